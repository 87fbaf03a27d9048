/*
 * mantis_ros.h — the ROS side of the drop-in, in plain C.
 *
 * The reference node's wire boundary, without roscpp:
 *   ingestion  quadDetection(const sensor_msgs::ImageConstPtr&,
 *              const sensor_msgs::CameraInfoConstPtr&)        src/mantis3.cpp:68-77
 *              (toCvShare(img, img->encoding) clone, get3x3FromVector(cam->K),
 *              cv::Mat(cam->D), frame_id; stamp never set — SURVEY Q15)
 *   egress     publishPose -> geometry_msgs/PoseWithCovarianceStamped on
 *              "mantis/pose_estimate"                         PosePub.h:12-61
 *   service    mantis/mantisService (Image[] image, CameraInfo[] camera_info,
 *              Vector3 delta_pos, Quaternion delta_quat ---
 *              Pose pose, float64 weight, int32 num_particles)  srv/mantisService.srv:1-13,
 *              server runMantis                              src/mantis_server.cpp:23-30
 *
 * Messages are handled in the ROS1 serialization (what TCPROS carries and a
 * rosbag record stores: little-endian scalars, uint32 length before every
 * string and variable array, fixed arrays inline), so a process that receives
 * those bytes — a thin TCPROS shim, a bag player, rosbridge — drives the
 * library with one call per message. Parsed messages point into the caller's
 * buffer (no copies of the pixel data); the library's own calls keep the
 * mantis.h ownership rules.
 */
#ifndef MANTIS_ROS_H
#define MANTIS_ROS_H
#include <stddef.h>
#include <stdint.h>

#include "mantis.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MANTIS_ROS_MAX_D 16

typedef struct mantis_ros_header { /* std_msgs/Header */
  uint32_t seq;
  uint32_t stamp_sec, stamp_nsec;
  const char* frame_id;            /* into the parsed buffer, not NUL-terminated */
  uint32_t frame_id_len;
} mantis_ros_header;

typedef struct mantis_ros_image {  /* sensor_msgs/Image */
  mantis_ros_header header;
  uint32_t height, width;
  const char* encoding;            /* into the buffer, not NUL-terminated */
  uint32_t encoding_len;
  uint8_t is_bigendian;
  uint32_t step;
  const uint8_t* data;             /* into the buffer */
  uint32_t data_len;
} mantis_ros_image;

typedef struct mantis_ros_camera_info { /* sensor_msgs/CameraInfo */
  mantis_ros_header header;
  uint32_t height, width;
  const char* distortion_model;
  uint32_t distortion_model_len;
  uint32_t D_len;                  /* entries of D present in the message */
  double D[MANTIS_ROS_MAX_D];      /* the first min(D_len, 16) */
  double K[9], R[9], P[12];
  uint32_t binning_x, binning_y;
  uint32_t roi_x_offset, roi_y_offset, roi_height, roi_width;
  uint8_t roi_do_rectify;
} mantis_ros_camera_info;

typedef struct mantis_ros_pose_stamped { /* geometry_msgs/PoseWithCovarianceStamped */
  uint32_t seq;
  uint32_t stamp_sec, stamp_nsec;
  char frame_id[32];               /* NUL-terminated; "world" (Mantis3Params.h WORLD_FRAME) */
  double position[3];
  double orientation_xyzw[4];
  double covariance[36];
} mantis_ros_pose_stamped;

typedef struct mantis_ros_service_response { /* mantisService response */
  double position[3];
  double orientation_xyzw[4];
  double weight;
  int32_t num_particles;
} mantis_ros_service_response;

/* --------------------------------------------------- ROS1 serialization */
/* Parse one message from buf; returns the bytes consumed, or -1 when buf is
 * short or a length field overruns it. */
int64_t mantis_ros_parse_image(const uint8_t* buf, size_t len, mantis_ros_image* out);
int64_t mantis_ros_parse_camera_info(const uint8_t* buf, size_t len, mantis_ros_camera_info* out);
/* mantisService request: fills up to max_cams images / camera infos (pointing
 * into buf), the counts, and motion (delta_pos, delta_quat). -1 when malformed
 * or when more than max_cams images are present. */
int64_t mantis_ros_parse_service_request(const uint8_t* buf, size_t len, mantis_ros_image* images,
                                         int32_t* n_images, mantis_ros_camera_info* infos, int32_t* n_infos,
                                         int32_t max_cams, mantis_motion* motion);
/* Serialize; return the bytes the message needs (writes only when cap is
 * large enough, so a call with cap = 0 sizes the buffer). */
int64_t mantis_ros_write_pose(const mantis_ros_pose_stamped* msg, uint8_t* buf, size_t cap);
int64_t mantis_ros_write_service_response(const mantis_ros_service_response* msg, uint8_t* buf, size_t cap);

/* ------------------------------------------ messages <-> library types */
/* sensor_msgs/Image + CameraInfo -> mantis_image (host memory, borrowed).
 * As the reference: the bytes are used as BGR whatever the 3-channel 8-bit
 * encoding says ("bgr8", "rgb8", "8UC3"; toCvShare keeps the encoding and
 * cvtColor(BGR2GRAY) follows, QuadDetection.h:209); any other encoding, a D
 * that is not the 4 fisheye coefficients (cv::fisheye asserts it), or a
 * data/step inconsistent with height x width gives MANTIS_ERR_ARG. The
 * camera is the rig base (T_base_cam = identity); frame_id is left NULL (the
 * caller keeps header.frame_id for its tf lookups). */
mantis_status mantis_ros_to_image(const mantis_ros_image* img, const mantis_ros_camera_info* cam, mantis_image* out);
/* publishPose (PosePub.h:12-61): fills the message and returns 1 when the
 * reference would publish (yaw gap > 4000), 0 otherwise, <0 on bad arguments.
 * stamp: the reference never sets the image stamp, so by default
 * (use_image_stamp = 0) the pose carries 0; 1 takes the image header's. */
int32_t mantis_ros_pose_from_result(const mantis_cam_result* r, const mantis_ros_header* image_header,
                                    int32_t use_image_stamp, mantis_ros_pose_stamped* out);
mantis_status mantis_ros_service_response_from_result(const mantis_result* r, mantis_ros_service_response* out);

/* --------------------------------------------------- whole callbacks */
/* quadDetection from the two serialized messages: parse, convert, process one
 * frame. pose_len receives the size of the serialized PoseWithCovarianceStamped
 * written to pose_buf when the frame publishes, 0 when it does not (0 quads,
 * 0 hypotheses, yaw ambiguous). cam_out (may be NULL) gets the frame result. */
mantis_status mantis_ros_image_callback(void* ctx, const uint8_t* image_msg, size_t image_len,
                                        const uint8_t* camera_info_msg, size_t camera_info_len,
                                        int32_t use_image_stamp, uint8_t* pose_buf, size_t pose_cap,
                                        int64_t* pose_len, mantis_cam_result* cam_out);
/* runMantis with the response filled (the reference leaves it empty): parse the
 * serialized request, process its cameras as one rig (T_base_cam = identity for
 * each; rigs with extrinsics use mantis_process), serialize the response. */
mantis_status mantis_ros_service_call(void* ctx, const uint8_t* request, size_t request_len, uint8_t* response_buf,
                                      size_t response_cap, int64_t* response_len, mantis_result* out);

#ifdef __cplusplus
}
#endif
#endif /* MANTIS_ROS_H */
