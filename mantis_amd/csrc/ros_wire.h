// ROS side of the drop-in (include/mantis_ros.h): ROS1
// serialization of sensor_msgs/Image, sensor_msgs/CameraInfo,
// geometry_msgs/PoseWithCovarianceStamped and the mantisService
// request/response, their conversion to the library types, and the whole
// quadDetection / runMantis callbacks over serialized messages. Host code;
// included at the end of api.hip (one translation unit).
//
// Reference semantics followed:
//   ingestion  src/mantis3.cpp:68-77 (toCvShare(img, img->encoding), K via
//              get3x3FromVector QuadDetection.h:189-201, D = cv::Mat(cam->D))
//   egress     PosePub.h:12-61 (publish iff yaw gap > MINIMUM_YAW_DIFFERENCE,
//              frame WORLD_FRAME, covariance diag(error / 600), stamp = the
//              never-set image stamp, i.e. 0 — SURVEY Q15)
//   service    srv/mantisService.srv:1-13
#pragma once
#include <cstring>

#include "../../include/mantis_ros.h"

namespace {

// little-endian reader over [p, end); every read is bounds-checked
struct RosReader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;
  bool need(size_t n) {
    if (!ok || (size_t)(end - p) < n) ok = false;
    return ok;
  }
  uint32_t u32() {
    uint32_t v = 0;
    if (need(4)) { std::memcpy(&v, p, 4); p += 4; }
    return v;
  }
  uint8_t u8() {
    uint8_t v = 0;
    if (need(1)) { v = *p; p += 1; }
    return v;
  }
  double f64() {
    double v = 0;
    if (need(8)) { std::memcpy(&v, p, 8); p += 8; }
    return v;
  }
  // string / uint8[]: length then bytes (returned in place)
  const uint8_t* bytes(uint32_t& n) {
    n = u32();
    if (!need(n)) { n = 0; return nullptr; }
    const uint8_t* b = p;
    p += n;
    return b;
  }
  void header(mantis_ros_header& h) {
    h.seq = u32();
    h.stamp_sec = u32();
    h.stamp_nsec = u32();
    h.frame_id = (const char*)bytes(h.frame_id_len);
  }
};

struct RosWriter {
  uint8_t* p;
  size_t cap, n = 0;
  void raw(const void* v, size_t k) {
    if (n + k <= cap) std::memcpy(p + n, v, k);
    n += k;
  }
  void u32(uint32_t v) { raw(&v, 4); }
  void i32(int32_t v) { raw(&v, 4); }
  void f64(double v) { raw(&v, 8); }
  void str(const char* s) {
    const uint32_t k = (uint32_t)std::strlen(s);
    u32(k);
    raw(s, k);
  }
};

bool ros_parse_image(RosReader& r, mantis_ros_image& o) {
  r.header(o.header);
  o.height = r.u32();
  o.width = r.u32();
  o.encoding = (const char*)r.bytes(o.encoding_len);
  o.is_bigendian = r.u8();
  o.step = r.u32();
  o.data = r.bytes(o.data_len);
  return r.ok;
}

bool ros_parse_camera_info(RosReader& r, mantis_ros_camera_info& o) {
  r.header(o.header);
  o.height = r.u32();
  o.width = r.u32();
  o.distortion_model = (const char*)r.bytes(o.distortion_model_len);
  o.D_len = r.u32();
  for (uint32_t i = 0; i < o.D_len && r.ok; i++) {
    const double d = r.f64();
    if (i < MANTIS_ROS_MAX_D) o.D[i] = d;
  }
  for (int i = 0; i < 9; i++) o.K[i] = r.f64();
  for (int i = 0; i < 9; i++) o.R[i] = r.f64();
  for (int i = 0; i < 12; i++) o.P[i] = r.f64();
  o.binning_x = r.u32();
  o.binning_y = r.u32();
  o.roi_x_offset = r.u32();
  o.roi_y_offset = r.u32();
  o.roi_height = r.u32();
  o.roi_width = r.u32();
  o.roi_do_rectify = r.u8();
  return r.ok;
}

bool enc_is(const mantis_ros_image& im, const char* e) {
  const size_t k = std::strlen(e);
  return im.encoding && im.encoding_len == k && std::memcmp(im.encoding, e, k) == 0;
}

}  // namespace

extern "C" {

int64_t mantis_ros_parse_image(const uint8_t* buf, size_t len, mantis_ros_image* out) {
  if (!buf || !out) return -1;
  RosReader r{buf, buf + len};
  *out = mantis_ros_image{};
  return ros_parse_image(r, *out) ? (int64_t)(r.p - buf) : -1;
}

int64_t mantis_ros_parse_camera_info(const uint8_t* buf, size_t len, mantis_ros_camera_info* out) {
  if (!buf || !out) return -1;
  RosReader r{buf, buf + len};
  *out = mantis_ros_camera_info{};
  return ros_parse_camera_info(r, *out) ? (int64_t)(r.p - buf) : -1;
}

int64_t mantis_ros_parse_service_request(const uint8_t* buf, size_t len, mantis_ros_image* images,
                                         int32_t* n_images, mantis_ros_camera_info* infos, int32_t* n_infos,
                                         int32_t max_cams, mantis_motion* motion) {
  if (!buf || !n_images || !n_infos || max_cams < 0 || (max_cams > 0 && (!images || !infos))) return -1;
  RosReader r{buf, buf + len};
  const uint32_t ni = r.u32();
  if (!r.ok || ni > (uint32_t)max_cams) return -1;
  for (uint32_t i = 0; i < ni; i++) {
    images[i] = mantis_ros_image{};
    if (!ros_parse_image(r, images[i])) return -1;
  }
  const uint32_t nc = r.u32();
  if (!r.ok || nc > (uint32_t)max_cams) return -1;
  for (uint32_t i = 0; i < nc; i++) {
    infos[i] = mantis_ros_camera_info{};
    if (!ros_parse_camera_info(r, infos[i])) return -1;
  }
  mantis_motion m{};
  for (int k = 0; k < 3; k++) m.delta_pos[k] = r.f64();
  for (int k = 0; k < 4; k++) m.delta_quat_xyzw[k] = r.f64();  // geometry_msgs/Quaternion: x, y, z, w
  if (!r.ok) return -1;
  if (motion) *motion = m;
  *n_images = (int32_t)ni;
  *n_infos = (int32_t)nc;
  return (int64_t)(r.p - buf);
}

int64_t mantis_ros_write_pose(const mantis_ros_pose_stamped* m, uint8_t* buf, size_t cap) {
  if (!m) return -1;
  RosWriter w{buf, buf ? cap : 0};
  w.u32(m->seq);
  w.u32(m->stamp_sec);
  w.u32(m->stamp_nsec);
  char fid[sizeof m->frame_id + 1];
  std::memcpy(fid, m->frame_id, sizeof m->frame_id);
  fid[sizeof m->frame_id] = 0;
  w.str(fid);
  for (int k = 0; k < 3; k++) w.f64(m->position[k]);
  for (int k = 0; k < 4; k++) w.f64(m->orientation_xyzw[k]);
  for (int k = 0; k < 36; k++) w.f64(m->covariance[k]);
  return (int64_t)w.n;
}

int64_t mantis_ros_write_service_response(const mantis_ros_service_response* m, uint8_t* buf, size_t cap) {
  if (!m) return -1;
  RosWriter w{buf, buf ? cap : 0};
  for (int k = 0; k < 3; k++) w.f64(m->position[k]);
  for (int k = 0; k < 4; k++) w.f64(m->orientation_xyzw[k]);
  w.f64(m->weight);
  w.i32(m->num_particles);
  return (int64_t)w.n;
}

mantis_status mantis_ros_to_image(const mantis_ros_image* img, const mantis_ros_camera_info* cam, mantis_image* out) {
  if (!img || !cam || !out) return MANTIS_ERR_ARG;
  if (!(enc_is(*img, "bgr8") || enc_is(*img, "rgb8") || enc_is(*img, "8UC3"))) return MANTIS_ERR_ARG;
  if (img->width < 1 || img->height < 1 || img->width > 0x7fffffffu / 3 || img->step < 3 * img->width)
    return MANTIS_ERR_ARG;
  if (!img->data || (uint64_t)img->data_len < (uint64_t)img->step * img->height) return MANTIS_ERR_ARG;
  if (cam->D_len != 4) return MANTIS_ERR_ARG;
  *out = mantis_image{};
  out->width = (int32_t)img->width;
  out->height = (int32_t)img->height;
  out->step_bytes = (int32_t)img->step;
  out->mem_kind = 0;
  out->bgr = img->data;
  for (int i = 0; i < 9; i++) out->K[i] = cam->K[i];
  for (int i = 0; i < 4; i++) out->D[i] = cam->D[i];
  for (int i = 0; i < 16; i++) out->T_base_cam[i] = (i % 5 == 0) ? 1.0 : 0.0;
  out->stamp_ns = (int64_t)img->header.stamp_sec * 1000000000LL + img->header.stamp_nsec;
  out->frame_id = nullptr;
  return MANTIS_OK;
}

int32_t mantis_ros_pose_from_result(const mantis_cam_result* r, const mantis_ros_header* image_header,
                                    int32_t use_image_stamp, mantis_ros_pose_stamped* out) {
  if (!r || !out) return -1;
  *out = mantis_ros_pose_stamped{};
  std::strncpy(out->frame_id, "world", sizeof out->frame_id - 1);
  if (use_image_stamp && image_header) {
    out->stamp_sec = image_header->stamp_sec;
    out->stamp_nsec = image_header->stamp_nsec;
  }
  for (int k = 0; k < 3; k++) out->position[k] = r->position[k];
  for (int k = 0; k < 4; k++) out->orientation_xyzw[k] = r->orientation_xyzw[k];
  for (int k = 0; k < 36; k++) out->covariance[k] = r->covariance[k];
  return r->publish ? 1 : 0;
}

mantis_status mantis_ros_service_response_from_result(const mantis_result* r, mantis_ros_service_response* out) {
  if (!r || !out) return MANTIS_ERR_ARG;
  *out = mantis_ros_service_response{};
  for (int k = 0; k < 3; k++) out->position[k] = r->position[k];
  for (int k = 0; k < 4; k++) out->orientation_xyzw[k] = r->orientation_xyzw[k];
  out->weight = r->weight;
  out->num_particles = r->num_particles;
  return MANTIS_OK;
}

mantis_status mantis_ros_image_callback(void* ctx, const uint8_t* image_msg, size_t image_len,
                                        const uint8_t* camera_info_msg, size_t camera_info_len,
                                        int32_t use_image_stamp, uint8_t* pose_buf, size_t pose_cap,
                                        int64_t* pose_len, mantis_cam_result* cam_out) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !pose_len) return MANTIS_ERR_ARG;
  *pose_len = 0;
  mantis_ros_image im;
  mantis_ros_camera_info ci;
  if (mantis_ros_parse_image(image_msg, image_len, &im) < 0 ||
      mantis_ros_parse_camera_info(camera_info_msg, camera_info_len, &ci) < 0) {
    c->err = "malformed sensor_msgs/Image or CameraInfo";
    return MANTIS_ERR_ARG;
  }
  mantis_image in;
  if (mantis_ros_to_image(&im, &ci, &in) != MANTIS_OK) {
    c->err = "unsupported image (3-channel 8-bit encoding, step >= 3 width, 4 fisheye D coefficients required)";
    return MANTIS_ERR_ARG;
  }
  mantis_result rr;
  mantis_cam_result cr;
  const mantis_status st = mantis_process(ctx, &in, 1, nullptr, &rr, &cr);
  if (st != MANTIS_OK) return st;
  if (cam_out) *cam_out = cr;
  mantis_ros_pose_stamped msg;
  if (mantis_ros_pose_from_result(&cr, &im.header, use_image_stamp, &msg) == 1) {
    const int64_t need = mantis_ros_write_pose(&msg, nullptr, 0);
    if (!pose_buf || (size_t)need > pose_cap) {
      c->err = "pose buffer too small";
      *pose_len = need;
      return MANTIS_ERR_CAPACITY;
    }
    *pose_len = mantis_ros_write_pose(&msg, pose_buf, pose_cap);
  }
  return MANTIS_OK;
}

mantis_status mantis_ros_service_call(void* ctx, const uint8_t* request, size_t request_len, uint8_t* response_buf,
                                      size_t response_cap, int64_t* response_len, mantis_result* out) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !response_len) return MANTIS_ERR_ARG;
  *response_len = 0;
  const int32_t cap = c->F;
  std::vector<mantis_ros_image> ims((size_t)cap);
  std::vector<mantis_ros_camera_info> cis((size_t)cap);
  int32_t ni = 0, nc = 0;
  mantis_motion m;
  if (mantis_ros_parse_service_request(request, request_len, ims.data(), &ni, cis.data(), &nc, cap, &m) < 0) {
    c->err = "malformed mantisService request (or more images than max_cams)";
    return MANTIS_ERR_ARG;
  }
  if (ni < 1 || ni != nc) {
    c->err = "mantisService request needs one CameraInfo per Image";
    return MANTIS_ERR_ARG;
  }
  std::vector<mantis_image> cams((size_t)ni);
  for (int32_t i = 0; i < ni; i++)
    if (mantis_ros_to_image(&ims[i], &cis[i], &cams[i]) != MANTIS_OK) {
      c->err = "unsupported image in mantisService request";
      return MANTIS_ERR_ARG;
    }
  mantis_result rr;
  const mantis_status st = mantis_process(ctx, cams.data(), ni, &m, &rr, nullptr);
  if (st != MANTIS_OK) return st;
  if (out) *out = rr;
  mantis_ros_service_response resp;
  mantis_ros_service_response_from_result(&rr, &resp);
  const int64_t need = mantis_ros_write_service_response(&resp, nullptr, 0);
  *response_len = need;
  if (!response_buf || (size_t)need > response_cap) {
    c->err = "response buffer too small";
    return MANTIS_ERR_CAPACITY;
  }
  mantis_ros_write_service_response(&resp, response_buf, response_cap);
  return MANTIS_OK;
}

}  // extern "C"
