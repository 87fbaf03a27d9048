"""ROS side of the drop-in (include/mantis_ros.h): ROS1-serialized
sensor_msgs/Image, sensor_msgs/CameraInfo, geometry_msgs/PoseWithCovarianceStamped
and the mantisService request/response (srv/mantisService.srv:1-13).

The writers/readers here are an independent restatement of the ROS1 wire
format (little-endian; uint32 length before strings and variable arrays;
fixed arrays inline) used by the tests to cross-check the library's C
parser/serializer; `image_callback` and `service_call` drive the library's
whole-callback entry points (mantis_ros_image_callback / mantis_ros_service_call)
with serialized messages, as a TCPROS shim or bag player would.
"""
import ctypes as C
import struct

import numpy as np

from . import (MantisCamResult, MantisError, MantisImage, MantisMotion, MantisResult, RosCameraInfo, RosImage,
               RosPoseStamped, RosServiceResponse, lib)


def _str(s):
    b = s.encode() if isinstance(s, str) else bytes(s)
    return struct.pack("<I", len(b)) + b


def header_bytes(seq=0, stamp=(0, 0), frame_id=""):
    """std_msgs/Header"""
    return struct.pack("<III", seq, stamp[0], stamp[1]) + _str(frame_id)


def image_bytes(img, encoding="bgr8", step=None, seq=0, stamp=(0, 0), frame_id="camera", is_bigendian=0):
    """sensor_msgs/Image from an H x W x 3 uint8 array (rows padded to step)."""
    h, w = img.shape[:2]
    step = step or 3 * w
    rows = np.zeros((h, step), np.uint8)
    rows[:, :3 * w] = img.reshape(h, 3 * w)
    data = rows.tobytes()
    return (header_bytes(seq, stamp, frame_id) + struct.pack("<II", h, w) + _str(encoding) +
            struct.pack("<BI", is_bigendian, step) + struct.pack("<I", len(data)) + data)


def camera_info_bytes(K, D, width, height, seq=0, stamp=(0, 0), frame_id="camera", distortion_model="fisheye"):
    """sensor_msgs/CameraInfo (R = identity, P = [K | 0], no binning / ROI)."""
    K = np.asarray(K, np.float64).reshape(9)
    P = np.zeros(12)
    P[[0, 1, 2, 4, 5, 6, 8, 9, 10]] = K
    out = header_bytes(seq, stamp, frame_id) + struct.pack("<II", height, width) + _str(distortion_model)
    out += struct.pack("<I", len(D)) + struct.pack(f"<{len(D)}d", *D)
    out += struct.pack("<9d", *K) + struct.pack("<9d", *np.eye(3).reshape(9)) + struct.pack("<12d", *P)
    out += struct.pack("<II", 0, 0) + struct.pack("<IIIIB", 0, 0, 0, 0, 0)
    return out


def service_request_bytes(images, infos, delta_pos=(0, 0, 0), delta_quat_xyzw=(0, 0, 0, 1)):
    """mantisService request: Image[] image, CameraInfo[] camera_info, Vector3, Quaternion."""
    out = struct.pack("<I", len(images)) + b"".join(images)
    out += struct.pack("<I", len(infos)) + b"".join(infos)
    return out + struct.pack("<3d", *delta_pos) + struct.pack("<4d", *delta_quat_xyzw)


def parse_pose_bytes(b):
    """geometry_msgs/PoseWithCovarianceStamped -> dict"""
    seq, sec, nsec, n = struct.unpack_from("<IIII", b, 0)
    o = 16
    frame = b[o:o + n].decode()
    o += n
    v = struct.unpack_from("<43d", b, o)
    assert o + 43 * 8 == len(b), "trailing bytes"
    return {"seq": seq, "stamp": (sec, nsec), "frame_id": frame, "position": v[0:3],
            "orientation_xyzw": v[3:7], "covariance": v[7:43]}


def parse_service_response_bytes(b):
    """mantisService response: Pose pose, float64 weight, int32 num_particles"""
    assert len(b) == 8 * 8 + 4
    v = struct.unpack_from("<8d", b, 0)
    return {"position": v[0:3], "orientation_xyzw": v[3:7], "weight": v[7],
            "num_particles": struct.unpack_from("<i", b, 64)[0]}


def _buf(b):
    return C.create_string_buffer(bytes(b), len(b))


def parse_image(b):
    """C parser: (RosImage, bytes consumed); the struct points into the returned buffer."""
    buf = _buf(b)
    im = RosImage()
    n = lib().mantis_ros_parse_image(buf, len(b), C.byref(im))
    return im, n, buf


def parse_camera_info(b):
    buf = _buf(b)
    ci = RosCameraInfo()
    n = lib().mantis_ros_parse_camera_info(buf, len(b), C.byref(ci))
    return ci, n, buf


def parse_service_request(b, max_cams=8):
    buf = _buf(b)
    ims = (RosImage * max_cams)()
    cis = (RosCameraInfo * max_cams)()
    ni, nc = C.c_int32(0), C.c_int32(0)
    m = MantisMotion()
    n = lib().mantis_ros_parse_service_request(buf, len(b), ims, C.byref(ni), cis, C.byref(nc), max_cams,
                                               C.byref(m))
    return n, list(ims[:ni.value]), list(cis[:nc.value]), m, buf


def to_image(im, ci):
    out = MantisImage()
    st = lib().mantis_ros_to_image(C.byref(im), C.byref(ci), C.byref(out))
    return st, out


def write_pose(msg):
    n = lib().mantis_ros_write_pose(C.byref(msg), None, 0)
    buf = C.create_string_buffer(int(n))
    lib().mantis_ros_write_pose(C.byref(msg), buf, n)
    return buf.raw


def pose_from_result(cam_result, image_header=None, use_image_stamp=0):
    msg = RosPoseStamped()
    pub = lib().mantis_ros_pose_from_result(C.byref(cam_result), C.byref(image_header) if image_header else None,
                                            use_image_stamp, C.byref(msg))
    return pub, msg


def image_callback(m, image_msg, camera_info_msg, use_image_stamp=0):
    """quadDetection over serialized messages: (serialized pose or None, MantisCamResult)."""
    ib, cb = _buf(image_msg), _buf(camera_info_msg)
    out = C.create_string_buffer(512)
    n = C.c_int64(0)
    cr = MantisCamResult()
    st = lib().mantis_ros_image_callback(m.h, ib, len(image_msg), cb, len(camera_info_msg), use_image_stamp, out,
                                         512, C.byref(n), C.byref(cr))
    if st != 0:
        raise MantisError(f"mantis_ros_image_callback: status {st}: {lib().mantis_last_error(m.h).decode()}")
    return (out.raw[:n.value] if n.value > 0 else None), cr


def service_call(m, request):
    """runMantis over a serialized request: (serialized response, MantisResult)."""
    rb = _buf(request)
    out = C.create_string_buffer(128)
    n = C.c_int64(0)
    r = MantisResult()
    st = lib().mantis_ros_service_call(m.h, rb, len(request), out, 128, C.byref(n), C.byref(r))
    if st != 0:
        raise MantisError(f"mantis_ros_service_call: status {st}: {lib().mantis_last_error(m.h).decode()}")
    return out.raw[:n.value], r
