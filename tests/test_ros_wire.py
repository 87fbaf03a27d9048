"""ROS side of the drop-in (include/mantis_ros.h) on the CPU:
the library's ROS1 parsers / serializers against an independent Python
restatement of the wire format (mantis_amd/ros.py), the message -> mantis_image
validation rules of the reference callback (src/mantis3.cpp:68-77), and the
publishPose mapping (PosePub.h:12-61). No GPU calls. Parity with roscpp's own
serializer is unpinned (no ROS in this image): the layouts follow the message
definitions field by field."""
import ctypes as C
import struct

import numpy as np

import mantis_amd as M
from mantis_amd import ros

K = [323.1511535644531, 0, 642.658203125, 0, 322.78955078125, 349.5538330078125, 0, 0, 1]
D = [0.0029509200248867273, -0.009944040328264236, 0.005587350111454725, -0.00205406011082232]
ERR_ARG = 1


def _bytes_at(ptr, n):
    return C.string_at(ptr, n)


def test_image_roundtrip_and_padding():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (7, 5, 3), dtype=np.uint8)
    b = ros.image_bytes(img, step=20, seq=9, stamp=(12, 34), frame_id="cam_front")
    im, n, keep = ros.parse_image(b)
    assert n == len(b)
    assert (im.header.seq, im.header.stamp_sec, im.header.stamp_nsec) == (9, 12, 34)
    assert _bytes_at(im.header.frame_id, im.header.frame_id_len) == b"cam_front"
    assert (im.height, im.width, im.step, im.is_bigendian) == (7, 5, 20, 0)
    assert _bytes_at(im.encoding, im.encoding_len) == b"bgr8"
    data = np.frombuffer(_bytes_at(im.data, im.data_len), np.uint8).reshape(7, 20)
    assert np.array_equal(data[:, :15].reshape(7, 5, 3), img)


def test_truncated_and_overrunning_messages_rejected():
    img = np.zeros((4, 4, 3), np.uint8)
    b = ros.image_bytes(img)
    for cut in (0, 3, 20, len(b) - 1):
        assert ros.parse_image(b[:cut])[1] == -1
    bad = bytearray(b)
    struct.pack_into("<I", bad, len(b) - 48 - 4, 10 ** 6)  # data length past the end
    assert ros.parse_image(bytes(bad))[1] == -1
    ci = ros.camera_info_bytes(K, D, 1280, 720)
    assert ros.parse_camera_info(ci[:-1])[1] == -1


def test_camera_info_fields():
    b = ros.camera_info_bytes(K, D, 1280, 720, seq=2, frame_id="cam")
    ci, n, keep = ros.parse_camera_info(b)
    assert n == len(b)
    assert (ci.width, ci.height, ci.D_len) == (1280, 720, 4)
    assert _bytes_at(ci.distortion_model, ci.distortion_model_len) == b"fisheye"
    assert list(ci.K) == K and list(ci.D)[:4] == D
    assert list(ci.R) == list(np.eye(3).reshape(9))


def test_to_image_rules_of_the_reference_callback():
    img = np.zeros((720, 1280, 3), np.uint8)
    ci, _, kc = ros.parse_camera_info(ros.camera_info_bytes(K, D, 1280, 720))
    for enc in ("bgr8", "rgb8", "8UC3"):  # used as BGR bytes, as toCvShare(img, img->encoding) + BGR2GRAY
        im, _, ki = ros.parse_image(ros.image_bytes(img, encoding=enc, step=3 * 1280 + 64, stamp=(5, 6)))
        st, out = ros.to_image(im, ci)
        assert st == 0
        assert (out.width, out.height, out.step_bytes, out.mem_kind) == (1280, 720, 3 * 1280 + 64, 0)
        assert list(out.K) == K and list(out.D) == D and out.stamp_ns == 5 * 10 ** 9 + 6
        assert list(out.T_base_cam) == list(np.eye(4).reshape(16))
    for enc in ("mono8", "bgra8", "16UC3", "bgr"):
        im, _, ki = ros.parse_image(ros.image_bytes(img, encoding=enc))
        assert ros.to_image(im, ci)[0] == ERR_ARG
    # the fisheye model needs exactly 4 coefficients (cv::fisheye asserts D.total() == 4)
    ci5, _, k5 = ros.parse_camera_info(ros.camera_info_bytes(K, D + [0.0], 1280, 720))
    im, _, ki = ros.parse_image(ros.image_bytes(img))
    assert ros.to_image(im, ci5)[0] == ERR_ARG
    # step below 3 * width, data shorter than step * height
    im, _, kb = ros.parse_image(ros.image_bytes(np.zeros((4, 4, 3), np.uint8)))
    ci4, _, k4 = ros.parse_camera_info(ros.camera_info_bytes(K, D, 4, 4))
    im.step = 11
    assert ros.to_image(im, ci4)[0] == ERR_ARG
    im.step = 12
    im.data_len = 47
    assert ros.to_image(im, ci4)[0] == ERR_ARG


def test_pose_from_result_and_wire():
    cr = M.MantisCamResult()
    cr.publish = 1
    cr.position[:] = [0.1, -0.2, 1.5]
    cr.orientation_xyzw[:] = [0.0, 0.0, 0.7071067811865476, 0.7071067811865476]
    for i in range(6):
        cr.covariance[7 * i] = 123.0 / 600.0
    hdr = M.RosHeader()
    hdr.stamp_sec, hdr.stamp_nsec = 77, 88
    pub, msg = ros.pose_from_result(cr, hdr, use_image_stamp=0)
    assert pub == 1 and msg.frame_id == b"world" and (msg.stamp_sec, msg.stamp_nsec) == (0, 0)
    d = ros.parse_pose_bytes(ros.write_pose(msg))
    assert d["frame_id"] == "world" and d["stamp"] == (0, 0)
    assert d["position"] == (0.1, -0.2, 1.5)
    assert d["orientation_xyzw"] == tuple(cr.orientation_xyzw)
    assert d["covariance"] == tuple(cr.covariance)
    pub, msg = ros.pose_from_result(cr, hdr, use_image_stamp=1)
    assert (msg.stamp_sec, msg.stamp_nsec) == (77, 88)
    cr.publish = 0
    assert ros.pose_from_result(cr, hdr)[0] == 0


def test_service_request_and_response_wire():
    rng = np.random.default_rng(5)
    imgs = [rng.integers(0, 256, (6, 8, 3), dtype=np.uint8) for _ in range(3)]
    req = ros.service_request_bytes([ros.image_bytes(i, frame_id=f"c{k}") for k, i in enumerate(imgs)],
                                    [ros.camera_info_bytes(K, D, 8, 6) for _ in imgs],
                                    delta_pos=(0.5, -1.0, 2.0), delta_quat_xyzw=(0.0, 0.1, 0.0, 0.99))
    n, ims, cis, m, keep = ros.parse_service_request(req)
    assert n == len(req) and len(ims) == 3 and len(cis) == 3
    assert [_bytes_at(im.header.frame_id, im.header.frame_id_len) for im in ims] == [b"c0", b"c1", b"c2"]
    for im, ref in zip(ims, imgs):
        assert np.array_equal(np.frombuffer(_bytes_at(im.data, im.data_len), np.uint8).reshape(6, 8, 3), ref)
    assert list(m.delta_pos) == [0.5, -1.0, 2.0] and list(m.delta_quat_xyzw) == [0.0, 0.1, 0.0, 0.99]
    assert ros.parse_service_request(req, max_cams=2)[0] == -1  # more images than the context holds
    assert ros.parse_service_request(req[:-1])[0] == -1
    r = M.MantisResult()
    r.position[:] = [1.0, 2.0, 3.0]
    r.orientation_xyzw[:] = [0.0, 0.0, 0.0, 1.0]
    r.weight, r.num_particles = 4567.25, 2468
    resp = M.RosServiceResponse()
    assert M.lib().mantis_ros_service_response_from_result(C.byref(r), C.byref(resp)) == 0
    n = M.lib().mantis_ros_write_service_response(C.byref(resp), None, 0)
    buf = C.create_string_buffer(int(n))
    assert M.lib().mantis_ros_write_service_response(C.byref(resp), buf, n) == n
    d = ros.parse_service_response_bytes(buf.raw)
    assert d == {"position": (1.0, 2.0, 3.0), "orientation_xyzw": (0.0, 0.0, 0.0, 1.0), "weight": 4567.25,
                 "num_particles": 2468}


def test_callbacks_reject_null_context():
    b = ros.image_bytes(np.zeros((4, 4, 3), np.uint8))
    n = C.c_int64(0)
    assert M.lib().mantis_ros_image_callback(None, b, len(b), b, len(b), 0, None, 0, C.byref(n), None) == ERR_ARG
    assert M.lib().mantis_ros_service_call(None, b, len(b), None, 0, C.byref(n), None) == ERR_ARG
