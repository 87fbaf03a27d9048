// Device/host math shared by the HIP kernels of libmantis_amd.so:
// the tf/LinearMath subset, the OpenCV fisheye projection and cvRound.
// FP64 throughout, built with -ffp-contract=off so the operation order below
// is the operation order executed (parity with the CPU oracle is ulp-exact
// except where the device libm differs from glibc by an ulp).
//
// Reference semantics:
//   Hypothesis::setC2W/setW2C/projectPoint   include/mantis3/Mantis3Types.h:68-93
//   distortPixel -> cv::fisheye::distortPoints include/mantis3/Mantis3Types.h:125-136
//   undistortPoints (normalized)             include/mantis3/QuadDetection.h:289-298
//   yaw copies rotZ * w2c                    include/mantis3/HypothesisGeneration.h:91-99
//   particle perturbation w2c * rand         include/mantis3/PoseAdjustment.h:13-23
#pragma once
#include <cmath>
#include <cstdint>

#include "mk_dmath.h"

#ifdef __HIPCC__
#define MK_HD __host__ __device__ inline
#else
#define MK_HD inline
#endif

namespace mk {

// Rigid transform: basis row-major R[9], origin t[3] (tf::Transform layout).
struct Xf {
  double R[9];
  double t[3];
};
struct Quat {
  double x, y, z, w;
};

MK_HD double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// tf Matrix3x3 * Matrix3x3: o[i][j] = m2[0][j]*m1[i][0] + m2[1][j]*m1[i][1] + m2[2][j]*m1[i][2]
MK_HD void mat_mul(const double* m1, const double* m2, double* o) {
  double r[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) r[i * 3 + j] = m2[j] * m1[i * 3] + m2[3 + j] * m1[i * 3 + 1] + m2[6 + j] * m1[i * 3 + 2];
  for (int k = 0; k < 9; k++) o[k] = r[k];
}
MK_HD void xf_apply(const Xf& T, const double* x, double* o) {
  double r0 = dot3(T.R, x) + T.t[0];
  double r1 = dot3(T.R + 3, x) + T.t[1];
  double r2 = dot3(T.R + 6, x) + T.t[2];
  o[0] = r0; o[1] = r1; o[2] = r2;
}
MK_HD Xf xf_mul(const Xf& a, const Xf& b) {
  Xf o;
  mat_mul(a.R, b.R, o.R);
  xf_apply(a, b.t, o.t);
  return o;
}
MK_HD Xf xf_inverse(const Xf& a) {
  Xf o;
  o.R[0] = a.R[0]; o.R[1] = a.R[3]; o.R[2] = a.R[6];
  o.R[3] = a.R[1]; o.R[4] = a.R[4]; o.R[5] = a.R[7];
  o.R[6] = a.R[2]; o.R[7] = a.R[5]; o.R[8] = a.R[8];
  double nt[3] = {-a.t[0], -a.t[1], -a.t[2]};
  o.t[0] = dot3(o.R, nt);
  o.t[1] = dot3(o.R + 3, nt);
  o.t[2] = dot3(o.R + 6, nt);
  return o;
}
// Matrix3x3::setRotation(q), s = 2/|q|^2
MK_HD void basis_from_quat(const Quat& q, double* R) {
  double d = q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w;
  double s = 2.0 / d;
  double xs = q.x * s, ys = q.y * s, zs = q.z * s;
  double wx = q.w * xs, wy = q.w * ys, wz = q.w * zs;
  double xx = q.x * xs, xy = q.x * ys, xz = q.x * zs;
  double yy = q.y * ys, yz = q.y * zs, zz = q.z * zs;
  R[0] = 1.0 - (yy + zz); R[1] = xy - wz; R[2] = xz + wy;
  R[3] = xy + wz; R[4] = 1.0 - (xx + zz); R[5] = yz - wx;
  R[6] = xz - wy; R[7] = yz + wx; R[8] = 1.0 - (xx + yy);
}
// Matrix3x3::getRotation (Shepperd)
MK_HD Quat basis_to_quat(const double* m) {
  double tr = m[0] + m[4] + m[8];
  double t[4];
  if (tr > 0.0) {
    double s = sqrt(tr + 1.0);
    t[3] = s * 0.5;
    s = 0.5 / s;
    t[0] = (m[7] - m[5]) * s;
    t[1] = (m[2] - m[6]) * s;
    t[2] = (m[3] - m[1]) * s;
  } else {
    int i = m[0] < m[4] ? (m[4] < m[8] ? 2 : 1) : (m[0] < m[8] ? 2 : 0);
    int j = (i + 1) % 3, k = (i + 2) % 3;
    double s = sqrt(m[i * 4] - m[j * 4] - m[k * 4] + 1.0);
    t[i] = s * 0.5;
    s = 0.5 / s;
    t[3] = (m[k * 3 + j] - m[j * 3 + k]) * s;
    t[j] = (m[j * 3 + i] + m[i * 3 + j]) * s;
    t[k] = (m[k * 3 + i] + m[i * 3 + k]) * s;
  }
  Quat q;
  q.x = t[0]; q.y = t[1]; q.z = t[2]; q.w = t[3];
  return q;
}
// setRPY(roll, pitch, yaw) = setEulerYPR(yaw, pitch, roll)
MK_HD void basis_from_rpy(double roll, double pitch, double yaw, double* R) {
  double ci = cos(roll), cj = cos(pitch), ch = cos(yaw);
  double si = sin(roll), sj = sin(pitch), sh = sin(yaw);
  double cc = ci * ch, cs = ci * sh, sc = si * ch, ss = si * sh;
  R[0] = cj * ch; R[1] = sj * sc - cs; R[2] = sj * cc + ss;
  R[3] = cj * sh; R[4] = sj * ss + cc; R[5] = sj * cs - sc;
  R[6] = -sj; R[7] = cj * si; R[8] = cj * ci;
}
// basis_from_rpy for |angles| < 2^30: on the device mk_dmath.h sincos_small
// (= ocml sin/cos without the large-argument path), glibc on the host
MK_HD void basis_from_rpy_small(double roll, double pitch, double yaw, double* R) {
#if !MK_DM_DEVICE
  basis_from_rpy(roll, pitch, yaw, R);
#else
  double si, ci, sj, cj, sh, ch;
  dm::sincos_small(roll, &si, &ci);
  dm::sincos_small(pitch, &sj, &cj);
  dm::sincos_small(yaw, &sh, &ch);
  double cc = ci * ch, cs = ci * sh, sc = si * ch, ss = si * sh;
  R[0] = cj * ch; R[1] = sj * sc - cs; R[2] = sj * cc + ss;
  R[3] = cj * sh; R[4] = sj * ss + cc; R[5] = sj * cs - sc;
  R[6] = -sj; R[7] = cj * si; R[8] = cj * ci;
#endif
}
// getRPY (getEulerYPR solution 1)
MK_HD void basis_to_rpy(const double* m, double* roll, double* pitch, double* yaw) {
  if (fabs(m[6]) >= 1) {
    *yaw = 0;
    double delta = atan2(m[7], m[8]);
    *pitch = (m[6] < 0) ? M_PI / 2.0 : -M_PI / 2.0;
    *roll = delta;
  } else {
    *pitch = -asin(m[6]);
    double cp = cos(*pitch);
    *roll = atan2(m[7] / cp, m[8] / cp);
    *yaw = atan2(m[3] / cp, m[0] / cp);
  }
}

// Hypothesis: c2w maps world points into the camera frame; w2c is the pose.
struct Hyp {
  Xf c2w, w2c;
  Quat q;
  double error;
};
MK_HD void hyp_set_c2w(Hyp& h, const Xf& T) { h.c2w = T; h.w2c = xf_inverse(T); h.q = basis_to_quat(h.w2c.R); }
MK_HD void hyp_set_w2c(Hyp& h, const Xf& T) { h.w2c = T; h.c2w = xf_inverse(T); h.q = basis_to_quat(h.w2c.R); }

MK_HD Xf make_rot_z90() {
  Xf t;
  Quat q{0, 0, 1 / sqrt(2.0), 1 / sqrt(2.0)};
  basis_from_quat(q, t.R);
  t.t[0] = t.t[1] = t.t[2] = 0;
  return t;
}

// Camera intrinsics as the reference sees them: K stored CV_32F
// (get3x3FromVector, QuadDetection.h:189-201) and promoted to double inside
// cv::fisheye; D CV_64F.
struct Cam {
  double fx, fy, cx, cy;
  double k[4];
};

// cv::fisheye::distortPoints on the normalized point (x/z, y/z), alpha = 0
MK_HD void distort(const Cam& cm, double X, double Y, double Z, double* u, double* v) {
  double x = X / Z, y = Y / Z;
  double r2 = x * x + y * y;
  double r = sqrt(r2);  // +0, positive or NaN
#if MK_DM_DEVICE
  const double inv_r0 = 1.0 / r;                // shared by atan's reduction and the 1/r below
  double theta = dm::atan_pos(r, inv_r0);       // ocml atan, op for op (mk_dmath.h)
#else
  const double inv_r0 = 1.0 / r;
  double theta = atan(r);
#endif
  double theta2 = theta * theta, theta3 = theta2 * theta, theta4 = theta2 * theta2, theta5 = theta4 * theta,
         theta6 = theta3 * theta3, theta7 = theta6 * theta, theta8 = theta4 * theta4, theta9 = theta8 * theta;
  double theta_d = theta + cm.k[0] * theta3 + cm.k[1] * theta5 + cm.k[2] * theta7 + cm.k[3] * theta9;
  double inv_r = r > 1e-8 ? inv_r0 : 1;
  double cdist = r > 1e-8 ? theta_d * inv_r : 1;
  double xd0 = x * cdist, xd1 = y * cdist;
  double xd3 = xd0 + 0.0 * xd1;
  *u = xd3 * cm.fx + cm.cx;
  *v = xd1 * cm.fy + cm.cy;
}
#ifdef __HIPCC__
// Filtered fisheye projection for the fast scorers. The scorers consume the
// projection only through decisions: in_frame (thresholds 0, cols, 0, rows)
// and cvRound (ties at k + 1/2). This version replaces the three IEEE
// divisions and the IEEE square root of distort() by the hardware reciprocal
// / reciprocal square root with Newton steps (same operation order
// otherwise); its pixel coordinates differ from distort()'s by ~2e-12 px
// (worst over 2^26 projections: tools/check_proj.hip). It returns whether
// every decision is certain -- a coordinate farther than kProjCert = 1e-7 px
// outside the frame, or both farther than that from the frame edges and
// from the rounding ties -- and the caller recomputes with distort()
// otherwise (~1 landmark in 3 million). r2 >= 1e200 (overflow: distort()
// then takes cdist = theta_d / inf = 0) and NaN are never certain.
// Measured in the PF scorer: 24.4 ms against 23.0 with distort() (the
// scorer waits on its gathers, not its FP64 pipe), so it is off by default
// (kernels.hip MK_FAST_PROJ) and kept, with its checker, for that A/B.
constexpr double kProjCert = 1e-7;
__device__ inline bool proj_in_certain(double a, int lim) {
  const double f = a - floor(a);
  return a > kProjCert && a < (double)lim - kProjCert && fabs(f - 0.5) > kProjCert;
}
__device__ inline bool proj_out_certain(double a, int lim) { return a < -kProjCert || a > (double)lim + kProjCert; }
__device__ inline bool distort_fast(const Cam& cm, double X, double Y, double Z, double* u, double* v, int W, int H) {
  double rz = __builtin_amdgcn_rcp(Z);
  double e = __builtin_fma(-Z, rz, 1.0);
  rz = __builtin_fma(rz, e, rz);
  e = __builtin_fma(-Z, rz, 1.0);
  rz = __builtin_fma(rz, e, rz);
  const double x = X * rz, y = Y * rz;
  const double r2 = x * x + y * y;
  double rs = __builtin_amdgcn_rsq(r2);
  rs = rs * __builtin_fma(-0.5 * r2, rs * rs, 1.5);
  const double r = r2 * rs;
  const double theta = dm::atan_pos(r, rs);
  const double theta2 = theta * theta, theta3 = theta2 * theta, theta4 = theta2 * theta2, theta5 = theta4 * theta,
               theta6 = theta3 * theta3, theta7 = theta6 * theta, theta8 = theta4 * theta4, theta9 = theta8 * theta;
  const double theta_d = theta + cm.k[0] * theta3 + cm.k[1] * theta5 + cm.k[2] * theta7 + cm.k[3] * theta9;
  const double cdist = r > 1e-8 ? theta_d * rs : 1;
  const double uu = (x * cdist) * cm.fx + cm.cx, vv = (y * cdist) * cm.fy + cm.cy;
  *u = uu;
  *v = vv;
  return r2 < 1e200 &&
         (proj_out_certain(uu, W) || proj_out_certain(vv, H) || (proj_in_certain(uu, W) && proj_in_certain(vv, H)));
}
#endif
// cv::fisheye::undistortPoints, no R/P (normalized output), 10 iterations,
// theta_d clamped to [-pi/2, pi/2] (OpenCV 3.3 form)
MK_HD void undistort(const Cam& cm, double px, double py, double* ox, double* oy) {
  double pwx = (px - cm.cx) / cm.fx, pwy = (py - cm.cy) / cm.fy;
  double scale = 1.0;
  double theta_d = sqrt(pwx * pwx + pwy * pwy);
  theta_d = fmin(fmax(-M_PI / 2., theta_d), M_PI / 2.);
  if (theta_d > 1e-8) {
    double theta = theta_d;
    for (int j = 0; j < 10; j++) {
      double theta2 = theta * theta, theta4 = theta2 * theta2, theta6 = theta4 * theta2, theta8 = theta6 * theta2;
      theta = theta_d / (1 + cm.k[0] * theta2 + cm.k[1] * theta4 + cm.k[2] * theta6 + cm.k[3] * theta8);
    }
    scale = tan(theta) / theta_d;
  }
  double pux = pwx * scale, puy = pwy * scale;
  double pr0 = 1.0 * pux + 0.0 * puy + 0.0 * 1.0;
  double pr1 = 0.0 * pux + 1.0 * puy + 0.0 * 1.0;
  double pr2 = 0.0 * pux + 0.0 * puy + 1.0 * 1.0;
  *ox = pr0 / pr2;
  *oy = pr1 / pr2;
}

// cvRound: round half to even (SSE2 cvtsd2si under the default MXCSR)
MK_HD int cv_round(double v) { return (int)rint(v); }

// inFrame (HypothesisEvaluation.h:388-398)
MK_HD bool in_frame(double x, double y, int rows, int cols) { return x < cols && y < rows && x >= 0 && y > 0; }

}  // namespace mk
