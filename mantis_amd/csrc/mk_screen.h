// FP32 screen of the fisheye landmark projection for the fast scorers
// (computePointErrorFAST / evaluateHypothesisWithImageWHITE,
// include/mantis3/HypothesisEvaluation.h:107-158, 218-227; projectPoint +
// distortPixel, include/mantis3/Mantis3Types.h:88-93, 125-136).
//
// The fast scorers consume a landmark's projection only through decisions:
// z > 0, inFrame (u in [0, cols), v in (0, rows), HypothesisEvaluation.h:
// 388-398) and the pixel cvRound(u), cvRound(v) (ties at k + 1/2). The exact
// FP64 projection (mk_math.h distort(), ~110 FP64 + ~100 other VALU
// instructions per landmark, FP64 issuing at half the FP32 rate on gfx950) is
// the same function evaluated in FP64; here it is evaluated in FP32 (~70 VALU
// instructions at full rate and three transcendental ops) together with a
// bound eps on |u_f32 - u_exact| and |v_f32 - v_exact|. A decision is taken
// from the FP32 values only when it cannot flip inside +-eps (a coordinate
// farther than eps outside the frame, or both farther than eps from the frame
// edges and from the rounding ties); otherwise the landmark is "unsure" and
// the caller recomputes it with the exact distort(). Decisions, pixels and
// therefore the integer error sums are identical to the exact path's.
//
// Error model (u = unit roundoff 2^-24; the derivation is in DESIGN.md §4):
//  * camera point p = R X + t by three FMAs per row from R, X, t rounded to
//    FP32: |dp_i| <= ez = 6 u (|X|_1 + |t|_1) per coordinate (|R_ij| <= 1);
//  * the pixel depends on p only through its direction: a direction error of
//    |dp| / |p| rad moves it by at most S px, S = f_max * max over theta in
//    [0, pi/2] of max(theta_d'(theta), theta_d(theta) / sin theta)
//    (ScreenCam.sens carries 2.2 S: sqrt(3) for the three coordinates, the
//    rest margin). S is an upper bound derived by interval subdivision
//    (screen_cam_from), not a sample;
//  * the FP32 evaluation itself: theta = atan2(rho, z) to <= 8 u rad (degree-6
//    minimax polynomial, 4.9e-8 rad, plus the roundings of q = min / max and of
//    pi/2 - atan), charged 16 u * S; the scale theta_d / rho and the products
//    to <= (8 + 9 M) u relative of (u - cx), M = max over theta of
//    (1 + sum |k_i| theta^(2i+2)) / F(theta), F = 1 + sum k_i theta^(2i+2)
//    (Horner with FMAs over theta^2 with one rounding, coefficients rounded to
//    FP32: the cancellation in F is what M measures), charged
//    crel = max(24, 1.25 (8 + 9 M)) u |u - cx|; the final add 0.5 u |u|,
//    charged 2 u |u| <= 2 u (|u - cx| + |cx|): with the constant parts folded
//    (round 5) eps = sens ez / |p| + (crel + 2u)(|du| + |dv|) + 16u sens +
//    2u (|cx| + |cy|), five operations.
#pragma once
#include <cmath>
#include <cstdint>

#include "mk_math.h"

namespace mk {

struct ScreenCam {
  float fx, fy, cx, cy;
  float k[4];
  float sens;   // 2.2 * S px per radian (see above); +inf disables the screen (every landmark unsure)
  float crel;   // relative error charge of the scale chain, max(24, 1.25 (8 + 9 M)) u (see above)
  // the bound's constant parts folded (round 5): |u| <= |du| + |cx| turns
  // crel (|du| + |dv|) + 2u (|u| + |v|) + sens 16u into
  // c2 (|du| + |dv|) + e0, with c2 = crel + 2u and e0 = sens 16u + 2u (|cx| + |cy|), both rounded up
  float c2, e0;
};
struct PoseF {   // c2w as FP32: rows of R, t, and 6u |t|_1 (the pose's part of the camera-point bound ez)
  float R[9];
  float t[3];
  float tn;
  float pad[3];
};

constexpr float kScrU = 5.9604644775390625e-8f;  // 2^-24
enum { SCR_OUT = 0, SCR_IN = 1, SCR_UNSURE = 2 };

MK_HD PoseF posef_from(const Xf& T) {
  PoseF p;
  for (int k = 0; k < 9; k++) p.R[k] = (float)T.R[k];
  for (int k = 0; k < 3; k++) p.t[k] = (float)T.t[k];
  p.tn = (float)((fabs(T.t[0]) + fabs(T.t[1]) + fabs(T.t[2])) * (6.0 * 5.9604644775390625e-8) * 1.000001);
  p.pad[0] = p.pad[1] = p.pad[2] = 0.f;
  return p;
}

#if defined(__HIPCC__) && defined(__HIP_DEVICE_COMPILE__)
__device__ inline float scr_rsq(float x) { return __builtin_amdgcn_rsqf(x); }
__device__ inline float scr_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
#else
MK_HD float scr_rsq(float x) { return 1.0f / sqrtf(x); }
MK_HD float scr_rcp(float x) { return 1.0f / x; }
#endif

// atan(q), q in [0, 1]: q + q s P(s), s = q^2, degree-6 P (|error| <= 4.9e-8)
MK_HD float scr_atan01(float q) {
  const float s = q * q;
  float p = fmaf(s, -0.004355372798310124f, 0.02304001704877514f);
  p = fmaf(s, p, -0.05777342045816491f);
  p = fmaf(s, p, 0.09794222509993752f);
  p = fmaf(s, p, -0.13976577679543017f);
  p = fmaf(s, p, 0.19962703195997453f);
  p = fmaf(s, p, -0.3333165898332249f);
  return fmaf(q * s, p, q);
}

// FP32 pixel coordinates of landmark (X, Y, Z) with xn = |X|_1 under pose P,
// with their error bound: state 0 = certainly z <= 0, 2 = unsure (z near 0 or
// on the optical axis), 1 = u, v, eps valid.
struct ScrUV {
  float u, v, eps;
  int state;
};
MK_HD ScrUV screen_uv(const PoseF& P, float X, float Y, float Z, float xn, const ScreenCam& c) {
  ScrUV r;
  r.u = r.v = r.eps = 0.f;
  const float x = fmaf(P.R[0], X, fmaf(P.R[1], Y, fmaf(P.R[2], Z, P.t[0])));
  const float y = fmaf(P.R[3], X, fmaf(P.R[4], Y, fmaf(P.R[5], Z, P.t[1])));
  const float z = fmaf(P.R[6], X, fmaf(P.R[7], Y, fmaf(P.R[8], Z, P.t[2])));
  const float ez = xn + P.tn;  // 6u (|X|_1 + |t|_1), both parts pre-scaled (screen_landmark, posef_from)
  if (!(z > ez)) {
    r.state = z < -ez ? 0 : 2;
    return r;
  }
  const float rho2 = fmaf(x, x, y * y);
  if (!(rho2 > 1e-12f * (z * z))) {  // on the optical axis (distort()'s r <= 1e-8 branch)
    r.state = 2;
    return r;
  }
  const float rinv = scr_rsq(fmaf(z, z, rho2));  // 1 / |p|
  const float irho = scr_rsq(rho2);
  const float rho = rho2 * irho;
  const bool wide = rho > z;  // theta > pi/4
  const float q = (wide ? z : rho) * scr_rcp(wide ? rho : z);
  const float a = scr_atan01(q);
  const float th = wide ? 1.57079632679489662f - a : a;
  const float t2 = th * th;
  const float thd = th * fmaf(t2, fmaf(t2, fmaf(t2, fmaf(t2, c.k[3], c.k[2]), c.k[1]), c.k[0]), 1.0f);
  const float sc = thd * irho;
  const float du = c.fx * (x * sc), dv = c.fy * (y * sc);
  r.u = du + c.cx;
  r.v = dv + c.cy;
  r.eps = fmaf(c.sens * ez, rinv, fmaf(c.c2, fabsf(du) + fabsf(dv), c.e0));
  r.state = 1;
  return r;
}

// Screen landmark (X, Y, Z) with xn = |X|_1 under pose P. SCR_IN: in frame,
// pixel (*px, *py) = (cvRound(u), cvRound(v)) exactly as distort() + cv_round
// give, and an interior pixel (1 <= px < W, 1 <= py < H: the linear offset
// py * W + px is the pixel itself); SCR_OUT: z <= 0 or outside the frame;
// SCR_UNSURE: recompute exactly (near a rounding tie, z ~ 0, the optical axis,
// or a pixel on the frame's first / last row or column, where inFrame and the
// linear offset need the exact value).
// Branch-free (screen_uv's early outs become predicates) and the range tests
// on the rounded pixel: with |d| = |u - rint(u)| < 1/2 - eps the exact u
// rounds to the same px, and px in [1, W - 1] puts u in (1/2, W - 1/2), inside
// [0, W); px < 0 or px > W puts u farther than 1/2 > eps outside.
MK_HD int screen_project(const PoseF& P, float X, float Y, float Z, float xn, const ScreenCam& c, int W, int H,
                         int* px, int* py) {
  const float x = fmaf(P.R[0], X, fmaf(P.R[1], Y, fmaf(P.R[2], Z, P.t[0])));
  const float y = fmaf(P.R[3], X, fmaf(P.R[4], Y, fmaf(P.R[5], Z, P.t[1])));
  const float z = fmaf(P.R[6], X, fmaf(P.R[7], Y, fmaf(P.R[8], Z, P.t[2])));
  const float ez = xn + P.tn;  // 6u (|X|_1 + |t|_1), both parts pre-scaled (screen_landmark, posef_from)
  const float rho2 = fmaf(x, x, y * y);
  const float z2 = z * z;
  const float irho = scr_rsq(rho2);
  const float rho = rho2 * irho;
  const bool wide = rho > z;
  // 1 / max(rho, z) >= 1 / |p| (|p| <= sqrt(2) max): the bound's 1 / |p| without
  // a third transcendental (round 5; the eps term it scales grows by <= sqrt(2))
  const float rinv = scr_rcp(wide ? rho : z);
  const float q = (wide ? z : rho) * rinv;
  const float a = scr_atan01(q);
  const float th = wide ? 1.57079632679489662f - a : a;
  const float t2 = th * th;
  const float thd = th * fmaf(t2, fmaf(t2, fmaf(t2, fmaf(t2, c.k[3], c.k[2]), c.k[1]), c.k[0]), 1.0f);
  const float sc = thd * irho;
  const float du = c.fx * (x * sc), dv = c.fy * (y * sc);
  const float u = du + c.cx, v = dv + c.cy;
  const float eps = fmaf(c.sens * ez, rinv, fmaf(c.c2, fabsf(du) + fabsf(dv), c.e0));
  // z certainly > 0, off the optical axis, and a bound below 1/4 px: the FP32
  // values are meaningful (NaN / inf fail every comparison)
  const bool valid = (int)(z > ez) & (int)(rho2 > 1e-12f * z2) & (int)(eps < 0.25f);
#if defined(__HIP_DEVICE_COMPILE__)
  // v_cvt_i32_f32 is defined for every input (NaN -> 0, out of range saturates);
  // a value that is not `valid` decides nothing below. Emitted as the
  // instruction itself: a C++ float -> int conversion of an
  // out-of-range value is poison in LLVM IR, which a compiler may fold into
  // anything, `valid & ...` included
  const float ru = rintf(u), rv = rintf(v);
  int iu, iv;
  asm("v_cvt_i32_f32 %0, %1" : "=v"(iu) : "v"(ru));
  asm("v_cvt_i32_f32 %0, %1" : "=v"(iv) : "v"(rv));
#else
  const float ru = rintf(valid ? u : 0.f), rv = rintf(valid ? v : 0.f);  // (int) of NaN / huge is UB on the host
  const int iu = (int)ru, iv = (int)rv;
#endif
  const bool round_ok = (int)(fabsf(u - ru) < 0.5f - eps) & (int)(fabsf(v - rv) < 0.5f - eps);
  const bool interior = (int)((unsigned)(iu - 1) < (unsigned)(W - 1)) & (int)((unsigned)(iv - 1) < (unsigned)(H - 1));
  const bool outside = (int)((unsigned)iu > (unsigned)W) | (int)((unsigned)iv > (unsigned)H);
  const bool sure = (int)valid & (int)round_ok & (int)interior;
  const bool out = (int)(z < -ez) | ((int)valid & (int)outside);
  *px = iu;
  *py = iv;
  return sure ? SCR_IN : (out ? SCR_OUT : SCR_UNSURE);
}

// landmark as the screen reads it: FP32 coordinates and 6u |X|_1 rounded up
// (the landmark's part of the camera-point bound ez)
MK_HD void screen_landmark(const double* X, float* o) {
  o[0] = (float)X[0];
  o[1] = (float)X[1];
  o[2] = (float)X[2];
  o[3] = (float)((fabs(X[0]) + fabs(X[1]) + fabs(X[2])) * (6.0 * 5.9604644775390625e-8) * 1.000001);
}

// Host: the screen constants of a camera, from bounds derived over [0, pi/2]
// by interval subdivision. On a piece theta in [a, b], x = theta^2 in
// [a^2, b^2]: every term c x^j of theta_d'(theta) = 1 + sum (2i+3) k_i x^(i+1),
// of F(theta) = 1 + sum k_i x^(i+1) and of A(theta) = sum |k_i| x^(i+1) is
// monotone in x >= 0, so the sum of the per-term maxima (minima) over the
// piece's ends bounds the polynomial from above (below) on the whole piece;
// theta / sin theta is increasing, so b / sin b bounds it. Then
//   S >= max(theta_d', theta_d / sin theta)  (upper bounds of both per piece),
//   M >= (1 + A) / F                           (upper bound of 1 + A over the
//                                              lower bound of F per piece),
// and the model needs theta_d increasing and positive: a piece whose lower
// bound of theta_d' or of F is not > 0 disables the screen (sens = inf: every
// landmark takes the exact path). The double arithmetic of the bounds is
// covered by a 1e-9 relative margin.
struct ScreenBounds {
  double S, M;  // S per unit focal length; M as above
  bool ok;
};
MK_HD ScreenBounds screen_bounds(const double* k, int pieces = 4096) {
  ScreenBounds r{1.0, 1.0, true};
  const double half_pi = 1.5707963267948966;
  for (int i = 0; i < pieces; i++) {
    const double a = half_pi * i / pieces, b = fmin(half_pi, half_pi * (i + 1) / pieces * (1 + 1e-15));
    const double xa = a * a, xb = b * b;
    double dhi = 1, dlo = 1, Fhi = 1, Flo = 1, Ahi = 0, pa = xa, pb = xb;
    for (int j = 0; j < 4; j++) {
      const double ta = k[j] * pa, tb = k[j] * pb;
      const double mx = fmax(ta, tb), mn = fmin(ta, tb);
      dhi += (2 * j + 3) * mx;
      dlo += (2 * j + 3) * mn;
      Fhi += mx;
      Flo += mn;
      Ahi += fmax(fabs(ta), fabs(tb));
      pa *= xa;
      pb *= xb;
    }
    if (!(dlo > 0) || !(Flo > 0)) r.ok = false;  // also false for NaN
    const double ratio = b / sin(b);
    r.S = fmax(r.S, fmax(dhi, ratio * Fhi));
    r.M = fmax(r.M, (1 + Ahi) / Flo);
  }
  r.S *= 1 + 1e-9;
  r.M *= 1 + 1e-9;
  return r;
}
MK_HD ScreenCam screen_cam_from(const Cam& cm) {
  ScreenCam s;
  s.fx = (float)cm.fx; s.fy = (float)cm.fy; s.cx = (float)cm.cx; s.cy = (float)cm.cy;
  for (int k = 0; k < 4; k++) s.k[k] = (float)cm.k[k];
  bool ok = cm.fx > 0 && cm.fy > 0 && cm.fx < 1e30 && cm.fy < 1e30;  // also false for NaN
  // the fp32 coefficients must reproduce theta_d closely: |k| bounded
  for (int k = 0; k < 4; k++) ok = ok && fabs(cm.k[k]) < 1.0;
  const ScreenBounds b = ok ? screen_bounds(cm.k) : ScreenBounds{1.0, 1.0, false};
  ok = ok && b.ok && b.M < 1e4;
  const double f = fmax(cm.fx, cm.fy);
  s.sens = ok ? (float)(2.2 * b.S * f) : INFINITY;
  s.crel = (float)(fmax(24.0, 1.25 * (8.0 + 9.0 * b.M)) * 5.9604644775390625e-8);
  const double u = 5.9604644775390625e-8;
  s.c2 = (float)(((double)s.crel + 2 * u) * 1.000001);
  s.e0 = ok ? (float)((16 * u * (double)s.sens + 2 * u * (fabs((double)s.cx) + fabs((double)s.cy))) * 1.000001)
            : INFINITY;
  return s;
}

}  // namespace mk
