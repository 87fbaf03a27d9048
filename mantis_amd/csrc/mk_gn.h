// Gauss–Newton pose refinement (new stage): the pieces
// shared by the HIP kernels (gn_impl.hip) and the host build used by the CPU
// tests (hostcheck.cpp).
//
// Residuals: r = pi(p) - u with p = R_cb inv(T_w_b) X + t_cb the world point X
// in camera c, u the observed normalized (undistorted) image point and
// pi(p) = (p_x/p_z, p_y/p_z). Right perturbation T_w_b <- T_w_b Exp(delta),
// delta = (rho, phi): dp/d(delta) = R_cb [ -I | [q]x ], q = inv(T_w_b) X.
// The 28 accumulated doubles are the upper triangle of J^T J (21), J^T r (6)
// and r^T r (1), i.e. entries of M^T M for M = [J | r].
//
// Two uses:
//  * rig GN (per rig after the fusion, configs 3/4): correspondences of quad
//    centres to grid-cell centres over all cameras (gn_quad_obs), camera
//    extrinsics T_base_cam;
//  * per-quad GN after RPP (quad_gn_refine): the quad's 4 corners to the
//    model square the reference fits with RPP (CoPlanarPoseEstimator.cpp:
//    16-58, model points +-GRID_SPACING/2), one camera with identity
//    extrinsics, the legacy cv::solvePnP ITERATIVE analogue
//    (include/legacy/mantis2/PoseEstimator.h:91-153, :103).
#pragma once
#include <cmath>

#include "mk_math.h"
#include "mk_types.h"

namespace mk {

// value of M[row][col] (col 0..5 = J, 6 = r, else 0) for residual row `row`
// (observation row >> 1, component row & 1); obs rows = [cam, u, v, X, Y, Z]
MK_HD double gn_entry(const double* Rwb_t, const double* twb, const GnCam* cams, const double* obs, int n_obs,
                      int row, int col) {
  if (col > 6) return 0.0;
  int i = row >> 1, comp = row & 1;
  if (i >= n_obs) return 0.0;
  const double* o = obs + 6 * (size_t)i;
  const GnCam& cm = cams[(int)o[0]];
  // q = inv(T_w_b) X = R_wb^T (X - t_wb)
  double d[3] = {o[3] - twb[0], o[4] - twb[1], o[5] - twb[2]};
  double q[3];
  for (int a = 0; a < 3; a++) q[a] = Rwb_t[3 * a] * d[0] + Rwb_t[3 * a + 1] * d[1] + Rwb_t[3 * a + 2] * d[2];
  double p[3];
  for (int a = 0; a < 3; a++)
    p[a] = cm.R_cb[3 * a] * q[0] + cm.R_cb[3 * a + 1] * q[1] + cm.R_cb[3 * a + 2] * q[2] + cm.t_cb[a];
  double iz = 1.0 / p[2];
  if (col == 6) return (comp == 0 ? p[0] : p[1]) * iz - (comp == 0 ? o[1] : o[2]);
  // dpi/dp row
  double g[3];
  if (comp == 0) { g[0] = iz; g[1] = 0; g[2] = -p[0] * iz * iz; }
  else { g[0] = 0; g[1] = iz; g[2] = -p[1] * iz * iz; }
  // h = g^T R_cb (1x3)
  double h[3];
  for (int b = 0; b < 3; b++) h[b] = g[0] * cm.R_cb[b] + g[1] * cm.R_cb[3 + b] + g[2] * cm.R_cb[6 + b];
  if (col < 3) return -h[col];
  // h [q]x column: [q]x = [[0,-qz,qy],[qz,0,-qx],[-qy,qx,0]]
  int k = col - 3;
  if (k == 0) return h[1] * q[2] - h[2] * q[1];
  if (k == 1) return -h[0] * q[2] + h[2] * q[0];
  return h[0] * q[1] - h[1] * q[0];
}

// the 28 accumulators of n_obs observations, rows summed in order (one lane)
MK_HD void gn_accumulate_seq(const double* Twb, const GnCam* cams, const double* obs, int n_obs, double* acc28) {
  double Rt[9], t[3];
  for (int a = 0; a < 3; a++) {
    for (int b = 0; b < 3; b++) Rt[3 * a + b] = Twb[4 * b + a];
    t[a] = Twb[4 * a + 3];
  }
  for (int e = 0; e < 28; e++) acc28[e] = 0.0;
  for (int row = 0; row < 2 * n_obs; row++) {
    double v[7];
    for (int col = 0; col < 7; col++) v[col] = gn_entry(Rt, t, cams, obs, n_obs, row, col);
    int n = 0;
    for (int a = 0; a < 6; a++)
      for (int b = a; b < 6; b++) acc28[n++] += v[a] * v[b];
    for (int a = 0; a < 6; a++) acc28[21 + a] += v[a] * v[6];
    acc28[27] += v[6] * v[6];
  }
}

// (J^T J + lambda I) delta = -J^T r from the 28 accumulators by Cholesky, then
// T_w_b <- T_w_b Exp(delta) (right perturbation: translation delta[0..2],
// rotation vector delta[3..5] through Rodrigues). Returns false when the
// normal matrix is not positive definite (too few observations).
MK_HD bool gn_solve6(const double* acc28, double lambda, double* T_w_b, double* delta6) {
  double A[6][6], b[6];
  int n = 0;
  for (int i = 0; i < 6; i++)
    for (int j = i; j < 6; j++) { A[i][j] = A[j][i] = acc28[n++]; }
  for (int i = 0; i < 6; i++) { A[i][i] += lambda; b[i] = -acc28[21 + i]; }
  double L[6][6];
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 6; j++) L[i][j] = 0;
  for (int i = 0; i < 6; i++)
    for (int j = 0; j <= i; j++) {
      double s = A[i][j];
      for (int k = 0; k < j; k++) s -= L[i][k] * L[j][k];
      if (i == j) {
        if (!(s > 0)) return false;
        L[i][i] = sqrt(s);
      } else {
        L[i][j] = s / L[j][j];
      }
    }
  double y[6], x[6];
  for (int i = 0; i < 6; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s -= L[i][k] * y[k];
    y[i] = s / L[i][i];
  }
  for (int i = 5; i >= 0; i--) {
    double s = y[i];
    for (int k = i + 1; k < 6; k++) s -= L[k][i] * x[k];
    x[i] = s / L[i][i];
  }
  if (delta6)
    for (int i = 0; i < 6; i++) delta6[i] = x[i];
  const double* w = x + 3;
  const double th = sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  const double K[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
  double a, bb;
  if (th < 1e-12) { a = 1.0; bb = 0.5; }
  else { a = sin(th) / th; bb = (1 - cos(th)) / (th * th); }
  double dR[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += K[i * 3 + k] * K[k * 3 + j];
      dR[i * 3 + j] = (i == j ? 1.0 : 0.0) + a * K[i * 3 + j] + bb * s;
    }
  const double D[16] = {dR[0], dR[1], dR[2], x[0], dR[3], dR[4], dR[5], x[1], dR[6], dR[7], dR[8], x[2], 0, 0, 0, 1};
  double r[16];
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      double s = 0;
      for (int k = 0; k < 4; k++) s += T_w_b[i * 4 + k] * D[k * 4 + j];
      r[i * 4 + j] = s;
    }
  for (int i = 0; i < 16; i++) T_w_b[i] = r[i];
  return true;
}

// Rig GN correspondence of one detected quad. A detected quad is the dark
// inside of one grid cell, so its centre is the cell centre; in the
// undistorted normalized image (a perspective view) the centre of the square
// is exactly where the quad's diagonals cross. That point, back-projected with
// the camera pose (Rwc, centre Cw) onto the floor and snapped to the nearest
// cell centre (-half + spacing (k + 1/2); accepted within 0.1 m), gives one
// observation o[1..5] = (u, v, X, Y, 0).
MK_HD bool gn_quad_obs(const Cam& cam, const int32_t* qc, const double* Rwc, const double* Cw, double half,
                       double spacing, double* o) {
  double u[4], v[4];
  for (int k = 0; k < 4; k++) undistort(cam, (double)qc[2 * k], (double)qc[2 * k + 1], &u[k], &v[k]);
  // diagonals p0-p2 and p1-p3: p0 + a (p2 - p0) = p1 + b (p3 - p1)
  const double d1x = u[2] - u[0], d1y = v[2] - v[0], d2x = u[3] - u[1], d2y = v[3] - v[1];
  const double den = d1x * d2y - d1y * d2x;
  if (fabs(den) < 1e-12) return false;
  const double a = ((u[1] - u[0]) * d2y - (v[1] - v[0]) * d2x) / den;
  if (!(a > 0 && a < 1)) return false;
  const double uc = u[0] + a * d1x, vc = v[0] + a * d1y;
  const double dw[3] = {Rwc[0] * uc + Rwc[1] * vc + Rwc[2], Rwc[3] * uc + Rwc[4] * vc + Rwc[5],
                        Rwc[6] * uc + Rwc[7] * vc + Rwc[8]};
  if (!(dw[2] < -1e-9)) return false;
  const double tt = -Cw[2] / dw[2];
  if (!(tt > 0)) return false;
  const double X = Cw[0] + tt * dw[0], Y = Cw[1] + tt * dw[1];
  const double c0 = -half + 0.5 * spacing;  // first cell centre
  const double kx = rint((X - c0) / spacing), ky = rint((Y - c0) / spacing);
  const double lim = rint(2 * half / spacing) - 1;
  if (kx < 0 || ky < 0 || kx > lim || ky > lim) return false;
  const double gx = c0 + spacing * kx, gy = c0 + spacing * ky;
  if (fabs(X - gx) > 0.1 || fabs(Y - gy) > 0.1) return false;
  o[1] = uc;
  o[2] = vc;
  o[3] = gx;
  o[4] = gy;
  o[5] = 0.0;
  return true;
}

// Per-quad GN after RPP: refine the pose R, t (model -> camera, the c2w
// naming of CoPlanarPoseEstimator.cpp:53-56) of one quad from its 4
// normalized image points img (4 x 2) and model points obj (4 x 3), starting
// from RPP's answer. The pose is held as T_w_b = inv([R | t]) (the camera in
// the model frame) with identity extrinsics, so the rows are gn_entry's.
// Stops after `iters` steps, when the step norm^2 < 1e-24 or when the normal
// matrix is singular (pose kept). Returns the steps taken; cost0 / cost =
// r^T r before / after.
MK_HD int quad_gn_refine(double* R, double* t, const double* img, const double* obj, int iters, double* cost0,
                         double* cost) {
  GnCam cam;
  for (int e = 0; e < 9; e++) cam.R_cb[e] = (e % 4 == 0) ? 1.0 : 0.0;
  cam.t_cb[0] = cam.t_cb[1] = cam.t_cb[2] = 0.0;
  double obs[24];
  for (int k = 0; k < 4; k++) {
    obs[6 * k] = 0.0;
    obs[6 * k + 1] = img[2 * k];
    obs[6 * k + 2] = img[2 * k + 1];
    for (int a = 0; a < 3; a++) obs[6 * k + 3 + a] = obj[3 * k + a];
  }
  double T[16];  // inv([R | t])
  for (int a = 0; a < 3; a++) {
    for (int b = 0; b < 3; b++) T[4 * a + b] = R[3 * b + a];
    T[4 * a + 3] = -(R[a] * t[0] + R[3 + a] * t[1] + R[6 + a] * t[2]);
  }
  T[12] = T[13] = T[14] = 0.0;
  T[15] = 1.0;
  double acc[28];
  gn_accumulate_seq(T, &cam, obs, 4, acc);
  *cost0 = acc[27];
  int it = 0;
  for (; it < iters; it++) {
    double Tn[16], d6[6];
    for (int e = 0; e < 16; e++) Tn[e] = T[e];
    if (!gn_solve6(acc, 1e-9, Tn, d6)) break;
    double acc_n[28];
    gn_accumulate_seq(Tn, &cam, obs, 4, acc_n);
    if (!(acc_n[27] <= acc[27])) break;  // no decrease: keep the previous pose
    for (int e = 0; e < 16; e++) T[e] = Tn[e];
    for (int e = 0; e < 28; e++) acc[e] = acc_n[e];
    double dn = 0;
    for (int e = 0; e < 6; e++) dn += d6[e] * d6[e];
    if (dn < 1e-24) { it++; break; }
  }
  *cost = acc[27];
  for (int a = 0; a < 3; a++) {
    for (int b = 0; b < 3; b++) R[3 * a + b] = T[4 * b + a];
    t[a] = -(T[a] * T[3] + T[4 + a] * T[7] + T[8 + a] * T[11]);
  }
  return it;
}

}  // namespace mk
