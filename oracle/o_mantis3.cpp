// ORACLE — test infrastructure only. Never linked into the product path.
//
// CPU restatement of the mantis3 per-frame callback and its stages:
//   quadDetection                     src/mantis3.cpp:68-135
//   Quadrilateral / removeDuplicate   include/mantis3/QuadDetection.h:13-66, 115-171
//   detectQuadrilaterals              include/mantis3/QuadDetection.h:203-287
//   undistortAndNormalize...          include/mantis3/QuadDetection.h:289-298
//   generate(Central)Hypotheses       include/mantis3/HypothesisGeneration.h:23-109
//   computeAllShiftedHypothesesFAST   include/mantis3/HypothesisGeneration.h:111-140
//   PoseClusterer BFcluster           include/mantis3/PoseClusterer.cpp:33-116, PoseClusterer.h:59-115
//   evaluate* / computePointError     include/mantis3/HypothesisEvaluation.h:23-275, 388-398
//   cleanImageByEdge                  include/mantis3/HypothesisEvaluation.h:319-386
//   getBestNHypotheses                include/mantis3/HypothesisEvaluation.h:484-518
//   determineBestYaw                  include/mantis3/HypothesisEvaluation.h:521-581
//   optimizeHypothesisWithParticleFilter include/mantis3/PoseAdjustment.h:13-60
//   publishPose                       include/mantis3/PosePub.h:12-61
//   parseCoordinatesFromString        include/mantis3/Mantis3Params.h:125-152
//   projectPoint / distortPixel       include/mantis3/Mantis3Types.h:88-136 (+ cv::fisheye [3P])
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "o_cvrng.hpp"
#include "o_imgproc.hpp"
#include "o_rpp.hpp"
#include "o_tf.hpp"
#include "oracle.h"

using namespace orc;

namespace {

constexpr double QUAD_STRETCH = 1.3;        // Mantis3Params.h:20
constexpr int GRID_SIZE = 9;                // :23
constexpr double GRID_SPACING = 0.32;       // :24
constexpr double MAX_QUAD_ERROR = 0.5;      // :26
constexpr double MAX_ANGLE_DIFF = 0.2;      // :28
constexpr double PROJ_BIAS = 1.1;           // :37, :55
constexpr double ROT_SIGMA = 0.03, TRANS_SIGMA = 0.01;  // :62-63
constexpr double MIN_YAW_DIFF = 4000;       // :67
constexpr double VAR_COEFF = 1.0 / 600.0;   // :68
constexpr int CANNY_LOW = 50;               // :162
constexpr int POLY_EPS = 10;                // :164
constexpr double SEARCH_MULT = 0.1;         // :166

struct Cam {
  double fx, fy, cx, cy;  // float K promoted (get3x3FromVector -> CV_32F)
  double k[4];
};
Cam make_cam(const double* K, const double* D) {
  Cam c;
  c.fx = (double)(float)K[0];
  c.fy = (double)(float)K[4];
  c.cx = (double)(float)K[2];
  c.cy = (double)(float)K[5];
  for (int i = 0; i < 4; i++) c.k[i] = D[i];
  return c;
}

// cv::fisheye::distortPoints for one normalized point (alpha = 0)
void distort_norm(const Cam& cm, double x, double y, double& u, double& v) {
  double r2 = x * x + y * y;
  double r = std::sqrt(r2);
  double theta = std::atan(r);
  double theta2 = theta * theta, theta3 = theta2 * theta, theta4 = theta2 * theta2, theta5 = theta4 * theta,
         theta6 = theta3 * theta3, theta7 = theta6 * theta, theta8 = theta4 * theta4, theta9 = theta8 * theta;
  double theta_d = theta + cm.k[0] * theta3 + cm.k[1] * theta5 + cm.k[2] * theta7 + cm.k[3] * theta9;
  double inv_r = r > 1e-8 ? 1.0 / r : 1;
  double cdist = r > 1e-8 ? theta_d * inv_r : 1;
  double xd0 = x * cdist, xd1 = y * cdist;
  double xd3 = xd0 + 0.0 * xd1;
  u = xd3 * cm.fx + cm.cx;
  v = xd1 * cm.fy + cm.cy;
}
// distortPixel(reproj) = distort(normalizePoint(reproj))
void distort_cam(const Cam& cm, const Vec3& p, double& u, double& v) {
  distort_norm(cm, p.x() / p.z(), p.y() / p.z(), u, v);
}
// cv::fisheye::undistortPoints, no R/P (normalized output); 10 fixed
// iterations, theta_d clamped to [-pi/2, pi/2] (OpenCV 3.3 form, [3P]).
void undistort_px(const Cam& cm, double px, double py, double& ox, double& oy) {
  double pwx = (px - cm.cx) / cm.fx, pwy = (py - cm.cy) / cm.fy;
  double scale = 1.0;
  double theta_d = std::sqrt(pwx * pwx + pwy * pwy);
  theta_d = std::min(std::max(-M_PI / 2., theta_d), M_PI / 2.);
  if (theta_d > 1e-8) {
    double theta = theta_d;
    for (int j = 0; j < 10; j++) {
      double theta2 = theta * theta, theta4 = theta2 * theta2, theta6 = theta4 * theta2, theta8 = theta6 * theta2;
      theta = theta_d / (1 + cm.k[0] * theta2 + cm.k[1] * theta4 + cm.k[2] * theta6 + cm.k[3] * theta8);
    }
    scale = std::tan(theta) / theta_d;
  }
  double pux = pwx * scale, puy = pwy * scale;
  // RR = I: pr = (1*pux + 0*puy + 0*1, 0*pux + 1*puy + 0*1, 0*pux + 0*puy + 1*1); fi = pr01 / pr2
  double pr0 = 1.0 * pux + 0.0 * puy + 0.0 * 1.0;
  double pr1 = 0.0 * pux + 1.0 * puy + 0.0 * 1.0;
  double pr2 = 0.0 * pux + 0.0 * puy + 1.0 * 1.0;
  ox = pr0 / pr2;
  oy = pr1 / pr2;
}

inline int cv_round(double v) { return (int)std::nearbyint(v); }

// BGR view with the defined out-of-buffer behaviour: pixel (x,y)
// lives at linear byte offset y*3W + 3x; offsets outside [0, 3WH) read 0.
struct View {
  const uint8_t* d;
  int w, h;
  inline void px(int x, int y, int& b, int& g, int& r) const {
    long off = (long)y * 3 * w + 3L * x;
    if (off < 0 || off + 2 >= 3L * w * h) { b = g = r = 0; return; }
    b = d[off]; g = d[off + 1]; r = d[off + 2];
  }
};
inline bool in_frame(double x, double y, int rows, int cols) { return x < cols && y < rows && x >= 0 && y > 0; }
inline int color_err(int b, int g, int r, int db, int dg, int dr) {
  int e0 = b - db, e1 = g - dg, e2 = r - dr;
  return e0 * e0 + e1 * e1 + e2 * e2;
}

struct Map {
  std::vector<Vec3> white, red, green;
};

// evaluateHypothesisWithImageWHITE (all three sets vs WHITE, fast path)
double eval_fast(const Hypothesis& h, const View& img, const Cam& cm, const Map& m, int& n) {
  double error = 0;
  n = 0;
  const std::vector<Vec3>* sets[3] = {&m.white, &m.red, &m.green};
  for (int s = 0; s < 3; s++)
    for (const Vec3& X : *sets[s]) {
      Vec3 rp = h.c2w(X);
      if (rp.z() > 0) {
        double u, v;
        distort_cam(cm, rp, u, v);
        if (in_frame(u, v, img.h, img.w)) {
          n++;
          int b, g, r;
          img.px(cv_round(u), cv_round(v), b, g, r);
          error += (double)color_err(b, g, r, 255, 255, 255);
        }
      }
    }
  return error;
}
double eval_hyp_fast(const Hypothesis& h, const View& img, const Cam& cm, const Map& m, int* nout = nullptr) {
  int n;
  double e = eval_fast(h, img, cm, m, n);
  if (nout) *nout = n;
  if (n <= 0) return DBL_MAX;
  return e / ((double)n * PROJ_BIAS);
}
// evaluateHypothesisCOLOR, GREEN_ONLY, 10x10 window (slow path)
double eval_hyp_color(const Hypothesis& h, const View& img, const Cam& cm, const Map& m, int* nout = nullptr) {
  double error = 0;
  int n = 0;
  for (const Vec3& X : m.green) {
    Vec3 rp = h.c2w(X);
    if (rp.z() > 0) {
      double u, v;
      distort_cam(cm, rp, u, v);
      if (in_frame(u, v, img.h, img.w)) {
        n++;
        double err = 0;
        for (double ox = -5.0; ox < 5.0; ox += 1)
          for (double oy = -5.0; oy < 5.0; oy += 1) {
            int b, g, r;
            img.px(cv_round(u + ox), cv_round(v + oy), b, g, r);
            err += (double)color_err(b, g, r, 50, 255, 85);
          }
        err /= (double)(10 * 10);
        error += err;
      }
    }
  }
  if (nout) *nout = n;
  if (n <= 0) return DBL_MAX;
  return error / ((double)n * PROJ_BIAS);
}

std::vector<Hypothesis> best_n(int n, std::vector<Hypothesis> hyps) {
  if ((int)hyps.size() <= n) return hyps;
  std::sort(hyps.begin(), hyps.end(), [](const Hypothesis& i, const Hypothesis& j) { return j.error < i.error; });
  return std::vector<Hypothesis>(hyps.end() - n, hyps.end());
}

const Transform& rot_z() {
  static Transform t(Quat(0, 0, 1 / std::sqrt(2), 1 / std::sqrt(2)));
  return t;
}

struct Quad {
  Pt c[4];
  float cx, cy;
  double side;
  double tp[4][2];
  bool neighbor = false;
};
Quad make_quad(const Contour& a) {
  Quad q;
  for (int i = 0; i < 4; i++) q.c[i] = a[i];
  int dx = a[0].x - a[1].x, dy = a[0].y - a[1].y;
  q.side = std::sqrt((double)(dx * dx + dy * dy));
  float xs = 0, ys = 0;
  for (int i = 0; i < 4; i++) { xs += (float)a[i].x; ys += (float)a[i].y; }
  q.cx = xs / (float)4;
  q.cy = ys / (float)4;
  for (int i = 0; i < 4; i++) {
    float dxf = (float)a[i].x - q.cx, dyf = (float)a[i].y - q.cy;
    float sx = (float)(dxf * QUAD_STRETCH), sy = (float)(dyf * QUAD_STRETCH);
    q.tp[i][0] = (double)(sx + q.cx);
    q.tp[i][1] = (double)(sy + q.cy);
  }
  return q;
}

// removeDuplicateQuads with FLANN radiusSearch semantics made exact:
// squared float distance <= (float)radius, results sorted by (dist, index),
// the 4-slot index vector zero-padded (quad 0 marked when < 4 hits).
void remove_duplicates(std::vector<Quad>& qs) {
  const int n = (int)qs.size();
  for (int i = 0; i < n; i++) {
    if (qs[i].neighbor) continue;
    float radius = (float)(SEARCH_MULT * qs[i].side);
    std::vector<std::pair<float, int>> hits;
    for (int j = 0; j < n; j++) {
      float d0 = qs[j].cx - qs[i].cx, d1 = qs[j].cy - qs[i].cy;
      float dist = 0.0f;
      dist += d0 * d0;
      dist += d1 * d1;
      if (dist <= radius) hits.push_back({dist, j});
    }
    std::sort(hits.begin(), hits.end());
    int idx[4] = {0, 0, 0, 0};
    for (int k = 0; k < 4 && k < (int)hits.size(); k++) idx[k] = hits[k].second;
    for (int k = 1; k < 4; k++) qs[idx[k]].neighbor = true;
  }
  std::vector<Quad> keep;
  for (auto& q : qs)
    if (!q.neighbor) keep.push_back(q);
  qs = keep;
}

void to12(const Transform& t, double* o) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) o[i * 3 + j] = t.basis.r[i][j];
  for (int i = 0; i < 3; i++) o[9 + i] = t.origin[i];
}
Transform from12(const double* o) {
  Transform t;
  t.basis = Mat3(o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7], o[8]);
  t.origin = Vec3(o[9], o[10], o[11]);
  return t;
}

Img8 clean_mask_from_canny(const Img8& canny) {
  Img8 grad = gradient_cross(canny);
  for (auto& v : grad.d) v = (uint8_t)~v;
  std::vector<Contour> cs = find_contours(grad, 1);
  Img8 small(canny.w, canny.h, 0);
  draw_contours(small, cs, 255);
  Img8 mask(canny.w, canny.h);
  for (size_t i = 0; i < mask.d.size(); i++) mask.d[i] = canny.d[i] | small.d[i];
  for (int i = 0; i < 3; i++) {
    mask = dilate_rect(mask, 3 + i);
    mask = erode_rect(mask, 3 + i);
  }
  mask = erode_rect(mask, 3);
  return mask;
}

}  // namespace

struct orc_ctx {
  Map map;
  CvRng rng;
  std::vector<std::vector<Vec3>> orientations;  // generatePossibleOrientations
};

extern "C" {

orc_ctx* orc_create(const double* white, int32_t nw, const double* red, int32_t nr, const double* green, int32_t ng,
                    uint64_t seed) {
  orc_ctx* c = new orc_ctx();
  for (int i = 0; i < nw; i++) c->map.white.push_back(Vec3(white[3 * i], white[3 * i + 1], white[3 * i + 2]));
  for (int i = 0; i < nr; i++) c->map.red.push_back(Vec3(red[3 * i], red[3 * i + 1], red[3 * i + 2]));
  for (int i = 0; i < ng; i++) c->map.green.push_back(Vec3(green[3 * i], green[3 * i + 1], green[3 * i + 2]));
  c->rng = CvRng(seed);
  const double g = GRID_SPACING;
  c->orientations = {{Vec3(g / 2, g / 2, 0), Vec3(-g / 2, g / 2, 0), Vec3(-g / 2, -g / 2, 0), Vec3(g / 2, -g / 2, 0)},
                     {Vec3(g / 2, -g / 2, 0), Vec3(-g / 2, -g / 2, 0), Vec3(-g / 2, g / 2, 0), Vec3(g / 2, g / 2, 0)}};
  return c;
}
void orc_destroy(orc_ctx* c) { delete c; }
uint64_t orc_rng_get(orc_ctx* c) { return c->rng.state; }
void orc_rng_set(orc_ctx* c, uint64_t s) { c->rng.state = s; }

int32_t orc_process_frame(orc_ctx* c, const uint8_t* bgr_in, int32_t w, int32_t h, int32_t step, const double* K,
                          const double* D, orc_frame_debug* dbg) {
  std::memset(dbg, 0, sizeof(*dbg));
  Cam cm = make_cam(K, D);
  // cv_bridge ... .clone(): continuous BGR copy
  std::vector<uint8_t> bgr((size_t)w * h * 3);
  for (int y = 0; y < h; y++) std::memcpy(&bgr[(size_t)y * w * 3], bgr_in + (size_t)y * step, (size_t)w * 3);

  // detectQuadrilaterals
  Img8 canny = orc::canny(gauss3x3(bgr2gray(bgr.data(), w, h, 3 * w)), CANNY_LOW, 3 * CANNY_LOW);
  Img8 det = erode_rect(dilate_rect(canny, 2), 1);
  std::vector<Contour> cs = find_contours(det, 2);
  std::vector<Quad> quads;
  for (const auto& ct : cs) {
    Contour ap = approx_poly_dp(ct, (double)POLY_EPS, true);
    if (ap.size() == 4) quads.push_back(make_quad(ap));
  }
  dbg->n_raw_quads = (int32_t)quads.size();
  if (!quads.empty()) remove_duplicates(quads);
  dbg->n_quads = (int32_t)quads.size();
  for (size_t i = 0; i < quads.size() && i < ORC_MAX_QUADS; i++)
    for (int k = 0; k < 4; k++) { dbg->quads[i][2 * k] = quads[i].c[k].x; dbg->quads[i][2 * k + 1] = quads[i].c[k].y; }
  dbg->rng_state_after = c->rng.state;
  if (quads.empty()) { dbg->reason = 1; return 0; }

  // undistortAndNormalizeQuadTestPoints
  for (size_t i = 0; i < quads.size(); i++)
    for (int k = 0; k < 4; k++) {
      double ox, oy;
      undistort_px(cm, quads[i].tp[k][0], quads[i].tp[k][1], ox, oy);
      quads[i].tp[k][0] = ox;
      quads[i].tp[k][1] = oy;
      if (i < ORC_MAX_QUADS) { dbg->test_pts[i][2 * k] = ox; dbg->test_pts[i][2 * k + 1] = oy; }
    }

  // generateHypotheses
  std::vector<Hypothesis> hyps;
  for (const Quad& q : quads) {
    Hypothesis hyp;
    double error = 0;
    bool dropped = false;
    for (const auto& e : c->orientations) {
      double model[12], ip[12];
      for (int k = 0; k < 4; k++) {
        ip[k] = q.tp[k][0]; ip[4 + k] = q.tp[k][1]; ip[8 + k] = 1.0;
        model[k] = e[k].x(); model[4 + k] = e[k].y(); model[8 + k] = e[k].z();
      }
      RppResult rr = rpp(model, ip, 4);
      if (rr.error == 1) { dropped = true; break; }  // reference exit(1): defined as "drop this quad"
      error = rr.img_err;
      Transform tr;
      tr.basis = Mat3(rr.R[0], rr.R[1], rr.R[2], rr.R[3], rr.R[4], rr.R[5], rr.R[6], rr.R[7], rr.R[8]);
      tr.origin = Vec3(rr.t[0], rr.t[1], rr.t[2]);
      hyp.setC2W(tr);
      if (hyp.position().z() >= 0) break;
    }
    if (dropped || error > MAX_QUAD_ERROR) continue;
    std::vector<Hypothesis> central;
    central.push_back(hyp);
    hyp.setW2C(rot_z() * central.back().w2c);
    central.push_back(hyp);
    hyp.setW2C(rot_z() * central.back().w2c);
    central.push_back(hyp);
    hyp.setW2C(rot_z() * central.back().w2c);
    central.push_back(hyp);
    hyps.insert(hyps.end(), central.begin(), central.end());
  }
  dbg->n_gen = (int32_t)hyps.size();

  // PoseClusterer(...).clusterByAngle(0.2).keepLargestCluster().convert2Hypotheses(hyps, false)
  {
    const int n = (int)hyps.size();
    struct P3 { float x, y, z; };
    std::vector<P3> ang(n);
    for (int i = 0; i < n; i++) {
      double r, p, y;
      Mat3(hyps[i].q).getRPY(r, p, y);
      ang[i] = {(float)r, (float)p, (float)y};
    }
    auto rad = [](const P3& a, const P3& b) {
      double dx = a.x - b.x, dy = a.y - b.y, dz = a.z - b.z;
      return std::sqrt(dx * dx + dy * dy + dz * dz);
    };
    std::vector<bool> nb(n, false);
    std::vector<std::vector<int>> clusters;
    for (int i = 0; i < n; i++) {
      if (nb[i]) continue;
      std::vector<int> idx;
      for (int j = 0; j < n; j++)
        if (!nb[j] && rad(ang[i], ang[j]) <= MAX_ANGLE_DIFF * 1.5) idx.push_back(j);
      P3 cen{0, 0, 0};
      for (int e : idx) { cen.x += ang[e].x; cen.y += ang[e].y; cen.z += ang[e].z; }
      double sz = (double)idx.size();
      cen = {(float)(cen.x / sz), (float)(cen.y / sz), (float)(cen.z / sz)};
      idx.clear();
      for (int j = 0; j < n; j++)
        if (!nb[j] && rad(cen, ang[j]) <= MAX_ANGLE_DIFF) idx.push_back(j);
      clusters.push_back(idx);
      for (int e : idx) nb[e] = true;
    }
    std::vector<Hypothesis> kept;
    if (!clusters.empty()) {
      size_t li = 0;
      for (size_t i = 0; i < clusters.size(); i++)
        if (clusters[i].size() > clusters[li].size()) li = i;
      for (int j : clusters[li]) kept.push_back(hyps[j]);
    }
    hyps = kept;
  }
  dbg->n_hyps = (int32_t)hyps.size();
  if (hyps.empty()) { dbg->reason = 2; return 0; }

  // cleanImageByEdge: canny recomputed with identical parameters == `canny`
  Img8 mask = clean_mask_from_canny(canny);
  std::vector<uint8_t> cleaned(bgr.size(), 0);
  for (size_t i = 0; i < mask.d.size(); i++)
    if (mask.d[i]) { cleaned[3 * i] = bgr[3 * i]; cleaned[3 * i + 1] = bgr[3 * i + 1]; cleaned[3 * i + 2] = bgr[3 * i + 2]; }
  View vc{cleaned.data(), w, h}, vo{bgr.data(), w, h};
  int n_scored = 0;

  for (size_t i = 0; i < hyps.size(); i++) {
    int n;
    hyps[i].error = eval_hyp_fast(hyps[i], vc, cm, c->map, &n);
    if (i < ORC_MAX_HYPS) { to12(hyps[i].c2w, dbg->hyp_c2w[i]); dbg->hyp_err[i] = hyps[i].error; dbg->hyp_n[i] = n; }
  }
  n_scored += (int)hyps.size();
  hyps = best_n(1, hyps);
  to12(hyps.back().c2w, dbg->best1_c2w);
  dbg->best1_err = hyps.back().error;

  // optimizeHypothesisWithParticleFilter(best, cleaned, 50, 10)
  Hypothesis cur = hyps.back();
  cur.error = eval_hyp_fast(cur, vc, cm, c->map);
  dbg->pf_iter_err[0] = cur.error;
  n_scored += 1;
  for (int it = 0; it < 10; it++) {
    Hypothesis sample = cur;
    for (int j = 0; j < 50; j++) {
      double yaw = c->rng.gaussian(ROT_SIGMA);
      double pitch = c->rng.gaussian(ROT_SIGMA);
      double roll = c->rng.gaussian(ROT_SIGMA);
      Mat3 rot;
      rot.setRPY(roll, pitch, yaw);
      double tz = c->rng.gaussian(TRANS_SIGMA);
      double ty = c->rng.gaussian(TRANS_SIGMA);
      double tx = c->rng.gaussian(TRANS_SIGMA);
      Transform rnd(rot, Vec3(tx, ty, tz));
      Hypothesis t = sample;
      t.setW2C(sample.w2c * rnd);
      t.error = eval_hyp_fast(t, vc, cm, c->map);
      if (t.error < cur.error) cur = t;
    }
    if (it + 1 < (int)(sizeof(dbg->pf_iter_err) / sizeof(double))) dbg->pf_iter_err[it + 1] = cur.error;  // the record holds 10 iterations
  }
  n_scored += 500;
  to12(cur.c2w, dbg->pf_c2w);
  dbg->pf_err = cur.error;

  // computeAllShiftedHypothesesFAST
  std::vector<Hypothesis> sh;
  for (double x = -((double)GRID_SIZE / 2.0) * GRID_SPACING + ((double)GRID_SPACING / 2.0);
       x < ((double)GRID_SIZE / 2.0) * GRID_SPACING; x += GRID_SPACING)
    for (double y = -((double)GRID_SIZE / 2.0) * GRID_SPACING + ((double)GRID_SPACING / 2.0);
         y < ((double)GRID_SIZE / 2.0) * GRID_SPACING; y += GRID_SPACING) {
      Transform nw = cur.w2c;
      nw.origin += Vec3(x, y, 0);
      Hypothesis nh;
      nh.setW2C(nw);
      sh.push_back(nh);
    }
  for (size_t i = 0; i < sh.size(); i++) {
    sh[i].error = eval_hyp_fast(sh[i], vc, cm, c->map);
    if (i < 81) dbg->shift_err[i] = sh[i].error;
  }
  n_scored += (int)sh.size();
  hyps = best_n(20, sh);
  for (size_t i = 0; i < hyps.size() && i < 20; i++) dbg->top20_err[i] = hyps[i].error;

  // determineBestYaw on the original image
  std::vector<std::vector<Hypothesis>> rots;
  rots.push_back(hyps);
  for (int i = 1; i < 4; i++) {
    rots.push_back(rots.back());
    for (size_t j = 0; j < hyps.size(); j++) {
      Hypothesis t = rots[i][j];
      t.setW2C(rot_z() * rots[i - 1][j].w2c);
      rots[i][j] = t;
    }
  }
  std::vector<Hypothesis> best;
  bool have_best = false;
  double best_error = DBL_MAX;
  std::vector<double> errors;
  for (int k = 0; k < 4; k++) {
    std::vector<Hypothesis> e = rots[k];
    double tot = 0;
    int succ = 0;
    for (auto& hh : e) {
      hh.error = eval_hyp_color(hh, vo, cm, c->map);
      if (std::fabs(hh.error - DBL_MAX) > 0.001) { succ++; tot += hh.error; }
    }
    double te = succ == 0 ? DBL_MAX : tot / (double)succ;
    dbg->yaw_err[k] = te;
    if (te < best_error) { best_error = te; best = e; have_best = true; dbg->yaw_best = k; }
    errors.push_back(te);
  }
  n_scored += 80;
  double min1 = DBL_MAX, min2 = DBL_MAX;
  for (double e : errors) {
    double diff = e - best_error;
    if (diff < min1) { min2 = min1; min1 = diff; }
    else if (diff < min2) { min2 = diff; }
  }
  dbg->min_yaw_diff = min2;
  dbg->n_scored = n_scored;
  dbg->rng_state_after = c->rng.state;
  if (!have_best) { dbg->reason = 4; dbg->yaw_best = -1; return 0; }
  const Hypothesis& pub = best.back();
  to12(pub.c2w, dbg->pub_c2w);
  dbg->pub_error = pub.error;
  for (int i = 0; i < 3; i++) dbg->position[i] = pub.w2c.origin[i];
  dbg->orientation_xyzw[0] = pub.q.x;
  dbg->orientation_xyzw[1] = pub.q.y;
  dbg->orientation_xyzw[2] = pub.q.z;
  dbg->orientation_xyzw[3] = pub.q.w;
  if (min2 > MIN_YAW_DIFF) {
    double var = pub.error * VAR_COEFF;
    for (int i = 0; i < 6; i++) dbg->covariance[i * 6 + i] = var;
    dbg->publish = 1;
    dbg->reason = 0;
  } else {
    dbg->reason = 3;
  }
  return 0;
}

void orc_gray(const uint8_t* bgr, int32_t w, int32_t h, int32_t step, uint8_t* out) {
  Img8 g = bgr2gray(bgr, w, h, step);
  std::memcpy(out, g.d.data(), g.d.size());
}
void orc_blur(const uint8_t* gray, int32_t w, int32_t h, uint8_t* out) {
  Img8 g(w, h);
  std::memcpy(g.d.data(), gray, g.d.size());
  Img8 b = gauss3x3(g);
  std::memcpy(out, b.d.data(), b.d.size());
}
void orc_canny(const uint8_t* bgr, int32_t w, int32_t h, int32_t step, uint8_t* out) {
  Img8 c = orc::canny(gauss3x3(bgr2gray(bgr, w, h, step)), CANNY_LOW, 3 * CANNY_LOW);
  std::memcpy(out, c.d.data(), c.d.size());
}
void orc_hysteresis(const uint8_t* cls, int32_t w, int32_t h, uint8_t* out) {
  Img8 c(w, h);
  std::memcpy(c.d.data(), cls, c.d.size());
  Img8 e = orc::hysteresis(c);
  std::memcpy(out, e.d.data(), e.d.size());
}
void orc_detector_binary(const uint8_t* canny, int32_t w, int32_t h, uint8_t* out) {
  Img8 c(w, h);
  std::memcpy(c.d.data(), canny, c.d.size());
  Img8 d = erode_rect(dilate_rect(c, 2), 1);
  std::memcpy(out, d.d.data(), d.d.size());
}
void orc_clean_mask(const uint8_t* canny, int32_t w, int32_t h, uint8_t* mask) {
  Img8 c(w, h);
  std::memcpy(c.d.data(), canny, c.d.size());
  Img8 m = clean_mask_from_canny(c);
  std::memcpy(mask, m.d.data(), m.d.size());
}
int32_t orc_find_contours(const uint8_t* bin, int32_t w, int32_t h, int32_t mode, int32_t* pts, int32_t max_pts,
                          int32_t* meta, int32_t max_contours) {
  Img8 b(w, h);
  std::memcpy(b.d.data(), bin, b.d.size());
  std::vector<int> holes;
  std::vector<Contour> cs = find_contours(b, mode, &holes);
  if ((int)cs.size() > max_contours) return -1;
  int off = 0;
  for (size_t i = 0; i < cs.size(); i++) {
    if (off + (int)cs[i].size() > max_pts) return -1;
    meta[3 * i] = off;
    meta[3 * i + 1] = (int)cs[i].size();
    meta[3 * i + 2] = holes[i];
    for (const Pt& p : cs[i]) { pts[2 * off] = p.x; pts[2 * off + 1] = p.y; off++; }
  }
  return (int32_t)cs.size();
}
int32_t orc_approx_poly(const int32_t* pts, int32_t n, double eps, int32_t closed, int32_t* out) {
  Contour c(n);
  for (int i = 0; i < n; i++) c[i] = {pts[2 * i], pts[2 * i + 1]};
  Contour a = approx_poly_dp(c, eps, closed != 0);
  for (size_t i = 0; i < a.size(); i++) { out[2 * i] = a[i].x; out[2 * i + 1] = a[i].y; }
  return (int32_t)a.size();
}
int32_t orc_parse_coordinates(const char* s, double* xyz, int32_t max_pts) {
  std::vector<std::string> rows;
  std::stringstream ts(s);
  std::string tmp;
  while (std::getline(ts, tmp, ';')) {
    tmp.erase(std::remove(tmp.begin(), tmp.end(), '\n'), tmp.end());
    tmp.erase(std::remove(tmp.begin(), tmp.end(), ' '), tmp.end());
    rows.push_back(tmp);
  }
  int n = 0;
  for (auto& e : rows) {
    std::stringstream rs(e);
    std::string rt;
    double v[3] = {0, 0, 0};
    for (int k = 0; k < 3; k++) {
      std::getline(rs, rt, ',');
      v[k] = std::atof(rt.data());
    }
    if (n < max_pts) { xyz[3 * n] = v[0]; xyz[3 * n + 1] = v[1]; xyz[3 * n + 2] = v[2]; }
    n++;
  }
  return n;
}
void orc_score(orc_ctx* c, const uint8_t* bgr, int32_t w, int32_t h, const double* K, const double* D,
               const double* c2w, int32_t n, int32_t fast, double* err, int32_t* nproj) {
  Cam cm = make_cam(K, D);
  View v{bgr, w, h};
  for (int i = 0; i < n; i++) {
    Hypothesis hh;
    hh.setC2W(from12(c2w + 12 * i));
    hh.c2w = from12(c2w + 12 * i);  // score exactly the given c2w
    int np = 0;
    err[i] = fast ? eval_hyp_fast(hh, v, cm, c->map, &np) : eval_hyp_color(hh, v, cm, c->map, &np);
    if (nproj) nproj[i] = np;
  }
}
// MonteCarlo::computeCameraError (include/legacy/mantis/MonteCarlo.cpp:183-226)
// for n world->camera poses c2w (n x 12) on one frame: every landmark of the
// three sets projected (project2d :169-181 has no z test) -- here with
// mantis3's fisheye projection (distortPixel, Mantis3Types.h:125-136) of the
// original frame instead of the legacy undistortImage + pinhole K -- the pixel
// as cv::Point2f strictly inside (0, cols) x (0, rows), Mat::at<Vec3b>(Point2f)
// = cvRound of the floats, colorError (:283-286) against the set's colour
// (colors = B, G, R of white, red, green). sums[2i] = error sum, sums[2i+1] = count.
void orc_camera_error(orc_ctx* c, const uint8_t* bgr, int32_t w, int32_t h, const double* K, const double* D,
                      const double* c2w, int32_t n, const int32_t* colors, double* sums) {
  Cam cm = make_cam(K, D);
  View v{bgr, w, h};
  const std::vector<Vec3>* sets[3] = {&c->map.white, &c->map.red, &c->map.green};
  for (int i = 0; i < n; i++) {
    Transform T = from12(c2w + 12 * i);
    double error = 0;
    int cnt = 0;
    for (int s = 0; s < 3; s++)
      for (const Vec3& X : *sets[s]) {
        double u, vv;
        distort_cam(cm, T(X), u, vv);
        const float fx = (float)u, fy = (float)vv;
        if (fx > 0 && fx < w && fy > 0 && fy < h) {
          int b, g, r;
          v.px((int)std::nearbyint(fx), (int)std::nearbyint(fy), b, g, r);
          error += (double)color_err(b, g, r, colors[3 * s], colors[3 * s + 1], colors[3 * s + 2]);
          cnt++;
        }
      }
    sums[2 * i] = error;
    sums[2 * i + 1] = cnt;
  }
}
void orc_distort(const double* xyz, int32_t n, const double* K, const double* D, double* px) {
  Cam cm = make_cam(K, D);
  for (int i = 0; i < n; i++) distort_cam(cm, Vec3(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]), px[2 * i], px[2 * i + 1]);
}
void orc_undistort(const double* px, int32_t n, const double* K, const double* D, double* out) {
  Cam cm = make_cam(K, D);
  for (int i = 0; i < n; i++) undistort_px(cm, px[2 * i], px[2 * i + 1], out[2 * i], out[2 * i + 1]);
}
int32_t orc_rpp(const double* model, const double* iprts, int32_t n, double* R, double* t, double* errs,
                int32_t* err_code) {
  RppResult r = rpp(model, iprts, n);
  std::memcpy(R, r.R, sizeof(r.R));
  std::memcpy(t, r.t, sizeof(r.t));
  errs[0] = r.obj_err;
  errs[1] = r.img_err;
  errs[2] = r.iterations;
  if (err_code) *err_code = r.error;
  return r.status;
}
int32_t orc_rpoly(const double* op, int32_t deg, double* zr, double* zi) { return rpoly(op, deg, zr, zi); }
void orc_svd(const double* A, int32_t m, int32_t n, double* w, double* u, double* vt) { cv_svd(A, m, n, w, u, vt); }
uint64_t orc_gaussians(uint64_t state, int32_t n, float* out) {
  CvRng r(state);
  for (int i = 0; i < n; i++) out[i] = r.gauss01();
  return r.state;
}
void orc_sort_desc(const double* err, int32_t n, int32_t* perm) {
  struct E { double e; int i; };
  std::vector<E> v(n);
  for (int i = 0; i < n; i++) v[i] = {err[i], i};
  std::sort(v.begin(), v.end(), [](const E& a, const E& b) { return b.e < a.e; });
  for (int i = 0; i < n; i++) perm[i] = v[i].i;
}

}  // extern "C"
