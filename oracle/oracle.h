/* ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py
 * cpu_baseline). The product library never links or calls this.
 *
 * C API over the CPU restatement of the reference mantis3 per-frame path
 * (src/mantis3.cpp:68-135). Layouts mirror include/mantis.h so parity tests
 * compare field by field. */
#ifndef MANTIS_ORACLE_H
#define MANTIS_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_QUADS 256
#define ORC_MAX_HYPS 1024

typedef struct orc_ctx orc_ctx;

/* Stage-by-stage record of one camera-frame (all in reference order). */
typedef struct orc_frame_debug {
  int32_t reason;            /* 0 published, 1 no quads, 2 no hyps, 3 yaw gap too small, 4 no yaw */
  int32_t publish;
  int32_t n_raw_quads;       /* 4-vertex approxPolyDP results before dedupe */
  int32_t n_quads;           /* after removeDuplicateQuads */
  int32_t quads[ORC_MAX_QUADS][8];       /* int corners x0,y0..x3,y3 */
  double test_pts[ORC_MAX_QUADS][8];     /* undistorted normalized test points */
  int32_t n_gen;             /* hypotheses from generateHypotheses (4 per passing quad) */
  int32_t n_hyps;            /* after keepLargestCluster (C) */
  double hyp_c2w[ORC_MAX_HYPS][12];      /* R row-major, t */
  double hyp_err[ORC_MAX_HYPS];          /* fast errors of the clustered hyps */
  int32_t hyp_n[ORC_MAX_HYPS];           /* projections counted */
  double best1_c2w[12];
  double best1_err;
  double pf_c2w[12];
  double pf_err;
  double pf_iter_err[11];
  double shift_err[81];
  double top20_err[20];
  double yaw_err[4];
  int32_t yaw_best;
  double min_yaw_diff;
  double pub_c2w[12];
  double pub_error;          /* COLOR error of the published hypothesis */
  double position[3];
  double orientation_xyzw[4];
  double covariance[36];
  uint64_t rng_state_after;
  int32_t n_scored;          /* hypotheses fast-scored + slow-scored */
} orc_frame_debug;

orc_ctx* orc_create(const double* white, int32_t nw, const double* red, int32_t nr, const double* green,
                    int32_t ng, uint64_t rng_seed);
void orc_destroy(orc_ctx* c);
uint64_t orc_rng_get(orc_ctx* c);
void orc_rng_set(orc_ctx* c, uint64_t state);

/* Full mantis3 callback on one BGR8 frame (K row-major 3x3, D fisheye k1..k4). */
int32_t orc_process_frame(orc_ctx* c, const uint8_t* bgr, int32_t w, int32_t h, int32_t step, const double* K,
                          const double* D, orc_frame_debug* dbg);

/* ---- stage entry points (images are W x H, row-major) ---- */
void orc_gray(const uint8_t* bgr, int32_t w, int32_t h, int32_t step, uint8_t* out);
void orc_blur(const uint8_t* gray, int32_t w, int32_t h, uint8_t* out);
void orc_canny(const uint8_t* bgr, int32_t w, int32_t h, int32_t step, uint8_t* out); /* gray+blur+Canny(50,150) */
void orc_hysteresis(const uint8_t* cls, int32_t w, int32_t h, uint8_t* out);          /* Canny's hysteresis walk on 0/1/2 classes */
void orc_detector_binary(const uint8_t* canny, int32_t w, int32_t h, uint8_t* out);   /* dilate x2, erode x1 */
void orc_clean_mask(const uint8_t* canny, int32_t w, int32_t h, uint8_t* mask);       /* cleanImageByEdge mask */
/* LIST/CCOMP contours: writes points (x,y pairs) and per-contour [offset,count,is_hole]; returns #contours or -1 */
int32_t orc_find_contours(const uint8_t* bin, int32_t w, int32_t h, int32_t mode, int32_t* pts, int32_t max_pts,
                          int32_t* meta, int32_t max_contours);
int32_t orc_approx_poly(const int32_t* pts, int32_t n, double eps, int32_t closed, int32_t* out);
int32_t orc_parse_coordinates(const char* s, double* xyz, int32_t max_pts);

/* fast (fast=1) or COLOR slow (fast=0) scoring of n hypotheses (c2w 12 doubles each)
 * against a BGR image (the cleaned image for fast scoring). */
void orc_score(orc_ctx* c, const uint8_t* bgr, int32_t w, int32_t h, const double* K, const double* D,
               const double* c2w, int32_t n, int32_t fast, double* err, int32_t* nproj);
void orc_camera_error(orc_ctx* c, const uint8_t* bgr, int32_t w, int32_t h, const double* K, const double* D,
                      const double* c2w, int32_t n, const int32_t* colors, double* sums);
void orc_distort(const double* xyz_cam, int32_t n, const double* K, const double* D, double* px);
void orc_undistort(const double* px, int32_t n, const double* K, const double* D, double* out);

/* RPP on n points: model/iprts 3 x n row-major. out: R[9], t[3], obj_err, img_err; returns status */
int32_t orc_rpp(const double* model, const double* iprts, int32_t n, double* R, double* t, double* errs,
                int32_t* err_code);
int32_t orc_rpoly(const double* op, int32_t deg, double* zr, double* zi);
void orc_svd(const double* A, int32_t m, int32_t n, double* w, double* u, double* vt);
/* n cv::RNG gaussian(1.0) float draws from `state`; returns the state after */
uint64_t orc_gaussians(uint64_t state, int32_t n, float* out);
/* Markov yaw filter (include/mantis3/Markov.cpp, o_markov.cpp): 360-bin planes, R = w2c basis (9) */
void orc_markov_init(const double* R, double* p);
void orc_markov_sense(double* p, const double* R);
void orc_markov_convolve(double* p, double dTheta, double dt);
void orc_markov_weight(const double* p, const double* R, int32_t n, double* error);
double orc_markov_yaw(const double* p, int32_t* argmax);
int32_t orc_markov_bin(const double* R);
/* std::sort(descending error) permutation as libstdc++ orders it */
void orc_sort_desc(const double* err, int32_t n, int32_t* perm);

#ifdef __cplusplus
}
#endif
#endif
