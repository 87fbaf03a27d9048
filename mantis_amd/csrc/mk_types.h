// Batch/workspace layouts shared by the HIP kernels (kernels.hip) and the
// host orchestration (api.hip). One "frame" = one camera image of one rig.
#pragma once
#include <cstdint>

#include "../../include/mantis.h"
#include "mk_math.h"
#include "mk_screen.h"

namespace mk {

constexpr int kLandmarksMax = 2048;
constexpr int kGaussPerFrame = 3000;  // 10 iterations x 50 particles x 6 draws (PoseAdjustment.h:15-16, 29)
constexpr int kMaxQuads = 256;
constexpr int kMaxHyps = 4 * kMaxQuads;
constexpr int kMaxBorders = 8192;

struct FrameDesc {
  const uint8_t* bgr;  // contiguous BGR8, stride 3W
  int32_t w, h;
  Cam cam;
  ScreenCam scam;      // FP32 projection screen of the fast scorers (mk_screen.h)
};

struct Border {  // one Suzuki–Abe border in the parallel formulation
  int32_t key;     // raster index (padded) where the scan would discover it
  int32_t start;   // padded index of the start pixel
  int32_t hole;    // 1 = hole border
  int32_t parent;  // CCOMP parent: key of the enclosing component's outer border (own key for outers); holes: -(root run + 1) until k_frame_contours resolves it
};

struct QuadRec {
  int32_t c[8];     // approxPolyDP corners (image coords)
  int32_t parent;   // CCOMP order key
  int32_t hole;
  int32_t key;
  int32_t keep;
  float cx, cy;
  double side;
  double tp[8];     // stretched test points, then undistorted normalized
};

struct RppOut {
  double R[9], t[3];
  double img_err, obj_err;
  int32_t status, error, iterations, pad;
};

struct HypRec {  // mk::Hyp + bookkeeping
  Xf c2w, w2c;
  Quat q;
  double error;
  int32_t nproj, pad;
};

// Stage-by-stage record of one camera-frame; field-for-field the layout of
// the oracle's orc_frame_debug (oracle/oracle.h) so parity tests compare them.
struct FrameDebug {
  int32_t reason;
  int32_t publish;
  int32_t n_raw_quads;
  int32_t n_quads;
  int32_t quads[kMaxQuads][8];
  double test_pts[kMaxQuads][8];
  int32_t n_gen;
  int32_t n_hyps;
  double hyp_c2w[kMaxHyps][12];
  double hyp_err[kMaxHyps];
  int32_t hyp_n[kMaxHyps];
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
  double pub_error;
  double position[3];
  double orientation_xyzw[4];
  double covariance[36];
  uint64_t rng_state_after;
  int32_t n_scored;
};

// Per-frame counters / status written by the kernels.

struct FrameState {
  int32_t n_borders;
  int32_t n_points;
  int32_t n_raw_quads;
  int32_t n_quads;
  int32_t n_gen;
  int32_t n_hyps;
  int32_t reaches_pf;
  int32_t gauss_offset;  // index into the gaussian stream (floats)
  int32_t overflow;      // bit 0 borders, 1 points, 2 quads, 3 hyps
  int32_t n_runs;        // runs of the detector binary (contour CCL, k_run_*)
  int32_t ticks[6];      // k_frame_contours phase ends, 10 ns wall-clock ticks from its start
  int32_t rpp_iters[2];  // AbsKernel calls of the first / candidate ObjPoses (k_objpose_q)
  int32_t trace_steps_max;  // longest border walk (steps) of k_trace_borders
  int32_t n_chunks;         // 64-point chunks handed out by k_trace_borders
  int32_t trace_steps_sum;  // all border walks' steps of the frame
  int32_t trace_ticks;      // k_trace_borders wall-clock time of the frame (10 ns ticks)
  int32_t seg_nc;           // border-walk checkpoint segments of the frame (k_seg_plan; 0: unsplit)
  int32_t seg_m;            // checkpoint row spacing in use (0: borders walked whole)
};

// Gauss–Newton rig refinement (gn_impl.hip): one camera's inv(T_base_cam)
struct GnCam {
  double R_cb[9];
  double t_cb[3];
};
// per-rig state of the rig GN kernels: base pose in, refined pose out.
// n_obs_local = this rank's correspondences (k_rig_gn_obs); n_obs = the whole
// rig's (summed with the accumulators); done = converged / failed / too few.
struct RigGnIO {
  double Twb[16];
  double T0[16];  // the fused pose the correspondences were formed with
  double cost0, cost;
  int32_t valid, iterations, n_obs, done;
  int32_t n_obs_local, pad[3];
};
// per-rig accumulator slot of the rig GN: upper-triangle J^T J (21), J^T r (6),
// r^T r (1), correspondence count (1), padding — summed across camera shards
constexpr int kGnSlot = 32;

// Markov yaw filter operation (markov_impl.hip, include/mantis3/Markov.cpp)
constexpr int kYawBins = 360;

struct MarkovOp {
  int32_t kind;  // -1 skip, 0 MarkovModel(Hypothesis), 1 senseFusion(Hypothesis), 2 convolve
  int32_t bin;   // yaw bin (kinds 0, 1)
  int32_t off;   // kind 2: aux[k] = p[(k + off) % 360] (Markov.cpp:230-248)
  int32_t pad;
  double den;    // stddev * sqrt(2 pi)
  double E[181]; // exp(-((d * d) / (2 * stddev * stddev))), d = 0..180
};


}  // namespace mk
