/*
 * mantis.h — C-ABI of the MI355X-native mantis3 hot path (libmantis_amd.so).
 *
 * Drop-in boundary for the reference's per-frame callback and service:
 *   void quadDetection(const sensor_msgs::ImageConstPtr&,
 *                      const sensor_msgs::CameraInfoConstPtr&)   src/mantis3.cpp:68-135
 *   srv/mantisService.srv:1-13 (Image[] image, CameraInfo[] camera_info,
 *        Vector3 delta_pos, Quaternion delta_quat -> Pose pose, float64 weight,
 *        int32 num_particles)                                    (server: src/mantis_server.cpp:23-30)
 * Plain C types only (no ROS/OpenCV/torch types). Every entry point returns a
 * mantis_status; mantis_last_error() describes the last failure on a context.
 * The library never calls exit()/abort() (the reference does: RPP.cpp:450-453).
 *
 * Ownership: input buffers are borrowed for the call only; host inputs are
 * staged through pinned memory. The context owns all device memory and its
 * HIP stream. Threading: one context per host thread; calls on one context are
 * serialized (matching the reference's single ros::spin thread,
 * src/mantis3.cpp:155). State carried across frames (the reference's globals
 * `cv::RNG rng(1)` Mantis3Params.h:87 and the map) lives in the context.
 */
#ifndef MANTIS_H
#define MANTIS_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MANTIS_ABI_VERSION 2

typedef enum mantis_status {
  MANTIS_OK = 0,
  MANTIS_ERR_ARG = 1,       /* bad argument (null pointer, size, channel count) */
  MANTIS_ERR_DEVICE = 2,    /* HIP runtime / kernel failure, or no GPU */
  MANTIS_ERR_OOM = 3,       /* device or pinned allocation failed */
  MANTIS_ERR_CAPACITY = 4,  /* a fixed-capacity workspace overflowed (see last_error) */
  MANTIS_ERR_STATE = 5,     /* map not set, comm not initialised, ... */
  MANTIS_ERR_COMM = 6       /* RCCL failure */
} mantis_status;

/* Per-frame outcome (reference early returns / gates, src/mantis3.cpp:82-132). */
typedef enum mantis_reason {
  MANTIS_PUBLISHED = 0,      /* yaw gap > MINIMUM_YAW_DIFFERENCE, pose published (PosePub.h:16) */
  MANTIS_NO_QUADS = 1,       /* "no quadrilaterlals detected!" early return (mantis3.cpp:82-84) */
  MANTIS_NO_HYPS = 2,        /* empty cluster (mantis3.cpp:94-97) */
  MANTIS_YAW_AMBIGUOUS = 3,  /* pose computed but gate not met: not published */
  MANTIS_NO_YAW = 4          /* every yaw set scored DBL_MAX (reference UB) */
} mantis_reason;

typedef struct mantis_config {
  int32_t struct_size;          /* sizeof(mantis_config) */
  int32_t device;               /* HIP device ordinal */
  int32_t max_cams;             /* camera-frames per mantis_process_batch call */
  int32_t max_width, max_height; /* width <= 8190, height <= 65533, width x height < 2^25 (else MANTIS_ERR_ARG) */
  uint64_t rng_seed;            /* cv::RNG seed, 1 in the reference (Mantis3Params.h:87) */
  int32_t canny_low;            /* ~canny_hysteresis, 50 (Mantis3Params.h:162); high = 3x */
  int32_t polygon_epsilon;      /* ~polygon_epsilon, 10 (:164) */
  double search_radius_multiplier; /* ~neighborhood_search_radius_multiplier, 0.1 (:166) */
  double grid_spacing;          /* ~grid_spacing, 0.32 (:167) */
  int32_t particles, iterations;/* 50, 10 (PoseAdjustment.h:29) */
  int32_t gn_enable;            /* 0 = reference-parity mode (no GN refinement) */
  int32_t gn_iterations;        /* rig GN iterations (0..10) */
  int32_t max_quads;            /* per-frame quad capacity: 256 (0 = default); other values are rejected */
  int32_t max_contour_points;   /* per-frame contour point pool (default 262144) */
  int32_t quad_gn_iterations;   /* per-quad GN after RPP (4 corners <-> model square), 0 = off (parity) */
  int32_t rig_weighting;        /* rig fusion: 0 = lowest-error published camera (default);
                                   1 = legacy MonteCarlo weighting (see mantis_get_rig_weights) */
} mantis_config;

typedef struct mantis_image {   /* sensor_msgs/Image (bgr8) + sensor_msgs/CameraInfo */
  int32_t width, height;
  int32_t step_bytes;           /* row stride, >= 3*width */
  int32_t mem_kind;             /* 0 = host pointer, 1 = device pointer (already in HBM) */
  const uint8_t* bgr;
  double K[9];                  /* CameraInfo.K, row-major; rounded to float as get3x3FromVector does */
  double D[4];                  /* fisheye k1..k4 (CameraInfo.D) */
  double T_base_cam[16];        /* camera pose in the rig/base frame (row-major 4x4); identity for 1 cam */
  int64_t stamp_ns;
  const char* frame_id;
} mantis_image;

typedef struct mantis_motion {  /* mantisService delta_pos / delta_quat ("applied to each particle") */
  double delta_pos[3];
  double delta_quat_xyzw[4];
} mantis_motion;

typedef struct mantis_cam_result {
  int32_t status;
  int32_t reason;               /* mantis_reason */
  int32_t publish;
  int32_t n_quads;              /* after removeDuplicateQuads */
  int32_t n_hyps;               /* after clustering (C) */
  int32_t n_scored;             /* hypotheses scored (fast + slow) */
  double position[3];           /* published camera position (w2c origin, PosePub.h:33-45) */
  double orientation_xyzw[4];
  double covariance[36];        /* diag(error / 600) (PosePub.h:47-56) */
  double error;                 /* hyp.error of the published hypothesis (COLOR error) */
  double min_yaw_diff;
  double pf_error;              /* fast error of the particle-filter optimum */
  double c2w[12];               /* published hypothesis, world->camera R (row-major) | t */
} mantis_cam_result;

typedef struct mantis_result {  /* one rig pose (mantisService response + diagnostics) */
  int32_t status;
  int32_t publish;
  int32_t n_cams_published;
  int32_t num_particles;        /* srv num_particles: hypotheses scored over the rig */
  double position[3];           /* srv pose (base frame in world) */
  double orientation_xyzw[4];
  double covariance[36];
  double weight;                /* srv weight: error of the chosen camera hypothesis */
  double min_yaw_diff;
  int32_t n_quads;
  int32_t gn_iterations;
  double gn_cost;               /* final GN cost (0 when GN disabled) */
  uint64_t rng_state_after;
} mantis_result;

/* ---------------------------------------------------------------- context */
void mantis_default_config(mantis_config* cfg);
mantis_status mantis_create(const mantis_config* cfg, void** out_ctx);
mantis_status mantis_destroy(void* ctx);
const char* mantis_last_error(void* ctx);
int32_t mantis_abi_version(void);

/* whiteMap / redMap / greenMap (params/map.yaml, parsed as Mantis3Params.h:125-152) */
mantis_status mantis_set_map(void* ctx, const double* white_xyz, int32_t nw, const double* red_xyz, int32_t nr,
                             const double* green_xyz, int32_t ng);
/* parseCoordinatesFromString (Mantis3Params.h:125-152); returns the row count, writes up to max_pts */
int32_t mantis_parse_coordinates(const char* s, double* xyz, int32_t max_pts);

/* cv::RNG state (checkpoint / resume of the cross-frame particle-filter stream) */
mantis_status mantis_rng_get(void* ctx, uint64_t* state);
mantis_status mantis_rng_set(void* ctx, uint64_t state);

/* ------------------------------------------------------------ hot path */
/* One rig pose from n_cams synchronized cameras (n_cams = 1 is exactly the
 * reference callback quadDetection, src/mantis3.cpp:68-135). cam_out may be
 * NULL; otherwise it receives n_cams per-camera results. motion (nullable) is
 * the mantisService delta_pos / delta_quat ("applied to each particle before
 * reevaluating", srv/mantisService.srv:4-8): the context keeps the last
 * published rig pose as the service's particle; with a motion and that prior,
 * T_prior * Transform(delta_quat, delta_pos) joins the rig candidates and all
 * are re-evaluated with the legacy weighting (mantis_get_rig_weights, last
 * candidate slot). Without a prior, or with |delta_quat|^2 < 0.5 (an unset
 * message), the call is the reference callback. */
mantis_status mantis_process(void* ctx, const mantis_image* cams, int32_t n_cams, const mantis_motion* motion,
                             mantis_result* out, mantis_cam_result* cam_out);
/* the motion prior (last published rig pose, T_w_b row-major 4x4): set (NULL clears) / get */
mantis_status mantis_set_prior_pose(void* ctx, const double* T_w_b);
mantis_status mantis_get_prior_pose(void* ctx, double* T_w_b, int32_t* has_prior);
/* n_rigs rigs of cams_per_rig cameras in one batched pass (throughput path):
 * cams[r * cams_per_rig + c]; frames are processed (and draw RNG) in that order. */
mantis_status mantis_process_batch(void* ctx, const mantis_image* cams, int32_t n_rigs, int32_t cams_per_rig,
                                   mantis_result* out, mantis_cam_result* cam_out);

/* Camera-sharded rig (BASELINE config 4: 8 cameras, one per GPU; SURVEY §8 e).
 * Every rank of the communicator (mantis_comm_init) calls this with the same
 * n_rigs / cams_per_rig and its own cameras: local_cams[r * n_local + j] is
 * camera cam_index[j] (ascending) of rig r; each camera belongs to exactly one
 * rank and n_local <= ceil(cams_per_rig / nranks). Exchanges (RCCL over xGMI):
 * one ncclAllGather of the frames' particle-filter flags, so every frame
 * draws the cv::RNG stream at the offset a sequential run over the rig's
 * cameras in rig-major order would (Mantis3Params.h:87, PoseAdjustment.h:15-16);
 * one ncclAllGather of the camera results for the rig fusion; with gn_enable one
 * ncclAllReduce of every rig's J^T J / J^T r accumulators per Gauss-Newton
 * iteration (each rank then solves the same 6x6 system). The multi-camera seam of
 * the reference is the base->camera extrinsic chain of
 * include/legacy/mantis/MonteCarlo.cpp:250-271. Every rank returns the same
 * out[n_rigs]; cam_out (nullable) receives all n_rigs * cams_per_rig camera
 * results in global order. With one rank this equals mantis_process_batch. */
mantis_status mantis_process_rig_sharded(void* ctx, const mantis_image* local_cams, int32_t n_rigs, int32_t n_local,
                                         const int32_t* cam_index, int32_t cams_per_rig, mantis_result* out,
                                         mantis_cam_result* cam_out);

/* Stage entry of the sharded call's cross-rank RNG bookkeeping (device
 * kernel k_gauss_offsets_global, for parity tests): `pairs` = the gathered
 * (global frame index, reaches-PF flag) pairs of every rank (npairs pairs,
 * padding slots (-1, 0)); each of the n_local frames with global index gidx[i]
 * gets offsets[i] = per_frame x (frames before it in global order that reach
 * the particle filter), i.e. where a sequential run over all cameras draws its
 * cv::RNG gaussians (Mantis3Params.h:87, PoseAdjustment.h:15-16); *total = the
 * gaussians drawn by all n_global frames. Host rule: mantis_amd/csrc/mk_shard.h. */
mantis_status mantis_shard_gauss_offsets(void* ctx, const int32_t* pairs, int32_t npairs, int32_t n_global,
                                         const int32_t* gidx, int32_t n_local, int32_t per_frame, int32_t* offsets,
                                         int32_t* total);

/* Rig Gauss-Newton record of rig `rig` of the last batch (cfg.gn_enable):
 * the fused pose the correspondences were formed with, the refined pose, the
 * cost before / after, and this rank's correspondences as rows of
 * [local camera index, u, v, X, Y, Z] (normalized undistorted point, world point). */
typedef struct mantis_rig_gn_info {
  double T_init[16];
  double T_final[16];
  double cost0, cost;
  int32_t valid, iterations, n_obs, n_obs_local;
} mantis_rig_gn_info;
mantis_status mantis_get_rig_gn(void* ctx, int32_t rig, mantis_rig_gn_info* info, double* obs, int32_t cap);

/* Rig weighting (cfg.rig_weighting = 1): the legacy particle
 * weight MonteCarlo::computeWeight / computeCameraError
 * (include/legacy/mantis/MonteCarlo.cpp:183-241) made to work with every
 * camera of the rig (the reference's "TODO make work with both cameras",
 * :250-271). Candidate k = the base pose implied by published camera k
 * (T_w_b = T_w_c inv(T_base_cam)); camera c scores it with
 * computeCameraError: every landmark projected into c (no z test, the float
 * pixel strictly inside (0, cols) x (0, rows), cvRound), the squared BGR
 * distance to its set's colour (white / red / green targets, mantis3's
 * palette Mantis3Params.h:40-42), error = sum / n, or 1e17 / n when n < 10.
 * The legacy undistortImage + pinhole projection is replaced by mantis3's
 * fisheye projection of the original frame (distortPixel, Mantis3Types.h:
 * 125-136). Weight = mean over the rig's cameras; the lowest weight wins
 * (first on ties) and is the rig's srv weight. Camera-sharded rigs sum the
 * per-camera (error sum, count) slots with one ncclAllReduce (exact integers).
 * Record of rig `rig` of the last batch, K = C + 1 candidate slots (C =
 * cams_per_rig; slot C = the mantisService motion prediction, see
 * mantis_process): weights[K] (DBL_MAX = not a candidate), c2w[K x C x 12]
 * (world->camera of candidate k in camera c, this rank's cameras; nullable),
 * sums[K x C x 2] (sum, count; nullable), chosen = winning slot or -1. */
mantis_status mantis_get_rig_weights(void* ctx, int32_t rig, double* weights, double* c2w, double* sums,
                                     int32_t* chosen);
/* Shape of the last batch's weighting record: rigs and C (cameras per rig), so
 * a caller sizes the buffers of mantis_get_rig_weights (K = C + 1 slots). */
mantis_status mantis_get_rig_weights_info(void* ctx, int32_t* n_rigs, int32_t* cams_per_rig);

/* Markov yaw filter (include/mantis3/Markov.{h,cpp}, MarkovModel,
 * included but unused upstream): n_filters 360-bin yaw distributions in the
 * context's HBM (one per camera stream or rig). w2c_R: hypothesis poses' w2c
 * bases (row-major 3x3, one per filter / hypothesis); yaw bin = getRPY yaw in
 * degrees wrapped to [0, 360). active (nullable): filter f is updated iff
 * active[f] != 0. Results are bit-identical to oracle/o_markov.cpp. */
/* MarkovModel(Hypothesis) (Markov.cpp:15-27): one-hot at the yaw bin, blurred (stddev 3) */
mantis_status mantis_markov_init(void* ctx, int32_t n_filters, const double* w2c_R);
/* senseFusion(Hypothesis) (:164-201): multiply by the measurement (stddev 3.5), normalize */
mantis_status mantis_markov_sense(void* ctx, const double* w2c_R, const int32_t* active);
/* convolve(dTheta, dt) (:227-258): shift by (int)dTheta*180/pi bins (dTheta truncated to whole
 * radians first, as the reference), blur with stddev dt * 11.5 / 90 */
mantis_status mantis_markov_convolve(void* ctx, const double* dtheta, const double* dt, const int32_t* active);
/* updateHypothesis (:207-222) with filter `filter`: error[i] = error[i] * 1 / p[bin(w2c_R[i])] */
mantis_status mantis_markov_weight(void* ctx, int32_t filter, const double* w2c_R, int32_t n, double* error);
/* planes (n_filters x 360, nullable); yaw = getYaw (:265-275: p[argmax] * pi / 180, the reference's
 * return value; nullable); argmax = first maximum bin (nullable) */
mantis_status mantis_markov_get(void* ctx, double* planes, double* yaw, int32_t* argmax);

/* ------------------------------------------- stage entry points (parity) */
/* gray -> GaussianBlur 3x3 -> Canny(50,150) (QuadDetection.h:209-212); out W*H bytes 0/255 */
mantis_status mantis_canny(void* ctx, const mantis_image* img, uint8_t* canny_out);
/* cv::Canny's hysteresis alone (the stack walk of QuadDetection.h:212 / HypothesisEvaluation.h:327's
 * Canny): cls W*H bytes, 0 = no candidate, 1 = weak candidate (NMS passed, mag > low), 2 = strong
 * (mag > high); out W*H bytes 0/255 = the candidates 8-connected to a strong pixel. Any other
 * class byte (e.g. a 0/255 plane) returns MANTIS_ERR_ARG */
mantis_status mantis_hysteresis(void* ctx, const uint8_t* cls, int32_t width, int32_t height, uint8_t* edges_out);
/* detector binary (dilate x2, erode x1, QuadDetection.h:213-214) and the
 * cleanImageByEdge mask (HypothesisEvaluation.h:319-386); either output may be NULL */
mantis_status mantis_masks(void* ctx, const mantis_image* img, uint8_t* det_out, uint8_t* mask_out);
/* detectQuadrilaterals (QuadDetection.h:203-287): int corners x0,y0..x3,y3 per quad,
 * after removeDuplicateQuads, in reference order */
mantis_status mantis_detect_quads(void* ctx, const mantis_image* img, int32_t* corners, int32_t max_quads,
                                  int32_t* n_quads);
/* evaluateHypotheses (HypothesisEvaluation.h:31-41, 71-158) fast=1 (1 px, all landmarks vs WHITE)
 * or evaluateHypothesisCOLOR (:89-105, 160-266) fast=0 (10x10 window, green vs GREEN).
 * c2w: n x 12 doubles (world->camera R row-major | t). mask: W*H bytes (nonzero = keep) or NULL
 * (score img as given). err: error per hypothesis (DBL_MAX if no projection), nproj: counts. */
mantis_status mantis_score_hypotheses(void* ctx, const mantis_image* img, const uint8_t* mask, const double* c2w,
                                      int32_t n, int32_t fast, double* err, int32_t* nproj);
/* RPP::Rpp on n 4-point problems (RPP.cpp:13-64): img_pts n x 4 x 2 normalized, obj_pts n x 4 x 3.
 * R n x 9, t n x 3, errs n x 2 (obj_err, img_err), rpp_status n (1 ok, 0 2nd-pose search failed,
 * -1 rotation check failed = the reference's exit(1)). */
mantis_status mantis_rpp_batch(void* ctx, const double* img_pts, const double* obj_pts, int32_t n, double* R,
                               double* t, double* errs, int32_t* rpp_status);
/* RPP::Rpp(model, iprts, ...) (RPP.h:92-93, RPP.cpp:13-64) on n problems of n_points points each,
 * 4 <= n_points <= 12 (the reference accepts any count; demo.cpp:17-38 solves 10): img_pts
 * n x n_points x 2 normalized (the homogeneous row is 1, as demo.cpp's Mat::ones), obj_pts
 * n x n_points x 3. Outputs as mantis_rpp_batch plus iterations (n, nullable: the reference's
 * `iterations` out-parameter). One device lane per problem; mantis_rpp_batch is the throughput
 * entry for 4-point problems (same arithmetic, bit-identical results). */
mantis_status mantis_rpp_solve(void* ctx, const double* img_pts, const double* obj_pts, int32_t n_points,
                               int32_t n, double* R, double* t, double* errs, int32_t* rpp_status,
                               int32_t* iterations);

/* Per-quad Gauss-Newton after RPP (new stage; legacy analogue
 * cv::solvePnP ITERATIVE, include/legacy/mantis2/PoseEstimator.h:91-153): n
 * problems of 4 normalized image points img_pts (n x 4 x 2) and model points
 * obj_pts (n x 4 x 3); R (n x 9), t (n x 3) hold the starting pose (model ->
 * camera, e.g. mantis_rpp_batch's) and receive the refined one. Up to
 * `iterations` steps minimizing the normalized reprojection error; a step is
 * kept only if the cost decreases. steps (n, nullable) = steps kept, costs
 * (n x 2, nullable) = r^T r before / after. The same refinement runs inside
 * the pipeline after RPP when cfg.quad_gn_iterations > 0. */
mantis_status mantis_quad_gn(void* ctx, const double* img_pts, const double* obj_pts, int32_t n, double* R,
                             double* t, int32_t iterations, int32_t* steps, double* costs);

/* Dense scoring with an argmin (BASELINE config 5: 81 shifts x 4 yaws x 50
 * perturbations = 16,200 hypotheses, SURVEY §8 d/e): the fast evaluator
 * (evaluateHypotheses, HypothesisEvaluation.h:31-41, 71-158) on n hypotheses,
 * then the lowest error with the first index on ties (the strict "<" the
 * reference's best-1 choice keeps). Hypothesis k of this call has global index
 * index_base + k. With use_comm (after mantis_comm_init) every rank passes its
 * shard and one ncclAllGather of (err, index) pairs gives all ranks the global
 * winner. best_idx = -1 when no hypothesis was scored. */
mantis_status mantis_score_argmin(void* ctx, const mantis_image* img, const uint8_t* mask, const double* c2w,
                                  int32_t n, int64_t index_base, int32_t use_comm, double* best_err,
                                  int64_t* best_idx);
/* The same with device-resident inputs: mask_dev (W*H bytes, or NULL) and c2w_dev
 * (n x 12 doubles) are device pointers on the context's GPU (mantis_device_alloc
 * or any allocation of that device), read in place -- no staging copy -- for
 * callers whose hypotheses are produced on the device or reused across calls. */
mantis_status mantis_score_argmin_dev(void* ctx, const mantis_image* img, const uint8_t* mask_dev,
                                      const double* c2w_dev, int32_t n, int64_t index_base, int32_t use_comm,
                                      double* best_err, int64_t* best_idx);
/* The cross-shard rule on its own (host only): pairs = nranks x (err, global index). */
mantis_status mantis_argmin_pick(const double* pairs, int32_t nranks, double* best_err, int64_t* best_idx);

/* mantis_score_argmin_dev over n_frames frames in one call (BASELINE config 5
 * batched): frame f's n_hyps[f] hypotheses (device c2w_dev[f], n x 12) scored
 * against its cleaned mask (device masks_dev[f], nullable array / entries)
 * in one launch, one argmin per frame, and with use_comm one ncclAllGather of
 * every frame's (err, global index) pair per rank; best_err / best_idx get
 * n_frames entries (global index = index_base[f] + local index). */
mantis_status mantis_score_argmin_batch(void* ctx, const mantis_image* imgs, int32_t n_frames,
                                        const uint8_t* const* masks_dev, const double* const* c2w_dev,
                                        const int32_t* n_hyps, const int64_t* index_base, int32_t use_comm,
                                        double* best_err, int64_t* best_idx);

/* ----------------------------------------- Gauss–Newton rig refinement (new) */
/* One GN step over m camera observations: for camera c, corr_c normalized image points u (2)
 * matched to world points X (3). Accumulates J^T J (21 upper-tri), J^T r (6), cost (1) into
 * acc28 for the base pose T_w_b (4x4 row-major) with right-perturbation exp(delta).
 * obs: rows of [cam_index, u_x, u_y, X, Y, Z]; T_base_cam: 16 doubles per camera. */
mantis_status mantis_gn_accumulate(void* ctx, const double* T_w_b, const double* T_base_cam, int32_t n_cams,
                                   const double* obs, int32_t n_obs, double* acc28);
/* Solve (JtJ + lambda I) delta = -Jtr from acc28 and update T_w_b in place. */
mantis_status mantis_gn_solve(const double* acc28, double lambda, double* T_w_b, double* delta6);

/* ------------------------------------------------- multi-GPU (RCCL, xGMI) */
/* 128-byte ncclUniqueId; rank 0 creates it, the caller broadcasts it. */
mantis_status mantis_comm_unique_id(void* id128);
mantis_status mantis_comm_init(void* ctx, const void* id128, int32_t nranks, int32_t rank);
/* the communicator's size and this context's rank (MANTIS_ERR_STATE without one) */
mantis_status mantis_comm_info(void* ctx, int32_t* nranks, int32_t* rank);
/* Camera-sharded rig: this rank contributes its cameras; the 28-double GN
 * accumulators are summed with one ncclAllReduce per iteration. */
mantis_status mantis_gn_allreduce(void* ctx, double* acc28);

/* ------------------------------------------------------------- tools */
/* Synthetic fisheye grid frames rendered in HBM (bench inputs). cams: n x mantis_synth_cam;
 * out_dev: device buffer n x H x W x 3 (stride 3W). */
typedef struct mantis_synth_cam {
  double fx, fy, cx, cy;
  double k[4];
  double R_wc[9];
  double pos[3];
  int32_t w, h;
  int32_t pad[2];
} mantis_synth_cam;
mantis_status mantis_synth_render(void* ctx, const mantis_synth_cam* cams, int32_t n, const uint64_t* seeds,
                                  uint8_t* out_dev);
/* Device buffers owned by the context (for device-resident benchmark inputs). */
mantis_status mantis_device_alloc(void* ctx, size_t bytes, void** dev_ptr);
mantis_status mantis_device_free(void* ctx, void* dev_ptr);
mantis_status mantis_memcpy_h2d(void* ctx, void* dst_dev, const void* src_host, size_t bytes);
mantis_status mantis_memcpy_d2h(void* ctx, void* dst_host, const void* src_dev, size_t bytes);
mantis_status mantis_synchronize(void* ctx);
/* Per-kernel timing of the last call (HIP events on the context stream), in ms. */
int32_t mantis_kernel_times(void* ctx, const char** names, float* ms, int32_t max);
/* Enable stage timing events (1) or not (0). */
mantis_status mantis_set_profiling(void* ctx, int32_t on);

/* ------------------------------------------------------- diagnostics */
/* Stage-by-stage record of camera-frame `frame` of the last batch (quads,
 * hypotheses, PF/shift/yaw errors); layout = oracle/oracle.h orc_frame_debug. */
size_t mantis_frame_debug_size(void);
mantis_status mantis_get_frame_debug(void* ctx, int32_t frame, void* out, size_t bytes);
/* The border-following output of camera-frame `frame` of the last batch
 * (findContours(RETR_CCOMP, CHAIN_APPROX_SIMPLE), QuadDetection.h:216, in the
 * library's border order): per border its point count and hole flag, and all
 * points (x, y pairs, image coordinates) border after border. Fails with
 * MANTIS_ERR_CAPACITY when max_borders / max_points are too small. */
mantis_status mantis_get_contours(void* ctx, int32_t frame, int32_t* counts, int32_t* holes, int32_t max_borders,
                                  int32_t* points, int32_t max_points, int32_t* n_borders);
/* Work counters of camera-frame `frame` of the last batch: borders, contour
 * points, raw/kept quads, generated/clustered hypotheses, PF flag, gaussian
 * offset, overflow flags, then 7 contour-kernel phase ends (10 ns ticks).
 * Returns the number of int32 written (<= max), -1 on a bad argument. */
int32_t mantis_frame_counters(void* ctx, int32_t frame, int32_t* out, int32_t max);
/* Batches of at most this many frames take the latency kernels (tile Canny, segmented
 * morphology walker, LDS border walks, 1024-thread contour blocks), larger ones the
 * throughput kernels; both give identical results (CUs / 4 by default,
 * MANTIS_FC_SMALL_FRAMES). No reference counterpart: a tuning query. */
int32_t mantis_small_batch_frames(void* ctx);

#ifdef __cplusplus
}
#endif
#endif /* MANTIS_H */
