// libmantis_amd.so — C-ABI (include/mantis.h) and host orchestration of the
// batched mantis3 hot path on one MI355X. One translation unit: the kernels
// are included below so every launch sees its definition.
//
// Batch flow per mantis_process_batch call (one HIP stream, no host sync
// until the results are copied back):
//   H2D frames (pinned staging)      | host: gaussian stream for the batch
//   image stages (all frames)        |   (cv::RNG, generated while the GPU
//   contours -> quads -> RPP -> hyps |    runs the detector)
//   offsets into the gaussian stream (frames that reach the PF, in order)
//   H2D gaussians -> scoring/PF/shift/yaw -> D2H results
#include <hip/hip_runtime.h>
#ifndef MK_FC_THREADS
#define MK_FC_THREADS 256  // k_frame_contours threads per frame for large batches
#endif

#include <algorithm>
#include <atomic>
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "kernels.hip"

using namespace mk;

namespace {

// ------------------------------------------------------------ cv::RNG (host)
// The reference's global `cv::RNG rng(1)` (Mantis3Params.h:87): MWC step and
// the float32 ziggurat of RNG::gaussian [OpenCV 3.x], generated on the host in
// draw order and consumed on the device from a per-batch stream.
struct ZigTables {
  uint32_t kn[128];
  float wn[128], fn[128];
  ZigTables() {
    const double m1 = 2147483648.0;
    double dn = 3.442619855899, tn = dn, vn = 9.91256303526217e-3;
    double q = vn / std::exp(-.5 * dn * dn);
    kn[0] = (uint32_t)((dn / q) * m1);
    kn[1] = 0;
    wn[0] = (float)(q / m1);
    wn[127] = (float)(dn / m1);
    fn[0] = 1.f;
    fn[127] = (float)std::exp(-.5 * dn * dn);
    for (int i = 126; i >= 1; i--) {
      dn = std::sqrt(-2. * std::log(vn / dn + std::exp(-.5 * dn * dn)));
      kn[i + 1] = (uint32_t)((dn / tn) * m1);
      tn = dn;
      fn[i] = (float)std::exp(-.5 * dn * dn);
      wn[i] = (float)(dn / m1);
    }
  }
};
const ZigTables& zig() {
  static ZigTables t;
  return t;
}
inline uint64_t rng_step(uint64_t x) { return (uint64_t)(uint32_t)x * 4164903690ULL + (x >> 32); }
inline float rng_gauss(uint64_t& state) {
  const ZigTables& T = zig();
  const float r = 3.442620f;
  const float rng_flt = 2.3283064365386962890625e-10f;
  uint64_t temp = state;
  float x, y;
  for (;;) {
    int hz = (int)(uint32_t)temp;
    temp = rng_step(temp);
    int iz = hz & 127;
    x = hz * T.wn[iz];
    if ((unsigned)std::abs(hz) < T.kn[iz]) break;
    if (iz == 0) {
      do {
        x = (unsigned)temp * rng_flt;
        temp = rng_step(temp);
        y = (unsigned)temp * rng_flt;
        temp = rng_step(temp);
        x = (float)(-std::log(x + FLT_MIN) * 0.2904764);
        y = (float)-std::log(y + FLT_MIN);
      } while (y + y < x * x);
      x = hz > 0 ? r + x : -r - x;
      break;
    }
    y = (unsigned)temp * rng_flt;
    temp = rng_step(temp);
    if (T.fn[iz] + y * (T.fn[iz - 1] - T.fn[iz]) < std::exp(-.5 * x * x)) break;
  }
  state = temp;
  return x;
}

#define HIP_OK(expr)                                                              \
  do {                                                                            \
    hipError_t e_ = (expr);                                                       \
    if (e_ != hipSuccess) {                                                       \
      c->err = std::string(#expr) + ": " + hipGetErrorString(e_);                 \
      return MANTIS_ERR_DEVICE;                                                   \
    }                                                                             \
  } while (0)

struct Ctx {
  mantis_config cfg{};
  hipStream_t s = nullptr;
  hipStream_t s_copy = nullptr;     // side stream: the gaussian stream's H2D, overlapped with RPP
  hipEvent_t ev_gauss = nullptr;    // ... which s waits on before scoring
  // batch calls wait for the stream on a blocking-sync event (the host thread
  // sleeps instead of spinning in hipStreamSynchronize: one spinning thread per
  // context was most of a step's host CPU time); calls of at most
  // spin_frames frames spin (latency).
  hipEvent_t ev_wait = nullptr;
  int spin_frames = 16;
  std::string err;
  uint64_t rng_state = 1;
  // map
  double* d_lm = nullptr;
  int nw = 0, nr = 0, ng = 0;
  // capacity
  int F = 0, Wmax = 0, Hmax = 0;
  int n_cu = 256;  // compute units of the device (block-size choices)
  // k_trace_borders_lds (bit plane in LDS) for batches of at most trace_lds_frames frames
  bool trace_lds_ok = false;
  size_t trace_lds_max = 0;
  int trace_lds_frames = 0;
  int fc_small_frames = 0;  // k_frame_contours at 1024 threads for batches of at most this many frames
  size_t plane = 0;
  int pool_cap = 0;
  // device workspace
  uint16_t* d_lroot = nullptr;  // hysteresis run extents (k_hyst_*), then contour run starts
  size_t lstride = 0;            // d_lroot entries per frame: max(plane, tiles x FTW x FTH)
  size_t fstride = 0;            // d_strong bytes per frame: plane rounded up to a dword (32-bit flag atomics)
  uint8_t *d_bgr = nullptr, *d_strong = nullptr, *d_edge = nullptr,
          *d_det = nullptr, *d_mask = nullptr;
  int32_t* d_lab = nullptr;
  uint32_t *d_eb = nullptr, *d_b1 = nullptr, *d_b2 = nullptr;  // bit planes
  uint32_t* d_mbits = nullptr;  // cleanImageByEdge mask bits (k_morph -> k_frame_score)
  size_t bstride = 0;                                           // words per frame
  int morph_bh = 48;       // k_morph output rows per band (MB_BH, or MB_BH_NARROW at wide max_width)
  int morph_walk = 1 << 20;  // k_morph_walk rows per segment (0: the LDS band kernel k_morph); MANTIS_MORPH_WALK
  bool runs_done = false;    // this batch's detector runs were numbered by the walker (one segment per frame)
  int morph_walk_small = 48; // walker segment rows for batches of at most fc_small_frames frames; MANTIS_MORPH_WALK_SMALL
  size_t pf_mask_lds = 0;  // bytes of dynamic LDS for k_score_pf's staged mask (0: global mask)
  int hyst_epoch = 3;      // hysteresis mark value of the current call (4..255; 3: the plane is not cleared yet)
  bool hyst_rec = true;    // hysteresis by bit-parallel reconstruction (k_hyst_rec) where the frame fits it; MANTIS_HYST_REC=0: run CCL
  size_t hyst_rec_lds = 0;  // dynamic LDS k_hyst_rec may take (a frame's candidate words)
  bool pf_split = true;    // small batches: each particle-filter iteration over several blocks per frame
                           // (k_score_pf_part); MANTIS_PF_SPLIT=0 keeps one block per frame
  uint32_t* d_dbits = nullptr;                                  // padded detector bits
  uint32_t* d_tbits = nullptr;                                  // the same in 32x32 tiles (k_trace_borders)
  size_t tstride = 0;
  int32_t* d_rowb = nullptr;  // run CCL row bases, rstride per frame
  size_t rstride = 0;
  size_t dstride = 0;
  FrameDesc* d_frames = nullptr;
  Border* d_borders = nullptr;
  int32_t *d_bcount = nullptr, *d_boff = nullptr, *d_pool = nullptr, *d_scratch = nullptr;
  QuadRec* d_quads = nullptr;
  RppOut* d_rpp = nullptr;
  RppItem* d_items = nullptr;
  rpp::Refine* d_refine = nullptr;
  int32_t *d_jobs0 = nullptr, *d_jobs1 = nullptr;  // RPP ObjPose job queues
  RppQueue* d_rq = nullptr;
  int rpp_blocks = 0;
  // ObjPose tail compaction (k_objpose_q rounds): two spill pools of op_cap
  // lanes (kOpFields doubles + a job id each), their counters, rounds per queue
  double* d_opool[2] = {nullptr, nullptr};
  int32_t* d_ojob[2] = {nullptr, nullptr};
  int32_t* d_octl = nullptr;  // [queue][round]: entries, next (zeroed once per RPP launch sequence)
  int32_t op_cap = 0;
  int op_rounds = 6, op_spill = 32;
  // small batches (latency): ObjPose jobs per wave and rounds (MANTIS_OP_LANES_SMALL, MANTIS_OP_ROUNDS_SMALL).
  // Fewer jobs per wave measured slower once correct (one per wave in one round:
  // rpp_first 3.28 -> 3.64 / 3.80 ms, profiles/r04_p50_objpose_lanes_fixed.txt)
  int op_lanes_small = 64, op_rounds_small = 6;
  int seg_m = 64;        // border-walk checkpoint rows (k_seg_plan; 0: borders walked whole)
  int canny_strip = 2;  // k_canny_strip: 2 = 8 columns per lane where W % 8 == 0, 1 = 4 columns; 0 = tiles (MANTIS_CANNY_STRIP)
  // the same for batches of at most fc_small_frames frames (the rig-latency
  // path): tiles, whose ~230 blocks per frame run at once, where the strip
  // walk of a frame is 720 dependent row steps (MANTIS_CANNY_STRIP sets both)
  int canny_small = 0;
#ifndef MK_SHIFT_SPLIT
#define MK_SHIFT_SPLIT 0
#endif
  bool shift_split = MK_SHIFT_SPLIT;
#ifndef MK_GN_FUSED_ALL
#define MK_GN_FUSED_ALL 1  // round 6: 29.2 / 29.3k -> 29.7 / 30.0k rig poses/s (6 contexts, A/B/A/B)
#endif
  bool gn_fused_all = MK_GN_FUSED_ALL;  // the rig GN as one k_rig_gn_fused launch for every batch size (MANTIS_GN_FUSED)
  bool pf_shifts = true;  // large batches: the 81 shifts at the end of k_score_pf (MANTIS_PF_SHIFTS)
  int pf_init = 1;  // large batches: k_score_init's work at the start of k_score_pf (MANTIS_PF_INIT; 2: its
                   // per-hypothesis arrays in global scratch, as for more hypotheses than its LDS buffer takes)  // large batches: the 81 shifts in k_score_shift_part blocks (MANTIS_SHIFT_SPLIT)
  bool canny_cat = true;  // k_canny_strip<2> over the frames side by side where W % 32 == 0 (MANTIS_CANNY_CAT=0: per frame)
  bool counted = false;  // included in g_live_ctx
  bool vec_ok = false;
  // dense scoring (mantis_score_argmin): hypotheses, errors, counts; (err, idx) pairs per rank
  double *d_dense_c2w = nullptr, *d_dense_err = nullptr, *d_pairs = nullptr;
  int32_t* d_dense_np = nullptr;
  size_t dense_cap = 0;
  void* d_dense_jobs = nullptr;  // mantis_score_argmin_batch: per-frame DenseJob records
  size_t dense_pairs_cap = 0;    // doubles d_pairs holds (0: the 64-rank single-frame buffer)
  size_t dense_jobs_cap = 0;     // DenseJob records d_dense_jobs holds
  // rig GN (cfg.gn_enable): per-camera inv(T_base_cam), per-rig poses, correspondences
  GnCam* d_gncam = nullptr;
  RigGnIO* d_rigio = nullptr;
  double* d_gnobs = nullptr;
  double* d_gnacc = nullptr;  // per-rig accumulator slots (kGnSlot doubles), all-reduced across camera shards
  int gn_rigs = 0, gn_cpr = 0;
  int gn_last_rigs = 0, gn_last_local = 0;  // shape of the last rig GN run (mantis_get_rig_gn)
  HypRec *d_gen = nullptr, *d_hyps = nullptr;
  FrameState* d_st = nullptr;
  ScoreState* d_sst = nullptr;  // scoring state between k_score_init / _pf / _final
  FrameDebug* d_dbg = nullptr;
  mantis_cam_result* d_res = nullptr;
  float* d_gauss = nullptr;
  int32_t* d_gtotal = nullptr;
  // pinned host
  float* h_gauss = nullptr;
  uint64_t* h_states = nullptr;
  mantis_cam_result* h_res = nullptr;
  FrameState* h_st = nullptr;
  int32_t* h_gtotal = nullptr;
  FrameDesc* h_frames = nullptr;
  // profiling
  bool prof = false;
  std::vector<std::string> ev_names;
  std::vector<hipEvent_t> ev;
  std::vector<float> last_ms;
  std::vector<std::string> last_names;
  std::vector<void*> user_allocs;
  // multi-GPU
  void* comm = nullptr;  // ncclComm_t
  int nranks = 1, rank = 0;
  double* d_gn28 = nullptr;
  // camera-sharded rigs (mantis_process_rig_sharded): local frames' global
  // indices, gathered (global index, PF flag) pairs, global PF flags, result records
  int32_t *d_sh_gidx = nullptr, *d_sh_pf = nullptr, *d_sh_flags = nullptr;
  int32_t* h_sh_flags = nullptr;
  size_t sh_cap = 0;  // global frames the shard buffers hold
  uint8_t *d_sh_rec = nullptr, *h_sh_rec = nullptr;
  size_t sh_rec_bytes = 0;
  int gauss_cap = 0;  // frames of gaussians h_gauss / d_gauss / h_states hold
  // legacy rig weighting (cfg.rig_weighting): jobs, (sum, count) per job, the
  // last batch's record per rig (mantis_get_rig_weights)
  RigWJob* d_rwjobs = nullptr;
  double* d_rwout = nullptr;
  size_t rw_cap = 0;
  int rw_rigs = 0, rw_C = 0;
  std::vector<double> rw_weights, rw_c2w, rw_sums;
  std::vector<int32_t> rw_chosen;
  // mantisService motion (mantis_process with a mantis_motion): the last published rig pose
  bool has_prior = false;
  double prior_Twb[16];
  // Markov yaw filters (markov_impl.hip): markov_n planes of 360 bins, per-filter operations
  double* d_markov = nullptr;
  MarkovOp* d_mops = nullptr;
  int markov_n = 0;
  int32_t* d_agree = nullptr;  // sharded calls: the failure flag all-reduced by agree()
  bool agreed_fail = false;     // the last failure was agreed on by every rank (agree())
  // hipGraphs of the rig-latency path (batches of at most fc_small_frames
  // frames): the call's device work as two graphs -- image stages .. RPP ..
  // gaussian offsets, then scoring + result copies -- captured once per call
  // shape and replayed (MANTIS_GRAPHS=0, or the runtime's graph packet
  // capture on: every kernel launched directly)
  struct CallGraph {
    int n = 0, W = 0, H = 0, live = 0, nw = 0, nr = 0, ng = 0;
    bool vec = false;
    const void* lm = nullptr;
    const void* gauss = nullptr;
    hipGraphExec_t pre = nullptr, post = nullptr;
  };
  std::vector<CallGraph> graphs;
  bool use_graphs = false;
  // MANTIS_SCREEN=0 at mantis_create: the fast scorers' FP32 projection screen is
  // off (every landmark takes the exact FP64 fallback; a test / A-B switch)
  bool screen_off = false;
  std::vector<std::pair<Cam, ScreenCam>> scam_cache;  // screen_cam_cached
};

// Camera-sharded calls: every rank must enter the same collectives in the same
// order. A rank-local failure (an image the staging rejects, an allocation, a
// launch error) is agreed on before each exchange phase with one small
// ncclAllReduce (max of a failure flag, 4 bytes), so every rank returns
// together -- the failing rank its own error, the others MANTIS_ERR_COMM --
// instead of leaving them blocked in an all-gather.
// `count` (>= 0): a size every rank must pass identically (the frame count of a
// batched exchange); ranks that disagree all fail with MANTIS_ERR_ARG instead
// of issuing collectives of different sizes.
mantis_status agree(Ctx* c, mantis_status local, int32_t count = -1) {
  c->agreed_fail = false;
  if (!c->comm || !c->d_agree) return local;
  int32_t v[3] = {local != MANTIS_OK ? 1 : 0, count, -count};  // max of each: flag, max count, -min count
  if (hipMemcpyAsync(c->d_agree, v, sizeof(v), hipMemcpyHostToDevice, c->s) != hipSuccess ||
      ncclAllReduce(c->d_agree, c->d_agree, 3, ncclInt32, ncclMax, (ncclComm_t)c->comm, c->s) != ncclSuccess ||
      hipMemcpyAsync(v, c->d_agree, sizeof(v), hipMemcpyDeviceToHost, c->s) != hipSuccess ||
      hipStreamSynchronize(c->s) != hipSuccess) {
    c->err = "agreement all-reduce failed";
    return MANTIS_ERR_COMM;
  }
  const bool mismatch = v[1] != -v[2];
  c->agreed_fail = v[0] != 0 || mismatch;
  if (local != MANTIS_OK) return local;
  if (v[0]) {
    c->err = "another rank of the communicator failed before this exchange (see its mantis_last_error)";
    return MANTIS_ERR_COMM;
  }
  if (mismatch) {
    c->err = "ranks passed different frame counts to a batched exchange (every rank must pass the same n_frames)";
    return MANTIS_ERR_ARG;
  }
  return MANTIS_OK;
}

// the map as the scoring kernels read it: FP64 triples, then the FP32 screen table
inline Landmarks lmk_of(const Ctx* c) {
  return Landmarks{c->d_lm, c->nw, c->nr, c->ng, c->d_lm ? (const float4*)(c->d_lm + kLmfOffset) : nullptr};
}

void mark(Ctx* c, const char* name) {
  if (!c->prof) return;
  if (c->ev.size() <= c->ev_names.size()) {
    hipEvent_t e;
    (void)hipEventCreate(&e);
    c->ev.push_back(e);
  }
  (void)hipEventRecord(c->ev[c->ev_names.size()], c->s);
  c->ev_names.push_back(name);
}

// Wait for everything queued on the ctx's stream: a blocking-sync event for
// batches of more than spin_frames frames (the thread sleeps), else a spin.
struct Ctx;
hipError_t wait_stream(Ctx* c, int frames);

// Entry points may be called from any host thread (one ctx per thread at a
// time): make the ctx's GPU current on the calling thread.
inline void bind_device(const Ctx* c) {
  int d = -1;
  if (hipGetDevice(&d) != hipSuccess || d != c->cfg.device) (void)hipSetDevice(c->cfg.device);
}

// dynamic LDS of k_morph: three band buffers of (bh + 2 MB_HALO) rows
inline size_t morph_lds(int W, int bh) { return (size_t)3 * (bh + 2 * MB_HALO) * ((W + 31) / 32) * sizeof(uint32_t); }

inline int blocks_for(size_t n, int per = 256, int cap = 4096) {
  size_t b = (n + per - 1) / per;
  return (int)std::min<size_t>(std::max<size_t>(b, 1), (size_t)cap);
}

Cam cam_from(const mantis_image& im) {
  Cam m;
  m.fx = (double)(float)im.K[0];
  m.fy = (double)(float)im.K[4];
  m.cx = (double)(float)im.K[2];
  m.cy = (double)(float)im.K[5];
  for (int k = 0; k < 4; k++) m.k[k] = im.D[k];
  return m;
}

// FP32 screen constants of a camera (mk_screen.h screen_cam_from bounds the
// distortion curve over 4096 pieces: ~0.1 ms), memoised per context on the
// intrinsics: the frames of a batch share a few cameras
ScreenCam screen_cam_cached(Ctx* c, const Cam& cm) {
  for (const auto& e : c->scam_cache)
    if (std::memcmp(&e.first, &cm, sizeof(Cam)) == 0) return e.second;
  ScreenCam sc = screen_cam_from(cm);
  if (c->screen_off) sc.sens = INFINITY;  // MANTIS_SCREEN=0: every landmark through the exact fallback
  if (c->scam_cache.size() >= 64) c->scam_cache.erase(c->scam_cache.begin());
  c->scam_cache.emplace_back(cm, sc);
  return sc;
}

template <class T>
mantis_status dalloc(Ctx* c, T** p, size_t count);

// Stage the frames into the batch: device-resident contiguous inputs are
// used in place; everything else is copied (pitch-converted) into d_bgr.
mantis_status stage_frames(Ctx* c, const mantis_image* cams, int n, int& W, int& H) {
  if (n <= 0 || n > c->F) { c->err = "frame count exceeds max_cams"; return MANTIS_ERR_ARG; }
  W = cams[0].width;
  H = cams[0].height;
  if (W <= 2 || H <= 2 || W > c->Wmax || H > c->Hmax) { c->err = "image size outside [3, max]"; return MANTIS_ERR_ARG; }
  const size_t fb = (size_t)W * H * 3;
  for (int i = 0; i < n; i++) {
    const mantis_image& im = cams[i];
    if (im.width != W || im.height != H) { c->err = "all cameras of a batch must share one size"; return MANTIS_ERR_ARG; }
    if (!im.bgr || im.step_bytes < 3 * W) { c->err = "bgr8 image with step >= 3*width required"; return MANTIS_ERR_ARG; }
    FrameDesc& fd = c->h_frames[i];
    fd.w = W;
    fd.h = H;
    fd.cam = cam_from(im);
    fd.scam = screen_cam_cached(c, fd.cam);
    if (im.mem_kind == 1 && im.step_bytes == 3 * W) {
      fd.bgr = im.bgr;
    } else {
      if (!c->d_bgr) {
        // the staging buffer only exists once a host (or pitched) frame arrives:
        // device-resident callers keep its max_cams x 3 W H bytes of HBM
        if (dalloc(c, &c->d_bgr, (size_t)c->F * c->Wmax * c->Hmax * 3) != MANTIS_OK) {
          c->d_bgr = nullptr;
          c->err = "hipMalloc of the frame staging buffer failed";
          return MANTIS_ERR_OOM;
        }
      }
      uint8_t* dst = c->d_bgr + (size_t)i * fb;
      HIP_OK(hipMemcpy2DAsync(dst, 3 * W, im.bgr, im.step_bytes, 3 * W, H,
                              im.mem_kind == 1 ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->s));
      fd.bgr = dst;
    }
  }
  c->vec_ok = (W % 4) == 0;
  for (int i = 0; i < n; i++) c->vec_ok = c->vec_ok && ((uintptr_t)c->h_frames[i].bgr & 3) == 0;
  HIP_OK(hipMemcpyAsync(c->d_frames, c->h_frames, sizeof(FrameDesc) * n, hipMemcpyHostToDevice, c->s));
  return MANTIS_OK;
}

mantis_status run_hyst_ccl(Ctx* c, int n, int W, int H, bool edge_bytes);
// border walks on an LDS copy of the padded plane (small batches) or on the tiled plane in L2
bool trace_on_lds(const Ctx* c, int n, int Wp, int Hp) {
  const size_t tb_lds = (size_t)dbits_wpw(Wp) * Hp * sizeof(uint32_t);
  return c->trace_lds_ok && tb_lds <= c->trace_lds_max && n <= c->trace_lds_frames;
}
mantis_status run_hysteresis(Ctx* c, int n, int W, int H, bool edge_bytes);
#ifndef MK_MW_ROLES
#define MK_MW_ROLES 2  // k_morph_walk waves per segment: detector and mask chains apart (1: one wave does both)
#endif

// gray..Canny, hysteresis, detector binary (padded) and clean mask
mantis_status run_image_stages(Ctx* c, int n, int W, int H, bool edge_bytes = false, bool det_bytes = false) {
  const size_t P = c->plane;
  mark(c, "start");
  const size_t B = c->bstride;
  const int tgx = (W + FTW - 1) / FTW, tgy = (H + FTH - 1) / FTH;
  const int cstrip = n <= c->fc_small_frames ? c->canny_small : c->canny_strip;
  if (cstrip >= 2 && c->vec_ok && W % 8 == 0 && W >= 16 && H >= 3) {
    // column strips walked by one wave each, 8 columns per lane (W % 8 == 0)
    // W % 32 == 0: the strips tile the frames laid side by side (no partial strip per frame)
    const int ns = (W + StripGeom<2>::cols - 1) / StripGeom<2>::cols;
    const bool cat = c->canny_cat && W % 32 == 0;
    const int nw = cat ? (int)(((int64_t)n * W + StripGeom<2>::cols - 1) / StripGeom<2>::cols) : ns * n;
    k_canny_strip<2><<<(unsigned)((nw + 3) / 4), 256, 0, c->s>>>(c->d_frames, c->cfg.canny_low, 3 * c->cfg.canny_low,
                                                                 c->d_b1, c->d_b2, B, ns, nw, cat ? 1 : 0, n);
    mark(c, "canny_nms/k_canny_strip<2>");
  } else if (cstrip && c->vec_ok && W >= 8 && H >= 3) {
    // 4 columns per lane (W % 4 == 0, dword-aligned rows)
    const int ns = (W + StripGeom<1>::cols - 1) / StripGeom<1>::cols, nw = ns * n;
    k_canny_strip<1><<<(unsigned)((nw + 3) / 4), 256, 0, c->s>>>(c->d_frames, c->cfg.canny_low, 3 * c->cfg.canny_low,
                                                                 c->d_b1, c->d_b2, B, ns, nw, 0, n);
    mark(c, "canny_nms/k_canny_strip<1>");
  } else {
    k_canny<<<(unsigned)(tgx * tgy * n), 256, 0, c->s>>>(c->d_frames, c->cfg.canny_low, 3 * c->cfg.canny_low,
                                                        c->vec_ok ? 1 : 0, c->d_b1, c->d_b2, B, tgx, tgy);
    mark(c, "canny_nms/k_canny");
  }
  if (mantis_status hs = run_hysteresis(c, n, W, H, edge_bytes); hs != MANTIS_OK) return hs;
  // detector binary (padded bit plane) and clean mask (bit plane), one fused pass
  // the contour stage's frame states are zeroed here: the walker's run
  // numbering writes n_runs
#ifdef MK_HYST_TICKS  // diagnostics: keep k_hyst_band's ticks
  {
    const size_t a = offsetof(FrameState, ticks), b = a + sizeof(FrameState::ticks);
    HIP_OK(hipMemset2DAsync(c->d_st, sizeof(FrameState), 0, a, n, c->s));
    HIP_OK(hipMemset2DAsync((char*)c->d_st + b, sizeof(FrameState), 0, sizeof(FrameState) - b, n, c->s));
  }
#else
  HIP_OK(hipMemsetAsync(c->d_st, 0, sizeof(FrameState) * n, c->s));
#endif
  c->runs_done = false;
  if (c->morph_walk > 0 && bits::words(W) <= 62 && dbits_wpw(W + 2) <= 63) {
    // register walker: one wave per (frame, row segment); with one segment per
    // frame it also numbers the detector runs (k_run_count / scan / emit)
    // small batches (latency): short segments, many waves per frame (the
    // walk down a whole frame is ~1 ms of dependent steps)
    const int seg = n <= c->fc_small_frames ? c->morph_walk_small : c->morph_walk;
    const int nseg = (H + seg - 1) / seg, nwv = nseg * n * MK_MW_ROLES;
    const WalkRuns wr{c->d_rowb, c->rstride, c->d_lroot, c->d_lab, c->plane, c->d_st};
    if (nseg == 1) {
      k_morph_walk<true><<<(unsigned)((nwv + 3) / 4), 256, 0, c->s>>>(c->d_eb, c->d_dbits, c->d_mbits, W, H, B,
                                                                      c->dstride, seg, nseg, nwv, wr, MK_MW_ROLES);
      c->runs_done = true;
    } else {
      k_morph_walk<false><<<(unsigned)((nwv + 3) / 4), 256, 0, c->s>>>(c->d_eb, c->d_dbits, c->d_mbits, W, H, B,
                                                                       c->dstride, seg, nseg, nwv, wr, MK_MW_ROLES);
    }
    mark(c, "morph/k_morph_walk");
  } else {
    dim3 gm((H + c->morph_bh - 1) / c->morph_bh, n);
    k_morph<<<gm, MB_THREADS, morph_lds(W, c->morph_bh), c->s>>>(c->d_eb, c->d_dbits, c->d_mbits, W, H, B, c->dstride,
                                                                c->morph_bh);
    mark(c, "morph/k_morph");
  }
  if (det_bytes) k_bits_to_bytes<<<blocks_for((size_t)(W + 2) * (H + 2)), 256, 0, c->s>>>(c->d_dbits, c->d_det, W + 2, H + 2,
                                                                                          dbits_wpw(W + 2));
  HIP_OK(hipGetLastError());
  return MANTIS_OK;
}

// cv::Canny's hysteresis on the candidate / strong planes (d_b1, d_b2) -> edge plane d_eb
mantis_status run_hysteresis(Ctx* c, int n, int W, int H, bool edge_bytes) {
  const size_t B = c->bstride;
  const size_t hr_lds = (size_t)((H + HR_ROWS - 1) / HR_ROWS) * HR_ROWS * bits::words(W) * sizeof(uint32_t);
  if (c->hyst_rec && bits::words(W) <= 63 && H <= HR_ROWS * HR_MAXW && hr_lds <= c->hyst_rec_lds) {
    // bit-parallel reconstruction: one block per frame, one wave per HR_ROWS-row band, the candidates in LDS
    k_hyst_rec<<<n, 64 * ((H + HR_ROWS - 1) / HR_ROWS), hr_lds, c->s>>>(c->d_b1, c->d_b2, c->d_eb, B, W, H, c->d_st);
    if (edge_bytes) k_bits_to_bytes<<<blocks_for((size_t)W * H), 256, 0, c->s>>>(c->d_eb, c->d_edge, W, H, 0);
    mark(c, "hysteresis/k_hyst_rec");
    HIP_OK(hipGetLastError());
    return MANTIS_OK;
  }
  return run_hyst_ccl(c, n, W, H, edge_bytes);
}

// hysteresis as a run CCL: frames past the reconstruction kernel's reach
// (W > 2016, H > 720 or the candidate plane past the LDS) and MANTIS_HYST_REC=0 (its planes are free again
// before the contour CCL reuses them)
mantis_status run_hyst_ccl(Ctx* c, int n, int W, int H, bool edge_bytes) {
  const size_t P = c->plane, B = c->bstride;
  // mark values 4..255 (the denser bands' flags are <= 3); the flag plane is cleared when they wrap
  c->hyst_epoch = c->hyst_epoch >= 255 ? 4 : c->hyst_epoch + 1;
  if (c->hyst_epoch == 4) HIP_OK(hipMemsetAsync(c->d_strong, 0, c->fstride * (size_t)c->F, c->s));
  HystRuns hr{(uint32_t*)c->d_lroot, c->d_lab, c->d_strong, c->d_rowb, c->lstride / 2, P, c->fstride, c->rstride, P / 2,
              HB_ROWS * ((W + 1) / 2), c->d_st, c->hyst_epoch};
  // list counters |A|, |B| of every frame (rowb[H + 1], rowb[H + 2])
  HIP_OK(hipMemset2DAsync(c->d_rowb + H + 1, c->rstride * sizeof(int32_t), 0, 2 * sizeof(int32_t), n, c->s));
  const int WWb = bits::words(W);
  k_hyst_band<<<dim3((H + HB_ROWS - 1) / HB_ROWS, n), HB_THREADS, 3 * sizeof(uint32_t) * HB_ROWS * WWb, c->s>>>(
      c->d_b1, c->d_b2, B, hr, c->d_eb, W, H);
  mark(c, "hysteresis/k_hyst_band");
  const int nseam = (H - 1) / HB_ROWS;
  if (nseam > 0) k_hyst_seam<<<dim3((nseam + 3) / 4, n), 256, 0, c->s>>>(hr, H);
  mark(c, "hysteresis/k_hyst_seam");
  k_hyst_mark<<<dim3(8, n), 256, 0, c->s>>>(hr, H);
  mark(c, "hysteresis/k_hyst_mark");
  k_hyst_fix<<<dim3(8, n), 256, 0, c->s>>>(hr, c->d_eb, B, W, H);
  if (edge_bytes) k_bits_to_bytes<<<blocks_for((size_t)W * H), 256, 0, c->s>>>(c->d_eb, c->d_edge, W, H, 0);
  mark(c, "hysteresis/k_hyst_fix");
  HIP_OK(hipGetLastError());
  return MANTIS_OK;
}

mantis_status run_contours(Ctx* c, int n, int W, int H) {
  const size_t P = c->plane;
  const int Wp = W + 2, Hp = H + 2;
  dim3 grow((Hp + 4 * RUN_RPW - 1) / (4 * RUN_RPW), n);  // k_run_count / emit / border: RUN_RPW rows per wave
  uint16_t* rx = c->d_lroot;  // free after hysteresis: run starts (u16, one run per pixel at most)
  if (!c->runs_done) {  // the morphology walker numbered the runs already
    k_run_count<<<grow, 256, 0, c->s>>>(c->d_dbits, c->dstride, c->d_rowb, c->rstride, Wp, Hp);
    k_run_scan<<<n, 256, 0, c->s>>>(c->d_rowb, c->rstride, c->d_st, Hp);
    k_run_emit<<<grow, 256, 0, c->s>>>(c->d_dbits, c->dstride, c->d_rowb, c->rstride, rx, c->d_lab, P, Wp, Hp);
  }
  k_run_band<<<dim3((Hp + RB_ROWS - 1) / RB_ROWS, n), RB_THREADS, 0, c->s>>>(c->d_rowb, c->rstride, rx, c->d_lab, P, Wp, Hp);
  const int seams = (Hp - 1) / RB_ROWS;
  if (seams > 0)
    k_run_seam<<<dim3((seams + 3) / 4, n), 256, 0, c->s>>>(c->d_rowb, c->rstride, rx, c->d_lab, P, Wp, Hp);
  k_run_border<<<grow, 256, 0, c->s>>>(c->d_rowb, c->rstride, rx, c->d_lab, P, c->d_borders, c->d_st, Wp, Hp,
                                       kMaxBorders);
  mark(c, "components");
  const size_t tb_lds = (size_t)dbits_wpw(Wp) * Hp * sizeof(uint32_t);
  k_seg_plan<<<n, 256, 0, c->s>>>(c->d_dbits, c->dstride, c->d_rowb, c->rstride, rx, c->d_lab, P, c->d_borders,
                                  c->d_st, c->d_scratch, c->pool_cap, Wp, Hp, kMaxBorders, c->seg_m);
  if (trace_on_lds(c, n, Wp, Hp)) {
    k_trace_borders_lds<<<n, 1024, tb_lds, c->s>>>(c->d_dbits, c->dstride, c->d_borders, c->d_st, c->d_scratch,
                                                   c->pool_cap, Wp, Hp, kMaxBorders, c->d_rowb, c->rstride, rx, P);
  } else {
    const int wpw = dbits_wpw(Wp);
    k_tile_bits<<<dim3((Hp + 31) / 32, n), 256, kTbRows * wpw * sizeof(uint32_t), c->s>>>(
        c->d_dbits, c->dstride, c->d_tbits, c->tstride, wpw, Wp, Hp);
    k_trace_borders<<<n, 64 * MK_TB_WAVES, 0, c->s>>>(c->d_tbits, c->tstride, c->d_borders, c->d_st, c->d_scratch, c->pool_cap, Wp,
                                        kMaxBorders, c->d_rowb, c->rstride, rx, P);
  }
  k_seg_chain<<<n, 256, 0, c->s>>>(c->d_st, c->d_bcount, c->d_scratch, c->pool_cap, kMaxBorders);
  mark(c, "border_trace");
  // small batches (latency): 1024 threads per frame; large ones: 256, so the
  // per-frame blocks fit beside other contexts' kernels on a CU
  k_frame_contours<<<n, n <= c->fc_small_frames ? 1024 : MK_FC_THREADS, 0, c->s>>>(c->d_dbits, c->dstride, c->d_borders, c->d_st, c->d_bcount, c->d_boff,
                                         c->d_pool, c->d_scratch, c->pool_cap, c->d_quads, c->d_dbg, c->d_frames, Wp,
                                         Hp, P, kMaxBorders, (double)c->cfg.polygon_epsilon,
                                         c->cfg.search_radius_multiplier, c->d_rowb, c->rstride, rx);
  mark(c, "contours_quads");
  HIP_OK(hipGetLastError());
  return MANTIS_OK;
}

// Live contexts per device in this process: the persistent ObjPose lanes are
// latency-bound (a long dependent FP64 chain per lane), and at 224 VGPRs two
// resident blocks per CU hold most of its register file, so with several
// contexts sharing a GPU each takes a proportional share of the CUs and
// leaves the rest to the other contexts' kernels (3 contexts: +5 % rig
// poses/s over filling every CU, bench sweep in DESIGN.md).
std::atomic<int> g_live_ctx[64];

// Grid of a persistent ObjPose launch: two lanes per job at the
// typical ~150 items per frame, at most 1.5 * CUs / (live contexts on the
// device) blocks (MANTIS_RPP_BLOCKS overrides).
unsigned objpose_blocks(const Ctx* c, size_t expected_jobs) {
  size_t b = (expected_jobs + 127) / 128;  // ~0.5 jobs per lane: small batches start every job at once
  const int live = std::max(1, g_live_ctx[c->cfg.device & 63].load());
  const size_t cap = c->rpp_blocks > 0 ? (size_t)c->rpp_blocks : (size_t)std::max(64, 3 * c->n_cu / (2 * live));
  return (unsigned)std::max<size_t>(1, std::min(b, cap));
}

// paired: pipeline items (orientation pairs of each quad, k_rpp_prep); the
// first queue holds orientation 0 only and op_end<0> mirrors its result
// One ObjPose queue as op_rounds launches over one grid (k_objpose_q, tail
// compaction): round 0 serves the job list, every later round the states the
// previous one spilled, the last runs every job to the end.
constexpr int kOpMaxRounds = 16;  // ObjPose tail-compaction rounds per queue at most
template <int MODE>
mantis_status run_objpose_rounds(Ctx* c, unsigned blocks, RppItem* items, rpp::Refine* rf, const int32_t* jobs,
                                 RppQueue* q, FrameState* st, int paired, int lanes = 64, int rounds = 0) {
  if (rounds <= 0) rounds = std::max(1, c->op_rounds);
  if ((size_t)blocks * 256 > (size_t)c->op_cap) blocks = (unsigned)(c->op_cap / 256);  // a pool holds a grid's lanes
  for (int r = 0; r < rounds; r++) {
    const int in = (r + 1) & 1, out = r & 1;
    OpRound rd;
    // counters per (queue, round), all zeroed before the first queue (no
    // memset launch between rounds); the data pools alternate
    int32_t* ctl = c->d_octl + 2 * (MODE * kOpMaxRounds);
    rd.in = OpPool{c->d_opool[in], c->d_ojob[in], ctl + 2 * (r > 0 ? r - 1 : 0)};
    rd.out = OpPool{c->d_opool[out], c->d_ojob[out], ctl + 2 * r};
    rd.cap = c->op_cap;
    rd.first = r == 0;
    rd.last = r == rounds - 1;
    rd.spill_below = c->op_spill;
    rd.lanes = lanes;
    rd.pad = 0;
    k_objpose_q<MODE><<<blocks, 256, 0, c->s>>>(items, rf, jobs, q, st, paired, rd);
  }
  return MANTIS_OK;
}

#ifndef MK_S1B_WPC
#define MK_S1B_WPC 32  // k_rpp_s1b waves per CU at most (a grid-stride loop over the items; 8: rpp_2nd 2.1 vs 1.8 ms per 4096 frames)
#endif
void launch_rpp_queues(Ctx* c, RppItem* items, rpp::Refine* rf, int32_t* jobs0, int32_t* jobs1, RppQueue* q,
                       RppOut* out, FrameState* st, size_t ni, size_t expected_items, const QuadRec* quads,
                       bool paired, bool small = false) {
  const int pr = paired ? 1 : 0;
  // every (queue, round) counter pair of this launch sequence, once
  (void)hipMemsetAsync(c->d_octl, 0, sizeof(int32_t) * 2 * 2 * kOpMaxRounds, c->s);
  // small batches: at most op_lanes_small jobs per wave, the grid sized for that
  const int lanes = small ? c->op_lanes_small : 64, rounds = small ? c->op_rounds_small : 0;
  auto blocks_for = [&](size_t jobs) {
    if (lanes >= 64) return objpose_blocks(c, jobs);
    return (unsigned)std::max<size_t>(1, std::min<size_t>((jobs + 4 * lanes - 1) / (4 * lanes), (size_t)c->op_cap / 256));
  };
  run_objpose_rounds<0>(c, blocks_for(paired ? expected_items / 2 : expected_items), items, rf, jobs0, q, st, pr,
                        lanes, rounds);
  mark(c, "rpp_first");
  k_rpp_s1b<<<(unsigned)std::min<size_t>((expected_items + 63) / 64, (size_t)c->n_cu * MK_S1B_WPC), 64, 0, c->s>>>(
      items, jobs0, jobs1, q, pr);
  mark(c, "rpp_2nd");
  run_objpose_rounds<1>(c, blocks_for(expected_items * 2), items, rf, jobs1, q, st, 0, lanes, rounds);
  mark(c, "rpp_cand");
  k_rpp_merge<<<(unsigned)((ni + 255) / 256), 256, 0, c->s>>>(items, ni, rf, out, quads,
                                                               quads ? c->cfg.quad_gn_iterations : 0);
  mark(c, "rpp_merge");
}

mantis_status run_pose(Ctx* c, int n) {
  HIP_OK(hipMemsetAsync(c->d_rq, 0, sizeof(RppQueue), c->s));
  dim3 gr((kMaxQuads * 2 + 255) / 256, n);
  k_rpp_prep<<<gr, 256, 0, c->s>>>(c->d_quads, c->d_st, c->d_items, c->d_jobs0, c->d_rq, c->cfg.grid_spacing / 2);
  const size_t ni = (size_t)n * kMaxQuads * 2;
  mark(c, "rpp_prep");
  launch_rpp_queues(c, c->d_items, c->d_refine, c->d_jobs0, c->d_jobs1, c->d_rq, c->d_rpp, c->d_st, ni, (size_t)n * 160,
                    c->d_quads, true, n <= c->fc_small_frames);
  k_frame_hyps<<<n, 256, 0, c->s>>>(c->d_rpp, c->d_st, c->d_gen, c->d_hyps, c->d_dbg, 0.5, 0.2);
  mark(c, "hyps_cluster");
  HIP_OK(hipGetLastError());
  return MANTIS_OK;
}

// Camera-sharded rig call (mantis_process_rig_sharded): this rank's frames are
// some cameras of each rig; the cv::RNG stream is consumed in global
// (rig-major camera) order, as one sequential run over all cameras would.
struct Shard {
  int n_global;         // frames over all ranks (n_rigs * cams_per_rig)
  int slots;            // (global index, PF flag) pairs each rank contributes
  const int32_t* gidx;  // host: global frame index of each local frame
};

// Gaussian-stream offsets of the frames that reach the particle filter. One
// rank: a prefix over the batch. Sharded: the frames' PF flags are gathered
// from every rank (ncclAllGather of (global index, flag) pairs) and each local
// frame takes the prefix at its global index.
mantis_status gauss_offsets(Ctx* c, int n, const Shard* sh) {
  const int per = c->cfg.particles * c->cfg.iterations * 6;
  if (!sh) {
    k_gauss_offsets<<<1, kGaussOffThreads, 0, c->s>>>(c->d_st, n, per, c->d_gtotal);
    HIP_OK(hipGetLastError());
    return MANTIS_OK;
  }
  HIP_OK(hipMemcpyAsync(c->d_sh_gidx, sh->gidx, sizeof(int32_t) * n, hipMemcpyHostToDevice, c->s));
  int32_t* send = c->d_sh_pf;
  int32_t* recv = c->d_sh_pf + 2 * (size_t)sh->slots;
  k_shard_pf_pack<<<(sh->slots + 255) / 256, 256, 0, c->s>>>(c->d_st, c->d_sh_gidx, n, sh->slots, send);
  ncclResult_t r = ncclAllGather(send, recv, 2 * (size_t)sh->slots, ncclInt32, (ncclComm_t)c->comm, c->s);
  if (r != ncclSuccess) { c->err = std::string("ncclAllGather (PF flags): ") + ncclGetErrorString(r); return MANTIS_ERR_COMM; }
  k_gauss_offsets_global<<<1, 1024, 0, c->s>>>(recv, sh->slots * c->nranks, c->d_sh_flags, sh->n_global, c->d_st,
                                               c->d_sh_gidx, n, per, c->d_gtotal);
  mark(c, "pf_exchange");
  HIP_OK(hipGetLastError());
  return MANTIS_OK;
}

// Gaussian stream for up to n frames (frames that skip the PF draw nothing,
// so the stream is contiguous and the device indexes it by prefix offsets).
void gen_gauss(Ctx* c, int n) {  // n <= c->gauss_cap
  const int per = c->cfg.particles * c->cfg.iterations * 6;
  uint64_t s = c->rng_state;
  c->h_states[0] = s;
  for (int f = 0; f < n; f++) {
    float* g = c->h_gauss + (size_t)f * per;
    for (int k = 0; k < per; k++) g[k] = rng_gauss(s);
    c->h_states[f + 1] = s;
  }
}

mantis_status run_score(Ctx* c, int n, int n_gauss, bool copy_gauss = true) {
  const int per = c->cfg.particles * c->cfg.iterations * 6;
  // on the side stream as soon as the host has drawn it (the caller joined the
  // drawing thread), so the copy overlaps the RPP kernels still queued on s;
  // s waits for it only before the scoring kernels. d_gauss / h_gauss are free:
  // the previous batch's call synchronised s, which had waited on this copy.
  // (the side-stream copy: score stage 11.13 / 11.34 -> 10.95 / 10.97 ms per 4096
  // frames in a 6-context A/B against k_score_init reading the pinned buffer)
  if (copy_gauss) {  // (graph calls copy on c->s before the scoring graph)
    HIP_OK(hipMemcpyAsync(c->d_gauss, c->h_gauss, sizeof(float) * per * n_gauss, hipMemcpyHostToDevice, c->s_copy));
    HIP_OK(hipEventRecord(c->ev_gauss, c->s_copy));
    HIP_OK(hipStreamWaitEvent(c->s, c->ev_gauss, 0));
  }
  mark(c, "gauss_h2d");
  Landmarks L = lmk_of(c);
  const bool split = c->pf_split && n <= c->fc_small_frames && c->cfg.particles <= kPfMaxParticles &&
                     c->cfg.iterations > 0;
  // large batches: k_score_init's work at the start of k_score_pf (pf_init), the
  // 81 shifts at its end (pf_shifts), both with the frame's mask in LDS
  const bool pf_shifts = !split && c->pf_shifts;
  const int pf_init = split ? 0 : c->pf_init;
  if (!pf_init) {
    k_score_init<kScoreInit><<<n, kScoreInit, 0, c->s>>>(c->d_frames, c->d_mbits, c->bstride, L, c->d_st, c->d_hyps,
                                                        c->d_res, c->d_dbg, c->d_sst);
    mark(c, "score_pf_yaw/k_score_init");
  }
  // particle filter: 16 waves per frame, each task one particle over a
  // 1/kPfSplit slice of the landmarks (the integer partial sums combine
  // exactly); the frame's mask plane goes to LDS when it fits (pf_mask_lds > 0:
  // 720p yes, 1080p no)
  const size_t ml = c->pf_mask_lds;
  constexpr int ppb = std::max(1, kPfThreads / 64 / kPfSplit);  // particles per block (one task per wave)
  // small batches split the filter's iterations over blocks (MANTIS_PF_SPLIT); the
  // end-of-filter writes (pf_error, the filter's pose) belong to the last
  // iteration's launch, so a config without iterations runs the one-block kernel
  if (split) {
    const int nblk = (c->cfg.particles + ppb - 1) / ppb;
    for (int it = 0; it < c->cfg.iterations; it++)
      k_score_pf_part<kPfThreads, kPfSplit><<<dim3(nblk, n), kPfThreads, 0, c->s>>>(
          c->d_frames, c->d_mbits, c->bstride, L, c->d_st, c->d_gauss, c->d_res, c->d_dbg, c->d_sst, c->cfg.particles,
          c->cfg.iterations, it, ppb, nblk);
  } else if (ml)
    k_score_pf<kPfThreads, kPfSplit, true><<<n, kPfThreads, ml, c->s>>>(
        c->d_frames, c->d_mbits, c->bstride, L, c->d_st, c->d_gauss, c->d_res, c->d_dbg, c->d_sst, c->cfg.particles,
        c->cfg.iterations, pf_shifts ? 1 : 0, c->cfg.grid_spacing, 9, pf_init, c->d_hyps,
        (unsigned char*)c->d_gen);
  else
    k_score_pf<kPfThreads, kPfSplit, false><<<n, kPfThreads, 0, c->s>>>(
        c->d_frames, c->d_mbits, c->bstride, L, c->d_st, c->d_gauss, c->d_res, c->d_dbg, c->d_sst, c->cfg.particles,
        c->cfg.iterations, pf_shifts ? 1 : 0, c->cfg.grid_spacing, 9, pf_init, c->d_hyps,
        (unsigned char*)c->d_gen);
  mark(c, "score_pf_yaw/k_score_pf");
  // the 81 shifts over several blocks per frame first (small batches; large
  // ones with shift_split: the shift tasks in a lean kernel instead of beside
  // k_score_final's sorting, COLOR and publishing code)
  const bool shifts_apart = !pf_shifts && (split || c->shift_split);
  if (shifts_apart) {
    constexpr int spb = kScoreTail / 128;
    k_score_shift_part<kScoreTail><<<dim3((81 + spb - 1) / spb, n), kScoreTail, 0, c->s>>>(
        c->d_frames, c->d_mbits, c->bstride, L, c->d_st, c->d_sst, c->cfg.grid_spacing, 9, spb);
    mark(c, "score_pf_yaw/k_score_shift_part");
  }
  k_score_final<kScoreTail><<<n, kScoreTail, 0, c->s>>>(c->d_frames, c->d_mbits, c->bstride, L, c->d_st, c->d_res, c->d_dbg,
                                               c->d_sst, c->cfg.grid_spacing, 9, shifts_apart || pf_shifts);
  mark(c, "score_pf_yaw/k_score_final");
  HIP_OK(hipGetLastError());
  return MANTIS_OK;
}

void finish_profile(Ctx* c, bool append = false) {
  if (!c->prof || c->ev_names.empty()) return;
  (void)hipEventSynchronize(c->ev[c->ev_names.size() - 1]);
  if (!append) {
    c->last_names.clear();
    c->last_ms.clear();
  }
  for (size_t i = 1; i < c->ev_names.size(); i++) {
    float ms = 0;
    (void)hipEventElapsedTime(&ms, c->ev[i - 1], c->ev[i]);
    c->last_names.push_back(c->ev_names[i]);
    c->last_ms.push_back(ms);
  }
  c->ev_names.clear();
}

hipError_t wait_stream(Ctx* c, int frames) {
  if (frames <= c->spin_frames || !c->ev_wait) return hipStreamSynchronize(c->s);
  hipError_t e = hipEventRecord(c->ev_wait, c->s);
  if (e != hipSuccess) return e;
  return hipEventSynchronize(c->ev_wait);
}

// rig fusion and 4x4 helpers: mk_shard.h (shared with the CPU test build)
using mk::shard::fuse_rig;
using mk::shard::mat4_inv_rigid;
using mk::shard::mat4_mul;
using mk::shard::quat_to_mat4;

template <class T>
mantis_status dalloc(Ctx* c, T** p, size_t count);
template <class T>
mantis_status halloc(Ctx* c, T** p, size_t count);

// gaussian buffers for n frames (a sharded call draws for every rig camera)
mantis_status ensure_gauss(Ctx* c, int n) {
  if (n <= c->gauss_cap) return MANTIS_OK;
  const int per = c->cfg.particles * c->cfg.iterations * 6;
  HIP_OK(hipStreamSynchronize(c->s));
  (void)hipFree(c->d_gauss);
  (void)hipHostFree(c->h_gauss);
  (void)hipHostFree(c->h_states);
  c->d_gauss = nullptr;
  c->h_gauss = nullptr;
  c->h_states = nullptr;
  c->gauss_cap = 0;
  if (dalloc(c, &c->d_gauss, (size_t)n * per) || halloc(c, &c->h_gauss, (size_t)n * per) ||
      halloc(c, &c->h_states, (size_t)n + 1))
    return MANTIS_ERR_OOM;
  c->gauss_cap = n;
  return MANTIS_OK;
}

// Stream capture of one part of a call into an executable graph. A failure
// inside the body ends the capture (the stream leaves capture mode either way)
// and discards what was captured.
template <class F>
mantis_status capture_graph(Ctx* c, hipGraphExec_t* out, F&& body) {
  HIP_OK(hipStreamBeginCapture(c->s, hipStreamCaptureModeThreadLocal));
  const mantis_status st = body();
  hipGraph_t gr = nullptr;
  const hipError_t e = hipStreamEndCapture(c->s, &gr);
  if (st != MANTIS_OK || e != hipSuccess) {
    if (gr) (void)hipGraphDestroy(gr);
    if (st != MANTIS_OK) return st;
    c->err = std::string("hipStreamEndCapture: ") + hipGetErrorString(e);
    return MANTIS_ERR_DEVICE;
  }
  const hipError_t ei = hipGraphInstantiate(out, gr, nullptr, nullptr, 0);
  (void)hipGraphDestroy(gr);
  if (ei != hipSuccess) {
    *out = nullptr;
    c->err = std::string("hipGraphInstantiate: ") + hipGetErrorString(ei);
    return MANTIS_ERR_DEVICE;
  }
  return MANTIS_OK;
}

// The cached graphs of a call shape (created empty, captured by the call), or
// null when the call takes the direct launches: sharded calls (collectives and
// host agreement between the parts), profiling (per-stage events), batches
// past the latency path, and frames whose hysteresis takes the run CCL (its
// per-call mark epoch is a kernel argument). Everything else a launch bakes in
// is part of the key: the shape, whether the frames allow dword loads, the
// live-context count (the ObjPose grid), the map and the gaussian buffer.
Ctx::CallGraph* call_graph(Ctx* c, int n, int W, int H, const Shard* sh) {
  if (!c->use_graphs || sh || c->prof || n > c->fc_small_frames) return nullptr;
  const size_t hr_lds = (size_t)((H + HR_ROWS - 1) / HR_ROWS) * HR_ROWS * bits::words(W) * sizeof(uint32_t);
  if (!(c->hyst_rec && bits::words(W) <= 63 && H <= HR_ROWS * HR_MAXW && hr_lds <= c->hyst_rec_lds)) return nullptr;
  const int live = std::max(1, g_live_ctx[c->cfg.device & 63].load());
  for (auto& g : c->graphs)
    if (g.n == n && g.W == W && g.H == H && g.vec == c->vec_ok && g.live == live && g.lm == c->d_lm &&
        g.nw == c->nw && g.nr == c->nr && g.ng == c->ng && g.gauss == c->d_gauss)
      return &g;
  if (c->graphs.size() >= 8) {  // the oldest shape goes
    if (c->graphs.front().pre) (void)hipGraphExecDestroy(c->graphs.front().pre);
    if (c->graphs.front().post) (void)hipGraphExecDestroy(c->graphs.front().post);
    c->graphs.erase(c->graphs.begin());
  }
  Ctx::CallGraph g;
  g.n = n; g.W = W; g.H = H; g.vec = c->vec_ok; g.live = live;
  g.lm = c->d_lm; g.nw = c->nw; g.nr = c->nr; g.ng = c->ng; g.gauss = c->d_gauss;
  c->graphs.push_back(g);
  return &c->graphs.back();
}

mantis_status process_frames(Ctx* c, const mantis_image* cams, int n, const Shard* sh = nullptr) {
  if (!c->d_lm) { c->err = "map not set (mantis_set_map)"; return MANTIS_ERR_STATE; }
  if (n <= 0 || n > c->F) { c->err = "frame count exceeds max_cams"; return MANTIS_ERR_ARG; }
  const int ng = sh ? sh->n_global : n;
  // the gaussian offsets are int32 on the device (FrameState::gauss_offset)
  if ((int64_t)c->cfg.particles * c->cfg.iterations * 6 * ng > INT32_MAX) {
    c->err = "particles x iterations x 6 x frames (all rig cameras when sharded) exceeds 2^31 gaussians per call";
    return MANTIS_ERR_ARG;
  }
  if (mantis_status e = ensure_gauss(c, ng)) return e;
  // The gaussian stream depends only on the RNG state, so a host thread draws
  // it while the device runs the image stages and RPP (the pinned buffer is
  // not in use: the previous call synchronised).
  struct Joiner {
    std::thread t;
    ~Joiner() { if (t.joinable()) t.join(); }
  } gauss;
  gauss.t = std::thread([c, ng] { gen_gauss(c, ng); });
  int W, H;
  mantis_status st = stage_frames(c, cams, n, W, H);
  const auto results_d2h = [&]() -> mantis_status {
    HIP_OK(hipMemcpyAsync(c->h_res, c->d_res, sizeof(mantis_cam_result) * n, hipMemcpyDeviceToHost, c->s));
    HIP_OK(hipMemcpyAsync(c->h_st, c->d_st, sizeof(FrameState) * n, hipMemcpyDeviceToHost, c->s));
    HIP_OK(hipMemcpyAsync(c->h_gtotal, c->d_gtotal, sizeof(int32_t), hipMemcpyDeviceToHost, c->s));
    return MANTIS_OK;
  };
  Ctx::CallGraph* g = st == MANTIS_OK ? call_graph(c, n, W, H, sh) : nullptr;
  if (g) {
    // the rig-latency path as two graph launches: the frames' descriptors (and
    // any host frames) were copied above, the gaussians are copied between the
    // two launches once the host thread has drawn them
    if (!g->pre)
      st = capture_graph(c, &g->pre, [&]() -> mantis_status {
        mantis_status s2 = run_image_stages(c, n, W, H);
        if (s2 == MANTIS_OK) s2 = run_contours(c, n, W, H);
        if (s2 == MANTIS_OK) s2 = run_pose(c, n);
        if (s2 == MANTIS_OK) s2 = gauss_offsets(c, n, nullptr);
        return s2;
      });
    if (st != MANTIS_OK) return st;
    HIP_OK(hipGraphLaunch(g->pre, c->s));
    gauss.t.join();
    const int per = c->cfg.particles * c->cfg.iterations * 6;
    HIP_OK(hipMemcpyAsync(c->d_gauss, c->h_gauss, sizeof(float) * per * ng, hipMemcpyHostToDevice, c->s));
    if (!g->post)
      st = capture_graph(c, &g->post, [&]() -> mantis_status {
        mantis_status s2 = run_score(c, n, ng, false);
        if (s2 == MANTIS_OK) s2 = results_d2h();
        return s2;
      });
    if (st != MANTIS_OK) return st;
    HIP_OK(hipGraphLaunch(g->post, c->s));
  } else {
    if (st == MANTIS_OK) st = run_image_stages(c, n, W, H);
    if (st == MANTIS_OK) st = run_contours(c, n, W, H);
    if (st == MANTIS_OK) st = run_pose(c, n);
    if (sh) st = agree(c, st);  // before the PF-flag all-gather
    if (st != MANTIS_OK) return st;
    if ((st = gauss_offsets(c, n, sh)) != MANTIS_OK) return st;
    gauss.t.join();
    if ((st = run_score(c, n, ng)) != MANTIS_OK) return st;
    if ((st = results_d2h()) != MANTIS_OK) return st;
  }
  if (sh) HIP_OK(hipMemcpyAsync(c->h_sh_flags, c->d_sh_flags, sizeof(int32_t) * ng, hipMemcpyDeviceToHost, c->s));
  HIP_OK(wait_stream(c, n));
  finish_profile(c);
  const int per = c->cfg.particles * c->cfg.iterations * 6;
  int used = 0;
  if (sh)
    for (int f = 0; f < ng; f++) used += c->h_sh_flags[f] ? 1 : 0;
  for (int f = 0; f < n; f++) {
    if (!sh && c->h_st[f].reaches_pf) used++;
    if (c->h_st[f].overflow) {
      std::ostringstream os;
      os << "frame " << f << ": workspace capacity exceeded (flags " << c->h_st[f].overflow << ", borders "
         << c->h_st[f].n_borders << ", points " << c->h_st[f].n_points << ", raw quads " << c->h_st[f].n_raw_quads
         << ")";
      c->err = os.str();
      c->h_res[f].status = MANTIS_ERR_CAPACITY;
    }
  }
  if (const char* fs = getenv("MANTIS_FRAME_STATS")) {  // diagnostics: one line per frame
    if (FILE* fp = fopen(fs, "a")) {
      for (int f = 0; f < n; f++)
        fprintf(fp, "%d %d %d %d %d %d %d\n", c->h_st[f].n_runs, c->h_st[f].n_borders, c->h_st[f].n_points,
                c->h_st[f].trace_steps_max, c->h_st[f].trace_steps_sum, c->h_st[f].n_chunks, c->h_st[f].trace_ticks);
      fclose(fp);
    }
  }
  if (used * per != *c->h_gtotal) { c->err = "internal: gaussian stream accounting mismatch"; return MANTIS_ERR_DEVICE; }
  c->rng_state = c->h_states[used];
  return MANTIS_OK;
}

template <class T>
mantis_status dalloc(Ctx* c, T** p, size_t count) {
  if (hipMalloc((void**)p, sizeof(T) * std::max<size_t>(count, 1)) != hipSuccess) {
    c->err = "hipMalloc failed";
    return MANTIS_ERR_OOM;
  }
  return MANTIS_OK;
}
// device scratch of one C-ABI call, freed on every return path
struct DevScratch {
  Ctx* c;
  std::vector<void*> p;
  explicit DevScratch(Ctx* ctx) : c(ctx) {}
  template <class T>
  bool get(T** q, size_t count) {  // true on failure (c->err set), like dalloc
    *q = nullptr;
    if (dalloc(c, q, count)) return true;
    p.push_back((void*)*q);
    return false;
  }
  ~DevScratch() {
    if (!p.empty()) (void)hipStreamSynchronize(c->s);
    for (void* q : p) (void)hipFree(q);
  }
};
template <class T>
mantis_status halloc(Ctx* c, T** p, size_t count) {
  if (hipHostMalloc((void**)p, sizeof(T) * std::max<size_t>(count, 1), hipHostMallocDefault) != hipSuccess) {
    c->err = "hipHostMalloc failed";
    return MANTIS_ERR_OOM;
  }
  return MANTIS_OK;
}

// T_base_cam of each camera, 16 doubles per camera
std::vector<double> gather_tbc(const mantis_image* cams, int n) {
  std::vector<double> T(16 * (size_t)n);
  for (int i = 0; i < n; i++) std::memcpy(&T[16 * (size_t)i], cams[i].T_base_cam, sizeof(double) * 16);
  return T;
}

thread_local std::string g_create_err;

}  // namespace

extern "C" {

int32_t mantis_abi_version(void) { return MANTIS_ABI_VERSION; }

void mantis_default_config(mantis_config* cfg) {
  std::memset(cfg, 0, sizeof(*cfg));
  cfg->struct_size = sizeof(mantis_config);
  cfg->device = 0;
  cfg->max_cams = 16;
  cfg->max_width = 1280;
  cfg->max_height = 720;
  cfg->rng_seed = 1;
  cfg->canny_low = 50;
  cfg->polygon_epsilon = 10;
  cfg->search_radius_multiplier = 0.1;
  cfg->grid_spacing = 0.32;
  cfg->particles = 50;
  cfg->iterations = 10;
  cfg->gn_enable = 0;
  cfg->gn_iterations = 10;
  cfg->max_quads = kMaxQuads;
  cfg->max_contour_points = 262144;
  cfg->quad_gn_iterations = 0;
  cfg->rig_weighting = 0;
}

mantis_status mantis_create(const mantis_config* cfg_in, void** out_ctx) {
  if (!out_ctx) return MANTIS_ERR_ARG;
  *out_ctx = nullptr;
  mantis_config cfg;
  mantis_default_config(&cfg);
  if (cfg_in) {
    if (cfg_in->struct_size != (int32_t)sizeof(mantis_config)) {
      g_create_err = "mantis_config.struct_size mismatch";
      return MANTIS_ERR_ARG;
    }
    cfg = *cfg_in;
  }
  if (cfg.max_quads == 0) cfg.max_quads = kMaxQuads;
  // gaussian offsets are int32 on the device (k_gauss_offsets): a batch of
  // max_cams frames must draw fewer than 2^31 (sharded calls check their
  // rig-wide count per call, process_frames)
  if ((int64_t)cfg.particles * cfg.iterations * 6 * (cfg.max_cams > 0 ? cfg.max_cams : 1) > INT32_MAX) {
    g_create_err = "particles x iterations x 6 x max_cams exceeds 2^31 gaussians per batch";
    return MANTIS_ERR_ARG;
  }
  if (cfg.particles < 1 || cfg.particles > 96 || cfg.iterations < 0 || cfg.iterations > 1000 || cfg.max_cams < 1 ||
      cfg.max_width < 3 || cfg.max_height < 3 || cfg.gn_iterations < 0 || cfg.gn_iterations > 10 ||
      cfg.quad_gn_iterations < 0 || cfg.quad_gn_iterations > 20 || cfg.rig_weighting < 0 || cfg.rig_weighting > 1) {
    g_create_err = "invalid config (particles 1..96, iterations 0..1000, gn_iterations 0..10, "
                   "quad_gn_iterations 0..20, max_cams >= 1, image >= 3x3)";
    return MANTIS_ERR_ARG;
  }
  if (cfg.max_width > 8190) {
    g_create_err = "max_width: at most 8190 (the hysteresis bands hold a row's worst-case runs in LDS)";
    return MANTIS_ERR_ARG;
  }
  if (cfg.max_height > 65533) {
    g_create_err = "max_height: at most 65533 (border walks and contour points pack y + 1 in 16 bits)";
    return MANTIS_ERR_ARG;
  }
  if ((int64_t)((cfg.max_height + HB_ROWS - 1) / HB_ROWS) * HB_ROWS * ((cfg.max_width + 1) / 2) >= (1 << 24)) {
    g_create_err = "max_width x max_height: at most 2^25 pixels (hysteresis run ids and their band row share a word)";
    return MANTIS_ERR_ARG;
  }
  if (cfg.max_quads != kMaxQuads) {
    g_create_err = "max_quads: the per-frame quad capacity is fixed at 256 in this build";
    return MANTIS_ERR_ARG;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= cfg.device) {
    g_create_err = "no HIP device available (libmantis_amd requires an MI355X / gfx950 GPU)";
    return MANTIS_ERR_DEVICE;
  }
  Ctx* c = new Ctx();
  c->cfg = cfg;
  c->rng_state = cfg.rng_seed ? cfg.rng_seed : 0xffffffffULL;
  if (hipSetDevice(cfg.device) != hipSuccess || hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->s_copy, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_gauss, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_wait, hipEventDisableTiming | hipEventBlockingSync) != hipSuccess) {
    g_create_err = "hipSetDevice/hipStreamCreate failed";
    if (c->s) (void)hipStreamDestroy(c->s);
    if (c->s_copy) (void)hipStreamDestroy(c->s_copy);
    delete c;
    return MANTIS_ERR_DEVICE;
  }
  if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, cfg.device) != hipSuccess || c->n_cu < 1)
    c->n_cu = 256;
  if (const char* e = std::getenv("MANTIS_RPP_BLOCKS")) c->rpp_blocks = std::atoi(e);
  if (const char* e = std::getenv("MANTIS_OP_ROUNDS")) c->op_rounds = std::max(1, std::min(kOpMaxRounds, std::atoi(e)));
  if (const char* e = std::getenv("MANTIS_OP_SPILL")) c->op_spill = std::max(0, std::min(64, std::atoi(e)));
  if (const char* e = std::getenv("MANTIS_OP_LANES_SMALL")) c->op_lanes_small = std::max(1, std::min(64, std::atoi(e)));
  if (const char* e = std::getenv("MANTIS_OP_ROUNDS_SMALL")) c->op_rounds_small = std::max(1, std::min(kOpMaxRounds, std::atoi(e)));
  if (const char* e = std::getenv("MANTIS_SEG_M")) c->seg_m = std::max(0, std::min(4096, std::atoi(e)));
  if (const char* e = std::getenv("MANTIS_CANNY_STRIP")) c->canny_strip = c->canny_small = std::atoi(e);
  if (const char* e = std::getenv("MANTIS_CANNY_CAT")) c->canny_cat = e[0] != '0';
  if (const char* e = std::getenv("MANTIS_SHIFT_SPLIT")) c->shift_split = e[0] != '0';
  if (const char* e = std::getenv("MANTIS_PF_SHIFTS")) c->pf_shifts = e[0] != '0';
  if (const char* e = std::getenv("MANTIS_GN_FUSED")) c->gn_fused_all = e[0] != '0';
  if (const char* e = std::getenv("MANTIS_PF_INIT")) c->pf_init = std::max(0, std::min(2, std::atoi(e)));
  if (const char* e = std::getenv("MANTIS_HYST_REC")) c->hyst_rec = e[0] != '0';
  {
    // graph replays need the HIP runtime's AQL packet capture of graphs off
    // (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 in the environment before HIP starts):
    // with it on (ROCm 7.2's default) a replay of the rig-latency graphs after
    // other contexts had come and gone faulted the GPU (illegal address) in the
    // round-6 GPU tests, and the same replay with it off ran clean (DESIGN.md
    // §4). Without that setting every kernel is launched directly.
    const char* pc = std::getenv("DEBUG_CLR_GRAPH_PACKET_CAPTURE");
    c->use_graphs = pc && pc[0] == '0';
    if (const char* e = std::getenv("MANTIS_GRAPHS")) c->use_graphs = c->use_graphs && e[0] != '0';
  }
  // tests: start the run CCL's mark epoch near its wrap (4..255; the flag plane is cleared at the wrap)
  if (const char* e = std::getenv("MANTIS_HYST_EPOCH0")) c->hyst_epoch = std::max(3, std::min(255, std::atoi(e)));
  c->F = cfg.max_cams;
  c->Wmax = cfg.max_width;
  c->Hmax = cfg.max_height;
  c->plane = (size_t)(c->Wmax + 2) * (c->Hmax + 2);
  c->bstride = bits::tiled_words(c->Wmax, c->Hmax);  // >= row-major words; the mask plane is tiled
  c->dstride = (size_t)dbits_wpw(c->Wmax + 2) * (c->Hmax + 2);
  c->pool_cap = cfg.max_contour_points;
  {
    // dynamic LDS budget of k_trace_borders_lds: 160 KB minus its static LUT
    c->trace_lds_max = 160 * 1024 - 512 * 8 - 64;
    c->trace_lds_ok = hipFuncSetAttribute((const void*)k_trace_borders_lds, hipFuncAttributeMaxDynamicSharedMemorySize,
                                          (int)c->trace_lds_max) == hipSuccess;
    const char* so = getenv("MANTIS_SCREEN");
    c->screen_off = so && so[0] == '0';
    const char* e = getenv("MANTIS_TRACE_LDS_FRAMES");
    c->trace_lds_frames = e ? atoi(e) : c->n_cu / 4;
    const char* e2 = getenv("MANTIS_FC_SMALL_FRAMES");
    c->fc_small_frames = e2 ? atoi(e2) : c->n_cu / 4;
    const char* e3 = getenv("MANTIS_PF_SPLIT");
    c->pf_split = !(e3 && e3[0] == '0');
  }
  {
    // LDS-staged mask for the particle filter: the tiled plane of a max-size
    // frame beside the kernel's static LDS
    const size_t ml = bits::tiled_words(c->Wmax, c->Hmax) * 4;
    hipFuncAttributes a1;
    c->pf_mask_lds = 0;
    if (!getenv("MANTIS_PF_MASK_GLOBAL") &&
        hipFuncGetAttributes(&a1, (const void*)k_score_pf<kPfThreads, kPfSplit, true>) == hipSuccess &&
        a1.sharedSizeBytes + ml <= 160 * 1024 &&
        hipFuncSetAttribute((const void*)k_score_pf<kPfThreads, kPfSplit, true>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)ml) == hipSuccess)
      c->pf_mask_lds = ml;
  }
  {
    // k_hyst_rec: the frame's candidate plane in LDS beside its static seam rows
    hipFuncAttributes a;
    if (hipFuncGetAttributes(&a, (const void*)k_hyst_rec) == hipSuccess) {
      const size_t budget = 160 * 1024 - a.sharedSizeBytes;
      if (hipFuncSetAttribute((const void*)k_hyst_rec, hipFuncAttributeMaxDynamicSharedMemorySize, (int)budget) ==
          hipSuccess)
        c->hyst_rec_lds = budget;
    }
  }
  // hysteresis bands: edge, strong and candidate words of HB_ROWS rows in LDS
  if (hipFuncSetAttribute((const void*)k_hyst_band, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)(3 * sizeof(uint32_t) * HB_ROWS * bits::words(c->Wmax))) != hipSuccess) {
    g_create_err = "max_width too large for the hysteresis band kernel";
    (void)hipStreamDestroy(c->s);
    delete c;
    return MANTIS_ERR_ARG;
  }
  c->morph_bh = morph_lds(c->Wmax, MB_BH) <= 160 * 1024 ? MB_BH : MB_BH_NARROW;
  if (const char* e = getenv("MANTIS_MORPH_WALK")) {  // an explicit choice applies to every batch size
    c->morph_walk = std::max(0, atoi(e));
    c->morph_walk_small = std::max(1, c->morph_walk);
  }
  if (const char* e = getenv("MANTIS_MORPH_WALK_SMALL")) c->morph_walk_small = std::max(1, atoi(e));
  if (morph_lds(c->Wmax, c->morph_bh) > 160 * 1024 ||
      hipFuncSetAttribute((const void*)k_morph, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)morph_lds(c->Wmax, c->morph_bh)) !=
          hipSuccess) {
    g_create_err = "max_width too large for the morphology band kernel";
    (void)hipStreamDestroy(c->s);
    delete c;
    return MANTIS_ERR_ARG;
  }
  const int F = c->F;
  const int per = cfg.particles * cfg.iterations * 6;
  mantis_status st = MANTIS_OK;
  auto chk = [&](mantis_status s) { if (st == MANTIS_OK) st = s; };
  c->fstride = (c->plane + 3) & ~(size_t)3;  // the hysteresis flags take dword atomics at (root & ~3)
  chk(dalloc(c, &c->d_strong, (size_t)F * c->fstride));
  c->lstride = (c->plane + 1) & ~(size_t)1;  // even: the hysteresis views it as u32 run extents
  chk(dalloc(c, &c->d_lroot, (size_t)F * c->lstride));
  chk(dalloc(c, &c->d_edge, c->plane));  // debug / single-frame byte planes (frame 0)
  chk(dalloc(c, &c->d_det, c->plane));
  chk(dalloc(c, &c->d_eb, (size_t)F * c->bstride));
  chk(dalloc(c, &c->d_b1, (size_t)F * c->bstride));
  chk(dalloc(c, &c->d_b2, (size_t)F * c->bstride));
  chk(dalloc(c, &c->d_dbits, (size_t)F * c->dstride));
  c->tstride = tbits_words(c->Wmax + 2, c->Hmax + 2);
  chk(dalloc(c, &c->d_tbits, (size_t)F * c->tstride));
  c->rstride = (size_t)c->Hmax + 3 + (c->Hmax + HB_ROWS - 1) / HB_ROWS;  // + the hysteresis band run counts
  chk(dalloc(c, &c->d_rowb, (size_t)F * c->rstride));
  chk(dalloc(c, &c->d_mask, c->plane));
  chk(dalloc(c, &c->d_mbits, (size_t)F * c->bstride));
  chk(dalloc(c, &c->d_lab, (size_t)F * c->plane));
  chk(dalloc(c, &c->d_frames, (size_t)F));
  chk(dalloc(c, &c->d_borders, (size_t)F * kMaxBorders));
  chk(dalloc(c, &c->d_bcount, (size_t)F * kMaxBorders));
  chk(dalloc(c, &c->d_boff, (size_t)F * kMaxBorders));
  chk(dalloc(c, &c->d_pool, (size_t)F * 2 * c->pool_cap));
  chk(dalloc(c, &c->d_scratch, (size_t)F * 4 * c->pool_cap));
  chk(dalloc(c, &c->d_quads, (size_t)F * kMaxQuads));
  chk(dalloc(c, &c->d_rpp, (size_t)F * kMaxQuads * 2));
  chk(dalloc(c, &c->d_items, (size_t)F * kMaxQuads * 2));
  chk(dalloc(c, &c->d_refine, (size_t)F * kMaxQuads * 2 * rpp::kCand));
  chk(dalloc(c, &c->d_jobs0, (size_t)F * kMaxQuads * 2));
  chk(dalloc(c, &c->d_jobs1, (size_t)F * kMaxQuads * 2 * rpp::kCand));
  chk(dalloc(c, &c->d_rq, 1));
  {
    // spill pools sized for the largest ObjPose grid objpose_blocks can return
    const size_t blocks = c->rpp_blocks > 0 ? (size_t)c->rpp_blocks : (size_t)std::max(64, 3 * c->n_cu / 2);
    c->op_cap = (int32_t)(blocks * 256);
    for (int k = 0; k < 2; k++) {
      chk(dalloc(c, &c->d_opool[k], (size_t)kOpFields * c->op_cap));
      chk(dalloc(c, &c->d_ojob[k], (size_t)c->op_cap));
    }
    chk(dalloc(c, &c->d_octl, 2 * 2 * kOpMaxRounds));
  }
  chk(dalloc(c, &c->d_gen, (size_t)F * kMaxHyps));
  chk(dalloc(c, &c->d_hyps, (size_t)F * kMaxHyps));
  chk(dalloc(c, &c->d_st, (size_t)F));
  chk(dalloc(c, &c->d_sst, (size_t)F));
  chk(dalloc(c, &c->d_dbg, (size_t)F));
  chk(dalloc(c, &c->d_res, (size_t)F));
  chk(dalloc(c, &c->d_gauss, (size_t)F * per));
  c->gauss_cap = F;
  chk(dalloc(c, &c->d_gtotal, 1));
  chk(halloc(c, &c->h_gauss, (size_t)F * per));
  chk(halloc(c, &c->h_states, (size_t)F + 1));
  chk(halloc(c, &c->h_res, (size_t)F));
  chk(halloc(c, &c->h_st, (size_t)F));
  chk(halloc(c, &c->h_gtotal, 1));
  chk(halloc(c, &c->h_frames, (size_t)F));
  if (st != MANTIS_OK) {
    g_create_err = c->err;
    mantis_destroy(c);
    return st;
  }
  (void)hipGetLastError();
  // the run CCL's mark plane starts clean: a first epoch set near the wrap
  // (MANTIS_HYST_EPOCH0) skips the clear at epoch 4, and k_hyst_fix reads the
  // flags of roots k_hyst_mark never wrote
  if (hipMemset(c->d_dbg, 0, sizeof(FrameDebug) * F) != hipSuccess ||
      hipMemset(c->d_strong, 0, c->fstride * (size_t)F) != hipSuccess) {
    g_create_err = "hipMemset failed";
    mantis_destroy(c);
    return MANTIS_ERR_DEVICE;
  }
  g_live_ctx[cfg.device & 63].fetch_add(1);
  c->counted = true;
  *out_ctx = c;
  return MANTIS_OK;
}

mantis_status mantis_destroy(void* ctx) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c) return MANTIS_ERR_ARG;
  if (c->counted) g_live_ctx[c->cfg.device & 63].fetch_sub(1);
  if (c->s) (void)hipStreamSynchronize(c->s);
  if (c->comm) (void)ncclCommDestroy((ncclComm_t)c->comm);
  for (auto& g : c->graphs) {
    if (g.pre) (void)hipGraphExecDestroy(g.pre);
    if (g.post) (void)hipGraphExecDestroy(g.post);
  }
  if (c->d_rwjobs) (void)hipFree(c->d_rwjobs);
  if (c->d_markov) (void)hipFree(c->d_markov);
  if (c->d_mops) (void)hipFree(c->d_mops);
  if (c->d_rwout) (void)hipFree(c->d_rwout);
  void* dptrs[] = {c->d_opool[0], c->d_opool[1], c->d_ojob[0], c->d_ojob[1], c->d_octl, c->d_dense_jobs, c->d_agree, c->d_gn28, c->d_bgr, c->d_lroot, c->d_strong, c->d_edge, c->d_det, c->d_mask, c->d_lab, c->d_eb, c->d_b1, c->d_b2, c->d_mbits, c->d_dbits, c->d_tbits, c->d_rowb,
                   c->d_frames, c->d_borders, c->d_bcount, c->d_boff, c->d_pool, c->d_scratch, c->d_quads, c->d_rpp, c->d_items, c->d_refine, c->d_jobs0, c->d_jobs1, c->d_rq,
                   c->d_dense_c2w, c->d_dense_err, c->d_dense_np, c->d_pairs, c->d_gncam, c->d_rigio, c->d_gnobs, c->d_gnacc, c->d_sh_gidx, c->d_sh_pf, c->d_sh_flags, c->d_sh_rec, c->d_gen, c->d_hyps, c->d_st, c->d_sst, c->d_dbg, c->d_res, c->d_gauss, c->d_gtotal, c->d_lm};
  for (void* p : dptrs)
    if (p) (void)hipFree(p);
  for (void* p : c->user_allocs) (void)hipFree(p);
  void* hptrs[] = {c->h_gauss, c->h_states, c->h_res, c->h_st, c->h_gtotal, c->h_frames, c->h_sh_flags, c->h_sh_rec};
  for (void* p : hptrs)
    if (p) (void)hipHostFree(p);
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  if (c->ev_gauss) (void)hipEventDestroy(c->ev_gauss);
  if (c->ev_wait) (void)hipEventDestroy(c->ev_wait);
  if (c->s_copy) (void)hipStreamDestroy(c->s_copy);
  if (c->s) (void)hipStreamDestroy(c->s);
  delete c;
  return MANTIS_OK;
}

const char* mantis_last_error(void* ctx) {
  if (!ctx) return g_create_err.c_str();
  return ((Ctx*)ctx)->err.c_str();
}

mantis_status mantis_set_map(void* ctx, const double* white, int32_t nw, const double* red, int32_t nr,
                             const double* green, int32_t ng) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || nw < 0 || nr < 0 || ng < 0 || nw + nr + ng > 768 || ng > 64 || (nw && !white) || (nr && !red) ||
      (ng && !green)) {
    if (c) c->err = "map: need nw+nr+ng <= 768 and ng <= 64";
    return MANTIS_ERR_ARG;
  }
  std::vector<double> all;
  all.insert(all.end(), white, white + 3 * nw);
  all.insert(all.end(), red, red + 3 * nr);
  all.insert(all.end(), green, green + 3 * ng);
  // then the screen's FP32 table (X, Y, Z, |X|_1 rounded up; mk_screen.h) at
  // double index kLmfOffset: 768 float4 = 1536 doubles
  const size_t nl = (size_t)nw + nr + ng;
  std::vector<double> buf(kLmfOffset + 2 * 768, 0.0);
  std::copy(all.begin(), all.end(), buf.begin());
  float* lf = (float*)(buf.data() + kLmfOffset);
  for (size_t i = 0; i < nl; i++) screen_landmark(all.data() + 3 * i, lf + 4 * i);
  if (c->d_lm) (void)hipFree(c->d_lm);
  c->d_lm = nullptr;
  if (dalloc(c, &c->d_lm, buf.size()) != MANTIS_OK) return MANTIS_ERR_OOM;
  HIP_OK(hipMemcpy(c->d_lm, buf.data(), sizeof(double) * buf.size(), hipMemcpyHostToDevice));
  c->nw = nw;
  c->nr = nr;
  c->ng = ng;
  return MANTIS_OK;
}

int32_t mantis_parse_coordinates(const char* s, double* xyz, int32_t max_pts) {
  if (!s) return 0;
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
    if (xyz && n < max_pts) { xyz[3 * n] = v[0]; xyz[3 * n + 1] = v[1]; xyz[3 * n + 2] = v[2]; }
    n++;
  }
  return n;
}

mantis_status mantis_rng_get(void* ctx, uint64_t* state) {
  if (!ctx || !state) return MANTIS_ERR_ARG;
  *state = ((Ctx*)ctx)->rng_state;
  return MANTIS_OK;
}
mantis_status mantis_rng_set(void* ctx, uint64_t state) {
  if (!ctx) return MANTIS_ERR_ARG;
  ((Ctx*)ctx)->rng_state = state ? state : 0xffffffffULL;
  return MANTIS_OK;
}

namespace {
mantis_status run_rig_gn(Ctx* c, const double* Tbc, int n_rigs, int cams_local, mantis_result* out,
                         bool use_comm);  // gn_impl.hip
}

namespace {
// cfg.rig_weighting = 1: the legacy particle weight (MonteCarlo::computeWeight /
// computeCameraError, include/legacy/mantis/MonteCarlo.cpp:183-241) over every
// camera of the rig, for each published camera's base pose (include/mantis.h,
// mantis_get_rig_weights). all / Tall: every camera's result and T_base_cam in
// global order (rig-major); gidx: the global index of each local frame of the
// last pipeline batch. With use_comm the (sum, count) slots of the local
// cameras are summed over the ranks (exact integers in doubles).
// Candidate slots per rig: K = C + 1, the last one the mantisService motion
// prediction pred_Twb[16 r] (nullable; mantis_process).
mantis_status weight_rigs(Ctx* c, int n_rigs, int C, const mantis_cam_result* all, const double* Tall,
                          const int32_t* gidx, int n_local, bool use_comm, mantis_result* out,
                          const double* pred_Twb = nullptr) {
  const int K = C + 1;
  const size_t nslot = (size_t)n_rigs * K * C;
  std::vector<double> Twb((size_t)n_rigs * K * 16);
  std::vector<char> cand((size_t)n_rigs * K, 0);
  for (int r = 0; r < n_rigs; r++) {
    for (int k = 0; k < C; k++) {
      const mantis_cam_result& cr = all[(size_t)r * C + k];
      if (!cr.publish) continue;
      double Twc[16], Tinv[16];
      quat_to_mat4(cr.orientation_xyzw, cr.position, Twc);
      mat4_inv_rigid(Tall + 16 * ((size_t)r * C + k), Tinv);
      mat4_mul(Twc, Tinv, &Twb[16 * ((size_t)r * K + k)]);
      cand[(size_t)r * K + k] = 1;
    }
    if (pred_Twb) {
      std::memcpy(&Twb[16 * ((size_t)r * K + C)], pred_Twb + 16 * (size_t)r, sizeof(double) * 16);
      cand[(size_t)r * K + C] = 1;
    }
  }
  c->rw_c2w.assign(nslot * 12, 0.0);  // this rank's cameras only
  std::vector<RigWJob> jobs;
  std::vector<size_t> slot_of;
  for (int i = 0; i < n_local; i++) {
    const int g = gidx ? gidx[i] : i;
    const int r = g / C, cam = g % C;
    for (int k = 0; k < K; k++) {
      if (!cand[(size_t)r * K + k]) continue;
      double Twc[16], Tcw[16];
      mat4_mul(&Twb[16 * ((size_t)r * K + k)], Tall + 16 * (size_t)g, Twc);
      mat4_inv_rigid(Twc, Tcw);
      RigWJob J;
      std::memset(&J, 0, sizeof(J));
      for (int a = 0; a < 3; a++) {
        for (int b = 0; b < 3; b++) J.c2w[3 * a + b] = Tcw[4 * a + b];
        J.c2w[9 + a] = Tcw[4 * a + 3];
      }
      J.frame = i;
      const size_t slot = ((size_t)r * K + k) * C + cam;
      std::memcpy(&c->rw_c2w[12 * slot], J.c2w, sizeof(J.c2w));
      jobs.push_back(J);
      slot_of.push_back(slot);
    }
  }
  const size_t nj = jobs.size();
  const size_t need = std::max(nj, nslot);
  if (need > c->rw_cap) {
    HIP_OK(hipStreamSynchronize(c->s));
    (void)hipFree(c->d_rwjobs);
    (void)hipFree(c->d_rwout);
    c->d_rwjobs = nullptr;
    c->d_rwout = nullptr;
    c->rw_cap = 0;
    mantis_status st = MANTIS_OK;
    if (dalloc(c, &c->d_rwjobs, need) || dalloc(c, &c->d_rwout, 2 * need)) st = MANTIS_ERR_OOM;
    if (use_comm) st = agree(c, st);  // before the (sum, count) all-reduce
    if (st != MANTIS_OK) return st;
    c->rw_cap = need;
  } else if (use_comm) {
    if (mantis_status st = agree(c, MANTIS_OK)) return st;
  }
  std::vector<double> sums(2 * nslot, 0.0);
  if (nj) {
    HIP_OK(hipMemcpyAsync(c->d_rwjobs, jobs.data(), sizeof(RigWJob) * nj, hipMemcpyHostToDevice, c->s));
    const RigWColors col{{255, 255, 255, 50, 85, 255, 50, 255, 85}};  // WHITE / RED / GREEN, Mantis3Params.h:40-42
    Landmarks L = lmk_of(c);
    k_rig_weight<<<(unsigned)((nj + 3) / 4), 256, 0, c->s>>>(c->d_frames, L, c->d_rwjobs, (int)nj, col, c->d_rwout);
    HIP_OK(hipGetLastError());
    std::vector<double> o(2 * nj);
    HIP_OK(hipMemcpyAsync(o.data(), c->d_rwout, sizeof(double) * 2 * nj, hipMemcpyDeviceToHost, c->s));
    HIP_OK(hipStreamSynchronize(c->s));
    for (size_t j = 0; j < nj; j++) {
      sums[2 * slot_of[j]] = o[2 * j];
      sums[2 * slot_of[j] + 1] = o[2 * j + 1];
    }
  }
  if (use_comm) {
    HIP_OK(hipMemcpyAsync(c->d_rwout, sums.data(), sizeof(double) * 2 * nslot, hipMemcpyHostToDevice, c->s));
    ncclResult_t rr = ncclAllReduce(c->d_rwout, c->d_rwout, 2 * nslot, ncclFloat64, ncclSum, (ncclComm_t)c->comm, c->s);
    if (rr != ncclSuccess) { c->err = std::string("ncclAllReduce (rig weights): ") + ncclGetErrorString(rr); return MANTIS_ERR_COMM; }
    HIP_OK(hipMemcpyAsync(sums.data(), c->d_rwout, sizeof(double) * 2 * nslot, hipMemcpyDeviceToHost, c->s));
    HIP_OK(hipStreamSynchronize(c->s));
  }
  c->rw_rigs = n_rigs;
  c->rw_C = C;
  c->rw_sums = sums;
  c->rw_weights.assign((size_t)n_rigs * K, DBL_MAX);
  c->rw_chosen.assign(n_rigs, -1);
  for (int r = 0; r < n_rigs; r++) {
    int best = -1;
    for (int k = 0; k < K; k++) {
      if (!cand[(size_t)r * K + k]) continue;
      double w = 0.0;
      for (int cam = 0; cam < C; cam++) {
        const size_t slot = ((size_t)r * K + k) * C + cam;
        const double e = sums[2 * slot], n = sums[2 * slot + 1];
        w += (n < 10 ? 1e17 : e) / n;  // computeCameraError :220-225 (n = 0 gives inf)
      }
      w /= (double)C;
      c->rw_weights[(size_t)r * K + k] = w;
      if (best < 0 || w < c->rw_weights[(size_t)r * K + best]) best = k;
    }
    c->rw_chosen[r] = best;
    if (best < 0 || !out) continue;  // nothing published, no prediction: keep the reference fusion's answer
    const double* T = &Twb[16 * ((size_t)r * K + best)];
    double R[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) R[i * 3 + j] = T[i * 4 + j];
    mk::Quat q = basis_to_quat(R);
    out[r].orientation_xyzw[0] = q.x; out[r].orientation_xyzw[1] = q.y;
    out[r].orientation_xyzw[2] = q.z; out[r].orientation_xyzw[3] = q.w;
    for (int i = 0; i < 3; i++) out[r].position[i] = T[i * 4 + 3];
    out[r].weight = c->rw_weights[(size_t)r * K + best];
    if (best < C) {
      const mantis_cam_result& cr = all[(size_t)r * C + best];
      for (int i = 0; i < 36; i++) out[r].covariance[i] = cr.covariance[i];
      out[r].min_yaw_diff = cr.min_yaw_diff;
      out[r].publish = 1;
    } else {  // the motion prediction: published only if a camera measured a pose this call
      out[r].publish = out[r].n_cams_published > 0 ? 1 : 0;
    }
  }
  return MANTIS_OK;
}
}  // namespace

namespace {
mantis_status process_batch_impl(Ctx* c, const mantis_image* cams, int32_t n_rigs, int32_t cams_per_rig,
                                 mantis_result* out, mantis_cam_result* cam_out, const double* pred_Twb);
}

mantis_status mantis_process_batch(void* ctx, const mantis_image* cams, int32_t n_rigs, int32_t cams_per_rig,
                                   mantis_result* out, mantis_cam_result* cam_out) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  return process_batch_impl(c, cams, n_rigs, cams_per_rig, out, cam_out, nullptr);
}

namespace {
mantis_status process_batch_impl(Ctx* c, const mantis_image* cams, int32_t n_rigs, int32_t cams_per_rig,
                                 mantis_result* out, mantis_cam_result* cam_out, const double* pred_Twb) {
  if (!c || !cams || n_rigs <= 0 || cams_per_rig <= 0) return MANTIS_ERR_ARG;
  const int n = n_rigs * cams_per_rig;
  mantis_status st = process_frames(c, cams, n);
  if (st != MANTIS_OK) return st;
  const std::vector<double> Tbc = gather_tbc(cams, n);
  if (out) {
    std::vector<int32_t> pf(n);
    for (int f = 0; f < n; f++) pf[f] = c->h_st[f].reaches_pf;
    mk::shard::rig_results(n_rigs, cams_per_rig, c->h_res, Tbc.data(), pf.data(), c->h_states, out);
  }
  if (out && (c->cfg.rig_weighting || pred_Twb)) {
    st = weight_rigs(c, n_rigs, cams_per_rig, c->h_res, Tbc.data(), nullptr, n, false, out, pred_Twb);
    if (st != MANTIS_OK) return st;
  }
  if (out && c->cfg.gn_enable) {
    st = run_rig_gn(c, Tbc.data(), n_rigs, cams_per_rig, out, false);
    if (st != MANTIS_OK) return st;
  }
  if (cam_out) std::memcpy(cam_out, c->h_res, sizeof(mantis_cam_result) * n);
  for (int f = 0; f < n; f++)
    if (c->h_res[f].status != 0) return MANTIS_ERR_CAPACITY;
  return MANTIS_OK;
}
}  // namespace

namespace {
using ShardRec = mk::shard::Rec;  // one camera's result as exchanged between the ranks
}  // namespace

mantis_status mantis_process_rig_sharded(void* ctx, const mantis_image* local_cams, int32_t n_rigs, int32_t n_local,
                                         const int32_t* cam_index, int32_t cams_per_rig, mantis_result* out,
                                         mantis_cam_result* cam_out) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !local_cams || !cam_index || !out || n_rigs <= 0 || n_local <= 0 || cams_per_rig <= 0)
    return MANTIS_ERR_ARG;
  if (!c->comm) { c->err = "comm not initialised (mantis_comm_init)"; return MANTIS_ERR_STATE; }
  // from here every failure is agreed on with the other ranks before an exchange (agree())
  mantis_status vst = MANTIS_OK;
  const int nl_max = (cams_per_rig + c->nranks - 1) / c->nranks;
  if (n_local * c->nranks < cams_per_rig && c->nranks == 1) {
    c->err = "sharded rig: a one-rank communicator must hold every camera";
    vst = MANTIS_ERR_ARG;
  }
  if (vst == MANTIS_OK && n_local > nl_max) {
    c->err = "sharded rig: at most ceil(cams_per_rig / nranks) cameras per rank";
    vst = MANTIS_ERR_ARG;
  }
  for (int j = 0; j < n_local && vst == MANTIS_OK; j++)
    if (cam_index[j] < 0 || cam_index[j] >= cams_per_rig || (j > 0 && cam_index[j] <= cam_index[j - 1])) {
      c->err = "sharded rig: cam_index must be ascending indices in [0, cams_per_rig)";
      vst = MANTIS_ERR_ARG;
    }
  const int n = n_rigs * n_local, ng = n_rigs * cams_per_rig, slots = n_rigs * nl_max;
  // exchange buffers: (index, flag) pairs and result records, send + nranks x recv
  if (vst == MANTIS_OK &&
      ((size_t)ng > c->sh_cap || (size_t)slots * (c->nranks + 1) * sizeof(ShardRec) > c->sh_rec_bytes)) {
    HIP_OK(hipStreamSynchronize(c->s));
    void* d[] = {c->d_sh_gidx, c->d_sh_pf, c->d_sh_flags, c->d_sh_rec};
    for (void* p : d) (void)hipFree(p);
    void* h[] = {c->h_sh_flags, c->h_sh_rec};
    for (void* p : h) (void)hipHostFree(p);
    c->d_sh_gidx = c->d_sh_pf = c->d_sh_flags = c->h_sh_flags = nullptr;
    c->d_sh_rec = c->h_sh_rec = nullptr;
    c->sh_cap = c->sh_rec_bytes = 0;
    const size_t rec_bytes = (size_t)slots * (c->nranks + 1) * sizeof(ShardRec);
    if (dalloc(c, &c->d_sh_gidx, (size_t)ng) || dalloc(c, &c->d_sh_pf, (size_t)2 * ng * (c->nranks + 1)) ||
        dalloc(c, &c->d_sh_flags, (size_t)2 * ng) || halloc(c, &c->h_sh_flags, (size_t)2 * ng) ||
        dalloc(c, &c->d_sh_rec, rec_bytes) || halloc(c, &c->h_sh_rec, rec_bytes)) {
      vst = MANTIS_ERR_OOM;
    } else {
      c->sh_cap = ng;
      c->sh_rec_bytes = rec_bytes;
    }
  }
  if ((vst = agree(c, vst)) != MANTIS_OK) return vst;
  std::vector<int32_t> gidx(n);
  mk::shard::global_indices(n_rigs, n_local, cam_index, cams_per_rig, gidx.data());
  Shard sh{ng, slots, gidx.data()};
  mantis_status st = process_frames(c, local_cams, n, &sh);
  // a failure process_frames agreed on returns everywhere; a later one (after
  // the PF-flag exchange) is agreed on before the result all-gather
  if (st != MANTIS_OK && c->agreed_fail) return st;
  if ((st = agree(c, st)) != MANTIS_OK) return st;
  // gather every camera's result (one ncclAllGather of fixed-size records)
  ShardRec* send = (ShardRec*)c->h_sh_rec;
  for (int s = 0; s < slots; s++) {
    std::memset(&send[s], 0, sizeof(ShardRec));
    send[s].gidx = -1;
    if (s < n) {
      send[s].res = c->h_res[s];
      std::memcpy(send[s].Tbc, local_cams[s].T_base_cam, sizeof(double) * 16);
      send[s].gidx = gidx[s];
    }
  }
  const size_t sbytes = (size_t)slots * sizeof(ShardRec);
  HIP_OK(hipMemcpyAsync(c->d_sh_rec, send, sbytes, hipMemcpyHostToDevice, c->s));
  ncclResult_t r = ncclAllGather(c->d_sh_rec, c->d_sh_rec + sbytes, sbytes, ncclUint8, (ncclComm_t)c->comm, c->s);
  if (r != ncclSuccess) { c->err = std::string("ncclAllGather (camera results): ") + ncclGetErrorString(r); return MANTIS_ERR_COMM; }
  HIP_OK(hipMemcpyAsync(c->h_sh_rec + sbytes, c->d_sh_rec + sbytes, sbytes * c->nranks, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  const ShardRec* recv = (const ShardRec*)(c->h_sh_rec + sbytes);
  std::vector<mantis_cam_result> all(ng);
  std::vector<double> Tall(16 * (size_t)ng);
  std::vector<int32_t> seen(ng);
  switch (mk::shard::merge_records(recv, slots * c->nranks, ng, all.data(), Tall.data(), seen.data())) {
    case 0: break;
    case 1: c->err = "sharded rig: a camera is owned by two ranks"; return MANTIS_ERR_ARG;
    case 2: c->err = "sharded rig: a camera is owned by no rank"; return MANTIS_ERR_ARG;
    default: c->err = "sharded rig: camera index out of range"; return MANTIS_ERR_ARG;
  }
  mk::shard::rig_results(n_rigs, cams_per_rig, all.data(), Tall.data(), c->h_sh_flags, c->h_states, out);
  if (c->cfg.rig_weighting) {
    st = weight_rigs(c, n_rigs, cams_per_rig, all.data(), Tall.data(), gidx.data(), n, true, out, nullptr);
    if (st != MANTIS_OK) return st;
  }
  if (c->cfg.gn_enable) {
    const std::vector<double> Tbc = gather_tbc(local_cams, n);
    st = run_rig_gn(c, Tbc.data(), n_rigs, n_local, out, true);
    if (st != MANTIS_OK) return st;
  }
  if (cam_out) std::memcpy(cam_out, all.data(), sizeof(mantis_cam_result) * ng);
  for (int g = 0; g < ng; g++)
    if (all[g].status != 0) return MANTIS_ERR_CAPACITY;
  return MANTIS_OK;
}

mantis_status mantis_shard_gauss_offsets(void* ctx, const int32_t* pairs, int32_t npairs, int32_t n_global,
                                         const int32_t* gidx, int32_t n_local, int32_t per_frame, int32_t* offsets,
                                         int32_t* total) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !pairs || npairs < 0 || n_global < 0 || !gidx || n_local < 0 || n_local > c->F || per_frame < 0 ||
      !offsets || !total)
    return MANTIS_ERR_ARG;
  if ((int64_t)per_frame * n_global > INT32_MAX) { c->err = "per_frame x n_global exceeds 2^31"; return MANTIS_ERR_ARG; }
  for (int i = 0; i < n_local; i++)
    if (gidx[i] < 0 || gidx[i] >= n_global) { c->err = "gidx outside [0, n_global)"; return MANTIS_ERR_ARG; }
  // the host rule (mk_shard.h offsets_from_pairs) rejects a gather naming a
  // frame >= n_global; so does the kernel (total -1), checked below as well
  for (int i = 0; i < npairs; i++)
    if (pairs[2 * i] >= n_global) { c->err = "pair index outside [0, n_global)"; return MANTIS_ERR_ARG; }
  int32_t *d_pairs = nullptr, *d_flags = nullptr, *d_gidx = nullptr, *d_total = nullptr;
  FrameState* d_st = nullptr;  // scratch frame states: the context's (last batch) are left alone
  DevScratch ds(c);
  if (ds.get(&d_pairs, (size_t)2 * npairs) || ds.get(&d_flags, (size_t)2 * n_global) ||
      ds.get(&d_gidx, (size_t)n_local) || ds.get(&d_total, 1) || ds.get(&d_st, (size_t)std::max(1, n_local)))
    return MANTIS_ERR_OOM;
  if (npairs) HIP_OK(hipMemcpyAsync(d_pairs, pairs, sizeof(int32_t) * 2 * npairs, hipMemcpyHostToDevice, c->s));
  if (n_local) HIP_OK(hipMemcpyAsync(d_gidx, gidx, sizeof(int32_t) * n_local, hipMemcpyHostToDevice, c->s));
  k_gauss_offsets_global<<<1, 1024, 0, c->s>>>(d_pairs, npairs, d_flags, n_global, d_st, d_gidx, n_local, per_frame,
                                               d_total);
  HIP_OK(hipGetLastError());
  std::vector<FrameState> st(std::max(1, n_local));
  if (n_local) HIP_OK(hipMemcpyAsync(st.data(), d_st, sizeof(FrameState) * n_local, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipMemcpyAsync(total, d_total, sizeof(int32_t), hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  if (*total < 0) { c->err = "pair index outside [0, n_global)"; return MANTIS_ERR_ARG; }
  for (int i = 0; i < n_local; i++) offsets[i] = st[i].gauss_offset;
  return MANTIS_OK;
}

mantis_status mantis_get_rig_weights_info(void* ctx, int32_t* n_rigs, int32_t* cams_per_rig) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !n_rigs || !cams_per_rig) return MANTIS_ERR_ARG;
  *n_rigs = c->rw_rigs;
  *cams_per_rig = c->rw_C;
  return MANTIS_OK;
}

mantis_status mantis_get_rig_weights(void* ctx, int32_t rig, double* weights, double* c2w, double* sums,
                                     int32_t* chosen) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !weights || rig < 0) return MANTIS_ERR_ARG;
  if (rig >= c->rw_rigs) { c->err = "no rig weighting record for that rig (cfg.rig_weighting, last batch)"; return MANTIS_ERR_STATE; }
  const int C = c->rw_C, K = C + 1;
  std::memcpy(weights, &c->rw_weights[(size_t)rig * K], sizeof(double) * K);
  if (c2w) std::memcpy(c2w, &c->rw_c2w[(size_t)rig * K * C * 12], sizeof(double) * K * C * 12);
  if (sums) std::memcpy(sums, &c->rw_sums[(size_t)rig * K * C * 2], sizeof(double) * K * C * 2);
  if (chosen) *chosen = c->rw_chosen[rig];
  return MANTIS_OK;
}

// mantisService motion (srv/mantisService.srv:4-8: "applied to each particle
// before reevaluating"; parsed into tf::Transform(delta_quat, delta_pos) by the
// legacy server, include/legacy/mantis/MonteCarlo.cpp:273-276, and composed on
// the right of a particle as runFilter does, :58). The mantis3 callback has no
// particles across frames, so the context keeps the last published
// rig pose as the one particle the service carries: with a motion and that
// prior, the prediction T_prior * Delta joins the rig candidates and all are
// re-evaluated with the legacy weighting (weight_rigs). A motion whose
// quaternion has |q|^2 < 0.5 (an unset message: all zeros) counts as none.
mantis_status mantis_process(void* ctx, const mantis_image* cams, int32_t n_cams, const mantis_motion* motion,
                             mantis_result* out, mantis_cam_result* cam_out) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c) return MANTIS_ERR_ARG;
  double pred[16];
  const double* pq = motion ? motion->delta_quat_xyzw : nullptr;
  const bool use_motion = motion && out && c->has_prior &&
                          pq[0] * pq[0] + pq[1] * pq[1] + pq[2] * pq[2] + pq[3] * pq[3] >= 0.5;
  if (use_motion) {
    double D[16];
    quat_to_mat4(motion->delta_quat_xyzw, motion->delta_pos, D);
    mat4_mul(c->prior_Twb, D, pred);
  }
  mantis_result tmp;
  mantis_result* o = out ? out : &tmp;
  const mantis_status st = process_batch_impl(c, cams, 1, n_cams, o, cam_out, use_motion ? pred : nullptr);
  if (st == MANTIS_OK && o->publish) {
    quat_to_mat4(o->orientation_xyzw, o->position, c->prior_Twb);
    c->has_prior = true;
  }
  return st;
}

mantis_status mantis_set_prior_pose(void* ctx, const double* T_w_b) {
  Ctx* c = (Ctx*)ctx;
  if (!c) return MANTIS_ERR_ARG;
  c->has_prior = T_w_b != nullptr;
  if (T_w_b) std::memcpy(c->prior_Twb, T_w_b, sizeof(c->prior_Twb));
  return MANTIS_OK;
}

mantis_status mantis_get_prior_pose(void* ctx, double* T_w_b, int32_t* has_prior) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !T_w_b || !has_prior) return MANTIS_ERR_ARG;
  *has_prior = c->has_prior ? 1 : 0;
  std::memcpy(T_w_b, c->prior_Twb, sizeof(c->prior_Twb));
  return MANTIS_OK;
}

mantis_status mantis_get_frame_debug(void* ctx, int32_t frame, void* out, size_t bytes) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !out || frame < 0 || frame >= c->F || bytes != sizeof(FrameDebug)) {
    if (c) c->err = "mantis_get_frame_debug: bad frame or size";
    return MANTIS_ERR_ARG;
  }
  HIP_OK(hipMemcpy(out, c->d_dbg + frame, sizeof(FrameDebug), hipMemcpyDeviceToHost));
  // the host-side RNG bookkeeping completes the record
  return MANTIS_OK;
}
size_t mantis_frame_debug_size(void) { return sizeof(FrameDebug); }

mantis_status mantis_get_contours(void* ctx, int32_t frame, int32_t* counts, int32_t* holes, int32_t max_borders,
                                  int32_t* points, int32_t max_points, int32_t* n_borders) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !counts || !holes || !points || !n_borders || frame < 0 || frame >= c->F || !c->h_st) return MANTIS_ERR_ARG;
  const int nb = std::min(c->h_st[frame].n_borders, kMaxBorders);
  *n_borders = nb;
  if (nb > max_borders) { c->err = "mantis_get_contours: max_borders too small"; return MANTIS_ERR_CAPACITY; }
  std::vector<int32_t> cnt(nb), off(nb);
  std::vector<Border> bs(nb);
  const size_t fb = (size_t)frame * kMaxBorders;
  if (nb > 0) {
    HIP_OK(hipMemcpy(cnt.data(), c->d_bcount + fb, sizeof(int32_t) * nb, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(off.data(), c->d_boff + fb, sizeof(int32_t) * nb, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(bs.data(), c->d_borders + fb, sizeof(Border) * nb, hipMemcpyDeviceToHost));
  }
  size_t total = 0;
  for (int b = 0; b < nb; b++) total += (size_t)cnt[b];
  if (total > (size_t)max_points) { c->err = "mantis_get_contours: max_points too small"; return MANTIS_ERR_CAPACITY; }
  std::vector<int32_t> pool((size_t)c->pool_cap);
  HIP_OK(hipMemcpy(pool.data(), c->d_pool + 2 * (size_t)frame * c->pool_cap, sizeof(int32_t) * pool.size(),
                   hipMemcpyDeviceToHost));
  // the device pool holds the points packed, x | y << 16 (k_frame_contours)
  const uint32_t* packed = (const uint32_t*)pool.data();
  size_t k = 0;
  for (int b = 0; b < nb; b++) {
    counts[b] = cnt[b];
    holes[b] = bs[b].hole;
    if ((size_t)off[b] + cnt[b] > (size_t)c->pool_cap) { c->err = "mantis_get_contours: pool overflow"; return MANTIS_ERR_CAPACITY; }
    for (int i = 0; i < cnt[b]; i++) {
      const uint32_t v = packed[(size_t)off[b] + i];
      points[2 * (k + i)] = (int32_t)(v & 0xffffu);
      points[2 * (k + i) + 1] = (int32_t)(v >> 16);
    }
    k += cnt[b];
  }
  return MANTIS_OK;
}

int32_t mantis_frame_counters(void* ctx, int32_t frame, int32_t* out, int32_t max) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !out || frame < 0 || frame >= c->F || !c->h_st) return -1;
  const int n = (int)(sizeof(FrameState) / sizeof(int32_t));
  const int k = max < n ? max : n;
  std::memcpy(out, &c->h_st[frame], sizeof(int32_t) * k);
  return k;
}

mantis_status mantis_canny(void* ctx, const mantis_image* img, uint8_t* canny_out) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !img || !canny_out) return MANTIS_ERR_ARG;
  int W, H;
  mantis_status st = stage_frames(c, img, 1, W, H);
  if (st != MANTIS_OK) return st;
  if ((st = run_image_stages(c, 1, W, H, true)) != MANTIS_OK) return st;
  HIP_OK(hipMemcpyAsync(canny_out, c->d_edge, (size_t)W * H, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  for (size_t i = 0; i < (size_t)W * H; i++) canny_out[i] = canny_out[i] ? 255 : 0;
  return MANTIS_OK;
}

mantis_status mantis_hysteresis(void* ctx, const uint8_t* cls, int32_t width, int32_t height, uint8_t* edges_out) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !cls || !edges_out) return MANTIS_ERR_ARG;
  const int W = width, H = height;
  if (W <= 2 || H <= 2 || W > c->Wmax || H > c->Hmax) { c->err = "image size outside [3, max]"; return MANTIS_ERR_ARG; }
  // class bytes are 0 / 1 / 2 only: k_cls_to_bits reads any non-zero byte as a
  // candidate, the oracle only 1 and 2, so other values are refused
  for (size_t i = 0; i < (size_t)W * H; i++)
    if (cls[i] > 2) { c->err = "class plane: bytes must be 0 (none), 1 (weak) or 2 (strong)"; return MANTIS_ERR_ARG; }
  HIP_OK(hipMemcpyAsync(c->d_edge, cls, (size_t)W * H, hipMemcpyHostToDevice, c->s));
  k_cls_to_bits<<<blocks_for((size_t)bits::words(W) * H), 256, 0, c->s>>>(c->d_edge, c->d_b1, c->d_b2, W, H);
  if (mantis_status st = run_hysteresis(c, 1, W, H, true); st != MANTIS_OK) return st;
  HIP_OK(hipMemcpyAsync(edges_out, c->d_edge, (size_t)W * H, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  for (size_t i = 0; i < (size_t)W * H; i++) edges_out[i] = edges_out[i] ? 255 : 0;
  return MANTIS_OK;
}

mantis_status mantis_masks(void* ctx, const mantis_image* img, uint8_t* det_out, uint8_t* mask_out) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !img) return MANTIS_ERR_ARG;
  int W, H;
  mantis_status st = stage_frames(c, img, 1, W, H);
  if (st != MANTIS_OK) return st;
  if ((st = run_image_stages(c, 1, W, H, false, det_out != nullptr)) != MANTIS_OK) return st;
  if (det_out) {
    HIP_OK(hipMemcpy2DAsync(det_out, W, c->d_det + (W + 2) + 1, W + 2, W, H, hipMemcpyDeviceToHost, c->s));
  }
  if (mask_out) {
    k_bits_to_bytes<<<blocks_for((size_t)W * H), 256, 0, c->s>>>(c->d_mbits, c->d_mask, W, H, -1);
    HIP_OK(hipMemcpyAsync(mask_out, c->d_mask, (size_t)W * H, hipMemcpyDeviceToHost, c->s));
  }
  HIP_OK(hipStreamSynchronize(c->s));
  for (size_t i = 0; det_out && i < (size_t)W * H; i++) det_out[i] = det_out[i] ? 255 : 0;
  for (size_t i = 0; mask_out && i < (size_t)W * H; i++) mask_out[i] = mask_out[i] ? 255 : 0;
  return MANTIS_OK;
}

mantis_status mantis_detect_quads(void* ctx, const mantis_image* img, int32_t* corners, int32_t max_quads,
                                  int32_t* n_quads) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !img || !n_quads) return MANTIS_ERR_ARG;
  int W, H;
  mantis_status st = stage_frames(c, img, 1, W, H);
  if (st != MANTIS_OK) return st;
  if ((st = run_image_stages(c, 1, W, H)) != MANTIS_OK) return st;
  if ((st = run_contours(c, 1, W, H)) != MANTIS_OK) return st;
  HIP_OK(hipMemcpyAsync(c->h_st, c->d_st, sizeof(FrameState), hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  if (c->h_st[0].overflow) { c->err = "detect_quads: workspace capacity exceeded"; return MANTIS_ERR_CAPACITY; }
  int nq = c->h_st[0].n_quads;
  *n_quads = nq;
  if (corners && max_quads > 0) {
    std::vector<QuadRec> q(nq);
    HIP_OK(hipMemcpy(q.data(), c->d_quads, sizeof(QuadRec) * nq, hipMemcpyDeviceToHost));
    for (int i = 0; i < nq && i < max_quads; i++)
      for (int k = 0; k < 8; k++) corners[8 * i + k] = q[i].c[k];
  }
  return MANTIS_OK;
}

mantis_status mantis_score_hypotheses(void* ctx, const mantis_image* img, const uint8_t* mask, const double* c2w,
                                      int32_t n, int32_t fast, double* err, int32_t* nproj) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !img || !c2w || n <= 0 || !err || !nproj) return MANTIS_ERR_ARG;
  if (!c->d_lm) { c->err = "map not set"; return MANTIS_ERR_STATE; }
  int W, H;
  mantis_status st = stage_frames(c, img, 1, W, H);
  if (st != MANTIS_OK) return st;
  double* d_c2w = nullptr;
  double* d_err = nullptr;
  int32_t* d_np = nullptr;
  if (dalloc(c, &d_c2w, (size_t)12 * n) != MANTIS_OK || dalloc(c, &d_err, (size_t)n) != MANTIS_OK ||
      dalloc(c, &d_np, (size_t)n) != MANTIS_OK)
    return MANTIS_ERR_OOM;
  const uint8_t* d_mask = nullptr;
  if (mask) {
    HIP_OK(hipMemcpyAsync(c->d_mask, mask, (size_t)W * H, hipMemcpyHostToDevice, c->s));
    d_mask = c->d_mask;
  }
  HIP_OK(hipMemcpyAsync(d_c2w, c2w, sizeof(double) * 12 * n, hipMemcpyHostToDevice, c->s));
  Landmarks L = lmk_of(c);
  mark(c, "start");
  k_score_api<<<(n + kApiHyps - 1) / kApiHyps, 64 * kApiHyps, 0, c->s>>>(c->d_frames, d_mask, L, d_c2w, n, fast, d_err, d_np);
  mark(c, "score_api");
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(err, d_err, sizeof(double) * n, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipMemcpyAsync(nproj, d_np, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  finish_profile(c);
  (void)hipFree(d_c2w);
  (void)hipFree(d_err);
  (void)hipFree(d_np);
  return MANTIS_OK;
}

mantis_status mantis_quad_gn(void* ctx, const double* img_pts, const double* obj_pts, int32_t n, double* R,
                             double* t, int32_t iterations, int32_t* steps, double* costs) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !img_pts || !obj_pts || n <= 0 || !R || !t || iterations < 0 || iterations > 100) return MANTIS_ERR_ARG;
  double *d_ip, *d_op, *d_R, *d_t, *d_c;
  int32_t* d_s;
  if (dalloc(c, &d_ip, (size_t)8 * n) || dalloc(c, &d_op, (size_t)12 * n) || dalloc(c, &d_R, (size_t)9 * n) ||
      dalloc(c, &d_t, (size_t)3 * n) || dalloc(c, &d_c, (size_t)2 * n) || dalloc(c, &d_s, (size_t)n))
    return MANTIS_ERR_OOM;
  HIP_OK(hipMemcpyAsync(d_ip, img_pts, sizeof(double) * 8 * n, hipMemcpyHostToDevice, c->s));
  HIP_OK(hipMemcpyAsync(d_op, obj_pts, sizeof(double) * 12 * n, hipMemcpyHostToDevice, c->s));
  HIP_OK(hipMemcpyAsync(d_R, R, sizeof(double) * 9 * n, hipMemcpyHostToDevice, c->s));
  HIP_OK(hipMemcpyAsync(d_t, t, sizeof(double) * 3 * n, hipMemcpyHostToDevice, c->s));
  k_quad_gn<<<(n + 255) / 256, 256, 0, c->s>>>(d_ip, d_op, n, d_R, d_t, iterations, d_s, d_c);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(R, d_R, sizeof(double) * 9 * n, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipMemcpyAsync(t, d_t, sizeof(double) * 3 * n, hipMemcpyDeviceToHost, c->s));
  if (steps) HIP_OK(hipMemcpyAsync(steps, d_s, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->s));
  if (costs) HIP_OK(hipMemcpyAsync(costs, d_c, sizeof(double) * 2 * n, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  void* ps[] = {d_ip, d_op, d_R, d_t, d_c, d_s};
  for (void* p : ps) (void)hipFree(p);
  return MANTIS_OK;
}

mantis_status mantis_rpp_batch(void* ctx, const double* img_pts, const double* obj_pts, int32_t n, double* R,
                               double* t, double* errs, int32_t* rpp_status) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !img_pts || !obj_pts || n <= 0 || !R || !t || !errs || !rpp_status) return MANTIS_ERR_ARG;
  double *d_ip, *d_op;
  RppItem* d_it;
  rpp::Refine* d_rf;
  RppOut* d_out;
  int32_t *d_j0, *d_j1;
  RppQueue* d_q;
  if (dalloc(c, &d_ip, (size_t)8 * n) || dalloc(c, &d_op, (size_t)12 * n) || dalloc(c, &d_it, (size_t)n) ||
      dalloc(c, &d_rf, (size_t)n * rpp::kCand) || dalloc(c, &d_out, (size_t)n) || dalloc(c, &d_j0, (size_t)n) ||
      dalloc(c, &d_j1, (size_t)n * rpp::kCand) || dalloc(c, &d_q, 1))
    return MANTIS_ERR_OOM;
  HIP_OK(hipMemcpyAsync(d_ip, img_pts, sizeof(double) * 8 * n, hipMemcpyHostToDevice, c->s));
  HIP_OK(hipMemcpyAsync(d_op, obj_pts, sizeof(double) * 12 * n, hipMemcpyHostToDevice, c->s));
  HIP_OK(hipMemsetAsync(d_q, 0, sizeof(RppQueue), c->s));
  mark(c, "start");
  k_rpp_prep_api<<<(n + 255) / 256, 256, 0, c->s>>>(d_ip, d_op, n, d_it, d_j0, d_q);
  mark(c, "rpp_prep");
  launch_rpp_queues(c, d_it, d_rf, d_j0, d_j1, d_q, d_out, nullptr, (size_t)n, (size_t)n, nullptr, false);
  HIP_OK(hipGetLastError());
  std::vector<RppOut> h(n);
  HIP_OK(hipMemcpyAsync(h.data(), d_out, sizeof(RppOut) * n, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  finish_profile(c);
  for (int i = 0; i < n; i++) {
    for (int k = 0; k < 9; k++) R[9 * i + k] = h[i].R[k];
    for (int k = 0; k < 3; k++) t[3 * i + k] = h[i].t[k];
    errs[2 * i] = h[i].obj_err;
    errs[2 * i + 1] = h[i].img_err;
    rpp_status[i] = h[i].error == 1 ? -1 : h[i].status;
  }
  void* ps[] = {d_ip, d_op, d_it, d_rf, d_out, d_j0, d_j1, d_q};
  for (void* p : ps) (void)hipFree(p);
  return MANTIS_OK;
}

mantis_status mantis_rpp_solve(void* ctx, const double* img_pts, const double* obj_pts, int32_t n_points,
                               int32_t n, double* R, double* t, double* errs, int32_t* rpp_status,
                               int32_t* iterations) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !img_pts || !obj_pts || n <= 0 || !R || !t || !errs || !rpp_status) return MANTIS_ERR_ARG;
  if (n_points < 4 || n_points > 12) {
    c->err = "mantis_rpp_solve: n_points must be in [4, 12]";
    return MANTIS_ERR_ARG;
  }
  double *d_ip, *d_op;
  RppOut* d_out;
  DevScratch ds(c);
  if (ds.get(&d_ip, (size_t)2 * n_points * n) || ds.get(&d_op, (size_t)3 * n_points * n) || ds.get(&d_out, (size_t)n))
    return MANTIS_ERR_OOM;
  HIP_OK(hipMemcpyAsync(d_ip, img_pts, sizeof(double) * 2 * n_points * n, hipMemcpyHostToDevice, c->s));
  HIP_OK(hipMemcpyAsync(d_op, obj_pts, sizeof(double) * 3 * n_points * n, hipMemcpyHostToDevice, c->s));
  const unsigned g = (unsigned)((n + 63) / 64);
  switch (n_points) {
#define MK_RPP_LAUNCH(k) \
    case k: k_rpp_solve<k><<<g, 64, 0, c->s>>>(d_ip, d_op, n, d_out); break;
    MK_RPP_LAUNCH(4)
    MK_RPP_INSTANCES(MK_RPP_LAUNCH)
#undef MK_RPP_LAUNCH
  }
  HIP_OK(hipGetLastError());
  std::vector<RppOut> h(n);
  HIP_OK(hipMemcpyAsync(h.data(), d_out, sizeof(RppOut) * n, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  for (int i = 0; i < n; i++) {
    for (int k = 0; k < 9; k++) R[9 * i + k] = h[i].R[k];
    for (int k = 0; k < 3; k++) t[3 * i + k] = h[i].t[k];
    errs[2 * i] = h[i].obj_err;
    errs[2 * i + 1] = h[i].img_err;
    rpp_status[i] = h[i].error == 1 ? -1 : h[i].status;
    if (iterations) iterations[i] = h[i].iterations;
  }
  return MANTIS_OK;
}

mantis_status mantis_synth_render(void* ctx, const mantis_synth_cam* cams, int32_t n, const uint64_t* seeds,
                                  uint8_t* out_dev) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !cams || n <= 0 || !seeds || !out_dev) return MANTIS_ERR_ARG;
  static_assert(sizeof(mantis_synth_cam) == sizeof(mantis_synth::Cam), "synth cam layout");
  mantis_synth::Cam* d_c;
  uint64_t* d_s;
  if (dalloc(c, &d_c, (size_t)n) || dalloc(c, &d_s, (size_t)n)) return MANTIS_ERR_OOM;
  HIP_OK(hipMemcpyAsync(d_c, cams, sizeof(mantis_synth::Cam) * n, hipMemcpyHostToDevice, c->s));
  HIP_OK(hipMemcpyAsync(d_s, seeds, sizeof(uint64_t) * n, hipMemcpyHostToDevice, c->s));
  size_t plane = (size_t)cams[0].w * cams[0].h * 3;
  dim3 g(blocks_for((size_t)cams[0].w * cams[0].h), n);
  k_synth<<<g, 256, 0, c->s>>>(d_c, d_s, out_dev, plane);
  HIP_OK(hipGetLastError());
  HIP_OK(hipStreamSynchronize(c->s));
  (void)hipFree(d_c);
  (void)hipFree(d_s);
  return MANTIS_OK;
}

mantis_status mantis_device_alloc(void* ctx, size_t bytes, void** dev_ptr) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !dev_ptr) return MANTIS_ERR_ARG;
  if (hipMalloc(dev_ptr, bytes) != hipSuccess) { c->err = "hipMalloc failed"; return MANTIS_ERR_OOM; }
  c->user_allocs.push_back(*dev_ptr);
  return MANTIS_OK;
}
mantis_status mantis_device_free(void* ctx, void* dev_ptr) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c) return MANTIS_ERR_ARG;
  auto it = std::find(c->user_allocs.begin(), c->user_allocs.end(), dev_ptr);
  if (it == c->user_allocs.end()) return MANTIS_ERR_ARG;
  c->user_allocs.erase(it);
  HIP_OK(hipFree(dev_ptr));
  return MANTIS_OK;
}
mantis_status mantis_memcpy_h2d(void* ctx, void* dst, const void* src, size_t bytes) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c) return MANTIS_ERR_ARG;
  HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  return MANTIS_OK;
}
mantis_status mantis_memcpy_d2h(void* ctx, void* dst, const void* src, size_t bytes) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c) return MANTIS_ERR_ARG;
  HIP_OK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  return MANTIS_OK;
}
mantis_status mantis_synchronize(void* ctx) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c) return MANTIS_ERR_ARG;
  HIP_OK(hipStreamSynchronize(c->s));
  return MANTIS_OK;
}
int32_t mantis_small_batch_frames(void* ctx) {
  const Ctx* c = (const Ctx*)ctx;
  return c ? c->fc_small_frames : -1;
}
int32_t mantis_kernel_times(void* ctx, const char** names, float* ms, int32_t max) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c) return 0;
  int n = (int)c->last_ms.size();
  for (int i = 0; i < n && i < max; i++) {
    if (names) names[i] = c->last_names[i].c_str();
    if (ms) ms[i] = c->last_ms[i];
  }
  return n;
}
mantis_status mantis_set_profiling(void* ctx, int32_t on) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c) return MANTIS_ERR_ARG;
  c->prof = on != 0;
  return MANTIS_OK;
}

}  // extern "C"

#include "gn_impl.hip"
#include "dense_impl.hip"
#include "markov_impl.hip"
#include "ros_wire.h"
