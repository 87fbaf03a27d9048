// Gauss–Newton rig refinement (new stage) and the RCCL
// exchange of its accumulators for camera-sharded rigs (§8 e). Included by
// api.hip (shares its Ctx). The residual rows, the 6x6 solve and the
// correspondences are in mk_gn.h (shared with the host build of the tests);
// here M^T M of M = [J | r] is built by one wave per rig with
// v_mfma_f64_16x16x4_f64, 4 residual rows per instruction.
#include <rccl/rccl.h>

#include "mk_gn.h"

namespace mk {

typedef double v4d __attribute__((ext_vector_type(4)));


__global__ __launch_bounds__(256) void k_gn_accum(const double* __restrict__ Twb, const GnCam* __restrict__ cams,
                                                  const double* __restrict__ obs, int n_obs, double* __restrict__ out28) {
  __shared__ double red[4][16][16];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double Rt[9], t[3];
  for (int a = 0; a < 3; a++) {
    for (int b = 0; b < 3; b++) Rt[3 * a + b] = Twb[4 * b + a];  // R_wb^T
    t[a] = Twb[4 * a + 3];
  }
  v4d acc = {0, 0, 0, 0};
  const int rows = 2 * n_obs;
  const int k = lane >> 4, m = lane & 15;
  for (int base = wave * 4; base < rows; base += 4 * 4) {
    double v = gn_entry(Rt, t, cams, obs, n_obs, base + k, m);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, acc, 0, 0, 0);
  }
  // D[row = (lane>>4) + 4r][col = lane & 15]
  for (int r = 0; r < 4; r++) red[wave][(lane >> 4) + 4 * r][lane & 15] = acc[r];
  __syncthreads();
  if (threadIdx.x == 0) {
    double D[7][7];
    for (int a = 0; a < 7; a++)
      for (int b = 0; b < 7; b++) D[a][b] = red[0][a][b] + red[1][a][b] + red[2][a][b] + red[3][a][b];
    int n = 0;
    for (int a = 0; a < 6; a++)
      for (int b = a; b < 6; b++) out28[n++] = D[a][b];
    for (int a = 0; a < 6; a++) out28[21 + a] = D[a][6];
    out28[27] = D[6][6];
  }
}

// ------------------------------------------------ batched rig GN (pipeline)
// cfg.gn_enable: after the per-camera pipeline and the rig fusion, the base
// pose of every rig is refined over all its cameras' quads, one quad-centre
// to cell-centre correspondence per quad (gn_quad_obs, mk_gn.h). The list is
// compacted in item order (block scan), so the MFMA sums are reproducible.

// The rig GN runs as (camera-sharded; one GPU: the same block functions in
// one launch, k_rig_gn_fused): k_rig_gn_obs (correspondences, once, with the fused
// pose) then, per iteration, k_rig_gn_acc (one block per rig builds M^T M with
// MFMA into a kGnSlot accumulator slot) -> [ncclAllReduce of every rig's slot
// when the rig's cameras are sharded over ranks] -> k_rig_gn_step (one lane
// per rig: Cholesky solve, SE(3) update, convergence flag). The single-GPU
// path is the same sequence without the all-reduce, so a camera-sharded run on
// a one-rank communicator is bit-identical to it, and with several ranks every
// rank solves the same summed system (no broadcast). The reference's
// multi-camera seam is the base->camera extrinsic chain of
// include/legacy/mantis/MonteCarlo.cpp:250-271 (T_w_c = T_w_b T_b_c).

// one rig, one block of 256: the accepted correspondences of this rank's
// cameras in item order (camera, quad), compacted by a block scan
// (R: the rig's state, in global memory or a block's LDS copy)
__device__ inline void gn_obs_block(const FrameDesc* __restrict__ frames, const FrameState* __restrict__ st,
                                    const QuadRec* __restrict__ quads, const GnCam* __restrict__ gncam, RigGnIO& R,
                                    int rig, int cams_local, double* obs_all, int obs_cap, double half,
                                    double spacing) {
  __shared__ double T[16];
  __shared__ int32_t scan[256];
  __shared__ int32_t nobs_s;
  const int t = threadIdx.x;
  if (t < 16) T[t] = R.Twb[t];
  __syncthreads();
  const GnCam* cams = gncam + (size_t)rig * cams_local;
  double* obs = obs_all + (size_t)rig * obs_cap * 6;
  const int n_items = cams_local * kMaxQuads;
  const int per = (n_items + 255) / 256;
  // pass 1: count accepted quads of this thread's item range; pass 2: write them in item order
  for (int pass = 0; pass < 2; pass++) {
    int pos = pass == 1 ? scan[t] : 0, cntv = 0;
    for (int it = t * per; it < n_items && it < (t + 1) * per; it++) {
      const int c = it / kMaxQuads, q = it % kMaxQuads;
      const int f = rig * cams_local + c;
      if (q >= st[f].n_quads) continue;
      // camera pose in the world from the base pose: T_wc = T_wb inv(T_cb)
      double Rbc[9], tbc[3], Rwc[9], Cw[3];
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) Rbc[3 * a + b] = cams[c].R_cb[3 * b + a];
      for (int a = 0; a < 3; a++) tbc[a] = -(Rbc[3 * a] * cams[c].t_cb[0] + Rbc[3 * a + 1] * cams[c].t_cb[1] +
                                              Rbc[3 * a + 2] * cams[c].t_cb[2]);
      for (int a = 0; a < 3; a++) {
        for (int b = 0; b < 3; b++)
          Rwc[3 * a + b] = T[4 * a] * Rbc[b] + T[4 * a + 1] * Rbc[3 + b] + T[4 * a + 2] * Rbc[6 + b];
        Cw[a] = T[4 * a] * tbc[0] + T[4 * a + 1] * tbc[1] + T[4 * a + 2] * tbc[2] + T[4 * a + 3];
      }
      double o[6];
      if (!gn_quad_obs(frames[f].cam, quads[(size_t)f * kMaxQuads + q].c, Rwc, Cw, half, spacing, o)) continue;
      if (pass == 1 && pos < obs_cap) {
        o[0] = (double)c;
        for (int e = 0; e < 6; e++) obs[(size_t)pos * 6 + e] = o[e];
      }
      pos++;
      cntv++;
    }
    if (pass == 0) {
      scan[t] = cntv;
      __syncthreads();
      if (t == 0) {
        int run = 0;
        for (int i = 0; i < 256; i++) { const int v = scan[i]; scan[i] = run; run += v; }
        nobs_s = run < obs_cap ? run : obs_cap;
      }
      __syncthreads();
    }
  }
  __syncthreads();
  if (t < 16) R.T0[t] = T[t];
  if (t == 0) {
    R.n_obs_local = nobs_s;
    R.n_obs = 0;
    R.iterations = 0;
    R.done = 0;
    R.cost0 = R.cost = 0;
  }
}
__global__ __launch_bounds__(256) void k_rig_gn_obs(const FrameDesc* __restrict__ frames,
                                                    const FrameState* __restrict__ st,
                                                    const QuadRec* __restrict__ quads,
                                                    const GnCam* __restrict__ gncam, RigGnIO* io, int cams_local,
                                                    double* __restrict__ obs_all, int obs_cap, double half,
                                                    double spacing) {
  RigGnIO& R = io[blockIdx.x];
  if (!R.valid) return;
  gn_obs_block(frames, st, quads, gncam, R, blockIdx.x, cams_local, obs_all, obs_cap, half, spacing);
}

// one rig, one block of 256: M^T M of M = [J | r] over this rank's
// correspondences about the current pose (4 waves, v_mfma_f64_16x16x4f64, 4
// residual rows per instruction), summed over the waves in a fixed order
// (out: the rig's kGnSlot accumulator slot, global or LDS)
__device__ inline void gn_acc_block(const GnCam* __restrict__ gncam, const RigGnIO& R, int rig, int cams_local,
                                    const double* obs_all, int obs_cap, double* out) {
  __shared__ double red[4][16][16];
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int n_obs = R.n_obs_local;
  const GnCam* cams = gncam + (size_t)rig * cams_local;
  const double* obs = obs_all + (size_t)rig * obs_cap * 6;
  double Rt[9], tw[3];
  for (int a = 0; a < 3; a++) {
    for (int b = 0; b < 3; b++) Rt[3 * a + b] = R.Twb[4 * b + a];
    tw[a] = R.Twb[4 * a + 3];
  }
  v4d acc = {0, 0, 0, 0};
  const int rows = 2 * n_obs;
  const int kk = lane >> 4, m = lane & 15;
  for (int base = wave * 4; base < rows; base += 16) {
    const double v = gn_entry(Rt, tw, cams, obs, n_obs, base + kk, m);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, acc, 0, 0, 0);
  }
  for (int r = 0; r < 4; r++) red[wave][(lane >> 4) + 4 * r][lane & 15] = acc[r];
  __syncthreads();
  if (t < kGnSlot) {
    double v = 0.0;
    if (t < 21) {  // upper triangle, row-major
      int a = 0, k = t;
      while (k >= 6 - a) { k -= 6 - a; a++; }
      const int b = a + k;
      v = red[0][a][b] + red[1][a][b] + red[2][a][b] + red[3][a][b];
    } else if (t < 27) {
      const int a = t - 21;
      v = red[0][a][6] + red[1][a][6] + red[2][a][6] + red[3][a][6];
    } else if (t == 27) {
      v = red[0][6][6] + red[1][6][6] + red[2][6][6] + red[3][6][6];
    } else if (t == 28) {
      v = (double)n_obs;
    }
    out[t] = v;
  }
}
__global__ __launch_bounds__(256) void k_rig_gn_acc(const GnCam* __restrict__ gncam, const RigGnIO* __restrict__ io,
                                                    int cams_local, const double* __restrict__ obs_all, int obs_cap,
                                                    double* __restrict__ acc_all) {
  const int rig = blockIdx.x;
  const RigGnIO& R = io[rig];
  double* out = acc_all + (size_t)rig * kGnSlot;
  if (!R.valid || R.done) {
    if (threadIdx.x < kGnSlot) out[threadIdx.x] = 0.0;
    return;
  }
  gn_acc_block(gncam, R, rig, cams_local, obs_all, obs_cap, out);
}

// one lane per rig: the summed system -> Cholesky solve -> T_w_b Exp(delta)
__device__ inline void gn_step_one(RigGnIO& R, const double* acc, int it) {
  if (!R.valid || R.done) return;
  if (it == 0) {
    R.n_obs = (int)acc[28];
    if (R.n_obs < 6) {  // too few correspondences over the rig: keep the fused pose
      R.done = 1;
      return;
    }
    R.cost0 = acc[27];
  }
  R.cost = acc[27];
  double Tn[16], d6[6];
  for (int e = 0; e < 16; e++) Tn[e] = R.Twb[e];
  if (!gn_solve6(acc, 1e-9, Tn, d6)) {
    R.done = 1;
  } else {
    for (int e = 0; e < 16; e++) R.Twb[e] = Tn[e];
    double dn = 0;
    for (int e = 0; e < 6; e++) dn += d6[e] * d6[e];
    if (dn < 1e-24) R.done = 1;
  }
  R.iterations = it + 1;
}
__global__ __launch_bounds__(64) void k_rig_gn_step(RigGnIO* io, const double* __restrict__ acc_all, int n_rigs,
                                                    int it) {
  const int rig = blockIdx.x * 64 + threadIdx.x;
  if (rig >= n_rigs) return;
  gn_step_one(io[rig], acc_all + (size_t)rig * kGnSlot, it);
}

// Single-GPU rig GN in one launch: one block per rig runs the correspondence
// pass and every iteration (accumulators -> solve -> update) on an LDS copy of
// the rig's state, stopping when the rig converges. The same block functions
// as the three-kernel sequence above (which the camera-sharded path keeps for
// its per-iteration all-reduce), so the results are bit-identical; what goes
// is 2 launches per iteration (the single-rig latency path's GN stage).
__global__ __launch_bounds__(256) void k_rig_gn_fused(const FrameDesc* __restrict__ frames,
                                                      const FrameState* __restrict__ st,
                                                      const QuadRec* __restrict__ quads,
                                                      const GnCam* __restrict__ gncam, RigGnIO* io, int cams_local,
                                                      double* obs_all, int obs_cap, double half, double spacing,
                                                      int iters) {
  __shared__ RigGnIO S;
  __shared__ double acc[kGnSlot];
  const int rig = blockIdx.x, t = threadIdx.x;
  if (t == 0) S = io[rig];
  __syncthreads();
  if (!S.valid) return;
  gn_obs_block(frames, st, quads, gncam, S, rig, cams_local, obs_all, obs_cap, half, spacing);
  __syncthreads();
  for (int it = 0; it < iters && !S.done; it++) {
    gn_acc_block(gncam, S, rig, cams_local, obs_all, obs_cap, acc);
    __syncthreads();
    if (t == 0) gn_step_one(S, acc, it);
    __syncthreads();
  }
  if (t == 0) io[rig] = S;
}

}  // namespace mk

namespace {
// cfg.gn_enable: refine every rig's fused base pose on the device. Tbc holds
// T_base_cam of this rank's cameras, rig-major (n_rigs x cams_local x 16); the
// frames of the last pipeline batch are those cameras in the same order. With
// a communicator (camera-sharded rigs) the accumulators are summed over ranks.
mantis_status run_rig_gn(Ctx* c, const double* Tbc, int n_rigs, int cams_local, mantis_result* out, bool use_comm) {
  const int n = n_rigs * cams_local;
  const int obs_cap = cams_local * kMaxQuads;
  std::vector<GnCam> gc(n);
  std::vector<RigGnIO> io(n_rigs);
  for (int f = 0; f < n; f++) {
    double inv[16];
    mat4_inv_rigid(Tbc + 16 * (size_t)f, inv);
    for (int a = 0; a < 3; a++) {
      for (int b = 0; b < 3; b++) gc[f].R_cb[3 * a + b] = inv[4 * a + b];
      gc[f].t_cb[a] = inv[4 * a + 3];
    }
  }
  for (int r = 0; r < n_rigs; r++) {
    std::memset(&io[r], 0, sizeof(RigGnIO));
    const double* q = out[r].orientation_xyzw;
    if (q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3] > 0.5) {
      quat_to_mat4(q, out[r].position, io[r].Twb);
      io[r].valid = 1;
    }
  }
  if (c->gn_rigs < n_rigs || c->gn_cpr != cams_local) {
    void* old[] = {c->d_gncam, c->d_rigio, c->d_gnobs, c->d_gnacc};
    for (void* p : old) (void)hipFree(p);
    c->d_gncam = nullptr;
    c->d_rigio = nullptr;
    c->d_gnobs = nullptr;
    c->d_gnacc = nullptr;
    c->gn_rigs = 0;
    mantis_status st = MANTIS_OK;
    if (dalloc(c, &c->d_gncam, (size_t)n) || dalloc(c, &c->d_rigio, (size_t)n_rigs) ||
        dalloc(c, &c->d_gnobs, (size_t)n_rigs * obs_cap * 6) || dalloc(c, &c->d_gnacc, (size_t)n_rigs * kGnSlot))
      st = MANTIS_ERR_OOM;
    if (use_comm) st = agree(c, st);  // the other ranks would wait in the per-iteration all-reduce
    if (st != MANTIS_OK) return st;
    c->gn_rigs = n_rigs;
    c->gn_cpr = cams_local;
  } else if (use_comm) {
    if (mantis_status st = agree(c, MANTIS_OK)) return st;
  }
  HIP_OK(hipMemcpyAsync(c->d_gncam, gc.data(), sizeof(GnCam) * n, hipMemcpyHostToDevice, c->s));
  HIP_OK(hipMemcpyAsync(c->d_rigio, io.data(), sizeof(RigGnIO) * n_rigs, hipMemcpyHostToDevice, c->s));
  const double spacing = c->cfg.grid_spacing, half = 4.5 * spacing;  // lines at -1.44 + 0.32 k, k = 0..9
  mark(c, "start");
  // small batches (latency): one launch, rig_gn 0.21 -> 0.17 ms at one rig per
  // call; large ones keep the three kernels (1024 rigs: 0.62 vs 0.89 ms fused).
  // Both forms are bit-identical (the camera-sharded path always takes the
  // three kernels: test_config4_8cam_1080p_rig_and_sharded_one_rank)
  if (!use_comm && (n <= c->fc_small_frames || c->gn_fused_all)) {
    k_rig_gn_fused<<<n_rigs, 256, 0, c->s>>>(c->d_frames, c->d_st, c->d_quads, c->d_gncam, c->d_rigio, cams_local,
                                              c->d_gnobs, obs_cap, half, spacing, c->cfg.gn_iterations);
  } else {
    k_rig_gn_obs<<<n_rigs, 256, 0, c->s>>>(c->d_frames, c->d_st, c->d_quads, c->d_gncam, c->d_rigio, cams_local,
                                            c->d_gnobs, obs_cap, half, spacing);
    for (int it = 0; it < c->cfg.gn_iterations; it++) {
      k_rig_gn_acc<<<n_rigs, 256, 0, c->s>>>(c->d_gncam, c->d_rigio, cams_local, c->d_gnobs, obs_cap, c->d_gnacc);
      if (use_comm) {
        ncclResult_t r = ncclAllReduce(c->d_gnacc, c->d_gnacc, (size_t)n_rigs * kGnSlot, ncclFloat64, ncclSum,
                                       (ncclComm_t)c->comm, c->s);
        if (r != ncclSuccess) { c->err = std::string("ncclAllReduce: ") + ncclGetErrorString(r); return MANTIS_ERR_COMM; }
      }
      k_rig_gn_step<<<(n_rigs + 63) / 64, 64, 0, c->s>>>(c->d_rigio, c->d_gnacc, n_rigs, it);
    }
  }
  mark(c, "rig_gn");
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(io.data(), c->d_rigio, sizeof(RigGnIO) * n_rigs, hipMemcpyDeviceToHost, c->s));
  HIP_OK(wait_stream(c, n));
  finish_profile(c, true);
  c->gn_last_rigs = n_rigs;
  c->gn_last_local = cams_local;
  for (int r = 0; r < n_rigs; r++) {
    if (!io[r].valid || io[r].iterations <= 0) continue;
    double R[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) R[i * 3 + j] = io[r].Twb[i * 4 + j];
    mk::Quat q = basis_to_quat(R);
    out[r].orientation_xyzw[0] = q.x;
    out[r].orientation_xyzw[1] = q.y;
    out[r].orientation_xyzw[2] = q.z;
    out[r].orientation_xyzw[3] = q.w;
    for (int i = 0; i < 3; i++) out[r].position[i] = io[r].Twb[i * 4 + 3];
    out[r].gn_iterations = io[r].iterations;
    out[r].gn_cost = io[r].cost;
  }
  return MANTIS_OK;
}
}  // namespace

extern "C" {

mantis_status mantis_gn_accumulate(void* ctx, const double* T_w_b, const double* T_base_cam, int32_t n_cams,
                                   const double* obs, int32_t n_obs, double* acc28) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !T_w_b || !T_base_cam || n_cams <= 0 || (n_obs > 0 && !obs) || !acc28) return MANTIS_ERR_ARG;
  std::vector<GnCam> cams(n_cams);
  for (int i = 0; i < n_cams; i++) {
    double inv[16];
    mat4_inv_rigid(T_base_cam + 16 * i, inv);
    for (int a = 0; a < 3; a++) {
      for (int b = 0; b < 3; b++) cams[i].R_cb[3 * a + b] = inv[4 * a + b];
      cams[i].t_cb[a] = inv[4 * a + 3];
    }
  }
  for (int i = 0; i < n_obs; i++)
    if ((int)obs[6 * i] < 0 || (int)obs[6 * i] >= n_cams) { c->err = "gn: observation camera index"; return MANTIS_ERR_ARG; }
  double* d_T;
  GnCam* d_c;
  double* d_o;
  double* d_out;
  if (dalloc(c, &d_T, 16) || dalloc(c, &d_c, (size_t)n_cams) || dalloc(c, &d_o, (size_t)6 * std::max(n_obs, 1)) ||
      dalloc(c, &d_out, 28))
    return MANTIS_ERR_OOM;
  HIP_OK(hipMemcpyAsync(d_T, T_w_b, sizeof(double) * 16, hipMemcpyHostToDevice, c->s));
  HIP_OK(hipMemcpyAsync(d_c, cams.data(), sizeof(GnCam) * n_cams, hipMemcpyHostToDevice, c->s));
  if (n_obs > 0) HIP_OK(hipMemcpyAsync(d_o, obs, sizeof(double) * 6 * n_obs, hipMemcpyHostToDevice, c->s));
  k_gn_accum<<<1, 256, 0, c->s>>>(d_T, d_c, d_o, n_obs, d_out);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(acc28, d_out, sizeof(double) * 28, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  void* ps[] = {d_T, d_c, d_o, d_out};
  for (void* p : ps) (void)hipFree(p);
  return MANTIS_OK;
}

mantis_status mantis_gn_solve(const double* acc28, double lambda, double* T_w_b, double* delta6) {
  if (!acc28 || !T_w_b) return MANTIS_ERR_ARG;
  return mk::gn_solve6(acc28, lambda, T_w_b, delta6) ? MANTIS_OK : MANTIS_ERR_ARG;
}

mantis_status mantis_comm_unique_id(void* id128) {
  if (!id128) return MANTIS_ERR_ARG;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return MANTIS_ERR_COMM;
  std::memcpy(id128, &id, sizeof(id));
  return MANTIS_OK;
}

mantis_status mantis_comm_init(void* ctx, const void* id128, int32_t nranks, int32_t rank) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !id128 || nranks <= 0 || rank < 0 || rank >= nranks) return MANTIS_ERR_ARG;
  ncclUniqueId id;
  std::memcpy(&id, id128, sizeof(id));
  ncclComm_t comm;
  HIP_OK(hipSetDevice(c->cfg.device));
  if (c->comm) {  // re-initialisation replaces the previous communicator
    HIP_OK(hipStreamSynchronize(c->s));
    (void)ncclCommDestroy((ncclComm_t)c->comm);
    c->comm = nullptr;
    c->nranks = 1;
    c->rank = 0;
  }
  ncclResult_t r = ncclCommInitRank(&comm, nranks, id, rank);
  if (r != ncclSuccess) { c->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r); return MANTIS_ERR_COMM; }
  int cnt = 0, me = -1;
  if (ncclCommCount(comm, &cnt) != ncclSuccess || ncclCommUserRank(comm, &me) != ncclSuccess || cnt != nranks ||
      me != rank) {
    (void)ncclCommDestroy(comm);
    c->err = "ncclCommCount/UserRank disagree with the requested rank layout";
    return MANTIS_ERR_COMM;
  }
  // the failure flag of the sharded call's agreement steps (agree(), api.hip):
  // allocated here so agreeing never needs an allocation
  if (!c->d_agree && dalloc(c, &c->d_agree, 4) != MANTIS_OK) {
    (void)ncclCommDestroy(comm);
    return MANTIS_ERR_OOM;
  }
  c->comm = comm;
  c->nranks = nranks;
  c->rank = rank;
  return MANTIS_OK;
}

mantis_status mantis_comm_info(void* ctx, int32_t* nranks, int32_t* rank) {
  Ctx* c = (Ctx*)ctx;
  if (!c || !nranks || !rank) return MANTIS_ERR_ARG;
  if (!c->comm) { c->err = "comm not initialised (mantis_comm_init)"; return MANTIS_ERR_STATE; }
  *nranks = c->nranks;
  *rank = c->rank;
  return MANTIS_OK;
}

mantis_status mantis_get_rig_gn(void* ctx, int32_t rig, mantis_rig_gn_info* info, double* obs, int32_t cap) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !info || rig < 0 || cap < 0 || (cap > 0 && !obs)) return MANTIS_ERR_ARG;
  if (rig >= c->gn_last_rigs || !c->d_rigio) { c->err = "no rig GN result for that rig (gn_enable, last batch)"; return MANTIS_ERR_STATE; }
  RigGnIO io;
  HIP_OK(hipMemcpyAsync(&io, c->d_rigio + rig, sizeof(io), hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  std::memcpy(info->T_init, io.T0, sizeof(io.T0));
  std::memcpy(info->T_final, io.Twb, sizeof(io.Twb));
  info->cost0 = io.cost0;
  info->cost = io.cost;
  info->valid = io.valid;
  info->iterations = io.iterations;
  info->n_obs = io.n_obs;
  info->n_obs_local = io.n_obs_local;
  const int k = std::min(cap, io.valid ? io.n_obs_local : 0);
  const size_t obs_cap = (size_t)c->gn_last_local * kMaxQuads;
  if (k > 0)
    HIP_OK(hipMemcpy(obs, c->d_gnobs + (size_t)rig * obs_cap * 6, sizeof(double) * 6 * k, hipMemcpyDeviceToHost));
  return MANTIS_OK;
}

mantis_status mantis_gn_allreduce(void* ctx, double* acc28) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !acc28) return MANTIS_ERR_ARG;
  if (!c->comm) { c->err = "comm not initialised (mantis_comm_init)"; return MANTIS_ERR_STATE; }
  if (!c->d_gn28 && dalloc(c, &c->d_gn28, 28) != MANTIS_OK) return MANTIS_ERR_OOM;
  HIP_OK(hipMemcpyAsync(c->d_gn28, acc28, sizeof(double) * 28, hipMemcpyHostToDevice, c->s));
  ncclResult_t r = ncclAllReduce(c->d_gn28, c->d_gn28, 28, ncclFloat64, ncclSum, (ncclComm_t)c->comm, c->s);
  if (r != ncclSuccess) { c->err = std::string("ncclAllReduce: ") + ncclGetErrorString(r); return MANTIS_ERR_COMM; }
  HIP_OK(hipMemcpyAsync(acc28, c->d_gn28, sizeof(double) * 28, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  return MANTIS_OK;
}

}  // extern "C"
