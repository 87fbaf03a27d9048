// Dense hypothesis scoring with an argmin (BASELINE config 5, SURVEY §8 d/e):
// n hypotheses (e.g. 81 shifts x 4 yaws x 50 perturbations = 16,200) scored
// against the 720 map.yaml landmarks with the fast evaluator
// (evaluateHypotheses, HypothesisEvaluation.h:31-41, 71-158; one wave per
// hypothesis, k_score_api), reduced on the device to the lowest error with
// the first index on ties (the strict "<" of the reference's best-1 choice).
// Sharded over ranks: every rank scores a contiguous block of the global
// hypothesis list; one ncclAllGather of (err, global index) per rank (16 B)
// and the same first-minimum rule give every rank the global winner. Included
// by api.hip (shares its Ctx).

namespace mk {

// one block: lowest err, then lowest index
__global__ __launch_bounds__(1024) void k_argmin(const double* __restrict__ err, int n, int64_t base,
                                                 double* __restrict__ out2) {
  __shared__ double se[1024];
  __shared__ int si[1024];
  const int t = threadIdx.x;
  double be = DBL_MAX;
  int bi = 0x7fffffff;
  for (int i = t; i < n; i += 1024) {
    const double e = err[i];
    if (e < be) { be = e; bi = i; }  // strided scan: ascending i within a thread
  }
  se[t] = be;
  si[t] = bi;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if (t < s) {
      const double e2 = se[t + s];
      const int i2 = si[t + s];
      if (e2 < se[t] || (e2 == se[t] && i2 < si[t])) { se[t] = e2; si[t] = i2; }
    }
    __syncthreads();
  }
  if (t == 0) {
    out2[0] = se[0];
    out2[1] = si[0] == 0x7fffffff ? -1.0 : (double)(base + si[0]);
  }
}

// Batched dense scoring (mantis_score_argmin_batch): one launch over every
// frame's hypothesis block (blockIdx.y = frame, kDenseHyps hypotheses per block,
// the screened fast scorer of k_score_api), then one argmin block per frame.
struct DenseJob {
  const uint8_t* mask;  // W*H bytes or null
  const double* c2w;    // n x 12
  int32_t n, err_off;   // hypotheses; offset into the batch's error array
  int64_t index_base;
};
__global__ __launch_bounds__(64 * kApiHyps) void k_score_api_batch(const FrameDesc* __restrict__ frames,
                                                                   const DenseJob* __restrict__ jobs, Landmarks lmk,
                                                                   double* __restrict__ err, int32_t* __restrict__ nproj) {
  const int f = blockIdx.y;
  const DenseJob J = jobs[f];
  if ((int)blockIdx.x * kDenseHyps >= J.n) return;
  const FrameDesc fd = frames[f];
  if (J.mask)
    score_api_fast<kDenseHyps>(fd, &frames[f].cam, MaskBytes{J.mask}, lmk, J.c2w, J.n, err + J.err_off,
                               nproj + J.err_off);
  else
    score_api_fast<kDenseHyps>(fd, &frames[f].cam, MaskNone{}, lmk, J.c2w, J.n, err + J.err_off, nproj + J.err_off);
}
__global__ __launch_bounds__(1024) void k_argmin_batch(const DenseJob* __restrict__ jobs, const double* __restrict__ err,
                                                       double* __restrict__ out2) {
  const DenseJob J = jobs[blockIdx.x];
  __shared__ double se[1024];
  __shared__ int si[1024];
  const int t = threadIdx.x;
  double be = DBL_MAX;
  int bi = 0x7fffffff;
  for (int i = t; i < J.n; i += 1024) {
    const double e = err[J.err_off + i];
    if (e < be) { be = e; bi = i; }
  }
  se[t] = be;
  si[t] = bi;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if (t < s) {
      const double e2 = se[t + s];
      const int i2 = si[t + s];
      if (e2 < se[t] || (e2 == se[t] && i2 < si[t])) { se[t] = e2; si[t] = i2; }
    }
    __syncthreads();
  }
  if (t == 0) {
    out2[2 * blockIdx.x] = se[0];
    out2[2 * blockIdx.x + 1] = si[0] == 0x7fffffff ? -1.0 : (double)(J.index_base + si[0]);
  }
}

}  // namespace mk

extern "C" {

// (err, global index) pairs of nranks shards -> the first minimum; an index
// of -1 marks an empty shard. Host function (also used by the CPU tests).
mantis_status mantis_argmin_pick(const double* pairs, int32_t nranks, double* best_err, int64_t* best_idx) {
  if (!pairs || nranks <= 0 || !best_err || !best_idx) return MANTIS_ERR_ARG;
  double be = DBL_MAX;
  int64_t bi = -1;
  for (int r = 0; r < nranks; r++) {
    const double e = pairs[2 * r];
    const int64_t i = (int64_t)pairs[2 * r + 1];
    if (i < 0) continue;
    if (bi < 0 || e < be || (e == be && i < bi)) { be = e; bi = i; }
  }
  *best_err = be;
  *best_idx = bi;
  return MANTIS_OK;
}

}  // extern "C"

namespace {
// dev: mask / c2w are device pointers read in place (mantis_score_argmin_dev)
mantis_status score_argmin_impl(void* ctx, const mantis_image* img, const uint8_t* mask, const double* c2w,
                                int32_t n, int64_t index_base, int32_t use_comm, double* best_err,
                                int64_t* best_idx, bool dev) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !img || !c2w || n < 0 || !best_err || !best_idx) return MANTIS_ERR_ARG;
  if (use_comm && !c->comm) { c->err = "comm not initialised (mantis_comm_init)"; return MANTIS_ERR_STATE; }
  // every rank-local failure from here to the exchange is agreed on first
  // (agree(), api.hip), so no rank is left alone in the all-gather
  const auto prepare = [&]() -> mantis_status {
    if (!c->d_lm) { c->err = "map not set"; return MANTIS_ERR_STATE; }
    if (use_comm && (c->nranks < 1 || c->nranks > 63)) { c->err = "argmin exchange supports 1..63 ranks"; return MANTIS_ERR_ARG; }
    int W, H;
    mantis_status st = stage_frames(c, img, 1, W, H);
    if (st != MANTIS_OK) return st;
    const size_t cap = (size_t)(n > 0 ? n : 1);
    if (cap > c->dense_cap) {
      (void)hipFree(c->d_dense_c2w);
      (void)hipFree(c->d_dense_err);
      (void)hipFree(c->d_dense_np);
      c->d_dense_c2w = nullptr;
      c->d_dense_err = nullptr;
      c->d_dense_np = nullptr;
      c->dense_cap = 0;
      if (dalloc(c, &c->d_dense_c2w, 12 * cap) != MANTIS_OK || dalloc(c, &c->d_dense_err, cap) != MANTIS_OK ||
          dalloc(c, &c->d_dense_np, cap) != MANTIS_OK)
        return MANTIS_ERR_OOM;
      c->dense_cap = cap;
    }
    if (!c->d_pairs) {
      if (dalloc(c, &c->d_pairs, (size_t)2 * 64) != MANTIS_OK) return MANTIS_ERR_OOM;
      c->dense_pairs_cap = 128;
    }
    return MANTIS_OK;
  };
  mantis_status st = prepare();
  if (use_comm) st = agree(c, st, 1);
  if (st != MANTIS_OK) return st;
  const int W = img->width, H = img->height;
  const uint8_t* d_mask = nullptr;
  const double* d_c2w = c->d_dense_c2w;
  if (dev) {
    d_mask = mask;
    d_c2w = c2w;
  } else {
    if (mask) {
      HIP_OK(hipMemcpyAsync(c->d_mask, mask, (size_t)W * H, hipMemcpyHostToDevice, c->s));
      d_mask = c->d_mask;
    }
    if (n > 0) HIP_OK(hipMemcpyAsync(c->d_dense_c2w, c2w, sizeof(double) * 12 * n, hipMemcpyHostToDevice, c->s));
  }
  Landmarks L = lmk_of(c);
  mark(c, "start");
  if (n > 0) {
    k_score_api<<<(n + kApiHyps - 1) / kApiHyps, 64 * kApiHyps, 0, c->s>>>(c->d_frames, d_mask, L, d_c2w, n, 1, c->d_dense_err,
                                               c->d_dense_np);
    mark(c, "score_dense");
  }
  k_argmin<<<1, 1024, 0, c->s>>>(c->d_dense_err, n, index_base, c->d_pairs);
  mark(c, "argmin");
  HIP_OK(hipGetLastError());
  int nr = 1;
  if (use_comm) {
    nr = c->nranks;  // checked against ncclCommCount in mantis_comm_init, range checked above
    ncclResult_t r = ncclAllGather(c->d_pairs, c->d_pairs + 2, 2, ncclFloat64, (ncclComm_t)c->comm, c->s);
    if (r != ncclSuccess) { c->err = std::string("ncclAllGather: ") + ncclGetErrorString(r); return MANTIS_ERR_COMM; }
    mark(c, "allgather");
  }
  double h[2 * 64];
  HIP_OK(hipMemcpyAsync(h, c->d_pairs + (use_comm ? 2 : 0), sizeof(double) * 2 * nr, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  finish_profile(c);
  return mantis_argmin_pick(h, nr, best_err, best_idx);
}
}  // namespace

extern "C" {

mantis_status mantis_score_argmin_batch(void* ctx, const mantis_image* imgs, int32_t n_frames,
                                        const uint8_t* const* masks_dev, const double* const* c2w_dev,
                                        const int32_t* n_hyps, const int64_t* index_base, int32_t use_comm,
                                        double* best_err, int64_t* best_idx) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !imgs || n_frames <= 0 || !c2w_dev || !n_hyps || !index_base || !best_err || !best_idx)
    return MANTIS_ERR_ARG;
  if (use_comm && !c->comm) { c->err = "comm not initialised (mantis_comm_init)"; return MANTIS_ERR_STATE; }
  std::vector<DenseJob> jobs(n_frames);
  int maxn = 0;
  // every rank-local failure up to the exchange (a rejected image, a bad
  // hypothesis block, an allocation) and the frame count are agreed on with
  // the other ranks first (agree(), api.hip): ranks fail together instead of
  // leaving the others in an all-gather, and never all-gather different sizes
  const auto prepare = [&]() -> mantis_status {
    if (!c->d_lm) { c->err = "map not set"; return MANTIS_ERR_STATE; }
    if (use_comm && (c->nranks < 1 || c->nranks > 63)) { c->err = "argmin exchange supports 1..63 ranks"; return MANTIS_ERR_ARG; }
    int W, H;
    mantis_status st = stage_frames(c, imgs, n_frames, W, H);
    if (st != MANTIS_OK) return st;
    size_t tot = 0;
    for (int f = 0; f < n_frames; f++) {
      if (n_hyps[f] < 0 || (n_hyps[f] > 0 && !c2w_dev[f])) { c->err = "bad hypothesis block"; return MANTIS_ERR_ARG; }
      jobs[f] = DenseJob{masks_dev ? masks_dev[f] : nullptr, c2w_dev[f], n_hyps[f], (int32_t)tot, index_base[f]};
      tot += (size_t)n_hyps[f];
      maxn = std::max(maxn, n_hyps[f]);
    }
    if (tot > (size_t)INT32_MAX) { c->err = "too many hypotheses in one batch"; return MANTIS_ERR_ARG; }
    const size_t cap = std::max<size_t>(tot, 1);
    if (cap > c->dense_cap) {
      (void)hipFree(c->d_dense_err);
      (void)hipFree(c->d_dense_np);
      (void)hipFree(c->d_dense_c2w);
      c->d_dense_err = c->d_dense_c2w = nullptr;
      c->d_dense_np = nullptr;
      c->dense_cap = 0;
      if (dalloc(c, &c->d_dense_c2w, 12 * cap) != MANTIS_OK || dalloc(c, &c->d_dense_err, cap) != MANTIS_OK ||
          dalloc(c, &c->d_dense_np, cap) != MANTIS_OK)
        return MANTIS_ERR_OOM;
      c->dense_cap = cap;
    }
    // at least the single-frame call's 64 pairs (mantis_score_argmin shares d_pairs)
    const size_t pair_cap = std::max<size_t>((size_t)2 * n_frames * (use_comm ? c->nranks + 1 : 1), 128);
    if (pair_cap > c->dense_pairs_cap) {
      (void)hipFree(c->d_pairs);
      c->d_pairs = nullptr;
      c->dense_pairs_cap = 0;
      if (dalloc(c, &c->d_pairs, pair_cap) != MANTIS_OK) return MANTIS_ERR_OOM;
      c->dense_pairs_cap = pair_cap;
    }
    // the job table has its own capacity: d_pairs may already be large enough
    // (single-frame call) when the first batch arrives
    if ((size_t)n_frames > c->dense_jobs_cap) {
      (void)hipFree(c->d_dense_jobs);
      c->d_dense_jobs = nullptr;
      c->dense_jobs_cap = 0;
      if (dalloc(c, (DenseJob**)&c->d_dense_jobs, (size_t)n_frames) != MANTIS_OK) return MANTIS_ERR_OOM;
      c->dense_jobs_cap = (size_t)n_frames;
    }
    return MANTIS_OK;
  };
  mantis_status st = prepare();
  if (use_comm) st = agree(c, st, n_frames);
  if (st != MANTIS_OK) return st;
  DenseJob* d_jobs = (DenseJob*)c->d_dense_jobs;
  HIP_OK(hipMemcpyAsync(d_jobs, jobs.data(), sizeof(DenseJob) * n_frames, hipMemcpyHostToDevice, c->s));
  Landmarks L = lmk_of(c);
  mark(c, "start");
  if (maxn > 0)
    k_score_api_batch<<<dim3((maxn + kDenseHyps - 1) / kDenseHyps, n_frames), 64 * kApiHyps, 0, c->s>>>(
        c->d_frames, d_jobs, L, c->d_dense_err, c->d_dense_np);
  mark(c, "score_dense");
  k_argmin_batch<<<n_frames, 1024, 0, c->s>>>(d_jobs, c->d_dense_err, c->d_pairs);
  mark(c, "argmin");
  HIP_OK(hipGetLastError());
  int nr = 1;
  if (use_comm) {
    nr = c->nranks;
    ncclResult_t r = ncclAllGather(c->d_pairs, c->d_pairs + 2 * n_frames, 2 * (size_t)n_frames, ncclFloat64,
                                   (ncclComm_t)c->comm, c->s);
    if (r != ncclSuccess) { c->err = std::string("ncclAllGather: ") + ncclGetErrorString(r); return MANTIS_ERR_COMM; }
    mark(c, "allgather");
  }
  std::vector<double> h((size_t)2 * n_frames * nr);
  HIP_OK(hipMemcpyAsync(h.data(), c->d_pairs + (use_comm ? 2 * n_frames : 0), sizeof(double) * h.size(),
                        hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  finish_profile(c);
  std::vector<double> pr((size_t)2 * nr);
  for (int f = 0; f < n_frames; f++) {
    for (int r = 0; r < nr; r++) {  // rank r's pair of frame f
      pr[2 * r] = h[(size_t)r * 2 * n_frames + 2 * f];
      pr[2 * r + 1] = h[(size_t)r * 2 * n_frames + 2 * f + 1];
    }
    mantis_argmin_pick(pr.data(), nr, &best_err[f], &best_idx[f]);
  }
  return MANTIS_OK;
}

mantis_status mantis_score_argmin(void* ctx, const mantis_image* img, const uint8_t* mask, const double* c2w,
                                  int32_t n, int64_t index_base, int32_t use_comm, double* best_err,
                                  int64_t* best_idx) {
  return score_argmin_impl(ctx, img, mask, c2w, n, index_base, use_comm, best_err, best_idx, false);
}

mantis_status mantis_score_argmin_dev(void* ctx, const mantis_image* img, const uint8_t* mask_dev,
                                      const double* c2w_dev, int32_t n, int64_t index_base, int32_t use_comm,
                                      double* best_err, int64_t* best_idx) {
  return score_argmin_impl(ctx, img, mask_dev, c2w_dev, n, index_base, use_comm, best_err, best_idx, true);
}

}  // extern "C"
