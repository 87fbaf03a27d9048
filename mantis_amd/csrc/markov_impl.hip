// Markov yaw filter: include/mantis3/Markov.cpp's MarkovModel
// (included but unused upstream) as a batch of 360-bin yaw distributions held
// in the context's HBM, one per camera stream / rig. Included by api.hip.
//
// Every operation is the reference's updateWeights (Markov.cpp:76-124): a
// circular Gaussian blur of the 360 bins, aux[i] = sum_j (y_j / (stddev
// sqrt(2 pi))) exp(-(i - mu_j)^2 / (2 stddev^2)), summed in the reference's j
// order, then normalized -- 130k terms per filter, one block of 384 lanes per
// filter (lane i owns bin i). The exp factors depend only on |i - mu_j| <= 180,
// so the host computes those 181 values per operation with the C library (the
// same values the oracle's calculateWeight evaluates) and the device does the
// divisions, products and ordered sums: the planes are bit-identical to the
// oracle's (oracle/o_markov.cpp). Yaw bins come from the hypotheses' w2c bases
// (getRPY, degrees, wrapped to [0, 360)) on the host.

namespace mk {

// updateWeights on y (LDS) into y, lane i = bin i; red = LDS scratch (1 double)
__device__ inline void markov_update(double* y, double* aux, double* red, const MarkovOp& op) {
  const int i = threadIdx.x;
  if (i < kYawBins) {
    double max = 0.0;
    const int diff = kYawBins / 2 + i;
    if (i <= kYawBins / 2) {
      for (int j = 0; j < diff; ++j) max += (y[j] / op.den) * op.E[i - j >= 0 ? i - j : j - i];
      for (int j = diff; j < kYawBins; ++j) max += (y[j] / op.den) * op.E[i + kYawBins - j];
    } else {
      for (int j = i; j < diff; ++j) max += (y[j % kYawBins] / op.den) * op.E[j - i];
      for (int j = diff % kYawBins; j < i; ++j) max += (y[j] / op.den) * op.E[i - j];
    }
    aux[i] = max;
  }
  __syncthreads();
  if (i == 0) {  // normalize (Markov.cpp:62-74): sum in bin order
    double sum = 0.0;
    for (int k = 0; k < kYawBins; ++k) sum += aux[k];
    *red = sum;
  }
  __syncthreads();
  if (i < kYawBins) y[i] = aux[i] / *red;
  __syncthreads();
}

__global__ __launch_bounds__(384) void k_markov(double* __restrict__ planes, const MarkovOp* __restrict__ ops) {
  __shared__ double y[kYawBins], aux[kYawBins], red;
  const int f = blockIdx.x, i = threadIdx.x;
  const MarkovOp& op = ops[f];
  if (op.kind < 0) return;
  double* p = planes + (size_t)f * kYawBins;
  if (i < kYawBins) {
    if (op.kind == 2) y[i] = p[(i + op.off) % kYawBins];  // convolve's displacement
    else y[i] = i == op.bin ? 1.0 : 0.0;                   // one-hot at the yaw bin
  }
  __syncthreads();
  markov_update(y, aux, &red, op);
  if (op.kind != 1) {
    if (i < kYawBins) p[i] = y[i];
    return;
  }
  // senseFusion(markovPlane) (Markov.cpp:164-183): both scaled by sqrt(DBL_MAX), multiplied, normalized
  const double newMax = 1.3407807929942596e+154;  // sqrt(DBL_MAX)
  if (i < kYawBins) aux[i] = (p[i] * newMax) * (y[i] * newMax);
  __syncthreads();
  if (i == 0) {
    double sum = 0.0;
    for (int k = 0; k < kYawBins; ++k) sum += aux[k];
    red = sum;
  }
  __syncthreads();
  if (i < kYawBins) p[i] = aux[i] / red;
}

// updateHypothesis (Markov.cpp:207-222): error = error * 1 / p[bin]
__global__ __launch_bounds__(256) void k_markov_weight(const double* __restrict__ plane,
                                                       const int32_t* __restrict__ bins, int n,
                                                       double* __restrict__ err) {
  const int h = blockIdx.x * 256 + threadIdx.x;
  if (h < n) err[h] = err[h] * 1 / plane[bins[h]];
}

}  // namespace mk

namespace {

// yaw bin of a hypothesis pose (w2c basis): getRPY, degrees, wrapped
// (Markov.cpp:15-27, 185-196); 360 after wrapping -> bin 0
int markov_bin(const double* R) {
  double roll, pitch, yaw;
  mk::basis_to_rpy(R, &roll, &pitch, &yaw);
  yaw *= 180.0 / M_PI;
  if (yaw < 0) yaw += mk::kYawBins;
  const int b = (int)yaw;
  return b >= mk::kYawBins ? b - mk::kYawBins : b;
}

void markov_gauss(MarkovOp& op, double stddev) {
  op.den = stddev * sqrt(2 * M_PI);
  for (int d = 0; d <= 180; d++) {
    const double x = (double)d;
    op.E[d] = exp(-(x * x / (2 * stddev * stddev)));
  }
}

mantis_status markov_run(Ctx* c, std::vector<MarkovOp>& ops) {
  const int n = c->markov_n;
  if (!c->d_mops && dalloc(c, &c->d_mops, (size_t)n) != MANTIS_OK) return MANTIS_ERR_OOM;
  HIP_OK(hipMemcpyAsync(c->d_mops, ops.data(), sizeof(MarkovOp) * n, hipMemcpyHostToDevice, c->s));
  k_markov<<<n, 384, 0, c->s>>>(c->d_markov, c->d_mops);
  HIP_OK(hipGetLastError());
  HIP_OK(hipStreamSynchronize(c->s));
  return MANTIS_OK;
}

}  // namespace

extern "C" {

mantis_status mantis_markov_init(void* ctx, int32_t n_filters, const double* w2c_R) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || n_filters <= 0 || n_filters > (1 << 20) || !w2c_R) return MANTIS_ERR_ARG;
  if (n_filters != c->markov_n) {
    HIP_OK(hipStreamSynchronize(c->s));
    (void)hipFree(c->d_markov);
    (void)hipFree(c->d_mops);
    c->d_markov = nullptr;
    c->d_mops = nullptr;
    c->markov_n = 0;
    if (dalloc(c, &c->d_markov, (size_t)n_filters * mk::kYawBins) != MANTIS_OK) return MANTIS_ERR_OOM;
    c->markov_n = n_filters;
  }
  std::vector<MarkovOp> ops(n_filters);
  for (int f = 0; f < n_filters; f++) {
    ops[f].kind = 0;
    ops[f].bin = markov_bin(w2c_R + 9 * (size_t)f);
    markov_gauss(ops[f], 3);
  }
  return markov_run(c, ops);
}

mantis_status mantis_markov_sense(void* ctx, const double* w2c_R, const int32_t* active) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !w2c_R) return MANTIS_ERR_ARG;
  if (!c->markov_n) { c->err = "markov filters not initialised (mantis_markov_init)"; return MANTIS_ERR_STATE; }
  std::vector<MarkovOp> ops(c->markov_n);
  for (int f = 0; f < c->markov_n; f++) {
    ops[f].kind = (!active || active[f]) ? 1 : -1;
    if (ops[f].kind < 0) continue;
    ops[f].bin = markov_bin(w2c_R + 9 * (size_t)f);
    markov_gauss(ops[f], 3.5);  // FWHM 8.25 deg (Markov.cpp:194-195)
  }
  return markov_run(c, ops);
}

mantis_status mantis_markov_convolve(void* ctx, const double* dtheta, const double* dt, const int32_t* active) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || !dtheta || !dt) return MANTIS_ERR_ARG;
  if (!c->markov_n) { c->err = "markov filters not initialised (mantis_markov_init)"; return MANTIS_ERR_STATE; }
  std::vector<MarkovOp> ops(c->markov_n);
  for (int f = 0; f < c->markov_n; f++) {
    ops[f].kind = (!active || active[f]) ? 2 : -1;
    if (ops[f].kind < 0) continue;
    if (!std::isfinite(dtheta[f]) || std::fabs(dtheta[f]) > 1e6) { c->err = "markov convolve: dTheta out of range"; return MANTIS_ERR_ARG; }
    int conv = (int)dtheta[f] * 180 / M_PI;  // (int) binds to dTheta first (Markov.cpp:230)
    if (dtheta[f] > 0) ops[f].off = (mk::kYawBins - conv % mk::kYawBins) % mk::kYawBins;
    else ops[f].off = (-conv) % mk::kYawBins;
    markov_gauss(ops[f], 1.0 / 3.0 * dt[f] * 11.5 / 30.0);  // GAUSSIAN_WIDTH_NOISE*dt*11.5/30.0 (:250)
  }
  return markov_run(c, ops);
}

mantis_status mantis_markov_weight(void* ctx, int32_t filter, const double* w2c_R, int32_t n, double* error) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c || n < 0 || (n > 0 && (!w2c_R || !error))) return MANTIS_ERR_ARG;
  if (filter < 0 || filter >= c->markov_n) { c->err = "markov: no such filter"; return MANTIS_ERR_STATE; }
  if (n == 0) return MANTIS_OK;
  std::vector<int32_t> bins(n);
  for (int h = 0; h < n; h++) bins[h] = markov_bin(w2c_R + 9 * (size_t)h);
  int32_t* d_b = nullptr;
  double* d_e = nullptr;
  struct Free {  // the temporaries are freed on every path (also the HIP_OK early returns)
    int32_t*& b;
    double*& e;
    ~Free() {
      (void)hipFree(b);
      (void)hipFree(e);
    }
  } fr{d_b, d_e};
  if (dalloc(c, &d_b, (size_t)n) || dalloc(c, &d_e, (size_t)n)) return MANTIS_ERR_OOM;
  HIP_OK(hipMemcpyAsync(d_b, bins.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c->s));
  HIP_OK(hipMemcpyAsync(d_e, error, sizeof(double) * n, hipMemcpyHostToDevice, c->s));
  k_markov_weight<<<(n + 255) / 256, 256, 0, c->s>>>(c->d_markov + (size_t)filter * mk::kYawBins, d_b, n, d_e);
  HIP_OK(hipGetLastError());
  HIP_OK(hipMemcpyAsync(error, d_e, sizeof(double) * n, hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  return MANTIS_OK;
}

mantis_status mantis_markov_get(void* ctx, double* planes, double* yaw, int32_t* argmax) {
  Ctx* c = (Ctx*)ctx;
  if (c) bind_device(c);
  if (!c) return MANTIS_ERR_ARG;
  if (!c->markov_n) { c->err = "markov filters not initialised (mantis_markov_init)"; return MANTIS_ERR_STATE; }
  std::vector<double> h((size_t)c->markov_n * mk::kYawBins);
  HIP_OK(hipMemcpyAsync(h.data(), c->d_markov, sizeof(double) * h.size(), hipMemcpyDeviceToHost, c->s));
  HIP_OK(hipStreamSynchronize(c->s));
  if (planes) std::memcpy(planes, h.data(), sizeof(double) * h.size());
  for (int f = 0; f < c->markov_n; f++) {  // getYaw (Markov.cpp:265-275): first maximum, p[max] * pi / 180
    const double* p = &h[(size_t)f * mk::kYawBins];
    int max = 0;
    for (int i = 0; i < mk::kYawBins; ++i)
      if (p[i] > p[max]) max = i;
    if (yaw) yaw[f] = p[max] * M_PI / 180;
    if (argmax) argmax[f] = max;
  }
  return MANTIS_OK;
}

}  // extern "C"
