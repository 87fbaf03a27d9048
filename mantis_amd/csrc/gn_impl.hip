// Gauss–Newton rig refinement (new stage) and the RCCL
// exchange of its accumulators for camera-sharded rigs (§8 e). Included by
// api.hip (shares its Ctx).
//
// Residuals: r = pi(p) - u with p = inv(T_b_c) inv(T_w_b) X the world point
// X in camera c, u the observed normalized (undistorted) image point and
// pi(p) = (p_x/p_z, p_y/p_z). Right perturbation T_w_b <- T_w_b Exp(delta),
// delta = (rho, phi): dp/d(delta) = R_cb [ -I | [q]x ], q = inv(T_w_b) X.
// The 28 accumulated doubles are the upper triangle of J^T J (21), J^T r (6)
// and r^T r (1): with M = [J | r] (rows = residual components) all of them
// are entries of M^T M, which one wave builds with v_mfma_f64_16x16x4_f64,
// 4 residual rows per instruction.
#include <rccl/rccl.h>

namespace mk {

typedef double v4d __attribute__((ext_vector_type(4)));

struct GnCam {
  double R_cb[9];  // inv(T_b_c) rotation
  double t_cb[3];
};

// value of M[row][col] (col 0..5 = J, 6 = r, else 0) for one residual row
__device__ inline double gn_entry(const double* Rwb_t, const double* twb, const GnCam* cams, const double* obs,
                                  int n_obs, int row, int col) {
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

}  // namespace mk

namespace {
void rodrigues(const double* w, double* R) {
  double th = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
  double K[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
  double a, b;
  if (th < 1e-12) { a = 1.0; b = 0.5; }
  else { a = std::sin(th) / th; b = (1 - std::cos(th)) / (th * th); }
  double K2[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += K[i * 3 + k] * K[k * 3 + j];
      K2[i * 3 + j] = s;
    }
  for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + a * K[i] + b * K2[i];
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
  double A[6][6], b[6];
  int n = 0;
  for (int i = 0; i < 6; i++)
    for (int j = i; j < 6; j++) { A[i][j] = A[j][i] = acc28[n++]; }
  for (int i = 0; i < 6; i++) { A[i][i] += lambda; b[i] = -acc28[21 + i]; }
  // Cholesky A = L L^T
  double L[6][6] = {{0}};
  for (int i = 0; i < 6; i++)
    for (int j = 0; j <= i; j++) {
      double s = A[i][j];
      for (int k = 0; k < j; k++) s -= L[i][k] * L[j][k];
      if (i == j) {
        if (!(s > 0)) return MANTIS_ERR_ARG;  // not positive definite (too few observations)
        L[i][i] = std::sqrt(s);
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
  double dR[9];
  rodrigues(x + 3, dR);
  double D[16] = {dR[0], dR[1], dR[2], x[0], dR[3], dR[4], dR[5], x[1], dR[6], dR[7], dR[8], x[2], 0, 0, 0, 1};
  mat4_mul(T_w_b, D, T_w_b);
  return MANTIS_OK;
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
  ncclResult_t r = ncclCommInitRank(&comm, nranks, id, rank);
  if (r != ncclSuccess) { c->err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r); return MANTIS_ERR_COMM; }
  c->comm = comm;
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
