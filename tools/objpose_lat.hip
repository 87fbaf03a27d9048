// ObjPose latency probe (GPU box): the 16 longest first-ObjPose problems of
// the bench scene (tools/objpose_long.bin, written by tools/rpp_iter_hist.py)
// run one lane at a time through mk_rpp.h's op_setup/op_step; prints the
// iterations, shader cycles per iteration and whether R, t, errors match the
// host build of the same code (iterations exactly, poses to 1e-9); with
// OBJPOSE_LAT_OUT set it writes the device results (R, t, errors, iterations
// and timings) for bit-for-bit comparisons between builds. Variants of the Jacobi/AbsKernel
// code are compared by building with -D flags.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/objpose_lat.hip -o tools/objpose_lat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#ifdef STAMPS  // per-part cycles of AbsKernel (diagnostic build: -DSTAMPS)
__device__ long long g_stamp[4], g_part[4];
#ifdef __HIP_DEVICE_COMPILE__
#define MK_OP_STAMP(k)                                                   \
  do {                                                                   \
    __builtin_amdgcn_s_waitcnt(0);                                       \
    const long long now_ = __builtin_readcyclecounter();                 \
    if (k > 0) g_part[k] += now_ - g_stamp[k - 1];                       \
    g_stamp[k] = now_;                                                   \
  } while (0)
#else
#define MK_OP_STAMP(k)
#endif
#endif
#include "../mantis_amd/csrc/mk_rpp.h"

using namespace mk::rpp;
struct Res {
  double R[9], t[3], oe, ie;
  long long cyc, wall;
  int it, code;
};

__global__ __launch_bounds__(64) void k_lat(const double* pr, Res* out) {
  if (threadIdx.x != 0) return;
  const double* p = pr + 24 * blockIdx.x;
  M34 P, Q;
  for (int k = 0; k < 12; k++) { P.a[k] = p[k]; Q.a[k] = p[12 + k]; }
  OpState s;
  const long long c0 = clock64(), w0 = wall_clock64();
  op_setup(P, Q, nullptr, s);
  int code;
  while (!(code = op_step(s))) {}
  M33 R;
  M31 t;
  Res& o = out[blockIdx.x];
  op_finish(s, R, t, o.oe, o.ie);
  o.cyc = clock64() - c0;
  o.wall = wall_clock64() - w0;
  for (int k = 0; k < 9; k++) o.R[k] = R.a[k];
  for (int k = 0; k < 3; k++) o.t[k] = t.a[k];
  o.it = s.it;
  o.code = code;
}

int main() {
  FILE* f = fopen("tools/objpose_long.bin", "rb");
  if (!f) { printf("objpose_long.bin missing\n"); return 2; }
  std::vector<double> h(16 * 24);
  const size_t n = fread(h.data(), 24 * sizeof(double), 16, f) ;
  fclose(f);
  double* d;
  Res* r;
  if (hipMalloc(&d, h.size() * 8) || hipMalloc(&r, sizeof(Res) * n)) return 2;
  if (hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice)) return 2;
  std::vector<Res> g(n);
  long long tot_c = 0, tot_i = 0;
  int bad = 0;
  for (size_t b = 0; b < n; b++) {  // one problem per launch: pure single-lane latency
    k_lat<<<1, 64>>>(d + 24 * b, r + b);
  }
  if (hipDeviceSynchronize() || hipMemcpy(g.data(), r, sizeof(Res) * n, hipMemcpyDeviceToHost)) return 2;
  int wall_rate = 0;
  (void)hipDeviceGetAttribute(&wall_rate, hipDeviceAttributeWallClockRate, 0);
  for (size_t b = 0; b < n; b++) {
    M34 P, Q;
    for (int k = 0; k < 12; k++) { P.a[k] = h[24 * b + k]; Q.a[k] = h[24 * b + 12 + k]; }
    OpState s;
    op_setup(P, Q, nullptr, s);
    int code;
    while (!(code = op_step(s))) {}
    M33 R;
    M31 t;
    double oe, ie;
    op_finish(s, R, t, oe, ie);
    double dmax = fabs(oe - g[b].oe) + fabs(ie - g[b].ie);
    for (int k = 0; k < 9; k++) dmax = fmax(dmax, fabs(R.a[k] - g[b].R[k]));
    for (int k = 0; k < 3; k++) dmax = fmax(dmax, fabs(t.a[k] - g[b].t[k]));
    // device libm (hypot) may differ from the host's by an ulp: poses to 1e-9
    const bool same = s.it == g[b].it && code == g[b].code && dmax <= 1e-9;
    bad += !same;
    tot_c += g[b].cyc;
    tot_i += g[b].it;
    printf("problem %2zu: %5d iterations, %7.0f cycles/iteration, %6.2f us/iteration, host %s\n", b, g[b].it,
           (double)g[b].cyc / g[b].it, wall_rate ? 1e3 * g[b].wall / wall_rate / g[b].it : 0.0,
           same ? "agrees (1e-9)" : "DIFFERENT");
  }
  // device results for device-vs-device comparisons of variants
  if (const char* o = getenv("OBJPOSE_LAT_OUT")) {
    if (FILE* fo = fopen(o, "wb")) { fwrite(g.data(), sizeof(Res), n, fo); fclose(fo); }
  }
#ifdef STAMPS
  long long part[4];
  if (hipMemcpyFromSymbol(part, HIP_SYMBOL(g_part), sizeof(part)) == hipSuccess)
    printf("AbsKernel cycles per iteration: before SVD %.0f, SVD %.0f, after SVD %.0f\n", (double)part[1] / tot_i,
           (double)part[2] / tot_i, (double)part[3] / tot_i);
#endif
  printf("objpose_lat: %lld iterations, mean %.0f cycles/iteration, %d mismatches\n", tot_i, (double)tot_c / tot_i, bad);
  return bad ? 1 : 0;
}
