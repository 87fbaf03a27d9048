// Microbenchmark (not part of the product): VALU throughput of FP64 / FP32
// FMA and FP64 reciprocal on this GPU, wave64, 8 independent chains per lane.
// Build: hipcc -O3 --offload-arch=gfx950 tools/fp64_rate.hip -o tools/fp64_rate
#include <hip/hip_runtime.h>
#include <cstdio>
template <class T, int OP>
__global__ __launch_bounds__(256) void kr(T* out, T a, T b, int iters) {
  T x[8];
#pragma unroll
  for (int k = 0; k < 8; k++) x[k] = (T)(threadIdx.x + k) * (T)1e-3;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (OP == 0) x[k] = __builtin_fma(x[k], a, b);
      else if (OP == 1) x[k] = x[k] * a;
      else x[k] = __builtin_amdgcn_rcp(x[k]) ;
    }
  }
  T s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s += x[k];
  if (s == (T)12345) out[threadIdx.x] = s;
}
template <class T, int OP>
void run(const char* name) {
  T* d;
  (void)hipMalloc(&d, 1024 * sizeof(T));
  const int blocks = 256 * 32, iters = 2048;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  kr<T, OP><<<blocks, 256>>>(d, (T)0.999, (T)1e-4, 16);
  (void)hipEventRecord(e0);
  kr<T, OP><<<blocks, 256>>>(d, (T)0.999, (T)1e-4, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  const double winst = (double)blocks * 4 * iters * 8;  // wave-instructions
  const double per_simd = winst / 1024.0;
  printf("%-10s %8.3f ms  %.3g wave-instr/SIMD  -> %.2f ns per wave-instr per SIMD (%.2f cyc @2.4GHz)  lane-ops %.1f T/s\n", name, ms,
         per_simd, ms * 1e6 / per_simd, ms * 1e6 / per_simd * 2.4, winst * 64 / (ms * 1e-3) / 1e12);
  (void)hipFree(d);
}
int main() {
  run<double, 0>("fma_f64");
  run<double, 1>("mul_f64");
  run<float, 0>("fma_f32");
  run<double, 2>("rcp_f64");
  run<float, 2>("rcp_f32");
  return 0;
}
