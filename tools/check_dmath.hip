// GPU check (not part of the product): mk_dmath.h replicas against the
// device libm they restate, bit for bit, over 2^24 inputs per function.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/check_dmath.hip -o tools/check_dmath
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../mantis_amd/csrc/mk_dmath.h"

__device__ inline uint64_t mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// inputs: uniform in [-range, range] with range = 2^(k-20), k = i % 32, plus raw bit patterns of small doubles
__device__ inline double input(uint64_t i) {
  const uint64_t r = mix(i);
  const int k = (int)(i % 32);
  const double u = (double)(r >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
  return u * ldexp(1.0, k - 20);
}
__global__ void kcheck(uint64_t n, unsigned long long* bad) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const double x = input(i);
    if (__double_as_longlong(mk::dm::atan(x)) != __double_as_longlong(::atan(x))) atomicAdd(&bad[0], 1ull);
    {  // the projection's form: x >= 0 with the shared reciprocal
      const double ax = __builtin_fabs(x);
      if (__double_as_longlong(mk::dm::atan_pos(ax, 1.0 / ax)) != __double_as_longlong(::atan(ax)))
        atomicAdd(&bad[0], 1ull);
    }
    if (__builtin_fabs(x) < 1073741824.0) {
      double s, c;
      mk::dm::sincos_small(x, &s, &c);
      if (__double_as_longlong(s) != __double_as_longlong(::sin(x))) atomicAdd(&bad[1], 1ull);
      if (__double_as_longlong(c) != __double_as_longlong(::cos(x))) atomicAdd(&bad[2], 1ull);
    }
  }
}
int main() {
  unsigned long long* d;
  unsigned long long h[3] = {0, 0, 0};
  if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 2;
  (void)hipMemset(d, 0, sizeof(h));
  const uint64_t n = 1ull << 24;
  kcheck<<<2048, 256>>>(n, d);
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  printf("check_dmath: %llu inputs, mismatches atan %llu sin %llu cos %llu\n", (unsigned long long)n, h[0], h[1], h[2]);
  return (h[0] | h[1] | h[2]) ? 1 : 0;
}
