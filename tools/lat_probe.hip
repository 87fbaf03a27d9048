// Microbenchmark (not part of the product): dependent-chain latency, in shader
// cycles per link, of the FP64 operations on ObjPose's Jacobi rotation chain
// (one wave, one lane's value feeding the next link): FMA, rcp, rsq, the
// compiler's IEEE division and square root, their unscaled instruction
// sequences (what the library forms reduce to when no operand needs scaling),
// ocml hypot, and the VALU -> SALU -> VALU scale decision.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/lat_probe.hip -o tools/lat_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

__device__ inline double div_seq(double n, double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double q = n * r;
  const double rem = __builtin_fma(-d, q, n);
  return __builtin_fma(rem, r, q);
}
__device__ inline double sqrt_seq(double x) {
  double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  double e = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, e, g);
  h = __builtin_fma(h, e, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  return __builtin_fma(d, h, g);
}

template <int OP>
__global__ __launch_bounds__(64) void k(double* out, long long* cyc, double a, double b, int iters) {
  double x = 0.75 + threadIdx.x * 1e-6;
  const long long c0 = clock64();
#pragma unroll 1
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if (OP == 0) x = __builtin_fma(x, a, b);                       // |x| stays ~1
      else if (OP == 1) x = __builtin_amdgcn_rcp(x);
      else if (OP == 2) x = __builtin_amdgcn_rsq(x) * 0.75;           // +1 mul
      else if (OP == 3) x = a / x;
      else if (OP == 4) x = div_seq(a, x);
      else if (OP == 5) x = sqrt(x) + 0.5;                            // +1 add
      else if (OP == 6) x = sqrt_seq(x) + 0.5;
      else if (OP == 7) x = hypot(x, a) * 0.5;                        // +1 mul
      else if (OP == 8) x = x + x * 0.0;                              // add(mul): 2 links
      else if (OP == 9) x = (x > a ? x : b) + 0.25;                   // cmp+cndmask+add
    }
  }
  const long long c1 = clock64();
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
  out[threadIdx.x] = x;
}

// issue rate of one wave: 8 independent chains per lane
template <int OP>
__global__ __launch_bounds__(64) void kt(double* out, long long* cyc, double a, double b, int iters) {
  double x[8];
  int m[8];
#pragma unroll
  for (int k = 0; k < 8; k++) { x[k] = 0.75 + threadIdx.x * 1e-6 + k; m[k] = threadIdx.x + k; }
  const long long c0 = clock64();
#pragma unroll 1
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 4; u++)
#pragma unroll
      for (int k = 0; k < 8; k++) {
        if (OP == 0) x[k] = __builtin_fma(x[k], a, b);
        else if (OP == 1) x[k] = x[k] * a;
        else if (OP == 2) x[k] = (x[k] > b) ? x[k] : a;   // cmp + 2 cndmask
        else if (OP == 3) m[k] = m[k] * 0x9E37 + 7;          // 32-bit integer
        else if (OP == 4) x[k] = __builtin_amdgcn_rcp(x[k]);
      }
  }
  const long long c1 = clock64();
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
  double s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s += x[k] + m[k];
  out[threadIdx.x] = s;
}
template <int OP>
void runt(const char* name, double instr) {
  double* d;
  long long* c;
  (void)hipMalloc(&d, 64 * sizeof(double));
  (void)hipMalloc(&c, sizeof(long long));
  const int iters = 2048;
  kt<OP><<<1, 64>>>(d, c, 0.999, 0.0001, 16);
  kt<OP><<<1, 64>>>(d, c, 0.999, 0.0001, iters);
  long long h = 0;
  (void)hipMemcpy(&h, c, sizeof(h), hipMemcpyDeviceToHost);
  printf("%-34s %8.1f cycles per independent op (%.1f per instruction)\n", name, (double)h / (iters * 32.0),
         h / (iters * 32.0) / instr);
  (void)hipFree(d);
  (void)hipFree(c);
}

template <int OP>
void run(const char* name, double links) {
  double* d;
  long long* c;
  (void)hipMalloc(&d, 64 * sizeof(double));
  (void)hipMalloc(&c, sizeof(long long));
  const int iters = 4096;
  k<OP><<<1, 64>>>(d, c, 0.999, 0.0001, 16);
  k<OP><<<1, 64>>>(d, c, 0.999, 0.0001, iters);
  long long h = 0;
  (void)hipMemcpy(&h, c, sizeof(h), hipMemcpyDeviceToHost);
  printf("%-34s %8.1f cycles per link (%.1f per op, %g ops)\n", name, (double)h / (iters * 8.0), h / (iters * 8.0) / links, links);
  (void)hipFree(d);
  (void)hipFree(c);
}

int main() {
  run<0>("fma f64", 1);
  run<1>("rcp f64", 1);
  run<2>("rsq f64 + mul", 2);
  run<3>("a / x (compiler IEEE div)", 1);
  run<4>("div sequence, unscaled", 1);
  run<5>("sqrt(x) + 0.5 (compiler)", 1);
  run<6>("sqrt sequence, unscaled, + 0.5", 1);
  run<7>("hypot(x, a) * 0.5 (ocml)", 1);
  run<8>("x + x * 0", 2);
  run<9>("select + add", 1);
  runt<0>("issue: fma f64", 1);
  runt<1>("issue: mul f64", 1);
  runt<2>("issue: cmp f64 + 2 cndmask", 3);
  runt<3>("issue: u32 mul + add", 2);
  runt<4>("issue: rcp f64", 1);
  return 0;
}
