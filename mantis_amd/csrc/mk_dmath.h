// Device replicas of the ROCm device-libm (ocml) double routines used on the
// scoring path, operation for operation, so results are bit-identical to
// ::atan / ::sin / ::cos on the device (tools/check_dmath.hip checks this on
// the GPU) while costing fewer VALU slots and registers:
//   * atan: the 19 polynomial coefficients are materialised in SGPRs with
//     scalar moves, so each Horner step is one v_fma_f64 (the library form
//     spends two v_mov_b32 per coefficient on literals);
//   * sin/cos: the small-argument reduction only (|x| < 2^30); the library's
//     large-argument Payne-Hanek path is what set the particle kernel's VGPR
//     count. Callers guarantee the bound (particle angles are float gaussians
//     x 0.03, |x| < 2 rad).
// Host builds (the CPU restatement in hostcheck.cpp) keep glibc.
#pragma once
#include <cmath>
#include <cstdint>

namespace mk {
namespace dm {

#if defined(__HIPCC__) && defined(__HIP_DEVICE_COMPILE__)
#define MK_DM_DEVICE 1
// 64-bit constant built from two scalar moves (SGPR pair): the compiler cannot
// turn it back into VGPR literal moves.
template <unsigned long long B>
__device__ inline double sk() {
#ifdef MK_DM_LITERAL_CONSTANTS  // A/B builds: let the compiler place the constants
  return __longlong_as_double((long long)B);
#endif
  unsigned lo, hi;
  asm("s_mov_b32 %0, %1" : "=s"(lo) : "i"((unsigned)(B & 0xffffffffu)));
  asm("s_mov_b32 %0, %1" : "=s"(hi) : "i"((unsigned)(B >> 32)));
  return __hiloint2double((int)hi, (int)lo);
}
__device__ inline double kd(unsigned long long b) { return __longlong_as_double((long long)b); }

// __ocmlpriv_atanred_f64 + __ocml_atan_f64 for x = +0, positive or NaN with
// inv = 1.0 / x already computed (the fisheye projection divides by r anyway:
// sharing the one IEEE division is exact, fabs(x) == x and copysign is a no-op)
__device__ inline double atan_pos(double x, double inv) {
  const double ax = x;
  const bool big = ax > 1.0;
  const double a = big ? inv : ax;
  const double s = a * a;
  double p = __builtin_fma(s, sk<0x3EEBA404B5E68A13ull>(), sk<0xBF23E260BD3237F4ull>());
  p = __builtin_fma(s, p, sk<0x3F4B2BB069EFB384ull>());
  p = __builtin_fma(s, p, sk<0xBF67952DAF56DE9Bull>());
  p = __builtin_fma(s, p, sk<0x3F7D6D43A595C56Full>());
  p = __builtin_fma(s, p, sk<0xBF8C6EA4A57D9582ull>());
  p = __builtin_fma(s, p, sk<0x3F967E295F08B19Full>());
  p = __builtin_fma(s, p, sk<0xBF9E9AE6FC27006Aull>());
  p = __builtin_fma(s, p, sk<0x3FA2C15B5711927Aull>());
  p = __builtin_fma(s, p, sk<0xBFA59976E82D3FF0ull>());
  p = __builtin_fma(s, p, sk<0x3FA82D5D6EF28734ull>());
  p = __builtin_fma(s, p, sk<0xBFAAE5CE6A214619ull>());
  p = __builtin_fma(s, p, sk<0x3FAE1BB48427B883ull>());
  p = __builtin_fma(s, p, sk<0xBFB110E48B207F05ull>());
  p = __builtin_fma(s, p, sk<0x3FB3B13657B87036ull>());
  p = __builtin_fma(s, p, sk<0xBFB745D119378E4Full>());
  p = __builtin_fma(s, p, sk<0x3FBC71C717E1913Cull>());
  p = __builtin_fma(s, p, sk<0xBFC2492492376B7Dull>());
  p = __builtin_fma(s, p, sk<0x3FC99999999952CCull>());
  p = __builtin_fma(s, p, sk<0xBFD5555555555523ull>());
  const double q = s * p;
  const double red = __builtin_fma(a, q, a);
  return big ? __builtin_fma(kd(0x3FEDD9AD336A0500ull), kd(0x3FFAF154EEB562D6ull), -red) : red;
}

// __ocmlpriv_atanred_f64 + __ocml_atan_f64
__device__ inline double atan(double x) {
  const double ax = __builtin_fabs(x);
  const bool big = ax > 1.0;
  const double inv = 1.0 / ax;
  const double a = big ? inv : ax;
  const double s = a * a;
  double p = __builtin_fma(s, sk<0x3EEBA404B5E68A13ull>(), sk<0xBF23E260BD3237F4ull>());
  p = __builtin_fma(s, p, sk<0x3F4B2BB069EFB384ull>());
  p = __builtin_fma(s, p, sk<0xBF67952DAF56DE9Bull>());
  p = __builtin_fma(s, p, sk<0x3F7D6D43A595C56Full>());
  p = __builtin_fma(s, p, sk<0xBF8C6EA4A57D9582ull>());
  p = __builtin_fma(s, p, sk<0x3F967E295F08B19Full>());
  p = __builtin_fma(s, p, sk<0xBF9E9AE6FC27006Aull>());
  p = __builtin_fma(s, p, sk<0x3FA2C15B5711927Aull>());
  p = __builtin_fma(s, p, sk<0xBFA59976E82D3FF0ull>());
  p = __builtin_fma(s, p, sk<0x3FA82D5D6EF28734ull>());
  p = __builtin_fma(s, p, sk<0xBFAAE5CE6A214619ull>());
  p = __builtin_fma(s, p, sk<0x3FAE1BB48427B883ull>());
  p = __builtin_fma(s, p, sk<0xBFB110E48B207F05ull>());
  p = __builtin_fma(s, p, sk<0x3FB3B13657B87036ull>());
  p = __builtin_fma(s, p, sk<0xBFB745D119378E4Full>());
  p = __builtin_fma(s, p, sk<0x3FBC71C717E1913Cull>());
  p = __builtin_fma(s, p, sk<0xBFC2492492376B7Dull>());
  p = __builtin_fma(s, p, sk<0x3FC99999999952CCull>());
  p = __builtin_fma(s, p, sk<0xBFD5555555555523ull>());
  const double q = s * p;
  const double red = __builtin_fma(a, q, a);
  const double r = big ? __builtin_fma(kd(0x3FEDD9AD336A0500ull), kd(0x3FFAF154EEB562D6ull), -red) : red;
  return __builtin_copysign(r, x);
}

// __ocmlpriv_trigredsmall_f64 (|x| < 2^30) + __ocmlpriv_sincosred2_f64, then
// the quadrant/sign selection of __ocml_sin_f64 / __ocml_cos_f64
__device__ inline void sincos_small(double x, double* s_out, double* c_out) {
  const double ax = __builtin_fabs(x);
  const double qd = __builtin_rint(ax * kd(0x3FE45F306DC9C883ull));
  const double a4 = __builtin_fma(qd, kd(0xBFF921FB54442D18ull), ax);
  const double a5 = __builtin_fma(qd, kd(0xBC91A62633145C00ull), a4);
  const double a6 = qd * kd(0x3C91A62633145C00ull);
  const double a8 = __builtin_fma(qd, kd(0x3C91A62633145C00ull), -a6);
  const double a9 = a4 - a6;
  const double a10 = a4 - a9;
  const double a11 = a10 - a6;
  const double a12 = a9 - a5;
  const double a13 = a12 + a11;
  const double a14 = a13 - a8;
  const double a15 = __builtin_fma(qd, kd(0xB97B839A252049C0ull), a14);
  const double rh = a5 + a15;
  const double a17 = rh - a5;
  const double rt = a15 - a17;
  const int q = (int)qd & 3;
  // sincosred2(rh, rt)
  const double x2 = rh * rh;
  const double h = x2 * 0.5;
  const double c1 = 1.0 - h;
  const double c2 = 1.0 - c1;
  const double c3 = c2 - h;
  const double x4 = x2 * x2;
  double pc = __builtin_fma(x2, kd(0xBDA907DB46CC5E42ull), kd(0x3E21EEB69037AB78ull));
  pc = __builtin_fma(x2, pc, kd(0xBE927E4FA17F65F6ull));
  pc = __builtin_fma(x2, pc, kd(0x3EFA01A019F4EC90ull));
  pc = __builtin_fma(x2, pc, kd(0xBF56C16C16C16967ull));
  pc = __builtin_fma(x2, pc, kd(0x3FA5555555555555ull));
  const double m = __builtin_fma(rh, -rt, c3);
  const double n = __builtin_fma(x4, pc, m);
  const double cv = c1 + n;
  double ps = __builtin_fma(x2, kd(0x3DE5E0B2F9A43BB8ull), kd(0xBE5AE600B42FDFA7ull));
  ps = __builtin_fma(x2, ps, kd(0x3EC71DE3796CDE01ull));
  ps = __builtin_fma(x2, ps, kd(0xBF2A01A019E83E5Cull));
  ps = __builtin_fma(x2, ps, kd(0x3F81111111110BB3ull));
  const double nx = rh * -x2;
  const double hy = rt * 0.5;
  const double u = __builtin_fma(nx, ps, hy);
  const double v = __builtin_fma(x2, u, -rt);
  const double w = __builtin_fma(nx, kd(0xBFC5555555555555ull), v);
  const double sv = rh - w;
  const unsigned flip = q > 1 ? 0x80000000u : 0u;
  // sin: odd, sign of x
  {
    const double sel = (q & 1) == 0 ? sv : cv;
    const unsigned long long b = (unsigned long long)__double_as_longlong(sel);
    const unsigned xs = (unsigned)((unsigned long long)__double_as_longlong(x) >> 32) & 0x80000000u;
    const unsigned hi = (unsigned)(b >> 32) ^ (flip ^ xs);
    *s_out = __longlong_as_double((long long)(((unsigned long long)hi << 32) | (b & 0xffffffffull)));
  }
  // cos: even
  {
    const double sel = (q & 1) == 0 ? cv : -sv;
    const unsigned long long b = (unsigned long long)__double_as_longlong(sel);
    const unsigned hi = (unsigned)(b >> 32) ^ flip;
    *c_out = __longlong_as_double((long long)(((unsigned long long)hi << 32) | (b & 0xffffffffull)));
  }
}
#else
#define MK_DM_DEVICE 0
#ifdef __HIPCC__
// host pass of a HIP translation unit: declarations only (never executed)
__host__ __device__ inline double atan(double x) { return ::atan(x); }
__host__ __device__ inline double atan_pos(double x, double) { return ::atan(x); }
__host__ __device__ inline void sincos_small(double x, double* s, double* c) {
  *s = ::sin(x);
  *c = ::cos(x);
}
#endif
#endif

}  // namespace dm
}  // namespace mk
