// HIP kernels (gfx950) of the mantis3 per-frame hot path. Host side: api.hip.
//
// Stage map (reference -> kernel):
//   cvtColor+GaussianBlur+Canny NMS  QuadDetection.h:209-212        k_canny (candidate / strong bit planes)
//   Canny hysteresis                 (OpenCV, [3P])                  k_hyst_band / _seam / _mark / _fix (run CCL)
//   dilate x2 / erode x1             QuadDetection.h:213-214         k_morph (bit planes, LDS bands)
//   cleanImageByEdge mask            HypothesisEvaluation.h:319-386  k_morph (same pass)
//   findContours(CCOMP, SIMPLE)      QuadDetection.h:216             k_run_count/_scan/_emit/_band/_seam/_border
//                                                                    (run CCL) + k_tile_bits + k_trace_borders
//                                                                    (+ _lds) + k_frame_contours
//   approxPolyDP / Quadrilateral /
//   removeDuplicateQuads / undistort QuadDetection.h:13-171, 219-228, 289-298   k_frame_contours
//   CoPlanarPoseEstimator -> RPP     CoPlanarPoseEstimator.cpp:16-58 k_rpp_prep, k_objpose_q<0>, k_rpp_s1b,
//                                                                    k_objpose_q<1>, k_rpp_merge (+ per-quad GN)
//   generateCentralHypotheses +
//   PoseClusterer                    HypothesisGeneration.h:57-109, PoseClusterer.cpp:33-116  k_frame_hyps
//   evaluate / PF / shifts / yaw /
//   publish gate                     src/mantis3.cpp:102-132          k_score_init / k_score_pf / k_score_final
//   legacy camera weighting          legacy/mantis/MonteCarlo.cpp:183-241  k_rig_weight
//   stage entries, dense grid        HypothesisEvaluation.h:31-41    k_score_api, k_argmin, k_quad_gn
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "mk_bits.h"
#include "mk_contour.h"
#include "mk_gn.h"
#include "mk_math.h"
#include "mk_rpp.h"
#include "mk_shard.h"
#include "mk_sort.h"
#include "mk_types.h"
#include "synth.h"

namespace mk {

// Wave scans on DPP (no LDS crossbar trips): Hillis-Steele inside each
// 16-lane row (row_shr 1, 2, 4, 8; lanes past the row's start read 0), then
// the rows' totals carried by row_bcast:15 (row r-1's last lane into rows 1
// and 3) and row_bcast:31 (lane 31 into rows 2 and 3). Every active lane must
// call them (inactive lanes read as 0 only inside the row steps).
#ifndef MK_DPP_SCAN
#define MK_DPP_SCAN 1
#endif
__device__ inline int wave_incl_scan(int v, int lane) {
#if MK_DPP_SCAN
  (void)lane;
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
#else
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o);
    if (lane >= o) v += u;
  }
#endif
  return v;
}
__device__ inline int wave_sum(int v) {
#if MK_DPP_SCAN
  return __builtin_amdgcn_readlane(wave_incl_scan(v, 0), 63);
#else
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
#endif
}

// Frame pointers come out of FrameDesc records in memory, so the compiler
// cannot tell they are global and emits flat loads (which also count against
// lgkmcnt, so every LDS wait waits for them too). Frames always live in
// device memory: these views make the loads global_load_*.
typedef __attribute__((address_space(1))) const uint8_t gu8;
typedef __attribute__((address_space(1))) const uint32_t gu32;
__device__ inline gu8* gbytes(const uint8_t* p) { return (gu8*)p; }
__device__ inline gu32* gwords(const void* p) { return (gu32*)p; }

// ======================================================== union-find (CCL)
// Concurrent union by index: roots are component minima, links point to
// smaller indices only, so finds terminate and stale reads only cost retries.
// Finds use path halving: only non-roots are rewritten (with an ancestor) and
// roots change only through the CAS in uf_union_c, so this is race-safe.
__device__ inline int uf_find_c(int32_t* lab, int x) {
  while (true) {
    int p = lab[x];
    if (p == x) return x;
    int g = lab[p];
    if (g == p) return p;
    lab[x] = g;
    x = g;
  }
}
__device__ inline void uf_union_c(int32_t* lab, int a, int b) {
  while (true) {
    a = uf_find_c(lab, a);
    b = uf_find_c(lab, b);
    if (a == b) return;
    if (a < b) { int t = a; a = b; b = t; }
    int old = atomicCAS(&lab[a], a, b);
    if (old == a) return;
    a = old;
  }
}
__device__ inline int lds_find(const int* L, int x) {
  int p;
  while ((p = L[x]) != x) x = p;
  return x;
}
__device__ inline void lds_union(int* L, int a, int b) {
  while (true) {
    a = lds_find(L, a);
    b = lds_find(L, b);
    if (a == b) return;
    if (a < b) { int t = a; a = b; b = t; }
    int old = atomicCAS(&L[a], a, b);
    if (old == a) return;
    a = old;
  }
}

// ============================================== Canny: classes + hysteresis
// cvtColor(BGR2GRAY) -> GaussianBlur 3x3 (x256 kernel [84,89,84], OpenCV <= 3.3,
// BORDER_REFLECT_101) -> Sobel 3x3 (REPLICATE) -> L1 magnitude -> NMS
// (QuadDetection.h:209-212, HypothesisEvaluation.h:323-327; one Canny serves
// both) and cv::Canny's hysteresis stack walk, i.e. the 8-connected components
// of the NMS candidates that hold a strong pixel. Nothing per-pixel reaches HBM
// but bit planes:
//   k_canny_strip / k_canny   column strips walked by one wave (DPP taps) /
//                128x16 tiles (LDS): BGR -> classes -> candidate and strong bit
//                planes
//   k_hyst_band  per 32-row band: the two planes' words into LDS, candidate
//                runs per row numbered inside the band, 8-connected run
//                unions in LDS; the edge words of every band component with a
//                strong pixel; lists of the components that reach a band seam
//   k_hyst_seam  the same unions across band seams (global labels)
//   k_hyst_mark  strong components at a seam mark their global root
//   k_hyst_fix   weak components at a seam whose global root is marked: edges
#ifndef MK_FTH
#define MK_FTH 16
#endif
constexpr int FTW = 128, FTH = MK_FTH;         // front-end tile
constexpr int FGW = FTW + 8, FGH = FTH + 6;    // gray tile: x0-4 .. x0+FTW+3 (4-aligned), y0-3 .. y0+FTH+2
constexpr int FRW = FTW + 4;                   // blurred columns x0-2 .. x0+FTW+1
constexpr int FMW = FTW + 2, FMH = FTH + 2;    // magnitude: x0-1 .. x0+FTW, y0-1 .. y0+FTH

__device__ inline int refl101(int i, int n) {  // BORDER_REFLECT_101
  if (n == 1) return 0;
  if (i < 0) return -i;
  if (i >= n) return 2 * n - 2 - i;
  return i;
}

template <class P>
__device__ inline uint8_t gray_px(P p) {
  return (uint8_t)((1868 * p[0] + 9617 * p[1] + 4899 * p[2] + 8192) >> 14);
}
// gray_px of the 4 pixels in three dwords (b0 g0 r0 b1 | g1 r1 b2 g2 | r2 b3 g3 r3)
// with byte dot products: each coefficient = 256 hi + lo, both bytes, so
// dot4(px, lo) + 256 dot4(px, hi) + 8192 is the same integer as gray_px's sum.
__device__ inline uint32_t gray4(uint32_t d0, uint32_t d1, uint32_t d2) {
  constexpr uint32_t LO = 0x0023914Cu, HI = 0x00132507u;  // (76, 145, 35), (7, 37, 19)
  const uint32_t p1 = __builtin_amdgcn_perm(d1, d0, 0x0c050403u), p2 = __builtin_amdgcn_perm(d2, d1, 0x0c040302u);
  const auto g = [](uint32_t p, uint32_t lo, uint32_t hi) {
    return __builtin_amdgcn_udot4(p, lo, (__builtin_amdgcn_udot4(p, hi, 0u, false) << 8) + 8192u, false) >> 14;
  };
  return g(d0, LO, HI) | (g(p1, LO, HI) << 8) | (g(p2, LO, HI) << 16) | (g(d2, LO << 8, HI << 8) << 24);
}

// gray4 as two u16 pairs (pixels 0, 1 and 2, 3): each dot sum is gray << 14
// plus a fraction under 2^14 and below 2^22, so (s << 2) holds gray in bits
// 16..23 (k_canny_strip's horizontal blur takes u16 pairs: no byte packing)
__device__ inline void gray4_pairs(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t& p01, uint32_t& p23) {
  constexpr uint32_t LO = 0x0023914Cu, HI = 0x00132507u;
  const uint32_t p1 = __builtin_amdgcn_perm(d1, d0, 0x0c050403u), p2 = __builtin_amdgcn_perm(d2, d1, 0x0c040302u);
  const auto s = [](uint32_t p, uint32_t lo, uint32_t hi) {
    return __builtin_amdgcn_udot4(p, lo, (__builtin_amdgcn_udot4(p, hi, 0u, false) << 8) + 8192u, false);
  };
  p01 = (s(d0, LO, HI) >> 14) | ((s(p1, LO, HI) << 2) & 0xffff0000u);
  p23 = (s(p2, LO, HI) >> 14) | ((s(d2, LO << 8, HI << 8) << 2) & 0xffff0000u);
}

// Interior tiles, four horizontally adjacent pixels per work-item: every
// stencil stage reads aligned dwords / qwords of LDS rows and writes one, so
// the per-pixel byte gathers and index arithmetic of the generic path go. All
// interior buffers share the gray tile's columns (x0-4 .. x0+FTW+3, FGW = 136
// = 34 groups of 4); columns outside a stage's valid range hold values that
// no later stage reads. Integer arithmetic as the generic path (the
// [84,89,84] sums are exact, so 84(a+c) + 89b is the same number).
constexpr int FG4 = FGW / 4;  // 4-pixel groups per interior row
static_assert(FGW % 4 == 0 && FGH * FGW * 2 <= 2 * FTW * FTH * 2, "interior blur rows fit the gradient buffer");
// Packed 16-bit pairs (VOP3P v_pk_* arithmetic, two pixels per instruction):
// for the 4-pixel group with bytes b1..b4 in wc, b0 = top byte of wp and b5 =
// low byte of wn, the 3-tap operands of pixels (0,1) and (2,3) as u16 pairs
// (l = left, m = centre, q = right; l23 = q01), built with v_perm_b32.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
struct Taps4 {
  uint32_t l01, m01, q01, m23, q23;
};
__device__ inline Taps4 taps4(uint32_t wp, uint32_t wc, uint32_t wn) {
  return {__builtin_amdgcn_perm(wc, wp, 0x0c040c03u), __builtin_amdgcn_perm(wc, wc, 0x0c010c00u),
          __builtin_amdgcn_perm(wc, wc, 0x0c020c01u), __builtin_amdgcn_perm(wc, wc, 0x0c030c02u),
          __builtin_amdgcn_perm(wn, wc, 0x0c040c03u)};
}
template <class V>
__device__ inline V vpk(uint32_t v) { return __builtin_bit_cast(V, v); }
template <class V>
__device__ inline uint32_t upk(V v) { return __builtin_bit_cast(uint32_t, v); }
// horizontal blur of gray rows 0 .. FGH-1 into hb (u16, FGH x FGW):
// 84 (l + q) + 89 m <= 257 * 255 fits u16 exactly
__device__ inline void hblur4(const uint8_t* g, uint16_t* hb, int t) {
  for (int u = t; u < FGH * FG4; u += 256) {
    const int ly = u / FG4, k = u - ly * FG4;
    const uint32_t* row = (const uint32_t*)(g + ly * FGW);
    const uint32_t wc = row[k], wp = row[k > 0 ? k - 1 : 0], wn = row[k + 1 < FG4 ? k + 1 : k];
    const Taps4 tp = taps4(wp, wc, wn);
    const u16x2 c84 = {84, 84}, c89 = {89, 89};
    const u16x2 o01 = (vpk<u16x2>(tp.l01) + vpk<u16x2>(tp.q01)) * c84 + vpk<u16x2>(tp.m01) * c89;
    const u16x2 o23 = (vpk<u16x2>(tp.q01) + vpk<u16x2>(tp.q23)) * c84 + vpk<u16x2>(tp.m23) * c89;
    *(uint2*)(hb + ly * FGW + 4 * k) = make_uint2(upk(o01), upk(o23));
  }
}
// vertical blur: bl rows 0 .. FTH+3 (image rows y0-2 ..) from hb rows ly .. ly+2
__device__ inline void vblur4(const uint16_t* hb, uint8_t* bl, int t) {
  constexpr int BLH = FTH + 4;
  for (int u = t; u < BLH * FG4; u += 256) {
    const int ly = u / FG4, k = u - ly * FG4;
    const uint2 a = *(const uint2*)(hb + ly * FGW + 4 * k);
    const uint2 b = *(const uint2*)(hb + (ly + 1) * FGW + 4 * k);
    const uint2 c = *(const uint2*)(hb + (ly + 2) * FGW + 4 * k);
    const uint32_t av[4] = {a.x & 0xffffu, a.x >> 16, a.y & 0xffffu, a.y >> 16};
    const uint32_t bv[4] = {b.x & 0xffffu, b.x >> 16, b.y & 0xffffu, b.y >> 16};
    const uint32_t cv[4] = {c.x & 0xffffu, c.x >> 16, c.y & 0xffffu, c.y >> 16};
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t r = (84u * (av[j] + cv[j]) + 89u * bv[j] + (1u << 15)) >> 16;
      w |= (r > 255u ? 255u : r) << (8 * j);
    }
    *(uint32_t*)(bl + ly * FGW + 4 * k) = w;
  }
}
// Sobel + L1 magnitude on rows 0 .. FTH+1 (image rows y0-1 ..), all columns;
// gx / gy kept for the tile's own pixels (rows 1 .. FTH, columns 4 .. FTW+3).
// Packed i16 pairs: |gx|, |gy| <= 1020, so every sum is exact in 16 bits.
__device__ inline void sobel4(const uint8_t* bl, int16_t* mag, int16_t* gx_s, int16_t* gy_s, int t) {
  for (int u = t; u < (FTH + 2) * FG4; u += 256) {
    const int ly = u / FG4, k = u - ly * FG4;
    s16x2 sm[3][2], df[3][2];
#pragma unroll
    for (int r = 0; r < 3; r++) {
      const uint32_t* row = (const uint32_t*)(bl + (ly + r) * FGW);
      const uint32_t wc = row[k], wp = row[k > 0 ? k - 1 : 0], wn = row[k + 1 < FG4 ? k + 1 : k];
      const Taps4 tp = taps4(wp, wc, wn);
      const s16x2 l01 = vpk<s16x2>(tp.l01), m01 = vpk<s16x2>(tp.m01), q01 = vpk<s16x2>(tp.q01);
      const s16x2 m23 = vpk<s16x2>(tp.m23), q23 = vpk<s16x2>(tp.q23);
      sm[r][0] = l01 + (m01 << 1) + q01;  // l + 2m + q
      sm[r][1] = q01 + (m23 << 1) + q23;
      df[r][0] = q01 - l01;               // q - l
      df[r][1] = q23 - q01;
    }
    s16x2 m[2], gx[2], gy[2];
#pragma unroll
    for (int p = 0; p < 2; p++) {
      gx[p] = df[0][p] + (df[1][p] << 1) + df[2][p];
      gy[p] = sm[2][p] - sm[0][p];
      m[p] = __builtin_elementwise_max(gx[p], -gx[p]) + __builtin_elementwise_max(gy[p], -gy[p]);
    }
    *(uint2*)(mag + ly * FGW + 4 * k) = make_uint2(upk(m[0]), upk(m[1]));
    if (ly >= 1 && ly <= FTH && k >= 1 && k <= FTW / 4) {
      const int jj = (ly - 1) * FTW + 4 * (k - 1);
      *(uint2*)(gx_s + jj) = make_uint2(upk(gx[0]), upk(gx[1]));
      *(uint2*)(gy_s + jj) = make_uint2(upk(gy[0]), upk(gy[1]));
    }
  }
}

// Sobel separated, vertical pass first (MK_CANNY_V): per column the
// smoothed sum vs = a + 2b + c and the difference vd = c - a of the three
// blurred rows, then gx = vs(x+1) - vs(x-1) and gy = vd(x-1) + 2 vd(x) +
// vd(x+1) -- the same integers as the 3x3 sums of sobel4, on u16 / i16 pairs
// of columns (-1, 0), (1, 2), (3, 4) of the group, with (0, 1) and (2, 3)
// taken from them by one v_perm each.
__device__ inline void sobel4v(const uint8_t* bl, int16_t* mag, int16_t* gx_s, int16_t* gy_s, int t) {
  for (int u = t; u < (FTH + 2) * FG4; u += 256) {
    const int ly = u / FG4, k = u - ly * FG4;
    u16x2 vs[3];
    s16x2 vd[3];
    u16x2 a[3], c[3];
#pragma unroll
    for (int r = 0; r < 3; r += 2) {
      const uint32_t* row = (const uint32_t*)(bl + (ly + r) * FGW);
      const uint32_t wc = row[k], wp = row[k > 0 ? k - 1 : 0], wn = row[k + 1 < FG4 ? k + 1 : k];
      u16x2* o = r == 0 ? a : c;
      o[0] = vpk<u16x2>(__builtin_amdgcn_perm(wc, wp, 0x0c040c03u));  // columns -1, 0
      o[1] = vpk<u16x2>(__builtin_amdgcn_perm(wc, wc, 0x0c020c01u));  // 1, 2
      o[2] = vpk<u16x2>(__builtin_amdgcn_perm(wn, wc, 0x0c040c03u));  // 3, 4
    }
    {
      const uint32_t* row = (const uint32_t*)(bl + (ly + 1) * FGW);
      const uint32_t wc = row[k], wp = row[k > 0 ? k - 1 : 0], wn = row[k + 1 < FG4 ? k + 1 : k];
      const u16x2 b0 = vpk<u16x2>(__builtin_amdgcn_perm(wc, wp, 0x0c040c03u));
      const u16x2 b1 = vpk<u16x2>(__builtin_amdgcn_perm(wc, wc, 0x0c020c01u));
      const u16x2 b2 = vpk<u16x2>(__builtin_amdgcn_perm(wn, wc, 0x0c040c03u));
      const u16x2 two = {2, 2};
      vs[0] = a[0] + c[0] + b0 * two;
      vs[1] = a[1] + c[1] + b1 * two;
      vs[2] = a[2] + c[2] + b2 * two;
    }
#pragma unroll
    for (int j = 0; j < 3; j++) vd[j] = vpk<s16x2>(upk(c[j])) - vpk<s16x2>(upk(a[j]));
    const s16x2 gx01 = vpk<s16x2>(upk(vs[1])) - vpk<s16x2>(upk(vs[0]));
    const s16x2 gx23 = vpk<s16x2>(upk(vs[2])) - vpk<s16x2>(upk(vs[1]));
    const s16x2 d01 = vpk<s16x2>(__builtin_amdgcn_perm(upk(vd[1]), upk(vd[0]), 0x05040302u));  // vd(0), vd(1)
    const s16x2 d23 = vpk<s16x2>(__builtin_amdgcn_perm(upk(vd[2]), upk(vd[1]), 0x05040302u));  // vd(2), vd(3)
    const s16x2 gy01 = vd[0] + vd[1] + (d01 << 1);
    const s16x2 gy23 = vd[1] + vd[2] + (d23 << 1);
    const s16x2 m01 = __builtin_elementwise_max(gx01, -gx01) + __builtin_elementwise_max(gy01, -gy01);
    const s16x2 m23 = __builtin_elementwise_max(gx23, -gx23) + __builtin_elementwise_max(gy23, -gy23);
    *(uint2*)(mag + ly * FGW + 4 * k) = make_uint2(upk(m01), upk(m23));
    if (ly >= 1 && ly <= FTH && k >= 1 && k <= FTW / 4) {
      const int jj = (ly - 1) * FTW + 4 * (k - 1);
      *(uint2*)(gx_s + jj) = make_uint2(upk(gx01), upk(gx23));
      *(uint2*)(gy_s + jj) = make_uint2(upk(gy01), upk(gy23));
    }
  }
}

// Interior NMS, four pixels per work-item on i16 pairs (MK_CANNY_V). Per
// pixel the reference's rule (cv::Canny, the direction from |gy| 2^15 against
// |gx| tan(22.5) 2^15 and |gx| tan(67.5) 2^15, the neighbour pair along it,
// m > a && (diagonal ? m > b : m >= b), then weak / strong against low / high)
// as masks: every comparison of values <= 2040 is the sign of a 16-bit
// difference (v_pk_sub + v_pk_ashr 15), the direction tests are the signs of
// two 24-bit multiply-adds, the neighbour choice is v_bfi on the pairs. The
// classes of a group go to cls (byte u: candidate nibble | strong nibble << 4).
// 0xffff per negative half: v_perm_b32's selectors 9 / 11 replicate bit 31 of
// its second / first operand into a byte, so one perm builds both halves
// (tools/perm_sign_check.hip: identical to the two-shift form on 2^24 pairs)
// a * b + c, a and b 24-bit signed (b wave-uniform): one v_mad_i32_i24
__device__ __forceinline__ int32_t mad24(int32_t a, int32_t b, int32_t c) {
  int32_t r;
  asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
  return r;
}
__device__ inline uint32_t sign_pair(int32_t lo, int32_t hi) {
  return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x0B0B0909u);
}
__device__ inline void nms4(const int16_t* mag, const int16_t* gx_s, const int16_t* gy_s, int low, int high,
                            uint8_t* cls, int t) {
  constexpr int SHIFT = 15;
  constexpr int TG22 = (int)(0.4142135623730950488016887242097 * (1 << SHIFT) + 0.5);
  const int lowc = low < -1 ? -1 : (low > 32767 ? 32767 : low);
  const int highc = high < -1 ? -1 : (high > 32767 ? 32767 : high);
  const s16x2 LOW = {(short)lowc, (short)lowc}, HIGH = {(short)highc, (short)highc};
  for (int u = t; u < FTH * FTW / 4; u += 256) {
    const int ly = u >> 5, k = u & 31;  // FTW / 4 = 32 groups per row
    uint32_t P[3][3], C[3][2];          // per row (up, centre, down): pairs (-1,0) (1,2) (3,4); (0,1) (2,3)
#pragma unroll
    for (int r = 0; r < 3; r++) {
      const int16_t* row = mag + (ly + r) * FGW + 4 * k;  // mag row ly + r = image row y0 + ly - 1 + r
      const uint32_t lo = *(const uint32_t*)(row + 2);
      const uint2 mid = *(const uint2*)(row + 4);
      const uint32_t hi = *(const uint32_t*)(row + 8);
      C[r][0] = mid.x;
      C[r][1] = mid.y;
      P[r][0] = __builtin_amdgcn_perm(mid.x, lo, 0x05040302u);
      P[r][1] = __builtin_amdgcn_perm(mid.y, mid.x, 0x05040302u);
      P[r][2] = __builtin_amdgcn_perm(hi, mid.y, 0x05040302u);
    }
    const uint2 gxw = *(const uint2*)(gx_s + ly * FTW + 4 * k);
    const uint2 gyw = *(const uint2*)(gy_s + ly * FTW + 4 * k);
    uint32_t push[2], strong[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t gxp = h ? gxw.y : gxw.x, gyp = h ? gyw.y : gyw.x;
      const s16x2 X = vpk<s16x2>(gxp), Y = vpk<s16x2>(gyp);
      const s16x2 AX = __builtin_elementwise_max(X, -X), AY = __builtin_elementwise_max(Y, -Y);
      const uint32_t ax = upk(AX), ay = upk(AY);
      const int ax0 = (int)(ax & 0xffffu), ax1 = (int)(ax >> 16);
      const int ay0 = (int)(ay & 0xffffu) << SHIFT, ay1 = (int)(ay >> 16) << SHIFT;
      // hor: ay 2^15 < ax TG22; ver: ay 2^15 > ax (TG22 + 2^16)
      const uint32_t HOR = sign_pair(ay0 - ax0 * TG22, ay1 - ax1 * TG22);
      const uint32_t VER = sign_pair(ax0 * (TG22 + (1 << (SHIFT + 1))) - ay0, ax1 * (TG22 + (1 << (SHIFT + 1))) - ay1);
      uint32_t NEG = upk(vpk<s16x2>(gxp ^ gyp) >> 15);  // gx gy < 0: the (up-right, down-left) diagonal
      asm volatile("" : "+v"(NEG));  // keeps the selects v_bfi (k_canny_strip)
      // neighbour pairs of pixels (2h, 2h+1): left / centre / right columns of each row
      const uint32_t UL = P[0][h], U = C[0][h], UR = P[0][h + 1];
      const uint32_t L = P[1][h], M = C[1][h], R = P[1][h + 1];
      const uint32_t DL = P[2][h], D = C[2][h], DR = P[2][h + 1];
      const uint32_t A = (HOR & L) | (~HOR & ((VER & U) | (~VER & ((NEG & UR) | (~NEG & UL)))));
      const uint32_t B = (HOR & R) | (~HOR & ((VER & D) | (~VER & ((NEG & DL) | (~NEG & DR)))));
      // push = m > max(A, low, B - [HOR or VER]) (k_canny_strip's form)
      const s16x2 Ms = vpk<s16x2>(M);
      const s16x2 Bp = vpk<s16x2>(B) + vpk<s16x2>(HOR | VER);
      const s16x2 T = __builtin_elementwise_max(__builtin_elementwise_max(vpk<s16x2>(A), LOW), Bp);
      push[h] = upk((T - Ms) >> 15);
      strong[h] = push[h] & upk((HIGH - Ms) >> 15);
    }
    // nibbles: pixel 2h + j <-> bit j of half h's word
    const uint32_t xp = (push[0] & 0x00020001u) | (push[1] & 0x00080004u);
    const uint32_t xs = (strong[0] & 0x00020001u) | (strong[1] & 0x00080004u);
    const uint32_t x = xp | (xs << 4);
    cls[u] = (uint8_t)(x | (x >> 16));
  }
}
// 32-bit word of candidate (strong: hi) bits from 8 class bytes (groups 0..7)
__device__ inline uint32_t nibbles32(uint64_t v, bool hi) {
  uint64_t x = (hi ? v >> 4 : v) & 0x0F0F0F0F0F0F0F0Full;
  x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
  x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
  return (uint32_t)(x | (x >> 16));
}
#ifndef MK_CANNY_V
#define MK_CANNY_V 1
#endif

// The Canny stages of one tile into the candidate / strong masks gm, sm (bit
// i & 63 of word i >> 6 = tile pixel i, i = ly * FTW + lx). IN: the tile and its halo
// (x0-4 .. x0+FTW+3, y0-3 .. y0+FTH+2) lie inside the image and the rows
// allow dword loads, so the border rules (reflect/replicate/zero) drop out.
template <bool IN>
__device__ inline void canny_classes(const FrameDesc& fd, int W, int H, int x0, int y0, int low, int high, int vec,
                                     uint8_t* g, uint8_t* bl, int16_t* mag, int16_t* gxy, uint64_t* gm, uint64_t* sm,
                                     int t) {
  constexpr int BLH = FTH + 4;
  int16_t* gx_s = gxy;
  int16_t* gy_s = gxy + FTW * FTH;
  // gray, 4-pixel groups
  for (int u = t; u < FGH * (FGW / 4); u += 256) {
    const int ly = u / (FGW / 4), lg = u % (FGW / 4);
    const int y = y0 - 3 + ly, xs = x0 - 4 + 4 * lg;
    uint8_t* o = g + ly * FGW + 4 * lg;
    if (IN) {
      // 32-bit offset from the frame base (frames are < 4 GB): global_load with
      // the base in SGPRs, no per-lane 64-bit address arithmetic
      gu32* q = gwords(fd.bgr + (uint32_t)(((uint32_t)y * (uint32_t)W + (uint32_t)xs) * 3u));
      *(uint32_t*)o = gray4(q[0], q[1], q[2]);
    } else if (y < 0 || y >= H) {
      o[0] = o[1] = o[2] = o[3] = 0;
    } else if (vec && xs >= 0 && xs + 3 < W) {
      gu32* q = gwords(fd.bgr + ((size_t)y * W + xs) * 3);
      *(uint32_t*)o = gray4(q[0], q[1], q[2]);
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int x = xs + k;
        o[k] = (x >= 0 && x < W) ? gray_px(gbytes(fd.bgr + ((size_t)y * W + x) * 3)) : 0;
      }
    }
  }
  __syncthreads();
  if (IN) {
    hblur4(g, (uint16_t*)gxy, t);
    __syncthreads();
    vblur4((const uint16_t*)gxy, bl, t);
    __syncthreads();
    if (MK_CANNY_V) sobel4v(bl, mag, gx_s, gy_s, t);
    else sobel4(bl, mag, gx_s, gy_s, t);
    __syncthreads();
    if (MK_CANNY_V) {
      nms4(mag, gx_s, gy_s, low, high, (uint8_t*)gm, t);  // gm, sm: one 512-byte class array here
      __syncthreads();
      return;
    }
  } else {
  // horizontal blur on rows y0-3 .. y0+FTH+2, columns x0-2 .. x0+FTW+1
  // (BORDER_REFLECT_101); staged in the gradient buffer, not live yet
  uint16_t* rowb = (uint16_t*)gxy;  // FGH * FRW <= 2 * FTW * FTH
  for (int i = t; i < FGH * FRW; i += 256) {
    const int ly = i / FRW, lx = i % FRW;
    const int x = x0 - 2 + lx, y = y0 - 3 + ly;
    int v = 0;
    if (IN || (x >= 0 && x < W && y >= 0 && y < H)) {
      const int xm = (IN ? x - 1 : refl101(x - 1, W)) - (x0 - 4), xc = x - (x0 - 4),
                xp = (IN ? x + 1 : refl101(x + 1, W)) - (x0 - 4);
      const uint8_t* gr = g + ly * FGW;
      v = 84 * gr[xm] + 89 * gr[xc] + 84 * gr[xp];
    }
    rowb[i] = (uint16_t)v;
  }
  __syncthreads();
  // vertical blur on rows y0-2 .. y0+FTH+1
  for (int i = t; i < BLH * FRW; i += 256) {
    const int ly = i / FRW, lx = i % FRW;
    const int x = x0 - 2 + lx, y = y0 - 2 + ly;
    uint8_t v = 0;
    if (IN || (x >= 0 && x < W && y >= 0 && y < H)) {
      const int ym = (IN ? y - 1 : refl101(y - 1, H)) - (y0 - 3), yc = y - (y0 - 3),
                yp = (IN ? y + 1 : refl101(y + 1, H)) - (y0 - 3);
      const int acc = 84 * rowb[ym * FRW + lx] + 89 * rowb[yc * FRW + lx] + 84 * rowb[yp * FRW + lx];
      const int r = (acc + (1 << 15)) >> 16;
      v = (uint8_t)(r > 255 ? 255 : r);
    }
    bl[i] = v;
  }
  __syncthreads();
  // Sobel (replicated border) -> L1 magnitude on x0-1 .. x0+FTW, y0-1 .. y0+FTH;
  // the tile's own pixels also keep gx, gy for the NMS
  for (int i = t; i < FMH * FMW; i += 256) {
    const int ly = i / FMW, lx = i % FMW;
    const int x = x0 - 1 + lx, y = y0 - 1 + ly;
    int m = 0;
    if (IN || (x >= 0 && x < W && y >= 0 && y < H)) {
      const int cl = (IN || x > 0 ? x - 1 : 0) - (x0 - 2), cm = x - (x0 - 2),
                cr = (IN || x + 1 < W ? x + 1 : W - 1) - (x0 - 2);
      const int ra = ((IN || y > 0 ? y - 1 : 0) - (y0 - 2)) * FRW, rb = (y - (y0 - 2)) * FRW,
                rc = ((IN || y + 1 < H ? y + 1 : H - 1) - (y0 - 2)) * FRW;
      const int l0 = bl[ra + cl], m0 = bl[ra + cm], q0 = bl[ra + cr];
      const int l1 = bl[rb + cl], q1 = bl[rb + cr];
      const int l2 = bl[rc + cl], m2 = bl[rc + cm], q2 = bl[rc + cr];
      const int gx = (q0 - l0) + 2 * (q1 - l1) + (q2 - l2);
      const int gy = (l2 - l0) + 2 * (m2 - m0) + (q2 - q0);
      m = abs(gx) + abs(gy);
      if (ly >= 1 && ly <= FTH && lx >= 1 && lx <= FTW) {
        const int j = (ly - 1) * FTW + lx - 1;
        gx_s[j] = (int16_t)gx;
        gy_s[j] = (int16_t)gy;
      }
    }
    mag[i] = (int16_t)m;
  }
  __syncthreads();
  }
  // NMS -> classes (0 none, 1 weak candidate, 2 strong); magnitude pitch and
  // column offset of the tile's pixels: interior FGW / 4, generic FMW / 1
  constexpr int MP = IN ? FGW : FMW, MO = IN ? 4 : 1;
  const int SHIFT = 15;
  const int TG22 = (int)(0.4142135623730950488016887242097 * (1 << SHIFT) + 0.5);
  for (int i = t; i < FTW * FTH; i += 256) {
    const int ly = i / FTW, lx = i % FTW;
    const int x = x0 + lx, y = y0 + ly;
    uint8_t c = 0;
    if (IN || (x < W && y < H)) {
      const int cy = ly + 1, cx = lx + MO;
      const int m = mag[cy * MP + cx];
      if (m > low) {
        // the three direction cases as selects (one pair of neighbour reads,
        // no divergent branches): horizontal m > left && m >= right, vertical
        // m > up && m >= down, diagonal m > both along the sign of gx * gy
        const int xs = gx_s[i], ys = gy_s[i];
        const int ax = abs(xs);
        const int ay = abs(ys) << SHIFT;
        const int tg22x = ax * TG22;
        const int tg67x = tg22x + (ax << (SHIFT + 1));
        const bool hor = ay < tg22x, ver = !hor && ay > tg67x, diag = !hor && !ver;
        const int sg = (xs ^ ys) < 0 ? -1 : 1;
        const int o = hor ? 1 : (ver ? MP : MP + sg);
        const int c0 = cy * MP + cx;
        const int a = mag[c0 - o], b = mag[c0 + o];
        const bool push = m > a && (diag ? m > b : m >= b);
        if (push) c = (m > high) ? 2 : 1;
      }
    }
    // a wave covers 64 consecutive tile pixels (uniform trip count)
    const uint64_t mc = __ballot(c != 0), ms = __ballot(c == 2);
    if ((t & 63) == 0) {
      gm[i >> 6] = mc;
      sm[i >> 6] = ms;
    }
  }
  __syncthreads();
}

// vec: every frame of the batch has W % 4 == 0 and a 4-byte aligned base, so a
// 4-pixel group is three aligned dwords.
// One-dimensional grid of gx * gy tiles per frame, remapped XCD-aware: blocks
// b and b + 8 share an XCD (round-robin dealing), so every group of blocks
// with the same b % 8 takes one contiguous run of tiles (frame-major,
// row-major within a frame) and a tile's halo rows, read again by the tile
// below, stay in that XCD's L2 (bijective remap, cdna_hip_programming.md T1).
__global__ __launch_bounds__(256) void k_canny(const FrameDesc* __restrict__ frames, int low, int high, int vec,
                                               uint32_t* __restrict__ cbits, uint32_t* __restrict__ sbits,
                                               size_t bstride, int gx, int gy) {
  const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rr = nwg & 7;
  const int wgid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
  const int f = wgid / (gx * gy), ti = wgid - f * (gx * gy);
  const FrameDesc fd = frames[f];
  const int W = fd.w, H = fd.h;
  const int x0 = (ti % gx) * FTW, y0 = (ti / gx) * FTH;
  if (x0 >= W || y0 >= H) return;
  // LDS regions reused across phases:
  //   R1: gray (x0-4 .., y0-3 ..) -> magnitude (x0-1 .., y0-1 ..)
  //   R2: blurred (x0-2 .., y0-2 ..)
  //   R3: horizontal blur -> gx | gy of the tile
  constexpr int BLH = FTH + 4;  // blurred rows y0-2 .. y0+FTH+1
  constexpr int R1 = FMH * FGW * 2 > FGH * FGW ? FMH * FGW * 2 : FGH * FGW;
  __shared__ __align__(16) uint8_t r1[R1];
  __shared__ __align__(16) uint8_t bl[BLH * FGW];
  __shared__ __align__(16) int16_t gxy[2 * FTW * FTH];
  // candidate / strong masks (generic tiles); interior tiles (MK_CANNY_V)
  // keep one class byte per 4-pixel group in the same 512 bytes
  __shared__ uint64_t gms[2 * FTW * FTH / 64];
  uint64_t* gm = gms;
  uint64_t* sm = gms + FTW * FTH / 64;
  const int t = threadIdx.x;
  const bool interior = vec && x0 >= 4 && x0 + FTW + 4 <= W && y0 >= 3 && y0 + FTH + 3 <= H;
  if (interior) canny_classes<true>(fd, W, H, x0, y0, low, high, vec, r1, bl, (int16_t*)r1, gxy, gm, sm, t);
  else canny_classes<false>(fd, W, H, x0, y0, low, high, vec, r1, bl, (int16_t*)r1, gxy, gm, sm, t);
  // 32-bit word j of the tile = row j / 4, quarter j % 4 = half j & 1 of mask
  // j / 2 (generic), class bytes 8j .. 8j + 7 (interior)
  const int WW = bits::words(W);
  static_assert(FTW == 128, "four 32-pixel words per tile row");
  for (int j = t; j < FTW * FTH / 32; j += 256) {
    const int y = y0 + (j >> 2), w = (x0 >> 5) + (j & 3);
    if (y < H && w < WW) {
      const size_t o = (size_t)f * bstride + (size_t)y * WW + w;
      if (MK_CANNY_V && interior) {
        const uint64_t v = ((const uint64_t*)gms)[j];
        cbits[o] = nibbles32(v, false);
        sbits[o] = nibbles32(v, true);
      } else {
        cbits[o] = (uint32_t)(gm[j >> 1] >> (32 * (j & 1)));
        sbits[o] = (uint32_t)(sm[j >> 1] >> (32 * (j & 1)));
      }
    }
  }
}

// ------------------------------------------------ Canny as column strips
// The same stages (gray, [84,89,84] blur with BORDER_REFLECT_101, Sobel with
// BORDER_REPLICATE, L1 magnitude, NMS, weak / strong classes) without LDS or
// barriers: a wave owns a strip of 64 x 4 columns and walks down the frame,
// each lane keeping its 4 columns' last rows of every stage in registers
// (the vertical taps) and taking the columns left and right of its own from
// the neighbouring lanes by DPP (the horizontal taps). Lanes 0..55 produce
// the strip's 224 columns (7 bit-plane words), lane 56 and lane 63 (the
// column group left of the strip, reached by the wave rotation) are the
// halo, lanes 57..62 idle. The stage outputs lag the input row: hblur(i),
// blur(i-1), Sobel(i-2), NMS(i-3). At the frame's edges the neighbour values
// are the border rules' (reflected gray, replicated blur, zero magnitude) in
// the first / last column groups and rows. Every value is the same integer
// as k_canny's (interior tiles), so the planes are identical.
__device__ inline uint32_t dpp_from_left(uint32_t v) {  // lane l gets lane l-1's v (lane 0: lane 63's)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x13C, 0xf, 0xf, false);
}
__device__ inline uint32_t dpp_from_right(uint32_t v) {  // lane l gets lane l+1's v (lane 63: lane 0's)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x134, 0xf, 0xf, false);
}
__device__ inline uint32_t dpp_row_shr(uint32_t v, int n) {  // lane l gets lane l-n of its 16-lane row, 0 past the row's start
  switch (n) {
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xf, 0xf, true);
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x112, 0xf, 0xf, true);
    default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x114, 0xf, 0xf, true);
  }
}
// K column groups of 4 per lane: K = 1 (W % 4 == 0) strips of 56 lanes x 4 =
// 224 columns (7 words, halo lanes 56 / 63); K = 2 (W % 8 == 0) strips of 60
// lanes x 8 = 480 columns (15 words, halo lanes 60 / 63): half the DPP,
// border selects and nibble packing per column, 6 % idle lanes instead of 12 %.
#ifndef MK_STRIP2_WAVES
#define MK_STRIP2_WAVES 4
#endif
template <int K>
struct StripGeom {
  static constexpr int out_lanes = K == 1 ? 56 : 60;       // lanes producing the strip's columns
  static constexpr int cols = out_lanes * 4 * K;            // columns per strip
  static constexpr int lanes_per_word = 8 / K;
};
// BGR rows a wave keeps in flight: K = 2 has the registers for MK_CANNY_PF
// (126 VGPRs at depth 2, under the 128 of 4 waves per SIMD; depth 3 spills),
// K = 1 (64 VGPRs for 8 waves) only for one
#ifndef MK_CANNY_PF
#define MK_CANNY_PF 1
#endif
template <int K>
constexpr int strip_pf() { return K == 2 ? MK_CANNY_PF : 1; }
// Per-wave state of a strip: three row slots per stage (row r in slot r % 3),
// so the walk unrolled by three indexes registers with constants and moves
// nothing between rows.
template <int K>
struct StripRegs {
  uint32_t hba[3][K], hbb[3][K];  // horizontal blur, 2 u16 pairs per group
  uint32_t bla[3][K], blb[3][K];  // blur, 2 u16 pairs per group
  uint32_t mga[3][K], mgb[3][K];  // L1 magnitude, 2 i16 pairs per group
  // |gx| with the sign of gx ^ gy in bit 15 of each half (NMS's diagonal
  // choice), |gy|: what the NMS reads, so it takes no absolute values
  uint32_t gxa[3][K], gxb[3][K], gya[3][K], gyb[3][K];
};
template <int K>
struct StripWave {
  const uint8_t* bgr;  // the frame (wave-uniform); lane offsets are 32-bit
  uint32_t loff;       // this lane's first byte in a row
  uint32_t rstep;
  int H, WW, lane;
  bool left_edge, right_edge, inside, store_lane;
  s16x2 LOW, HIGH;
  int KH, KV;  // -2 TG22, -2 (TG22 + 2^16) (v_mad_i32_i24 operands)
  uint32_t TWO;  // (2, 2) in an SGPR the compiler cannot see through: x 2 + y stays one v_pk_mad
  uint32_t* cb;
  uint32_t* sbp;
  // BGR rows in flight (strip_pf): 1 = row i, 2 = rows i, i+1 (shifted down a
  // slot per row), 3 = rows i .. i+2 in slots i % 3 (the walk's unroll)
  uint32_t rows[strip_pf<K>()][K][3];
};
template <int K>
__device__ __forceinline__ void strip_load_to(const StripWave<K>& w, int row, uint32_t (&d)[K][3]) {
#pragma unroll
  for (int k = 0; k < K; k++) {
    gu32* q = gwords(w.bgr + (w.loff + 12u * k + (uint32_t)row * w.rstep));
    d[k][0] = q[0];
    d[k][1] = q[1];
    d[k][2] = q[2];
  }
}
// the input row of iteration i (S = i % 3) and the load that replaces it:
// row i + strip_pf (the last row again past the end)
template <int K, int S>
__device__ __forceinline__ const uint32_t (&strip_row(const StripWave<K>& w))[K][3] {
  return w.rows[strip_pf<K>() == 3 ? S : 0];
}
template <int K, int S>
__device__ __forceinline__ void strip_advance(StripWave<K>& w, int i) {
  constexpr int PF = strip_pf<K>();
  const int r = i + PF < w.H ? i + PF : w.H - 1;
  if constexpr (PF == 3) {
    strip_load_to(w, r, w.rows[S]);
  } else {
#pragma unroll
    for (int p = 0; p + 1 < PF; p++)
#pragma unroll
      for (int k = 0; k < K; k++)
#pragma unroll
        for (int j = 0; j < 3; j++) w.rows[p][k][j] = w.rows[p + 1][k][j];
    strip_load_to(w, r, w.rows[PF - 1]);
  }
}
// Iteration i of the walk (S = i % 3): hblur(i), blur(i-1), Sobel(i-2), NMS(i-3).
// ROWS: the frame's first / last rows may be among them (else all four rows
// are inside the frame and no row rule applies: 6 <= i <= H - 1); EDGE: the
// strip holds the frame's first or last column group (else no lane needs a
// column rule). Group k's left / right neighbours are the lane's groups k-1 /
// k+1, or the neighbouring lanes' last / first group by DPP.
template <int K, int S, bool ROWS, bool EDGE>
__device__ __forceinline__ void strip_step(StripWave<K>& w, StripRegs<K>& R, int i) {
  // the nibble packing below (WK) has weights for groups 0 and 1 only: bits 0..7 of a lane's byte
  static_assert(K == 1 || K == 2, "k_canny_strip packs at most two 4-column groups per lane");
  constexpr int S1 = (S + 1) % 3, S2 = (S + 2) % 3;  // slots of rows i-2 / i+1, i-1
  constexpr int SHIFT = 15;
  constexpr int TG22 = (int)(0.4142135623730950488016887242097 * (1 << SHIFT) + 0.5);
  const u16x2 c84 = {84, 84}, c89 = {89, 89};
  const int H = w.H;
  // ---- gray and horizontal blur of input row i
  if (!ROWS || i < H) {
    uint32_t g01[K], g23[K];  // gray as u16 pairs: pixels (0, 1), (2, 3) of each group
    {
      const uint32_t(&nx)[K][3] = strip_row<K, S>(w);
#pragma unroll
      for (int k = 0; k < K; k++) gray4_pairs(nx[k][0], nx[k][1], nx[k][2], g01[k], g23[k]);
    }
    strip_advance<K, S>(w, i);
    // the left group's (2, 3) pair, the right group's (0, 1) pair
    uint32_t gl = dpp_from_left(g23[K - 1]), gr = dpp_from_right(g01[0]);
    if (EDGE && w.left_edge) gl = g01[0];        // gray(-1) = gray(1): the high half
    if (EDGE && w.right_edge) gr = g23[K - 1];   // gray(W) = gray(W-2): the low half
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t l23 = k ? g23[k - 1] : gl, r01 = k + 1 < K ? g01[k + 1] : gr;
      const u16x2 l01 = vpk<u16x2>(__builtin_amdgcn_perm(g01[k], l23, 0x05040302u));     // pixels -1, 0
      const u16x2 q01 = vpk<u16x2>(__builtin_amdgcn_perm(g23[k], g01[k], 0x05040302u));  // 1, 2
      const u16x2 q23 = vpk<u16x2>(__builtin_amdgcn_perm(r01, g23[k], 0x05040302u));     // 3, 4
      const u16x2 o01 = (l01 + q01) * c84 + vpk<u16x2>(g01[k]) * c89;
      const u16x2 o23 = (q01 + q23) * c84 + vpk<u16x2>(g23[k]) * c89;
      R.hba[S][k] = upk(o01);
      R.hbb[S][k] = upk(o23);
    }
  } else if (ROWS && i == H) {  // row H = row H-2 (reflect), for the blur of row H-1
#pragma unroll
    for (int k = 0; k < K; k++) {
      R.hba[S][k] = R.hba[S1][k];
      R.hbb[S][k] = R.hbb[S1][k];
    }
  }
  // ---- vertical blur of row j = i - 1 (hblur rows j-1, j, j+1 = slots S1, S2, S)
  const int j = i - 1;
  if (!ROWS || (j >= 0 && j < H)) {
    const bool top = ROWS && j == 0;
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t aa = top ? R.hba[S][k] : R.hba[S1][k], ab = top ? R.hbb[S][k] : R.hbb[S1][k];  // row -1 = row 1
      // pixel b: 84 (a + c) + 89 m + 2^15 as three v_dot2_u32_u16 on the packed
      // u16 pairs themselves, the other half's coefficient 0 (no unpacking)
      const uint32_t A2[2] = {aa, ab}, B2[2] = {R.hba[S2][k], R.hbb[S2][k]}, C2[2] = {R.hba[S][k], R.hbb[S][k]};
      uint32_t o[2];
#pragma unroll
      for (int p = 0; p < 2; p++) {
        uint32_t r[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
          const u16x2 c84 = h ? u16x2{0, 84} : u16x2{84, 0}, c89 = h ? u16x2{0, 89} : u16x2{89, 0};
          r[h] = __builtin_amdgcn_udot2(vpk<u16x2>(B2[p]), c89, 1u << 15, false);
          r[h] = __builtin_amdgcn_udot2(vpk<u16x2>(C2[p]), c84, r[h], false);
          r[h] = __builtin_amdgcn_udot2(vpk<u16x2>(A2[p]), c84, r[h], false);
        }
        // the high halves (sum >> 16, at most 257) as a u16 pair, clamped to 255
        const u16x2 q = vpk<u16x2>(__builtin_amdgcn_perm(r[1], r[0], 0x07060302u));
        o[p] = upk(__builtin_elementwise_min(q, (u16x2){255, 255}));
      }
      R.bla[S2][k] = o[0];
      R.blb[S2][k] = o[1];
    }
  } else if (ROWS && j == H) {
#pragma unroll
    for (int k = 0; k < K; k++) {  // row H = row H-1 (replicate), for the Sobel of row H-1
      R.bla[S2][k] = R.bla[S1][k];
      R.blb[S2][k] = R.blb[S1][k];
    }
  }
  // ---- Sobel of row m = i - 2 (blur rows m-1, m, m+1 = slots S, S1, S2)
  const int m = i - 2;
  if (!ROWS || (m >= 0 && m < H)) {
    uint32_t vs01[K], vs23[K], vd01[K], vd23[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      const bool top = ROWS && m == 0;  // row -1 = row 0
      const u16x2 A01 = vpk<u16x2>(top ? R.bla[S1][k] : R.bla[S][k]), A23 = vpk<u16x2>(top ? R.blb[S1][k] : R.blb[S][k]);
      const u16x2 B01 = vpk<u16x2>(R.bla[S1][k]), B23 = vpk<u16x2>(R.blb[S1][k]);
      const u16x2 C01 = vpk<u16x2>(R.bla[S2][k]), C23 = vpk<u16x2>(R.blb[S2][k]);
      vs01[k] = upk(B01 * vpk<u16x2>(w.TWO) + (A01 + C01));
      vs23[k] = upk(B23 * vpk<u16x2>(w.TWO) + (A23 + C23));
      vd01[k] = upk(vpk<s16x2>(upk(C01)) - vpk<s16x2>(upk(A01)));
      vd23[k] = upk(vpk<s16x2>(upk(C23)) - vpk<s16x2>(upk(A23)));
    }
    uint32_t VL0 = dpp_from_left(vs23[K - 1]), VRK = dpp_from_right(vs01[0]);
    uint32_t DL0 = dpp_from_left(vd23[K - 1]), DRK = dpp_from_right(vd01[0]);
    if (EDGE && w.left_edge) { VL0 = vs01[0] << 16; DL0 = vd01[0] << 16; }                  // blur(-1) = blur(0)
    if (EDGE && w.right_edge) { VRK = vs23[K - 1] >> 16; DRK = vd23[K - 1] >> 16; }        // blur(W) = blur(W-1)
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t VL = k ? vs23[k - 1] : VL0, VR = k + 1 < K ? vs01[k + 1] : VRK;
      const uint32_t DL = k ? vd23[k - 1] : DL0, DR = k + 1 < K ? vd01[k + 1] : DRK;
      const s16x2 S0v = vpk<s16x2>(__builtin_amdgcn_perm(vs01[k], VL, 0x05040302u));     // columns -1, 0
      const s16x2 S1v = vpk<s16x2>(__builtin_amdgcn_perm(vs23[k], vs01[k], 0x05040302u)); // 1, 2
      const s16x2 S2v = vpk<s16x2>(__builtin_amdgcn_perm(VR, vs23[k], 0x05040302u));      // 3, 4
      const s16x2 D0 = vpk<s16x2>(__builtin_amdgcn_perm(vd01[k], DL, 0x05040302u));
      const s16x2 D1 = vpk<s16x2>(__builtin_amdgcn_perm(vd23[k], vd01[k], 0x05040302u));
      const s16x2 D2 = vpk<s16x2>(__builtin_amdgcn_perm(DR, vd23[k], 0x05040302u));
      const s16x2 gx01 = S1v - S0v, gx23 = S2v - S1v;
      const s16x2 gy01 = vpk<s16x2>(vd01[k]) * vpk<s16x2>(w.TWO) + (D0 + D1);
      const s16x2 gy23 = vpk<s16x2>(vd23[k]) * vpk<s16x2>(w.TWO) + (D1 + D2);
      const s16x2 ax01 = __builtin_elementwise_max(gx01, -gx01), ay01 = __builtin_elementwise_max(gy01, -gy01);
      const s16x2 ax23 = __builtin_elementwise_max(gx23, -gx23), ay23 = __builtin_elementwise_max(gy23, -gy23);
      R.mga[S1][k] = upk(ax01 + ay01);
      R.mgb[S1][k] = upk(ax23 + ay23);
      R.gxa[S1][k] = upk(ax01) | ((upk(gx01) ^ upk(gy01)) & 0x80008000u);
      R.gxb[S1][k] = upk(ax23) | ((upk(gx23) ^ upk(gy23)) & 0x80008000u);
      R.gya[S1][k] = upk(ay01);
      R.gyb[S1][k] = upk(ay23);
    }
  } else if (ROWS && m == H) {
#pragma unroll
    for (int k = 0; k < K; k++) {
      R.mga[S1][k] = 0;  // magnitude below the frame: zero
      R.mgb[S1][k] = 0;
    }
  }
  // ---- NMS of row n = i - 3 (magnitude rows n-1, n, n+1 = slots S2, S, S1)
  const int n = i - 3;
  if (ROWS && n < 0) return;
  const bool first = ROWS && n == 0;
  uint32_t P[3][K][3], Cw[3][K][2];
#pragma unroll
  for (int r = 0; r < 3; r++) {
    uint32_t rwa[K], rwb[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
      rwa[k] = r == 0 ? (first ? 0u : R.mga[S2][k]) : r == 1 ? R.mga[S][k] : R.mga[S1][k];  // above the frame: zero
      rwb[k] = r == 0 ? (first ? 0u : R.mgb[S2][k]) : r == 1 ? R.mgb[S][k] : R.mgb[S1][k];
    }
    uint32_t Lw0 = dpp_from_left(rwb[K - 1]), RwK = dpp_from_right(rwa[0]);
    if (EDGE && w.left_edge) Lw0 = 0u;
    if (EDGE && w.right_edge) RwK = 0u;
#pragma unroll
    for (int k = 0; k < K; k++) {
      const uint32_t Lw = k ? rwb[k - 1] : Lw0, Rw = k + 1 < K ? rwa[k + 1] : RwK;
      Cw[r][k][0] = rwa[k];
      Cw[r][k][1] = rwb[k];
      P[r][k][0] = __builtin_amdgcn_perm(rwa[k], Lw, 0x05040302u);
      P[r][k][1] = __builtin_amdgcn_perm(rwb[k], rwa[k], 0x05040302u);
      P[r][k][2] = __builtin_amdgcn_perm(Rw, rwb[k], 0x05040302u);
    }
  }
  uint32_t cw = 0, sw = 0;
#pragma unroll
  for (int k = 0; k < K; k++) {
    uint32_t dp[2], ds[2];  // per half: sign bits = push / strong
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t axn = h ? R.gxb[S][k] : R.gxa[S][k], ay = h ? R.gyb[S][k] : R.gya[S][k];
      const int ax0 = (int)(axn & 0x7fffu), ax1 = (int)((axn >> 16) & 0x7fffu);
      // OpenCV's tests at twice the scale, each a single v_mad_i32_i24 per
      // pixel: hor: ay 2^16 < ax 2 TG22; ver: ay 2^16 > ax 2 (TG22 + 2^16).
      // VERN = ~ver but at gx = gy = 0, where m = 0 never pushes
      const int ay0 = (int)(ay << 16), ay1 = (int)(ay & 0xffff0000u);
      // (asm: left to itself the compiler derives VERN from HOR's product
      // with a shift and a subtract per pixel)
      const uint32_t HOR = sign_pair(mad24(ax0, w.KH, ay0), mad24(ax1, w.KH, ay1));
      const uint32_t VERN = sign_pair(mad24(ax0, w.KV, ay0), mad24(ax1, w.KV, ay1));
      uint32_t NEG = upk(vpk<s16x2>(axn) >> 15);
      // opaque: seen as a sign mask, the selects below become per-half
      // compares + v_cndmask + repacking (12 ops per half instead of 2 v_bfi)
      asm volatile("" : "+v"(NEG));
      const uint32_t UL = P[0][k][h], U = Cw[0][k][h], UR = P[0][k][h + 1];
      const uint32_t L = P[1][k][h], Mm = Cw[1][k][h], Rr = P[1][k][h + 1];
      const uint32_t DLw = P[2][k][h], Dd = Cw[2][k][h], DRw = P[2][k][h + 1];
      const uint32_t A = (HOR & L) | (~HOR & ((VERN & ((NEG & UR) | (~NEG & UL))) | (~VERN & U)));
      const uint32_t B = (HOR & Rr) | (~HOR & ((VERN & ((NEG & DLw) | (~NEG & DRw))) | (~VERN & Dd)));
      // push = m > A && m > low && (m >= B horizontally / vertically, m > B on
      // the diagonals) = m > max(A, low, B - [HOR or VER]): one compare (the
      // masks are 0 / -1 per half, so adding HOR | VER subtracts 1 there)
      const s16x2 Ms = vpk<s16x2>(Mm);
      const s16x2 Bp = vpk<s16x2>(B) + vpk<s16x2>(HOR | ~VERN);
      const s16x2 T = __builtin_elementwise_max(__builtin_elementwise_max(vpk<s16x2>(A), w.LOW), Bp);
      dp[h] = upk(T - Ms);                                     // m > T: push
      ds[h] = upk(__builtin_elementwise_max(T, w.HIGH) - Ms);  // m > T and m > high: strong
    }
    // the four sign bits as bytes 0 / -1 (v_perm sign replication), then one
    // signed byte dot with weights -2^(4k + t): group k's nibble added in place
    const int WK = k == 0 ? (int)0xf8fcfeffu : (int)0x80c0e0f0u;  // (-1, -2, -4, -8), (-16, .., -128)
    const uint32_t bp = __builtin_amdgcn_perm(dp[1], dp[0], 0x0b0a0908u), bs = __builtin_amdgcn_perm(ds[1], ds[0], 0x0b0a0908u);
    cw = (uint32_t)__builtin_amdgcn_sdot4((int)bp, WK, (int)cw, false);
    sw = (uint32_t)__builtin_amdgcn_sdot4((int)bs, WK, (int)sw, false);
  }
  // the lane's 4K bits into 32-bit words of 8 / K lanes (outside the frame:
  // lanes past the last column group of an edge strip)
  constexpr int LPW = StripGeom<K>::lanes_per_word;
  const int sh = 4 * K * (w.lane & (LPW - 1));
  cw = !EDGE || w.inside ? cw << sh : 0u;
  sw = !EDGE || w.inside ? sw << sh : 0u;
  cw |= dpp_row_shr(cw, 1);
  sw |= dpp_row_shr(sw, 1);
  cw |= dpp_row_shr(cw, 2);
  sw |= dpp_row_shr(sw, 2);
  if (LPW == 8) {
    cw |= dpp_row_shr(cw, 4);
    sw |= dpp_row_shr(sw, 4);
  }
  if (w.store_lane) {
    const uint32_t o = 4u * ((uint32_t)n * (uint32_t)w.WW + (uint32_t)(w.lane / LPW));  // byte offset
    *(uint32_t*)((char*)w.cb + o) = cw;
    *(uint32_t*)((char*)w.sbp + o) = sw;
  }
}
// rows 0 .. H+2 in triples (row i in slot i % 3): the first two triples and
// the last ones with the row rules, the triples between without
template <int K, bool EDGE>
__device__ __forceinline__ void strip_walk(StripWave<K>& w, StripRegs<K>& R) {
  const int rows = w.H + 3;
  int i = 0;
#pragma unroll 1
  for (; i < 6 && i < rows; i += 3) {
    strip_step<K, 0, true, EDGE>(w, R, i);
    if (i + 1 < rows) strip_step<K, 1, true, EDGE>(w, R, i + 1);
    if (i + 2 < rows) strip_step<K, 2, true, EDGE>(w, R, i + 2);
  }
#pragma unroll 1
  for (; i + 2 < w.H; i += 3) {
    strip_step<K, 0, false, EDGE>(w, R, i);
    strip_step<K, 1, false, EDGE>(w, R, i + 1);
    strip_step<K, 2, false, EDGE>(w, R, i + 2);
  }
#pragma unroll 1
  for (; i < rows; i += 3) {
    strip_step<K, 0, true, EDGE>(w, R, i);
    if (i + 1 < rows) strip_step<K, 1, true, EDGE>(w, R, i + 1);
    if (i + 2 < rows) strip_step<K, 2, true, EDGE>(w, R, i + 2);
  }
}
// one wave per (frame, strip); needs W % (4K) == 0, W >= 8K, H >= 3.
// cat (W % 32 == 0, round 6): the strips tile the batch's frames laid side by
// side -- strip s covers columns [s cols, (s + 1) cols) of that n W-column
// band, so a strip may hold the end of one frame and the start of the next
// (frame boundaries fall on 32-column words, so every output word belongs to
// one frame; a lane takes its frame's rows, the border rules apply per lane
// at each frame's own edges, and DPP neighbours across a boundary are never
// read). ceil(n W / cols) waves instead of n ceil(W / cols): at 1280 columns
// and 480-column strips 2.67 instead of 3 waves per frame, the partial third
// strip's idle lanes gone.
template <int K>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(K == 1 ? 8 : MK_STRIP2_WAVES))) void k_canny_strip(const FrameDesc* __restrict__ frames, int low, int high,
                                                     uint32_t* __restrict__ cbits, uint32_t* __restrict__ sbits,
                                                     size_t bstride, int nstrip, int nwaves, int cat, int nframes) {
  // the wave index is wave-uniform: frame fields and row conditions stay scalar
  const int wv = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
  if (wv >= nwaves) return;
  StripWave<K> w;
  w.lane = threadIdx.x & 63;
  constexpr int G = 4 * K;  // columns per lane
  constexpr int LPW = StripGeom<K>::lanes_per_word;
  const int W = frames[0].w;  // one size per batch
  w.H = frames[0].h;
  w.WW = bits::words(W);
  int f, base, c0;
  bool edge_strip;
  if (cat) {
    const int vbase = wv * StripGeom<K>::cols;                        // the strip's first column in the band
    const int vc = w.lane == 63 ? vbase - G : vbase + G * w.lane;     // this lane's
    const int fl = vc < 0 ? 0 : vc / W;
    f = fl < nframes ? fl : nframes - 1;
    c0 = vc - f * W;                                                  // frame-local (outside [0, W) past the band)
    base = c0 - G * w.lane;                                           // for the store-lane test below (lanes < 60)
    edge_strip = true;
  } else {
    f = wv / nstrip;
    const int sidx = wv - f * nstrip;
    base = sidx * StripGeom<K>::cols;
    c0 = w.lane == 63 ? base - G : base + G * w.lane;
    edge_strip = sidx == 0 || sidx == nstrip - 1;
  }
  const int lc = c0 < 0 ? 0 : (c0 > W - G ? W - G : c0);           // loads stay inside the row
  w.left_edge = c0 == 0;                                           // columns -1.. come from the border rules
  w.right_edge = c0 == W - G;
  w.inside = c0 >= 0 && c0 <= W - G;
  if (cat) edge_strip = __builtin_amdgcn_ballot_w64(w.left_edge || w.right_edge || !w.inside) != 0;
  const int lowc = low < -1 ? -1 : (low > 32767 ? 32767 : low);
  const int highc = high < -1 ? -1 : (high > 32767 ? 32767 : high);
  w.LOW = s16x2{(short)lowc, (short)lowc};
  w.HIGH = s16x2{(short)highc, (short)highc};
  {
    constexpr int TG22 = (int)(0.4142135623730950488016887242097 * (1 << 15) + 0.5);
    w.KH = -2 * TG22;
    w.KV = -(2 * TG22 + (1 << 17));
    w.TWO = 0x00020002u;
    asm volatile("" : "+s"(w.TWO));
  }
  w.rstep = (uint32_t)W * 3u;
  if (cat) {
    // per lane: its frame's pixels and planes (at most two frames per wave)
    w.bgr = frames[f].bgr;
    w.loff = (uint32_t)lc * 3u;
    const size_t wo = (size_t)f * bstride + (size_t)((c0 < 0 ? 0 : c0) >> 5) - (size_t)(w.lane / LPW);
    w.cb = cbits + wo;
    w.sbp = sbits + wo;
    w.store_lane = (w.lane & (LPW - 1)) == LPW - 1 && w.lane < StripGeom<K>::out_lanes && w.inside;
  } else {
    w.bgr = frames[f].bgr;
    w.loff = (uint32_t)lc * 3u;
    w.cb = cbits + (size_t)f * bstride + (size_t)(base >> 5);
    w.sbp = sbits + (size_t)f * bstride + (size_t)(base >> 5);
    w.store_lane = (w.lane & (LPW - 1)) == LPW - 1 && w.lane < StripGeom<K>::out_lanes &&
                   base + G * (w.lane & ~(LPW - 1)) < W;
  }
  StripRegs<K> R = {};
#pragma unroll
  for (int p = 0; p < strip_pf<K>(); p++) strip_load_to(w, p < w.H ? p : w.H - 1, w.rows[p]);
  if (edge_strip) strip_walk<K, true>(w, R);
  else strip_walk<K, false>(w, R);
}

// ------------------------------------------------ hysteresis: run CCL
// Runs = maximal spans of candidates in a row, numbered in raster order per
// frame (k_run_scan gives the row bases); 8-connected unions between
// consecutive rows, first inside 32-row bands in LDS, then across the band
// seams on the global labels (the contour CCL's two-level scheme); roots are
// a component's smallest run id. Run extents (packed u32), labels (int32) and
// flags (u8) live in planes sized for one run per pixel.
// run starts / ends of word w of a row (bits past W are zero)
__device__ inline uint32_t hb_starts(const uint32_t* row, int w) {
  const uint32_t cur = row[w], prv = w > 0 ? row[w - 1] : 0u;
  return cur & ~((cur << 1) | (prv >> 31));
}
__device__ inline uint32_t hb_ends(const uint32_t* row, int w, int WW) {
  const uint32_t cur = row[w], nxt = w + 1 < WW ? row[w + 1] : 0u;
  return cur & ~((cur >> 1) | (nxt << 31));
}
// mask of bits [a, b] of word w
__device__ inline uint32_t span_mask(int w, int a, int b) {
  const uint32_t lo = w == (a >> 5) ? (0xffffffffu << (a & 31)) : 0xffffffffu;
  const uint32_t hi = w == (b >> 5) ? (0xffffffffu >> (31 - (b & 31))) : 0xffffffffu;
  return lo & hi;
}
// first run k of [0, n) whose end reaches v, n if none (packed extents)
__device__ inline int hx_first_end(const uint32_t* x, int n, int v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((int)(x[mid] >> 16) >= v) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}
// unions of row y's runs [by, by + ny) with row y-1's [bp, bp + np), 8-connected
template <class UF>
__device__ inline void hyst_row_union(const uint32_t* x, int bp, int np, int by, int ny, int lane, const UF& uni) {
  for (int j = lane; j < ny; j += 64) {
    const int a = x[by + j] & 0xffff, b = x[by + j] >> 16;
    for (int k = hx_first_end(x + bp, np, a - 1); k < np && (int)(x[bp + k] & 0xffff) <= b + 1; k++)
      uni(by + j, bp + k);
  }
}
// does the run [a, b] of srow hold a strong pixel
__device__ inline bool run_strong(const uint32_t* srow, int a, int b) {
  for (int w = a >> 5; w <= (b >> 5); w++)
    if (srow[w] & span_mask(w, a, b)) return true;
  return false;
}

struct HystRuns {  // per-frame planes (frame f at + f * stride)
  uint32_t* x;     // run extents: start | end << 16 (seam rows, list B runs; every run of a dense band)
  int32_t* lab;    // run labels
  uint8_t* flag;   // per root: == epoch: the global component holds a strong pixel (denser bands: bits 0 / 1
                   // = strong / reaches a seam, per band root, values <= 3)
  int32_t* rowb;   // per row: its first run's index inside the band; [H + 1], [H + 2] = |A|, |B|;
                   // [H + 3 + b] = runs of band b
  size_t x_stride, lab_stride, flag_stride, rstride, half;
  int bs;          // run ids per band: run i of band b is b * bs + i (bs = band rows x ceil(W / 2))
  FrameState* st;  // diagnostics only (MK_HYST_TICKS: phase ends of one band per frame into st[f].ticks)
  int epoch;       // this call's mark value, 4..255: a root is marked when its flag byte equals it, so the
                   // band kernel never clears the flags of its roots (a scattered byte per root); the host
                   // clears the plane when the value wraps
};

// Per band of HB_ROWS rows: unions in LDS (labels = band roots, written to
// the global labels for the seams), then the band's edge words: the runs of
// band components holding a strong pixel are edges whatever the rest of the
// frame holds; a band component without one that reaches the band's first or
// last row (inside the frame) may still meet a strong pixel across a seam, so
// its runs go to list B; the roots of strong components that reach them go to
// list A. Lists live in the label plane above the labels (A from hr.half up,
// B from the top of the plane down; |A| + |B| <= runs <= half). Denser bands
// (more than HB_CAP runs) take the same steps on the global labels.
#ifndef MK_HB_ROWS
#define MK_HB_ROWS 32
#endif
#ifndef MK_HB_THREADS
#define MK_HB_THREADS 512
#endif
constexpr int HB_ROWS = MK_HB_ROWS, HB_CAP = 4096, HB_THREADS = MK_HB_THREADS, HB_WAVES = HB_THREADS / 64;
// global id of row y's first run and the row's run count
__device__ inline void hr_row(const int32_t* rb, int H, int bs, int y, int& g, int& cnt) {
  const int b = y / HB_ROWS, s = rb[y];
  const int e = (y + 1 < H && (y + 1) % HB_ROWS != 0) ? rb[y + 1] : rb[H + 3 + b];
  g = b * bs + s;
  cnt = e - s;
}
// band-local union-find on 16-bit labels in LDS (roots = smallest id); the
// link is a 32-bit CAS on the dword holding the 16-bit slot
// (bits 12..13 of a root's slot hold its band flags once the unions are done:
// ids are < HB_CAP = 4096, so the low 12 bits are the link)
__device__ inline int hb_find(const uint16_t* L, int x) {
  int p;
  while ((p = L[x] & 0xfff) != x) x = p;
  return x;
}
__device__ inline void hb_union(uint16_t* L, int a, int b) {
  while (true) {
    a = hb_find(L, a);
    b = hb_find(L, b);
    if (a == b) return;
    if (a < b) { const int tt = a; a = b; b = tt; }
    uint32_t* wp = (uint32_t*)(L + (a & ~1));
    const int sh = (a & 1) * 16;
    const uint32_t old = *(volatile uint32_t*)wp;
    if (((old >> sh) & 0xffffu) != (uint32_t)a) continue;  // a was linked meanwhile: find again
    const uint32_t nw = (old & ~(0xffffu << sh)) | ((uint32_t)b << sh);
    if (atomicCAS(wp, old, nw) == old) return;
  }
}
// wave-aggregated list append (one atomic per wave and call; every active lane calls it)
__device__ inline void hyst_push(int32_t* list, int32_t* count, int v, bool push, bool down, size_t top) {
  const uint64_t m = __ballot(push);
  if (!m) return;
  const int lane = threadIdx.x & 63, leader = __ffsll((unsigned long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(count, __popcll(m));
  base = __shfl(base, leader);
  if (push) {
    const int k = base + __popcll(m & ((1ull << lane) - 1));
    list[down ? top - 1 - k : k] = v;
  }
}
// run extents of a band row (candidate words cw in LDS) from local index o:
// its k-th start bit and k-th end bit bound run k (two wave scans, no search)
template <class P>
__device__ inline void hb_emit_runs(const uint32_t* cw, int WW, P* X16, int o, int lane) {
  int bs = o, be = o;
  for (int w0 = 0; w0 < WW; w0 += 64) {
    const int w = w0 + lane;
    uint32_t S = w < WW ? hb_starts(cw, w) : 0u;
    uint32_t E = w < WW ? hb_ends(cw, w, WW) : 0u;
    const int cs = __popc(S), ce = __popc(E);
    const int is = wave_incl_scan(cs, lane), ie = wave_incl_scan(ce, lane);
    for (int os = bs + is - cs; S; S &= S - 1, os++) X16[2 * os] = (uint16_t)(32 * w + __ffs(S) - 1);
    for (int oe = be + ie - ce; E; E &= E - 1, oe++) X16[2 * oe + 1] = (uint16_t)(32 * w + __ffs(E) - 1);
    bs += __builtin_amdgcn_readlane(is, 63);
    be += __builtin_amdgcn_readlane(ie, 63);
  }
}
// One block per band: the band's candidate and strong words into LDS, its
// runs counted and numbered (band-local ids: no frame-wide scan), unions,
// classes, edge words, lists. Global traffic: the two bit planes' words once,
// the edge words once, labels / extents of the rows and runs later kernels read.
__global__ __launch_bounds__(HB_THREADS) void k_hyst_band(const uint32_t* __restrict__ cbits,
                                                          const uint32_t* __restrict__ sbits, size_t bstride, HystRuns hr,
                                                          uint32_t* __restrict__ ebits, int W, int H) {
  __shared__ uint16_t Ll[HB_CAP];
  __shared__ uint32_t Xl[HB_CAP];
  __shared__ int32_t rbl[HB_ROWS + 1];
  extern __shared__ uint32_t Ew[];     // the band's edge words (rows x WW), then its strong words, then its candidates
  const int f = blockIdx.y, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int band = blockIdx.x, y0 = band * HB_ROWS;
  if (y0 >= H) return;
  const int y1 = min(y0 + HB_ROWS, H), WW = bits::words(W), nr = y1 - y0;
  int32_t* rb = hr.rowb + (size_t)f * hr.rstride;
  int32_t* cnt = rb + H + 1;
  uint32_t* X = hr.x + (size_t)f * hr.x_stride;
  int32_t* L = hr.lab + (size_t)f * hr.lab_stride;
  int32_t* lists = L + hr.half;
  const size_t top = hr.lab_stride - hr.half;
  uint8_t* fl = hr.flag + (size_t)f * hr.flag_stride;
  uint32_t* eb = ebits + (size_t)f * bstride + (size_t)y0 * WW;
  const int g0 = band * hr.bs;
  uint32_t* Sw = Ew + nr * WW;
  uint32_t* Cw = Sw + nr * WW;
  const uint32_t* sb = sbits + (size_t)f * bstride + (size_t)y0 * WW;
  const uint32_t* cb = cbits + (size_t)f * bstride + (size_t)y0 * WW;
#ifdef MK_HYST_TICKS  // diagnostics: phase ends of the middle band's block (10 ns), tools/hyst_ticks.py
  const uint64_t tk0 = wall_clock64();
#define MK_HTICK(k) \
  if (t == 0 && band == (H / HB_ROWS) / 2) hr.st[f].ticks[k] = (int32_t)(wall_clock64() - tk0);
#else
#define MK_HTICK(k)
#endif
  for (int i = t; i < nr * WW; i += HB_THREADS) {
    Ew[i] = 0u;
    Sw[i] = sb[i];
    Cw[i] = cb[i];
  }
  __syncthreads();
  MK_HTICK(0);
  // runs per row (wave per row), then the band's row bases
  for (int q = wave; q < nr; q += HB_WAVES) {
    int c = 0;
    for (int w = lane; w < WW; w += 64) c += __popc(hb_starts(Cw + q * WW, w));
    c = wave_sum(c);
    if (lane == 0) rbl[q + 1] = c;
  }
  __syncthreads();
  if (t < 64) {
    const int v = t < nr ? rbl[t + 1] : 0;
    const int s = wave_incl_scan(v, t);
    if (t < nr) {
      rbl[t + 1] = s;
      rb[y0 + t] = s - v;
    }
    if (t == 0) rbl[0] = 0;
    if (t == nr - 1) rb[H + 3 + band] = s;
  }
  __syncthreads();
  MK_HTICK(1);
  const int n = rbl[nr];
  // a row whose components may continue past the band: its first / last row inside the frame
  const auto edge_row = [&](int q) { return (q == 0 && y0 > 0) || (q == nr - 1 && y1 < H); };
  if (n > HB_CAP) {
    for (int q = wave; q < nr; q += HB_WAVES) hb_emit_runs(Cw + q * WW, WW, (uint16_t*)(X + g0), rbl[q], lane);
    for (int i = t; i < n; i += HB_THREADS) {
      L[g0 + i] = g0 + i;
      fl[g0 + i] = 0;
    }
    __syncthreads();
    const auto uni = [L](int a, int b) { uf_union_c(L, a, b); };
    for (int q = 1 + wave; q < nr; q += HB_WAVES)
      hyst_row_union(X, g0 + rbl[q - 1], rbl[q] - rbl[q - 1], g0 + rbl[q], rbl[q + 1] - rbl[q], lane, uni);
    __syncthreads();
    for (int q = wave; q < nr; q += HB_WAVES)
      for (int j = g0 + rbl[q] + lane; j < g0 + rbl[q + 1]; j += 64) {
        const int root = uf_find_c(L, j);
        const uint32_t b = (run_strong(Sw + q * WW, X[j] & 0xffff, X[j] >> 16) ? 1u : 0u) | (edge_row(q) ? 2u : 0u);
        if (b) atomicOr((uint32_t*)(fl + (root & ~3)), b << (8 * (root & 3)));
      }
    __syncthreads();
    for (int q = wave; q < nr; q += HB_WAVES)
      for (int j = g0 + rbl[q] + lane; j < g0 + rbl[q + 1]; j += 64) {
        const int root = uf_find_c(L, j);
        const int fb = fl[root] & 3;
        if (fb & 1) {
          const int a = X[j] & 0xffff, b = X[j] >> 16;
          for (int w = a >> 5; w <= (b >> 5); w++) atomicOr(&Ew[q * WW + w], span_mask(w, a, b));
        }
        hyst_push(lists, cnt + 1, j | (q << 24), fb == 2, true, top);  // list B: run id | its band row << 24
        hyst_push(lists, cnt, j, root == j && fb == 3, false, top);
      }
    __syncthreads();
    for (int i = t; i < nr * WW; i += HB_THREADS) eb[i] = Ew[i];
    return;
  }
  for (int q = wave; q < nr; q += HB_WAVES) hb_emit_runs(Cw + q * WW, WW, (uint16_t*)Xl, rbl[q], lane);
  for (int i = t; i < n; i += HB_THREADS) Ll[i] = (uint16_t)i;
  __syncthreads();
  MK_HTICK(2);
  uint16_t* Li = Ll;
  const auto uni = [Li](int a, int b) { hb_union(Li, a, b); };
  for (int q = 1 + wave; q < nr; q += HB_WAVES)
    hyst_row_union(Xl, rbl[q - 1], rbl[q] - rbl[q - 1], rbl[q], rbl[q + 1] - rbl[q], lane, uni);
  __syncthreads();
  MK_HTICK(3);
  for (int q = wave; q < nr; q += HB_WAVES) {
    for (int j = rbl[q] + lane; j < rbl[q + 1]; j += 64) {
      const int root = hb_find(Ll, j);
      const uint32_t b = (run_strong(Sw + q * WW, Xl[j] & 0xffff, Xl[j] >> 16) ? 1u : 0u) | (edge_row(q) ? 2u : 0u);
      // the band flags go to bits 12..13 of the root's own slot (its link
      // bits stay == root, so concurrent finds still stop there); a root
      // never stores its own slot, which would drop flags already set
      if (root != j) Ll[j] = (uint16_t)root;
      if (b) atomicOr((uint32_t*)(Ll + (root & ~1)), (b << 12) << (16 * (root & 1)));
    }
  }
  __syncthreads();
  MK_HTICK(4);
  for (int q = wave; q < nr; q += HB_WAVES) {
    for (int j = rbl[q] + lane; j < rbl[q + 1]; j += 64) {
      const int root = Ll[j] & 0xfff;
      const int fb = (Ll[root] >> 12) & 3;
      // global labels / extents only where a later kernel looks: the band's
      // seam rows (its first / last row where another band lies beyond:
      // k_hyst_seam's unions), list B runs (fb == 2: k_hyst_fix) and the roots
      // of components that reach a seam (finds end there; their flag byte is
      // what k_hyst_mark / k_hyst_fix use) -- no later kernel finds its way to
      // the other roots
      const bool seam_row = edge_row(q);
      if (seam_row || fb == 2 || (root == j && (fb & 2))) L[g0 + j] = g0 + root;
      if (seam_row || fb == 2) X[g0 + j] = Xl[j];
      if (fb & 1) {
        const int a = Xl[j] & 0xffff, b = Xl[j] >> 16;
        for (int w = a >> 5; w <= (b >> 5); w++) atomicOr(&Ew[q * WW + w], span_mask(w, a, b));
      }
      hyst_push(lists, cnt + 1, (g0 + j) | (q << 24), fb == 2, true, top);
      hyst_push(lists, cnt, g0 + j, root == j && fb == 3, false, top);
    }
  }
  __syncthreads();
  MK_HTICK(5);
  for (int i = t; i < nr * WW; i += HB_THREADS) eb[i] = Ew[i];
}

// one wave per band boundary row y = k * HB_ROWS against row y-1
__global__ __launch_bounds__(256) void k_hyst_seam(HystRuns hr, int H) {
  const int f = blockIdx.y, lane = threadIdx.x & 63;
  const int y = (blockIdx.x * 4 + (threadIdx.x >> 6) + 1) * HB_ROWS;
  if (y >= H) return;
  const int32_t* rb = hr.rowb + (size_t)f * hr.rstride;
  int32_t* L = hr.lab + (size_t)f * hr.lab_stride;
  const auto uni = [L](int a, int b) { uf_union_c(L, a, b); };
  int gp, np, gy, ny;
  hr_row(rb, H, hr.bs, y - 1, gp, np);
  hr_row(rb, H, hr.bs, y, gy, ny);
  hyst_row_union(hr.x + (size_t)f * hr.x_stride, gp, np, gy, ny, lane, uni);
}

// list A: strong band components reaching a seam mark their global root (bit 2)
__global__ __launch_bounds__(256) void k_hyst_mark(HystRuns hr, int H) {
  const int f = blockIdx.y;
  const int n = hr.rowb[(size_t)f * hr.rstride + H + 1];
  int32_t* L = hr.lab + (size_t)f * hr.lab_stride;
  const int32_t* A = L + hr.half;
  uint8_t* fl = hr.flag + (size_t)f * hr.flag_stride;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int root = uf_find_c(L, A[i]);
    if (fl[root] != (uint8_t)hr.epoch) fl[root] = (uint8_t)hr.epoch;  // byte stores of one value: races are benign
  }
}

// list B: runs of weak band components whose global root is marked become edges
__global__ __launch_bounds__(256) void k_hyst_fix(HystRuns hr, uint32_t* __restrict__ ebits, size_t bstride, int W,
                                                  int H) {
  const int f = blockIdx.y;
  const int32_t* rb = hr.rowb + (size_t)f * hr.rstride;
  const int n = rb[H + 2];
  int32_t* L = hr.lab + (size_t)f * hr.lab_stride;
  const int32_t* Bl = L + hr.lab_stride - 1;  // B[i] = Bl[-i]
  const uint8_t* fl = hr.flag + (size_t)f * hr.flag_stride;
  const uint32_t* X = hr.x + (size_t)f * hr.x_stride;
  const int WW = bits::words(W);
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int e = Bl[-i], j = e & 0xffffff;  // run id | band row << 24 (ids < 2^24: bands x bs)
    if (fl[uf_find_c(L, j)] != (uint8_t)hr.epoch) continue;
    const int y = (j / hr.bs) * HB_ROWS + (e >> 24);
    const int a = X[j] & 0xffff, b = X[j] >> 16;
    uint32_t* eb = ebits + (size_t)f * bstride + (size_t)y * WW;
    for (int w = a >> 5; w <= (b >> 5); w++) atomicOr(&eb[w], span_mask(w, a, b));
  }
}

// ================================= hysteresis as bit-parallel reconstruction
// cv::Canny's hysteresis (the stack walk from every strong pixel over the
// 8-connected candidates, QuadDetection.h:212 / HypothesisEvaluation.h:327)
// marks exactly the candidate components that hold a strong pixel: the
// morphological reconstruction of the candidate plane C from the strong plane
// S, the least E with E = (S ∪ dilate8(E)) ∩ C. No labels: one block per frame,
// wave w owns rows [w HR_ROWS, (w + 1) HR_ROWS) with its band's C and E words
// in VGPRs (lane = 32-pixel word column, W <= 2016) and reaches the fixpoint
// with row sweeps:
//   row fill   every candidate run of a row that holds a seed, as two
//              additions along the row: c + s carries from each run's lowest
//              seed to the run's end (rightward), and the same on bit-reversed
//              words in reversed lane order (leftward); the carries between
//              words are one 64-bit scalar addition over the lanes' generate /
//              propagate ballots
//   sweeps     seed(y) = E(y) ∪ (dilate3(E(y ∓ 1)) ∩ C(y)), then the row fill,
//              down and up the band alternately until a sweep adds nothing
//              (each sweep carries a change any distance in its direction)
//   seams      the bands trade their first / last rows through LDS; a band
//              whose edge row gains seeds sweeps again; the block stops when
//              no band gains any (__syncthreads_or)
// C and S are read once and E written once: 3 W H / 8 bytes per frame.
#ifndef MK_HR_ROWS
#define MK_HR_ROWS 45
#endif
constexpr int HR_ROWS = MK_HR_ROWS, HR_MAXW = 16;  // rows per wave; waves per block (frames up to 720 rows)
// 8-neighbour row dilation of a row's words (lanes past the row hold 0; lane
// 0's left and lane 63's right neighbour wrap to lanes past the row)
__device__ inline uint32_t hr_dil3(uint32_t e) {
  return e | __builtin_amdgcn_alignbit(e, dpp_from_left(e), 31) | __builtin_amdgcn_alignbit(dpp_from_right(e), e, 1);
}
// carry into lane i (bit i) of a word-wise addition whose lanes generate G / propagate P
__device__ inline uint64_t hr_carries(uint64_t G, uint64_t P) {
  const uint64_t A = G | P;
  return (A + G) ^ A ^ G;
}
// word-wise addition across the row's lanes: carry out of each lane's c + s as
// a lane mask (v_add_co's carry, straight into an SGPR pair), and t + the
// carry into the lane (v_addc_co's carry-in operand is the lane mask k)
__device__ inline uint32_t hr_add(uint32_t c, uint32_t s, uint64_t& g) {
  uint32_t t;
  asm("v_add_co_u32 %0, %1, %2, %3" : "=v"(t), "=s"(g) : "v"(c), "v"(s));
  return t;
}
__device__ inline uint32_t hr_addc(uint32_t t, uint64_t k) {
  uint32_t u;
  uint64_t co;
  asm("v_addc_co_u32 %0, %1, %2, 0, %3" : "=v"(u), "=s"(co) : "v"(t), "s"(k));
  return u;
}
// every candidate run of the row (this lane's word c) that holds a seed bit of s (s ⊆ c)
__device__ inline uint32_t hr_fill(uint32_t c, uint32_t s) {
  uint64_t gr, gl;
  const uint32_t t = hr_add(c, s, gr);  // rightward: each run from its lowest seed to its end
  const uint32_t rt = s | ((hr_addc(t, hr_carries(gr, __ballot(t == 0xffffffffu))) ^ c ^ s) & c);
  const uint32_t cr = __builtin_bitreverse32(c), sr = __builtin_bitreverse32(s);
  const uint32_t u = hr_add(cr, sr, gl);  // leftward: the same on the reversed row (carries from lane i + 1 into lane i)
  const uint64_t kl = __builtin_bitreverse64(
      hr_carries(__builtin_bitreverse64(gl), __builtin_bitreverse64(__ballot(u == 0xffffffffu))));
  const uint32_t lf = __builtin_bitreverse32(sr | ((hr_addc(u, kl) ^ cr ^ sr) & cr));
  return rt | lf;
}
__global__ __launch_bounds__(64 * HR_MAXW) void k_hyst_rec(const uint32_t* __restrict__ cbits,
                                                           const uint32_t* __restrict__ sbits,
                                                           uint32_t* __restrict__ ebits, size_t bstride, int W,
                                                           int H, FrameState* st) {
  __shared__ uint32_t xt[HR_MAXW][64], xb[HR_MAXW][64];  // every band's first / last row of E
  extern __shared__ uint32_t hr_c[];                     // the bands' candidate words (waves x HR_ROWS x WW)
  const int f = blockIdx.x, lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), nwv = blockDim.x >> 6;
  const int WW = bits::words(W);
  const int y0 = wave * HR_ROWS, nr = min(HR_ROWS, H - y0);  // nr >= 1: nwv = ceil(H / HR_ROWS)
  const bool on = lane < WW;
  const uint32_t vm = on ? bits::valid(lane, W) : 0u;
  // band bases are wave-uniform (scalar); the lane's word offset is 32-bit
  const size_t band = (size_t)f * bstride + (size_t)y0 * WW;
  const gu32* cb = gwords(cbits + band);
  const gu32* sb = gwords(sbits + band);
  // C goes to LDS, E stays in VGPRs. The band's LDS slice holds its WW word
  // columns HR_ROWS words apart (lane-major: the rows of a lane are one base
  // VGPR plus immediate offsets, and the odd pitch keeps the lanes on distinct
  // banks); rows past the frame hold 0, so the sweeps leave their E 0 and the
  // up sweep reaches a short band's last row with the zero row below it. Every
  // global load is issued (rows past the frame re-read its last row, lanes past
  // the row word 0; the row test and vm zero the extra words), and lanes past
  // the row read lane 0's LDS column and drop it (onm).
  const int lw = on ? lane : 0;
  const uint32_t onm = on ? ~0u : 0u;
  uint32_t* cl = hr_c + (y0 * WW + lw * HR_ROWS);
  uint32_t e[HR_ROWS];
#pragma unroll
  for (int r = 0; r < HR_ROWS; r++) {
    const int o = min(r, nr - 1) * WW + lw;
    const uint32_t cw = r < nr ? cb[o] & vm : 0u;
    e[r] = sb[o] & cw;
    if (on) cl[r] = cw;
  }
  const auto c = [&](int r) -> uint32_t { return cl[r] & onm; };
  uint32_t top = 0u, bot = 0u;  // the rows of E above / below the band (the neighbours' edge rows)
  // Sweep windows: a down sweep re-examines row r only if the row above it
  // (row -1: top) changed since r was last made consistent from above, i.e.
  // it starts below the first row the previous sweep changed, runs through the
  // row after its last one, and goes on past it while rows keep changing; an
  // up sweep likewise from below (row HR_ROWS: bot). [clo, chi] are the rows
  // the previous sweep changed; a sweep that changes nothing ends the settle.
  // The very first sweep fills every seeded row (S is not run-closed yet) and
  // the up sweep after it examines every row.
  bool go = true, down = true, all = true, pend_bot = false;
  int clo = -1, chi = HR_ROWS - 1;
#ifdef MK_HYST_TICKS  // diagnostics (tools/hyst_ticks.py rec): seam rounds, sweeps, filled rows, phase ticks
  __shared__ int hs_cnt[3];
  const uint64_t tk0 = wall_clock64();
  int n_sweeps = 0, n_fills = 0, n_rounds = 0, t_settle = 0;
  if (threadIdx.x < 3) hs_cnt[threadIdx.x] = 0;
#endif
  while (true) {
    while (go) {
      asm volatile("" ::: "memory");  // the LDS reads of C stay in the sweeps (hoisted, they would take the VGPRs back)
      int nlo = HR_ROWS + 1, nhi = -2;  // rows this sweep changes
      bool live = false;                // the previous row of this sweep changed
      if (down) {
        const int from = clo + 1, upto = chi + 1;
#pragma unroll
        for (int r = 0; r < HR_ROWS; r++) {
          if (r < from) continue;
          const uint32_t cw = c(r);
          if (r > upto && !live) break;
          const uint32_t sd = e[r] | (hr_dil3(r == 0 ? top : e[r - 1]) & cw);
          live = false;
          if (__ballot(all ? sd != 0u : sd != e[r])) {
#ifdef MK_HYST_TICKS
            n_fills++;
#endif
            const uint32_t n = hr_fill(cw, sd);
            if (__ballot(n != e[r])) {
              live = true;
              nlo = min(nlo, r);
              nhi = r;
            }
            e[r] = n;
          }
        }
      } else {
        const int from = chi - 1, upto = clo - 1;
#pragma unroll
        for (int r = HR_ROWS - 1; r >= 0; r--) {
          if (r > from) continue;
          const uint32_t cw = c(r);
          if (r < upto && !live) break;
          const uint32_t sd = e[r] | (hr_dil3(r == HR_ROWS - 1 ? bot : e[r + 1]) & cw);
          live = false;
          if (__ballot(sd != e[r])) {
#ifdef MK_HYST_TICKS
            n_fills++;
#endif
            const uint32_t n = hr_fill(cw, sd);
            if (__ballot(n != e[r])) {
              live = true;
              nhi = max(nhi, r);
              nlo = r;
            }
            e[r] = n;
          }
        }
      }
#ifdef MK_HYST_TICKS
      n_sweeps++;
#endif
      if (all) {
        all = false;
        clo = 0;
        chi = HR_ROWS;
      } else {
        clo = nlo;
        chi = nhi;
        if (pend_bot) {  // the up sweep after a seam round's first (down) sweep also takes the bottom seeds
          pend_bot = false;
          if (clo > chi) clo = HR_ROWS;
          chi = HR_ROWS;
        }
      }
      go = clo <= chi;
      down = !down;
    }
#ifdef MK_HYST_TICKS
    if (n_rounds++ == 0) t_settle = (int)(wall_clock64() - tk0);
#endif
    // seams: a band whose first / last row gains seeds from its neighbour sweeps again
    xt[wave][lane] = e[0];
    xb[wave][lane] = e[HR_ROWS - 1];  // read only by the next band: this band is full then
    __syncthreads();
    top = wave > 0 ? xb[wave - 1][lane] : 0u;
    bot = wave + 1 < nwv ? xt[wave + 1][lane] : 0u;
    const bool nt = __ballot((hr_dil3(top) & c(0) & ~e[0]) != 0u) != 0;
    const bool nb = __ballot((hr_dil3(bot) & c(HR_ROWS - 1) & ~e[HR_ROWS - 1]) != 0u) != 0;
    go = nt || nb;
    down = nt;
    pend_bot = nt && nb;
    clo = nt ? -1 : HR_ROWS;
    chi = nt ? -1 : HR_ROWS;
    if (!__syncthreads_or(go)) break;
  }
#ifdef MK_HYST_TICKS
  if (lane == 0) {
    atomicMax(&hs_cnt[0], n_sweeps);
    atomicAdd(&hs_cnt[1], n_sweeps);
    atomicAdd(&hs_cnt[2], n_fills);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    st[f].ticks[0] = n_rounds;         // seam rounds (1: the first settle sufficed)
    st[f].ticks[1] = hs_cnt[0];        // most sweeps of one band
    st[f].ticks[2] = hs_cnt[1];        // sweeps of all bands
    st[f].ticks[3] = hs_cnt[2];        // row fills of all bands
    st[f].ticks[4] = t_settle;         // first settle (wave 0), 10 ns ticks
    st[f].ticks[5] = (int)(wall_clock64() - tk0);
  }
#endif
  // the store offsets are recomputed here rather than kept alive from the loads
  int lo = lane, nrs = nr;
  asm volatile("" : "+v"(lo), "+s"(nrs));
  uint32_t* eb = ebits + band;
#pragma unroll
  for (int r = 0; r < HR_ROWS; r++)
    if (lo < WW && r < nrs) eb[r * WW + lo] = e[r];
}

// mantis_hysteresis stage entry: class bytes (0 none, 1 weak candidate, 2
// strong) -> the candidate / strong bit planes (a strong byte is a candidate)
__global__ __launch_bounds__(256) void k_cls_to_bits(const uint8_t* __restrict__ cls, uint32_t* __restrict__ cb,
                                                     uint32_t* __restrict__ sb, int W, int H) {
  const int WW = bits::words(W);
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < WW * H; k += gridDim.x * blockDim.x) {
    const int y = k / WW, w = k - y * WW;
    uint32_t cw = 0, sw = 0;
    for (int b = 0; b < 32 && 32 * w + b < W; b++) {
      const uint8_t v = cls[(size_t)y * W + 32 * w + b];
      cw |= (uint32_t)(v != 0) << b;
      sw |= (uint32_t)(v == 2) << b;
    }
    cb[k] = cw;
    sb[k] = sw;
  }
}

// Padded detector binary as a row-aligned bit plane: (W+2) x (H+2) with the
// zero ring, WPW = ceil((W+2)/32) + 1 words per row (the spare word lets a
// 64-bit window at any x be read without a bounds test).
__device__ __host__ inline int dbits_wpw(int Wp) { return (Wp + 31) / 32 + 1; }
// ============================================================== morphology
// output rows per band: MB_BH when the three band buffers fit in LDS at the
// context's max width (<= 2496 px), else MB_BH_NARROW (bands at 1280 px:
// 3 x (112 + 2 x 29) rows x 40 words x 4 B = 82 KB, one per CU; measured
// 4.75 -> 3.34 ms per 4096 frames against 48 rows at 256 threads)
#ifndef MK_MB_BH
#define MK_MB_BH 112
#endif
#ifndef MK_MB_THREADS
#define MK_MB_THREADS 512
#endif
constexpr int MB_BH = MK_MB_BH, MB_BH_NARROW = 48;
constexpr int MB_THREADS = MK_MB_THREADS;
constexpr int MB_HALO = 29;   // mask chain reach: M0 2 + (3+3+4+4+5+5) + 3
struct RowRange {
  int lo, hi;  // absolute rows [lo, hi) valid in a buffer
  __device__ RowRange shrink(int r, int H) const { return {lo == 0 ? 0 : lo + r, hi == H ? H : hi - r}; }
};
// Work-item layout inside a band: work-item (w, g) owns word column w and the
// g-th of G contiguous row segments of each pass's output range, so the
// vertical window slides down its column in registers (one new row per output
// row) instead of re-reading 2r + 1 rows, and no index is divided per word.
struct MbLane {
  int w, g, G;
  __device__ bool active() const { return g < G; }
  __device__ void seg(RowRange rr, int& a, int& b) const {
    const int s = (rr.hi - rr.lo + G - 1) / G;
    a = rr.lo + g * s;
    b = min(rr.hi, a + s);
  }
};
// One separable rectangle pass (radius R; dilate or erode), horizontal and
// vertical fused: out(y) = OP_{|k|<=R, 0<=y+k<H} hword(in, y+k). src/dst hold
// absolute rows [y0, ...) at row pitch WW; dst row y goes to dst + (y - y0) * WW.
template <int R, bool DIL>
__device__ inline void mb_hv(const uint32_t* src, uint32_t* dst, RowRange out, int y0, int WW, int W, int H,
                             const MbLane& L) {
  if (!L.active()) return;
  int a, b;
  L.seg(out, a, b);
  if (a >= b) return;
  const uint32_t ident = DIL ? 0u : 0xffffffffu;
  const uint32_t vmask = bits::valid(L.w, W);
  uint32_t ring[2 * R + 1];
#pragma unroll
  for (int k = 0; k < 2 * R; k++) {
    const int yy = a - R + k;
    ring[k] = (yy >= 0 && yy < H) ? bits::hword(src + (yy - y0) * WW, L.w, W, R, DIL) : ident;
  }
  for (int y = a; y < b; y++) {
    const int yy = y + R;
    ring[2 * R] = yy < H ? bits::hword(src + (yy - y0) * WW, L.w, W, R, DIL) : ident;
    uint32_t acc = ring[0];
#pragma unroll
    for (int k = 1; k <= 2 * R; k++) acc = DIL ? (acc | ring[k]) : (acc & ring[k]);
    dst[(y - y0) * WW + L.w] = acc & vmask;
#pragma unroll
    for (int k = 0; k < 2 * R; k++) ring[k] = ring[k + 1];
  }
}

// Detector binary and cleanImageByEdge mask in one pass over the edge bit
// plane (mk_bits.h word semantics). A block owns a band of bh output rows of
// one frame and keeps the band plus a MB_HALO-row halo on each side in LDS
// (three row buffers), so the stages of the two chains never touch HBM between
// them: each stage recomputes the rows its successors still need (its valid
// range shrinks by its vertical reach, except at the image edge, where the
// clipped-window rules of mk_bits.h apply).
//   detector  QuadDetection.h:213-214: dilate 5x5 (iterations 2), erode 3x3
//             -> padded bit plane (zero ring) for the contour CCL
//   mask      HypothesisEvaluation.h:319-363: NG = NOT(gradient), M0 = edge |
//             border(NG), 3 x {dilate, erode}(3 + i), erode(3) -> mask bit plane
__global__ __launch_bounds__(MB_THREADS) void k_morph(const uint32_t* __restrict__ eb, uint32_t* __restrict__ dbits,
                                               uint32_t* __restrict__ mbits, int W, int H, size_t bstride,
                                               size_t dstride, int bh) {
  extern __shared__ uint32_t mb_lds[];
  const int f = blockIdx.y, t = threadIdx.x, nt = blockDim.x;
  const int WW = bits::words(W);
  const MbLane L{t % WW, t / WW, nt / WW};
  const int yb = blockIdx.x * bh, ye = min(H, yb + bh);
  const int y0 = max(0, yb - MB_HALO), y1 = min(H, ye + MB_HALO);
  const int rows = bh + 2 * MB_HALO;
  uint32_t* A = mb_lds;
  uint32_t* B = A + rows * WW;
  uint32_t* Cb = B + rows * WW;
  const uint32_t* E = eb + (size_t)f * bstride;
  for (int k = t; k < (y1 - y0) * WW; k += nt) A[k] = E[(size_t)y0 * WW + k];
  __syncthreads();
  const RowRange rr{y0, y1};
  const uint32_t vmask = bits::valid(L.w, W);
  // NG (reach 1): A -> Cb
  const RowRange rng = rr.shrink(1, H);
  if (L.active()) {
    int a, b;
    L.seg(rng, a, b);
    const uint32_t* base = A - (ptrdiff_t)y0 * WW;
    for (int y = a; y < b; y++) Cb[(y - y0) * WW + L.w] = bits::ngword(base, L.w, y, W, H);
  }
  __syncthreads();
  // M0 = edge | border(NG) (reach 2): (A, Cb) -> B
  const RowRange rm0 = rng.shrink(1, H);
  if (L.active()) {
    int a, b;
    L.seg(rm0, a, b);
    const int w = L.w;
    for (int y = a; y < b; y++) {
      const uint32_t* nr = Cb + (y - y0) * WW;
      const uint32_t ng = nr[w];
      const uint32_t ngl = w > 0 ? nr[w - 1] : 0u;
      const uint32_t ngr = w + 1 < WW ? nr[w + 1] : 0u;
      const uint32_t left = (ng << 1) | (ngl >> 31);   // ng(x - 1), 0 left of the image
      const uint32_t right = (ng >> 1) | (ngr << 31);  // ng(x + 1), 0 right of the image
      const uint32_t up = y > 0 ? nr[w - WW] : 0u;
      const uint32_t down = y + 1 < H ? nr[w + WW] : 0u;
      const uint32_t bd = ng & (~left | ~right | ~up | ~down);
      B[(y - y0) * WW + w] = (A[(y - y0) * WW + w] | bd) & vmask;
    }
  }
  __syncthreads();
  // detector: dilate r2 (A -> Cb), erode r1 (Cb -> A)
  RowRange d = rr.shrink(2, H);
  mb_hv<2, true>(A, Cb, d, y0, WW, W, H, L);
  __syncthreads();
  d = d.shrink(1, H);
  mb_hv<1, false>(Cb, A, d, y0, WW, W, H, L);
  __syncthreads();
  // padded detector rows py = y + 1 of this band (ring rows 0 and Hp - 1 by the edge bands)
  {
    const int wpw = dbits_wpw(W + 2);
    uint32_t* D = dbits + (size_t)f * dstride;
    const int py0 = yb == 0 ? 0 : yb + 1, py1 = ye == H ? H + 2 : ye + 1;
    for (int k = t; k < (py1 - py0) * wpw; k += nt) {
      const int py = py0 + k / wpw, w = k - (k / wpw) * wpw;
      uint32_t v = 0;
      if (py > 0 && py < H + 1) {
        const uint32_t* row = A + (py - 1 - y0) * WW;
        const uint32_t cur = w < WW ? row[w] : 0u;
        const uint32_t prv = (w > 0 && w - 1 < WW) ? row[w - 1] : 0u;
        v = (cur << 1) | (prv >> 31);  // padded x = image x + 1
      }
      D[(size_t)py * wpw + w] = v;
    }
  }
  // mask: {dilate, erode}(3), (4), (5) ping-pong B <-> A, then erode(3) -> HBM
  RowRange m = rm0.shrink(3, H);
  __syncthreads();
  mb_hv<3, true>(B, A, m, y0, WW, W, H, L);
  __syncthreads();
  m = m.shrink(3, H);
  mb_hv<3, false>(A, B, m, y0, WW, W, H, L);
  __syncthreads();
  m = m.shrink(4, H);
  mb_hv<4, true>(B, A, m, y0, WW, W, H, L);
  __syncthreads();
  m = m.shrink(4, H);
  mb_hv<4, false>(A, B, m, y0, WW, W, H, L);
  __syncthreads();
  m = m.shrink(5, H);
  mb_hv<5, true>(B, A, m, y0, WW, W, H, L);
  __syncthreads();
  m = m.shrink(5, H);
  mb_hv<5, false>(A, B, m, y0, WW, W, H, L);
  __syncthreads();
  // final erode(3): output rows [yb, ye) -> A, then to the tiled mask plane
  // (bits::tiled_word), lanes down a word column so the stores stay contiguous
  mb_hv<3, false>(B, A, RowRange{yb, ye}, y0, WW, W, H, L);
  __syncthreads();
  uint32_t* M = mbits + (size_t)f * bstride;
  const int nr = ye - yb;
  for (int k = t; k < nr * WW; k += nt) {
    const int w = k / nr, y = yb + (k - w * nr);
    M[bits::tiled_word(y, w, bits::tiled_rows(H))] = A[(y - y0) * WW + w];
  }
}

// The same two chains as k_morph, walked down the frame by one wave per
// (frame, row segment) with every stage's window in registers (no LDS, no
// barriers): lane w owns word column w (W <= 2016: the row fits one wave),
// the horizontal part of each stage takes the neighbour words from lanes
// w - 1 / w + 1 by DPP (lanes past the row hold the stage's identity, so the
// clipped-window rule at the left / right edge falls out), and the vertical
// part keeps the stage's last 2R + 1 horizontally processed input rows in a
// register ring. Stage outputs lag the input row i: NG(i - 1), M0 and the
// detector dilation (i - 2), detector erosion (i - 3), then the mask chain's
// seven passes (i - 5 ... i - 29). A row outside [0, H) enters a ring as the
// stage's identity (the clipped window of mk_bits.h). A segment starts its
// walk MB_HALO rows above its first output row, so every stored row is exact.
// Bit-identical to k_morph (tests/test_gpu_parity.py: masks and detector).
template <int R, bool DIL>
struct MwStage {
  // rows y - R .. y + 1 + R of the horizontally processed input: a step pushes
  // two rows and yields two output rows, so the ring shifts and the window's
  // OP over its middle 2R rows are shared by the pair (half the register moves
  // and vertical OPs of a one-row step)
  uint32_t ring[2 * R + 2];
  __device__ void init() {
#pragma unroll
    for (int k = 0; k < 2 * R + 2; k++) ring[k] = DIL ? 0u : ~0u;
  }
  // horizontal OP over x - R .. x + R of word `cur` (prev / next: the lanes
  // beside; every word already carries the identity outside the image)
  __device__ static uint32_t hop(uint32_t cur) {
    const uint32_t prev = dpp_from_left(cur), next = dpp_from_right(cur);
    uint32_t acc = cur;
#pragma unroll
    for (int k = 1; k <= R; k++) {
      const uint32_t rt = __builtin_amdgcn_alignbit(next, cur, k);       // in(x + k)
      const uint32_t lf = __builtin_amdgcn_alignbit(cur, prev, 32 - k);  // in(x - k)
      acc = DIL ? (acc | rt | lf) : (acc & rt & lf);
    }
    return acc;
  }
  // push input rows y + R, y + R + 1 (present: inside the image; the words
  // already carry this stage's identity outside it); yields rows y, y + 1
  __device__ void push2(uint32_t in0, bool p0, uint32_t in1, bool p1, uint32_t& o0, uint32_t& o1) {
#pragma unroll
    for (int k = 0; k < 2 * R; k++) ring[k] = ring[k + 2];
    ring[2 * R] = p0 ? hop(in0) : (DIL ? 0u : ~0u);
    ring[2 * R + 1] = p1 ? hop(in1) : (DIL ? 0u : ~0u);
    uint32_t mid = ring[1];
#pragma unroll
    for (int k = 2; k <= 2 * R; k++) mid = DIL ? (mid | ring[k]) : (mid & ring[k]);
    o0 = DIL ? (mid | ring[0]) : (mid & ring[0]);
    o1 = DIL ? (mid | ring[2 * R + 1]) : (mid & ring[2 * R + 1]);
  }
};
// NOT(gradient) word of the row with rows up / down (their presence: inside the image)
__device__ inline uint32_t mw_ng(uint32_t up, bool hu, uint32_t c0, uint32_t dn, bool hd, uint32_t vm) {
  const uint32_t c1 = c0 | ~vm;  // horizontal identities 0 / 1 outside the image
  uint32_t mx = c0 | __builtin_amdgcn_alignbit(dpp_from_right(c0), c0, 1) |
                __builtin_amdgcn_alignbit(c0, dpp_from_left(c0), 31);
  uint32_t mn = c1 & __builtin_amdgcn_alignbit(dpp_from_right(c1), c1, 1) &
                __builtin_amdgcn_alignbit(c1, dpp_from_left(c1), 31);
  if (hu) { mx |= up; mn &= up; }
  if (hd) { mx |= dn; mn &= dn; }
  return ~(mx ^ mn) & vm;
}
// M0 = edge | border(NG) word of the row (NG rows up / down: 0 outside the image)
__device__ inline uint32_t mw_m0(uint32_t e, uint32_t nu, uint32_t n, uint32_t nd, uint32_t vm) {
  const uint32_t left = __builtin_amdgcn_alignbit(n, dpp_from_left(n), 31);   // ng(x - 1)
  const uint32_t right = __builtin_amdgcn_alignbit(dpp_from_right(n), n, 1);  // ng(x + 1)
  return (e | (n & (~left | ~right | ~nu | ~nd))) & vm;
}
// RUNS (one segment per frame): the walker also numbers the runs of each
// padded detector row as it produces it -- the outputs of k_run_count /
// k_run_scan / k_run_emit (row bases, run starts, labels = own ids, n_runs),
// with a running id in an SGPR instead of a frame-wide scan.
struct WalkRuns {
  int32_t* rowb;
  size_t rstride;
  uint16_t* rx;
  int32_t* lab;
  size_t plane;
  FrameState* st;
};
#ifndef MK_MW_PF
#define MK_MW_PF 1  // k_morph_walk: steps of E-row prefetch
#endif
template <bool RUNS>
__global__ __launch_bounds__(256) void k_morph_walk(const uint32_t* __restrict__ eb, uint32_t* __restrict__ dbits,
                                                    uint32_t* __restrict__ mbits, int W, int H, size_t bstride,
                                                    size_t dstride, int seg_rows, int nseg, int nwaves, WalkRuns wr,
                                                    int roles) {
  const int gw0 = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
  if (gw0 >= nwaves) return;
  // roles == 2 (round 5): two waves per segment, the detector chain (dilate 5,
  // erode 3, runs) on one and the mask chain (NOT gradient, border, seven
  // stages) on the other, each reading the edge rows itself: the per-row
  // dependent chain of a wave is about half as long and twice the waves run
  const int role = roles == 2 ? (gw0 & 1) : -1;  // 0 detector, 1 mask, -1 both
  const bool det = role != 1, msk = role != 0;
  const int gw = roles == 2 ? gw0 >> 1 : gw0;
  const int lane = threadIdx.x & 63;
  const int f = gw / nseg, sg = gw - f * nseg;
  const int ys = sg * seg_rows, ye = min(H, ys + seg_rows);
  const int WW = bits::words(W), wpw = dbits_wpw(W + 2), Hp = bits::tiled_rows(H);
  const uint32_t vm = lane < WW ? bits::valid(lane, W) : 0u;  // valid pixels of this lane's word
  const uint32_t* E = eb + (size_t)f * bstride;
  uint32_t* D = dbits + (size_t)f * dstride;
  uint32_t* M = mbits + (size_t)f * bstride;
  // padded detector ring rows (zero) by the first / last segment
  if (det && sg == 0 && lane < wpw) D[lane] = 0u;
  if (det && ye == H && lane < wpw) D[(size_t)(H + 1) * wpw + lane] = 0u;
  int32_t* RB = RUNS ? wr.rowb + (size_t)f * wr.rstride : nullptr;
  uint16_t* RX = RUNS ? wr.rx + (size_t)f * wr.plane : nullptr;
  int32_t* RL = RUNS ? wr.lab + (size_t)f * wr.plane : nullptr;
  int run_id = 0;  // next run id (wave-uniform)
  // runs of padded row py (words v, lanes < wpw): the ring run at x = 0, then
  // one run per transition, in lane (word) order
  const auto emit_runs = [&](uint32_t v, int py) {
    const uint32_t prv = dpp_from_left(v);
    const uint32_t T = v ^ ((v << 1) | (prv >> 31));
    const int c = __popc(T);
    const int inc = wave_incl_scan(c, lane);
    if (lane == 0) {
      RB[py] = run_id;
      RX[run_id] = 0;
      RL[run_id] = run_id;
    }
    int o = run_id + 1 + inc - c;
    for (uint32_t t = T; t; t &= t - 1, o++) {
      RX[o] = (uint16_t)(32 * lane + __ffs(t) - 1);
      RL[o] = o;
    }
    run_id += 1 + __builtin_amdgcn_readlane(inc, 63);
  };
  if (RUNS && det) emit_runs(0u, 0);
  MwStage<2, true> d1;   // detector dilate 5x5 of E
  MwStage<1, false> d2;  // detector erode 3x3
  MwStage<3, true> s1;
  MwStage<3, false> s2;
  MwStage<4, true> s3;
  MwStage<4, false> s4;
  MwStage<5, true> s5;
  MwStage<5, false> s6;
  MwStage<3, false> s7;
  d1.init(); d2.init(); s1.init(); s2.init(); s3.init(); s4.init(); s5.init(); s6.init(); s7.init();
  const auto in = [H](int y) { return (unsigned)y < (unsigned)H; };
  uint32_t eA = 0, eB = 0;  // E rows i - 2, i - 1 (masked to the image, 0 outside it)
  uint32_t nA = 0, nB = 0;  // NG rows i - 3, i - 2
  // input rows a segment needs: the detector's output row y reads E rows y - 3 .. y + 3 (dilate 2 +
  // erode 1), the mask's y - 29 .. y + 29; a detector-only wave walks its own reach
  const int halo = role == 0 ? 3 : MB_HALO;
  const int i0 = max(0, ys - halo), i1 = min(H, ye) + halo;
  const auto ld = [&](int y) { return (in(y) && lane < WW) ? E[(size_t)y * WW + lane] & vm : 0u; };
  // E rows prefetched MK_MW_PF steps (2 MK_MW_PF rows) ahead
  uint32_t q[2 * MK_MW_PF];
#pragma unroll
  for (int k = 0; k < 2 * MK_MW_PF; k++) q[k] = ld(i0 + k);
  for (int i = i0; i < i1; i += 2) {
    const uint32_t e0 = q[0], e1 = q[1];  // E rows i, i + 1
#pragma unroll
    for (int k = 0; k + 2 < 2 * MK_MW_PF; k++) q[k] = q[k + 2];
    q[2 * MK_MW_PF - 2] = ld(i + 2 * MK_MW_PF);
    q[2 * MK_MW_PF - 1] = ld(i + 2 * MK_MW_PF + 1);
    // NOT(gradient) rows i - 1, i; M0 rows i - 2, i - 1
    uint32_t m0 = 0u, m1 = 0u;
    if (msk) {
      const uint32_t g0 = in(i - 1) ? mw_ng(eA, in(i - 2), eB, e0, in(i), vm) : 0u;
      const uint32_t g1 = in(i) ? mw_ng(eB, in(i - 1), e0, e1, in(i + 1), vm) : 0u;
      m0 = in(i - 2) ? mw_m0(eA, nA, nB, g0, vm) : 0u;
      m1 = in(i - 1) ? mw_m0(eB, nB, g0, g1, vm) : 0u;
      nA = g0;
      nB = g1;
    }
    eA = e0;
    eB = e1;
    uint32_t a0, a1, b0, b1;
    if (det) {
    // detector: dilate r2 of E (rows i, i + 1 in; i - 2, i - 1 out), erode r1 (i - 3, i - 2 out)
    d1.push2(e0, in(i), e1, in(i + 1), a0, a1);
    d2.push2((a0 & vm) | ~vm, in(i - 2), (a1 & vm) | ~vm, in(i - 1), b0, b1);
    b0 &= vm;
    b1 &= vm;
    {
      const uint32_t p0 = dpp_from_left(b0), p1 = dpp_from_left(b1);
      const int y = i - 3;
      const uint32_t v0 = lane < wpw ? (b0 << 1) | (p0 >> 31) : 0u, v1 = lane < wpw ? (b1 << 1) | (p1 >> 31) : 0u;
      if (y >= ys && y < ye) {
        if (lane < wpw) D[(size_t)(y + 1) * wpw + lane] = v0;
        if (RUNS) emit_runs(v0, y + 1);
      }
      if (y + 1 >= ys && y + 1 < ye) {
        if (lane < wpw) D[(size_t)(y + 2) * wpw + lane] = v1;
        if (RUNS) emit_runs(v1, y + 2);
      }
    }
    }
    if (!msk) continue;
    // mask: {dilate, erode}(3), (4), (5), erode(3): M0 rows i - 2, i - 1 in; i - 29, i - 28 out
    s1.push2(m0, in(i - 2), m1, in(i - 1), a0, a1);
    s2.push2((a0 & vm) | ~vm, in(i - 5), (a1 & vm) | ~vm, in(i - 4), b0, b1);
    s3.push2(b0 & vm, in(i - 8), b1 & vm, in(i - 7), a0, a1);
    s4.push2((a0 & vm) | ~vm, in(i - 12), (a1 & vm) | ~vm, in(i - 11), b0, b1);
    s5.push2(b0 & vm, in(i - 16), b1 & vm, in(i - 15), a0, a1);
    s6.push2((a0 & vm) | ~vm, in(i - 21), (a1 & vm) | ~vm, in(i - 20), b0, b1);
    s7.push2((b0 & vm) | ~vm, in(i - 26), (b1 & vm) | ~vm, in(i - 25), a0, a1);
    const int y = i - MB_HALO;
    if (y >= ys && y < ye && lane < WW) M[bits::tiled_word(y, lane, Hp)] = a0 & vm;
    if (y + 1 >= ys && y + 1 < ye && lane < WW) M[bits::tiled_word(y + 1, lane, Hp)] = a1 & vm;
  }
  if (RUNS && det) {
    emit_runs(0u, H + 1);
    if (lane == 0) {
      RB[H + 2] = run_id;
      wr.st[f].n_runs = run_id;
    }
  }
}

// debug bytes (frame 0): a W x H bit plane (wpw = 0: ceil(W/32) words per
// row; wpw = -1: the tiled mask plane) or the padded detector plane (wpw = its
// words per row) -> one byte per pixel
__global__ __launch_bounds__(256) void k_bits_to_bytes(const uint32_t* __restrict__ src, uint8_t* __restrict__ out,
                                                       int W, int H, int wpw) {
  const int WW = wpw > 0 ? wpw : bits::words(W);
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < W * H; k += gridDim.x * blockDim.x) {
    const int y = k / W, x = k - y * W;
    const size_t i = wpw < 0 ? bits::tiled_word(y, x >> 5, bits::tiled_rows(H)) : (size_t)y * WW + (x >> 5);
    out[k] = (uint8_t)((src[i] >> (x & 31)) & 1u);
  }
}

// ==================================================== contour components
// Run-length CCL of the zero-ringed detector binary (Wp x Hp, row-aligned bit
// plane): foreground 8-connected, background 4-connected. A row's runs
// (maximal spans of equal bits) alternate bg / fg from the ring pixel at
// x = 0 and are numbered in raster order, so the smallest run of a component
// starts at its raster-first pixel: where the sequential Suzuki–Abe scan
// (findContours, QuadDetection.h:216) discovers the component's border. A
// 720p detector frame has ~36k runs against 0.93 M pixels. Run starts go to
// a u16 plane (x), labels to an int32 plane (run ids, frame-local), both
// sized for one run per pixel, so nothing can overflow.
//   k_run_count   wave per row: transitions -> runs of the row
//   k_run_scan    block per frame: row bases (exclusive scan)
//   k_run_emit    wave per row: run starts, labels = own ids
//   k_run_band    block per 32-row band: unions with the overlapping same-colour
//                 runs of the row above (fg: [a-1, b+1], bg: [a, b]) in LDS
//   k_run_seam    wave per band boundary: the same unions across bands
//   k_run_border  wave per row: component roots -> border records
// Transitions of word w of a padded row: bit b set where x = 32 w + b starts a run.
__device__ inline uint32_t run_starts(const uint32_t* row, int w) {
  const uint32_t cur = row[w], prv = w > 0 ? row[w - 1] : 0u;
  return cur ^ ((cur << 1) | (prv >> 31));
}

// The per-row kernels of the run CCL (count, emit, border) take RUN_RPW rows
// per wave (a block = 4 waves = 4 RUN_RPW rows): a row is a few dozen runs,
// so with one row per wave the grid was 181 blocks per 720p frame (741k per
// 4096-frame batch) and the launches were bound by workgroup dispatch
#ifndef MK_RUN_RPW
#define MK_RUN_RPW 8
#endif
constexpr int RUN_RPW = MK_RUN_RPW;
__global__ __launch_bounds__(256) void k_run_count(const uint32_t* __restrict__ dbits, size_t dstride,
                                                   int32_t* __restrict__ rowb, size_t rstride, int Wp, int Hp) {
  const int f = blockIdx.y, lane = threadIdx.x & 63;
  const int ya = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RUN_RPW, yb = min(ya + RUN_RPW, Hp);
  const int nw = (Wp + 31) / 32;
  for (int y = ya; y < yb; y++) {
    const uint32_t* row = dbits + (size_t)f * dstride + (size_t)y * dbits_wpw(Wp);
    int c = 0;
    for (int w = lane; w < nw; w += 64) c += __popc(run_starts(row, w));
    c = wave_sum(c);
    if (lane == 0) rowb[(size_t)f * rstride + y] = c + 1;
  }
}

__global__ __launch_bounds__(256) void k_run_scan(int32_t* __restrict__ rowb, size_t rstride, FrameState* st,
                                                   int Hp) {
  __shared__ int32_t wsum[4];  // 256 threads: fits beside other contexts' kernels
  const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  int32_t* r = rowb + (size_t)f * rstride;
  const int per = (Hp + 255) / 256, y0 = t * per;
  int loc = 0;
  for (int k = 0; k < per; k++)
    if (y0 + k < Hp) loc += r[y0 + k];
  const int inc = wave_incl_scan(loc, lane);
  if (lane == 63) wsum[wave] = inc;
  __syncthreads();
  int off = 0;
  for (int k = 0; k < wave; k++) off += wsum[k];
  int acc = off + inc - loc;
  for (int k = 0; k < per; k++)
    if (y0 + k < Hp) {
      const int v = r[y0 + k];
      r[y0 + k] = acc;
      acc += v;
    }
  if (t == 255) {
    r[Hp] = acc;
    st[f].n_runs = acc;
  }
}

__global__ __launch_bounds__(256) void k_run_emit(const uint32_t* __restrict__ dbits, size_t dstride,
                                                  const int32_t* __restrict__ rowb, size_t rstride,
                                                  uint16_t* __restrict__ rx, int32_t* __restrict__ lab, size_t plane,
                                                  int Wp, int Hp) {
  const int f = blockIdx.y, lane = threadIdx.x & 63;
  const int ya = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RUN_RPW, yb = min(ya + RUN_RPW, Hp);
  uint16_t* X = rx + (size_t)f * plane;
  int32_t* L = lab + (size_t)f * plane;
  const int nw = (Wp + 31) / 32;
  for (int y = ya; y < yb; y++) {
    const uint32_t* row = dbits + (size_t)f * dstride + (size_t)y * dbits_wpw(Wp);
    int base = rowb[(size_t)f * rstride + y];
    if (lane == 0) { X[base] = 0; L[base] = base; }
    base++;
    for (int w0 = 0; w0 < nw; w0 += 64) {
      const int w = w0 + lane;
      uint32_t T = w < nw ? run_starts(row, w) : 0u;
      const int c = __popc(T);
      const int inc = wave_incl_scan(c, lane);
      int o = base + inc - c;
      while (T) {
        const int b = __ffs(T) - 1;
        T &= T - 1;
        X[o] = (uint16_t)(32 * w + b);
        L[o] = o;
        o++;
      }
      base += __builtin_amdgcn_readlane(inc, 63);
    }
  }
}

// largest k in [0, n) with x[k] <= v (x[0] == 0 <= v)
__device__ inline int run_at(const uint16_t* x, int n, int v) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((int)x[mid] <= v) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// Unions of row y's runs (ids by .. by+ny-1, starts X[by..]) with the
// overlapping same-colour runs of row y-1 (ids bp .. bp+np-1): fg runs
// 8-connected ([a-1, b+1]), bg runs 4-connected ([a, b]); one wave, lanes over
// the runs. UF is lds_union on band-local ids or uf_union_c on frame ids.
template <class UF>
__device__ inline void run_row_union(const uint16_t* X, int bp, int np, int by, int ny, int Wp, int lane,
                                     const UF& uni) {
  const uint16_t* Xp = X + bp;
  for (int j = lane; j < ny; j += 64) {
    const int fg = j & 1;
    const int a = X[by + j], b = (j + 1 < ny ? (int)X[by + j + 1] : Wp) - 1;
    const int lo = a - fg, hi = b + fg;
    for (int k = run_at(Xp, np, lo); k < np && (int)Xp[k] <= hi; k++)
      if ((k & 1) == fg) uni(by + j, bp + k);
  }
}

// Run unions in two levels, so the union-find paths stay short (a
// frame-wide chain of per-row links had every find walk up to ~700 global
// hops). k_run_band: one block per band of RB_ROWS rows, its runs' starts and
// labels in LDS, unions inside the band, then every run's label = its band
// root (the band component's smallest run id). k_run_seam: the unions across
// band boundaries on the global labels. Roots stay the component's smallest
// run id either way (both unions link the larger root under the smaller).
// A band with more than RB_CAP runs does its in-band unions on the global
// labels instead.
#ifndef MK_RB_ROWS
#define MK_RB_ROWS 32
#endif
constexpr int RB_ROWS = MK_RB_ROWS, RB_CAP = 128 * MK_RB_ROWS;
#ifndef MK_RB_THREADS
#define MK_RB_THREADS 512  // 8 waves per 32-row band: components 2.70 -> 2.57 ms per 4096 frames (1024: 3.2)
#endif
constexpr int RB_THREADS = MK_RB_THREADS, RB_WAVES = RB_THREADS / 64;
__global__ __launch_bounds__(RB_THREADS) void k_run_band(const int32_t* __restrict__ rowb, size_t rstride,
                                                  const uint16_t* __restrict__ rx, int32_t* lab, size_t plane, int Wp,
                                                  int Hp) {
  __shared__ int32_t Ll[RB_CAP];
  __shared__ uint16_t Xl[RB_CAP];
  __shared__ int32_t rbl[RB_ROWS + 1];
  const int f = blockIdx.y, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int y0 = blockIdx.x * RB_ROWS;
  if (y0 >= Hp) return;
  const int y1 = min(y0 + RB_ROWS, Hp);
  const int32_t* r = rowb + (size_t)f * rstride;
  const uint16_t* X = rx + (size_t)f * plane;
  int32_t* L = lab + (size_t)f * plane;
  const int g0 = r[y0], n = r[y1] - g0;
  if (n > RB_CAP) {
    const auto uni = [L](int a, int b) { uf_union_c(L, a, b); };
    for (int y = y0 + 1 + wave; y < y1; y += RB_WAVES) run_row_union(X, r[y - 1], r[y] - r[y - 1], r[y], r[y + 1] - r[y], Wp, lane, uni);
    return;
  }
  for (int i = t; i <= y1 - y0; i += RB_THREADS) rbl[i] = r[y0 + i] - g0;
  for (int i = t; i < n; i += RB_THREADS) {
    Xl[i] = X[g0 + i];
    Ll[i] = i;
  }
  __syncthreads();
  int* Li = Ll;
  const auto uni = [Li](int a, int b) { lds_union(Li, a, b); };
  for (int y = y0 + 1 + wave; y < y1; y += RB_WAVES) {
    const int q = y - y0;
    run_row_union(Xl, rbl[q - 1], rbl[q] - rbl[q - 1], rbl[q], rbl[q + 1] - rbl[q], Wp, lane, uni);
  }
  __syncthreads();
  for (int i = t; i < n; i += RB_THREADS) L[g0 + i] = g0 + lds_find(Ll, i);
}

// one wave per band boundary row y = k * RB_ROWS (k >= 1) against row y-1
__global__ __launch_bounds__(256) void k_run_seam(const int32_t* __restrict__ rowb, size_t rstride,
                                                  const uint16_t* __restrict__ rx, int32_t* lab, size_t plane, int Wp,
                                                  int Hp) {
  const int f = blockIdx.y;
  const int y = (blockIdx.x * 4 + (threadIdx.x >> 6) + 1) * RB_ROWS, lane = threadIdx.x & 63;
  if (y >= Hp) return;
  const int32_t* r = rowb + (size_t)f * rstride;
  int32_t* L = lab + (size_t)f * plane;
  const auto uni = [L](int a, int b) { uf_union_c(L, a, b); };
  run_row_union(rx + (size_t)f * plane, r[y - 1], r[y] - r[y - 1], r[y], r[y + 1] - r[y], Wp, lane, uni);
}

// row of run id: largest y with rowb[y] <= id
__device__ inline int run_at_row(const int32_t* rowb, int Hp, int id) {
  int lo = 0, hi = Hp - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (rowb[mid] <= id) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__global__ __launch_bounds__(256) void k_run_border(const int32_t* __restrict__ rowb, size_t rstride,
                                                    const uint16_t* __restrict__ rx, int32_t* lab, size_t plane,
                                                    Border* __restrict__ borders, FrameState* st, int Wp, int Hp,
                                                    int cap) {
  const int f = blockIdx.y, lane = threadIdx.x & 63;
  const int ya = (blockIdx.x * 4 + (threadIdx.x >> 6)) * RUN_RPW, yb = min(ya + RUN_RPW, Hp);
  if (ya >= Hp) return;
  const int32_t* r = rowb + (size_t)f * rstride;
  const uint16_t* X = rx + (size_t)f * plane;
  int32_t* L = lab + (size_t)f * plane;
  // the wave's rows' run bases in one load (lane q: row ya + q, q <= rows);
  // its runs are the contiguous ids [base of ya, base of yb), taken 64 at a
  // time whatever their rows (no pass per row)
  const int nrow = yb - ya;
  const int rbq = lane <= nrow ? r[ya + lane] : 0x7fffffff;
  const int g0 = __builtin_amdgcn_readlane(rbq, 0), g1 = __builtin_amdgcn_readlane(rbq, nrow);
  const int nruns = r[Hp];
  const uint64_t below = (1ull << lane) - 1;
  for (int id = g0 + lane; __ballot(id < g1); id += 64) {
    const bool live = id < g1;
    // row of run id: the last row base <= id
    int y = ya, by = g0;
#pragma unroll
    for (int k = 1; k < RUN_RPW; k++) {
      const int bk = __builtin_amdgcn_readlane(rbq, k);
      if (k < nrow && bk <= id) { y = ya + k; by = bk; }
    }
    const int j = id - by;
    // a root is a run whose label is itself: one load (a find would walk, and
    // path-halve, the chain of every non-root; halving never makes a non-root
    // point to itself, so the test is exact while other lanes compress).
    // Run 0 (ring) is the outside background.
    const bool root = live && id != 0 && L[id] == id;
    Border b;
    if (root) {
      const int key = y * Wp + X[id];
      b.key = key;
      if (j & 1) {
        b.start = key; b.hole = 0; b.parent = key;
      } else {
        // hole: the run on its left is foreground; its component's root run
        // starts at the key of the enclosing outer border. Kept as -(root + 1):
        // k_frame_contours turns it into that key for the few borders that
        // become quads (the root's row is a binary search of dependent loads,
        // the longest chain of this kernel when it ran for every hole here)
        const int pr = uf_find_c(L, id - 1);
        b.start = key - 1; b.hole = 1; b.parent = -(pr + 1);
      }
    }
    // one counter atomic per wave trip for all its roots
    const uint64_t m = __ballot(root);
    if (!m) continue;
    const int leader = __ffsll((unsigned long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(&st[f].n_borders, __popcll(m));
    base = __builtin_amdgcn_readlane(base, leader);
    if (!root) continue;
    const int idx = base + __popcll(m & below);
    if (idx < cap) {
      borders[(size_t)f * cap + idx] = b;
      // border index of the root run, above the labels (k_seg_plan; it checks the fit)
      if (2 * (size_t)nruns <= plane) L[nruns + id] = idx;
    } else {
      atomicOr(&st[f].overflow, 1);
    }
  }
}

// ============================================ per-frame contour -> quads
// direction code -> (dx + 1), (dy + 1), two bits per code (branch-free code_dx/code_dy)
__device__ inline int fdx(int s) { return (int)((0x901Au >> (2 * s)) & 3u) - 1; }
__device__ inline int fdy(int s) { return (int)((0xA901u >> (2 * s)) & 3u) - 1; }

// Next-direction table of the border follower: for the 3x3 pattern
// p9 = up | mid << 3 | dn << 6 (each 3 bits = columns x-1, x, x+1) and the
// search start s (the code pointing back to the previous pixel), the first
// set neighbour counter-clockwise after s (8: none). One LDS byte per step
// replaces building the packed 8-neighbourhood and the rotate + ctz search.
__device__ inline void build_next_lut(uint8_t* lut, int tid, int nthreads) {
  for (int e = tid; e < 512 * 8; e += nthreads) {
    const uint32_t p9 = (uint32_t)e >> 3;
    const int s = e & 7;
    const uint32_t m = nb8_from_rows(p9 & 7u, (p9 >> 3) & 7u, (p9 >> 6) & 7u);
    const uint32_t r = ((m | (m << 8)) >> (s + 1)) & 0xffu;
    lut[e] = r ? (uint8_t)((s + 1 + __builtin_ctz(r)) & 7) : (uint8_t)8;
  }
}

// Single-pass border tracing: points go to 64-point chunks handed out by an
// LDS bump allocator; a wave per chunk then compacts them by border.
// 16-point chunks: a segmented walk (k_seg_plan) leaves one partial chunk per
// segment, so the chunk storage (the pool's size in points) must hold the
// points plus < 16 per segment (64-point chunks overflowed it on dense frames)
constexpr int kChunk = 16;
#ifndef MK_CHUNK_BUF
#define MK_CHUNK_BUF 2  // border-walk points staged per half chunk (packed): border_trace 5.75 / 6.16 -> 4.67 / 4.64 ms per 4096 frames
#endif
// Chunk c holds ccount[c] points that go to positions ordv[c] .. of its
// owner's point list (owner = border; during segmented walks the segment,
// k_seg_chain then adds the segment's offset in its border and maps the owner).
struct ChunkEmit {
  int32_t* chunks;  // [chunk][kChunk] packed points (x | y << 16)
  int32_t* owner;   // border (or segment) of each chunk
  int32_t* ordv;    // first point position of the chunk within its owner
  int32_t* ccount;  // points in the chunk
  int32_t* counter; // LDS
  int max_chunks, border, cur, k, nch;
  bool ovf;
  int n_pts = 0;  // the walk's point count (walk_segment_lds)
#if MK_CHUNK_BUF
  // points of the current half chunk (8 points = 64 B) held in registers and
  // stored at once: a chunk's 128-B line gets two full-width writes instead
  // of sixteen 8-byte ones spread over the walk (a selected slot per point:
  // the index is per lane)
#if MK_CHUNK_BUF == 2  // packed x | y << 16 (points are image coordinates >= 0): one register per point
  uint32_t bp[8];
  __device__ uint32_t pk(int j) const { return bp[j]; }
#else
  int bx[8], by[8];
  __device__ uint32_t pk(int j) const { return (uint32_t)bx[j] | ((uint32_t)by[j] << 16); }
#endif
  // chunk points packed x | y << 16 (PtPacked, what the contour pool holds):
  // a half chunk is two 16-byte stores
  __device__ void store8(int k0) {
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    u32x4* d = (u32x4*)((uint32_t*)chunks + ((size_t)cur * kChunk + k0));
#pragma unroll
    for (int j = 0; j < 2; j++)
      d[j] = u32x4{pk(4 * j), pk(4 * j + 1), pk(4 * j + 2), pk(4 * j + 3)};
  }
#endif
  __device__ void operator()(int px, int py) {
    if (cur < 0 || k == kChunk) {
      if (ovf) return;
      if (cur >= 0) ccount[cur] = kChunk;
      const int c = atomicAdd(counter, 1);
      if (c >= max_chunks) { ovf = true; return; }
      cur = c;
      k = 0;
      owner[c] = border;
      ordv[c] = kChunk * nch++;
    }
#if MK_CHUNK_BUF
    const int i = k & 7;
#pragma unroll
    for (int j = 0; j < 8; j++) {
#if MK_CHUNK_BUF == 2
      bp[j] = j == i ? (uint32_t)px | ((uint32_t)py << 16) : bp[j];
#else
      bx[j] = j == i ? px : bx[j];
      by[j] = j == i ? py : by[j];
#endif
    }
    k++;
    if ((k & 7) == 0) store8(k - 8);
#else
    ((uint32_t*)chunks)[(size_t)cur * kChunk + k] = (uint32_t)px | ((uint32_t)py << 16);  // one 4-byte store
    k++;
#endif
  }
  __device__ void flush() {
    if (cur < 0) return;
#if MK_CHUNK_BUF
    if (k & 7) store8(k & ~7);  // the open half (slots past k: stale, never read: ccount bounds the chunk)
#endif
    ccount[cur] = k;
  }
};

// max over the wave of (d, idx) with ties to the smaller idx (the first
// strict maximum of a sequential scan in idx order)
__device__ inline void wave_argmax(double& d, int& idx) {
  for (int o = 32; o > 0; o >>= 1) {
    const double d2 = __shfl_xor(d, o);
    const int i2 = __shfl_xor(idx, o);
    if (d2 > d || (d2 == d && i2 < idx)) { d = d2; idx = i2; }
  }
}

// approx_poly (mk_contour.h, closed, quad early exit) executed by one wave:
// the farthest-point scans are lane-parallel reductions; lane 0 owns the DP
// stack and the output (single-lane memory order), control is wave-uniform.
// STK: the DP stack's storage -- global scratch (int32_t*, as many slices as
// points) or a wave's LDS slice of `cap` slices (lds_i32*): a push past cap
// returns -1 and the caller runs the border again on the global stack (the DP
// is deterministic, dst is rewritten)
typedef __attribute__((address_space(3))) int32_t lds_i32;
#ifndef MK_WAVE_STK
#define MK_WAVE_STK 14  // 16 waves x 14 slices x 8 B: k_frame_contours stays under 32 KB of LDS (5 blocks per CU)
#endif
constexpr int kWaveStk = MK_WAVE_STK;  // DP stack slices per wave in LDS
template <class STK>
__device__ int approx_poly_wave(const uint32_t* __restrict__ src, int count, double eps, int32_t* dst, STK stk,
                                int max_dp, int cap = 0x7fffffff) {  // src: packed points (PtPacked)
  const int lane = threadIdx.x & 63;
  if (count == 0) return 0;
  eps *= eps;
  int top = 0, nc = 0, rs_s = 0, pos = 0;
  bool le_eps = false;
  int spx = 0, spy = 0;
  for (int it = 0; it < 3; it++) {
    pos = (pos + rs_s) % count;
    spx = PtPacked::x(src[pos]);
    spy = PtPacked::y(src[pos]);
    double best = 0;
    int bj = 0x7fffffff;
    for (int j = 1 + lane; j < count; j += 64) {
      int q = pos + j;
      if (q >= count) q -= count;
      const uint32_t v = src[q];
      const double dx = PtPacked::x(v) - spx, dy = PtPacked::y(v) - spy;
      const double d = dx * dx + dy * dy;
      if (d > best) { best = d; bj = j; }
    }
    wave_argmax(best, bj);
    if (best > 0) rs_s = bj;
    le_eps = best <= eps;
  }
  if (!le_eps) {
    const int sl_s = pos % count, sl_e = (rs_s + sl_s) % count;
    if (lane == 0) {
      stk[0] = sl_e; stk[1] = sl_s;  // PUSH(rs_s, rs_e)
      stk[2] = sl_s; stk[3] = sl_e;  // PUSH(sl_s, sl_e)
    }
    top = 2;
  } else {
    if (lane == 0) { dst[0] = spx; dst[1] = spy; }
    nc = 1;
  }
  while (top > 0) {
    top--;
    int a0 = 0, a1 = 0;
    if (lane == 0) { a0 = stk[2 * top]; a1 = stk[2 * top + 1]; }
    const int sl_s = __shfl(a0, 0), sl_e = __shfl(a1, 0);
    const int epx = PtPacked::x(src[sl_e]), epy = PtPacked::y(src[sl_e]);
    int p0 = sl_s + 1;
    if (p0 >= count) p0 = 0;
    spx = PtPacked::x(src[sl_s]);
    spy = PtPacked::y(src[sl_s]);
    if (p0 != sl_e) {
      const double dx = epx - spx, dy = epy - spy;
      int L = sl_e - p0;
      if (L < 0) L += count;
      double best = 0;
      int bt = 0x7fffffff;
      for (int t = lane; t < L; t += 64) {
        int q = p0 + t;
        if (q >= count) q -= count;
        const uint32_t v = src[q];
        const double dist = fabs((PtPacked::y(v) - spy) * dx - (PtPacked::x(v) - spx) * dy);
        if (dist > best) { best = dist; bt = t; }
      }
      wave_argmax(best, bt);
      if (best > 0) rs_s = (p0 + bt) % count;
      le_eps = best * best <= eps * (dx * dx + dy * dy);
    } else {
      le_eps = true;
    }
    if (le_eps) {
      if (lane == 0) { dst[2 * nc] = spx; dst[2 * nc + 1] = spy; }
      nc++;
      if (max_dp > 0 && nc >= max_dp) return max_dp + 1;
    } else {
      if (top + 2 > cap) return -1;  // wave-uniform
      if (lane == 0) {
        stk[2 * top] = rs_s; stk[2 * top + 1] = sl_e;      // PUSH(rs_s, rs_e = sl_e)
        stk[2 * top + 2] = sl_s; stk[2 * top + 3] = rs_s;  // PUSH(sl_s, sl_e = rs_s)
      }
      top += 2;
    }
  }
  int r = 0;
  if (lane == 0) r = approx_cleanup(dst, nc, eps, true);
  return __shfl(r, 0);
}

// CCOMP output order (OpenCV tree pre-order): outers by key descending, each
// followed by its holes by key descending.
__device__ inline bool ccomp_before(int pa, int ha, int ka, int pb, int hb, int kb) {
  if (pa != pb) return pa > pb;
  if (ha != hb) return ha < hb;
  return ka > kb;
}

#ifndef MK_LONG_BORDER
#define MK_LONG_BORDER 128
#endif
constexpr int kLongBorder = MK_LONG_BORDER;  // points; longer borders get a whole wave for approxPolyDP
static_assert(kLongBorder <= 128, "k_frame_contours' length buckets (count / 4) hold counts up to 128");
constexpr int kMaxLong = 512;

struct RawQuad {
  int32_t c[8];
  int32_t parent, hole, key;
};

// The detector bit plane again for the walks (round 6 layout): for each
// 32-row tile ty and 16-pixel group g, kTbRows = 34 32-bit words -- rows
// 32 ty - 1 .. 32 ty + 32 of the 32-pixel window 16 g - 8 .. 16 g + 23. A walk
// step at (x, y) needs pixels x - 1 .. x + 1 of rows y - 1 .. y + 1: group
// x >> 4, bit (x & 15) + 7 of three consecutive words (entries y & 31 ..
// + 2 of the tile), so ONE 12-byte load per step instead of three 8-byte
// ones of round 5's 64-bit row windows (the walks were bound by the vector
// memory pipeline: TA 64 %, TD 77 % busy, profiles/r05_pmc.json); a walk
// moving vertically stays in the lines it holds. Same size as before (~250 KB
// per 720p frame).
constexpr int kTbRows = 34;
__device__ __host__ inline int tb_groups(int Wp) { return ((Wp - 2) >> 4) + 1; }
__device__ __host__ inline size_t tbits_words(int Wp, int Hp) {
  return (size_t)tb_groups(Wp) * kTbRows * (size_t)((Hp + 31) >> 5);
}
// word offset of the three rows y - 1 .. y + 1 around pixel x (1 <= x <= Wp - 2, 1 <= y <= Hp - 2)
__device__ inline uint32_t tb_off(int x, int y, int G) {
  return (uint32_t)(((y >> 5) * G + (x >> 4)) * kTbRows + (y & 31));
}
__global__ __launch_bounds__(256) void k_tile_bits(const uint32_t* __restrict__ dbits, size_t dstride,
                                                   uint32_t* __restrict__ tbits, size_t tstride, int wpw, int Wp,
                                                   int Hp) {
  extern __shared__ uint32_t tl_band[];  // kTbRows rows x wpw words
  const int f = blockIdx.y, ty = blockIdx.x, t = threadIdx.x;
  const uint32_t* src = dbits + (size_t)f * dstride;
  const int r0 = 32 * ty - 1;
  for (int i = t; i < kTbRows * wpw; i += 256) {
    const int e = i / wpw, r = r0 + e;
    tl_band[i] = r >= 0 && r < Hp ? src[(size_t)r * wpw + (i - e * wpw)] : 0u;
  }
  __syncthreads();
  const int G = tb_groups(Wp);
  uint32_t* dst = tbits + (size_t)f * tstride + (size_t)ty * G * kTbRows;
  for (int o = t; o < G * kTbRows; o += 256) {
    const int g = o / kTbRows, e = o - g * kTbRows;
    const int p = 16 * g - 8, w = p >> 5, sh = p & 31;  // sh is 8 or 24
    const uint32_t lo = w >= 0 ? tl_band[e * wpw + w] : 0u, hi = w + 1 < wpw ? tl_band[e * wpw + w + 1] : 0u;
    dst[o] = (lo >> sh) | (hi << (32 - sh));
  }
}
struct BitsTiled {
  const uint32_t* __restrict__ b;
  int G;
  __device__ uint32_t operator()(int x, int y) const {
    const uint32_t* p = b + tb_off(x, y, G);
    const int sh = (x & 15) + 7;
    return nb8_from_rows((p[0] >> sh) & 7u, (p[1] >> sh) & 7u, (p[2] >> sh) & 7u);
  }
};

// trace_border_lut as a resumable walk (one step per call), so a lane whose
// border closed can take the next one while its wave's long walks go on. A
// step is a serial chain and its wave issues it for one or a few lanes, so it
// is kept short: the position packed as x | y << 16 (one add moves it; the
// emitted point is (x - 1, y - 1), as trace_border_lut's px, py), 32-bit byte
// offsets into the tiled plane (scalar base + vector offset addressing).
#ifndef MK_WALK_WINDOW
#define MK_WALK_WINDOW 1  // walk_step keeps a 4-word window of the tiled plane (0: a load per step)
#endif
struct Walk {
  uint32_t pos, spos, p1;  // current, start, and the start's last neighbour
  int s, prev_s, n, steps;
  int first;               // the next step is the segment's first (never a checkpoint stop)
  // walk_step's window: 4 consecutive words of one (tile, group) column of the
  // tiled plane, ck = (tile * G + group) << 5 | first word (~0u: none)
  uint32_t ck, c0, c1, c2, c3;
};
__device__ inline uint32_t wpos(int x, int y) { return (uint32_t)x | ((uint32_t)y << 16); }
__device__ inline uint32_t wdelta(int s) { return (uint32_t)(fdx(s) + (fdy(s) << 16)); }
// the walk's first pixel and search; false: a single-point border (emitted)
template <class NB, class EM>
__device__ inline bool walk_start(const NB& nb, int sx, int sy, bool hole, EM& em, Walk& w) {
  const uint32_t m = nb(sx, sy);
  const int s_end0 = hole ? 0 : 4;
  int s = s_end0;
  do {
    s = (s - 1) & 7;
  } while (!((m >> s) & 1u) && s != s_end0);
  w.n = 0;
  w.steps = 0;
  if (s == s_end0) {
    em(sx - 1, sy - 1);
    w.n = 1;
    return false;
  }
  w.spos = w.pos = wpos(sx, sy);
  w.p1 = wpos(sx + fdx(s), sy + fdy(s));
  w.prev_s = s ^ 4;
  w.s = s;
  w.ck = ~0u;
  return true;
}
// ------------------------------------------------ segmented border walks
// A long border (the outer border of the grid's net, the large holes: 4.5k-
// 9k steps, the frame's critical path) is walked as segments in parallel.
// Checkpoints are fixed visits of the walk: in every row y = M k (padded
// coordinates), each foreground run [a, b] gives the visit of pixel a whose
// swept background arc holds its west neighbour and the visit of b whose arc
// holds its east neighbour. Each such visit lies on exactly one border (the
// one between the run's component and the background component on that side)
// and occurs exactly once in that border's walk, and its walk state follows
// from the 3x3 neighbourhood alone: the search start is the first foreground
// direction clockwise from the arc's direction. So a segment starts at a
// checkpoint with the state the whole walk would have there, emits exactly
// the points the whole walk emits, and stops on arriving at the next
// checkpoint visit (a local test: row y = M k and the arc about to be swept
// holds west or east) or at its border's closing move. k_seg_chain then links
// the segments of each border from its start in walk order: the point
// sequence is findContours' (QuadDetection.h:216), bit for bit.
constexpr int kSegRows = 512;     // sampled rows per frame (Hp <= 512 M)
constexpr int kSegCap = 65536;    // segments per frame
struct SegTab {
  int32_t* rowbase;  // first checkpoint id of each sampled row (2 per foreground run)
  int32_t *border, *pos, *sdir, *next, *cnt, *off;
  int cap;
};
// in the scratch after the chunk planes (chunks 2 pc, owner / ordv / ccount 3 mc)
__device__ inline SegTab seg_tab(int32_t* sc, int pool_cap) {
  const long mc = pool_cap / kChunk;
  int32_t* base = sc + 2 * (size_t)pool_cap + 3 * (size_t)mc;
  const long avail = 4L * pool_cap - (2L * pool_cap + 3L * mc) - kSegRows;
  SegTab t;
  t.cap = (int)(avail / 6 < kSegCap ? avail / 6 : kSegCap);
  t.rowbase = base;
  int32_t* q = base + kSegRows;
  t.border = q;
  t.pos = q + t.cap;
  t.sdir = q + 2 * (size_t)t.cap;
  t.next = q + 3 * (size_t)t.cap;
  t.cnt = q + 4 * (size_t)t.cap;
  t.off = q + 5 * (size_t)t.cap;
  return t;
}
// sdir codes of a segment: >= 0 checkpoint (search start), -1 unused (the
// right visit of a one-pixel run that is its left visit), -2 start segment
// aliased to the checkpoint at its border's start (next = that id), -3 start
// segment walked from the border start, -4 isolated pixel (one point)
constexpr int kSegUnused = -1, kSegAlias = -2, kSegStart = -3, kSegSingle = -4;
// checkpoint id of the visit of pixel (x, y) on the west (side 0) / east (1)
// arc: its foreground run in the row's run list (run 0 of a row is the
// background ring, foreground runs have odd local indices)
__device__ inline int seg_id_at(int x, int y, int side, int M, const int32_t* r, const uint16_t* X,
                                const int32_t* rowbase) {
  const int j0 = r[y];
  const int j = j0 + run_at(X + j0, r[y + 1] - j0, x);
  return rowbase[y / M - 1] + 2 * ((j - j0 - 1) >> 1) + side;
}
// does the arc swept from search start s to the found direction sn (both
// exclusive, counter-clockwise) hold direction d
__device__ inline bool arc_has(int s, int sn, int d) { return ((d - s - 1) & 7) < ((sn - s - 1) & 7); }
// first foreground direction clockwise from d - 1 (the search start of the
// visit whose arc holds d); d if there is none (an isolated pixel)
__device__ inline int first_cw(uint32_t m, int d) {
  int s = d;
  do {
    s = (s - 1) & 7;
  } while (!((m >> s) & 1u) && s != d);
  return s;
}
// the walk at a checkpoint visit
template <class NB>
__device__ inline void seg_begin(const NB& nb, const Border& b, int Wp, uint32_t pos, int sd, Walk& w) {
  const int sx = b.start % Wp, sy = b.start / Wp;
  const int s0 = first_cw(nb(sx, sy), b.hole ? 0 : 4);  // the border start's last neighbour (walk_start)
  w.spos = wpos(sx, sy);
  w.p1 = wpos(sx + fdx(s0), sy + fdy(s0));
  w.pos = pos;
  w.s = sd;
  w.prev_s = (sd + 4) & 7;
  w.n = 0;
  w.steps = 0;
  w.first = 1;
  w.ck = ~0u;
}
// one step of the follower on the tiled plane (BitsTiled layout, wpw32 = 32 *
// words per row); false once the segment ended: nx = the next segment's
// checkpoint id, -1 when the border closed
template <class EM>
__device__ inline bool walk_step(const uint32_t* __restrict__ tb, int G, const uint8_t* lut, EM& em, Walk& w,
                                 int M, const int32_t* r, const uint16_t* X, const int32_t* rowbase, int& nx) {
  const int x = (int)(w.pos & 0xffffu), y = (int)(w.pos >> 16);
#if MK_WALK_WINDOW
  // rows y - 1 .. y + 1 are the words (y & 31) .. + 2 of the (tile, group)
  // column tg. A lane keeps 4 consecutive words of one column: a step that
  // stays inside them (moves along the 16-pixel group, or one row on in the
  // direction the window was placed) needs no load. The long segments that
  // end a frame's walks run with one or two busy lanes per wave, so a step
  // the window covers costs the lane's LDS lookup instead of an L2 round trip.
  const uint32_t tg = (uint32_t)((y >> 5) * G + (x >> 4));
  const int yr = y & 31;
  int d = yr - (int)(w.ck & 31u);
  if ((w.ck >> 5) != tg || (unsigned)d > 1u) {
    // place the window so the next row in the walk's direction is inside it
    // (words s0 .. s0 + 3 <= 33: inside the column's 34)
    const int s0 = fdy(w.s ^ 4) < 0 ? max(yr - 1, 0) : min(yr, 30);
    typedef unsigned int u32x4a __attribute__((ext_vector_type(4), aligned(4)));
    const u32x4a v = *(const __attribute__((address_space(1))) u32x4a*)((const char*)tb + ((tg * kTbRows + s0) << 2));
    w.c0 = v.x; w.c1 = v.y; w.c2 = v.z; w.c3 = v.w;
    w.ck = (tg << 5) | (uint32_t)s0;
    d = yr - s0;
  }
  const uint32_t va = d ? w.c1 : w.c0, vb = d ? w.c2 : w.c1, vc = d ? w.c3 : w.c2;
  const int sh = (x & 15) + 7;
  const uint32_t p9 = ((va >> sh) & 7u) | (((vb >> sh) & 7u) << 3) | (((vc >> sh) & 7u) << 6);
#else
  // rows y - 1 .. y + 1 as three consecutive words: one 12-byte load (scalar
  // base + 32-bit byte offset)
  typedef unsigned int u32x3a __attribute__((ext_vector_type(3), aligned(4)));
  const u32x3a v = *(const __attribute__((address_space(1))) u32x3a*)((const char*)tb + (tb_off(x, y, G) << 2));
  const int sh = (x & 15) + 7;
  const uint32_t p9 = ((v.x >> sh) & 7u) | (((v.y >> sh) & 7u) << 3) | (((v.z >> sh) & 7u) << 6);
#endif
  const int s = lut[(p9 << 3) | w.s];
  if (M > 0 && !w.first && y % M == 0) {
    const bool west = arc_has(w.s, s, 4);
    if (west || arc_has(w.s, s, 0)) {
      nx = seg_id_at(x, y, west ? 0 : 1, M, r, X, rowbase);
      return false;
    }
  }
  w.first = 0;
  if (s != w.prev_s) {
    em(x - 1, y - 1);
    w.n++;
    w.prev_s = s;
  }
  const uint32_t np = w.pos + wdelta(s);
  if (np == w.spos && w.pos == w.p1) {
    nx = -1;
    return false;
  }
  w.pos = np;
  w.s = (s + 4) & 7;
  w.steps++;
  return true;
}

// The frame's segments (before the walks; one block per frame): checkpoints
// of the sampled rows with their border (the run's component, or the hole on
// that side when the run's component encloses it: the hole's root run has the
// component's run on its left, k_run_border's parent rule), search start and
// kind; then one start segment per border, aliased to its start's checkpoint
// when the start lies in a sampled row. M = 0, too many rows or segments, or
// a label plane too full for the border-index map: borders walked whole.
struct BitsRows {  // the padded bit plane, row-major (dbits)
  const uint32_t* b;
  int wpw;
  __device__ uint32_t row3(int x, int y) const {
    const uint32_t* p = b + (size_t)y * wpw + ((x - 1) >> 5);
    const uint64_t v = ((uint64_t)p[1] << 32) | p[0];
    return (uint32_t)(v >> ((x - 1) & 31)) & 7u;
  }
  __device__ uint32_t operator()(int x, int y) const { return nb8_from_rows(row3(x, y - 1), row3(x, y), row3(x, y + 1)); }
};
__global__ __launch_bounds__(256) void k_seg_plan(const uint32_t* __restrict__ dbits, size_t dstride,
                                                  const int32_t* __restrict__ rowb, size_t rstride,
                                                  const uint16_t* __restrict__ rx, int32_t* lab, size_t plane,
                                                  const Border* __restrict__ borders, FrameState* st,
                                                  int32_t* __restrict__ scratch, int pool_cap, int Wp, int Hp,
                                                  int border_cap, int M) {
  __shared__ int32_t rb[kSegRows + 1];
  __shared__ int32_t wsum[4];
  const int f = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int32_t* r = rowb + (size_t)f * rstride;
  const uint16_t* X = rx + (size_t)f * plane;
  int32_t* L = lab + (size_t)f * plane;
  const int nruns = r[Hp];
  const int32_t* bidx = L + nruns;  // k_run_border: border index of each root run
  int nb = st[f].n_borders;
  if (nb > border_cap) nb = border_cap;
  SegTab T = seg_tab(scratch + 4 * (size_t)f * pool_cap, pool_cap);
  if (nb > T.cap) {  // a contour pool too small for one record per border
    if (t == 0) atomicOr(&st[f].overflow, 2);
    nb = T.cap;
  }
  const Border* bs = borders + (size_t)f * border_cap;
  const int nsr = M > 0 ? (Hp - 2) / M : 0;  // sampled rows y = M, 2M, .. <= Hp - 2
  bool split = M > 0 && nsr > 0 && nsr <= kSegRows && 2 * (size_t)nruns <= plane;
  // checkpoint ids: 2 per foreground run of each sampled row
  static_assert(kSegRows <= 512, "two passes of 256 sampled rows");
  int carry = 0;
  for (int pass = 0; pass < 2; pass++) {
    int v = 0;
    const int k = pass * 256 + t;
    if (split && k < nsr) {
      const int y = (k + 1) * M;
      v = 2 * ((r[y + 1] - r[y] - 1) >> 1);
    }
    const int inc = wave_incl_scan(v, lane);
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    int o = carry;
    for (int q = 0; q < wave; q++) o += wsum[q];
    if (k < kSegRows) rb[k] = o + inc - v;
    carry += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  int NC = split ? carry : 0;
  if (NC + nb > T.cap) {
    split = false;
    NC = 0;
  }
  if (t == 0) {
    st[f].seg_nc = NC;
    st[f].seg_m = split ? M : 0;
  }
  for (int k = t; k < nsr && split; k += 256) T.rowbase[k] = rb[k];
  const BitsRows nbh{dbits + (size_t)f * dstride, dbits_wpw(Wp)};
  if (split) {
    for (int k = 0; k < nsr; k++) {
      const int y = (k + 1) * M, j0 = r[y], nfg = (r[y + 1] - j0 - 1) >> 1;
      for (int i = t; i < nfg; i += 256) {
        const int g = j0 + 2 * i + 1;
        const int x0 = X[g], x1 = (int)X[g + 1] - 1;
        const int fr = uf_find_c(L, g);
        const int id = rb[k] + 2 * i;
        // west visit of x0: the border against the background run on the left
        {
          const int bg = uf_find_c(L, g - 1);
          const int own = (bg != 0 && uf_find_c(L, bg - 1) == fr) ? bg : fr;
          const uint32_t m = nbh(x0, y);
          const int sd = first_cw(m, 4);
          T.border[id] = bidx[own];
          T.pos[id] = (int32_t)wpos(x0, y);
          T.sdir[id] = sd == 4 ? kSegSingle : sd;
          T.next[id] = -1;
          T.cnt[id] = 0;
        }
        // east visit of x1 (for a one-pixel run, the west visit when its arc also holds east)
        {
          const int bg = uf_find_c(L, g + 1);
          const int own = (bg != 0 && uf_find_c(L, bg - 1) == fr) ? bg : fr;
          const uint32_t m = nbh(x1, y);
          int sd = first_cw(m, 0);
          if (sd == 0) {
            sd = kSegUnused;  // isolated pixel: its west visit is the border
          } else if (x1 == x0) {
            const int sw = first_cw(m, 4);
            const uint32_t rr = ((m | (m << 8)) >> (sw + 1)) & 0xffu;
            if (arc_has(sw, (sw + 1 + __builtin_ctz(rr)) & 7, 0)) sd = kSegUnused;
          }
          T.border[id + 1] = bidx[own];
          T.pos[id + 1] = (int32_t)wpos(x1, y);
          T.sdir[id + 1] = sd;
          T.next[id + 1] = -1;
          T.cnt[id + 1] = 0;
        }
      }
    }
  }
  __syncthreads();  // the checkpoints' kinds, for the aliases below
  // start segments
  for (int b = t; b < nb; b += 256) {
    const Border bb = bs[b];
    const int sx = bb.start % Wp, sy = bb.start / Wp, id = NC + b;
    T.border[id] = b;
    T.cnt[id] = 0;
    T.pos[id] = (int32_t)wpos(sx, sy);
    if (split && sy % M == 0 && sy <= Hp - 2) {
      T.sdir[id] = kSegAlias;
      int c = seg_id_at(sx, sy, bb.hole ? 1 : 0, M, r, X, rb);
      if (T.sdir[c] == kSegUnused) c--;  // a one-pixel run whose west visit is also its east one
      T.next[id] = c;
    } else {
      T.sdir[id] = kSegStart;
      T.next[id] = -1;
    }
  }
}

// Per border, its segments in walk order from the start: offsets of their
// points, the border's point count; then every chunk gets its border and
// its points' positions in the border's list. A chain that does not close
// within the frame's segment count, or that passes a segment planned for
// another border, marks the frame overflowed (its quads are dropped).
__global__ __launch_bounds__(256) void k_seg_chain(FrameState* st, int32_t* __restrict__ counts,
                                                   int32_t* __restrict__ scratch, int pool_cap, int border_cap) {
  const int f = blockIdx.x, t = threadIdx.x;
  int nb = st[f].n_borders;
  if (nb > border_cap) nb = border_cap;
  int32_t* sc = scratch + 4 * (size_t)f * pool_cap;
  SegTab T = seg_tab(sc, pool_cap);
  int32_t* cnt = counts + (size_t)f * border_cap;
  for (int b = T.cap + t; b < nb; b += 256) cnt[b] = 0;  // past the segment table (overflow flagged)
  if (nb > T.cap) nb = T.cap;
  const int NC = st[f].seg_nc, NS = NC + nb;
  for (int b = t; b < nb; b += 256) {
    // from the start's segment until the walk is back at the start: a segment
    // ends at the start checkpoint (aliased starts) or on the closing move (-1)
    const int start = T.sdir[NC + b] == kSegAlias ? T.next[NC + b] : NC + b;
    int cur = start, acc = 0, k = 0;
    bool bad = false;
    do {
      if (++k > NS || T.border[cur] != b) {
        bad = true;
        break;
      }
      T.off[cur] = acc;
      acc += T.cnt[cur];
      cur = T.next[cur];
    } while (cur >= 0 && cur != start);
    cnt[b] = acc;
    if (bad) atomicOr(&st[f].overflow, 2);
  }
  __syncthreads();
  const int max_chunks = pool_cap / kChunk;
  int nch = st[f].n_chunks;
  if (nch > max_chunks) nch = max_chunks;
  int32_t* owner = sc + 2 * (size_t)pool_cap;
  int32_t* ordv = owner + max_chunks;
  for (int c = t; c < nch; c += 256) {
    const int sg = owner[c];
    owner[c] = T.border[sg];
    ordv[c] += T.off[sg];
  }
}

// 1. follow every border once: MK_TB_WAVES waves per frame (the tiled bit
// plane in L2), each lane walking one segment at a time (k_seg_plan; a whole
// border when the frame is not split) and refilled from the frame's segment
// list (an LDS counter) once a quarter of its wave is idle, so a frame costs
// about its steps over its lanes instead of its longest border (the outer
// border of the grid lines, ~5-9k steps). Points go to 16-point chunks handed
// out by a per-frame counter; k_seg_chain orders them.
#ifndef MK_TB_WAVES
#define MK_TB_WAVES 4
#endif
__global__ __launch_bounds__(64 * MK_TB_WAVES) void k_trace_borders(const uint32_t* __restrict__ tbits, size_t tstride,
                                                      const Border* __restrict__ borders, FrameState* st,
                                                      int32_t* __restrict__ scratch, int pool_cap, int Wp,
                                                      int border_cap, const int32_t* __restrict__ rowb,
                                                      size_t rstride, const uint16_t* __restrict__ rx, size_t plane) {
  const uint64_t t_start = wall_clock64();
  __shared__ uint8_t next_lut[512 * 8];
  __shared__ int32_t next_job;
  const int f = blockIdx.x, lane = threadIdx.x & 63;
  build_next_lut(next_lut, threadIdx.x, blockDim.x);
  if (threadIdx.x == 0) next_job = 0;
  __syncthreads();
  int nb = st[f].n_borders;
  if (nb > border_cap) nb = border_cap;
  const uint32_t* B = tbits + (size_t)f * tstride;
  const int wpw = dbits_wpw(Wp);
  const Border* bs = borders + (size_t)f * border_cap;
  int32_t* sc = scratch + 4 * (size_t)f * pool_cap;
  const int max_chunks = pool_cap / kChunk;
  int32_t* chunks = sc;                        // [0, 2 pool_cap)
  int32_t* owner = sc + 2 * (size_t)pool_cap;  // [2 pool_cap, + max_chunks)
  int32_t* ordv = owner + max_chunks;
  int32_t* ccount = ordv + max_chunks;
  const SegTab T = seg_tab(sc, pool_cap);
  if (nb > T.cap) nb = T.cap;  // k_seg_plan flagged the frame
  const int NC = st[f].seg_nc, M = st[f].seg_m, NS = NC + nb;
  const int32_t* r = rowb + (size_t)f * rstride;
  const uint16_t* X = rx + (size_t)f * plane;
  const BitsTiled nbh{B, tb_groups(Wp)};
  int32_t* smax = &st[f].trace_steps_max;
  ChunkEmit em{chunks, owner, ordv, ccount, &st[f].n_chunks, max_chunks, 0, -1, 0, 0, false};
  Walk w;
  int i = -1;
  bool act = false;
  bool exhausted = NS == 0;  // wave-uniform
  const uint64_t below = (1ull << lane) - 1;
  const auto finish = [&](int nx) {
    T.cnt[i] = w.n;
    T.next[i] = nx;
    em.flush();
    if (em.ovf) atomicOr(&st[f].overflow, 2);
    atomicMax(smax, w.steps);
    atomicAdd(&st[f].trace_steps_sum, w.steps);
  };
  for (;;) {
    const uint64_t idle = __ballot(!act);
    const int nidle = __popcll(idle);
    if (!exhausted && (nidle >= 16 || nidle == 64)) {
      const int leader = __ffsll((unsigned long long)idle) - 1;
      int next = 0;
      if (lane == leader) next = atomicAdd(&next_job, nidle);
      next = __shfl(next, leader);
      if (next + nidle >= NS) exhausted = true;
      if (!act) {
        const int j = next + __popcll(idle & below);
        if (j < NS) {
          const int sd = T.sdir[j];
          if (sd != kSegUnused && sd != kSegAlias) {
            i = j;
            const Border b = bs[T.border[j]];
            em.border = j; em.cur = -1; em.k = 0; em.nch = 0; em.ovf = false;
            if (sd == kSegStart) {
              act = walk_start(nbh, b.start % Wp, b.start / Wp, b.hole != 0, em, w);
              w.first = 0;
              if (!act) finish(-1);
            } else if (sd == kSegSingle) {
              const uint32_t p = (uint32_t)T.pos[j];
              em((int)(p & 0xffffu) - 1, (int)(p >> 16) - 1);
              w.n = 1;
              w.steps = 0;
              finish(-1);
            } else {
              seg_begin(nbh, b, Wp, (uint32_t)T.pos[j], sd, w);
              act = true;
            }
          }
        }
      }
      continue;
    }
    if (nidle == 64) {
      if (exhausted) break;
      continue;
    }
    int nx = -1;
    if (act && !walk_step(nbh.b, nbh.G, next_lut, em, w, M, r, X, T.rowbase, nx)) {
      act = false;
      finish(nx);
    }
  }
  if (lane == 0) atomicMax(&st[f].trace_ticks, (int32_t)(wall_clock64() - t_start));
}

// Latency variant of k_trace_borders for small batches: one 1024-thread block
// per frame stages the padded bit plane in LDS (when it fits), so each step of
// a walk waits on an LDS read instead of an L2 round trip -- the longest walk of
// a frame is on the per-rig latency path.
extern __shared__ uint32_t tb_lds[];
struct BitsNBLds {
  int wpw;
  __device__ uint32_t row3(int x, int y) const {
    const int o = y * wpw + ((x - 1) >> 5);
    const uint64_t v = ((uint64_t)tb_lds[o + 1] << 32) | tb_lds[o];
    return (uint32_t)(v >> ((x - 1) & 31)) & 7u;
  }
  __device__ uint32_t operator()(int x, int y) const { return nb8_from_rows(row3(x, y - 1), row3(x, y), row3(x, y + 1)); }
};
// one segment (k_seg_plan) on the LDS plane: the same walk as walk_step
template <class NB, class EM>
__device__ inline int walk_segment_lds(const NB& nb, const uint8_t* lut, EM& em, const Border& b, int Wp,
                                       uint32_t pos, int sd, int M, const int32_t* r, const uint16_t* X,
                                       const int32_t* rowbase, int& steps) {
  Walk w;
  if (sd == kSegStart) {
    if (!walk_start(nb, b.start % Wp, b.start / Wp, b.hole != 0, em, w)) {
      steps = 0;
      return -1;
    }
    w.first = 0;
  } else {
    seg_begin(nb, b, Wp, pos, sd, w);
  }
  for (;;) {
    const int x = (int)(w.pos & 0xffffu), y = (int)(w.pos >> 16);
    const uint32_t p9 = nb.row3(x, y - 1) | (nb.row3(x, y) << 3) | (nb.row3(x, y + 1) << 6);
    const int s = lut[(p9 << 3) | w.s];
    if (M > 0 && !w.first && y % M == 0) {
      const bool west = arc_has(w.s, s, 4);
      if (west || arc_has(w.s, s, 0)) {
        steps = w.steps;
        em.n_pts = w.n;
        return seg_id_at(x, y, west ? 0 : 1, M, r, X, rowbase);
      }
    }
    w.first = 0;
    if (s != w.prev_s) {
      em(x - 1, y - 1);
      w.n++;
      w.prev_s = s;
    }
    const uint32_t np = w.pos + wdelta(s);
    if (np == w.spos && w.pos == w.p1) break;
    w.pos = np;
    w.s = (s + 4) & 7;
    w.steps++;
  }
  steps = w.steps;
  em.n_pts = w.n;
  return -1;
}
// Latency path (small batches): one 1024-thread block per frame, the padded
// bit plane in LDS (ds_read per step instead of an L2 round trip), threads
// taking the frame's segments from an LDS counter (a frame's longest border,
// ~5-9k steps, was the rig latency's walk; split it is a few hundred).
__global__ __launch_bounds__(1024) void k_trace_borders_lds(const uint32_t* __restrict__ dbits, size_t dstride,
                                                            const Border* __restrict__ borders, FrameState* st,
                                                            int32_t* __restrict__ scratch, int pool_cap, int Wp,
                                                            int Hp, int border_cap, const int32_t* __restrict__ rowb,
                                                            size_t rstride, const uint16_t* __restrict__ rx,
                                                            size_t plane) {
  __shared__ uint8_t next_lut[512 * 8];
  __shared__ int32_t next_job;
  const int f = blockIdx.x;
  build_next_lut(next_lut, threadIdx.x, blockDim.x);
  if (threadIdx.x == 0) next_job = 0;
  const int wpw = dbits_wpw(Wp);
  const uint32_t* B = dbits + (size_t)f * dstride;
  for (int k = threadIdx.x; k < wpw * Hp; k += blockDim.x) tb_lds[k] = B[k];
  __syncthreads();
  int nb = st[f].n_borders;
  if (nb > border_cap) nb = border_cap;
  const Border* bs = borders + (size_t)f * border_cap;
  int32_t* sc = scratch + 4 * (size_t)f * pool_cap;
  const int max_chunks = pool_cap / kChunk;
  int32_t* chunks = sc;
  int32_t* owner = sc + 2 * (size_t)pool_cap;
  int32_t* ordv = owner + max_chunks;
  const SegTab T = seg_tab(sc, pool_cap);
  if (nb > T.cap) nb = T.cap;  // k_seg_plan flagged the frame
  const int NC = st[f].seg_nc, M = st[f].seg_m, NS = NC + nb;
  const int32_t* r = rowb + (size_t)f * rstride;
  const uint16_t* X = rx + (size_t)f * plane;
  const BitsNBLds nbh{wpw};
  for (;;) {
    int j = 0;
    j = atomicAdd(&next_job, 1);
    if (j >= NS) break;
    const int sd = T.sdir[j];
    if (sd == kSegUnused || sd == kSegAlias) continue;
    const Border b = bs[T.border[j]];
    ChunkEmit em{chunks, owner, ordv, ordv + max_chunks, &st[f].n_chunks, max_chunks, j, -1, 0, 0, false};
    int steps = 0, nx = -1;
    if (sd == kSegSingle) {
      const uint32_t p = (uint32_t)T.pos[j];
      em((int)(p & 0xffffu) - 1, (int)(p >> 16) - 1);
      em.n_pts = 1;
    } else {
      nx = walk_segment_lds(nbh, next_lut, em, b, Wp, (uint32_t)T.pos[j], sd, M, r, X, T.rowbase, steps);
    }
    T.cnt[j] = em.n_pts;
    T.next[j] = nx;
    em.flush();
    if (em.ovf) atomicOr(&st[f].overflow, 2);
    atomicMax(&st[f].trace_steps_max, steps);
  }
}

#ifndef MK_FC_CPL
#define MK_FC_CPL 2  // compaction points per lane (k_frame_contours step 3)
#endif
#ifndef MK_FC_CU
#define MK_FC_CU 8  // compaction trips in flight per wave (k_frame_contours step 3)
#endif
// 5 waves per SIMD (96 VGPRs, 32 B of spills) rather than the 106 VGPRs / 4
// waves the 1024-thread bound allows: in throughput mode (256-thread blocks)
// a fifth block per CU, 5.34 -> 4.75 ms per 4096 frames
#ifndef MK_FC_WPE
#define MK_FC_WPE 5
#endif
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(MK_FC_WPE))) void k_frame_contours(const uint32_t* __restrict__ dbits, size_t dstride,
                                                         const Border* __restrict__ borders,
                                                         FrameState* st, int32_t* __restrict__ counts,
                                                         int32_t* __restrict__ offs, int32_t* __restrict__ pool,
                                                         int32_t* __restrict__ scratch, int pool_cap,
                                                         QuadRec* __restrict__ quads, FrameDebug* dbg,
                                                         const FrameDesc* __restrict__ frames, int Wp, int Hp,
                                                         size_t plane, int border_cap, double eps, double search_mult,
                                                         const int32_t* __restrict__ rowb, size_t rstride,
                                                         const uint16_t* __restrict__ rx) {
  __shared__ int32_t scan[1024];
  __shared__ RawQuad raw[kMaxQuads];
  __shared__ int32_t nraw, total, nkeep;
  __shared__ int32_t idx4[kMaxQuads][4];
  __shared__ int32_t nbr[kMaxQuads];
  __shared__ int32_t kpos[kMaxQuads];
  __shared__ int32_t ord[kMaxQuads];
  __shared__ float qcx[kMaxQuads], qcy[kMaxQuads];
  __shared__ double qside[kMaxQuads];
  __shared__ int32_t nchunk, nlong;
  __shared__ int32_t longs[kMaxLong];
  const int f = blockIdx.x;
  const int tid = threadIdx.x;
  const uint32_t* B = dbits + (size_t)f * dstride;
  const int wpw = dbits_wpw(Wp);
  const Border* bs = borders + (size_t)f * border_cap;
  int32_t* cnt = counts + (size_t)f * border_cap;
  int32_t* off = offs + (size_t)f * border_cap;
  uint32_t* pl = (uint32_t*)(pool + 2 * (size_t)f * pool_cap);  // the border points, packed (PtPacked)
  int32_t* sc = scratch + 4 * (size_t)f * pool_cap;
  int nb = st[f].n_borders;
  if (nb > border_cap) nb = border_cap;
  auto emit_raw = [&](int i, const int32_t* q4) {
    const int q = atomicAdd(&nraw, 1);
    if (q < kMaxQuads) {
      for (int k = 0; k < 8; k++) raw[q].c[k] = q4[k];
      int par = bs[i].parent;
      if (par < 0) {  // a hole's parent as its component's root run (k_run_border): that run's key
        const int pr = -par - 1;
        par = run_at_row(rowb + (size_t)f * rstride, Hp, pr) * Wp + rx[(size_t)f * plane + pr];
      }
      raw[q].parent = par;
      raw[q].hole = bs[i].hole;
      raw[q].key = bs[i].key;
    } else {
      atomicOr(&st[f].overflow, 4);
    }
  };
  const uint64_t t0 = wall_clock64();
#ifdef MK_HYST_TICKS  // the ticks are k_hyst_band's
#define MK_TICK(k)
#else
#define MK_TICK(k) \
  if (tid == 0) st[f].ticks[k] = (int32_t)(wall_clock64() - t0);
#endif
  if (tid == 0) { nraw = 0; total = 0; nlong = 0; nchunk = st[f].n_chunks; }
  __syncthreads();

  const int max_chunks = pool_cap / kChunk;
  int32_t* chunks = sc;                              // [0, 2 pool_cap), filled by k_trace_borders
  int32_t* owner = sc + 2 * (size_t)pool_cap;        // [2 pool_cap, + max_chunks)
  int32_t* ordv = owner + max_chunks;

  // 2. exclusive scan of the point counts, blockDim at a time: wave scans,
  // then the wave totals (two barriers per chunk; the running total is kept
  // by every thread in a register)
  {
    const int lane = tid & 63, wv = tid >> 6, nwv = blockDim.x >> 6;
    int run = 0;
    for (int base = 0; base < nb; base += blockDim.x) {
      const int i = base + tid;
      const int v = i < nb ? cnt[i] : 0;
      const int inc = wave_incl_scan(v, lane);
      if (lane == 63) scan[wv] = inc;
      __syncthreads();
      int pre = 0, tot = 0;
      for (int k = 0; k < nwv; k++) {
        const int s = scan[k];
        pre += k < wv ? s : 0;
        tot += s;
      }
      if (i < nb) off[i] = run + pre + inc - v;
      run += tot;
      __syncthreads();
    }
    if (tid == 0) total = run;
    __syncthreads();
  }
  if (total > pool_cap || nchunk > max_chunks) {
    if (tid == 0) {
      atomicOr(&st[f].overflow, 2);
      st[f].n_points = total;
      st[f].n_quads = 0;
      st[f].n_raw_quads = 0;
    }
    return;
  }
  MK_TICK(0);  // scan
  // 3. compact: kCPL points per lane (one 4- or 8-byte load of the packed
  // chunk), 64 kCPL / kChunk chunks per wave, kCU wave trips at once: every
  // load of the kCU trips is issued (at a clamped, valid chunk) before any is
  // used, so a trip's chain (chunk count / owner / order, then the border's
  // offset, then the stores) costs one round trip per kCU trips instead of per
  // trip
  if (nchunk > 0) {
    constexpr int kCPL = MK_FC_CPL, LPC = kChunk / kCPL, CPW = 64 / LPC, kCU = MK_FC_CU;
    static_assert(kCPL == 1 || kCPL == 2, "points per lane");
    const int wave = tid >> 6, lane = tid & 63, nwaves = blockDim.x >> 6;
    const int32_t* ccount = ordv + max_chunks;
    const int l = (lane % LPC) * kCPL;  // the lane's first point in its chunk
    const uint32_t* ch = (const uint32_t*)chunks;  // packed points (ChunkEmit)
    typedef __attribute__((aligned(8))) uint2 u2a;
    for (int c0 = wave * CPW * kCU; c0 < nchunk; c0 += nwaves * CPW * kCU) {
      int cc[kCU], b[kCU], k[kCU], o[kCU];
      uint32_t v[kCU][kCPL];
#pragma unroll
      for (int u = 0; u < kCU; u++) {
        const int c = min(c0 + u * CPW + lane / LPC, nchunk - 1);
        cc[u] = c0 + u * CPW + lane / LPC < nchunk ? ccount[c] : 0;
        b[u] = owner[c];
        k[u] = ordv[c] + l;
        if (kCPL == 2) {
          const uint2 w = *(const u2a*)(ch + (size_t)c * kChunk + l);
          v[u][0] = w.x;
          v[u][kCPL - 1] = w.y;
        } else {
          v[u][0] = ch[(size_t)c * kChunk + l];
        }
      }
#pragma unroll
      for (int u = 0; u < kCU; u++) o[u] = off[b[u]];
#pragma unroll
      for (int u = 0; u < kCU; u++)  // packed x | y << 16 (PtPacked)
#pragma unroll
        for (int e = 0; e < kCPL; e++)
          if (l + e < cc[u]) pl[(size_t)o[u] + k[u] + e] = v[u][e];
    }
  }
  __syncthreads();
  MK_TICK(1);  // compaction
  // 4. approxPolyDP per border (eps = POLYGON_EPSILON, closed, quad early
  // exit). Borders longer than kLongBorder points take a whole wave
  // (approx_poly_wave); the others one lane each, ordered by length (counting
  // sort on count / 4, longest first) so the 64 lanes of a wave trip walk
  // borders of about one length instead of idling behind the longest of a
  // random 64 (DP per lane is a serial loop; a trip lasts its longest lane).
  // Waves take the long borders first, then 64 short ones at a time, from LDS
  // counters. The result does not depend on the order: emit_raw's slots are
  // re-ordered by CCOMP key below.
  __shared__ int32_t hist[33], nshort, next_long, next_short;
  __shared__ int32_t wstk[16][2 * kWaveStk];  // each wave's DP stack for the long borders
  if (tid < 33) hist[tid] = 0;
  if (tid == 0) { next_long = 0; next_short = 0; }
  __syncthreads();
  bool sorted = nb <= 1024;  // the order lives in scan[] (free after step 2)
  if (sorted) {
    for (int i = tid; i < nb; i += blockDim.x) {
      const int c = cnt[i];
      if (c > kLongBorder) {
        const int k = atomicAdd(&nlong, 1);
        if (k < kMaxLong) longs[k] = i;
      } else {
        atomicAdd(&hist[c >> 2], 1);
      }
    }
    __syncthreads();
    sorted = nlong <= kMaxLong;
    if (sorted) {
      if (tid == 0) {
        int acc = 0;
        for (int b = 32; b >= 0; b--) {
          const int h = hist[b];
          hist[b] = acc;
          acc += h;
        }
        nshort = acc;
      }
      __syncthreads();
      for (int i = tid; i < nb; i += blockDim.x) {
        const int c = cnt[i];
        if (c <= kLongBorder) scan[atomicAdd(&hist[c >> 2], 1)] = i;
      }
      __syncthreads();
      const int lane = tid & 63;
      for (;;) {
        int k = 0;
        if (lane == 0) k = atomicAdd(&next_long, 1);
        k = __shfl(k, 0);
        if (k >= nlong) break;
        const int i = longs[k], o = off[i], c = cnt[i];
        int32_t* dst = sc + 4 * (size_t)o;
        int32_t* stk = dst + 2 * (size_t)c;
        // the DP stack in the wave's LDS slice (one L2 round trip less per DP
        // step); a deeper stack runs the border again on the global one
        int m = approx_poly_wave(pl + o, c, eps, dst, (lds_i32*)wstk[tid >> 6], 10, kWaveStk);
        if (m < 0) m = approx_poly_wave(pl + o, c, eps, dst, stk, 10);
        if (m == 4 && lane == 0) emit_raw(i, dst);
      }
#ifdef MK_FC_TICK_SPLIT  // diagnostics (tools/fc_ticks.py): tick 2 = the long borders' end, tick 3 = the short ones'
      MK_TICK(2);
#endif
      for (;;) {
        int k = 0;
        if (lane == 0) k = atomicAdd(&next_short, 64);
        k = __shfl(k, 0);
        if (k >= nshort) break;
        if (k + lane < nshort) {
          const int i = scan[k + lane], o = off[i], c = cnt[i];
          int32_t* dst = sc + 4 * (size_t)o;
          int32_t* stk = dst + 2 * (size_t)c;
          const int m = approx_poly(PtPacked{pl + o}, c, eps, true, dst, stk, 10);
          if (m == 4) emit_raw(i, dst);
        }
      }
      __syncthreads();
#ifdef MK_FC_TICK_SPLIT
      MK_TICK(3);
#else
      MK_TICK(2);  // approx (sorted)
#endif
    } else {
      __syncthreads();
      if (tid == 0) nlong = 0;
      __syncthreads();
    }
  }
  if (!sorted) {  // more than 1024 borders or kMaxLong long ones: borders in index order
    for (int i = tid; i < nb; i += blockDim.x) {
      const int o = off[i], c = cnt[i];
      if (c > kLongBorder) {
        const int k = atomicAdd(&nlong, 1);
        if (k < kMaxLong) { longs[k] = i; continue; }
      }
      int32_t* dst = sc + 4 * (size_t)o;
      int32_t* stk = dst + 2 * (size_t)c;
      int m = approx_poly(PtPacked{pl + o}, c, eps, true, dst, stk, 10);
      if (m == 4) emit_raw(i, dst);
    }
    __syncthreads();
    MK_TICK(2);  // short-border approx (threads)
    {
      const int wave = tid >> 6, nwaves = blockDim.x >> 6;
      const int nl = nlong < kMaxLong ? nlong : kMaxLong;
      for (int k = wave; k < nl; k += nwaves) {
        const int i = longs[k], o = off[i], c = cnt[i];
        int32_t* dst = sc + 4 * (size_t)o;
        int32_t* stk = dst + 2 * (size_t)c;
        const int m = approx_poly_wave(pl + o, c, eps, dst, stk, 10);
        if (m == 4 && (tid & 63) == 0) emit_raw(i, dst);
      }
    }
  }
  __syncthreads();
#ifndef MK_FC_TICK_SPLIT
  MK_TICK(3);  // long-border approx (waves)
#endif
  const int nq = nraw < kMaxQuads ? nraw : kMaxQuads;
  // position in the CCOMP output order (keys are distinct)
  for (int i = tid; i < nq; i += blockDim.x) {
    int r = 0;
    for (int j = 0; j < nq; j++)
      if (ccomp_before(raw[j].parent, raw[j].hole, raw[j].key, raw[i].parent, raw[i].hole, raw[i].key)) r++;
    ord[r] = i;
  }
  __syncthreads();
  // Quadrilateral(approx) (QuadDetection.h:23-61): float centre, int side
  for (int r = tid; r < nq; r += blockDim.x) {
    const RawQuad& q = raw[ord[r]];
    int dx = q.c[0] - q.c[2], dy = q.c[1] - q.c[3];
    qside[r] = sqrt((double)(dx * dx + dy * dy));
    float xs = 0, ys = 0;
    for (int k = 0; k < 4; k++) { xs += (float)q.c[2 * k]; ys += (float)q.c[2 * k + 1]; }
    qcx[r] = xs / (float)4;
    qcy[r] = ys / (float)4;
  }
  __syncthreads();
  // removeDuplicateQuads (QuadDetection.h:115-171) with an exact radius
  // search: squared float distance <= radius, the 4 smallest (dist, index)
  // hits per query zero-padded; then the order-dependent sweep.
  for (int i = tid; i < nq; i += blockDim.x) {
    float radius = (float)(search_mult * qside[i]);
    float bd[4] = {0, 0, 0, 0};
    int bi[4] = {0, 0, 0, 0};
    int nh = 0;
    for (int j = 0; j < nq; j++) {
      float d0 = qcx[j] - qcx[i], d1 = qcy[j] - qcy[i];
      float dist = 0.0f;
      dist += d0 * d0;
      dist += d1 * d1;
      if (dist <= radius) {
        int pos = nh < 4 ? nh : 4;
        while (pos > 0 && (dist < bd[pos - 1] || (dist == bd[pos - 1] && j < bi[pos - 1]))) {
          if (pos < 4) { bd[pos] = bd[pos - 1]; bi[pos] = bi[pos - 1]; }
          pos--;
        }
        if (pos < 4) { bd[pos] = dist; bi[pos] = j; }
        if (nh < 4) nh++;
      }
    }
    for (int k = 0; k < 4; k++) idx4[i][k] = k < nh ? bi[k] : 0;
    nbr[i] = 0;
  }
  __syncthreads();
  if (tid == 0) {
    for (int i = 0; i < nq; i++) {
      if (nbr[i]) continue;
      for (int k = 1; k < 4; k++) nbr[idx4[i][k]] = 1;
    }
    int n = 0;
    for (int i = 0; i < nq; i++) {
      kpos[i] = nbr[i] ? -1 : n;
      if (!nbr[i]) n++;
    }
    nkeep = n;
    st[f].n_raw_quads = nraw;
    st[f].n_quads = n;
    st[f].n_points = total;
    dbg[f].n_raw_quads = nraw;
    dbg[f].n_quads = n;
  }
  __syncthreads();
  MK_TICK(4);  // CCOMP order, duplicates
  const FrameDesc fd = frames[f];
  for (int r = tid; r < nq; r += blockDim.x) {
    int k = kpos[r];
    if (k < 0) continue;
    const RawQuad& rq = raw[ord[r]];
    QuadRec q;
    for (int c = 0; c < 8; c++) q.c[c] = rq.c[c];
    q.parent = rq.parent; q.hole = rq.hole; q.key = rq.key; q.keep = 1;
    q.cx = qcx[r]; q.cy = qcy[r]; q.side = qside[r];
    for (int c = 0; c < 4; c++) {
      // test points: float((pt - centre) * 1.3) + centre, widened to double
      float dxf = (float)q.c[2 * c] - q.cx, dyf = (float)q.c[2 * c + 1] - q.cy;
      float sx = (float)(dxf * 1.3), sy = (float)(dyf * 1.3);
      double ox, oy;
      undistort(fd.cam, (double)(sx + q.cx), (double)(sy + q.cy), &ox, &oy);
      q.tp[2 * c] = ox;
      q.tp[2 * c + 1] = oy;
    }
    quads[(size_t)f * kMaxQuads + k] = q;
    for (int c = 0; c < 8; c++) { dbg[f].quads[k][c] = q.c[c]; dbg[f].test_pts[k][c] = q.tp[c]; }
  }
  __syncthreads();
  MK_TICK(5);  // end
#undef MK_TICK
}

// ================================================================ RPP
// Phases (mk_rpp.h): first ObjPose per (frame, quad, orientation); Get2ndPose
// per item; one ObjPose per surviving 2nd-pose candidate; ordered merge.
// The two ObjPose phases are job queues served by persistent lanes
// (k_objpose_q): a lane whose ObjPose converged writes it out and takes the
// next job, so a wave is not held by its slowest lane (first-ObjPose
// iteration counts run from ~10 to ~600, candidate ones from 1 to ~800).
// gridSquarePossibilities (Mantis3Params.h:102-123): #0 CCW, #1 mirrored.
struct RppItem {
  rpp::Stage1 s;   // s.Q holds the image points until the first ObjPose rewrites them
  double P[12];
  int32_t active, pad;
};
// queue control per phase: [0] job count, [1] next job
struct RppQueue {
  int32_t n0, next0, n1, next1;
};

__global__ __launch_bounds__(256) void k_rpp_prep(const QuadRec* __restrict__ quads, const FrameState* __restrict__ st,
                                                  RppItem* __restrict__ items, int32_t* __restrict__ jobs,
                                                  RppQueue* q, double half) {
  const int f = blockIdx.y;
  const int item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= kMaxQuads * 2) return;
  const int qd = item >> 1, o = item & 1;
  const size_t slot = (size_t)f * kMaxQuads * 2 + item;
  RppItem& it = items[slot];
  if (qd >= st[f].n_quads) { it.active = 0; return; }
  const QuadRec& Q = quads[(size_t)f * kMaxQuads + qd];
  const double sx0[4] = {half, -half, -half, half};
  const double sy0[4] = {half, half, -half, -half};
  const double sy1[4] = {-half, -half, half, half};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    it.P[k] = sx0[k];
    it.P[4 + k] = o == 0 ? sy0[k] : sy1[k];
    it.P[8 + k] = 0.0;
    it.s.Q[k] = Q.tp[2 * k];
    it.s.Q[4 + k] = Q.tp[2 * k + 1];
    it.s.Q[8 + k] = 1.0;
  }
  it.active = 1;
  // the first ObjPose of orientation 1 is orientation 0's mirrored (op_end<0>):
  // only orientation 0 items enter the first queue
  if (o == 0) jobs[atomicAdd(&q->n0, 1)] = (int32_t)slot;
}

__global__ __launch_bounds__(256) void k_rpp_prep_api(const double* __restrict__ img_pts,
                                                      const double* __restrict__ obj_pts, int n,
                                                      RppItem* __restrict__ items, int32_t* __restrict__ jobs,
                                                      RppQueue* q) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  RppItem& it = items[i];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    it.P[k] = obj_pts[12 * i + 3 * k];
    it.P[4 + k] = obj_pts[12 * i + 3 * k + 1];
    it.P[8 + k] = obj_pts[12 * i + 3 * k + 2];
    it.s.Q[k] = img_pts[8 * i + 2 * k];
    it.s.Q[4 + k] = img_pts[8 * i + 2 * k + 1];
    it.s.Q[8 + k] = 1.0;
  }
  it.active = 1;
  jobs[i] = i;
  if (i == 0) q->n0 = n;
}

// Persistent ObjPose lanes. MODE 0: job = item slot, first ObjPose (no initial
// rotation) into items[].s. MODE 1: job = item * kCand + j, candidate ObjPose
// from s.sR[j] into rf[job]. A wave refills its idle lanes with one atomic
// when at least a quarter of them are idle (or all are), so the setup of new
// jobs is shared by many lanes.
template <int MODE>
__device__ inline void op_begin(RppItem* items, int32_t job, rpp::OpState& s) {
  const int32_t p = MODE == 0 ? job : job / rpp::kCand;
  rpp::M34 P, Q;
  const RppItem& it = items[p];
#pragma unroll
  for (int k = 0; k < 12; k++) { P.a[k] = it.P[k]; Q.a[k] = it.s.Q[k]; }
  if (MODE == 0) {
    rpp::op_setup(P, Q, nullptr, s);
#pragma unroll
    for (int k = 0; k < 12; k++) items[p].s.Q[k] = Q.a[k];
  } else {
    const int j = job - p * rpp::kCand;
    rpp::M33 R0;
#pragma unroll
    for (int k = 0; k < 9; k++) R0.a[k] = it.s.sR[j][k];
    rpp::op_setup(P, Q, &R0, s);
  }
}

// Pipeline items come in orientation pairs (k_rpp_prep: slot = 2 quad + o)
// whose model squares are mirror images in y (sy1 = -sy0, z = 0). The first
// ObjPose of the pair is then one computation: every quantity it forms is
// the same for both or changes sign exactly (negation is exact), and the
// result of orientation 1 is R1 = R0 diag(1, -1, -1) with t, both errors, the
// iteration count, the stop code and the rewritten image points identical --
// R1 P1 = R0 P0 since the model's z row is zero. Checked bit for bit on the
// host build (mk_rpp.h) over the bench scene's quads (tools/rpp_mirror_check.py)
// and end to end by the GPU parity tests against the oracle, which computes
// both orientations.
template <int MODE>
__device__ inline void op_end(RppItem* items, rpp::Refine* rf, FrameState* st, int32_t job, const rpp::OpState& s,
                              int code, bool paired) {
  if (st) {
    const int32_t p = MODE == 0 ? job : job / rpp::kCand;
    atomicAdd(&st[p / (kMaxQuads * 2)].rpp_iters[MODE], s.it);
  }
  rpp::M33 R;
  rpp::M31 t;
  double oe, ie;
  rpp::op_finish(s, R, t, oe, ie);
  if (MODE == 0) {
    rpp::Stage1& o = items[job].s;
#pragma unroll
    for (int k = 0; k < 9; k++) o.R[k] = R.a[k];
#pragma unroll
    for (int k = 0; k < 3; k++) o.t[k] = t.a[k];
    o.obj_err = oe;
    o.img_err = ie;
    o.iterations = s.it;
    o.error = code == 2 ? 2 : 0;
    o.keep_mask = 0;
    if (paired) {
      rpp::Stage1& m = items[job + 1].s;
#pragma unroll
      for (int r = 0; r < 3; r++) {
        m.R[3 * r] = R.a[3 * r];
        m.R[3 * r + 1] = -R.a[3 * r + 1];
        m.R[3 * r + 2] = -R.a[3 * r + 2];
      }
#pragma unroll
      for (int k = 0; k < 3; k++) m.t[k] = t.a[k];
#pragma unroll
      for (int k = 0; k < 12; k++) m.Q[k] = o.Q[k];
      m.obj_err = oe;
      m.img_err = ie;
      m.iterations = s.it;
      m.error = code == 2 ? 2 : 0;
      m.keep_mask = 0;
    }
  } else {
    rpp::Refine& o = rf[job];
#pragma unroll
    for (int k = 0; k < 9; k++) o.R[k] = R.a[k];
#pragma unroll
    for (int k = 0; k < 3; k++) o.t[k] = t.a[k];
    o.obj_err = oe;
    o.img_err = ie;
    o.iterations = s.it;
    o.capped = code == 2 ? 1 : 0;
  }
}

// Tail compaction. A queue's jobs run from ~10 to ~2,700 iterations, so once
// the queue is empty a wave is kept alive by its last few long jobs while its
// other lanes idle -- and it still issues every instruction for 64 lanes
// (rocprofv3: ~10.8k VALU instructions per wave trip against ~2.7k for one
// lane's AbsKernel, profiles/r03_pmc_objpose.json). The queue therefore runs as
// a few rounds (launches) over one grid: in every round but the last, a wave
// whose queue is exhausted and whose busy lanes drop below `spill_below` writes
// their ObjPose states to a pool and exits; the next round starts from that
// pool with the surviving long jobs packed into full waves. A state is copied
// bit for bit (OpState fields as doubles), so every job runs exactly the
// iterations it would have run in place.
constexpr int kOpFields = 80;  // doubles per spilled OpState (76 values + 3 ints + pad)
struct OpPool {
  double* state;   // [kOpFields][cap], SoA so a wave's stores coalesce
  int32_t* job;    // [cap]
  int32_t* ctl;    // [0] entries, [1] next entry to take
};
struct OpRound {
  OpPool in, out;  // in: unused in round 0 (the queue's job list instead)
  int32_t cap;     // entries a pool holds (>= the grid's lanes)
  int32_t first, last, spill_below;
  int32_t lanes;   // lanes per wave that take jobs (64; fewer spreads a small queue over more waves)
  int32_t pad;
};
__device__ inline void op_save(const OpPool& p, int32_t cap, int k, const rpp::OpState& s) {
  double* d = p.state + k;
  int f = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[(size_t)cap * f++] = s.P.a[i];
#pragma unroll
  for (int i = 0; i < 12; i++) d[(size_t)cap * f++] = s.Qi.a[i];
#pragma unroll
  for (int i = 0; i < rpp::NP; i++)
#pragma unroll
    for (int j = 0; j < 6; j++) d[(size_t)cap * f++] = s.F6[i][j];
#pragma unroll
  for (int i = 0; i < 9; i++) d[(size_t)cap * f++] = s.G.a[i];
#pragma unroll
  for (int i = 0; i < 9; i++) d[(size_t)cap * f++] = s.R.a[i];
#pragma unroll
  for (int i = 0; i < 3; i++) d[(size_t)cap * f++] = s.t.a[i];
#pragma unroll
  for (int i = 0; i < 3; i++) d[(size_t)cap * f++] = s.pbar.a[i];
  d[(size_t)cap * f++] = s.old_err;
  d[(size_t)cap * f++] = s.new_err;
  d[(size_t)cap * f++] = s.qx0;
  d[(size_t)cap * f++] = s.qy0;
  d[(size_t)cap * f++] = (double)s.it;
  d[(size_t)cap * f++] = (double)s.init_pass;
  d[(size_t)cap * f++] = (double)s.first;
}
__device__ inline void op_load(const OpPool& p, int32_t cap, int k, rpp::OpState& s) {
  const double* d = p.state + k;
  int f = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s.P.a[i] = d[(size_t)cap * f++];
#pragma unroll
  for (int i = 0; i < 12; i++) s.Qi.a[i] = d[(size_t)cap * f++];
#pragma unroll
  for (int i = 0; i < rpp::NP; i++)
#pragma unroll
    for (int j = 0; j < 6; j++) s.F6[i][j] = d[(size_t)cap * f++];
#pragma unroll
  for (int i = 0; i < 9; i++) s.G.a[i] = d[(size_t)cap * f++];
#pragma unroll
  for (int i = 0; i < 9; i++) s.R.a[i] = d[(size_t)cap * f++];
#pragma unroll
  for (int i = 0; i < 3; i++) s.t.a[i] = d[(size_t)cap * f++];
#pragma unroll
  for (int i = 0; i < 3; i++) s.pbar.a[i] = d[(size_t)cap * f++];
  s.old_err = d[(size_t)cap * f++];
  s.new_err = d[(size_t)cap * f++];
  s.qx0 = d[(size_t)cap * f++];
  s.qy0 = d[(size_t)cap * f++];
  s.it = (int)d[(size_t)cap * f++];
  s.init_pass = (int)d[(size_t)cap * f++];
  s.first = (int)d[(size_t)cap * f++];
}
static_assert(12 + 12 + 6 * rpp::NP + 9 + 9 + 3 + 3 + 4 + 3 <= kOpFields, "OpState fields");

#ifndef MK_OP_WPE
#define MK_OP_WPE 1  // k_objpose_q waves per SIMD the compiler targets (1: up to 512 registers)
#endif
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MK_OP_WPE))) void k_objpose_q(RppItem* __restrict__ items, rpp::Refine* __restrict__ rf,
                                                   const int32_t* __restrict__ jobs, RppQueue* q, FrameState* st,
                                                   int paired, OpRound rd) {
  const int lane = threadIdx.x & 63;
  const int32_t njobs = rd.first ? (MODE == 0 ? q->n0 : q->n1) : min(rd.in.ctl[0], rd.cap);
  int32_t* next = rd.first ? (MODE == 0 ? &q->next0 : &q->next1) : &rd.in.ctl[1];
  rpp::OpState s;
  int32_t job = -1;
  bool exhausted = false;
  const bool eligible = lane < rd.lanes;
  const int refill_at = min(16, rd.lanes);
#pragma unroll 1
  while (true) {
    const uint64_t idle = __ballot(job < 0 && eligible);
    const int nidle = __popcll(idle);
    if (!exhausted && nidle >= refill_at) {
      const int leader = __ffsll((unsigned long long)idle) - 1;
      int base = 0;
      if (lane == leader) base = atomicAdd(next, nidle);
      base = __shfl(base, leader);
      if (base + nidle >= njobs) exhausted = true;
      if (job < 0 && eligible) {  // only the reserved lanes (idle & eligible) take one
        const int k = base + __popcll(idle & ((1ull << lane) - 1));
        if (k < njobs) {
          if (rd.first) {
            job = jobs[k];
            op_begin<MODE>(items, job, s);
          } else {
            job = rd.in.job[k];
            op_load(rd.in, rd.cap, k, s);
          }
        }
      }
    }
    const uint64_t busy = __ballot(job >= 0);
    if (busy == 0) {
      if (exhausted) break;
      continue;
    }
    const int nbusy = __popcll(busy);
    if (exhausted && !rd.last && nbusy < rd.spill_below) {
      // hand the long jobs to the next round and free the SIMD slot. A lane
      // spills at most once per round and the pool holds the grid's lanes
      // (launch_rpp_queues checks), so the reservation always fits; the test
      // below only keeps a misconfigured launch in bounds (the wave then runs on)
      const int leader = __ffsll((unsigned long long)busy) - 1;
      int base = 0;
      if (lane == leader) base = atomicAdd(&rd.out.ctl[0], nbusy);
      base = __shfl(base, leader);
      if (base + nbusy <= rd.cap) {
        if (job >= 0) {
          const int k = base + __popcll(busy & ((1ull << lane) - 1));
          op_save(rd.out, rd.cap, k, s);
          rd.out.job[k] = job;
        }
        break;
      }
      rd.last = 1;
    }
    if (job >= 0) {
      const int code = rpp::op_step(s);
      if (code) {
        op_end<MODE>(items, rf, st, job, s, code, paired != 0);
        job = -1;
      }
    }
  }
}

// Get2ndPose setup (candidate rotations from the quartic) per active item;
// every candidate that enters the search becomes a MODE-1 job. One wave per
// block over the first-ObjPose job list (the active items only): the stage
// needs ~390 registers per lane, so a 64-thread block fits on one SIMD
// instead of waiting for a whole CU to drain.
// two waves per SIMD (256 registers, spilling to scratch) instead of the 512
// (256 VGPRs + 256 AGPRs) the compiler takes by default, which let a wave run
// only on an otherwise empty SIMD: 2.45 -> 2.11 ms isolated per 4096 frames,
// and it fits beside the other contexts' waves
#ifndef MK_S1B_WPE
#define MK_S1B_WPE 2
#endif
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(MK_S1B_WPE))) void k_rpp_s1b(RppItem* __restrict__ items, const int32_t* __restrict__ jobs0,
                                                int32_t* __restrict__ jobs1, RppQueue* q, int paired) {
  const int n0 = q->n0 << (paired ? 1 : 0);  // paired: both orientations of every first-queue job
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n0; k += gridDim.x * blockDim.x) {
    const int32_t i = paired ? jobs0[k >> 1] + (k & 1) : jobs0[k];
    if (!items[i].active) continue;
    double model[12];
#pragma unroll
    for (int j = 0; j < 12; j++) model[j] = items[i].P[j];
    rpp::stage1b(model, items[i].s);
    const int m = items[i].s.error == 1 ? 0 : items[i].s.keep_mask;
    if (m) {
      int b = atomicAdd(&q->n1, __popc(m));
      for (int j = 0; j < rpp::kCand; j++)
        if ((m >> j) & 1) jobs1[b++] = (int32_t)(i * rpp::kCand + j);
    }
  }
}

// RPP's answer per item; with quad_gn_its > 0 (pipeline items, quads given)
// the pose is then refined by the per-quad GN on the quad's 4 undistorted
// test points against the model square (mk_gn.h quad_gn_refine); RPP's
// img_err stays the generateCentralHypotheses gate (HypothesisGeneration.h:80-85)
__global__ __launch_bounds__(256) void k_rpp_merge(const RppItem* __restrict__ items, size_t n_items,
                                                   const rpp::Refine* __restrict__ rf, RppOut* __restrict__ out,
                                                   const QuadRec* __restrict__ quads, int quad_gn_its) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items || !items[i].active) return;
  rpp::Result r = rpp::merge(items[i].s, rf + i * rpp::kCand);
  if (quads && quad_gn_its > 0 && r.error != 1) {
    const QuadRec& Q = quads[i >> 1];  // item = (frame * kMaxQuads + quad) * 2 + orientation
    double obj[12], c0, c1;
    for (int k = 0; k < 4; k++) {
      obj[3 * k] = items[i].P[k];
      obj[3 * k + 1] = items[i].P[4 + k];
      obj[3 * k + 2] = items[i].P[8 + k];
    }
    quad_gn_refine(r.R, r.t, Q.tp, obj, quad_gn_its, &c0, &c1);
  }
  RppOut& R = out[i];
  for (int k = 0; k < 9; k++) R.R[k] = r.R[k];
  for (int k = 0; k < 3; k++) R.t[k] = r.t[k];
  R.img_err = r.img_err;
  R.obj_err = r.obj_err;
  R.status = r.status;
  R.error = r.error;
  R.iterations = r.iterations;
}

// mantis_rpp_solve: RPP::Rpp (RPP.cpp:13-64) on N-point problems, the whole
// solve on one lane (stage1 + candidate ObjPoses + merge, the same functions
// the 4-point queues run in pieces). Off the per-frame path: it exists so any
// point count the reference accepts runs the device code, e.g. demo.cpp:17-38's
// 10-point known answer. img: n x N x 2 normalized (homogeneous z = 1, as
// demo.cpp's Mat::ones and CoPlanarPoseEstimator.cpp:19-34 pack them), obj:
// n x N x 3.
template <int N> struct RppN;
template <> struct RppN<4> {
  static __device__ rpp::Result solve(const double* m, const double* q) { return rpp::solve(m, q); }
};
#define MK_RPP_SOLVE_N(k)                                                                         \
  template <> struct RppN<k> {                                                                    \
    static __device__ rpp::Result solve(const double* m, const double* q) { return rpp::n##k::solve(m, q); } \
  };
MK_RPP_INSTANCES(MK_RPP_SOLVE_N)
#undef MK_RPP_SOLVE_N
template <int N>
__global__ __launch_bounds__(64) void k_rpp_solve(const double* __restrict__ img, const double* __restrict__ obj,
                                                  int n, RppOut* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double model[3 * N], ip[3 * N];
  for (int k = 0; k < N; k++) {
    const size_t p = (size_t)i * N + k;
    model[k] = obj[3 * p];
    model[N + k] = obj[3 * p + 1];
    model[2 * N + k] = obj[3 * p + 2];
    ip[k] = img[2 * p];
    ip[N + k] = img[2 * p + 1];
    ip[2 * N + k] = 1.0;
  }
  const rpp::Result r = RppN<N>::solve(model, ip);
  RppOut& R = out[i];
  for (int k = 0; k < 9; k++) R.R[k] = r.R[k];
  for (int k = 0; k < 3; k++) R.t[k] = r.t[k];
  R.img_err = r.img_err;
  R.obj_err = r.obj_err;
  R.status = r.status;
  R.error = r.error;
  R.iterations = r.iterations;
}

// stage entry mantis_quad_gn: one lane per problem
__global__ __launch_bounds__(256) void k_quad_gn(const double* __restrict__ img, const double* __restrict__ obj, int n,
                                                 double* __restrict__ R, double* __restrict__ t, int its,
                                                 int32_t* __restrict__ steps, double* __restrict__ costs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double Ri[9], ti[3], ip[8], op[12], c0, c1;
  for (int k = 0; k < 9; k++) Ri[k] = R[9 * i + k];
  for (int k = 0; k < 3; k++) ti[k] = t[3 * i + k];
  for (int k = 0; k < 8; k++) ip[k] = img[8 * i + k];
  for (int k = 0; k < 12; k++) op[k] = obj[12 * i + k];
  steps[i] = quad_gn_refine(Ri, ti, ip, op, its, &c0, &c1);
  for (int k = 0; k < 9; k++) R[9 * i + k] = Ri[k];
  for (int k = 0; k < 3; k++) t[3 * i + k] = ti[k];
  costs[2 * i] = c0;
  costs[2 * i + 1] = c1;
}

// ===================================== hypotheses generation + clustering
__device__ inline Xf xf_from_rpp(const RppOut& r) {
  Xf t;
  for (int k = 0; k < 9; k++) t.R[k] = r.R[k];
  for (int k = 0; k < 3; k++) t.t[k] = r.t[k];
  return t;
}

__global__ __launch_bounds__(256) void k_frame_hyps(const RppOut* __restrict__ rpp, FrameState* st,
                                                    HypRec* __restrict__ gen, HypRec* __restrict__ hyps,
                                                    FrameDebug* dbg, double max_quad_error, double max_angle) {
  const int f = blockIdx.x;
  const int tid = threadIdx.x;
  __shared__ int32_t pass_slot[kMaxQuads];
  __shared__ float ax[kMaxHyps], ay[kMaxHyps], az[kMaxHyps];
  __shared__ int32_t cid[kMaxHyps];
  __shared__ int32_t flag[kMaxHyps];
  __shared__ int32_t csize[kMaxHyps];
  __shared__ float cen[3];
  __shared__ int32_t ngen_s, nclus;
  const int nq = st[f].n_quads;
  HypRec* G = gen + (size_t)f * kMaxHyps;
  // per quad: orientation loop with break on camera z >= 0, gate on the last img_err
  for (int q = tid; q < nq; q += blockDim.x) {
    const RppOut& r0 = rpp[((size_t)f * kMaxQuads + q) * 2 + 0];
    const RppOut& r1 = rpp[((size_t)f * kMaxQuads + q) * 2 + 1];
    int ok = 1;
    double err;
    Hyp h;
    if (r0.error == 1) {
      ok = 0;
      err = 0;
    } else {
      hyp_set_c2w(h, xf_from_rpp(r0));
      err = r0.img_err;
      if (!(h.w2c.t[2] >= 0)) {
        if (r1.error == 1) ok = 0;
        else { hyp_set_c2w(h, xf_from_rpp(r1)); err = r1.img_err; }
      }
    }
    pass_slot[q] = (ok && !(err > max_quad_error)) ? 1 : 0;
  }
  __syncthreads();
  if (tid == 0) {
    int n = 0;
    for (int q = 0; q < nq; q++) {
      int p = pass_slot[q];
      pass_slot[q] = p ? n : -1;
      n += p;
    }
    ngen_s = 4 * n;
  }
  __syncthreads();
  const Xf rz = make_rot_z90();
  for (int q = tid; q < nq; q += blockDim.x) {
    int slot = pass_slot[q];
    if (slot < 0) continue;
    const RppOut& r0 = rpp[((size_t)f * kMaxQuads + q) * 2 + 0];
    const RppOut& r1 = rpp[((size_t)f * kMaxQuads + q) * 2 + 1];
    Hyp h;
    hyp_set_c2w(h, xf_from_rpp(r0));
    if (!(h.w2c.t[2] >= 0)) hyp_set_c2w(h, xf_from_rpp(r1));
    for (int k = 0; k < 4; k++) {
      if (k > 0) {
        Hyp n2;
        hyp_set_w2c(n2, xf_mul(rz, h.w2c));
        h = n2;
      }
      HypRec& o = G[4 * slot + k];
      o.c2w = h.c2w; o.w2c = h.w2c; o.q = h.q; o.error = 0; o.nproj = 0;
    }
  }
  __syncthreads();
  const int n = ngen_s;
  // PoseClusterer: RPY (tf getRPY of Matrix3x3(q)) as float
  for (int i = tid; i < n; i += blockDim.x) {
    double m[9], r, p, y;
    basis_from_quat(G[i].q, m);
    basis_to_rpy(m, &r, &p, &y);
    ax[i] = (float)r; ay[i] = (float)p; az[i] = (float)y;
    cid[i] = -1;
  }
  if (tid == 0) nclus = 0;
  __syncthreads();
  // BFcluster (PoseClusterer.cpp:51-116): seeds in index order; the members
  // within 1.5 r of the seed are found in parallel (ballot words), their
  // float centre is summed by one thread in index order (float adds are
  // order-sensitive) over the set bits only, then the members within r of the
  // centre join the cluster in parallel.
  __shared__ uint64_t hitw[kMaxHyps / 64];
  __shared__ int32_t csz;
  const int lane = tid & 63;
  for (int i = 0; i < n; i++) {
    if (cid[i] >= 0) continue;  // uniform: cid[] is shared and stable here
    for (int j0 = 0; j0 < n; j0 += blockDim.x) {
      const int j = j0 + tid;
      int hit = 0;
      if (j < n && cid[j] < 0) {
        double dx = ax[i] - ax[j], dy = ay[i] - ay[j], dz = az[i] - az[j];
        hit = sqrt(dx * dx + dy * dy + dz * dz) <= max_angle * 1.5;
      }
      const uint64_t m = __ballot(hit);
      if (lane == 0 && j0 + (tid & ~63) < n) hitw[(j0 + (tid & ~63)) >> 6] = m;
    }
    if (tid == 0) csz = 0;
    __syncthreads();
    if (tid == 0) {
      float cx = 0, cy = 0, cz = 0;
      int cntm = 0;
      for (int w = 0; w < (n + 63) / 64; w++) {
        uint64_t m = hitw[w];
        while (m) {
          const int j = 64 * w + __ffsll((unsigned long long)m) - 1;
          m &= m - 1;
          cx += ax[j]; cy += ay[j]; cz += az[j];
          cntm++;
        }
      }
      double sz = (double)cntm;
      cen[0] = (float)(cx / sz); cen[1] = (float)(cy / sz); cen[2] = (float)(cz / sz);
    }
    __syncthreads();
    const int c = nclus;
    for (int j = tid; j < n; j += blockDim.x) {
      int hit = 0;
      if (cid[j] < 0) {
        double dx = cen[0] - ax[j], dy = cen[1] - ay[j], dz = cen[2] - az[j];
        hit = sqrt(dx * dx + dy * dy + dz * dz) <= max_angle;
      }
      flag[j] = hit;
    }
    __syncthreads();
    for (int j = tid; j < n; j += blockDim.x) {
      if (flag[j]) {
        cid[j] = c;
        atomicAdd(&csz, 1);
      }
    }
    __syncthreads();
    if (tid == 0) {
      csize[c] = csz;
      nclus = c + 1;
    }
    __syncthreads();
  }
  __shared__ int32_t best_c, nC;
  if (tid == 0) {
    int b = 0;
    for (int c = 1; c < nclus; c++)
      if (csize[c] > csize[b]) b = c;
    best_c = nclus > 0 ? b : -1;
    // the best cluster's members in index order: positions here (flag[] is
    // free again), the record copies below by the whole block
    int k = 0;
    for (int j = 0; j < n; j++) flag[j] = (best_c >= 0 && cid[j] == best_c) ? k++ : -1;
    nC = k;
    st[f].n_gen = n;
    st[f].n_hyps = k;
    st[f].reaches_pf = (nq > 0 && k > 0) ? 1 : 0;
    dbg[f].n_gen = n;
    dbg[f].n_hyps = k;
  }
  __syncthreads();
  HypRec* Hh = hyps + (size_t)f * kMaxHyps;
  for (int j = tid; j < n; j += blockDim.x)
    if (flag[j] >= 0) Hh[flag[j]] = G[j];
}

// prefix over frames: draws of the shared cv::RNG stream happen only for
// frames that reach the particle filter, in frame order
// (one 1024-thread block: per-thread serial chunk, wave scans, block scan)
// 256 threads (round 6; 1024 before): under the other contexts' load a
// 16-wave block waits for a whole CU to drain (9 ms of stream time per batch in
// the 6-context bench's gauss_h2d span), four waves fit beside them
constexpr int kGaussOffThreads = 256;
__global__ __launch_bounds__(kGaussOffThreads) void k_gauss_offsets(FrameState* st, int nf, int per_frame, int32_t* total) {
  constexpr int NT = kGaussOffThreads;
  __shared__ int wsum[NT / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int chunk = (nf + NT - 1) / NT;
  const int f0 = min(nf, t * chunk), f1 = min(nf, f0 + chunk);
  int mine = 0;
  for (int f = f0; f < f1; f++) mine += st[f].reaches_pf ? per_frame : 0;
  int incl = mine;  // inclusive scan over the wave
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wave; w++) base += wsum[w];
  int acc = base + incl - mine;
  for (int f = f0; f < f1; f++) {
    st[f].gauss_offset = acc;
    if (st[f].reaches_pf) acc += per_frame;
  }
  if (t == NT - 1) *total = base + incl;
}

// Camera-sharded rigs: this rank's (global frame index, reaches-PF flag) pairs,
// padded to `slots` with (-1, 0) so every rank contributes the same count.
__global__ __launch_bounds__(256) void k_shard_pf_pack(const FrameState* __restrict__ st,
                                                       const int32_t* __restrict__ gidx, int n_local, int slots,
                                                       int32_t* __restrict__ pairs) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= slots) return;
  pairs[2 * s] = s < n_local ? gidx[s] : -1;
  pairs[2 * s + 1] = s < n_local ? (st[s].reaches_pf ? 1 : 0) : 0;
}

// The gathered pairs of every rank -> flags[0, ng) in global frame order, the
// exclusive prefix of flags * per_frame in flags[ng, 2 ng), and each local
// frame's gaussian offset at its global index (one block).
__global__ __launch_bounds__(1024) void k_gauss_offsets_global(const int32_t* __restrict__ pairs, int npairs,
                                                               int32_t* flags, int ng, FrameState* st,
                                                               const int32_t* __restrict__ gidx, int n_local,
                                                               int per_frame, int32_t* total) {
  __shared__ int wsum[16];
  __shared__ int bad;  // a pair names a frame >= ng: mk_shard.h offsets_from_pairs rejects the gather (-1)
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0) bad = 0;
  for (int i = t; i < ng; i += 1024) flags[i] = 0;
  __syncthreads();
  for (int i = t; i < npairs; i += 1024) {
    const int g = pairs[2 * i];
    if (g >= ng) bad = 1;
    else if (g >= 0) flags[g] = pairs[2 * i + 1];
  }
  __syncthreads();
  const int chunk = (ng + 1023) / 1024;
  const int f0 = min(ng, t * chunk), f1 = min(ng, f0 + chunk);
  int mine = 0;
  for (int f = f0; f < f1; f++) mine += flags[f] ? per_frame : 0;
  int incl = mine;
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < wave; w++) base += wsum[w];
  int acc = base + incl - mine;
  for (int f = f0; f < f1; f++) {
    flags[ng + f] = acc;
    if (flags[f]) acc += per_frame;
  }
  if (t == 1023) *total = bad ? -1 : base + incl;
  __syncthreads();
  for (int f = t; f < n_local; f += 1024) st[f].gauss_offset = flags[ng + gidx[f]];
}

// ============================================================== scoring
struct Landmarks {
  const double* xyz;  // n x 3 (white, red, green in map order)
  int32_t nw, nr, ng;
  const float4* xyzf;  // the same as the FP32 screen reads them: X, Y, Z, |X|_1 (mk_screen.h screen_landmark)
};
constexpr int kLmfOffset = 3 * 768;  // double index of the FP32 table in the map buffer (mantis_set_map)

// Masks of the cleaned image (HypothesisEvaluation.h:364 img.copyTo(out, mask)):
// none (original image), host bytes (standalone scoring API) or the k_morph
// bit plane (pipeline). Pixels are addressed by linear offset (below).
// Each mask offers a split test for the pipelined fast scorer: word() issues
// the load of the mask word holding pixel (x, y) (x already normalised to
// [0, W)), test() extracts the bit. Out-of-buffer offsets (cvRound(px) == W /
// == H) read as black; the caller never passes them in.
struct MaskNone {
  __device__ uint32_t word(int, int, int) const { return 1u; }
  __device__ bool test(uint32_t, int) const { return true; }
};
struct MaskBytes {
  const uint8_t* m;
  __device__ uint32_t word(int lin, int, int) const { return m[lin]; }
  __device__ bool test(uint32_t w, int) const { return w != 0; }
};
// the frame's tiled mask plane staged in LDS (k_score_pf, when it fits
// beside the kernel's static LDS: a 720p plane is 115 KB): ds_read lookups
// instead of mask-word gathers through the L1
typedef __attribute__((address_space(3))) const uint32_t lds_cu32;
// lookups of word (y, x >> 5) of the tiled plane (bits::tiled_word) in 32-bit
// arithmetic: x, y >= 0 and a plane holds < 2^31 words
struct MaskLds {
  lds_cu32* m;
  int Hp;  // bits::tiled_rows(H)
  // (24-bit multiplies: x >> 5 and Hp are far below 2^24; v_mul_lo_u32 is quarter rate)
  __device__ uint32_t word(int, int x, int y) const { return m[__umul24((uint32_t)(x >> 5), (uint32_t)Hp) + y]; }
  __device__ bool test(uint32_t w, int x) const { return (w >> (x & 31)) & 1u; }
};
struct MaskBits {
  const uint32_t* m;
  int Hp, W;
  __device__ uint32_t word(int, int x, int y) const { return m[__umul24((uint32_t)(x >> 5), (uint32_t)Hp) + y]; }
  __device__ bool test(uint32_t w, int x) const { return (w >> (x & 31)) & 1u; }
};
// B, G, R of pixel lin as the low 24 bits of one (unaligned) dword load; the
// last pixel of the frame reads one byte early so the load stays in the buffer.
__device__ inline uint32_t load_bgr(const uint8_t* bgr, int lin, int npx) {
  const bool last = lin == npx - 1;
  typedef __attribute__((address_space(1), aligned(1))) const uint32_t gu32u;  // unaligned dword
  const uint32_t v = *(gu32u*)(bgr + (3 * lin - (last ? 1 : 0)));
  return last ? (v >> 8) : v;
}

// COLOR (slow) error of one hypothesis (computePointError, HypothesisEvaluation.h:
// 233-266): for each green landmark with z > 0 in frame, the mean over the
// 10 x 10 window cvRound(px + ox, py + oy), o in -5..4 (no bounds check:
// linear offset, out-of-buffer reads 0), of the squared BGR
// distance to GREEN (50, 255, 85); the error is the sum of the means in map
// order / (n * 1.1). One wave per hypothesis: lanes project the landmarks
// once, then take (landmark, window row) items -- ten independent pixel
// gathers each -- and add their integer row sums into the landmark's LDS
// accumulator (the window sum is an exact integer, so its order is free);
// lane 0 sums the means in landmark order.
struct ColorLds {
  double u[64], v[64];
  int32_t acc[64], ok[64];
  int32_t x0[64], run[64];  // cvRound(u - 5); whether the 10 columns are x0 .. x0 + 9
};
// Window-row sum of the COLOR error over the 10 pixels lin0 .. lin0 + 9 (the
// common case: the columns cvRound(u - 5 + k) are x0 + k, and the row lies
// inside the buffer with 36 bytes to spare): two 16-byte loads and one dword
// of the 30 bytes from the dword-aligned start, realigned with v_alignbyte,
// instead of ten unaligned pixel loads. Same pixels, same integer sum.
typedef unsigned int cu32x4 __attribute__((ext_vector_type(4)));
// the row sum from its 36 loaded bytes (dword-aligned start, m = the row's
// byte offset in the first dword)
__device__ inline int color_row_words(cu32x4 q0, cu32x4 q1, uint32_t d8, uint32_t m) {
  const uint32_t d[9] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, d8};
  uint32_t w[8];
#pragma unroll
  for (int j = 0; j < 8; j++) w[j] = __builtin_amdgcn_alignbyte(d[j + 1], d[j], m);
  w[7] &= 0xffffu;  // bytes 28, 29: the stream's 30 bytes end there
  // sum over the 30 bytes c of (c - t)^2, t = GREEN's channel of the byte
  // (50, 255, 85 repeating): sum c^2 - 2 sum c t + 10 |GREEN|^2, both sums as
  // v_dot4_u32_u8 chains over the realigned dwords (dword j starts at byte 4j,
  // channel 4j mod 3 = j mod 3)
  constexpr uint32_t T0 = 50u | 255u << 8 | 85u << 16 | 50u << 24;   // channels 0 1 2 0
  constexpr uint32_t T1 = 255u | 85u << 8 | 50u << 16 | 255u << 24;  // 1 2 0 1
  constexpr uint32_t T2 = 85u | 50u << 8 | 255u << 16 | 85u << 24;   // 2 0 1 2
  uint32_t sq = 0, ct = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    sq = __builtin_amdgcn_udot4(w[j], w[j], sq, false);
    ct = __builtin_amdgcn_udot4(w[j], j % 3 == 0 ? T0 : (j % 3 == 1 ? T1 : T2), ct, false);
  }
  return (int)sq - 2 * (int)ct + 10 * (50 * 50 + 255 * 255 + 85 * 85);
}
__device__ inline int color_row_run(const uint8_t* bgr, long lin0) {
  const long b = 3 * lin0;
  const uint32_t m = (uint32_t)(b & 3);
  typedef __attribute__((address_space(1), aligned(4))) const cu32x4 gu4a;
  const uint8_t* a = bgr + (b - m);
  // the ninth dword only when the row starts at byte 3 of its first dword
  // (bytes m + 28, m + 29 are the last ones used: inside the first eight for m <= 2)
  uint32_t d8 = 0u;
  if (m == 3u) d8 = *(gu32*)(a + 32);
  return color_row_words(*(gu4a*)a, *(gu4a*)(a + 16), d8, m);
}
__device__ inline void wave_score_color(const Xf& c2w, const double* green, int ngr, const Cam& cm,
                                        const uint8_t* bgr, int W, int H, ColorLds* cl, double* err_out,
                                        int* n_out) {
  const int lane = threadIdx.x & 63;
  const long npx = (long)W * H;
  double total = 0;
  int n = 0;
  for (int base = 0; base < ngr; base += 64) {
    const int nb = min(64, ngr - base);
    {
      const int l = base + lane;
      int ok = 0;
      double u = 0, v = 0;
      if (lane < nb) {
        double rp[3];
        xf_apply(c2w, green + 3 * l, rp);
        distort(cm, rp[0], rp[1], rp[2], &u, &v);
        ok = rp[2] > 0 && in_frame(u, v, H, W);
      }
      const int x0 = cv_round(u + (-5.0 + 0.0));
      int run = 1;
#pragma unroll
      for (int ox = 1; ox < 10; ox++) run &= cv_round(u + (-5.0 + (double)ox)) == x0 + ox;
      cl->u[lane] = u;
      cl->v[lane] = v;
      cl->ok[lane] = ok;
      cl->acc[lane] = 0;
      cl->x0[lane] = x0;
      cl->run[lane] = run;
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    for (int k = lane; k < nb * 10; k += 64) {
      const int li = k / 10, r = k - 10 * li;
      if (!cl->ok[li]) continue;
      const double u = cl->u[li];
      const int y = cv_round(cl->v[li] + (-5.0 + (double)r));
      const long lin0 = (long)y * W + cl->x0[li];
      if (cl->run[li] && lin0 >= 0 && lin0 + 12 <= npx) {
        atomicAdd(&cl->acc[li], color_row_run(bgr, lin0));
        continue;
      }
      int rs = 0;
#pragma unroll
      for (int ox = 0; ox < 10; ox++) {
        const int x = cv_round(u + (-5.0 + (double)ox));
        const long lin = (long)y * W + x;
        int b = 0, g = 0, rr = 0;
        if (lin >= 0 && lin < npx) {
          const uint32_t pv = load_bgr(bgr, lin, npx);
          b = (int)(pv & 0xffu);
          g = (int)((pv >> 8) & 0xffu);
          rr = (int)((pv >> 16) & 0xffu);
        }
        const int e0 = b - 50, e1 = g - 255, e2 = rr - 85;
        rs += e0 * e0 + e1 * e1 + e2 * e2;
      }
      atomicAdd(&cl->acc[li], rs);
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
    if (lane == 0) {
      for (int l = 0; l < nb; l++)
        if (cl->ok[l]) {
          total += (double)cl->acc[l] / (double)(10 * 10);
          n++;
        }
    }
    __builtin_amdgcn_wave_barrier();
    __threadfence_block();
  }
  if (lane == 0) {
    *n_out = n;
    *err_out = n <= 0 ? DBL_MAX : total / ((double)n * 1.1);
  }
}

// The same COLOR errors for a block's whole hypothesis set at once
// (k_score_final's 80 yaw-set hypotheses): phase 1 projects every
// (hypothesis, green landmark) pair (exact FP64, one per thread), phase 2 takes
// the window rows -- (pair, row) items spread over every thread of the block,
// several row loads in flight per thread, integer row sums added into the
// pair's LDS slot (exact, order-free) -- and phase 3 sums each hypothesis's
// window means in landmark order. Same pixels, same sums and the same ordered
// double sum as wave_score_color, without its per-hypothesis chain of
// dependent row trips.
constexpr int kColorPairs = 3072;  // (hypothesis, green landmark) pairs the block path holds (80 x 37 = 2960)
struct ColorPairs {
  int32_t x0[kColorPairs];  // cvRound(u - 5)
  int32_t yf[kColorPairs];  // cvRound(v - 5) << 3 | yrun << 2 | xrun << 1 | ok
  int32_t acc[kColorPairs]; // window sum
};
// window row r of pair (T, X) when a column or row of the window does not
// follow from x0 / y0 (a rounding of u - 5 + k or v - 5 + r that moves the
// pixel by other than k / r: only within an ulp of a half-integer)
__device__ __attribute__((noinline)) int color_row_exact(const Xf& T, const double* X, const Cam& cm,
                                                         const uint8_t* bgr, int W, int H, int r) {
  double rp[3], u, v;
  xf_apply(T, X, rp);
  distort(cm, rp[0], rp[1], rp[2], &u, &v);
  const long npx = (long)W * H;
  const int y = cv_round(v + (-5.0 + (double)r));
  int rs = 0;
  for (int ox = 0; ox < 10; ox++) {
    const int x = cv_round(u + (-5.0 + (double)ox));
    const long lin = (long)y * W + x;
    int b = 0, g = 0, rr = 0;
    if (lin >= 0 && lin < npx) {
      const uint32_t pv = load_bgr(bgr, lin, npx);
      b = (int)(pv & 0xffu);
      g = (int)((pv >> 8) & 0xffu);
      rr = (int)((pv >> 16) & 0xffu);
    }
    const int e0 = b - 50, e1 = g - 255, e2 = rr - 85;
    rs += e0 * e0 + e1 * e1 + e2 * e2;
  }
  return rs;
}
// COLOR errors of nh hypotheses (pose_of(h) = FP64 c2w) into err[h]; the whole
// block calls it (nh * ngr <= kColorPairs)
// MK_SCORE_TICKS == 3 (diagnostics): the ends of COLOR's projection and row
// phases into ctk[1], ctk[2] (k_score_final's ticks, 10 ns from ctk0)
#define MK_CTICK(k) \
  if (ctk && threadIdx.x == 0) ctk[1 + (k)] = (int32_t)(wall_clock64() - ctk0);
template <int NT, class PoseOf>
__device__ inline void block_score_color(const PoseOf& pose_of, int nh, const double* green, int ngr, const Cam& cm,
                                         const uint8_t* bgr, int W, int H, ColorPairs* cp, double* err, int32_t* ctk = nullptr, uint64_t ctk0 = 0) {
  const int tid = threadIdx.x;
  const int np = nh * ngr;
  const long npx = (long)W * H;
  for (int i = tid; i < np; i += NT) {
    const int h = i / ngr, l = i - h * ngr;
    double rp[3], u, v;
    xf_apply(pose_of(h), green + 3 * l, rp);
    distort(cm, rp[0], rp[1], rp[2], &u, &v);
    const int ok = rp[2] > 0 && in_frame(u, v, H, W);
    const int x0 = cv_round(u + (-5.0 + 0.0)), y0 = cv_round(v + (-5.0 + 0.0));
    int xrun = 1, yrun = 1;
#pragma unroll
    for (int k = 1; k < 10; k++) {
      xrun &= cv_round(u + (-5.0 + (double)k)) == x0 + k;
      yrun &= cv_round(v + (-5.0 + (double)k)) == y0 + k;
    }
    cp->x0[i] = x0;
    cp->yf[i] = (int32_t)((uint32_t)y0 << 3) | (yrun << 2) | (xrun << 1) | ok;
    cp->acc[i] = 0;
  }
  __syncthreads();
  MK_CTICK(0);
  // (pair, row) items, row-major over the pairs so a wave's lanes add into
  // different pairs; 4 items per thread per trip (their row loads in flight together)
  const int ni = 10 * np;
  constexpr int kU = 4;
  for (int q0 = tid; q0 < ni; q0 += kU * NT) {
    int rsum[kU], slot[kU];
#pragma unroll
    for (int k = 0; k < kU; k++) {
      const int q = q0 + k * NT;
      slot[k] = -1;
      rsum[k] = 0;
      if (q >= ni) continue;
      const int r = q / np, i = q - r * np;
      const int yf = cp->yf[i];
      if (!(yf & 1)) continue;
      slot[k] = i;
      const int x0 = cp->x0[i], y = (yf >> 3) + r;
      const long lin0 = (long)y * W + x0;
      if ((yf & 6) == 6 && lin0 >= 0 && lin0 + 12 <= npx) {
        rsum[k] = color_row_run(bgr, lin0);
      } else if ((yf & 6) == 6) {  // rows reaching past the buffer: pixel by pixel, out-of-buffer reads 0 (Q10)
        int rs = 0;
        for (int ox = 0; ox < 10; ox++) {
          const long lin = lin0 + ox;
          int b = 0, g = 0, rr = 0;
          if (lin >= 0 && lin < npx) {
            const uint32_t pv = load_bgr(bgr, lin, npx);
            b = (int)(pv & 0xffu);
            g = (int)((pv >> 8) & 0xffu);
            rr = (int)((pv >> 16) & 0xffu);
          }
          const int e0 = b - 50, e1 = g - 255, e2 = rr - 85;
          rs += e0 * e0 + e1 * e1 + e2 * e2;
        }
        rsum[k] = rs;
      } else {
        const int h = i / ngr;
        rsum[k] = color_row_exact(pose_of(h), green + 3 * (i - h * ngr), cm, bgr, W, H, r);
      }
    }
#pragma unroll
    for (int k = 0; k < kU; k++)
      if (slot[k] >= 0) atomicAdd(&cp->acc[slot[k]], rsum[k]);
  }
  __syncthreads();
  MK_CTICK(1);
  for (int h = tid; h < nh; h += NT) {
    double total = 0;
    int n = 0;
    for (int l = 0; l < ngr; l++) {
      const int i = h * ngr + l;
      if (cp->yf[i] & 1) {
        total += (double)cp->acc[i] / (double)(10 * 10);
        n++;
      }
    }
    err[h] = n <= 0 ? DBL_MAX : total / ((double)n * 1.1);
  }
  __syncthreads();
}

// ------------------------------------------------------ screened fast scoring
// Every landmark is first projected with the FP32 screen (mk_screen.h), whose
// decision (z > 0, inFrame, cvRound pixel) is taken where it is certain; the
// rare unsure landmarks (about 1 % of the in-frame ones on the bench frames,
// tools/check_screen.hip) are appended to a per-block queue in LDS as
// (tag, landmark) and recomputed with the exact FP64 projection by the whole
// block after the screened pass -- full waves, whichever wave pushed them --
// their integer terms added into the tag's sums with LDS atomics. The sums are
// exact integers, so the order is free and the errors are identical to the
// exact path's (HypothesisEvaluation.h:107-158, 218-227). A wave that finds the
// queue full recomputes its own unsure landmarks in place.
#ifndef MK_SCR_UNROLL
#define MK_SCR_UNROLL 6
#endif
constexpr int kScrUnroll = MK_SCR_UNROLL;  // landmarks per lane in flight (their pixel loads overlap)
struct UQueue {
  uint32_t* e;  // entries: tag << 16 | landmark
  int32_t* n;   // entries pushed (past cap: those were recomputed in place)
  int cap;
};
// exact term of one landmark: the FP64 path the screen stands in for. Not
// inlined: it runs for ~1 % of the landmarks, and inlined its FP64 constants
// (mk_dmath.h atan coefficients in SGPRs) stay live across the screened loop
// and spill it.
template <class MK>
__device__ __attribute__((noinline)) bool exact_term(const Xf& T, const double* X, const Cam& cm, int W, int H, const uint8_t* bgr,
                                  const MK& mask, int& e) {
  double rp[3], u, v;
  xf_apply(T, X, rp);
  distort(cm, rp[0], rp[1], rp[2], &u, &v);
  if (!(rp[2] > 0 && in_frame(u, v, H, W))) return false;
  const int npx = W * H;
  int x = cv_round(u), y = cv_round(v);
  const int li = y * W + x;
  const bool ok = li >= 0 && li < npx;
  if (x >= W) { x -= W; y += 1; }  // cvRound(u) == W: next row (linear offset)
  e = 3 * 255 * 255;
  if (ok && mask.test(mask.word(li, x, y), x)) {
    const uint32_t pv = load_bgr(bgr, li, npx);
    const int b = (int)(pv & 0xffu) - 255, g = (int)((pv >> 8) & 0xffu) - 255, r = (int)((pv >> 16) & 0xffu) - 255;
    e = b * b + g * g + r * r;
  }
  return true;
}
// wave-uniform FP32 pose into SGPRs
__device__ inline float rfl(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}
__device__ inline PoseF rfl(const PoseF& P) {
  PoseF u;
#pragma unroll
  for (int k = 0; k < 9; k++) u.R[k] = rfl(P.R[k]);
#pragma unroll
  for (int k = 0; k < 3; k++) u.t[k] = rfl(P.t[k]);
  u.tn = rfl(P.tn);
  u.pad[0] = u.pad[1] = u.pad[2] = 0.f;
  return u;
}
// One wave, pose P (wave-uniform), landmarks [lb, le): integer error sum and
// count of the screened landmarks (wave-reduced); unsure ones go to q under
// `tag` (Tx, lmd, cmp: the exact pose, the FP64 landmarks and the camera, read
// only when the queue is full). States: 0 out, 1 in frame (pixel in the
// buffer), 2 unsure, 3 in frame past the end of the buffer (cvRound == rows:
// reads as black).
// LM(k, l): landmark l (already clamped to [lb, le)) of slot k of the trip
template <int U, class MK, class LM>
__device__ inline void wave_sums_screen_t(const PoseF& P, const LM& lm_at, int lb, int le, const ScreenCam& sc, int W,
                                          int H, const uint8_t* bgr, const MK& mask, UQueue q, int tag, const Xf* Tx,
                                          const double* lmd, const Cam* cmp, long long& s_out, int& n_out) {
  const int lane = threadIdx.x & 63;
  int s = 0, n = 0;  // per lane: <= 12 landmarks x 3 * 255^2, exact in int32
  for (int b0 = lb; b0 < le; b0 += 64 * U) {  // wave-uniform trips
    int st[U], lin[U], px[U], py[U];
#pragma unroll
    for (int k = 0; k < U; k++) {
      const int l = b0 + lane + 64 * k;
      const float4 L = lm_at(k, l < le ? l : le - 1);
      int x, y;
      const int t = screen_project(P, L.x, L.y, L.z, L.w, sc, W, H, &x, &y);
      st[k] = l < le ? t : SCR_OUT;
      const bool in = st[k] == SCR_IN;  // interior pixel: no wrap, inside the buffer
      px[k] = in ? x : 0;
      py[k] = in ? y : 0;
      lin[k] = in ? (int)__umul24((uint32_t)y, (uint32_t)W) + x : 0;  // y, W < 2^13
    }
    // mask words and pixel loads issued unconditionally (address 0 when not
    // needed), so the U loads of a lane are in flight together
    uint32_t mw[U];
#pragma unroll
    for (int k = 0; k < U; k++) mw[k] = mask.word(lin[k], px[k], py[k]);
    // a hit's pixel is interior (lin >= W + 1), so the dword one byte before
    // it (the previous pixel's R, then B, G, R) is inside the buffer for every
    // pixel, the frame's last included: one load form, the value >> 8
    uint32_t pv[U];
    int hm[U];
#pragma unroll
    for (int k = 0; k < U; k++) {
      const bool hit = st[k] == SCR_IN && mask.test(mw[k], px[k]);
      hm[k] = hit ? -1 : 0;
      // 3 lin - 1 as one v_lshl_add_u32 and a v_add (asm: otherwise it becomes a
      // quarter-rate 64-bit v_mad_u64_u32 and a 64-bit address add per load,
      // instead of the scalar-base + 32-bit-offset form)
      uint32_t l3;
      asm("v_lshl_add_u32 %0, %1, 1, %1" : "=v"(l3) : "v"(lin[k]));
      const uint32_t off = hit ? l3 - 1u : 0u;  // 32-bit offset from the scalar base
      typedef __attribute__((address_space(1), aligned(1))) const uint32_t gu32u;
      pv[k] = *(gu32u*)(gbytes(bgr) + off);
    }
    // every load issued, none sunk into a branch behind its mask test: the U
    // loads of a lane stay in flight together
#pragma unroll
    for (int k = 0; k < U; k++) asm volatile("" : "+v"(pv[k]));
    // the terms as masks, not selects: every loaded value is consumed, so the
    // compiler keeps the U loads unconditional (in flight together) instead
    // of sinking each into a branch with its own wait
    int cu = 0;
#pragma unroll
    for (int k = 0; k < U; k++) {
      cu += st[k] == SCR_UNSURE;
      const uint32_t d = ~(pv[k] >> 8) & 0xffffffu;  // 255 - B, 255 - G, 255 - R as bytes
      const int term = (int)__builtin_amdgcn_udot4(d, d, 0u, false);  // sum of their squares (v_dot4_u32_u8)
      constexpr int kBlack = 3 * 255 * 255;  // masked out
      const int e = kBlack ^ ((term ^ kBlack) & hm[k]);
      const int im = st[k] == SCR_IN ? -1 : 0;
      n -= im;
      s += e & im;
    }
    if (__ballot(cu > 0)) {  // wave-aggregated queue append: one LDS atomic
      const int incl = wave_incl_scan(cu, lane);
      int base = 0;
      if (lane == 63) base = atomicAdd(q.n, incl);
      base = __builtin_amdgcn_readlane(base, 63);
      int idx = base + incl - cu;
#pragma unroll
      for (int k = 0; k < U; k++) {
        if (st[k] != SCR_UNSURE) continue;
        const int l = b0 + lane + 64 * k;
        if (idx < q.cap) {
          q.e[idx] = ((uint32_t)tag << 16) | (uint32_t)l;
        } else {
          int e;
          if (exact_term(*Tx, lmd + 3 * l, *cmp, W, H, bgr, mask, e)) { n++; s += e; }
        }
        idx++;
      }
    }
  }
  // wave totals in int32 (<= 64 lanes x 12 landmarks x 3 * 255^2 < 2^31)
  s_out = wave_sum(s);
  n_out = wave_sum(n);
}
template <int U, class MK>
__device__ inline void wave_sums_screen(const PoseF& P, const float4* lmf, int lb, int le, const ScreenCam& sc, int W,
                                        int H, const uint8_t* bgr, const MK& mask, UQueue q, int tag, const Xf* Tx,
                                        const double* lmd, const Cam* cmp, long long& s_out, int& n_out) {
  wave_sums_screen_t<U>(P, [&](int, int l) { return lmf[l]; }, lb, le, sc, W, H, bgr, mask, q, tag, Tx, lmd, cmp,
                        s_out, n_out);
}
// A wave whose tasks all cover the same landmark slice [lb, le) of at most
// 64 U landmarks (the scorers' (hypothesis, half) tasks when the block's wave
// count is even) keeps that slice in registers for all of them instead of
// reading it from LDS on every trip: WaveLms::load once, then sums().
template <int U>
struct WaveLms {
  float4 L[U];
  int lb, le;
  __device__ void load(const float4* lmf, int lb_, int le_) {
    lb = lb_;
    le = le_;
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < U; k++) {
      const int l = lb + lane + 64 * k;
      L[k] = lmf[l < le ? l : le - 1];
    }
  }
  template <class MK>
  __device__ void sums(const PoseF& P, const ScreenCam& sc, int W, int H, const uint8_t* bgr, const MK& mask, UQueue q,
                       int tag, const Xf* Tx, const double* lmd, const Cam* cmp, long long& s_out, int& n_out) const {
    wave_sums_screen_t<U>(P, [&](int k, int) { return L[k]; }, lb, le, sc, W, H, bgr, mask, q, tag, Tx, lmd, cmp, s_out,
                          n_out);
  }
};
// the block recomputes the queued landmarks exactly: add(tag, term) for those
// in frame (pose_of(tag) = the tag's FP64 c2w)
template <class MK, class PoseOf, class Add>
__device__ inline void block_drain(UQueue q, const double* lmd, const Cam* cmp, int W, int H, const uint8_t* bgr,
                                   const MK& mask, const PoseOf& pose_of, const Add& add) {
  const int n = min(*q.n, q.cap);
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t en = q.e[i];
    const int tag = (int)(en >> 16), l = (int)(en & 0xffffu);
    int e;
    if (exact_term(pose_of(tag), lmd + 3 * l, *cmp, W, H, bgr, mask, e)) add(tag, e);
  }
}

// Scoring is three kernels per frame batch (one block per frame each), so
// the particle filter -- 500 of the ~620 scored hypotheses of a frame -- runs
// in a lean kernel whose register budget is not set by the sorting and
// publishing code (VGPRs bound the waves a CU keeps in flight):
//   k_score_init   evaluateHypotheses(C hyps) + getBestNHypotheses(1)
//   k_score_pf     optimizeHypothesisWithParticleFilter (10 x 50)
//   k_score_final  81 shifts, top-20, determineBestYaw, publish gate
// init / final: 10 waves per frame. Particle filter block: 16 waves, tasks = (particle, 1/kPfSplit of the
// landmarks): 100 tasks over 16 waves at split 2 -- 18.3 ms per 4096 frames
// against 20.5 for 10 waves with one task per particle (50 tasks, 5 rounds)
#ifndef MK_PF_THREADS
#define MK_PF_THREADS 1024
#endif
constexpr int kPfThreads = MK_PF_THREADS;
#ifndef MK_PF_SPLIT
#define MK_PF_SPLIT 2
#endif
constexpr int kPfSplit = MK_PF_SPLIT;
#ifndef MK_SCORE_TAIL_THREADS
#define MK_SCORE_TAIL_THREADS 1024
#endif
// k_score_final block size (>= 128: 81 shift lanes): 16 waves take the 81
// shifted hypotheses in 6 rounds instead of 9 (128 VGPRs with some spills;
// score stage 18.4 -> 17.5 ms per 4096 frames)
constexpr int kScoreTail = MK_SCORE_TAIL_THREADS;
#ifndef MK_SCORE_INIT_THREADS
#define MK_SCORE_INIT_THREADS 1024
#endif
constexpr int kScoreInit = MK_SCORE_INIT_THREADS;  // k_score_init block size
// unsure-landmark queues (entries per block pass): init (C hypotheses), particle filter (one iteration), tail (81 shifts)
constexpr int kInitQueue = 1024, kPfQueue = 1024, kTailQueue = 512;
static_assert(kScoreTail >= 128 && kScoreTail % 64 == 0, "score tail block");

struct PoseLds {
  Xf c2w, w2c;
  Quat q;
  double err;
};
// per-frame state handed from one scoring kernel to the next; psum / pcnt /
// ctr: the split particle filter's per-particle partial results and its
// last-block counter (small batches, k_score_pf_part)
constexpr int kPfMaxParticles = 96;
struct ScoreState {
  PoseLds cur;
  int32_t nsc, ctr;
  long long psum[kPfMaxParticles];
  int32_t pcnt[kPfMaxParticles];
};

// wave-uniform double into SGPRs (pose operands of the projection loop)
__device__ inline double rfl(double v) {
  const unsigned long long b = (unsigned long long)__double_as_longlong(v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
__device__ inline Xf rfl(const Xf& T) {
  Xf u;
#pragma unroll
  for (int k = 0; k < 9; k++) u.R[k] = rfl(T.R[k]);
#pragma unroll
  for (int k = 0; k < 3; k++) u.t[k] = rfl(T.t[k]);
  return u;
}

// A frame that returns before scoring (no quadrilaterals / no hypotheses,
// src/mantis3.cpp:82-97): its result record
__device__ inline void score_early_result(const FrameState& s, mantis_cam_result& R, FrameDebug& D) {
  R.status = 0;
  R.reason = s.n_quads == 0 ? MANTIS_NO_QUADS : MANTIS_NO_HYPS;
  R.publish = 0;
  R.n_quads = s.n_quads;
  R.n_hyps = s.n_hyps;
  R.n_scored = 0;
  D.reason = R.reason;
  D.publish = 0;
}

// evaluateHypotheses(C hyps) + getBestNHypotheses(1) of one frame, by the
// whole block (k_score_init, or k_score_pf taking the init itself): screened
// tasks (hypothesis, landmark half; a wave's half in wl), the unsure
// landmarks exactly, errors and debug records, the best one by a unique-
// minimum reduction or, on ties, the libstdc++-order sort. ei / hs / hn hold
// C entries (LDS, or global scratch for more hypotheses than the LDS takes);
// the first npfi hypotheses' screen poses are staged in pfi. Leaves the best
// in cur (and sst), the scored count in nsc. Ends on a barrier.
template <int NT, class MK>
__device__ inline void block_score_init(const FrameDesc& fd, const Cam* cmp, const MK& mask, const Landmarks& lmk,
                                        const WaveLms<kScrUnroll>& wl, HypRec* Hh, int C, FrameDebug& D, ErrIdx* ei,
                                        unsigned long long* hs, int32_t* hn, PoseF* pfi, int npfi, UQueue q,
                                        int32_t* uqn, PoseLds& cur, int32_t& nsc, int32_t& uniq_bi, ScoreState& S) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int W = fd.w, H = fd.h;
  if (tid == 0) *uqn = 0;
  for (int h = tid; h < C; h += NT) {
    hs[h] = 0;
    hn[h] = 0;
    if (h < npfi) pfi[h] = posef_from(Hh[h].c2w);
  }
  __syncthreads();
  // tasks = (hypothesis, half of the landmarks); the halves' sums add exactly
  for (int t = __builtin_amdgcn_readfirstlane(wave); t < 2 * C; t += (NT / 64)) {
    const int h = t >> 1;
    long long s;
    int n;
    const PoseF P = h < npfi ? pfi[h] : posef_from(Hh[h].c2w);
    wl.sums(P, fd.scam, W, H, fd.bgr, mask, q, h, &Hh[h].c2w, lmk.xyz, cmp, s, n);
    if (lane == 0) {
      atomicAdd(&hs[h], (unsigned long long)s);
      atomicAdd(&hn[h], n);
    }
  }
  __syncthreads();
  block_drain(q, lmk.xyz, cmp, W, H, fd.bgr, mask, [&](int t) -> const Xf& { return Hh[t].c2w; },
              [&](int t, int e) {
                atomicAdd(&hs[t], (unsigned long long)e);
                atomicAdd(&hn[t], 1);
              });
  __syncthreads();
  for (int h = tid; h < C; h += NT) {
    const int n = hn[h];
    const double e = n <= 0 ? DBL_MAX : (double)(long long)hs[h] / ((double)n * 1.1);
    Hh[h].error = e;
    Hh[h].nproj = n;
    ei[h].e = e;
    ei[h].i = h;
    for (int k = 0; k < 9; k++) D.hyp_c2w[h][k] = Hh[h].c2w.R[k];
    for (int k = 0; k < 3; k++) D.hyp_c2w[h][9 + k] = Hh[h].c2w.t[k];
    D.hyp_err[h] = e;
    D.hyp_n[h] = n;
  }
  __syncthreads();
  // getBestNHypotheses(1): std::sort, keep back(). When the minimum error is
  // unique, back() is that element whatever the sort's tie order, so wave 0
  // finds it with a reduction and the serial sort runs only on ties.
  if (wave == 0) {
    double be = DBL_MAX;
    int bj = 0x7fffffff, cnt = 0;
    for (int h = lane; h < C; h += 64) {
      const double e = ei[h].e;
      if (e < be || bj == 0x7fffffff) { be = e; bj = h; cnt = 1; }
      else if (e == be) cnt++;
    }
    for (int o = 32; o > 0; o >>= 1) {
      const double oe = __shfl_xor(be, o);
      const int oj = __shfl_xor(bj, o), oc = __shfl_xor(cnt, o);
      if (oe < be) { be = oe; bj = oj; cnt = oc; }
      else if (oe == be) { cnt += oc; if (oj < bj) bj = oj; }
    }
    if (lane == 0) uniq_bi = cnt == 1 ? bj : -1;
  }
  __syncthreads();
  if (tid == 0) {
    int bi = 0;
    if (C > 1) {
      if (uniq_bi >= 0) {
        bi = uniq_bi;
      } else {
        std_sort_desc(ei, ei + C);
        bi = ei[C - 1].i;
      }
    }
    cur.c2w = Hh[bi].c2w; cur.w2c = Hh[bi].w2c; cur.q = Hh[bi].q; cur.err = Hh[bi].error;
    for (int k = 0; k < 9; k++) D.best1_c2w[k] = cur.c2w.R[k];
    for (int k = 0; k < 3; k++) D.best1_c2w[9 + k] = cur.c2w.t[k];
    D.best1_err = cur.err;
    D.pf_iter_err[0] = cur.err;
    nsc = C + 1;
    S.cur = cur;
    S.nsc = nsc;
    S.ctr = 0;
  }
  __syncthreads();
}

template <int NT>
__global__ __launch_bounds__(NT) void k_score_init(
    const FrameDesc* __restrict__ frames, const uint32_t* __restrict__ mbits, size_t bstride, Landmarks lmk,
    FrameState* st, HypRec* __restrict__ hyps, mantis_cam_result* __restrict__ res, FrameDebug* dbg,
    ScoreState* __restrict__ sst) {
  const int f = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6;
  const FrameDesc fd = frames[f];
  const MaskBits mask{mbits + (size_t)f * bstride, bits::tiled_rows(fd.h), fd.w};
  FrameDebug& D = dbg[f];
  const int nl = lmk.nw + lmk.nr + lmk.ng;
  __shared__ float4 lmf[768];
  __shared__ ErrIdx ei[kMaxHyps];
  __shared__ unsigned long long hs[kMaxHyps];  // per hypothesis: integer error sum, count
  __shared__ int32_t hn[kMaxHyps];
  __shared__ uint32_t uqe[kInitQueue];
  __shared__ int32_t uqn;
  __shared__ PoseLds cur;
  __shared__ int32_t nsc, uniq_bi;
  // the first kInitPoses hypotheses' screen poses staged in LDS once (a task
  // then reads its pose from LDS instead of global memory)
  constexpr int kInitPoses = 128;
  __shared__ PoseF pfi[kInitPoses];
  if (!st[f].reaches_pf) {
    if (tid == 0) score_early_result(st[f], res[f], D);
    return;
  }
  for (int i = tid; i < nl; i += blockDim.x) lmf[i] = lmk.xyzf[i];
  __syncthreads();
  static_assert((NT / 64) % 2 == 0 && 64 * kScrUnroll * 2 >= 768, "one register trip per half");
  WaveLms<kScrUnroll> wl;
  wl.load(lmf, nl * (wave & 1) / 2, nl * ((wave & 1) + 1) / 2);
  block_score_init<NT>(fd, &frames[f].cam, mask, lmk, wl, hyps + (size_t)f * kMaxHyps, st[f].n_hyps, D, ei, hs, hn,
                       pfi, kInitPoses, UQueue{uqe, &uqn, kInitQueue}, &uqn, cur, nsc, uniq_bi, sst[f]);
}

// computeAllShiftedHypothesesFAST (HypothesisEvaluation.h): the 9 x 9 grid of
// translations of the optimum by whole grid cells
__device__ inline void shift_values(int grid_size, double grid_spacing, double* shv) {
  double x = -((double)grid_size / 2.0) * grid_spacing + ((double)grid_spacing / 2.0);
  int k = 0;
  for (; x < ((double)grid_size / 2.0) * grid_spacing && k < 9; x += grid_spacing) shv[k++] = x;
}
__device__ inline void shift_pose(const Xf& w2c, const double* shv, int j, PoseLds& o) {
  Xf nw = w2c;
  nw.t[0] += shv[j / 9];
  nw.t[1] += shv[j % 9];
  nw.t[2] += 0.0;
  Hyp h;
  hyp_set_w2c(h, nw);
  o.c2w = h.c2w; o.w2c = h.w2c; o.q = h.q;
}

// particle pose of the six gaussians g6 around the current pose
__device__ inline void pf_particle(const Xf& cur_w2c, const float* g6, Xf& w2c, Xf& c2w) {
  double yaw = (double)g6[0] * 0.03, pitch = (double)g6[1] * 0.03, roll = (double)g6[2] * 0.03;
  double tz = (double)g6[3] * 0.01, ty = (double)g6[4] * 0.01, tx = (double)g6[5] * 0.01;
  Xf rnd;
  basis_from_rpy_small(roll, pitch, yaw, rnd.R);  // |angle| < 2 rad: float gaussian x 0.03
  rnd.t[0] = tx; rnd.t[1] = ty; rnd.t[2] = tz;
  w2c = xf_mul(cur_w2c, rnd);
  c2w = xf_inverse(w2c);
}

// optimizeHypothesisWithParticleFilter (PoseAdjustment.h:13-60): particles are
// w2c_sample * rand, rand = Transform(setRPY(g,g,g), (g,g,g)) drawn yaw, pitch,
// roll, z, y, x; best = first strict minimum (argmin by (error, index) over
// the 50, taken only when strictly below the current error).
template <int NT, int SPLIT, bool LM>
__global__ __launch_bounds__(NT) void k_score_pf(
    const FrameDesc* __restrict__ frames, const uint32_t* __restrict__ mbits, size_t bstride, Landmarks lmk,
    const FrameState* __restrict__ st, const float* __restrict__ gauss, mantis_cam_result* __restrict__ res,
    FrameDebug* dbg, ScoreState* __restrict__ sst, int particles, int iterations, int shifts, double grid_spacing,
    int grid_size, int init, HypRec* __restrict__ hyps, unsigned char* __restrict__ init_scratch) {
  const int f = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (!st[f].reaches_pf) {
    if (init && tid == 0) score_early_result(st[f], res[f], dbg[f]);
    return;
  }
  const FrameDesc fd = frames[f];
  const int W = fd.w, H = fd.h;
  const uint32_t* fm = mbits + (size_t)f * bstride;
  extern __shared__ __align__(16) uint32_t pf_mask[];
  if (LM) {  // stage the tiled plane (bits::tiled_words: a multiple of 32 words, 16-byte aligned)
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
    const int n4 = (int)(bits::tiled_words(W, H) / 4);
    const u32x4* src = (const u32x4*)fm;
    u32x4* dst = (u32x4*)pf_mask;
    for (int i = tid; i < n4; i += NT) dst[i] = src[i];
  }
  FrameDebug& D = dbg[f];
  const int nl = lmk.nw + lmk.nr + lmk.ng;
  __shared__ float4 lmf[768];
  // the particles' poses and sums (Pc, Pw, Pf, Pe, Ps, Pn) in one buffer, which
  // the init phase (init: k_score_init's work done here, the mask already in
  // LDS) uses first for its per-hypothesis errors, sums and counts
  constexpr int kPfBuf = 96 * (2 * (int)sizeof(Xf) + (int)sizeof(PoseF) + 8 + SPLIT * 12);
  __shared__ __align__(16) unsigned char pbuf[kPfBuf];
  Xf* Pc = (Xf*)pbuf;
  Xf* Pw = Pc + 96;
  PoseF* Pf = (PoseF*)(Pw + 96);
  double* Pe = (double*)(Pf + 96);
  unsigned long long* Ps = (unsigned long long*)(Pe + 96);
  int32_t* Pn = (int32_t*)(Ps + 96 * SPLIT);
  __shared__ uint32_t uqe[kPfQueue];
  __shared__ int32_t uqn;
  constexpr int kW = NT / 64;
  __shared__ Xf cur_c2w, cur_w2c;
  __shared__ double cur_err;
  for (int i = tid; i < nl; i += blockDim.x) lmf[i] = lmk.xyzf[i];
  if (tid == 0 && !init) {
    cur_c2w = sst[f].cur.c2w;
    cur_w2c = sst[f].cur.w2c;
    cur_err = sst[f].cur.err;
  }
  __syncthreads();
#if defined(MK_SCORE_TICKS) && MK_SCORE_TICKS == 2  // diagnostics: this kernel's phases summed over the iterations
  // into st[f].ticks (10 ns): staging, particles, screened tasks, drain, sums, argmin (tools/score_ticks.py pf)
  uint64_t tkp = wall_clock64();
  int32_t tka[6] = {0, 0, 0, 0, 0, 0};
#define MK_PTICK(k)                                \
  if (tid == 0) {                                  \
    const uint64_t nw = wall_clock64();            \
    tka[k] += (int32_t)(nw - tkp);                 \
    tkp = nw;                                      \
  }
#else
#define MK_PTICK(k)
#endif
  MK_PTICK(0);
  const float* gs = gauss + st[f].gauss_offset;
  const UQueue q{uqe, &uqn, kPfQueue};
  const MaskLds mlds{(lds_cu32*)pf_mask, bits::tiled_rows(H)};
  const MaskBits mglb{fm, bits::tiled_rows(H), W};
  // a wave's tasks are (particle, slice wave % SPLIT): its slice of the
  // landmarks stays in registers for every task and iteration
  static_assert(kW % SPLIT == 0 && 64 * kScrUnroll * SPLIT >= 768, "one register trip per slice");
  WaveLms<kScrUnroll> wl;
  {
    const int h = wave % SPLIT;
    wl.load(lmf, nl * h / SPLIT, nl * (h + 1) / SPLIT);
  }
  if (init) {
    // evaluateHypotheses + getBestNHypotheses(1) (k_score_init's block
    // function) with the mask lookups from LDS; the init's landmark halves are
    // the particle tasks' slices (SPLIT == 2)
    static_assert(SPLIT == 2, "the init tasks use landmark halves");
    __shared__ PoseLds icur;
    __shared__ int32_t insc, iuniq;
    const int C = st[f].n_hyps;
    HypRec* Hh = hyps + (size_t)f * kMaxHyps;
    constexpr int kPer = (int)(sizeof(ErrIdx) + sizeof(unsigned long long) + sizeof(int32_t));
    const auto run = [&](unsigned char* buf) {
      ErrIdx* ei = (ErrIdx*)buf;
      unsigned long long* hs = (unsigned long long*)(ei + C);
      int32_t* hn = (int32_t*)(hs + C);
      const UQueue qi{uqe, &uqn, kPfQueue};
      if (LM) block_score_init<NT>(fd, &frames[f].cam, mlds, lmk, wl, Hh, C, D, ei, hs, hn, nullptr, 0, qi, &uqn,
                                   icur, insc, iuniq, sst[f]);
      else block_score_init<NT>(fd, &frames[f].cam, mglb, lmk, wl, Hh, C, D, ei, hs, hn, nullptr, 0, qi, &uqn, icur,
                                insc, iuniq, sst[f]);
    };
    if (C * kPer <= kPfBuf && init != 2) run(pbuf);  // init == 2 (tests): the global-scratch path
    else run(init_scratch + (size_t)f * kMaxHyps * kPer);  // more hypotheses than the LDS buffer takes: global scratch
    if (tid == 0) {
      cur_c2w = icur.c2w;
      cur_w2c = icur.w2c;
      cur_err = icur.err;
    }
    __syncthreads();
  }
  // the frame's gaussians in LDS (round 6): the landmark table's bytes, free
  // once every wave holds its slice (wl) -- the particle phase then reads them
  // by ds_read instead of a global round trip per iteration
  const int ngs = particles * iterations * 6;
  const bool gl = ngs <= (int)(sizeof(lmf) / sizeof(float));
  float* glds = (float*)lmf;
  __syncthreads();
  if (gl)
    for (int i = tid; i < ngs; i += NT) glds[i] = gs[i];
  const float* gsrc = gl ? (const float*)glds : gs;
  const auto particle = [&](int it, int j, const Xf& w2c_cur) {
    Xf w2c, c2w;
    pf_particle(w2c_cur, gsrc + (size_t)(it * particles + j) * 6, w2c, c2w);
    Pw[j] = w2c;
    Pc[j] = c2w;
    Pf[j] = posef_from(c2w);
  };
  __syncthreads();
  if (iterations > 0)
    for (int j = tid; j < particles; j += NT) particle(0, j, cur_w2c);
  if (tid == 0) uqn = 0;
  __syncthreads();
  MK_PTICK(1);
  // each iteration: tasks, the unsure landmarks, then wave 0 alone: the
  // particles' errors, the first strict minimum, the current pose, and the
  // next iteration's particles (three barriers an iteration; round 5 had five)
  for (int it = 0; it < iterations; it++) {
    // SPLIT waves per particle (landmark slices; integer sums, so the
    // partials combine exactly in any order); a wave's tasks pipelined
    for (int task = __builtin_amdgcn_readfirstlane(wave); task < particles * SPLIT; task += kW) {
      const int j = task / SPLIT;
      long long sum;
      int cnt;
      if (LM) wl.sums(Pf[j], fd.scam, W, H, fd.bgr, mlds, q, j, &Pc[j], lmk.xyz, &frames[f].cam, sum, cnt);
      else wl.sums(Pf[j], fd.scam, W, H, fd.bgr, mglb, q, j, &Pc[j], lmk.xyz, &frames[f].cam, sum, cnt);
      if (lane == 0) {
        Ps[task] = (unsigned long long)sum;
        Pn[task] = cnt;
      }
    }
    __syncthreads();
    MK_PTICK(2);
    const auto pose_of = [&](int t) -> const Xf& { return Pc[t]; };
    const auto add = [&](int t, int e) {
      atomicAdd(&Ps[t * SPLIT], (unsigned long long)e);
      atomicAdd(&Pn[t * SPLIT], 1);
    };
    if (LM) block_drain(q, lmk.xyz, &frames[f].cam, W, H, fd.bgr, mlds, pose_of, add);
    else block_drain(q, lmk.xyz, &frames[f].cam, W, H, fd.bgr, mglb, pose_of, add);
    __syncthreads();
    MK_PTICK(3);
    if (wave == 0) {
      double be = DBL_MAX;
      int bj = 0x7fffffff;
      for (int j = lane; j < particles; j += 64) {
        long long sum = 0;
        int cnt = 0;
        for (int h = 0; h < SPLIT; h++) {
          sum += (long long)Ps[j * SPLIT + h];
          cnt += Pn[j * SPLIT + h];
        }
        const double e = cnt <= 0 ? DBL_MAX : (double)sum / ((double)cnt * 1.1);
        if (e < be || bj == 0x7fffffff) { be = e; bj = j; }
      }
      for (int o = 32; o > 0; o >>= 1) {
        const double oe = __shfl_xor(be, o);
        const int oj = __shfl_xor(bj, o);
        if (oe < be || (oe == be && oj < bj)) { be = oe; bj = oj; }
      }
      MK_PTICK(4);
      // the winner (wave-uniform) read by every lane before any lane
      // overwrites the particle arrays with the next iteration's
      const bool upd = bj < particles && be < cur_err;
      const Xf nw = upd ? Pw[bj] : cur_w2c;
      if (lane == 0) {
        if (upd) {
          cur_err = be;
          cur_c2w = Pc[bj];
          cur_w2c = nw;
        }
        if (it + 1 < (int)(sizeof(D.pf_iter_err) / sizeof(double))) D.pf_iter_err[it + 1] = upd ? be : cur_err;  // the record holds 10 iterations
        uqn = 0;
      }
      if (it + 1 < iterations)
        for (int j = lane; j < particles; j += 64) particle(it + 1, j, nw);
    }
    __syncthreads();
    MK_PTICK(5);
  }
#if defined(MK_SCORE_TICKS) && MK_SCORE_TICKS == 2
  if (tid == 0)
    for (int k = 0; k < 6; k++) const_cast<FrameState*>(st)[f].ticks[k] = tka[k];
#endif
#undef MK_PTICK
  if (tid == 0) {
    ScoreState& S = sst[f];
    S.cur.c2w = cur_c2w;
    S.cur.w2c = cur_w2c;
    S.cur.q = basis_to_quat(cur_w2c.R);
    S.cur.err = cur_err;
    S.nsc += iterations * particles;
    for (int k = 0; k < 9; k++) D.pf_c2w[k] = cur_c2w.R[k];
    for (int k = 0; k < 3; k++) D.pf_c2w[9 + k] = cur_c2w.t[k];
    D.pf_err = cur_err;
    res[f].pf_error = cur_err;
  }
  if (!shifts) return;
  // shifts (round 6): the 81 shifted hypotheses of k_score_final scored here,
  // while the frame's mask is still in LDS (lookups by ds_read instead of L2
  // gathers); their integer sums and counts go to ScoreState, where
  // k_score_final (pre) takes them, as after k_score_shift_part. Same poses
  // (shift_pose of the same optimum), same sums.
  constexpr int NS = 81;
  static_assert(NS <= 96, "shift poses in the particle arrays");
  __shared__ double shv[9];
  if (tid == 0) {
    uqn = 0;
    shift_values(grid_size, grid_spacing, shv);
  }
  __syncthreads();
  if (tid < NS) {
    PoseLds o;
    shift_pose(cur_w2c, shv, tid, o);
    Pc[tid] = o.c2w;
    Pf[tid] = posef_from(o.c2w);
  }
  for (int i = tid; i < NS * SPLIT; i += NT) {
    Ps[i] = 0;
    Pn[i] = 0;
  }
  __syncthreads();
  for (int task = __builtin_amdgcn_readfirstlane(wave); task < NS * SPLIT; task += kW) {
    const int j = task / SPLIT;
    long long sum;
    int cnt;
    if (LM) wl.sums(Pf[j], fd.scam, W, H, fd.bgr, mlds, q, j, &Pc[j], lmk.xyz, &frames[f].cam, sum, cnt);
    else wl.sums(Pf[j], fd.scam, W, H, fd.bgr, mglb, q, j, &Pc[j], lmk.xyz, &frames[f].cam, sum, cnt);
    if (lane == 0) {
      Ps[task] = (unsigned long long)sum;
      Pn[task] = cnt;
    }
  }
  __syncthreads();
  {
    const auto pose_of = [&](int t) -> const Xf& { return Pc[t]; };
    const auto add = [&](int t, int e) {
      atomicAdd(&Ps[t * SPLIT], (unsigned long long)e);
      atomicAdd(&Pn[t * SPLIT], 1);
    };
    if (LM) block_drain(q, lmk.xyz, &frames[f].cam, W, H, fd.bgr, mlds, pose_of, add);
    else block_drain(q, lmk.xyz, &frames[f].cam, W, H, fd.bgr, mglb, pose_of, add);
  }
  __syncthreads();
  if (tid < NS) {
    long long sum = 0;
    int cnt = 0;
    for (int h = 0; h < SPLIT; h++) {
      sum += (long long)Ps[tid * SPLIT + h];
      cnt += Pn[tid * SPLIT + h];
    }
    sst[f].psum[tid] = sum;
    sst[f].pcnt[tid] = cnt;
  }
}

// One iteration of the particle filter spread over `nblk` blocks per frame
// (small batches, where one block per frame leaves the chip idle and the
// iterations' chain is the latency): block b takes particles [b * ppb, (b+1)
// * ppb), each a task per landmark slice (one per wave), over the global
// mask plane; it writes its particles' integer sums and counts, and the
// frame's last block to finish (counter in ScoreState) takes the argmin and
// moves the current pose, as k_score_pf does at the end of an iteration.
// Same sums, same first strict minimum, same poses (pf_particle recomputes
// the winner's), so the results are identical to k_score_pf's.
template <int NT, int SPLIT>
__global__ __launch_bounds__(NT) void k_score_pf_part(
    const FrameDesc* __restrict__ frames, const uint32_t* __restrict__ mbits, size_t bstride, Landmarks lmk,
    const FrameState* __restrict__ st, const float* __restrict__ gauss, mantis_cam_result* __restrict__ res,
    FrameDebug* dbg, ScoreState* __restrict__ sst, int particles, int iterations, int it, int ppb, int nblk) {
  const int f = blockIdx.y, b = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (!st[f].reaches_pf) return;
  const FrameDesc fd = frames[f];
  const int W = fd.w, H = fd.h;
  const int nl = lmk.nw + lmk.nr + lmk.ng;
  constexpr int kW = NT / 64, kPP = kW / SPLIT > 0 ? kW / SPLIT : 1;  // particles per block (one task per wave)
  __shared__ float4 lmf[768];
  __shared__ Xf Pc[kPP];
  __shared__ PoseF Pf[kPP];
  __shared__ unsigned long long Ps[kPP];
  __shared__ int32_t Pn[kPP];
  __shared__ uint32_t uqe[kPfQueue];
  __shared__ int32_t uqn, last;
  ScoreState& S = sst[f];
  const int p0 = b * ppb, np = max(0, min(ppb, particles - p0));
  const float* gs = gauss + st[f].gauss_offset + (size_t)it * particles * 6;
  for (int i = tid; i < nl; i += NT) lmf[i] = lmk.xyzf[i];
  if (tid < np) {
    Xf w2c, c2w;
    pf_particle(S.cur.w2c, gs + (size_t)(p0 + tid) * 6, w2c, c2w);
    Pc[tid] = c2w;
    Pf[tid] = posef_from(c2w);
    Ps[tid] = 0;
    Pn[tid] = 0;
  }
  if (tid == 0) uqn = 0;
  __syncthreads();
  const UQueue q{uqe, &uqn, kPfQueue};
  const MaskBits mglb{mbits + (size_t)f * bstride, bits::tiled_rows(H), W};
  static_assert(kW % SPLIT == 0 && 64 * kScrUnroll * SPLIT >= 768, "one register trip per slice");
  WaveLms<kScrUnroll> wl;
  {
    const int h = wave % SPLIT;
    wl.load(lmf, nl * h / SPLIT, nl * (h + 1) / SPLIT);
  }
  for (int task = __builtin_amdgcn_readfirstlane(wave); task < np * SPLIT; task += kW) {
    const int j = task / SPLIT;
    long long sum;
    int cnt;
    wl.sums(Pf[j], fd.scam, W, H, fd.bgr, mglb, q, j, &Pc[j], lmk.xyz, &frames[f].cam, sum, cnt);
    if (lane == 0) {
      atomicAdd(&Ps[j], (unsigned long long)sum);
      atomicAdd(&Pn[j], cnt);
    }
  }
  __syncthreads();
  block_drain(q, lmk.xyz, &frames[f].cam, W, H, fd.bgr, mglb, [&](int t) -> const Xf& { return Pc[t]; },
              [&](int t, int e) {
                atomicAdd(&Ps[t], (unsigned long long)e);
                atomicAdd(&Pn[t], 1);
              });
  __syncthreads();
  if (tid < np) {
    S.psum[p0 + tid] = (long long)Ps[tid];
    S.pcnt[p0 + tid] = Pn[tid];
  }
  __threadfence();
  __syncthreads();
  if (tid == 0) last = atomicAdd(&S.ctr, 1) == nblk - 1;
  __syncthreads();
  if (!last || wave != 0) return;
  // the frame's last block: argmin by (error, index), taken only when strictly
  // below the current error
  __threadfence();
  const volatile long long* vs = S.psum;
  const volatile int32_t* vc = S.pcnt;
  double be = DBL_MAX;
  int bj = 0x7fffffff;
  for (int j = lane; j < particles; j += 64) {
    const int cnt = vc[j];
    const double e = cnt <= 0 ? DBL_MAX : (double)vs[j] / ((double)cnt * 1.1);
    if (e < be || bj == 0x7fffffff) { be = e; bj = j; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const double oe = __shfl_xor(be, o);
    const int oj = __shfl_xor(bj, o);
    if (oe < be || (oe == be && oj < bj)) { be = oe; bj = oj; }
  }
  if (lane == 0) {
    FrameDebug& D = dbg[f];
    if (bj < particles && be < S.cur.err) {
      Xf w2c, c2w;
      pf_particle(S.cur.w2c, gs + (size_t)bj * 6, w2c, c2w);
      S.cur.c2w = c2w;
      S.cur.w2c = w2c;
      S.cur.err = be;
    }
    if (it + 1 < (int)(sizeof(D.pf_iter_err) / sizeof(double))) D.pf_iter_err[it + 1] = S.cur.err;
    S.ctr = 0;
    if (it == iterations - 1) {
      S.cur.q = basis_to_quat(S.cur.w2c.R);
      S.nsc += iterations * particles;
      for (int k = 0; k < 9; k++) D.pf_c2w[k] = S.cur.c2w.R[k];
      for (int k = 0; k < 3; k++) D.pf_c2w[9 + k] = S.cur.c2w.t[k];
      D.pf_err = S.cur.err;
      res[f].pf_error = S.cur.err;
    }
  }
}

// computeAllShiftedHypothesesFAST's shift values (accumulated in double as the
// reference loop does) and shifted pose j = (j / 9, j % 9) of the optimum
// The 81 shifted hypotheses' screened sums spread over `nblk` blocks per frame
// (small batches): block b takes shifts [b * spb, (b+1) * spb), one task per
// (shift, landmark half), drains its own unsure landmarks, and writes each
// shift's integer sum and count to ScoreState; k_score_final (pre = true)
// takes them from there instead of scoring the shifts itself. Same sums.
template <int NT>
__global__ __launch_bounds__(NT) void k_score_shift_part(
    const FrameDesc* __restrict__ frames, const uint32_t* __restrict__ mbits, size_t bstride, Landmarks lmk,
    const FrameState* __restrict__ st, ScoreState* __restrict__ sst, double grid_spacing, int grid_size, int spb) {
  const int f = blockIdx.y, b = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (!st[f].reaches_pf) return;
  const FrameDesc fd = frames[f];
  const int W = fd.w, H = fd.h;
  const MaskBits mask{mbits + (size_t)f * bstride, bits::tiled_rows(H), W};
  const int nl = lmk.nw + lmk.nr + lmk.ng;
  constexpr int NS = 81, kMaxSpb = NT / 128 > 0 ? NT / 128 : 1;  // shifts per block: two tasks each, one per wave
  __shared__ float4 lmf[768];
  __shared__ PoseLds P[kMaxSpb];
  __shared__ double shv[9];
  __shared__ unsigned long long hs[kMaxSpb];
  __shared__ int32_t hn[kMaxSpb];
  __shared__ uint32_t uqe[kTailQueue];
  __shared__ int32_t uqn;
  const int j0 = b * spb, ns = max(0, min(min(spb, kMaxSpb), NS - j0));
  for (int i = tid; i < nl; i += NT) lmf[i] = lmk.xyzf[i];
  if (tid == 0) {
    uqn = 0;
    shift_values(grid_size, grid_spacing, shv);
  }
  __syncthreads();
  if (tid < ns) {
    shift_pose(sst[f].cur.w2c, shv, j0 + tid, P[tid]);
    hs[tid] = 0;
    hn[tid] = 0;
  }
  __syncthreads();
  const UQueue q{uqe, &uqn, kTailQueue};
  static_assert((NT / 64) % 2 == 0 && 64 * kScrUnroll * 2 >= 768, "one register trip per half");
  WaveLms<kScrUnroll> wl;
  wl.load(lmf, nl * (wave & 1) / 2, nl * ((wave & 1) + 1) / 2);
  for (int t = __builtin_amdgcn_readfirstlane(wave); t < 2 * ns; t += NT / 64) {
    const int j = t >> 1;
    long long sum;
    int n;
    wl.sums(posef_from(P[j].c2w), fd.scam, W, H, fd.bgr, mask, q, j, &P[j].c2w, lmk.xyz, &frames[f].cam, sum, n);
    if (lane == 0) {
      atomicAdd(&hs[j], (unsigned long long)sum);
      atomicAdd(&hn[j], n);
    }
  }
  __syncthreads();
  block_drain(q, lmk.xyz, &frames[f].cam, W, H, fd.bgr, mask, [&](int t) -> const Xf& { return P[t].c2w; },
              [&](int t, int e) {
                atomicAdd(&hs[t], (unsigned long long)e);
                atomicAdd(&hn[t], 1);
              });
  __syncthreads();
  if (tid < ns) {
    sst[f].psum[j0 + tid] = (long long)hs[tid];
    sst[f].pcnt[j0 + tid] = hn[tid];
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void k_score_final(
    const FrameDesc* __restrict__ frames, const uint32_t* __restrict__ mbits, size_t bstride, Landmarks lmk,
    const FrameState* __restrict__ st, mantis_cam_result* __restrict__ res, FrameDebug* dbg,
    const ScoreState* __restrict__ sst, double grid_spacing, int grid_size, bool pre) {
  const int f = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  if (!st[f].reaches_pf) return;
  const FrameDesc fd = frames[f];
  const int W = fd.w, H = fd.h;
  const MaskBits mask{mbits + (size_t)f * bstride, bits::tiled_rows(H), W};
  mantis_cam_result& R = res[f];
  FrameDebug& D = dbg[f];
  const int nl = lmk.nw + lmk.nr + lmk.ng;
  __shared__ float4 lmf[768];
  __shared__ PoseLds P[96];
  __shared__ ErrIdx ei[96];
  // COLOR phase: the block path's pair table, or (maps with more than
  // kColorPairs / 80 green landmarks) the per-wave path's scratch in the same bytes
  static_assert(sizeof(ColorPairs) >= sizeof(ColorLds) * (NT / 64), "color scratch");
  __shared__ ColorPairs cpairs;
  __shared__ PoseLds cur;
  __shared__ double shv[9];
  __shared__ double yerr[4];
  __shared__ int32_t nsc;
  __shared__ unsigned long long hs[96];
  __shared__ int32_t hn[96];
  __shared__ uint32_t uqe[kTailQueue];
  __shared__ int32_t uqn;
#if defined(MK_SCORE_TICKS) && MK_SCORE_TICKS != 2  // diagnostics: phase ends of this kernel into st[f].ticks (10 ns), tools/score_ticks.py
  const uint64_t tk0 = wall_clock64();
  int32_t* tk = const_cast<FrameState*>(st)[f].ticks;
#define MK_STICK(k) \
  if (tid == 0 && (MK_SCORE_TICKS != 3 || ((k) != 1 && (k) != 2))) tk[k] = (int32_t)(wall_clock64() - tk0);
#else
#define MK_STICK(k)
#endif
  for (int i = tid; i < nl; i += blockDim.x) lmf[i] = lmk.xyzf[i];
  if (tid == 0) {
    uqn = 0;
    cur = sst[f].cur;
    nsc = sst[f].nsc;
    shift_values(grid_size, grid_spacing, shv);
  }
  __syncthreads();
  // computeAllShiftedHypothesesFAST: 81 shifted copies of the optimum
  const int NS = 81;
  if (tid < NS) shift_pose(cur.w2c, shv, tid, P[tid]);
  __syncthreads();
  const UQueue q{uqe, &uqn, kTailQueue};
  if (tid < NS) {
    hs[tid] = pre ? (unsigned long long)sst[f].psum[tid] : 0ull;  // pre: k_score_shift_part's sums
    hn[tid] = pre ? sst[f].pcnt[tid] : 0;
  }
  __syncthreads();
  if (!pre) {
  // tasks = (shift, half of the landmarks): 162 one-trip tasks over the waves
  // instead of 81 two-trip ones (the last round of whole hypotheses kept one
  // wave busy); the halves' integer sums combine exactly
  static_assert((NT / 64) % 2 == 0 && 64 * kScrUnroll * 2 >= 768, "one register trip per half");
  WaveLms<kScrUnroll> wl;
  wl.load(lmf, nl * (wave & 1) / 2, nl * ((wave & 1) + 1) / 2);
  for (int t = __builtin_amdgcn_readfirstlane(wave); t < 2 * NS; t += (NT / 64)) {
    const int j = t >> 1;
    long long sum;
    int n;
    wl.sums(posef_from(P[j].c2w), fd.scam, W, H, fd.bgr, mask, q, j, &P[j].c2w, lmk.xyz, &frames[f].cam, sum, n);
    if (lane == 0) {
      atomicAdd(&hs[j], (unsigned long long)sum);
      atomicAdd(&hn[j], n);
    }
  }
  __syncthreads();
  MK_STICK(0);
  block_drain(q, lmk.xyz, &frames[f].cam, W, H, fd.bgr, mask, [&](int t) -> const Xf& { return P[t].c2w; },
              [&](int t, int e) {
                atomicAdd(&hs[t], (unsigned long long)e);
                atomicAdd(&hn[t], 1);
              });
  __syncthreads();
  }
  if (tid < NS) {
    const int n = hn[tid];
    const double e = n <= 0 ? DBL_MAX : (double)(long long)hs[tid] / ((double)n * 1.1);
    P[tid].err = e;
    ei[tid].e = e;
    ei[tid].i = tid;
    D.shift_err[tid] = e;
  }
  __syncthreads();
  MK_STICK(1);
  // getBestNHypotheses(20) (HypothesisEvaluation.h:484-518): std::sort by
  // descending error, keep the last 20. When the 20 smallest errors are all
  // distinct from every other error, their sorted positions follow from
  // their ranks (no tie order involved); otherwise tid 0 runs the
  // libstdc++-order sort.
  __shared__ int32_t top[20];
  __shared__ int32_t tie20;
  if (tid == 0) tie20 = 0;
  __syncthreads();
  if (tid < NS) {
    const double e = ei[tid].e;
    int lt = 0, eq = 0;
    for (int j = 0; j < NS; j++) {
      const double o = ei[j].e;
      lt += o < e;
      eq += o == e;
    }
    if (lt < 20) {
      if (eq != 1) tie20 = 1;
      else top[19 - lt] = tid;
    }
  }
  __syncthreads();
  if (tid == 0) {
    if (tie20) {
      std_sort_desc(ei, ei + NS);
      for (int k = 0; k < 20; k++) top[k] = ei[NS - 20 + k].i;
    }
    for (int k = 0; k < 20; k++) D.top20_err[k] = P[top[k]].err;
    nsc += NS;
  }
  __syncthreads();
  MK_STICK(2);
  // determineBestYaw: 4 yaw sets (rotZ^k * w2c, left-multiplied), COLOR errors
  // on the original image. Set k derives from set k-1; all four are built
  // first (P[20k + i], the shifts are no longer needed) so their 80 scorings
  // share one pass over the waves (5 rounds at 16 waves instead of 4 x 2).
  // the top 20 staged in the COLOR scratch (not in use yet): LDS per block
  // 83.2 -> 78.5 KB, under half a CU's 160 KB
  static_assert(sizeof(ColorPairs) >= 20 * sizeof(PoseLds), "top-20 staging");
  PoseLds* Y = (PoseLds*)&cpairs;
  if (tid < 20) {
    const PoseLds& s = P[top[tid]];
    Y[tid] = s;
  }
  __syncthreads();
  const Xf rz = make_rot_z90();
  if (tid < 20) {
    P[tid] = Y[tid];
    for (int k = 1; k < 4; k++) {
      Hyp h;
      hyp_set_w2c(h, xf_mul(rz, P[20 * (k - 1) + tid].w2c));
      PoseLds& d = P[20 * k + tid];
      d.c2w = h.c2w; d.w2c = h.w2c; d.q = h.q;
    }
  }
  __syncthreads();
  MK_STICK(3);
  const double* green = lmk.xyz + 3 * (lmk.nw + lmk.nr);
  __shared__ double yset_err[80];
  if (80 * lmk.ng <= kColorPairs) {
    block_score_color<NT>([&](int h) -> const Xf& { return P[h].c2w; }, 80, green, lmk.ng, fd.cam, fd.bgr, W, H,
                          &cpairs, yset_err
#if defined(MK_SCORE_TICKS) && MK_SCORE_TICKS == 3
                          , tk, tk0
#endif
                          );
  } else {
    ColorLds* cls = (ColorLds*)&cpairs;
    for (int j = wave; j < 80; j += (NT / 64)) {
      double e;
      int n;
      wave_score_color(P[j].c2w, green, lmk.ng, fd.cam, fd.bgr, W, H, &cls[wave], &e, &n);
      if (lane == 0) yset_err[j] = e;
    }
    __syncthreads();
  }
  MK_STICK(4);
  if (tid == 0) {
    double best_error = DBL_MAX;
    int best_k = -1;
    for (int k = 0; k < 4; k++) {
      double tot = 0;
      int succ = 0;
      for (int j = 0; j < 20; j++)
        if (fabs(yset_err[20 * k + j] - DBL_MAX) > 0.001) { succ++; tot += yset_err[20 * k + j]; }
      double te = succ == 0 ? DBL_MAX : tot / (double)succ;
      yerr[k] = te;
      D.yaw_err[k] = te;
      if (te < best_error) {
        best_error = te;
        best_k = k;
      }
    }
    // the published pose is the last of the best set (its last assignment)
    PoseLds& pb = P[20 * (best_k < 0 ? 0 : best_k) + 19];
    if (best_k >= 0) pb.err = yset_err[20 * best_k + 19];
    nsc += 80;
    double min1 = DBL_MAX, min2 = DBL_MAX;
    for (int k = 0; k < 4; k++) {
      double diff = yerr[k] - best_error;
      if (diff < min1) { min2 = min1; min1 = diff; }
      else if (diff < min2) { min2 = diff; }
    }
    R.status = 0;
    R.n_quads = st[f].n_quads;
    R.n_hyps = st[f].n_hyps;
    R.n_scored = nsc;
    R.min_yaw_diff = min2;
    D.min_yaw_diff = min2;
    D.yaw_best = best_k;
    D.n_scored = nsc;
    for (int i = 0; i < 36; i++) R.covariance[i] = 0;
    if (best_k < 0) {
      R.reason = MANTIS_NO_YAW;
      R.publish = 0;
      D.reason = R.reason;
      D.publish = 0;
    } else {
      for (int k = 0; k < 3; k++) { R.position[k] = pb.w2c.t[k]; D.position[k] = pb.w2c.t[k]; }
      R.orientation_xyzw[0] = pb.q.x; R.orientation_xyzw[1] = pb.q.y;
      R.orientation_xyzw[2] = pb.q.z; R.orientation_xyzw[3] = pb.q.w;
      for (int k = 0; k < 4; k++) D.orientation_xyzw[k] = R.orientation_xyzw[k];
      for (int k = 0; k < 9; k++) { R.c2w[k] = pb.c2w.R[k]; D.pub_c2w[k] = pb.c2w.R[k]; }
      for (int k = 0; k < 3; k++) { R.c2w[9 + k] = pb.c2w.t[k]; D.pub_c2w[9 + k] = pb.c2w.t[k]; }
      R.error = pb.err;
      D.pub_error = pb.err;
      if (min2 > 4000) {
        double var = pb.err * (1.0 / 600.0);
        for (int i = 0; i < 6; i++) R.covariance[i * 6 + i] = var;
        R.publish = 1;
        R.reason = MANTIS_PUBLISHED;
      } else {
        R.publish = 0;
        R.reason = MANTIS_YAW_AMBIGUOUS;
      }
      for (int i = 0; i < 36; i++) D.covariance[i] = R.covariance[i];
      D.reason = R.reason;
      D.publish = R.publish;
    }
  }
  MK_STICK(5);
#undef MK_STICK
}

// ============================================ legacy rig weighting (f-4)
// MonteCarlo::computeCameraError (include/legacy/mantis/MonteCarlo.cpp:183-226)
// for one (candidate, camera) job per wave: every landmark projected (no z
// test, as project2d :169-181), the pixel as a float strictly inside the
// frame, cvRound, colorError (:283-286) to the landmark set's colour; integer
// sum and count (exact, so the lane order does not matter). Pixels past the
// end of the buffer (cvRound == cols / rows) read black, as the oracle's View.
struct RigWJob {
  double c2w[12];
  int32_t frame, pad;
};
struct RigWColors {
  int32_t c[9];  // B, G, R of white, red, green
};
__global__ __launch_bounds__(256) void k_rig_weight(const FrameDesc* __restrict__ frames, Landmarks lmk,
                                                    const RigWJob* __restrict__ jobs, int n, RigWColors col,
                                                    double* __restrict__ out2) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= n) return;
  const RigWJob& J = jobs[j];
  const FrameDesc fd = frames[J.frame];
  Xf T;
  for (int k = 0; k < 9; k++) T.R[k] = J.c2w[k];
  for (int k = 0; k < 3; k++) T.t[k] = J.c2w[9 + k];
  const int nl = lmk.nw + lmk.nr + lmk.ng;
  const long npx = (long)fd.w * fd.h;
  long long s = 0;
  int cnt = 0;
  for (int l = lane; l < nl; l += 64) {
    double rp[3], u, v;
    xf_apply(T, lmk.xyz + 3 * l, rp);
    distort(fd.cam, rp[0], rp[1], rp[2], &u, &v);
    const float fu = (float)u, fv = (float)v;  // cv::Point2f out (:175-177)
    if (!(fu > 0 && fu < (float)fd.w && fv > 0 && fv < (float)fd.h)) continue;
    cnt++;
    const int x = (int)rintf(fu), y = (int)rintf(fv);
    const long lin = (long)y * fd.w + x;
    const int set = l < lmk.nw ? 0 : (l < lmk.nw + lmk.nr ? 1 : 2);
    int b = 0, g = 0, r = 0;
    if (lin >= 0 && lin < npx) {
      const uint32_t pv = load_bgr(fd.bgr, lin, npx);
      b = (int)(pv & 0xffu);
      g = (int)((pv >> 8) & 0xffu);
      r = (int)((pv >> 16) & 0xffu);
    }
    const int e0 = b - col.c[3 * set], e1 = g - col.c[3 * set + 1], e2 = r - col.c[3 * set + 2];
    s += e0 * e0 + e1 * e1 + e2 * e2;
  }
  for (int o = 32; o > 0; o >>= 1) {
    s += __shfl_xor(s, o);
    cnt += __shfl_xor(cnt, o);
  }
  if (lane == 0) {
    out2[2 * j] = (double)s;
    out2[2 * j + 1] = (double)cnt;
  }
}

// ================================================ standalone scoring API
// Fast errors: HPB hypotheses per block of kApiHyps waves, tasks =
// (hypothesis, half of the landmarks) with a wave's half in registers
// (WaveLms), one drain per block: k_score_api (a call's few hundred
// hypotheses, HPB = 16: many blocks) and the dense batch (thousands per
// frame, HPB = 64: the landmark staging, barriers and drain shared by four
// times as many). COLOR errors: one wave per hypothesis, exact FP64.
#ifndef MK_DENSE_HYPS
#define MK_DENSE_HYPS 64
#endif
constexpr int kApiHyps = 16, kApiQueue = 1024, kDenseHyps = MK_DENSE_HYPS;
template <int HPB, class MK>
__device__ inline void score_api_fast(const FrameDesc& fd, const Cam* cmp, const MK& mask, Landmarks lmk,
                                      const double* c2w, int n, double* err, int32_t* nproj) {
  constexpr int NW = kApiHyps;  // waves per block
  static_assert(NW % 2 == 0 && 64 * kScrUnroll * 2 >= 768, "one register trip per half");
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int h0 = blockIdx.x * HPB, nh = min(HPB, n - h0);
  const int nl = lmk.nw + lmk.nr + lmk.ng;
  __shared__ float4 lmf[768];
  __shared__ unsigned long long hs[HPB];
  __shared__ int32_t hn[HPB];
  __shared__ uint32_t uqe[kApiQueue];
  __shared__ int32_t uqn;
  __shared__ PoseF pf[HPB];  // the block's poses as the screen reads them, staged once
  for (int i = tid; i < nl; i += blockDim.x) lmf[i] = lmk.xyzf[i];
  for (int i = tid; i < HPB; i += blockDim.x) {
    hs[i] = 0;
    hn[i] = 0;
    if (i < nh) pf[i] = posef_from(*(const Xf*)(c2w + 12 * (size_t)(h0 + i)));
  }
  if (tid == 0) uqn = 0;
  __syncthreads();
  const UQueue q{uqe, &uqn, kApiQueue};
  WaveLms<kScrUnroll> wl;
  wl.load(lmf, nl * (wave & 1) / 2, nl * ((wave & 1) + 1) / 2);
  for (int t = __builtin_amdgcn_readfirstlane(wave); t < 2 * nh; t += NW) {
    const int j = t >> 1;
    const Xf* T = (const Xf*)(c2w + 12 * (size_t)(h0 + j));  // R[9], t[3] = mk::Xf
    long long s;
    int c;
    wl.sums(pf[j], fd.scam, fd.w, fd.h, fd.bgr, mask, q, j, T, lmk.xyz, cmp, s, c);
    if (lane == 0) {
      atomicAdd(&hs[j], (unsigned long long)s);
      atomicAdd(&hn[j], c);
    }
  }
  __syncthreads();
  block_drain(q, lmk.xyz, cmp, fd.w, fd.h, fd.bgr, mask,
              [&](int t) -> const Xf& { return *(const Xf*)(c2w + 12 * (size_t)(h0 + t)); },
              [&](int t, int e) {
                atomicAdd(&hs[t], (unsigned long long)e);
                atomicAdd(&hn[t], 1);
              });
  __syncthreads();
  for (int i = tid; i < nh; i += blockDim.x) {
    const int c = hn[i];
    err[h0 + i] = c <= 0 ? DBL_MAX : (double)(long long)hs[i] / ((double)c * 1.1);
    nproj[h0 + i] = c;
  }
}
__global__ __launch_bounds__(64 * kApiHyps) void k_score_api(const FrameDesc* __restrict__ frames, const uint8_t* mask,
                                                             Landmarks lmk, const double* __restrict__ c2w, int n,
                                                             int fast, double* __restrict__ err,
                                                             int32_t* __restrict__ nproj) {
  const FrameDesc fd = frames[0];
  if (fast) {
    if (mask) score_api_fast<kApiHyps>(fd, &frames[0].cam, MaskBytes{mask}, lmk, c2w, n, err, nproj);
    else score_api_fast<kApiHyps>(fd, &frames[0].cam, MaskNone{}, lmk, c2w, n, err, nproj);
    return;
  }
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int h = blockIdx.x * kApiHyps + wave;
  __shared__ ColorLds cls[kApiHyps];
  if (h >= n) return;
  Xf T;
  for (int k = 0; k < 9; k++) T.R[k] = c2w[12 * h + k];
  for (int k = 0; k < 3; k++) T.t[k] = c2w[12 * h + 9 + k];
  double e;
  int np;
  wave_score_color(T, lmk.xyz + 3 * (lmk.nw + lmk.nr), lmk.ng, fd.cam, fd.bgr, fd.w, fd.h, &cls[wave], &e, &np);
  if (lane == 0) {
    err[h] = e;
    nproj[h] = np;
  }
}

// ============================================================ synth render
__global__ __launch_bounds__(256) void k_synth(const mantis_synth::Cam* __restrict__ cams, const uint64_t* seeds,
                                               uint8_t* out, size_t plane) {
  const int f = blockIdx.y;
  const mantis_synth::Cam c = cams[f];
  const size_t n = (size_t)c.w * c.h;
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (size_t)gridDim.x * blockDim.x)
    mantis_synth::render_pixel(c, (int)(p % c.w), (int)(p / c.w), seeds[f], out + (size_t)f * plane + 3 * p);
}

}  // namespace mk
