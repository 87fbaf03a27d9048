// Border following and polygon approximation for the quad detector
// (detectQuadrilaterals, include/mantis3/QuadDetection.h:216-226), as
// device/host code.
//
// The reference calls cv::findContours(RETR_CCOMP, CHAIN_APPROX_SIMPLE) and
// cv::approxPolyDP(eps = POLYGON_EPSILON, closed) [3P, OpenCV >= 3.2]. The
// sequential Suzuki–Abe raster scan is replaced by an equivalent parallel
// formulation: every 8-connected foreground component
// has one outer border starting at its raster-first pixel, every enclosed
// 4-connected background component (hole) one hole border starting left of
// its raster-first pixel; each border is then followed independently here.
// The path depends only on the binary image (OpenCV's NBD marks never change
// which pixels are nonzero), so one work-item per border reproduces
// icvFetchContour's point sequence exactly.
#pragma once
#include <cstdint>

#include "mk_math.h"

namespace mk {

// Direction codes 0..7: right, up-right, up, up-left, left, down-left, down, down-right.
MK_HD int code_dx(int s) { return (s == 0 || s == 1 || s == 7) ? 1 : ((s >= 3 && s <= 5) ? -1 : 0); }
MK_HD int code_dy(int s) { return (s >= 1 && s <= 3) ? -1 : ((s >= 5 && s <= 7) ? 1 : 0); }

// Follow one border of the zero-padded binary image (Wp = W + 2 columns).
// `nz(idx)` tests a padded pixel. Writes CHAIN_APPROX_SIMPLE points (image
// coordinates = padded - 1) when out != nullptr (up to cap); returns the count.
template <class NZ>
MK_HD int trace_border(const NZ& nz, int Wp, int sx, int sy, bool hole, int32_t* out, int cap) {
  int deltas[16];
  for (int k = 0; k < 8; k++) deltas[k] = deltas[k + 8] = code_dy(k) * Wp + code_dx(k);
  int i0 = sy * Wp + sx;
  int s_end, s;
  s_end = s = hole ? 0 : 4;
  int i1;
  do {
    s = (s - 1) & 7;
    i1 = i0 + deltas[s];
  } while (!nz(i1) && s != s_end);
  int px = sx - 1, py = sy - 1;
  int n = 0;
  if (s == s_end) {
    if (out && n < cap) { out[0] = px; out[1] = py; }
    return 1;
  }
  int i3 = i0, i4;
  int prev_s = s ^ 4;
  for (;;) {
    s_end = s;
    for (;;) {
      i4 = i3 + deltas[++s];
      if (nz(i4)) break;
    }
    s &= 7;
    if (s != prev_s) {
      if (out && n < cap) { out[2 * n] = px; out[2 * n + 1] = py; }
      n++;
      prev_s = s;
    }
    px += code_dx(s);
    py += code_dy(s);
    if (i4 == i0 && i3 == i1) break;
    i3 = i4;
    s = (s + 4) & 7;
  }
  return n;
}

// Same border following driven by the packed 8-neighbourhood of the current
// pixel: bit k of nb(x, y) = pixel in direction code k is nonzero (padded
// coordinates). One neighbourhood fetch per step replaces up to 8 probes;
// the next direction is a rotate + count-trailing-zeros. Equal to
// trace_border point for point (tests/test_host_logic.py).
MK_HD uint32_t nb8_from_rows(uint32_t up, uint32_t mid, uint32_t dn) {
  // each argument: 3 bits (x-1, x, x+1) of one row
  return ((mid >> 2) & 1u) | (((up >> 2) & 1u) << 1) | (((up >> 1) & 1u) << 2) | ((up & 1u) << 3) |
         ((mid & 1u) << 4) | ((dn & 1u) << 5) | (((dn >> 1) & 1u) << 6) | (((dn >> 2) & 1u) << 7);
}
MK_HD int ctz32(uint32_t v) {
#ifdef __HIP_DEVICE_COMPILE__
  return __builtin_ctz(v);
#else
  int k = 0;
  while (!(v & 1u)) { v >>= 1; k++; }
  return k;
#endif
}
// em(px, py) receives each CHAIN_APPROX_SIMPLE point in order (image
// coordinates); returns the point count.
template <class NB, class EM>
MK_HD int trace_border_nb_em(const NB& nb, int sx, int sy, bool hole, EM& em) {
  int x = sx, y = sy;
  uint32_t m = nb(x, y);
  const int s_end0 = hole ? 0 : 4;
  int s = s_end0;
  do {
    s = (s - 1) & 7;
  } while (!((m >> s) & 1u) && s != s_end0);
  int px = sx - 1, py = sy - 1;
  if (s == s_end0) {
    em(px, py);
    return 1;
  }
  const int x1 = sx + code_dx(s), y1 = sy + code_dy(s);  // i1
  int n = 0;
  int prev_s = s ^ 4;
  // (x, y) = i3
  for (;;) {
    // first set direction after s, counter-clockwise: s+1, s+2, ...
    const uint32_t r = ((m | (m << 8)) >> (s + 1)) & 0xffu;
    s = (s + 1 + ctz32(r)) & 7;
    if (s != prev_s) {
      em(px, py);
      n++;
      prev_s = s;
    }
    const int dx = code_dx(s), dy = code_dy(s);
    px += dx;
    py += dy;
    const int x4 = x + dx, y4 = y + dy;
    if (x4 == sx && y4 == sy && x == x1 && y == y1) break;
    x = x4;
    y = y4;
    m = nb(x, y);
    s = (s + 4) & 7;
  }
  return n;
}
struct ArrayEmit {
  int32_t* out;
  int cap, n;
  MK_HD void operator()(int px, int py) {
    if (out && n < cap) { out[2 * n] = px; out[2 * n + 1] = py; }
    n++;
  }
};
template <class NB>
MK_HD int trace_border_nb(const NB& nb, int sx, int sy, bool hole, int32_t* out, int cap) {
  ArrayEmit em{out, cap, 0};
  return trace_border_nb_em(nb, sx, sy, hole, em);
}

// approxPolyDP's final clean-up of [almost] straight runs on the n_dp
// Douglas–Peucker points in dst (eps = squared epsilon); returns the count.
MK_HD int approx_cleanup(int32_t* dst, int new_count, double eps, bool closed0) {
  bool is_closed = closed0;
  int count = new_count;
  int pos, wpos, spx, spy, ptx, pty, epx, epy;
#define MK_READD(X, Y, P)           \
  do {                              \
    X = dst[2 * (P)];               \
    Y = dst[2 * (P) + 1];           \
    if (++(P) >= count) (P) = 0;    \
  } while (0)
  pos = is_closed ? count - 1 : 0;
  MK_READD(spx, spy, pos);
  wpos = pos;
  MK_READD(ptx, pty, pos);
  for (int i = !is_closed; i < count - !is_closed && new_count > 2; i++) {
    double dx, dy, dist, succ;
    MK_READD(epx, epy, pos);
    dx = epx - spx;
    dy = epy - spy;
    dist = fabs((ptx - spx) * dy - (pty - spy) * dx);
    succ = (ptx - spx) * (epx - ptx) + (pty - spy) * (epy - pty);
    if (dist * dist <= 0.5 * eps * (dx * dx + dy * dy) && dx != 0 && dy != 0 && succ >= 0) {
      new_count--;
      dst[2 * wpos] = spx = epx;
      dst[2 * wpos + 1] = spy = epy;
      if (++wpos >= count) wpos = 0;
      MK_READD(ptx, pty, pos);
      i++;
      continue;
    }
    dst[2 * wpos] = spx = ptx;
    dst[2 * wpos + 1] = spy = pty;
    if (++wpos >= count) wpos = 0;
    ptx = epx;
    pty = epy;
  }
  if (!is_closed) { dst[2 * wpos] = ptx; dst[2 * wpos + 1] = pty; }
#undef MK_READD
  return new_count;
}

// Point sources of approx_poly: x, y int pairs, or (on the device's contour
// pool) one 32-bit word per point, x | y << 16 (image coordinates < 65536): a
// point is one load and one register, so a lane's read-ahead holds twice the
// points in the same registers. `Raw` is what a read-ahead slot keeps.
struct PtPairs {
  const int32_t* p;
  static constexpr int kAhead = 4;
  struct Raw { int x, y; };
  MK_HD Raw ld(int i) const { return Raw{p[2 * i], p[2 * i + 1]}; }
  MK_HD static int x(const Raw& r) { return r.x; }
  MK_HD static int y(const Raw& r) { return r.y; }
};
#ifndef MK_APPROX_AHEAD_PACKED
#define MK_APPROX_AHEAD_PACKED 8
#endif
struct PtPacked {
  const uint32_t* p;
  static constexpr int kAhead = MK_APPROX_AHEAD_PACKED;
  typedef uint32_t Raw;
  MK_HD Raw ld(int i) const { return p[i]; }
  MK_HD static int x(Raw r) { return (int)(r & 0xffffu); }
  MK_HD static int y(Raw r) { return (int)(r >> 16); }
};

// cv::approxPolyDP (approxPolyDP_<int>, closed or open) on n points `src`
// (x,y int pairs, or a point source above). dst needs n pairs, stack n slices
// (2 ints each). Returns the output count.
// max_dp > 0: stop once the Douglas-Peucker stage has emitted max_dp points
// and return max_dp + 1 (the quad detector passes 10: the clean-up removes at
// most every other point, so 10 or more DP points can never end as 4).
template <class PS>
MK_HD int approx_poly(const PS& src, int count0, double eps, bool closed0, int32_t* dst, int32_t* stack,
                      int max_dp = 0);
MK_HD int approx_poly(const int32_t* src, int count0, double eps, bool closed0, int32_t* dst, int32_t* stack,
                      int max_dp = 0) {
  return approx_poly(PtPairs{src}, count0, eps, closed0, dst, stack, max_dp);
}
template <class PS>
MK_HD int approx_poly(const PS& src, int count0, double eps, bool closed0, int32_t* dst, int32_t* stack,
                      int max_dp) {
  int count = count0;
  if (count == 0) return 0;
  int top = 0;
  int init_iters = 3;
  int sl_s = 0, sl_e = 0, rs_s = 0, rs_e = 0;
  int spx = -1000000, spy = -1000000, epx = 0, epy = 0, ptx = 0, pty = 0;
  int i = 0, j, pos = 0, wpos, new_count = 0;
  bool is_closed = closed0;
  bool le_eps = false;
#define MK_READ(X, Y, P)            \
  do {                              \
    const auto r_ = src.ld(P);      \
    X = PS::x(r_);                  \
    Y = PS::y(r_);                  \
    if (++(P) >= count) (P) = 0;    \
  } while (0)
#define MK_PUSH(S, E) \
  do {                \
    stack[2 * top] = (S); stack[2 * top + 1] = (E); top++; \
  } while (0)
  eps *= eps;
  if (!is_closed) {
    rs_s = count;
    epx = PS::x(src.ld(0)); epy = PS::y(src.ld(0));
    spx = PS::x(src.ld(count - 1)); spy = PS::y(src.ld(count - 1));
    if (spx != epx || spy != epy) {
      sl_s = 0;
      sl_e = count - 1;
      MK_PUSH(sl_s, sl_e);
    } else {
      is_closed = true;
      init_iters = 1;
    }
  }
  // The point reads of the scans below go kApproxAhead at a time (indices
  // wrapped, every load issued before the first is used): one memory round
  // trip per group instead of per point on the device, where one lane walks a
  // border and each read is an L2 trip. Same points, same order, same
  // arithmetic as cv::approxPolyDP's scans.
  constexpr int kApproxAhead = PS::kAhead;
  if (is_closed) {
    rs_s = 0;
    for (i = 0; i < init_iters; i++) {
      double dist, max_dist = 0;
      pos = (pos + rs_s) % count;
      MK_READ(spx, spy, pos);
      for (j = 1; j < count; j += kApproxAhead) {
        typename PS::Raw g[kApproxAhead];
        int p = pos;
        for (int k = 0; k < kApproxAhead; k++) {  // wrapped indices stay inside the border
          g[k] = src.ld(p);
          if (++p >= count) p = 0;
        }
        const int nk = count - j < kApproxAhead ? count - j : kApproxAhead;
        for (int k = 0; k < kApproxAhead; k++) {
          if (k >= nk) break;
          double dx, dy;
          dx = PS::x(g[k]) - spx;
          dy = PS::y(g[k]) - spy;
          dist = dx * dx + dy * dy;
          if (dist > max_dist) {
            max_dist = dist;
            rs_s = j + k;
          }
        }
        ptx = PS::x(g[nk - 1]);
        pty = PS::y(g[nk - 1]);
        pos += nk;
        if (pos >= count) pos -= count;
      }
      le_eps = max_dist <= eps;
    }
    if (!le_eps) {
      rs_e = sl_s = pos % count;
      sl_e = rs_s = (rs_s + sl_s) % count;
      MK_PUSH(rs_s, rs_e);
      MK_PUSH(sl_s, sl_e);
    } else {
      dst[2 * new_count] = spx; dst[2 * new_count + 1] = spy; new_count++;
    }
  }
  while (top > 0) {
    top--;
    sl_s = stack[2 * top];
    sl_e = stack[2 * top + 1];
    {
      const auto e_ = src.ld(sl_e);
      epx = PS::x(e_); epy = PS::y(e_);
    }
    pos = sl_s;
    MK_READ(spx, spy, pos);
    if (pos != sl_e) {
      double dx, dy, dist, max_dist = 0;
      dx = epx - spx;
      dy = epy - spy;
      int left = sl_e - pos;  // reads until pos reaches sl_e
      if (left < 0) left += count;
      while (left > 0) {
        typename PS::Raw g[kApproxAhead];
        int p = pos;
        for (int k = 0; k < kApproxAhead; k++) {
          g[k] = src.ld(p);
          if (++p >= count) p = 0;
        }
        const int nk = left < kApproxAhead ? left : kApproxAhead;
        for (int k = 0; k < kApproxAhead; k++) {
          if (k >= nk) break;
          ptx = PS::x(g[k]);
          pty = PS::y(g[k]);
          if (++pos >= count) pos = 0;
          dist = fabs((pty - spy) * dx - (ptx - spx) * dy);
          if (dist > max_dist) {
            max_dist = dist;
            rs_s = (pos + count - 1) % count;
          }
        }
        left -= nk;
      }
      le_eps = max_dist * max_dist <= eps * (dx * dx + dy * dy);
    } else {
      le_eps = true;
      const auto s_ = src.ld(sl_s);
      spx = PS::x(s_); spy = PS::y(s_);
    }
    if (le_eps) {
      dst[2 * new_count] = spx; dst[2 * new_count + 1] = spy; new_count++;
      if (max_dp > 0 && new_count >= max_dp) return max_dp + 1;
    } else {
      rs_e = sl_e;
      sl_e = rs_s;
      MK_PUSH(rs_s, rs_e);
      MK_PUSH(sl_s, sl_e);
    }
  }
  if (!is_closed) {
    const auto l_ = src.ld(count - 1);
    dst[2 * new_count] = PS::x(l_); dst[2 * new_count + 1] = PS::y(l_); new_count++;
  }
#undef MK_READ
#undef MK_PUSH
  return approx_cleanup(dst, new_count, eps, closed0);
}

}  // namespace mk
