// ORACLE — test infrastructure only. Never linked into the product path.
// See o_imgproc.hpp for the reference call sites each function restates.
#include "o_imgproc.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <functional>

namespace orc {

Img8 bgr2gray(const uint8_t* bgr, int w, int h, int step) {
  Img8 g(w, h);
  for (int y = 0; y < h; y++) {
    const uint8_t* row = bgr + (size_t)y * step;
    for (int x = 0; x < w; x++) {
      int b = row[3 * x], gg = row[3 * x + 1], r = row[3 * x + 2];
      g.at(x, y) = (uint8_t)((1868 * b + 9617 * gg + 4899 * r + 8192) >> 14);
    }
  }
  return g;
}

static inline int reflect101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = (i < 0) ? -i : 2 * n - 2 - i;
  return i;
}

Img8 gauss3x3(const Img8& s) {
  const int k0 = 84, k1 = 89;  // getGaussianKernel(3, 3) x 256, rounded
  std::vector<int> rows((size_t)s.w * s.h);
  for (int y = 0; y < s.h; y++)
    for (int x = 0; x < s.w; x++)
      rows[(size_t)y * s.w + x] = k0 * s.at(reflect101(x - 1, s.w), y) + k1 * s.at(x, y) +
                                  k0 * s.at(reflect101(x + 1, s.w), y);
  Img8 o(s.w, s.h);
  for (int y = 0; y < s.h; y++)
    for (int x = 0; x < s.w; x++) {
      int acc = k0 * rows[(size_t)reflect101(y - 1, s.h) * s.w + x] + k1 * rows[(size_t)y * s.w + x] +
                k0 * rows[(size_t)reflect101(y + 1, s.h) * s.w + x];
      int v = (acc + (1 << 15)) >> 16;
      o.at(x, y) = (uint8_t)std::min(255, std::max(0, v));
    }
  return o;
}

Img8 canny(const Img8& g, int low, int high) {
  const int W = g.w, H = g.h;
  auto px = [&](int x, int y) -> int {
    x = std::min(std::max(x, 0), W - 1);
    y = std::min(std::max(y, 0), H - 1);
    return g.at(x, y);
  };
  std::vector<int> dx((size_t)W * H), dy((size_t)W * H);
  // magnitude with a zero ring: (W+2) x (H+2)
  std::vector<int> mag((size_t)(W + 2) * (H + 2), 0);
  auto M = [&](int x, int y) -> int& { return mag[(size_t)(y + 1) * (W + 2) + (x + 1)]; };
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      int gx = (px(x + 1, y - 1) - px(x - 1, y - 1)) + 2 * (px(x + 1, y) - px(x - 1, y)) +
               (px(x + 1, y + 1) - px(x - 1, y + 1));
      int gy = (px(x - 1, y + 1) - px(x - 1, y - 1)) + 2 * (px(x, y + 1) - px(x, y - 1)) +
               (px(x + 1, y + 1) - px(x + 1, y - 1));
      dx[(size_t)y * W + x] = gx;
      dy[(size_t)y * W + x] = gy;
      M(x, y) = std::abs(gx) + std::abs(gy);
    }
  const int SHIFT = 15;
  const int TG22 = (int)(0.4142135623730950488016887242097 * (1 << SHIFT) + 0.5);
  // map: 0 = candidate, 1 = not an edge, 2 = edge (ring of 1)
  std::vector<uint8_t> map((size_t)(W + 2) * (H + 2), 1);
  auto MP = [&](int x, int y) -> uint8_t& { return map[(size_t)(y + 1) * (W + 2) + (x + 1)]; };
  std::vector<std::pair<int, int>> stack;
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      int m = M(x, y);
      bool push = false;
      if (m > low) {
        int xs = dx[(size_t)y * W + x], ys = dy[(size_t)y * W + x];
        int ax = std::abs(xs);
        int ay = std::abs(ys) << SHIFT;
        int tg22x = ax * TG22;
        if (ay < tg22x) {
          push = m > M(x - 1, y) && m >= M(x + 1, y);
        } else {
          int tg67x = tg22x + (ax << (SHIFT + 1));
          if (ay > tg67x) {
            push = m > M(x, y - 1) && m >= M(x, y + 1);
          } else {
            int s = (xs ^ ys) < 0 ? -1 : 1;
            push = m > M(x - s, y - 1) && m > M(x + s, y + 1);
          }
        }
      }
      if (!push) {
        MP(x, y) = 1;
      } else if (m > high) {
        MP(x, y) = 2;
        stack.push_back({x, y});
      } else {
        MP(x, y) = 0;
      }
    }
  return hysteresis_walk(map, W, H, stack);
}

// cv::Canny's hysteresis: from every strong pixel on the stack, the 8-neighbours
// still marked candidate (0) become edges (2) and are pushed in turn
// (OpenCV imgproc canny.cpp, the CANNY_POP loop); map is (W+2) x (H+2) with a ring of 1
Img8 hysteresis_walk(std::vector<uint8_t>& map, int W, int H, std::vector<std::pair<int, int>>& stack) {
  auto MP = [&](int x, int y) -> uint8_t& { return map[(size_t)(y + 1) * (W + 2) + (x + 1)]; };
  while (!stack.empty()) {
    auto [x, y] = stack.back();
    stack.pop_back();
    for (int oy = -1; oy <= 1; oy++)
      for (int ox = -1; ox <= 1; ox++) {
        if (!ox && !oy) continue;
        uint8_t& v = MP(x + ox, y + oy);
        if (v == 0) { v = 2; stack.push_back({x + ox, y + oy}); }
      }
  }
  Img8 o(W, H);
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) o.at(x, y) = MP(x, y) == 2 ? 255 : 0;
  return o;
}

// the same walk on a class plane (0 none, 1 weak candidate, 2 strong), pushed in raster order
Img8 hysteresis(const Img8& cls) {
  const int W = cls.w, H = cls.h;
  std::vector<uint8_t> map((size_t)(W + 2) * (H + 2), 1);
  std::vector<std::pair<int, int>> stack;
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++) {
      const uint8_t v = cls.at(x, y);
      uint8_t& m = map[(size_t)(y + 1) * (W + 2) + (x + 1)];
      if (v == 2) {
        m = 2;
        stack.push_back({x, y});
      } else {
        m = v == 1 ? 0 : 1;
      }
    }
  return hysteresis_walk(map, W, H, stack);
}

static Img8 morph_rect(const Img8& s, int r, bool dil) {
  Img8 t(s.w, s.h), o(s.w, s.h);
  for (int y = 0; y < s.h; y++)
    for (int x = 0; x < s.w; x++) {
      int v = dil ? 0 : 255;
      for (int k = std::max(0, x - r); k <= std::min(s.w - 1, x + r); k++)
        v = dil ? std::max(v, (int)s.at(k, y)) : std::min(v, (int)s.at(k, y));
      t.at(x, y) = (uint8_t)v;
    }
  for (int y = 0; y < s.h; y++)
    for (int x = 0; x < s.w; x++) {
      int v = dil ? 0 : 255;
      for (int k = std::max(0, y - r); k <= std::min(s.h - 1, y + r); k++)
        v = dil ? std::max(v, (int)t.at(x, k)) : std::min(v, (int)t.at(x, k));
      o.at(x, y) = (uint8_t)v;
    }
  return o;
}
Img8 dilate_rect(const Img8& s, int r) { return morph_rect(s, r, true); }
Img8 erode_rect(const Img8& s, int r) { return morph_rect(s, r, false); }

Img8 gradient_cross(const Img8& s) {
  Img8 o(s.w, s.h);
  const int ox[5] = {0, -1, 1, 0, 0}, oy[5] = {0, 0, 0, -1, 1};
  for (int y = 0; y < s.h; y++)
    for (int x = 0; x < s.w; x++) {
      int mx = 0, mn = 255;
      for (int k = 0; k < 5; k++) {
        int xx = x + ox[k], yy = y + oy[k];
        if (xx < 0 || yy < 0 || xx >= s.w || yy >= s.h) continue;
        mx = std::max(mx, (int)s.at(xx, yy));
        mn = std::min(mn, (int)s.at(xx, yy));
      }
      o.at(x, y) = (uint8_t)(mx - mn);
    }
  return o;
}

// ---------------------------------------------------------------- contours
namespace {
struct CInfo {
  Contour pts;
  bool hole;
  int parent;               // index into infos, -1 = frame
  std::vector<int> kids;    // prepended (reverse discovery order)
};
}  // namespace

std::vector<Contour> find_contours(const Img8& bin, int mode, std::vector<int>* is_hole_out) {
  const int Wp = bin.w + 2, Hp = bin.h + 2;
  std::vector<int> img((size_t)Wp * Hp, 0);
  for (int y = 0; y < bin.h; y++)
    for (int x = 0; x < bin.w; x++) img[(size_t)(y + 1) * Wp + (x + 1)] = bin.at(x, y) ? 1 : 0;
  // direction codes 0..7: right, up-right, up, up-left, left, down-left, down, down-right
  const int cdx[8] = {1, 1, 0, -1, -1, -1, 0, 1}, cdy[8] = {0, -1, -1, -1, 0, 1, 1, 1};
  int deltas[16];
  for (int k = 0; k < 8; k++) deltas[k] = deltas[k + 8] = cdy[k] * Wp + cdx[k];

  std::vector<CInfo> infos;
  std::vector<int> frame_kids;
  auto trace = [&](int sx, int sy, bool hole, int id) {
    Contour pts;
    int i0 = sy * Wp + sx;
    int s_end, s;
    s_end = s = hole ? 0 : 4;
    int i1;
    do {
      s = (s - 1) & 7;
      i1 = i0 + deltas[s];
    } while (img[i1] == 0 && s != s_end);
    Pt pt{sx - 1, sy - 1};
    if (s == s_end) {  // single pixel domain
      img[i0] = -id;
      pts.push_back(pt);
      return pts;
    }
    int i3 = i0, i4;
    int prev_s = s ^ 4;
    for (;;) {
      s_end = s;
      for (;;) {
        i4 = i3 + deltas[++s];
        if (img[i4] != 0) break;
      }
      s &= 7;
      if ((unsigned)(s - 1) < (unsigned)s_end)
        img[i3] = -id;
      else if (img[i3] == 1)
        img[i3] = id;
      if (s != prev_s) {
        pts.push_back(pt);
        prev_s = s;
      }
      pt.x += cdx[s];
      pt.y += cdy[s];
      if (i4 == i0 && i3 == i1) break;
      i3 = i4;
      s = (s + 4) & 7;
    }
    return pts;
  };

  int next_id = 2;
  for (int y = 1; y < Hp; y++) {
    int lnbd_x = 0;
    int prev = 0;
    for (int x = 1; x < Wp; x++) {
      int p = img[(size_t)y * Wp + x];
      if (p == prev) continue;
      bool found = false, hole = false;
      if (prev == 0 && p == 1) {
        found = true;
      } else if (p == 0 && prev >= 1) {
        if (prev != 0 && prev != 1) lnbd_x = x - 1;
        found = true;
        hole = true;
      }
      if (!found) {
        prev = p;
        if (prev != 0 && prev != 1) lnbd_x = x;
        continue;
      }
      int parent = -1;
      if (!(mode <= 1 || (!hole && mode == 2) || lnbd_x <= 0)) {
        int lval = std::abs(img[(size_t)y * Wp + lnbd_x]);
        int par = lval - 2;
        if (infos[par].hole == hole) par = infos[par].parent;
        parent = par;
      }
      lnbd_x = x - (hole ? 1 : 0);
      int id = next_id++;
      CInfo ci;
      ci.hole = hole;
      ci.parent = parent;
      ci.pts = trace(x - (hole ? 1 : 0), y, hole, id);
      infos.push_back(std::move(ci));
      int me = (int)infos.size() - 1;
      if (parent < 0) frame_kids.insert(frame_kids.begin(), me);
      else infos[parent].kids.insert(infos[parent].kids.begin(), me);
      prev = img[(size_t)y * Wp + x];
    }
  }
  std::vector<Contour> out;
  std::function<void(int)> visit = [&](int i) {
    out.push_back(infos[i].pts);
    if (is_hole_out) is_hole_out->push_back(infos[i].hole ? 1 : 0);
    for (int k : infos[i].kids) visit(k);
  };
  for (int k : frame_kids) visit(k);
  return out;
}

Contour approx_poly_dp(const Contour& src, double eps, bool closed0) {
  int count = (int)src.size();
  Contour dst(count > 0 ? count : 0);
  if (count == 0) return {};
  struct Slice { int start, end; };
  std::vector<Slice> stack;
  int init_iters = 3;
  Slice slice{0, 0}, right_slice{0, 0};
  Pt start_pt{-1000000, -1000000}, end_pt{0, 0}, pt{0, 0};
  int i = 0, j, pos = 0, wpos, new_count = 0;
  bool is_closed = closed0;
  bool le_eps = false;
  auto READ = [&](Pt& p, int& ps) { p = src[ps]; if (++ps >= count) ps = 0; };
  eps *= eps;
  if (!is_closed) {
    right_slice.start = count;
    end_pt = src[0];
    start_pt = src[count - 1];
    if (start_pt.x != end_pt.x || start_pt.y != end_pt.y) {
      slice.start = 0;
      slice.end = count - 1;
      stack.push_back(slice);
    } else {
      is_closed = true;
      init_iters = 1;
    }
  }
  if (is_closed) {
    right_slice.start = 0;
    for (i = 0; i < init_iters; i++) {
      double dist, max_dist = 0;
      pos = (pos + right_slice.start) % count;
      READ(start_pt, pos);
      for (j = 1; j < count; j++) {
        double dx, dy;
        READ(pt, pos);
        dx = pt.x - start_pt.x;
        dy = pt.y - start_pt.y;
        dist = dx * dx + dy * dy;
        if (dist > max_dist) {
          max_dist = dist;
          right_slice.start = j;
        }
      }
      le_eps = max_dist <= eps;
    }
    if (!le_eps) {
      right_slice.end = slice.start = pos % count;
      slice.end = right_slice.start = (right_slice.start + slice.start) % count;
      stack.push_back(right_slice);
      stack.push_back(slice);
    } else {
      dst[new_count++] = start_pt;
    }
  }
  while (!stack.empty()) {
    slice = stack.back();
    stack.pop_back();
    end_pt = src[slice.end];
    pos = slice.start;
    READ(start_pt, pos);
    if (pos != slice.end) {
      double dx, dy, dist, max_dist = 0;
      dx = end_pt.x - start_pt.x;
      dy = end_pt.y - start_pt.y;
      while (pos != slice.end) {
        READ(pt, pos);
        dist = std::fabs((pt.y - start_pt.y) * dx - (pt.x - start_pt.x) * dy);
        if (dist > max_dist) {
          max_dist = dist;
          right_slice.start = (pos + count - 1) % count;
        }
      }
      le_eps = max_dist * max_dist <= eps * (dx * dx + dy * dy);
    } else {
      le_eps = true;
      start_pt = src[slice.start];
    }
    if (le_eps) {
      dst[new_count++] = start_pt;
    } else {
      right_slice.end = slice.end;
      slice.end = right_slice.start;
      stack.push_back(right_slice);
      stack.push_back(slice);
    }
  }
  if (!is_closed) dst[new_count++] = src[count - 1];

  // final clean-up of [almost] straight runs
  is_closed = closed0;
  count = new_count;
  auto READD = [&](Pt& p, int& ps) { p = dst[ps]; if (++ps >= count) ps = 0; };
  pos = is_closed ? count - 1 : 0;
  READD(start_pt, pos);
  wpos = pos;
  READD(pt, pos);
  for (i = !is_closed; i < count - !is_closed && new_count > 2; i++) {
    double dx, dy, dist, succ;
    READD(end_pt, pos);
    dx = end_pt.x - start_pt.x;
    dy = end_pt.y - start_pt.y;
    dist = std::fabs((pt.x - start_pt.x) * dy - (pt.y - start_pt.y) * dx);
    succ = (pt.x - start_pt.x) * (end_pt.x - pt.x) + (pt.y - start_pt.y) * (end_pt.y - pt.y);
    if (dist * dist <= 0.5 * eps * (dx * dx + dy * dy) && dx != 0 && dy != 0 && succ >= 0) {
      new_count--;
      dst[wpos] = start_pt = end_pt;
      if (++wpos >= count) wpos = 0;
      READD(pt, pos);
      i++;
      continue;
    }
    dst[wpos] = start_pt = pt;
    if (++wpos >= count) wpos = 0;
    pt = end_pt;
  }
  if (!is_closed) dst[wpos] = pt;
  dst.resize(new_count);
  return dst;
}

// OpenCV LineIterator(connectivity 8, leftToRight) + Line()
static void draw_line(Img8& img, Pt p1, Pt p2, uint8_t val) {
  int dx = p2.x - p1.x, dy = p2.y - p1.y;
  int s = dx < 0 ? -1 : 0;
  dx = (dx ^ s) - s;
  dy = (dy ^ s) - s;
  p1.x ^= (p1.x ^ p2.x) & s;
  p1.y ^= (p1.y ^ p2.y) & s;
  long step_pix = 1, istep = img.w;
  s = dy < 0 ? -1 : 0;
  dy = (dy ^ s) - s;
  istep = (istep ^ s) - s;
  s = dy > dx ? -1 : 0;
  dx ^= dy & s; dy ^= dx & s; dx ^= dy & s;
  step_pix ^= istep & s; istep ^= step_pix & s; step_pix ^= istep & s;
  int err = dx - (dy + dy), plusDelta = dx + dx, minusDelta = -(dy + dy);
  long plusStep = istep, minusStep = step_pix;
  int cnt = dx + 1;
  long off = (long)p1.y * img.w + p1.x;
  for (int k = 0; k < cnt; k++) {
    img.d[off] = val;
    int mask = err < 0 ? -1 : 0;
    err += minusDelta + (plusDelta & mask);
    off += minusStep + (plusStep & mask);
  }
}

void draw_contours(Img8& dst, const std::vector<Contour>& cs, uint8_t val) {
  for (const auto& c : cs) {
    if (c.empty()) continue;
    Pt prev = c.back();
    for (const Pt& p : c) {
      draw_line(dst, prev, p, val);
      prev = p;
    }
  }
}

}  // namespace orc
