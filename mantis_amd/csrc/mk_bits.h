// Bit-packed binary planes for the detector/mask morphology
// (mantis3.cpp:84-94 dilate/erode, HypothesisEvaluation.h:337-351
// cleanImageByEdge): one bit per pixel, rows of WW = ceil(W/32) uint32 words,
// pixel x of a row at bit (x & 31) of word (x >> 5). A 32-pixel word is one
// work-item, so a pass moves W*H/8 bytes instead of W*H.
//
// Rectangle dilate/erode use OpenCV's clipped window (the default border
// value makes outside pixels neutral): outside the image a dilation reads 0
// and an erosion reads 1.
#pragma once
#include <cstdint>

#include "mk_math.h"

namespace mk {
namespace bits {

MK_HD int words(int W) { return (W + 31) >> 5; }
// Tiled mask plane (the scorers' cleanImageByEdge mask): word (y, w) -- 32
// pixels of row y -- at w * Hp + y, word columns of Hp = H rounded up to 32
// rows, so one 128-byte line holds a 32 x 32 pixel tile and a pixel
// neighbourhood touches a few lines instead of one line per row; a lookup is
// (x >> 5) * Hp + y (one multiply-add, no 64-bit index).
MK_HD int tiled_rows(int H) { return (H + 31) & ~31; }
MK_HD size_t tiled_word(int y, int w, int Hp) { return (size_t)w * Hp + y; }
MK_HD size_t tiled_words(int W, int H) { return (size_t)words(W) * tiled_rows(H); }

// mask of the valid pixels of word w
MK_HD uint32_t valid(int w, int W) {
  const int rem = W - (w << 5);
  return rem >= 32 ? 0xffffffffu : (rem <= 0 ? 0u : ((1u << rem) - 1u));
}

// word w of a row with the outside filled with the neutral element
MK_HD uint32_t load(const uint32_t* row, int w, int W, uint32_t ident) {
  const int WW = words(W);
  if (w < 0 || w >= WW) return ident;
  const uint32_t v = valid(w, W);
  return (row[w] & v) | (ident & ~v);
}

// horizontal pass: out(x) = OP_{|k|<=r} in(x+k), 0 < r < 32
MK_HD uint32_t hword(const uint32_t* row, int w, int W, int r, bool dil) {
  const uint32_t ident = dil ? 0u : 0xffffffffu;
  const uint32_t prev = load(row, w - 1, W, ident), cur = load(row, w, W, ident), next = load(row, w + 1, W, ident);
  uint32_t acc = cur;
  for (int k = 1; k <= r; k++) {
    const uint32_t right = (cur >> k) | (next << (32 - k));  // in(x + k)
    const uint32_t left = (cur << k) | (prev >> (32 - k));   // in(x - k)
    if (dil) acc |= right | left;
    else acc &= right & left;
  }
  return acc & valid(w, W);
}

// vertical pass: out(y) = OP_{|k|<=r, 0<=y+k<H} in(y+k)
MK_HD uint32_t vword(const uint32_t* plane, int w, int y, int W, int H, int r, bool dil) {
  const int WW = words(W);
  uint32_t acc = dil ? 0u : 0xffffffffu;
  const int lo = y - r < 0 ? 0 : y - r, hi = y + r >= H ? H - 1 : y + r;
  for (int yy = lo; yy <= hi; yy++) {
    const uint32_t v = plane[(size_t)yy * WW + w];
    if (dil) acc |= v;
    else acc &= v;
  }
  return acc & valid(w, W);
}

// NOT(morphological gradient, 3x3 cross) at word (w, y): 1 where the clipped
// cross max equals the clipped cross min
MK_HD uint32_t ngword(const uint32_t* E, int w, int y, int W, int H) {
  const int WW = words(W);
  const uint32_t* row = E + (size_t)y * WW;
  const uint32_t p0 = load(row, w - 1, W, 0u), c0 = load(row, w, W, 0u), n0 = load(row, w + 1, W, 0u);
  const uint32_t p1 = load(row, w - 1, W, ~0u), c1 = load(row, w, W, ~0u), n1 = load(row, w + 1, W, ~0u);
  uint32_t mx = c0 | ((c0 >> 1) | (n0 << 31)) | ((c0 << 1) | (p0 >> 31));
  uint32_t mn = c1 & ((c1 >> 1) | (n1 << 31)) & ((c1 << 1) | (p1 >> 31));
  if (y > 0) {
    const uint32_t u = load(E + (size_t)(y - 1) * WW, w, W, 0u);
    mx |= u;
    mn &= u;
  }
  if (y + 1 < H) {
    const uint32_t d = load(E + (size_t)(y + 1) * WW, w, W, 0u);
    mx |= d;
    mn &= d;
  }
  return ~(mx ^ mn) & valid(w, W);
}

// M0 = edge | (border pixels of NOT(gradient)): a NOT-gradient pixel on the
// image edge or with a 4-neighbour that is not NOT-gradient — the union of
// all RETR_LIST contours drawn with thickness 1 (DESIGN.md "Mask")
MK_HD uint32_t m0word(const uint32_t* E, int w, int y, int W, int H) {
  const int WW = words(W);
  const uint32_t ng = ngword(E, w, y, W, H);
  const uint32_t ngl = w > 0 ? ngword(E, w - 1, y, W, H) : 0u;
  const uint32_t ngr = w + 1 < WW ? ngword(E, w + 1, y, W, H) : 0u;
  const uint32_t left = (ng << 1) | (ngl >> 31);   // ng(x - 1), 0 left of the image
  const uint32_t right = (ng >> 1) | (ngr << 31);  // ng(x + 1), 0 right of the image
  const uint32_t up = y > 0 ? ngword(E, w, y - 1, W, H) : 0u;
  const uint32_t down = y + 1 < H ? ngword(E, w, y + 1, W, H) : 0u;
  const uint32_t b = ng & (~left | ~right | ~up | ~down);
  return (E[(size_t)y * WW + w] | b) & valid(w, W);
}

}  // namespace bits
}  // namespace mk
