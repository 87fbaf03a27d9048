// ORACLE — test infrastructure only. Never linked into the product path.
//
// CPU restatement of the OpenCV 3.x imgproc calls on the mantis3 hot path
// (OpenCV is not vendored in the reference and not installed here, so every
// semantic below is restated from the published 3.3-era sources [3P] and
// documented in DESIGN.md §Oracle):
//   cvtColor BGR2GRAY       QuadDetection.h:209, HypothesisEvaluation.h:323
//   GaussianBlur 3x3 s=3    QuadDetection.h:211, HypothesisEvaluation.h:326
//   Canny(50,150,3,L1)      QuadDetection.h:212, HypothesisEvaluation.h:327
//   dilate/erode            QuadDetection.h:213-214, HypothesisEvaluation.h:353-372
//   morphologyEx GRADIENT   HypothesisEvaluation.h:338
//   findContours            QuadDetection.h:216 (CCOMP), HypothesisEvaluation.h:342 (LIST)
//   approxPolyDP            QuadDetection.h:221
//   drawContours            HypothesisEvaluation.h:348
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace orc {

struct Img8 {
  int w = 0, h = 0;
  std::vector<uint8_t> d;
  Img8() {}
  Img8(int w_, int h_, uint8_t v = 0) : w(w_), h(h_), d((std::size_t)w_ * h_, v) {}
  uint8_t& at(int x, int y) { return d[(std::size_t)y * w + x]; }
  uint8_t at(int x, int y) const { return d[(std::size_t)y * w + x]; }
};

struct Pt { int x, y; };
using Contour = std::vector<Pt>;

// BGR (row step in bytes) -> gray, (1868 B + 9617 G + 4899 R + 8192) >> 14
Img8 bgr2gray(const uint8_t* bgr, int w, int h, int step);
// 3x3 Gaussian, sigma 3, OpenCV <= 3.3 fixed point: kernel [84,89,84] (x256,
// sum 257) in both passes, (acc + 2^15) >> 16 with saturation, REFLECT_101.
Img8 gauss3x3(const Img8& src);
// Canny with 3x3 Sobel (REPLICATE), L1 magnitude, TG22 NMS, hysteresis.
// Pixels outside the image have magnitude 0, so border pixels may be edges.
Img8 canny(const Img8& gray, int low, int high);
// cv::Canny's hysteresis alone on a class plane (0 none, 1 weak candidate, 2 strong)
Img8 hysteresis(const Img8& cls);
Img8 hysteresis_walk(std::vector<uint8_t>& map, int W, int H, std::vector<std::pair<int, int>>& stack);
// Morphology with a (2r+1)x(2r+1) rectangle; the border never contributes
// (default DBL_MAX border and BORDER_REPLICATE are equivalent for rect max/min).
Img8 dilate_rect(const Img8& src, int r);
Img8 erode_rect(const Img8& src, int r);
// morphologyEx(MORPH_GRADIENT, ellipse 3x3 == cross)
Img8 gradient_cross(const Img8& src);

// findContours (OpenCV >= 3.2: 1-px zero pad, offset -1) sequential
// Suzuki–Abe border following, CHAIN_APPROX_SIMPLE. mode 1 = LIST, 2 = CCOMP.
// Output is in OpenCV's tree pre-order.
std::vector<Contour> find_contours(const Img8& bin, int mode, std::vector<int>* is_hole = nullptr);
// approxPolyDP (closed) on int points
Contour approx_poly_dp(const Contour& src, double eps, bool closed);
// drawContours(img, contours, i, 255, thickness 1, LINE_8) for every i
void draw_contours(Img8& dst, const std::vector<Contour>& cs, uint8_t val);

}  // namespace orc
