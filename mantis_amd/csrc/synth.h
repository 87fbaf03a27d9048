// Synthetic fisheye grid renderer (SURVEY §8(d) scene), shared by the HIP
// render kernel (bench inputs generated in HBM) and the host build used by
// CPU tests (tools/libmantis_synth.so). It replaces the reference's OpenGL
// GridRenderer (include/mantis3/GridRenderer.cpp:211-353, not on the path).
//
// Scene: plane z = 0, 10 lines per axis at -1.44 + 0.32 k (k = 0..9) over the
// extent |x|,|y| <= 1.44 (+ half width), width 0.04 m. y = +1.44 is GREEN
// (50,255,85), y = -1.44 is RED (50,85,255), every other line WHITE; the
// colored lines win at their corners (as params/map.yaml assigns the corner
// landmarks). Floor BGR (120,110,105) + per-channel integer noise in [-20,20]
// from a counter-based PCG hash of (seed, pixel, channel); rays that miss the
// floor render (40,40,40). No anti-aliasing: one ray through each pixel
// centre, inverted through the equidistant fisheye model with Newton steps.
#pragma once
#include <cmath>
#include <cstdint>

#ifdef __HIPCC__
#define MANTIS_HD __host__ __device__
#else
#define MANTIS_HD
#endif

namespace mantis_synth {

struct Cam {
  double fx, fy, cx, cy;
  double k[4];
  double R_wc[9];  // camera axes in world (columns), row-major
  double pos[3];   // camera centre in world
  int32_t w, h;
  int32_t pad[2];
};

MANTIS_HD inline uint32_t pcg_hash(uint64_t v) {
  uint64_t s = v * 6364136223846793005ULL + 1442695040888963407ULL;
  s ^= s >> 33;
  s *= 0xff51afd7ed558ccdULL;
  s ^= s >> 33;
  s *= 0xc4ceb9fe1a85ec53ULL;
  s ^= s >> 33;
  uint32_t xorshifted = (uint32_t)(((s >> 18u) ^ s) >> 27u);
  uint32_t rot = (uint32_t)(s >> 59u);
  return (xorshifted >> rot) | (xorshifted << ((-rot) & 31));
}

// theta_d = theta (1 + k1 t^2 + k2 t^4 + k3 t^6 + k4 t^8), solved for theta
MANTIS_HD inline double inv_fisheye(const double* k, double td) {
  double th = td;
  for (int it = 0; it < 30; it++) {
    double t2 = th * th, t4 = t2 * t2, t6 = t4 * t2, t8 = t4 * t4;
    double f = th * (1 + k[0] * t2 + k[1] * t4 + k[2] * t6 + k[3] * t8) - td;
    double df = 1 + 3 * k[0] * t2 + 5 * k[1] * t4 + 7 * k[2] * t6 + 9 * k[3] * t8;
    double step = f / df;
    th -= step;
    if (fabs(step) < 1e-15) break;
  }
  return th;
}

MANTIS_HD inline void render_pixel(const Cam& c, int x, int y, uint64_t seed, uint8_t* bgr) {
  double mx = ((double)x - c.cx) / c.fx, my = ((double)y - c.cy) / c.fy;
  double td = sqrt(mx * mx + my * my);
  double dx, dy, dz;
  if (td < 1e-12) {
    dx = 0; dy = 0; dz = 1;
  } else {
    double th = inv_fisheye(c.k, td);
    double s = sin(th) / td;
    dx = mx * s; dy = my * s; dz = cos(th);
  }
  // ray in world
  double wx = c.R_wc[0] * dx + c.R_wc[1] * dy + c.R_wc[2] * dz;
  double wy = c.R_wc[3] * dx + c.R_wc[4] * dy + c.R_wc[5] * dz;
  double wz = c.R_wc[6] * dx + c.R_wc[7] * dy + c.R_wc[8] * dz;
  int b = 40, g = 40, r = 40;
  if (wz < -1e-9) {
    double t = -c.pos[2] / wz;
    double X = c.pos[0] + t * wx, Y = c.pos[1] + t * wy;
    const double half = 0.02, lo = -1.44, sp = 0.32, ext = 1.44 + half;
    int col = 0;  // 0 floor, 1 white, 2 red, 3 green
    if (fabs(X) <= ext && fabs(Y) <= ext) {
      double fy = (Y - lo) / sp, fx = (X - lo) / sp;
      double ky = floor(fy + 0.5), kx = floor(fx + 0.5);
      bool onh = ky >= 0 && ky <= 9 && fabs(Y - (lo + ky * sp)) <= half;
      bool onv = kx >= 0 && kx <= 9 && fabs(X - (lo + kx * sp)) <= half;
      if (onh && ky == 0) col = 2;
      else if (onh && ky == 9) col = 3;
      else if (onh || onv) col = 1;
    }
    if (col == 1) { b = 255; g = 255; r = 255; }
    else if (col == 2) { b = 50; g = 85; r = 255; }
    else if (col == 3) { b = 50; g = 255; r = 85; }
    else {
      uint64_t idx = ((uint64_t)y * (uint64_t)c.w + (uint64_t)x) * 3ULL;
      b = 120 + (int)(pcg_hash(seed ^ (idx + 0)) % 41u) - 20;
      g = 110 + (int)(pcg_hash(seed ^ (idx + 1)) % 41u) - 20;
      r = 105 + (int)(pcg_hash(seed ^ (idx + 2)) % 41u) - 20;
    }
  }
  bgr[0] = (uint8_t)b;
  bgr[1] = (uint8_t)g;
  bgr[2] = (uint8_t)r;
}

}  // namespace mantis_synth
