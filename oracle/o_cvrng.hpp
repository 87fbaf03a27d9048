// ORACLE — test infrastructure only. Never linked into the product path.
//
// CPU restatement of cv::RNG as used by the reference: the global
// `cv::RNG rng(1)` (include/mantis3/Mantis3Params.h:87) drawn by
// generateRandomHypothesis (include/mantis3/PoseAdjustment.h:15-16), and the
// `cv::RNG rng(10)` noise of test/unit_test.cpp:196-203.
// OpenCV 3.x semantics [3P, unpinned]: multiply-with-carry step
//   state = (uint64)(uint32)state * 4164903690 + (state >> 32)
// and RNG::gaussian(sigma) = (float) Marsaglia–Tsang ziggurat (128 strips,
// r = 3.442619855899, v = 9.91256303526217e-3) times sigma.
#pragma once
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>

namespace orc {

struct CvRng {
  uint64_t state;
  explicit CvRng(uint64_t s = 0xffffffffULL) : state(s ? s : 0xffffffffULL) {}

  static inline uint64_t step(uint64_t x) { return (uint64_t)(uint32_t)x * 4164903690ULL + (x >> 32); }
  uint32_t next() { state = step(state); return (uint32_t)state; }

  struct Tables {
    uint32_t kn[128];
    float wn[128], fn[128];
    Tables() {
      const double m1 = 2147483648.0;
      double dn = 3.442619855899, tn = dn, vn = 9.91256303526217e-3;
      double q = vn / std::exp(-.5 * dn * dn);
      kn[0] = (uint32_t)((dn / q) * m1);
      kn[1] = 0;
      wn[0] = (float)(q / m1);
      wn[127] = (float)(dn / m1);
      fn[0] = 1.f;
      fn[127] = (float)std::exp(-.5 * dn * dn);
      for (int i = 126; i >= 1; i--) {
        dn = std::sqrt(-2. * std::log(vn / dn + std::exp(-.5 * dn * dn)));
        kn[i + 1] = (uint32_t)((dn / tn) * m1);
        tn = dn;
        fn[i] = (float)std::exp(-.5 * dn * dn);
        wn[i] = (float)(dn / m1);
      }
    }
  };
  static const Tables& tables() { static Tables t; return t; }

  // randn_0_1_32f for one value
  float gauss01() {
    const Tables& T = tables();
    const float r = 3.442620f;
    const float rng_flt = 2.3283064365386962890625e-10f;
    uint64_t temp = state;
    float x, y;
    for (;;) {
      int hz = (int)(uint32_t)temp;
      temp = step(temp);
      int iz = hz & 127;
      x = hz * T.wn[iz];
      if ((unsigned)std::abs(hz) < T.kn[iz]) break;
      if (iz == 0) {
        do {
          x = (unsigned)temp * rng_flt;
          temp = step(temp);
          y = (unsigned)temp * rng_flt;
          temp = step(temp);
          x = (float)(-std::log(x + FLT_MIN) * 0.2904764);
          y = (float)-std::log(y + FLT_MIN);
        } while (y + y < x * x);
        x = hz > 0 ? r + x : -r - x;
        break;
      }
      y = (unsigned)temp * rng_flt;
      temp = step(temp);
      if (T.fn[iz] + y * (T.fn[iz - 1] - T.fn[iz]) < std::exp(-.5 * x * x)) break;
    }
    state = temp;
    return x;
  }
  double gaussian(double sigma) { float t = gauss01(); return t * sigma; }
};

}  // namespace orc
