// ORACLE (test infrastructure only): CPU restatement of the mantis3 Markov
// yaw filter, include/mantis3/Markov.cpp (MarkovModel) and Markov.h
// (DEGREES = 360, markovPlane = std::array<double, 360>). Included but unused
// upstream; the library's HIP version is
// mantis_amd/csrc/markov_impl.hip. Quirks kept: convolve's `(int)dTheta*180/M_PI`
// truncates dTheta to whole radians first (Markov.cpp:230); getYaw returns
// p[argmax] * pi / 180, not the argmax angle (:265-275); updateHypothesis
// divides the error by p[bin] (`error * 1/(p)` = (error * 1) / p, :207-222).
// Defined (reference UB): senseFusion(Hypothesis)'s zero-fill loop never
// terminates (`for(int i=0; sense.size(); ++i)`, :190) -- here it fills the 360
// bins; a yaw of exactly 360 after wrapping maps to bin 0.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "o_tf.hpp"

namespace {
constexpr int kDeg = 360;

// MarkovModel::calculateWeight (Markov.cpp:29-32)
inline double weight(double x, double mu, double stddev, double y) {
  return (y / (stddev * std::sqrt(2 * M_PI))) * std::exp(-((x - mu) * (x - mu) / (2 * stddev * stddev)));
}

// MarkovModel::normalize(input, output) (:62-74)
void normalize_to(const double* in, double* out) {
  double sum = 0.0;
  for (int i = 0; i < kDeg; ++i) sum += in[i];
  for (int i = 0; i < kDeg; ++i) out[i] = in[i] / sum;
}

// MarkovModel::updateWeights (:76-124)
void update_weights(double* yaw, double stddev) {
  double aux[kDeg];
  for (int i = 0; i < kDeg; ++i) {
    double max = 0.0;
    const int diff = kDeg / 2 + i;
    if (i <= kDeg / 2) {
      for (int j = 0; j < diff; ++j) max += weight((double)i, (double)j, stddev, yaw[j]);
      for (int j = diff; j < kDeg; ++j) max += weight((double)i, (double)(-(kDeg - j)), stddev, yaw[j]);
    } else {
      for (int j = i; j < diff; ++j) max += weight((double)i, (double)j, stddev, yaw[j % kDeg]);
      for (int j = diff % kDeg; j < i; ++j) max += weight((double)i, (double)j, stddev, yaw[j]);
    }
    aux[i] = max;
  }
  normalize_to(aux, yaw);
}

// yaw bin of a hypothesis: getW2C().getBasis().getRPY, degrees, wrapped (:15-27, :185-196)
int yaw_bin(const double* R) {
  orc::Mat3 m(R[0], R[1], R[2], R[3], R[4], R[5], R[6], R[7], R[8]);
  double roll, pitch, yaw;
  m.getRPY(roll, pitch, yaw);
  yaw *= 180.0 / M_PI;
  if (yaw < 0) yaw += kDeg;
  const int b = (int)yaw;
  return b >= kDeg ? b - kDeg : b;
}
}  // namespace

extern "C" {

// MarkovModel(Hypothesis) (:15-27): one-hot at the yaw bin, updateWeights(p, 3)
void orc_markov_init(const double* R, double* p) {
  for (int i = 0; i < kDeg; ++i) p[i] = 0.0;
  p[yaw_bin(R)] = 1;
  update_weights(p, 3);
}

// senseFusion(Hypothesis) (:185-201) -> senseFusion(markovPlane) (:164-183)
void orc_markov_sense(double* p, const double* R) {
  double sense[kDeg];
  for (int i = 0; i < kDeg; ++i) sense[i] = 0.0;
  sense[yaw_bin(R)] = 1;
  update_weights(sense, 3.5);
  const double newMax = std::sqrt(DBL_MAX);
  for (int i = 0; i < kDeg; ++i) {
    p[i] = p[i] * newMax;
    sense[i] = sense[i] * newMax;
  }
  for (int i = 0; i < kDeg; ++i) p[i] *= sense[i];
  normalize_to(p, p);
}

// convolve(dTheta, dt) (:227-258)
void orc_markov_convolve(double* p, double dTheta, double dt) {
  double aux[kDeg];
  int convDisplacement = (int)dTheta * 180 / M_PI;
  if (dTheta > 0) {
    for (int i = convDisplacement; i < kDeg + convDisplacement; ++i) aux[i % kDeg] = p[i - convDisplacement];
  } else {
    convDisplacement *= -1;
    for (int i = 0; i < kDeg; ++i) aux[i] = p[(convDisplacement + i) % kDeg];
  }
  std::memcpy(p, aux, sizeof(aux));
  update_weights(p, 1.0 / 3.0 * dt * 11.5 / 30.0);
}

// updateHypothesis (:207-222)
void orc_markov_weight(const double* p, const double* R, int32_t n, double* error) {
  for (int i = 0; i < n; i++) error[i] = error[i] * 1 / (p[yaw_bin(R + 9 * i)]);
}

// getYaw (:265-275): p[argmax] * pi / 180 (quirk), first maximum
double orc_markov_yaw(const double* p, int32_t* argmax) {
  int max = 0;
  for (int i = 0; i < kDeg; ++i)
    if (p[i] > p[max]) max = i;
  if (argmax) *argmax = max;
  return p[max] * M_PI / 180;
}

int32_t orc_markov_bin(const double* R) { return yaw_bin(R); }

}  // extern "C"
