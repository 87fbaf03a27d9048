// FP64 operation count of the RPP ObjPose iteration (test/measurement tool):
// the device-logic header mk_rpp.h compiled for the host with `double`
// replaced by a counting scalar. Every +, -, *, /, sqrt, hypot, trig and pow
// on an FP64 value counts one flop (comparisons, fabs and copies count none),
// so the figure is the arithmetic the reference's ObjPose performs per
// AbsKernel call (RPP.cpp:229-332, OpenCV's one-sided Jacobi included).
// Problems: synthetic 4-corner squares seen from random poses with pixel-level
// noise, both gridSquarePossibilities orientations. Prints JSON.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

static long long g_ops = 0;
struct CD {
  double v;
  constexpr CD() : v(0) {}
  constexpr CD(double x) : v(x) {}
  constexpr CD(int x) : v(x) {}
  constexpr CD(long double x) : v((double)x) {}
  explicit operator double() const { return v; }
  explicit operator int() const { return (int)v; }
  CD operator-() const { return CD(-v); }
  CD& operator+=(CD o) { ++g_ops; v += o.v; return *this; }
  CD& operator-=(CD o) { ++g_ops; v -= o.v; return *this; }
  CD& operator*=(CD o) { ++g_ops; v *= o.v; return *this; }
  CD& operator/=(CD o) { ++g_ops; v /= o.v; return *this; }
};
inline CD operator+(CD a, CD b) { ++g_ops; return CD(a.v + b.v); }
inline CD operator-(CD a, CD b) { ++g_ops; return CD(a.v - b.v); }
inline CD operator*(CD a, CD b) { ++g_ops; return CD(a.v * b.v); }
inline CD operator/(CD a, CD b) { ++g_ops; return CD(a.v / b.v); }
inline bool operator<(CD a, CD b) { return a.v < b.v; }
inline bool operator>(CD a, CD b) { return a.v > b.v; }
inline bool operator<=(CD a, CD b) { return a.v <= b.v; }
inline bool operator>=(CD a, CD b) { return a.v >= b.v; }
inline bool operator==(CD a, CD b) { return a.v == b.v; }
inline bool operator!=(CD a, CD b) { return a.v != b.v; }
inline CD fabs(CD a) { return CD(std::fabs(a.v)); }
inline CD fmax(CD a, CD b) { return CD(std::fmax(a.v, b.v)); }
inline CD fmin(CD a, CD b) { return CD(std::fmin(a.v, b.v)); }
inline CD sqrt(CD a) { ++g_ops; return CD(std::sqrt(a.v)); }
inline CD hypot(CD a, CD b) { ++g_ops; return CD(std::hypot(a.v, b.v)); }
inline CD atan2(CD a, CD b) { ++g_ops; return CD(std::atan2(a.v, b.v)); }
inline CD acos(CD a) { ++g_ops; return CD(std::acos(a.v)); }
inline CD sin(CD a) { ++g_ops; return CD(std::sin(a.v)); }
inline CD cos(CD a) { ++g_ops; return CD(std::cos(a.v)); }
inline CD pow(CD a, CD b) { ++g_ops; return CD(std::pow(a.v, b.v)); }
inline CD ldexp(CD a, int e) { return CD(std::ldexp(a.v, e)); }
inline CD log(CD a) { ++g_ops; return CD(std::log(a.v)); }
inline CD exp(CD a) { ++g_ops; return CD(std::exp(a.v)); }

#include "../mantis_amd/csrc/mk_math.h"
#define double CD
#include "../mantis_amd/csrc/mk_rpp.h"
#undef double

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4000;
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> U(0, 1);
  std::normal_distribution<double> N(0, 1);
  const double s = 0.16;
  const double m0[12] = {s, -s, -s, s, s, s, -s, -s, 0, 0, 0, 0};
  const double m1[12] = {s, -s, -s, s, -s, -s, s, s, 0, 0, 0, 0};
  long long it_total = 0, ops_loop = 0, ops_total = 0, problems = 0;
  for (int k = 0; k < n; k++) {
    // camera looking down from 0.8-3 m, yaw random, tilt ~N(0, 0.3)
    double yaw = U(rng) * 6.283, tilt = N(rng) * 0.3, h = 0.8 + 2.2 * U(rng);
    double cy = std::cos(yaw), sy = std::sin(yaw), ct = std::cos(tilt), st = std::sin(tilt);
    double Rz[9] = {cy, -sy, 0, sy, cy, 0, 0, 0, 1}, Rx[9] = {1, 0, 0, 0, ct, -st, 0, st, ct};
    double Rn[9] = {1, 0, 0, 0, -1, 0, 0, 0, -1};  // nadir
    double A[9], R[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        A[i * 3 + j] = 0;
        for (int q = 0; q < 3; q++) A[i * 3 + j] += Rz[i * 3 + q] * Rn[q * 3 + j];
      }
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        R[i * 3 + j] = 0;
        for (int q = 0; q < 3; q++) R[i * 3 + j] += A[i * 3 + q] * Rx[q * 3 + j];
      }
    double t[3] = {N(rng) * 0.3, N(rng) * 0.3, h};
    for (int o = 0; o < 2; o++) {
      const double* m = o ? m1 : m0;
      CD model[12], ip[12];
      for (int c = 0; c < 4; c++) {
        double X[3] = {m[c], m[4 + c], m[8 + c]}, Q[3];
        for (int r = 0; r < 3; r++) Q[r] = R[0 * 3 + r] * X[0] + R[1 * 3 + r] * X[1] + R[2 * 3 + r] * X[2] + t[r];
        for (int r = 0; r < 3; r++) model[r * 4 + c] = CD(m[r * 4 + c]);
        ip[c] = CD(Q[0] / Q[2] + N(rng) * 0.003);
        ip[4 + c] = CD(Q[1] / Q[2] + N(rng) * 0.003);
        ip[8 + c] = CD(1.0);
      }
      // count the ObjPose loop separately: one AbsKernel per op_step
      mk::rpp::M34 P, Qp;
      for (int q = 0; q < 12; q++) { P.a[q] = model[q]; Qp.a[q] = ip[q]; }
      mk::rpp::OpState st;
      mk::rpp::op_setup(P, Qp, nullptr, st);
      long long before = g_ops;
      while (mk::rpp::op_step(st) == 0) {
      }
      ops_loop += g_ops - before;
      it_total += st.it;
      long long b2 = g_ops;
      mk::rpp::solve(model, ip);
      ops_total += g_ops - b2;
      problems++;
    }
  }
  std::printf("{\"problems\": %lld, \"first_objpose_iterations\": %lld, \"flops_per_iteration\": %.1f, "
              "\"flops_per_problem\": %.1f}\n",
              problems, it_total, (double)ops_loop / it_total, (double)ops_total / problems);
  return 0;
}
