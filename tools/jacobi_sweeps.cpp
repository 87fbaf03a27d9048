// Jacobi sweep counts of the AbsKernel SVD (measurement tool): the host build
// of mk_rpp.h with hooks that record, for every svd3 call inside an ObjPose
// iteration (abs_kernel, between MK_OP_STAMP(1) and (2)), how many sweeps ran
// and whether the noise fast-forward ended them. A wave of 64 lanes runs the
// sweep loop as long as its slowest lane, so the distribution's tail sets the
// per-wave cost of k_objpose_q. Input: problems from tools/jacobi_sweeps.py
// (model 3x4, image points 3x4 row-major float64 each). Prints JSON.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

static int g_in_svd = 0, g_sweeps = 0, g_ff = 0;
static std::vector<int> g_calls;  // sweeps per svd3 call, ff-ended calls negative
#define MK_OP_STAMP(k)                                  \
  do {                                                  \
    if ((k) == 1) { g_in_svd = 1; g_sweeps = 0; g_ff = 0; } \
    if ((k) == 2) { g_in_svd = 0; g_calls.push_back(g_ff ? -g_sweeps : g_sweeps); } \
  } while (0)
#define MK_JACOBI_COUNT(M, N, iter, changed) \
  do {                                       \
    if (g_in_svd && (M) == 3 && (N) == 3) g_sweeps = (iter) + 1; \
  } while (0)
#include "../mantis_amd/csrc/mk_math.h"
#include "../mantis_amd/csrc/mk_rpp.h"

int main(int argc, char** argv) {
  if (argc < 2) { std::fprintf(stderr, "usage: jacobi_sweeps problems.bin\n"); return 1; }
  FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 1;
  std::vector<double> buf;
  double tmp[24];
  while (std::fread(tmp, sizeof(double), 24, f) == 24) buf.insert(buf.end(), tmp, tmp + 24);
  std::fclose(f);
  const size_t n = buf.size() / 24;
  std::vector<int> first, cand;
  for (size_t i = 0; i < n; i++) {
    const double* model = &buf[24 * i];
    const double* ip = model + 12;
    g_calls.clear();
    mk::rpp::Stage1 s;
    mk::rpp::stage1(model, ip, s);
    first.insert(first.end(), g_calls.begin(), g_calls.end());
    if (s.error == 1) continue;
    for (int j = 0; j < mk::rpp::kCand; j++) {
      if (!((s.keep_mask >> j) & 1)) continue;
      g_calls.clear();
      mk::rpp::Refine r;
      mk::rpp::refine(model, s.Q, s.sR[j], r);
      cand.insert(cand.end(), g_calls.begin(), g_calls.end());
    }
  }
  // histogram and the expected wave maximum over 64 random calls
  std::mt19937_64 rng(7);
  std::printf("{");
  const char* names[2] = {"first", "cand"};
  std::vector<int>* sets[2] = {&first, &cand};
  for (int k = 0; k < 2; k++) {
    std::vector<int>& v = *sets[k];
    long hist[32] = {0}, ffc = 0;
    double mean = 0;
    for (int x : v) {
      int a = x < 0 ? -x : x;
      if (x < 0) ffc++;
      hist[a < 31 ? a : 31]++;
      mean += a;
    }
    mean /= v.empty() ? 1 : v.size();
    double wmax = 0;
    const int T = 20000;
    for (int t = 0; t < T && !v.empty(); t++) {
      int m = 0;
      for (int l = 0; l < 64; l++) {
        int x = v[rng() % v.size()];
        m = std::max(m, x < 0 ? -x : x);
      }
      wmax += m;
    }
    std::printf("%s\"%s\": {\"calls\": %zu, \"ff_ended\": %ld, \"mean_sweeps\": %.3f, \"wave64_max_sweeps\": %.3f, \"hist\": [",
                k ? ", " : "", names[k], v.size(), ffc, mean, wmax / T);
    for (int i = 0; i < 32; i++) std::printf("%s%ld", i ? ", " : "", hist[i]);
    std::printf("]}");
  }
  std::printf("}\n");
  return 0;
}
