// Host-side rate of the cv::RNG gaussian stream (api.hip's rng_gauss): one
// batch of the default bench (4096 frames x 50 particles x 10 iterations x 6)
// drawn on one thread, as gen_gauss does per context while the device runs
// the image stages and RPP. Build: hipcc -O3 tools/gauss_rate.hip -o tools/gauss_rate -lrccl
#include "../mantis_amd/csrc/api.hip"
int main() {
  const size_t n = 4096ull * 50 * 10 * 6;
  std::vector<float> g(n);
  uint64_t s = 1;
  const auto t0 = std::chrono::steady_clock::now();
  for (size_t k = 0; k < n; k++) g[k] = rng_gauss(s);
  const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  double acc = 0;
  for (size_t k = 0; k < n; k += 4096) acc += g[k];
  printf("gauss_rate: %zu draws in %.1f ms (%.2f ns each), checksum %.6f\n", n, ms, 1e6 * ms / n, acc);
}
