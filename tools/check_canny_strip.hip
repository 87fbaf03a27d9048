// GPU check of k_canny_strip against k_canny (measurement tool): both on
// the same frames (blob noise, gradients, random bytes; several sizes with
// W % 4 == 0), candidate and strong bit planes compared word for word; the
// first mismatching pixels are printed with both bits.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize tools/check_canny_strip.hip -o tools/check_canny_strip
#include "../mantis_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

using namespace mk;

// time mode: N copies of one 1280x720 noise frame, both kernels timed with
// HIP events (best of 5); for rocprofv3 --pmc passes on the kernels alone.
static int time_mode(int N) {
  const int W = 1280, H = 720;
  const size_t fb = (size_t)W * H * 3;
  std::vector<uint8_t> img(fb);
  std::mt19937 rng(9);
  for (size_t i = 0; i < fb; i++) img[i] = (uint8_t)((((i / 3) % W) / 6 + (i / 3 / W) / 6) & 1 ? 200 + (rng() & 31) : 30 + (rng() & 31));
  uint8_t* dimg;
  hipMalloc(&dimg, fb * N);
  for (int f = 0; f < N; f++) hipMemcpy(dimg + fb * f, img.data(), fb, hipMemcpyHostToDevice);
  std::vector<FrameDesc> fd(N);
  for (int f = 0; f < N; f++) { fd[f] = FrameDesc{}; fd[f].bgr = dimg + fb * f; fd[f].w = W; fd[f].h = H; }
  FrameDesc* dfd;
  hipMalloc(&dfd, sizeof(FrameDesc) * N);
  hipMemcpy(dfd, fd.data(), sizeof(FrameDesc) * N, hipMemcpyHostToDevice);
  const size_t B = (size_t)bits::words(W) * H;
  uint32_t *c, *s;
  hipMalloc(&c, B * 4 * N);
  hipMalloc(&s, B * 4 * N);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int tgx = (W + FTW - 1) / FTW, tgy = (H + FTH - 1) / FTH;
  const int ns1 = (W + StripGeom<1>::cols - 1) / StripGeom<1>::cols, ns2 = (W + StripGeom<2>::cols - 1) / StripGeom<2>::cols;
  for (int kind = 0; kind < 3; kind++) {
    float best = 1e9f;
    for (int r = 0; r < 5; r++) {
      hipEventRecord(e0);
      if (kind == 0) k_canny<<<tgx * tgy * N, 256>>>(dfd, 30, 90, 1, c, s, B, tgx, tgy);
      else if (kind == 1) k_canny_strip<1><<<(ns1 * N + 3) / 4, 256>>>(dfd, 30, 90, c, s, B, ns1, ns1 * N);
      else k_canny_strip<2><<<(ns2 * N + 3) / 4, 256>>>(dfd, 30, 90, c, s, B, ns2, ns2 * N);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      best = ms < best ? ms : best;
    }
    printf("%s: %d frames %.3f ms (%.3f ms per 4096 frames)\n", kind == 2 ? "k_canny_strip<2>" : kind ? "k_canny_strip<1>" : "k_canny", N, best, best * 4096.0 / N);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 2 && std::string(argv[1]) == "time") return time_mode(std::atoi(argv[2]));
  const int sizes[][2] = {{1280, 720}, {640, 480}, {1000, 611}, {232, 40}, {8, 3}, {448, 17}, {1284, 33}, {16, 3}, {24, 5}, {488, 9}};
  int fails = 0;
  std::mt19937 rng(5);
  for (auto& sz : sizes) {
    const int W = sz[0], H = sz[1];
    for (int kind = 0; kind < 3; kind++) {
      std::vector<uint8_t> img((size_t)W * H * 3);
      for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++)
          for (int c = 0; c < 3; c++) {
            uint8_t v;
            if (kind == 0) v = (((x / 7) + (y / 5)) & 1) ? 210 : 25;
            else if (kind == 1) v = (uint8_t)((x * 3 + y * 5 + c * 40) & 255);
            else v = (uint8_t)(rng() & 255);
            img[((size_t)y * W + x) * 3 + c] = v;
          }
      uint8_t* dimg;
      hipMalloc(&dimg, img.size());
      hipMemcpy(dimg, img.data(), img.size(), hipMemcpyHostToDevice);
      FrameDesc fd{};
      fd.bgr = dimg;
      fd.w = W;
      fd.h = H;
      FrameDesc* dfd;
      hipMalloc(&dfd, sizeof(FrameDesc));
      hipMemcpy(dfd, &fd, sizeof(fd), hipMemcpyHostToDevice);
      const int WW = bits::words(W);
      const size_t B = (size_t)WW * H;
      uint32_t *c1, *s1, *c2, *s2;
      hipMalloc(&c1, B * 4); hipMalloc(&s1, B * 4); hipMalloc(&c2, B * 4); hipMalloc(&s2, B * 4);
      hipMemset(c1, 0, B * 4); hipMemset(s1, 0, B * 4);
      const int low = 30, high = 90;
      const int tgx = (W + FTW - 1) / FTW, tgy = (H + FTH - 1) / FTH;
      k_canny<<<tgx * tgy, 256>>>(dfd, low, high, 1, c1, s1, B, tgx, tgy);
      std::vector<uint32_t> h1(B), h2(B), g1(B), g2(B);
      hipMemcpy(h1.data(), c1, B * 4, hipMemcpyDeviceToHost);
      hipMemcpy(g1.data(), s1, B * 4, hipMemcpyDeviceToHost);
      for (int K = 1; K <= 2; K++) {
        if (K == 2 && (W % 8 != 0 || W < 16)) continue;
        hipMemset(c2, 0xff, B * 4); hipMemset(s2, 0xff, B * 4);
        if (K == 1) {
          const int ns = (W + StripGeom<1>::cols - 1) / StripGeom<1>::cols;
          k_canny_strip<1><<<(ns + 3) / 4, 256>>>(dfd, low, high, c2, s2, B, ns, ns);
        } else {
          const int ns = (W + StripGeom<2>::cols - 1) / StripGeom<2>::cols;
          k_canny_strip<2><<<(ns + 3) / 4, 256>>>(dfd, low, high, c2, s2, B, ns, ns);
        }
        hipMemcpy(h2.data(), c2, B * 4, hipMemcpyDeviceToHost);
        hipMemcpy(g2.data(), s2, B * 4, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int y = 0; y < H; y++)
          for (int x = 0; x < W; x++) {
            const size_t w = (size_t)y * WW + (x >> 5);
            const int b = x & 31;
            const int a1 = (h1[w] >> b) & 1, a2 = (h2[w] >> b) & 1, t1 = (g1[w] >> b) & 1, t2 = (g2[w] >> b) & 1;
            if (a1 != a2 || t1 != t2) {
              if (bad < 8) printf("  %dx%d kind %d K %d: (%d, %d) cand %d/%d strong %d/%d\n", W, H, kind, K, x, y, a1, a2, t1, t2);
              bad++;
            }
          }
        printf("%dx%d kind %d K %d: %d pixel mismatches\n", W, H, kind, K, bad);
        fails += bad != 0;
      }
      hipFree(dimg); hipFree(dfd); hipFree(c1); hipFree(s1); hipFree(c2); hipFree(s2);
    }
  }
  printf("check_canny_strip: %s\n", fails ? "FAIL" : "ok");
  return fails ? 1 : 0;
}
