// GPU check of the filtered projection (mk_math.h distort_fast) against the
// exact distort(): max |du|, |dv| over random camera-frame points, and that
// every certified point makes the exact decisions (in_frame, cvRound).
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/check_proj.hip -o tools/check_proj
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../mantis_amd/csrc/mk_math.h"

__device__ inline uint64_t mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ inline double unif(uint64_t i, int k) { return (double)(mix(i * 4 + k) >> 11) * (1.0 / 9007199254740992.0); }

__global__ void kcheck(uint64_t n, mk::Cam cm, int W, int H, unsigned long long* cnt, double* maxd) {
  double md = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    // points in front of / beside the camera, as landmarks 0.5..6 m away at any angle
    const double X = (unif(i, 0) * 2 - 1) * 6, Y = (unif(i, 1) * 2 - 1) * 6;
    double Z = (unif(i, 2) * 2 - 0.2) * 4;
    if ((i & 1023) == 0) Z = (unif(i, 3) - 0.5) * 1e-9;  // near the image plane
    double ue, ve, uf, vf;
    mk::distort(cm, X, Y, Z, &ue, &ve);
    const bool sure = mk::distort_fast(cm, X, Y, Z, &uf, &vf, W, H);
    if (!sure) { atomicAdd(&cnt[1], 1ull); continue; }
    atomicAdd(&cnt[0], 1ull);
    if (fabs(ue) < 1e4 && fabs(ve) < 1e4) md = fmax(md, fmax(fabs(ue - uf), fabs(ve - vf)));
    const bool in_e = mk::in_frame(ue, ve, H, W), in_f = mk::in_frame(uf, vf, H, W);
    if (in_e != in_f || (in_e && (mk::cv_round(ue) != mk::cv_round(uf) || mk::cv_round(ve) != mk::cv_round(vf))))
      atomicAdd(&cnt[2], 1ull);
  }
  for (int o = 32; o > 0; o >>= 1) md = fmax(md, __shfl_xor(md, o));
  if ((threadIdx.x & 63) == 0) atomicMax((unsigned long long*)maxd, (unsigned long long)__double_as_longlong(md));
}
int main() {
  mk::Cam cm;
  cm.fx = (double)(float)323.1511535644531; cm.fy = (double)(float)322.78955078125;
  cm.cx = (double)(float)642.658203125; cm.cy = (double)(float)349.5538330078125;
  const double k[4] = {0.0029509200248867273, -0.009944040328264236, 0.005587350111454725, -0.00205406011082232};
  for (int i = 0; i < 4; i++) cm.k[i] = k[i];
  unsigned long long* c;
  double* md;
  if (hipMalloc(&c, 24) || hipMalloc(&md, 8)) return 2;
  (void)hipMemset(c, 0, 24);
  (void)hipMemset(md, 0, 8);
  const uint64_t n = 1ull << 26;
  kcheck<<<4096, 256>>>(n, cm, 1280, 720, c, md);
  unsigned long long h[3];
  double m;
  if (hipMemcpy(h, c, 24, hipMemcpyDeviceToHost) || hipMemcpy(&m, md, 8, hipMemcpyDeviceToHost)) return 2;
  printf("check_proj: %llu points, certified %llu, fallback %llu, decision mismatches %llu, max |d| %.3e px\n",
         (unsigned long long)n, h[0], h[1], h[2], m);
  return h[2] ? 1 : 0;
}
