// GPU validation of the FP32 projection screen (mantis_amd/csrc/mk_screen.h)
// against the exact FP64 projection the scorers use (mk_math.h xf_apply +
// distort + in_frame + cv_round, device libm restated in mk_dmath.h): every
// decision the screen takes (SCR_IN with its pixel, SCR_OUT) must equal the
// exact one. Reports the unsure rate and the largest |u_f32 - u_exact| / eps.
// Pose / landmark distributions:
//   0 scene: camera 0.9..2.1 m above the grid plane, optical axis within 45 deg
//     of nadir, landmarks from the map (params/map.yaml) or the floor square
//   1 any: uniform random rotation, camera and landmarks in a 6 m box
//   2 near: landmarks 2..60 cm from the camera, any direction
// and three cameras: the 720p and 1080p rig intrinsics, random K/D per trial.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/check_screen.hip -o tools/check_screen
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../mantis_amd/csrc/mk_screen.h"

__device__ inline uint64_t mix(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__device__ inline double unif(uint64_t i, int k) { return (double)(mix(i * 16 + k) >> 11) * (1.0 / 9007199254740992.0); }
__device__ inline double gaus(uint64_t i, int k) {
  const double a = fmax(unif(i, k), 1e-300), b = unif(i, k + 1);
  return sqrt(-2 * log(a)) * cos(6.283185307179586 * b);
}

struct Out {
  unsigned long long n, in_exact, sure_in, sure_out, unsure, bad, unsure_in;
  unsigned long long maxratio_bits;  // max |u_f - u_e| / eps as double bits
};

// rotation from a unit quaternion
__device__ void quat_rot(double a, double b, double c, double d, double* R) {
  const double n = sqrt(a * a + b * b + c * c + d * d);
  a /= n; b /= n; c /= n; d /= n;
  R[0] = a * a + b * b - c * c - d * d; R[1] = 2 * (b * c - a * d); R[2] = 2 * (b * d + a * c);
  R[3] = 2 * (b * c + a * d); R[4] = a * a - b * b + c * c - d * d; R[5] = 2 * (c * d - a * b);
  R[6] = 2 * (b * d - a * c); R[7] = 2 * (c * d + a * b); R[8] = a * a - b * b - c * c + d * d;
}

__global__ void kcheck(uint64_t n, uint64_t seed, int mode, int camk, const double* map, int nmap, Out* out) {
  double mr = 0;
  unsigned long long cnt[7] = {0, 0, 0, 0, 0, 0, 0};
  // camera: fixed per thread (random intrinsics per thread for camk 2)
  const uint64_t tid = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 0x9e3779b97f4a7c15ull + seed;
  // camera
  mk::Cam cm;
  int W = 1280, H = 720;
  if (camk == 0 || camk == 1) {
    const double s = camk == 1 ? 1.5 : 1.0;
    W = camk == 1 ? 1920 : 1280;
    H = camk == 1 ? 1080 : 720;
    cm.fx = (double)(float)(323.1511535644531 * s); cm.fy = (double)(float)(322.78955078125 * s);
    cm.cx = (double)(float)(642.658203125 * s); cm.cy = (double)(float)(349.5538330078125 * s);
    cm.k[0] = 0.0029509200248867273; cm.k[1] = -0.009944040328264236;
    cm.k[2] = 0.005587350111454725; cm.k[3] = -0.00205406011082232;
  } else {
    W = 320 + (int)(unif(tid, 0) * 1800);
    H = 240 + (int)(unif(tid, 1) * 1000);
    cm.fx = (double)(float)(150 + unif(tid, 2) * 800);
    cm.fy = (double)(float)(cm.fx * (0.9 + 0.2 * unif(tid, 3)));
    cm.cx = (double)(float)(W * (0.3 + 0.4 * unif(tid, 4)));
    cm.cy = (double)(float)(H * (0.3 + 0.4 * unif(tid, 5)));
    for (int k = 0; k < 4; k++) cm.k[k] = (unif(tid, 6 + k) * 2 - 1) * 0.02;
  }
  const mk::ScreenCam sc = mk::screen_cam_from(cm);
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t id = i * 0x100000001b3ull + seed;
    // pose (c2w: world -> camera) and landmark
    double R[9], C[3], X[3];
    if (mode == 0) {
      // nadir-looking camera tilted up to 45 deg, any yaw
      const double yaw = unif(id, 10) * 6.283185307179586, tilt = unif(id, 11) * 0.785, tdir = unif(id, 12) * 6.2832;
      double Rw[9];  // camera-to-world: z axis = viewing direction
      const double vx = sin(tilt) * cos(tdir), vy = sin(tilt) * sin(tdir), vz = -cos(tilt);
      // build an orthonormal frame around v with a yaw about v
      double ax[3] = {cos(yaw), sin(yaw), 0};
      double d = ax[0] * vx + ax[1] * vy + ax[2] * vz;
      ax[0] -= d * vx; ax[1] -= d * vy; ax[2] -= d * vz;
      double nn = sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
      ax[0] /= nn; ax[1] /= nn; ax[2] /= nn;
      const double ay[3] = {vy * ax[2] - vz * ax[1], vz * ax[0] - vx * ax[2], vx * ax[1] - vy * ax[0]};
      Rw[0] = ax[0]; Rw[1] = ay[0]; Rw[2] = vx;
      Rw[3] = ax[1]; Rw[4] = ay[1]; Rw[5] = vy;
      Rw[6] = ax[2]; Rw[7] = ay[2]; Rw[8] = vz;
      for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) R[r * 3 + c] = Rw[c * 3 + r];
      C[0] = (unif(id, 13) * 2 - 1) * 0.9; C[1] = (unif(id, 14) * 2 - 1) * 0.9; C[2] = 0.9 + 1.2 * unif(id, 15);
      if ((i & 3) != 3 && nmap > 0) {
        const int l = (int)(unif(id, 16) * nmap) % nmap;
        X[0] = map[3 * l]; X[1] = map[3 * l + 1]; X[2] = map[3 * l + 2];
      } else {
        X[0] = (unif(id, 17) * 2 - 1) * 1.6; X[1] = (unif(id, 18) * 2 - 1) * 1.6; X[2] = 0;
      }
    } else {
      quat_rot(gaus(id, 10), gaus(id, 12), unif(id, 14) * 2 - 1, unif(id, 15) * 2 - 1, R);
      for (int k = 0; k < 3; k++) C[k] = (unif(id, 16 + k) * 2 - 1) * 3;
      if (mode == 1) {
        for (int k = 0; k < 3; k++) X[k] = (unif(id, 20 + k) * 2 - 1) * 3;
      } else {
        const double rr = 0.02 + 0.58 * unif(id, 20);
        double dv[3] = {gaus(id, 21), gaus(id, 23), unif(id, 25) * 2 - 1};
        const double nd = sqrt(dv[0] * dv[0] + dv[1] * dv[1] + dv[2] * dv[2]);
        for (int k = 0; k < 3; k++) X[k] = C[k] + rr * dv[k] / nd;
      }
    }
    mk::Xf T;
    for (int k = 0; k < 9; k++) T.R[k] = R[k];
    for (int r = 0; r < 3; r++) T.t[r] = -(R[3 * r] * C[0] + R[3 * r + 1] * C[1] + R[3 * r + 2] * C[2]);
    // exact
    double rp[3], ue, ve;
    mk::xf_apply(T, X, rp);
    mk::distort(cm, rp[0], rp[1], rp[2], &ue, &ve);
    const bool in_e = rp[2] > 0 && mk::in_frame(ue, ve, H, W);
    cnt[0]++;
    cnt[1] += in_e;
    // screen
    const mk::PoseF P = mk::posef_from(T);
    float xl[4];
    mk::screen_landmark(X, xl);
    int px = 0, py = 0;
    const int s = mk::screen_project(P, xl[0], xl[1], xl[2], xl[3], sc, W, H, &px, &py);
    if (s == mk::SCR_IN) {
      cnt[2]++;
      if (!in_e || px != mk::cv_round(ue) || py != mk::cv_round(ve)) cnt[5]++;
    } else if (s == mk::SCR_OUT) {
      cnt[3]++;
      if (in_e) cnt[5]++;
    } else {
      cnt[4]++;
      cnt[6] += in_e;
    }
    const mk::ScrUV r = mk::screen_uv(P, xl[0], xl[1], xl[2], xl[3], sc);
    if (r.state == 1 && rp[2] > 0 && fabs(ue) < 1e5 && fabs(ve) < 1e5 && r.eps > 0)
      mr = fmax(mr, fmax(fabs((double)r.u - ue), fabs((double)r.v - ve)) / (double)r.eps);
  }
  for (int k = 0; k < 7; k++) {
    unsigned long long v = cnt[k];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    cnt[k] = v;
  }
  for (int o = 32; o > 0; o >>= 1) mr = fmax(mr, __shfl_xor(mr, o));
  if ((threadIdx.x & 63) == 0) {
    unsigned long long* o = &out->n;
    for (int k = 0; k < 7; k++) atomicAdd(o + k, cnt[k]);
    atomicMax(&out->maxratio_bits, (unsigned long long)__double_as_longlong(mr));
  }
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 0) : (1ull << 28);
  std::vector<double> map;
  if (argc > 2) {  // landmarks as text triples
    FILE* f = fopen(argv[2], "r");
    double a, b, c;
    while (f && fscanf(f, "%lf %lf %lf", &a, &b, &c) == 3) { map.push_back(a); map.push_back(b); map.push_back(c); }
    if (f) fclose(f);
  }
  double* dmap = nullptr;
  Out* d;
  if (hipMalloc(&d, sizeof(Out))) return 2;
  if (!map.empty() && (hipMalloc(&dmap, map.size() * 8) || hipMemcpy(dmap, map.data(), map.size() * 8, hipMemcpyHostToDevice)))
    return 2;
  int fails = 0;
  for (int mode = 0; mode < 3; mode++)
    for (int camk = 0; camk < 3; camk++) {
      (void)hipMemset(d, 0, sizeof(Out));
      kcheck<<<8192, 256>>>(n, 0x5eed0000ull + 131 * mode + camk, mode, camk, dmap, (int)map.size() / 3, d);
      Out h;
      if (hipMemcpy(&h, d, sizeof(Out), hipMemcpyDeviceToHost)) return 2;
      double mr;
      memcpy(&mr, &h.maxratio_bits, 8);
      printf("check_screen mode %d cam %d: %llu projections, exact in-frame %llu; screen in %llu out %llu unsure %llu "
             "(%.3f %% of all, %.3f %% of in-frame); decision mismatches %llu; max |d|/eps %.4f\n",
             mode, camk, h.n, h.in_exact, h.sure_in, h.sure_out, h.unsure, 100.0 * h.unsure / h.n,
             100.0 * h.unsure_in / (h.in_exact ? h.in_exact : 1), h.bad, mr);
      fflush(stdout);
      fails += h.bad != 0 || mr >= 1.0;
    }
  printf("check_screen: %s\n", fails ? "FAIL" : "ok");
  return fails ? 1 : 0;
}
