// Host build of the device-logic headers (mk_*.h) for CPU unit tests only:
// lets tests/ check the per-work-item algorithms (RPP, Jenkins–Traub, the
// libstdc++ sort port, border following + approxPolyDP, and the parallel
// contour formulation) against the oracle without a GPU. The product path is
// the HIP build in libmantis_amd.so; nothing here is loaded by it.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

// runtime switch for the Jacobi noise-phase fast-forward (mk_rpp.h), so the
// tests can compare it bit for bit against the full sweep sequence
static int g_jacobi_ff = 1;
#define MK_JACOBI_FF g_jacobi_ff
#include "mk_bits.h"
#include "mk_contour.h"
#include "mk_gn.h"
#include "mk_math.h"
#include "mk_rpp.h"
#include "mk_screen.h"
#include "mk_shard.h"
#include "mk_sort.h"

extern "C" {

void hc_set_jacobi_ff(int on) { g_jacobi_ff = on; }

int hc_rpp(const double* model, const double* iprts, double* R, double* t, double* errs, int* err_code) {
  mk::rpp::Result r = mk::rpp::solve(model, iprts);
  std::memcpy(R, r.R, sizeof(r.R));
  std::memcpy(t, r.t, sizeof(r.t));
  errs[0] = r.obj_err;
  errs[1] = r.img_err;
  errs[2] = r.iterations;
  *err_code = r.error;
  return r.status;
}

// RPP::Rpp on n points (4..12) through the per-count instances mantis_rpp_solve runs
int hc_rpp_n(const double* model, const double* iprts, int n, double* R, double* t, double* errs, int* err_code) {
  mk::rpp::Result r;
  switch (n) {
    case 4: r = mk::rpp::solve(model, iprts); break;
#define MK_HC_RPP(k) \
    case k: r = mk::rpp::n##k::solve(model, iprts); break;
    MK_RPP_INSTANCES(MK_HC_RPP)
#undef MK_HC_RPP
    default: return -100;
  }
  std::memcpy(R, r.R, sizeof(r.R));
  std::memcpy(t, r.t, sizeof(r.t));
  errs[0] = r.obj_err;
  errs[1] = r.img_err;
  errs[2] = r.iterations;
  *err_code = r.error;
  return r.status;
}

// first ObjPose (stage1a): R[9], t[3], obj_err, img_err, iterations, Q after (12)
void hc_first_objpose(const double* model, const double* iprts, double* R, double* t, double* errs, int32_t* it,
                      double* Qout) {
  mk::rpp::Stage1 s;
  mk::rpp::stage1a(model, iprts, s);
  std::memcpy(R, s.R, sizeof(s.R));
  std::memcpy(t, s.t, sizeof(s.t));
  errs[0] = s.obj_err;
  errs[1] = s.img_err;
  *it = s.iterations;
  std::memcpy(Qout, s.Q, sizeof(s.Q));
}

// stage1 (first ObjPose + Get2ndPose setup): candidate initial rotations sR (kCand x 9), keep mask, error;
// refine each kept candidate: R (kCand x 9), t (kCand x 3), errs (kCand x 2), iterations (kCand)
int hc_stage1_cands(const double* model, const double* iprts, double* sR, double* R, double* t, double* errs,
                    int32_t* its, int32_t* error) {
  mk::rpp::Stage1 s;
  mk::rpp::stage1(model, iprts, s);
  *error = s.error;
  std::memcpy(sR, s.sR, sizeof(s.sR));
  for (int j = 0; j < mk::rpp::kCand; j++) {
    its[j] = -1;
    if (s.error != 1 && ((s.keep_mask >> j) & 1)) {
      mk::rpp::Refine r;
      mk::rpp::refine(model, s.Q, s.sR[j], r);
      std::memcpy(R + 9 * j, r.R, sizeof(r.R));
      std::memcpy(t + 3 * j, r.t, sizeof(r.t));
      errs[2 * j] = r.obj_err;
      errs[2 * j + 1] = r.img_err;
      its[j] = r.iterations;
    }
  }
  return s.keep_mask;
}

// iteration counts of the phases: it[0] first ObjPose, it[1..5] candidate ObjPoses (-1 if absent)
void hc_rpp_iters(const double* model, const double* iprts, int32_t* it) {
  mk::rpp::Stage1 s;
  mk::rpp::stage1(model, iprts, s);
  it[0] = s.iterations;
  for (int j = 0; j < mk::rpp::kCand; j++) {
    it[1 + j] = -1;
    if (s.error != 1 && ((s.keep_mask >> j) & 1)) {
      mk::rpp::Refine r;
      mk::rpp::refine(model, s.Q, s.sR[j], r);
      it[1 + j] = r.iterations;
    }
  }
}

// longest-first scheduling predictor (mk_rpp.h op_predict) for the first
// ObjPose (sR == nullptr) or a candidate ObjPose from initial rotation sR
float hc_objpose_predict(const double* model, const double* iprts, const double* sR, int kprobe) {
  mk::rpp::M34 P, Q;
  for (int i = 0; i < 12; i++) { P.a[i] = model[i]; Q.a[i] = iprts[i]; }
  mk::rpp::OpState s;
  mk::rpp::M33 R0;
  if (sR)
    for (int k = 0; k < 9; k++) R0.a[k] = sR[k];
  mk::rpp::op_setup(P, Q, sR ? &R0 : nullptr, s);
  return mk::rpp::op_predict(s, kprobe);
}

// the ObjPose error sequence (new_err after each AbsKernel, first n) and its
// total AbsKernel count (predictor studies, tools/)
int hc_objpose_trace(const double* model, const double* iprts, const double* sR, int n, double* errs) {
  mk::rpp::M34 P, Q;
  for (int i = 0; i < 12; i++) { P.a[i] = model[i]; Q.a[i] = iprts[i]; }
  mk::rpp::OpState s;
  mk::rpp::M33 R0;
  if (sR)
    for (int k = 0; k < 9; k++) R0.a[k] = sR[k];
  mk::rpp::op_setup(P, Q, sR ? &R0 : nullptr, s);
  int k = 0;
  while (!mk::rpp::op_step(s)) {
    if (k < n) errs[k] = s.new_err;
    k++;
  }
  return s.it;
}

int hc_rpoly(const double* op, int deg, double* zr, double* zi) { return mk::rpp::rpoly(op, deg, zr, zi); }

void hc_sort_desc(const double* err, int n, int* perm) {
  std::vector<mk::ErrIdx> v(n);
  for (int i = 0; i < n; i++) v[i] = {err[i], i};
  mk::std_sort_desc(v.data(), v.data() + n);
  for (int i = 0; i < n; i++) perm[i] = v[i].i;
}

int hc_approx(const int32_t* pts, int n, double eps, int closed, int32_t* out, int max_dp) {
  std::vector<int32_t> dst(2 * n + 2), stack(2 * n + 2);
  int m = mk::approx_poly(pts, n, eps, closed != 0, dst.data(), stack.data(), max_dp);
  if (m > n) return m;
  std::memcpy(out, dst.data(), sizeof(int32_t) * 2 * m);
  return m;
}

// Parallel contour formulation (what the GPU kernels compute), sequential here:
// fg 8-connected / bg 4-connected labels with root = minimum padded index,
// one border per fg component (outer, start = root) and per enclosed bg
// component (hole, start = root - 1), CCOMP/LIST output order from the keys.
int hc_find_contours(const uint8_t* bin, int w, int h, int mode, int32_t* pts, int max_pts, int32_t* meta,
                     int max_c) {
  const int Wp = w + 2, Hp = h + 2;
  std::vector<uint8_t> img((size_t)Wp * Hp, 0);
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) img[(size_t)(y + 1) * Wp + x + 1] = bin[(size_t)y * w + x] ? 1 : 0;
  std::vector<int> lab((size_t)Wp * Hp);
  for (size_t i = 0; i < lab.size(); i++) lab[i] = (int)i;
  auto find = [&](int x) {
    while (lab[x] != x) x = lab[x] = lab[lab[x]];
    return x;
  };
  auto unite = [&](int a, int b) {
    a = find(a); b = find(b);
    if (a == b) return;
    if (a < b) lab[b] = a; else lab[a] = b;
  };
  for (int y = 0; y < Hp; y++)
    for (int x = 0; x < Wp; x++) {
      int p = y * Wp + x;
      if (img[p]) {
        const int dx[4] = {-1, -1, 0, 1}, dy[4] = {0, -1, -1, -1};
        for (int k = 0; k < 4; k++) {
          int xx = x + dx[k], yy = y + dy[k];
          if (xx < 0 || yy < 0 || xx >= Wp) continue;
          int q = yy * Wp + xx;
          if (img[q]) unite(p, q);
        }
      } else {
        if (x > 0 && !img[p - 1]) unite(p, p - 1);
        if (y > 0 && !img[p - Wp]) unite(p, p - Wp);
      }
    }
  for (size_t i = 0; i < lab.size(); i++) lab[i] = find((int)i);
  struct B { long long key; int start; int hole; int parent; };
  std::vector<B> bs;
  for (int p = 0; p < Wp * Hp; p++) {
    if (lab[p] != p) continue;
    if (img[p]) bs.push_back({p, p, 0, p});
    else if (p != 0) bs.push_back({p, p - 1, 1, lab[p - 1]});
  }
  // CCOMP: outers by key desc, each followed by its holes by key desc; LIST: all by key desc
  std::sort(bs.begin(), bs.end(), [&](const B& a, const B& b) {
    if (mode == 2) {
      if (a.parent != b.parent) return a.parent > b.parent;
      if (a.hole != b.hole) return a.hole < b.hole;
    }
    return a.key > b.key;
  });
  if ((int)bs.size() > max_c) return -1;
  // the device tracer: packed 8-neighbourhood per step
  auto nb = [&](int x, int y) {
    auto row = [&](int yy) {
      const uint8_t* r = img.data() + (size_t)yy * Wp;
      return (uint32_t)(r[x - 1] != 0) | ((uint32_t)(r[x] != 0) << 1) | ((uint32_t)(r[x + 1] != 0) << 2);
    };
    return mk::nb8_from_rows(row(y - 1), row(y), row(y + 1));
  };
  int off = 0;
  for (size_t i = 0; i < bs.size(); i++) {
    int sx = bs[i].start % Wp, sy = bs[i].start / Wp;
    int n = mk::trace_border_nb(nb, sx, sy, bs[i].hole != 0, nullptr, 0);
    if (off + n > max_pts) return -1;
    mk::trace_border_nb(nb, sx, sy, bs[i].hole != 0, pts + 2 * off, n);
    meta[3 * i] = off;
    meta[3 * i + 1] = n;
    meta[3 * i + 2] = bs[i].hole;
    off += n;
  }
  return (int)bs.size();
}

// The bit-packed detector/mask chains (what the GPU passes compute), word by word.
void hc_masks_bits(const uint8_t* edge, int W, int H, uint8_t* det, uint8_t* mask) {
  namespace B = mk::bits;
  const int WW = B::words(W);
  std::vector<uint32_t> E((size_t)WW * H, 0), a((size_t)WW * H), b((size_t)WW * H);
  for (int y = 0; y < H; y++)
    for (int x = 0; x < W; x++)
      if (edge[(size_t)y * W + x]) E[(size_t)y * WW + (x >> 5)] |= 1u << (x & 31);
  auto hpass = [&](const std::vector<uint32_t>& src, std::vector<uint32_t>& dst, int r, bool dil) {
    for (int y = 0; y < H; y++)
      for (int w = 0; w < WW; w++) dst[(size_t)y * WW + w] = B::hword(src.data() + (size_t)y * WW, w, W, r, dil);
  };
  auto vpass = [&](const std::vector<uint32_t>& src, std::vector<uint32_t>& dst, int r, bool dil) {
    for (int y = 0; y < H; y++)
      for (int w = 0; w < WW; w++) dst[(size_t)y * WW + w] = B::vword(src.data(), w, y, W, H, r, dil);
  };
  auto unpack = [&](const std::vector<uint32_t>& src, uint8_t* out) {
    for (int y = 0; y < H; y++)
      for (int x = 0; x < W; x++) out[(size_t)y * W + x] = (src[(size_t)y * WW + (x >> 5)] >> (x & 31)) & 1u;
  };
  hpass(E, a, 2, true);
  vpass(a, b, 2, true);
  hpass(b, a, 1, false);
  vpass(a, b, 1, false);
  unpack(b, det);
  for (int y = 0; y < H; y++)
    for (int w = 0; w < WW; w++) a[(size_t)y * WW + w] = B::m0word(E.data(), w, y, W, H);
  for (int i = 0; i < 3; i++) {
    hpass(a, b, 3 + i, true);
    vpass(b, a, 3 + i, true);
    hpass(a, b, 3 + i, false);
    vpass(b, a, 3 + i, false);
  }
  hpass(a, b, 3, false);
  vpass(b, a, 3, false);
  unpack(a, mask);
}

void hc_distort(const double* xyz, int n, const double* K, const double* D, double* px) {
  mk::Cam cm{(double)(float)K[0], (double)(float)K[4], (double)(float)K[2], (double)(float)K[5], {D[0], D[1], D[2], D[3]}};
  for (int i = 0; i < n; i++) mk::distort(cm, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2], px + 2 * i, px + 2 * i + 1);
}
void hc_undistort(const double* px, int n, const double* K, const double* D, double* out) {
  mk::Cam cm{(double)(float)K[0], (double)(float)K[4], (double)(float)K[2], (double)(float)K[5], {D[0], D[1], D[2], D[3]}};
  for (int i = 0; i < n; i++) mk::undistort(cm, px[2 * i], px[2 * i + 1], out + 2 * i, out + 2 * i + 1);
}

// screen constants (mk_screen.h screen_cam_from / screen_bounds): out = sens,
// crel, S (per unit focal length), M; returns the bound's admissibility
int hc_screen_consts(const double* K, const double* D, int pieces, double* out) {
  mk::Cam cm;
  cm.fx = (double)(float)K[0];
  cm.fy = (double)(float)K[4];
  cm.cx = (double)(float)K[2];
  cm.cy = (double)(float)K[5];
  for (int k = 0; k < 4; k++) cm.k[k] = D[k];
  const mk::ScreenCam sc = mk::screen_cam_from(cm);
  const mk::ScreenBounds b = mk::screen_bounds(cm.k, pieces);
  out[0] = sc.sens;
  out[1] = sc.crel;
  out[2] = b.S;
  out[3] = b.M;
  return b.ok ? 1 : 0;
}

// FP32 projection screen (mk_screen.h) against the exact projection on n
// (c2w, landmark) pairs: res[4 i] = screen state (0 out, 1 in, 2 unsure),
// res[4 i + 1] = exact in-frame (z > 0 and inFrame), res[4 i + 2 / + 3] = the
// screened pixel when in (else the exact pixel). Returns the number of
// screened decisions that differ from the exact ones.
int hc_screen_check(const double* c2w, const double* X, int n, const double* K, const double* D, int W, int H,
                    int32_t* res) {
  mk::Cam cm{(double)(float)K[0], (double)(float)K[4], (double)(float)K[2], (double)(float)K[5], {D[0], D[1], D[2], D[3]}};
  const mk::ScreenCam sc = mk::screen_cam_from(cm);
  int bad = 0;
  for (int i = 0; i < n; i++) {
    mk::Xf T;
    for (int k = 0; k < 12; k++) (k < 9 ? T.R[k] : T.t[k - 9]) = c2w[12 * i + k];
    double rp[3], u, v;
    mk::xf_apply(T, X + 3 * i, rp);
    mk::distort(cm, rp[0], rp[1], rp[2], &u, &v);
    const bool in = rp[2] > 0 && mk::in_frame(u, v, H, W);
    float xl[4];
    mk::screen_landmark(X + 3 * i, xl);
    int px = 0, py = 0;
    const int st = mk::screen_project(mk::posef_from(T), xl[0], xl[1], xl[2], xl[3], sc, W, H, &px, &py);
    res[4 * i] = st;
    res[4 * i + 1] = in;
    res[4 * i + 2] = st == mk::SCR_IN ? px : (in ? mk::cv_round(u) : 0);
    res[4 * i + 3] = st == mk::SCR_IN ? py : (in ? mk::cv_round(v) : 0);
    if ((st == mk::SCR_IN && (!in || px != mk::cv_round(u) || py != mk::cv_round(v))) || (st == mk::SCR_OUT && in))
      bad++;
  }
  return bad;
}

// cross-rank bookkeeping of mantis_process_rig_sharded (mk_shard.h): the
// library's own rules, for the gloo tests
int hc_sizeof_cam_result(void) { return (int)sizeof(mantis_cam_result); }
int hc_sizeof_result(void) { return (int)sizeof(mantis_result); }
int hc_sizeof_shard_rec(void) { return (int)sizeof(mk::shard::Rec); }
void hc_shard_global_indices(int n_rigs, int n_local, const int32_t* cam_index, int cams_per_rig, int32_t* gidx) {
  mk::shard::global_indices(n_rigs, n_local, cam_index, cams_per_rig, gidx);
}
void hc_shard_pack_pairs(const int32_t* gidx, const int32_t* pf, int n_local, int slots, int32_t* pairs) {
  mk::shard::pack_pairs(gidx, pf, n_local, slots, pairs);
}
int64_t hc_shard_offsets(const int32_t* pairs, int npairs, int ng, int64_t per, int32_t* flags, int64_t* offset) {
  return mk::shard::offsets_from_pairs(pairs, npairs, ng, per, flags, offset);
}
// records of n local frames padded to slots (gidx -1)
void hc_shard_make_recs(const mantis_cam_result* res, const double* Tbc, const int32_t* gidx, int n, int slots,
                        mk::shard::Rec* out) {
  for (int s = 0; s < slots; s++) {
    std::memset(&out[s], 0, sizeof(out[s]));
    out[s].gidx = -1;
    if (s < n) {
      out[s].res = res[s];
      std::memcpy(out[s].Tbc, Tbc + 16 * (size_t)s, sizeof(double) * 16);
      out[s].gidx = gidx[s];
    }
  }
}
int hc_shard_merge(const mk::shard::Rec* recv, int nrec, int ng, mantis_cam_result* all, double* Tall) {
  std::vector<int32_t> seen(ng > 0 ? ng : 1);
  return mk::shard::merge_records(recv, nrec, ng, all, Tall, seen.data());
}
void hc_rig_results(int n_rigs, int cams_per_rig, const mantis_cam_result* all, const double* Tall, const int32_t* pf,
                    const uint64_t* states, mantis_result* out) {
  mk::shard::rig_results(n_rigs, cams_per_rig, all, Tall, pf, states, out);
}

// rig GN accumulators of n_obs observations [cam, u, v, X, Y, Z] about T_w_b
// (camera c has extrinsic T_base_cam[16 c]): the same residual rows as the
// device's MFMA accumulation (mk_gn.h gn_entry), summed in row order
void hc_gn_accumulate(const double* Twb, const double* Tbc, int n_cams, const double* obs, int n_obs, double* acc28) {
  std::vector<mk::GnCam> cams(n_cams);
  for (int i = 0; i < n_cams; i++) {
    const double* a = Tbc + 16 * i;
    for (int r = 0; r < 3; r++) {
      for (int k = 0; k < 3; k++) cams[i].R_cb[3 * r + k] = a[4 * k + r];
      cams[i].t_cb[r] = -(a[r] * a[3] + a[4 + r] * a[7] + a[8 + r] * a[11]);
    }
  }
  mk::gn_accumulate_seq(Twb, cams.data(), obs, n_obs, acc28);
}

// per-quad GN after RPP (mk_gn.h quad_gn_refine) on n problems
void hc_quad_gn(int n, double* R, double* t, const double* img, const double* obj, int iters, int32_t* steps,
                double* cost0, double* cost) {
  for (int i = 0; i < n; i++)
    steps[i] = mk::quad_gn_refine(R + 9 * i, t + 3 * i, img + 8 * i, obj + 12 * i, iters, cost0 + i, cost + i);
}

}  // extern "C"
