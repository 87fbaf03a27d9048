// Cross-rank bookkeeping of the camera-sharded rig call
// (mantis_process_rig_sharded, include/mantis.h; the reference's multi-camera
// seam is include/legacy/mantis/MonteCarlo.cpp:250-271) as plain host
// functions, shared by the library (api.hip) and the CPU test build
// (hostcheck.cpp), so the gloo tests run the very rules the library runs:
//   * global frame order: rig-major, camera c of rig r is frame r * C + c;
//   * the cv::RNG stream (global cv::RNG rng(1), Mantis3Params.h:87) is consumed
//     by the frames that reach the particle filter (PoseAdjustment.h:15-16,
//     `per` gaussians each), in global order, as one sequential run over all
//     cameras would: a frame's offset is per x (PF frames before it);
//   * each rank sends (global index, PF flag) pairs padded to a common slot
//     count with (-1, 0), and camera records padded with gidx -1; every global
//     frame must arrive exactly once;
//   * the rig result is the published camera with the lowest error mapped
//     through T_base_cam (fuse_rig), and rng_state_after of rig r is the RNG
//     state after the PF frames of rigs 0..r.
// The device form of offsets_from_pairs is k_gauss_offsets_global
// (kernels.hip); tests/test_gpu_multi.py compares them on fabricated gathers.
#pragma once
#include <cstdint>
#include <cstring>

#include "../../include/mantis.h"
#include "mk_math.h"

namespace mk {
namespace shard {

// global index of each local frame (rig-major: rig r, local camera j)
inline void global_indices(int n_rigs, int n_local, const int32_t* cam_index, int cams_per_rig, int32_t* gidx) {
  for (int r = 0; r < n_rigs; r++)
    for (int j = 0; j < n_local; j++) gidx[(size_t)r * n_local + j] = r * cams_per_rig + cam_index[j];
}

// this rank's (global index, PF flag) pairs, padded to `slots` with (-1, 0)
inline void pack_pairs(const int32_t* gidx, const int32_t* pf, int n_local, int slots, int32_t* pairs) {
  for (int s = 0; s < slots; s++) {
    pairs[2 * s] = s < n_local ? gidx[s] : -1;
    pairs[2 * s + 1] = s < n_local ? (pf[s] ? 1 : 0) : 0;
  }
}

// the gathered pairs of every rank (npairs = slots x ranks) -> flags[ng] in
// global order and offset[ng] = per x (PF frames before g); returns the total
// gaussians drawn, or -1 if a global index is out of range
inline int64_t offsets_from_pairs(const int32_t* pairs, int npairs, int ng, int64_t per, int32_t* flags,
                                  int64_t* offset) {
  for (int g = 0; g < ng; g++) flags[g] = 0;
  for (int i = 0; i < npairs; i++) {
    const int g = pairs[2 * i];
    if (g < 0) continue;
    if (g >= ng) return -1;
    flags[g] = pairs[2 * i + 1];
  }
  int64_t acc = 0;
  for (int g = 0; g < ng; g++) {
    offset[g] = acc;
    if (flags[g]) acc += per;
  }
  return acc;
}

// one camera's result as exchanged between the ranks
struct Rec {
  mantis_cam_result res;
  double Tbc[16];
  int32_t gidx, pad;
};

// received records -> every camera's result and T_base_cam in global order:
// 0 ok, 1 a camera arrived twice, 2 a camera never arrived, 3 index out of range
inline int merge_records(const Rec* recv, int nrec, int ng, mantis_cam_result* all, double* Tall, int32_t* seen) {
  for (int g = 0; g < ng; g++) seen[g] = 0;
  for (int i = 0; i < nrec; i++) {
    const int g = recv[i].gidx;
    if (g < 0) continue;
    if (g >= ng) return 3;
    if (seen[g]++) return 1;
    all[g] = recv[i].res;
    std::memcpy(Tall + 16 * (size_t)g, recv[i].Tbc, sizeof(double) * 16);
  }
  for (int g = 0; g < ng; g++)
    if (!seen[g]) return 2;
  return 0;
}

// 4x4 helpers for rig results (row-major)
inline void mat4_mul(const double* a, const double* b, double* o) {
  double r[16];
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++) {
      double s = 0;
      for (int k = 0; k < 4; k++) s += a[i * 4 + k] * b[k * 4 + j];
      r[i * 4 + j] = s;
    }
  std::memcpy(o, r, sizeof(r));
}
inline void mat4_inv_rigid(const double* a, double* o) {
  double r[16] = {0};
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) r[i * 4 + j] = a[j * 4 + i];
  for (int i = 0; i < 3; i++) r[i * 4 + 3] = -(r[i * 4 + 0] * a[3] + r[i * 4 + 1] * a[7] + r[i * 4 + 2] * a[11]);
  r[15] = 1;
  std::memcpy(o, r, sizeof(r));
}
inline void quat_to_mat4(const double* q, const double* p, double* T) {
  Quat qq{q[0], q[1], q[2], q[3]};
  double R[9];
  basis_from_quat(qq, R);
  for (int i = 0; i < 16; i++) T[i] = 0;
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) T[i * 4 + j] = R[i * 3 + j];
    T[i * 4 + 3] = p[i];
  }
  T[15] = 1;
}

// Rig pose from per-camera results (reference-parity mode: no GN): the
// published camera with the lowest error, mapped through T_base_cam.
inline void fuse_rig(const double* Tbc, const mantis_cam_result* cr, int nc, mantis_result* out) {
  std::memset(out, 0, sizeof(*out));
  int best = -1;
  int npub = 0, nscored = 0, nq = 0;
  for (int i = 0; i < nc; i++) {
    nscored += cr[i].n_scored;
    nq += cr[i].n_quads;
    if (cr[i].publish) {
      npub++;
      if (best < 0 || cr[i].error < cr[best].error) best = i;
    }
  }
  out->num_particles = nscored;
  out->n_quads = nq;
  out->n_cams_published = npub;
  out->status = MANTIS_OK;
  if (best < 0) {
    // nothing passes the yaw gate: report the first camera that produced a pose, unpublished
    for (int i = 0; i < nc && best < 0; i++)
      if (cr[i].reason == MANTIS_PUBLISHED || cr[i].reason == MANTIS_YAW_AMBIGUOUS) best = i;
    out->publish = 0;
    if (best < 0) return;
  } else {
    out->publish = 1;
  }
  double Twc[16], Tbc_inv[16], Twb[16];
  quat_to_mat4(cr[best].orientation_xyzw, cr[best].position, Twc);
  mat4_inv_rigid(Tbc + 16 * (size_t)best, Tbc_inv);
  mat4_mul(Twc, Tbc_inv, Twb);
  double R[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) R[i * 3 + j] = Twb[i * 4 + j];
  Quat q = basis_to_quat(R);
  out->orientation_xyzw[0] = q.x; out->orientation_xyzw[1] = q.y;
  out->orientation_xyzw[2] = q.z; out->orientation_xyzw[3] = q.w;
  for (int i = 0; i < 3; i++) out->position[i] = Twb[i * 4 + 3];
  for (int i = 0; i < 36; i++) out->covariance[i] = cr[best].covariance[i];
  out->weight = cr[best].error;
  out->min_yaw_diff = cr[best].min_yaw_diff;
}

// every rig's fused result and RNG state after it: all / Tall in global
// order, pf[g] the global PF flags, states[k] the RNG state after k PF frames
inline void rig_results(int n_rigs, int cams_per_rig, const mantis_cam_result* all, const double* Tall,
                        const int32_t* pf, const uint64_t* states, mantis_result* out) {
  int k = 0;
  for (int r = 0; r < n_rigs; r++) {
    fuse_rig(Tall + 16 * (size_t)r * cams_per_rig, all + (size_t)r * cams_per_rig, cams_per_rig, &out[r]);
    for (int i = 0; i < cams_per_rig; i++) k += pf[r * cams_per_rig + i] ? 1 : 0;
    out[r].rng_state_after = states[k];
  }
}

}  // namespace shard
}  // namespace mk
