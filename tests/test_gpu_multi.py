"""GPU tests of the multi-GPU code paths on one MI355X (SURVEY §8 e):

* the RCCL call sites through a one-rank communicator (mantis_comm_init,
  mantis_gn_allreduce, mantis_score_argmin(use_comm=1)), which must leave the
  single-GPU answers unchanged;
* BASELINE config 4 — one 8-camera 1920x1080 rig — per camera against the CPU
  oracle, its rig Gauss-Newton against the FP64 restatement
  (tests/_gn_ref.rig_gn_reference), and the camera-sharded call
  (mantis_process_rig_sharded: PF-flag all-gather, result all-gather, per-
  iteration all-reduce of the J^T J / J^T r slots) equal to the batched call.

Tolerances: the rig GN correspondences and pose 1e-9 absolute against the
FP64 restatement (device MFMA sums vs numpy matmul order, device vs glibc
tan/sin/cos ulps); the one-rank sharded run is bit-identical to the batch.
"""
import ctypes as C

import numpy as np
import pytest

import _gn_ref as G
import _oracle as O
from mantis_amd import synth
from test_gpu_parity import _cmp_debug

pytestmark = pytest.mark.gpu
GN_TOL = 1e-9


def _render_rigs(n_rigs, n_cams, W, H, seed, cfg_id):
    import mantis_amd as M

    K, D = synth.intrinsics(W, H)
    ext = synth.rig_extrinsics(n_cams)
    rng = np.random.default_rng(seed)
    host, imgs, truth = [], [], []
    for r in range(n_rigs):
        Twb = synth.random_base_pose(rng)
        truth.append(Twb)
        for c in range(n_cams):
            Twc = Twb @ ext[c]
            fr = synth.render_host(synth.make_cam(Twc[:3, :3], Twc[:3, 3], W, H), synth.frame_seed(cfg_id, 100 * r + c))
            host.append(fr)
            imgs.append(M.make_image(fr, K, D, T_base_cam=ext[c]))
    return K, D, ext, host, imgs, truth


def check_rig_gn_against_restatement(m, ext, n_rigs, K, D, iterations, frame_base=0):
    """The device rig GN of every rig of the last batch against the FP64
    restatement: same correspondences (count, order, values), same pose."""
    Kf = np.asarray(K, np.float64).astype(np.float32).astype(np.float64)  # get3x3FromVector rounds K to float
    und = lambda px: O.undistort(px, Kf, D)
    n_cams = len(ext)
    checked = 0
    for r in range(n_rigs):
        info, obs = m.rig_gn(r)
        if not info.valid:
            continue
        cam_quads = []
        for c in range(n_cams):
            d = m.frame_debug(frame_base + r * n_cams + c)
            cam_quads.append(np.array(d.quads)[: d.n_quads])
        T0 = np.array(info.T_init).reshape(4, 4)
        obs_ref, T_ref, its, cost0, cost = G.rig_gn_reference(T0, ext, cam_quads, [und] * n_cams, iterations)
        assert info.n_obs == len(obs_ref) == info.n_obs_local, (r, info.n_obs, len(obs_ref))
        np.testing.assert_allclose(obs, obs_ref, atol=GN_TOL, rtol=0)
        np.testing.assert_allclose(np.array(info.T_final).reshape(4, 4), T_ref, atol=GN_TOL, rtol=0)
        if len(obs_ref) >= 6:
            assert abs(info.iterations - its) <= 1  # the 1e-12 step threshold may fall either side by an ulp
            np.testing.assert_allclose(info.cost0, cost0, rtol=1e-9, atol=1e-18)
        checked += 1
    return checked


def test_rccl_one_rank_communicator(landmark_map):
    import mantis_amd as M
    from mantis_amd import dense

    m = M.Mantis(max_cams=1)
    m.set_map(*landmark_map)
    with pytest.raises(M.MantisError):
        m.comm_info()  # no communicator yet: MANTIS_ERR_STATE
    acc = np.random.default_rng(3).normal(size=28)
    a = acc.copy()
    assert M.lib().mantis_gn_allreduce(m.h, a.ctypes.data) == 5  # MANTIS_ERR_STATE without comm
    m.comm_init(0, 1)
    assert m.comm_info() == (1, 0)
    assert M.lib().mantis_gn_allreduce(m.h, a.ctypes.data) == 0
    assert np.array_equal(a, acc)  # a sum over one rank is the identity
    rng = np.random.default_rng(8)
    R, pos = synth.random_pose(rng)
    K, D = synth.intrinsics()
    img = synth.render_host(synth.make_cam(R, pos), synth.frame_seed(5, 9))
    im = M.make_image(img, K, D)
    _, mask = m.masks(im)
    hyps = dense.config5_hypotheses(R, pos, np.random.default_rng(4), n_particles=2)
    local = m.score_argmin(im, hyps, 0, False, mask)
    shared = m.score_argmin(im, hyps, 0, True, mask)
    assert local == shared and local[1] >= 0
    base = m.score_argmin(im, hyps, 1000, True, mask)
    assert base == (local[0], local[1] + 1000)
    m.comm_init(0, 1)  # re-initialisation replaces the communicator
    assert m.comm_info() == (1, 0)
    assert m.score_argmin(im, hyps, 0, True, mask) == local
    m.close()


def test_config4_8cam_1080p_rig_and_sharded_one_rank(landmark_map):
    import mantis_amd as M

    W, H, n_rigs, n_cams, its = 1920, 1080, 2, 8, 8
    K, D, ext, host, imgs, truth = _render_rigs(n_rigs, n_cams, W, H, 44, 4)
    cfg = dict(max_cams=n_rigs * n_cams, max_width=W, max_height=H, gn_enable=1, gn_iterations=its)
    mb = M.Mantis(M.default_config(**cfg))
    mb.set_map(*landmark_map)
    mb.rng_state = 1
    rb, cb = mb.process(imgs, rigs=n_rigs)
    orc = O.Oracle(*landmark_map, seed=1)
    states = []
    for i, fr in enumerate(host):
        _cmp_debug(mb.frame_debug(i), orc.process(fr, K, D), f"config4 rig {i // n_cams} cam {i % n_cams}")
        states.append(orc.rng_state)
    for r in range(n_rigs):
        assert rb[r].rng_state_after == states[n_cams * r + n_cams - 1]
    assert mb.rng_state == orc.rng_state
    assert sum(r.n_quads for r in rb) > 0
    assert check_rig_gn_against_restatement(mb, ext, n_rigs, K, D, its) >= 1
    # the camera-sharded call on a one-rank communicator: every exchange runs
    # (PF flags, camera results, GN accumulators) and the answer is the batch's
    ms = M.Mantis(M.default_config(**cfg))
    ms.set_map(*landmark_map)
    ms.comm_init(0, 1)
    ms.rng_state = 1
    rs, cs = ms.process_sharded(imgs, n_rigs, list(range(n_cams)), n_cams)
    assert ms.rng_state == mb.rng_state
    for a, b in zip(rb, rs):
        assert bytes(a) == bytes(b)
    for a, b in zip(cb, cs):
        assert bytes(a) == bytes(b)
    for r in range(n_rigs):
        ia, oa = mb.rig_gn(r)
        ib, ob = ms.rig_gn(r)
        assert bytes(ia) == bytes(ib) and np.array_equal(oa, ob)
    # a rank that does not hold every camera of a one-rank rig is rejected up front
    with pytest.raises(M.MantisError):
        ms.process_sharded(imgs[:n_rigs * 4], n_rigs, [0, 1, 2, 3], n_cams)
    # a rank-local staging failure (row step < 3 W) goes through the agreement
    # all-reduce before the PF-flag exchange and returns an error (with more
    # ranks the others return MANTIS_ERR_COMM instead of blocking in the
    # all-gather); the communicator stays usable and the next call is correct
    bad = [M.make_image(host[i], K, D, T_base_cam=ext[i % n_cams]) for i in range(n_rigs * n_cams)]
    bad[3].step_bytes = 3 * W - 3
    with pytest.raises(M.MantisError, match="step"):
        ms.process_sharded(bad, n_rigs, list(range(n_cams)), n_cams)
    ms.rng_state = 1
    rs2, _ = ms.process_sharded(imgs, n_rigs, list(range(n_cams)), n_cams)
    for a, b in zip(rb, rs2):
        assert bytes(a) == bytes(b)
    mb.close()
    ms.close()


def test_gauss_offsets_global_fabricated_gathers():
    """k_gauss_offsets_global (the device half of the sharded call's cv::RNG
    bookkeeping, mantis_shard_gauss_offsets) on fabricated all-gathers of 2 and
    8 ranks -- uneven camera splits with padding slots (-1, 0), random PF
    flags -- against the library's host rule (mk_shard.h, CPU build) and the
    sequential prefix a single run over all cameras consumes."""
    import _hostcheck as HC
    import mantis_amd as M
    from mantis_amd import rig

    m = M.Mantis(max_cams=64, max_width=64, max_height=64)
    try:
        rng = np.random.default_rng(31)
        per = 3000
        for world, n_rigs, cams in [(2, 5, 4), (8, 3, 8), (3, 7, 8), (8, 2, 5)]:
            ng = n_rigs * cams
            pf = (rng.random(ng) < 0.7).astype(np.int32)
            nl_max = -(-cams // world)
            slots = n_rigs * nl_max
            gathered, locals_ = [], []
            for r in range(world):
                ci = rig.shard_cameras(cams, r, world)
                g = HC.shard_global_indices(n_rigs, ci, cams) if ci else np.zeros(0, np.int32)
                locals_.append(g)
                gathered.append(HC.shard_pack_pairs(g, pf[g], slots))
            pairs = np.concatenate(gathered)
            flags, off_host, tot_host = HC.shard_offsets(pairs, ng, per)
            seq = per * np.concatenate([[0], np.cumsum(pf)[:-1]])
            assert np.array_equal(off_host, seq) and tot_host == per * pf.sum()
            for r in range(world):
                if len(locals_[r]) == 0:
                    continue
                off, tot = m.shard_gauss_offsets(pairs, ng, locals_[r], per)
                assert np.array_equal(off, seq[locals_[r]]), f"world {world} rank {r}"
                assert tot == tot_host
            # a malformed gather (a frame index >= n_global) is rejected by both
            # halves: the host rule returns -1, the entry point an error
            badp = pairs.copy()
            badp[0] = ng
            assert HC.shard_offsets(badp, ng, per)[2] == -1
            with pytest.raises(M.MantisError, match="pair index"):
                m.shard_gauss_offsets(badp, ng, locals_[0], per)
    finally:
        m.close()
