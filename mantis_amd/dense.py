"""Dense hypothesis scoring, sharded (BASELINE config 5, SURVEY §8 d/e).

The global hypothesis list (81 shifts x 4 yaws x 50 perturbations = 16,200 for
config 5) is split into contiguous blocks, one per rank; each rank scores its
block with mantis_score_argmin (device first-minimum), and one ncclAllGather of
(err, global index) per rank plus the same first-minimum rule give every rank
the global winner — the reference's strict "<" best-1 choice over the whole
list (HypothesisEvaluation.h:490-518).
"""
import numpy as np

from . import synth


def shard_range(n, rank, world):
    """Contiguous block [lo, hi) of rank (the first n % world ranks get one more)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def config5_hypotheses(R_wc, pos, rng, n_particles=50, sigma_rot=0.03, sigma_t=0.01, spacing=0.32):
    """81 grid shifts x 4 yaw copies x n_particles perturbations of a camera
    pose (SURVEY §8 d config 5), as world->camera 3x4 rows (c2w layout of
    mantis_score_hypotheses): shifts as computeAllShiftedHypothesesFAST
    (HypothesisGeneration.h:125-140, +-1.28 m step 0.32), yaws as
    determineBestYaw's rotZ(k*90 deg) about the world origin
    (HypothesisEvaluation.h:521-581), perturbations as the particle filter's
    gaussian pose noise (PoseAdjustment.h:13-27, sigma 0.03 rad / 0.01 m)."""
    out = []
    steps = [-1.28 + spacing * k for k in range(9)]
    for dx in steps:
        for dy in steps:
            for k in range(4):
                Rz = synth.rot_z(k * np.pi / 2)
                Rw = Rz @ R_wc
                p = Rz @ (pos + np.array([dx, dy, 0.0]))
                for _ in range(n_particles):
                    a = rng.normal(size=3) * sigma_rot
                    Rp = Rw @ synth.rot_z(a[2]) @ synth.rot_y(a[1]) @ synth.rot_x(a[0])
                    pp = p + rng.normal(size=3) * sigma_t
                    Rcw = Rp.T
                    out.append(np.concatenate([Rcw.reshape(9), -Rcw @ pp]))
    return np.array(out)
