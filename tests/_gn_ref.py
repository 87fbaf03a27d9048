"""Plain-numpy FP64 reference of the rig Gauss-Newton accumulators
(mantis_amd/csrc/gn_impl.hip): residual r = pi(p) - u, p = inv(T_b_c) inv(T_w_b) X,
right perturbation T_w_b <- T_w_b Exp(rho, phi). Returns the 28 doubles
(upper-triangle J^T J row-major, J^T r, r^T r). Test infrastructure only.
"""
import numpy as np


def skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def rigid_inv(T):
    R, t = T[:3, :3], T[:3, 3]
    Ti = np.eye(4)
    Ti[:3, :3] = R.T
    Ti[:3, 3] = -R.T @ t
    return Ti


def gn_rows(T_w_b, T_b_c, obs):
    """obs rows: (cam, u, v, X, Y, Z). Returns M = [J | r] (2N x 7)."""
    Rwb, twb = T_w_b[:3, :3], T_w_b[:3, 3]
    rows = []
    for o in obs:
        c = int(o[0])
        Tcb = rigid_inv(T_b_c[c])
        q = Rwb.T @ (o[3:6] - twb)
        p = Tcb[:3, :3] @ q + Tcb[:3, 3]
        iz = 1.0 / p[2]
        r = np.array([p[0] * iz - o[1], p[1] * iz - o[2]])
        dpi = np.array([[iz, 0, -p[0] * iz * iz], [0, iz, -p[1] * iz * iz]])
        dp = Tcb[:3, :3] @ np.hstack([-np.eye(3), skew(q)])
        J = dpi @ dp
        for k in range(2):
            rows.append(np.concatenate([J[k], [r[k]]]))
    return np.array(rows).reshape(-1, 7)


def gn_accumulate(T_w_b, T_b_c, obs):
    M = gn_rows(T_w_b, T_b_c, obs)
    D = M.T @ M
    iu = np.triu_indices(6)
    return np.concatenate([D[:6, :6][iu], D[:6, 6], [D[6, 6]]])


def exp_se3_right(T, delta):
    rho, phi = delta[:3], delta[3:]
    th = np.linalg.norm(phi)
    K = skew(phi)
    if th < 1e-12:
        a, b = 1.0, 0.5
    else:
        a, b = np.sin(th) / th, (1 - np.cos(th)) / th ** 2
    dR = np.eye(3) + a * K + b * K @ K
    D = np.eye(4)
    D[:3, :3] = dR
    D[:3, 3] = rho
    return T @ D


def gn_solve(acc28, lam, T_w_b):
    A = np.zeros((6, 6))
    A[np.triu_indices(6)] = acc28[:21]
    A = A + np.triu(A, 1).T + lam * np.eye(6)
    x = np.linalg.solve(A, -np.asarray(acc28[21:27]))
    return exp_se3_right(T_w_b, x), x


def synth_rig_obs(rng, T_w_b, T_b_c, n_per_cam=24, noise=1e-3):
    """World points in front of each camera and their noisy normalized projections."""
    obs = []
    for c, Tbc in enumerate(T_b_c):
        Twc = T_w_b @ Tbc
        for _ in range(n_per_cam):
            pc = np.array([rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5), rng.uniform(1.0, 3.0)])
            X = Twc[:3, :3] @ pc + Twc[:3, 3]
            u = pc[:2] / pc[2] + rng.normal(size=2) * noise
            obs.append([c, u[0], u[1], X[0], X[1], X[2]])
    return np.array(obs)
