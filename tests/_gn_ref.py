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


def quad_cell_obs(corners, undistort, Rwc, Cw, half=1.44, spacing=0.32):
    """FP64 restatement of gn_quad_obs (mantis_amd/csrc/gn_impl.hip): the
    crossing of the quad's undistorted diagonals, back-projected with the
    camera pose onto the floor z = 0 and snapped to the nearest cell centre
    (accepted within 0.1 m). corners: 4 x 2 pixel ints; undistort(px) -> 4 x 2
    normalized. Returns (u, v, X, Y, 0) or None."""
    uv = undistort(np.asarray(corners, np.float64).reshape(4, 2))
    u, v = uv[:, 0], uv[:, 1]
    d1x, d1y, d2x, d2y = u[2] - u[0], v[2] - v[0], u[3] - u[1], v[3] - v[1]
    den = d1x * d2y - d1y * d2x
    if abs(den) < 1e-12:
        return None
    a = ((u[1] - u[0]) * d2y - (v[1] - v[0]) * d2x) / den
    if not (0 < a < 1):
        return None
    uc, vc = u[0] + a * d1x, v[0] + a * d1y
    dw = Rwc @ np.array([uc, vc, 1.0])
    if not dw[2] < -1e-9:
        return None
    tt = -Cw[2] / dw[2]
    if not tt > 0:
        return None
    X, Y = Cw[0] + tt * dw[0], Cw[1] + tt * dw[1]
    c0 = -half + 0.5 * spacing
    kx, ky = np.rint((X - c0) / spacing), np.rint((Y - c0) / spacing)
    lim = np.rint(2 * half / spacing) - 1
    if kx < 0 or ky < 0 or kx > lim or ky > lim:
        return None
    gx, gy = c0 + spacing * kx, c0 + spacing * ky
    if abs(X - gx) > 0.1 or abs(Y - gy) > 0.1:
        return None
    return np.array([uc, vc, gx, gy, 0.0])


def rig_gn_reference(T0, T_b_c, cam_quads, undistorters, iterations, lam=1e-9, half=1.44, spacing=0.32):
    """FP64 restatement of the pipeline's rig Gauss-Newton (k_rig_gn_obs /
    _acc / _step): correspondences formed once with the fused pose T0 in
    (camera, quad) order, then up to `iterations` solves of the summed normal
    equations, stopping when the step is below 1e-12 or the system is not
    positive definite; fewer than 6 correspondences keep T0.
    Returns (obs rows [cam, u, v, X, Y, Z], T, iterations, cost0, cost)."""
    obs = []
    for c, quads in enumerate(cam_quads):
        Twc = T0 @ T_b_c[c]
        for q in quads:
            o = quad_cell_obs(np.asarray(q).reshape(4, 2), undistorters[c], Twc[:3, :3], Twc[:3, 3], half, spacing)
            if o is not None:
                obs.append(np.concatenate([[c], o]))
    obs = np.array(obs).reshape(-1, 6)
    T = np.array(T0, np.float64)
    if len(obs) < 6:
        return obs, T, 0, 0.0, 0.0
    cost0 = cost = None
    it_done = 0
    for it in range(iterations):
        acc = gn_accumulate(T, T_b_c, obs)
        if it == 0:
            cost0 = acc[27]
        cost = acc[27]
        it_done = it + 1
        A = np.zeros((6, 6))
        A[np.triu_indices(6)] = acc[:21]
        A = A + np.triu(A, 1).T + lam * np.eye(6)
        try:
            np.linalg.cholesky(A)
        except np.linalg.LinAlgError:
            break
        T, x = gn_solve(acc, lam, T)
        if float(x @ x) < 1e-24:
            break
    return obs, T, it_done, cost0, cost


def quad_gn_reference(R, t, img, obj, iterations, lam=1e-9):
    """FP64 restatement of the per-quad GN after RPP (mk_gn.h quad_gn_refine):
    the pose R, t (model -> camera) of one quad refined on its 4 normalized
    image points img (4 x 2) against the model points obj (4 x 3), as the
    camera pose T = inv([R | t]) with identity extrinsics; a step is kept only
    if the cost decreases; stops when the step norm^2 < 1e-24 or the normal
    matrix is singular. Returns (R, t, steps, cost0, cost)."""
    obs = np.hstack([np.zeros((4, 1)), np.asarray(img, np.float64).reshape(4, 2),
                     np.asarray(obj, np.float64).reshape(4, 3)])
    ext = [np.eye(4)]
    Tcw = np.eye(4)
    Tcw[:3, :3] = np.asarray(R, np.float64).reshape(3, 3)
    Tcw[:3, 3] = np.asarray(t, np.float64).reshape(3)
    T = rigid_inv(Tcw)
    acc = gn_accumulate(T, ext, obs)
    cost0 = acc[27]
    steps = 0
    for _ in range(iterations):
        A = np.zeros((6, 6))
        A[np.triu_indices(6)] = acc[:21]
        A = A + np.triu(A, 1).T + lam * np.eye(6)
        try:
            np.linalg.cholesky(A)
        except np.linalg.LinAlgError:
            break
        Tn, x = gn_solve(acc, lam, T)
        acc_n = gn_accumulate(Tn, ext, obs)
        if not acc_n[27] <= acc[27]:
            break
        T, acc = Tn, acc_n
        steps += 1
        if float(x @ x) < 1e-24:
            break
    Tc = rigid_inv(T)
    return Tc[:3, :3], Tc[:3, 3], steps, cost0, acc[27]


def quad_problems(rng, n, noise=2e-3, pose_noise=0.02, half=0.16):
    """n synthetic per-quad problems: the model square +-half seen by a random
    camera 0.8..2.5 m away, noisy normalized corners, and a perturbed start
    pose. Returns (img n x 4 x 2, obj n x 4 x 3, R0 n x 3 x 3, t0 n x 3,
    R_true, t_true)."""
    obj = np.array([[half, half, 0], [-half, half, 0], [-half, -half, 0], [half, -half, 0]], np.float64)
    imgs, R0s, t0s, Rts, tts = [], [], [], [], []
    for _ in range(n):
        a = rng.normal(size=3) * 0.4
        Rt = exp_se3_right(np.eye(4), np.concatenate([[0, 0, 0], a]))[:3, :3]
        Rt = Rt @ np.diag([1.0, -1.0, -1.0])  # camera looks down at the plane
        tt = np.array([rng.uniform(-0.3, 0.3), rng.uniform(-0.3, 0.3), rng.uniform(0.8, 2.5)])
        pc = (Rt @ obj.T).T + tt
        imgs.append(pc[:, :2] / pc[:, 2:3] + rng.normal(size=(4, 2)) * noise)
        Tp = exp_se3_right(rigid_inv(np.vstack([np.hstack([Rt, tt[:, None]]), [0, 0, 0, 1]])),
                           rng.normal(size=6) * pose_noise)
        Tc = rigid_inv(Tp)
        R0s.append(Tc[:3, :3])
        t0s.append(Tc[:3, 3])
        Rts.append(Rt)
        tts.append(tt)
    return (np.array(imgs), np.repeat(obj[None], n, 0), np.array(R0s), np.array(t0s), np.array(Rts),
            np.array(tts))
