"""numpy restatement of the reference's tracker Gauss-Newton (frame -> keyframe
relative Sim(3) pose).

TEST INFRASTRUCTURE ONLY (checker for the device tracker path and the CPU
baseline's tracker leg). Follows, line for line in behaviour:

* ``FrameTracker.opt_pose_ray_dist_sim3``  tracker.py:173-214
* ``FrameTracker.opt_pose_calib_sim3``     tracker.py:216-266
* ``FrameTracker.solve``                   tracker.py:156-171
* ``point_to_ray_dist`` / ``act_Sim3`` / ``project_calib``
                                           geometry.py:17-34, 45-52, 63-104
* ``huber`` / ``check_convergence``        nonlinear_optimizer.py:5-33

Group arithmetic (lietorch, third-party, absent offline) follows the
reference's CUDA restatement gn_kernels.cu:172-413 — parity for that part is
pinned only through tests/golden (reference tracker run with the same Sim3).
Pinned against tests/golden/tracker_*.npz (the reference's own tracker code).
"""
from __future__ import annotations

import math

import numpy as np

F32 = np.float32


class CholeskyFailed(RuntimeError):
    pass


# ------------------------------------------------------------ Sim3 (f32) --
def qmul(a, b):
    ax, ay, az, aw = a[..., 0], a[..., 1], a[..., 2], a[..., 3]
    bx, by, bz, bw = b[..., 0], b[..., 1], b[..., 2], b[..., 3]
    return np.stack(
        [
            aw * bx + ax * bw + ay * bz - az * by,
            aw * by - ax * bz + ay * bw + az * bx,
            aw * bz + ax * by - ay * bx + az * bw,
            aw * bw - ax * bx - ay * by - az * bz,
        ],
        -1,
    ).astype(F32)


def qrot(q, X):
    qv, w = q[..., :3], q[..., 3:4]
    uv = F32(2.0) * np.cross(qv, X)
    return (X + w * uv + np.cross(qv, uv)).astype(F32)


def act(T, X):
    return (T[..., 7:8] * qrot(T[..., 3:7], X) + T[..., 0:3]).astype(F32)


def inv(T):
    qi = np.concatenate([-T[..., 0 + 3 : 6], T[..., 6:7]], -1)
    si = F32(1.0) / T[..., 7:8]
    ti = -si * qrot(qi, T[..., 0:3])
    return np.concatenate([ti, qi, si], -1).astype(F32)


def mul(A, B):
    q = qmul(A[..., 3:7], B[..., 3:7])
    t = A[..., 0:3] + A[..., 7:8] * qrot(A[..., 3:7], B[..., 0:3])
    return np.concatenate([t, q, A[..., 7:8] * B[..., 7:8]], -1).astype(F32)


def exp_sim3(xi):
    xi = np.asarray(xi, F32).reshape(7)
    tau, phi, sigma = xi[0:3].copy(), xi[3:6], F32(xi[6])
    scale = F32(np.exp(sigma))
    th2 = F32(phi @ phi)
    if th2 < 1e-6:
        th4 = th2 * th2
        im = F32(0.5 - th2 / 48.0 + th4 / 3840.0)
        re = F32(1.0 - th2 / 8.0 + th4 / 384.0)
    else:
        th = F32(np.sqrt(th2))
        im = F32(np.sin(0.5 * th) / th)
        re = F32(np.cos(0.5 * th))
    q = np.array([im * phi[0], im * phi[1], im * phi[2], re], F32)
    th = F32(np.sqrt(th2))
    if abs(sigma) < 1e-6:
        C = F32(1.0)
        if abs(th) < 1e-6:
            A, B = F32(0.5), F32(1.0 / 6.0)
        else:
            A = F32((1.0 - np.cos(th)) / th2)
            B = F32((th - np.sin(th)) / (th2 * th))
    else:
        C = F32((scale - 1.0) / sigma)
        if abs(th) < 1e-6:
            sg2 = sigma * sigma
            A = F32(((sigma - 1.0) * scale + 1.0) / sg2)
            B = F32((scale * 0.5 * sg2 + scale - 1.0 - sigma * scale) / (sg2 * sigma))
        else:
            a, b = F32(scale * np.sin(th)), F32(scale * np.cos(th))
            c = F32(th2 + sigma * sigma)
            A = F32((a * sigma + (1.0 - b) * th) / (th * c))
            B = F32((C - ((b - 1.0) * sigma + a * th) / c) / th2)
    p1 = np.cross(phi, tau).astype(F32)
    p2 = np.cross(phi, p1).astype(F32)
    t = (C * tau + A * p1 + B * p2).astype(F32)
    return np.concatenate([t, q, [scale]]).astype(F32)


def retr(T, xi):
    return mul(exp_sim3(xi)[None], T)


# -------------------------------------------------------------- geometry --
def skew(x):
    o = np.zeros_like(x[..., 0])
    X, Y, Z = x[..., 0], x[..., 1], x[..., 2]
    return np.stack([o, -Z, Y, Z, o, -X, -Y, X, o], -1).reshape(*x.shape[:-1], 3, 3)


def point_to_ray_dist(X, jacobian=False):
    d = np.linalg.norm(X, axis=-1, keepdims=True).astype(F32)
    d_inv = (F32(1.0) / d).astype(F32)
    r = d_inv * X
    rd = np.concatenate([r, d], -1)
    if not jacobian:
        return rd
    d_inv_2 = d_inv**2
    I = np.broadcast_to(np.eye(3, dtype=F32), X.shape[:-1] + (3, 3))
    dr_dX = d_inv[..., None] * (I - d_inv_2[..., None] * (X[..., :, None] @ X[..., None, :]))
    dd_dX = r[..., None, :]
    return rd, np.concatenate([dr_dX, dd_dX], -2).astype(F32)


def act_sim3_jac(T, X):
    pW = act(T, X)
    I = np.broadcast_to(np.eye(3, dtype=F32), pW.shape[:-1] + (3, 3))
    J = np.concatenate([I, -skew(pW), pW[..., None]], -1)
    return pW, J.astype(F32)


def project_calib(P, K, img_size, border, z_eps):
    p = (P @ K.T).astype(F32)
    p = p / p[..., 2:3]
    p = p[..., :2]
    u, v = p[..., 0:1], p[..., 1:2]
    x, y, z = P[..., 0:1], P[..., 1:2], P[..., 2:3]
    valid = (u > border) & (u < img_size[1] - 1 - border)
    valid &= (v > border) & (v < img_size[0] - 1 - border)
    valid_z = z > z_eps
    valid &= valid_z
    with np.errstate(divide="ignore", invalid="ignore"):
        logz = np.log(z)
    logz = np.where(valid_z, logz, F32(0.0))
    pz = np.concatenate([p, logz], -1).astype(F32)
    fx, fy = K[0, 0], K[1, 1]
    with np.errstate(divide="ignore", invalid="ignore"):
        z_inv = F32(1.0) / z[..., 0]
    J = np.zeros(P.shape[:-1] + (3, 3), F32)
    J[..., 0, 0] = fx
    J[..., 1, 1] = fy
    J[..., 0, 2] = -fx * x[..., 0] * z_inv
    J[..., 1, 2] = -fy * y[..., 0] * z_inv
    J *= z_inv[..., None, None]
    J[..., 2, 2] = z_inv
    return pz, J, valid


def huber(r, k):
    a = np.abs(r)
    with np.errstate(divide="ignore"):
        return np.where(a < k, F32(1.0), (F32(k) / a)).astype(F32)


# ------------------------------------------------------------------ solve --
def solve(sqrt_info, r, J, k):
    whitened = sqrt_info * r
    robust = sqrt_info * np.sqrt(huber(whitened, k))
    A = (robust[..., None] * J).reshape(-1, J.shape[-1]).astype(F32)
    b = (robust * r).reshape(-1, 1).astype(F32)
    H = A.T @ A
    g = -A.T @ b
    cost = 0.5 * float((b.T @ b)[0, 0])
    try:
        L = np.linalg.cholesky(H)
    except np.linalg.LinAlgError as e:
        raise CholeskyFailed(str(e))
    y = np.linalg.solve(L, g)
    tau = np.linalg.solve(L.T, y).reshape(1, -1).astype(F32)
    solve.last_gscale = (np.abs(A).astype(np.float64).T @ np.abs(b).astype(np.float64))[:, 0]
    return tau, cost, H, g


def converged(rel_thresh, delta_thresh, old_cost, new_cost, tau):
    diff = old_cost - new_cost
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = math.fabs(diff / old_cost) if old_cost != float("inf") else float("nan")
    return rel < rel_thresh or float(np.linalg.norm(tau)) < delta_thresh


def track_rays(Xf, Xk, T_WCf, T_WCk, Qk, valid, cfg, record=None):
    """opt_pose_ray_dist_sim3 (tracker.py:173-214). Returns (T_WCf, T_CkCf, iters)."""
    valid = valid.astype(F32)
    si_r = F32(1.0 / cfg["sigma_ray"]) * valid * np.sqrt(Qk)
    si_d = F32(1.0 / cfg["sigma_dist"]) * valid * np.sqrt(Qk)
    sqrt_info = np.concatenate([np.repeat(si_r, 3, 1), si_d], 1).astype(F32)
    T = mul(inv(T_WCk), T_WCf)
    rd_k = point_to_ray_dist(Xk)
    old = float("inf")
    it = 0
    for step in range(cfg["max_iters"]):
        it = step + 1
        Xf_Ck, dX = act_sim3_jac(T, Xf)
        rd_f, drd = point_to_ray_dist(Xf_Ck, True)
        r = rd_k - rd_f
        J = -(drd @ dX)
        tau, cost, H, g = solve(sqrt_info, r, J, cfg["huber"])
        if record is not None:
            record.append(dict(tau=tau, cost=cost, H=H, g=g, gscale=solve.last_gscale))
        T = retr(T, tau)
        if converged(cfg["rel_error"], cfg["delta_norm"], old, cost, tau):
            break
        old = cost
    return mul(T_WCk, T), T, it


def calib_meas(Xk, img_size, depth_eps):
    """meas_k / valid_meas_k of get_points_poses (tracker.py:146-152)."""
    h, w = img_size
    v, u = np.meshgrid(np.arange(h, dtype=F32), np.arange(w, dtype=F32), indexing="ij")
    uv = np.stack([u.reshape(-1), v.reshape(-1)], -1)
    with np.errstate(divide="ignore", invalid="ignore"):
        logz = np.log(Xk[..., 2:3])
    meas = np.concatenate([uv, logz], -1).astype(F32)
    valid = Xk[..., 2:3] > depth_eps
    meas[~np.repeat(valid, 3, 1)] = 0.0
    return meas, valid


def constrain_points_to_ray(img_size, X, K):
    """geometry.py:37-42 + backproject :107-115 for one pointmap [HW,3]."""
    h, w = img_size
    v, u = np.meshgrid(np.arange(h, dtype=F32), np.arange(w, dtype=F32), indexing="ij")
    x = (u.reshape(-1) - K[0, 2]) / K[0, 0]
    y = (v.reshape(-1) - K[1, 2]) / K[1, 1]
    z = X[..., 2]
    return np.stack([z * x, z * y, z], -1).astype(F32)


def track_calib(Xf, Xk, T_WCf, T_WCk, Qk, valid, meas_k, valid_meas_k, K, img_size, cfg, record=None):
    """opt_pose_calib_sim3 (tracker.py:216-266). Xf/Xk already ray-constrained."""
    valid = valid.astype(F32)
    si_p = F32(1.0 / cfg["sigma_pixel"]) * valid * np.sqrt(Qk)
    si_z = F32(1.0 / cfg["sigma_depth"]) * valid * np.sqrt(Qk)
    sqrt_info = np.concatenate([np.repeat(si_p, 2, 1), si_z], 1).astype(F32)
    T = mul(inv(T_WCk), T_WCf)
    old = float("inf")
    it = 0
    for step in range(cfg["max_iters"]):
        it = step + 1
        Xf_Ck, dX = act_sim3_jac(T, Xf)
        pz, dpz, vproj = project_calib(Xf_Ck, K, img_size, cfg["pixel_border"], cfg["depth_eps"])
        si2 = (vproj & valid_meas_k).astype(F32) * sqrt_info
        r = meas_k - pz
        J = -(dpz @ dX)
        with np.errstate(invalid="ignore"):
            tau, cost, H, g = solve(si2, r, J, cfg["huber"])
        if record is not None:
            record.append(dict(tau=tau, cost=cost, H=H, g=g, gscale=solve.last_gscale))
        T = retr(T, tau)
        if converged(cfg["rel_error"], cfg["delta_norm"], old, cost, tau):
            break
        old = cost
    return mul(T_WCk, T), T, it


TRACKING_CFG = dict(  # config/base.yaml:16-33
    max_iters=50, C_conf=0.0, Q_conf=1.5, rel_error=1e-3, delta_norm=1e-3, huber=1.345,
    sigma_ray=0.003, sigma_dist=10.0, sigma_pixel=1.0, sigma_depth=10.0, pixel_border=-10,
    depth_eps=1e-6,
)
LOCAL_OPT_CFG = dict(  # config/base.yaml:35-50
    pin=1, C_conf=0.0, Q_conf=1.5, pixel_border=-10, depth_eps=1e-6, max_iters=10,
    sigma_ray=0.003, sigma_dist=10.0, sigma_pixel=1.0, sigma_depth=10.0, sigma_point=0.05,
    delta_norm=1e-8,
)
