"""PyTorch-CPU restatement of the reference's tracker Gauss-Newton — the
reference's own CPU/PyTorch path, op for op.

TEST INFRASTRUCTURE ONLY: the tracker leg of bench.py's cpu_baseline (timed on
all host cores) and a checker in tests/. The product
path never imports it. It runs the same torch tensor program the reference
runs (materialised [HW,3,7] / [HW,4,3] / [4HW,7] intermediates, a GEMM for
H = A^T A, fp32 Cholesky, one .item() per iteration), so its time is what the
reference's tracker costs on these cores:

* ``opt_pose_ray_dist_sim3``  tracker.py:173-214
* ``opt_pose_calib_sim3``     tracker.py:216-266
* ``solve``                   tracker.py:156-171
* ``point_to_ray_dist`` / ``act_Sim3`` / ``project_calib`` / ``skew_sym``
                              geometry.py:5-34, 45-52, 63-104
* ``huber`` / ``check_convergence``  nonlinear_optimizer.py:5-33

Group arithmetic: mast3r_slam_amd.sim3 (the lietorch restatement, pinned by
tests/test_sim3_math.py). Pinned against tests/golden/tracker_*.npz
(tests/test_oracle_golden.py::test_torch_tracker_matches_reference_tracker).
"""
from __future__ import annotations

import math

import torch

from mast3r_slam_amd.sim3 import Sim3


def skew_sym(x):  # geometry.py:5-9
    b = x.shape[:-1]
    x, y, z = x.unbind(dim=-1)
    o = torch.zeros_like(x)
    return torch.stack([o, -z, y, z, o, -x, -y, x, o], dim=-1).view(*b, 3, 3)


def point_to_ray_dist(X, jacobian=False):  # geometry.py:17-34
    b = X.shape[:-1]
    d = torch.linalg.norm(X, dim=-1, keepdim=True)
    d_inv = 1.0 / d
    r = d_inv * X
    rd = torch.cat((r, d), dim=-1)
    if not jacobian:
        return rd
    d_inv_2 = d_inv ** 2
    I = torch.eye(3, dtype=X.dtype).repeat(*b, 1, 1)
    dr_dX = d_inv.unsqueeze(-1) * (I - d_inv_2.unsqueeze(-1) * (X.unsqueeze(-1) @ X.unsqueeze(-2)))
    dd_dX = r.unsqueeze(-2)
    return rd, torch.cat((dr_dX, dd_dX), dim=-2)


def act_Sim3(T: Sim3, pC, jacobian=False):  # geometry.py:45-52
    pW = T.act(pC)
    if not jacobian:
        return pW
    dpC_dt = torch.eye(3).repeat(*pW.shape[:-1], 1, 1)
    dpC_dR = -skew_sym(pW)
    dpc_ds = pW.reshape(*pW.shape[:-1], -1, 1)
    return pW, torch.cat([dpC_dt, dpC_dR, dpc_ds], dim=-1)


def project_calib(P, K, img_size, border=0, z_eps=0.0):  # geometry.py:63-104 (jacobian=True)
    b = P.shape[:-1]
    K_rep = K.repeat(*b, 1, 1)
    p = (K_rep @ P[..., None]).squeeze(-1)
    p = p / p[..., 2:3]
    p = p[..., :2]
    u, v = p.split([1, 1], dim=-1)
    x, y, z = P.split([1, 1, 1], dim=-1)
    valid = (u > border) & (u < img_size[1] - 1 - border) & (v > border) & (v < img_size[0] - 1 - border)
    valid_z = z > z_eps
    valid = valid & valid_z
    logz = torch.log(z)
    logz[torch.logical_not(valid_z)] = 0.0
    pz = torch.cat((p, logz), dim=-1)
    fx, fy = K[0, 0], K[1, 1]
    z_inv = 1.0 / z[..., 0]
    dpz_dP = torch.zeros(*b + (3, 3), dtype=P.dtype)
    dpz_dP[..., 0, 0] = fx
    dpz_dP[..., 1, 1] = fy
    dpz_dP[..., 0, 2] = -fx * x[..., 0] * z_inv
    dpz_dP[..., 1, 2] = -fy * y[..., 0] * z_inv
    dpz_dP *= z_inv[..., None, None]
    dpz_dP[..., 2, 2] = z_inv
    return pz, dpz_dP, valid


def huber(r, k=1.345):  # nonlinear_optimizer.py:28-33
    unit = torch.ones((1), dtype=r.dtype)
    r_abs = torch.abs(r)
    mask = r_abs < k
    w = torch.where(mask, unit, k / r_abs)
    return w


def check_convergence(iter, rel_error_threshold, delta_norm_threshold, old_cost, new_cost, delta):
    # nonlinear_optimizer.py:5-25
    cost_diff = old_cost - new_cost
    rel_dec = math.fabs(cost_diff / old_cost) if old_cost != float("inf") else float("nan")
    delta_norm = torch.linalg.norm(delta)
    return rel_dec < rel_error_threshold or delta_norm < delta_norm_threshold


def solve(cfg, sqrt_info, r, J):  # tracker.py:156-171
    whitened_r = sqrt_info * r
    robust_sqrt_info = sqrt_info * torch.sqrt(huber(whitened_r, k=cfg["huber"]))
    mdim = J.shape[-1]
    A = (robust_sqrt_info[..., None] * J).view(-1, mdim)
    b = (robust_sqrt_info * r).view(-1, 1)
    H = A.T @ A
    g = -A.T @ b
    cost = 0.5 * (b.T @ b).item()
    L = torch.linalg.cholesky(H, upper=False)
    tau_j = torch.cholesky_solve(g, L, upper=False).view(1, -1)
    return tau_j, cost


def track_rays(Xf, Xk, T_WCf, T_WCk, Qk, valid, cfg):
    """opt_pose_ray_dist_sim3 (tracker.py:173-214). torch CPU float32
    tensors; T_* as [1, 8] data. Returns (T_WCf, T_CkCf, iters)."""
    T_WCf, T_WCk = Sim3(T_WCf), Sim3(T_WCk)
    sqrt_info_ray = 1 / cfg["sigma_ray"] * valid * torch.sqrt(Qk)
    sqrt_info_dist = 1 / cfg["sigma_dist"] * valid * torch.sqrt(Qk)
    sqrt_info = torch.cat((sqrt_info_ray.repeat(1, 3), sqrt_info_dist), dim=1)
    T_CkCf = T_WCk.inv() * T_WCf
    rd_k = point_to_ray_dist(Xk, jacobian=False)
    old_cost = float("inf")
    it = 0
    for step in range(cfg["max_iters"]):
        it = step + 1
        Xf_Ck, dXf_Ck_dT_CkCf = act_Sim3(T_CkCf, Xf, jacobian=True)
        rd_f_Ck, drd_f_Ck_dXf_Ck = point_to_ray_dist(Xf_Ck, jacobian=True)
        r = rd_k - rd_f_Ck
        J = -drd_f_Ck_dXf_Ck @ dXf_Ck_dT_CkCf
        tau, new_cost = solve(cfg, sqrt_info, r, J)
        T_CkCf = T_CkCf.retr(tau)
        if check_convergence(step, cfg["rel_error"], cfg["delta_norm"], old_cost, new_cost, tau):
            break
        old_cost = new_cost
    return (T_WCk * T_CkCf).data, T_CkCf.data, it


def track_calib(Xf, Xk, T_WCf, T_WCk, Qk, valid, meas_k, valid_meas_k, K, img_size, cfg):
    """opt_pose_calib_sim3 (tracker.py:216-266)."""
    T_WCf, T_WCk = Sim3(T_WCf), Sim3(T_WCk)
    sqrt_info_pixel = 1 / cfg["sigma_pixel"] * valid * torch.sqrt(Qk)
    sqrt_info_depth = 1 / cfg["sigma_depth"] * valid * torch.sqrt(Qk)
    sqrt_info = torch.cat((sqrt_info_pixel.repeat(1, 2), sqrt_info_depth), dim=1)
    T_CkCf = T_WCk.inv() * T_WCf
    old_cost = float("inf")
    it = 0
    for step in range(cfg["max_iters"]):
        it = step + 1
        Xf_Ck, dXf_Ck_dT_CkCf = act_Sim3(T_CkCf, Xf, jacobian=True)
        pzf_Ck, dpzf_Ck_dXf_Ck, valid_proj = project_calib(Xf_Ck, K, img_size, border=cfg["pixel_border"],
                                                            z_eps=cfg["depth_eps"])
        valid2 = valid_proj & valid_meas_k
        sqrt_info2 = valid2 * sqrt_info
        r = meas_k - pzf_Ck
        J = -dpzf_Ck_dXf_Ck @ dXf_Ck_dT_CkCf
        tau, new_cost = solve(cfg, sqrt_info2, r, J)
        T_CkCf = T_CkCf.retr(tau)
        if check_convergence(step, cfg["rel_error"], cfg["delta_norm"], old_cost, new_cost, tau):
            break
        old_cost = new_cost
    return (T_WCk * T_CkCf).data, T_CkCf.data, it
