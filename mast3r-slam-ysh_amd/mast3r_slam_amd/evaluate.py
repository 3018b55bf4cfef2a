"""Trajectory error (ATE) of keyframe poses — the parity figure the north star
quotes ("pose ATE delta < 1e-5 m").

The reference writes keyframe poses as SE(3) TUM lines (``evaluate.py:23-44``:
``as_SE3(T_WC)`` keeps ``t`` and ``q``, drops the scale) and scores them with
``evo_ape tum <gt> <est> -as`` (``scripts/eval_tum.sh:48-50``): the estimate's
positions are aligned to the ground truth by the Umeyama least-squares Sim(3)
(``-a`` align, ``-s`` correct scale) and the APE of the translation part is
reported as an RMSE. ``evo`` is not installed here; this restates its
published algorithm (Umeyama 1991, eqs. 38-42) in numpy fp64. No reference
test pins it ("parity unpinned" for the evo restatement itself); what the
tests compare is the ATE of the HIP backend's poses against the ATE of the
oracle's poses on the same synthetic graph, both through this function.

Host-side evaluation only: nothing here is on the GN hot path.
"""
from __future__ import annotations

import numpy as np


def positions(Twc) -> np.ndarray:
    """``[N,8]`` lietorch Sim3 data (t, q_xyzw, s) -> ``[N,3]`` camera centres
    as written by ``save_traj`` (``evaluate.py:40-44``)."""
    T = np.asarray(Twc.cpu() if hasattr(Twc, "cpu") else Twc, dtype=np.float64)
    return T.reshape(-1, 8)[:, :3].copy()


def umeyama_sim3(src: np.ndarray, dst: np.ndarray):
    """Least-squares ``s, R, t`` minimising ``sum ||dst - (s R src + t)||^2``
    (Umeyama 1991; what ``evo``'s ``align(correct_scale=True)`` computes).
    ``src, dst``: ``[N,3]``. Returns ``(s, R [3,3], t [3])``."""
    src = np.asarray(src, np.float64)
    dst = np.asarray(dst, np.float64)
    if src.shape != dst.shape or src.ndim != 2 or src.shape[1] != 3:
        raise ValueError("umeyama_sim3: src and dst must both be [N,3]")
    n = src.shape[0]
    if n < 3:
        raise ValueError("umeyama_sim3: need at least 3 positions")
    mu_s, mu_d = src.mean(0), dst.mean(0)
    xs, xd = src - mu_s, dst - mu_d
    var_s = (xs * xs).sum() / n
    cov = xd.T @ xs / n
    U, D, Vt = np.linalg.svd(cov)
    S = np.eye(3)
    if np.linalg.det(U) * np.linalg.det(Vt) < 0:
        S[2, 2] = -1.0
    R = U @ S @ Vt
    s = float(np.trace(np.diag(D) @ S) / var_s) if var_s > 0 else 1.0
    t = mu_d - s * R @ mu_s
    return s, R, t


def ate_rmse(est_Twc, gt_Twc, correct_scale: bool = True) -> float:
    """APE RMSE (metres) of the translation part after Umeyama alignment of the
    estimate onto the ground truth (``evo_ape tum gt est -as``)."""
    pe, pg = positions(est_Twc), positions(gt_Twc)
    if correct_scale:
        s, R, t = umeyama_sim3(pe, pg)
    else:
        _, R, t = umeyama_sim3(pe, pg)
        s = 1.0
        t = pg.mean(0) - R @ pe.mean(0)
    aligned = (s * (R @ pe.T)).T + t
    return float(np.sqrt(((aligned - pg) ** 2).sum(1).mean()))
