"""Host-side mirror of the reference tracker's pose refinement
(FrameTracker.opt_pose_ray_dist_sim3 / opt_pose_calib_sim3, tracker.py:173-266)
on top of the HIP entry points ``mast3r_slam_backends.track_rays_sim3`` /
``track_calib_sim3``.

Same arguments and return values as the reference methods: poses in and out
are Sim3 objects (``mast3r_slam_amd.sim3.Sim3``, the lietorch subset the
reference uses; ``.data`` is the same [..., 8] layout), results are
``(T_WCf, T_CkCf)``. A failed Cholesky raises ``torch.linalg.LinAlgError``
like the reference's ``torch.linalg.cholesky`` (tracker.py:167, caught at
:91-93). The whole GN loop — residuals, Huber whitening, 7x7 normal equations,
fp64 Cholesky, retraction and the reference's convergence rule
(nonlinear_optimizer.py:5-25) — runs on the device; the host reads the
convergence flag every ``sync_every`` iterations only.
"""
from __future__ import annotations

import torch

import mast3r_slam_backends as be

from .sim3 import Sim3

# config/base.yaml:16-31
TRACKING_CFG = dict(max_iters=50, rel_error=1e-3, delta_norm=1e-3, huber=1.345, sigma_ray=0.003,
                    sigma_dist=1e1, sigma_pixel=1.0, sigma_depth=1e1, pixel_border=-10,
                    depth_eps=1e-6)


def _flat_pose(T) -> torch.Tensor:
    d = T.data if hasattr(T, "data") else T
    return d.reshape(-1, 8)[0].contiguous()


def _result(T_f, T_r, info):
    if int(info[be.INFO_SOLVE_FAIL]):
        raise torch.linalg.LinAlgError("tracker: Cholesky of the 7x7 normal equations failed")
    return Sim3(T_f), Sim3(T_r)


def opt_pose_ray_dist_sim3(Xf, Xk, T_WCf, T_WCk, Qk, valid, cfg=TRACKING_CFG, sync_every=5):
    """tracker.py:173-214. Xf [HW,3] (gathered by idx_f2k), Xk [HW,3], Qk [HW,1],
    valid [HW,1] bool; T_WCf / T_WCk Sim3 -> (T_WCf, T_CkCf)."""
    T_f, T_r, info = be.track_rays_sim3(
        Xf.contiguous(), Xk.contiguous(), _flat_pose(T_WCf), _flat_pose(T_WCk), Qk.contiguous(),
        valid.contiguous(), cfg["sigma_ray"], cfg["sigma_dist"], cfg["huber"], cfg["max_iters"],
        cfg["rel_error"], cfg["delta_norm"], sync_every=sync_every)
    return _result(T_f, T_r, info)


def opt_pose_calib_sim3(Xf, Xk, T_WCf, T_WCk, Qk, valid, meas_k, valid_meas_k, K, img_size,
                        cfg=TRACKING_CFG, sync_every=5):
    """tracker.py:216-266. Xf / Xk ray-constrained as get_points_poses leaves
    them (tracker.py:142-144); meas_k / valid_meas_k are formed on the device
    from the pixel grid and Xk exactly as get_points_poses does (:146-152), so
    the arguments are accepted for signature parity and not read."""
    del meas_k, valid_meas_k
    T_f, T_r, info = be.track_calib_sim3(
        Xf.contiguous(), Xk.contiguous(), _flat_pose(T_WCf), _flat_pose(T_WCk), Qk.contiguous(),
        valid.contiguous(), K.contiguous(), img_size, cfg["sigma_pixel"], cfg["sigma_depth"],
        cfg["huber"], cfg["max_iters"], cfg["rel_error"], cfg["delta_norm"], cfg["pixel_border"],
        cfg["depth_eps"], sync_every=sync_every)
    return _result(T_f, T_r, info)
