"""Generate golden fixtures by running the REFERENCE's own tracker GN code.

Run in the development container only (``/root/reference`` does not exist on
the GPU box); the resulting ``*.npz`` files are committed and are pure data:
inputs (synthetic pointmaps, poses, confidences) and the outputs the reference
code produced from them.

What executes here is the reference's
``mast3r_slam/tracker.py`` (``FrameTracker.opt_pose_ray_dist_sim3`` :173-214,
``opt_pose_calib_sim3`` :216-266, ``solve`` :156-171, ``get_points_poses``
:129-154), ``mast3r_slam/geometry.py`` and ``mast3r_slam/nonlinear_optimizer.py``
with the parameters of ``config/base.yaml``. Three modules the reference imports
are absent offline and are replaced by stand-ins that are NOT on the GN path:

* ``lietorch``              -> this build's ``mast3r_slam_amd.sim3.Sim3``
                               (third-party group arithmetic; parity unpinned,
                               restated from gn_kernels.cu:172-413)
* ``mast3r_slam.mast3r_utils`` -> stub (network inference; never called)
* ``mast3r_slam_backends``  -> stub (the CUDA extension; never called)

Usage: ``python tests/golden/make_golden.py`` (writes tests/golden/*.npz)
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "mast3r-slam-ysh_amd"))

from mast3r_slam_amd.sim3 import Sim3  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402


def install_shims():
    lt = types.ModuleType("lietorch")
    lt.Sim3 = Sim3
    lt.SE3 = type("SE3", (), {})
    sys.modules["lietorch"] = lt
    mu = types.ModuleType("mast3r_slam.mast3r_utils")

    def _absent(*a, **k):
        raise RuntimeError("MASt3R network is not part of the GN oracle")

    mu.mast3r_match_asymmetric = _absent
    mu.mast3r_match_symmetric = _absent
    mu.resize_img = _absent
    sys.modules["mast3r_slam.mast3r_utils"] = mu
    be = types.ModuleType("mast3r_slam_backends")
    sys.modules["mast3r_slam_backends"] = be
    sys.path.insert(0, REF)


class Recorder:
    """Wraps FrameTracker.solve to capture per-iteration H, g, tau, cost."""

    def __init__(self, tracker):
        self.tracker = tracker
        self.orig = tracker.solve
        self.rec = []
        tracker.solve = self

    def __call__(self, sqrt_info, r, J):
        whitened_r = sqrt_info * r
        from mast3r_slam.nonlinear_optimizer import huber

        robust = sqrt_info * torch.sqrt(huber(whitened_r, k=self.tracker.cfg["huber"]))
        A = (robust[..., None] * J).view(-1, J.shape[-1])
        b = (robust * r).view(-1, 1)
        H = (A.T @ A).double().numpy()
        g = (-A.T @ b).double().numpy()[:, 0]
        try:
            tau, cost = self.orig(sqrt_info, r, J)
        except Exception:
            self.rec.append(dict(H=H, g=g, tau=np.full(7, np.nan), cost=np.nan, failed=True))
            raise
        self.rec.append(dict(H=H, g=g, tau=tau.double().numpy()[0], cost=cost, failed=False))
        return tau, cost


def run_case(name, calib, H, W, seed, identity_idx=False, max_iters=None, kill_valid=False):
    from mast3r_slam.config import config, load_config
    from mast3r_slam.frame import Frame
    from mast3r_slam.tracker import FrameTracker

    load_config(os.path.join(REF, "config", "base.yaml"))
    config["use_calib"] = bool(calib)
    tr = FrameTracker(model=None, frames=None, device="cpu")
    if max_iters is not None:
        tr.cfg = dict(tr.cfg)
        tr.cfg["max_iters"] = max_iters
    torch.manual_seed(0)
    p = synthetic.make_pair(H, W, seed=seed, identity_idx=identity_idx)
    if kill_valid:
        p.valid[:] = False

    # Frame stand-ins carry exactly what get_points_poses reads.
    img = torch.zeros(3, H, W)
    fr = Frame(1, img, None, None, None, p.T_WCf_init, X_canon=None, C=None, N=1)
    kf = Frame(0, img, None, None, None, p.T_WCk, X_canon=p.Xk.clone(), C=p.Ck.clone(), N=1)
    # the frame's un-gathered pointmap: our pair stores Xf already gathered, so
    # pass identity idx to get_points_poses with the gathered map as X_canon
    fr.X_canon = p.Xf.clone()
    fr.C = p.Cf.clone()
    idx = torch.arange(H * W)
    K = p.K if calib else None
    Xf, Xk, T_WCf, T_WCk, Cf, Ck, meas_k, valid_meas_k = tr.get_points_poses(
        fr, kf, idx, (H, W), calib, K
    )
    rec = Recorder(tr)
    failed = False
    try:
        if not calib:
            T_WCf_out, T_CkCf = tr.opt_pose_ray_dist_sim3(Xf, Xk, T_WCf, T_WCk, p.Qk, p.valid)
        else:
            T_WCf_out, T_CkCf = tr.opt_pose_calib_sim3(
                Xf, Xk, T_WCf, T_WCk, p.Qk, p.valid, meas_k, valid_meas_k, K, (H, W)
            )
        T_WCf_np = T_WCf_out.data.numpy().astype(np.float32)
        T_CkCf_np = T_CkCf.data.numpy().astype(np.float32)
    except Exception:
        failed = True
        T_WCf_np = np.full((1, 8), np.nan, np.float32)
        T_CkCf_np = np.full((1, 8), np.nan, np.float32)

    out = dict(
        calib=np.int32(calib),
        H=np.int32(H),
        W=np.int32(W),
        K=p.K.numpy(),
        Xf_raw=p.Xf.numpy(),
        Xk_raw=p.Xk.numpy(),
        Xf=Xf.numpy(),
        Xk=Xk.numpy(),
        Qk=p.Qk.numpy(),
        valid=p.valid.numpy(),
        T_WCk=p.T_WCk.data.numpy(),
        T_WCf_init=p.T_WCf_init.data.numpy(),
        T_WCf=T_WCf_np,
        T_CkCf=T_CkCf_np,
        failed=np.int32(failed),
        n_iters=np.int32(len(rec.rec)),
        H_iter=np.stack([r["H"] for r in rec.rec]),
        g_iter=np.stack([r["g"] for r in rec.rec]),
        tau_iter=np.stack([r["tau"] for r in rec.rec]),
        cost_iter=np.array([r["cost"] for r in rec.rec]),
        max_iters=np.int32(tr.cfg["max_iters"]),
        sigma_ray=np.float32(tr.cfg["sigma_ray"]),
        sigma_dist=np.float32(tr.cfg["sigma_dist"]),
        sigma_pixel=np.float32(tr.cfg["sigma_pixel"]),
        sigma_depth=np.float32(tr.cfg["sigma_depth"]),
        pixel_border=np.int32(tr.cfg["pixel_border"]),
        depth_eps=np.float32(tr.cfg["depth_eps"]),
        rel_error=np.float32(tr.cfg["rel_error"]),
        delta_norm=np.float32(tr.cfg["delta_norm"]),
        huber=np.float32(tr.cfg["huber"]),
    )
    if calib:
        out["meas_k"] = meas_k.numpy()
        out["valid_meas_k"] = valid_meas_k.numpy()
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: iters={len(rec.rec)} failed={failed} -> {os.path.relpath(path, REPO)}")


def main():
    install_shims()
    torch.set_num_threads(8)
    run_case("tracker_rays_64x48", calib=False, H=48, W=64, seed=1001)
    run_case("tracker_calib_64x48", calib=True, H=48, W=64, seed=1002)
    run_case("tracker_rays_identity_64x48", calib=False, H=48, W=64, seed=1011, identity_idx=True)
    run_case("tracker_calib_identity_64x48", calib=True, H=48, W=64, seed=1012, identity_idx=True)
    # one-step cases pin the backend kernels through the tracker<->backend
    # equivalence
    run_case("onestep_rays_identity_32x24", calib=False, H=24, W=32, seed=1021, identity_idx=True, max_iters=1)
    run_case("onestep_calib_identity_32x24", calib=True, H=24, W=32, seed=1022, identity_idx=True, max_iters=1)
    # edge case: nothing valid -> H = 0 -> Cholesky raises -> track failure
    run_case("tracker_rays_allinvalid_32x24", calib=False, H=24, W=32, seed=1031, kill_valid=True)


if __name__ == "__main__":
    main()
