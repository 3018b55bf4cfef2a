"""GPU parity of the kernels either side of the GN/matching path
(SURVEY §8f #2, #4): keyframe pointmap fusion (m3s_fuse_pointmap) and the
iter_proj input prep (m3s_prep_rays), against oracle/fusion_oracle.py (the
reference's torch expressions on CPU / their numpy restatement).

Tolerances: the fused filter is elementwise fp32 in the reference's operation
order, compared to 1 ulp-scale (rtol 1e-6); with a Sim3 applied first the
lietorch act differs by FMA contraction (atol 1e-6 relative to the scene
scale). Ray prep: unit rays to 1e-6, Scharr gradients to 1e-6 (torch's conv
sums the 9 taps in its own order).
"""
import numpy as np
import pytest
import torch

import mast3r_slam_backends as be
from mast3r_slam_amd import frame, synthetic
from mast3r_slam_amd.sim3 import Sim3
from oracle import fusion_oracle as fo

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _pair(H=48, W=64, seed=7):
    g = torch.Generator().manual_seed(seed)
    Xc = torch.randn(H * W, 3, generator=g) + torch.tensor([0.0, 0.0, 3.0])
    C = 1.0 + torch.rand(H * W, 1, generator=g) * 5
    Xn = Xc + 0.01 * torch.randn(H * W, 3, generator=g)
    Cn = 1.0 + torch.rand(H * W, 1, generator=g) * 5
    return Xc, C, Xn, Cn


@pytest.mark.parametrize("mode", ["weighted_pointmap", "indep_conf", "recent", "weighted_spherical"])
@pytest.mark.parametrize("with_T", [False, True])
def test_fuse_pointmap_matches_oracle(mode, with_T):
    Xc, C, Xn, Cn = _pair()
    T = None
    if with_T:
        xi = torch.tensor([[0.02, -0.01, 0.03, 0.01, -0.02, 0.015, 0.01]])
        T = Sim3.exp(xi).data[0]
    ref_X, ref_C = fo.fuse_pointmap(Xc.numpy(), C.numpy(), Xn.numpy(), Cn.numpy(),
                                    None if T is None else T.numpy(), mode)
    Xd, Cd = Xc.to(DEV), C.to(DEV)
    be.fuse_pointmap(Xd, Cd, Xn.to(DEV), Cn.to(DEV), None if T is None else T.to(DEV), mode)
    tol = dict(rtol=1e-6, atol=1e-6 if with_T else 0.0)
    if mode == "weighted_spherical":
        # atan2 / acos / sin / cos: device libm vs torch's CPU kernels differ
        # by a few ulp, and acos(z / r) amplifies an input ulp by 1/sin(theta)
        # (the T.act input differs by ulps too): 1e-4 absolute on ~3 m points
        tol = dict(rtol=2e-5, atol=1e-4)
    np.testing.assert_allclose(Xd.cpu().numpy(), ref_X, **tol)
    np.testing.assert_allclose(Cd.cpu().numpy(), ref_C, rtol=1e-6)


def test_pointmap_mirror_counts_and_modes():
    """Frame.update_pointmap bookkeeping (N, N_updates, first / best_score)."""
    Xc, C, Xn, Cn = _pair(8, 8)
    pm = frame.Pointmap("weighted_pointmap")
    pm.update_pointmap(Xc.to(DEV), C.to(DEV))
    assert pm.N == 1 and torch.equal(pm.X_canon.cpu(), Xc)
    pm.update_pointmap(Xn.to(DEV), Cn.to(DEV))
    assert pm.N == 2 and pm.N_updates == 2
    ref_X, ref_C = fo.fuse_pointmap(Xc.numpy(), C.numpy(), Xn.numpy(), Cn.numpy())
    np.testing.assert_allclose(pm.X_canon.cpu().numpy(), ref_X, rtol=1e-6)
    np.testing.assert_allclose(pm.get_average_conf().cpu().numpy(), ref_C / 2, rtol=1e-6)
    # "first" (frame.py:55-58): the update after the initialisation replaces
    # it (N_updates == 1 then), later ones are ignored
    first = frame.Pointmap("first")
    first.update_pointmap(Xc.to(DEV), C.to(DEV))
    first.update_pointmap(Xn.to(DEV), Cn.to(DEV))
    first.update_pointmap(Xc.to(DEV), C.to(DEV))
    assert torch.equal(first.X_canon.cpu(), Xn) and first.N_updates == 3
    sph = frame.Pointmap("weighted_spherical")
    sph.update_pointmap(Xc.to(DEV), C.to(DEV))
    sph.update_pointmap(Xn.to(DEV), Cn.to(DEV))
    assert sph.N == 2 and sph.N_updates == 2
    ref_X, ref_C = fo.fuse_pointmap(Xc.numpy(), C.numpy(), Xn.numpy(), Cn.numpy(), mode="weighted_spherical")
    np.testing.assert_allclose(sph.X_canon.cpu().numpy(), ref_X, rtol=2e-5, atol=2e-5)


def test_fuse_tracked_points_applies_pose():
    Xc, C, Xn, Cn = _pair(16, 16)
    xi = torch.tensor([[0.05, 0.0, -0.02, 0.0, 0.03, 0.0, -0.01]])
    T = Sim3.exp(xi)
    kf = frame.Pointmap()
    kf.update_pointmap(Xc.to(DEV), C.to(DEV))
    frame.fuse_tracked_points(kf, Sim3(T.data.to(DEV)), Xn.to(DEV), Cn.to(DEV))
    ref_X, _ = fo.fuse_pointmap(Xc.numpy(), C.numpy(), Xn.numpy(), Cn.numpy(), T.data.numpy())
    np.testing.assert_allclose(kf.X_canon.cpu().numpy(), ref_X, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("H,W,B", [(48, 64, 1), (17, 23, 2), (2, 2, 1)])
def test_prep_rays_matches_reference_expressions(H, W, B):
    m = synthetic.make_match_inputs(max(H, 3), max(W, 3))
    g = torch.Generator().manual_seed(3)
    X11 = (torch.randn(B, H, W, 3, generator=g) + torch.tensor([0.0, 0.0, 2.0])).contiguous()
    X21 = (torch.randn(B, H, W, 3, generator=g) + torch.tensor([0.0, 0.0, 2.0])).contiguous()
    ref_img, ref_pts = fo.prep_rays(X11.numpy(), X21.numpy())
    img, pts = be.prep_rays(X11.to(DEV), X21.to(DEV))
    np.testing.assert_allclose(img.cpu().numpy(), ref_img, atol=1e-6)
    np.testing.assert_allclose(pts.cpu().numpy(), ref_pts, atol=1e-6)
    del m
