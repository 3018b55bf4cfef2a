"""GPU parity of the HIP matching kernels (mast3r_slam_backends.iter_proj /
refine_matches -> m3s_match.hip) against the numpy restatement of
matching_kernels.cu (oracle/matching_oracle.py; parity unpinned, see there).

Tolerances: refine_matches returns integer pixels and must agree exactly
(float16 descriptors, the reference's path); iter_proj's float pixels follow
the same IEEE operation sequence and are compared bitwise on >= 99% of points
and within 1e-4 px on all; converged flags agree on >= 99%.
"""
import numpy as np
import pytest
import torch

import mast3r_slam_backends as be
from mast3r_slam_amd import matching, synthetic
from oracle import fusion_oracle as fo
from oracle import matching_oracle as mo

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _inputs(H=48, W=64, seed=1005):
    """CPU inputs built with the reference's torch expressions (oracle)."""
    m = synthetic.make_match_inputs(H, W, seed=seed)
    img, pts = fo.prep_rays(m.X11.numpy(), m.X21.numpy())
    ar = torch.arange(H * W)
    p0 = torch.stack((ar % W, ar // W), -1)[None].float().contiguous()
    return m, torch.from_numpy(img), torch.from_numpy(pts), p0


@pytest.mark.parametrize("H,W,max_iter", [(48, 64, 10), (37, 53, 3), (3, 3, 10)])
def test_iter_proj_matches_oracle(H, W, max_iter):
    m, img, pts, p0 = _inputs(H, W)
    p_ref, c_ref = mo.iter_proj(img.numpy(), pts.numpy(), p0.numpy(), max_iter, 1e-8, 1e-6)
    p, c = be.iter_proj(img.to(DEV), pts.to(DEV), p0.to(DEV), max_iter, 1e-8, 1e-6)
    p, c = p.cpu().numpy(), c.cpu().numpy()
    assert p.dtype == np.float32 and c.dtype == bool and p.shape == p_ref.shape
    assert np.abs(p - p_ref).max() < 1e-4
    assert (p == p_ref).all(-1).mean() >= 0.99
    assert (c == c_ref).mean() >= 0.99


def test_iter_proj_batched_and_clamped_init():
    m, img, pts, p0 = _inputs(32, 40)
    img2 = torch.cat([img, img.flip(1)]).contiguous()
    pts2 = torch.cat([pts, pts.flip(1)]).contiguous()
    p02 = torch.cat([p0, p0 * 1.7 - 5.0]).contiguous()  # second batch partly outside the image
    p_ref, c_ref = mo.iter_proj(img2.numpy(), pts2.numpy(), p02.numpy(), 10, 1e-8, 1e-6)
    p, c = be.iter_proj(img2.to(DEV), pts2.to(DEV), p02.to(DEV), 10, 1e-8, 1e-6)
    assert np.abs(p.cpu().numpy() - p_ref).max() < 1e-4
    assert (c.cpu().numpy() == c_ref).mean() >= 0.99


@pytest.mark.parametrize("dtype", [torch.float16, torch.float32])
@pytest.mark.parametrize("radius,dilation", [(3, 5), (2, 1), (0, 3)])
def test_refine_matches_matches_oracle(dtype, radius, dilation):
    m = synthetic.make_match_inputs(48, 64)
    rng = np.random.default_rng(1)
    p_start = np.clip(m.p_true.numpy() + rng.integers(-4, 5, m.p_true.shape), 0, [63, 47])
    D11, D21 = m.D11.to(dtype), m.D21.to(dtype)
    ref = mo.refine_matches(D11.numpy(), D21.numpy(), p_start, radius, dilation)
    (out,) = be.refine_matches(D11.to(DEV), D21.to(DEV), torch.from_numpy(p_start).to(DEV), radius, dilation)
    out = out.cpu().numpy()
    assert out.dtype == np.int64 and out.shape == ref.shape
    agree = (out == ref).all(-1).mean()
    assert agree == 1.0 if dtype == torch.float16 else agree >= 0.999


def test_refine_matches_odd_feature_width():
    m = synthetic.make_match_inputs(24, 32, F=20)  # F not specialised in registers
    p = m.p_true.numpy()
    ref = mo.refine_matches(m.D11.numpy(), m.D21.numpy(), p, 3, 5)
    (out,) = be.refine_matches(m.D11.to(DEV), m.D21.to(DEV), m.p_true.to(DEV), 3, 5)
    assert np.array_equal(out.cpu().numpy(), ref)


def test_match_pipeline_recovers_correspondences():
    """mast3r_slam_amd.matching.match (matching.py:8-90 mirror) end to end."""
    m = synthetic.make_match_inputs(96, 128)
    idx, valid = matching.match(m.X11.to(DEV), m.X21.to(DEV), m.D11.to(DEV), m.D21.to(DEV))
    idx, valid = idx.cpu()[0], valid.cpu()[0, :, 0]
    p_true = m.p_true[0]
    true_idx = p_true[:, 0] + 128 * p_true[:, 1]
    ok = valid & m.vis[0]
    assert ok.float().mean() > 0.6
    u, v = idx % 128, idx // 128
    near = ((u - p_true[:, 0]).abs() <= 1) & ((v - p_true[:, 1]).abs() <= 1)
    assert near[ok].float().mean() > 0.95
    assert (idx[ok] == true_idx[ok]).float().mean() > 0.8


def test_matching_rejects_bad_inputs():
    m, img, pts, p0 = _inputs(16, 16)
    with pytest.raises(RuntimeError, match="contiguous"):
        be.iter_proj(img.to(DEV).transpose(1, 2), pts.to(DEV), p0.to(DEV), 10, 1e-8, 1e-6)
    with pytest.raises(RuntimeError):
        be.refine_matches(m.D11.to(DEV), m.D21.to(DEV).float(), m.p_true.to(DEV), 3, 5)


@pytest.mark.parametrize("F", [16, 24, 32])
def test_refine_matches_f16_kernel_batches_and_far_centres(F):
    """refine_f16_kernel (round 5: XCD bands, zero-returning out-of-image
    loads; round 6: the reference's c10::Half chains): batched (a wave straddles the two batches: 37 x 53
    pixels is not a multiple of 64), centres near and past the borders and far
    outside (|p| up to 2^40: no candidate is inside, p is returned as is),
    F = 16 / 24 / 32; integer output equal to the oracle."""
    H, W = 37, 53
    ms = [synthetic.make_match_inputs(H, W, seed=1100 + k, F=F) for k in range(2)]
    D11 = torch.cat([m.D11 for m in ms]).contiguous()
    D21 = torch.cat([m.D21 for m in ms]).contiguous()
    rng = np.random.default_rng(F)
    p = np.concatenate([m.p_true.numpy() for m in ms]).astype(np.int64)
    p = p + rng.integers(-6, 7, p.shape)
    sel = rng.random(p.shape[:2]) < 0.05
    p[sel] = rng.integers(-25, 80, (int(sel.sum()), 2))  # near and past the borders
    far = rng.random(p.shape[:2]) < 0.01
    p[far] = rng.choice(np.array([-(1 << 40), (1 << 40), -(1 << 31) - 3, (1 << 31) + 5]), (int(far.sum()), 2))
    ref = mo.refine_matches(D11.numpy(), D21.numpy(), p, 3, 5)
    (out,) = be.refine_matches(D11.to(DEV), D21.to(DEV), torch.from_numpy(p).to(DEV), 3, 5)
    out = out.cpu().numpy()
    assert np.array_equal(out, ref), (out != ref).any(-1).sum()
    assert np.array_equal(out[far], p[far])


@pytest.mark.parametrize("F,radius", [(16, 3), (8, 1)])
def test_refine_matches_subnormal_score_moves_centre(F, radius):
    """Both refine kernels (refine_f16_kernel: F = 16, radius 3; refine_kernel:
    F = 8, radius 1) start the running maximum at c10::Half's numeric_limits
    min() as libcu++ leaves it, 0 (matching_kernels.cu:47): a candidate whose
    c10::Half score is the smallest positive subnormal wins; every other
    candidate scores 0 and the first-maximum rule keeps the planted one."""
    H, W = 9, 11
    D11 = torch.zeros(1, H, W, F, dtype=torch.float16)
    D11[0, 6, 2, 0] = 2.0 ** -12
    D21 = torch.zeros(1, 1, F, dtype=torch.float16)
    D21[0, 0, 0] = 2.0 ** -12
    p = np.array([[[3, 5]]], np.int64)
    ref = mo.refine_matches(D11.numpy(), D21.numpy(), p, radius, 1)
    (out,) = be.refine_matches(D11.to(DEV), D21.to(DEV), torch.from_numpy(p).to(DEV), radius, 1)
    assert np.array_equal(ref, np.array([[[2, 6]]])) and np.array_equal(out.cpu().numpy(), ref)
