"""CPU checks of the matching oracle (oracle/matching_oracle.py, the numpy
restatement of matching_kernels.cu that the GPU tests compare against).

Parity unpinned (no reference fixtures exist for these kernels): these tests
pin the restatement's behaviour on a synthetic view pair with known
correspondences instead.
"""
import numpy as np
import torch
import torch.nn.functional as F

from mast3r_slam_amd import synthetic
from oracle import matching_oracle as mo


def _prep(m):
    b, h, w, _ = m.X11.shape
    rays = F.normalize(m.X11, dim=-1).permute(0, 3, 1, 2)
    k = torch.tensor([[-3.0, 0, 3], [-10, 0, 10], [-3, 0, 3]]) / 32
    pad = F.pad(rays, (1, 1, 1, 1), mode="reflect")
    gx = F.conv2d(pad, k.repeat(3, 1, 1, 1), groups=3)
    gy = F.conv2d(pad, k.t().contiguous().repeat(3, 1, 1, 1), groups=3)
    img = torch.cat((rays, gx, gy), 1).permute(0, 2, 3, 1).contiguous()
    pts = F.normalize(m.X21.reshape(1, -1, 3), dim=-1)
    ar = torch.arange(h * w)
    p0 = torch.stack((ar % w, ar // w), -1)[None].float()
    return img.numpy(), pts.numpy(), p0.numpy()


def test_iter_proj_recovers_projections():
    m = synthetic.make_match_inputs(48, 64)
    img, pts, p0 = _prep(m)
    p, conv = mo.iter_proj(img, pts, p0, 10, 1e-8, 1e-6)
    vis = m.vis[0].numpy()
    ok = vis & conv[0]
    assert ok.mean() > 0.7
    err = np.abs(np.round(p[0]) - m.p_true[0].numpy()).max(-1)
    assert (err[ok] <= 1).mean() > 0.99


def test_iter_proj_zero_iterations_clamps_init():
    img = np.zeros((1, 5, 6, 9), np.float32)
    p0 = np.array([[[-3.0, 10.0], [2.5, 2.5], [np.nan, 0.0]]], np.float32)
    p, conv = mo.iter_proj(img, np.zeros((1, 3, 3), np.float32), p0, 0, 1e-8, 1e-6)
    assert np.array_equal(p[0], np.array([[1, 3], [2.5, 2.5], [1, 1]], np.float32))
    assert not conv.any()


def test_refine_finds_planted_matches():
    m = synthetic.make_match_inputs(48, 64)
    vis = m.vis[0].numpy()
    # start 2-4 px away from the truth: the dilated search must come back
    rng = np.random.default_rng(0)
    p_true = m.p_true.numpy()
    p_start = np.clip(p_true + rng.integers(-4, 5, p_true.shape), 0, [63, 47])
    p1 = mo.refine_matches(m.D11.numpy(), m.D21.numpy(), p_start, 3, 5)
    near = np.abs(p1[0] - p_true[0]).max(-1) <= 1
    assert near[vis].mean() > 0.98


def test_refine_keeps_centre_when_no_positive_score():
    D11 = -np.ones((1, 4, 4, 8), np.float16)
    D21 = np.ones((1, 2, 8), np.float16)
    p1 = np.array([[[1, 2], [3, 0]]], np.int64)
    assert np.array_equal(mo.refine_matches(D11, D21, p1, 1, 2), p1)
