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


def test_refine_score_chain_is_c10_half_arithmetic():
    """The oracle's fp16 score step (a rounded product, then a rounded sum per
    feature) is c10::Half's `score += a * b`, the reference kernel's arithmetic
    for its .half() descriptors (matching_kernels.cu:58-60, :103): checked
    bitwise against torch's own CPU Half tensors, whose operators are c10's
    (compute in float, convert back). A fused multiply-add chain differs from
    it on these inputs, so the test tells the two apart."""
    g = torch.Generator().manual_seed(71)
    n, fd = 4096, 24
    a = F.normalize(torch.randn(n, fd, generator=g), dim=-1).half()
    b = F.normalize(torch.randn(n, fd, generator=g), dim=-1).half()
    s_t = torch.zeros(n, dtype=torch.float16)
    s_o = np.zeros(n, np.float16)
    s_f = np.zeros(n, np.float16)
    for k in range(fd):
        s_t = s_t + a[:, k] * b[:, k]
        s_o = mo._score_step(a[:, k].numpy(), b[:, k].numpy(), s_o, np.float16)
        s_f = (a[:, k].numpy().astype(np.float64) * b[:, k].numpy().astype(np.float64)
               + s_f.astype(np.float64)).astype(np.float16)
    assert np.array_equal(s_o.view(np.uint16), s_t.numpy().view(np.uint16))
    assert not np.array_equal(s_f.view(np.uint16), s_t.numpy().view(np.uint16))


def test_refine_tiny_positive_score_moves_the_centre():
    """max_score starts at c10::Half's numeric_limits min() as libcu++ defines
    it for an unspecialised type, T() = 0 (matching_kernels.cu:47): a
    candidate whose score is a positive subnormal (below the smallest normal
    half, 6.1e-5) still wins over the centre."""
    D11 = np.zeros((1, 3, 3, 2), np.float16)
    D11[0, 1, 2] = [np.float16(2.0 ** -12), 0]  # score 2^-12 * 2^-12 = 2^-24, the smallest subnormal
    D21 = np.zeros((1, 1, 2), np.float16)
    D21[0, 0] = [np.float16(2.0 ** -12), 0]
    p1 = np.array([[[1, 1]]], np.int64)
    assert np.array_equal(mo.refine_matches(D11, D21, p1, 1, 1), np.array([[[2, 1]]]))
