"""Seeded synthetic pointmap graphs and frame pairs.

There are no datasets or MASt3R weights offline, so every workload is built from
a ray-cast box room:

* N camera poses on a smooth loop (radius ``radius`` m, small height wobble,
  yaw wobble so that every pair of views overlaps), scale 1;
* per-KF canonical pointmaps ``X = z K^-1 [u v 1] + N(0, 0.002 z)``, the layout
  of ``SharedKeyframes.X`` (``frame.py:240``): ``[N, H*W, 3]`` float32;
* confidences ``C = 1 + exp(N(1.0, 0.5))`` and match qualities
  ``Q = 1 + exp(N(0.3, 0.8))`` — both >= 1 like MASt3R's ``exp`` conf mode;
* correspondences ``idx_ii2jj[e, k]``: KF j's pixel k projected into KF i with
  a depth test; invalid entries are 0, as ``matching.py`` leaves them;
* edges: consecutive + loop edges to random earlier KFs, then doubled into
  both directions exactly as ``FactorGraph.prep_two_way_edges``
  (``global_opt.py:104-110``);
* initial poses: GT (+) noise (rot 1 deg, trans 2 cm, log-scale 0.01), KF 0 exact.

Everything is torch so it runs on the device where the benchmark lives.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .sim3 import Sim3

ROOM_LO = (-4.0, -2.5, -1.5)
ROOM_HI = (4.0, 2.5, 5.0)


def intrinsics(H: int, W: int, device=None) -> torch.Tensor:
    f = 0.8 * W
    return torch.tensor(
        [[f, 0.0, W / 2.0], [0.0, f, H / 2.0], [0.0, 0.0, 1.0]],
        dtype=torch.float32,
        device=device,
    )


def _yaw_pitch_quat(yaw: torch.Tensor, pitch: torch.Tensor) -> torch.Tensor:
    """q = q_yaw(about y) * q_pitch(about x), xyzw."""
    cy, sy = torch.cos(yaw / 2), torch.sin(yaw / 2)
    cp, sp = torch.cos(pitch / 2), torch.sin(pitch / 2)
    # q_y = (0, sy, 0, cy), q_x = (sp, 0, 0, cp)
    x = cy * sp
    y = sy * cp
    z = -sy * sp
    w = cy * cp
    return torch.stack((x, y, z, w), dim=-1)


def loop_trajectory(N: int, gen: torch.Generator, radius=0.6, device=None) -> Sim3:
    k = torch.arange(N, dtype=torch.float64)
    th = 2 * math.pi * k / max(N, 1)
    px = radius * torch.cos(th) - radius
    pz = radius * torch.sin(th)
    py = 0.1 * torch.sin(3 * th)
    yaw = math.radians(20.0) * torch.sin(th)
    pitch = math.radians(5.0) * torch.cos(2 * th)
    q = _yaw_pitch_quat(yaw, pitch)
    t = torch.stack((px, py, pz), dim=-1)
    data = torch.cat((t, q, torch.ones(N, 1, dtype=torch.float64)), dim=-1)
    return Sim3(data.to(torch.float32).to(device))


def pixel_rays(H: int, W: int, K: torch.Tensor) -> torch.Tensor:
    """K^-1 [u v 1] for the row-major pixel grid, [H*W, 3] (z = 1)."""
    dev = K.device
    v, u = torch.meshgrid(
        torch.arange(H, device=dev, dtype=torch.float32),
        torch.arange(W, device=dev, dtype=torch.float32),
        indexing="ij",
    )
    x = (u.reshape(-1) - K[0, 2]) / K[0, 0]
    y = (v.reshape(-1) - K[1, 2]) / K[1, 1]
    return torch.stack((x, y, torch.ones_like(x)), dim=-1)


def raycast_depth(T_WC: Sim3, rays_c: torch.Tensor) -> torch.Tensor:
    """Camera-frame z of the first box-wall hit for each pixel ray; [N, HW]."""
    N = T_WC.shape[0]
    d = T_WC.data
    t = d[:, None, 0:3]
    q = d[:, None, 3:7].expand(N, rays_c.shape[0], 4)
    from .sim3 import quat_rotate

    dw = quat_rotate(q, rays_c[None].expand(N, -1, 3))
    lo = torch.tensor(ROOM_LO, device=rays_c.device)
    hi = torch.tensor(ROOM_HI, device=rays_c.device)
    bound = torch.where(dw > 0, hi, lo)
    tt = (bound - t) / torch.where(dw.abs() < 1e-9, torch.full_like(dw, 1e-9), dw)
    tt = torch.where(tt > 0, tt, torch.full_like(tt, float("inf")))
    z = tt.min(dim=-1).values
    return z  # ray z-component is 1, so the hit parameter is the depth


@dataclass
class Graph:
    H: int
    W: int
    K: torch.Tensor  # [3,3]
    T_gt: Sim3  # [N]
    T_init: Sim3  # [N]
    Xs: torch.Tensor  # [N, HW, 3]
    Cs: torch.Tensor  # [N, HW, 1]
    ii: torch.Tensor  # [E_dir] int64 (global KF ids)
    jj: torch.Tensor
    idx_ii2jj: torch.Tensor  # [E_dir, HW] int64
    valid_match: torch.Tensor  # [E_dir, HW, 1] bool
    Q: torch.Tensor  # [E_dir, HW, 1] float32
    kf_ids: torch.Tensor  # [N] global ids of the KFs (sorted)

    @property
    def n_edges(self):
        return int(self.ii.numel())


def perturb(T: Sim3, gen: torch.Generator, rot_deg=1.0, trans=0.02, log_s=0.01, fix_first=True) -> Sim3:
    N = T.shape[0]
    xi = torch.zeros(N, 7, dtype=torch.float32)
    xi[:, 0:3] = torch.randn(N, 3, generator=gen) * trans
    xi[:, 3:6] = torch.randn(N, 3, generator=gen) * math.radians(rot_deg)
    xi[:, 6] = torch.randn(N, generator=gen) * log_s
    if fix_first:
        xi[0] = 0
    return Sim3.exp(xi.to(T.device)) * T


def make_edges(N: int, gen: torch.Generator, loop_frac=0.55):
    """Consecutive edges + ~loop_frac*N loop edges to random earlier KFs."""
    ii = list(range(N - 1))
    jj = list(range(1, N))
    n_loop = int(round(loop_frac * N))
    cands = list(range(2, N))
    if n_loop and cands:
        pick = torch.randperm(len(cands), generator=gen)[: min(n_loop, len(cands))]
        for p in sorted(pick.tolist()):
            j = cands[p]
            i = int(torch.randint(0, j - 1, (1,), generator=gen))
            ii.append(i)
            jj.append(j)
    return ii, jj


def correspondences(Xw_j: torch.Tensor, T_i: Sim3, depth_i: torch.Tensor, K: torch.Tensor, H: int, W: int):
    """Project KF j's world points into KF i; idx (row-major) + validity."""
    P = T_i.inv().act(Xw_j)  # [HW,3] in camera i
    z = P[:, 2]
    zs = torch.where(z.abs() < 1e-6, torch.full_like(z, 1e-6), z)
    u = K[0, 0] * P[:, 0] / zs + K[0, 2]
    v = K[1, 1] * P[:, 1] / zs + K[1, 2]
    ur = torch.round(u)
    vr = torch.round(v)
    inside = (z > 1e-3) & (ur >= 0) & (ur <= W - 1) & (vr >= 0) & (vr <= H - 1)
    idx = (vr.clamp(0, H - 1) * W + ur.clamp(0, W - 1)).to(torch.int64)
    zi = depth_i[idx]
    vis = inside & ((zi - z).abs() < 0.05 * z)
    idx = torch.where(vis, idx, torch.zeros_like(idx))
    return idx, vis


def make_graph(
    N: int,
    H: int,
    W: int,
    seed: int = 1003,
    device=None,
    loop_frac: float = 0.55,
    edges=None,
    kf_ids=None,
    noise=True,
    edge_range=None,
    edge_ids=None,
) -> Graph:
    """Build a synthetic FactorGraph problem (already in the two-way edge form
    that ``FactorGraph.prep_two_way_edges`` hands to the backend).

    ``edge_range=(b, e)`` builds idx/valid/Q only for directed edges [b, e)
    (a rank's shard); every per-edge random draw is seeded by the edge index,
    so shards are slices of the full graph. ``edge_ids`` (a list of directed
    edge ids, e.g. ``distributed.edge_shard``'s) builds exactly those edges in
    that order instead. ii/jj are always the full lists."""
    gen = torch.Generator().manual_seed(seed)
    K = intrinsics(H, W, device)
    T_gt = loop_trajectory(N, gen, device=device)
    rays = pixel_rays(H, W, K)
    depth = raycast_depth(T_gt, rays)  # [N, HW]
    X_clean = depth[..., None] * rays[None]
    if noise:
        nz = torch.randn(X_clean.shape, generator=gen).to(device) * (0.002 * depth[..., None])
        Xs = (X_clean + nz).contiguous()
    else:
        Xs = X_clean.contiguous()
    Cs = (1.0 + torch.exp(1.0 + 0.5 * torch.randn(N, H * W, 1, generator=gen))).to(device)

    if edges is None:  # own generator: the edge set must not depend on H x W
        ii_u, jj_u = make_edges(N, torch.Generator().manual_seed(seed + 7), loop_frac)
    else:
        ii_u, jj_u = edges
    # two-way edges: (i,j) then (j,i) — global_opt.py:104-110
    ii_dir = ii_u + jj_u
    jj_dir = jj_u + ii_u
    E = len(ii_dir)
    HW = H * W
    if edge_ids is not None:
        sel = [int(e) for e in edge_ids]
        assert all(0 <= e < E for e in sel)
    else:
        eb, ee = (0, E) if edge_range is None else (max(0, edge_range[0]), min(E, edge_range[1]))
        sel = list(range(eb, max(ee, eb)))
    n_loc = len(sel)
    idx = torch.empty(n_loc, HW, dtype=torch.int64, device=device)
    valid = torch.empty(n_loc, HW, 1, dtype=torch.bool, device=device)
    Q = torch.empty(n_loc, HW, 1, dtype=torch.float32, device=device)
    for k, e in enumerate(sel):
        i, j = ii_dir[e], jj_dir[e]
        Xw_j = T_gt[j : j + 1].act(X_clean[j])
        ie, ve = correspondences(Xw_j, T_gt[i : i + 1], depth[i], K, H, W)
        idx[k] = ie
        valid[k, :, 0] = ve
        ge = torch.Generator().manual_seed(seed * 1000003 + e)
        Q[k] = (1.0 + torch.exp(0.3 + 0.8 * torch.randn(HW, 1, generator=ge))).to(device)
    T_init = perturb(T_gt, torch.Generator().manual_seed(seed + 13)) if noise else T_gt.clone()
    if kf_ids is None:
        kf_ids = torch.arange(N, dtype=torch.int64)
    kf_ids = torch.as_tensor(kf_ids, dtype=torch.int64)
    ii_t = kf_ids[torch.tensor(ii_dir, dtype=torch.int64)].to(device)
    jj_t = kf_ids[torch.tensor(jj_dir, dtype=torch.int64)].to(device)
    return Graph(H, W, K, T_gt, T_init, Xs, Cs, ii_t, jj_t, idx, valid, Q, kf_ids.to(device))


@dataclass
class Pair:
    """Tracker inputs for one frame -> keyframe registration (tracker.py:54-64)."""

    H: int
    W: int
    K: torch.Tensor
    T_WCk: Sim3  # [1]
    T_WCf_gt: Sim3  # [1]
    T_WCf_init: Sim3  # [1]
    Xf: torch.Tensor  # [HW,3] frame points already gathered by idx_f2k
    Xk: torch.Tensor  # [HW,3]
    Qk: torch.Tensor  # [HW,1]
    valid: torch.Tensor  # [HW,1] bool (valid_opt)
    Cf: torch.Tensor  # [HW,1] (gathered)
    Ck: torch.Tensor  # [HW,1]


def make_pair(H: int, W: int, seed: int = 1001, device=None, identity_idx=False) -> Pair:
    """A keyframe (pose 0) and a frame (pose 1) of the loop trajectory."""
    gen = torch.Generator().manual_seed(seed)
    K = intrinsics(H, W, device)
    T_gt = loop_trajectory(16, gen, device=device)[0:2]
    rays = pixel_rays(H, W, K)
    depth = raycast_depth(T_gt, rays)
    X_clean = depth[..., None] * rays[None]
    nz = torch.randn(X_clean.shape, generator=gen).to(device) * (0.002 * depth[..., None])
    X = X_clean + nz
    C = (1.0 + torch.exp(1.0 + 0.5 * torch.randn(2, H * W, 1, generator=gen))).to(device)
    # idx_f2k: for each KF pixel, the frame pixel seeing the same point
    if identity_idx:
        idx = torch.arange(H * W, device=device)
        vis = torch.ones(H * W, dtype=torch.bool, device=device)
    else:
        Xw_k = T_gt[0:1].act(X_clean[0])
        idx, vis = correspondences(Xw_k, T_gt[1:2], depth[1], K, H, W)
    Qk = (1.0 + torch.exp(0.3 + 0.8 * torch.randn(H * W, 1, generator=gen))).to(device)
    Xf = X[1][idx].contiguous()
    Cf = C[1][idx].contiguous()
    Xk = X[0].contiguous()
    Ck = C[0].contiguous()
    valid = (vis[:, None] & (Cf > 0.0) & (Ck > 0.0) & (Qk > 1.5)).contiguous()
    T_WCk = T_gt[0:1]
    T_WCf_gt = T_gt[1:2]
    xi = torch.zeros(1, 7)
    xi[:, 0:3] = torch.randn(1, 3, generator=gen) * 0.02
    xi[:, 3:6] = torch.randn(1, 3, generator=gen) * math.radians(1.0)
    xi[:, 6] = torch.randn(1, generator=gen) * 0.01
    T_WCf_init = Sim3.exp(xi.to(device)) * T_WCf_gt
    return Pair(H, W, K, T_WCk, T_WCf_gt, T_WCf_init, Xf, Xk, Qk, valid, Cf, Ck)


@dataclass
class MatchInputs:
    """Inputs of matching.match (matching.py:8-10) for one view pair: X11 is view
    1's pointmap in camera 1, X21 view 2's pointmap expressed in camera 1 (what
    MASt3R's pairwise head returns), D11 / D21 per-pixel descriptors. p_true is
    the pixel of view 1 each view-2 pixel projects to (vis marks visible ones)."""
    H: int
    W: int
    X11: torch.Tensor  # [1, H, W, 3] f32
    X21: torch.Tensor  # [1, H, W, 3] f32
    D11: torch.Tensor  # [1, H, W, F] f16
    D21: torch.Tensor  # [1, H*W, F] f16
    p_true: torch.Tensor  # [1, H*W, 2] int64
    vis: torch.Tensor  # [1, H*W] bool


def make_match_inputs(H: int, W: int, seed: int = 1005, device=None, F: int = 24) -> MatchInputs:
    gen = torch.Generator().manual_seed(seed)
    K = intrinsics(H, W, device)
    T = loop_trajectory(16, gen, device=device)[0:2]
    rays = pixel_rays(H, W, K)
    depth = raycast_depth(T, rays)
    X = depth[..., None] * rays[None]
    Xw2 = T[1:2].act(X[1])
    idx, vis = correspondences(Xw2, T[0:1], depth[0], K, H, W)
    X21 = T[0:1].inv().act(Xw2)
    p_true = torch.stack((idx % W, idx // W), -1)
    # descriptors: a spatially smooth unit feature field for view 1 (blurred
    # noise plus a fine-scale part), view 2 = the matched view-1 feature plus
    # noise where visible (random elsewhere)
    raw = torch.randn(1, F, H, W, generator=gen)
    g = torch.exp(-0.5 * (torch.arange(-6, 7, dtype=torch.float32) / 3.0) ** 2)
    g = g / g.sum()
    sm = torch.nn.functional.conv2d(torch.nn.functional.pad(raw, (6, 6, 0, 0), mode="replicate"),
                                    g.view(1, 1, 1, 13).repeat(F, 1, 1, 1), groups=F)
    sm = torch.nn.functional.conv2d(torch.nn.functional.pad(sm, (0, 0, 6, 6), mode="replicate"),
                                    g.view(1, 1, 13, 1).repeat(F, 1, 1, 1), groups=F)
    field = sm / sm.std() + 0.15 * torch.randn(1, F, H, W, generator=gen)
    D11 = torch.nn.functional.normalize(field[0].permute(1, 2, 0).reshape(H * W, F), dim=-1).to(device)
    noise = torch.nn.functional.normalize(torch.randn(H * W, F, generator=gen), dim=-1).to(device)
    D21 = torch.where(vis[:, None], torch.nn.functional.normalize(D11[idx] + 0.3 * noise, dim=-1), noise)
    return MatchInputs(H, W, X[0].reshape(1, H, W, 3).contiguous(), X21.reshape(1, H, W, 3).contiguous(),
                       D11.reshape(1, H, W, F).half().contiguous(), D21[None].half().contiguous(),
                       p_true[None].contiguous(), vis[None].contiguous())
