"""Host-side mirror of the reference's matching.py (the caller of the matching
kernels), on top of the HIP entry points ``mast3r_slam_backends.iter_proj`` /
``refine_matches``.

Same functions, arguments and semantics as
/root/reference/mast3r_slam/matching.py:1-90; the matching configuration is
passed explicitly (the reference reads ``config["matching"]``; MATCHING_CFG
holds its base.yaml:8-14 values). The ray-image prep (normalise + Scharr
gradient of image.py:5-38 + pack) and both per-pixel searches run in HIP;
torch is only the glue the reference also uses (index math, the occlusion
gather).
"""
from __future__ import annotations

import torch

import mast3r_slam_backends as be

# config/base.yaml:8-14
MATCHING_CFG = dict(max_iter=10, lambda_init=1e-8, convergence_thresh=1e-6, dist_thresh=1e-1,
                    radius=3, dilation_max=5)


def pixel_to_lin(p1, w):
    return p1[..., 0] + (w * p1[..., 1])


def lin_to_pixel(idx_1_to_2, w):
    return torch.stack((idx_1_to_2 % w, idx_1_to_2 // w), dim=-1)


def prep_for_iter_proj(X11, X21, idx_1_to_2_init=None):
    """matching.py:25-49: ray image + gradients [b,h,w,9], unit rays [b,hw,3],
    p_init [b,hw,2]. The normalise + Scharr + pack chain is one HIP pass
    (mast3r_slam_backends.prep_rays; device tensors only)."""
    b, h, w, _ = X11.shape
    rays_with_grad_img, pts3d_norm = be.prep_rays(X11.contiguous(), X21.contiguous())
    if idx_1_to_2_init is None:
        idx_1_to_2_init = torch.arange(h * w, device=X11.device)[None, :].repeat(b, 1)
    p_init = lin_to_pixel(idx_1_to_2_init, w).float().contiguous()
    return rays_with_grad_img, pts3d_norm, p_init


def match_iterative_proj(X11, X21, D11, D21, idx_1_to_2_init=None, cfg=MATCHING_CFG):
    """matching.py:52-90 -> (idx_1_to_2 [b,hw] int64, valid [b,hw,1] bool)."""
    b, h, w = X21.shape[:3]
    rays_with_grad_img, pts3d_norm, p_init = prep_for_iter_proj(X11, X21, idx_1_to_2_init)
    p1, valid_proj2 = be.iter_proj(rays_with_grad_img, pts3d_norm, p_init, cfg["max_iter"],
                                   cfg["lambda_init"], cfg["convergence_thresh"])
    p1 = p1.long()
    # occlusion check on 3D distances (matching.py:69-75)
    batch_inds = torch.arange(b, device=X11.device)[:, None].repeat(1, h * w)
    dists2 = torch.linalg.norm(
        X11[batch_inds, p1[..., 1], p1[..., 0], :].reshape(b, h, w, 3) - X21, dim=-1)
    valid_proj2 = valid_proj2 & (dists2 < cfg["dist_thresh"]).view(b, -1)
    if cfg["radius"] > 0:
        (p1,) = be.refine_matches(D11.half().contiguous(), D21.reshape(b, h * w, -1).half().contiguous(),
                                  p1.contiguous(), cfg["radius"], cfg["dilation_max"])
    return pixel_to_lin(p1, w), valid_proj2.unsqueeze(-1)


def match(X11, X21, D11, D21, idx_1_to_2_init=None, cfg=MATCHING_CFG):
    """matching.py:8-10."""
    return match_iterative_proj(X11, X21, D11, D21, idx_1_to_2_init, cfg)
