"""NumPy restatement of the steps either side of the GN/matching path
(SURVEY.md §8f #2 and #4).

TEST INFRASTRUCTURE ONLY — imported by tests/ as the checker; the product path
(mast3r_slam_backends.fuse_pointmap / prep_rays -> m3s_fuse.hip) never imports it.

* ``fuse_pointmap``  tracker.py:98-99 (Xkk = T_CkCf.act(Xkf)) + Frame.update_pointmap
                     (frame.py:41-100) for an initialised keyframe, modes
                     weighted_pointmap (:73-76), indep_conf (:68-72), recent (:59-62),
                     weighted_spherical (:78-100, the reference's torch expressions
                     on CPU tensors); elementwise fp32 in the torch expressions'
                     operation order.
* ``prep_rays``      prep_for_iter_proj (matching.py:25-49): F.normalize (eps 1e-12),
                     Scharr x/y kernels / 32 with reflect padding (image.py:5-38).

Pinned by the reference's own expressions, evaluated here with torch on the
CPU (the same torch ops the reference calls) — see tests/test_gpu_fusion.py.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from oracle import tracker_oracle as tro

F32 = np.float32


def fuse_pointmap(X_canon, C, X_new, C_new, T=None, mode="weighted_pointmap"):
    X = np.asarray(X_new, F32).reshape(-1, 3)
    if T is not None:
        X = tro.act(np.asarray(T, F32).reshape(1, 8), X).astype(F32)
    Xc = np.asarray(X_canon, F32).reshape(-1, 3).copy()
    Co = np.asarray(C, F32).reshape(-1, 1).copy()
    Cn = np.asarray(C_new, F32).reshape(-1, 1)
    if mode == "weighted_pointmap":
        Xc = (((Co * Xc).astype(F32) + (Cn * X).astype(F32)).astype(F32) / (Co + Cn).astype(F32)).astype(F32)
        Co = (Co + Cn).astype(F32)
    elif mode == "indep_conf":
        m = (Cn > Co)[:, 0]
        Xc[m] = X[m]
        Co[m] = Cn[m]
    elif mode == "recent":
        Xc, Co = X.copy(), Cn.copy()
    elif mode == "weighted_spherical":  # frame.py:78-100, the same torch ops
        def to_sph(P):
            r = torch.linalg.norm(P, dim=-1, keepdim=True)
            x, y, z = torch.tensor_split(P, 3, dim=-1)
            return torch.cat((r, torch.atan2(y, x), torch.acos(z / r)), dim=-1)

        def to_cart(S):
            r, phi, theta = torch.tensor_split(S, 3, dim=-1)
            return torch.cat((r * torch.sin(theta) * torch.cos(phi), r * torch.sin(theta) * torch.sin(phi),
                              r * torch.cos(theta)), dim=-1)

        tC, tCn = torch.as_tensor(Co), torch.as_tensor(Cn)
        s = ((tC * to_sph(torch.as_tensor(Xc))) + (tCn * to_sph(torch.as_tensor(X)))) / (tC + tCn)
        Xc = to_cart(s).numpy().astype(F32)
        Co = (Co + Cn).astype(F32)
    else:
        raise ValueError(mode)
    return Xc, Co


def prep_rays(X11, X21):
    """The reference's torch expressions, on CPU tensors."""
    X11 = torch.as_tensor(np.asarray(X11, F32))
    X21 = torch.as_tensor(np.asarray(X21, F32))
    b, h, w, _ = X11.shape
    rays = F.normalize(X11, dim=-1).permute(0, 3, 1, 2)
    kx = (1.0 / 32.0) * torch.tensor([[-3.0, 0.0, 3.0], [-10.0, 0.0, 10.0], [-3.0, 0.0, 3.0]])
    ky = (1.0 / 32.0) * torch.tensor([[-3.0, -10.0, -3.0], [0.0, 0.0, 0.0], [3.0, 10.0, 3.0]])
    pad = F.pad(rays, (1, 1, 1, 1), mode="reflect")
    gx = F.conv2d(pad, kx.repeat(3, 1, 1, 1), groups=3)
    gy = F.conv2d(pad, ky.repeat(3, 1, 1, 1), groups=3)
    img = torch.cat((rays, gx, gy), dim=1).permute(0, 2, 3, 1).contiguous()
    pts = F.normalize(X21.reshape(b, -1, 3), dim=-1)
    return img.numpy(), pts.numpy()
