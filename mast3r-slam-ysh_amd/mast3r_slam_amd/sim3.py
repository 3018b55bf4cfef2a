"""Sim(3) group on torch tensors — the subset of lietorch's ``Sim3`` that the
reference's GN path uses.

Data layout is lietorch's ``[tx, ty, tz, qx, qy, qz, qw, s]`` (embedded_dim 8),
tangent layout ``[tau(3), phi(3), sigma(1)]``.

lietorch itself is a third-party dependency of the reference
(``/root/reference/pyproject.toml:14``, an unpinned git URL) and is not vendored,
so its arithmetic is restated here from the reference's own CUDA restatement of
it, which is the in-repo spec:

* quaternion product / inverse  — ``gn_kernels.cu:177-193``
* rotation of a point           — ``gn_kernels.cu:195-205``
* Sim3 action ``s R X + t``     — ``gn_kernels.cu:207-219``
* Exp (SO3 and Sim3, EPS=1e-6)  — ``gn_kernels.cu:299-390``
* left retraction Exp(xi) * T   — ``gn_kernels.cu:392-413``

Call sites this type replaces: ``tracker.py:98,180,187,195,212``,
``geometry.py:46``, ``global_opt.py:115``, ``frame.py:24,239``.

This module is host plumbing (the tracker/FactorGraph mirror and the synthetic
generator); the hot path applies the same formulas on device in
``csrc/m3s_device.h`` (exposed for tests by ``m3s_debug_sim3``). Both are
checked against the group's mathematics in ``tests/test_sim3_math.py`` /
``tests/test_gpu_sim3.py``: Exp is the matrix exponential of the sim(3)
generator, compose / inverse / act are 4x4 matrix products, and the
reference's Jacobian rows are the derivatives of its residuals.
"""
from __future__ import annotations

import torch

EPS = 1e-6


def quat_mul(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Hamilton product a*b, xyzw (gn_kernels.cu:179-184)."""
    ax, ay, az, aw = a.unbind(-1)
    bx, by, bz, bw = b.unbind(-1)
    return torch.stack(
        (
            aw * bx + ax * bw + ay * bz - az * by,
            aw * by - ax * bz + ay * bw + az * bx,
            aw * bz + ax * by - ay * bx + az * bw,
            aw * bw - ax * bx - ay * by - az * bz,
        ),
        dim=-1,
    )


def quat_inv(q: torch.Tensor) -> torch.Tensor:
    return torch.cat((-q[..., :3], q[..., 3:]), dim=-1)


def quat_rotate(q: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
    """R(q) X via uv = 2 q_v x X ; X + w uv + q_v x uv (gn_kernels.cu:195-205)."""
    qv = q[..., :3]
    w = q[..., 3:]
    uv = 2.0 * torch.linalg.cross(qv, X, dim=-1)
    return X + w * uv + torch.linalg.cross(qv, uv, dim=-1)


def _bcast(a: torch.Tensor, b: torch.Tensor):
    shape = torch.broadcast_shapes(a.shape[:-1], b.shape[:-1])
    return a.expand(*shape, a.shape[-1]), b.expand(*shape, b.shape[-1])


def exp_so3(phi: torch.Tensor) -> torch.Tensor:
    """SO3 Exp as quaternion; Taylor branch when theta^2 < EPS (gn_kernels.cu:299-321)."""
    theta_sq = (phi * phi).sum(-1, keepdim=True)
    theta_p4 = theta_sq * theta_sq
    small = theta_sq < EPS
    theta = torch.sqrt(theta_sq)
    safe_theta = torch.where(small, torch.ones_like(theta), theta)
    imag = torch.where(
        small,
        0.5 - (1.0 / 48.0) * theta_sq + (1.0 / 3840.0) * theta_p4,
        torch.sin(0.5 * safe_theta) / safe_theta,
    )
    real = torch.where(
        small,
        1.0 - (1.0 / 8.0) * theta_sq + (1.0 / 384.0) * theta_p4,
        torch.cos(0.5 * safe_theta),
    )
    return torch.cat((imag * phi, real), dim=-1)


def exp_sim3(xi: torch.Tensor):
    """Sim3 Exp -> (t, q, s) with lietorch's RxSO3 W = C I + A Phi + B Phi^2
    and its small-sigma / small-theta branches (gn_kernels.cu:323-390)."""
    tau = xi[..., 0:3]
    phi = xi[..., 3:6]
    sigma = xi[..., 6:7]
    scale = torch.exp(sigma)
    q = exp_so3(phi)
    theta_sq = (phi * phi).sum(-1, keepdim=True)
    theta = torch.sqrt(theta_sq)

    small_s = sigma.abs() < EPS
    small_t = theta.abs() < EPS
    one = torch.ones_like(sigma)
    # guards only keep the unused branches finite; selection below is exact
    sg = torch.where(small_s, one, sigma)
    th = torch.where(small_t, one, theta)
    th_sq = torch.where(small_t, one, theta_sq)

    # sigma ~ 0
    A0t = 0.5 * one
    B0t = one / 6.0
    A0 = (1.0 - torch.cos(th)) / th_sq
    B0 = (th - torch.sin(th)) / (th_sq * th)
    # sigma != 0
    C1 = (scale - 1.0) / sg
    sg_sq = sg * sg
    A1t = ((sg - 1.0) * scale + 1.0) / sg_sq
    B1t = (scale * 0.5 * sg_sq + scale - 1.0 - sg * scale) / (sg_sq * sg)
    a = scale * torch.sin(th)
    b = scale * torch.cos(th)
    c = th_sq + sg * sg
    A1 = (a * sg + (1.0 - b) * th) / (th * c)
    B1 = (C1 - ((b - 1.0) * sg + a * th) / c) / th_sq

    C = torch.where(small_s, one, C1)
    A = torch.where(small_s, torch.where(small_t, A0t, A0), torch.where(small_t, A1t, A1))
    B = torch.where(small_s, torch.where(small_t, B0t, B0), torch.where(small_t, B1t, B1))

    phi_x_tau = torch.linalg.cross(phi, tau, dim=-1)
    phi_x_phi_x_tau = torch.linalg.cross(phi, phi_x_tau, dim=-1)
    t = C * tau + A * phi_x_tau + B * phi_x_phi_x_tau
    return t, q, scale


class Sim3:
    """lietorch.Sim3-compatible container (data [..., 8])."""

    embedded_dim = 8
    manifold_dim = 7

    def __init__(self, data: torch.Tensor):
        if isinstance(data, Sim3):
            data = data.data
        self.data = data

    # -- constructors -----------------------------------------------------
    @classmethod
    def Identity(cls, *batch, device=None, dtype=torch.float32):
        if len(batch) == 1 and isinstance(batch[0], (tuple, list)):
            batch = tuple(batch[0])
        d = torch.zeros(*batch, 8, device=device, dtype=dtype)
        d[..., 6] = 1.0
        d[..., 7] = 1.0
        return cls(d)

    @classmethod
    def exp(cls, xi: torch.Tensor) -> "Sim3":
        t, q, s = exp_sim3(xi)
        return cls(torch.cat((t, q, s), dim=-1))

    # -- accessors --------------------------------------------------------
    @property
    def shape(self):
        return self.data.shape[:-1]

    @property
    def device(self):
        return self.data.device

    @property
    def dtype(self):
        return self.data.dtype

    def translation(self):
        return self.data[..., 0:3]

    def quat(self):
        return self.data[..., 3:7]

    def scale(self):
        return self.data[..., 7:8]

    def __getitem__(self, idx):
        return Sim3(self.data[idx])

    def __len__(self):
        return self.data.shape[0]

    def clone(self):
        return Sim3(self.data.clone())

    def to(self, *args, **kwargs):
        return Sim3(self.data.to(*args, **kwargs))

    def cpu(self):
        return Sim3(self.data.cpu())

    # -- group operations -------------------------------------------------
    def act(self, X: torch.Tensor) -> torch.Tensor:
        """s R X + t, broadcasting the group batch over point batch."""
        d, Xb = _bcast(self.data, X)
        t, q, s = d[..., 0:3], d[..., 3:7], d[..., 7:8]
        return s * quat_rotate(q, Xb) + t

    def inv(self) -> "Sim3":
        t, q, s = self.translation(), self.quat(), self.scale()
        qi = quat_inv(q)
        si = 1.0 / s
        ti = -si * quat_rotate(qi, t)
        return Sim3(torch.cat((ti, qi, si), dim=-1))

    def __mul__(self, other: "Sim3") -> "Sim3":
        a, b = _bcast(self.data, other.data)
        t1, q1, s1 = a[..., 0:3], a[..., 3:7], a[..., 7:8]
        t2, q2, s2 = b[..., 0:3], b[..., 3:7], b[..., 7:8]
        q = quat_mul(q1, q2)
        t = t1 + s1 * quat_rotate(q1, t2)
        return Sim3(torch.cat((t, q, s1 * s2), dim=-1))

    def retr(self, xi: torch.Tensor) -> "Sim3":
        """Left retraction Exp(xi) * self (gn_kernels.cu:392-413)."""
        return Sim3.exp(xi) * self

    def __repr__(self):
        return f"Sim3({self.data})"
