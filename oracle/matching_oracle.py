"""NumPy restatement of the reference matching kernels (CPU oracle).

TEST INFRASTRUCTURE ONLY — imported by tests/ as the checker. The product path
(mast3r_slam_backends.iter_proj / refine_matches -> m3s_match.hip) never
imports it.

* ``iter_proj``       follows matching_kernels.cu:119-296 (iter_proj_kernel),
                      vectorised over pixels, with the kernel's fp32 operation
                      order and its fp64-promoted literals (`1.0 - du` :161-163,
                      `1.0 / r_norm` :186, `1.0 / det` :214, `lambda *= 0.1`
                      :271, `*= 10.0` :276), no fused multiply-add.
* ``refine_matches``  follows matching_kernels.cu:25-78 (refine_matches_kernel):
                      dilation d = dilation_max..1, window offsets u outer / v
                      inner, strict `score > max_score`, centre moved to the best
                      match after every dilation level (:75-76). Scores
                      accumulate in feature order in the arithmetic of the
                      dispatched scalar_t (AT_DISPATCH_FLOATING_TYPES_AND_HALF,
                      :103):
                      - c10::Half (the reference's caller passes .half()
                        descriptors, matching.py:80): c10::Half's operators
                        compute in float and convert back (c10/util/Half-inl.h),
                        so `score += a * b` (:58-60) rounds the product to half
                        and then the sum to half; max_score starts at
                        ::cuda::std::numeric_limits<c10::Half>::min() (:47),
                        which libcu++ does not specialise for c10::Half: the
                        primary template's T() = 0;
                      - float: nvcc contracts `score += a * b` to one fused
                        multiply-add; max_score starts at FLT_MIN.

Parity unpinned: the reference's own tests hold no fixtures for these kernels
 and the CUDA module cannot be built or run here, so this
restatement (and the HIP kernel, which implements the same arithmetic) follows
the kernel source and the c10 / libcu++ semantics above, not reference outputs.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
F64 = np.float64


def _clamp(x, lo, hi):
    return np.fmin(np.fmax(x, F32(lo)), F32(hi)).astype(F32)


def _bilinear(img, b, u, v, c0, nc):
    """matching_kernels.cu:154-182 for channels [c0, c0+nc)."""
    u11 = np.floor(u).astype(np.int64)
    v11 = np.floor(v).astype(np.int64)
    du = (u - u11.astype(F32)).astype(F32)
    dv = (v - v11.astype(F32)).astype(F32)
    w11 = (du * dv).astype(F32)
    w12 = ((1.0 - du.astype(F64)) * dv.astype(F64)).astype(F32)
    w21 = (du.astype(F64) * (1.0 - dv.astype(F64))).astype(F32)
    w22 = ((1.0 - du.astype(F64)) * (1.0 - dv.astype(F64))).astype(F32)
    r11 = img[b, v11 + 1, u11 + 1, c0:c0 + nc]
    r12 = img[b, v11 + 1, u11, c0:c0 + nc]
    r21 = img[b, v11, u11 + 1, c0:c0 + nc]
    r22 = img[b, v11, u11, c0:c0 + nc]
    out = (w11[:, None] * r11).astype(F32)
    out = (out + (w12[:, None] * r12).astype(F32)).astype(F32)
    out = (out + (w21[:, None] * r21).astype(F32)).astype(F32)
    out = (out + (w22[:, None] * r22).astype(F32)).astype(F32)
    return out


def _dot3(a, b):
    s = (a[:, 0] * b[:, 0]).astype(F32)
    s = (s + (a[:, 1] * b[:, 1]).astype(F32)).astype(F32)
    return (s + (a[:, 2] * b[:, 2]).astype(F32)).astype(F32)


def _normalized_err(r, p):
    r_norm = np.sqrt(_dot3(r, r)).astype(F32)
    r_norm_inv = (1.0 / r_norm.astype(F64)).astype(F32)
    rn = (r * r_norm_inv[:, None]).astype(F32)
    err = (rn - p).astype(F32)
    return err, _dot3(err, err)


def iter_proj(rays_img, pts_3d_norm, p_init, max_iter, lambda_init, cost_thresh):
    """Returns (p_new [B,N,2] f32, converged [B,N] bool)."""
    img = np.ascontiguousarray(rays_img, F32)
    B, H, W, C = img.shape
    assert C == 9
    pts = np.ascontiguousarray(pts_3d_norm, F32).reshape(-1, 3)
    p0 = np.ascontiguousarray(p_init, F32).reshape(-1, 2)
    N = p_init.shape[1]
    b = np.repeat(np.arange(B), N)
    u = _clamp(p0[:, 0], 1, W - 2)
    v = _clamp(p0[:, 1], 1, H - 2)
    lam = np.full(u.shape, F32(lambda_init), F32)
    conv = np.zeros(u.shape, bool)
    ct = F32(cost_thresh)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        for _ in range(int(max_iter)):
            r = _bilinear(img, b, u, v, 0, 3)
            gx = _bilinear(img, b, u, v, 3, 3)
            gy = _bilinear(img, b, u, v, 6, 3)
            err, cost = _normalized_err(r, pts)
            A00 = _dot3(gx, gx)
            A01 = _dot3(gx, gy)
            A11 = _dot3(gy, gy)
            b0 = (-_dot3(err, gx)).astype(F32)
            b1 = (-_dot3(err, gy)).astype(F32)
            A00 = (A00 + lam).astype(F32)
            A11 = (A11 + lam).astype(F32)
            det = ((A00 * A11).astype(F32) - (A01 * A01).astype(F32)).astype(F32)
            det_inv = (1.0 / det.astype(F64)).astype(F32)
            du_ = (det_inv * ((A11 * b0).astype(F32) - (A01 * b1).astype(F32)).astype(F32)).astype(F32)
            dv_ = (det_inv * (((-A01) * b0).astype(F32) + (A00 * b1).astype(F32)).astype(F32)).astype(F32)
            u_new = _clamp((u + du_).astype(F32), 1, W - 2)
            v_new = _clamp((v + dv_).astype(F32), 1, H - 2)
            _, new_cost = _normalized_err(_bilinear(img, b, u_new, v_new, 0, 3), pts)
            better = new_cost < cost
            u = np.where(better, u_new, u)
            v = np.where(better, v_new, v)
            lam = np.where(better, (lam.astype(F64) * 0.1).astype(F32),
                           (lam.astype(F64) * 10.0).astype(F32))
            conv = np.where(better, new_cost < ct, cost < ct)
    return np.stack([u, v], -1).reshape(B, N, 2), conv.reshape(B, N)


def _score_step(a, b, s, dt):
    """score + a * b in the reference's arithmetic for dt: fp16 (c10::Half) a
    product rounded to half, then the sum rounded to half (both exact in fp64
    before their one rounding); fp32 one correctly rounded fused multiply-add."""
    if dt == np.float16:
        p = (a.astype(F64) * b.astype(F64)).astype(np.float16)
        return (s.astype(F64) + p.astype(F64)).astype(np.float16)
    return (a.astype(F64) * b.astype(F64) + s.astype(F64)).astype(dt)


def refine_matches(D11, D21, p1, radius, dilation_max):
    """Returns p1_new [B,N,2] int64."""
    D11 = np.ascontiguousarray(D11)
    dt = D11.dtype
    assert dt in (np.float16, np.float32)
    B, H, W, Fd = D11.shape
    D21 = np.ascontiguousarray(D21, dt).reshape(-1, Fd)
    N = p1.shape[1]
    b = np.repeat(np.arange(B), N)
    u0 = np.ascontiguousarray(p1, np.int64).reshape(-1, 2)[:, 0].copy()
    v0 = np.ascontiguousarray(p1, np.int64).reshape(-1, 2)[:, 1].copy()
    # numeric_limits<T>::min() (:47): c10::Half -> T() = 0; float -> FLT_MIN
    start = 0.0 if dt == np.float16 else np.finfo(dt).tiny
    best = np.full(u0.shape, start, dt)
    u_new, v_new = u0.copy(), v0.copy()
    for d in range(int(dilation_max), 0, -1):
        rd = radius * d
        diam = 2 * rd + 1
        for i in range(0, diam, d):
            u = u0 - rd + i
            for j in range(0, diam, d):
                v = v0 - rd + j
                inside = (v >= 0) & (v < H) & (u >= 0) & (u < W)
                x = D11[b, np.clip(v, 0, H - 1), np.clip(u, 0, W - 1)]
                s = np.zeros(u.shape, dt)
                for k in range(Fd):
                    s = _score_step(D21[:, k], x[:, k], s, dt)
                upd = inside & (s > best)
                best = np.where(upd, s, best)
                u_new = np.where(upd, u, u_new)
                v_new = np.where(upd, v, v_new)
        u0, v0 = u_new.copy(), v_new.copy()
    return np.stack([u_new, v_new], -1).reshape(B, N, 2)
