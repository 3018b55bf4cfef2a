"""Sim(3) pinned by mathematics (row a14).

lietorch is not importable here and no reference test pins it, so the
restatement (mast3r_slam_amd/sim3.py, restating gn_kernels.cu:172-413) is
checked against the group's defining properties in fp64:

* Exp(xi) equals torch.linalg.matrix_exp of the 4x4 sim(3) generator
  [[hat(phi) + sigma I, tau], [0, 0]] on all four branches of the reference's
  expSim3 (sigma and theta each below / above EPS = 1e-6, gn_kernels.cu:34,
  :344-389), and the SO(3) part on both sides of its theta^2 < EPS test
  (:305-315);
* compose, inverse and act are 4x4 matrix products / the inverse matrix;
* the left retraction T.retr(xi) is Exp(xi) T (retrSim3, :392-413);
* the reference's per-pixel Jacobian rows (oracle/gn_oracle.c rows_for_pixel,
  restating gn_kernels.cu:990-1073 rays and :1422-1479 calib, mapped to the
  world-pose blocks J_j = Adj(T_i)^-T J_local, J_i = -J_j, :999-1000) are
  the derivatives of the residuals under left perturbations Exp(d) T of the
  world poses, checked by central finite differences in fp64.

Status: pinned by mathematics; parity with lietorch's own code unpinned.
The device helpers (csrc/m3s_device.h) get the same checks on the GPU in
tests/test_gpu_sim3.py.
"""
import math

import numpy as np
import pytest
import torch

from mast3r_slam_amd.sim3 import EPS, Sim3, exp_sim3

D = torch.float64


def hat(phi):
    x, y, z = phi.unbind(-1)
    o = torch.zeros_like(x)
    return torch.stack((torch.stack((o, -z, y), -1), torch.stack((z, o, -x), -1),
                        torch.stack((-y, x, o), -1)), -2)


def generator(xi):
    """4x4 sim(3) Lie algebra element of tangent [tau, phi, sigma]."""
    G = torch.zeros(*xi.shape[:-1], 4, 4, dtype=xi.dtype)
    G[..., :3, :3] = hat(xi[..., 3:6]) + xi[..., 6:7, None] * torch.eye(3, dtype=xi.dtype)
    G[..., :3, 3] = xi[..., 0:3]
    return G


def quat_to_R(q):
    x, y, z, w = q.unbind(-1)
    return torch.stack((
        torch.stack((1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)), -1),
        torch.stack((2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)), -1),
        torch.stack((2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)), -1)), -2)


def to_mat(T):
    d = T.data if isinstance(T, Sim3) else T
    M = torch.zeros(*d.shape[:-1], 4, 4, dtype=d.dtype)
    M[..., :3, :3] = d[..., 7:8, None] * quat_to_R(d[..., 3:7])
    M[..., :3, 3] = d[..., 0:3]
    M[..., 3, 3] = 1.0
    return M


def random_xi(n, gen, rot, trans, sig):
    xi = torch.empty(n, 7, dtype=D)
    xi[:, 0:3] = torch.randn(n, 3, generator=gen, dtype=D) * trans
    phi = torch.randn(n, 3, generator=gen, dtype=D)
    phi = phi / phi.norm(dim=-1, keepdim=True) * rot
    xi[:, 3:6] = phi
    xi[:, 6] = sig * torch.sign(torch.randn(n, generator=gen, dtype=D))
    return xi


def random_T(n, gen):
    return Sim3.exp(random_xi(n, gen, 0.9, 1.5, 0.3))


# (theta, sigma) per branch of expSim3 (gn_kernels.cu:344-389): the small
# values sit below EPS; the SO(3) Taylor branch is theta^2 < EPS (theta < 1e-3)
BRANCHES = {
    "sigma~0,theta~0": (3e-7, 4e-7),
    "sigma~0,theta": (0.7, 2e-7),
    "sigma,theta~0": (5e-7, 0.4),
    "sigma,theta": (1.3, -0.25),
    "sigma,theta_so3_taylor": (5e-4, 0.2),
    "large": (2.9, 1.1),
}


@pytest.mark.parametrize("branch", list(BRANCHES))
def test_exp_is_matrix_exponential_of_generator(branch):
    theta, sigma = BRANCHES[branch]
    gen = torch.Generator().manual_seed(7)
    xi = random_xi(64, gen, abs(theta), 0.8, sigma)
    if sigma < 0:
        xi[:, 6] = sigma
    assert bool(((xi[:, 3:6].norm(dim=-1) < EPS) == (abs(theta) < EPS)).all())
    assert bool(((xi[:, 6].abs() < EPS) == (abs(sigma) < EPS)).all())
    ref = torch.linalg.matrix_exp(generator(xi))
    got = to_mat(Sim3.exp(xi))
    # the small-sigma branches take C = 1 and sigma-free A, B (gn_kernels.cu
    # :344-352): a first-order truncation, |W - W_exact| <= |sigma| |tau|;
    # the small-theta branches are second order in theta (below 1e-12)
    tol = 1e-12 + (abs(sigma) * float(xi[:, 0:3].norm(dim=-1).max()) if abs(sigma) < EPS else 0.0)
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=0, atol=tol)
    q = Sim3.exp(xi).quat()
    np.testing.assert_allclose(q.norm(dim=-1).numpy(), 1.0, atol=1e-12)


def test_exp_continuous_across_branch_boundaries():
    """Each branch boundary (|sigma| = EPS, |theta| = EPS, theta^2 = EPS): the
    two formulas agree on either side (no jump in the reference's Exp)."""
    gen = torch.Generator().manual_seed(3)
    base = random_xi(8, gen, 1.0, 0.5, 0.2)
    tmax = float(base[:, 0:3].norm(dim=-1).max())
    # (boundary, value, allowed jump): the small-sigma branch is a first-order
    # truncation in sigma (jump ~ EPS |tau|); the small-theta ones are second
    # order, but the general formulas lose ~eps / theta^2 to cancellation there
    for which, val, tol in (("sigma", EPS, 1.5 * EPS * tmax), ("theta", EPS, 1e-4 * tmax),
                            ("theta", math.sqrt(EPS), 1e-8)):  # (inputs 2e-9 apart there)
        lo, hi = base.clone(), base.clone()
        for x, f in ((lo, 1 - 1e-6), (hi, 1 + 1e-6)):
            if which == "sigma":
                x[:, 6] = val * f
            else:
                x[:, 3:6] = x[:, 3:6] / x[:, 3:6].norm(dim=-1, keepdim=True) * val * f
        a, b = to_mat(Sim3.exp(lo)), to_mat(Sim3.exp(hi))
        print(which, val, float((a - b).abs().max()))
        np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=0, atol=tol)


def test_compose_inverse_act_are_matrix_products():
    gen = torch.Generator().manual_seed(11)
    A, B = random_T(32, gen), random_T(32, gen)
    MA, MB = to_mat(A), to_mat(B)
    np.testing.assert_allclose(to_mat(A * B).numpy(), (MA @ MB).numpy(), rtol=0, atol=1e-12)
    np.testing.assert_allclose(to_mat(A.inv()).numpy(), torch.linalg.inv(MA).numpy(), rtol=0, atol=1e-12)
    X = torch.randn(32, 3, generator=gen, dtype=D) * 3
    Xh = torch.cat((X, torch.ones(32, 1, dtype=D)), -1)
    np.testing.assert_allclose(A.act(X).numpy(), (MA @ Xh[..., None])[:, :3, 0].numpy(), rtol=0, atol=1e-12)
    # identities
    I = to_mat(A * A.inv())
    np.testing.assert_allclose(I.numpy(), np.broadcast_to(np.eye(4), I.shape), atol=1e-12)
    C = random_T(32, gen)
    np.testing.assert_allclose(to_mat((A * B) * C).numpy(), to_mat(A * (B * C)).numpy(), atol=1e-12)


def test_left_retraction_is_exp_times_T():
    gen = torch.Generator().manual_seed(5)
    T = random_T(32, gen)
    xi = random_xi(32, gen, 0.05, 0.02, 0.01)
    got = to_mat(T.retr(xi))
    ref = torch.linalg.matrix_exp(generator(xi)) @ to_mat(T)
    np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=0, atol=1e-12)


def small_steps(n, gen):
    """GN-sized steps in the regime where the reference's fp32 Exp cancels:
    |sigma| log-uniform in [1.5e-6, 1e-3] (just above EPS), theta log-uniform
    in [2e-6, 3e-2], |tau| ~ 0.1, random signs."""
    u = torch.rand(n, 2, generator=gen, dtype=D)
    sig = 10 ** (math.log10(1.5e-6) + u[:, 0] * (math.log10(1e-3) - math.log10(1.5e-6)))
    th = 10 ** (math.log10(2e-6) + u[:, 1] * (math.log10(3e-2) - math.log10(2e-6)))
    xi = random_xi(n, gen, 1.0, 0.1, 1.0)
    xi[:, 3:6] *= th[:, None]
    xi[:, 6] = sig * torch.sign(torch.randn(n, generator=gen, dtype=D))
    return xi.to(torch.float32)


def pose_err(T, M_exact):
    """Per-pose max |entry| of the 3x4 [sR | t] difference to the exact matrix."""
    return (to_mat(torch.as_tensor(np.asarray(T, np.float64))) - M_exact)[..., :3, :].abs().amax((-2, -1)).numpy()


def test_oracle_retractions_against_matrix_exponential():
    """The C oracle's two retractions on identical fp32 (xi, T): the fp32 one
    (the reference's retrSim3 arithmetic, gn_kernels.cu:323-413) and the fp64
    one of the exact-arithmetic yardstick (libgn_oracle_f64.so), against
    expm(generator(xi)) T in fp64. The fp64 one is within fp32 rounding of the
    pose entries; the fp32 one carries the reference's cancellation,
    C = (e^sigma - 1) / sigma with the rounding of e^sigma over |sigma|:
    |dt| ~ 6e-8 |tau| / |sigma|."""
    from oracle import oracle as orc

    gen = torch.Generator().manual_seed(61)
    xi = small_steps(400, gen)
    T = random_T(400, gen).data.to(torch.float32)
    M_x = torch.linalg.matrix_exp(generator(xi.to(D))) @ to_mat(T.to(D))
    T32 = np.stack([orc.retract(xi[k].numpy(), T[k].numpy()) for k in range(400)])
    T64 = np.stack([orc.retract(xi[k].numpy(), T[k].numpy(), f64=True) for k in range(400)])
    e32, e64 = pose_err(T32, M_x), pose_err(T64, M_x)
    scale = 1.0 + M_x[..., :3, :].abs().amax((-2, -1)).numpy()
    model = 6e-8 * xi[:, 0:3].to(D).norm(dim=-1).numpy() / xi[:, 6].abs().to(D).numpy()
    print(f"fp64 retraction max err {e64.max():.2e}; fp32 (reference arithmetic) max err {e32.max():.2e}, "
          f"median {np.median(e32):.2e}; cancellation model max {model.max():.2e}")
    assert np.all(e64 <= 4e-7 * scale)
    assert np.all(e32 <= 4 * model + 4e-7 * scale)  # the error is the model's, no other
    assert e32.max() > 30 * e64.max()  # and it is real at these steps


def test_exp_log_consistency_small_steps():
    """Exp is a local diffeomorphism: d/dh Exp(h xi)|0 = generator(xi)."""
    gen = torch.Generator().manual_seed(9)
    xi = random_xi(16, gen, 0.6, 0.7, 0.4)
    h = 1e-6
    d = (to_mat(Sim3.exp(h * xi)) - to_mat(Sim3.exp(-h * xi))) / (2 * h)
    np.testing.assert_allclose(d.numpy(), generator(xi).numpy(), rtol=0, atol=1e-8)


# ----------------------------------------------- Jacobian rows of the kernels
def _residual(mode, Ti, Tj, Xi, Xj, K, u_t, v_t):
    """fp64 residuals of gn_kernels.cu for one pixel: rays [r(Y) - r(Xi),
    |Y| - |Xi|] (:944-947), calib [u - u_t, v - v_t, log Y_z - log Xi_z]
    (:1361-1399); Y = (Ti^-1 Tj) Xj."""
    Y = (Ti.inv() * Tj).act(Xj)
    if mode == "rays":
        nY, nX = Y.norm(), Xi.norm()
        return torch.cat((Y / nY - Xi / nX, (nY - nX)[None]))
    x, y = Y[0] / Y[2], Y[1] / Y[2]
    return torch.stack((K[0, 0] * x + K[0, 2] - u_t, K[1, 1] * y + K[1, 2] - v_t,
                        torch.log(Y[2]) - torch.log(Xi[2])))


@pytest.mark.parametrize("mode", ["rays", "calib"])
def test_reference_jacobian_rows_are_derivatives(mode):
    from oracle import oracle as orc

    lib = orc.lib()
    import ctypes

    P = ctypes.c_void_p
    lib.oracle_pixel_rows.restype = ctypes.c_int
    lib.oracle_pixel_rows.argtypes = [ctypes.POINTER(orc.Params), P, P, P, P, ctypes.c_int64, P, P, P]
    H, W = 48, 64
    K = torch.tensor([[0.8 * W, 0, W / 2], [0, 0.8 * W, H / 2], [0, 0, 1]], dtype=D)
    if mode == "rays":
        params = orc.make_params(orc.MODE_RAYS, 0.003, 10.0, 0.0, 1.5)
    else:
        params = orc.make_params(orc.MODE_CALIB, 1.0, 10.0, 0.0, 1.5, K=K.numpy(), height=H, width=W,
                                 pixel_border=-10, z_eps=1e-6)
    gen = torch.Generator().manual_seed(21 if mode == "rays" else 22)
    worst = 0.0
    for _ in range(24):
        Ti = Sim3.exp(random_xi(1, gen, 0.3, 0.5, 0.1))[0]
        Tj = Sim3.exp(random_xi(1, gen, 0.3, 0.5, 0.1))[0]
        # a point in front of camera i, its (noisy) match, and the point in camera j
        Xi0 = torch.tensor([0.2, -0.15, 2.0], dtype=D) + torch.randn(3, generator=gen, dtype=D) * 0.2
        Xj = (Tj.inv() * Ti).act(Xi0)
        Xi = Xi0 + torch.randn(3, generator=gen, dtype=D) * 0.01
        u_t, v_t, id_i = 0.0, 0.0, 0
        if mode == "calib":
            pi = K @ (Xi / Xi[2])
            u_t, v_t = float(torch.round(pi[0]).clamp(0, W - 1)), float(torch.round(pi[1]).clamp(0, H - 1))
            id_i = int(v_t) * W + int(u_t)
        f32 = lambda t: np.ascontiguousarray(t.numpy(), np.float32)  # noqa: E731
        Ji = np.zeros((4, 7), np.float32)
        Jj = np.zeros((4, 7), np.float32)
        e = np.zeros(4, np.float32)
        ins = [f32(t) for t in (Ti.data, Tj.data, Xi, Xj)]  # kept alive across the call
        nr = lib.oracle_pixel_rows(ctypes.byref(params), *(a.ctypes.data for a in ins), id_i, Ji.ctypes.data,
                                   Jj.ctypes.data, e.ctypes.data)
        assert nr == (4 if mode == "rays" else 3)
        e_ref = _residual(mode, Ti, Tj, Xi, Xj, K, u_t, v_t)
        np.testing.assert_allclose(e[:nr], e_ref.numpy(), rtol=1e-4, atol=1e-5 * float(e_ref.abs().max() + 1))
        h = 1e-6
        for side, J in (("i", Ji), ("j", Jj)):
            num = np.zeros((nr, 7))
            for k in range(7):
                d = torch.zeros(7, dtype=D)
                d[k] = h
                Tp, Tm = (Sim3.exp(d[None])[0] * (Ti if side == "i" else Tj),
                          Sim3.exp(-d[None])[0] * (Ti if side == "i" else Tj))
                if side == "i":
                    ep, em = _residual(mode, Tp, Tj, Xi, Xj, K, u_t, v_t), _residual(mode, Tm, Tj, Xi, Xj, K, u_t, v_t)
                else:
                    ep, em = _residual(mode, Ti, Tp, Xi, Xj, K, u_t, v_t), _residual(mode, Ti, Tm, Xi, Xj, K, u_t, v_t)
                num[:, k] = ((ep - em) / (2 * h)).numpy()
            scale = np.abs(num).max(axis=1, keepdims=True) + 1e-12
            err = np.abs(J[:nr] - num) / scale
            worst = max(worst, float(err.max()))
            assert err.max() < 2e-4, (mode, side, J[:nr], num)
    print(f"{mode}: worst row error vs finite differences {worst:.2e} (relative to the row's largest entry)")
