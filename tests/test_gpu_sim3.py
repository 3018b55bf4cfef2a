"""The device Sim(3) helpers of the hot path (csrc/m3s_device.h, run through
the m3s_debug_sim3 C entry) against the group's mathematics in fp64 — the GPU
half of row a14 (tests/test_sim3_math.py checks the host restatement and the
reference's Jacobian rows the same way).

fp32 on device vs fp64 matrices: tolerances are a few fp32 ulps of the
magnitudes involved (stated per check). The small-sigma Exp branch keeps the
reference's first-order truncation (|W - W_exact| <= |sigma| |tau|,
gn_kernels.cu:344-352), below fp32 resolution at |sigma| < 1e-6."""
import numpy as np
import pytest
import torch

from test_sim3_math import BRANCHES, generator, random_T, random_xi, to_mat

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
D = torch.float64


@pytest.fixture(scope="module")
def be():
    import mast3r_slam_backends as be

    return be


def dev32(t):
    return t.to(torch.float32).to(DEV).contiguous()


def host64(t):
    return t.cpu().to(D)


@pytest.mark.parametrize("branch", list(BRANCHES))
def test_device_exp_is_matrix_exponential(be, branch):
    theta, sigma = BRANCHES[branch]
    gen = torch.Generator().manual_seed(17)
    xi = random_xi(256, gen, abs(theta), 0.8, sigma)
    if sigma < 0:
        xi[:, 6] = sigma
    xi32 = xi.to(torch.float32).to(D)  # the exact inputs the device sees
    got = to_mat(host64(be.debug_sim3("exp", dev32(xi))))
    ref = torch.linalg.matrix_exp(generator(xi32))
    err = float((got - ref).abs().max())
    print(f"{branch}: max |Exp_dev - expm| = {err:.2e}")
    assert err < 3e-6 * (1.0 + float(ref.abs().max()))
    q = host64(be.debug_sim3("exp", dev32(xi)))[:, 3:7]
    assert float((q.norm(dim=-1) - 1).abs().max()) < 1e-6


def test_device_group_ops_are_matrix_products(be):
    gen = torch.Generator().manual_seed(19)
    A, B = random_T(512, gen), random_T(512, gen)
    A32, B32 = A.data.to(torch.float32), B.data.to(torch.float32)
    MA, MB = to_mat(A32.to(D)), to_mat(B32.to(D))
    tol = 4e-6
    comp = to_mat(host64(be.debug_sim3("compose", dev32(A32), dev32(B32))))
    assert float((comp - MA @ MB).abs().max()) < tol * float((MA @ MB).abs().max())
    inv = to_mat(host64(be.debug_sim3("inverse", dev32(A32))))
    Minv = torch.linalg.inv(MA)
    assert float((inv - Minv).abs().max()) < tol * float(Minv.abs().max())
    rel = to_mat(host64(be.debug_sim3("relative", dev32(A32), dev32(B32))))
    Mrel = Minv @ MB
    assert float((rel - Mrel).abs().max()) < tol * float(Mrel.abs().max())
    X = torch.randn(512, 3, generator=gen, dtype=D) * 3
    Xh = torch.cat((X.to(torch.float32).to(D), torch.ones(512, 1, dtype=D)), -1)
    ref = (MA @ Xh[..., None])[:, :3, 0]
    for op in ("act", "act_matrix"):  # quaternion form and the linearize kernels' 3x4 form
        Y = host64(be.debug_sim3(op, dev32(A32), dev32(X)))
        assert float((Y - ref).abs().max()) < tol * float(ref.abs().max()), op


def test_device_retraction_is_exp_times_T(be):
    gen = torch.Generator().manual_seed(23)
    T = random_T(512, gen)
    xi = random_xi(512, gen, 0.05, 0.02, 0.01)
    T32, xi32 = T.data.to(torch.float32), xi.to(torch.float32)
    got = to_mat(host64(be.debug_sim3("retract", dev32(xi32), dev32(T32))))
    ref = torch.linalg.matrix_exp(generator(xi32.to(D))) @ to_mat(T32.to(D))
    assert float((got - ref).abs().max()) < 4e-6 * float(ref.abs().max())


def test_device_adjoint_maps_local_rows_to_world_rows(be):
    """Adj(T)^-T (apply_Sim3_adj_inv): for a left perturbation of T_j by d,
    T_i^-1 Exp(d) T_j = Exp(Adj(T_i^-1) d) T_i^-1 T_j, so a row a of the local
    Jacobian becomes a Adj(T_i)^-1 = (Adj(T_i)^-T a^T)^T. Checked against the
    matrix adjoint: hat(Adj(T) d) = T hat(d) T^-1 for every basis d."""
    gen = torch.Generator().manual_seed(29)
    T = random_T(64, gen)
    T32 = T.data.to(torch.float32)
    M = host64(be.debug_sim3("adjT_inv", dev32(T32))).reshape(-1, 7, 7)
    MT = to_mat(T32.to(D))
    MTi = torch.linalg.inv(MT)
    for k in range(7):
        d = torch.zeros(64, 7, dtype=D)
        d[:, k] = 1.0
        # Adj(T^-1) e_k from matrices: T^-1 hat(e_k) T = hat(Adj(T^-1) e_k)
        G = MTi @ generator(d) @ MT
        col = torch.cat((G[:, :3, 3], torch.stack((G[:, 2, 1], G[:, 0, 2], G[:, 1, 0]), -1),
                         (G[:, 0, 0] + G[:, 1, 1] + G[:, 2, 2])[:, None] / 3.0), -1)
        # row k of Adj(T)^-T equals column k of Adj(T)^-1 = Adj(T^-1)
        got = M[:, k, :]
        assert float((got - col).abs().max()) < 5e-6 * (1.0 + float(col.abs().max())), k


def test_backend_retraction_same_inputs_three_ways(be):
    """Identical fp32 (xi, T) in the small-step regime where the reference's
    fp32 Exp cancels (tests/test_sim3_math.small_steps), retracted by the
    backend's device retraction (op "retract", fp64 evaluation), by the
    oracle's fp32 restatement of retrSim3 (gn_kernels.cu:323-413) and in fp64
    by expm(generator(xi)) T. Per pose |T_hip - T_f64| <= |T_ref32 - T_f64| +
    1e-6, and T_hip within fp32 rounding of the exact pose. The device's fp32
    form (op "retract_f32", the tracker's) is the reference's arithmetic: it
    sits where the oracle's fp32 restatement sits."""
    from oracle import oracle as orc
    from test_sim3_math import pose_err, small_steps

    gen = torch.Generator().manual_seed(67)
    n = 400
    xi = small_steps(n, gen)
    T = random_T(n, gen).data.to(torch.float32)
    M_x = torch.linalg.matrix_exp(generator(xi.to(D))) @ to_mat(T.to(D))
    T_hip = host64(be.debug_sim3("retract", dev32(xi), dev32(T))).numpy()
    T_h32 = host64(be.debug_sim3("retract_f32", dev32(xi), dev32(T))).numpy()
    T_ref = np.stack([orc.retract(xi[k].numpy(), T[k].numpy()) for k in range(n)])
    e_hip, e_h32, e_ref = pose_err(T_hip, M_x), pose_err(T_h32, M_x), pose_err(T_ref, M_x)
    scale = 1.0 + M_x[..., :3, :].abs().amax((-2, -1)).numpy()
    print(f"max|T - T_f64|: hip (fp64 eval) {e_hip.max():.2e}, hip fp32 form {e_h32.max():.2e}, "
          f"oracle fp32 {e_ref.max():.2e} (median {np.median(e_ref):.2e})")
    assert np.all(e_hip <= e_ref + 1e-6)
    assert np.all(e_hip <= 4e-7 * scale)
    # the device's fp32 form and the oracle's restatement: the same arithmetic,
    # apart from ulp-level differences of expf/sinf/cosf between the two libms
    # (each amplified by the same cancellation)
    assert np.median(np.abs(e_h32 - e_ref)) <= 1e-6
