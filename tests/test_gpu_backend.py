"""GPU parity of the backend GN (gauss_newton_{rays,calib,points}) against the
CPU oracle (oracle/gn_oracle.c, pinned to the reference in
tests/test_oracle_golden.py), through the C ABI.

Tolerances (DESIGN.md "Parity tolerances"): per-edge normal equations within
2e-5 of the entry scale (fp32 sums of ~10^4-10^5 terms in a different order
and grouping than the reference's 14x14 form); poses after GN within
1e-5 + 1e-4 * sum of step lengths.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import oracle as orc  # noqa: E402

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def be():
    import mast3r_slam_backends as be

    return be


def params_for(mode, g):
    if mode == "rays":
        return orc.make_params(orc.MODE_RAYS, 0.003, 10.0, 0.0, 1.5)
    if mode == "calib":
        return orc.make_params(orc.MODE_CALIB, 1.0, 10.0, 0.0, 1.5, K=g.K.numpy(), height=g.H,
                               width=g.W, pixel_border=-10, z_eps=1e-6)
    return orc.make_params(orc.MODE_POINTS, 0.05, 0.0, 0.0, 1.5)


def run_gpu(be, mode, g, max_iter, delta, Twc0=None, Xs=None, valid=None):
    Twc = (g.T_init.data if Twc0 is None else torch.as_tensor(Twc0)).clone().to(DEV).contiguous()
    Xs = (g.Xs if Xs is None else Xs).to(DEV).contiguous()
    valid = (g.valid_match if valid is None else valid).to(DEV).contiguous()
    Cs, ii, jj, idx, Q = (t.to(DEV).contiguous() for t in (g.Cs, g.ii, g.jj, g.idx_ii2jj, g.Q))
    info = torch.zeros(8, dtype=torch.int32, device=DEV)
    if mode == "rays":
        (dx,) = be.gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx, valid, Q, 0.003, 10.0, 0.0, 1.5,
                                     max_iter, delta, info=info)
    elif mode == "calib":
        (dx,) = be.gauss_newton_calib(Twc, Xs, Cs, g.K.to(DEV), ii, jj, idx, valid, Q, g.H, g.W,
                                      -10, 1e-6, 1.0, 10.0, 0.0, 1.5, max_iter, delta, info=info)
    else:
        (dx,) = be.gauss_newton_points(Twc, Xs, Cs, ii, jj, idx, valid, Q, 0.05, 0.0, 1.5,
                                       max_iter, delta, info=info)
    torch.cuda.synchronize()
    return Twc.cpu().numpy(), dx.cpu().numpy(), info.cpu().numpy()


def run_oracle(mode, g, max_iter, delta, Twc0=None, Xs=None, valid=None, f64=False):
    p = params_for(mode, g)
    T0 = g.T_init.data.numpy() if Twc0 is None else np.asarray(Twc0)
    return orc.gn(p, T0, (g.Xs if Xs is None else Xs).numpy(), g.Cs.numpy(), g.ii.numpy(),
                  g.jj.numpy(), g.idx_ii2jj.numpy(),
                  (g.valid_match if valid is None else valid).numpy(), g.Q.numpy(), max_iter, delta,
                  f64=f64)


def constrained(g):
    """Calib inputs are ray-constrained by the caller (global_opt.py:172)."""
    from oracle.tracker_oracle import constrain_points_to_ray

    K = g.K.numpy()
    return torch.from_numpy(np.stack([constrain_points_to_ray((g.H, g.W), x, K) for x in g.Xs.numpy()]))


@pytest.fixture(scope="module")
def graph_small():
    from mast3r_slam_amd import synthetic

    return synthetic.make_graph(6, 48, 64, seed=31)


@pytest.mark.parametrize("mode", ["rays", "calib", "points"])
def test_edge_normal_equations_match_oracle(be, graph_small, mode):
    """m3s_gn_linearize's per-edge (L, l) mapped through M = Adj(T_i)^-T equal
    the oracle's Hs[3] / gs[1] blocks; Hs[0]=Hs[3], Hs[1]=Hs[2]=-Hs[3]."""
    g = graph_small
    Xs = constrained(g) if mode == "calib" else g.Xs
    Twc = g.T_init.data.clone().to(DEV)
    tens = dict(Xs=Xs.to(DEV), Cs=g.Cs.to(DEV), ii=g.ii.to(DEV), jj=g.jj.to(DEV),
                idx=g.idx_ii2jj.to(DEV), valid=g.valid_match.to(DEV), Q=g.Q.to(DEV))
    mode_id = {"rays": be.MODE_RAYS, "calib": be.MODE_CALIB, "points": be.MODE_POINTS}[mode]
    sig = {"rays": (0.003, 10.0), "calib": (1.0, 10.0), "points": (0.05, 0.0)}[mode]
    a, keep = be.make_gn_args(mode_id, Twc, tens["Xs"], tens["Cs"], tens["ii"], tens["jj"],
                              tens["idx"], tens["valid"], tens["Q"],
                              g.K.to(DEV) if mode == "calib" else None, sigma_a=sig[0],
                              sigma_b=sig[1], C_thresh=0.0, Q_thresh=1.5, height=g.H, width=g.W,
                              pixel_border=-10, z_eps=1e-6, max_iter=1, delta_thresh=0.0)
    E = g.n_edges
    es = torch.zeros(E, be.EDGE_SUM_STRIDE, dtype=torch.float64, device=DEV)
    be.gn_prepare(a, keep)
    be.gn_linearize(a, keep, 0, E, es)
    torch.cuda.synchronize()
    es = es.cpu().numpy()
    Hs, gs = orc.edge_blocks(params_for(mode, g), g.T_init.data.numpy(), Xs.numpy(), g.Cs.numpy(),
                             g.ii.numpy(), g.jj.numpy(), g.idx_ii2jj.numpy(),
                             g.valid_match.numpy(), g.Q.numpy())
    iu = np.triu_indices(7)
    for e in range(E):
        L = np.zeros((7, 7))
        L[iu] = es[e, :28]
        L = L + L.T - np.diag(np.diag(L))
        M = orc.adjT_inv_matrix(g.T_init.data.numpy()[int(g.ii[e])]).astype(np.float64)
        Hjj = M @ L @ M.T
        gj = M @ es[e, 28:35]
        scale = np.abs(Hs[3, e]).max() + 1e-30
        assert np.abs(Hjj - Hs[3, e]).max() <= 2e-5 * scale, (mode, e)
        gscale = np.abs(gs[1, e]).max() + 1e-3 * scale ** 0.5
        assert np.abs(gj - gs[1, e]).max() <= 1e-4 * gscale + 1e-6, (mode, e)


@pytest.mark.parametrize("mode", ["rays", "calib", "points"])
def test_gn_poses_match_oracle(be, graph_small, mode):
    g = graph_small
    Xs = constrained(g) if mode == "calib" else g.Xs
    T_gpu, dx_gpu, info = run_gpu(be, mode, g, 10, 0.0, Xs=Xs)
    T_ref, dx_ref, it, failed = run_oracle(mode, g, 10, 0.0, Xs=Xs)
    assert info[be.INFO_ITERS] == it == 10
    assert info[be.INFO_SOLVE_FAIL] == failed == 0
    assert info[be.INFO_N_UNIQUE] == 6
    np.testing.assert_array_equal(T_gpu[0], g.T_init.data.numpy()[0])  # fixed pose
    np.testing.assert_allclose(T_gpu, T_ref, atol=1e-4)
    np.testing.assert_allclose(dx_gpu, dx_ref, atol=1e-5)


def test_gn_natural_termination_matches_oracle(be, graph_small):
    """delta_thresh between two consecutive step norms stops the loop at the
    same iteration as the reference loop (gn_kernels.cu:1219-1222)."""
    g = graph_small
    p = params_for("rays", g)
    T = g.T_init.data.numpy()
    norms = []
    for _ in range(8):
        T, dx, _, _ = orc.gn(p, T, g.Xs.numpy(), g.Cs.numpy(), g.ii.numpy(), g.jj.numpy(),
                             g.idx_ii2jj.numpy(), g.valid_match.numpy(), g.Q.numpy(), 1, 0.0)
        norms.append(float(np.linalg.norm(dx)))
    k = 4
    assert norms[k + 1] < 0.9 * norms[k]
    delta = float(np.sqrt(norms[k] * norms[k + 1]))
    T_gpu, dx_gpu, info = run_gpu(be, "rays", g, 10, delta)
    T_ref, dx_ref, it, _ = run_oracle("rays", g, 10, delta)
    assert info[be.INFO_ITERS] == it == k + 2
    assert info[be.INFO_CONVERGED] == 1
    np.testing.assert_allclose(T_gpu, T_ref, atol=1e-4)


def test_gn_global_ids_are_remapped(be):
    """ii/jj carry global KF ids (sorted-unique rank order, gn_kernels.cu:161-170)."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(5, 24, 32, seed=33, kf_ids=[3, 7, 8, 20, 41])
    T_gpu, _, info = run_gpu(be, "rays", g, 3, 0.0)
    T_ref, _, it, _ = run_oracle("rays", g, 3, 0.0)
    assert info[be.INFO_N_UNIQUE] == 5 and info[be.INFO_BAD_EDGE] == 0
    np.testing.assert_allclose(T_gpu, T_ref, atol=1e-4)


@pytest.mark.parametrize("mode,N,ids", [("rays", 6, [-5, 0, 9, 1 << 40, 77, 78]), ("calib", 32, None),
                                        ("points", 12, "spread"), ("rays", 140, "spread")])
def test_device_prologue_matches_host_prepare_bitwise(be, knobs, mode, N, ids):
    """The call prologue on the device (the ids ranked by a bitonic sort in LDS,
    the task table, flags / info / dx init; gn_prepare_async) against the host
    prepare (knob prologue = 0): poses, dx and info agree bitwise, for global
    ids that are negative, far apart or unsorted, on the one-workgroup and the
    chip-wide solver paths, with a cold and a cached plan."""
    from mast3r_slam_amd import synthetic

    if ids == "spread":
        ids = sorted(np.random.default_rng(N).choice(1 << 20, size=N, replace=False).tolist())
    H, W = (24, 32) if N < 64 else (12, 16)
    g = synthetic.make_graph(N, H, W, seed=700 + N, kf_ids=ids)
    Xs = constrained(g) if mode == "calib" else None
    res = []
    for pro in (1, 0, 1):  # the last call hits the plan cached by the first two
        knobs("prologue", pro)
        res.append(run_gpu(be, mode, g, 3, 0.0, Xs=Xs))
    for T, dx, info in res[1:]:
        np.testing.assert_array_equal(info, res[0][2])
        np.testing.assert_array_equal(dx, res[0][1])
        np.testing.assert_array_equal(T, res[0][0])
    assert res[0][2][be.INFO_N_UNIQUE] == N and res[0][2][be.INFO_ITERS] == 3


@pytest.mark.parametrize("N,ids", [(5, [40, -3, 1 << 45, 7, 8]), (32, None), (256, "spread")])
def test_device_prologue_ranks_and_edge_order(be, N, ids):
    """gn_prologue_kernel's outputs in the workspace after m3s_gn_prepare:
    ranks = the sorted-unique inverse of cat(ii, jj) (gn_kernels.cu:1154-1160),
    the edge order a permutation of the edges grouped by KF j, info's
    N_UNIQUE, zeroed dx_out; the ids copied to the host are those passed."""
    from mast3r_slam_amd import synthetic
    from mast3r_slam_amd.distributed import HipOps

    if ids == "spread":
        ids = sorted(np.random.default_rng(N).choice(1 << 40, size=N, replace=False).tolist())
    g = synthetic.make_graph(N, 8, 8, seed=800 + N, kf_ids=ids)
    E = g.n_edges
    ii, jj = g.ii.to(DEV).contiguous(), g.jj.to(DEV).contiguous()
    ops = HipOps(be.MODE_RAYS, g.T_init.data.clone().to(DEV).contiguous(), g.Xs.to(DEV).contiguous(),
                 g.Cs.to(DEV).contiguous(), ii, jj, g.idx_ii2jj.to(DEV).contiguous(),
                 g.valid_match.to(DEV).contiguous(), g.Q.to(DEV).contiguous(), E, sigma_a=0.003, sigma_b=10.0)
    ops.dx.fill_(7.0)
    ops.prepare(0.0)
    torch.cuda.synchronize()
    lay = be.workspace_layout(N, 64, E)
    ws = ops.ws.cpu().numpy()
    rank_i = ws[lay["rank_i"]:lay["rank_i"] + 4 * E].view(np.int32)
    rank_j = ws[lay["rank_j"]:lay["rank_j"] + 4 * E].view(np.int32)
    order = ws[lay["eorder"]:lay["eorder"] + 4 * E].view(np.int32)
    u, inv = np.unique(np.concatenate([g.ii.numpy(), g.jj.numpy()]), return_inverse=True)
    np.testing.assert_array_equal(rank_i, inv[:E])
    np.testing.assert_array_equal(rank_j, inv[E:])
    np.testing.assert_array_equal(np.sort(order), np.arange(E))
    assert np.all(np.diff(rank_j[order]) >= 0)
    info = ops.info.cpu().numpy()
    assert info[be.INFO_N_UNIQUE] == len(u) == N and info[be.INFO_BAD_EDGE] == 0
    assert np.all(ops.dx.cpu().numpy() == 0)
    ops.close()


def test_gn_singular_system_zero_dx(be):
    """No valid residual -> LLT fails -> dx = 0, poses untouched (gn_kernels.cu:147-150)."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(4, 24, 32, seed=34)
    valid = torch.zeros_like(g.valid_match)
    T_gpu, dx, info = run_gpu(be, "rays", g, 10, 1e-8, valid=valid)
    assert info[be.INFO_SOLVE_FAIL] == 1 and info[be.INFO_ITERS] == 1
    assert np.all(dx == 0)
    np.testing.assert_array_equal(T_gpu, g.T_init.data.numpy())


@pytest.mark.parametrize("N,tail", [(12, None), (140, 8)])
def test_gn_broken_plan_times_out_as_solve_failure(test_lib, be, knobs, N, tail):
    """A plan bug must end as a solve failure, never a hang (the LLT's flag
    waits are bounded). The debug_drop_item knob removes the first item of the
    dispatch list (a leaf DIAG): the items reading its blocks time out, the
    iteration reports INFO_SOLVE_FAIL with dx = 0 and the poses untouched.
    N = 12: the one-workgroup dataflow (sparse_llt_kernel); N = 140 with a
    dense tail: the
    chip-wide path (df_factor_kernel's epoch flags, tail_cyc_kernel's tagged
    granules, col_backsub_kernel)."""
    import time

    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(N, 12 if N > 64 else 24, 16 if N > 64 else 32, seed=37)
    if tail is not None:
        knobs("dense_tail_min", tail)
    knobs("debug_drop_item", "0")
    t0 = time.time()
    T_gpu, dx, info = run_gpu(be, "rays", g, 1, 0.0)
    dt = time.time() - t0
    assert info[be.INFO_SOLVE_FAIL] == 1 and info[be.INFO_ITERS] == 1
    assert np.all(dx == 0)
    np.testing.assert_array_equal(T_gpu, g.T_init.data.numpy())
    assert dt < 60.0
    knobs("debug_drop_item", -1)
    T_ok, _, info = run_gpu(be, "rays", g, 1, 0.0)  # the same graph, intact plan
    assert info[be.INFO_SOLVE_FAIL] == 0 and not np.array_equal(T_ok, g.T_init.data.numpy())


def test_workspace_reuse_across_solver_paths(be, knobs):
    """One workspace for a chip-wide solve (global factor, dense tail: epoch
    flags and tagged granules), then an LDS-resident solve, then the chip-wide
    one again: flags, granules and tickets left by an earlier call must not be
    taken for this call's; each dx equals a fresh-workspace run bitwise."""
    from mast3r_slam_amd import synthetic

    knobs("dense_tail_min", 8)
    big = synthetic.make_graph(140, 12, 16, seed=61)
    small = synthetic.make_graph(12, 12, 16, seed=62)

    def call(g, ws):
        Twc = g.T_init.data.clone().to(DEV).contiguous()
        args = [t.to(DEV).contiguous() for t in (g.Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q)]
        a, keep = be.make_gn_args(be.MODE_RAYS, Twc, *args, sigma_a=0.003, sigma_b=10.0, C_thresh=0.0,
                                  Q_thresh=1.5, max_iter=3, delta_thresh=0.0, workspace=ws)
        (dx,) = be._run_gn("m3s_gauss_newton_rays", a, keep)
        torch.cuda.synchronize()
        return Twc.cpu().numpy(), dx.cpu().numpy(), keep["info"].cpu().numpy()

    nbytes = max(be._lib.m3s_gn_workspace_size(g.Xs.shape[0], g.Xs.shape[1], g.n_edges) for g in (big, small))
    ws = torch.zeros(nbytes, dtype=torch.uint8, device=DEV)
    seq = [call(g, ws) for g in (big, small, big)]
    for g, got in zip((big, small, big), seq):
        ref = call(g, None)
        assert got[2][be.INFO_SOLVE_FAIL] == 0 and got[2][be.INFO_ITERS] == 3
        np.testing.assert_array_equal(got[1], ref[1])
        np.testing.assert_array_equal(got[0], ref[0])


def test_gn_bad_edge_ids_flagged(be):
    """More unique ids than poses -> flagged, nothing computed (the reference
    would read out of bounds)."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(4, 24, 32, seed=35)
    g.ii[0] = 99  # a 5th unique id with only 4 pointmaps
    T_gpu, dx, info = run_gpu(be, "rays", g, 2, 0.0)
    assert info[be.INFO_BAD_EDGE] == 1 and info[be.INFO_ITERS] == 0
    np.testing.assert_array_equal(T_gpu, g.T_init.data.numpy())


def test_gn_ragged_pixel_count_scalar_path(be):
    """HW % 4 != 0 takes the scalar load path; still matches the oracle."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(4, 17, 30, seed=36)
    assert (g.H * g.W) % 4 != 0
    T_gpu, _, info = run_gpu(be, "rays", g, 4, 0.0)
    T_ref, _, _, _ = run_oracle("rays", g, 4, 0.0)
    np.testing.assert_allclose(T_gpu, T_ref, atol=1e-4)


def test_gn_two_pose_onestep_golden(be, golden_dir):
    """Reference tracker fixture through the backend."""
    import os

    for name in ("onestep_rays_identity_32x24", "onestep_calib_identity_32x24"):
        d = dict(np.load(os.path.join(golden_dir, name + ".npz")))
        HW = d["Xf"].shape[0]
        Twc = torch.from_numpy(np.concatenate([d["T_WCk"], d["T_WCf_init"]])).to(DEV)
        Xs = torch.from_numpy(np.stack([d["Xk"], d["Xf"]])).to(DEV)
        Cs = torch.ones(2, HW, 1, device=DEV)
        ii = torch.tensor([0], device=DEV)
        jj = torch.tensor([1], device=DEV)
        idx = torch.arange(HW, device=DEV)[None].contiguous()
        valid = torch.from_numpy(d["valid"]).reshape(1, HW, 1).to(DEV)
        Q = torch.from_numpy(d["Qk"]).reshape(1, HW, 1).to(DEV)
        if int(d["calib"]):
            be.gauss_newton_calib(Twc, Xs, Cs, torch.from_numpy(d["K"]).to(DEV), ii, jj, idx, valid,
                                  Q, int(d["H"]), int(d["W"]), -10, 1e-6, 1.0, 10.0, 0.0, 1.5, 1, 0.0)
        else:
            be.gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx, valid, Q, 0.003, 10.0, 0.0, 1.5, 1, 0.0)
        torch.cuda.synchronize()
        tol = 1e-5 + 1e-4 * float(np.linalg.norm(d["tau_iter"], axis=-1).sum())
        np.testing.assert_allclose(Twc[1].cpu().numpy(), d["T_WCf"][0], atol=tol)


def test_gn_is_deterministic(be, graph_small):
    a = run_gpu(be, "rays", graph_small, 5, 0.0)
    b = run_gpu(be, "rays", graph_small, 5, 0.0)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


def test_gn_c3_shape_one_iteration_matches_oracle(be):
    """32 KFs (C3 graph shape) at 128x96: one iteration vs the oracle."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(32, 96, 128, seed=1003)
    assert 7 * 31 + 1 <= 224
    T_gpu, dx_gpu, info = run_gpu(be, "rays", g, 1, 0.0)
    T_ref, dx_ref, it, _ = run_oracle("rays", g, 1, 0.0)
    np.testing.assert_allclose(dx_gpu, dx_ref, atol=2e-5)
    np.testing.assert_allclose(T_gpu, T_ref, atol=2e-5)


def test_gn_input_checks(be, graph_small):
    g = graph_small
    Twc = g.T_init.data.clone().to(DEV)
    args = [t.to(DEV) for t in (g.Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q)]
    nc = args[0].transpose(0, 1)
    with pytest.raises(RuntimeError, match="Xs must be contiguous"):
        be.gauss_newton_rays(Twc, nc, *args[1:], 0.003, 10.0, 0.0, 1.5, 1, 0.0)
    with pytest.raises(RuntimeError, match="ROCm device"):
        be.gauss_newton_rays(Twc.cpu(), *args, 0.003, 10.0, 0.0, 1.5, 1, 0.0)


@pytest.mark.parametrize("N", [33, 70])
def test_gn_tiled_cholesky_path_matches_oracle(test_lib, be, knobs, N):
    """The dense fallback forced on (test build, knob dense=1) at 7(N-1)+1 >
    224: the tiled 64x64 fp64 Cholesky + blocked back-substitution. One step
    from identical inputs is tight; after 3 steps the fp32 H/g noise (x
    cond(H)) has moved the linearisation point, so poses get the step-scaled
    tolerance."""
    from mast3r_slam_amd import synthetic

    knobs("dense", 1)
    g = synthetic.make_graph(N, 24, 32, seed=40 + N)
    _, dx1_gpu, _ = run_gpu(be, "rays", g, 1, 0.0)
    _, dx1_ref, _, _ = run_oracle("rays", g, 1, 0.0)
    np.testing.assert_allclose(dx1_gpu, dx1_ref, atol=1e-6 + 1e-4 * np.abs(dx1_ref).max())
    T_gpu, dx_gpu, info = run_gpu(be, "rays", g, 3, 0.0)
    T_ref, dx_ref, it, failed = run_oracle("rays", g, 3, 0.0)
    assert info[be.INFO_ITERS] == it == 3 and failed == info[be.INFO_SOLVE_FAIL]
    np.testing.assert_allclose(T_gpu, T_ref, atol=1e-5 + 3e-4 * np.abs(dx1_ref).max())


def test_gn_over_capacity_plan_takes_dense_fallback(be):
    """The product library's own dense fallback: a complete graph of 201
    keyframes fills all m (m + 1) / 2 = 20100 blocks of its factor, more than
    the workspace's sparse-slot capacity (64 m + 4096 + 1), so the call solves
    by the tiled fp64 Cholesky (n = 1400) instead of the block-sparse LLT;
    against the oracle (gn_kernels.cu:57-159 builds the same system as
    triplets). The yardstick is the oracle with fp64 sums and the fp64
    retraction (exact-arithmetic stand-in, as tests/test_gpu_large.py).

    Every GN step must be as accurate as the reference's fp32 step from the
    SAME linearisation point: step 1 from the initial poses, and step 2 (the
    packed linearize + the tiled solve of a 2-iteration call) from HIP's own
    poses after step 1, each within the fp32 reference's distance to the
    exact step + 1e-6. The retraction of step 2 is then checked on identical
    inputs (T1, dx2) three ways: the device's, the oracle's fp32 restatement
    of retrSim3 and fp64 expm(generator(dx2)) T1. The reference's fp32 Exp
    cancels for this graph's small scale steps (C = (e^sigma - 1) / sigma,
    tests/test_sim3_math.py), which is what moved its poses 1e-5..1e-3 off
    the exact ones with the last bit of a step (round 5); the backend's
    retraction is evaluated in fp64 (round 6), so HIP's poses are bounded
    against the exact ones as its steps are."""
    from mast3r_slam_amd import synthetic
    from test_sim3_math import generator, pose_err, to_mat

    N = 201
    ii_u = [i for j in range(N) for i in range(j)]
    jj_u = [j for j in range(N) for i in range(j)]
    g = synthetic.make_graph(N, 8, 12, seed=45, edges=(ii_u, jj_u))
    m = N - 1
    assert m * (m + 1) // 2 > 64 * m + 4096 + 1
    # step 1 from the initial poses
    T1_gpu, dx1_gpu, info1 = run_gpu(be, "rays", g, 1, 0.0)
    _, dx1_ref, _, failed = run_oracle("rays", g, 1, 0.0)
    T1_x, dx1_x, _, failed_x = run_oracle("rays", g, 1, 0.0, f64=True)
    assert failed == 0 == failed_x and info1[be.INFO_SOLVE_FAIL] == 0
    e1_hip, e1_ref = float(np.abs(dx1_gpu - dx1_x).max()), float(np.abs(dx1_ref - dx1_x).max())
    p1_hip = float(np.abs(T1_gpu - T1_x).max())
    # step 2: a 2-iteration call (its first iteration is bitwise the call above)
    # against the exact and the fp32 reference step from HIP's poses after step 1
    T2_gpu, dx2_gpu, info = run_gpu(be, "rays", g, 2, 0.0)
    assert info[be.INFO_ITERS] == 2 and info[be.INFO_SOLVE_FAIL] == 0
    T2_ref_h, dx2_ref, _, f2 = run_oracle("rays", g, 1, 0.0, Twc0=T1_gpu)
    T2_x_h, dx2_x, _, f2x = run_oracle("rays", g, 1, 0.0, Twc0=T1_gpu, f64=True)
    assert f2 == 0 == f2x
    e2_hip, e2_ref = float(np.abs(dx2_gpu - dx2_x).max()), float(np.abs(dx2_ref - dx2_x).max())
    p2_hip, p2_ref = float(np.abs(T2_gpu - T2_x_h).max()), float(np.abs(T2_ref_h - T2_x_h).max())
    # the retraction of step 2 on identical inputs (T1, dx2), three ways
    xi = torch.from_numpy(dx2_gpu.reshape(m, 7).astype(np.float32))
    T1p = torch.from_numpy(T1_gpu[1:].astype(np.float32))
    M_x = torch.linalg.matrix_exp(generator(xi.double())) @ to_mat(T1p.double())
    T_dev = be.debug_sim3("retract", xi.to(DEV), T1p.to(DEV)).cpu().numpy()
    T_r32 = np.stack([orc.retract(xi[k].numpy(), T1p[k].numpy()) for k in range(m)])
    r_dev, r_ref = pose_err(T_dev, M_x), pose_err(T_r32, M_x)
    np.testing.assert_array_equal(T_dev, T2_gpu[1:])  # the call's own retraction
    # the trajectories after 2 iterations
    T_ref, _, _, _ = run_oracle("rays", g, 2, 0.0)
    T_x, _, _, _ = run_oracle("rays", g, 2, 0.0, f64=True)
    t_hip, t_ref = float(np.abs(T2_gpu - T_x).max()), float(np.abs(T_ref - T_x).max())
    print(f"dense fallback N={N}: max|dx - dx_exact| step 1 hip {e1_hip:.3e} ref {e1_ref:.3e}; "
          f"step 2 (from HIP's T1) hip {e2_hip:.3e} ref {e2_ref:.3e}, poses hip {p2_hip:.3e} ref {p2_ref:.3e}; "
          f"retraction of (T1, dx2) vs fp64 expm: device {r_dev.max():.3e} oracle fp32 {r_ref.max():.3e}; "
          f"poses after step 1 hip {p1_hip:.3e}; trajectories after 2 iterations max|T - T_exact| "
          f"hip {t_hip:.3e} ref {t_ref:.3e} (max|dx1| {np.abs(dx1_x).max():.3f})")
    assert e1_hip <= e1_ref + 1e-6
    assert e2_hip <= e2_ref + 1e-6
    assert np.all(r_dev <= r_ref + 1e-6)
    assert p2_hip <= p2_ref + 1e-6
    assert t_hip <= t_ref + 1e-6
    # the second step inside the 2-iteration call (packed linearize) is the step
    # a 1-iteration call takes from HIP's T1 (gathering linearize) to fp32
    # round-off, and so are the poses it retracts to
    T2_one, dx2_one, _ = run_gpu(be, "rays", g, 1, 0.0, Twc0=T1_gpu)
    assert float(np.abs(dx2_gpu - dx2_one).max()) <= 1e-6
    assert float(np.abs(T2_gpu - T2_one).max()) <= 1e-5


def test_gn_singular_global_factor_zero_dx(be):
    """As above at 40 KFs: every iteration's block-sparse LLT fails, dx = 0,
    poses untouched."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(40, 12, 16, seed=77)
    valid = torch.zeros_like(g.valid_match)
    T_gpu, dx, info = run_gpu(be, "rays", g, 5, 0.0, valid=valid)
    assert info[be.INFO_SOLVE_FAIL] == 5 and info[be.INFO_ITERS] == 5
    assert np.all(dx == 0)
    np.testing.assert_array_equal(T_gpu, g.T_init.data.numpy())


@pytest.mark.parametrize("N,tail", [(6, "8"), (32, "8"), (70, "8"), (32, "3"), (70, "0"), (140, "8"), (256, "24")])
def test_sparse_llt_matches_dense_llt(test_lib, be, N, tail, knobs):
    """Block-sparse LLT (default; LDS-resident for small plans, global for
    N >= 70; the top clique as a dense right-looking tail when it has at least
    M3S_DENSE_TAIL_MIN columns, 0 = never) against the dense fallback
    (M3S_DENSE=1) on identical inputs."""
    from mast3r_slam_amd import synthetic

    knobs("dense_tail_min", tail)
    g = synthetic.make_graph(N, 24, 32, seed=90 + N)
    T_s, dx_s, info_s = run_gpu(be, "rays", g, 3, 0.0)
    knobs("dense", "1")
    T_d, dx_d, info_d = run_gpu(be, "rays", g, 3, 0.0)
    knobs("dense", 0)
    assert info_s[be.INFO_ITERS] == info_d[be.INFO_ITERS] == 3
    np.testing.assert_allclose(dx_s, dx_d, atol=1e-6 + 1e-5 * np.abs(dx_d).max())
    np.testing.assert_allclose(T_s, T_d, atol=1e-5)


def test_mfma_tail_matches_block_tail_and_is_deterministic(test_lib, be, knobs):
    """Global factor with a dense tail: tail_llt_kernel (the top clique on the
    f64 MFMA, 16x16 tiles, the default) against the 7x7-block tail of
    sparse_llt_kernel (M3S_TAIL_MFMA=0) on identical inputs; the MFMA path is
    bitwise reproducible run to run (the sharded ranks rely on it)."""
    from mast3r_slam_amd import synthetic

    knobs("dense_tail_min", "8")
    g = synthetic.make_graph(140, 24, 32, seed=77)
    T_a, dx_a, info_a = run_gpu(be, "rays", g, 3, 0.0)
    T_a2, dx_a2, _ = run_gpu(be, "rays", g, 3, 0.0)
    knobs("tail_mfma", "0")
    T_b, dx_b, info_b = run_gpu(be, "rays", g, 3, 0.0)
    assert info_a[be.INFO_ITERS] == info_b[be.INFO_ITERS] == 3
    assert info_a[be.INFO_SOLVE_FAIL] == info_b[be.INFO_SOLVE_FAIL] == 0
    np.testing.assert_array_equal(T_a, T_a2)
    np.testing.assert_array_equal(dx_a, dx_a2)
    np.testing.assert_allclose(dx_a, dx_b, atol=1e-6 + 1e-5 * np.abs(dx_b).max())
    np.testing.assert_allclose(T_a, T_b, atol=1e-5)


@pytest.mark.parametrize("N", [150, 256, 400])
def test_mfma_tail_one_step_matches_oracle(be, N):
    """One GN step through the MFMA tail (tails of ~14-64 block columns at
    these sizes) against the oracle's dense fp64 LLT on identical inputs."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(N, 12, 16, seed=500 + N)
    p = be.sparse_plan(N, *np.unique(np.concatenate([g.ii.numpy(), g.jj.numpy()]), return_inverse=True)[1]
                       .reshape(2, -1))
    assert p["nc"] >= 8  # a dense tail exists
    _, dx_gpu, info = run_gpu(be, "rays", g, 1, 0.0)
    _, dx_ref, it, failed = run_oracle("rays", g, 1, 0.0)
    p64 = params_for("rays", g)
    _, dx_x, _, _ = orc.gn(p64, g.T_init.data.numpy(), g.Xs.numpy(), g.Cs.numpy(), g.ii.numpy(), g.jj.numpy(),
                           g.idx_ii2jj.numpy(), g.valid_match.numpy(), g.Q.numpy(), 1, 0.0, f64=True)
    assert info[be.INFO_SOLVE_FAIL] == failed == 0
    # yardstick: the oracle with fp64 sums (tests/test_gpu_large.py)
    e_gpu, e_ref = np.abs(dx_gpu - dx_x).max(), np.abs(dx_ref - dx_x).max()
    print(f"N={N} nc={p['nc']} max|dx|={np.abs(dx_x).max():.3e} |hip-exact|={e_gpu:.3e} |ref-exact|={e_ref:.3e}")
    assert e_gpu <= max(2.0 * e_ref, 1e-6 + 1e-5 * np.abs(dx_x).max())


@pytest.mark.parametrize("N", [90, 140, 256])
def test_block_dataflow_matches_column_tasks_bitwise(test_lib, be, N, knobs):
    """Large graphs: the wave-level block dataflow (df_factor_kernel, the
    default: DIAG / OFF / tail-border items over the chip) sums every block's
    update list in the same order as the column tasks + border_kernel path
    (M3S_DF=0), so poses and dx agree bitwise; no solve fails."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(N, 12, 16, seed=700 + N)
    T_a, dx_a, info_a = run_gpu(be, "rays", g, 3, 0.0)
    knobs("df", "0")
    T_b, dx_b, info_b = run_gpu(be, "rays", g, 3, 0.0)
    assert info_a[be.INFO_ITERS] == info_b[be.INFO_ITERS] == 3
    assert info_a[be.INFO_SOLVE_FAIL] == info_b[be.INFO_SOLVE_FAIL] == 0
    np.testing.assert_array_equal(dx_a, dx_b)
    np.testing.assert_array_equal(T_a, T_b)


@pytest.mark.parametrize("N", [128, 140, 256, 400])
def test_tail_pairs_match_tail_columns_bitwise(test_lib, be, N, knobs):
    """The dense tail with two tile columns per workgroup (tail_pair_kernel,
    the default, round 4) applies every tile update in tail_cyc_kernel's order
    (knob tail_pair=0; the pair's own first column last) and shares its
    back-substitution: poses and dx agree bitwise, odd and even tile counts."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(N, 12, 16, seed=850 + N)
    knobs("gcomb", "0")  # both with col_backsub_kernel (tail_cyc_kernel has no workers)
    T_a, dx_a, info_a = run_gpu(be, "rays", g, 3, 0.0)
    knobs("tail_pair", "0")
    T_b, dx_b, info_b = run_gpu(be, "rays", g, 3, 0.0)
    assert info_a[be.INFO_ITERS] == info_b[be.INFO_ITERS] == 3
    assert info_a[be.INFO_SOLVE_FAIL] == info_b[be.INFO_SOLVE_FAIL] == 0
    np.testing.assert_array_equal(dx_a, dx_b)
    np.testing.assert_array_equal(T_a, T_b)


@pytest.mark.parametrize("N", [140, 256, 400])
def test_tail_over_workgroups_matches_one_workgroup(test_lib, be, N, knobs):
    """The dense tail with one workgroup per tile column (tail_cyc_kernel, the
    default) applies every tile update of the factor in the single-workgroup
    kernel's order (tail_llt_kernel, M3S_TAIL_CYC=0); its back-substitution
    runs on the f64 MFMA (a different fp64 summation order), so dx agrees to
    fp64 round-off seen through the fp32 output; no failures."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(N, 12, 16, seed=800 + N)
    T_a, dx_a, info_a = run_gpu(be, "rays", g, 3, 0.0)
    knobs("tail_cyc", "0")
    T_b, dx_b, info_b = run_gpu(be, "rays", g, 3, 0.0)
    assert info_a[be.INFO_ITERS] == info_b[be.INFO_ITERS] == 3
    assert info_a[be.INFO_SOLVE_FAIL] == info_b[be.INFO_SOLVE_FAIL] == 0
    np.testing.assert_allclose(dx_a, dx_b, rtol=0, atol=1e-6 * np.abs(dx_b).max() + 1e-9)
    np.testing.assert_allclose(T_a, T_b, rtol=0, atol=1e-6)
    knobs("tail_cyc", 1)  # and the default is bitwise reproducible run to run
    T_a2, dx_a2, _ = run_gpu(be, "rays", g, 3, 0.0)
    np.testing.assert_array_equal(dx_a, dx_a2)
    np.testing.assert_array_equal(T_a, T_a2)



@pytest.mark.parametrize("mode", ["rays", "calib", "points"])
def test_gn_partial_trip_pixel_count_matches_oracle(be, mode):
    """HW = 20 x 52 = 1040 pixels: a multiple of 4 (the vector, packed and
    pipelined gathering paths) but not of a 1024-pixel trip, so the last trip
    of the last chunk is partial: its lanes past the end take no part and their
    LDS-DMA loads take an offset past the buffer range (zeros, no access).
    The pointmaps sit at the very end of their own allocation (a fresh 12-MiB
    segment of the caching allocator), so the last keyframe's partial trip
    has no bytes of the allocation left behind it to read."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(6, 20, 52, seed=37)
    Xs = constrained(g) if mode == "calib" else g.Xs
    buf = torch.empty(3 << 20, dtype=torch.float32, device=DEV)
    Xs_end = buf[buf.numel() - Xs.numel():].view(Xs.shape)
    Xs_end.copy_(Xs.to(DEV))
    assert Xs_end.data_ptr() + 4 * Xs.numel() == buf.data_ptr() + 4 * buf.numel()
    T_gpu, dx_gpu, info = run_gpu(be, mode, g, 5, 0.0, Xs=Xs_end)
    T_ref, dx_ref, it, failed = run_oracle(mode, g, 5, 0.0, Xs=Xs)
    assert info[be.INFO_ITERS] == it == 5
    assert info[be.INFO_SOLVE_FAIL] == failed == 0
    np.testing.assert_allclose(T_gpu, T_ref, atol=1e-4)
    np.testing.assert_allclose(dx_gpu, dx_ref, atol=1e-5)


@pytest.mark.parametrize("mode,idx32", [("calib", False), ("rays", False), ("rays", True), ("points", False)])
def test_pipelined_gathering_launch_matches_round2_kernel_bitwise(test_lib, be, knobs, mode, idx32):
    """The first GN iteration's pipelined kernel (linearize_gather_kernel:
    streams by LDS-DMA, gathers before the refill) against the round-2
    VGPR-staged linearize_kernel it replaced (test-build knob gather_lds=0):
    the same per-pixel calls in the same order, so poses, dx and info are
    bitwise equal after several iterations; int64 and int32 ids."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(10, 64, 96, seed=38)
    Xs = (constrained(g) if mode == "calib" else g.Xs).to(DEV).contiguous()
    idx = g.idx_ii2jj.to(torch.int32) if idx32 else g.idx_ii2jj
    out = []
    for knob in (0, 1):
        knobs("gather_lds", knob)
        Twc = g.T_init.data.clone().to(DEV).contiguous()
        info = torch.zeros(8, dtype=torch.int32, device=DEV)
        Cs, ii, jj, ix, valid, Q = (t.to(DEV).contiguous() for t in (g.Cs, g.ii, g.jj, idx, g.valid_match, g.Q))
        if mode == "calib":
            (dx,) = be.gauss_newton_calib(Twc, Xs, Cs, g.K.to(DEV), ii, jj, ix, valid, Q, g.H, g.W, -10, 1e-6,
                                          1.0, 10.0, 0.0, 1.5, 4, 0.0, info=info)
        elif mode == "rays":
            (dx,) = be.gauss_newton_rays(Twc, Xs, Cs, ii, jj, ix, valid, Q, 0.003, 10.0, 0.0, 1.5, 4, 0.0, info=info)
        else:
            (dx,) = be.gauss_newton_points(Twc, Xs, Cs, ii, jj, ix, valid, Q, 0.05, 0.0, 1.5, 4, 0.0, info=info)
        torch.cuda.synchronize()
        out.append((Twc.cpu().numpy(), dx.cpu().numpy(), info.cpu().numpy()))
    for a, b in zip(out[0], out[1]):
        np.testing.assert_array_equal(a, b)
    assert int(out[1][2][be.INFO_SOLVE_FAIL]) == 0


@pytest.mark.parametrize("N", [140, 256])
def test_tail_warmup_leaves_factor_bitwise(test_lib, be, N, knobs):
    """The warm-up run of the tail's diagonal factor on a dummy tile (round 4:
    the code is hot when the real tile arrives) writes only scratch that the
    real factor overwrites: poses and dx agree bitwise with it off."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(N, 12, 16, seed=950 + N)
    T_a, dx_a, info_a = run_gpu(be, "rays", g, 3, 0.0)
    knobs("tail_warm", "0")
    T_b, dx_b, info_b = run_gpu(be, "rays", g, 3, 0.0)
    assert info_a[be.INFO_ITERS] == info_b[be.INFO_ITERS] == 3
    assert info_a[be.INFO_SOLVE_FAIL] == info_b[be.INFO_SOLVE_FAIL] == 0
    np.testing.assert_array_equal(dx_a, dx_b)
    np.testing.assert_array_equal(T_a, T_b)


@pytest.mark.parametrize("N", [90, 128, 140, 256, 400])
def test_sparse_backsub_workers_match_column_tasks(test_lib, be, N, knobs):
    """Round 5: the sparse columns' back-substitution as x_k = a_k + B_k x_t
    (X_k = [a_k | B_k] by the extra workgroups of the dense tail's launch
    while the tail factors, gcol_worker, the default) against the column
    tasks after the tail (col_backsub_kernel, knob gcomb=0): the same factor,
    a different fp64 summation order, so dx agrees to fp64 round-off seen
    through the fp32 output; bitwise run to run; no failures."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(N, 12, 16, seed=880 + N)
    knobs("gcomb_min_nc", "0")  # the workers on every tail size (the product takes them from 32 columns)
    T_a, dx_a, info_a = run_gpu(be, "rays", g, 3, 0.0)
    knobs("gcomb", "0")
    T_b, dx_b, info_b = run_gpu(be, "rays", g, 3, 0.0)
    assert info_a[be.INFO_ITERS] == info_b[be.INFO_ITERS] == 3
    assert info_a[be.INFO_SOLVE_FAIL] == info_b[be.INFO_SOLVE_FAIL] == 0
    np.testing.assert_allclose(dx_a, dx_b, rtol=0, atol=1e-6 * np.abs(dx_b).max() + 1e-9)
    np.testing.assert_allclose(T_a, T_b, rtol=0, atol=1e-6)
    knobs("gcomb", "1")
    T_a2, dx_a2, _ = run_gpu(be, "rays", g, 3, 0.0)
    np.testing.assert_array_equal(dx_a, dx_a2)
    np.testing.assert_array_equal(T_a, T_a2)


def test_broken_plan_through_workers_is_solve_failure(test_lib, be, knobs):
    """The bounded waits of the tail launch's back-substitution workers: a
    dropped leaf DIAG item (df_factor_kernel) with the workers forced on a
    small tail ends as one failed iteration (dx = 0, poses untouched), and the
    intact plan then solves (round 5: the finishing wave must see every
    failure flag, stored before the flags that release the step)."""
    from mast3r_slam_amd import synthetic

    g = synthetic.make_graph(140, 12, 16, seed=37)
    knobs("dense_tail_min", 8)
    knobs("gcomb_min_nc", "0")
    knobs("debug_drop_item", "0")
    T_gpu, dx, info = run_gpu(be, "rays", g, 1, 0.0)
    assert info[be.INFO_SOLVE_FAIL] == 1 and info[be.INFO_ITERS] == 1
    assert np.all(dx == 0)
    np.testing.assert_array_equal(T_gpu, g.T_init.data.numpy())
    knobs("debug_drop_item", -1)
    T_ok, _, info = run_gpu(be, "rays", g, 1, 0.0)
    assert info[be.INFO_SOLVE_FAIL] == 0 and info[be.INFO_ITERS] == 1
    assert not np.array_equal(T_ok, g.T_init.data.numpy())
