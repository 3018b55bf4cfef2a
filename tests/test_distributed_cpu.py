"""Multi-process (gloo, CPU) tests of the edge-sharded GN orchestration
(mast3r_slam_amd/distributed.py, the N>1 path of bench.py).

The per-rank compute is the CPU oracle here (test infrastructure): each rank
linearises its contiguous edge slice into per-edge reference blocks
(Hs[0..3], gs[0..1] of gn_kernels.cu), the payloads travel through the real
``dist.all_gather_into_tensor`` on gloo, and every rank assembles and solves
the same fp64 system (SparseBlock semantics, gn_kernels.cu:57-159) and
retracts its replicated poses. Checked: slices cover every edge once, every
rank ends with bitwise-identical poses, and they match the single-process
oracle GN (oracle.gn) on the same graph.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "mast3r-slam-ysh_amd")


def _paths():
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)


_paths()
from mast3r_slam_amd.distributed import (ShardedGN, edge_shard, edge_slice, payload_edges,  # noqa: E402
                                         payload_ids)

N_KF, H, W, ITERS = 7, 12, 16, 3
SIG = (0.003, 10.0)


class OracleOps:
    """CPU stand-in for HipOps: payload = the reference blocks of one edge."""

    stride = 4 * 49 + 2 * 7

    def __init__(self, Twc, Xs, Cs, ii, jj, idx_loc, valid_loc, Q_loc):
        from oracle import oracle as orc

        self.orc = orc
        self.params = orc.make_params(orc.MODE_RAYS, SIG[0], SIG[1], 0.0, 1.5)
        self.Twc = Twc  # torch [N, 8], updated in place like the device path
        self.Xs, self.Cs = Xs.numpy(), Cs.numpy()
        self.ii, self.jj = ii.numpy(), jj.numpy()
        self.idx, self.valid, self.Q = idx_loc.numpy(), valid_loc.numpy(), Q_loc.numpy()
        u = np.unique(np.concatenate([self.ii, self.jj]))
        self.ri, self.rj = np.searchsorted(u, self.ii), np.searchsorted(u, self.jj)
        self.device = torch.device("cpu")
        self.dx = torch.zeros(Twc.shape[0] - 1, 7)
        self.stop = False

    def prepare(self, delta):
        self.delta, self.stop = float(delta), False

    def linearize(self, eb, ee, es_loc):
        T = self.Twc.numpy()
        for k, e in enumerate(range(eb, ee)):
            a, b = int(self.ri[e]), int(self.rj[e])
            lo, hi = min(a, b), max(a, b)
            sel = [lo, hi] if lo != hi else [lo]
            Hs, gs = self.orc.edge_blocks(
                self.params, T[sel], self.Xs[sel], self.Cs[sel],
                np.array([self.ii[e]]), np.array([self.jj[e]]), self.idx[k:k + 1],
                self.valid[k:k + 1], self.Q[k:k + 1])
            es_loc[k] = torch.from_numpy(np.concatenate([Hs[:, 0].reshape(-1), gs[:, 0].reshape(-1)]))

    def solve(self, es):
        if self.stop:
            return
        N = self.Twc.shape[0]
        n = 7 * (N - 1)
        Hm, g = np.zeros((n, n)), np.zeros(n)
        P = es.numpy()
        for e in range(len(self.ri)):
            Hs = P[e, :196].reshape(4, 7, 7)
            gs = P[e, 196:].reshape(2, 7)
            a, b = int(self.ri[e]) - 1, int(self.rj[e]) - 1
            for (x, y), blk in zip(((a, a), (a, b), (b, a), (b, b)), Hs):
                if x >= 0 and y >= 0:
                    Hm[7 * x:7 * x + 7, 7 * y:7 * y + 7] += blk
            if a >= 0:
                g[7 * a:7 * a + 7] += gs[0]
            if b >= 0:
                g[7 * b:7 * b + 7] += gs[1]
        dx = -np.linalg.solve(Hm, g).reshape(N - 1, 7).astype(np.float32)
        T = self.Twc.numpy()
        for k in range(1, N):
            T[k] = self.orc.retract(dx[k - 1], T[k])
        self.dx.copy_(torch.from_numpy(dx))
        if np.linalg.norm(dx) < self.delta:
            self.stop = True


class LocalFormOracleOps(OracleOps):
    """CPU stand-in with the HIP path's payload: per edge the 36 fp64 values of
    m3s_gn_linearize (include/m3s_gn.h) — L's upper triangle (28, row-major),
    l (7), cost (1) in the frame of the residual — and a solve that maps them
    through M = Adj(T_i)^-T exactly as the device finalize does (H_jj = M L M^T,
    g_j = M l; Hs[0] = Hs[3] = H_jj, Hs[1] = Hs[2] = -H_jj, gs[0] = -g_j,
    gs[1] = g_j). L and l come from the oracle's reference blocks
    (L = M^-1 Hs[3] M^-T, l = M^-1 gs[1])."""

    stride = 36

    def linearize(self, eb, ee, es_loc):
        T = self.Twc.numpy()
        iu = np.triu_indices(7)
        for k, e in enumerate(range(eb, ee)):
            a, b = int(self.ri[e]), int(self.rj[e])
            lo, hi = min(a, b), max(a, b)
            sel = [lo, hi] if lo != hi else [lo]
            Hs, gs = self.orc.edge_blocks(
                self.params, T[sel], self.Xs[sel], self.Cs[sel],
                np.array([self.ii[e]]), np.array([self.jj[e]]), self.idx[k:k + 1],
                self.valid[k:k + 1], self.Q[k:k + 1])
            Mi = np.linalg.inv(self.orc.adjT_inv_matrix(T[a]).astype(np.float64))
            L = Mi @ Hs[3, 0].astype(np.float64) @ Mi.T
            l = Mi @ gs[1, 0].astype(np.float64)
            es_loc[k] = torch.from_numpy(np.concatenate([L[iu], l, [0.0]]))

    def solve(self, es):
        if self.stop:
            return
        N = self.Twc.shape[0]
        T = self.Twc.numpy()
        P = es.numpy()
        iu = np.triu_indices(7)
        Hs = np.zeros((len(self.ri), 4, 7, 7))
        gs = np.zeros((len(self.ri), 2, 7))
        for e in range(len(self.ri)):
            L = np.zeros((7, 7))
            L[iu] = P[e, :28]
            L = L + L.T - np.diag(np.diag(L))
            M = self.orc.adjT_inv_matrix(T[int(self.ri[e])]).astype(np.float64)
            Hjj, gj = M @ L @ M.T, M @ P[e, 28:35]
            Hs[e] = (Hjj, -Hjj, -Hjj, Hjj)
            gs[e] = (-gj, gj)
        full = np.concatenate([Hs.reshape(len(self.ri), -1), gs.reshape(len(self.ri), -1)], 1)
        super().solve(torch.from_numpy(full))


def _graph():
    from mast3r_slam_amd import synthetic

    return synthetic.make_graph(N_KF, H, W, seed=41)


def _rank_main(rank, world, port, out_dir, local_form=False):
    _paths()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = _graph()
        E = g.n_edges
        ids, _ = edge_shard(E, rank, world)  # both halves of each undirected edge
        Twc = g.T_init.data.clone()
        cls = LocalFormOracleOps if local_form else OracleOps
        ii_p, jj_p = payload_ids(g.ii, g.jj, world)  # the solve's edge list (gathered-row order)
        loc = (g.idx_ii2jj[ids], g.valid_match[ids], g.Q[ids])
        ops = cls(Twc, g.Xs, g.Cs, ii_p, jj_p, *loc)
        solver = ShardedGN(1, Twc, g.Xs, g.Cs, g.ii, g.jj, *loc, E, sigma_a=SIG[0], sigma_b=SIG[1],
                           ops=ops)
        solver.solve(ITERS, 0.0)
        np.save(os.path.join(out_dir, f"T_{rank}.npy"), Twc.numpy())
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,local_form", [(2, False), (3, False), (2, True), (4, True)])
def test_sharded_gn_matches_single_process_oracle(world, local_form, tmp_path):
    """local_form: the 36-double per-edge payload of the HIP path
    (m3s_gn_linearize) travels through the gloo all-gather."""
    from oracle import oracle as orc

    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path), local_form), nprocs=world, join=True)
    Ts = [np.load(tmp_path / f"T_{r}.npy") for r in range(world)]
    for r in range(1, world):
        assert np.array_equal(Ts[0], Ts[r]), f"rank {r} poses differ from rank 0"
    g = _graph()
    p = orc.make_params(orc.MODE_RAYS, SIG[0], SIG[1], 0.0, 1.5)
    T_ref, _, it, _ = orc.gn(p, g.T_init.data.numpy(), g.Xs.numpy(), g.Cs.numpy(), g.ii.numpy(),
                             g.jj.numpy(), g.idx_ii2jj.numpy(), g.valid_match.numpy(),
                             g.Q.numpy(), ITERS, 0.0)
    assert it == ITERS
    err = np.abs(Ts[0] - T_ref).max()
    assert err < 1e-4, f"sharded GN vs single-process oracle: {err}"


@pytest.mark.parametrize("E,world", [(98, 2), (98, 8), (5, 4), (1, 3), (0, 2), (792, 8)])
def test_edge_slices_partition_edges(E, world):
    seen = []
    for r in range(world):
        b, e, per = edge_slice(E, r, world)
        assert 0 <= b <= e <= E and e - b <= per
        assert b == min(r * per, E)  # row k of the gathered payload is edge k
        seen.extend(range(b, e))
    assert seen == list(range(E))


@pytest.mark.parametrize("E,world", [(98, 2), (98, 8), (96, 3), (6, 4), (2, 3), (0, 2), (792, 8),
                                     (2048, 8), (7, 3)])
def test_edge_shards_keep_pairs_and_cover_edges(E, world):
    """edge_shard: every directed edge on exactly one rank; for a two-way list
    (E even: [fwd | bwd], global_opt.py:104-110) edge u and edge E/2 + u on
    the same rank; payload_edges: rank r's rows start at r * per, padding rows
    repeat an edge of the same rank."""
    seen = []
    rows = payload_edges(E, world)
    for r in range(world):
        ids, per = edge_shard(E, r, world)
        assert len(ids) <= per
        seen.extend(ids)
        assert rows[r * per:r * per + len(ids)] == ids
        pad = rows[r * per + len(ids):(r + 1) * per]
        assert all(p == (ids[0] if ids else 0) for p in pad)
        if E % 2 == 0 and world > 1:
            U = E // 2
            own = set(ids)
            for u in ids:
                assert (u + U if u < U else u - U) in own, f"pair of edge {u} not on rank {r}"
    assert sorted(seen) == list(range(E))
    assert len(rows) == (len(rows) // world) * world


def test_payload_order_zero_padding_rows_leave_the_system_unchanged():
    """A padding row (duplicate edge, zero sums) adds exact zeros: the solve on
    the payload-ordered edge list equals the solve on the reference order up
    to the fp64 summation order of duplicate blocks."""
    g = _graph()
    Twc0 = g.T_init.data.clone()
    E = g.n_edges
    world = 4
    ii_p, jj_p = payload_ids(g.ii, g.jj, world)
    rows = payload_edges(E, world)
    ops_ref = LocalFormOracleOps(Twc0.clone(), g.Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q)
    es = torch.zeros(E, 36, dtype=torch.float64)
    ops_ref.linearize(0, E, es)
    es_pay = torch.zeros(len(rows), 36, dtype=torch.float64)
    real = set()
    for k, e in enumerate(rows):
        if e not in real:  # the first occurrence carries the edge, repeats are padding
            es_pay[k] = es[e]
            real.add(e)
    ops_pay = LocalFormOracleOps(Twc0.clone(), g.Xs, g.Cs, ii_p, jj_p, g.idx_ii2jj, g.valid_match, g.Q)
    ops_ref.prepare(0.0)
    ops_pay.prepare(0.0)
    ops_ref.solve(es)
    ops_pay.solve(es_pay)
    np.testing.assert_allclose(ops_pay.Twc.numpy(), ops_ref.Twc.numpy(), rtol=0, atol=1e-6)


def test_sharded_gn_rejects_wrong_slice():
    g = _graph()
    Twc = g.T_init.data.clone()
    with pytest.raises(ValueError):
        ShardedGN(1, Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj[:3], g.valid_match[:3], g.Q[:3],
                  g.n_edges, sigma_a=SIG[0], ops=OracleOps(Twc, g.Xs, g.Cs, g.ii, g.jj,
                                                           g.idx_ii2jj[:3], g.valid_match[:3],
                                                           g.Q[:3]))
