"""Edge-sharded backend GN across the GPUs of one node.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
The directed edges of a FactorGraph are independent residual blocks
(one block per edge in the reference, gn_kernels.cu:1183), so each rank
linearises a contiguous slice of them and the only exchange per GN iteration
is an all-gather of the per-edge normal-equation sums (36 fp64 per edge:
~290 KB at 1024 edges). Every rank then assembles and solves the identical
(N-1)*7 system with identical inputs and deterministic kernels, so the
retracted poses agree bitwise across ranks and nothing is broadcast.

Per GN iteration on each rank:
    m3s_gn_linearize(slice)  ->  all_gather_into_tensor  ->  m3s_gn_solve
all enqueued asynchronously; convergence (||dx|| < delta) is a device flag
that makes the remaining launches no-ops, exactly like the single-GPU call.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

import mast3r_slam_backends as be


def edge_slice(E: int, rank: int, world: int):
    per = (E + world - 1) // world
    b = min(rank * per, E)
    e = min(b + per, E)
    return b, e, per


class ShardedGN:
    """Holds the per-rank state of one sharded GN problem.

    Edge data tensors (idx, valid, Q) are this rank's slice [e_end - e_begin,
    HW(,1)]; ii/jj are the full [E] id lists (every rank needs all of them to
    assemble the system); Xs/Cs/Twc are replicated.
    """

    def __init__(self, mode, Twc, Xs, Cs, ii, jj, idx_loc, valid_loc, Q_loc, E, K=None, *,
                 sigma_a, sigma_b=0.0, C_thresh=0.0, Q_thresh=1.5, height=0, width=0,
                 pixel_border=0, z_eps=0.0, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.E = int(E)
        self.eb, self.ee, self.per = edge_slice(self.E, self.rank, self.world)
        n_loc = self.ee - self.eb
        HW = int(Xs.shape[1])
        assert idx_loc.shape[0] == n_loc and valid_loc.shape[0] == n_loc and Q_loc.shape[0] == n_loc
        for name, t in (("Twc", Twc), ("Xs", Xs), ("Cs", Cs), ("ii", ii), ("jj", jj),
                        ("idx", idx_loc), ("valid", valid_loc), ("Q", Q_loc)):
            be._check(t, name)
        dev = Xs.device
        N = int(Xs.shape[0])
        self.dx = torch.zeros(max(N - 1, 0), 7, dtype=torch.float32, device=dev)
        self.info = torch.zeros(8, dtype=torch.int32, device=dev)
        self.ws = be._workspace(be._lib.m3s_gn_workspace_size(N, HW, self.E), dev)
        self.es_loc = torch.zeros(self.per, be.EDGE_SUM_STRIDE, dtype=torch.float64, device=dev)
        self.es_all = torch.zeros(self.per * self.world, be.EDGE_SUM_STRIDE, dtype=torch.float64,
                                  device=dev)
        a = be.GnArgs()
        P = be._p
        a.Twc, a.Xs, a.Cs, a.ii, a.jj = P(Twc), P(Xs), P(Cs), P(ii), P(jj)
        # edge-slice base pointers: the C side addresses edge data relative to
        # edge_begin (include/m3s_gn.h, stepwise API)
        a.idx_ii2jj, a.valid_match, a.Q, a.K = P(idx_loc), P(valid_loc), P(Q_loc), P(K)
        a.N, a.HW, a.E, a.mode = N, HW, self.E, mode
        a.sigma_a, a.sigma_b, a.C_thresh, a.Q_thresh = sigma_a, sigma_b, C_thresh, Q_thresh
        a.height, a.width, a.pixel_border, a.z_eps = height, width, pixel_border, z_eps
        a.max_iter, a.delta_thresh = 0, 0.0
        a.dx_out, a.info = P(self.dx), P(self.info)
        a.workspace, a.workspace_bytes = P(self.ws), self.ws.numel()
        self.args = a
        self.keep = dict(Twc=Twc, Xs=Xs, Cs=Cs, ii=ii, jj=jj, idx=idx_loc, valid=valid_loc,
                         Q=Q_loc, K=K)
        self.stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def solve(self, max_iter: int, delta_thresh: float):
        """gauss_newton_{mode} semantics over the sharded edges; Twc in place."""
        a = self.args
        a.delta_thresh = float(delta_thresh)
        be._raise(be._lib.m3s_gn_prepare(ctypes.byref(a), self.stream), "m3s_gn_prepare")
        n_loc = self.ee - self.eb
        for _ in range(int(max_iter)):
            if n_loc > 0:
                be._raise(
                    be._lib.m3s_gn_linearize(ctypes.byref(a), self.eb, self.ee,
                                             be._p(self.es_loc), self.stream),
                    "m3s_gn_linearize",
                )
            if self.world > 1:
                dist.all_gather_into_tensor(self.es_all, self.es_loc, group=self.group)
                es = self.es_all
            else:
                es = self.es_loc
            be._raise(be._lib.m3s_gn_solve(ctypes.byref(a), be._p(es), self.stream), "m3s_gn_solve")
        return [self.dx]

    def linearize_only(self):
        """Timing hook: just the linearize kernel on this rank's slice."""
        if self.ee > self.eb:
            be._raise(
                be._lib.m3s_gn_linearize(ctypes.byref(self.args), self.eb, self.ee, None, self.stream),
                "m3s_gn_linearize",
            )
