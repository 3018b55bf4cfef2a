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
    linearize(slice)  ->  all_gather_into_tensor  ->  solve
all enqueued asynchronously; convergence (||dx|| < delta) is a device flag
that makes the remaining launches no-ops, exactly like the single-GPU call.

The per-rank compute is behind a small ops object (prepare / linearize /
solve + the per-edge payload width). ``HipOps`` is the product path (the
m3s_gn stepwise C ABI, include/m3s_gn.h); tests substitute a CPU
implementation to exercise the slicing and the collective on gloo.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist


def edge_slice(E: int, rank: int, world: int):
    """Contiguous edge range [b, e) of `rank` and the per-rank stride `per`
    (the plain split; ShardedGN uses :func:`edge_shard`)."""
    per = (E + world - 1) // world if world > 0 else E
    b = min(rank * per, E)
    e = min(b + per, E)
    return b, e, per


def edge_shard(E: int, rank: int, world: int):
    """The directed edges of `rank`, keeping each undirected edge's two halves
    together: the reference hands the backend the two-way
    list [fwd | bwd] (``prep_two_way_edges``, global_opt.py:104-110), so edge
    u < E/2 and edge E/2 + u are one pair. Rank r owns the pairs of a
    contiguous range [ub, ue) of undirected edges: directed ids
    [ub, ue) ++ [E/2 + ub, E/2 + ue), in that order. An odd E (not a two-way
    list) falls back to the contiguous split.

    Returns (ids, per): rank r's rows of the gathered [per * world, S]
    payload are [r * per, r * per + len(ids)); rows past len(ids) are padding
    (zero sums). :func:`payload_edges` gives the edge of every payload row."""
    if world <= 1:
        return list(range(E)), E
    if E % 2:
        b, e, per = edge_slice(E, rank, world)
        return list(range(b, e)), per
    U = E // 2
    per_u = (U + world - 1) // world
    ub = min(rank * per_u, U)
    ue = min(ub + per_u, U)
    return list(range(ub, ue)) + list(range(U + ub, U + ue)), 2 * per_u


def payload_edges(E: int, world: int):
    """The directed edge id of every row of the gathered payload
    ([per * world] rows, rank-major). A padding row repeats a real edge of the
    same rank (or edge 0): its sums are zero, so the assembled system, the
    fill pattern and the keyframe set are those of the E real edges."""
    rows = []
    for r in range(world):
        ids, per = edge_shard(E, r, world)
        pad = ids[0] if ids else 0
        rows += ids + [pad] * (per - len(ids))
    return rows


def payload_ids(ii: torch.Tensor, jj: torch.Tensor, world: int):
    """ii/jj in payload order (the edge list every rank's solve is given; the
    reference's order itself at world 1)."""
    if world <= 1:
        return ii, jj
    rows = torch.tensor(payload_edges(int(ii.numel()), world), dtype=torch.int64, device=ii.device)
    return ii[rows].contiguous(), jj[rows].contiguous()


class HipOps:
    """Stepwise m3s_gn C ABI on this rank's device (m3s_gn_prepare /
    m3s_gn_linearize / m3s_gn_solve)."""

    def __init__(self, mode, Twc, Xs, Cs, ii, jj, idx_loc, valid_loc, Q_loc, E, K=None, *,
                 sigma_a, sigma_b=0.0, C_thresh=0.0, Q_thresh=1.5, height=0, width=0,
                 pixel_border=0, z_eps=0.0):
        import mast3r_slam_backends as be

        self.be = be
        self.stride = be.EDGE_SUM_STRIDE
        f32, i64 = torch.float32, torch.int64
        # the same dtype contract as the single-call path (make_gn_args): idx
        # is int64 as the reference passes it, or int32 from the device edge
        # store (factor_graph.EdgeStore) — the C side is told which
        for name, t, dt in (("Twc", Twc, f32), ("Xs", Xs, f32), ("Cs", Cs, f32), ("ii", ii, i64),
                            ("jj", jj, i64), ("idx", idx_loc, (i64, torch.int32)),
                            ("valid", valid_loc, torch.bool), ("Q", Q_loc, f32)):
            be._check(t, name, dt)
        if K is not None:
            be._check(K, "K", f32)
        dev = Xs.device
        self.device = dev
        N, HW = int(Xs.shape[0]), int(Xs.shape[1])
        self.dx = torch.zeros(max(N - 1, 0), 7, dtype=torch.float32, device=dev)
        self.info = torch.zeros(8, dtype=torch.int32, device=dev)
        self.ws = be._workspace(be._lib.m3s_gn_workspace_size(N, HW, int(E)), dev)
        a = be.GnArgs()
        P = be._p
        a.Twc, a.Xs, a.Cs, a.ii, a.jj = P(Twc), P(Xs), P(Cs), P(ii), P(jj)
        # edge-slice base pointers: the C side addresses edge data relative to
        # edge_begin (include/m3s_gn.h, stepwise API)
        a.idx_ii2jj, a.valid_match, a.Q, a.K = P(idx_loc), P(valid_loc), P(Q_loc), P(K)
        a.idx_i32 = 1 if idx_loc.dtype == torch.int32 else 0
        a.N, a.HW, a.E, a.mode = N, HW, int(E), mode
        a.sigma_a, a.sigma_b, a.C_thresh, a.Q_thresh = sigma_a, sigma_b, C_thresh, Q_thresh
        a.height, a.width, a.pixel_border, a.z_eps = height, width, pixel_border, z_eps
        a.max_iter, a.delta_thresh = 0, 0.0
        a.dx_out, a.info = P(self.dx), P(self.info)
        a.workspace, a.workspace_bytes = P(self.ws), self.ws.numel()
        self.args = a
        self.keep = dict(Twc=Twc, Xs=Xs, Cs=Cs, ii=ii, jj=jj, idx=idx_loc, valid=valid_loc,
                         Q=Q_loc, K=K)
        self.stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def prepare(self, delta_thresh: float):
        self.args.delta_thresh = float(delta_thresh)
        self.be._raise(self.be._lib.m3s_gn_prepare(ctypes.byref(self.args), self.stream),
                       "m3s_gn_prepare")

    def linearize(self, eb: int, ee: int, es_loc):
        ptr = self.be._p(es_loc) if es_loc is not None else None
        self.be._raise(self.be._lib.m3s_gn_linearize(ctypes.byref(self.args), eb, ee, ptr,
                                                     self.stream), "m3s_gn_linearize")

    def solve(self, es):
        self.be._raise(self.be._lib.m3s_gn_solve(ctypes.byref(self.args), self.be._p(es),
                                                 self.stream), "m3s_gn_solve")

    def close(self):
        """Drop the library's host state of this workspace (m3s_gn_release)."""
        if self.args is not None:
            self.be._raise(self.be._lib.m3s_gn_release(ctypes.byref(self.args), self.stream),
                           "m3s_gn_release")
            self.args = None


class ShardedGN:
    """Per-rank state of one sharded GN problem.

    Edge data tensors (idx, valid, Q) are this rank's edges
    (:func:`edge_shard`: both halves of each of its undirected edges, in the
    order ``edge_shard`` lists them), [n_loc, HW(,1)]; ii/jj are the full [E]
    id lists in the reference's order (every rank needs all of them to
    assemble the system); Xs/Cs/Twc are replicated. ``ops`` defaults to
    :class:`HipOps` over the same arguments.

    The solve sees the edges in payload order (:func:`payload_edges`: the
    gathered rows, rank-major), so the all-gathered tensor is consumed as it
    lands: this rank linearizes the contiguous payload rows
    [rank * per, rank * per + n_loc) and nothing is permuted per iteration.
    """

    def __init__(self, mode, Twc, Xs, Cs, ii, jj, idx_loc, valid_loc, Q_loc, E, K=None, *,
                 sigma_a, sigma_b=0.0, C_thresh=0.0, Q_thresh=1.5, height=0, width=0,
                 pixel_border=0, z_eps=0.0, group=None, ops=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.E = int(E)
        ids, self.per = edge_shard(self.E, self.rank, self.world)
        self.edge_ids = ids
        n_loc = len(ids)
        self.eb = self.rank * self.per if self.world > 1 else 0
        self.ee = self.eb + n_loc
        if not (idx_loc.shape[0] == n_loc and valid_loc.shape[0] == n_loc
                and Q_loc.shape[0] == n_loc):
            raise ValueError(f"rank {self.rank}: edge data must hold this rank's {n_loc} edges "
                             f"(edge_shard)")
        ii, jj = payload_ids(ii, jj, self.world)  # padding rows: zero sums
        self.E_pay = int(ii.numel())
        if ops is None:
            ops = HipOps(mode, Twc, Xs, Cs, ii, jj, idx_loc, valid_loc, Q_loc, self.E_pay, K,
                         sigma_a=sigma_a, sigma_b=sigma_b, C_thresh=C_thresh, Q_thresh=Q_thresh,
                         height=height, width=width, pixel_border=pixel_border, z_eps=z_eps)
        self.ops = ops
        dev = getattr(ops, "device", Xs.device)
        self.es_loc = torch.zeros(self.per, ops.stride, dtype=torch.float64, device=dev)
        self.es_all = torch.zeros(self.per * self.world, ops.stride, dtype=torch.float64, device=dev)

    # convenience views of the HIP ops state (bench / tests)
    @property
    def args(self):
        return self.ops.args

    @property
    def keep(self):
        return self.ops.keep

    @property
    def dx(self):
        return self.ops.dx

    @property
    def info(self):
        return self.ops.info

    def solve(self, max_iter: int, delta_thresh: float):
        """gauss_newton_{mode} semantics over the sharded edges; Twc in place."""
        self.ops.prepare(delta_thresh)
        n_loc = self.ee - self.eb
        for _ in range(int(max_iter)):
            if n_loc > 0:
                self.ops.linearize(self.eb, self.ee, self.es_loc)
            if self.world > 1:
                dist.all_gather_into_tensor(self.es_all, self.es_loc, group=self.group)
                es = self.es_all
            else:
                es = self.es_loc
            self.ops.solve(es)
        return [self.ops.dx]

    def solve_timed(self, max_iter: int, delta_thresh: float, stream):
        """solve() with HIP event pairs on `stream` around every linearize
        launch (the kernel plus its small per-edge reduce) and every solve
        launch, in the solve's own launch pattern. Returns the per-iteration
        durations in ms: (linearize, solve)."""
        self.ops.prepare(delta_thresh)
        evs = []
        for _ in range(int(max_iter)):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            e[0].record(stream)
            if self.ee > self.eb:
                self.ops.linearize(self.eb, self.ee, self.es_loc)
            e[1].record(stream)
            if self.world > 1:
                dist.all_gather_into_tensor(self.es_all, self.es_loc, group=self.group)
                es = self.es_all
            else:
                es = self.es_loc
            e[2].record(stream)
            self.ops.solve(es)
            e[3].record(stream)
            evs.append(e)
        torch.cuda.synchronize()
        return [e[0].elapsed_time(e[1]) for e in evs], [e[2].elapsed_time(e[3]) for e in evs]

    def linearize_only(self):
        """Timing hook: just the linearize kernel on this rank's slice."""
        if self.ee > self.eb:
            self.ops.linearize(self.eb, self.ee, None)
