"""Single-GPU emulation of one rank of the N-GPU weak-scaling bench.

Per GN iteration a rank linearizes its slice (~98 directed edges at 32 KFs per
GPU) and then runs the replicated solve of the whole 32*N-KF system. This
builds the FULL synthetic graph of the N-GPU run (bench.py's generator and
seed), linearizes every edge once so that the edge sums are the real system,
then times, per iteration, rank 0's linearize of its own slice followed by the
solve of the whole system, with HIP events. The poses are reset before every
timed iteration, so each one solves the same real system. Any failed
factorisation aborts the run. Rank 0's slice is its pair-preserving shard
(distributed.edge_shard) and the solve sees the payload edge order, as
ShardedGN runs it.

Two terms a one-GPU box cannot time are added and printed separately:
  * the all-gather of the per-edge sums (36 fp64 per edge; ~28 KB per rank
    at 98 edges): a STATED latency AG_US (default 25 us for world > 1: RCCL
    small-message all-gather over xGMI, SURVEY.md §8e's 10-30 us band);
  * the cold-plan cost of a solve call whose edge set changed (SLAM adds
    edges every keyframe): two 10-iteration stepwise calls are timed on the
    host clock, plan cache off and on; the difference is what the host
    symbolic analysis adds per call after overlapping the first linearize,
    shown per call and per iteration (/ 10).

Prints t_iter(N) and the predicted efficiency t_iter(1) / t_iter(N), warm
(edge set unchanged) and cold (every call re-plans), both with the
all-gather term.

env: MODES=calib,rays  WORLDS=1,2,4,8  HW_SIDE=512  REPS=20  AG_US=25  CALLS=5
     M3S_LIB=variants/lib_X.so
"""
import time
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402

if os.environ.get("M3S_LIB"):  # a library variant (tools/mkvar.sh) for A/B
    be._lib = be._load(os.path.abspath(os.environ["M3S_LIB"]))
from mast3r_slam_amd import synthetic  # noqa: E402
from mast3r_slam_amd.distributed import HipOps, edge_shard, payload_edges  # noqa: E402

dev = torch.device("cuda:0")
H = W = int(os.environ.get("HW_SIDE", "512"))
REPS = int(os.environ.get("REPS", "20"))
modes = os.environ.get("MODES", "calib,rays").split(",")
SIG = {"calib": (1.0, 10.0), "rays": (0.003, 10.0)}
AG_US = float(os.environ.get("AG_US", "25"))
CALLS = int(os.environ.get("CALLS", "5"))


def ev():
    return torch.cuda.Event(enable_timing=True)


base = {}
for world in [int(x) for x in os.environ.get("WORLDS", "1,2,4,8").split(",")]:
    N = 32 * world
    g = synthetic.make_graph(N, H, W, seed=1003, device=dev)
    E = g.n_edges
    rows = torch.tensor(payload_edges(E, world) if world > 1 else list(range(E)), device=dev)
    ids0, _ = edge_shard(E, 0, world)
    ee0 = len(ids0)  # rank 0's rows lead the payload
    ii, jj = g.ii[rows].contiguous(), g.jj[rows].contiguous()
    idx, valid, Q = g.idx_ii2jj[rows].contiguous(), g.valid_match[rows].contiguous(), g.Q[rows].contiguous()
    Ep = int(rows.numel())
    rays = synthetic.pixel_rays(H, W, g.K)
    for m in modes:
        Xs = (g.Xs[..., 2:3] * rays[None]).contiguous() if m == "calib" else g.Xs.contiguous()
        T0 = g.T_init.data.contiguous().clone()
        Twc = T0.clone()
        mid = be.MODE_CALIB if m == "calib" else be.MODE_RAYS
        ops = HipOps(mid, Twc, Xs, g.Cs.contiguous(), ii, jj, idx, valid, Q, Ep, g.K if m == "calib" else None,
                     sigma_a=SIG[m][0], sigma_b=SIG[m][1], C_thresh=0.0, Q_thresh=1.5, height=H, width=W,
                     pixel_border=-10, z_eps=1e-6)
        es = torch.zeros(Ep, be.EDGE_SUM_STRIDE, dtype=torch.float64, device=dev)
        ops.prepare(0.0)
        ops.linearize(0, Ep, es)  # every edge: the real system of the N-GPU run
        for _ in range(3):
            Twc.copy_(T0)
            ops.linearize(0, ee0, es[:ee0])
            ops.solve(es)
        torch.cuda.synchronize()
        t_lin, t_sol = [], []
        for _ in range(REPS):
            Twc.copy_(T0)
            a, b, c = ev(), ev(), ev()
            a.record()
            ops.linearize(0, ee0, es[:ee0])
            b.record()
            ops.solve(es)
            c.record()
            t_lin.append((a, b))
            t_sol.append((b, c))
        torch.cuda.synchronize()
        lin = sum(x.elapsed_time(y) for x, y in t_lin) / REPS * 1e3
        sol = sum(x.elapsed_time(y) for x, y in t_sol) / REPS * 1e3
        fail = int(ops.info[be.INFO_SOLVE_FAIL])
        assert fail == 0, f"{m} N={N}: {fail} failed factorisations"

        # cold vs warm calls: prepare + 10 x (rank 0's linearize + solve of the
        # whole system), host clock, synchronised; the edge sums of the other
        # ranks are the ones computed above (es rows past ee0 are untouched)
        def call():
            Twc.copy_(T0)
            ops.prepare(0.0)
            for _ in range(10):
                ops.linearize(0, ee0, es[:ee0])
                ops.solve(es)

        def timed_calls():
            call()
            torch.cuda.synchronize()
            ts = []
            for _ in range(CALLS):
                t0 = time.perf_counter()
                call()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            return sorted(ts)[len(ts) // 2] * 1e6

        warm_call = timed_calls()
        with be.knob("plan_cache", 0):
            cold_call = timed_calls()
        assert int(ops.info[be.INFO_SOLVE_FAIL]) == 0
        cold = max(0.0, cold_call - warm_call)
        ops.close()
        del ops, es
        torch.cuda.empty_cache()
        ag = AG_US if world > 1 else 0.0
        t = lin + sol + ag
        tc = t + cold / 10
        base.setdefault(m, t)
        print(f"{m:5s} world {world} N={N} E={E} rank0={ee0}: linearize {lin:7.1f} us  solve {sol:7.1f} us  "
              f"all-gather {ag:5.1f} us (stated)  iteration {t:7.1f} us -> eff {base[m] / t:.3f} | "
              f"call warm {warm_call:8.1f} us cold {cold_call:8.1f} us: cold-plan {cold:7.1f} us/call "
              f"({cold / 10:6.1f} us/it) -> eff cold {base[m] / tc:.3f}  (fail 0)", flush=True)
    del g
    torch.cuda.empty_cache()
