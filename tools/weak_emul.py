"""Single-GPU emulation of one rank of the N-GPU weak-scaling bench.

Per GN iteration a rank linearizes its slice (~98 directed edges at 32 KFs per
GPU) and then runs the replicated solve of the whole 32*N-KF system. This
times both parts with HIP events on one GPU (the all-gather is not included)
and prints the predicted efficiency t_iter(1) / t_iter(N), for the sparse LLT,
the persistent dense LLT (M3S_SOLVER=pdense) and the dense fallback (M3S_DENSE=1). Calib model, 512x512 (bench.py).
"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402
from mast3r_slam_amd.distributed import HipOps, edge_slice  # noqa: E402

dev = torch.device("cuda:0")
H = W = int(os.environ.get("HW_SIDE", "512"))
REPS = int(os.environ.get("REPS", "20"))
modes = os.environ.get("MODES", "sparse,pdense").split(",")


def ev():
    return torch.cuda.Event(enable_timing=True)


base = None
for world in [int(x) for x in os.environ.get("WORLDS", "1,2,4,8").split(",")]:
    N = 32 * world
    probe = synthetic.make_graph(N, 4, 4, seed=1003, edge_range=(0, 0))
    E = probe.n_edges
    eb, ee, per = edge_slice(E, 0, world)
    g = synthetic.make_graph(N, H, W, seed=1003, device=dev, edge_range=(eb, ee))
    rays = synthetic.pixel_rays(H, W, g.K)
    Xs = (g.Xs[..., 2:3] * rays[None]).contiguous()
    Twc = g.T_init.data.contiguous().clone()
    row = {}
    for m in modes:
        os.environ["M3S_DENSE"] = "1" if m == "dense" else "0"
        os.environ["M3S_SOLVER"] = "pdense" if m == "pdense" else "sparse"
        ops = HipOps(be.MODE_CALIB, Twc, Xs, g.Cs.contiguous(), g.ii.contiguous(), g.jj.contiguous(),
                     g.idx_ii2jj, g.valid_match, g.Q, E, g.K, sigma_a=1.0, sigma_b=10.0, C_thresh=0.0,
                     Q_thresh=1.5, height=H, width=W, pixel_border=-10, z_eps=1e-6)
        es = torch.zeros(per * world, be.EDGE_SUM_STRIDE, dtype=torch.float64, device=dev)
        ops.prepare(0.0)
        ops.linearize(eb, ee, es[: ee - eb])  # gathering kernel + planes
        # the other ranks' rows: copies of this rank's (a well-posed stand-in)
        for r in range(1, world):
            b, e, _ = edge_slice(E, r, world)
            k = e - b
            es[r * per: r * per + k] = es[:k].repeat((k + ee - eb - 1) // (ee - eb), 1)[:k]
        for _ in range(3):
            ops.linearize(eb, ee, es[: ee - eb])
            ops.solve(es)
        torch.cuda.synchronize()
        t_lin, t_sol = [], []
        for _ in range(REPS):
            a, b, c = ev(), ev(), ev()
            a.record()
            ops.linearize(eb, ee, es[: ee - eb])
            b.record()
            ops.solve(es)
            c.record()
            t_lin.append((a, b))
            t_sol.append((b, c))
        torch.cuda.synchronize()
        lin = sum(x.elapsed_time(y) for x, y in t_lin) / REPS
        sol = sum(x.elapsed_time(y) for x, y in t_sol) / REPS
        fail = int(ops.info[be.INFO_SOLVE_FAIL])
        row[m] = (lin, sol, fail)
        del ops
        torch.cuda.empty_cache()
    best = min(row.values(), key=lambda v: v[0] + v[1])
    if base is None:
        base = best[0] + best[1]
    txt = "  ".join(f"{m}: lin {v[0] * 1e3:.1f} us solve {v[1] * 1e3:.1f} us (fail {v[2]})" for m, v in row.items())
    print(f"world {world} N={N} E={E} slice={ee - eb}: {txt}  -> eff {base / (best[0] + best[1]):.3f}",
          flush=True)
    del g, Xs
    torch.cuda.empty_cache()
