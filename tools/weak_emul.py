"""Single-GPU emulation of one rank of the N-GPU weak-scaling bench.

Per GN iteration a rank linearizes its slice (~98 directed edges at 32 KFs per
GPU) and then runs the replicated solve of the whole 32*N-KF system. This
builds the FULL synthetic graph of the N-GPU run (bench.py's generator and
seed), linearizes every edge once so that the edge sums are the real system,
then times, per iteration, rank 0's linearize of its own slice followed by the
solve of the whole system, with HIP events. The poses are reset before every
timed iteration, so each one solves the same real system. The all-gather
(36 fp64 per edge) is not included. Any failed factorisation aborts the run.

Prints t_iter(N) and the predicted efficiency t_iter(1) / t_iter(N).

env: MODES=calib,rays  WORLDS=1,2,4,8  HW_SIDE=512  REPS=20  M3S_LIB=variants/lib_X.so
"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402

if os.environ.get("M3S_LIB"):  # a library variant (tools/mkvar.sh) for A/B
    be._lib = be._load(os.path.abspath(os.environ["M3S_LIB"]))
from mast3r_slam_amd import synthetic  # noqa: E402
from mast3r_slam_amd.distributed import HipOps, edge_slice  # noqa: E402

dev = torch.device("cuda:0")
H = W = int(os.environ.get("HW_SIDE", "512"))
REPS = int(os.environ.get("REPS", "20"))
modes = os.environ.get("MODES", "calib,rays").split(",")
SIG = {"calib": (1.0, 10.0), "rays": (0.003, 10.0)}


def ev():
    return torch.cuda.Event(enable_timing=True)


base = {}
for world in [int(x) for x in os.environ.get("WORLDS", "1,2,4,8").split(",")]:
    N = 32 * world
    g = synthetic.make_graph(N, H, W, seed=1003, device=dev)
    E = g.n_edges
    _, ee0, _ = edge_slice(E, 0, world)
    rays = synthetic.pixel_rays(H, W, g.K)
    for m in modes:
        Xs = (g.Xs[..., 2:3] * rays[None]).contiguous() if m == "calib" else g.Xs.contiguous()
        T0 = g.T_init.data.contiguous().clone()
        Twc = T0.clone()
        mid = be.MODE_CALIB if m == "calib" else be.MODE_RAYS
        ops = HipOps(mid, Twc, Xs, g.Cs.contiguous(), g.ii.contiguous(), g.jj.contiguous(), g.idx_ii2jj,
                     g.valid_match, g.Q, E, g.K if m == "calib" else None, sigma_a=SIG[m][0],
                     sigma_b=SIG[m][1], C_thresh=0.0, Q_thresh=1.5, height=H, width=W, pixel_border=-10,
                     z_eps=1e-6)
        es = torch.zeros(E, be.EDGE_SUM_STRIDE, dtype=torch.float64, device=dev)
        ops.prepare(0.0)
        ops.linearize(0, E, es)  # every edge: the real system of the N-GPU run
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
        ops.close()
        del ops, es
        torch.cuda.empty_cache()
        t = lin + sol
        base.setdefault(m, t)
        print(f"{m:5s} world {world} N={N} E={E} slice={ee0}: linearize {lin:7.1f} us  solve {sol:7.1f} us  "
              f"iteration {t:7.1f} us  -> eff {base[m] / t:.3f}  (fail 0)", flush=True)
    del g
    torch.cuda.empty_cache()
