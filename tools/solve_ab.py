"""Solve-kernel A/B at the multi-GPU graph sizes: whole drop-in GN calls on a
32*G-KF graph (bench.py's edges, seed 1003) with tiny images, so the call
time is the solve's. Runs the test build (knobs), alternating the knob
settings in SOLVE_AB ("name=v;name=v|name=v" groups), prints the median call
time per setting and whether poses agree bitwise with the first setting.
Under rocprofv3 --kernel-trace --stats the per-kernel times come out too.

usage: python tools/solve_ab.py   (env: SOLVE_N="128,256" SOLVE_AB="tail_pair=1|tail_pair=0"
                                    SOLVE_MODE=calib SOLVE_ITERS=3 SOLVE_ROUNDS=7
                                    LIB=variants/lib_X_test.so: another test build)
"""
import os
import statistics
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]

import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402


def main():
    be._lib = be._load(os.path.abspath(os.environ["LIB"])) if os.environ.get("LIB") else be.load_test_library()
    dev = torch.device("cuda:0")
    mode = os.environ.get("SOLVE_MODE", "calib")
    iters = int(os.environ.get("SOLVE_ITERS", "3"))
    rounds = int(os.environ.get("SOLVE_ROUNDS", "7"))
    groups = [dict(kv.split("=") for kv in g.split(";") if kv) for g in os.environ.get("SOLVE_AB", "tail_pair=1|tail_pair=0").split("|")]
    H, W = 12, 16
    for N in [int(x) for x in os.environ.get("SOLVE_N", "128,256").split(",")]:
        g = synthetic.make_graph(N, H, W, seed=1003, device=dev)
        calib = mode == "calib"
        Xs = (g.Xs[..., 2:3] * synthetic.pixel_rays(H, W, g.K)[None]).contiguous() if calib else g.Xs.contiguous()
        times = [[] for _ in groups]
        outs = [None] * len(groups)
        for rnd in range(rounds):
            # rotate the order every round (no setting always runs first)
            order = list(range(len(groups)))
            for gi in order[rnd % len(order):] + order[:rnd % len(order)]:
                grp = groups[gi]
                old = {k: be.set_knob(k, int(v)) for k, v in grp.items()}
                Twc = g.T_init.data.clone().contiguous()
                info = torch.zeros(8, dtype=torch.int32, device=dev)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if calib:
                    (dx,) = be.gauss_newton_calib(Twc, Xs, g.Cs, g.K, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q, H, W,
                                                  -10, 1e-6, 1.0, 10.0, 0.0, 1.5, iters, 0.0, info=info)
                else:
                    (dx,) = be.gauss_newton_rays(Twc, Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q, 0.003,
                                                 10.0, 0.0, 1.5, iters, 0.0, info=info)
                e1.record()
                torch.cuda.synchronize()
                if rnd:
                    times[gi].append(e0.elapsed_time(e1))
                outs[gi] = (Twc.cpu(), dx.cpu(), info.cpu())
                for k, v in old.items():
                    be.set_knob(k, v)
        for gi, grp in enumerate(groups):
            same = all(torch.equal(a, b) for a, b in zip(outs[gi], outs[0]))
            inf = outs[gi][2].tolist()
            print(f"N={N} {mode} {grp}: {statistics.median(times[gi]):.4f} ms/call ({iters} it) "
                  f"info={inf[:4]} bitwise_vs_first={same}", flush=True)


if __name__ == "__main__":
    main()
