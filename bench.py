#!/usr/bin/env python
"""Benchmark: backend Gauss-Newton over dense 512x512 pointmap pairs on MI355X.

Workload (BASELINE.json configs[2], "C3"): a 32-keyframe loop-closure
FactorGraph in the calib residual model (config/calib.yaml -> use_calib), i.e.
``mast3r_slam_backends.gauss_newton_calib`` as ``FactorGraph.solve_GN_calib``
calls it (global_opt.py:190-210), 512x512 synthetic pointmaps, two-way edges
(E_dir ~ 98), max_iter = 10 with delta_thresh = 0 so every step runs exactly 10
GN iterations.

One "step" = one full solve call (10 GN iterations). Multi-GPU (weak scaling):
N GPUs solve a graph of 32*N keyframes (~98*N directed edges) with the edges
sharded across ranks and one RCCL all-gather of per-edge normal equations per
GN iteration (mast3r_slam_amd/distributed.py).

value = directed 512x512 pair-linearisations inside full GN iterations per
second, whole job (= E_dir * GN iterations / s); ``gn_iters_per_s`` is given
beside it. Inputs are resident in HBM before the timed region.

Extra legs on rank 0 at N = 1:
  roofline     — the linearize kernel timed alone with HIP events on its stream
  cpu_baseline — the CPU oracle (C restatement of gn_kernels.cu, OpenMP) on one
                 GN iteration of the same graph
  tracker_c2   — configs[1]: single-pair tracker GN at 512x512, fixed 10 iters
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "mast3r-slam-ysh_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--kf-per-gpu", type=int, default=32)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--lin-reps", type=int, default=30)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-tracker", action="store_true")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import mast3r_slam_backends as be
    from mast3r_slam_amd import synthetic
    from mast3r_slam_amd.distributed import ShardedGN, edge_slice

    H, W = args.height, args.width
    HW = H * W
    N = args.kf_per_gpu * world
    # full edge list first (cheap), then only this rank's slice of edge data
    probe = synthetic.make_graph(N, 4, 4, seed=1003, edge_range=(0, 0))
    E = probe.n_edges
    eb, ee, _ = edge_slice(E, rank, world)
    t0 = time.time()
    g = synthetic.make_graph(N, H, W, seed=1003, device=dev, edge_range=(eb, ee))
    assert g.n_edges == E
    # calib inputs are ray-constrained by the caller (global_opt.py:172)
    rays = synthetic.pixel_rays(H, W, g.K)
    Xs = (g.Xs[..., 2:3] * rays[None]).contiguous()
    Cs = g.Cs.contiguous()
    T_init = g.T_init.data.contiguous()
    Twc = T_init.clone()
    ii, jj = g.ii.contiguous(), g.jj.contiguous()
    idx, valid, Q = g.idx_ii2jj, g.valid_match, g.Q
    torch.cuda.synchronize()
    log(f"[rank {rank}] graph N={N} E_dir={E} slice=[{eb},{ee}) built in {time.time() - t0:.1f}s")

    calib = dict(sigma_a=1.0, sigma_b=10.0, C_thresh=0.0, Q_thresh=1.5, height=H, width=W,
                 pixel_border=-10, z_eps=1e-6)
    solver = ShardedGN(be.MODE_CALIB, Twc, Xs, Cs, ii, jj, idx, valid, Q, E, g.K, **calib)
    info = torch.zeros(8, dtype=torch.int32, device=dev)

    def step():
        Twc.copy_(T_init)
        if world == 1:  # the drop-in entry point itself
            be.gauss_newton_calib(Twc, Xs, Cs, g.K, ii, jj, idx, valid, Q, H, W, -10, 1e-6, 1.0,
                                  10.0, 0.0, 1.5, args.iters, 0.0, info=info)
        else:
            solver.solve(args.iters, 0.0)

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    iters_total = args.iters * args.steps
    gn_iters_per_s = iters_total / elapsed
    value = E * gn_iters_per_s
    if world == 1:
        assert int(info[be.INFO_ITERS]) == args.iters and int(info[be.INFO_BAD_EDGE]) == 0

    # ---- roofline: the dominant kernel, HIP events on its stream ----
    # GN iterations 2..10 of a call run linearize_packed_kernel (the first one
    # runs the gathering kernel that also stores the target-side planes). It
    # is timed in the solve's own launch pattern (linearize -> LLT -> ...):
    # an event pair around each linearize launch of stepwise solves of the
    # same graph (the pair also covers the launch's ~3 us per-edge reduce).
    # The same kernel launched back to back is timed too, for reference.
    n_loc = ee - eb
    kf_touched = torch.unique(torch.cat([ii[eb:ee], jj[eb:ee]])).numel() if n_loc else 0
    bytes_alg = HW * (13 * n_loc + 16 * kf_touched)  # SURVEY.md §8(d) per (edge, px) and (KF, px)
    stream = torch.cuda.current_stream(dev)
    in_solve = []
    for rep in range(4):
        Twc.copy_(T_init)
        t = solver.solve_timed(args.iters, 0.0, stream)
        if rep:  # the first call is a warm-up
            in_solve += t[1:]  # iterations 2.. (packed kernel)
    lin_ms = sum(in_solve) / len(in_solve)
    Twc.copy_(T_init)
    be.gn_prepare(solver.args, solver.keep)
    solver.linearize_only()  # first launch: gathering kernel + planes
    for _ in range(5):  # warm launches right before the timed ones
        solver.linearize_only()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(args.lin_reps):
        solver.linearize_only()
    ev1.record(stream)
    torch.cuda.synchronize()
    b2b_ms = ev0.elapsed_time(ev1) / args.lin_reps  # back-to-back launches, per-launch average
    achieved = bytes_alg / (lin_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_linearize_c3.json")
    if os.path.exists(pmc_path) and world == 1:
        try:
            traffic = json.load(open(pmc_path)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "512x512-pair GN iterations/s (E_dir x GN iterations per second, whole job)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded ray-cast room, SURVEY.md §8d); no datasets/weights offline",
        "config": {
            "workload": "C3: %d-KF loop-closure FactorGraph, gauss_newton_calib, %dx%d, "
                        "%d GN iterations per step (delta_thresh=0)" % (N, H, W, args.iters),
            "keyframes": N,
            "directed_edges": E,
            "pixels_per_pointmap": HW,
            "gn_iters_per_step": args.iters,
            "solve": "fp64 block-sparse 7x7 LLT on device (min-degree order), n=%d" % (7 * (N - 1)),
            "parallelism": "edge-sharded x%d, RCCL all-gather of per-edge normal equations" % world
            if world > 1 else "single GPU",
        },
        "gn_iters_per_s": round(gn_iters_per_s, 2),
        "roofline": {
            "bound": "hbm",
            "kernel": "linearize_packed_kernel<calib> (%d edges x %d px per launch; GN "
                      "iterations 2..%d of each call)" % (n_loc, HW, args.iters),
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "algorithmic_bytes_per_launch": bytes_alg,
            "avg_launch_ms": round(lin_ms, 5),
            "timing": "HIP events around each linearize launch of stepwise solves (its launch pattern "
                      "in the timed region); back_to_back_ms = the same kernel launched back to back",
            "back_to_back_ms": round(b2b_ms, 5),
            "iteration_level": {
                "achieved": round(bytes_alg * gn_iters_per_s / 1e9, 1) if world == 1 else None,
                "note": "SURVEY.md §8(d) B_iter x GN iterations/s (whole iteration: linearize, "
                        "reduce, assemble, LLT, retraction)",
            },
        },
    }

    if rank == 0 and world == 1 and not args.no_tracker:
        out["tracker_c2"] = tracker_leg(be, synthetic, dev, H, W)
        out["matching_512"] = matching_leg(be, synthetic, dev, H, W)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_leg(g, Xs, ii, jj, idx, valid, Q, T_init, H, W, E)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def tracker_leg(be, synthetic, dev, H, W, iters=10, reps=50):
    """configs[1]: single-keyframe tracking GN at 512x512 (replicas only)."""
    p = synthetic.make_pair(H, W, seed=1002, device=dev)
    a = (p.Xf.contiguous(), p.Xk.contiguous(), p.T_WCf_init.data.contiguous(), p.T_WCk.data.contiguous(),
         p.Qk.contiguous(), p.valid.contiguous())
    call = lambda: be.track_rays_sim3(*a, 0.003, 10.0, 1.345, iters, 0.0, 0.0, sync_every=0)  # noqa: E731
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = call()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert int(out[2][0]) == iters
    return {"workload": "C2: 1 frame->keyframe pair, rays+dist Sim3 GN, %dx%d, %d fixed iterations"
                        % (H, W, iters),
            "gn_iters_per_s": round(reps * iters / dt, 1), "ms_per_solve": round(dt / reps * 1e3, 4)}


def matching_leg(be, synthetic, dev, H, W, reps=20):
    """iter_proj + refine_matches on one 512x512 view pair
    (matching.py:52-90 with base.yaml's matching config)."""
    from mast3r_slam_amd import matching

    m = synthetic.make_match_inputs(H, W, device=dev)
    img, pts, p0 = matching.prep_for_iter_proj(m.X11, m.X21)
    X11, X21 = m.X11.contiguous(), m.X21.contiguous()
    cfg = matching.MATCHING_CFG
    p1 = be.iter_proj(img, pts, p0, cfg["max_iter"], cfg["lambda_init"], cfg["convergence_thresh"])[0].long()
    times = {}
    for name, fn in (
        ("iter_proj", lambda: be.iter_proj(img, pts, p0, cfg["max_iter"], cfg["lambda_init"],
                                           cfg["convergence_thresh"])),
        ("refine_matches", lambda: be.refine_matches(m.D11, m.D21, p1, cfg["radius"], cfg["dilation_max"])),
        ("prep_rays", lambda: be.prep_rays(X11, X21)),
    ):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        times[name] = round(e0.elapsed_time(e1) / reps, 4)
    return {"workload": "one %dx%d view pair, F=%d float16 descriptors, matching config of base.yaml"
                        % (H, W, m.D11.shape[-1]),
            "ms_iter_proj": times["iter_proj"], "ms_refine_matches": times["refine_matches"],
            "ms_prep_rays": times["prep_rays"]}


def cpu_leg(g, Xs, ii, jj, idx, valid, Q, T_init, H, W, E):
    """The CPU oracle (oracle/gn_oracle.c, OpenMP) on one GN iteration of the
    same graph; reported, not the target."""
    from oracle import oracle as orc

    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    p = orc.make_params(orc.MODE_CALIB, 1.0, 10.0, 0.0, 1.5, K=g.K.cpu().numpy(), height=H, width=W,
                        pixel_border=-10, z_eps=1e-6)
    host = [t.cpu().numpy() for t in (T_init, Xs, g.Cs, ii, jj, idx, valid, Q)]
    t0 = time.perf_counter()
    _, _, it, _ = orc.gn(p, *host, 1, 0.0)
    dt = time.perf_counter() - t0
    return {"value": round(E * it / dt, 2), "unit": "512x512-pair GN iterations/s", "cores": cores,
            "kind": "port",
            "sample": "1 full GN iteration (linearise %d directed edges + fp64 solve) of the same graph, "
                      "%.1f s" % (E, dt)}


if __name__ == "__main__":
    main()
