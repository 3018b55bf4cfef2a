#!/usr/bin/env python
"""Benchmark: backend Gauss-Newton over dense 512x512 pointmap pairs on MI355X.

Workload (BASELINE.json configs[2], "C3"): a 32-keyframe loop-closure
FactorGraph in the calib residual model (config/calib.yaml -> use_calib), i.e.
``mast3r_slam_backends.gauss_newton_calib`` as ``FactorGraph.solve_GN_calib``
calls it (global_opt.py:190-210), 512x512 synthetic pointmaps, two-way edges
(E_dir = 98), max_iter = 10 with delta_thresh = 0 so every step runs exactly 10
GN iterations.

One "step" = one full solve call (10 GN iterations). Multi-GPU (weak scaling):
N GPUs solve one graph of 32*N keyframes (~98*N directed edges) with the edges
sharded across ranks and one RCCL all-gather of per-edge normal equations per
GN iteration (mast3r_slam_amd/distributed.py).

value = GN iterations per second in units of the C3 graph (SURVEY.md §8d
"completed backend GN iterations / wall time"): at N = 1 exactly the GN
iterations/s of the 32-KF graph; at N GPUs the whole job's E_dir * GN it/s
divided by the C3 graph's E_dir, so that a weak-scaling run that keeps every
GPU as busy as one GPU on C3 reports N x the single-GPU value. The raw GN
iterations/s of the run's own graph (``gn_iters_per_s``) and the directed
512x512 pair-linearisations per second (``pair_iters_per_s``) are given
beside it. Inputs are resident in HBM before the timed region.

Launch: ``python bench.py --gpus N`` spawns N ranks (one process per GPU,
RCCL) when it is not already running under torch.distributed.run; under a
launcher, --gpus must equal WORLD_SIZE (else exit 2). ``--dry-run`` runs the
same orchestration on CPU/gloo with no-op per-rank compute (a plumbing check:
its timings mean nothing).

Extra legs on rank 0 at N = 1:
  cold         — the same steps with the host plan cache off (knob plan_cache=0):
                 the per-call symbolic analysis inside the timed region
  roofline     — the linearize kernel timed with HIP events on its stream
                 (+ the first-iteration gathering kernel and the solve launches)
  hbm_copy     — a measured streaming-copy rate (16-B nt copy kernel) next to the 8 TB/s spec
  cpu_baseline — the CPU oracle (C restatement of gn_kernels.cu, OpenMP) on one
                 GN iteration of the same graph (median of 5), and the PyTorch-CPU
                 tracker program of tracker.py on the C2 pair, all cores (median of 3)
  tracker_c2   — configs[1]: single-pair tracker GN at 512x512, fixed 10 iters
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import statistics
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
# shipped with the tree (profiles/ stays on the build host): the PMC record of the benched library
PMC_PATH = os.path.join(ROOT, "pmc", "linearize_c3.json")
SEED = 1003  # 1000 + config number


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--kf-per-gpu", type=int, default=32)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--width", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--mode", choices=("calib", "rays"), default="calib")
    ap.add_argument("--lin-reps", type=int, default=30)
    ap.add_argument("--cold-steps", type=int, default=5)
    ap.add_argument("--natural-steps", type=int, default=10)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-tracker", action="store_true")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU/gloo orchestration check with no-op compute (no GPU)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal of the N-rank path on a one-GPU box: every rank on cuda:0, gloo "
                         "collectives (RCCL refuses two ranks on one device); not a scaling measurement")
    return ap.parse_args(argv)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class NullOps:
    """--dry-run per-rank compute: the HipOps interface with no work, so the
    spawn / gloo collective / timing / JSON path runs on a CPU-only host."""

    stride = 36

    def __init__(self, N):
        self.device = torch.device("cpu")
        self.dx = torch.zeros(max(N - 1, 0), 7)
        self.info = torch.zeros(8, dtype=torch.int32)
        self.args = self.keep = None

    def prepare(self, delta):
        pass

    def linearize(self, eb, ee, es_loc):
        if es_loc is not None:
            es_loc.zero_()

    def solve(self, es):
        self.info[0] += 1

    def close(self):
        pass


def lib_digest():
    import mast3r_slam_backends as be

    h = hashlib.sha256()
    with open(be.LIB_PATH, "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def base_edges(args):
    """E_dir of the one-GPU (C3) graph: the unit of `value`."""
    from mast3r_slam_amd import synthetic

    return synthetic.make_graph(args.kf_per_gpu, 4, 4, seed=SEED, edge_range=(0, 0)).n_edges


def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dry = args.dry_run
    if dry:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    elif args.share_gpu:
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        if world > 1:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if world > 1:
            dist.init_process_group("nccl", device_id=dev)
    if world > 1:
        log(f"[rank {rank}] backend={dist.get_backend()} world_size={dist.get_world_size()} "
            f"local_rank={local} device={dev}")

    from mast3r_slam_amd import synthetic
    from mast3r_slam_amd.distributed import ShardedGN, edge_shard

    H, W = (8, 8) if dry else (args.height, args.width)
    HW = H * W
    N = args.kf_per_gpu * world
    calib_mode = args.mode == "calib"
    # full edge list first (cheap), then only this rank's slice of edge data
    probe = synthetic.make_graph(N, 4, 4, seed=SEED, edge_range=(0, 0))
    E = probe.n_edges
    E_base = base_edges(args)
    ids, _ = edge_shard(E, rank, world)  # both halves of each of this rank's undirected edges
    t0 = time.time()
    g = synthetic.make_graph(N, H, W, seed=SEED, device=dev, edge_ids=ids)
    assert g.n_edges == E
    if calib_mode:  # calib inputs are ray-constrained by the caller (global_opt.py:172)
        rays = synthetic.pixel_rays(H, W, g.K)
        Xs = (g.Xs[..., 2:3] * rays[None]).contiguous()
    else:
        Xs = g.Xs.contiguous()
    Cs = g.Cs.contiguous()
    T_init = g.T_init.data.contiguous()
    Twc = T_init.clone()
    ii, jj = g.ii.contiguous(), g.jj.contiguous()
    idx, valid, Q = g.idx_ii2jj, g.valid_match, g.Q
    if not dry:
        torch.cuda.synchronize()
    log(f"[rank {rank}] graph N={N} E_dir={E} {len(ids)} edges (pair-preserving shard) built in "
        f"{time.time() - t0:.1f}s")

    if dry:
        sig = dict(sigma_a=1.0)
        ops = NullOps(N)
        be = None
    else:
        import mast3r_slam_backends as be

        if calib_mode:
            sig = dict(sigma_a=1.0, sigma_b=10.0, C_thresh=0.0, Q_thresh=1.5, height=H, width=W,
                       pixel_border=-10, z_eps=1e-6)
        else:
            sig = dict(sigma_a=0.003, sigma_b=10.0, C_thresh=0.0, Q_thresh=1.5)
        ops = None
    mode_id = 2 if calib_mode else 1  # M3S_MODE_CALIB / M3S_MODE_RAYS (include/m3s_gn.h)
    solver = ShardedGN(mode_id, Twc, Xs, Cs, ii, jj, idx, valid, Q, E, g.K if calib_mode else None,
                       ops=ops, **sig)
    info = torch.zeros(8, dtype=torch.int32, device=dev)

    def step(delta=0.0, iters=None):
        iters = args.iters if iters is None else iters
        Twc.copy_(T_init)
        if world == 1 and not dry:  # the drop-in entry point itself
            if calib_mode:
                be.gauss_newton_calib(Twc, Xs, Cs, g.K, ii, jj, idx, valid, Q, H, W, -10, 1e-6, 1.0,
                                      10.0, 0.0, 1.5, iters, delta, info=info)
            else:
                be.gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx, valid, Q, 0.003, 10.0, 0.0, 1.5,
                                     iters, delta, info=info)
        else:
            solver.solve(iters, delta)

    def sync():
        if not dry:
            torch.cuda.synchronize()

    def timed(nsteps, delta=0.0):
        if world > 1:
            dist.barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(nsteps):
            step(delta)
        sync()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t)
        return el

    for _ in range(args.warmup):
        step()
    elapsed = timed(args.steps)
    iters_total = args.iters * args.steps
    gn_iters_per_s = iters_total / elapsed
    pair_iters_per_s = E * gn_iters_per_s
    value = pair_iters_per_s / E_base
    if world == 1 and not dry:
        assert int(info[be.INFO_ITERS]) == args.iters and int(info[be.INFO_BAD_EDGE]) == 0
        assert int(info[be.INFO_SOLVE_FAIL]) == 0

    # cold calls: the host symbolic analysis (ordering, fill, schedule) inside
    # the timed region, as a SLAM backend call whose edge set changed pays it
    if dry:
        cold_el = None
    else:
        with be.knob("plan_cache", 0):
            cold_el = timed(args.cold_steps) if args.cold_steps > 0 else None

    # natural termination (reported separately): the same calls
    # with the reference's delta_thresh = 1e-8 (config/base.yaml:49) and
    # max_iter = 10; the device stop flag ends the loop when a step's norm
    # falls below delta, and the iterations actually run are counted
    natural = None
    if not dry and args.natural_steps > 0:
        step(1e-8)  # warm-up of the delta path
        nat_el = timed(args.natural_steps, 1e-8)
        nat_iters = int(solver.ops.info[0]) if world > 1 else int(info[be.INFO_ITERS])
        natural = {
            "delta_thresh": 1e-8, "max_iter": args.iters, "calls": args.natural_steps,
            "iters_per_call": nat_iters,
            "ms_per_call": round(nat_el / args.natural_steps * 1e3, 4),
            "gn_iters_per_s": round(nat_iters * args.natural_steps / nat_el, 2),
            "note": "config/base.yaml:49 delta; the fp32 steps of this seeded graph stay above 1e-8, so "
                    "every call runs max_iter iterations (tests/test_gpu_large.py checks the same)"}

    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GN iterations/s of the 32-KF C3 graph (E_dir x GN it/s / 98; = GN it/s at N=1), whole job",
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
            "workload": "%s: %d-KF loop-closure FactorGraph, gauss_newton_%s, %dx%d, "
                        "%d GN iterations per step (delta_thresh=0)"
                        % ("C3" if world == 1 and calib_mode else "weak-scaled C3", N, args.mode, H, W,
                           args.iters),
            "keyframes": N,
            "directed_edges": E,
            "pixels_per_pointmap": HW,
            "gn_iters_per_step": args.iters,
            "solve": "fp64 block-sparse 7x7 LLT on device (min-degree order), n=%d" % (7 * (N - 1)),
            "parallelism": "edge-sharded x%d (pair-preserving), %s all-gather of per-edge normal equations"
            % (world, "RCCL" if dist.get_backend() == "nccl" else dist.get_backend())
            if world > 1 else "single GPU",
        },
        "gn_iters_per_s": round(gn_iters_per_s, 2),
        "pair_iters_per_s": round(pair_iters_per_s, 1),
        "natural_termination": natural,
        "cold": {
            "ms_per_step": round(cold_el / args.cold_steps * 1e3, 4) if cold_el else None,
            "gn_iters_per_s": round(args.iters * args.cold_steps / cold_el, 2) if cold_el else None,
            "note": "plan cache off (knob plan_cache=0): every call re-runs the host symbolic "
                    "analysis, as a call on a changed edge set does",
        },
    }
    if dry:
        out["dry_run"] = True
        out["data"] = "dry run: CPU/gloo orchestration with no-op compute; timings are meaningless"
    elif args.share_gpu and world > 1:
        out["share_gpu"] = True
        out["data"] = ("rehearsal: %d ranks sharing ONE GPU over gloo (the product path, HIP compute); "
                       "not a scaling measurement" % world)
    else:
        out["roofline"] = roofline_leg(args, solver, be, Twc, T_init, ii, jj, ids, HW, gn_iters_per_s,
                                       world, dev, step if world == 1 else None, elapsed / args.steps)

    if rank == 0 and world == 1 and not dry:
        out["hbm_copy"] = copy_leg(be, dev)
        out["roofline"]["frac_of_measured_copy"] = round(out["roofline"]["achieved"] / out["hbm_copy"]["GB_per_s"], 4)
        if not args.no_tracker:
            out["tracker_c2"] = tracker_leg(be, synthetic, dev, H, W)
            out["matching_512"] = matching_leg(be, synthetic, dev, H, W)
        if not args.no_cpu:
            out["cpu_baseline"] = cpu_leg(g, Xs, ii, jj, idx, valid, Q, T_init, H, W, E, calib_mode,
                                          not args.no_tracker)
    solver.ops.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def roofline_leg(args, solver, be, Twc, T_init, ii, jj, ids, HW, gn_iters_per_s, world, dev, call=None,
                 step_s=None):
    """The dominant kernel: GN iterations 2..10 of a call run
    linearize_packed_kernel (the first runs the gathering kernel that also
    stores the target-side planes).

    At N = 1 (round 6, reconciled with the timed steps): the packed kernel's
    time per launch in the benched calls themselves is
        (T_10 - T_1) / 9 - solve,
    T_10 / T_1 the per-call times of un-instrumented drop-in calls with 10 and
    1 GN iterations (HIP events around batches of calls, interleaved), solve
    the LLT dispatch's own span. The instrumented calls (m3s_debug_call_timing:
    each linearize and the one-launch solve through hipExtLaunchKernel with
    the dispatch's begin / end events) give the gathering launch, the solve
    and the packed kernel's dispatch span as a cross-check; spans x launches
    is reported beside ms_per_step. A sharded rank times its stepwise solve's
    linearize launches (their per-edge reduce included). The same kernel
    launched back to back is timed too."""
    n_loc = len(ids)
    sel = torch.tensor(ids, dtype=torch.int64, device=ii.device)
    kf_touched = torch.unique(torch.cat([ii[sel], jj[sel]])).numel() if n_loc else 0
    bytes_alg = HW * (13 * n_loc + 16 * kf_touched)  # SURVEY.md §8(d) per (edge, px) and (KF, px)
    stream = torch.cuda.current_stream(dev)
    lin, first, slv = [], [], []
    if call is not None:
        call()  # warm-up
        torch.cuda.synchronize()
        be.debug_call_timing(True)
        for _ in range(5):
            call()
        spans = be.debug_call_times()
        be.debug_call_timing(False)
        assert len(spans) == 5 * 2 * args.iters, len(spans)
        first = [ms for k, ms in spans if k == 0]
        lin = [ms for k, ms in spans if k == 1]
        slv = [ms for k, ms in spans if k == 2]
        # un-instrumented calls of 10 and 1 GN iterations, interleaved batches
        t_n, t_1 = [], []
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _ in range(4):
            for iters, acc in ((args.iters, t_n), (1, t_1)):
                call(iters=iters)
                ev[0].record()
                for _ in range(10):
                    call(iters=iters)
                ev[1].record()
                torch.cuda.synchronize()
                acc.append(ev[0].elapsed_time(ev[1]) / 10)
        call_n, call_1 = statistics.median(t_n), statistics.median(t_1)
        slv_ms = sum(slv) / len(slv)
        lin_step = (call_n - call_1) / (args.iters - 1) - slv_ms
        timing = ("packed launch time in the benched calls: (T_%d - T_1) / %d - solve, T_k = per-call time of "
                  "un-instrumented drop-in calls of k GN iterations (HIP events around 4 x 10 calls each, "
                  "interleaved; medians), solve = the LLT dispatch's own span (hipExtLaunchKernel); "
                  "dispatch_span_ms = the packed dispatch's own span in 5 instrumented calls; back_to_back_ms = "
                  "the same kernel launched back to back (HIP events around the run)"
                  % (args.iters, args.iters - 1))
    else:
        for rep in range(4):
            Twc.copy_(T_init)
            t_lin, t_slv = solver.solve_timed(args.iters, 0.0, stream)
            if rep:  # the first call is a warm-up
                first.append(t_lin[0])
                lin += t_lin[1:]  # iterations 2.. (packed kernel)
                slv += t_slv
        timing = ("HIP events around each linearize launch (+ its per-edge reduce) of this rank's "
                  "stepwise solves; back_to_back_ms = the same kernel launched back to back")
    span_ms = sum(lin) / len(lin)
    lin_ms = lin_step if call is not None else span_ms
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
    b2b_ms = ev0.elapsed_time(ev1) / args.lin_reps
    achieved = bytes_alg / (lin_ms * 1e-3) / 1e9
    first_ms = sum(first) / len(first)
    traffic, traffic_note, gather_traffic = None, "no PMC record", None
    if os.path.exists(PMC_PATH) and world == 1 and args.mode == "calib":
        rec = json.load(open(PMC_PATH))
        if rec.get("lib_sha256_16") == lib_digest() and rec.get("kf") == args.kf_per_gpu:
            traffic = rec.get("hbm_bytes_per_launch")
            traffic_note = rec.get("note", "PMC pass of this library build")
            g = rec.get("gather") or {}
            if g.get("lib_sha256_16") == rec.get("lib_sha256_16"):
                gather_traffic = {"read": g.get("hbm_bytes_per_launch"), "write": g.get("hbm_write_bytes_per_launch")}
        else:
            traffic_note = "PMC record is of another library build: not reported"
    return {
        "bound": "hbm",
        "kernel": "linearize_packed_kernel<%s> (%d edges x %d px per launch; GN iterations 2..%d "
                  "of each call)" % (args.mode, n_loc, HW, args.iters),
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "traffic_note": traffic_note,
        "algorithmic_bytes_per_launch": bytes_alg,
        "avg_launch_ms": round(lin_ms, 5),
        "timing": timing,
        "dispatch_span_ms": round(span_ms, 5),
        "in_call_ms_min_max": [round(min(lin), 5), round(max(lin), 5)],
        "back_to_back_ms": round(b2b_ms, 5),
        "gather_kernel": {
            "kernel": "linearize_gather_kernel (first GN iteration: streams prefetched by LDS-DMA, gathers Xi/Ci through idx, stores planes)",
            "avg_launch_ms": round(first_ms, 5),
            "achieved": round(bytes_alg / (first_ms * 1e-3) / 1e9, 1),
            "frac": round(bytes_alg / (first_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "traffic": gather_traffic,
        },
        "solve": {
            "kernels": "fp64 block-sparse LLT + retraction: every solve launch of one GN iteration "
                       "(at N = 1 the one sparse_llt_kernel dispatch's own span; the stepwise path's finalize + "
                       "assemble included at N > 1)",
            "avg_ms": round(sum(slv) / len(slv), 5),
            "bound": "latency (elimination-tree critical path, DESIGN.md §4)",
        },
        "reconcile": None if call is None else {
            "ms_per_step": round(step_s * 1e3, 5) if step_s else None,
            "call_ms": {str(args.iters): round(call_n, 5), "1": round(call_1, 5)},
            "spans_x_launches_ms": round(first_ms + (args.iters - 1) * lin_ms + args.iters * slv_ms, 5),
            "ratio_to_ms_per_step": round((first_ms + (args.iters - 1) * lin_ms + args.iters * slv_ms)
                                          / (step_s * 1e3), 4) if step_s else None,
            "note": "gathering span + %d x packed + %d x solve; the rest of a call is its prologue kernel and "
                    "the inter-call gap" % (args.iters - 1, args.iters)},
        "iteration_level": {
            "achieved": round(bytes_alg * gn_iters_per_s / 1e9, 1) if world == 1 else None,
            "note": "SURVEY.md §8(d) B_iter x GN iterations/s (whole iteration: linearize, "
                    "reduce, assemble, LLT, retraction)",
        },
    }


def copy_leg(be, dev, nbytes=1 << 30, reps=20):
    """Measured HBM ceiling beside the 8 TB/s spec: the 16-B non-temporal
    streaming copy kernel (m3s_debug_copy; the guide's float4 copy reaches
    6.29 TB/s) over 1 GiB, best grid of a small sweep, read + write bytes;
    torch's copy_ timed beside it."""
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev).fill_(1.0)
    b = torch.empty_like(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def rate(fn):
        fn()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return 2 * nbytes / (e0.elapsed_time(e1) / reps * 1e-3) / 1e9

    sweep = {blk: rate(lambda blk=blk: be.debug_copy(a, b, blk)) for blk in (1024, 2048, 4096, 8192)}
    best = max(sweep, key=sweep.get)
    out = {"GB_per_s": round(sweep[best], 1), "bytes_moved": 2 * nbytes, "blocks": best,
           "sweep_GB_per_s": {str(k): round(v, 1) for k, v in sweep.items()},
           "torch_copy_GB_per_s": round(rate(lambda: b.copy_(a)), 1),
           "note": "m3s_debug_copy: 16-B nt loads/stores, 4 in flight per lane, 1 GiB, read + write bytes"}
    assert torch.equal(a, b)
    return out


def tracker_leg(be, synthetic, dev, H, W, iters=10, reps=50):
    """configs[1]: single-keyframe tracking GN at 512x512 (replicas only).
    The default path is the persistent one-launch tracker; the launch-per-
    iteration path (knob track_persistent=0) is timed beside it."""
    p = synthetic.make_pair(H, W, seed=1002, device=dev)
    a = (p.Xf.contiguous(), p.Xk.contiguous(), p.T_WCf_init.data.contiguous(), p.T_WCk.data.contiguous(),
         p.Qk.contiguous(), p.valid.contiguous())
    call = lambda: be.track_rays_sim3(*a, 0.003, 10.0, 1.345, iters, 0.0, 0.0, sync_every=0)  # noqa: E731

    def timed():
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            out = call()
        torch.cuda.synchronize()
        assert int(out[2][0]) == iters
        return time.perf_counter() - t0

    dt = timed()
    with be.knob("track_persistent", 0):
        dt_l = timed()
    return {"workload": "C2: 1 frame->keyframe pair, rays+dist Sim3 GN, %dx%d, %d fixed iterations"
                        % (H, W, iters),
            "gn_iters_per_s": round(reps * iters / dt, 1), "ms_per_solve": round(dt / reps * 1e3, 4),
            "path": "persistent (one launch per solve; pixel inputs register-resident after iteration 1)",
            "bytes_per_solve": 45 * H * W,
            "bound": "latency: one grid-wide arrival + all-partials read per iteration",
            "launch_per_iter": {"gn_iters_per_s": round(reps * iters / dt_l, 1),
                                "ms_per_solve": round(dt_l / reps * 1e3, 4),
                                "note": "knob track_persistent=0: one linearize launch per iteration, "
                                        "45 B per pixel re-read each time"}}


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


def cpu_leg(g, Xs, ii, jj, idx, valid, Q, T_init, H, W, E, calib_mode, with_tracker, runs=5):
    """Reported, not the target. Backend: the C oracle (oracle/gn_oracle.c,
    OpenMP over edges) on one full GN iteration of the same graph, median of
    `runs`. Tracker: the PyTorch-CPU restatement of tracker.py on the C2 pair, 10
    fixed iterations of the reference's PyTorch program on all cores, median of 3."""
    from mast3r_slam_amd import synthetic
    from oracle import oracle as orc
    from oracle import tracker_oracle as tro

    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    if calib_mode:
        p = orc.make_params(orc.MODE_CALIB, 1.0, 10.0, 0.0, 1.5, K=g.K.cpu().numpy(), height=H, width=W,
                            pixel_border=-10, z_eps=1e-6)
    else:
        p = orc.make_params(orc.MODE_RAYS, 0.003, 10.0, 0.0, 1.5)
    host = [t.cpu().numpy() for t in (T_init, Xs, g.Cs, ii, jj, idx, valid, Q)]
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        _, _, it, _ = orc.gn(p, *host, 1, 0.0)
        ts.append(time.perf_counter() - t0)
    med = statistics.median(ts)
    out = {"value": round(it / med, 3), "unit": "GN iterations/s of the same graph (C oracle)",
           "cores": cores, "kind": "port",
           "pair_iters_per_s": round(E * it / med, 2),
           "sample": "1 full GN iteration (linearise %d directed edges + fp64 solve) of the same graph, "
                     "median of %d runs: %.3f s (min %.3f, max %.3f)" % (E, runs, med, min(ts), max(ts))}
    if with_tracker:
        # the reference's own CPU/PyTorch tracker program (oracle/tracker_torch.py,
        # pinned by the tracker fixtures) on all host cores
        from oracle import tracker_torch as trt

        pr = synthetic.make_pair(H, W, seed=1002)
        cfg = dict(tro.TRACKING_CFG, max_iters=10, rel_error=0.0, delta_norm=0.0)
        threads_before = torch.get_num_threads()
        torch.set_num_threads(cores)
        try:
            targs = (pr.Xf, pr.Xk, pr.T_WCf_init.data, pr.T_WCk.data, pr.Qk, pr.valid, cfg)
            trt.track_rays(*targs)  # warm-up
            tt = []
            for _ in range(3):
                t0 = time.perf_counter()
                _, _, it2 = trt.track_rays(*targs)
                tt.append(time.perf_counter() - t0)
        finally:
            torch.set_num_threads(threads_before)
        tm = statistics.median(tt)
        out["tracker"] = {"gn_iters_per_s": round(it2 / tm, 3), "cores": cores, "kind": "port",
                          "sample": "C2 pair %dx%d, %d fixed iterations of the PyTorch-CPU restatement of "
                                    "tracker.py (the reference's tensor program), torch threads %d, median of 3: "
                                    "%.3f s" % (H, W, it2, cores, tm)}
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_entry(local_rank, argv, world, port):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run(parse(argv))


def main(argv=None):
    args = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            log(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}; refusing to run")
            sys.exit(2)
        run(args)
        return
    if args.gpus <= 1:
        run(args)
        return
    # one process per GPU, spawned before this process touches the GPU
    import torch.multiprocessing as mp

    log(f"bench.py: spawning {args.gpus} ranks")
    mp.start_processes(_rank_entry, args=(sys.argv[1:] if argv is None else argv, args.gpus, _free_port()),
                       nprocs=args.gpus, join=True, start_method="spawn")


if __name__ == "__main__":
    main()
