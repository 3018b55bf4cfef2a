"""Per-call time of the GN solve under solver-knob settings (GPU box).

  KNOBS='[{"df": 1}, {"df": 0}]' python tools/knob_ab.py
  (M3S_LIB=variants/lib_X.so in the env for a variant library)

Small images (linearize negligible) so the call time is the solve path:
median of 20 calls (HIP events) per (graph, knob setting), in one process,
settings interleaved round-robin to cancel drift."""
import json
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402

if os.environ.get("M3S_LIB"):
    be._lib = be._load(os.path.abspath(os.environ["M3S_LIB"]))
from mast3r_slam_amd import synthetic  # noqa: E402

dev = torch.device("cuda:0")
GRAPHS = [("calib", 32, 64, 64, 10), ("rays", 140, 32, 32, 3), ("rays", 256, 32, 32, 3)]
SETTINGS = json.loads(os.environ.get("KNOBS", "[{}]"))
REPS = int(os.environ.get("REPS", "20"))

for mode, N, H, W, iters in GRAPHS:
    g = synthetic.make_graph(N, H, W, seed=4242 + N, device=dev)
    Xs = (g.Xs[..., 2:3] * synthetic.pixel_rays(H, W, g.K)[None]).contiguous() if mode == "calib" else g.Xs

    def call():
        Twc = g.T_init.data.clone().contiguous()
        if mode == "calib":
            be.gauss_newton_calib(Twc, Xs, g.Cs, g.K, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q, H, W, -10, 1e-6,
                                  1.0, 10.0, 0.0, 1.5, iters, 0.0)
        else:
            be.gauss_newton_rays(Twc, Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q, 0.003, 10.0, 0.0, 1.5,
                                 iters, 0.0)

    times = {i: [] for i in range(len(SETTINGS))}
    for rep in range(REPS + 2):
        for i, st in enumerate(SETTINGS):
            try:
                old = {k: be.set_knob(k, v) for k, v in st.items()}
            except RuntimeError:  # a library variant without these knobs: its defaults only
                if i:
                    continue
                old = {}
            call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            call()
            e1.record()
            torch.cuda.synchronize()
            if rep >= 2:
                times[i].append(e0.elapsed_time(e1) * 1e3)
            for k, v in old.items():
                be.set_knob(k, v)
    for i, st in enumerate(SETTINGS):
        if not times[i]:
            continue
        t = sorted(times[i])[len(times[i]) // 2]
        print(f"{mode:5s} N={N:3d} {iters:2d} it {st}: {t:8.1f} us per call ({t / iters:6.1f} us/it)", flush=True)
