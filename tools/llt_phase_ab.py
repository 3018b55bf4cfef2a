"""Phase timing of the one-workgroup sparse LLT at C3 by early-exit builds:
tools/mkvar.sh x1 -DM3S_LLT_EXIT=1 (after assembly), x2 -DM3S_LLT_EXIT=2
(after the factor dataflow); the full library times the whole kernel. Each
library runs the C3 drop-in call (bench.py's graph, 10 GN iterations) with HIP
events; the per-iteration difference between two builds is the phase's time.

usage: python tools/llt_phase_ab.py lib_full.so variants/lib_x1.so variants/lib_x2.so"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402

dev = torch.device("cuda:0")
H = W = 512
g = synthetic.make_graph(32, H, W, seed=1003, device=dev)
rays = synthetic.pixel_rays(H, W, g.K)
Xs = (g.Xs[..., 2:3] * rays[None]).contiguous()
T0 = g.T_init.data.contiguous()
Twc = T0.clone()
info = torch.zeros(8, dtype=torch.int32, device=dev)


def call():
    Twc.copy_(T0)
    be.gauss_newton_calib(Twc, Xs, g.Cs.contiguous(), g.K, g.ii.contiguous(), g.jj.contiguous(), g.idx_ii2jj,
                          g.valid_match, g.Q, H, W, -10, 1e-6, 1.0, 10.0, 0.0, 1.5, 10, 0.0, info=info)


res = {p: [] for p in sys.argv[1:]}
for rnd in range(3):
    for p in sys.argv[1:]:
        be._lib = be._load(os.path.abspath(p))
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            call()
        e.record()
        torch.cuda.synchronize()
        res[p].append(s.elapsed_time(e) / 10)
for p, v in res.items():
    print(f"{os.path.basename(p)}: {sorted(v)[1] * 1e3:8.1f} us per call (median of 3 rounds)")
