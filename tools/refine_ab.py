"""Interleaved A/B of refine_matches builds on bench.py's 512x512 matching
pair (GPU box). Each argument is a shared library exporting
m3s_refine_matches (tools/mkmatch.sh builds match-only variants); the product
library's result is the reference: every variant must equal it bitwise.
python tools/refine_ab.py variants/match_A.so variants/match_B.so ..."""
import ctypes
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import matching, synthetic  # noqa: E402

dev = torch.device("cuda:0")
H = W = 512
m = synthetic.make_match_inputs(H, W, device=dev)
img, pts, p0 = matching.prep_for_iter_proj(m.X11, m.X21)
cfg = matching.MATCHING_CFG
p1 = be.iter_proj(img, pts, p0, cfg["max_iter"], cfg["lambda_init"], cfg["convergence_thresh"])[0].long()
ref = be.refine_matches(m.D11, m.D21, p1, cfg["radius"], cfg["dilation_max"])[0]
torch.cuda.synchronize()
libs = [("product", be._lib)] + [(os.path.basename(p), ctypes.CDLL(os.path.abspath(p))) for p in sys.argv[1:]]
B, N, F = 1, H * W, m.D11.shape[-1]
stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def call(lib, out):
    a = be.RefineArgs()
    a.D11, a.D21, a.p1 = m.D11.data_ptr(), m.D21.data_ptr(), p1.data_ptr()
    a.B, a.H, a.W, a.N, a.F = B, H, W, N, F
    a.dtype, a.radius, a.dilation_max = 0, cfg["radius"], cfg["dilation_max"]
    a.p1_new = out.data_ptr()
    rc = lib.m3s_refine_matches(ctypes.byref(a), stream)
    assert rc == 0, rc


outs = {}
for name, lib in libs:
    out = torch.zeros_like(ref)
    call(lib, out)
    torch.cuda.synchronize()
    outs[name] = out
    moved = int((out != p1).any(-1).sum())
    print(f"{name}: bitwise equal to product: {bool(torch.equal(out, ref))} (moved {moved} of {N})", flush=True)
reps, rounds = 20, 7
times = {name: [] for name, _ in libs}
for r in range(rounds):
    for name, lib in libs:
        out = outs[name]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        call(lib, out)
        e0.record()
        for _ in range(reps):
            call(lib, out)
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / reps * 1e3)
for name, t in times.items():
    t = sorted(t)
    print(f"{name}: median {t[len(t) // 2]:.1f} us  min {t[0]:.1f}  max {t[-1]:.1f}  (us per 512x512 call, F={F})")
