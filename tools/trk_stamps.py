"""Phase timing of the persistent tracker (library built with
-DM3S_TRK_STAMPS, e.g. tools/mkvar.sh trkst -DM3S_TRK_STAMPS): runs the C2
tracker solve a few times and prints, per iteration, the phases of workgroups
0 and G-1 in us: compute | block reduce + partial store | arrival (+ level-1 sum on a shard reducer) | top reducer:
partial sums, else: poll | reducer: solve + publish, else: record read |
(next iteration start).

usage: python tools/trk_stamps.py variants/lib_trkst.so"""
import ctypes
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402

lib = ctypes.CDLL(os.path.abspath(sys.argv[1]))
be._lib = be._load(os.path.abspath(sys.argv[1]))  # the wrapper runs the stamped build
lib = be._lib
dev = torch.device("cuda:0")
p = synthetic.make_pair(512, 512, seed=1002, device=dev)
a = (p.Xf.contiguous(), p.Xk.contiguous(), p.T_WCf_init.data.contiguous(), p.T_WCk.data.contiguous(),
     p.Qk.contiguous(), p.valid.contiguous())
for _ in range(5):
    be.track_rays_sim3(*a, 0.003, 10.0, 1.345, 10, 0.0, 0.0, sync_every=0)
torch.cuda.synchronize()
st = np.zeros((2, 16, 8), np.int64)
assert lib.m3s_debug_stamps(0, st.ctypes.data_as(ctypes.c_void_p)) == 1
t0 = st[0, 0, 0]
for w in range(2):
    print("workgroup", "0" if w == 0 else "G-1")
    for it in range(10):
        r = st[w, it]
        nxt = st[w, it + 1, 0] if it < 9 else r[5]
        ph = [(r[k + 1] - r[k]) * 0.01 for k in range(5)] + [(nxt - r[5]) * 0.01]
        upd = f"   (update {(r[6] - r[4]) * 0.01:5.2f})" if w == 0 else ""
        print(f"  it {it}: start {(r[0] - t0) * 0.01:7.2f} us  " + "  ".join(f"{x:5.2f}" for x in ph) + upd)
