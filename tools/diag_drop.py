"""Bounded-wait diagnostic: drop one df dispatch item on the 140-KF dense-tail
graph and print the reported info per knob setting (gcomb 0 / 1)."""
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402
from test_gpu_backend import run_gpu  # noqa: E402

be._lib = be._load(os.environ["LIB"]) if os.environ.get("LIB") else be.load_test_library()
g = synthetic.make_graph(140, 12, 16, seed=37)
be.set_knob("dense_tail_min", 8)
for gc in (0, 1, 0, 1):
    for d in (0, 1, 5):
        be.set_knob("gcomb", gc)
        be.set_knob("debug_drop_item", d)
        t0 = time.time()
        T, dx, info = run_gpu(be, "rays", g, 1, 0.0)
        be.set_knob("debug_drop_item", -1)
        T2, dx2, info2 = run_gpu(be, "rays", g, 1, 0.0)
        print(f"gcomb={gc} drop={d}: info {info.tolist()} |dx| {abs(dx).max():.3e} {time.time()-t0:.2f}s; intact after: {info2.tolist()}", flush=True)
