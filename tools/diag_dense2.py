"""Dense-fallback 2-iteration diagnostic: is the 2-iteration call's result the
1-iteration call applied twice? (complete 201-KF graph, rays)"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402
from test_gpu_backend import run_gpu  # noqa: E402

N = 201
ii_u = [i for j in range(N) for i in range(j)]
jj_u = [j for j in range(N) for i in range(j)]
g = synthetic.make_graph(N, 8, 12, seed=45, edges=(ii_u, jj_u))
T1a, dx1a, _ = run_gpu(be, "rays", g, 1, 0.0)
T1b, dx1b, _ = run_gpu(be, "rays", g, 1, 0.0)
print("1-it run to run: max|dT| %.3e max|ddx| %.3e" % (np.abs(T1a - T1b).max(), np.abs(dx1a - dx1b).max()))
T2, dx2, info = run_gpu(be, "rays", g, 2, 0.0)
T2s, dx2s, _ = run_gpu(be, "rays", g, 1, 0.0, Twc0=T1a)
print("2-it call vs two 1-it calls: max|dT2| %.3e max|ddx2| %.3e; max|dx2| %.3e max|dx1| %.3e info %s" % (
    np.abs(T2 - T2s).max(), np.abs(dx2 - dx2s).max(), np.abs(dx2).max(), np.abs(dx1a).max(), info.tolist()))
T3, dx3, _ = run_gpu(be, "rays", g, 2, 0.0)
print("2-it run to run: max|dT| %.3e" % np.abs(T2 - T3).max())
