"""Debug driver: gauss_newton_rays through the persistent dense LLT
(M3S_SOLVER=pdense) at a few graph sizes; prints info and timing."""
import os
import sys
import time

sys.path[:0] = ['.', 'mast3r-slam-ysh_amd']
os.environ["M3S_SOLVER"] = "pdense"
import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402

DEV = torch.device("cuda:0")
for N in [int(x) for x in os.environ.get("NS", "2,6,33").split(",")]:
    g = synthetic.make_graph(N, 24, 32, seed=190 + N)
    Twc = g.T_init.data.clone().to(DEV)
    info = torch.zeros(8, dtype=torch.int32, device=DEV)
    d = [t.to(DEV).contiguous() for t in (g.Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q)]
    t0 = time.time()
    be.gauss_newton_rays(Twc, *d, 0.003, 10.0, 0.0, 1.5, int(os.environ.get("ITERS", "3")), 0.0, info=info)
    torch.cuda.synchronize()
    print("N", N, "info", info.cpu().tolist(), "%.3f s" % (time.time() - t0), flush=True)
