"""Per-step wall-clock stamps of tail_llt_kernel (variant library built with
-DM3S_TAIL_STAMPS, tools/mkvar.sh): one stepwise GN iteration of a rays graph
of N keyframes, then the stamps read from the workspace (100 MHz clock)."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402
from mast3r_slam_amd.distributed import HipOps  # noqa: E402

N = int(os.environ.get("N", "256"))
dev = torch.device("cuda:0")
g = synthetic.make_graph(N, 64, 64, seed=1003, device=dev)
Twc = g.T_init.data.clone().contiguous()
E = g.n_edges
ops = HipOps(be.MODE_RAYS, Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q, E, None,
             sigma_a=0.003, sigma_b=10.0, C_thresh=0.0, Q_thresh=1.5)
es = torch.zeros(E, 36, dtype=torch.float64, device=dev)
lay = be.workspace_layout(N, 64 * 64, E)
for rep in range(3):
    ops.prepare(0.0)
    ops.linearize(0, E, es)
    ops.solve(es)
    torch.cuda.synchronize()
TMAX = 32
off = lay["tail"] + 8 * (512 * 512 + TMAX * (TMAX + 1) // 2 * 256 + TMAX * 256)
st = ops.ws[off:off + 8 * 128].view(torch.int64).cpu().numpy()
p = be.sparse_plan(N, *np.unique(np.concatenate([g.ii.cpu().numpy(), g.jj.cpu().numpy()]),
                                 return_inverse=True)[1].reshape(2, -1))
n = 7 * p["nc"]
TC = (n + 15) // 16
t0 = st[0]
print(f"N={N} nc={p['nc']} n={n} TC={TC}; us from kernel start (update done / diag done / step done):")
for k in range(TC):
    a, b, c = (st[1 + 3 * k:4 + 3 * k] - t0) / 100.0
    print(f"  k={k:2d}  {a:8.2f} {b:8.2f} {c:8.2f}")
print(f"  back-substitution done {(st[100] - t0) / 100.0:.2f} us")
