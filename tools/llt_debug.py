import ctypes, os, sys
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch
import mast3r_slam_backends as be
from mast3r_slam_amd import synthetic
dev = torch.device("cuda:0")
N = int(os.environ.get("N", 4))
g = synthetic.make_graph(N, 16, 16, seed=3, device=dev)
Twc = g.T_init.data.contiguous()
info = torch.zeros(8, dtype=torch.int32, device=dev)
print("calling", flush=True)
be.gauss_newton_rays(Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q, 0.003, 10.0, 0.0, 1.5, 1, 0.0, info=info)
torch.cuda.synchronize()
print("info", info.tolist(), flush=True)
