"""Debug: planes written by the first linearize vs torch recomputation, and
packed (2nd call) vs gathering (1st call) edge sums. usage: MODE=rays python tools/debug_planes.py"""
import ctypes, os, sys
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch
import mast3r_slam_backends as be
from mast3r_slam_amd import synthetic

mode = os.environ.get("MODE", "rays")
H, W, N = int(os.environ.get("H", 64)), int(os.environ.get("W", 64)), int(os.environ.get("N", 4))
dev = torch.device("cuda:0")
g = synthetic.make_graph(N, H, W, seed=5, device=dev)
mid = {"calib": be.MODE_CALIB, "rays": be.MODE_RAYS, "points": be.MODE_POINTS}[mode]
Xs = g.Xs.contiguous()
E, HW = g.n_edges, H * W
wst = torch.zeros(int(be._lib.m3s_gn_workspace_size(N, HW, E)), dtype=torch.uint8, device=dev)
a, keep = be.make_gn_args(mid, g.T_init.data.contiguous(), Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj,
                          g.valid_match, g.Q, g.K if mode == "calib" else None, sigma_a=0.003,
                          sigma_b=10.0, C_thresh=0.0, Q_thresh=1.5, height=H, width=W,
                          pixel_border=-10, z_eps=1e-6, max_iter=1, delta_thresh=0.0,
                          workspace=wst)
st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
lay = be.workspace_layout(N, HW, E)
es1 = torch.zeros(E, 36, dtype=torch.float64, device=dev)
es2 = torch.zeros_like(es1)
L = be._lib
assert L.m3s_gn_prepare(ctypes.byref(a), st) == 0
assert L.m3s_gn_linearize(ctypes.byref(a), 0, E, ctypes.c_void_p(es1.data_ptr()), st) == 0
torch.cuda.synchronize()
npl = {"points": 4, "rays": 5, "calib": 3}[mode]
nbytes = 4 * npl * E * HW
planes = wst[lay["planes"]:lay["planes"] + nbytes].clone().view(torch.float32).view(E, npl, HW).cpu()
assert L.m3s_gn_linearize(ctypes.byref(a), 0, E, ctypes.c_void_p(es2.data_ptr()), st) == 0
torch.cuda.synchronize()
print("edge-sum diff 2nd vs 1st per edge:", (es2 - es1).abs().amax(1).cpu().numpy())
# expected planes
ii, jj = g.ii.cpu(), g.jj.cpu()
u = torch.unique(torch.cat([ii, jj]))
ri = torch.searchsorted(u, ii); rj = torch.searchsorted(u, jj)
Xc, Cc = Xs.cpu(), g.Cs.cpu().reshape(N, HW)
idx, vm, Q = g.idx_ii2jj.cpu(), g.valid_match.cpu().reshape(E, HW), g.Q.cpu().reshape(E, HW)
for e in range(E):
    id_ = torch.where(vm[e], idx[e], torch.zeros_like(idx[e]))
    Xi = Xc[ri[e]][id_]
    ok = vm[e] & (Q[e] > 1.5) & (Cc[ri[e]][id_] > 0) & (Cc[rj[e]] > 0)
    if mode == "rays":
        ni = Xi.norm(dim=1)
        exp = torch.stack([Xi[:, 0] / ni, Xi[:, 1] / ni, Xi[:, 2] / ni, ni, torch.where(ok, Q[e].sqrt(), 0)])
    elif mode == "points":
        exp = torch.stack([Xi[:, 0], Xi[:, 1], Xi[:, 2], torch.where(ok, Q[e].sqrt(), 0)])
    else:
        exp = None
    if exp is not None:
        d = (planes[e] - exp).abs().amax(1)
        if d.max() > 1e-3:
            bad = ((planes[e] - exp).abs() > 1e-3).nonzero()[:5]
            print("edge", e, "plane maxdiff", d.numpy(), "first bad (plane,px):", bad.tolist(),
                  [(planes[e][p, k].item(), exp[p, k].item()) for p, k in bad.tolist()])
print("done")
