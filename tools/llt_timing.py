"""Phase timing of sparse_llt_kernel (lib built with -DM3S_LLT_TIMING=1):
assembly / factorisation / back-substitution / retraction, in microseconds."""
import ctypes, os, sys
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch
import mast3r_slam_backends as be
from mast3r_slam_amd import synthetic
dev = torch.device("cuda:0")
for N in [int(x) for x in os.environ.get("NS", "32,64,128").split(",")]:
    H = W = 64
    g = synthetic.make_graph(N, H, W, seed=1003, device=dev)
    E, HW = g.n_edges, H * W
    wst = torch.zeros(int(be._lib.m3s_gn_workspace_size(N, HW, E)), dtype=torch.uint8, device=dev)
    Twc = g.T_init.data.contiguous()
    a, keep = be.make_gn_args(be.MODE_RAYS, Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match,
                              g.Q, None, sigma_a=0.003, sigma_b=10.0, C_thresh=0.0, Q_thresh=1.5,
                              max_iter=1, delta_thresh=0.0, workspace=wst)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    lay = be.workspace_layout(N, HW, E)
    res = []
    for rep in range(6):
        assert be._lib.m3s_gauss_newton_rays(ctypes.byref(a), st) == 0
        torch.cuda.synchronize()
        ts = wst[lay["flags"] + 64: lay["flags"] + 64 + 64].clone().view(torch.int64).cpu().tolist()
        us = lambda a, b: (ts[b] - ts[a]) / 100.0
        # stamps: 0 start, 1 assembled, 5 items done, 6 tail border, 7 tail factor, 2 factor+tail, 3 backsub, 4 end
        tail = [us(1, 5), us(5, 6), us(6, 7), us(7, 2)] if ts[7] > ts[6] > ts[5] > 0 else None
        res.append([us(0, 1), us(1, 2), us(2, 3), us(3, 4), tail])
        for i in (5, 6, 7):
            wst[lay["flags"] + 64 + 8 * i: lay["flags"] + 72 + 8 * i] = 0
    r = res[-1]
    plan = be.sparse_plan(N, *[torch.searchsorted(torch.unique(torch.cat([g.ii, g.jj])), t).cpu().numpy() for t in (g.ii, g.jj)])
    import numpy as np
    m = N - 1
    if os.environ.get("CYC") == "1":
        d = wst[lay["A"]: lay["A"] + 8 * 48].clone().view(torch.int64).cpu().numpy().reshape(16, 3)
        print("  per-wave factor cycles: total %.0f, waiting %.0f (%.0f%%), update products %.0f (%.0f%%)"
              % (d[:, 0].mean(), d[:, 1].mean(), 100 * d[:, 1].mean() / d[:, 0].mean(),
                 d[:, 2].mean(), 100 * d[:, 2].mean() / d[:, 0].mean()))
        S_ = plan["S"]
        it_ = wst[lay["A"] + 8 * 64: lay["A"] + 8 * (64 + S_)].clone().view(torch.int64).cpu().numpy()
        dur, nt = it_ & ((1 << 40) - 1), it_ >> 40
        for name, sel in (("DIAG", slice(0, m)), ("OFF", slice(m, S_))):
            dd, nn = dur[sel], nt[sel]
            for lo, hi in ((0, 1), (1, 3), (3, 8), (8, 100)):
                mk = (nn >= lo) & (nn < hi)
                if mk.any():
                    print(f"    {name} items with {lo}-{hi - 1} updates: n={mk.sum()} mean {dd[mk].mean():.0f} cycles")
    print(f"N={N} levels={plan['levels']} S={plan['S']}: assembly {r[0]:.1f} us, factor {r[1]:.1f} us, "
          f"backsub {r[2]:.1f} us, retract {r[3]:.1f} us")
    if r[4] and os.environ.get("BT") == "1":
        bt = wst[lay["A"]: lay["A"] + 48].clone().view(torch.int64).cpu().tolist()
        print("    wave 0 tail cycles: diag %d, barrier %d, off %d, barrier %d, trailing %d, barrier %d" % tuple(bt))
    if r[4]:
        print(f"    dense tail {plan['nc']} columns: items {r[4][0]:.1f} us, border {r[4][1]:.1f} us, "
              f"tail factor {r[4][2]:.1f} us, tail backsub {r[4][3]:.1f} us")
