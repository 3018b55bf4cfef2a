"""A/B timing of linearize-kernel library variants in ONE process, interleaved
rounds (cdna_hip_programming.md §5.4 rule 24). Each variant .so is loaded with
its own ctypes handle; all run the same C3 workload (calib, 32 KF, 512x512).

usage: python tools/ab_linearize.py variants/lib_A.so variants/lib_B.so ...
"""
import ctypes
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]

import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402


def main():
    libs = sys.argv[1:]
    dev = torch.device("cuda:0")
    H = W = int(os.environ.get("AB_HW", "512"))
    N = int(os.environ.get("AB_N", "32"))
    mode = os.environ.get("AB_MODE", "calib")
    g = synthetic.make_graph(N, H, W, seed=1003, device=dev)
    rays = synthetic.pixel_rays(H, W, g.K)
    Xs = (g.Xs[..., 2:3] * rays[None]).contiguous() if mode == "calib" else g.Xs.contiguous()
    Twc = g.T_init.data.contiguous()
    mid = {"calib": be.MODE_CALIB, "rays": be.MODE_RAYS, "points": be.MODE_POINTS}[mode]
    sig = {"calib": (1.0, 10.0), "rays": (0.003, 10.0), "points": (0.05, 0.0)}[mode]
    a, keep = be.make_gn_args(mid, Twc, Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q,
                              g.K if mode == "calib" else None, sigma_a=sig[0], sigma_b=sig[1],
                              C_thresh=0.0, Q_thresh=1.5, height=H, width=W, pixel_border=-10,
                              z_eps=1e-6, max_iter=1, delta_thresh=0.0)
    E = g.n_edges
    wkeep = {}
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    handles, wargs = [], []
    for p in libs:
        L = ctypes.CDLL(os.path.abspath(p))
        L.m3s_gn_workspace_size.restype = ctypes.c_size_t
        L.m3s_gn_workspace_size.argtypes = [ctypes.c_int64] * 3
        nb = L.m3s_gn_workspace_size(N, H * W, E)
        ws = torch.empty(nb + 256, dtype=torch.uint8, device=dev)
        aa = be.GnArgs.from_buffer_copy(a)
        aa.workspace, aa.workspace_bytes = ws.data_ptr(), nb
        wkeep[p] = ws
        wargs.append(aa)
        L.m3s_gn_prepare.argtypes = [ctypes.POINTER(be.GnArgs), ctypes.c_void_p]
        L.m3s_gn_linearize.argtypes = [ctypes.POINTER(be.GnArgs), ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_void_p, ctypes.c_void_p]
        handles.append(L)
    # correctness: edge sums of each variant vs the first
    ref = None
    for p, L, aa in zip(libs, handles, wargs):
        es = torch.zeros(E, 36, dtype=torch.float64, device=dev)
        es2 = torch.zeros(E, 36, dtype=torch.float64, device=dev)
        assert L.m3s_gn_prepare(ctypes.byref(aa), st) == 0
        assert L.m3s_gn_linearize(ctypes.byref(aa), 0, E, ctypes.c_void_p(es.data_ptr()), st) == 0
        assert L.m3s_gn_linearize(ctypes.byref(aa), 0, E, ctypes.c_void_p(es2.data_ptr()), st) == 0
        torch.cuda.synchronize()
        if ref is None:
            ref, ref2 = es.clone(), es2.clone()
        err = ((es - ref).abs().max() / ref.abs().max()).item()
        # packed (2nd) call: L and l only (entry 35, the cost, is not summed there)
        err2 = ((es2[:, :35] - ref2[:, :35]).abs().max() / ref2[:, :35].abs().max()).item()
        d12 = ((es2[:, :35] - es[:, :35]).abs().max() / es[:, :35].abs().max()).item()
        print(f"{os.path.basename(p)}: max rel diff vs first: gathering call {err:.2e}, packed call {err2:.2e};"
              f" packed vs gathering call {d12:.2e}")
    reps, rounds = 20, int(os.environ.get("AB_ROUNDS", "5"))
    times = {p: [] for p in libs}
    first = {p: [] for p in libs}
    trio = list(zip(libs, handles, wargs))
    for rnd in range(rounds):
        # the list order rotates every round: the first-listed library read
        # ~2-3 % slow when it always ran first (profiles/r05/ab_pkw_order*.txt)
        for p, L, aa in trio[rnd % len(trio):] + trio[:rnd % len(trio)]:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            assert L.m3s_gn_prepare(ctypes.byref(aa), st) == 0
            s.record()
            L.m3s_gn_linearize(ctypes.byref(aa), 0, E, None, st)
            e.record()
            torch.cuda.synchronize()
            first[p].append(s.elapsed_time(e))
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            L.m3s_gn_linearize(ctypes.byref(aa), 0, E, None, st)
            s.record()
            for _ in range(reps):
                L.m3s_gn_linearize(ctypes.byref(aa), 0, E, None, st)
            e.record()
            torch.cuda.synchronize()
            times[p].append(s.elapsed_time(e) / reps)
    HW = H * W
    bytes_alg = HW * (13 * E + 16 * N)
    for p in libs:
        t = sorted(times[p])
        f = sorted(first[p])
        print(f"{os.path.basename(p)}: median {t[len(t)//2]*1e3:.1f} us  min {t[0]*1e3:.1f} us  "
              f"-> {bytes_alg / (t[len(t)//2] * 1e-3) / 1e9:.0f} GB/s algorithmic; "
              f"first call after prepare {f[len(f)//2]*1e3:.1f} us")


if __name__ == "__main__":
    main()
