"""Interleaved A/B of whole GN calls (the drop-in entry point) across library
builds in ONE process (cdna_hip_programming.md §5.4 rule 24): every library
gets its own ctypes handle, workspace, poses and info; rounds alternate the
libraries so box-level drift hits all of them alike. Prints the median call
time per library per case and whether the final poses / dx / info are bitwise
equal to the first library's.

usage: python tools/ab_calls.py variants/lib_A.so variants/lib_B.so ...
  AB_CASES="calib:32:128:128:10:16,rays:140:24:32:3:8"  (mode:N:H:W:iters:dense_tail_min[:seed])
  (seed defaults to 4242 + N; bench.py's C3 graph is seed 1003)
"""
import ctypes
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]

import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402

DEFAULT = "calib:32:128:128:10:16,calib:32:512:512:10:16,rays:140:24:32:3:8,rays:256:12:16:3:16"


def main():
    libs = sys.argv[1:]
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    handles = []
    for p in libs:
        L = ctypes.CDLL(os.path.abspath(p))
        L.m3s_gn_workspace_size.restype = ctypes.c_size_t
        L.m3s_gn_workspace_size.argtypes = [ctypes.c_int64] * 3
        for f in ("m3s_gauss_newton_calib", "m3s_gauss_newton_rays", "m3s_gn_release"):
            getattr(L, f).argtypes = [ctypes.POINTER(be.GnArgs), ctypes.c_void_p]
        L.m3s_set_knob.argtypes = [ctypes.c_char_p, ctypes.c_int]
        handles.append(L)
    rounds = int(os.environ.get("AB_ROUNDS", "7"))
    for case in os.environ.get("AB_CASES", DEFAULT).split(","):
        mode, N, H, W, iters, tail, *sd = case.split(":")
        N, H, W, iters, tail = int(N), int(H), int(W), int(iters), int(tail)
        g = synthetic.make_graph(N, H, W, seed=int(sd[0]) if sd else 4242 + N, device=dev)
        calib = mode == "calib"
        Xs = (g.Xs[..., 2:3] * synthetic.pixel_rays(H, W, g.K)[None]).contiguous() if calib else g.Xs.contiguous()
        mid = be.MODE_CALIB if calib else be.MODE_RAYS
        sig = (1.0, 10.0) if calib else (0.003, 10.0)
        per = []
        for L in handles:
            L.m3s_set_knob(b"dense_tail_min", tail)
            Twc = g.T_init.data.clone().contiguous()
            info = torch.zeros(8, dtype=torch.int32, device=dev)
            dx = torch.zeros(N - 1, 7, dtype=torch.float32, device=dev)
            nb = L.m3s_gn_workspace_size(N, H * W, g.n_edges)
            ws = torch.empty(nb + 256, dtype=torch.uint8, device=dev)
            a, keep = be.make_gn_args(mid, Twc, Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q,
                                      g.K if calib else None, sigma_a=sig[0], sigma_b=sig[1], C_thresh=0.0,
                                      Q_thresh=1.5, height=H, width=W, pixel_border=-10, z_eps=1e-6,
                                      max_iter=iters, delta_thresh=0.0, dx=dx, info=info, workspace=ws)
            per.append(dict(a=a, keep=keep, Twc=Twc, info=info, dx=dx, t=[]))
        fn = "m3s_gauss_newton_calib" if calib else "m3s_gauss_newton_rays"
        pairs = list(zip(handles, per))
        for r in range(rounds + 1):
            # rotate the order every round (no library always runs first)
            for L, d in pairs[r % len(pairs):] + pairs[:r % len(pairs)]:
                d["Twc"].copy_(g.T_init.data)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                rc = getattr(L, fn)(ctypes.byref(d["a"]), sp)
                e.record()
                L.m3s_gn_release(ctypes.byref(d["a"]), sp)
                torch.cuda.synchronize()
                assert rc == 0, rc
                if r:  # round 0 warms the plan cache
                    d["t"].append(s.elapsed_time(e))
        ref = per[0]
        for p, d in zip(libs, per):
            same = (torch.equal(d["Twc"], ref["Twc"]) and torch.equal(d["dx"], ref["dx"])
                    and torch.equal(d["info"], ref["info"]))
            t = sorted(d["t"])
            print(f"{mode}_{N}_{H}x{W} {os.path.basename(p):24s} median {t[len(t) // 2]:.4f} ms  min {t[0]:.4f}"
                  f"  {'bitwise EQUAL' if same else 'DIFFERENT max|dT| %.3e' % (d['Twc'] - ref['Twc']).abs().max().item()}"
                  f"  fails {int(d['info'][1])}")


if __name__ == "__main__":
    main()
