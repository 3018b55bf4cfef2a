"""Bitwise A/B of two library builds on the same solves (GPU box).

  python tools/ab_bitwise.py variants/lib_OLD.so      # vs the in-tree library

Each library runs in its own process (M3S_LIB) on identical seeded graphs:
C3-shaped calib (32 KFs), a small rays graph, and the chip-wide path (140 KFs
with a dense tail), a few GN iterations each; poses, dx and info are compared
bit for bit and the solve time of each is printed (HIP events, median)."""
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))

CASES = [("calib", 32, 128, 128, 10, 16), ("rays", 12, 48, 64, 5, 16), ("rays", 140, 24, 32, 3, 8),
         ("rays", 256, 12, 16, 3, 16)]


def child(out_path):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
    import numpy as np
    import torch

    import mast3r_slam_backends as be
    from mast3r_slam_amd import synthetic

    dev = torch.device("cuda:0")
    res = {}
    for mode, N, H, W, iters, tail in CASES:
        be.set_knob("dense_tail_min", tail)
        g = synthetic.make_graph(N, H, W, seed=4242 + N, device=dev)
        Xs = (g.Xs[..., 2:3] * synthetic.pixel_rays(H, W, g.K)[None]).contiguous() if mode == "calib" else g.Xs
        times = []
        for rep in range(5):
            Twc = g.T_init.data.clone().contiguous()
            info = torch.zeros(8, dtype=torch.int32, device=dev)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if mode == "calib":
                (dx,) = be.gauss_newton_calib(Twc, Xs, g.Cs, g.K, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q, H, W,
                                              -10, 1e-6, 1.0, 10.0, 0.0, 1.5, iters, 0.0, info=info)
            else:
                (dx,) = be.gauss_newton_rays(Twc, Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q, 0.003,
                                             10.0, 0.0, 1.5, iters, 0.0, info=info)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        key = f"{mode}_{N}"
        res[key + "_T"] = Twc.cpu().numpy()
        res[key + "_dx"] = dx.cpu().numpy()
        res[key + "_info"] = info.cpu().numpy()
        res[key + "_ms"] = np.array(sorted(times)[2])
    np.savez(out_path, **res)


def main():
    import numpy as np

    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    variant = os.path.abspath(sys.argv[1])
    outs = []
    for tag, lib in (("tree", None), ("variant", variant)):
        env = dict(os.environ)
        if lib:
            env["M3S_LIB"] = lib
        path = os.path.join(ROOT, "gpurun_out", f"ab_{tag}.npz")
        os.makedirs(os.path.dirname(path), exist_ok=True)
        subprocess.run([sys.executable, __file__, "--child", path], check=True, env=env, timeout=600)
        outs.append(np.load(path))
    a, b = outs
    ok = True
    for mode, N, *_ in CASES:
        key = f"{mode}_{N}"
        same = all(np.array_equal(a[key + s], b[key + s]) for s in ("_T", "_dx", "_info"))
        ok &= same
        print(f"{key:10s} bitwise {'EQUAL' if same else 'DIFFERENT'}  max|dT| {np.abs(a[key + '_T'] - b[key + '_T']).max():.3e}"
              f"  call ms: tree {float(a[key + '_ms']):.4f} variant {float(b[key + '_ms']):.4f}  "
              f"fails {a[key + '_info'][1]}/{b[key + '_info'][1]}")
    print("ALL EQUAL" if ok else "SOME DIFFERENT")


if __name__ == "__main__":
    main()
