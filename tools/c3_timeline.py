"""Launch timeline of the C3 drop-in call (GPU box, under rocprofv3).

  rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python tools/c3_timeline.py
  python tools/c3_timeline.py --analyze DIR/.../run_kernel_trace.csv

The first form runs bench.py's C3 call (calib, 32 KFs, 512x512, 10 GN
iterations) 8 times; the second prints, for the last call, every launch with
its start offset, duration and the idle gap before it, and the totals: kernel
time, gaps, and the call's span."""
import csv
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def run():
    sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
    import torch

    import mast3r_slam_backends as be
    from mast3r_slam_amd import synthetic

    dev = torch.device("cuda:0")
    H = W = 512
    g = synthetic.make_graph(32, H, W, seed=1003, device=dev)
    Xs = (g.Xs[..., 2:3] * synthetic.pixel_rays(H, W, g.K)[None]).contiguous()
    T0 = g.T_init.data.contiguous()
    Twc = T0.clone()
    info = torch.zeros(8, dtype=torch.int32, device=dev)
    Cs, ii, jj = g.Cs.contiguous(), g.ii.contiguous(), g.jj.contiguous()
    for _ in range(8):
        Twc.copy_(T0)
        be.gauss_newton_calib(Twc, Xs, Cs, g.K, ii, jj, g.idx_ii2jj, g.valid_match, g.Q, H, W, -10, 1e-6,
                              1.0, 10.0, 0.0, 1.5, 10, 0.0, info=info)
    torch.cuda.synchronize()


def between_calls(path, t_end, t_start):
    """Memory copies and HIP API calls of the gap between two calls (the
    traces next to the kernel trace, when recorded)."""
    d = os.path.dirname(path)
    ev = []
    for f in os.listdir(d):
        if f.endswith("memory_copy_trace.csv"):
            for r in csv.DictReader(open(os.path.join(d, f))):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")))
        if f.endswith("hip_api_trace.csv"):
            for r in csv.DictReader(open(os.path.join(d, f))):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api " + r.get("Function", "")))
        if f.endswith("kernel_trace.csv"):
            for r in csv.DictReader(open(os.path.join(d, f))):
                if "anonymous namespace" not in r["Kernel_Name"]:
                    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kern " + r["Kernel_Name"][:40]))
    for s, e, n in sorted(ev):
        if t_end - 1000 <= s <= t_start:
            print(f"    {(s - t_end) / 1e3:+9.1f} us  dur {(e - s) / 1e3:7.2f}  {n[:80]}")


def analyze(path):
    rows = list(csv.DictReader(open(path)))
    seq = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    ours = [(s, e, n.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0])
            for s, e, n in seq if "anonymous namespace" in n]
    # calls start at the gathering linearize launch (first GN iteration)
    starts = [i for i, (_, _, n) in enumerate(ours) if n.startswith(("linearize_kernel", "linearize_gather_kernel"))]
    b = starts[-1]
    call = ours[b:]
    print(f"between the last two calls: previous call ends, this call's first kernel at "
          f"{(ours[b][0] - ours[b - 1][1]) / 1e3:.1f} us")
    between_calls(path, ours[b - 1][1], ours[b][0])
    print("during the first linearize of the call:")
    between_calls(path, call[0][0], call[1][0] + 1)
    # the last call ends at its 10th solve launch
    t0 = call[0][0]
    busy = gaps = 0
    prev = None
    for s, e, n in call:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        gaps += max(gap, 0.0)
        busy += (e - s) / 1e3
        print(f"  +{(s - t0) / 1e3:8.1f} us  dur {(e - s) / 1e3:8.2f}  gap {gap:6.2f}  {n[:70]}")
        prev = e
    span = (call[-1][1] - t0) / 1e3
    print(f"launches {len(call)}  kernel {busy:.1f} us  gaps {gaps:.1f} us  span {span:.1f} us")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run()
