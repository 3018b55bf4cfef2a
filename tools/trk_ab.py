import os, sys
ROOT = "/root/repo" if os.path.exists("/root/repo") else os.getcwd()
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch
import bench
import mast3r_slam_backends as be
from mast3r_slam_amd import synthetic
dev = torch.device("cuda:0")
libs = sys.argv[1:]
for rnd in range(4):
    # rotate the order every round (no library always runs first)
    for p in libs[rnd % len(libs):] + libs[:rnd % len(libs)]:
        be._lib = be._load(os.path.abspath(p))
        r = bench.tracker_leg(be, synthetic, dev, 512, 512, reps=50)
        print(os.path.basename(p), r["gn_iters_per_s"], r["ms_per_solve"], flush=True)
