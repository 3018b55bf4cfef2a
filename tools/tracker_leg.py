"""bench.py's tracker leg alone (configs[1]: 512x512 frame->keyframe GN,
10 fixed iterations), for rocprofv3 kernel traces of the tracker path."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402

dev = torch.device("cuda:0")
print(bench.tracker_leg(be, synthetic, dev, 512, 512, reps=int(os.environ.get("REPS", "50"))), flush=True)
