"""refine_matches / iter_proj timing on bench.py's 512x512 matching pair
(GPU box): python tools/refine_time.py  (M3S_REFINE_STAGED=0: global kernel)."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402

print(os.environ.get("M3S_REFINE_STAGED", "1"), bench.matching_leg(be, synthetic, torch.device("cuda:0"), 512, 512))
