"""refine_matches / iter_proj timing on bench.py's 512x512 matching pair
(GPU box): python tools/refine_time.py (round 4 timed its kernel variants
with it: profiles/r04/refine_variants.txt, the label is the variant)."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402

print(bench.matching_leg(be, synthetic, torch.device("cuda:0"), 512, 512))
