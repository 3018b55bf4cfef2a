"""Spread of refine_matches centres per 16x16 query tile on bench.py's
512x512 matching pair (GPU box): the LDS box a tile-staged kernel would need
per dilation. Prints percentiles of the centres' bounding box (w, h) and the
fraction of tiles whose box fits a budget."""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import matching, synthetic  # noqa: E402

dev = torch.device("cuda:0")
H = W = 512
m = synthetic.make_match_inputs(H, W, device=dev)
img, pts, p0 = matching.prep_for_iter_proj(m.X11, m.X21)
cfg = matching.MATCHING_CFG
p1 = be.iter_proj(img, pts, p0, cfg["max_iter"], cfg["lambda_init"], cfg["convergence_thresh"])[0].long()
cur = p1.clone()
T = 16
fin = be.refine_matches(m.D11, m.D21, p1, cfg["radius"], cfg["dilation_max"])[0]
for name, cur in (("p1", p1), ("refined", fin)):
  print(name)
  for d in range(cfg["dilation_max"], 0, -1):
      c = cur[0].view(H // T, T, W // T, T, 2).permute(0, 2, 1, 3, 4).reshape(-1, T * T, 2).float()
      w = (c[..., 0].amax(1) - c[..., 0].amin(1) + 1 + 6 * d)
      h = (c[..., 1].amax(1) - c[..., 1].amin(1) + 1 + 6 * d)
      area = (w * h)
      q = torch.tensor([0.1, 0.5, 0.9, 0.99], device=dev)
      print(f"d={d}: box w pct {w.quantile(q).tolist()} h pct {h.quantile(q).tolist()} "
            f"area<=2560 {float((area <= 2560).float().mean()):.3f} <=4096 {float((area <= 4096).float().mean()):.3f}",
            flush=True)
print("vis fraction", float(m.vis.float().mean()))
# p1 vs p_true
err = (p1[0] - m.p_true[0]).abs().amax(-1)
print("iter_proj |p1 - p_true| pct", err.float().quantile(torch.tensor([0.5, 0.9, 0.99], device=dev)).tolist())
