"""Per-column timing of the large-graph solve (library built with
-DM3S_COL_STAMPS [-DM3S_TAIL_STAMPS], tools/mkvar.sh): one stepwise GN
iteration of an N-keyframe rays graph (64x64 pixels: the solve does not depend
on the image size), then per elimination-tree level of the sparse columns the
spread of (ticket -> dependencies ready -> DIAG done -> column published) in
us from the first column's ticket, and the back-substitution likewise.

usage: N=256 python tools/col_stamps.py variants/lib_colst.so"""
import os
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402

be._lib = be._load(os.path.abspath(sys.argv[1]))
from mast3r_slam_amd import synthetic  # noqa: E402
from mast3r_slam_amd.distributed import HipOps  # noqa: E402

N = int(os.environ.get("N", "256"))
dev = torch.device("cuda:0")
g = synthetic.make_graph(N, 64, 64, seed=1003, device=dev)
Twc = g.T_init.data.clone().contiguous()
E = g.n_edges
ops = HipOps(be.MODE_RAYS, Twc, g.Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj, g.valid_match, g.Q, E, None,
             sigma_a=0.003, sigma_b=10.0, C_thresh=0.0, Q_thresh=1.5)
es = torch.zeros(E, 36, dtype=torch.float64, device=dev)
for rep in range(3):
    ops.prepare(0.0)
    ops.linearize(0, E, es)
    torch.cuda.synchronize()
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    ops.solve(es)
    s1.record()
    torch.cuda.synchronize()
print(f"N={N}: solve {s0.elapsed_time(s1) * 1e3:.1f} us (HIP events, last rep)")
st = np.zeros((4, 2048, 4), np.int64)
assert be._lib.m3s_debug_stamps(1, st.ctypes.data_as(__import__("ctypes").c_void_p)) == 1
ri = np.unique(np.concatenate([g.ii.cpu().numpy(), g.jj.cpu().numpy()]), return_inverse=True)[1].reshape(2, -1)
p = be.sparse_plan(N, ri[0], ri[1], split=32)
m, nc = p["m"], p["nc"]
c0 = m - nc
cols = np.arange(c0)
parent = np.full(m, -1)
for k in range(m):
    rows = p["col_row"][p["col_ptr"][k]:p["col_ptr"][k + 1]]
    if len(rows):
        parent[k] = rows.min()
lev = np.zeros(m, int)
for k in range(m):
    if parent[k] >= 0:
        lev[parent[k]] = max(lev[parent[k]], lev[k] + 1)
F = st[0, :c0]
t0 = F[:, 0].min()
O = st[3]  # OFF items by destination slot: ticket, updates ready, DIAG(k) ready, published
tdst = p["task_dst"]
tcol = p["task_col"]
us = lambda x: (x - t0) / 100.0  # noqa: E731
print(f"sparse columns {c0}, tail columns {nc}; factor: first ticket -> last publish {us(F[:, 3].max()):.1f} us")
print("level  cols   ticket(min/max)   ready(max)   diag(max)   publish(min/max)   per-column ready->publish (mean)"
      "   OFF: publish(max)  DIAG->OFF published (mean/max)")
for L in range(lev[:c0].max() + 1):
    ks = cols[lev[:c0] == L]
    if not len(ks):
        continue
    f = F[ks]
    print(f"{L:5d} {len(ks):5d}   {us(f[:, 0].min()):7.1f}/{us(f[:, 0].max()):7.1f}   {us(f[:, 1].max()):9.1f}"
          f"   {us(f[:, 2].max()):9.1f}   {us(f[:, 3].min()):7.1f}/{us(f[:, 3].max()):7.1f}"
          f"   {((f[:, 3] - f[:, 1]) / 100.0).mean():8.2f}", end="")
    offs = [t for t in range(len(tdst)) if tcol[t] in set(ks.tolist())]
    if offs:
        op = np.array([O[tdst[t], 3] for t in offs])
        gap = np.array([(O[tdst[t], 3] - F[tcol[t], 3]) / 100.0 for t in offs])
        print(f"   {us(op.max()):9.1f}   {gap.mean():6.2f}/{gap.max():6.2f}")
    else:
        print()
B = st[1, :c0]
tb = B[:, 0].min()
print(f"back-substitution: first ticket -> last x {((B[:, 2].max() - tb) / 100.0):.1f} us; per column ready->done "
      f"mean {((B[:, 2] - B[:, 1]) / 100.0).mean():.2f} us; wait (ticket->ready) max {((B[:, 1] - B[:, 0]) / 100.0).max():.1f} us")
T = st[2]
TC = (7 * nc + 15) // 16
if TC:
    tt0 = T[0, 1]
    print(f"dense tail over {TC} workgroups (us from workgroup 0's updates done): column: updates done / "
          f"diag done / first tile published early / published")
    for J in range(TC):
        a, b, c = ((T[J, 1:4] - tt0) / 100.0)
        e = (T[J, 0] - tt0) / 100.0 if J + 1 < TC else float("nan")
        dg = (T[J, 2] - T[600 + J, 0]) / 100.0 if T[600 + J, 0] else float("nan")
        print(f"  J={J:2d} {a:8.2f} {b:8.2f} {e:8.2f} {c:8.2f}   (diagonal factor alone {dg:5.2f})")
    if T[800, 1]:
        print("  pair kernel, wave 1 per pair (J0): deferred update done / W_J0 seen / J0 panels stored / "
              "J1 updates done / W_J1 seen")
        for J0 in range(0, TC - 1, 2):
            v = [(T[800 + J0, i] - tt0) / 100.0 for i in range(4)] + [(T[900 + J0, 0] - tt0) / 100.0]
            print(f"  J0={J0:2d} " + " ".join(f"{x:8.2f}" for x in v))
    if T[1000 + 15, 1]:
        print("  pair kernel, waves 1..3: k-loop done / each row done (us)")
        for J0 in range(0, min(TC - 1, 8), 2):
            for w in (1, 2, 3):
                row = [T[1000 + 16 * J0 + 15, w]] + [T[1000 + 16 * J0 + u, w] for u in range(11)]
                print(f"  J0={J0:2d} w{w} " + " ".join(f"{(x - tt0) / 100.0:7.2f}" for x in row if x))
    if T[1300, 1]:
        print("  pair kernel, wave 1 rows: (row start, J0 tile stored, J1 tile stored) us")
        for J0 in range(0, min(TC - 1, 6), 2):
            cells = []
            for u in range(8):
                r = T[1300 + 16 * J0 + u]
                if r[0]:
                    cells.append("(" + ",".join(f"{(r[i] - tt0) / 100.0:.2f}" for i in (0, 1, 3)) + ")")
            print(f"  J0={J0:2d} " + " ".join(cells))
    print(f"  back-substitution done {(T[511, 0] - tt0) / 100.0:.2f} us")
    if B[:, 3].max() > 0:  # gcol_worker (knob gcomb): X_k recursion during the tail, then x_k = a_k + B_k x_t
        print(f"  sparse workers (us from the tail's t0): first ticket {(B[:, 0].min() - tt0) / 100.0:.2f}, "
              f"last X_k {(B[:, 2].max() - tt0) / 100.0:.2f}, last x_k {(B[:, 3].max() - tt0) / 100.0:.2f}; "
              f"per column ready->X_k mean {((B[:, 2] - B[:, 1]) / 100.0).mean():.2f} us")
        for L in range(lev[:c0].max() + 1):
            ks = cols[lev[:c0] == L]
            if len(ks):
                b = B[ks]
                print(f"    level {L:2d} cols {len(ks):4d}: ticket min {(b[:, 0].min() - tt0) / 100.0:8.2f}  ready max "
                      f"{(b[:, 1].max() - tt0) / 100.0:8.2f}  X_k max {(b[:, 2].max() - tt0) / 100.0:8.2f}  "
                      f"ready->X_k mean {((b[:, 2] - b[:, 1]) / 100.0).mean():6.2f}")
    if T[699, 0]:
        print(f"  back-substitution: flags seen {(T[698, 0] - tt0) / 100.0:.2f}, loop start {(T[699, 0] - tt0) / 100.0:.2f}; "
              "x_K published at " + " ".join(f"{(T[700 + K, 0] - tt0) / 100.0:.2f}" for K in range(TC - 1, -1, -1)))
