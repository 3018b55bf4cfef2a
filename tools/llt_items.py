"""Per-item timeline of sparse_llt_kernel's factorisation (lib built with
-DM3S_LLT_ITEMS=1, M3S_LIB=...): busy/wait per item kind and the critical
path through the dataflow (which items and waits the factor time is made of).
Clock: s_memtime (shader clock cycles)."""
import ctypes, os, sys
from collections import defaultdict
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import numpy as np
import torch
import mast3r_slam_backends as be
from mast3r_slam_amd import synthetic

dev = torch.device("cuda:0")
for N in [int(x) for x in os.environ.get("NS", "32,64,128").split(",")]:
    H = W = 64
    g = synthetic.make_graph(N, H, W, seed=1003, device=dev)
    E, HW = g.n_edges, H * W
    wst = torch.zeros(int(be._lib.m3s_gn_workspace_size(N, HW, E)), dtype=torch.uint8, device=dev)
    a, keep = be.make_gn_args(be.MODE_RAYS, g.T_init.data.contiguous(), g.Xs, g.Cs, g.ii, g.jj, g.idx_ii2jj,
                              g.valid_match, g.Q, None, sigma_a=0.003, sigma_b=10.0, C_thresh=0.0,
                              Q_thresh=1.5, max_iter=1, delta_thresh=0.0, workspace=wst)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    lay = be.workspace_layout(N, HW, E)
    u = torch.unique(torch.cat([g.ii, g.jj]))
    ri, rj = [torch.searchsorted(u, t).cpu().numpy() for t in (g.ii, g.jj)]
    m = N - 1
    p = be.sparse_plan(N, ri, rj)
    if 8 * ((p["S"] + m) * 49 + m * 7) > 150 * 1024:  # global factor: split updates as the solver does
        slot_cap = min(m * (m + 1) // 2, 64 * m + 4096) + 1
        p = be.sparse_plan(N, ri, rj, 8, slot_cap - 1)
    n_it = len(p["witems"])
    for rep in range(4):
        assert be._lib.m3s_gauss_newton_rays(ctypes.byref(a), st) == 0
        torch.cuda.synchronize()
    ts = wst[lay["A"]: lay["A"] + 32 * n_it].clone().view(torch.int64).cpu().numpy().reshape(n_it, 4)
    T = len(p["task_dst"])
    # dynamic dispatch: the wave that ran an item is in bits 58.. of stamp 0
    wave_of = (ts[:, 0] >> 58).astype(int)
    ts[:, 0] &= (1 << 58) - 1
    items = p["witems"]
    pos = {int(v): i for i, v in enumerate(items)}
    t0 = ts[:, 0].min()
    ts = ts - t0
    kind = np.where(items >= T, 2, np.where(items < 0, 0, 1))
    names = ["DIAG", "OFF", "PART"]
    span = ts[:, 2].max()
    print(f"N={N} S={p['S']} items={n_it} (DIAG {m}, OFF {T}, PART {p['n_parts']}) factor span {span} cycles")
    for k in range(3):
        sel = kind == k
        if sel.any():
            print(f"  {names[k]:5s} n={sel.sum():4d} busy mean {np.mean(ts[sel, 2] - ts[sel, 1]):7.0f} "
                  f"wait mean {np.mean(ts[sel, 1] - ts[sel, 0]):7.0f}")
    if (kind == 0).any():
        sel = kind == 0
        print(f"  DIAG to sdone (chol + W) mean {np.mean(ts[sel, 3] - ts[sel, 1]):.0f}, forward step "
              f"{np.mean(ts[sel, 2] - ts[sel, 3]):.0f}")
    # producers: slot -> (item position, stamp index of its publish)
    slot_pub, y_pub = {}, {}
    for i, v in enumerate(items):
        v = int(v)
        if v < 0:
            slot_pub[-1 - v] = (i, 3)
            y_pub[-1 - v] = (i, 2)
        elif v < T:
            slot_pub[int(p["task_dst"][v])] = (i, 2)

    def deps(v):
        out = []
        if v >= T:
            pi = v - T
            for q in range(p["part_q0"][pi], p["part_q1"][pi]):
                if p["part_tgt"][pi] < 0:
                    out += [slot_pub[int(p["dtr_slot"][q])], y_pub[int(p["dtr_p"][q])]]
                else:
                    out += [slot_pub[int(p["tr_a"][q])], slot_pub[int(p["tr_b"][q])]]
            return out
        sp = len(p["dpart_ptr"]) > 0
        if v < 0:
            k = -1 - v
            ps = range(p["dpart_ptr"][k], p["dpart_ptr"][k + 1]) if sp else []
            out += [(pos[T + pi], 2) for pi in ps]
            for q in range(p["dtr_ptr"][k], p["dtr_ptr"][k + 1]):
                out.append(slot_pub[int(p["dtr_slot"][q])])
            return out
        ps = range(p["opart_ptr"][v], p["opart_ptr"][v + 1]) if sp else []
        out += [(pos[T + pi], 2) for pi in ps]
        out.append(slot_pub[int(p["task_col"][v])])
        for q in range(p["task_tr_ptr"][v], p["task_tr_ptr"][v + 1]):
            out.append(slot_pub[int(p["tr_a"][q])])
        return out

    # dense top clique: trailing columns whose structure is every later column
    cnt = np.diff(p["col_ptr"])
    cq = 0
    for k in range(m - 1, -1, -1):
        if cnt[k] != m - 1 - k:
            break
        cq += 1
    dk = np.where(items < 0, -1 - items, -1)
    pre = (items < 0) & (dk < m - cq)
    cl = (items < 0) & (dk >= m - cq)
    if pre.any() and cl.any():
        print(f"  clique {cq} columns: last non-clique L_kk at {ts[pre, 3].max()}, clique L_kk from "
              f"{ts[cl, 3].min()} to {ts[cl, 3].max()} cycles")
    cur, stamp = int(np.argmax(ts[:, 2])), 2
    comp = defaultdict(float)
    chain = 0
    while True:
        chain += 1
        comp[names[kind[cur]] + " busy"] += ts[cur, stamp] - ts[cur, 1]
        dl = deps(int(items[cur]))
        same = [i for i in range(n_it) if wave_of[i] == wave_of[cur] and ts[i, 0] < ts[cur, 0]]
        prev_same = max(same, key=lambda i: ts[i, 0]) if same else None
        dmax = max(dl, key=lambda d: ts[d[0], d[1]]) if dl else None
        # what the item started after: its wave's previous item or its last input
        if dmax is not None and ts[dmax[0], dmax[1]] > ts[cur, 0]:
            comp["flag latency"] += ts[cur, 1] - ts[dmax[0], dmax[1]]
            cur, stamp = dmax
        elif prev_same is not None:
            comp["wave switch"] += ts[cur, 1] - ts[prev_same, 2]
            cur, stamp = prev_same, 2
        else:
            comp["start"] += ts[cur, 1]
            break
    print(f"  critical path: {chain} items; " + ", ".join(f"{k} {v:.0f}" for k, v in sorted(comp.items())))
