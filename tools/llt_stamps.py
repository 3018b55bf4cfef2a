"""Item timeline of the one-workgroup sparse LLT at C3 (GPU box).

  tools/mkvar.sh lst -DM3S_LLT_STAMPS && python tools/llt_stamps.py variants/lib_lst.so

Runs bench.py's C3 call (calib, 32 KFs, 512x512) with 2 GN iterations on the
stamped build (sparse_llt_kernel<1> records the shader clock per dispatched
item: ticket, inputs summed, published, forward step done; and its phases),
then prints the phase split, per-kind means and the critical path of the
factorisation: from the last item to finish, back through the input that
arrived last (DIAG(k) <- the L_kp blocks of its update list; OFF(i,k) <- its
update blocks and DIAG(k)), with the time each hop spent waiting (flag hand-
off) and computing."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mast3r-slam-ysh_amd")]
import torch  # noqa: E402

import mast3r_slam_backends as be  # noqa: E402
from mast3r_slam_amd import synthetic  # noqa: E402

be._lib = be._load(os.path.abspath(sys.argv[1]))
dev = torch.device("cuda:0")
N = int(os.environ.get("LS_N", "32"))
H = W = 512 if N <= 32 else 64
g = synthetic.make_graph(N, H, W, seed=1003, device=dev)
Xs = (g.Xs[..., 2:3] * synthetic.pixel_rays(H, W, g.K)[None]).contiguous()
Twc = g.T_init.data.clone().contiguous()
info = torch.zeros(8, dtype=torch.int32, device=dev)
for _ in range(3):
    Twc.copy_(g.T_init.data)
    be.gauss_newton_calib(Twc, Xs, g.Cs.contiguous(), g.K, g.ii.contiguous(), g.jj.contiguous(), g.idx_ii2jj,
                          g.valid_match, g.Q, H, W, -10, 1e-6, 1.0, 10.0, 0.0, 1.5, 2, 0.0, info=info)
torch.cuda.synchronize()
be._lib.m3s_debug_stamps.argtypes = [ctypes.c_int, ctypes.c_void_p]
buf = np.zeros(2048 * 4 + 2048 * 2 + 8, np.int64)
if be._lib.m3s_debug_stamps(2, ctypes.c_void_p(buf.ctypes.data)) != 1:
    sys.exit("library built without -DM3S_LLT_STAMPS")
st = buf[:2048 * 4].reshape(2048, 4)
items = buf[2048 * 4:2048 * 6].reshape(2048, 2)
ph = buf[2048 * 6:2048 * 6 + 8]

ii, jj = g.ii.cpu().numpy(), g.jj.cpu().numpy()
u, inv = np.unique(np.concatenate([ii, jj]), return_inverse=True)
ri, rj = inv[:len(ii)], inv[len(ii):]
P = be.sparse_plan(N, ri, rj)
m, T = P["m"], len(P["task_dst"])
n = m + T  # dispatch slots used (no PART items at this size)
t0 = ph[0]
span = ph[4] - ph[0]
print(f"N={N} m={m} OFF tasks={T}; kernel span {span} clk: assembly {ph[1] - ph[0]}, factor {ph[2] - ph[1]}, "
      f"back-sub {ph[3] - ph[2]}, retraction {ph[4] - ph[3]}")
rec = {}
for it in range(n):
    item, wave = int(items[it, 0]), int(items[it, 1])
    rec[item] = dict(it=it, wave=wave, t=st[it] - t0)
diag = {k: rec[-1 - k] for k in range(m) if -1 - k in rec}
off = {t: rec[t] for t in range(T) if t in rec}
# DIAG: ticket -> summed (t1) -> published (t2) -> fwd (t3); OFF: ticket -> summed (t1) -> W_k ready (t3) -> published (t2)
d_sum = np.mean([d["t"][1] - d["t"][0] for d in diag.values()])
d_fac = np.mean([d["t"][2] - d["t"][1] for d in diag.values()])
d_fwd = np.mean([d["t"][3] - d["t"][2] for d in diag.values()])
o_sum = np.mean([o["t"][1] - o["t"][0] for o in off.values()])
o_w = np.mean([o["t"][3] - o["t"][1] for o in off.values()])
o_x = np.mean([o["t"][2] - o["t"][3] for o in off.values()])
print(f"DIAG n={len(diag)}: ticket->summed {d_sum:.0f}, factor+publish {d_fac:.0f}, forward step {d_fwd:.0f} clk")
print(f"OFF  n={len(off)}: ticket->summed {o_sum:.0f}, wait W_k {o_w:.0f}, product+publish {o_x:.0f} clk")
# slot -> producer (DIAG k for slot k < m, else the OFF task storing it)
prod = {k: ("D", k) for k in range(m)}
for t in range(T):
    prod[int(P["task_dst"][t])] = ("O", t)


def done(p):
    kind, x = p
    return (diag[x]["t"][2] if kind == "D" else off[x]["t"][2])


def inputs(p):
    kind, x = p
    if kind == "D":
        sl = P["dtr_slot"][P["dtr_ptr"][x]:P["dtr_ptr"][x + 1]]
        return [prod[int(s)] for s in sl]
    q0, q1 = P["task_tr_ptr"][x], P["task_tr_ptr"][x + 1]
    return [prod[int(s)] for s in P["tr_a"][q0:q1]] + [prod[int(s)] for s in P["tr_b"][q0:q1]] + \
        [("D", int(P["task_col"][x]))]


last = max([("D", k) for k in diag] + [("O", t) for t in off], key=done)
path = []
cur = last
while True:
    ins = inputs(cur)
    path.append(cur)
    if not ins:
        break
    cur = max(ins, key=done)
path.reverse()
print(f"critical path: {len(path)} items, factor ends at {done(last)} clk")
tot_wait = tot_busy = 0
prev_done = ph[1] - t0
for p in path:
    r = diag[p[1]] if p[0] == "D" else off[p[1]]
    t = r["t"]
    start = t[0]
    wait = max(0, start - prev_done)  # inputs final -> item picked up by a wave (dispatch / wave switch)
    ready_gap = max(0, (t[1] if p[0] == "D" else t[3]) - max(start, prev_done))
    busy = t[2] - max(t[1] if p[0] == "D" else t[3], prev_done)
    tot_wait += wait
    tot_busy += busy
    print(f"  {p[0]}{p[1]:4d} wave {r['wave']:2d}  ticket {t[0]:6d}  inputs-final {prev_done:6d}  "
          f"summed/W {t[1] if p[0] == 'D' else t[3]:6d}  published {t[2]:6d}  (pickup {wait}, in-item wait+sum "
          f"{ready_gap}, compute {busy})")
    prev_done = t[2]
print(f"critical path totals: pickup {tot_wait} clk, compute {tot_busy} clk")
