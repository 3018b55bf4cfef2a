"""Device-resident FactorGraph: the host-side mirror of
global_opt.py:12-213 over a preallocated edge store and keyframe store.

The reference keeps its edges as growing torch tensors and, on every solve,
concatenates them into the two-way form (`prep_two_way_edges`,
global_opt.py:104-110 — a copy of all edge data, 2 x 13 B per directed edge
pixel) and stacks the keyframe pointmaps (`get_poses_points`, :112-119). Here:

* ``EdgeStore`` holds the directed edges already in two-way form, each
  undirected edge as two adjacent rows (i->j, j->i), in capacity-doubling
  device buffers: a solve passes views, nothing is copied. Match indices are
  int32 (a pixel index of one keyframe, < 2^31): the GN's first iteration
  reads 9 B of edge data per pixel instead of 13 (m3s_gn_args.idx_i32);
* ``KeyframeStore`` holds X_canon / C / N / T_WC in [capacity, ...] buffers
  like SharedKeyframes (frame.py:220-247), plus C / N and (calib) the
  ray-constrained pointmaps, kept current on every write; when the graph's
  keyframes are a contiguous id range (the usual case) the solve passes views
  — no per-solve copy of pointmaps or confidences — and the GN updates the
  stored poses in place.

The per-edge order differs from the reference's (interleaved instead of all
forward then all reverse); the normal equations are order-independent up to
fp64 rounding of the per-slot sums (tests/test_factor_graph.py checks the
mirror against the oracle fed the reference's concatenated edge order).
X / C keep the SharedKeyframes array-of-structs layout [cap, HW, 3]: the GN
gathers X_i through idx, and one 12-B point per gathered pixel stays within
one cache line (three separate planes would touch three). ``add_factors`` takes the outputs of
mast3r_match_symmetric (the network is out of scope) and applies the
reference's edge filter (global_opt.py:56-78).
"""
from __future__ import annotations

import torch

import mast3r_slam_backends as be

# config/base.yaml:35-50
LOCAL_OPT_CFG = dict(pin=1, window_size=1e6, C_conf=0.0, Q_conf=1.5, min_match_frac=0.1,
                     pixel_border=-10, depth_eps=1e-6, max_iters=10, sigma_ray=0.003, sigma_dist=1e1,
                     sigma_pixel=1.0, sigma_depth=1e1, sigma_point=0.05, delta_norm=1e-8)


class EdgeStore:
    """Two-way directed edges: row 2k = (ii_k -> jj_k), row 2k+1 = (jj_k -> ii_k)."""

    def __init__(self, HW: int, device, capacity: int = 64):
        self.HW, self.device, self.n = int(HW), device, 0
        self._alloc(max(int(capacity), 1))

    def _alloc(self, cap):
        grow = hasattr(self, "_ii")
        d, HW = self.device, self.HW
        new = dict(ii=torch.empty(2 * cap, dtype=torch.int64, device=d),
                   jj=torch.empty(2 * cap, dtype=torch.int64, device=d),
                   idx=torch.empty(2 * cap, HW, dtype=torch.int32, device=d),
                   valid=torch.empty(2 * cap, HW, 1, dtype=torch.bool, device=d),
                   Q=torch.empty(2 * cap, HW, 1, dtype=torch.float32, device=d))
        if grow:
            for k, t in new.items():
                t[: 2 * self.n].copy_(getattr(self, "_" + k)[: 2 * self.n])
        for k, t in new.items():
            setattr(self, "_" + k, t)
        self.capacity = cap

    def append(self, ii, jj, idx_i2j, idx_j2i, valid_j, valid_i, Qj, Qi):
        e = int(ii.numel())
        if self.n + e > self.capacity:
            self._alloc(max(2 * self.capacity, self.n + e))
        r0, r1 = 2 * self.n, 2 * (self.n + e)
        self._ii[r0:r1:2], self._ii[r0 + 1:r1:2] = ii, jj
        self._jj[r0:r1:2], self._jj[r0 + 1:r1:2] = jj, ii
        self._idx[r0:r1:2], self._idx[r0 + 1:r1:2] = idx_i2j.reshape(e, -1), idx_j2i.reshape(e, -1)
        self._valid[r0:r1:2] = valid_j.reshape(e, -1, 1)
        self._valid[r0 + 1:r1:2] = valid_i.reshape(e, -1, 1)
        self._Q[r0:r1:2], self._Q[r0 + 1:r1:2] = Qj.reshape(e, -1, 1), Qi.reshape(e, -1, 1)
        self.n += e

    def directed(self):
        """Views (ii, jj, idx_ii2jj, valid_match, Q) of the 2n directed edges."""
        m = 2 * self.n
        return self._ii[:m], self._jj[:m], self._idx[:m], self._valid[:m], self._Q[:m]


class KeyframeStore:
    """X_canon [cap,HW,3], C [cap,HW,1], N [cap], T_WC [cap,8] (SharedKeyframes
    layout), plus what the GN reads, kept current on every write so a solve
    passes views instead of building them:

    * ``Cn`` [cap,HW,1] = C / N, the average confidence the reference forms per
      solve (``get_average_conf``, frame.py:107-108; global_opt.py:114-117);
    * ``Xr`` [cap,HW,3] (when the store has intrinsics K): X_canon constrained to
      the pixel rays, z * [(u-cx)/fx, (v-cy)/fy, 1], which solve_GN_calib forms
      per solve (constrain_points_to_ray, global_opt.py:172)."""

    def __init__(self, H: int, W: int, device, capacity: int = 512, K=None):
        self.H, self.W, self.device, self.n = H, W, device, 0
        HW = H * W
        self.X = torch.zeros(capacity, HW, 3, device=device)
        self.C = torch.zeros(capacity, HW, 1, device=device)
        self.N = torch.zeros(capacity, dtype=torch.int32, device=device)
        self.T_WC = torch.zeros(capacity, 8, device=device)
        self.Cn = torch.zeros(capacity, HW, 1, device=device)
        self.K = None if K is None else torch.as_tensor(K, dtype=torch.float32, device=device)
        self.Xr = torch.zeros(capacity, HW, 3, device=device) if K is not None else None
        if K is not None:
            self._rays = _pixel_rays(H, W, self.K)

    def append(self, X, C, T_WC, N=1):
        k = self.n
        self.n += 1
        self.T_WC[k].copy_(T_WC.reshape(8))
        self.set_pointmap(k, X, C, N)
        return k

    def set_pointmap(self, k, X, C, N):
        """Keyframe k's canonical pointmap, accumulated confidence and update
        count (after Frame.update_pointmap, frame.py:41-105), with the derived
        Cn / Xr rows."""
        self.X[k].copy_(X.reshape(-1, 3))
        self.C[k].copy_(C.reshape(-1, 1))
        self.N[k] = int(N)
        torch.div(self.C[k], float(N), out=self.Cn[k])
        if self.Xr is not None:
            torch.mul(self.X[k][:, 2:3], self._rays, out=self.Xr[k])

    def update_T_WCs(self, T_WCs, idx):  # frame.py:309-311
        self.T_WC[idx] = T_WCs


def _pixel_rays(H, W, K):
    """[(u-cx)/fx, (v-cy)/fy, 1] of the row-major pixel grid, [H*W, 3]."""
    v, u = torch.meshgrid(torch.arange(H, device=K.device, dtype=torch.float32),
                          torch.arange(W, device=K.device, dtype=torch.float32), indexing="ij")
    return torch.stack(((u.reshape(-1) - K[0, 2]) / K[0, 0], (v.reshape(-1) - K[1, 2]) / K[1, 1],
                        torch.ones(H * W, device=K.device)), -1)


def ray_constrained(Xs, K, H, W):
    """constrain_points_to_ray (geometry.py:37-42) of [n, HW, 3] pointmaps."""
    return (Xs[..., 2:3] * _pixel_rays(H, W, torch.as_tensor(K, device=Xs.device))).contiguous()


class FactorGraph:
    def __init__(self, keyframes: KeyframeStore, K=None, cfg=LOCAL_OPT_CFG, edge_capacity=64):
        self.frames, self.K, self.cfg = keyframes, K, cfg
        self.edges = EdgeStore(keyframes.H * keyframes.W, keyframes.device, edge_capacity)
        self.ii_u = torch.empty(0, dtype=torch.int64, device=keyframes.device)  # undirected, for ids
        self.jj_u = torch.empty(0, dtype=torch.int64, device=keyframes.device)
        self._workspace = None

    def add_factors(self, ii, jj, idx_i2j, idx_j2i, valid_match_j, valid_match_i, Qj, Qi,
                    min_match_frac, is_reloc=False):
        """global_opt.py:31-100 after mast3r_match_symmetric: Qj/Qi are the
        already combined qualities sqrt(Q_ii[idx] * Q_ji) (:53-55)."""
        dev = self.frames.device
        ii = torch.as_tensor(ii, device=dev)
        jj = torch.as_tensor(jj, device=dev)
        valid_j = valid_match_j & (Qj > self.cfg["Q_conf"])
        valid_i = valid_match_i & (Qi > self.cfg["Q_conf"])
        frac_j = valid_j.reshape(valid_j.shape[0], -1).float().mean(1)
        frac_i = valid_i.reshape(valid_i.shape[0], -1).float().mean(1)
        invalid = (torch.minimum(frac_j, frac_i) < min_match_frac) & ~(ii == (jj - 1))
        if bool(invalid.any()) and is_reloc:
            return False
        keep = ~invalid
        if not bool(keep.any()):
            return False
        self.edges.append(ii[keep], jj[keep], idx_i2j[keep], idx_j2i[keep], valid_match_j[keep],
                          valid_match_i[keep], Qj[keep], Qi[keep])
        self.ii_u = torch.cat([self.ii_u, ii[keep]])
        self.jj_u = torch.cat([self.jj_u, jj[keep]])
        return True

    def get_unique_kf_idx(self):
        return torch.unique(torch.cat([self.ii_u, self.jj_u]), sorted=True)

    def _poses_points(self, uk, calib):
        """Views when the keyframes are ids [a, a+n) (no copy); gathers
        otherwise. Xs is the ray-constrained store for calib."""
        n = uk.numel()
        a = int(uk[0])
        F = self.frames
        X = F.Xr if calib else F.X
        contiguous = int(uk[-1]) - a + 1 == n
        if contiguous:
            return X[a:a + n], F.Cn[a:a + n], F.T_WC[a:a + n], contiguous
        return X[uk], F.Cn[uk], F.T_WC[uk].contiguous(), contiguous

    def _solve(self, calib):
        pin = self.cfg["pin"]
        uk = self.get_unique_kf_idx()
        if uk.numel() <= pin:
            return
        if calib and self.frames.Xr is None:
            raise RuntimeError("solve_GN_calib needs a KeyframeStore built with K")
        Xs, Cs, T, contiguous = self._poses_points(uk, calib)
        # the reference GN holds rank 0 fixed and writes back poses [pin:]
        # (global_opt.py:158); in place, poses 1..pin-1 are restored after
        held = T[1:pin].clone() if contiguous and pin > 1 else None
        ii, jj, idx, valid, Q = self.edges.directed()
        c = self.cfg
        if calib:
            H, W = self.frames.H, self.frames.W
            be.gauss_newton_calib(T, Xs, Cs, self.K, ii, jj, idx, valid, Q,
                                  H, W, c["pixel_border"], c["depth_eps"], c["sigma_pixel"],
                                  c["sigma_depth"], c["C_conf"], c["Q_conf"], c["max_iters"],
                                  c["delta_norm"])
        else:
            be.gauss_newton_rays(T, Xs, Cs, ii, jj, idx, valid, Q, c["sigma_ray"], c["sigma_dist"],
                                 c["C_conf"], c["Q_conf"], c["max_iters"], c["delta_norm"])
        if held is not None:
            T[1:pin].copy_(held)
        if not contiguous:  # the GN updated a gathered copy: write back (global_opt.py:158)
            self.frames.update_T_WCs(T[pin:], uk[pin:])

    def solve_GN_rays(self):  # global_opt.py:121-158
        self._solve(calib=False)

    def solve_GN_calib(self):  # global_opt.py:160-213
        self._solve(calib=True)
