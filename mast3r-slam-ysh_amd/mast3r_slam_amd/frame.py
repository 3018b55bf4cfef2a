"""Host-side mirror of the reference keyframe pointmap bookkeeping
(Frame.update_pointmap / get_average_conf, frame.py:41-104) and of the
tracker's fusion step (tracker.py:98-99), with the per-pixel work in the HIP
kernel ``mast3r_slam_backends.fuse_pointmap``.

``Pointmap`` holds what the reference ``Frame`` holds for this purpose
(X_canon [HW,3], C [HW,1], N, N_updates, score) and applies the same
filtering modes (config tracking.filtering_mode). weighted_pointmap (the
default), weighted_spherical, indep_conf and recent run in one fused device
pass; first and best_score are whole-tensor copies decided on the host as the
reference does.
"""
from __future__ import annotations

import torch

import mast3r_slam_backends as be


class Pointmap:
    def __init__(self, filtering_mode: str = "weighted_pointmap", filtering_score: str = "median"):
        self.mode = filtering_mode
        self.filtering_score = filtering_score
        self.X_canon = None
        self.C = None
        self.N = 0
        self.N_updates = 0
        self.score = None

    def get_score(self, C):  # frame.py:33-39
        return torch.median(C) if self.filtering_score == "median" else torch.mean(C)

    def get_average_conf(self):  # frame.py:102-103
        return self.C / self.N if self.C is not None else None

    def update_pointmap(self, X: torch.Tensor, C: torch.Tensor, T=None):
        """frame.py:41-100; if T (Sim3 data [8] / [1,8]) is given the points
        are X' = T.act(X) first, fused into the same pass (tracker.py:98-99)."""
        if self.N == 0 or self.mode in ("first", "best_score"):
            if T is not None:
                X = _act(T, X)
            if self.N == 0:
                self.X_canon, self.C = X.clone(), C.clone()
                self.N = self.N_updates = 1
                if self.mode == "best_score":
                    self.score = self.get_score(C)
                return
            if self.mode == "first":
                if self.N_updates == 1:
                    self.X_canon, self.C, self.N = X.clone(), C.clone(), 1
            else:
                new_score = self.get_score(C)
                if new_score > self.score:
                    self.X_canon, self.C, self.N, self.score = X.clone(), C.clone(), 1, new_score
            self.N_updates += 1
            return
        if self.mode not in be.FILTER_MODES:
            raise NotImplementedError(f"filtering_mode {self.mode!r} is not built on the device path")
        be.fuse_pointmap(self.X_canon, self.C, X.contiguous(), C.contiguous(),
                         None if T is None else _pose(T), self.mode)
        self.N = self.N + 1 if self.mode in ("weighted_pointmap", "weighted_spherical") else 1
        self.N_updates += 1


def _pose(T):
    d = T.data if hasattr(T, "data") else T
    return d.reshape(-1, 8)[0].contiguous()


def _act(T, X):
    """T.act(X) through the fusion kernel in 'recent' mode (no torch math)."""
    out = torch.empty_like(X)
    c = torch.zeros(X.shape[0], 1, dtype=X.dtype, device=X.device)
    be.fuse_pointmap(out, c, X.contiguous(), c.clone(), _pose(T), "recent")
    return out


def fuse_tracked_points(keyframe: Pointmap, T_CkCf, Xkf, Ckf):
    """tracker.py:98-99: keyframe.update_pointmap(T_CkCf.act(Xkf), Ckf)."""
    keyframe.update_pointmap(Xkf, Ckf, T=T_CkCf)
