"""ctypes/numpy front end of the CPU oracle.

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker. The product path never imports it.

* ``gn(...)`` / ``edge_blocks(...)``  -> oracle/gn_oracle.c (restatement of
  gn_kernels.cu; see that file's header for citations and pinning)
* ``tracker_*``                       -> oracle/tracker_oracle.py (numpy
  restatement of tracker.py / geometry.py / nonlinear_optimizer.py)
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libgn_oracle.so")
LIB_F64_PATH = os.path.join(HERE, "libgn_oracle_f64.so")  # fp64 per-edge sums (yardstick)

MODE_POINTS, MODE_RAYS, MODE_CALIB = 0, 1, 2


class Params(ctypes.Structure):
    _fields_ = [
        ("mode", ctypes.c_int),
        ("sigma_a", ctypes.c_float),
        ("sigma_b", ctypes.c_float),
        ("C_thresh", ctypes.c_float),
        ("Q_thresh", ctypes.c_float),
        ("fx", ctypes.c_float),
        ("fy", ctypes.c_float),
        ("cx", ctypes.c_float),
        ("cy", ctypes.c_float),
        ("height", ctypes.c_int),
        ("width", ctypes.c_int),
        ("pixel_border", ctypes.c_int),
        ("z_eps", ctypes.c_float),
    ]


_libs = {}


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib(f64=False):
    path = LIB_F64_PATH if f64 else LIB_PATH
    if path not in _libs:
        if not os.path.exists(path):
            build()
        _lib = ctypes.CDLL(path)
        _libs[path] = _lib
        P = ctypes.c_void_p
        _lib.oracle_gn.restype = ctypes.c_int
        _lib.oracle_gn.argtypes = [
            ctypes.POINTER(Params), P, P, P, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int,
            P, P, P, ctypes.c_int, ctypes.c_float, P, P,
        ]
        _lib.oracle_edge_blocks.restype = ctypes.c_int
        _lib.oracle_edge_blocks.argtypes = [
            ctypes.POINTER(Params), P, P, P, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_int,
            P, P, P, P, P,
        ]
        for f in ("oracle_retract", "oracle_adjT_inv", "oracle_relative"):
            getattr(_lib, f).restype = None
            getattr(_lib, f).argtypes = [P, P, P] if f != "oracle_retract" else [P, P]
    return _libs[path]


def _c(a, dtype):
    a = np.ascontiguousarray(np.asarray(a), dtype=dtype)
    return a


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def make_params(mode, sigma_a=0.0, sigma_b=0.0, C_thresh=0.0, Q_thresh=1.5, K=None,
                height=0, width=0, pixel_border=0, z_eps=0.0):
    p = Params()
    p.mode = mode
    p.sigma_a, p.sigma_b = sigma_a, sigma_b
    p.C_thresh, p.Q_thresh = C_thresh, Q_thresh
    if K is not None:
        K = np.asarray(K, np.float32)
        p.fx, p.fy, p.cx, p.cy = float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])
    p.height, p.width, p.pixel_border, p.z_eps = int(height), int(width), int(pixel_border), z_eps
    return p


def _inputs(Twc, Xs, Cs, ii, jj, idx, valid, Q):
    Twc = _c(Twc, np.float32).reshape(-1, 8).copy()
    Xs = _c(Xs, np.float32)
    Cs = _c(Cs, np.float32)
    ii = _c(ii, np.int64).reshape(-1)
    jj = _c(jj, np.int64).reshape(-1)
    idx = _c(idx, np.int64)
    valid = _c(valid, np.uint8)
    Q = _c(Q, np.float32)
    N, HW = Xs.shape[0], Xs.shape[1]
    E = ii.shape[0]
    assert idx.size == E * HW and valid.size == E * HW and Q.size == E * HW
    assert Cs.size == N * HW
    return Twc, Xs, Cs, ii, jj, idx, valid, Q, N, HW, E


def gn(params, Twc, Xs, Cs, ii, jj, idx, valid, Q, max_iter, delta_thresh, f64=False):
    """Returns (Twc_out [N,8], dx [N-1,7], iters, solve_failed). f64: the
    fp64-accumulator build (not the reference's arithmetic; a yardstick)."""
    Twc, Xs, Cs, ii, jj, idx, valid, Q, N, HW, E = _inputs(Twc, Xs, Cs, ii, jj, idx, valid, Q)
    dx = np.zeros((max(N - 1, 0), 7), np.float32)
    failed = ctypes.c_int(0)
    it = lib(f64).oracle_gn(
        ctypes.byref(params), _ptr(Twc), _ptr(Xs), _ptr(Cs), N, HW, _ptr(ii), _ptr(jj), E,
        _ptr(idx), _ptr(valid), _ptr(Q), int(max_iter), float(delta_thresh), _ptr(dx),
        ctypes.byref(failed),
    )
    if it < 0:
        raise ValueError("oracle_gn: invalid input (edge references a pose >= N)")
    return Twc, dx, it, failed.value


def edge_blocks(params, Twc, Xs, Cs, ii, jj, idx, valid, Q):
    """Returns (Hs [4,E,7,7], gs [2,E,7]) at the given poses."""
    Twc, Xs, Cs, ii, jj, idx, valid, Q, N, HW, E = _inputs(Twc, Xs, Cs, ii, jj, idx, valid, Q)
    Hs = np.zeros((4, E, 7, 7), np.float32)
    gs = np.zeros((2, E, 7), np.float32)
    rc = lib().oracle_edge_blocks(
        ctypes.byref(params), _ptr(Twc), _ptr(Xs), _ptr(Cs), N, HW, _ptr(ii), _ptr(jj), E,
        _ptr(idx), _ptr(valid), _ptr(Q), _ptr(Hs), _ptr(gs),
    )
    if rc != 0:
        raise ValueError("oracle_edge_blocks: invalid input")
    return Hs, gs


def retract(xi, T, f64=False):
    """T <- Exp(xi) T for one pose. f64=False: the reference's fp32 retrSim3
    (gn_kernels.cu:323-413); f64=True: the exact-arithmetic yardstick's fp64
    evaluation of the same map (gn_oracle.c retract_exact)."""
    xi = _c(xi, np.float32).reshape(7)
    T = _c(T, np.float32).reshape(8).copy()
    lib(f64).oracle_retract(_ptr(xi), _ptr(T))
    return T


def adjT_inv_matrix(Ti):
    """M (7x7) with Jj = M @ J_local (columns = images of unit vectors)."""
    Ti = _c(Ti, np.float32).reshape(8)
    M = np.zeros((7, 7), np.float32)
    for c in range(7):
        e = np.zeros(7, np.float32)
        e[c] = 1.0
        out = np.zeros(7, np.float32)
        lib().oracle_adjT_inv(_ptr(Ti), _ptr(e), _ptr(out))
        M[:, c] = out
    return M


def relative(Ti, Tj):
    Ti = _c(Ti, np.float32).reshape(8)
    Tj = _c(Tj, np.float32).reshape(8)
    out = np.zeros(8, np.float32)
    lib().oracle_relative(_ptr(Ti), _ptr(Tj), _ptr(out))
    return out
