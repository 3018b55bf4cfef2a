"""``mast3r_slam_backends`` — drop-in for the reference's CUDA extension module,
backed by the MI355X HIP library ``libm3s_gn.so`` through its C ABI
(``include/m3s_gn.h``, ``include/m3s_match.h``).

Reference interface (``/root/reference/mast3r_slam/backend/src/gn.cpp:116-122``):
same module name, same function names, same positional arguments, same
in-place update of ``Twc`` and the same return value ``[dx]`` (the last GN step,
``[N-1, 7]`` float32). Callers: ``global_opt.py:140-155`` (rays) and
``global_opt.py:190-210`` (calib).

Error behaviour: like ``TORCH_CHECK(x.is_contiguous())`` (``gn.cpp:14-21``) a
non-contiguous input raises ``RuntimeError("<name> must be contiguous")``. In
addition, tensors that are not on a ROCm device, or have the wrong dtype,
raise ``RuntimeError`` — there is no CPU fallback: without the HIP library this
module fails at import.

New entry points (the reference tracker has no backend call, tracker.py:173-266):
``track_rays_sim3`` and ``track_calib_sim3``.

``iter_proj`` / ``refine_matches`` (gn.cpp:84-114, matching_kernels.cu) run
the HIP matching kernels with the reference's signatures and return values.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libm3s_gn.so"
LIB_PATH = os.environ.get("M3S_LIB") or os.path.join(_HERE, LIB_NAME)  # override: experiments only
# the same sources built with -DM3S_TEST_PATHS: the A/B reference solver paths
# and test hooks, for the tests that compare against them (never the product)
TEST_LIB_PATH = os.path.join(_HERE, "libm3s_gn_test.so")

M3S_OK, M3S_EINVAL, M3S_ELAUNCH, M3S_ETOOLARGE = 0, 1, 2, 3
MODE_POINTS, MODE_RAYS, MODE_CALIB = 0, 1, 2
INFO_ITERS, INFO_SOLVE_FAIL, INFO_BAD_EDGE, INFO_CONVERGED, INFO_N_UNIQUE = 0, 1, 2, 3, 4
EDGE_SUM_STRIDE = 36

_VP = ctypes.c_void_p


class GnArgs(ctypes.Structure):
    """Mirror of ``m3s_gn_args`` (include/m3s_gn.h)."""

    _fields_ = [
        ("Twc", _VP), ("Xs", _VP), ("Cs", _VP), ("ii", _VP), ("jj", _VP),
        ("idx_ii2jj", _VP), ("valid_match", _VP), ("Q", _VP), ("K", _VP),
        ("N", ctypes.c_int64), ("HW", ctypes.c_int64), ("E", ctypes.c_int64),
        ("mode", ctypes.c_int),
        ("sigma_a", ctypes.c_float), ("sigma_b", ctypes.c_float),
        ("C_thresh", ctypes.c_float), ("Q_thresh", ctypes.c_float),
        ("height", ctypes.c_int), ("width", ctypes.c_int), ("pixel_border", ctypes.c_int),
        ("z_eps", ctypes.c_float),
        ("max_iter", ctypes.c_int), ("delta_thresh", ctypes.c_float),
        ("dx_out", _VP), ("info", _VP),
        ("workspace", _VP), ("workspace_bytes", ctypes.c_size_t),
        ("idx_i32", ctypes.c_int),
    ]


class IterProjArgs(ctypes.Structure):
    """Mirror of ``m3s_iter_proj_args`` (include/m3s_match.h)."""

    _fields_ = [
        ("rays_img", _VP), ("pts_3d_norm", _VP), ("p_init", _VP),
        ("B", ctypes.c_int64), ("H", ctypes.c_int64), ("W", ctypes.c_int64), ("N", ctypes.c_int64),
        ("max_iter", ctypes.c_int), ("lambda_init", ctypes.c_float), ("cost_thresh", ctypes.c_float),
        ("p_new", _VP), ("converged", _VP),
    ]


class RefineArgs(ctypes.Structure):
    """Mirror of ``m3s_refine_args`` (include/m3s_match.h)."""

    _fields_ = [
        ("D11", _VP), ("D21", _VP), ("p1", _VP),
        ("B", ctypes.c_int64), ("H", ctypes.c_int64), ("W", ctypes.c_int64), ("N", ctypes.c_int64),
        ("F", ctypes.c_int64), ("dtype", ctypes.c_int), ("radius", ctypes.c_int),
        ("dilation_max", ctypes.c_int), ("p1_new", _VP),
    ]


class FuseArgs(ctypes.Structure):
    """Mirror of ``m3s_fuse_args`` (include/m3s_fuse.h)."""

    _fields_ = [
        ("X_canon", _VP), ("C", _VP), ("X_new", _VP), ("C_new", _VP), ("T", _VP),
        ("HW", ctypes.c_int64), ("mode", ctypes.c_int),
    ]


class PrepRaysArgs(ctypes.Structure):
    """Mirror of ``m3s_prep_rays_args`` (include/m3s_fuse.h)."""

    _fields_ = [
        ("X11", _VP), ("X21", _VP), ("B", ctypes.c_int64), ("H", ctypes.c_int64),
        ("W", ctypes.c_int64), ("rays_img", _VP), ("pts_norm", _VP),
    ]


class TrackArgs(ctypes.Structure):
    """Mirror of ``m3s_track_args`` (include/m3s_gn.h)."""

    _fields_ = [
        ("Xf", _VP), ("Xk", _VP), ("Qk", _VP), ("valid", _VP), ("T_WCf", _VP), ("T_WCk", _VP),
        ("K", _VP), ("HW", ctypes.c_int64),
        ("height", ctypes.c_int), ("width", ctypes.c_int), ("pixel_border", ctypes.c_int),
        ("z_eps", ctypes.c_float), ("sigma_a", ctypes.c_float), ("sigma_b", ctypes.c_float),
        ("huber_k", ctypes.c_float), ("max_iters", ctypes.c_int),
        ("rel_error", ctypes.c_float), ("delta_norm", ctypes.c_float),
        ("sync_every", ctypes.c_int),
        ("T_WCf_out", _VP), ("T_CkCf_out", _VP), ("info", _VP),
        ("workspace", _VP), ("workspace_bytes", ctypes.c_size_t),
    ]


# every symbol include/m3s_gn.h declares
EXPORTS = (
    "m3s_gn_workspace_size", "m3s_gauss_newton_points", "m3s_gauss_newton_rays",
    "m3s_gauss_newton_calib", "m3s_gn_prepare", "m3s_gn_linearize", "m3s_gn_solve", "m3s_gn_release",
    "m3s_track_workspace_size", "m3s_track_rays_sim3", "m3s_track_calib_sim3", "m3s_version",
    "m3s_sparse_plan_debug", "m3s_gn_layout_debug", "m3s_iter_proj", "m3s_refine_matches",
    "m3s_fuse_pointmap", "m3s_prep_rays", "m3s_debug_stamps", "m3s_debug_sim3",
    "m3s_debug_copy", "m3s_set_knob", "m3s_debug_call_timing", "m3s_debug_call_times",
)
FILTER_MODES = {"weighted_pointmap": 0, "indep_conf": 1, "recent": 2, "weighted_spherical": 3}


def _load(path=LIB_PATH):
    if not os.path.exists(path):
        raise ImportError(
            f"mast3r_slam_backends: {path} is missing; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)"
        )
    lib = ctypes.CDLL(path)
    P = ctypes.POINTER
    lib.m3s_gn_workspace_size.restype = ctypes.c_size_t
    lib.m3s_gn_workspace_size.argtypes = [ctypes.c_int64] * 3
    for f in ("m3s_gauss_newton_points", "m3s_gauss_newton_rays", "m3s_gauss_newton_calib",
              "m3s_gn_prepare"):
        getattr(lib, f).restype = ctypes.c_int
        getattr(lib, f).argtypes = [P(GnArgs), _VP]
    lib.m3s_gn_linearize.restype = ctypes.c_int
    lib.m3s_gn_linearize.argtypes = [P(GnArgs), ctypes.c_int64, ctypes.c_int64, _VP, _VP]
    lib.m3s_gn_solve.restype = ctypes.c_int
    lib.m3s_gn_solve.argtypes = [P(GnArgs), _VP, _VP]
    lib.m3s_gn_release.restype = ctypes.c_int
    lib.m3s_gn_release.argtypes = [P(GnArgs), _VP]
    lib.m3s_track_workspace_size.restype = ctypes.c_size_t
    lib.m3s_track_workspace_size.argtypes = [ctypes.c_int64]
    for f in ("m3s_track_rays_sim3", "m3s_track_calib_sim3"):
        getattr(lib, f).restype = ctypes.c_int
        getattr(lib, f).argtypes = [P(TrackArgs), _VP]
    lib.m3s_version.restype = ctypes.c_char_p
    lib.m3s_version.argtypes = []
    lib.m3s_sparse_plan_debug.restype = ctypes.c_int64
    lib.m3s_sparse_plan_debug.argtypes = [ctypes.c_int32, ctypes.c_int64, _VP, _VP, ctypes.c_int32, ctypes.c_int32, _VP,
                                          ctypes.c_int64, _VP]
    lib.m3s_fuse_pointmap.restype = ctypes.c_int
    lib.m3s_fuse_pointmap.argtypes = [P(FuseArgs), _VP]
    lib.m3s_prep_rays.restype = ctypes.c_int
    lib.m3s_prep_rays.argtypes = [P(PrepRaysArgs), _VP]
    lib.m3s_iter_proj.restype = ctypes.c_int
    lib.m3s_iter_proj.argtypes = [P(IterProjArgs), _VP]
    lib.m3s_refine_matches.restype = ctypes.c_int
    lib.m3s_refine_matches.argtypes = [P(RefineArgs), _VP]
    lib.m3s_debug_stamps.restype = ctypes.c_int
    lib.m3s_debug_stamps.argtypes = [ctypes.c_int, _VP]
    lib.m3s_debug_sim3.restype = ctypes.c_int
    lib.m3s_debug_sim3.argtypes = [ctypes.c_int, _VP, _VP, _VP, ctypes.c_int64, _VP]
    lib.m3s_set_knob.restype = ctypes.c_int
    lib.m3s_set_knob.argtypes = [ctypes.c_char_p, ctypes.c_int]
    lib.m3s_debug_copy.restype = ctypes.c_int
    lib.m3s_debug_copy.argtypes = [_VP, _VP, ctypes.c_int64, ctypes.c_int, _VP]
    lib.m3s_debug_call_timing.restype = ctypes.c_int
    lib.m3s_debug_call_timing.argtypes = [ctypes.c_int]
    lib.m3s_debug_call_times.restype = ctypes.c_int
    lib.m3s_debug_call_times.argtypes = [_VP, _VP, ctypes.c_int]
    lib.m3s_gn_layout_debug.restype = ctypes.c_size_t
    lib.m3s_gn_layout_debug.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _VP]
    return lib


_lib = _load()


def load_test_library():
    """The test build of the library (A/B reference paths, test hooks)."""
    return _load(TEST_LIB_PATH)


def version() -> str:
    return _lib.m3s_version().decode()


PLAN_SECTIONS = ("perm", "col_ptr", "col_row", "col_slot", "lev_ptr", "lev_col", "dtr_ptr",
                 "dtr_slot", "dtr_p", "task_lev_ptr", "task_dst", "task_col", "task_tr_ptr", "tr_a",
                 "tr_b", "asm_ptr", "asm_edge", "g_ptr", "g_edge", "ctask_ptr", "items", "wave_ptr", "witems",
                 "part_q0", "part_q1", "part_tgt", "dpart_ptr", "opart_ptr", "clq", "corder", "ctask0")


LAYOUT_SECTIONS = ("flags", "rank_i", "rank_j", "first", "partials", "edge_sums", "A", "fin",
                   "plan", "Lblk", "Dinv", "tail", "eorder", "planes", "total")


SIM3_OPS = {"exp": (0, 7, None, 8), "retract": (1, 7, 8, 8), "compose": (2, 8, 8, 8), "inverse": (3, 8, None, 8),
            "relative": (4, 8, 8, 8), "act": (5, 8, 3, 3), "act_matrix": (6, 8, 3, 3), "adjT_inv": (7, 8, None, 49),
            "retract_f32": (8, 7, 8, 8)}


def debug_sim3(op: str, a: torch.Tensor, b: torch.Tensor = None) -> torch.Tensor:
    """The device Sim(3) helpers of the hot path on [n, ...] float32 device
    tensors (m3s_debug_sim3; diagnostics/tests). op in SIM3_OPS."""
    code, wa, wb, wo = SIM3_OPS[op]
    a = a.contiguous()
    _check(a, "a", torch.float32)
    n = a.numel() // wa
    if a.numel() != n * wa:
        raise RuntimeError(f"debug_sim3({op}): a must be [n, {wa}]")
    if wb is not None:
        if b is None:
            raise RuntimeError(f"debug_sim3({op}) needs b")
        b = b.contiguous()
        _check(b, "b", torch.float32)
        if b.numel() != n * wb:
            raise RuntimeError(f"debug_sim3({op}): b must be [n, {wb}]")
    out = torch.empty(n, wo, dtype=torch.float32, device=a.device)
    _raise(_lib.m3s_debug_sim3(code, _p(a), _p(b), _p(out), n, _stream(a.device)), "m3s_debug_sim3")
    return out


def set_knob(name: str, value: int) -> int:
    """Set a solver knob for the calls that follow (include/m3s_gn.h
    m3s_set_knob); returns the previous value."""
    old = _lib.m3s_set_knob(name.encode(), int(value))
    if old == -(1 << 30):
        raise RuntimeError(f"unknown knob {name!r}")
    return old


class knob:
    """``with knob("df", 0): ...`` — a knob set for the block, restored after."""

    def __init__(self, name: str, value: int):
        self.name, self.value = name, value

    def __enter__(self):
        self.old = set_knob(self.name, self.value)
        return self

    def __exit__(self, *exc):
        set_knob(self.name, self.old)


def debug_call_timing(enable: bool) -> None:
    """Turn in-call launch timing on or off (m3s_debug_call_timing); the
    record of the calls that follow is read by debug_call_times()."""
    _raise(_lib.m3s_debug_call_timing(1 if enable else 0), "m3s_debug_call_timing")


def debug_call_times(cap: int = 4096):
    """[(kind, ms)] of the timed calls since debug_call_timing(True), in launch
    order; kind 0 = first-iteration (gathering) linearize, 1 = packed
    linearize, 2 = solve launches of one iteration."""
    import numpy as np

    ms = np.zeros(cap, np.float32)
    kinds = np.zeros(cap, np.int32)
    n = _lib.m3s_debug_call_times(ms.ctypes.data, kinds.ctypes.data, cap)
    if n < 0:
        _raise(n, "m3s_debug_call_times")
    n = min(n, cap)
    return [(int(kinds[k]), float(ms[k])) for k in range(n)]


def debug_copy(src: torch.Tensor, dst: torch.Tensor, blocks: int = 4096):
    """dst <- src by the 16-B streaming copy kernel (m3s_debug_copy)."""
    _check(src, "src")
    _check(dst, "dst")
    nb = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() < nb:
        raise RuntimeError("debug_copy: dst too small")
    _raise(_lib.m3s_debug_copy(_p(src), _p(dst), nb, int(blocks), _stream(src.device)), "m3s_debug_copy")


def workspace_layout(N, HW, E):
    """Byte offsets of the GN workspace sections (diagnostics/tests)."""
    offs = (ctypes.c_size_t * len(LAYOUT_SECTIONS))()
    _lib.m3s_gn_layout_debug(int(N), int(HW), int(E), offs)
    return dict(zip(LAYOUT_SECTIONS, list(offs)))


def sparse_plan(N, ri, rj, split=0, max_parts=0):
    """Host symbolic plan of the block-sparse LLT (diagnostics/tests; CPU only).
    split > 0: long update lists cut into PART items (global-factor solves).
    The dense tail (clq) follows M3S_DENSE_TAIL_MIN like the solver."""
    import numpy as np

    ri = np.ascontiguousarray(ri, dtype=np.int32)
    rj = np.ascontiguousarray(rj, dtype=np.int32)
    meta = np.zeros(4 + len(PLAN_SECTIONS), np.int32)
    P = ctypes.c_void_p
    args = (int(N), ri.size, P(ri.ctypes.data), P(rj.ctypes.data), int(split), int(max_parts))
    n = _lib.m3s_sparse_plan_debug(*args, None, 0, P(meta.ctypes.data))
    out = np.zeros(max(n, 1), np.int32)
    _lib.m3s_sparse_plan_debug(*args, P(out.ctypes.data), n, P(meta.ctypes.data))
    offs = list(meta[3:3 + len(PLAN_SECTIONS)]) + [n]
    plan = {"m": int(meta[0]), "S": int(meta[1]), "levels": int(meta[2]),
            "n_parts": int(meta[3 + len(PLAN_SECTIONS)])}
    for k, name in enumerate(PLAN_SECTIONS):
        plan[name] = out[offs[k]:]
    m, S, L, NP = plan["m"], plan["S"], plan["levels"], plan["n_parts"]
    T = int(plan["task_lev_ptr"][L])
    sp = NP > 0 or split > 0
    nc = int(plan["clq"][0])  # dense-tail columns: not dataflow items
    plan["nc"] = nc
    n_items = (m - nc) + (T - nc * (nc - 1) // 2) + NP
    lens = {"perm": m, "col_ptr": m + 1, "lev_ptr": L + 1, "lev_col": m, "dtr_ptr": m + 1,
            "task_lev_ptr": L + 1, "task_dst": T, "task_col": T, "task_tr_ptr": T + 1,
            "asm_ptr": S + 1, "g_ptr": m + 1, "ctask_ptr": m + 1, "clq": 2 + nc + nc * nc,
            "items": n_items, "wave_ptr": 2, "witems": n_items,
            "part_q0": NP, "part_q1": NP, "part_tgt": NP,
            "dpart_ptr": m + 1 if sp else 0, "opart_ptr": T + 1 if sp else 0,
            "corder": m - nc, "ctask0": m}
    for name, ln in lens.items():
        plan[name] = plan[name][:ln]
    nnz = int(plan["col_ptr"][m])
    plan["col_row"], plan["col_slot"] = plan["col_row"][:nnz], plan["col_slot"][:nnz]
    nd = int(plan["dtr_ptr"][m])
    plan["dtr_slot"], plan["dtr_p"] = plan["dtr_slot"][:nd], plan["dtr_p"][:nd]
    nt = int(plan["task_tr_ptr"][T])
    plan["tr_a"], plan["tr_b"] = plan["tr_a"][:nt], plan["tr_b"][:nt]
    plan["asm_edge"] = plan["asm_edge"][:int(plan["asm_ptr"][S])]
    plan["g_edge"] = plan["g_edge"][:int(plan["g_ptr"][m])]
    return plan


# ------------------------------------------------------------------ checks --
def _check(t: torch.Tensor, name: str, dtype=None):
    if not isinstance(t, torch.Tensor):
        raise RuntimeError(f"{name} must be a tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name} must be on a ROCm device (got {t.device}); no CPU path")
    if dtype is not None and t.dtype not in (dtype if isinstance(dtype, tuple) else (dtype,)):
        raise RuntimeError(f"{name} must be {dtype} (got {t.dtype})")


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _raise(rc, fn):
    if rc == M3S_OK:
        return
    msg = {M3S_EINVAL: "invalid argument", M3S_ELAUNCH: "HIP launch failed",
           M3S_ETOOLARGE: "problem size exceeds this build's limits"}.get(rc, f"error {rc}")
    raise RuntimeError(f"{fn}: {msg}")


def _workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=device)


def make_gn_args(mode, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, K=None, *, sigma_a=0.0,
                 sigma_b=0.0, C_thresh=0.0, Q_thresh=0.0, height=0, width=0, pixel_border=0,
                 z_eps=0.0, max_iter=0, delta_thresh=0.0, dx=None, info=None, workspace=None):
    """Validate reference-layout tensors and fill an ``m3s_gn_args``. Returns
    (args, keepalive) — keepalive holds every tensor the struct points to."""
    _check(Twc, "Twc", torch.float32)
    _check(Xs, "Xs", torch.float32)
    _check(Cs, "Cs", torch.float32)
    if K is not None:
        _check(K, "K", torch.float32)
    _check(ii, "ii", torch.int64)
    _check(jj, "jj", torch.int64)
    # int64 as the reference passes it; int32 from the device edge store
    _check(idx_ii2jj, "idx_ii2jj", (torch.int64, torch.int32))
    _check(valid_match, "valid_match", torch.bool)
    _check(Q, "Q", torch.float32)
    N, HW = int(Xs.shape[0]), int(Xs.shape[1])
    E = int(ii.shape[0])
    if Xs.dim() != 3 or Xs.shape[2] != 3:
        raise RuntimeError("Xs must be [N, HW, 3]")
    if Twc.numel() != 8 * N:
        raise RuntimeError(f"Twc must be [N, 8] with N = Xs.size(0) = {N}")
    if Cs.numel() != N * HW:
        raise RuntimeError("Cs must be [N, HW, 1]")
    if jj.numel() != E or idx_ii2jj.numel() != E * HW or valid_match.numel() != E * HW or Q.numel() != E * HW:
        raise RuntimeError("edge tensors must be [E, HW(,1)] with E = ii.size(0)")
    dev = Xs.device
    # no fill launches: m3s_gn_prepare zeroes dx and uploads info on the stream
    if dx is None:
        dx = torch.empty(max(N - 1, 0), 7, dtype=torch.float32, device=dev)
    if info is None:
        info = torch.empty(8, dtype=torch.int32, device=dev)
    ws_bytes = int(_lib.m3s_gn_workspace_size(N, HW, E))
    if workspace is None or workspace.numel() < ws_bytes:
        workspace = _workspace(ws_bytes, dev)
    a = GnArgs()
    a.Twc, a.Xs, a.Cs, a.ii, a.jj = _p(Twc), _p(Xs), _p(Cs), _p(ii), _p(jj)
    a.idx_ii2jj, a.valid_match, a.Q, a.K = _p(idx_ii2jj), _p(valid_match), _p(Q), _p(K)
    a.idx_i32 = 1 if idx_ii2jj.dtype == torch.int32 else 0
    a.N, a.HW, a.E, a.mode = N, HW, E, mode
    a.sigma_a, a.sigma_b = float(sigma_a), float(sigma_b)
    a.C_thresh, a.Q_thresh = float(C_thresh), float(Q_thresh)
    a.height, a.width, a.pixel_border = int(height), int(width), int(pixel_border)
    a.z_eps = float(z_eps)
    a.max_iter, a.delta_thresh = int(max_iter), float(delta_thresh)
    a.dx_out, a.info = _p(dx), _p(info)
    a.workspace, a.workspace_bytes = _p(workspace), workspace.numel()
    keep = dict(Twc=Twc, Xs=Xs, Cs=Cs, ii=ii, jj=jj, idx=idx_ii2jj, valid=valid_match, Q=Q, K=K,
                dx=dx, info=info, workspace=workspace)
    return a, keep


def _run_gn(fn_name, a, keep):
    st = _stream(keep["Xs"].device)
    rc = getattr(_lib, fn_name)(ctypes.byref(a), st)
    # the per-call workspace goes back to the caching allocator: drop its host
    # state too (m3s_gn_release: no stream sync; the call returns as soon as
    # its launches are queued)
    rc_rel = _lib.m3s_gn_release(ctypes.byref(a), st)
    _raise(rc, fn_name)
    _raise(rc_rel, "m3s_gn_release")
    return [keep["dx"]]


# ------------------------------------------------- reference entry points --
def gauss_newton_points(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, sigma_point, C_thresh,
                        Q_thresh, max_iter, delta_thresh, *, info=None):
    """gn.cpp:3-27 / gn_kernels.cu:725-811."""
    a, keep = make_gn_args(MODE_POINTS, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q,
                           sigma_a=sigma_point, C_thresh=C_thresh, Q_thresh=Q_thresh,
                           max_iter=max_iter, delta_thresh=delta_thresh, info=info)
    return _run_gn("m3s_gauss_newton_points", a, keep)


def gauss_newton_rays(Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, sigma_ray, sigma_dist,
                      C_thresh, Q_thresh, max_iter, delta_thresh, *, info=None):
    """gn.cpp:29-54 / gn_kernels.cu:1140-1228."""
    a, keep = make_gn_args(MODE_RAYS, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q,
                           sigma_a=sigma_ray, sigma_b=sigma_dist, C_thresh=C_thresh,
                           Q_thresh=Q_thresh, max_iter=max_iter, delta_thresh=delta_thresh,
                           info=info)
    return _run_gn("m3s_gauss_newton_rays", a, keep)


def gauss_newton_calib(Twc, Xs, Cs, K, ii, jj, idx_ii2jj, valid_match, Q, height, width,
                       pixel_border, z_eps, sigma_pixel, sigma_depth, C_thresh, Q_thresh, max_iter,
                       delta_thresh, *, info=None):
    """gn.cpp:56-85 / gn_kernels.cu:1546-1638."""
    a, keep = make_gn_args(MODE_CALIB, Twc, Xs, Cs, ii, jj, idx_ii2jj, valid_match, Q, K,
                           sigma_a=sigma_pixel, sigma_b=sigma_depth, C_thresh=C_thresh,
                           Q_thresh=Q_thresh, height=height, width=width,
                           pixel_border=pixel_border, z_eps=z_eps, max_iter=max_iter,
                           delta_thresh=delta_thresh, info=info)
    return _run_gn("m3s_gauss_newton_calib", a, keep)


def iter_proj(rays_img_with_grad, pts_3d_norm, p_init, max_iter, lambda_init, cost_thresh):
    """gn.cpp:84-99 / matching_kernels.cu:119-296: per-pixel LM projection.

    rays_img_with_grad [B,H,W,9] f32, pts_3d_norm [B,N,3] f32, p_init [B,N,2]
    f32 -> [p_new [B,N,2] f32, converged [B,N] bool] (new tensors)."""
    for name, t in (("rays_img_with_grad", rays_img_with_grad), ("pts_3d_norm", pts_3d_norm),
                    ("p_init", p_init)):
        _check(t, name, torch.float32)
    B, H, W, C = rays_img_with_grad.shape
    Bn, N = int(p_init.shape[0]), int(p_init.shape[1])
    if C != 9 or Bn != B or tuple(pts_3d_norm.shape) != (B, N, 3) or tuple(p_init.shape) != (B, N, 2):
        raise RuntimeError("iter_proj: expected rays [B,H,W,9], pts_3d_norm [B,N,3], p_init [B,N,2]")
    dev = p_init.device
    p_new = torch.zeros(B, N, 2, dtype=torch.float32, device=dev)
    converged = torch.zeros(B, N, dtype=torch.bool, device=dev)
    a = IterProjArgs()
    a.rays_img, a.pts_3d_norm, a.p_init = _p(rays_img_with_grad), _p(pts_3d_norm), _p(p_init)
    a.B, a.H, a.W, a.N = B, H, W, N
    a.max_iter, a.lambda_init, a.cost_thresh = int(max_iter), float(lambda_init), float(cost_thresh)
    a.p_new, a.converged = _p(p_new), _p(converged)
    _raise(_lib.m3s_iter_proj(ctypes.byref(a), _stream(dev)), "m3s_iter_proj")
    return [p_new, converged]


def refine_matches(D11, D21, p1, radius, dilation_max):
    """gn.cpp:101-114 / matching_kernels.cu:25-116: dilated local search.

    D11 [B,H,W,F] f16 (or f32), D21 [B,N,F] same dtype, p1 [B,N,2] int64 (u, v)
    -> [p1_new [B,N,2] int64] (new tensor)."""
    _check(D11, "D11")
    _check(D21, "D21", D11.dtype)
    _check(p1, "p1", torch.int64)
    dt = {torch.float16: 0, torch.float32: 1}.get(D11.dtype)
    if dt is None:
        raise RuntimeError(f"refine_matches: descriptors must be float16 or float32 (got {D11.dtype})")
    B, H, W, F = D11.shape
    N = int(p1.shape[1])
    if tuple(D21.shape) != (B, N, F) or tuple(p1.shape) != (B, N, 2):
        raise RuntimeError("refine_matches: expected D11 [B,H,W,F], D21 [B,N,F], p1 [B,N,2]")
    p1_new = torch.zeros(B, N, 2, dtype=torch.int64, device=p1.device)
    a = RefineArgs()
    a.D11, a.D21, a.p1 = _p(D11), _p(D21), _p(p1)
    a.B, a.H, a.W, a.N, a.F = B, H, W, N, F
    a.dtype, a.radius, a.dilation_max = dt, int(radius), int(dilation_max)
    a.p1_new = _p(p1_new)
    _raise(_lib.m3s_refine_matches(ctypes.byref(a), _stream(p1.device)), "m3s_refine_matches")
    return [p1_new]


def fuse_pointmap(X_canon, C, X_new, C_new, T=None, mode="weighted_pointmap"):
    """Keyframe pointmap fusion after tracking, in place (new entry point):
    X_canon/C <- filter(X_canon, C, T.act(X_new), C_new) — tracker.py:98-99 +
    Frame.update_pointmap (frame.py:41-100) for an initialised keyframe.
    X_canon, X_new [HW,3] f32; C, C_new [HW,1] (or [HW]) f32; T [8] or [1,8]."""
    _check(X_canon, "X_canon", torch.float32)
    _check(C, "C", torch.float32)
    _check(X_new, "X_new", torch.float32)
    _check(C_new, "C_new", torch.float32)
    if mode not in FILTER_MODES:
        raise RuntimeError(f"fuse_pointmap: unsupported filtering mode {mode!r}")
    HW = int(X_canon.shape[0])
    if X_canon.numel() != 3 * HW or X_new.numel() != 3 * HW or C.numel() != HW or C_new.numel() != HW:
        raise RuntimeError("fuse_pointmap: expected X [HW,3] and C [HW,1]")
    if T is not None:
        T = T.contiguous()
        _check(T, "T", torch.float32)
    a = FuseArgs()
    a.X_canon, a.C, a.X_new, a.C_new, a.T = _p(X_canon), _p(C), _p(X_new), _p(C_new), _p(T)
    a.HW, a.mode = HW, FILTER_MODES[mode]
    _raise(_lib.m3s_fuse_pointmap(ctypes.byref(a), _stream(X_canon.device)), "m3s_fuse_pointmap")


def prep_rays(X11, X21):
    """iter_proj inputs in one pass (new entry point; prep_for_iter_proj,
    matching.py:25-49): X11 [B,H,W,3], X21 [B,H,W,3] (or [B,HW,3]) f32 ->
    (rays_with_grad [B,H,W,9], pts3d_norm [B,HW,3])."""
    _check(X11, "X11", torch.float32)
    _check(X21, "X21", torch.float32)
    B, H, W, _ = X11.shape
    if X21.numel() != B * H * W * 3:
        raise RuntimeError("prep_rays: X21 must hold B*H*W points")
    dev = X11.device
    rays = torch.empty(B, H, W, 9, dtype=torch.float32, device=dev)
    pts = torch.empty(B, H * W, 3, dtype=torch.float32, device=dev)
    a = PrepRaysArgs()
    a.X11, a.X21, a.B, a.H, a.W, a.rays_img, a.pts_norm = _p(X11), _p(X21), B, H, W, _p(rays), _p(pts)
    _raise(_lib.m3s_prep_rays(ctypes.byref(a), _stream(dev)), "m3s_prep_rays")
    return rays, pts


# ------------------------------------------------------------ tracker ---
def _track(fn, Xf, Xk, T_WCf, T_WCk, Qk, valid, K, img_size, sigma_a, sigma_b, huber_k,
           max_iters, rel_error, delta_norm, pixel_border=0, z_eps=0.0, sync_every=5, workspace=None):
    _check(Xf, "Xf", torch.float32)
    _check(Xk, "Xk", torch.float32)
    _check(Qk, "Qk", torch.float32)
    _check(valid, "valid", torch.bool)
    T_WCf = T_WCf.contiguous()
    T_WCk = T_WCk.contiguous()
    _check(T_WCf, "T_WCf", torch.float32)
    _check(T_WCk, "T_WCk", torch.float32)
    if K is not None:
        _check(K, "K", torch.float32)
    HW = int(Xk.shape[0])
    if Xf.numel() != 3 * HW or Xk.numel() != 3 * HW or Qk.numel() != HW or valid.numel() != HW:
        raise RuntimeError("tracker inputs must be Xf/Xk [HW,3], Qk/valid [HW,1]")
    dev = Xk.device
    out_f = torch.empty(1, 8, dtype=torch.float32, device=dev)
    out_r = torch.empty(1, 8, dtype=torch.float32, device=dev)
    info = torch.zeros(8, dtype=torch.int32, device=dev)
    need = _lib.m3s_track_workspace_size(HW)
    if workspace is None:
        ws = _workspace(need, dev)
    else:  # caller-owned (tests: reused / poisoned workspaces)
        _check(workspace, "workspace", torch.uint8)
        if workspace.device != dev or workspace.numel() < need:
            raise RuntimeError(f"tracker workspace must be a uint8 tensor of >= {need} bytes on {dev}")
        ws = workspace
    a = TrackArgs()
    a.Xf, a.Xk, a.Qk, a.valid = _p(Xf), _p(Xk), _p(Qk), _p(valid)
    a.T_WCf, a.T_WCk, a.K = _p(T_WCf), _p(T_WCk), _p(K)
    a.HW = HW
    h, w = (int(img_size[0]), int(img_size[1])) if img_size is not None else (0, 0)
    a.height, a.width, a.pixel_border, a.z_eps = h, w, int(pixel_border), float(z_eps)
    a.sigma_a, a.sigma_b, a.huber_k = float(sigma_a), float(sigma_b), float(huber_k)
    a.max_iters, a.rel_error, a.delta_norm = int(max_iters), float(rel_error), float(delta_norm)
    a.sync_every = int(sync_every)
    a.T_WCf_out, a.T_CkCf_out, a.info = _p(out_f), _p(out_r), _p(info)
    a.workspace, a.workspace_bytes = _p(ws), ws.numel()
    rc = getattr(_lib, fn)(ctypes.byref(a), _stream(dev))
    _raise(rc, fn)
    del ws  # stream-ordered by the caching allocator
    return out_f, out_r, info


def track_workspace_size(HW):
    """Bytes of the tracker workspace for an image of HW pixels."""
    return int(_lib.m3s_track_workspace_size(int(HW)))


def track_rays_sim3(Xf, Xk, T_WCf, T_WCk, Qk, valid, sigma_ray, sigma_dist, huber_k, max_iters,
                    rel_error, delta_norm, sync_every=5, workspace=None):
    """Device form of FrameTracker.opt_pose_ray_dist_sim3 (tracker.py:173-214).
    Returns (T_WCf [1,8], T_CkCf [1,8], info int32[8]); info[1] != 0 means the
    Cholesky failed (the reference raises; tracker.py:91-93)."""
    return _track("m3s_track_rays_sim3", Xf, Xk, T_WCf, T_WCk, Qk, valid, None, None, sigma_ray,
                  sigma_dist, huber_k, max_iters, rel_error, delta_norm, sync_every=sync_every,
                  workspace=workspace)


def track_calib_sim3(Xf, Xk, T_WCf, T_WCk, Qk, valid, K, img_size, sigma_pixel, sigma_depth,
                     huber_k, max_iters, rel_error, delta_norm, pixel_border, z_eps, sync_every=5,
                     workspace=None):
    """Device form of FrameTracker.opt_pose_calib_sim3 (tracker.py:216-266);
    Xf/Xk already constrained to rays, meas_k formed on device."""
    return _track("m3s_track_calib_sim3", Xf, Xk, T_WCf, T_WCk, Qk, valid, K, img_size,
                  sigma_pixel, sigma_depth, huber_k, max_iters, rel_error, delta_norm,
                  pixel_border=pixel_border, z_eps=z_eps, sync_every=sync_every, workspace=workspace)


# -------------------------------------------------- stepwise (sharded) ---
def gn_prepare(a, keep):
    _raise(_lib.m3s_gn_prepare(ctypes.byref(a), _stream(keep["Xs"].device)), "m3s_gn_prepare")


def gn_linearize(a, keep, edge_begin, edge_end, edge_sums):
    _check(edge_sums, "edge_sums", torch.float64)
    rc = _lib.m3s_gn_linearize(ctypes.byref(a), int(edge_begin), int(edge_end), _p(edge_sums),
                               _stream(keep["Xs"].device))
    _raise(rc, "m3s_gn_linearize")


def gn_release(a, keep):
    _raise(_lib.m3s_gn_release(ctypes.byref(a), _stream(keep["Xs"].device)), "m3s_gn_release")


def gn_solve(a, keep, edge_sums):
    _check(edge_sums, "edge_sums", torch.float64)
    rc = _lib.m3s_gn_solve(ctypes.byref(a), _p(edge_sums), _stream(keep["Xs"].device))
    _raise(rc, "m3s_gn_solve")
