/*
 * m3s_gn.h — C ABI of the MI355X Gauss-Newton backend for MASt3R-SLAM.
 *
 * Drop-in for the reference's `mast3r_slam_backends` GN entry points
 * (pybind module, /root/reference/mast3r_slam/backend/src/gn.cpp:116-122,
 * declarations gn.h:11-80). Everything here is plain C: device pointers,
 * sizes, a hipStream_t passed as `void *`, an int status. No torch types.
 *
 * Layouts are exactly the reference's tensors (all contiguous, device memory):
 *   Twc        float  [N, 8]      t(3) q(xyzw) s      — updated IN PLACE
 *   Xs         float  [N, HW, 3]  canonical pointmaps (rank order)
 *   Cs         float  [N, HW]     (the reference's [N, HW, 1]) average conf
 *   ii, jj     int64  [E]         global keyframe ids of each directed edge
 *   idx_ii2jj  int64  [E, HW]     pixel of KF ii matched to pixel k of KF jj
 *                                 (int32 when idx_i32 = 1)
 *   valid_match uint8 [E, HW]     (torch.bool, [E, HW, 1] in the reference)
 *   Q          float  [E, HW]     match quality
 *   K          float  [3, 3]      calib only
 * ii/jj are remapped to ranks in sorted-unique(cat(ii, jj)) as the reference
 * does (gn_kernels.cu:161-170); pose rank 0 is held fixed (num_fix = 1,
 * gn_kernels.cu:1157).
 *
 * Per solve call the host reads ii/jj once (like the reference's _unique /
 * searchsorted) to rank them and to build the block-sparse LLT plan; every GN
 * iteration after that is launched asynchronously on `stream` with no host
 * synchronisation. Nothing is allocated (the caller passes a workspace of
 * m3s_gn_workspace_size() bytes, 256-byte aligned). Device-side outcomes
 * (iterations run, solve failures, invalid edge ids) land in `info`.
 */
#ifndef M3S_GN_H
#define M3S_GN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* return codes (host side) */
#define M3S_OK 0
#define M3S_EINVAL 1     /* bad sizes / null pointers / workspace too small */
#define M3S_ELAUNCH 2    /* a HIP launch failed */
#define M3S_ETOOLARGE 3  /* problem size beyond this build's limits */

/* residual models (gn_kernels.cu kernels) */
#define M3S_MODE_POINTS 0 /* point_align_kernel  :455-723  */
#define M3S_MODE_RAYS 1   /* ray_align_kernel    :813-1138 */
#define M3S_MODE_CALIB 2  /* calib_proj_kernel   :1231-1543 */

/* device-side info block, int32[8], written by the GN launches */
#define M3S_INFO_ITERS 0        /* GN iterations executed                     */
#define M3S_INFO_SOLVE_FAIL 1   /* iterations whose LLT failed (dx = 0 then)   */
#define M3S_INFO_BAD_EDGE 2     /* 1 if an edge id maps to a rank >= N         */
#define M3S_INFO_CONVERGED 3    /* 1 if ||dx|| < delta_thresh stopped the loop */
#define M3S_INFO_N_UNIQUE 4     /* number of unique keyframe ids in ii/jj      */

typedef struct m3s_gn_args {
  float *Twc;
  const float *Xs;
  const float *Cs;
  const int64_t *ii;
  const int64_t *jj;
  const int64_t *idx_ii2jj;
  const uint8_t *valid_match;
  const float *Q;
  const float *K; /* calib only, else NULL */
  int64_t N, HW, E;
  int mode;
  /* residual parameters: points: sigma_a = sigma_point
   *                      rays:   sigma_a = sigma_ray,   sigma_b = sigma_dist
   *                      calib:  sigma_a = sigma_pixel, sigma_b = sigma_depth */
  float sigma_a, sigma_b;
  float C_thresh, Q_thresh;
  int height, width, pixel_border; /* calib */
  float z_eps;                     /* calib */
  int max_iter;
  float delta_thresh;
  float *dx_out;  /* [N-1, 7] float: the last GN step (the reference's return) */
  int32_t *info;  /* [8] int32 device */
  void *workspace;
  size_t workspace_bytes;
  /* 0: idx_ii2jj is the reference's int64 [E, HW]; 1: it holds int32 (the
   * device edge store of mast3r_slam_amd.factor_graph: 4 B less per edge
   * pixel on the first GN iteration's reads) */
  int idx_i32;
} m3s_gn_args;

/* Bytes of scratch the GN entry points need for this problem size. */
size_t m3s_gn_workspace_size(int64_t N, int64_t HW, int64_t E);

/* Replaces gauss_newton_points (gn.cpp:3-27 -> gn_kernels.cu:725-811). */
int m3s_gauss_newton_points(const m3s_gn_args *a, void *stream);
/* Replaces gauss_newton_rays   (gn.cpp:29-54 -> gn_kernels.cu:1140-1228). */
int m3s_gauss_newton_rays(const m3s_gn_args *a, void *stream);
/* Replaces gauss_newton_calib  (gn.cpp:56-85 -> gn_kernels.cu:1546-1638). */
int m3s_gauss_newton_calib(const m3s_gn_args *a, void *stream);

/* ---- stepwise API (edge-sharded multi-GPU path; same math as above) ----
 * m3s_gn_prepare:   one prologue kernel ranks ii/jj on the device, writes the
 *                   task table, zeroes info/flags/dx_out and copies the ids to
 *                   pinned host memory; no stream synchronisation. The host
 *                   reads the ids when it first needs them (the first solve,
 *                   or a linearize of a sub-range: it then waits for the
 *                   prologue only) to fetch or build the sparse plan, which is
 *                   uploaded on a side stream while the first linearize runs.
 *                   E > 2048 (or knob prologue = 0): the host prepare, with
 *                   one stream synchronisation.
 * m3s_gn_linearize: per-edge local normal equations for edges
 *                   [edge_begin, edge_end) into edge_sums (double[E_loc][36]:
 *                   28 upper-triangular J^T W J, 7 J^T W r, 1 cost, in the
 *                   frame of the residual).
 * m3s_gn_solve:     given edge_sums for ALL E edges: assemble the
 *                   (N-1)*7 system, fp64 LLT, dx = -H^-1 g, retract Twc, update
 *                   info/convergence flag. Iterations after convergence are
 *                   skipped on device. */
int m3s_gn_prepare(const m3s_gn_args *a, void *stream);
int m3s_gn_linearize(const m3s_gn_args *a, int64_t edge_begin, int64_t edge_end,
                     double *edge_sums, void *stream);
int m3s_gn_solve(const m3s_gn_args *a, const double *edge_sums, void *stream);
/* m3s_gn_release:   drop the host-side state m3s_gn_prepare keyed by
 *                   a->workspace (no synchronisation: queued uploads read the
 *                   library's pinned staging, never this state). Call it
 *                   before the workspace is freed or reused for another
 *                   problem; the gauss_newton_* wrappers of mast3r_slam_backends
 *                   do. */
int m3s_gn_release(const m3s_gn_args *a, void *stream);
#define M3S_EDGE_SUM_STRIDE 36

/* ---- tracker (new entry points; the reference tracker is pure PyTorch,
 *      tracker.py:173-266) ----
 * Frame -> keyframe relative Sim(3) GN with the reference's convergence rule
 * (nonlinear_optimizer.py:5-25). Inputs are the tensors opt_pose_* receive:
 *   Xf [HW,3] (frame points gathered by idx_f2k), Xk [HW,3], Qk [HW],
 *   valid [HW] uint8, T_WCf / T_WCk [8]; calib additionally K [3,3] and the
 *   image size (meas_k is formed on device from the pixel grid and Xk).
 * Outputs: T_WCf_out [8], T_CkCf_out [8], info [8] (ITERS, SOLVE_FAIL=1 if
 * the Cholesky failed — the reference raises, tracker.py:91-93). */
typedef struct m3s_track_args {
  const float *Xf;
  const float *Xk;
  const float *Qk;
  const uint8_t *valid;
  const float *T_WCf;
  const float *T_WCk;
  const float *K; /* calib only */
  int64_t HW;
  int height, width, pixel_border;
  float z_eps;
  float sigma_a, sigma_b; /* (sigma_ray, sigma_dist) or (sigma_pixel, sigma_depth) */
  float huber_k;          /* config tracking.huber (1.345) */
  int max_iters;
  float rel_error, delta_norm;
  int sync_every; /* 0: launch all max_iters (device-side early exit);
                     k>0: read the convergence flag every k iterations */
  float *T_WCf_out;
  float *T_CkCf_out;
  int32_t *info;
  void *workspace;
  size_t workspace_bytes;
} m3s_track_args;

size_t m3s_track_workspace_size(int64_t HW);
int m3s_track_rays_sim3(const m3s_track_args *a, void *stream);
int m3s_track_calib_sim3(const m3s_track_args *a, void *stream);

/* build identification (for the loaded-library check) */
const char *m3s_version(void);

/* Diagnostic: the host symbolic plan of the block-sparse LLT for N poses and
 * edge ranks (ri, rj) (pose rank 0 fixed); split > 0 cuts update lists longer
 * than split into PART items (at most max_parts, widening split to fit), as
 * the solver does for factors that live in global memory. Writes the
 * flattened int32 plan to out (if cap suffices) and meta[0..34] = {m, S,
 * levels, 31 section offsets in the order of m3s_symbolic.h, n_parts}.
 * Returns the plan length in int32 words. */
int64_t m3s_sparse_plan_debug(int32_t N, int64_t E, const int32_t *ri, const int32_t *rj, int32_t split,
                              int32_t max_parts, int32_t *out, int64_t cap, int32_t *meta);

/* Diagnostic: byte offsets of the workspace sections for (N, HW, E), in the
 * order flags, rank_i, rank_j, first, partials, edge_sums, A, fin, plan, Lblk,
 * Dinv, tail, tasks, planes, total (offs[15]). Returns the total. */
size_t m3s_gn_layout_debug(int64_t N, int64_t HW, int64_t E, size_t *offs);
/* instrumented builds only: which = 0 persistent-tracker phase stamps
 * [2][16][8] (-DM3S_TRK_STAMPS), 1 column-task stamps [4][2048][4]
 * (-DM3S_COL_STAMPS); wall-clock ticks. 1 if present, 0 otherwise
 * (tools/trk_stamps.py, tools/col_stamps.py) */
int m3s_debug_stamps(int which, int64_t *out);
/* Diagnostic (tests/test_gpu_sim3.py): the device Sim(3) helpers of the hot
 * path (csrc/m3s_device.h; lietorch semantics, gn_kernels.cu:172-413) on n
 * elements, asynchronously on `stream`. Device arrays; Sim3 = 8 floats
 * (t, q_xyzw, s), tangent = 7 floats (tau, phi, sigma), point = 3 floats.
 *   op 0 exp(a: tangent)            -> out Sim3      (expSim3 :323-390)
 *   op 1 retract(a: tangent, b: T)  -> out Exp(a) b  (retrSim3 :392-413), the
 *        backend's retraction: evaluated in fp64, rounded once
 *   op 2 compose(a, b)              -> out a * b
 *   op 3 inverse(a)                 -> out a^-1
 *   op 4 relative(a, b)             -> out a^-1 b    (relSim3 :252-272)
 *   op 5 act(a, b: point)           -> out point     (actSim3 :207-219)
 *   op 6 act as the 3x4 matrix form the linearize kernels use -> out point
 *   op 7 Adj(a)^-T as a row-major 7x7 (apply_Sim3_adj_inv :274-297) -> out 49
 *   op 8 retract as op 1 in the reference's fp32 arithmetic (the tracker's) */
int m3s_debug_sim3(int op, const float *a, const float *b, float *out, int64_t n, void *stream);
/* Solver knobs (experiments / A/B tests). Defaults are the measured best;
 * the environment (M3S_PLAN_CACHE, M3S_DENSE, M3S_DENSE_TAIL_MIN, M3S_COLS,
 * M3S_DF, M3S_TAIL_CYC, M3S_TAIL_MFMA, M3S_BORDER_SPLIT,
 * M3S_TRACK_PERSISTENT, M3S_PROLOGUE) is read once per process; this sets a
 * knob at run time for the calls that follow. Names: plan_cache, dense,
 * dense_tail_min, cols, df, tail_cyc, tail_mfma, border_split,
 * track_persistent, prologue (0: host-side prepare),
 * debug_drop_item (test hook: drop one dispatch item of the one-workgroup
 * LLT so its bounded waits time out). Returns the previous value, or
 * -2^30 for an unknown name. */
int m3s_set_knob(const char *name, int value);
/* Diagnostic (bench.py's measured HBM ceiling): copy nbytes (a multiple of
 * 16, 16-B aligned device pointers) with 16-B non-temporal loads and stores,
 * `blocks` workgroups of 256 lanes, asynchronously on `stream`. */
int m3s_debug_copy(const void *src, void *dst, int64_t nbytes, int blocks, void *stream);
/* Diagnostic (bench.py's roofline leg): in-call launch timing. enable != 0
 * makes every following drop-in call record timing events on its stream
 * around each iteration's linearize launch and solve launches (and resets
 * the record); m3s_debug_call_times waits for the last event and returns
 * the recorded spans in launch order (ms[k], kinds[k]: 0 first-iteration
 * gathering linearize, 1 packed linearize, 2 solve), at most cap of them;
 * the return value is the number of spans (or a negative status). The
 * record is cleared after reading. Linearize spans are the dispatch's own
 * begin / end timestamps: the call launches each linearize through
 * hipExtLaunchKernel with a start / stop event pair (round 4: events recorded
 * around the launch read 6-12% above the kernel trace). A small graph's solve
 * (one sparse_llt_kernel launch) is timed the same way (round 6: the events
 * around it read ~19% above the trace). A linearize that does not go through
 * that launch (the non-vectorised first iteration) and a large graph's
 * multi-launch solve use the events recorded around the launches. */
int m3s_debug_call_timing(int enable);
int m3s_debug_call_times(float *ms, int32_t *kinds, int cap);

#ifdef __cplusplus
}
#endif
#endif /* M3S_GN_H */
