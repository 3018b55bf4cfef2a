// m3s_device.h — device helpers for the MI355X GN path: Sim(3) algebra,
// residual-row builders, packed normal-equation accumulation.
//
// Sim(3) algebra follows the reference's CUDA helpers (lietorch semantics):
//   quaternion xyzw product / rotation  gn_kernels.cu:177-205
//   relative pose T_i^-1 T_j            gn_kernels.cu:252-272
//   Exp / left retraction               gn_kernels.cu:299-413
// The Jacobian design differs from the reference on purpose: the reference
// builds the 14-wide [J_i, J_j] row per pixel and accumulates the 105-entry
// upper triangle of [J_i J_j]^T W [J_i J_j] (gn_kernels.cu:990-1089). Since
// J_j = M(T_i) J_local and J_i = -J_j exactly (:999-1000), every block of the
// 14x14 matrix is +-M L M^T with L = sum w J_local J_local^T. We accumulate
// only L (28 entries, and only the structurally non-zero ones per row) and
// the 7-vector l = sum w e J_local, and apply M once per edge in fp64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace m3s {

constexpr int kNP = 36;  // per-edge partial: 28 (upper-tri L) + 7 (l) + 1 (cost)
constexpr int kL = 0, kG = 28, kCost = 35;

// packed upper-triangular index of (m, n), m <= n < 7
__host__ __device__ constexpr int tri(int m, int n) { return m * 7 - (m * (m - 1)) / 2 + (n - m); }

// ------------------------------------------------------------------ Sim3 --
struct Sim3f {
  float t[3];
  float q[4];  // x y z w
  float s;
};

__device__ __forceinline__ Sim3f load_sim3(const float *p) {
  Sim3f T;
  T.t[0] = p[0], T.t[1] = p[1], T.t[2] = p[2];
  T.q[0] = p[3], T.q[1] = p[4], T.q[2] = p[5], T.q[3] = p[6];
  T.s = p[7];
  return T;
}

__device__ __forceinline__ void store_sim3(float *p, const Sim3f &T) {
  p[0] = T.t[0], p[1] = T.t[1], p[2] = T.t[2];
  p[3] = T.q[0], p[4] = T.q[1], p[5] = T.q[2], p[6] = T.q[3];
  p[7] = T.s;
}

__device__ __forceinline__ void quat_mul(const float *a, const float *b, float *o) {
  const float x = a[3] * b[0] + a[0] * b[3] + a[1] * b[2] - a[2] * b[1];
  const float y = a[3] * b[1] - a[0] * b[2] + a[1] * b[3] + a[2] * b[0];
  const float z = a[3] * b[2] + a[0] * b[1] - a[1] * b[0] + a[2] * b[3];
  const float w = a[3] * b[3] - a[0] * b[0] - a[1] * b[1] - a[2] * b[2];
  o[0] = x, o[1] = y, o[2] = z, o[3] = w;
}

// R(q) X = X + 2w (v x X) + v x (2 v x X)
__device__ __forceinline__ void quat_rot(const float *q, const float *X, float *Y) {
  const float ux = 2.0f * (q[1] * X[2] - q[2] * X[1]);
  const float uy = 2.0f * (q[2] * X[0] - q[0] * X[2]);
  const float uz = 2.0f * (q[0] * X[1] - q[1] * X[0]);
  const float y0 = X[0] + q[3] * ux + (q[1] * uz - q[2] * uy);
  const float y1 = X[1] + q[3] * uy + (q[2] * ux - q[0] * uz);
  const float y2 = X[2] + q[3] * uz + (q[0] * uy - q[1] * ux);
  Y[0] = y0, Y[1] = y1, Y[2] = y2;
}

__device__ __forceinline__ void act(const Sim3f &T, const float *X, float *Y) {
  quat_rot(T.q, X, Y);
  Y[0] = Y[0] * T.s + T.t[0];
  Y[1] = Y[1] * T.s + T.t[1];
  Y[2] = Y[2] * T.s + T.t[2];
}

// Y = s R(q) X + t as a 3x4 matrix: 9 FMAs per point instead of the
// quaternion form's ~24 operations (same map; rounding differs at the ulp level).
struct Sim3Mat {
  float m[9], t[3];
};
__device__ __forceinline__ Sim3Mat sim3_matrix(const Sim3f &T) {
  const float x = T.q[0], y = T.q[1], z = T.q[2], w = T.q[3], s = T.s;
  Sim3Mat M;
  M.m[0] = s * (1.0f - 2.0f * (y * y + z * z));
  M.m[1] = s * (2.0f * (x * y - z * w));
  M.m[2] = s * (2.0f * (x * z + y * w));
  M.m[3] = s * (2.0f * (x * y + z * w));
  M.m[4] = s * (1.0f - 2.0f * (x * x + z * z));
  M.m[5] = s * (2.0f * (y * z - x * w));
  M.m[6] = s * (2.0f * (x * z - y * w));
  M.m[7] = s * (2.0f * (y * z + x * w));
  M.m[8] = s * (1.0f - 2.0f * (x * x + y * y));
  M.t[0] = T.t[0], M.t[1] = T.t[1], M.t[2] = T.t[2];
  return M;
}
__device__ __forceinline__ void act(const Sim3Mat &M, const float *X, float *Y) {
  // rows 0 and 1 as one float2 chain (v_pk_fma_f32), row 2 scalar
  typedef float v2 __attribute__((ext_vector_type(2)));
  v2 y = __builtin_elementwise_fma(v2{M.m[2], M.m[5]}, v2{X[2], X[2]}, v2{M.t[0], M.t[1]});
  y = __builtin_elementwise_fma(v2{M.m[1], M.m[4]}, v2{X[1], X[1]}, y);
  y = __builtin_elementwise_fma(v2{M.m[0], M.m[3]}, v2{X[0], X[0]}, y);
  Y[0] = y.x, Y[1] = y.y;
  Y[2] = __builtin_fmaf(M.m[6], X[0], __builtin_fmaf(M.m[7], X[1], __builtin_fmaf(M.m[8], X[2], M.t[2])));
}

__device__ __forceinline__ Sim3f inverse(const Sim3f &T) {
  Sim3f R;
  R.q[0] = -T.q[0], R.q[1] = -T.q[1], R.q[2] = -T.q[2], R.q[3] = T.q[3];
  R.s = 1.0f / T.s;
  float d[3];
  quat_rot(R.q, T.t, d);
  R.t[0] = -R.s * d[0], R.t[1] = -R.s * d[1], R.t[2] = -R.s * d[2];
  return R;
}

// A * B
__device__ __forceinline__ Sim3f compose(const Sim3f &A, const Sim3f &B) {
  Sim3f C;
  quat_mul(A.q, B.q, C.q);
  float d[3];
  quat_rot(A.q, B.t, d);
  C.t[0] = A.t[0] + A.s * d[0];
  C.t[1] = A.t[1] + A.s * d[1];
  C.t[2] = A.t[2] + A.s * d[2];
  C.s = A.s * B.s;
  return C;
}

// T_i^-1 T_j  (relSim3, gn_kernels.cu:252-272)
__device__ __forceinline__ Sim3f relative(const Sim3f &Ti, const Sim3f &Tj) {
  Sim3f R;
  const float inv_si = 1.0f / Ti.s;
  const float qc[4] = {-Ti.q[0], -Ti.q[1], -Ti.q[2], Ti.q[3]};
  R.s = inv_si * Tj.s;
  quat_mul(qc, Tj.q, R.q);
  float d[3] = {Tj.t[0] - Ti.t[0], Tj.t[1] - Ti.t[1], Tj.t[2] - Ti.t[2]};
  quat_rot(qc, d, d);
  R.t[0] = d[0] * inv_si, R.t[1] = d[1] * inv_si, R.t[2] = d[2] * inv_si;
  return R;
}

// Exp: tangent [tau, phi, sigma] -> Sim3 (lietorch RxSO3 W, gn_kernels.cu:299-390)
__device__ inline Sim3f exp_sim3(const float *xi) {
  const float EPSV = 1e-6f;
  Sim3f E;
  const float tau[3] = {xi[0], xi[1], xi[2]};
  const float phi[3] = {xi[3], xi[4], xi[5]};
  const float sg = xi[6];
  const float scale = expf(sg);
  const float th2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  float im, re;
  if (th2 < EPSV) {
    const float th4 = th2 * th2;
    im = 0.5f - (1.0f / 48.0f) * th2 + (1.0f / 3840.0f) * th4;
    re = 1.0f - (1.0f / 8.0f) * th2 + (1.0f / 384.0f) * th4;
  } else {
    const float th = sqrtf(th2);
    im = sinf(0.5f * th) / th;
    re = cosf(0.5f * th);
  }
  E.q[0] = im * phi[0], E.q[1] = im * phi[1], E.q[2] = im * phi[2], E.q[3] = re;
  E.s = scale;
  const float th = sqrtf(th2);
  float A, B, C;
  if (fabsf(sg) < EPSV) {
    C = 1.0f;
    if (th < EPSV) {
      A = 0.5f;
      B = 1.0f / 6.0f;
    } else {
      A = (1.0f - cosf(th)) / th2;
      B = (th - sinf(th)) / (th2 * th);
    }
  } else {
    C = (scale - 1.0f) / sg;
    if (th < EPSV) {
      const float sg2 = sg * sg;
      A = ((sg - 1.0f) * scale + 1.0f) / sg2;
      B = (scale * 0.5f * sg2 + scale - 1.0f - sg * scale) / (sg2 * sg);
    } else {
      const float a = scale * sinf(th), b = scale * cosf(th), c = th2 + sg * sg;
      A = (a * sg + (1.0f - b) * th) / (th * c);
      B = (C - ((b - 1.0f) * sg + a * th) / c) / th2;
    }
  }
  // W tau = C tau + A phi x tau + B phi x (phi x tau)
  const float p1[3] = {phi[1] * tau[2] - phi[2] * tau[1], phi[2] * tau[0] - phi[0] * tau[2],
                       phi[0] * tau[1] - phi[1] * tau[0]};
  const float p2[3] = {phi[1] * p1[2] - phi[2] * p1[1], phi[2] * p1[0] - phi[0] * p1[2],
                       phi[0] * p1[1] - phi[1] * p1[0]};
  for (int c = 0; c < 3; c++) E.t[c] = C * tau[c] + A * p1[c] + B * p2[c];
  return E;
}

// T <- Exp(xi) T  (retrSim3 / pose_retr_kernel, gn_kernels.cu:392-453), in the
// reference's fp32 arithmetic: the tracker's update (its parity is pinned by
// the reference tracker's own outputs, tests/golden)
__device__ inline Sim3f retract(const float *xi, const Sim3f &T) { return compose(exp_sim3(xi), T); }

// The backend's retraction: the same map, the same branches and formulas,
// evaluated in fp64 from the fp32 step and pose and rounded once (round 6).
// The reference's fp32 expSim3 (gn_kernels.cu:323-389) is ill-conditioned
// for small steps: C = (e^sigma - 1) / sigma keeps the rounding of e^sigma
// (6e-8) over |sigma|, 0.6 % of C at sigma = 1e-5, so t = W tau moves by up to
// 6e-3 |tau| with the last bit of sigma; A and B lose more when theta and
// sigma are both small. In fp64 those terms are exact to ~1e-16 / |sigma|
// and the pose lands within an fp32 ulp of Exp(xi) T
// (tests/test_gpu_sim3.py::test_backend_retraction_same_inputs_three_ways).
// One lane per pose, once per GN iteration: the cost is off the hot loop.
__device__ inline Sim3f retract_f64(const float *xi, const Sim3f &T) {
  const double EPSV = 1e-6;
  const double tau[3] = {xi[0], xi[1], xi[2]};
  const double phi[3] = {xi[3], xi[4], xi[5]};
  const double sg = xi[6];
  // one expm1 and one sincos of theta / 2 carry every transcendental:
  // e^sigma = 1 + em1, sin theta = 2 sh ch, 1 - cos theta = 2 sh^2 (no
  // cancellation), 1 - e^sigma cos theta = 2 e^sigma sh^2 - em1
  const double em1 = expm1(sg), scale = 1.0 + em1;
  const double th2 = phi[0] * phi[0] + phi[1] * phi[1] + phi[2] * phi[2];
  const double th = sqrt(th2);
  double sh, ch;
  sincos(0.5 * th, &sh, &ch);
  double im, re;
  if (th2 < EPSV) {
    const double th4 = th2 * th2;
    im = 0.5 - (1.0 / 48.0) * th2 + (1.0 / 3840.0) * th4;
    re = 1.0 - (1.0 / 8.0) * th2 + (1.0 / 384.0) * th4;
  } else {
    im = sh / th;
    re = ch;
  }
  const double eq[4] = {im * phi[0], im * phi[1], im * phi[2], re};
  const double sin_th = 2.0 * sh * ch, omc = 2.0 * sh * sh;  // sin theta, 1 - cos theta
  double A, B, C;
  if (fabs(sg) < EPSV) {
    C = 1.0;
    if (th < EPSV) {
      A = 0.5;
      B = 1.0 / 6.0;
    } else {
      A = omc / th2;
      B = (th - sin_th) / (th2 * th);
    }
  } else {
    C = em1 / sg;
    if (th < EPSV) {
      const double sg2 = sg * sg;
      A = ((sg - 1.0) * scale + 1.0) / sg2;
      B = (scale * 0.5 * sg2 + scale - 1.0 - sg * scale) / (sg2 * sg);
    } else {
      const double a = scale * sin_th, omb = scale * omc - em1, c = th2 + sg * sg;  // omb = 1 - b
      A = (a * sg + omb * th) / (th * c);
      B = (C - (a * th - omb * sg) / c) / th2;
    }
  }
  const double p1[3] = {phi[1] * tau[2] - phi[2] * tau[1], phi[2] * tau[0] - phi[0] * tau[2],
                        phi[0] * tau[1] - phi[1] * tau[0]};
  const double p2[3] = {phi[1] * p1[2] - phi[2] * p1[1], phi[2] * p1[0] - phi[0] * p1[2],
                        phi[0] * p1[1] - phi[1] * p1[0]};
  // compose: q = eq * T.q, t = et + scale R(eq) T.t, s = scale T.s
  const double bq[4] = {T.q[0], T.q[1], T.q[2], T.q[3]};
  const double bt[3] = {T.t[0], T.t[1], T.t[2]};
  Sim3f R;
  R.q[0] = (float)(eq[3] * bq[0] + eq[0] * bq[3] + eq[1] * bq[2] - eq[2] * bq[1]);
  R.q[1] = (float)(eq[3] * bq[1] - eq[0] * bq[2] + eq[1] * bq[3] + eq[2] * bq[0]);
  R.q[2] = (float)(eq[3] * bq[2] + eq[0] * bq[1] - eq[1] * bq[0] + eq[2] * bq[3]);
  R.q[3] = (float)(eq[3] * bq[3] - eq[0] * bq[0] - eq[1] * bq[1] - eq[2] * bq[2]);
  const double ux = 2.0 * (eq[1] * bt[2] - eq[2] * bt[1]);
  const double uy = 2.0 * (eq[2] * bt[0] - eq[0] * bt[2]);
  const double uz = 2.0 * (eq[0] * bt[1] - eq[1] * bt[0]);
  const double rt[3] = {bt[0] + eq[3] * ux + (eq[1] * uz - eq[2] * uy),
                        bt[1] + eq[3] * uy + (eq[2] * ux - eq[0] * uz),
                        bt[2] + eq[3] * uz + (eq[0] * uy - eq[1] * ux)};
  for (int c = 0; c < 3; c++) R.t[c] = (float)(C * tau[c] + A * p1[c] + B * p2[c] + scale * rt[c]);
  R.s = (float)(scale * (double)T.s);
  return R;
}

// M = Adj(T_i)^-T as a dense 7x7 (double), so that J_j = M J_local
// (apply_Sim3_adj_inv, gn_kernels.cu:274-297):
//   [ s^-1 R          0   0 ]
//   [ s^-1 [t]x R     R   0 ]
//   [ s^-1 t^T R      0   1 ]
// Entry (r, c) of M = Adj(T)^-T (tau 0-2, phi 3-5, sigma 6): one lane per
// entry (round 5: the edge finalize's 49 lanes form M side by side instead of
// one lane forming all of it); adjT_inv_matrix is the same entries in a loop.
__device__ inline double adjT_inv_entry(const float *Tp, int r, int c) {
  if (r == 6 && c == 6) return 1.0;
  if (c >= 3 && (r < 3 || r == 6 || c == 6)) return 0.0;
  const double tx = Tp[0], ty = Tp[1], tz = Tp[2];
  const double qx = Tp[3], qy = Tp[4], qz = Tp[5], qw = Tp[6];
  // rotation matrix of the (not renormalised) quaternion, matching actSO3's
  // formula X + 2w(v x X) + v x (2 v x X) applied to unit vectors (entries
  // picked by selects, not an indexed array: r, c vary by lane -> scratch)
  const double R00 = 1.0 - 2.0 * (qy * qy + qz * qz), R01 = 2.0 * (qx * qy - qw * qz),
               R02 = 2.0 * (qx * qz + qw * qy), R10 = 2.0 * (qx * qy + qw * qz),
               R11 = 1.0 - 2.0 * (qx * qx + qz * qz), R12 = 2.0 * (qy * qz - qw * qx),
               R20 = 2.0 * (qx * qz - qw * qy), R21 = 2.0 * (qy * qz + qw * qx),
               R22 = 1.0 - 2.0 * (qx * qx + qy * qy);
  const int j = c >= 3 ? c - 3 : c;
  const double R0 = j == 0 ? R00 : (j == 1 ? R01 : R02);  // column j of R
  const double R1 = j == 0 ? R10 : (j == 1 ? R11 : R12);
  const double R2 = j == 0 ? R20 : (j == 1 ? R21 : R22);
  if (c >= 3) return r == 3 ? R0 : (r == 4 ? R1 : R2);  // the phi block
  const double is = 1.0 / (double)Tp[7];
  if (r < 3) return is * (r == 0 ? R0 : (r == 1 ? R1 : R2));
  if (r == 3) return is * (ty * R2 - tz * R1);  // [t]x R
  if (r == 4) return is * (tz * R0 - tx * R2);
  if (r == 5) return is * (tx * R1 - ty * R0);
  return is * (tx * R0 + ty * R1 + tz * R2);
}
__device__ inline void adjT_inv_matrix(const float *Tp, double M[7][7]) {
  for (int r = 0; r < 7; r++)
    for (int c = 0; c < 7; c++) M[r][c] = adjT_inv_entry(Tp, r, c);
}

// ----------------------------------------------------- fast scalar math --
// One-ulp hardware ops for the per-pixel path (v_rcp_f32 / v_sqrt_f32 /
// v_log_f32); the reference uses correctly rounded double-promoted forms —
// the difference is below the fp32 summation noise (DESIGN.md tolerances).
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float fsqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
// natural log: v_log_f32 (log2, ~1 ulp on normal inputs) * ln 2; callers only
// use it on z > z_eps (>= FLT_MIN) or select the result away
__device__ __forceinline__ float flog(float x) {
  return __builtin_amdgcn_logf(x) * 0.693147180559945309f;
}

// branch-free: both sides are always computed, then selected
__device__ __forceinline__ float huber_w(float r, float k) {
  // min(1, k/|r|): 1 below the threshold (k/|r| > 1 there), k/|r| above; one
  // v_min_f32 instead of a compare and a select
  return fminf(1.0f, k * frcp(fabsf(r)));
}

// non-zero patterns of the local Jacobian rows (bits: tau0..2 phi0..2 sigma)
constexpr unsigned kRayX = 0x37, kRayY = 0x2F, kRayZ = 0x1F, kRayD = 0x47;
constexpr unsigned kCalU = 0x3D, kCalV = 0x3E, kCalZ = 0x5C;
constexpr unsigned kPtX = 0x71, kPtY = 0x6A, kPtZ = 0x5C;

// ------------------------------------------ packed-fp32 row accumulation --
// gfx950 issues v_pk_fma_f32 (two fp32 FMAs per lane) at the rate of one
// v_fma_f32, so two residual rows with the same number of non-zero Jacobian
// entries are accumulated as one row of float2: lane .x is row A, lane .y is
// row B, each into its own sums (the shared L entries of the two rows are
// added once, at the end of the block, in fold()). The per-pixel products are
// the reference's (w a_m a_n, w e a_m, w e^2); only the order of the fp32 sums
// differs (per row, then combined).
typedef float f32x2 __attribute__((ext_vector_type(2)));

__host__ __device__ constexpr int popc7(unsigned m) {
  int n = 0;
  for (int c = 0; c < 7; c++) n += (m >> c) & 1u;
  return n;
}
// column of the p-th set bit of m, -1 past the last
__host__ __device__ constexpr int nth_col(unsigned m, int p) {
  for (int c = 0; c < 7; c++)
    if (m & (1u << c)) {
      if (p == 0) return c;
      p--;
    }
  return -1;
}

// Two rows A (mask MA) and B (mask MB, popc(MB) <= popc(MA)); a[p] holds the
// p-th non-zero entry of each (B padded with 0 past its last).
template <unsigned MA, unsigned MB>
struct PairAcc {
  static constexpr int K = popc7(MA);
  static constexpr int NT = K * (K + 1) / 2;
  f32x2 h[NT], g[K], c;
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int t = 0; t < NT; t++) h[t] = f32x2{0.0f, 0.0f};
#pragma unroll
    for (int p = 0; p < K; p++) g[p] = f32x2{0.0f, 0.0f};
    c = f32x2{0.0f, 0.0f};
  }
  __device__ __forceinline__ void add(const f32x2 (&a)[K], f32x2 w, f32x2 e) {
    f32x2 wa[K];
#pragma unroll
    for (int p = 0; p < K; p++) wa[p] = w * a[p];
    int t = 0;
#pragma unroll
    for (int p = 0; p < K; p++)
#pragma unroll
      for (int q = p; q < K; q++, t++) h[t] = __builtin_elementwise_fma(wa[p], a[q], h[t]);
    const f32x2 we = w * e;
#pragma unroll
    for (int p = 0; p < K; p++) g[p] = __builtin_elementwise_fma(we, a[p], g[p]);
    c = __builtin_elementwise_fma(we, e, c);
  }
  __device__ __forceinline__ void fold(float *acc) const {
    int t = 0;
#pragma unroll
    for (int p = 0; p < K; p++)
#pragma unroll
      for (int q = p; q < K; q++, t++) {
        acc[kL + tri(nth_col(MA, p), nth_col(MA, q))] += h[t].x;
        if (nth_col(MB, q) >= 0) acc[kL + tri(nth_col(MB, p), nth_col(MB, q))] += h[t].y;
      }
#pragma unroll
    for (int p = 0; p < K; p++) {
      acc[kG + nth_col(MA, p)] += g[p].x;
      if (nth_col(MB, p) >= 0) acc[kG + nth_col(MB, p)] += g[p].y;
    }
    acc[kCost] += c.x + c.y;
  }
};

// One row (mask M), a[p] = its p-th non-zero entry.
template <unsigned M>
struct RowAcc {
  static constexpr int K = popc7(M);
  static constexpr int NT = K * (K + 1) / 2;
  float h[NT], g[K], c;
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int t = 0; t < NT; t++) h[t] = 0.0f;
#pragma unroll
    for (int p = 0; p < K; p++) g[p] = 0.0f;
    c = 0.0f;
  }
  __device__ __forceinline__ void add(const float (&a)[K], float w, float e) {
    float wa[K];
#pragma unroll
    for (int p = 0; p < K; p++) wa[p] = w * a[p];
    int t = 0;
#pragma unroll
    for (int p = 0; p < K; p++)
#pragma unroll
      for (int q = p; q < K; q++, t++) h[t] = __builtin_fmaf(wa[p], a[q], h[t]);
    const float we = w * e;
#pragma unroll
    for (int p = 0; p < K; p++) g[p] = __builtin_fmaf(we, a[p], g[p]);
    c = __builtin_fmaf(we, e, c);
  }
  __device__ __forceinline__ void fold(float *acc) const {
    int t = 0;
#pragma unroll
    for (int p = 0; p < K; p++)
#pragma unroll
      for (int q = p; q < K; q++, t++) acc[kL + tri(nth_col(M, p), nth_col(M, q))] += h[t];
#pragma unroll
    for (int p = 0; p < K; p++) acc[kG + nth_col(M, p)] += g[p];
    acc[kCost] += c;
  }
};

// Scalar twin of the packed accumulators that adds straight into one
// 36-float layout (fewer registers: the first, gathering GN iteration keeps 4
// pixels of raw inputs live and uses it). Same products, the reference's order
// per entry (rows u/x, then v/y, then the third row).
struct AccumFlat {
  float s[kNP];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int k = 0; k < kNP; k++) s[k] = 0.0f;
  }
  __device__ __forceinline__ void fold(float *acc) const {
#pragma unroll
    for (int k = 0; k < kNP; k++) acc[k] += s[k];
  }
  template <unsigned MA, unsigned MB, int K>
  __device__ __forceinline__ void add2(const f32x2 (&a)[K], f32x2 w, f32x2 e) {
    f32x2 wa[K];
#pragma unroll
    for (int p = 0; p < K; p++) wa[p] = w * a[p];
#pragma unroll
    for (int p = 0; p < K; p++)
#pragma unroll
      for (int q = p; q < K; q++) {
        const int ta = kL + tri(nth_col(MA, p), nth_col(MA, q));
        s[ta] = __builtin_fmaf(wa[p].x, a[q].x, s[ta]);
        if (nth_col(MB, q) >= 0) {
          const int tb = kL + tri(nth_col(MB, p), nth_col(MB, q));
          s[tb] = __builtin_fmaf(wa[p].y, a[q].y, s[tb]);
        }
      }
    const f32x2 we = w * e;
#pragma unroll
    for (int p = 0; p < K; p++) {
      s[kG + nth_col(MA, p)] = __builtin_fmaf(we.x, a[p].x, s[kG + nth_col(MA, p)]);
      if (nth_col(MB, p) >= 0) s[kG + nth_col(MB, p)] = __builtin_fmaf(we.y, a[p].y, s[kG + nth_col(MB, p)]);
    }
    s[kCost] = __builtin_fmaf(we.x, e.x, s[kCost]);
    s[kCost] = __builtin_fmaf(we.y, e.y, s[kCost]);
  }
  template <unsigned M, int K>
  __device__ __forceinline__ void add1(const float (&a)[K], float w, float e) {
    float wa[K];
#pragma unroll
    for (int p = 0; p < K; p++) wa[p] = w * a[p];
#pragma unroll
    for (int p = 0; p < K; p++)
#pragma unroll
      for (int q = p; q < K; q++) {
        const int t = kL + tri(nth_col(M, p), nth_col(M, q));
        s[t] = __builtin_fmaf(wa[p], a[q], s[t]);
      }
    const float we = w * e;
#pragma unroll
    for (int p = 0; p < K; p++) s[kG + nth_col(M, p)] = __builtin_fmaf(we, a[p], s[kG + nth_col(M, p)]);
    s[kCost] = __builtin_fmaf(we, e, s[kCost]);
  }
};

// Per-lane accumulators of one residual model: rays pairs (x, y) and
// (z, dist); calib pairs (u, v) plus the log-depth row; points pairs (x, y)
// plus z. fold() adds them into the 36-float layout (kL / kG / kCost).
template <int MODE>
struct Accum;
// add2<MA, MB>(a, w, e) / add1<M>(a, w, e) route a row pair / a row to its
// accumulator (the same calls drive AccumFlat).
template <>
struct Accum<1> {
  PairAcc<kRayX, kRayY> xy;
  PairAcc<kRayZ, kRayD> zd;
  __device__ __forceinline__ void zero() { xy.zero(), zd.zero(); }
  __device__ __forceinline__ void fold(float *acc) const { xy.fold(acc), zd.fold(acc); }
  template <unsigned MA, unsigned MB, int K>
  __device__ __forceinline__ void add2(const f32x2 (&a)[K], f32x2 w, f32x2 e) {
    if constexpr (MA == kRayX) xy.add(a, w, e);
    else zd.add(a, w, e);
  }
};
template <>
struct Accum<2> {
  PairAcc<kCalU, kCalV> uv;
  RowAcc<kCalZ> z;
  __device__ __forceinline__ void zero() { uv.zero(), z.zero(); }
  __device__ __forceinline__ void fold(float *acc) const { uv.fold(acc), z.fold(acc); }
  template <unsigned MA, unsigned MB, int K>
  __device__ __forceinline__ void add2(const f32x2 (&a)[K], f32x2 w, f32x2 e) { uv.add(a, w, e); }
  template <unsigned M, int K>
  __device__ __forceinline__ void add1(const float (&a)[K], float w, float e) { z.add(a, w, e); }
};
template <>
struct Accum<0> {
  PairAcc<kPtX, kPtY> xy;
  RowAcc<kPtZ> z;
  __device__ __forceinline__ void zero() { xy.zero(), z.zero(); }
  __device__ __forceinline__ void fold(float *acc) const { xy.fold(acc), z.fold(acc); }
  template <unsigned MA, unsigned MB, int K>
  __device__ __forceinline__ void add2(const f32x2 (&a)[K], f32x2 w, f32x2 e) { xy.add(a, w, e); }
  template <unsigned M, int K>
  __device__ __forceinline__ void add1(const float (&a)[K], float w, float e) { z.add(a, w, e); }
};

struct ResidualParams {
  float inv_sig_a, inv_sig_b;  // 1/sigma
  float C_thresh, Q_thresh;
  float fx, fy, cx, cy;
  int width, height;
  float border, z_eps;
  float huber_k;
};

// Per (edge, pixel) target-side inputs of the residual: everything that does
// not depend on the poses. The backend computes them once per solve call and
// stores them as per-edge planes (see linearize_packed_kernel), so later GN
// iterations read 12-20 B per pixel and never gather from KF i. Both the
// gathering and the packed kernels go through make_pixin + pixel_contrib (same
// formulas; the sums differ only by FMA-contraction rounding between kernels).
//   points: {Xi.x, Xi.y, Xi.z, sq}          rays: {Xi.x, Xi.y, Xi.z, sq} (the unit
//   ray X_i / |X_i| and |X_i| are formed where they are used: 16 B per pixel)
//   calib:  {(v_t << 16 | u_t) as bits, sq, log z_i}
// sq = sqrt(q) if the match is valid (valid_match, q > Q_thresh, ci/cj >
// C_thresh; calib also z_i > z_eps), else 0: a zero weight zeroes the
// pixel's contribution exactly as the reference's `valid ? ... : 0` does.
template <int MODE>
struct PixIn;
template <>
struct PixIn<0> {
  static constexpr int kPlanes = 4;
  float v[4];
};
template <>
struct PixIn<1> {  // {X_i, sq}: the unit ray and |X_i| are formed from X_i in pixel_contrib
  static constexpr int kPlanes = 4;
  float v[4];
};
template <>
struct PixIn<2> {
  static constexpr int kPlanes = 3;
  float v[3];
};

template <int MODE>
__device__ __forceinline__ PixIn<MODE> make_pixin(const ResidualParams &P, const float *Xi, bool ok,
                                                  float q, int u_t, int v_t) {
  PixIn<MODE> r;
  if (MODE == 1) {  // ray_align_kernel :924-963 (the ray of X_i is formed per use)
    r.v[0] = Xi[0], r.v[1] = Xi[1], r.v[2] = Xi[2];
    r.v[3] = ok ? fsqrt(q) : 0.0f;
  } else if (MODE == 2) {  // calib_proj_kernel :1360-1405
    const bool vzi = Xi[2] > P.z_eps;
    const float li = flog(Xi[2]);
    r.v[0] = __int_as_float((v_t << 16) | u_t);
    r.v[1] = (ok && vzi) ? fsqrt(q) : 0.0f;
    r.v[2] = vzi ? li : 0.0f;
  } else {  // point_align_kernel :564-586
    r.v[0] = Xi[0], r.v[1] = Xi[1], r.v[2] = Xi[2];
    r.v[3] = ok ? fsqrt(q) : 0.0f;
  }
  return r;
}

// One (edge, pixel) contribution from the target-side inputs and
// Y = T_ij Xj (source point in frame i).
template <int MODE, typename ACC>
__device__ __forceinline__ void pixel_contrib(ACC &acc, const ResidualParams &P, const PixIn<MODE> &in,
                                              const float *Y) {
  if constexpr (MODE == 1) {  // rays + distance  (ray_align_kernel :924-1089)
    const float ni = fsqrt(in.v[0] * in.v[0] + in.v[1] * in.v[1] + in.v[2] * in.v[2]);
    const float ini = frcp(ni);
    const float nj2 = Y[0] * Y[0] + Y[1] * Y[1] + Y[2] * Y[2];
    const float nj = fsqrt(nj2);
    const float inj = frcp(nj);
    const float rx = Y[0] * inj, ry = Y[1] * inj, rz = Y[2] * inj;
    const float e0 = rx - in.v[0] * ini, e1 = ry - in.v[1] * ini, e2 = rz - in.v[2] * ini;
    const float e3 = nj - ni;
    const float sq = in.v[3];
    const float swr = P.inv_sig_a * sq;
    const float swd = P.inv_sig_b * sq;
    const float kr = swr * swr, kd = swd * swd;
    const float w0 = huber_w(swr * e0, P.huber_k) * kr;
    const float w1 = huber_w(swr * e1, P.huber_k) * kr;
    const float w2 = huber_w(swr * e2, P.huber_k) * kr;
    const float w3 = huber_w(swd * e3, P.huber_k) * kd;
    // d r / d P = (I - r r^T) / |P|
    const float dxx = inj - rx * rx * inj, dyy = inj - ry * ry * inj, dzz = inj - rz * rz * inj;
    const float dxy = -rx * ry * inj, dxz = -rx * rz * inj, dyz = -ry * rz * inj;
    // non-zero entries of the rows (kRayX..kRayD order of columns)
    //   x: {dxx, dxy, dxz, rz, -ry}   y: {dxy, dyy, dyz, -rz, rx}
    //   z: {dxz, dyz, dzz, ry, -rx}   d: {rx, ry, rz, nj}
    const f32x2 axy[5] = {{dxx, dxy}, {dxy, dyy}, {dxz, dyz}, {rz, -rz}, {-ry, rx}};
    const f32x2 azd[5] = {{dxz, rx}, {dyz, ry}, {dzz, rz}, {ry, nj}, {-rx, 0.0f}};
    acc.template add2<kRayX, kRayY>(axy, f32x2{w0, w1}, f32x2{e0, e1});
    acc.template add2<kRayZ, kRayD>(azd, f32x2{w2, w3}, f32x2{e2, e3});
  } else if constexpr (MODE == 2) {  // pinhole pixel + log-depth (calib_proj_kernel :1360-1495)
    // The u / v rows in focal-normalised form: with f = (fx, fy), a' = a / f,
    // e' = e / f and W = w f^2 the sums are unchanged (W a' a'^T = w a a^T,
    // W e' a' = w e a, W e'^2 = w e^2), and W needs no extra work:
    //   w = huber(sw e) sw^2 = min(sw^2, k sw / |e|)  (|sw e| < k -> sw^2)
    //   W = min((sw f)^2, k (sw f) / |e'|)
    const bool vz = Y[2] > P.z_eps;  // z_i > z_eps is folded into sq
    const float zr = frcp(Y[2]), lj_ = flog(Y[2]);
    const float zinv = vz ? zr : 0.0f;
    const float e2 = vz ? lj_ - in.v[2] : 0.0f;  // log z_j - log z_i (both 0 when !vz)
    const int uvt = __float_as_int(in.v[0]);
    const f32x2 tuv = {(float)(uvt & 0xffff), (float)(uvt >> 16)};
    const f32x2 fxy = {P.fx, P.fy};
    const f32x2 xy = f32x2{Y[0], Y[1]} * zinv;
    const f32x2 uv = __builtin_elementwise_fma(fxy, xy, f32x2{P.cx, P.cy});
    const bool vu = (uv.x > P.border) && (uv.x < (float)P.width - 1.0f - P.border);
    const bool vv = (uv.y > P.border) && (uv.y < (float)P.height - 1.0f - P.border);
    const bool good = vu && vv && vz;
    const float sq = good ? in.v[1] : 0.0f;
    const f32x2 et = (uv - tuv) * f32x2{1.0f / P.fx, 1.0f / P.fy};
    const f32x2 swf = sq * (P.inv_sig_a * fxy);
    const f32x2 kpf = swf * swf, ksf = swf * P.huber_k;
    const f32x2 W = {fminf(kpf.x, ksf.x * frcp(fabsf(et.x))), fminf(kpf.y, ksf.y * frcp(fabsf(et.y)))};
    const float swz = sq * P.inv_sig_b;
    const float w2 = fminf(swz * swz, (swz * P.huber_k) * frcp(fabsf(e2)));
    const float x = xy.x, y = xy.y;
    // u / fx: {1/z, -x/z, -x y, 1 + x^2, -y}   (columns 0 2 3 4 5)
    // v / fy: {1/z, -y/z, -(1 + y^2), x y, x}  (columns 1 2 3 4 5)
    // log z:  {1/z, y, -x, 1}                  (columns 2 3 4 6)
    const float xyp = x * y;
    const f32x2 auv[5] = {{zinv, zinv}, -(xy * zinv), {-xyp, -__builtin_fmaf(y, y, 1.0f)},
                          {__builtin_fmaf(x, x, 1.0f), xyp}, {-y, x}};
    acc.template add2<kCalU, kCalV>(auv, W, et);
    const float az[4] = {zinv, y, -x, 1.0f};
    acc.template add1<kCalZ>(az, w2, e2);
  } else {  // 3D point (point_align_kernel :564-674)
    const float e0 = Y[0] - in.v[0], e1 = Y[1] - in.v[1], e2 = Y[2] - in.v[2];
    const float sw = P.inv_sig_a * in.v[3];
    const float k2 = sw * sw;
    const float w0 = huber_w(sw * e0, P.huber_k) * k2;
    const float w1 = huber_w(sw * e1, P.huber_k) * k2;
    const float w2 = huber_w(sw * e2, P.huber_k) * k2;
    // x: {1, Y2, -Y1, Y0} (columns 0 4 5 6)  y: {1, -Y2, Y0, Y1} (1 3 5 6)
    // z: {1, Y1, -Y0, Y2} (columns 2 3 4 6)
    const f32x2 axy[4] = {{1.0f, 1.0f}, {Y[2], -Y[2]}, {-Y[1], Y[0]}, {Y[0], Y[1]}};
    const float az[4] = {1.0f, Y[1], -Y[0], Y[2]};
    acc.template add2<kPtX, kPtY>(axy, f32x2{w0, w1}, f32x2{e0, e1});
    acc.template add1<kPtZ>(az, w2, e2);
  }
}

// ------------------------------------- pixel-pair packed accumulation --
// Two PIXELS per lane in the halves of a float2: every per-pixel operation
// (the Sim(3) transform, the residuals, the Jacobian entries, the Huber
// weights and all 36 normal-equation sums) is one v_pk_* instruction for
// both pixels; only the transcendentals (v_sqrt / v_rcp / v_log) stay
// scalar. Entries no row of the model touches stay compile-time zeros and
// take no registers (rays 33, calib 32 live sums). Same per-pixel products as
// pixel_contrib; the fp32 sums are per half, then combined in fold().
struct AccumPP {
  f32x2 s[kNP];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int k = 0; k < kNP; k++) s[k] = f32x2{0.0f, 0.0f};
  }
  __device__ __forceinline__ void fold(float *acc) const {
#pragma unroll
    for (int k = 0; k < kNP; k++) acc[k] += s[k].x + s[k].y;
  }
  // Calib (packed backend iterations, round 5): L(2,5) is not summed but
  // formed here as -(L(0,3) + L(1,4)). With zi = 1/z, per pixel the u row
  // adds -W_u x y zi to L(0,3) and +W_u x y zi to L(2,5), the v row +W_v x y zi
  // to L(1,4) and -W_v x y zi to L(2,5), and the log-depth row has no column
  // 5. Two fewer FMAs per pixel pair; only the fp32 rounding of L(2,5) differs.
  __device__ __forceinline__ void cal25_fixup() {
    s[kL + tri(2, 5)] = -(s[kL + tri(0, 3)] + s[kL + tri(1, 4)]);
  }
  // one residual row (non-zero columns M, a[p] = the p-th entry) of both pixels;
  // COST false: no cost sum (the backend's solve never reads it; the tracker's
  // convergence rule does)
  // SKIP: a sum this row leaves out (one the caller forms afterwards)
  template <unsigned M, int K, bool COST = true, int SKIP = -1>
  __device__ __forceinline__ void add(const f32x2 (&a)[K], f32x2 w, f32x2 e) {
    f32x2 wa[K];
#pragma unroll
    for (int p = 0; p < K; p++) wa[p] = w * a[p];
#pragma unroll
    for (int p = 0; p < K; p++)
#pragma unroll
      for (int q = p; q < K; q++) {
        const int t = kL + tri(nth_col(M, p), nth_col(M, q));
        if (t == SKIP) continue;
        s[t] = __builtin_elementwise_fma(wa[p], a[q], s[t]);
      }
    const f32x2 we = w * e;
#pragma unroll
    for (int p = 0; p < K; p++) s[kG + nth_col(M, p)] = __builtin_elementwise_fma(we, a[p], s[kG + nth_col(M, p)]);
    if (COST) s[kCost] = __builtin_elementwise_fma(we, e, s[kCost]);
  }
};

// keeps the scheduler from hoisting the next row's products over this row's
// sums (register pressure of the pixel-pair kernels)
#define M3S_ROW_BARRIER() __builtin_amdgcn_sched_barrier(0)
__device__ __forceinline__ f32x2 splat2(float v) { return f32x2{v, v}; }
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 rcp2(f32x2 x) { return f32x2{frcp(x.x), frcp(x.y)}; }
__device__ __forceinline__ f32x2 sqrt2(f32x2 x) { return f32x2{fsqrt(x.x), fsqrt(x.y)}; }
__device__ __forceinline__ f32x2 abs2(f32x2 x) { return f32x2{fabsf(x.x), fabsf(x.y)}; }
__device__ __forceinline__ f32x2 min2(f32x2 a, f32x2 b) { return f32x2{fminf(a.x, b.x), fminf(a.y, b.y)}; }
__device__ __forceinline__ f32x2 sel2(bool cx, bool cy, f32x2 a, f32x2 b) {
  return f32x2{cx ? a.x : b.x, cy ? a.y : b.y};
}

// Y = T X for two points (same FMA order per element as act(Sim3Mat))
__device__ __forceinline__ void act2(const Sim3Mat &M, const f32x2 (&X)[3], f32x2 (&Y)[3]) {
#pragma unroll
  for (int r = 0; r < 3; r++)
    Y[r] = fma2(splat2(M.m[3 * r]), X[0],
                fma2(splat2(M.m[3 * r + 1]), X[1], fma2(splat2(M.m[3 * r + 2]), X[2], splat2(M.t[r]))));
}

// pixel_contrib for two pixels: in[k] = plane k of both, Y = T_ij Xj of both.
// COST false (the backend's packed iterations): no cost sum, and the calib
// model takes 1/z and log z of max(z, z_floor) instead of selecting them away
// when z <= z_eps (that pixel's weight is 0 either way; both stay finite), and
// forms log z_j - log z_i as one fma on log2 z_j
template <int MODE, int NPL, bool COST = true>
__device__ __forceinline__ void pixel_contrib2(AccumPP &acc, const ResidualParams &P, const f32x2 (&in)[NPL],
                                               const f32x2 (&Y)[3]) {
  if constexpr (MODE == 1) {  // rays + distance  (ray_align_kernel :924-1089)
    const f32x2 ni = sqrt2(fma2(in[0], in[0], fma2(in[1], in[1], in[2] * in[2])));
    const f32x2 ini = rcp2(ni);
    const f32x2 nj2 = fma2(Y[0], Y[0], fma2(Y[1], Y[1], Y[2] * Y[2]));
    const f32x2 nj = sqrt2(nj2);
    const f32x2 inj = rcp2(nj);
    const f32x2 rx = Y[0] * inj, ry = Y[1] * inj, rz = Y[2] * inj;
    const f32x2 e0 = rx - in[0] * ini, e1 = ry - in[1] * ini, e2 = rz - in[2] * ini, e3 = nj - ni;
    const f32x2 swr = in[3] * P.inv_sig_a, swd = in[3] * P.inv_sig_b;
    const f32x2 kr = swr * swr, kd = swd * swd;
    const f32x2 hk = splat2(P.huber_k);
    // huber(sw e) sw^2 = min(1, k / |sw e|) sw^2 (= sw min(sw, k / |e|): one
    // product fewer, the packed backend iterations)
    f32x2 w0, w1, w2, w3;
    if (COST) {
      w0 = min2(splat2(1.0f), hk * rcp2(abs2(swr * e0))) * kr;
      w1 = min2(splat2(1.0f), hk * rcp2(abs2(swr * e1))) * kr;
      w2 = min2(splat2(1.0f), hk * rcp2(abs2(swr * e2))) * kr;
      w3 = min2(splat2(1.0f), hk * rcp2(abs2(swd * e3))) * kd;
    } else {
      w0 = swr * min2(swr, hk * rcp2(abs2(e0)));
      w1 = swr * min2(swr, hk * rcp2(abs2(e1)));
      w2 = swr * min2(swr, hk * rcp2(abs2(e2)));
      w3 = swd * min2(swd, hk * rcp2(abs2(e3)));
    }
    // d r / d P = (I - r r^T) / |P|
    const f32x2 rxi = rx * inj, ryi = ry * inj, rzi = rz * inj;
    const f32x2 dxx = inj - rx * rxi, dyy = inj - ry * ryi, dzz = inj - rz * rzi;
    const f32x2 dxy = -(ry * rxi), dxz = -(rz * rxi), dyz = -(rz * ryi);
    const f32x2 ax[5] = {dxx, dxy, dxz, rz, -ry};  // kRayX: tau0 tau1 tau2 phi1 phi2
    const f32x2 ay[5] = {dxy, dyy, dyz, -rz, rx};  // kRayY: tau0 tau1 tau2 phi0 phi2
    const f32x2 az[5] = {dxz, dyz, dzz, ry, -rx};  // kRayZ: tau0 tau1 tau2 phi0 phi1
    const f32x2 ad[4] = {rx, ry, rz, nj};          // kRayD: tau0 tau1 tau2 sigma
    acc.add<kRayX, 5, COST>(ax, w0, e0);
    M3S_ROW_BARRIER();
    acc.add<kRayY, 5, COST>(ay, w1, e1);
    M3S_ROW_BARRIER();
    acc.add<kRayZ, 5, COST>(az, w2, e2);
    M3S_ROW_BARRIER();
    acc.add<kRayD, 4, COST>(ad, w3, e3);
    M3S_ROW_BARRIER();
  } else if constexpr (MODE == 2) {  // pinhole pixel + log-depth (calib_proj_kernel :1360-1495)
    // focal-normalised u / v rows as in pixel_contrib
    const bool vzx = Y[2].x > P.z_eps, vzy = Y[2].y > P.z_eps;
    const f32x2 zero2 = splat2(0.0f);
    f32x2 zinv, e2;
    if (COST) {
      const f32x2 zr = rcp2(Y[2]);
      const f32x2 lj = f32x2{flog(Y[2].x), flog(Y[2].y)};
      zinv = sel2(vzx, vzy, zr, zero2);
      e2 = sel2(vzx, vzy, lj - in[2], zero2);
    } else {
      // z_floor = max(z_eps, FLT_MIN): z > z_eps leaves z unchanged
      const float zf = fmaxf(P.z_eps, 1.17549435e-38f);
      const f32x2 zc = {fmaxf(Y[2].x, zf), fmaxf(Y[2].y, zf)};
      zinv = rcp2(zc);
      const f32x2 l2 = {__builtin_amdgcn_logf(zc.x), __builtin_amdgcn_logf(zc.y)};
      e2 = fma2(l2, splat2(0.693147180559945309f), -in[2]);
    }
    const int ux = __float_as_int(in[0].x), uy = __float_as_int(in[0].y);
    const f32x2 tu = {(float)(ux & 0xffff), (float)(uy & 0xffff)};
    const f32x2 tv = {(float)(ux >> 16), (float)(uy >> 16)};
    const f32x2 x = Y[0] * zinv, y = Y[1] * zinv;
    const f32x2 u = fma2(splat2(P.fx), x, splat2(P.cx)), v = fma2(splat2(P.fy), y, splat2(P.cy));
    const float ulim = (float)P.width - 1.0f - P.border, vlim = (float)P.height - 1.0f - P.border;
    const bool gx = (u.x > P.border) && (u.x < ulim) && (v.x > P.border) && (v.x < vlim) && vzx;
    const bool gy = (u.y > P.border) && (u.y < ulim) && (v.y > P.border) && (v.y < vlim) && vzy;
    const f32x2 sq = sel2(gx, gy, in[1], zero2);
    const f32x2 etu = (u - tu) * (1.0f / P.fx), etv = (v - tv) * (1.0f / P.fy);
    const f32x2 swu = sq * (P.inv_sig_a * P.fx), swv = sq * (P.inv_sig_a * P.fy);
    const f32x2 hk = splat2(P.huber_k);
    const f32x2 swz = sq * P.inv_sig_b;
    f32x2 Wu, Wv, Wz;
    if (COST) {
      Wu = min2(swu * swu, (swu * hk) * rcp2(abs2(etu)));
      Wv = min2(swv * swv, (swv * hk) * rcp2(abs2(etv)));
      Wz = min2(swz * swz, (swz * hk) * rcp2(abs2(e2)));
    } else {  // the same weights as sw min(sw, k / |e|): two products instead of three
      Wu = swu * min2(swu, hk * rcp2(abs2(etu)));
      Wv = swv * min2(swv, hk * rcp2(abs2(etv)));
      Wz = swz * min2(swz, hk * rcp2(abs2(e2)));
    }
    const f32x2 xyp = x * y;
    const f32x2 one = splat2(1.0f);
    const f32x2 au[5] = {zinv, -(x * zinv), -xyp, fma2(x, x, one), -y};  // kCalU: 0 2 3 4 5
    const f32x2 av[5] = {zinv, -(y * zinv), -fma2(y, y, one), xyp, x};  // kCalV: 1 2 3 4 5
    const f32x2 az[4] = {zinv, y, -x, one};                              // kCalZ: 2 3 4 6
    constexpr int kSkip25 = !COST ? kL + tri(2, 5) : -1;  // AccumPP::cal25_fixup
    acc.add<kCalU, 5, COST, kSkip25>(au, Wu, etu);
    M3S_ROW_BARRIER();
    acc.add<kCalV, 5, COST, kSkip25>(av, Wv, etv);
    M3S_ROW_BARRIER();
    acc.add<kCalZ, 4, COST>(az, Wz, e2);
    M3S_ROW_BARRIER();
  } else {  // 3D point (point_align_kernel :564-674)
    const f32x2 e0 = Y[0] - in[0], e1 = Y[1] - in[1], e2 = Y[2] - in[2];
    const f32x2 sw = in[3] * P.inv_sig_a;
    const f32x2 k2 = sw * sw;
    const f32x2 hk = splat2(P.huber_k);
    f32x2 w0, w1, w2;
    if (COST) {
      w0 = min2(splat2(1.0f), hk * rcp2(abs2(sw * e0))) * k2;
      w1 = min2(splat2(1.0f), hk * rcp2(abs2(sw * e1))) * k2;
      w2 = min2(splat2(1.0f), hk * rcp2(abs2(sw * e2))) * k2;
    } else {
      w0 = sw * min2(sw, hk * rcp2(abs2(e0)));
      w1 = sw * min2(sw, hk * rcp2(abs2(e1)));
      w2 = sw * min2(sw, hk * rcp2(abs2(e2)));
    }
    const f32x2 one = splat2(1.0f);
    const f32x2 ax[4] = {one, Y[2], -Y[1], Y[0]};  // kPtX: 0 4 5 6
    const f32x2 ay[4] = {one, -Y[2], Y[0], Y[1]};  // kPtY: 1 3 5 6
    const f32x2 az[4] = {one, Y[1], -Y[0], Y[2]};  // kPtZ: 2 3 4 6
    acc.add<kPtX, 4, COST>(ax, w0, e0);
    M3S_ROW_BARRIER();
    acc.add<kPtY, 4, COST>(ay, w1, e1);
    M3S_ROW_BARRIER();
    acc.add<kPtZ, 4, COST>(az, w2, e2);
    M3S_ROW_BARRIER();
  }
}

// wave64 butterfly sum
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

}  // namespace m3s
