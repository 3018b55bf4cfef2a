// m3s_match.hip — MI355X (gfx950) matching kernels of MASt3R-SLAM:
// iter_proj and refine_matches (include/m3s_match.h).
//
// Both are per-pixel independent searches: one lane per (batch, pixel), 256
// lanes per block, grid over B*N. Their reads are gathers around the pixel's
// own neighbourhood, so neighbouring lanes hit the same 128-B lines and the
// working set stays in the CU's L1/L2 (no LDS tiling: iter_proj's window
// moves with every LM step and refine_matches' centre drifts up to
// radius*(dilation_max+...+1) pixels, so a fixed halo would not fit).
//
// Arithmetic follows the reference kernels operation by operation, including
// their double-precision literals (`1.0 - du`, `1.0 / r_norm`, `lambda *= 0.1`
// promote to fp64 in matching_kernels.cu) and without FMA contraction, so the
// fp32 results reproduce the reference's IEEE sequence.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "m3s_gn.h"
#include "m3s_match.h"

namespace {

constexpr int kMatchThreads = 256;

inline int launch_status() { return hipGetLastError() == hipSuccess ? M3S_OK : M3S_ELAUNCH; }

// ------------------------------------------------------------ iter_proj --
#pragma clang fp contract(off)

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// bilinear weights of matching_kernels.cu:160-164 (w12, w21, w22 via fp64)
struct Bilin {
  int u11, v11;
  float w11, w12, w21, w22;
};
__device__ __forceinline__ Bilin bilin(float u, float v) {
  Bilin B;
  B.u11 = (int)floorf(u);
  B.v11 = (int)floorf(v);
  const float du = u - (float)B.u11;
  const float dv = v - (float)B.v11;
  B.w11 = du * dv;
  B.w12 = (float)((1.0 - (double)du) * (double)dv);
  B.w21 = (float)((double)du * (1.0 - (double)dv));
  B.w22 = (float)((1.0 - (double)du) * (1.0 - (double)dv));
  return B;
}

// channels [c0, c0+n) of the bilinear sample; "pixels are opposite the area"
// (matching_kernels.cu:166-170): r11 <- (v+1, u+1), r12 <- (v+1, u), r21 <- (v, u+1), r22 <- (v, u)
template <int NC>
__device__ __forceinline__ void sample(const float *img, int64_t W, const Bilin &B, int c0, float *out) {
  const float *r11 = img + ((int64_t)(B.v11 + 1) * W + (B.u11 + 1)) * 9 + c0;
  const float *r12 = img + ((int64_t)(B.v11 + 1) * W + B.u11) * 9 + c0;
  const float *r21 = img + ((int64_t)B.v11 * W + (B.u11 + 1)) * 9 + c0;
  const float *r22 = img + ((int64_t)B.v11 * W + B.u11) * 9 + c0;
#pragma unroll
  for (int j = 0; j < NC; j++) out[j] = B.w11 * r11[j] + B.w12 * r12[j] + B.w21 * r21[j] + B.w22 * r22[j];
}

__device__ __forceinline__ float normalized_cost(float *r, const float *p) {
  const float r_norm = sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
  const float r_norm_inv = (float)(1.0 / (double)r_norm);
  float err[3];
#pragma unroll
  for (int j = 0; j < 3; j++) {
    r[j] *= r_norm_inv;
    err[j] = r[j] - p[j];
  }
  return err[0] * err[0] + err[1] * err[1] + err[2] * err[2];
}

__global__ void __launch_bounds__(kMatchThreads) iter_proj_kernel(m3s_iter_proj_args A) {
  const int64_t gid = (int64_t)blockIdx.x * kMatchThreads + threadIdx.x;
  if (gid >= A.B * A.N) return;
  const int64_t b = gid / A.N;
  const float *img = A.rays_img + b * A.H * A.W * 9;
  const float W2 = (float)(A.W - 2), H2 = (float)(A.H - 2);
  float u = clampf(A.p_init[2 * gid], 1.0f, W2);
  float v = clampf(A.p_init[2 * gid + 1], 1.0f, H2);
  const float p[3] = {A.pts_3d_norm[3 * gid], A.pts_3d_norm[3 * gid + 1], A.pts_3d_norm[3 * gid + 2]};
  float lambda = A.lambda_init;
  bool conv = false;
  for (int it = 0; it < A.max_iter; it++) {
    const Bilin B = bilin(u, v);
    float r[3], gx[3], gy[3];
    sample<3>(img, A.W, B, 0, r);
    sample<3>(img, A.W, B, 3, gx);
    sample<3>(img, A.W, B, 6, gy);
    // error of the normalised ray (matching_kernels.cu:184-198)
    const float r_norm = sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    const float r_norm_inv = (float)(1.0 / (double)r_norm);
    float err[3];
#pragma unroll
    for (int j = 0; j < 3; j++) {
      r[j] *= r_norm_inv;
      err[j] = r[j] - p[j];
    }
    const float cost = err[0] * err[0] + err[1] * err[1] + err[2] * err[2];
    // 2x2 LM system (matching_kernels.cu:200-218)
    float A00 = gx[0] * gx[0] + gx[1] * gx[1] + gx[2] * gx[2];
    const float A01 = gx[0] * gy[0] + gx[1] * gy[1] + gx[2] * gy[2];
    float A11 = gy[0] * gy[0] + gy[1] * gy[1] + gy[2] * gy[2];
    const float b0 = -(err[0] * gx[0] + err[1] * gx[1] + err[2] * gx[2]);
    const float b1 = -(err[0] * gy[0] + err[1] * gy[1] + err[2] * gy[2]);
    A00 += lambda;
    A11 += lambda;
    const float det_inv = (float)(1.0 / (double)(A00 * A11 - A01 * A01));
    const float delta_u = det_inv * (A11 * b0 - A01 * b1);
    const float delta_v = det_inv * (-A01 * b0 + A00 * b1);
    const float u_new = clampf(u + delta_u, 1.0f, W2);
    const float v_new = clampf(v + delta_v, 1.0f, H2);
    // cost at the candidate (matching_kernels.cu:229-262)
    const Bilin Bn = bilin(u_new, v_new);
    float rn[3];
    sample<3>(img, A.W, Bn, 0, rn);
    const float new_cost = normalized_cost(rn, p);
    if (new_cost < cost) {
      u = u_new;
      v = v_new;
      lambda = (float)((double)lambda * 0.1);
      conv = new_cost < A.cost_thresh;
    } else {
      lambda = (float)((double)lambda * 10.0);
      conv = cost < A.cost_thresh;
    }
  }
  A.p_new[2 * gid] = u;
  A.p_new[2 * gid + 1] = v;
  A.converged[gid] = conv ? 1 : 0;
}

#pragma clang fp contract(on)

// ------------------------------------------------------- refine_matches --
// Scores accumulate as the reference's `score += D21[k] * D11[k]`
// (matching_kernels.cu:58-60) in feature order. fp16 descriptors (scalar_t =
// c10::Half, the reference's only caller, matching.py:80): a rounded product
// and a rounded sum per feature (c10::Half computes in float and converts back,
// score2_f16 below), the running maximum starting at 0 (libcu++'s
// numeric_limits has no c10::Half specialization: T() = 0, :47). fp32
// descriptors: nvcc contracts the float expression to one fused multiply-add
// per feature, the maximum starts at FLT_MIN. A window whose scores never
// exceed the start keeps its centre. Ties keep the first candidate in scan
// order (dilation descending, u offset outer, v inner).
template <typename T>
__device__ __forceinline__ T score_start();
template <>
__device__ __forceinline__ _Float16 score_start<_Float16>() {
  return (_Float16)0.0f;
}
template <>
__device__ __forceinline__ float score_start<float>() {
  return 1.17549435082228750797e-38f;
}
// score + a * b in the reference's arithmetic for T
__device__ __forceinline__ float score_step(float a, float b, float s) { return __builtin_fmaf(a, b, s); }
__device__ __forceinline__ _Float16 score_step(_Float16 a, _Float16 b, _Float16 s) {
#pragma clang fp contract(off)
  const _Float16 p = a * b;
  return s + p;
}

// Round 4 measured four restructurings of this kernel on one 512 x 512 pair
// (F = 24, base.yaml config; all bitwise equal to it; DESIGN.md section 4,
// profiles/r04/refine_variants.txt): this kernel 205-210 us; the windows of a
// 16 x 16 tile staged in LDS per dilation 555 us (boxes ~8x the tile's pixels
// at dilation 5, one workgroup per CU); four candidates interleaved per lane
// 269-275 us; four lanes per query 306 us; D11 rewritten as 16-B feature
// planes 305 us. Neighbouring lanes here score neighbouring queries, so one
// load instruction reads the same few D11 lines for the whole wave and a
// candidate's 48 B sit in one line: the L1 serves it; each variant lost that.
template <typename T, int FMAX>
__global__ void __launch_bounds__(kMatchThreads) refine_kernel(m3s_refine_args A) {
  const int64_t gid = (int64_t)blockIdx.x * kMatchThreads + threadIdx.x;
  if (gid >= A.B * A.N) return;
  const int64_t b = gid / A.N;
  const int64_t H = A.H, W = A.W, F = A.F;
  const T *D11 = static_cast<const T *>(A.D11) + b * H * W * F;
  const T *d21 = static_cast<const T *>(A.D21) + gid * F;
  T q[FMAX > 0 ? FMAX : 1];
  if (FMAX > 0) {
#pragma unroll
    for (int k = 0; k < FMAX; k++) q[k] = d21[k];
  }
  int64_t u0 = A.p1[2 * gid], v0 = A.p1[2 * gid + 1];
  T max_score = score_start<T>();
  int64_t u_new = u0, v_new = v0;
  for (int d = A.dilation_max; d > 0; d--) {
    const int rd = A.radius * d;
    const int diam = 2 * rd + 1;
    for (int i = 0; i < diam; i += d) {
      const int64_t u = u0 - rd + i;
      for (int j = 0; j < diam; j += d) {
        const int64_t v = v0 - rd + j;
        if (v >= 0 && v < H && u >= 0 && u < W) {
          const T *x = D11 + (v * W + u) * F;
          T score = (T)0.0f;
          if (FMAX > 0) {
#pragma unroll
            for (int k = 0; k < FMAX; k++) score = score_step(q[k], x[k], score);
          } else {
            for (int64_t k = 0; k < F; k++) score = score_step(d21[k], x[k], score);
          }
          if (score > max_score) {
            max_score = score;
            u_new = u;
            v_new = v;
          }
        }
      }
    }
    u0 = u_new;
    v0 = v_new;
  }
  A.p1_new[2 * gid] = u_new;
  A.p1_new[2 * gid + 1] = v_new;
}

// ---- round 5: refine_f16_kernel (fp16 descriptors, F in {16, 24, 32}) ----
// The same scan, the same per-candidate fp16 chain (score2_f16, the
// reference's c10::Half arithmetic) and the same first-maximum rule as
// refine_kernel (bitwise equal outputs), re-cut for the memory path:
// * XCD bands: hardware block b runs on XCD b % 8; logical block
//   (b % 8) * per + b / 8 gives each XCD one contiguous band of queries
//   (image rows), so the D11 rows its windows read (+-radius*dilation_max
//   rows) stay in that XCD's 4 MB L2 instead of every XCD streaming the
//   whole descriptor image;
// * buffer loads whose offset is past the descriptor image when the
//   candidate lies outside it (the hardware returns zeros without an access):
//   no branch per candidate, and a zero score never beats max_score (>= 0,
//   strict >), as a skipped candidate never does;
// * the next candidate's 16-B loads are issued before the current one's FMA
//   chain (one candidate in flight per lane besides the one computing);
// * the odd features are read from the high halves by op_sel (no shifts).
#ifndef M3S_REF_XCD
#define M3S_REF_XCD 1
#endif
// M3S_REF_ROWS: candidates in image-row order (measured 153 -> 136 us per
// 512 x 512 pair, profiles/r05/refine_ab_rows.txt)
#ifndef M3S_REF_ROWS
#define M3S_REF_ROWS 1
#endif
typedef unsigned int u32x4m __attribute__((ext_vector_type(4)));
constexpr int kRefFar = 0x7fff0000;  // past any descriptor image (the kernel takes images < 2^30 B): loads return zeros, and o + 16 l stays below 2^31

// Two candidates' scores in the reference's c10::Half arithmetic. The
// reference dispatches refine_matches_kernel on scalar_t = c10::Half
// (AT_DISPATCH_FLOATING_TYPES_AND_HALF, matching_kernels.cu:103; matching.py:80
// passes .half() descriptors), and c10::Half's operators compute in float and
// convert back (c10/util/Half-inl.h): `score += a * b` (:58-60) is
// p = Half(float(a) * float(b)), score = Half(float(score) + float(p)) -- a
// rounded product and a rounded sum per feature, in feature order, with no
// contraction across the conversions. On gfx950: v_pk_mul_f16 forms two
// features' products at once (a product of two halves is exact in fp32, so
// its one rounding equals the reference's multiply-then-convert), and
// v_add_f16 adds them in order (fp32 carries >= 2 * 11 + 2 bits, so the
// float add then convert equals the correctly rounded half add).
// Parity unpinned against reference outputs (no fixtures):
// this follows the source semantics.
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
template <int NL>
__device__ __forceinline__ void score2_f16(const h2v (&q)[4 * NL], const u32x4m (&xa)[NL], const u32x4m (&xb)[NL],
                                           _Float16 &sa, _Float16 &sb) {
#pragma clang fp contract(off)
  _Float16 a = 0, b = 0;
#pragma unroll
  for (int w = 0; w < 4 * NL; w++) {
    const h2v pa = q[w] * __builtin_bit_cast(h2v, (unsigned)xa[w >> 2][w & 3]);
    const h2v pb = q[w] * __builtin_bit_cast(h2v, (unsigned)xb[w >> 2][w & 3]);
    a = a + pa.x;
    b = b + pb.x;
    a = a + pa.y;
    b = b + pb.y;
  }
  sa = a, sb = b;
}

template <int FMAX, int NR>
__global__ void __launch_bounds__(kMatchThreads) refine_f16_kernel(m3s_refine_args A, int per_xcd) {
  constexpr int NL = FMAX / 8;  // 16-B loads per descriptor
  constexpr int N1 = 2 * NR + 1, NN = N1 * N1;
  constexpr int F2 = FMAX * 2;  // bytes per descriptor
  const int bh = (int)blockIdx.x;
  const int64_t lb = M3S_REF_XCD ? (int64_t)(bh & 7) * per_xcd + (bh >> 3) : bh;
  const int64_t gid = lb * kMatchThreads + threadIdx.x;
  if (gid >= A.B * A.N) return;
  const int64_t b = gid / A.N;
  const int H = (int)A.H, W = (int)A.W;
  // one wave-uniform resource over every batch's image (a per-batch base
  // would not be uniform: a wave may straddle two batches)
  const __amdgpu_buffer_rsrc_t R = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void *>(A.D11), 0, (int)(A.B * A.H * A.W * F2), 0x00020000);
  const int base = (int)(b * A.H * A.W * F2);
  h2v q[4 * NL];
  {
    const u32x4m *d21 = reinterpret_cast<const u32x4m *>(static_cast<const _Float16 *>(A.D21) + gid * FMAX);
#pragma unroll
    for (int l = 0; l < NL; l++) {
      const u32x4m v = d21[l];
#pragma unroll
      for (int k = 0; k < 4; k++) q[4 * l + k] = __builtin_bit_cast(h2v, (unsigned)v[k]);
    }
  }
  const int64_t pu = A.p1[2 * gid], pv = A.p1[2 * gid + 1];
  // a centre this far out has no candidate inside the image at any dilation
  // (radius * dilation_max < 2^20): the reference returns it unchanged
  const bool far = pu < -(1 << 30) || pu > (1 << 30) || pv < -(1 << 30) || pv > (1 << 30);
  int u0 = far ? -(1 << 30) : (int)pu, v0 = far ? -(1 << 30) : (int)pv;
  // ::cuda::std::numeric_limits<c10::Half>::min() (:47): libcu++ has no
  // specialization for c10::Half, so the primary template's T() = 0
  _Float16 max_score = (_Float16)0.0f;
  bool moved = false;
  for (int d = A.dilation_max; d > 0; d--) {
    const int rd = NR * d;
    const int ub = u0 - rd, vb = v0 - rd;
    // candidate c = i * N1 + j: u = ub + i d (outer), v = vb + j d (inner)
    // (bitwise & / selects only: a short-circuit && becomes a branch per candidate)
    unsigned uok = 0, vok = 0;
#pragma unroll
    for (int k = 0; k < N1; k++) {
      uok |= ((unsigned)(ub + k * d) < (unsigned)W ? 1u : 0u) << k;
      vok |= ((unsigned)(vb + k * d) < (unsigned)H ? 1u : 0u) << k;
    }
    // offsets stepped by wave-uniform increments (no per-candidate products)
    // unsigned: a centre far outside wraps (every candidate is then masked)
    const unsigned o0 = (unsigned)base + ((unsigned)vb * (unsigned)W + (unsigned)ub) * (unsigned)F2;
    const unsigned du = (unsigned)(d * F2), dv = (unsigned)d * (unsigned)W * (unsigned)F2;
    unsigned oi = o0, oij = o0;  // offset of the line start and of the last candidate formed
    // processing position p -> candidate (i, j): scan order (i outer) or, with
    // M3S_REF_ROWS, image rows (j outer: consecutive candidates of a wave are
    // the same row shifted by d pixels, so their lines are still in L1)
    auto cand_i = [](int p) { return M3S_REF_ROWS ? p % N1 : p / N1; };
    auto cand_j = [](int p) { return M3S_REF_ROWS ? p / N1 : p % N1; };
    auto load = [&](int p, u32x4m (&x)[NL]) {  // p in order; p >= NN: the pair's dummy (zeros)
      const int i = cand_i(p), j = cand_j(p);
      if (p > 0 && p < NN) {
        if (p % N1 == 0) oi += M3S_REF_ROWS ? dv : du, oij = oi;
        else oij += M3S_REF_ROWS ? du : dv;
      }
      const unsigned ok = p < NN ? (uok >> i) & (vok >> j) & 1u : 0u;
      const int o = ok ? (int)oij : kRefFar;
#pragma unroll
      for (int l = 0; l < NL; l++) x[l] = __builtin_amdgcn_raw_buffer_load_b128(R, o + 16 * l, 0, 0);
    };
    // pairs of candidates; the next pair's loads go out before this pair is scored
    u32x4m x[2][2][NL];
    load(0, x[0][0]);
    load(1, x[0][1]);
    int best = -1;
#pragma unroll
    for (int c = 0; c < NN; c += 2) {
      const int s = (c >> 1) & 1;
      if (c + 2 < NN) {
        load(c + 2, x[s ^ 1][0]);
        load(c + 3, x[s ^ 1][1]);
      }
      _Float16 sa, sb;
      score2_f16<NL>(q, x[s][0], x[s][1], sa, sb);
      // scan index of the two (the reference's order: u offset outer); in row
      // order a tie keeps the smaller scan index, as the reference's first
      // maximum (a score equal to the initial minimum never wins)
      const int ca = cand_i(c) * N1 + cand_j(c), cb = cand_i(c + 1) * N1 + cand_j(c + 1);
      const bool wa = sa > max_score || (M3S_REF_ROWS && sa == max_score && best >= 0 && ca < best);
      max_score = wa ? sa : max_score;
      best = wa ? ca : best;
      const bool wb = sb > max_score || (M3S_REF_ROWS && sb == max_score && best >= 0 && cb < best);
      max_score = wb ? sb : max_score;
      best = wb ? cb : best;
      __builtin_amdgcn_sched_barrier(0);  // one pair in flight: no loads hoisted further up
    }
    if (best >= 0) {
      moved = true;
      u0 = ub + (best / N1) * d;
      v0 = vb + (best % N1) * d;
    }
  }
  A.p1_new[2 * gid] = moved ? (int64_t)u0 : pu;
  A.p1_new[2 * gid + 1] = moved ? (int64_t)v0 : pv;
}

#ifndef M3S_REF_V2
#define M3S_REF_V2 1
#endif
template <typename T>
int launch_refine(const m3s_refine_args &a, hipStream_t st) {
  const unsigned blocks = (unsigned)((a.B * a.N + kMatchThreads - 1) / kMatchThreads);
  if (M3S_REF_V2 && sizeof(T) == 2 && (a.F == 16 || a.F == 24 || a.F == 32) && a.radius == 3 &&
      a.B * a.H * a.W * a.F * 2 < (1ll << 30) && a.dilation_max < (1 << 16) && a.H < (1 << 20) &&
      a.W < (1 << 20)) {
    const int per = (int)((blocks + 7) / 8);
    const unsigned grid = M3S_REF_XCD ? 8u * (unsigned)per : blocks;
    switch (a.F) {
      case 16: refine_f16_kernel<16, 3><<<grid, kMatchThreads, 0, st>>>(a, per); break;
      case 24: refine_f16_kernel<24, 3><<<grid, kMatchThreads, 0, st>>>(a, per); break;
      default: refine_f16_kernel<32, 3><<<grid, kMatchThreads, 0, st>>>(a, per); break;
    }
    return launch_status();
  }
  switch (a.F) {  // descriptor width in registers for the common sizes
    case 16: refine_kernel<T, 16><<<blocks, kMatchThreads, 0, st>>>(a); break;
    case 24: refine_kernel<T, 24><<<blocks, kMatchThreads, 0, st>>>(a); break;
    case 32: refine_kernel<T, 32><<<blocks, kMatchThreads, 0, st>>>(a); break;
    default: refine_kernel<T, 0><<<blocks, kMatchThreads, 0, st>>>(a); break;
  }
  return launch_status();
}

}  // namespace

extern "C" {

int m3s_iter_proj(const m3s_iter_proj_args *a, void *stream) {
  if (!a || !a->rays_img || !a->pts_3d_norm || !a->p_init || !a->p_new || !a->converged) return M3S_EINVAL;
  if (a->B < 0 || a->N < 0 || a->H < 3 || a->W < 3 || a->max_iter < 0) return M3S_EINVAL;
  if (a->B * a->N == 0) return M3S_OK;
  const unsigned blocks = (unsigned)((a->B * a->N + kMatchThreads - 1) / kMatchThreads);
  iter_proj_kernel<<<blocks, kMatchThreads, 0, static_cast<hipStream_t>(stream)>>>(*a);
  return launch_status();
}

int m3s_refine_matches(const m3s_refine_args *a, void *stream) {
  if (!a || !a->D11 || !a->D21 || !a->p1 || !a->p1_new) return M3S_EINVAL;
  if (a->B < 0 || a->N < 0 || a->H < 1 || a->W < 1 || a->F < 1 || a->radius < 0 || a->dilation_max < 0)
    return M3S_EINVAL;
  if (a->B * a->N == 0) return M3S_OK;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (a->dtype == M3S_DESC_F16) return launch_refine<_Float16>(*a, st);
  if (a->dtype == M3S_DESC_F32) return launch_refine<float>(*a, st);
  return M3S_EINVAL;
}

}  // extern "C"
