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
// Scores accumulate in the descriptor type, one fused multiply-add per
// feature in feature order (the reference's `score += D21[k] * D11[k]` on
// __half, matching_kernels.cu:65-67). The running maximum starts at the
// type's smallest positive normal (numeric_limits<T>::min(), :47): a window
// whose scores are all below it keeps its centre. Ties keep the first
// candidate in scan order (dilation descending, u offset outer, v inner).
template <typename T>
__device__ __forceinline__ T min_normal();
template <>
__device__ __forceinline__ _Float16 min_normal<_Float16>() {
  return (_Float16)6.103515625e-05f;
}
template <>
__device__ __forceinline__ float min_normal<float>() {
  return 1.17549435082228750797e-38f;
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
  T max_score = min_normal<T>();
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
            for (int k = 0; k < FMAX; k++) score = __builtin_elementwise_fma(q[k], x[k], score);
          } else {
            for (int64_t k = 0; k < F; k++) score = __builtin_elementwise_fma(d21[k], x[k], score);
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

template <typename T>
int launch_refine(const m3s_refine_args &a, hipStream_t st) {
  const unsigned blocks = (unsigned)((a.B * a.N + kMatchThreads - 1) / kMatchThreads);
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
