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

// M3S_REFINE_STAGED (A/B): 0 = the round-3 global-read kernel, 1 = windows
// staged in LDS, 2 = four candidates interleaved per lane, 3 (default) = four
// lanes per query (refine_split_kernel)
int refine_staged_knob() {
  static const int v = [] {
    const char *e = std::getenv("M3S_REFINE_STAGED");
    return e ? std::atoi(e) : 3;
  }();
  return v;
}

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

// Round 4: the window rows staged in LDS. A workgroup takes a 16 x 16 tile of
// query pixels (N = H W, query n = pixel (n % W, n / W) of image 2, whose
// matches p1 in image 1 move smoothly, so their windows overlap) or 256
// consecutive queries otherwise. Per dilation d (dilation_max .. 1) the
// workgroup reduces the bounding box of its current windows (centres +-
// radius d, clipped to the image), copies those D11 pixels into LDS with
// coalesced 16-B loads (rows of the box are contiguous in D11), and every
// lane scores its candidates from LDS; a candidate outside the box (a box too
// large for LDS is not staged at all) reads D11 directly. Each score is the
// same fp16 FMA chain in feature order and candidates keep the scan order and
// strict comparison, so the integer result is bitwise the global kernel's.
// (matching_kernels.cu:25-81.)
constexpr int kRefTile = 16;
constexpr int kRefLdsBytes = 144 * 1024;
constexpr int kRefNear = 32;  // centres within this many pixels of the anchor set the box

template <typename T, int FMAX, bool STAGE>
__global__ void __launch_bounds__(kMatchThreads) refine_lds_kernel(m3s_refine_args A, int tiles_x, int tiles_per_b,
                                                                   int tiled) {
  constexpr int EV = 16 / (int)sizeof(T);  // elements per 16-B vector
  static_assert(FMAX % EV == 0, "16-B vectors per pixel");
  constexpr int NV = FMAX / EV;            // vectors per pixel
  typedef T TV __attribute__((ext_vector_type(EV)));
  extern __shared__ __attribute__((aligned(16))) unsigned char rsm[];
  TV *Ls = reinterpret_cast<TV *>(rsm);
  __shared__ int red[8];
  const int tid = threadIdx.x;
  const int b = (int)(blockIdx.x / tiles_per_b);
  const int tb = (int)(blockIdx.x - (unsigned)b * tiles_per_b);
  const int H = (int)A.H, W = (int)A.W;
  int n;
  bool valid;
  if (tiled) {
    const int x = (tb % tiles_x) * kRefTile + tid % kRefTile, y = (tb / tiles_x) * kRefTile + tid / kRefTile;
    valid = x < W && y < H;
    n = y * W + x;
  } else {
    n = tb * kMatchThreads + tid;
    valid = n < A.N;
  }
  const int64_t gid = (int64_t)b * A.N + n;
  const TV *Dv = reinterpret_cast<const TV *>(static_cast<const T *>(A.D11) + (int64_t)b * H * W * FMAX);
  TV q[NV];
  int u0 = 0, v0 = 0;
  {
    const TV *d21 = reinterpret_cast<const TV *>(static_cast<const T *>(A.D21) + (valid ? gid : 0) * FMAX);
#pragma unroll
    for (int c = 0; c < NV; c++) q[c] = d21[c];
    if (valid) u0 = (int)A.p1[2 * gid], v0 = (int)A.p1[2 * gid + 1];
  }
  T max_score = min_normal<T>();
  int u_new = u0, v_new = v0;
  const int cap_px = kRefLdsBytes / (16 * NV);
  for (int d = A.dilation_max; d > 0; d--) {
    const int rd = A.radius * d;
    // the box of this dilation's windows over the centres near the tile's
    // anchor (its middle query, or the first valid one): a few far-off
    // matches (occluded pixels) would otherwise blow the box past LDS and
    // leave the whole tile on global reads; they read D11 directly instead
    if (tid == 0) red[0] = INT32_MAX, red[1] = INT32_MIN, red[2] = INT32_MAX, red[3] = INT32_MIN, red[4] = INT32_MAX;
    __syncthreads();
    if (valid) atomicMin(&red[4], tid == kMatchThreads / 2 + kRefTile / 2 ? -1 : tid);
    __syncthreads();
    const int at = red[4] < 0 ? kMatchThreads / 2 + kRefTile / 2 : red[4];
    if (tid == at) red[5] = u0, red[6] = v0;
    __syncthreads();
    if (valid && abs(u0 - red[5]) <= kRefNear && abs(v0 - red[6]) <= kRefNear)
      atomicMin(&red[0], u0), atomicMax(&red[1], u0), atomicMin(&red[2], v0), atomicMax(&red[3], v0);
    __syncthreads();
    const int bx0 = max(red[0] - rd, 0), bx1 = min(red[1] + rd, W - 1);
    const int by0 = max(red[2] - rd, 0), by1 = min(red[3] + rd, H - 1);
    const int bw = bx1 - bx0 + 1, bh = by1 - by0 + 1;
    const bool staged = STAGE && red[0] <= red[1] && bw > 0 && bh > 0 && bw * bh <= cap_px;
    __syncthreads();  // red read by every lane before the next dilation rewrites it
    if (staged) {
      // box rows are contiguous in D11: 16-B loads, four in flight per lane
      const int nvec = bw * bh * NV;
      for (int i0 = 0; i0 < nvec; i0 += 4 * kMatchThreads) {
        TV v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int i = min(i0 + u * kMatchThreads + tid, nvec - 1);
          const int px = i / NV, c = i - px * NV;
          const int yy = by0 + px / bw, xx = bx0 + px % bw;
          v[u] = Dv[(yy * W + xx) * NV + c];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int i = i0 + u * kMatchThreads + tid;
          if (i < nvec) Ls[i] = v[u];
        }
      }
    }
    __syncthreads();
    if (valid) {
      // candidates in scan order (u offset outer, v inner), four v offsets at a
      // time: their FMA chains run interleaved, then they are compared in order
      const int nw = 2 * A.radius + 1;
      constexpr int G = 4;
      for (int i = 0; i < nw; i++) {
        const int u = u0 - rd + i * d;
        const bool ucol = u >= 0 && u < W, ubox = staged && u >= bx0 && u <= bx1;
        for (int j0 = 0; j0 < nw; j0 += G) {
          TV x[G][NV];
          bool ok[G];
#pragma unroll
          for (int g = 0; g < G; g++) {
            const int v = v0 - rd + (j0 + g) * d;
            ok[g] = j0 + g < nw && ucol && v >= 0 && v < H;
            if (ubox && v >= by0 && v <= by1) {
              const TV *pl = Ls + ((v - by0) * bw + (u - bx0)) * NV;
#pragma unroll
              for (int c = 0; c < NV; c++) x[g][c] = pl[c];
            } else {  // (a candidate outside the image reads pixel 0 and is discarded)
              const TV *pg = Dv + (ok[g] ? (v * W + u) * NV : 0);
#pragma unroll
              for (int c = 0; c < NV; c++) x[g][c] = pg[c];
            }
          }
          T score[G];
#pragma unroll
          for (int g = 0; g < G; g++) score[g] = (T)0.0f;
#pragma unroll
          for (int k = 0; k < FMAX; k++)
#pragma unroll
            for (int g = 0; g < G; g++) score[g] = __builtin_elementwise_fma(q[k / EV][k % EV], x[g][k / EV][k % EV], score[g]);
#pragma unroll
          for (int g = 0; g < G; g++) {
            if (ok[g] && score[g] > max_score) {
              max_score = score[g];
              u_new = u;
              v_new = v0 - rd + (j0 + g) * d;
            }
          }
        }
      }
    }
    u0 = u_new;
    v0 = v_new;
    __syncthreads();  // the box is read before the next dilation restages it
  }
  if (valid) {
    A.p1_new[2 * gid] = u_new;
    A.p1_new[2 * gid + 1] = v_new;
  }
}

// Round 4 (default, M3S_REFINE_STAGED=3): S = 4 lanes per query. The round-3
// kernel (one lane per query, ~245 candidates in a row, each a dependent
// 24-FMA chain behind its loads) had only ~4 waves per SIMD for a 512 x 512
// pair: latency-bound. Here lane s of a query's group scores the candidates
// c = s, s + S, ... of each dilation (two at a time), keeps the first
// occurrence of its best score (strict >, ascending c), and the group
// combines (higher score; equal scores: lower c) with two lane shuffles: the
// first candidate in scan order that attains the dilation's maximum, taken if
// it beats the running maximum - exactly the sequential scan's result
// (strict >, ties to the earlier candidate). Same fp16 FMA chain per score.
constexpr int kRefS = 4;
template <typename T, int FMAX>
__global__ void __launch_bounds__(kMatchThreads) refine_split_kernel(m3s_refine_args A) {
  constexpr int EV = 16 / (int)sizeof(T);
  constexpr int NV = FMAX / EV;
  typedef T TV __attribute__((ext_vector_type(EV)));
  const int tid = threadIdx.x, sub = tid % kRefS;
  const int64_t gq = (int64_t)blockIdx.x * (kMatchThreads / kRefS) + tid / kRefS;  // (batch, query)
  const bool valid = gq < A.B * A.N;
  const int64_t gid = valid ? gq : 0;
  const int64_t b = gid / A.N;
  const int H = (int)A.H, W = (int)A.W;
  const TV *Dv = reinterpret_cast<const TV *>(static_cast<const T *>(A.D11) + b * (int64_t)H * W * FMAX);
  TV q[NV];
  {
    const TV *d21 = reinterpret_cast<const TV *>(static_cast<const T *>(A.D21) + gid * FMAX);
#pragma unroll
    for (int c = 0; c < NV; c++) q[c] = d21[c];
  }
  int u0 = (int)A.p1[2 * gid], v0 = (int)A.p1[2 * gid + 1];
  T max_score = min_normal<T>();
  const int nw = 2 * A.radius + 1, ncand = nw * nw;
  for (int d = A.dilation_max; d > 0; d--) {
    const int rd = A.radius * d;
    T best = (T)0.0f;
    int bi = INT32_MAX;  // no candidate yet
    for (int c0 = sub; c0 < ncand; c0 += 2 * kRefS) {
      int cc[2];
      bool ok[2];
      TV x[2][NV];
#pragma unroll
      for (int g = 0; g < 2; g++) {
        cc[g] = c0 + g * kRefS;
        const int i = cc[g] / nw, j = cc[g] - (cc[g] / nw) * nw;
        const int u = u0 - rd + i * d, v = v0 - rd + j * d;
        ok[g] = cc[g] < ncand && u >= 0 && u < W && v >= 0 && v < H;
        const TV *pg = Dv + (ok[g] ? (v * W + u) * NV : 0);
#pragma unroll
        for (int c = 0; c < NV; c++) x[g][c] = pg[c];
      }
      T sc[2] = {(T)0.0f, (T)0.0f};
#pragma unroll
      for (int k = 0; k < FMAX; k++)
#pragma unroll
        for (int g = 0; g < 2; g++) sc[g] = __builtin_elementwise_fma(q[k / EV][k % EV], x[g][k / EV][k % EV], sc[g]);
#pragma unroll
      for (int g = 0; g < 2; g++)
        if (ok[g] && (bi == INT32_MAX || sc[g] > best)) best = sc[g], bi = cc[g];
    }
    // the group's first maximum (lanes of a group are adjacent: xor 1, 2)
#pragma unroll
    for (int o = 1; o < kRefS; o <<= 1) {
      const float bo = __shfl_xor((float)best, o, 64);
      const int io = __shfl_xor(bi, o, 64);
      const T bt = (T)bo;
      if (io != INT32_MAX && (bi == INT32_MAX || bt > best || (bt == best && io < bi))) best = bt, bi = io;
    }
    if (bi != INT32_MAX && best > max_score) {
      max_score = best;
      u0 = u0 - rd + (bi / nw) * d;
      v0 = v0 - rd + (bi - (bi / nw) * nw) * d;
    }
  }
  if (valid && sub == 0) {
    A.p1_new[2 * gid] = u0;
    A.p1_new[2 * gid + 1] = v0;
  }
}

template <typename T>
int launch_refine(const m3s_refine_args &a, hipStream_t st) {
  // LDS-staged windows for 16-B multiples of descriptor bytes (f16: F = 8k)
  // (int image arithmetic: H W F and the pixel coordinates fit 31 bits)
  const bool vec = (a.F * (int64_t)sizeof(T)) % 16 == 0 && (a.F == 16 || a.F == 24 || a.F == 32) &&
                   reinterpret_cast<uintptr_t>(a.D11) % 16 == 0 && reinterpret_cast<uintptr_t>(a.D21) % 16 == 0 &&
                   a.H * a.W * a.F < (int64_t)1 << 30 && a.N < (int64_t)1 << 30;
  if (vec && refine_staged_knob() == 3) {
    const unsigned blocks = (unsigned)((a.B * a.N + kMatchThreads / kRefS - 1) / (kMatchThreads / kRefS));
    switch (a.F) {
      case 16: refine_split_kernel<T, 16><<<blocks, kMatchThreads, 0, st>>>(a); break;
      case 24: refine_split_kernel<T, 24><<<blocks, kMatchThreads, 0, st>>>(a); break;
      default: refine_split_kernel<T, 32><<<blocks, kMatchThreads, 0, st>>>(a); break;
    }
    return launch_status();
  }
  if (vec && refine_staged_knob() != 0) {
    const bool tiled = a.N == a.H * a.W;
    const int tiles_x = (int)((a.W + kRefTile - 1) / kRefTile);
    const int tiles_per_b = tiled ? tiles_x * (int)((a.H + kRefTile - 1) / kRefTile)
                                  : (int)((a.N + kMatchThreads - 1) / kMatchThreads);
    const unsigned blocks = (unsigned)(a.B * tiles_per_b);
    static bool attr = false;
    if (!attr) {
      for (const void *f : {reinterpret_cast<const void *>(refine_lds_kernel<T, 16, true>),
                            reinterpret_cast<const void *>(refine_lds_kernel<T, 24, true>),
                            reinterpret_cast<const void *>(refine_lds_kernel<T, 32, true>)})
        (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kRefLdsBytes);
      attr = true;
    }
    if (refine_staged_knob() == 1) {
      switch (a.F) {
        case 16: refine_lds_kernel<T, 16, true><<<blocks, kMatchThreads, kRefLdsBytes, st>>>(a, tiles_x, tiles_per_b, tiled); break;
        case 24: refine_lds_kernel<T, 24, true><<<blocks, kMatchThreads, kRefLdsBytes, st>>>(a, tiles_x, tiles_per_b, tiled); break;
        default: refine_lds_kernel<T, 32, true><<<blocks, kMatchThreads, kRefLdsBytes, st>>>(a, tiles_x, tiles_per_b, tiled); break;
      }
    } else {
      switch (a.F) {
        case 16: refine_lds_kernel<T, 16, false><<<blocks, kMatchThreads, 0, st>>>(a, tiles_x, tiles_per_b, tiled); break;
        case 24: refine_lds_kernel<T, 24, false><<<blocks, kMatchThreads, 0, st>>>(a, tiles_x, tiles_per_b, tiled); break;
        default: refine_lds_kernel<T, 32, false><<<blocks, kMatchThreads, 0, st>>>(a, tiles_x, tiles_per_b, tiled); break;
      }
    }
    return launch_status();
  }
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
