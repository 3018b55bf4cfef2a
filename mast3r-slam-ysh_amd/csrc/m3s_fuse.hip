// m3s_fuse.hip — MI355X (gfx950) kernels either side of the GN/matching path
// (include/m3s_fuse.h): keyframe pointmap fusion and the iter_proj input prep.
//
// Both are pure streaming elementwise passes (HBM-bound; a 512x512 pointmap
// is 3 MB), one lane per pixel, so each replaces a chain of 5-12 torch
// kernels (and their intermediate tensors) of the reference with one launch.
// Element arithmetic follows the reference's torch expressions operation by
// operation without FMA contraction.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "m3s_device.h"
#include "m3s_fuse.h"
#include "m3s_gn.h"

using namespace m3s;

namespace {

constexpr int kFuseThreads = 256;

inline int launch_status() { return hipGetLastError() == hipSuccess ? M3S_OK : M3S_ELAUNCH; }

#pragma clang fp contract(off)

// Frame.update_pointmap (frame.py:41-100) on Xkk = T_CkCf.act(Xkf)
// (tracker.py:98-99) for an already initialised keyframe.
__global__ void __launch_bounds__(kFuseThreads) fuse_pointmap_kernel(m3s_fuse_args A) {
  const int64_t p = (int64_t)blockIdx.x * kFuseThreads + threadIdx.x;
  if (p >= A.HW) return;
  float x[3] = {A.X_new[3 * p], A.X_new[3 * p + 1], A.X_new[3 * p + 2]};
  if (A.T) {  // lietorch Sim3 act: s R(q) x + t (gn_kernels.cu:232-250 form)
    const Sim3f T = load_sim3(A.T);
    float y[3];
    act(T, x, y);
    x[0] = y[0], x[1] = y[1], x[2] = y[2];
  }
  const float cn = A.C_new[p];
  const float co = A.C[p];
  float *xc = A.X_canon + 3 * p;
  if (A.mode == M3S_FILTER_WEIGHTED_POINTMAP) {  // frame.py:73-76
    const float den = co + cn;
#pragma unroll
    for (int k = 0; k < 3; k++) xc[k] = ((co * xc[k]) + (cn * x[k])) / den;
    A.C[p] = co + cn;
  } else if (A.mode == M3S_FILTER_INDEP_CONF) {  // frame.py:68-72
    if (cn > co) {
      xc[0] = x[0], xc[1] = x[1], xc[2] = x[2];
      A.C[p] = cn;
    }
  } else if (A.mode == M3S_FILTER_WEIGHTED_SPHERICAL) {  // frame.py:78-100
    // cartesian_to_spherical: r = ||P||, phi = atan2(y, x), theta = acos(z / r)
    float so[3], sn[3];
    {
      const float r = sqrtf(xc[0] * xc[0] + xc[1] * xc[1] + xc[2] * xc[2]);
      so[0] = r, so[1] = atan2f(xc[1], xc[0]), so[2] = acosf(xc[2] / r);
    }
    {
      const float r = sqrtf(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
      sn[0] = r, sn[1] = atan2f(x[1], x[0]), sn[2] = acosf(x[2] / r);
    }
    const float den = co + cn;
    float sp[3];
#pragma unroll
    for (int k = 0; k < 3; k++) sp[k] = ((co * so[k]) + (cn * sn[k])) / den;
    // spherical_to_cartesian
    const float st = sinf(sp[2]);
    xc[0] = sp[0] * st * cosf(sp[1]);
    xc[1] = sp[0] * st * sinf(sp[1]);
    xc[2] = sp[0] * cosf(sp[2]);
    A.C[p] = co + cn;
  } else {  // recent (frame.py:59-62)
    xc[0] = x[0], xc[1] = x[1], xc[2] = x[2];
    A.C[p] = cn;
  }
}

// F.normalize(v, dim=-1): v / max(||v||, 1e-12)
__device__ __forceinline__ void unit(const float *v, float *r) {
  const float n = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  const float d = fmaxf(n, 1e-12f);
  r[0] = v[0] / d, r[1] = v[1] / d, r[2] = v[2] / d;
}

__device__ __forceinline__ int64_t reflect(int64_t i, int64_t n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

// prep_for_iter_proj (matching.py:25-49): rays = normalize(X11), Scharr x/y
// gradients /32 with reflect padding (image.py:5-38), pts = normalize(X21).
__global__ void __launch_bounds__(kFuseThreads) prep_rays_kernel(m3s_prep_rays_args A) {
  const int64_t HW = A.H * A.W;
  const int64_t g = (int64_t)blockIdx.x * kFuseThreads + threadIdx.x;
  if (g >= A.B * HW) return;
  const int64_t b = g / HW, p = g - b * HW;
  const int64_t y = p / A.W, x = p - y * A.W;
  const float *X = A.X11 + b * HW * 3;
  float r[3][3][3];  // [dy][dx][c] unit rays of the 3x3 neighbourhood
#pragma unroll
  for (int dy = 0; dy < 3; dy++) {
    const int64_t yy = reflect(y + dy - 1, A.H);
#pragma unroll
    for (int dx = 0; dx < 3; dx++) {
      const int64_t xx = reflect(x + dx - 1, A.W);
      const float *v = X + (yy * A.W + xx) * 3;
      const float vv[3] = {v[0], v[1], v[2]};
      unit(vv, r[dy][dx]);
    }
  }
  constexpr float k3 = 3.0f / 32.0f, k10 = 10.0f / 32.0f;
  float *o = A.rays_img + g * 9;
#pragma unroll
  for (int c = 0; c < 3; c++) {
    o[c] = r[1][1][c];
    o[3 + c] = -k3 * r[0][0][c] + k3 * r[0][2][c] - k10 * r[1][0][c] + k10 * r[1][2][c] - k3 * r[2][0][c] +
               k3 * r[2][2][c];
    o[6 + c] = -k3 * r[0][0][c] - k10 * r[0][1][c] - k3 * r[0][2][c] + k3 * r[2][0][c] + k10 * r[2][1][c] +
               k3 * r[2][2][c];
  }
  const float *q = A.X21 + g * 3;
  const float qq[3] = {q[0], q[1], q[2]};
  unit(qq, A.pts_norm + g * 3);
}

#pragma clang fp contract(on)

}  // namespace

extern "C" {

int m3s_fuse_pointmap(const m3s_fuse_args *a, void *stream) {
  if (!a || !a->X_canon || !a->C || !a->X_new || !a->C_new || a->HW < 0) return M3S_EINVAL;
  if (a->mode < 0 || a->mode > M3S_FILTER_WEIGHTED_SPHERICAL) return M3S_EINVAL;
  if (a->HW == 0) return M3S_OK;
  const unsigned blocks = (unsigned)((a->HW + kFuseThreads - 1) / kFuseThreads);
  fuse_pointmap_kernel<<<blocks, kFuseThreads, 0, static_cast<hipStream_t>(stream)>>>(*a);
  return launch_status();
}

int m3s_prep_rays(const m3s_prep_rays_args *a, void *stream) {
  if (!a || !a->X11 || !a->X21 || !a->rays_img || !a->pts_norm) return M3S_EINVAL;
  if (a->B < 0 || a->H < 2 || a->W < 2) return M3S_EINVAL;
  if (a->B == 0) return M3S_OK;
  const unsigned blocks = (unsigned)((a->B * a->H * a->W + kFuseThreads - 1) / kFuseThreads);
  prep_rays_kernel<<<blocks, kFuseThreads, 0, static_cast<hipStream_t>(stream)>>>(*a);
  return launch_status();
}

}  // extern "C"
