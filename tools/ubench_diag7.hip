// Micro-benchmark of the 7x7 DIAG factor of sparse_llt_kernel (gfx950): the
// same algorithm as m3s_gn.hip's diag_factor<false, RL=true> (restated here,
// hot code, one wave alone on its SIMD), with shader-clock stamps after the
// entry -> row relayout, after the pivot loop and after the stores, and
// variants of the pivot loop.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_diag7.hip -o variants/ubench_diag7
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double rsqrt_nr(double d) {
  double x = __builtin_amdgcn_rsq(d);
  const double hd = 0.5 * d;
  x = x * (1.5 - hd * x * x);
  return x;
}
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// VAR 0: the product form (row layout, readlane broadcasts, W by columns)
// VAR 1: the same, the row -> per-lane relayout through readlanes of the
//        entry layout instead of an LDS round trip
template <int VAR>
__device__ __noinline__ bool diag7(double v, double *Lb, double *Di, double *scr, int lane, long long *ts) {
  const int l7 = (lane < 7 ? lane : 0) * 7;
  double a[7];
  if (VAR == 1) {
#pragma unroll
    for (int qq = 0; qq < 7; qq++) {
      double s = 0.0;
#pragma unroll
      for (int r = 0; r < 7; r++) {
        const double e = readlane_d(v, 7 * r + qq);
        s = lane == r ? e : s;
      }
      a[qq] = s;
    }
  } else {
    if (lane < 49) scr[lane] = v;
    wave_lds_fence();
#pragma unroll
    for (int qq = 0; qq < 7; qq++) a[qq] = scr[l7 + qq];
    wave_lds_fence();
  }
  ts[1] = clock64();
  double sw[7], wcol[7];
#pragma unroll
  for (int r = 0; r < 7; r++) sw[r] = (r == lane) ? 1.0 : 0.0;
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 7; j++) {
    const double d = readlane_d(a[j], j);
    bad |= !(d > 0.0);
    const double inv = rsqrt_nr(d);
    a[j] *= inv;
    wcol[j] = sw[j] * inv;
#pragma unroll
    for (int cc = j + 1; cc < 7; cc++) {
      const double lcj = readlane_d(a[j], cc);
      a[cc] -= a[j] * lcj;
      sw[cc] -= lcj * wcol[j];
    }
  }
  ts[2] = clock64();
  if (lane < 7) {
#pragma unroll
    for (int qq = 0; qq < 7; qq++) {
      Lb[lane * 7 + qq] = (qq <= lane) ? a[qq] : 0.0;
      Di[qq * 7 + lane] = wcol[qq];
    }
  }
  return bad;
}

template <int VAR>
__global__ void k_diag7(double *out, long long *t) {
  __shared__ double Lb[49], Di[49], scr[64];
  const int lane = threadIdx.x;
  const int r = lane / 7, c = lane % 7;
  double v = lane < 49 ? (r == c ? 10.0 + r : 1.0 / (2 + r + c)) : 0.0;
  long long ts[3];
  for (int it = 0; it < 6; it++) {
    const long long c0 = clock64();
    const bool bad = diag7<VAR>(v, Lb, Di, scr, lane, ts);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    const long long c1 = clock64();
    if (lane == 0 && it == 5) {
      t[0] = ts[1] - c0, t[1] = ts[2] - ts[1], t[2] = c1 - ts[2], t[3] = c1 - c0;
    }
    v += bad ? 1.0 : (lane < 49 ? Lb[lane] * 1e-12 + Di[lane] * 1e-12 : 0.0);
  }
  out[lane] = v;
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main() {
  double *out;
  long long *t, h[4];
  CK(hipMalloc(&out, 64 * 8));
  CK(hipMalloc(&t, 32));
  for (int rep = 0; rep < 2; rep++) {
    k_diag7<0><<<1, 64>>>(out, t);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, t, 32, hipMemcpyDeviceToHost));
    printf("7x7 DIAG (LDS relayout):      relayout %lld  pivots %lld  stores %lld  total %lld cycles\n", h[0], h[1], h[2], h[3]);
    k_diag7<1><<<1, 64>>>(out, t);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, t, 32, hipMemcpyDeviceToHost));
    printf("7x7 DIAG (readlane relayout): relayout %lld  pivots %lld  stores %lld  total %lld cycles\n", h[0], h[1], h[2], h[3]);
  }
  return 0;
}
