// Micro-benchmarks, part 2 (gfx950): straight-line code run cold vs hot
// (instruction-cache misses in one-shot chain code), dependent f64 FMA and
// v_rsq_f64 latencies, and the dense tail's 16x16 diagonal factor (the same
// algorithm as m3s_gn.hip's tail_diag_mfma_t, restated here) per call, first
// call vs later calls.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_icache.hip -o variants/ubench_icache
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

#define R4(x) x x x x
#define R16(x) R4(R4(x))
#define R256(x) R16(R16(x))

// 2 x 256 independent VALU ops (4 chains): cold first pass, hot second pass
__global__ void k_icache(double *out, long long *t) {
  double a = threadIdx.x, b = 1.0001, c = 0.5, d = 0.25;
  for (int pass = 0; pass < 3; pass++) {
    const long long c0 = clock64();
    asm volatile(R256("v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4\n")
                 : "+v"(a), "+v"(c), "+v"(d), "+v"(b)
                 : "v"(1.0));
    const long long c1 = clock64();
    if (threadIdx.x == 0) t[pass] = c1 - c0;
  }
  out[threadIdx.x] = a + b + c + d;
}

__global__ void k_fma_dep(double *out, long long *t, int n) {
  double a = threadIdx.x * 1e-3, b = 1.0000001;
  const long long c0 = clock64();
  for (int i = 0; i < n; i++) a = __builtin_fma(a, b, 1e-9);
  const long long c1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) t[0] = c1 - c0;
}

__global__ void k_rsq_dep(double *out, long long *t, int n) {
  double a = 1.0 + threadIdx.x * 1e-3;
  const long long c0 = clock64();
  for (int i = 0; i < n; i++) a = __builtin_amdgcn_rsq(a) + 0.5;
  const long long c1 = clock64();
  out[threadIdx.x] = a;
  if (threadIdx.x == 0) t[0] = c1 - c0;
}

__device__ __forceinline__ double rsqrt_nr(double d) {
  double x = __builtin_amdgcn_rsq(d);
  const double hd = 0.5 * d;
  x = x * (1.5 - hd * x * x);
  x = x * (1.5 - hd * x * x);
  return x;
}
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// the round-2 blocked diagonal factor (4 steps of 4 columns), FULL tile
__device__ __noinline__ bool diag16(f64x4 a, double (*Wk)[17], int lane) {
  __shared__ double xd[4][16], xw[4][16];
  const int lr = lane & 15, lk = lane >> 4;
  f64x4 M;
#pragma unroll
  for (int r = 0; r < 4; r++) M[r] = (lk + 4 * r == lr) ? 1.0 : 0.0;
  bool bad = false;
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const int c0 = 4 * b;
    if (lr >= c0 && lr < c0 + 4) xd[b][4 * lk + lr - c0] = a[b];
    wave_lds_fence();
    double D[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) D[i][j] = xd[b][4 * i + j];
    double L[4][4], Wd[4][4], iv[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      double d = D[j][j];
      bad |= !(d > 0.0);
      d = d > 0.0 ? d : 1.0;
      iv[j] = rsqrt_nr(d);
#pragma unroll
      for (int i = j + 1; i < 4; i++) L[i][j] = D[i][j] * iv[j];
#pragma unroll
      for (int i = j + 1; i < 4; i++)
#pragma unroll
        for (int k = j + 1; k <= i; k++) D[i][k] -= L[i][j] * L[k][j];
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      Wd[i][i] = iv[i];
#pragma unroll
      for (int j = 0; j < i; j++) {
        double s = 0.0;
#pragma unroll
        for (int k = j; k < i; k++) s += L[i][k] * Wd[k][j];
        Wd[i][j] = -s * iv[i];
      }
    }
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int k = 0; k < 4; k++) xw[b][4 * i + k] = k <= i ? Wd[i][k] : 0.0;
    }
    wave_lds_fence();
    const double wpad = lr < 4 ? xw[b][4 * lr + lk] : 0.0;
    const double a1 = (lr >= c0 && lr < c0 + 4) ? xw[b][4 * (lr - c0) + lk] - (lr - c0 == lk ? 1.0 : 0.0) : 0.0;
    double p = __builtin_amdgcn_mfma_f64_16x16x4f64(wpad, a[b], f64x4{0.0, 0.0, 0.0, 0.0}, 0, 0, 0)[0];
    p = (lr >= c0) ? p : 0.0;
    a = __builtin_amdgcn_mfma_f64_16x16x4f64(-p, p, a, 0, 0, 0);
    const f64x4 Y = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, M[b], M, 0, 0, 0);
    const double a2 = (lr >= c0 + 4) ? -p : 0.0;
    M = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, Y[b], Y, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) Wk[lk + 4 * r][lr] = M[r];
  return bad;
}

// the same with shader-clock stamps per step phase (ps[5 b + 0..4])
__device__ __noinline__ bool diag16s(f64x4 a, double (*Wk)[17], int lane, long long *ps) {
  __shared__ double xd[4][16], xw[4][16];
  const int lr = lane & 15, lk = lane >> 4;
  f64x4 M;
#pragma unroll
  for (int r = 0; r < 4; r++) M[r] = (lk + 4 * r == lr) ? 1.0 : 0.0;
  bool bad = false;
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const int c0 = 4 * b;
    if (lr >= c0 && lr < c0 + 4) xd[b][4 * lk + lr - c0] = a[b];
    wave_lds_fence();
    ps[5 * b + 0] = clock64();
    double D[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) D[i][j] = xd[b][4 * i + j];
    double L[4][4], Wd[4][4], iv[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      double d = D[j][j];
      bad |= !(d > 0.0);
      d = d > 0.0 ? d : 1.0;
      iv[j] = rsqrt_nr(d);
#pragma unroll
      for (int i = j + 1; i < 4; i++) L[i][j] = D[i][j] * iv[j];
#pragma unroll
      for (int i = j + 1; i < 4; i++)
#pragma unroll
        for (int k = j + 1; k <= i; k++) D[i][k] -= L[i][j] * L[k][j];
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      Wd[i][i] = iv[i];
#pragma unroll
      for (int j = 0; j < i; j++) {
        double s = 0.0;
#pragma unroll
        for (int k = j; k < i; k++) s += L[i][k] * Wd[k][j];
        Wd[i][j] = -s * iv[i];
      }
    }
    __builtin_amdgcn_s_waitcnt(0);
    ps[5 * b + 1] = clock64() + (long long)(Wd[3][0] != 0.0 ? 0 : 1);
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 4; i++)
#pragma unroll
        for (int k = 0; k < 4; k++) xw[b][4 * i + k] = k <= i ? Wd[i][k] : 0.0;
    }
    wave_lds_fence();
    const double wpad = lr < 4 ? xw[b][4 * lr + lk] : 0.0;
    const double a1 = (lr >= c0 && lr < c0 + 4) ? xw[b][4 * (lr - c0) + lk] - (lr - c0 == lk ? 1.0 : 0.0) : 0.0;
    ps[5 * b + 2] = clock64() + (long long)(wpad + a1 != 0.0 ? 0 : 1);
    double p = __builtin_amdgcn_mfma_f64_16x16x4f64(wpad, a[b], f64x4{0.0, 0.0, 0.0, 0.0}, 0, 0, 0)[0];
    ps[5 * b + 3] = clock64() + (long long)(p != 0.0 ? 0 : 1);
    p = (lr >= c0) ? p : 0.0;
    a = __builtin_amdgcn_mfma_f64_16x16x4f64(-p, p, a, 0, 0, 0);
    const f64x4 Y = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, M[b], M, 0, 0, 0);
    const double a2 = (lr >= c0 + 4) ? -p : 0.0;
    M = __builtin_amdgcn_mfma_f64_16x16x4f64(a2, Y[b], Y, 0, 0, 0);
    ps[5 * b + 4] = clock64() + (long long)(a[b < 3 ? b + 1 : 3] != 0.0 ? 0 : 1);
  }
#pragma unroll
  for (int r = 0; r < 4; r++) Wk[lk + 4 * r][lr] = M[r];
  return bad;
}

__global__ void k_diag(double *out, long long *t) {
  __shared__ double Wk[16][17];
  const int lane = threadIdx.x, lr = lane & 15, lk = lane >> 4;
  f64x4 a;
#pragma unroll
  for (int r = 0; r < 4; r++) a[r] = (lk + 4 * r == lr) ? 20.0 : 1.0 / (1 + lr + lk + 4 * r);
  for (int c = 0; c < 4; c++) {
    const long long c0 = clock64();
    const bool bad = diag16(a, Wk, lane);
    wave_lds_fence();
    const long long c1 = clock64();
    if (lane == 0) t[c] = c1 - c0;
    a[0] += bad ? 1.0 : Wk[lr][lk] * 1e-12;
  }
  long long ps[20];
  const long long s0 = clock64();
  (void)diag16s(a, Wk, lane, ps);
  if (lane == 0)
    for (int i = 0; i < 20; i++) t[4 + i] = ps[i] - s0;
  out[lane] = a[0] + a[1] + a[2] + a[3];
}

// accuracy of v_rsq_f64 and of one / two Newton steps on it, vs 1/sqrt in fp64
__global__ void k_rsq_acc(double *err, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  double e0 = 0.0, e1 = 0.0, e2 = 0.0;
  for (int i = t; i < n; i += gridDim.x * blockDim.x) {
    const double d = ldexp(1.0 + (double)((i * 2654435761u) % 1000003u) / 1000003.0, (i % 61) - 30);
    const double ref = 1.0 / sqrt(d);
    double x = __builtin_amdgcn_rsq(d);
    e0 = fmax(e0, fabs(x - ref) / ref);
    const double hd = 0.5 * d;
    x = x * (1.5 - hd * x * x);
    e1 = fmax(e1, fabs(x - ref) / ref);
    x = x * (1.5 - hd * x * x);
    e2 = fmax(e2, fabs(x - ref) / ref);
  }
  atomicMax(reinterpret_cast<unsigned long long *>(err + 0), (unsigned long long)__double_as_longlong(e0));
  atomicMax(reinterpret_cast<unsigned long long *>(err + 1), (unsigned long long)__double_as_longlong(e1));
  atomicMax(reinterpret_cast<unsigned long long *>(err + 2), (unsigned long long)__double_as_longlong(e2));
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
  CK(hipMalloc(&t, 24 * 8));
  {
    double *err, he[3];
    CK(hipMalloc(&err, 24));
    CK(hipMemset(err, 0, 24));
    k_rsq_acc<<<256, 256>>>(err, 1 << 24);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(he, err, 24, hipMemcpyDeviceToHost));
    printf("v_rsq_f64 max rel error: raw %.3e, 1 Newton step %.3e, 2 steps %.3e (2^-52 = 2.2e-16)\n", he[0], he[1], he[2]);
  }
  for (int rep = 0; rep < 2; rep++) {
    k_icache<<<1, 64>>>(out, t);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, t, 24, hipMemcpyDeviceToHost));
    printf("1024 straight-line v_fma_f64 (4 chains): pass 1 %lld, pass 2 %lld, pass 3 %lld cycles\n", h[0], h[1], h[2]);
    k_fma_dep<<<1, 64>>>(out, t, 256);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, t, 8, hipMemcpyDeviceToHost));
    printf("dependent f64 FMA: %.1f cycles\n", h[0] / 256.0);
    k_rsq_dep<<<1, 64>>>(out, t, 256);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, t, 8, hipMemcpyDeviceToHost));
    printf("dependent v_rsq_f64 + add: %.1f cycles\n", h[0] / 256.0);
    k_diag<<<1, 64>>>(out, t);
    CK(hipDeviceSynchronize());
    long long hh[24];
    CK(hipMemcpy(hh, t, 24 * 8, hipMemcpyDeviceToHost));
    printf("16x16 diagonal factor: calls 1..4: %lld %lld %lld %lld cycles\n", hh[0], hh[1], hh[2], hh[3]);
    printf("  stamped call, per step: D in / chol+inv done / W_D in / panel MFMA done / step end (cycles from entry)\n");
    for (int b = 0; b < 4; b++)
      printf("    step %d: %6lld %6lld %6lld %6lld %6lld\n", b, hh[4 + 5 * b], hh[5 + 5 * b], hh[6 + 5 * b], hh[7 + 5 * b], hh[8 + 5 * b]);
  }
  return 0;
}
