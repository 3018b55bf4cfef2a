// Micro-benchmark (gfx950): the dense tail's 16x16 diagonal factor on DPP row
// broadcasts (m3s_gn.hip tail_diag_full, restated) on one wave, hot calls,
// shader clock; plus the latency of its building blocks (dependent f64 FMA,
// v_mov_b64_dpp row_newbcast -> FMA, rsqrt_nr) with no loop overhead.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_diag16.hip -o variants/ubench_diag16
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));

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
template <int I>
__device__ __forceinline__ double row_bcast_c(double v) {
  return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + I, 0xf, 0xf, false);
}
__device__ __forceinline__ double row_bcast(double v, int i) {
  switch (i) {
    case 0: return row_bcast_c<0>(v);
    case 1: return row_bcast_c<1>(v);
    case 2: return row_bcast_c<2>(v);
    case 3: return row_bcast_c<3>(v);
    case 4: return row_bcast_c<4>(v);
    case 5: return row_bcast_c<5>(v);
    case 6: return row_bcast_c<6>(v);
    case 7: return row_bcast_c<7>(v);
    case 8: return row_bcast_c<8>(v);
    case 9: return row_bcast_c<9>(v);
    case 10: return row_bcast_c<10>(v);
    case 11: return row_bcast_c<11>(v);
    case 12: return row_bcast_c<12>(v);
    case 13: return row_bcast_c<13>(v);
    case 14: return row_bcast_c<14>(v);
    default: return row_bcast_c<15>(v);
  }
}
__device__ __noinline__ bool diag_dpp(f64x4 a4, double (*Wk)[17], int lane, long long *st) {
  __shared__ double xt[16][17];
  const int lr = lane & 15, lk = lane >> 4;
  const long long c0 = __builtin_readcyclecounter();
#pragma unroll
  for (int r = 0; r < 4; r++) xt[lr][lk + 4 * r] = a4[r];
  wave_lds_fence();
  double a[16], R[16];
#pragma unroll
  for (int i = 0; i < 16; i++) {
    a[i] = xt[lr][i];
    R[i] = i == lr ? 1.0 : 0.0;
  }
  const long long c1 = __builtin_readcyclecounter();
  bool bad = false;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const double d0 = row_bcast(a[k], k);
    bad |= !(d0 > 0.0);
    const double r = rsqrt_nr(d0 > 0.0 ? d0 : 1.0);
    const double l = a[k] * r;
    const double w = R[k] * r;
    if (lk == 0) Wk[k][lr] = w;
#pragma unroll
    for (int i = k + 1; i < 16; i++) {
      const double li = row_bcast(l, i);
      a[i] = __builtin_fma(-li, l, a[i]);
      R[i] = __builtin_fma(-li, w, R[i]);
    }
  }
  wave_lds_fence();
  const long long c2 = __builtin_readcyclecounter();
  if (lane == 0) st[0] = c1 - c0, st[1] = c2 - c1;
  return bad;
}

__global__ void k_diag(const double *A, double *W, long long *t) {
  __shared__ double Wk[16][17];
  const int lane = threadIdx.x, lr = lane & 15, lk = lane >> 4;
  f64x4 a;
  for (int r = 0; r < 4; r++) a[r] = A[16 * (lk + 4 * r) + lr];
  bool bad = false;
  for (int call = 0; call < 4; call++) {
    const long long c0 = __builtin_readcyclecounter();
    bad |= diag_dpp(a, Wk, lane, t + 8 + 2 * call);
    const long long c1 = __builtin_readcyclecounter();
    if (lane == 0) t[call] = c1 - c0;
  }
  for (int e = lane; e < 256; e += 64) W[e] = Wk[e / 16][e % 16];
  if (lane == 0) t[7] = bad;
}

#define R8(x) x x x x x x x x
__global__ void k_lat(double *out, long long *t) {
  double a = 1.0 + threadIdx.x * 1e-3, b = 1.0000001;
  long long c0 = __builtin_readcyclecounter();
  asm volatile(R8(R8("v_fma_f64 %0, %0, %1, %1\n")) : "+v"(a) : "v"(b));
  long long c1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) t[0] = c1 - c0;
  c0 = __builtin_readcyclecounter();
  for (int k = 0; k < 64; k++) a = __builtin_fma(row_bcast_c<3>(a), b, 1e-9);
  c1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) t[1] = c1 - c0;
  c0 = __builtin_readcyclecounter();
#pragma unroll
  for (int k = 0; k < 64; k++) a = rsqrt_nr(a) + 0.5;
  c1 = __builtin_readcyclecounter();
  if (threadIdx.x == 0) t[2] = c1 - c0;
  out[threadIdx.x] = a;
}

int main() {
  double hA[256], *dA, *dW, *dout;
  long long *dt, ht[16];
  // SPD: M M^T + 16 I
  double M[256];
  for (int i = 0; i < 256; i++) M[i] = ((i * 7919) % 97) / 97.0 - 0.5;
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 16; j++) {
      double s = i == j ? 16.0 : 0.0;
      for (int k = 0; k < 16; k++) s += M[16 * i + k] * M[16 * j + k];
      hA[16 * i + j] = s;
    }
  hipMalloc(&dA, 2048), hipMalloc(&dW, 2048), hipMalloc(&dt, 128), hipMalloc(&dout, 512);
  hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice);
  k_diag<<<1, 64>>>(dA, dW, dt);
  hipMemcpy(ht, dt, 128, hipMemcpyDeviceToHost);
  double hW[256];
  hipMemcpy(hW, dW, 2048, hipMemcpyDeviceToHost);
  // check W A W^T = I
  double err = 0;
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 16; j++) {
      double s = 0;
      for (int p = 0; p < 16; p++)
        for (int q = 0; q < 16; q++) s += hW[16 * i + p] * hA[16 * p + q] * hW[16 * j + q];
      err = fmax(err, fabs(s - (i == j)));
    }
  printf("DPP 16x16 diagonal factor: calls 1..4: %lld %lld %lld %lld cycles (bad %lld); |W A W^T - I| = %.2e\n",
         ht[0], ht[1], ht[2], ht[3], ht[7], err);
  printf("  inside, per call: transpose in %lld / factor %lld | %lld / %lld | %lld / %lld | %lld / %lld\n", ht[8],
         ht[9], ht[10], ht[11], ht[12], ht[13], ht[14], ht[15]);
  k_lat<<<1, 64>>>(dout, dt);
  hipMemcpy(ht, dt, 64, hipMemcpyDeviceToHost);
  printf("dependent v_fma_f64 (64, straight-line): %.1f cycles each; DPP broadcast -> FMA (64): %.1f; rsqrt_nr + add "
         "(64): %.1f\n",
         ht[0] / 64.0, ht[1] / 64.0, ht[2] / 64.0);
  return 0;
}
