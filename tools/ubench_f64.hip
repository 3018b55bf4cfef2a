// Micro-benchmarks of the latencies the dense-tail chain is made of (gfx950):
// dependent / independent v_mfma_f64_16x16x4f64, an LDS write->read round
// trip, a write-through 16-B store followed by a load of another line (the
// vmcnt wait covers the store), and an L2-hit load. One wave each; cycles
// from s_memtime (clock64) and ns from s_memrealtime (100 MHz).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_f64.hip -o variants/ubench_f64
#include <hip/hip_runtime.h>

#include <cstdio>

typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_mfma_dep(double *out, long long *t, int n) {
  const int lane = threadIdx.x;
  f64x4 acc = {1.0 * lane, 0.5, 0.25, 0.125};
  double a = 1.0 + 1e-9 * lane, b = 1.0 - 1e-9 * lane;
  __syncthreads();
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < n; i++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  const long long c1 = clock64(), w1 = wall_clock64();
  out[lane] = acc[0] + acc[1] + acc[2] + acc[3];
  if (lane == 0) t[0] = c1 - c0, t[1] = w1 - w0;
}

__global__ void k_mfma_ind(double *out, long long *t, int n) {
  const int lane = threadIdx.x;
  f64x4 a0 = {1.0 * lane, 0.5, 0.25, 0.125}, a1 = a0, a2 = a0, a3 = a0;
  double a = 1.0 + 1e-9 * lane, b = 1.0 - 1e-9 * lane;
  __syncthreads();
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < n; i++) {
    a0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, a0, 0, 0, 0);
    a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, a1, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, a2, 0, 0, 0);
    a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, a3, 0, 0, 0);
  }
  const long long c1 = clock64(), w1 = wall_clock64();
  out[lane] = a0[0] + a1[1] + a2[2] + a3[3];
  if (lane == 0) t[0] = c1 - c0, t[1] = w1 - w0;
}

// MFMA result feeding the next MFMA's A operand (the panel -> update chain)
__global__ void k_mfma_dep_ab(double *out, long long *t, int n) {
  const int lane = threadIdx.x;
  f64x4 acc = {1.0 * lane, 0.5, 0.25, 0.125};
  __syncthreads();
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < n; i++) {
    const f64x4 z = {0.0, 0.0, 0.0, 0.0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(acc[0] * 1e-3, acc[1], z, 0, 0, 0);
  }
  const long long c1 = clock64(), w1 = wall_clock64();
  out[lane] = acc[0] + acc[1] + acc[2] + acc[3];
  if (lane == 0) t[0] = c1 - c0, t[1] = w1 - w0;
}

__global__ void k_lds_rt(double *out, long long *t, int n) {
  __shared__ double s[64];
  const int lane = threadIdx.x;
  double v = lane;
  __syncthreads();
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < n; i++) {
    s[lane] = v;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    v = s[(lane + 1) & 63] + 1.0;
  }
  const long long c1 = clock64(), w1 = wall_clock64();
  out[lane] = v;
  if (lane == 0) t[0] = c1 - c0, t[1] = w1 - w0;
}

// store (write-through, sc0 sc1) then a dependent load of another buffer
__global__ void k_store_load(double *buf, double *out, long long *t, int n) {
  const int lane = threadIdx.x;
  double v = lane;
  const __amdgpu_buffer_rsrc_t R = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 1 << 20, 0x00020000);
  __syncthreads();
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < n; i++) {
    __builtin_amdgcn_raw_buffer_store_b32((unsigned)__double_as_longlong(v), R, (4096 + (i & 63) * 64 + lane) * 4, 0, 3);
    const unsigned x = __builtin_amdgcn_raw_buffer_load_b32(R, lane * 4, 0, 3);
    v += (double)x * 1e-30;
  }
  const long long c1 = clock64(), w1 = wall_clock64();
  out[lane] = v;
  if (lane == 0) t[0] = c1 - c0, t[1] = w1 - w0;
}

// dependent loads of one line (sc1: past L1, an L2 hit)
__global__ void k_load_l2(double *buf, double *out, long long *t, int n) {
  const int lane = threadIdx.x;
  const __amdgpu_buffer_rsrc_t R = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 1 << 20, 0x00020000);
  int off = lane * 4;
  double v = 0.0;
  __syncthreads();
  const long long c0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < n; i++) {
    const unsigned x = __builtin_amdgcn_raw_buffer_load_b32(R, off, 0, 2);
    v += (double)x;
    off = (lane * 4) + (int)(x & 0u);  // dependent address
  }
  const long long c1 = clock64(), w1 = wall_clock64();
  out[lane] = v;
  if (lane == 0) t[0] = c1 - c0, t[1] = w1 - w0;
}

// store throughput of one wave: n x 16-B stores per lane (1 KB per wave
// instruction) to distinct lines, then a full drain; AUX = cache policy
// (0 plain, 1 sc0, 2 sc1, 3 sc0 sc1); mode 1 times the issue only (no drain)
template <int AUX>
__global__ void k_store_bw(double *buf, long long *t, int n, int drain) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t R = __builtin_amdgcn_make_buffer_rsrc(buf, 0, 1 << 24, 0x00020000);
  __syncthreads();
  const long long c0 = clock64();
  for (int i = 0; i < n; i++) {
    const u32x4 w = {(unsigned)i, (unsigned)lane, (unsigned)wv, 0u};
    __builtin_amdgcn_raw_buffer_store_b128(w, R, ((wv * n + i) * 64 + lane) * 16, 0, AUX);
  }
  if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const long long c1 = clock64();
  if (threadIdx.x == 0) t[0] = c1 - c0;
}

#define CK(x)                                                  \
  do {                                                         \
    hipError_t e = (x);                                        \
    if (e != hipSuccess) {                                     \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                \
    }                                                          \
  } while (0)

int main() {
  double *buf, *out;
  long long *t;
  CK(hipMalloc(&buf, 1 << 20));
  CK(hipMemset(buf, 0, 1 << 20));
  CK(hipMalloc(&out, 64 * 8));
  CK(hipMalloc(&t, 16));
  const int n = 256;
  long long h[2];
  auto rep = [&](const char *name, int per) {
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, t, 16, hipMemcpyDeviceToHost));
    printf("%-34s %8.1f cycles  %7.1f ns  per op (clock %.2f GHz)\n", name, (double)h[0] / (n * per),
           h[1] * 10.0 / (n * per), (double)h[0] / (h[1] * 10.0));
    return 0;
  };
  {
    double *sb;
    CK(hipMalloc(&sb, 1 << 24));
    for (int waves = 1; waves <= 4; waves *= 4)
      for (int drain = 0; drain < 2; drain++) {
        k_store_bw<0><<<1, 64 * waves>>>(sb, t, 64, drain);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, t, 8, hipMemcpyDeviceToHost));
        const long long plain = h[0];
        k_store_bw<2><<<1, 64 * waves>>>(sb, t, 64, drain);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, t, 8, hipMemcpyDeviceToHost));
        const long long wt = h[0];
        k_store_bw<3><<<1, 64 * waves>>>(sb, t, 64, drain);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, t, 8, hipMemcpyDeviceToHost));
        printf("64 x 16-B stores per lane, %d wave(s) on one CU, %s: plain %.1f, sc1 %.1f, sc0 sc1 %.1f cycles per wave instruction\n",
               waves, drain ? "drained" : "issue only", plain / 64.0, wt / 64.0, h[0] / 64.0);
      }
  }
  for (int pass = 0; pass < 2; pass++) {
    k_mfma_dep<<<1, 64>>>(out, t, n);
    rep("mfma f64 16x16x4, dependent (C)", 1);
    k_mfma_ind<<<1, 64>>>(out, t, n);
    rep("mfma f64 16x16x4, 4 independent", 4);
    k_mfma_dep_ab<<<1, 64>>>(out, t, n);
    rep("mfma f64 16x16x4, result -> A,B", 1);
    k_lds_rt<<<1, 64>>>(out, t, n);
    rep("LDS write -> read round trip", 1);
    k_store_load<<<1, 64>>>(buf, out, t, n);
    rep("store (sc0 sc1) + load, vmcnt", 1);
    k_load_l2<<<1, 64>>>(buf, out, t, n);
    rep("dependent load (sc1, L2 hit)", 1);
  }
  return 0;
}
