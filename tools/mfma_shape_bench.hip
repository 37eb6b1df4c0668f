// mfma_shape_bench.hip — which bf16 MFMA shape sustains more FLOP/s on this chip under load?
// (cdna_hip_programming.md §5.4 rule 28: the clock the chip holds can depend on the shape.)
//
// Both kernels compute the same 64 x 64 output tile per wave with k = 32 per iteration over
// operands re-read from LDS by ds_read_b128 (random bf16, 8 reads per iteration in both), one
// wave per SIMD, 4 workgroups per CU slot's worth of grid:
//   shape 0: v_mfma_f32_32x32x16_bf16, 2 x 2 blocks x 2 k-steps = 8 MFMAs per iteration
//   shape 1: v_mfma_f32_16x16x32_bf16, 4 x 4 blocks x 1 k-step  = 16 MFMAs per iteration
// Prints one JSON line per shape: TFLOP/s (median of rounds) and the in-kernel clock.
//   hipcc --offload-arch=gfx950 -O3 -o mfma_shape_bench tools/mfma_shape_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int LDS_BYTES = 64 * 1024;

template <int SHAPE>
__global__ __launch_bounds__(256, 1) void mfma_loop(const bf16x8* __restrict__ src, int iters,
                                                    float* __restrict__ out,
                                                    unsigned long long* __restrict__ clk) {
  __shared__ bf16x8 lds[LDS_BYTES / 16];
  for (int i = threadIdx.x; i < LDS_BYTES / 16; i += blockDim.x) lds[i] = src[i];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bf16x8* base = lds + wave * 512;  // 8 KiB per wave
  unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  float sink = 0.f;
  if constexpr (SHAPE == 0) {
    floatx16 acc[2][2] = {};
    for (int it = 0; it < iters; ++it) {
      const int o = (it & 7) * 64;
      bf16x8 a[2][2], b[2][2];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          a[m][k] = base[(o + lane + 128 * (2 * m + k)) & 511];
          b[m][k] = base[(o + lane + 64 + 128 * (2 * m + k)) & 511];
        }
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n)
            acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[m][k], b[n][k], acc[m][n], 0, 0, 0);
    }
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int r = 0; r < 16; ++r) sink += acc[m][n][r];
  } else {
    floatx4 acc[4][4] = {};
    for (int it = 0; it < iters; ++it) {
      const int o = (it & 7) * 64;
      bf16x8 a[4], b[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        a[m] = base[(o + lane + 128 * m) & 511];
        b[m] = base[(o + lane + 64 + 128 * m) & 511];
      }
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m], b[n], acc[m][n], 0, 0, 0);
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) sink += acc[m][n][r];
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = sink;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 4, iters = 20000;
  std::vector<unsigned short> h(LDS_BYTES / 2);
  unsigned s = 12345;
  for (auto& x : h) {  // random finite bf16 in about [-2, 2]
    s = s * 1664525u + 1013904223u;
    x = (unsigned short)(0x3c00 + ((s >> 16) & 0x7ff)) | (unsigned short)(((s >> 8) & 1) << 15);
  }
  bf16x8* src;
  float* out;
  unsigned long long* clk;
  CK(hipMalloc(&src, LDS_BYTES));
  CK(hipMalloc(&out, (size_t)grid * 256 * 4));
  CK(hipMalloc(&clk, (size_t)grid * 16));
  CK(hipMemcpy(src, h.data(), LDS_BYTES, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double flop = (double)grid * 4 * iters * 64.0 * 64 * 32 * 2;
  std::vector<double> t[2];
  std::vector<double> ghz[2];
  for (int round = 0; round < 7; ++round) {
    for (int sh = 0; sh < 2; ++sh) {
      CK(hipEventRecord(e0, 0));
      for (int rep = 0; rep < 3; ++rep) {
        if (sh == 0) hipLaunchKernelGGL(mfma_loop<0>, dim3(grid), dim3(256), 0, 0, src, iters, out, clk);
        else hipLaunchKernelGGL(mfma_loop<1>, dim3(grid), dim3(256), 0, 0, src, iters, out, clk);
      }
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[sh].push_back(ms / 3);
      std::vector<unsigned long long> c(2 * grid);
      CK(hipMemcpy(c.data(), clk, c.size() * 8, hipMemcpyDeviceToHost));
      std::vector<double> g;
      for (int b = 0; b < grid; ++b) g.push_back((double)c[2 * b] / (double)c[2 * b + 1] * 0.1);
      std::sort(g.begin(), g.end());
      ghz[sh].push_back(g[g.size() / 2]);
    }
  }
  for (int sh = 0; sh < 2; ++sh) {
    std::sort(t[sh].begin(), t[sh].end());
    std::sort(ghz[sh].begin(), ghz[sh].end());
    const double ms = t[sh][t[sh].size() / 2];
    printf("{\"shape\": \"%s\", \"ms\": %.3f, \"tflops\": %.1f, \"clock_ghz\": %.3f}\n",
           sh == 0 ? "32x32x16" : "16x16x32", ms, flop / ms / 1e9, ghz[sh][ghz[sh].size() / 2]);
  }
  return 0;
}
