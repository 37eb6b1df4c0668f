// common.h — shared device helpers for the gfx950 kernels of the victim-query engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <map>
#include <mutex>
#include <utility>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef short shortx8 __attribute__((ext_vector_type(8)));
typedef unsigned short ushortx4 __attribute__((ext_vector_type(4)));

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device): the attribute is
// per device, so a process driving two GPUs sets it on each; thread-safe.
inline hipError_t ensure_dynamic_lds(const void* fn, size_t lds) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, size_t> done;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> g(mu);
  size_t& have = done[{fn, dev}];
  if (have >= lds) return hipSuccess;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess) have = lds;
  return e;
}

#define AE_HIDDEN 768
#define AE_HEAD_DIM 64

// 32x32 MFMA C/D layout (gfx950, dtype independent): register r of lane l holds
// row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31.
__device__ __forceinline__ int mfma32_row(int r, int half) { return (r & 3) + 8 * (r >> 2) + 4 * half; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

__device__ __forceinline__ float gelu_erf(float x) {
  // exact-erf GELU (HF "gelu" = nn.functional.gelu, approximate='none')
  return 0.5f * x * (1.0f + erff(x * 0.70710678118654752440f));
}

// exact-erf GELU through a rational erfc (Abramowitz & Stegun 7.1.26, |erf error| <= 1.5e-7):
// erfc(z) = t·P5(t)·exp(-z²) = E, t = 1/(1 + 0.3275911 z), z = |x|/√2.  With u = x/2,
// GELU(x) = u + |u| - |u|·E (x >= 0: x - u·E; x < 0: u·E), so no compare / select: one FMA ends
// it.  Over [-12, 12] it is within 3.3e-7 absolute of the float64 GELU (torch's f32 GELU: 1.2e-6
// absolute), 5 Horner FMAs + rcp + exp2 — the split-precision FFN1 epilogue is VALU-bound on
// this (tools/gemm_bench.py diag 4 vs 0).
__device__ __forceinline__ float gelu_erfc_fast(float x) {
  const float u = 0.5f * x, au = fabsf(u);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.46328380415598320f, au, 1.0f));
  float p = 1.061405429f;
  p = fmaf(p, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(u * (-2.88539008177792680f * u));  // exp(-x²/2)
  return fmaf(-au, (p * t) * e, u + au);
}

// gelu_erfc_fast on a pair, written on 2-wide vectors so every non-transcendental step is one
// packed-f32 instruction (v_pk_fma / v_pk_mul / v_pk_add: the same IEEE operation per element,
// so the results equal two gelu_erfc_fast calls bit for bit); the rcp and exp2 stay scalar.
typedef float gelu_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ gelu_f2 gelu_erfc_fast2(gelu_f2 x) {
  const gelu_f2 u = x * 0.5f;
  const gelu_f2 au = {fabsf(u.x), fabsf(u.y)};
  const gelu_f2 d = __builtin_elementwise_fma(gelu_f2(0.46328380415598320f), au, gelu_f2(1.0f));
  const gelu_f2 t = {__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
  gelu_f2 p = gelu_f2(1.061405429f);
  p = __builtin_elementwise_fma(p, t, gelu_f2(-1.453152027f));
  p = __builtin_elementwise_fma(p, t, gelu_f2(1.421413741f));
  p = __builtin_elementwise_fma(p, t, gelu_f2(-0.284496736f));
  p = __builtin_elementwise_fma(p, t, gelu_f2(0.254829592f));
  const gelu_f2 a = u * (-2.88539008177792680f * u);
  const gelu_f2 e = {__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
  return __builtin_elementwise_fma(-au, (p * t) * e, u + au);
}

// bf16 round-to-nearest-even of an f32 (NaN-preserving cast lowered to v_cvt_pk_bf16_f32).
__device__ __forceinline__ unsigned short f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5, T1):
// blocks b and b+8 share an XCD, so give each XCD a contiguous chunk of the tile order.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7, idx = orig >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}
