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

typedef float gelu_f2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

// exact-erf GELU (HF "gelu") of NP2 pairs x, in place:  GELU(x) = max(x, 0) - s·E',
// s = min(|x|, 6), E' = erfc(s/√2) / 2 = exp2(P6(s)), P6 the degree-6 polynomial of
// tools/fit_gelu.py (a weighted minimax fit of log2 erfc(s/√2) - 1 on the GELU error itself,
// s·E'·ln2·ΔP).  For |x| <= 6 this is the identity x·Φ(x) = max(x, 0) - |x|·Φ(-|x|); past it the
// s·E' term is at most 6·E'(6) = 6.6e-9, so large |x| give x (x > 0) or -6.6e-9 (x < 0).  Over
// every f32 x within 2.9e-7 absolute of the float64 GELU and 8.2e-8 beyond the f32 rounding of
// the result (the Abramowitz & Stegun 7.1.26 form it replaced — rcp + exp + five FMAs — 2.1e-7
// beyond rounding; torch's f32 GELU 1.2e-6).  Per pair: two v_min (|x| as a source modifier), six
// packed FMAs, two v_exp_f32, two v_maximum and one packed FMA — no reciprocal; written step-major
// over the pairs so that independent chains interleave (no VOP3P dependency stalls).
template <int NP2>
__device__ __forceinline__ void gelu_exp2_pairs(gelu_f2 (&x)[NP2]) {
  gelu_f2 s[NP2], p[NP2];
#pragma unroll
  for (int k = 0; k < NP2; ++k)
    s[k] = __builtin_elementwise_min(__builtin_elementwise_abs(x[k]), gelu_f2(6.0f));
#pragma unroll
  for (int k = 0; k < NP2; ++k)
    p[k] = __builtin_elementwise_fma(gelu_f2(3.309332169e-05f), s[k], gelu_f2(-7.692241343e-04f));
#pragma unroll
  for (int k = 0; k < NP2; ++k) p[k] = __builtin_elementwise_fma(p[k], s[k], gelu_f2(8.080731146e-03f));
#pragma unroll
  for (int k = 0; k < NP2; ++k) p[k] = __builtin_elementwise_fma(p[k], s[k], gelu_f2(-5.341212824e-02f));
#pragma unroll
  for (int k = 0; k < NP2; ++k) p[k] = __builtin_elementwise_fma(p[k], s[k], gelu_f2(-4.587709606e-01f));
#pragma unroll
  for (int k = 0; k < NP2; ++k) p[k] = __builtin_elementwise_fma(p[k], s[k], gelu_f2(-1.151201725e+00f));
#pragma unroll
  for (int k = 0; k < NP2; ++k) p[k] = __builtin_elementwise_fma(p[k], s[k], gelu_f2(-9.999930859e-01f));
#pragma unroll
  for (int k = 0; k < NP2; ++k) {
    const gelu_f2 e = {__builtin_amdgcn_exp2f(p[k].x), __builtin_amdgcn_exp2f(p[k].y)};
    // IEEE maximum (v_maximum3_f32), not maxnum: a NaN pre-activation stays NaN (maxnum would
    // return 0 and the result a finite -6.6e-9 — an upstream overflow must not give finite scores)
    x[k] = __builtin_elementwise_fma(-s[k], e, __builtin_elementwise_maximum(x[k], gelu_f2(0.0f)));
  }
}

// split of an f32 pair into bf16 hi / lo planes (hi = rne(y), lo = rne(y - hi)), each plane's pair
// as one 32-bit word (element 0 in the low half): two v_cvt_pk_bf16_f32, the hi pair widened back
// to f32 by a shift and a mask, one packed subtract
__device__ __forceinline__ void split_pair(gelu_f2 y, uint32_t& hw, uint32_t& lw) {
  hw = __builtin_bit_cast(uint32_t, __builtin_convertvector(y, bf16x2_t));
  const gelu_f2 hf = {__builtin_bit_cast(float, hw << 16), __builtin_bit_cast(float, hw & 0xffff0000u)};
  lw = __builtin_bit_cast(uint32_t, __builtin_convertvector(y - hf, bf16x2_t));
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
