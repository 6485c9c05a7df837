// Shared device-side helpers for the FER-ViT gfx950 kernels.
//
// Storage conventions:
//   * activations are token-major [M = B*N rows][D cols], row-major, bf16 (fast path)
//     or fp32 (parity path); weights follow nn.Linear's [out][in] layout.
//   * bf16 is the compiler's __bf16 (lowered to v_cvt_pk_bf16_f32 on gfx950).
//   * dropout keep-masks are never stored: they are regenerated from
//     (seed, linear element index) by `drop_keep`, in forward and backward.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <map>
#include <mutex>

#define FER_DEV __device__ __forceinline__

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) short short4_t;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
// Global-typed 16-byte load (kernel-argument structs hold generic pointers: flat loads otherwise)
FER_DEV f32x4 ldg_f32x4(const float* p) { return *(const __attribute__((address_space(1))) f32x4*)(const void*)p; }
// A volatile int in LDS through an LDS-typed pointer: a plain `volatile int*` into a __shared__ array is a
// generic pointer, compiled to flat_load / flat_store, which count in vmcnt AND lgkmcnt -- the compiler
// then waits vmcnt(0) for the word, i.e. for every outstanding global store of the wave as well.
typedef volatile __attribute__((address_space(3))) int lds_vint;
typedef volatile __attribute__((address_space(3))) unsigned lds_vuint;
#define FER_LDS_INT(p) ((lds_vint*)(__attribute__((address_space(3))) void*)(void*)(p))
#define FER_LDS_UINT(p) ((lds_vuint*)(__attribute__((address_space(3))) void*)(void*)(p))
// Two 4 x bf16 halves (e.g. two ds_read_b64_tr_b16 results) as one 8 x bf16 MFMA operand by
// register concatenation: element-wise construction made hipcc repack every 16-bit element
// (shift / and / or per element: ~8 VALU per operand in the attention and MN GEMM loops).
FER_DEV bf16x8 cat8(short4_t a, short4_t b) {
  const u32x2 x = __builtin_bit_cast(u32x2, a), y = __builtin_bit_cast(u32x2, b);
  return __builtin_bit_cast(bf16x8, u32x4{x[0], x[1], y[0], y[1]});
}

enum { FER_ACT_NONE = 0, FER_ACT_GELU = 1, FER_ACT_RELU = 2, FER_ACT_MUL = 3 /* aux_act only: v *= aux */ };
// act flag: `pre` receives the backward GATE act'(v) * keep * drop_scale instead of the
// pre-activation v (the input-gradient GEMM then only multiplies by it: aux_act = FER_ACT_MUL).
enum { FER_PRE_GATE = 16 };

FER_DEV float bf2f(bf16 x) { return (float)x; }
FER_DEV bf16 f2bf(float x) { return (bf16)x; }

template <typename T> FER_DEV float to_f(T x);
template <> FER_DEV float to_f<float>(float x) { return x; }
template <> FER_DEV float to_f<bf16>(bf16 x) { return (float)x; }
template <typename T> FER_DEV T from_f(float x);
template <> FER_DEV float from_f<float>(float x) { return x; }
template <> FER_DEV bf16 from_f<bf16>(float x) { return (bf16)x; }

// 4 consecutive elements <-> float4 (8 B for bf16, 16 B for fp32).
template <typename T> FER_DEV f32x4 load4(const T* p);
template <> FER_DEV f32x4 load4<float>(const float* p) { return *(const f32x4*)p; }
template <> FER_DEV f32x4 load4<bf16>(const bf16* p) {
  bf16x4 v = *(const bf16x4*)p;
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
}
// Raw (unconverted) 4-element vectors, for loads whose conversion is deferred to the use.
template <typename T> struct Raw4;
template <> struct Raw4<float> { typedef f32x4 type; };
template <> struct Raw4<bf16> { typedef bf16x4 type; };
FER_DEV f32x4 raw4_to_f(f32x4 v) { return v; }
FER_DEV f32x4 raw4_to_f(bf16x4 v) { return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]}; }
template <typename T> FER_DEV void store4(T* p, f32x4 v);
template <> FER_DEV void store4<float>(float* p, f32x4 v) { *(f32x4*)p = v; }
template <> FER_DEV void store4<bf16>(bf16* p, f32x4 v) {
  *(bf16x4*)p = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
}

// ---------------------------------------------------------------- activations
// erf via Abramowitz-Stegun 7.1.26 (|err| <= 1.5e-7), sharing exp(-x^2/2) with the
// GELU derivative's pdf term; ~15 VALU ops instead of the libm erff path.
FER_DEV float fast_erf_from_exp(float z, float e /* = exp(-z*z) */) {
  const float az = fabsf(z);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, az, 1.0f));
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  const float r = 1.0f - y * t * e;
  return copysignf(r, z);
}
FER_DEV float gelu_erf(float x) {
  const float e = __expf(-0.5f * x * x);
  return 0.5f * x * (1.0f + fast_erf_from_exp(x * 0.70710678118654752f, e));
}
// GELU for the bf16 GEMM epilogue (VALU-bound there): erf by Abramowitz-Stegun 7.1.28,
// 1 - (1 + a1 z + ... + a6 z^6)^-16 — one reciprocal, no exponential; |GELU error| <= 9e-7 in
// fp32, two orders below the bf16 rounding of the stored activation.
FER_DEV float gelu_erf_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  float p = fmaf(4.30638e-5f, z, 2.765672e-4f);
  p = fmaf(p, z, 1.520143e-4f);
  p = fmaf(p, z, 9.2705272e-3f);
  p = fmaf(p, z, 4.22820123e-2f);
  p = fmaf(p, z, 7.05230784e-2f);
  p = fmaf(p, z, 1.0f);
  p *= p;
  p *= p;
  p *= p;
  p *= p;
  const float e = 1.0f - __builtin_amdgcn_rcpf(p);  // erf(|x| / sqrt 2); rcp(inf) = 0
  return 0.5f * x * (1.0f + copysignf(e, x));
}
// The same on two values with packed fp32 math (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth
// per instruction); identical arithmetic per element, so bit-identical to gelu_erf_fast.
typedef __attribute__((ext_vector_type(2))) float f32x2;
// A packed-math constant materialised where it is used: without the barrier the compiler hoists
// every such constant into an SGPR pair for the whole kernel, and the GEMM's main loop then
// spills SGPRs.
FER_DEV f32x2 kpk(float c) {
  asm volatile("" : "+s"(c));
  return f32x2(c);
}
FER_DEV f32x2 gelu_erf_fast2(f32x2 x) {
  const f32x2 z = __builtin_elementwise_abs(x) * 0.70710678118654752f;
  f32x2 p = __builtin_elementwise_fma(kpk(4.30638e-5f), z, kpk(2.765672e-4f));
  p = __builtin_elementwise_fma(p, z, kpk(1.520143e-4f));
  p = __builtin_elementwise_fma(p, z, kpk(9.2705272e-3f));
  p = __builtin_elementwise_fma(p, z, kpk(4.22820123e-2f));
  p = __builtin_elementwise_fma(p, z, kpk(7.05230784e-2f));
  p = __builtin_elementwise_fma(p, z, f32x2(1.0f));
  p *= p;
  p *= p;
  p *= p;
  p *= p;
  const f32x2 e = 1.0f - f32x2{__builtin_amdgcn_rcpf(p[0]), __builtin_amdgcn_rcpf(p[1])};
  return 0.5f * x * (1.0f + __builtin_elementwise_copysign(e, x));
}
FER_DEV float gelu_erf_grad(float x) {
  const float e = __expf(-0.5f * x * x);
  const float cdf = 0.5f * (1.0f + fast_erf_from_exp(x * 0.70710678118654752f, e));
  return fmaf(x * 0.39894228040143268f, e, cdf);
}
FER_DEV f32x2 gelu_erf_grad2(f32x2 x) {  // packed gelu_erf_grad, same arithmetic per element
  const f32x2 h = -0.5f * x * x;
  const f32x2 e = f32x2{__expf(h[0]), __expf(h[1])};
  const f32x2 z = x * 0.70710678118654752f;
  const f32x2 d = __builtin_elementwise_fma(kpk(0.3275911f), __builtin_elementwise_abs(z), f32x2(1.0f));
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f32x2 y = __builtin_elementwise_fma(kpk(1.061405429f), t, kpk(-1.453152027f));
  y = __builtin_elementwise_fma(y, t, kpk(1.421413741f));
  y = __builtin_elementwise_fma(y, t, kpk(-0.284496736f));
  y = __builtin_elementwise_fma(y, t, kpk(0.254829592f));
  const f32x2 r = 1.0f - y * t * e;
  const f32x2 cdf = 0.5f * (1.0f + __builtin_elementwise_copysign(r, z));
  return __builtin_elementwise_fma(x * 0.39894228040143268f, e, cdf);
}
// GELU and its derivative together, packed: erf by Abramowitz-Stegun 7.1.26 from e = exp(-x^2/2),
// which is also the derivative's pdf term -- one exponential and one reciprocal per element for
// both (|erf error| <= 1.5e-7).
FER_DEV f32x2 gelu_and_grad2(f32x2 x, f32x2& grad) {
  const f32x2 h = -0.5f * x * x;
  const f32x2 e = f32x2{__expf(h[0]), __expf(h[1])};
  const f32x2 z = x * 0.70710678118654752f;
  const f32x2 d = __builtin_elementwise_fma(kpk(0.3275911f), __builtin_elementwise_abs(z), f32x2(1.0f));
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f32x2 y = __builtin_elementwise_fma(kpk(1.061405429f), t, kpk(-1.453152027f));
  y = __builtin_elementwise_fma(y, t, kpk(1.421413741f));
  y = __builtin_elementwise_fma(y, t, kpk(-0.284496736f));
  y = __builtin_elementwise_fma(y, t, kpk(0.254829592f));
  const f32x2 r = 1.0f - y * t * e;
  const f32x2 cdf = 0.5f * (1.0f + __builtin_elementwise_copysign(r, z));
  grad = __builtin_elementwise_fma(x * 0.39894228040143268f, e, cdf);
  return x * cdf;
}
// Four independent pairs stage by stage (the same per-element operations as gelu_and_grad2): a
// dependent packed-f32 op right after its producer costs a hazard s_nop, and one pair's
// polynomial is a chain of them; interleaving the pairs fills those slots.
FER_DEV void gelu_and_grad8(f32x2 (&x)[4], f32x2 (&grad)[4]) {
  f32x2 e[4], z[4], t[4], y[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2 h = -0.5f * x[i] * x[i];
    e[i] = f32x2{__expf(h[0]), __expf(h[1])};
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) z[i] = x[i] * 0.70710678118654752f;
  const f32x2 ka = kpk(0.3275911f);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2 d = __builtin_elementwise_fma(ka, __builtin_elementwise_abs(z[i]), f32x2(1.0f));
    t[i] = f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  }
  const f32x2 k0 = kpk(1.061405429f), k1 = kpk(-1.453152027f);
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = __builtin_elementwise_fma(k0, t[i], k1);
  const f32x2 k2 = kpk(1.421413741f);
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = __builtin_elementwise_fma(y[i], t[i], k2);
  const f32x2 k3 = kpk(-0.284496736f);
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = __builtin_elementwise_fma(y[i], t[i], k3);
  const f32x2 k4 = kpk(0.254829592f);
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = __builtin_elementwise_fma(y[i], t[i], k4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const f32x2 r = 1.0f - y[i] * t[i] * e[i];
    const f32x2 cdf = 0.5f * (1.0f + __builtin_elementwise_copysign(r, z[i]));
    grad[i] = __builtin_elementwise_fma(x[i] * 0.39894228040143268f, e[i], cdf);
    x[i] = x[i] * cdf;
  }
}
// gelu_and_grad8 with an output scale s folded into its constants (the GEMM epilogue's dropout
// scale: x <- x * cdf * s, grad <- (x * pdf + cdf) * s) and exp(-x^2/2) taken as exp2 of
// x^2 * (-log2(e)/2): same formulas, roundings in a different order.
// hs = {s/2, s/2}, ps = {s/sqrt(2 pi), s/sqrt(2 pi)} (computed once by the caller, outside any
// divergent branch).
template <int P>
FER_DEV void gelu_and_grad_ps(f32x2 (&x)[P], f32x2 (&grad)[P], f32x2 hs, f32x2 ps) {
  f32x2 e[P], z[P], t[P], y[P];
  // z = |x| sqrt(log2(e) / 2): exp(-x^2/2) = exp2(-z^2), and |x| / sqrt(2) = z * 0.83255461 is folded
  // into the A-S constant (one multiply per pair less than scaling x twice); the sign comes from x
  const f32x2 kz = kpk(0.84932180028801907f);
#pragma unroll
  for (int i = 0; i < P; ++i) {
    // |z| by two scalar multiplies with the abs modifier (packed f32 has none: v_and per element)
    float z0 = __builtin_fabsf(x[i][0]) * kz[0], z1 = __builtin_fabsf(x[i][1]) * kz[1];
    asm volatile("" : "+v"(z0), "+v"(z1));
    z[i] = f32x2{z0, z1};
  }
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const f32x2 h = -(z[i] * z[i]);
    e[i] = f32x2{__builtin_amdgcn_exp2f(h[0]), __builtin_amdgcn_exp2f(h[1])};
  }
  const f32x2 ka = kpk(0.27273748087922250f);  // 0.3275911 / sqrt(2) / 0.84932180
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const f32x2 d = __builtin_elementwise_fma(ka, z[i], f32x2(1.0f));
    t[i] = f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  }
  const f32x2 k0 = kpk(1.061405429f), k1 = kpk(-1.453152027f);
#pragma unroll
  for (int i = 0; i < P; ++i) y[i] = __builtin_elementwise_fma(k0, t[i], k1);
  const f32x2 k2 = kpk(1.421413741f);
#pragma unroll
  for (int i = 0; i < P; ++i) y[i] = __builtin_elementwise_fma(y[i], t[i], k2);
  const f32x2 k3 = kpk(-0.284496736f);
#pragma unroll
  for (int i = 0; i < P; ++i) y[i] = __builtin_elementwise_fma(y[i], t[i], k3);
  const f32x2 k4 = kpk(0.254829592f);
#pragma unroll
  for (int i = 0; i < P; ++i) y[i] = __builtin_elementwise_fma(y[i], t[i], k4);
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const f32x2 r = 1.0f - y[i] * t[i] * e[i];
    const f32x2 cdf = __builtin_elementwise_fma(hs, __builtin_elementwise_copysign(r, x[i]), hs);  // s * Phi(x)
    grad[i] = __builtin_elementwise_fma(x[i] * ps, e[i], cdf);
    x[i] = x[i] * cdf;
  }
}
FER_DEV void gelu_and_grad8s(f32x2 (&x)[4], f32x2 (&grad)[4], f32x2 hs, f32x2 ps) { gelu_and_grad_ps<4>(x, grad, hs, ps); }
FER_DEV float act_fwd(int act, float x) {
  return act == FER_ACT_GELU ? gelu_erf(x) : (act == FER_ACT_RELU ? fmaxf(x, 0.f) : x);
}
FER_DEV float act_grad(int act, float x) {
  return act == FER_ACT_GELU ? gelu_erf_grad(x)
                             : (act == FER_ACT_RELU ? (x > 0.f ? 1.f : 0.f) : (act == FER_ACT_MUL ? x : 1.f));
}

// ---------------------------------------------------------------- dropout RNG
// Counter-based and stateless: keep(seed, idx) is a pure function of the element's
// linear index, so backward regenerates the forward mask. One 32-bit hash yields two 16-bit
// uniforms: element idx uses half (idx & 1) of hash(seed, idx >> 1). Drop iff u16 < thresh,
// thresh = round(p * 65536). The key enters by xor/add (a relabelling of the counter), the
// lowbias32 finaliser does the mixing: 2 integer multiplies per pair of elements.
// Element indices are 32-bit: every C-ABI entry point with dropout checks idx < 2^32
// (fer::check_drop_range); index arithmetic is done mod 2^32 by the callers.
FER_DEV uint32_t fer_mix(uint32_t x) {  // the lowbias32 finaliser
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
// fer_mix split for keep tests: returns x before the last step (h = x ^ (x >> 16) has x's high half, so
// h >> 16 == x >> 16 and h >= t << 16 iff x >= t << 16) and sets lo = h & 0xFFFF by one SDWA xor (the
// compiler's form is a shift and a bitop3)
FER_DEV uint32_t fer_mix_pre(uint32_t x, uint32_t& lo) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  asm("v_xor_b32_sdwa %0, %1, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:WORD_0" : "=v"(lo) : "v"(x));
  return x;
}
FER_DEV uint32_t fer_hash(uint64_t seed, uint32_t pair) {
  return fer_mix((pair ^ (uint32_t)seed) + (uint32_t)(seed >> 32));
}
// Device-side step counter for graph-replayed training steps (fer_set_step_counter): a
// captured launch keeps its host seed, so every dropout kernel mixes the current step into it.
// One pointer per code object (each .hip file is its own code object); null = no counter.
static __device__ const uint64_t* fer_step_ptr = nullptr;
FER_DEV uint64_t step_seed(uint64_t seed) {
  const uint64_t* p = fer_step_ptr;
  if (!p) return seed;
  // global-typed load (a generic pointer compiles to a flat load: vmcnt AND lgkmcnt waits)
  const uint64_t c = *(const __attribute__((address_space(1))) uint64_t*)(const void*)p;
  uint64_t z = seed ^ (c * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// host side, per code object
static inline hipError_t set_step_ptr_here(const uint64_t* p) {
  return hipMemcpyToSymbol(HIP_SYMBOL(fer_step_ptr), &p, sizeof(p));
}
FER_DEV bool drop_keep(uint64_t seed, uint32_t idx, uint32_t thresh) {
  if (thresh == 0u) return true;
  const uint32_t h = fer_hash(seed, idx >> 1);
  return ((h >> ((idx & 1) * 16)) & 0xFFFFu) >= thresh;
}
// Keep bits of 4 consecutive elements starting at an even index (two hashes): bit r = element r.
FER_DEV uint32_t keep4(uint64_t seed, uint32_t idx, uint32_t thresh) {
  const uint32_t h0 = fer_hash(seed, idx >> 1), h1 = fer_hash(seed, (idx >> 1) + 1);
  return (uint32_t)((h0 & 0xFFFFu) >= thresh) | ((uint32_t)((h0 >> 16) >= thresh) << 1) |
         ((uint32_t)((h1 & 0xFFFFu) >= thresh) << 2) | ((uint32_t)((h1 >> 16) >= thresh) << 3);
}
// 4 consecutive elements starting at an even index: two hashes.
FER_DEV void drop4(uint64_t seed, uint32_t idx, uint32_t thresh, float scale, f32x4& v) {
  if (thresh == 0u) return;
  const uint32_t h0 = fer_hash(seed, idx >> 1), h1 = fer_hash(seed, (idx >> 1) + 1);
  v[0] = (h0 & 0xFFFFu) >= thresh ? v[0] * scale : 0.f;
  v[1] = (h0 >> 16) >= thresh ? v[1] * scale : 0.f;
  v[2] = (h1 & 0xFFFFu) >= thresh ? v[2] * scale : 0.f;
  v[3] = (h1 >> 16) >= thresh ? v[3] * scale : 0.f;
}

// ---------------------------------------------------------------- reductions
// Combine a value with the other 32-lane half of the wave (lane l with l ^ 32) by
// v_permlane32_swap: VALU only, no ds_bpermute round trip through the LDS pipe. The swap of v with
// itself gives {own, partner} in lanes 0-31 and {partner, own} in 32-63; max / sum are symmetric,
// so both halves get bit-identical results.
FER_DEV float xhalf_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
FER_DEV float xhalf_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
FER_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
FER_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------- buffer rsrc
// Raw buffer descriptor. Loads whose voffset >= num_records return 0: kernels
// s_waitcnt vmcnt(N): all but this wave's N youngest vector-memory ops (loads, stores, LDS-DMA,
// in issue order) are done.
template <int N>
FER_DEV void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// mask out-of-tile lanes by giving them FER_OOB as voffset.
#define FER_OOB 0x80000000u

// Buffer descriptor as four dwords (same fields as make_rsrc) for the inline-asm LDS-DMA below.
FER_DEV u32x4 rsrc4(const void* base) {
  const uint64_t a = (uint64_t)base;
  return u32x4{(uint32_t)a, (uint32_t)(a >> 32) & 0xFFFFu, 0x7FFFFFF0u, 0x00020000u};
}
FER_DEV uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p; }
// LDS-DMA (buffer_load ... lds; lane l's 16 or 4 bytes land at lds + 16*l / 4*l) issued by inline
// asm: the compiler's wait-count pass does not see the LDS write, so it neither pads every later
// LDS read with s_waitcnt vmcnt(0) (it cannot tell the DMA target from the other LDS data) nor
// orders anything against it -- the issuing wave waits (wait_vm) before the data is read.
// s_nop: an SALU write of M0 needs one wait state before an LDS-DMA reads it. M0 is reserved by the
// compiler (a clobber is not honoured), so the asm saves and restores it.
FER_DEV void dma16_asm(const void* lds, const u32x4& rs, uint32_t voff) {
  uint32_t t;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(t) : "s"(lds_addr(lds)), "v"(voff), "s"(rs) : "memory");
}
FER_DEV void dma4_asm(const void* lds, const u32x4& rs, uint32_t voff) {
  uint32_t t;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dword %2, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(t) : "s"(lds_addr(lds)), "v"(voff), "s"(rs) : "memory");
}
// Workgroup barrier for LDS data only: no vmcnt(0) (__syncthreads' release fence waits for every
// outstanding global load and store of the wave -- prefetches and stores would be exposed at
// every barrier). Data that arrived by LDS-DMA must be waited for by its issuing wave first.
FER_DEV void bar_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
FER_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)0x7FFFFFF0, 0x00020000);
}

// ---------------------------------------------------------------- dynamic work queues
// Persistent kernels (one workgroup per CU) claim their work items from a device counter instead
// of walking a fixed blockIdx stride. With a fixed stride, a workgroup whose CU is held by another
// stream's kernel (RCCL's all-reduce during the DDP-overlapped backward, the weight-gradient
// stream) only starts once some other workgroup of this kernel has EXITED, i.e. after all of its
// items: the kernels ran 55-80 % longer with 16 of 256 CUs held (tools/hog_bench.py). Claiming
// items dynamically, a late workgroup finds the queue drained.
// Items are split into 8 classes (item & 7; blockIdx & 7 is the XCD a round-robin dispatch puts a
// block on, so an XCD keeps walking its own L2-friendly share). Workgroup b's first item is b
// itself (no claim at kernel start); the rest of class c is claimed from counter c, each on its own
// 4 KB page. The counters are never reset: the host keeps each one's value at the start of the
// launch (`base`, exact because every launch makes a known number of claims: one per dynamic
// item plus one failing claim per workgroup that held an item), so a launch needs no exit
// counter and no reset. Slots are per code object and per stream; under stream capture (the
// replayed graph could not keep the bases current) the kernels walk the fixed stride.
constexpr int FER_WQ_SLOTS = 32;
constexpr int FER_WQ_PAD = 1024;
static __device__ int fer_wq[FER_WQ_SLOTS][8 * FER_WQ_PAD];

struct WqArgs {
  int* q;  // null: fixed stride
  uint32_t base[8];
};

// First item of this workgroup (-1: none).
FER_DEV int wq_first(int n) { return (int)blockIdx.x < n ? (int)blockIdx.x : -1; }
// Next item of this workgroup's class; -1 when drained (then claim no more).
FER_DEV int wq_claim(int* q, const uint32_t* base, int n) {
  const int cls = blockIdx.x & 7;
  const uint32_t t =
      (uint32_t)__hip_atomic_fetch_add(q + cls * FER_WQ_PAD, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
      base[cls];
  const int nwg = ((int)gridDim.x - cls + 7) >> 3, items = (n - cls + 7) >> 3;
  return (long)t < (long)items - nwg ? cls + 8 * (nwg + (int)t) : -1;
}
// The same claim in two halves: issue the atomic early, read its result only where it is needed (an
// atomic with return counts in vmcnt: consuming it right away exposes the whole round trip).
// The atomic is inline asm (a vector global_atomic_add with return, agent scope): the compiler's atomic
// optimizer would otherwise wrap it in a wave reduction whose readfirstlane waits for the result at once.
// The caller waits (s_waitcnt vmcnt) before reading the result, then passes it through an empty asm.
FER_DEV uint32_t wq_claim_issue(int* q) {
  uint32_t r;
  int* p = q + (blockIdx.x & 7) * FER_WQ_PAD;
  asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(r) : "v"(p), "v"(1) : "memory");
  return r;
}
FER_DEV int wq_claim_finish(uint32_t raw, const uint32_t* base, int n) {
  const int cls = blockIdx.x & 7;
  const uint32_t t = raw - base[cls];
  const int nwg = ((int)gridDim.x - cls + 7) >> 3, items = (n - cls + 7) >> 3;
  return (long)t < (long)items - nwg ? cls + 8 * (nwg + (int)t) : -1;
}
// Host state of this code object's queues: slots keyed by (device, stream) -- the counters live in
// the device's own copy of fer_wq, whose address is looked up per device -- and a slot whose
// launch failed is retired (the bases it advanced no longer match the counters), after which that
// (device, stream) walks the fixed stride.
struct WqHost {
  struct Slot {
    int* dev;
    uint32_t base[8];
    bool dead;
  };
  std::mutex mu;
  std::map<std::pair<int, hipStream_t>, Slot> slots;
  std::map<int, std::pair<int*, int>> pools;  // device -> (fer_wq on that device, slots used)
};
static inline WqHost& wq_host() {
  static WqHost h;
  return h;
}
// Host: the queue of this code object for a launch of `grid` workgroups over `n` items on `st`
// (q = null: fixed stride). Advances the slot's bases by the claims the launch will make.
static inline WqArgs wq_prepare_here(hipStream_t st, int grid, int n) {
  WqArgs a{};
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return a;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return a;
  WqHost& h = wq_host();
  std::lock_guard<std::mutex> lk(h.mu);
  auto pit = h.pools.find(dev);
  if (pit == h.pools.end()) {
    int* pool = nullptr;
    if (hipGetSymbolAddress((void**)&pool, HIP_SYMBOL(fer_wq)) != hipSuccess) pool = nullptr;
    pit = h.pools.emplace(dev, std::make_pair(pool, 0)).first;
  }
  if (!pit->second.first) return a;
  const auto key = std::make_pair(dev, st);
  auto it = h.slots.find(key);
  if (it == h.slots.end()) {
    if (pit->second.second >= FER_WQ_SLOTS) return a;  // more streams than slots: fixed stride
    WqHost::Slot sl{pit->second.first + 8 * FER_WQ_PAD * pit->second.second++, {}, false};
    it = h.slots.emplace(key, sl).first;
  }
  WqHost::Slot& sl = it->second;
  if (sl.dead) return a;
  a.q = sl.dev;
  for (int c = 0; c < 8; ++c) {
    a.base[c] = sl.base[c];
    const int nwg = std::max(0, (grid - c + 7) / 8), items = std::max(0, (n - c + 7) / 8);
    sl.base[c] += (uint32_t)(std::max(0, items - nwg) + std::min(nwg, items));
  }
  return a;
}
// Host: call right after a work-queue launch; when the launch did not go out, the slot of
// (current device, st) is retired (fixed stride from then on) instead of desynchronising silently.
static inline void wq_check_launch(hipStream_t st, const WqArgs& a) {
  if (!a.q || hipPeekAtLastError() == hipSuccess) return;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;
  WqHost& h = wq_host();
  std::lock_guard<std::mutex> lk(h.mu);
  auto it = h.slots.find(std::make_pair(dev, st));
  if (it != h.slots.end()) it->second.dead = true;
}
