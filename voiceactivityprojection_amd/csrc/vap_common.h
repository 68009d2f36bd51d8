// Shared device helpers for the VAP MI355X engine (gfx950 / CDNA4 only).
//
// Precision model: "storage" type T feeds the matrix cores.
//   T = __bf16 : perf mode, v_mfma_f32_16x16x32_bf16 (fp32 accumulate)
//   T = float  : parity mode, v_mfma_f32_16x16x4_f32 (exact fp32 fmaf chain)
// Both share one fragment geometry: every lane reads 16 contiguous bytes of a K-contiguous
// row ([row][k] layout) -- 8 bf16 (one 16x16x32 MFMA) or 4 floats (four 16x16x4 MFMAs covering
// k-slots (lane>>4) with k = 4*(lane>>4)+j).  Accumulator (C/D) layout for both:
//   col = lane & 15, row = (lane >> 4) * 4 + r,  r = 0..3.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

#define VAP_DEV __device__ __forceinline__

VAP_DEV float to_f32(float x) { return x; }
VAP_DEV float to_f32(bf16 x) { return (float)x; }
template <typename T> VAP_DEV T from_f32(float x);
template <> VAP_DEV float from_f32<float>(float x) { return x; }
template <> VAP_DEV bf16 from_f32<bf16>(float x) { return (bf16)x; }

// 16-byte fragment chunk: 8 bf16 or 4 floats.
typedef u32x4 chunk16;

// One "16-byte k-chunk" MFMA step: acc += A_chunk(row=lane&15) x B_chunk(col=lane&15).
// bf16: 16x16x32 (chunk = k 8*(lane>>4)..+7 of a 32-wide k-step)
// f32 : 4 x 16x16x4 (chunk = k 4*(lane>>4)..+3 of a 16-wide k-step)
template <typename T> VAP_DEV f32x4 mfma_chunk(chunk16 a, chunk16 b, f32x4 acc);
template <> VAP_DEV f32x4 mfma_chunk<bf16>(chunk16 a, chunk16 b, f32x4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc,
                                                 0, 0, 0);
}
// NOTE: bit-cast the WHOLE vector.  hipcc (ROCm 7.2 clang) lowers __builtin_bit_cast(float, v[i]) on
// an ext_vector element to a load of element 0 whatever i is (verified in the .ll / .s).
template <> VAP_DEV f32x4 mfma_chunk<float>(chunk16 a, chunk16 b, f32x4 acc) {
  const f32x4 fa = __builtin_bit_cast(f32x4, a), fb = __builtin_bit_cast(f32x4, b);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[0], fb[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[1], fb[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[2], fb[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[3], fb[3], acc, 0, 0, 0);
  return acc;
}

// elements of T per 16-byte chunk
template <typename T> struct ChunkElems { static constexpr int v = 16 / sizeof(T); };

VAP_DEV float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
VAP_DEV float sigmoidf_(float x) { return 1.0f / (1.0f + __expf(-x)); }

// wave64 reductions without the LDS crossbar: DPP within rows of 16 (quad swaps, then half-row and
// row mirrors, each pairing two partial results of equal extent), then v_permlane16/32_swap across
// rows (inline asm: the builtins given equal operands are miscompiled).  Every pair is combined in
// both orders, so all 64 lanes end with the bit-identical result.
template <int CTRL>
VAP_DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <typename Op>
VAP_DEV float wave_reduce(float v, Op op) {
  v = op(v, dpp_f<0xB1>(v));   // quad_perm [1,0,3,2]: lane ^ 1
  v = op(v, dpp_f<0x4E>(v));   // quad_perm [2,3,0,1]: lane ^ 2
  v = op(v, dpp_f<0x141>(v));  // row_half_mirror: the other quad of the 8
  v = op(v, dpp_f<0x140>(v));  // row_mirror: the other 8 of the row
  float a = v, b = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  float c = op(a, b), d = c;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(c), "+v"(d));
  return op(c, d);
}
VAP_DEV float wave_sum(float v) {
  return wave_reduce(v, [](float x, float y) { return x + y; });
}
VAP_DEV float wave_max(float v) {
  return wave_reduce(v, [](float x, float y) { return fmaxf(x, y); });
}

// store 4 consecutive values as T
VAP_DEV void store4(float* p, float a, float b, float c, float d) { *(f32x4*)p = f32x4{a, b, c, d}; }
VAP_DEV void store4(bf16* p, float a, float b, float c, float d) {
  bf16x4 v = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
  *(bf16x4*)p = v;
}

// Buffer resource over [p, p + bytes) for raw buffer loads: out-of-range reads return 0 (the
// hardware range check replaces per-lane bounds branches).  p and bytes must be wave-uniform.
VAP_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* pu = (void*)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pu, 0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
VAP_DEV chunk16 buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(chunk16, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, (int)soff, 0));
}

// Range-checked buffer stores: a lane whose offset lies outside the resource writes nothing, so
// bounds are handled without branches (conditional stores also defeat the compiler's vmcnt
// bookkeeping for the loads issued after them).
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
VAP_DEV void buf_store8(__amdgpu_buffer_rsrc_t r, uint32_t voff, u32x2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)voff, 0, 0);
}
VAP_DEV void buf_store16(__amdgpu_buffer_rsrc_t r, uint32_t voff, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)voff, 0, 0);
}
// write-through (sc1) 16-B store: the line leaves the XCD's L2 with the store instead of staying
// dirty, so the kernel's end-of-launch L2 write-back (~ dirty bytes / 6 TB/s on the next launch's
// critical path) has nothing to do.  16-B only: narrower sc1 stores are one fabric write each.
VAP_DEV void buf_store16_wt(__amdgpu_buffer_rsrc_t r, uint32_t voff, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)voff, 0, 16);
}
VAP_DEV u32x2 pack_bf16x4(float a, float b, float c, float d) {
  const bf16x4 v = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
  return __builtin_bit_cast(u32x2, v);
}

// GELU(x) = x * Phi(x) with Phi from the erfc approximation of Abramowitz & Stegun 7.1.26
// (|erf error| <= 1.5e-7, i.e. |GELU error| <= 7.5e-8 |x|): one v_rcp, one v_exp and ~10 FMAs
// instead of the ~50-instruction erff.  Used where the result is rounded to bf16.
VAP_DEV float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, z, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float h = 0.5f * p * t * __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f);  // erfc(z) / 2
  return x * (x >= 0.f ? 1.0f - h : h);
}

// gelu_fast on two values with packed f32 math (v_pk_mul/v_pk_fma: two lanes' worth per
// instruction) and the constants folded: z = |x| sqrt(log2e / 2) so that exp(-x^2 / 2) = exp2(-z^2),
// and GELU = max(x, 0) - |x| erfc(|x| / sqrt2) / 2 = ((x + |x|) - z h) / 2 with the A&S 7.1.26
// coefficients pre-scaled by 1 / sqrt(log2e / 2) (no sign select, no max).
typedef float f32x2 __attribute__((ext_vector_type(2)));
VAP_DEV f32x2 gelu_fast2(f32x2 x) {
  const f32x2 a = __builtin_elementwise_abs(x);
  const f32x2 z = a * 0.84932180028801907f;
  const f32x2 d = __builtin_elementwise_fma(z, (f32x2)0.27273748087922250f, (f32x2)1.0f);
  const f32x2 t = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f32x2 p = __builtin_elementwise_fma(t, (f32x2)1.249709390056937f, (f32x2)-1.7109557608284776f);
  p = __builtin_elementwise_fma(p, t, (f32x2)1.673586784794615f);
  p = __builtin_elementwise_fma(p, t, (f32x2)-0.334969308339339f);
  p = __builtin_elementwise_fma(p, t, (f32x2)0.3000389156543292f);
  const f32x2 e = z * -z;
  const f32x2 h = p * t * (f32x2){__builtin_amdgcn_exp2f(e[0]), __builtin_amdgcn_exp2f(e[1])};
  return __builtin_elementwise_fma(-z, h, x + a) * 0.5f;
}
