// Shared device helpers for libsam2hip (gfx950 / CDNA4 only).
//
// Element types: every compute kernel is templated on the storage type T of its
// activations: `float` (fp32-parity mode, f32-input MFMA 16x16x4) or `__bf16`
// (performance mode, bf16 MFMA 16x16x32).  Accumulation is always fp32.
#pragma once

// frames one frame-batched launch can cover (the tracking loop's frames, T <= 32)
#define S2H_MAX_FRAMES 32
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

enum S2HDtype { S2H_F32 = 0, S2H_BF16 = 1 };

#define S2H_WAVE 64

__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f32<bf16>(float x) { return (bf16)x; }

// ---------------------------------------------------------------------------
// MFMA traits.  Both shapes are 16x16 output tiles with the dtype-independent
// C/D layout: lane l holds column (l & 15), rows 4*(l >> 4) + r, r = 0..3.
// Operand layout: lane l supplies A[row l&15][k = (l>>4)*KPL + j] and
// B[k = (l>>4)*KPL + j][col l&15], j < KPL, one instruction covers KSTEP = 4*KPL.
// ---------------------------------------------------------------------------
template <typename T> struct Mfma;
template <> struct Mfma<bf16> {
  static constexpr int KPL = 8;
  static constexpr int KSTEP = 32;
  typedef bf16x8 frag;
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ frag load(const bf16* p) { return *(const bf16x8*)p; }
  static __device__ __forceinline__ frag zero() { frag z; for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f; return z; }
};
template <> struct Mfma<float> {
  static constexpr int KPL = 1;
  static constexpr int KSTEP = 4;
  typedef float frag;
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ frag load(const float* p) { return *p; }
  static __device__ __forceinline__ frag zero() { return 0.f; }
};

// 16-byte vector of T (8 bf16 or 4 f32) for coalesced global loads.
template <typename T> struct Vec16;
template <> struct Vec16<bf16> { static constexpr int N = 8; typedef uint4 raw; };
template <> struct Vec16<float> { static constexpr int N = 4; typedef uint4 raw; };

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
// reduce across the 16 lanes that share (lane >> 4) -- one MFMA row group
__device__ __forceinline__ float row16_sum(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Counter-based dropout RNG.  keep(i) is a pure function of (seed, element index), so
// forward and backward regenerate the same mask without storing it.  One 32-bit hash
// (lowbias32 finaliser: 2 multiplies, 3 xor-shifts) serves an even/odd PAIR of elements
// (16 bits each, drop probability quantised to 1/65536): dropout sits inside the
// attention softmax, where a 64-bit splitmix per element cost more VALU than the math.
__device__ __forceinline__ uint32_t s2h_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t s2h_hash_pair(uint64_t seed, uint64_t pair) {
  const uint32_t key = s2h_mix32((uint32_t)seed ^ 0x5bd1e995u) ^ (uint32_t)(seed >> 32);
  return s2h_mix32(((uint32_t)pair + (uint32_t)(pair >> 32) * 0x9E3779B9u) ^ key);
}
// the two halves of s2h_hash_pair, for kernels that hoist the seed key and the high word:
// s2h_hash_pair(seed, pair) == s2h_hash_mixed(s2h_hash_key(seed), lo(pair) + hi(pair) * 0x9E3779B9)
__device__ __forceinline__ uint32_t s2h_hash_key(uint64_t seed) {
  return s2h_mix32((uint32_t)seed ^ 0x5bd1e995u) ^ (uint32_t)(seed >> 32);
}
__device__ __forceinline__ uint32_t s2h_hash_mixed(uint32_t key, uint32_t x) { return s2h_mix32(x ^ key); }
// thresh = p * 2^32 (the 16 high bits are used)
__device__ __forceinline__ bool s2h_keep(uint64_t seed, uint64_t idx, uint32_t thresh) {
  const uint32_t h = s2h_hash_pair(seed, idx >> 1);
  const uint32_t u = (idx & 1) ? (h >> 16) : (h & 0xFFFFu);
  return u >= (thresh >> 16);
}
// keep flags of elements 2*pair and 2*pair + 1 from one hash
__device__ __forceinline__ void s2h_keep_pair(uint64_t seed, uint64_t pair, uint32_t thresh, bool& k0, bool& k1) {
  const uint32_t h = s2h_hash_pair(seed, pair);
  k0 = (h & 0xFFFFu) >= (thresh >> 16);
  k1 = (h >> 16) >= (thresh >> 16);
}

// Device-resident RNG offset.  The host binds one uint64 in device memory with s2h_rng_bind;
// every dropout site folds its value into the per-launch seed when the kernel starts, so a
// captured HIP graph replays with fresh dropout masks after the host advances the offset
// (forward and backward of one step read the same value, so the backward regenerates the
// forward's masks).  Offset 0 (or nothing bound) leaves the seed unchanged.
const uint64_t* s2h_rng_offset_ptr();  // host side (runtime.hip)
__device__ __forceinline__ uint64_t s2h_seed(uint64_t seed, const uint64_t* off) {
  if (!off) return seed;
  const uint64_t o = *off;
  return o ? seed ^ (o * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) : seed;
}

// GELU (exact erf form, nn.GELU() of the reference's MLPs / CXBlock / mask decoder) through the normal
// CDF Phi(x) = 0.5 erfc(-x / sqrt 2), with erfc(a) = t exp(-a^2 + P(t)), t = 1 / (1 + a / 2), a >= 0: the
// Chebyshev fit of Numerical Recipes' erfcc (fractional error < 1.2e-7 for every a), one v_rcp, one
// v_exp and 9 FMAs, branch-free.  Round 6: it replaces ocml erff (~35 VALU with a |x| < 1 branch that
// divergent lanes take both ways) in the GEMM epilogues of the Hiera MLP fc1 (462 M elements per bench
// step, forward and backward) and the memory fuser; erfc's relative accuracy also holds in the far
// negative tail where 1 + erff(x) cancelled to a few bits.
__device__ __forceinline__ float s2h_erfc_exp_arg(float a, float t) {  // -a^2 + P(t): erfc(a) = t exp(this)
  float p = 0.17087277f;
  p = fmaf(t, p, -0.82215223f);
  p = fmaf(t, p, 1.48851587f);
  p = fmaf(t, p, -1.13520398f);
  p = fmaf(t, p, 0.27886807f);
  p = fmaf(t, p, -0.18628806f);
  p = fmaf(t, p, 0.09678418f);
  p = fmaf(t, p, 0.37409196f);
  p = fmaf(t, p, 1.00002368f);
  p = fmaf(t, p, -1.26551223f);
  return fmaf(-a, a, p);
}
__device__ __forceinline__ float s2h_normal_cdf(float x) {  // Phi(x)
  const float a = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.5f, a, 1.f));
  const float h = 0.5f * t * __builtin_amdgcn_exp2f(s2h_erfc_exp_arg(a, t) * 1.4426950408889634f);  // 0.5 erfc(a)
  return x >= 0.f ? 1.f - h : h;
}
__device__ __forceinline__ float gelu_erf(float x) { return x * s2h_normal_cdf(x); }
__device__ __forceinline__ float gelu_erf_grad(float x) {
  const float pdf = 0.39894228040143268f * __builtin_amdgcn_exp2f(-0.72134752044448170f * x * x);  // phi(x)
  return fmaf(x, pdf, s2h_normal_cdf(x));
}

enum S2HAct { S2H_ACT_NONE = 0, S2H_ACT_RELU = 1, S2H_ACT_GELU = 2, S2H_ACT_SIGMOID = 3 };

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == S2H_ACT_RELU) return fmaxf(v, 0.f);
  if (act == S2H_ACT_GELU) return gelu_erf(v);
  if (act == S2H_ACT_SIGMOID) return 1.f / (1.f + expf(-v));
  return v;
}

// derivative of the activation, evaluated at the pre-activation value x
__device__ __forceinline__ float act_grad(float x, int act) {
  if (act == S2H_ACT_RELU) return x > 0.f ? 1.f : 0.f;
  if (act == S2H_ACT_GELU) return gelu_erf_grad(x);
  if (act == S2H_ACT_SIGMOID) { float s = 1.f / (1.f + expf(-x)); return s * (1.f - s); }
  return 1.f;
}

#define S2H_LAUNCH_CHECK() return (int)hipGetLastError()

// Zero-fill as a KERNEL on `st` (elementwise.hip).  Used instead of hipMemset*Async: inside a
// captured HIP graph the memset nodes were observed to break stream order against the kernel
// nodes around them on ROCm 7.2 (garbage loss values in replays), kernel nodes never do.
// rows x cols floats with row stride ld (ld == cols: one contiguous range).
void s2h_zero_f32(float* p, int64_t rows, int64_t cols, int64_t ld, hipStream_t st);

// Deterministic reductions (round 5): the workspace registered by s2h_wgrad_workspace (gemm_wgrad.hip)
// for kernels that write per-block partials and add them in fixed order in a second pass instead of
// float atomics; nullptr when none is registered, it is switched off or smaller than `bytes` (the caller
// then keeps its atomic path).  Users are stream-ordered (one stream).
float* s2h_det_ws(int64_t bytes);
// its usable size in bytes (0: none registered or switched off)
int64_t s2h_det_ws_bytes();
// Deferred second pass (grad_defer.hip): inside a s2h_grad_defer scope, partial storage for nb rows of
// n0 + n1 columns whose fixed-order column sums go to out0[0:n0] (+=) and out1[0:n1] (+=), recorded for
// s2h_grad_defer_flush; nullptr when no scope is open or a destination is outside the registered sink
// (the caller then runs its own second pass).
float* s2h_defer_sink(int nb, int n0, float* out0, int n1, float* out1, hipStream_t st);

// LDS-DMA (global_load_lds_dwordx4 / _dword: 16 / 4 B per lane into lds_piece + lane * size)
// issued through inline asm.  Issued through the builtin, the compiler's waitcnt pass sees an
// LDS write it cannot tell apart from later ds_reads and puts s_waitcnt vmcnt(0) before the
// first ds_read after it -- draining every DMA still in flight and serialising a multi-stage
// ring.  Callers order these with their own counted s_waitcnt vmcnt + s_barrier.
__device__ __forceinline__ void lds_dma16(const void* src, const void* lds_piece) {
  const uint32_t m0 =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)lds_piece);
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
}
// one 1-KiB LDS-DMA piece from a wave-uniform row base (SGPR pair) + this lane's 32-bit byte offset
// (global_load_lds_dwordx4, saddr form): the building block of PadDma and of the backward kernels'
// precomputed-offset stage loads
__device__ __forceinline__ uint64_t sgpr_base(const void* p) {
  const uint64_t b = (uint64_t)(uintptr_t)p;
  // (readfirstlane returns int: through uint32_t, or the low word's sign bit smears into the high one)
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(b >> 32)) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)b);
}
__device__ __forceinline__ void lds_dma16_so(uint64_t sbase, uint32_t voff, const void* lds_piece) {
  const uint32_t m0 =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)lds_piece);
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(m0) : "memory", "m0");
}
// the same with the piece's LDS byte address given as an integer (lds_u32 of the __shared__ array plus
// an offset): no generic -> LDS pointer cast at the call (its null test came out as an illegal VALU
// compare against src_shared_base in some GEMM instantiations)
__device__ __forceinline__ void lds_dma16_sm(uint64_t sbase, uint32_t voff, uint32_t lds_addr) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile("s_mov_b32 m0, %2\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "s"(m0) : "memory", "m0");
}
// LDS byte address of a __shared__ array (call it on the array itself)
template <typename T>
__device__ __forceinline__ uint32_t lds_u32(T* shared_array) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) T*)shared_array;
}

// lds_dma16 with the LDS byte address as an integer (see lds_dma16_sm)
__device__ __forceinline__ void lds_dma16_m(const void* src, uint32_t lds_addr) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_addr);
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
}
__device__ __forceinline__ void lds_dma4(const void* src, const void* lds_piece) {
  const uint32_t m0 =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)lds_piece);
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dword %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
}
