// GEMM epilogue shared by the bf16 (gemm_bf16.hip) and MX-fp8 (gemm_mx8.hip) kernels: the
// fp32 accumulator tile of one wave goes through a wave-private LDS slab and is finished
// 4 / 8 columns per lane (bias, activation or act' of a saved pre-activation, column scale,
// dropout, residual, beta, bf16 / fp32 / split-K atomic stores).
#pragma once
#include <type_traits>

#include "gemm16.h"

// Output stores are non-temporal (streamed past the caches toward HBM): GEMM outputs are read
// back by a later kernel, not by this one, and tools/epi_bench.py measured them 5-25 % faster
// than plain stores at every tiling (93184x2048x256 bf16: 297 -> 223 us; the MX-fp8 kernel
// 229 -> 165 us).  GemmArgs16::dbg bit 8 restores plain stores for A/B measurements.
typedef uint32_t s2h_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t s2h_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st16_nt(void* ptr, uint4 v, bool plain) {
  if (plain) { *(uint4*)ptr = v; return; }
  __builtin_nontemporal_store(s2h_u32x4{v.x, v.y, v.z, v.w}, (s2h_u32x4*)ptr);
}
__device__ __forceinline__ void st8b_nt(void* ptr, uint2 v, bool plain) {
  if (plain) { *(uint2*)ptr = v; return; }
  __builtin_nontemporal_store(s2h_u32x2{v.x, v.y}, (s2h_u32x2*)ptr);
}

// Finishes outputs (row, col0..col0+3) of batch bz from the fp32 accumulators v4.
// Every epilogue option is tested ONCE per 4-column group (uniform scalar branches around
// 4-wide straight-line code), never per element: per-element option tests made the epilogue
// SALU-bound (~1.7k SALU + 1.2k VALU instructions per wave for 32 MFMAs at K = 64).
// `bcol` holds the lane's 4 column biases (loaded once per tile by the caller).
__device__ __forceinline__ uint2 ld4_bf16(const bf16* ptr, bool full) {
  if (full) return *(const uint2*)ptr;
  return make_uint2(0, 0);
}
// axial RoPE of NV consecutive output columns (col0 even) of `row` (GemmArgs16 rope_* fields)
template <int NV>
__device__ __forceinline__ void rope_cols(const GemmArgs16& p, int row, int col0, float* v) {
  if (p.rope_cos == nullptr || col0 >= p.rope_ncol) return;
  const int l = row % p.rope_L;
  if (l >= p.rope_nrot) return;
  const int half = p.rope_dh / 2;
  const int t = (l % p.rope_period) * half + (col0 % p.rope_dh) / 2;
#pragma unroll
  for (int j = 0; j < NV / 2; ++j) {
    const float co = p.rope_cos[t + j], si = p.rope_sin[t + j];
    const float x0 = v[2 * j], x1 = v[2 * j + 1];
    v[2 * j] = x0 * co - x1 * si;
    v[2 * j + 1] = x0 * si + x1 * co;
  }
}

__device__ __forceinline__ void epilogue4(const GemmArgs16& p, int bz, int row, int col0, float4 v4, const float* bcol,
                                          int split = 0) {
  float v[4] = {v4.x, v4.y, v4.z, v4.w};
  const int nval = p.N - col0;
  if (nval <= 0) return;
  const bool full = nval >= 4 && p.vecC;
  if (p.splits > 1) {  // split-K: the partial tile (gemm16.h), or fp32 atomics (beta handled on the host side)
    if (p.X) {
      float* P = (float*)p.X + split * p.sX + ((int64_t)bz * p.M + row) * p.N + col0;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (e < nval) P[e] = p.alpha * v[e];
      return;
    }
    float* C = (float*)p.C + (int64_t)bz * p.sC + (int64_t)row * p.ldc + col0;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (e < nval) atomicAdd(C + e, p.alpha * v[e]);
    return;
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = p.alpha * v[e] + bcol[e];
  if (p.bias_mode == 2) {
    const float br = p.bias[row];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] += br;
  }
  if (p.aux_mode == 1) {  // store the pre-activation
    bf16* X = (bf16*)p.X + (int64_t)bz * p.sX + (int64_t)row * p.ldx + col0;
    if (full && p.ldx % 4 == 0) {
      bf16 t[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] = (bf16)v[e];
      st8b_nt(X, *(const uint2*)t, p.dbg & 8);
    } else {
      _Pragma("unroll") for (int e = 0; e < 4; ++e) if (e < nval) X[e] = (bf16)v[e];
    }
  }
  if (p.aux_mode == 2) {  // multiply by act'(pre-activation)
    const bf16* X = (const bf16*)p.X + (int64_t)bz * p.sX + (int64_t)row * p.ldx + col0;
    float xs[4];
    if (full && p.ldx % 4 == 0) {
      const uint2 r = *(const uint2*)X;
      const bf16* rb = (const bf16*)&r;
#pragma unroll
      for (int e = 0; e < 4; ++e) xs[e] = (float)rb[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) xs[e] = e < nval ? (float)X[e] : 0.f;
    }
    if (p.act == S2H_ACT_RELU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = xs[e] > 0.f ? v[e] : 0.f;
    } else if (p.act != S2H_ACT_NONE) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] *= act_grad(xs[e], p.act);
    }
  } else if (p.act == S2H_ACT_RELU) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
  } else if (p.act != S2H_ACT_NONE) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = apply_act(v[e], p.act);
  }
  rope_cols<4>(p, row, col0, v);
  if (p.cscale) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] *= e < nval ? p.cscale[col0 + e] : 0.f;
  }
  if (p.drop_p > 0.f) {
    const uint32_t thresh = (uint32_t)(p.drop_p * 4294967296.0);
    const float inv_keep = 1.f / (1.f - p.drop_p);
    const uint64_t idx0 = p.drop_idx0 + (uint64_t)bz * p.M * p.N + (uint64_t)row * p.N + col0;
    bool k[4];
    if ((idx0 & 1) == 0) {
      s2h_keep_pair(p.seed, idx0 >> 1, thresh, k[0], k[1]);
      s2h_keep_pair(p.seed, (idx0 >> 1) + 1, thresh, k[2], k[3]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) k[e] = s2h_keep(p.seed, idx0 + e, thresh);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = k[e] ? v[e] * inv_keep : 0.f;
  }
  if (p.R) {
    const bf16* R = (const bf16*)p.R + (int64_t)bz * p.sR + (int64_t)row * p.ldr + col0;
    if (full && p.ldr % 4 == 0) {
      const uint2 r = *(const uint2*)R;
      const bf16* rb = (const bf16*)&r;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += (float)rb[e];
    } else {
      _Pragma("unroll") for (int e = 0; e < 4; ++e) if (e < nval) v[e] += (float)R[e];
    }
  }
  const int64_t co = (int64_t)bz * p.sC + (int64_t)row * p.ldc + col0;
  if (p.out_f32) {
    float* C = (float*)p.C + co;
    if (full) {
      float4 o = {v[0], v[1], v[2], v[3]};
      if (p.beta != 0.f) {
        const float4 c = *(const float4*)C;
        o.x += p.beta * c.x; o.y += p.beta * c.y; o.z += p.beta * c.z; o.w += p.beta * c.w;
      }
      st16_nt(C, *(const uint4*)&o, p.dbg & 8);
    } else {
      _Pragma("unroll") for (int e = 0; e < 4; ++e) if (e < nval) C[e] = v[e] + (p.beta != 0.f ? p.beta * C[e] : 0.f);
    }
  } else {
    bf16* C = (bf16*)p.C + co;
    if (full) {
      bf16 o[4];
      if (p.beta != 0.f) {
        const uint2 c = *(const uint2*)C;
        const bf16* cb = (const bf16*)&c;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)(v[e] + p.beta * (float)cb[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (bf16)v[e];
      }
      st8b_nt(C, *(const uint2*)o, p.dbg & 8);
    } else {
      _Pragma("unroll") for (int e = 0; e < 4; ++e) if (e < nval) C[e] = (bf16)(v[e] + (p.beta != 0.f ? p.beta * (float)C[e] : 0.f));
    }
  }
}

// 8 consecutive bf16 outputs (row, col0..col0+7) with one 16-B access per operand -- the
// store-issue-bound tail of a GEMM costs per instruction, not per byte (the 4-column form
// issues twice the stores).  Requires (checked by the caller) 8 valid columns, no split-K, a
// bf16 output and vec8 bit 0; X / R fall back to two 8-B accesses when their bit is clear.
__device__ __forceinline__ void ld8_bf16(const bf16* ptr, bool wide, float* out) {
  if (wide) {
    const uint4 r = *(const uint4*)ptr;
    const bf16* rb = (const bf16*)&r;
#pragma unroll
    for (int e = 0; e < 8; ++e) out[e] = (float)rb[e];
  } else {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint2 r = *(const uint2*)(ptr + 4 * h);
      const bf16* rb = (const bf16*)&r;
#pragma unroll
      for (int e = 0; e < 4; ++e) out[4 * h + e] = (float)rb[e];
    }
  }
}
__device__ __forceinline__ void st8_bf16(bf16* ptr, bool wide, const float* v, bool plain) {
  bf16 t[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) t[e] = (bf16)v[e];
  if (wide) {
    st16_nt(ptr, *(const uint4*)t, plain);
  } else {
    st8b_nt(ptr, *(const uint2*)t, plain);
    st8b_nt(ptr + 4, *(const uint2*)(t + 4), plain);
  }
}
__device__ __forceinline__ void epilogue8(const GemmArgs16& p, int bz, int row, int col0, const float* vin,
                                          const float* bcol) {
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = p.alpha * vin[e] + bcol[e];
  if (p.bias_mode == 2) {
    const float br = p.bias[row];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += br;
  }
  const bool wx = (p.vec8 & 2) != 0, wr = (p.vec8 & 4) != 0;
  if (p.aux_mode == 1) st8_bf16((bf16*)p.X + (int64_t)bz * p.sX + (int64_t)row * p.ldx + col0, wx, v, p.dbg & 8);
  if (p.aux_mode == 2) {
    float xs[8];
    ld8_bf16((const bf16*)p.X + (int64_t)bz * p.sX + (int64_t)row * p.ldx + col0, wx, xs);
    if (p.act == S2H_ACT_RELU) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = xs[e] > 0.f ? v[e] : 0.f;
    } else if (p.act != S2H_ACT_NONE) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] *= act_grad(xs[e], p.act);
    }
  } else if (p.act == S2H_ACT_RELU) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
  } else if (p.act != S2H_ACT_NONE) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = apply_act(v[e], p.act);
  }
  rope_cols<8>(p, row, col0, v);
  if (p.cscale) {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= p.cscale[col0 + e];
  }
  if (p.drop_p > 0.f) {
    const uint32_t thresh = (uint32_t)(p.drop_p * 4294967296.0);
    const float inv_keep = 1.f / (1.f - p.drop_p);
    const uint64_t idx0 = p.drop_idx0 + (uint64_t)bz * p.M * p.N + (uint64_t)row * p.N + col0;
    bool k[8];
    if ((idx0 & 1) == 0) {
#pragma unroll
      for (int h = 0; h < 4; ++h) s2h_keep_pair(p.seed, (idx0 >> 1) + h, thresh, k[2 * h], k[2 * h + 1]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) k[e] = s2h_keep(p.seed, idx0 + e, thresh);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = k[e] ? v[e] * inv_keep : 0.f;
  }
  if (p.R) {
    float rs[8];
    ld8_bf16((const bf16*)p.R + (int64_t)bz * p.sR + (int64_t)row * p.ldr + col0, wr, rs);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += rs[e];
  }
  bf16* C = (bf16*)p.C + (int64_t)bz * p.sC + (int64_t)row * p.ldc + col0;
  if (p.beta != 0.f) {
    float cs[8];
    ld8_bf16(C, true, cs);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += p.beta * cs[e];
  }
  st8_bf16(C, true, v, p.dbg & 8);
}

// epilogue8 + LayerNorm of the row (GemmArgs16 ln_*): the CPR lanes of one output row each hold 8
// of its columns (CPR * 8 == N), so the row statistics are a CPR-lane xor reduction.  x' = R +
// drop(alpha acc + bias) is rounded to bf16 (the residual stream as stored) before the statistics,
// as the standalone LayerNorm kernel reads it (norm.hip ln_fwd_vec_kernel: two-pass variance).
// Every lane of the wave calls this (the shuffles need them all); `live` guards the stores.
template <int CPR>
__device__ __forceinline__ void epilogue8_ln(const GemmArgs16Ln& p, int bz, int row, int col0, const float* vin,
                                             const float* bcol, bool live) {
  float v[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = p.alpha * vin[e] + bcol[e];
  if (p.drop_p > 0.f) {
    const uint32_t thresh = (uint32_t)(p.drop_p * 4294967296.0);
    const float inv_keep = 1.f / (1.f - p.drop_p);
    const uint64_t idx0 = p.drop_idx0 + (uint64_t)bz * p.M * p.N + (uint64_t)row * p.N + col0;
    bool k[8];
    if ((idx0 & 1) == 0) {
#pragma unroll
      for (int h = 0; h < 4; ++h) s2h_keep_pair(p.seed, (idx0 >> 1) + h, thresh, k[2 * h], k[2 * h + 1]);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) k[e] = s2h_keep(p.seed, idx0 + e, thresh);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = k[e] ? v[e] * inv_keep : 0.f;
  }
  if (p.R && live) {
    float rs[8];
    ld8_bf16((const bf16*)p.R + (int64_t)bz * p.sR + (int64_t)row * p.ldr + col0, (p.vec8 & 4) != 0, rs);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] += rs[e];
  }
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    v[e] = (float)(bf16)v[e];
    s += v[e];
  }
#pragma unroll
  for (int o = CPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mu = s / p.N;
  float q = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float d = v[e] - mu;
    q += d * d;
  }
#pragma unroll
  for (int o = CPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rs = 1.f / sqrtf(q / p.N + p.ln_eps);
  if (!live) return;
  st8_bf16((bf16*)p.C + (int64_t)bz * p.sC + (int64_t)row * p.ldc + col0, true, v, p.dbg & 8);
  float y[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) y[e] = (v[e] - mu) * rs * p.ln_gamma[col0 + e] + p.ln_beta[col0 + e];
  st8_bf16((bf16*)p.ln_y + (int64_t)bz * p.M * p.ln_ldy + (int64_t)row * p.ln_ldy + col0, true, y, p.dbg & 8);
  if (col0 == 0) {
    p.ln_mean[(int64_t)bz * p.M + row] = mu;
    p.ln_rstd[(int64_t)bz * p.M + row] = rs;
  }
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// the lane's 4 column biases (zeros when the bias is absent or per row)
template <int V = 4>
__device__ __forceinline__ void load_bcol(const GemmArgs16& p, int col0, float* bcol) {
#pragma unroll
  for (int e = 0; e < V; ++e) bcol[e] = (p.splits == 1 && p.bias_mode == 1 && col0 + e < p.N) ? p.bias[col0 + e] : 0.f;
}

// the fused row sum of A over one split's K chunk (GemmArgs16::rowsum): into the split's partial slot
// when the launch has partial storage (gemm16.h), else a float atomic (one adder per element unsplit)
__device__ __forceinline__ void store_rowsum(const GemmArgs16& p, int bz, int split, int m, float rs) {
  if (p.splits > 1 && p.X) {
    const int batch = gridDim.z / p.splits;
    ((float*)p.X)[p.splits * p.sX + ((int64_t)split * batch + bz) * p.M + m] = rs;
  } else {
    atomicAdd(&p.rowsum[(int64_t)bz * p.M + m], rs);
  }
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Epilogue of one wave's WM x WN accumulator block through a wave-private LDS slab `ep`
// (16 x (WN + 4) fp32): per 16-row slab, stage the accumulators, then every lane finishes 4
// consecutive columns of a row (epilogue4) with 8-/16-byte stores -- rows of a
// wave-instruction are 128-B column runs.  The slab is private to the wave, so no workgroup
// barrier: LDS operations of one wave retire in order.  (A register-direct variant with
// swapped MFMA operands -- 4 consecutive columns per lane, no staging -- measured 1.5-2.6x
// slower: its stores scatter 16 rows x 32 B per instruction, and split-K atomics likewise.)
// a LayerNorm epilogue requested (only the full-row tilings' argument block carries one)
__device__ __forceinline__ bool ln_epilogue_on(const GemmArgs16&) { return false; }
__device__ __forceinline__ bool ln_epilogue_on(const GemmArgs16Ln& p) { return p.ln_gamma != nullptr; }

template <int WM, int WN, int MI, int NI, typename PA = GemmArgs16>
__device__ __forceinline__ void tile_epilogue(const PA& p, f32x4 (&acc)[MI][NI], float* ep, int bz, int mw,
                                              int nw, int lane, int split = 0) {
  constexpr int EPLD = WN + 4;
  float bcol[4], bcol8[8];
  load_bcol(p, nw + 4 * (lane % (WN / 4)), bcol);
  load_bcol<8>(p, nw + 8 * (lane % (WN / 8 > 0 ? WN / 8 : 1)), bcol8);
  // compile-time slab index (a rolled loop would index acc dynamically -> scratch)
  static_for<0, MI>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) ep[(4 * (lane >> 4) + r) * EPLD + j * 16 + (lane & 15)] = acc[i][j][r];
    __builtin_amdgcn_wave_barrier();
    if (p.splits > 1) {
      // split-K: consecutive lanes on consecutive columns (256 B per instruction): RPI rows of
      // WN <= 64 columns, or 64-column pieces of one row for the full-row tiles (WN 128 / 256); plain
      // stores of the partial tile when the split has one (gemm16.h), else float atomics into C
      const bool part = p.X != nullptr;
      float* C = part ? (float*)p.X + split * p.sX + (int64_t)bz * p.M * p.N : (float*)p.C + (int64_t)bz * p.sC;
      const int64_t ldc = part ? (int64_t)p.N : p.ldc;
      if constexpr (WN <= 64) {
        constexpr int RPI = 64 / WN;  // rows per instruction
        const int col = nw + lane % WN;
        for (int rr = lane / WN; rr < 16; rr += RPI) {
          const int row = mw + i * 16 + rr;
          if (row < p.M && col < p.N) {
            const float v = p.alpha * ep[rr * EPLD + lane % WN];
            if (part) C[(int64_t)row * ldc + col] = v;
            else atomicAdd(&C[(int64_t)row * ldc + col], v);
          }
        }
      } else {
        for (int rr = 0; rr < 16; ++rr) {
          const int row = mw + i * 16 + rr;
#pragma unroll
          for (int cc = lane; cc < WN; cc += 64) {
            const int col = nw + cc;
            if (row < p.M && col < p.N) {
              const float v = p.alpha * ep[rr * EPLD + cc];
              if (part) C[(int64_t)row * ldc + col] = v;
              else atomicAdd(&C[(int64_t)row * ldc + col], v);
            }
          }
        }
      }
    } else if (WN >= 128 && WN % 32 == 0 && ln_epilogue_on(p)) {
      // LayerNorm of whole rows (s2h_linear_add_ln checked: N == WN, one wave per 16 full rows).
      // Instantiated for the full-row tiles only: compiled into every tiling, the extra epilogue
      // raised the 64x64 tile's VGPRs 63 -> 81 and cost 1.5 % of the step with the fusion unused
      if constexpr (WN >= 128 && WN % 32 == 0 && std::is_same_v<PA, GemmArgs16Ln>) {
        constexpr int CPR = WN / 8, RPP = 64 / CPR;
        const int c8 = lane % CPR, rg = lane / CPR;
        for (int ps = 0; ps < 16 / RPP; ++ps) {
          const int rl = rg + ps * RPP;
          const float4 lo = *(const float4*)&ep[rl * EPLD + 8 * c8];
          const float4 hi = *(const float4*)&ep[rl * EPLD + 8 * c8 + 4];
          const float v8[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
          const int row = mw + i * 16 + rl;
          epilogue8_ln<CPR>(p, bz, row, nw + 8 * c8, v8, bcol8, row < p.M && !(p.dbg & 1));
        }
      }
    } else if (WN % 32 == 0 && (p.vec8 & 1) && nw + WN <= p.N) {
      // 8 columns per lane, one 16-B store each (the wave's column block is entirely valid)
      constexpr int CPR = WN / 8, RPP = 64 / CPR;
      const int c8 = lane % CPR, rg = lane / CPR;
      for (int ps = 0; ps < 16 / RPP; ++ps) {
        const int rl = rg + ps * RPP;
        const float4 lo = *(const float4*)&ep[rl * EPLD + 8 * c8];
        const float4 hi = *(const float4*)&ep[rl * EPLD + 8 * c8 + 4];
        const float v8[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        const int row = mw + i * 16 + rl;
        if (row < p.M && !(p.dbg & 1)) epilogue8(p, bz, row, nw + 8 * c8, v8, bcol8);
      }
    } else {
      constexpr int CPR = WN / 4, RPP = 64 / CPR;
      const int c4 = lane % CPR, rg = lane / CPR;
      for (int ps = 0; ps < 16 / RPP; ++ps) {
        const int rl = rg + ps * RPP;
        const float4 v4 = *(const float4*)&ep[rl * EPLD + 4 * c4];
        const int row = mw + i * 16 + rl;
        if (row < p.M && !(p.dbg & 1)) epilogue4(p, bz, row, nw + 4 * c4, v4, bcol);
      }
    }
    __builtin_amdgcn_wave_barrier();
  });
}


// LayerNorm backward over whole output rows in the dgrad GEMM's epilogue (GemmArgs16 lnb_*; full-row
// tiles, N == WN, the WGM waves stacked along M).  With dy = alpha * acc (fp32, never rounded),
// g = dy * gamma, xhat = (x - mean) * rstd:
//   dx = rstd * (g - mean_c(g) - xhat * mean_c(g * xhat)) [+ dres]     (norm.hip ln_bwd_vec_kernel)
// and the tile's (sum_rows dy * xhat, sum_rows dy) partial row goes to lnb_part[tile] (fixed-order
// sums: lanes, then the waves through LDS; ln_wgrad_finalize_kernel adds the rows up).  Every wave of
// the workgroup calls this (one workgroup barrier for the cross-wave sum).
template <int WM, int WN, int MI, int NI, int NW>
__device__ __forceinline__ void tile_epilogue_lnbwd(const GemmArgs16Ln& p, f32x4 (&acc)[MI][NI], char* smem, int mw,
                                                    int tile, int lane, int w) {
  constexpr int EPLD = WN + 4, CPR = WN / 8, RPP = 64 / CPR;
  float* ep = reinterpret_cast<float*>(smem) + w * 16 * EPLD;
  float* red = reinterpret_cast<float*>(smem) + NW * 16 * EPLD;  // [NW][2 WN]
  const int c8 = lane % CPR, rg = lane / CPR, col0 = 8 * c8;
  const bf16* X = (const bf16*)p.lnb_x;
  const bf16* R = (const bf16*)p.R;
  float gam[8], pg[8], pb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    gam[e] = p.ln_gamma[col0 + e];
    pg[e] = 0.f;
    pb[e] = 0.f;
  }
  const float inv_n = 1.f / WN;
  static_for<0, MI>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) ep[(4 * (lane >> 4) + r) * EPLD + j * 16 + (lane & 15)] = acc[i][j][r];
    __builtin_amdgcn_wave_barrier();
    for (int ps = 0; ps < 16 / RPP; ++ps) {
      const int rl = rg + ps * RPP;
      const int row = mw + i * 16 + rl;
      const bool live = row < p.M;
      const float4 lo = *(const float4*)&ep[rl * EPLD + col0];
      const float4 hi = *(const float4*)&ep[rl * EPLD + col0 + 4];
      const float a8[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      float xv[8], rv[8], dy[8], xh[8], g[8];
      float mu = 0.f, rs = 0.f;
      if (live) {
        ld8_bf16(X + (int64_t)row * p.lnb_ldx + col0, true, xv);
        mu = p.ln_mean[row];
        rs = p.ln_rstd[row];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) xv[e] = 0.f;
      }
      if (live && R) {
        ld8_bf16(R + (int64_t)row * p.ldr + col0, true, rv);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) rv[e] = 0.f;
      }
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dy[e] = live ? p.alpha * a8[e] : 0.f;  // rows past M hold clamped-operand garbage
        xh[e] = live ? (xv[e] - mu) * rs : 0.f;
        pg[e] += dy[e] * xh[e];
        pb[e] += dy[e];
        g[e] = dy[e] * gam[e];
        s1 += g[e];
        s2 += g[e] * xh[e];
      }
#pragma unroll
      for (int o = CPR / 2; o > 0; o >>= 1) {
        s1 += __shfl_xor(s1, o, 64);
        s2 += __shfl_xor(s2, o, 64);
      }
      s1 *= inv_n;
      s2 *= inv_n;
      if (live && !(p.dbg & 1)) {
        float o8[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o8[e] = rs * (g[e] - s1 - xh[e] * s2) + rv[e];
        st8_bf16((bf16*)p.C + (int64_t)row * p.ldc + col0, true, o8, p.dbg & 8);
      }
    }
    __builtin_amdgcn_wave_barrier();
  });
  if (p.lnb_part == nullptr) return;  // uniform: no weight gradient of the LayerNorm wanted
  // the RPP row groups of the wave (lanes with equal c8), then the NW waves through LDS
#pragma unroll
  for (int o = 32; o >= CPR; o >>= 1) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      pg[e] += __shfl_xor(pg[e], o, 64);
      pb[e] += __shfl_xor(pb[e], o, 64);
    }
  }
  if (lane < CPR) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[w * 2 * WN + col0 + e] = pg[e];
      red[w * 2 * WN + WN + col0 + e] = pb[e];
    }
  }
  __syncthreads();
  for (int c = w * 64 + lane; c < 2 * WN; c += NW * 64) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < NW; ++k) s += red[k * 2 * WN + c];
    p.lnb_part[(int64_t)tile * 2 * WN + c] = s;
  }
}

// output-vector flags of the epilogue (host side)
static void gemm_plan_vec(GemmArgs16& a, int batch) {
  // 4-column output groups: 16-B (f32) / 8-B (bf16) aligned
  a.vecC = ((uintptr_t)a.C % (a.out_f32 ? 16 : 8) == 0) && a.ldc % 4 == 0 && (batch == 1 || a.sC % 4 == 0);
  // 8-column groups with one 16-B access per operand (bf16: base 16-B aligned, strides % 8)
  auto ok8 = [&](const void* ptr, int64_t ld, int64_t sb) {
    return ptr && (uintptr_t)ptr % 16 == 0 && ld % 8 == 0 && (batch == 1 || sb % 8 == 0);
  };
  a.vec8 = (!a.out_f32 && ok8(a.C, a.ldc, a.sC) ? 1 : 0) | (ok8(a.X, a.ldx, a.sX) ? 2 : 0) |
           (ok8(a.R, a.ldr, a.sR) ? 4 : 0);
}
