// Two-way transformer, token side, forward (round 5): reference sam/transformer.py:112-187 (the
// TwoWayAttentionBlock) and :19-109 (TwoWayTransformer's final token -> image attention).
//
// Per tracked frame the mask decoder's token side is 13 objects x 8 tokens = 104 rows of width 256:
// every projection, the token self-attention (8 x 8 per object and head), the LayerNorms and the
// positional adds are launch-latency sized (a 104 x 256 x 256 GEMM is ~8 us of mostly fixed cost).
// Here one workgroup (8 waves) carries up to 16 token rows (whole objects) through a chain of them with
// the activations in LDS and the weight fragments straight from global / L2:
//   dt_self  (a block's first half):  [q = x + pe] -> q / k / v projections -> self-attention ->
//            out-projection (+ x) -> norm1 -> x1;  qt = x1 + pe -> the token -> image q projection
//   dt_post_a (after the token -> image attention): out-projection (+ x1) -> norm2 -> x2
//            [the MLP: its two GEMM launches]
//   dt_post_b norm3 -> x3;  q2 = x3 + pe -> the image -> token k / v projections [and for the last
//            block the final token -> image q projection]
//   dt_final the final out-projection (+ x3) -> norm_final
// Every intermediate the frame tape's backward reads is written to its tape slot, with the values the
// separate launches would produce up to fp32 summation order (bf16 rounding at the same points: each
// projection output, each add, each LayerNorm output; attention P rounded to bf16 for P V as in the
// attention kernels, lse = ln sum exp).  The image-side projections and both cross-attentions stay
// separate launches (frametape.py dec_* record the token ops in program order around them).
#include "common.h"

namespace {

constexpr int DT_R = 16;          // token rows per workgroup (MFMA tile height)
constexpr int DT_C = 256;         // embedding width
constexpr int DT_I = 128;         // cross-attention internal width (downsample 2)
constexpr int DT_PA = DT_C + 8;   // LDS pitch (bf16 elements) of 256-wide rows
constexpr int DT_PI = DT_I + 8;   // of 128-wide rows
constexpr int DT_PF = DT_C + 4;   // fp32 pitch
constexpr int DT_HEADS = 8;       // self-attention heads (head dim 32)
constexpr int DT_NW = 8;          // waves per workgroup
constexpr int DT_NT = DT_NW * 64;


struct DtLin { const bf16* w; const float* b; };          // weight [N][K] bf16 row-major, bias [N] fp32
struct DtNorm { const float* g; const float* b; float eps; };

struct DtSelfArgs {
  int R, T, skip;
  float scale;
  const bf16* x; const bf16* pe;
  DtLin q, k, v, o, qc;
  DtNorm n1;
  bf16* qa; bf16* qs; bf16* ks; bf16* vs; bf16* os; float* lse; bf16* y1; bf16* x1; float* mean1; float* rstd1;
  bf16* qt; bf16* qq;
};

struct DtPostArgs {
  int R, T, final_q;
  const bf16* ot; const bf16* x1; const bf16* y3; const bf16* pe;
  DtLin o, ki, vi, qf;
  DtNorm n2, n3;
  bf16* y2; bf16* x2; float* mean2; float* rstd2; bf16* x3; float* mean3; float* rstd3;
  bf16* q2; bf16* kio; bf16* vio; bf16* qfa; bf16* qqf;
};

struct DtFinalArgs {
  int R, T;
  const bf16* of; const bf16* x3;
  DtLin o;
  DtNorm n;
  bf16* y; bf16* hs; float* mean; float* rstd;
};

// the workgroup's rows: whole objects, at most 16 rows
__device__ __forceinline__ void dt_rows(int R, int T, int& r0, int& nr) {
  const int per = DT_R / T;  // objects per workgroup
  r0 = blockIdx.x * per * T;
  nr = min(per * T, R - r0);
}

// global [nr][N] bf16 (row stride N) -> LDS [16][pitch], rows >= nr zero
template <int N>
__device__ __forceinline__ void dt_load(bf16* lds, int pitch, const bf16* g, int r0, int nr) {
  constexpr int CH = N / 8;
  for (int i = threadIdx.x; i < DT_R * CH; i += blockDim.x) {
    const int r = i / CH, c = (i % CH) * 8;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r < nr) v = *(const uint4*)(g + (int64_t)(r0 + r) * N + c);
    *(uint4*)(lds + r * pitch + c) = v;
  }
}
// LDS [16][pitch] -> global [nr][N]
template <int N>
__device__ __forceinline__ void dt_store(bf16* g, const bf16* lds, int pitch, int r0, int nr) {
  constexpr int CH = N / 8;
  for (int i = threadIdx.x; i < nr * CH; i += blockDim.x) {
    const int r = i / CH, c = (i % CH) * 8;
    *(uint4*)(g + (int64_t)(r0 + r) * N + c) = *(const uint4*)(lds + r * pitch + c);
  }
}
// out = bf16(a + b) elementwise over [16][256] (the positional adds), also stored to global
__device__ __forceinline__ void dt_add(bf16* out, const bf16* a, const bf16* b, bf16* g, int r0, int nr) {
  for (int i = threadIdx.x; i < DT_R * DT_C / 8; i += blockDim.x) {
    const int r = i / (DT_C / 8), c = (i % (DT_C / 8)) * 8;
    const bf16x8 x = *(const bf16x8*)(a + r * DT_PA + c), y = *(const bf16x8*)(b + r * DT_PA + c);
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (bf16)((float)x[j] + (float)y[j]);
    *(bf16x8*)(out + r * DT_PA + c) = z;
    if (g && r < nr) *(bf16x8*)(g + (int64_t)(r0 + r) * DT_C + c) = z;
  }
}

// C[16][N] = A[16][K] W^T on the 8 waves, every weight fragment straight from global (L2).  The chip is
// idle around these launches, so what counts is round trips: the waves split N (WN groups of n-blocks)
// and, for long K, K (WK groups; their partial tiles are added in fixed order through LDS afterwards), and
// each wave loads up to 4 n-blocks x 8 k-steps of fragments (32 x 16 B per lane) before their MFMAs.
// part == nullptr (WK 1): epi(nb, acc) finishes 16 columns (lane: rows 4 (lane >> 4) + e, column nb * 16 +
// (lane & 15)).  Else the (partial) tiles go to part [WK][16][N] fp32 (may alias A: written after a
// barrier), and dt_gemm_reduce calls epi_el(row, col, sum) for every element.
template <int K, int N, int WK, typename Epi>
__device__ __forceinline__ void dt_gemm(const bf16* A, int pa, const bf16* W, float* part, Epi epi) {
  constexpr int NB = N / 16, KS = K / 32;
  constexpr int WN = DT_NW / WK;
  constexpr int NBW = (NB + WN - 1) / WN;   // n-blocks per wave
  constexpr int KSW = KS / WK;              // k-steps per wave
  constexpr int NG = NBW < 4 ? NBW : 4;
  constexpr int CH = KSW < 8 ? KSW : 8;
  static_assert(KS % WK == 0 && KSW % CH == 0, "k split");
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = w % WN, wk = w / WN;
  f32x4 keep[NBW];
#pragma unroll
  for (int gi = 0; gi < NBW; gi += NG) {
    f32x4 acc[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k0 = 0; k0 < KSW; k0 += CH) {
      bf16x8 b[NG][CH];
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const int nb = min(wn * NBW + gi + g, NB - 1);
        const bf16* wp = W + (int64_t)(nb * 16 + (lane & 15)) * K + (wk * KSW + k0) * 32 + 8 * (lane >> 4);
#pragma unroll
        for (int s = 0; s < CH; ++s) b[g][s] = *(const bf16x8*)(wp + s * 32);
      }
#pragma unroll
      for (int s = 0; s < CH; ++s) {
        const bf16x8 a = *(const bf16x8*)(A + (lane & 15) * pa + (wk * KSW + k0 + s) * 32 + 8 * (lane >> 4));
#pragma unroll
        for (int g = 0; g < NG; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[g][s], acc[g], 0, 0, 0);
      }
    }
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      const int nb = wn * NBW + gi + g;
      if (part) keep[gi + g] = acc[g];
      else if (nb < NB) epi(nb, acc[g]);
    }
  }
  if (part) {
    __syncthreads();  // every wave is done reading A (part may alias it)
#pragma unroll
    for (int g = 0; g < NBW; ++g) {
      const int nb = wn * NBW + g;
      if (nb < NB) {
#pragma unroll
        for (int e = 0; e < 4; ++e) part[(wk * DT_R + 4 * (lane >> 4) + e) * N + nb * 16 + (lane & 15)] = keep[g][e];
      }
    }
  }
}
// The weight fragments of one C[16][N] = A[16][256] W^T (dt_gemm with WK = 1: 8 waves split N, each
// wave the whole K) held apart from their MFMAs, so a later GEMM's weights can be issued a phase early
// and their memory round trip overlaps the work before it (round 6; the same MFMAs in the same order as
// dt_gemm, bit for bit).  N = 256, K = 256: 2 n-blocks x 8 k-steps per wave (64 VGPRs), N = 128: 1 x 8.
template <int N, int K = DT_C>
struct DtWFrag {
  static constexpr int NBW = N / 16 / DT_NW, KS = K / 32;
  bf16x8 b[NBW][KS];
  __device__ __forceinline__ void load(const bf16* W) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int g = 0; g < NBW; ++g) {
      const bf16* wp = W + (int64_t)((w * NBW + g) * 16 + (lane & 15)) * K + 8 * (lane >> 4);
#pragma unroll
      for (int s = 0; s < KS; ++s) b[g][s] = *(const bf16x8*)(wp + s * 32);
    }
  }
  template <typename Epi>
  __device__ __forceinline__ void mma(const bf16* A, int pa, Epi epi) const {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    f32x4 acc[NBW];
#pragma unroll
    for (int g = 0; g < NBW; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const bf16x8 a = *(const bf16x8*)(A + (lane & 15) * pa + s * 32 + 8 * (lane >> 4));
#pragma unroll
      for (int g = 0; g < NBW; ++g) acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[g][s], acc[g], 0, 0, 0);
    }
#pragma unroll
    for (int g = 0; g < NBW; ++g) epi(w * NBW + g, acc[g]);
  }
};

template <int N, int WK, typename EpiEl>
__device__ __forceinline__ void dt_gemm_reduce(const float* part, EpiEl epi_el) {
  __syncthreads();
  for (int i = threadIdx.x; i < DT_R * N; i += blockDim.x) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < WK; ++k) v += part[k * DT_R * N + i];
    epi_el(i / N, i % N, v);
  }
}

// bf16(acc + bias) -> LDS [16][pitch] (bf16)
__device__ __forceinline__ void dt_epi_bf16(bf16* out, int pitch, const float* bias, int nb, const f32x4& acc,
                                            bool relu = false) {
  const int lane = threadIdx.x & 63;
  const int col = nb * 16 + (lane & 15);
  const float b = bias ? bias[col] : 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float v = acc[e] + b;
    if (relu) v = fmaxf(v, 0.f);
    out[(4 * (lane >> 4) + e) * pitch + col] = (bf16)v;
  }
}
// fp32 of bf16(acc + bias + residual) -> LDS [16][DT_PF] (the stored projection output, LayerNorm input)
__device__ __forceinline__ void dt_epi_res(float* out, const float* bias, const bf16* res, int nb, const f32x4& acc) {
  const int lane = threadIdx.x & 63;
  const int col = nb * 16 + (lane & 15);
  const float b = bias[col];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int r = 4 * (lane >> 4) + e;
    float v = acc[e] + b;
    if (res) v += (float)res[r * DT_PA + col];
    out[r * DT_PF + col] = (float)(bf16)v;
  }
}
// y (fp32 [16][DT_PF], bf16-exact values) -> global bf16 rows
__device__ __forceinline__ void dt_store_f(bf16* g, const float* y, int r0, int nr) {
  for (int i = threadIdx.x; i < nr * DT_C / 8; i += blockDim.x) {
    const int r = i / (DT_C / 8), c = (i % (DT_C / 8)) * 8;
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (bf16)y[r * DT_PF + c + j];
    *(bf16x8*)(g + (int64_t)(r0 + r) * DT_C + c) = z;
  }
}
// LayerNorm of the 16 rows of y: 16 threads per row, 16 columns each (two-pass, as the LayerNorm kernel)
__device__ __forceinline__ void dt_layernorm(bf16* out, const float* y, DtNorm n, float* mean, float* rstd, int r0,
                                             int nr) {
  if (threadIdx.x >= DT_R * 16) return;  // 16 threads per row
  const int r = threadIdx.x >> 4, j = threadIdx.x & 15;
  float v[16];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) { v[i] = y[r * DT_PF + j + 16 * i]; s += v[i]; }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const float mu = s / DT_C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) { const float d = v[i] - mu; q += d * d; }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
  const float rs = 1.f / sqrtf(q / DT_C + n.eps);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int c = j + 16 * i;
    out[r * DT_PA + c] = (bf16)((v[i] - mu) * rs * n.g[c] + n.b[c]);
  }
  if (j == 0 && r < nr) { mean[r0 + r] = mu; rstd[r0 + r] = rs; }
}

// -------------------------------------------------------------------------------- dt_self
template <bool SCHED>
__global__ __launch_bounds__(DT_NT) void dt_self_kernel(DtSelfArgs p) {
  __shared__ __attribute__((aligned(16))) bf16 sx[DT_R * DT_PA], spe[DT_R * DT_PA], sqa[DT_R * DT_PA],
      sq[DT_R * DT_PA], sk[DT_R * DT_PA], sv[DT_R * DT_PA], so[DT_R * DT_PA], sx1[DT_R * DT_PA];
  __shared__ __attribute__((aligned(16))) float sy[DT_R * DT_PF];
  int r0, nr;
  dt_rows(p.R, p.T, r0, nr);
  // the q / k / v weights first (one round trip for all three, under the row loads); the out- and
  // q-projection weights are issued ahead of the attention and of norm1 below
  DtWFrag<DT_C> wq, wk, wv;
  if constexpr (SCHED) { wq.load(p.q.w); wk.load(p.k.w); wv.load(p.v.w); }
  dt_load<DT_C>(sx, DT_PA, p.x, r0, nr);
  dt_load<DT_C>(spe, DT_PA, p.pe, r0, nr);
  __syncthreads();
  if (!p.skip) dt_add(sqa, sx, spe, p.qa, r0, nr);
  __syncthreads();
  const bf16* qin = p.skip ? sx : sqa;
  if constexpr (SCHED) {
    wq.mma(qin, DT_PA, [&](int nb, const f32x4& a) { dt_epi_bf16(sq, DT_PA, p.q.b, nb, a); });
    wk.mma(qin, DT_PA, [&](int nb, const f32x4& a) { dt_epi_bf16(sk, DT_PA, p.k.b, nb, a); });
    wv.mma(sx, DT_PA, [&](int nb, const f32x4& a) { dt_epi_bf16(sv, DT_PA, p.v.b, nb, a); });
  } else {
    dt_gemm<DT_C, DT_C, 1>(qin, DT_PA, p.q.w, nullptr, [&](int nb, const f32x4& a) { dt_epi_bf16(sq, DT_PA, p.q.b, nb, a); });
    dt_gemm<DT_C, DT_C, 1>(qin, DT_PA, p.k.w, nullptr, [&](int nb, const f32x4& a) { dt_epi_bf16(sk, DT_PA, p.k.b, nb, a); });
    dt_gemm<DT_C, DT_C, 1>(sx, DT_PA, p.v.w, nullptr, [&](int nb, const f32x4& a) { dt_epi_bf16(sv, DT_PA, p.v.b, nb, a); });
  }
  DtWFrag<DT_C> wo;
  if constexpr (SCHED) wo.load(p.o.w);
  __syncthreads();
  dt_store<DT_C>(p.qs, sq, DT_PA, r0, nr);
  dt_store<DT_C>(p.ks, sk, DT_PA, r0, nr);
  dt_store<DT_C>(p.vs, sv, DT_PA, r0, nr);
  // self-attention: thread = (object, head, query); scores over the object's T tokens in fp32, P rounded
  // to bf16 for P V, lse = ln sum exp (the attention kernels' conventions)
  {
    const int T = p.T, nobj = nr / T;
    const float sl2 = p.scale * 1.4426950408889634f;
    for (int t = threadIdx.x; t < nobj * DT_HEADS * T; t += blockDim.x) {
      const int i = t % T, h = (t / T) % DT_HEADS, o = t / (T * DT_HEADS);
      const int r = o * T + i;
      float s[DT_R], mx = -INFINITY;
      for (int j = 0; j < T; ++j) {
        float d = 0.f;
#pragma unroll
        for (int c = 0; c < 32; c += 8) {
          const bf16x8 a = *(const bf16x8*)(sq + r * DT_PA + h * 32 + c);
          const bf16x8 b = *(const bf16x8*)(sk + (o * T + j) * DT_PA + h * 32 + c);
#pragma unroll
          for (int e = 0; e < 8; ++e) d += (float)a[e] * (float)b[e];
        }
        s[j] = d * sl2;
        mx = fmaxf(mx, s[j]);
      }
      float l = 0.f;
      for (int j = 0; j < T; ++j) {
        const float e = exp2f(s[j] - mx);
        l += e;
        s[j] = (float)(bf16)e;
      }
      const float inv = 1.f / l;
#pragma unroll
      for (int c = 0; c < 32; c += 8) {
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int j = 0; j < T; ++j) {
          const bf16x8 b = *(const bf16x8*)(sv + (o * T + j) * DT_PA + h * 32 + c);
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += s[j] * (float)b[e];
        }
        bf16x8 z;
#pragma unroll
        for (int e = 0; e < 8; ++e) z[e] = (bf16)(acc[e] * inv);
        *(bf16x8*)(so + r * DT_PA + h * 32 + c) = z;
      }
      const int ob = r0 / T + o;
      p.lse[((int64_t)ob * DT_HEADS + h) * T + i] = (mx + log2f(l)) * 0.6931471805599453f;
    }
  }
  // rows of objects past the last (nr < 16): zero attention output
  for (int i = threadIdx.x; i < (DT_R - nr) * DT_C; i += blockDim.x) so[(nr + i / DT_C) * DT_PA + i % DT_C] = (bf16)0.f;
  __syncthreads();
  dt_store<DT_C>(p.os, so, DT_PA, r0, nr);
  if constexpr (SCHED)
    wo.mma(so, DT_PA, [&](int nb, const f32x4& a) { dt_epi_res(sy, p.o.b, p.skip ? nullptr : sx, nb, a); });
  else
    dt_gemm<DT_C, DT_C, 1>(so, DT_PA, p.o.w, nullptr,
                           [&](int nb, const f32x4& a) { dt_epi_res(sy, p.o.b, p.skip ? nullptr : sx, nb, a); });
  DtWFrag<DT_I> wc;
  if constexpr (SCHED) wc.load(p.qc.w);
  __syncthreads();
  dt_store_f(p.y1, sy, r0, nr);
  dt_layernorm(sx1, sy, p.n1, p.mean1, p.rstd1, r0, nr);
  __syncthreads();
  dt_store<DT_C>(p.x1, sx1, DT_PA, r0, nr);
  dt_add(sqa, sx1, spe, p.qt, r0, nr);
  __syncthreads();
  if constexpr (SCHED)
    wc.mma(sqa, DT_PA, [&](int nb, const f32x4& a) { dt_epi_bf16(sq, DT_PI, p.qc.b, nb, a); });
  else
    dt_gemm<DT_C, DT_I, 1>(sqa, DT_PA, p.qc.w, nullptr, [&](int nb, const f32x4& a) { dt_epi_bf16(sq, DT_PI, p.qc.b, nb, a); });
  __syncthreads();
  dt_store<DT_I>(p.qq, sq, DT_PI, r0, nr);
}

// -------------------------------------------------------------------------------- dt_post
// The MLP between the two halves stays two GEMM launches: its 2 MB of weights streamed through one CU
// per workgroup took longer (a single-launch dt_post with the MLP inside: 79 us per launch) than the
// separate GEMMs, which spread them over the chip.
// dt_post_a: token -> image out-projection (+ x1) -> norm2
template <bool SCHED>
__global__ __launch_bounds__(DT_NT) void dt_post_a_kernel(DtPostArgs p) {
  __shared__ __attribute__((aligned(16))) bf16 sot[DT_R * DT_PI], sx1[DT_R * DT_PA], sx2[DT_R * DT_PA];
  __shared__ __attribute__((aligned(16))) float sy[DT_R * DT_PF];
  int r0, nr;
  dt_rows(p.R, p.T, r0, nr);
  DtWFrag<DT_C, DT_I> wo;  // under the row loads (SCHED)
  if constexpr (SCHED) wo.load(p.o.w);
  dt_load<DT_I>(sot, DT_PI, p.ot, r0, nr);
  dt_load<DT_C>(sx1, DT_PA, p.x1, r0, nr);
  __syncthreads();
  if constexpr (SCHED)
    wo.mma(sot, DT_PI, [&](int nb, const f32x4& a) { dt_epi_res(sy, p.o.b, sx1, nb, a); });
  else
    dt_gemm<DT_I, DT_C, 1>(sot, DT_PI, p.o.w, nullptr, [&](int nb, const f32x4& a) { dt_epi_res(sy, p.o.b, sx1, nb, a); });
  __syncthreads();
  dt_store_f(p.y2, sy, r0, nr);
  dt_layernorm(sx2, sy, p.n2, p.mean2, p.rstd2, r0, nr);
  __syncthreads();
  dt_store<DT_C>(p.x2, sx2, DT_PA, r0, nr);
}

// dt_post_b: norm3 of the MLP output (fc2's GEMM already added x2) -> x3; q2 = x3 + pe -> the image ->
// token k / v projections [and the final token -> image query]
template <bool SCHED>
__global__ __launch_bounds__(DT_NT) void dt_post_b_kernel(DtPostArgs p) {
  __shared__ __attribute__((aligned(16))) bf16 spe[DT_R * DT_PA], sx3[DT_R * DT_PA], sq2[DT_R * DT_PA],
      sk[DT_R * DT_PI], sv[DT_R * DT_PI];
  __shared__ __attribute__((aligned(16))) float sy[DT_R * DT_PF];
  int r0, nr;
  dt_rows(p.R, p.T, r0, nr);
  DtWFrag<DT_I> wki, wvi;  // under the row loads and norm3 (SCHED)
  if constexpr (SCHED) { wki.load(p.ki.w); wvi.load(p.vi.w); }
  dt_load<DT_C>(spe, DT_PA, p.pe, r0, nr);
  for (int i = threadIdx.x; i < DT_R * DT_C; i += blockDim.x) {
    const int r = i / DT_C, c = i % DT_C;
    sy[r * DT_PF + c] = r < nr ? (float)p.y3[(int64_t)(r0 + r) * DT_C + c] : 0.f;
  }
  __syncthreads();
  dt_layernorm(sx3, sy, p.n3, p.mean3, p.rstd3, r0, nr);
  __syncthreads();
  dt_store<DT_C>(p.x3, sx3, DT_PA, r0, nr);
  dt_add(sq2, sx3, spe, p.q2, r0, nr);
  __syncthreads();
  if constexpr (SCHED) {
    wki.mma(sq2, DT_PA, [&](int nb, const f32x4& a) { dt_epi_bf16(sk, DT_PI, p.ki.b, nb, a); });
    wvi.mma(sx3, DT_PA, [&](int nb, const f32x4& a) { dt_epi_bf16(sv, DT_PI, p.vi.b, nb, a); });
  } else {
    dt_gemm<DT_C, DT_I, 1>(sq2, DT_PA, p.ki.w, nullptr, [&](int nb, const f32x4& a) { dt_epi_bf16(sk, DT_PI, p.ki.b, nb, a); });
    dt_gemm<DT_C, DT_I, 1>(sx3, DT_PA, p.vi.w, nullptr, [&](int nb, const f32x4& a) { dt_epi_bf16(sv, DT_PI, p.vi.b, nb, a); });
  }
  __syncthreads();
  dt_store<DT_I>(p.kio, sk, DT_PI, r0, nr);
  dt_store<DT_I>(p.vio, sv, DT_PI, r0, nr);
  if (p.final_q) {  // TwoWayTransformer's final token -> image query: its own add (x3 + pe) and q projection
    dt_store<DT_C>(p.qfa, sq2, DT_PA, r0, nr);
    __syncthreads();
    dt_gemm<DT_C, DT_I, 1>(sq2, DT_PA, p.qf.w, nullptr, [&](int nb, const f32x4& a) { dt_epi_bf16(sk, DT_PI, p.qf.b, nb, a); });
    __syncthreads();
    dt_store<DT_I>(p.qqf, sk, DT_PI, r0, nr);
  }
}

// -------------------------------------------------------------------------------- dt_final
template <bool SCHED>
__global__ __launch_bounds__(DT_NT) void dt_final_kernel(DtFinalArgs p) {
  __shared__ __attribute__((aligned(16))) bf16 sof[DT_R * DT_PI], sx3[DT_R * DT_PA], shs[DT_R * DT_PA];
  __shared__ __attribute__((aligned(16))) float sy[DT_R * DT_PF];
  int r0, nr;
  dt_rows(p.R, p.T, r0, nr);
  DtWFrag<DT_C, DT_I> wo;  // under the row loads (SCHED)
  if constexpr (SCHED) wo.load(p.o.w);
  dt_load<DT_I>(sof, DT_PI, p.of, r0, nr);
  dt_load<DT_C>(sx3, DT_PA, p.x3, r0, nr);
  __syncthreads();
  if constexpr (SCHED)
    wo.mma(sof, DT_PI, [&](int nb, const f32x4& a) { dt_epi_res(sy, p.o.b, sx3, nb, a); });
  else
    dt_gemm<DT_I, DT_C, 1>(sof, DT_PI, p.o.w, nullptr, [&](int nb, const f32x4& a) { dt_epi_res(sy, p.o.b, sx3, nb, a); });
  __syncthreads();
  dt_store_f(p.y, sy, r0, nr);
  dt_layernorm(shs, sy, p.n, p.mean, p.rstd, r0, nr);
  __syncthreads();
  dt_store<DT_C>(p.hs, shs, DT_PA, r0, nr);
}

bool dt_shape_ok(int R, int T) { return R > 0 && T > 0 && T <= DT_R && R % T == 0; }
int dt_blocks(int R, int T) {
  const int per = DT_R / T;
  return (R / T + per - 1) / per;
}
DtLin lin(const void* w, const float* b) { return DtLin{(const bf16*)w, b}; }
int g_dt_sched = 1;  // the dt_* kernels <true>: weights issued a phase ahead (s2h_dec_sched A/B knob)

}  // namespace

// Token side of a TwoWayAttentionBlock's first half (transformer.py:150-170), bf16, R = objects x T rows
// of width 256 (T <= 16 tokens per object; 8 heads of 32; cross-attention width 128):
//   qa = x + pe (skip == 0)                     q/k/v = (skip ? x : qa | skip ? x : qa | x) W^T + b
//   os = softmax(scale q k^T per object, head) v     (lse [objects, 8, T], natural log)
//   y1 = os Wo^T + bo (+ x if !skip)    x1 = norm1(y1) (mean1 / rstd1)    qt = x1 + pe    qq = qt Wqc^T + bqc
// Weights [N, K] bf16, biases fp32; outputs at the given slots (row-major, contiguous).
// A/B knob (round 6): 1 (default) the token-side kernels with their weight fragments issued a phase ahead
// (DtWFrag), 0 each projection loading its own before its MFMAs.  Returns the previous setting
// (mode < 0: query only).
extern "C" int s2h_dec_sched(int mode) {
  const int prev = g_dt_sched;
  if (mode >= 0) g_dt_sched = mode;
  return prev;
}
extern "C" int s2h_dec_self(int R, int T, int skip, float scale, const void* x, const void* pe, const void* wq,
                            const float* bq, const void* wk, const float* bk, const void* wv, const float* bv,
                            const void* wo, const float* bo, const float* g1, const float* b1, float eps1,
                            const void* wqc, const float* bqc, void* qa, void* qs, void* ks, void* vs, void* os,
                            float* lse, void* y1, void* x1, float* mean1, float* rstd1, void* qt, void* qq,
                            hipStream_t st) {
  if (!dt_shape_ok(R, T)) return (int)hipErrorInvalidValue;
  DtSelfArgs p;
  p.R = R; p.T = T; p.skip = skip; p.scale = scale;
  p.x = (const bf16*)x; p.pe = (const bf16*)pe;
  p.q = lin(wq, bq); p.k = lin(wk, bk); p.v = lin(wv, bv); p.o = lin(wo, bo); p.qc = lin(wqc, bqc);
  p.n1 = DtNorm{g1, b1, eps1};
  p.qa = (bf16*)qa; p.qs = (bf16*)qs; p.ks = (bf16*)ks; p.vs = (bf16*)vs; p.os = (bf16*)os; p.lse = lse;
  p.y1 = (bf16*)y1; p.x1 = (bf16*)x1; p.mean1 = mean1; p.rstd1 = rstd1; p.qt = (bf16*)qt; p.qq = (bf16*)qq;
  if (g_dt_sched)
    hipLaunchKernelGGL(dt_self_kernel<true>, dim3(dt_blocks(R, T)), dim3(DT_NT), 0, st, p);
  else
    hipLaunchKernelGGL(dt_self_kernel<false>, dim3(dt_blocks(R, T)), dim3(DT_NT), 0, st, p);
  return (int)hipGetLastError();
}

// Its second half's token side around the MLP GEMMs (transformer.py:170-173):
//   s2h_dec_post_a: y2 = ot Wo^T + bo + x1, x2 = norm2(y2)
//   s2h_dec_post_b: x3 = norm3(y3) (y3 = the MLP output + x2), q2 = x3 + pe, kio = q2 Wki^T + bki,
//     vio = x3 Wvi^T + bvi (the image -> token keys / values); final_q: qfa = x3 + pe, qqf = qfa Wqf^T + bqf
//     (TwoWayTransformer's final token -> image query, :194-196)
extern "C" int s2h_dec_post_a(int R, int T, const void* ot, const void* x1, const void* wo, const float* bo,
                              const float* g2, const float* b2n, float eps2, void* y2, void* x2, float* mean2,
                              float* rstd2, hipStream_t st) {
  if (!dt_shape_ok(R, T)) return (int)hipErrorInvalidValue;
  DtPostArgs p = {};
  p.R = R; p.T = T;
  p.ot = (const bf16*)ot; p.x1 = (const bf16*)x1;
  p.o = lin(wo, bo);
  p.n2 = DtNorm{g2, b2n, eps2};
  p.y2 = (bf16*)y2; p.x2 = (bf16*)x2; p.mean2 = mean2; p.rstd2 = rstd2;
  if (g_dt_sched)
    hipLaunchKernelGGL(dt_post_a_kernel<true>, dim3(dt_blocks(R, T)), dim3(DT_NT), 0, st, p);
  else
    hipLaunchKernelGGL(dt_post_a_kernel<false>, dim3(dt_blocks(R, T)), dim3(DT_NT), 0, st, p);
  return (int)hipGetLastError();
}

extern "C" int s2h_dec_post_b(int R, int T, int final_q, const void* y3, const void* pe, const float* g3,
                              const float* b3n, float eps3, const void* wki, const float* bki, const void* wvi,
                              const float* bvi, const void* wqf, const float* bqf, void* x3, float* mean3,
                              float* rstd3, void* q2, void* kio, void* vio, void* qfa, void* qqf, hipStream_t st) {
  if (!dt_shape_ok(R, T) || (final_q && (!qfa || !qqf || !wqf))) return (int)hipErrorInvalidValue;
  DtPostArgs p = {};
  p.R = R; p.T = T; p.final_q = final_q;
  p.y3 = (const bf16*)y3; p.pe = (const bf16*)pe;
  p.ki = lin(wki, bki); p.vi = lin(wvi, bvi); p.qf = lin(wqf, bqf);
  p.n3 = DtNorm{g3, b3n, eps3};
  p.x3 = (bf16*)x3; p.mean3 = mean3; p.rstd3 = rstd3; p.q2 = (bf16*)q2; p.kio = (bf16*)kio; p.vio = (bf16*)vio;
  p.qfa = (bf16*)qfa; p.qqf = (bf16*)qqf;
  if (g_dt_sched)
    hipLaunchKernelGGL(dt_post_b_kernel<true>, dim3(dt_blocks(R, T)), dim3(DT_NT), 0, st, p);
  else
    hipLaunchKernelGGL(dt_post_b_kernel<false>, dim3(dt_blocks(R, T)), dim3(DT_NT), 0, st, p);
  return (int)hipGetLastError();
}

// TwoWayTransformer's final token side (transformer.py:196-197): y = of Wo^T + bo + x3, hs = norm(y)
extern "C" int s2h_dec_final(int R, int T, const void* of, const void* x3, const void* wo, const float* bo,
                             const float* g, const float* bn, float eps, void* y, void* hs, float* mean, float* rstd,
                             hipStream_t st) {
  if (!dt_shape_ok(R, T)) return (int)hipErrorInvalidValue;
  DtFinalArgs p;
  p.R = R; p.T = T;
  p.of = (const bf16*)of; p.x3 = (const bf16*)x3;
  p.o = lin(wo, bo);
  p.n = DtNorm{g, bn, eps};
  p.y = (bf16*)y; p.hs = (bf16*)hs; p.mean = mean; p.rstd = rstd;
  if (g_dt_sched)
    hipLaunchKernelGGL(dt_final_kernel<true>, dim3(dt_blocks(R, T)), dim3(DT_NT), 0, st, p);
  else
    hipLaunchKernelGGL(dt_final_kernel<false>, dim3(dt_blocks(R, T)), dim3(DT_NT), 0, st, p);
  return (int)hipGetLastError();
}
