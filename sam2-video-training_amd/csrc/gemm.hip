// MFMA-tiled GEMM with fused epilogue for every projection / MLP / 1x1-conv /
// im2col-conv / hypernetwork product on the SAM2 training step.
//
//   C[b](m,n) = act(alpha * sum_k A[b](m,k) B[b](k,n) + bias) + R[b](m,n) + beta*C[b](m,n)
//
// A and B are addressed through (row, k) strides so the three products of a
// Linear layer (fwd Y = X W^T, dgrad dX = dY W, wgrad dW = dY^T X) all run
// without transposed copies: each operand is either K-contiguous ("KC") or
// M/N-contiguous, selected at compile time.  Tiles are staged through LDS in a
// K-contiguous [row][k] image so both MFMA operands read 16-B fragments.
#include "gemm_bf16.h"

struct GemmArgs {
  int M, N, K;
  const void* A; int64_t lda_m, lda_k, sA;
  const void* B; int64_t ldb_k, ldb_n, sB;
  void* C; int64_t ldc, sC;
  const float* bias; int bias_mode;  // 0 none, 1 per column n, 2 per row m
  const void* R; int64_t ldr, sR;
  void* X; int64_t ldx, sX;  // aux: aux_mode 1 stores pre-activation, 2 multiplies by act'(X)
  int aux_mode;
  const float* cscale;        // optional per-column scale applied after the activation
  float drop_p; uint64_t seed; const uint64_t* seed_off; // optional dropout after the activation (index = row*N + col)
  uint64_t drop_idx0;  // dropout element-index offset (frame slot of a frame-stacked activation)
  float alpha, beta; int act;
  int vecA, vecB;
};

template <typename T, int ROWS, int BK, bool KC, int NTHR>
struct TileLoader {
  // Loads a ROWS x BK tile (row = m or n, k) into registers, then LDS [row][k].
  static constexpr int VEC = 16 / sizeof(T);
  static constexpr int NV = ROWS * BK / VEC / NTHR;
  static_assert(NV >= 1, "tile too small for thread count");
  uint4 r[NV];

  __device__ __forceinline__ void load(const T* base, int64_t ld_row, int64_t ld_k, int row0, int k0,
                                       int nrows, int K, bool vec_ok, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int v = tid + i * NTHR;
      int row, k;
      if (KC) { row = v / (BK / VEC); k = (v % (BK / VEC)) * VEC; }
      else    { k = v / (ROWS / VEC); row = (v % (ROWS / VEC)) * VEC; }
      int gr = row0 + row, gk = k0 + k;
      bool full = KC ? (gr < nrows && gk + VEC <= K) : (gk < K && gr + VEC <= nrows);
      if (full && vec_ok) {
        const T* ptr = base + (int64_t)gr * ld_row + (int64_t)gk * ld_k;
        r[i] = *(const uint4*)ptr;
      } else {
        T tmp[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          int rr = KC ? gr : gr + j;
          int kk = KC ? gk + j : gk;
          tmp[j] = (rr < nrows && kk < K) ? base[(int64_t)rr * ld_row + (int64_t)kk * ld_k] : from_f32<T>(0.f);
        }
        r[i] = *(uint4*)tmp;
      }
    }
  }
  __device__ __forceinline__ void store(T* lds, int lds_stride, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      int v = tid + i * NTHR;
      if (KC) {
        int row = v / (BK / VEC), k = (v % (BK / VEC)) * VEC;
        *(uint4*)(lds + row * lds_stride + k) = r[i];
      } else {
        int k = v / (ROWS / VEC), row = (v % (ROWS / VEC)) * VEC;
        const T* t = (const T*)&r[i];
#pragma unroll
        for (int j = 0; j < VEC; ++j) lds[(row + j) * lds_stride + k] = t[j];
      }
    }
  }
};

template <typename T, typename TC, int BM, int BN, bool AKC, bool BKC>
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs p) {
  if (p.drop_p > 0.f) p.seed = s2h_seed(p.seed, p.seed_off);
  constexpr int BK = 32;
  constexpr int VEC = 16 / sizeof(T);
  constexpr int LS = BK + VEC;  // LDS row stride (elements): +16 B pad
  constexpr int WM = BM / 2, WN = BN / 2, MI = WM / 16, NI = WN / 16;
  using MF = Mfma<T>;
  __shared__ __attribute__((aligned(16))) T As[BM * LS];
  __shared__ __attribute__((aligned(16))) T Bs[BN * LS];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int bz = blockIdx.z;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const T* A = (const T*)p.A + (int64_t)bz * p.sA;
  const T* B = (const T*)p.B + (int64_t)bz * p.sB;

  TileLoader<T, BM, BK, AKC, 256> la;
  TileLoader<T, BN, BK, BKC, 256> lb;
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  la.load(A, p.lda_m, p.lda_k, m0, 0, p.M, p.K, p.vecA, tid);
  lb.load(B, p.ldb_n, p.ldb_k, n0, 0, p.N, p.K, p.vecB, tid);
  for (int kt = 0; kt < nk; ++kt) {
    la.store(As, LS, tid);
    lb.store(Bs, LS, tid);
    __syncthreads();
    if (kt + 1 < nk) {
      la.load(A, p.lda_m, p.lda_k, m0, (kt + 1) * BK, p.M, p.K, p.vecA, tid);
      lb.load(B, p.ldb_n, p.ldb_k, n0, (kt + 1) * BK, p.N, p.K, p.vecB, tid);
    }
#pragma unroll
    for (int ks = 0; ks < BK; ks += MF::KSTEP) {
      typename MF::frag a[MI], b[NI];
      const int kof = ks + (lane >> 4) * MF::KPL;
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = MF::load(&As[(wm * WM + i * 16 + (lane & 15)) * LS + kof]);
#pragma unroll
      for (int j = 0; j < NI; ++j) b[j] = MF::load(&Bs[(wn * WN + j * 16 + (lane & 15)) * LS + kof]);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = MF::mma(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }

  TC* C = (TC*)p.C + (int64_t)bz * p.sC;
  const TC* R = p.R ? (const TC*)p.R + (int64_t)bz * p.sR : nullptr;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      int col = n0 + wn * WN + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int row = m0 + wm * WM + i * 16 + (lane >> 4) * 4 + r;
        if (row < p.M && col < p.N) {
          float v = p.alpha * acc[i][j][r];
          if (p.bias_mode == 1) v += p.bias[col];
          else if (p.bias_mode == 2) v += p.bias[row];
          if (p.aux_mode == 1) ((TC*)p.X)[(int64_t)bz * p.sX + (int64_t)row * p.ldx + col] = from_f32<TC>(v);
          if (p.aux_mode == 2) v *= act_grad(to_f32(((const TC*)p.X)[(int64_t)bz * p.sX + (int64_t)row * p.ldx + col]), p.act);
          else v = apply_act(v, p.act);
          if (p.cscale) v *= p.cscale[col];
          if (p.drop_p > 0.f) {
            const uint64_t idx = p.drop_idx0 + (uint64_t)bz * p.M * p.N + (uint64_t)row * p.N + col;
            v = s2h_keep(p.seed, idx, (uint32_t)(p.drop_p * 4294967296.0)) ? v / (1.f - p.drop_p) : 0.f;
          }
          if (R) v += to_f32(R[(int64_t)row * p.ldr + col]);
          int64_t off = (int64_t)row * p.ldc + col;
          if (p.beta != 0.f) v += p.beta * to_f32(C[off]);
          C[off] = from_f32<TC>(v);
        }
      }
    }
}

template <typename T, typename TC, int BM, int BN>
static int launch_gemm_tiles(const GemmArgs& a, int batch, hipStream_t st) {
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, batch);
  bool akc = a.lda_k == 1, bkc = a.ldb_k == 1;
  if (akc && bkc) hipLaunchKernelGGL((gemm_kernel<T, TC, BM, BN, true, true>), grid, dim3(256), 0, st, a);
  else if (akc && !bkc) hipLaunchKernelGGL((gemm_kernel<T, TC, BM, BN, true, false>), grid, dim3(256), 0, st, a);
  else if (!akc && bkc) hipLaunchKernelGGL((gemm_kernel<T, TC, BM, BN, false, true>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((gemm_kernel<T, TC, BM, BN, false, false>), grid, dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

static int g_gemm32_small = 1;  // A/B knob (s2h_gemm_f32_small): fp32 GEMMs of < 64 tiles on 32 x 32 tiles
extern "C" int s2h_gemm_f32_small(int mode) {
  const int prev = g_gemm32_small;
  if (mode >= 0) g_gemm32_small = mode;
  return prev;
}

template <typename T, typename TC>
static int launch_gemm(const GemmArgs& a, int batch, hipStream_t st) {
  // Small problems: 64x64 tiles keep enough workgroups in flight on 256 CUs.
  long tiles128 = (long)((a.M + 127) / 128) * ((a.N + 127) / 128) * batch;
  if (tiles128 >= 512) return launch_gemm_tiles<T, TC, 128, 128>(a, batch, st);
  // fp32 problems of fewer than 64 tiles of 64^2 (the V-fold weight gradients dWo += G V^T, 256 x 256 x 72,
  // and dV = Wo^T G, 256 x 72 x 256, once per layer and step): 32 x 32 tiles, 4x the workgroups
  if constexpr (sizeof(T) == 4) {
    const long tiles64 = (long)((a.M + 63) / 64) * ((a.N + 63) / 64) * batch;
    if (g_gemm32_small && tiles64 < 64) return launch_gemm_tiles<T, TC, 32, 32>(a, batch, st);
  }
  return launch_gemm_tiles<T, TC, 64, 64>(a, batch, st);
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

extern "C" int s2h_gemm(int dt_ab, int dt_c, int batch, int M, int N, int K,
                        const void* A, int64_t lda_m, int64_t lda_k, int64_t sA,
                        const void* B, int64_t ldb_k, int64_t ldb_n, int64_t sB,
                        void* C, int64_t ldc, int64_t sC,
                        const float* bias, int bias_mode,
                        const void* R, int64_t ldr, int64_t sR,
                        void* X, int64_t ldx, int64_t sX, int aux_mode,
                        const float* cscale, float drop_p, uint64_t seed, uint64_t drop_idx0,
                        float alpha, float beta, int act, hipStream_t stream) {
  if (M <= 0 || N <= 0 || batch <= 0) return 0;
  if (!(lda_k == 1 || lda_m == 1) || !(ldb_k == 1 || ldb_n == 1)) return (int)hipErrorInvalidValue;
  if (dt_ab == S2H_F32 && dt_c != S2H_F32) return (int)hipErrorInvalidValue;
  GemmArgs a;
  a.M = M; a.N = N; a.K = K;
  a.A = A; a.lda_m = lda_m; a.lda_k = lda_k; a.sA = sA;
  a.B = B; a.ldb_k = ldb_k; a.ldb_n = ldb_n; a.sB = sB;
  a.C = C; a.ldc = ldc; a.sC = sC;
  a.bias = bias; a.bias_mode = bias ? bias_mode : 0;
  a.R = R; a.ldr = ldr; a.sR = sR;
  a.X = X; a.ldx = ldx; a.sX = sX; a.aux_mode = X ? aux_mode : 0;
  a.cscale = cscale; a.drop_p = drop_p; a.seed = seed; a.seed_off = s2h_rng_offset_ptr();
  a.drop_idx0 = drop_idx0;
  a.alpha = alpha; a.beta = beta; a.act = act;
  const int esz = dt_ab == S2H_BF16 ? 2 : 4;
  const int vec = 16 / esz;
  // vector loads need a 16-B aligned base, and every row start 16-B aligned
  int64_t lda_row = (lda_k == 1) ? lda_m : lda_k;
  int64_t ldb_row = (ldb_k == 1) ? ldb_n : ldb_k;
  a.vecA = aligned16(A) && (lda_row % vec == 0) && (batch == 1 || sA % vec == 0);
  a.vecB = aligned16(B) && (ldb_row % vec == 0) && (batch == 1 || sB % vec == 0);
  if (K <= 0) {
    a.K = 0;
  }
  // profiler record: (batch, M, N, K, layout = 2*A_kcontig + B_kcontig + 4*bf16)
  const int slot = s2h_prof_begin(stream, 4, batch, M, N, K, 2 * (lda_k == 1) + (ldb_k == 1) + 4 * (dt_ab == S2H_BF16));
  int rc;
  if (dt_ab == S2H_F32) {
    rc = launch_gemm<float, float>(a, batch, stream);
    s2h_prof_end(slot, stream);
    return rc;
  }
  GemmArgs16 b = {};
  b.M = a.M; b.N = a.N; b.K = a.K;
  b.A = (const bf16*)A; b.lda_m = lda_m; b.lda_k = lda_k; b.sA = sA;
  b.B = (const bf16*)B; b.ldb_k = ldb_k; b.ldb_n = ldb_n; b.sB = sB;
  b.C = C; b.ldc = ldc; b.sC = sC;
  b.bias = a.bias; b.bias_mode = a.bias_mode;
  b.R = R; b.ldr = ldr; b.sR = sR;
  b.X = X; b.ldx = ldx; b.sX = sX; b.aux_mode = a.aux_mode;
  b.cscale = cscale; b.drop_p = drop_p; b.seed = seed; b.seed_off = s2h_rng_offset_ptr();
  b.drop_idx0 = drop_idx0;
  b.alpha = alpha; b.beta = beta; b.act = act;
  b.vecA = a.vecA; b.vecB = a.vecB;
  b.out_f32 = dt_c == S2H_F32;
  b.rowsum = nullptr;
  rc = s2h_gemm_bf16(b, batch, stream);
  s2h_prof_end(slot, stream);
  return rc;
}

// Linear + axial RoPE of its output in one launch (bf16): Y[b] = A[b] W^T + bias, then rows
// r < nrot of every block of L rows rotated in (2i, 2i+1) pairs of the columns c < ncol with table
// row (r % period) and column (c % dh) / 2 -- the memory attention's q / k projections followed by
// apply_rotary_enc (transformer.py:275-311), and the fused q/k/v projection with q and k rotated.
extern "C" int s2h_linear_rope(int M, int N, int K, const void* A, int64_t lda, const void* W, int64_t ldw,
                               const float* bias, void* Y, int64_t ldy, const float* cosv, const float* sinv, int L,
                               int nrot, int period, int ncol, int dh, hipStream_t stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || L <= 0 || period <= 0 || dh <= 0 || dh % 8 || ncol % 8 || nrot < 0 || nrot > L || !cosv || !sinv)
    return (int)hipErrorInvalidValue;
  const int slot = s2h_prof_begin(stream, 4, 1, M, N, K, 2 + 1 + 4);
  GemmArgs16 b = {};
  b.M = M; b.N = N; b.K = K;
  b.A = (const bf16*)A; b.lda_m = lda; b.lda_k = 1;
  b.B = (const bf16*)W; b.ldb_k = 1; b.ldb_n = ldw;
  b.C = Y; b.ldc = ldy;
  b.bias = bias; b.bias_mode = bias ? 1 : 0;
  b.seed_off = s2h_rng_offset_ptr();
  b.alpha = 1.f;
  b.vecA = aligned16(A) && lda % 8 == 0;
  b.vecB = aligned16(W) && ldw % 8 == 0;
  b.rope_cos = cosv; b.rope_sin = sinv;
  b.rope_L = L; b.rope_nrot = nrot; b.rope_period = period; b.rope_ncol = ncol; b.rope_dh = dh;
  const int rc = s2h_gemm_bf16(b, 1, stream);
  s2h_prof_end(slot, stream);
  return rc;
}

// Projection + dropout + residual + LayerNorm in one launch (bf16; round 4):
//   X' = R + drop(A W^T + bias)   (C, the residual stream)      Y = LN(X') * gamma + beta
// with mean / rstd per row -- a Linear followed by the residual add + LayerNorm that reads it
// (memory_attention.py:60-98 out_proj / cross-attention output / linear2 -> norm2 / norm3 / the
// next layer's norm1).  Full-row tiles (64 rows x N, N = 128 or 256, gemm_cfg6.hip).
extern "C" int s2h_linear_add_ln(int M, int N, int K, const void* A, int64_t lda, const void* W, int64_t ldw,
                                 const float* bias, const void* R, int64_t ldr, float drop_p, uint64_t seed,
                                 uint64_t drop_idx0, void* C, int64_t ldc, const float* gamma, const float* beta,
                                 float eps, void* Y, int64_t ldy, float* mean, float* rstd, hipStream_t stream) {
  if (M <= 0) return 0;
  if ((N != 256 && N != 128) || K <= 0 || !A || !W || !C || !Y || !gamma || !beta || !mean || !rstd ||
      !aligned16(A) || !aligned16(W) || !aligned16(C) || !aligned16(Y) || (R && !aligned16(R)) || lda % 8 ||
      ldw % 8 || ldc % 8 || ldy % 8 || (R && ldr % 8) || K % 8 || (int64_t)M * lda >= (1ll << 31) ||
      (int64_t)N * ldw >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  const int slot = s2h_prof_begin(stream, 4, 1, M, N, K, 2 + 1 + 4);
  GemmArgs16Ln b = {};
  b.M = M; b.N = N; b.K = K;
  b.A = (const bf16*)A; b.lda_m = lda; b.lda_k = 1;
  b.B = (const bf16*)W; b.ldb_k = 1; b.ldb_n = ldw;
  b.C = C; b.ldc = ldc;
  b.bias = bias; b.bias_mode = bias ? 1 : 0;
  b.R = R; b.ldr = ldr;
  b.drop_p = drop_p; b.seed = seed; b.seed_off = s2h_rng_offset_ptr(); b.drop_idx0 = drop_idx0;
  b.alpha = 1.f;
  b.vecA = 1; b.vecB = 1;
  b.ln_gamma = gamma; b.ln_beta = beta; b.ln_eps = eps; b.ln_y = Y; b.ln_ldy = ldy; b.ln_mean = mean; b.ln_rstd = rstd;
  const int cfg = N == 128 ? CFG_64x128_W41_NS4 : (K <= 256 ? CFG_64x256_W41_NS4 : CFG_64x256_W41_NS3);
  const int rc = gemm_cfg_launch_6_ln(cfg, b, 1, stream);
  s2h_prof_end(slot, stream);
  return rc;
}

// Input gradient of a Linear whose input is a LayerNorm output it alone reads, with the LayerNorm
// backward in the GEMM epilogue (bf16; round 4):
//   dy = alpha * G W        (G [M, K] the Linear's output gradient, W [K, N] its weight)
//   dx = LN_bwd(dy; X, gamma, mean, rstd) + dres                         (C [M, N], bf16)
//   dgamma += sum_rows dy * xhat, dbeta += sum_rows dy                   (when dgamma != null)
// -- memory_attention.py:60-98 norm1 -> q/k/v, norm2 -> cross-attention q, norm3 -> linear1 in the
// backward: the LayerNorm output's gradient stays in registers (never stored as bf16 and re-read).
// `part` holds ceil(M / 64) * 2N floats (s2h_linear_dgrad_ln_bwd_ws_bytes).  Full-row tiles.
extern "C" int s2h_ln_wgrad_finalize(int nb, int C, const float* part, float* dgamma, float* dbeta, hipStream_t st);
extern "C" int64_t s2h_linear_dgrad_ln_bwd_ws_bytes(int M, int N) {
  return M <= 0 ? 0 : (int64_t)((M + 63) / 64) * 2 * N * sizeof(float);
}
extern "C" int s2h_linear_dgrad_ln_bwd(int M, int N, int K, const void* G, int64_t ldg, const void* W, int64_t ldw,
                                       float alpha, const void* X, int64_t ldx, const float* gamma, const float* mean,
                                       const float* rstd, const void* dres, int64_t ldr, void* dx, int64_t lddx,
                                       float* part, float* dgamma, float* dbeta, hipStream_t stream) {
  if (M <= 0) return 0;
  if ((N != 256 && N != 128) || K <= 0 || !G || !W || !X || !dx || !gamma || !mean || !rstd ||
      ((dgamma == nullptr) != (dbeta == nullptr)) || (dgamma && !part) || !aligned16(G) || !aligned16(W) ||
      !aligned16(X) || !aligned16(dx) || (dres && !aligned16(dres)) || ldg % 8 || ldw % 8 || ldx % 8 || lddx % 8 ||
      (dres && ldr % 8) || K % 8 || (int64_t)M * ldg >= (1ll << 31) || (int64_t)K * ldw >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  const int slot = s2h_prof_begin(stream, 4, 1, M, N, K, 2 + 0 + 4);
  GemmArgs16Ln b = {};
  b.M = M; b.N = N; b.K = K;
  b.A = (const bf16*)G; b.lda_m = ldg; b.lda_k = 1;
  b.B = (const bf16*)W; b.ldb_k = ldw; b.ldb_n = 1;
  b.C = dx; b.ldc = lddx;
  b.R = dres; b.ldr = ldr;
  b.seed_off = s2h_rng_offset_ptr();
  b.alpha = alpha;
  b.vecA = 1; b.vecB = 1;
  b.ln_gamma = gamma; b.ln_mean = const_cast<float*>(mean); b.ln_rstd = const_cast<float*>(rstd);
  b.lnb_x = X; b.lnb_ldx = ldx; b.lnb_part = dgamma ? part : nullptr;
  const int cfg = N == 128 ? CFG_64x128_W41_NS4 : (K <= 256 ? CFG_64x256_W41_NS4 : CFG_64x256_W41_NS3);
  int rc = gemm_cfg_launch_6_ln(cfg, b, 1, stream);
  s2h_prof_end(slot, stream);
  if (rc || !dgamma) return rc;
  return s2h_ln_wgrad_finalize((M + 63) / 64, N, part, dgamma, dbeta, stream);
}

extern "C" int s2h_colsum(int dt, int64_t rows, int cols, const void* x, int64_t ld, float* out, int accum,
                          hipStream_t st);

// Weight (and bias) gradient of a Linear layer y = x W^T + b over `rows` rows:
//   dw[N, K] (+)= dy[rows, N]^T x[rows, K]      db[N] (+)= sum_rows dy
// bf16: one GEMM launch (split over the row reduction when the N x K tiles cannot fill the
// chip) with the bias gradient summed from the staged dy tiles; fp32: GEMM + column sum.
extern "C" int s2h_linear_wgrad(int dt, int64_t rows, int N, int K, const void* dy, int64_t lddy, const void* x,
                                int64_t ldx, float* dw, int64_t lddw, float* db, int accumulate, hipStream_t stream) {
  if (N <= 0 || K <= 0) return 0;
  if (rows > INT32_MAX) return (int)hipErrorInvalidValue;
  if (!accumulate && db) s2h_zero_f32(db, 1, N, N, stream);
  if (dt == S2H_F32) {
    int rc = s2h_gemm(S2H_F32, S2H_F32, 1, N, K, (int)rows, dy, 1, lddy, 0, x, ldx, 1, 0, dw, lddw, 0, nullptr, 0,
                      nullptr, 0, 0, nullptr, 0, 0, 0, nullptr, 0.f, 0, 0, 1.f, accumulate ? 1.f : 0.f, 0, stream);
    if (rc || !db) return rc;
    return s2h_colsum(dt, rows, N, dy, lddy, db, 1, stream);
  }
  const int slot = s2h_prof_begin(stream, 4, 1, N, K, rows, 4);
  GemmArgs16 b = {};
  b.M = N; b.N = K; b.K = (int)rows;
  b.A = (const bf16*)dy; b.lda_m = 1; b.lda_k = lddy; b.sA = 0;
  b.B = (const bf16*)x; b.ldb_k = ldx; b.ldb_n = 1; b.sB = 0;
  b.C = dw; b.ldc = lddw; b.sC = 0;
  b.alpha = 1.f; b.beta = accumulate ? 1.f : 0.f;
  b.vecA = aligned16(dy) && lddy % 8 == 0;
  b.vecB = aligned16(x) && ldx % 8 == 0;
  b.out_f32 = 1;
  b.rowsum = db;
  const int rc = s2h_gemm_bf16(b, 1, stream);
  s2h_prof_end(slot, stream);
  return rc;
}
