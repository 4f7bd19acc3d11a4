// Argument block of the bf16 MFMA GEMM (gemm_bf16.hip), shared with the C-ABI entry in gemm.hip.
#pragma once
#include "common.h"

struct GemmArgs16 {
  int M, N, K;
  const bf16* A; int64_t lda_m, lda_k, sA;
  const bf16* B; int64_t ldb_k, ldb_n, sB;
  void* C; int64_t ldc, sC;
  const float* bias; int bias_mode;
  const void* R; int64_t ldr, sR;
  void* X; int64_t ldx, sX;
  int aux_mode;
  const float* cscale;
  float drop_p; uint64_t seed; const uint64_t* seed_off; uint64_t drop_idx0;
  float alpha, beta; int act;
  int vecA, vecB;
  // split-K: blockIdx.z = batch * splits + split.  With the deterministic-reduction workspace registered
  // (s2h_det_ws) a split launch stores its partial tiles there instead of adding them into C with float
  // atomics, and gemm_split_reduce_kernel adds them in split order: X then points at the partials
  // (unused otherwise -- a split GEMM has no epilogue operands), sX is one split's stride
  // (batch x M x N floats, rows of N), the rowsum partials follow at splits x sX
  int splits, kchunk;
  int out_f32;
  int vecC;  // 4-column output groups are vector-aligned
  int vec8;  // 8-column groups take 16-B accesses: bit 0 C (bf16 out), bit 1 X, bit 2 R
  float* rowsum;  // optional: rowsum[b*M + m] += sum_k A[b](m, k)  (fused bias gradient)
  // optional axial RoPE of the output (memory-attention q / k projections, transformer.py:275-311):
  // row r (within batch bz) is rotated when (r % rope_L) < rope_nrot, with table row
  // (r % rope_L) % rope_period; columns c < rope_ncol are rotated in pairs (2i, 2i+1) with the
  // tables' column (c % rope_dh) / 2.  rope_cos == nullptr: no rotation.
  const float* rope_cos; const float* rope_sin;
  int rope_L, rope_nrot, rope_period, rope_ncol, rope_dh;
  int dbg;       // measurement-only ablations (s2h_gemm_config bits 8+): 1 skip epilogue stores, 2 skip MFMAs, 4 skip operand DMA, 8 plain stores, 16 tile-major split-K order, 32 split-K by float atomics, 64 per-piece DMA address arithmetic (gemm16g_kernel)
};

// The LayerNorm epilogues' extra arguments (round 4), in a derived block that only the full-row tilings
// (gemm_cfg6.hip) take, so the plain GEMM kernels compile exactly as before: with 88 more bytes in
// every GEMM's block the bench step lost 0.35 ms (in-call A/B of the round-4 checkpoint with its block
// padded by 88 bytes: 56.57 -> 56.95 ms).  Not the bytes themselves -- a graph of 1000 launches costs
// 1.53-1.54 us per launch for any block from 64 B to 2 KB (tools/kernarg_probe.hip) -- but the code
// generated around them
struct GemmArgs16Ln : GemmArgs16 {
  // optional LayerNorm of the finished output rows (s2h_linear_add_ln): the tile spans the whole
  // output width (N <= 256, one wave per 16 full rows); C receives x' = R + drop(A W^T + b) (bf16, the
  // residual stream), ln_y = LN(x') with gamma / beta / eps, ln_mean / ln_rstd per row -- the
  // residual add + LayerNorm that follows a projection (memory_attention.py:60-98), fused
  const float* ln_gamma; const float* ln_beta; float ln_eps;
  void* ln_y; int64_t ln_ldy; float* ln_mean; float* ln_rstd;
  // optional LayerNorm BACKWARD of the finished rows (s2h_linear_dgrad_ln_bwd): the GEMM is the dgrad of
  // the LayerNorm output's only consumer, alpha * acc = dL/dy over whole rows; lnb_x is the LayerNorm
  // input (bf16), ln_gamma / ln_mean / ln_rstd its saved parameters and statistics, R the
  // residual-stream gradient added to dx (may be null); C receives dx; lnb_part (may be null) one
  // (sum dy * xhat, sum dy) row of 2N floats per 64-row tile for ln_wgrad_finalize_kernel
  const void* lnb_x; int64_t lnb_ldx; float* lnb_part;
};

int s2h_gemm_bf16(const GemmArgs16& a, int batch, hipStream_t st);
int s2h_prof_begin(hipStream_t st, int kind, int64_t m0, int64_t m1, int64_t m2, int64_t m3, int64_t m4);
void s2h_prof_end(int slot, hipStream_t st);
void s2h_prof_tag(int64_t tag);  // runtime.hip: the kernel of the current profiler record
// profiler tag of a GEMM tiling (include/sam2hip.h, s2h_prof_read_tags)
static inline int64_t gemm_tag(int BM, int BN, int WGM, int WGN, int NS, int BK, bool akc, bool bkc, bool regs,
                               bool mx8, bool areg = false) {
  return (int64_t)BM | ((int64_t)BN << 10) | ((int64_t)WGM << 20) | ((int64_t)WGN << 24) | ((int64_t)NS << 28) |
         ((int64_t)(BK / 32) << 32) | ((int64_t)akc << 36) | ((int64_t)bkc << 37) | ((int64_t)regs << 38) |
         ((int64_t)mx8 << 39) | ((int64_t)areg << 40);
}
