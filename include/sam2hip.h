/*
 * sam2hip.h -- C ABI of libsam2hip.so, the MI355X (gfx950) compute path of the
 * SAM2 video fine-tuning step (SAM2LightningModule.training_step,
 * reference sam2_video/training/trainer.py:256-289).
 *
 * Every entry point takes raw device pointers, int64 element strides, a dtype
 * tag, scalar parameters and the hipStream_t to launch on.  Nothing allocates
 * (workspaces are passed in), nothing synchronises, and every call returns a
 * hipError_t value (0 = success).  Element strides are in elements, not bytes.
 * Tensors are owned by the caller (the Python host package uses PyTorch's
 * caching allocator).  The library keeps no per-thread state; forward launches
 * come from the Python thread, backward launches from the autograd worker.
 *
 * Each declaration names the reference operation it replaces (file:line in the
 * reference repository, sam2_video/... paths; the modeling files are the
 * vendored SAM2.1 sources under sam2_video/model/modeling/).
 */
#ifndef SAM2HIP_H
#define SAM2HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same definition as hip_runtime_api.h, so the two headers can be combined. */
typedef struct ihipStream_t* hipStream_t;

/* dtype tags (`dt` arguments) */
enum { S2H_F32 = 0, S2H_BF16 = 1 };
/* fused activations (`act` arguments) */
enum { S2H_ACT_NONE = 0, S2H_ACT_RELU = 1, S2H_ACT_GELU = 2, S2H_ACT_SIGMOID = 3 };

/* ---------------------------------------------------------------- library */
/* ABI version (1). */
int s2h_version(void);
/* Bind a device-resident uint64 RNG offset (NULL unbinds).  Every dropout site
 * (s2h_gemm epilogue, s2h_attn_fwd/bwd, s2h_dropout) folds its current value into
 * the seed it was launched with, at kernel start: a captured HIP graph of the step
 * replays with fresh dropout masks (memory_attention.py:40-48, transformer.py:304-306
 * dropout_p) once the host advances the offset between replays; 0 = unchanged seed. */
int s2h_rng_bind(const void* dev_u64);
/* In-library launch profiler: `cap` > 0 pre-creates `cap` HIP event pairs and
 * brackets every launch of a selected kind on the stream it is launched on; 0 disables. */
int s2h_prof_enable(int cap);
/* kinds recorded: bit 1 attention forward, 2 attention backward, 4 GEMM, 8 trace markers (default 1) */
int s2h_prof_select(int mask);
int s2h_prof_reset(void);
int s2h_prof_count(void);
/* Copies up to `max` records: ms[i] (event elapsed time) and meta[6*i..] = (kind, shape):
 * attention (1, 2): (batch*heads, Lq, Lk, head_dim, element size);
 * GEMM (4): (batch, M, N, K, 2*A_kcontig + B_kcontig + 4*bf16).  Synchronises the events. */
int s2h_prof_read(int max, float* ms, int64_t* meta);
/* tags[i] = the kernel record i launched (0 = not tagged): GEMM tilings as
 * BM | BN << 10 | WGM << 20 | WGN << 24 | NS << 28 | (BK / 32) << 32 | A_kcontig << 36 |
 * B_kcontig << 37 | register_staged << 38 | mx_fp8 << 39 | a_in_registers << 40 |
 * deterministic_wgrad << 41 | ffn_bwd_dgrad << 42 | ffn_fwd << 43 -- the template arguments of the kernel rocprofv3 names (bench.py: the
 * roofline's dominant kernel). */
int s2h_prof_read_tags(int max, int64_t* tags);
/* Launches a one-lane no-op kernel (s2h_trace_marker_kernel) on `st`: brackets a region of a
 * rocprofv3 kernel trace (bench.py's timed steps, tools/step_profile.py). */
int s2h_trace_marker(int tag, hipStream_t st);

/* ---------------------------------------------------------------- GEMM
 * C[b](m,n) = act(alpha * sum_k A[b](m,k) B[b](k,n) + bias) * cscale[n], dropout(p, seed),
 *             + R[b](m,n) + beta * C[b](m,n)
 * (dropout element index drop_idx0 + (b*M + m)*N + n: a launch over frame f of a frame-stacked
 *  activation passes f*M*N so the frame-batched backward regenerates the same mask)
 * A addressed as A[m*lda_m + k*lda_k] (one of lda_m, lda_k must be 1), B as
 * B[k*ldb_k + n*ldb_n] (one of ldb_k, ldb_n must be 1), batch strides sA/sB/sC.
 * dt_ab: S2H_F32 (fp32 MFMA, parity mode; dt_c must be F32) or S2H_BF16 (bf16 MFMA,
 * fp32 accumulate; dt_c BF16 or F32).  bias_mode 1 = per column, 2 = per row.
 * aux_mode 1 stores the pre-activation into X; 2 multiplies by act'(X) (the
 * activation gradient of the layer that produced X) instead of applying act.
 * Replaces every nn.Linear / 1x1 nn.Conv2d / im2col conv / matmul on the path:
 *   hieradet.py:56-81 (qkv, proj), :140 (dim-change proj), sam2_utils.py:112-139 (MLP),
 *   transformer.py:230-243, 275-311 (q/k/v/out proj), memory_attention.py:58-99 (FFN),
 *   image_encoder.py:79 (FPN lateral 1x1), mask_decoder.py:66-81 (ConvT 2x2 / conv_s0/s1),
 *   utils.py:85 (PatchEmbed 7x7/4 conv), memory_encoder.py:43-156 (mask downsampler,
 *   CXBlock pwconv, pix_feat_proj, out_proj), mask_decoder.py:168-245 (hypernetwork
 *   product), hieradet.py:273-281 (bicubic pos-embed resize as two GEMMs),
 *   and their autograd backward (dgrad / wgrad). */
int s2h_gemm(int dt_ab, int dt_c, int batch, int M, int N, int K,
             const void* A, int64_t lda_m, int64_t lda_k, int64_t sA,
             const void* B, int64_t ldb_k, int64_t ldb_n, int64_t sB,
             void* C, int64_t ldc, int64_t sC,
             const float* bias, int bias_mode,
             const void* R, int64_t ldr, int64_t sR,
             void* X, int64_t ldx, int64_t sX, int aux_mode,
             const float* cscale, float drop_p, uint64_t seed, uint64_t drop_idx0,
             float alpha, float beta, int act, hipStream_t stream);

/* A/B switch (tests, benchmarks) for the bf16 GEMM tiling; returns the previous setting.
 * 0 = automatic by shape, -1 = register-staged kernel, LDS-DMA tilings: 1 = 64x64,
 * 2 = 128x128, 3 = 128x128 with a 3-deep ring, 4 = 256x128, 5 = 256x256, 6 = 128x256,
 * 7 = 128x64, 8 = 64x128, 9 = 64x64 with a 3-deep ring, 10 = 64x64 32-deep 4-deep ring,
 * 11 / 12 / 13 = 128x64 32-deep 3- / 4-deep ring and 64-deep 3-deep ring, 14 / 15 = 256x128 on 4 waves
 * (32-deep 3-deep ring / 64-deep 2-deep), 16 = 128x128 32-deep 3-deep ring, 17 = 256x64 on 4 waves;
 * bits 8+ are measurement-only ablations of the LDS-DMA kernel (results are wrong):
 * 256 = skip the epilogue stores, 512 = skip the MFMAs. */
int s2h_gemm_config(int cfg);

/* A/B knob (tests, benchmarks): workgroups a split-K weight-gradient GEMM aims at (default 768;
 * t <= 0 leaves it unchanged); returns the previous value. */
int s2h_gemm_split_target(int t);

/* A/B knob (tests, benchmarks): tiling of the GEMMs with M <= 128 rows (0 = automatic, values as
 * s2h_gemm_config); returns the previous setting. */
int s2h_gemm_tiny_config(int cfg);
/* A/B knob: the bf16-output GEMMs on 4 x 1 wave grids (whole 64-column rows per wave) instead of
 * 2 x 2 (1: all, the default; 2: only N >= 768; 0: off); results are bit-identical.  Returns the
 * previous mode. */
int s2h_gemm_w41(int mode);
/* A/B knob (round 6): tiling (values as s2h_gemm_config, 0 = the shape rules) of one class of
 * bf16-output GEMMs with M > 128 -- class 0: K >= 1024 and N <= 512; 1: K <= 256, N <= 256 and
 * M >= 8192; 2: K <= 512 and N >= 768; 3: 256 < K < 1024 and N <= 512; 4 / 5: K < 256 not a multiple
 * of 64 with M >= 65536 / with M < 65536 and K >= 128.  Returns the previous setting (-1: no such class). */
int s2h_gemm_class_config(int cls, int cfg);
/* A/B knob (round 6): bf16-output GEMMs with M <= 128, K >= 1024 and at most 16 64 x 64 output tiles as
 * one split-K fp32 launch into the weight-gradient workspace + one fixed-order reduce running the
 * GEMM epilogue (1: on; 0: the one-launch tiling, the default -- measured step-neutral); mode < 0 only queries.  Returns the
 * previous mode. */
int s2h_gemm_tiny_splitk(int mode);
/* A/B knob: GEMMs with a short K that is not a multiple of 64 (K < 256, K-contiguous A, bf16 output)
 * on the A-in-registers tiling (1: on, the default; 0: off); results are bit-identical.  Returns the
 * previous mode. */
int s2h_gemm_areg(int mode);
/* flash forward: 16-query sets per wave (1 or 2; bits 0-3 V-fold launches, 4-7 plain launches with
   head dim <= 128); returns the previous mode, < 0 only queries.  Same results either way. */
int s2h_flash_fwd_sets(int mode);

/* Weight and bias gradient of a Linear layer (autograd of nn.Linear, e.g. hieradet.py:56-81,
 * memory_attention.py:58-99): dw[N, K] (+)= dy[rows, N]^T x[rows, K] (dw row stride lddw),
 * db[N] (+)= sum over rows of dy (db may be NULL); `accumulate` 0 overwrites both.
 * bf16 dy/x: one launch, the bias gradient summed from the GEMM's staged dy tiles. */
int s2h_linear_wgrad(int dt, int64_t rows, int N, int K, const void* dy, int64_t lddy, const void* x,
                     int64_t ldx, float* dw, int64_t lddw, float* db, int accumulate, hipStream_t stream);

/* Workspace of the deterministic weight-gradient GEMM (round 5, csrc/gemm_wgrad.hip): bf16 GEMMs with
 * an fp32 output, both operands row-contiguous over a reduction of >= kmin rows (the Linear weight
 * gradients of s2h_linear_wgrad / s2h_gemm, e.g. memory_attention.py:97's FFN over 93184 rows) run on
 * 256 x 256-class tiles, write per-split fp32 partial tiles here and add them in fixed split order:
 * the gradient arena is bit-identical from run to run (the split-K path added with fp32 atomics).
 * ws: device memory of `bytes` owned by the caller (NULL: none, the atomic path runs); launches
 * using it must be stream-ordered.  kmin 0 turns the kernel off, -1 keeps the current value (4096).
 * Returns 0. */
int s2h_wgrad_workspace(void* ws, int64_t bytes, int kmin);
/* Measurement knob (tools/wgrad_bench.py): force that kernel's tile (0 = 256x256, 1 = 256x128,
 * 2 = 128x256, 3 = 128x128, 4 = 256x64, 5 = 64x256; -1 = its cost model) and split count (0 = the cost
 * model's).  Results stay bit-identical for a given choice.  Returns 0. */
int s2h_wgrad_force(int tile, int splits);

/* Deferred gradient sums (round 5, csrc/grad_defer.hip).  No reference counterpart: the reference's
 * parameter gradients come from torch autograd's per-op accumulation (the LayerNorm / Linear bias
 * backward inside nn.LayerNorm / nn.Linear, hieradet.py:98-166, memory_attention.py:58-99,
 * transformer.py:137-311).  Here those column reductions run as per-block partial rows + a fixed-order
 * sum; between s2h_grad_defer(ws, ...) and s2h_grad_defer(NULL, ...) the fixed-order sums whose
 * destinations lie inside [sink, sink + sink_bytes) (the gradient arena) are recorded instead of
 * launched, their partials kept in ws (device memory owned by the caller, 256-B aligned), and
 * s2h_grad_defer_flush adds them all in a few launches on `stream` (64 records per launch, in record
 * order for overlapping destinations).  Nothing may read those destinations before the flush.
 * s2h_grad_defer(NULL, ...) with records pending returns hipErrorNotReady. */
int s2h_grad_defer(void* ws, int64_t ws_bytes, void* sink, int64_t sink_bytes);
int s2h_grad_defer_flush(hipStream_t stream);
/* ends the deferral scope unconditionally, dropping unflushed records (cleanup after a failed flush).
 * Records are taken from one stream per scope (the first record's); s2h_grad_defer_flush on another
 * stream with records pending returns hipErrorInvalidResourceHandle. */
int s2h_grad_defer_reset(void);
/* records waiting for s2h_grad_defer_flush (not a hipError_t) */
int s2h_grad_defer_pending(void);

/* ---------------------------------------------------------------- MX-fp8 (BASELINE config 5)
 * No reference counterpart: the reference trains in fp32 / bf16 autocast only
 * (trainer.py:256-289 under Lightning `precision`); this is the fp8 variant of the projection
 * and FFN GEMMs the north_star asks for (`s2h_gemm` replaces nn.Linear in hieradet.py:56-91,
 * memory_attention.py:58-99, transformer.py:137-311).  OCP MX v1.0 MXFP8-E4M3: 32-element
 * blocks along the reduction dimension, one E8M0 scale each.
 *
 * s2h_mx8_quant: element (r, c) of X (bf16 / fp32) at X[r*ld_row + c*ld_col], r < rows, c < cols,
 * blocks along c.  Q [rows][ldq] u8 e4m3 (ldq >= cols rounded up to 128, ldq % 16 == 0, Q 16-B
 * aligned; columns cols..ldq-1 of the first round-up written as zeros); S [ceil(cols/128)][lds]
 * int32 scale words (lds >= rows): byte b of word (kt, r) = E8M0 scale of block 4kt+b of row r.
 * ld_row == 1 selects the row-walking lane order (a transposed source). */
int s2h_mx8_quant(int rows, int cols, int dt_x, const void* X, int64_t ld_row, int64_t ld_col, uint8_t* Q,
                  int64_t ldq, int32_t* S, int64_t lds, hipStream_t stream);

/* C[M, N] = epilogue(alpha * A B^T) for MX-fp8 A [M, K] (Q lda, scales SA, row stride lsa >= M)
 * and B [N, K] (ldb, SB, lsb >= N) as s2h_mx8_quant writes them; K is the logical depth (both
 * operands zero-padded to a multiple of 128).  Epilogue as s2h_gemm with bias per column:
 * act (aux_mode 1 stores the pre-activation to X, 2 multiplies by act'(X)), dropout, residual R,
 * beta.  C bf16 (dt_c 1) or fp32 (0). */
int s2h_gemm_mx8(int M, int N, int K, const uint8_t* A, int64_t lda, const int32_t* SA, int64_t lsa,
                 const uint8_t* B, int64_t ldb, const int32_t* SB, int64_t lsb, void* C, int dt_c, int64_t ldc,
                 const float* bias, const void* R, int64_t ldr, void* X, int64_t ldx, int aux_mode, float drop_p,
                 uint64_t seed, uint64_t drop_idx0, float alpha, float beta, int act, hipStream_t stream);

/* MX-fp8 GEMM tiling override for measurements: 0 automatic, 1 64x64, 2 128x64, 3 128x128;
 * bits 8+ measurement-only ablations (1 skip epilogue stores, 2 skip MFMAs, 4 skip operand DMA);
 * returns the previous value. */
int s2h_mx8_config(int cfg);

/* ---------------------------------------------------------------- attention
 * Fused multi-head attention, tensors [B, L, H, D] addressed through
 * (batch, head, row) strides with contiguous D; lse [B, H, Lq] fp32 (natural log).
 * Optional attention-probability dropout p_drop with a counter-based hash keyed by
 * `seed` (regenerated identically in the backward) over the element index
 * idx0 + ((b*H + h)*Lq + q)*Lk + k.  D in {32, 64, 96, 128, 256}
 * for bf16, 32..256 (multiple of 4) for fp32.
 * Replaces F.scaled_dot_product_attention at hieradet.py:70 (windowed / global
 * Hiera attention), transformer.py:243 (two-way decoder attention) and
 * transformer.py:306 (memory-attention RoPE self / cross attention).
 * bf16 with head_dim 256, or 32..128 in steps of 8 (run in a zero-padded 64 / 128 image: Hiera-B+'s
 * 56, Hiera-L's 72), and >= 128 query rows takes the flash path
 * (16x16x32 MFMA, LDS-DMA K/V ring, key range split over workgroups): it wants a
 * device workspace of s2h_attn_fwd_ws_bytes(...) bytes (ws = NULL / too small
 * just disables the key split). */
int64_t s2h_attn_fwd_ws_bytes(int dt, int B, int H, int Lq, int Lk, int D);
/* A/B switch (tests, benchmarks): bit 0 of flash_enable = 0 sends every attention to the
 * generic kernels; bits 8+ (if non-zero) set the workgroup count the flash forward key split
 * aims at (default 256).  Returns the previous setting in the same encoding. */
/* A/B knob: 1 (default) runs bf16 attentions with Lq, Lk <= 64, head dim <= 64 and no dropout (the
 * Hiera windows) on the whole-instance small-window kernels (attention.hip attn_win_*), 0 on the
 * tile kernels.  Returns the previous setting. */
int s2h_attn_win(int on);
int s2h_attn_config(int flash_enable);
/* A/B bits (round 6, default 0) of the non-V-fold flash kernels: 1 the head-dim-256 self-attention dQ
 * kernel with 8 fragment reads ahead, 2 the head-dim <= 128 dQ kernel on a 3-stage ring, 4 the
 * head-dim <= 128 forward on a 3-stage ring, 8 the 32x32 dK / dV kernel on a 3-stage ring, 16 the
 * one-row-per-wave key-split combine (all flash forwards, V-fold included).  Returns the previous bits
 * (mode < 0: query only). */
int s2h_flash_variant2(int mode);
/* A/B knob (round 6): fp32 GEMMs of fewer than 64 tiles of 64 x 64 on 32 x 32 tiles (1, default) or 64 x 64
 * (0).  Returns the previous mode (mode < 0: query only). */
int s2h_gemm_f32_small(int mode);
int s2h_attn_fwd(int dt, int B, int H, int Lq, int Lk, int D,
                 const void* q, int64_t sqb, int64_t sqh, int64_t sql,
                 const void* k, int64_t skb, int64_t skh, int64_t skl,
                 const void* v, int64_t svb, int64_t svh, int64_t svl,
                 void* o, int64_t sob, int64_t soh, int64_t sol,
                 float* lse, float scale, float p_drop, uint64_t seed, uint64_t idx0, uint32_t* keep,
                 void* ws, int64_t ws_bytes, hipStream_t st);
/* Dropout keep bitmap (`keep`, nullable, p_drop > 0 only): the flash forward at head_dim 256
 * also writes each element's keep flag -- bit (k & 31) of word [(b*H + h) * Lq + q] * kw + k/32,
 * kw = 2 * ceil(Lk / 64); s2h_attn_keep_words(...) words -- and the backward reads it instead
 * of re-hashing.  A non-NULL keep on a launch that does not take that path is an error. */
int64_t s2h_attn_keep_words(int B, int H, int Lq, int Lk);
/* Backward of s2h_attn_fwd; di_ws: fp32 workspace [B*H*Lq].  The flash forward's domain takes
 * the flash path (dQ kernel with key-split fp32 partials in
 * `ws` of s2h_attn_bwd_ws_bytes(...) bytes, dK/dV kernel per 128-key block). */
int64_t s2h_attn_bwd_ws_bytes(int dt, int B, int H, int Lq, int Lk, int D);
int s2h_attn_bwd(int dt, int B, int H, int Lq, int Lk, int D,
                 const void* q, int64_t sqb, int64_t sqh, int64_t sql,
                 const void* k, int64_t skb, int64_t skh, int64_t skl,
                 const void* v, int64_t svb, int64_t svh, int64_t svl,
                 const void* o, int64_t sob, int64_t soh, int64_t sol,
                 const void* dout, int64_t sgb, int64_t sgh, int64_t sgl,
                 void* dq, int64_t sdqb, int64_t sdqh, int64_t sdql,
                 void* dk, int64_t sdkb, int64_t sdkh, int64_t sdkl,
                 void* dv, int64_t sdvb, int64_t sdvh, int64_t sdvl,
                 const float* lse, float* di_ws, float scale, float p_drop, uint64_t seed, uint64_t idx0,
                 const uint32_t* keep, void* ws, int64_t ws_bytes, hipStream_t st);
/* Frame-batched flash backward (the flash domain: bf16, head_dim 32..128 / 256, Lq >= 128):
 * nfr frames x bpf batches x H heads of the tracking loop in one launch per kernel -- Q / O / dO /
 * dQ / lse uniform [nfr*bpf] batches, K / V / dK / dV packed per frame (frame f: bpf blocks of fr_lk[f] rows
 * starting at row fr_krow[f]); frame f's dropout indices start at fr_idx0[f] (host arrays of
 * nfr <= 32 entries); keep (nullable) = the frames' forward keep bitmaps, frame f's from word
 * fr_koff[f].  The memory-attention backward of every frame at once
 * (transformer.py:275-311 for frames 1..T-1, memory_attention.py:58-99). */
/* 1 when s2h_flash_bwd_frames takes (dt, Lq, head_dim); 0 = run the frames one by one. */
int s2h_flash_bwd_ok(int dt, int Lq, int D);
int s2h_flash_bwd_frames(int nfr, int bpf, int H, int Lq, int D, const int* fr_lk, const int64_t* fr_krow,
                         const uint64_t* fr_idx0, const void* q, int64_t sqb, int64_t sqh, int64_t sql,
                         const void* k, int64_t skh, int64_t skl, const void* v, int64_t svh, int64_t svl,
                         const void* o, int64_t sob, int64_t soh, int64_t sol, const void* dout, int64_t sgb,
                         int64_t sgh, int64_t sgl, void* dq, int64_t sdqb, int64_t sdqh, int64_t sdql, void* dk,
                         int64_t sdkh, int64_t sdkl, void* dv, int64_t sdvh, int64_t sdvl, const float* lse,
                         float* di_ws, float scale, float p_drop, uint64_t seed, const uint32_t* keep,
                         const int64_t* fr_koff, hipStream_t st);
/* s2h_flash_bwd_frames with the q projection's RoPE epilogue transposed into the dQ store
 * (position_encoding.py:212-239 apply_rotary_enc, transposed; head dim 256; replaces the separate
 * rotation pass over dq of the memory self-attention, transformer.py:296-307): query rows
 * < fr_nrotq[f] of every batch block of frame f are rotated back with table row (row % rope_period)
 * of cos / sin [period, 128] fp32 (fr_nrotq NULL: unrotated); dk is stored unrotated. */
int s2h_flash_bwd_frames_rope(int nfr, int bpf, int H, int Lq, int D, const int* fr_lk, const int64_t* fr_krow,
                              const uint64_t* fr_idx0, const void* q, int64_t sqb, int64_t sqh, int64_t sql,
                              const void* k, int64_t skh, int64_t skl, const void* v, int64_t svh, int64_t svl,
                              const void* o, int64_t sob, int64_t soh, int64_t sol, const void* dout, int64_t sgb,
                              int64_t sgh, int64_t sgl, void* dq, int64_t sdqb, int64_t sdqh, int64_t sdql, void* dk,
                              int64_t sdkh, int64_t sdkl, void* dv, int64_t sdvh, int64_t sdvl, const float* lse,
                              float* di_ws, float scale, float p_drop, uint64_t seed, const uint32_t* keep,
                              const int64_t* fr_koff, const float* rope_cos, const float* rope_sin, int rope_period,
                              const int* fr_nrotq, hipStream_t st);

/* V-fold of the memory-attention cross-attention (RoPEAttention, transformer.py:275-311, with
 * kv_in_dim 64: memory_attention.py:66-81, sam2.1_hiera_t.yaml:49-58).  Its values are a projection
 * of the 64-channel memory bank M, V = M Wv^T + bv, so with D = dropout(softmax(scale q k^T))
 * (the dropped, normalised probabilities) attention(q, k, V) = u' [Wv | bv]^T where
 * u' = [D M | rowsum(D) | 0 x 7] (72 columns).  Single head, q / k head_dim 256, bf16, Lq >= 128.
 * s2h_attn_fwd_vfold: q [B, Lq, 256], k [B, Lk, 256] (RoPE applied), mem [B, Lk, 64] -> u [B, Lq,
 * sul >= 72], lse [B, Lq]; strides (batch, row) in elements, 16-B aligned rows; ws of
 * s2h_attn_fwd_vfold_ws_bytes bytes enables the key split; keep: as s2h_attn_fwd (B, H = 1).
 * Replaces v_proj(memory) + the SDPA of the cross-attention (transformer.py:296-307). */
int64_t s2h_attn_fwd_vfold_ws_bytes(int B, int Lq, int Lk);
int s2h_attn_fwd_vfold(int B, int Lq, int Lk, const void* q, int64_t sqb, int64_t sql, const void* k, int64_t skb,
                       int64_t skl, const void* mem, int64_t smb, int64_t sml, void* u, int64_t sub, int64_t sul,
                       float* lse, float scale, float p_drop, uint64_t seed, uint64_t idx0, uint32_t* keep, void* ws,
                       int64_t ws_bytes, hipStream_t st);
/* Frame-batched backward of s2h_attn_fwd_vfold (layout as s2h_flash_bwd_frames, H = 1): du = the
 * gradient of u' (dO [Wv | bv | 0], 72 columns), dq, dk; no value gradient (the memory bank is
 * detached, sam2model.py:345-358).  di_ws: fp32 [nfr * bpf * Lq]. */
int s2h_flash_bwd_frames_vfold(int nfr, int bpf, int Lq, const int* fr_lk, const int64_t* fr_krow,
                               const uint64_t* fr_idx0, const void* q, int64_t sqb, int64_t sql, const void* k,
                               int64_t skl, const void* mem, int64_t sml, const void* u, int64_t sub, int64_t sul,
                               const void* du, int64_t sgb, int64_t sgl, void* dq, int64_t sdqb, int64_t sdql, void* dk,
                               int64_t sdkl, const float* lse, float* di_ws, float scale, float p_drop, uint64_t seed,
                               const uint32_t* keep, const int64_t* fr_koff, hipStream_t st);
/* The same with the keys' inverse RoPE fused into the dK store (position_encoding.py:212-239
 * apply_rotary_enc with repeat_freqs_k, transposed; replaces the separate rotation pass over dk):
 * key rows < fr_nrot[f] of every batch block of frame f are rotated back with table row
 * key % rope_period of cos / sin [period, 128] fp32 (head dim 256, every column rotated); the
 * remaining rows (object-pointer keys) are stored as computed.  rope_cos == NULL: no rotation. */
int s2h_flash_bwd_frames_vfold_rope(int nfr, int bpf, int Lq, const int* fr_lk, const int64_t* fr_krow,
                                    const uint64_t* fr_idx0, const void* q, int64_t sqb, int64_t sql, const void* k,
                                    int64_t skl, const void* mem, int64_t sml, const void* u, int64_t sub, int64_t sul,
                                    const void* du, int64_t sgb, int64_t sgl, void* dq, int64_t sdqb, int64_t sdql,
                                    void* dk, int64_t sdkl, const float* lse, float* di_ws, float scale, float p_drop,
                                    uint64_t seed, const uint32_t* keep, const int64_t* fr_koff, const float* rope_cos,
                                    const float* rope_sin, int rope_period, const int* fr_nrot, hipStream_t st);
/* + the query projection's inverse RoPE in the dQ store (query rows < fr_nrotq[f], same tables;
 * transformer.py:296 q rotation transposed).  fr_nrot / fr_nrotq each NULL: that gradient unrotated. */
int s2h_flash_bwd_frames_vfold_rope_qk(int nfr, int bpf, int Lq, const int* fr_lk, const int64_t* fr_krow,
                                       const uint64_t* fr_idx0, const void* q, int64_t sqb, int64_t sql, const void* k,
                                       int64_t skl, const void* mem, int64_t sml, const void* u, int64_t sub,
                                       int64_t sul, const void* du, int64_t sgb, int64_t sgl, void* dq, int64_t sdqb,
                                       int64_t sdql, void* dk, int64_t sdkl, const float* lse, float* di_ws,
                                       float scale, float p_drop, uint64_t seed, const uint32_t* keep,
                                       const int64_t* fr_koff, const float* rope_cos, const float* rope_sin,
                                       int rope_period, const int* fr_nrot, const int* fr_nrotq, hipStream_t st);
/* [Wv | bv | 0] as a bf16 [N, ld] matrix (ld >= K + 1) from the bf16 weight [N, K] and the fp32 bias,
 * and its fp32 gradient g [N, ld] scattered back: gwv [N, K] += g[:, :K], gbv [N] += g[:, K]
 * (either nullable).  The value projection's parameters of the folded cross-attention. */
int s2h_vfold_weight(int N, int K, int ld, const void* wv, const float* bv, void* out, hipStream_t st);
int s2h_vfold_grad(int N, int K, int ld, const float* g, float* gwv, float* gbv, hipStream_t st);

/* bf16 Linear whose output is rotated by the axial RoPE in the GEMM epilogue: Y = A W^T + bias
 * (A [M, K], W [N, K] rows K-contiguous), then in every block of L rows the rows r < nrot are
 * rotated in (2i, 2i+1) column pairs for columns c < ncol with table row r % period and column
 * (c % dh) / 2 (cosv / sinv [period, dh / 2] fp32, as s2h_rope).  Replaces q_proj / k_proj +
 * apply_rotary_enc (transformer.py:275-311, position_encoding.py:212-239) and the fused
 * q / k / v projection of the memory self-attention with q and k rotated (ncol = 2 x 256). */
int s2h_linear_rope(int M, int N, int K, const void* A, int64_t lda, const void* W, int64_t ldw, const float* bias,
                    void* Y, int64_t ldy, const float* cosv, const float* sinv, int L, int nrot, int period, int ncol,
                    int dh, hipStream_t stream);
/* Linear + dropout + residual + LayerNorm in one launch (bf16): C = R + dropout(A W^T + bias)
 * (the residual stream x'), Y = LN(C) * gamma + beta, mean / rstd per row -- a projection and the
 * residual add + LayerNorm that reads it (memory_attention.py:60-98: out_proj -> norm2, the
 * cross-attention output -> norm3, linear2 -> the next layer's norm1; nn.LayerNorm).  N = 128 or 256
 * (one workgroup per 64 full rows); A [M, K] (lda), W [N, K] (ldw), R / C / Y with row strides;
 * 16-B aligned rows.  R may be NULL (no residual); dropout index = drop_idx0 + row * N + col. */
int s2h_linear_add_ln(int M, int N, int K, const void* A, int64_t lda, const void* W, int64_t ldw,
                      const float* bias, const void* R, int64_t ldr, float drop_p, uint64_t seed,
                      uint64_t drop_idx0, void* C, int64_t ldc, const float* gamma, const float* beta, float eps,
                      void* Y, int64_t ldy, float* mean, float* rstd, hipStream_t st);
/* Backward twin: input gradient of a Linear whose input is a LayerNorm output read by nothing else,
 * with that LayerNorm's backward in the GEMM epilogue (bf16): dy = alpha * G W (G [M, K] the Linear's
 * output gradient, W [K, N] its weight), dx = LN'(dy; X, gamma, mean, rstd) + dres (C [M, N]),
 * dgamma / dbeta += (both or neither; `part` = s2h_linear_dgrad_ln_bwd_ws_bytes(M, N) bytes of
 * per-tile partial rows).  Replaces linear dgrad + s2h_layernorm_bwd for memory_attention.py:60-98
 * norm1 -> q/k/v, norm2 -> cross-attention q, norm3 -> linear1 (torch autograd of nn.Linear +
 * nn.LayerNorm).  N = 128 or 256; 16-B aligned rows; dres may be NULL. */
/* Memory-attention FFN backward, input-gradient side, one launch (bf16; memory_attention.py:97,
 * replacing torch autograd's linear2 input gradient -> ReLU/dropout backward -> linear1 input gradient):
 *   dh [R, H] = alpha * (dy [R, 256] w2 [256, H]) * [hid > 0]     (alpha = 1 / keep)
 *   dx [R, 256] = dh w1 [H, 256]
 * hid = linear2's saved input (ReLU -> dropout output).  R a multiple of 64, H of 128; 16-B aligned
 * bases, row strides multiples of 8 elements. */
int s2h_ffn_bwd_dgrad(int R, int H, const void* dy, int64_t lddy, const void* w2, const void* w1, const void* hid,
                      int64_t ldh, float alpha, void* dh, int64_t lddh, void* dx, int64_t lddx, hipStream_t st);
/* Memory-attention FFN forward, one launch (bf16; memory_attention.py:97, replacing linear1 + ReLU +
 * dropout and linear2 + dropout as two GEMM launches):
 *   hid [R, H] = drop1(relu(x [R, 256] w1 [H, 256]^T + b1))      (saved for the backward)
 *   y [R, 256] = drop2(hid w2 [256, H]^T + b2)
 * b1 / b2 fp32; dropout p with the GEMM epilogue's counter hash (seed1, element idx1 + row * H + h;
 * seed2, idx2 + row * 256 + n), each seed folded with the bound RNG offset.  R a multiple of 64, H 1024
 * or 2048; 16-B aligned bases, row strides multiples of 8 elements. */
int s2h_ffn_fwd(int R, int H, const void* x, int64_t ldx, const void* w1, const float* b1, const void* w2,
                const float* b2, float p, uint64_t seed1, uint64_t idx1, uint64_t seed2, uint64_t idx2, void* hid,
                int64_t ldh, void* y, int64_t ldy, hipStream_t st);
/* Two-way transformer token side, forward (bf16; sam/transformer.py:112-197, replacing per block ~17
 * of ~17 launches (13 objects x 8 tokens) to five).  R = objects x T rows (T <= 16
 * tokens per object, an object never split), width 256, self-attention 8 heads of 32, cross-attention
 * width 128, MLP 256 -> 2048 -> 256 ReLU; weights [N, K] bf16 row-major, biases / LayerNorm fp32.  Every
 * intermediate is written where the frame tape stores the corresponding op's output (lse [objects, 8,
 * T] natural log; mean / rstd per row).
 * s2h_dec_self (transformer.py:163-170): qa = x + pe (skip == 0, else unused), q / k from (skip ? x : qa),
 *   v from x, os = self-attention, y1 = os Wo^T + bo (+ x unless skip), x1 = norm1(y1), qt = x1 + pe,
 *   qq = qt Wqc^T + bqc (the token -> image query). */
int s2h_dec_self(int R, int T, int skip, float scale, const void* x, const void* pe, const void* wq, const float* bq,
                 const void* wk, const float* bk, const void* wv, const float* bv, const void* wo, const float* bo,
                 const float* g1, const float* b1, float eps1, const void* wqc, const float* bqc, void* qa, void* qs,
                 void* ks, void* vs, void* os, float* lse, void* y1, void* x1, float* mean1, float* rstd1, void* qt,
                 void* qq, hipStream_t st);
/* A/B knob (round 6): 1 (default) the s2h_dec_* kernels issue each projection's weight fragments a phase
 * ahead (s2h_dec_self: the q / k / v weights together, the out- and q-projection weights under the
 * attention and norm1; the others: under their row loads and LayerNorms), 0 each projection loads its own
 * before its MFMAs; the same sums either way.  Returns the previous setting
 * (mode < 0: query only). */
int s2h_dec_sched(int mode);
/* The second half's token side around the MLP (whose two GEMMs stay s2h_gemm launches; transformer.py:170-173):
 * s2h_dec_post_a: y2 = ot Wo^T + bo + x1, x2 = norm2(y2);
 * s2h_dec_post_b: x3 = norm3(y3) (y3 = MLP output + x2), q2 = x3 + pe, kio = q2 Wki^T + bki,
 *   vio = x3 Wvi^T + bvi (the image -> token keys / values); final_q: qfa = x3 + pe, qqf = qfa Wqf^T + bqf
 *   (TwoWayTransformer's final token -> image query, :194-196). */
int s2h_dec_post_a(int R, int T, const void* ot, const void* x1, const void* wo, const float* bo, const float* g2,
                   const float* b2n, float eps2, void* y2, void* x2, float* mean2, float* rstd2, hipStream_t st);
int s2h_dec_post_b(int R, int T, int final_q, const void* y3, const void* pe, const float* g3, const float* b3n,
                   float eps3, const void* wki, const float* bki, const void* wvi, const float* bvi, const void* wqf,
                   const float* bqf, void* x3, float* mean3, float* rstd3, void* q2, void* kio, void* vio, void* qfa,
                   void* qqf, hipStream_t st);
/* s2h_dec_final (transformer.py:196-197): y = of Wo^T + bo + x3, hs = norm(y). */
int s2h_dec_final(int R, int T, const void* of, const void* x3, const void* wo, const float* bo, const float* g,
                  const float* bn, float eps, void* y, void* hs, float* mean, float* rstd, hipStream_t st);
int64_t s2h_linear_dgrad_ln_bwd_ws_bytes(int M, int N);
int s2h_linear_dgrad_ln_bwd(int M, int N, int K, const void* G, int64_t ldg, const void* W, int64_t ldw, float alpha,
                            const void* X, int64_t ldx, const float* gamma, const float* mean, const float* rstd,
                            const void* dres, int64_t ldr, void* dx, int64_t lddx, float* part, float* dgamma,
                            float* dbeta, hipStream_t st);
/* dgamma += sum_b part[b][0:C], dbeta += sum_b part[b][C:2C] over nb partial rows of 2C floats. */
int s2h_ln_wgrad_finalize(int nb, int C, const float* part, float* dgamma, float* dbeta, hipStream_t st);

/* Per-object MLP heads under no_grad in ONE launch (bf16): for each of nheads (<= 4) heads, rows
 * x[h] [M, dims[4h]] (row stride ldx[h]) through nl[h] (<= 3) Linear layers w[3h + l]
 * [dims[4h+l+1], dims[4h+l]] (+ fp32 bias b[3h + l] or NULL), ReLU between layers, act_last[h]
 * (S2HAct) after the last, into y[h] [M, dims[4h + nl]] (row stride ldy[h]); widths <= 256 (hidden
 * ones multiples of 8), 16-B aligned rows.  Bit-identical to the per-layer GEMMs.  Replaces the
 * object-score head (mask_decoder.py:234-238) and the object-pointer projection (sam2_base.py:296-305
 * obj_ptr_proj): 6 launches of 13 rows per frame -> 1.  Argument arrays are host memory. */
int s2h_mlp_heads(int nheads, int M, const void* const* x, const int64_t* ldx, const void* const* w,
                  const float* const* b, const int* dims, const int* nl, const int* act_last, void* const* y,
                  const int64_t* ldy, void* const* hid, void* const* pre, hipStream_t st);
/* (hid[2h + l], optional: layer l's ReLU output [M, dims[4h+l+1]] for l < nl - 1; pre[h], optional:
 * the last layer's pre-activation -- saved for the backward of trained heads: the mask decoder's
 * hypernetwork MLP and IoU head, mask_decoder.py:227-233, in the frame-batched tape) */

/* ---------------------------------------------------------------- normalisation
 * Row LayerNorm over C (<= 1280) with an optional fused pre-add:
 * xsum = x + badd (badd broadcast over rows when b_bcast), y = LN(xsum) * gamma + beta;
 * saves per-row mean / rstd (fp32).  Replaces nn.LayerNorm (hieradet.py:134-166,
 * memory_attention.py:43-45,115, transformer.py:63,137-149) and LayerNorm2d
 * (sam2_utils.py:141-151, NHWC rows) and the residual adds feeding them. */
int s2h_layernorm_fwd(int dt, int rows, int C, const void* x, int64_t ldx, const void* badd, int64_t ldb,
                      int b_bcast, void* xsum, const float* gamma, const float* beta, float eps, void* y,
                      int64_t ldy, float* mean, float* rstd, hipStream_t st);
/* bf16 LayerNorm of contiguous rows that also stores ype = y + pe[row % pe_rows] (the two-way
 * transformer's keys + key_pe after norm4, transformer.py:182-185 feeding the next block's
 * k = keys + key_pe, transformer.py:170 / :102): y bit-identical to s2h_layernorm_fwd, ype to the
 * broadcast add it replaces.  16-B aligned rows, C / 8 <= 64. */
int s2h_layernorm_fwd_pe(int dt, int rows, int C, const void* x, const float* gamma, const float* beta, float eps,
                         void* y, float* mean, float* rstd, const void* pe, int pe_rows, void* ype, hipStream_t st);
/* dx = LN'(dy) (+= when dx_accum, or + dres: the residual-stream gradient of the fused
 * pre-add, so the caller needs no copy), dgamma += , dbeta += (fp32, both or neither).
 * The weight gradients go through per-block partials in `ws`
 * (s2h_layernorm_bwd_ws_bytes(dt, rows, C) bytes; may be NULL when dgamma is NULL). */
int64_t s2h_layernorm_bwd_ws_bytes(int dt, int rows, int C);
int s2h_layernorm_bwd(int dt, int rows, int C, const void* x, int64_t ldx, const void* dy, int64_t lddy,
                      const float* gamma, const float* mean, const float* rstd, void* dx, int64_t lddx,
                      int dx_accum, const void* dres, int64_t ldres, float* dgamma, float* dbeta, void* ws,
                      hipStream_t st);

/* ---------------------------------------------------------------- elementwise / layout
 * out = alpha*a + beta*b (residual adds, sam2_base.py:680-684 no_mem_embed,
 * memory_attention.py:140-141 curr + 0.1*pos). */
int s2h_add(int dt, int64_t n, const void* a, const void* b, float alpha, float beta, void* out, hipStream_t st);
/* out[o, i] = alpha*a[o, i] + beta*b[i % b_period] (bias / embedding broadcast:
 * mask_decoder.py:201-209 dense prompt add, sam2_base.py:761-767 no_obj_embed_spatial). */
int s2h_add_bcast(int dt, int64_t outer, int64_t inner, const void* a, float alpha, const void* b,
                  int64_t b_period, float beta, void* out, hipStream_t st);
/* y = act(scale*x + shift) (GELU / ReLU / sigmoid; sam2_base.py:742-747 mask_for_mem). */
int s2h_act_fwd(int dt, int64_t n, const void* x, int act, float scale, float shift, void* y, hipStream_t st);
/* dx (=, or += when accum) = dy * act'(x). */
int s2h_act_bwd(int dt, int64_t n, const void* x, const void* dy, int act, void* dx, int accum, hipStream_t st);
/* dtype conversion (fp32 <-> bf16; sam2_base.py:391-399 `.float()` of the logits). */
int s2h_cast(int dt_in, int dt_out, int64_t n, const void* x, void* y, hipStream_t st);
/* out = a + dropout(b) (b may be NULL: out = dropout(a)), element index idx0 + i; nn.Dropout at
 * memory_attention.py:40-48 and the post-attention / FFN dropouts. */
int s2h_dropout(int dt, int64_t n, const void* a, const void* b, float p, uint64_t seed, uint64_t idx0, void* out,
                hipStream_t st);
/* dx = act'(x_pre) * keep(i) / (1 - p) * dy in one pass: the backward of a Linear epilogue's
 * act -> dropout (memory_attention.py:95-98); x_pre NULL = no activation. */
int s2h_act_dropout_bwd(int dt, int64_t n, const void* x_pre, const void* dy, int act, float p, uint64_t seed,
                        uint64_t idx0, void* dx, hipStream_t st);
/* dx = scale * [y > 0] * dy: the backward of ReLU (-> dropout, scale = 1/(1-p)) from the layer's
 * output y, which is positive exactly where the pre-activation was and the element was kept
 * (memory_attention.py:95-98 linear1 + ReLU + dropout; no pre-activation stored, no re-hash). */
int s2h_relu_mask_bwd(int dt, int64_t n, const void* y, const void* dy, float scale, void* dx, hipStream_t st);
/* Axial rotary embedding of the first `nrot` rows of each batch (cos/sin tables
 * [period, D/2], row r uses entry r % period; inverse = 1 applies the transpose
 * rotation for the backward).  Replaces apply_rotary_enc (position_encoding.py:212-239)
 * with compute_axial_cis tables (:192-201) and the key-repeat at transformer.py:291-299. */
int s2h_rope(int dt, int64_t nb, int nrot, int D, const void* x, int64_t sxb, int64_t sxl, void* y,
             int64_t syb, int64_t syl, const float* cosv, const float* sinv, int period, int inverse,
             hipStream_t st);
/* 2x2/2 max pooling, NHWC with pixel stride ldx (do_pool, hieradet.py:25-36). */
int s2h_maxpool2_fwd(int dt, int B, int H, int W, int C, const void* x, int64_t ldx, void* y, hipStream_t st);
int s2h_maxpool2_bwd(int dt, int B, int H, int W, int C, const void* x, int64_t ldx, const void* dy,
                     void* dx, int64_t lddx, hipStream_t st);
/* Up to 16 strided 2-D copies in one launch (replaces torch.cat / copy_ of the memory bank
 * assembly, reference sam2_base.py:649-676, and the tracking loop's per-frame gradient packing):
 * segment s copies rows[s] rows of row_bytes[s] bytes from src[s] (pitch src_ld[s] bytes) to dst[s]
 * (pitch dst_ld[s]; destination rows must not overlap, a source pitch of 0 broadcasts).  Host arrays
 * of n entries; bases, pitches and row lengths 4-B aligned (16-B aligned segments move in 16-B
 * pieces), else hipErrorInvalidValue. */
int s2h_copy2d_batch(int n, const void* const* src, void* const* dst, const int64_t* rows, const int64_t* row_bytes,
                     const int64_t* src_ld, const int64_t* dst_ld, hipStream_t st);
/* window_partition (dir 0) / window_unpartition (dir 1) with zero padding
 * (backbones/utils.py:16-60); accum adds into dst. */
int s2h_window(int dt, int B, int H, int W, int C, int ws, const void* src, void* dst, int dir, int accum,
               hipStream_t st);
/* window_partition of a per-token projection's output with the padded positions set to padrow
 * (fp32 [C], rounded to dt): with padrow = the projection's bias this equals the projection of the
 * zero-padded partition (hieradet.py:146 pads before attn.qkv), so the projection runs over the real
 * tokens only.  C a multiple of 16 B, 16-B aligned tensors. */
int s2h_window_pad(int dt, int B, int H, int W, int C, int ws, const void* src, const float* padrow, void* dst,
                   hipStream_t st);
/* Its bias gradient: out[c] += sum of win[row][c] over the padded rows of the windowed tensor
 * (fixed-order partial sums). */
int s2h_window_pad_colsum(int dt, int B, int H, int W, int C, int ws, const void* win, float* out, hipStream_t st);
/* FPN top-down: out = lat + nearest_up2(prev) (image_encoder.py:102-134). */
int s2h_up2_add(int dt, int B, int H, int W, int C, const void* lat, const void* prev, void* out, hipStream_t st);
/* Backward of the nearest 2x upsample: dprev (+)= 2x2 sum of dout. */
int s2h_pool2_sum(int dt, int B, int Ho, int Wo, int C, const void* dout, void* dprev, int accum, hipStream_t st);
/* Bilinear resize, align_corners=False, fp32 [N, hi, wi] -> [N, ho, wo]
 * (F.interpolate at sam2_base.py:393-399, low-res -> high-res mask logits). */
int s2h_bilinear_fwd(int N, int hi, int wi, int ho, int wo, const float* x, float* y, hipStream_t st);
int s2h_bilinear_bwd(int N, int hi, int wi, int ho, int wo, const float* dy, float* dx, hipStream_t st);
/* out[c] (=, or += when accum) = sum_r x[r, c] (bias gradients). */
int s2h_colsum(int dt, int64_t rows, int cols, const void* x, int64_t ld, float* out, int accum, hipStream_t st);
/* Segmented column sums, one launch: out[dsts[s], c] += sum_{r < rows} x[offs[s] + r, c] for s < nseg
 * (<= 64; cols a multiple of the 16-B vector, <= 256 vectors).  The memory positions' temporal-code
 * gradient (sam2_base.py:605-611: maskmem_tpos_enc added per memory slot), all slots of all frames. */
int s2h_colsum_seg(int dt, int nseg, int64_t rows, int cols, const void* x, int64_t ld, const int64_t* offs,
                   const int* dsts, float* out, hipStream_t st);
/* Memory positions, one launch: out[j L + l, :] = pos[l, :] + tpos[idx[j], :] for j < n (<= 16)
 * (sam2_base.py:605-611: the memory encoder position + maskmem_tpos_enc[t] per memory slot). */
int s2h_memory_pos(int dt, int n, int L, int Dm, const void* pos, const void* tpos, const int* idx, void* out,
                   hipStream_t st);
/* out[i] (=/+=) sum_o x[o, i] (gradient of a per-object broadcast of shared
 * features: sam2model.py:307-311, mask_decoder.py:201,209 repeat_interleave). */
int s2h_sum_outer(int dt, int O, int64_t inner, const void* x, void* out, int accum, hipStream_t st);
/* out[f][:] (+)= sum over o < O of x[f][o][:] for F frames in one launch (x [F, O, inner], out [F, inner];
 * the frame-batched backward of a broadcast over objects, tracking.py / mask_decoder.py); each element
 * summed in o order (the values of F s2h_sum_outer launches). */
int s2h_sum_outer_batched(int dt, int F, int O, int64_t inner, const void* x, void* out, int accum,
                          hipStream_t st);
/* NHWC im2col in PyTorch weight order (c, ky, kx) for the strided convolutions
 * (PatchEmbed utils.py:85; MaskDownSampler memory_encoder.py:43): rows of ldcol >= C*kh*kw elements,
 * the columns past C*kh*kw written as zeros. */
int s2h_im2col(int dt, int B, int H, int W, int C, int kh, int kw, int stride, int pad, int Ho, int Wo,
               int64_t ldcol, const void* x, void* col, hipStream_t st);
/* Mask down-sampler stage, fused 3x3/2 pad-1 conv + LayerNorm2d(cout) + GELU, NHWC
 * (memory_encoder.py:17-55 MaskDownSampler.encoder[3i..3i+2] with the SAM2.1 config
 * kernel_size 3, stride 2, padding 1).  Supported (cin, cout): (1, 4), (4, 16), (16, 64).
 * x_logit: x is the fp32 high-res mask logits [O, H, W] and the stage applies
 * sigmoid(x) * scale + shift first (sam2_base.py:742-747).  Weights fp32 [cout, cin, 3, 3].
 * y [O, ceil(H/2), ceil(W/2), cout]. */
int s2h_mask_down_stage(int dt, int O, int H, int W, int cin, int cout, const void* x, int x_logit, float scale,
                        float shift, const float* w, const float* bias, const float* gamma, const float* beta,
                        float eps, void* y, hipStream_t st);
/* Depthwise KxK conv, NHWC, fp32 weights [C, K, K] (CXBlock dwconv, memory_encoder.py:84). */
int s2h_dwconv(int dt, int B, int H, int W, int C, int K, int pad, const void* x, const float* w,
               const float* bias, void* y, hipStream_t st);
/* ConvTranspose2d k=2 s=2 as GEMM + scatter (dir 0: out = scatter(Y) + bias (+ add));
 * dir 1 gathers the output gradient into GEMM layout (mask_decoder.py:66-75). */
int s2h_convt2(int dt, int B, int H, int W, int Co, const void* Y, const float* bias, const void* add,
               void* out, int dir, hipStream_t st);
/* The forward scatter vectorised with the bias and the residual add fused (round 5; mask_decoder.py:105-107
 * dc1(x) + feat_s1, dc2(x) + feat_s0): out[b, 2y+dy, 2x+dx, co] = Y[(b,y,x)][co*4 + dy*2 + dx] + bias[co]
 * (+ add[b or 0 when add_bcast, 2y+dy, 2x+dx, co]), rounded after the bias and after the add as the
 * two launches it replaces.  Co % (16 B / element) == 0, 16-B aligned buffers. */
int s2h_convt2_store(int dt, int B, int H, int W, int Co, const void* Y, const float* bias, const void* add,
                     int add_bcast, void* out, hipStream_t st);
/* The mask decoder's last upscaling step and mask head in one pass (mask_decoder.py:105-113, bf16,
 * Co = 32): pre = the s2h_convt2_store values, post = gelu(pre) (as s2h_act_fwd rounds it), masks[b][p] =
 * sum_c hyper[b][c] post[b][p][c] (fp32 sum, bf16 store); pre / post [B, 2H, 2W, 32], masks [B, 2H * 2W]. */
int s2h_convt2_tail(int dt, int B, int H, int W, int Co, const void* Y, const float* bias, const void* add,
                    int add_bcast, const void* hyper, void* pre, void* post, void* masks, hipStream_t st);
/* The first upscaling step in one pass (mask_decoder.py:105-106, bf16, Co = 64): pre = the s2h_convt2_store
 * values, y / mean / rstd = LayerNorm2d(pre) over the channels (gamma, beta, eps; the values of
 * s2h_layernorm_fwd), post = gelu(y) (as s2h_act_fwd rounds it); mean / rstd [B * 2H * 2W] fp32. */
int s2h_convt2_ln_gelu(int dt, int B, int H, int W, int Co, const void* Y, const float* bias, const void* add,
                       int add_bcast, const float* gamma, const float* beta, float eps, void* pre, void* y,
                       float* mean, float* rstd, void* post, hipStream_t st);
/* y[r, :] = gate[r] > 0 ? x[r, :] : fill; dir 1 = backward (object-score gating to
 * NO_OBJ_SCORE, sam2_base.py:380-389). */
int s2h_row_gate(int dt, int64_t rows, int64_t inner, const void* x, const float* gate, float fill,
                 void* y, int dir, hipStream_t st);
/* s2h_row_gate with input type dt_in and output type dt_out (the low-res mask logits' cast to fp32
 * fused with the gate; its backward back to bf16); gate_out (nullable): gate[0:rows] copied. */
int s2h_row_gate_cast(int dt_in, int dt_out, int64_t rows, int64_t inner, const void* x, const float* gate,
                      float fill, void* y, int dir, float* gate_out, hipStream_t st);
/* y = (scale_x ? g*x : x) + (1-g)*vec for g = (gate > 0) (obj_ptr / no_obj_ptr mix,
 * sam2_base.py:413-424; no_obj_embed_spatial sam2_base.py:761-767). */
int s2h_gate_mix(int dt, int64_t rows, int64_t inner, const void* x, const float* gate, const void* vec,
                 int vec_period, int scale_x, void* y, hipStream_t st);
/* Hiera positional embedding: out[h, w, c] = Y[c, h, w] + win[c, h % ws, w % ws]
 * (bicubic-resized background + tiled window embedding, hieradet.py:273-281). */
int s2h_pos_embed(int dt, int C, int h, int w, int ws, const float* Y, const float* win, void* out,
                  hipStream_t st);
int s2h_pos_embed_bwd(int dt, int C, int h, int w, int ws, const void* dout, float* dY, float* dwin,
                      hipStream_t st);
/* Point prompt embedding: out[r] = pe[r] + table[label[r] + 1] (label -1 = pad:
 * table row 0 = not_a_point_embed, pe zeroed), prompt_encoder.py:79-104; labels_out (nullable):
 * the labels copied (kept for the backward). */
int s2h_point_embed(int dt, int R, int D, const float* pe, const int* labels, const void* table, void* out,
                    int* labels_out, hipStream_t st);
int s2h_point_embed_bwd(int dt, int R, int D, const int* labels, const void* dout, float* dtable, hipStream_t st);
/* the same with the 5 label rows' gradients at their own addresses (host array of 5 fp32 [D] rows:
 * not_a_point_embed, point_embeddings[0..3] -- the parameters' arena gradients), accumulated in row order. */
int s2h_point_embed_bwd_rows(int dt, int R, int D, const int* labels, const void* dout, float* const* drows,
                             hipStream_t st);

/* ---------------------------------------------------------------- loss + category merge
 * Per-row mask statistics of logits x/T vs uint8 targets: stats[6*r..] = (focal sum,
 * sigmoid sum, target sum, sigmoid.target sum, (x>0) & tgt count, (x>0) | tgt count).
 * sigmoid_focal_loss / dice_loss / iou_loss inputs, losses.py:20-76, 111-248. */
int s2h_mask_stats(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt,
                   float inv_temp, float* stats, hipStream_t st);
/* losses[4] = (loss_mask, loss_dice, loss_iou, weighted total) with per-frame
 * normalisation by valid categories (valid = NULL: target sum > 0); coef[3*N] are the
 * gradient coefficients consumed by s2h_mask_loss_bwd. */
int s2h_mask_loss_finalize(int N, int64_t P, const float* stats, const float* pred_iou, const int* valid,
                           float w_mask, float w_dice, float w_iou, float gscale, float* losses,
                           float* coef, hipStream_t st);
/* dx = d(total)/d(logits) * gtot[3] (device scalar upstream gradient); dious likewise. */
int s2h_mask_loss_bwd(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt,
                      float inv_temp, const float* coef, float* dx, int64_t lddx, const float* gtot,
                      float* dious, hipStream_t st);
/* BCECategoryLoss (losses.py:251-372, loss.type=bce): per-row stats[2*r..] = (sum of
 * binary_cross_entropy_with_logits(x/T, t, pos_weight[r]), target sum); pos_weight may be NULL. */
int s2h_bce_stats(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt,
                  float inv_temp, const float* pos_weight, float* stats, hipStream_t st);
/* losses[0] += frame_scale * (mean (reduction 0) or sum (1) over the rows with target pixels);
 * coef[N] are the backward coefficients. */
int s2h_bce_finalize(int N, int64_t P, const float* stats, int reduction, float frame_scale, float* losses,
                     float* coef, hipStream_t st);
/* dx = gtot[0] * d(loss)/d(logits) (gtot: device scalar upstream gradient, NULL = 1). */
int s2h_bce_bwd(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt, float inv_temp,
                const float* pos_weight, const float* coef, const float* gtot, float* dx, int64_t lddx,
                hipStream_t st);
/* Evaluation counts of one frame (eval/eval.py:16-40 caculate_iou / _dice / _mae on the
 * binarised category-merged mask pred = logits > 0): counts[4n..4n+3] = |pred & gt|,
 * |pred | gt|, |pred|, |gt| as uint64 (zeroed by the call).  Validation only, no gradient. */
int s2h_mask_eval_counts(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt,
                         uint64_t* counts, hipStream_t st);
/* Pixelwise max of each category's object masks (CSR cat_off / cat_obj), argmax
 * saved for the backward (merge_object_results_to_category, masks.py:98-115). */
int s2h_group_max_fwd(int Ncat, int64_t P, const int* cat_off, const int* cat_obj, const float* x,
                      int64_t ldx, float* y, int64_t ldy, int* arg, hipStream_t st);
int s2h_group_max_bwd(int O, int64_t P, const int* obj_cat, const int* arg, const float* dy, int64_t lddy,
                      float* dx, int64_t lddx, hipStream_t st);
/* Sigmoid-mass weighted mean of per-object scalars (IoU / object scores) per
 * category, weights = stats (masks.py:98-140); bwd also yields d(weights). */
int s2h_group_wavg_fwd(int Ncat, int K, const int* cat_off, const int* cat_obj, const float* stats,
                       const float* x, float* y, hipStream_t st);
int s2h_group_wavg_bwd(int O, int K, const int* obj_cat, const int* cat_off, const float* stats,
                       const float* x, const float* y, const float* dy, float* dx, float* dw, hipStream_t st);
/* dx[r, :] += coef[r] * sigmoid'(x[r, :]) (gradient of the sigmoid-mass weights). */
int s2h_sigmoid_grad_axpy(int R, int64_t P, const float* x, int64_t ldx, const float* coef, float* dx,
                          int64_t lddx, hipStream_t st);

/* ---------------------------------------------------------------- optimizer
 * Global L2 norm of the flat fp32 gradient arena (times grad_scale) and the clip
 * factor: out[0] = norm, out[1] = min(1, max_norm / (norm + 1e-6)) * grad_scale.
 * partial_ws: fp32 workspace of >= 1024 floats.  Replaces gradient_clip_val
 * (torch clip_grad_norm_, configured at trainer / best.yaml:106). */
int s2h_grad_norm(int64_t n, const float* g, float* partial_ws, float max_norm, float grad_scale,
                  float* out, hipStream_t st);
/* Fused AdamW over the flat arena (torch.optim.AdamW semantics, trainer.py:125):
 * g' = g*clip[1]; p *= 1 - lr*wd; m = b1 m + (1-b1) g'; v = b2 v + (1-b2) g'^2;
 * p -= lr/(1-b1^step) * m / (sqrt(v)/sqrt(1-b2^step) + eps); optional bf16 shadow copy. */
int s2h_adamw(int64_t n, float* p, const float* g, float* m, float* v, const float* clip, float lr,
              float beta1, float beta2, float eps, float wd, int step, void* bf16_shadow, hipStream_t st);

/* ---------------------------------------------------------------- prompt stage (host CPU code)
 * The per-step host work of prepare_prompt_inputs (sam2model.py:181-236) on frame 0, native and
 * multi-threaded (one thread per category, `threads` at most); no device calls.
 * s2h_prompt_objects replaces cat_to_obj_mask + find_connected_components (masks.py:13-50, the
 * cv2 5x5-ellipse opening + 8-connected components): N category masks [N, H, W] of 0/1 bytes ->
 * objects numbered category-major, raster order of first pixel within a category; obj_cat[o],
 * stats[o * 7 ..] = (count, sum_y, sum_x, y_min, y_max, x_min, x_max), optional lab[N, H, W] =
 * 1 + object index (0 background).  Returns 0, 2 with *n_obj = the count needed when it
 * exceeds max_obj, 1 on bad arguments.
 * s2h_prompt_object_masks: lab -> float object masks [n_obj, H, W] (cat_to_obj_mask's output).
 * s2h_mask_moments: the same 7 moments of B whole masks [B, H, W] -- the centre-of-mass click of
 * generate_point_prompt (prompts.py:13-75) and the corners of generate_box_prompt (prompts.py:78-97). */
int s2h_prompt_objects(int N, int H, int W, const uint8_t* masks, int max_obj, int* n_obj, int32_t* obj_cat,
                       int64_t* stats, int32_t* lab, int threads);
int s2h_prompt_object_masks(int N, int H, int W, const int32_t* lab, int n_obj, float* out, int threads);
int s2h_mask_moments(int B, int H, int W, const uint8_t* masks, int64_t* stats, int threads);

#ifdef __cplusplus
}
#endif

#endif /* SAM2HIP_H */
