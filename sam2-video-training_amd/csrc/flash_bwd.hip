// Flash attention backward for the long-sequence bf16 attentions (the partner of flash.hip):
// memory-attention RoPE self / cross attention (transformer.py:275-311, head_dim 256).
//
// P is recomputed from Q, K and the forward's LSE; dropout masks are regenerated from the
// same counter hash.  Three kernels, no atomics:
//   * Di = rowsum(dO * O)                                 (inside the dQ kernel)
//   * dQ:  per 128-query block, K / V tiles streamed by LDS-DMA exactly like the forward;
//          S^T = K Q^T and dP^T = V dO^T keep the query on the lane, so P, dS are
//          lane-local; dQ^T += K^T dS^T with K^T fragments from transposing LDS reads.
//          The key range is split over workgroups when the query blocks cannot fill the
//          chip; fp32 partials are summed (and scaled, cast) by a combine kernel.
//   * dK / dV: per 128-key block (8 waves x 16 keys, K and V fragments held in registers),
//          Q / dO tiles of 32 queries streamed by LDS-DMA; S = Q K^T and dP = dO V^T keep
//          the key on the lane, so P_drop and dS are already the B operands of
//          dV^T += dO^T P_drop and dK^T += Q^T dS (dO^T / Q^T by transposing reads).
// V-fold (DV != DP, s2h_flash_bwd_frames_vfold; the forward's flash.hip header): the memory bank M
// (64 wide) stands in for V = M Wv^T + bv and the upstream gradient arrives as
// du' = dO [Wv | bv] = [dO Wv | dO . bv] (72 columns): dD = du M^T + dr (dr = du'[:, 64]),
// Di = rowsum(dO * O) = du . u + dr * rowsum(D) from u' = [D M | rowsum(D)].  No dV: the bank is
// detached (sam2model.py:345-358) and the value projection's weight gradient is dO^T u'.
#include <type_traits>

#include "flash_common.h"

int s2h_prof_begin(hipStream_t st, int kind, int64_t m0, int64_t m1, int64_t m2, int64_t m3, int64_t m4);
int s2h_flash_variant();  // flash.hip: A/B selection of older kernels
int s2h_flash_v2();       // flash.hip: round-6 A/B bits (s2h_flash_variant2)
void s2h_prof_end(int slot, hipStream_t st);

struct FlashBwdArgs {
  int BH, H, Lq, Lk;
  int D;  // head dim (<= DP: head dims <= 64 run in a 64 image, zero operand columns past D)
  const bf16* q; int64_t sqb, sqh, sql;
  const bf16* k; int64_t skb, skh, skl;
  const bf16* v; int64_t svb, svh, svl;
  const bf16* o; int64_t sob, soh, sol;
  const bf16* g; int64_t sgb, sgh, sgl;  // dO
  bf16* dq; int64_t sdqb, sdqh, sdql;
  bf16* dk; int64_t sdkb, sdkh, sdkl;
  bf16* dv; int64_t sdvb, sdvh, sdvl;
  const float* lse;  // [BH*Lq] natural log
  float* di;         // [BH*Lq] rowsum(dO*O)
  float scale, sl2;
  float p_drop; uint32_t thresh; float inv_keep; uint64_t seed; const uint64_t* seed_off;
  int splits, tiles_per_split;
  float* ws_dq;  // [splits][BH*Lq][DP] fp32 partial dQ (splits > 1)
  int kv_splits, kv_tiles_per_split;  // dK/dV kernel: query range split over workgroups
  float* ws_dkv;  // [kv_splits][BH*Lk][2][DP] fp32 partial (dK, dV) (kv_splits > 1)
  uint64_t idx0;  // dropout element-index offset (single-frame launches)
  // dropout keep bitmap of the forward (nullable; flash.hip layout: bit (k & 31) of word
  // [(bh * Lq + q) * kw + k / 32]); read instead of re-hashing every element
  const uint32_t* keep; int kw;
  // Frame table (nfr > 0): the batch is nfr frames x bpf batches, Q / O / dO / dQ / LSE uniform,
  // K / V / dK / dV PACKED per frame: batch bl of frame f has fr_lk[f] keys starting at row
  // fr_krow[f] + bl * fr_lk[f]; dropout indices of frame f start at fr_idx0[f] (the offsets its
  // forward launch used).  One launch covers the frame-batched backward of every frame.
  int nfr, bpf;
  int fr_lk[S2H_MAX_FRAMES];
  int64_t fr_krow[S2H_MAX_FRAMES];
  uint64_t fr_idx0[S2H_MAX_FRAMES];
  int64_t fr_koff[S2H_MAX_FRAMES];  // word offset of frame f's keep bitmap
  // optional inverse RoPE of dQ / dK (s2h_flash_bwd_frames_rope: dQ; s2h_flash_bwd_frames_vfold_rope_qk;
  // head dim 256, frame-table launches): with rope_k, key rows < fr_nrot[f] of every batch block are
  // rotated back with table row key % rope_period (the k projection's RoPE epilogue, transposed);
  // with rope_q, query rows < fr_nrotq[f] the same way (the q projection's).  Tables [period][D / 2].
  const float* rope_cos; const float* rope_sin; int rope_period;
  int rope_k, rope_q;
  int fr_nrot[S2H_MAX_FRAMES];
  int fr_nrotq[S2H_MAX_FRAMES];
  int prio;  // bit 0: dK kernel, bit 1: dQ kernel -- waves 4-7 at s_setprio 1 (A/B: s2h_flash_variant bits 1-2)
};

// The frame table is read straight from the kernarg segment (scalar loads): indexing the by-value
// argument's arrays with a runtime frame made the compiler copy the whole struct (1.3 KB) into
// per-lane scratch at every kernel start.
typedef __attribute__((address_space(4))) const FlashBwdArgs KFlashBwdArgs;
__device__ __forceinline__ KFlashBwdArgs* kargs() { return (KFlashBwdArgs*)__builtin_amdgcn_kernarg_segment_ptr(); }

// K / V / dK / dV bases, key count and dropout index base (query 0) of batch-head bh
struct KvFrame {
  const bf16* k; const bf16* v; bf16* dk; bf16* dv;
  int Lk;
  uint64_t drow0;
  const uint32_t* keep;  // keep bitmap of query 0 of this batch-head (nullptr: hash)
  int kw;                // its words per query row
};
__device__ __forceinline__ KvFrame kv_frame(const FlashBwdArgs& a, int bh) {
  const int b = bh / a.H, h = bh % a.H;
  KvFrame r;
  if (a.nfr > 0) {
    const int f = b / a.bpf, bl = b - f * a.bpf;
    KFlashBwdArgs* ka = kargs();
    r.Lk = ka->fr_lk[f];
    const int64_t row = ka->fr_krow[f] + (int64_t)bl * r.Lk;
    r.k = a.k + row * a.skl + h * a.skh;
    r.v = a.v + row * a.svl + h * a.svh;
    r.dk = a.dk + row * a.sdkl + h * a.sdkh;
    r.dv = a.dv + row * a.sdvl + h * a.sdvh;
    r.drow0 = ka->fr_idx0[f] + (uint64_t)(bl * a.H + h) * (uint64_t)a.Lq * (uint64_t)r.Lk;
    r.kw = 2 * ((r.Lk + 63) / 64);
    r.keep = a.keep ? a.keep + ka->fr_koff[f] + (int64_t)(bl * a.H + h) * a.Lq * r.kw : nullptr;
  } else {
    r.Lk = a.Lk;
    r.k = a.k + b * a.skb + h * a.skh;
    r.v = a.v + b * a.svb + h * a.svh;
    r.dk = a.dk + b * a.sdkb + h * a.sdkh;
    r.dv = a.dv + b * a.sdvb + h * a.sdvh;
    r.drow0 = a.idx0 + (uint64_t)bh * (uint64_t)a.Lq * (uint64_t)a.Lk;
    r.kw = a.kw;
    r.keep = a.keep ? a.keep + (int64_t)bh * a.Lq * a.kw : nullptr;
  }
  return r;
}

// the RoPE table row of gradient row `row` when it is rotated (row < nrot), else nullptr
__device__ __forceinline__ const float* rope_row(const FlashBwdArgs& a, int row, int nrot, const float* tab) {
  if (row >= nrot) return nullptr;
  return tab + (int64_t)(row % a.rope_period) * (a.D / 2);
}

// the table entries of the 4 consecutive gradient columns c0..c0+3 (2 rotation pairs, c0 % 4 == 0):
// one 8-B load per table.  Store loops load every entry they need BEFORE their first store (a load
// after a global store waits for it: vmcnt counts both).  What remains is one exposed table-load
// latency per workgroup (these kernels run one workgroup per CU): +13..15 us per launch of the
// 1664-workgroup dQ kernels, about what the separate rotation launch cost (profiles/r05_v29-v30;
// an L2 warm-up at kernel start did not change it, holding the entries from kernel start spilled)
struct RopeCS { float2 c, s; };
__device__ __forceinline__ RopeCS rope_load(const float* rc, const float* rsn, int c0) {
  return RopeCS{*(const float2*)(rc + c0 / 2), *(const float2*)(rsn + c0 / 2)};
}
// the inverse rotation (the projection epilogue's, transposed) of those 4 columns
__device__ __forceinline__ void rope_apply(float (&v)[4], const RopeCS& t) {
  const float cs[2] = {t.c.x, t.c.y}, sns[2] = {t.s.x, t.s.y};
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float c = cs[j], sn = sns[j], x0 = v[2 * j], x1 = v[2 * j + 1];
    v[2 * j] = x0 * c + x1 * sn;
    v[2 * j + 1] = x1 * c - x0 * sn;
  }
}

// dropout handling of the backward kernels (a template parameter: a runtime test per element
// made the compiler branch around every element's exp2 / hash, SALU + exec churn in the loop)
enum { DROP_NONE = 0, DROP_BITS = 1, DROP_HASH = 2 };

// ------------------------------------------------------------------ dQ
// NSB: stages in the K / V ring (2, or 3: a tile in flight across the next one's compute, one barrier
// per tile); PF: LDS fragment reads kept ahead of their MFMAs in the S / dP phase.
template <int DP, int DROP, int DV = DP, int NSB = 2, int PF = 4>
__global__ __launch_bounds__(FL_WAVES * 64, 1) void flash_bwd_dq_kernel(FlashBwdArgs a) {
  static_assert(NSB == 2 || NSB == 3, "ring depth");
  constexpr bool FOLD = DV != DP;
  const uint64_t seed = DROP == DROP_HASH ? s2h_seed(a.seed, a.seed_off) : 0;
  using C = FlashCfg<DP, 64>;
  using I = PadImg<DP>;   // padded K image (the forward's: conflict-free b128 and transposing reads)
  using IV = PadImg<DV>;  // padded V image (V-fold: memory rows)
  constexpr int NTV = DV / 32;  // 32-deep d steps of dP
  constexpr int STG = I::TILEB + IV::TILEB;
  // [stage][K | V] + [stage][wave][16 queries x 2 keep words]
  __shared__ __attribute__((aligned(1024))) char smem[NSB * STG + NSB * FL_WAVES * 256];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, ql = lane & 15;
  if ((a.prio & 2) && w >= 4) __builtin_amdgcn_s_setprio(1);
  const WgIdx wi = wg_xcd_order();
  if (wi.y >= a.BH) return;  // grid padding
  const int bh = wi.y, b = bh / a.H, h = bh % a.H;
  const int split = wi.z;
  const int q = wi.x * FL_QB + w * 16 + ql;
  const bf16* Q = a.q + b * a.sqb + h * a.sqh;
  const bf16* G = a.g + b * a.sgb + h * a.sgh;
  const KvFrame fr = kv_frame(a, bh);
  const bf16* K = fr.k;
  const bf16* V = fr.v;
  const int Lk = fr.Lk;
  const int ntiles_all = (Lk + C::KT - 1) / C::KT;
  const int t0 = split * a.tiles_per_split;
  const int nt = min(ntiles_all, t0 + a.tiles_per_split) - t0;
  // keep words of this wave's 16 queries for the 64 keys of a tile: lane 2i + j (< 32) fetches
  // word j of query i (lanes 32..63 repeat them); LDS holds them as one uint2 per query
  constexpr bool bits = DROP == DROP_BITS;
  const uint32_t* KEEPQ = bits ? fr.keep + (int64_t)min(wi.x * FL_QB + w * 16 + ((lane >> 1) & 15), a.Lq - 1) * fr.kw
                               : nullptr;
  char* bits_lds = smem + NSB * STG + w * 256;
  const int npw = I::pieces(w), npv = IV::pieces(w);
  auto dma_bits = [&](int stage, int k0) { lds_dma4(KEEPQ + (k0 >> 5) + (lane & 1), bits_lds + stage * FL_WAVES * 256); };

  if (nt > 0) {
    dma_tile_pad<DP, 64, FL_WAVES, true>(smem, K, a.skl, t0 * C::KT, Lk, w, lane, a.D);
    dma_tile_pad<DV, 64, FL_WAVES, true>(smem + I::TILEB, V, a.svl, t0 * C::KT, Lk, w, lane, FOLD ? DV : a.D);
    if constexpr (bits) dma_bits(0, t0 * C::KT);
  }
  if (NSB == 3 && nt > 1) {
    dma_tile_pad<DP, 64, FL_WAVES, true>(smem + STG, K, a.skl, (t0 + 1) * C::KT, Lk, w, lane, a.D);
    dma_tile_pad<DV, 64, FL_WAVES, true>(smem + STG + I::TILEB, V, a.svl, (t0 + 1) * C::KT, Lk, w, lane, FOLD ? DV : a.D);
    if constexpr (bits) dma_bits(1, (t0 + 1) * C::KT);
  }
  const bool qv = q < a.Lq;
  bf16x8 qf[C::NT], gf[NTV];
#pragma unroll
  for (int t = 0; t < C::NT; ++t) {
    const bool ok = qv && 32 * t + 8 * g < a.D;  // zero past the head dim
    qf[t] = ok ? *(const bf16x8*)(Q + (int64_t)q * a.sql + 32 * t + 8 * g) : bf16x8{};
  }
#pragma unroll
  for (int t = 0; t < NTV; ++t) {
    const bool ok = qv && (FOLD || 32 * t + 8 * g < a.D);
    gf[t] = ok ? *(const bf16x8*)(G + (int64_t)q * a.sgl + 32 * t + 8 * g) : bf16x8{};
  }
  // V-fold: dr = du'[q, DV] (dO . bv), constant over the keys of the row
  const float dr = FOLD && qv ? (float)G[(int64_t)q * a.sgl + DV] : 0.f;
  const float lse2 = qv ? a.lse[(int64_t)bh * a.Lq + q] * FL_LOG2E : 0.f;
  // Di = rowsum(dO * O) of this lane's query from the dO fragments already in registers and the
  // matching O fragments, reduced over the 4 lanes (g) of the query: replaces a separate
  // one-wave-per-row pass over O and dO.  Split 0 stores it for the dK/dV kernel that follows.
  float di = 0.f;
  {
    const bf16* O = a.o + b * a.sob + h * a.soh;
#pragma unroll
    for (int t = 0; t < NTV; ++t) {
      if (qv && (FOLD || 32 * t + 8 * g < a.D)) {
        const bf16x8 of = *(const bf16x8*)(O + (int64_t)q * a.sol + 32 * t + 8 * g);
#pragma unroll
        for (int j = 0; j < 8; ++j) di += (float)gf[t][j] * (float)of[j];
      }
    }
    di += __shfl_xor(di, 16, 64);
    di += __shfl_xor(di, 32, 64);
    if constexpr (FOLD) {  // + dr * rowsum(D)
      if (qv) di += dr * (float)O[(int64_t)q * a.sol + DV];
    }
  }
  // compiler-visible vmcnt(0): the compiler's own bookkeeping retires these loads here instead
  // of waiting vmcnt(0) inside the key loop (which would also drain the asm K/V prefetch)
  __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0) expcnt(7) lgkmcnt(15)
  if (split == 0 && g == 0 && qv) a.di[(int64_t)bh * a.Lq + q] = di;
  f32x4 acc[C::ND];  // dQ^T: row d = 16*db + 4g + r, column q
#pragma unroll
  for (int d = 0; d < C::ND; ++d) acc[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint64_t drow = fr.drow0 + (uint64_t)q * (uint64_t)Lk;

  int cur = 0;  // it % NSB
  for (int it = 0; it < nt; ++it) {
    const int k0 = (t0 + it) * C::KT;
    char* Kb = smem + cur * STG;
    char* Vb = Kb + I::TILEB;
    const int bstage = cur;
    // this wave's pieces of tile `it` have landed once all but one later tile's retired
    auto wait_one_ahead = [&]() {
      if constexpr (bits) wait_kv_pieces<I::PPW_LO + 1, IV::PPW_LO>(npw + 1, npv);
      else wait_kv_pieces<I::PPW_LO, IV::PPW_LO>(npw, npv);
    };
    auto issue = [&](int stage, int kk) {
      char* Kn = smem + stage * STG;
      dma_tile_pad<DP, 64, FL_WAVES, true>(Kn, K, a.skl, kk, Lk, w, lane, a.D);
      dma_tile_pad<DV, 64, FL_WAVES, true>(Kn + I::TILEB, V, a.svl, kk, Lk, w, lane, FOLD ? DV : a.D);
      if constexpr (bits) dma_bits(stage, kk);
    };
    if constexpr (NSB == 2) {
      if (it + 1 < nt) {
        issue(cur ^ 1, k0 + C::KT);
        wait_one_ahead();
      } else {
        wait_vmcnt<0>();
      }
      wg_barrier();
    } else {
      // tile it + 1 stays in flight across this one; tile it + 2 goes after the barrier into the
      // buffer every wave finished reading in iteration it - 1
      if (it + 1 < nt) wait_one_ahead();
      else wait_vmcnt<0>();
      wg_barrier();
      if (it + 2 < nt) issue(cur == 0 ? 2 : cur - 1, k0 + 2 * C::KT);
    }
    cur = cur == NSB - 1 ? 0 : cur + 1;

    f32x4 s[4], dp[4];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int row = kb * 16 + ql;
#pragma unroll
      for (int t = 0; t < C::NT; ++t) {
        const bf16x8 kf = *(const bf16x8*)(Kb + row * I::ROWB + 16 * (4 * t + g));
        s[kb] = mfma16(kf, qf[t], s[kb]);
        if (t < NTV) {
          const bf16x8 vf = *(const bf16x8*)(Vb + row * IV::ROWB + 16 * (4 * t + g));
          dp[kb] = mfma16(vf, gf[t], dp[kb]);
        }
      }
    }
    sched_reads_ahead<4 * (C::NT + (NTV < C::NT ? NTV : C::NT)), PF, 1>();
    __builtin_amdgcn_sched_barrier(0);
    const bool full = k0 + C::KT <= Lk;
    uint32_t kwords[2] = {0u, 0u};
    if constexpr (bits) {
      const uint2 t2 = *(const uint2*)(bits_lds + bstage * FL_WAVES * 256 + ql * 8);
      kwords[0] = t2.x;
      kwords[1] = t2.y;
    }
    // the key-tail test as a separate code path: an in-line `if (!full)` compiled to a compare and a
    // select per element on every tile (31 of the loop's 276 VALU instructions, gfx950 ISA)
    auto softmax = [&](auto tail) {
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) {
        bool kp[4] = {true, true, true, true};
        if constexpr (bits) {
          const uint32_t wd = kwords[kb >> 1] >> (16 * (kb & 1) + 4 * g);
#pragma unroll
          for (int e = 0; e < 4; ++e) kp[e] = (wd >> e) & 1u;
        } else if constexpr (DROP == DROP_HASH) {
          const uint64_t e0 = drow + k0 + kb * 16 + 4 * g;
          if ((e0 & 1) == 0) {
            s2h_keep_pair(seed, e0 >> 1, a.thresh, kp[0], kp[1]);
            s2h_keep_pair(seed, (e0 >> 1) + 1, a.thresh, kp[2], kp[3]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) kp[e] = s2h_keep(seed, e0 + e, a.thresh);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = __builtin_amdgcn_exp2f(s[kb][r] * a.sl2 - lse2);
          if constexpr (decltype(tail)::value) p = (k0 + kb * 16 + 4 * g + r < Lk) ? p : 0.f;
          const float dpr = FOLD ? dp[kb][r] + dr : dp[kb][r];
          if constexpr (DROP == DROP_NONE) {
            s[kb][r] = p * (dpr - di);  // dS (scale applied at the end)
          } else {
            const float dpd = kp[r] ? dpr : 0.f;
            s[kb][r] = p * fmaf(dpd, a.inv_keep, -di);
          }
        }
      }
    };
    if (full) softmax(std::false_type{});
    else softmax(std::true_type{});
    bf16x8 dsb[2];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) dsb[c][j] = (bf16)s[2 * c + (j >> 2)][j & 3];
    // dQ^T += K^T dS^T
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int d = 0; d < C::ND; ++d) acc[d] = mfma16(tr_frag_pad<I::ROWB>(Kb, 32 * c, 16 * d, lane), dsb[c], acc[d]);
    sched_reads_ahead<2 * C::ND, 4, 2>();
    __builtin_amdgcn_sched_barrier(0);

    if constexpr (NSB == 2) {  // every wave's reads of this stage retired before it is refilled
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wg_barrier();
    }
  }

  if (!qv) return;
  if (a.splits == 1) {
    bf16* DQ = a.dq + b * a.sdqb + h * a.sdqh + (int64_t)q * a.sdql;
    // inverse RoPE of the query gradient (frame-table launches, rope_q)
    const int nrq = a.rope_q ? (a.nfr > 0 ? kargs()->fr_nrotq[b / a.bpf] : a.Lq) : 0;
    const float* rc = rope_row(a, q, nrq, a.rope_cos);
    const float* rsn = rope_row(a, q, nrq, a.rope_sin);
    RopeCS tab[C::ND];
    if (rc != nullptr) {
#pragma unroll
      for (int d = 0; d < C::ND; ++d) tab[d] = rope_load(rc, rsn, min(16 * d + 4 * g, a.D - 4));
    }
#pragma unroll
    for (int d = 0; d < C::ND; ++d) {
      if (16 * d + 4 * g >= a.D) continue;
      float v4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v4[e] = acc[d][e] * a.scale;
      if (rc != nullptr) rope_apply(v4, tab[d]);
      bf16 t4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) t4[e] = (bf16)v4[e];
      *(uint2*)(DQ + 16 * d + 4 * g) = *(const uint2*)t4;
    }
  } else {
    float* W = a.ws_dq + ((int64_t)split * a.BH * a.Lq + (int64_t)bh * a.Lq + q) * DP;
#pragma unroll
    for (int d = 0; d < C::ND; ++d) *(float4*)(W + 16 * d + 4 * g) = float4{acc[d][0], acc[d][1], acc[d][2], acc[d][3]};
  }
}

template <int DP>
__global__ __launch_bounds__(256) void flash_bwd_dq_combine_kernel(FlashBwdArgs a) {
  const int64_t rows = (int64_t)a.BH * a.Lq;
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;  // 4 consecutive d
  if (i >= rows * DP) return;
  const int64_t row = i / DP;
  const int d = i % DP;
  float4 s = *(const float4*)(a.ws_dq + i);
  for (int sp = 1; sp < a.splits; ++sp) {
    const float4 t = *(const float4*)(a.ws_dq + sp * rows * DP + i);
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  }
  if (d >= a.D) return;
  const int bh = row / a.Lq, q = row % a.Lq, b = bh / a.H, h = bh % a.H;
  bf16 t4[4] = {(bf16)(s.x * a.scale), (bf16)(s.y * a.scale), (bf16)(s.z * a.scale), (bf16)(s.w * a.scale)};
  *(uint2*)(a.dq + b * a.sdqb + h * a.sdqh + (int64_t)q * a.sdql + d) = *(const uint2*)t4;
}

// ------------------------------------------------------------------ dK / dV
// head_dim 72..128 in a 128 image, or 32..64 in a 64 image (Hiera, hieradet.py:56-81; B+ 56, L 72):
// 8 waves x 16 keys, K / V
// fragments in registers; Q / dO tiles of QT queries (64 for the 64 image: a 32-row tile would be
// half a DMA piece per wave) consumed in 32-query halves.
template <int DP, int DROP>
__global__ __launch_bounds__(FL_WAVES * 64, 1) void flash_bwd_dkv_kernel(FlashBwdArgs a) {
  const uint64_t seed = DROP == DROP_HASH ? s2h_seed(a.seed, a.seed_off) : 0;
  constexpr int QT = DP == 64 ? 64 : 32;
  using C = FlashCfg<DP, QT>;
  __shared__ __attribute__((aligned(1024))) char smem[2 * 2 * C::TILEB];  // [stage][Q | dO]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, kl = lane & 15;
  const WgIdx wi = wg_xcd_order();
  if (wi.y >= a.BH) return;  // grid padding
  const int bh = wi.y, b = bh / a.H, h = bh % a.H;
  const int key = wi.x * FL_QB + w * 16 + kl;  // this lane's key (B-operand column)
  const KvFrame fr = kv_frame(a, bh);
  if (wi.x * FL_QB >= fr.Lk) return;  // frame-table launch: past this frame's keys
  const bool kv = key < fr.Lk;
  const bf16* Q = a.q + b * a.sqb + h * a.sqh;
  const bf16* G = a.g + b * a.sgb + h * a.sgh;
  const bf16* K = fr.k;
  const bf16* V = fr.v;
  const int nt = (a.Lq + QT - 1) / QT;

  dma_tile<DP, QT, FL_WAVES, true>(smem, Q, a.sql, 0, a.Lq, w, lane, a.D);
  dma_tile<DP, QT, FL_WAVES, true>(smem + C::TILEB, G, a.sgl, 0, a.Lq, w, lane, a.D);
  bf16x8 kf[C::NT], vf[C::NT];  // B operands: K^T / V^T [k = d][n = key]; zero past the head dim
#pragma unroll
  for (int t = 0; t < C::NT; ++t) {
    const bool ok = kv && 32 * t + 8 * g < a.D;
    kf[t] = ok ? *(const bf16x8*)(K + (int64_t)key * a.skl + 32 * t + 8 * g) : bf16x8{};
    vf[t] = ok ? *(const bf16x8*)(V + (int64_t)key * a.svl + 32 * t + 8 * g) : bf16x8{};
  }
  // compiler-visible vmcnt(0) for the fragment loads (see the dQ kernel)
  __builtin_amdgcn_s_waitcnt(0xF70);
  f32x4 dk[C::ND], dv[C::ND];  // dK^T / dV^T: row d = 16*db + 4g + r, column key
#pragma unroll
  for (int d = 0; d < C::ND; ++d) {
    dk[d] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float* LSE = a.lse + (int64_t)bh * a.Lq;
  const float* DI = a.di + (int64_t)bh * a.Lq;

  for (int it = 0; it < nt; ++it) {
    const int q0 = it * QT;
    char* Qb = smem + (it & 1) * 2 * C::TILEB;
    char* Gb = Qb + C::TILEB;
    // this tile's queries of this lane: q0 + 32*hf + 16*qb + 4g + r  (hf < QT/32; qb = 0, 1; r = 0..3)
    float4 lse4[QT / 16], di4[QT / 16];
#pragma unroll
    for (int qb = 0; qb < QT / 16; ++qb) {
      const int qr = q0 + 16 * qb + 4 * g;
      if (qr + 3 < a.Lq && (a.Lq & 3) == 0) {
        lse4[qb] = *(const float4*)(LSE + qr);
        di4[qb] = *(const float4*)(DI + qr);
      } else {
        float lt[4], dt[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          lt[e] = qr + e < a.Lq ? LSE[qr + e] : INFINITY;  // exp2(-inf) = 0: padded queries drop out
          dt[e] = qr + e < a.Lq ? DI[qr + e] : 0.f;
        }
        lse4[qb] = float4{lt[0], lt[1], lt[2], lt[3]};
        di4[qb] = float4{dt[0], dt[1], dt[2], dt[3]};
      }
    }
    if (it + 1 < nt) {
      char* Qn = smem + ((it + 1) & 1) * 2 * C::TILEB;
      dma_tile<DP, QT, FL_WAVES, true>(Qn, Q, a.sql, q0 + QT, a.Lq, w, lane, a.D);
      dma_tile<DP, QT, FL_WAVES, true>(Qn + C::TILEB, G, a.sgl, q0 + QT, a.Lq, w, lane, a.D);
      wait_vmcnt<2 * C::PPW>();
    } else {
      wait_vmcnt<0>();
    }
    wg_barrier();

#pragma unroll
    for (int hf = 0; hf < QT / 32; ++hf) {
      f32x4 s[2], dp[2];  // S / dP: row q = 32*hf + 16*qb + 4g + r, column key
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        s[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
        dp[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
        const int row = 32 * hf + qb * 16 + kl;
#pragma unroll
        for (int t = 0; t < C::NT; ++t) {
          const bf16x8 qa = *(const bf16x8*)(Qb + swz<DP>(row, 4 * t + g));
          s[qb] = mfma16(qa, kf[t], s[qb]);
          const bf16x8 ga = *(const bf16x8*)(Gb + swz<DP>(row, 4 * t + g));
          dp[qb] = mfma16(ga, vf[t], dp[qb]);
        }
      }
      sched_reads_ahead<4 * C::NT, 4, 1>();
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 pdb, dsb;  // B operands over 32 queries: k index 8g + j <-> q 16(j>>2) + 4g + (j&3)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const float4 l4 = lse4[2 * hf + qb], d4 = di4[2 * hf + qb];
        const float lt[4] = {l4.x, l4.y, l4.z, l4.w};
        const float dt[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __builtin_amdgcn_exp2f(s[qb][r] * a.sl2 - lt[r] * FL_LOG2E);
          if constexpr (DROP == DROP_NONE) {
            pdb[4 * qb + r] = (bf16)p;
            dsb[4 * qb + r] = (bf16)(p * (dp[qb][r] - dt[r]));
          } else {
            const int qi = q0 + 32 * hf + 16 * qb + 4 * g + r;
            const bool keep = s2h_keep(seed, fr.drow0 + (uint64_t)qi * (uint64_t)fr.Lk + key, a.thresh);
            const float pd = keep ? p * a.inv_keep : 0.f;
            const float dpd = keep ? dp[qb][r] * a.inv_keep : 0.f;
            pdb[4 * qb + r] = (bf16)pd;
            dsb[4 * qb + r] = (bf16)(p * (dpd - dt[r]));
          }
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int d = 0; d < C::ND; ++d) {
        dv[d] = mfma16(tr_frag_perm<DP>(Gb, 32 * hf, 16 * d, lane), pdb, dv[d]);
        dk[d] = mfma16(tr_frag_perm<DP>(Qb, 32 * hf, 16 * d, lane), dsb, dk[d]);
      }
      sched_reads_ahead<2 * C::ND, 4, 2>();
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    wg_barrier();
  }

  if (!kv) return;
  bf16* DK = fr.dk + (int64_t)key * a.sdkl;
  bf16* DV = fr.dv + (int64_t)key * a.sdvl;
#pragma unroll
  for (int d = 0; d < C::ND; ++d) {
    if (16 * d + 4 * g >= a.D) continue;
    bf16 tk[4], tv[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      tk[e] = (bf16)(dk[d][e] * a.scale);
      tv[e] = (bf16)dv[d][e];
    }
    *(uint2*)(DK + 16 * d + 4 * g) = *(const uint2*)tk;
    *(uint2*)(DV + 16 * d + 4 * g) = *(const uint2*)tv;
  }
}

// dK / dV for head_dim 256: 16-wide MFMAs would need K, V fragments (64) + dK^T, dV^T
// (128) + S, dP registers beyond 256 per wave, so this form runs one wave per SIMD with
// the 512-register file: 4 waves x 32 keys on v_mfma_f32_32x32x16_bf16 (also half the LDS
// operand traffic per FLOP), dK^T / dV^T in 2 x 128 accumulator registers.
// KREG: K fragments held in registers like V (64 more VGPRs, no K block in LDS): the S / dP
// phase re-read the constant K block from LDS every 32-query tile -- a third of that phase's
// LDS traffic, and the phase is LDS-bandwidth-bound (4 waves x 48 b128 reads against 32 MFMAs).
// NSB: stages of the Q / dO ring -- 2 (two barriers per tile), 3 (one barrier per tile, tile it + 1
// in flight across tile it; the dkv16 / dQ kernels' round-6 ring)
template <int DP, int DROP, bool KREG = true, int DV = DP, int NSB = 2>
__global__ __launch_bounds__(256, 1) void flash_bwd_dkv32_kernel(FlashBwdArgs a) {
  static_assert(NSB == 2 || NSB == 3, "ring depth");
  constexpr bool FOLD = DV != DP;  // V-fold: dO tile = du' (DV wide + dr), no dV
  const uint64_t seed = DROP == DROP_HASH ? s2h_seed(a.seed, a.seed_off) : 0;
  constexpr int NWV = 4, QT = 32;
  using C = FlashCfg<DP, QT, NWV>;
  using CG = FlashCfg<DV, QT, NWV>;  // dO (du') tile
  constexpr int SWG = DV >= 128 ? 1 : 0;
  constexpr int NT = DP / 16, ND = DP / 32, NTV = DV / 16;
  // [K block: 128 keys (!KREG)][stage][Q | dO] + [stage][wave][lse(32) | Di(32)] (each wave DMAs
  // its own copy of the row constants).  V (and with KREG, K) live in registers.
  using CK = FlashCfg<DP, NWV * 32, NWV>;
  constexpr int RWB = FOLD ? 768 : 512;  // per wave [lse | Di | keep words (x2) | dr words (x2, V-fold)]
  constexpr int STAGE = C::TILEB + CG::TILEB + NWV * RWB;
  constexpr int KBLK = KREG ? 0 : CK::TILEB;
  __shared__ __attribute__((aligned(1024))) char smem[KBLK + NSB * STAGE];
  char* Kblk = smem;
  char* stages = smem + KBLK;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, hi = lane >> 5, kl = lane & 31;
  const WgIdx wi = wg_xcd_order();
  if (wi.y >= a.BH) return;  // grid padding
  const int bh = wi.y, b = bh / a.H, h = bh % a.H;
  const int key = wi.x * (NWV * 32) + w * 32 + kl;
  const KvFrame fr = kv_frame(a, bh);
  if (wi.x * (NWV * 32) >= fr.Lk) return;  // frame-table launch: past this frame's keys
  const bool kv = key < fr.Lk;
  const bf16* Q = a.q + b * a.sqb + h * a.sqh;
  const bf16* G = a.g + b * a.sgb + h * a.sgh;
  const bf16* K = fr.k;
  const bf16* V = fr.v;
  // query tiles [qt0, qt0 + nt) of this workgroup (kv_splits > 1: partial dK / dV)
  const int nt_all = (a.Lq + QT - 1) / QT;
  const int qt0 = wi.z * a.kv_tiles_per_split;
  const int nt = max(0, min(nt_all, qt0 + a.kv_tiles_per_split) - qt0);
  const int qbase = qt0 * QT;

  const float* LSE = a.lse + (int64_t)bh * a.Lq;
  const float* DI = a.di + (int64_t)bh * a.Lq;
  // one 4-B-per-lane DMA per stage: lanes 0..31 lse[q0 + lane], lanes 32..63 Di[q0 + lane - 32]
  auto dma_rows = [&](char* stage, int q0) {
    const int qi = min(q0 + (lane & 31), a.Lq - 1);
    const float* src = (lane < 32 ? LSE : DI) + qi;
    lds_dma4(src, stage + C::TILEB + CG::TILEB + w * RWB);
  };
  // keep words of this wave's 32 keys (word key / 32) for the 32 queries of a tile (lanes 32..63
  // repeat lanes 0..31)
  constexpr bool bits = DROP == DROP_BITS;
  const uint32_t* KEEPW = bits ? fr.keep + min(wi.x * NWV + w, fr.kw - 1) : nullptr;
  auto dma_bits = [&](char* stage, int q0) {
    lds_dma4(KEEPW + (int64_t)min(q0 + (lane & 31), a.Lq - 1) * fr.kw, stage + C::TILEB + CG::TILEB + w * RWB + 256);
  };
  // V-fold: dr of the tile's 32 queries = du'[q, DV] (bf16, read as the word of columns DV, DV + 1)
  auto dma_dr = [&](char* stage, int q0) {
    lds_dma4(G + (int64_t)min(q0 + (lane & 31), a.Lq - 1) * a.sgl + DV, stage + C::TILEB + CG::TILEB + w * RWB + 512);
  };
  if constexpr (!KREG) dma_tile<DP, NWV * 32, NWV, true, 1>(Kblk, K, a.skl, wi.x * (NWV * 32), fr.Lk, w, lane);
  dma_tile<DP, QT, NWV, true, 1>(stages, Q, a.sql, qbase, a.Lq, w, lane);
  dma_tile<DV, QT, NWV, true, SWG>(stages + C::TILEB, G, a.sgl, qbase, a.Lq, w, lane);
  dma_rows(stages, qbase);
  if constexpr (bits) dma_bits(stages, qbase);
  if constexpr (FOLD) dma_dr(stages, qbase);
  auto issue = [&](char* Qn, int qn) {
    dma_tile<DP, QT, NWV, true, 1>(Qn, Q, a.sql, qn, a.Lq, w, lane);
    dma_tile<DV, QT, NWV, true, SWG>(Qn + C::TILEB, G, a.sgl, qn, a.Lq, w, lane);
    dma_rows(Qn, qn);
    if constexpr (bits) dma_bits(Qn, qn);
    if constexpr (FOLD) dma_dr(Qn, qn);
  };
  if (NSB == 3 && nt > 1) issue(stages + STAGE, qbase + QT);
  bf16x8 vf[NTV];  // B operand V^T (V-fold: M^T): [k = d = 16t + 8hi + j][n = key]
  const int64_t vkey = min(key, fr.Lk - 1);
#pragma unroll
  for (int t = 0; t < NTV; ++t) vf[t] = *(const bf16x8*)(V + vkey * a.svl + 16 * t + 8 * hi);
  bf16x8 kf[KREG ? NT : 1];  // B operand K^T of S = Q K^T: [k = d = 16t + 8hi + j][n = key]
  if constexpr (KREG) {
#pragma unroll
    for (int t = 0; t < NT; ++t) kf[t] = *(const bf16x8*)(K + vkey * a.skl + 16 * t + 8 * hi);
  }
  __builtin_amdgcn_s_waitcnt(0xF70);  // retire the V (K) loads in the compiler's bookkeeping (see dq)
  const int krow = w * 32 + kl;  // this lane's key row in the K block
  constexpr int NDV = FOLD ? 1 : ND;
  f32x16 dk[ND], dv[NDV];  // dK^T / dV^T: row d = 32*db + 8(r>>2) + 4hi + (r&3), column key
#pragma unroll
  for (int d = 0; d < ND; ++d) dk[d] = f32x16{};
#pragma unroll
  for (int d = 0; d < NDV; ++d) dv[d] = f32x16{};
  int cur = 0;  // it % NSB
  for (int it = 0; it < nt; ++it) {
    const int q0 = qbase + it * QT;
    char* Qb = stages + cur * STAGE;
    char* Gb = Qb + C::TILEB;
    // [lse(32) | Di(32) | keep(32) | - | dr words(32) | -]
    const float* rows = (const float*)(Qb + C::TILEB + CG::TILEB + w * RWB);
    const uint32_t* kwd = (const uint32_t*)(rows + 64);
    const uint32_t* drw = (const uint32_t*)(rows + 128);
    constexpr int PER_STAGE = C::PPW + CG::PPW + 1 + (bits ? 1 : 0) + (FOLD ? 1 : 0);  // DMAs per wave and stage
    if constexpr (NSB == 2) {
      if (it + 1 < nt) {
        issue(stages + (cur ^ 1) * STAGE, q0 + QT);
        wait_vmcnt<PER_STAGE>();
      } else {
        wait_vmcnt<0>();
      }
      wg_barrier();
    } else {
      // tile it + 1 stays in flight across this one; tile it + 2 goes after the barrier into the buffer
      // every wave finished reading in iteration it - 1
      if (it + 1 < nt) wait_vmcnt<PER_STAGE>();
      else wait_vmcnt<0>();
      wg_barrier();
      if (it + 2 < nt) issue(stages + (cur == 0 ? 2 : cur - 1) * STAGE, q0 + 2 * QT);
    }
    cur = cur == NSB - 1 ? 0 : cur + 1;

    f32x16 s = f32x16{}, dp = f32x16{};  // S / dP: row q = 8(r>>2) + 4hi + (r&3), column key
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const bf16x8 qa = *(const bf16x8*)(Qb + swz<DP, 1>(kl, 2 * t + hi));
      if constexpr (KREG) {
        s = mfma32(qa, kf[t], s);
      } else {
        const bf16x8 kb = *(const bf16x8*)(Kblk + swz<DP, 1>(krow, 2 * t + hi));
        s = mfma32(qa, kb, s);
      }
      if (t < NTV) {
        const bf16x8 ga = *(const bf16x8*)(Gb + swz<DV, SWG>(kl, 2 * t + hi));
        dp = mfma32(ga, vf[t], dp);
      }
      if ((t & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // bound the fragment prefetch depth
    }
    bf16x8 pdb[2], dsb[2];  // 16-query steps c: k index 8hi + j <-> r = 8c + j
    const bool qfull = q0 + QT <= a.Lq;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ql = 8 * (r >> 2) + 4 * hi + (r & 3);
      const int qi = q0 + ql;
      const float lse_r = rows[ql], di_r = rows[32 + ql];
      float p = __builtin_amdgcn_exp2f(fmaf(s[r], a.sl2, -lse_r * FL_LOG2E));
      if (!qfull) p = qi < a.Lq ? p : 0.f;  // wave-uniform test, then a select
      if constexpr (FOLD) dp[r] += __uint_as_float(drw[ql] << 16);  // + dr (bf16 in the low half)
      if constexpr (DROP == DROP_NONE) {
        pdb[r >> 3][r & 7] = (bf16)p;
        dsb[r >> 3][r & 7] = (bf16)(p * (dp[r] - di_r));
      } else {
        bool keep;
        if constexpr (bits) keep = (kwd[ql] >> kl) & 1u;
        else keep = s2h_keep(seed, fr.drow0 + (uint64_t)qi * (uint64_t)fr.Lk + key, a.thresh);
        // dV accumulates the kept P unscaled (x 1/keep at the store); dS = P (keep dP / keep_p - Di)
        const float pk = keep ? p : 0.f;
        const float dpd = keep ? dp[r] : 0.f;
        pdb[r >> 3][r & 7] = (bf16)pk;
        dsb[r >> 3][r & 7] = (bf16)(p * fmaf(dpd, a.inv_keep, -di_r));
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int d = 0; d < ND; ++d) {
        if constexpr (!FOLD) dv[d] = mfma32(tr_frag_perm32<DP, 1>(Gb, 16 * c, 32 * d, lane), pdb[c], dv[d]);
        dk[d] = mfma32(tr_frag_perm32<DP, 1>(Qb, 16 * c, 32 * d, lane), dsb[c], dk[d]);
        if (d & 1) __builtin_amdgcn_sched_barrier(0);
      }
    if constexpr (NSB == 2) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wg_barrier();
    }
  }

  if (!kv) return;
  if (!FOLD && a.kv_splits > 1) {  // fp32 partials, summed (and scaled, cast) by flash_bwd_dkv_combine_kernel
    float* W = a.ws_dkv + (((int64_t)wi.z * a.BH + bh) * a.Lk + key) * 2 * DP;  // single-frame only
#pragma unroll
    for (int d = 0; d < ND; ++d)
#pragma unroll
      for (int G4 = 0; G4 < 4; ++G4) {
        const int d0 = 32 * d + 8 * G4 + 4 * hi;
        *(float4*)(W + d0) = float4{dk[d][4 * G4], dk[d][4 * G4 + 1], dk[d][4 * G4 + 2], dk[d][4 * G4 + 3]};
        const int dvd = FOLD ? 0 : d;
        *(float4*)(W + DP + d0) = float4{dv[dvd][4 * G4] * a.inv_keep, dv[dvd][4 * G4 + 1] * a.inv_keep,
                                         dv[dvd][4 * G4 + 2] * a.inv_keep, dv[dvd][4 * G4 + 3] * a.inv_keep};
      }
    return;
  }
  bf16* DK = fr.dk + (int64_t)key * a.sdkl;
  bf16* DVp = FOLD ? nullptr : fr.dv + (int64_t)key * a.sdvl;
  // inverse RoPE of the key gradient (V-fold instance only: rope_k; in the DV = 256 instance the table
  // entries held over the dV stores spilled, and loads issued between stores serialise on them)
  const int nrk = FOLD && a.rope_k ? (a.nfr > 0 ? kargs()->fr_nrot[b / a.bpf] : fr.Lk) : 0;
  const float* rc = rope_row(a, key, nrk, a.rope_cos);
  const float* rsn = rope_row(a, key, nrk, a.rope_sin);
  RopeCS tab[FOLD ? ND : 1][4];
  if constexpr (FOLD) {
    if (rc != nullptr) {
#pragma unroll
      for (int d = 0; d < ND; ++d)
#pragma unroll
        for (int j = 0; j < 4; ++j) tab[d][j] = rope_load(rc, rsn, 32 * d + 8 * j + 4 * hi);
    }
  }
#pragma unroll
  for (int d = 0; d < ND; ++d)
#pragma unroll
    for (int G4 = 0; G4 < 4; ++G4) {
      bf16 tk[4], tv[4];
      const int dvd = FOLD ? 0 : d;
      float k4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) k4[e] = dk[d][4 * G4 + e] * a.scale;
      if constexpr (FOLD) {
        if (rc != nullptr) rope_apply(k4, tab[d][G4]);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        tk[e] = (bf16)k4[e];
        tv[e] = (bf16)(dv[dvd][4 * G4 + e] * a.inv_keep);
      }
      const int d0 = 32 * d + 8 * G4 + 4 * hi;
      *(uint2*)(DK + d0) = *(const uint2*)tk;
      if constexpr (!FOLD) *(uint2*)(DVp + d0) = *(const uint2*)tv;
    }
}

// ------------------------------------------------------------------ dK / dV, head dim 256, two waves per SIMD
// 8 waves x 16 keys per workgroup, 16x16x32 MFMA, two waves per SIMD (<= 256 VGPRs): each wave's
// softmax / dropout VALU issues under its partner's MFMAs.  (flash_bwd_dkv32_kernel, one wave per
// SIMD on 32x32x16, measured 15 % MFMA-busy at 13.7 VALU per MFMA on the V-fold: its 512-register
// allocation moved S / dP through the accumulator file every tile and each swizzled fragment read
// was waited for alone; the DV = 256 instance also spilled.)
//   DV = 64 (V-fold, s2h_flash_bwd_frames_vfold): the value is the 64-wide memory bank M, dO is
//     du' = [du | dr | 0] and there is no dV: K^T (32 VGPRs) + M^T (8) fragments, dK^T (64).
//   DV = 256 (memory self-attention): K^T + V^T fragments (64), dK^T + dV^T accumulators (128).
// Per 32-query tile and wave: S = Q K^T (16 MFMA), dP = dO V^T (4 / 16), dK^T += Q^T dS (16),
// dV^T += dO^T P_drop (16, DV = 256).  Q and dO tiles sit in padded images (one base register +
// immediate offsets for every fragment, conflict-free b128 and transposing reads); the row
// constants (lse, Di, dr, keep words [word][query]) are DMA'd beside them so a lane reads its 4
// consecutive queries with one b128.  DMA pieces per stage and wave: Q pieces w, w + 8 (16: wave 0);
// DV = 256 dO the same (16: wave 1), DV = 64 du' pieces 0..4 on waves 1..5; lse | Di on wave 6;
// dr (DV = 64) and the keep words on wave 7.
// NSB: stages in the Q / du' ring -- 3 (default): tile it + 1 in flight across tile it's compute, one
// barrier per tile; 2: the round-5 ring, two barriers per tile.  PF: LDS fragment reads kept ahead of
// their MFMAs in the S / dP phase.  3 stages + 8 ahead: V-fold backward 1.231 -> 1.192 ms (dQ + dK,
// tools/vfold_bwd_bench.py).  Measured and dropped: waves 4-7 staggered by one phase (each tile's dK
// phase after the next barrier, 4-stage ring): 1.213 vs 1.177 ms (profiles/r06_v28_vfold_bwd.log).
template <int DV, int DROP, int NSB = 3, int PF = 8>
__global__ __launch_bounds__(512, 1) void flash_bwd_dkv16_kernel(FlashBwdArgs a) {
  static_assert(NSB == 2 || NSB == 3, "ring depth");
  const uint64_t seed = DROP == DROP_HASH ? s2h_seed(a.seed, a.seed_off) : 0;
  constexpr int DP = 256, QT = 32, NW = 8;
  constexpr bool FOLD = DV != DP;
  using IQ = PadImg<DP, QT, NW>;  // 32 rows x 544 B, 17 pieces
  using IG = PadImg<DV, QT, 1>;   // dO / du': 32 rows x 544 B (17 pieces) or x 160 B (5 pieces)
  constexpr int RB_LSE = 0, RB_DI = 128, RB_DR = 256, RB_KEEP = 384;  // row block: + keep [4 words][32 q]
  constexpr int RB = 384 + 512;
  constexpr int STAGE = IQ::TILEB + IG::TILEB + RB;
  constexpr bool bits = DROP == DROP_BITS;
  __shared__ __attribute__((aligned(1024))) char smem[NSB * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, kl = lane & 15;
  const WgIdx wi = wg_xcd_order();
  if (wi.y >= a.BH) return;  // grid padding
  const int bh = wi.y, b = bh / a.H, h = bh % a.H;
  const KvFrame fr = kv_frame(a, bh);
  if (wi.x * (NW * 16) >= fr.Lk) return;  // frame-table launch: past this frame's keys
  if ((a.prio & 1) && w >= 4) __builtin_amdgcn_s_setprio(1);
  const int key = wi.x * (NW * 16) + w * 16 + kl;
  const bool kv = key < fr.Lk;
  const bf16* Q = a.q + b * a.sqb + h * a.sqh;
  const bf16* G = a.g + b * a.sgb + h * a.sgh;
  const float* LSE = a.lse + (int64_t)bh * a.Lq;
  const float* DI = a.di + (int64_t)bh * a.Lq;
  const int nt = (a.Lq + QT - 1) / QT;
  const int Lq1 = a.Lq - 1;

  // one 1-KiB piece of a padded [32][C] image of rows q0.. of src (row stride ld)
  auto dma_piece = [&](char* img, const bf16* src, int64_t ld, int spr, int ncol, int q0, int piece) {
    const int slot = piece * 64 + lane;
    const int row = slot / spr, c = slot % spr;
    lds_dma16(src + (min(q0 + row, Lq1) * (int)ld + (c < ncol / 8 ? 8 * c : 0)), img + piece * 1024);
  };
  auto issue = [&](char* st, int q0) {
    dma_piece(st, Q, a.sql, IQ::SPR, DP, q0, w);
    dma_piece(st, Q, a.sql, IQ::SPR, DP, q0, w + 8);
    if (w == 0) dma_piece(st, Q, a.sql, IQ::SPR, DP, q0, 16);
    char* gimg = st + IQ::TILEB;
    if constexpr (FOLD) {
      if (w >= 1 && w <= 5) dma_piece(gimg, G, a.sgl, IG::SPR, DV, q0, w - 1);
    } else {
      dma_piece(gimg, G, a.sgl, IG::SPR, DV, q0, w);
      dma_piece(gimg, G, a.sgl, IG::SPR, DV, q0, w + 8);
      if (w == 1) dma_piece(gimg, G, a.sgl, IG::SPR, DV, q0, 16);
    }
    char* rb = st + IQ::TILEB + IG::TILEB;
    if (w == 6) {  // lanes 0..31 lse, 32..63 Di
      lds_dma4((lane < 32 ? LSE : DI) + min(q0 + (lane & 31), Lq1), rb + RB_LSE);
    } else if (w == 7) {
      // dr = du'[q, DV] (bf16 in the low half of the word); lanes 32..63 repeat 0..31
      if constexpr (FOLD) lds_dma4(G + (min(q0 + (lane & 31), Lq1) * (int)a.sgl + DV), rb + RB_DR);
      if constexpr (bits) {  // keep words (key / 32) of the block's 128 keys: [word][query]
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int word = min(wi.x * 4 + 2 * j + (lane >> 5), fr.kw - 1);
          lds_dma4(fr.keep + (int64_t)min(q0 + (lane & 31), Lq1) * fr.kw + word, rb + RB_KEEP + j * 256);
        }
      }
    }
  };
  // vmcnt that leaves this wave's DMAs of the next stage in flight (wave-uniform counts)
  auto wait_stage = [&]() {
    if constexpr (FOLD) {  // 3 on every wave, 5 on wave 7 with the bitmap
      if (bits && w == 7) wait_vmcnt<5>();
      else wait_vmcnt<3>();
    } else {  // 4, + 1 on waves 0, 1, 6, + 2 on wave 7 with the bitmap
      if (w == 0 || w == 1 || w == 6) wait_vmcnt<5>();
      else if (bits && w == 7) wait_vmcnt<6>();
      else wait_vmcnt<4>();
    }
  };

  issue(smem, 0);
  if (NSB >= 3 && nt > 1) issue(smem + STAGE, QT);
  bf16x8 kf[DP / 32], vf[DV / 32];  // B operands K^T / V^T: [k = d = 32t + 8g + j][n = key]
  const int64_t vkey = min(key, fr.Lk - 1);
#pragma unroll
  for (int t = 0; t < DP / 32; ++t) kf[t] = *(const bf16x8*)(fr.k + vkey * a.skl + 32 * t + 8 * g);
#pragma unroll
  for (int t = 0; t < DV / 32; ++t) vf[t] = *(const bf16x8*)(fr.v + vkey * a.svl + 32 * t + 8 * g);
  __builtin_amdgcn_s_waitcnt(0xF70);  // retire the fragment loads in the compiler's bookkeeping
  constexpr int NDV = FOLD ? 1 : DP / 16;
  f32x4 dk[DP / 16], dv[NDV];  // dK^T / dV^T: row d = 16 db + 4g + r, column key
#pragma unroll
  for (int d = 0; d < DP / 16; ++d) dk[d] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int d = 0; d < NDV; ++d) dv[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int kword = (w & 1) * 16 + kl;  // this lane's bit in its keep word
  const int kwsel = w >> 1;             // which of the block's 4 words

  // dK^T += Q^T dS, dV^T += dO^T P_drop (transposing reads of the padded Q / dO images)
  auto dk_phase = [&](const char* Qb, const char* Gb, bf16x8 ds, bf16x8 pd) {
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int d = 0; d < DP / 16; ++d) {
      dk[d] = mfma16(tr_frag_pad<IQ::ROWB>(Qb, 0, 16 * d, lane), ds, dk[d]);
      if constexpr (!FOLD) dv[d] = mfma16(tr_frag_pad<IG::ROWB>(Gb, 0, 16 * d, lane), pd, dv[d]);
    }
    sched_reads_ahead<(FOLD ? 1 : 2) * DP / 16, 4, 2>();
    __builtin_amdgcn_sched_barrier(0);
  };

  int cur = 0;  // it % NSB
  for (int it = 0; it < nt; ++it) {
    const int q0 = it * QT;
    char* st = smem + cur * STAGE;
    if constexpr (NSB == 2) {
      if (it + 1 < nt) {
        issue(smem + (cur ^ 1) * STAGE, q0 + QT);
        wait_stage();
      } else {
        wait_vmcnt<0>();
      }
      wg_barrier();
    } else {
      // one barrier per tile: tile it + 1 stays in flight across it; tile it + 2 is issued after the
      // barrier into the buffer every wave finished reading in iteration it - 1
      if (it + 1 < nt) wait_stage();
      else wait_vmcnt<0>();
      wg_barrier();
      if (it + 2 < nt) issue(smem + ((cur + 2) % NSB) * STAGE, q0 + 2 * QT);
    }
    cur = cur == NSB - 1 ? 0 : cur + 1;
    const char* Qi = st;
    const char* Gi = st + IQ::TILEB;
    const char* rb = st + IQ::TILEB + IG::TILEB;

    f32x4 s[2], dp[2];  // row q = 16 qb + 4g + r, column key
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      s[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[qb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const char* qrow = Qi + (16 * qb + kl) * IQ::ROWB + 16 * g;
      const char* grow = Gi + (16 * qb + kl) * IG::ROWB + 16 * g;
#pragma unroll
      for (int t = 0; t < DP / 32; ++t) s[qb] = mfma16(*(const bf16x8*)(qrow + 64 * t), kf[t], s[qb]);
#pragma unroll
      for (int t = 0; t < DV / 32; ++t) dp[qb] = mfma16(*(const bf16x8*)(grow + 64 * t), vf[t], dp[qb]);
    }
    sched_reads_ahead<2 * (DP / 32 + DV / 32), PF, 1>();
    __builtin_amdgcn_sched_barrier(0);
    // B operands over 32 queries: k index 8g + j <-> q 16(j >> 2) + 4g + (j & 3)
    bf16x8 dsb, pdb;
    // the query-tail test as a separate code path (an in-line `if` became per-element selects)
    auto softmax = [&](auto tail) {
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const int qo = 16 * qb + 4 * g;
        const float4 l4 = *(const float4*)(rb + RB_LSE + 4 * qo);
        const float4 d4 = *(const float4*)(rb + RB_DI + 4 * qo);
        uint4 r4 = uint4{0u, 0u, 0u, 0u}, k4 = uint4{0u, 0u, 0u, 0u};
        if constexpr (FOLD) r4 = *(const uint4*)(rb + RB_DR + 4 * qo);
        if constexpr (bits) k4 = *(const uint4*)(rb + RB_KEEP + kwsel * 128 + 4 * qo);
        const float lt[4] = {l4.x, l4.y, l4.z, l4.w};
        const float dt[4] = {d4.x, d4.y, d4.z, d4.w};
        const uint32_t rt[4] = {r4.x, r4.y, r4.z, r4.w};
        const uint32_t kt[4] = {k4.x, k4.y, k4.z, k4.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float p = __builtin_amdgcn_exp2f(fmaf(s[qb][r], a.sl2, -lt[r] * FL_LOG2E));
          if constexpr (decltype(tail)::value) p = q0 + qo + r < a.Lq ? p : 0.f;
          const float dpr = FOLD ? dp[qb][r] + __uint_as_float(rt[r] << 16) : dp[qb][r];
          float dsv, pk = p;
          if constexpr (DROP != DROP_NONE) {
            bool keep;
            if constexpr (bits) keep = (kt[r] >> kword) & 1u;
            else keep = s2h_keep(seed, fr.drow0 + (uint64_t)(q0 + qo + r) * (uint64_t)fr.Lk + key, a.thresh);
            dsv = p * fmaf(keep ? dpr : 0.f, a.inv_keep, -dt[r]);
            pk = keep ? p : 0.f;  // dV accumulates the kept P unscaled (x 1/keep at the store)
          } else {
            dsv = p * (dpr - dt[r]);
          }
          dsb[4 * qb + r] = (bf16)dsv;
          if constexpr (!FOLD) pdb[4 * qb + r] = (bf16)pk;
        }
      }
    };
    if (q0 + QT <= a.Lq) softmax(std::false_type{});
    else softmax(std::true_type{});
    dk_phase(Qi, Gi, dsb, pdb);
    if constexpr (NSB == 2) {  // every wave's reads of this stage retired before it is refilled
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wg_barrier();
    }
  }

  if (!kv) return;
  bf16* DK = fr.dk + (int64_t)key * a.sdkl;
  // inverse RoPE of the key gradient: the lane's 4 consecutive columns are 2 rotation pairs
  const int nrk = a.rope_k ? (a.nfr > 0 ? kargs()->fr_nrot[b / a.bpf] : fr.Lk) : 0;
  const float* rc = rope_row(a, key, nrk, a.rope_cos);
  const float* rsn = rope_row(a, key, nrk, a.rope_sin);
  RopeCS tab[DP / 16];
  if (rc != nullptr) {
#pragma unroll
    for (int d = 0; d < DP / 16; ++d) tab[d] = rope_load(rc, rsn, 16 * d + 4 * g);
  }
#pragma unroll
  for (int d = 0; d < DP / 16; ++d) {
    float v4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v4[e] = dk[d][e] * a.scale;
    if (rc != nullptr) rope_apply(v4, tab[d]);
    bf16 t4[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) t4[e] = (bf16)v4[e];
    *(uint2*)(DK + 16 * d + 4 * g) = *(const uint2*)t4;
  }
  if constexpr (!FOLD) {
    bf16* DVp = fr.dv + (int64_t)key * a.sdvl;
#pragma unroll
    for (int d = 0; d < DP / 16; ++d) {
      bf16 t4[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) t4[e] = (bf16)(dv[d][e] * a.inv_keep);
      *(uint2*)(DVp + 16 * d + 4 * g) = *(const uint2*)t4;
    }
  }
}

// dK = scale * sum_s partial_dK[s], dV = sum_s partial_dV[s]; 4 consecutive d per thread
template <int DP>
__global__ __launch_bounds__(256) void flash_bwd_dkv_combine_kernel(FlashBwdArgs a) {
  const int64_t rows = (int64_t)a.BH * a.Lk;
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;  // over rows * 2 * DP
  if (i >= rows * 2 * DP) return;
  float4 s = *(const float4*)(a.ws_dkv + i);
  for (int sp = 1; sp < a.kv_splits; ++sp) {
    const float4 t = *(const float4*)(a.ws_dkv + sp * rows * 2 * DP + i);
    s.x += t.x; s.y += t.y; s.z += t.z; s.w += t.w;
  }
  const int64_t row = i / (2 * DP);
  const int part = (int)((i / DP) & 1), d = (int)(i % DP);
  const int bh = row / a.Lk, key = row % a.Lk, b = bh / a.H, h = bh % a.H;
  const float f = part == 0 ? a.scale : 1.f;
  bf16 t4[4] = {(bf16)(s.x * f), (bf16)(s.y * f), (bf16)(s.z * f), (bf16)(s.w * f)};
  bf16* dst = part == 0 ? a.dk + b * a.sdkb + h * a.sdkh + (int64_t)key * a.sdkl + d
                        : a.dv + b * a.sdvb + h * a.sdvh + (int64_t)key * a.sdvl + d;
  *(uint2*)dst = *(const uint2*)t4;
}

// ------------------------------------------------------------------ host
// dK/dV (head_dim 256): 128-key workgroups, one per CU; when they cannot fill the chip
// (short key ranges: the memory-attention self-attention, Lk = 1024 x 13 objects = 104
// blocks) the query range is split over workgroups with fp32 partials.
static void flash_bwd_kv_plan(int BH, int Lq, int Lk, int& kv_splits, int& tps) {
  const int base = ((Lk + 127) / 128) * BH;
  const int nt = (Lq + 31) / 32;
  int s = base >= 256 ? 1 : 256 / base;
  s = std::max(1, std::min(s, nt / 4));
  tps = (nt + s - 1) / s;
  kv_splits = (nt + tps - 1) / tps;
}

static void flash_bwd_plan(int BH, int Lq, int Lk, int& splits, int& tps) {
  const int base = ((Lq + FL_QB - 1) / FL_QB) * BH;
  const int ntiles = (Lk + 63) / 64;
  int s = (512 + base - 1) / base;
  s = std::max(1, std::min(s, ntiles / 2));
  tps = (ntiles + s - 1) / s;
  splits = (ntiles + tps - 1) / tps;
}

// [dQ partials][dK/dV partials], each present only when its kernel splits
static void flash_bwd_ws_layout(int BH, int Lq, int Lk, int D, int64_t& dq_bytes, int64_t& dkv_bytes) {
  int splits, tps, kvs, ktps;
  flash_bwd_plan(BH, Lq, Lk, splits, tps);
  flash_bwd_kv_plan(BH, Lq, Lk, kvs, ktps);
  const int DPd = flash_dp(D);  // padded image width of the dQ partials
  dq_bytes = splits > 1 ? (int64_t)splits * BH * Lq * DPd * 4 : 0;
  dkv_bytes = (D == 256 && kvs > 1) ? (int64_t)kvs * BH * Lk * 2 * D * 4 : 0;
}

int64_t s2h_flash_bwd_ws_bytes(int B, int H, int Lq, int Lk, int D) {
  int64_t dq_bytes, dkv_bytes;
  flash_bwd_ws_layout(B * H, Lq, Lk, D, dq_bytes, dkv_bytes);
  return dq_bytes + dkv_bytes;
}

template <int DP, int DV = DP>
static int flash_bwd_launch(FlashBwdArgs& a, hipStream_t st) {
  const int64_t rows = (int64_t)a.BH * a.Lq;
  a.prio = (s2h_flash_variant() >> 1) & 3;
  // Di = rowsum(dO * O) is computed by the dQ kernel and stored for the dK / dV kernel
  const int drop = a.p_drop <= 0.f ? DROP_NONE : (a.keep ? DROP_BITS : DROP_HASH);
  const dim3 gq((a.Lq + FL_QB - 1) / FL_QB, pad_bh8(a.BH), a.splits);
  // the V-fold dQ kernel on the 3-stage ring with 8 reads ahead (A/B: variant bit 6 the 2-stage form)
  bool dq_done = false;
  if constexpr (DP == 256 && DV == 64) {
    if (((s2h_flash_variant() >> 6) & 1) == 0) {
      if (drop == DROP_NONE) hipLaunchKernelGGL((flash_bwd_dq_kernel<DP, DROP_NONE, DV, 3, 8>), gq, dim3(FL_WAVES * 64), 0, st, a);
      else if (drop == DROP_BITS) hipLaunchKernelGGL((flash_bwd_dq_kernel<DP, DROP_BITS, DV, 3, 8>), gq, dim3(FL_WAVES * 64), 0, st, a);
      else hipLaunchKernelGGL((flash_bwd_dq_kernel<DP, DROP_HASH, DV, 3, 8>), gq, dim3(FL_WAVES * 64), 0, st, a);
      dq_done = true;
    }
  }
  if constexpr (DV == DP && DP == 256) {  // self-attention: 8 reads ahead (A/B bit 1 of s2h_flash_variant2)
    if (s2h_flash_v2() & 1) {
      if (drop == DROP_NONE) hipLaunchKernelGGL((flash_bwd_dq_kernel<DP, DROP_NONE, DV, 2, 8>), gq, dim3(FL_WAVES * 64), 0, st, a);
      else if (drop == DROP_BITS) hipLaunchKernelGGL((flash_bwd_dq_kernel<DP, DROP_BITS, DV, 2, 8>), gq, dim3(FL_WAVES * 64), 0, st, a);
      else hipLaunchKernelGGL((flash_bwd_dq_kernel<DP, DROP_HASH, DV, 2, 8>), gq, dim3(FL_WAVES * 64), 0, st, a);
      dq_done = true;
    }
  }
  if constexpr (DV == DP && DP <= 128) {  // Hiera: the 3-stage ring, 8 ahead (A/B bit 2)
    if (s2h_flash_v2() & 2) {
      if (drop == DROP_NONE) hipLaunchKernelGGL((flash_bwd_dq_kernel<DP, DROP_NONE, DV, 3, 8>), gq, dim3(FL_WAVES * 64), 0, st, a);
      else if (drop == DROP_BITS) hipLaunchKernelGGL((flash_bwd_dq_kernel<DP, DROP_BITS, DV, 3, 8>), gq, dim3(FL_WAVES * 64), 0, st, a);
      else hipLaunchKernelGGL((flash_bwd_dq_kernel<DP, DROP_HASH, DV, 3, 8>), gq, dim3(FL_WAVES * 64), 0, st, a);
      dq_done = true;
    }
  }
  if (!dq_done) {
    if (drop == DROP_NONE) hipLaunchKernelGGL((flash_bwd_dq_kernel<DP, DROP_NONE, DV>), gq, dim3(FL_WAVES * 64), 0, st, a);
    else if (drop == DROP_BITS) hipLaunchKernelGGL((flash_bwd_dq_kernel<DP, DROP_BITS, DV>), gq, dim3(FL_WAVES * 64), 0, st, a);
    else hipLaunchKernelGGL((flash_bwd_dq_kernel<DP, DROP_HASH, DV>), gq, dim3(FL_WAVES * 64), 0, st, a);
  }
  if (a.splits > 1)
    hipLaunchKernelGGL((flash_bwd_dq_combine_kernel<DP>), dim3((unsigned)((rows * DP / 4 + 255) / 256)), dim3(256), 0,
                       st, a);
  if constexpr (DP == 256) {
    const dim3 gk((a.Lk + 127) / 128, pad_bh8(a.BH), a.kv_splits);
    // V-fold: two waves per SIMD (flash_bwd_dkv16_kernel) unless variant bit 1 asks for the 32x32
    // kernel below; it takes a single query range per workgroup (no fp32 partials).  The DV = 256
    // instance (memory self-attention) spilled at 256 VGPRs and measured slower than the 32x32 kernel
    // (tools/attn_ab.py --variants: self-attention backward 0.565 vs 0.513 ms), so it is not built.
    if constexpr (DV == 64) {
      if (a.kv_splits == 1 && (s2h_flash_variant() & 1) == 0) {
        if ((s2h_flash_variant() >> 4) & 1) {  // A/B: variant bit 4 the round-5 2-stage ring
          if (drop == DROP_NONE) hipLaunchKernelGGL((flash_bwd_dkv16_kernel<DV, DROP_NONE, 2, 4>), gk, dim3(512), 0, st, a);
          else if (drop == DROP_BITS) hipLaunchKernelGGL((flash_bwd_dkv16_kernel<DV, DROP_BITS, 2, 4>), gk, dim3(512), 0, st, a);
          else hipLaunchKernelGGL((flash_bwd_dkv16_kernel<DV, DROP_HASH, 2, 4>), gk, dim3(512), 0, st, a);
        } else {
          if (drop == DROP_NONE) hipLaunchKernelGGL((flash_bwd_dkv16_kernel<DV, DROP_NONE>), gk, dim3(512), 0, st, a);
          else if (drop == DROP_BITS) hipLaunchKernelGGL((flash_bwd_dkv16_kernel<DV, DROP_BITS>), gk, dim3(512), 0, st, a);
          else hipLaunchKernelGGL((flash_bwd_dkv16_kernel<DV, DROP_HASH>), gk, dim3(512), 0, st, a);
        }
        return (int)hipGetLastError();
      }
    }
    if (s2h_flash_v2() & 8) {  // the 3-stage ring (A/B bit 8 of s2h_flash_variant2)
      if (drop == DROP_NONE) hipLaunchKernelGGL((flash_bwd_dkv32_kernel<DP, DROP_NONE, true, DV, 3>), gk, dim3(256), 0, st, a);
      else if (drop == DROP_BITS) hipLaunchKernelGGL((flash_bwd_dkv32_kernel<DP, DROP_BITS, true, DV, 3>), gk, dim3(256), 0, st, a);
      else hipLaunchKernelGGL((flash_bwd_dkv32_kernel<DP, DROP_HASH, true, DV, 3>), gk, dim3(256), 0, st, a);
    } else if (drop == DROP_NONE) {
      hipLaunchKernelGGL((flash_bwd_dkv32_kernel<DP, DROP_NONE, true, DV>), gk, dim3(256), 0, st, a);
    } else if (drop == DROP_BITS) {
      hipLaunchKernelGGL((flash_bwd_dkv32_kernel<DP, DROP_BITS, true, DV>), gk, dim3(256), 0, st, a);
    } else {
      hipLaunchKernelGGL((flash_bwd_dkv32_kernel<DP, DROP_HASH, true, DV>), gk, dim3(256), 0, st, a);
    }
    if (DV == DP && a.kv_splits > 1) {
      const int64_t n4 = (int64_t)a.BH * a.Lk * 2 * DP / 4;
      hipLaunchKernelGGL((flash_bwd_dkv_combine_kernel<DP>), dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, a);
    }
  } else if constexpr (DV == DP) {
    const dim3 gk((a.Lk + FL_QB - 1) / FL_QB, pad_bh8(a.BH));
    if (drop == DROP_NONE) hipLaunchKernelGGL((flash_bwd_dkv_kernel<DP, DROP_NONE>), gk, dim3(FL_WAVES * 64), 0, st, a);
    else hipLaunchKernelGGL((flash_bwd_dkv_kernel<DP, DROP_HASH>), gk, dim3(FL_WAVES * 64), 0, st, a);
  }
  return (int)hipGetLastError();
}

// the dQ kernel reads O (for Di = rowsum(dO * O)) with 16-B loads: base and strides 16-B aligned
static bool flash_bwd_o_aligned(const void* o, int64_t sob, int64_t soh, int64_t sol) {
  return ((uintptr_t)o & 15) == 0 && (sob & 7) == 0 && (soh & 7) == 0 && (sol & 7) == 0;
}

int s2h_flash_bwd(int B, int H, int Lq, int Lk, int D,
                  const void* q, int64_t sqb, int64_t sqh, int64_t sql,
                  const void* k, int64_t skb, int64_t skh, int64_t skl,
                  const void* v, int64_t svb, int64_t svh, int64_t svl,
                  const void* o, int64_t sob, int64_t soh, int64_t sol,
                  const void* dout, int64_t sgb, int64_t sgh, int64_t sgl,
                  void* dq, int64_t sdqb, int64_t sdqh, int64_t sdql,
                  void* dk, int64_t sdkb, int64_t sdkh, int64_t sdkl,
                  void* dv, int64_t sdvb, int64_t sdvh, int64_t sdvl,
                  const float* lse, float* di_ws, float scale, float p_drop, uint64_t seed, uint64_t idx0,
                  const uint32_t* keep, void* ws, int64_t ws_bytes, hipStream_t st) {
  FlashBwdArgs a = {};
  a.idx0 = idx0;
  a.D = D;
  if (keep && D != 256) return (int)hipErrorInvalidValue;  // the head-dim-256 kernels read the bitmap
  if (!flash_bwd_o_aligned(o, sob, soh, sol)) return (int)hipErrorInvalidValue;
  a.keep = keep;
  a.kw = 2 * ((Lk + 63) / 64);
  a.BH = B * H; a.H = H; a.Lq = Lq; a.Lk = Lk;
  a.q = (const bf16*)q; a.sqb = sqb; a.sqh = sqh; a.sql = sql;
  a.k = (const bf16*)k; a.skb = skb; a.skh = skh; a.skl = skl;
  a.v = (const bf16*)v; a.svb = svb; a.svh = svh; a.svl = svl;
  a.o = (const bf16*)o; a.sob = sob; a.soh = soh; a.sol = sol;
  a.g = (const bf16*)dout; a.sgb = sgb; a.sgh = sgh; a.sgl = sgl;
  a.dq = (bf16*)dq; a.sdqb = sdqb; a.sdqh = sdqh; a.sdql = sdql;
  a.dk = (bf16*)dk; a.sdkb = sdkb; a.sdkh = sdkh; a.sdkl = sdkl;
  a.dv = (bf16*)dv; a.sdvb = sdvb; a.sdvh = sdvh; a.sdvl = sdvl;
  a.lse = lse; a.di = di_ws;
  a.scale = scale; a.sl2 = scale * FL_LOG2E;
  a.p_drop = p_drop;
  a.thresh = (uint32_t)(p_drop * 4294967296.0);
  a.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.seed = seed;
  a.seed_off = s2h_rng_offset_ptr();
  flash_bwd_plan(a.BH, Lq, Lk, a.splits, a.tiles_per_split);
  flash_bwd_kv_plan(a.BH, Lq, Lk, a.kv_splits, a.kv_tiles_per_split);
  int64_t dq_bytes, dkv_bytes;
  flash_bwd_ws_layout(a.BH, Lq, Lk, D, dq_bytes, dkv_bytes);
  if (dq_bytes + dkv_bytes > ws_bytes || (dq_bytes + dkv_bytes > 0 && ws == nullptr)) {
    return (int)hipErrorInvalidValue;  // the caller sizes ws with s2h_attn_bwd_ws_bytes
  }
  if (a.splits > 1) a.ws_dq = (float*)ws;
  if (dkv_bytes > 0) a.ws_dkv = (float*)((char*)ws + dq_bytes);
  else { a.kv_splits = 1; a.kv_tiles_per_split = (Lq + 31) / 32; }
  if (D == 256) return flash_bwd_launch<256>(a, st);
  if (D > 64) return flash_bwd_launch<128>(a, st);  // 72..128: padded 128 image
  return flash_bwd_launch<64>(a, st);               // 32..64: padded 64 image
}

// eligible: the flash forward's domain (bf16, head_dim 256 or 32..128 padded to 64 / 128, >= 128
// query rows)
int s2h_flash_bwd_eligible(int dt, int Lq, int D);
int s2h_flash_eligible(int dt, int Lq, int D);
int s2h_flash_bwd_eligible(int dt, int Lq, int D) { return s2h_flash_eligible(dt, Lq, D); }

// Frame-batched backward: nfr frames x bpf batches x H heads in ONE launch per kernel.  Q / O /
// dO / dQ / LSE are [nfr * bpf] uniform batches (batch stride sqb ...); K / V / dK / dV are
// packed per frame (frame f: bpf blocks of fr_lk[f] rows from row fr_krow[f]; row stride skl,
// head stride skh); dropout indices of frame f start at fr_idx0[f]; keep (nullable) holds frame
// f's forward keep bitmap from word fr_koff[f] (flash.hip layout: bpf * H * Lq rows of
// 2 * ceil(fr_lk[f] / 64) words).  nfr * bpf * (Lq / 128)
// query blocks fill the chip without key or query splits, so no fp32 partials or combines.
// the frame-table launches' optional inverse RoPE of dQ (fr_nrotq) and / or dK (fr_nrotk), head dim 256
static int flash_bwd_rope_args(FlashBwdArgs& a, int nfr, int D, const float* cos, const float* sin, int period,
                               const int* fr_nrotq, const int* fr_nrotk) {
  if (fr_nrotq == nullptr && fr_nrotk == nullptr) return 0;
  if (D != 256 || cos == nullptr || sin == nullptr || period <= 0 || ((uintptr_t)cos & 7) || ((uintptr_t)sin & 7))
    return (int)hipErrorInvalidValue;
  a.rope_cos = cos; a.rope_sin = sin; a.rope_period = period;
  a.rope_q = fr_nrotq != nullptr;
  a.rope_k = fr_nrotk != nullptr;
  for (int f = 0; f < nfr; ++f) {
    a.fr_nrotq[f] = fr_nrotq ? fr_nrotq[f] : 0;
    a.fr_nrot[f] = fr_nrotk ? fr_nrotk[f] : 0;
  }
  return 0;
}

extern "C" int s2h_flash_bwd_frames_rope(int nfr, int bpf, int H, int Lq, int D, const int* fr_lk,
                                         const int64_t* fr_krow, const uint64_t* fr_idx0, const void* q, int64_t sqb,
                                         int64_t sqh, int64_t sql, const void* k, int64_t skh, int64_t skl,
                                         const void* v, int64_t svh, int64_t svl, const void* o, int64_t sob,
                                         int64_t soh, int64_t sol, const void* dout, int64_t sgb, int64_t sgh,
                                         int64_t sgl, void* dq, int64_t sdqb, int64_t sdqh, int64_t sdql, void* dk,
                                         int64_t sdkh, int64_t sdkl, void* dv, int64_t sdvh, int64_t sdvl,
                                         const float* lse, float* di_ws, float scale, float p_drop, uint64_t seed,
                                         const uint32_t* keep, const int64_t* fr_koff, const float* rope_cos,
                                         const float* rope_sin, int rope_period, const int* fr_nrotq,
                                         hipStream_t st);
extern "C" int s2h_flash_bwd_frames(int nfr, int bpf, int H, int Lq, int D, const int* fr_lk, const int64_t* fr_krow,
                                    const uint64_t* fr_idx0, const void* q, int64_t sqb, int64_t sqh, int64_t sql,
                                    const void* k, int64_t skh, int64_t skl, const void* v, int64_t svh, int64_t svl,
                                    const void* o, int64_t sob, int64_t soh, int64_t sol, const void* dout,
                                    int64_t sgb, int64_t sgh, int64_t sgl, void* dq, int64_t sdqb, int64_t sdqh,
                                    int64_t sdql, void* dk, int64_t sdkh, int64_t sdkl, void* dv, int64_t sdvh,
                                    int64_t sdvl, const float* lse, float* di_ws, float scale, float p_drop,
                                    uint64_t seed, const uint32_t* keep, const int64_t* fr_koff, hipStream_t st) {
  return s2h_flash_bwd_frames_rope(nfr, bpf, H, Lq, D, fr_lk, fr_krow, fr_idx0, q, sqb, sqh, sql, k, skh, skl, v, svh,
                                   svl, o, sob, soh, sol, dout, sgb, sgh, sgl, dq, sdqb, sdqh, sdql, dk, sdkh, sdkl, dv,
                                   sdvh, sdvl, lse, di_ws, scale, p_drop, seed, keep, fr_koff, nullptr, nullptr, 1,
                                   nullptr, st);
}
// s2h_flash_bwd_frames with the q projection's RoPE epilogue transposed into the dQ store (head dim
// 256): query rows < fr_nrotq[f] of every batch block of frame f come out rotated back with table row
// (row % rope_period) of rope_cos / rope_sin [period][D / 2] (fr_nrotq == nullptr: unrotated).  The
// key gradient stays unrotated: the DV = 256 dK kernel's store did not take the rotation without
// spilling (see flash_bwd_dkv32_kernel)
extern "C" int s2h_flash_bwd_frames_rope(int nfr, int bpf, int H, int Lq, int D, const int* fr_lk,
                                         const int64_t* fr_krow, const uint64_t* fr_idx0, const void* q, int64_t sqb,
                                         int64_t sqh, int64_t sql, const void* k, int64_t skh, int64_t skl,
                                         const void* v, int64_t svh, int64_t svl, const void* o, int64_t sob,
                                         int64_t soh, int64_t sol, const void* dout, int64_t sgb, int64_t sgh,
                                         int64_t sgl, void* dq, int64_t sdqb, int64_t sdqh, int64_t sdql, void* dk,
                                         int64_t sdkh, int64_t sdkl, void* dv, int64_t sdvh, int64_t sdvl,
                                         const float* lse, float* di_ws, float scale, float p_drop, uint64_t seed,
                                         const uint32_t* keep, const int64_t* fr_koff, const float* rope_cos,
                                         const float* rope_sin, int rope_period, const int* fr_nrotq,
                                         hipStream_t st) {
  if (nfr <= 0 || bpf <= 0 || H <= 0 || Lq <= 0) return 0;
  if (nfr > S2H_MAX_FRAMES || !s2h_flash_bwd_eligible(S2H_BF16, Lq, D)) return (int)hipErrorInvalidValue;
  if (keep && (D != 256 || fr_koff == nullptr)) return (int)hipErrorInvalidValue;
  if (!flash_bwd_o_aligned(o, sob, soh, sol)) return (int)hipErrorInvalidValue;
  FlashBwdArgs a = {};
  if (flash_bwd_rope_args(a, nfr, D, rope_cos, rope_sin, rope_period, fr_nrotq, nullptr) != 0)
    return (int)hipErrorInvalidValue;
  a.D = D;
  a.nfr = nfr; a.bpf = bpf;
  a.keep = keep;
  int lk_max = 0;
  if ((int64_t)Lq * std::max(sql, sgl) >= (1ll << 31)) return (int)hipErrorInvalidValue;  // 32-bit DMA offsets
  for (int f = 0; f < nfr; ++f) {
    if (fr_lk[f] <= 0 || (int64_t)fr_lk[f] * std::max(skl, svl) >= (1ll << 31)) return (int)hipErrorInvalidValue;
    a.fr_lk[f] = fr_lk[f]; a.fr_krow[f] = fr_krow[f]; a.fr_idx0[f] = fr_idx0[f];
    a.fr_koff[f] = keep ? fr_koff[f] : 0;
    lk_max = std::max(lk_max, fr_lk[f]);
  }
  a.BH = nfr * bpf * H; a.H = H; a.Lq = Lq; a.Lk = lk_max;
  a.q = (const bf16*)q; a.sqb = sqb; a.sqh = sqh; a.sql = sql;
  a.k = (const bf16*)k; a.skh = skh; a.skl = skl;
  a.v = (const bf16*)v; a.svh = svh; a.svl = svl;
  a.o = (const bf16*)o; a.sob = sob; a.soh = soh; a.sol = sol;
  a.g = (const bf16*)dout; a.sgb = sgb; a.sgh = sgh; a.sgl = sgl;
  a.dq = (bf16*)dq; a.sdqb = sdqb; a.sdqh = sdqh; a.sdql = sdql;
  a.dk = (bf16*)dk; a.sdkh = sdkh; a.sdkl = sdkl;
  a.dv = (bf16*)dv; a.sdvh = sdvh; a.sdvl = sdvl;
  a.lse = lse; a.di = di_ws;
  a.scale = scale; a.sl2 = scale * FL_LOG2E;
  a.p_drop = p_drop;
  a.thresh = (uint32_t)(p_drop * 4294967296.0);
  a.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.seed = seed;
  a.seed_off = s2h_rng_offset_ptr();
  a.splits = 1; a.tiles_per_split = (lk_max + 63) / 64;
  a.kv_splits = 1; a.kv_tiles_per_split = (Lq + 31) / 32;
  // profiler record: per-frame batch-heads and the keys summed over frames (flops = 10 * m0 m1 m2 m3)
  int64_t lk_sum = 0;
  for (int f = 0; f < nfr; ++f) lk_sum += fr_lk[f];
  const int slot = s2h_prof_begin(st, 2, (int64_t)bpf * H, Lq, lk_sum, D, 3);
  const int rc = D == 256 ? flash_bwd_launch<256>(a, st) : D > 64 ? flash_bwd_launch<128>(a, st)
                                                                  : flash_bwd_launch<64>(a, st);
  s2h_prof_end(slot, st);
  return rc;
}

// the frame-batched backward's domain for the host (bf16, head_dim 256 or 32..128, >= 128 query
// rows, flash path not switched off by s2h_attn_config)
extern "C" int s2h_flash_bwd_ok(int dt, int Lq, int D) { return s2h_flash_bwd_eligible(dt, Lq, D); }

// V-fold frame-batched backward (header comment; the forward is s2h_attn_fwd_vfold): single head,
// q / u / du / dq [nfr * bpf, Lq, ...] uniform (batch, row strides), k / m / dk PACKED per frame
// like s2h_flash_bwd_frames (row strides), u / du rows of >= 72 columns; no dV (the memory is
// detached).  Di is computed by the dQ kernel into di_ws [nfr * bpf * Lq].
extern "C" int s2h_flash_bwd_frames_vfold_rope(int nfr, int bpf, int Lq, const int* fr_lk, const int64_t* fr_krow,
                                               const uint64_t* fr_idx0, const void* q, int64_t sqb, int64_t sql,
                                               const void* k, int64_t skl, const void* mem, int64_t sml, const void* u,
                                               int64_t sub, int64_t sul, const void* du, int64_t sgb, int64_t sgl,
                                               void* dq, int64_t sdqb, int64_t sdql, void* dk, int64_t sdkl,
                                               const float* lse, float* di_ws, float scale, float p_drop, uint64_t seed,
                                               const uint32_t* keep, const int64_t* fr_koff, const float* rope_cos,
                                               const float* rope_sin, int rope_period, const int* fr_nrot,
                                               hipStream_t st);
extern "C" int s2h_flash_bwd_frames_vfold(int nfr, int bpf, int Lq, const int* fr_lk, const int64_t* fr_krow,
                                          const uint64_t* fr_idx0, const void* q, int64_t sqb, int64_t sql,
                                          const void* k, int64_t skl, const void* mem, int64_t sml, const void* u,
                                          int64_t sub, int64_t sul, const void* du, int64_t sgb, int64_t sgl, void* dq,
                                          int64_t sdqb, int64_t sdql, void* dk, int64_t sdkl, const float* lse,
                                          float* di_ws, float scale, float p_drop, uint64_t seed, const uint32_t* keep,
                                          const int64_t* fr_koff, hipStream_t st) {
  return s2h_flash_bwd_frames_vfold_rope(nfr, bpf, Lq, fr_lk, fr_krow, fr_idx0, q, sqb, sql, k, skl, mem, sml, u, sub,
                                         sul, du, sgb, sgl, dq, sdqb, sdql, dk, sdkl, lse, di_ws, scale, p_drop, seed,
                                         keep, fr_koff, nullptr, nullptr, 1, nullptr, st);
}
extern "C" int s2h_flash_bwd_frames_vfold_rope_qk(
    int nfr, int bpf, int Lq, const int* fr_lk, const int64_t* fr_krow, const uint64_t* fr_idx0, const void* q,
    int64_t sqb, int64_t sql, const void* k, int64_t skl, const void* mem, int64_t sml, const void* u, int64_t sub,
    int64_t sul, const void* du, int64_t sgb, int64_t sgl, void* dq, int64_t sdqb, int64_t sdql, void* dk,
    int64_t sdkl, const float* lse, float* di_ws, float scale, float p_drop, uint64_t seed, const uint32_t* keep,
    const int64_t* fr_koff, const float* rope_cos, const float* rope_sin, int rope_period, const int* fr_nrot,
    const int* fr_nrotq, hipStream_t st);
extern "C" int s2h_flash_bwd_frames_vfold_rope(int nfr, int bpf, int Lq, const int* fr_lk, const int64_t* fr_krow,
                                               const uint64_t* fr_idx0, const void* q, int64_t sqb, int64_t sql,
                                               const void* k, int64_t skl, const void* mem, int64_t sml, const void* u,
                                               int64_t sub, int64_t sul, const void* du, int64_t sgb, int64_t sgl,
                                               void* dq, int64_t sdqb, int64_t sdql, void* dk, int64_t sdkl,
                                               const float* lse, float* di_ws, float scale, float p_drop, uint64_t seed,
                                               const uint32_t* keep, const int64_t* fr_koff, const float* rope_cos,
                                               const float* rope_sin, int rope_period, const int* fr_nrot,
                                               hipStream_t st) {
  return s2h_flash_bwd_frames_vfold_rope_qk(nfr, bpf, Lq, fr_lk, fr_krow, fr_idx0, q, sqb, sql, k, skl, mem, sml, u,
                                            sub, sul, du, sgb, sgl, dq, sdqb, sdql, dk, sdkl, lse, di_ws, scale,
                                            p_drop, seed, keep, fr_koff, rope_cos, rope_sin, rope_period,
                                            rope_cos ? fr_nrot : nullptr, nullptr, st);
}
// + the q projection's RoPE transposed into the dQ store (query rows < fr_nrotq[f]; nullable)
extern "C" int s2h_flash_bwd_frames_vfold_rope_qk(
    int nfr, int bpf, int Lq, const int* fr_lk, const int64_t* fr_krow, const uint64_t* fr_idx0, const void* q,
    int64_t sqb, int64_t sql, const void* k, int64_t skl, const void* mem, int64_t sml, const void* u, int64_t sub,
    int64_t sul, const void* du, int64_t sgb, int64_t sgl, void* dq, int64_t sdqb, int64_t sdql, void* dk,
    int64_t sdkl, const float* lse, float* di_ws, float scale, float p_drop, uint64_t seed, const uint32_t* keep,
    const int64_t* fr_koff, const float* rope_cos, const float* rope_sin, int rope_period, const int* fr_nrot,
    const int* fr_nrotq, hipStream_t st) {
  constexpr int D = 256, DV = 64;
  if (nfr <= 0 || bpf <= 0 || Lq <= 0) return 0;
  if (nfr > S2H_MAX_FRAMES || !s2h_flash_bwd_eligible(S2H_BF16, Lq, D)) return (int)hipErrorInvalidValue;
  if (keep && fr_koff == nullptr) return (int)hipErrorInvalidValue;
  if (sul < DV + 8 || sgl < DV + 8) return (int)hipErrorInvalidValue;
  auto rows_ok = [](const void* p, int64_t sb, int64_t sl) {
    return ((uintptr_t)p & 15) == 0 && (sb & 7) == 0 && (sl & 7) == 0;
  };
  if (!rows_ok(q, sqb, sql) || !rows_ok(k, 0, skl) || !rows_ok(mem, 0, sml) || !rows_ok(u, sub, sul) ||
      !rows_ok(du, sgb, sgl) || !rows_ok(dq, sdqb, sdql) || !rows_ok(dk, 0, sdkl))
    return (int)hipErrorInvalidValue;
  FlashBwdArgs a = {};
  a.D = D;
  a.nfr = nfr; a.bpf = bpf;
  a.keep = keep;
  int lk_max = 0;
  if ((int64_t)Lq * std::max(sql, sgl) >= (1ll << 31)) return (int)hipErrorInvalidValue;  // 32-bit DMA offsets
  for (int f = 0; f < nfr; ++f) {
    if (fr_lk[f] <= 0 || (int64_t)fr_lk[f] * std::max(skl, sml) >= (1ll << 31)) return (int)hipErrorInvalidValue;
    a.fr_lk[f] = fr_lk[f]; a.fr_krow[f] = fr_krow[f]; a.fr_idx0[f] = fr_idx0[f];
    a.fr_koff[f] = keep ? fr_koff[f] : 0;
    lk_max = std::max(lk_max, fr_lk[f]);
  }
  a.BH = nfr * bpf; a.H = 1; a.Lq = Lq; a.Lk = lk_max;
  a.q = (const bf16*)q; a.sqb = sqb; a.sqh = 0; a.sql = sql;
  a.k = (const bf16*)k; a.skh = 0; a.skl = skl;
  a.v = (const bf16*)mem; a.svh = 0; a.svl = sml;
  a.o = (const bf16*)u; a.sob = sub; a.soh = 0; a.sol = sul;
  a.g = (const bf16*)du; a.sgb = sgb; a.sgh = 0; a.sgl = sgl;
  a.dq = (bf16*)dq; a.sdqb = sdqb; a.sdqh = 0; a.sdql = sdql;
  a.dk = (bf16*)dk; a.sdkh = 0; a.sdkl = sdkl;
  a.dv = nullptr;
  a.lse = lse; a.di = di_ws;
  a.scale = scale; a.sl2 = scale * FL_LOG2E;
  a.p_drop = p_drop;
  a.thresh = (uint32_t)(p_drop * 4294967296.0);
  a.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.seed = seed;
  a.seed_off = s2h_rng_offset_ptr();
  a.splits = 1; a.tiles_per_split = (lk_max + 63) / 64;
  a.kv_splits = 1; a.kv_tiles_per_split = (Lq + 31) / 32;
  if (flash_bwd_rope_args(a, nfr, D, rope_cos, rope_sin, rope_period, fr_nrotq, fr_nrot) != 0)
    return (int)hipErrorInvalidValue;
  int64_t lk_sum = 0;
  for (int f = 0; f < nfr; ++f) lk_sum += fr_lk[f];
  // profiler record: m4 = 1000 + DV (bench.py prices 2 (2 D + DV) per pair: dP over DV, dQ, dK)
  const int slot = s2h_prof_begin(st, 2, (int64_t)bpf, Lq, lk_sum, D, 1000 + DV);
  const int rc = flash_bwd_launch<D, DV>(a, st);
  s2h_prof_end(slot, st);
  return rc;
}
