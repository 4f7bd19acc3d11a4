// Flash attention forward for the long-sequence attentions of the step (bf16):
// memory-attention RoPE self / cross attention (transformer.py:275-311; head_dim 256,
// Lq = 1024, Lk <= 7*1028) and Hiera global attention (hieradet.py:56-81).
//
// CDNA4 structure (one workgroup = 8 waves x 16 query rows, two waves per SIMD so one
// wave's softmax VALU work overlaps the other's MFMAs):
//   * S^T = K Q^T on v_mfma_f32_16x16x32_bf16 with the KEY on the accumulator row and
//     the QUERY on the lane: a lane owns one query row, so the online softmax (max, exp2,
//     sum) runs on lane-local values plus a 4-way cross-lane reduction.
//   * The probabilities never leave registers: converted to bf16 they ARE the B operand of
//     O^T = V^T P^T (the key order inside each 32-key MFMA step is permuted identically on
//     both operands), and O^T keeps the query on the lane, so the online-softmax rescale is
//     lane-local too (and deferred until a row max grows by 2^8).
//   * K / V tiles (64 keys) are streamed by LDS-DMA (global_load_lds, 16 B per lane) into a
//     2-deep ring; 16-B chunks are XOR-swizzled by row on the SOURCE address so the
//     lane-linear DMA image is read conflict-free by ds_read_b128 (K) and by the
//     transposing ds_read_b64_tr_b16 (V).  One barrier pair per tile, counted vmcnt.
//   * Too few query rows to fill 256 CUs (13 objects x 1024 rows = 104 query blocks) ->
//     the key range is split over workgroups; partial (O, m, l) go to a workspace and a
//     combine kernel merges them (flash-decoding style).
//   * V-fold (DV != DP, s2h_attn_fwd_vfold): the memory-attention cross-attention's values are a
//     projection of the 64-channel memory bank, V = M Wv^T + bv (memory_attention.py:66-81,
//     kv_in_dim 64).  With D = P_drop / l the dropped, normalised probabilities,
//     D V = (D M) Wv^T + rowsum(D) bv: the kernel streams M (64 wide) instead of V (256 wide) and
//     writes u' = [D M | rowsum(D) | 0 x 7] (72 columns); one [rows x 72] x [72 x 256] GEMM with
//     [Wv | bv] finishes O.  P V costs a quarter of its MFMAs and V tiles a quarter of their bytes;
//     the V projection of the whole bank (up to 7196 x 13 rows per frame and layer) disappears.
#include "flash_common.h"

int s2h_prof_begin(hipStream_t st, int kind, int64_t m0, int64_t m1, int64_t m2, int64_t m3, int64_t m4);
void s2h_prof_end(int slot, hipStream_t st);

struct FlashArgs {
  int BH, H, Lq, Lk;
  int D;  // head dim (<= DP; DP = 64 pads e.g. Hiera's 56: zero Q columns, unstored O columns)
  const bf16* q; int64_t sqb, sqh, sql;
  const bf16* k; int64_t skb, skh, skl;
  const bf16* v; int64_t svb, svh, svl;
  bf16* o; int64_t sob, soh, sol;
  float* lse;
  float sl2;  // scale * log2(e)
  float p_drop; uint32_t thresh; float inv_keep; uint64_t seed; const uint64_t* seed_off;
  uint64_t idx0;  // dropout element-index offset (this launch's frame slot in a frame-stacked batch)
  // keep bitmap (nullable): bit (k & 31) of word keep[(bh * Lq + q) * kw + k / 32] = this launch's
  // dropout keep flag of (q, k); kw = 2 * ceil(Lk / 64).  The backward reads it instead of
  // re-hashing (flash_bwd.hip).
  uint32_t* keep; int kw;
  int pair_ok;  // idx0 and Lk even: every element pair (2i, 2i + 1) of a 4-key group shares one hash
  int splits, tiles_per_split;
  float* ws_o;   // [splits][BH*Lq][DP] unnormalised partial O (splits > 1)
  float* ws_ml;  // [splits][BH*Lq][2] (m in log2 units, l)
  int prio;      // waves 4-7 at s_setprio 1 (A/B: s2h_flash_variant bit 3)
};

// dropout: none / counter hash / counter hash + keep bitmap store (template: no per-tile tests)
enum { FDROP_NONE = 0, FDROP_HASH = 1, FDROP_BITS = 2 };

// columns of the V-fold output row u' = [D M (DV) | rowsum(D) | 0 x 7]
#define FL_VFOLD_COLS(DV) ((DV) + 8)
// partial-row scalars in the key-split workspace: (m, l) or, V-fold, (m, l, rowsum(D), -)
#define FL_MLW(FOLD) ((FOLD) ? 4 : 2)

// QS: 16-query sets per wave (QS = 2: every K / V fragment read from LDS feeds two MFMAs -- the
// kernel's LDS read traffic per query halves; the workgroup covers 128 QS query rows)
// NSB: stages in the K / V ring -- 2: two barriers per tile; 3 (the V-fold default, flash_launch): tile
// it + 1 in flight across tile it's compute, one barrier per tile (the backward's round-6 ring)
template <int DP, int DROP, int DV = DP, int QS = 1, int NSB = 2>
__global__ __launch_bounds__(FL_WAVES * 64, 1) void flash_fwd_kernel(FlashArgs a) {
  static_assert(NSB == 2 || NSB == 3, "ring depth");
  constexpr bool FOLD = DV != DP;
  constexpr int QB = FL_QB * QS;
  const uint32_t hkey = DROP != FDROP_NONE ? s2h_hash_key(s2h_seed(a.seed, a.seed_off)) : 0u;
  const uint32_t t16 = a.thresh >> 16;
  using C = FlashCfg<DP>;
  using I = PadImg<DP>;   // padded K image (affine read addresses, no swizzle)
  using IV = PadImg<DV>;  // padded V image (V-fold: the 64-channel memory rows)
  constexpr int NDV = DV / 16;
  constexpr int STG = I::TILEB + IV::TILEB;
  // one LDS array: [NSB stages][K tile | V tile]
  __shared__ __attribute__((aligned(1024))) char smem[NSB * STG];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, ql = lane & 15;
  if (a.prio && w >= 4) __builtin_amdgcn_s_setprio(1);  // the second-dispatched half (MI355X_MICROARCH item 4)
  const WgIdx wi = wg_xcd_order();
  if (wi.y >= a.BH) return;  // grid padding
  const int bh = wi.y, b = bh / a.H, h = bh % a.H;
  const int split = wi.z;
  int q[QS];  // this lane's query row in each set
#pragma unroll
  for (int u = 0; u < QS; ++u) q[u] = wi.x * QB + (w * QS + u) * 16 + ql;
  const bf16* Q = a.q + b * a.sqb + h * a.sqh;
  const bf16* K = a.k + b * a.skb + h * a.skh;
  const bf16* V = a.v + b * a.svb + h * a.svh;
  const int ntiles_all = (a.Lk + C::KT - 1) / C::KT;
  const int t0 = split * a.tiles_per_split;
  const int t1 = min(ntiles_all, t0 + a.tiles_per_split);
  const int nt = t1 - t0;

  if (nt > 0) {
    dma_tile_pad<DP, 64, FL_WAVES, true>(smem, K, a.skl, t0 * C::KT, a.Lk, w, lane, a.D);
    dma_tile_pad<DV, 64, FL_WAVES, true>(smem + I::TILEB, V, a.svl, t0 * C::KT, a.Lk, w, lane, FOLD ? DV : a.D);
  }
  const int npw = I::pieces(w), npv = IV::pieces(w);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  PadDma<DP> kdma;
  PadDma<DV> vdma;
  kdma.init(a.skl, w, lane, a.D);
  vdma.init(a.svl, w, lane, FOLD ? DV : a.D);
  auto issue = [&](char* Kn, int kk) {  // the K / V tile of keys kk.. into stage Kn
    if (kk + C::KT <= a.Lk) {  // whole tile: precomputed offsets on an SGPR row base
      kdma.issue(Kn, K, a.skl, kk, wu);
      vdma.issue(Kn + I::TILEB, V, a.svl, kk, wu);
    } else {
      dma_tile_pad<DP, 64, FL_WAVES, true>(Kn, K, a.skl, kk, a.Lk, w, lane, a.D);
      dma_tile_pad<DV, 64, FL_WAVES, true>(Kn + I::TILEB, V, a.svl, kk, a.Lk, w, lane, FOLD ? DV : a.D);
    }
  };
  if (NSB == 3 && nt > 1) issue(smem + STG, (t0 + 1) * C::KT);

  // Q^T fragments (B operand of K Q^T): lane -> query q, d = 32t + 8g + j
  bf16x8 qf[QS][C::NT];
#pragma unroll
  for (int u = 0; u < QS; ++u)
#pragma unroll
    for (int t = 0; t < C::NT; ++t) {
      if (q[u] < a.Lq && 32 * t + 8 * g < a.D)
        qf[u][t] = *(const bf16x8*)(Q + (int64_t)q[u] * a.sql + 32 * t + 8 * g);
      else
        qf[u][t] = bf16x8{};
    }
  // compiler-visible vmcnt(0): retires the Q loads in the compiler's own bookkeeping too;
  // otherwise it keeps them "maybe pending" around the key loop and waits vmcnt(0) before
  // the first MFMA of every tile -- which also drains the (asm, invisible) K/V prefetch
  __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0) expcnt(7) lgkmcnt(15)

  f32x4 o[QS][NDV];  // O^T: row d = 16*db + 4g + r, column q
#pragma unroll
  for (int u = 0; u < QS; ++u)
#pragma unroll
    for (int d = 0; d < NDV; ++d) o[u][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[QS], l[QS], rd[QS];  // rd: V-fold with dropout, running rowsum of the dropped probabilities
  uint64_t drow[QS];
#pragma unroll
  for (int u = 0; u < QS; ++u) {
    m[u] = -INFINITY, l[u] = 0.f, rd[u] = 0.f;
    drow[u] = a.idx0 + ((uint64_t)bh * a.Lq + q[u]) * (uint64_t)a.Lk;
  }
  const int qq = (lane >> 2) & 3, pp = lane & 3;  // transposing-read lane roles

  int cur = 0;  // it % NSB
  for (int it = 0; it < nt; ++it) {
    const int kt = t0 + it;
    const int k0 = kt * C::KT;
    char* Kb = smem + cur * STG;
    char* Vb = Kb + I::TILEB;
    if constexpr (NSB == 2) {
      if (it + 1 < nt) {
        issue(smem + (cur ^ 1) * STG, k0 + C::KT);
        // this wave's pieces of tile `it` have landed once all but the npw + npv just issued retired
        wait_kv_pieces<I::PPW_LO, IV::PPW_LO>(npw, npv);
      } else {
        wait_vmcnt<0>();
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    } else {
      // tile it + 1 (issued after the previous barrier) stays in flight; tile it + 2 goes after this
      // barrier into the buffer every wave finished reading in iteration it - 1
      if (it + 1 < nt) wait_kv_pieces<I::PPW_LO, IV::PPW_LO>(npw, npv);
      else wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (it + 2 < nt) issue(smem + (cur == 0 ? 2 : cur - 1) * STG, k0 + 2 * C::KT);
    }
    cur = cur == NSB - 1 ? 0 : cur + 1;

    // ---- S^T = K Q^T: four 16-key blocks, key = 16*kb + 4g + r on the accumulator row
    f32x4 s[QS][4];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
      for (int u = 0; u < QS; ++u) s[u][kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int row = kb * 16 + ql;
#pragma unroll
      for (int t = 0; t < C::NT; ++t) {
        const bf16x8 kf = *(const bf16x8*)(Kb + row * I::ROWB + 16 * (4 * t + g));
#pragma unroll
        for (int u = 0; u < QS; ++u) s[u][kb] = mfma16(kf, qf[u][t], s[u][kb]);
      }
    }
    sched_reads_ahead<4 * C::NT, 4, 1, QS>();  // fragment reads 4 ahead of their MFMAs
    __builtin_amdgcn_sched_barrier(0);
    // ---- online softmax per query set (lane-local query row; keys spread over the 4 lane groups)
    bf16x8 pb[QS][2];
#pragma unroll
    for (int u = 0; u < QS; ++u) {
      float mx = -INFINITY;
      if (k0 + C::KT <= a.Lk) {  // full tile (wave-uniform): no key mask
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s[u][kb][r] *= a.sl2;
            mx = fmaxf(mx, s[u][kb][r]);
          }
      } else {
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int key = k0 + kb * 16 + 4 * g + r;
            const float x = key < a.Lk ? s[u][kb][r] * a.sl2 : -INFINITY;
            s[u][kb][r] = x;
            mx = fmaxf(mx, x);
          }
      }
      mx = quad_max(mx);
      // deferred rescale: keep the running reference max until a row's max grows by more
      // than 2^8 (p <= 256 stays exact enough in bf16 / fp32)
      const float mn = (mx > m[u] + 8.f) ? mx : m[u];
      const float alpha = (m[u] == -INFINITY) ? (mn == -INFINITY ? 1.f : 0.f) : __builtin_amdgcn_exp2f(m[u] - mn);
      const float mref = (mn == -INFINITY) ? 0.f : mn;
      m[u] = mn;
      float rs = 0.f;
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          s[u][kb][r] = __builtin_amdgcn_exp2f(s[u][kb][r] - mref);
          rs += s[u][kb][r];
        }
      float rdt = 0.f;  // V-fold: this tile's dropped-probability sum (lane part)
      if constexpr (DROP != FDROP_NONE) {
        uint32_t kbits[2] = {0u, 0u};  // this lane's keep flags: bit 16kb + 4g + e of the tile's 64 keys
        // the 4 keys of a (kb) block are consecutive: with even element indices (a.pair_ok) key pair
        // (16 kb + 4g + 2j, + 1) is hash pair pt + 8 kb + j, pt = (drow + k0) / 2 + 2g, and while no lane's
        // low word carries within the tile (wave-uniform test) the hash input lo + hi * C is xt + 8 kb + j
        // -- 32-bit adds instead of 64-bit index arithmetic and a multiply-add per hash (same hashes)
        const uint64_t pt = (drow[u] + (uint64_t)k0) / 2 + 2 * g;
        const uint32_t ptl = (uint32_t)pt;
        const bool fast = a.pair_ok && !__builtin_amdgcn_ballot_w64(ptl > 0xFFFFFFFFu - 32u);
        const uint32_t xt = ptl + (uint32_t)(pt >> 32) * 0x9E3779B9u;
        // keep masks as integers: (int)(t16 - 1 - u16) >> 31 is all ones iff u16 >= t16 (kept) -- the
        // product is masked and the bitmap bit or-ed in without materialised booleans
        const int t16m1 = (int)t16 - 1;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
          const uint64_t e0 = drow[u] + k0 + kb * 16 + 4 * g;
          uint32_t km[4];
          if (fast) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const uint32_t hsh = s2h_hash_mixed(hkey, xt + (uint32_t)(8 * kb + j));
              km[2 * j] = (uint32_t)((t16m1 - (int)(hsh & 0xFFFFu)) >> 31);
              km[2 * j + 1] = (uint32_t)((t16m1 - (int)(hsh >> 16)) >> 31);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const uint64_t pr = (e0 + e) >> 1;
              const uint32_t hsh = s2h_hash_mixed(hkey, (uint32_t)pr + (uint32_t)(pr >> 32) * 0x9E3779B9u);
              km[e] = (uint32_t)((t16m1 - (int)(((e0 + e) & 1) ? (hsh >> 16) : (hsh & 0xFFFFu))) >> 31);
            }
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            s[u][kb][e] = __uint_as_float(__float_as_uint(s[u][kb][e] * a.inv_keep) & km[e]);
            kbits[kb >> 1] |= km[e] & (1u << (16 * (kb & 1) + 4 * g + e));
          }
          if constexpr (FOLD) {
#pragma unroll
            for (int e = 0; e < 4; ++e) rdt += s[u][kb][e];
          }
        }
        if constexpr (DROP == FDROP_BITS) {  // OR the 4 key groups of the query row, one 8-B store per row and tile
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) kbits[h2] = quad_or(kbits[h2]);
          if (g == 0 && q[u] < a.Lq)
            *(uint2*)(a.keep + ((int64_t)bh * a.Lq + q[u]) * a.kw + (k0 >> 5)) = uint2{kbits[0], kbits[1]};
        }
      }
      rs = quad_sum(rs);
      l[u] = l[u] * alpha + rs;
      if constexpr (FOLD && DROP != FDROP_NONE) {
        rdt = quad_sum(rdt);
        rd[u] = rd[u] * alpha + rdt;
      }
      if (__builtin_amdgcn_ballot_w64(alpha != 1.f)) {
#pragma unroll
        for (int d = 0; d < NDV; ++d) o[u][d] *= alpha;
      }
      // P^T as the B operand: 32-key step c, k index 8g + j <-> key 32c + 16(j>>2) + 4g + (j&3)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[u][c][j] = (bf16)s[u][2 * c + (j >> 2)][j & 3];
    }

    // ---- O^T += V^T P^T, V^T fragments by transposing LDS reads (same key permutation)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int r0 = 32 * c + 4 * g + qq;
#pragma unroll
      for (int d = 0; d < NDV; ++d) {
        const int dcol = 16 * d + 4 * pp;  // first of the 4 d this lane addresses
        v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(Vb + r0 * IV::ROWB + 2 * dcol));
        v4i16 hv = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(Vb + (r0 + 16) * IV::ROWB + 2 * dcol));
        v8i16 cat = __builtin_shufflevector(lo, hv, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int u = 0; u < QS; ++u) o[u][d] = mfma16(__builtin_bit_cast(bf16x8, cat), pb[u][c], o[u][d]);
      }
    }
    sched_reads_ahead<2 * NDV, 4, 2, QS>();
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (NSB == 2) {  // every wave done reading this stage before it is refilled (LDS reads retired first)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }

#pragma unroll
  for (int u = 0; u < QS; ++u) {
    if (q[u] >= a.Lq) continue;
    if (a.splits == 1) {
      bf16* O = a.o + b * a.sob + h * a.soh + (int64_t)q[u] * a.sol;
      const float inv = l[u] > 0.f ? 1.f / l[u] : 0.f;
#pragma unroll
      for (int d = 0; d < NDV; ++d) {
        bf16 t4[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) t4[e] = (bf16)(o[u][d][e] * inv);
        if (FOLD || 16 * d + 4 * g < a.D) *(uint2*)(O + 16 * d + 4 * g) = *(const uint2*)t4;
      }
      if constexpr (FOLD) {  // rowsum(D): exactly 1 without dropout (l is the sum of the same p)
        if (g == 0) {
          bf16 t8[8] = {};
          t8[0] = (bf16)(DROP == FDROP_NONE ? (l[u] > 0.f ? 1.f : 0.f) : rd[u] * inv);
          *(uint4*)(O + DV) = *(const uint4*)t8;
        }
      }
      if (g == 0) a.lse[(int64_t)bh * a.Lq + q[u]] = (m[u] + log2f(l[u])) * FL_LN2;
    } else {
      const int64_t row = (int64_t)split * a.BH * a.Lq + (int64_t)bh * a.Lq + q[u];
      float* W = a.ws_o + row * DV;
#pragma unroll
      for (int d = 0; d < NDV; ++d)
        *(float4*)(W + 16 * d + 4 * g) = float4{o[u][d][0], o[u][d][1], o[u][d][2], o[u][d][3]};
      if (g == 0) {
        a.ws_ml[FL_MLW(FOLD) * row] = m[u];
        a.ws_ml[FL_MLW(FOLD) * row + 1] = l[u];
        if constexpr (FOLD) a.ws_ml[FL_MLW(FOLD) * row + 2] = DROP == FDROP_NONE ? l[u] : rd[u];
      }
    }
  }
}

// Merge the key-split partials: one wave per query row, DP/64 columns per lane.
// V-fold (DV != DP): the partials carry rowsum(D) beside (m, l), merged like l; the output row is
// u' = [DV columns | rowsum(D) / L | 0 x 7].
template <int DP, int DV = DP>
__global__ __launch_bounds__(256) void flash_combine_kernel(FlashArgs a) {
  constexpr bool FOLD = DV != DP;
  constexpr int MLW = FL_MLW(FOLD);
  const int lane = threadIdx.x & 63;
  const int64_t rowg = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // bh*Lq + q
  if (rowg >= (int64_t)a.BH * a.Lq) return;
  const int bh = rowg / a.Lq, q = rowg % a.Lq, b = bh / a.H, h = bh % a.H;
  const int64_t stride = (int64_t)a.BH * a.Lq;
  float M = -INFINITY;
  for (int s = 0; s < a.splits; ++s) M = fmaxf(M, a.ws_ml[MLW * (s * stride + rowg)]);
  const float Mr = M == -INFINITY ? 0.f : M;
  float L = 0.f, R = 0.f;
  constexpr int PER = DV / 64;
  float acc[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) acc[j] = 0.f;
  for (int s = 0; s < a.splits; ++s) {
    const int64_t r = s * stride + rowg;
    const float ms = a.ws_ml[MLW * r], ls = a.ws_ml[MLW * r + 1];
    const float f = ms == -INFINITY ? 0.f : exp2f(ms - Mr);
    L += ls * f;
    if constexpr (FOLD) R += a.ws_ml[MLW * r + 2] * f;
#pragma unroll
    for (int j = 0; j < PER; ++j) acc[j] += f * a.ws_o[r * DV + lane * PER + j];
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  bf16* O = a.o + b * a.sob + h * a.soh + (int64_t)q * a.sol;
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (FOLD || lane * PER + j < a.D) O[lane * PER + j] = (bf16)(acc[j] * inv);
  if constexpr (FOLD) {
    if (lane < 8) O[DV + lane] = (bf16)(lane == 0 ? R * inv : 0.f);
  }
  if (lane == 0) a.lse[rowg] = (Mr + log2f(L)) * FL_LN2;
}

// Round 6: the same merge with DV / 4 lanes per query row and 4 columns per lane, so each split's
// partial row and its (m, l[, r]) record are 16-B loads (flash_combine_kernel above gives the V-fold's
// 64-wide rows one float per lane and one row per wave); the same sums in the same order, bit for bit
// (variant2 bit 16 launches the kernel above)
// SPL > 0: the split count as a constant (the loops unroll and every load issues before the merge)
template <int DP, int DV = DP, int SPL = 0>
__global__ __launch_bounds__(256) void flash_combine_vec_kernel(FlashArgs a) {
  constexpr bool FOLD = DV != DP;
  constexpr int MLW = FL_MLW(FOLD);
  constexpr int LPR = DV / 4, RPB = 256 / LPR;
  const int sub = threadIdx.x & (LPR - 1);
  const int64_t rowg = (int64_t)blockIdx.x * RPB + threadIdx.x / LPR;  // bh*Lq + q
  if (rowg >= (int64_t)a.BH * a.Lq) return;
  const int bh = rowg / a.Lq, q = rowg % a.Lq, b = bh / a.H, h = bh % a.H;
  const int64_t stride = (int64_t)a.BH * a.Lq;
  const int ns = SPL > 0 ? SPL : a.splits;
  float M = -INFINITY;
  for (int s = 0; s < ns; ++s) M = fmaxf(M, a.ws_ml[MLW * (s * stride + rowg)]);
  const float Mr = M == -INFINITY ? 0.f : M;
  float L = 0.f, R = 0.f, acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < ns; ++s) {
    const int64_t r = s * stride + rowg;
    float ms, ls, rs = 0.f;
    if constexpr (FOLD) {
      const f32x4 ml = *(const f32x4*)(a.ws_ml + 4 * r);
      ms = ml[0]; ls = ml[1]; rs = ml[2];
    } else {
      ms = a.ws_ml[2 * r]; ls = a.ws_ml[2 * r + 1];
    }
    const float f = ms == -INFINITY ? 0.f : exp2f(ms - Mr);
    L += ls * f;
    if constexpr (FOLD) R += rs * f;
    const f32x4 o = *(const f32x4*)(a.ws_o + r * DV + sub * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] += f * o[j];
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  bf16* O = a.o + b * a.sob + h * a.soh + (int64_t)q * a.sol;
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (FOLD || sub * 4 + j < a.D) O[sub * 4 + j] = (bf16)(acc[j] * inv);
  if constexpr (FOLD) {
    if (sub < 2) {
#pragma unroll
      for (int j = 0; j < 4; ++j) O[DV + sub * 4 + j] = (bf16)(sub == 0 && j == 0 ? R * inv : 0.f);
    }
  }
  if (sub == 0) a.lse[rowg] = (Mr + log2f(L)) * FL_LN2;
}

// Split count: as many key splits as keep the grid within one round of 256 workgroups (one
// per CU), never fewer than 2 key tiles per split.  Measured on the memory-attention shapes
// (13 objects x 1024 queries x 1024..7196 keys, d 256, tools/attn_bench.py --targets): 2 splits
// 50 / 110 / 218 us against 92 / 129 / 247 us for the earlier ~3-round target (768) -- every
// extra split adds an fp32 [rows][D] partial written and re-read by the combine.
static int g_flash_fwd_target = 256;  // workgroups the key split aims at (s2h_attn_config bits 8+)

// 16-query sets per wave of the forward (flash_fwd_kernel QS): V-fold launches (bits 0-3) and plain
// launches with head dims <= 128 (bits 4-7); the 256-wide plain form keeps 1 (its O^T alone would take
// 128 VGPRs per set).  A/B knob s2h_flash_fwd_sets (S2H_FLASH_QS).
static int g_flash_qs = 1 | (1 << 4);
extern "C" int s2h_flash_fwd_sets(int mode) {
  const int prev = g_flash_qs;
  if (mode >= 0) g_flash_qs = mode;
  return prev;
}
static int flash_qs(bool vfold, int D) {
  const int v = vfold ? (g_flash_qs & 15) : D <= 128 ? ((g_flash_qs >> 4) & 15) : 1;
  return v == 2 ? 2 : 1;
}

static void flash_plan(int BH, int Lq, int Lk, int& splits, int& tps, int qs = 1) {
  const int qblocks = (Lq + FL_QB * qs - 1) / (FL_QB * qs);
  const int base = qblocks * BH;
  const int ntiles = (Lk + 63) / 64;
  int s = g_flash_fwd_target / base;
  s = std::max(1, std::min(s, ntiles / 2));
  tps = (ntiles + s - 1) / s;
  splits = (ntiles + tps - 1) / tps;
}

static int g_flash_enabled = 1;
// bits 1+ of the flash switch select older kernel variants for A/B runs (flash_bwd.hip)
int s2h_flash_variant() { return g_flash_enabled >> 1; }
// round-6 A/B bits of the non-V-fold flash kernels (default 0): 1 the self-attention dQ kernel (head dim
// 256) with 8 fragment reads ahead; 2 the head-dim <= 128 dQ kernel on the 3-stage ring with 8 ahead;
// 4 the head-dim <= 128 forward on the 3-stage ring; 8 the 32x32 dK / dV kernel (self-attention) on the
// 3-stage ring; 16 the one-row-per-wave key-split combine (flash_combine_kernel).  Returns the previous
// bits (mode < 0: query).
static int g_flash_v2 = 0;
extern "C" int s2h_flash_variant2(int mode) {
  const int prev = g_flash_v2;
  if (mode >= 0) g_flash_v2 = mode;
  return prev;
}
int s2h_flash_v2() { return g_flash_v2; }

// A/B switch for tests and benchmarks: 0 routes every attention to the generic kernels;
// 3 keeps the flash path with the one-wave-per-SIMD V-fold dK kernel (flash_bwd_dkv32_kernel).
extern "C" int s2h_attn_config(int flash_enable) {
  const int prev = g_flash_enabled | (g_flash_fwd_target << 8);
  g_flash_enabled = flash_enable & 0xff;
  g_flash_fwd_target = (flash_enable >> 8) > 0 ? (flash_enable >> 8) : 256;
  return prev;
}

// eligible: bf16, head_dim 256 or 32..128 in steps of 8 (padded to a 64 / 128 image: Hiera-B+'s
// 56, Hiera-L's 72), >= 128 query rows, 16-B aligned rows
int s2h_flash_eligible(int dt, int Lq, int D) {
  const bool dok = D == 256 || (D >= 32 && D <= 128 && D % 8 == 0);
  return g_flash_enabled && dt == S2H_BF16 && dok && Lq >= 128;
}

int64_t s2h_flash_ws_bytes(int B, int H, int Lq, int Lk, int D) {
  int splits, tps;
  flash_plan(B * H, Lq, Lk, splits, tps, flash_qs(false, D));
  if (splits <= 1) return 0;
  const int DPd = flash_dp(D);  // padded image width
  return (int64_t)splits * B * H * Lq * (DPd + 2) * 4;
}

template <int DP, int DV = DP, int QS = 1>
static int flash_launch(FlashArgs& a, hipStream_t st) {
  a.prio = (s2h_flash_variant() >> 3) & 1;
  dim3 grid((a.Lq + FL_QB * QS - 1) / (FL_QB * QS), pad_bh8(a.BH), a.splits);
  bool done = false;
  if constexpr (DV == 64 && DP == 256) {  // V-fold: the 3-stage ring (A/B: variant bit 5 the 2-stage one)
    if (((s2h_flash_variant() >> 5) & 1) == 0) {
      if (a.p_drop <= 0.f)
        hipLaunchKernelGGL((flash_fwd_kernel<DP, FDROP_NONE, DV, QS, 3>), grid, dim3(FL_WAVES * 64), 0, st, a);
      else if (a.keep)
        hipLaunchKernelGGL((flash_fwd_kernel<DP, FDROP_BITS, DV, QS, 3>), grid, dim3(FL_WAVES * 64), 0, st, a);
      else
        hipLaunchKernelGGL((flash_fwd_kernel<DP, FDROP_HASH, DV, QS, 3>), grid, dim3(FL_WAVES * 64), 0, st, a);
      done = true;
    }
  }
  if constexpr (DV == DP && DP <= 128) {
    if (s2h_flash_v2() & 4) {
      if (a.p_drop <= 0.f)
        hipLaunchKernelGGL((flash_fwd_kernel<DP, FDROP_NONE, DV, QS, 3>), grid, dim3(FL_WAVES * 64), 0, st, a);
      else if (a.keep)
        hipLaunchKernelGGL((flash_fwd_kernel<DP, FDROP_BITS, DV, QS, 3>), grid, dim3(FL_WAVES * 64), 0, st, a);
      else
        hipLaunchKernelGGL((flash_fwd_kernel<DP, FDROP_HASH, DV, QS, 3>), grid, dim3(FL_WAVES * 64), 0, st, a);
      done = true;
    }
  }
  if (!done) {
    if (a.p_drop <= 0.f)
      hipLaunchKernelGGL((flash_fwd_kernel<DP, FDROP_NONE, DV, QS>), grid, dim3(FL_WAVES * 64), 0, st, a);
    else if (a.keep)
      hipLaunchKernelGGL((flash_fwd_kernel<DP, FDROP_BITS, DV, QS>), grid, dim3(FL_WAVES * 64), 0, st, a);
    else
      hipLaunchKernelGGL((flash_fwd_kernel<DP, FDROP_HASH, DV, QS>), grid, dim3(FL_WAVES * 64), 0, st, a);
  }
  if (a.splits > 1) {
    const int64_t rows = (int64_t)a.BH * a.Lq;
    constexpr int RPB = 256 / (DV / 4);
    if ((s2h_flash_v2() & 16) || (((uintptr_t)a.ws_o | (uintptr_t)a.ws_ml) & 15))
      hipLaunchKernelGGL((flash_combine_kernel<DP, DV>), dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, a);
    else if (a.splits == 2)
      hipLaunchKernelGGL((flash_combine_vec_kernel<DP, DV, 2>), dim3((unsigned)((rows + RPB - 1) / RPB)), dim3(256), 0,
                         st, a);
    else
      hipLaunchKernelGGL((flash_combine_vec_kernel<DP, DV>), dim3((unsigned)((rows + RPB - 1) / RPB)), dim3(256), 0,
                         st, a);
  }
  return (int)hipGetLastError();
}

int s2h_flash_fwd(int B, int H, int Lq, int Lk, int D,
                  const void* q, int64_t sqb, int64_t sqh, int64_t sql,
                  const void* k, int64_t skb, int64_t skh, int64_t skl,
                  const void* v, int64_t svb, int64_t svh, int64_t svl,
                  void* o, int64_t sob, int64_t soh, int64_t sol,
                  float* lse, float scale, float p_drop, uint64_t seed, uint64_t idx0, uint32_t* keep, void* ws,
                  int64_t ws_bytes, hipStream_t st) {
  FlashArgs a = {};
  a.idx0 = idx0;
  a.D = D;
  a.keep = p_drop > 0.f ? keep : nullptr;
  a.kw = 2 * ((Lk + 63) / 64);
  a.pair_ok = ((idx0 | (uint64_t)Lk) & 1) == 0;
  a.BH = B * H; a.H = H; a.Lq = Lq; a.Lk = Lk;
  a.q = (const bf16*)q; a.sqb = sqb; a.sqh = sqh; a.sql = sql;
  a.k = (const bf16*)k; a.skb = skb; a.skh = skh; a.skl = skl;
  a.v = (const bf16*)v; a.svb = svb; a.svh = svh; a.svl = svl;
  a.o = (bf16*)o; a.sob = sob; a.soh = soh; a.sol = sol;
  a.lse = lse;
  a.sl2 = scale * FL_LOG2E;
  a.p_drop = p_drop;
  a.thresh = (uint32_t)(p_drop * 4294967296.0);
  a.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.seed = seed;
  a.seed_off = s2h_rng_offset_ptr();
  const int DPd = flash_dp(D);  // padded image width of the partials
  const int qs = flash_qs(false, D);
  flash_plan(a.BH, Lq, Lk, a.splits, a.tiles_per_split, qs);
  const int64_t need = a.splits > 1 ? (int64_t)a.splits * a.BH * Lq * (DPd + 2) * 4 : 0;
  if (need > ws_bytes || (need > 0 && ws == nullptr)) {  // no workspace: one split
    a.splits = 1;
    a.tiles_per_split = (Lk + 63) / 64;
  } else if (a.splits > 1) {
    a.ws_o = (float*)ws;
    a.ws_ml = a.ws_o + (int64_t)a.splits * a.BH * Lq * DPd;
  }
  if (D == 256) return flash_launch<256>(a, st);
  if (D > 64) return qs == 2 ? flash_launch<128, 128, 2>(a, st) : flash_launch<128>(a, st);  // 72..128
  return qs == 2 ? flash_launch<64, 64, 2>(a, st) : flash_launch<64>(a, st);                 // 32..64
}

// ---------------------------------------------------------------------------- V-fold
// Memory-attention cross-attention with the value projection folded out (header comment):
// q [B, Lq, 256], k [B, Lk, 256] (RoPE applied), m [B, Lk, 64] (the memory bank rows, the
// value projection's INPUT), single head -> u [B, Lq, >= 72]: u[:, :, 0:64] = D m,
// u[:, :, 64] = rowsum(D), u[:, :, 65:72] = 0, lse [B, Lq].  Strides in elements, (batch, row).
#define VF_D 256
#define VF_DV 64

extern "C" int64_t s2h_attn_fwd_vfold_ws_bytes(int B, int Lq, int Lk) {
  int splits, tps;
  flash_plan(B, Lq, Lk, splits, tps, flash_qs(true, VF_D));
  if (splits <= 1) return 0;
  return (int64_t)splits * B * Lq * (VF_DV + FL_MLW(true)) * 4;
}

static bool vf_rows_ok(const void* p, int64_t sb, int64_t sl) {
  return ((uintptr_t)p & 15) == 0 && (sb & 7) == 0 && (sl & 7) == 0;
}

extern "C" int s2h_attn_fwd_vfold(int B, int Lq, int Lk, const void* q, int64_t sqb, int64_t sql, const void* k, int64_t skb,
                       int64_t skl, const void* mem, int64_t smb, int64_t sml, void* u, int64_t sub, int64_t sul,
                       float* lse, float scale, float p_drop, uint64_t seed, uint64_t idx0, uint32_t* keep, void* ws,
                       int64_t ws_bytes, hipStream_t st) {
  if (B <= 0 || Lq <= 0) return 0;
  if (Lk <= 0 || !s2h_flash_eligible(S2H_BF16, Lq, VF_D) || sul < FL_VFOLD_COLS(VF_DV)) return (int)hipErrorInvalidValue;
  if (!vf_rows_ok(q, sqb, sql) || !vf_rows_ok(k, skb, skl) || !vf_rows_ok(mem, smb, sml) || !vf_rows_ok(u, sub, sul))
    return (int)hipErrorInvalidValue;
  if ((int64_t)Lk * std::max(skl, sml) >= (1ll << 31)) return (int)hipErrorInvalidValue;  // 32-bit DMA offsets
  FlashArgs a = {};
  a.idx0 = idx0;
  a.D = VF_D;
  a.keep = p_drop > 0.f ? keep : nullptr;
  a.kw = 2 * ((Lk + 63) / 64);
  a.pair_ok = ((idx0 | (uint64_t)Lk) & 1) == 0;
  a.BH = B; a.H = 1; a.Lq = Lq; a.Lk = Lk;
  a.q = (const bf16*)q; a.sqb = sqb; a.sqh = 0; a.sql = sql;
  a.k = (const bf16*)k; a.skb = skb; a.skh = 0; a.skl = skl;
  a.v = (const bf16*)mem; a.svb = smb; a.svh = 0; a.svl = sml;
  a.o = (bf16*)u; a.sob = sub; a.soh = 0; a.sol = sul;
  a.lse = lse;
  a.sl2 = scale * FL_LOG2E;
  a.p_drop = p_drop;
  a.thresh = (uint32_t)(p_drop * 4294967296.0);
  a.inv_keep = p_drop > 0.f ? 1.f / (1.f - p_drop) : 1.f;
  a.seed = seed;
  a.seed_off = s2h_rng_offset_ptr();
  const int qs = flash_qs(true, VF_D);
  flash_plan(a.BH, Lq, Lk, a.splits, a.tiles_per_split, qs);
  const int64_t need = a.splits > 1 ? (int64_t)a.splits * a.BH * Lq * (VF_DV + FL_MLW(true)) * 4 : 0;
  if (need > ws_bytes || (need > 0 && ws == nullptr)) {
    a.splits = 1;
    a.tiles_per_split = (Lk + 63) / 64;
  } else if (a.splits > 1) {
    a.ws_o = (float*)ws;
    a.ws_ml = a.ws_o + (int64_t)a.splits * a.BH * Lq * VF_DV;
  }
  // profiler record: m4 = 1000 + DV marks the folded value width (bench.py prices 2 (D + DV) per pair)
  const int slot = s2h_prof_begin(st, 1, (int64_t)B, Lq, Lk, VF_D, 1000 + VF_DV);
  const int rc = qs == 2 ? flash_launch<VF_D, VF_DV, 2>(a, st) : flash_launch<VF_D, VF_DV>(a, st);
  s2h_prof_end(slot, st);
  return rc;
}
