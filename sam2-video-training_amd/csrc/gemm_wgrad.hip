// Weight-gradient GEMM over a long reduction with a DETERMINISTIC split-K reduction (round 5).
//
//   C[M x N] = beta C + alpha sum_k A[k, m] B[k, n]        (+ rowsum[m] += sum_k A[k, m])
//
// the layout of every Linear / 1x1-conv weight gradient dW = dY^T X (hieradet.py, memory_attention.py,
// transformer.py projections and FFNs): dY [rows, out] and X [rows, in] are both row-contiguous over the
// reduction (K = rows = 8192 .. 374192 per step).  The split-K path of gemm16g_kernel reduced its K chunks
// with fp32 atomics into C: 128 x 64 tiles (24 KB of operands per 64-deep K step for 256 MFMA cycles --
// L2-bound, 10-18 % MFMA-busy, profiles/r04_v25_gemm_pmc.json) and a summation order that changed from run
// to run.  Here:
//  * 256 x 256 / 256 x 128 / 128 x 256 / 128 x 128 / 256 x 64 / 64 x 256 tiles on 8 waves (two per SIMD), both
//    operands through the LDS-DMA images of gemm_bf16.h ([64 k][rows], transposing fragment reads), one
//    workgroup per CU: 64 KB of operands per K step against 2048 MFMA cycles per SIMD at 256 x 256;
//  * the (split, tile) pairs in split-major XCD order (gemm16g_kernel): an XCD runs whole K chunks with all
//    their tiles, each chunk fetched once into its L2;
//  * each workgroup stores its fp32 partial tile in MFMA-fragment order (16 B per lane, 1 KB per wave
//    instruction, no LDS staging) to a workspace; gemm_wg_reduce_kernel adds the partials in split order
//    0, 1, ..., S-1 and applies alpha / beta: the result is bit-identical from run to run;
//  * the bias gradient (rowsum over k of A) as MFMAs against a ones fragment, spread over the wave
//    columns of the n-tile-0 workgroups, reduced the same way.
// The workspace is registered once per process (s2h_wgrad_workspace): launches that use it must be
// ordered (one stream, or streams joined in between) -- the opt-in side stream for weight gradients
// (S2H_WGRAD_STREAM) turns this kernel off.  A shape that does not fit takes the atomic split-K path.
#include "gemm_bf16.h"

struct WgArgs {
  int M, N, K;     // M / N: extents the operand DMA covers (multiples of 8)
  int Mo, No;      // output extents (<= M / N: a row pitch padded past a 147-column im2col matrix)
  const bf16* A; int64_t lda;  // A[k * lda + m]
  const bf16* B; int64_t ldb;  // B[k * ldb + n]
  int splits, kchunk, ntm, ntn;
  float* part;     // [splits][tiles][BM * BN] in fragment order
  float* part_rs;  // [splits][ntm][BM] (nullptr: no rowsum)
};

template <int BM, int BN, int WGM, int WGN, int NS>
__global__ __launch_bounds__(WGM * WGN * 64, 1) void gemm_wg_kernel(WgArgs p) {
  constexpr int NW = WGM * WGN;
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 16, NI = WN / 16;
  constexpr int BK = 64;
  using IA = GImg<BM, false, NW, BK>;
  using IB = GImg<BN, false, NW, BK>;
  constexpr int STAGE = IA::BYTES + IB::BYTES;
  constexpr int DPS = IA::PPW + IB::PPW;  // DMA instructions per stage per wave
  constexpr int RI = (MI + WGN - 1) / WGN;  // rowsum fragments per wave: i = wn + WGN * ri < MI
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  // the wave index through an SGPR: the rowsum branches below are then scalar branches, not
  // exec-masked regions around MFMAs
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w / WGN, wn = w % WGN;
  const int tiles = p.ntm * p.ntn;
  const int total = gridDim.x, lin = blockIdx.x;
  const int x8 = lin % 8, q8 = total / 8, r8 = total % 8;
  const int w2 = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + lin / 8;
  const int tile = w2 % tiles, split = w2 / tiles;
  const int mt = tile / p.ntn, nt = tile % p.ntn;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const bool do_rs = p.part_rs != nullptr && nt == 0;

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 rsacc[RI];
#pragma unroll
  for (int r = 0; r < RI; ++r) rsacc[r] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (bf16)1.f;

  // the operands' DMA on precomputed per-lane offsets + one SGPR base per K step (GDma, gemm_bf16.h)
  GDma<IA, false> adma;
  GDma<IB, false> bdma;
  adma.init(1, p.lda, m0, p.M, w, lane);
  bdma.init(1, p.ldb, n0, p.N, w, lane);
  const uint32_t smem_lds = lds_u32(smem);
  auto stage_dma = [&](int stg, int k) {
    adma.issue(smem + stg * STAGE, smem_lds + stg * STAGE, p.A, 1, p.lda, m0, k, p.M, kend, w, w, lane);
    bdma.issue(smem + stg * STAGE + IA::BYTES, smem_lds + stg * STAGE + IA::BYTES, p.B, 1, p.ldb, n0, k, p.N, kend, w,
               w, lane);
  };
#pragma unroll
  for (int st = 0; st < NS - 1; ++st) {
    if (st < nk) stage_dma(st, kbeg + st * BK);
  }
  for (int kt = 0; kt < nk; ++kt) {
    char* sa = smem + (kt % NS) * STAGE;
    char* sb = sa + IA::BYTES;
    if (kt + NS - 2 < nk) vm_wait<(NS - 2) * DPS>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NS - 1 < nk) stage_dma((kt + NS - 1) % NS, kbeg + (kt + NS - 1) * BK);
    const int kvalid = kend - (kbeg + kt * BK);
    if (kvalid < BK) {  // K tail: zero the invalid k of both images (last step only)
      IA::zero_tail(sa, kvalid, tid);
      IB::zero_tail(sb, kvalid, tid);
      __syncthreads();
    }
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 a[MI], b[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = IA::frag(sa, wm * WM + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) b[j] = IB::frag(sb, wn * WN + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      if (do_rs) {  // workgroup-uniform: the wave's rowsum fragments read again from the image
#pragma unroll
        for (int ri = 0; ri < RI; ++ri) {
          const int i = wn + WGN * ri;
          if (i < MI) {
            const bf16x8 ar = IA::frag(sa, wm * WM + i * 16, ks, lane);
            rsacc[ri] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ar, ones, rsacc[ri], 0, 0, 0);
          }
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");

  // partial tile in fragment order: slot ((w * MI + i) * NI + j) * 64 + lane, one f32x4 per lane
  f32x4* P = reinterpret_cast<f32x4*>(p.part + ((int64_t)split * tiles + tile) * (BM * BN));
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) P[((w * MI + i) * NI + j) * 64 + lane] = acc[i][j];
  if (do_rs && (lane & 15) == 0) {
    float* R = p.part_rs + ((int64_t)split * p.ntm + mt) * BM;
#pragma unroll
    for (int ri = 0; ri < RI; ++ri) {
      const int i = wn + WGN * ri;
      if (i < MI) {
#pragma unroll
        for (int r = 0; r < 4; ++r) R[wm * WM + i * 16 + 4 * (lane >> 4) + r] = rsacc[ri][r];
      }
    }
  }
}

// The split reduction, deterministic, one launch: a 256-thread workgroup covers 256 / SL fragment slots
// x SL slices of the splits; slice q sums splits q, q + SL, ... with eight independent f32x4 chains
// (eight 16-B loads in flight per thread), the SL slice sums are added in a fixed tree through LDS and
// slice 0 writes C = beta C + alpha sum.  Workgroups past the slots do the same for the bias gradient,
// rowsum[m] += sum_s part_rs[s][m].  Every assignment is fixed by the launch shape: the result does not
// depend on timing.
template <int BM, int BN, int WGM, int WGN, int SL>
__global__ __launch_bounds__(256) void gemm_wg_reduce_kernel(WgArgs p, float* C, int64_t ldc, float alpha, float beta,
                                                             float* rowsum) {
  constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 16, NI = WN / 16;
  constexpr int SLOTS = BM * BN / 4, CPB = 256 / SL;
  __shared__ f32x4 red[SL][CPB];
  const int tiles = p.ntm * p.ntn;
  const int64_t nslots = (int64_t)tiles * SLOTS;
  const int64_t nsb = (nslots + CPB - 1) / CPB;  // workgroups of fragment slots
  const int c = threadIdx.x % CPB, q = threadIdx.x / CPB;
  const int S = p.splits;
  if ((int64_t)blockIdx.x >= nsb) {  // bias gradient
    const int64_t m = ((int64_t)blockIdx.x - nsb) * CPB + c;
    const int64_t nm = (int64_t)p.ntm * BM;
    float ch[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (m < nm) {
      int s = q;
      for (; s + 7 * SL < S; s += 8 * SL) {
#pragma unroll
        for (int j = 0; j < 8; ++j) ch[j] += p.part_rs[(int64_t)(s + j * SL) * nm + m];
      }
#pragma unroll
      for (int j = 0; j < 7; ++j)
        if (s + j * SL < S) ch[j] += p.part_rs[(int64_t)(s + j * SL) * nm + m];
    }
    float* rf = reinterpret_cast<float*>(&red[0][0]);
    rf[q * CPB + c] = ((ch[0] + ch[1]) + (ch[2] + ch[3])) + ((ch[4] + ch[5]) + (ch[6] + ch[7]));
    __syncthreads();
#pragma unroll
    for (int h = SL / 2; h >= 1; h >>= 1) {
      if (q < h) rf[q * CPB + c] += rf[(q + h) * CPB + c];
      __syncthreads();
    }
    if (q == 0 && m < nm && m < p.Mo) rowsum[m] += rf[c];
    return;
  }
  const int64_t slot = (int64_t)blockIdx.x * CPB + c;
  const f32x4* P = reinterpret_cast<const f32x4*>(p.part);
  f32x4 ch[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) ch[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (slot < nslots) {
    int s = q;
    for (; s + 7 * SL < S; s += 8 * SL) {
#pragma unroll
      for (int j = 0; j < 8; ++j) ch[j] += P[(int64_t)(s + j * SL) * nslots + slot];
    }
#pragma unroll
    for (int j = 0; j < 7; ++j)
      if (s + j * SL < S) ch[j] += P[(int64_t)(s + j * SL) * nslots + slot];
  }
  red[q][c] = ((ch[0] + ch[1]) + (ch[2] + ch[3])) + ((ch[4] + ch[5]) + (ch[6] + ch[7]));
  __syncthreads();
#pragma unroll
  for (int h = SL / 2; h >= 1; h >>= 1) {
    if (q < h) red[q][c] += red[q + h][c];
    __syncthreads();
  }
  if (q != 0 || slot >= nslots) return;
  const f32x4 v = red[0][c];
  const int tile = (int)(slot / SLOTS);
  int rem = (int)(slot % SLOTS);
  const int lane = rem % 64;
  rem /= 64;
  const int j = rem % NI;
  rem /= NI;
  const int i = rem % MI;
  const int w = rem / MI;
  const int wm = w / WGN, wn = w % WGN;
  const int mt = tile / p.ntn, nt = tile % p.ntn;
  const int row0 = mt * BM + wm * WM + i * 16 + 4 * (lane >> 4);
  const int col = nt * BN + wn * WN + j * 16 + (lane & 15);
  if (col >= p.No) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = row0 + r;
    if (row < p.Mo) {
      float* cp = C + (int64_t)row * ldc + col;
      *cp = beta != 0.f ? beta * *cp + alpha * v[r] : alpha * v[r];
    }
  }
}

template <int BM, int BN, int WGM, int WGN, int SL>
static void wg_reduce_launch(const WgArgs& p, const GemmArgs16& a, hipStream_t st) {
  constexpr int CPB = 256 / SL;
  const int64_t nslots = (int64_t)p.ntm * p.ntn * (BM * BN / 4);
  const int64_t nsb = (nslots + CPB - 1) / CPB;
  const int64_t nrb = a.rowsum ? ((int64_t)p.ntm * BM + CPB - 1) / CPB : 0;
  hipLaunchKernelGGL((gemm_wg_reduce_kernel<BM, BN, WGM, WGN, SL>), dim3((unsigned)(nsb + nrb)), dim3(256), 0, st, p,
                     (float*)a.C, a.ldc, a.alpha, a.beta, a.rowsum);
}

static float* g_wg_ws = nullptr;
static int64_t g_wg_ws_bytes = 0;
static int g_wg_kmin = 4096;  // reductions at least this long take the deterministic kernel (0: off)
static int g_wg_force_tile = -1, g_wg_force_splits = 0;  // measurement override (s2h_wgrad_force)

// Measurement knob (tools/wgrad_bench.py): force the tile (0 256x256, 1 256x128, 2 128x256, 3 128x128,
// 4 256x64, 5 64x256; -1 = the cost model) and the split count (0 = the cost model's).  Returns 0.
extern "C" int s2h_wgrad_force(int tile, int splits) {
  g_wg_force_tile = tile;
  g_wg_force_splits = splits;
  return 0;
}

// Register the weight-gradient workspace (device memory of `bytes`, owned by the caller; nullptr
// unregisters it); kmin: the shortest reduction routed here (0 turns the kernel off, -1 keeps the
// current value).  Returns 0 (hipSuccess).
extern "C" int s2h_wgrad_workspace(void* ws, int64_t bytes, int kmin) {
  g_wg_ws = (float*)ws;
  g_wg_ws_bytes = ws ? bytes : 0;
  if (kmin >= 0) g_wg_kmin = kmin;
  return 0;
}

float* s2h_det_ws(int64_t bytes) {
  return (g_wg_kmin > 0 && g_wg_ws != nullptr && bytes <= g_wg_ws_bytes) ? g_wg_ws : nullptr;
}
int64_t s2h_det_ws_bytes() { return (g_wg_kmin > 0 && g_wg_ws != nullptr) ? g_wg_ws_bytes : 0; }

template <int BM, int BN, int WGM, int WGN, int NS>
static int wg_launch(const GemmArgs16& a, int Md, int Nd, int s, hipStream_t st) {
  WgArgs p;
  p.M = Md; p.N = Nd; p.K = a.K;
  p.Mo = a.M; p.No = a.N;
  p.A = a.A; p.lda = a.lda_k;
  p.B = a.B; p.ldb = a.ldb_k;
  p.ntm = (a.M + BM - 1) / BM;
  p.ntn = (a.N + BN - 1) / BN;
  const int tiles = p.ntm * p.ntn;
  if (s < 1) s = 1;
  const int64_t tile_bytes = (int64_t)BM * BN * 4;
  const int64_t rs_bytes = a.rowsum ? (int64_t)p.ntm * BM * 4 : 0;
  const int64_t fit = g_wg_ws_bytes / ((int64_t)tiles * tile_bytes + rs_bytes);
  if (fit < 1) return -1;
  if (s > fit) s = (int)fit;
  p.kchunk = ((a.K + s - 1) / s + 63) / 64 * 64;
  p.splits = (a.K + p.kchunk - 1) / p.kchunk;
  p.part = g_wg_ws;
  p.part_rs = a.rowsum ? g_wg_ws + (int64_t)p.splits * tiles * BM * BN : nullptr;
  s2h_prof_tag(gemm_tag(BM, BN, WGM, WGN, NS, 64, false, false, false, false) | ((int64_t)1 << 41));
  hipLaunchKernelGGL((gemm_wg_kernel<BM, BN, WGM, WGN, NS>), dim3(tiles * p.splits), dim3(WGM * WGN * 64), 0, st, p);
  // reduction: SL slices per slot so that about 2^17 threads (eight 16-B loads in flight each) read
  // the partials
  const int64_t slots = (int64_t)tiles * (BM * BN / 4);
  int sl = 1;
  while (sl < 16 && slots * sl < 131072 && sl * 2 <= p.splits) sl *= 2;
  switch (sl) {
    case 16: wg_reduce_launch<BM, BN, WGM, WGN, 16>(p, a, st); break;
    case 8: wg_reduce_launch<BM, BN, WGM, WGN, 8>(p, a, st); break;
    case 4: wg_reduce_launch<BM, BN, WGM, WGN, 4>(p, a, st); break;
    case 2: wg_reduce_launch<BM, BN, WGM, WGN, 2>(p, a, st); break;
    default: wg_reduce_launch<BM, BN, WGM, WGN, 1>(p, a, st); break;
  }
  return (int)hipGetLastError();
}

// -1: not this kernel's case (the caller's split-K path runs)
int s2h_gemm_wgrad_det(const GemmArgs16& a, int batch, hipStream_t st) {
  if (g_wg_kmin <= 0 || g_wg_ws == nullptr || batch != 1) return -1;
  const bool plain = a.out_f32 && !a.bias && !a.R && !a.X && !a.cscale && a.drop_p == 0.f && a.act == 0 &&
                     (a.beta == 1.f || a.beta == 0.f) && a.rope_cos == nullptr;
  // every reduction the split-K path would split (plan_splits: < 512 tiles of 128 x 64, K >= 1024), and
  // every reduction of >= kmin rows
  const long t128x64 = (long)((a.M + 127) / 128) * ((a.N + 63) / 64);
  // round 6: also the mid-length reductions (512 <= K < 1024) of few output tiles -- the two-way decoder's
  // frame-batched weight gradients (832 token rows: 256 x 256, 256 x 2048, ...), which ran as 16-64
  // unsplit 64 x 64 workgroups of 13 K steps (~23 us each, profiles/r06_v3_shape_table.txt)
  const bool mid = a.K >= 512 && a.K < 1024 && t128x64 <= 64;
  if (!plain || (a.K < 1024 && !mid) || (a.K < g_wg_kmin && t128x64 >= 512)) return -1;
  if (a.lda_m != 1 || a.ldb_n != 1 || a.M < 16 || a.N < 64) return -1;
  // operand extents rounded up to 8 inside the row pitch (the DMA moves 8-element pieces; the extra
  // rows / columns are read, never stored)
  const int Md = (a.M + 7) / 8 * 8, Nd = (a.N + 7) / 8 * 8;
  if (Md > a.lda_k || Nd > a.ldb_k || a.lda_k % 8 || a.ldb_k % 8 || ((uintptr_t)a.A & 15) || ((uintptr_t)a.B & 15))
    return -1;
  if ((int64_t)a.K * a.lda_k >= (1ll << 31) - 8 || (int64_t)a.K * a.ldb_k >= (1ll << 31)) return -1;
  // tile and split count from a cost model (one workgroup per CU): rounds of workgroups x (the
  // K chunk's MFMA work at the tile's measured rate + a fixed prologue / epilogue) + the partial tiles
  // written and read back once each.  Per-CU rates (TF/s) fitted to tools/wgrad_sweep.py
  // (profiles/r05_v2_wgrad_sweep.log: the model's pick within ~10 % of the best forced tile x split).
  struct Cand { int bm, bn; double rate; };
  const Cand cands[] = {{256, 256, 4.2}, {256, 128, 3.4}, {128, 256, 3.4}, {128, 128, 2.4}, {256, 64, 2.0},
                        {64, 256, 2.0}};
  int best = -1, best_s = 1;
  double best_t = 1e30;
  for (int c = 0; c < 6; ++c) {
    const int bm = cands[c].bm, bn = cands[c].bn;
    const long tiles = (long)((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
    const int smax = std::max(1, std::min(256, a.K / (mid ? 128 : 512)));
    for (int sp = 1; sp <= smax; ++sp) {
      const long kchunk = ((a.K + sp - 1) / sp + 63) / 64 * 64;
      const long wgs = tiles * sp;
      const long rounds = (wgs + 255) / 256;
      const double t = rounds * (2.0 * bm * bn * kchunk / (cands[c].rate * 1e6) + 2.5) +
                       (sp > 1 ? 2.0 * wgs * bm * bn * 4 / 4.5e6 : 0.0);  // us
      if (t < best_t) { best_t = t; best = c; best_s = sp; }
    }
  }
  if (g_wg_force_tile >= 0 && g_wg_force_tile < 6) best = g_wg_force_tile;
  if (g_wg_force_splits > 0) best_s = g_wg_force_splits;
  switch (best) {
    case 0: return wg_launch<256, 256, 2, 4, 2>(a, Md, Nd, best_s, st);
    case 1: return wg_launch<256, 128, 4, 2, 2>(a, Md, Nd, best_s, st);
    case 2: return wg_launch<128, 256, 2, 4, 2>(a, Md, Nd, best_s, st);
    case 3: return wg_launch<128, 128, 2, 4, 3>(a, Md, Nd, best_s, st);
    case 4: return wg_launch<256, 64, 4, 2, 3>(a, Md, Nd, best_s, st);
    default: return wg_launch<64, 256, 1, 8, 3>(a, Md, Nd, best_s, st);
  }
}
