// bf16 MFMA GEMM for the compute path (fwd / dgrad / wgrad of every projection): the kernel
// templates and their launchers.  The tilings are instantiated in gemm_cfg*.hip (one translation
// unit per group, compiled in parallel); gemm_bf16.hip picks one per shape.
//
// Each operand is staged into LDS in the layout its source already has, with
// 16-B vector loads and 16-B LDS stores (no transposing scalar writes):
//   K-contiguous source  -> LDS [row][k]  -> fragments by ds_read_b128
//   row-contiguous source-> LDS [k][row]  -> fragments by ds_read_b64_tr_b16
//                                            (CDNA4 transposing LDS read, two per fragment)
// so Y = X W^T (both K-contiguous), dX = dY W (W row-contiguous) and the weight
// gradient dW = dY^T X (both row-contiguous over the reduction) all run at full
// LDS bandwidth.  Rows are padded by 16 B (conflict-free ds_read_b128 and
// transposed reads).  K is split over workgroups when the output tile count cannot
// fill the 256 CUs -- the weight gradients reduce over 10^4-10^5 rows into a few
// hundred KB -- the splits' partial tiles added in fixed order by a second launch
// (fp32 atomics into the output only without the workspace).
#pragma once
#include "gemm_epi.h"

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

__device__ __forceinline__ bf16x8 tr_frag(const bf16* lds_row0, int ld, int lane) {
  // rows (8g + q) and (8g + 4 + q) of a [k][row] image, columns 4p..4p+3 of the 16-wide block
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const bf16* a0 = lds_row0 + (8 * g + q) * ld + 4 * p;
  const bf16* a1 = a0 + 4 * ld;
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a0);
  v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a1);
  typedef short v8i16 __attribute__((ext_vector_type(8)));
  v8i16 c = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, c);
}

template <int ROWS, int BK, bool KC>
struct Stage16 {
  // ROWS x BK tile; KC: source (row, k) with k contiguous -> LDS [ROWS][BK+8]
  //                !KC: source (row, k) with row contiguous -> LDS [BK][ROWS+8]
  static constexpr int NV = ROWS * BK / 8 / 256;
  static constexpr int LDS_LD = KC ? BK + 8 : ROWS + 8;
  static constexpr int LDS_ELEMS = KC ? ROWS * (BK + 8) : BK * (ROWS + 8);
  uint4 r[NV];

  __device__ __forceinline__ void load(const bf16* base, int64_t ld_row, int64_t ld_k, int row0, int k0, int nrows,
                                       int kend, bool vec_ok, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + i * 256;
      int row, k;
      if (KC) { row = v / (BK / 8); k = (v % (BK / 8)) * 8; }
      else    { k = v / (ROWS / 8); row = (v % (ROWS / 8)) * 8; }
      const int gr = row0 + row, gk = k0 + k;
      const bool full = KC ? (gr < nrows && gk + 8 <= kend) : (gk < kend && gr + 8 <= nrows);
      if (full && vec_ok) {
        r[i] = *(const uint4*)(base + (int64_t)gr * ld_row + (int64_t)gk * ld_k);
      } else {
        bf16 t[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int rr = KC ? gr : gr + j, kk = KC ? gk + j : gk;
          t[j] = (rr < nrows && kk < kend) ? base[(int64_t)rr * ld_row + (int64_t)kk * ld_k] : (bf16)0.f;
        }
        r[i] = *(const uint4*)t;
      }
    }
  }
  __device__ __forceinline__ void store(bf16* lds, int tid) {
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int v = tid + i * 256;
      if (KC) {
        const int row = v / (BK / 8), k = (v % (BK / 8)) * 8;
        *(uint4*)(lds + row * LDS_LD + k) = r[i];
      } else {
        const int k = v / (ROWS / 8), row = (v % (ROWS / 8)) * 8;
        *(uint4*)(lds + k * LDS_LD + row) = r[i];
      }
    }
  }
  // MFMA operand fragment for the 16 rows starting at `row0`, k-step offset ks (32 wide)
  __device__ __forceinline__ bf16x8 frag(const bf16* lds, int row0, int ks, int lane) const {
    if (KC) return *(const bf16x8*)(lds + (row0 + (lane & 15)) * LDS_LD + ks + (lane >> 4) * 8);
    return tr_frag(lds + ks * LDS_LD + row0, LDS_LD, lane);
  }
};

template <int BM, int BN, bool AKC, bool BKC>
__global__ __launch_bounds__(256) void gemm16_kernel(GemmArgs16 p) {
  if (p.drop_p > 0.f) p.seed = s2h_seed(p.seed, p.seed_off);
  constexpr int BK = 64;
  constexpr int WM = BM / 2, WN = BN / 2, MI = WM / 16, NI = WN / 16;
  using SA = Stage16<BM, BK, AKC>;
  using SB = Stage16<BN, BK, BKC>;
  __shared__ __attribute__((aligned(16))) bf16 smem[SA::LDS_ELEMS + SB::LDS_ELEMS];
  bf16* As = smem;
  bf16* Bs = smem + SA::LDS_ELEMS;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int bz = blockIdx.z / p.splits, split = blockIdx.z % p.splits;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const bf16* A = p.A + (int64_t)bz * p.sA;
  const bf16* B = p.B + (int64_t)bz * p.sB;
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);

  SA la;
  SB lb;
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (nk > 0) {
    la.load(A, p.lda_m, p.lda_k, m0, kbeg, p.M, kend, p.vecA, tid);
    lb.load(B, p.ldb_n, p.ldb_k, n0, kbeg, p.N, kend, p.vecB, tid);
  }
  // optional fused row sums of A (the bias gradient of a Linear's weight-gradient GEMM):
  // the first column tile's threads < BM sum their A row out of the staged LDS tile
  const bool do_rs = p.rowsum != nullptr && blockIdx.x == 0 && tid < BM;
  float rs = 0.f;
  for (int kt = 0; kt < nk; ++kt) {
    la.store(As, tid);
    lb.store(Bs, tid);
    __syncthreads();
    if (do_rs) {
#pragma unroll 8
      for (int k = 0; k < BK; ++k) rs += (float)(AKC ? As[tid * SA::LDS_LD + k] : As[k * SA::LDS_LD + tid]);
    }
    if (kt + 1 < nk) {
      la.load(A, p.lda_m, p.lda_k, m0, kbeg + (kt + 1) * BK, p.M, kend, p.vecA, tid);
      lb.load(B, p.ldb_n, p.ldb_k, n0, kbeg + (kt + 1) * BK, p.N, kend, p.vecB, tid);
    }
#pragma unroll
    for (int ks = 0; ks < BK; ks += 32) {
      bf16x8 a[MI], b[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) a[i] = la.frag(As, wm * WM + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) b[j] = lb.frag(Bs, wn * WN + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }

  // Epilogue through LDS: each wave stages one 16-row slab of its accumulators (static
  // register indices -- no scratch), then every lane finishes 4 consecutive columns of a
  // row with a compact loop and vectorised stores.
  constexpr int EPLD = WN + 4;
  constexpr int CPR = WN / 4;    // lanes per row
  constexpr int RPP = 64 / CPR;  // rows per pass
  static_assert(4 * 16 * EPLD * 4 <= (SA::LDS_ELEMS + SB::LDS_ELEMS) * 2, "epilogue staging fits the tile LDS");
  float* ep = reinterpret_cast<float*>(smem) + w * 16 * EPLD;
  const int c4 = lane % CPR, rg = lane / CPR;
  float bcol[4];
  load_bcol(p, n0 + wn * WN + 4 * c4, bcol);
  if (do_rs && m0 + tid < p.M) store_rowsum(p, bz, split, m0 + tid, rs);
  if (nk == 0) __syncthreads();
#pragma unroll
  for (int i = 0; i < MI; ++i) {
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) ep[(4 * (lane >> 4) + r) * EPLD + j * 16 + (lane & 15)] = acc[i][j][r];
    __syncthreads();
    for (int ps = 0; ps < 16 / RPP; ++ps) {
      const int rl = rg + ps * RPP;
      const float4 v4 = *(const float4*)&ep[rl * EPLD + 4 * c4];
      const int row = m0 + wm * WM + i * 16 + rl;
      if (row < p.M) epilogue4(p, bz, row, n0 + wn * WN + 4 * c4, v4, bcol, split);
    }
    __syncthreads();
  }
}

// ======================================================================================
// LDS-DMA form (the fast path).  Each operand tile is moved global -> LDS by
// global_load_lds (16 B per lane, no register staging), into a 2-deep ring with ONE
// barrier per 64-deep K step (the DMA of step k+1 is issued right after the barrier that
// retires step k, and runs under step k's MFMAs).  The DMA destination is lane-linear, so
// bank-conflict avoidance is an XOR swizzle of 16-B chunks applied to the per-lane SOURCE
// address:
//   K-contiguous operand  -> image [row][64 k] (128-B rows), chunk ^= (row >> 1) & 7,
//                            fragments by ds_read_b128
//   row-contiguous operand-> image [64 k][ROWS] (128/256-B rows), chunk ^= 2 * (k & 3),
//                            fragments by ds_read_b64_tr_b16 (two per fragment)
// Workgroups are remapped so that consecutive tiles of one row block share an XCD (L2).
// Requirements (else the register-staged kernel above runs): 16-B aligned bases, row
// strides and batch strides multiple of 8 elements, the contiguous extent of every
// operand a multiple of 8.
template <int ROWS, bool KC, int NW = 4, int BK_ = 64>
struct GImg {
  static constexpr int BK = BK_;                       // 64 or 32 k per stage
  static constexpr int RB = KC ? BK * 2 : ROWS * 2;    // bytes per image row
  static constexpr int CPR = BK / 8;                   // 16-B chunks per K-contiguous row
  static constexpr int BYTES = ROWS * BK * 2;
  static constexpr int PIECES = BYTES / 1024;          // 1-KiB DMA pieces
  static constexpr int PPW = PIECES / NW;              // per wave
  static constexpr int LPR = RB / 16;                  // lanes (16-B chunks) per image row
  static_assert(PPW >= 1 && PIECES % NW == 0, "tile too small");
  static_assert(BK == 64 || BK == 32, "stage depth");

  // K-contiguous: chunk ^= (row >> 1) mod CPR -- conflict-free ds_read_b128 fragments for
  // both 128-B (BK 64) and 64-B (BK 32) image rows (checked against the b128 lane groups)
  // Row-contiguous: a transposing fragment read's 32-lane half covers image rows k = 8g + q
  // (g = 0, 1; q = 0..3) x two 16-B chunks, so the XOR must separate k and k + 8 as well:
  //   256-/512-B rows (one row per bank row): chunk ^= 2 (k & 3) | 8 ((k >> 3) & 1)
  //   128-B rows (two rows per bank row, k & 1 picks the half): chunk ^= 2 ((k >> 1) & 1) | 4 ((k >> 3) & 1)
  // (the round-2 form 2 (k & 3) mapped k and k + 8 onto the same banks: PMC 1.65 conflict cycles
  // per LDS instruction on the weight-gradient tiles)
  __device__ static __forceinline__ int swz(int r, int c) {
    if constexpr (KC) return c ^ ((r >> 1) & (CPR - 1));
    if constexpr (RB >= 256) return c ^ ((2 * (r & 3)) | (8 * ((r >> 3) & 1)));
    return c ^ ((2 * ((r >> 1) & 1)) | (4 * ((r >> 3) & 1)));
  }
  // DMA rows/k of the tile at (row0, k0); rows >= nrows / k >= kend are clamped to valid
  // addresses (garbage rows are never stored; the K tail is zeroed in LDS afterwards)
  // (img_lds: the image's LDS byte address when the caller has it as an integer -- GDma -- else ~0u)
  __device__ static __forceinline__ void dma(char* img, const bf16* base, int64_t ld_row, int64_t ld_k, int row0, int k0,
                                            int nrows, int kend, int w, int lane, uint32_t img_lds = ~0u) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int piece = w * PPW + i;
      const int irow = piece * (1024 / RB) + lane / LPR;  // image row
      const int c = swz(irow, lane % LPR);                 // logical 16-B chunk held at this slot
      const bf16* src;
      // 32-bit element offsets: gemm_glds_ok keeps operands past 2^31 elements on the
      // register-staged kernel (a 64-bit multiply per piece was a third of the step's VALU here)
      if (KC) {
        const int r = min(row0 + irow, nrows - 1);
        const int k = k0 + 8 * c < kend ? k0 + 8 * c : k0;
        src = base + (r * (int)ld_row + k);
      } else {
        const int k = min(k0 + irow, kend - 1);
        const int r = row0 + 8 * c < nrows ? row0 + 8 * c : row0;
        src = base + (k * (int)ld_k + r);
      }
      if (img_lds != ~0u) lds_dma16_m(src, img_lds + piece * 1024);
      else lds_dma16(src, img + piece * 1024);
    }
  }
  // zero the k >= kvalid part of the image (last K step only)
  __device__ static __forceinline__ void zero_tail(char* img, int kvalid, int tid) {
    bf16* e = (bf16*)img;
    for (int i = tid; i < ROWS * BK; i += NW * 64) {
      int r, k;
      if (KC) { r = i / BK; k = i % BK; } else { k = i / ROWS; r = i % ROWS; }
      if (k < kvalid) continue;
      const int byte = KC ? r * RB + 16 * swz(r, k >> 3) + 2 * (k & 7) : k * RB + 16 * swz(k, r >> 3) + 2 * (r & 7);
      e[byte >> 1] = (bf16)0.f;
    }
  }
  // byte offset of element (row r, k) in the image
  __device__ static __forceinline__ int at(int r, int k) {
    return KC ? r * RB + 16 * swz(r, k >> 3) + 2 * (k & 7) : k * RB + 16 * swz(k, r >> 3) + 2 * (r & 7);
  }
  // MFMA operand fragment: rows rb..rb+15 of the tile, k step ks (32 deep)
  __device__ static __forceinline__ bf16x8 frag(const char* img, int rb, int ks, int lane) {
    const int g = lane >> 4;
    if (KC) {
      const int r = rb + (lane & 15);
      return *(const bf16x8*)(img + r * RB + 16 * swz(r, 4 * ks + g));
    }
    const int q = (lane >> 2) & 3, p = lane & 3;
    const int k = 32 * ks + 8 * g + q;
    const int col = rb + 4 * p;
    const char* a0 = img + k * RB + 16 * swz(k, col >> 3) + 2 * (col & 7);
    const char* a1 = img + (k + 4) * RB + 16 * swz(k + 4, col >> 3) + 2 * (col & 7);
    v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a0);
    v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)a1);
    typedef short v8i16 __attribute__((ext_vector_type(8)));
    v8i16 cat = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, cat);
  }
};

// GImg::dma with the lane-constant part of every piece's source address computed once per workgroup:
// a whole K step (k0 + BK <= kend) is one SGPR base (the operand at k0) + this lane's 32-bit byte
// offset per piece (global_load_lds_dwordx4, saddr form) -- no VALU per piece (GImg::dma spent 27 VALU
// per K step of the 64 x 64 tile on clamps and 64-bit address arithmetic, gfx950 ISA).  The ragged last
// step takes GImg::dma.  Same bytes into the same image slots.
template <class IMG, bool KC>
struct GDma {
  uint32_t off[IMG::PPW];
  __device__ __forceinline__ void init(int64_t ld_row, int64_t ld_k, int row0, int nrows, int w, int lane) {
#pragma unroll
    for (int i = 0; i < IMG::PPW; ++i) {
      const int piece = w * IMG::PPW + i;
      const int irow = piece * (1024 / IMG::RB) + lane / IMG::LPR;
      const int c = IMG::swz(irow, lane % IMG::LPR);
      if (KC) off[i] = (uint32_t)(min(row0 + irow, nrows - 1) * (int)ld_row + 8 * c) * 2u;
      else off[i] = (uint32_t)(irow * (int)ld_k + (row0 + 8 * c < nrows ? row0 + 8 * c : row0)) * 2u;
    }
  }
  // img: the stage image; img_lds: its LDS byte address
  __device__ __forceinline__ void issue(char* img, uint32_t img_lds, const bf16* base, int64_t ld_row, int64_t ld_k,
                                        int row0, int k0, int nrows, int kend, int w, int wu, int lane) const {
    if (k0 + IMG::BK > kend) {  // ragged last step: clamped addresses
      IMG::dma(img, base, ld_row, ld_k, row0, k0, nrows, kend, w, lane, img_lds);
      return;
    }
    const uint64_t bs = sgpr_base(KC ? base + k0 : base + (int64_t)k0 * ld_k);
#pragma unroll
    for (int i = 0; i < IMG::PPW; ++i) lds_dma16_sm(bs, off[i], img_lds + (wu * IMG::PPW + i) * 1024);
  }
};

// Tile BM x BN on a WGM x WGN grid of waves (each wave WM x WN of 16x16 accumulators),
// NS-deep LDS-DMA ring: at the top of K step kt the DMA of stage kt is retired with a counted
// `s_waitcnt vmcnt` that leaves the NS-2 later stages in flight (raw s_barrier, never
// __syncthreads inside the loop: its fence would drain them), then stage kt+NS-1 is issued
// into the buffer step kt-1 just finished reading.
template <int BM, int BN, int WGM, int WGN, int NS, int BK = 64>
struct GemmShape {
  static constexpr int NW = WGM * WGN, NT = NW * 64;
  static constexpr int WM = BM / WGM, WN = BN / WGN, MI = WM / 16, NI = WN / 16;
  static constexpr int STAGE_BYTES = 2 * BK * (BM + BN);
  static constexpr int MINB = NS * STAGE_BYTES <= 80 * 1024 ? 2 : 1;  // workgroups per CU the LDS allows
};

template <int BM, int BN, int WGM, int WGN, int NS, int BK, bool AKC, bool BKC, typename PA = GemmArgs16>
__global__ __launch_bounds__((GemmShape<BM, BN, WGM, WGN, NS, BK>::NT), (GemmShape<BM, BN, WGM, WGN, NS, BK>::MINB))
void gemm16g_kernel(PA p) {
  if (p.drop_p > 0.f) p.seed = s2h_seed(p.seed, p.seed_off);
  using SH = GemmShape<BM, BN, WGM, WGN, NS, BK>;
  constexpr int NW = SH::NW, NT = SH::NT;
  constexpr int WM = SH::WM, WN = SH::WN, MI = SH::MI, NI = SH::NI;
  using IA = GImg<BM, AKC, NW, BK>;
  using IB = GImg<BN, BKC, NW, BK>;
  constexpr int STAGE = IA::BYTES + IB::BYTES;
  constexpr int DPS = IA::PPW + IB::PPW;  // DMA instructions per stage per wave
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w / WGN, wn = w % WGN;
  // XCD-aware tile order (bijective remap): blocks id, id+8, ... share an XCD; give them
  // consecutive tiles of one row block so its A tile stays in that XCD's L2
  const int nwg = gridDim.x;
  int wg, zi;  // tile, z index (batch * splits + split)
  if (p.splits > 1 && !(p.dbg & 16)) {
    // split-K (the weight gradients): the same remap over the (split, tile) pairs in split-major
    // order, from the dispatch order x + gridDim.x * z -- an XCD runs whole K chunks with all their
    // tiles side by side, so each chunk of both operands is read from HBM once and shared through
    // that XCD's L2 (tile-major, every XCD read the whole of the narrow operand: the memory-attention
    // FFN weight gradients fetched ~2.8x their algorithmic bytes, profiles/r04_v8_gemm_pmc.json)
    const int total = nwg * gridDim.z, lin = blockIdx.x + nwg * blockIdx.z;
    const int x8 = lin % 8, q8 = total / 8, r8 = total % 8;
    const int w2 = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + lin / 8;
    wg = w2 % nwg;
    zi = w2 / nwg;
  } else {
    const int id = blockIdx.x;
    const int xcd = id % 8, qd = nwg / 8, rm = nwg % 8;
    wg = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + id / 8;
    zi = blockIdx.z;
  }
  const int ntn = (p.N + BN - 1) / BN;
  const int m0 = (wg / ntn) * BM, n0 = (wg % ntn) * BN;
  const int bz = zi / p.splits, split = zi % p.splits;
  const bf16* A = p.A + (int64_t)bz * p.sA;
  const bf16* B = p.B + (int64_t)bz * p.sB;
  const int kbeg = split * p.kchunk;
  const int kend = min(p.K, kbeg + p.kchunk);
  const int nk = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_rs = p.rowsum != nullptr && n0 == 0 && tid < BM;
  float rs = 0.f;
  GDma<IA, AKC> adma;
  GDma<IB, BKC> bdma;
  adma.init(p.lda_m, p.lda_k, m0, p.M, w, lane);
  bdma.init(p.ldb_n, p.ldb_k, n0, p.N, w, lane);
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const uint32_t smem_lds = lds_u32(smem);
  auto stage_dma = [&](int stg, int k) {  // dbg 64: the per-piece address arithmetic (A/B)
    char* sa = smem + stg * STAGE;
    if (p.dbg & 64) {
      IA::dma(sa, A, p.lda_m, p.lda_k, m0, k, p.M, kend, w, lane, smem_lds + stg * STAGE);
      IB::dma(sa + IA::BYTES, B, p.ldb_n, p.ldb_k, n0, k, p.N, kend, w, lane, smem_lds + stg * STAGE + IA::BYTES);
    } else {
      adma.issue(sa, smem_lds + stg * STAGE, A, p.lda_m, p.lda_k, m0, k, p.M, kend, w, wu, lane);
      bdma.issue(sa + IA::BYTES, smem_lds + stg * STAGE + IA::BYTES, B, p.ldb_n, p.ldb_k, n0, k, p.N, kend, w, wu,
                 lane);
    }
  };

#pragma unroll
  for (int st = 0; st < NS - 1; ++st) {  // prologue: stages 0 .. NS-2 in flight
    if (st < nk && !(p.dbg & 4)) stage_dma(st, kbeg + st * BK);
  }
  for (int kt = 0; kt < nk; ++kt) {
    char* sa = smem + (kt % NS) * STAGE;
    char* sb = sa + IA::BYTES;
    if (kt + NS - 2 < nk) vm_wait<(NS - 2) * DPS>();  // stage kt retired, NS-2 later ones stay in flight
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NS - 1 < nk && !(p.dbg & 4))  // refill the buffer step kt-1 read; runs under this step's MFMAs
      stage_dma((kt + NS - 1) % NS, kbeg + (kt + NS - 1) * BK);
    const int kvalid = kend - (kbeg + kt * BK);
    if (kvalid < BK) {  // K tail: zero the invalid k of both images (last step only)
      IA::zero_tail(sa, kvalid, tid);
      IB::zero_tail(sb, kvalid, tid);
      __syncthreads();
    }
    if (do_rs) {
#pragma unroll 8
      for (int k = 0; k < BK; ++k) rs += (float)*(const bf16*)(sa + IA::at(tid, k));
    }
    if (p.dbg & 2) continue;
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
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();

  if (do_rs && m0 + tid < p.M) store_rowsum(p, bz, split, m0 + tid, rs);
  if constexpr (WGN == 1 && WN >= 128 && WN % 32 == 0 && std::is_same_v<PA, GemmArgs16Ln>) {
    if (p.lnb_x != nullptr) {  // full-row tiles: LayerNorm backward epilogue
      static_assert(NW * 16 * (WN + 4) * 4 + NW * 2 * WN * 4 <= NS * STAGE, "LayerNorm-backward epilogue LDS");
      tile_epilogue_lnbwd<WM, WN, MI, NI, NW>(p, acc, smem, m0 + wm * WM, m0 / BM, lane, w);
      return;
    }
  }
  tile_epilogue<WM, WN, MI, NI, PA>(p, acc, reinterpret_cast<float*>(smem) + w * 16 * (WN + 4), bz, m0 + wm * WM,
                                n0 + wn * WN, lane, split);
}

// Short-K variant (round 4, K <= KMAX = 256 -- the step's projections, FFN linear1 forward and the
// K = 256 dgrads): the waves are stacked along M (16 rows each), so no wave reads another's A rows;
// every wave loads ITS A panel (16 rows x K) straight into registers as MFMA fragments (lane l: row
// l & 15, k 32 ks + 8 (l >> 4); one 16-B load per fragment), and only B -- shared by the 4 waves --
// goes through LDS, all of its K stages issued at once.  LDS per workgroup is B alone (BN x K x 2 B:
// 32 KB at BN 64), so 4-5 workgroups fit a CU where the two-operand 64 x 64 tile with all K in flight
// fits 2 (64 KB).  The A loads are plain (compiler-visible) loads issued before the B DMA: the one
// wait before the first MFMA (vmcnt(0)) retires both.  Requirements: K-contiguous A, K <= KMAX,
// no split-K, no fused row sums (gemm_areg_ok).
template <int BN, int KMAX, bool BKC>
__global__ __launch_bounds__(256, 4) void gemm16a_kernel(GemmArgs16 p) {
  if (p.drop_p > 0.f) p.seed = s2h_seed(p.seed, p.seed_off);
  constexpr int BM = 64, NW = 4, WM = 16, WN = BN, MI = 1, NI = BN / 16, KS = KMAX / 32, NST = KMAX / 64;
  using IB = GImg<BN, BKC, NW, 64>;
  __shared__ __attribute__((aligned(1024))) char smem[NST * IB::BYTES > NW * 16 * (WN + 4) * 4 ? NST * IB::BYTES
                                                                                              : NW * 16 * (WN + 4) * 4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nwg = gridDim.x, id = blockIdx.x;
  const int xcd = id % 8, qd = nwg / 8, rm = nwg % 8;
  const int wg = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + id / 8;
  const int ntn = (p.N + BN - 1) / BN;
  const int m0 = (wg / ntn) * BM, n0 = (wg % ntn) * BN;
  const int bz = blockIdx.z;
  const bf16* A = p.A + (int64_t)bz * p.sA;
  const bf16* B = p.B + (int64_t)bz * p.sB;
  const int K = p.K;
  const int nk = (K + 63) / 64;

  // A fragments of this wave's 16 rows (rows past M clamped; k >= K zero)
  bf16x8 af[KS];
  {
    const int r = min(m0 + w * WM + (lane & 15), p.M - 1);
    const bf16* arow = A + (int64_t)r * p.lda_m;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = 32 * ks + 8 * (lane >> 4);
      if (32 * ks < K) af[ks] = k < K ? *(const bf16x8*)(arow + k) : bf16x8{};
      else af[ks] = bf16x8{};
    }
  }
  // B: every K stage in flight at once
#pragma unroll
  for (int st = 0; st < NST; ++st)
    if (st < nk && !(p.dbg & 4)) IB::dma(smem + st * IB::BYTES, B, p.ldb_n, p.ldb_k, n0, st * 64, p.N, K, w, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (K % 64) {  // zero the K tail of the last stage's image
    IB::zero_tail(smem + (nk - 1) * IB::BYTES, K - (nk - 1) * 64, tid);
    __syncthreads();
  }
  f32x4 acc[MI][NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) acc[0][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (!(p.dbg & 2)) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (32 * ks >= K) break;
      const char* sb = smem + (ks / 2) * IB::BYTES;
      bf16x8 b[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) b[j] = IB::frag(sb, j * 16, ks % 2, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], b[j], acc[0][j], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();  // the B images are reused as the epilogue slabs
  tile_epilogue<WM, WN, MI, NI>(p, acc, reinterpret_cast<float*>(smem) + w * 16 * (WN + 4), bz, m0 + w * WM, n0,
                                lane);
}

static bool gemm_areg_ok(const GemmArgs16& a, int kmax) {
  return a.lda_k == 1 && a.K <= kmax && a.K > 0 && a.rowsum == nullptr && ((uintptr_t)a.A & 15) == 0 &&
         a.lda_m % 8 == 0 && a.K % 8 == 0 && (a.sA % 8 == 0);
}

static bool gemm_glds_ok(const GemmArgs16& a, int batch) {
  auto al = [](const void* ptr) { return ((uintptr_t)ptr & 15) == 0; };
  const bool akc = a.lda_k == 1, bkc = a.ldb_k == 1;
  const int64_t lda = akc ? a.lda_m : a.lda_k, ldb = bkc ? a.ldb_n : a.ldb_k;
  const int aext = akc ? a.K : a.M, bext = bkc ? a.K : a.N;  // contiguous extents
  // per-batch operand extents addressed with 32-bit element offsets in GImg::dma
  const int64_t aspan = akc ? (int64_t)a.M * lda : (int64_t)a.K * lda;
  const int64_t bspan = bkc ? (int64_t)a.N * ldb : (int64_t)a.K * ldb;
  return al(a.A) && al(a.B) && lda % 8 == 0 && ldb % 8 == 0 && aext % 8 == 0 && bext % 8 == 0 &&
         (batch == 1 || (a.sA % 8 == 0 && a.sB % 8 == 0)) && a.K > 0 && aspan < (1ll << 31) &&
         bspan < (1ll << 31);
}

// weight gradients over a long reduction, deterministic split-K (gemm_wgrad.hip); -1: not its case
int s2h_gemm_wgrad_det(const GemmArgs16& a, int batch, hipStream_t st);

// workgroups a split-K launch aims at (s2h_gemm_split_target; gemm_bf16.hip)
extern int g_gemm_split_target;

// the second launch of a split launch with partial tiles (gemm16.h): C (beta 0 / 1) and rowsum get the
// splits' sums in split order (gemm_bf16.hip)
int s2h_gemm_split_reduce(const GemmArgs16& a, int batch, hipStream_t st);

// split-K decision + output-group alignment for a BM x BN tiling
static void plan_splits(GemmArgs16& a, int batch, int BM, int BN, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN) * batch;
  a.splits = 1;
  a.kchunk = a.K;
  const bool plain = a.out_f32 && !a.bias && !a.R && !a.X && !a.cscale && a.drop_p == 0.f && a.act == 0 &&
                     (a.beta == 1.f || a.beta == 0.f);
  if (plain && tiles < 512 && a.K >= 1024) {
    int s = (g_gemm_split_target + tiles - 1) / tiles;
    int maxs = a.K / 512;
    if (s > maxs) s = maxs;
    // up to 256 splits: the memory K / V projection weight gradients (256 x 64 over 374k rows)
    // have 2-4 output tiles, which 64 splits left at half a wave of workgroups
    if (s > 256) s = 256;
    // deterministic (round 6): the splits' partial tiles in the workspace, added in split order by
    // gemm_split_reduce_kernel -- the float atomics' arrival order made e.g. the hypernetwork-mask
    // gradient (104 batched 1 x 32 x 65536 products, mask_decoder.py) differ between identical runs.
    // As many splits as the workspace holds; none when it holds fewer than two.
    const int64_t per = (int64_t)batch * a.M * a.N + (a.rowsum ? (int64_t)batch * a.M : 0);
    const int64_t cap = (a.dbg & 32) ? 0 : s2h_det_ws_bytes() / 4;  // dbg 32: the atomic form (A/B)
    if (cap > 0 && s > 1 && (int64_t)s * per > cap) s = (int)std::min<int64_t>(s, cap / per);
    if (s > 1) {
      a.splits = s;
      a.kchunk = ((a.K + s - 1) / s + 63) / 64 * 64;
      a.splits = (a.K + a.kchunk - 1) / a.kchunk;
      if (cap > 0) {
        a.X = s2h_det_ws((int64_t)a.splits * per * 4);
        a.sX = (int64_t)batch * a.M * a.N;
      } else if (a.beta == 0.f && a.ldc == a.N && (batch == 1 || a.sC == (int64_t)a.M * a.N)) {
        s2h_zero_f32((float*)a.C, (int64_t)batch * a.M, a.N, a.N, st);
      } else if (a.beta == 0.f) {
        for (int b = 0; b < batch; ++b) s2h_zero_f32((float*)a.C + (int64_t)b * a.sC, a.M, a.N, a.ldc, st);
      }
    }
  }
  gemm_plan_vec(a, batch);
}

template <int BM, int BN, int WGM, int WGN, int NS, int BK = 64, typename PA = GemmArgs16>
static int launch_glds(PA& a, int batch, hipStream_t st) {
  plan_splits(a, batch, BM, BN, st);
  const bool akc = a.lda_k == 1, bkc = a.ldb_k == 1;
  constexpr int NT = GemmShape<BM, BN, WGM, WGN, NS, BK>::NT;
  s2h_prof_tag(gemm_tag(BM, BN, WGM, WGN, NS, BK, akc, bkc, false, false));
  dim3 g1(((a.N + BN - 1) / BN) * ((a.M + BM - 1) / BM), 1, batch * a.splits);
  if constexpr (std::is_same_v<PA, GemmArgs16Ln>) {
    if (akc && bkc) hipLaunchKernelGGL((gemm16g_kernel<BM, BN, WGM, WGN, NS, BK, true, true, GemmArgs16Ln>), g1, dim3(NT), 0, st, a);
    else if (akc && !bkc) hipLaunchKernelGGL((gemm16g_kernel<BM, BN, WGM, WGN, NS, BK, true, false, GemmArgs16Ln>), g1, dim3(NT), 0, st, a);
    else if (!akc && bkc) hipLaunchKernelGGL((gemm16g_kernel<BM, BN, WGM, WGN, NS, BK, false, true, GemmArgs16Ln>), g1, dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((gemm16g_kernel<BM, BN, WGM, WGN, NS, BK, false, false, GemmArgs16Ln>), g1, dim3(NT), 0, st, a);
  } else {
    if (akc && bkc) hipLaunchKernelGGL((gemm16g_kernel<BM, BN, WGM, WGN, NS, BK, true, true>), g1, dim3(NT), 0, st, a);
    else if (akc && !bkc) hipLaunchKernelGGL((gemm16g_kernel<BM, BN, WGM, WGN, NS, BK, true, false>), g1, dim3(NT), 0, st, a);
    else if (!akc && bkc) hipLaunchKernelGGL((gemm16g_kernel<BM, BN, WGM, WGN, NS, BK, false, true>), g1, dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((gemm16g_kernel<BM, BN, WGM, WGN, NS, BK, false, false>), g1, dim3(NT), 0, st, a);
  }
  if (a.splits > 1 && a.X) return s2h_gemm_split_reduce(a, batch, st);
  return (int)hipGetLastError();
}

template <int BN, int KMAX = 256>
static int launch_areg(GemmArgs16& a, int batch, hipStream_t st) {
  plan_splits(a, batch, 64, BN, st);
  if (a.splits != 1) {  // not this tiling's case: undo the plan for the caller's next launcher
    a.splits = 1;
    a.kchunk = a.K;
    a.X = nullptr;
    a.sX = 0;
    return -1;
  }
  const bool bkc = a.ldb_k == 1;
  s2h_prof_tag(gemm_tag(64, BN, 4, 1, 1, 64, true, bkc, false, false, true));
  dim3 g(((a.N + BN - 1) / BN) * ((a.M + 63) / 64), 1, batch);
  if (bkc) hipLaunchKernelGGL((gemm16a_kernel<BN, KMAX, true>), g, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((gemm16a_kernel<BN, KMAX, false>), g, dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

template <int BM, int BN>
static int launch16_regs(GemmArgs16& a, int batch, hipStream_t st) {
  plan_splits(a, batch, BM, BN, st);
  const bool akc = a.lda_k == 1, bkc = a.ldb_k == 1;
  s2h_prof_tag(gemm_tag(BM, BN, 2, 2, 1, 64, akc, bkc, true, false));
  dim3 grid((a.N + BN - 1) / BN, (a.M + BM - 1) / BM, batch * a.splits);
  if (akc && bkc) hipLaunchKernelGGL((gemm16_kernel<BM, BN, true, true>), grid, dim3(256), 0, st, a);
  else if (akc && !bkc) hipLaunchKernelGGL((gemm16_kernel<BM, BN, true, false>), grid, dim3(256), 0, st, a);
  else if (!akc && bkc) hipLaunchKernelGGL((gemm16_kernel<BM, BN, false, true>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((gemm16_kernel<BM, BN, false, false>), grid, dim3(256), 0, st, a);
  if (a.splits > 1 && a.X) return s2h_gemm_split_reduce(a, batch, st);
  return (int)hipGetLastError();
}

// LDS-DMA tilings (s2h_gemm_config selects one for A/B measurements; 0 = automatic)
enum GemmCfg {
  CFG_AUTO = 0, CFG_64 = 1, CFG_128 = 2, CFG_128_NS3 = 3, CFG_256x128 = 4, CFG_256 = 5, CFG_128x256 = 6,
  CFG_128x64 = 7, CFG_64x128 = 8, CFG_64_NS3 = 9, CFG_64_K32_NS4 = 10, CFG_128x64_K32_NS3 = 11,
  CFG_128x64_K32_NS4 = 12, CFG_128x64_NS3 = 13, CFG_256x128_W4_K32_NS3 = 14, CFG_256x128_W4_K64 = 15,
  CFG_128_K32_NS3 = 16, CFG_256x64_W4_K32_NS3 = 17, CFG_64_NS4 = 18, CFG_64_K32_NS8 = 19,
  // 4 x 1 wave grids: every wave owns whole 64-column rows of the tile (128-B bf16 output rows)
  CFG_64_W41 = 20, CFG_128x64_W41 = 21, CFG_128x64_W41_K32_NS3 = 22, CFG_64_W41_NS4 = 23, CFG_128x64_W41_NS3 = 24,
  // full-row tiles (round 4): one workgroup owns 64 rows x the whole N <= 256 output width, the four
  // waves stacked along M (16 full rows each), the K ring 4 stages deep (K <= 256 in one round trip)
  CFG_64x256_W41_NS4 = 25, CFG_64x128_W41_NS4 = 26, CFG_64x256_W41_NS3 = 27, CFG_64x256_W41_K32_NS4 = 28,
  // short K (round 4): A in registers, only B through LDS (gemm16a_kernel), K <= 256
  CFG_64_AREG = 29, CFG_64x128_AREG = 30,
  CFG_REGS = 99
};
// per-translation-unit launchers: return -1 when `cfg` is not one of the unit's tilings
int gemm_cfg_launch_1(int cfg, GemmArgs16& a, int batch, hipStream_t st);
int gemm_cfg_launch_2(int cfg, GemmArgs16& a, int batch, hipStream_t st);
int gemm_cfg_launch_3(int cfg, GemmArgs16& a, int batch, hipStream_t st);
int gemm_cfg_launch_4(int cfg, GemmArgs16& a, int batch, hipStream_t st);
int gemm_cfg_launch_5(int cfg, GemmArgs16& a, int batch, hipStream_t st);
int gemm_cfg_launch_6(int cfg, GemmArgs16& a, int batch, hipStream_t st);
int gemm_cfg_launch_6_ln(int cfg, GemmArgs16Ln& a, int batch, hipStream_t st);  // the LayerNorm epilogues
int gemm_cfg_launch_7(int cfg, GemmArgs16& a, int batch, hipStream_t st);
