// Shared pieces of the flash-attention kernels (flash.hip forward, flash_bwd.hip backward):
// 16x16x32 bf16 MFMA, the XOR-swizzled [rows][DP] LDS image, LDS-DMA of one 64-row tile,
// counted vmcnt waits.
#pragma once
#include "common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef short v8i16 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

#define FL_LOG2E 1.4426950408889634f
#define FL_LN2 0.6931471805599453f
#define FL_WAVES 8
#define FL_QB (FL_WAVES * 16)  // query (or key) rows per workgroup

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Reductions over the 4 lane groups (lanes l, l ^ 16, l ^ 32, l ^ 48) on v_permlane16/32_swap (VALU
// exchanges) instead of ds_bpermute (an LDS-pipe op and an lgkmcnt wait inside the softmax).  With
// both operands the same register the swap leaves, in every lane, the two values of its pair in the
// two results, so op(r[0], r[1]) is op(own, partner) up to commutativity: the same bits as the
// __shfl_xor form.
template <int W>
__device__ __forceinline__ void lane_pair(uint32_t x, uint32_t& a, uint32_t& b) {
  if constexpr (W == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    a = r[0], b = r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    a = r[0], b = r[1];
  }
}
__device__ __forceinline__ float quad_max(float x) {
  uint32_t a, b;
  lane_pair<16>(__float_as_uint(x), a, b);
  x = fmaxf(__uint_as_float(a), __uint_as_float(b));
  lane_pair<32>(__float_as_uint(x), a, b);
  return fmaxf(__uint_as_float(a), __uint_as_float(b));
}
__device__ __forceinline__ float quad_sum(float x) {
  uint32_t a, b;
  lane_pair<16>(__float_as_uint(x), a, b);
  x = __uint_as_float(a) + __uint_as_float(b);
  lane_pair<32>(__float_as_uint(x), a, b);
  return __uint_as_float(a) + __uint_as_float(b);
}
__device__ __forceinline__ uint32_t quad_or(uint32_t x) {
  uint32_t a, b;
  lane_pair<16>(x, a, b);
  lane_pair<32>(a | b, a, b);
  return a | b;
}

template <int DP, int ROWS = 64, int NWV = FL_WAVES>
struct FlashCfg {
  static constexpr int KT = ROWS;            // rows per streamed tile
  static constexpr int ROWB = DP * 2;        // bytes per LDS row (unpadded)
  static constexpr int NCH = DP / 8;         // 16-B chunks per row
  static constexpr int RPP = 1024 / ROWB;    // rows per 1-KiB DMA piece
  static constexpr int TILEB = KT * ROWB;    // bytes per tile
  static constexpr int PIECES = TILEB / 1024;
  static constexpr int PPW = PIECES / NWV;   // pieces per wave per operand
  static constexpr int ND = DP / 16;         // 16-wide d blocks
  static constexpr int NT = DP / 32;         // 32-deep d steps
  static_assert(PPW >= 1, "tile smaller than one DMA piece per wave");
};

// XOR applied to the 16-B chunk index of image row `row`.
//  SW 0: row mod (chunks per row) -- conflict-free for 16-row ds_read_b128 fragments and for
//        transposing reads that span 8 rows x one 16-B chunk.
//  SW 1: ((row & 3) << 2) | ((row >> 2) & 3) -- for the dK/dV kernel, whose transposing reads
//        cover 4 rows x 4 consecutive chunks (32x32x16 fragments): under SW 0 the row only
//        reached the low 2 chunk bits there and every read was a 4-way bank conflict (PMC:
//        SQ_LDS_BANK_CONFLICT = half of SQ_LDS_IDX_ACTIVE).  Still conflict-free for its
//        32-row ds_read_b128 reads.  Needs >= 16 chunks per row (DP >= 128).
template <int DP, int SW = 0>
__device__ __forceinline__ int swz_x(int row) {
  if constexpr (SW == 0) return row & (DP / 8 - 1);
  static_assert(SW == 0 || DP >= 128, "SW 1 needs 16 chunks per row");
  return ((row & 3) << 2) | ((row >> 2) & 3);
}
// LDS byte offset of (row, 16-B chunk c) in a swizzled [rows][DP] image
template <int DP, int SW = 0>
__device__ __forceinline__ int swz(int row, int c) {
  return row * (DP * 2) + ((c ^ swz_x<DP, SW>(row)) << 4);
}

// DMA one tile (rows r0.., clamped to [0, nrows)) into a swizzled LDS image; the chunk
// permutation is applied to the per-lane SOURCE address (the DMA destination is lane-linear)
// ASM: issue through inline asm (lds_dma16) so the compiler's waitcnt pass does not put
// vmcnt(0) before later ds_reads; the builtin form is kept where it measured faster (the
// forward kernel, whose spilled address registers make every scratch reload a vmcnt wait).
// dvalid < DP (head dims padded to DP, e.g. Hiera's 56 in a 64 image): chunks at or past dvalid
// re-read chunk 0 of the row -- finite values the kernels cancel (zero operand columns) or never store
template <int DP, int ROWS, int NWV = FL_WAVES, bool ASM = false, int SW = 0>
__device__ __forceinline__ void dma_tile(char* lds_tile, const bf16* src, int64_t ld, int r0, int nrows, int w, int lane,
                                         int dvalid = DP) {
  using C = FlashCfg<DP, ROWS, NWV>;
#pragma unroll
  for (int i = 0; i < C::PPW; ++i) {
    const int piece = w * C::PPW + i;
    const int row = piece * C::RPP + lane / C::NCH;
    const int pos = lane % C::NCH;
    const int c = pos ^ swz_x<DP, SW>(row);
    const int gr = min(r0 + row, nrows - 1);
    const bf16* g = src + (gr * (int)ld + (c * 8 < dvalid ? c * 8 : 0));  // 32-bit offsets (host-checked)
    if constexpr (ASM)
      lds_dma16(g, lds_tile + piece * 1024);
    else
      __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)(lds_tile + piece * 1024),
                                       16, 0, 0);
  }
}

// Padded [rows][DP] image: rows of DP*2 + 32 bytes instead of an XOR swizzle.  Reads of
// 16 rows x 16-B chunks (ds_read_b128) and transposing ds_read_b64_tr_b16 reads of 8 rows
// are bank-conflict-free for DP 64 / 128 / 256 (row starts step by 8 banks), and a lane's
// addresses are affine in the column (one base register + immediate offsets) -- the
// swizzled image needs one address per column block, which in the forward kernel meant
// ~64 live address VGPRs and scratch spills inside the key loop.  The lane-linear DMA
// writes the pad slots too (with a copy of chunk 0 of the row: 6 % extra bytes).
template <int DP, int ROWS = 64, int NWV = FL_WAVES>
struct PadImg {
  static constexpr int SPR = DP / 8 + 2;               // 16-B slots per row, 2 of them pad
  static constexpr int ROWB = SPR * 16;                // bytes per row
  static constexpr int TILEB = ROWS * ROWB;
  static constexpr int PIECES = ROWS * SPR / 64;       // 1-KiB DMA pieces
  static constexpr int PPW_LO = PIECES / NWV;          // pieces of waves >= NHI
  static constexpr int NHI = PIECES % NWV;             // waves < NHI take one more
  static_assert((ROWS * SPR) % 64 == 0 && PPW_LO >= 1, "tile shape");
  __device__ static __forceinline__ int pieces(int w) { return PPW_LO + (w < NHI ? 1 : 0); }
};

// Transposing fragment read from a padded image (PadImg row pitch): A[m = column c0 + (lane & 15)]
// [k = 8g + j] with k <-> image row rbase + 4g + j (j < 4) and rbase + 16 + 4g + (j - 4) (j >= 4)
// -- tr_frag_perm's layout, conflict-free on the padded pitch.
template <int ROWB>
__device__ __forceinline__ bf16x8 tr_frag_pad(const char* img, int rbase, int c0, int lane) {
  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int r0 = rbase + 4 * g + qq;
  const int dcol = c0 + 4 * pp;
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + r0 * ROWB + 2 * dcol));
  v4i16 hv = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + (r0 + 16) * ROWB + 2 * dcol));
  v8i16 cat = __builtin_shufflevector(lo, hv, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, cat);
}

template <int DP, int ROWS = 64, int NWV = FL_WAVES, bool ASM = false>
__device__ __forceinline__ void dma_tile_pad(char* lds_tile, const bf16* src, int64_t ld, int r0, int nrows, int w,
                                             int lane, int dvalid = DP) {
  using I = PadImg<DP, ROWS, NWV>;
#pragma unroll
  for (int i = 0; i < I::PPW_LO + (I::NHI ? 1 : 0); ++i) {
    if (i == I::PPW_LO && w >= I::NHI) break;  // wave-uniform
    const int piece = w + i * NWV;
    const int slot = piece * 64 + lane;
    const int row = slot / I::SPR, c = slot % I::SPR;
    const int gr = min(r0 + row, nrows - 1);
    const bf16* g = src + (gr * (int)ld + (c < DP / 8 && c * 8 < dvalid ? c * 8 : 0));  // 32-bit offsets
    if constexpr (ASM)
      lds_dma16(g, lds_tile + piece * 1024);
    else
      __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)(lds_tile + piece * 1024),
                                       16, 0, 0);
  }
}

// dma_tile_pad with the lane-constant part of the addresses computed once (init) and the tile's row
// base a wave-uniform SGPR pair: per piece one s_mov m0 + global_load_lds_dwordx4 on a 32-bit VGPR
// byte offset (the saddr form) -- dma_tile_pad's per-tile VALU address arithmetic (a division by the
// padded row pitch, a clamp, a 64-bit multiply-add per piece) is gone.  Whole tiles only: a ragged
// last tile takes dma_tile_pad's clamped rows.  Same bytes, same LDS image.
template <int DP, int ROWS = 64, int NWV = FL_WAVES>
struct PadDma {
  using I = PadImg<DP, ROWS, NWV>;
  static constexpr int NP = I::PPW_LO + (I::NHI ? 1 : 0);
  uint32_t off[NP];
  __device__ __forceinline__ void init(int64_t ld, int w, int lane, int dvalid) {
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int slot = (w + i * NWV) * 64 + lane;
      const int row = slot / I::SPR, c = slot % I::SPR;
      off[i] = (uint32_t)((int64_t)row * ld + (c < DP / 8 && c * 8 < dvalid ? c * 8 : 0)) * 2u;
    }
  }
  // wu: the wave index as a provably wave-uniform value (readfirstlane)
  __device__ __forceinline__ void issue(char* lds_tile, const bf16* src, int64_t ld, int r0, int wu) const {
    const uint64_t bs = sgpr_base(src + (int64_t)r0 * ld);
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      if (i == I::PPW_LO && wu >= I::NHI) break;  // wave-uniform
      lds_dma16_so(bs, off[i], lds_tile + (wu + i * NWV) * 1024);
    }
  }
};

// XCD-aware work order: workgroup `id` (x fastest) runs on XCD id % 8, so round-robin placed the
// workgroups that re-read one (batch, head)'s operands -- the query blocks of a forward / dQ
// launch, the key blocks of a dK/dV launch -- on 8 different L2s.  Here XCD j runs every x (and z)
// of the batch-heads y = j, j + 8, ... in order: they share its L2, and consecutive batch-heads
// (different frames of a frame-table launch, different key counts) still spread over all XCDs.
// The host pads gridDim.y to a multiple of 8 (pad_bh8); workgroups with y >= BH return at once.
struct WgIdx {
  int x, y, z;
};
__device__ __forceinline__ WgIdx wg_xcd_order() {
  const int gx = gridDim.x, gy8 = gridDim.y / 8;
  const int id = blockIdx.x + gx * (blockIdx.y + gridDim.y * blockIdx.z);
  const int xcd = id % 8, m = id / 8;
  const int x = m % gx, t = m / gx;
  return WgIdx{x, (t % gy8) * 8 + xcd, t / gy8};
}
static inline unsigned pad_bh8(int bh) { return (unsigned)((bh + 7) / 8 * 8); }
// LDS image width of a head dim: 32..64 -> 64, 72..128 -> 128 (zero-extended columns), 256
static inline int flash_dp(int D) { return D <= 64 ? 64 : D <= 128 ? 128 : D; }

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// vmcnt(M * pieces) for a wave-uniform piece count in {LO, LO + 1}
template <int M, int LO>
__device__ __forceinline__ void wait_vmcnt_pieces(int n) {
  if (n > LO) wait_vmcnt<M * (LO + 1)>();
  else wait_vmcnt<M * LO>();
}

// vmcnt wait that leaves the K and V pieces of the next tile in flight (nk in {LOK, LOK + 1},
// nv in {LOV, LOV + 1}, wave-uniform)
template <int LOK, int LOV>
__device__ __forceinline__ void wait_kv_pieces(int nk, int nv) {
  if (nk > LOK) {
    if (nv > LOV) wait_vmcnt<LOK + LOV + 2>();
    else wait_vmcnt<LOK + LOV + 1>();
  } else {
    if (nv > LOV) wait_vmcnt<LOK + LOV + 1>();
    else wait_vmcnt<LOK + LOV>();
  }
}

// Scheduling groups for a phase of N (fragment read, MFMA) pairs: the compiler issued every
// fragment read right before its MFMA and waited for it (s_waitcnt lgkmcnt(0) per MFMA); this
// pins the order  R^PF (M R)^(N-PF) M^PF  so PF fragments are always in flight (R = LDS read
// instructions per fragment: 1 for ds_read_b128, 2 for a transposing b64 pair).  Call right after
// the phase's code, between __builtin_amdgcn_sched_barrier(0) fences.
template <int K, typename F>
__device__ __forceinline__ void sched_rep(F&& f) {
  if constexpr (K > 0) {
    f();
    sched_rep<K - 1>(f);
  }
}
// (MM: MFMAs per fragment -- 2 when one fragment feeds two 16-query sets, flash_fwd_kernel QS = 2)
template <int N, int PF, int R, int MM = 1>
__device__ __forceinline__ void sched_reads_ahead() {
  static_assert(PF <= N, "prefetch depth");
  sched_rep<PF>([] { __builtin_amdgcn_sched_group_barrier(0x100, R, 0); });
  sched_rep<N - PF>([] {
    __builtin_amdgcn_sched_group_barrier(0x008, MM, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, R, 0);
  });
  sched_rep<PF>([] { __builtin_amdgcn_sched_group_barrier(0x008, MM, 0); });
}

__device__ __forceinline__ void wg_barrier() {
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// 32x32x16 form of the transposing read: A[m = column c0 + (lane & 31)][k = 8hi + j] where
// k <-> image row  rbase + 4hi + j (j < 4)  and  rbase + 8 + 4hi + (j - 4) (j >= 4), hi = lane >> 5
// (the row order of a 32x32 accumulator's registers r = 8(j>>2) + ... within a 16-row step).
template <int DP, int SW = 0>
__device__ __forceinline__ bf16x8 tr_frag_perm32(const char* img, int rbase, int c0, int lane) {
  const int G = lane >> 4, hi = G >> 1, qq = (lane >> 2) & 3, pp = lane & 3;
  const int r0 = rbase + 4 * hi + qq;
  const int dcol = c0 + 16 * (G & 1) + 4 * pp;
  const int ch = dcol >> 3, off = (dcol & 7) * 2;
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + swz<DP, SW>(r0, ch) + off));
  v4i16 hv = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + swz<DP, SW>(r0 + 8, ch) + off));
  v8i16 cat = __builtin_shufflevector(lo, hv, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, cat);
}

// Transposing fragment read: A[m = column c0 + (lane & 15)][k = 8g + j] of a swizzled image
// where k <-> image row  rbase + 4g + j (j < 4)  and  rbase + 16 + 4g + (j - 4) (j >= 4).
template <int DP>
__device__ __forceinline__ bf16x8 tr_frag_perm(const char* img, int rbase, int c0, int lane) {
  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int r0 = rbase + 4 * g + qq;
  const int dcol = c0 + 4 * pp;
  const int ch = dcol >> 3, off = (dcol & 7) * 2;
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + swz<DP>(r0, ch) + off));
  v4i16 hv = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + swz<DP>(r0 + 16, ch) + off));
  v8i16 cat = __builtin_shufflevector(lo, hv, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, cat);
}
