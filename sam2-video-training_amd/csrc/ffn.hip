// Memory-attention FFN backward, input-gradient side, as ONE kernel (round 5).
//
// Reference: memory_attention.py:97, y = linear2(dropout(relu(linear1(x)))).  With hid = the saved
// linear2 input (= dropout(relu(pre)), zero exactly where the ReLU or the dropout cut) and dY the
// gradient at linear2's output, the frame-batched backward (R = 93 184 rows per layer at the bench
// shape) needs
//   dH = (dY W2) * [hid > 0] / keep       (linear1's pre-activation gradient; its weight gradient and
//                                          bias gradient read it: dW1 = dH^T X, db1 = colsum dH)
//   dX = dH W1                            (the gradient at linear1's input, i.e. norm3's output)
// The unfused path ran two GEMMs: dH (93184 x 2048 x 256, the mask read from hid in the epilogue) and
// dX (93184 x 256 x 2048), the second re-reading the 381 MB dH the first had written.  Here a
// workgroup owns BM rows (128; 64 when there are too few rows to fill the chip) and walks the hidden
// units in chunks of 128:
//   phase A  dH_c^T = W2[:, c]^T dY^T     (K = 256; dY's BM x 256 tile stays in LDS for all chunks)
//   mask     [hid > 0] / keep, bf16, in place: the chunk's hid tile is LDS-DMA'd into the very image
//            phase C reads dH from (same layout), each lane overwriting the 4 elements it read
//   store    the chunk to dH, 16 B per lane
//   phase C  dX^T += W1[c, :]^T dH_c^T    (K = 128; accumulated in registers over all chunks)
// Both products are computed transposed so each lane holds 4 consecutive columns of one row (8-byte
// LDS accesses, no shuffles).  The weight operands stream through one 4-deep LDS-DMA ring of 16 KB
// steps: per chunk four 64-deep W2 steps (128 hidden x 64) and four 32-deep W1 steps (32 x 256); the
// chunk's hid tile rides with its last W2 step.  Four waves, each a 64 x BM/2 (phase A) and
// 128 x BM/2 (phase C) tile; DMA sources are per-lane 32-bit offsets from wave-uniform SGPR bases.
// Measured on the bench shape (tools/ffn_bench.py): BM = 64 374 us, BM = 128 294 us, against 456 us
// for the two GEMMs it replaces.  What bounds it is data movement, not the MFMAs (with every MFMA
// switched off it still took ~300 us): the 2 MB of weights are re-read through L2 once per row tile
// (1.5 GB), hid is read (381 MB) and dH written (381 MB) once, and the per-chunk mask/store epilogue
// runs with the MFMA pipes idle.  (A variant with dY's fragments held in registers and a 6-deep ring
// was slower: 321 us, accumulator copies between AGPRs and VGPRs.)  dH is never read back from HBM.
#include "gemm_bf16.h"
#include "flash_common.h"

namespace {

constexpr int FFN_D = 256;   // d_model (memory attention)
constexpr int FFN_HC = 128;  // hidden units per chunk
constexpr int FFN_NS = 4;    // ring steps
constexpr int FFN_RING = 16 * 1024;

using IW2 = GImg<FFN_HC, false, 4, 64>;    // W2 step: [64 k (d)][128 h], A operand of phase A
using IW1 = GImg<FFN_D, false, 4, 32>;     // W1 step: [32 k (h)][256 n], A operand of phase C
static_assert(IW2::BYTES == FFN_RING && IW1::BYTES == FFN_RING, "ring step size");
static_assert(IW2::PPW == 4 && IW1::PPW == 4, "DMA pieces per wave");

template <int BM>
struct FfnShape {
  using IDY = GImg<BM, true, 4, 64>;   // dY tile: 4 x [BM r][64 k (d)], B operand of phase A
  using IDH = GImg<BM, true, 4, 64>;   // hid tile -> dH chunk (in place): 2 x [BM r][64 k (h)]
  static constexpr int NI = BM / 32;   // 16-row blocks per wave (r)
  static constexpr int OFF_DY = 0;
  static constexpr int OFF_RING = OFF_DY + 4 * IDY::BYTES;
  static constexpr int OFF_DH = OFF_RING + FFN_NS * FFN_RING;
  static constexpr int OFF_HID = OFF_DH;
  static constexpr int LDS = OFF_DH + 2 * IDH::BYTES;  // 160 KB at BM = 128
  static constexpr int HIDW = 2 * IDH::PPW;            // hid DMA pieces per wave
  static constexpr int STW = BM / 16;                  // dH 16-B stores per lane per chunk
  static constexpr int XLD = FFN_D * 2 + 16;           // dX staging row pitch (bytes), over the whole LDS
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(BM * XLD <= LDS, "dX staging fits");
  static_assert(FFN_NS == 4, "the hid tile (DMA'd into the dH image) goes out with step 3 = at the top of step 0, "
                "after every wave has finished the previous chunk's phase C");
};

struct FfnArgs {
  int R, H;                  // rows, hidden width (a multiple of 128)
  const bf16* dy; int64_t lddy;
  const bf16* w2;            // [256][H]   (linear2.weight, row-major)
  const bf16* w1;            // [H][256]   (linear1.weight, row-major)
  const bf16* hid; int64_t ldh;
  bf16* dh; int64_t lddh;
  bf16* dx; int64_t lddx;
  float alpha;               // 1 / keep
};

// Per-lane byte offsets of this wave's DMA pieces (the images' swizzled source addresses, GImg::dma's
// arithmetic done once: whole tiles, no clamping); each step then issues from a wave-uniform SGPR base
// (global_load_lds saddr form).  Keeping one 64-bit address per step x piece live across the loop was
// what spilled registers.
template <int BM>
struct FfnDma {
  using IDH = typename FfnShape<BM>::IDH;
  uint32_t w2[4], w1[4], h[IDH::PPW];
  __device__ __forceinline__ void init(const FfnArgs& p, int w, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int piece = w * 4 + i;
      int k = piece * (1024 / IW2::RB) + lane / IW2::LPR;
      w2[i] = (uint32_t)(k * p.H + 8 * IW2::swz(k, lane % IW2::LPR)) * 2u;
      k = piece * (1024 / IW1::RB) + lane / IW1::LPR;
      w1[i] = (uint32_t)(k * FFN_D + 8 * IW1::swz(k, lane % IW1::LPR)) * 2u;
    }
#pragma unroll
    for (int i = 0; i < IDH::PPW; ++i) {
      const int piece = w * IDH::PPW + i;
      const int r = piece * (1024 / IDH::RB) + lane / IDH::LPR;
      h[i] = (uint32_t)(r * (int)p.ldh + 8 * IDH::swz(r, lane % IDH::LPR)) * 2u;
    }
  }
};

// ring step q: chunk q / 8; steps 0-3 of a chunk are W2 (the chunk's hid tile with step 3), 4-7 W1
template <int BM>
__device__ __forceinline__ void ffn_issue(char* smem, const FfnArgs& p, const FfnDma<BM>& d, int q, int r0, int w) {
  using S = FfnShape<BM>;
  using IDH = typename S::IDH;
  char* slot = smem + S::OFF_RING + (q % FFN_NS) * FFN_RING;
  const int c = q >> 3, sub = q & 7;
  if (sub < 4) {
    const uint64_t b = sgpr_base(p.w2 + (int64_t)sub * 64 * p.H + c * FFN_HC);
#pragma unroll
    for (int i = 0; i < 4; ++i) lds_dma16_so(b, d.w2[i], slot + (w * 4 + i) * 1024);
    if (sub == 3) {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint64_t hb = sgpr_base(p.hid + (int64_t)r0 * p.ldh + c * FFN_HC + s * 64);
#pragma unroll
        for (int i = 0; i < IDH::PPW; ++i)
          lds_dma16_so(hb, d.h[i], smem + S::OFF_HID + s * IDH::BYTES + (w * IDH::PPW + i) * 1024);
      }
    }
  } else {
    const uint64_t b = sgpr_base(p.w1 + (int64_t)(c * FFN_HC + (sub - 4) * 32) * FFN_D);
#pragma unroll
    for (int i = 0; i < 4; ++i) lds_dma16_so(b, d.w1[i], slot + (w * 4 + i) * 1024);
  }
}

// vmcnt allowance at the top of ring step SUB: the DMAs of the NS-2 later steps in flight (4 per wave,
// + the hid tile on step 3) + the dH stores younger than this step's DMA.  Step q's DMA is issued at the
// top of step q-NS+1, a chunk's stores at the end of its step 3: they are younger than q's DMA and
// already issued for this chunk's steps 4 .. NS+2 (NS+2 >= 8: the next chunk's first steps too).
template <int BM>
constexpr int ffn_cnt(int x) { return 4 + ((x % 8) == 3 ? FfnShape<BM>::HIDW : 0); }
template <int BM, int SUB>
__device__ __forceinline__ void ffn_wait(bool first_chunk, bool last_chunk) {
  using S = FfnShape<BM>;
  constexpr int later = [] { int n = 0; for (int i = 1; i <= FFN_NS - 2; ++i) n += ffn_cnt<BM>(SUB + i); return n; }();
  constexpr int own = (SUB >= 4 && SUB <= FFN_NS + 2) ? S::STW : 0;
  constexpr bool prev = SUB + 8 <= FFN_NS + 2;  // the previous chunk's stores (none before chunk 1)
  if (SUB + FFN_NS - 2 >= 8 && last_chunk) vm_wait<0>();  // no next chunk: fewer DMAs in flight
  else if (prev && !first_chunk) vm_wait<later + own + S::STW>();
  else vm_wait<later + own>();
}

__device__ __forceinline__ void raw_barrier_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int BM>
__global__ __launch_bounds__(256, 1) void ffn_bwd_dgrad_kernel(FfnArgs p) {
  using S = FfnShape<BM>;
  using IDH = typename S::IDH;
  constexpr int NI = S::NI;
  __shared__ __attribute__((aligned(1024))) char smem[S::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r0 = blockIdx.x * BM;
  const int nchunk = p.H / FFN_HC;
  const int nq = nchunk * 8;
  // phase A (dH^T, 128 h x BM r) and phase C (dX^T, 256 n x BM r): waves 2 (h / n) x 2 (r)
  const int wc = w & 1, wr = w >> 1;
  constexpr int WR = BM / 2;

  using IDY = typename S::IDY;
#pragma unroll
  for (int s = 0; s < 4; ++s) IDY::dma(smem + S::OFF_DY + s * IDY::BYTES, p.dy, p.lddy, 1, r0, s * 64, p.R, FFN_D, w, lane);
  FfnDma<BM> dma;
  dma.init(p, w, lane);
#pragma unroll
  for (int q = 0; q < FFN_NS - 1; ++q) ffn_issue<BM>(smem, p, dma, q, r0, w);

  f32x4 acc1[4][NI], acc2[8][NI];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int c = 0; c < nchunk; ++c) {
    const bool last = c + 1 == nchunk;
    static_for<0, 8>([&](auto subc) {
      constexpr int SUB = decltype(subc)::value;
      const int q = c * 8 + SUB;
      ffn_wait<BM, SUB>(c == 0, last);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (q + FFN_NS - 1 < nq) ffn_issue<BM>(smem, p, dma, q + FFN_NS - 1, r0, w);
      const char* slot = smem + S::OFF_RING + (q % FFN_NS) * FFN_RING;
      if constexpr (SUB < 4) {
        if constexpr (SUB == 0) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        const char* dyi = smem + S::OFF_DY + SUB * IDY::BYTES;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          bf16x8 a[4], b[NI];
#pragma unroll
          for (int i = 0; i < 4; ++i) a[i] = IW2::frag(slot, wc * 64 + i * 16, ks, lane);
#pragma unroll
          for (int j = 0; j < NI; ++j) b[j] = IDY::frag(dyi, wr * WR + j * 16, ks, lane);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc1[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc1[i][j], 0, 0, 0);
        }
        if constexpr (SUB == 3) {
          // the hid tile (step 3's DMA, retired at the top of this step) -> mask + scale -> bf16 dH image
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) {
              const int h = wc * 64 + i * 16 + 4 * (lane >> 4);
              const int r = wr * WR + j * 16 + (lane & 15);
              const int off = (h >> 6) * IDH::BYTES + IDH::at(r, h & 63);
              const uint2 hv = *(const uint2*)(smem + S::OFF_HID + off);
              const bf16* hb = (const bf16*)&hv;
              bf16 t[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) t[e] = (bf16)((float)hb[e] > 0.f ? p.alpha * acc1[i][j][e] : 0.f);
              *(uint2*)(smem + S::OFF_DH + off) = *(const uint2*)t;
            }
          // raw barrier (a __syncthreads fence would also drain the ring's DMAs in flight)
          raw_barrier_lds();
          // dH chunk to global: BM rows x 16 chunks of 16 B
#pragma unroll
          for (int e = 0; e < S::STW; ++e) {
            const int id = tid + 256 * e;
            const int r = id >> 4, kc = id & 15;
            const uint4 v = *(const uint4*)(smem + S::OFF_DH + (kc >> 3) * IDH::BYTES + IDH::at(r, (kc & 7) * 8));
            st16_nt(p.dh + (int64_t)(r0 + r) * p.lddh + c * FFN_HC + 8 * kc, v, false);
          }
        }
      } else {
        constexpr int KS = SUB - 4;  // 32-deep step of the chunk's 128 hidden units
        const char* dhi = smem + S::OFF_DH + (KS >> 1) * IDH::BYTES;
        bf16x8 b[NI];
#pragma unroll
        for (int j = 0; j < NI; ++j) b[j] = IDH::frag(dhi, wr * WR + j * 16, KS & 1, lane);
#pragma unroll
        for (int ih = 0; ih < 2; ++ih) {  // A fragments four at a time (register budget: dY's live in VGPRs)
          bf16x8 a[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) a[i] = IW1::frag(slot, wc * 128 + (ih * 4 + i) * 16, 0, lane);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j)
              acc2[ih * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc2[ih * 4 + i][j], 0, 0, 0);
        }
      }
    });
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // dX: 4 consecutive n of one row per lane -> bf16 staging [BM r][256 n] (padded rows) over the LDS
  char* xs = smem;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = wc * 128 + i * 16 + 4 * (lane >> 4);
      const int r = wr * WR + j * 16 + (lane & 15);
      bf16 t[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] = (bf16)acc2[i][j][e];
      *(uint2*)(xs + r * S::XLD + n * 2) = *(const uint2*)t;
    }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < BM / 8; ++e) {
    const int id = tid + 256 * e;
    const int r = id >> 5, nc = id & 31;
    const uint4 v = *(const uint4*)(xs + r * S::XLD + nc * 16);
    *(uint4*)(p.dx + (int64_t)(r0 + r) * p.lddx + 8 * nc) = v;
  }
}

// ================================================================================ forward
// The same walk for the forward (memory_attention.py:97, per tracked frame: 13 312 rows):
//   phase A  H_c^T = W1[c, :] x^T           (K = 256; x's tile resident in LDS)
//   epilogue + b1, ReLU, dropout (the GEMM epilogue's counter hash, seed1 / element index
//            idx1 + row * H + h), bf16 -> the hid image (phase C's operand) and, 16 B per lane, the
//            saved hid (the backward's mask and dW2 operand)
//   phase C  y^T += W2[:, c] H_c^T          (K = 128, registers)
//   epilogue + b2, dropout (seed2, idx2 + row * 256 + n), bf16 -> y
// = linear2(dropout(relu(linear1(x)))) -> dropout as two GEMM launches compute it, without writing and
// re-reading hid between them.  Both weights are K-contiguous here (W1 [H][256] rows = hidden units,
// W2 [256][H] rows = outputs): the ring steps are plain K-contiguous images (b128 fragment reads).
#ifndef FFN_FWD_NS64
#define FFN_FWD_NS64 6
#endif
constexpr int FFN_FWD_HMAX = 2048;
using IF1 = GImg<FFN_HC, true, 4, 64>;  // W1 step: [128 h][64 k (d)], A operand of phase A
using IF2 = GImg<FFN_D, true, 4, 32>;   // W2 step: [256 n][32 k (h)], A operand of phase C
static_assert(IF1::BYTES == FFN_RING && IF2::BYTES == FFN_RING && IF1::PPW == 4 && IF2::PPW == 4, "ring steps");

template <int BM, int NS>
struct FfnFwdShape {
  using IX = GImg<BM, true, 4, 64>;   // x tile: 4 x [BM r][64 k (d)], B operand of phase A
  using IH = GImg<BM, true, 4, 64>;   // hid chunk: 2 x [BM r][64 k (h)], B operand of phase C
  static constexpr int NI = BM / 32;
  static constexpr int OFF_X = 0;
  static constexpr int OFF_RING = OFF_X + 4 * IX::BYTES;
  static constexpr int OFF_H = OFF_RING + NS * FFN_RING;
  static constexpr int OFF_B1 = OFF_H + 2 * IH::BYTES;  // b1 (fp32, H <= FFN_FWD_HMAX), DMA'd at the start
  static constexpr int LDS = OFF_B1 + FFN_FWD_HMAX * 4;
  static constexpr int STW = BM / 16;            // hid 16-B stores per lane per chunk
  static constexpr int XLD = FFN_D * 2 + 16;     // y staging row pitch (bytes)
  static_assert(LDS <= 160 * 1024 && BM * XLD <= LDS, "LDS");
};

struct FfnFwdArgs {
  int R, H;
  const bf16* x; int64_t ldx;
  const bf16* w1; const float* b1;   // [H][256], [H]   (linear1)
  const bf16* w2; const float* b2;   // [256][H], [256] (linear2)
  bf16* hid; int64_t ldh;
  bf16* y; int64_t ldy;
  float p;
  uint64_t seed1, seed2, idx1, idx2;
  const uint64_t* seed_off;
};

struct FfnFwdDma {
  uint32_t w1[4], w2[4];
  __device__ __forceinline__ void init(const FfnFwdArgs& p, int w, int lane) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int piece = w * 4 + i;
      int r = piece * (1024 / IF1::RB) + lane / IF1::LPR;
      w1[i] = (uint32_t)(r * FFN_D + 8 * IF1::swz(r, lane % IF1::LPR)) * 2u;
      r = piece * (1024 / IF2::RB) + lane / IF2::LPR;
      w2[i] = (uint32_t)(r * p.H + 8 * IF2::swz(r, lane % IF2::LPR)) * 2u;
    }
  }
};

// ring step q: chunk q / 8; steps 0-3 W1 (64-deep over d), 4-7 W2 (32-deep over the chunk's h)
template <int BM, int NS>
__device__ __forceinline__ void ffn_fwd_issue(char* smem, const FfnFwdArgs& p, const FfnFwdDma& d, int q, int w) {
  using S = FfnFwdShape<BM, NS>;
  char* slot = smem + S::OFF_RING + (q % NS) * FFN_RING;
  const int c = q >> 3, sub = q & 7;
  if (sub < 4) {
    const uint64_t b = sgpr_base(p.w1 + (int64_t)c * FFN_HC * FFN_D + sub * 64);
#pragma unroll
    for (int i = 0; i < 4; ++i) lds_dma16_so(b, d.w1[i], slot + (w * 4 + i) * 1024);
  } else {
    const uint64_t b = sgpr_base(p.w2 + c * FFN_HC + (sub - 4) * 32);
#pragma unroll
    for (int i = 0; i < 4; ++i) lds_dma16_so(b, d.w2[i], slot + (w * 4 + i) * 1024);
  }
}

// as ffn_wait: 4 DMAs per wave per step, the hid stores at the end of step 3
template <int BM, int NS, int SUB>
__device__ __forceinline__ void ffn_fwd_wait(bool first_chunk, bool last_chunk) {
  using S = FfnFwdShape<BM, NS>;
  constexpr int later = 4 * (NS - 2);
  constexpr int own = (SUB >= 4 && SUB <= NS + 2) ? S::STW : 0;
  constexpr bool prev = SUB + 8 <= NS + 2;
  if (SUB + NS - 2 >= 8 && last_chunk) vm_wait<0>();
  else if (prev && !first_chunk) vm_wait<later + own + S::STW>();
  else vm_wait<later + own>();
}

// dropout keep flags of 4 consecutive elements starting at idx (the GEMM epilogue's form)
__device__ __forceinline__ void keep4(uint64_t seed, uint64_t idx, uint32_t thresh, bool* k) {
  if ((idx & 1) == 0) {
    s2h_keep_pair(seed, idx >> 1, thresh, k[0], k[1]);
    s2h_keep_pair(seed, (idx >> 1) + 1, thresh, k[2], k[3]);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) k[e] = s2h_keep(seed, idx + e, thresh);
  }
}

template <int BM, int NS>
__global__ __launch_bounds__(256, 1) void ffn_fwd_kernel(FfnFwdArgs p) {
  using S = FfnFwdShape<BM, NS>;
  using IX = typename S::IX;
  using IH = typename S::IH;
  constexpr int NI = S::NI;
  __shared__ __attribute__((aligned(1024))) char smem[S::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r0 = blockIdx.x * BM;
  const int nchunk = p.H / FFN_HC;
  const int nq = nchunk * 8;
  const int wc = w & 1, wr = w >> 1;
  constexpr int WR = BM / 2;
  const bool drop = p.p > 0.f;
  const uint32_t thresh = drop ? (uint32_t)(p.p * 4294967296.0) : 0u;
  const float inv_keep = drop ? 1.f / (1.f - p.p) : 1.f;
  const uint64_t seed1 = drop ? s2h_seed(p.seed1, p.seed_off) : 0, seed2 = drop ? s2h_seed(p.seed2, p.seed_off) : 0;

  // b1 into LDS first (H / 256 pieces of 1 KB, H % 1024 == 0: the same count per wave): the epilogue
  // reads it from there -- a plain global load inside the loop would make the compiler wait for
  // vmcnt(0), draining the ring's DMAs every chunk
  for (int i = w; i < p.H / 256; i += 4) lds_dma16(p.b1 + i * 256 + lane * 4, smem + S::OFF_B1 + i * 1024);
#pragma unroll
  for (int s = 0; s < 4; ++s) IX::dma(smem + S::OFF_X + s * IX::BYTES, p.x, p.ldx, 1, r0, s * 64, p.R, FFN_D, w, lane);
  FfnFwdDma dma;
  dma.init(p, w, lane);
#pragma unroll
  for (int q = 0; q < NS - 1; ++q) ffn_fwd_issue<BM, NS>(smem, p, dma, q, w);

  f32x4 acc1[4][NI], acc2[8][NI];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int c = 0; c < nchunk; ++c) {
    const bool last = c + 1 == nchunk;
    static_for<0, 8>([&](auto subc) {
      constexpr int SUB = decltype(subc)::value;
      const int q = c * 8 + SUB;
      ffn_fwd_wait<BM, NS, SUB>(c == 0, last);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (q + NS - 1 < nq) ffn_fwd_issue<BM, NS>(smem, p, dma, q + NS - 1, w);
      const char* slot = smem + S::OFF_RING + (q % NS) * FFN_RING;
      if constexpr (SUB < 4) {
        if constexpr (SUB == 0) {
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc1[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        const char* xi = smem + S::OFF_X + SUB * IX::BYTES;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          bf16x8 a[4], b[NI];
#pragma unroll
          for (int i = 0; i < 4; ++i) a[i] = IF1::frag(slot, wc * 64 + i * 16, ks, lane);
#pragma unroll
          for (int j = 0; j < NI; ++j) b[j] = IX::frag(xi, wr * WR + j * 16, ks, lane);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc1[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc1[i][j], 0, 0, 0);
        }
        if constexpr (SUB == 3) {
          // + b1, ReLU, dropout, bf16 -> the hid image
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int hl = wc * 64 + i * 16 + 4 * (lane >> 4);
            const int hg = c * FFN_HC + hl;
            const float4 bb = *(const float4*)(smem + S::OFF_B1 + hg * 4);
            const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
            for (int j = 0; j < NI; ++j) {
              const int r = wr * WR + j * 16 + (lane & 15);
              float v[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = fmaxf(acc1[i][j][e] + bv[e], 0.f);
              if (drop) {
                bool k[4];
                keep4(seed1, p.idx1 + (uint64_t)(r0 + r) * p.H + hg, thresh, k);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = k[e] ? v[e] * inv_keep : 0.f;
              }
              bf16 t[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) t[e] = (bf16)v[e];
              *(uint2*)(smem + S::OFF_H + (hl >> 6) * IH::BYTES + IH::at(r, hl & 63)) = *(const uint2*)t;
            }
          }
          raw_barrier_lds();
#pragma unroll
          for (int e = 0; e < S::STW; ++e) {
            const int id = tid + 256 * e;
            const int r = id >> 4, kc = id & 15;
            const uint4 v = *(const uint4*)(smem + S::OFF_H + (kc >> 3) * IH::BYTES + IH::at(r, (kc & 7) * 8));
            st16_nt(p.hid + (int64_t)(r0 + r) * p.ldh + c * FFN_HC + 8 * kc, v, false);
          }
        }
      } else {
        constexpr int KS = SUB - 4;
        const char* hi = smem + S::OFF_H + (KS >> 1) * IH::BYTES;
        bf16x8 b[NI];
#pragma unroll
        for (int j = 0; j < NI; ++j) b[j] = IH::frag(hi, wr * WR + j * 16, KS & 1, lane);
#pragma unroll
        for (int ih = 0; ih < 2; ++ih) {
          bf16x8 a[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) a[i] = IF2::frag(slot, wc * 128 + (ih * 4 + i) * 16, 0, lane);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j)
              acc2[ih * 4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc2[ih * 4 + i][j], 0, 0, 0);
        }
      }
    });
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  // y = drop(acc + b2), 4 consecutive n of one row per lane -> bf16 staging -> 16-B row stores
  char* ys = smem;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int n = wc * 128 + i * 16 + 4 * (lane >> 4);
    const float4 bb = *(const float4*)(p.b2 + n);
    const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int r = wr * WR + j * 16 + (lane & 15);
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = acc2[i][j][e] + bv[e];
      if (drop) {
        bool k[4];
        keep4(seed2, p.idx2 + (uint64_t)(r0 + r) * FFN_D + n, thresh, k);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = k[e] ? v[e] * inv_keep : 0.f;
      }
      bf16 t[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] = (bf16)v[e];
      *(uint2*)(ys + r * S::XLD + n * 2) = *(const uint2*)t;
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < BM / 8; ++e) {
    const int id = tid + 256 * e;
    const int r = id >> 5, nc = id & 31;
    const uint4 v = *(const uint4*)(ys + r * S::XLD + nc * 16);
    *(uint4*)(p.y + (int64_t)(r0 + r) * p.ldy + 8 * nc) = v;
  }
}

}  // namespace

// Memory-attention FFN forward in one launch (memory_attention.py:97, bf16):
//   hid[R, H] = drop1(relu(x w1^T + b1))       (saved for the backward)
//   y[R, 256] = drop2(hid w2^T + b2)
// x [R, 256], w1 [H, 256] (linear1.weight), b1 [H] fp32, w2 [256, H] (linear2.weight), b2 [256] fp32;
// dropout p with the GEMM epilogue's counter hash: seed1 / element index idx1 + row * H + h for hid,
// seed2 / idx2 + row * 256 + n for y (so the backward's regenerated masks are the two GEMMs' own).
// R a multiple of 64, H a multiple of 1024 up to 2048; 16-B aligned bases, row strides multiples of 8.
extern "C" int s2h_ffn_fwd(int R, int H, const void* x, int64_t ldx, const void* w1, const float* b1, const void* w2,
                           const float* b2, float p, uint64_t seed1, uint64_t idx1, uint64_t seed2, uint64_t idx2,
                           void* hid, int64_t ldh, void* y, int64_t ldy, hipStream_t st) {
  if (R <= 0) return 0;
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (R % 64 || H <= 0 || H % 1024 || H > FFN_FWD_HMAX || !al(x) || !al(w1) || !al(w2) || !al(b1) || !al(b2) || !al(hid) || !al(y) ||
      ldx % 8 || ldh % 8 || ldy % 8 || (int64_t)R * ldx >= (1ll << 31) || (int64_t)H * H >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  FfnFwdArgs a;
  a.R = R; a.H = H;
  a.x = (const bf16*)x; a.ldx = ldx;
  a.w1 = (const bf16*)w1; a.b1 = b1;
  a.w2 = (const bf16*)w2; a.b2 = b2;
  a.hid = (bf16*)hid; a.ldh = ldh;
  a.y = (bf16*)y; a.ldy = ldy;
  a.p = p; a.seed1 = seed1; a.seed2 = seed2; a.idx1 = idx1; a.idx2 = idx2;
  a.seed_off = s2h_rng_offset_ptr();
  const bool big = R % 128 == 0 && R / 128 >= 512;
  const int slot = s2h_prof_begin(st, 4, 1, R, 2 * H, FFN_D, 4 | 16);
  s2h_prof_tag(((int64_t)1 << 43) | (big ? 128 : 64));
  // 64-row tiles (a tracked frame's 13 312 rows: 208 workgroups, one per CU) take a 6-deep ring to
  // hide the weight steps' DMA latency
  if (big)
    hipLaunchKernelGGL((ffn_fwd_kernel<128, 3>), dim3(R / 128), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((ffn_fwd_kernel<64, FFN_FWD_NS64>), dim3(R / 64), dim3(256), 0, st, a);
  s2h_prof_end(slot, st);
  return (int)hipGetLastError();
}

// Memory-attention FFN backward, input-gradient side (memory_attention.py:97): from dy (the gradient
// at linear2's output, [R, 256]), hid (linear2's saved input, [R, H]) and the bf16 weights w2
// ([256, H], linear2.weight) and w1 ([H, 256], linear1.weight):
//   dh[R, H] = (dy w2) * [hid > 0] * alpha        (alpha = 1 / keep of the dropout after the ReLU)
//   dx[R, 256] = dh w1
// One launch; dh is written once (for dW1 / db1) and never re-read here.  Requirements: R a multiple
// of 64, H of 128, 16-B aligned bases, row strides multiples of 8 elements.
extern "C" int s2h_ffn_bwd_dgrad(int R, int H, const void* dy, int64_t lddy, const void* w2, const void* w1,
                                 const void* hid, int64_t ldh, float alpha, void* dh, int64_t lddh, void* dx,
                                 int64_t lddx, hipStream_t st) {
  if (R <= 0) return 0;
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  // whole row tiles: every wave issues the same number of dH stores per chunk (the counted vmcnt
  // waits rely on it)
  if (R % 64 || H <= 0 || H % FFN_HC || !al(dy) || !al(w2) || !al(w1) || !al(hid) || !al(dh) || !al(dx) ||
      lddy % 8 || ldh % 8 || lddh % 8 || lddx % 8 || (int64_t)R * ldh >= (1ll << 31) ||
      (int64_t)R * lddy >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  FfnArgs p;
  p.R = R; p.H = H;
  p.dy = (const bf16*)dy; p.lddy = lddy;
  p.w2 = (const bf16*)w2; p.w1 = (const bf16*)w1;
  p.hid = (const bf16*)hid; p.ldh = ldh;
  p.dh = (bf16*)dh; p.lddh = lddh;
  p.dx = (bf16*)dx; p.lddx = lddx;
  p.alpha = alpha;
  // 128-row tiles when they still give >= 2 waves of workgroups over the 256 CUs
  const bool big = R % 128 == 0 && R / 128 >= 512;
  const int slot = s2h_prof_begin(st, 4, 1, R, 2 * H, FFN_D, 4 | 16);  // 4 R H 256 flop
  s2h_prof_tag(((int64_t)1 << 42) | (big ? 128 : 64));
  if (big)
    hipLaunchKernelGGL(ffn_bwd_dgrad_kernel<128>, dim3(R / 128), dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL(ffn_bwd_dgrad_kernel<64>, dim3(R / 64), dim3(256), 0, st, p);
  s2h_prof_end(slot, st);
  return (int)hipGetLastError();
}
