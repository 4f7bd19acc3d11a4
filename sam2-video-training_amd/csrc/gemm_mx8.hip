// MX-fp8 path (BASELINE config 5): OCP MX block-scaled e4m3 operands on the gfx950
// block-scaled MFMA (v_mfma_scale_f32_16x16x128_f8f6f4: twice the bf16 rate per clock).
//
// Format (OCP Microscaling v1.0, MXFP8 E4M3): blocks of 32 consecutive elements along the
// reduction dimension share one E8M0 scale 2^(e-127); e = floor(log2(amax)) - 8 + 127
// (8 = emax of e4m3), clamped to [0, 254]; elements are v / 2^(e-127) clamped to +-448 and
// rounded to nearest-even e4m3 (v_cvt_pk_fp8_f32).  Storage:
//   Q  [rows][Kp] u8, Kp = K rounded up to 128 (zero padding: no K tail in the GEMM)
//   S  [Kp / 128][lds] int32: word (kt, row) holds the scales of blocks 4kt..4kt+3 of `row`,
//      byte b = block 4kt+b -- the MFMA takes one scale byte per lane (row l&15, block l>>4),
//      and 16 consecutive rows are 16 consecutive words.
// Lane map of the 16x16x128 f8f6f4 operand (tools/probe_mx.hip): lane l holds row l&15,
// bytes 0..15 = k 16g..16g+15 and bytes 16..31 = k 64+16g..64+16g+15 (g = l>>4) of the
// 128-deep step; its scale byte covers block g (k 32g..32g+31) of that row.  Both operands
// use the same map, so a product over K is exact up to fp32 summation order.
#include "gemm_epi.h"

typedef int v8i32 __attribute__((ext_vector_type(8)));

// ------------------------------------------------------------------ quantiser
struct Mx8QArgs {
  const void* X; int dt; int64_t ld_row, ld_col;
  uint8_t* Q; int64_t ldq;
  int32_t* S; int64_t lds;
  int rows, cols, nkt, vec;
};

__device__ __forceinline__ int floor_log2_pos(float a) {
  const uint32_t b = __float_as_uint(a);
  const int e = (int)((b >> 23) & 0xff);
  if (e) return e - 127;
  const uint32_t m = b & 0x7fffff;  // subnormal: m * 2^-149
  return (31 - __builtin_clz(m)) - 149;
}

__device__ __forceinline__ uint32_t pack4_e4m3(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

// 8 lanes per (row, 128-column group): lane `sub` converts columns 16*sub .. 16*sub+15, lanes
// (2b, 2b+1) share block b's amax.  TRANS: consecutive groups walk rows (the source is
// row-contiguous: a transposed weight), else 128-column groups of one row.
template <bool TRANS>
__global__ __launch_bounds__(256) void mx8_quant_kernel(Mx8QArgs p) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t grp = t >> 3;
  const int sub = threadIdx.x & 7;
  if (grp >= (int64_t)p.rows * p.nkt) return;  // whole 8-lane groups retire together
  int row, kt;
  if (TRANS) { kt = (int)(grp / p.rows); row = (int)(grp % p.rows); }
  else       { row = (int)(grp / p.nkt); kt = (int)(grp % p.nkt); }
  const int c0 = kt * 128 + 16 * sub;
  float v[16];
  if (!TRANS && p.vec && c0 + 16 <= p.cols) {
    const bf16* src = (const bf16*)p.X + (int64_t)row * p.ld_row + c0;
    const uint4 r0 = *(const uint4*)src, r1 = *(const uint4*)(src + 8);
    const bf16* b0 = (const bf16*)&r0;
    const bf16* b1 = (const bf16*)&r1;
#pragma unroll
    for (int j = 0; j < 8; ++j) { v[j] = (float)b0[j]; v[8 + j] = (float)b1[j]; }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int c = c0 + j;
      const int64_t o = (int64_t)row * p.ld_row + (int64_t)c * p.ld_col;
      v[j] = c < p.cols ? (p.dt == S2H_BF16 ? (float)((const bf16*)p.X)[o] : ((const float*)p.X)[o]) : 0.f;
    }
  }
  float amax = 0.f;
#pragma unroll
  for (int j = 0; j < 16; ++j) amax = fmaxf(amax, fabsf(v[j]));
  amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
  int e8 = 127;
  if (amax > 0.f) e8 = min(max(floor_log2_pos(amax) - 8 + 127, 0), 254);
  const float inv = ldexpf(1.f, 127 - e8);
  uint32_t w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float x[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = fminf(fmaxf(v[4 * q + e] * inv, -448.f), 448.f);
    w[q] = pack4_e4m3(x[0], x[1], x[2], x[3]);
  }
  *(uint4*)(p.Q + (int64_t)row * p.ldq + c0) = make_uint4(w[0], w[1], w[2], w[3]);
  const int base = (threadIdx.x & 63) & ~7;
  const uint32_t word = (uint32_t)__shfl(e8, base + 0, 64) | ((uint32_t)__shfl(e8, base + 2, 64) << 8) |
                        ((uint32_t)__shfl(e8, base + 4, 64) << 16) | ((uint32_t)__shfl(e8, base + 6, 64) << 24);
  if (sub == 0) p.S[(int64_t)kt * p.lds + row] = (int32_t)word;
}

extern "C" int s2h_mx8_quant(int rows, int cols, int dt_x, const void* X, int64_t ld_row, int64_t ld_col, uint8_t* Q,
                             int64_t ldq, int32_t* S, int64_t lds, hipStream_t st) {
  if (rows <= 0 || cols <= 0) return 0;
  const int nkt = (cols + 127) / 128;
  if (ldq < 128 * nkt || ldq % 16 || ((uintptr_t)Q & 15) || lds < rows || (dt_x != S2H_BF16 && dt_x != S2H_F32))
    return (int)hipErrorInvalidValue;
  Mx8QArgs p;
  p.X = X; p.dt = dt_x; p.ld_row = ld_row; p.ld_col = ld_col;
  p.Q = Q; p.ldq = ldq; p.S = S; p.lds = lds;
  p.rows = rows; p.cols = cols; p.nkt = nkt;
  p.vec = dt_x == S2H_BF16 && ld_col == 1 && ld_row % 8 == 0 && ((uintptr_t)X & 15) == 0;
  const int64_t threads = (int64_t)rows * nkt * 8;
  const dim3 grid((unsigned)((threads + 255) / 256));
  const int slot = s2h_prof_begin(st, 8, rows, cols, 0, 0, 0);
  if (ld_row == 1 && ld_col != 1) hipLaunchKernelGGL(mx8_quant_kernel<true>, grid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL(mx8_quant_kernel<false>, grid, dim3(256), 0, st, p);
  s2h_prof_end(slot, st);
  S2H_LAUNCH_CHECK();
}

// ------------------------------------------------------------------ GEMM
struct Mx8Args {
  GemmArgs16 e;  // shapes + epilogue (A / B of it unused)
  const uint8_t* A; int64_t lda; const int32_t* SA; int64_t lsa;
  const uint8_t* B; int64_t ldb; const int32_t* SB; int64_t lsb;
  int nkt;
};

// ROWS x 128-byte operand image: 16-B chunk c of row r stored at chunk c ^ ((r >> 1) & 7)
// (conflict-free ds_read_b128 for the 16-row fragment reads); filled by LDS-DMA, 1 KiB
// (8 rows) per wave instruction, the swizzle applied to the per-lane source address.
template <int ROWS, int NW>
struct MxImg {
  static constexpr int BYTES = ROWS * 128;
  static constexpr int PIECES = BYTES / 1024;
  static constexpr int PPW = PIECES / NW;
  static_assert(PPW >= 1 && PIECES % NW == 0, "tile too small");
  __device__ static __forceinline__ int swz(int r, int c) { return c ^ ((r >> 1) & 7); }
  __device__ static __forceinline__ void dma(char* img, const uint8_t* base, int ld, int row0, int k0, int nrows,
                                            int w, int lane) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int piece = w * PPW + i;
      const int irow = piece * 8 + (lane >> 3);
      const int c = swz(irow, lane & 7);
      const int r = min(row0 + irow, nrows - 1);  // rows past the edge: valid address, never stored
      lds_dma16(base + (r * ld + k0 + 16 * c), img + piece * 1024);
    }
  }
  __device__ static __forceinline__ v8i32 frag(const char* img, int rb, int lane) {
    const int r = rb + (lane & 15), g = lane >> 4;
    const uint4 lo = *(const uint4*)(img + r * 128 + 16 * swz(r, g));
    const uint4 hi = *(const uint4*)(img + r * 128 + 16 * swz(r, 4 + g));
    v8i32 f;
    f[0] = lo.x; f[1] = lo.y; f[2] = lo.z; f[3] = lo.w;
    f[4] = hi.x; f[5] = hi.y; f[6] = hi.z; f[7] = hi.w;
    return f;
  }
};

template <int BM, int BN>
__global__ __launch_bounds__(256, (2 * 128 * (BM + BN) <= 80 * 1024 ? 2 : 1)) void gemm_mx8_kernel(Mx8Args p) {
  if (p.e.drop_p > 0.f) p.e.seed = s2h_seed(p.e.seed, p.e.seed_off);
  constexpr int NW = 4, WM = BM / 2, WN = BN / 2, MI = WM / 16, NI = WN / 16;
  using IA = MxImg<BM, NW>;
  using IB = MxImg<BN, NW>;
  constexpr int STAGE = IA::BYTES + IB::BYTES;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int nwg = gridDim.x, id = blockIdx.x;  // XCD-aware order, as the bf16 kernel
  const int xcd = id % 8, qd = nwg / 8, rm = nwg % 8;
  const int wg = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + id / 8;
  const int M = p.e.M, N = p.e.N;
  const int ntn = (N + BN - 1) / BN;
  const int m0 = (wg / ntn) * BM, n0 = (wg % ntn) * BN;
  const int nk = p.nkt;
  const int lda = (int)p.lda, ldb = (int)p.ldb;

  // scale words: one per 16-row fragment and K step; lane group g takes byte g
  int arow[MI], brow[NI];
#pragma unroll
  for (int i = 0; i < MI; ++i) arow[i] = min(m0 + wm * WM + i * 16 + (lane & 15), M - 1);
#pragma unroll
  for (int j = 0; j < NI; ++j) brow[j] = min(n0 + wn * WN + j * 16 + (lane & 15), N - 1);
  const int sh = 8 * (lane >> 4);
  int sa_n[MI], sb_n[NI];

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const bool dma_on = !(p.e.dbg & 4);
  if (nk > 0) {
    if (dma_on) {
      IA::dma(smem, p.A, lda, m0, 0, M, w, lane);
      IB::dma(smem + IA::BYTES, p.B, ldb, n0, 0, N, w, lane);
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) sa_n[i] = p.SA[arow[i]];
#pragma unroll
    for (int j = 0; j < NI; ++j) sb_n[j] = p.SB[brow[j]];
  }
  for (int kt = 0; kt < nk; ++kt) {
    char* sa = smem + (kt & 1) * STAGE;
    char* sb = sa + IA::BYTES;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage kt and its scale words landed
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    int sca[MI], scb[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) sca[i] = (sa_n[i] >> sh) & 0xff;
#pragma unroll
    for (int j = 0; j < NI; ++j) scb[j] = (sb_n[j] >> sh) & 0xff;
    if (kt + 1 < nk) {  // next stage into the buffer step kt-1 read; runs under this step's MFMAs
      char* na = smem + ((kt + 1) & 1) * STAGE;
      if (dma_on) {
        IA::dma(na, p.A, lda, m0, (kt + 1) * 128, M, w, lane);
        IB::dma(na + IA::BYTES, p.B, ldb, n0, (kt + 1) * 128, N, w, lane);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) sa_n[i] = p.SA[(int64_t)(kt + 1) * p.lsa + arow[i]];
#pragma unroll
      for (int j = 0; j < NI; ++j) sb_n[j] = p.SB[(int64_t)(kt + 1) * p.lsb + brow[j]];
    }
    if (p.e.dbg & 2) continue;
    v8i32 a[MI], b[NI];
#pragma unroll
    for (int i = 0; i < MI; ++i) a[i] = IA::frag(sa, wm * WM + i * 16, lane);
#pragma unroll
    for (int j = 0; j < NI; ++j) b[j] = IB::frag(sb, wn * WN + j * 16, lane);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[i], b[j], acc[i][j], 0, 0, 0, sca[i], 0, scb[j]);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  tile_epilogue<WM, WN, MI, NI>(p.e, acc, reinterpret_cast<float*>(smem) + w * 16 * (WN + 4), 0, m0 + wm * WM,
                                n0 + wn * WN, lane);
}

static int g_mx8_cfg = 0;  // 0 automatic, 1: 64x64, 2: 128x64, 3: 128x128
static int g_mx8_dbg = 0;  // measurement-only ablations (bits 8+): as GemmArgs16::dbg
extern "C" int s2h_mx8_config(int cfg) {
  const int prev = g_mx8_cfg | (g_mx8_dbg << 8);
  g_mx8_cfg = cfg & 0xff;
  g_mx8_dbg = cfg >> 8;
  return prev;
}

template <int BM, int BN>
static void launch_mx8(const Mx8Args& a, hipStream_t st) {
  s2h_prof_tag(gemm_tag(BM, BN, 2, 2, 2, 128, true, true, false, true));
  const dim3 grid(((a.e.N + BN - 1) / BN) * ((a.e.M + BM - 1) / BM));
  hipLaunchKernelGGL((gemm_mx8_kernel<BM, BN>), grid, dim3(256), 0, st, a);
}

extern "C" int s2h_gemm_mx8(int M, int N, int K, const uint8_t* A, int64_t lda, const int32_t* SA, int64_t lsa,
                            const uint8_t* B, int64_t ldb, const int32_t* SB, int64_t lsb, void* C, int dt_c,
                            int64_t ldc, const float* bias, const void* R, int64_t ldr, void* X, int64_t ldx,
                            int aux_mode, float drop_p, uint64_t seed, uint64_t drop_idx0, float alpha, float beta,
                            int act, hipStream_t st) {
  if (M <= 0 || N <= 0) return 0;
  const int nkt = (K + 127) / 128;
  auto al16 = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  // 32-bit DMA offsets; 16-B aligned operand rows (the quantiser's Kp layout)
  if (K <= 0 || lda < 128 * nkt || ldb < 128 * nkt || lda % 16 || ldb % 16 || !al16(A) || !al16(B) ||
      (int64_t)M * lda >= (1ll << 31) || (int64_t)N * ldb >= (1ll << 31) || lsa < M || lsb < N)
    return (int)hipErrorInvalidValue;
  Mx8Args a = {};
  GemmArgs16& e = a.e;
  e.M = M; e.N = N; e.K = K;
  e.C = C; e.ldc = ldc; e.sC = 0;
  e.bias = bias; e.bias_mode = bias ? 1 : 0;
  e.R = R; e.ldr = ldr; e.sR = 0;
  e.X = X; e.ldx = ldx; e.sX = 0; e.aux_mode = X ? aux_mode : 0;
  e.cscale = nullptr; e.drop_p = drop_p; e.seed = seed; e.seed_off = s2h_rng_offset_ptr(); e.drop_idx0 = drop_idx0;
  e.alpha = alpha; e.beta = beta; e.act = act;
  e.splits = 1; e.kchunk = K;
  e.out_f32 = dt_c == S2H_F32;
  e.rowsum = nullptr;
  e.dbg = g_mx8_dbg;
  gemm_plan_vec(e, 1);
  a.A = A; a.lda = lda; a.SA = SA; a.lsa = lsa;
  a.B = B; a.ldb = ldb; a.SB = SB; a.lsb = lsb;
  a.nkt = nkt;
  const int slot = s2h_prof_begin(st, 4, 1, M, N, K, 8 + 2 + 1);  // layout flag 8: MX-fp8 operands
  int cfg = g_mx8_cfg;
  if (!cfg) {
    // graph-replay timings of the config-5 shapes (tools/mx8_bench.py): 128x64 wins everywhere
    // but on long K (16384x448x1792: 128x128 23.5 us vs 28.5) and on small grids (64x64)
    const long t128 = (long)((M + 127) / 128) * ((N + 127) / 128);
    const long t128x64 = (long)((M + 127) / 128) * ((N + 63) / 64);
    cfg = (K >= 1024 && t128 >= 256) ? 3 : (t128x64 >= 256 ? 2 : 1);
  }
  if (cfg == 3) launch_mx8<128, 128>(a, st);
  else if (cfg == 2) launch_mx8<128, 64>(a, st);
  else launch_mx8<64, 64>(a, st);
  s2h_prof_end(slot, st);
  S2H_LAUNCH_CHECK();
}
