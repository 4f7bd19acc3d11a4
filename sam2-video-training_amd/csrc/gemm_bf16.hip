// bf16 GEMM dispatch: the tiling per shape (kernels in gemm_bf16.h, instantiated in gemm_cfg*.hip).
#include "gemm_bf16.h"

static int g_gemm_cfg = CFG_AUTO;
static int g_gemm_tiny_cfg = CFG_AUTO;  // A/B knob: tiling of GEMMs with M <= 128 (s2h_gemm_tiny_config)

extern "C" int s2h_gemm_tiny_config(int cfg) {
  const int prev = g_gemm_tiny_cfg;
  g_gemm_tiny_cfg = cfg;
  return prev;
}
// (512 -- one round of two workgroups per CU -- won the hot-cache sweep, profiles/r03_v6_wgrad_sweep.log,
// but lost inside the step, profiles/r03_v6_trace_diff.log: kept at 768)
int g_gemm_split_target = 768;

// A/B knob: workgroups a split-K weight-gradient launch aims at (returns the previous value)
extern "C" int s2h_gemm_split_target(int t) {
  const int prev = g_gemm_split_target;
  if (t > 0) g_gemm_split_target = t;
  return prev;
}
static int g_gemm_dbg = 0;

// 4 x 1 wave grids instead of the 2 x 2 ones for bf16 outputs (1: every such GEMM, the default;
// 2: only N >= 768; 0: off); bit-identical results.  In-step env A/B (tools/gpu_r3q.sh,
// S2H_GEMM_W41 0 / 1 / 2, two rounds): 136.77 / 136.71, 136.98 / 137.05, 136.68 / 136.86 clip-frames/s
static int g_gemm_w41 = 1;
extern "C" int s2h_gemm_w41(int mode) {
  const int prev = g_gemm_w41;
  g_gemm_w41 = mode;
  return prev;
}
static int w41_of(int cfg) {
  switch (cfg) {
    case CFG_64: return CFG_64_W41;
    case CFG_128x64: return CFG_128x64_W41;
    case CFG_128x64_K32_NS3: return CFG_128x64_W41_K32_NS3;
    case CFG_64_NS4: return CFG_64_W41_NS4;
    case CFG_128x64_NS3: return CFG_128x64_W41_NS3;
    default: return cfg;
  }
}

// Short K that is not a whole number of 64-deep stages (Hiera's 112 / 224 channels, the V-fold's 72,
// the memory encoder's 64 + 8 ...) on the A-in-registers tiling: no zero-filled tail stage, no
// extra barrier, 5 workgroups per CU (tools/areg_bench.py, profiles/r04_v11_areg.log: 32768x224x224
// 22.1 -> 17.2 us, 8192x448x112 9.3 -> 8.3, 13312x256x72 9.7 -> 8.4; at K = 128 / 256 the LDS-DMA
// tilings stay ahead).  1 = on (default), 0 = off (A/B, S2H_GEMM_AREG)
static int g_gemm_areg = 1;
extern "C" int s2h_gemm_areg(int mode) {
  const int prev = g_gemm_areg;
  g_gemm_areg = mode;
  return prev;
}

// A/B knob (round 6): the tiling of one class of bf16-output GEMMs (M > 128), 0 = the shape rules below.
//   class 0: K >= 1024, N <= 512 (long reduction, narrow output: the memory-attention FFN linear2, the
//            memory fuser pwconv2, Hiera MLP fc2)
//   class 1: K <= 256, N <= 256, M >= 8192 (short reduction, narrow output: per-frame projections)
//   class 2: K <= 512, N >= 768 (wide output: FFN linear1, Hiera qkv / fc1)
//   class 3: 256 < K < 1024, N <= 512 (mid reduction, narrow output: Hiera proj)
//   class 4: K < 256 not a multiple of 64 (the A-in-registers domain), M >= 65536 (Hiera stage 1 at
//            112 channels: 131072 rows at 512^2)
//   class 5: the same with M < 65536 and K >= 128 (Hiera stage 2 at 224 channels)
// Defaults (round 6): classes 4 / 5 on the 128 x 64 4 x 1 LDS-DMA tiling with 32-deep stages, 3-deep ring
// (cfg 22) instead of the A-in-registers kernel: in-step sweeps 47.59 / 47.52 -> 47.45 / 47.44 ms
// (profiles/r06_v12_gemm_class4_sweep.log, r06_v13_gemm_class45_sweep.log); every other class keeps its rules.
static int g_gemm_class_cfg[6] = {0, 0, 0, 0, CFG_128x64_W41_K32_NS3, CFG_128x64_W41_K32_NS3};
extern "C" int s2h_gemm_class_config(int cls, int cfg) {
  if (cls < 0 || cls > 5) return -1;
  const int prev = g_gemm_class_cfg[cls];
  g_gemm_class_cfg[cls] = cfg;
  return prev;
}
static int gemm_class(const GemmArgs16& a) {
  if (a.out_f32 || a.M <= 128) return -1;
  // (K < 128 with M < 65536 -- the V-fold out projection, 13312x256x72 -- stays on the A-in-registers
  // rule: 12.45 us there vs 14.21 on cfg 22, profiles/r06_v3 vs r06_v37 shape tables)
  if (a.K < 256 && a.K % 64 != 0) return a.M >= 65536 ? 4 : (a.K >= 128 ? 5 : -1);
  if (a.K >= 1024 && a.N <= 512) return 0;
  if (a.K <= 256 && a.N <= 256 && a.M >= 8192) return 1;
  if (a.K <= 512 && a.N >= 768) return 2;
  if (a.K > 256 && a.K < 1024 && a.N <= 512) return 3;
  return -1;
}

extern "C" int s2h_gemm_config(int cfg) {
  const int prev = g_gemm_cfg | (g_gemm_dbg << 8);
  g_gemm_cfg = cfg < 0 ? cfg : (cfg & 0xff);
  g_gemm_dbg = cfg < 0 ? 0 : (cfg >> 8);
  return prev;
}

// Tiling by shape.  rocprofv3 kernel traces of tools/gemm_one.py (tools/kt_gemm.sh,
// profiles/r01_v14_gemm_tilings.txt) and the per-shape table of a profiled training step
// (bench.py --kernel-table with S2H_GEMM_CFG forced to 1 / 7, profiles/r01_v14_gemm_cfg_step.txt):
//  * 128x64 (4 waves of 32x32, 24 KB per stage) wins where it still yields >= 1024 tiles --
//    13312x2048x256 35.7 us vs 38.2 (64^2) / 40.0 (128^2), 131072x448x112 70.1 vs 77.5 --
//    and on split-K weight gradients with >= 64 of its tiles (2048x256x13312: -17 %);
//  * 64^2 wins on the narrow outputs (N = 128..256 of 13312 rows, 416 tiles at 128x64: the
//    occupancy of the smaller tile hides the LDS-DMA latency) and on tiny weight gradients;
//  * 256^2 (8 waves) only pays on large square problems (4096^3: 146 us vs 170 for 128^2).
static int pick_cfg(const GemmArgs16& a, int batch) {
  // M <= 128 (decoder tokens, pooled heads): 64^2 tiles with a 4-deep ring -- the in-step env A/B
  // (tools/gpu_r3n.sh, S2H_GEMM_TINY_CFG 0 / 19 / 18, two rounds) measured 137.5 / 137.3 clip-frames/s
  // for the default rules, 136.9 / 137.0 for the 8-deep K32 ring and 137.8 / 138.0 for this one
  if (a.M <= 128) return CFG_64_NS4;
  const long t256 = (long)((a.M + 255) / 256) * ((a.N + 255) / 256) * batch;
  if (a.M >= 1024 && a.N >= 1024 && a.K >= 1024 && t256 >= 128) return CFG_256;
  const long t128x64 = (long)((a.M + 127) / 128) * ((a.N + 63) / 64) * batch;
  const bool split = a.out_f32 && a.K >= 1024 && t128x64 < 512;  // plan_splits' split-K regime
  // deep K on large grids: 128x128 (tools/epi_bench.py: 93184x256x2048 175 -> 139 us; below
  // 512 of its tiles the 128x64 form stays ahead, e.g. 8192x448x1792 24 vs 29 us)
  const long t128 = (long)((a.M + 127) / 128) * ((a.N + 127) / 128) * batch;
  // >= 1024 tiles of 128^2 with K >= 256 on the frame-batched backward's row counts: 32-deep
  // stages, 3-deep ring (tools/gemm_cfg_sweep.py, profiles/r03_v4_gemm_cfg_sweep.log: dgrad
  // 93184x256x2048 215 -> 188 us, 93184x256x256 32.6 -> 29.3, 93184x2048x256 148 -> 142; the
  // 13312-row forward shapes won in isolation but lost inside the step: 13312x2048x256 with its
  // ReLU + dropout epilogue 50.7 -> 57.8 us per launch, profiles/r03_v5_kernel_table.txt)
  if (!split && a.M >= 32768 && a.K >= 256 && a.N >= 256 && t128 >= 1024) return CFG_128_K32_NS3;
  if (!split && a.K >= 1024 && t128 >= 512) return CFG_128;
  // shallow K (<= 256) on large grids: 32-deep stages, 3-deep ring (tools/epi_bench.py graph
  // replays: 131072x448x112 70 -> 58 us, 32768x672x224 35 -> 28, 93184x2048x256 222 -> 216;
  // below ~2k tiles or at K >= 448 the 64-deep 2-stage form stays ahead)
  // (tools/dgrad_bench.py: the same holds for narrow outputs up to K = 1024 -- dgrad 32768x224
  // over K = 672: 29.2 -> 24.4 us, 131072x112 over K = 448: 43.9 -> 40.3)
  if (!split && t128x64 >= 1024 && (a.K <= 256 ? t128x64 >= 2048 : (a.N <= 256 && a.K <= 1024)))
    return CFG_128x64_K32_NS3;
  if (split ? t128x64 >= 64 : t128x64 >= 1024) return CFG_128x64;
  return CFG_64;
}

// Tiny-M long-K GEMMs with a bf16 output (M <= 128, K >= 1024, <= 16 output tiles of 64 x 64; round 6):
// the two-way decoder's token MLP second layer, 104 x 256 x 2048 (transformer.py:219-245, frame-batched
// forward per frame), ran as 8 workgroups of 32 K steps each (21 us, profiles/r06_v3_shape_table.txt).
// The K range is split over S batch entries of ONE fp32 launch into the weight-gradient workspace
// (no epilogue), then ONE launch adds the S partials in fixed order and runs the GEMM epilogue (bias,
// activation, dropout, residual, pre-activation store: epilogue4) -- deterministic, the fp32 sum rounded
// once.  Opt-in (S2H_GEMM_TINY_SPLITK=1, s2h_gemm_tiny_splitk): 47.73 / 47.81 ms per bench step against
// 47.63 / 47.83 for the one-launch tiling (in-call A/B) -- no gain, so the one-launch tiling stays.
float* s2h_det_ws(int64_t bytes);  // gemm_wgrad.hip: the registered workspace (nullptr: none / off)
static int g_gemm_tiny_splitk = 0;  // measured neutral in-step (profiles/r06_v9_tiny_splitk_ab.log): opt-in
extern "C" int s2h_gemm_tiny_splitk(int mode) {
  const int prev = g_gemm_tiny_splitk;
  if (mode >= 0) g_gemm_tiny_splitk = mode;
  return prev;
}

__global__ __launch_bounds__(256) void gemm_splitk_epi_kernel(GemmArgs16 p, const float* part, int S) {
  if (p.drop_p > 0.f) p.seed = s2h_seed(p.seed, p.seed_off);  // the device RNG offset, as every dropout site
  const int nq = (p.N + 3) / 4;
  const int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (q >= (int64_t)p.M * nq) return;
  const int row = (int)(q / nq), col0 = (int)(q % nq) * 4;
  const int64_t MN = (int64_t)p.M * p.N;
  const float* pp = part + (int64_t)row * p.N + col0;
  float v[4] = {0.f, 0.f, 0.f, 0.f};
  if (col0 + 4 <= p.N && (p.N & 3) == 0) {
    for (int sp = 0; sp < S; ++sp) {
      const float4 t = *(const float4*)(pp + sp * MN);
      v[0] += t.x; v[1] += t.y; v[2] += t.z; v[3] += t.w;
    }
  } else {
    for (int sp = 0; sp < S; ++sp)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (col0 + e < p.N) v[e] += pp[sp * MN + e];
  }
  float bcol[4];
  load_bcol(p, col0, bcol);
  epilogue4(p, 0, row, col0, float4{v[0], v[1], v[2], v[3]}, bcol);
}

static int gemm_tiny_splitk(const GemmArgs16& a, int batch, hipStream_t st) {
  if (!g_gemm_tiny_splitk || batch != 1 || a.out_f32 || a.M > 128 || a.K < 1024 || a.lda_k != 1 || a.ldb_k != 1 ||
      a.rowsum != nullptr || a.rope_cos != nullptr)
    return -1;
  const int tiles = ((a.M + 63) / 64) * ((a.N + 63) / 64);
  if (tiles > 16) return -1;
  int S = 16;
  while (S > 1 && (a.K % (64 * S) != 0 || tiles * S > 256)) S /= 2;
  if (S < 4 || a.K / S >= 1024) return -1;  // (a K chunk of >= 1024 would be split again, into the same workspace)
  float* ws = s2h_det_ws((int64_t)S * a.M * a.N * 4);
  if (ws == nullptr) return -1;
  GemmArgs16 b = {};
  b.M = a.M; b.N = a.N; b.K = a.K / S;
  b.A = a.A; b.lda_m = a.lda_m; b.lda_k = 1; b.sA = a.K / S;
  b.B = a.B; b.ldb_k = 1; b.ldb_n = a.ldb_n; b.sB = a.K / S;
  b.C = ws; b.ldc = a.N; b.sC = (int64_t)a.M * a.N;
  b.alpha = 1.f; b.beta = 0.f; b.out_f32 = 1;
  b.vecA = a.vecA; b.vecB = a.vecB;
  b.dbg = a.dbg;
  if (!gemm_glds_ok(b, S)) return -1;
  int rc = gemm_cfg_launch_1(CFG_64_NS4, b, S, st);
  if (rc != 0) return rc;
  GemmArgs16 e = a;
  e.splits = 1;
  e.kchunk = a.K;
  gemm_plan_vec(e, 1);
  const int64_t nq = (int64_t)a.M * ((a.N + 3) / 4);
  hipLaunchKernelGGL(gemm_splitk_epi_kernel, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, e, ws, S);
  return (int)hipGetLastError();
}

// The fixed-order sum of a split launch's partial tiles (gemm16.h, plan_splits): one thread per output
// element (then per rowsum element), eight independent chains over the splits (split q on chain q % 8,
// eight loads in flight) combined in a fixed tree -- the same sum for any timing of the split launch.
__global__ __launch_bounds__(256) void gemm_split_reduce_kernel(const float* part, int S, int64_t sX, int batch, int M,
                                                                int N, float* C, int64_t ldc, int64_t sC, int beta1,
                                                                float* rowsum) {
  const int64_t nc = (int64_t)batch * M * N, nr = rowsum ? (int64_t)batch * M : 0;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nc + nr) return;
  const float* pp = i < nc ? part + i : part + S * sX + (i - nc);
  const int64_t stride = i < nc ? sX : nr;
  float ch[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int s = 0;
  for (; s + 8 <= S; s += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) ch[j] += pp[(s + j) * stride];
#pragma unroll
  for (int j = 0; j < 7; ++j)
    if (s + j < S) ch[j] += pp[(s + j) * stride];
  const float v = ((ch[0] + ch[1]) + (ch[2] + ch[3])) + ((ch[4] + ch[5]) + (ch[6] + ch[7]));
  if (i < nc) {
    const int64_t b = i / ((int64_t)M * N), r = (i / N) % M, c = i % N;
    float* o = C + b * sC + r * ldc + c;
    *o = beta1 ? *o + v : v;
  } else {
    rowsum[i - nc] += v;
  }
}

int s2h_gemm_split_reduce(const GemmArgs16& a, int batch, hipStream_t st) {
  const int64_t n = (int64_t)batch * a.M * a.N + (a.rowsum ? (int64_t)batch * a.M : 0);
  hipLaunchKernelGGL(gemm_split_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (const float*)a.X,
                     a.splits, a.sX, batch, a.M, a.N, (float*)a.C, a.ldc, a.sC, a.beta == 1.f ? 1 : 0, a.rowsum);
  return (int)hipGetLastError();
}

// K = 1 (an outer product, e.g. the hypernetwork-mask gradient dup[o] = g[o]^T h[o] over 104 frames x
// objects of 16384 x 32, frametape._hyper_bw): C = alpha * a b^T element-wise, 8 output columns per lane
// with one 16-B store.  The bf16 x bf16 product is exact in fp32 and rounded once, as the MFMA tile's
// single accumulation is -- the same bits as the tiled GEMM, which spent 134 us per launch on K-step
// prologue / tail zeroing for 109 MB of output.
__global__ __launch_bounds__(256) void gemm_outer_kernel(GemmArgs16 p, int batch) {
  const int ng = (p.N + 7) / 8;
  const int64_t total = (int64_t)batch * p.M * ng;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int gcol = (int)(i % ng);
    const int64_t r = i / ng;
    const int m = (int)(r % p.M), bz = (int)(r / p.M);
    const float av = p.alpha * (float)p.A[(int64_t)bz * p.sA + (int64_t)m * p.lda_m];
    const bf16* B = p.B + (int64_t)bz * p.sB;
    const int n0 = gcol * 8;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = n0 + e < p.N ? av * (float)B[(int64_t)(n0 + e) * p.ldb_n] : 0.f;
    if (p.out_f32) {
      float* C = (float*)p.C + (int64_t)bz * p.sC + (int64_t)m * p.ldc + n0;
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (n0 + e < p.N) C[e] = v[e];
    } else {
      bf16* C = (bf16*)p.C + (int64_t)bz * p.sC + (int64_t)m * p.ldc + n0;
      bf16 t[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) t[e] = (bf16)v[e];
      if (n0 + 8 <= p.N && (((uintptr_t)C) & 15) == 0) {
        *(uint4*)C = *(const uint4*)t;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (n0 + e < p.N) C[e] = t[e];
      }
    }
  }
}
static int gemm_outer(const GemmArgs16& a, int batch, hipStream_t st) {
  if (a.K != 1 || a.beta != 0.f || a.bias || a.R || a.X || a.cscale || a.drop_p != 0.f || a.act != 0 || a.rowsum ||
      a.rope_cos != nullptr)
    return -1;
  const int64_t total = (int64_t)batch * a.M * ((a.N + 7) / 8);
  if (total <= 0) return 0;
  const int64_t blocks = std::min<int64_t>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(gemm_outer_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a, batch);
  return (int)hipGetLastError();
}

int s2h_gemm_bf16(const GemmArgs16& in, int batch, hipStream_t st) {
  GemmArgs16 a = in;
  a.dbg = g_gemm_dbg;
  if (!g_gemm_cfg) {
    const int rc = gemm_outer(a, batch, st);
    if (rc >= 0) return rc;
  }
  if (!g_gemm_cfg && !g_gemm_tiny_cfg) {
    const int rc = gemm_tiny_splitk(a, batch, st);
    if (rc >= 0) return rc;
  }
  if (!g_gemm_cfg && a.out_f32 && a.K >= 512) {  // long / mid-reduction weight gradients (gemm_wgrad.hip)
    const int rc = s2h_gemm_wgrad_det(a, batch, st);
    if (rc >= 0) return rc;
  }
  int cfg = g_gemm_cfg ? g_gemm_cfg : pick_cfg(a, batch);
  if (g_gemm_tiny_cfg && !g_gemm_cfg && a.M <= 128) cfg = g_gemm_tiny_cfg;
  if (g_gemm_w41 && !g_gemm_cfg && !a.out_f32 && (g_gemm_w41 == 1 || a.N >= 768)) cfg = w41_of(cfg);
  if (g_gemm_areg && !g_gemm_cfg && a.K < 256 && a.K % 64 != 0 && !a.out_f32 && a.M > 128 && gemm_areg_ok(a, 256))
    cfg = CFG_64_AREG;
  if (!g_gemm_cfg) {  // A/B override per GEMM class (s2h_gemm_class_config)
    const int cls = gemm_class(a);
    if (cls >= 0 && g_gemm_class_cfg[cls]) cfg = g_gemm_class_cfg[cls];
  }
  if (cfg < 0 || !gemm_glds_ok(a, batch)) return gemm_cfg_launch_1(CFG_REGS, a, batch, st);  // register-staged
  int rc;
  if ((rc = gemm_cfg_launch_1(cfg, a, batch, st)) >= 0) return rc;
  if ((rc = gemm_cfg_launch_2(cfg, a, batch, st)) >= 0) return rc;
  if ((rc = gemm_cfg_launch_3(cfg, a, batch, st)) >= 0) return rc;
  if ((rc = gemm_cfg_launch_4(cfg, a, batch, st)) >= 0) return rc;
  if ((rc = gemm_cfg_launch_5(cfg, a, batch, st)) >= 0) return rc;
  if ((rc = gemm_cfg_launch_6(cfg, a, batch, st)) >= 0) return rc;
  if ((rc = gemm_cfg_launch_7(cfg, a, batch, st)) >= 0) return rc;
  return gemm_cfg_launch_3(CFG_128, a, batch, st);
}
