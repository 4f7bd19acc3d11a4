// Row LayerNorm forward/backward.
// Covers nn.LayerNorm (Hiera eps 1e-6, hieradet.py:100; memory attention /
// decoder eps 1e-5, memory_attention.py:43-45, transformer.py:137-149) and
// LayerNorm2d (sam2_utils.py:141-153) because every feature map is kept NHWC,
// which turns the channel norm into a row norm over C.
//
// Optional fused pre-add: x = a + b (b broadcast over rows when b_bcast), the
// sum is written to `xsum` so the residual stream is materialised once.
//
// Layout of the vector kernels: a row is split into NC = C / VEC chunks of 16 B
// (VEC = 8 bf16 or 4 f32).  G lanes (a power of two, G <= 64) own one row, lane j
// of the group holds chunks j, j + G, ... (K of them), so one wave normalises
// 64 / G rows per pass with 16-byte loads and stores and group-local shuffles.
// HBM-bound: fwd reads C*(1 [+1 add]) and writes C*(1 [+1 sum]) elements per row,
// bwd reads x, dy (+ the residual-stream gradient) and writes dx.
//
// Backward weight gradients: each block folds its rows' dy*xhat / dy into per-
// block partials in the caller's workspace and a second kernel reduces the
// partials column-wise into dgamma / dbeta (+=).  No same-address atomics: with
// ~10^3 blocks hitting the same 2C words they serialised at L2 and dominated.
#include <algorithm>
#include <initializer_list>

#include "common.h"

// ------------------------------------------------------------ group helpers
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T> struct Chunk;
template <> struct Chunk<bf16> {
  static constexpr int VEC = 8;
  static __device__ __forceinline__ void load(const bf16* p, float* v) {
    const bf16x8 r = *(const bf16x8*)p;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)r[j];
  }
  static __device__ __forceinline__ void store(bf16* p, const float* v) {
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (bf16)v[j];
    *(bf16x8*)p = r;
  }
};
template <> struct Chunk<float> {
  static constexpr int VEC = 4;
  static __device__ __forceinline__ void load(const float* p, float* v) {
    const f32x4 r = *(const f32x4*)p;
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = r[j];
  }
  static __device__ __forceinline__ void store(float* p, const float* v) {
    f32x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = v[j];
    *(f32x4*)p = r;
  }
};

// VEC consecutive fp32 parameters (gamma / beta): 16-B loads when aligned (parameter arena
// slices need not be), scalar loads otherwise
template <int VEC>
__device__ __forceinline__ void load_param(const float* p, float* out) {
  if (((uintptr_t)p & 15) == 0) {
#pragma unroll
    for (int h = 0; h < VEC / 4; ++h) {
      const f32x4 v = ((const f32x4*)p)[h];
#pragma unroll
      for (int j = 0; j < 4; ++j) out[4 * h + j] = v[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) out[j] = p[j];
  }
}

// ------------------------------------------------------------ forward (vector)
// PE: also ype = y + pe[row % pe_rows] (the stored y, rounded to T, plus a positional table; the
// add_bcast it replaces rounds the same fp32 sum) -- the two-way transformer's keys + key_pe after
// norm4 (transformer.py:182-185 feeding :170 / :102)
template <typename T, int G, int K, bool PE = false>
__global__ __launch_bounds__(256) void ln_fwd_vec_kernel(int rows, int C, const T* a, int64_t lda, const T* badd,
                                                         int64_t ldb, int b_bcast, T* xsum, const float* gamma,
                                                         const float* beta, float eps, T* y, int64_t ldy,
                                                         float* mean, float* rstd, const T* pe, int pe_rows,
                                                         T* ype) {
  constexpr int VEC = Chunk<T>::VEC;
  constexpr int RPW = 64 / G;  // rows per wave
  const int lane = threadIdx.x & 63;
  const int gl = lane & (G - 1);
  const int64_t row = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / G;
  const bool live = row < rows;
  const int NC = C / VEC;
  // gamma / beta first: their loads then overlap the row loads instead of adding a memory
  // round trip after the two reductions (the kernel is one short latency chain per wave)
  float gv[K][VEC], bv[K][VEC];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int ch = gl + k * G;
    if (gamma && ch < NC) {
      load_param<VEC>(gamma + ch * VEC, gv[k]);
      load_param<VEC>(beta + ch * VEC, bv[k]);
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) { gv[k][j] = 1.f; bv[k][j] = 0.f; }
    }
  }
  float v[K][VEC];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int ch = gl + k * G;
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[k][j] = 0.f;
    if (live && ch < NC) {
      Chunk<T>::load(a + row * lda + ch * VEC, v[k]);
      if (badd) {
        float b[VEC];
        Chunk<T>::load(badd + (b_bcast ? 0 : row * ldb) + ch * VEC, b);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          v[k][j] += b[j];
          if constexpr (sizeof(T) == 2) v[k][j] = (float)(bf16)v[k][j];  // residual stream stored in T
        }
        if (xsum) Chunk<T>::store(xsum + row * (int64_t)C + ch * VEC, v[k]);
      }
#pragma unroll
      for (int j = 0; j < VEC; ++j) s += v[k][j];
    }
  }
  const float mu = group_sum<G>(s) / C;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (gl + k * G < NC) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) { const float d = v[k][j] - mu; q += d * d; }
    }
  }
  const float rs = 1.f / sqrtf(group_sum<G>(q) / C + eps);
  if (!live) return;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int ch = gl + k * G;
    if (ch < NC) {
      float o[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = (v[k][j] - mu) * rs * gv[k][j] + bv[k][j];
      Chunk<T>::store(y + row * ldy + ch * VEC, o);
      if constexpr (PE) {
        float t[VEC];
        Chunk<T>::load(pe + (row % pe_rows) * (int64_t)C + ch * VEC, t);
#pragma unroll
        for (int j = 0; j < VEC; ++j) t[j] += (float)(T)o[j];
        Chunk<T>::store(ype + row * (int64_t)C + ch * VEC, t);
      }
    }
  }
  if (gl == 0) { mean[row] = mu; rstd[row] = rs; }
}

// ------------------------------------------------------------ backward (vector)
// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)) [+ dres],  g = dy * gamma
// partial[block] = (sum_rows dy * xhat, sum_rows dy)  -> ln_wgrad_finalize_kernel
template <typename T, int G, int K>
__global__ __launch_bounds__(256) void ln_bwd_vec_kernel(int rows, int C, const T* x, int64_t ldx, const T* dy,
                                                         int64_t lddy, const float* gamma, const float* mean,
                                                         const float* rstd, T* dx, int64_t lddx, int dx_accum,
                                                         const T* dres, int64_t ldres, float* part) {
  constexpr int VEC = Chunk<T>::VEC;
  constexpr int RPW = 64 / G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int gl = lane & (G - 1);
  const int NC = C / VEC;
  float pg[K][VEC], pb[K][VEC];
#pragma unroll
  for (int k = 0; k < K; ++k)
#pragma unroll
    for (int j = 0; j < VEC; ++j) { pg[k][j] = 0.f; pb[k][j] = 0.f; }
  float gk[K][VEC];  // gamma of this lane's chunks, loaded once (row-independent)
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int ch = gl + k * G;
    if (gamma && ch < NC) {
      load_param<VEC>(gamma + ch * VEC, gk[k]);
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) gk[k][j] = 1.f;
    }
  }
  const int64_t stride = (int64_t)gridDim.x * 4 * RPW;
  for (int64_t row = ((int64_t)blockIdx.x * 4 + w) * RPW + lane / G; row - lane / G < rows; row += stride) {
    const bool live = row < rows;
    const float mu = live ? mean[row] : 0.f, rs = live ? rstd[row] : 0.f;
    float xh[K][VEC], g[K][VEC], r[K][VEC];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int ch = gl + k * G;
#pragma unroll
      for (int j = 0; j < VEC; ++j) { xh[k][j] = 0.f; g[k][j] = 0.f; r[k][j] = 0.f; }
      if (live && ch < NC) {
        float xv[VEC], d[VEC];
        Chunk<T>::load(x + row * ldx + ch * VEC, xv);
        Chunk<T>::load(dy + row * lddy + ch * VEC, d);
        // the addend now, not after the reductions: one memory round trip per row instead of two
        if (dx_accum || dres)
          Chunk<T>::load(dx_accum ? dx + row * lddx + ch * VEC : dres + row * ldres + ch * VEC, r[k]);
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          xh[k][j] = (xv[j] - mu) * rs;
          pg[k][j] += d[j] * xh[k][j];
          pb[k][j] += d[j];
          g[k][j] = d[j] * gk[k][j];
          s1 += g[k][j];
          s2 += g[k][j] * xh[k][j];
        }
      }
    }
    s1 = group_sum<G>(s1) / C;
    s2 = group_sum<G>(s2) / C;
    if (live) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int ch = gl + k * G;
        if (ch < NC) {
          float o[VEC];
#pragma unroll
          for (int j = 0; j < VEC; ++j) o[j] = rs * (g[k][j] - s1 - xh[k][j] * s2) + r[k][j];
          Chunk<T>::store(dx + row * lddx + ch * VEC, o);
        }
      }
    }
  }
  if (!part) return;
  // fold the RPW row groups of the wave (lanes with equal gl), then the 4 waves via LDS
#pragma unroll
  for (int o = 32; o >= G; o >>= 1) {
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        pg[k][j] += __shfl_xor(pg[k][j], o, 64);
        pb[k][j] += __shfl_xor(pb[k][j], o, 64);
      }
  }
  extern __shared__ float sh[];  // [4 waves][2C]
  if (lane < G) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int ch = gl + k * G;
      if (ch < NC) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          sh[w * 2 * C + ch * VEC + j] = pg[k][j];
          sh[w * 2 * C + C + ch * VEC + j] = pb[k][j];
        }
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * C; c += 256)
    part[(int64_t)blockIdx.x * 2 * C + c] = sh[c] + sh[2 * C + c] + sh[4 * C + c] + sh[6 * C + c];
}

// dgamma[c] += sum_b part[b][c], dbeta[c] += sum_b part[b][C + c], deterministic: one workgroup per 64
// columns, 1024 threads = 64 columns x 16 slices; slice s sums the rows b = s, s + 16, ... in order
// (independent loads in flight), the 16 slice sums are added in a fixed tree through LDS, and one thread
// per column updates it (no atomics: the round-4 form added up to 32 slices with float atomics, in an
// order that changed from run to run)
__global__ __launch_bounds__(1024) void ln_wgrad_finalize_kernel(int nb, int C, const float* part, float* dgamma,
                                                                 float* dbeta) {
  __shared__ float sh[16][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sl = threadIdx.x >> 6;
  float s = 0.f;
  if (col < 2 * C) {
#pragma unroll 8
    for (int b = sl; b < nb; b += 16) s += part[(int64_t)b * 2 * C + col];
  }
  sh[sl][threadIdx.x & 63] = s;
  __syncthreads();
#pragma unroll
  for (int h = 8; h >= 1; h >>= 1) {
    if (sl < h) sh[sl][threadIdx.x & 63] += sh[sl + h][threadIdx.x & 63];
    __syncthreads();
  }
  if (sl == 0 && col < 2 * C) {
    float* d = col < C ? &dgamma[col] : &dbeta[col - C];
    *d += sh[0][threadIdx.x];
  }
}

// ------------------------------------------------------------ scalar fallback (C % VEC != 0, unaligned rows)
template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int rows, int C, const T* a, int64_t lda, const T* badd,
                                                     int64_t ldb, int b_bcast, T* xsum, const float* gamma,
                                                     const float* beta, float eps, T* y, int64_t ldy, float* mean,
                                                     float* rstd) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* x = a + row * lda;
  const T* bb = badd ? badd + (b_bcast ? 0 : row * ldb) : nullptr;
  T* xs = xsum ? xsum + row * (int64_t)C : nullptr;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) {
    float t = to_f32(x[c]);
    if (bb) {
      t += to_f32(bb[c]);
      if constexpr (sizeof(T) == 2) t = (float)(bf16)t;
      if (xs) xs[c] = from_f32<T>(t);
    }
    s += t;
  }
  const float mu = wave_sum(s) / C;
  float q = 0.f;
  for (int c = lane; c < C; c += 64) {
    float t = to_f32(x[c]);
    if (bb) {
      t += to_f32(bb[c]);
      if constexpr (sizeof(T) == 2) t = (float)(bf16)t;
    }
    q += (t - mu) * (t - mu);
  }
  const float rs = 1.f / sqrtf(wave_sum(q) / C + eps);
  T* yr = y + row * ldy;
  for (int c = lane; c < C; c += 64) {
    float t = to_f32(x[c]);
    if (bb) {
      t += to_f32(bb[c]);
      if constexpr (sizeof(T) == 2) t = (float)(bf16)t;
    }
    float o = (t - mu) * rs;
    if (gamma) o = o * gamma[c] + beta[c];
    yr[c] = from_f32<T>(o);
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int rows, int C, const T* x, int64_t ldx, const T* dy,
                                                     int64_t lddy, const float* gamma, const float* mean,
                                                     const float* rstd, T* dx, int64_t lddx, int dx_accum,
                                                     const T* dres, int64_t ldres, float* part) {
  extern __shared__ float sh[];  // [4 waves][2C] floats: each wave's own partial row (no LDS atomics)
  for (int c = threadIdx.x; c < 8 * C; c += 256) sh[c] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* shw = sh + w * 2 * C;
  for (int64_t row = (int64_t)blockIdx.x * 4 + w; row < rows; row += (int64_t)gridDim.x * 4) {
    const T* xr = x + row * ldx;
    const T* gr = dy + row * lddy;
    const float mu = mean[row], rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
    for (int c = lane; c < C; c += 64) {
      const float d = to_f32(gr[c]);
      const float xh = (to_f32(xr[c]) - mu) * rs;
      const float g = gamma ? d * gamma[c] : d;
      s1 += g;
      s2 += g * xh;
      if (part) { shw[c] += d * xh; shw[C + c] += d; }  // lane-exclusive columns of the wave's row
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
    T* dxr = dx + row * lddx;
    for (int c = lane; c < C; c += 64) {
      const float d = to_f32(gr[c]);
      const float xh = (to_f32(xr[c]) - mu) * rs;
      const float g = gamma ? d * gamma[c] : d;
      float o = rs * (g - s1 - xh * s2);
      if (dx_accum) o += to_f32(dxr[c]);
      else if (dres) o += to_f32(dres[row * ldres + c]);
      dxr[c] = from_f32<T>(o);
    }
  }
  if (!part) return;
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * C; c += 256)
    part[(int64_t)blockIdx.x * 2 * C + c] = (sh[c] + sh[2 * C + c]) + (sh[4 * C + c] + sh[6 * C + c]);
}

// ------------------------------------------------------------ launch plumbing
namespace {
constexpr int kMaxBwdBlocks = 1024;

struct LnPlan {
  bool vec;
  int G, K;
};

template <typename T>
LnPlan plan(int C, std::initializer_list<int64_t> lds, std::initializer_list<const void*> ptrs) {
  constexpr int VEC = 16 / sizeof(T);
  LnPlan p{false, 64, 1};
  if (C % VEC) return p;
  for (int64_t ld : lds)
    if (ld % VEC) return p;
  for (const void* q : ptrs)
    if (q && ((uintptr_t)q & 15)) return p;
  const int NC = C / VEC;
  if (NC <= 64) {
    int G = 1;
    while (G < NC) G <<= 1;
    p = {true, G, 1};
  } else {
    const int K = (NC + 63) / 64;
    if (K > 5) return p;
    p = {true, 64, K == 4 ? 5 : K};
  }
  return p;
}

int bwd_blocks(int rows, const LnPlan& p) {
  const int rpb = p.vec ? 4 * (64 / p.G) : 4;
  int nb = (rows + rpb - 1) / rpb;
  return nb > kMaxBwdBlocks ? kMaxBwdBlocks : nb;
}

template <typename T, int G, int K>
void fwd_launch(int rows, dim3 blk, hipStream_t st, int C, const T* x, int64_t ldx, const T* badd, int64_t ldb,
                int b_bcast, T* xsum, const float* gamma, const float* beta, float eps, T* y, int64_t ldy,
                float* mean, float* rstd) {
  const int rpb = 4 * (64 / G);
  hipLaunchKernelGGL((ln_fwd_vec_kernel<T, G, K>), dim3((rows + rpb - 1) / rpb), blk, 0, st, rows, C, x, ldx, badd,
                     ldb, b_bcast, xsum, gamma, beta, eps, y, ldy, mean, rstd, nullptr, 1, nullptr);
}

template <typename T, int G, int K>
void bwd_launch(int nb, hipStream_t st, int rows, int C, const T* x, int64_t ldx, const T* dy, int64_t lddy,
                const float* gamma, const float* mean, const float* rstd, T* dx, int64_t lddx, int dx_accum,
                const T* dres, int64_t ldres, float* part) {
  hipLaunchKernelGGL((ln_bwd_vec_kernel<T, G, K>), dim3(nb), dim3(256), part ? 8 * C * sizeof(float) : 0, st, rows,
                     C, x, ldx, dy, lddy, gamma, mean, rstd, dx, lddx, dx_accum, dres, ldres, part);
}

#define S2H_LN_DISPATCH(FN, P, ...)                                   \
  do {                                                                \
    if ((P).K == 1) {                                                 \
      switch ((P).G) {                                                \
        case 1: FN<T, 1, 1>(__VA_ARGS__); break;                      \
        case 2: FN<T, 2, 1>(__VA_ARGS__); break;                      \
        case 4: FN<T, 4, 1>(__VA_ARGS__); break;                      \
        case 8: FN<T, 8, 1>(__VA_ARGS__); break;                      \
        case 16: FN<T, 16, 1>(__VA_ARGS__); break;                    \
        case 32: FN<T, 32, 1>(__VA_ARGS__); break;                    \
        default: FN<T, 64, 1>(__VA_ARGS__); break;                    \
      }                                                               \
    } else if ((P).K == 2) {                                          \
      FN<T, 64, 2>(__VA_ARGS__);                                      \
    } else if ((P).K == 3) {                                          \
      FN<T, 64, 3>(__VA_ARGS__);                                      \
    } else {                                                          \
      FN<T, 64, 5>(__VA_ARGS__);                                      \
    }                                                                 \
  } while (0)

template <typename T>
int ln_fwd(int rows, int C, const T* x, int64_t ldx, const T* badd, int64_t ldb, int b_bcast, T* xsum,
           const float* gamma, const float* beta, float eps, T* y, int64_t ldy, float* mean, float* rstd,
           hipStream_t st) {
  const LnPlan p = plan<T>(C, {ldx, b_bcast ? 0 : ldb, ldy}, {x, badd, xsum, y});
  if (p.vec) {
    S2H_LN_DISPATCH(fwd_launch, p, rows, dim3(256), st, C, x, ldx, badd, ldb, b_bcast, xsum, gamma, beta, eps, y,
                    ldy, mean, rstd);
  } else {
    hipLaunchKernelGGL(ln_fwd_kernel<T>, dim3((rows + 3) / 4), dim3(256), 0, st, rows, C, x, ldx, badd, ldb, b_bcast,
                       xsum, gamma, beta, eps, y, ldy, mean, rstd);
  }
  return (int)hipGetLastError();
}

template <typename T>
int ln_bwd(int rows, int C, const T* x, int64_t ldx, const T* dy, int64_t lddy, const float* gamma, const float* mean,
           const float* rstd, T* dx, int64_t lddx, int dx_accum, const T* dres, int64_t ldres, float* dgamma,
           float* dbeta, float* ws, hipStream_t st) {
  const LnPlan p = plan<T>(C, {ldx, lddy, lddx, dres ? ldres : 0}, {x, dy, dx, dres});
  const int nb = bwd_blocks(rows, p);
  // gamma / beta gradients into the arena inside a deferral scope: the fixed-order sum of the block
  // partials runs later, batched with the step's other deferred sums (grad_defer.hip)
  float* deferred = dgamma ? s2h_defer_sink(nb, C, dgamma, C, dbeta, st) : nullptr;
  float* part = deferred ? deferred : dgamma ? ws : nullptr;
  if (dgamma && !part) return (int)hipErrorInvalidValue;
  if (p.vec) {
    S2H_LN_DISPATCH(bwd_launch, p, nb, st, rows, C, x, ldx, dy, lddy, gamma, mean, rstd, dx, lddx, dx_accum, dres,
                    ldres, part);
  } else {
    hipLaunchKernelGGL(ln_bwd_kernel<T>, dim3(nb), dim3(256), 8 * C * sizeof(float), st, rows, C, x, ldx, dy, lddy,
                       gamma, mean, rstd, dx, lddx, dx_accum, dres, ldres, part);
  }
  if (part && !deferred)
    hipLaunchKernelGGL(ln_wgrad_finalize_kernel, dim3((2 * C + 63) / 64), dim3(1024), 0, st, nb, C, part, dgamma, dbeta);
  return (int)hipGetLastError();
}
}  // namespace

extern "C" int s2h_layernorm_fwd(int dt, int rows, int C, const void* x, int64_t ldx, const void* badd, int64_t ldb,
                                 int b_bcast, void* xsum, const float* gamma, const float* beta, float eps, void* y,
                                 int64_t ldy, float* mean, float* rstd, hipStream_t st) {
  if (rows <= 0) return 0;
  if (C <= 0 || C > 1280) return (int)hipErrorInvalidValue;
  if (dt == S2H_BF16)
    return ln_fwd<bf16>(rows, C, (const bf16*)x, ldx, (const bf16*)badd, ldb, b_bcast, (bf16*)xsum, gamma, beta, eps,
                        (bf16*)y, ldy, mean, rstd, st);
  return ln_fwd<float>(rows, C, (const float*)x, ldx, (const float*)badd, ldb, b_bcast, (float*)xsum, gamma, beta,
                       eps, (float*)y, ldy, mean, rstd, st);
}

// LayerNorm of contiguous bf16 rows (C / 8 lanes per row, the vector plan) that also stores
// ype = y + pe[row % pe_rows]: y bit-identical to s2h_layernorm_fwd, ype to its add_bcast
extern "C" int s2h_layernorm_fwd_pe(int dt, int rows, int C, const void* x, const float* gamma, const float* beta,
                                    float eps, void* y, float* mean, float* rstd, const void* pe, int pe_rows,
                                    void* ype, hipStream_t st) {
  if (rows <= 0) return 0;
  if (dt != S2H_BF16 || C <= 0 || C > 1280 || pe == nullptr || ype == nullptr || pe_rows <= 0)
    return (int)hipErrorInvalidValue;
  const LnPlan p = plan<bf16>(C, {C, 0, C}, {x, nullptr, nullptr, y});
  if (!p.vec || p.K != 1 || ((uintptr_t)pe & 15) || ((uintptr_t)ype & 15)) return (int)hipErrorInvalidValue;
  const int rpb = 4 * (64 / p.G);
  const dim3 grid((rows + rpb - 1) / rpb);
  const bf16* xb = (const bf16*)x;
#define S2H_LN_PE(GG)                                                                                           \
  hipLaunchKernelGGL((ln_fwd_vec_kernel<bf16, GG, 1, true>), grid, dim3(256), 0, st, rows, C, xb, (int64_t)C,   \
                     (const bf16*)nullptr, (int64_t)0, 0, (bf16*)nullptr, gamma, beta, eps, (bf16*)y, (int64_t)C, \
                     mean, rstd, (const bf16*)pe, pe_rows, (bf16*)ype)
  switch (p.G) {
    case 8: S2H_LN_PE(8); break;
    case 16: S2H_LN_PE(16); break;
    case 32: S2H_LN_PE(32); break;
    case 64: S2H_LN_PE(64); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef S2H_LN_PE
  return (int)hipGetLastError();
}

// dgamma += sum_b part[b][0:C], dbeta += sum_b part[b][C:2C] (partial rows written by a fused
// LayerNorm-backward epilogue, gemm.hip s2h_linear_dgrad_ln_bwd)
extern "C" int s2h_ln_wgrad_finalize(int nb, int C, const float* part, float* dgamma, float* dbeta, hipStream_t st) {
  if (nb <= 0) return 0;
  if (C <= 0 || !part || !dgamma || !dbeta) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ln_wgrad_finalize_kernel, dim3((2 * C + 63) / 64), dim3(1024), 0, st, nb, C, part, dgamma, dbeta);
  return (int)hipGetLastError();
}

extern "C" int64_t s2h_layernorm_bwd_ws_bytes(int dt, int rows, int C) {
  if (rows <= 0 || C <= 0) return 0;
  const LnPlan p = dt == S2H_BF16 ? plan<bf16>(C, {}, {}) : plan<float>(C, {}, {});
  // the scalar fallback may use more blocks than the vector plan: size for the larger
  const int nb = std::max(bwd_blocks(rows, p), bwd_blocks(rows, LnPlan{false, 64, 1}));
  return (int64_t)nb * 2 * C * sizeof(float);
}

extern "C" int s2h_layernorm_bwd(int dt, int rows, int C, const void* x, int64_t ldx, const void* dy, int64_t lddy,
                                 const float* gamma, const float* mean, const float* rstd, void* dx, int64_t lddx,
                                 int dx_accum, const void* dres, int64_t ldres, float* dgamma, float* dbeta, void* ws,
                                 hipStream_t st) {
  if (rows <= 0) return 0;
  if (C <= 0 || C > 1280 || (dx_accum && dres) || ((dgamma == nullptr) != (dbeta == nullptr)))
    return (int)hipErrorInvalidValue;
  if (dt == S2H_BF16)
    return ln_bwd<bf16>(rows, C, (const bf16*)x, ldx, (const bf16*)dy, lddy, gamma, mean, rstd, (bf16*)dx, lddx,
                        dx_accum, (const bf16*)dres, ldres, dgamma, dbeta, (float*)ws, st);
  return ln_bwd<float>(rows, C, (const float*)x, ldx, (const float*)dy, lddy, gamma, mean, rstd, (float*)dx, lddx,
                       dx_accum, (const float*)dres, ldres, dgamma, dbeta, (float*)ws, st);
}
