// Row LayerNorm forward/backward (wavefront-reduced, one wave per row).
// Covers nn.LayerNorm (Hiera eps 1e-6, hieradet.py:100; memory attention /
// decoder eps 1e-5, memory_attention.py:43-45, transformer.py:137-149) and
// LayerNorm2d (sam2_utils.py:141-153) because every feature map is kept NHWC,
// which turns the channel norm into a row norm over C.
//
// Optional fused pre-add: x = a + b (b broadcast over rows when b_rows == 1),
// the sum is written to `xsum` so the residual stream is materialised once.
#include "common.h"

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
  constexpr int MAXE = 20;  // C <= 1280
  float v[MAXE];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXE; ++i) {
    int c = lane + i * 64;
    float t = 0.f;
    if (c < C) {
      t = to_f32(x[c]);
      if (bb) {
        t += to_f32(bb[c]);
        if constexpr (sizeof(T) == 2) t = (float)(bf16)t;  // residual stream stored in T
      }
      if (xs) xs[c] = from_f32<T>(t);
    }
    v[i] = t;
    s += t;
  }
  const float mu = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXE; ++i) {
    int c = lane + i * 64;
    if (c < C) { float d = v[i] - mu; q += d * d; }
  }
  const float var = wave_sum(q) / C;
  const float rs = 1.f / sqrtf(var + eps);
  T* yr = y + row * ldy;
#pragma unroll
  for (int i = 0; i < MAXE; ++i) {
    int c = lane + i * 64;
    if (c < C) {
      float o = (v[i] - mu) * rs;
      if (gamma) o = o * gamma[c] + beta[c];
      yr[c] = from_f32<T>(o);
    }
  }
  if (lane == 0) { mean[row] = mu; rstd[row] = rs; }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * gamma
// dgamma += sum_rows dy * xhat ; dbeta += sum_rows dy   (LDS partials + one atomic per column per block)
template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int rows, int C, const T* x, int64_t ldx, const T* dy,
                                                     int64_t lddy, const float* gamma, const float* mean,
                                                     const float* rstd, T* dx, int64_t lddx, int dx_accum,
                                                     float* dgamma, float* dbeta) {
  extern __shared__ float sh[];  // 2*C floats
  float* sg = sh;
  float* sb = sh + C;
  for (int c = threadIdx.x; c < 2 * C; c += 256) sh[c] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int MAXE = 20;
  float pg[MAXE], pb[MAXE];
#pragma unroll
  for (int i = 0; i < MAXE; ++i) { pg[i] = 0.f; pb[i] = 0.f; }
  for (int64_t row = (int64_t)blockIdx.x * 4 + w; row < rows; row += (int64_t)gridDim.x * 4) {
    const T* xr = x + row * ldx;
    const T* gr = dy + row * lddy;
    const float mu = mean[row], rs = rstd[row];
    float xh[MAXE], g[MAXE];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
      int c = lane + i * 64;
      xh[i] = 0.f; g[i] = 0.f;
      if (c < C) {
        float d = to_f32(gr[c]);
        xh[i] = (to_f32(xr[c]) - mu) * rs;
        pg[i] += d * xh[i];
        pb[i] += d;
        g[i] = gamma ? d * gamma[c] : d;
        s1 += g[i];
        s2 += g[i] * xh[i];
      }
    }
    s1 = wave_sum(s1) / C;
    s2 = wave_sum(s2) / C;
    T* dxr = dx + row * lddx;
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
      int c = lane + i * 64;
      if (c < C) {
        float o = rs * (g[i] - s1 - xh[i] * s2);
        if (dx_accum) o += to_f32(dxr[c]);
        dxr[c] = from_f32<T>(o);
      }
    }
  }
  if (dgamma) {
#pragma unroll
    for (int i = 0; i < MAXE; ++i) {
      int c = lane + i * 64;
      if (c < C) { atomicAdd(&sg[c], pg[i]); atomicAdd(&sb[c], pb[i]); }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += 256) {
      atomicAdd(&dgamma[c], sg[c]);
      atomicAdd(&dbeta[c], sb[c]);
    }
  }
}

extern "C" int s2h_layernorm_fwd(int dt, int rows, int C, const void* x, int64_t ldx, const void* badd, int64_t ldb,
                                 int b_bcast, void* xsum, const float* gamma, const float* beta, float eps, void* y,
                                 int64_t ldy, float* mean, float* rstd, hipStream_t st) {
  if (rows <= 0) return 0;
  if (C > 1280) return (int)hipErrorInvalidValue;
  dim3 grid((rows + 3) / 4);
  if (dt == S2H_BF16)
    hipLaunchKernelGGL(ln_fwd_kernel<bf16>, grid, dim3(256), 0, st, rows, C, (const bf16*)x, ldx, (const bf16*)badd,
                       ldb, b_bcast, (bf16*)xsum, gamma, beta, eps, (bf16*)y, ldy, mean, rstd);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<float>, grid, dim3(256), 0, st, rows, C, (const float*)x, ldx,
                       (const float*)badd, ldb, b_bcast, (float*)xsum, gamma, beta, eps, (float*)y, ldy, mean, rstd);
  return (int)hipGetLastError();
}

extern "C" int s2h_layernorm_bwd(int dt, int rows, int C, const void* x, int64_t ldx, const void* dy, int64_t lddy,
                                 const float* gamma, const float* mean, const float* rstd, void* dx, int64_t lddx,
                                 int dx_accum, float* dgamma, float* dbeta, hipStream_t st) {
  if (rows <= 0) return 0;
  if (C > 1280) return (int)hipErrorInvalidValue;
  int nb = (rows + 3) / 4;
  if (nb > 1024) nb = 1024;
  size_t sh = 2 * C * sizeof(float);
  if (dt == S2H_BF16)
    hipLaunchKernelGGL(ln_bwd_kernel<bf16>, dim3(nb), dim3(256), sh, st, rows, C, (const bf16*)x, ldx,
                       (const bf16*)dy, lddy, gamma, mean, rstd, (bf16*)dx, lddx, dx_accum, dgamma, dbeta);
  else
    hipLaunchKernelGGL(ln_bwd_kernel<float>, dim3(nb), dim3(256), sh, st, rows, C, (const float*)x, ldx,
                       (const float*)dy, lddy, gamma, mean, rstd, (float*)dx, lddx, dx_accum, dgamma, dbeta);
  return (int)hipGetLastError();
}
