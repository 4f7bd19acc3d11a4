// Fused mask loss of MultiStepMultiMasksAndIous (losses.py:20-76, 143-238):
// sigmoid focal (alpha .25, gamma 2) + Dice (+1 smoothing) + IoU-L1, with the
// per-frame valid-category filter and logit temperature; plus the category
// merge of masks.py:53-213 (pixelwise max for masks, sigmoid-mass weighted mean
// for IoU predictions) with its backward.
//
// stats[n] = {sum focal, sum sigma, sum t, sum sigma*t, |pred & gt|, |pred | gt|}
#include "common.h"
#include "reduce_det.h"

#define NSTAT 6

// sigmoid(x) and the binary cross-entropy with logits from ONE exponential: e = exp(-|x|),
// sigma = 1 / (1 + e) or e / (1 + e), ce = max(x, 0) - x t + log(1 + e) (hardware exp / log / rcp;
// the libm expf / log1pf / division made the loss kernels compute-bound)
__device__ __forceinline__ float sig_ce(float x, float t, float& ce) {
  const float e = __expf(-fabsf(x));
  const float r = __builtin_amdgcn_rcpf(1.f + e);
  ce = fmaxf(x, 0.f) - x * t + __logf(1.f + e);
  return x >= 0.f ? r : e * r;
}

__device__ __forceinline__ float focal_elem(float x, float t, float& p) {
  float ce;
  p = sig_ce(x, t, ce);
  const float pt = p * t + (1.f - p) * (1.f - t);
  const float at = 0.25f * t + 0.75f * (1.f - t);
  const float q = 1.f - pt;
  return at * ce * q * q;
}

// grid (chunks, N): block-reduce partial sums, atomically added into stats (zeroed by caller)
__global__ __launch_bounds__(256) void mask_stats_kernel(int N, int64_t P, const float* x, int64_t ldx,
                                                         const uint8_t* tgt, int64_t ldt, float inv_temp,
                                                         float* stats, float* part) {
  const int n = blockIdx.y;
  const int64_t chunk = (P + gridDim.x - 1) / gridDim.x;
  const int64_t p0 = blockIdx.x * chunk, p1 = min(P, p0 + chunk);
  float acc[NSTAT] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int64_t p = p0 + threadIdx.x; p < p1; p += 256) {
    const float xv = x[n * ldx + p] * inv_temp;
    const float t = tgt ? (tgt[n * ldt + p] ? 1.f : 0.f) : 0.f;
    float s;
    const float f = focal_elem(xv, t, s);
    const bool pr = xv > 0.f, gt = t > 0.f;
    acc[0] += f; acc[1] += s; acc[2] += t; acc[3] += s * t;
    acc[4] += (pr && gt) ? 1.f : 0.f;
    acc[5] += (pr || gt) ? 1.f : 0.f;
  }
  __shared__ float red[4][NSTAT];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NSTAT; ++k) {
    float v = wave_sum(acc[k]);
    if (lane == 0) red[w][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < NSTAT) {
    float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (part) part[((int64_t)n * gridDim.x + blockIdx.x) * NSTAT + threadIdx.x] = v;
    else atomicAdd(&stats[n * NSTAT + threadIdx.x], v);
  }
}

// 4 consecutive pixels per vector, MV vectors per thread: every load of the thread is issued before
// any arithmetic (the scalar form waited on one dependent load per pixel, ~25 us per 13 x 512^2
// frame; fewer, larger workgroups were slower still -- the kernel is load-latency bound).
// Requires P, ldx, ldt multiples of 4 and 16-B / 4-B aligned bases (checked by the host).
template <int MV>
__global__ __launch_bounds__(256) void mask_stats_vec_kernel(int N, int64_t P, const float* x, int64_t ldx,
                                                             const uint8_t* tgt, int64_t ldt, float inv_temp,
                                                             float* stats, float* part) {
  const int n = blockIdx.y;
  const int64_t p0 = (int64_t)blockIdx.x * (256 * 4 * MV);
  float4 xv[MV];
  uint32_t tv[MV];
#pragma unroll
  for (int j = 0; j < MV; ++j) {
    const int64_t p = p0 + 4 * (threadIdx.x + 256 * j);
    const bool ok = p < P;
    xv[j] = ok ? *(const float4*)(x + n * ldx + p) : float4{0.f, 0.f, 0.f, 0.f};
    tv[j] = ok && tgt ? *(const uint32_t*)(tgt + n * ldt + p) : 0u;
  }
  float acc[NSTAT] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < MV; ++j) {
    if (p0 + 4 * (threadIdx.x + 256 * j) >= P) continue;
    const float xs[4] = {xv[j].x, xv[j].y, xv[j].z, xv[j].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float xe = xs[e] * inv_temp;
      const float t = (tv[j] >> (8 * e)) & 0xffu ? 1.f : 0.f;
      float sg;
      const float f = focal_elem(xe, t, sg);
      const bool pr = xe > 0.f, gt = t > 0.f;
      acc[0] += f; acc[1] += sg; acc[2] += t; acc[3] += sg * t;
      acc[4] += (pr && gt) ? 1.f : 0.f;
      acc[5] += (pr || gt) ? 1.f : 0.f;
    }
  }
  __shared__ float red[4][NSTAT];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NSTAT; ++k) {
    float v = wave_sum(acc[k]);
    if (lane == 0) red[w][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < NSTAT) {
    float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (part) part[((int64_t)n * gridDim.x + blockIdx.x) * NSTAT + threadIdx.x] = v;
    else atomicAdd(&stats[n * NSTAT + threadIdx.x], v);
  }
}

static bool mask_vec4_ok(int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt) {
  return P % 4 == 0 && ldx % 4 == 0 && ((uintptr_t)x & 15) == 0 &&
         (tgt == nullptr || (ldt % 4 == 0 && ((uintptr_t)tgt & 3) == 0));
}

extern "C" int s2h_mask_stats(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt,
                              float inv_temp, float* stats, hipStream_t st) {
  if (N <= 0) return 0;
  constexpr int MV = 2;  // vector kernel: 2 x 4 pixels per thread, 2048 per workgroup
  const bool vec = mask_vec4_ok(P, x, ldx, tgt, ldt);
  int64_t nch = vec ? (P + 256 * 4 * MV - 1) / (256 * 4 * MV) : (P + 4095) / 4096;
  if (!vec && nch > 256) nch = 256;
  if (nch < 1) nch = 1;
  if (nch > 65535) return (int)hipErrorInvalidValue;
  // one partial row per workgroup + a fixed-order finalize (deterministic) when the workspace is
  // there; otherwise float atomics into the zeroed statistics
  float* part = s2h_det_ws((int64_t)N * nch * NSTAT * (int64_t)sizeof(float));
  if (!part) s2h_zero_f32(stats, 1, (int64_t)N * NSTAT, (int64_t)N * NSTAT, st);
  if (vec)
    hipLaunchKernelGGL(mask_stats_vec_kernel<MV>, dim3((unsigned)nch, N), dim3(256), 0, st, N, P, x, ldx, tgt, ldt,
                       inv_temp, stats, part);
  else
    hipLaunchKernelGGL(mask_stats_kernel, dim3((unsigned)nch, N), dim3(256), 0, st, N, P, x, ldx, tgt, ldt, inv_temp,
                       stats, part);
  if (part) det_colsum(N, (int)nch, NSTAT, part, stats, 0, st);
  return (int)hipGetLastError();
}

// One frame: losses[0..3] += {mask, dice, iou, total}; per-row backward coefficients.
// coef[n*4 + 0] = focal coefficient, [1] dice A, [2] dice B, [3] d pred_iou.
__global__ void mask_loss_finalize_kernel(int N, int64_t P, const float* stats, const float* pred_iou,
                                          const int* valid, float w_mask, float w_dice, float w_iou, float gscale,
                                          float* losses, float* coef) {
  if (threadIdx.x != 0) return;
  // valid = categories with ground-truth pixels (losses.py:149-152); derived from the stats
  // when no explicit flags are given
  int nv = 0;
  for (int n = 0; n < N; ++n) nv += (valid ? valid[n] != 0 : stats[n * NSTAT + 2] > 0.f) ? 1 : 0;
  const float inv_nv = nv > 0 ? 1.f / (float)nv : 0.f;
  float lm = 0.f, ld = 0.f, li = 0.f;
  for (int n = 0; n < N; ++n) {
    const float* s = stats + n * NSTAT;
    float* c = coef + n * 4;
    const bool vn = valid ? valid[n] != 0 : s[2] > 0.f;
    if (!vn) { c[0] = c[1] = c[2] = c[3] = 0.f; continue; }
    lm += s[0] / (float)P;
    const float den = s[1] + s[2] + 1.f;
    ld += 1.f - (2.f * s[3] + 1.f) / den;
    const float actual = s[4] / fmaxf(s[5], 1.f);
    const float diff = pred_iou[n] - actual;
    li += fabsf(diff);
    const float cd = gscale * w_dice * inv_nv;
    c[0] = gscale * w_mask * inv_nv / (float)P;
    c[1] = cd * 2.f / den;
    c[2] = cd * (2.f * s[3] + 1.f) / (den * den);
    c[3] = gscale * w_iou * inv_nv * (diff > 0.f ? 1.f : (diff < 0.f ? -1.f : 0.f));
  }
  lm *= inv_nv; ld *= inv_nv; li *= inv_nv;
  losses[0] += lm;
  losses[1] += ld;
  losses[2] += li;
  losses[3] += w_mask * lm + w_dice * ld + w_iou * li;
}
extern "C" int s2h_mask_loss_finalize(int N, int64_t P, const float* stats, const float* pred_iou, const int* valid,
                                      float w_mask, float w_dice, float w_iou, float gscale, float* losses,
                                      float* coef, hipStream_t st) {
  hipLaunchKernelGGL(mask_loss_finalize_kernel, dim3(1), dim3(64), 0, st, N, P, stats, pred_iou, valid, w_mask,
                     w_dice, w_iou, gscale, losses, coef);
  return (int)hipGetLastError();
}

// dx[n,p] = inv_temp * ( cf * dfocal/dx + (-(A t - B)) * sigma' )
__global__ void mask_loss_bwd_kernel(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt,
                                     float inv_temp, const float* coef, float* dx, int64_t lddx, const float* gtot,
                                     float* dious) {
  const int64_t n_all = (int64_t)N * P;
  const float gs = gtot ? gtot[3] : 1.f;  // upstream gradient of the weighted total (device scalar)
  if (dious && blockIdx.x == 0 && threadIdx.x < N) dious[threadIdx.x] = coef[threadIdx.x * 4 + 3] * gs;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_all; i += (int64_t)gridDim.x * blockDim.x) {
    const int n = i / P;
    const int64_t p = i - (int64_t)n * P;
    const float* c = coef + n * 4;
    float g = 0.f;
    if (c[0] != 0.f || c[1] != 0.f || c[2] != 0.f) {
      const float xv = x[n * ldx + p] * inv_temp;
      const float t = tgt[n * ldt + p] ? 1.f : 0.f;
      float ce;
      const float s = sig_ce(xv, t, ce);
      const float ds = s * (1.f - s);
      const float pt = s * t + (1.f - s) * (1.f - t);
      const float at = 0.25f * t + 0.75f * (1.f - t);
      const float q = 1.f - pt;
      const float dfocal = at * (-2.f * q * (2.f * t - 1.f) * ds * ce + q * q * (s - t));
      g = c[0] * dfocal - (c[1] * t - c[2]) * ds;
    }
    dx[n * lddx + p] = g * inv_temp * gs;
  }
}
// 4 consecutive pixels per thread (16-B logit / gradient accesses, 4-B targets); same arithmetic
__global__ void mask_loss_bwd_vec_kernel(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt,
                                         int64_t ldt, float inv_temp, const float* coef, float* dx, int64_t lddx,
                                         const float* gtot, float* dious) {
  const int64_t n4 = (int64_t)N * P / 4;
  const float gs = gtot ? gtot[3] : 1.f;
  if (dious && blockIdx.x == 0 && threadIdx.x < N) dious[threadIdx.x] = coef[threadIdx.x * 4 + 3] * gs;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int n = (4 * i) / P;
    const int64_t p = 4 * i - (int64_t)n * P;
    const float* c = coef + n * 4;
    float g[4] = {0.f, 0.f, 0.f, 0.f};
    if (c[0] != 0.f || c[1] != 0.f || c[2] != 0.f) {
      const float4 x4 = *(const float4*)(x + n * ldx + p);
      const uint32_t t4 = *(const uint32_t*)(tgt + n * ldt + p);
      const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float xv = xs[e] * inv_temp;
        const float t = (t4 >> (8 * e)) & 0xffu ? 1.f : 0.f;
        float ce;
        const float s = sig_ce(xv, t, ce);
        const float ds = s * (1.f - s);
        const float pt = s * t + (1.f - s) * (1.f - t);
        const float at = 0.25f * t + 0.75f * (1.f - t);
        const float q = 1.f - pt;
        const float dfocal = at * (-2.f * q * (2.f * t - 1.f) * ds * ce + q * q * (s - t));
        g[e] = c[0] * dfocal - (c[1] * t - c[2]) * ds;
      }
    }
    const float f = inv_temp * gs;
    *(float4*)(dx + n * lddx + p) = float4{g[0] * f, g[1] * f, g[2] * f, g[3] * f};
  }
}

extern "C" int s2h_mask_loss_bwd(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt,
                                 float inv_temp, const float* coef, float* dx, int64_t lddx, const float* gtot,
                                 float* dious, hipStream_t st) {
  const int64_t n = (int64_t)N * P;
  if (n <= 0) return 0;
  if (N > 256) return (int)hipErrorInvalidValue;
  if (tgt != nullptr && mask_vec4_ok(P, x, ldx, tgt, ldt) && lddx % 4 == 0 && ((uintptr_t)dx & 15) == 0) {
    int64_t b = (n / 4 + 255) / 256;
    if (b > 8192) b = 8192;
    hipLaunchKernelGGL(mask_loss_bwd_vec_kernel, dim3((unsigned)b), dim3(256), 0, st, N, P, x, ldx, tgt, ldt, inv_temp,
                       coef, dx, lddx, gtot, dious);
    return (int)hipGetLastError();
  }
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  hipLaunchKernelGGL(mask_loss_bwd_kernel, dim3((unsigned)b), dim3(256), 0, st, N, P, x, ldx, tgt, ldt, inv_temp,
                     coef, dx, lddx, gtot, dious);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------- BCE category loss
// BCECategoryLoss (losses.py:251-372): per frame, binary_cross_entropy_with_logits over the
// categories with ground-truth pixels (logits / T, optional per-category pos_weight), mean (or
// sum) reduction, averaged over frames.  bce = (1 - t) x + (1 + (pw - 1) t) softplus(-x).
// stats[n] = {sum bce, sum t}
__global__ __launch_bounds__(256) void bce_stats_kernel(int N, int64_t P, const float* x, int64_t ldx,
                                                        const uint8_t* tgt, int64_t ldt, float inv_temp,
                                                        const float* pos_weight, float* stats, float* part) {
  const int n = blockIdx.y;
  const int64_t chunk = (P + gridDim.x - 1) / gridDim.x;
  const int64_t p0 = blockIdx.x * chunk, p1 = min(P, p0 + chunk);
  const float pw = pos_weight ? pos_weight[n] : 1.f;
  float a0 = 0.f, a1 = 0.f;
  for (int64_t p = p0 + threadIdx.x; p < p1; p += 256) {
    const float xv = x[n * ldx + p] * inv_temp;
    const float t = tgt[n * ldt + p] ? 1.f : 0.f;
    const float lw = 1.f + (pw - 1.f) * t;
    a0 += (1.f - t) * xv + lw * (log1pf(expf(-fabsf(xv))) + fmaxf(-xv, 0.f));
    a1 += t;
  }
  __shared__ float red[4][2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  a0 = wave_sum(a0);
  a1 = wave_sum(a1);
  if (lane == 0) { red[w][0] = a0; red[w][1] = a1; }
  __syncthreads();
  if (threadIdx.x < 2) {
    const float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (part) part[((int64_t)n * gridDim.x + blockIdx.x) * 2 + threadIdx.x] = v;
    else atomicAdd(&stats[n * 2 + threadIdx.x], v);
  }
}
extern "C" int s2h_bce_stats(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt,
                             float inv_temp, const float* pos_weight, float* stats, hipStream_t st) {
  if (N <= 0) return 0;
  int chunks = (int)((P + 4095) / 4096);
  if (chunks > 256) chunks = 256;
  if (chunks < 1) chunks = 1;
  float* part = s2h_det_ws((int64_t)N * chunks * 2 * (int64_t)sizeof(float));
  if (!part) s2h_zero_f32(stats, 1, (int64_t)N * 2, (int64_t)N * 2, st);
  hipLaunchKernelGGL(bce_stats_kernel, dim3(chunks, N), dim3(256), 0, st, N, P, x, ldx, tgt, ldt, inv_temp,
                     pos_weight, stats, part);
  if (part) det_colsum(N, chunks, 2, part, stats, 0, st);
  return (int)hipGetLastError();
}
// losses[0] += frame_scale * frame loss; coef[n] = d(frame_scale * loss) / d(bce sum of row n).
// reduction 0 = mean over the valid rows' elements (0/0 = NaN when no row is valid, as torch's
// mean of an empty tensor), 1 = sum.
__global__ void bce_finalize_kernel(int N, int64_t P, const float* stats, int reduction, float frame_scale,
                                    float* losses, float* coef) {
  if (threadIdx.x != 0) return;
  int nv = 0;
  float tot = 0.f;
  for (int n = 0; n < N; ++n) {
    if (stats[n * 2 + 1] > 0.f) { ++nv; tot += stats[n * 2]; }
  }
  const float den = reduction == 0 ? (float)nv * (float)P : 1.f;
  const float c = nv > 0 ? frame_scale / den : 0.f;
  for (int n = 0; n < N; ++n) coef[n] = stats[n * 2 + 1] > 0.f ? c : 0.f;
  losses[0] += frame_scale * (tot / den);
}
extern "C" int s2h_bce_finalize(int N, int64_t P, const float* stats, int reduction, float frame_scale,
                                float* losses, float* coef, hipStream_t st) {
  hipLaunchKernelGGL(bce_finalize_kernel, dim3(1), dim3(64), 0, st, N, P, stats, reduction, frame_scale, losses,
                     coef);
  return (int)hipGetLastError();
}
// dx = gtot * coef[n] * inv_temp * ((1 - t) - (1 + (pw - 1) t) * sigmoid(-x))
__global__ void bce_bwd_kernel(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt,
                               float inv_temp, const float* pos_weight, const float* coef, const float* gtot,
                               float* dx, int64_t lddx) {
  const int64_t n_all = (int64_t)N * P;
  const float gs = gtot ? gtot[0] : 1.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_all; i += (int64_t)gridDim.x * blockDim.x) {
    const int n = i / P;
    const int64_t p = i - (int64_t)n * P;
    float g = 0.f;
    const float c = coef[n];
    if (c != 0.f) {
      const float xv = x[n * ldx + p] * inv_temp;
      const float t = tgt[n * ldt + p] ? 1.f : 0.f;
      const float pw = pos_weight ? pos_weight[n] : 1.f;
      const float lw = 1.f + (pw - 1.f) * t;
      const float sneg = 1.f / (1.f + expf(xv));
      g = c * inv_temp * ((1.f - t) - lw * sneg);
    }
    dx[n * lddx + p] = g * gs;
  }
}
extern "C" int s2h_bce_bwd(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt,
                           float inv_temp, const float* pos_weight, const float* coef, const float* gtot, float* dx,
                           int64_t lddx, hipStream_t st) {
  const int64_t n = (int64_t)N * P;
  if (n <= 0) return 0;
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  hipLaunchKernelGGL(bce_bwd_kernel, dim3((unsigned)b), dim3(256), 0, st, N, P, x, ldx, tgt, ldt, inv_temp,
                     pos_weight, coef, gtot, dx, lddx);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------- category merge
// cat_off[c]..cat_off[c+1] index into cat_obj (object ids of category c).
__global__ void group_max_fwd_kernel(int Ncat, int64_t P, const int* cat_off, const int* cat_obj, const float* x,
                                     int64_t ldx, float* y, int64_t ldy, int* arg) {
  const int64_t n = (int64_t)Ncat * P;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = i / P;
    const int64_t p = i - (int64_t)c * P;
    float m = 0.f;
    int best = -1;
    for (int k = cat_off[c]; k < cat_off[c + 1]; ++k) {
      const int o = cat_obj[k];
      const float v = x[o * ldx + p];
      // first maximum wins ties; the first NaN wins outright (torch.max(dim) semantics)
      if (best < 0 || v > m || (v != v && m == m)) { m = v; best = o; }
    }
    y[c * ldy + p] = m;
    if (arg) arg[i] = best;
  }
}
// dx[o,p] = (arg[cat(o),p] == o) ? dy[cat(o),p] : 0
__global__ void group_max_bwd_kernel(int O, int64_t P, const int* obj_cat, const int* arg, const float* dy,
                                     int64_t lddy, float* dx, int64_t lddx) {
  const int64_t n = (int64_t)O * P;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int o = i / P;
    const int64_t p = i - (int64_t)o * P;
    const int c = obj_cat[o];
    dx[o * lddx + p] = (arg[(int64_t)c * P + p] == o) ? dy[c * lddy + p] : 0.f;
  }
}
// 4 pixels per lane (16-B loads / stores) with the category (object) from blockIdx.y: the scalar forms'
// 64-bit division per element dominated them (11 / 16 us per launch over 13 x 512^2 masks).  Same rule,
// same results.
__global__ __launch_bounds__(256) void group_max_fwd_vec_kernel(int64_t P4, const int* cat_off, const int* cat_obj,
                                                                const float4* x, int64_t ldx4, float4* y, int64_t ldy4,
                                                                int4* arg) {
  const int c = blockIdx.y;
  const int k0 = cat_off[c], k1 = cat_off[c + 1];
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < P4; q += (int64_t)gridDim.x * 256) {
    float m[4] = {0.f, 0.f, 0.f, 0.f};
    int best[4] = {-1, -1, -1, -1};
    for (int k = k0; k < k1; ++k) {
      const int o = cat_obj[k];
      const float4 v4 = x[o * ldx4 + q];
      const float v[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (best[e] < 0 || v[e] > m[e] || (v[e] != v[e] && m[e] == m[e])) { m[e] = v[e]; best[e] = o; }
    }
    y[c * ldy4 + q] = float4{m[0], m[1], m[2], m[3]};
    if (arg) arg[(int64_t)c * P4 + q] = int4{best[0], best[1], best[2], best[3]};
  }
}
__global__ __launch_bounds__(256) void group_max_bwd_vec_kernel(int64_t P4, const int* obj_cat, const int4* arg,
                                                                const float4* dy, int64_t lddy4, float4* dx,
                                                                int64_t lddx4) {
  const int o = blockIdx.y;
  const int c = obj_cat[o];
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < P4; q += (int64_t)gridDim.x * 256) {
    const int4 a = arg[(int64_t)c * P4 + q];
    const float4 g = dy[c * lddy4 + q];
    dx[o * lddx4 + q] = float4{a.x == o ? g.x : 0.f, a.y == o ? g.y : 0.f, a.z == o ? g.z : 0.f, a.w == o ? g.w : 0.f};
  }
}
static bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

extern "C" int s2h_group_max_fwd(int Ncat, int64_t P, const int* cat_off, const int* cat_obj, const float* x,
                                 int64_t ldx, float* y, int64_t ldy, int* arg, hipStream_t st) {
  if (Ncat > 0 && P > 0 && P % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && al16(x) && al16(y) && al16(arg) &&
      Ncat <= 65535) {
    const int64_t P4 = P / 4;
    const dim3 g((unsigned)std::min<int64_t>((P4 + 255) / 256, 2048), (unsigned)Ncat);
    hipLaunchKernelGGL(group_max_fwd_vec_kernel, g, dim3(256), 0, st, P4, cat_off, cat_obj, (const float4*)x, ldx / 4,
                       (float4*)y, ldy / 4, (int4*)arg);
    return (int)hipGetLastError();
  }
  const int64_t n = (int64_t)Ncat * P;
  if (n <= 0) return 0;
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  hipLaunchKernelGGL(group_max_fwd_kernel, dim3((unsigned)b), dim3(256), 0, st, Ncat, P, cat_off, cat_obj, x, ldx, y,
                     ldy, arg);
  return (int)hipGetLastError();
}
extern "C" int s2h_group_max_bwd(int O, int64_t P, const int* obj_cat, const int* arg, const float* dy, int64_t lddy,
                                 float* dx, int64_t lddx, hipStream_t st) {
  if (O > 0 && P > 0 && P % 4 == 0 && lddy % 4 == 0 && lddx % 4 == 0 && al16(arg) && al16(dy) && al16(dx) &&
      O <= 65535) {
    const int64_t P4 = P / 4;
    const dim3 g((unsigned)std::min<int64_t>((P4 + 255) / 256, 2048), (unsigned)O);
    hipLaunchKernelGGL(group_max_bwd_vec_kernel, g, dim3(256), 0, st, P4, obj_cat, (const int4*)arg, (const float4*)dy,
                       lddy / 4, (float4*)dx, lddx / 4);
    return (int)hipGetLastError();
  }
  const int64_t n = (int64_t)O * P;
  if (n <= 0) return 0;
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  hipLaunchKernelGGL(group_max_bwd_kernel, dim3((unsigned)b), dim3(256), 0, st, O, P, obj_cat, arg, dy, lddy, dx,
                     lddx);
  return (int)hipGetLastError();
}

// weighted mean per category: y[c] = sum w_o x_o / sum w_o  (plain mean when sum w == 0; 0 if empty)
// w_o = sum of sigmoid of object o's high-res logits (stats[o*NSTAT + 1]); K values per object.
__global__ void group_wavg_kernel(int Ncat, int K, const int* cat_off, const int* cat_obj, const float* stats,
                                  const float* x, float* y) {
  const int i = threadIdx.x + blockIdx.x * blockDim.x;
  if (i >= Ncat * K) return;
  const int c = i / K, k = i % K;
  float sw = 0.f, sx = 0.f, sm = 0.f;
  const int cnt = cat_off[c + 1] - cat_off[c];
  for (int j = cat_off[c]; j < cat_off[c + 1]; ++j) {
    const int o = cat_obj[j];
    const float w = stats[o * NSTAT + 1];
    sw += w; sx += w * x[o * K + k]; sm += x[o * K + k];
  }
  y[i] = cnt == 0 ? 0.f : (sw == 0.f ? sm / cnt : sx / sw);
}
// backward: dx[o,k] = dy[c,k] * w_o / W ; dw[o] = sum_k dy[c,k] (x_o - y_c) / W   (mean form when W == 0)
__global__ void group_wavg_bwd_kernel(int O, int K, const int* obj_cat, const int* cat_off, const float* stats,
                                      const float* x, const float* y, const float* dy, float* dx, float* dw) {
  const int o = threadIdx.x + blockIdx.x * blockDim.x;
  if (o >= O) return;
  const int c = obj_cat[o];
  const int cnt = cat_off[c + 1] - cat_off[c];
  float sw = 0.f, acc_w = 0.f;
  for (int oo = 0; oo < O; ++oo)
    if (obj_cat[oo] == c) sw += stats[oo * NSTAT + 1];
  const float wo = stats[o * NSTAT + 1];
  for (int k = 0; k < K; ++k) {
    const float g = dy[c * K + k];
    if (sw == 0.f) {
      dx[o * K + k] = g / cnt;
    } else {
      dx[o * K + k] = g * wo / sw;
      acc_w += g * (x[o * K + k] - y[c * K + k]) / sw;
    }
  }
  dw[o] = acc_w;
}
extern "C" int s2h_group_wavg_fwd(int Ncat, int K, const int* cat_off, const int* cat_obj, const float* stats,
                                  const float* x, float* y, hipStream_t st) {
  if (Ncat * K <= 0) return 0;
  hipLaunchKernelGGL(group_wavg_kernel, dim3((Ncat * K + 63) / 64), dim3(64), 0, st, Ncat, K, cat_off, cat_obj, stats,
                     x, y);
  return (int)hipGetLastError();
}
extern "C" int s2h_group_wavg_bwd(int O, int K, const int* obj_cat, const int* cat_off, const float* stats,
                                  const float* x, const float* y, const float* dy, float* dx, float* dw,
                                  hipStream_t st) {
  if (O <= 0) return 0;
  hipLaunchKernelGGL(group_wavg_bwd_kernel, dim3((O + 63) / 64), dim3(64), 0, st, O, K, obj_cat, cat_off, stats, x, y,
                     dy, dx, dw);
  return (int)hipGetLastError();
}

// dx[r,p] += coef[r] * sigma'(x[r,p])   (gradient through the sigmoid-mass merge weights)
__global__ void sigmoid_grad_axpy_kernel(int R, int64_t P, const float* x, int64_t ldx, const float* coef, float* dx,
                                         int64_t lddx) {
  const int64_t n = (int64_t)R * P;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = i / P;
    const int64_t p = i - (int64_t)r * P;
    const float c = coef[r];
    if (c == 0.f) continue;
    const float s = 1.f / (1.f + expf(-x[r * ldx + p]));
    dx[r * lddx + p] += c * s * (1.f - s);
  }
}
extern "C" int s2h_sigmoid_grad_axpy(int R, int64_t P, const float* x, int64_t ldx, const float* coef, float* dx,
                                     int64_t lddx, hipStream_t st) {
  const int64_t n = (int64_t)R * P;
  if (n <= 0) return 0;
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  hipLaunchKernelGGL(sigmoid_grad_axpy_kernel, dim3((unsigned)b), dim3(256), 0, st, R, P, x, ldx, coef, dx, lddx);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ evaluation counts
// Per category n of one frame: counts[n] = {|pred & gt|, |pred | gt|, |pred|, |gt|} with
// pred = (logits > 0) (the binarised category-merged high-res mask the reference writes out
// for evaluation) -- exactly the integer sums behind caculate_iou / caculate_dice /
// caculate_mae (eval/eval.py:16-40): iou = i / (u + 1e-7), dice = 2 i / (|p| + |g| + 1e-7),
// mae = (|p| + |g| - 2 i) / P.  Integer counts: bit-exact against the CPU restatement.
__global__ __launch_bounds__(256) void mask_eval_counts_kernel(int64_t P, const float* x, int64_t ldx,
                                                               const uint8_t* tgt, int64_t ldt,
                                                               unsigned long long* counts) {
  const int n = blockIdx.y;
  const int64_t chunk = (P + gridDim.x - 1) / gridDim.x;
  const int64_t p0 = blockIdx.x * chunk, p1 = min(P, p0 + chunk);
  uint32_t c[4] = {0, 0, 0, 0};
  for (int64_t p = p0 + threadIdx.x; p < p1; p += 256) {
    const bool pr = x[n * ldx + p] > 0.f;
    const bool gt = tgt[n * ldt + p] != 0;
    c[0] += pr && gt;
    c[1] += pr || gt;
    c[2] += pr;
    c[3] += gt;
  }
  __shared__ uint32_t red[4][4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t v = c[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if (lane == 0) red[w][k] = v;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const uint32_t v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(&counts[n * 4 + threadIdx.x], (unsigned long long)v);
  }
}

__global__ void zero_u64_kernel(unsigned long long* p, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = 0ull;
}

extern "C" int s2h_mask_eval_counts(int N, int64_t P, const float* x, int64_t ldx, const uint8_t* tgt, int64_t ldt,
                                    uint64_t* counts, hipStream_t st) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(zero_u64_kernel, dim3((4 * N + 255) / 256), dim3(256), 0, st, (unsigned long long*)counts, 4 * N);
  int chunks = (int)((P + 8191) / 8192);
  if (chunks > 256) chunks = 256;
  if (chunks < 1) chunks = 1;
  hipLaunchKernelGGL(mask_eval_counts_kernel, dim3(chunks, N), dim3(256), 0, st, P, x, ldx, tgt, ldt,
                     (unsigned long long*)counts);
  return (int)hipGetLastError();
}
