// Optimizer step over the flat fp32 parameter / gradient arena:
// global grad-norm (deterministic two-stage reduction), clip_grad_norm_ factor
// computed on device (no host sync), and a fused AdamW update that applies the
// clip factor on the fly (torch.optim.AdamW semantics, trainer.py:124-130:
// decoupled decay p *= 1 - lr*wd, m.lerp_(g, 1-b1), v = b2*v + (1-b2) g^2,
// p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)).
// Also: fp32 -> bf16 shadow-weight refresh for the bf16 compute path.
#include "common.h"

// partial[b] = sum over block b of x^2
// 16-B loads, four loads in flight per thread and four accumulator chains (the scalar grid-stride
// loop read the 316 MB arena at 2.4 TB/s); the assignment of elements to threads and the order of
// every sum are fixed by the launch shape (deterministic)
__global__ __launch_bounds__(256) void sumsq_kernel(int64_t n, const float* x, float* partial) {
  float acc = 0.f;
  if (((uintptr_t)x & 15) == 0) {
    const int64_t n4 = n / 4, stride = (int64_t)gridDim.x * 256;
    const float4* x4 = (const float4*)x;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + 3 * stride < n4; i += 4 * stride) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = x4[i + u * stride];
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += v[u].x * v[u].x + v[u].y * v[u].y + v[u].z * v[u].z + v[u].w * v[u].w;
    }
    for (; i < n4; i += stride) {
      const float4 v = x4[i];
      a[0] += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    acc = (a[0] + a[1]) + (a[2] + a[3]);
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) acc += x[4 * n4 + threadIdx.x] * x[4 * n4 + threadIdx.x];
  } else {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) acc += x[i] * x[i];
  }
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
// out[0] = sqrt(sum partial); out[1] = clip coefficient min(1, max_norm / (norm + 1e-6)) (1 if max_norm <= 0)
// grad_scale: the stored gradient is scaled by this factor before use (1/world after a
// SUM all-reduce); out[1] = grad_scale * clip coefficient, the factor AdamW applies.
__global__ __launch_bounds__(256) void norm_finalize_kernel(int nb, const float* partial, float max_norm,
                                                            float grad_scale, float* out) {
  float acc = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) acc += partial[i];
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float norm = sqrtf(red[0] + red[1] + red[2] + red[3]) * grad_scale;
    out[0] = norm;
    float c = 1.f;
    if (max_norm > 0.f) {
      c = max_norm / (norm + 1e-6f);
      if (c > 1.f) c = 1.f;
    }
    out[1] = c * grad_scale;
  }
}
#define NORM_BLOCKS 1024
extern "C" int s2h_grad_norm(int64_t n, const float* g, float* partial_ws, float max_norm, float grad_scale,
                             float* out, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(NORM_BLOCKS), dim3(256), 0, st, n, g, partial_ws);
  hipLaunchKernelGGL(norm_finalize_kernel, dim3(1), dim3(256), 0, st, NORM_BLOCKS, partial_ws, max_norm, grad_scale,
                     out);
  return (int)hipGetLastError();
}

// One element's AdamW update (torch.optim.AdamW, decoupled weight decay), every rounding step written
// out (explicit fmaf) so the scalar and the 16-B kernels below produce the same bits for any compiler
// contraction choice
__device__ __forceinline__ void adamw_elem(float g, float& p, float& m, float& v, float cf, float decay, float w1,
                                           float beta2, float omb2, float eps, float step_size, float bc2_sqrt) {
  const float gi = g * cf;
  const float mi = fmaf(w1, gi - m, m);
  const float vi = fmaf(omb2, gi * gi, v * beta2);
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  p = fmaf(-step_size, mi / denom, p * decay);
  m = mi;
  v = vi;
}
__global__ __launch_bounds__(256) void adamw_kernel(int64_t n, float* p, const float* g, float* m, float* v,
                                                    const float* clip, float lr, float beta1, float beta2, float eps,
                                                    float wd, float step_size, float bc2_sqrt, bf16* shadow) {
  const float cf = clip ? clip[1] : 1.f;
  const float decay = 1.f - lr * wd, w1 = 1.f - beta1, omb2 = 1.f - beta2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float pi = p[i], mi = m[i], vi = v[i];
    adamw_elem(g[i], pi, mi, vi, cf, decay, w1, beta2, omb2, eps, step_size, bc2_sqrt);
    p[i] = pi; m[i] = mi; v[i] = vi;
    if (shadow) shadow[i] = (bf16)pi;
  }
}
// The same update 4 elements per lane with 16-B loads / stores (8-B shadow stores): one pass over the
// arena is 30 B per parameter (p, g, m, v read; p, m, v, shadow written) -- HBM-bound, and the scalar
// form's 4-B accesses reached 4.7 TB/s on the B+ arena (484 us per step).  Bit-identical per element.
__global__ __launch_bounds__(256) void adamw_vec_kernel(int64_t n4, float4* p, const float4* g, float4* m, float4* v,
                                                        const float* clip, float lr, float beta1, float beta2, float eps,
                                                        float wd, float step_size, float bc2_sqrt, uint2* shadow) {
  const float cf = clip ? clip[1] : 1.f;
  const float decay = 1.f - lr * wd, w1 = 1.f - beta1, omb2 = 1.f - beta2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 g4 = g[i], p4 = p[i], m4 = m[i], v4 = v[i];
    const float ga[4] = {g4.x, g4.y, g4.z, g4.w};
    float po[4] = {p4.x, p4.y, p4.z, p4.w}, mo[4] = {m4.x, m4.y, m4.z, m4.w}, vo[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
      adamw_elem(ga[e], po[e], mo[e], vo[e], cf, decay, w1, beta2, omb2, eps, step_size, bc2_sqrt);
    p[i] = float4{po[0], po[1], po[2], po[3]};
    m[i] = float4{mo[0], mo[1], mo[2], mo[3]};
    v[i] = float4{vo[0], vo[1], vo[2], vo[3]};
    if (shadow) {
      bf16 t4[4] = {(bf16)po[0], (bf16)po[1], (bf16)po[2], (bf16)po[3]};
      shadow[i] = *(const uint2*)t4;
    }
  }
}
extern "C" int s2h_adamw(int64_t n, float* p, const float* g, float* m, float* v, const float* clip, float lr,
                         float beta1, float beta2, float eps, float wd, int step, void* bf16_shadow, hipStream_t st) {
  if (n <= 0) return 0;
  const double bc1 = 1.0 - pow((double)beta1, (double)step);
  const double bc2 = 1.0 - pow((double)beta2, (double)step);
  const float step_size = (float)(lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const bool vec = (((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) == 0 &&
                   ((uintptr_t)bf16_shadow & 7) == 0;
  const int64_t n4 = vec ? n / 4 : 0;
  if (n4 > 0) {
    int64_t b = (n4 + 255) / 256;
    if (b > 8192) b = 8192;
    hipLaunchKernelGGL(adamw_vec_kernel, dim3((unsigned)b), dim3(256), 0, st, n4, (float4*)p, (const float4*)g,
                       (float4*)m, (float4*)v, clip, lr, beta1, beta2, eps, wd, step_size, bc2_sqrt, (uint2*)bf16_shadow);
  }
  const int64_t done = 4 * n4, rest = n - done;  // the tail (or everything when unaligned)
  if (rest > 0) {
    int64_t b = (rest + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)b), dim3(256), 0, st, rest, p + done, g + done, m + done, v + done,
                       clip, lr, beta1, beta2, eps, wd, step_size, bc2_sqrt,
                       bf16_shadow ? (bf16*)bf16_shadow + done : (bf16*)nullptr);
  }
  return (int)hipGetLastError();
}
