// Bandwidth-bound helpers of the SAM2 step: residual adds, broadcast adds,
// activations, casts, dropout, 2-D axial RoPE, q-pool max-pool, window
// (un)partition, FPN nearest top-down, bilinear mask resampling, column sums,
// NHWC im2col / depthwise conv / transposed-conv scatter.  All grid-stride,
// coalesced along the contiguous (channel) dimension.
#include "common.h"
#include "reduce_det.h"

#include <algorithm>
#include <initializer_list>

#define GRID_STRIDE(i, n) for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (n); i += (int64_t)gridDim.x * blockDim.x)

static inline dim3 ew_grid(int64_t n) {
  int64_t b = (n + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return dim3((unsigned)b);
}

#define DISPATCH_T(dt, KERNEL, grid, ...)                                      \
  do {                                                                         \
    if ((dt) == S2H_BF16) hipLaunchKernelGGL(KERNEL<bf16>, grid, dim3(256), 0, st, __VA_ARGS__); \
    else hipLaunchKernelGGL(KERNEL<float>, grid, dim3(256), 0, st, __VA_ARGS__); \
  } while (0)

// 16 B of T as floats (VEC = 8 bf16 / 4 f32)
template <typename T> struct V16 {
  static constexpr int VEC = 16 / sizeof(T);
  static __device__ __forceinline__ void load(const T* p, float* v) {
    const uint4 r = *(const uint4*)p;
    const T* e = (const T*)&r;
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = to_f32(e[j]);
  }
  static __device__ __forceinline__ void store(T* p, const float* v) {
    uint4 r;
    T* e = (T*)&r;
#pragma unroll
    for (int j = 0; j < VEC; ++j) e[j] = from_f32<T>(v[j]);
    *(uint4*)p = r;
  }
};
static inline bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// 16-B vector forms of the element-wise kernels (VEC = 8 bf16 / 4 f32 per lane, 32-bit vector
// indices): the scalar forms move 2 B per load and, for the broadcast add, paid a 64-bit
// division and modulo per element (rocprofv3: add 11 us, add_bcast 9 us per launch on 3-7 MB).
template <typename T>
__global__ void add_vec_kernel(int nv, const void* a, const void* b, float alpha, float beta, void* out) {
  constexpr int VEC = V16<T>::VEC;
  GRID_STRIDE(i, nv) {
    float v[VEC], w[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = 0.f;
    if (a) {
      V16<T>::load((const T*)a + (int64_t)i * VEC, w);
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[j] = alpha * w[j];
    }
    if (b) {
      V16<T>::load((const T*)b + (int64_t)i * VEC, w);
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[j] += beta * w[j];
    }
    V16<T>::store((T*)out + (int64_t)i * VEC, v);
  }
}
// rows of `inner` elements (inner % VEC == 0): out[r] = alpha * a[r] + beta * b[r % period]
template <typename T>
__global__ void add_bcast_vec_kernel(int nv, int cpr, const void* a, float alpha, const void* b, int b_period,
                                     float beta, void* out) {
  constexpr int VEC = V16<T>::VEC;
  GRID_STRIDE(i, nv) {
    const int ii = (int)i;
    const int r = ii / cpr, c = ii - r * cpr;
    float v[VEC], w[VEC];
    V16<T>::load((const T*)b + ((int64_t)(r % b_period) * cpr + c) * VEC, v);
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] *= beta;
    if (a) {
      V16<T>::load((const T*)a + (int64_t)ii * VEC, w);
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[j] += alpha * w[j];
    }
    V16<T>::store((T*)out + (int64_t)ii * VEC, v);
  }
}
template <typename T>
__global__ void act_fwd_vec_kernel(int nv, const void* x, int act, float scale, float shift, void* y) {
  constexpr int VEC = V16<T>::VEC;
  GRID_STRIDE(i, nv) {
    float v[VEC];
    V16<T>::load((const T*)x + (int64_t)i * VEC, v);
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = apply_act(v[j], act) * scale + shift;
    V16<T>::store((T*)y + (int64_t)i * VEC, v);
  }
}
template <typename T>
__global__ void act_bwd_vec_kernel(int nv, const void* x, const void* dy, int act, void* dx, int accum) {
  constexpr int VEC = V16<T>::VEC;
  GRID_STRIDE(i, nv) {
    float g[VEC], xv[VEC];
    V16<T>::load((const T*)dy + (int64_t)i * VEC, g);
    V16<T>::load((const T*)x + (int64_t)i * VEC, xv);
#pragma unroll
    for (int j = 0; j < VEC; ++j) g[j] *= act_grad(xv[j], act);
    if (accum) {
      V16<T>::load((const T*)dx + (int64_t)i * VEC, xv);
#pragma unroll
      for (int j = 0; j < VEC; ++j) g[j] += xv[j];
    }
    V16<T>::store((T*)dx + (int64_t)i * VEC, g);
  }
}
// keep flags of VEC consecutive elements from idx: one hash per even/odd pair when idx is even
template <int VEC>
__device__ __forceinline__ void keep_vec(uint64_t seed, uint64_t idx, uint32_t thresh, bool* k) {
  if ((idx & 1) == 0) {
#pragma unroll
    for (int j = 0; j < VEC / 2; ++j) s2h_keep_pair(seed, (idx >> 1) + j, thresh, k[2 * j], k[2 * j + 1]);
  } else {
#pragma unroll
    for (int j = 0; j < VEC; ++j) k[j] = s2h_keep(seed, idx + j, thresh);
  }
}
template <typename T>
__global__ void act_dropout_bwd_vec_kernel(int nv, const void* x, const void* dy, int act, float p, uint64_t seed,
                                           const uint64_t* seed_off, uint64_t idx0, void* dx) {
  constexpr int VEC = V16<T>::VEC;
  seed = s2h_seed(seed, seed_off);
  const uint32_t thresh = (uint32_t)(p * 4294967296.0);
  const float inv = p > 0.f ? 1.f / (1.f - p) : 1.f;
  GRID_STRIDE(i, nv) {
    float g[VEC], xv[VEC];
    bool k[VEC];
    V16<T>::load((const T*)dy + (int64_t)i * VEC, g);
    if (p > 0.f) keep_vec<VEC>(seed, idx0 + (uint64_t)i * VEC, thresh, k);
    if (x) V16<T>::load((const T*)x + (int64_t)i * VEC, xv);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float v = (p > 0.f && !k[j]) ? 0.f : g[j] * inv;
      if (x) v *= act_grad(xv[j], act);
      g[j] = v;
    }
    V16<T>::store((T*)dx + (int64_t)i * VEC, g);
  }
}
template <typename T>
__global__ void dropout_vec_kernel(int nv, const void* a, const void* b, float p, uint64_t seed,
                                   const uint64_t* seed_off, uint64_t idx0, void* out) {
  constexpr int VEC = V16<T>::VEC;
  seed = s2h_seed(seed, seed_off);
  const uint32_t thresh = (uint32_t)(p * 4294967296.0);
  const float inv = 1.f / (1.f - p);
  GRID_STRIDE(i, nv) {
    float v[VEC], w[VEC];
    bool k[VEC];
    V16<T>::load((const T*)b + (int64_t)i * VEC, v);
    keep_vec<VEC>(seed, idx0 + (uint64_t)i * VEC, thresh, k);
#pragma unroll
    for (int j = 0; j < VEC; ++j) v[j] = k[j] ? v[j] * inv : 0.f;
    if (a) {
      V16<T>::load((const T*)a + (int64_t)i * VEC, w);
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[j] += w[j];
    }
    V16<T>::store((T*)out + (int64_t)i * VEC, v);
  }
}
static inline bool ew_vec_ok(int dt, int64_t n, std::initializer_list<const void*> ptrs) {
  const int vec = dt == S2H_BF16 ? 8 : 4;
  if (n % vec || n / vec >= (1ll << 31)) return false;
  for (const void* q : ptrs)
    if (q && !al16(q)) return false;
  return true;
}

// ---------------------------------------------------------------- add / axpy
// out = alpha*a + beta*b   (a or b may be null -> treated as 0)
template <typename T>
__global__ void add_kernel(int64_t n, const void* a, const void* b, float alpha, float beta, void* out) {
  GRID_STRIDE(i, n) {
    float v = 0.f;
    if (a) v += alpha * to_f32(((const T*)a)[i]);
    if (b) v += beta * to_f32(((const T*)b)[i]);
    ((T*)out)[i] = from_f32<T>(v);
  }
}
extern "C" int s2h_add(int dt, int64_t n, const void* a, const void* b, float alpha, float beta, void* out,
                       hipStream_t st) {
  if (n <= 0) return 0;
  const int vec = dt == S2H_BF16 ? 8 : 4;
  if (n % vec == 0 && n / vec < (1ll << 31) && (!a || al16(a)) && (!b || al16(b)) && al16(out)) {
    DISPATCH_T(dt, add_vec_kernel, ew_grid(n / vec), (int)(n / vec), a, b, alpha, beta, out);
  } else {
    DISPATCH_T(dt, add_kernel, ew_grid(n), n, a, b, alpha, beta, out);
  }
  return (int)hipGetLastError();
}

// out[i, j] = alpha*a[i, j] + beta*bvec[(i % b_period) * inner + j]   (b row broadcast / periodic)
template <typename T>
__global__ void add_bcast_kernel(int64_t outer, int64_t inner, const void* a, float alpha, const void* b,
                                 int64_t b_period, float beta, void* out) {
  const int64_t n = outer * inner;
  GRID_STRIDE(i, n) {
    const int64_t r = i / inner, c = i - r * inner;
    float v = beta * to_f32(((const T*)b)[(r % b_period) * inner + c]);
    if (a) v += alpha * to_f32(((const T*)a)[i]);
    ((T*)out)[i] = from_f32<T>(v);
  }
}
extern "C" int s2h_add_bcast(int dt, int64_t outer, int64_t inner, const void* a, float alpha, const void* b,
                             int64_t b_period, float beta, void* out, hipStream_t st) {
  if (outer * inner <= 0) return 0;
  const int vec = dt == S2H_BF16 ? 8 : 4;
  if (inner % vec == 0 && outer * inner / vec < (1ll << 31) && b_period < (1ll << 31) && (!a || al16(a)) && al16(b) &&
      al16(out)) {
    DISPATCH_T(dt, add_bcast_vec_kernel, ew_grid(outer * inner / vec), (int)(outer * inner / vec), (int)(inner / vec), a,
               alpha, b, (int)b_period, beta, out);
  } else {
    DISPATCH_T(dt, add_bcast_kernel, ew_grid(outer * inner), outer, inner, a, alpha, b, b_period, beta, out);
  }
  return (int)hipGetLastError();
}

// ----------------------------------------------------------- activations
// y = act(x) * scale + shift
template <typename T>
__global__ void act_fwd_kernel(int64_t n, const void* x, int act, float scale, float shift, void* y) {
  GRID_STRIDE(i, n) ((T*)y)[i] = from_f32<T>(apply_act(to_f32(((const T*)x)[i]), act) * scale + shift);
}
extern "C" int s2h_act_fwd(int dt, int64_t n, const void* x, int act, float scale, float shift, void* y,
                           hipStream_t st) {
  if (n <= 0) return 0;
  if (ew_vec_ok(dt, n, {x, y})) {
    const int vec = dt == S2H_BF16 ? 8 : 4;
    DISPATCH_T(dt, act_fwd_vec_kernel, ew_grid(n / vec), (int)(n / vec), x, act, scale, shift, y);
    return (int)hipGetLastError();
  }
  DISPATCH_T(dt, act_fwd_kernel, ew_grid(n), n, x, act, scale, shift, y);
  return (int)hipGetLastError();
}
// dx = dy * act'(x_pre) (+ dx if accum)
template <typename T>
__global__ void act_bwd_kernel(int64_t n, const void* x, const void* dy, int act, void* dx, int accum) {
  GRID_STRIDE(i, n) {
    float v = to_f32(((const T*)dy)[i]) * act_grad(to_f32(((const T*)x)[i]), act);
    if (accum) v += to_f32(((T*)dx)[i]);
    ((T*)dx)[i] = from_f32<T>(v);
  }
}
extern "C" int s2h_act_bwd(int dt, int64_t n, const void* x, const void* dy, int act, void* dx, int accum,
                           hipStream_t st) {
  if (n <= 0) return 0;
  if (ew_vec_ok(dt, n, {x, dy, dx})) {
    const int vec = dt == S2H_BF16 ? 8 : 4;
    DISPATCH_T(dt, act_bwd_vec_kernel, ew_grid(n / vec), (int)(n / vec), x, dy, act, dx, accum);
    return (int)hipGetLastError();
  }
  DISPATCH_T(dt, act_bwd_kernel, ew_grid(n), n, x, dy, act, dx, accum);
  return (int)hipGetLastError();
}

// dx = scale * [y > 0] * dy: the backward of ReLU (-> dropout) from the layer's OUTPUT y --
// y > 0 exactly where the pre-activation was positive and the element kept, so neither the
// pre-activation nor the dropout hash is needed (scale = 1 / (1 - p), or 1 without dropout).
// 8 bf16 per lane when the buffers allow 16-B accesses.
template <typename T>
__global__ void relu_mask_bwd_kernel(int64_t n, const T* y, const T* dy, float scale, T* dx) {
  constexpr int V = 16 / sizeof(T);
  const bool vec = ((uintptr_t)y % 16 == 0) && ((uintptr_t)dy % 16 == 0) && ((uintptr_t)dx % 16 == 0);
  const int64_t nv = vec ? n / V : 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nv; i += stride) {
    const uint4 yv = ((const uint4*)y)[i], gv = ((const uint4*)dy)[i];
    const T* yy = (const T*)&yv;
    const T* gg = (const T*)&gv;
    T o[V];
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = from_f32<T>(to_f32(yy[e]) > 0.f ? to_f32(gg[e]) * scale : 0.f);
    ((uint4*)dx)[i] = *(const uint4*)o;
  }
  for (int64_t i = nv * V + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    dx[i] = from_f32<T>(to_f32(y[i]) > 0.f ? to_f32(dy[i]) * scale : 0.f);
}
extern "C" int s2h_relu_mask_bwd(int dt, int64_t n, const void* y, const void* dy, float scale, void* dx,
                                 hipStream_t st) {
  if (n <= 0) return 0;
  const int64_t work = (n + 7) / 8;
  const dim3 grid((unsigned)std::min<int64_t>((work + 255) / 256, 8192));
  if (dt == S2H_BF16)
    hipLaunchKernelGGL(relu_mask_bwd_kernel<bf16>, grid, dim3(256), 0, st, n, (const bf16*)y, (const bf16*)dy, scale,
                       (bf16*)dx);
  else
    hipLaunchKernelGGL(relu_mask_bwd_kernel<float>, grid, dim3(256), 0, st, n, (const float*)y, (const float*)dy,
                       scale, (float*)dx);
  return (int)hipGetLastError();
}

// dx = act'(x_pre) * keep(i) / (1 - p) * dy: the backward of act -> dropout in one pass (the
// Linear epilogue's forward order, memory_attention.py:95-98 linear1 + ReLU + dropout).  The
// mask is the forward's counter hash of the flat output index.  x_pre may be null (no act).
template <typename T>
__global__ void act_dropout_bwd_kernel(int64_t n, const void* x, const void* dy, int act, float p, uint64_t seed,
                                       const uint64_t* seed_off, uint64_t idx0, void* dx) {
  seed = s2h_seed(seed, seed_off);
  const uint32_t thresh = (uint32_t)(p * 4294967296.0);
  const float inv = p > 0.f ? 1.f / (1.f - p) : 1.f;
  GRID_STRIDE(i, n) {
    float v = (p > 0.f && !s2h_keep(seed, idx0 + (uint64_t)i, thresh)) ? 0.f : to_f32(((const T*)dy)[i]) * inv;
    if (x) v *= act_grad(to_f32(((const T*)x)[i]), act);
    ((T*)dx)[i] = from_f32<T>(v);
  }
}
extern "C" int s2h_act_dropout_bwd(int dt, int64_t n, const void* x_pre, const void* dy, int act, float p,
                                   uint64_t seed, uint64_t idx0, void* dx, hipStream_t st) {
  if (n <= 0) return 0;
  if (ew_vec_ok(dt, n, {x_pre, dy, dx})) {
    const int vec = dt == S2H_BF16 ? 8 : 4;
    DISPATCH_T(dt, act_dropout_bwd_vec_kernel, ew_grid(n / vec), (int)(n / vec), x_pre, dy, act, p, seed,
               s2h_rng_offset_ptr(), idx0, dx);
    return (int)hipGetLastError();
  }
  DISPATCH_T(dt, act_dropout_bwd_kernel, ew_grid(n), n, x_pre, dy, act, p, seed, s2h_rng_offset_ptr(), idx0, dx);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ casts
__global__ void cast_f32_bf16_kernel(int64_t n, const float* x, bf16* y) { GRID_STRIDE(i, n) y[i] = (bf16)x[i]; }
__global__ void cast_bf16_f32_kernel(int64_t n, const bf16* x, float* y) { GRID_STRIDE(i, n) y[i] = (float)x[i]; }
__global__ void copy_f32_kernel(int64_t n, const float* x, float* y) { GRID_STRIDE(i, n) y[i] = x[i]; }
extern "C" int s2h_cast(int dt_in, int dt_out, int64_t n, const void* x, void* y, hipStream_t st) {
  if (n <= 0) return 0;
  if (dt_in == S2H_F32 && dt_out == S2H_BF16)
    hipLaunchKernelGGL(cast_f32_bf16_kernel, ew_grid(n), dim3(256), 0, st, n, (const float*)x, (bf16*)y);
  else if (dt_in == S2H_BF16 && dt_out == S2H_F32)
    hipLaunchKernelGGL(cast_bf16_f32_kernel, ew_grid(n), dim3(256), 0, st, n, (const bf16*)x, (float*)y);
  else if (dt_in == S2H_F32 && dt_out == S2H_F32)
    hipLaunchKernelGGL(copy_f32_kernel, ew_grid(n), dim3(256), 0, st, n, (const float*)x, (float*)y);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- dropout
// mode 0: out = a + keep(i)*b/(1-p)     mode 1: out = keep(i)*b/(1-p)   (also the backward)
template <typename T>
__global__ void dropout_kernel(int64_t n, const void* a, const void* b, float p, uint64_t seed, const uint64_t* seed_off,
                               uint64_t idx0, void* out) {
  seed = s2h_seed(seed, seed_off);
  const uint32_t thresh = (uint32_t)(p * 4294967296.0);
  const float inv = 1.f / (1.f - p);
  GRID_STRIDE(i, n) {
    float v = s2h_keep(seed, idx0 + (uint64_t)i, thresh) ? to_f32(((const T*)b)[i]) * inv : 0.f;
    if (a) v += to_f32(((const T*)a)[i]);
    ((T*)out)[i] = from_f32<T>(v);
  }
}
extern "C" int s2h_dropout(int dt, int64_t n, const void* a, const void* b, float p, uint64_t seed, uint64_t idx0,
                           void* out, hipStream_t st) {
  if (n <= 0) return 0;
  if (ew_vec_ok(dt, n, {a, b, out})) {
    const int vec = dt == S2H_BF16 ? 8 : 4;
    DISPATCH_T(dt, dropout_vec_kernel, ew_grid(n / vec), (int)(n / vec), a, b, p, seed, s2h_rng_offset_ptr(), idx0,
               out);
    return (int)hipGetLastError();
  }
  DISPATCH_T(dt, dropout_kernel, ew_grid(n), n, a, b, p, seed, s2h_rng_offset_ptr(), idx0, out);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------ axial RoPE
// Rotates consecutive pairs (2c, 2c+1) of the first `nrot` rows of every batch:
// row t uses table row (t % period); inverse=1 rotates by -theta (backward).
template <typename T>
__global__ void rope_kernel(int64_t nb, int nrot, int D, const void* x, int64_t sxb, int64_t sxl, void* y,
                            int64_t syb, int64_t syl, const float* cosv, const float* sinv, int period, int inverse) {
  const int half = D / 2;
  const int64_t n = nb * nrot * half;
  GRID_STRIDE(i, n) {
    const int c = i % half;
    const int64_t rt = i / half;
    const int t = rt % nrot;
    const int64_t b = rt / nrot;
    const T* xp = (const T*)x + b * sxb + (int64_t)t * sxl + 2 * c;
    T* yp = (T*)y + b * syb + (int64_t)t * syl + 2 * c;
    const int pr = t % period;
    const float co = cosv[pr * half + c];
    const float si = inverse ? -sinv[pr * half + c] : sinv[pr * half + c];
    const float xr = to_f32(xp[0]), xi = to_f32(xp[1]);
    yp[0] = from_f32<T>(xr * co - xi * si);
    yp[1] = from_f32<T>(xr * si + xi * co);
  }
}
// 16 B (VEC/2 complex pairs) per thread, 32-bit index math: the scalar form above spent
// four 64-bit divisions on every 4-byte pair.  rows = nb * nrot < 2^31.
template <typename T>
__global__ void rope_vec_kernel(int rows, int nrot, int D, const void* x, int64_t sxb, int64_t sxl, void* y,
                                int64_t syb, int64_t syl, const float* cosv, const float* sinv, int period,
                                int inverse) {
  constexpr int VEC = V16<T>::VEC, NP = VEC / 2;
  const int half = D / 2, cpr = D / VEC;  // 16-B chunks per row
  const int64_t n = (int64_t)rows * cpr;
  GRID_STRIDE(i, n) {
    const int ii = (int)i;
    const int row = ii / cpr, ch = ii - row * cpr;
    const int b = row / nrot, t = row - b * nrot;
    const int pr = t % period;
    float v[VEC], o[VEC];
    V16<T>::load((const T*)x + (int64_t)b * sxb + (int64_t)t * sxl + ch * VEC, v);
    const float* cp = cosv + pr * half + ch * NP;
    const float* sp = sinv + pr * half + ch * NP;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
      const float co = cp[j], si = inverse ? -sp[j] : sp[j];
      o[2 * j] = v[2 * j] * co - v[2 * j + 1] * si;
      o[2 * j + 1] = v[2 * j] * si + v[2 * j + 1] * co;
    }
    V16<T>::store((T*)y + (int64_t)b * syb + (int64_t)t * syl + ch * VEC, o);
  }
}

extern "C" int s2h_rope(int dt, int64_t nb, int nrot, int D, const void* x, int64_t sxb, int64_t sxl, void* y,
                        int64_t syb, int64_t syl, const float* cosv, const float* sinv, int period, int inverse,
                        hipStream_t st) {
  const int64_t n = nb * nrot * (D / 2);
  if (n <= 0) return 0;
  const int vec = dt == S2H_BF16 ? 8 : 4;
  if (D % vec == 0 && al16(x) && al16(y) && sxb % vec == 0 && sxl % vec == 0 && syb % vec == 0 &&
      syl % vec == 0 && nb * nrot * (D / vec) < (1ll << 31)) {
    const int rows = (int)(nb * nrot);
    DISPATCH_T(dt, rope_vec_kernel, ew_grid((int64_t)rows * (D / vec)), rows, nrot, D, x, sxb, sxl, y, syb, syl,
               cosv, sinv, period, inverse);
  } else {
    DISPATCH_T(dt, rope_kernel, ew_grid(n), nb, nrot, D, x, sxb, sxl, y, syb, syl, cosv, sinv, period, inverse);
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------------- 2x2 max-pool NHWC
// x viewed as [B, H, W, C] with row stride ldx (elements between consecutive (b,h,w) pixels)
template <typename T>
__global__ void maxpool2_fwd_kernel(int B, int H, int W, int C, const void* x, int64_t ldx, void* y) {
  const int Ho = H / 2, Wo = W / 2;
  const int64_t n = (int64_t)B * Ho * Wo * C;
  GRID_STRIDE(i, n) {
    const int c = i % C;
    int64_t p = i / C;
    const int xo = p % Wo; p /= Wo;
    const int yo = p % Ho;
    const int b = p / Ho;
    const T* xb = (const T*)x;
    float m = -INFINITY;
    for (int dy = 0; dy < 2; ++dy)
      for (int dx = 0; dx < 2; ++dx) {
        int64_t pix = ((int64_t)b * H + 2 * yo + dy) * W + 2 * xo + dx;
        float v = to_f32(xb[pix * ldx + c]);
        if (v > m || isnan(v)) m = v;
      }
    ((T*)y)[i] = from_f32<T>(m);
  }
}
// routes dy to the first maximal element of each window (PyTorch's scan order); writes (not accumulates) dx
template <typename T>
__global__ void maxpool2_bwd_kernel(int B, int H, int W, int C, const void* x, int64_t ldx, const void* dy,
                                    void* dx, int64_t lddx) {
  const int Ho = H / 2, Wo = W / 2;
  const int64_t n = (int64_t)B * Ho * Wo * C;
  GRID_STRIDE(i, n) {
    const int c = i % C;
    int64_t p = i / C;
    const int xo = p % Wo; p /= Wo;
    const int yo = p % Ho;
    const int b = p / Ho;
    const T* xb = (const T*)x;
    float m = -INFINITY;
    int best = 0;
    for (int k = 0; k < 4; ++k) {
      int64_t pix = ((int64_t)b * H + 2 * yo + (k >> 1)) * W + 2 * xo + (k & 1);
      float v = to_f32(xb[pix * ldx + c]);
      if (v > m || isnan(v)) { m = v; best = k; }
    }
    const float g = to_f32(((const T*)dy)[i]);
    for (int k = 0; k < 4; ++k) {
      int64_t pix = ((int64_t)b * H + 2 * yo + (k >> 1)) * W + 2 * xo + (k & 1);
      ((T*)dx)[pix * lddx + c] = from_f32<T>(k == best ? g : 0.f);
    }
  }
}
// 16-B forms (round 6): VEC channels per lane, 32-bit index math -- the scalar kernels above move 2 B
// per load and pay a 64-bit division chain per element (19.7 / 24.0 us per Hiera q-pool launch).
// The same per-channel scan (window order, NaN propagates, first maximum gets the gradient).
template <typename T>
__global__ void maxpool2_fwd_vec_kernel(int B, int H, int W, int C, const T* x, int ldx, T* y) {
  constexpr int VEC = V16<T>::VEC;
  const int Ho = H / 2, Wo = W / 2, cc = C / VEC;
  const int n = B * Ho * Wo * cc;
  GRID_STRIDE(i, n) {
    const int ii = (int)i;
    int p = ii / cc;
    const int c = (ii - p * cc) * VEC;
    const int xo = p % Wo; p /= Wo;
    const int yo = p % Ho;
    const int b = p / Ho;
    float m[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) m[j] = -INFINITY;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int pix = (b * H + 2 * yo + (k >> 1)) * W + 2 * xo + (k & 1);
      float v[VEC];
      V16<T>::load(x + (int64_t)pix * ldx + c, v);
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (v[j] > m[j] || isnan(v[j])) m[j] = v[j];
    }
    V16<T>::store(y + (int64_t)ii * VEC, m);
  }
}
template <typename T>
__global__ void maxpool2_bwd_vec_kernel(int B, int H, int W, int C, const T* x, int ldx, const T* dy, T* dx,
                                        int lddx) {
  constexpr int VEC = V16<T>::VEC;
  const int Ho = H / 2, Wo = W / 2, cc = C / VEC;
  const int n = B * Ho * Wo * cc;
  GRID_STRIDE(i, n) {
    const int ii = (int)i;
    int p = ii / cc;
    const int c = (ii - p * cc) * VEC;
    const int xo = p % Wo; p /= Wo;
    const int yo = p % Ho;
    const int b = p / Ho;
    float v[4][VEC], m[VEC], g[VEC];
    int best[VEC];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      V16<T>::load(x + (int64_t)((b * H + 2 * yo + (k >> 1)) * W + 2 * xo + (k & 1)) * ldx + c, v[k]);
    V16<T>::load(dy + (int64_t)ii * VEC, g);
#pragma unroll
    for (int j = 0; j < VEC; ++j) { m[j] = -INFINITY; best[j] = 0; }
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int j = 0; j < VEC; ++j)
        if (v[k][j] > m[j] || isnan(v[k][j])) { m[j] = v[k][j]; best[j] = k; }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float o[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) o[j] = best[j] == k ? g[j] : 0.f;
      V16<T>::store(dx + (int64_t)((b * H + 2 * yo + (k >> 1)) * W + 2 * xo + (k & 1)) * lddx + c, o);
    }
  }
}
// the 16-B forms need VEC | C, VEC | the row strides, 16-B aligned pointers and 32-bit indices
static bool maxpool_vec_ok(int dt, int B, int H, int W, int C, int64_t ld0, int64_t ld1, const void* p0,
                           const void* p1, const void* p2) {
  const int vec = dt == S2H_BF16 ? 8 : 4;
  return (dt == S2H_BF16 || dt == S2H_F32) && C % vec == 0 && ld0 % vec == 0 && ld1 % vec == 0 && al16(p0) &&
         al16(p1) && (!p2 || al16(p2)) && (int64_t)B * H * W * std::max(ld0, ld1) < (1ll << 31);
}
extern "C" int s2h_maxpool2_fwd(int dt, int B, int H, int W, int C, const void* x, int64_t ldx, void* y,
                                hipStream_t st) {
  const int64_t n = (int64_t)B * (H / 2) * (W / 2) * C;
  if (n <= 0) return 0;
  if (maxpool_vec_ok(dt, B, H, W, C, ldx, C, x, y, nullptr)) {
    const int vec = dt == S2H_BF16 ? 8 : 4;
    if (dt == S2H_BF16)
      hipLaunchKernelGGL(maxpool2_fwd_vec_kernel<bf16>, ew_grid(n / vec), dim3(256), 0, st, B, H, W, C,
                         (const bf16*)x, (int)ldx, (bf16*)y);
    else
      hipLaunchKernelGGL(maxpool2_fwd_vec_kernel<float>, ew_grid(n / vec), dim3(256), 0, st, B, H, W, C,
                         (const float*)x, (int)ldx, (float*)y);
    return (int)hipGetLastError();
  }
  DISPATCH_T(dt, maxpool2_fwd_kernel, ew_grid(n), B, H, W, C, x, ldx, y);
  return (int)hipGetLastError();
}
extern "C" int s2h_maxpool2_bwd(int dt, int B, int H, int W, int C, const void* x, int64_t ldx, const void* dy,
                                void* dx, int64_t lddx, hipStream_t st) {
  const int64_t n = (int64_t)B * (H / 2) * (W / 2) * C;
  if (n <= 0) return 0;
  if (maxpool_vec_ok(dt, B, H, W, C, ldx, lddx, x, dx, dy)) {
    const int vec = dt == S2H_BF16 ? 8 : 4;
    if (dt == S2H_BF16)
      hipLaunchKernelGGL(maxpool2_bwd_vec_kernel<bf16>, ew_grid(n / vec), dim3(256), 0, st, B, H, W, C,
                         (const bf16*)x, (int)ldx, (const bf16*)dy, (bf16*)dx, (int)lddx);
    else
      hipLaunchKernelGGL(maxpool2_bwd_vec_kernel<float>, ew_grid(n / vec), dim3(256), 0, st, B, H, W, C,
                         (const float*)x, (int)ldx, (const float*)dy, (float*)dx, (int)lddx);
    return (int)hipGetLastError();
  }
  DISPATCH_T(dt, maxpool2_bwd_kernel, ew_grid(n), B, H, W, C, x, ldx, dy, dx, lddx);
  return (int)hipGetLastError();
}

// ------------------------------------------------ window (un)partition NHWC
// partition (dir 0): win[(b*nh + wy)*nw + wx][iy][ix][c] = x[b][wy*ws+iy][wx*ws+ix][c]  (0 outside H, W)
// unpartition (dir 1): x[b][y][x][c] = win[...]   (padding dropped)
// accum: the destination is accumulated into (used for residual-stream backward)
template <typename T>
__global__ void window_kernel(int B, int H, int W, int C, int ws, const void* src, void* dst, int dir, int accum) {
  const int nh = (H + ws - 1) / ws, nw = (W + ws - 1) / ws;
  const int64_t n = dir == 0 ? (int64_t)B * nh * nw * ws * ws * C : (int64_t)B * H * W * C;
  GRID_STRIDE(i, n) {
    const int c = i % C;
    int64_t p = i / C;
    int b, yy, xx;
    int64_t widx;
    if (dir == 0) {
      const int ix = p % ws; p /= ws;
      const int iy = p % ws; p /= ws;
      const int wx = p % nw; p /= nw;
      const int wy = p % nh;
      b = p / nh;
      yy = wy * ws + iy; xx = wx * ws + ix;
      float v = 0.f;
      if (yy < H && xx < W) v = to_f32(((const T*)src)[(((int64_t)b * H + yy) * W + xx) * C + c]);
      if (accum) v += to_f32(((T*)dst)[i]);
      ((T*)dst)[i] = from_f32<T>(v);
    } else {
      xx = p % W; p /= W;
      yy = p % H;
      b = p / H;
      widx = ((((int64_t)b * nh + yy / ws) * nw + xx / ws) * ws + yy % ws) * ws + xx % ws;
      float v = to_f32(((const T*)src)[widx * C + c]);
      if (accum) v += to_f32(((T*)dst)[i]);
      ((T*)dst)[i] = from_f32<T>(v);
    }
  }
}
// 16 B of channels per thread, 32-bit pixel index math (pixels < 2^31 / chunks)
template <typename T>
__global__ void window_vec_kernel(int B, int H, int W, int C, int ws, const void* src, void* dst, int dir,
                                  int accum) {
  constexpr int VEC = V16<T>::VEC;
  const int nh = (H + ws - 1) / ws, nw = (W + ws - 1) / ws, cc = C / VEC;
  const int64_t n = (dir == 0 ? (int64_t)B * nh * nw * ws * ws : (int64_t)B * H * W) * cc;
  GRID_STRIDE(i, n) {
    const int ii = (int)i;
    int p = ii / cc;
    const int c = (ii - p * cc) * VEC;
    float v[VEC];
    if (dir == 0) {
      const int ix = p % ws; p /= ws;
      const int iy = p % ws; p /= ws;
      const int wx = p % nw; p /= nw;
      const int wy = p % nh;
      const int b = p / nh;
      const int yy = wy * ws + iy, xx = wx * ws + ix;
      if (yy < H && xx < W) {
        V16<T>::load((const T*)src + (((int64_t)b * H + yy) * W + xx) * C + c, v);
      } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) v[j] = 0.f;
      }
    } else {
      const int xx = p % W; p /= W;
      const int yy = p % H;
      const int b = p / H;
      const int64_t widx = ((((int64_t)b * nh + yy / ws) * nw + xx / ws) * ws + yy % ws) * ws + xx % ws;
      V16<T>::load((const T*)src + widx * C + c, v);
    }
    T* d = (T*)dst + (int64_t)ii * VEC;
    if (accum) {
      float a[VEC];
      V16<T>::load(d, a);
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[j] += a[j];
    }
    V16<T>::store(d, v);
  }
}

// Window partition of a per-token projection's OUTPUT (round 5): the padded positions get `padrow`
// (fp32, rounded to T) instead of zeros -- the projection of a zero-padded input row is its bias, so
// partition(linear(x)) with padrow = bias equals linear(partition(x)) bit for bit, and the
// projection runs over the real tokens only (hieradet.py:146 pads before the qkv projection).
template <typename T>
__global__ void window_pad_vec_kernel(int B, int H, int W, int C, int ws, const T* src, const float* padrow, T* dst) {
  constexpr int VEC = V16<T>::VEC;
  const int nh = (H + ws - 1) / ws, nw = (W + ws - 1) / ws, cc = C / VEC;
  const int64_t n = (int64_t)B * nh * nw * ws * ws * cc;
  GRID_STRIDE(i, n) {
    const int ii = (int)i;
    int p = ii / cc;
    const int c = (ii - p * cc) * VEC;
    const int ix = p % ws; p /= ws;
    const int iy = p % ws; p /= ws;
    const int wx = p % nw; p /= nw;
    const int wy = p % nh;
    const int b = p / nh;
    const int yy = wy * ws + iy, xx = wx * ws + ix;
    float v[VEC];
    if (yy < H && xx < W) {
      V16<T>::load(src + (((int64_t)b * H + yy) * W + xx) * C + c, v);
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) v[j] = padrow[c + j];
    }
    V16<T>::store(dst + (int64_t)ii * VEC, v);
  }
}

extern "C" int s2h_window_pad(int dt, int B, int H, int W, int C, int ws, const void* src, const float* padrow, void* dst,
                              hipStream_t st) {
  const int nh = (H + ws - 1) / ws, nw = (W + ws - 1) / ws;
  const int64_t n = (int64_t)B * nh * nw * ws * ws * C;
  if (n <= 0) return 0;
  const int vec = dt == S2H_BF16 ? 8 : 4;
  if (C % vec || !al16(src) || !al16(dst) || n / vec >= (1ll << 31) || !padrow) return (int)hipErrorInvalidValue;
  if (dt == S2H_BF16)
    hipLaunchKernelGGL(window_pad_vec_kernel<bf16>, ew_grid(n / vec), dim3(256), 0, st, B, H, W, C, ws,
                       (const bf16*)src, padrow, (bf16*)dst);
  else
    hipLaunchKernelGGL(window_pad_vec_kernel<float>, ew_grid(n / vec), dim3(256), 0, st, B, H, W, C, ws,
                       (const float*)src, padrow, (float*)dst);
  return (int)hipGetLastError();
}

// Its bias gradient: out[c] += sum over the PADDED rows of the windowed gradient (the rows whose
// input was the zero padding; their projection output was the bias).  Padded positions of one image,
// in the padded (Hp, Wp) frame: rows y >= H (all x), then rows y < H with x >= W.  Block = 32 column
// groups of 16 B x 8 row lanes over one chunk of padded rows; the 8 lanes' sums are added in fixed
// order through LDS, the chunk's partial row goes to the workspace and det_colsum finishes (or float
// atomics without the deterministic workspace).
template <typename T>
__global__ __launch_bounds__(256) void window_pad_colsum_kernel(int B, int H, int W, int C, int ws, const T* win,
                                                                int rows_per_chunk, float* out, float* part) {
  constexpr int VEC = V16<T>::VEC;
  const int cg = threadIdx.x & 31, lane = threadIdx.x >> 5;
  const int c = (blockIdx.x * 32 + cg) * VEC;
  const int nh = (H + ws - 1) / ws, nw = (W + ws - 1) / ws, Hp = nh * ws, Wp = nw * ws;
  const int P = Hp * Wp - H * W, rows = B * P, top = (Hp - H) * Wp;
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(rows, r0 + rows_per_chunk);
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  if (c < C) {
    for (int r = r0 + lane; r < r1; r += 8) {
      const int b = r / P;
      int q = r - b * P, y, x;
      if (q < top) { y = H + q / Wp; x = q - (q / Wp) * Wp; }
      else { q -= top; y = q / (Wp - W); x = W + q - y * (Wp - W); }
      const int64_t wrow = (((int64_t)(b * nh + y / ws) * nw + x / ws) * ws + y % ws) * ws + x % ws;
      float v[VEC];
      V16<T>::load(win + wrow * C + c, v);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += v[j];
    }
  }
  __shared__ float red[8][32 * 8 + 4];
#pragma unroll
  for (int j = 0; j < VEC; ++j) red[lane][cg * VEC + j] = acc[j];
  __syncthreads();
  // 256 threads finish the block's 32 * VEC columns: thread t -> column t (VEC 8: 256 columns)
  const int cl = threadIdx.x;
  if (cl < 32 * VEC) {
    const int cc = blockIdx.x * 32 * VEC + cl;
    if (cc < C) {
      float s2 = 0.f;
#pragma unroll
      for (int l = 0; l < 8; ++l) s2 += red[l][cl];
      if (part) part[(int64_t)blockIdx.y * C + cc] = s2;
      else atomicAdd(&out[cc], s2);
    }
  }
}

extern "C" int s2h_window_pad_colsum(int dt, int B, int H, int W, int C, int ws, const void* win, float* out,
                                     hipStream_t st) {
  const int nh = (H + ws - 1) / ws, nw = (W + ws - 1) / ws;
  const int64_t rows = (int64_t)B * ((int64_t)nh * ws * nw * ws - (int64_t)H * W);
  const int vec = dt == S2H_BF16 ? 8 : 4;
  if (C % vec || !al16(win) || rows >= (1ll << 31)) return (int)hipErrorInvalidValue;
  if (rows <= 0 || C <= 0) return 0;
  // chunks of >= 32 rows, <= 256 of them (the fixed-order finalize's partial rows)
  int rpc = 32;
  int nchunk = (int)((rows + rpc - 1) / rpc);
  if (nchunk > 256) {
    rpc = (int)((rows + 255) / 256);
    nchunk = (int)((rows + rpc - 1) / rpc);
  }
  float* deferred = s2h_defer_sink(nchunk, C, out, 0, nullptr, st);
  float* part = deferred ? deferred : s2h_det_ws(nchunk * C * (int64_t)sizeof(float));
  const dim3 grid((unsigned)((C / vec + 31) / 32), (unsigned)nchunk);
  if (dt == S2H_BF16)
    hipLaunchKernelGGL(window_pad_colsum_kernel<bf16>, grid, dim3(256), 0, st, B, H, W, C, ws, (const bf16*)win, rpc,
                       out, part);
  else
    hipLaunchKernelGGL(window_pad_colsum_kernel<float>, grid, dim3(256), 0, st, B, H, W, C, ws, (const float*)win, rpc,
                       out, part);
  if (part && !deferred) det_colsum(1, nchunk, C, part, out, 1, st);
  return (int)hipGetLastError();
}

extern "C" int s2h_window(int dt, int B, int H, int W, int C, int ws, const void* src, void* dst, int dir, int accum,
                          hipStream_t st) {
  const int nh = (H + ws - 1) / ws, nw = (W + ws - 1) / ws;
  const int64_t n = dir == 0 ? (int64_t)B * nh * nw * ws * ws * C : (int64_t)B * H * W * C;
  if (n <= 0) return 0;
  const int vec = dt == S2H_BF16 ? 8 : 4;
  if (C % vec == 0 && al16(src) && al16(dst) && n / vec < (1ll << 31)) {
    DISPATCH_T(dt, window_vec_kernel, ew_grid(n / vec), B, H, W, C, ws, src, dst, dir, accum);
  } else {
    DISPATCH_T(dt, window_kernel, ew_grid(n), B, H, W, C, ws, src, dst, dir, accum);
  }
  return (int)hipGetLastError();
}

// ----------------------------------------------- FPN nearest x2 top-down
// out[b,y,x,c] = lat[b,y,x,c] + prev[b,y/2,x/2,c]
template <typename T>
__global__ void up2_add_kernel(int B, int H, int W, int C, const void* lat, const void* prev, void* out) {
  const int64_t n = (int64_t)B * H * W * C;
  GRID_STRIDE(i, n) {
    const int c = i % C;
    int64_t p = i / C;
    const int xx = p % W; p /= W;
    const int yy = p % H;
    const int b = p / H;
    float v = to_f32(((const T*)lat)[i]);
    v += to_f32(((const T*)prev)[(((int64_t)b * (H / 2) + yy / 2) * (W / 2) + xx / 2) * C + c]);
    ((T*)out)[i] = from_f32<T>(v);
  }
}
// dprev[b,y,x,c] = sum_{2x2} dout[b,2y+dy,2x+dx,c]   (+= if accum)
template <typename T>
__global__ void pool2_sum_kernel(int B, int Ho, int Wo, int C, const void* dout, void* dprev, int accum) {
  const int64_t n = (int64_t)B * Ho * Wo * C;
  GRID_STRIDE(i, n) {
    const int c = i % C;
    int64_t p = i / C;
    const int xx = p % Wo; p /= Wo;
    const int yy = p % Ho;
    const int b = p / Ho;
    float v = 0.f;
    for (int k = 0; k < 4; ++k)
      v += to_f32(((const T*)dout)[(((int64_t)b * 2 * Ho + 2 * yy + (k >> 1)) * 2 * Wo + 2 * xx + (k & 1)) * C + c]);
    if (accum) v += to_f32(((T*)dprev)[i]);
    ((T*)dprev)[i] = from_f32<T>(v);
  }
}
extern "C" int s2h_up2_add(int dt, int B, int H, int W, int C, const void* lat, const void* prev, void* out,
                           hipStream_t st) {
  const int64_t n = (int64_t)B * H * W * C;
  if (n <= 0) return 0;
  DISPATCH_T(dt, up2_add_kernel, ew_grid(n), B, H, W, C, lat, prev, out);
  return (int)hipGetLastError();
}
extern "C" int s2h_pool2_sum(int dt, int B, int Ho, int Wo, int C, const void* dout, void* dprev, int accum,
                             hipStream_t st) {
  const int64_t n = (int64_t)B * Ho * Wo * C;
  if (n <= 0) return 0;
  DISPATCH_T(dt, pool2_sum_kernel, ew_grid(n), B, Ho, Wo, C, dout, dprev, accum);
  return (int)hipGetLastError();
}

// --------------------------------------- bilinear resample (align_corners=False)
// planes [N, hi, wi] f32 -> [N, ho, wo] f32, PyTorch upsample_bilinear2d index rule.
__device__ __forceinline__ void bil_src(int o, float scale, int in, int& i0, int& i1, float& l1) {
  float s = scale * (o + 0.5f) - 0.5f;
  if (s < 0.f) s = 0.f;
  i0 = (int)s;
  if (i0 > in - 1) i0 = in - 1;
  i1 = i0 + (i0 < in - 1 ? 1 : 0);
  l1 = s - (float)i0;
}
__global__ void bilinear_fwd_kernel(int N, int hi, int wi, int ho, int wo, const float* x, float* y) {
  const float sh = (float)hi / ho, sw = (float)wi / wo;
  const int64_t n = (int64_t)N * ho * wo;
  GRID_STRIDE(i, n) {
    const int ox = i % wo;
    const int64_t r = i / wo;
    const int oy = r % ho;
    const int p = r / ho;
    int y0, y1, x0, x1;
    float ly, lx;
    bil_src(oy, sh, hi, y0, y1, ly);
    bil_src(ox, sw, wi, x0, x1, lx);
    const float* xp = x + (int64_t)p * hi * wi;
    const float v = (1.f - ly) * ((1.f - lx) * xp[y0 * wi + x0] + lx * xp[y0 * wi + x1]) +
                    ly * ((1.f - lx) * xp[y1 * wi + x0] + lx * xp[y1 * wi + x1]);
    y[i] = v;
  }
}
// gather form of the backward (deterministic): dx[p,iy,ix] = sum over outputs whose taps hit (iy,ix)
__global__ void bilinear_bwd_kernel(int N, int hi, int wi, int ho, int wo, const float* dy, float* dx) {
  const float sh = (float)hi / ho, sw = (float)wi / wo;
  const int64_t n = (int64_t)N * hi * wi;
  const int ry = (int)ceilf(1.f / sh) + 2, rx = (int)ceilf(1.f / sw) + 2;
  GRID_STRIDE(i, n) {
    const int ix = i % wi;
    const int64_t r = i / wi;
    const int iy = r % hi;
    const int p = r / hi;
    // the outputs whose taps can reach (iy, ix): source coordinate s = scale (o + 0.5) - 0.5 within
    // (i - 1, i + 1), widened by one output on each side (the weight tests below are exact, so the
    // contributing outputs and their order are those of the wider cy +- (ry + 1) search: 10 x 10
    // candidates instead of 15 x 15 at a 4x upsampling)
    const int oy0 = max(0, (int)floorf((iy - 0.5f) / sh - 0.5f) - 1);
    const int oy1 = min(ho - 1, (int)ceilf((iy + 1.5f) / sh - 0.5f) + 1);
    const int ox0 = max(0, (int)floorf((ix - 0.5f) / sw - 0.5f) - 1);
    const int ox1 = min(wo - 1, (int)ceilf((ix + 1.5f) / sw - 0.5f) + 1);
    (void)ry;
    (void)rx;
    float acc = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy) {
      int y0, y1; float ly;
      bil_src(oy, sh, hi, y0, y1, ly);
      float wy = (y0 == iy ? 1.f - ly : 0.f) + (y1 == iy ? ly : 0.f);
      if (wy == 0.f) continue;
      for (int ox = ox0; ox <= ox1; ++ox) {
        int x0, x1; float lx;
        bil_src(ox, sw, wi, x0, x1, lx);
        float wx = (x0 == ix ? 1.f - lx : 0.f) + (x1 == ix ? lx : 0.f);
        if (wx == 0.f) continue;
        acc += wy * wx * dy[((int64_t)p * ho + oy) * wo + ox];
      }
    }
    dx[i] = acc;
  }
}
extern "C" int s2h_bilinear_fwd(int N, int hi, int wi, int ho, int wo, const float* x, float* y, hipStream_t st) {
  const int64_t n = (int64_t)N * ho * wo;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(bilinear_fwd_kernel, ew_grid(n), dim3(256), 0, st, N, hi, wi, ho, wo, x, y);
  return (int)hipGetLastError();
}
// The same gather with the column taps' weights computed once per input pixel (MAXC candidate output
// columns in registers) instead of once per (candidate row, candidate column): the same candidates, the
// same skipped zeros, the same (wy * wx) * dy products added in the same order -- bit-identical.  The
// per-candidate index arithmetic made the kernel VALU-bound (126 us for the 104-plane 256^2 -> 512^2
// mask upsampling backward).
// F: exact integer upsampling (ho = F hi, wo = F wi; 0 otherwise): the taps of input i come from outputs
// F i - F / 2 .. F i + 3 F / 2 - 1 only (the wider search's other candidates all have zero weight), so
// 2F x 2F candidates (2x: 4 x 4 instead of 8 x 8, 4x: 8 x 8 instead of 12 x 16) -- the same nonzero terms
// in the same order
template <int MAXC, int F = 0>
__global__ __launch_bounds__(256) void bilinear_bwd_hoist_kernel(int N, int hi, int wi, int ho, int wo, const float* dy,
                                                                 float* dx) {
  const float sh = (float)hi / ho, sw = (float)wi / wo;
  const int64_t n = (int64_t)N * hi * wi;
  GRID_STRIDE(i, n) {
    const int ix = i % wi;
    const int64_t r = i / wi;
    const int iy = r % hi;
    const int p = r / hi;
    const int oy0 = F ? max(0, F * iy - F / 2) : max(0, (int)floorf((iy - 0.5f) / sh - 0.5f) - 1);
    const int oy1 = F ? min(ho - 1, F * iy + 3 * F / 2 - 1) : min(ho - 1, (int)ceilf((iy + 1.5f) / sh - 0.5f) + 1);
    const int ox0 = F ? max(0, F * ix - F / 2) : max(0, (int)floorf((ix - 0.5f) / sw - 0.5f) - 1);
    const int ox1 = F ? min(wo - 1, F * ix + 3 * F / 2 - 1) : min(wo - 1, (int)ceilf((ix + 1.5f) / sw - 0.5f) + 1);
    float wxs[MAXC];
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      int x0, x1; float lx;
      bil_src(ox0 + c, sw, wi, x0, x1, lx);
      wxs[c] = ox0 + c <= ox1 ? (x0 == ix ? 1.f - lx : 0.f) + (x1 == ix ? lx : 0.f) : 0.f;
    }
    float acc = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy) {
      int y0, y1; float ly;
      bil_src(oy, sh, hi, y0, y1, ly);
      const float wy = (y0 == iy ? 1.f - ly : 0.f) + (y1 == iy ? ly : 0.f);
      if (wy == 0.f) continue;
      const float* row = dy + ((int64_t)p * ho + oy) * wo + ox0;
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
        if (wxs[c] != 0.f) acc += wy * wxs[c] * row[c];
    }
    dx[i] = acc;
  }
}
extern "C" int s2h_bilinear_bwd(int N, int hi, int wi, int ho, int wo, const float* dy, float* dx, hipStream_t st) {
  const int64_t n = (int64_t)N * hi * wi;
  if (n <= 0) return 0;
  // candidate output columns per input column: ox1 - ox0 + 1 <= ceil(2 wo / wi) + 4 (2x: 8)
  const int maxc = (int)ceilf(2.f * wo / wi) + 4;
  if (ho == 2 * hi && wo == 2 * wi)
    hipLaunchKernelGGL((bilinear_bwd_hoist_kernel<4, 2>), ew_grid(n), dim3(256), 0, st, N, hi, wi, ho, wo, dy, dx);
  else if (ho == 4 * hi && wo == 4 * wi)
    hipLaunchKernelGGL((bilinear_bwd_hoist_kernel<8, 4>), ew_grid(n), dim3(256), 0, st, N, hi, wi, ho, wo, dy, dx);
  else if (maxc <= 8) hipLaunchKernelGGL((bilinear_bwd_hoist_kernel<8>), ew_grid(n), dim3(256), 0, st, N, hi, wi, ho, wo, dy, dx);
  else if (maxc <= 16) hipLaunchKernelGGL((bilinear_bwd_hoist_kernel<16>), ew_grid(n), dim3(256), 0, st, N, hi, wi, ho, wo, dy, dx);
  else hipLaunchKernelGGL(bilinear_bwd_kernel, ew_grid(n), dim3(256), 0, st, N, hi, wi, ho, wo, dy, dx);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------ column sums
// out[c] (+)= sum_r x[r*ld + c]  -> f32 (bias gradients, reductions over objects)
// part != nullptr: the block's sums go to part[block row][c] for colsum_finalize_kernel (fixed order,
// deterministic); otherwise float atomics into out
template <typename T>
__global__ void colsum_kernel(int64_t rows, int cols, const void* x, int64_t ld, float* out, float* part) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  const int64_t chunk = (rows + gridDim.y - 1) / gridDim.y;
  const int64_t r0 = blockIdx.y * chunk, r1 = min(rows, r0 + chunk);
  float acc = 0.f;
  for (int64_t r = r0; r < r1; ++r) acc += to_f32(((const T*)x)[r * ld + c]);
  if (part) part[(int64_t)blockIdx.y * cols + c] = acc;
  else atomicAdd(&out[c], acc);
}
template <typename T>
__global__ __launch_bounds__(256) void colsum_vec_kernel(int64_t rows, int cols, const T* x, int64_t ld,
                                                         int64_t rows_per_block, float* out, float* part) {
  constexpr int V = 16 / sizeof(T);
  const int G = cols / V;
  const int lanes = 256 / G;  // row lanes per pass
  const int g = threadIdx.x % G, lane = threadIdx.x / G;
  __shared__ float red[256 * 8];
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
  const int64_t r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  if (lane < lanes) {
    for (int64_t r = r0 + lane; r < r1; r += lanes) {
      const uint4 u = *(const uint4*)(x + r * ld + g * V);
      const T* t = (const T*)&u;
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] += to_f32(t[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) red[threadIdx.x * V + j] = (lane < lanes) ? acc[j] : 0.f;
  __syncthreads();
  for (int c = threadIdx.x; c < cols; c += 256) {
    const int gg = c / V, j = c % V;
    float s = 0.f;
    for (int l = 0; l < lanes; ++l) s += red[(l * G + gg) * V + j];
    if (part) part[(int64_t)blockIdx.x * cols + c] = s;
    else atomicAdd(&out[c], s);
  }
}

extern "C" int s2h_colsum(int dt, int64_t rows, int cols, const void* x, int64_t ld, float* out, int accum,
                          hipStream_t st) {
  if (cols <= 0) return 0;
  if (!accum) s2h_zero_f32(out, 1, cols, cols, st);
  if (rows <= 0) return (int)hipGetLastError();
  const int V = dt == S2H_BF16 ? 8 : 4;
  if (cols % V == 0 && cols / V <= 256 && ld % V == 0 && ((uintptr_t)x & 15) == 0) {
    // ~1024 blocks, each >= 16 rows
    int64_t rpb = (rows + 1023) / 1024;
    if (rpb < 16) rpb = 16;
    int64_t nb = (rows + rpb - 1) / rpb;
    // deterministic: <= 256 partial rows for the second pass (deferred into the arena inside a
    // s2h_grad_defer scope, grad_defer.hip)
    const int64_t rpb_d = nb > 256 ? (rows + 255) / 256 : rpb;
    const int64_t nb_d = (rows + rpb_d - 1) / rpb_d;
    float* deferred = s2h_defer_sink((int)nb_d, cols, out, 0, nullptr, st);
    float* part = deferred ? deferred : s2h_det_ws(nb * cols * (int64_t)sizeof(float));
    if (part) {
      rpb = rpb_d;
      nb = nb_d;
    }
    if (dt == S2H_BF16)
      hipLaunchKernelGGL(colsum_vec_kernel<bf16>, dim3((unsigned)nb), dim3(256), 0, st, rows, cols,
                         (const bf16*)x, ld, rpb, out, part);
    else
      hipLaunchKernelGGL(colsum_vec_kernel<float>, dim3((unsigned)nb), dim3(256), 0, st, rows, cols,
                         (const float*)x, ld, rpb, out, part);
    if (part && !deferred) det_colsum(1, (int)nb, cols, part, out, 1, st);
    return (int)hipGetLastError();
  }
  const int cb = (cols + 255) / 256;
  int64_t ry = (rows + 255) / 256;
  int64_t want = 2048 / cb;
  if (want < 1) want = 1;
  if (ry > want) ry = want;
  dim3 grid(cb, (unsigned)ry);
  float* deferred = s2h_defer_sink((int)ry, cols, out, 0, nullptr, st);
  float* part = deferred ? deferred : s2h_det_ws(ry * cols * (int64_t)sizeof(float));
  if (dt == S2H_BF16) hipLaunchKernelGGL(colsum_kernel<bf16>, grid, dim3(256), 0, st, rows, cols, x, ld, out, part);
  else hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, st, rows, cols, x, ld, out, part);
  if (part && !deferred) det_colsum(1, (int)ry, cols, part, out, 1, st);
  return (int)hipGetLastError();
}
// out[j] = sum_{o<O} x[o*inner + j]   written in T (broadcast-input gradients)
template <typename T>
__global__ void sum_outer_kernel(int O, int64_t inner, const void* x, void* out, int accum) {
  GRID_STRIDE(j, inner) {
    float v = 0.f;
    for (int o = 0; o < O; ++o) v += to_f32(((const T*)x)[(int64_t)o * inner + j]);
    if (accum) v += to_f32(((T*)out)[j]);
    ((T*)out)[j] = from_f32<T>(v);
  }
}
extern "C" int s2h_sum_outer(int dt, int O, int64_t inner, const void* x, void* out, int accum, hipStream_t st) {
  if (inner <= 0) return 0;
  DISPATCH_T(dt, sum_outer_kernel, ew_grid(inner), O, inner, x, out, accum);
  return (int)hipGetLastError();
}
// out[f][j] = sum_{o<O} x[f][o][j] for F frames in one launch (the frame-batched backward of a broadcast
// over objects), 16 B per thread; each element's sum in o order, as sum_outer_kernel adds it
template <typename T>
__global__ __launch_bounds__(256) void sum_outer_vec_kernel(int F, int O, int64_t inner, const T* x, T* out, int accum) {
  constexpr int V = 16 / sizeof(T);
  const int64_t nv = inner / V;
  GRID_STRIDE(i, (int64_t)F * nv) {
    const int64_t f = i / nv, jv = i - f * nv;
    const T* xp = x + f * O * inner + jv * V;
    float acc[V];
#pragma unroll
    for (int j = 0; j < V; ++j) acc[j] = 0.f;
    for (int o = 0; o < O; ++o) {
      T t[V];
      *(uint4*)t = *(const uint4*)(xp + (int64_t)o * inner);
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] += to_f32(t[j]);
    }
    T* op = out + f * inner + jv * V;
    T r[V];
    if (accum) {
      T prev[V];
      *(uint4*)prev = *(const uint4*)op;
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] += to_f32(prev[j]);
    }
#pragma unroll
    for (int j = 0; j < V; ++j) r[j] = from_f32<T>(acc[j]);
    *(uint4*)op = *(const uint4*)r;
  }
}
extern "C" int s2h_sum_outer_batched(int dt, int F, int O, int64_t inner, const void* x, void* out, int accum,
                                     hipStream_t st) {
  if (inner <= 0 || F <= 0) return 0;
  const int V = dt == S2H_BF16 ? 8 : 4;
  if (inner % V == 0 && al16(x) && al16(out)) {
    const int64_t n = (int64_t)F * (inner / V);
    if (dt == S2H_BF16)
      hipLaunchKernelGGL(sum_outer_vec_kernel<bf16>, ew_grid(n), dim3(256), 0, st, F, O, inner, (const bf16*)x,
                         (bf16*)out, accum);
    else
      hipLaunchKernelGGL(sum_outer_vec_kernel<float>, ew_grid(n), dim3(256), 0, st, F, O, inner, (const float*)x,
                         (float*)out, accum);
    return (int)hipGetLastError();
  }
  for (int f = 0; f < F; ++f) {
    const int64_t esz = dt == S2H_BF16 ? 2 : 4;
    DISPATCH_T(dt, sum_outer_kernel, ew_grid(inner), O, inner, (const char*)x + f * O * inner * esz,
               (char*)out + f * inner * esz, accum);
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------------------ NHWC im2col
// col[(b*Ho+oy)*Wo+ox][c*kh*kw + ky*kw + kx] = x[b][oy*s-p+ky][ox*s-p+kx][c]  (PyTorch weight order);
// rows of ldc >= C*kh*kw elements, the columns past C*kh*kw zero (a row pitch that is a multiple of 8
// keeps the patch embedding's 147-column weight gradient on the LDS-DMA GEMM)
template <typename T>
__global__ void im2col_kernel(int B, int H, int W, int C, int kh, int kw, int stride, int pad, int Ho, int Wo,
                              int ldc, const void* x, void* col) {
  const int Kc = C * kh * kw;
  const int64_t n = (int64_t)B * Ho * Wo * ldc;
  GRID_STRIDE(i, n) {
    const int k = i % ldc;
    const int64_t p = i / ldc;
    float v = 0.f;
    if (k < Kc) {
      const int ox = p % Wo;
      const int oy = (p / Wo) % Ho;
      const int b = p / ((int64_t)Wo * Ho);
      const int c = k / (kh * kw), r = k % (kh * kw), ky = r / kw, kx = r % kw;
      const int yy = oy * stride - pad + ky, xx = ox * stride - pad + kx;
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) v = to_f32(((const T*)x)[(((int64_t)b * H + yy) * W + xx) * C + c]);
    }
    ((T*)col)[i] = from_f32<T>(v);
  }
}
// bf16, ldcol % 8 == 0: 8 consecutive columns per lane (one 16-B store) with the (c, ky, kx) and pixel
// decomposition done once per lane and stepped incrementally -- the per-element integer divisions made
// the scalar form VALU-bound (36.6 us per launch for the 131072 x 152 patch-embedding matrix).  Same
// values in the same places.
__global__ __launch_bounds__(256) void im2col_vec8_kernel(int B, int H, int W, int C, int kh, int kw, int stride,
                                                          int pad, int Ho, int Wo, int ldc, const bf16* x, bf16* col) {
  const int Kc = C * kh * kw;
  const int ng = ldc / 8;
  const int64_t n = (int64_t)B * Ho * Wo * ng;
  GRID_STRIDE(i, n) {
    const int gk = (int)(i % ng);
    const int64_t p = i / ng;
    const int ox = (int)(p % Wo);
    const int oy = (int)((p / Wo) % Ho);
    const int b = (int)(p / ((int64_t)Wo * Ho));
    int k = gk * 8;
    int c = k / (kh * kw), r = k - c * (kh * kw), ky = r / kw, kx = r - ky * kw;
    const int y0 = oy * stride - pad, x0 = ox * stride - pad;
    const bf16* xb = x + (int64_t)b * H * W * C;
    bf16 t[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      bf16 v = (bf16)0.f;
      const int yy = y0 + ky, xx = x0 + kx;
      if (k + e < Kc && yy >= 0 && yy < H && xx >= 0 && xx < W) v = xb[((int64_t)yy * W + xx) * C + c];
      t[e] = v;
      if (++kx == kw) {
        kx = 0;
        if (++ky == kh) { ky = 0; ++c; }
      }
    }
    *(uint4*)(col + p * ldc + gk * 8) = *(const uint4*)t;
  }
}
extern "C" int s2h_im2col(int dt, int B, int H, int W, int C, int kh, int kw, int stride, int pad, int Ho, int Wo,
                          int64_t ldcol, const void* x, void* col, hipStream_t st) {
  if (ldcol < (int64_t)C * kh * kw) return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)B * Ho * Wo * ldcol;
  if (n <= 0) return 0;
  if (dt == S2H_BF16 && ldcol % 8 == 0 && ((uintptr_t)col & 15) == 0) {
    hipLaunchKernelGGL(im2col_vec8_kernel, ew_grid(n / 8), dim3(256), 0, st, B, H, W, C, kh, kw, stride, pad, Ho, Wo,
                       (int)ldcol, (const bf16*)x, (bf16*)col);
    return (int)hipGetLastError();
  }
  DISPATCH_T(dt, im2col_kernel, ew_grid(n), B, H, W, C, kh, kw, stride, pad, Ho, Wo, (int)ldcol, x, col);
  return (int)hipGetLastError();
}

// ------------------------------------------------- depthwise KxK conv NHWC
template <typename T>
__global__ void dwconv_kernel(int B, int H, int W, int C, int K, int pad, const void* x, const float* w,
                              const float* bias, void* y) {
  const int64_t n = (int64_t)B * H * W * C;
  GRID_STRIDE(i, n) {
    const int c = i % C;
    int64_t p = i / C;
    const int xx = p % W; p /= W;
    const int yy = p % H;
    const int b = p / H;
    float acc = bias ? bias[c] : 0.f;
    for (int ky = 0; ky < K; ++ky) {
      const int sy = yy - pad + ky;
      if (sy < 0 || sy >= H) continue;
      for (int kx = 0; kx < K; ++kx) {
        const int sx = xx - pad + kx;
        if (sx < 0 || sx >= W) continue;
        acc += w[(c * K + ky) * K + kx] * to_f32(((const T*)x)[(((int64_t)b * H + sy) * W + sx) * C + c]);
      }
    }
    ((T*)y)[i] = from_f32<T>(acc);
  }
}
// Channel-vectorised form: a block owns a 64-channel slice of 32 consecutive pixels of one
// row; the slice's K*K taps are staged in LDS as [tap][64] so every lane reads its 8
// channels' weights with two 16-B LDS loads, and the 8 channels of x with one 16-B load.
template <typename T>
__global__ __launch_bounds__(256) void dwconv_vec_kernel(int B, int H, int W, int C, int K, int pad, const T* x,
                                                         const float* w, const float* bias, T* y) {
  __shared__ __attribute__((aligned(16))) float wl[49 * 64];
  const int cg = threadIdx.x & 7, px = threadIdx.x >> 3;  // 8 channel groups x 32 pixels
  const int c0 = blockIdx.z * 64;
  const int row = blockIdx.y;  // b*H + yy
  const int yy = row % H, b = row / H;
  const int xx = blockIdx.x * 32 + px;
  for (int i = threadIdx.x; i < K * K * 64; i += 256) {
    const int t = i / 64, c = i % 64;
    wl[t * 64 + c] = w[(int64_t)(c0 + c) * K * K + t];
  }
  __syncthreads();
  if (xx >= W) return;
  const int cc = c0 + cg * 8;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = bias ? bias[cc + j] : 0.f;
  for (int ky = 0; ky < K; ++ky) {
    const int sy = yy - pad + ky;
    if (sy < 0 || sy >= H) continue;
    const T* xr = x + (((int64_t)b * H + sy) * W) * C + cc;
    for (int kx = 0; kx < K; ++kx) {
      const int sx = xx - pad + kx;
      if (sx < 0 || sx >= W) continue;
      T v[8];
      if (sizeof(T) == 2) {
        *(uint4*)v = *(const uint4*)(xr + (int64_t)sx * C);
      } else {
        *(uint4*)v = *(const uint4*)(xr + (int64_t)sx * C);
        *(uint4*)(v + 4) = *(const uint4*)(xr + (int64_t)sx * C + 4);
      }
      const float4 w0 = *(const float4*)&wl[(ky * K + kx) * 64 + cg * 8];
      const float4 w1 = *(const float4*)&wl[(ky * K + kx) * 64 + cg * 8 + 4];
      acc[0] += w0.x * to_f32(v[0]); acc[1] += w0.y * to_f32(v[1]);
      acc[2] += w0.z * to_f32(v[2]); acc[3] += w0.w * to_f32(v[3]);
      acc[4] += w1.x * to_f32(v[4]); acc[5] += w1.y * to_f32(v[5]);
      acc[6] += w1.z * to_f32(v[6]); acc[7] += w1.w * to_f32(v[7]);
    }
  }
  T o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = from_f32<T>(acc[j]);
  T* yp = y + (((int64_t)b * H + yy) * W + xx) * C + cc;
  if (sizeof(T) == 2) {
    *(uint4*)yp = *(const uint4*)o;
  } else {
    *(uint4*)yp = *(const uint4*)o;
    *(uint4*)(yp + 4) = *(const uint4*)(o + 4);
  }
}

// Row-blocked bf16 form for K = 7 (the memory fuser's CXBlock depthwise 7x7): a thread computes R
// vertically adjacent outputs of 8 channels; per kernel column kx it loads the R + K - 1 input rows
// once (16 B each) and applies that column's K taps to all R outputs from registers -- 17.5 input
// loads per output at R = 4 instead of 49 (the one-output form above is load-issue bound).
// Out-of-image taps read zeros (the one-output form skips them: same sum, other order).
template <int K, int R>
__global__ __launch_bounds__(256) void dwconv_rows_kernel(int B, int H, int W, int C, int pad, const bf16* x,
                                                          const float* w, const float* bias, bf16* y) {
  __shared__ __attribute__((aligned(16))) float wl[K * K * 64];
  const int cg = threadIdx.x & 7, px = threadIdx.x >> 3;  // 8 channel groups x 32 pixels
  const int c0 = blockIdx.z * 64;
  const int HB = (H + R - 1) / R;
  const int y0 = (blockIdx.y % HB) * R, b = blockIdx.y / HB;
  const int xx = blockIdx.x * 32 + px;
  for (int i = threadIdx.x; i < K * K * 64; i += 256) {
    const int t = i / 64, c = i % 64;
    wl[t * 64 + c] = w[(int64_t)(c0 + c) * K * K + t];
  }
  __syncthreads();
  if (xx >= W) return;
  const int cc = c0 + cg * 8;
  float acc[R][8];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[r][j] = bias ? bias[cc + j] : 0.f;
  const bf16* xb = x + (int64_t)b * H * W * C + cc;
#pragma unroll 1
  for (int kx = 0; kx < K; ++kx) {  // rolled: unrolled, all K*K weight taps get hoisted into VGPRs
    const int sx = xx - pad + kx;
    const bool xok = sx >= 0 && sx < W;
    uint4 in[R + K - 1];
#pragma unroll
    for (int i = 0; i < R + K - 1; ++i) {
      const int sy = y0 - pad + i;
      in[i] = (xok && sy >= 0 && sy < H) ? *(const uint4*)(xb + ((int64_t)sy * W + sx) * C) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int ky = 0; ky < K; ++ky) {
      const float4 w0 = *(const float4*)&wl[(ky * K + kx) * 64 + cg * 8];
      const float4 w1 = *(const float4*)&wl[(ky * K + kx) * 64 + cg * 8 + 4];
      const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const bf16* v = (const bf16*)&in[r + ky];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[r][j] += wv[j] * (float)v[j];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (y0 + r >= H) break;
    bf16 o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)acc[r][j];
    *(uint4*)(y + (((int64_t)b * H + y0 + r) * W + xx) * C + cc) = *(const uint4*)o;
  }
}

extern "C" int s2h_dwconv(int dt, int B, int H, int W, int C, int K, int pad, const void* x, const float* w,
                          const float* bias, void* y, hipStream_t st) {
  const int64_t n = (int64_t)B * H * W * C;
  if (n <= 0) return 0;
  if (dt == S2H_BF16 && K == 7 && C % 64 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    constexpr int R = 4;
    dim3 grid((W + 31) / 32, B * ((H + R - 1) / R), C / 64);
    hipLaunchKernelGGL((dwconv_rows_kernel<7, R>), grid, dim3(256), 0, st, B, H, W, C, pad, (const bf16*)x, w, bias,
                       (bf16*)y);
    return (int)hipGetLastError();
  }
  if (C % 64 == 0 && K <= 7 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    dim3 grid((W + 31) / 32, B * H, C / 64);
    if (dt == S2H_BF16)
      hipLaunchKernelGGL(dwconv_vec_kernel<bf16>, grid, dim3(256), 0, st, B, H, W, C, K, pad, (const bf16*)x, w,
                         bias, (bf16*)y);
    else
      hipLaunchKernelGGL(dwconv_vec_kernel<float>, grid, dim3(256), 0, st, B, H, W, C, K, pad, (const float*)x, w,
                         bias, (float*)y);
    return (int)hipGetLastError();
  }
  DISPATCH_T(dt, dwconv_kernel, ew_grid(n), B, H, W, C, K, pad, x, w, bias, y);
  return (int)hipGetLastError();
}

// -------------------------------------------- ConvTranspose2d(k=2, s=2) NHWC
// GEMM output Y[(b,y,x)][co*4 + dy*2 + dx] (PyTorch weight [Ci, Co, 2, 2] as [Ci, Co*4])
// scatter (dir 0): out[b,2y+dy,2x+dx,co] = Y[...] + bias[co] (+ add[...])
// gather  (dir 1): dY[(b,y,x)][co*4+dy*2+dx] = dout[b,2y+dy,2x+dx,co]
template <typename T>
__global__ void convt2_kernel(int B, int H, int W, int Co, const void* Y, const float* bias, const void* add,
                              void* out, int dir) {
  const int64_t n = (int64_t)B * 2 * H * 2 * W * Co;
  GRID_STRIDE(i, n) {
    const int co = i % Co;
    int64_t p = i / Co;
    const int ox = p % (2 * W); p /= 2 * W;
    const int oy = p % (2 * H);
    const int b = p / (2 * H);
    const int64_t yi = (((int64_t)b * H + oy / 2) * W + ox / 2) * (4 * Co) + co * 4 + (oy & 1) * 2 + (ox & 1);
    if (dir == 0) {
      float v = to_f32(((const T*)Y)[yi]) + (bias ? bias[co] : 0.f);
      if (add) v += to_f32(((const T*)add)[i]);
      ((T*)out)[i] = from_f32<T>(v);
    } else {
      ((T*)out)[yi] = ((const T*)Y)[i];
    }
  }
}
// gather (dir 1), vectorised: one thread per (pixel, 16-B channel group) reads the 2 x 2 output
// pixels' V channels (4 16-B loads) and writes the group's 4 x V contiguous dY entries (co*4 + s:
// 4 16-B stores); the scalar form wrote 2-B elements at stride 4 (98 us per frame-batched launch)
template <typename T>
__global__ __launch_bounds__(256) void convt2_gather_vec_kernel(int B, int H, int W, int Co, const T* dout, T* dY) {
  constexpr int V = 16 / sizeof(T);
  const int CG = Co / V;
  const int64_t n = (int64_t)B * H * W * CG;
  GRID_STRIDE(i, n) {
    const int cg = (int)(i % CG);
    const int64_t p = i / CG;
    const int x = (int)(p % W);
    const int64_t t = p / W;
    const int y = (int)(t % H);
    const int b = (int)(t / H);
    T g[4][V];
#pragma unroll
    for (int sidx = 0; sidx < 4; ++sidx) {
      const int dy = sidx >> 1, dx = sidx & 1;
      const int64_t o = (((int64_t)b * 2 * H + 2 * y + dy) * 2 * W + 2 * x + dx) * Co + cg * V;
      *(uint4*)g[sidx] = *(const uint4*)(dout + o);
    }
    T e[4 * V];
#pragma unroll
    for (int j = 0; j < V; ++j)
#pragma unroll
      for (int sidx = 0; sidx < 4; ++sidx) e[4 * j + sidx] = g[sidx][j];
    uint4* yr = (uint4*)(dY + p * 4 * Co + (int64_t)cg * V * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) yr[u] = *(const uint4*)(e + u * V);
  }
}

extern "C" int s2h_convt2(int dt, int B, int H, int W, int Co, const void* Y, const float* bias, const void* add,
                          void* out, int dir, hipStream_t st) {
  const int64_t n = (int64_t)B * 4 * H * W * Co;
  if (n <= 0) return 0;
  const int V = dt == S2H_BF16 ? 8 : 4;
  if (dir == 1 && Co % V == 0 && al16(Y) && al16(out)) {
    const int64_t nv = n / 4 / V;
    if (dt == S2H_BF16)
      hipLaunchKernelGGL(convt2_gather_vec_kernel<bf16>, ew_grid(nv), dim3(256), 0, st, B, H, W, Co, (const bf16*)Y,
                         (bf16*)out);
    else
      hipLaunchKernelGGL(convt2_gather_vec_kernel<float>, ew_grid(nv), dim3(256), 0, st, B, H, W, Co,
                         (const float*)Y, (float*)out);
    return (int)hipGetLastError();
  }
  DISPATCH_T(dt, convt2_kernel, ew_grid(n), B, H, W, Co, Y, bias, add, out, dir);
  return (int)hipGetLastError();
}

// Vectorised scatter with the bias and the residual add fused (round 5, the mask decoder's upscaling
// dc1(x) + feat_s1 / dc2(x) + feat_s0, mask_decoder.py:105-107): one thread per (pixel, 16-B channel
// group) reads the group's 4 x V contiguous GEMM outputs (4 16-B loads: co*4 + s for its V channels)
// and writes the 2 x 2 output pixels (4 16-B stores), + bias[co] + add (add_bcast: one batch broadcast
// over B), bit-identical to the scalar scatter (2-B accesses at stride 4) followed by the separate
// (broadcast) add it replaces.
template <typename T>
__global__ __launch_bounds__(256) void convt2_store_kernel(int B, int H, int W, int Co, const T* Y,
                                                           const float* bias, const T* add, int add_bcast, T* out) {
  constexpr int V = 16 / sizeof(T);
  const int CG = Co / V;
  const int64_t n = (int64_t)B * H * W * CG;
  GRID_STRIDE(i, n) {
    const int cg = (int)(i % CG);
    const int64_t p = i / CG;  // (b * H + y) * W + x
    const int x = (int)(p % W);
    const int64_t t = p / W;
    const int y = (int)(t % H);
    const int b = (int)(t / H);
    T e[4 * V];
    const uint4* yr = (const uint4*)(Y + p * 4 * Co + (int64_t)cg * V * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) *(uint4*)(e + u * V) = yr[u];
    float bv[V];
#pragma unroll
    for (int j = 0; j < V; ++j) bv[j] = bias ? bias[cg * V + j] : 0.f;
#pragma unroll
    for (int sidx = 0; sidx < 4; ++sidx) {
      const int dy = sidx >> 1, dx = sidx & 1;
      const int64_t pix = ((int64_t)(2 * y + dy) * 2 * W + 2 * x + dx);  // within batch b
      const int64_t o = ((int64_t)b * 4 * H * W + pix) * Co + cg * V;
      float v[V];
      // rounded to T after the bias and again after the add: the values of the scatter + add launches
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] = to_f32(from_f32<T>(to_f32(e[4 * j + sidx]) + bv[j]));
      if (add) {
        T ad[V];
        *(uint4*)ad = *(const uint4*)(add + (add_bcast ? pix * Co + cg * V : o));
#pragma unroll
        for (int j = 0; j < V; ++j) v[j] += to_f32(ad[j]);
      }
      T r[V];
#pragma unroll
      for (int j = 0; j < V; ++j) r[j] = from_f32<T>(v[j]);
      *(uint4*)(out + o) = *(const uint4*)r;
    }
  }
}
extern "C" int s2h_convt2_store(int dt, int B, int H, int W, int Co, const void* Y, const float* bias, const void* add,
                                int add_bcast, void* out, hipStream_t st) {
  const int V = dt == S2H_BF16 ? 8 : 4;
  if (Co % V || !al16(Y) || !al16(out) || (add && !al16(add))) return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)B * H * W * (Co / V);
  if (n <= 0) return 0;
  if (dt == S2H_BF16)
    hipLaunchKernelGGL(convt2_store_kernel<bf16>, ew_grid(n), dim3(256), 0, st, B, H, W, Co, (const bf16*)Y, bias,
                       (const bf16*)add, add_bcast, (bf16*)out);
  else
    hipLaunchKernelGGL(convt2_store_kernel<float>, ew_grid(n), dim3(256), 0, st, B, H, W, Co, (const float*)Y, bias,
                       (const float*)add, add_bcast, (float*)out);
  return (int)hipGetLastError();
}

// The mask decoder's last upscaling step and mask head in one pass (round 5; mask_decoder.py:105-113:
// u = gelu(dc2(x) + feat_s0), masks = hyper0 . u per pixel): the convt2_store values (pre, the GEMM
// output scattered + bias + add, rounded as the separate launches round it), post = gelu(pre) rounded
// as act_fwd rounds it, and masks[b][pixel] = sum_c hyper[b][c] post[c] (fp32, the CG lanes of a pixel
// reduced by xor shuffles).  pre and post are stored for the backward (the GELU' and the hyper
// product's gradients).  Replaces the scatter, the activation and a batched M = 1 GEMM (30 us per
// frame, 13 row-vector products).
template <typename T, int CG>
__global__ __launch_bounds__(256) void convt2_tail_kernel(int B, int H, int W, const T* Y, const float* bias,
                                                          const T* add, int add_bcast, const T* hyper, T* pre, T* post,
                                                          T* masks) {
  constexpr int V = 16 / sizeof(T);
  constexpr int Co = CG * V;
  const int64_t n = (int64_t)B * H * W * CG;
  GRID_STRIDE(i, n) {  // (n is a multiple of CG: a pixel's CG lanes stay together)
    const int cg = (int)(i % CG);
    const int64_t p = i / CG;  // (b * H + y) * W + x
    const int x = (int)(p % W);
    const int64_t t = p / W;
    const int y = (int)(t % H);
    const int b = (int)(t / H);
    T e[4 * V];
    const uint4* yr = (const uint4*)(Y + p * 4 * Co + (int64_t)cg * V * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) *(uint4*)(e + u * V) = yr[u];
    float bv[V], hv[V];
    T hb[V];
    *(uint4*)hb = *(const uint4*)(hyper + (int64_t)b * Co + cg * V);
#pragma unroll
    for (int j = 0; j < V; ++j) {
      bv[j] = bias ? bias[cg * V + j] : 0.f;
      hv[j] = to_f32(hb[j]);
    }
#pragma unroll
    for (int sidx = 0; sidx < 4; ++sidx) {
      const int dy = sidx >> 1, dx = sidx & 1;
      const int64_t pix = ((int64_t)(2 * y + dy) * 2 * W + 2 * x + dx);  // within batch b
      const int64_t o = ((int64_t)b * 4 * H * W + pix) * Co + cg * V;
      float v[V];
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] = to_f32(from_f32<T>(to_f32(e[4 * j + sidx]) + bv[j]));
      if (add) {
        T ad[V];
        *(uint4*)ad = *(const uint4*)(add + (add_bcast ? pix * Co + cg * V : o));
#pragma unroll
        for (int j = 0; j < V; ++j) v[j] += to_f32(ad[j]);
      }
      T r[V], g[V];
      float dot = 0.f;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        r[j] = from_f32<T>(v[j]);
        g[j] = from_f32<T>(gelu_erf(to_f32(r[j])) + 0.f);  // (+ 0: act_fwd's `* 1 + 0`, -0 -> +0)
        dot += hv[j] * to_f32(g[j]);
      }
      *(uint4*)(pre + o) = *(const uint4*)r;
      *(uint4*)(post + o) = *(const uint4*)g;
#pragma unroll
      for (int m = 1; m < CG; m <<= 1) dot += __shfl_xor(dot, m, 64);
      if (cg == 0) masks[(int64_t)b * 4 * H * W + pix] = from_f32<T>(dot);
    }
  }
}
extern "C" int s2h_convt2_tail(int dt, int B, int H, int W, int Co, const void* Y, const float* bias, const void* add,
                               int add_bcast, const void* hyper, void* pre, void* post, void* masks, hipStream_t st) {
  if (dt != S2H_BF16 || Co != 32 || !al16(Y) || !al16(pre) || !al16(post) || !al16(hyper) || (add && !al16(add)))
    return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)B * H * W * 4;
  if (n <= 0) return 0;
  hipLaunchKernelGGL((convt2_tail_kernel<bf16, 4>), ew_grid(n), dim3(256), 0, st, B, H, W, (const bf16*)Y, bias,
                     (const bf16*)add, add_bcast, (const bf16*)hyper, (bf16*)pre, (bf16*)post, (bf16*)masks);
  return (int)hipGetLastError();
}

// The mask decoder's first upscaling step in one pass (round 5; mask_decoder.py:105-106:
// u = gelu(LayerNorm2d(dc1(x) + feat_s1))): pre = the convt2_store values, y = LayerNorm over the Co
// channels of each output pixel with the arithmetic of norm.hip ln_fwd_vec_kernel<bf16, CG, 1> (the CG
// lanes of a pixel each sum their 8 channels in order, then xor 4, 2, 1; two-pass variance) -- so y,
// mean and rstd are bit-identical to that kernel's -- and post = gelu(y) as act_fwd rounds it.  pre,
// mean / rstd and y / post are what the LayerNorm's, the GELU's and dc2's backward read.
template <typename T, int CG>
__global__ __launch_bounds__(256) void convt2_ln_gelu_kernel(int B, int H, int W, const T* Y, const float* bias,
                                                             const T* add, int add_bcast, const float* gamma,
                                                             const float* beta, float eps, T* pre, T* y, float* mean,
                                                             float* rstd, T* post) {
  constexpr int V = 16 / sizeof(T);
  constexpr int Co = CG * V;
  const int64_t n = (int64_t)B * H * W * CG;
  GRID_STRIDE(i, n) {  // (n is a multiple of CG: a pixel's CG lanes stay together)
    const int cg = (int)(i % CG);
    const int64_t p = i / CG;  // (b * H + y) * W + x
    const int x = (int)(p % W);
    const int64_t t = p / W;
    const int yy = (int)(t % H);
    const int b = (int)(t / H);
    T e[4 * V];
    const uint4* yr = (const uint4*)(Y + p * 4 * Co + (int64_t)cg * V * 4);
#pragma unroll
    for (int u = 0; u < 4; ++u) *(uint4*)(e + u * V) = yr[u];
    float bv[V], gv[V], be[V];
#pragma unroll
    for (int j = 0; j < V; ++j) {
      bv[j] = bias ? bias[cg * V + j] : 0.f;
      gv[j] = gamma[cg * V + j];
      be[j] = beta[cg * V + j];
    }
#pragma unroll
    for (int sidx = 0; sidx < 4; ++sidx) {
      const int dy = sidx >> 1, dx = sidx & 1;
      const int64_t pix = ((int64_t)(2 * yy + dy) * 2 * W + 2 * x + dx);  // within batch b
      const int64_t row = (int64_t)b * 4 * H * W + pix;
      const int64_t o = row * Co + cg * V;
      float v[V];
#pragma unroll
      for (int j = 0; j < V; ++j) v[j] = to_f32(from_f32<T>(to_f32(e[4 * j + sidx]) + bv[j]));
      if (add) {
        T ad[V];
        *(uint4*)ad = *(const uint4*)(add + (add_bcast ? pix * Co + cg * V : o));
#pragma unroll
        for (int j = 0; j < V; ++j) v[j] += to_f32(ad[j]);
      }
      T r[V];
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        r[j] = from_f32<T>(v[j]);
        v[j] = to_f32(r[j]);
        s += v[j];
      }
      *(uint4*)(pre + o) = *(const uint4*)r;
#pragma unroll
      for (int m = CG / 2; m > 0; m >>= 1) s += __shfl_xor(s, m, 64);
      const float mu = s / Co;
      float q = 0.f;
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const float d = v[j] - mu;
        q += d * d;
      }
#pragma unroll
      for (int m = CG / 2; m > 0; m >>= 1) q += __shfl_xor(q, m, 64);
      const float rs = 1.f / sqrtf(q / Co + eps);
      T yo[V], g[V];
#pragma unroll
      for (int j = 0; j < V; ++j) {
        yo[j] = from_f32<T>((v[j] - mu) * rs * gv[j] + be[j]);
        g[j] = from_f32<T>(gelu_erf(to_f32(yo[j])) + 0.f);  // (+ 0: act_fwd's `* 1 + 0`)
      }
      *(uint4*)(y + o) = *(const uint4*)yo;
      *(uint4*)(post + o) = *(const uint4*)g;
      if (cg == 0) {
        mean[row] = mu;
        rstd[row] = rs;
      }
    }
  }
}
extern "C" int s2h_convt2_ln_gelu(int dt, int B, int H, int W, int Co, const void* Y, const float* bias,
                                  const void* add, int add_bcast, const float* gamma, const float* beta, float eps,
                                  void* pre, void* y, float* mean, float* rstd, void* post, hipStream_t st) {
  if (dt != S2H_BF16 || Co != 64 || !al16(Y) || !al16(pre) || !al16(y) || !al16(post) || (add && !al16(add)) ||
      !gamma || !beta)
    return (int)hipErrorInvalidValue;
  const int64_t n = (int64_t)B * H * W * 8;
  if (n <= 0) return 0;
  hipLaunchKernelGGL((convt2_ln_gelu_kernel<bf16, 8>), ew_grid(n), dim3(256), 0, st, B, H, W, (const bf16*)Y, bias,
                     (const bf16*)add, add_bcast, gamma, beta, eps, (bf16*)pre, (bf16*)y, mean, rstd, (bf16*)post);
  return (int)hipGetLastError();
}

// -------------------------------------------------- per-row gate / select
// y[r, j] = gate[r] > 0 ? x[r, j] : fill ;  backward (dir 1): dx = gate > 0 ? dy : 0
template <typename T>
__global__ void row_gate_kernel(int64_t rows, int64_t inner, const void* x, const float* gate, float fill, void* y,
                                int dir) {
  const int64_t n = rows * inner;
  GRID_STRIDE(i, n) {
    const bool on = gate[i / inner] > 0.f;
    float v = on ? to_f32(((const T*)x)[i]) : (dir == 0 ? fill : 0.f);
    ((T*)y)[i] = from_f32<T>(v);
  }
}
extern "C" int s2h_row_gate(int dt, int64_t rows, int64_t inner, const void* x, const float* gate, float fill,
                            void* y, int dir, hipStream_t st) {
  if (rows * inner <= 0) return 0;
  DISPATCH_T(dt, row_gate_kernel, ew_grid(rows * inner), rows, inner, x, gate, fill, y, dir);
  return (int)hipGetLastError();
}
// row_gate with its own input and output types: the low-res mask logits' cast to fp32 and the
// object-score gate of sam2_base.py:380-389 in one pass (forward bf16 -> fp32; backward fp32 ->
// bf16, dx = gate > 0 ? dy : 0); gate_out (nullable): the gate copied for the backward
template <typename TI, typename TO>
__global__ void row_gate_cast_kernel(int64_t rows, int64_t inner, const TI* x, const float* gate, float fill, TO* y,
                                     int dir, float* gate_out) {
  const int64_t n = rows * inner;
  GRID_STRIDE(i, n) {
    const bool on = gate[i / inner] > 0.f;
    y[i] = from_f32<TO>(on ? to_f32(x[i]) : (dir == 0 ? fill : 0.f));
    if (gate_out != nullptr && i < rows) gate_out[i] = gate[i];
  }
}
extern "C" int s2h_row_gate_cast(int dt_in, int dt_out, int64_t rows, int64_t inner, const void* x, const float* gate,
                                 float fill, void* y, int dir, float* gate_out, hipStream_t st) {
  if (rows * inner <= 0) return 0;
  const dim3 g = ew_grid(rows * inner);
  if (dt_in == S2H_BF16 && dt_out == S2H_F32)
    hipLaunchKernelGGL((row_gate_cast_kernel<bf16, float>), g, dim3(256), 0, st, rows, inner, (const bf16*)x, gate,
                       fill, (float*)y, dir, gate_out);
  else if (dt_in == S2H_F32 && dt_out == S2H_BF16)
    hipLaunchKernelGGL((row_gate_cast_kernel<float, bf16>), g, dim3(256), 0, st, rows, inner, (const float*)x, gate,
                       fill, (bf16*)y, dir, gate_out);
  else if (dt_in == S2H_F32 && dt_out == S2H_F32)
    hipLaunchKernelGGL((row_gate_cast_kernel<float, float>), g, dim3(256), 0, st, rows, inner, (const float*)x, gate,
                       fill, (float*)y, dir, gate_out);
  else if (dt_in == S2H_BF16 && dt_out == S2H_BF16)
    hipLaunchKernelGGL((row_gate_cast_kernel<bf16, bf16>), g, dim3(256), 0, st, rows, inner, (const bf16*)x, gate,
                       fill, (bf16*)y, dir, gate_out);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
// y[r, j] = x[r, j] + (1 - (gate[r] > 0)) * vec[j]   (no-object embedding / pointer mixing)
// if scale_x: y = (gate>0)*x + (1-(gate>0))*vec  (fixed_no_obj_ptr form)
template <typename T>
__global__ void gate_mix_kernel(int64_t rows, int64_t inner, const void* x, const float* gate, const void* vec,
                                int vec_period, int scale_x, void* y) {
  const int64_t n = rows * inner;
  GRID_STRIDE(i, n) {
    const float lam = gate[i / inner] > 0.f ? 1.f : 0.f;
    float xv = to_f32(((const T*)x)[i]);
    if (scale_x) xv *= lam;
    const float v = xv + (1.f - lam) * to_f32(((const T*)vec)[(i % inner) % vec_period]);
    ((T*)y)[i] = from_f32<T>(v);
  }
}
extern "C" int s2h_gate_mix(int dt, int64_t rows, int64_t inner, const void* x, const float* gate, const void* vec,
                            int vec_period, int scale_x, void* y, hipStream_t st) {
  if (rows * inner <= 0) return 0;
  DISPATCH_T(dt, gate_mix_kernel, ew_grid(rows * inner), rows, inner, x, gate, vec, vec_period, scale_x, y);
  return (int)hipGetLastError();
}

// ------------------------------------------ Hiera windowed pos-embed finish
// out[i, j, c] = Y[c, i, j] + win[c, i % ws, j % ws]   (Y = bicubic(pos_embed), fp32 CHW -> T HWC)
template <typename T>
__global__ void pos_embed_fwd_kernel(int C, int h, int w, int ws, const float* Y, const float* win, void* out) {
  const int64_t n = (int64_t)h * w * C;
  GRID_STRIDE(i, n) {
    const int c = i % C;
    const int64_t p = i / C;
    const int x = p % w, y = p / w;
    const float v = Y[((int64_t)c * h + y) * w + x] + win[(c * ws + y % ws) * ws + x % ws];
    ((T*)out)[i] = from_f32<T>(v);
  }
}
// dY[c, i, j] = dout[i, j, c] (f32) ; dwin[c, a, b] += sum over (i%ws==a, j%ws==b) dout[i, j, c]
template <typename T>
__global__ void pos_embed_bwd_kernel(int C, int h, int w, int ws, const void* dout, float* dY, float* dwin) {
  const int64_t n = (int64_t)h * w * C;
  GRID_STRIDE(i, n) {
    const int c = i % C;
    const int64_t p = i / C;
    const int x = p % w, y = p / w;
    const float g = to_f32(((const T*)dout)[i]);
    if (dY) dY[((int64_t)c * h + y) * w + x] = g;
    if (dwin) atomicAdd(&dwin[(c * ws + y % ws) * ws + x % ws], g);
  }
}
extern "C" int s2h_pos_embed(int dt, int C, int h, int w, int ws, const float* Y, const float* win, void* out,
                             hipStream_t st) {
  const int64_t n = (int64_t)h * w * C;
  if (n <= 0) return 0;
  DISPATCH_T(dt, pos_embed_fwd_kernel, ew_grid(n), C, h, w, ws, Y, win, out);
  return (int)hipGetLastError();
}
// dwin[c, a, b] += sum over (i % ws == a, j % ws == b) dout[i, j, c]: one thread per window element,
// the positions in row-major order (deterministic; the scatter form added with float atomics)
// (16 slices per window element: slice sl takes the copies k = sl, sl + 16, ... in row-major order,
// the slice sums added in a fixed LDS tree -- one serial chain of (h / ws) * (w / ws) loads per element
// and only C * ws^2 threads took 68 us for Hiera-B+ at 512^2)
template <typename T>
__global__ __launch_bounds__(256) void pos_win_bwd_kernel(int C, int h, int w, int ws, const void* dout, float* dwin) {
  constexpr int SL = 16;
  const int n = C * ws * ws;
  const int e = blockIdx.x * 16 + (threadIdx.x & 15);
  const int sl = threadIdx.x >> 4;
  __shared__ float red[SL][16];
  float s = 0.f;
  if (e < n) {
    const int c = e % C, ab = e / C, a = ab / ws, b = ab % ws;
    const int ny = (h - a + ws - 1) / ws, nx = (w - b + ws - 1) / ws;
    for (int k = sl; k < ny * nx; k += SL) {
      const int y = a + (k / nx) * ws, x = b + (k % nx) * ws;
      s += to_f32(((const T*)dout)[((int64_t)y * w + x) * C + c]);
    }
  }
  red[sl][threadIdx.x & 15] = s;
  __syncthreads();
#pragma unroll
  for (int hh = SL / 2; hh >= 1; hh >>= 1) {
    if (sl < hh) red[sl][threadIdx.x & 15] += red[sl + hh][threadIdx.x & 15];
    __syncthreads();
  }
  if (sl == 0 && e < n) {
    const int c = e % C, ab = e / C, a = ab / ws, b = ab % ws;
    dwin[(c * ws + a) * ws + b] += red[0][threadIdx.x & 15];
  }
}
extern "C" int s2h_pos_embed_bwd(int dt, int C, int h, int w, int ws, const void* dout, float* dY, float* dwin,
                                 hipStream_t st) {
  const int64_t n = (int64_t)h * w * C;
  if (n <= 0) return 0;
  if (dY) DISPATCH_T(dt, pos_embed_bwd_kernel, ew_grid(n), C, h, w, ws, dout, dY, (float*)nullptr);
  if (dwin) {
    const dim3 g((C * ws * ws + 15) / 16);
    if (dt == S2H_BF16) hipLaunchKernelGGL(pos_win_bwd_kernel<bf16>, g, dim3(256), 0, st, C, h, w, ws, dout, dwin);
    else hipLaunchKernelGGL(pos_win_bwd_kernel<float>, g, dim3(256), 0, st, C, h, w, ws, dout, dwin);
  }
  return (int)hipGetLastError();
}

// ------------------------------------------------ point-prompt embeddings
// out[r, :] = pe[r, :] * (label != -1) + table[label + 1, :]   (table rows: not_a_point, pe0..pe3)
// backward: dtable[label + 1, :] += dout[r, :]  (f32, serial over rows -> deterministic)
// labels_out (nullable): the labels copied (the frame tape keeps them for the backward)
template <typename T>
__global__ void point_embed_kernel(int R, int D, const float* pe, const int* labels, const void* table, void* out,
                                   int* labels_out) {
  const int64_t n = (int64_t)R * D;
  GRID_STRIDE(i, n) {
    const int r = i / D, d = i % D;
    const int l = labels[r];
    float v = (l == -1 ? 0.f : pe[i]) + to_f32(((const T*)table)[(l + 1) * D + d]);
    ((T*)out)[i] = from_f32<T>(v);
    if (labels_out != nullptr && d == 0) labels_out[r] = l;
  }
}
// one thread per column; the 5 label rows' sums in registers in row order (the same additions, in the
// same order, as adding into dtable row by row -- which made every row wait for the previous row's
// store: 53 us for the step's ~200 click rows)
// the 5 label rows' gradient destinations (rows of one table, or the 5 parameters' own gradients)
struct PeRows {
  float* r[5];
};
template <typename T>
__global__ void point_embed_bwd_kernel(int R, int D, const int* labels, const void* dout, PeRows rows) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= D) return;
  float acc[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) acc[k] = rows.r[k][d];
#pragma unroll 8
  for (int r = 0; r < R; ++r) {
    const int l = labels[r] + 1;
    const float v = to_f32(((const T*)dout)[(int64_t)r * D + d]);
#pragma unroll
    for (int k = 0; k < 5; ++k)
      if (l == k) acc[k] += v;
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) rows.r[k][d] = acc[k];
}
extern "C" int s2h_point_embed(int dt, int R, int D, const float* pe, const int* labels, const void* table, void* out,
                               int* labels_out, hipStream_t st) {
  if (R * D <= 0) return 0;
  DISPATCH_T(dt, point_embed_kernel, ew_grid((int64_t)R * D), R, D, pe, labels, table, out, labels_out);
  return (int)hipGetLastError();
}
extern "C" int s2h_point_embed_bwd(int dt, int R, int D, const int* labels, const void* dout, float* dtable,
                                   hipStream_t st) {
  if (R * D <= 0) return 0;
  PeRows rows;
  for (int k = 0; k < 5; ++k) rows.r[k] = dtable + (int64_t)k * D;
  DISPATCH_T(dt, point_embed_bwd_kernel, dim3((D + 255) / 256), R, D, labels, dout, rows);
  return (int)hipGetLastError();
}
extern "C" int s2h_point_embed_bwd_rows(int dt, int R, int D, const int* labels, const void* dout,
                                        float* const* drows, hipStream_t st) {
  if (R * D <= 0) return 0;
  PeRows rows;
  for (int k = 0; k < 5; ++k) {
    if (drows[k] == nullptr) return (int)hipErrorInvalidValue;
    rows.r[k] = drows[k];
  }
  DISPATCH_T(dt, point_embed_bwd_kernel, dim3((D + 255) / 256), R, D, labels, dout, rows);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ zero fill
__global__ __launch_bounds__(256) void zero_f32_kernel(float* p, int64_t rows, int64_t cols, int64_t ld) {
  const int64_t n = rows * cols;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / cols;
    p[r * ld + (i - r * cols)] = 0.f;
  }
}
__global__ __launch_bounds__(256) void zero_f32x4_kernel(float4* p, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    p[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}
void s2h_zero_f32(float* p, int64_t rows, int64_t cols, int64_t ld, hipStream_t st) {
  const int64_t n = rows * cols;
  if (n <= 0) return;
  if (ld == cols && (uintptr_t)p % 16 == 0 && n % 4 == 0) {
    const int64_t n4 = n / 4;
    int64_t b = (n4 + 255) / 256;
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(zero_f32x4_kernel, dim3((unsigned)b), dim3(256), 0, st, (float4*)p, n4);
    return;
  }
  int64_t b = (n + 255) / 256;
  if (b > 4096) b = 4096;
  hipLaunchKernelGGL(zero_f32_kernel, dim3((unsigned)b), dim3(256), 0, st, p, rows, cols, ld);
}

// ------------------------------------------------------------------ V-fold value projection
// [Wv | bv | 0] (bf16 [N, ld], ld >= K + 8): the value projection's weight with its bias as an
// extra input column, the B operand of u' [rows, K + 8] x [Wv | bv | 0]^T (flash.hip V-fold).
// wv is the compute-dtype (bf16) weight [N, K], bv the fp32 bias [N].
__global__ __launch_bounds__(256) void vfold_weight_kernel(int N, int K, int ld, const bf16* wv, const float* bv,
                                                           bf16* out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)N * ld) return;
  const int n = (int)(i / ld), k = (int)(i % ld);
  out[i] = k < K ? wv[(int64_t)n * K + k] : (k == K ? (bf16)bv[n] : (bf16)0.f);
}
extern "C" int s2h_vfold_weight(int N, int K, int ld, const void* wv, const float* bv, void* out, hipStream_t st) {
  if (N <= 0) return 0;
  if (ld < K + 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(vfold_weight_kernel, dim3((unsigned)(((int64_t)N * ld + 255) / 256)), dim3(256), 0, st, N, K, ld,
                     (const bf16*)wv, bv, (bf16*)out);
  return (int)hipGetLastError();
}

// the weight gradient of [Wv | bv | 0] (fp32 [N, ld]) scattered back: gwv [N, K] += g[:, :K],
// gbv [N] += g[:, K] (either may be null: frozen)
__global__ __launch_bounds__(256) void vfold_grad_kernel(int N, int K, int ld, const float* g, float* gwv, float* gbv) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)N * (K + 1)) return;
  const int n = (int)(i / (K + 1)), k = (int)(i % (K + 1));
  const float v = g[(int64_t)n * ld + k];
  if (k < K) {
    if (gwv) gwv[(int64_t)n * K + k] += v;
  } else if (gbv) {
    gbv[n] += v;
  }
}
extern "C" int s2h_vfold_grad(int N, int K, int ld, const float* g, float* gwv, float* gbv, hipStream_t st) {
  if (N <= 0) return 0;
  if (ld < K + 1) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(vfold_grad_kernel, dim3((unsigned)(((int64_t)N * (K + 1) + 255) / 256)), dim3(256), 0, st, N, K,
                     ld, g, gwv, gbv);
  return (int)hipGetLastError();
}

// ------------------------------------------------------- memory positional rows
// The memory attention's key positions (sam2_base memory pos; functional_sam.memory_pos): slot j of
// the memory bank gets out[j L + l] = spatial_pos[l] + tpos[idx[j]] -- all slots in one launch
// (the per-slot broadcast adds were one launch each).  Backward: the tpos rows' gradient is the
// column sum of each slot's rows, all slots of all frames in one segmented launch.
struct MposTable { int idx[16]; };
template <typename T>
__global__ __launch_bounds__(256) void memory_pos_vec_kernel(int nvec, int L, int dv, const T* pos, const T* tpos,
                                                             MposTable tb, T* out) {
  constexpr int V = V16<T>::VEC;
  for (int v = blockIdx.x * 256 + threadIdx.x; v < nvec; v += gridDim.x * 256) {
    const int c = (v % dv) * V, row = v / dv, j = row / L, l = row - j * L;
    float a[V], b[V];
    V16<T>::load(pos + (int64_t)l * dv * V + c, a);
    V16<T>::load(tpos + (int64_t)tb.idx[j] * dv * V + c, b);
#pragma unroll
    for (int e = 0; e < V; ++e) a[e] += b[e];
    V16<T>::store(out + (int64_t)row * dv * V + c, a);
  }
}
extern "C" int s2h_memory_pos(int dt, int n, int L, int Dm, const void* pos, const void* tpos, const int* idx, void* out,
                              hipStream_t st) {
  if (n <= 0 || L <= 0) return 0;
  const int V = dt == S2H_BF16 ? 8 : 4;
  if (n > 16 || Dm % V != 0 || !al16(pos) || !al16(tpos) || !al16(out) || (int64_t)n * L * Dm / V >= (1ll << 31))
    return (int)hipErrorInvalidValue;
  MposTable tb = {};
  for (int j = 0; j < n; ++j) tb.idx[j] = idx[j];
  const int nvec = n * L * (Dm / V);
  if (dt == S2H_BF16)
    hipLaunchKernelGGL(memory_pos_vec_kernel<bf16>, ew_grid(nvec), dim3(256), 0, st, nvec, L, Dm / V, (const bf16*)pos,
                       (const bf16*)tpos, tb, (bf16*)out);
  else
    hipLaunchKernelGGL(memory_pos_vec_kernel<float>, ew_grid(nvec), dim3(256), 0, st, nvec, L, Dm / V, (const float*)pos,
                       (const float*)tpos, tb, (float*)out);
  return (int)hipGetLastError();
}

// segmented column sums: out[dst[s]][:] += sum over rows r < rows of x[off[s] + r][:]  (s < nseg <= 64,
// blockIdx.y = segment; colsum_vec_kernel's row-lane plan within each segment)
struct SegTable { int64_t off[64]; int dst[64]; };
template <typename T>
__global__ __launch_bounds__(256) void colsum_seg_kernel(int64_t rows, int cols, const T* x, int64_t ld,
                                                         int64_t rows_per_block, SegTable tb, float* out, float* part) {
  constexpr int V = 16 / sizeof(T);
  const int G = cols / V;
  const int lanes = 256 / G;
  const int g = threadIdx.x % G, lane = threadIdx.x / G;
  __shared__ float red[256 * 8];
  x += tb.off[blockIdx.y] * ld;
  out += (int64_t)tb.dst[blockIdx.y] * cols;
  if (part) part += ((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * cols;
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
  const int64_t r0 = blockIdx.x * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  if (lane < lanes) {
    for (int64_t r = r0 + lane; r < r1; r += lanes) {
      const uint4 u = *(const uint4*)(x + r * ld + g * V);
      const T* t = (const T*)&u;
#pragma unroll
      for (int j = 0; j < V; ++j) acc[j] += to_f32(t[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < V; ++j) red[threadIdx.x * V + j] = (lane < lanes) ? acc[j] : 0.f;
  __syncthreads();
  for (int c = threadIdx.x; c < cols; c += 256) {
    const int gg = c / V, j = c % V;
    float s = 0.f;
    for (int l = 0; l < lanes; ++l) s += red[(l * G + gg) * V + j];
    if (part) part[c] = s;
    else atomicAdd(&out[c], s);
  }
}
// out[d][c] += the partials of every segment s with dst[s] == d (segments in order, then blocks in
// order): one thread per (destination row, column), deterministic
// one workgroup per (destination row, 64 columns), 1024 threads = 64 columns x 16 slices: the
// destination's partial rows (its segments in order, nbx blocks each) are dealt to the slices
// round-robin, the slice sums added in a fixed LDS tree (one thread per column walking every
// segment's blocks took 56 us)
__global__ __launch_bounds__(1024) void colsum_seg_finalize_kernel(int nseg, int nbx, int ndst, int cols, SegTable tb,
                                                                   const float* part, float* out) {
  const int d = blockIdx.y;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int sl = threadIdx.x >> 6;
  __shared__ float red[16][64];
  float s = 0.f;
  bool any = false;
  int q = 0;  // index of this destination's partial rows
  for (int sg = 0; sg < nseg; ++sg) {
    if (tb.dst[sg] != d) continue;
    any = true;
    if (c < cols) {
      const float* p = part + (int64_t)sg * nbx * cols + c;
      // rows b of this segment with (q + b) % 16 == sl
      for (int b = (sl - q % 16 + 16) % 16; b < nbx; b += 16) s += p[(int64_t)b * cols];
    }
    q += nbx;
  }
  red[sl][threadIdx.x & 63] = s;
  __syncthreads();
#pragma unroll
  for (int hh = 8; hh >= 1; hh >>= 1) {
    if (sl < hh) red[sl][threadIdx.x & 63] += red[sl + hh][threadIdx.x & 63];
    __syncthreads();
  }
  if (sl == 0 && any && c < cols) out[(int64_t)d * cols + c] += red[0][threadIdx.x & 63];
}
extern "C" int s2h_colsum_seg(int dt, int nseg, int64_t rows, int cols, const void* x, int64_t ld, const int64_t* offs,
                              const int* dsts, float* out, hipStream_t st) {
  if (nseg <= 0 || rows <= 0 || cols <= 0) return 0;
  const int V = dt == S2H_BF16 ? 8 : 4;
  if (nseg > 64 || cols % V != 0 || cols / V > 256 || ld % V != 0 || !al16(x)) return (int)hipErrorInvalidValue;
  SegTable tb = {};
  for (int s = 0; s < nseg; ++s) {
    tb.off[s] = offs[s];
    tb.dst[s] = dsts[s];
  }
  int64_t rpb = (rows + 63) / 64;  // ~64 blocks per segment, each >= 16 rows
  if (rpb < 16) rpb = 16;
  const dim3 grid((unsigned)((rows + rpb - 1) / rpb), (unsigned)nseg);
  float* part = s2h_det_ws((int64_t)grid.x * nseg * cols * (int64_t)sizeof(float));
  if (dt == S2H_BF16)
    hipLaunchKernelGGL(colsum_seg_kernel<bf16>, grid, dim3(256), 0, st, rows, cols, (const bf16*)x, ld, rpb, tb, out,
                       part);
  else
    hipLaunchKernelGGL(colsum_seg_kernel<float>, grid, dim3(256), 0, st, rows, cols, (const float*)x, ld, rpb, tb, out,
                       part);
  if (part) {
    int ndst = 0;
    for (int sg = 0; sg < nseg; ++sg) ndst = std::max(ndst, dsts[sg] + 1);
    hipLaunchKernelGGL(colsum_seg_finalize_kernel, dim3((cols + 63) / 64, ndst), dim3(1024), 0, st, nseg,
                       (int)grid.x, ndst, cols, tb, part, out);
  }
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------- batched 2-D copies
// Up to 16 strided 2-D copies in ONE launch: the per-frame memory bank assembly (the reference's
// torch.cat of the spatial memories and object pointers, sam2_base.py:649-676) and the tracking
// loop's per-frame gradient packing, which otherwise cost one copy launch per bank entry / frame.
// Segment s: rows[s] rows of row_bytes[s] bytes, source / destination pitches in bytes; every base,
// pitch and row length a multiple of 16 B (16-B pieces) or of 4 B (4-B pieces: the per-frame IoU
// gradients of the tracking loop, 13 floats); destination rows may not overlap, source rows may (a
// source pitch of 0 broadcasts one row block: the decoder's learned tokens into every object).
// One lane per piece, grid-stride over the pieces of all segments (segment found by a scan of the
// <= 16 prefix offsets, uniform in most waves).
constexpr int kCopySegs = 16;
struct CopySegs {
  const char* src[kCopySegs];
  char* dst[kCopySegs];
  int64_t start[kCopySegs + 1];  // first piece of each segment
  int64_t src_ld[kCopySegs], dst_ld[kCopySegs];  // pitches in bytes
  uint32_t row_pieces[kCopySegs];
  int shift[kCopySegs];  // log2 of the segment's piece size: 4 (16 B) or 2 (4 B)
  int n;
};
__global__ __launch_bounds__(256) void copy_segs_kernel(CopySegs a) {
  const int64_t total = a.start[a.n];
  GRID_STRIDE(i, total) {
    int s = 0;
    while (s + 1 < a.n && i >= a.start[s + 1]) ++s;
    const uint32_t c = (uint32_t)(i - a.start[s]);
    const uint32_t r = c / a.row_pieces[s], col = c - r * a.row_pieces[s];
    const int sh = a.shift[s];
    const char* sp = a.src[s] + (int64_t)r * a.src_ld[s] + ((int64_t)col << sh);
    char* dp = a.dst[s] + (int64_t)r * a.dst_ld[s] + ((int64_t)col << sh);
    if (sh == 4) *(uint4*)dp = *(const uint4*)sp;
    else *(uint32_t*)dp = *(const uint32_t*)sp;
  }
}
extern "C" int s2h_copy2d_batch(int n, const void* const* src, void* const* dst, const int64_t* rows,
                                const int64_t* row_bytes, const int64_t* src_ld, const int64_t* dst_ld,
                                hipStream_t st) {
  if (n <= 0) return 0;
  if (n > kCopySegs) return (int)hipErrorInvalidValue;
  CopySegs a = {};
  a.n = n;
  a.start[0] = 0;
  auto al = [](int64_t v, int64_t m) { return v % m == 0; };
  for (int s = 0; s < n; ++s) {
    const bool v16 = al16(src[s]) && al16(dst[s]) && al(row_bytes[s], 16) && al(src_ld[s], 16) && al(dst_ld[s], 16);
    const bool v4 = ((uintptr_t)src[s] & 3) == 0 && ((uintptr_t)dst[s] & 3) == 0 && al(row_bytes[s], 4) &&
                    al(src_ld[s], 4) && al(dst_ld[s], 4);
    if ((!v16 && !v4) || rows[s] < 0 || row_bytes[s] <= 0 || src_ld[s] < 0 ||
        (rows[s] > 1 && dst_ld[s] < row_bytes[s]))
      return (int)hipErrorInvalidValue;
    a.shift[s] = v16 ? 4 : 2;
    const int64_t pieces = rows[s] * (row_bytes[s] >> a.shift[s]);
    if (pieces >= (1ll << 32)) return (int)hipErrorInvalidValue;
    a.src[s] = (const char*)src[s];
    a.dst[s] = (char*)dst[s];
    a.row_pieces[s] = (uint32_t)(row_bytes[s] >> a.shift[s]);
    a.src_ld[s] = src_ld[s];
    a.dst_ld[s] = dst_ld[s];
    a.start[s + 1] = a.start[s] + pieces;
  }
  if (a.start[n] == 0) return 0;
  hipLaunchKernelGGL(copy_segs_kernel, ew_grid(a.start[n]), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}
