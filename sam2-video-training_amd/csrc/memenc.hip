// Memory-encoder mask down-sampler stage, fused: 3x3 / stride 2 / pad 1 conv +
// LayerNorm2d (over the output channels) + GELU, NHWC, one thread per output pixel.
// Replaces MaskDownSampler.encoder[3i .. 3i+2] (memory_encoder.py:17-55:
// Conv2d(cin, cin*4, 3, 2, 1) -> LayerNorm2d -> GELU; sam2.1_hiera_*.yaml
// mask_downsampler kernel_size 3, stride 2, padding 1) for the narrow stages
// (cin 1 -> 4, 4 -> 16, 16 -> 64) where an im2col GEMM wastes the MFMA tile on
// 4..64 columns and the LayerNorm wastes a wave on 4..64 channels.
//
// The first stage can read the decoder's fp32 high-res logits directly and apply
// the memory-encoder input transform sigmoid(x) * scale + shift
// (sam2_base.py:742-747, sigmoid_scale_for_mem_enc / sigmoid_bias_for_mem_enc),
// rounded to the compute dtype as the unfused path stores it; zero padding is
// applied to the transformed mask (F.conv2d pads its input with zeros).
//
// Weights arrive in PyTorch order [cout][cin][3][3] (fp32) and are transposed into LDS as
// [tap][cin][cout] per block (4 output channels per broadcast ds_read_b128; per-weight scalar
// loads in a rolled tap loop measured 180 us for the 16 -> 64 stage).  HBM-bound: reads
// O*H*W*cin, writes O*H/2*W/2*cout elements.
#include "common.h"

// SPLIT lanes per output pixel (adjacent lanes), each accumulating COUT / SPLIT channels: the 16 -> 64
// stage at one thread per pixel ran ~1 wave per SIMD with 9216 dependent-free FMAs each and no latency
// hiding (65 us per frame, profiles/r05_v16_kernel_stats.csv); the LayerNorm statistics gather the
// pixel's channels from its SPLIT lanes and sum them in channel order.
template <typename T, int CIN, int COUT, bool LOGIT, int SPLIT = 1>
__global__ __launch_bounds__(256) void mask_down_kernel(int O, int H, int W, int Ho, int Wo, const void* xin,
                                                        float scale, float shift, const float* __restrict__ w,
                                                        const float* __restrict__ bias,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps, T* y) {
  constexpr int CPT = COUT / SPLIT;
  static_assert(CPT % 4 == 0 && (SPLIT & (SPLIT - 1)) == 0, "channel split");
  // weights transposed into LDS as [tap][ci][co]: the inner loop reads 4 output channels per
  // ds_read_b128, the same address on every lane of a channel group (broadcast)
  __shared__ __attribute__((aligned(16))) float wl[9 * CIN * COUT];
  {  // every load issued before the first LDS store (a rolled load -> store loop paid one L2 round trip
     // per element: 36 of them per thread in the 16 -> 64 stage)
    constexpr int NWT = 9 * CIN * COUT, PER = (NWT + 255) / 256;
    float tw[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int e = threadIdx.x + 256 * j;
      const int co = e % COUT, ci = (e / COUT) % CIN, tap = e / (COUT * CIN);
      tw[j] = e < NWT ? w[(co * CIN + ci) * 9 + tap] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j)
      if (threadIdx.x + 256 * j < NWT) wl[threadIdx.x + 256 * j] = tw[j];
  }
  __syncthreads();
  const int64_t p = ((int64_t)blockIdx.x * 256 + threadIdx.x) / SPLIT;
  const int c0 = (int)(threadIdx.x % SPLIT) * CPT;
  const int64_t total = (int64_t)O * Ho * Wo;
  // (a pixel's SPLIT lanes are adjacent and 256 % SPLIT == 0: whole pixel groups leave together)
  if (p >= total) return;
  const int ox = (int)(p % Wo);
  const int64_t t = p / Wo;
  const int oy = (int)(t % Ho);
  const int o = (int)(t / Ho);
  float acc[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) acc[c] = bias[c0 + c];
  for (int tap = 0; tap < 9; ++tap) {
    const int iy = 2 * oy - 1 + tap / 3, ix = 2 * ox - 1 + tap % 3;
    if (iy < 0 || iy >= H || ix < 0 || ix >= W) continue;
    const int64_t pix = ((int64_t)o * H + iy) * W + ix;
    float in[CIN];
    if constexpr (LOGIT) {
      const float v = ((const float*)xin)[pix];
      in[0] = to_f32(from_f32<T>(scale / (1.f + expf(-v)) + shift));
    } else {
      const T* xp = (const T*)xin + pix * CIN;
#pragma unroll
      for (int ci = 0; ci < CIN; ++ci) in[ci] = to_f32(xp[ci]);
    }
    const float* wt = wl + tap * CIN * COUT + c0;
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
      for (int c = 0; c < CPT; c += 4) {
        const float4 w4 = *(const float4*)&wt[ci * COUT + c];
        acc[c] += in[ci] * w4.x;
        acc[c + 1] += in[ci] * w4.y;
        acc[c + 2] += in[ci] * w4.z;
        acc[c + 3] += in[ci] * w4.w;
      }
  }
  // the LayerNorm statistics over all COUT channels in channel order, as one thread per pixel sums
  // them (bit-identical to SPLIT = 1): every lane of the pixel gathers the other lanes' channels
  float all[COUT];
  const int lane0 = (threadIdx.x & 63) & ~(SPLIT - 1);
#pragma unroll
  for (int j = 0; j < SPLIT; ++j)
#pragma unroll
    for (int c = 0; c < CPT; ++c) all[j * CPT + c] = SPLIT == 1 ? acc[c] : __shfl(acc[c], lane0 + j, 64);
  float s = 0.f;
#pragma unroll
  for (int co = 0; co < COUT; ++co) s += all[co];
  const float mu = s / COUT;
  float q = 0.f;
#pragma unroll
  for (int co = 0; co < COUT; ++co) q += (all[co] - mu) * (all[co] - mu);
  const float rs = 1.f / sqrtf(q / COUT + eps);
  T* yp = y + p * COUT + c0;
#pragma unroll
  for (int c = 0; c < CPT; c += 4) {
    T r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      r[j] = from_f32<T>(gelu_erf((acc[c + j] - mu) * rs * gamma[c0 + c + j] + beta[c0 + c + j]));
    if constexpr (sizeof(T) == 2) {
      bf16x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = r[j];
      *(bf16x4*)(yp + c) = v;
    } else {
      f32x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = r[j];
      *(f32x4*)(yp + c) = v;
    }
  }
}

template <typename T>
static int mask_down(int O, int H, int W, int cin, int cout, const void* x, int x_logit, float scale, float shift,
                     const float* w, const float* b, const float* g, const float* be, float eps, void* y,
                     hipStream_t st) {
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;  // (H + 2 - 3) / 2 + 1
  const int64_t total = (int64_t)O * Ho * Wo;
  const dim3 grid((unsigned)((total + 255) / 256)), blk(256);
  const dim3 grid4((unsigned)((4 * total + 255) / 256));  // 4 lanes per pixel
  if (cin == 1 && cout == 4 && x_logit)
    hipLaunchKernelGGL((mask_down_kernel<T, 1, 4, true>), grid, blk, 0, st, O, H, W, Ho, Wo, x, scale, shift, w, b, g,
                       be, eps, (T*)y);
  else if (cin == 1 && cout == 4)
    hipLaunchKernelGGL((mask_down_kernel<T, 1, 4, false>), grid, blk, 0, st, O, H, W, Ho, Wo, x, scale, shift, w, b,
                       g, be, eps, (T*)y);
  else if (cin == 4 && cout == 16 && !x_logit)
    hipLaunchKernelGGL((mask_down_kernel<T, 4, 16, false>), grid, blk, 0, st, O, H, W, Ho, Wo, x, scale, shift, w, b,
                       g, be, eps, (T*)y);
  else if (cin == 16 && cout == 64 && !x_logit)
    hipLaunchKernelGGL((mask_down_kernel<T, 16, 64, false, 4>), grid4, blk, 0, st, O, H, W, Ho, Wo, x, scale, shift, w,
                       b, g, be, eps, (T*)y);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

extern "C" int s2h_mask_down_stage(int dt, int O, int H, int W, int cin, int cout, const void* x, int x_logit,
                                   float scale, float shift, const float* w, const float* bias, const float* gamma,
                                   const float* beta, float eps, void* y, hipStream_t st) {
  if (O <= 0 || H <= 0 || W <= 0) return 0;
  if (dt == S2H_BF16)
    return mask_down<bf16>(O, H, W, cin, cout, x, x_logit, scale, shift, w, bias, gamma, beta, eps, y, st);
  return mask_down<float>(O, H, W, cin, cout, x, x_logit, scale, shift, w, bias, gamma, beta, eps, y, st);
}
