// Per-object MLP heads in one launch (round 4): the SAM2 heads that run under no_grad on the
// objects' tokens -- the object-score head (mask_decoder.py:234-238, MLP 256 -> 256 -> 256 -> 1) and
// the object-pointer projection (sam2_base.py:296-305 obj_ptr_proj, MLP 256 -> 256 -> 256 -> 256) --
// were 3 + 3 GEMM launches of 13 rows each per frame.  Here one workgroup carries 16 rows of one head
// through all of its layers: the activation rows stay in LDS between layers, each wave computes
// 16-column output tiles with 16x16x32 MFMAs whose weight fragments are loaded straight from global
// memory (lane l: output column l & 15, k 32 ks + 8 (l >> 4)), and the bias / activation / bf16
// rounding follow every layer exactly as the GEMM epilogue does -- so the outputs are bit-identical
// to the per-layer GEMMs (same K order per output element, same epilogue arithmetic).
#include "common.h"

namespace {

constexpr int HD_MAXH = 4;    // heads per launch
constexpr int HD_MAXL = 3;    // layers per head
constexpr int HD_MAXK = 256;  // widest layer input / output
constexpr int HD_LD = HD_MAXK + 8;  // LDS activation row (bf16), padded: conflict-free b128 reads

struct HeadDesc {
  const bf16* x;  // [M, dims[0]] rows, row stride ldx
  int64_t ldx;
  const bf16* w[HD_MAXL];     // [dims[l + 1], dims[l]] row-major (the Linear weight)
  const float* b[HD_MAXL];    // [dims[l + 1]] or null
  int dims[HD_MAXL + 1];
  int nl;        // layers
  int act_last;  // S2HAct of the last layer (the hidden layers are ReLU)
  bf16* y;       // [M, dims[nl]], row stride ldy
  int64_t ldy;
  bf16* hid[HD_MAXL - 1];  // optional [M, dims[l + 1]] hidden outputs (after ReLU), contiguous rows
  bf16* pre;               // optional [M, dims[nl]] last layer's pre-activation, contiguous rows
};

struct HeadsArgs {
  HeadDesc h[HD_MAXH];
  int nheads, M;
};

typedef __attribute__((ext_vector_type(8))) __bf16 hd_bf16x8;
typedef __attribute__((ext_vector_type(4))) float hd_f32x4;

// 16 waves: wave w owns output columns 16w .. 16w + 15 of every layer (widths <= 256), and loads ALL
// of its weight fragments for all layers at kernel start -- they do not depend on the activations --
// so the head costs one global round trip plus three LDS exchanges (the first form, 4 waves looping
// over tiles with a load before every MFMA, was slower than the 6 GEMM launches it replaced)
__global__ __launch_bounds__(1024) void mlp_heads_kernel(HeadsArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 act[2][16 * HD_LD];
  const HeadDesc& d = a.h[blockIdx.y];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r0 = blockIdx.x * 16;
  const int nl = d.nl;
  const int n = 16 * w + (lane & 15);
  hd_bf16x8 bfr[HD_MAXL][HD_MAXK / 32];
#pragma unroll
  for (int l = 0; l < HD_MAXL; ++l) {
    const int K = l < nl ? d.dims[l] : 0, N = l < nl ? d.dims[l + 1] : 0;
    const bf16* W = d.w[l];
#pragma unroll
    for (int ks = 0; ks < HD_MAXK / 32; ++ks) {
      const int k = 32 * ks + 8 * (lane >> 4);
      bfr[l][ks] = (n < N && k < K) ? *(const hd_bf16x8*)(W + (int64_t)n * K + k) : hd_bf16x8{};
    }
  }
  // layer-0 input rows (rows past M and columns past K zero), 8 columns per thread
  {
    const int K0 = d.dims[0];
    if (tid < 16 * (HD_MAXK / 8)) {
      const int r = tid / (HD_MAXK / 8), c = (tid % (HD_MAXK / 8)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (r0 + r < a.M && c < K0) v = *(const uint4*)(d.x + (int64_t)(r0 + r) * d.ldx + c);
      *(uint4*)(act[0] + r * HD_LD + c) = v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int l = 0; l < HD_MAXL; ++l) {
    if (l < nl) {
      const int K = d.dims[l], N = d.dims[l + 1];
      const bool last = l == nl - 1;
      const int act_fn = last ? d.act_last : S2H_ACT_RELU;
      const bf16* in = act[l & 1];
      bf16* out = act[(l & 1) ^ 1];
      if (16 * w < N) {
        hd_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < HD_MAXK / 32; ++ks) {
          if (32 * ks < K) {
            const hd_bf16x8 af = *(const hd_bf16x8*)(in + (lane & 15) * HD_LD + 32 * ks + 8 * (lane >> 4));
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[l][ks], acc, 0, 0, 0);
          }
        }
        // lane holds rows 4 (lane >> 4) + e of column n
        const float bn = (d.b[l] != nullptr && n < N) ? d.b[l][n] : 0.f;
        bf16* hid = last ? nullptr : d.hid[l];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * (lane >> 4) + e;
          const float pv = acc[e] + bn;
          const bf16 v = (bf16)apply_act(pv, act_fn);
          if (n < N) {
            out[r * HD_LD + n] = v;
            if (r0 + r < a.M) {
              if (last) {
                d.y[(int64_t)(r0 + r) * d.ldy + n] = v;
                if (d.pre) d.pre[(int64_t)(r0 + r) * N + n] = (bf16)pv;
              } else if (hid) {
                hid[(int64_t)(r0 + r) * N + n] = v;
              }
            }
          }
        }
      }
      // columns [N, N rounded up to 32) of the next layer's input read as zero
      if (!last && tid < 16 * 32) {
        const int r = tid / 32, c = N + tid % 32;
        if (c < ((N + 31) / 32) * 32) out[r * HD_LD + c] = (bf16)0.f;
      }
      __syncthreads();
    }
  }
}

}  // namespace

// heads[h]: x [M, dims[h*4]] (row stride ldx[h]), weights w[h*3 + l] [dims[h*4+l+1], dims[h*4+l]],
// biases b[h*3 + l] (fp32 or null), nl[h] layers (<= 3; hidden layers ReLU, the last act_last[h]),
// y [M, dims[h*4 + nl]] (row stride ldy[h]); bf16; every width <= 256 and a multiple of 8 (the last
// may be any width <= 256); 16-B aligned rows.
// hid (optional, may be NULL): hid[2h + l] receives layer l's output (after ReLU, [M, dims[4h+l+1]]
// contiguous) for l < nl - 1; pre (optional): pre[h] the last layer's pre-activation [M, dims[4h+nl]] --
// what the backward of a trained head reads (tape op frametape.mlp_heads)
extern "C" int s2h_mlp_heads(int nheads, int M, const void* const* x, const int64_t* ldx, const void* const* w,
                             const float* const* b, const int* dims, const int* nl, const int* act_last,
                             void* const* y, const int64_t* ldy, void* const* hid, void* const* pre,
                             hipStream_t st) {
  if (M <= 0 || nheads <= 0) return 0;
  if (nheads > HD_MAXH) return (int)hipErrorInvalidValue;
  HeadsArgs a = {};
  a.nheads = nheads;
  a.M = M;
  for (int h = 0; h < nheads; ++h) {
    HeadDesc& d = a.h[h];
    d.nl = nl[h];
    if (d.nl < 1 || d.nl > HD_MAXL || !x[h] || !y[h] || ((uintptr_t)x[h] & 15) || ldx[h] % 8)
      return (int)hipErrorInvalidValue;
    d.x = (const bf16*)x[h];
    d.ldx = ldx[h];
    d.y = (bf16*)y[h];
    d.ldy = ldy[h];
    d.act_last = act_last[h];
    for (int l = 0; l <= d.nl; ++l) {
      d.dims[l] = dims[h * (HD_MAXL + 1) + l];
      if (d.dims[l] <= 0 || d.dims[l] > HD_MAXK || (l < d.nl && d.dims[l] % 8)) return (int)hipErrorInvalidValue;
    }
    for (int l = 0; l < HD_MAXL - 1; ++l) d.hid[l] = hid ? (bf16*)hid[h * (HD_MAXL - 1) + l] : nullptr;
    d.pre = pre ? (bf16*)pre[h] : nullptr;
    for (int l = 0; l < d.nl; ++l) {
      d.w[l] = (const bf16*)w[h * HD_MAXL + l];
      d.b[l] = b[h * HD_MAXL + l];
      if (!d.w[l] || ((uintptr_t)d.w[l] & 15)) return (int)hipErrorInvalidValue;
    }
  }
  hipLaunchKernelGGL(mlp_heads_kernel, dim3((M + 15) / 16, nheads), dim3(1024), 0, st, a);
  return (int)hipGetLastError();
}
