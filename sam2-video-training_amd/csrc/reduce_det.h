// Deterministic column reduction of per-workgroup partial rows (round 5): the second pass of the
// kernels that used to add their workgroup sums with float atomics (column sums, loss statistics).
//
//   out[b][i] (+)= sum_{r < nr} part[b][r][i]
//
// One 256-thread workgroup covers 256 / SL columns x SL row slices: slice s sums rows s, s + SL, ...
// with eight independent chains (eight loads in flight per thread), the SL slice sums are added in a
// fixed tree through LDS.  Every assignment is fixed by the launch shape, so the result does not
// depend on timing; SL grows as the columns get few, so the rows are read by enough threads.
#pragma once
#include "common.h"

template <int SL>
__global__ __launch_bounds__(256) void det_colsum_kernel(int nr, int n, const float* part, float* out, int accumulate) {
  constexpr int CPB = 256 / SL;
  __shared__ float red[SL][CPB];
  const int c = threadIdx.x % CPB, sl = threadIdx.x / CPB;
  const int col = blockIdx.x * CPB + c;
  const int b = blockIdx.y;
  part += (int64_t)b * nr * n;
  float ch[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col < n) {
    int r = sl;
    for (; r + 7 * SL < nr; r += 8 * SL) {
#pragma unroll
      for (int q = 0; q < 8; ++q) ch[q] += part[(int64_t)(r + q * SL) * n + col];
    }
#pragma unroll
    for (int q = 0; q < 7; ++q)  // static indices (a dynamic index would put ch[] in scratch)
      if (r + q * SL < nr) ch[q] += part[(int64_t)(r + q * SL) * n + col];
  }
  red[sl][c] = ((ch[0] + ch[1]) + (ch[2] + ch[3])) + ((ch[4] + ch[5]) + (ch[6] + ch[7]));
  __syncthreads();
#pragma unroll
  for (int h = SL / 2; h >= 1; h >>= 1) {
    if (sl < h) red[sl][c] += red[sl + h][c];
    __syncthreads();
  }
  if (sl == 0 && col < n) {
    float* o = out + (int64_t)b * n + col;
    *o = accumulate ? *o + red[0][c] : red[0][c];
  }
}

// out[b][:] (+)= the nr partial rows of batch b; B batches of n columns
static inline void det_colsum(int B, int nr, int n, const float* part, float* out, int accumulate, hipStream_t st) {
  const int64_t cols = (int64_t)B * n;
  int sl = cols <= 2048 ? 16 : cols <= 8192 ? 8 : cols <= 32768 ? 4 : 1;
  while (sl > 1 && sl > nr) sl >>= 1;
  const int cpb = 256 / sl;
  const dim3 g((n + cpb - 1) / cpb, B);
  switch (sl) {
    case 16: hipLaunchKernelGGL(det_colsum_kernel<16>, g, dim3(256), 0, st, nr, n, part, out, accumulate); break;
    case 8: hipLaunchKernelGGL(det_colsum_kernel<8>, g, dim3(256), 0, st, nr, n, part, out, accumulate); break;
    case 4: hipLaunchKernelGGL(det_colsum_kernel<4>, g, dim3(256), 0, st, nr, n, part, out, accumulate); break;
    case 2: hipLaunchKernelGGL(det_colsum_kernel<2>, g, dim3(256), 0, st, nr, n, part, out, accumulate); break;
    default: hipLaunchKernelGGL(det_colsum_kernel<1>, g, dim3(256), 0, st, nr, n, part, out, accumulate); break;
  }
}
