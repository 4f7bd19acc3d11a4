// Workgroup dispatch cost: near-empty kernels over grids of 256-thread workgroups with
// 0 / 32 KiB of LDS, timed with HIP events (20 launches each).  hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>

template <int LDS>
__global__ __launch_bounds__(256) void empty_kernel(float* out) {
  __shared__ float s[LDS / 4 > 0 ? LDS / 4 : 1];
  s[threadIdx.x % (LDS / 4 > 0 ? LDS / 4 : 1)] = threadIdx.x;
  __syncthreads();
  if (threadIdx.x == 0 && s[1] == -1.f) out[blockIdx.x] = s[0];
}

template <int LDS>
static float run(int wgs, float* out) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(empty_kernel<LDS>, dim3(wgs), dim3(256), 0, 0, out);
  hipEventRecord(a);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(empty_kernel<LDS>, dim3(wgs), dim3(256), 0, 0, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1000.f / 20.f;
}

int main() {
  float* out;
  hipMalloc(&out, 1 << 20);
  for (int wgs : {256, 832, 1664, 3328, 6656, 13312, 26624}) {
    printf("wgs %6d  lds0 %7.2f us  lds32K %7.2f us  lds64K %7.2f us\n", wgs, run<0>(wgs, out), run<32768>(wgs, out),
           run<65536>(wgs, out));
  }
  return 0;
}
