// Does the size of a kernel's argument block change its launch cost inside a HIP graph?
// A graph of N back-to-back launches of a small kernel (256 workgroups, each wave loads the first and
// the last 8 bytes of its by-value argument block) per argument size; prints the replay time per
// launch.  Measurement only (round 4: 88 more bytes in GemmArgs16 cost 0.35 ms per bench step).
//   hipcc --offload-arch=gfx950 -O3 tools/kernarg_probe.hip -o tools/bin/kernarg_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

template <int BYTES>
struct Blob {
  long long v[BYTES / 8];
};

template <int BYTES>
__global__ void probe_kernel(Blob<BYTES> b, float* out) {
  // first and last word of the block, so the wave's scalar loads span it
  const long long s = b.v[0] + b.v[BYTES / 8 - 1];
  if (threadIdx.x == 0 && s == 12345) out[blockIdx.x] = 1.f;
}

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));          \
      return 1;                                                         \
    }                                                                   \
  } while (0)

template <int BYTES>
int run(int n, int reps, float* out, hipStream_t st) {
  Blob<BYTES> b{};
  b.v[0] = 1;
  hipGraph_t g;
  hipGraphExec_t ge;
  CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int i = 0; i < n; ++i) hipLaunchKernelGGL(probe_kernel<BYTES>, dim3(256), dim3(256), 0, st, b, out);
  CHECK(hipStreamEndCapture(st, &g));
  CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) CHECK(hipGraphLaunch(ge, st));
  CHECK(hipStreamSynchronize(st));
  std::vector<float> t;
  for (int r = 0; r < reps; ++r) {
    CHECK(hipEventRecord(e0, st));
    CHECK(hipGraphLaunch(ge, st));
    CHECK(hipEventRecord(e1, st));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    t.push_back(ms);
  }
  float best = t[0], sum = 0.f;
  for (float x : t) {
    best = x < best ? x : best;
    sum += x;
  }
  std::printf("arg block %5d B: %7.3f us per launch (best), %7.3f (mean) over %d launches x %d replays\n", BYTES,
              1e3f * best / n, 1e3f * sum / reps / n, n, reps);
  CHECK(hipGraphExecDestroy(ge));
  CHECK(hipGraphDestroy(g));
  return 0;
}

int main() {
  float* out;
  CHECK(hipMalloc(&out, 4096 * sizeof(float)));
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  const int n = 1000, reps = 10;
  int rc = 0;
  for (int pass = 0; pass < 2; ++pass) {
    rc |= run<64>(n, reps, out, st);
    rc |= run<256>(n, reps, out, st);
    rc |= run<320>(n, reps, out, st);
    rc |= run<408>(n, reps, out, st);
    rc |= run<512>(n, reps, out, st);
    rc |= run<1024>(n, reps, out, st);
    rc |= run<2048>(n, reps, out, st);
  }
  CHECK(hipStreamDestroy(st));
  CHECK(hipFree(out));
  return rc;
}
