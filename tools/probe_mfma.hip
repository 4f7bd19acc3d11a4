// Layout probe (GPU box): checks the register layouts the flash-attention kernels assume for
// v_mfma_f32_32x32x16_bf16, ds_read_b64_tr_b16 and global_load_lds.  Prints PASS/FAIL lines.
//   hipcc --offload-arch=gfx950 -O3 tools/probe_mfma.hip -o /tmp/probe && /tmp/probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short v4i16 __attribute__((ext_vector_type(4)));

__global__ void mfma32(const float* A, const float* B, float* C) {
  // A [32][16], B [16][32] row-major fp32 (exact in bf16: small integers)
  const int l = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (__bf16)A[(l & 31) * 16 + 8 * (l >> 5) + j];
    b[j] = (__bf16)B[(8 * (l >> 5) + j) * 32 + (l & 31)];
  }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    const int row = 8 * (r >> 2) + 4 * (l >> 5) + (r & 3), col = l & 31;
    C[row * 32 + col] = acc[r];
  }
}

__global__ void trread(const short* src, short* out) {
  // 8 rows x 32 cols of shorts in LDS; each 16-lane group reads rows 4*(g&1).., cols 16*(g>>1)..
  __shared__ short t[8 * 32];
  for (int i = threadIdx.x; i < 256; i += 64) t[i] = src[i];
  __syncthreads();
  const int l = threadIdx.x, g = l >> 4, q = (l >> 2) & 3, p = l & 3;
  const short* a = t + (4 * (g & 1) + q) * 32 + 16 * (g >> 1) + 4 * p;
  v4i16 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16*)a);
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}

__global__ void glds(const int4* src, int* out) {
  __shared__ int4 lds[128];
  for (int i = threadIdx.x; i < 128; i += 64) lds[i] = make_int4(-1, -1, -1, -1);
  __syncthreads();
  __builtin_amdgcn_global_load_lds((const void*)(src + 63 - threadIdx.x), (__attribute__((address_space(3))) void*)(lds + 32), 16, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  for (int i = threadIdx.x; i < 128; i += 64) out[i] = lds[i].x;
}

int main() {
  std::vector<float> A(32 * 16), B(16 * 32), C(32 * 32), R(32 * 32, 0.f);
  for (int i = 0; i < 32 * 16; ++i) A[i] = (float)((i * 7) % 5 - 2);
  for (int i = 0; i < 16 * 32; ++i) B[i] = (float)((i * 3) % 7 - 3);
  for (int r = 0; r < 32; ++r)
    for (int c = 0; c < 32; ++c)
      for (int k = 0; k < 16; ++k) R[r * 32 + c] += A[r * 16 + k] * B[k * 32 + c];
  float *dA, *dB, *dC;
  hipMalloc(&dA, 4 * A.size()); hipMalloc(&dB, 4 * B.size()); hipMalloc(&dC, 4 * C.size());
  hipMemcpy(dA, A.data(), 4 * A.size(), hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), 4 * B.size(), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(mfma32, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  hipMemcpy(C.data(), dC, 4 * C.size(), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 32 * 32; ++i) bad += C[i] != R[i];
  printf("mfma_f32_32x32x16_bf16 layout: %s (%d mismatches)\n", bad ? "FAIL" : "PASS", bad);

  std::vector<short> S(256), O(256);
  for (int i = 0; i < 256; ++i) S[i] = (short)i;
  short *dS, *dO;
  hipMalloc(&dS, 512); hipMalloc(&dO, 512);
  hipMemcpy(dS, S.data(), 512, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(trread, dim3(1), dim3(64), 0, 0, dS, dO);
  hipMemcpy(O.data(), dO, 512, hipMemcpyDeviceToHost);
  bad = 0;
  for (int l = 0; l < 64; ++l) {
    const int g = l >> 4, i = l & 15;
    for (int e = 0; e < 4; ++e) bad += O[l * 4 + e] != S[(4 * (g & 1) + e) * 32 + 16 * (g >> 1) + i];
  }
  printf("ds_read_b64_tr_b16 layout: %s (%d mismatches)\n", bad ? "FAIL" : "PASS", bad);

  std::vector<int> G(64 * 4), GO(128);
  for (int i = 0; i < 64; ++i) G[4 * i] = i;
  int *dG, *dGO;
  hipMalloc(&dG, 4 * G.size()); hipMalloc(&dGO, 4 * GO.size());
  hipMemcpy(dG, G.data(), 4 * G.size(), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(glds, dim3(1), dim3(64), 0, 0, (const int4*)dG, dGO);
  hipMemcpy(GO.data(), dGO, 4 * GO.size(), hipMemcpyDeviceToHost);
  bad = 0;
  for (int i = 0; i < 128; ++i) {
    const int want = (i >= 32 && i < 96) ? 63 - (i - 32) : -1;
    bad += GO[i] != want;
  }
  printf("global_load_lds lane-linear destination: %s (%d mismatches)\n", bad ? "FAIL" : "PASS", bad);
  return 0;
}
