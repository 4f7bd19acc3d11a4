// Short-K tilings with A in registers (gemm_bf16.h gemm16a_kernel, CFG_64_AREG / CFG_64x128_AREG).
#include "gemm_bf16.h"

int gemm_cfg_launch_7(int cfg, GemmArgs16& a, int batch, hipStream_t st) {
  if (cfg != CFG_64_AREG && cfg != CFG_64x128_AREG) return -1;
  if (!gemm_areg_ok(a, 256)) return -1;  // a forced tiling the shape cannot take: the caller's default
  return cfg == CFG_64_AREG ? launch_areg<64>(a, batch, st) : launch_areg<128>(a, batch, st);
}
