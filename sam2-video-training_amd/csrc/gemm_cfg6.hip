// Full-row bf16 GEMM tilings (gemm_bf16.h CFG_64x256_* / CFG_64x128_*): a workgroup owns 64 rows
// across the whole (<= 256-column) output, four waves of 16 full rows, K <= 256 in flight at once.
#include "gemm_bf16.h"

int gemm_cfg_launch_6_ln(int cfg, GemmArgs16Ln& a, int batch, hipStream_t st) {
  switch (cfg) {
    case CFG_64x256_W41_NS4: return launch_glds<64, 256, 4, 1, 4, 64, GemmArgs16Ln>(a, batch, st);
    case CFG_64x128_W41_NS4: return launch_glds<64, 128, 4, 1, 4, 64, GemmArgs16Ln>(a, batch, st);
    case CFG_64x256_W41_NS3: return launch_glds<64, 256, 4, 1, 3, 64, GemmArgs16Ln>(a, batch, st);
    case CFG_64x256_W41_K32_NS4: return launch_glds<64, 256, 4, 1, 4, 32, GemmArgs16Ln>(a, batch, st);
    default: return -1;
  }
}

// a plain GEMM forced onto a full-row tiling (s2h_gemm_config 25-28): the same kernels, no LayerNorm
int gemm_cfg_launch_6(int cfg, GemmArgs16& a, int batch, hipStream_t st) {
  GemmArgs16Ln l{};
  static_cast<GemmArgs16&>(l) = a;
  return gemm_cfg_launch_6_ln(cfg, l, batch, st);
}
