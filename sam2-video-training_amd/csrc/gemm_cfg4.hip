// GEMM tilings, translation unit 4 (see gemm_bf16.h)
#include "gemm_bf16.h"

int gemm_cfg_launch_4(int cfg, GemmArgs16& a, int batch, hipStream_t st) {
  switch (cfg) {
    case CFG_256: return launch_glds<256, 256, 2, 4, 2>(a, batch, st);
    case CFG_256x128: return launch_glds<256, 128, 4, 2, 2>(a, batch, st);
    case CFG_256x128_W4_K32_NS3: return launch_glds<256, 128, 2, 2, 3, 32>(a, batch, st);
    case CFG_256x128_W4_K64: return launch_glds<256, 128, 2, 2, 2>(a, batch, st);
    case CFG_256x64_W4_K32_NS3: return launch_glds<256, 64, 4, 1, 3, 32>(a, batch, st);
    default: return -1;
  }
}
