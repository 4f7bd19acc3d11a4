// GEMM tilings, translation unit 3 (see gemm_bf16.h)
#include "gemm_bf16.h"

int gemm_cfg_launch_3(int cfg, GemmArgs16& a, int batch, hipStream_t st) {
  switch (cfg) {
    case CFG_128: return launch_glds<128, 128, 2, 2, 2>(a, batch, st);
    case CFG_128_NS3: return launch_glds<128, 128, 2, 2, 3>(a, batch, st);
    case CFG_128_K32_NS3: return launch_glds<128, 128, 2, 2, 3, 32>(a, batch, st);
    case CFG_128x256: return launch_glds<128, 256, 2, 4, 2>(a, batch, st);
    default: return -1;
  }
}
