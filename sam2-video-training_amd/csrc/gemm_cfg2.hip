// GEMM tilings, translation unit 2 (see gemm_bf16.h)
#include "gemm_bf16.h"

int gemm_cfg_launch_2(int cfg, GemmArgs16& a, int batch, hipStream_t st) {
  switch (cfg) {
    case CFG_128x64: return launch_glds<128, 64, 2, 2, 2>(a, batch, st);
    case CFG_128x64_K32_NS3: return launch_glds<128, 64, 2, 2, 3, 32>(a, batch, st);
    case CFG_128x64_K32_NS4: return launch_glds<128, 64, 2, 2, 4, 32>(a, batch, st);
    case CFG_128x64_NS3: return launch_glds<128, 64, 2, 2, 3>(a, batch, st);
    default: return -1;
  }
}
