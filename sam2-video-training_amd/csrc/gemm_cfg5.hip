// GEMM tilings, translation unit 5: 4 x 1 wave grids (gemm_bf16.h).  Each wave computes whole
// 64-column rows of the tile, so the epilogue's 16-B stores cover full 128-B lines of a bf16
// output row (the 2 x 2 grids' 32-column waves write half lines, whose partial-line stores
// dominated the short-K forward GEMMs: tools/gemm_breakdown.py, profiles/r03_v10_*).
#include "gemm_bf16.h"

int gemm_cfg_launch_5(int cfg, GemmArgs16& a, int batch, hipStream_t st) {
  switch (cfg) {
    case CFG_64_W41: return launch_glds<64, 64, 4, 1, 2>(a, batch, st);
    case CFG_128x64_W41: return launch_glds<128, 64, 4, 1, 2>(a, batch, st);
    case CFG_128x64_W41_K32_NS3: return launch_glds<128, 64, 4, 1, 3, 32>(a, batch, st);
    case CFG_64_W41_NS4: return launch_glds<64, 64, 4, 1, 4>(a, batch, st);
    case CFG_128x64_W41_NS3: return launch_glds<128, 64, 4, 1, 3>(a, batch, st);
    default: return -1;
  }
}
