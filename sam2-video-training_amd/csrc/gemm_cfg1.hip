// GEMM tilings, translation unit 1 (see gemm_bf16.h)
#include "gemm_bf16.h"

int gemm_cfg_launch_1(int cfg, GemmArgs16& a, int batch, hipStream_t st) {
  switch (cfg) {
    case CFG_64: return launch_glds<64, 64, 2, 2, 2>(a, batch, st);
    case CFG_64_NS3: return launch_glds<64, 64, 2, 2, 3>(a, batch, st);
    case CFG_64_K32_NS4: return launch_glds<64, 64, 2, 2, 4, 32>(a, batch, st);
    case CFG_64x128: return launch_glds<64, 128, 2, 2, 2>(a, batch, st);
    case CFG_64_NS4: return launch_glds<64, 64, 2, 2, 4>(a, batch, st);
    case CFG_64_K32_NS8: return launch_glds<64, 64, 2, 2, 8, 32>(a, batch, st);
    case CFG_REGS: {  // register-staged kernel (unaligned operands)
      const long t128 = (long)((a.M + 127) / 128) * ((a.N + 127) / 128) * batch;
      if (t128 >= 256 || (a.M >= 128 && a.N >= 128 && a.K >= 1024)) return launch16_regs<128, 128>(a, batch, st);
      return launch16_regs<64, 64>(a, batch, st);
    }
    default: return -1;
  }
}
