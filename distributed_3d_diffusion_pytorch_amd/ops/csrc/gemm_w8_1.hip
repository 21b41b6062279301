// gemm_fw_k instantiations: 256 x 256 tile, F_MF (packed, mask-free) epilogues (see gemm_kernel.h).
#include "gemm_kernel.h"

int gemm_dispatch_w8_1(int F, bool deep, const GArgs& a) { return g_dispatch<8>(F, deep, a, GFlagsMF{}); }
