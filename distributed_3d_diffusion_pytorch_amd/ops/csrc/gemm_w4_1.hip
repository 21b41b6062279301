// gemm_fw_k instantiations: 128 x 128 tile, F_MF (packed, mask-free) epilogues (see gemm_kernel.h).
#include "gemm_kernel.h"

int gemm_dispatch_w4_1(int F, bool deep, const GArgs& a) { return g_dispatch<4>(F, deep, a, GFlagsMF{}); }
