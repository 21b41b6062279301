// gemm_fw_k instantiations: 64 x 64 tile, F_MF (packed, mask-free) epilogues (see gemm_kernel.h).
#include "gemm_kernel.h"

int gemm_dispatch_w2_1(int F, bool deep, const GArgs& a) { return g_dispatch<2>(F, deep, a, GFlagsMF{}); }
