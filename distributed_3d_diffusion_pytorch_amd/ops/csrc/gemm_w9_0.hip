// gemm_fw_k instantiations: 256 x 256 tile on 8 waves (8 x 4 fragments each), plain and concat epilogues (see gemm_kernel.h).
#include "gemm_kernel.h"

int gemm_dispatch_w9_0(int F, bool deep, const GArgs& a) { return g_dispatch<9>(F, deep, a, GFlagsPlain{}); }
