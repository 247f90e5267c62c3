// Macro-tile GEMM launchers for operand layout 0 (see xgemm_impl.h).
#include "xgemm_impl.h"

RKX_DECLARE(0) { return launch_layout<false, false>(g, cfg, h, a_bytes, b_bytes, num_cus, s); }
