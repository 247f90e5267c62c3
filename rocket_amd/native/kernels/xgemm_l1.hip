// Macro-tile GEMM launchers for operand layout 1 (see xgemm_impl.h).
#include "xgemm_impl.h"

RKX_DECLARE(1) { return launch_layout<false, true>(g, cfg, h, a_bytes, b_bytes, num_cus, s); }
