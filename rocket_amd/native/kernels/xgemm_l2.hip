// Macro-tile GEMM launchers for operand layout 2 (see xgemm_impl.h).
#include "xgemm_impl.h"

RKX_DECLARE(2) { return launch_layout<true, true>(g, cfg, h, a_bytes, b_bytes, num_cus, s); }
