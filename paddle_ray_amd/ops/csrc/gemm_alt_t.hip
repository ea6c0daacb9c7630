// TS-schedule GEMM configurations (gemm_core.h kstep_t; dispatcher in gemm_w4.hip).
#include "gemm_alt.h"

namespace pra {
namespace {
using W4T = WCfg<2, 2, 256, 256, true, false, false, true>;  // W4 with the TS schedule
using W8T = WCfg<2, 4, 256, 256, true, false, false, true>;  // W8 with the TS schedule
}  // namespace
}  // namespace pra

PRA_GEMM_ALT_ENTRY(pra_gemm_w4t, pra::W4T)
PRA_GEMM_ALT_ENTRY(pra_gemm_w8t, pra::W8T)
