// MUBUF-DMA (W4B / W8B) and two-barrier early-refill (W4P / W8P) GEMM configurations
// (gemm_core.h; dispatcher in gemm_w4.hip).
#include "gemm_alt.h"

namespace pra {
namespace {
using W4B = WCfg<2, 2, 256, 256, true, true>;         // W4 with MUBUF operand DMA
using W8B = WCfg<2, 4, 256, 256, false, true>;        // W8 (burst schedule) with MUBUF operand DMA
using W4P = WCfg<2, 2, 256, 256, true, false, true>;  // W4 with the two-barrier early-refill schedule
using W8P = WCfg<2, 4, 256, 256, true, false, true>;  // W8 with the two-barrier early-refill schedule
}  // namespace
}  // namespace pra

PRA_GEMM_ALT_ENTRY(pra_gemm_w4b, pra::W4B)
PRA_GEMM_ALT_ENTRY(pra_gemm_w8b, pra::W8B)
PRA_GEMM_ALT_ENTRY(pra_gemm_w4p, pra::W4P)
PRA_GEMM_ALT_ENTRY(pra_gemm_w8p, pra::W8P)
