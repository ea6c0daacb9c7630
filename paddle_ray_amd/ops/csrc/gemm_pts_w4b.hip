// Persistent TS GEMM, 4-wave configuration with MUBUF LDS-DMA (buffer_load_dwordx4 ... lds
// instead of global_load_lds_dwordx4); selected by PRA_PTS_BUF=1 (gemm_lds.hip).
#include "gemm_pts_entry.h"
namespace pra {
namespace {
using W4TB = WCfg<2, 2, 256, 256, true, true, false, true>;
}
}  // namespace pra
PRA_GEMM_PTS_ENTRY(pra_gemm_pts_w4b, pra::W4TB, 3)
