// Persistent TS GEMM, 4-wave 128x128-per-wave configuration (gemm_pts.h; dispatcher in gemm_lds.hip).
#include "gemm_pts_entry.h"
// dy·Wᵀ and x·W (xᵀ·dy spills at 4 waves: 15-18 VGPRs)
PRA_GEMM_PTS_ENTRY(pra_gemm_pts_w4, pra::W4T, 3)
