// Persistent TS GEMM, 4-wave 128x128-per-wave configuration (gemm_pts.h; dispatcher in gemm_lds.hip).
#include "gemm_pts_entry.h"
// layout 1 (dy·Wᵀ) only: the x·W / xᵀ·dy variants spill at 4 waves
PRA_GEMM_PTS_ENTRY(pra_gemm_pts_w4, pra::W4T, 2)
