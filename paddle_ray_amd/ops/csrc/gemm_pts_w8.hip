// Persistent TS GEMM, 8-wave 128x64-per-wave configuration (gemm_pts.h; dispatcher in gemm_lds.hip).
#include "gemm_pts_entry.h"
// all layouts
PRA_GEMM_PTS_ENTRY(pra_gemm_pts_w8, pra::W8T, 7)
