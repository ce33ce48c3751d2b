// shade_kernels_bal.hip -- the wave-balanced point-light kernels (shade_tile_kernel BAL 1 and 2, pbr_balanced.h)
// in a translation unit of their own, compiled with the default machine scheduler (shade_kernels.hip, top of
// its launch section, says why). Profiling builds (PBR_BAL_PROFILE) compile them in shade_kernels.hip instead.
#if !(defined(PBR_BAL_PROFILE) && PBR_BAL_PROFILE)
#define PBR_BAL_TU 1
#include "shade_kernels.hip"
#endif
