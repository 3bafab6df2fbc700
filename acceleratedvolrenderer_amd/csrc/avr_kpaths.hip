// avr_kpaths.hip — explicit instantiations of the persistent path kernel k_paths for ONE
// medium kind (AVR_KP_MED: 0 GridMedium, 1 Homogeneous/Cloud, 3 NanoVDB, 4 RGBGridMedium)
// and render mode (AVR_KP_FAST: 0 replay, 1 fast). build.py compiles one object per
// (medium, mode) in parallel — the 112 instantiations are most of the library's compile
// time — and links them with avr_capi.hip, which declares them (AVR_KP_SPLIT).
#define AVR_KPATHS_TU   // only the kernels' templates and device helpers, no host-launched kernels
#include "avr_kernels.hip"
#include "avr_kpaths_list.h"

#if !defined(AVR_KP_MED) || !defined(AVR_KP_FAST)
#error "build with -DAVR_KP_MED=<0|1|3|4> -DAVR_KP_FAST=<0|1>"
#endif

namespace avr {
#define AVR_KP_INST(em, gr, zs, med, im, fa) template __global__ void k_paths<em, gr, zs, med, im, fa>(Params);
#if AVR_KP_MED == 4
AVR_KP_MEDIUM_RGB(AVR_KP_INST, (AVR_KP_FAST != 0))
#else
AVR_KP_MEDIUM(AVR_KP_INST, AVR_KP_MED, (AVR_KP_FAST != 0))
#endif
#undef AVR_KP_INST
}  // namespace avr
