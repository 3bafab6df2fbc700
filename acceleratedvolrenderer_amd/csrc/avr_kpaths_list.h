// avr_kpaths_list.h — the k_paths instantiations, as X-macro lists shared by the translation
// units that define them (avr_kpaths.hip, one medium x render mode per unit, built in
// parallel) and the C-ABI unit that declares them (avr_capi.hip, AVR_KP_SPLIT).
// X(emissive, gray, sampler, medium, image, fast); sampler 0 IndependentSampler, 2 / 3
// ZSobolSampler with a 32-bit / 64-bit sample index. RGBGridMedium (medium 4) carries
// per-voxel spectra and has no gray variant.
#pragma once

#define AVR_KP_GRAY_BOTH(X, em, zs, med, im, fa) X(em, false, zs, med, im, fa) X(em, true, zs, med, im, fa)
#define AVR_KP_GRAY_NONE(X, em, zs, med, im, fa) X(em, false, zs, med, im, fa)
#define AVR_KP_VARIANTS_IM(X, G, med, im, fa)                                                          \
    G(X, false, 0, med, im, fa) G(X, true, 0, med, im, fa) G(X, false, 2, med, im, fa) G(X, true, 2, med, im, fa) \
    G(X, false, 3, med, im, fa) G(X, true, 3, med, im, fa)
#define AVR_KP_VARIANTS(X, G, med, fa) AVR_KP_VARIANTS_IM(X, G, med, false, fa) AVR_KP_VARIANTS_IM(X, G, med, true, fa)
// every instantiation of one medium kind and render mode (fa: false replay, true fast)
#define AVR_KP_MEDIUM(X, med, fa) AVR_KP_VARIANTS(X, AVR_KP_GRAY_BOTH, med, fa)
#define AVR_KP_MEDIUM_RGB(X, fa) AVR_KP_VARIANTS(X, AVR_KP_GRAY_NONE, 4, fa)
#define AVR_KP_ALL(X)                                                                                     \
    AVR_KP_MEDIUM(X, 0, false) AVR_KP_MEDIUM(X, 1, false) AVR_KP_MEDIUM(X, 3, false) AVR_KP_MEDIUM_RGB(X, false) \
    AVR_KP_MEDIUM(X, 0, true) AVR_KP_MEDIUM(X, 1, true) AVR_KP_MEDIUM(X, 3, true) AVR_KP_MEDIUM_RGB(X, true)
