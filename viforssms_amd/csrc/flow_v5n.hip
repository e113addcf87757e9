// The bf16 flow kernels for three hidden layers (LV / SV / FHN heads): flow_v5.hip compiled a second time, by the
// Makefile with -fno-slp-vectorize, in namespace flow5n with the entry points suffixed _nh3 (flow_api.hip
// dispatches the shapes of the two-sample three-layer backward here: LV, FHN, SV).  Without the SLP vectorizer the element-wise work beside the matrix-core chains
// stays in scalar VALU instructions instead of v_pk_fma_f32 / v_pk_mul_f32, which cost more than two scalar ones
// between MFMAs (MI355X_MICROARCH.md, filler prices): LV-cfg backward 18.1 -> 16.8 ms per launch (A/B,
// profiles/r03/ab_misc_r03.log), FHN 3.7 -> 3.5 ms, SV 7.2 -> 6.7 ms; the one-hidden-layer AR kernels (+0.3 ms per
// launch) and the one-sample three-layer backward (SV's k = 50: 10.3 -> 10.8 ms) measured slower that way and keep
// the vectorizer.
#define VISSM_FLOW5_NS flow5n
#define VISSM_FLOW5_API(name) name##_nh3
#include "flow_v5.hip"
