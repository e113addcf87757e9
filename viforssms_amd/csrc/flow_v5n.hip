// The bf16 flow kernels for three hidden layers (LV / SV / FHN heads): flow_v5.hip compiled a second time, by the
// Makefile with -fno-slp-vectorize, in namespace flow5n with the entry points suffixed _nh3 (flow_api.hip
// dispatches the shapes of the two-sample three-layer backward here: LV, FHN, SV).  Without the SLP vectorizer the element-wise work beside the matrix-core chains
// stays in scalar VALU instructions instead of v_pk_fma_f32 / v_pk_mul_f32, which cost more than two scalar ones
// between MFMAs (MI355X_MICROARCH.md, filler prices): LV-cfg backward 18.1 -> 16.8 ms per launch (A/B,
// profiles/r03/ab_misc_r03.log), FHN 3.7 -> 3.5 ms, SV 7.2 -> 6.7 ms; the one-hidden-layer AR kernels (+0.3 ms per
// launch) and the one-sample three-layer backward (SV's k = 50: 10.3 -> 10.8 ms) measured slower that way and keep
// the vectorizer.
// Also built with -mllvm -amdgpu-mfma-vgpr-form=1: with 512 registers per wave the compiler otherwise writes the
// chain's MFMA results (the recompute, dX, dcon) into AGPRs and copies every element back for the element-wise work
// (508 v_accvgpr_read + 215 v_accvgpr_mov of 2021 VALU instructions per pair unit at LV); in the VGPR form, with the
// item-lifetime dW / dW_eps / dW_head accumulators pinned to the AGPRs by inline asm (mfma32_a*, flow_v5.hip), the
// pair unit issues 1535-1685 VALU instructions: LV backward 16.6 -> 14.6 ms per launch, FHN 3.45 -> 3.06 ms
// (profiles/r04/ab_families_vgpr_form.log).
#define VISSM_BWD2N_AACC 1
#define VISSM_FLOW5_NS flow5n
#define VISSM_FLOW5_API(name) name##_nh3
#include "flow_v5.hip"
