// The bf16 flow kernels for three hidden layers at 32 < k <= 64 (SV, stride 1): flow_v5.hip compiled a third time, by the
// Makefile with -fno-slp-vectorize as flow_v5n.hip but with the compiler's own MFMA register form, in namespace flow5s
// with the entry points suffixed _nh3s (flow_api.hip dispatches those shapes here).  Built in the VGPR form of
// flow_v5n.hip these kernels' gradients moved away from the oracle (SV k = 50 case: weight-gradient error 0.012 ->
// 0.51, profiles/r04/sv_vgpr_form_errs.log) while the k <= 24 kernels' did not; their time did not change (SV step
// 44.4 -> 44.2 ms), so they keep this build.
#define VISSM_FLOW5_NS flow5s
#define VISSM_FLOW5_API(name) name##_nh3s
#include "flow_v5.hip"
