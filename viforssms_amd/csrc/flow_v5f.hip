// The fused last AR flow (vissm_flow_ar_elbo_fused): flow_v5.hip compiled once more, in namespace flow5f with the
// entry points suffixed _fz, by the Makefile with LLVM's AMDGPU register-pressure trackers in the scheduler
// (-mllvm -amdgpu-use-amdgpu-trackers=1).  That build runs the fused backward (bwd2_kernel<FZ = true>) 23.42 ->
// 22.74 ms per launch but the other flows' backward slower (first 18.28 -> 18.50 ms, middle 20.57 -> 21.02 ms),
// profiles/r05/ab_sched_strategies.log; flow_api.hip sends only the fused entry points here.  Like flow_v5.o it is
// built without the SLP vectorizer (the f16-derivative products, VISSM_DERIV16).
#define VISSM_FLOW5_NS flow5f
#define VISSM_FLOW5_API(name) name##_fz
#include "flow_v5.hip"
