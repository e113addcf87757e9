#!/bin/bash
# Build the phase-ablation variants of libvissm.so (compile-time mask, flow_v5.hip kAbl) into
# abl_mask/ for scripts/gpu_ablate.sh; rebuilds the production library at the end.
cd "$(dirname "$0")/.." && mkdir -p abl_mask
for A in 1 2 4 8 16 31; do
  touch viforssms_amd/csrc/flow_v5.hip
  make -C viforssms_amd/csrc -j8 EXTRA=-DVISSM_V5_ABLATE=$A > /dev/null && cp viforssms_amd/libvissm.so abl_mask/lib_abl$A.so
done
touch viforssms_amd/csrc/flow_v5.hip && make -C viforssms_amd/csrc -j8 > /dev/null
