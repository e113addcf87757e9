#!/bin/bash
# A/B of the forward kernels in 8-wave blocks (weights from LDS): bf16x2 flow forward and bf16x2f step (lib c), LV /
# FHN steps (lib d) against lib a, and the bf16x2 parity cases on lib c
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
IMPL=bf16x2 ROUNDS=2 bash scripts/ab_libs.sh > gpurun_out/ab_x2fwd_flow.log 2>&1; cat gpurun_out/ab_x2fwd_flow.log
EXTRA="--precision bf16x2f" ROUNDS=1 STEPS=6 bash scripts/ab_step.sh abl/lib_a_base.so abl/lib_c_x2nw8.so > gpurun_out/ab_x2fwd_step.log 2>&1; cat gpurun_out/ab_x2fwd_step.log
MODELS="lv fhn" ROUNDS=1 bash scripts/ab_families.sh abl/lib_a_base.so abl/lib_d_n3nw8.so > gpurun_out/ab_n3fwd.log 2>&1; cat gpurun_out/ab_n3fwd.log
VISSM_LIB=$PWD/abl/lib_c_x2nw8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_config_parity.py tests/test_gpu_fused.py -k "bf16x2" -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_x2nw8.log 2>&1; tail -3 gpurun_out/pytest_x2nw8.log
ROUNDS=1 STEPS=8 bash scripts/ab_step.sh abl/lib_a_base.so abl/lib_e_n1nw8.so > gpurun_out/ab_n1fwd_step.log 2>&1; cat gpurun_out/ab_n1fwd_step.log
