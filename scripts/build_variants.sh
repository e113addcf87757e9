#!/bin/bash
# Build libvissm.so variants into abl/ for scripts/ab_libs.sh: each argument is NAME=FLAGS
# (compile-time switches, e.g. m3="-DVISSM_BWD_MED3=1"); rebuilds the production library at the end.
cd "$(dirname "$0")/.." && rm -rf abl && mkdir -p abl
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  touch viforssms_amd/csrc/flow_v5.hip viforssms_amd/csrc/flow_v5n.hip viforssms_amd/csrc/flow_api.hip viforssms_amd/csrc/elbo.hip
  make -C viforssms_amd/csrc -j8 EXTRA="$flags" > /dev/null 2>&1 || { echo "build failed: $spec"; exit 1; }
  cp viforssms_amd/libvissm.so "abl/lib_$name.so"; echo "built abl/lib_$name.so ($flags)"
done
touch viforssms_amd/csrc/flow_v5.hip viforssms_amd/csrc/flow_v5n.hip viforssms_amd/csrc/flow_api.hip viforssms_amd/csrc/elbo.hip && make -C viforssms_amd/csrc -j8 > /dev/null 2>&1
