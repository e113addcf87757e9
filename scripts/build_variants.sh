#!/bin/bash
# Build libvissm.so variants into abl/lib_NAME.so for A/B timing (scripts/ab_libs.sh): each argument is NAME=FLAGS
# (compile-time switches, e.g. nox="-DVISSM_ABL_STORES=1").  Each variant has its own object directory; the
# production library and its objects are not touched (a GPU push taken meanwhile still carries the built library).
# NAME=make:ARGS passes ARGS to make verbatim instead (per-file flags: 'V5_EXTRA=-fno-slp-vectorize EXTRA=-DX').
cd "$(dirname "$0")/.." && mkdir -p abl
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  if [ "${flags#make:}" != "$flags" ]; then margs=(${flags#make:}); else margs=(EXTRA="$flags"); fi
  mkdir -p abl/v_$name && make -C viforssms_amd/csrc -j8 OUTDIR=../../abl/v_$name BUILD=build_abl_$name "${margs[@]}" \
      ../../abl/v_$name/libvissm.so > /dev/null 2>&1 || { echo "build failed: $spec"; exit 1; }
  mv abl/v_$name/libvissm.so "abl/lib_$name.so" && rmdir abl/v_$name; echo "built abl/lib_$name.so ($flags)"
done
