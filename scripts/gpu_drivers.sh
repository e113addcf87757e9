#!/bin/bash
# The drop-in drivers run a few steps on the GPU (pre-training + ELBO steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
D=$(mktemp -d); cp -r dat hyperparameters.txt $D/ 2>/dev/null; chmod -R u+w $D; R=$PWD
run() { echo "== $*"; (cd $D && timeout -k 10 300 python "$@" > $R/gpurun_out/drv.log 2>&1); rc=$?; tail -3 $R/gpurun_out/drv.log | cut -c1-300; [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }; }
run $R/main.py hyperparameters.txt --steps 30
run $R/main.py hyperparameters.txt --steps 8 --precision bf16 --no-pretrain
run $R/lotka_volterra_partial.py --steps 6 --no-pretrain
run $R/SV_dense.py --steps 6
run $R/fitz_nag_NVP.py --steps 6 --train --T 400 --no-pretrain
