cd "${GRAFT_REPO_ROOT}"
for r in 1 2 3 4; do for L in abl/*.so; do
  echo -n "$L "
  VISSM_LIB=$PWD/$L timeout -k 10 300 python scripts/flow_bench.py --B 65536 --only bf16 --rounds 3 | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['results']['bf16'])"
done; done
