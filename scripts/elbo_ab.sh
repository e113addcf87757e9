cd "${GRAFT_REPO_ROOT}"
for r in 1 2; do for L in abl/*.so; do
  VISSM_LIB=$PWD/$L timeout -k 10 200 python bench.py --steps 3 --warmup 1 --cpu-baseline off 2>/dev/null | python -c "
import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$L', round(d['ms_per_step'],2), [(round(s['avg_launch_ms'],3), round(s['frac'],3)) for s in d['streaming_rooflines']])" || exit 1
done; done
