# Same-box A/B of the settle phase at the driver's settings: bench.py --steps 20 --warmup 5 with and without it.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r03settle; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/settle_$r.json 2> $O/s$r.err || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-settle > $O/nosettle_$r.json 2> $O/n$r.err || exit 1
done
for f in $O/*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', '%.4f ms'%d['ms_per_step'], 'frac %.3f'%d['roofline']['frac'], d.get('settle'))"; done
