#!/bin/bash
# Round-2 closing check: -m gpu suite, smoke, the driver's bench line, and one line per configuration.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -B10 -A40 "Error\|assert" $O/pytest_gpu.log | head -120; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
for cfg in north_star c2 c3 c4 c5 c4_topk ns_topk; do
timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -5 $O/bench_$cfg.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_$cfg.json').read().strip().splitlines()[-1])
print('$cfg', d['config']['algorithm'], '%.4f ms'%d['ms_per_step'], '%.4g win/s'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done
python3 -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('default', '%.4f ms'%d['ms_per_step'], '%.4g win/s'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'])"
