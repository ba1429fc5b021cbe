#!/bin/bash
# Session 3n: compile-time nt loads for the phase outputs: parity (phase tests) + ns_phase / ns_topk_phase / inverse bench.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullgrid.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -80; exit $rc; }
for cfg in ns_phase ns_topk_phase north_star ns_topk; do
timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -5 $O/bench_$cfg.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_$cfg.json').read().strip().splitlines()[-1])
print('$cfg', '%.4f ms'%d['ms_per_step'], 'frac %.3f'%d['roofline']['frac'])"
done
