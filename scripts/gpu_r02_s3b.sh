#!/bin/bash
# Session 3b: seeded sliding DFT (hop = 1): parity tests, C4/C5 bench slide vs FFT.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_slide.py tests/test_gpu_fullgrid.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_slide.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest_slide.log | tail -15
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest_slide.log | head -80; exit $rc; }
for cfg in c4 c5; do for algo in slide fft; do
timeout -k 10 300 python bench.py --config $cfg --algo $algo --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_${cfg}_$algo.json 2> $O/bench_${cfg}_$algo.err || { tail -5 $O/bench_${cfg}_$algo.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_${cfg}_$algo.json').read().strip().splitlines()[-1])
print('$cfg $algo', d['config']['algorithm'], '%.3f ms'%d['ms_per_step'], '%.3g win/s'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done; done
