#!/bin/bash
# Session 3f: sliding DFT with plain stores: parity, C4/C5 bench, rocprof C4/C5 + FFT ablations.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_slide.py tests/test_gpu_fullgrid.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_slide.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_slide.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest_slide.log | head -80; exit $rc; }
for cfg in c4 c5; do
timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 20 > $O/bench_${cfg}.json 2> $O/bench_${cfg}.err || { tail -5 $O/bench_${cfg}.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_${cfg}.json').read().strip().splitlines()[-1])
print('$cfg', d['config']['algorithm'], '%.3f ms'%d['ms_per_step'], '%.3g win/s'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done
for cfg in c4 c5; do bash scripts/gpu_profile.sh r02s3f $cfg > $O/prof_$cfg.log 2>&1 || { tail -5 $O/prof_$cfg.log; exit 1; }; grep -A4 '"kernels"' $O/prof_$cfg.log | head -6; grep hbm_bytes $O/prof_$cfg.log; done
cp profiles/traffic.json $O/traffic.json
