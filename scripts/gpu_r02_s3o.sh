#!/bin/bash
# Session 3o: hop = 1 top-k records by the sliding DFT: parity + C4-topk bench (slide vs FFT) + C4/C5 after the refactor.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_slide.py tests/test_gpu_fullgrid.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_slide.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_slide.log
[ $rc -eq 0 ] || { grep -B10 -A40 "Error\|assert" $O/pytest_slide.log | head -120; exit $rc; }
for cfg in "c4_topk slide" "c4_topk fft" "c4 auto" "c5 auto"; do set -- $cfg
timeout -k 10 300 python bench.py --config $1 --algo $2 --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err || { tail -5 $O/bench_$1_$2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_$1_$2.json').read().strip().splitlines()[-1])
print('$1 $2', d['config']['algorithm'], '%.4f ms'%d['ms_per_step'], '%.3g win/s'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done
