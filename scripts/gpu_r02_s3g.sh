#!/bin/bash
# Session 3g: two bins per thread for N <= 1024: parity + C5 bench (3 runs) + segment sweep.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_slide.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_slide.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_slide.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest_slide.log | head -80; exit $rc; }
for seg in 0 0 0 16 48 64; do
timeout -k 10 300 python bench.py --config c5 --slide-seg $seg --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_c5_$seg.json 2> $O/bench_c5_$seg.err || { tail -5 $O/bench_c5_$seg.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c5_$seg.json').read().strip().splitlines()[-1])
print('c5 seg $seg', d['config']['algorithm'], '%.3f ms'%d['ms_per_step'], '%.3g win/s'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config c5 --steps 50 --warmup 10 --no-cpu-baseline > $O/trace.log 2>&1 && grep slide_kernel $O/trace/*/run_kernel_stats.csv $O/trace/run_kernel_stats.csv 2>/dev/null | cut -c1-200
true
timeout -k 10 120 fft-wavespec_amd/bin/kbench store 20 4 > $O/kbench_store.log 2>&1; cat $O/kbench_store.log
