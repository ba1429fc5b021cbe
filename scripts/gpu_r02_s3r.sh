#!/bin/bash
# Session 3r: seed pass at N/4 threads: parity + C4-topk bench.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_slide.py tests/test_gpu_fullgrid.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_slide.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_slide.log
[ $rc -eq 0 ] || { grep -B10 -A40 "Error\|assert" $O/pytest_slide.log | head -120; exit $rc; }
for seg in 0 128; do
timeout -k 10 300 python bench.py --config c4_topk --slide-seg $seg --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_c4_topk_$seg.json 2> $O/bench_c4_topk_$seg.err || { tail -5 $O/bench_c4_topk_$seg.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c4_topk_$seg.json').read().strip().splitlines()[-1])
print('c4_topk seg $seg', d['config']['algorithm'], '%.4f ms'%d['ms_per_step'], '%.3g win/s'%d['value'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config c4_topk --steps 50 --warmup 10 --no-cpu-baseline > $O/trace.log 2>&1 || exit 1
grep slide $O/trace/run_kernel_stats.csv | cut -c1-160
