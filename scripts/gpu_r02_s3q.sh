#!/bin/bash
# Session 3q: HEAD check: full -m gpu suite, smoke, driver-style bench; rocprof trace of c4_topk (slide) and c4/c5.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3q; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -B10 -A40 "Error\|assert" $O/pytest_gpu.log | head -120; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_ns.json 2> $O/bench_ns.err || { tail -5 $O/bench_ns.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_ns.json').read().strip().splitlines()[-1])
print('north_star', '%.4f ms'%d['ms_per_step'], '%.4g win/s'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4_topk -o run -- python3 bench.py --config c4_topk --steps 50 --warmup 10 --no-cpu-baseline > $O/trace_c4_topk.log 2>&1 || exit 1
grep slide $O/trace_c4_topk/run_kernel_stats.csv | cut -c1-160
