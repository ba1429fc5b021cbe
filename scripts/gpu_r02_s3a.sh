#!/bin/bash
# Session 3a: HEAD check after the container re-creation: -m gpu suite, smoke, driver-style bench.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_ns.json 2> $O/bench_ns.err || { tail -5 $O/bench_ns.err; exit 1; }
cat $O/bench_ns.json
