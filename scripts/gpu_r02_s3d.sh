#!/bin/bash
# Session 3d: radix-4 seed FFT with LDS twiddles; windows-per-workgroup sweep for C4 / C5.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_slide.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_slide.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_slide.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest_slide.log | head -80; exit $rc; }
sweep() { cfg=$1; shift; for seg in "$@"; do
timeout -k 10 300 python bench.py --config $cfg --slide-seg $seg --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_${cfg}_$seg.json 2> $O/bench_${cfg}_$seg.err || { tail -5 $O/bench_${cfg}_$seg.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_${cfg}_$seg.json').read().strip().splitlines()[-1])
print('$cfg seg $seg', d['config']['algorithm'], '%.3f ms'%d['ms_per_step'], '%.3g win/s'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
done; }
sweep c4 0 128 256 384 512 1024 && sweep c5 0 16 32 64 128
