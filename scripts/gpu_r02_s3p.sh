#!/bin/bash
# Session 3p: slide top-k segment sweep (C4 top-8) + C5 repeat.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3p; mkdir -p $O
for cfg in "c4_topk 32" "c4_topk 64" "c4_topk 128" "c4_topk 256" "c5 0" "c5 0"; do set -- $cfg
timeout -k 10 300 python bench.py --config $1 --slide-seg $2 --steps 50 --warmup 10 --no-cpu-baseline > $O/bench_$1_$2.json 2> $O/bench_$1_$2.err || { tail -5 $O/bench_$1_$2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_$1_$2.json').read().strip().splitlines()[-1])
print('$1 seg $2', d['config']['algorithm'], '%.4f ms'%d['ms_per_step'], '%.3g win/s'%d['value'])"
done
