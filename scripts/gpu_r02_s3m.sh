#!/bin/bash
# Session 3m: C5 stream layouts (length / greedy by output bytes / greedy by N log N) and stream counts, same box.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3m; mkdir -p $O
for rep in 1 2; do for lay in "length 3" "greedy 3" "nlogn 3" "greedy 2" "greedy 4"; do set -- $lay
tag=${1}_$2_$rep
timeout -k 10 300 python bench.py --config c5 --c5-layout $1 --c5-streams $2 --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -5 $O/bench_$tag.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1])
print('$tag', '%.4f ms'%d['ms_per_step'], 'frac %.3f'%d['roofline']['frac'], d['config']['c5'])"
done; done
