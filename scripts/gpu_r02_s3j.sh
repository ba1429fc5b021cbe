#!/bin/bash
# Session 3j: rocprofv3 kernel trace + FETCH/WRITE passes for the HEAD kernels; driver-style bench lines.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02s3j; mkdir -p $O
for cfg in north_star c3 ns_topk; do bash scripts/gpu_profile.sh r02s3j $cfg > $O/prof_$cfg.log 2>&1 || { tail -5 $O/prof_$cfg.log; exit 1; }; grep -A4 '"kernels"' $O/prof_$cfg.log | grep -E "avg_us|void" | head -4; grep hbm_bytes $O/prof_$cfg.log; done
cp profiles/traffic.json $O/traffic.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_ns_20_5.json 2> $O/bench_ns_20_5.err || { tail -5 $O/bench_ns_20_5.err; exit 1; }
cat $O/bench_ns_20_5.json
for cfg in c3 c4 c5; do
timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 20 > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -5 $O/bench_$cfg.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_$cfg.json').read().strip().splitlines()[-1])
print('$cfg', '%.4f ms'%d['ms_per_step'], 'kernel %.4f'%d['roofline']['kernel_ms'], 'frac %.3f'%d['roofline']['frac'], 'traffic', d['roofline']['traffic'])"
done
