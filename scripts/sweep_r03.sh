#!/bin/bash
# ablation sweep for c4_topk / c5 (round 3); one line per variant
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r03d; mkdir -p $O
b() { local tag=$1; shift; timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || { echo "FAIL $tag"; tail -3 $O/$tag.err; exit 1; }; python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print('%-28s %.4f ms  kernel %.4f'%('$tag', d['ms_per_step'], d['roofline']['kernel_ms']))"; }
b topk_v1 --config c4_topk --variant 1
b topk_v2 --config c4_topk --variant 2
b topk_v3 --config c4_topk --variant 3
b topk_v2_s256 --config c4_topk --variant 2 --slide-seg 256
b topk_v3_s256 --config c4_topk --variant 3 --slide-seg 256
b topk_v3_s512 --config c4_topk --variant 3 --slide-seg 512
b topk_v3_s64 --config c4_topk --variant 3 --slide-seg 64
b c5_st1 --config c5
b c5_st2 --config c5 --c5-streams 2
b c5_st3 --config c5 --c5-streams 3
b c5_st1_s128 --config c5 --slide-seg 128
b c5_st1_s256 --config c5 --slide-seg 256
b c5_st3_s128 --config c5 --c5-streams 3 --slide-seg 128
b c5_st3_s256 --config c5 --c5-streams 3 --slide-seg 256
b c5_plans3 --config c5 --c5-mode plans --c5-streams 3
