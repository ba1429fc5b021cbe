#!/bin/bash
# Round-3 ablation sweeps, one bench line per variant (50 timed steps after 10 warm-up):
#   gpurun -- bash scripts/sweep_r03.sh <tag> [topk] [c5] [large] [c3]
#   topk   hop = 1 top-8 records (C4 shape): scan forms (default probe threshold, --variant 1 one-wave,
#          2 / 3 transposed 16 / 8 windows per batch) x segment lengths
#   c5     grouped plan: internal streams x segment lengths; the per-symbol plans (round-2 form)
#   large  4096 x 65536: two-pass (default), pipelined quarter chunks on two streams (--variant 2), fused
#          one-workgroup-per-window (--variant 3); 1024 x 262144 (two-pass)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
b() {
    local tag=$1; shift
    timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu-baseline "$@" > $O/$tag.json 2> $O/$tag.err || {
        echo "FAIL $tag"; tail -3 $O/$tag.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1])
print('%-28s %.4f ms  kernel %.4f  frac %.3f' % ('$tag', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac']))"
}
for what in "$@"; do
    case $what in
    topk)
        for sg in 128 256 512 1024; do b topk_v0_s$sg --config c4_topk --slide-seg $sg; done
        b topk_v1 --config c4_topk --variant 1
        for v in 2 3; do for sg in 128 512; do b topk_v${v}_s$sg --config c4_topk --variant $v --slide-seg $sg; done; done
        ;;
    c5)
        b c5_st1 --config c5
        b c5_st3 --config c5 --c5-streams 3
        b c5_st3_s256 --config c5 --c5-streams 3 --slide-seg 256
        b c5_st1_s256 --config c5 --slide-seg 256
        b c5_plans3 --config c5 --c5-mode plans --c5-streams 3
        ;;
    large)
        b large_v0 --config large
        b large_v2 --config large --variant 2
        b large_v3 --config large --variant 3
        b large262k --config large_262144
        ;;
    c3)
        b c3 --config c3
        ;;
    esac
done
