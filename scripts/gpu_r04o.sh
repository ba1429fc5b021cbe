# round-4 session check o: C4 top-8 strong-shard segment length (the one-eighth shard's 131072 windows give
# 2048 segments at the policy's floor of 64 -- half the 4096 resident waves): sweep --slide-seg on 1/8 and 1/4
# shards and the full batch.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
b() {  # b <tag> <bench args...>
    local tag=$1; shift
    timeout -k 10 300 python bench.py "$@" --steps 50 --warmup 10 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1])
print('$tag', '%.4f ms'%d['ms_per_step'], '%.4g win/s'%d['value'])"
}
b full --config c4_topk
b s8_auto --config c4_topk --emulate-shard 0/8
for seg in 16 24 32 48 96 128; do b s8_seg$seg --config c4_topk --emulate-shard 0/8 --slide-seg $seg; done
b s4_auto --config c4_topk --emulate-shard 0/4
for seg in 32 64 128; do b s4_seg$seg --config c4_topk --emulate-shard 0/4 --slide-seg $seg; done
b full_seg128 --config c4_topk --slide-seg 128
