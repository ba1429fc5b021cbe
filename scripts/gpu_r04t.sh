# round-4 session check t: C5's default now halves the shortest class's segments only above the segment floor
# (large batches).  Group tests, then the full batch and the 1/8 and 6/8 shards: default vs mode 4 (one length).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_slide.py tests/test_gpu_fullgrid.py -m gpu -q -p no:cacheprovider -k "group or c5" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
b() {  # b <tag> <bench args...>
    local tag=$1; shift
    timeout -k 10 300 python bench.py "$@" --steps 100 --warmup 20 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1])
print('$tag', '%.4f ms'%d['ms_per_step'], '%.4g win/s'%d['value'])"
}
b c5_auto --config c5
b c5_uniform --config c5 --c5-mode group-mixed-uniform
b c5_auto2 --config c5
b c5_uniform2 --config c5 --c5-mode group-mixed-uniform
b s18_auto --config c5 --emulate-shard 1/8
b s18_uniform --config c5 --emulate-shard 1/8 --c5-mode group-mixed-uniform
b s68_auto --config c5 --emulate-shard 6/8
b s68_uniform --config c5 --emulate-shard 6/8 --c5-mode group-mixed-uniform
b s02_auto --config c5 --emulate-shard 0/2
b s02_uniform --config c5 --emulate-shard 0/2 --c5-mode group-mixed-uniform
