# round-4 session check n: N = 65536 two-pass with 8-column column workgroups (variant 8, the N = 262144 lever)
# against the fused default and the 16-column two-pass form (variant 1); chunk sweep of variant 8.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
b() {  # b <tag> <bench args...>
    local tag=$1; shift
    timeout -k 10 300 python bench.py "$@" --steps 50 --warmup 10 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1])
print('$tag', '%.4f ms'%d['ms_per_step'], '%.4g win/s'%d['value'])"
}
b large_v0 --config large
b large_v1 --config large --variant 1
b large_v8 --config large --variant 8
b large_v8_c256 --config large --variant 8 --chunk 256
b large_v8_c768 --config large --variant 8 --chunk 768
b large_v8_c1024 --config large --variant 8 --chunk 1024
b large_v8_c4096 --config large --variant 8 --chunk 4096
b large_v0b --config large
b large_v8b --config large --variant 8
