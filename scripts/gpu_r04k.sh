# round-4 session check k: the hop = 1 top-k probe minimum by scalar readlanes over the slot's probe lanes
# instead of a 64-lane DPP / permlane min.  Top-k tests first, then C4 top-8 A/B against the library built
# without the change (WSP_MTBRIDGE_LIB=fft-wavespec_amd/lib/libmtbridge_base.so), alternating on one box.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_slide.py tests/test_gpu_fullgrid.py -k "topk" -v -m gpu -p no:cacheprovider \
    --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
ab() {  # ab <tag> <lib or ''> <bench args...>
    local tag=$1 lib=$2; shift 2
    if [ -n "$lib" ]; then
        WSP_MTBRIDGE_LIB=$lib timeout -k 10 300 python bench.py "$@" --steps 100 --warmup 20 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || exit $?
    else
        timeout -k 10 300 python bench.py "$@" --steps 100 --warmup 20 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || exit $?
    fi
    python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1])
print('$tag', '%.4f ms'%d['ms_per_step'], '%.4g win/s'%d['value'])"
}
BASE=fft-wavespec_amd/lib/libmtbridge_base.so
ab c4_topk_new '' --config c4_topk
ab c4_topk_base $BASE --config c4_topk
ab c4_topk_new2 '' --config c4_topk
ab c4_topk_base2 $BASE --config c4_topk
ab c3_new '' --config c3
ab c3_base $BASE --config c3
