# round-4 session check i: packed fp32 complex arithmetic in the spectrum kernel (C3's fp32 spectrum pass is
# VALU-issue-bound).  The whole GPU suite first, then C3 A/B against the library built without the change
# (fft-wavespec_amd/lib/libmtbridge_base.so via WSP_MTBRIDGE_LIB, same box, alternating),
# and the SQ pass over C3 with the new library (VALU issue after; profiles/r04/sq/c3_sq_counters.csv is before).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
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
ab c3_new '' --config c3
ab c3_base $BASE --config c3
ab c3_new2 '' --config c3
ab c3_base2 $BASE --config c3
bash scripts/gpu_run.sh r04i sq=c3,SQ_WAIT_ANY,SQ_INSTS_VALU,SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_LDS,SQ_WAIT_INST_ANY \
    prof=c3
