# round-4 session check m: ns_phase neighbour-bin phases shared through LDS (phase_chunk kNb) and the C5 mixed
# launch back on one segment length by default (tail-half = mode 3).  The whole GPU suite first, then ns_phase
# A/B against the library built without the phase change (fft-wavespec_amd/lib/libmtbridge_base.so via
# WSP_MTBRIDGE_LIB, same box, alternating), and C5 once with the new default.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04m
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
ab ns_phase_new '' --config ns_phase
ab ns_phase_base $BASE --config ns_phase
ab ns_phase_new2 '' --config ns_phase
ab ns_phase_base2 $BASE --config ns_phase
ab c5_new '' --config c5
ab c5_tailhalf '' --config c5 --c5-mode group-mixed-tail-half
