# round-4 session check u: C5 tail segments, A/B on one box through WSP_MTBRIDGE_LIB (alternating): the default
# (shortest class at S/2 above the floor) against (a) the shortest class at S/4 and (b) the two shortest at S/2.
# The variant libraries are built from the default's sources with that one line changed (not committed).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
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
A=fft-wavespec_amd/lib/libmtbridge_a.so
B=fft-wavespec_amd/lib/libmtbridge_b.so
for i in 1 2; do
    ab c5_default$i '' --config c5
    ab c5_quarter$i $A --config c5
    ab c5_two$i $B --config c5
done
