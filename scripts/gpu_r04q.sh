# round-4 session check q: chunk sweep (windows per two-pass chunk; default = 192 MiB of column results, i.e. 192
# windows at N = 131072 and 96 at N = 262144) for the two-pass large-N forms after the round's column / row changes;
# then the new N = 131072 full-batch parity case.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
b() {  # b <tag> <bench args...>
    local tag=$1; shift
    timeout -k 10 300 python bench.py "$@" --steps 50 --warmup 10 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1])
print('$tag', '%.4f ms'%d['ms_per_step'], '%.4g win/s'%d['value'])"
}
b l131_auto --config large_131072
for c in 48 96 128 256 512; do b l131_c$c --config large_131072 --chunk $c; done
b l262_auto --config large_262144
for c in 24 48 64 128 256; do b l262_c$c --config large_262144 --chunk $c; done
b l131_auto2 --config large_131072
b l262_auto2 --config large_262144
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullgrid.py -m gpu -q -p no:cacheprovider -k large_full --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
