# round-4 session check p: N = 131072 (2048 windows, fp64 Hann; VERDICT r03 item 5 "extend the fused form to
# N = 131072"): the two-pass default against the fused kernel (variant 3: 512 threads, one 1 MiB slot per CU;
# variant 4: 256 threads with register prefetch) and the 8-column two-pass form (variant 8).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
b() {  # b <tag> <bench args...>
    local tag=$1; shift
    timeout -k 10 300 python bench.py "$@" --steps 50 --warmup 10 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || exit $?
    python3 -c "
import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1])
print('$tag', '%.4f ms'%d['ms_per_step'], '%.4g win/s'%d['value'])"
}
b l131_v0 --config large_131072
b l131_v3 --config large_131072 --variant 3
b l131_v4 --config large_131072 --variant 4
b l131_v8 --config large_131072 --variant 8
b l131_v0b --config large_131072
b l131_v3b --config large_131072 --variant 3
