# round-4 session check f: the mixed C5 launch with non-temporal power-row stores (mode 3) against the default,
# the C5 strong-shard emulation under the new defaults (two bins per thread, segment floor 128), and kernel traces
# plus PMC passes of the new C5 default and of large_262144 (the two-pass N = 262144 form: which pass bounds it),
# whose column pass now runs 8 columns per workgroup (two workgroups per CU) against 16 (variant 6) and whose row
# pass maps blocks XCD-aware (variant 7: plain order).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
t() {  # t <log> <pytest args...>
    local log=$1; shift
    timeout -k 10 500 python -u -m pytest "$@" -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/$log 2>&1
    local rc=$?
    tail -4 $O/$log
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
t t_group.log tests/test_gpu_slide.py -k group tests/test_gpu_fullgrid.py::test_c5_grouped_plan
t t_large.log tests/test_gpu_large.py
bash scripts/gpu_run.sh r04f bench=c5 bench=c5,--c5-mode,group-mixed-nt bench=c5,--steps,101 bench=c5,--c5-mode,group-mixed-nt,--steps,101 \
    bench=large_262144 bench=large_262144,--variant,6 bench=large_262144,--variant,7 bench=large_262144,--steps,101 bench=large_262144,--variant,6,--steps,101 bench=large_262144,--variant,7,--steps,101 \
    prof=c5 prof=large_262144 shards=--configs,c5,--c5-shards,split
