# round-4 session check e: the split top-k + phase form without spills (atan2 as a call, one pass of atan2 over
# the 3k winner items), the AoS top-k + phase forms after the same change, the mixed C5 launch with two bins per
# thread as the default and the segment floor of 128, then the phase kernel's PMC traffic.
# A failed assertion (pytest rc 1) does not stop the benches; a fault, abort or time limit does.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
t() {  # t <log> <pytest args...>
    local log=$1; shift
    timeout -k 10 500 python -u -m pytest "$@" -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/$log 2>&1
    local rc=$?
    tail -4 $O/$log
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
t t_phase.log tests/test_gpu_parity.py -k "phase" tests/test_gpu_fullgrid.py::test_ns_topk_full_grid
t t_group.log tests/test_gpu_slide.py -k group tests/test_gpu_fullgrid.py::test_c5_grouped_plan
S8=--emulate-shard,0/8
bash scripts/gpu_run.sh r04e bench=ns_topk_phase bench=ns_topk_phase,--variant,1 bench=ns_topk_phase bench=ns_phase \
    bench=c5 bench=c5,--c5-mode,group-mixed-b4 bench=c5 bench=c5,$S8 bench=c5,$S8,--slide-seg,192 \
    prof=ns_topk_phase
