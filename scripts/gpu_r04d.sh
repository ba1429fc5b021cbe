# round-4 session check d: the mixed C5 launch at B=4 (mode 0) against B=2 (mode 2) and the per-length launches,
# the split top-k + phase form after its spill cut (112 -> 80 B/lane) against the AoS form, the C5 segment floor
# on a one-eighth shard and on the full batch, and the phase kernel's PMC traffic.
# A failed assertion (pytest rc 1) does not stop the benches; a fault, abort or time limit does.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
t() {  # t <log> <pytest args...>
    local log=$1; shift
    timeout -k 10 500 python -u -m pytest "$@" -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/$log 2>&1
    local rc=$?
    tail -4 $O/$log
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
t t_group.log tests/test_gpu_slide.py -k group -x
t t_phase.log tests/test_gpu_parity.py -k topk_phase tests/test_gpu_fullgrid.py::test_c5_grouped_plan \
    tests/test_gpu_fullgrid.py::test_ns_topk_full_grid
S8=--emulate-shard,0/8
bash scripts/gpu_run.sh r04d bench=c5 bench=c5,--c5-mode,group-mixed-b2 bench=c5,--c5-mode,group-per-length bench=c5 \
    bench=ns_topk_phase bench=ns_topk_phase,--variant,1 bench=ns_topk_phase \
    bench=c5,$S8 bench=c5,$S8,--slide-seg,64 bench=c5,$S8,--slide-seg,128 bench=c5,$S8,--slide-seg,192 \
    bench=c5,$S8,--slide-seg,256 bench=c5,$S8,--c5-mode,group-mixed-b2 bench=c5,$S8,--c5-mode,group-mixed-b2,--slide-seg,128 \
    bench=c5,--slide-seg,128 bench=c5,--slide-seg,256 \
    prof=ns_topk_phase
