# round-4 session check: the mixed-length grouped launch first (its own short limit), then the new parity tests,
# A/B benches (C5 mixed vs per-length, ns_topk_phase split vs AoS, inverse forms) and the strong-shard emulation.
# A failed assertion (pytest rc 1) does not stop the benches; a fault, abort or time limit does.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
t() {  # t <log> <pytest args...>
    local log=$1; shift
    timeout -k 10 500 python -u -m pytest "$@" -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/$log 2>&1
    local rc=$?
    tail -4 $O/$log
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
t t_group.log tests/test_gpu_slide.py -k group -x
t t_phase.log tests/test_gpu_parity.py -k "topk_phase or inverse"
t t_new.log -s tests/test_gpu_slide.py::test_slide_topk_exact_ties tests/test_gpu_slide.py::test_plan_workspace_growth_frees_old_block \
    tests/test_gpu_fullgrid.py::test_c4_topk_probe_scan_vs_oracle_full_size tests/test_gpu_fullgrid.py::test_c5_grouped_plan \
    tests/test_gpu_fullgrid.py::test_ns_topk_full_grid tests/test_gpu_large.py::test_large_set_chunk
bash scripts/gpu_run.sh r04b bench=c5 bench=c5,--c5-mode,group-per-length bench=c5 bench=c5,--c5-mode,group-per-length \
    bench=ns_topk_phase bench=ns_topk_phase,--variant,1 bench=inverse bench=inverse,--variant,1 bench=inverse,--variant,2 shards
