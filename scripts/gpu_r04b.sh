# round-4 session check: the mixed-length grouped launch first (its own short limit), then the new parity tests,
# A/B benches (C5 mixed vs per-length, ns_topk_phase split vs AoS) and the strong-shard emulation
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04b
timeout -k 10 400 python -u -m pytest tests/test_gpu_slide.py -k "group" -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04b/t_group.log 2>&1
rc=$?; tail -25 gpurun_out/r04b/t_group.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "topk_phase or inverse" -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/r04b/t_phase.log 2>&1
rc=$?; tail -25 gpurun_out/r04b/t_phase.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc  # a failed assertion: go on
bash scripts/gpu_run.sh r04b tests=tests/test_gpu_slide.py::test_slide_topk_exact_ties,tests/test_gpu_slide.py::test_plan_workspace_growth_frees_old_block,tests/test_gpu_fullgrid.py::test_c4_topk_probe_scan_vs_oracle_full_size,tests/test_gpu_fullgrid.py::test_c5_grouped_plan,tests/test_gpu_fullgrid.py::test_ns_topk_full_grid,-s bench=c5 bench=c5,--c5-mode,group-per-length bench=c5 bench=c5,--c5-mode,group-per-length bench=ns_topk_phase bench=ns_topk_phase,--variant,1 bench=inverse bench=inverse,--variant,1 bench=inverse,--variant,2 shards
