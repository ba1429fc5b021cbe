# round-4 session check h: the mixed C5 launch with one-wave 512-point sub-workgroups (wave fences, own trip
# counts; the new default) against the lockstep two-wave form (mode 3), on the full batch, per length and on the
# one-eighth shards; group and large-N tests first.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_slide.py tests/test_gpu_large.py tests/test_gpu_fullgrid.py::test_c5_grouped_plan \
    -k "group or large" -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
S0=--emulate-shard,0/8
bash scripts/gpu_run.sh r04h bench=c5 bench=c5,--c5-mode,group-mixed-lockstep bench=c5,--steps,101 \
    bench=c5,--c5-mode,group-mixed-lockstep,--steps,101 harness=c5_len_sweep.py,30,0,--lens,512,1024 \
    harness=c5_len_sweep.py,30,0,--lens,512,--mode,mixed-lockstep bench=c5,$S0 bench=c5,$S0,--c5-mode,group-mixed-lockstep \
    shards=--configs,c5,--c5-shards,split
