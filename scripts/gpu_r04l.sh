# round-4 session check l: half-length segments for the mixed C5 launch's last class (the shortest windows, which
# drain the launch) against one segment length for every class (mode 3); group tests first.
# (As run at commit 0a9c387, where tail-half was the default and mode 3 "mixed-uniform" the one-length ablation;
# since b47fafe one length is the default and mode 3 is "mixed-tail-half", so this script no longer runs as is.)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_slide.py tests/test_gpu_fullgrid.py::test_c5_grouped_plan -k "group" -v -m gpu \
    -p no:cacheprovider --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
S1=--emulate-shard,1/8
S6=--emulate-shard,6/8
bash scripts/gpu_run.sh r04l bench=c5 bench=c5,--c5-mode,group-mixed-uniform bench=c5,--steps,101 \
    bench=c5,--c5-mode,group-mixed-uniform,--steps,101 bench=c5,$S1 bench=c5,$S1,--c5-mode,group-mixed-uniform \
    bench=c5,$S6 bench=c5,$S6,--c5-mode,group-mixed-uniform
