# round-4 session check g: the mixed C5 launch per window length (one-length groups: which class runs below the
# write rate), two vs four bins per thread there, and the segment length of the slowest one-eighth C5 shards
# (rank 1 = the N = 1024 symbols, rank 4 = N = 4096); first the two-ended task order (mode 3: every other group
# of 8 workgroups takes the shortest tasks first, so seed phases stop coinciding) against the default; last the
# fused N = 65536 kernel with wave-local column FFTs (variant 8) and wave-local rows too (9) against the default.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_slide.py -k group tests/test_gpu_large.py -v -m gpu -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/t_group.log 2>&1
rc=$?; tail -3 $O/t_group.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
S1=--emulate-shard,1/8
S4=--emulate-shard,4/8
bash scripts/gpu_run.sh r04g bench=c5 bench=c5,--c5-mode,group-mixed-two-ended bench=c5,--steps,101 \
    bench=c5,--c5-mode,group-mixed-two-ended,--steps,101 harness=c5_len_sweep.py,30,0,128,256 harness=c5_len_sweep.py,30,0,128,--mode,mixed-b4 \
    harness=c5_len_sweep.py,30,0,--mode,per-length \
    bench=c5,$S1 bench=c5,$S1,--slide-seg,64 bench=c5,$S1,--slide-seg,96 bench=c5,$S1,--slide-seg,192 \
    bench=c5,$S1,--c5-mode,group-mixed-b4 bench=c5,$S4 bench=c5,$S4,--slide-seg,64 bench=c5,$S4,--slide-seg,192 \
    bench=c5,$S4,--c5-mode,group-mixed-b4 bench=large bench=large,--variant,8 bench=large,--steps,101 \
    bench=large,--variant,8,--steps,101 bench=large,--variant,9 bench=large,--variant,9,--steps,101
