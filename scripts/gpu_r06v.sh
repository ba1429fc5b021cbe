#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_run.sh r06v "tests=tests/test_gpu_large.py,tests/test_gpu_fullgrid.py,-k,large" "harness=large_timeline.py,gpurun_out/r06v/large_tl.json" && \
bash scripts/ab_lib.sh r06v fft-wavespec_amd/lib/libmtbridge_a.so fft-wavespec_amd/lib/libmtbridge_b.so 3 large
