#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_run.sh r06x "tests=tests/test_gpu_large.py,tests/test_gpu_fullgrid.py,-k,large" "harness=large_timeline.py,gpurun_out/r06x/large_tl.json" && \
bash scripts/ab_lib.sh r06x fft-wavespec_amd/lib/libmtbridge_a.so fft-wavespec_amd/lib/libmtbridge_b.so 3 large large_131072 large_262144
