#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_run.sh r06r "tests=tests/test_gpu_large.py" "harness=large_timeline.py,gpurun_out/r06r/large_tl.json" && \
bash scripts/ab_lib.sh r06r fft-wavespec_amd/lib/libmtbridge_a.so fft-wavespec_amd/lib/libmtbridge_b.so 2 large large_262144
