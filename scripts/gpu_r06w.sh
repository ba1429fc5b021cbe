#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_run.sh r06w "tests=tests/test_gpu_parity.py,tests/test_gpu_fullgrid.py,-k,phase" && \
bash scripts/ab_lib.sh r06w fft-wavespec_amd/lib/libmtbridge_a.so fft-wavespec_amd/lib/libmtbridge_b.so 3 ns_phase
