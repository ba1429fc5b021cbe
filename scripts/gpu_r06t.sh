#!/bin/bash
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_run.sh r06t "tests=tests/test_gpu_large.py,tests/test_gpu_fullgrid.py,-k,large" sq=large_262144,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE sq=large,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE && \
bash scripts/ab_lib.sh r06t fft-wavespec_amd/lib/libmtbridge_a.so fft-wavespec_amd/lib/libmtbridge_b.so 2 large large_131072 large_262144
