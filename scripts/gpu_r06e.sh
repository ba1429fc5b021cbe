#!/bin/bash
# round 6: DPP neighbour phases -- the probe, the phase parity tests, the benchmarked record
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06e
timeout -k 10 60 fft-wavespec_amd/bin/dpp_probe > gpurun_out/r06e/dpp_probe.log 2>&1 && cat gpurun_out/r06e/dpp_probe.log && \
bash scripts/gpu_run.sh r06e "tests=tests/test_gpu_parity.py,tests/test_gpu_fullgrid.py,-k,phase" bench=ns_phase bench=ns_topk_phase bench=ns_phase
