#!/bin/bash
# Session 2k: Infinity-Cache probe for a fused large-N design (recycled per-workgroup slot).
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 120 fft-wavespec_amd/bin/mall_probe 1 > $O/mall_probe_1.log 2>&1 && timeout -k 10 120 fft-wavespec_amd/bin/mall_probe 2 > $O/mall_probe_2.log 2>&1 || { cat $O/mall_probe_*.log; exit 1; }
cat $O/mall_probe_1.log $O/mall_probe_2.log
