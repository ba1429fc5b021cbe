#!/bin/bash
# Session 2f: full GPU suite; PCIe-inclusive rate staged vs registered; C3 profile refresh (pk2 Kalman).
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02b; mkdir -p $O
export WSP_PARITY_LOG=$O/parity_metrics.json
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 180 python3 scripts/pcie_rate.py north_star > $O/pcie_staged.json 2>&1 || { cat $O/pcie_staged.json; exit 1; }
timeout -k 10 180 python3 scripts/pcie_rate.py north_star --registered > $O/pcie_registered.json 2>&1 || { cat $O/pcie_registered.json; exit 1; }
python3 -c "
import json
for f in ('staged','registered'):
    d=json.loads(open('$O/pcie_'+f+'.json').read().strip().splitlines()[-1]); print(f, ['%.4f'%t for t in d['seconds']], '%.3g windows/s'%d['windows_per_s'], '%.1f GB/s host bytes'%(d['host_bytes_per_s']/1e9), d.get('register_seconds'))"
bash scripts/gpu_profile.sh r02b c3 > gpurun_out/prof_r02b_c3.summary 2>&1 || { tail -20 gpurun_out/prof_r02b_c3.summary; exit 1; }
tail -c 1500 gpurun_out/prof_r02b_c3.summary
