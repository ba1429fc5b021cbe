#!/bin/bash
# Full GPU suite + bench lines + PMC traffic of the main configs (round-2 HEAD kernels).
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02; mkdir -p $O
export WSP_PARITY_LOG=$O/parity_metrics.json
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 fft-wavespec_amd/bin/kbench hop1 11 1048576 5 > $O/kbench_hop1_n2048_pad.log 2>&1 || exit 1
grep "round 1" $O/kbench_hop1_n2048_pad.log | head -3
for c in north_star ns_topk c4; do bash scripts/gpu_profile.sh r02 $c > gpurun_out/prof_r02_$c.summary 2>&1 || exit 1; done
for c in north_star ns_topk c4; do python3 -c "
import json;t=open('gpurun_out/prof_r02_$c.summary').read();d=json.loads(t[t.find('{'):])
print('$c', {k[:60]:v for k,v in d.get('kernels',{}).items()}, 'hbm/launch', d.get('hbm_bytes_per_launch'))"; done
