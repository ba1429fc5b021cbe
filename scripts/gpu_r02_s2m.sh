#!/bin/bash
# Session 2m: end-to-end (host memory) C4: power vs fused top-k; staged vs registered.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02h; mkdir -p $O
for mode in "" "--registered" "--topk"; do
tag=$(echo "c4$mode" | tr -d ' -')
timeout -k 10 300 python3 scripts/pcie_rate.py c4 $mode > $O/pcie_$tag.json 2> $O/pcie_$tag.err || { tail -5 $O/pcie_$tag.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/pcie_$tag.json').read().strip().splitlines()[-1]); print('$tag', ['%.4f'%t for t in d['seconds']], '%.3g windows/s'%d['windows_per_s'], '%.1f GB/s host bytes'%(d['host_bytes_per_s']/1e9))"
done
