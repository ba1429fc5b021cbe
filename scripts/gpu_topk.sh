#!/bin/bash
# Top-k rework: parity tests, output-mode ablation, bench line.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r02; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "topk" > $O/pytest_topk.log 2>&1 || { tail -40 $O/pytest_topk.log; exit 1; }
tail -2 $O/pytest_topk.log
timeout -k 10 120 fft-wavespec_amd/bin/kbench out 20 > $O/kbench_outputs_r02.log 2>&1 || { cat $O/kbench_outputs_r02.log; exit 1; }
cat $O/kbench_outputs_r02.log
timeout -k 10 180 python3 bench.py --config ns_topk --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_ns_topk.json || exit 1
python3 -c "import json;d=json.load(open('$O/bench_ns_topk.json'));print('ns_topk', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
