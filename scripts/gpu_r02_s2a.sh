#!/bin/bash
# Session 2a: top-k + phase on the split exchange (parity + bench), C4 stall counters, counter list.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "topk or phase" > $O/pytest_topk_phase.log 2>&1 || { tail -40 $O/pytest_topk_phase.log; exit 1; }
tail -2 $O/pytest_topk_phase.log
timeout -k 10 180 python3 bench.py --config ns_topk_phase --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_ns_topk_phase.json || exit 1
python3 -c "import json;d=json.load(open('$O/bench_ns_topk_phase.json'));print('ns_topk_phase', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
timeout -k 10 120 fft-wavespec_amd/bin/kbench out 10 > $O/kbench_outputs.log 2>&1 || { cat $O/kbench_outputs.log; exit 1; }
cat $O/kbench_outputs.log
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace --output-format csv -d $O/sq_c4 -o run -- \
  python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $O/sq_c4.log 2>&1 || exit 1
python3 - $O/sq_c4 <<'PY'
import csv, glob, sys, collections
vals = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'spectrum_kernel' in r['Kernel_Name']:
            vals[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(vals.items()):
    print(k, sum(v) / len(v))
PY
