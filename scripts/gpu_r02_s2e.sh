#!/bin/bash
# Session 2e: counter list; SQ stall/fetch counters of the Kalman pre-pass (C3) and the hop=1 spectrum (C4).
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -oE "SQ_[A-Z0-9_]+|SQC_[A-Z0-9_]+" $O/counters.txt | sort -u | tr '\n' ' ' | head -c 6000; echo
for c in c3 c4; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d $O/sqf_$c -o run -- \
  python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-settle > $O/sqf_$c.log 2>&1 || { tail -5 $O/sqf_$c.log; exit 1; }
python3 - $O/sqf_$c <<'PY'
import csv, glob, sys, collections
vals = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'spectrum_kernel' in r['Kernel_Name'] or 'kalman' in r['Kernel_Name']:
            vals[(r['Kernel_Name'][:50], r['Counter_Name'])].append(float(r['Counter_Value']))
for k, v in sorted(vals.items()):
    print(k[0], k[1], '%.4g' % (sum(v) / len(v)))
PY
done
