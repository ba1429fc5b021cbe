#!/bin/bash
# Split-exchange padding (C4 / north star): tests, ablation, bench lines, LDS counters.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "kalman or c3 or c4 or north_star or sizes or overlap or topk or full_size" > $O/pytest_b.log 2>&1 || { tail -30 $O/pytest_b.log; exit 1; }
tail -2 $O/pytest_b.log
timeout -k 10 180 fft-wavespec_amd/bin/kbench hop1 11 1048576 5 > $O/kbench_hop1_n2048_pad.log 2>&1 || { cat $O/kbench_hop1_n2048_pad.log; exit 1; }
tail -4 $O/kbench_hop1_n2048_pad.log
for c in north_star c4 c3; do
  timeout -k 10 180 python3 bench.py --config $c --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_$c.json || exit 1
done
for f in bench_north_star bench_c4 bench_c3; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), d['value'])"; done
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --kernel-trace --output-format csv -d $O/sq_c4 -o run -- python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-settle > $O/sq_c4.log 2>&1 || { tail -5 $O/sq_c4.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES --kernel-trace --output-format csv -d $O/sq_ns -o run -- python3 bench.py --config north_star --steps 3 --warmup 1 --no-cpu-baseline --no-settle > $O/sq_ns.log 2>&1 || { tail -5 $O/sq_ns.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, collections
for tag in ("sq_c4", "sq_ns"):
    vals = collections.defaultdict(list)
    for f in glob.glob(sys.argv[1] + "/" + tag + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "spectrum_kernel" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: sum(v) / len(v) for k, v in vals.items()}
    print(tag, out, "conflict/active_lds = %.3f" % (out.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, out.get("SQ_ACTIVE_INST_LDS", 1))))
PY
