#!/bin/bash
# SQ instruction-mix / LDS counters for one bench config (own PMC pass, no traces).
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; CFG=$2
OUT=gpurun_out/sq_${TAG}_${CFG}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/a -o run -- \
  python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $OUT/a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/b -o run -- \
  python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline > $OUT/b.log 2>&1 || exit $?
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
vals = collections.defaultdict(list)
for f in glob.glob(out + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'spectrum_kernel' in r['Kernel_Name'] or 'kalman' in r['Kernel_Name']:
            vals[(r['Kernel_Name'][:60], r['Counter_Name'])].append(float(r['Counter_Value']))
for k, v in sorted(vals.items()):
    print(k[0], k[1], sum(v) / len(v))
PY
