#!/bin/bash
# SQ counters of the C3 step (Kalman pre-pass alternating with the spectrum kernel).
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/kalman_alt_$1; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/sq -o run -- \
  fft-wavespec_amd/bin/kbench kalman 4 2 > $OUT/sq.log 2>&1 || exit $?
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
rows = collections.defaultdict(dict)
for f in glob.glob(out + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'kalman' in r['Kernel_Name']:
            rows[(int(r['Dispatch_Id']), r['Kernel_Name'][60:125])][r['Counter_Name']] = float(r['Counter_Value'])
for k in sorted(rows):
    v = rows[k]
    print(k, ' '.join(f"{c}={v[c]:.4g}" for c in sorted(v)))
PY
cat $OUT/sq.log
