#!/bin/bash
# Kalman pre-pass: GPU parity tests, kbench ablation, one SQ counter pass over it.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1
OUT=gpurun_out/kalman_$TAG; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "kalman or f32_detrends" > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 fft-wavespec_amd/bin/kbench kalman 10 > $OUT/kbench.log 2>&1; rc=$?
cat $OUT/kbench.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/sq -o run -- \
  fft-wavespec_amd/bin/kbench kalman 1 > $OUT/sq.log 2>&1 || exit $?
python3 - $OUT > $OUT/sq_summary.txt <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
vals = collections.defaultdict(list)
for f in glob.glob(out + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'kalman' in r['Kernel_Name']:
            vals[(r['Kernel_Name'][:110], r['Counter_Name'])].append(float(r['Counter_Value']))
for k, v in sorted(vals.items()):
    print(k[0], k[1], sum(v) / len(v))
PY
