# round-4 profiles: kernel traces + PMC traffic of the changed paths, SQ counters of the VALU-bound configs,
# the C5 strong-shard segment sweep and the large-N chunk sweep
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
t() {  # t <log> <pytest args...>: a failed assertion (rc 1) does not stop the run
    local log=$1; shift
    timeout -k 10 500 python -u -m pytest "$@" -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/$log 2>&1
    local rc=$?
    tail -4 $O/$log
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
t t_new.log -s tests/test_gpu_slide.py::test_slide_topk_exact_ties tests/test_gpu_fullgrid.py::test_c4_topk_probe_scan_vs_oracle_full_size
bash scripts/gpu_run.sh r04c prof=c5 prof=c5,auto,0,per_length,--c5-mode+group-per-length prof=ns_topk_phase prof=inverse \
    sq=c3,SQ_WAIT_ANY,SQ_INSTS_VALU,SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_LDS,SQ_WAIT_INST_ANY \
    || exit $?
bash scripts/gpu_run.sh r04c sq=c4_topk,SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU || exit $?
for mode in symbols split; do
  for seg in 32 48 64 96 128 192; do
    timeout -k 10 120 python bench.py --config c5 --emulate-shard 0/8 --c5-shard $mode --slide-seg $seg --steps 50 --warmup 10 --no-cpu-baseline > $O/c5_shard0of8_${mode}_seg$seg.json 2>$O/c5_shard_err.log || exit $?
    python3 -c "import json; d=json.loads(open('$O/c5_shard0of8_${mode}_seg$seg.json').read().strip().splitlines()[-1]); print('c5 shard 0/8 $mode seg $seg', '%.4f ms'%d['ms_per_step'])"
  done
done
for seg in 96 128 160 256 320 448; do
  timeout -k 10 120 python bench.py --config c5 --slide-seg $seg --steps 100 --warmup 20 --no-cpu-baseline > $O/c5_seg$seg.json 2>$O/c5_err.log || exit $?
  python3 -c "import json; d=json.loads(open('$O/c5_seg$seg.json').read().strip().splitlines()[-1]); print('c5 seg $seg', '%.4f ms'%d['ms_per_step'])"
done
for ch in 24 48 192; do
  timeout -k 10 120 python bench.py --config large_262144 --chunk $ch --steps 30 --warmup 5 --no-cpu-baseline > $O/large262144_chunk$ch.json 2>$O/large_err.log || exit $?
  python3 -c "import json; d=json.loads(open('$O/large262144_chunk$ch.json').read().strip().splitlines()[-1]); print('large_262144 chunk $ch', '%.4f ms'%d['ms_per_step'])"
done
timeout -k 10 120 python bench.py --config large_262144 --variant 2 --steps 30 --warmup 5 --no-cpu-baseline > $O/large262144_v2.json 2>>$O/large_err.log || exit $?
python3 -c "import json; d=json.loads(open('$O/large262144_v2.json').read().strip().splitlines()[-1]); print('large_262144 v2', '%.4f ms'%d['ms_per_step'])"
