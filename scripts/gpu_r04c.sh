# round-4 profiles: kernel traces + PMC traffic of the changed paths, SQ counters of the VALU-bound configs,
# the C5 strong-shard segment sweep and the large-N chunk sweep
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
bash scripts/gpu_run.sh r04c prof=c5 prof=c5,auto,0,per_length,--c5-mode+group-per-length prof=ns_topk_phase prof=inverse \
    sq=c3,SQ_WAIT_ANY,SQ_INSTS_VALU,SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_LDS,SQ_WAIT_INST_ANY \
    || exit $?
bash scripts/gpu_run.sh r04c sq=c4_topk,SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_INSTS_SALU || exit $?
for seg in 32 48 64 96 128; do
  timeout -k 10 120 python bench.py --config c5 --emulate-shard 0/8 --slide-seg $seg --steps 50 --warmup 10 --no-cpu-baseline > $O/c5_shard0of8_seg$seg.json 2>$O/c5_shard_err.log || exit $?
  tail -1 $O/c5_shard0of8_seg$seg.json | cut -c1-200
done
for ch in 24 48 192; do
  timeout -k 10 120 python bench.py --config large_262144 --chunk $ch --steps 30 --warmup 5 --no-cpu-baseline > $O/large262144_chunk$ch.json 2>$O/large_err.log || exit $?
  tail -1 $O/large262144_chunk$ch.json | cut -c1-200
done
timeout -k 10 120 python bench.py --config large_262144 --variant 2 --steps 30 --warmup 5 --no-cpu-baseline > $O/large262144_v2.json 2>>$O/large_err.log || exit $?
tail -1 $O/large262144_v2.json | cut -c1-200
