#!/bin/bash
# rocprofv3 passes over bench.py for one config:
#   1) --kernel-trace --stats      (per-kernel durations)
#   2) --pmc FETCH_SIZE            (own pass; HBM read bytes, x2 gfx950 correction)
#   3) --pmc WRITE_SIZE            (own pass)
# Usage: bash scripts/gpu_profile.sh <tag> [config] [algo: auto|fft|slide] [variant] [key suffix] [extra bench args...]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; CFG=${2:-north_star}; ALGO=${3:-auto}; VAR=${4:-0}; SUF=${5:-}
shift $(( $# < 5 ? $# : 5 ))
EXTRA="$*"
KEY=$CFG; [ "$ALGO" = auto ] || KEY=${CFG}_$ALGO
[ "$VAR" = 0 ] || KEY=${KEY}_v$VAR
[ -z "$SUF" ] || KEY=${KEY}_$SUF
OUT=gpurun_out/prof_${TAG}_${KEY}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --config $CFG --steps 100 --warmup 20 --no-cpu-baseline --algo $ALGO --variant $VAR $EXTRA > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/fetch -o run -- \
  python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --algo $ALGO --variant $VAR $EXTRA > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/write -o run -- \
  python3 bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --algo $ALGO --variant $VAR $EXTRA > $OUT/write.log 2>&1 || exit $?
python3 scripts/parse_prof.py $OUT $CFG $KEY
