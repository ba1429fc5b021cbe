#!/bin/bash
# Same-box A/B of two builds of libmtbridge.so: alternates bench.py runs of each config against library A and
# library B (WSP_MTBRIDGE_LIB), `rounds` times, and prints one line per run.  Lines land in gpurun_out/<tag>/ab.log.
#   bash scripts/ab_lib.sh <tag> <libA> <libB> <rounds> <config[,args]> [<config[,args]> ...]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; A=$2; B=$3; R=$4
shift 4
O=gpurun_out/$TAG
mkdir -p $O
for ((i = 0; i < R; i++)); do
    for spec in "$@"; do
        cfg=${spec%%,*}
        extra=""
        [ "$cfg" != "$spec" ] && extra=${spec#*,}
        for lib in "$A" "$B"; do
            WSP_MTBRIDGE_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 20 --no-cpu-baseline ${extra//,/ } > $O/one.json 2> $O/one.err || { echo "bench failed ($lib $spec)"; tail -20 $O/one.err; exit 1; }
            python3 -c "
import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1])
print('$TAG round $i', '$(basename $lib)', '$spec', '%.4f ms' % d['ms_per_step'], 'frac %.3f' % d['roofline']['frac'])" | tee -a $O/ab.log
        done
    done
done
