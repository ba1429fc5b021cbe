# round-6 closing check, in parts that each fit one gpurun call (gpu_run.sh stops at the first failing step):
#   PART=a  the whole GPU suite, smoke, the default bench line (the driver's command), then the north-star kernel
#           trace + PMC passes on the same lease
#   PART=b  every configuration's line WITH the CPU baseline beside it (the oracle on 1 core)
#   PART=c  strong-scaling shards emulated one rank at a time (G = 2, 4, 8; each rank the median of 3 passes)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
case "${PART:-a}" in
a)
    bash scripts/gpu_run.sh ${TAG:-r06final} tests smoke default prof=north_star
    ;;
b)
    bash scripts/gpu_run.sh ${TAG:-r06finalb} benchc=north_star benchc=c2 benchc=c3 benchc=c4 benchc=c4_topk \
        benchc=c5 benchc=ns_topk benchc=ns_phase benchc=ns_topk_phase benchc=inverse benchc=large benchc=large_131072 \
        benchc=large_262144
    ;;
c)
    bash scripts/gpu_run.sh ${TAG:-r06finalc} "shards=--configs,north_star+c4+c5+c4_topk,--gpus,2+4+8,--repeat,3,--c5-shards,split"
    ;;
esac
