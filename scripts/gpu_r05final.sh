# round-5 closing check, in parts that each fit one gpurun call (gpu_run.sh stops at the first failing step):
#   PART=a  the whole GPU suite, smoke, the default bench line (the driver's command), then the north-star kernel
#           trace + PMC passes on the same lease
#   PART=b  every configuration's line WITH the CPU baseline beside it (1 core + the job's cores: VERDICT r04 item 7)
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
case "${PART:-a}" in
a)
    bash scripts/gpu_run.sh ${TAG:-r05final} tests smoke default prof=north_star
    ;;
b)
    bash scripts/gpu_run.sh ${TAG:-r05finalb} benchc=north_star benchc=c2 benchc=c3 benchc=c4 benchc=c4_topk \
        benchc=c5 benchc=ns_topk benchc=ns_phase benchc=ns_topk_phase benchc=inverse benchc=large benchc=large_262144
    ;;
esac
