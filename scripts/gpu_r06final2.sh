# round-6 closing check, second session (after the Newton-basis Kalman step, the window fold and bench's own PMC
# passes), in parts that each fit one gpurun call (gpu_run.sh stops at the first failing step):
#   PART=a  the whole GPU suite, smoke, the default bench line (the driver's command: now with its own PMC passes),
#           then the north-star and C3 kernel traces + PMC passes on the same lease
#   PART=b  every configuration's line with the CPU baseline (1 core + the job's cores) and its own PMC passes
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
case "${PART:-a}" in
a)
    bash scripts/gpu_run.sh ${TAG:-r06z} tests smoke default prof=north_star prof=c3
    ;;
b)
    bash scripts/gpu_run.sh ${TAG:-r06zb} benchc=north_star benchc=c2 benchc=c3 benchc=c4 benchc=c4_topk \
        benchc=c5 benchc=ns_topk benchc=ns_phase benchc=ns_topk_phase benchc=inverse benchc=large benchc=large_131072 \
        benchc=large_262144
    ;;
esac
