# round-5 closing check on ONE box: the whole GPU suite, smoke, the default bench line (the driver's command), every
# configuration's line WITH the CPU baseline beside it (1 core + the job's cores: VERDICT r04 item 7), then the
# north-star kernel trace + PMC passes on the same lease.  gpu_run.sh stops at the first failing step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_run.sh ${TAG:-r05final} tests smoke default benchc=north_star benchc=c2 benchc=c3 benchc=c4 benchc=c4_topk \
    benchc=c5 benchc=ns_topk benchc=ns_phase benchc=ns_topk_phase benchc=inverse benchc=large benchc=large_262144 \
    prof=north_star
