# round-4 closing check on ONE box: the whole GPU suite, smoke, the default bench line (the driver's command),
# every configuration's bench line, then the north-star kernel trace + PMC passes on the same lease (VERDICT r03
# item 7: traced average and ms_per_step from one box).  gpu_run.sh stops at the first failing step.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_run.sh ${TAG:-r04final} tests smoke default bench=north_star bench=c2 bench=c3 bench=c4 bench=c4_topk bench=c5 \
    bench=ns_topk bench=ns_phase bench=ns_topk_phase bench=inverse bench=large bench=large_262144 prof=north_star
