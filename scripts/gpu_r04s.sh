# round-4 session check s: the ns_topk_phase bench line with its VALU roofline (profiles/valu.json, r04r) and the
# new large_131072 config's line, as the driver would print them.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 300 python bench.py --config ns_topk_phase --steps 100 --warmup 20 --no-cpu-baseline > $O/ns_topk_phase.json 2> $O/ns_topk_phase.err || exit $?
tail -1 $O/ns_topk_phase.json
timeout -k 10 300 python bench.py --config large_131072 --steps 50 --warmup 10 > $O/large_131072.json 2> $O/large_131072.err || exit $?
tail -1 $O/large_131072.json
