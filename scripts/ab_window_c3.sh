set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06win
for i in 1 2; do
for w in hann none; do
  WSP_BENCH_WINDOW=$w timeout -k 10 200 python bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/r06win/c3_$w.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/r06win/c3_$w.json').read().strip().splitlines()[-1]); print('$w', d['ms_per_step'])" | tee -a gpurun_out/r06win/ab.log
done; done
