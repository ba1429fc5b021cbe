# Driver-style bench lines (the round-end driver runs `python bench.py --gpus 1 --steps 20 --warmup 5`, and
# torchrun for N > 1): two plain runs, one single-rank torchrun run, and C2 (the settle phase of a 10-us step).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r03drv; mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5_a.json 2> $O/a.err || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_20_5_b.json 2> $O/b.err || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_torchrun_1rank.json 2> $O/c.err || exit 1
for f in $O/*.json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', '%.4f ms'%d['ms_per_step'], '%.4g win/s'%d['value'], 'frac %.3f'%d['roofline']['frac'], 'cpu', d.get('cpu_baseline',{}).get('value'))"; done
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_20_5.json 2> $O/d.err || exit 1
python3 -c "
import json; d=json.loads(open('$O/bench_c2_20_5.json').read().strip().splitlines()[-1]); print('c2', '%.4f ms'%d['ms_per_step'], d['settle'])"
