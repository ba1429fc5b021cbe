#!/bin/bash
# Session 2i: C5 stream layouts (3 balanced streams vs 1), torchrun rehearsal of the driver's N>1 launch with one rank.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r02e; mkdir -p $O
for ns in 3; do
C5_STREAMS=$ns timeout -k 10 180 python3 bench.py --config c5 --steps 100 --warmup 20 --no-cpu-baseline > $O/bench_c5_s$ns.json || exit 1
python3 -c "import json;d=json.load(open('$O/bench_c5_s$ns.json'));print('c5 streams=$ns', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o run -- python3 bench.py --config c5 --steps 30 --warmup 10 --no-cpu-baseline > $O/trace_c5.log 2>&1 || exit 1
timeout -k 10 240 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 5 > $O/torchrun_1.json 2> $O/torchrun_1.err || { tail -20 $O/torchrun_1.err; exit 1; }
tail -1 $O/torchrun_1.json | cut -c1-400
