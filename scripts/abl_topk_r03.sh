cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r03j; mkdir -p $O
for sg in 128 512; do for v in 2 4 5; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_${v}_$sg -o run -- python3 bench.py --config c4_topk --variant $v --slide-seg $sg --steps 30 --warmup 5 --no-cpu-baseline > $O/b_${v}_$sg.json 2> $O/b_${v}_$sg.err || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('$O/tr_${v}_$sg/run_kernel_stats.csv')):
    if 'slide' in r['Name']: print('v$v seg$sg', r['Name'][40:75], '%.1f us'%(float(r['AverageNs'])/1e3))"
done; done
