# round-4 session check j: the new full-size parity tests (C2 at 4096 x 1024, the large-N batches of the bench
# against torch.fft window by window, the ns_phase record on both grid-stride iterations).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
WSP_PARITY_LOG=$O/parity_metrics.json timeout -k 10 500 python -u -m pytest tests/test_gpu_fullgrid.py \
    -k "c2_full or large_full or ns_phase_full" -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/t.log 2>&1
rc=$?; tail -8 $O/t.log; exit $rc
