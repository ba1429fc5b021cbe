# round-4 session check r: SQ counter passes (VALU issue) over the secondary outputs and the large-N kernels, to
# state their bounds: ns_phase, ns_topk_phase, inverse, large (fused), large_262144 (two passes), C5 (mixed).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
C=SQ_WAIT_ANY,SQ_INSTS_VALU,SQ_WAVES,SQ_BUSY_CYCLES,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_LDS,SQ_WAIT_INST_ANY
bash scripts/gpu_run.sh r04r sq=ns_phase,$C sq=ns_topk_phase,$C sq=inverse,$C sq=large,$C sq=large_262144,$C sq=c5,$C
