# round-5 PMC refresh of profiles/traffic.json on the closing tree: for each configuration given,
# rocprofv3 kernel trace + FETCH_SIZE + WRITE_SIZE in separate passes (scripts/gpu_profile.sh, parsed by
# scripts/parse_prof.py).  Usage: TAG=r05pmc bash scripts/gpu_r05pmc.sh c3 c5 ...
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
steps=()
for c in "$@"; do steps+=("prof=$c"); done
bash scripts/gpu_run.sh ${TAG:-r05pmc} "${steps[@]}"
