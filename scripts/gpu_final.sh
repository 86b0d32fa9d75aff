# round-end evidence: full GPU tests + smoke + fp32 bench/profile, bf16-mode profile
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_cycle.sh r1end || exit $?
bash scripts/gpu_prof.sh r1end_bf16 --dtype bf16 || exit $?
