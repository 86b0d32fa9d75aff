# round-2 first GPU call: tuned bench + kernel table of the inherited tree, then the RCCL
# two-ranks-on-one-GPU probe (decides how multi-rank native tests can run on a 1-GPU box)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/gpu_prof.sh r2base || exit $?
NCCL_DEBUG=WARN timeout -k 5 90 python3 scripts/rccl_dup_probe.py > gpurun_out/rccl_dup_probe.log 2>&1
echo "dup probe exit $?"; tail -20 gpurun_out/rccl_dup_probe.log
