# A/B of the single-launch BN row threshold
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export CS744_TUNE_CACHE=$GRAFT_REPO_ROOT/gpurun_out/tune_bnf.json
for R in 0 256 1024 4096 0; do
  CS_BN_FUSED_ROWS=$R timeout -k 10 300 python bench.py --steps 300 --warmup 20 > gpurun_out/bnf_$R.log 2>&1 || exit $?
  echo "rows=$R $(tail -1 gpurun_out/bnf_$R.log | cut -c60-140)"
done
