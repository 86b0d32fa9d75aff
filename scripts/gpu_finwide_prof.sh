# kernel times of the two BN finalize kernels (wide vs one wave per channel)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export CS744_TUNE_CACHE=$R/gpurun_out/tune_finwide.json
for W in 2048 0; do
  cd /tmp && CS_BN_FIN_WIDE=$W timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fw$W -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof_fw$W.log 2>&1 || exit $?
  cd $R
  python3 scripts/prof_summary.py gpurun_out/prof_fw$W --steps 25 --timeline 10 > gpurun_out/prof_fw${W}_summary.txt 2>&1
  grep -E "^#|finalize" gpurun_out/prof_fw${W}_summary.txt
done
