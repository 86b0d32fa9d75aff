# kernel tables for the two BN launch paths (tuned tiles cached first)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export CS744_TUNE_CACHE=$R/gpurun_out/tune_bnprof.json
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 > gpurun_out/bench_bnprof_warm.log 2>&1 || exit $?
for b in 1 0; do
  cd /tmp
  CS_BN_PATH=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bn$b -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof_bn$b.log 2>&1 || exit $?
  cd $R
  python3 scripts/prof_summary.py gpurun_out/prof_bn$b --steps 25 --timeline 70 > gpurun_out/prof_bn${b}_summary.txt 2>&1
  head -3 gpurun_out/prof_bn${b}_summary.txt
done
