# kernel timeline of the one-GPU DP plumbing probe (eager)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export CS744_TUNE_CACHE=$R/gpurun_out/tune_commprof.json
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 > gpurun_out/bench_commprof_warm.log 2>&1 || exit $?
cd /tmp
CS_COMM_PROBE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_commprobe -o run -- python3 $R/bench.py --steps 20 --warmup 5 --graph none > $R/gpurun_out/prof_commprobe.log 2>&1 || exit $?
cd $R
python3 scripts/prof_summary.py gpurun_out/prof_commprobe --steps 25 --timeline 110 > gpurun_out/prof_commprobe_summary.txt 2>&1
head -3 gpurun_out/prof_commprobe_summary.txt
