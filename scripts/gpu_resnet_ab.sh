# ResNet-50 layout / dtype A/B + a kernel trace of the slow configuration
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export MIOPEN_FIND_MODE=FAST TMPDIR=/tmp
for CFG in "1 bf16" "0 bf16" "1 fp32" "0 fp32"; do
  set -- $CFG
  CS744_CHANNELS_LAST=$1 timeout -k 10 200 python bench.py --model resnet50 --dtype $2 --steps 10 --warmup 5 > gpurun_out/rn_$1_$2.log 2>&1 || exit $?
  echo "channels_last=$1 $2: $(tail -1 gpurun_out/rn_$1_$2.log | cut -c60-140)"
done
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn -o run -- python3 $R/bench.py --model resnet50 --dtype bf16 --steps 5 --warmup 3 > $R/gpurun_out/prof_rn.log 2>&1
rc=$?; cd $R; python3 scripts/prof_summary.py gpurun_out/prof_rn --steps 8 > gpurun_out/prof_rn_summary.txt 2>&1; head -25 gpurun_out/prof_rn_summary.txt | cut -c1-160; exit $rc
