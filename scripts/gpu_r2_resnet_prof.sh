# ResNet-50 (torch path, NCHW) kernel profile: where a step's time goes on MI355X
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for dt in bf16 fp32; do
  timeout -k 10 300 python3 bench.py --model resnet50 --dtype $dt --steps 10 --warmup 3 > gpurun_out/rn_$dt.log 2>&1 || exit $?
  tail -1 gpurun_out/rn_$dt.log
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_rn_bf16 -o run -- python3 $R/bench.py --model resnet50 --dtype bf16 --steps 3 --warmup 2 > $R/gpurun_out/prof_rn_bf16.log 2>&1) || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_rn_bf16 --steps 5 --top 30 > gpurun_out/prof_rn_bf16_summary.txt 2>&1
head -34 gpurun_out/prof_rn_bf16_summary.txt
