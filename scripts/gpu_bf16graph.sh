# host-launch headroom: eager vs full-step graph for the faster bf16 step (and fp32 B=256)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export CS744_TUNE_CACHE=gpurun_out/tune_bf16graph.json
for cfg in "bf16 64 none" "bf16 64 full" "fp32 256 none" "fp32 256 full" "bf16 256 none" "bf16 256 full"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 --dtype $1 --batch-size $2 --graph $3 > gpurun_out/bench_bg.log 2>&1 || exit $?
  echo "$1 B=$2 graph=$3 $(tail -1 gpurun_out/bench_bg.log | cut -c60-100)"
done
