# eager step: per-bucket SGD overlap on/off (cross-stream event cost outside graphs), full graph for reference
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export CS744_TUNE_CACHE=gpurun_out/tune_eager.json
for cfg in "none 0" "none 1" "full 0" "none 0" "none 1" "full 0"; do
  set -- $cfg
  CS_SGD_OVERLAP=$2 timeout -k 10 300 python3 bench.py --steps 400 --warmup 20 --graph $1 > gpurun_out/bench_eager.log 2>&1 || exit $?
  echo "graph=$1 sgd_overlap=$2 $(tail -1 gpurun_out/bench_eager.log | cut -c60-100)"
done
