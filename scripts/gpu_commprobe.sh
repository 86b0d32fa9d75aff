# price of the DP plumbing on one GPU: one-rank RCCL communicator, bucketed all-reduce + buffer
# broadcast + stream fork/join (CS_COMM_PROBE=1), eager and full-graph, vs no communicator
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export CS744_TUNE_CACHE=gpurun_out/tune_commprobe.json
for cfg in "none 0" "none 1" "full 1" "full 0"; do
  set -- $cfg
  CS_COMM_PROBE=$2 timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 --graph $1 > gpurun_out/bench_commprobe.log 2>&1 || { tail -20 gpurun_out/bench_commprobe.log; exit 1; }
  echo "graph=$1 probe=$2 $(tail -1 gpurun_out/bench_commprobe.log | cut -c60-100)"
done
