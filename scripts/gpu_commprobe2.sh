# DP plumbing price on one GPU by fork/join event flavour (CS_COMM_EVENT_FLAGS 0/1/2), eager
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export CS744_TUNE_CACHE=gpurun_out/tune_commprobe2.json
for cfg in "0 0" "1 0" "1 1" "1 2" "0 0" "1 1"; do
  set -- $cfg
  CS_COMM_PROBE=$1 CS_COMM_EVENT_FLAGS=$2 timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 --graph none > gpurun_out/bench_commprobe2.log 2>&1 || { tail -20 gpurun_out/bench_commprobe2.log; exit 1; }
  echo "probe=$1 evflags=$2 $(tail -1 gpurun_out/bench_commprobe2.log | cut -c60-100)"
done
