# DP plumbing price on one GPU: event fork/join vs stream-memory-op fork/join; bucket count
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export CS744_TUNE_CACHE=gpurun_out/tune_commprobe3.json
for cfg in "0 0 4" "1 0 4" "1 1 4" "1 0 12" "1 1 12" "1 0 1000" "0 0 4"; do
  set -- $cfg
  CS_COMM_PROBE=$1 CS_COMM_FORK=$2 timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 --graph none --bucket-mb $3 > gpurun_out/bench_commprobe3.log 2>&1 || { tail -20 gpurun_out/bench_commprobe3.log; exit 1; }
  echo "probe=$1 valuefork=$2 bucket_mb=$3 $(tail -1 gpurun_out/bench_commprobe3.log | cut -c60-100)"
done
