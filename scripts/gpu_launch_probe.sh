# price of one kernel boundary inside the replayed step graph
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export CS744_TUNE_CACHE=$GRAFT_REPO_ROOT/gpurun_out/tune_probe.json
for K in 0 0; do
  CS_PROBE_EXTRA_LAUNCHES=$K timeout -k 10 300 python bench.py --steps 300 --warmup 20 > gpurun_out/probe_$K.log 2>&1 || exit $?
  echo "extra=$K $(tail -1 gpurun_out/probe_$K.log | cut -c60-150)"
done
