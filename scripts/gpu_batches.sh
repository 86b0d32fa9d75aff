# native engine at other per-GPU batches (part1 = 256) + VGG-16
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for cfg in "VGG11 256" "VGG11 128" "VGG16 64"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --model $1 --batch-size $2 --steps 200 --warmup 20 --json-out gpurun_out/bench_batches.jsonl > gpurun_out/bench_batches.log 2>&1 || { tail -20 gpurun_out/bench_batches.log; exit 1; }
  echo "$1 B=$2 $(tail -1 gpurun_out/bench_batches.log | cut -c1-150)"
done
