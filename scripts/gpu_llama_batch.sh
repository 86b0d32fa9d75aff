# Llama-3-8B bf16 (torch path + framework kernels): tokens/s vs per-GPU batch (optimizer amortisation)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 2 4; do
  timeout -k 10 400 python bench.py --model llama3-8b --dtype bf16 --batch-size $b --seq-len 2048 --steps 5 --warmup 2 --json-out gpurun_out/bench_llama_batch.jsonl > gpurun_out/bench_llama_b$b.log 2>&1 || { echo "B=$b failed"; tail -5 gpurun_out/bench_llama_b$b.log; exit 0; }
  echo "B=$b $(tail -1 gpurun_out/bench_llama_b$b.log | cut -c1-160)"
done
