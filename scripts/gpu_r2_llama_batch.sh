# round-2: Llama-3-8B per-GPU batch sweep (x 2048 tokens) on the final kernels
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for b in 6 8; do
  timeout -k 10 300 python bench.py --model llama3-8b --batch-size $b --steps 4 --warmup 2 > gpurun_out/bench_llama_b$b.log 2>&1 || exit $?
  echo "B=$b: $(tail -1 gpurun_out/bench_llama_b$b.log | cut -c1-200)"
  python -c "import torch; print('peak GiB n/a in parent')" > /dev/null
done
