# round-2: Llama-3-8B step with the shipped TunableOp GEMM table vs hipBLASLt's heuristic picks (same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --model llama3-8b --steps 4 --warmup 2 > gpurun_out/bench_llama_table.log 2>&1 || exit $?
echo "table: $(tail -1 gpurun_out/bench_llama_table.log | cut -c1-400)"
CS744_GEMM_TABLE=0 timeout -k 10 300 python bench.py --model llama3-8b --steps 4 --warmup 2 > gpurun_out/bench_llama_notable.log 2>&1 || exit $?
echo "heuristic: $(tail -1 gpurun_out/bench_llama_notable.log | cut -c1-200)"
