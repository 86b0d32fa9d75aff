# round-2: Llama-3-8B (bf16, B=4 x 2048) bench + rocprofv3 kernel table
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --model llama3-8b --steps 4 --warmup 2 > gpurun_out/bench_llama.log 2>&1 || exit $?
tail -1 gpurun_out/bench_llama.log | cut -c1-300
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_llama -o run -- python3 $R/bench.py --model llama3-8b --steps 2 --warmup 1 > $R/gpurun_out/prof_llama.log 2>&1) || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_llama --steps 3 > gpurun_out/prof_llama_summary.txt 2>&1
head -45 gpurun_out/prof_llama_summary.txt | cut -c1-200
