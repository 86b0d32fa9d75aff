# round-2: LM kernel tests, then Llama-3-8B bench + kernel profile after the RMSNorm rewrite
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_lm_gpu.py tests/test_ops_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_lm.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -8 gpurun_out/pytest_lm.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --model llama3-8b --steps 4 --warmup 2 > gpurun_out/bench_llama.log 2>&1 || exit $?
tail -1 gpurun_out/bench_llama.log | cut -c1-300
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_llama4 -o run -- python3 $R/bench.py --model llama3-8b --steps 2 --warmup 1 > $R/gpurun_out/prof_llama4.log 2>&1) || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_llama4 --steps 3 > gpurun_out/prof_llama4_summary.txt 2>&1
head -30 gpurun_out/prof_llama4_summary.txt | cut -c1-200
