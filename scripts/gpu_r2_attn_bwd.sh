# round-2: attention backward — heaviest-first dK/dV grid (default) and the one-launch fused variant:
# attention GPU tests, then the Llama-3-8B step A/B and a kernel profile of the default
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py tests/test_lm_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_attn.log
[ $rc -eq 0 ] || exit $rc
CS_ATTN_BWD_FUSED=1 timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_attn_fused.log 2>&1
rc=$?; echo "pytest (fused) exit $rc"; tail -2 gpurun_out/pytest_attn_fused.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model llama3-8b --steps 4 --warmup 2 > gpurun_out/bench_llama_lpt.log 2>&1 || exit $?
echo "lpt: $(tail -1 gpurun_out/bench_llama_lpt.log | cut -c1-200)"
CS_ATTN_BWD_FUSED=1 timeout -k 10 300 python bench.py --model llama3-8b --steps 4 --warmup 2 > gpurun_out/bench_llama_fused.log 2>&1 || exit $?
echo "fused: $(tail -1 gpurun_out/bench_llama_fused.log | cut -c1-200)"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_llama5 -o run -- python3 $R/bench.py --model llama3-8b --steps 2 --warmup 1 > $R/gpurun_out/prof_llama5.log 2>&1) || exit $?
python3 scripts/prof_summary.py gpurun_out/prof_llama5 --steps 3 > gpurun_out/prof_llama5_summary.txt 2>&1
grep -E "attn_" gpurun_out/prof_llama5_summary.txt | head -6 | cut -c1-160
