# classifier head kernels (register-cached W, prefetched dW rows): tests, bench, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_native_engine_gpu.py tests/test_native_distributed_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/hd_tests.log 2>&1 || { tail -30 gpurun_out/hd_tests.log; exit 1; }
tail -1 gpurun_out/hd_tests.log
export CS744_TUNE_CACHE=$R/gpurun_out/tune_hd.json
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 300 --warmup 20 > gpurun_out/hd_$i.log 2>&1 || exit $?
  echo "run $i $(tail -1 gpurun_out/hd_$i.log | cut -c60-140)"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_hd -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof_hd.log 2>&1 || exit $?
cd $R && python3 scripts/prof_summary.py gpurun_out/prof_hd --steps 25 --timeline 80 > gpurun_out/prof_hd_summary.txt 2>&1
head -30 gpurun_out/prof_hd_summary.txt | cut -c1-160
