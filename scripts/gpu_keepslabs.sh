# kept split-K dgrad slabs: engine + BN tests, A/B bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_native_engine_gpu.py tests/test_conv_bn_gpu.py -k "engine or slabs or bn_relu or dual or fp64 or graph" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_keep.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_keep.log; [ $rc -eq 0 ] || exit $rc
export CS744_TUNE_CACHE=gpurun_out/tune_keep.json
for k in 1 0 1 0; do
  CS_KEEP_SLABS=$k timeout -k 10 300 python3 bench.py --steps 400 --warmup 20 > gpurun_out/bench_keep.log 2>&1 || exit $?
  echo "keep=$k $(tail -1 gpurun_out/bench_keep.log | cut -c60-100)"
done
