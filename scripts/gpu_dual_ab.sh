# engine + conv numerics, then bench A/B of the dual wgrad+dgrad launch
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_native_engine_gpu.py tests/test_conv_bn_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_conv.log; [ $rc -eq 0 ] || exit $rc

for D in 1 0; do
  CS_TUNE_VERBOSE=1 CS_CONV_DUAL=$D CS744_TUNE_CACHE=$GRAFT_REPO_ROOT/gpurun_out/tune_dual$D.json timeout -k 10 300 python bench.py --steps 200 --warmup 20 > gpurun_out/bench_dual$D.log 2>&1 || exit $?
  grep "\[tune\]" gpurun_out/bench_dual$D.log; echo "dual=$D $(tail -1 gpurun_out/bench_dual$D.log | cut -c1-160)"
done
