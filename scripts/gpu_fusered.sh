# BN partial-sum pass appended to the weight-gradient launch: engine tests, A/B bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_native_engine_gpu.py tests/test_conv_bn_gpu.py -k "not conv_fwd and not conv_dgrad and not conv_wgrad" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_fusered.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_fusered.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_conv_bn_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_fusered_conv.log 2>&1
rc=$?; echo "conv pytest exit $rc"; tail -2 gpurun_out/pytest_fusered_conv.log; [ $rc -eq 0 ] || exit $rc
export CS744_TUNE_CACHE=gpurun_out/tune_fusered.json
for f in 1 0 1 0; do
  CS_FUSE_BN_RED=$f timeout -k 10 300 python3 bench.py --steps 400 --warmup 20 > gpurun_out/bench_fusered.log 2>&1 || exit $?
  echo "fuse=$f $(tail -1 gpurun_out/bench_fusered.log | cut -c60-100)"
done
