# engine + conv GPU tests, then a tuned bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_native_engine_gpu.py tests/test_native_distributed_gpu.py tests/test_conv_bn_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_quick.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_launch_probe.sh
