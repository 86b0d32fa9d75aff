# conv numerics incl. LDS-DMA staging + engine tests + tuned bench (autotune picks staging per GEMM)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_bn_gpu.py tests/test_native_engine_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_conv.log; [ $rc -eq 0 ] || exit $rc
CS744_TUNE_CACHE=$GRAFT_REPO_ROOT/gpurun_out/tune_stage.json timeout -k 10 400 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_stage.log 2>&1 || exit $?
tail -1 gpurun_out/bench_stage.log | cut -c1-220
