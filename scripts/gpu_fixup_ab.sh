# conv numerics (incl. in-launch split-K fixup) + engine tests + bench A/B of CS_CONV_FIXUP
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_bn_gpu.py tests/test_native_engine_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_conv.log; [ $rc -eq 0 ] || exit $rc
for F in 1 0; do
  CS_CONV_FIXUP=$F CS744_TUNE_CACHE=$GRAFT_REPO_ROOT/gpurun_out/tune_fix$F.json timeout -k 10 300 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_fix$F.log 2>&1 || exit $?
  echo "fixup=$F $(tail -1 gpurun_out/bench_fix$F.log | cut -c1-200)"
done
