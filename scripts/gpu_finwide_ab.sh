# BN finalize: wide (8-channel / 1024-thread) kernel for >= 512 partials vs one wave per channel
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_conv_bn_gpu.py tests/test_native_engine_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "finalize_many or bn_relu_pool or bn_eval or engine" > gpurun_out/finwide_tests.log 2>&1 || { tail -30 gpurun_out/finwide_tests.log; exit 1; }
tail -1 gpurun_out/finwide_tests.log
export CS744_TUNE_CACHE=$R/gpurun_out/tune_finwide.json
for W in 512 0 512 0; do
  CS_BN_FIN_WIDE=$W timeout -k 10 300 python bench.py --steps 300 --warmup 20 > gpurun_out/finwide_$W.log 2>&1 || exit $?
  echo "wide_min=$W $(tail -1 gpurun_out/finwide_$W.log | cut -c60-140)"
done
for W in 512 0; do
  cd /tmp && CS_BN_FIN_WIDE=$W timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_fw$W -o run -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof_fw$W.log 2>&1 || exit $?
  cd $R
done
