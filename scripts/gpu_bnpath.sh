# BN launch path A/B: numerics (BN + engine tests), then tuned bench with CS_BN_PATH=1/0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_bn_gpu.py -k "bn" tests/test_native_engine_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_bnpath.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_bnpath.log; [ $rc -eq 0 ] || exit $rc
export CS744_TUNE_CACHE=gpurun_out/tune_bnpath.json
for b in 1 0 1; do
  CS_BN_PATH=$b timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 > gpurun_out/bench_bnpath_$b.log 2>&1 || exit $?
  echo "bnpath=$b $(tail -1 gpurun_out/bench_bnpath_$b.log | cut -c1-130)"
done
