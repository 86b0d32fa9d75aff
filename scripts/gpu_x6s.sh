# X6S (split at LDS store) numerics + x6-family and all-math tuned benches
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_bn_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_x6s.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -15 gpurun_out/pytest_x6s.log; [ $rc -eq 0 ] || exit $rc
for m in 2 1; do
  CS_CONV_MATH=$m CS744_TUNE_CACHE=gpurun_out/tune_x6s_$m.json timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 > gpurun_out/bench_x6s_$m.log 2>&1 || exit $?
  echo "math=$m $(tail -1 gpurun_out/bench_x6s_$m.log | cut -c1-130)"
done
