# per-bucket SGD overlap: engine GPU tests, then A/B bench (tuned tiles reused)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_native_engine_gpu.py tests/test_native_distributed_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_sgdovl.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_sgdovl.log; [ $rc -eq 0 ] || exit $rc
export CS744_TUNE_CACHE=gpurun_out/tune_sgdovl.json
for o in 1 0 1; do
  CS_SGD_OVERLAP=$o timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 > gpurun_out/bench_sgdovl_$o.log 2>&1 || exit $?
  echo "overlap=$o $(tail -1 gpurun_out/bench_sgdovl_$o.log | cut -c1-130)"
done
