# dual X6S backward launch: engine tests, then tuned bench (verbose dual choice)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_native_engine_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_dualxs.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 gpurun_out/pytest_dualxs.log; [ $rc -eq 0 ] || exit $rc
CS_TUNE_VERBOSE=1 CS744_TUNE_CACHE=gpurun_out/tune_dualxs.json timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 > gpurun_out/bench_dualxs.log 2>&1 || exit $?
grep "dual" gpurun_out/bench_dualxs.log | tail -8; tail -1 gpurun_out/bench_dualxs.log | cut -c1-130
