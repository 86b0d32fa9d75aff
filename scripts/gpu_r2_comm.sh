# round 2: multi-rank C++ step (staged comm), ordering probe, abort path, entrypoint defaults,
# native resume; then the engine tests and a quick bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
  tests/test_native_distributed_gpu.py tests/test_entrypoints_gpu.py > gpurun_out/pytest_r2comm.log 2>&1
rc=$?; echo "pytest(comm) exit $rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_r2comm.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_native_engine_gpu.py tests/test_ops_gpu.py > gpurun_out/pytest_r2eng.log 2>&1
rc=$?; echo "pytest(engine) exit $rc"; tail -5 gpurun_out/pytest_r2eng.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_r2comm.log 2>&1; rc=$?
tail -1 gpurun_out/bench_r2comm.log; exit $rc
