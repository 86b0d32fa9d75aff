set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_native_engine_gpu.py -x -q -p no:cacheprovider > gpurun_out/pytest_engine.log 2>&1
rc=$?
echo "pytest exit $rc"; tail -30 gpurun_out/pytest_engine.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -3 gpurun_out/smoke.log && \
timeout -k 10 300 python bench.py --steps 100 --warmup 20 > gpurun_out/bench_native.log 2>&1; rc=$?
tail -5 gpurun_out/bench_native.log
exit $rc
