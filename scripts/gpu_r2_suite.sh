# full GPU suite + smoke + default bench (what the driver runs at round end)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -5 gpurun_out/pytest_gpu_full.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke exit $rc"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1; rc=$?
tail -1 gpurun_out/bench_default.log; exit $rc
