# side-stream SGD: engine + distributed tests, then A/B bench on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_native_engine_gpu.py > gpurun_out/pytest_sgds_eng.log 2>&1
rc=$?; echo "pytest(engine) exit $rc"; tail -5 gpurun_out/pytest_sgds_eng.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
  tests/test_native_distributed_gpu.py > gpurun_out/pytest_sgds_comm.log 2>&1
rc=$?; echo "pytest(comm) exit $rc"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_sgds_comm.log | tail -30
[ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  CS_SGD_SIDE=$v timeout -k 10 200 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_sgds_$v.log 2>&1 || exit $?
  echo "CS_SGD_SIDE=$v $(tail -1 gpurun_out/bench_sgds_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
