set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
  tests/test_asan_runtime_gpu.py > gpurun_out/pytest_asan.log 2>&1
rc=$?; echo "asan test exit $rc"; tail -3 gpurun_out/pytest_asan.log
ASAN_OPTIONS=detect_leaks=0:detect_container_overflow=0 timeout -k 10 200 ./cs744_pytorch_distributed_tutorial_amd/bin/asan_runtime_test > gpurun_out/asan_run.log 2>&1; echo "asan exe rc $?"; grep -v amdgpu.ids gpurun_out/asan_run.log | tail -15
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r2_sgd.sh
