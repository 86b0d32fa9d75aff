set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -s -p no:cacheprovider --timeout 240 --timeout-method thread \
  tests/test_native_engine_gpu.py -k "fp64 or ragged" > gpurun_out/pytest_r2parity.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASS|FAIL|Error|assert|\[parity\]" gpurun_out/pytest_r2parity.log | tail -40; exit $rc
