#!/bin/bash
# Round-4 measurement 3: side-stream weight gradients restored on the pruned engine (.ab/r4c), with
# and without the in-launch BN finalize, against round 2 (.ab/r2) and round 3 (.ab/r3) on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
(cd .ab/r4d && timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_native_engine_gpu.py -k "side_stream or long_run or bench_config_b64 or sgd_in_wgrad or graph" \
  > ../../gpurun_out/r4d_tests.log 2>&1)
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4d_tests.log | tail -20; echo "r4d pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
V=".ab/r2 .ab/r3 .ab/r4c .ab/r4d .ab/r4d:CS_BN_FIN=0 .ab/r4d:CS_OVERLAP_WGRAD=0"
bash scripts/ab_trees.sh 3 $V -- --steps 20 --warmup 5 > gpurun_out/ab3_20_5.log 2>&1 || exit $?
tail -5 gpurun_out/ab3_20_5.log
bash scripts/ab_trees.sh 2 $V -- --steps 100 --warmup 10 > gpurun_out/ab3_100_10.log 2>&1 || exit $?
tail -5 gpurun_out/ab3_100_10.log
(cd .ab/r4d && GRAFT_REPO_ROOT=$PWD bash scripts/gpu.sh trace r4d_trace --steps 10 --warmup 5) && mkdir -p gpurun_out/r4d && cp -r .ab/r4d/gpurun_out/. gpurun_out/r4d/
