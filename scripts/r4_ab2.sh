#!/bin/bash
# Round-4, second measurement: the appended BN-apply tree (.ab/r4b) — its GPU tests, then an
# interleaved A/B against the finalize-only tree (.ab/r4a) at 20/5 and 100/10, then its step trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
(cd .ab/r4b && timeout -k 10 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_native_engine_gpu.py -k "appended or in_launch or b64_matches_fp64 or long_run or graph or ragged or sgd_in_wgrad" \
  tests/test_conv_bn_gpu.py -k "in_launch" \
  > ../../gpurun_out/r4b_tests.log 2>&1)
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4b_tests.log | tail -40; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_trees.sh 3 .ab/r4a .ab/r4b -- --steps 20 --warmup 5 > gpurun_out/ab2_20_5.log 2>&1 || exit $?
tail -2 gpurun_out/ab2_20_5.log
bash scripts/ab_trees.sh 2 .ab/r4a .ab/r4b -- --steps 100 --warmup 10 > gpurun_out/ab2_100_10.log 2>&1 || exit $?
tail -2 gpurun_out/ab2_100_10.log
(cd .ab/r4b && GRAFT_REPO_ROOT=$PWD bash scripts/gpu.sh trace r4_app --steps 10 --warmup 5) && mkdir -p gpurun_out/r4b && cp -r .ab/r4b/gpurun_out/. gpurun_out/r4b/
