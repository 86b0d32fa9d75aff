#!/bin/bash
# Round-4 measurement 19: the BN/engine GPU tests after dropping the BN backward's slab inputs; a
# same-box A/B of the single-launch small-layer BatchNorm threshold (CS_BN_FUSED_ROWS: 256 =
# blocks 6-7, the default; 1024 = blocks 4-7; 0 = none).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 180 --timeout-method thread \
  tests/test_native_engine_gpu.py tests/test_conv_bn_gpu.py > gpurun_out/r19_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r19_tests.log; [ $rc -eq 0 ] || exit $rc
V=". .:CS_BN_FUSED_ROWS=1024 .:CS_BN_FUSED_ROWS=0"
bash scripts/ab_trees.sh 3 $V -- --steps 20 --warmup 5 > gpurun_out/ab10_20_5.log 2>&1 || exit $?
tail -3 gpurun_out/ab10_20_5.log
bash scripts/ab_trees.sh 2 $V -- --steps 100 --warmup 10 > gpurun_out/ab10_100_10.log 2>&1 || exit $?
tail -3 gpurun_out/ab10_100_10.log
