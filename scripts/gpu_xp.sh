#!/bin/bash
# XP (pre-split) conv GEMMs: numerics tests (+ extra test files given as args), then the graph-timed
# VGG-11 shape sweep (only if nothing crashed)
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_xp_gpu.py "$@" \
  > gpurun_out/xp_tests.log 2>&1
rc=$?
tail -15 gpurun_out/xp_tests.log
echo "pytest rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 600 python -u scripts/xp_bench.py 64 10 > gpurun_out/xp_bench.log 2>&1
  echo "bench rc=$?"
  grep -v amdgpu.ids gpurun_out/xp_bench.log
fi
