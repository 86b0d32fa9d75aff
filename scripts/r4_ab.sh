#!/bin/bash
# Round-4 measurement on one box: GPU tests of the appended BN-apply tree (.ab/r4b: fp64 parity at
# every in-launch finalize / apply site, bitwise apply equivalence), then round-2 (.ab/r2 =
# d2c2e4c), round-3 (.ab/r3 = 5ac3e03), r4a (in-launch finalize) and r4b interleaved at the
# driver's 20/5 config and at 100/10, then kernel traces. Test failures are reported, not fatal;
# a crash / abort / time limit ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
(cd .ab/r4b && timeout -k 10 600 python -u -m pytest -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_native_engine_gpu.py -k "bench_config_b64 or appended or in_launch" \
  > ../../gpurun_out/r4b_tests.log 2>&1)
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r4b_tests.log | tail -30; echo "r4b pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
TREES=".ab/r2 .ab/r3 .ab/r4a .ab/r4b"
bash scripts/ab_trees.sh 3 $TREES -- --steps 20 --warmup 5 > gpurun_out/ab_20_5.log 2>&1 || exit $?
tail -4 gpurun_out/ab_20_5.log
bash scripts/ab_trees.sh 2 $TREES -- --steps 100 --warmup 10 > gpurun_out/ab_100_10.log 2>&1 || exit $?
tail -4 gpurun_out/ab_100_10.log
for t in r4a r4b; do
  (cd .ab/$t && GRAFT_REPO_ROOT=$PWD bash scripts/gpu.sh trace ${t}_trace --steps 10 --warmup 5) || exit $?
  mkdir -p gpurun_out/$t && cp -r .ab/$t/gpurun_out/. gpurun_out/$t/
done
