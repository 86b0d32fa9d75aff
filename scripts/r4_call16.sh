#!/bin/bash
# Round-4 measurement 16: small-layer BN backward from the data gradient's split-K slabs —
# numerics, then same-box A/B (default = forward tail + backward slabs) vs each turned off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
timeout -k 10 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_native_engine_gpu.py -k "from_slabs or bench_config_b64 or side_stream or long_run or fp64 or graph" \
  > gpurun_out/slab_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/slab_tests.log | tail -30; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
V=". .:CS_BN_BWD_SLABS=0"
bash scripts/ab_trees.sh 3 $V -- --steps 20 --warmup 5 > gpurun_out/ab8_20_5.log 2>&1 || exit $?
tail -3 gpurun_out/ab8_20_5.log
bash scripts/ab_trees.sh 2 $V -- --steps 100 --warmup 10 > gpurun_out/ab8_100_10.log 2>&1 || exit $?
tail -3 gpurun_out/ab8_100_10.log
