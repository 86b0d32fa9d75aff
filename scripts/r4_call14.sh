#!/bin/bash
# Round-4 measurement 14: BatchNorm-backward partial sums in the data-gradient epilogue (default)
# vs the BN backward's own reduce pass (CS_BN_EPI_RED=0), side-stream schedule, one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_native_engine_gpu.py -k "bench_config_b64 and (autotuned or dual)" > gpurun_out/ered_tests.log 2>&1 || exit $?
CS_BN_EPI_RED=0 timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
  tests/test_native_engine_gpu.py -k "bench_config_b64 and (autotuned or dual or split)" >> gpurun_out/ered_tests.log 2>&1 || exit $?
tail -2 gpurun_out/ered_tests.log
V=". .:CS_BN_EPI_RED=0"
bash scripts/ab_trees.sh 3 $V -- --steps 20 --warmup 5 > gpurun_out/ab6_20_5.log 2>&1 || exit $?
tail -2 gpurun_out/ab6_20_5.log
bash scripts/ab_trees.sh 2 $V -- --steps 100 --warmup 10 > gpurun_out/ab6_100_10.log 2>&1 || exit $?
tail -2 gpurun_out/ab6_100_10.log
bash scripts/ab_trees.sh 1 .ab/r2 .ab/r3 .:CS_LM_GEMM=blas . -- --model llama3-8b --steps 6 --warmup 3 \
  > gpurun_out/ab_llama_r2r3r4.log 2>&1 || exit $?
tail -4 gpurun_out/ab_llama_r2r3r4.log
