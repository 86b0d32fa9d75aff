#!/bin/bash
# Round-4 measurement 20: ResNet-50 bf16 B=256 with the conv weight gradients on the native bf16
# GEMM (CS_CONV_GEMM=wgrad) vs hipBLASLt, same box, interleaved; its GPU test first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 180 --timeout-method thread \
  tests/test_gemm_bf16_gpu.py -k "bottleneck" > gpurun_out/r20_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r20_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_trees.sh 3 .:CS_CONV_GEMM=blas .:CS_CONV_GEMM=wgrad -- --model resnet50 --dtype bf16 --steps 10 --warmup 4 \
  > gpurun_out/ab_resnet_wgrad.log 2>&1 || exit $?
tail -3 gpurun_out/ab_resnet_wgrad.log
