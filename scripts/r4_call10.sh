#!/bin/bash
# Round-4 measurement 10: bench window-length experiment, warm-up ramp and probe projection with
# the side stream kept (>= 8 HIP queues), extension A/Bs after the split-K / policy fixes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
timeout -k 10 600 python -u scripts/bench_windows.py --rounds 2 > gpurun_out/bench_windows.log 2>&1 || exit $?
cat gpurun_out/bench_windows.log
timeout -k 10 300 python -u scripts/bench_ramp.py --warmup 5 --window 20 --windows 8 > gpurun_out/ramp.log 2>&1 || exit $?
grep window gpurun_out/ramp.log | head -3
timeout -k 10 500 python -u scripts/dp_projection.py --steps 40 --warmup 10 --gbps 150,300 --ctas 0,16 \
  > gpurun_out/dp_projection.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/dp_projection.log | cut -c1-220
bash scripts/ab_trees.sh 2 .:CS_LM_GEMM=blas .:CS_LM_GEMM=wgrad -- --model llama3-8b --steps 6 --warmup 3 \
  > gpurun_out/ab_llama_gemm.log 2>&1 || exit $?
tail -2 gpurun_out/ab_llama_gemm.log
bash scripts/ab_trees.sh 2 .:CS_CONV_GEMM=blas .:CS_CONV_GEMM=auto -- --model resnet50 --dtype bf16 --steps 10 \
  --warmup 4 > gpurun_out/ab_resnet_gemm.log 2>&1 || exit $?
tail -2 gpurun_out/ab_resnet_gemm.log
