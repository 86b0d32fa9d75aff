#!/bin/bash
# Round-4 measurement 7: extension configs on the native bf16 GEMM vs hipBLASLt, same box,
# interleaved: Llama-3-8B (CS_LM_GEMM) and ResNet-50 bf16 B=256 (CS_CONV_GEMM, with the GEMM-epilogue
# BatchNorm statistics), plus a rocprofv3 kernel table of the GEMM A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
bash scripts/ab_trees.sh 2 .:CS_LM_GEMM=blas .:CS_LM_GEMM=native -- --model llama3-8b --steps 6 --warmup 3 \
  > gpurun_out/ab_llama_gemm.log 2>&1 || exit $?
tail -2 gpurun_out/ab_llama_gemm.log
bash scripts/ab_trees.sh 2 .:CS_CONV_GEMM=blas .:CS_CONV_GEMM=auto .:CS_CONV_GEMM=native -- --model resnet50 \
  --dtype bf16 --steps 10 --warmup 4 > gpurun_out/ab_resnet_gemm.log 2>&1 || exit $?
tail -3 gpurun_out/ab_resnet_gemm.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/gemm_prof -o run -- \
  python3 $R/scripts/gemm_bench.py --rounds 1 --reps 3 > $R/gpurun_out/gemm_prof.log 2>&1)
echo "rocprofv3 rc=$?"
