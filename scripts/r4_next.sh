#!/bin/bash
# Round-4 measurement 4 (working tree): the warm-up ramp of the 20/5 driver config, the N>1
# projection on one GPU (xGMI-model probe communicator), and Llama-3-8B / ResNet-50 extension
# benches of round 2, round 3 and the working tree on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
timeout -k 10 300 python -u scripts/bench_ramp.py --warmup 5 --window 20 --windows 10 > gpurun_out/ramp.log 2>&1 || exit $?
tail -4 gpurun_out/ramp.log
timeout -k 10 600 python -u scripts/dp_projection.py --steps 40 --warmup 10 > gpurun_out/dp_projection.log 2>&1 || exit $?
cat gpurun_out/dp_projection.log | grep -v amdgpu
bash scripts/ab_trees.sh 1 .ab/r2 .ab/r3 . -- --model llama3-8b --steps 6 --warmup 3 > gpurun_out/ab_llama.log 2>&1 || exit $?
tail -3 gpurun_out/ab_llama.log
bash scripts/ab_trees.sh 1 .ab/r3 . -- --model resnet50 --dtype bf16 --steps 10 --warmup 4 > gpurun_out/ab_resnet.log 2>&1 || exit $?
tail -2 gpurun_out/ab_resnet.log
