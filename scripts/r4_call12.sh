#!/bin/bash
# Round-4 measurement 12: bench window experiment after moving the GC pass before the warmup.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
timeout -k 10 600 python -u scripts/bench_windows.py --rounds 2 > gpurun_out/bench_windows2.log 2>&1 || exit $?
cat gpurun_out/bench_windows2.log
V=".ab/r2 . .:CS_BN_FIN=0"
bash scripts/ab_trees.sh 3 $V -- --steps 20 --warmup 5 > gpurun_out/ab5_20_5.log 2>&1 || exit $?
tail -3 gpurun_out/ab5_20_5.log
bash scripts/ab_trees.sh 2 $V -- --steps 100 --warmup 10 > gpurun_out/ab5_100_10.log 2>&1 || exit $?
tail -3 gpurun_out/ab5_100_10.log
