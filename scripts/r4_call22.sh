#!/bin/bash
# Round-4 measurement 22 (experiment): the step's main stream at high hardware-queue priority
# (CS_MAIN_PRIO=1, bench.py) vs the default-priority current stream, next to the low-priority
# side stream; same box, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -c "import torch; print(torch.cuda.Stream(priority=-1).priority, torch.cuda.Stream().priority)" || exit $?
V=". .:CS_MAIN_PRIO=1"
bash scripts/ab_trees.sh 3 $V -- --steps 20 --warmup 5 > gpurun_out/ab12_20_5.log 2>&1 || exit $?
tail -2 gpurun_out/ab12_20_5.log
bash scripts/ab_trees.sh 2 $V -- --steps 100 --warmup 10 > gpurun_out/ab12_100_10.log 2>&1 || exit $?
tail -2 gpurun_out/ab12_100_10.log
