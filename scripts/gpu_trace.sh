#!/bin/bash
# Kernel + marker trace of the default bench step (side-stream weight gradients): per-kernel table,
# one-step per-queue timeline (scripts/step_timeline.py). Args: tag [extra bench args]
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
TAG=${1:-trace}; shift
timeout -k 10 200 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?
(cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --marker-trace --stats -d $R/gpurun_out/$TAG -o run -- \
  python3 $R/bench.py --steps 10 --warmup 5 "$@" > $R/gpurun_out/$TAG.log 2>&1)
rc=$?; echo "rocprofv3 rc=$rc"; tail -1 gpurun_out/$TAG.log
[ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py gpurun_out/$TAG --steps 15 --top 45 > gpurun_out/${TAG}_kernels.txt 2>&1
python3 scripts/step_timeline.py gpurun_out/$TAG > gpurun_out/${TAG}_timeline.txt 2>&1
head -3 gpurun_out/${TAG}_kernels.txt; grep -E "^# one step|^## queue|^# queue|^# main" gpurun_out/${TAG}_timeline.txt
