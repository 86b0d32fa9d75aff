#!/bin/bash
# Round-4 measurement 17 (end of round): every GPU test, smoke(), the default bench; the default
# step's kernel trace; the probe projection on the final engine.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
bash scripts/gpu.sh suite || exit $?
bash scripts/gpu.sh trace r4_end --steps 10 --warmup 5 || exit $?
timeout -k 10 500 python -u scripts/dp_projection.py --steps 40 --warmup 10 --gbps 150,300 --ctas 0,16 \
  > gpurun_out/dp_projection_end.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/dp_projection_end.log | cut -c1-200
