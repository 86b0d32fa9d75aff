#!/bin/bash
# Round-4 measurement 13: the round-end set on the new defaults (every GPU test, smoke(), the
# default bench), then a kernel trace of the default step for profiles/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
bash scripts/gpu.sh suite || exit $?
bash scripts/gpu.sh trace r4_final --steps 10 --warmup 5
