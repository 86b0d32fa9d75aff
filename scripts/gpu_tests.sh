#!/bin/bash
# Selected GPU test files (args), one pytest process, each test bounded; then optional trace tag
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 180 --timeout-method thread "$@" > gpurun_out/tests_sel.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tests_sel.log | tail -40
echo "pytest rc=$rc"
exit $rc
