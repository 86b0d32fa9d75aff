#!/bin/bash
# A/B of engine env toggles on one box: bash scripts/ab_env.sh "VAR=a" "VAR=b" [rounds] [bench args]
# Alternates the configs `rounds` times (default 2), one bench.py process per run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
A=$1; B=$2; N=${3:-2}; shift 3 || shift $#
[ $# -eq 0 ] && set -- --steps 100 --warmup 10
for i in $(seq 1 "$N"); do
  for cfg in "$A" "$B"; do
    out=$(env $cfg timeout -k 10 300 python -u bench.py "$@" 2>>gpurun_out/ab_env.err | tail -1) || exit $?
    echo "$cfg => $(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['value'], d['ms_per_step'])" "$out")"
  done
done
