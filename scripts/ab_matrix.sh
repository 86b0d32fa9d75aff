#!/bin/bash
# Interleaved A/B/... of bench.py configs on one box: bash scripts/ab_matrix.sh ROUNDS "ENV ARGS" ...
# Each config is "VAR=v VAR2=w -- --bench-arg x" (env before --, bench.py args after); every round
# runs each config once (one process each), default 100 timed / 10 warmup steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
N=$1; shift
for i in $(seq 1 "$N"); do
  for cfg in "$@"; do
    envs=${cfg%%--*}; args=""
    [[ "$cfg" == *--* ]] && args=${cfg#*--}
    out=$(env $envs timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 $args 2>>gpurun_out/ab_matrix.err | tail -1) || exit $?
    echo "[$cfg] => $(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['value'], d['ms_per_step'])" "$out")"
  done
done
