#!/bin/bash
# Cross-process A/B of the conv math on the VGG-11 step: one process per run, arms alternating
# (scripts/f3_probe.py), N rounds. Usage (GPU box): bash scripts/f3_ab.sh N "arm1 arm2 ..." [probe args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
N=${1:-3}; ARMS=${2:-"base f3"}; shift 2 || true
for i in $(seq 1 "$N"); do
  for arm in $ARMS; do
    timeout -k 10 180 python3 scripts/f3_probe.py --arm "$arm" "$@" >> gpurun_out/f3_ab.jsonl 2> gpurun_out/f3_ab_err.log || exit $?
    tail -1 gpurun_out/f3_ab.jsonl
  done
done
