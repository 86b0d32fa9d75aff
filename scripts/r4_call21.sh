#!/bin/bash
# Round-4 measurement 21: the shipped conv tile table (tuned in round 1) vs a table re-tuned on
# this round's kernels (CS744_TUNE=1, written to a cache by the first run and reused by the rest),
# same box, interleaved; the re-tuned table is kept in gpurun_out/ for shipping.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
rm -f /tmp/tune_r4.json
V=". .:CS744_TUNE=1,CS744_TUNE_CACHE=/tmp/tune_r4.json"
bash scripts/ab_trees.sh 3 $V -- --steps 20 --warmup 5 > gpurun_out/ab11_20_5.log 2>&1 || exit $?
tail -2 gpurun_out/ab11_20_5.log
cp /tmp/tune_r4.json gpurun_out/tune_r4.json || exit 1
bash scripts/ab_trees.sh 2 $V -- --steps 100 --warmup 10 > gpurun_out/ab11_100_10.log 2>&1 || exit $?
tail -2 gpurun_out/ab11_100_10.log
