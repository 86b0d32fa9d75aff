#!/bin/bash
# Same-box A/B of source trees (each with its own built _C.so), interleaved:
#   bash scripts/ab_trees.sh ROUNDS TREE[:VAR=VAL[,VAR=VAL]]... [-- bench.py args]
# e.g. TREE = .ab/r2 (a `git worktree add .ab/r2 <commit>` built in place), . (the working tree), or
# .:CS_ENGINE_OFF=side_sgd_tail (the working tree with an environment override). One bench.py process per run,
# the variants alternating ROUNDS times, so clock and thermal drift on the box hit every variant
# alike. Prints one line per run and a median per variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
N=$1; shift
TREES=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do TREES+=("$1"); shift; done
[ "$1" = "--" ] && shift
[ $# -eq 0 ] && set -- --steps 20 --warmup 5
R=$PWD
: > gpurun_out/ab_trees.tmp
for i in $(seq 1 "$N"); do
  for spec in "${TREES[@]}"; do
    t=${spec%%:*}; envs=""
    [ "$spec" != "$t" ] && envs=${spec#*:}
    out=$(cd "$t" && env ${envs//,/ } timeout -k 10 300 python -u bench.py "$@" 2>>"$R/gpurun_out/ab_trees.err" | tail -1) || exit $?
    v=$(python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(d['value'], d['ms_per_step'], (d.get('calibration') or {}).get('mfma_bf16_gemm_tflops'))" "$out") || exit $?
    echo "$spec $v" | tee -a gpurun_out/ab_trees.tmp
  done
done
python3 - "$*" "${TREES[@]}" <<'PY'
import statistics, sys
rows = [l.split() for l in open("gpurun_out/ab_trees.tmp") if l.strip()]
for t in sys.argv[2:]:
    v = [float(r[1]) for r in rows if r[0] == t]
    print(f"# {t}: median {statistics.median(v):.0f} img/s over {len(v)} runs ({sys.argv[1]}); all {v}")
PY
