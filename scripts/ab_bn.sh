set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
for cfg in "CS_BN_PATH=2 CS_DEFER_SIGNALS=1" "CS_BN_PATH=0 CS_DEFER_SIGNALS=1" "CS_BN_PATH=2 CS_DEFER_SIGNALS=0" "CS_BN_PATH=0 CS_DEFER_SIGNALS=0" "CS_BN_PATH=1 CS_DEFER_SIGNALS=0" "CS_BN_PATH=2 CS_DEFER_SIGNALS=1"; do
  env $cfg timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > gpurun_out/ab.log 2>&1 || exit $?
  echo "$cfg $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
