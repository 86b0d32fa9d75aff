# Step-level A/B of engine knobs on one GPU (100 timed steps each): BN path x grid-barrier version,
# kept split-K slabs, in-launch split-K combine. One bench.py process per configuration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
CFGS=${AB_CFGS:-"CS_BN_PATH=0|CS_BN_PATH=2 CS_BN_GRID_BARV=1|CS_BN_PATH=2 CS_BN_GRID_BARV=2|CS_BN_PATH=0 CS_KEEP_SLABS=1|CS_BN_PATH=0 CS_CONV_FIXUP=1|CS_BN_PATH=2 CS_BN_GRID_BARV=2 CS_KEEP_SLABS=1|CS_BN_PATH=0"}
IFS='|'
for cfg in $CFGS; do
  IFS=' ' read -r -a kv <<< "$cfg"
  env "${kv[@]}" timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 > gpurun_out/ab.log 2>&1 || { rc=$?; tail -5 gpurun_out/ab.log; exit $rc; }
  echo "$cfg => $(tail -1 gpurun_out/ab.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
