# short-run bench variance: 5 fresh processes at --steps 20 --warmup 10
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2 3 4 5; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 10 > gpurun_out/short_$i.log 2>&1 || exit $?
  echo "run $i $(tail -1 gpurun_out/short_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
for i in 1 2; do
  CS_OVERLAP_WGRAD=0 timeout -k 10 120 python bench.py --steps 20 --warmup 10 > gpurun_out/short_s$i.log 2>&1 || exit $?
  echo "serial $i $(tail -1 gpurun_out/short_s$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
