# (1) bench warmup/steps sensitivity on one box; (2) X6S split-arithmetic probe (wrong numbers,
# timing only) against the normal build
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # tag, dir, args...
  local tag=$1 dir=$2; shift 2
  timeout -k 10 200 python $dir/bench.py "$@" > gpurun_out/bp_$tag.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/bp_$tag.log; return 1; }
  echo "$tag $(tail -1 gpurun_out/bp_$tag.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run s20w10 . --steps 20 --warmup 10 && run s50w10 . --steps 50 --warmup 10 && run s300w30 . --steps 300 --warmup 30 && \
run s20w300 . --steps 20 --warmup 300 && run probe_s300 _probe --steps 300 --warmup 30 && run s300w30b . --steps 300 --warmup 30
