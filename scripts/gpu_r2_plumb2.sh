set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="timeout -k 10 120 python bench.py --steps 300 --warmup 30"
run() { echo "== $1"; shift; env "$@" $B > gpurun_out/plumb.log 2>&1 || { tail -5 gpurun_out/plumb.log; exit 1; }; tail -1 gpurun_out/plumb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
run none CS_COMM_PROBE=0
run none_stream CS_COMM_PROBE=0 CS_STEP_STREAM=1
run events_only_stream CS_COMM_PROBE=order CS_PROBE_SPIN=-1 CS_STEP_STREAM=1
run rccl_stream CS_COMM_PROBE=1 CS_STEP_STREAM=1
run events_only CS_COMM_PROBE=order CS_PROBE_SPIN=-1
