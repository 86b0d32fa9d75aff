# round 2: price the data-parallel plumbing of the C++ step on one GPU (world 1):
# none | fork/join events only (ProbeComm nop) | one-rank RCCL (+ event flag variants, 1 bucket)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="timeout -k 10 120 python bench.py --steps 300 --warmup 30"
run() { echo "== $1"; shift; env "$@" $B > gpurun_out/plumb.log 2>&1 || { tail -5 gpurun_out/plumb.log; exit 1; }; tail -1 gpurun_out/plumb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
run none CS_COMM_PROBE=0
run events_only CS_COMM_PROBE=order CS_PROBE_SPIN=-1
run rccl CS_COMM_PROBE=1
run rccl_flags0 CS_COMM_PROBE=1 CS_COMM_EVENT_FLAGS=0
run rccl_flags2 CS_COMM_PROBE=1 CS_COMM_EVENT_FLAGS=2
run none2 CS_COMM_PROBE=0
run rccl2 CS_COMM_PROBE=1
run events_only2 CS_COMM_PROBE=order CS_PROBE_SPIN=-1
