# round 2: price the C++ step's data-parallel plumbing on one GPU (world 1) by bucket count,
# HIP-event fork/join (CS_COMM_FORK=0) vs kernel stream links (CS_COMM_FORK=2); then the
# ordering-probe tests under stream links
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="timeout -k 10 120 python bench.py --steps 300 --warmup 30"
run() { echo "== $1"; shift; env "$@" > gpurun_out/plumb.log 2>&1 || { tail -5 gpurun_out/plumb.log; exit 1; }; tail -1 gpurun_out/plumb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
run none CS_COMM_PROBE=0 $B
for f in 0 2; do
for mb in 1000000 9 4 1; do
run fork${f}_events_bucket$mb CS_COMM_FORK=$f CS_COMM_PROBE=order CS_PROBE_SPIN=-1 $B --bucket-mb $mb
done
run fork${f}_rccl_bucket4 CS_COMM_FORK=$f CS_COMM_PROBE=1 $B
done
run none2 CS_COMM_PROBE=0 $B
CS_COMM_FORK=2 timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  tests/test_native_distributed_gpu.py -k "probe or abort or staged" > gpurun_out/pytest_links.log 2>&1
rc=$?; echo "link tests exit $rc"; tail -3 gpurun_out/pytest_links.log; exit $rc
