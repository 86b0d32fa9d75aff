# the side stream reserved before other streams exist: does it keep its own hardware queue?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
one() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 200 python scripts/bench_ramp.py --windows 3 "$@" > gpurun_out/q4_$tag.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/q4_$tag.log; return 1; }
  echo "$tag $(grep window gpurun_out/q4_$tag.log | tail -1)"
}
one reserved_x40 --reserve-first --extra-streams 40 && one reserved_ncclpg_x8 --reserve-first --nccl-pg --extra-streams 8 && \
one late_x40 --extra-streams 40 && timeout -k 10 120 python bench.py --steps 100 --warmup 20 > gpurun_out/q4_bench.log 2>&1 && tail -1 gpurun_out/q4_bench.log
