# 16 hardware queues: base step time, and the one-rank NCCL group + 8 extra streams case that
# shared the side stream's queue at 8
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
one() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 200 python scripts/bench_ramp.py --windows 3 "$@" > gpurun_out/q3_$tag.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/q3_$tag.log; return 1; }
  echo "$tag $(grep window gpurun_out/q3_$tag.log | tail -1)"
}
export GPU_MAX_HW_QUEUES=16
one q16_base && one q16_ncclpg_x8 --nccl-pg --extra-streams 8 && one q16_x12 --extra-streams 12 && \
GPU_MAX_HW_QUEUES=8 one q8_base
