# which stream is hurt by hardware-queue sharing, and does a one-rank NCCL process group (what a
# multi-GPU job brings up before the trainer) reproduce it?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
one() {  # tag, args...
  local tag=$1; shift
  timeout -k 10 200 python scripts/bench_ramp.py --windows 3 "$@" > gpurun_out/q2_$tag.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/q2_$tag.log; return 1; }
  echo "$tag $(grep window gpurun_out/q2_$tag.log | tail -1)"
}
one ovl_before --extra-streams 40 && { export CS_OVERLAP_WGRAD=0; one serial_before --extra-streams 40; rc=$?; unset CS_OVERLAP_WGRAD; [ $rc -eq 0 ]; } && \
one ncclpg --nccl-pg && one ncclpg_x8 --nccl-pg --extra-streams 8 && one base
