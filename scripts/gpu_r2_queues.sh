# HIP hardware-queue sharing vs the engine's kernel stream links: step time with 40 extra busy
# streams, by queue count and stream creation order
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # tag, env..., -- args
  local tag=$1; shift
  env "$@" timeout -k 10 200 python scripts/bench_ramp.py --windows 3 --extra-streams 40 ${EXTRA_ARGS} > gpurun_out/q_$tag.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/q_$tag.log; return 1; }
  echo "$tag $(grep window gpurun_out/q_$tag.log | tail -1) $(grep -c 'links ok' gpurun_out/q_$tag.log)"
}
run q8_before GPU_MAX_HW_QUEUES=8 && EXTRA_ARGS=--extra-after run q8_after GPU_MAX_HW_QUEUES=8 && \
run q16_before GPU_MAX_HW_QUEUES=16 && run q32_before GPU_MAX_HW_QUEUES=32 && \
EXTRA_ARGS=--extra-after run q16_after GPU_MAX_HW_QUEUES=16
