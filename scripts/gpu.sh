#!/bin/bash
# One parametrised driver for every GPU measurement of this repo (replaces the round-1/2 one-off
# lease scripts). Run on the box as one gpurun command, e.g.
#   gpurun --timeout 1200 -- 'bash scripts/gpu.sh suite'
#   gpurun --timeout 900  -- 'bash scripts/gpu.sh tests tests/test_conv_bn_gpu.py -k grid'
#   gpurun --timeout 600  -- 'bash scripts/gpu.sh trace r3 --steps 10'
# Every GPU step runs under its own timeout and the steps chain with && (a crash, abort or time
# limit ends the command; nothing is retried). Results land in gpurun_out/.
#
#   suite                      every GPU test, smoke(), default bench   (the driver's round-end set)
#   tests FILES... [pytest -k]  selected GPU tests, one pytest process
#   bench [bench.py args]      one bench.py run (default: 20 timed / 5 warmup steps)
#   trace TAG [bench args]     rocprofv3 kernel + marker trace -> per-kernel table and a one-step
#                              per-queue timeline (scripts/prof_summary.py, scripts/step_timeline.py)
#   pmc TAG "COUNTERS" [args]  one rocprofv3 counter pass over a short bench (kernel trace only,
#                              never combined with other trace domains) -> scripts/pmc_summary.py
#   extras                     part1 batch (B=256), stock PyTorch-ROCm baseline, ResNet-50, Llama-3-8B
#   projection                 N>1 projection with the RCCL CTA budget priced (a model)
#   ramp [STEPS]               start-up ramp per kernel: kernel trace + one GRBM/SQ counter pass
#   ahead TAG [args]           kernel-trace timeline of steps enqueued behind a device sleep, so the
#                              profiler's per-dispatch host cost does not open gaps (step_trace_ahead.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
what=${1:-suite}
shift || true

page_in() { timeout -k 10 300 python3 -c "import torch, cs744_pytorch_distributed_tutorial_amd" || exit $?; }

case "$what" in
  suite)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 \
      --timeout-method thread > gpurun_out/pytest_gpu_full.log 2>&1
    rc=$?; echo "pytest exit $rc"; tail -5 gpurun_out/pytest_gpu_full.log
    [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    rc=$?; echo "smoke exit $rc"; tail -3 gpurun_out/smoke.log
    [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1
    rc=$?; tail -1 gpurun_out/bench_default.log; exit $rc
    ;;
  tests)
    timeout -k 10 1000 python -u -m pytest -x -v --timeout 180 --timeout-method thread "$@" \
      > gpurun_out/tests_sel.log 2>&1
    rc=$?
    grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/tests_sel.log | tail -60
    echo "pytest rc=$rc"; exit $rc
    ;;
  bench)
    [ $# -eq 0 ] && set -- --steps 20 --warmup 5
    timeout -k 10 400 python -u bench.py "$@" > gpurun_out/bench.log 2>&1
    rc=$?; grep -v amdgpu.ids gpurun_out/bench.log | tail -3; exit $rc
    ;;
  trace)
    TAG=${1:-trace}; shift || true
    [ $# -eq 0 ] && set -- --steps 10 --warmup 5
    page_in
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d $R/gpurun_out/$TAG -o run -- \
      python3 $R/bench.py "$@" > $R/gpurun_out/$TAG.log 2>&1)
    rc=$?; echo "rocprofv3 rc=$rc"; tail -1 gpurun_out/$TAG.log
    [ $rc -eq 0 ] || exit $rc
    python3 scripts/prof_summary.py gpurun_out/$TAG --steps ${PS_STEPS:-15} --top 45 > gpurun_out/${TAG}_kernels.txt 2>&1
    python3 scripts/step_timeline.py gpurun_out/$TAG > gpurun_out/${TAG}_timeline.txt 2>&1
    head -3 gpurun_out/${TAG}_kernels.txt
    grep -E "^# one step|^## queue|^# queue|^# main" gpurun_out/${TAG}_timeline.txt || true
    ;;
  pmc)
    TAG=${1:-pmc}; P=$2; shift 2 || true
    [ $# -eq 0 ] && set -- --steps 3 --warmup 2
    page_in
    (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/$TAG -o run -- \
      python3 $R/bench.py "$@" > $R/gpurun_out/$TAG.log 2>&1)
    rc=$?; echo "pmc pass exit $rc"; tail -2 gpurun_out/$TAG.log
    [ $rc -eq 0 ] || exit $rc
    python3 scripts/pmc_summary.py gpurun_out/$TAG > gpurun_out/${TAG}_summary.txt 2>&1
    head -40 gpurun_out/${TAG}_summary.txt
    ;;
  ramp)
    # start-up ramp, kernel by kernel: one long run under a kernel trace (scripts/ramp_table.py),
    # then one counter pass (GRBM_GUI_ACTIVE, SQ_BUSY_CYCLES; kernel trace only) over the same run
    # (scripts/ramp_pmc.py)
    N=${1:-230}
    page_in
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/ramp -o run -- \
      python3 $R/scripts/ramp_run.py --steps $N > $R/gpurun_out/ramp.log 2>&1)
    rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 scripts/ramp_table.py gpurun_out/ramp > gpurun_out/ramp_table.txt 2>&1; head -30 gpurun_out/ramp_table.txt
    (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace --output-format csv \
      -d $R/gpurun_out/ramp_pmc -o run -- python3 $R/scripts/ramp_run.py --steps $N > $R/gpurun_out/ramp_pmc.log 2>&1)
    rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 scripts/ramp_pmc.py gpurun_out/ramp_pmc --steps $N > gpurun_out/ramp_pmc.txt 2>&1; head -30 gpurun_out/ramp_pmc.txt
    ;;
  ahead)
    TAG=${1:-ahead}; shift || true
    page_in
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/$TAG -o run -- \
      python3 $R/scripts/step_trace_ahead.py "$@" > $R/gpurun_out/$TAG.log 2>&1)
    rc=$?; echo "rocprofv3 rc=$rc"; grep '^{' gpurun_out/$TAG.log || true
    [ $rc -eq 0 ] || exit $rc
    python3 scripts/step_timeline.py gpurun_out/$TAG --last 10 > gpurun_out/${TAG}_timeline.txt 2>&1
    head -14 gpurun_out/${TAG}_timeline.txt
    grep -E "^## queue|^# queue|^# main" gpurun_out/${TAG}_timeline.txt || true
    ;;
  extras)
    # end-of-round side measurements (each its own bench.py process, JSON lines appended to
    # gpurun_out/extras.jsonl): the tutorial's part1 batch (B=256, master/part1/part1.py:17), the
    # stock PyTorch-ROCm (MIOpen) VGG-11 baseline on this chip, the BASELINE.json extension configs
    : > gpurun_out/extras.jsonl
    for args in "--batch-size 256 --steps 20 --warmup 5" "--engine torch --steps 20 --warmup 5" \
                "--model resnet50 --dtype bf16 --steps 10 --warmup 4" "--model llama3-8b --steps 6 --warmup 3"; do
      timeout -k 10 500 python -u bench.py $args 2>>gpurun_out/extras.err | tail -1 >> gpurun_out/extras.jsonl || exit $?
      tail -1 gpurun_out/extras.jsonl | cut -c1-200
    done
    ;;
  projection)
    # N > 1 projection with the RCCL CTA budget priced (scripts/dp_projection.py --cta-gbps; a model)
    timeout -k 10 600 python -u scripts/dp_projection.py --steps 40 --warmup 10 --gbps ${PJ_GBPS:-150,300} \
      --worlds ${PJ_WORLDS:-8} --ctas ${PJ_CTAS:-8,16,32} --cta-gbps ${PJ_CTA_GBPS:-10} > gpurun_out/projection.jsonl \
      2> gpurun_out/projection.err || exit $?
    cut -c1-220 gpurun_out/projection.jsonl
    ;;
  *)
    echo "usage: bash scripts/gpu.sh suite|tests|bench|trace|ahead|pmc|ramp|extras|projection ..."; exit 2
    ;;
esac
