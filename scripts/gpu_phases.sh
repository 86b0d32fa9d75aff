# per-phase device timing of the native step (no comm, and the one-rank RCCL probe)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_native_engine_gpu.py -k phase -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_phase.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_phase.log; [ $rc -eq 0 ] || exit $rc
export CS744_TUNE_CACHE=gpurun_out/tune_phases.json
timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --phases 20 > gpurun_out/phases_1gpu.log 2>&1 || exit $?
grep phases gpurun_out/phases_1gpu.log
CS_COMM_PROBE=1 timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --phases 20 > gpurun_out/phases_probe.log 2>&1 || exit $?
grep phases gpurun_out/phases_probe.log
