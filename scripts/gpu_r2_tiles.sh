# round 2: tile tables for the shipped gfx950 JSON, then the B=64/ragged fp64 parity tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/tiles_gfx950.json
CS744_TUNE=1 CS744_TUNE_CACHE=gpurun_out/tiles_gfx950.json timeout -k 10 600 python -u scripts/make_tile_table.py \
  > gpurun_out/make_tiles.log 2>&1; rc=$?; cat gpurun_out/make_tiles.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
cp gpurun_out/tiles_gfx950.json cs744_pytorch_distributed_tutorial_amd/runtime/tiles_gfx950.json
timeout -k 10 600 python -u -m pytest -x -v -p no:cacheprovider --timeout 240 --timeout-method thread \
  tests/test_native_engine_gpu.py > gpurun_out/pytest_r2parity.log 2>&1
rc=$?; echo "pytest exit $rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_r2parity.log | tail -40; exit $rc
