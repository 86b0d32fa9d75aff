# BN variants at the VGG shapes, per grid-barrier version (-1 = barriers skipped, timing only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
: > gpurun_out/bn_grid.log
for v in 0 1 2 -1; do
  CS_BN_GRID_BARV=$v timeout -k 10 200 python -u scripts/bn_grid_bench.py 64 20 >> gpurun_out/bn_grid.log 2>&1 || { rc=$?; grep -v amdgpu.ids gpurun_out/bn_grid.log; exit $rc; }
done
grep -v amdgpu.ids gpurun_out/bn_grid.log
