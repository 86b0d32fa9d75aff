# the tutorial's entrypoints on one MI355X with the native engine: part1 (B=256, one full epoch +
# full test-set eval, reference print formats) and part3 (DDP loop, world 1), checkpoint + resume
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m cs744_pytorch_distributed_tutorial_amd.entrypoints.part1 --engine native --device cuda --checkpoint gpurun_out/ck_part1.pt > gpurun_out/entry_part1.log 2>&1 || { tail -20 gpurun_out/entry_part1.log; exit 1; }
head -4 gpurun_out/entry_part1.log; tail -4 gpurun_out/entry_part1.log
timeout -k 10 300 python -m cs744_pytorch_distributed_tutorial_amd.entrypoints.part3 --engine native --device cuda --resume gpurun_out/ck_part1.pt --steps 100 > gpurun_out/entry_part3.log 2>&1 || { tail -20 gpurun_out/entry_part3.log; exit 1; }
head -3 gpurun_out/entry_part3.log; tail -3 gpurun_out/entry_part3.log
rm -f gpurun_out/ck_part1.pt
