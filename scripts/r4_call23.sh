#!/bin/bash
# Round-4 measurement 23 (end of round): the extension configs' bench lines on the final tree —
# ResNet-50 bf16 B=256 and Llama-3-8B bf16 8 x 2048 tokens — plus the VGG-11 default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/bench_ext_end.jsonl
timeout -k 10 400 python -u bench.py --model resnet50 --dtype bf16 --steps 10 --warmup 4 2>gpurun_out/ext_err.log \
  | tail -1 >> gpurun_out/bench_ext_end.jsonl || exit $?
tail -1 gpurun_out/bench_ext_end.jsonl | cut -c1-200
timeout -k 10 500 python -u bench.py --model llama3-8b --steps 6 --warmup 3 2>>gpurun_out/ext_err.log \
  | tail -1 >> gpurun_out/bench_ext_end.jsonl || exit $?
tail -1 gpurun_out/bench_ext_end.jsonl | cut -c1-200
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 2>>gpurun_out/ext_err.log \
  | tail -1 >> gpurun_out/bench_ext_end.jsonl || exit $?
tail -1 gpurun_out/bench_ext_end.jsonl | cut -c1-200
