"""MI355X-native data-parallel training framework with the capabilities of the
CS744 PyTorch Distributed Tutorial (kkyyhh96/CS744_PyTorch_Distributed_Tutorial).

Subpackages:
  models/    VGG11/13/16/19 (reference layout), ResNet-50, Llama-style decoder
  ops/       hand-written HIP/CDNA4 kernels (gfx950) + autograd wrappers
  parallel/  gradient-sync strategies, DDP (bucketed, overlapped), RCCL communicator
  runtime/   fused, graph-captured native training engine
  utils/     data (synthetic CIFAR, sampler, device loader), metrics, checkpoint, faults
  entrypoints/ part1, part1_pingpong, part2a, part2a_extra, part2b, part3
"""
__version__ = "0.1.0"

from . import distributed  # noqa: F401
