"""part2b: per-parameter all_reduce(SUM) of grad/N (reference `master/part2b/part2b.py:43-45`).

One script serves every rank (the reference ships separate master/ and slave/
copies; rank-dependent logic lives in `parallel.sync`). Usage::

    python -m cs744_pytorch_distributed_tutorial_amd.entrypoints.part2b --master-ip 127.0.0.1 --num-nodes 4 --rank R

or under torchrun (RANK/WORLD_SIZE/LOCAL_RANK from the environment). Extra flags:
`--sync`, `--engine {torch,native}`, `--comm {torch,rccl}`, `--bucket-mb`, `--steps`, ...
"""
from __future__ import annotations

import sys

from ..config import config_from_args
from ..train import run


def main(argv=None) -> int:
    cfg = config_from_args("part2b", argv)
    run(cfg)
    return 0


if __name__ == "__main__":
    sys.exit(main())
