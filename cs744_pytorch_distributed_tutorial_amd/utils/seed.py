"""Deterministic seeding (reference `master/part2b/part2b.py:82-83`,
`master/part1/part1.py:107`: ``torch.manual_seed(5000)`` + ``np.random.seed(5000)``).

In part2a/2b this is the *only* mechanism that gives identical initial weights on
every rank (there is no broadcast), so the same seed must be applied before the
model is built on every rank.
"""
from __future__ import annotations

import random

import numpy as np
import torch

REFERENCE_SEED = 5000


def seed_everything(seed: int = REFERENCE_SEED) -> None:
    torch.manual_seed(seed)
    np.random.seed(seed)
    random.seed(seed)
