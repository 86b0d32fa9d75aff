"""gfx950 (MI355X) kernels: see csrc/kernels/*.hip; Python entry points in ``native``
and autograd/module wrappers in ``functional`` and ``optim``."""
from . import native  # noqa: F401
