from .buckets import build_buckets  # noqa: F401
from .comm import Comm, TorchComm, make_comm  # noqa: F401
from .ddp import DistributedDataParallel  # noqa: F401
from .sync import SYNC_MODES, make_sync  # noqa: F401
