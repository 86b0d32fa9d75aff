import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")
    # the test session is an entry point like bench.py: HIP's hardware queues are raised before
    # any test initialises HIP (the engine's side stream + a communicator need >= 8 queues)
    import cs744_pytorch_distributed_tutorial_amd as pkg
    pkg.ensure_hw_queues()


class HostedStore:
    """A rendezvous store the TEST process owns for the whole life of a spawned world.

    The server binds port 0 and keeps the socket, so no other socket can take the port between
    "pick a port" and "rank 0 listens on it" (the round-5 EADDRINUSE race of bind(0)-then-close).
    Ranks connect as clients: ``TORCHELASTIC_USE_AGENT_STORE=True`` makes torch's env://
    rendezvous create a client on every rank, rank 0 included — exactly what torchrun's agent
    does with its own store. One store per world: process-group keys restart in every process.
    """

    def __init__(self, world: int):
        from torch.distributed import TCPStore
        self.store = TCPStore("127.0.0.1", 0, world, is_master=True, wait_for_workers=False)
        self.port = self.store.port

    def env(self, base=None) -> dict:
        e = dict(os.environ if base is None else base)
        e.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(self.port), TORCHELASTIC_USE_AGENT_STORE="True")
        return e


def torchrun_cmd(nproc: int) -> list:
    """torchrun with a standalone rendezvous: the launcher's agent binds port 0 and hands its store
    to the workers, so there is no port to race for."""
    return [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1",
            "--nnodes=1", f"--nproc-per-node={nproc}"]


@pytest.fixture
def hosted_store(monkeypatch):
    """A one-rank HostedStore whose port/env the test's child processes inherit."""
    hs = HostedStore(1)
    for k, v in hs.env({}).items():
        monkeypatch.setenv(k, v)
    yield hs
    del hs.store
