import os
import socket
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


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.fixture
def port():
    return free_port()
