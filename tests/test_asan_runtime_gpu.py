"""Host-side AddressSanitizer run of the native C++ runtime: the standalone
program csrc/tests/asan_runtime_test.cpp, built with -Xarch_host -fsanitize=address
(`python -m cs744_pytorch_distributed_tutorial_amd._build --asan`), drives the VGG engine,
the C++ DDP step through the ordering-probe communicator (stream links and HIP events), a
one-rank RCCL step, abort and teardown on an MI355X; an ASan report fails it."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "cs744_pytorch_distributed_tutorial_amd", "bin", "asan_runtime_test")


def test_runtime_under_host_asan():
    if not os.path.exists(EXE):
        pytest.skip("ASan runtime test not built (python -m cs744_pytorch_distributed_tutorial_amd._build --asan)")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:detect_container_overflow=0:abort_on_error=0")
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=200, env=env, cwd=ROOT)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0 and "done, 0 failure(s)" in r.stdout, out[-3000:]
