import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs via gpurun on the GPU box)")
    config.addinivalue_line("markers", "multigpu: needs >=2 GPUs")
    config.addinivalue_line("markers", "slow: long-running test")


def _gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords or "multigpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def native_lib():
    """The HIP kernel library MUST load on a GPU box (no silent fallback)."""
    from llmctl.ops import _lib
    assert os.environ.get("LLMCTL_FORCE_REF") != "1", "LLMCTL_FORCE_REF must not be set for kernel tests"
    assert _lib.load(), f"HIP library failed to load: {_lib._error}"
    import torch
    return torch.ops.llmctl


@pytest.fixture(autouse=True)
def _reset_perf_knobs():
    """Engines configure the process-wide performance knobs (llmctl.config.knobs); every test
    starts and ends with the defaults (+ LLMCTL_KNOBS of the environment, if any)."""
    from llmctl.config import knobs

    knobs.configure()
    yield
    knobs.configure()
