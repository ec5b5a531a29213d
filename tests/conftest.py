import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def _gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


GPU = _gpu_available()


def pytest_collection_modifyitems(config, items):
    if GPU:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def oracle():
    import oracle_lib
    return oracle_lib.load()


@pytest.fixture(scope="session")
def built_lib():
    """The product library, built in-tree if this checkout has not built it yet."""
    from huffman_amd import build
    build.build()
    import huffman_amd
    return huffman_amd.load()


@pytest.fixture(scope="module", autouse=True)
def _default_torch_stream():
    """StreamCodec makes its own (non-blocking) stream torch's current stream for the process;
    restore the default stream after every module, so a later module's Device(0) (the null
    stream) and its torch tensors are ordered again."""
    yield
    if "torch" in sys.modules:
        import torch
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()
            torch.cuda.set_stream(torch.cuda.default_stream())
