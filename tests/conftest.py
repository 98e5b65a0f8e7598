import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "hgnn-2_amd")
for p in (REPO, PKG, os.path.join(REPO, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

os.environ.setdefault("HGNN_STRICT", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    mark = (config.getoption("markexpr", "") or "").replace(" ", "")
    if "gpu" in mark and "notgpu" not in mark:
        # Multi-process GPU tests fork their ranks from a forkserver started here, before this
        # process initialises the GPU (collection below asks torch whether a GPU is present):
        # the ranks are then never exec'd from a process that holds GPU state.
        import multiprocessing as mp
        ctx = mp.get_context("forkserver")
        ctx.set_forkserver_preload([])
        from multiprocessing import forkserver
        forkserver.ensure_running()


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(REPO, "tests", "golden", name + ".npz"))
    return load
