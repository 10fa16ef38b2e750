import contextlib
import glob
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, os.path.join(REPO, "oracle"), os.path.join(REPO, "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_collection_modifyitems(config, items):
    # a test that takes the ``cuda`` fixture needs the GPU whether or not it
    # carries the marker: mark it, so ``-m gpu`` selects it (and ``-m "not gpu"``
    # does not collect a test that could only skip)
    for item in items:
        if "cuda" in getattr(item, "fixturenames", ()) and item.get_closest_marker("gpu") is None:
            item.add_marker(pytest.mark.gpu)


@contextlib.contextmanager
def knobs(*pairs):
    """Run the block with A/B knobs (key, value) set: on the product library
    when every value is 0 (the product's own choices), else on the diagnostic
    library (gsvc_amd._lib.diagnostic(), the only one with knobs).  Yields the
    library the block's ops use."""
    from gsvc_amd import _lib
    if all(v == 0 for _, v in pairs):
        yield _lib.load()
        return
    with _lib.diagnostic() as lib:
        olds = [(k, lib.gsvc_debug_set(k, v)) for k, v in pairs]
        # an unknown key returns -1 and sets nothing: an A/B that would test nothing
        assert all(o >= 0 for _, o in olds), f"knob key out of range: {pairs}"
        try:
            yield lib
        finally:
            for k, v in reversed(olds):
                lib.gsvc_debug_set(k, v)


def load_golden(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return {k: z[k] for k in z.files}


def golden_names(prefix):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from gsvc_amd import _lib
    _lib.load()
    return torch.device("cuda:0")
