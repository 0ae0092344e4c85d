import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'deepwalk-and-node2vec_amd')
GOLDEN = os.path.join(REPO, 'tests', 'golden')
for p in (PKG, REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP device) and libdw_hip.so')
    config.addinivalue_line('markers', 'slow: long-running parity case')


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope='session')
def hip_device():
    import torch
    from shallow_encoders import _native
    if not torch.cuda.is_available():
        pytest.fail('GPU test selected but no HIP device is visible')
    _native.load()
    return torch.device('cuda', 0)
