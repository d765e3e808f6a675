import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / 'x-transformers-rl_amd'))
os.environ.setdefault('TQDM_DISABLE', '1')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through the HIP C-ABI library)')


@pytest.fixture(scope='session')
def golden():
    import numpy as np

    def load(name):
        return np.load(REPO / 'tests' / 'golden' / f'{name}.npz', allow_pickle=False)
    return load
