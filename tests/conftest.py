import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "jwave-pro_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test requires a HIP device")
    return torch.device("cuda:0")


class _Knobs:
    """Engine settings (JW_*) through jw_set_knob, restored after the test: monkeypatch's
    setenv/delenv shape, without setenv racing the engine's threads."""

    def __init__(self):
        from jwave import _native
        self._n = _native
        self._saved = {}

    def setenv(self, name, value):
        if name not in self._saved:
            self._saved[name] = self._n.get_knob(name)
        self._n.set_knob(name, value)

    def delenv(self, name):
        self.setenv(name, None)

    def restore(self):
        for k, v in self._saved.items():
            self._n.set_knob(k, v)


@pytest.fixture
def knobs():
    k = _Knobs()
    yield k
    k.restore()
