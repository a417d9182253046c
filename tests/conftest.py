import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP engine")


def gpu_available() -> bool:
    try:
        from leanfe_amd._lib import load_library
        import ctypes
        load_library()
        hip = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_int(0)
        return hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    except Exception:
        return False


class Knobs:
    """The engine's test / A-B knobs (lfe_test_set_knob), with monkeypatch's setenv / delenv shape.
    The engine reads no environment variables: a test that wants a non-default kernel path sets a
    knob, and every knob it set is removed at teardown."""

    def __init__(self):
        self.names = set()

    def setenv(self, name: str, value) -> None:
        from leanfe_amd._lib import set_knob
        set_knob(name, str(value))
        self.names.add(name)

    def delenv(self, name: str, raising: bool = False) -> None:
        from leanfe_amd._lib import set_knob
        set_knob(name, None)
        self.names.discard(name)


@pytest.fixture
def knob():
    k = Knobs()
    yield k
    if k.names:
        from leanfe_amd._lib import clear_knobs
        clear_knobs()
