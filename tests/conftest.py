import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_sessionfinish(session, exitstatus):
    """Write every error the parity tests measured (tests/parity.py) to $PARITY_LOG."""
    path = os.environ.get("PARITY_LOG")
    if not path:
        return
    parity = sys.modules.get("parity")  # tests import it as `from parity import check`
    if parity is None:
        return
    import json
    recs = parity.RECORDS
    if recs:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(recs, f, indent=1)


@pytest.fixture
def switch():
    """set_switch(name, value) for one test (gonova_tts_amd.engine.set_switch: the process-wide
    kernel-path switches of include/tts_hip.h); every switch it touched goes back to the value
    it had before the test (an environment setting included)."""
    from gonova_tts_amd.engine import get_switch, set_switch
    saved = {}

    def setter(name, value):
        if name not in saved:
            saved[name] = get_switch(name)
        set_switch(name, -1 if value is None else int(value))

    yield setter
    for name, v in saved.items():
        set_switch(name, v)
