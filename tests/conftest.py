import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run on the GPU box")


def pytest_sessionfinish(session, exitstatus):
    """Write the parity margins the GPU tests recorded (tests/margins.py)."""
    try:
        import margins
    except ImportError:
        return
    rec = margins.records()
    if not rec:
        return
    import json

    out = os.environ.get("WBC_MARGINS_OUT", os.path.join(ROOT, "gpurun_out", "parity_margins.json"))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(rec, f, indent=1, sort_keys=True)
