import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    # Native pieces are built in-tree; build them on demand (no-op when up to date).
    from flodbadd_amd.build import build_oracle, build_synth
    build_synth()
    build_oracle()


@pytest.fixture(scope="session")
def gpu_capture():
    """One context for the GPU session (few processes on the card, see gpurun rules)."""
    from flodbadd_amd.capture import FlodbaddGpuCapture
    from flodbadd_amd.sessions import SessionFilter
    cap = FlodbaddGpuCapture(0, session_filter=SessionFilter.All, flow_capacity=1 << 22)
    yield cap
    cap.close()
