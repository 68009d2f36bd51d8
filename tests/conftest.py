import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: multi-second CPU oracle runs")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))

    return load


@pytest.fixture(scope="session")
def sd_np():
    from voiceactivityprojection_amd.weights import synthetic_state_dict

    return synthetic_state_dict(seed=0)


@pytest.fixture
def drop_ready(monkeypatch):
    """Robustness tests: every native handle a VapGPT creates from now on never publishes the recurrence's
    ready flag of time chunk 1 (test ABI vap_test_drop_ready), so the bounded hand-off wait times out."""
    from voiceactivityprojection_amd import _native as N
    from voiceactivityprojection_amd.model import VapGPT

    orig = VapGPT._native

    def patched(self, device):
        h = orig(self, device)
        N.check(N.lib().vap_test_drop_ready(h, 1), "vap_test_drop_ready")
        return h

    monkeypatch.setattr(VapGPT, "_native", patched)
