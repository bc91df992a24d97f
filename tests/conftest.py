import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

# Known-answer trace of the 128^2 Re=100 cavity (dt = 1/1024, 200 steps), printed by the
# reference's monitor (FluidSolver.cpp:559-560); recorded in SURVEY.md section 6 / 8(c).
KNOWN_TRACE_128 = {
    1: (-0.037102, 0.254838, -0.102481, 0.102481),
    10: (-0.113792, 0.758282, -0.293865, 0.270659),
    50: (-0.140046, 0.891198, -0.367546, 0.316163),
    100: (-0.149054, 0.920759, -0.395207, 0.317666),
    150: (-0.154963, 0.933707, -0.409960, 0.318302),
    200: (-0.160059, 0.941389, -0.419694, 0.318126),
}


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libnsgpu.so)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def printed_equal(a, b):
    """Equal as printed by printf("%lf"), allowing a last-digit flip."""
    return abs(round(a, 6) - round(b, 6)) <= 1.000001e-6


@pytest.fixture(scope="session")
def gpu():
    import torch  # noqa: F401  (device presence only; the product path is libnsgpu.so)
    import navierstokessolver_amd as nsa
    nsa._lib.lib()
    return nsa
