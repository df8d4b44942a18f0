import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device; parity tests of the HIP path against the oracle")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(autouse=True)
def _checker_jacobian_arithmetic(request):
    """GPU tests check the HIP path against the oracle in the library's own pixel-node Jacobian arithmetic (the FMA form
    of csrc/fitter_kernels.hip, NNRT_JAC_FMA: bit-identical terms, so H / g stay held to 1e-6); the reference CPU path's
    unfused arithmetic is the oracle's default and is checked against the GPU at north_star's tolerance in
    tests/test_gpu_parity.py::test_fused_jacobians_vs_reference_arithmetic."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    O = request.getfixturevalue("oracle_mod")
    from dynamicfuion_python_amd import _native
    O.set_fused_jacobians(_native.jacobian_fma())
    yield
    O.set_fused_jacobians(False)
