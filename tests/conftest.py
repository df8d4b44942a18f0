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
    """GPU tests check the HIP path against the oracle in the library's own pixel-node Jacobian arithmetic: the product
    build forms them as the reference CPU path's unfused products (the oracle's default, NNRT_JAC_FMA=0), so every GPU
    test runs against the reference arithmetic; a development build with FMA-formed Jacobians switches the oracle to its
    bit-identical fused mode, and tests/test_gpu_parity.py::test_reference_arithmetic_margins then holds that build
    against the reference arithmetic at north_star's tolerance."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    O = request.getfixturevalue("oracle_mod")
    from dynamicfuion_python_amd import _native
    O.set_fused_jacobians(_native.jacobian_fma())
    yield
    O.set_fused_jacobians(False)
