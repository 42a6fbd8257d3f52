"""Test configuration: `gpu` marker, import paths, shared helpers.

CPU tests (`-m "not gpu"`) cover the oracle against its independent Python restatement and
hand-derived known answers, the consumer (parse_umi_clusters) against golden fixtures produced by
the reference itself, argv/parameter handling and that the C-ABI library exports every symbol
include/umiclust.h declares.  GPU tests (`-m gpu`) are the parity tests proper and call through
the C ABI; they never read /root/reference.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ont-tcrconsensus_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))  # fixture writers (data only)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def gpu_ctx():
    from umiclust import _lib
    ctx = _lib.Context(0)
    yield ctx
    ctx.close()
