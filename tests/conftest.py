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


_BINSETS = {}


@pytest.fixture(scope="session")
def config_binset():
    """Synthetic BASELINE multi-bin inputs (umiclust.synth.config_bins, deterministic per bin), built once per session
    and shared by the tests that cluster them (config 3 at full size is ~9.9M reads)."""
    def get(cfg: int, scale: float, shard_ids=None):
        from umiclust import synth
        key = (cfg, scale, tuple(shard_ids) if shard_ids is not None else None)
        if key not in _BINSETS:
            _BINSETS[key] = synth.concat_bins(synth.config_bins(cfg, scale, workers=min(16, os.cpu_count() or 4),
                                                                shard_ids=shard_ids))
        return _BINSETS[key]
    return get
