import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")
    config.addinivalue_line("markers", "slow: longer CPU-side oracle runs")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def ref_tables(tmp_path_factory):
    """phi-phi tables on the reference's exact axes and record counts ({5000, 100}, {1000, 1000, 100}; 1.6 GB
    of records, synthetic values), written once per session (nusiprop_amd.phiphi_tables)."""
    from nusiprop_amd.phiphi_tables import write_synthetic_tables
    d = str(tmp_path_factory.mktemp("pp_ref"))
    return write_synthetic_tables(d)
