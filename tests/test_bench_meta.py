"""
bench.py's host-side bookkeeping (CPU): the committed PMC summary it reads the roofline `traffic`
from exists and covers the configs whose dominant kernel was profiled.
"""
import importlib.util
import os

from tests.conftest import ROOT


def load_bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    module = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(module)
    return module


def test_measured_traffic_reads_the_pmc_summary():
    bench = load_bench()
    for cfg in ("c2", "c3", "c5"):
        traffic, source = bench.measured_traffic(cfg)
        assert traffic is not None and traffic > 0, cfg
        assert source.startswith("profiles/r") and source.endswith("_pmc.json")
    assert bench.measured_traffic("c1") == (None, None)
