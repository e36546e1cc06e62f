"""The measured-peak probe behind bench.py's roofline (tfidf_hbm_probe): plausible
streaming read / copy rates for an MI355X (HBM3E, 8 TB/s spec peak)."""
import pytest

pytestmark = pytest.mark.gpu


def test_hbm_probe_plausible(engine):
    r = engine.hbm_probe(1 << 30, 3)
    assert 1000.0 < r["read_GBps"] < 8200.0, r
    assert 1000.0 < r["copy_GBps"] < 8200.0, r
