"""The bench line's PMC traffic and in-network clock come from committed profiles keyed by the conv
source hash (bench.py pmc_traffic / conv_clock): present for the dominant classes at the tree's
conv source, null (stale) as soon as the kernel source differs.  CPU only: reads profiles/*.json."""
import importlib.util
import os

import pytest

from conftest import REPO

HEAD = "conv3x3 256->256 @32x512 d1"


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(REPO, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_profiles_match_the_tree(bench):
    traffic, src = bench.pmc_traffic("fp32x3", 4, HEAD)
    assert traffic is not None and traffic > 136_577_024, src   # above the algorithmic bytes
    assert "conv source" in src
    for cls in (HEAD, "conv3x3 128->128 @64x1024 d1"):
        clk = bench.conv_clock(cls)
        assert clk is not None, cls
        assert 1.0 < clk["clock_GHz"] < 2.5 and 0.0 < clk["mfma_busy_frac"] <= 1.0


def test_stale_source_gives_null(bench, monkeypatch):
    from sdp import _build
    monkeypatch.setattr(_build, "conv_source_hash", lambda: "0" * 64)
    traffic, src = bench.pmc_traffic("fp32x3", 4, HEAD)
    assert traffic is None and src.startswith("stale")
    assert bench.conv_clock(HEAD) is None
