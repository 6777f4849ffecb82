"""Planted-model query paths (tests/planted.py) are SAT by construction, and the recall harness
(scripts/planted_recall.py) counts them right.  Host only: the fake device stands in (small
rounds); the measured recall on the GPU is tests/test_gpu_recall.py and DESIGN §6."""
import pytest

from tests import fake_device
from tests.planted import FAMILIES, planted_path


@pytest.mark.parametrize("family", sorted(FAMILIES))
def test_every_prefix_has_the_planted_model(family):
    kinds = set()
    for seed in range(12):
        ctx, cs, m, ks = planted_path(family, seed, 16)
        assert len(cs) == len(ks) >= 12
        assert all(m.holds(ctx, c) for c in cs), (family, seed)
        kinds.update(ks)
        again = planted_path(family, seed, 16)
        assert len(again[1]) == len(cs) and again[3] == ks  # deterministic
    want = {"random": {"store", "keccak_pair", "keccak_bound", "wide_eq", "pinned", "eq", "ult"},
            "laser": {"dispatch", "size_guard", "arg_range", "overflow", "actors", "owner",
                      "value", "storage", "mapping", "suicide", "ether_thief"}}[family]
    assert want <= kinds, want - kinds


def test_recall_harness_on_fake_device(monkeypatch):
    """No planted query is refuted (M is a model of it) and every hit is oracle-valid."""
    from mythril_amd.sieve import Sieve
    from scripts.planted_recall import run_family

    fake_device.install(monkeypatch)
    s = Sieve(rows=256)
    for family in sorted(FAMILIES):
        out = run_family(s, family, 2, 8)
        assert out["refuted"] == 0 and out["invalid_witnesses"] == 0, out
        assert out["error"] == 0, out
        assert out["queries"] >= 16 and out["recall"] > 0, out
