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


@pytest.mark.parametrize("keccak_reads", [False, True])
@pytest.mark.parametrize("seed", [3, 9])
def test_lowered_rows_are_models_on_random_paths(seed, keccak_reads):
    """Every guided row the lowered query accepts is a model of the original query (ORACLE),
    on planted random paths (arrays read at keys that lower to constants no harvest saw, e.g.
    select(K(7), i) as an index; keccak at symbolic and constant arguments), in both lowering
    modes.  Seed 9 prefix 5 had a row that was not (a constant key outside the harvested cells
    read the else column while a read at an equal index took another value; r06c GPU recall
    run: 7 invalid witnesses)."""
    from mythril_amd.candidates import build_guide
    from mythril_amd.lower import lower_query
    from oracle import smt_eval as E
    from oracle.guided_gen import generate_row
    from tests.test_reference_fixtures import holds_original

    ctx, cs, _, _ = planted_path("random", seed, 16)
    nodes = [c.node for c in cs]
    b = ctx.b
    accepted = 0
    for k in range(1, len(nodes) + 1):
        root, schema = lower_query(b, nodes[:k], keccak_reads=keccak_reads)
        cols = list(schema.columns)
        if not cols:
            continue
        guide = build_guide(b, root, schema, cols).arrays()
        names = [n for n, _ in sorted(b.var_index.items(), key=lambda kv: kv[1])]
        tape = b.finish(root)
        for r in range(48):
            row = dict(zip(cols, generate_row(0x5EED, r, guide)))
            if E.evaluate(tape.nodes, b.pool.values, [row.get(n, 0) for n in names]):
                accepted += 1
                assert holds_original(ctx, cs[:k], schema, row), (seed, k, r)
    assert accepted > 0
