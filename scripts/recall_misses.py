#!/usr/bin/env python3
"""Where the planted random family's misses come from (diagnostics for the recall
work of VERDICT r5 next 3).

Paths of tests/planted.py asked in LASER order on one Sieve (as scripts/planted_recall.py).  Per
path the outcome of every prefix; per *first* miss (a miss whose parent was answered) the
newest constraint's kind and whether the planted model M's row satisfies the lowered query --
if it does, the miss is the candidate search's (a row exists in the sieve's model space; the
guided rounds did not draw it), else the lowering's (no row denotes M).  One JSON line.

    python scripts/recall_misses.py [n_paths=100] [path_len=24] [--fake]
"""
import json
import os
import sys
from collections import Counter

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

from mythril_amd.lower import READ_KINDS, lower_query  # noqa: E402
from mythril_amd.sieve import Sieve  # noqa: E402
from oracle import smt_eval as E  # noqa: E402
from oracle.term_eval import evaluate_term  # noqa: E402
from tests.planted import planted_path  # noqa: E402


def m_row_accepted(ctx, nodes, m, keccak_reads=False):
    """The planted model's row of the lowered query, and whether the lowered root holds there."""
    b = ctx.b
    names = [n for n, _ in sorted(b.var_index.items(), key=lambda kv: kv[1])]

    def mval(node):
        return evaluate_term(b.finish(node).nodes, b.pool.values, names, b.symbols.array_names,
                             b.symbols.function_names, m.vars, m.arrays, m.funcs)

    root, schema = lower_query(b, nodes, keccak_reads=keccak_reads)
    row = {}
    for c in schema.columns.values():
        if c.kind == "var":
            row[c.name] = m.vars.get(c.name, 0)
        elif c.kind in ("cell", "else", "read"):
            tab, els = m.arrays.get(c.symbol, ({}, 0))
            key = c.key if c.kind == "cell" else mval(c.key) if c.kind == "read" else None
            row[c.name] = els if key is None else tab.get(key, els)
        elif c.kind in ("ufcell", "ufread", "kread"):
            f = m.funcs.get(c.symbol)
            key = c.key if c.kind == "ufcell" else mval(c.key)
            row[c.name] = f(key) if f else 0
        else:
            row[c.name] = 0
    names = [n for n, _ in sorted(b.var_index.items(), key=lambda kv: kv[1])]  # with the columns
    return bool(E.evaluate(b.finish(root).nodes, b.pool.values, [row.get(n, 0) for n in names]))


def main():
    args = [int(a) for a in sys.argv[1:] if not a.startswith("--")]
    n_paths = args[0] if args else 100
    path_len = args[1] if len(args) > 1 else 24
    if "--fake" in sys.argv:
        import pytest

        from tests import fake_device

        fake_device.install(pytest.MonkeyPatch())
        s = Sieve(rows=256, budget_s=60.0)
    else:
        s = Sieve()
    seqs, first = [], Counter()
    space = Counter()
    first_pos = []
    for seed in range(n_paths):
        ctx, cs, m, kinds = planted_path("random", seed, path_len)
        nodes = [c.node for c in cs]
        seq, prev = "", True
        for k in range(1, len(nodes) + 1):
            try:
                w = s.solve(ctx.b, nodes[:k], key=tuple(nodes[:k]))
            except Exception:  # noqa: BLE001
                w = None
            hit = w is not None
            seq += "h" if hit else "m"
            if not hit and prev:
                first[kinds[k - 1]] += 1
                first_pos.append(k)
                try:
                    acc = m_row_accepted(ctx, nodes[:k], m)
                    acc2 = m_row_accepted(ctx, nodes[:k], m, keccak_reads=True)
                except Exception:  # noqa: BLE001
                    acc = acc2 = None
                space[("search" if acc else "lowering" if acc is False else "error",
                       "search" if acc2 else "lowering" if acc2 is False else "error")] += 1
            prev = hit
        seqs.append(seq)
    s.close()
    n = sum(len(x) for x in seqs)
    misses = sum(x.count("m") for x in seqs)
    after_miss = sum(1 for x in seqs for i in range(1, len(x)) if x[i] == "m" and x[i - 1] == "m")
    recovered = sum(1 for x in seqs for i in range(1, len(x)) if x[i] == "h" and x[i - 1] == "m")
    print(json.dumps({
        "paths": n_paths, "queries": n, "misses": misses,
        "first_misses": sum(first.values()), "misses_after_a_miss": after_miss,
        "hits_after_a_miss": recovered,
        "first_miss_by_newest_constraint": dict(first.most_common()),
        "first_miss_cause (default, keccak_reads)": {"%s/%s" % k: v for k, v in space.items()},
        "first_miss_prefix_len_mean": round(sum(first_pos) / max(len(first_pos), 1), 2),
        "sequences": seqs[:20],
    }), flush=True)


if __name__ == "__main__":
    main()
