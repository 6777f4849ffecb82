#!/usr/bin/env python3
"""Recall of the sieve on queries that are SAT by construction.

Paths of tests/planted.py (a model drawn first, every constraint oriented to hold under it and
checked by the oracle) are asked in LASER order on one Sieve -- every prefix a query, its parent
solved first (svm.py:257-262) -- so every query is satisfiable and every miss is a query the
sieve could have answered and z3 must.  Per query: the outcome (a hit in the first, 256-row round
or only in the second, 2^16-row round; a miss; a refutation -- a soundness failure, since M is a
model; an unsupported shape), the wall time, and for a hit that the witness is a model of the
original query (oracle/term_eval.py).  One JSON line per family with the recall overall, per
round, per shape class of the query's newest constraint, latency percentiles, the hits of the
keccak second chance (SIEVE_KECCAK2=0 turns it off); with --extended,
the misses are asked again of a sieve with 2^20-row second rounds (how many more rows would
recover).

    python scripts/planted_recall.py [n_paths=100] [path_len=24] [--extended] [--fake]
                                     [--round2=always|progress|never] [--feedback]

--feedback: after a miss, the planted model M is learnt as the missed query's witness
(Sieve.learn, what frontend.learn_from_fallback does with the fallback's model), as if z3 had
answered the miss with M -- an upper bound on what learning z3's models gives, since z3's model of
a prefix need not satisfy the path's later constraints as M does.

--fake runs on tests/fake_device.py (CPU; use small sizes).
"""
import json
import os
import sys
import time
from collections import Counter, defaultdict

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402

from mythril_amd.sieve import Sieve  # noqa: E402
from tests.planted import FAMILIES, planted_path  # noqa: E402
from tests.test_reference_fixtures import holds_original  # noqa: E402


def _pct(v):
    if not v:
        return {"n": 0}
    a = np.array(v)
    return {"n": len(v), "p50": round(float(np.percentile(a, 50)), 3),
            "p90": round(float(np.percentile(a, 90)), 3),
            "p99": round(float(np.percentile(a, 99)), 3), "max": round(float(a.max()), 3)}


def planted_value(m, ctx=None):
    """value_of(column) for Sieve.learn under the planted model M (a read column at its index
    term's value under M, given the term context)."""
    def at(node):
        b = ctx.b
        names = [n for n, _ in sorted(b.var_index.items(), key=lambda kv: kv[1])]
        from oracle.term_eval import evaluate_term

        return evaluate_term(b.finish(node).nodes, b.pool.values, names, b.symbols.array_names,
                             b.symbols.function_names, m.vars, m.arrays, m.funcs)

    def value_of(col):
        if col.kind == "var":
            return m.vars.get(col.symbol)
        if col.kind in ("cell", "else") and col.symbol in m.arrays:
            table, els = m.arrays[col.symbol]
            return els if col.kind == "else" else table.get(col.key, els)
        if col.kind == "ufcell" and col.symbol in m.funcs:
            return m.funcs[col.symbol](col.key)
        if ctx is not None and col.kind == "read" and col.symbol in m.arrays:
            table, els = m.arrays[col.symbol]
            return table.get(at(col.key), els)
        if ctx is not None and col.kind in ("ufread", "kread") and col.symbol in m.funcs:
            return m.funcs[col.symbol](at(col.key))
        return None
    return value_of


def run_family(s, family, n_paths, path_len, big=None, check=True, feedback=False):
    """Every prefix of n_paths planted paths in LASER order on sieve `s`.  Returns the summary
    and the list of missed (seed, prefix) pairs."""
    outcomes = Counter()
    by_kind = defaultdict(Counter)
    progress = Counter()  # first-round progress (some groups solved) of round-2 hits and misses
    times = defaultdict(list)
    bad, missed = [], []
    learnt0 = s.stats.extra.get("learnt", 0)
    k2t0 = s.stats.extra.get("keccak2_tries", 0)
    k2hits = 0
    for seed in range(n_paths):
        ctx, cs, m, kinds = planted_path(family, seed, path_len)
        nodes = [c.node for c in cs]
        for k in range(1, len(nodes) + 1):
            r0 = s.stats.extra.get("refuted", 0)
            t0 = time.perf_counter()
            try:
                w = s.solve(ctx.b, nodes[:k], key=tuple(nodes[:k]))
                dt = (time.perf_counter() - t0) * 1e3
                if w is not None:
                    kind = "hit_r%d" % w.rounds
                    k2hits += bool(getattr(w.schema, "keccak_reads", False))
                    if check and not holds_original(ctx, cs[:k], w.schema, w.values):
                        bad.append((seed, k))
                elif s.stats.extra.get("refuted", 0) > r0:
                    kind = "refuted"
                else:
                    kind = "miss"
                    missed.append((seed, k))
                    if feedback:
                        s.learn(tuple(nodes[:k]), planted_value(m, ctx))
            except Exception as e:  # noqa: BLE001 - the front end falls back on any error
                dt = (time.perf_counter() - t0) * 1e3
                kind = "unsupported" if "Unsupported" in type(e).__name__ else "error"
            outcomes[kind] += 1
            by_kind[kinds[k - 1]][kind] += 1
            lr = s.last_rounds
            if kind in ("hit_r2", "miss") and lr:
                part = 0 < lr.get("r1_solved", 0) < lr.get("groups", 0)
                progress[kind + ("_r1_partial" if part else "_r1_none")] += 1
            times[kind].append(dt)
    n = sum(outcomes.values())
    hits = outcomes["hit_r1"] + outcomes["hit_r2"]
    out = {
        "family": family, "paths": n_paths, "path_len": path_len, "queries": n,
        "recall": round(hits / max(n, 1), 4),
        "hit_round1": outcomes["hit_r1"], "hit_round2_only": outcomes["hit_r2"],
        "miss": outcomes["miss"], "refuted": outcomes["refuted"],
        "unsupported": outcomes["unsupported"], "error": outcomes["error"],
        "invalid_witnesses": len(bad),
        "second_round": s.second_round,
        # hits of the keccak second chance (keccak applications as read columns, Sieve.solve)
        "keccak_second_chance": s.keccak_second_chance, "keccak2_hits": k2hits,
        "keccak2_tries": s.stats.extra.get("keccak2_tries", 0) - k2t0,
        "feedback": feedback, "learnt": s.stats.extra.get("learnt", 0) - learnt0,
        "first_round_progress": dict(progress),
        "by_newest_constraint": {
            k: {"n": sum(c.values()), "recall": round((c["hit_r1"] + c["hit_r2"]) /
                                                      max(sum(c.values()), 1), 4),
                "round2_only": c["hit_r2"], "miss": c["miss"]}
            for k, c in sorted(by_kind.items())},
        "ms": {k: _pct(v) for k, v in sorted(times.items())},
    }
    if big is not None and missed:
        rec = 0
        for seed, k in missed:
            ctx, cs, m, kinds = planted_path(family, seed, path_len)
            nodes = [c.node for c in cs]
            try:
                w = big.solve(ctx.b, nodes[:k])
            except Exception:  # noqa: BLE001
                w = None
            rec += w is not None
        out["extended_rows"] = big.rows
        out["misses_recovered_by_extended"] = rec
    return out


def main():
    argv = [a for a in sys.argv[1:] if not a.startswith("--")]
    n_paths = int(argv[0]) if argv else 100
    path_len = int(argv[1]) if len(argv) > 1 else 24
    fake = "--fake" in sys.argv
    if fake:
        import pytest

        from tests import fake_device

        fake_device.install(pytest.MonkeyPatch())
    policy = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--round2=")), None)
    # the stand-in is slow: a budget that does not cut its rounds short
    s = (Sieve(rows=256, second_round=policy, budget_s=60.0) if fake
         else Sieve(second_round=policy))
    big = None
    if "--extended" in sys.argv:
        big = Sieve(rows=1 << 20)
    for family in FAMILIES:
        out = run_family(s, family, n_paths, path_len, big, feedback="--feedback" in sys.argv)
        out["device"] = "fake (CPU)" if fake else "gpu"
        print(json.dumps(out), flush=True)
    s.close()
    if big is not None:
        big.close()


if __name__ == "__main__":
    main()
