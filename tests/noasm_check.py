"""The C++ step() build of the interpreter (libmythril_hip_noasm.so, `make noasm`: every op through
exec.h, no asm core) on short-circuited tapes, against the oracle.  Run in its own process with
MYTHRIL_HIP_LIB naming that library (tests/test_gpu_parity.py::test_cpp_step_build_matches_oracle):

    MYTHRIL_HIP_LIB=mythril_amd/libmythril_hip_noasm.so python -m tests.noasm_check

The tape compiler reorders every Bool-root AND chain newest conjunct first with D_BANDZ between
the conjuncts (compile.cpp short_circuit); the asm core leaves a tape at a D_BANDZ whose running
conjunction is 0 in every lane, and the C++ driver must run the D_BANDZ and leave only then
(it used to stop before running it, so a tape's root was its first conjunct alone).
Checks per-tape hit counts and first witnesses (both modes) of config-5 tapes, and one LASER query
(KillBilly's) answered by the interpreter with a witness that is a model of the query.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main() -> int:
    lib_path = os.environ.get("MYTHRIL_HIP_LIB", "")
    assert lib_path.endswith("libmythril_hip_noasm.so"), lib_path
    from mythril_amd import native, synth
    from oracle import smt_eval

    native.load()
    ctx = native.Context(0)
    ts = synth.generate(48)
    seed, rows, base = 0x5EED, 1024, 333
    assigns = [smt_eval.gen_assignment(seed, ts.n_vars, base + r) for r in range(rows)]
    counts, first = [], []
    for t in ts.tapes:
        hits = [r for r in range(rows) if smt_eval.evaluate(t.nodes, ts.pool.values, assigns[r])]
        counts.append(len(hits))
        first.append(base + hits[0] if hits else native.NO_HIT)
    ct = ctx.compile(ts)
    a = ctx.assignments(ts.n_vars, rows)
    a.generate(seed, base)
    fh, hc = native.run(ctx, ct, a, index_base=base, mode=native.MODE_COUNT_ALL)
    assert [int(x) for x in hc] == counts, ([int(x) for x in hc], counts)
    assert [int(x) for x in fh] == first
    fh2, _ = native.run(ctx, ct, a, index_base=base, mode=native.MODE_FIRST_HIT)
    assert [int(x) for x in fh2] == first
    ctx.close()
    n_sat = sum(1 for c in counts if c)

    from mythril_amd.sieve import Sieve
    from mythril_amd.smt import And
    from oracle.term_eval import evaluate_term
    from tests.laser_like import queries
    from tests.test_lowering import model_of

    qctx, qs = queries()
    cs = dict(qs)["killbilly"]
    s = Sieve()
    try:
        w = s.solve(qctx.b, [c.node for c in cs])
    finally:
        s.close()
    assert w is not None, "no witness for KillBilly's query"
    names = [n for n, _ in sorted(qctx.b.var_index.items(), key=lambda kv: kv[1])]
    vars_, arrays, funcs = model_of(w.schema, w.values, qctx.b)
    tape = qctx.b.finish(And(*cs).node)
    assert evaluate_term(tape.nodes, qctx.b.pool.values, names, qctx.b.symbols.array_names,
                         qctx.b.symbols.function_names, vars_, arrays, funcs)
    print("noasm ok: %d tapes x %d rows (%d with hits) equal the oracle; KillBilly answered"
          % (len(ts.tapes), rows, n_sat))
    return 0


if __name__ == "__main__":
    sys.exit(main())
