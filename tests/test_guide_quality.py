"""The harvested guide solves every SAT LASER-shaped query within the sieve's first round.

The first launch of ``Sieve.solve`` is ``first_rows`` (256) guided rows; the front end's latency
figures assume every SAT shape of tests/laser_like.py is found there.  This checks
it on the CPU with the oracle restatements of the generator (oracle/guided_gen.py) and of tape
evaluation (oracle/smt_eval.py): each variable-disjoint group (one device tape) has a satisfying
row among the first 256, so the sieve's first round returns a witness for the query.
"""
import pytest

from mythril_amd.candidates import build_guide
from mythril_amd.lower import lower_query
from mythril_amd.sieve import Sieve, local_tape
from mythril_amd.tape import Op
from oracle import smt_eval as E
from oracle.guided_gen import generate_row
from tests.laser_like import queries

FIRST_ROWS = 256
SEED = 0x5EED5EED  # Sieve's default seed


SAT_SHAPES = [n for n, _ in queries()[1] if not n.startswith("unsat")]


@pytest.mark.parametrize("name", SAT_SHAPES)
def test_first_round_solves_the_sat_queries(name):
    ctx, qs = queries()
    cs = dict(qs)[name]
    b = ctx.b
    root, schema = lower_query(b, [c.node for c in cs])
    cols = list(schema.columns)
    guide = build_guide(b, root, schema, cols).arrays()
    rows = [generate_row(SEED, (1 << 24) + r, guide) for r in range(FIRST_ROWS)]
    for conj, _ in Sieve.buckets(b, root):
        acc = conj[0]
        for x in conj[1:]:
            acc = b.op(Op.AND, acc, x)
        nodes = local_tape(b, acc, cols)
        assert any(E.evaluate(nodes, b.pool.values, row) for row in rows), (name, len(conj))
