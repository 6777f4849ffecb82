"""z3-style SMT-LIB text of one constraint (test helper): what ``z3.Solver().sexpr()`` prints for
a LASER constraint — the symbols it reads as ``declare-fun``s, then one ``assert`` whose shared
sub-terms are bound by nested ``let``s named ``a!1``, ``a!2``, ... (z3's printer introduces a let
for a sub-term it meets more than once).  z3 is absent here and on the GPU box; this printer
produces text of that shape from mythril_amd.smt terms, to time and test the import stage
(mythril_amd/smtlib.py Reader / Z3Importer, mh_smtlib_read) on LASER-shaped queries.
"""
from __future__ import annotations

from typing import Dict, List

from mythril_amd.smtlib import _OPNAME, _bv, _sort_str, _sym
from mythril_amd.tape import ARITY, F_ARRAY, Op


def z3_sexpr(c, head: str = "assert") -> str:
    """The declarations and the assert of Bool term `c`, z3-style (shared terms as lets).
    head="minimize": what ``z3.Optimize().minimize(t).sexpr()`` prints for a bit-vector term
    (the import of a single term, smtlib._z3_term_sexpr)."""
    b = c.ctx.b
    order: List[int] = []
    uses: Dict[int, int] = {}
    seen = set()
    stack = [(c.node, False)]
    while stack:
        n, done = stack.pop()
        if done:
            order.append(n)
            continue
        uses[n] = uses.get(n, 0) + 1
        if n in seen:
            continue
        seen.add(n)
        stack.append((n, True))
        for ch in reversed(b.nodes[n][2:2 + ARITY[Op(b.nodes[n][0])]]):
            stack.append((ch, False))
    var_names = {v: k for k, v in b.var_index.items()}
    decls, declared = [], set()
    for n in order:
        op, w, a, bb, cc, i0, i1 = b.nodes[n]
        op = Op(op)
        name = None
        if op == Op.VAR:
            name, sort = var_names[i0], "(_ BitVec %d)" % w
        elif op == Op.ARRAY:
            name, sort = b.symbols.array_names[i0], _sort_str(b, n)
        elif op == Op.UF:
            name = b.symbols.function_names[i0]
            _, dom, rng = b.symbols.functions[name]
            sort = None
            if name not in declared:
                declared.add(name)
                decls.append("(declare-fun %s ((_ BitVec %d)) (_ BitVec %d))"
                             % (_sym(name), dom, rng))
            continue
        if name is not None and name not in declared:
            declared.add(name)
            decls.append("(declare-fun %s () %s)" % (_sym(name), sort))
    names: Dict[int, str] = {}

    def expr(n: int) -> str:
        if n in names:
            return names[n]
        op, w, a, bb, cc, i0, i1 = b.nodes[n]
        op = Op(op)
        if op == Op.CONST:
            return _bv(b.pool.values[i0], w)
        if op == Op.TRUE:
            return "true"
        if op == Op.FALSE:
            return "false"
        if op == Op.VAR:
            return _sym(var_names[i0])
        if op == Op.ARRAY:
            return _sym(b.symbols.array_names[i0])
        if op == Op.CONST_ARRAY:
            return "((as const %s) %s)" % (_sort_str(b, n), expr(a))
        if op == Op.UF:
            return "(%s %s)" % (_sym(b.symbols.function_names[i0]), expr(a))
        if op == Op.EXTRACT:
            return "((_ extract %d %d) %s)" % (i0, i1, expr(a))
        if op == Op.ZEXT:
            return "((_ zero_extend %d) %s)" % (i0, expr(a))
        if op == Op.SEXT:
            return "((_ sign_extend %d) %s)" % (i0, expr(a))
        if op == Op.BVADD_NOOVFL_U:
            wa = b.widths[a]
            return ("(= ((_ extract %d %d) (bvadd ((_ zero_extend 1) %s) ((_ zero_extend 1) %s)))"
                    " #b0)" % (wa, wa, expr(a), expr(bb)))
        if op == Op.BVSUB_NOUDFL_U:
            return "(bvule %s %s)" % (expr(bb), expr(a))
        k = ARITY[op]
        return "(%s %s)" % (_OPNAME[op], " ".join(expr(x) for x in (a, bb, cc)[:k]))

    binds = []
    for n in order:
        op = Op(b.nodes[n][0])
        if uses.get(n, 0) > 1 and ARITY[op] > 0 and not (b.flags[n] & F_ARRAY) and n != c.node:
            text = expr(n)
            names[n] = "a!%d" % (len(binds) + 1)
            binds.append((names[n], text))
    body = expr(c.node)
    for name, text in reversed(binds):
        body = "(let ((%s %s))\n  %s)" % (name, text, body)
    return "\n".join(decls + ["(%s %s)" % (head, body)]) + "\n"
