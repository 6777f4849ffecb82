"""SMT-LIB2 <-> sieve terms: the ``--solver-log`` format and the z3 import path.

* ``parse(text)`` reads what the reference writes with ``--solver-log``
  (mythril/support/model.py:44-55: ``Optimize.sexpr()`` — declarations, ``assert``s,
  ``minimize`` / ``maximize``, ``check-sat``), and what ``z3.Solver.sexpr()`` prints for any set
  of LASER constraints, into mythril_amd.smt terms.  It covers the QF_ABV fragment LASER
  produces: every ``bv*`` operator including z3's ``bv*_i`` internal division
  names (identical to the plain ones for the non-zero divisors z3 emits them for), ``concat``,
  ``(_ extract i j)``, ``(_ zero_extend k)``, ``(_ sign_extend k)``, ``(_ repeat k)``,
  ``(_ rotate_left k)``, ``(_ rotate_right k)``, ``bvcomp``, ``bvumul_noovfl``, Boolean
  connectives (n-ary ``and``/``or``/``=``/``distinct``, ``=>``, ``xor``, ``ite``), ``let``,
  ``define-fun`` (0-ary), ``select``/``store``, ``((as const (Array ..)) v)`` and uninterpreted
  function application (keccak UFs).  Literals: ``#x..``, ``#b..``, ``(_ bvN w)``.
* ``to_smtlib(constraints, minimize, maximize)`` prints sieve terms in the same format
  (shared sub-terms as ``define-fun``), so ``--solver-log`` keeps working when the sieve
  front end answers, and ``parse(to_smtlib(q))`` round-trips.
* ``from_z3(constraints)`` imports the reference's z3-backed ``Bool``s (``.raw``) through
  ``sexpr()``, memoised per z3 AST (``get_id``), for the get_model front end; the text is read
  by the C++ session behind ``mh_smtlib_read`` (``NativeReader``), ``Reader`` below is its
  Python statement and parity reference.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple, Union

from . import smt
from .tape import ARITY, BOOL, F_ARRAY, Op, TapeError

Sexp = Union[str, list]


class SmtlibError(TapeError):
    pass


# -- reader ----------------------------------------------------------------------------------
_TOKEN = re.compile(r"""\s*(?:(;[^\n]*)|(\()|(\))|(\|[^|]*\|)|("(?:[^"]|"")*")|([^\s()|";]+))""")


def read_sexps(text: str) -> List[Sexp]:
    out: List[Sexp] = []
    stack: List[list] = []
    pos, n = 0, len(text)
    while pos < n:
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                break
            raise SmtlibError("cannot tokenize at %d: %r" % (pos, text[pos:pos + 20]))
        pos = m.end()
        comment, lp, rp, qsym, string, atom = m.groups()
        if comment is not None:
            continue
        if lp:
            stack.append([])
            continue
        if rp:
            if not stack:
                raise SmtlibError("unbalanced ')'")
            done = stack.pop()
            (stack[-1] if stack else out).append(done)
            continue
        tok = qsym[1:-1] if qsym is not None else (string if string is not None else atom)
        if qsym is not None:
            tok = _Quoted(tok)
        (stack[-1] if stack else out).append(tok)
    if stack:
        raise SmtlibError("unbalanced '('")
    return out


class _Quoted(str):
    """A |quoted| symbol: never a literal or keyword."""


# -- sorts -----------------------------------------------------------------------------------
@dataclass
class Sort:
    kind: str            # "bool" | "bv" | "array"
    width: int = 0       # bv width / array range width
    domain: int = 0      # array domain width


def _sort(s: Sexp) -> Sort:
    if s == "Bool":
        return Sort("bool")
    if isinstance(s, list) and len(s) == 3 and s[0] == "_" and s[1] == "BitVec":
        return Sort("bv", int(s[2]))
    if isinstance(s, list) and len(s) == 3 and s[0] == "Array":
        d, r = _sort(s[1]), _sort(s[2])
        if d.kind != "bv" or r.kind != "bv":
            raise SmtlibError("arrays must map bit-vectors to bit-vectors")
        return Sort("array", r.width, d.width)
    raise SmtlibError("unsupported sort %r" % (s,))


# -- term interpretation ---------------------------------------------------------------------
@dataclass
class Query:
    ctx: smt.Context
    constraints: List[smt.Bool] = field(default_factory=list)
    minimize: List[smt.BitVec] = field(default_factory=list)
    maximize: List[smt.BitVec] = field(default_factory=list)


_BV_BIN = {
    "bvadd": Op.BVADD, "bvsub": Op.BVSUB, "bvmul": Op.BVMUL, "bvudiv": Op.BVUDIV,
    "bvudiv_i": Op.BVUDIV, "bvurem": Op.BVUREM, "bvurem_i": Op.BVUREM, "bvsdiv": Op.BVSDIV,
    "bvsdiv_i": Op.BVSDIV, "bvsrem": Op.BVSREM, "bvsrem_i": Op.BVSREM, "bvsmod": Op.BVSMOD,
    "bvsmod_i": Op.BVSMOD, "bvand": Op.BVAND, "bvor": Op.BVOR, "bvxor": Op.BVXOR,
    "bvshl": Op.BVSHL, "bvlshr": Op.BVLSHR, "bvashr": Op.BVASHR,
}
_NARY_ASSOC = {"bvadd", "bvmul", "bvand", "bvor", "bvxor"}
_BV_CMP = {
    "bvult": Op.BVULT, "bvule": Op.BVULE, "bvugt": Op.BVUGT, "bvuge": Op.BVUGE,
    "bvslt": Op.BVSLT, "bvsle": Op.BVSLE, "bvsgt": Op.BVSGT, "bvsge": Op.BVSGE,
    "bvumul_noovfl": Op.BVMUL_NOOVFL_U,
}


class Reader:
    """Interprets SMT-LIB2 commands into terms of one smt.Context (node ids of its builder)."""

    def __init__(self, ctx: Optional[smt.Context] = None):
        self.ctx = ctx if ctx is not None else smt.Context()
        self.b = self.ctx.b
        self.decls: Dict[str, Tuple[str, Sort, Optional[Sort]]] = {}  # name -> (kind, sort, dom)
        self.defs: Dict[str, int] = {}

    # nodes carry their own sort: width (0 = Bool) and the array flag
    def _is_bool(self, n: int) -> bool:
        return self.b.widths[n] == BOOL and not self.b.is_array(n)

    def command(self, cmd: Sexp, q: Query) -> None:
        if not isinstance(cmd, list) or not cmd:
            raise SmtlibError("not a command: %r" % (cmd,))
        head = cmd[0]
        if head in ("set-option", "set-info", "set-logic", "check-sat", "get-model", "exit",
                    "get-objectives", "push", "pop", "echo"):
            return
        if head == "declare-fun":
            name, args_, res = cmd[1], cmd[2], cmd[3]
            if args_:
                if len(args_) != 1:
                    raise SmtlibError("only unary functions are supported: %s" % name)
                self.decls[name] = ("fun", _sort(res), _sort(args_[0]))
            else:
                self.decls[name] = ("const", _sort(res), None)
            return
        if head == "declare-const":
            self.decls[cmd[1]] = ("const", _sort(cmd[2]), None)
            return
        if head == "define-fun":
            name, args_, _res, body = cmd[1], cmd[2], cmd[3], cmd[4]
            if args_:
                raise SmtlibError("define-fun with arguments is not supported: %s" % name)
            self.defs[name] = self.term(body, {})
            return
        if head == "assert":
            n = self.term(cmd[1], {})
            if not self._is_bool(n):
                raise SmtlibError("assert of a non-Bool term")
            q.constraints.append(smt.Bool(n, self.ctx))
            return
        if head in ("minimize", "maximize"):
            n = self.term(cmd[1], {})
            (q.minimize if head == "minimize" else q.maximize).append(smt.BitVec(n, self.ctx))
            return
        raise SmtlibError("unsupported command %r" % (head,))

    def term(self, t: Sexp, env: Dict[str, int]) -> int:
        """The node of term `t`.  An explicit work stack, not recursion: LASER terms nest
        thousands deep (store chains of every SSTORE, ite chains of symbolic-index reads, folded
        Ands), far past Python's recursion limit."""
        vals: List[int] = []
        work: list = [(0, t, env)]
        steps = 0
        while work:
            item = work.pop()
            kind = item[0]
            steps += 1
            if kind == 0:  # evaluate item[1] in env item[2]
                _, t, env = item
                if isinstance(t, str):
                    vals.append(self._atom(t, env))
                    continue
                if not t:
                    raise SmtlibError("empty application")
                head = t[0]
                if head == "let":  # parallel let: every binding in the outer env
                    binds = t[1]
                    work.append((1, t[2], env, [name for name, _ in binds]))
                    work += [(0, val, env) for _, val in reversed(binds)]
                    continue
                if isinstance(head, list):
                    if len(t) != 2:
                        raise SmtlibError("indexed application takes 1 argument: %r" % (head,))
                    work.append((3, head))
                    work.append((0, t[1], env))
                    continue
                if head == "_":  # (_ bvN w)
                    if isinstance(t[1], str) and t[1].startswith("bv"):
                        vals.append(self.b.const(int(t[1][2:]), int(t[2])))
                        continue
                    raise SmtlibError("unsupported indexed term %r" % (t,))
                work.append((2, head, len(t) - 1))
                work += [(0, x, env) for x in reversed(t[1:])]
            elif kind == 1:  # let body, bindings on the value stack
                _, body, env, names = item
                k = len(names)
                bound = vals[len(vals) - k:] if k else []
                del vals[len(vals) - k:]
                env2 = dict(env)
                env2.update(zip(names, bound))
                work.append((0, body, env2))
            elif kind == 2:  # application of a named operator
                _, head, n = item
                a = vals[len(vals) - n:] if n else []
                del vals[len(vals) - n:]
                vals.append(self._apply(head, a))
            else:  # indexed operator / (as const ..) over the value on top
                vals.append(self._indexed(item[1], vals.pop()))
        assert len(vals) == 1
        return vals[0]

    def _atom(self, t: str, env: Dict[str, int]) -> int:
        b = self.b
        if not isinstance(t, _Quoted):
            if t == "true":
                return b.true()
            if t == "false":
                return b.false()
            if t.startswith("#x"):
                return b.const(int(t[2:], 16), 4 * (len(t) - 2))
            if t.startswith("#b"):
                return b.const(int(t[2:], 2), len(t) - 2)
        if t in env:
            return env[t]
        if t in self.defs:
            return self.defs[t]
        d = self.decls.get(t)
        if d is None:
            raise SmtlibError("undeclared symbol %r" % t)
        kind, sort, _ = d
        if kind != "const":
            raise SmtlibError("function %r used as a constant" % t)
        if sort.kind == "bool":
            v = b.user_var(t, 1)
            b.symbols.bool_vars.add(t)
            return b.op(Op.EQ, v, b.const(1, 1))
        if sort.kind == "bv":
            return b.user_var(t, sort.width)
        return b.array(t, sort.domain, sort.width)

    def _indexed(self, head: list, x: int) -> int:
        b = self.b
        if head[0] == "as" and head[1] == "const":
            s = _sort(head[2])
            return b.const_array(s.domain, x)
        if head[0] != "_":
            raise SmtlibError("unsupported application head %r" % (head,))
        name, idx = head[1], [int(x) for x in head[2:]]
        w = b.widths[x]
        if name == "extract":
            return b.op(Op.EXTRACT, x, imm0=idx[0], imm1=idx[1])
        if name == "zero_extend":
            return x if idx[0] == 0 else b.op(Op.ZEXT, x, imm0=idx[0])
        if name == "sign_extend":
            return x if idx[0] == 0 else b.op(Op.SEXT, x, imm0=idx[0])
        if name == "repeat":
            acc = x
            for _ in range(idx[0] - 1):
                acc = b.op(Op.CONCAT, acc, x)
            return acc
        if name in ("rotate_left", "rotate_right"):
            k = idx[0] % w
            if name == "rotate_right":
                k = (w - k) % w
            if k == 0:
                return x
            hi = b.op(Op.EXTRACT, x, imm0=w - k - 1, imm1=0)
            lo = b.op(Op.EXTRACT, x, imm0=w - 1, imm1=w - k)
            return b.op(Op.CONCAT, hi, lo)
        raise SmtlibError("unsupported indexed operator %r" % (name,))

    def _fold(self, op: Op, args_: List[int]) -> int:
        acc = args_[0]
        for x in args_[1:]:
            acc = self.b.op(op, acc, x)
        return acc

    def _add_noovfl(self, e: int, z: int) -> Optional[int]:
        """z3's BVAddNoOverflow(x, y, False) (bitvec_helper.py:178-189 builds it; z3 prints
        (= ((_ extract w w) (bvadd ((_ zero_extend 1) x) ((_ zero_extend 1) y))) #b0)) back to
        the one predicate, so the tape stays within 256 bits and the guide sees the overflow
        shape.  None when (e, z) is not that form."""
        nodes, pool = self.b.nodes, self.b.pool.values
        zo, zw, *_, zi0, _ = nodes[z]
        if Op(zo) != Op.CONST or zw != 1 or pool[zi0] & 1:
            return None
        eo, ew, ea, _, _, hi, lo = nodes[e]
        if Op(eo) != Op.EXTRACT or hi != lo or ew != 1:
            return None
        so, sw, sa, sb, *_ = nodes[ea]
        if Op(so) != Op.BVADD or sw != hi + 1:
            return None
        inner = []
        for k in (sa, sb):
            ko, kw, ka, _, _, ki0, _ = nodes[k]
            if Op(ko) != Op.ZEXT or ki0 != 1 or nodes[ka][1] != hi:
                return None
            inner.append(ka)
        return self.b.op(Op.BVADD_NOOVFL_U, inner[0], inner[1])

    def _apply(self, head: str, a: List[int]) -> int:
        b = self.b
        if head in _BV_BIN:
            if len(a) > 2 and head not in _NARY_ASSOC and head != "bvsub":
                raise SmtlibError("%s takes 2 arguments" % head)
            return self._fold(_BV_BIN[head], a)
        if head in _BV_CMP:
            return b.op(_BV_CMP[head], a[0], a[1])
        if head == "bvneg":
            return b.op(Op.BVNEG, a[0])
        if head == "bvnot":
            return b.op(Op.BVNOT, a[0])
        if head in ("bvnand", "bvnor", "bvxnor"):
            inner = {"bvnand": Op.BVAND, "bvnor": Op.BVOR, "bvxnor": Op.BVXOR}[head]
            return b.op(Op.BVNOT, b.op(inner, a[0], a[1]))
        if head == "bvcomp":
            return b.op(Op.ITE, b.op(Op.EQ, a[0], a[1]), b.const(1, 1), b.const(0, 1))
        if head == "concat":
            return self._fold(Op.CONCAT, a)
        if head == "and":
            return b.true() if not a else self._fold(Op.AND, a)
        if head == "or":
            return b.false() if not a else self._fold(Op.OR, a)
        if head == "xor":
            return self._fold(Op.XOR, a)
        if head == "not":
            return b.op(Op.NOT, a[0])
        if head == "=>":
            return b.op(Op.OR, b.op(Op.NOT, a[0]), a[1])
        if head == "=":
            if any(b.is_array(x) for x in a):
                raise SmtlibError("equality between arrays is not supported")
            if len(a) == 2:
                nov = self._add_noovfl(a[0], a[1])
                if nov is None:
                    nov = self._add_noovfl(a[1], a[0])
                if nov is not None:
                    return nov
            eqs = [b.op(Op.EQ, a[i], a[i + 1]) for i in range(len(a) - 1)]
            return self._fold(Op.AND, eqs)
        if head == "distinct":
            ne = [b.op(Op.NOT, b.op(Op.EQ, a[i], a[j]))
                  for i in range(len(a)) for j in range(i + 1, len(a))]
            return self._fold(Op.AND, ne)
        if head == "ite":
            if b.is_array(a[1]):
                raise SmtlibError("ite over arrays is not supported")
            return b.op(Op.ITE, a[0], a[1], a[2])
        if head == "select":
            return b.select(a[0], a[1])
        if head == "store":
            return b.store(a[0], a[1], a[2])
        d = self.decls.get(head)
        if d is not None and d[0] == "fun":
            _, res, dom = d
            if res.kind != "bv" or dom.kind != "bv":
                raise SmtlibError("function %s must map bit-vectors to bit-vectors" % head)
            return b.apply(head, dom.width, res.width, a[0])
        raise SmtlibError("unsupported operator %r" % (head,))


def parse(text: str, ctx: Optional[smt.Context] = None) -> Query:
    r = Reader(ctx)
    q = Query(r.ctx)
    for cmd in read_sexps(text):
        r.command(cmd, q)
    return q


# -- writer ----------------------------------------------------------------------------------
_SIMPLE = re.compile(r"^[A-Za-z~!@$%^&*_+=<>.?/\-][0-9A-Za-z~!@$%^&*_+=<>.?/\-]*$")
_RESERVED = {"true", "false", "let", "as", "_", "!", "par", "forall", "exists", "assert"}
_OPNAME = {
    Op.BVADD: "bvadd", Op.BVSUB: "bvsub", Op.BVMUL: "bvmul", Op.BVUDIV: "bvudiv",
    Op.BVUREM: "bvurem", Op.BVSDIV: "bvsdiv", Op.BVSREM: "bvsrem", Op.BVSMOD: "bvsmod",
    Op.BVNEG: "bvneg", Op.BVNOT: "bvnot", Op.BVAND: "bvand", Op.BVOR: "bvor",
    Op.BVXOR: "bvxor", Op.BVSHL: "bvshl", Op.BVLSHR: "bvlshr", Op.BVASHR: "bvashr",
    Op.EQ: "=", Op.BVULT: "bvult", Op.BVULE: "bvule", Op.BVUGT: "bvugt", Op.BVUGE: "bvuge",
    Op.BVSLT: "bvslt", Op.BVSLE: "bvsle", Op.BVSGT: "bvsgt", Op.BVSGE: "bvsge",
    Op.AND: "and", Op.OR: "or", Op.XOR: "xor", Op.NOT: "not", Op.ITE: "ite",
    Op.CONCAT: "concat", Op.BVMUL_NOOVFL_U: "bvumul_noovfl", Op.SELECT: "select",
    Op.STORE: "store",
}


def _sym(name: str) -> str:
    return name if _SIMPLE.match(name) and name not in _RESERVED else "|%s|" % name


def _bv(value: int, width: int) -> str:
    if width % 4 == 0:
        return "#x%0*x" % (width // 4, value)
    return "#b%s" % format(value, "0%db" % width)


def _sort_str(b, n: int) -> str:
    if b.is_array(n):
        return "(Array (_ BitVec %d) (_ BitVec %d))" % (b.nodes[n][6], b.widths[n])
    w = b.widths[n]
    return "Bool" if w == BOOL else "(_ BitVec %d)" % w


def to_smtlib(constraints: Sequence, minimize: Sequence = (), maximize: Sequence = ()) -> str:
    """SMT-LIB2 text of sieve terms (the shape of ``Optimize.sexpr()``)."""
    items = list(constraints) + list(minimize) + list(maximize)
    if not items:
        return "(check-sat)\n"
    ctx = items[0].ctx
    b = ctx.b
    roots = [x.node for x in items]
    order, uses = [], {}
    seen = set()
    stack = [(r, False) for r in reversed(roots)]
    while stack:
        n, done = stack.pop()
        if done:
            order.append(n)
            continue
        if n in seen:
            uses[n] = uses.get(n, 0) + 1
            continue
        seen.add(n)
        uses[n] = uses.get(n, 0) + 1
        stack.append((n, True))
        op = b.nodes[n][0]
        for ch in reversed(b.nodes[n][2:2 + ARITY[Op(op)]]):
            stack.append((ch, False))
    names: Dict[int, str] = {}
    lines: List[str] = []
    var_names = {v: k for k, v in b.var_index.items()}
    declared = set()
    for n in order:
        op, w, a, bb, c, i0, i1 = b.nodes[n]
        op = Op(op)
        if op == Op.VAR:
            name = var_names[i0]
            if name not in declared:
                declared.add(name)
                lines.append("(declare-fun %s () %s)" % (_sym(name), "(_ BitVec %d)" % w))
        elif op == Op.ARRAY:
            name = b.symbols.array_names[i0]
            if name not in declared:
                declared.add(name)
                lines.append("(declare-fun %s () %s)" % (_sym(name), _sort_str(b, n)))
        elif op == Op.UF:
            name = b.symbols.function_names[i0]
            if name not in declared:
                declared.add(name)
                _, dom, rng = b.symbols.functions[name]
                lines.append("(declare-fun %s ((_ BitVec %d)) (_ BitVec %d))"
                             % (_sym(name), dom, rng))
    body: List[str] = []

    def expr(n: int) -> str:
        op, w, a, bb, c, i0, i1 = b.nodes[n]
        op = Op(op)
        if n in names:
            return names[n]
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
        if op == Op.BVADD_NOOVFL_U:  # (= ((_ extract w w) (bvadd zext1 a, zext1 b)) #b0)
            wa = b.widths[a]
            return ("(= ((_ extract %d %d) (bvadd ((_ zero_extend 1) %s) ((_ zero_extend 1) %s)))"
                    " #b0)" % (wa, wa, expr(a), expr(bb)))
        if op == Op.BVSUB_NOUDFL_U:
            return "(bvule %s %s)" % (expr(bb), expr(a))
        if op == Op.KECCAK:
            raise SmtlibError("KECCAK (concrete hash) has no SMT-LIB form")
        if op in (Op.EVM_ADDMOD, Op.EVM_MULMOD):  # z3's exact form (mythril_hip.h)
            zx = lambda k: "((_ zero_extend 256) %s)" % expr(k)
            r = "((_ extract 255 0) (bvurem (%s %s %s) %s))" % (
                "bvadd" if op == Op.EVM_ADDMOD else "bvmul", zx(a), zx(bb), zx(c))
            if i0 == 1:
                return r
            zero = "#x" + "0" * 64
            return "(ite (= %s %s) %s %s)" % (expr(c), zero, zero, r)
        if op in (Op.EVM_EXP, Op.EVM_SIGNEXTEND, Op.EVM_BYTE):
            raise SmtlibError("%s has no SMT-LIB form" % op.name)
        k = ARITY[op]
        return "(%s %s)" % (_OPNAME[op], " ".join(expr(x) for x in (a, bb, c)[:k]))

    for n in order:
        op = Op(b.nodes[n][0])
        if uses.get(n, 0) > 1 and ARITY[op] > 0 and not (b.flags[n] & F_ARRAY):
            name = "|$%d|" % n
            body.append("(define-fun %s () %s %s)" % (name, _sort_str(b, n), expr(n)))
            names[n] = name
    for x in constraints:
        body.append("(assert %s)" % expr(x.node))
    for x in minimize:
        body.append("(minimize %s)" % expr(x.node))
    for x in maximize:
        body.append("(maximize %s)" % expr(x.node))
    body.append("(check-sat)")
    return "\n".join(lines + body) + "\n"


class NativeReader:
    """The product path's SMT-LIB reader: the C++ session behind mh_smtlib_read (same fragment
    and the same terms as ``Reader``, tests/test_smtlib_native.py), hash-consing against what it
    has already handed to this context's builder, so a constraint that extends its parent's only
    builds its new nodes on the host."""

    def __init__(self, ctx: Optional[smt.Context] = None):
        from . import native

        self.ctx = ctx if ctx is not None else smt.Context()
        self.b = self.ctx.b
        self.session = native.SmtlibSession()

    def read(self, text: str, q: Query) -> None:
        from . import native

        try:
            items = self.session.read(text, self.b)
        except native.SieveError as e:
            raise SmtlibError(str(e)) from None
        for kind, node in items:
            if kind == native.SMT_ASSERT:
                q.constraints.append(smt.Bool(node, self.ctx))
            elif kind == native.SMT_MINIMIZE:
                q.minimize.append(smt.BitVec(node, self.ctx))
            else:
                q.maximize.append(smt.BitVec(node, self.ctx))


def parse_native(text: str, ctx: Optional[smt.Context] = None) -> Query:
    """``parse`` through the C++ reader."""
    r = NativeReader(ctx)
    q = Query(r.ctx)
    r.read(text, q)
    return q


# -- z3 import -------------------------------------------------------------------------------
def _z3_sexpr(raw) -> str:
    import z3  # only on a box where the reference runs

    s = z3.Solver()
    s.add(raw)
    return s.sexpr()


def _z3_term_sexpr(raw) -> str:
    """SMT-LIB2 of one reference term of any sort, as z3 prints it: a Bool as an assert, a
    bit-vector as an Optimize objective (``(minimize t)``: the reader hands its node back)."""
    import z3

    if z3.is_bool(raw):
        return _z3_sexpr(raw)
    o = z3.Optimize()
    o.minimize(raw)
    return o.sexpr()


class Z3Importer:
    """z3-backed reference terms -> sieve terms, memoised per z3 AST id (callable as the
    front end's ``to_terms``).

    Memory stays bounded over a long ``myth analyze`` run: the memo is an LRU of at most
    ``max_memo`` ASTs, and once the reader's term store holds more than ``max_nodes`` nodes the
    importer starts over with a fresh context (between two queries, never inside one) and calls
    ``on_reset`` — the front end drops every cache keyed by the old context's node ids then (the
    sieve's parent-witness table).  ``sexpr_of`` prints one reference term as SMT-LIB2 (z3's
    ``Solver.sexpr()`` by default)."""

    def __init__(self, ctx: Optional[smt.Context] = None, max_memo: int = 1 << 16,
                 max_nodes: int = 1 << 21, sexpr_of=None, on_reset=None, term_sexpr_of=None):
        from collections import OrderedDict

        self.reader = NativeReader(ctx)
        self.memo: "OrderedDict[int, Tuple[object, int]]" = OrderedDict()
        self.max_memo = max_memo
        self.max_nodes = max_nodes
        self.sexpr_of = sexpr_of or _z3_sexpr
        # one term of any sort (Model.eval / Model[decl] of reference terms): _z3_term_sexpr
        self.term_sexpr_of = term_sexpr_of or _z3_term_sexpr
        self.on_reset = on_reset
        self.resets = 0

    def reset(self) -> None:
        self.reader.session.close()
        self.reader = NativeReader()
        self.memo.clear()
        self.resets += 1
        if self.on_reset is not None:
            self.on_reset()

    def n_nodes(self) -> int:
        return len(self.reader.b.nodes)

    def __call__(self, constraints):
        if self.n_nodes() > self.max_nodes:
            self.reset()
        out = []
        for c in constraints:
            raw = getattr(c, "raw", c)
            key = raw.get_id()
            got = self.memo.get(key)
            if got is None or got[0] is not raw:
                q = Query(self.reader.ctx)
                self.reader.read(self.sexpr_of(raw), q)
                node = q.constraints[-1].node if len(q.constraints) == 1 else \
                    smt.And(*q.constraints).node
                got = self.memo[key] = (raw, node)
                while len(self.memo) > self.max_memo:
                    self.memo.popitem(last=False)
            else:
                self.memo.move_to_end(key)
            out.append(smt.Bool(got[1], self.reader.ctx))
        return self.reader.ctx, out

    @property
    def ctx(self) -> smt.Context:
        return self.reader.ctx

    def term(self, raw) -> "smt.Expression":
        """One reference term of any sort (a z3 ``ExprRef``: Bool or bit-vector, up to 512 bits
        and beyond) as a term of this importer's context, for Model.eval / Model[decl] of the
        reference's callers (calldata.py:240-244, analysis/solver.py:141,174-176,
        keccak_function_manager.py:113).  Memoised with the constraints; never resets the
        context (a model's terms must stay in the context its witness was found in)."""
        key = ("term", raw.get_id())
        got = self.memo.get(key)
        if got is None or got[0] is not raw:
            q = Query(self.reader.ctx)
            self.reader.read(self.term_sexpr_of(raw), q)
            if len(q.constraints) == 1 and not q.minimize and not q.maximize:
                node, is_bool = q.constraints[0].node, True
            elif len(q.minimize) == 1 and not q.constraints:
                node, is_bool = q.minimize[0].node, False
            else:
                raise SmtlibError("a single term was expected, got %d asserts and %d objectives"
                                  % (len(q.constraints), len(q.minimize) + len(q.maximize)))
            got = self.memo[key] = (raw, (node, is_bool))
            while len(self.memo) > self.max_memo:
                self.memo.popitem(last=False)
        else:
            self.memo.move_to_end(key)
        node, is_bool = got[1]
        return (smt.Bool if is_bool else smt.BitVec)(node, self.reader.ctx)
