"""Queries whose satisfiability is known by construction: planted models (test helper; VERDICT r4
next 4).

A random model M is drawn first -- scalar symbols, array tables with an else value, tables of
uninterpreted functions, keccak functions that obey the keccak manager's interval / mod-64 /
inverse conditions -- and then constraints of a query family are generated one at a time and
ORIENTED to hold under M: a comparison that M falsifies is swapped or negated, an equality is
pinned to M's value of its term.  Every constraint is checked by the ORACLE (oracle/term_eval.py)
under M before it joins the path, and one that does not hold is dropped, so every prefix of a
path is satisfiable (M is a model of it) whatever the sieve does.  The sieve's recall on such
paths -- the share of SAT queries it answers -- is what decides whether a query pays z3 at all
(svm.py:257-262: LASER asks is_possible for every new state).

Families:
* ``random``: the shapes of tests/test_query_native._random_query (free and K arrays, stores,
  selects at constant and symbolic keys, a tabled function, keccak pairs / bounds / inverses,
  wide equalities);
* ``laser``: 1-3 message calls: dispatcher checks, ABI calldata-size guards, argument range checks,
  SafeMath and the IntegerArithmetics module's no-overflow predicates (integer.py:141-157),
  senders in ACTORS and the Suicide module's caller checks (suicide.py:68-81), call values against
  balances and the EtherThief module's balance growth (ether_thief.py:65-73), storage slots and
  mappings through the keccak manager (keccak_function_manager.py:83-149).
"""
from __future__ import annotations

import random
from typing import Callable, Dict, List, Tuple

from mythril_amd import smt
from mythril_amd.smt import (And, Array, BVAddNoOverflow, BVMulNoOverflow, Concat, Function, If,
                             K, Not, UGE, UGT, ULE, ULT, symbol_factory)
from oracle.keccak import keccak256
from oracle.term_eval import evaluate_term
from tests import laser_like as L
from tests.laser_paths import SELECTORS

BVV = symbol_factory.BitVecVal
BVS = symbol_factory.BitVecSym
M256 = (1 << 256) - 1


class Planted:
    """A model: vars {name: int}, arrays {name: (table, else)}, functions {name: callable}."""

    def __init__(self):
        self.vars: Dict[str, int] = {}
        self.arrays: Dict[str, Tuple[dict, int]] = {}
        self.funcs: Dict[str, Callable[[int], int]] = {}

    def value(self, ctx, term) -> int:
        b = ctx.b
        names = [n for n, _ in sorted(b.var_index.items(), key=lambda kv: kv[1])]
        tape = b.finish(term.node)
        return evaluate_term(tape.nodes, b.pool.values, names, b.symbols.array_names,
                             b.symbols.function_names, self.vars, self.arrays, self.funcs)

    def holds(self, ctx, c) -> bool:
        return bool(self.value(ctx, c))


def _keccak_pair(m: Planted, name: str, nbytes: int, image: Callable[[int], int]):
    """keccak256_N and its inverse in M: f(x) = image(x), inv(f(x)) = x for every x met."""
    inv: Dict[int, int] = {}

    def f(x):
        y = image(x)
        inv[y] = x
        return y

    m.funcs[name] = f
    m.funcs[name + "-1"] = lambda y: inv.get(y, 0)


def _real_keccak(nbytes):
    return lambda x: int.from_bytes(keccak256(x.to_bytes(nbytes, "big")), "big")


class _Path:
    def __init__(self, ctx, m: Planted):
        self.ctx, self.m = ctx, m
        self.cs: List[smt.Bool] = []
        self.kinds: List[str] = []  # the shape class of each constraint
        self.kind = ""
        self.dropped = 0

    def add(self, c) -> None:
        """Append `c` if it holds under M (the oracle decides); count it dropped otherwise."""
        if self.m.holds(self.ctx, c):
            self.cs.append(c)
            self.kinds.append(self.kind)
        else:
            self.dropped += 1

    def orient(self, c) -> None:
        """`c` or its negation, whichever holds under M."""
        self.add(c if self.m.holds(self.ctx, c) else Not(c))

    def ult(self, a, b) -> None:
        """ULT(a, b) oriented: swapped when M has a > b, negated when equal."""
        va, vb = self.m.value(self.ctx, a), self.m.value(self.ctx, b)
        self.add(ULT(a, b) if va < vb else ULT(b, a) if vb < va else Not(ULT(a, b)))

    def pin(self, t) -> None:
        """t == M(t)."""
        self.add(t == BVV(self.m.value(self.ctx, t), t.size()))


def _draw256(rng) -> int:
    r = rng.random()
    if r < 0.3:
        return rng.randrange(64)
    if r < 0.5:
        return rng.choice((0, 1, 4, 36, 1 << 160))
    if r < 0.7:
        return rng.getrandbits(160)
    return rng.getrandbits(256)


# -- random family --------------------------------------------------------------------------------

def planted_random(rng: random.Random, n: int):
    """(ctx, constraints, model, kinds): n attempts at _random_query's shapes, oriented to M."""
    ctx = smt.set_context(smt.Context())
    m = Planted()
    xs = [BVS("x%d" % i, 256) for i in range(3)]
    for i in range(3):
        m.vars["x%d" % i] = _draw256(rng)
    keys = [0, 1, 4, 36, 1 << 160]
    arrs = [Array("A", 256, 256), Array("B", 256, 8)]
    m.arrays["A"] = ({k: _draw256(rng) for k in keys if rng.random() < 0.6}, _draw256(rng))
    m.arrays["B"] = ({k: rng.randrange(256) for k in keys if rng.random() < 0.6},
                     rng.randrange(256))
    kar = K(256, 256, 7)
    f = Function("f", 256, 256)
    ftab = {k: _draw256(rng) for k in keys if rng.random() < 0.5}
    fels = _draw256(rng)
    m.funcs["f"] = lambda x: ftab.get(x, fels)
    # keccak as LASER builds it: every application through the keccak manager, whose condition
    # (interval / mod 64 / inverse, or a remembered concrete pair) joins the path before the
    # constraint that uses it (keccak_function_manager.py:83-149).  M: the real hash on the keys
    # the family hashes concretely, the manager's interval elsewhere (a multiple of 64)
    km = L.KeccakManager()
    km.functions(256)
    real = _real_keccak(32)
    keyset = set(keys)

    fixed: Dict[int, int] = {}  # M is a function: a point's value never changes once read

    def kimage(x):
        if x not in fixed:
            if x in keyset or (x, 256) in km.concrete or 256 not in km.hooks:
                fixed[x] = real(x)
            else:
                fixed[x] = km.hooks[256] * L.PART + ((real(x) >> 139) << 6)
        return fixed[x]

    _keccak_pair(m, "keccak256_256", 32, kimage)
    pending: List[smt.Bool] = []

    def kec(t):
        h, cond = km.create(t)
        pending.append(cond)
        return h

    kv = [BVV(k, 256) for k in keys]

    def term(d=0):
        r = rng.random()
        if d > 2 or r < 0.25:
            return rng.choice(xs + kv)
        if r < 0.45:
            a = rng.choice(arrs + [kar])
            idx = rng.choice(kv) if rng.random() < 0.6 else term(d + 1)
            return smt.ZeroExt(248, a[idx]) if a.range == 8 else a[idx]
        if r < 0.55:
            return f(rng.choice(kv) if rng.random() < 0.5 else term(d + 1))
        if r < 0.7:
            return kec(term(d + 1))
        if r < 0.85:
            return term(d + 1) + term(d + 1)
        return If(ULT(term(d + 1), term(d + 1)), term(d + 1), term(d + 1))

    p = _Path(ctx, m)

    class _Keccak(_Path):  # the manager's conditions first, then the constraint
        def add(self, c):
            kind, self.kind = self.kind, "keccak_cond"
            for x in pending:
                _Path.add(self, x)
            pending.clear()
            self.kind = kind
            _Path.add(self, c)

    p.__class__ = _Keccak
    for _ in range(n):
        r = rng.random()
        if r < 0.1:  # a store into the free array, read back
            p.kind = "store"
            a = arrs[0]
            a[rng.choice(kv)] = term(1)
            t = a[term(2)]
            p.pin(t) if rng.random() < 0.5 else p.orient(t == term(2))
        elif r < 0.2:  # a concrete keccak pair
            p.kind = "keccak_pair"
            p.pin(kec(rng.choice(kv)))
        elif r < 0.3:  # a keccak bound
            p.kind = "keccak_bound"
            p.orient(UGT(kec(term(1)), BVV(rng.getrandbits(200) << 40, 256)))
        elif r < 0.38:  # a wide equality
            p.kind = "wide_eq"
            t = Concat(term(1), term(1))
            p.pin(t) if rng.random() < 0.5 else p.orient(t == Concat(term(1), term(1)))
        elif r < 0.55:
            p.kind = "pinned"
            p.pin(term())
        elif r < 0.7:
            p.kind = "eq"
            p.orient(term() == term())
        else:
            p.kind = "ult"
            p.ult(term(), term())
    return ctx, p.cs, m, p.kinds


# -- LASER family ---------------------------------------------------------------------------------

ACTORS = (L.CREATOR, L.ATTACKER, L.SOMEGUY)


def planted_laser(rng: random.Random, n: int):
    """(ctx, constraints, model, kinds): a path of up to 3 message calls, n constraint attempts."""
    ctx = smt.set_context(smt.Context())
    m = Planted()
    n_tx = rng.choice((1, 1, 2, 3))
    km = L.KeccakManager()
    # the keccak functions M needs: mapping slots hash 512-bit (key . slot) inputs into the
    # manager's interval for that width (the same hook the manager gives it), multiples of 64
    txs = []
    balances = Array("balance", 256, 256)
    starting = Array("balance", 256, 256)  # world_state.py:34: the copy before any transaction
    storage = Array("Storage", 256, 256)
    m.arrays["balance"] = ({a: rng.choice((0, 10 ** 18, rng.getrandbits(80))) for a in ACTORS},
                           rng.getrandbits(64))
    m.arrays["Storage"] = ({s: _draw256(rng) for s in range(4) if rng.random() < 0.7}, 0)
    for t in range(1, n_tx + 1):
        cd = L.Calldata(str(t))
        sender = BVS("sender_%d" % t, 256)
        value = BVS("call_value%d" % t, 256)
        sel = rng.choice(SELECTORS)
        n_args = rng.randrange(3)
        args = [rng.choice((rng.randrange(1 << 16), rng.getrandbits(160), rng.getrandbits(256)))
                for _ in range(n_args)]
        size = 4 + 32 * n_args + rng.choice((0, 0, 0, 1, 5))
        data = sel.to_bytes(4, "big") + b"".join(a.to_bytes(32, "big") for a in args)
        data += bytes(rng.randrange(256) for _ in range(size - len(data)))
        m.vars["%d_calldatasize" % t] = size
        m.arrays["%d_calldata" % t] = ({i: x for i, x in enumerate(data)}, rng.randrange(256))
        m.vars["sender_%d" % t] = rng.choice(ACTORS)
        m.vars["call_value%d" % t] = rng.choice((0, 0, rng.randrange(1, 1 << 20)))
        txs.append((cd, sender, value, sel, n_args))

    def kimage(x):
        lo = km.hooks[512] * L.PART
        h = int.from_bytes(keccak256(x.to_bytes(64, "big")), "big")
        return lo + ((h >> 139) << 6)

    _keccak_pair(m, "keccak256_512", 64, kimage)
    p = _Path(ctx, m)
    dispatched = set()
    for _ in range(n):
        cd, sender, value, sel, n_args = txs[rng.randrange(len(txs))]
        t = txs.index((cd, sender, value, sel, n_args)) + 1
        words = [cd.word(4 + 32 * j) for j in range(n_args)]
        kind = rng.randrange(12)
        if kind == 0 or t not in dispatched:  # the dispatcher: this function's selector
            dispatched.add(t)
            p.kind = "dispatch"
            p.add(L.selector_is(cd, sel))
        elif kind == 1:  # a selector tested before this one, not taken
            p.kind = "dispatch"
            p.add(Not(L.selector_is(cd, rng.choice([s for s in SELECTORS if s != sel]))))
        elif kind == 2:  # the ABI decoder's size guards
            p.kind = "size_guard"
            k = rng.randrange(n_args + 1)
            p.add(Not(ULT(cd.size, BVV(4 + 32 * k, 256))))
            if rng.random() < 0.3:
                p.add(ULT(cd.size, BVV(rng.choice((5000, 4 + 32 * n_args + 32)), 256)))
        elif kind == 3 and words:  # argument cleaning / require(arg < bound)
            p.kind = "arg_range"
            p.orient(ULT(rng.choice(words), BVV(1 << rng.choice((8, 16, 160, 192, 255)), 256)))
        elif kind == 4 and len(words) == 2:  # SafeMath, and IntegerArithmetics' predicates
            p.kind = "overflow"
            a, b = words
            r = rng.random()
            if r < 0.4:
                p.orient(UGE(a + b, a))
            elif r < 0.7:
                p.orient(BVAddNoOverflow(a, b, False))
            else:
                p.orient(BVMulNoOverflow(a, b, False))
        elif kind == 5:  # sender in ACTORS (transaction/symbolic.py:87-104)
            p.kind = "actors"
            p.add(L.sender_is_actor(sender))
        elif kind == 6:  # an owner check, taken or not
            p.kind = "owner"
            p.orient(sender == BVV(rng.choice(ACTORS), 256))
        elif kind == 7:  # the call value against the sender's balance, non-payable checks
            p.kind = "value"
            if rng.random() < 0.5:
                p.orient(value == BVV(0, 256))
            else:
                p.orient(UGE(balances[sender], value))
        elif kind == 8:  # a storage slot read
            p.kind = "storage"
            p.pin(storage[BVV(rng.randrange(4), 256)])
        elif kind == 9:  # a mapping read: keccak(key . slot) with the manager's conditions
            p.kind = "mapping"
            key = rng.choice([sender] + [w & BVV((1 << 160) - 1, 256) for w in words])
            slot_t, cond = L.mapping_slot(km, key, rng.randrange(1, 4))
            p.add(cond)
            p.pin(storage[slot_t])
        elif kind == 10:  # the Suicide module: caller == attacker and caller == origin
            p.kind = "suicide"
            p.orient(And(sender == BVV(L.ATTACKER, 256), sender == sender))
        else:  # EtherThief: the attacker's balance after a transfer, against the start
            p.kind = "ether_thief"
            amount = words[0] if words else value
            bal = balances[sender]
            p.orient(UGT(bal + amount, starting[sender]))
    return ctx, p.cs, m, p.kinds


FAMILIES = {"random": planted_random, "laser": planted_laser}


def planted_path(family: str, seed: int, n: int):
    """(ctx, constraints, model, kinds) of one planted path (deterministic per family, seed, n):
    kinds[i] is the shape class of constraints[i]."""
    salt = {"random": 0, "laser": 1 << 24}[family]
    return FAMILIES[family](random.Random(salt + seed * 7919 + n), n)
