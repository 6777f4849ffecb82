"""LASER-shaped path conditions grown to real path lengths (test helper).

The shapes of tests/laser_like.py stop at 8-22 constraints; a path at ``-t 2/3`` holds hundreds
(SURVEY §8(a) a1).  ``grow(base, n)`` keeps a base shape's constraints in order and interleaves
the constraints LASER adds along a path (svm.py:257-262: each new state's condition is its
parent's plus one), until the path holds ``n``:

* dispatcher fall-throughs: ``Not(Extract(255, 224, calldata[0:32]) == selector')`` for the
  other functions' selectors a Solidity dispatcher tests first (instructions.py:1543-1619);
* calldata-size guards of the ABI decoder: ``Not(ULT(calldatasize, 4 + 32 k))``;
* argument range checks (address / uint cleaning, require): ``ULT(arg_k, 2^m)``;
* SafeMath's overflow checks on the arguments: ``UGE(a + b, a)`` (``c >= a`` after an add);
* repeated storage reads of slots the path wrote (K(0) storage with stores, account.py:18-82);
* ``Not(sender == 0)`` and call-value bounds against the sender's balance.

Every filler holds under the base shape's intended witnesses (calldata of the right size, small
arguments, the selected function), so a grown SAT base stays SAT; ``unsat=True`` appends one
contradicting constraint (what an infeasible JUMPI branch costs).  Deterministic per seed.
"""
from __future__ import annotations

import random

from mythril_amd import smt
from mythril_amd.smt import (Not, ULT, UGE, ULE, symbol_factory)
from tests import laser_like as L

SELECTORS = [0x06FDDE03, 0x095EA7B3, 0x18160DDD, 0x23B872DD, 0x313CE567, 0x70A08231,
             0x8DA5CB5B, 0x95D89B41, 0xA9059CBB, 0xDD62ED3E, 0xF2FDE38B, 0x3CCFD60B,
             0x2E1A7D4D, 0xD0E30DB0, 0x41C0E1B5, 0x9FA299CC, 0x84057065, 0x7C11DA20]


def _base(name):
    if name == "killbilly":
        cs = L.killbilly()
        return cs, 2, ["1", "2", "3"]
    if name == "ether_thief":
        cs = L.ether_thief()
        return cs, 3, ["1"]
    if name == "overflow":
        cd = L.Calldata("1")
        x, y = cd.word(4), cd.word(36)
        cs = [L.sender_is_actor(symbol_factory.BitVecSym("sender_1", 256)),
              L.selector_is(cd, 0xA9059CBB),
              UGE(cd.size, symbol_factory.BitVecVal(68, 256)),
              ULT(cd.size, symbol_factory.BitVecVal(5000, 256)),
              Not(smt.BVAddNoOverflow(x, y, False))]
        return cs, 1, ["1"]
    raise ValueError(name)


def _selector_of(name, tx):
    return {("killbilly", "1"): 0x9FA299CC, ("killbilly", "2"): 0x84057065,
            ("killbilly", "3"): 0x7C11DA20, ("ether_thief", "1"): 0x2E1A7D4D,
            ("overflow", "1"): 0xA9059CBB}[(name, tx)]


def _fillers(name, tx, rng):
    """An endless stream of filler constraints for transaction `tx` of base `name`."""
    cd = L.Calldata(tx)
    sender = symbol_factory.BitVecSym("sender_%s" % tx, 256)
    value = symbol_factory.BitVecSym("call_value%s" % tx, 256)
    sel = _selector_of(name, tx)
    others = [s for s in SELECTORS if s != sel]
    rng.shuffle(others)
    n_args = 2 if name != "killbilly" or tx == "1" else 0
    k = 0
    while True:
        k += 1
        kind = rng.randrange(6)
        if kind == 0 and others:
            yield Not(L.selector_is(cd, others.pop()))
        elif kind == 1:
            yield Not(ULT(cd.size, symbol_factory.BitVecVal(4 + 32 * rng.randrange(1 + n_args),
                                                           256)))
        elif kind == 2 and n_args and name != "overflow":  # (an overflow needs large args)
            j = rng.randrange(n_args)
            yield ULT(cd.word(4 + 32 * j), symbol_factory.BitVecVal(1 << rng.choice(
                (160, 192, 224, 255)), 256))
        elif kind == 3 and n_args == 2 and name != "overflow":
            a, b = cd.word(4), cd.word(36)
            yield UGE(a + b, a)
        elif kind == 4:
            yield Not(sender == symbol_factory.BitVecVal(rng.randrange(1, 1 << 16), 256))
        elif kind == 5 and name == "ether_thief":
            yield ULE(value, symbol_factory.BitVecVal(10 ** 18 * (1 + rng.randrange(100)), 256))
        else:
            yield Not(ULT(cd.size, symbol_factory.BitVecVal(4, 256)))


def grow(name: str, n: int, seed: int = 0, unsat: bool = False):
    """(smt.Context, constraints): base shape `name` grown to `n` constraints (in LASER order:
    the base's constraints keep their order, fillers of each transaction follow its own
    constraints; the base's final goal constraints stay last)."""
    ctx = smt.Context()
    smt.set_context(ctx)
    rng = random.Random(seed * 1000 + n)
    base, goal_n, txs = _base(name)
    body, goal = base[:-goal_n], base[-goal_n:]
    extra = max(0, n - len(base) - (1 if unsat else 0))
    streams = {t: _fillers(name, t, rng) for t in txs}
    per = [extra // len(txs) + (1 if i < extra % len(txs) else 0) for i in range(len(txs))]
    # place each transaction's fillers after the body constraints that mention its calldata
    out, tx_i = [], 0
    chunks = [[] for _ in txs]
    for i, c in enumerate(body):
        chunks[min(len(txs) - 1, i * len(txs) // max(len(body), 1))].append(c)
    for t, chunk, m in zip(txs, chunks, per):
        out += chunk
        out += [next(streams[t]) for _ in range(m)]
        tx_i += 1
    out += goal
    if unsat:
        out.append(_contradiction(name))
    return ctx, out


def _contradiction(name):
    """One constraint that contradicts the grown path in a way folding cannot see."""
    if name == "killbilly":
        return symbol_factory.BitVecSym("sender_3", 256) == symbol_factory.BitVecVal(
            L.CREATOR, 256)
    if name == "ether_thief":
        return ULE(L.Calldata("1").word(4), symbol_factory.BitVecSym("call_value1", 256))
    cd = L.Calldata("1")
    lim = symbol_factory.BitVecVal(1 << 128, 256)
    return smt.And(ULT(cd.word(4), lim), ULT(cd.word(36), lim))
