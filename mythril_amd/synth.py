"""Synthetic constraint-tape generator for BASELINE.json config 5.

10^4 seeded random tapes over V = 4 free 256-bit variables (calldata word, caller, callvalue,
storage value), the shape of LASER path constraints: arithmetic/bitwise/shift/ext-concat
chains over the variables and the constants mythril's constraints carry (the ACTORS addresses,
mythril/laser/ethereum/transaction/symbolic.py:22-31; 4-byte function selectors), compared and
conjoined at the root.  Generation is a postfix stack machine driven by splitmix64 seeded with
``seed_base + tape_id`` and the frozen op mix in ``synth_spec.json``; each tape is independent,
so any shard of the tape set can be regenerated anywhere.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

from .tape import Op, TapeSet

SPEC_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "synth_spec.json")
M64 = (1 << 64) - 1


def load_spec(path: str = SPEC_PATH) -> Dict:
    with open(path) as f:
        return json.load(f)


class SplitMix64:
    def __init__(self, seed: int):
        self.s = seed & M64

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)

    def below(self, n: int) -> int:
        return self.next() % n

    def unit(self) -> float:
        return (self.next() >> 11) / float(1 << 53)

    def word(self) -> int:
        return self.next() | self.next() << 64 | self.next() << 128 | self.next() << 192


def _weighted(rng: SplitMix64, items: List[tuple]) -> str:
    total = sum(w for _, w in items)
    x = rng.below(total)
    for name, w in items:
        if x < w:
            return name
        x -= w
    return items[-1][0]


def gen_tape(ts: TapeSet, tape_id: int, spec: Optional[Dict] = None, keccak: bool = False) -> int:
    """One config-5 tape.  keccak=True is SURVEY §8d's keccak variant: the same program plus one
    keccak256 of a 512-bit (word . word) input, the mapping-slot shape of
    keccak_function_manager.py, compared against a pool constant and conjoined at the root."""
    spec = spec or load_spec()
    rng = SplitMix64(spec["seed_base"] + tape_id)
    b = ts.builder()
    var_nodes = [b.var(v, 256) for v in spec["vars"]]
    pool = [int(c, 16) for c in spec["const_pool"]]
    pool += [rng.word() for _ in range(spec["random_words_per_tape"])]
    mix = sorted(spec["mix"].items())
    n_ops = spec["ops_min"] + rng.below(spec["ops_max"] - spec["ops_min"] + 1)

    def leaf() -> int:
        if rng.unit() < spec["leaf_var_prob"]:
            return var_nodes[rng.below(len(var_nodes))]
        return b.const(pool[rng.below(len(pool))], 256)

    stack: List[int] = []
    bools: List[int] = []
    done = 0

    def pop() -> int:
        return stack.pop() if stack else leaf()

    def compare(x: int, y: int) -> int:
        op = [Op.BVULT, Op.BVULE, Op.BVUGT, Op.BVUGE, Op.BVSLT, Op.BVSLE, Op.BVSGT, Op.BVSGE,
              Op.EQ][rng.below(9)]
        return b.op(op, x, y)

    while done < n_ops:
        cls = _weighted(rng, mix)
        if cls == "add_sub":
            y, x = pop(), pop()
            stack.append(b.op(Op.BVADD if rng.below(2) == 0 else Op.BVSUB, x, y))
            done += 1
        elif cls == "mul":
            y, x = pop(), pop()
            stack.append(b.op(Op.BVMUL, x, y))
            done += 1
        elif cls == "logic":
            k = rng.below(4)
            if k == 3:
                stack.append(b.op(Op.BVNOT, pop()))
            else:
                y, x = pop(), pop()
                stack.append(b.op([Op.BVAND, Op.BVOR, Op.BVXOR][k], x, y))
            done += 1
        elif cls == "shift":
            op = [Op.BVSHL, Op.BVLSHR, Op.BVASHR][rng.below(3)]
            if rng.unit() < spec["shift_const_prob"]:
                amt = b.const(rng.below(260), 256)
            else:
                amt = pop()
            stack.append(b.op(op, pop(), amt))
            done += 1
        elif cls == "compare":
            y, x = pop(), pop()
            bools.append(compare(x, y))
            done += 1
        elif cls == "ite":
            if bools:
                c = bools.pop()
            else:
                c = compare(leaf(), leaf())
                done += 1
            e, t = pop(), pop()
            stack.append(b.op(Op.ITE, c, t, e))
            done += 1
        elif cls == "extract_concat_zext":
            if rng.below(2) == 0:
                k = [8, 32, 128, 160][rng.below(4)]
                lo = 8 * rng.below((256 - k) // 8 + 1)
                ex = b.op(Op.EXTRACT, pop(), imm0=lo + k - 1, imm1=lo)
                stack.append(b.op(Op.ZEXT, ex, imm0=256 - k))
                done += 2
            else:
                y, x = pop(), pop()
                lo_half = b.op(Op.EXTRACT, x, imm0=127, imm1=0)
                hi_half = b.op(Op.EXTRACT, y, imm0=255, imm1=128)
                stack.append(b.op(Op.CONCAT, lo_half, hi_half))
                done += 3
        else:  # div
            op = [Op.BVUDIV, Op.BVUREM, Op.BVSDIV, Op.BVSREM][rng.below(4)]
            y, x = pop(), pop()
            stack.append(b.op(op, x, y))
            done += 1
    if keccak:  # drawn after the main program, so the plain variant's tapes are unchanged
        key = pop()
        slot = var_nodes[rng.below(len(var_nodes))]
        h = b.op(Op.KECCAK, b.op(Op.CONCAT, key, slot))
        bools.append(compare(h, leaf()))
    # every remaining value feeds a comparison so the whole program is live
    while stack:
        bools.append(compare(stack.pop(), leaf()))
    if not bools:
        bools.append(compare(leaf(), leaf()))
    root = bools[0]
    for x in bools[1:]:
        root = b.op(Op.AND, root, x)
    return ts.add(b.finish(root))


def generate(n_tapes: Optional[int] = None, first: int = 0, spec: Optional[Dict] = None,
             keccak: bool = False) -> TapeSet:
    spec = spec or load_spec()
    n = spec["n_tapes"] if n_tapes is None else n_tapes
    ts = TapeSet(spec["vars"])
    for t in range(first, first + n):
        gen_tape(ts, t, spec, keccak=keccak)
    return ts
