"""The reference's own SAT/UNSAT outcome tests for the solver layer, restated over the
mythril_amd.smt term API (test helpers; data, not copied source).

Each case names the reference test it restates and the outcome that test asserts:

* tests/laser/keccak_tests.py:7-138 — keccak UF equalities through the keccak function
  manager (restated exactly as tests/laser_like.KeccakManager, keccak_function_manager.py:24-149),
  in two variants: a fresh manager per case (``CASES``), and one manager shared by all the
  module's cases in file order (``shared_keccak_cases``), as the reference's module-level
  manager is -- its remembered concrete hashes then enter later cases' Or-chains.  Where the
  restated query is satisfiable against the test's asserted "unsat" (the reference's code and
  its assertion diverge), ``DIVERGENT`` names the case and the witness that shows it;
* tests/laser/state/calldata_test.py:14-91 — concrete and symbolic calldata (calldata.py);
* tests/laser/state/storage_test.py:11-58 — concrete (K) and symbolic storage (account.py:18-82);
* tests/laser/smt/independece_solver_test.py:42-145 — the DependenceMap partition and the
  IndependenceSolver's outcomes;
* tests/laser/smt/model_test.py:1-56 — decls / __getitem__ / eval(...).as_long() of a model.

An assertion on a *simplified value* (``calldata[100] == 0`` is True after z3's simplify) is
restated as two ground queries: ``value == want`` must be SAT and ``value != want`` UNSAT.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple

from mythril_amd import smt
from mythril_amd.smt import And, Array, BitVec, Concat, If, K, symbol_factory
from tests.laser_like import Calldata as SymbolicCalldata
from tests.laser_like import KeccakManager

BVV = symbol_factory.BitVecVal
BVS = symbol_factory.BitVecSym


class ConcreteCalldata:
    """calldata.py:118-166: a K(256, 8, 0) array with one store per concrete byte."""

    def __init__(self, tx_id, calldata: List[int]):
        self.tx_id = tx_id
        self._concrete = list(calldata)
        self._calldata = K(256, 8, 0)
        for i, element in enumerate(calldata):
            self._calldata[BVV(i, 256)] = BVV(element, 8)

    def __getitem__(self, item) -> BitVec:
        item = BVV(item, 256) if isinstance(item, int) else item
        return self._calldata[item]

    def get_word_at(self, offset: int) -> BitVec:
        return Concat([self[offset + k] for k in range(32)])

    @property
    def calldatasize(self) -> BitVec:
        return BVV(len(self._concrete), 256)


class Storage:
    """account.py:18-82 without a dynamic loader: K(256, 256, 0) when concrete, else the free
    array ``Storage{address}``."""

    def __init__(self, concrete: bool = False, address=None):
        self._standard = K(256, 256, 0) if concrete else Array("Storage%s" % (address,), 256, 256)

    def __getitem__(self, item: BitVec) -> BitVec:
        return self._standard[item]

    def __setitem__(self, key: BitVec, value) -> None:
        self._standard[key] = value


@dataclass
class Case:
    name: str
    ref: str                      # reference test (file:line)
    build: Callable[[], Tuple[smt.Context, list]]
    expected: str                 # "sat" | "unsat" (the reference's assertion)
    # a SAT case the sieve does not answer: why (the test asserts the fallback is asked)
    fallback_reason: Optional[str] = None


def _fresh():
    ctx = smt.Context()
    smt.set_context(ctx)
    return ctx


# -- keccak_tests.py --------------------------------------------------------------------------

def _keccak_basic(mk1, mk2):
    def build(km=None):
        ctx = _fresh()
        km = km or KeccakManager()
        o1, c1 = km.create(mk1())
        o2, c2 = km.create(mk2())
        return ctx, [And(c1, c2), o1 == o2]
    return build


def _keccak_symbol_and_val(km=None):
    ctx = _fresh()
    km = km or KeccakManager()
    n = BVS("n", 256)
    o1, c1 = km.create(BVV(100, 256))
    o2, c2 = km.create(n)
    return ctx, [And(c1, c2), o1 == o2, n == BVV(10, 256)]


def _keccak_complex(distinct: bool):
    def build(km=None):
        ctx = _fresh()
        km = km or KeccakManager()
        a, b = BVS("a", 160), BVS("b", 160)
        o1, c1 = km.create(a)
        o2, c2 = km.create(b)
        cs = [And(c1, c2)]
        two = BVV(2, 256)
        o1, c1 = km.create(two * o1)
        o2, c2 = km.create(two * o2)
        cs += [And(c1, c2), o1 == o2]
        if distinct:
            cs.append(a != b)
        return ctx, cs
    return build


def _keccak_simple_number(km=None):
    ctx = _fresh()
    km = km or KeccakManager()
    o, c = km.create(BVS("a", 160))
    return ctx, [c, BVV(10, 256) == o]


def _keccak_other_num(km=None):
    ctx = _fresh()
    km = km or KeccakManager()
    a, b = BVS("a", 160), BVS("b", 256)
    o, c = km.create(a)
    cs = [c]
    o, c = km.create(BVV(2, 256) * o)
    cs += [c, b == o]
    return ctx, cs


KECCAK_BASIC = [
    ("val8_100_val8_101", lambda: BVV(100, 8), lambda: BVV(101, 8), "unsat"),
    ("val8_100_val16_100", lambda: BVV(100, 8), lambda: BVV(100, 16), "unsat"),
    ("val8_100_val8_100", lambda: BVV(100, 8), lambda: BVV(100, 8), "sat"),
    ("sym_N1_sym_N2", lambda: BVS("N1", 256), lambda: BVS("N2", 256), "sat"),
    ("val256_100_sym_N1", lambda: BVV(100, 256), lambda: BVS("N1", 256), "sat"),
    ("val8_100_sym_N1", lambda: BVV(100, 8), lambda: BVS("N1", 256), "unsat"),
]


# -- calldata_test.py -------------------------------------------------------------------------

def _ground_eq(make, want: int, negate: bool):
    def build():
        ctx = _fresh()
        v = make()
        c = v == BVV(want, v.size())
        return ctx, [smt.Not(c) if negate else c]
    return build


def _concrete_cd_uninit(data, which):
    def make():
        cd = ConcreteCalldata(0, data)
        return cd[100] if which == "byte" else cd.get_word_at(200)
    return make


def _concrete_cd_constrain_index():
    ctx = _fresh()
    cd = ConcreteCalldata(0, [1, 4, 7, 3, 7, 2, 9])
    return ctx, [cd[2] == BVV(3, 8)]


def _symbolic_cd_constrain_index():
    ctx = _fresh()
    cd = SymbolicCalldata("0")
    value = cd.load(51)
    return ctx, [value == BVV(1, 8), cd.size == BVV(50, 256)]


def _symbolic_cd_equal_indices():
    ctx = _fresh()
    cd = SymbolicCalldata("0")
    ia, ib = BVS("index_a", 256), BVS("index_b", 256)
    a, b = cd.load(ia), cd.load(ib)
    return ctx, [ia == ib, a != b]


# -- storage_test.py --------------------------------------------------------------------------

STORAGE_DATA = [({}, 1), ({1: 5}, 2), ({1: 5, 3: 10}, 2)]


def _concrete_storage_uninit(init, key):
    def make():
        st = Storage(concrete=True)
        for k, v in init.items():
            st[BVV(k, 256)] = BVV(v, 256)
        return st[BVV(key, 256)]
    return make


def _storage_set(values):
    def make():
        st = Storage()
        for v in values:
            st[BVV(1, 256)] = BVV(v, 256)
        return st[BVV(1, 256)]
    return make


# -- independece_solver_test.py ---------------------------------------------------------------

def _xyzab():
    return [BVS(n, 256) for n in ("x", "y", "z", "a", "b")]


def _indep(kind):
    def build():
        ctx = _fresh()
        x, y, z, a, b = _xyzab()
        cs = {"unsat": [x > y, y == z, y != z, a == b],
              "unsat_second": [x > y, y == z, a == b, a != b],
              "sat": [x > y, y == z, a == b]}[kind]
        return ctx, cs
    return build


# -- model_test.py ----------------------------------------------------------------------------

def _model_x_eq_2():
    ctx = _fresh()
    x = BVS("x", 256)
    return ctx, [x == BVV(2, 256)]


KT = "tests/laser/keccak_tests.py"
CT = "tests/laser/state/calldata_test.py"
ST = "tests/laser/state/storage_test.py"
IT = "tests/laser/smt/independece_solver_test.py"

CASES: List[Case] = []
for _n, _m1, _m2, _e in KECCAK_BASIC:
    CASES.append(Case("keccak_basic_" + _n, KT + ":7-38", _keccak_basic(_m1, _m2), _e))
CASES += [
    Case("keccak_symbol_and_val", KT + ":41-54", _keccak_symbol_and_val, "unsat"),
    Case("keccak_complex_eq", KT + ":57-78", _keccak_complex(True), "unsat"),
    Case("keccak_complex_eq2", KT + ":81-103", _keccak_complex(False), "sat"),
    Case("keccak_simple_number", KT + ":106-119", _keccak_simple_number, "unsat"),
    Case("keccak_other_num", KT + ":122-138", _keccak_other_num, "sat"),
]
for _i, _data in enumerate(([], [1, 4, 5, 3, 4, 72, 230, 53])):
    for _which in ("byte", "word"):
        for _neg in (False, True):
            CASES.append(Case("calldata_uninit_%d_%s_%s" % (_i, _which, "ne" if _neg else "eq"),
                              CT + ":14-25", _ground_eq(_concrete_cd_uninit(_data, _which), 0,
                                                        _neg),
                              "unsat" if _neg else "sat"))
CASES += [
    Case("calldata_constrain_index", CT + ":42-55", _concrete_cd_constrain_index, "unsat"),
    Case("symbolic_calldata_constrain_index", CT + ":58-73", _symbolic_cd_constrain_index,
         "unsat"),
    Case("symbolic_calldata_equal_indices", CT + ":76-91", _symbolic_cd_equal_indices, "unsat"),
]
for _i, (_init, _key) in enumerate(STORAGE_DATA):
    for _neg in (False, True):
        CASES.append(Case("storage_uninit_%d_%s" % (_i, "ne" if _neg else "eq"), ST + ":11-22",
                          _ground_eq(_concrete_storage_uninit(_init, _key), 0, _neg),
                          "unsat" if _neg else "sat"))
for _name, _vals, _want, _ref in (("storage_set_item", (13,), 13, ":39-47"),
                                  ("storage_change_item", (12, 14), 14, ":50-58")):
    for _neg in (False, True):
        CASES.append(Case("%s_%s" % (_name, "ne" if _neg else "eq"), ST + _ref,
                          _ground_eq(_storage_set(_vals), _want, _neg),
                          "unsat" if _neg else "sat"))
CASES += [
    Case("independence_unsat", IT + ":88-105", _indep("unsat"), "unsat"),
    Case("independence_unsat_second_bucket", IT + ":108-125", _indep("unsat_second"), "unsat"),
    Case("independence_sat", IT + ":128-145", _indep("sat"), "sat"),
    Case("model_x_eq_2", "tests/laser/smt/model_test.py:5-56", _model_x_eq_2, "sat"),
]

BY_NAME = {c.name: c for c in CASES}


def case_ids():
    return [c.name for c in CASES]


KECCAK_MODULE = [c.name for c in CASES if c.ref.startswith(KT)]  # keccak_tests.py, file order


def _k(value: int, nbytes: int) -> int:
    from oracle.keccak import keccak256

    return int.from_bytes(keccak256(value.to_bytes(nbytes, "big")), "big")


# Cases whose restated query -- the reference's own construction, exactly -- is satisfiable
# although the reference test asserts "unsat": the reference's code and its assertion diverge.
# Each entry: why, and a model (vars, functions) the ORACLE checks against the query
# (tests/test_reference_fixtures.py::test_divergent_cases_are_satisfiable).  The sieve answers
# neither with a witness (its keccak lowering gives keccak256_256 its own interval values, so it
# cannot make keccak256_256(100) equal an 8-bit input's hash); the query reaches the fallback,
# where z3 decides it.
DIVERGENT = {
    "keccak_basic_val8_100_sym_N1": (
        "keccak_function_manager.py:145-148 ORs every remembered concrete pair into N1's "
        "condition, and `key == func_input` zero-pads the 8-bit key 100 (bitvec.py:16-22): "
        "N1 = 100 with keccak256_256(100) = keccak(0x64) satisfies o1 == o2",
        {"N1": 100},
        {"keccak256_8": {100: _k(100, 1)}, "keccak256_8-1": {_k(100, 1): 100},
         "keccak256_256": {100: _k(100, 1)}, "keccak256_256-1": {_k(100, 1): 100}}),
}


def shared_keccak_cases():
    """keccak_tests.py's cases in file order over ONE manager (the reference's module-level
    ``keccak_function_manager``): [(case, ctx, constraints)], each case in a fresh context."""
    km = KeccakManager()
    out = []
    for name in KECCAK_MODULE:
        case = BY_NAME[name]
        ctx, cs = case.build(km)
        out.append((case, ctx, cs))
    return out


def dependence_map_case():
    """independece_solver_test.py:54-85: conditions [x > y, y == z, a == b] give two buckets,
    ({x, y, z}: conditions 0 and 1) and ({a, b}: condition 2)."""
    ctx = _fresh()
    x, y, z, a, b = _xyzab()
    return ctx, [x > y, y == z, a == b], ({"x", "y", "z"}, {"a", "b"}), ([0, 1], [2])


def expr_variables_case():
    """independece_solver_test.py:12-39: If(x, y, z + b) reads x, y, z, b; b + 2 reads b."""
    ctx = _fresh()
    x = symbol_factory.BoolSym("x")
    y, z, b = BVS("y", 256), BVS("z", 256), BVS("b", 256)
    return ctx, [(If(x, y, z + b), {"x", "y", "z", "b"}), (b + BVV(2, 256), {"b"})]
