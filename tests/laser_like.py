"""Builders of LASER-shaped path conditions with the mythril_amd.smt term API (test helpers).

Each builder follows the reference construction it names, so the queries the tests hand to the
lowering / sieve have the shapes ``myth analyze`` produces:

* calldata reads: ``If(i < calldatasize, calldata[i], 0)`` per byte, words as ``Concat`` of 32
  bytes (mythril/laser/ethereum/state/calldata.py:48-54, 219-232; ``<`` is signed, bitvec.py);
* the function-selector check of a Solidity dispatcher (JUMPI on
  ``Extract(255, 224, calldataload(0)) == selector``, instructions.py:1543-1619);
* ``sender in ACTORS`` (transaction/symbolic.py:22-67, 87-104);
* ``UGE(balance[sender], value)`` (transaction_models.py:129-133, world_state.py:33-34);
* storage reads of a free ``Storage`` array (account.py:18-82);
* keccak UF applications with the manager's interval / mod-64 / inverse / concrete-pair
  conditions (keccak_function_manager.py:83-149) — concrete hashes from the oracle's Keccak-256;
* the integer-overflow module's ``BVAddNoOverflow``/``BVMulNoOverflow`` (integer.py:141-157);
* the EtherThief and Suicide modules' queries (ether_thief.py:65-73, suicide.py:68-81) over the
  world state LASER builds: per message call the ACTORS constraint and the call value's transfer
  (transaction/symbolic.py:165-167, transaction_models.py:121-133), a CALL's transfer_ether
  (instructions.py:71-92).
"""
from __future__ import annotations

from mythril_amd import smt
from mythril_amd.smt import (And, Array, BitVec, Concat, Extract, Function, If, K, Not, Or, ULE,
                             ULT, UGE, UGT, URem, symbol_factory)
from oracle.keccak import keccak256

CREATOR = 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE
ATTACKER = 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF
SOMEGUY = 0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA

TOTAL_PARTS = 10 ** 40
PART = (2 ** 256 - 1) // TOTAL_PARTS
INTERVAL_DIFFERENCE = 10 ** 30


class Calldata:
    """SymbolicCalldata (calldata.py:207-255)."""

    def __init__(self, tx_id: str):
        self.size = symbol_factory.BitVecSym("%s_calldatasize" % tx_id, 256)
        self.data = Array("%s_calldata" % tx_id, 256, 8)

    def load(self, i) -> BitVec:
        item = symbol_factory.BitVecVal(i, 256) if isinstance(i, int) else i
        return If(item < self.size, self.data[item], symbol_factory.BitVecVal(0, 8))

    def word(self, offset: int) -> BitVec:
        return Concat([self.load(offset + k) for k in range(32)])


def selector_is(cd: Calldata, selector: int) -> smt.Bool:
    return Extract(255, 224, cd.word(0)) == symbol_factory.BitVecVal(selector, 32)


def sender_is_actor(sender: BitVec) -> smt.Bool:
    return Or(*[sender == symbol_factory.BitVecVal(a, 256) for a in (CREATOR, ATTACKER, SOMEGUY)])


class KeccakManager:
    """keccak_function_manager.py:24-149 restated over the test term API, exactly: a concrete
    input's hash is remembered (``concrete_hashes``, keyed by value and width as the reference's
    dict of BitVecVals is) and every later symbolic input's condition ORs over ALL remembered
    pairs, whatever their width -- ``key == func_input`` zero-pads the narrower side
    (bitvec.py:16-22), so an 8-bit key 100 admits a 256-bit input 100 (:145-148).  The state is
    plain integers, so one manager can serve several term contexts in turn, as the reference's
    module-level manager serves every test of a pytest session."""

    def __init__(self):
        self.store = {}
        self.hooks = {}
        self.counter = TOTAL_PARTS - 34534
        self.concrete = {}  # (value, width) -> hash, in insertion order (:40, :95)

    def functions(self, length: int):
        # terms of the CURRENT context (a shared manager outlives the contexts of its cases)
        ctx = smt.context()
        got = self.store.get(length)
        if got is None or got[0] is not ctx:
            got = self.store[length] = (ctx, Function("keccak256_%d" % length, length, 256),
                                        Function("keccak256_%d-1" % length, 256, length))
        return got[1], got[2]

    def create(self, data: BitVec):
        length = data.size()
        f, inv = self.functions(length)
        if data.value is not None:  # :92-97
            h = int.from_bytes(keccak256(data.value.to_bytes(length // 8, "big")), "big")
            hv = symbol_factory.BitVecVal(h, 256)
            self.concrete[(data.value, length)] = h
            return hv, And(f(data) == hv, inv(f(data)) == data)
        if length not in self.hooks:  # :128-133
            self.hooks[length] = self.counter
            self.counter -= INTERVAL_DIFFERENCE
        lo = self.hooks[length] * PART
        hi = lo + PART
        cond = And(inv(f(data)) == data,
                   ULE(symbol_factory.BitVecVal(lo, 256), f(data)),
                   ULT(f(data), symbol_factory.BitVecVal(hi, 256)),
                   URem(f(data), symbol_factory.BitVecVal(64, 256)) == 0)
        conc = symbol_factory.Bool(False)
        for (value, width), h in self.concrete.items():  # :145-148, every width
            key = symbol_factory.BitVecVal(value, width)
            conc = Or(conc, And(f(data) == symbol_factory.BitVecVal(h, 256), key == data))
        return f(data), And(inv(f(data)) == data, Or(cond, conc))


def mapping_slot(km: KeccakManager, key: BitVec, slot: int):
    """keccak256(key . slot): the storage slot of mapping[key] (Solidity layout)."""
    return km.create(Concat(key, symbol_factory.BitVecVal(slot, 256)))


def killbilly():
    """The path condition at ``selfdestruct`` in the 3-transaction KillBilly sequence of
    README.md:54-76 (killerize(addr); activatekillability(); commencekilling()): three
    calldata arrays and dispatcher checks, senders in ACTORS, non-payable functions, and the
    created contract's storage (K(0), account.py:26-29) carrying
    approved_killers[addr] = 1 (mapping slot keccak(addr . 1)) from tx 1 to tx 2 and
    is_killable = 1 (slot 0) from tx 2 to tx 3, with the keccak manager's conditions."""
    km = KeccakManager()
    zero = symbol_factory.BitVecVal(0, 256)
    one = symbol_factory.BitVecVal(1, 256)
    storage = K(256, 256, 0)
    cs = []
    txs = []
    for t, sel in ((1, 0x9FA299CC), (2, 0x84057065), (3, 0x7C11DA20)):
        cd = Calldata(str(t))
        sender = symbol_factory.BitVecSym("sender_%d" % t, 256)
        value = symbol_factory.BitVecSym("call_value%d" % t, 256)
        cs += [sender_is_actor(sender), selector_is(cd, sel), value == zero,
               ULT(cd.size, symbol_factory.BitVecVal(5000, 256))]
        txs.append((cd, sender))
    cd1, _ = txs[0]
    cs.append(UGE(cd1.size, symbol_factory.BitVecVal(36, 256)))
    addr = cd1.word(4) & symbol_factory.BitVecVal((1 << 160) - 1, 256)
    slot_a, cond_a = mapping_slot(km, addr, 1)
    storage[slot_a] = one                                   # tx 1: approved_killers[addr] = 1
    _, sender2 = txs[1]
    slot_s, cond_s = mapping_slot(km, sender2, 1)
    cs += [cond_a, cond_s, storage[slot_s] == one]          # tx 2: require(approved[msg.sender])
    storage[zero] = one                                     # tx 2: is_killable = 1
    _, sender3 = txs[2]
    cs += [Not(storage[zero] == zero),                      # tx 3: require(is_killable)
           sender3 == symbol_factory.BitVecVal(ATTACKER, 256)]
    return cs


CONTRACT = 0x901D12EBE1B195E5AA8748E62BD7734AE19B51F


def message_call(t: int, balances, callee: int = CONTRACT):
    """A symbolic message call's environment and its world-state constraints: the sender is one of
    the ACTORS (transaction/symbolic.py:86-104, 165-167; origin is the same symbol as the caller),
    and the call value moves from the sender to the callee (transaction_models.py:121-133)."""
    sender = symbol_factory.BitVecSym("sender_%d" % t, 256)
    value = symbol_factory.BitVecSym("call_value%d" % t, 256)
    cs = [sender_is_actor(sender), UGE(balances[sender], value)]
    callee_bv = symbol_factory.BitVecVal(callee, 256)
    balances[callee_bv] += value
    balances[sender] -= value
    return sender, sender, value, cs


def transfer_ether(cs, balances, sender, receiver, value):
    """instructions.py:71-92: UGE(balance[sender], value), then the two balance updates."""
    cs.append(UGE(balances[sender], value))
    balances[receiver] += value
    balances[sender] -= value


def ether_thief():
    """EtherThief (analysis/module/modules/ether_thief.py:65-73) at the CALL of a `withdraw(uint256
    amount)` that sends `amount` to msg.sender without an ownership check: the transaction's
    world-state constraints, the dispatcher check, the CALL's transfer, then the module's
    UGT(balances[attacker], starting_balances[attacker]), sender == attacker, caller == origin."""
    balances = Array("balance", 256, 256)
    starting = Array("balance", 256, 256)  # world_state.py:34: a copy taken before any transaction
    cd = Calldata("1")
    caller, origin, value, cs = message_call(1, balances)
    cs += [selector_is(cd, 0x2E1A7D4D), ULT(cd.size, symbol_factory.BitVecVal(5000, 256))]
    amount = cd.word(4)
    transfer_ether(cs, balances, symbol_factory.BitVecVal(CONTRACT, 256), caller, amount)
    attacker = symbol_factory.BitVecVal(ATTACKER, 256)
    cs += [UGT(balances[attacker], starting[attacker]), caller == attacker, caller == origin]
    return cs


def suicide_arg():
    """Suicide (analysis/module/modules/suicide.py:68-81) at the SELFDESTRUCT of a
    `kill(address to)` with no ownership check: per message-call transaction
    And(caller == attacker, caller == origin), and to == attacker, where `to` is the ABI-decoded
    address argument (calldata word 4 masked to 160 bits)."""
    balances = Array("balance", 256, 256)
    cd = Calldata("1")
    caller, origin, value, cs = message_call(1, balances)
    cs += [selector_is(cd, 0xCBF0B0C0), value == symbol_factory.BitVecVal(0, 256),
           UGE(cd.size, symbol_factory.BitVecVal(36, 256))]
    to = cd.word(4) & symbol_factory.BitVecVal((1 << 160) - 1, 256)
    attacker = symbol_factory.BitVecVal(ATTACKER, 256)
    cs += [And(caller == attacker, caller == origin), to == attacker]
    return cs


def suicide_killbilly():
    """The Suicide module's query on KillBilly's 3-transaction sequence (README.md:54-76): the
    path condition at SELFDESTRUCT (killbilly()) plus, per transaction, And(caller == attacker,
    caller == origin), and the beneficiary (msg.sender of the third call) == attacker."""
    cs = killbilly()
    attacker = symbol_factory.BitVecVal(ATTACKER, 256)
    for t in (1, 2, 3):
        s = symbol_factory.BitVecSym("sender_%d" % t, 256)
        cs.append(And(s == attacker, s == s))
    cs.append(symbol_factory.BitVecSym("sender_3", 256) == attacker)
    return cs


def queries():
    """A list of (name, [constraints]) LASER-shaped feasibility queries, most of them SAT."""
    out = []
    ctx = smt.Context()
    smt.set_context(ctx)
    cd = Calldata("1")
    sender = symbol_factory.BitVecSym("sender_1", 256)
    value = symbol_factory.BitVecSym("call_value1", 256)
    balance = Array("balance", 256, 256)
    storage = Array("Storage0x901d12ebe1b195e5aa8748e62bd7734ae19b51f", 256, 256)
    out.append(("selector", [selector_is(cd, 0x9FA299CC), sender_is_actor(sender)]))
    out.append(("selector_size", [selector_is(cd, 0x13AF4035),
                                  UGE(cd.size, symbol_factory.BitVecVal(36, 256)),
                                  ULT(cd.size, symbol_factory.BitVecVal(5000, 256))]))
    out.append(("owner_check", [sender_is_actor(sender), storage[symbol_factory.BitVecVal(0, 256)]
                                == sender, Not(sender == symbol_factory.BitVecVal(CREATOR, 256))]))
    out.append(("balance", [sender_is_actor(sender), UGE(balance[sender], value),
                            Not(value == symbol_factory.BitVecVal(0, 256))]))
    arg = Extract(159, 0, cd.word(4))
    out.append(("address_arg", [selector_is(cd, 0x9FA299CC),
                                arg == Extract(159, 0, sender)]))
    x = cd.word(4)
    y = cd.word(36)
    out.append(("overflow", [selector_is(cd, 0xA9059CBB),
                             Not(smt.BVAddNoOverflow(x, y, False))]))
    out.append(("mul_overflow", [Not(smt.BVMulNoOverflow(x, symbol_factory.BitVecVal(3, 256),
                                                          False))]))
    km = KeccakManager()
    h_c, cond_c = mapping_slot(km, symbol_factory.BitVecVal(CREATOR, 256), 1)
    h_s, cond_s = mapping_slot(km, sender, 1)
    out.append(("keccak_mapping", [cond_c, cond_s, sender_is_actor(sender),
                                   storage[h_s] == symbol_factory.BitVecVal(7, 256)]))
    out.append(("keccak_alias", [cond_c, cond_s, h_s == h_c]))
    st = K(256, 256, 0)
    st[symbol_factory.BitVecVal(0, 256)] = sender
    st[cd.word(4)] = value
    out.append(("k_storage", [st[symbol_factory.BitVecVal(0, 256)] == symbol_factory.BitVecVal(
        ATTACKER, 256), sender_is_actor(sender)]))
    out.append(("killbilly", killbilly()))
    out.append(("ether_thief", ether_thief()))
    out.append(("suicide_arg", suicide_arg()))
    out.append(("suicide_killbilly", suicide_killbilly()))
    out.append(("unsat_actor", [sender_is_actor(sender), sender == symbol_factory.BitVecVal(5,
                                                                                            256)]))
    return ctx, out


def hard_queries():
    """UNSAT variants of the largest SAT shapes: each adds a conjunct that contradicts the path
    condition in a way constant folding cannot see, so the sieve runs every round and misses
    (what an infeasible JUMPI branch costs LASER on top of z3, svm.py:257-262)."""
    ctx, qs = queries()
    d = dict(qs)
    out = []
    # KillBilly: the third transaction's sender is both ATTACKER and CREATOR
    sender3 = symbol_factory.BitVecSym("sender_3", 256)
    out.append(("killbilly_unsat", d["killbilly"] + [sender3 == symbol_factory.BitVecVal(
        CREATOR, 256)]))
    # transfer overflow of two words that are both below 2^128
    cd = Calldata("1")
    lim = symbol_factory.BitVecVal(1 << 128, 256)
    out.append(("overflow_unsat", d["overflow"] + [ULT(cd.word(4), lim), ULT(cd.word(36), lim)]))
    # storage slot 0 holds the sender (or a zero value when the key word is 0) and must be the
    # attacker, while the sender is not and the value is zero
    sender = symbol_factory.BitVecSym("sender_1", 256)
    value = symbol_factory.BitVecSym("call_value1", 256)
    out.append(("k_storage_unsat", d["k_storage"] + [
        Not(sender == symbol_factory.BitVecVal(ATTACKER, 256)),
        value == symbol_factory.BitVecVal(0, 256)]))
    # EtherThief on a withdraw that pays out at most the call's own value: the attacker's
    # balance cannot grow (b - v + amount <= b with amount <= v and no underflow, UGE(b, v))
    cd4 = Calldata("1").word(4)
    out.append(("ether_thief_unsat", d["ether_thief"] + [
        ULE(cd4, symbol_factory.BitVecSym("call_value1", 256))]))
    return ctx, out


def query_tapeset(b, constraints):
    """The tape set the sieve builds for one query (Sieve.solve's steps 1-3): lowered root,
    schema, one tape per variable-disjoint bucket, and the harvested guide."""
    from mythril_amd.candidates import build_guide
    from mythril_amd.lower import lower_query
    from mythril_amd.sieve import Sieve, local_tape
    from mythril_amd.tape import Op, Tape, TapeSet

    root, schema = lower_query(b, [c.node for c in constraints])
    cols = list(schema.columns)
    ts = TapeSet(cols)
    ts.pool = b.pool
    for conj, _ in Sieve.buckets(b, root):
        acc = conj[0]
        for x in conj[1:]:
            acc = b.op(Op.AND, acc, x)
        ts.tapes.append(Tape(local_tape(b, acc, cols)))
    guide = build_guide(b, root, schema, cols, None).arrays()
    return ts, schema, guide

