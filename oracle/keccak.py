"""ORACLE (test infrastructure only — never imported by the product path).

Keccak-256 restated in plain Python: the hash the reference computes for concrete inputs through
pyethereum ``utils.sha3`` (mythril/laser/ethereum/keccak_function_manager.py:43-57,
find_concrete_keccak; also ``_pysha3`` in mythril/support/support_utils.py:36).  Neither
dependency is installed here (pyethereum ``ethereum>=2.3.2``, ``pysha3``; no lock
file pins them).  The published algorithm restated: Keccak-f[1600] (24 rounds of theta, rho, pi,
chi, iota on 25 64-bit lanes), sponge with rate 1088 bits (136 bytes), original Keccak padding
0x01 ... 0x80, 32-byte output.

Pinned by: hashlib.sha3_256 (same permutation and rate, pad byte 0x06 instead of 0x01) on
arbitrary inputs, and the reference's own known answers (VMTests vmSha3Test post-storage,
keccak("") at keccak_function_manager.py:80, the 4-byte selectors of tests/cmd_line_test.py and
README.md) — see tests/test_oracle_keccak.py.
"""
from __future__ import annotations

MASK64 = (1 << 64) - 1

ROUND_CONSTANTS = [
    0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
    0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
    0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
    0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
    0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
    0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008,
]

# rotation offsets r[x][y]
ROTATIONS = [
    [0, 36, 3, 41, 18],
    [1, 44, 10, 45, 2],
    [62, 6, 43, 15, 61],
    [28, 55, 25, 21, 56],
    [27, 20, 39, 8, 14],
]

RATE = 136


def _rol(x: int, n: int) -> int:
    n %= 64
    return ((x << n) | (x >> (64 - n))) & MASK64 if n else x


def keccak_f1600(state):
    """state: list of 25 ints, lane (x, y) at index x + 5*y.  Returns the permuted list."""
    a = list(state)
    for rc in ROUND_CONSTANTS:
        # theta
        c = [a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20] for x in range(5)]
        d = [c[(x - 1) % 5] ^ _rol(c[(x + 1) % 5], 1) for x in range(5)]
        a = [a[i] ^ d[i % 5] for i in range(25)]
        # rho + pi: B[y, 2x+3y] = rot(A[x, y], r[x, y])
        b = [0] * 25
        for x in range(5):
            for y in range(5):
                b[y + 5 * ((2 * x + 3 * y) % 5)] = _rol(a[x + 5 * y], ROTATIONS[x][y])
        # chi
        a = [b[i] ^ ((~b[(i % 5 + 1) % 5 + 5 * (i // 5)]) & b[(i % 5 + 2) % 5 + 5 * (i // 5)])
             for i in range(25)]
        a = [v & MASK64 for v in a]
        # iota
        a[0] ^= rc
    return a


def _sponge(data: bytes, pad: int, out_len: int = 32) -> bytes:
    msg = bytearray(data)
    msg.append(pad)
    while len(msg) % RATE:
        msg.append(0)
    msg[-1] |= 0x80
    state = [0] * 25
    for off in range(0, len(msg), RATE):
        block = msg[off:off + RATE]
        for i in range(RATE // 8):
            state[i] ^= int.from_bytes(block[8 * i:8 * i + 8], "little")
        state = keccak_f1600(state)
    out = b"".join(state[i].to_bytes(8, "little") for i in range(RATE // 8))
    return out[:out_len]


def keccak256(data: bytes) -> bytes:
    """Keccak-256 (Ethereum's sha3), pad byte 0x01."""
    return _sponge(bytes(data), 0x01)


def sha3_256_fips(data: bytes) -> bytes:
    """FIPS-202 SHA3-256 (pad byte 0x06) — only used to pin the permutation against hashlib."""
    return _sponge(bytes(data), 0x06)


def keccak256_int(value: int, nbytes: int) -> int:
    """find_concrete_keccak: keccak of value.to_bytes(size // 8, 'big') as a 256-bit int."""
    return int.from_bytes(keccak256(value.to_bytes(nbytes, "big")), "big")
