"""The division algorithm of the asm core (gen_asm_core.py Core.div_body), modelled step for step
in Python (IEEE doubles, u32 limbs) and checked against exact integer division.  It pins the
algorithm -- f64 digit estimates over 32-bit digits without normalisation, one add-back and one
subtract per digit, start digit from the f64 quotient with a factor-2 margin -- independently of
the GPU; tests/test_gpu_parity.py checks the assembly itself against the oracle."""
import math
import random

M32 = (1 << 32) - 1


def _limbs(v):
    return [(v >> (32 * k)) & M32 for k in range(8)]


def _val(l):
    return sum(x << (32 * k) for k, x in enumerate(l))


def _to_f64(l):  # Horner with fma, as the asm (v_cvt_f64_u32 + v_fma_f64)
    d = float(l[7])
    for k in range(6, -1, -1):
        d = math.fma(d, 4294967296.0, float(l[k])) if hasattr(math, "fma") else d * 4294967296.0 + l[k]
    return d


def _cvt_u32(d):  # v_min_f64 clamp + v_cvt_u32_f64
    d = min(d, 4294967295.0)
    return 0 if d != d or d <= 0 else int(d)


def model_udivrem(x, y):
    R, Y, Q = _limbs(x), _limbs(y), [0] * 8
    if y == 0:
        return (1 << 256) - 1, x
    if x < y:
        return 0, x
    fy = 1.0 / _to_f64(Y)
    qd = _to_f64(R) * fy
    start = next((j for j in range(7, 0, -1) if 2.0 ** (32 * j - 1) <= qd), 0)
    for j in range(start, -1, -1):
        c = _cvt_u32(_to_f64(R) * fy * 2.0 ** (-32 * j))
        carry = borrow = 0
        for k in range(8):  # R[j..] -= c * y (limbs above 7 only feed the borrow)
            t = c * Y[k] + carry
            lo, carry = t & M32, t >> 32
            d = (R[j + k] if j + k <= 7 else 0) - lo - borrow
            if j + k <= 7:
                R[j + k] = d & M32
            borrow = int(d < 0)
        if 0 - carry - borrow < 0:  # negative: add y << 32j back
            cy = 0
            for k in range(8 - j):
                s = R[j + k] + Y[k] + cy
                R[j + k], cy = s & M32, s >> 32
            c -= 1
        br = 0
        for k in range(8):
            d = (R[j + k] if k < 8 - j else 0) - Y[k] - br
            br = int(d < 0)
        if not br:  # R >= y << 32j: subtract once more
            br = 0
            for k in range(8 - j):
                d = R[j + k] - Y[k] - br
                R[j + k], br = d & M32, int(d < 0)
            c += 1
        assert 0 <= c <= M32
        Q[j] = c
    return _val(Q), _val(R)


def test_division_model_matches_exact_division():
    rng = random.Random(7)
    cases = [((1 << 256) - 1, 2), ((1 << 256) - 2, 2), ((1 << 256) - 1, 1), (1 << 255, 3),
             ((1 << 256) - 1, (1 << 256) - 1), (12345, 0), (0, 5)]
    for _ in range(4000):
        x = rng.getrandbits(rng.choice([8, 64, 128, 255, 256]))
        y = rng.getrandbits(rng.choice([1, 8, 31, 32, 33, 64, 96, 128, 200, 256]))
        cases.append((x, y))
        cases.append((x, (1 << rng.randrange(256)) + rng.getrandbits(8)))
    for x, y in cases:
        want = ((1 << 256) - 1, x) if y == 0 else (x // y, x % y)
        assert model_udivrem(x, y) == want, (hex(x), hex(y))
