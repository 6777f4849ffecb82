"""ORACLE (test infrastructure only — never imported by the product path).

Restatement of the guided candidate generator ``mh_assign_generate_guided``
(include/mythril_hip.h, mythril_amd/csrc/generate.hip ``guided_kernel`` / ``guided_lds_kernel``), bit for bit:

    g = global_base + row
    per column v (width w, pool P_v):
        m0, m1 = gen_limb(seed ^ SALT_MODE, v, g, 0), gen_limb(seed ^ SALT_MODE, v, g, 1)
        mode = m0 & 0xff
        mode <  64                 -> (m0 >> 8) & 0xff                       ("small")
        mode < 128 or P_v is empty -> limbs gen_limb(seed, v, g, k), k = 0..7 ("uniform")
        otherwise                  -> P_v[m1 % |P_v|]                        ("pool")
        masked to w bits
    per set j, in order:
        s = gen_limb(seed ^ SALT_SET, j, g, 0)
        if (s & 0xff) < prob_j and set j has alternatives:
            apply alternative set_off[j] + (s >> 8) % n_alt_j: every (column, value) entry,
            value masked to the column's width (later sets override earlier ones); an entry
            whose column has bit 31 set is a copy: limbs [src, dst_lo, src_lo, nbits] put bits
            [src_lo, src_lo + nbits) of column src (its value at that point) into bits
            [dst_lo, dst_lo + nbits) of the destination column

gen_limb is the plain generator's counter-based splitmix64 (oracle/smt_eval.py gen_limb).
"""
from __future__ import annotations

from typing import Dict, List

try:
    from .smt_eval import gen_limb
except ImportError:  # pragma: no cover
    from smt_eval import gen_limb  # type: ignore

SALT_MODE = 0x6A09E667F3BCC909
SALT_SET = 0xBB67AE8584CAA73B
COPY_FLAG = 0x80000000


def _limbs_to_int(row) -> int:
    return sum(int(x) << (32 * k) for k, x in enumerate(row))


def generate_row(seed: int, g: int, arrays: Dict) -> List[int]:
    """Column values of global row index g for a guide given as mh_guide arrays."""
    width = [int(x) for x in arrays["width"]]
    pool_off = arrays["pool_off"]
    pool = arrays["pool"]
    out = []
    for v, w in enumerate(width):
        m0 = gen_limb(seed ^ SALT_MODE, v, g, 0)
        m1 = gen_limb(seed ^ SALT_MODE, v, g, 1)
        mode = m0 & 0xFF
        lo, hi = int(pool_off[v]), int(pool_off[v + 1])
        if mode < 64:
            val = (m0 >> 8) & 0xFF
        elif mode < 128 or hi == lo:
            val = sum(gen_limb(seed, v, g, k) << (32 * k) for k in range(8))
        else:
            val = _limbs_to_int(pool[lo + m1 % (hi - lo)])
        out.append(val & ((1 << w) - 1))
    set_off, prob = arrays["set_off"], arrays["set_prob"]
    alt_off, e_col, e_val = arrays["alt_off"], arrays["entry_col"], arrays["entry_val"]
    for j in range(len(set_off) - 1):
        s = gen_limb(seed ^ SALT_SET, j, g, 0)
        n_alt = int(set_off[j + 1]) - int(set_off[j])
        if (s & 0xFF) < int(prob[j]) and n_alt:
            alt = int(set_off[j]) + (s >> 8) % n_alt
            for e in range(int(alt_off[alt]), int(alt_off[alt + 1])):
                col = int(e_col[e])
                if col & COPY_FLAG:  # bits [src_lo, src_lo+n) of src into [dst_lo, ...) of dst
                    dst = col & ~COPY_FLAG
                    src, dlo, slo, nb = (int(x) for x in e_val[e][:4])
                    m = ((1 << nb) - 1) << dlo
                    bits = ((out[src] >> slo) << dlo) & m
                    out[dst] = ((out[dst] & ~m) | bits) & ((1 << width[dst]) - 1)
                else:
                    out[col] = _limbs_to_int(e_val[e]) & ((1 << width[col]) - 1)
    return out
