// One interpreter step of the sieve machine (dev_isa.h), shared by the HIP kernels
// (sieve_kernels.hip: the complex ops) and the test-only host emulator (tests/native/emu.cpp:
// every op).  For the ops the device runs in the assembly core, step() is the reference
// semantics the assembly is tested against (tests/test_gpu_parity.py, via the oracle).
//
// M is the machine: the register file (accumulator X = R[nrx()]) and the read-only environment.
//   u32  nrx();                       index of the accumulator
//   void read(u32 r, u32* v);         R[r], 8 limbs         (device: indexed VGPR moves)
//   u32  read0(u32 r);                limb 0 of R[r]
//   void write(u32 r, const u32* v);  R[r] = v
//   void iconst(u32 slot, u32* v);    the inline constant in slots slot..slot+3 of the tape
//   void var(u32 col, u32* v);        assignment column col of this lane's row
// FEAT (dev_isa.h F_DIV | F_KECCAK | F_EVM) compiles the heavy handlers in or out, so a tape
// set without them runs a kernel with a smaller register budget (higher occupancy).
#pragma once
#include "dev_isa.h"
#include "u256_ops.h"

namespace mh {

// Keccak-256 of a message of nw (1..3) LEFT-aligned 32-byte words W0, W1, W2 (big-endian byte
// order, the host has already cut the message into words and placed the 0x01 pad byte when the
// message ends inside a word; full = the message ends on a word boundary, so the pad starts the
// next word).  One 136-byte block; every state position is static, so no byte gathering.
MH_FN void keccak_absorb_word(u64* st, const u32* W) {
#pragma unroll
    for (int t = 0; t < 4; ++t)
        st[t] = (u64)bswap32(W[7 - 2 * t]) | ((u64)bswap32(W[6 - 2 * t]) << 32);
}

MH_FN void keccak_words(const u32* W0, const u32* W1, const u32* W2, u32 nw, u32 full, u32* z) {
    u64 st[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) st[i] = 0;
    keccak_absorb_word(st, W0);
    if (nw >= 2u) keccak_absorb_word(st + 4, W1);  // wave-uniform
    if (nw >= 3u) keccak_absorb_word(st + 8, W2);
    if (full) {
        if (nw == 1u) st[4] |= 0x01ull;
        else if (nw == 2u) st[8] |= 0x01ull;
        else st[12] |= 0x01ull;
    }
    st[16] |= 0x8000000000000000ull;  // byte 135 of the 136-byte block
    keccak_f1600(st);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int i = 7 - k;  // u32 word i of the output bytes
        const u32 wv = (i & 1) ? (u32)(st[i >> 1] >> 32) : (u32)st[i >> 1];
        z[k] = bswap32(wv);
    }
}

MH_FN void zero8(u32* z) {
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = 0;
}

MH_FN void copy8(u32* z, const u32* x) {
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = x[k];
}

// z = f(x, y, c3) for a complex op (op >= D_FIRST_COMPLEX): x = R[a'], y = R[b] or the inline
// constant, c3 = R[c] (KECCAK's third piece, ADDMOD / MULMOD's modulus).  Width-w semantics on canonical operands.  E
// provides var(col, v) for D_LOADVAR.  Shared by the device's C++ path and step().
template <int FEAT, class E>
MH_FN void complex_op(const E& env, u32 w1, const u32* x, const u32* y, const u32* c3, u32* z) {
    const u32 op = w1 & 0xFFu, w = (w1 >> 8) & 0x1FFu, aux = (w1 >> 17) & MH_AUX_MAX;
    copy8(z, x);
    switch (op) {
        case D_UADD_NOOVFL: {
            u32 t[8];
            const u32 cy = add256(x, y, t);
            u32 hi = 0;
            if (w < 256) {
#pragma unroll
                for (int k = 0; k < 8; ++k) hi |= t[k] & ~width_mask(k, w);
            }
            z[0] = !(cy || hi);
            break;
        }
        case D_UMUL_NOOVFL: {
            u32 f[16];
            mul_full256(x, y, f);
            u32 hi = 0;
#pragma unroll
            for (int k = 8; k < 16; ++k) hi |= f[k];
            if (w < 256) {
#pragma unroll
                for (int k = 0; k < 8; ++k) hi |= f[k] & ~width_mask(k, w);
            }
            z[0] = hi == 0;
            break;
        }
        case D_EXP:
            if constexpr ((FEAT & F_EVM) != 0) evm_exp(x, y, z, w);
            break;
        case D_SIGNEXT:
            if constexpr ((FEAT & F_EVM) != 0) evm_signextend(x, y, z);
            break;
        case D_BYTE:
            if constexpr ((FEAT & F_EVM) != 0) evm_byte(x, y, z);
            break;
        case D_ADDMOD: case D_MULMOD:
            if constexpr ((FEAT & F_EVM) != 0) evm_modop(op == D_MULMOD, x, y, c3, z, aux & 1u);
            break;
        case D_KECCAK:
            if constexpr ((FEAT & F_KECCAK) != 0) {
                u32 W2[8];
                copy8(W2, c3);
                keccak_words(x, y, W2, (w1 >> 8) & 3u, (w1 >> 10) & 1u, z);
            }
            break;
        case D_LOADVAR: env.var(aux, z); break;
        default:
            break;
    }
}

// True for the asm-core ops whose y is the inline constant (the *_C forms and D_LOADC).
MH_FN bool asm_op_yconst(u32 op) { return mh_pair_form(op) == 2 || op == D_LOADC; }

// asm-core ops that read y = R[b] in full
MH_FN bool asm_op_yreg(u32 op) {
    return mh_pair_form(op) == 1 || op == D_ITEC || op == D_SHL_V || op == D_LSHR_V ||
           op == D_ASHR_V;
}

// One instruction at slot ip (words w0, w1): X = f(R[a'], y, ...), R[d'] = X.  Returns the slots
// it occupies (1, or 5 with an inline constant).  D_END / D_WINDOW are the caller's business.
// SIMPLE = false drops the asm-core ops (the device runs those in assembly), so the device's
// C++ path only carries the code of the complex ops.
template <int FEAT, bool SIMPLE, class M>
MH_FN u32 step(M& m, u32 w0, u32 w1, u32 ip) {
    const u32 a = w0 & 0xFFu, b = (w0 >> 8) & 0xFFu, d = (w0 >> 16) & 0xFFu, c = w0 >> 24;
    const u32 op = mh_base_op(w1 & 0xFFu), aux = (w1 >> 17) & MH_AUX_MAX;
    u32 x[8], y[8], z[8];
    m.read(a, x);
    u32 len = 1;
    bool full_y;
    bool yconst;
    if (op < D_FIRST_COMPLEX) {
        yconst = asm_op_yconst(op);
        full_y = asm_op_yreg(op);
    } else {
        yconst = (w1 & F_YC) != 0;
        full_y = op != D_LOADVAR;
    }
    if (yconst) {
        m.iconst(ip + 1, y);
        len = 5;
    } else if (op == D_LOADVAR) {
        // no register operand: b / c carry the next column the tape loads (the asm core's
        // prefetch, compile.cpp), so neither is read
        zero8(y);
    } else if (full_y) {
        m.read(b, y);
    } else {
        y[0] = m.read0(b);
    }
    copy8(z, x);
    switch (op) {
        // ---- asm-core ops (reference semantics of asm_core_*.inc)
        case D_NOP: if constexpr (SIMPLE) {} break;
        case D_ADD_R: case D_ADD_C: if constexpr (SIMPLE) add256(x, y, z); break;
        case D_SUB_R: case D_SUB_C: if constexpr (SIMPLE) sub256(x, y, z); break;
        case D_RSUB_R: case D_RSUB_C: if constexpr (SIMPLE) sub256(y, x, z); break;
        case D_AND_R: case D_AND_C:
            if constexpr (SIMPLE) {
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = x[k] & y[k];
            }
            break;
        case D_OR_R: case D_OR_C:
            if constexpr (SIMPLE) {
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = x[k] | y[k];
            }
            break;
        case D_XOR_R: case D_XOR_C:
            if constexpr (SIMPLE) {
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = x[k] ^ y[k];
            }
            break;
        case D_EQ_R: case D_EQ_C: if constexpr (SIMPLE) z[0] = eq256(x, y); break;
        case D_ULT_R: case D_ULT_C: if constexpr (SIMPLE) z[0] = ult256(x, y); break;
        case D_UGT_R: case D_UGT_C: if constexpr (SIMPLE) z[0] = ult256(y, x); break;
        case D_ULE_R: case D_ULE_C: if constexpr (SIMPLE) z[0] = !ult256(y, x); break;
        case D_UGE_R: case D_UGE_C: if constexpr (SIMPLE) z[0] = !ult256(x, y); break;
        case D_SLT_R: case D_SLT_C: if constexpr (SIMPLE) z[0] = slt_w(x, y, 256); break;
        case D_SGT_R: case D_SGT_C: if constexpr (SIMPLE) z[0] = slt_w(y, x, 256); break;
        case D_SLE_R: case D_SLE_C: if constexpr (SIMPLE) z[0] = !slt_w(y, x, 256); break;
        case D_SGE_R: case D_SGE_C: if constexpr (SIMPLE) z[0] = !slt_w(x, y, 256); break;
        // Bool operands are canonical 0/1 in limb 0 (dev_isa.h), so, exactly like the asm core,
        // no mask: a producer that left other bits set would show here as a non-0/1 result,
        // which the host emulator rejects (tests/native/emu.cpp, mh_produces_bool)
        case D_BAND: case D_BANDZ: if constexpr (SIMPLE) z[0] = x[0] & y[0]; break;
        case D_BOR: if constexpr (SIMPLE) z[0] = x[0] | y[0]; break;
        case D_BXOR: if constexpr (SIMPLE) z[0] = x[0] ^ y[0]; break;
        case D_BEQ: if constexpr (SIMPLE) z[0] = x[0] ^ y[0] ^ 1u; break;
        case D_BNOT: if constexpr (SIMPLE) z[0] = x[0] ^ 1u; break;
        case D_TRUE: if constexpr (SIMPLE) z[0] = 1u; break;
        case D_FALSE: if constexpr (SIMPLE) z[0] = 0u; break;
        case D_ITE:
            if constexpr (SIMPLE) {
                u32 e[8];
                m.read(c, e);
                const bool cnd = (y[0] & 1u) != 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = cnd ? x[k] : e[k];
            }
            break;
        case D_ITEC:
            if constexpr (SIMPLE) {
                u32 e[8];
                m.read(c, e);
                const bool cnd = (x[0] & 1u) != 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = cnd ? y[k] : e[k];
            }
            break;
        case D_BITE:
            if constexpr (SIMPLE) z[0] = (x[0] & 1u) ? (y[0] & 1u) : (m.read0(c) & 1u);
            break;
        case D_LOADC: if constexpr (SIMPLE) copy8(z, y); break;
        case D_SHR0: case D_SHR1: case D_SHR2: case D_SHR3: case D_SHR4: case D_SHR5:
        case D_SHR6: case D_SHR7:
            if constexpr (SIMPLE) shr256_u(x, 32u * (op - D_SHR0) + (aux & 31u), z, 0u);
            break;
        case D_SHL0: case D_SHL1: case D_SHL2: case D_SHL3: case D_SHL4: case D_SHL5:
        case D_SHL6: case D_SHL7:
            if constexpr (SIMPLE) {
                const u32 p = op - D_SHL0, f = aux & 31u;
                const u32 s = f ? 32u * p + 32u - f : 32u * (p + 1u);
                if (s >= 256u) zero8(z);
                else shl256_u(x, s, z);
            }
            break;
        case D_MUL_R: case D_MUL_C: if constexpr (SIMPLE) mul_lo256(x, y, z); break;
        case D_SHL_V: if constexpr (SIMPLE) bvshl_v(x, shift_amount(y), z, 256); break;
        case D_LSHR_V: if constexpr (SIMPLE) bvlshr_v(x, shift_amount(y), z, 256); break;
        case D_ASHR_V: if constexpr (SIMPLE) bvashr_v(x, shift_amount(y), z, 256); break;
        case D_UDIV_R: case D_UDIV_C: case D_UREM_R: case D_UREM_C: case D_SDIV_R: case D_SDIV_C:
        case D_SREM_R: case D_SREM_C: case D_SMOD_R: case D_SMOD_C:
            if constexpr (SIMPLE) divmod_family((op - D_UDIV_R) >> 1, x, y, z, 256);
            break;
        default:
            if (op >= D_FIRST_COMPLEX) {
                u32 c3[8];
                if (op == D_LOADVAR) zero8(c3);
                else m.read(c, c3);
                complex_op<FEAT>(m, w1, x, y, c3, z);
            }
            break;
    }
    m.write(m.nrx(), z);
    m.write(d, z);
    return len;
}

}  // namespace mh
