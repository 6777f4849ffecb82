// TEST-ONLY host emulator of the device interpreter (not part of libmythril_hip).
//
// Runs the tape compiler (mythril_amd/csrc/compile.cpp) and then the device instruction stream
// on the host CPU, using the same limb routines the kernel uses (mythril_amd/csrc/u256_ops.h).
// It lets tests/test_emulator.py check the compiler (lowering, register allocation, encoding)
// and the 256-bit algorithms (division, shifts, signed ops, keccak-f) against the Python oracle
// without a GPU.  The dispatch below mirrors exec_tape() in sieve_kernels.hip; the keccak message
// assembly is restated with a byte buffer (the device version is covered by the GPU tests).
#include <stdint.h>
#include <string.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "compile.h"
#include "u256_ops.h"

using namespace mh;

static void keccak_msg(const u32* P0, const u32* P1, const u32* P2, u32 n0, u32 n1, u32 n2,
                       u32* z) {
    uint8_t msg[136];
    memset(msg, 0, sizeof(msg));
    const u32* P[3] = {P0, P1, P2};
    const u32 n[3] = {n0, n1, n2};
    u32 off = 0;
    for (int p = 0; p < 3; ++p) {
        for (u32 j = 0; j < n[p]; ++j) {
            const u32 e = n[p] - 1 - j;
            msg[off + j] = (uint8_t)(P[p][e >> 2] >> (8 * (e & 3)));
        }
        off += n[p];
    }
    msg[off] |= 0x01;
    msg[135] |= 0x80;
    u64 st[25];
    memset(st, 0, sizeof(st));
    for (int i = 0; i < 17; ++i) {
        u64 v = 0;
        for (int b = 0; b < 8; ++b) v |= (u64)msg[8 * i + b] << (8 * b);
        st[i] = v;
    }
    keccak_f1600(st);
    for (int k = 0; k < 8; ++k) {
        const int i = 7 - k;
        const u32 wv = (i & 1) ? (u32)(st[i >> 1] >> 32) : (u32)st[i >> 1];
        z[k] = bswap32(wv);
    }
}

static void exec(u32 R[MH_NUM_REGS][8], const u32* ip, u32 n, const u32* consts,
                 const u32* assign, u64 cap, u64 row) {
    for (u32 i = 0; i < n; ++i) {
        const u32 w0 = ip[2 * i], w1 = ip[2 * i + 1];
        const u32 op = w0 & 0xFFu, d = (w0 >> 8) & 0xFFu, a = (w0 >> 16) & 0xFFu, b = w0 >> 24;
        const u32 flags = ((MH_CONST_OPERAND_OK >> op) & 1u) ? (w1 & 3u) : 0u;
        const u32 w = (w1 >> 2) & 0x1FFu, aux = w1 >> 11;
        // z starts as garbage, as in the kernel: a handler that leaves limbs unwritten is a bug
        u32 x[8], y[8], z[8];
        for (int k = 0; k < 8; ++k) z[k] = 0xA5A5A5A5u ^ (u32)k;
        memcpy(x, (flags & F_ACONST) ? consts + 8ull * aux : R[a], 32);
        memcpy(y, (flags & F_BCONST) ? consts + 8ull * aux : R[b], 32);
        switch (op) {
            case D_ADD: add256(x, y, z); mask_w(z, w); break;
            case D_SUB: sub256(x, y, z); mask_w(z, w); break;
            case D_MUL: mul_lo256(x, y, z); mask_w(z, w); break;
            case D_AND: for (int k = 0; k < 8; ++k) z[k] = x[k] & y[k]; break;
            case D_OR: for (int k = 0; k < 8; ++k) z[k] = x[k] | y[k]; break;
            case D_XOR: for (int k = 0; k < 8; ++k) z[k] = x[k] ^ y[k]; break;
            case D_SHL: bvshl_v(x, shift_amount(y), z, w); break;
            case D_LSHR: bvlshr_v(x, shift_amount(y), z, w); break;
            case D_ASHR: bvashr_v(x, shift_amount(y), z, w); break;
            case D_CONCAT: {
                u32 t[8];
                shl256(x, aux, t);
                for (int k = 0; k < 8; ++k) z[k] = t[k] | y[k];
                break;
            }
            case D_UDIV: case D_UREM: case D_SDIV: case D_SREM: case D_SMOD:
                divmod_family(op - D_UDIV, x, y, z, w);
                break;
            case D_EXP: evm_exp(x, y, z, w); break;
            case D_SIGNEXT: evm_signextend(x, y, z); break;
            case D_BYTE: evm_byte(x, y, z); break;
            case D_NEG: neg256(x, z); mask_w(z, w); break;
            case D_NOT: for (int k = 0; k < 8; ++k) z[k] = ~x[k]; mask_w(z, w); break;
            case D_SHLI: if (aux < w) { shl256(x, aux, z); mask_w(z, w); } else memset(z, 0, 32); break;
            case D_LSHRI: if (aux < w) shr256(x, aux, z, 0u); else memset(z, 0, 32); break;
            case D_ASHRI: bvashr_v(x, aux, z, w); break;
            case D_EXTRACT: shr256(x, aux, z, 0u); mask_w(z, w); break;
            case D_SEXT: sext_to256(x, aux, z); mask_w(z, w); break;
            case D_MOV: memcpy(z, x, 32); break;
            case D_EQ: z[0] = eq256(x, y); break;
            case D_ULT: z[0] = ult256(x, y); break;
            case D_ULE: z[0] = !ult256(y, x); break;
            case D_SLT: z[0] = slt_w(x, y, w); break;
            case D_SLE: z[0] = !slt_w(y, x, w); break;
            case D_UADD_NOOVFL: {
                u32 t[8];
                const u32 cy = add256(x, y, t);
                u32 hi = 0;
                if (w < 256) for (int k = 0; k < 8; ++k) hi |= t[k] & ~width_mask(k, w);
                z[0] = !(cy || hi);
                break;
            }
            case D_UMUL_NOOVFL: {
                u32 t[16];
                mul_full256(x, y, t);
                u32 hi = 0;
                for (int k = 8; k < 16; ++k) hi |= t[k];
                if (w < 256) for (int k = 0; k < 8; ++k) hi |= t[k] & ~width_mask(k, w);
                z[0] = hi == 0;
                break;
            }
            case D_BAND: z[0] = x[0] & y[0] & 1u; break;
            case D_BOR: z[0] = (x[0] | y[0]) & 1u; break;
            case D_BXOR: z[0] = (x[0] ^ y[0]) & 1u; break;
            case D_BEQ: z[0] = ((x[0] ^ y[0]) & 1u) ^ 1u; break;
            case D_BNOT: z[0] = (x[0] & 1u) ^ 1u; break;
            case D_TRUE: z[0] = 1u; break;
            case D_FALSE: z[0] = 0u; break;
            case D_ITE: {
                const bool cnd = (x[0] & 1u) != 0;
                for (int k = 0; k < 8; ++k) z[k] = cnd ? y[k] : R[aux][k];
                break;
            }
            case D_BITE: z[0] = (x[0] & 1u) ? (y[0] & 1u) : (R[aux][0] & 1u); break;
            case D_LOADC: memcpy(z, consts + 8ull * aux, 32); break;
            case D_LOADVAR:
                for (int k = 0; k < 8; ++k) z[k] = assign[((u64)aux * 8 + k) * cap + row];
                break;
            case D_KECCAK: {
                const u32 np = (w1 >> 26) & 3u;
                const u32 n0 = (w1 >> 8) & 63u, n1 = (w1 >> 14) & 63u, n2 = (w1 >> 20) & 63u;
                keccak_msg(x, y, R[w1 & 0xFFu], n0, np > 1 ? n1 : 0u, np > 2 ? n2 : 0u, z);
                break;
            }
            default: break;
        }
        memcpy(R[d], z, 32);
    }
}

extern "C" int32_t emu_eval(const mh_node* nodes, const uint64_t* offs, uint32_t n_tapes,
                            const uint32_t* consts, uint32_t n_consts, uint32_t n_vars,
                            uint32_t tape, const uint32_t* assign, uint64_t rows, uint32_t* out,
                            uint32_t* n_regs_out, char* err, int errlen) {
    std::vector<uint32_t> dconsts, words;
    std::unordered_map<std::string, uint32_t> dindex;
    CompiledTape sel{};
    uint32_t sel_off = 0;
    for (uint32_t t = 0; t < n_tapes; ++t) {
        CompiledTape ct;
        std::string e;
        const uint32_t first = (uint32_t)(words.size() / 2);
        int32_t r = compile_tape(nodes + offs[t], (size_t)(offs[t + 1] - offs[t]), consts,
                                 n_consts, n_vars, dconsts, dindex, words, ct, e);
        if (r != MH_OK) {
            snprintf(err, errlen, "tape %u: %s", t, e.c_str());
            return r;
        }
        if (t == tape) {
            sel = ct;
            sel_off = first;
        }
    }
    if (n_regs_out) *n_regs_out = sel.n_regs;
    const uint32_t n_pre = n_vars <= MH_MAX_PRELOAD ? n_vars : 0;
    for (uint64_t row = 0; row < rows; ++row) {
        u32 R[MH_NUM_REGS][8];
        memset(R, 0xCD, sizeof(R));  // poison: reads of never-written registers show up
        for (uint32_t v = 0; v < n_pre; ++v)
            for (int k = 0; k < 8; ++k) R[v][k] = assign[((u64)v * 8 + k) * rows + row];
        exec(R, words.data() + 2ull * sel_off, sel.n_insns, dconsts.data(), assign, rows, row);
        u32 res[8];
        memcpy(res, R[sel.root_reg], 32);
        if (sel.root_bool) {
            res[0] &= 1u;
            for (int k = 1; k < 8; ++k) res[k] = 0;
        }
        for (int k = 0; k < 8; ++k) out[(u64)k * rows + row] = res[k];
    }
    return MH_OK;
}
