// Tape compiler: mh_node IR (include/mythril_hip.h) -> device code (dev_isa.h, ISA v4).
//
// Per tape:
//  1. reachability from the root and legalisation: values wider than 256 bits exist only as
//     Concat/ZeroExt chains feeding Keccak, kept as lists of byte-aligned pieces;
//  2. lowering, in a Sethi-Ullman post-order, to device ops on SSA virtual registers: the asm-core
//     ops (add/sub/logic/compares/selects/immediate shifts, with explicit AND masks where a
//     narrow result could overflow its width) and the complex ops run in C++ (mul, division,
//     variable shifts, narrow signed compares, keccak, EVM helpers); a constant second operand
//     becomes an inline constant (the *_C forms);
//  3. the accumulator pass: each instruction's first operand is the previous result (kept in X)
//     whenever possible, through operand swaps and mirrored ops (a - b = rsub(b, a), a < b =
//     b > a); a result is written back to the register file only if something reads it again
//     from there;
//  4. linear-scan allocation of the written-back values onto at most MH_NR_MAX registers
//     (assignment columns 0..3 pinned in R0..R3), which fixes the kernel variant (NR) and hence
//     the accumulator index NRX used in the encoding;
//  5. slot layout: inline constants, 64-slot windows closed by D_WINDOW, D_END.
// Anything the device path does not cover returns MH_E_UNSUPPORTED so the caller falls back to
// z3, as get_model's contract requires.
#include "compile.h"
#include "exec.h"

#include <algorithm>
#include <numeric>
#include <cstdlib>
#include <functional>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace mh {

namespace {

// algorithmic u32 ALU ops per IR node (SURVEY.md §8d op-cost table)
uint64_t op_cost(const mh_node& n, const std::vector<mh_node>& t) {
    switch (n.op) {
        case MH_OP_CONST: case MH_OP_VAR: case MH_OP_TRUE: case MH_OP_FALSE: return 0;
        case MH_OP_BVADD: case MH_OP_BVSUB: case MH_OP_BVNEG: return 8;
        case MH_OP_BVAND: case MH_OP_BVOR: case MH_OP_BVXOR: case MH_OP_BVNOT: return 8;
        case MH_OP_EQ: return t[n.a].width == 0 ? 1 : 15;
        case MH_OP_BVULT: case MH_OP_BVULE: case MH_OP_BVUGT: case MH_OP_BVUGE:
        case MH_OP_BVSLT: case MH_OP_BVSLE: case MH_OP_BVSGT: case MH_OP_BVSGE: return 16;
        case MH_OP_ITE: return n.width == 0 ? 1 : 8;
        case MH_OP_BVSHL: case MH_OP_BVLSHR: case MH_OP_BVASHR:
            return t[n.b].op == MH_OP_CONST ? 8 : 24;
        case MH_OP_EXTRACT: case MH_OP_CONCAT: case MH_OP_ZEXT: case MH_OP_SEXT: return 8;
        case MH_OP_BVMUL: return 64;
        case MH_OP_BVUDIV: case MH_OP_BVUREM: case MH_OP_BVSDIV: case MH_OP_BVSREM:
        case MH_OP_BVSMOD: return 1100;
        case MH_OP_AND: case MH_OP_OR: case MH_OP_XOR: case MH_OP_NOT: return 1;
        case MH_OP_KECCAK: return 9600ull * ((t[n.a].width / 8) / 136 + 1);
        case MH_OP_BVADD_NOOVFL_U: case MH_OP_BVSUB_NOUDFL_U: return 16;
        case MH_OP_BVMUL_NOOVFL_U: return 128;
        case MH_OP_EVM_EXP: return 256ull * 2 * 64;
        case MH_OP_EVM_SIGNEXTEND: case MH_OP_EVM_BYTE: return 24;
        case MH_OP_EVM_ADDMOD: return 8 + 2200;              // sum + 512-bit remainder
        case MH_OP_EVM_MULMOD: return 128 + 2200;            // product + 512-bit remainder
        default: return 0;
    }
}

// ops whose y may be an inline constant: asm pairs (given as the *_R form) and binary complex ops
bool y_const_ok(uint8_t op) {
    if (mh_pair_form(op)) return mh_pair_form(op) == 1;
    switch (op) {
        case D_UADD_NOOVFL: case D_UMUL_NOOVFL: case D_EXP: case D_SIGNEXT: case D_BYTE:
            return true;
        default:
            return false;
    }
}

bool commutes(uint8_t op) {
    switch (op) {
        case D_ADD_R: case D_AND_R: case D_OR_R: case D_XOR_R: case D_EQ_R: case D_MUL_R:
        case D_UADD_NOOVFL: case D_UMUL_NOOVFL: case D_BAND: case D_BOR: case D_BXOR: case D_BEQ:
        case D_BANDZ:
            return true;
        default:
            return false;
    }
}

uint8_t mirror(uint8_t op) {  // op(a, b) == mirror(op)(b, a), or 0
    switch (op) {
        case D_SUB_R: return D_RSUB_R;
        case D_RSUB_R: return D_SUB_R;
        case D_ULT_R: return D_UGT_R;
        case D_UGT_R: return D_ULT_R;
        case D_ULE_R: return D_UGE_R;
        case D_UGE_R: return D_ULE_R;
        case D_SLT_R: return D_SGT_R;
        case D_SGT_R: return D_SLT_R;
        case D_SLE_R: return D_SGE_R;
        case D_SGE_R: return D_SLE_R;
        default: return 0;
    }
}

// Diagnostic switch: MH_XFORM_MASK (env, default all) enables X forms per group --
// 1 add/sub R, 2 add/sub C, 4 logic R, 8 logic C, 16 eq, 32 compares R, 64 compares C,
// 256 mul, 512 loadc.
bool xform_enabled(uint32_t op) {
    static const uint32_t mask = [] {
        const char* e = std::getenv("MH_XFORM_MASK");
        return e ? (uint32_t)std::strtoul(e, nullptr, 0) : ~0u;
    }();
    uint32_t g = 0;
    switch (op) {
        case D_ADD_R: case D_SUB_R: case D_RSUB_R: g = 1; break;
        case D_ADD_C: case D_SUB_C: case D_RSUB_C: g = 2; break;
        case D_AND_R: case D_OR_R: case D_XOR_R: g = 4; break;
        case D_AND_C: case D_OR_C: case D_XOR_C: g = 8; break;
        case D_EQ_R: case D_EQ_C: g = 16; break;
        case D_MUL_R: case D_MUL_C: g = 256; break;
        case D_LOADC: g = 512; break;
        default:
            if (op >= D_ULT_R && op <= D_SGE_C) g = ((op - D_ULT_R) & 1) ? 64 : 32;
            break;
    }
    return (mask & g) != 0;
}

typedef SsaInsn VInsn;

struct Piece {
    int vreg;
    uint32_t bits;
};

// A lowered IR value: a virtual register (<= 256 bits or Bool), or a piece list (> 256 bits,
// most significant piece first).
struct Val {
    int vreg = -1;
    int remat = -1;  // constant node re-materialised at every use (keeps pressure low)
    std::vector<Piece> pieces;
    bool wide() const { return !pieces.empty(); }
};

uint32_t lane_mask(int k, uint32_t w) {
    const int rem = (int)w - 32 * k;
    return rem >= 32 ? 0xFFFFFFFFu : rem <= 0 ? 0u : ((1u << rem) - 1u);
}

struct Lowering {
    const std::vector<mh_node>& t;
    const uint32_t* consts;
    uint32_t n_consts;
    uint32_t n_vars;
    bool pinned;
    std::vector<uint32_t>& pool;  // deduplicated 256-bit constants (8 limbs each)
    ConstIndex& pool_index;
    std::vector<VInsn> code;
    int n_vregs = 0;
    uint32_t features = 0;
    std::string err;
    std::vector<Val>* vals_ = nullptr;

    Lowering(const std::vector<mh_node>& tape, const uint32_t* c, uint32_t nc, uint32_t nv,
             std::vector<uint32_t>& pl, ConstIndex& pi)
        : t(tape), consts(c), n_consts(nc), n_vars(nv), pinned(nv <= MH_MAX_PRELOAD),
          pool(pl), pool_index(pi) {
        if (pinned) n_vregs = (int)nv;  // vregs 0..nv-1 are the pinned columns
    }

    int fresh() { return n_vregs++; }

    int emit(uint8_t op, int a = -1, int b = -1, int c = -1, uint32_t width = 256,
             uint32_t aux = 0, int cidx = -1) {
        VInsn v{op, fresh(), a, b, c, width, aux, cidx, 0};
        code.push_back(v);
        return v.d;
    }

    bool fail(const std::string& m) {
        if (err.empty()) err = m;
        return false;
    }

    uint32_t const_index(const uint32_t* limbs, uint32_t width) {
        ConstKey key;
        for (int k = 0; k < 8; ++k) key.w[k] = limbs[k] & lane_mask(k, width);
        auto it = pool_index.find(key);
        if (it != pool_index.end()) return it->second;
        uint32_t idx = (uint32_t)(pool.size() / 8);
        pool.insert(pool.end(), key.w, key.w + 8);
        pool_index.emplace(key, idx);
        return idx;
    }

    int mask_const(uint32_t w) {
        static const uint32_t ones[8] = {~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u, ~0u};
        return (int)const_index(ones, w);
    }

    int zero_const() {
        static const uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        return (int)const_index(z, 256);
    }

    // r & (2^w - 1) when w < 256 (keeps narrow values canonical)
    int masked(int r, uint32_t w) {
        if (w >= 256 || r < 0) return r;
        return emit(D_AND_R, r, -1, -1, w, 0, mask_const(w));
    }

    int bit_const(uint32_t b) {  // 2^b, b < 256
        uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        m[b >> 5] = 1u << (b & 31);
        return (int)const_index(m, 256);
    }

    // sign extension of a canonical wa-bit value to 256 bits: (x ^ 2^(wa-1)) - 2^(wa-1)
    int sext256(int r, uint32_t wa) {
        if (wa >= 256 || r < 0) return r;
        const int m = bit_const(wa - 1);
        return emit(D_SUB_R, emit(D_XOR_R, r, -1, -1, 256, 0, m), -1, -1, 256, 0, m);
    }

    // arithmetic shift right by a uniform s at width w:
    // ((x ^ 2^(w-1)) >> s') - 2^(w-1-s'), s' = min(s, w-1), then masked to w
    int ashr_imm(int r, uint32_t s, uint32_t w) {
        const uint32_t sp = s < w - 1 ? s : w - 1;
        int u = emit(D_XOR_R, r, -1, -1, 256, 0, bit_const(w - 1));
        if (sp) u = shr_imm(u, sp);
        u = emit(D_SUB_R, u, -1, -1, 256, 0, bit_const(w - 1 - sp));
        return masked(u, w);
    }

    // op(sext256(a), sext256(b)) for a binary op on signed operands of width w < 256 (a
    // constant operand is sign-extended on the host and becomes the inline constant)
    int emit_sext_bin(uint8_t op, uint32_t na, uint32_t nb, uint32_t w) {
        auto sext_const = [&](uint32_t k) {
            const mh_node& c = t[(size_t)(*vals_)[k].remat];
            uint32_t m[8];
            for (int i = 0; i < 8; ++i) m[i] = consts[8ull * c.imm0 + i] & lane_mask(i, w);
            if ((m[(w - 1) >> 5] >> ((w - 1) & 31)) & 1u)
                for (int i = 0; i < 8; ++i) m[i] |= ~lane_mask(i, w);
            return (int)const_index(m, 256);
        };
        auto sx = [&](uint32_t k) {
            const int r = vreg_of(k);
            return r < 0 ? -1 : sext256(r, w);
        };
        if (is_const_node(nb)) return emit(op, sx(na), -1, -1, 256, 0, sext_const(nb));
        const int a = sx(na), b = sx(nb);
        if (a < 0 || b < 0) return -1;
        return emit(op, a, b, -1, 256);
    }

    // signed compare at width w < 256 as the unsigned compare of the biased values
    // x ^ 2^(w-1) (a constant operand is biased on the host)
    int emit_scmp(uint8_t uop, uint32_t na, uint32_t nb, uint32_t w) {
        auto biased_const = [&](uint32_t k) {
            const mh_node& c = t[(size_t)(*vals_)[k].remat];
            uint32_t m[8];
            for (int i = 0; i < 8; ++i) m[i] = consts[8ull * c.imm0 + i] & lane_mask(i, w);
            m[(w - 1) >> 5] ^= 1u << ((w - 1) & 31);
            return (int)const_index(m, 256);
        };
        auto bias = [&](uint32_t k) {
            const int r = vreg_of(k);
            return r < 0 ? -1 : emit(D_XOR_R, r, -1, -1, 256, 0, bit_const(w - 1));
        };
        if (is_const_node(nb)) return emit(uop, bias(na), -1, -1, 256, 0, biased_const(nb));
        if (is_const_node(na))
            return emit(mirror(uop), bias(nb), -1, -1, 256, 0, biased_const(na));
        const int a = bias(na), b = bias(nb);
        if (a < 0 || b < 0) return -1;
        return emit(uop, a, b, -1, 256);
    }

    bool is_const_node(uint32_t k) const {
        const Val& v = (*vals_)[k];
        return !v.wide() && v.remat >= 0 && t[(size_t)v.remat].op == MH_OP_CONST;
    }

    int const_of(uint32_t k) {
        const mh_node& c = t[(size_t)(*vals_)[k].remat];
        return (int)const_index(consts + 8ull * c.imm0, c.width);
    }

    // register holding narrow value k (constants, and assignment columns that are not pinned in
    // registers, are re-materialised at each use: a column load costs less than keeping a value
    // live, and a query over many columns would otherwise exceed the register file)
    int vreg_of(uint32_t k) {
        const Val& v = (*vals_)[k];
        if (v.wide()) return -1;
        if (v.remat >= 0) {
            const mh_node& c = t[(size_t)v.remat];
            if (c.op == MH_OP_TRUE) return emit(D_TRUE, -1, -1, -1, 1);
            if (c.op == MH_OP_FALSE) return emit(D_FALSE, -1, -1, -1, 1);
            if (c.op == MH_OP_VAR) {
                const uint64_t key = (uint64_t)c.imm0 << 16 | c.width;
                bool hold = false;
                if (hold_vars) {
                    auto u = uses_.find(key);
                    hold = u != uses_.end() && u->second >= kHoldUses;
                }
                if (hold) {
                    auto it = held_.find(key);
                    if (it != held_.end()) return it->second;
                }
                const int r = masked(emit(D_LOADVAR, -1, -1, -1, 256, c.imm0), c.width);
                if (hold) held_.emplace(key, r);
                return r;
            }
            return emit(D_LOADC, -1, -1, -1, 256, 0,
                        (int)const_index(consts + 8ull * c.imm0, c.width));
        }
        return v.vreg;
    }

    // Binary op on IR nodes na, nb: a constant operand becomes the inline constant y (swapping
    // through commutativity or the mirrored op when the constant is the first operand).
    int emit_bin(uint8_t op, uint32_t na, uint32_t nb, uint32_t width) {
        if (y_const_ok(op)) {
            const bool ca = is_const_node(na), cb = is_const_node(nb);
            if (cb || (ca && (commutes(op) || mirror(op)))) {
                uint8_t o = op;
                uint32_t kc = nb, kr = na;
                if (!cb) {
                    kc = na;
                    kr = nb;
                    if (!commutes(op)) o = mirror(op);
                }
                const int r = vreg_of(kr);
                if (r < 0) return -1;
                return emit(o, r, -1, -1, width, 0, const_of(kc));
            }
        }
        const int a = vreg_of(na), b = vreg_of(nb);
        if (a < 0 || b < 0) return -1;
        return emit(op, a, b, -1, width);
    }

    // logical shift left by a uniform amount s (0 < s < 256), result mod 2^256: the limb-count
    // op D_SHL0 + p with the alignbit field (dev_isa.h)
    int shl_imm(int r, uint32_t s) {
        const uint32_t q = s >> 5, b = s & 31;
        if (b) return emit((uint8_t)(D_SHL0 + q), r, -1, -1, 256, 32 - b);
        return emit((uint8_t)(D_SHL0 + q - 1), r, -1, -1, 256, 0);
    }

    // logical shift right by a uniform amount s (0 < s < 256)
    int shr_imm(int r, uint32_t s) {
        return emit((uint8_t)(D_SHR0 + (s >> 5)), r, -1, -1, 256, s & 31);
    }

    // bits [lo, lo + w) of a wa-bit canonical value
    int extract(int r, uint32_t lo, uint32_t w, uint32_t wa) {
        if (lo) r = shr_imm(r, lo);
        if (lo + w < wa) r = masked(r, w);
        return r;
    }

    // (hi << wb) | lo for canonical parts, wb + width(hi) <= 256
    int concat(int hi, int lo, uint32_t wb) { return emit(D_OR_R, shl_imm(hi, wb), lo, -1); }

    // ---- native-code forms (jit = true, the JIT's lowering): the complex ops the JIT has no
    // machine code for, restated on ops it has.  Same values as exec.h complex_op on canonical
    // operands (tests/test_jit.py checks each against the oracle).
    bool jit = false;
    // interpreter: a loaded-on-use column read by at least kHoldUses operands is loaded once and
    // kept in a register (each load is a complex op, ~1 us of a wave's time; calldata bytes all
    // compare their index with calldatasize) -- off again when the tape runs out of registers
    bool hold_vars = false;
    // (uses are counted per column and width: a rematerialised tape gives every use of a column
    // a VAR node of its own)
    static constexpr uint32_t kHoldUses = 3;
    std::unordered_map<uint64_t, uint32_t> uses_;
    std::unordered_map<uint64_t, int> held_;

    int small_const(uint32_t x) {
        const uint32_t m[8] = {x, 0, 0, 0, 0, 0, 0, 0};
        return (int)const_index(m, 256);
    }
    // limbs of constant node k masked to w bits
    void const_limbs(uint32_t k, uint32_t w, uint32_t* m) const {
        const mh_node& c = t[(size_t)(*vals_)[k].remat];
        for (int i = 0; i < 8; ++i) m[i] = consts[8ull * c.imm0 + i] & lane_mask(i, w);
    }
    // 248 - 8 k mod 2^256: the right shift that brings big-endian byte k of a word to the bottom
    int byte_shift(int k) {
        return emit(D_RSUB_R, shl_imm(k, 3), -1, -1, 256, 0, small_const(248));
    }
    // SIGNEXTEND(k, x): for k < 31, x shifted left and arithmetically right by 248 - 8k (the sign
    // bit 8k + 7 lands on bit 255 and is copied back down); x itself otherwise
    int jit_signextend(uint32_t nk, uint32_t nx) {
        if (is_const_node(nk)) {
            uint32_t m[8];
            const_limbs(nk, 256, m);
            const int x = vreg_of(nx);
            if (m[1] | m[2] | m[3] | m[4] | m[5] | m[6] | m[7] || m[0] > 30) return x;
            const uint32_t s = 248 - 8 * m[0];
            return ashr_imm(shl_imm(x, s), s, 256);
        }
        const int k = vreg_of(nk), x = vreg_of(nx);
        if (k < 0 || x < 0) return -1;
        const int s = byte_shift(k);
        const int u = emit(D_ASHR_V, emit(D_SHL_V, x, s, -1, 256), s, -1, 256);
        const int in_range = emit(D_ULT_R, k, -1, -1, 256, 0, small_const(31));
        return emit(D_ITE, in_range, u, x, 256);
    }
    // BYTE(i, x): (x >> (248 - 8 i)) & 0xff for i < 32, else 0
    int jit_byte(uint32_t ni, uint32_t nx) {
        if (is_const_node(ni)) {
            uint32_t m[8];
            const_limbs(ni, 256, m);
            if (m[1] | m[2] | m[3] | m[4] | m[5] | m[6] | m[7] || m[0] > 31)
                return emit(D_LOADC, -1, -1, -1, 256, 0, zero_const());
            const uint32_t s = 248 - 8 * m[0];
            int x = vreg_of(nx);
            if (x < 0) return -1;
            if (s) x = shr_imm(x, s);
            return emit(D_AND_R, x, -1, -1, 256, 0, small_const(0xFF));
        }
        const int i = vreg_of(ni), x = vreg_of(nx);
        if (i < 0 || x < 0) return -1;
        const int u = emit(D_AND_R, emit(D_LSHR_V, x, byte_shift(i), -1, 256), -1, -1, 256, 0,
                           small_const(0xFF));
        const int in_range = emit(D_ULT_R, i, -1, -1, 256, 0, small_const(32));
        return emit(D_ITE, in_range, u, emit(D_LOADC, -1, -1, -1, 256, 0, zero_const()), 256);
    }
    // EXP(b, e) mod 2^w: a constant exponent as left-to-right square and multiply, a symbolic one
    // stays D_EXP (the native code's loop, jit.cpp op_exp)
    int jit_exp(uint32_t nb, uint32_t ne, uint32_t w) {
        if (!is_const_node(ne)) {  // a per-lane exponent: the native code's EXP loop
            const int b = vreg_of(nb), x = vreg_of(ne);
            return b < 0 || x < 0 ? -1 : masked(emit(D_EXP, b, x, -1, 256), w);
        }
        uint32_t e[8];
        const_limbs(ne, w, e);
        int top = -1;
        for (int i = 255; i >= 0 && top < 0; --i)
            if ((e[i >> 5] >> (i & 31)) & 1u) top = i;
        if (top < 0) return emit(D_LOADC, -1, -1, -1, 256, 0, small_const(1));
        const int b = vreg_of(nb);
        if (b < 0) return -1;
        int r = b;
        for (int i = top - 1; i >= 0; --i) {
            r = emit(D_MUL_R, r, r, -1, 256);
            if ((e[i >> 5] >> (i & 31)) & 1u) r = emit(D_MUL_R, r, b, -1, 256);
        }
        return masked(r, w);
    }
    // BVAddNoOverflow(a, b, False) at width w: b <= a ^ (2^w - 1)  (a + b < 2^w)
    int jit_add_noovfl(uint32_t na, uint32_t nb, uint32_t w) {
        if (is_const_node(nb) && !is_const_node(na)) std::swap(na, nb);
        if (is_const_node(na)) {
            uint32_t m[8];
            const_limbs(na, w, m);
            for (int i = 0; i < 8; ++i) m[i] = ~m[i] & lane_mask(i, w);
            const int b = vreg_of(nb);
            return b < 0 ? -1 : emit(D_ULE_R, b, -1, -1, 256, 0, (int)const_index(m, 256));
        }
        const int a = vreg_of(na);
        if (a < 0) return -1;
        const int na_ = emit(D_XOR_R, a, -1, -1, 256, 0, mask_const(w));
        if (is_const_node(nb)) return emit(D_UGE_R, na_, -1, -1, 256, 0, const_of(nb));
        const int b = vreg_of(nb);
        return b < 0 ? -1 : emit(D_ULE_R, b, na_, -1, 256);
    }
    // BVMulNoOverflow(a, b, False) at width w: b <= floor((2^w - 1) / a)  (a = 0: the quotient
    // is 2^256 - 1, SMT-LIB x / 0, and the compare holds, as a * b = 0 does not overflow)
    int jit_mul_noovfl(uint32_t na, uint32_t nb, uint32_t w) {
        if (is_const_node(nb) && !is_const_node(na)) std::swap(na, nb);
        if (is_const_node(na)) {
            uint32_t c[8], mw[8], q[8];
            const_limbs(na, w, c);
            if (!(c[0] | c[1] | c[2] | c[3] | c[4] | c[5] | c[6] | c[7]))
                return emit(D_TRUE, -1, -1, -1, 1);
            for (int i = 0; i < 8; ++i) mw[i] = lane_mask(i, w);
            divmod_family(0, mw, c, q, 256);
            const int b = vreg_of(nb);
            return b < 0 ? -1 : emit(D_ULE_R, b, -1, -1, 256, 0, (int)const_index(q, 256));
        }
        const int a = vreg_of(na), b = vreg_of(nb);
        if (a < 0 || b < 0) return -1;
        const int q = emit(D_UDIV_R, emit(D_LOADC, -1, -1, -1, 256, 0, mask_const(w)), a, -1, 256);
        return emit(D_ULE_R, b, q, -1, 256);
    }
    // yellow-paper ADDMOD (exact sum): t = (a mod n) + (b mod n) mod 2^256, minus n when the
    // exact sum (carry or t >= n) reaches n; n = 0 leaves t = a + b mod 2^256 (zero_low) or 0
    int jit_addmod(int a, int b, int n, bool zero_low) {
        const int r1 = emit(D_UREM_R, a, n, -1, 256), r2 = emit(D_UREM_R, b, n, -1, 256);
        const int t_ = emit(D_ADD_R, r1, r2, -1, 256);
        const int ge = emit(D_BOR, emit(D_ULT_R, t_, r1, -1, 256), emit(D_UGE_R, t_, n, -1, 256),
                            -1, 1);
        int r = emit(D_ITE, ge, emit(D_SUB_R, t_, n, -1, 256), t_, 256);
        if (!zero_low) {
            const int nz = emit(D_EQ_R, n, -1, -1, 256, 0, zero_const());
            r = emit(D_ITE, nz, emit(D_LOADC, -1, -1, -1, 256, 0, zero_const()), r, 256);
        }
        return r;
    }
    // yellow-paper MULMOD (exact product): (a mod n) * (b mod n) mod n by the native code's
    // double-and-add loop (D_MULMOD with aux bit 1: operands reduced); n = 0 gives the low 256
    // bits of a * b (zero_low) or 0
    int jit_mulmod(int a, int b, int n, bool zero_low) {
        const int x = emit(D_UREM_R, a, n, -1, 256), y = emit(D_UREM_R, b, n, -1, 256);
        const int r = emit(D_MULMOD, x, y, n, 256, zero_low ? 3u : 2u);
        const int nz = emit(D_EQ_R, n, -1, -1, 256, 0, zero_const());
        const int z = zero_low ? emit(D_MUL_R, a, b, -1, 256)
                               : emit(D_LOADC, -1, -1, -1, 256, 0, zero_const());
        return emit(D_ITE, nz, z, r, 256);
    }

    std::vector<Piece> pieces_of(uint32_t k, uint32_t width) {
        const Val& v = (*vals_)[k];
        if (!v.wide()) return {Piece{vreg_of(k), width}};
        return v.pieces;
    }

    bool lower(std::vector<Val>& vals);
};

int arity(const mh_node& nd) {
    if (nd.op <= MH_OP_FALSE) return 0;
    if (nd.op == MH_OP_ITE || nd.op == MH_OP_EVM_ADDMOD || nd.op == MH_OP_EVM_MULMOD) return 3;
    if (nd.op == MH_OP_BVNEG || nd.op == MH_OP_BVNOT || nd.op == MH_OP_NOT ||
        nd.op == MH_OP_EXTRACT || nd.op == MH_OP_ZEXT || nd.op == MH_OP_SEXT ||
        nd.op == MH_OP_KECCAK)
        return 1;
    return 2;
}

bool Lowering::lower(std::vector<Val>& vals) {
    const size_t n = t.size();
    // operand validation (every node) and reachability from the root
    std::vector<char> live(n, 0);
    live[n - 1] = 1;
    for (size_t i = n; i-- > 0;) {
        const mh_node& nd = t[i];
        const int ar = arity(nd);
        const uint32_t ops[3] = {nd.a, nd.b, nd.c};
        for (int k = 0; k < ar; ++k) {
            if (ops[k] >= i) return fail("operand index not before node " + std::to_string(i));
            if (live[i]) live[ops[k]] = 1;
        }
    }
    vals.assign(n, Val());
    vals_ = &vals;
    if (hold_vars) {  // operand references per (column, width), live nodes
        for (size_t i = 0; i < n; ++i) {
            if (!live[i]) continue;
            const mh_node& nd = t[i];
            const int ar = arity(nd);
            const uint32_t ops[3] = {nd.a, nd.b, nd.c};
            for (int k = 0; k < ar; ++k) {
                const mh_node& o = t[ops[k]];
                if (o.op == MH_OP_VAR) ++uses_[(uint64_t)o.imm0 << 16 | o.width];
            }
        }
    }
    // evaluation order: post-order DFS from the root, operands with the larger Sethi-Ullman
    // register need first (the input order is only required to be topological)
    std::vector<uint32_t> need(n, 1);
    auto children = [&](size_t i, uint32_t* ch) -> int {
        const mh_node& nd = t[i];
        const int ar = arity(nd);
        const uint32_t ops[3] = {nd.a, nd.b, nd.c};
        for (int k = 0; k < ar; ++k) ch[k] = ops[k];
        // stable insertion sort of at most three (std::stable_sort allocates a buffer per call)
        for (int k = 1; k < ar; ++k)
            for (int j = k; j > 0 && need[ch[j]] > need[ch[j - 1]]; --j) std::swap(ch[j], ch[j - 1]);
        return ar;
    };
    for (size_t i = 0; i < n; ++i) {
        const mh_node& nd = t[i];
        if ((nd.op == MH_OP_VAR && pinned) || nd.op == MH_OP_CONST) { need[i] = 0; continue; }
        uint32_t ch[3];
        const int ar = children(i, ch);
        uint32_t m = 1;
        for (int k = 0; k < ar; ++k) m = std::max<uint32_t>(m, need[ch[k]] + (uint32_t)k);
        need[i] = m;
    }
    std::vector<uint32_t> order;
    order.reserve(n);
    {
        std::vector<char> seen(n, 0);
        std::vector<std::pair<uint32_t, bool>> st;
        st.push_back({(uint32_t)(n - 1), false});
        while (!st.empty()) {
            auto [x, done] = st.back();
            st.pop_back();
            if (done) { order.push_back(x); continue; }
            if (seen[x]) continue;
            seen[x] = 1;
            st.push_back({x, true});
            uint32_t ch[3];
            const int ar = children(x, ch);
            for (int k = ar - 1; k >= 0; --k)
                if (!seen[ch[k]]) st.push_back({ch[k], false});
        }
    }
    for (const uint32_t i : order) {
        const mh_node& nd = t[i];
        const uint32_t w = nd.width;
        if (w > 1088) return fail("width > 1088");
        auto V = [&](uint32_t k) -> const Val& { return vals[k]; };
        auto W = [&](uint32_t k) -> uint32_t { return t[k].width; };
        auto narrow = [&](uint32_t k) -> int { return vreg_of(k); };
        Val out;
        switch (nd.op) {
            case MH_OP_CONST: {
                if (nd.imm0 >= n_consts) return fail("const index out of range");
                if (w == 0 || w > 256) return fail("const width");
                out.remat = (int)i;
                break;
            }
            case MH_OP_VAR: {
                if (nd.imm0 >= n_vars) return fail("var column out of range");
                if (w == 0 || w > 256) return fail("var width");
                if (!pinned) {
                    features |= F_CPLX;
                    out.remat = (int)i;  // loaded at each use (vreg_of)
                    break;
                }
                out.vreg = masked((int)nd.imm0, w);  // a w-bit variable: low w bits of its column
                break;
            }
            case MH_OP_TRUE: case MH_OP_FALSE: out.remat = (int)i; break;
            case MH_OP_BVADD: case MH_OP_BVSUB: case MH_OP_BVMUL: case MH_OP_BVAND:
            case MH_OP_BVOR: case MH_OP_BVXOR: case MH_OP_BVUDIV: case MH_OP_BVUREM:
            case MH_OP_BVSDIV: case MH_OP_BVSREM: case MH_OP_BVSMOD: case MH_OP_EVM_EXP:
            case MH_OP_EVM_SIGNEXTEND: case MH_OP_EVM_BYTE: {
                if (V(nd.a).wide() || V(nd.b).wide() || w == 0 || w > 256 || W(nd.a) != w ||
                    W(nd.b) != w)
                    return fail("bit-vector op wider than 256 bits");
                uint8_t op = 0;
                bool mask = false;
                switch (nd.op) {
                    case MH_OP_BVADD: op = D_ADD_R; mask = true; break;
                    case MH_OP_BVSUB: op = D_SUB_R; mask = true; break;
                    case MH_OP_BVMUL: op = D_MUL_R; mask = true; break;
                    case MH_OP_BVAND: op = D_AND_R; break;
                    case MH_OP_BVOR: op = D_OR_R; break;
                    case MH_OP_BVXOR: op = D_XOR_R; break;
                    case MH_OP_BVUDIV: op = D_UDIV_R; mask = true; features |= F_DIV; break;
                    case MH_OP_BVUREM: op = D_UREM_R; features |= F_DIV; break;
                    case MH_OP_BVSDIV: op = D_SDIV_R; features |= F_DIV; break;
                    case MH_OP_BVSREM: op = D_SREM_R; features |= F_DIV; break;
                    case MH_OP_BVSMOD: op = D_SMOD_R; features |= F_DIV; break;
                    case MH_OP_EVM_EXP: op = D_EXP; features |= F_EVM; break;
                    case MH_OP_EVM_SIGNEXTEND: op = D_SIGNEXT; features |= F_EVM; break;
                    case MH_OP_EVM_BYTE: op = D_BYTE; features |= F_EVM; break;
                }
                if ((op == D_SIGNEXT || op == D_BYTE) && w != 256)
                    return fail("EVM word ops are 256-bit");
                if (jit && (op == D_SIGNEXT || op == D_BYTE || op == D_EXP)) {
                    out.vreg = op == D_SIGNEXT ? jit_signextend(nd.a, nd.b)
                               : op == D_BYTE  ? jit_byte(nd.a, nd.b)
                                               : jit_exp(nd.a, nd.b, w);
                    if (out.vreg < 0) return fail(err.empty() ? "EVM word op operand" : err);
                    break;
                }
                if (w < 256 && (op == D_SDIV_R || op == D_SREM_R || op == D_SMOD_R)) {
                    // signed division at width w = 256-bit signed division of the sign-extended
                    // operands, masked (all SMT-LIB sign cases agree mod 2^w)
                    out.vreg = masked(emit_sext_bin(op, nd.a, nd.b, w), w);
                    break;
                }
                int r = emit_bin(op, nd.a, nd.b, w);
                out.vreg = mask ? masked(r, w) : r;
                break;
            }
            case MH_OP_BVSHL: case MH_OP_BVLSHR: case MH_OP_BVASHR: {
                if (V(nd.a).wide() || V(nd.b).wide() || w == 0 || w > 256)
                    return fail("shift wider than 256");
                const mh_node& sn = t[nd.b];
                if (sn.op == MH_OP_CONST) {  // uniform shift amount
                    const uint32_t* lim = consts + 8ull * sn.imm0;
                    uint32_t hi = 0;
                    for (int k = 1; k < 8; ++k) hi |= lim[k] & lane_mask(k, sn.width);
                    uint32_t s = lim[0] & lane_mask(0, sn.width);
                    if (hi || s > 511) s = 511;
                    const int a = narrow(nd.a);
                    if (nd.op == MH_OP_BVASHR) {
                        out.vreg = s ? ashr_imm(a, s, w) : a;
                    } else if (s >= w) {
                        out.vreg = emit(D_LOADC, -1, -1, -1, 256, 0, zero_const());
                    } else if (s == 0) {
                        out.vreg = a;
                    } else if (nd.op == MH_OP_BVLSHR) {
                        out.vreg = shr_imm(a, s);
                    } else {
                        out.vreg = masked(shl_imm(a, s), w);
                    }
                } else {  // per-lane amount: 256-bit shifts of canonical / sign-extended values
                    const int a = narrow(nd.a), b = narrow(nd.b);
                    if (nd.op == MH_OP_BVSHL)
                        out.vreg = masked(emit(D_SHL_V, a, b, -1, 256), w);
                    else if (nd.op == MH_OP_BVLSHR)
                        out.vreg = emit(D_LSHR_V, a, b, -1, 256);
                    else
                        out.vreg = masked(emit(D_ASHR_V, sext256(a, w), b, -1, 256), w);
                }
                break;
            }
            case MH_OP_EVM_ADDMOD: case MH_OP_EVM_MULMOD: {
                if (w != 256 || W(nd.a) != 256 || W(nd.b) != 256 || W(nd.c) != 256 ||
                    nd.imm0 > 1)
                    return fail("ADDMOD / MULMOD take three 256-bit words");
                const int a = narrow(nd.a), b = narrow(nd.b), c = narrow(nd.c);
                if (a < 0 || b < 0 || c < 0) return fail("ADDMOD / MULMOD operand wider than 256");
                if (jit) {
                    out.vreg = nd.op == MH_OP_EVM_ADDMOD ? jit_addmod(a, b, c, nd.imm0 != 0)
                                                         : jit_mulmod(a, b, c, nd.imm0 != 0);
                    break;
                }
                features |= F_EVM;
                out.vreg = emit(nd.op == MH_OP_EVM_ADDMOD ? D_ADDMOD : D_MULMOD, a, b, c, 256,
                                nd.imm0);
                break;
            }
            case MH_OP_BVNEG: {
                const int a = narrow(nd.a);
                if (a < 0 || w == 0 || w > 256) return fail("unary op wider than 256");
                out.vreg = masked(emit(D_RSUB_R, a, -1, -1, w, 0, zero_const()), w);  // 0 - a
                break;
            }
            case MH_OP_BVNOT: {
                const int a = narrow(nd.a);
                if (a < 0 || w == 0 || w > 256) return fail("unary op wider than 256");
                out.vreg = emit(D_XOR_R, a, -1, -1, w, 0, mask_const(w));  // a ^ (2^w - 1)
                break;
            }
            case MH_OP_EQ: {
                const uint32_t wa = W(nd.a);
                if (wa != W(nd.b)) return fail("EQ sort mismatch");
                if (V(nd.a).wide() || V(nd.b).wide()) return fail("EQ wider than 256 bits");
                if (wa == 0) out.vreg = emit(D_BEQ, narrow(nd.a), narrow(nd.b), -1, 1);
                else out.vreg = emit_bin(D_EQ_R, nd.a, nd.b, wa);
                break;
            }
            case MH_OP_BVULT: case MH_OP_BVULE: case MH_OP_BVUGT: case MH_OP_BVUGE:
            case MH_OP_BVSLT: case MH_OP_BVSLE: case MH_OP_BVSGT: case MH_OP_BVSGE:
            case MH_OP_BVADD_NOOVFL_U: case MH_OP_BVMUL_NOOVFL_U: case MH_OP_BVSUB_NOUDFL_U: {
                const uint32_t wa = W(nd.a);
                if (V(nd.a).wide() || V(nd.b).wide() || wa == 0 || wa > 256 || W(nd.b) != wa)
                    return fail("compare wider than 256 bits");
                const bool full = wa == 256;
                uint8_t op = 0;
                switch (nd.op) {
                    case MH_OP_BVULT: op = D_ULT_R; break;
                    case MH_OP_BVULE: op = D_ULE_R; break;
                    case MH_OP_BVUGT: op = D_UGT_R; break;
                    case MH_OP_BVUGE: op = D_UGE_R; break;
                    case MH_OP_BVSLT: op = full ? D_SLT_R : D_ULT_R; break;
                    case MH_OP_BVSLE: op = full ? D_SLE_R : D_ULE_R; break;
                    case MH_OP_BVSGT: op = full ? D_SGT_R : D_UGT_R; break;
                    case MH_OP_BVSGE: op = full ? D_SGE_R : D_UGE_R; break;
                    case MH_OP_BVADD_NOOVFL_U: op = D_UADD_NOOVFL; features |= F_CPLX; break;
                    case MH_OP_BVMUL_NOOVFL_U: op = D_UMUL_NOOVFL; features |= F_CPLX; break;
                    case MH_OP_BVSUB_NOUDFL_U: op = D_UGE_R; break;  // b <= a
                }
                if (jit && (op == D_UADD_NOOVFL || op == D_UMUL_NOOVFL)) {
                    out.vreg = op == D_UADD_NOOVFL ? jit_add_noovfl(nd.a, nd.b, wa)
                                                   : jit_mul_noovfl(nd.a, nd.b, wa);
                    if (out.vreg < 0) return fail("overflow predicate operand");
                    break;
                }
                const bool narrow_signed = !full && (nd.op == MH_OP_BVSLT || nd.op == MH_OP_BVSLE ||
                                                     nd.op == MH_OP_BVSGT || nd.op == MH_OP_BVSGE);
                out.vreg = narrow_signed ? emit_scmp(op, nd.a, nd.b, wa) : emit_bin(op, nd.a, nd.b, wa);
                break;
            }
            case MH_OP_AND: case MH_OP_OR: case MH_OP_XOR: {
                if (W(nd.a) != 0 || W(nd.b) != 0) return fail("Bool op on bit-vectors");
                const uint8_t op = nd.op == MH_OP_AND ? D_BAND : nd.op == MH_OP_OR ? D_BOR : D_BXOR;
                out.vreg = emit(op, narrow(nd.a), narrow(nd.b), -1, 1);
                break;
            }
            case MH_OP_NOT: {
                if (W(nd.a) != 0) return fail("NOT on a bit-vector");
                out.vreg = emit(D_BNOT, narrow(nd.a), -1, -1, 1);
                break;
            }
            case MH_OP_ITE: {
                if (W(nd.a) != 0) return fail("ITE condition must be Bool");
                if (V(nd.b).wide() || V(nd.c).wide() || W(nd.b) != W(nd.c))
                    return fail("ITE wider than 256");
                const int c = narrow(nd.a), a = narrow(nd.b), b = narrow(nd.c);
                if (a < 0 || b < 0 || c < 0) return fail("ITE wider than 256");
                // generic select (cond, then, else); the accumulator pass picks the form
                out.vreg = emit(w == 0 ? D_BITE : D_ITE, c, a, b, w == 0 ? 1 : w);
                break;
            }
            case MH_OP_EXTRACT: {
                const uint32_t hi = nd.imm0, lo = nd.imm1, wa = W(nd.a);
                if (wa == 0 || lo > hi || hi >= wa || hi - lo + 1 != w) return fail("bad extract");
                if (!V(nd.a).wide()) {
                    out.vreg = extract(narrow(nd.a), lo, w, wa);
                    break;
                }
                if (w > 256) return fail("extract result wider than 256");
                // gather the parts of the pieces covering [lo, hi]
                const auto& ps = V(nd.a).pieces;
                uint32_t top = wa;  // bit just above the current piece
                int acc = -1;
                for (const Piece& p : ps) {
                    const uint32_t plo = top - p.bits, phi = top - 1;
                    top = plo;
                    if (phi < lo || plo > hi) continue;
                    const uint32_t elo = std::max(lo, plo) - plo, ehi = std::min(hi, phi) - plo;
                    const uint32_t pw = ehi - elo + 1;
                    const int part = extract(p.vreg, elo, pw, p.bits);
                    acc = acc < 0 ? part : concat(acc, part, pw);
                }
                out.vreg = acc;
                break;
            }
            case MH_OP_CONCAT: {
                const uint32_t wa = W(nd.a), wb = W(nd.b);
                if (wa == 0 || wb == 0 || wa + wb != w) return fail("bad concat");
                if (w <= 256) {
                    const int hi = narrow(nd.a);
                    if (is_const_node(nd.b))
                        out.vreg = emit(D_OR_R, shl_imm(hi, wb), -1, -1, 256, 0, const_of(nd.b));
                    else
                        out.vreg = concat(hi, narrow(nd.b), wb);
                } else {
                    out.pieces = pieces_of(nd.a, wa);
                    auto pb = pieces_of(nd.b, wb);
                    out.pieces.insert(out.pieces.end(), pb.begin(), pb.end());
                }
                break;
            }
            case MH_OP_ZEXT: {
                const uint32_t wa = W(nd.a);
                if (wa == 0 || wa + nd.imm0 != w) return fail("bad zero_extend");
                if (w <= 256) {
                    out.vreg = V(nd.a).vreg;  // canonical values: zero extension is free
                    out.remat = V(nd.a).remat;
                } else {
                    const int z = emit(D_LOADC, -1, -1, -1, 256, 0, zero_const());
                    uint32_t left = nd.imm0;
                    while (left) {
                        const uint32_t take = left > 256 ? 256 : left;
                        out.pieces.push_back(Piece{z, take});
                        left -= take;
                    }
                    auto pa = pieces_of(nd.a, wa);
                    out.pieces.insert(out.pieces.end(), pa.begin(), pa.end());
                }
                break;
            }
            case MH_OP_SEXT: {
                const uint32_t wa = W(nd.a);
                if (wa == 0 || wa + nd.imm0 != w || w > 256) return fail("sign_extend > 256");
                out.vreg = nd.imm0 ? masked(sext256(narrow(nd.a), wa), w) : narrow(nd.a);
                break;
            }
            case MH_OP_KECCAK: {
                const uint32_t wa = W(nd.a);
                if (wa == 0 || wa % 8 || w != 256) return fail("bad keccak input");
                auto ps = pieces_of(nd.a, wa);
                // merge into byte-aligned chunks of <= 256 bits
                std::vector<Piece> chunks;
                int cur = -1;
                uint32_t curw = 0;
                for (const Piece& p : ps) {
                    if (cur >= 0 && curw + p.bits <= 256) {
                        cur = concat(cur, p.vreg, p.bits);
                        curw += p.bits;
                    } else {
                        if (cur >= 0) {
                            if (curw % 8) return fail("keccak piece not byte aligned");
                            chunks.push_back(Piece{cur, curw});
                        }
                        cur = p.vreg;
                        curw = p.bits;
                    }
                }
                if (curw % 8) return fail("keccak piece not byte aligned");
                chunks.push_back(Piece{cur, curw});
                if (chunks.size() > 3) return fail("keccak input of more than 3 chunks");
                uint32_t total = 0;
                for (auto& ch : chunks) total += ch.bits / 8;
                if (total == 0 || total > 96) return fail("keccak input longer than 96 bytes");
                features |= F_KECCAK;
                // re-cut the message (big-endian bytes of the chunks, in order) into LEFT-aligned
                // 32-byte words and put the 0x01 pad byte in place, so the device absorbs whole
                // words at static state positions (exec.h keccak_words)
                const uint32_t nw = (total + 31) / 32;
                std::vector<int> words;
                for (uint32_t i = 0; i < nw; ++i) {
                    int word = -1;
                    uint32_t o = 0;
                    for (const Piece& ch : chunks) {
                        const uint32_t nb = ch.bits / 8;
                        if (o < 32 * i + 32 && o + nb > 32 * i) {
                            const int sh = (int)(32 * i + 32) - (int)(o + nb);  // bytes left
                            int part = ch.vreg;
                            if (sh > 0) part = shl_imm(part, 8u * (uint32_t)sh);
                            else if (sh < 0) part = shr_imm(part, 8u * (uint32_t)(-sh));
                            word = word < 0 ? part : emit(D_OR_R, word, part, -1);
                        }
                        o += nb;
                    }
                    words.push_back(word);
                }
                const uint32_t rem = total % 32;
                if (rem) {  // pad byte right after the message, inside the last word
                    uint32_t pad[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                    const uint32_t bit = 8 * (31 - rem);
                    pad[bit >> 5] = 1u << (bit & 31);
                    words.back() = emit(D_OR_R, words.back(), -1, -1, 256, 0,
                                        (int)const_index(pad, 256));
                }
                const uint32_t w1 = D_KECCAK | (nw << 8) | ((rem ? 0u : 1u) << 10);
                VInsn v{D_KECCAK, fresh(), words[0], nw > 1 ? words[1] : -1,
                        nw > 2 ? words[2] : -1, 256, 0, -1, w1};
                code.push_back(v);
                out.vreg = v.d;
                break;
            }
            default:
                return fail("unknown op " + std::to_string(nd.op));
        }
        if (!out.wide() && out.vreg < 0 && out.remat < 0)
            return fail("operand wider than 256 bits");
        vals[i] = std::move(out);
    }
    if (vals[n - 1].wide()) return fail("root wider than 256 bits");
    return true;
}

// Host machine for exec.h's step() over one instruction: x = R[0], y = R[1], third operand R[2],
// result in R[3] (the accumulator).  Folding runs the device's own instruction semantics, so a
// folded value is bit-identical to what the kernel would have computed in every lane.
struct FoldMachine {
    u32 R[4][8];
    u32 nrx() const { return 3; }
    void read(u32 r, u32* v) const { std::memcpy(v, R[r], 32); }
    u32 read0(u32 r) const { return R[r][0]; }
    void write(u32 r, const u32* v) { std::memcpy(R[r], v, 32); }
    void iconst(u32, u32* v) const { std::memcpy(v, R[1], 32); }
    void var(u32, u32* v) const { std::memset(v, 0, 32); }  // never reached: LOADVAR is not folded
};

bool bool_result(uint8_t op) {
    switch (op) {
        case D_EQ_R: case D_BAND: case D_BOR: case D_BXOR: case D_BEQ: case D_BNOT:
        case D_TRUE: case D_FALSE: case D_BITE: case D_UADD_NOOVFL: case D_UMUL_NOOVFL:
            return true;
        default:
            return op >= D_ULT_R && op <= D_SGE_C;
    }
}

// Constant folding and dead-code elimination on the lowered SSA code (before the accumulator
// pass).  An instruction whose operands are all known constants becomes a LOADC (TRUE / FALSE
// for a Bool) of its value; a select with a known condition becomes its chosen operand; a known
// y operand of an op with a *_C form becomes the inline constant (a known x of a commutative or
// mirrored op likewise, by swapping).  This is what z3's simplify does to mythril's constraints
// before any solver sees them (laser/smt/bitvec.py, `simplify` calls); nodes whose value does not
// depend on the assignment are not counted as per-evaluation work (compile_tape's alg_ops).
// Returns the root's register after aliasing; recomputes the feature bits.
int fold_constants(Lowering& L, int root_v, int value_numbering) {
    std::vector<VInsn>& code = L.code;
    const int nv = L.n_vregs;
    std::vector<char> known(nv, 0);
    std::vector<u32> val((size_t)nv * 8, 0u);
    std::vector<int> rep(nv);
    for (int r = 0; r < nv; ++r) rep[r] = r;
    auto R = [&](int r) { return r < 0 ? r : rep[r]; };
    auto K = [&](int r) { return r >= 0 && known[r]; };
    // value numbering (native code only: the interpreter's 15 registers rely on cheap shared
    // terms being duplicated, Sieve.rematerialize): an instruction with the same op, operands and
    // immediates as an earlier one is that one (every op is pure)
    std::unordered_map<std::string, int> seen_insn;
    auto set_bool = [&](VInsn& v, bool b) {
        known[v.d] = 1;
        u32* z = &val[(size_t)v.d * 8];
        for (int k = 0; k < 8; ++k) z[k] = 0;
        z[0] = b ? 1u : 0u;
        v = VInsn{b ? (uint8_t)D_TRUE : (uint8_t)D_FALSE, v.d, -1, -1, -1, 1, 0, -1, 0};
    };
    for (VInsn& v : code) {
        v.a = R(v.a);
        v.b = R(v.b);
        v.c = R(v.c);
        if (value_numbering && !(value_numbering == kVnNoLoads && v.op == D_LOADVAR)) {
            const int key[8] = {v.op, v.a, v.b, v.c, (int)v.width, (int)v.aux, v.cidx,
                                (int)v.w1raw};
            std::string k(reinterpret_cast<const char*>(key), sizeof(key));
            auto it = seen_insn.find(k);
            if (it != seen_insn.end()) {
                rep[v.d] = it->second;  // uses are renamed; the copy is dead code below
                continue;
            }
            seen_insn.emplace(std::move(k), v.d);
        }
        // identities of an op applied to one value twice (what z3's simplify does to x - x,
        // x ^ x, x & x, x == x, ...): the result is a constant or the operand itself
        if (v.cidx < 0 && v.a >= 0 && v.a == v.b) {
            switch (v.op) {
                case D_SUB_R: case D_RSUB_R: case D_XOR_R:
                    known[v.d] = 1;
                    std::memset(&val[(size_t)v.d * 8], 0, 32);
                    v = VInsn{D_LOADC, v.d, -1, -1, -1, 256, 0, L.zero_const(), 0};
                    continue;
                case D_AND_R: case D_OR_R: case D_BAND: case D_BOR:
                    rep[v.d] = v.a;
                    continue;
                case D_EQ_R: case D_ULE_R: case D_UGE_R: case D_SLE_R: case D_SGE_R: case D_BEQ:
                    set_bool(v, true);
                    continue;
                case D_ULT_R: case D_UGT_R: case D_SLT_R: case D_SGT_R: case D_BXOR:
                    set_bool(v, false);
                    continue;
                default:
                    break;
            }
        }
        if ((v.op == D_ITE || v.op == D_BITE) && v.b >= 0 && v.b == v.c) {  // (cond, t, t)
            rep[v.d] = v.b;
            continue;
        }
        const uint8_t op = v.op;
        if (op == D_LOADC) {
            known[v.d] = 1;
            std::memcpy(&val[(size_t)v.d * 8], L.pool.data() + 8ull * (uint32_t)v.cidx, 32);
            continue;
        }
        if (op == D_TRUE || op == D_FALSE) {
            known[v.d] = 1;
            val[(size_t)v.d * 8] = op == D_TRUE ? 1u : 0u;
            continue;
        }
        if (op == D_LOADVAR || op == D_KECCAK) continue;
        if (op == D_ITE || op == D_BITE) {  // (cond a, then b, else c)
            if (K(v.a)) rep[v.d] = (val[(size_t)v.a * 8] & 1u) ? v.b : v.c;
            continue;
        }
        const bool ka = v.a < 0 || K(v.a);
        const bool kb = v.cidx >= 0 || v.b < 0 || K(v.b);
        const bool kc = v.c < 0 || K(v.c);
        if (ka && kb && kc && v.aux <= MH_AUX_MAX) {
            FoldMachine m;
            std::memset(m.R, 0, sizeof(m.R));
            if (v.a >= 0) std::memcpy(m.R[0], &val[(size_t)v.a * 8], 32);
            if (v.cidx >= 0)
                std::memcpy(m.R[1], L.pool.data() + 8ull * (uint32_t)v.cidx, 32);
            else if (v.b >= 0)
                std::memcpy(m.R[1], &val[(size_t)v.b * 8], 32);
            if (v.c >= 0) std::memcpy(m.R[2], &val[(size_t)v.c * 8], 32);
            const u32 w1 = op | ((v.width & 0x1FFu) << 8) | (v.aux << 17);
            step<F_CPLX | F_KECCAK | F_EVM | F_DIV, true>(m, 0u | 1u << 8 | 3u << 16 | 2u << 24,
                                                           w1, 0u);
            u32* z = &val[(size_t)v.d * 8];
            std::memcpy(z, m.R[3], 32);
            known[v.d] = 1;
            if (bool_result(op)) {
                z[0] &= 1u;
                for (int k = 1; k < 8; ++k) z[k] = 0;
                v = VInsn{z[0] ? (uint8_t)D_TRUE : (uint8_t)D_FALSE, v.d, -1, -1, -1, 1, 0, -1, 0};
            } else {
                v = VInsn{D_LOADC, v.d, -1, -1, -1, 256, 0, (int)L.const_index(z, 256), 0};
            }
            continue;
        }
        // a known operand of a pair op becomes the inline constant
        if (v.cidx < 0 && v.b >= 0 && y_const_ok(op) && op < D_FIRST_COMPLEX) {
            if (K(v.b)) {
                v.cidx = (int)L.const_index(&val[(size_t)v.b * 8], 256);
                v.b = -1;
            } else if (K(v.a) && (commutes(op) || mirror(op))) {
                if (!commutes(op)) v.op = mirror(op);
                v.cidx = (int)L.const_index(&val[(size_t)v.a * 8], 256);
                v.a = v.b;
                v.b = -1;
            }
        }
    }
    root_v = R(root_v);
    // dead code: everything the root does not read (every op is pure)
    std::vector<char> used(nv, 0);
    used[root_v] = 1;
    std::vector<char> keep(code.size(), 0);
    for (size_t i = code.size(); i-- > 0;) {
        const VInsn& v = code[i];
        if (!used[v.d]) continue;
        keep[i] = 1;
        for (int r : {v.a, v.b, v.c})
            if (r >= 0) used[r] = 1;
    }
    std::vector<VInsn> live;
    live.reserve(code.size());
    uint32_t feats = 0;
    for (size_t i = 0; i < code.size(); ++i) {
        if (!keep[i]) continue;
        const uint8_t op = code[i].op;
        if (op >= D_UDIV_R && op <= D_SMOD_C) feats |= F_DIV;
        else if (op == D_KECCAK) feats |= F_KECCAK;
        else if (op == D_EXP || op == D_SIGNEXT || op == D_BYTE || op == D_ADDMOD ||
                 op == D_MULMOD)
            feats |= F_EVM;
        else if (op >= D_FIRST_COMPLEX) feats |= F_CPLX;
        live.push_back(code[i]);
    }
    code.swap(live);
    L.features = feats;
    return root_v;
}

}  // namespace

void sample_bools(const SsaTape& st, const std::vector<uint32_t>& pool, uint32_t n_rows,
                  uint64_t seed, const std::vector<int>& want,
                  std::vector<std::vector<uint8_t>>& out) {
    out.assign(want.size(), std::vector<uint8_t>(n_rows, 0));
    std::vector<u32> val((size_t)st.n_vregs * 8, 0u);
    uint64_t s = seed;
    auto next = [&]() {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    };
    for (uint32_t r = 0; r < n_rows; ++r) {
        for (int c = 0; c < st.n_pinned; ++c)
            for (int k = 0; k < 8; k += 2) {
                const uint64_t x = next();
                val[(size_t)c * 8 + k] = (u32)x;
                val[(size_t)c * 8 + k + 1] = (u32)(x >> 32);
            }
        for (const SsaInsn& v : st.code) {
            FoldMachine m;
            std::memset(m.R, 0, sizeof(m.R));
            auto ld = [&](int slot, int reg) {
                if (reg >= 0) std::memcpy(m.R[slot], &val[(size_t)reg * 8], 32);
            };
            if (v.op == D_ITE) {  // SSA select (a = cond, b = then, c = else) -> step's D_ITE
                ld(0, v.b);
                ld(1, v.a);
                ld(2, v.c);
            } else {
                ld(0, v.a);
                if (v.cidx >= 0) std::memcpy(m.R[1], pool.data() + 8ull * (uint32_t)v.cidx, 32);
                else ld(1, v.b);
                ld(2, v.c);
            }
            if (v.op == D_LOADC) {
                std::memcpy(m.R[3], pool.data() + 8ull * (uint32_t)v.cidx, 32);
            } else if (v.op == D_LOADVAR) {  // a column not pinned: uniform too, per (row, column)
                uint64_t h = seed ^ (0xD1B54A32D192ED03ull * (r + 1)) ^ (0x8CB92BA72F3D8DD7ull * (v.aux + 1));
                for (int k = 0; k < 8; ++k) {
                    h += 0x9E3779B97F4A7C15ull;
                    uint64_t z = h;
                    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
                    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
                    m.R[3][k] = (u32)(z ^ (z >> 31));
                }
            }
            else {
                const u32 w1 = v.op == D_KECCAK ? v.w1raw
                                                : (v.op | ((v.width & 0x1FFu) << 8) | (v.aux << 17));
                step<F_CPLX | F_KECCAK | F_EVM | F_DIV, true>(m, 0u | 1u << 8 | 3u << 16 | 2u << 24,
                                                               w1, 0u);
            }
            std::memcpy(&val[(size_t)v.d * 8], m.R[3], 32);
        }
        for (size_t i = 0; i < want.size(); ++i)
            out[i][r] = want[i] >= 0 ? (uint8_t)(val[(size_t)want[i] * 8] & 1u) : 0;
    }
}

namespace {

// z3's form of the yellow-paper ADDMOD / MULMOD (what LASER would build with exact semantics, and
// what a z3 term carries into the SMT-LIB reader):
//     extract[255:0](bvurem(zext256(a) op zext256(b), zext256(n)))      op = bvadd / bvmul
// becomes MH_OP_EVM_ADDMOD / MULMOD(a, b, n) with imm0 = 1 (n == 0: bvurem returns the 512-bit
// dividend, whose low 256 bits are a op b), so the 512-bit intermediates never reach the device.
// The node keeps its index; the wide nodes it no longer reads become dead.
void rewrite_wide_modops(std::vector<mh_node>& t) {
    auto zext256 = [&](uint32_t k, uint32_t* inner) {
        const mh_node& z = t[k];
        if (z.op != MH_OP_ZEXT || z.width != 512 || z.imm0 != 256 || z.a >= k ||
            t[z.a].width != 256)
            return false;
        *inner = z.a;
        return true;
    };
    for (size_t i = 0; i < t.size(); ++i) {
        mh_node& e = t[i];
        if (e.op != MH_OP_EXTRACT || e.imm0 != 255 || e.imm1 != 0 || e.width != 256 || e.a >= i)
            continue;
        const mh_node& r = t[e.a];
        if (r.op != MH_OP_BVUREM || r.width != 512 || r.a >= e.a || r.b >= e.a) continue;
        const mh_node& s = t[r.a];
        if ((s.op != MH_OP_BVADD && s.op != MH_OP_BVMUL) || s.width != 512 || s.a >= r.a ||
            s.b >= r.a)
            continue;
        uint32_t a, b, n;
        if (!zext256(s.a, &a) || !zext256(s.b, &b) || !zext256(r.b, &n)) continue;
        const uint8_t op = s.op == MH_OP_BVADD ? MH_OP_EVM_ADDMOD : MH_OP_EVM_MULMOD;
        e = mh_node{};
        e.op = op;
        e.width = 256;
        e.a = a;
        e.b = b;
        e.c = n;
        e.imm0 = 1;
    }
}

}  // namespace

int32_t lower_tape_ssa(const mh_node* nodes, size_t n_nodes, const uint32_t* consts,
                       uint32_t n_consts, uint32_t n_vars, std::vector<uint32_t>& dconsts,
                       ConstIndex& dconst_index, SsaTape& st,
                       std::string& err, int value_numbering, bool jit_forms, bool hold_vars) {
    if (n_nodes == 0) {
        err = "empty tape";
        return MH_E_INVALID;
    }
    std::vector<mh_node> t(nodes, nodes + n_nodes);
    rewrite_wide_modops(t);
    Lowering L(t, consts, n_consts, n_vars, dconsts, dconst_index);
    L.jit = jit_forms;
    L.hold_vars = hold_vars;
    std::vector<Val> vals;
    if (!L.lower(vals)) {
        err = L.err;
        return MH_E_UNSUPPORTED;
    }
    // algorithmic work per evaluation: the nodes whose value depends on the assignment (the
    // others are folded to constants on the host, fold_constants)
    st.alg_ops = 0;
    std::vector<char> dep(n_nodes, 0);
    for (size_t i = 0; i < n_nodes; ++i) {
        const mh_node& nd = t[i];
        if (nd.op == MH_OP_VAR) { dep[i] = 1; continue; }
        const int ar = arity(nd);
        const uint32_t ops[3] = {nd.a, nd.b, nd.c};
        for (int k = 0; k < ar; ++k) dep[i] |= dep[ops[k]];
        if (dep[i]) st.alg_ops += op_cost(nd, t);
    }
    // root: X after the last instruction must hold it
    int root_v = L.vreg_of((uint32_t)(n_nodes - 1));
    if (root_v < 0) {
        err = "root wider than 256 bits";
        return MH_E_UNSUPPORTED;
    }
    if (!std::getenv("MH_NO_FOLD")) root_v = fold_constants(L, root_v, value_numbering);
    st.code.swap(L.code);
    st.root = root_v;
    st.n_vregs = L.n_vregs;
    st.n_pinned = L.pinned ? (int)n_vars : 0;
    st.features = L.features;
    st.root_bool = t.back().width == 0;
    return MH_OK;
}

namespace {

// Cheap shared sub-terms (at most max_size nodes, no multiply / divide / keccak / exp) duplicated
// at every use instead of kept live: a path condition reads the same calldata bytes in several
// overlapping words (calldata.py:48-54: word(0) and word(4) share 28 byte terms), which otherwise
// holds more values live than the register file has; the copies cost a few cheap instructions.
std::vector<mh_node> rematerialize(const mh_node* t, size_t n, uint32_t max_size) {
    std::vector<uint32_t> uses(n, 0), size(n, 0);
    std::vector<char> cheap(n, 0), dup(n, 0);
    for (size_t i = 0; i < n; ++i) {
        const mh_node& nd = t[i];
        const int ar = arity(nd);
        const uint32_t ops[3] = {nd.a, nd.b, nd.c};
        uint64_t sz = 1;
        bool ok = nd.width <= 256;
        for (int k = 0; k < ar; ++k) {
            ++uses[ops[k]];
            sz += size[ops[k]];
            ok = ok && cheap[ops[k]];
        }
        size[i] = (uint32_t)std::min<uint64_t>(sz, 1u << 30);
        switch (nd.op) {
            case MH_OP_BVMUL: case MH_OP_BVUDIV: case MH_OP_BVUREM: case MH_OP_BVSDIV:
            case MH_OP_BVSREM: case MH_OP_BVSMOD: case MH_OP_KECCAK: case MH_OP_EVM_EXP:
            case MH_OP_BVMUL_NOOVFL_U: case MH_OP_EVM_ADDMOD: case MH_OP_EVM_MULMOD:
                ok = false;
                break;
            default:
                break;
        }
        cheap[i] = ok && size[i] <= max_size;
    }
    for (size_t i = 0; i < n; ++i) dup[i] = cheap[i] && uses[i] > 1;
    std::vector<mh_node> out;
    std::vector<uint32_t> remap(n, 0);
    // inside a duplicated sub-term every cheap node is copied too, so copies share nothing
    // (a recursive lambda called through itself: no std::function per call)
    auto copy = [&](auto&& self, uint32_t k, bool deep) -> uint32_t {
        mh_node nd = t[k];
        const int ar = arity(nd);
        uint32_t* ops[3] = {&nd.a, &nd.b, &nd.c};
        for (int j = 0; j < ar; ++j) {
            const uint32_t x = *ops[j];
            *ops[j] = (cheap[x] && (deep || dup[x])) ? self(self, x, true) : remap[x];
        }
        out.push_back(nd);
        return (uint32_t)(out.size() - 1);
    };
    for (size_t i = 0; i < n; ++i) {
        if (dup[i] && i != n - 1) continue;
        remap[i] = copy(copy, (uint32_t)i, false);
    }
    return out;
}

int32_t compile_tape_once(const mh_node* nodes, size_t n_nodes, const uint32_t* consts,
                          uint32_t n_consts, uint32_t n_vars, std::vector<uint32_t>& dconsts,
                          ConstIndex& dconst_index,
                          std::vector<uint32_t>& words, CompiledTape& out, std::string& err,
                          bool hold_vars, bool sc);

}  // namespace

// A tape that runs out of registers is retried without held columns (Lowering::hold_vars), then
// with cheap shared sub-terms duplicated at their uses, widening what counts as cheap (8, 32, 256
// nodes) -- each size first with held columns, then without; and each of those first with the
// short-circuit order (short_circuit), then, if that runs out of registers, in the order as
// lowered, whose live ranges may fit where the reordered ones do not.
// The attempt that fitted the last tape compiled on this thread is tried first: a LASER query's
// tapes grow by one conjunct per query (svm.py:257-262), and a long path's tape needs the same
// rematerialisation as its parent's, so the attempts that ran out of registers for the parent are
// not repeated for every child (the code differs, the values do not).
int32_t compile_tape(const mh_node* nodes, size_t n_nodes, const uint32_t* consts,
                     uint32_t n_consts, uint32_t n_vars, std::vector<uint32_t>& dconsts,
                     ConstIndex& dconst_index,
                     std::vector<uint32_t>& words, CompiledTape& out, std::string& err) {
    static thread_local int hint = 0;  // index into the attempt list of the last success
    const bool hold = n_vars > MH_MAX_PRELOAD && !std::getenv("MH_NO_HOLD_VARS");
    static const uint32_t kSizes[4] = {0u, 8u, 32u, 256u};
    std::vector<int> order;  // a = 4 * size index + 2 * (no hold) + (no short circuit)
    for (int a = 0; a < 16; ++a)
        if (!((a & 2) == 0 && !hold)) order.push_back(a);
    auto it = std::find(order.begin(), order.end(), hint);
    if (it != order.end()) std::rotate(order.begin(), it, it + 1);  // the hint first, then in order
    int32_t r = MH_E_UNSUPPORTED;
    const size_t words0 = words.size(), dconsts0 = dconsts.size();
    for (int a : order) {
        const uint32_t sz = kSizes[a >> 2];
        const bool h = (a & 2) == 0, sc = (a & 1) == 0;
        std::vector<mh_node> t2;
        if (sz) t2 = rematerialize(nodes, n_nodes, sz);
        const mh_node* tn = sz ? t2.data() : nodes;
        const size_t nn = sz ? t2.size() : n_nodes;
        err.clear();
        words.resize(words0);  // a failed attempt leaves nothing behind
        if (dconsts.size() != dconsts0) {
            dconsts.resize(dconsts0);
            for (auto i = dconst_index.begin(); i != dconst_index.end();)
                i = i->second >= dconsts0 / 8 ? dconst_index.erase(i) : std::next(i);
        }
        r = compile_tape_once(tn, nn, consts, n_consts, n_vars, dconsts, dconst_index, words, out,
                              err, h, sc);
        out.n_nodes = (uint32_t)n_nodes;
        if (r != MH_E_UNSUPPORTED || err.find("register pressure") == std::string::npos) {
            if (r == MH_OK) hint = a;
            return r;
        }
    }
    return r;
}

namespace {

// Short-circuit conjunctions of the interpreter (the native code orders its own, jit.cpp): the
// root's AND chain -- the BANDs reachable from the root through single-use BANDs -- is flattened
// and emitted again conjunct by conjunct: each conjunct's cone (the instructions it needs that no
// earlier conjunct emitted, in their lowered order) just before the AND that takes it in, every
// AND but the last a D_BANDZ, where a wave with no lane left true leaves the tape (its root is 0
// in every lane).  Newest conjunct first: a LASER query's tape is its parent's conjunction and the
// new constraint (svm.py:257-262), the conjunct that rows guided by the parent's witness are the
// least likely to satisfy.  MH_INTERP_SC=0 keeps the tape as lowered, =given the conjuncts' order.
// Counts, first witnesses and root values are those of the tape as lowered.
void short_circuit(SsaTape& st) {
    static const int mode = [] {
        const char* e = std::getenv("MH_INTERP_SC");
        return !e ? 2 : std::strcmp(e, "0") == 0 ? 0 : std::strcmp(e, "given") == 0 ? 1 : 2;
    }();
    if (!mode || !st.root_bool || st.root < 0) return;
    std::vector<SsaInsn>& code = st.code;
    const int n = (int)code.size();
    std::vector<int> def(st.n_vregs, -1), uses(st.n_vregs, 0);
    for (int i = 0; i < n; ++i) {
        def[code[i].d] = i;
        for (int r : {code[i].a, code[i].b, code[i].c})
            if (r >= 0) ++uses[r];
    }
    if (def[st.root] < 0 || code[def[st.root]].op != D_BAND) return;
    std::vector<char> chain(n, 0), is_conj(st.n_vregs, 0);
    std::vector<int> conj, stack{st.root};
    while (!stack.empty()) {
        const int r = stack.back();
        stack.pop_back();
        const int i = def[r];
        if (i >= 0 && code[i].op == D_BAND && code[i].cidx < 0 && code[i].b >= 0 &&
            (r == st.root || uses[r] == 1)) {
            chain[i] = 1;
            stack.push_back(code[i].b);
            stack.push_back(code[i].a);
        } else if (!is_conj[r]) {
            is_conj[r] = 1;
            conj.push_back(r);
        }
    }
    if (conj.size() < 2) return;
    if (mode == 2) std::reverse(conj.begin(), conj.end());
    std::vector<SsaInsn> out;
    out.reserve(code.size() + conj.size());
    std::vector<char> emitted(n, 0);
    int acc = -1;
    for (size_t k = 0; k < conj.size(); ++k) {
        std::vector<int> cone;
        if (def[conj[k]] >= 0 && !emitted[def[conj[k]]]) {
            stack.assign(1, def[conj[k]]);
            emitted[def[conj[k]]] = 1;
            while (!stack.empty()) {
                const int i = stack.back();
                stack.pop_back();
                if (chain[i]) return;  // a chain AND read inside a conjunct: keep the tape
                cone.push_back(i);
                for (int r : {code[i].a, code[i].b, code[i].c}) {
                    if (r < 0 || def[r] < 0 || emitted[def[r]]) continue;
                    emitted[def[r]] = 1;
                    stack.push_back(def[r]);
                }
            }
            std::sort(cone.begin(), cone.end());
        }
        for (int i : cone) out.push_back(code[i]);
        const bool last = k + 1 == conj.size();
        const int d = st.n_vregs++;
        // the first conjunct is tested alone (x & x)
        out.push_back(SsaInsn{last ? (uint8_t)D_BAND : (uint8_t)D_BANDZ, d, k ? acc : conj[k],
                              conj[k], -1, 1, 0, -1, 0});
        acc = d;
    }
    size_t n_chain = 0;
    for (int i = 0; i < n; ++i) n_chain += chain[i];
    if (out.size() != code.size() - n_chain + conj.size()) return;  // something outside: keep
    code.swap(out);
    st.root = acc;
}

int32_t compile_tape_once(const mh_node* nodes, size_t n_nodes, const uint32_t* consts,
                          uint32_t n_consts, uint32_t n_vars, std::vector<uint32_t>& dconsts,
                          ConstIndex& dconst_index,
                          std::vector<uint32_t>& words, CompiledTape& out, std::string& err,
                          bool hold_vars, bool sc) {
    SsaTape st;
    if (int32_t r = lower_tape_ssa(nodes, n_nodes, consts, n_consts, n_vars, dconsts,
                                   dconst_index, st, err, 0, false, hold_vars))
        return r;
    out.alg_ops = st.alg_ops;
    out.n_nodes = (uint32_t)n_nodes;
    if (sc) short_circuit(st);
    std::vector<VInsn>& code = st.code;
    const int n_pinned = st.n_pinned;
    int root_v = st.root;
    if (code.empty() || code.back().d != root_v)
        code.push_back(VInsn{D_NOP, st.n_vregs++, root_v, -1, -1, 256, 0, -1, 0});
    out.features = st.features;

    // ---- accumulator pass: which operand each instruction finds in X ----
    std::vector<char> lda(code.size(), 0);
    int acc = -1;
    for (size_t i = 0; i < code.size(); ++i) {
        VInsn& v = code[i];
        int prim = v.a;  // operand that goes through X
        switch (v.op) {
            case D_LOADC: case D_LOADVAR: case D_TRUE: case D_FALSE:
                prim = -1;
                break;
            case D_ITE: {  // generic select from lowering: a = cond, b = then, c = else
                const int cnd = v.a, thn = v.b;
                if (acc == cnd && thn != cnd) {
                    v.op = D_ITEC;  // X = cond, R[b] = then
                } else {
                    v.op = D_ITE;  // X = then, R[b] = cond
                    v.a = thn;
                    v.b = cnd;
                }
                prim = v.a;
                break;
            }
            case D_BITE:  // X = cond, R[b] = then, R[c] = else
                break;
            default:
                if (v.cidx < 0 && v.b >= 0 && acc == v.b && acc != v.a) {
                    if (commutes(v.op)) {
                        std::swap(v.a, v.b);
                    } else if (uint8_t mo = mirror(v.op)) {
                        v.op = mo;
                        std::swap(v.a, v.b);
                    }
                }
                prim = v.a;
                break;
        }
        if (prim >= 0 && acc != prim) lda[i] = 1;
        acc = v.d;
    }
    // register uses: loads of the first operand (LDA), y operands, the third operand
    const int nv = st.n_vregs;
    std::vector<int> last_use(nv, -1);
    std::vector<char> needs_reg(nv, 0);
    for (int r = 0; r < n_pinned; ++r) needs_reg[r] = 1;
    auto reg_use = [&](int r, int i) {
        if (r < 0) return;
        last_use[r] = std::max(last_use[r], i);
        needs_reg[r] = 1;
    };
    for (int i = 0; i < (int)code.size(); ++i) {
        const VInsn& v = code[i];
        if (lda[i]) reg_use(v.a, i);
        if (v.cidx < 0) reg_use(v.b, i);
        reg_use(v.c, i);
    }
    // ---- linear-scan allocation of the written-back values ----
    std::vector<int> phys(nv, -1);
    for (int r = 0; r < n_pinned; ++r) phys[r] = r;
    std::vector<int> free_regs;
    for (int r = MH_NR_MAX - 1; r >= n_pinned; --r) free_regs.push_back(r);
    std::vector<char> wb(code.size(), 0);
    int peak = n_pinned;  // highest register index used + 1
    for (int i = 0; i < (int)code.size(); ++i) {
        const VInsn& v = code[i];
        const int ops[3] = {lda[i] ? v.a : -1, v.cidx >= 0 ? -1 : v.b, v.c};
        for (int k = 0; k < 3; ++k) {
            const int r = ops[k];
            if (r < n_pinned) continue;
            bool dup = false;
            for (int j = 0; j < k; ++j) dup |= ops[j] == r;
            if (!dup && last_use[r] == i) free_regs.push_back(phys[r]);
        }
        if (!needs_reg[v.d]) continue;
        if (free_regs.empty()) {
            err = "register pressure exceeds " + std::to_string(MH_NR_MAX) + " registers";
            return MH_E_UNSUPPORTED;
        }
        // lowest free register keeps small tapes in the small-register kernel
        auto it = std::min_element(free_regs.begin(), free_regs.end());
        phys[v.d] = *it;
        free_regs.erase(it);
        peak = std::max(peak, phys[v.d] + 1);
        wb[i] = 1;
    }
    const uint32_t nrx = mh_nrx_of((uint32_t)peak);
    out.n_regs = (uint32_t)std::max(peak, 1);
    out.root_bool = st.root_bool;

    // ---- encode + slot layout ----
    std::vector<uint32_t> slots;  // pairs (w0, w1)
    auto put = [&](uint32_t w0, uint32_t w1) {
        slots.push_back(w0);
        slots.push_back(w1);
    };
    auto pos = [&]() { return (uint32_t)(slots.size() / 2); };
    // D_LOADVAR names the NEXT column the tape loads in its b | c << 8 fields (0xffff: none): the
    // asm core prefetches it while the instructions in between run (gen_asm_core.py LOADVAR)
    int64_t last_lv = -1;
    for (size_t i = 0; i < code.size(); ++i) {
        const VInsn& v = code[i];
        auto P = [&](int r) -> uint32_t { return (r < 0 || phys[r] < 0) ? 0u : (uint32_t)phys[r]; };
        const uint32_t a = lda[i] ? P(v.a) : nrx;
        const uint32_t d = wb[i] ? P(v.d) : nrx;
        const uint32_t b = v.cidx >= 0 ? 0u : P(v.b);
        const uint32_t c = P(v.c);
        uint32_t op = v.op;
        uint32_t w1;
        if (v.op == D_KECCAK) {
            w1 = v.w1raw;
        } else {
            if (v.aux > MH_AUX_MAX) {
                err = "immediate exceeds 14 bits";
                return MH_E_UNSUPPORTED;
            }
            if (v.cidx >= 0 && op < D_FIRST_COMPLEX && op != D_LOADC) op += 1;  // *_C form
            // first operand already in X and no write-back: the X form (a' = d' = X)
            if (op < D_FIRST_COMPLEX && a == nrx && d == nrx && mh_xform(op) &&
                xform_enabled(op))
                op = mh_xform(op);
            w1 = op | ((v.width & 0x1FFu) << 8) | (v.aux << 17);
            if (v.cidx >= 0 && op >= D_FIRST_COMPLEX) w1 |= F_YC;
        }
        const uint32_t len = v.cidx >= 0 ? 5u : 1u;
        if (pos() % MH_WINDOW + len > MH_WINDOW - 1) {  // keep the last slot for D_WINDOW
            put(0, D_WINDOW);
            while (pos() % MH_WINDOW) put(0, 0);
        }
        if (v.op == D_LOADVAR) {
            if (last_lv >= 0) {  // the previous LOADVAR prefetches this column
                uint32_t& pw0 = slots[2 * (size_t)last_lv];
                pw0 = (pw0 & 0x00FF00FFu) | ((v.aux & 0xFFu) << 8) | ((v.aux >> 8) << 24);
            }
            last_lv = pos();
            put(a | (0xFFu << 8) | (d << 16) | (0xFFu << 24), w1);
        } else {
            put(a | (b << 8) | (d << 16) | (c << 24), w1);
        }
        if (v.cidx >= 0) {
            const uint32_t* lim = dconsts.data() + 8ull * (uint32_t)v.cidx;
            for (int k = 0; k < 4; ++k) put(lim[2 * k], lim[2 * k + 1]);
        }
    }
    put(0, D_END);
    out.n_insns = pos();
    words.insert(words.end(), slots.begin(), slots.end());
    return MH_OK;
}

}  // namespace

static int ir_arity(uint8_t op) {
    switch (op) {
        case MH_OP_CONST: case MH_OP_VAR: case MH_OP_TRUE: case MH_OP_FALSE: return 0;
        case MH_OP_BVNEG: case MH_OP_BVNOT: case MH_OP_NOT: case MH_OP_EXTRACT: case MH_OP_ZEXT:
        case MH_OP_SEXT: case MH_OP_KECCAK: return 1;
        case MH_OP_ITE: case MH_OP_EVM_ADDMOD: case MH_OP_EVM_MULMOD: return 3;
        default: return 2;
    }
}

// compile.h split_conjunction
bool split_conjunction(const mh_node* nd, uint32_t n, uint32_t want,
                       std::vector<std::vector<mh_node>>& out) {
    std::vector<uint32_t> conj, st{n - 1};
    while (!st.empty()) {  // the root's AND chain, left to right
        const uint32_t u = st.back();
        st.pop_back();
        if (nd[u].op == MH_OP_AND && nd[u].width == 0 && nd[u].a < u && nd[u].b < u) {
            st.push_back(nd[u].b);
            st.push_back(nd[u].a);
        } else {
            conj.push_back(u);
        }
    }
    if (conj.size() < 2 || want < 2) return false;
    std::vector<uint32_t> mark(n, 0), cone(conj.size(), 0);
    uint32_t stamp = 0;
    auto reach = [&](uint32_t root, uint32_t s, std::vector<uint32_t>* keep) {
        uint32_t cnt = 0;
        std::vector<uint32_t> stk{root};
        while (!stk.empty()) {
            const uint32_t u = stk.back();
            stk.pop_back();
            if (u >= n || mark[u] == s) continue;
            mark[u] = s;
            ++cnt;
            if (keep) keep->push_back(u);
            const int k = ir_arity(nd[u].op);
            if (k >= 1) stk.push_back(nd[u].a);
            if (k >= 2) stk.push_back(nd[u].b);
            if (k >= 3) stk.push_back(nd[u].c);
        }
        return cnt;
    };
    uint64_t total = 0;
    for (size_t i = 0; i < conj.size(); ++i) total += cone[i] = reach(conj[i], ++stamp, nullptr);
    const uint32_t parts = std::min<uint32_t>(want, (uint32_t)conj.size());
    out.clear();
    size_t i = 0;
    for (uint32_t p = 0; p < parts && i < conj.size(); ++p) {
        // consecutive conjuncts up to this part's share of what is left
        const uint64_t left = std::accumulate(cone.begin() + (long)i, cone.end(), (uint64_t)0);
        const uint64_t share = (left + (parts - p) - 1) / (parts - p);
        const size_t rest_parts = parts - p - 1;
        std::vector<uint32_t> mine;
        uint64_t sum = 0;
        while (i < conj.size() && (mine.empty() || (sum < share && conj.size() - i > rest_parts))) {
            sum += cone[i];
            mine.push_back(conj[i++]);
        }
        if (p + 1 == parts)
            while (i < conj.size()) mine.push_back(conj[i++]);
        std::vector<uint32_t> keep;
        ++stamp;
        for (uint32_t r : mine) reach(r, stamp, &keep);
        std::sort(keep.begin(), keep.end());
        std::vector<uint32_t> idx(n, UINT32_MAX);
        std::vector<mh_node> tp;
        tp.reserve(keep.size() + mine.size());
        for (uint32_t u : keep) {
            mh_node x = nd[u];
            const int k = ir_arity(x.op);
            if (k >= 1) x.a = idx[x.a];
            if (k >= 2) x.b = idx[x.b];
            if (k >= 3) x.c = idx[x.c];
            idx[u] = (uint32_t)tp.size();
            tp.push_back(x);
        }
        uint32_t acc = idx[mine[0]];
        for (size_t j = 1; j < mine.size(); ++j) {
            mh_node a{};
            a.op = MH_OP_AND;
            a.width = 0;
            a.a = acc;
            a.b = idx[mine[j]];
            acc = (uint32_t)tp.size();
            tp.push_back(a);
        }
        if (acc != tp.size() - 1) {  // a lone conjunct that is not its cone's last node
            mh_node a{};
            a.op = MH_OP_AND;
            a.a = acc;
            a.b = acc;
            tp.push_back(a);
        }
        out.push_back(std::move(tp));
    }
    return out.size() >= 2;
}


}  // namespace mh
