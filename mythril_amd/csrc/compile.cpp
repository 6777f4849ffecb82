// Tape compiler: mh_node IR (include/mythril_hip.h) -> device register code (dev_isa.h).
//
// Per tape: reachability from the root, legalisation (values wider than 256 bits exist only as
// Concat/ZeroExt chains feeding Keccak, kept as lists of byte-aligned pieces), lowering to
// device ops with virtual registers, then linear-scan allocation onto MH_NUM_REGS registers.
// Assignment columns 0..3 are pinned in R0..R3 when the tape set has at most 4 columns.
// Anything the device path does not cover returns MH_E_UNSUPPORTED so the caller falls back
// to z3, as get_model's contract requires.
#include "compile.h"

#include <algorithm>
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
        default: return 0;
    }
}

struct VInsn {
    uint8_t op;
    int d, a, b, c;   // virtual registers (-1 = none)
    uint32_t width;   // 1..256
    uint32_t aux;     // 21-bit immediate (constant index for D_LOADC / constant operands)
    uint32_t w1raw;   // full second word (D_KECCAK); used when raw == true
    bool raw;
    uint8_t flags;    // F_ACONST / F_BCONST
};

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

struct Lowering {
    const std::vector<mh_node>& t;
    const uint32_t* consts;
    uint32_t n_consts;
    uint32_t n_vars;
    bool pinned;
    std::vector<uint32_t>& dconsts;           // device const pool (8 limbs each)
    std::unordered_map<std::string, uint32_t>& dconst_index;
    std::vector<VInsn> code;
    int n_vregs = 0;
    uint32_t features = 0;
    std::string err;

    Lowering(const std::vector<mh_node>& tape, const uint32_t* c, uint32_t nc, uint32_t nv,
             std::vector<uint32_t>& dc, std::unordered_map<std::string, uint32_t>& di)
        : t(tape), consts(c), n_consts(nc), n_vars(nv), pinned(nv <= MH_MAX_PRELOAD),
          dconsts(dc), dconst_index(di) {
        if (pinned) n_vregs = (int)nv;  // vregs 0..nv-1 are the pinned columns
    }

    int fresh() { return n_vregs++; }

    int emit(uint8_t op, int a = -1, int b = -1, int c = -1, uint32_t width = 256,
             uint32_t aux = 0) {
        VInsn v{op, fresh(), a, b, c, width, aux, 0, false, 0};
        code.push_back(v);
        return v.d;
    }

    bool is_const_node(uint32_t k) const {
        const Val& v = (*vals_)[k];
        return !v.wide() && v.remat >= 0 && t[(size_t)v.remat].op == MH_OP_CONST;
    }

    uint32_t const_of(uint32_t k) {
        const mh_node& c = t[(size_t)(*vals_)[k].remat];
        return const_index(consts + 8ull * c.imm0, c.width);
    }

    // Binary op on IR nodes na, nb; a constant operand is folded into the instruction (read by
    // the scalar unit from the constant pool) instead of being loaded into a register.
    int emit_bin(uint8_t op, uint32_t na, uint32_t nb, uint32_t width, bool commutative) {
        if ((MH_CONST_OPERAND_OK >> op) & 1) {
            const bool ca = is_const_node(na), cb = is_const_node(nb);
            if (cb || (ca && commutative)) {
                const uint32_t kc = cb ? nb : na, kr = cb ? na : nb;
                const int r = vreg_of(kr);
                if (r < 0) return -1;
                VInsn v{op, fresh(), r, -1, -1, width, const_of(kc), 0, false, F_BCONST};
                code.push_back(v);
                return v.d;
            }
        }
        const int a = vreg_of(na), b = vreg_of(nb);
        if (a < 0 || b < 0) return -1;
        return emit(op, a, b, -1, width);
    }

    uint32_t const_index(const uint32_t* limbs, uint32_t width) {
        uint32_t m[8];
        for (int k = 0; k < 8; ++k) {
            int rem = (int)width - 32 * k;
            uint32_t mask = rem >= 32 ? 0xFFFFFFFFu : rem <= 0 ? 0u : ((1u << rem) - 1u);
            m[k] = limbs[k] & mask;
        }
        std::string key(reinterpret_cast<const char*>(m), sizeof(m));
        auto it = dconst_index.find(key);
        if (it != dconst_index.end()) return it->second;
        uint32_t idx = (uint32_t)(dconsts.size() / 8);
        dconsts.insert(dconsts.end(), m, m + 8);
        dconst_index.emplace(key, idx);
        return idx;
    }

    int load_const(const uint32_t* limbs, uint32_t width) {
        VInsn v{D_LOADC, fresh(), -1, -1, -1, width, const_index(limbs, width), 0, false, 0};
        code.push_back(v);
        return v.d;
    }

    int zero_reg() {
        static const uint32_t z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        return load_const(z, 256);
    }

    bool fail(const std::string& m) {
        if (err.empty()) err = m;
        return false;
    }

    std::vector<Val>* vals_ = nullptr;

    // register holding narrow value k (constants are re-loaded at each use)
    int vreg_of(uint32_t k) {
        const Val& v = (*vals_)[k];
        if (v.wide()) return -1;
        if (v.remat >= 0) {
            const mh_node& c = t[(size_t)v.remat];
            if (c.op == MH_OP_TRUE) return emit(D_TRUE, -1, -1, -1, 1);
            if (c.op == MH_OP_FALSE) return emit(D_FALSE, -1, -1, -1, 1);
            return load_const(consts + 8ull * c.imm0, c.width);
        }
        return v.vreg;
    }

    // pieces of a value (a narrow value is one piece)
    std::vector<Piece> pieces_of(uint32_t k, uint32_t width) {
        const Val& v = (*vals_)[k];
        if (!v.wide()) return {Piece{vreg_of(k), width}};
        return v.pieces;
    }

    bool lower(std::vector<Val>& vals, uint32_t* root_reg, uint32_t* root_bool);
};

bool Lowering::lower(std::vector<Val>& vals, uint32_t* root_reg, uint32_t* root_bool) {
    const size_t n = t.size();
    // operand validation (every node) and reachability from the root
    std::vector<char> live(n, 0);
    live[n - 1] = 1;
    for (size_t i = n; i-- > 0;) {
        const mh_node& nd = t[i];
        int ar = (nd.op <= MH_OP_FALSE) ? 0
                 : (nd.op == MH_OP_ITE) ? 3
                 : (nd.op == MH_OP_BVNEG || nd.op == MH_OP_BVNOT || nd.op == MH_OP_NOT ||
                    nd.op == MH_OP_EXTRACT || nd.op == MH_OP_ZEXT || nd.op == MH_OP_SEXT ||
                    nd.op == MH_OP_KECCAK) ? 1 : 2;
        const uint32_t ops[3] = {nd.a, nd.b, nd.c};
        for (int k = 0; k < ar; ++k) {
            if (ops[k] >= i) return fail("operand index not before node " + std::to_string(i));
            if (live[i]) live[ops[k]] = 1;
        }
    }
    vals.assign(n, Val());
    vals_ = &vals;
    // evaluation order: post-order DFS from the root, operands with the larger Sethi-Ullman
    // register need first (the input order is only required to be topological)
    std::vector<uint32_t> need(n, 1);
    auto arity = [&](const mh_node& nd) -> int {
        return (nd.op <= MH_OP_FALSE) ? 0 : (nd.op == MH_OP_ITE) ? 3
               : (nd.op == MH_OP_BVNEG || nd.op == MH_OP_BVNOT || nd.op == MH_OP_NOT ||
                  nd.op == MH_OP_EXTRACT || nd.op == MH_OP_ZEXT || nd.op == MH_OP_SEXT ||
                  nd.op == MH_OP_KECCAK) ? 1 : 2;
    };
    auto children = [&](size_t i, uint32_t* ch) -> int {
        const mh_node& nd = t[i];
        const int ar = arity(nd);
        const uint32_t ops[3] = {nd.a, nd.b, nd.c};
        for (int k = 0; k < ar; ++k) ch[k] = ops[k];
        std::stable_sort(ch, ch + ar, [&](uint32_t x, uint32_t y) { return need[x] > need[y]; });
        return ar;
    };
    for (size_t i = 0; i < n; ++i) {
        const mh_node& nd = t[i];
        if (nd.op == MH_OP_VAR && pinned) { need[i] = 0; continue; }
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
                int r;
                if (pinned) {
                    r = (int)nd.imm0;
                } else {
                    r = emit(D_LOADVAR, -1, -1, -1, 256, nd.imm0);
                }
                if (w < 256) r = emit(D_EXTRACT, r, -1, -1, w, 0);
                out.vreg = r;
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
                switch (nd.op) {
                    case MH_OP_BVADD: op = D_ADD; break;
                    case MH_OP_BVSUB: op = D_SUB; break;
                    case MH_OP_BVMUL: op = D_MUL; break;
                    case MH_OP_BVAND: op = D_AND; break;
                    case MH_OP_BVOR: op = D_OR; break;
                    case MH_OP_BVXOR: op = D_XOR; break;
                    case MH_OP_BVUDIV: op = D_UDIV; features |= F_DIV; break;
                    case MH_OP_BVUREM: op = D_UREM; features |= F_DIV; break;
                    case MH_OP_BVSDIV: op = D_SDIV; features |= F_DIV; break;
                    case MH_OP_BVSREM: op = D_SREM; features |= F_DIV; break;
                    case MH_OP_BVSMOD: op = D_SMOD; features |= F_DIV; break;
                    case MH_OP_EVM_EXP: op = D_EXP; features |= F_EVM; break;
                    case MH_OP_EVM_SIGNEXTEND: op = D_SIGNEXT; features |= F_EVM; break;
                    case MH_OP_EVM_BYTE: op = D_BYTE; features |= F_EVM; break;
                }
                if ((op == D_SIGNEXT || op == D_BYTE) && w != 256)
                    return fail("EVM word ops are 256-bit");
                const bool comm = op == D_ADD || op == D_MUL || op == D_AND || op == D_OR ||
                                  op == D_XOR;
                out.vreg = emit_bin(op, nd.a, nd.b, w, comm);
                break;
            }
            case MH_OP_BVSHL: case MH_OP_BVLSHR: case MH_OP_BVASHR: {
                if (V(nd.a).wide() || V(nd.b).wide() || w == 0 || w > 256)
                    return fail("shift wider than 256");
                const mh_node& sn = t[nd.b];
                if (sn.op == MH_OP_CONST) {  // uniform shift amount
                    const uint32_t* lim = consts + 8ull * sn.imm0;
                    uint32_t hi = 0;
                    for (int k = 1; k < 8; ++k) hi |= lim[k];
                    uint32_t s = lim[0];
                    if (sn.width < 32) s &= (1u << sn.width) - 1u;
                    else if (hi && sn.width > 32) s = 511;
                    if (s > 511) s = 511;
                    uint8_t op = nd.op == MH_OP_BVSHL ? D_SHLI : nd.op == MH_OP_BVLSHR ? D_LSHRI
                                                                                        : D_ASHRI;
                    out.vreg = emit(op, narrow(nd.a), -1, -1, w, s);
                } else {
                    uint8_t op = nd.op == MH_OP_BVSHL ? D_SHL : nd.op == MH_OP_BVLSHR ? D_LSHR
                                                                                       : D_ASHR;
                    out.vreg = emit_bin(op, nd.a, nd.b, w, false);
                }
                break;
            }
            case MH_OP_BVNEG: case MH_OP_BVNOT: {
                int a = narrow(nd.a);
                if (a < 0 || w == 0 || w > 256) return fail("unary op wider than 256");
                out.vreg = emit(nd.op == MH_OP_BVNEG ? D_NEG : D_NOT, a, -1, -1, w);
                break;
            }
            case MH_OP_EQ: {
                uint32_t wa = W(nd.a);
                if (wa != W(nd.b)) return fail("EQ sort mismatch");
                if (V(nd.a).wide() || V(nd.b).wide()) return fail("EQ wider than 256 bits");
                if (wa == 0) out.vreg = emit(D_BEQ, narrow(nd.a), narrow(nd.b), -1, 1);
                else out.vreg = emit_bin(D_EQ, nd.a, nd.b, wa, true);
                break;
            }
            case MH_OP_BVULT: case MH_OP_BVULE: case MH_OP_BVUGT: case MH_OP_BVUGE:
            case MH_OP_BVSLT: case MH_OP_BVSLE: case MH_OP_BVSGT: case MH_OP_BVSGE:
            case MH_OP_BVADD_NOOVFL_U: case MH_OP_BVMUL_NOOVFL_U: case MH_OP_BVSUB_NOUDFL_U: {
                uint32_t wa = W(nd.a);
                if (V(nd.a).wide() || V(nd.b).wide() || wa == 0 || wa > 256 || W(nd.b) != wa)
                    return fail("compare wider than 256 bits");
                uint8_t op = 0;
                bool swap = false;
                switch (nd.op) {
                    case MH_OP_BVULT: op = D_ULT; break;
                    case MH_OP_BVULE: op = D_ULE; break;
                    case MH_OP_BVUGT: op = D_ULT; swap = true; break;
                    case MH_OP_BVUGE: op = D_ULE; swap = true; break;
                    case MH_OP_BVSLT: op = D_SLT; break;
                    case MH_OP_BVSLE: op = D_SLE; break;
                    case MH_OP_BVSGT: op = D_SLT; swap = true; break;
                    case MH_OP_BVSGE: op = D_SLE; swap = true; break;
                    case MH_OP_BVADD_NOOVFL_U: op = D_UADD_NOOVFL; break;
                    case MH_OP_BVMUL_NOOVFL_U: op = D_UMUL_NOOVFL; break;
                    case MH_OP_BVSUB_NOUDFL_U: op = D_ULE; swap = true; break;  // b <= a
                }
                out.vreg = swap ? emit_bin(op, nd.b, nd.a, wa, false)
                                : emit_bin(op, nd.a, nd.b, wa, op == D_UADD_NOOVFL ||
                                                               op == D_UMUL_NOOVFL);
                break;
            }
            case MH_OP_AND: case MH_OP_OR: case MH_OP_XOR: {
                int a = narrow(nd.a), b = narrow(nd.b);
                if (W(nd.a) != 0 || W(nd.b) != 0) return fail("Bool op on bit-vectors");
                uint8_t op = nd.op == MH_OP_AND ? D_BAND : nd.op == MH_OP_OR ? D_BOR : D_BXOR;
                out.vreg = emit(op, a, b, -1, 1);
                break;
            }
            case MH_OP_NOT: {
                if (W(nd.a) != 0) return fail("NOT on a bit-vector");
                out.vreg = emit(D_BNOT, narrow(nd.a), -1, -1, 1);
                break;
            }
            case MH_OP_ITE: {
                if (W(nd.a) != 0) return fail("ITE condition must be Bool");
                int c = narrow(nd.a), a = narrow(nd.b), b = narrow(nd.c);
                if (a < 0 || b < 0 || W(nd.b) != W(nd.c)) return fail("ITE wider than 256");
                if (w == 0) out.vreg = emit(D_BITE, c, a, b, 1);
                else out.vreg = emit(D_ITE, c, a, b, w);
                break;
            }
            case MH_OP_EXTRACT: {
                const uint32_t hi = nd.imm0, lo = nd.imm1, wa = W(nd.a);
                if (wa == 0 || lo > hi || hi >= wa || hi - lo + 1 != w) return fail("bad extract");
                if (!V(nd.a).wide()) {
                    out.vreg = emit(D_EXTRACT, narrow(nd.a), -1, -1, w, lo);
                    break;
                }
                if (w > 256) return fail("extract result wider than 256");
                // gather the parts of the pieces covering [lo, hi]
                const auto& ps = V(nd.a).pieces;
                uint32_t top = wa;  // bit just above the current piece
                int acc = -1;
                uint32_t accw = 0;
                for (const Piece& p : ps) {
                    const uint32_t plo = top - p.bits, phi = top - 1;
                    top = plo;
                    if (phi < lo || plo > hi) continue;
                    const uint32_t elo = std::max(lo, plo) - plo, ehi = std::min(hi, phi) - plo;
                    int part = (elo == 0 && ehi + 1 == p.bits)
                                   ? p.vreg
                                   : emit(D_EXTRACT, p.vreg, -1, -1, ehi - elo + 1, elo);
                    const uint32_t pw = ehi - elo + 1;
                    if (acc < 0) { acc = part; accw = pw; }
                    else {
                        acc = emit(D_CONCAT, acc, part, -1, accw + pw, pw);
                        accw += pw;
                    }
                }
                out.vreg = acc;
                break;
            }
            case MH_OP_CONCAT: {
                const uint32_t wa = W(nd.a), wb = W(nd.b);
                if (wa == 0 || wb == 0 || wa + wb != w) return fail("bad concat");
                if (w <= 256) {
                    out.vreg = emit(D_CONCAT, narrow(nd.a), narrow(nd.b), -1, w, wb);
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
                    int z = zero_reg();
                    uint32_t left = nd.imm0;
                    while (left) {
                        uint32_t take = left > 256 ? 256 : left;
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
                out.vreg = emit(D_SEXT, narrow(nd.a), -1, -1, w, wa);
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
                        cur = emit(D_CONCAT, cur, p.vreg, -1, curw + p.bits, p.bits);
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
                if (total > 135) return fail("multi-block keccak");
                features |= F_KECCAK;
                VInsn v{D_KECCAK, fresh(), chunks[0].vreg,
                        chunks.size() > 1 ? chunks[1].vreg : -1,
                        chunks.size() > 2 ? chunks[2].vreg : -1, 256, 0, 0, true, 0};
                uint32_t w1 = 0;
                for (size_t k = 0; k < chunks.size(); ++k)
                    w1 |= (chunks[k].bits / 8) << (8 + 6 * k);
                w1 |= (uint32_t)chunks.size() << 26;
                v.w1raw = w1;  // c is filled at encode time
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
    const Val& rv = vals[n - 1];
    if (rv.wide()) return fail("root wider than 256 bits");
    *root_reg = (uint32_t)vreg_of((uint32_t)(n - 1));
    *root_bool = t[n - 1].width == 0;
    return true;
}

}  // namespace

int32_t compile_tape(const mh_node* nodes, size_t n_nodes, const uint32_t* consts,
                     uint32_t n_consts, uint32_t n_vars, std::vector<uint32_t>& dconsts,
                     std::unordered_map<std::string, uint32_t>& dconst_index,
                     std::vector<uint32_t>& words, CompiledTape& out, std::string& err) {
    if (n_nodes == 0) {
        err = "empty tape";
        return MH_E_INVALID;
    }
    std::vector<mh_node> t(nodes, nodes + n_nodes);
    Lowering L(t, consts, n_consts, n_vars, dconsts, dconst_index);
    std::vector<Val> vals;
    uint32_t root_v = 0, root_bool = 0;
    if (!L.lower(vals, &root_v, &root_bool)) {
        err = L.err;
        return MH_E_UNSUPPORTED;
    }
    out.alg_ops = 0;
    out.n_nodes = (uint32_t)n_nodes;
    for (size_t i = 0; i < n_nodes; ++i) out.alg_ops += op_cost(t[i], t);
    out.features = L.features;

    // ---- linear-scan register allocation ----
    const int nv = L.n_vregs;
    const int n_pinned = L.pinned ? (int)n_vars : 0;
    std::vector<int> last_use(nv, -1);
    auto use = [&](int r, int i) { if (r >= 0) last_use[r] = std::max(last_use[r], i); };
    for (int i = 0; i < (int)L.code.size(); ++i) {
        use(L.code[i].a, i);
        use(L.code[i].b, i);
        use(L.code[i].c, i);
    }
    use((int)root_v, (int)L.code.size());  // root stays live to the end
    std::vector<int> phys(nv, -1);
    for (int r = 0; r < n_pinned; ++r) phys[r] = r;
    std::vector<int> free_regs;
    for (int r = MH_NUM_REGS - 1; r >= n_pinned; --r) free_regs.push_back(r);
    int peak = n_pinned;
    std::vector<int> in_use_count(MH_NUM_REGS, 0);
    int used = n_pinned;
    for (int i = 0; i < (int)L.code.size(); ++i) {
        VInsn& v = L.code[i];
        // release operands whose last use is this instruction (the kernel reads operands
        // before writing the destination, so d may reuse an operand's register)
        int ops[3] = {v.a, v.b, v.c};
        for (int k = 0; k < 3; ++k) {
            int r = ops[k];
            if (r < n_pinned || r < 0) continue;
            bool dup = false;
            for (int j = 0; j < k; ++j) dup |= ops[j] == r;
            if (!dup && last_use[r] == i) {
                free_regs.push_back(phys[r]);
                --used;
            }
        }
        if (last_use[v.d] < 0) {
            // dead result (only possible for unused keccak chunks etc.) — still needs a slot
            last_use[v.d] = i;
        }
        if (free_regs.empty()) {
            err = "register pressure exceeds " + std::to_string(MH_NUM_REGS) + " registers";
            return MH_E_UNSUPPORTED;
        }
        phys[v.d] = free_regs.back();
        free_regs.pop_back();
        ++used;
        peak = std::max(peak, used);
        if (last_use[v.d] == i) {  // dead immediately
            free_regs.push_back(phys[v.d]);
            --used;
        }
    }
    out.n_regs = (uint32_t)peak;
    out.n_insns = (uint32_t)L.code.size();
    out.root_reg = (uint32_t)phys[root_v];
    out.root_bool = root_bool;

    // ---- encode ----
    for (const VInsn& v : L.code) {
        auto P = [&](int r) -> uint32_t { return r < 0 ? 0u : (uint32_t)phys[r]; };
        const uint32_t w0 = (uint32_t)v.op | (P(v.d) << 8) | (P(v.a) << 16) | (P(v.b) << 24);
        uint32_t w1;
        if (v.op == D_KECCAK) {
            w1 = v.w1raw | P(v.c);
        } else {
            const uint32_t aux = (v.op == D_ITE || v.op == D_BITE) ? P(v.c) : v.aux;
            if (aux > MH_AUX_MAX) {
                err = "immediate / constant index exceeds 21 bits";
                return MH_E_UNSUPPORTED;
            }
            w1 = (uint32_t)v.flags | ((v.width & 0x1FF) << 2) | (aux << 11);
        }
        words.push_back(w0);
        words.push_back(w1);
    }
    return MH_OK;
}

}  // namespace mh
