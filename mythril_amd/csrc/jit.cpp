// Native-code emitter of the sieve JIT (see jit.h for the design).
//
// Per tape (SSA from compile.cpp lower_tape_ssa, constants folded):
//   1. last use of every virtual register, and the limbs each value must provide (demanded
//      limbs, a backward pass: a consumer that reads limb k of its result asks its operands for
//      the limbs limb k depends on -- carries reach up, shifts move, masks cut);
//   2. forward emission: a value is 8 limbs, each a constant (no code) or one VGPR; every op
//      computes only its demanded limbs, with limb-level constant folding and renaming
//      (x + (c << 128) copies nothing below limb 4, x & 0xff..ff is x, a shift by 64 is a rename);
//      Bool values are lane masks in SGPR pairs; registers are reference counted and freed at
//      the last use;
//   3. the root's mask goes to s[S_RES:S_RES+1] (values mode also reports the root's limbs).
// Encoding rules of gfx950 honoured here: a VOP2/VOPC (e32) src1 must be a VGPR; a VOP2 that
// reads VCC implicitly (addc/subb/cndmask e32) takes no literal or SGPR in src0; VOP3 takes no
// literal and at most one SGPR (a carry-in or mask pair counts).  Constants that break a rule are
// first moved into a VGPR (v_mov, a 2-cycle instruction) or staged in an SGPR (s_mov).
#include "jit.h"

#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace mh {
namespace jit {

namespace {

struct Fail {
    std::string why;
};

[[noreturn]] void fail(const std::string& w) { throw Fail{w}; }

enum LK : uint8_t { L_UNDEF, L_CONST, L_VGPR };
struct Limb {
    uint8_t k = L_UNDEF;
    uint32_t v = 0;
    static Limb C(uint32_t x) { Limb l; l.k = L_CONST; l.v = x; return l; }
    static Limb R(uint32_t r) { Limb l; l.k = L_VGPR; l.v = r; return l; }
    bool is_c() const { return k == L_CONST; }
    bool is_r() const { return k == L_VGPR; }
    bool is_c(uint32_t x) const { return k == L_CONST && v == x; }
};

struct Val {
    bool is_bool = false;
    int bconst = -1;  // Bool: 0/1 when known, -1 = lane mask in SGPR pair `pair`
    int pair = -1;
    Limb l[8];
    bool defined = false;
};

enum : uint32_t { LBL_SC_SKIP = 0xFFF0, LBL_SC_END = 0xFFF1 };  // tape-local labels

int top_bit(uint32_t m) { return m ? 31 - __builtin_clz(m) : -1; }
uint32_t prefix_mask(uint32_t m) { int t = top_bit(m); return t < 0 ? 0u : ((2u << t) - 1u); }

class Emitter {
public:
    Emitter(const SsaTape& st, const std::vector<uint32_t>& pool, uint32_t n_vars,
            const Options& opt, const std::vector<uint8_t>* check = nullptr,
            std::vector<double>* insn_cost = nullptr)
        : st_(st), pool_(pool), n_vars_(n_vars), opt_(opt), check_(check),
          insn_cost_(insn_cost) {}

    TapeCode run();

private:
    const SsaTape& st_;
    const std::vector<uint32_t>& pool_;
    uint32_t n_vars_;
    Options opt_;
    const std::vector<uint8_t>* check_;  // short-circuit test after these vregs (or null)
    std::vector<double>* insn_cost_;     // out: VALU emitted per SSA instruction (or null)
    bool sc_used_ = false;
    std::vector<MI> code_;
    std::vector<Val> vals_;
    std::vector<int> last_;
    std::vector<uint8_t> dem_;
    int vref_[512] = {};
    uint32_t vbase_ = 0, vmax_ = 0, vhigh_ = 0;
    int pref_[N_BOOL_PAIRS] = {};
    uint32_t kstage_ = 0;
    uint32_t n_valu_ = 0, n_wide_ = 0, n_salu_ = 0;
    // VALU emitted on the unlikely side of a uniform branch (cold_ > 0): static counts keep
    // them, the scheduler's cost model (insn_cost_) does not
    uint32_t n_valu_cold_ = 0;
    int cold_ = 0;
    bool calls_div_ = false;
    bool uses_lds_ = false;
    bool calls_kec_ = false;
    int cur_op_ = -1;  // SSA op being emitted (diagnostic attribution)
public:
    static uint64_t op_valu[256], op_wide[256], op_count[256];
private:

    // ---- emission
    void emit(uint16_t op, std::initializer_list<Opnd> ops, bool e64 = false) {
        MI m;
        m.op = op;
        m.e64 = e64 ? 1 : 0;
        m.tag = cur_op_ >= 0 ? (uint8_t)cur_op_ : 0xFF;
        int i = 0;
        for (const Opnd& o : ops) m.o[i++] = o;
        code_.push_back(m);
        if (op <= M_V_CMP_LE_F64) {
            ++n_valu_;
            if (cold_ > 0) ++n_valu_cold_;
            const bool wide = e64 || op == M_V_ADD_CO || op == M_V_ADDC_CO || op == M_V_SUB_CO ||
                              op == M_V_SUBB_CO || op == M_V_SUBREV_CO || op == M_V_SUBBREV_CO ||
                              op == M_V_OR3 || op == M_V_ALIGNBIT || op == M_V_MAD_U64_U32 ||
                              op == M_V_LSHL_ADD || op == M_V_PERM || op == M_V_BFI ||
                              op == M_V_LSHLREV || op == M_V_LSHRREV || op == M_V_ASHRREV ||
                              (op >= M_V_CMP_EQ && op <= M_V_CMP_GT_I32) || op >= M_V_CVT_F64_U32 ||
                              op == M_V_RCP_F32 || op == M_V_CMP_GT_F32 || op == M_V_CMP_LE_F32;
            if (wide) ++n_wide_;
            if (cur_op_ >= 0) { ++op_valu[cur_op_]; op_wide[cur_op_] += wide; }
        } else if (op <= M_S_CMP_LT_U32) {
            ++n_salu_;
        }
    }

    uint32_t next_lbl_ = 0x1000;  // tape-local labels of in-op branches

    // ---- VGPRs (reference counted; columns and fixed registers are never freed)
    uint32_t valloc() {
        for (uint32_t r = vbase_; r < vmax_; ++r)
            if (vref_[r] == 0) {
                vref_[r] = 1;
                vhigh_ = std::max(vhigh_, r + 1);
                return r;
            }
        fail("VGPR pressure");
    }
    uint32_t valloc_pair() {
        for (uint32_t r = (vbase_ + 1) & ~1u; r + 1 < vmax_; r += 2)
            if (vref_[r] == 0 && vref_[r + 1] == 0) {
                vref_[r] = vref_[r + 1] = 1;
                vhigh_ = std::max(vhigh_, r + 2);
                return r;
            }
        fail("VGPR pressure (pair)");
    }
    void vretain(uint32_t r) { if (r >= vbase_) ++vref_[r]; }
    void vrelease(uint32_t r) {
        if (r < vbase_) return;
        if (vref_[r] <= 0) fail("internal: VGPR refcount");
        --vref_[r];
    }

    // ---- Bool pairs
    int palloc() {
        for (int i = 0; i < (int)N_BOOL_PAIRS; ++i)
            if (pref_[i] == 0) {
                pref_[i] = 1;
                return i;
            }
        fail("SGPR pressure (Bool masks)");
    }
    static Opnd P(int i) { return S(S_BOOL0 + 2 * (uint32_t)i, 2); }

    // ---- values
    void retain(const Val& v) {
        if (v.is_bool) {
            if (v.bconst < 0) ++pref_[v.pair];
            return;
        }
        for (const Limb& l : v.l)
            if (l.is_r()) vretain(l.v);
    }
    void release(const Val& v) {
        if (v.is_bool) {
            if (v.bconst < 0) {
                if (pref_[v.pair] <= 0) fail("internal: pair refcount");
                --pref_[v.pair];
            }
            return;
        }
        for (const Limb& l : v.l)
            if (l.is_r()) vrelease(l.v);
    }
    const Val& val(int r) const {
        if (r < 0 || r >= (int)vals_.size() || !vals_[r].defined) fail("internal: undefined vreg");
        return vals_[r];
    }
    Val const_val(int cidx) const {
        Val v;
        v.defined = true;
        for (int k = 0; k < 8; ++k) v.l[k] = Limb::C(pool_[8ull * (uint32_t)cidx + k]);
        return v;
    }
    static Val bool_const(bool b) {
        Val v;
        v.defined = true;
        v.is_bool = true;
        v.bconst = b ? 1 : 0;
        return v;
    }
    Val bool_mask(int pair) {
        Val v;
        v.defined = true;
        v.is_bool = true;
        v.pair = pair;
        return v;
    }
    // a Bool as a mask pair (constants materialised in a fresh pair; caller releases)
    int mask_of(const Val& b, std::vector<int>& tmp_pairs) {
        if (b.bconst < 0) return b.pair;
        const int p = palloc();
        tmp_pairs.push_back(p);
        emit(M_S_MOV_B64, {P(p), IMM(b.bconst ? 0xFFFFFFFFu : 0u)});
        return p;
    }

    static Opnd src(const Limb& l) {
        if (l.k == L_UNDEF) fail("internal: read of an undemanded limb");
        return l.is_c() ? IMM(l.v) : V(l.v);
    }
    // a VGPR holding limb l (constants moved into a temporary, released by the caller)
    uint32_t vgpr_of(const Limb& l, std::vector<uint32_t>& tmp) {
        if (l.k == L_UNDEF) fail("internal: read of an undemanded limb");
        if (l.is_r()) return l.v;
        const uint32_t t = valloc();
        tmp.push_back(t);
        emit(M_V_MOV, {V(t), IMM(l.v)});
        return t;
    }
    // VGPR or inline constant
    Opnd vi_of(const Limb& l, std::vector<uint32_t>& tmp) {
        if (l.is_c() && is_inline(l.v)) return IMM(l.v);
        return V(vgpr_of(l, tmp));
    }
    // SGPR-staged constant (one per VOP3 at most)
    Opnd staged(uint32_t x) {
        if (is_inline(x)) return IMM(x);
        const uint32_t s = S_KSTAGE + (kstage_++ % N_KSTAGE);
        emit(M_S_MOV_B32, {S(s), IMM(x)});
        return S(s);
    }
    void free_tmp(std::vector<uint32_t>& tmp) {
        for (uint32_t r : tmp) vrelease(r);
        tmp.clear();
    }
    void free_tmp_pairs(std::vector<int>& tp) {
        for (int p : tp) --pref_[p];
        tp.clear();
    }

    // ---- building blocks
    int chain(bool sub, const Limb* a, const Limb* b, int top, Limb* res, uint32_t junk,
              std::vector<uint32_t>& tmp);
    void op_addsub(int d, const Val& A, const Val& B, bool sub);
    void op_logic(int d, const Val& A, const Val& B, int kind);
    Val op_eq(const Val& A, const Val& B);
    void and_all_zero(const std::vector<uint32_t>& regs, int* p, std::vector<uint32_t>& tmp);
    Val op_ult(const Val& A, const Val& B, bool signed_, bool negate);
    void op_ite(int d, const Val& C, const Val& T, const Val& E);
    Val op_bite(const Val& C, const Val& T, const Val& E);
    Val op_bool2(uint8_t op, const Val& A, const Val& B);
    void op_shr(int d, const Val& A, uint32_t s);
    void op_shl(int d, const Val& A, uint32_t s);
    void op_vshift(int d, const Val& A, const Val& B, uint8_t op);
    void op_mul(int d, const Val& A, const Val& B);
    void op_div(int d, int a, int b, int cidx, uint32_t kind, int cur);
    void rescue_div_regs(int cur, uint32_t end = R_TEMP0);
    void op_keccak(const SsaInsn& v, int cur);
    void op_exp(int d, const Val& A, const Val& E);
    void addmod_regs(const uint32_t* u, const uint32_t* v, const uint32_t* n, uint32_t* r,
                     int when = -1);
    void op_mulmod(int d, const Val& X, const Val& Y, const Val& N);
    int scratch_ = -1;  // a virtual register past the tape's own (op_exp's products)
    void demand();
    void sc_check(const Val& v);
    Val& out(int d) {
        Val& v = vals_[d];
        v = Val();
        v.defined = true;
        return v;
    }
};

// Carry / borrow chain over limbs 0..top: res[k] = a[k] +- b[k] +- carry (res == nullptr: the
// limbs go to `junk`, only the final carry matters).  Returns the final carry state: 0 / 1 when
// known at compile time, 2 when it is in VCC.
int Emitter::chain(bool sub, const Limb* a, const Limb* b, int top, Limb* res, uint32_t junk,
                   std::vector<uint32_t>& tmp) {
    int cs = 0;
    uint32_t same = ~0u;  // register holding the value of the last "carry passes through" limb
    for (int k = 0; k <= top; ++k) {
        const Limb x = a[k], y = b[k];
        if (x.k == L_UNDEF || y.k == L_UNDEF) fail("internal: chain over an undemanded limb");
        if (cs == 2 && x.is_c() && y.is_c()) {
            // carry / borrow c in VCC, both limbs constant: x - x - c = -c and 2^32-1 + c wrap
            // with the carry passing through unchanged, so a run of such limbs (the top of a
            // narrow value's sign extension, say) shares one register; any other constant pair
            // decides the carry out at compile time
            const bool through = sub ? x.v == y.v : (uint64_t)x.v + y.v == 0xFFFFFFFFull;
            if (through) {
                if (res) {
                    if (same == ~0u) {
                        same = valloc();
                        emit(M_V_ADDC_CO, {V(same), S(S_DIV_DUMMY, 2), IMM(sub ? 0u : ~0u),
                                           IMM(sub ? 0u : 0u), VCC()}, true);
                        if (sub) code_.back().op = M_V_SUBB_CO;
                    } else {
                        vretain(same);
                    }
                    res[k] = Limb::R(same);
                }
                continue;
            }
            same = ~0u;
            if (!res) {  // only the final carry matters: it is known from here on
                cs = sub ? (x.v < y.v ? 1 : 0) : ((uint64_t)x.v + y.v > 0xFFFFFFFFull ? 1 : 0);
                continue;
            }
            const uint32_t dst = valloc();
            if (sub) {
                if (is_inline(x.v) && is_inline(y.v))
                    emit(M_V_SUBB_CO, {V(dst), S(S_DIV_DUMMY, 2), IMM(x.v), IMM(y.v), VCC()}, true);
                else
                    emit(M_V_SUBB_CO, {V(dst), S(S_DIV_DUMMY, 2), V(vgpr_of(x, tmp)),
                                       V(vgpr_of(y, tmp)), VCC()}, true);
                cs = x.v < y.v ? 1 : 0;
            } else {
                const uint32_t sv = x.v + y.v;  // < 2^32 - 1 or wrapped: carry out known
                if (is_inline(sv))
                    emit(M_V_ADDC_CO, {V(dst), S(S_DIV_DUMMY, 2), IMM(sv), IMM(0), VCC()}, true);
                else
                    emit(M_V_ADDC_CO, {V(dst), S(S_DIV_DUMMY, 2), V(vgpr_of(Limb::C(sv), tmp)),
                                       IMM(0), VCC()}, true);
                cs = (uint64_t)x.v + y.v > 0xFFFFFFFFull ? 1 : 0;
            }
            res[k] = Limb::R(dst);
            continue;
        }
        same = ~0u;
        if (cs != 2 && x.is_c() && y.is_c()) {
            const uint64_t xv = x.v, yv = y.v;
            if (sub) {
                if (res) res[k] = Limb::C((uint32_t)(xv - yv - (uint64_t)cs));
                cs = xv < yv + (uint64_t)cs ? 1 : 0;
            } else {
                const uint64_t r = xv + yv + (uint64_t)cs;
                if (res) res[k] = Limb::C((uint32_t)r);
                cs = (int)(r >> 32);
            }
            continue;
        }
        if (cs == 0 && y.is_c(0)) {  // x +- 0, no carry: x
            if (res) { res[k] = x; if (x.is_r()) vretain(x.v); }
            continue;
        }
        if (cs == 0 && !sub && x.is_c(0)) {
            if (res) { res[k] = y; if (y.is_r()) vretain(y.v); }
            continue;
        }
        const uint32_t dst = res ? valloc() : junk;
        if (cs == 1) {
            emit(M_S_MOV_B64, {VCC(), IMM(0xFFFFFFFFu)});
            cs = 2;
        }
        if (cs == 0) {  // first instruction of the chain: carry-out only
            if (!sub) {
                if (y.is_r()) emit(M_V_ADD_CO, {V(dst), VCC(), src(x), V(y.v)});
                else if (x.is_r()) emit(M_V_ADD_CO, {V(dst), VCC(), src(y), V(x.v)});
                else emit(M_V_ADD_CO, {V(dst), VCC(), src(x), V(vgpr_of(y, tmp))});
            } else {
                if (y.is_r()) emit(M_V_SUB_CO, {V(dst), VCC(), src(x), V(y.v)});        // x - y
                else if (x.is_r()) emit(M_V_SUBREV_CO, {V(dst), VCC(), src(y), V(x.v)});  // x - y
                else emit(M_V_SUB_CO, {V(dst), VCC(), src(x), V(vgpr_of(y, tmp))});
            }
        } else {  // carry-in in VCC
            if (!sub) {
                Limb p = x, q = y;
                if (!q.is_r() && p.is_r()) std::swap(p, q);
                if (!q.is_r() && !p.is_r() && is_inline(p.v) && is_inline(q.v)) {
                    emit(M_V_ADDC_CO, {V(dst), VCC(), IMM(p.v), IMM(q.v), VCC()}, true);
                } else {
                    const uint32_t qr = vgpr_of(q, tmp);
                    emit(M_V_ADDC_CO, {V(dst), VCC(), vi_of(p, tmp), V(qr), VCC()});
                }
            } else {
                if (y.is_r()) {
                    emit(M_V_SUBB_CO, {V(dst), VCC(), vi_of(x, tmp), V(y.v), VCC()});
                } else if (x.is_r()) {
                    emit(M_V_SUBBREV_CO, {V(dst), VCC(), vi_of(y, tmp), V(x.v), VCC()});
                } else if (is_inline(x.v) && is_inline(y.v)) {
                    emit(M_V_SUBB_CO, {V(dst), VCC(), IMM(x.v), IMM(y.v), VCC()}, true);
                } else {
                    emit(M_V_SUBB_CO, {V(dst), VCC(), vi_of(x, tmp), V(vgpr_of(y, tmp)), VCC()});
                }
            }
        }
        cs = 2;
        if (res) res[k] = Limb::R(dst);
    }
    return cs;
}

void Emitter::op_addsub(int d, const Val& A, const Val& B, bool sub) {
    const int top = top_bit(dem_[d]);
    Val& R = out(d);
    if (top < 0) return;
    std::vector<uint32_t> tmp;
    chain(sub, A.l, B.l, top, R.l, 0, tmp);
    free_tmp(tmp);
}

// kind 0 and, 1 or, 2 xor
void Emitter::op_logic(int d, const Val& A, const Val& B, int kind) {
    const uint32_t dm = dem_[d];
    Val& R = out(d);
    for (int k = 0; k < 8; ++k) {
        if (!((dm >> k) & 1)) continue;
        Limb x = A.l[k], y = B.l[k];
        if (x.is_c() && !y.is_c()) std::swap(x, y);  // constant (if any) in y
        if (y.is_c() && ((kind == 0 && y.v == 0) || (kind == 1 && y.v == ~0u))) {
            R.l[k] = Limb::C(y.v);  // the constant decides (the other limb was not demanded)
            continue;
        }
        if (x.k == L_UNDEF || y.k == L_UNDEF) fail("internal: logic over an undemanded limb");
        auto alias = [&](const Limb& l) { R.l[k] = l; if (l.is_r()) vretain(l.v); };
        if (x.is_c() && y.is_c()) {
            R.l[k] = Limb::C(kind == 0 ? (x.v & y.v) : kind == 1 ? (x.v | y.v) : (x.v ^ y.v));
            continue;
        }
        if (y.is_c()) {
            const uint32_t c = y.v;
            if (kind == 0 && c == 0) { R.l[k] = Limb::C(0); continue; }
            if (kind == 0 && c == ~0u) { alias(x); continue; }
            if (kind == 1 && c == 0) { alias(x); continue; }
            if (kind == 1 && c == ~0u) { R.l[k] = Limb::C(~0u); continue; }
            if (kind == 2 && c == 0) { alias(x); continue; }
            const uint32_t dst = valloc();
            if (kind == 2 && c == ~0u) emit(M_V_NOT, {V(dst), V(x.v)});
            else emit(kind == 0 ? M_V_AND : kind == 1 ? M_V_OR : M_V_XOR, {V(dst), IMM(c), V(x.v)});
            R.l[k] = Limb::R(dst);
            continue;
        }
        if (x.v == y.v) {  // same register
            if (kind == 2) R.l[k] = Limb::C(0);
            else alias(x);
            continue;
        }
        const uint32_t dst = valloc();
        emit(kind == 0 ? M_V_AND : kind == 1 ? M_V_OR : M_V_XOR, {V(dst), V(x.v), V(y.v)});
        R.l[k] = Limb::R(dst);
    }
}

// a lane mask "all of these VGPR limbs are zero" folded into the pair *p (allocated on first
// use): v_or (2-cycle) reduction, one compare
void Emitter::and_all_zero(const std::vector<uint32_t>& regs, int* p, std::vector<uint32_t>& tmp) {
    if (regs.empty()) return;
    uint32_t acc = regs[0];
    if (regs.size() > 1) {
        acc = valloc();
        tmp.push_back(acc);
        emit(M_V_OR, {V(acc), V(regs[0]), V(regs[1])});
        for (size_t i = 2; i < regs.size(); ++i) emit(M_V_OR, {V(acc), V(regs[i]), V(acc)});
    }
    emit(M_V_CMP_EQ, {VCC(), IMM(0), V(acc)});
    if (*p < 0) {
        *p = palloc();
        emit(M_S_MOV_B64, {P(*p), VCC()});
    } else {
        emit(M_S_AND_B64, {P(*p), P(*p), VCC()});
    }
}

Val Emitter::op_eq(const Val& A, const Val& B) {
    int p = -1;
    std::vector<uint32_t> zero_regs, tmp;  // VGPR limbs compared against a known zero
    std::vector<std::pair<Limb, Limb>> cmps;  // (constant or VGPR, VGPR) limb pairs
    for (int k = 0; k < 8; ++k) {
        Limb x = A.l[k], y = B.l[k];
        if (x.is_c() && y.is_c()) {
            if (x.v != y.v) return bool_const(false);
            continue;
        }
        if (x.is_r() && y.is_r() && x.v == y.v) continue;
        if (!y.is_r()) std::swap(x, y);
        if (x.is_c(0)) {
            zero_regs.push_back(y.v);
            continue;
        }
        cmps.push_back({x, y});
    }
    // once the first compare finds no equal lane (full-width operands: nearly always) the
    // value is false in every lane: the other compares are skipped
    const size_t rest = cmps.size() + (zero_regs.empty() ? 0 : 1);
    const uint32_t l_end = rest >= 3 ? next_lbl_++ : 0;
    for (size_t i = 0; i < cmps.size(); ++i) {
        emit(M_V_CMP_EQ, {VCC(), src(cmps[i].first), V(cmps[i].second.v)});
        if (p < 0) {
            p = palloc();
            emit(M_S_MOV_B64, {P(p), VCC()});
            if (l_end) {
                emit(M_S_CMP_EQ_U64, {P(p), IMM(0)});
                emit(M_S_CBRANCH_SCC1, {LBL(l_end)});
            }
            if (l_end) ++cold_;
        } else {
            emit(M_S_AND_B64, {P(p), P(p), VCC()});
        }
    }
    and_all_zero(zero_regs, &p, tmp);
    free_tmp(tmp);
    if (l_end && p >= 0) {
        --cold_;
        emit(M_LABEL, {LBL(l_end)});
    }
    if (p < 0) return bool_const(true);
    return bool_mask(p);
}

// A < B (unsigned, or signed 256-bit), optionally negated (>=).  Limbs where both sides are
// equal constants at the top do not take part; a run of top limbs known zero on one side only
// is an OR-reduction of the other side's limbs plus the compare of the limbs below:
//   A < B  =  A[hi] == 0 && A[lo] < B[lo]   (B zero in hi)
//          =  B[hi] != 0 || A[lo] < B[lo]   (A zero in hi)
Val Emitter::op_ult(const Val& A, const Val& B, bool signed_, bool negate) {
    std::vector<uint32_t> tmp;
    Limb a[8], b[8];
    for (int k = 0; k < 8; ++k) { a[k] = A.l[k]; b[k] = B.l[k]; }
    // signed: bias the sign bit (signed order = unsigned order of x ^ 2^255); constant limbs
    // now, register limbs where the borrow chain needs them (the uniform path compares the
    // unbiased top limbs as signed words)
    bool bias_regs = false;
    if (signed_) {
        for (Limb* l : {&a[7], &b[7]}) {
            if (l->is_c()) l->v ^= 0x80000000u;
            else bias_regs = true;
        }
    }
    auto bias = [&]() {
        if (!bias_regs) return;
        bias_regs = false;
        for (Limb* l : {&a[7], &b[7]}) {
            if (l->is_c()) continue;
            const uint32_t t = valloc();
            tmp.push_back(t);
            emit(M_V_XOR, {V(t), IMM(0x80000000u), V(l->v)});
            *l = Limb::R(t);
        }
    };
    int top = 7;
    while (top > 0 && a[top].is_c() && b[top].is_c() && a[top].v == b[top].v) --top;
    if (top < 7) bias();  // (limb 7 constant on both sides: no register bias anyway)
    if (a[top].is_c() && b[top].is_c() && a[top].v != b[top].v) {
        // the highest limb that differs is known on both sides: it decides, whatever is below
        free_tmp(tmp);
        return bool_const((a[top].v < b[top].v) != negate);
    }
    // top run where exactly one side is known zero
    int hi_side = 0;  // 1: b zero on [m+1, top], 2: a zero there
    int m = top;
    if (b[top].is_c(0) && !a[top].is_c()) {
        hi_side = 1;
        while (m > 0 && b[m].is_c(0)) --m;
    } else if (a[top].is_c(0) && !b[top].is_c()) {
        hi_side = 2;
        while (m > 0 && a[m].is_c(0)) --m;
    }
    if (hi_side && m == top) hi_side = 0;
    if (hi_side) bias();
    int p = -1;  // the high-run mask (A[hi] == 0 / B[hi] == 0)
    std::vector<uint32_t> regs;
    const Limb* o = hi_side == 1 ? a : b;  // the side that is not zero there
    if (hi_side) {
        for (int k = m + 1; k <= top; ++k) {
            if (o[k].is_c()) {
                if (o[k].v) {  // decided by a known nonzero limb
                    free_tmp(tmp);
                    if (p >= 0) --pref_[p];
                    return bool_const((hi_side == 2) != negate);
                }
                continue;
            }
            regs.push_back(o[k].v);
        }
    }
    auto finish = [&]() -> Val {
        if (hi_side) and_all_zero(regs, &p, tmp);
        // uniform fast path: when the top limbs differ in every lane -- all but certain for
        // full-width operands -- the top limb alone decides: one compare tests that, one decides
        const bool fast = p < 0 && m == top && top >= 2 && !(a[top].is_c() && b[top].is_c());
        uint32_t l_join = 0;
        if (fast) {
            l_join = next_lbl_++;
            const uint32_t l_chain = next_lbl_++;
            // v_cmp_<op> vcc, x, y (x may be a constant; a constant y swaps the operands)
            auto cmp = [&](uint16_t op, Limb x, Limb y) {
                if (y.is_c() && !x.is_c()) {
                    const uint16_t rev = op == M_V_CMP_LT ? M_V_CMP_GT
                                       : op == M_V_CMP_LT_I32 ? M_V_CMP_GT_I32 : op;
                    emit(rev, {VCC(), IMM(y.v), V(x.v)});
                } else {
                    emit(op, {VCC(), src(x), V(y.v)});
                }
            };
            // signed top limbs compare unbiased as signed words (constants were biased above)
            Limb xa = a[top], xb = b[top];
            const bool sgn_top = signed_ && top == 7;
            if (sgn_top) {
                if (xa.is_c()) xa.v ^= 0x80000000u;
                if (xb.is_c()) xb.v ^= 0x80000000u;
            }
            cmp(M_V_CMP_NE, xa, xb);
            emit(M_S_CMP_EQ_U64, {VCC(), IMM(0xFFFFFFFFu)});
            emit(M_S_CBRANCH_SCC0, {LBL(l_chain)});
            cmp(sgn_top ? M_V_CMP_LT_I32 : M_V_CMP_LT, xa, xb);  // the borrow of A - B
            emit(M_S_BRANCH, {LBL(l_join)});
            emit(M_LABEL, {LBL(l_chain)});
            ++cold_;
            bias();
            --cold_;
        }
        bias();
        if (fast) ++cold_;
        const uint32_t junk = valloc();
        tmp.push_back(junk);
        const int cs = chain(true, a, b, m, nullptr, junk, tmp);
        if (fast) {
            if (cs != 2) fail("internal: uniform compare path over a known borrow");
            --cold_;
            emit(M_LABEL, {LBL(l_join)});
        }
        free_tmp(tmp);
        // combine: lo = borrow (A[lo] < B[lo]); result = hi_side 1: p && lo; 2: !p || lo
        if (p < 0) {
            if (cs != 2) return bool_const((cs == 1) != negate);
            const int q = palloc();
            emit(negate ? M_S_NOT_B64 : M_S_MOV_B64, {P(q), VCC()});
            return bool_mask(q);
        }
        // p holds "the other side's high run is zero"
        if (cs != 2) {
            const bool lo = cs == 1;
            if (hi_side == 1) {  // p && lo
                if (!lo) { --pref_[p]; return bool_const(negate); }
                if (negate) emit(M_S_NOT_B64, {P(p), P(p)});
                return bool_mask(p);
            }
            // !p || lo
            if (lo) { --pref_[p]; return bool_const(!negate); }
            if (!negate) emit(M_S_NOT_B64, {P(p), P(p)});
            return bool_mask(p);
        }
        if (hi_side == 1) emit(M_S_AND_B64, {P(p), P(p), VCC()});
        else emit(M_S_ORN2_B64, {P(p), VCC(), P(p)});  // lo || !p
        if (negate) emit(M_S_NOT_B64, {P(p), P(p)});
        return bool_mask(p);
    };
    // uniform path of a high run: when the nonzero side's top limb is nonzero in every lane
    // (a full-width value against a narrow one), that side is the larger one in every lane
    if (hi_side && !regs.empty() && o[top].is_r()) {
        const int q = palloc();
        const uint32_t l_slow = next_lbl_++, l_join2 = next_lbl_++;
        emit(M_V_CMP_NE, {VCC(), IMM(0), V(o[top].v)});
        emit(M_S_CMP_EQ_U64, {VCC(), IMM(0xFFFFFFFFu)});
        emit(M_S_CBRANCH_SCC0, {LBL(l_slow)});
        const bool lt = hi_side == 2;  // B has the nonzero high part: A < B
        emit(M_S_MOV_B64, {P(q), IMM((lt != negate) ? 0xFFFFFFFFu : 0u)});
        emit(M_S_BRANCH, {LBL(l_join2)});
        emit(M_LABEL, {LBL(l_slow)});
        ++cold_;
        const Val r = finish();
        --cold_;
        if (r.bconst >= 0) {
            emit(M_S_MOV_B64, {P(q), IMM(r.bconst ? 0xFFFFFFFFu : 0u)});
        } else {
            emit(M_S_MOV_B64, {P(q), P(r.pair)});
            release(r);
        }
        emit(M_LABEL, {LBL(l_join2)});
        return bool_mask(q);
    }
    return finish();
}

void Emitter::op_ite(int d, const Val& C, const Val& T, const Val& E) {
    if (C.bconst >= 0) {
        Val v = C.bconst ? T : E;
        retain(v);
        vals_[d] = v;
        return;
    }
    const uint32_t dm = dem_[d];
    Val& R = out(d);
    std::vector<uint32_t> tmp;
    for (int k = 0; k < 8; ++k) {
        if (!((dm >> k) & 1)) continue;
        const Limb t = T.l[k], e = E.l[k];
        if (t.k == L_UNDEF || e.k == L_UNDEF) fail("internal: ite over an undemanded limb");
        if (t.k == e.k && t.v == e.v) {
            R.l[k] = t;
            if (t.is_r()) vretain(t.v);
            continue;
        }
        const uint32_t dst = valloc();
        emit(M_V_CNDMASK, {V(dst), vi_of(e, tmp), vi_of(t, tmp), P(C.pair)}, true);
        R.l[k] = Limb::R(dst);
    }
    free_tmp(tmp);
}

Val Emitter::op_bite(const Val& C, const Val& T, const Val& E) {
    if (C.bconst >= 0) {
        Val v = C.bconst ? T : E;
        retain(v);
        return v;
    }
    if (T.bconst >= 0 && E.bconst >= 0) {
        if (T.bconst == E.bconst) return bool_const(T.bconst != 0);
        const int p = palloc();
        emit(T.bconst ? M_S_MOV_B64 : M_S_NOT_B64, {P(p), P(C.pair)});
        return bool_mask(p);
    }
    std::vector<int> tp;
    const int t = mask_of(T, tp), e = mask_of(E, tp);
    const int p = palloc();
    const int q = palloc();
    emit(M_S_AND_B64, {P(p), P(C.pair), P(t)});
    emit(M_S_ANDN2_B64, {P(q), P(e), P(C.pair)});
    emit(M_S_OR_B64, {P(p), P(p), P(q)});
    --pref_[q];
    free_tmp_pairs(tp);
    return bool_mask(p);
}

Val Emitter::op_bool2(uint8_t op, const Val& A, const Val& B) {
    const Val* a = &A;
    const Val* b = &B;
    if (a->bconst >= 0 && b->bconst >= 0) {
        const bool x = a->bconst, y = b->bconst;
        switch (op) {
            case D_BAND: return bool_const(x && y);
            case D_BOR: return bool_const(x || y);
            case D_BXOR: return bool_const(x != y);
            default: return bool_const(x == y);  // D_BEQ
        }
    }
    if (a->bconst >= 0) std::swap(a, b);  // constant (if any) in b
    if (b->bconst >= 0) {
        const bool y = b->bconst;
        const bool same = (op == D_BAND && y) || (op == D_BOR && !y) || (op == D_BXOR && !y) ||
                          (op == D_BEQ && y);
        if (same) { retain(*a); return *a; }
        if (op == D_BAND) return bool_const(false);
        if (op == D_BOR) return bool_const(true);
        const int p = palloc();  // xor 1 / eq 0: not
        emit(M_S_NOT_B64, {P(p), P(a->pair)});
        return bool_mask(p);
    }
    const int p = palloc();
    const uint16_t m = op == D_BAND ? M_S_AND_B64 : op == D_BOR ? M_S_OR_B64 :
                       op == D_BXOR ? M_S_XOR_B64 : M_S_XNOR_B64;
    emit(m, {P(p), P(a->pair), P(b->pair)});
    return bool_mask(p);
}

// logical right shift by a constant s (0 < s < 256)
void Emitter::op_shr(int d, const Val& A, uint32_t s) {
    const uint32_t q = s >> 5, bsh = s & 31, dm = dem_[d];
    Val& R = out(d);
    std::vector<uint32_t> tmp;
    for (int k = 0; k < 8; ++k) {
        if (!((dm >> k) & 1)) continue;
        const int i = k + (int)q;
        const Limb lo = i < 8 ? A.l[i] : Limb::C(0);
        const Limb hi = i + 1 < 8 ? A.l[i + 1] : Limb::C(0);
        if (bsh == 0) {
            R.l[k] = lo;
            if (lo.is_r()) vretain(lo.v);
            continue;
        }
        if (lo.k == L_UNDEF || hi.k == L_UNDEF) fail("internal: shift of an undemanded limb");
        if (lo.is_c() && hi.is_c()) {
            R.l[k] = Limb::C((uint32_t)((((uint64_t)hi.v << 32) | lo.v) >> bsh));
            continue;
        }
        const uint32_t dst = valloc();
        if (hi.is_c(0)) emit(M_V_LSHRREV, {V(dst), IMM(bsh), V(lo.v)});
        else if (lo.is_c(0)) emit(M_V_LSHLREV, {V(dst), IMM(32 - bsh), V(hi.v)});
        else emit(M_V_ALIGNBIT, {V(dst), vi_of(hi, tmp), vi_of(lo, tmp), IMM(bsh)});
        R.l[k] = Limb::R(dst);
    }
    free_tmp(tmp);
}

// left shift by a constant s (0 < s < 256), mod 2^256
void Emitter::op_shl(int d, const Val& A, uint32_t s) {
    const uint32_t q = s >> 5, bsh = s & 31, dm = dem_[d];
    Val& R = out(d);
    std::vector<uint32_t> tmp;
    for (int k = 0; k < 8; ++k) {
        if (!((dm >> k) & 1)) continue;
        const int i = k - (int)q;
        const Limb hi = i >= 0 ? A.l[i] : Limb::C(0);       // supplies the high bits
        const Limb lo = i - 1 >= 0 ? A.l[i - 1] : Limb::C(0);
        if (bsh == 0) {
            R.l[k] = hi;
            if (hi.is_r()) vretain(hi.v);
            continue;
        }
        if (lo.k == L_UNDEF || hi.k == L_UNDEF) fail("internal: shift of an undemanded limb");
        if (lo.is_c() && hi.is_c()) {
            R.l[k] = Limb::C((uint32_t)((((uint64_t)hi.v << 32) | lo.v) >> (32 - bsh)));
            continue;
        }
        const uint32_t dst = valloc();
        if (lo.is_c(0)) emit(M_V_LSHLREV, {V(dst), IMM(bsh), V(hi.v)});
        else if (hi.is_c(0)) emit(M_V_LSHRREV, {V(dst), IMM(32 - bsh), V(lo.v)});
        else emit(M_V_ALIGNBIT, {V(dst), vi_of(hi, tmp), vi_of(lo, tmp), IMM(32 - bsh)});
        R.l[k] = Limb::R(dst);
    }
    free_tmp(tmp);
}

// per-lane shift amount B (>= 256 saturates: 0 / sign fill): limb-select network + alignbit
void Emitter::op_vshift(int d, const Val& A, const Val& B, uint8_t op) {
    const bool right = op != D_SHL_V, arith = op == D_ASHR_V;
    bool bconst = true;
    for (int k = 0; k < 8; ++k) bconst &= B.l[k].is_c();
    if (bconst) {  // uniform amount after folding: the constant-shift forms
        uint32_t hi = 0;
        for (int k = 1; k < 8; ++k) hi |= B.l[k].v;
        const uint32_t s = hi || B.l[0].v > 255u ? 256u : B.l[0].v;
        if (s == 0) { retain(A); vals_[d] = A; return; }
        if (!arith && s >= 256) {
            Val& R = out(d);
            for (int k = 0; k < 8; ++k) R.l[k] = Limb::C(0);
            return;
        }
        if (!arith) {
            if (right) op_shr(d, A, s); else op_shl(d, A, s);
            return;
        }
    }
    // Through the lane's LDS window (R_LDS): the operand's limbs go to words [D, D+8) between
    // zero words, and result limb k is the funnel of window words (base + k + 1, base + k) by
    // the bit part of the amount, base = D + q for right shifts (q = amount >> 5) and
    // D - q' for left shifts (q' = ceil(amount / 32), bit part (-amount) & 31, a right funnel);
    // amounts >= 256 read the zero words (q = q' = 8, bit part 0).  Arithmetic right shifts are
    // logical ones of x ^ s, xor s (s = the sign mask).  This replaces a three-stage select
    // network of 24 v_cndmask (4-cycle VALU) with 4 LDS writes and <= 5 LDS reads.
    uses_lds_ = true;
    std::vector<uint32_t> tmp;
    std::vector<int> tp;
    const uint32_t dm = dem_[d];
    // every lane shifting by >= 256 (a full-width symbolic amount, the common case): the result
    // is 0, or the sign for arithmetic shifts, written by the uniform branch at the end; a
    // nonzero top limb of the amount in every lane decides it with one compare
    const uint32_t l_fast = next_lbl_++, l_end = next_lbl_++;
    const bool fast_likely = B.l[7].is_r();
    if (fast_likely) {
        emit(M_V_CMP_NE, {VCC(), IMM(0), V(B.l[7].v)});
        emit(M_S_CMP_EQ_U64, {VCC(), IMM(0xFFFFFFFFu)});
        emit(M_S_CBRANCH_SCC1, {LBL(l_fast)});
        ++cold_;
    }
    const uint32_t y0 = vgpr_of(B.l[0], tmp);
    const int big = palloc();
    tp.push_back(big);
    emit(M_V_CMP_LT, {VCC(), IMM(0xFFu), V(y0)});  // 255 < y0
    emit(M_S_MOV_B64, {P(big), VCC()});
    uint32_t orr = ~0u;
    for (int k = 1; k < 8; ++k) {
        const Limb l = B.l[k];
        if (l.is_c()) {
            if (l.v) { emit(M_S_MOV_B64, {P(big), IMM(0xFFFFFFFFu)}); }
            continue;
        }
        if (orr == ~0u) {
            orr = valloc();
            tmp.push_back(orr);
            emit(M_V_MOV, {V(orr), V(l.v)});
        } else {
            emit(M_V_OR, {V(orr), V(l.v), V(orr)});
        }
    }
    if (orr != ~0u) {
        emit(M_V_CMP_NE, {VCC(), IMM(0), V(orr)});
        emit(M_S_OR_B64, {P(big), P(big), VCC()});
    }
    free_tmp(tmp);  // the amount's temporaries (y0 stays live in B or is re-read below)
    emit(M_S_CMP_EQ_U64, {P(big), IMM(0xFFFFFFFFu)});
    emit(M_S_CBRANCH_SCC1, {LBL(l_fast)});
    // operand limbs into VGPRs (ASHR: x ^ s), two at a time, each pair's temporaries freed as
    // soon as it is in LDS (register pressure: the network's eight temporaries are gone)
    uint32_t sgn = ~0u;
    if (arith) {
        sgn = valloc();
        const Opnd c7 = vi_of(A.l[7], tmp);
        if (c7.k == O_V) emit(M_V_ASHRREV, {V(sgn), IMM(31), c7});
        else emit(M_V_MOV, {V(sgn), IMM((c7.v >> 31) ? ~0u : 0u)});
        free_tmp(tmp);
    }
    for (int i = 0; i < 4; ++i) {
        uint32_t src[2];
        for (int h = 0; h < 2; ++h) {
            const Limb& l = A.l[2 * i + h];
            if (arith) {
                src[h] = valloc();
                const Opnd x = vi_of(l, tmp);
                tmp.push_back(src[h]);
                emit(M_V_XOR, {V(src[h]), x, V(sgn)});
            } else {
                src[h] = vgpr_of(l, tmp);
            }
        }
        emit(M_DS_WRITE2ST64, {V(R_LDS), V(src[0]), V(src[1]), IMM(LDS_D + 2 * i),
                               IMM(LDS_D + 2 * i + 1)});
        free_tmp(tmp);
    }
    const uint32_t y0r = vgpr_of(B.l[0], tmp);
    const uint32_t qv = valloc(), rv = valloc(), av = valloc();
    tmp.push_back(qv); tmp.push_back(rv); tmp.push_back(av);
    if (right) {
        emit(M_V_LSHRREV, {V(qv), IMM(5), V(y0r)});
        emit(M_V_AND, {V(rv), IMM(31), V(y0r)});
    } else {
        emit(M_V_ADD_U32, {V(qv), IMM(31), V(y0r)});
        emit(M_V_LSHRREV, {V(qv), IMM(5), V(qv)});
        emit(M_V_SUB_U32, {V(rv), IMM(0), V(y0r)});
        emit(M_V_AND, {V(rv), IMM(31), V(rv)});
    }
    emit(M_V_CNDMASK, {V(qv), V(qv), IMM(8), P(big)}, true);
    emit(M_V_CNDMASK, {V(rv), V(rv), IMM(0), P(big)}, true);
    // base word: D + q (right) or D - q' = 8 - q' (left); the reads add their word offsets
    if (!right) emit(M_V_SUB_U32, {V(qv), IMM(LDS_D), V(qv)});
    emit(M_V_LSHL_ADD, {V(av), V(qv), IMM(8), V(R_LDS)});
    const uint32_t off0 = right ? LDS_D : 0u;
    // window words k, k+1 of every demanded result limb k, two per read
    uint32_t need = 0;
    for (int k = 0; k < 8; ++k)
        if ((dm >> k) & 1) need |= 3u << k;
    std::vector<int> words;
    for (int j = 0; j < 9; ++j)
        if ((need >> j) & 1) words.push_back(j);
    uint32_t w[9];
    for (size_t i = 0; i < words.size(); i += 2) {
        if (i + 1 < words.size()) {
            const uint32_t pr = valloc_pair();
            tmp.push_back(pr); tmp.push_back(pr + 1);
            emit(M_DS_READ2ST64, {V(pr, 2), V(av), IMM(off0 + words[i]),
                                  IMM(off0 + words[i + 1])});
            w[words[i]] = pr;
            w[words[i + 1]] = pr + 1;
        } else {
            const uint32_t r1 = valloc();
            tmp.push_back(r1);
            emit(M_DS_READ_B32, {V(r1), V(av), IMM((off0 + words[i]) * 256u)});
            w[words[i]] = r1;
        }
    }
    emit(M_S_WAITCNT_LGKM, {IMM(0)});
    Val& R = out(d);
    for (int k = 0; k < 8; ++k) {
        if (!((dm >> k) & 1)) continue;
        const uint32_t o = valloc();
        emit(M_V_ALIGNBIT, {V(o), V(w[k + 1]), V(w[k]), V(rv)});
        if (arith) emit(M_V_XOR, {V(o), V(o), V(sgn)});
        R.l[k] = Limb::R(o);
    }
    if (fast_likely) --cold_;
    emit(M_S_BRANCH, {LBL(l_end)});
    emit(M_LABEL, {LBL(l_fast)});
    uint32_t first = ~0u;
    for (int k = 0; k < 8; ++k) {
        if (!((dm >> k) & 1)) continue;
        const uint32_t o = R.l[k].v;
        if (!arith) {
            emit(M_V_MOV, {V(o), IMM(0)});
        } else if (first != ~0u) {
            emit(M_V_MOV, {V(o), V(first)});
        } else {
            if (A.l[7].is_c()) emit(M_V_MOV, {V(o), IMM((A.l[7].v >> 31) ? ~0u : 0u)});
            else emit(M_V_ASHRREV, {V(o), IMM(31), V(A.l[7].v)});
            first = o;
        }
    }
    emit(M_LABEL, {LBL(l_end)});
    if (arith) vrelease(sgn);
    free_tmp(tmp);
    free_tmp_pairs(tp);
}

// x * y mod 2^256, product scanning over the demanded columns: column k accumulates its terms
// with v_mad_u64_u32 into a 64-bit pair; carries out of the pair (only where the column can
// exceed 2^64) are counted into the next column's high word.
void Emitter::op_mul(int d, const Val& A, const Val& B) {
    const int top = top_bit(dem_[d]);
    Val& R = out(d);
    if (top < 0) return;
    std::vector<uint32_t> tmp;
    typedef unsigned __int128 u128;
    const u128 M32 = 0xFFFFFFFFull;
    auto maxv = [&](const Limb& l) -> u128 { return l.is_c() ? (u128)l.v : M32; };
    int init = -1;          // VGPR pair (lo = carry-in, hi = carried overflows) of this column
    u128 init_max = 0;
    for (int k = 0; k <= top; ++k) {
        std::vector<std::pair<int, int>> terms;
        u128 colmax = init_max;
        for (int i = 0; i <= k; ++i) {
            const Limb x = A.l[i], y = B.l[k - i];
            if (x.k == L_UNDEF || y.k == L_UNDEF) fail("internal: mul over an undemanded limb");
            if (x.is_c(0) || y.is_c(0)) continue;
            terms.push_back({i, k - i});
            colmax += maxv(x) * maxv(y);
        }
        if (terms.empty()) {
            if (init < 0) { R.l[k] = Limb::C(0); continue; }
            // the column is its carry-in: limb = init.lo, the next carry-in = (init.hi, 0)
            R.l[k] = Limb::R((uint32_t)init);
            if (k < top) {
                const uint32_t np = valloc_pair();
                emit(M_V_MOV, {V(np), V((uint32_t)init + 1)});
                if (k + 1 < top) emit(M_V_MOV, {V(np + 1), IMM(0)});
                vrelease((uint32_t)init + 1);
                init = (int)np;
                init_max >>= 32;
            } else {
                vrelease((uint32_t)init + 1);
            }
            continue;
        }
        // overflows out of column k's pair weigh 2^(32 (k + 2)): they matter only below the
        // top column (the top column keeps just its low word, which they cannot change)
        const bool count = k + 1 < top && colmax >> 64;
        const uint32_t acc = valloc_pair();
        uint32_t np = 0;
        if (k < top) np = valloc_pair();
        bool first = true, first_count = true;
        u128 run = init_max;  // bound of the column's accumulator so far
        const u128 M64 = ((u128)1 << 64) - 1;
        for (auto [i, j] : terms) {
            Limb x = A.l[i], y = B.l[j];
            if (x.is_c() && !y.is_c()) std::swap(x, y);
            Opnd s0, s1;
            if (x.is_c() && y.is_c()) {
                s0 = staged(x.v);
                s1 = V(vgpr_of(y, tmp));
            } else if (y.is_c()) {
                s0 = staged(y.v);
                s1 = V(x.v);
            } else {
                s0 = V(x.v);
                s1 = V(y.v);
            }
            const Opnd s2 = first ? (init >= 0 ? V((uint32_t)init, 2) : IMM(0)) : V(acc, 2);
            // this product can carry out of the pair only if the bound so far plus its own
            // reaches 2^64 (the first product over a small carry-in cannot)
            const u128 pm = maxv(A.l[i]) * maxv(B.l[j]);
            const bool c_here = count && run + pm > M64;
            run = std::min(run + pm, M64);
            emit(M_V_MAD_U64_U32, {V(acc, 2), c_here ? VCC() : S(S_DIV_DUMMY, 2), s0, s1, s2});
            if (c_here) {
                if (first_count) emit(M_V_ADDC_CO, {V(np + 1), VCC(), IMM(0), IMM(0), VCC()}, true);
                else emit(M_V_ADDC_CO, {V(np + 1), VCC(), IMM(0), V(np + 1), VCC()});
                first_count = false;
            }
            first = false;
        }
        if (count && first_count) emit(M_V_MOV, {V(np + 1), IMM(0)});  // no product could carry
        if (init >= 0) {
            vrelease((uint32_t)init);
            vrelease((uint32_t)init + 1);
        }
        R.l[k] = Limb::R(acc);
        if (k < top) {
            // the top column reads only the low word of its carry-in pair
            if (!count && k + 1 < top) emit(M_V_MOV, {V(np + 1), IMM(0)});
            emit(M_V_MOV, {V(np), V(acc + 1)});
            init = (int)np;
            init_max = colmax >> 32;
        }
        vrelease(acc + 1);
    }
    free_tmp(tmp);
}

// EXP(b, e) mod 2^256 for a per-lane exponent (EVM EXP, exec.h evm_exp): square and multiply from
// the exponent's low bit up, in a loop that runs while some valid lane still has exponent bits
// left (a wave-uniform exit, as evm_exp's any_lane test); the running result, the running square
// and the exponent are loop-carried registers.  The result is the full 256 bits (the lowering
// masks narrower widths).
void Emitter::op_exp(int d, const Val& A, const Val& E) {
    uint32_t res[8], b[8], e[8];
    for (int k = 0; k < 8; ++k) {
        res[k] = valloc();
        emit(M_V_MOV, {V(res[k]), IMM(k == 0 ? 1u : 0u)});
    }
    for (int k = 0; k < 8; ++k) {
        b[k] = valloc();
        emit(M_V_MOV, {V(b[k]), src(A.l[k])});
    }
    for (int k = 0; k < 8; ++k) {
        e[k] = valloc();
        emit(M_V_MOV, {V(e[k]), src(E.l[k])});
    }
    const uint32_t t = valloc();
    const int p = palloc();
    const uint32_t top = next_lbl_++, done = next_lbl_++;
    emit(M_LABEL, {LBL(top)});
    emit(M_V_OR3, {V(t), V(e[0]), V(e[1]), V(e[2])});
    emit(M_V_OR3, {V(t), V(t), V(e[3]), V(e[4])});
    emit(M_V_OR3, {V(t), V(t), V(e[5]), V(e[6])});
    emit(M_V_OR, {V(t), V(e[7]), V(t)});
    emit(M_V_CMP_NE, {VCC(), IMM(0), V(t)});
    emit(M_S_AND_B64, {S(S_SCRATCH, 2), VCC(), S(S_VALID, 2)});
    emit(M_S_CBRANCH_SCC0, {LBL(done)});
    emit(M_V_AND, {V(t), IMM(1), V(e[0])});
    emit(M_V_CMP_NE, {P(p), IMM(0), V(t)}, true);
    Val R, B;
    R.defined = B.defined = true;
    for (int k = 0; k < 8; ++k) {
        R.l[k] = Limb::R(res[k]);
        B.l[k] = Limb::R(b[k]);
    }
    op_mul(scratch_, R, B);  // res = bit ? res * b : res
    {
        Val prod = vals_[scratch_];
        for (int k = 0; k < 8; ++k)
            emit(M_V_CNDMASK, {V(res[k]), V(res[k]), src(prod.l[k]), P(p)}, true);
        release(prod);
    }
    op_mul(scratch_, B, B);  // b = b * b
    {
        Val sq = vals_[scratch_];
        for (int k = 0; k < 8; ++k) emit(M_V_MOV, {V(b[k]), src(sq.l[k])});
        release(sq);
    }
    for (int k = 0; k < 7; ++k) emit(M_V_ALIGNBIT, {V(e[k]), V(e[k + 1]), V(e[k]), IMM(1)});
    emit(M_V_LSHRREV, {V(e[7]), IMM(1), V(e[7])});
    emit(M_S_BRANCH, {LBL(top)});
    emit(M_LABEL, {LBL(done)});
    --pref_[p];
    vrelease(t);
    for (int k = 0; k < 8; ++k) {
        vrelease(b[k]);
        vrelease(e[k]);
    }
    Val& O = out(d);
    for (int k = 0; k < 8; ++k) O.l[k] = Limb::R(res[k]);
}

// r = (u + v) mod n for u, v < n (8-limb VGPR arrays; r may be u or v): the exact sum minus n
// when the sum carries out or s - n does not borrow.  n = 0 leaves r = u + v mod 2^256.  With a
// Bool pair `when`, lanes outside it keep r.
void Emitter::addmod_regs(const uint32_t* u, const uint32_t* v, const uint32_t* n, uint32_t* r,
                          int when) {
    uint32_t sm[8], df[8];
    for (int k = 0; k < 8; ++k) {
        sm[k] = valloc();
        df[k] = valloc();
    }
    emit(M_V_ADD_CO, {V(sm[0]), VCC(), V(u[0]), V(v[0])});
    for (int k = 1; k < 8; ++k) emit(M_V_ADDC_CO, {V(sm[k]), VCC(), V(u[k]), V(v[k]), VCC()});
    const int pc = palloc();
    emit(M_S_MOV_B64, {P(pc), VCC()});
    emit(M_V_SUB_CO, {V(df[0]), VCC(), V(sm[0]), V(n[0])});
    for (int k = 1; k < 8; ++k) emit(M_V_SUBB_CO, {V(df[k]), VCC(), V(sm[k]), V(n[k]), VCC()});
    emit(M_S_ORN2_B64, {P(pc), P(pc), VCC()});  // carry out, or no borrow: s >= n
    for (int k = 0; k < 8; ++k) {
        if (when < 0) {
            emit(M_V_CNDMASK, {V(r[k]), V(sm[k]), V(df[k]), P(pc)}, true);
        } else {
            emit(M_V_CNDMASK, {V(sm[k]), V(sm[k]), V(df[k]), P(pc)}, true);
            emit(M_V_CNDMASK, {V(r[k]), V(r[k]), V(sm[k]), P(when)}, true);
        }
    }
    --pref_[pc];
    for (int k = 0; k < 8; ++k) {
        vrelease(sm[k]);
        vrelease(df[k]);
    }
}

// Yellow-paper MULMOD on operands the lowering has already reduced mod n (x, y < n; exec.h
// evm_modop): x * y mod n by double and add over y's bits from the low end, r += p and
// p = 2 p mod n, in a loop that runs while some valid lane has bits of y left.  The lowering
// selects the n = 0 result around it.
void Emitter::op_mulmod(int d, const Val& X, const Val& Y, const Val& N) {
    uint32_t r[8], p[8], y[8], n[8];
    for (int k = 0; k < 8; ++k) {
        r[k] = valloc();
        emit(M_V_MOV, {V(r[k]), IMM(0)});
        p[k] = valloc();
        emit(M_V_MOV, {V(p[k]), src(X.l[k])});
        y[k] = valloc();
        emit(M_V_MOV, {V(y[k]), src(Y.l[k])});
        if (N.l[k].is_r()) {  // read where it lives (never written here)
            n[k] = N.l[k].v;
            vretain(n[k]);
        } else {
            n[k] = valloc();
            emit(M_V_MOV, {V(n[k]), src(N.l[k])});
        }
    }
    const uint32_t t = valloc();
    const int pb = palloc();
    const uint32_t top = next_lbl_++, done = next_lbl_++;
    emit(M_LABEL, {LBL(top)});
    emit(M_V_OR3, {V(t), V(y[0]), V(y[1]), V(y[2])});
    emit(M_V_OR3, {V(t), V(t), V(y[3]), V(y[4])});
    emit(M_V_OR3, {V(t), V(t), V(y[5]), V(y[6])});
    emit(M_V_OR, {V(t), V(y[7]), V(t)});
    emit(M_V_CMP_NE, {VCC(), IMM(0), V(t)});
    emit(M_S_AND_B64, {S(S_SCRATCH, 2), VCC(), S(S_VALID, 2)});
    emit(M_S_CBRANCH_SCC0, {LBL(done)});
    emit(M_V_AND, {V(t), IMM(1), V(y[0])});
    emit(M_V_CMP_NE, {P(pb), IMM(0), V(t)}, true);
    addmod_regs(r, p, n, r, pb);  // r = bit ? r + p mod n : r
    addmod_regs(p, p, n, p);      // p = 2 p mod n
    for (int k = 0; k < 7; ++k) emit(M_V_ALIGNBIT, {V(y[k]), V(y[k + 1]), V(y[k]), IMM(1)});
    emit(M_V_LSHRREV, {V(y[7]), IMM(1), V(y[7])});
    emit(M_S_BRANCH, {LBL(top)});
    emit(M_LABEL, {LBL(done)});
    --pref_[pb];
    vrelease(t);
    for (int k = 0; k < 8; ++k) {
        vrelease(p[k]);
        vrelease(y[k]);
        vrelease(n[k]);
    }
    Val& O = out(d);
    for (int k = 0; k < 8; ++k) O.l[k] = Limb::R(r[k]);
}

// The result stays where the subroutine leaves it (the quotient / signed remainders in DQ, the
// unsigned remainder in DR) until the next call: limbs of live values that sit in the
// subroutine's registers are moved out just before it (rescue_div_regs).
void Emitter::rescue_div_regs(int cur, uint32_t end) {
    std::vector<std::pair<uint32_t, uint32_t>> moved;  // (div register, new register)
    for (size_t r = 0; r < vals_.size(); ++r) {
        Val& v = vals_[r];
        if (!v.defined || v.is_bool || last_[r] <= cur) continue;
        for (Limb& l : v.l) {
            if (!l.is_r() || l.v < R_DIV0 || l.v >= end) continue;
            uint32_t nr = ~0u;
            for (auto& m : moved)
                if (m.first == l.v) nr = m.second;
            if (nr == ~0u) {
                nr = valloc();
                emit(M_V_MOV, {V(nr), V(l.v)});
                moved.push_back({l.v, nr});
            } else {
                vretain(nr);
            }
            l.v = nr;
        }
    }
}

void Emitter::op_div(int d, int a, int b, int cidx, uint32_t kind, int cur) {
    calls_div_ = true;
    // values still live after this call move out of the subroutine's registers first; then y
    // before x, so an operand sitting in R (a previous remainder read for the last time here)
    // is read before R is overwritten
    rescue_div_regs(cur);
    const Val& A = val(a);
    const Val B = cidx >= 0 ? const_val(cidx) : val(b);
    // bvsdiv / bvsrem / bvsmod of operands whose sign bits are known clear are bvudiv / bvurem
    // (every SMT-LIB sign rule reduces to the unsigned form for non-negative x and y)
    if (kind >= 2 && A.l[7].is_c() && !(A.l[7].v >> 31) && B.l[7].is_c() && !(B.l[7].v >> 31))
        kind = kind == 2 ? 0u : 1u;
    if (kind < 2) {
        for (int k = 0; k < 8; ++k) emit(M_V_MOV, {V(R_DY + k), src(B.l[k])});
        for (int k = 0; k < 8; ++k) emit(M_V_MOV, {V(R_DR + k), src(A.l[k])});
    } else {
        // signed kinds: the subroutine divides |x| by |y| and takes the signs from v[R_SX],
        // v[R_SY]; |v| = (v ^ m) - m (m = the sign mask) is formed here, reading the operand
        // where it lives, instead of a copy plus the same work inside the subroutine.  Both sign
        // masks first (an operand may sit in R, which the second load overwrites).
        auto sign_of = [&](const Val& X, uint32_t sreg) {
            if (X.l[7].is_c()) emit(M_V_MOV, {V(sreg), IMM((X.l[7].v >> 31) ? ~0u : 0u)});
            else emit(M_V_ASHRREV, {V(sreg), IMM(31), V(X.l[7].v)});
        };
        auto load_abs = [&](uint32_t base, uint32_t sreg, const Val& X) {
            bool allc = true;
            for (int k = 0; k < 8; ++k) allc = allc && X.l[k].is_c();
            const bool known = X.l[7].is_c(), neg = known && (X.l[7].v >> 31);
            if (allc) {  // |X| on the host
                uint32_t c[8];
                uint64_t borrow = neg ? 1 : 0;
                for (int k = 0; k < 8; ++k) {
                    const uint64_t t = (uint64_t)(neg ? ~X.l[k].v : X.l[k].v) + borrow;
                    c[k] = (uint32_t)t;
                    borrow = t >> 32;
                }
                for (int k = 0; k < 8; ++k) emit(M_V_MOV, {V(base + k), IMM(c[k])});
                return;
            }
            if (known && !neg) {
                for (int k = 0; k < 8; ++k) emit(M_V_MOV, {V(base + k), src(X.l[k])});
                return;
            }
            for (int k = 0; k < 8; ++k) {
                if (X.l[k].is_c(0)) emit(M_V_MOV, {V(base + k), V(sreg)});
                else emit(M_V_XOR, {V(base + k), src(X.l[k]), V(sreg)});
            }
            emit(M_V_SUB_CO, {V(base), VCC(), V(base), V(sreg)});
            for (int k = 1; k < 8; ++k)
                emit(M_V_SUBB_CO, {V(base + k), VCC(), V(base + k), V(sreg), VCC()});
        };
        sign_of(B, R_SY);
        sign_of(A, R_SX);
        load_abs(R_DY, R_SY, B);
        load_abs(R_DR, R_SX, A);
    }
    emit(M_S_MOV_B32, {S(S_DIV_KIND), IMM(kind)});
    emit(M_CALL_DIV, {IMM((uint32_t)code_.size())});
    Val& R = out(d);
    const uint32_t dm = dem_[d], base = kind == 1 ? R_DR : R_DQ;
    for (int k = 0; k < 8; ++k)
        if ((dm >> k) & 1) R.l[k] = Limb::R(base + k);
}

// KECCAK (exec.h keccak_words): the caller absorbs the message words straight into the
// subroutine's state registers (byte-swapped by v_perm_b32; constants swapped on the host),
// zeroes the rest, sets the pad bits, calls the permutation and byte-swaps the first 8 output
// words out of wherever the subroutine's renaming leaves them.
void Emitter::op_keccak(const SsaInsn& v, int cur) {
    calls_kec_ = true;
    rescue_div_regs(cur, R_TEMP_KEC);
    const uint32_t nw = (v.w1raw >> 8) & 3u, full = (v.w1raw >> 10) & 1u;
    if (nw < 1 || nw > 3) fail("keccak: bad word count");
    const int ops[3] = {v.a, v.b, v.c};
    // message limbs; a dying operand inside the state registers is copied out first (the
    // absorb overwrites those registers)
    Limb src[3][8];
    std::vector<uint32_t> tmp;
    for (uint32_t i = 0; i < nw; ++i) {
        const Val& W = val(ops[i]);
        for (int k = 0; k < 8; ++k) {
            src[i][k] = W.l[k];
            if (src[i][k].k == L_UNDEF) fail("internal: keccak over an undemanded limb");
            if (src[i][k].is_r() && src[i][k].v >= R_KEC0 && src[i][k].v < R_TEMP_KEC) {
                const uint32_t r = valloc();
                tmp.push_back(r);
                emit(M_V_MOV, {V(r), V(src[i][k].v)});
                src[i][k] = Limb::R(r);
            }
        }
    }
    emit(M_S_MOV_B32, {S(S_PERM_SEL), IMM(0x00010203u)});  // byte swap
    for (uint32_t i = 0; i < nw; ++i)
        for (int t = 0; t < 4; ++t)
            for (int h = 0; h < 2; ++h) {
                const uint32_t dst = R_KEC0 + 2 * (4 * i + t) + h;
                const Limb& l = src[i][h ? 6 - 2 * t : 7 - 2 * t];
                if (l.is_c()) emit(M_V_MOV, {V(dst), IMM(__builtin_bswap32(l.v))});
                else emit(M_V_PERM, {V(dst), IMM(0), V(l.v), S(S_PERM_SEL)});
            }
    free_tmp(tmp);
    for (uint32_t lane = 4 * nw; lane < 25; ++lane)
        for (uint32_t h = 0; h < 2; ++h) {
            uint32_t x = 0;
            if (full && lane == 4 * nw && h == 0) x = 1u;         // pad byte 0x01
            if (lane == 16 && h == 1) x = 0x80000000u;            // byte 135: 0x80
            emit(M_V_MOV, {V(R_KEC0 + 2 * lane + h), IMM(x)});
        }
    emit(M_CALL_KEC, {IMM((uint32_t)code_.size())});
    const KecCode& kc = kec_routine();
    Val& R = out(v.d);
    const uint32_t dm = dem_[v.d];
    for (int k = 0; k < 8; ++k) {
        if (!((dm >> k) & 1)) continue;
        const uint32_t r = valloc();
        emit(M_V_PERM, {V(r), IMM(0), V(kc.out[7 - k]), S(S_PERM_SEL)});
        R.l[k] = Limb::R(r);
    }
}

void Emitter::demand() {
    const auto& code = st_.code;
    const int nv = st_.n_vregs;
    dem_.assign(nv, 0);
    if (st_.root >= 0) dem_[st_.root] = 0xFF;
    auto D = [&](int r, uint32_t m) { if (r >= 0) dem_[r] |= (uint8_t)m; };
    for (size_t i = code.size(); i-- > 0;) {
        const SsaInsn& v = code[i];
        const uint32_t dd = dem_[v.d];
        const uint8_t op = v.op;
        switch (op) {
            case D_NOP: D(v.a, dd); break;
            case D_ADD_R: case D_SUB_R: case D_RSUB_R: case D_MUL_R:
                D(v.a, prefix_mask(dd));
                D(v.b, prefix_mask(dd));
                break;
            case D_AND_R: case D_OR_R: case D_XOR_R: {
                uint32_t ma = dd;
                if (v.cidx >= 0) {
                    for (int k = 0; k < 8; ++k) {
                        const uint32_t c = pool_[8ull * (uint32_t)v.cidx + k];
                        if ((op == D_AND_R && c == 0) || (op == D_OR_R && c == ~0u))
                            ma &= ~(1u << k);
                    }
                }
                D(v.a, ma);
                D(v.b, dd);
                break;
            }
            case D_ITE: D(v.b, dd); D(v.c, dd); break;
            case D_EXP: case D_MULMOD:
                D(v.a, 0xFF);
                D(v.b, 0xFF);
                D(v.c, 0xFF);
                break;
            case D_SHL_V: case D_LSHR_V: case D_ASHR_V:
                D(v.a, 0xFF);
                D(v.b, 0xFF);
                break;
            default:
                if (op >= D_SHR0 && op <= D_SHR7) {
                    const uint32_t s = 32u * (op - D_SHR0) + (v.aux & 31u);
                    const uint32_t q = s >> 5, bsh = s & 31;
                    uint32_t m = 0;
                    for (int k = 0; k < 8; ++k)
                        if ((dd >> k) & 1) {
                            if (k + q < 8) m |= 1u << (k + q);
                            if (bsh && k + q + 1 < 8) m |= 1u << (k + q + 1);
                        }
                    D(v.a, m);
                } else if (op >= D_SHL0 && op <= D_SHL7) {
                    const uint32_t p = op - D_SHL0, f = v.aux & 31u;
                    const uint32_t s = f ? 32u * p + 32u - f : 32u * (p + 1u);
                    if (s < 256) {
                        const int q = (int)(s >> 5), bsh = (int)(s & 31);
                        uint32_t m = 0;
                        for (int k = 0; k < 8; ++k)
                            if ((dd >> k) & 1) {
                                if (k - q >= 0) m |= 1u << (k - q);
                                if (bsh && k - q - 1 >= 0) m |= 1u << (k - q - 1);
                            }
                        D(v.a, m);
                    }
                } else if ((op >= D_EQ_R && op <= D_SGE_C) ||
                           (op >= D_UDIV_R && op <= D_SMOD_C)) {
                    D(v.a, 0xFF);
                    D(v.b, 0xFF);
                } else if (op == D_KECCAK) {
                    D(v.a, 0xFF);
                    D(v.b, 0xFF);
                    D(v.c, 0xFF);
                } else {  // Bool ops, constants
                    D(v.a, 0);
                }
                break;
        }
    }
}

uint64_t Emitter::op_valu[256], Emitter::op_wide[256], Emitter::op_count[256];

// Short-circuit test after a conjunct (or partial conjunction): leave the tape when no valid lane
// of the wave is still true.  s_and_b64 sets SCC = (result != 0).
void Emitter::sc_check(const Val& v) {
    if (!v.is_bool || v.bconst == 1) return;
    sc_used_ = true;
    if (v.bconst == 0) {
        emit(M_S_BRANCH, {LBL(LBL_SC_SKIP)});
        return;
    }
    emit(M_S_AND_B64, {S(S_SCRATCH, 2), P(v.pair), S(S_VALID, 2)});
    emit(M_S_CBRANCH_SCC0, {LBL(LBL_SC_SKIP)});
}

namespace {

// Rough VALU cost of an SSA op in the native code (jit_mix.json's per-op averages), for ordering
// conjuncts only.
double sc_cost(const SsaInsn& v) {
    const uint8_t op = v.op;
    if (op == D_MUL_R) return 60;
    if (op >= D_UDIV_R && op <= D_SMOD_C) return 130;
    if (op == D_SHL_V || op == D_LSHR_V || op == D_ASHR_V) return 35;
    if (op == D_KECCAK) return 7000;
    if (op == D_EXP) return 40000;
    if (op == D_MULMOD) return 20000;
    if (op == D_ADD_R || op == D_SUB_R || op == D_RSUB_R) return 10;
    if (op >= D_EQ_R && op <= D_SGE_C) return 9;
    if (op == D_AND_R || op == D_OR_R || op == D_XOR_R || op == D_ITE) return 6;
    if ((op >= D_SHR0 && op <= D_SHR7) || (op >= D_SHL0 && op <= D_SHL7)) return 4;
    if (op >= D_BAND && op <= D_BITE) return 1;
    return 0.5;
}

}  // namespace

// Order the conjuncts of a root AND chain for short-circuit evaluation.  Each conjunct needs the
// SSA instructions of its operand cone that are not computed yet; conjuncts are taken greedily by
// (cost of that remainder) / (probability the conjunct ends the evaluation), the classic order
// for filters.  The probability is measured on sample rows (sample_bools: uniform columns, by
// the device's semantics), per 64-row wave and conditioned on the conjuncts already placed;
// without samples, static guesses: an equality rarely holds (0.02), its negation nearly always
// (0.98), anything else half the time.  The order only moves work, never changes a result.  The
// chain's ANDs are rebuilt in that order (the last one defines the root), each operand cone is
// emitted just before the AND that consumes it, in the original relative order.
bool order_search_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("MH_SC_SEARCH");
        return e == nullptr || atoi(e) != 0;
    }();
    return on;
}

bool schedule_impl(const SsaTape& st, const std::vector<uint32_t>& pool, uint32_t sample_rows,
                   const std::vector<double>* insn_cost, SsaTape& out,
                   std::vector<uint8_t>& check) {
    auto cost = [&](int i) {
        return insn_cost && (size_t)i < insn_cost->size() ? (*insn_cost)[i] + 0.5
                                                           : sc_cost(st.code[i]);
    };
    const auto& code = st.code;
    const int n = (int)code.size();
    if (st.root < 0 || !st.root_bool || n == 0) return false;
    std::vector<int> def(st.n_vregs, -1), uses(st.n_vregs, 0);
    for (int i = 0; i < n; ++i) {
        if (code[i].d < 0 || code[i].d >= st.n_vregs) return false;
        def[code[i].d] = i;
        for (int r : {code[i].a, code[i].b, code[i].c})
            if (r >= 0 && r < st.n_vregs) ++uses[r];
    }
    if (def[st.root] < 0 || code[def[st.root]].op != D_BAND) return false;
    // the chain: BANDs reachable from the root through single-use BANDs
    std::vector<char> chain(n, 0);
    std::vector<int> conj, stack{st.root};
    while (!stack.empty()) {
        const int r = stack.back();
        stack.pop_back();
        const int i = r >= 0 ? def[r] : -1;
        if (i >= 0 && code[i].op == D_BAND && (r == st.root || uses[r] == 1)) {
            chain[i] = 1;
            stack.push_back(code[i].b);
            stack.push_back(code[i].a);
        } else if (std::find(conj.begin(), conj.end(), r) == conj.end()) {
            conj.push_back(r);
        }
    }
    if (conj.size() < 2) return false;
    for (int r : conj)
        if (r < st.n_pinned || def[r] < 0) return false;
    // operand cone of each conjunct (chain ANDs excluded), in instruction order
    std::vector<std::vector<int>> cone(conj.size());
    for (size_t k = 0; k < conj.size(); ++k) {
        std::vector<char> seen(n, 0);
        std::vector<int> st2{def[conj[k]]};
        seen[def[conj[k]]] = 1;
        while (!st2.empty()) {
            const int i = st2.back();
            st2.pop_back();
            cone[k].push_back(i);
            for (int r : {code[i].a, code[i].b, code[i].c}) {
                if (r < 0 || def[r] < 0 || seen[def[r]]) continue;
                if (chain[def[r]]) return false;  // a chain AND used inside a conjunct
                seen[def[r]] = 1;
                st2.push_back(def[r]);
            }
        }
        std::sort(cone[k].begin(), cone[k].end());
    }
    auto reject_p = [&](int r) -> double {
        const SsaInsn& v = code[def[r]];
        double pass = 0.5;
        if (v.op == D_EQ_R) pass = 0.02;
        else if (v.op == D_FALSE) pass = 0.0;
        else if (v.op == D_TRUE) pass = 1.0;
        else if (v.op == D_BNOT && v.a >= 0 && def[v.a] >= 0 && code[def[v.a]].op == D_EQ_R)
            pass = 0.98;
        return std::max(1.0 - pass, 0.02);
    };
    // measured rejection: each conjunct on sample rows, conditioned on the rows that passed the
    // conjuncts already placed (correlated conjuncts), counted in waves of 64 rows as the device
    // leaves a tape per wave; the static guess when no sample row is left
    std::vector<std::vector<uint8_t>> bits;
    if (sample_rows) sample_bools(st, pool, sample_rows, 0x5A4D91C3E7B2F601ull, conj, bits);
    std::vector<uint8_t> alive(sample_rows, 1);
    uint32_t n_alive = sample_rows;
    std::vector<char> done(n, 0), taken(conj.size(), 0);
    std::vector<int> order;
    for (size_t step = 0; step < conj.size(); ++step) {
        int best = -1;
        double best_s = 0;
        for (size_t k = 0; k < conj.size(); ++k) {
            if (taken[k]) continue;
            double c = 0;
            for (int i : cone[k])
                if (!done[i]) c += cost(i);
            double rej = reject_p(conj[k]);
            if (n_alive) {
                uint32_t fails = 0;
                for (uint32_t r = 0; r < sample_rows; ++r) fails += alive[r] && !bits[k][r];
                rej = (fails + 0.5) / (n_alive + 1.0);
                {  // a wave leaves only when all its rows fail: the fraction of the sample's
                   // 64-row waves still alive that this conjunct would end, the row rate as
                   // the tie-breaker when it ends none
                    uint32_t wa = 0, wk = 0;
                    for (uint32_t w0 = 0; w0 + 64 <= sample_rows; w0 += 64) {
                        bool al = false, st = false;
                        for (uint32_t r = w0; r < w0 + 64; ++r) {
                            al |= alive[r] != 0;
                            st |= alive[r] && bits[k][r];
                        }
                        wa += al;
                        wk += al && !st;
                    }
                    if (wa) rej = (wk + rej) / (wa + 1.0);
                }
            }
            const double sc = c / rej;
            if (best < 0 || sc < best_s) { best = (int)k; best_s = sc; }
        }
        taken[best] = 1;
        order.push_back(best);
        for (int i : cone[best]) done[i] = 1;
        if (n_alive)
            for (uint32_t r = 0; r < sample_rows; ++r)
                if (alive[r] && !bits[best][r]) { alive[r] = 0; --n_alive; }
    }
    // local search on the sample: the expected VALU of an order is the sum over conjuncts of
    // (the cost of its cone's new part) x (fraction of the sample's 64-row waves still alive
    // before it); moving a conjunct to another position is kept when that sum drops
    if (sample_rows >= 64 && conj.size() > 2 && order_search_enabled()) {
        const uint32_t nw = sample_rows / 64;
        auto expected = [&](const std::vector<int>& ord) {
            std::vector<char> dn(n, 0);
            std::vector<uint8_t> al(sample_rows, 1);
            double total = 0;
            uint32_t waves = nw;
            for (int k : ord) {
                double c = 0;
                for (int i : cone[k])
                    if (!dn[i]) { c += cost(i); dn[i] = 1; }
                total += c * (double)waves / (double)nw;
                waves = 0;
                for (uint32_t w0 = 0; w0 + 64 <= sample_rows; w0 += 64) {
                    bool any = false;
                    for (uint32_t r = w0; r < w0 + 64; ++r) {
                        al[r] = al[r] && bits[k][r];
                        any |= al[r] != 0;
                    }
                    waves += any;
                }
            }
            return total;
        };
        double best_e = expected(order);
        for (int pass = 0; pass < 4; ++pass) {
            bool improved = false;
            for (size_t i = 0; i < order.size(); ++i)
                for (size_t j = 0; j < order.size(); ++j) {
                    if (i == j) continue;
                    std::vector<int> o2 = order;
                    const int k = o2[i];
                    o2.erase(o2.begin() + (long)i);
                    o2.insert(o2.begin() + (long)j, k);
                    const double e = expected(o2);
                    if (e < best_e - 1e-9) { best_e = e; order.swap(o2); improved = true; }
                }
            if (!improved) break;
        }
    }
    // every instruction is either in the chain or in some cone (dead code was dropped)
    for (int i = 0; i < n; ++i)
        if (!chain[i] && !done[i]) return false;
    std::vector<int> chain_d;
    for (int i = 0; i < n; ++i)
        if (chain[i] && code[i].d != st.root) chain_d.push_back(code[i].d);
    if (chain_d.size() + 2 < conj.size()) return false;
    out = st;
    out.code.clear();
    check.assign(st.n_vregs, 0);
    std::fill(done.begin(), done.end(), 0);
    int acc = -1;
    size_t next_d = 0;
    for (size_t s = 0; s < order.size(); ++s) {
        const int k = order[s];
        for (int i : cone[k])
            if (!done[i]) { out.code.push_back(code[i]); done[i] = 1; }
        if (acc < 0) {
            acc = conj[k];
            check[acc] = 1;
            continue;
        }
        SsaInsn a{};
        a.op = D_BAND;
        a.d = s + 1 == order.size() ? st.root : chain_d[next_d++];
        a.a = acc;
        a.b = conj[k];
        a.c = -1;
        a.width = 1;
        a.cidx = -1;
        out.code.push_back(a);
        acc = a.d;
        if (acc != st.root) check[acc] = 1;
    }
    return true;
}

TapeCode Emitter::run() {
    TapeCode tc;
    tc.alg_ops = st_.alg_ops;
    try {
        const auto& code = st_.code;
        const int nv = st_.n_vregs;
        if (insn_cost_) insn_cost_->assign(code.size(), 0.0);
        const uint32_t n_pin = pinned_cols(n_vars_);
        if (st_.n_pinned != (int)n_pin) fail("assignment columns not pinned as the module pins them");
        bool has_div = false, has_kec = false;
        for (const SsaInsn& v : code) {
            if (v.op == D_KECCAK) { has_kec = true; continue; }
            if (v.op == D_LOADVAR || v.op == D_EXP) continue;
            if (v.op == D_MULMOD && (v.aux & 2u)) continue;  // operands reduced by the lowering
            if (v.op >= D_FIRST_COMPLEX) {
                fail(v.op == D_EXP ? "EXP with a symbolic exponent (interpreter only)"
                     : v.op == D_MULMOD ? "MULMOD (interpreter only)"
                                        : "complex op (interpreter only)");
            }
            if (v.op >= D_UDIV_R && v.op <= D_SMOD_C) has_div = true;
        }
        // without pinned columns v[R_COL0..R_DIV0) are free for temporaries (below the
        // subroutines' registers only when no subroutine is called)
        vbase_ = has_kec ? R_TEMP_KEC : has_div ? R_TEMP0 : n_pin ? R_TEMP_NODIV : R_COL0;
        vmax_ = std::min<uint32_t>(has_kec ? std::max(opt_.max_vgpr, opt_.max_vgpr_keccak)
                                           : opt_.max_vgpr, 256);
        if (vmax_ <= vbase_ + 16) fail("VGPR budget too small");
        vhigh_ = R_COL0 + 8 * n_pin;
        vals_.assign(nv, Val());
        for (int c = 0; c < st_.n_pinned; ++c) {
            Val& v = vals_[c];
            v.defined = true;
            for (int k = 0; k < 8; ++k) v.l[k] = Limb::R(R_COL0 + 8u * (uint32_t)c + k);
        }
        last_.assign(nv, -1);
        for (int i = 0; i < (int)code.size(); ++i)
            for (int r : {code[i].a, code[i].b, code[i].c})
                if (r >= 0) last_[r] = i;
        if (st_.root >= 0) last_[st_.root] = INT_MAX;
        demand();
        // op_exp's products: one virtual register past the tape's, all limbs demanded
        scratch_ = nv;
        vals_.push_back(Val());
        last_.push_back(-1);
        dem_.push_back(0xFF);
        for (int i = 0; i < (int)code.size(); ++i) {
            const SsaInsn& v = code[i];
            const uint8_t op = v.op;
            cur_op_ = op;
            const uint32_t valu_before = n_valu_, cold_before = n_valu_cold_;
            ++op_count[op];
            auto Y = [&]() -> Val { return v.cidx >= 0 ? const_val(v.cidx) : val(v.b); };
            switch (op) {
                case D_NOP: {
                    const Val& a = val(v.a);
                    retain(a);
                    vals_[v.d] = a;
                    break;
                }
                case D_LOADC: vals_[v.d] = const_val(v.cidx); break;
                case D_LOADVAR: {  // a column not pinned: the demanded limbs, one load each
                    const uint32_t dm = dem_[v.d];
                    Val& R = out(v.d);
                    for (int k = 0; k < 8; ++k)
                        if ((dm >> k) & 1u) {
                            const uint32_t r = valloc();
                            emit(M_LOADCOL, {V(r), IMM(8u * v.aux + (uint32_t)k)});
                            R.l[k] = Limb::R(r);
                        }
                    if (dm) emit(M_S_WAITCNT_VM, {IMM(0)});
                    break;
                }
                case D_TRUE: vals_[v.d] = bool_const(true); break;
                case D_FALSE: vals_[v.d] = bool_const(false); break;
                case D_ADD_R: op_addsub(v.d, val(v.a), Y(), false); break;
                case D_SUB_R: op_addsub(v.d, val(v.a), Y(), true); break;
                case D_RSUB_R: op_addsub(v.d, Y(), val(v.a), true); break;
                case D_AND_R: op_logic(v.d, val(v.a), Y(), 0); break;
                case D_OR_R: op_logic(v.d, val(v.a), Y(), 1); break;
                case D_XOR_R: op_logic(v.d, val(v.a), Y(), 2); break;
                case D_EQ_R: vals_[v.d] = op_eq(val(v.a), Y()); break;
                case D_ULT_R: vals_[v.d] = op_ult(val(v.a), Y(), false, false); break;
                case D_UGE_R: vals_[v.d] = op_ult(val(v.a), Y(), false, true); break;
                case D_UGT_R: vals_[v.d] = op_ult(Y(), val(v.a), false, false); break;
                case D_ULE_R: vals_[v.d] = op_ult(Y(), val(v.a), false, true); break;
                case D_SLT_R: vals_[v.d] = op_ult(val(v.a), Y(), true, false); break;
                case D_SGE_R: vals_[v.d] = op_ult(val(v.a), Y(), true, true); break;
                case D_SGT_R: vals_[v.d] = op_ult(Y(), val(v.a), true, false); break;
                case D_SLE_R: vals_[v.d] = op_ult(Y(), val(v.a), true, true); break;
                case D_BAND: case D_BOR: case D_BXOR: case D_BEQ:
                    vals_[v.d] = op_bool2(op, val(v.a), val(v.b));
                    break;
                case D_BNOT: {
                    const Val& a = val(v.a);
                    if (a.bconst >= 0) {
                        vals_[v.d] = bool_const(!a.bconst);
                    } else {
                        const int p = palloc();
                        emit(M_S_NOT_B64, {P(p), P(a.pair)});
                        vals_[v.d] = bool_mask(p);
                    }
                    break;
                }
                case D_ITE: op_ite(v.d, val(v.a), val(v.b), val(v.c)); break;
                case D_BITE: vals_[v.d] = op_bite(val(v.a), val(v.b), val(v.c)); break;
                case D_MUL_R: op_mul(v.d, val(v.a), Y()); break;
                case D_SHL_V: case D_LSHR_V: case D_ASHR_V:
                    op_vshift(v.d, val(v.a), val(v.b), op);
                    break;
                case D_UDIV_R: case D_UREM_R: case D_SDIV_R: case D_SREM_R: case D_SMOD_R:
                    op_div(v.d, v.a, v.b, v.cidx, (uint32_t)(op - D_UDIV_R) >> 1, i);
                    break;
                case D_KECCAK: op_keccak(v, i); break;
                case D_EXP: op_exp(v.d, val(v.a), Y()); break;
                case D_MULMOD: op_mulmod(v.d, val(v.a), val(v.b), val(v.c)); break;
                default:
                    if (op >= D_SHR0 && op <= D_SHR7) {
                        const uint32_t s = 32u * (op - D_SHR0) + (v.aux & 31u);
                        if (s == 0) { const Val& a = val(v.a); retain(a); vals_[v.d] = a; }
                        else op_shr(v.d, val(v.a), s);
                    } else if (op >= D_SHL0 && op <= D_SHL7) {
                        const uint32_t p = op - D_SHL0, f = v.aux & 31u;
                        const uint32_t s = f ? 32u * p + 32u - f : 32u * (p + 1u);
                        if (s >= 256) {
                            Val& R = out(v.d);
                            for (int k = 0; k < 8; ++k) R.l[k] = Limb::C(0);
                        } else {
                            op_shl(v.d, val(v.a), s);
                        }
                    } else {
                        fail("op " + std::to_string(op) + " not in the JIT");
                    }
                    break;
            }
            vals_[v.d].defined = true;
            // operands whose last use this was
            int seen[3] = {-1, -1, -1};
            int ns = 0;
            for (int r : {v.a, v.b, v.c}) {
                if (r < 0 || last_[r] != i) continue;
                bool dup = false;
                for (int j = 0; j < ns; ++j) dup |= seen[j] == r;
                if (dup) continue;
                seen[ns++] = r;
                release(vals_[r]);
            }
            if (check_ && (*check_)[v.d]) sc_check(vals_[v.d]);
            if (insn_cost_) {
                // a division-family call runs ~90 VALU in the subroutine (tests/tools/jit_mix.py)
                const bool call = op >= D_UDIV_R && op <= D_SMOD_C;
                (*insn_cost_)[i] = (double)(n_valu_ - valu_before) -
                                   (double)(n_valu_cold_ - cold_before) + (call ? 90.0 : 0.0) +
                                   (op == D_KECCAK ? 7000.0 : 0.0);
            }
        }
        // root
        const Val& root = val(st_.root);
        tc.root_bool = root.is_bool;
        if (root.is_bool) {
            if (root.bconst >= 0) emit(M_S_MOV_B64, {S(S_RES, 2), IMM(root.bconst ? ~0u : 0u)});
            else emit(M_S_MOV_B64, {S(S_RES, 2), P(root.pair)});
            if (sc_used_) {  // a wave with no valid lane left: root mask 0
                emit(M_S_BRANCH, {LBL(LBL_SC_END)});
                emit(M_LABEL, {LBL(LBL_SC_SKIP)});
                emit(M_S_MOV_B64, {S(S_RES, 2), IMM(0)});
                emit(M_LABEL, {LBL(LBL_SC_END)});
            }
            for (int k = 0; k < 8; ++k) { tc.root_limbs[k] = ~0u; tc.root_const[k] = 0; }
        } else {
            // hit = value != 0
            uint32_t acc = ~0u, cacc = 0;
            for (int k = 0; k < 8; ++k) {
                const Limb l = root.l[k];
                if (l.is_c()) { cacc |= l.v; tc.root_limbs[k] = ~0u; tc.root_const[k] = l.v; continue; }
                tc.root_limbs[k] = l.v;
                tc.root_const[k] = 0;
                if (acc == ~0u) { acc = valloc(); emit(M_V_MOV, {V(acc), V(l.v)}); }
                else emit(M_V_OR, {V(acc), V(l.v), V(acc)});
            }
            if (cacc) emit(M_S_MOV_B64, {S(S_RES, 2), IMM(~0u)});
            else if (acc == ~0u) emit(M_S_MOV_B64, {S(S_RES, 2), IMM(0)});
            else {
                emit(M_V_CMP_NE, {VCC(), IMM(0), V(acc)});
                emit(M_S_MOV_B64, {S(S_RES, 2), VCC()});
            }
        }
        tc.ok = true;
    } catch (const Fail& f) {
        tc.ok = false;
        tc.why = f.why;
        code_.clear();
    }
    tc.code.swap(code_);
    tc.max_vgpr = vhigh_;
    tc.calls_div = calls_div_;
    tc.uses_lds = uses_lds_;
    tc.calls_kec = calls_kec_;
    tc.n_valu = n_valu_;
    tc.n_valu_wide = n_wide_;
    tc.n_salu = n_salu_;
    return tc;
}

// ---- printer ---------------------------------------------------------------------------
struct OpInfo {
    const char* name;
};
const char* op_name(uint16_t op) {
    switch (op) {
        case M_V_MOV: return "v_mov_b32";
        case M_V_ADD_U32: return "v_add_u32";
        case M_V_SUB_U32: return "v_sub_u32";
        case M_V_SUBREV_U32: return "v_subrev_u32";
        case M_V_ADD_CO: return "v_add_co_u32";
        case M_V_ADDC_CO: return "v_addc_co_u32";
        case M_V_SUB_CO: return "v_sub_co_u32";
        case M_V_SUBB_CO: return "v_subb_co_u32";
        case M_V_SUBREV_CO: return "v_subrev_co_u32";
        case M_V_SUBBREV_CO: return "v_subbrev_co_u32";
        case M_V_AND: return "v_and_b32";
        case M_V_OR: return "v_or_b32";
        case M_V_XOR: return "v_xor_b32";
        case M_V_NOT: return "v_not_b32";
        case M_V_XNOR: return "v_xnor_b32";
        case M_V_OR3: return "v_or3_b32";
        case M_V_ALIGNBIT: return "v_alignbit_b32";
        case M_V_LSHLREV: return "v_lshlrev_b32";
        case M_V_LSHRREV: return "v_lshrrev_b32";
        case M_V_ASHRREV: return "v_ashrrev_i32";
        case M_V_CNDMASK: return "v_cndmask_b32";
        case M_V_CMP_EQ: return "v_cmp_eq_u32";
        case M_V_CMP_NE: return "v_cmp_ne_u32";
        case M_V_CMP_LT: return "v_cmp_lt_u32";
        case M_V_CMP_LE: return "v_cmp_le_u32";
        case M_V_CMP_GT: return "v_cmp_gt_u32";
        case M_V_CMP_GE: return "v_cmp_ge_u32";
        case M_V_CMP_LT_I32: return "v_cmp_lt_i32";
        case M_V_CMP_GT_I32: return "v_cmp_gt_i32";
        case M_V_MAD_U64_U32: return "v_mad_u64_u32";
        case M_V_LSHL_ADD: return "v_lshl_add_u32";
        case M_V_PERM: return "v_perm_b32";
        case M_V_BFI: return "v_bfi_b32";
        case M_V_BITOP3: return "v_bitop3_b32";
        case M_V_CVT_F32_U32: return "v_cvt_f32_u32";
        case M_V_FMA_F32: return "v_fma_f32";
        case M_V_RCP_F32: return "v_rcp_f32";
        case M_V_MUL_F32: return "v_mul_f32";
        case M_V_CVT_U32_F32: return "v_cvt_u32_f32";
        case M_V_FRACT_F32: return "v_fract_f32";
        case M_V_CMP_GT_F32: return "v_cmp_gt_f32";
        case M_V_CMP_LE_F32: return "v_cmp_le_f32";
        case M_V_CVT_F64_U32: return "v_cvt_f64_u32";
        case M_V_FMA_F64: return "v_fma_f64";
        case M_V_RCP_F64: return "v_rcp_f64";
        case M_V_MUL_F64: return "v_mul_f64";
        case M_V_MIN_F64: return "v_min_f64";
        case M_V_CVT_U32_F64: return "v_cvt_u32_f64";
        case M_V_FRACT_F64: return "v_fract_f64";
        case M_V_CMP_LE_F64: return "v_cmp_le_f64";
        case M_S_MOV_B32: return "s_mov_b32";
        case M_S_MOV_B64: return "s_mov_b64";
        case M_S_AND_B64: return "s_and_b64";
        case M_S_OR_B64: return "s_or_b64";
        case M_S_XOR_B64: return "s_xor_b64";
        case M_S_XNOR_B64: return "s_xnor_b64";
        case M_S_ANDN2_B64: return "s_andn2_b64";
        case M_S_ORN2_B64: return "s_orn2_b64";
        case M_S_NOT_B64: return "s_not_b64";
        case M_S_CMP_EQ_U64: return "s_cmp_eq_u64";
        case M_S_CMP_LG_U64: return "s_cmp_lg_u64";
        case M_S_CMP_EQ_U32: return "s_cmp_eq_u32";
        case M_S_CMP_LT_U32: return "s_cmp_lt_u32";
        case M_S_CBRANCH_SCC0: return "s_cbranch_scc0";
        case M_S_CBRANCH_SCC1: return "s_cbranch_scc1";
        case M_S_BRANCH: return "s_branch";
        case M_S_NOP: return "s_nop";
        default: return "?";
    }
}

std::string opnd_str(const Opnd& o, const std::string& prefix) {
    char b[64];
    switch (o.k) {
        case O_V:
            if (o.n == 1) snprintf(b, sizeof b, "%sv%u", o.neg ? "-" : "", o.v);
            else snprintf(b, sizeof b, "%sv[%u:%u]", o.neg ? "-" : "", o.v, o.v + o.n - 1);
            return b;
        case O_S:
            if (o.n == 1) snprintf(b, sizeof b, "s%u", o.v);
            else snprintf(b, sizeof b, "s[%u:%u]", o.v, o.v + o.n - 1);
            return b;
        case O_VCC: return "vcc";
        case O_EXEC: return "exec";
        case O_IMM:
            if (o.v <= 64u) snprintf(b, sizeof b, "%u", o.v);
            else if (o.v >= 0xFFFFFFF0u) snprintf(b, sizeof b, "%d", (int32_t)o.v);
            else snprintf(b, sizeof b, "0x%x", o.v);
            return b;
        case O_LABEL: return prefix + "_L" + std::to_string(o.v);
        case O_FONE: return "1.0";
        default: return "";
    }
}

}  // namespace

bool schedule_conjuncts(const SsaTape& st, const std::vector<uint32_t>& pool,
                        uint32_t sample_rows, const std::vector<double>* insn_cost, SsaTape& out,
                        std::vector<uint8_t>& check) {
    return schedule_impl(st, pool, sample_rows, insn_cost, out, check);
}

// ---- the division subroutine ---------------------------------------------------------------
// 256-bit division by f64 digit estimates over 32-bit digits, no normalisation shifts (the
// round-1 interpreter's algorithm, gen_asm_core.py div_body, over fixed registers).  Step j
// (7..0, entered at the highest j any lane needs): c = trunc(R / (y 2^(32j))) from f64 (relative
// error ~2^-48, so c is the digit or off by one), R -= c*y*2^(32j) (8 mads), then one add-back if
// R went negative, one subtract if R >= y 2^(32j).  Lanes with y = 0 keep R = |x| and get
// q = 2^256 - 1 (SMT-LIB); signed kinds divide |x| by |y| and fix the signs by the bvsdiv /
// bvsrem / bvsmod rules.
std::vector<MI> div_routine() {
    std::vector<MI> o;
    auto E = [&](uint16_t op, std::initializer_list<Opnd> ops, bool e64 = false) {
        MI m;
        m.op = op;
        m.e64 = e64 ? 1 : 0;
        int i = 0;
        for (const Opnd& x : ops) m.o[i++] = x;
        o.push_back(m);
    };
    auto L = [&](uint32_t id) { E(M_LABEL, {LBL(id)}); };
    auto Yr = [](int k) { return V(R_DY + k); };
    auto Rr = [](int k) { return V(R_DR + k); };
    auto Xr = [](int k) { return V(R_DQ + k); };
    const Opnd FY = V(R_FY, 2), FR = V(R_FR, 2), FC = V(R_FC, 2), FT = V(R_FT, 2);
    const Opnd CARRY = V(R_CARRY, 2), MAD = V(R_MAD, 2);
    const Opnd C = V(R_C), T1 = V(R_T1), SX = V(R_SX), SY = V(R_SY);
    const Opnd YNZ = S(S_DIV_YNZ, 2), DUMMY = S(S_DIV_DUMMY, 2), MSK = S(S_DIV_MSK, 2),
               TM = S(S_DIV_TM, 2), K64 = S(S_DIV_F64K, 2), KIND = S(S_DIV_KIND);
    const Opnd K64LO = S(S_DIV_F64K), K64HI = S(S_DIV_F64K + 1);
    enum : uint32_t { L_UNS = 1, L_DONE, L_TOP3, L_CONV, L_ZQ, L_NOZQ, L_STEP0 = 10, L_NONEG0 = 20, L_NOGE0 = 30, L_WB = 40,
                      L_SDIV, L_SREM, L_SMOD, L_NARROW = 50, L_NNEG0 = 60, L_NGE0 = 70,
                      L_NOYZ = 80, L_CZ0 = 90, L_RLT = 100, L_RLTD, L_YSLOW, L_YDONE, L_TOPALL,
                      L_F32 = 110, L_F32OK, L_STEP0_BODY };
    auto to_f64 = [&](Opnd dst, Opnd (*limb)(int)) {
        E(M_S_MOV_B32, {K64LO, IMM(0)});
        E(M_S_MOV_B32, {K64HI, IMM(0x41f00000u)});
        E(M_V_CVT_F64_U32, {dst, limb(7)});
        for (int k = 6; k >= 0; --k) {
            E(M_V_CVT_F64_U32, {FT, limb(k)});
            E(M_V_FMA_F64, {dst, dst, K64, FT});
        }
    };
    auto Rl = [](int k) { return V(R_DR + k); };
    auto Yl = [](int k) { return V(R_DY + k); };
    // signed kinds arrive as |x|, |y| with the sign masks in SX, SY (the call site forms them)
    L(L_UNS);
    // the quotient registers start at 0 for the kinds that return the quotient (the digit steps
    // write only the digits they compute); remainder kinds leave them as they are
    E(M_S_CMP_EQ_U32, {KIND, IMM(0)});
    E(M_S_CBRANCH_SCC1, {LBL(L_ZQ)});
    E(M_S_CMP_EQ_U32, {KIND, IMM(2)});
    E(M_S_CBRANCH_SCC0, {LBL(L_NOZQ)});
    L(L_ZQ);
    for (int k = 0; k < 8; ++k) E(M_V_MOV, {Xr(k), IMM(0)});
    L(L_NOZQ);
    // TM = lanes with y >= 2^32, YNZ = lanes with y != 0: every lane when every lane's top limb
    // is nonzero (full-width divisors), else from an OR over the limbs
    E(M_V_CMP_NE, {VCC(), IMM(0), Yr(7)});
    E(M_S_CMP_EQ_U64, {VCC(), IMM(0xFFFFFFFFu)});
    E(M_S_CBRANCH_SCC0, {LBL(L_YSLOW)});
    E(M_S_MOV_B64, {TM, IMM(0xFFFFFFFFu)});
    E(M_S_MOV_B64, {YNZ, IMM(0xFFFFFFFFu)});
    E(M_S_BRANCH, {LBL(L_YDONE)});
    L(L_YSLOW);
    E(M_V_OR3, {T1, Yr(1), Yr(2), Yr(3)});
    E(M_V_OR3, {T1, T1, Yr(4), Yr(5)});
    E(M_V_OR3, {T1, T1, Yr(6), Yr(7)});
    E(M_V_CMP_NE, {TM, IMM(0), T1}, true);  // lanes with y >= 2^32
    E(M_V_OR, {T1, T1, Yr(0)});
    E(M_V_CMP_NE, {YNZ, IMM(0), T1}, true);
    L(L_YDONE);
    // lanes with x < y (no digit): the top limbs decide when they differ in every lane, else
    // the borrow chain
    E(M_V_CMP_NE, {VCC(), Rr(7), Yr(7)});
    E(M_S_CMP_EQ_U64, {VCC(), IMM(0xFFFFFFFFu)});
    E(M_S_CBRANCH_SCC0, {LBL(L_RLT)});
    E(M_V_CMP_LT, {VCC(), Rr(7), Yr(7)});
    E(M_S_BRANCH, {LBL(L_RLTD)});
    L(L_RLT);
    E(M_V_SUB_CO, {T1, VCC(), Rr(0), Yr(0)});
    for (int k = 1; k < 8; ++k) E(M_V_SUBB_CO, {T1, VCC(), Rr(k), Yr(k), VCC()});
    L(L_RLTD);
    E(M_S_ANDN2_B64, {MSK, YNZ, VCC()});
    E(M_S_CMP_EQ_U64, {MSK, IMM(0)});
    E(M_S_CBRANCH_SCC1, {LBL(L_DONE)});
    // every lane's divisor below 2^32: digit-by-digit 64/32 division (L_NARROW)
    E(M_S_CMP_EQ_U64, {TM, IMM(0)});
    E(M_S_CBRANCH_SCC1, {LBL(L_NARROW)});
    // 1/yd, qd = R/y for the start digit.  When every lane that needs a digit has y >= 2^224,
    // y's and R's top three limbs give both to 2^-64 relative (R >= y there; lower limbs of R
    // only shift the estimate by < 2^-64, which the +-1 corrections absorb): 6 f64 ops per
    // conversion instead of 15
    // 1/y: v_rcp_f64 is an approximation (LLVM's f64 divide refines it twice); two Newton
    // steps bring it to f64 rounding, which the skipped-correction test below relies on (one
    // step left digit estimates off by up to ~2^-12 on MI355X: a digit one short, found at 2^24
    // config-5 rows)
    auto recip = [&]() {
        E(M_V_RCP_F64, {FC, FY});
        E(M_S_NOP, {IMM(1)});  // trans result -> non-trans VALU use needs a wait state
        E(M_V_FMA_F64, {FT, NEG(FY), FC, FONE()});
        E(M_V_FMA_F64, {FC, FC, FT, FC});
        E(M_V_FMA_F64, {FT, NEG(FY), FC, FONE()});
        E(M_V_FMA_F64, {FY, FC, FT, FC});
    };
    auto top3_f64 = [&](Opnd dst, Opnd (*limb)(int)) {
        E(M_S_MOV_B32, {K64LO, IMM(0)});
        E(M_S_MOV_B32, {K64HI, IMM(0x41f00000u)});  // 2^32
        E(M_V_CVT_F64_U32, {dst, limb(7)});
        for (int k = 6; k >= 5; --k) {
            E(M_V_CVT_F64_U32, {FT, limb(k)});
            E(M_V_FMA_F64, {dst, dst, K64, FT});
        }
        E(M_S_MOV_B32, {K64HI, IMM((uint32_t)(1023 + 160) << 20)});  // 2^160
        E(M_V_MUL_F64, {dst, dst, K64});
    };
    E(M_V_CMP_NE, {VCC(), IMM(0), Yr(7)});
    E(M_S_ANDN2_B64, {TM, MSK, VCC()});
    E(M_S_CBRANCH_SCC0, {LBL(L_F32)});
    to_f64(FY, Yl);
    recip();
    to_f64(FR, Rl);
    E(M_S_BRANCH, {LBL(L_CONV)});
    // Small quotients of full-width divisors (every lane that needs a digit has y >= 2^224, and
    // its estimate is below 2^10: random full-width x / y almost always): the digit from f32
    // estimates of the top two limbs, R7:R6 / Y7:Y6.  Truncating both to 64 bits moves R / y by
    // < 2^-32 relative (Y7 >= 1); the two conversions, the reciprocal (1 ulp) and the product add
    // < 2^-20.5 relative, so for an estimate below 2^10 the error is < 2^-9.9 absolute: the
    // digit is exact or one off, an estimate one high leaves R negative (the add-back below) and
    // one low has a fraction above 1 - 2^-9.9 (the "R >= y" test runs in waves with such a
    // lane).  4 f32 conversions, 2 fma, a reciprocal and a product instead of 19 f64 ops.
    L(L_F32);
    E(M_S_MOV_B32, {K64LO, IMM(0x4f800000u)});  // 2^32 as f32
    E(M_V_CVT_F32_U32, {V(R_FT), Rr(7)});
    E(M_V_CVT_F32_U32, {V(R_FT + 1), Rr(6)});
    E(M_V_FMA_F32, {V(R_FR), V(R_FT), K64LO, V(R_FT + 1)});
    E(M_V_CVT_F32_U32, {V(R_FT), Yr(7)});
    E(M_V_CVT_F32_U32, {V(R_FT + 1), Yr(6)});
    E(M_V_FMA_F32, {V(R_FY), V(R_FT), K64LO, V(R_FT + 1)});
    E(M_V_RCP_F32, {V(R_FY), V(R_FY)});
    E(M_S_NOP, {IMM(1)});  // trans result -> non-trans VALU use needs a wait state
    E(M_V_MUL_F32, {V(R_FC), V(R_FR), V(R_FY)});
    E(M_V_CMP_GT_F32, {VCC(), IMM(0x44800000u), V(R_FC)});  // estimate < 2^10
    E(M_S_ANDN2_B64, {TM, MSK, VCC()});
    E(M_S_CBRANCH_SCC0, {LBL(L_F32OK)});
    E(M_V_CMP_NE, {VCC(), IMM(0), Yr(7)});  // the f64 path reads y7 != 0 from VCC
    E(M_S_BRANCH, {LBL(L_TOP3)});
    L(L_F32OK);
    E(M_V_CVT_U32_F32, {C, V(R_FC)});
    E(M_V_CNDMASK, {C, IMM(0), C, MSK}, true);  // lanes without a digit (x < y, y = 0): 0
    E(M_V_FRACT_F32, {V(R_FT), V(R_FC)});
    E(M_V_CMP_LE_F32, {VCC(), IMM(0x3f7f8000u), V(R_FT)});  // 1 - 2^-9 <= fraction
    E(M_S_AND_B64, {TM, VCC(), MSK});
    E(M_S_BRANCH, {LBL(L_STEP0_BODY)});
    L(L_TOP3);
    top3_f64(FY, Yl);
    recip();
    // lanes outside MSK (x < y, or y = 0) may have y < 2^224, where the top limbs say nothing:
    // 1/y := 0 there, so every digit estimate is 0 and R keeps x, as their results need.  Not
    // needed when every lane has y >= 2^224 (VCC still holds y's top limb != 0 per lane): an
    // x < y lane then estimates a digit of 0, or 1 that the add-back corrects
    E(M_S_CMP_EQ_U64, {VCC(), IMM(0xFFFFFFFFu)});
    E(M_S_CBRANCH_SCC1, {LBL(L_TOPALL)});
    E(M_V_CNDMASK, {V(R_FY), IMM(0), V(R_FY), MSK}, true);
    E(M_V_CNDMASK, {V(R_FY + 1), IMM(0), V(R_FY + 1), MSK}, true);
    L(L_TOPALL);
    top3_f64(FR, Rl);
    L(L_CONV);
    E(M_V_MUL_F64, {FC, FR, FY});
    // common case first: every active lane's quotient estimate below 2^31 -> the last step only
    E(M_S_MOV_B32, {K64LO, IMM(0)});
    E(M_S_MOV_B32, {K64HI, IMM((uint32_t)(1023 + 31) << 20)});
    E(M_V_CMP_LE_F64, {VCC(), K64, FC});
    E(M_S_AND_B64, {TM, VCC(), MSK});
    E(M_S_CMP_EQ_U64, {TM, IMM(0)});
    E(M_S_CBRANCH_SCC1, {LBL(L_STEP0)});
    for (int j = 7; j >= 1; --j) {  // start at the highest j with qd >= 2^(32j - 1) in some lane
        const uint32_t hi = (uint32_t)(1023 + 32 * j - 1) << 20;
        E(M_S_MOV_B32, {K64LO, IMM(0)});
        E(M_S_MOV_B32, {K64HI, IMM(hi)});
        E(M_V_CMP_LE_F64, {VCC(), K64, FC});
        E(M_S_AND_B64, {TM, VCC(), MSK});
        E(M_S_CMP_LG_U64, {TM, IMM(0)});
        E(M_S_CBRANCH_SCC1, {LBL(L_STEP0 + j)});
    }
    E(M_S_BRANCH, {LBL(L_STEP0)});
    // FC = R * (1/y) is valid on entry to every step: computed above for the first step the
    // dispatch picks, recomputed at the end of each step for the next one
    for (int j = 7; j >= 0; --j) {
        L(L_STEP0 + j);
        if (j) {
            E(M_S_MOV_B32, {K64LO, IMM(0)});
            E(M_S_MOV_B32, {K64HI, IMM((uint32_t)(1023 - 32 * j) << 20)});
            E(M_V_MUL_F64, {FC, FC, K64});
        }
        // clamp to 2^32 - 1 (NaN from y = 0 lanes becomes the clamp and is zeroed below)
        E(M_S_MOV_B32, {K64LO, IMM(0xffe00000u)});
        E(M_S_MOV_B32, {K64HI, IMM(0x41efffffu)});
        E(M_V_MIN_F64, {FC, FC, K64});
        E(M_V_CVT_U32_F64, {C, FC});
        // y = 0 lanes (their NaN estimate became the clamp) take digit 0; skipped when no lane
        // divides by zero
        E(M_S_CMP_EQ_U64, {YNZ, IMM(0xFFFFFFFFu)});
        E(M_S_CBRANCH_SCC1, {LBL(L_CZ0 + j)});
        E(M_V_CNDMASK, {C, IMM(0), C, YNZ}, true);
        L(L_CZ0 + j);
        // the estimate is within 2^-19 of R / (y 2^32j), so c is one too small only in lanes
        // whose estimate has a fraction above 1 - 2^-18: without such a lane the "R >= y" test
        // below (a 9-instruction borrow chain) is skipped
        E(M_V_FRACT_F64, {FT, FC});
        E(M_S_MOV_B32, {K64LO, IMM(0)});
        E(M_S_MOV_B32, {K64HI, IMM(0x3feffff8u)});  // 1 - 2^-18
        E(M_V_CMP_LE_F64, {VCC(), K64, FT});
        E(M_S_AND_B64, {TM, VCC(), YNZ});
        // R[j..] -= c * y (the product's limbs above limb 7 only feed the borrow); the carry
        // pair's high word stays 0 from the first copy on (the first product adds nothing)
        if (j == 0) L(L_STEP0_BODY);
        for (int k = 0; k < 8; ++k) {
            E(M_V_MAD_U64_U32, {MAD, DUMMY, C, Yr(k), k ? CARRY : IMM(0)});
            if (k == 0) E(M_V_MOV, {V(R_CARRY + 1), IMM(0)});
            E(M_V_MOV, {V(R_CARRY), V(R_MAD + 1)});
            const int limb = j + k;
            if (limb <= 7) {
                if (k == 0) E(M_V_SUB_CO, {Rr(limb), VCC(), Rr(limb), V(R_MAD)});
                else E(M_V_SUBB_CO, {Rr(limb), VCC(), Rr(limb), V(R_MAD), VCC()});
            } else {
                E(M_V_SUBB_CO, {T1, VCC(), IMM(0), V(R_MAD), VCC()});
            }
        }
        E(M_V_SUBB_CO, {T1, VCC(), IMM(0), V(R_CARRY), VCC()});  // limb j + 8 > 7
        // negative: add y << 32j back, c - 1
        E(M_S_MOV_B64, {MSK, VCC()});
        E(M_S_CMP_EQ_U64, {MSK, IMM(0)});
        E(M_S_CBRANCH_SCC1, {LBL(L_NONEG0 + j)});
        for (int k = 0; k < 8 - j; ++k) {
            E(M_V_CNDMASK, {T1, IMM(0), Yr(k), MSK}, true);
            if (k == 0) E(M_V_ADD_CO, {Rr(j + k), VCC(), Rr(j + k), T1});
            else E(M_V_ADDC_CO, {Rr(j + k), VCC(), Rr(j + k), T1, VCC()});
        }
        E(M_V_CNDMASK, {T1, IMM(0), IMM(1), MSK}, true);
        E(M_V_SUB_U32, {C, C, T1});
        L(L_NONEG0 + j);
        // R >= y << 32j (y = 0 lanes excluded): subtract once more, c + 1
        E(M_S_CMP_EQ_U64, {TM, IMM(0)});
        E(M_S_CBRANCH_SCC1, {LBL(L_NOGE0 + j)});
        E(M_V_SUB_CO, {T1, VCC(), Rr(j), Yr(0)});
        for (int k = 1; k < 8 - j; ++k) E(M_V_SUBB_CO, {T1, VCC(), Rr(j + k), Yr(k), VCC()});
        for (int k = 8 - j; k < 8; ++k) E(M_V_SUBB_CO, {T1, VCC(), IMM(0), Yr(k), VCC()});
        E(M_S_ANDN2_B64, {MSK, YNZ, VCC()});
        E(M_S_CMP_EQ_U64, {MSK, IMM(0)});
        E(M_S_CBRANCH_SCC1, {LBL(L_NOGE0 + j)});
        for (int k = 0; k < 8 - j; ++k) {
            E(M_V_CNDMASK, {T1, IMM(0), Yr(k), MSK}, true);
            if (k == 0) E(M_V_SUB_CO, {Rr(j + k), VCC(), Rr(j + k), T1});
            else E(M_V_SUBB_CO, {Rr(j + k), VCC(), Rr(j + k), T1, VCC()});
        }
        E(M_V_CNDMASK, {T1, IMM(0), IMM(1), MSK}, true);
        E(M_V_ADD_U32, {C, C, T1});
        L(L_NOGE0 + j);
        E(M_V_MOV, {Xr(j), C});
        if (j) {  // the next step's estimate from the reduced remainder
            to_f64(FR, Rl);
            E(M_V_MUL_F64, {FC, FR, FY});
        }
    }
    E(M_S_BRANCH, {LBL(L_DONE)});
    // ---- narrow divisor (d = y0 < 2^32 in every lane, y = 0 lanes masked by YNZ): for
    // k = 7..0, q_k = floor((r 2^32 + R[k]) / d) from an f64 estimate (the 64-bit numerator and
    // the refined reciprocal round to 2^-52 relative, so the estimate is the digit or off by
    // one), R[k] = the low word of the exact difference, corrected by one add-back / subtract;
    // it is the next digit's r
    L(L_NARROW);
    E(M_V_CVT_F64_U32, {FY, Yr(0)});
    E(M_V_RCP_F64, {FC, FY});
    E(M_S_NOP, {IMM(1)});
    E(M_V_FMA_F64, {FT, NEG(FY), FC, FONE()});
    E(M_V_FMA_F64, {FC, FC, FT, FC});
    E(M_V_FMA_F64, {FT, NEG(FY), FC, FONE()});
    E(M_V_FMA_F64, {FY, FC, FT, FC});          // FY = 1/d (two Newton steps, as above)
    // y = 0 lanes: 1/d := 0, so their digit estimates are 0, nothing is subtracted and R keeps
    // |x| (the SMT-LIB x % 0 = x); their quotient is fixed to 2^256 - 1 at the end
    E(M_V_CNDMASK, {V(R_FY), IMM(0), V(R_FY), YNZ}, true);
    E(M_V_CNDMASK, {V(R_FY + 1), IMM(0), V(R_FY + 1), YNZ}, true);
    E(M_S_MOV_B32, {K64LO, IMM(0)});
    E(M_S_MOV_B32, {K64HI, IMM(0x41f00000u)});  // 2^32
    E(M_V_MOV, {C, IMM(0)});                    // running remainder r < d
    for (int k = 7; k >= 0; --k) {
        E(M_V_CVT_F64_U32, {FR, C});
        E(M_V_CVT_F64_U32, {FT, Rr(k)});
        E(M_V_FMA_F64, {FR, FR, K64, FT});      // r 2^32 + R[k]
        E(M_V_MUL_F64, {FC, FR, FY});
        E(M_S_MOV_B32, {K64LO, IMM(0xffe00000u)});
        E(M_S_MOV_B32, {K64HI, IMM(0x41efffffu)});
        E(M_V_MIN_F64, {FC, FC, K64});
        E(M_S_MOV_B32, {K64LO, IMM(0)});
        E(M_S_MOV_B32, {K64HI, IMM(0x41f00000u)});
        E(M_V_CVT_U32_F64, {Xr(k), FC});          // digit estimate
        E(M_V_MAD_U64_U32, {MAD, DUMMY, Xr(k), Yr(0), IMM(0)});
        E(M_V_SUB_CO, {Rr(k), VCC(), Rr(k), V(R_MAD)});        // low word of the difference
        E(M_V_SUBB_CO, {T1, VCC(), C, V(R_MAD + 1), VCC()});    // borrow: estimate one too high
        E(M_S_MOV_B64, {TM, VCC()});
        E(M_S_CMP_EQ_U64, {TM, IMM(0)});
        E(M_S_CBRANCH_SCC1, {LBL(L_NNEG0 + k)});
        E(M_V_CNDMASK, {T1, IMM(0), Yr(0), TM}, true);
        E(M_V_CNDMASK, {C, IMM(0), IMM(1), TM}, true);
        E(M_V_ADD_U32, {Rr(k), Rr(k), T1});
        E(M_V_SUB_U32, {Xr(k), Xr(k), C});
        L(L_NNEG0 + k);
        E(M_V_CMP_GE, {VCC(), Rr(k), Yr(0)});              // one too low: r >= d
        E(M_S_AND_B64, {TM, VCC(), YNZ});
        E(M_S_CMP_EQ_U64, {TM, IMM(0)});
        E(M_S_CBRANCH_SCC1, {LBL(L_NGE0 + k)});
        E(M_V_CNDMASK, {T1, IMM(0), Yr(0), TM}, true);
        E(M_V_CNDMASK, {C, IMM(0), IMM(1), TM}, true);
        E(M_V_SUB_U32, {Rr(k), Rr(k), T1});
        E(M_V_ADD_U32, {Xr(k), Xr(k), C});
        L(L_NGE0 + k);
        E(M_V_MOV, {C, Rr(k)});                  // r
    }
    // R[0] is the remainder; R[1..7] hold the intermediate remainders: zero them (y != 0 lanes)
    for (int k = 1; k < 8; ++k) E(M_V_CNDMASK, {Rr(k), Rr(k), IMM(0), YNZ}, true);
    L(L_DONE);
    auto cneg = [&](uint32_t dst, uint32_t srcb, Opnd m) {  // dst = (src ^ m) - m
        for (int k = 0; k < 8; ++k) E(M_V_XOR, {V(dst + k), V(srcb + k), m});
        E(M_V_SUB_CO, {V(dst), VCC(), V(dst), m});
        for (int k = 1; k < 8; ++k) E(M_V_SUBB_CO, {V(dst + k), VCC(), V(dst + k), m, VCC()});
    };
    // UREM: the remainder stays in R (the caller reads it there); x % 0 = x needs no fix-up
    E(M_S_CMP_EQ_U32, {KIND, IMM(1)});
    E(M_S_CBRANCH_SCC1, {LBL(L_WB)});
    E(M_S_CMP_EQ_U32, {KIND, IMM(4)});
    E(M_S_CBRANCH_SCC1, {LBL(L_SMOD)});
    E(M_S_CMP_EQ_U32, {KIND, IMM(3)});
    E(M_S_CBRANCH_SCC1, {LBL(L_SREM)});
    // y = 0: q = 2^256 - 1 (R already holds |x|); nothing to do when no lane divides by zero
    E(M_S_CMP_EQ_U64, {YNZ, IMM(0xFFFFFFFFu)});
    E(M_S_CBRANCH_SCC1, {LBL(L_NOYZ)});
    for (int k = 0; k < 8; ++k) E(M_V_CNDMASK, {Xr(k), IMM(0xFFFFFFFFu), Xr(k), YNZ}, true);
    L(L_NOYZ);
    E(M_S_CMP_EQ_U32, {KIND, IMM(0)});
    E(M_S_CBRANCH_SCC1, {LBL(L_WB)});
    L(L_SDIV);  // q negated when the signs differ
    E(M_V_XOR, {T1, SX, SY});
    cneg(R_DQ, R_DQ, T1);
    E(M_S_BRANCH, {LBL(L_WB)});
    L(L_SREM);  // r takes the sign of x
    cneg(R_DQ, R_DR, SX);
    E(M_S_BRANCH, {LBL(L_WB)});
    L(L_SMOD);  // u = |x| % |y|: (x<0 ? -u : u) + (signs differ && u ? +-|y| : 0)
    cneg(R_DQ, R_DR, SX);
    E(M_V_OR3, {T1, Rr(0), Rr(1), Rr(2)});
    E(M_V_OR3, {T1, T1, Rr(3), Rr(4)});
    E(M_V_OR3, {T1, T1, Rr(5), Rr(6)});
    E(M_V_OR, {T1, T1, Rr(7)});
    E(M_V_CMP_NE, {MSK, IMM(0), T1}, true);
    E(M_V_XOR, {T1, SX, SY});
    E(M_V_CMP_NE, {VCC(), IMM(0), T1});
    E(M_S_AND_B64, {MSK, MSK, VCC()});
    cneg(R_DY, R_DY, SY);  // t = +-|y| (the original y)
    for (int k = 0; k < 8; ++k) {
        E(M_V_CNDMASK, {T1, IMM(0), Yr(k), MSK}, true);
        if (k == 0) E(M_V_ADD_CO, {Xr(k), VCC(), Xr(k), T1});
        else E(M_V_ADDC_CO, {Xr(k), VCC(), Xr(k), T1, VCC()});
    }
    L(L_WB);
    E(M_RET, {});
    return o;
}

// ---- the Keccak-f[1600] subroutine ---------------------------------------------------------
// 24 rounds fully unrolled, each lane's halves renamed instead of moved: theta's column parities
// and rho's rotations (two v_alignbit per 64-bit lane) and chi's new rows go to free registers and
// the old ones are freed, so pi costs nothing and the state never moves; the final lane ->
// register map is fixed at build time (KecCode::out).  chi = b0 ^ (~b1 & b2) as
// v_bfi_b32(b1, b0, b0 ^ b2).  Per round: 152 two-cycle-class VALU (xor), 108 four-cycle (alignbit,
// bfi).  Restates keccak_f1600 (u256_ops.h).
namespace {
const uint64_t kKeccakRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
// rho + pi along the pi cycle from lane 1: (destination lane, rotation of the lane moved there)
const int kRhoPi[24][2] = {{10, 1}, {7, 3},   {11, 6},  {17, 10}, {18, 15}, {3, 21},
                           {5, 28}, {16, 36}, {8, 45},  {21, 55}, {24, 2},  {4, 14},
                           {15, 27}, {23, 41}, {19, 56}, {13, 8},  {12, 25}, {2, 43},
                           {20, 62}, {14, 18}, {22, 39}, {9, 61},  {6, 20},  {1, 44}};
}  // namespace

namespace {

// Complement states through theta: a column parity is stored complemented when an odd number of
// its lanes are, D[x] = C[x-1] ^ rot(C[x+1], 1) when exactly one of the two is, and lane (x, y) ^= D[x].
void kec_theta_states(uint8_t* comp) {
    uint8_t c[5] = {0}, d[5];
    for (int i = 0; i < 25; ++i) c[i % 5] ^= comp[i];
    for (int x = 0; x < 5; ++x) d[x] = c[(x + 4) % 5] ^ c[(x + 1) % 5];
    for (int i = 0; i < 25; ++i) comp[i] ^= d[i % 5];
}

// ... and through rho + pi (rotations keep a complement; pi moves it with the lane).
void kec_rhopi_states(uint8_t* comp) {
    uint8_t cur = comp[1];
    for (int step = 0; step < 24; ++step) {
        const int dst = kRhoPi[step][0];
        const uint8_t t = comp[dst];
        comp[dst] = cur;
        cur = t;
    }
}

// The complement plan (scripts/kec_plan.py, a beam search over the issue cost): lanes stored
// complemented at entry (two v_not each), and per round the state of every chi output (bit
// x + 5y).  Positions whose operands share a state keep b0's state whatever the plan says (v_bfi);
// the free ones take the planned state (xor, or xnor when it is not the natural one).  Over the
// 24 rounds: 132 v_bfi positions of 600 and 34 xnor positions, vs 600 v_bfi without complements.
const uint32_t kKecInit = 0x0400000u;
const uint32_t kKecPlan[24] = {
    0x068bb68u, 0x02e4e13u, 0x1c06466u, 0x0c37227u, 0x0c4310cu, 0x1102786u, 0x19c30d0u, 0x0766471u,
    0x110c621u, 0x0601678u, 0x10ce186u, 0x1c8e266u, 0x04310c6u, 0x0096583u, 0x138e181u, 0x191c4ecu,
    0x0431886u, 0x0a3c580u, 0x11c1863u, 0x1889592u, 0x1319212u, 0x03218c6u, 0x0c5a310u, 0x0cc2090u};

}  // namespace

bool kec_bitop3() {
    static const bool on = [] {
        const char* e = std::getenv("MH_JIT_KEC_BITOP3");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

const KecCode& kec_routine() {
    static const KecCode kc = [] {
        KecCode k;
        std::vector<MI>& o = k.code;
        auto E = [&](uint16_t op, std::initializer_list<Opnd> ops) {
            MI m;
            m.op = op;
            int i = 0;
            for (const Opnd& x : ops) m.o[i++] = x;
            o.push_back(m);
        };
        uint32_t map[25][2];
        for (uint32_t i = 0; i < 25; ++i) {
            map[i][0] = R_KEC0 + 2 * i;
            map[i][1] = R_KEC0 + 2 * i + 1;
        }
        std::vector<uint32_t> spare;
        for (uint32_t r = R_KEC0 + N_KEC_REGS; r-- > R_KEC0 + 50;) spare.push_back(r);
        auto take = [&]() {
            const uint32_t r = spare.back();
            spare.pop_back();
            return r;
        };
        auto give = [&](uint32_t r) { spare.push_back(r); };
        // lane complementing (MH_JIT_KEC_COMPLEMENT=0 turns it off): per-lane stored-complemented
        // flags, tracked through theta and rho-pi at build time, and the chi output states of
        // every round (kKecPlan)
        static const bool complement = [] {
            const char* e = std::getenv("MH_JIT_KEC_COMPLEMENT");
            return !(e && atoi(e) == 0);
        }();
        uint8_t comp[25] = {0};
        uint8_t plan[24][25];
        for (int r = 0; r < 24; ++r)
            for (int i = 0; i < 25; ++i) plan[r][i] = (uint8_t)((kKecPlan[r] >> i) & 1);
        if (complement && !kec_bitop3())
            for (int i = 0; i < 25; ++i)
                if ((kKecInit >> i) & 1) {
                    comp[i] = 1;
                    for (int h = 0; h < 2; ++h) E(M_V_NOT, {V(map[i][h]), V(map[i][h])});
                }
        // rotl64 of (lo, hi) by r (1..63, not 32) into two fresh registers
        auto rotl = [&](uint32_t lo, uint32_t hi, int r, uint32_t* out) {
            if (r > 32) { std::swap(lo, hi); r -= 32; }
            out[0] = take();
            out[1] = take();
            E(M_V_ALIGNBIT, {V(out[0]), V(lo), V(hi), IMM((uint32_t)(32 - r))});
            E(M_V_ALIGNBIT, {V(out[1]), V(hi), V(lo), IMM((uint32_t)(32 - r))});
        };
        // gfx950's v_bitop3_b32 (MH_JIT_KEC_BITOP3=0: the complement plan below instead): a
        // three-input bitwise op at the issue rate of v_xor (profiles/r05j/valu_bitop3.json:
        // 2.6-2.8 cycles per wave instruction at 2-8 waves per SIMD, v_xor 2.9, v_alignbit 4.7).
        // theta's column parities are two XOR3 per half, D[x] folds into the XOR3 that applies
        // it (lane ^ C[x-1] ^ rot(C[x+1], 1)), chi is one op per half (table 0xd2: b0 ^ (~b1 &
        // b2)).  Per round 120 bitop3 + 58 alignbit + iota's xor, against 196 two-cycle and 64
        // four-cycle ops of the complement plan.  No lane is stored complemented.
        const bool bitop3 = kec_bitop3();
        auto B3 = [&](uint32_t d, uint32_t a, uint32_t b, uint32_t c, uint32_t tt) {
            E(M_V_BITOP3, {V(d), V(a), V(b), V(c), IMM(tt)});
        };
        for (int round = 0; bitop3 && round < 24; ++round) {
            uint32_t c[5][2];
            for (int x = 0; x < 5; ++x)  // the ten parities interleaved (dependent ops 10 apart)
                for (int h = 0; h < 2; ++h) {
                    c[x][h] = take();
                    B3(c[x][h], map[x][h], map[x + 5][h], map[x + 10][h], 0x96);
                }
            for (int x = 0; x < 5; ++x)
                for (int h = 0; h < 2; ++h)
                    B3(c[x][h], c[x][h], map[x + 15][h], map[x + 20][h], 0x96);
            for (int x = 0; x < 5; ++x) {
                uint32_t d[2];
                rotl(c[(x + 1) % 5][0], c[(x + 1) % 5][1], 1, d);
                for (int h = 0; h < 2; ++h)
                    for (int y = 0; y < 5; ++y)
                        B3(map[x + 5 * y][h], map[x + 5 * y][h], c[(x + 4) % 5][h], d[h], 0x96);
                give(d[0]);
                give(d[1]);
            }
            for (int x = 0; x < 5; ++x) { give(c[x][0]); give(c[x][1]); }
            uint32_t cur[2] = {map[1][0], map[1][1]};
            for (int step = 0; step < 24; ++step) {
                const int dst = kRhoPi[step][0];
                const uint32_t t[2] = {map[dst][0], map[dst][1]};
                uint32_t nv[2];
                rotl(cur[0], cur[1], kRhoPi[step][1], nv);
                map[dst][0] = nv[0];
                map[dst][1] = nv[1];
                give(cur[0]);
                give(cur[1]);
                cur[0] = t[0];
                cur[1] = t[1];
            }
            for (int y = 0; y < 25; y += 5) {
                uint32_t nrow[5][2];
                for (int x = 0; x < 5; ++x)
                    for (int h = 0; h < 2; ++h) {
                        nrow[x][h] = take();
                        B3(nrow[x][h], map[y + x][h], map[y + (x + 1) % 5][h],
                           map[y + (x + 2) % 5][h], 0xd2);
                    }
                for (int x = 0; x < 5; ++x)
                    for (int h = 0; h < 2; ++h) {
                        give(map[y + x][h]);
                        map[y + x][h] = nrow[x][h];
                    }
            }
            const uint64_t rc = kKeccakRC[round];
            for (int h = 0; h < 2; ++h) {
                const uint32_t w = (uint32_t)(rc >> (32 * h));
                if (w) E(M_V_XOR, {V(map[0][h]), IMM(w), V(map[0][h])});
            }
        }
        for (int round = 0; !bitop3 && round < 24; ++round) {
            // theta
            // (the ten column-parity chains interleaved: a wave's dependent VALU ops 10 apart)
            uint32_t c[5][2];
            for (int x = 0; x < 5; ++x)
                for (int h = 0; h < 2; ++h) {
                    c[x][h] = take();
                    E(M_V_XOR, {V(c[x][h]), V(map[x][h]), V(map[x + 5][h])});
                }
            for (int y = 2; y < 5; ++y)
                for (int x = 0; x < 5; ++x)
                    for (int h = 0; h < 2; ++h)
                        E(M_V_XOR, {V(c[x][h]), V(map[x + 5 * y][h]), V(c[x][h])});
            for (int x = 0; x < 5; ++x) {
                uint32_t d[2];
                rotl(c[(x + 1) % 5][0], c[(x + 1) % 5][1], 1, d);
                for (int h = 0; h < 2; ++h) {
                    E(M_V_XOR, {V(d[h]), V(c[(x + 4) % 5][h]), V(d[h])});
                    for (int y = 0; y < 5; ++y)
                        E(M_V_XOR, {V(map[x + 5 * y][h]), V(d[h]), V(map[x + 5 * y][h])});
                }
                give(d[0]);
                give(d[1]);
            }
            for (int x = 0; x < 5; ++x) { give(c[x][0]); give(c[x][1]); }
            kec_theta_states(comp);
            // rho + pi
            uint32_t cur[2] = {map[1][0], map[1][1]};
            for (int step = 0; step < 24; ++step) {
                const int dst = kRhoPi[step][0];
                const uint32_t t[2] = {map[dst][0], map[dst][1]};
                uint32_t nv[2];
                rotl(cur[0], cur[1], kRhoPi[step][1], nv);
                map[dst][0] = nv[0];
                map[dst][1] = nv[1];
                give(cur[0]);
                give(cur[1]);
                cur[0] = t[0];
                cur[1] = t[1];
                // the last step's t is lane 1's original registers, freed by the first step
            }
            kec_rhopi_states(comp);
            // chi, on lanes that may be stored complemented (comp[i]: register value = ~lane i).
            // Row y, position x: o = b0 ^ (~b1 & b2).  With b1, b2 in opposite complement states
            // ~b1 & b2 is one AND (b1 stored complemented) or the complement of one OR (b2 stored
            // complemented), and the output's complement state is free: xor or xnor with b0.
            // With equal states it is v_bfi over the stored values (state of b0 kept).  The
            // states chosen for the free outputs (kKecPlan) keep both rare.  Per row the ten
            // first operations come first and the ten second ones then write in place, so
            // dependent operations are ten apart.
            for (int y = 0; y < 25; y += 5) {
                uint32_t nrow[5][2];
                uint8_t ncomp[5];
                for (int x = 0; x < 5; ++x) {
                    const int i0 = y + x, i1 = y + (x + 1) % 5, i2 = y + (x + 2) % 5;
                    const bool r1 = comp[i1], r2 = comp[i2];
                    for (int h = 0; h < 2; ++h) {
                        const uint32_t b0 = map[i0][h], b1 = map[i1][h], b2 = map[i2][h];
                        nrow[x][h] = take();
                        if (!complement || r1 == r2)
                            E(M_V_XOR, {V(nrow[x][h]), V(b0), V(r1 ? b1 : b2)});
                        else
                            E(r1 ? M_V_AND : M_V_OR, {V(nrow[x][h]), V(b1), V(b2)});
                    }
                }
                for (int x = 0; x < 5; ++x) {
                    const int i0 = y + x, i1 = y + (x + 1) % 5, i2 = y + (x + 2) % 5;
                    const bool r1 = comp[i1], r2 = comp[i2];
                    for (int h = 0; h < 2; ++h) {
                        const uint32_t b0 = map[i0][h], b1 = map[i1][h], b2 = map[i2][h];
                        const uint32_t t = nrow[x][h];
                        if (!complement || r1 == r2) {
                            // r1 = r2 = 0: b0' ^ (~b1' & b2') = bfi(b1', b0', b0' ^ b2');
                            // r1 = r2 = 1: ~b1 & b2 = b1' & ~b2' -> bfi(b2', b0', b0' ^ b1')
                            E(M_V_BFI, {V(t), V(r1 ? b2 : b1), V(b0), V(t)});
                        } else {
                            // natural state of b0' ^ t: comp[i0] (AND), comp[i0] ^ 1 (OR)
                            const bool nat = comp[i0] ^ !r1;
                            E(nat == plan[round][i0] ? M_V_XOR : M_V_XNOR, {V(t), V(b0), V(t)});
                        }
                    }
                    ncomp[x] = (!complement || r1 == r2) ? comp[i0] : plan[round][i0];
                }
                for (int x = 0; x < 5; ++x) {
                    comp[y + x] = ncomp[x];
                    for (int h = 0; h < 2; ++h) {
                        give(map[y + x][h]);
                        map[y + x][h] = nrow[x][h];
                    }
                }
            }
            // iota
            const uint64_t rc = kKeccakRC[round];
            for (int h = 0; h < 2; ++h) {
                const uint32_t w = (uint32_t)(rc >> (32 * h));
                if (w) E(M_V_XOR, {V(map[0][h]), IMM(w), V(map[0][h])});
            }
        }
        for (int i = 0; i < 4; ++i) {
            for (int h = 0; h < 2 && comp[i]; ++h) E(M_V_NOT, {V(map[i][h]), V(map[i][h])});
            k.out[2 * i] = map[i][0];
            k.out[2 * i + 1] = map[i][1];
        }
        E(M_RET, {});
        return k;
    }();
    return kc;
}

void op_stats(uint64_t* valu, uint64_t* wide, uint64_t* count, bool reset) {
    for (int i = 0; i < 256; ++i) {
        valu[i] = Emitter::op_valu[i];
        wide[i] = Emitter::op_wide[i];
        count[i] = Emitter::op_count[i];
        if (reset) Emitter::op_valu[i] = Emitter::op_wide[i] = Emitter::op_count[i] = 0;
    }
}

std::string print(const MI& m, const std::string& prefix) {
    if (m.op == M_LABEL) return prefix + "_L" + std::to_string(m.o[0].v) + ":";
    if (m.op == M_CALL_DIV || m.op == M_CALL_KEC) {
        const std::string l = prefix + "_c" + std::to_string(m.o[0].v);
        const char* tgt = m.op == M_CALL_DIV ? "mh_div" : "mh_kec";
        char b[512];
        snprintf(b, sizeof b,
                 "s_getpc_b64 s[%u:%u]\n%s:\n"
                 "s_add_u32 s%u, s%u, %s - %s\n"
                 "s_addc_u32 s%u, s%u, 0\n"
                 "s_swappc_b64 s[%u:%u], s[%u:%u]",
                 S_DIV_TGT, S_DIV_TGT + 1, l.c_str(), S_DIV_TGT, S_DIV_TGT, tgt, l.c_str(),
                 S_DIV_TGT + 1, S_DIV_TGT + 1, S_DIV_RA, S_DIV_RA + 1, S_DIV_TGT, S_DIV_TGT + 1);
        return b;
    }
    if (m.op == M_RET) {
        char b[64];
        snprintf(b, sizeof b, "s_setpc_b64 s[%u:%u]", S_DIV_RA, S_DIV_RA + 1);
        return b;
    }
    if (m.op == M_LOADCOL) {
        char b[320];
        const uint32_t j = m.o[1].v;
        snprintf(b, sizeof b,
                 "s_mul_i32 s28, s27, 0x%x\n"
                 "s_mul_hi_u32 s29, s27, 0x%x\n"
                 "s_add_u32 s28, s28, s4\n"
                 "s_addc_u32 s29, s29, s5\n"
                 "global_load_dword v%u, v2, s[28:29]",
                 j, j, m.o[0].v);
        return b;
    }
    if (m.op == M_S_WAITCNT_VM) {
        char b[64];
        snprintf(b, sizeof b, "s_waitcnt vmcnt(%u)", m.o[0].v);
        return b;
    }
    if (m.op == M_DS_WRITE2ST64 || m.op == M_DS_READ2ST64 || m.op == M_DS_READ_B32 ||
        m.op == M_S_WAITCNT_LGKM) {
        char b[128];
        const Opnd* o = m.o;
        if (m.op == M_DS_WRITE2ST64)
            snprintf(b, sizeof b, "ds_write2st64_b32 v%u, v%u, v%u offset0:%u offset1:%u", o[0].v,
                     o[1].v, o[2].v, o[3].v, o[4].v);
        else if (m.op == M_DS_READ2ST64)
            snprintf(b, sizeof b, "ds_read2st64_b32 v[%u:%u], v%u offset0:%u offset1:%u", o[0].v,
                     o[0].v + 1, o[1].v, o[2].v, o[3].v);
        else if (m.op == M_DS_READ_B32)
            snprintf(b, sizeof b, "ds_read_b32 v%u, v%u offset:%u", o[0].v, o[1].v, o[2].v);
        else
            snprintf(b, sizeof b, "s_waitcnt lgkmcnt(%u)", o[0].v);
        return b;
    }
    std::string s = op_name(m.op);
    if (m.e64) s += "_e64";
    if (m.op == M_S_NOP) return s + " " + std::to_string(m.o[0].v);
    if (m.op == M_V_BITOP3) {
        char b[128];
        snprintf(b, sizeof b, "v_bitop3_b32 v%u, v%u, v%u, v%u bitop3:0x%x", m.o[0].v, m.o[1].v,
                 m.o[2].v, m.o[3].v, m.o[4].v & 0xFFu);
        return b;
    }
    bool first = true;
    for (const Opnd& o : m.o) {
        if (o.k == O_NONE) break;
        s += first ? " " : ", ";
        s += opnd_str(o, prefix);
        first = false;
    }
    return s;
}

void print_list(const std::vector<MI>& code, const std::string& prefix, std::string& out) {
    for (const MI& m : code) {
        out += print(m, prefix);
        out += '\n';
    }
}

uint32_t code_bytes(const TapeCode& tc) {
    uint32_t b = 0;
    for (const MI& m : tc.code) {
        if (m.op == M_LABEL) continue;
        if (m.op == M_CALL_DIV || m.op == M_CALL_KEC) { b += 24; continue; }
        if (m.op == M_LOADCOL) { b += 36; continue; }
        bool lit = false;
        for (const Opnd& o : m.o) lit |= o.k == O_IMM && !is_inline(o.v);
        const bool vop3 = m.e64 || m.op == M_V_OR3 || m.op == M_V_ALIGNBIT ||
                          m.op == M_V_MAD_U64_U32 || m.op == M_V_FMA_F64 || m.op == M_V_MUL_F64 ||
                          m.op == M_V_MIN_F64 || m.op == M_V_LSHL_ADD || m.op == M_V_PERM ||
                          m.op == M_V_BFI || m.op == M_V_BITOP3 || m.op == M_DS_WRITE2ST64 ||
                          m.op == M_DS_READ2ST64 || m.op == M_DS_READ_B32;
        b += (vop3 || lit) ? 8 : 4;
    }
    return b;
}

namespace {

void line(std::string& out, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
void line(std::string& out, const char* fmt, ...) {
    char b[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(b, sizeof b, fmt, ap);
    va_end(ap);
    out += b;
    out += '\n';
}

}  // namespace

// Kernel `mh_jit` (register map in jit.h):
//   s[0:1] kernarg pointer, s2 = workgroup id x (row block), s3 = workgroup id y (tape group);
//   kernel arguments in s4..s23 (KernArgs); s24 = this wave's first row (buffer-local),
//   s25 = its end, s26 = current 64-row chunk, s27 = column stride in bytes, s[28:29] load
//   address, s[30:31] valid-lane mask, s[32:33] the tape's root mask, s34/s35 scratch,
//   s[36:37] jump-table address, s38 = group index.
//   v0 = workitem id, v1 = lane, v2 = row offset in bytes, v3 = per-tape hit counts (lane t =
//   the group's tape t), v4 = per-tape first hit + 1 (0 = none), v5..v7 atomics / stores,
//   v[8:39] the assignment columns (tape sets of <= 4 columns; above that the tape code loads
//   the limbs it demands, M_LOADCOL), v[40:79] the division subroutine, v80.. tape temporaries.
Module build_module(const std::vector<const TapeCode*>& codes,
                    const std::vector<uint32_t>& tape_ids, uint32_t n_vars, bool values,
                    uint32_t group_bytes) {
    Module m;
    std::string& o = m.text;
    // groups: consecutive tapes up to group_bytes of code (and at most 64: one lane per tape)
    uint32_t cur = 0, first = 0;
    for (uint32_t i = 0; i < codes.size(); ++i) {
        const uint32_t b = code_bytes(*codes[i]) + 96;
        if (i > first && (cur + b > group_bytes || i - first >= 64)) {
            m.group_first.push_back(first);
            m.group_count.push_back(i - first);
            first = i;
            cur = 0;
        }
        cur += b;
    }
    if (first < codes.size()) {
        m.group_first.push_back(first);
        m.group_count.push_back((uint32_t)codes.size() - first);
    }
    const uint32_t n_pin = pinned_cols(n_vars);
    uint32_t maxv = R_COL0 + 8 * n_pin;
    bool any_div = false, any_lds = false, any_kec = false;
    for (const TapeCode* tc : codes) {
        maxv = std::max(maxv, tc->max_vgpr);
        any_div |= tc->calls_div;
        any_lds |= tc->uses_lds;
        any_kec |= tc->calls_kec;
    }
    if (any_kec) maxv = std::max<uint32_t>(maxv, R_TEMP_KEC);
    if (any_div) maxv = std::max<uint32_t>(maxv, R_TEMP0);
    maxv = std::max<uint32_t>(maxv, 8);
    static const uint32_t pad = [] {  // diagnostic: MH_JIT_PAD_VGPR (occupancy A/B)
        const char* e = std::getenv("MH_JIT_PAD_VGPR");
        const uint32_t v = e ? (uint32_t)atoi(e) : 0u;
        return v <= 512 ? v : 0u;
    }();
    maxv = std::max(maxv, pad);
    maxv = (maxv + 7) & ~7u;
    m.max_vgpr = maxv;
    m.n_sgpr = S_NEXT_FREE;

    line(o, ".amdgcn_target \"amdgcn-amd-amdhsa--gfx950\"");
    line(o, ".amdhsa_code_object_version 5");
    line(o, ".text");
    line(o, ".globl mh_jit");
    line(o, ".p2align 8");
    line(o, ".type mh_jit,@function");
    line(o, "mh_jit:");
    line(o, "s_load_dwordx16 s[4:19], s[0:1], 0x0");
    line(o, "s_load_dwordx4 s[20:23], s[0:1], 0x40");
    line(o, "v_and_b32 v1, 63, v0");
    line(o, "v_lshrrev_b32 v2, 6, v0");
    // a VALU write of a VGPR -> v_readfirstlane / v_readlane of it needs a wait state (CDNA3/4
    // manually inserted wait states); without it the wave reads a stale wave index
    line(o, "s_nop 1");
    line(o, "v_readfirstlane_b32 s24, v2");
    if (any_lds) {
        // this lane's shift window (R_LDS) and its zero words [0, D) and [D + 8, LDS_WORDS)
        line(o, "v_mul_u32_u24 v%u, 0x%x, v2", R_LDS, LDS_WAVE_BYTES);
        line(o, "v_lshl_add_u32 v%u, v1, 2, v%u", R_LDS, R_LDS);
        line(o, "v_mov_b32 v5, 0");
        for (uint32_t w = 0; w < LDS_WORDS; ++w) {
            if (w >= LDS_D && w < LDS_D + 8) continue;
            const uint32_t w2 = w + 1;
            if (w2 < LDS_WORDS && !(w2 >= LDS_D && w2 < LDS_D + 8)) {
                line(o, "ds_write2st64_b32 v%u, v5, v5 offset0:%u offset1:%u", R_LDS, w, w2);
                ++w;
            } else {
                line(o, "ds_write_b32 v%u, v5 offset:%u", R_LDS, w * 256);
            }
        }
    }
    line(o, "s_waitcnt lgkmcnt(0)");
    line(o, "s_lshr_b32 s25, s19, 2");        // rows per wave
    line(o, "s_mul_i32 s26, s2, s19");        // row block * rows per workgroup
    line(o, "s_mul_i32 s27, s24, s25");       // wave * rows per wave
    line(o, "s_add_u32 s24, s8, s26");
    line(o, "s_add_u32 s24, s24, s27");       // first row of this wave
    line(o, "s_add_u32 s25, s24, s25");
    line(o, "s_add_u32 s26, s8, s10");        // row_first + row_count
    line(o, "s_min_u32 s25, s25, s26");
    line(o, "s_cmp_ge_u32 s24, s25");
    line(o, "s_cbranch_scc1 mh_done");
    line(o, "s_lshl_b32 s27, s6, 2");         // column stride (bytes)
    line(o, "v_mov_b32 v3, 0");
    line(o, "v_mov_b32 v4, 0");
    line(o, "s_add_u32 s38, s3, s22");        // group
    line(o, "s_getpc_b64 s[36:37]");
    line(o, "mh_pc:");
    line(o, "s_add_u32 s36, s36, mh_tab - mh_pc");
    line(o, "s_addc_u32 s37, s37, 0");
    line(o, "s_lshl_b32 s34, s38, 2");
    line(o, "s_load_dword s35, s[36:37], s34");
    line(o, "s_waitcnt lgkmcnt(0)");
    line(o, "s_add_u32 s36, s36, s35");
    line(o, "s_addc_u32 s37, s37, 0");
    line(o, "s_setpc_b64 s[36:37]");
    line(o, "mh_done:");
    line(o, "s_endpgm");
    line(o, ".p2align 2");
    line(o, "mh_tab:");
    for (size_t g = 0; g < m.group_first.size(); ++g) line(o, ".long mh_g%zu - mh_tab", g);
    for (size_t g = 0; g < m.group_first.size(); ++g) {
        const uint32_t g0 = m.group_first[g], gn = m.group_count[g];
        line(o, ".p2align 6");
        line(o, "mh_g%zu:", g);
        line(o, "s_mov_b32 s26, s24");
        line(o, "mh_g%zu_chunk:", g);
        // rows of this chunk, validity, clamped load offsets
        line(o, "v_add_u32 v2, s26, v1");
        line(o, "v_cmp_gt_u32 vcc, s25, v2");
        line(o, "s_mov_b64 s[30:31], vcc");
        line(o, "s_sub_u32 s34, s25, 1");
        line(o, "v_min_u32 v2, s34, v2");
        line(o, "v_lshlrev_b32 v2, 2, v2");
        line(o, "s_mov_b64 s[28:29], s[4:5]");
        for (uint32_t j = 0; j < 8 * n_pin; ++j) {
            if (j) {
                line(o, "s_add_u32 s28, s28, s27");
                line(o, "s_addc_u32 s29, s29, 0");
            }
            line(o, "global_load_dword v%u, v2, s[28:29]", R_COL0 + j);
        }
        if (n_pin) line(o, "s_waitcnt vmcnt(0)");
        for (uint32_t t = 0; t < gn; ++t) {
            const TapeCode& tc = *codes[g0 + t];
            char pre[64];
            snprintf(pre, sizeof pre, "mh_g%zut%u", g, t);
            print_list(tc.code, pre, o);
            if (values) {
                const uint32_t id = tape_ids[g0 + t];
                line(o, "s_mov_b64 exec, s[30:31]");
                line(o, "s_nop 1");
                line(o, "s_sub_u32 s34, s26, s8");
                line(o, "v_add_u32 v5, s34, v1");
                line(o, "v_lshlrev_b32 v5, 2, v5");
                for (int k = 0; k < 8; ++k) {
                    const uint64_t mult = ((uint64_t)id * 8 + (uint64_t)k) * 4ull;
                    if (mult >> 32) { line(o, "s_endpgm"); break; }
                    line(o, "s_mul_i32 s34, s10, 0x%x", (uint32_t)mult);
                    line(o, "s_mul_hi_u32 s35, s10, 0x%x", (uint32_t)mult);
                    line(o, "s_add_u32 s28, s20, s34");
                    line(o, "s_addc_u32 s29, s21, s35");
                    if (tc.root_bool) {
                        if (k == 0) line(o, "v_cndmask_b32_e64 v6, 0, 1, s[32:33]");
                        else line(o, "v_mov_b32 v6, 0");
                        line(o, "global_store_dword v5, v6, s[28:29]");
                    } else if (tc.root_limbs[k] != ~0u) {
                        line(o, "global_store_dword v5, v%u, s[28:29]", tc.root_limbs[k]);
                    } else {
                        line(o, "v_mov_b32 v6, 0x%x", tc.root_const[k]);
                        line(o, "global_store_dword v5, v6, s[28:29]");
                    }
                }
                line(o, "s_mov_b64 exec, -1");
                continue;
            }
            // no valid row of this chunk satisfies the tape (the common case): nothing to count
            line(o, "s_and_b64 s[32:33], s[32:33], s[30:31]");
            line(o, "s_cbranch_scc0 %s_nf", pre);
            line(o, "s_bcnt1_i32_b64 s34, s[32:33]");
            line(o, "v_readlane_b32 s35, v3, %u", t);
            line(o, "s_add_u32 s35, s35, s34");
            line(o, "v_writelane_b32 v3, s35, %u", t);
            line(o, "s_nop 4");
            line(o, "v_readlane_b32 s35, v4, %u", t);
            line(o, "s_cmp_lg_u32 s35, 0");
            line(o, "s_cbranch_scc1 %s_nf", pre);
            line(o, "s_ff1_i32_b64 s34, s[32:33]");
            line(o, "s_add_u32 s34, s34, s26");
            line(o, "s_add_u32 s34, s34, 1");
            line(o, "v_writelane_b32 v4, s34, %u", t);
            line(o, "s_nop 4");
            line(o, "%s_nf:", pre);
        }
        line(o, "s_add_u32 s26, s26, 64");
        line(o, "s_cmp_lt_u32 s26, s25");
        line(o, "s_cbranch_scc1 mh_g%zu_chunk", g);
        if (!values) {
            line(o, "s_nop 4");
            for (uint32_t t = 0; t < gn; ++t) {
                const uint32_t id = tape_ids[g0 + t];
                line(o, "v_readlane_b32 s34, v3, %u", t);
                line(o, "s_cmp_eq_u32 s34, 0");
                line(o, "s_cbranch_scc1 mh_g%zue%u_nc", g, t);
                line(o, "s_mov_b64 exec, 1");
                line(o, "s_nop 1");
                line(o, "v_mov_b32 v6, s34");
                line(o, "v_mov_b32 v7, 0");
                line(o, "v_mov_b32 v5, 0x%x", id * 8u);
                line(o, "global_atomic_add_x2 v5, v[6:7], s[16:17]");
                line(o, "s_mov_b64 exec, -1");
                line(o, "mh_g%zue%u_nc:", g, t);
                line(o, "v_readlane_b32 s34, v4, %u", t);
                line(o, "s_cmp_eq_u32 s34, 0");
                line(o, "s_cbranch_scc1 mh_g%zue%u_nf", g, t);
                line(o, "s_sub_u32 s34, s34, 1");
                line(o, "s_add_u32 s34, s34, s12");
                line(o, "s_addc_u32 s35, s13, 0");
                line(o, "s_mov_b64 exec, 1");
                line(o, "s_nop 1");
                line(o, "v_mov_b32 v6, s34");
                line(o, "v_mov_b32 v7, s35");
                line(o, "v_mov_b32 v5, 0x%x", id * 8u);
                line(o, "global_atomic_umin_x2 v5, v[6:7], s[14:15]");
                line(o, "s_mov_b64 exec, -1");
                line(o, "mh_g%zue%u_nf:", g, t);
            }
        }
        line(o, "s_endpgm");
    }
    if (any_div) {
        line(o, ".p2align 6");
        line(o, "mh_div:");
        print_list(div_routine(), "mh_dv", o);
    }
    if (any_kec) {
        line(o, ".p2align 6");
        line(o, "mh_kec:");
        print_list(kec_routine().code, "mh_kc", o);
    }
    line(o, ".Lmh_jit_end:");
    line(o, ".size mh_jit, .Lmh_jit_end-mh_jit");
    // kernel descriptor
    line(o, ".rodata");
    line(o, ".p2align 6");
    line(o, ".amdhsa_kernel mh_jit");
    line(o, "  .amdhsa_group_segment_fixed_size %u", any_lds ? (uint32_t)LDS_WG_BYTES : 0u);
    line(o, "  .amdhsa_private_segment_fixed_size 0");
    line(o, "  .amdhsa_kernarg_size %u", (uint32_t)sizeof(KernArgs));
    line(o, "  .amdhsa_user_sgpr_count 2");
    line(o, "  .amdhsa_user_sgpr_kernarg_segment_ptr 1");
    line(o, "  .amdhsa_system_sgpr_workgroup_id_x 1");
    line(o, "  .amdhsa_system_sgpr_workgroup_id_y 1");
    line(o, "  .amdhsa_system_vgpr_workitem_id 0");
    line(o, "  .amdhsa_next_free_vgpr %u", maxv);
    line(o, "  .amdhsa_next_free_sgpr %u", (uint32_t)S_NEXT_FREE);
    line(o, "  .amdhsa_accum_offset %u", (maxv + 3) & ~3u);
    line(o, "  .amdhsa_reserve_vcc 1");
    line(o, "  .amdhsa_ieee_mode 1");
    line(o, "  .amdhsa_dx10_clamp 1");
    line(o, ".end_amdhsa_kernel");
    line(o, ".amdgpu_metadata");
    line(o, "---");
    line(o, "amdhsa.kernels:");
    line(o, "  - .args:");
    line(o, "      - .offset: 0");
    line(o, "        .size: %u", (uint32_t)sizeof(KernArgs));
    line(o, "        .value_kind: by_value");
    line(o, "    .group_segment_fixed_size: %u", any_lds ? (uint32_t)LDS_WG_BYTES : 0u);
    line(o, "    .kernarg_segment_align: 8");
    line(o, "    .kernarg_segment_size: %u", (uint32_t)sizeof(KernArgs));
    line(o, "    .max_flat_workgroup_size: 256");
    line(o, "    .name: mh_jit");
    line(o, "    .private_segment_fixed_size: 0");
    line(o, "    .sgpr_count: %u", (uint32_t)S_NEXT_FREE + 6);
    line(o, "    .sgpr_spill_count: 0");
    line(o, "    .symbol: mh_jit.kd");
    line(o, "    .vgpr_count: %u", maxv);
    line(o, "    .vgpr_spill_count: 0");
    line(o, "    .agpr_count: 0");
    line(o, "    .wavefront_size: 64");
    line(o, "amdhsa.target: amdgcn-amd-amdhsa--gfx950");
    line(o, "amdhsa.version:");
    line(o, "  - 1");
    line(o, "  - 2");
    line(o, "...");
    line(o, ".end_amdgpu_metadata");
    return m;
}

// Code bytes per tape group (MH_JIT_GROUP_KB for A/B; a group's chunk loop branches back over
// the whole group, and s_cbranch reaches +-128 KB, so at most 112 KB).  Measured on MI355X,
// config 5 (profiles/r02y): 24 KB 2.52e11 evals/s, 40 KB 2.91e11, 56 KB 3.09e11, 80 KB 3.18e11,
// 96 KB 3.20e11, 128 KB 3.20e11 -- fewer, larger groups reload the assignment columns less
// often; the instruction cache streams the larger groups fine.
uint32_t default_group_bytes() {
    static const uint32_t g = [] {
        const char* e = std::getenv("MH_JIT_GROUP_KB");
        const uint32_t kb = e ? (uint32_t)atoi(e) : 0u;
        return (kb >= 4 && kb <= 112) ? kb * 1024u : 96u * 1024u;
    }();
    return g;
}

// VGPRs a code object holding tape `tc` allocates (build_module's rule for one tape).
uint32_t module_vgprs(const TapeCode& tc, uint32_t n_vars) {
    uint32_t v = std::max<uint32_t>(R_COL0 + 8 * pinned_cols(n_vars), tc.max_vgpr);
    if (tc.calls_kec) v = std::max<uint32_t>(v, R_TEMP_KEC);
    if (tc.calls_div) v = std::max<uint32_t>(v, R_TEMP0);
    return (std::max<uint32_t>(v, 8) + 7) & ~7u;
}

// Occupancy classes below the budget (MH_JIT_CLASSES, comma-separated VGPR ceilings): a code
// object's waves per SIMD are set by its worst tape, so tapes can be binned by the VGPRs their
// code object needs, each bin its own code object(s).  Off by default: on MI355X, config 5
// (profiles/r02ad), one class 3.383e11 evals/s, {64, 80, 96} 3.384-3.386e11, {72, 80, 96}
// 3.389e11, {80, 96} 3.392e11 -- within run-to-run noise, as an issue-bound kernel predicts
// (more waves per SIMD do not add VALU issue slots).
std::vector<uint32_t> occupancy_classes(uint32_t budget) {
    std::vector<uint32_t> c;
    if (const char* e = std::getenv("MH_JIT_CLASSES")) {
        c.clear();
        for (const char* p = e; *p;) {
            char* q = nullptr;
            const unsigned long x = strtoul(p, &q, 10);
            if (q == p) break;
            if (x >= 16 && x < budget) c.push_back((uint32_t)x);
            p = *q ? q + 1 : q;
        }
    }
    std::sort(c.begin(), c.end());
    c.erase(std::unique(c.begin(), c.end()), c.end());
    while (!c.empty() && c.back() >= budget) c.pop_back();
    c.push_back(budget);
    return c;
}

static uint64_t fnv1a64(const void* p, size_t n, uint64_t h) {
    const unsigned char* c = (const unsigned char*)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 0x100000001b3ull;
    return h;
}

uint32_t default_threads() {
    uint32_t threads = std::max(1u, std::min(4u, std::thread::hardware_concurrency()));
    if (const char* e = std::getenv("MH_JIT_THREADS")) threads = (uint32_t)std::max(1, atoi(e));
    return threads;
}

uint64_t code_id(const std::vector<Built>& built) {
    uint64_t h = 0xcbf29ce484222325ull;
    for (const Built& b : built) {
        h = fnv1a64(&b.text_hash, sizeof b.text_hash, h);
        h = fnv1a64(&b.n_groups, sizeof b.n_groups, h);
    }
    return h;
}

bool build_tapeset(const mh_node* nodes, const uint64_t* offs, uint32_t n_tapes,
                   const uint32_t* consts, uint32_t n_consts, uint32_t n_vars, bool values,
                   const Options& opt, uint32_t threads, std::vector<Built>& out,
                   BuildStats& stats, std::string& err) {
    threads = std::max<uint32_t>(1, std::min<uint32_t>(threads, (n_tapes + 63) / 64));
    out.clear();
    stats.jitted.assign(n_tapes, 0);
    stats.why.assign(n_tapes, std::string());
    // 1. emission, one slice of consecutive tapes per thread; tapes over the register budget go
    //    to `over` (null: they stay on the interpreter)
    struct Slice {
        std::vector<TapeCode> codes;
        std::vector<uint32_t> ids, over;
    };
    std::vector<Slice> slices(threads + 1);
    auto emit_list = [&](const std::vector<uint32_t>& list, const Options& o, Slice& sl,
                         bool keep_over) {
        std::vector<uint32_t> pool;
        ConstIndex index;
        sl.codes.reserve(list.size());
        for (uint32_t t : list) {
            SsaTape st;
            std::string e;
            if (lower_tape_ssa(nodes + offs[t], (size_t)(offs[t + 1] - offs[t]), consts, n_consts,
                               n_vars, pool, index, st, e, true, true) != MH_OK) {
                stats.why[t] = "lowering: " + e;
                continue;
            }
            TapeCode tc = emit_tape(st, pool, n_vars, o);
            if (!tc.ok && !keep_over && pinned_cols(n_vars) == 0 &&
                tc.why.find("VGPR pressure") != std::string::npos) {
                // still over the larger budget: every column use loads again instead of one
                // load kept live across the tape
                SsaTape st2;
                if (lower_tape_ssa(nodes + offs[t], (size_t)(offs[t + 1] - offs[t]), consts,
                                   n_consts, n_vars, pool, index, st2, e, kVnNoLoads,
                                   true) == MH_OK)
                    tc = emit_tape(st2, pool, n_vars, o);
            }
            if (tc.ok && code_bytes(tc) > 96 * 1024) {
                tc.ok = false;
                tc.why = "tape code larger than 96 KB";
            }
            if (!tc.ok) {
                stats.why[t] = tc.why;
                if (keep_over && tc.why.find("VGPR pressure") != std::string::npos)
                    sl.over.push_back(t);
                continue;
            }
            stats.jitted[t] = 1;
            stats.why[t].clear();
            sl.codes.push_back(std::move(tc));
            sl.ids.push_back(t);
        }
    };
    auto work = [&](uint32_t s) {
        const uint32_t lo = (uint32_t)((uint64_t)n_tapes * s / threads);
        const uint32_t hi = (uint32_t)((uint64_t)n_tapes * (s + 1) / threads);
        std::vector<uint32_t> list;
        for (uint32_t t = lo; t < hi; ++t) list.push_back(t);
        emit_list(list, opt, slices[s], true);
    };
    {
        std::vector<std::thread> pool;
        for (uint32_t s = 1; s < threads; ++s) pool.emplace_back(work, s);
        work(0);
        for (auto& th : pool) th.join();
    }
    // the tapes over the register budget, emitted with the larger one (fewer waves per SIMD for
    // them only) instead of the interpreter
    std::vector<uint32_t> big;
    for (uint32_t s = 0; s < threads; ++s)
        big.insert(big.end(), slices[s].over.begin(), slices[s].over.end());
    const uint32_t big_budget = std::max(opt.max_vgpr, opt.max_vgpr_keccak);
    if (!big.empty() && big_budget > opt.max_vgpr) {
        Options o2 = opt;
        o2.max_vgpr = big_budget;
        emit_list(big, o2, slices[threads], false);
    }
    // 2. occupancy classes over every emitted tape (tape order kept inside a class), each class
    //    cut into pieces of about n_tapes / threads tapes: one code object per piece
    const std::vector<uint32_t> cls = occupancy_classes(opt.max_vgpr);
    struct Piece {
        std::vector<const TapeCode*> codes;
        std::vector<uint32_t> ids;
    };
    std::vector<std::vector<std::pair<const TapeCode*, uint32_t>>> bins(cls.size() + 1);
    for (const Slice& sl : slices)
        for (size_t i = 0; i < sl.codes.size(); ++i) {
            const TapeCode& tc = sl.codes[i];
            stats.code_bytes += code_bytes(tc);
            stats.valu_static += tc.n_valu;
            stats.valu_wide_static += tc.n_valu_wide;
            const uint32_t need = module_vgprs(tc, n_vars);
            size_t c = 0;
            while (c < cls.size() && need > cls[c]) ++c;
            bins[c].push_back({&tc, sl.ids[i]});
        }
    const size_t per_piece = std::max<size_t>(64, (n_tapes + threads - 1) / threads);
    std::vector<Piece> pieces;
    for (auto& bin : bins) {
        if (bin.empty()) continue;
        std::stable_sort(bin.begin(), bin.end(),
                         [](const auto& a, const auto& b) { return a.second < b.second; });
        const size_t n_p = (bin.size() + per_piece - 1) / per_piece;
        for (size_t p = 0; p < n_p; ++p) {
            pieces.emplace_back();
            const size_t lo = bin.size() * p / n_p, hi = bin.size() * (p + 1) / n_p;
            for (size_t i = lo; i < hi; ++i) {
                pieces.back().codes.push_back(bin[i].first);
                pieces.back().ids.push_back(bin[i].second);
            }
        }
    }
    // 3. module text and assembly, the pieces shared out over the threads
    out.assign(pieces.size(), Built());
    const uint32_t group_bytes = default_group_bytes();
    std::atomic<size_t> next{0};
    auto assemble_work = [&]() {
        for (size_t p; (p = next.fetch_add(1)) < pieces.size();) {
            Built& b = out[p];
            b.tape_ids = pieces[p].ids;
            Module m = build_module(pieces[p].codes, pieces[p].ids, n_vars, false, group_bytes);
            b.n_groups = (uint32_t)m.group_first.size();
            b.max_vgpr = m.max_vgpr;
            b.text_hash = fnv1a64(m.text.data(), m.text.size(), 0xcbf29ce484222325ull);
            if (!opt.assemble) continue;
            std::string log;
            if (!assemble(m.text, b.hsaco, log)) {
                b.err = "assemble: " + log.substr(0, 2000);
                continue;
            }
            if (values) {
                Module mv = build_module(pieces[p].codes, pieces[p].ids, n_vars, true, group_bytes);
                if (!assemble(mv.text, b.hsaco_values, log))
                    b.err = "assemble (values): " + log.substr(0, 2000);
            }
        }
    };
    {
        std::vector<std::thread> pool;
        const size_t nt = std::min<size_t>(std::max<uint32_t>(threads, 1), pieces.size());
        for (size_t s = 1; s < nt; ++s) pool.emplace_back(assemble_work);
        assemble_work();
        for (auto& th : pool) th.join();
    }
    for (const Built& b : out) {
        if (!b.err.empty()) {
            err = b.err;
            return false;
        }
    }
    return true;
}

namespace {

// VGPRs an instruction writes (first, count); count 0 = none.  VALU ops write o[0] (a pair for
// v_mad_u64_u32 and the f64 ops) except the compares, which write an SGPR pair / VCC; LDS reads
// write o[0]; nothing else writes VGPRs.
std::pair<uint32_t, uint32_t> vgpr_writes(const MI& m) {
    const bool valu = m.op <= M_V_CMP_LE_F64 &&
                      !(m.op >= M_V_CMP_EQ && m.op <= M_V_CMP_GT_I32) && m.op != M_V_CMP_LE_F64 &&
                      m.op != M_V_CMP_GT_F32 && m.op != M_V_CMP_LE_F32;
    const bool lds_read = m.op == M_DS_READ2ST64 || m.op == M_DS_READ_B32;
    if ((valu || lds_read) && m.o[0].k == O_V) return {m.o[0].v, m.o[0].n};
    return {0, 0};
}

bool touches(const Opnd& o, uint32_t r) { return o.k == O_V && r >= o.v && r < o.v + o.n; }

// Copy coalescing at division call sites: `v_mov DY+k / DR+k, vX` where vX was written by one
// single-register VALU instruction earlier in the same straight-line stretch and is dead after
// the copy -- that instruction writes DY+k / DR+k directly (its reads of vX in between follow)
// and the copy goes.  Returns the number of copies removed.
uint32_t coalesce_div_moves(std::vector<MI>& code) {
    uint32_t removed = 0;
    std::vector<char> gone(code.size(), 0);
    for (size_t p = 0; p < code.size(); ++p) {
        const MI& mv = code[p];
        if (mv.op != M_V_MOV || mv.e64 || mv.o[0].k != O_V || mv.o[0].n != 1 ||
            mv.o[1].k != O_V || mv.o[1].n != 1)
            continue;
        const uint32_t t = mv.o[0].v, x = mv.o[1].v;
        if (!((t >= R_DY && t < R_DY + 8) || (t >= R_DR && t < R_DR + 8)) || x < R_TEMP0) continue;
        // the call this copy feeds: only copies / scalar moves until it
        size_t c = p + 1;
        while (c < code.size() && (code[c].op == M_V_MOV || code[c].op == M_S_MOV_B32)) ++c;
        if (c >= code.size() || code[c].op != M_CALL_DIV) continue;
        // x dead after the copy (forward, to the tape's end: the subroutine keeps to v40-v79)
        bool live = false;
        for (size_t f = p + 1; f < code.size() && !live; ++f) {
            if (gone[f]) continue;
            const MI& m = code[f];
            const auto w = vgpr_writes(m);
            for (int k = 0; k < 5; ++k) {
                if (w.second && k == 0) continue;
                if (touches(m.o[k], x)) live = true;
            }
            if (!live && w.second && x >= w.first && x < w.first + w.second) break;  // rewritten
        }
        if (live) continue;
        // the producer: the last writer of x, in straight-line code, with t untouched since
        size_t q = p;
        bool ok = false;
        while (q-- > 0) {
            if (gone[q]) continue;
            const MI& m = code[q];
            if (m.op == M_LABEL || m.op == M_CALL_DIV || m.op == M_CALL_KEC || m.op == M_RET ||
                m.op == M_S_CBRANCH_SCC0 || m.op == M_S_CBRANCH_SCC1 || m.op == M_S_BRANCH)
                break;
            bool tt = false, pair_read = false;
            const auto w = vgpr_writes(m);
            for (int k = 0; k < 5; ++k) {
                tt |= touches(m.o[k], t);
                if (!(w.second && k == 0) && m.o[k].n > 1 && touches(m.o[k], x)) pair_read = true;
            }
            if (w.second && x >= w.first && x < w.first + w.second) {
                ok = w.second == 1 && w.first == x && !tt;
                break;
            }
            if (tt || pair_read) break;
        }
        if (!ok) continue;
        code[q].o[0].v = t;
        for (size_t i = q + 1; i < p; ++i)
            for (int k = 0; k < 5; ++k)
                if (code[i].o[k].k == O_V && code[i].o[k].n == 1 && code[i].o[k].v == x)
                    code[i].o[k].v = t;
        gone[p] = 1;
        ++removed;
    }
    if (removed) {
        std::vector<MI> out;
        out.reserve(code.size() - removed);
        for (size_t i = 0; i < code.size(); ++i)
            if (!gone[i]) out.push_back(code[i]);
        code.swap(out);
    }
    return removed;
}

}  // namespace

static std::atomic<uint64_t> g_sc_fallbacks{0};

uint64_t sc_fallbacks(bool reset) {
    return reset ? g_sc_fallbacks.exchange(0) : g_sc_fallbacks.load();
}

TapeCode emit_tape(const SsaTape& st, const std::vector<uint32_t>& pool, uint32_t n_vars,
                   const Options& opt) {
    TapeCode tc = emit_tape_body(st, pool, n_vars, opt);
    if (tc.ok && opt.coalesce) {
        const uint32_t r = coalesce_div_moves(tc.code);
        tc.n_valu -= r;
    }
    return tc;
}

TapeCode emit_tape_body(const SsaTape& st, const std::vector<uint32_t>& pool, uint32_t n_vars,
                        const Options& opt) {
    // source order first: the tape's code when there is no conjunction to reorder, and the VALU
    // each SSA instruction costs (the scheduler's cost model) when there is
    std::vector<double> cost;
    Emitter e(st, pool, n_vars, opt, nullptr, opt.short_circuit ? &cost : nullptr);
    TapeCode tc0 = e.run();
    if (opt.short_circuit) {
        SsaTape sc;
        std::vector<uint8_t> check;
        if (schedule_conjuncts(st, pool, opt.sample_rows, tc0.ok ? &cost : nullptr, sc, check)) {
            Emitter e2(sc, pool, n_vars, opt, &check);
            TapeCode tc = e2.run();
            if (tc.ok) return tc;  // else (register pressure of the new order): source order
            g_sc_fallbacks.fetch_add(1, std::memory_order_relaxed);
        }
    }
    return tc0;
}

}  // namespace jit
}  // namespace mh
