// The query compiler behind the C-ABI (mh_terms_*, mh_query_*): lowering, bucketing and tape
// linearisation of one get_model query in C++ (Sieve.solve's host stages).
//
// A session (mh_terms) mirrors the host's hash-consed term store (mythril_amd/tape.py
// TapeBuilder): its nodes with their flags, its 256-bit constant pool and the symbol tables
// (variable, array and function names), appended incrementally.  mh_query_build then does what
// mythril_amd/lower.py lower_query, sieve.py Sieve.bucket_roots and sieve.py local_tapeset do for
// the conjunction of some root nodes, with the same results (tests/test_query_native.py):
//
//  * pass 1 (lower.py Lowering.collect / apply_harvest): the constant keys each free array and
//    each non-keccak function is read at, the concrete keccak pairs keccak256_N(c) == k and the
//    greatest lower bound a keccak application is compared with;
//  * pass 2 (Lowering.lower / _rewrite): only nodes that are or read host-only terms (F_HOST) are
//    rewritten -- select / store chains to ite chains over the store keys and the array's cell
//    columns (name "A[0x..]", else column "A[*]"), K(v) to v, keccak256_N to ite(x == c_i, k_i,
//    base + ((keccak(x) >> 139) << 6)), keccak256_N-1(keccak256_N(x)) to x, other functions
//    tabled like arrays, equalities wider than 256 bits split on both sides' concat boundaries;
//  * the AND leaves of the lowered conjunction split into column-disjoint groups (Sieve.buckets,
//    the DependenceMap of laser/smt/solver/independence_solver.py:38-83), ordered by their first
//    conjunct, ground conjuncts one group per node;
//  * the root tape (the guide's input) and, with more than one group, one tape per group (the
//    AND of its conjuncts in path order), over the query's own columns and constants.
//
// A query whose lowered conjuncts have the shape of a symbol definition (sieve.py
// eliminate_definitions: variable == computed term) is flagged MH_QUERY_DEFINITIONS; the host
// then takes its Python stages.  A session is used by one thread at a time (scratch is shared).
#include <algorithm>
#include <array>
#include <cstdint>
#include <cstring>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/mythril_hip.h"

int32_t mh_detail_set_err(int32_t code, const char* msg);  // capi.cpp

namespace {

enum : uint8_t {
    CONST = 0, VAR = 1, TRUE_ = 2, FALSE_ = 3, BVADD = 10, BVSHL = 23, BVLSHR = 24, EQ = 30,
    BVULT = 31, BVSGE = 38, AND = 40, ITE = 45, EXTRACT = 50, CONCAT = 51, ZEXT = 52, SEXT = 53,
    KECCAK = 60, ARRAY = 80, CONST_ARRAY = 81, STORE = 82, SELECT = 83, UF = 84,
};
constexpr uint8_t F_ARRAY = 1, F_HOST = 2;
constexpr uint32_t KECCAK_SHIFT = 139, KECCAK_ALIGN = 6;  // lower.py KECCAK_SHIFT / KECCAK_ALIGN
constexpr int NL = MH_QUERY_KEY_LIMBS;                     // 1152-bit host values (<= 1088 used)
constexpr uint32_t OWN = 0x80000000u;       // node id of a query-made node: OWN | index into ov
constexpr uint32_t OV_CONST = 0x80000000u;  // query-made CONST imm0: index into the query's values
constexpr uint32_t CELL_COL = 0x40000000u;  // query-made VAR imm0: index into the query's cells

struct Fail {
    int32_t code;
    std::string msg;
};
[[noreturn]] void unsupported(const std::string& m) { throw Fail{MH_E_UNSUPPORTED, m}; }
[[noreturn]] void invalid(const std::string& m) { throw Fail{MH_E_INVALID, m}; }

int arity(uint8_t op) {  // tape.py ARITY
    switch (op) {
        case CONST: case VAR: case TRUE_: case FALSE_: case ARRAY: return 0;
        case MH_OP_BVNEG: case MH_OP_BVNOT: case MH_OP_NOT: case EXTRACT: case ZEXT: case SEXT:
        case KECCAK: case CONST_ARRAY: case UF: return 1;
        case ITE: case MH_OP_EVM_ADDMOD: case MH_OP_EVM_MULMOD: case STORE: return 3;
        default: return 2;
    }
}

struct Big {  // unsigned, little-endian u32 limbs
    uint32_t w[NL] = {};
    bool operator==(const Big& o) const { return memcmp(w, o.w, sizeof w) == 0; }
    bool operator<(const Big& o) const {
        for (int i = NL - 1; i >= 0; --i)
            if (w[i] != o.w[i]) return w[i] < o.w[i];
        return false;
    }
    bool zero() const {
        for (uint32_t x : w)
            if (x) return false;
        return true;
    }
    Big shr(uint32_t s) const {
        Big r;
        const uint32_t q = s / 32, b = s % 32;
        for (uint32_t i = 0; i + q < NL; ++i) {
            uint64_t v = w[i + q] >> b;
            if (b && i + q + 1 < NL) v |= (uint64_t)w[i + q + 1] << (32 - b);
            r.w[i] = (uint32_t)v;
        }
        return r;
    }
    Big shl(uint32_t s) const {
        Big r;
        const uint32_t q = s / 32, b = s % 32;
        for (uint32_t i = q; i < NL; ++i) {
            uint64_t v = (uint64_t)w[i - q] << b;
            if (b && i > q) v |= w[i - q - 1] >> (32 - b);
            r.w[i] = (uint32_t)v;
        }
        return r;
    }
    Big masked(uint32_t bits) const {
        Big r = *this;
        for (uint32_t i = 0; i < NL; ++i) {
            const uint32_t lo = 32 * i;
            if (lo >= bits) r.w[i] = 0;
            else if (bits - lo < 32) r.w[i] &= (1u << (bits - lo)) - 1u;
        }
        return r;
    }
    Big operator|(const Big& o) const {
        Big r;
        for (int i = 0; i < NL; ++i) r.w[i] = w[i] | o.w[i];
        return r;
    }
    Big plus(uint32_t v) const {
        Big r = *this;
        uint64_t c = v;
        for (int i = 0; i < NL && c; ++i) {
            c += r.w[i];
            r.w[i] = (uint32_t)c;
            c >>= 32;
        }
        return r;
    }
    Big minus_one() const {  // *this - 1, for *this > 0
        Big r = *this;
        for (int i = 0; i < NL; ++i)
            if (r.w[i]--) break;
        return r;
    }
    Big times(const Big& o) const {  // exact for operands below 2^576
        Big r;
        for (int i = 0; i < NL / 2; ++i) {
            uint64_t carry = 0;
            for (int j = 0; i + j < NL; ++j) {
                const uint64_t cur = (uint64_t)w[i] * (j < NL / 2 ? o.w[j] : 0u) + r.w[i + j] + carry;
                r.w[i + j] = (uint32_t)cur;
                carry = cur >> 32;
            }
        }
        return r;
    }
    Big operator+(const Big& o) const {
        Big r;
        uint64_t c = 0;
        for (int i = 0; i < NL; ++i) {
            c += (uint64_t)w[i] + o.w[i];
            r.w[i] = (uint32_t)c;
            c >>= 32;
        }
        return r;
    }
    bool bit(uint32_t i) const { return (w[i / 32] >> (i % 32)) & 1u; }
    std::string hex() const {  // Python's "%#x"
        static const char* d = "0123456789abcdef";
        int i = NL * 8 - 1;
        while (i > 0 && !((w[i / 8] >> (4 * (i % 8))) & 15u)) --i;
        std::string s = "0x";
        for (; i >= 0; --i) s += d[(w[i / 8] >> (4 * (i % 8))) & 15u];
        return s;
    }
};
struct BigHash {
    size_t operator()(const Big& b) const {
        uint64_t h = 1469598103934665603ull;
        for (int i = 0; i < 9; ++i) h = (h ^ b.w[i]) * 1099511628211ull;  // low 288 bits
        return (size_t)h;
    }
};

struct Key {
    uint32_t op, width, a, b, c, imm0, imm1;
    bool operator==(const Key& o) const {
        return op == o.op && width == o.width && a == o.a && b == o.b && c == o.c &&
               imm0 == o.imm0 && imm1 == o.imm1;
    }
};
struct KeyHash {
    size_t operator()(const Key& k) const {
        uint64_t h = 0x9E3779B97F4A7C15ull * (k.op + 1);
        const uint32_t v[6] = {k.width, k.a, k.b, k.c, k.imm0, k.imm1};
        for (uint32_t x : v) h = (h ^ x) * 0xFF51AFD7ED558CCDull + (h >> 29);
        return (size_t)h;
    }
};
Key key_of(const mh_node& x) { return Key{x.op, x.width, x.a, x.b, x.c, x.imm0, x.imm1}; }

// a node -> value map valid for one epoch (reset in O(1) between queries)
struct Stamped {
    std::vector<uint32_t> stamp, val;
    uint32_t epoch = 1;
    void reset(size_t n) {
        if (++epoch == 0) {
            std::fill(stamp.begin(), stamp.end(), 0u);
            epoch = 1;
        }
        if (stamp.size() < n) {
            stamp.resize(n, 0u);
            val.resize(n);
        }
    }
    bool has(size_t i) const { return i < stamp.size() && stamp[i] == epoch; }
    void unset(size_t i) {
        if (i < stamp.size()) stamp[i] = 0u;  // epochs start at 1
    }
    uint32_t get(size_t i) const { return val[i]; }
    void set(size_t i, uint32_t v) {
        if (i >= stamp.size()) {
            const size_t n = std::max(i + 1, 2 * stamp.size());
            stamp.resize(n, 0u);
            val.resize(n);
        }
        stamp[i] = epoch;
        val[i] = v;
    }
};

}  // namespace

struct mh_terms {
    std::vector<mh_node> nodes;
    std::unordered_map<Key, uint32_t, KeyHash> memo;  // TapeBuilder._memo
    std::vector<Big> pool;
    std::unordered_map<Big, uint32_t, BigHash> pool_index;
    std::vector<std::string> var_names, array_names, fn_names;
    // const_value of the mirrored nodes (immutable): 0 unknown, 1 none, k + 2 = cv_vals[k]
    std::vector<uint32_t> cv_state;
    std::vector<Big> cv_vals;
    Stamped memo_lower, seen, local;  // per-query scratch (mirrored node ids)
    std::unique_ptr<class QueryState> last;  // the last query, kept for a child that extends it
    uint32_t options = 0;                     // MH_TERMS_*
};

namespace {

struct Column {
    std::string name, symbol;
    uint32_t width, kind;
    bool has_key;
    Big key;
};

struct KeccakMap {
    Big bound, base;
    bool has_bound = false;
    std::vector<std::pair<Big, Big>> pairs;  // (argument, hash); a later statement of a key wins
    bool put(const Big& arg, const Big& h) {  // true: the table changed
        for (auto& p : pairs)
            if (p.first == arg) {
                const bool changed = !(p.second == h);
                p.second = h;
                return changed;
            }
        pairs.emplace_back(arg, h);
        return true;
    }
};

using Tables = std::vector<std::pair<std::string, std::vector<Big>>>;

class Query {
public:
    // a fresh query: the per-query scratch starts a new epoch (the lowering memo too, unless the
    // caller may adopt the last query's lowering: adopt_lowering, or reset_lowering if not)
    explicit Query(mh_terms& t, bool keep_lowering = false) : T(t) {
        if (!keep_lowering) T.memo_lower.reset(T.nodes.size());
        T.seen.reset(T.nodes.size());
        T.local.reset(T.nodes.size());
        sync();
    }
    void reset_lowering() { T.memo_lower.reset(T.nodes.size()); }
    // the lowering memo (T.memo_lower, kept) is valid for this query when its harvest equals the
    // one the memo was made under: take over the nodes, constants and cell columns it refers to
    bool same_harvest(const Query& o) const {
        if (cells != o.cells || uf_cells != o.uf_cells || keccak.size() != o.keccak.size())
            return false;
        for (size_t i = 0; i < keccak.size(); ++i) {
            const KeccakMap& a = keccak[i].second;
            const KeccakMap& b = o.keccak[i].second;
            if (keccak[i].first != o.keccak[i].first || !(a.base == b.base) ||
                a.has_bound != b.has_bound || !(a.bound == b.bound) || a.pairs != b.pairs)
                return false;
        }
        return true;
    }
    void adopt_lowering(Query& o) {
        ov = std::move(o.ov);
        ov_memo = std::move(o.ov_memo);
        ov_vals = std::move(o.ov_vals);
        ov_index = std::move(o.ov_index);
        ov_cv = std::move(o.ov_cv);
        ov_cv_vals = std::move(o.ov_cv_vals);
        ccols = std::move(o.ccols);
        cell_index = std::move(o.cell_index);
        read_li = std::move(o.read_li);
    }
    // the harvest tables, copied whole (a state keeps one per depth at which its harvest grew)
    struct HarvestCopy {
        Tables cells, uf_cells;
        std::unordered_map<std::string, size_t> cell_of, uf_of, kidx;
        std::vector<std::pair<std::string, KeccakMap>> keccak;
        uint64_t hver = 0;
    };
    HarvestCopy save_harvest() const {
        return HarvestCopy{cells, uf_cells, cell_of, uf_of, kidx, keccak, hver};
    }
    void restore_harvest(const HarvestCopy& h) {
        cells = h.cells;
        uf_cells = h.uf_cells;
        cell_of = h.cell_of;
        uf_of = h.uf_of;
        kidx = h.kidx;
        keccak = h.keccak;
        hver = h.hver;
    }
    void sync() {  // the mirror may have grown since the query was made
        if (T.cv_state.size() < T.nodes.size()) T.cv_state.resize(T.nodes.size(), 0u);
    }

    // ---- nodes: mirrored ids below OWN, the query's own OWN | i -------------------------------
    const mh_node& nd(uint32_t n) const { return n & OWN ? ov[n & ~OWN] : T.nodes[n]; }
    uint32_t width(uint32_t n) const { return nd(n).width; }

    uint32_t add(uint8_t op, uint32_t w, uint32_t a = 0, uint32_t b = 0, uint32_t c = 0,
                 uint32_t i0 = 0, uint32_t i1 = 0) {
        const Key k{op, w, a, b, c, i0, i1};
        auto it = ov_memo.find(k);  // the query's own first (a node the host made later is the same)
        if (it != ov_memo.end()) return it->second;
        auto m = T.memo.find(k);  // hash-consed against the host's nodes
        if (m != T.memo.end()) return m->second;
        mh_node x{};
        x.op = op;
        x.width = (uint16_t)w;
        x.a = a;
        x.b = b;
        x.c = c;
        x.imm0 = i0;
        x.imm1 = i1;
        ov.push_back(x);
        const uint32_t id = OWN | (uint32_t)(ov.size() - 1);
        ov_memo.emplace(k, id);
        return id;
    }
    uint32_t konst(const Big& v, uint32_t w) {  // TapeBuilder.const
        if (w > 256) {
            const uint32_t lo = konst(v.masked(256), 256);
            const uint32_t hi = konst(v.shr(256), w - 256);
            return add(CONCAT, w, hi, lo);
        }
        const Big m = v.masked(w);
        auto p = T.pool_index.find(m);
        if (p != T.pool_index.end()) return add(CONST, w, 0, 0, 0, p->second);
        auto it = ov_index.find(m);
        if (it == ov_index.end()) {
            it = ov_index.emplace(m, (uint32_t)ov_vals.size()).first;
            ov_vals.push_back(m);
        }
        return add(CONST, w, 0, 0, 0, OV_CONST | it->second);
    }
    const Big& const_of(uint32_t n) const {  // a CONST node's value
        const uint32_t i0 = nd(n).imm0;
        return (n & OWN) && (i0 & OV_CONST) ? ov_vals[i0 & ~OV_CONST] : T.pool.at(i0);
    }

    // TapeBuilder.const_value: CONST / TRUE / FALSE and CONCAT / EXTRACT / ZEXT / SEXT over them
    const Big* const_value(uint32_t n) {
        if (!(n & OWN)) {
            const uint32_t s = T.cv_state[n];
            if (s) return s == 1 ? nullptr : &T.cv_vals[s - 2];
        } else {
            auto it = ov_cv.find(n);
            if (it != ov_cv.end()) return it->second < 0 ? nullptr : &ov_cv_vals[(size_t)it->second];
        }
        const mh_node x = nd(n);
        bool ok = false;
        Big v;
        if (x.op == CONST) {
            ok = true;
            v = const_of(n);
        } else if (x.op == TRUE_) {
            ok = true;
            v.w[0] = 1;
        } else if (x.op == FALSE_) {
            ok = true;
        } else if (x.op == CONCAT) {
            if (const Big* hi = const_value(x.a)) {
                const Big h = *hi;
                if (const Big* lo = const_value(x.b)) {
                    ok = true;
                    v = h.shl(width(x.b)) | *lo;
                }
            }
        } else if (x.op == EXTRACT || x.op == ZEXT || x.op == SEXT) {
            if (const Big* a = const_value(x.a)) {
                ok = true;
                if (x.op == EXTRACT) {
                    v = a->shr(x.imm1).masked(x.imm0 - x.imm1 + 1);
                } else if (x.op == SEXT && a->bit(width(x.a) - 1)) {
                    Big ones;
                    for (uint32_t i = 0; i < x.imm0; ++i) ones.w[i / 32] |= 1u << (i % 32);
                    v = *a | ones.shl(width(x.a));
                } else {
                    v = *a;
                }
            }
        }
        // callers copy a value before the next const_value (the vectors may grow)
        if (!(n & OWN)) {
            if (!ok) {
                T.cv_state[n] = 1;
                return nullptr;
            }
            T.cv_vals.push_back(v);
            T.cv_state[n] = (uint32_t)T.cv_vals.size() + 1;
            return &T.cv_vals.back();
        }
        if (!ok) {
            ov_cv[n] = -1;
            return nullptr;
        }
        ov_cv_vals.push_back(v);
        ov_cv[n] = (int64_t)ov_cv_vals.size() - 1;
        return &ov_cv_vals.back();
    }

    // ---- pass 1: lower.py Lowering.collect + apply_harvest -----------------------------------
    const std::string& array_name(uint32_t n) const { return T.array_names.at(nd(n).imm0); }
    const std::string& fn_name(uint32_t n) const { return T.fn_names.at(nd(n).imm0); }
    static bool inverse(const std::string& f) {
        return f.size() >= 2 && f.compare(f.size() - 2, 2, "-1") == 0;
    }
    static bool keccak_fn(const std::string& f) { return f.rfind("keccak256_", 0) == 0 && !inverse(f); }

    int64_t array_base(uint32_t arr) const {  // the ARRAY under a store chain, -1 for K(...)
        for (;;) {
            const uint8_t op = nd(arr).op;
            if (op == STORE) arr = nd(arr).a;
            else if (op == ARRAY) return arr;
            else if (op == CONST_ARRAY) return -1;
            else unsupported("array term is not a store chain");
        }
    }
    static std::vector<Big>& keys_of(Tables& tabs, std::unordered_map<std::string, size_t>& idx,
                                     const std::string& n) {
        auto it = idx.find(n);
        if (it == idx.end()) {
            it = idx.emplace(n, tabs.size()).first;
            tabs.emplace_back(n, std::vector<Big>());
        }
        return tabs[it->second].second;
    }
    KeccakMap& keccak_map(const std::string& f) {
        auto it = kidx.find(f);
        if (it == kidx.end()) {
            it = kidx.emplace(f, keccak.size()).first;
            keccak.emplace_back(f, KeccakMap());
        }
        return keccak[it->second].second;
    }

    void harvest(const std::vector<uint32_t>& roots) {
        // per root, in order, children before parents, host-only nodes and their parents only
        // (lower.py _walk over each constraint; Harvest.merge: a later root's keccak pair wins)
        std::vector<int64_t> st;
        for (uint32_t r : roots) {
            if (!(nd(r).flags & F_HOST)) continue;
            polarity(r);
            T.seen.reset(T.nodes.size());
            st.assign(1, r);
            walk_host(st);
        }
        finish_harvest();
    }
    // lower.py _polarity: the host-only comparisons / equalities reached from the root through
    // AND / OR / NOT only, 1 positive | 2 negative (NOT flips); absent = positive
    std::unordered_map<uint32_t, uint8_t> pol;
    void polarity(uint32_t r) {
        pol.clear();
        std::vector<std::pair<uint32_t, uint8_t>> st{{r, 0}};
        std::unordered_set<uint64_t> vis;
        while (!st.empty()) {
            const auto [n, neg] = st.back();
            st.pop_back();
            if (!vis.insert((uint64_t)n << 1 | neg).second) continue;
            const mh_node& x = nd(n);
            if (x.op == AND || x.op == MH_OP_OR) {
                for (uint32_t k : {x.a, x.b})
                    if (nd(k).flags & F_HOST) st.push_back({k, neg});
            } else if (x.op == MH_OP_NOT) {
                if (nd(x.a).flags & F_HOST) st.push_back({x.a, (uint8_t)(neg ^ 1)});
            } else {
                pol[n] |= neg ? 2 : 1;
            }
        }
    }
    void walk_host(std::vector<int64_t>& st) {
        while (!st.empty()) {
            const int64_t s = st.back();
            st.pop_back();
            if (s < 0) {
                collect((uint32_t)~s);
                continue;
            }
            if (T.seen.has((size_t)s)) continue;
            T.seen.set((size_t)s, 1);
            st.push_back(~s);
            const mh_node& x = nd((uint32_t)s);
            const uint32_t kids[3] = {x.a, x.b, x.c};
            for (int j = arity(x.op) - 1; j >= 0; --j)
                if (!T.seen.has(kids[j]) && (nd(kids[j]).flags & F_HOST)) st.push_back(kids[j]);
        }
    }
    // changes whenever the harvest does (a key, a keccak function, a pair or a bound added):
    // start() finds the depth from which a state's prefixes all have its harvest
    std::array<uint64_t, 4> harvest_sig() const {
        uint64_t nc = 0, nu = 0;
        for (const auto& kv : cells) nc += kv.second.size() + 1;
        for (const auto& kv : uf_cells) nu += kv.second.size() + 1;
        return {nc, nu, (uint64_t)keccak.size(), hver};
    }
    void finish_harvest() {  // lower.py apply_harvest: sorted keys, the keccak bases
        for (Tables* tabs : {&cells, &uf_cells})
            for (auto& kv : *tabs) {
                std::sort(kv.second.begin(), kv.second.end());
                kv.second.erase(std::unique(kv.second.begin(), kv.second.end()), kv.second.end());
            }
        for (auto& kv : keccak) {
            KeccakMap& km = kv.second;
            km.base = km.has_bound ? km.bound.plus(63) : Big();
            km.base.w[0] &= ~63u;
            km.base = km.base.masked(256);
        }
    }
    void collect(uint32_t n) {
        const mh_node x = nd(n);
        if (x.op == SELECT) {
            const int64_t base = array_base(x.a);
            if (base >= 0) {
                auto& keys = keys_of(cells, cell_of, array_name((uint32_t)base));
                if (const Big* k = const_value(x.b)) keys.push_back(*k);
            }
        } else if (x.op == UF) {
            const std::string& f = fn_name(n);
            if (keccak_fn(f)) {
                keccak_map(f);
            } else if (!inverse(f)) {
                auto& keys = keys_of(uf_cells, uf_of, f);
                if (const Big* k = const_value(x.a)) keys.push_back(*k);
            }
        } else if (x.op == EQ || (x.op >= BVULT && x.op <= BVSGE)) {
            uint8_t op = x.op;
            auto pi = pol.find(n);
            if (pi != pol.end() && pi->second == 2) {
                // reached only under an odd number of NOTs: the negated comparison (ADVICE r5:
                // Not(UGT(f(x), c)) is an upper bound); a disequality states no pair
                if (op == EQ) return;
                static const uint8_t neg_of[8] = {MH_OP_BVUGE, MH_OP_BVUGT, MH_OP_BVULE,
                                                  MH_OP_BVULT, MH_OP_BVSGE, MH_OP_BVSGT,
                                                  MH_OP_BVSLE, MH_OP_BVSLT};
                op = neg_of[op - BVULT];
            }
            const uint32_t sides[2][2] = {{x.a, x.b}, {x.b, x.a}};
            for (const auto& s : sides) {
                const mh_node& app = nd(s[0]);
                if (app.op != UF || !keccak_fn(fn_name(s[0]))) continue;
                const Big* kv = const_value(s[1]);
                if (!kv) continue;
                const Big hv = *kv;
                KeccakMap& km = keccak_map(fn_name(s[0]));
                if (x.op == EQ) {
                    if (const Big* arg = const_value(app.a)) hver += km.put(*arg, hv);
                    continue;
                }
                // a lower bound on the application (f > k, f >= k, k < f, k <= f): the
                // interval's base is the greatest of them; upper bounds and signed orders
                // bound nothing here (lower.py Lowering.collect)
                const bool left = &s == &sides[0];
                bool lower = false, strict = false;
                if (left && (op == MH_OP_BVUGT || op == MH_OP_BVUGE)) {
                    lower = true;
                    strict = op == MH_OP_BVUGT;
                } else if (!left && (op == BVULT || op == MH_OP_BVULE)) {
                    lower = true;
                    strict = op == BVULT;
                }
                if (!lower) continue;
                const Big lb = strict ? hv.plus(1) : hv;
                if (!km.has_bound || km.bound < lb) {
                    km.bound = lb;
                    km.has_bound = true;
                    ++hver;
                }
            }
        }
    }

    // ---- pass 2: lower.py Lowering.lower / _rewrite -------------------------------------------
    uint32_t cell_column(const std::string& name, uint32_t w, uint32_t kind,
                         const std::string& sym, const Big* key, uint32_t li = UINT32_MAX) {
        auto it = cell_index.find(name);
        if (it == cell_index.end()) {
            it = cell_index.emplace(name, (uint32_t)ccols.size()).first;
            ccols.push_back(Column{name, sym, w, kind, key != nullptr, key ? *key : Big()});
            read_li.push_back(li);  // a read's index term (the first lowering that made it)
        }
        return add(VAR, w, 0, 0, 0, CELL_COL | it->second);
    }
    static bool read_kind(uint32_t k) {
        return k == MH_COL_READ || k == MH_COL_UFREAD || k == MH_COL_KREAD;
    }

    void deps(uint32_t n, std::vector<uint32_t>& d) {  // Lowering._deps
        d.clear();
        const mh_node& x = nd(n);
        if (x.op == SELECT) {
            d.push_back(x.b);
            uint32_t arr = x.a;
            while (nd(arr).op == STORE) {
                d.push_back(nd(arr).b);
                d.push_back(nd(arr).c);
                arr = nd(arr).a;
            }
            if (nd(arr).op == CONST_ARRAY) d.push_back(nd(arr).a);
            else if (nd(arr).op != ARRAY) unsupported("array term is not a store chain");
            return;
        }
        if (x.op == UF) {
            const std::string& f = fn_name(n);
            if (inverse(f)) {
                const mh_node& in = nd(x.a);
                const std::string fwd = f.substr(0, f.size() - 2);
                if (in.op != UF || T.fn_names.at(in.imm0) != fwd)
                    unsupported(f + " applied to something other than " + fwd + "(...)");
                d.push_back(in.a);
            } else {
                d.push_back(x.a);
            }
            return;
        }
        if (x.flags & F_ARRAY) unsupported("array-sorted term used as a value");
        const uint32_t kids[3] = {x.a, x.b, x.c};
        for (int j = 0; j < arity(x.op); ++j) {
            if (nd(kids[j]).flags & F_ARRAY) unsupported("operator over arrays");
            d.push_back(kids[j]);
        }
    }

    uint32_t low(uint32_t n) const {  // the lowered form of an operand
        return T.memo_lower.has(n) ? T.memo_lower.get(n) : n;
    }
    uint32_t lower(uint32_t root) {
        if (!(nd(root).flags & F_HOST)) return root;  // reads no host-only term: itself
        std::vector<std::pair<uint32_t, bool>> st{{root, false}};
        std::vector<uint32_t> d;
        while (!st.empty()) {
            const auto [n, expanded] = st.back();
            st.pop_back();
            if (T.memo_lower.has(n)) continue;
            if (!expanded) {
                st.push_back({n, true});
                deps(n, d);
                for (uint32_t x : d)
                    if ((nd(x).flags & F_HOST) && !T.memo_lower.has(x)) st.push_back({x, false});
                continue;
            }
            T.memo_lower.set(n, rewrite(n));
        }
        return T.memo_lower.get(root);
    }

    uint32_t rewrite(uint32_t n) {
        const mh_node x = nd(n);
        if (x.op == SELECT) return select(x.a, low(x.b), x.b);
        if (x.op == UF) return apply(n);
        const int k = arity(x.op);
        if (k == 0) return n;
        const uint32_t kids[3] = {x.a, x.b, x.c};
        uint32_t args[3] = {0, 0, 0};
        bool same = true;
        for (int j = 0; j < k; ++j) {
            args[j] = low(kids[j]);
            same = same && args[j] == kids[j];
        }
        if (x.op == EQ && width(args[0]) > 256) return eq(args[0], args[1]);
        if (same) return n;
        return add(x.op, x.width, args[0], args[1], args[2], x.imm0, x.imm1);
    }

    uint32_t eq(uint32_t x, uint32_t y) {  // Lowering.eq
        const uint32_t w = width(x);
        if (w <= 256) return add(EQ, 0, x, y);
        struct Seg {
            uint32_t lo, hi, p;
        };
        std::vector<Seg> sides[2];
        std::vector<uint32_t> cuts{w};
        const uint32_t ts[2] = {x, y};
        for (int s = 0; s < 2; ++s) {
            uint32_t pos = w;
            for (uint32_t p : pieces(ts[s])) {
                const uint32_t pw = width(p);
                sides[s].push_back({pos - pw, pos, p});
                cuts.push_back(pos - pw);
                pos -= pw;
            }
        }
        std::sort(cuts.begin(), cuts.end());
        cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
        int64_t acc = -1;
        for (size_t i = 0; i + 1 < cuts.size(); ++i) {
            const uint32_t lo = cuts[i], hi = cuts[i + 1];
            uint32_t parts[2] = {0, 0};
            for (int s = 0; s < 2; ++s)
                for (const Seg& g : sides[s])
                    if (g.lo <= lo && hi <= g.hi) {
                        parts[s] = slice(g.p, hi - g.lo, lo - g.lo);
                        break;
                    }
            const uint32_t e = add(EQ, 0, parts[0], parts[1]);
            acc = acc < 0 ? e : add(AND, 0, (uint32_t)acc, e);
        }
        return (uint32_t)acc;
    }
    std::vector<uint32_t> pieces(uint32_t n) {  // Lowering._pieces: CONCAT leaves, high first
        std::vector<uint32_t> out, st{n};
        while (!st.empty()) {
            const uint32_t x = st.back();
            st.pop_back();
            const mh_node v = nd(x);
            if (v.op == CONCAT) {
                st.push_back(v.b);
                st.push_back(v.a);
            } else if (v.op == ZEXT) {
                st.push_back(v.a);
                st.push_back(konst(Big(), v.imm0));
            } else if (v.width > 256 && !const_value(x)) {
                unsupported(std::to_string(v.width) + "-bit operand of a wide equality");
            } else {
                out.push_back(x);
            }
        }
        return out;
    }
    uint32_t slice(uint32_t piece, uint32_t hi, uint32_t lo) {  // bits [lo, hi) (Lowering._slice)
        if (lo == 0 && hi == width(piece)) return piece;
        if (const Big* c = const_value(piece)) {
            const Big v = c->shr(lo);
            return konst(v, hi - lo);
        }
        return add(EXTRACT, hi - lo, piece, 0, 0, hi - 1, lo);
    }

    uint32_t select(uint32_t arr, uint32_t idx, uint32_t idx_orig) {  // Lowering._select
        const mh_node a = nd(arr);
        if (a.op == STORE) {
            const uint32_t key = low(a.b), val = low(a.c);
            const uint32_t rest = select(a.a, idx, idx_orig);
            return add(ITE, width(val), eq(idx, key), val, rest);
        }
        if (a.op == CONST_ARRAY) return low(a.a);
        const std::string& name = array_name(arr);
        auto it = cell_of.find(name);
        return table(name, a.width, idx, it == cell_of.end() ? nullptr : &cells[it->second].second,
                     MH_COL_CELL, MH_COL_READ, idx_orig);
    }
    // _table: a constant key's cell; any other index the cells' ite chain over its read column
    // name[@idx_orig] (Ackermann's reduction)
    uint32_t table(const std::string& name, uint32_t rng, uint32_t idx,
                   const std::vector<Big>* keys, uint32_t kcell, uint32_t kread,
                   uint32_t idx_orig) {
        const Big* kp = const_value(idx);
        const Big key = kp ? *kp : Big();
        if (kp && keys && std::binary_search(keys->begin(), keys->end(), key))
            return cell_column(name + "[" + key.hex() + "]", rng, kcell, name, &key);
        Big ik;
        ik.w[0] = idx_orig;
        uint32_t acc = cell_column(name + "[@" + std::to_string(idx_orig) + "]", rng, kread, name,
                                   &ik, idx);
        // an index that lowers to a constant no harvest saw: a read of its own (an else value
        // there would let a read at an equal index take another value)
        if (kp || !keys) return acc;
        for (size_t i = keys->size(); i-- > 0;) {
            const Big k = (*keys)[i];
            const uint32_t cell = cell_column(name + "[" + k.hex() + "]", rng, kcell, name, &k);
            const uint32_t kn = konst(k, width(idx));
            acc = add(ITE, rng, eq(idx, kn), cell, acc);
        }
        return acc;
    }
    uint32_t apply(uint32_t n) {  // Lowering._apply
        const mh_node x = nd(n);
        const std::string& f = fn_name(n);
        if (inverse(f)) return low(nd(x.a).a);
        const uint32_t a = low(x.a);
        if (keccak_fn(f)) {
            auto it = kidx.find(f);
            if (it == kidx.end()) unsupported("keccak function " + f + " not harvested");
            const KeccakMap km = keccak[it->second].second;
            if (x.width != 256)
                unsupported("keccak function " + f + " has range " + std::to_string(x.width));
            uint32_t acc;
            if (T.options & MH_TERMS_KECCAK_READS) {  // Lowering._keccak_read: f[@a], free
                Big ik;
                ik.w[0] = x.a;
                const Big* cx = const_value(a);
                if (cx)  // a stated pair's hash, else a read no pair's ite chain can take
                    for (const auto& pr : km.pairs)
                        if (pr.first == *cx) return konst(pr.second, 256);
                acc = cell_column(f + "[@" + std::to_string(x.a) + "]", 256, MH_COL_KREAD, f, &ik, a);
                if (cx) return acc;
            } else {
                Big s1, s2;
                s1.w[0] = KECCAK_SHIFT;
                s2.w[0] = KECCAK_ALIGN;
                uint32_t h = add(KECCAK, 256, a);
                h = add(BVLSHR, 256, h, konst(s1, 256));
                h = add(BVSHL, 256, h, konst(s2, 256));
                acc = km.base.zero() ? h : add(BVADD, 256, h, konst(km.base, 256));
            }
            std::vector<std::pair<Big, Big>> pairs = km.pairs;
            std::sort(pairs.begin(), pairs.end(),
                      [](const std::pair<Big, Big>& p, const std::pair<Big, Big>& q) {
                          return q.first < p.first;
                      });
            for (const auto& pr : pairs) {
                const uint32_t c = eq(a, konst(pr.first, width(a)));
                acc = add(ITE, 256, c, konst(pr.second, 256), acc);
            }
            return acc;
        }
        auto it = uf_of.find(f);
        return table(f, x.width, a, it == uf_of.end() ? nullptr : &uf_cells[it->second].second,
                     MH_COL_UFCELL, MH_COL_UFREAD, x.a);
    }

    // ---- the root tape (sieve.py local_tapeset): VAR imm0 = query column, CONST imm0 = query
    // constant; has_col = the node reads a column ----------------------------------------------
    // continues the tape of an earlier call (a child query's root extends its parent's); equal
    // tape nodes are one (a node the host made after the query made its own copy)
    bool lhas(uint32_t n) const {
        return n & OWN ? (n & ~OWN) < local_own.size() && local_own[n & ~OWN] >= 0 : T.local.has(n);
    }
    uint32_t lget(uint32_t n) const {
        return n & OWN ? (uint32_t)local_own[n & ~OWN] : T.local.get(n);
    }
    void lset(uint32_t n, uint32_t v) {
        local_log.push_back(n);  // undone by rollback (a sibling query takes the tape back)
        if (n & OWN) {
            if (local_own.size() <= (n & ~OWN)) local_own.resize(ov.size(), -1);
            local_own[n & ~OWN] = v;
        } else {
            T.local.set(n, v);
        }
    }
    void linearise(uint32_t root) {
        std::vector<std::pair<uint32_t, bool>> st{{root, false}};
        while (!st.empty()) {
            const auto [n, done] = st.back();
            st.pop_back();
            if (lhas(n)) continue;
            const mh_node& x = nd(n);
            const int k = arity(x.op);
            const uint32_t kids[3] = {x.a, x.b, x.c};
            if (!done) {
                st.push_back({n, true});
                for (int j = k - 1; j >= 0; --j)
                    if (!lhas(kids[j])) st.push_back({kids[j], false});
                continue;
            }
            if (x.op >= ARRAY || (x.flags & F_ARRAY)) invalid("a host-only term survived lowering");
            mh_node y = x;
            y.flags = 0;
            uint8_t hc = 0;
            uint32_t* opnd[3] = {&y.a, &y.b, &y.c};
            for (int j = 0; j < 3; ++j) {
                *opnd[j] = j < k ? lget(kids[j]) : 0;
                if (j < k) hc |= has_col[*opnd[j]];
            }
            if (x.op == VAR) {
                y.imm0 = column_of(n);
                hc = 1;
            } else if (x.op == CONST) {
                y.imm0 = const_index(n);
            }
            auto ins = tape_memo.emplace(key_of(y), (uint32_t)tape.size());
            lset(n, ins.first->second);
            if (!ins.second) continue;
            tape.push_back(y);
            has_col.push_back(hc);
        }
    }
    uint32_t column_of(uint32_t n) {  // a VAR node's query column (numbered by first use)
        const mh_node& x = nd(n);
        const bool cell = (n & OWN) && (x.imm0 & CELL_COL);
        auto& m = cell ? cell_cols : var_cols;
        const uint32_t k = cell ? x.imm0 & ~CELL_COL : x.imm0;
        auto it = m.find(k);
        if (it != m.end()) return it->second;
        const uint32_t q = (uint32_t)cols.size();
        if (cell) {
            cols.push_back(ccols.at(k));
        } else {
            const std::string& name = T.var_names.at(k);
            cols.push_back(Column{name, name, x.width, MH_COL_VAR, false, Big()});
        }
        m.emplace(k, q);
        map_log.push_back({cell ? 1u : 0u, k});
        return q;
    }
    uint32_t const_index(uint32_t n) {
        const uint32_t i0 = nd(n).imm0;
        auto& m = (n & OWN) && (i0 & OV_CONST) ? own_consts : pool_consts;
        auto it = m.find(i0);
        if (it != m.end()) return it->second;
        const uint32_t q = (uint32_t)qpool.size();
        qpool.push_back(const_of(n));
        m.emplace(i0, q);
        map_log.push_back({(n & OWN) && (i0 & OV_CONST) ? 3u : 2u, i0});
        return q;
    }

    // ---- checkpoints of the root tape: a query that is not a child of this one (a JUMPI's
    // other branch, svm.py:257-262; the next state a BFS pops) takes the tape back to the common
    // prefix of their roots and extends it from there.  The lowering overlay is not rolled back:
    // it is a function of the harvest, which is the same at every depth of one state.
    struct Mark {
        size_t tape, cols, qpool, local_log, map_log;
    };
    Mark mark() const {
        return Mark{tape.size(), cols.size(), qpool.size(), local_log.size(), map_log.size()};
    }
    void rollback(const Mark& m) {
        for (size_t i = local_log.size(); i-- > m.local_log;) {
            const uint32_t n = local_log[i];
            if (n & OWN) local_own[n & ~OWN] = -1;
            else T.local.unset(n);
        }
        local_log.resize(m.local_log);
        for (size_t i = map_log.size(); i-- > m.map_log;) {
            const auto& e = map_log[i];
            (e.first == 0 ? var_cols : e.first == 1 ? cell_cols : e.first == 2 ? pool_consts
                                                                                  : own_consts)
                .erase(e.second);
        }
        map_log.resize(m.map_log);
        for (size_t n = m.tape; n < tape.size(); ++n) tape_memo.erase(key_of(tape[n]));
        tape.resize(m.tape);
        has_col.resize(m.tape);
        cols.resize(m.cols);
        qpool.resize(m.qpool);
    }

    mh_terms& T;
    std::vector<mh_node> ov;  // nodes the query made
    std::unordered_map<Key, uint32_t, KeyHash> ov_memo;
    std::vector<Big> ov_vals;  // constants outside the host's pool
    std::unordered_map<Big, uint32_t, BigHash> ov_index;
    std::unordered_map<uint32_t, int64_t> ov_cv;
    std::vector<Big> ov_cv_vals;
    // the harvest (Schema.cells / uf_cells / keccak), in first-seen order
    Tables cells, uf_cells;
    std::unordered_map<std::string, size_t> cell_of, uf_of, kidx;
    std::vector<std::pair<std::string, KeccakMap>> keccak;
    uint64_t hver = 0;          // keccak pairs / bounds changed (harvest_sig)
    std::vector<Column> ccols;  // every cell / else / read column lowering made
    std::vector<uint32_t> read_li;  // per ccol: a read's lowered index term (else UINT32_MAX)
    std::unordered_map<std::string, uint32_t> cell_index;
    // the root tape
    std::vector<mh_node> tape;
    std::vector<uint8_t> has_col;
    std::vector<int64_t> local_own;  // tape index of the query's own nodes, -1 none
    std::unordered_map<Key, uint32_t, KeyHash> tape_memo;
    std::vector<Column> cols;  // query columns, in first-use order
    std::unordered_map<uint32_t, uint32_t> var_cols, cell_cols, pool_consts, own_consts;
    std::vector<Big> qpool;
    // what linearise set since the state began (rollback's undo records): nodes given a tape
    // index (OWN bit for the query's own), and (map, key) of new column / constant entries
    std::vector<uint32_t> local_log;
    std::vector<std::pair<uint32_t, uint32_t>> map_log;
};

}  // namespace

struct mh_query {
    std::vector<mh_node> nodes;
    std::vector<uint64_t> tape_off;
    std::vector<uint32_t> consts;
    std::vector<mh_query_column> columns;
    std::string names;
    std::vector<uint32_t> key_limbs, group_cols, group_off, table_limbs;
    std::vector<mh_query_table> tables;
    std::vector<uint32_t> def_cols;  // the column each definition tape (the last ones) gives
    uint32_t parent_len = 0;         // root tape nodes of the query without its last root
    std::vector<uint32_t> root_ends;  // [d - 1]: root tape nodes of its first d roots
};

namespace {

void put_big(std::vector<uint32_t>& v, const Big& b) { v.insert(v.end(), b.w, b.w + 8); }
void put_key(std::vector<uint32_t>& v, const Big& b) { v.insert(v.end(), b.w, b.w + NL); }
uint32_t put_name(std::string& s, const std::string& n) {
    const uint32_t off = (uint32_t)s.size();
    s += n;
    return off;
}

// sieve.py _may_define, narrowed to what eliminate_definitions can use: a plain variable on one
// side, a computed term that reads columns on the other
bool may_define(const std::vector<mh_node>& tape, const std::vector<uint8_t>& has_col,
                const std::vector<Column>& cols, uint32_t cj) {
    const mh_node& x = tape[cj];
    if (x.op != EQ) return false;
    const uint32_t s[2][2] = {{x.a, x.b}, {x.b, x.a}};
    for (const auto& p : s) {
        const mh_node& v = tape[p[0]];
        const uint8_t t = tape[p[1]].op;
        if (v.op == VAR && cols[v.imm0].kind == MH_COL_VAR && t != VAR && t != CONST && has_col[p[1]])
            return true;
    }
    return false;
}

struct Cmp {
    uint8_t op;
    uint32_t t, c;  // tape nodes: the term, the constant
};

// t op c for a comparison node of a bit-vector term t with a constant c (either side; a constant on
// the left mirrors the comparison)
bool cmp_of_plain(const std::vector<mh_node>& tape, uint32_t n, Cmp& out) {
    const mh_node& x = tape[n];
    uint8_t op = x.op;
    if (op != EQ && !(op >= BVULT && op <= MH_OP_BVUGE)) return false;
    const bool ca = tape[x.a].op == CONST, cb = tape[x.b].op == CONST;
    if (ca == cb || tape[x.a].width == 0) return false;
    if (ca)
        op = op == BVULT ? MH_OP_BVUGT : op == MH_OP_BVULE ? MH_OP_BVUGE
           : op == MH_OP_BVUGT ? BVULT : op == MH_OP_BVUGE ? MH_OP_BVULE : op;
    out = {op, ca ? x.b : x.a, ca ? x.a : x.b};
    return true;
}

// A conjunction that contradicts itself syntactically (sound, not complete): a FALSE conjunct, a
// conjunct and its negation, or one term pinned by its conjuncts -- t == c, t != c, unsigned
// comparisons of t with constants and their negations -- to an empty range.  Over the lowered
// root tape, whose nodes are hash-consed (equal terms are one node).  Such a query cannot have a
// witness: the device rounds are skipped (the query still goes to the fallback solver).
// Scratch of refuted(), kept per thread across queries: per tape node an epoch stamp for "asserted"
// and one for "has a range" (with the range's index), so a query costs its conjuncts, not a hash
// map built afresh (a 400-constraint path's refutation was ~45 % of its query build).
struct RefuteScratch {
    struct Range {
        Big lo, hi;
        std::vector<uint32_t> ne;  // constants t must differ from
    };
    uint32_t epoch = 0;
    std::vector<uint32_t> asserted, has_range, range_of;
    std::vector<Range> ranges;
    std::vector<uint32_t> range_terms;
    void begin(size_t n) {
        if (++epoch == 0) {  // wrapped: every stamp is stale again
            std::fill(asserted.begin(), asserted.end(), 0);
            std::fill(has_range.begin(), has_range.end(), 0);
            epoch = 1;
        }
        if (asserted.size() < n) {
            asserted.resize(n, 0);
            has_range.resize(n, 0);
            range_of.resize(n, 0);
        }
        ranges.clear();
        range_terms.clear();
    }
};

// 2^w - 1 (w bits set, at most the 32 NL a Big holds)
Big ones(uint32_t w) {
    Big r;
    const uint32_t n = std::min<uint32_t>(w, 32u * NL);
    for (uint32_t i = 0; i < n / 32; ++i) r.w[i] = ~0u;
    if (n % 32) r.w[n / 32] = (1u << (n % 32)) - 1u;
    return r;
}

bool refuted(const Query& Q, const std::vector<uint32_t>& conj) {
    const std::vector<mh_node>& tape = Q.tape;
    thread_local RefuteScratch S;
    S.begin(tape.size());
    const uint32_t ep = S.epoch;
    for (uint32_t cj : conj) S.asserted[cj] = ep;
    auto range = [&](uint32_t t) -> RefuteScratch::Range& {
        if (S.has_range[t] != ep) {
            S.has_range[t] = ep;
            S.range_of[t] = (uint32_t)S.ranges.size();
            S.range_terms.push_back(t);
            S.ranges.emplace_back();
            S.ranges.back().hi = ones(tape[t].width);
        }
        return S.ranges[S.range_of[t]];
    };
    // smt.py's ULE / UGE (bitvec_helper.py: Or(ULT(a, b), a == b)) read as BVULE / BVUGE
    auto cmp_of = [&](uint32_t n, Cmp& out) -> bool {
        const mh_node& x = tape[n];
        if (x.op == MH_OP_OR) {
            Cmp p, e;
            if (!cmp_of_plain(tape, x.a, p) || !cmp_of_plain(tape, x.b, e)) return false;
            if (p.op == EQ) std::swap(p, e);
            if (e.op != EQ || p.t != e.t || p.c != e.c) return false;
            if (p.op != BVULT && p.op != MH_OP_BVUGT) return false;
            out = {(uint8_t)(p.op == BVULT ? MH_OP_BVULE : MH_OP_BVUGE), p.t, p.c};
            return true;
        }
        return cmp_of_plain(tape, n, out);
    };
    for (uint32_t cj : conj) {
        const mh_node& x0 = tape[cj];
        if (x0.op == FALSE_) return true;
        bool neg = false;
        uint32_t n = cj;
        if (x0.op == MH_OP_NOT) {
            if (S.asserted[x0.a] == ep) return true;
            neg = true;
            n = x0.a;
        }
        Cmp k;
        if (!cmp_of(n, k)) continue;
        uint8_t op = k.op;
        const uint32_t t = k.t;
        const Big* c = &Q.qpool[tape[k.c].imm0];
        if (neg)  // not (t < c) is t >= c, ...; not (t == c) is t != c
            op = op == BVULT ? MH_OP_BVUGE : op == MH_OP_BVULE ? MH_OP_BVUGT
               : op == MH_OP_BVUGT ? MH_OP_BVULE : op == MH_OP_BVUGE ? BVULT : op;
        RefuteScratch::Range& r = range(t);
        if (op == EQ && neg) {
            r.ne.push_back(k.c);
            continue;
        }
        if (op == EQ || op == MH_OP_BVULE || op == BVULT) {  // an upper bound
            if (op == BVULT && c->zero()) return true;
            const Big h = op == BVULT ? c->minus_one() : *c;
            if (h < r.hi) r.hi = h;
        }
        if (op == EQ || op == MH_OP_BVUGE || op == MH_OP_BVUGT) {  // a lower bound
            Big l = *c;
            if (op == MH_OP_BVUGT) {
                if (!(*c < r.hi) && !(r.hi < *c)) return true;  // t > max of the range so far
                l = c->plus(1);
            }
            if (r.lo < l) r.lo = l;
        }
        if (r.hi < r.lo) return true;
    }
    for (const RefuteScratch::Range& r : S.ranges) {  // a range pinned to one value that a
        if (r.lo == r.hi)                             // disequality excludes
            for (uint32_t ne : r.ne)
                if (Q.qpool[tape[ne].imm0] == r.lo) return true;
    }
    // second pass: comparisons of two terms and the no-overflow predicates
    // (bitvec_helper.py:178-227) decided by the terms' ranges
    auto bounds = [&](uint32_t t, Big& lo, Big& hi) {
        if (tape[t].op == CONST) {
            lo = hi = Q.qpool[tape[t].imm0];
            return;
        }
        if (S.has_range[t] == ep) {
            lo = S.ranges[S.range_of[t]].lo;
            hi = S.ranges[S.range_of[t]].hi;
            return;
        }
        lo = Big();
        hi = ones(tape[t].width);
    };
    auto le = [](const Big& a, const Big& b) { return !(b < a); };
    // 1 = true under every value in the ranges, 0 = false under every one, -1 = either
    auto decide = [&](auto& self, uint32_t n, int depth) -> int {
        const mh_node& x = tape[n];
        if (depth > 8) return -1;
        switch (x.op) {
            case TRUE_: return 1;
            case FALSE_: return 0;
            case MH_OP_NOT: {
                const int v = self(self, x.a, depth + 1);
                return v < 0 ? -1 : 1 - v;
            }
            case MH_OP_OR: case AND: {
                const int a = self(self, x.a, depth + 1), b = self(self, x.b, depth + 1);
                if (x.op == MH_OP_OR) return a == 1 || b == 1 ? 1 : (a == 0 && b == 0 ? 0 : -1);
                return a == 0 || b == 0 ? 0 : (a == 1 && b == 1 ? 1 : -1);
            }
            default: break;
        }
        const bool cmp = x.op == EQ || (x.op >= BVULT && x.op <= MH_OP_BVUGE);
        const bool pred = x.op == MH_OP_BVADD_NOOVFL_U || x.op == MH_OP_BVMUL_NOOVFL_U ||
                          x.op == MH_OP_BVSUB_NOUDFL_U;
        if ((!cmp && !pred) || tape[x.a].width == 0) return -1;
        Big la, ha, lb, hb;
        bounds(x.a, la, ha);
        bounds(x.b, lb, hb);
        Big top;  // 2^width
        const uint32_t w = tape[x.a].width;
        top.w[w / 32] |= 1u << (w % 32);
        switch (x.op) {
            case EQ: return hb < la || ha < lb ? 0 : (la == ha && lb == hb && la == lb ? 1 : -1);
            case BVULT: return ha < lb ? 1 : (le(hb, la) ? 0 : -1);
            case MH_OP_BVULE: return le(ha, lb) ? 1 : (hb < la ? 0 : -1);
            case MH_OP_BVUGT: return hb < la ? 1 : (le(ha, lb) ? 0 : -1);
            case MH_OP_BVUGE: return le(hb, la) ? 1 : (ha < lb ? 0 : -1);
            case MH_OP_BVADD_NOOVFL_U: return (ha + hb) < top ? 1 : (le(top, la + lb) ? 0 : -1);
            case MH_OP_BVMUL_NOOVFL_U:
                if (w > 512) return -1;
                return ha.times(hb) < top ? 1 : (le(top, la.times(lb)) ? 0 : -1);
            case MH_OP_BVSUB_NOUDFL_U: return le(hb, la) ? 1 : (ha < lb ? 0 : -1);
            default: return -1;
        }
    };
    for (uint32_t cj : conj)
        if (decide(decide, cj, 0) == 0) return true;
    return false;
}

// the AND leaves of tape node n, left to right (Sieve.conjuncts)
void and_leaves(const std::vector<mh_node>& tape, uint32_t n, std::vector<uint32_t>& out) {
    std::vector<uint32_t> st{n};
    while (!st.empty()) {
        const uint32_t x = st.back();
        st.pop_back();
        if (tape[x].op == AND) {
            st.push_back(tape[x].b);
            st.push_back(tape[x].a);
        } else {
            out.push_back(x);
        }
    }
}


// The query's tapes: the root's (tape 0), then with several groups each group's AND chain over
// the root tape's nodes (sieve.py local_tapeset(b, [root] + accs, columns))
void emit_tapes(mh_query& q, const std::vector<mh_node>& tape,
                const std::vector<std::vector<uint32_t>>& gconj) {
    const uint32_t N = (uint32_t)tape.size();
    const uint32_t G = (uint32_t)gconj.size();
    q.nodes = tape;
    q.tape_off = {0, N};
    if (G <= 1) return;
    std::vector<int32_t> remap(N, -1);
    std::vector<uint32_t> touched;
    std::vector<std::pair<uint32_t, bool>> s2;
    for (uint32_t g = 0; g < G; ++g) {
        const size_t base = q.nodes.size();
        for (uint32_t n : touched) remap[n] = -1;
        touched.clear();
        int64_t acc = -1;
        for (uint32_t cj : gconj[g]) {
            s2.assign(1, {cj, false});
            while (!s2.empty()) {
                const auto [n, done] = s2.back();
                s2.pop_back();
                if (remap[n] >= 0) continue;
                const mh_node& x = tape[n];
                const int k = arity(x.op);
                const uint32_t kids[3] = {x.a, x.b, x.c};
                if (!done) {
                    s2.push_back({n, true});
                    for (int j = k - 1; j >= 0; --j)
                        if (remap[kids[j]] < 0) s2.push_back({kids[j], false});
                    continue;
                }
                mh_node y = x;
                y.a = k > 0 ? (uint32_t)remap[x.a] : 0;
                y.b = k > 1 ? (uint32_t)remap[x.b] : 0;
                y.c = k > 2 ? (uint32_t)remap[x.c] : 0;
                remap[n] = (int32_t)(q.nodes.size() - base);
                touched.push_back(n);
                q.nodes.push_back(y);
            }
            if (acc < 0) {
                acc = remap[cj];
                continue;
            }
            mh_node a{};
            a.op = AND;
            a.a = (uint32_t)acc;
            a.b = (uint32_t)remap[cj];
            acc = (int64_t)(q.nodes.size() - base);
            q.nodes.push_back(a);
        }
        if ((size_t)acc != q.nodes.size() - base - 1) invalid("group tape root is not its last node");
        q.tape_off.push_back(q.nodes.size());
    }
}

void put_groups(mh_query& q, std::vector<std::vector<uint32_t>>& gcols) {
    q.group_off.assign(1, 0);
    for (auto& gc : gcols) {
        std::sort(gc.begin(), gc.end());
        gc.erase(std::unique(gc.begin(), gc.end()), gc.end());
        q.group_cols.insert(q.group_cols.end(), gc.begin(), gc.end());
        q.group_off.push_back((uint32_t)q.group_cols.size());
    }
}

// Column-disjoint groups of `conj` on a tape (the DependenceMap; QueryState keeps the same
// union-find incrementally): conjuncts reaching a common column-reading node are one group,
// groups in order of their first conjunct, a ground conjunct its own group per node
void group_conjuncts(const std::vector<mh_node>& tape, const std::vector<uint8_t>& hc,
                     const std::vector<uint32_t>& conj,
                     std::vector<std::vector<uint32_t>>& gconj,
                     std::vector<std::vector<uint32_t>>& gcols) {
    std::vector<int32_t> owner(tape.size(), -1);
    std::vector<uint32_t> uf(conj.size());
    auto find = [&](uint32_t x) {
        while (uf[x] != x) x = uf[x] = uf[uf[x]];
        return x;
    };
    std::vector<uint32_t> st;
    for (uint32_t i = 0; i < conj.size(); ++i) {
        uf[i] = i;
        st.assign(1, conj[i]);
        while (!st.empty()) {
            const uint32_t n = st.back();
            st.pop_back();
            if (!hc[n]) continue;
            if (owner[n] >= 0) {
                const uint32_t a = find(i), b = find((uint32_t)owner[n]);
                uf[std::max(a, b)] = std::min(a, b);
                continue;
            }
            owner[n] = (int32_t)i;
            const mh_node& x = tape[n];
            const uint32_t kids[3] = {x.a, x.b, x.c};
            for (int j = 0; j < arity(x.op); ++j) st.push_back(kids[j]);
        }
    }
    std::unordered_map<int64_t, uint32_t> gid;
    std::vector<uint32_t> group_of(conj.size(), UINT32_MAX);
    for (uint32_t i = 0; i < conj.size(); ++i) {
        const int64_t key = hc[conj[i]] ? (int64_t)find(i) : -(int64_t)conj[i] - 1;
        auto it = gid.find(key);
        if (it == gid.end()) {
            it = gid.emplace(key, (uint32_t)gconj.size()).first;
            gconj.emplace_back();
        }
        gconj[it->second].push_back(conj[i]);
        if (key >= 0) group_of[(size_t)key] = it->second;
    }
    gcols.assign(gconj.size(), {});
    for (uint32_t n = 0; n < tape.size(); ++n)
        if (tape[n].op == VAR && owner[n] >= 0)
            gcols[group_of[find((uint32_t)owner[n])]].push_back(tape[n].imm0);
}

// sieve.py eliminate_definitions over a copy of the root tape (the session's tape stays the
// linearisation a LASER child extends): nodes hash-consed as in the tape, VAR imm0 = column
struct DefTape {
    std::vector<mh_node> t;
    std::vector<uint8_t> hc;
    std::unordered_map<Key, uint32_t, KeyHash> memo;

    uint32_t add(mh_node y) {
        y.flags = 0;
        auto ins = memo.emplace(key_of(y), (uint32_t)t.size());
        if (!ins.second) return ins.first->second;
        uint8_t h = y.op == VAR;
        const uint32_t kids[3] = {y.a, y.b, y.c};
        for (int j = 0; j < arity(y.op); ++j) h |= hc[kids[j]];
        t.push_back(y);
        hc.push_back(h);
        return ins.first->second;
    }
    // sieve.py substitute: `root` with every VAR of a column in env replaced by env's term
    uint32_t subst(uint32_t root, const std::unordered_map<uint32_t, uint32_t>& env) {
        std::unordered_map<uint32_t, uint32_t> out;
        std::vector<uint32_t> st{root};
        while (!st.empty()) {
            const uint32_t n = st.back();
            if (out.count(n)) {
                st.pop_back();
                continue;
            }
            const mh_node x = t[n];
            if (x.op == VAR) {
                auto e = env.find(x.imm0);
                out[n] = e == env.end() ? n : e->second;
                st.pop_back();
                continue;
            }
            if (!hc[n]) {  // reads no column: itself
                out[n] = n;
                st.pop_back();
                continue;
            }
            const int k = arity(x.op);
            const uint32_t kids[3] = {x.a, x.b, x.c};
            bool todo = false;
            for (int j = 0; j < k; ++j)
                if (!out.count(kids[j])) {
                    st.push_back(kids[j]);
                    todo = true;
                }
            if (todo) continue;
            st.pop_back();
            mh_node y = x;
            uint32_t* o[3] = {&y.a, &y.b, &y.c};
            bool same = true;
            for (int j = 0; j < k; ++j) {
                *o[j] = out[kids[j]];
                same = same && *o[j] == kids[j];
            }
            out[n] = same ? n : add(y);
        }
        return out[root];
    }
    // the columns a term reads (lower.node_columns)
    void reads(uint32_t root, std::vector<uint32_t>& cols) const {
        std::vector<uint32_t> st{root};
        std::unordered_map<uint32_t, bool> seen;
        cols.clear();
        while (!st.empty()) {
            const uint32_t n = st.back();
            st.pop_back();
            if (!hc[n] || !seen.emplace(n, true).second) continue;
            const mh_node& x = t[n];
            if (x.op == VAR) {
                cols.push_back(x.imm0);
                continue;
            }
            const uint32_t kids[3] = {x.a, x.b, x.c};
            for (int j = 0; j < arity(x.op); ++j) st.push_back(kids[j]);
        }
    }
    // the nodes below `root` in post order (operands first, a before b before c), as
    // TapeBuilder.finish / local_tapeset number them
    void linearise(uint32_t root, std::vector<mh_node>& out, std::vector<uint8_t>* ohc) const {
        std::unordered_map<uint32_t, uint32_t> at;
        std::vector<std::pair<uint32_t, bool>> st{{root, false}};
        while (!st.empty()) {
            const auto [n, done] = st.back();
            st.pop_back();
            if (at.count(n)) continue;
            const mh_node& x = t[n];
            const int k = arity(x.op);
            const uint32_t kids[3] = {x.a, x.b, x.c};
            if (!done) {
                st.push_back({n, true});
                for (int j = k - 1; j >= 0; --j)
                    if (!at.count(kids[j])) st.push_back({kids[j], false});
                continue;
            }
            mh_node y = x;
            uint32_t* o[3] = {&y.a, &y.b, &y.c};
            for (int j = 0; j < 3; ++j) *o[j] = j < k ? at.at(kids[j]) : 0;
            at.emplace(n, (uint32_t)out.size());
            out.push_back(y);
            if (ohc) ohc->push_back(hc[n]);
        }
    }
};

// Harvest tables compared before and after a new constraint (lower.py Harvest.fingerprint)
struct Fingerprint {
    Tables cells, uf_cells;
    std::vector<std::pair<std::string, std::pair<Big, std::vector<std::pair<Big, Big>>>>> keccak;
    explicit Fingerprint(const Query& Q) : cells(Q.cells), uf_cells(Q.uf_cells) {
        for (const auto& kv : Q.keccak) keccak.push_back({kv.first, {kv.second.base, kv.second.pairs}});
    }
    bool same(const Query& Q) const {
        if (cells != Q.cells || uf_cells != Q.uf_cells || keccak.size() != Q.keccak.size()) return false;
        for (size_t i = 0; i < keccak.size(); ++i)
            if (keccak[i].first != Q.keccak[i].first || !(keccak[i].second.first == Q.keccak[i].second.base) ||
                keccak[i].second.second != Q.keccak[i].second.pairs)
                return false;
        return true;
    }
};

}  // namespace

// One query's state, kept on the session (mh_terms.last): a child query whose roots are its
// parent's plus one constraint (svm.py:257-262) extends it when the new constraint adds nothing to
// the harvest -- only that constraint is harvested, lowered, linearised and grouped (lower.py
// _lower_extend / sieve.py _bucket_state do the same in Python); otherwise the query is built
// afresh.  Either way the result equals the from-scratch one (tests/test_query_native.py).
class QueryState {
public:
    explicit QueryState(mh_terms& t, bool keep_lowering = false) : Q(t, keep_lowering) {}

    // A fresh state for the query `rs` (n roots).  warm: the last query's state, whose lowering
    // this one takes over when their harvests are equal (the same path with another condition:
    // only what is new is lowered afresh, the rest are memo hits).
    void start(const uint32_t* rs, uint32_t n, QueryState* warm = nullptr) {
        // the harvest root by root (the same tables as over all roots at once), a copy of the
        // tables kept at every depth where they grew (rollback restores the prefix's harvest)
        marks.clear();
        snaps.clear();
        snaps.push_back({0, Q.save_harvest()});
        harvest_roots(rs, 0, n);
        if (warm && Q.same_harvest(warm->Q)) Q.adopt_lowering(warm->Q);
        else if (warm) Q.reset_lowering();
        roots.clear();
        if (!n) {
            root = Q.add(TRUE_, 0);
            Q.linearise(root);
            add_conjuncts(Q.lget(root));
            return;
        }
        lower_roots(rs, 0, n);
    }

    // The query `rs` (n roots) from this state: taken back to depth d (the length of the common
    // prefix of their roots), the harvest of the prefix extended by the rest -- which must end
    // where this state's harvest is, or the lowering memo would not hold (false: build afresh,
    // the state is spent) -- then the rest lowered, linearised and grouped root by root.  A
    // child of the last query is d = all its roots, a JUMPI's other branch d = all but one
    // (svm.py:257-262), the next state a BFS pops d = where their paths parted (cli.py:417-419).
    bool advance(const uint32_t* rs, uint32_t n, size_t d) {
        Q.sync();
        const Fingerprint before(Q);
        rollback(d);
        harvest_roots(rs, d, n);
        if (!before.same(Q)) return false;
        lower_roots(rs, d, n);
        return true;
    }

    void emit(mh_query& q, uint32_t& flags);

    Query Q;
    std::vector<uint32_t> roots;

private:
    void harvest_roots(const uint32_t* rs, size_t from, size_t to) {
        std::array<uint64_t, 4> sig = Q.harvest_sig();
        for (size_t i = from; i < to; ++i) {
            Q.harvest({rs[i]});
            const std::array<uint64_t, 4> s2 = Q.harvest_sig();
            if (s2 != sig) snaps.push_back({i + 1, Q.save_harvest()});
            sig = s2;
        }
    }
    void lower_roots(const uint32_t* rs, size_t from, size_t to) {
        // lower_query: the AND of the lowered roots, linearised root by root (the tape of
        // AND(x, y) is x's followed by y's new nodes), a checkpoint before every root
        for (size_t i = from; i < to; ++i) {
            marks.push_back(Mark{Q.mark(), root, defines, conj.size(), uf_log.size(),
                                 owner_log.size(), qreads.size()});
            const uint32_t x = lowered(rs[i]);
            roots.push_back(rs[i]);
            root = i == 0 ? x : Q.add(AND, 0, root, x);
            Q.linearise(root);
            add_conjuncts(Q.lget(x));
            congruence(x);
        }
    }
    // lower.py congruence: the read columns x reads first in this query (directly or in a read's
    // index term), by (symbol, index term), each paired with every earlier read of its symbol:
    // Or(Not(i == j), A[@i] == A[@j]) ANDed on as a conjunct of its own
    void congruence(uint32_t x) {
        std::vector<uint32_t> found, st{x};
        std::unordered_set<uint32_t> vis, fs;
        while (!st.empty()) {
            const uint32_t n = st.back();
            st.pop_back();
            if (!vis.insert(n).second) continue;
            const mh_node& v = Q.nd(n);
            if (v.op == VAR && (n & OWN) && (v.imm0 & CELL_COL)) {
                const uint32_t k = v.imm0 & ~CELL_COL;
                if (Query::read_kind(Q.ccols.at(k).kind) && fs.insert(k).second) {
                    found.push_back(k);
                    st.push_back(Q.read_li.at(k));
                }
                continue;
            }
            const uint32_t kids[3] = {v.a, v.b, v.c};
            for (int j = 0; j < arity(v.op); ++j) st.push_back(kids[j]);
        }
        std::vector<uint32_t> fresh;
        for (uint32_t k : found)
            if (!qseen.count(k)) fresh.push_back(k);
        std::sort(fresh.begin(), fresh.end(), [&](uint32_t a, uint32_t b) {
            const Column& ca = Q.ccols[a];
            const Column& cb = Q.ccols[b];
            if (ca.symbol != cb.symbol) return ca.symbol < cb.symbol;
            return ca.key < cb.key;
        });
        for (uint32_t p : fresh) {
            const Column& cp = Q.ccols[p];
            for (size_t qi = 0; qi < qreads.size(); ++qi) {
                const uint32_t q = qreads[qi];
                const Column& cq = Q.ccols[q];
                if (cq.symbol != cp.symbol || cq.kind != cp.kind) continue;
                const uint32_t vq = Q.add(VAR, cq.width, 0, 0, 0, CELL_COL | q);
                const uint32_t vp = Q.add(VAR, cp.width, 0, 0, 0, CELL_COL | p);
                const uint32_t eqv = Q.add(EQ, 0, vq, vp);
                const Big* cq_ = Q.const_value(Q.read_li[q]);
                const Big* cp_ = Q.const_value(Q.read_li[p]);
                if (cp.kind == MH_COL_KREAD && cq_ && cp_) {  // both at constant arguments
                    conjoin(*cq_ == *cp_ ? eqv : Q.add(MH_OP_NOT, 0, eqv));
                    continue;
                }
                const uint32_t same = Q.eq(Q.read_li[q], Q.read_li[p]);
                conjoin(Q.add(MH_OP_OR, 0, Q.add(MH_OP_NOT, 0, same), eqv));
                if (cp.kind == MH_COL_KREAD)  // injective too: Or(i == j, Not(f_i == f_j))
                    conjoin(Q.add(MH_OP_OR, 0, same, Q.add(MH_OP_NOT, 0, eqv)));
            }
            if (cp.kind == MH_COL_KREAD) {  // apart from the stated pairs (the inverse reads them)
                const uint32_t li = Q.read_li[p];
                const uint32_t vp = Q.add(VAR, cp.width, 0, 0, 0, CELL_COL | p);
                std::vector<std::pair<Big, Big>> pairs = Q.keccak.at(Q.kidx.at(cp.symbol)).second.pairs;
                std::sort(pairs.begin(), pairs.end(),
                          [](const std::pair<Big, Big>& u, const std::pair<Big, Big>& v) {
                              return u.first < v.first;
                          });
                const bool lc = Q.const_value(li) != nullptr;  // no pair's argument
                for (const auto& pr : pairs) {
                    const uint32_t ne = Q.add(MH_OP_NOT, 0, Q.add(EQ, 0, vp, Q.konst(pr.second, 256)));
                    conjoin(lc ? ne : Q.add(MH_OP_OR, 0, Q.eq(li, Q.konst(pr.first, Q.width(li))), ne));
                }
            }
            qreads.push_back(p);
            qseen.insert(p);
        }
    }
    void conjoin(uint32_t y) {  // one more conjunct of its own
        root = Q.add(AND, 0, root, y);
        Q.linearise(root);
        add_conjuncts(Q.lget(y));
    }
    // Back to depth d <= roots.size(): every root since undone (tape, columns, constants,
    // conjuncts, union-find, owners; the harvest as it was after the first d roots).  The
    // lowering overlay and memo stay: they hold for any query with this harvest.
    void rollback(size_t d) {
        if (d >= roots.size()) return;
        const Mark m = marks.at(d);
        for (size_t i = uf_log.size(); i-- > m.uf_log;) uf[uf_log[i].first] = uf_log[i].second;
        uf_log.resize(m.uf_log);
        for (size_t i = owner_log.size(); i-- > m.owner_log;)
            owner[owner_log[i].first] = owner_log[i].second;
        owner_log.resize(m.owner_log);
        conj.resize(m.conj);
        uf.resize(m.conj);
        while (qreads.size() > m.qreads) {
            qseen.erase(qreads.back());
            qreads.pop_back();
        }
        Q.rollback(m.q);
        owner.resize(Q.tape.size(), -1);
        root = m.root;
        defines = m.defines;
        roots.resize(d);
        marks.resize(d);
        while (snaps.size() > 1 && snaps.back().first > d) snaps.pop_back();
        Q.restore_harvest(snaps.back().second);
    }
    uint32_t lowered(uint32_t r) {
        const uint32_t x = Q.lower(r);
        if (Q.width(x) != 0 || (Q.nd(x).flags & F_ARRAY)) invalid("constraints must be Bool");
        return x;
    }
    // new conjuncts: definitions flag, column-disjoint groups by a union-find over the conjuncts
    // that reach a common node reading columns
    void add_conjuncts(uint32_t tape_node) {
        const size_t first = conj.size();
        and_leaves(Q.tape, tape_node, conj);
        owner.resize(Q.tape.size(), -1);
        std::vector<uint32_t> st;
        for (size_t i = first; i < conj.size(); ++i) {
            uf.push_back((uint32_t)i);
            defines = defines || may_define(Q.tape, Q.has_col, Q.cols, conj[i]);
            st.assign(1, conj[i]);
            while (!st.empty()) {
                const uint32_t n = st.back();
                st.pop_back();
                if (!Q.has_col[n]) continue;
                if (owner[n] >= 0) {
                    const uint32_t a = find((uint32_t)i), b = find((uint32_t)owner[n]);
                    set_uf(std::max(a, b), std::min(a, b));  // the earlier conjunct stays the root
                    continue;
                }
                owner_log.push_back({n, owner[n]});
                owner[n] = (int32_t)i;
                const mh_node& x = Q.tape[n];
                const uint32_t kids[3] = {x.a, x.b, x.c};
                for (int j = 0; j < arity(x.op); ++j) st.push_back(kids[j]);
            }
        }
    }
    uint32_t find(uint32_t x) {
        while (uf[x] != x) {
            set_uf(x, uf[uf[x]]);
            x = uf[x];
        }
        return x;
    }
    void set_uf(uint32_t i, uint32_t v) {  // every write logged: rollback restores them
        if (uf[i] == v) return;
        uf_log.push_back({i, uf[i]});
        uf[i] = v;
    }
    bool emit_definitions(mh_query& q);

    uint32_t root = 0;            // node id of the lowered conjunction
    std::vector<uint32_t> conj;   // its AND leaves (tape nodes), in order
    std::vector<int32_t> owner;   // per tape node: the first conjunct reaching it
    std::vector<uint32_t> uf;     // union-find over conj
    bool defines = false;
    // checkpoints: marks[k] is the state at depth k (before root k); snaps the harvest tables
    // after the first `first` roots, at 0 and at every depth where they grew
    struct Mark {
        Query::Mark q;
        uint32_t root;
        bool defines;
        size_t conj, uf_log, owner_log, qreads;
    };
    std::vector<Mark> marks;
    std::vector<uint32_t> qreads;        // read columns (ccol) in the order the query met them
    std::unordered_set<uint32_t> qseen;
    std::vector<std::pair<size_t, Query::HarvestCopy>> snaps;
    std::vector<std::pair<uint32_t, uint32_t>> uf_log;   // (index, previous value)
    std::vector<std::pair<uint32_t, int32_t>> owner_log;  // (tape node, previous owner)
};

void QueryState::emit(mh_query& q, uint32_t& flags) {
    const std::vector<mh_node>& tape = Q.tape;
    const uint32_t N = (uint32_t)tape.size();
    if (Q.lget(root) != N - 1) unsupported("the query's root is not the last node of its tape");
    {
        // a variable named like a cell of this query would make two columns one (the cell
        // columns the lowering made for other queries of the state do not count)
        std::unordered_set<std::string> cells;
        for (const Column& c : Q.cols)
            if (c.kind != MH_COL_VAR) cells.insert(c.name);
        if (!cells.empty())
            for (const Column& c : Q.cols)
                if (c.kind == MH_COL_VAR && cells.count(c.name))
                    unsupported("variable " + c.name + " is named like an array cell");
    }
    if (refuted(Q, conj)) flags |= MH_QUERY_REFUTED;
    if (defines && emit_definitions(q)) {
        flags |= MH_QUERY_DEFINITIONS;
    } else {
        // the root tape lists the query without its last root first (linearised root by root)
        for (size_t d = 1; d < roots.size(); ++d) q.root_ends.push_back(Q.lget(marks[d].root) + 1);
        if (roots.size() >= 2) q.parent_len = q.root_ends.back();
        std::vector<std::vector<uint32_t>> gconj;  // conjunct tape nodes per group, path order
        std::unordered_map<int64_t, uint32_t> gid;
        std::vector<uint32_t> group_of(conj.size(), UINT32_MAX);  // by union-find root
        for (uint32_t i = 0; i < conj.size(); ++i) {
            const int64_t key = Q.has_col[conj[i]] ? (int64_t)find(i) : -(int64_t)conj[i] - 1;
            auto it = gid.find(key);
            if (it == gid.end()) {
                it = gid.emplace(key, (uint32_t)gconj.size()).first;
                gconj.emplace_back();
            }
            gconj[it->second].push_back(conj[i]);
            if (key >= 0) group_of[(size_t)key] = it->second;
        }
        std::vector<std::vector<uint32_t>> gcols(gconj.size());
        for (uint32_t n = 0; n < N; ++n)
            if (tape[n].op == VAR && owner[n] >= 0)
                gcols[group_of[find((uint32_t)owner[n])]].push_back(tape[n].imm0);
        emit_tapes(q, tape, gconj);
        put_groups(q, gcols);
    }
    for (const Big& v : Q.qpool) put_big(q.consts, v);
    if (Q.qpool.empty()) put_big(q.consts, Big());
    // columns; a ground query reads one Bool column (Sieve.solve's "__ground__")
    std::vector<Column> cols = Q.cols;
    if (cols.empty()) cols.push_back(Column{"__ground__", "__ground__", 1, MH_COL_VAR, false, Big()});
    for (const Column& c : cols) {
        mh_query_column mc{};
        mc.name_off = put_name(q.names, c.name);
        mc.name_len = (uint32_t)c.name.size();
        mc.symbol_off = put_name(q.names, c.symbol);
        mc.symbol_len = (uint32_t)c.symbol.size();
        mc.width = c.width;
        mc.kind = c.kind;
        mc.key_off = c.has_key ? (uint32_t)(q.key_limbs.size() / NL) : UINT32_MAX;
        if (c.has_key) put_key(q.key_limbs, c.key);
        q.columns.push_back(mc);
    }
    // the schema's tables: every harvested key (read or not), keccak bases and pairs
    for (int t = 0; t < 2; ++t)
        for (const auto& kv : t == 0 ? Q.cells : Q.uf_cells) {
            mh_query_table tb{};
            tb.kind = t == 0 ? MH_TABLE_CELLS : MH_TABLE_UF_CELLS;
            tb.name_off = put_name(q.names, kv.first);
            tb.name_len = (uint32_t)kv.first.size();
            tb.limb_off = (uint32_t)(q.table_limbs.size() / NL);
            tb.n_items = (uint32_t)kv.second.size();
            for (const Big& k : kv.second) put_key(q.table_limbs, k);
            q.tables.push_back(tb);
        }
    for (const auto& kv : Q.keccak) {
        mh_query_table tb{};
        tb.kind = MH_TABLE_KECCAK;
        tb.name_off = put_name(q.names, kv.first);
        tb.name_len = (uint32_t)kv.first.size();
        tb.limb_off = (uint32_t)(q.table_limbs.size() / NL);
        tb.n_items = (uint32_t)kv.second.pairs.size();
        put_key(q.table_limbs, kv.second.base);  // then (argument, hash) pairs
        for (const auto& pr : kv.second.pairs) {
            put_key(q.table_limbs, pr.first);
            put_key(q.table_limbs, pr.second);
        }
        q.tables.push_back(tb);
    }
}

// sieve.py solve_definitions / eliminate_definitions, natively: a conjunct
// `v == t` with a plain variable v on one side and a computed term t over other columns on the
// other (not a constant, not a symbol: the guide proposes those) defines v; it is dropped and v
// replaced by t in every other conjunct, definitions kept closed (every defining term reads
// undefined columns only).  The remaining conjunction is the query's root, grouped afresh; one
// tape per definition follows the group tapes, whose value under the witness row is v's.
// Equisatisfiable: a row satisfying the rest extends to a model with v = t(row).  false: no
// conjunct defines anything (the query is emitted as it is).
bool QueryState::emit_definitions(mh_query& q) {
    DefTape D{Q.tape, Q.has_col, Q.tape_memo};
    std::unordered_map<uint32_t, uint32_t> env;  // column -> defining term
    std::vector<uint32_t> def_cols, rest, rd;
    for (uint32_t cn : conj) {
        const mh_node x = D.t[cn];
        bool done = false;
        if (x.op == EQ) {
            const uint32_t sides[2][2] = {{x.a, x.b}, {x.b, x.a}};
            for (const auto& sd : sides) {
                const mh_node v = D.t[sd[0]];
                if (v.op != VAR || Q.cols.at(v.imm0).kind != MH_COL_VAR || env.count(v.imm0))
                    continue;
                const uint8_t top = D.t[sd[1]].op;
                if (top == VAR || top == CONST) continue;
                const uint32_t t2 = env.empty() ? sd[1] : D.subst(sd[1], env);
                D.reads(t2, rd);
                if (rd.empty() || std::find(rd.begin(), rd.end(), v.imm0) != rd.end()) continue;
                const std::unordered_map<uint32_t, uint32_t> one{{v.imm0, t2}};
                for (auto& e : env) e.second = D.subst(e.second, one);
                env[v.imm0] = t2;
                def_cols.push_back(v.imm0);
                done = true;
                break;
            }
        }
        if (!done) rest.push_back(cn);
    }
    if (env.empty()) return false;
    uint32_t r;
    if (rest.empty()) {
        mh_node t{};
        t.op = TRUE_;
        r = D.add(t);
    } else {
        r = D.subst(rest[0], env);
        for (size_t i = 1; i < rest.size(); ++i) {
            mh_node a{};
            a.op = AND;
            a.a = r;
            a.b = D.subst(rest[i], env);
            r = D.add(a);
        }
    }
    std::vector<mh_node> tape;
    std::vector<uint8_t> hc;
    D.linearise(r, tape, &hc);
    std::vector<uint32_t> leaves;
    and_leaves(tape, (uint32_t)tape.size() - 1, leaves);
    std::vector<std::vector<uint32_t>> gconj, gcols;
    group_conjuncts(tape, hc, leaves, gconj, gcols);
    emit_tapes(q, tape, gconj);
    put_groups(q, gcols);
    for (uint32_t c : def_cols) {  // the definitions' tapes, in definition order
        std::vector<mh_node> dt;
        D.linearise(env.at(c), dt, nullptr);
        q.nodes.insert(q.nodes.end(), dt.begin(), dt.end());
        q.tape_off.push_back(q.nodes.size());
        q.def_cols.push_back(c);
    }
    return true;
}

extern "C" {

int32_t mh_terms_create(mh_terms** out) {
    if (!out) return mh_detail_set_err(MH_E_INVALID, "null out");
    *out = new (std::nothrow) mh_terms();
    return *out ? MH_OK : mh_detail_set_err(MH_E_NOMEM, "mh_terms_create");
}

int32_t mh_terms_destroy(mh_terms* t) {
    if (!t) return mh_detail_set_err(MH_E_INVALID, "null terms");
    delete t;
    return MH_OK;
}

int32_t mh_terms_set_options(mh_terms* t, uint32_t options) {
    if (!t) return mh_detail_set_err(MH_E_INVALID, "null terms");
    if (options & ~MH_TERMS_KECCAK_READS) return mh_detail_set_err(MH_E_INVALID, "unknown option");
    t->options = options;
    t->last.reset();
    return MH_OK;
}

int32_t mh_terms_append(mh_terms* t, const mh_node* nodes, uint64_t n_nodes,
                        const uint32_t* consts, uint64_t n_consts, const char* var_names,
                        uint64_t n_vars, const char* array_names, uint64_t n_arrays,
                        const char* fn_names, uint64_t n_fns) {
    if (!t || (n_nodes && !nodes) || (n_consts && !consts) || (n_vars && !var_names) ||
        (n_arrays && !array_names) || (n_fns && !fn_names))
        return mh_detail_set_err(MH_E_INVALID, "null argument");
    // validate every node against the store as it will be after this append, then append:
    // a rejected batch changes nothing (TermMirror.sync sends it again after an error)
    const size_t n0 = t->nodes.size(), p0 = t->pool.size();
    const size_t v0 = t->var_names.size(), a0 = t->array_names.size(), f0 = t->fn_names.size();
    for (uint64_t i = 0; i < n_nodes; ++i) {
        const mh_node& x = nodes[i];
        const uint64_t id = n0 + i;
        const int k = arity(x.op);
        if ((k > 0 && x.a >= id) || (k > 1 && x.b >= id) || (k > 2 && x.c >= id) ||
            (x.op == CONST && x.imm0 >= p0 + n_consts))
            return mh_detail_set_err(MH_E_INVALID, "node operand outside the term store");
    }
    try {
        for (uint64_t i = 0; i < n_consts; ++i) {
            Big v;
            memcpy(v.w, consts + 8 * i, 32);
            t->pool_index.emplace(v, (uint32_t)t->pool.size());
            t->pool.push_back(v);
        }
        for (uint64_t i = 0; i < n_nodes; ++i) {
            t->nodes.push_back(nodes[i]);
            t->memo.emplace(key_of(nodes[i]), (uint32_t)(n0 + i));
        }
        auto names = [](const char* p, uint64_t n, std::vector<std::string>& out) {
            for (uint64_t i = 0; i < n; ++i) {  // NUL-terminated, back to back
                const size_t len = strlen(p);
                out.emplace_back(p, len);
                p += len + 1;
            }
        };
        names(var_names, n_vars, t->var_names);
        names(array_names, n_arrays, t->array_names);
        names(fn_names, n_fns, t->fn_names);
    } catch (const std::bad_alloc&) {
        // back to the sizes on entry; map entries are dropped only where they point at an
        // appended element (an equal earlier constant or node keeps its own entry)
        for (size_t j = n0; j < t->nodes.size(); ++j) {
            auto it = t->memo.find(key_of(t->nodes[j]));
            if (it != t->memo.end() && it->second >= n0) t->memo.erase(it);
        }
        for (size_t j = p0; j < t->pool.size(); ++j) {
            auto it = t->pool_index.find(t->pool[j]);
            if (it != t->pool_index.end() && it->second >= p0) t->pool_index.erase(it);
        }
        t->nodes.resize(n0);
        t->pool.resize(p0);
        t->var_names.resize(v0);
        t->array_names.resize(a0);
        t->fn_names.resize(f0);
        return mh_detail_set_err(MH_E_NOMEM, "mh_terms_append");
    }
    return MH_OK;
}

int32_t mh_terms_sizes(const mh_terms* t, uint64_t* out /* [5] */) {
    if (!t || !out) return mh_detail_set_err(MH_E_INVALID, "null argument");
    out[0] = t->nodes.size();
    out[1] = t->pool.size();
    out[2] = t->var_names.size();
    out[3] = t->array_names.size();
    out[4] = t->fn_names.size();
    return MH_OK;
}

int32_t mh_query_build(mh_terms* t, const uint32_t* roots, uint32_t n_roots, mh_query** out,
                       mh_query_info* info) {
    if (!t || !out || !info || (n_roots && !roots)) return mh_detail_set_err(MH_E_INVALID, "null argument");
    *out = nullptr;
    for (uint32_t i = 0; i < n_roots; ++i)
        if (roots[i] >= t->nodes.size()) return mh_detail_set_err(MH_E_INVALID, "root outside the term store");
    std::unique_ptr<mh_query> q(new (std::nothrow) mh_query());
    if (!q) return mh_detail_set_err(MH_E_NOMEM, "mh_query_build");
    uint32_t flags = 0;
    try {
        QueryState* st = t->last.get();
        // The state keeps a checkpoint per root: a query sharing a prefix of d > 0 roots with it
        // takes it back to depth d and extends it by the rest (QueryState::advance) -- a child
        // of the last query, a JUMPI's other branch, the next state a BFS pops.  Otherwise, or
        // when the rest changes the harvest, the query is built afresh, taking over the
        // state's lowering when the harvests agree (start).
        size_t d = 0;
        if (st) {
            const size_t m = std::min<size_t>(st->roots.size(), n_roots);
            while (d < m && st->roots[d] == roots[d]) ++d;
        }
        if (st && d > 0 && st->advance(roots, n_roots, d)) {
            flags |= MH_QUERY_INCREMENTAL;
        } else if (st && d > 0) {
            // the rest changed the harvest: afresh (a new epoch of the scratch maps)
            t->last.reset();
            t->last.reset(new QueryState(*t));
            t->last->start(roots, n_roots);
        } else {
            std::unique_ptr<QueryState> prev = std::move(t->last);
            t->last.reset(new QueryState(*t, prev != nullptr));
            t->last->start(roots, n_roots, prev.get());
        }
        t->last->emit(*q, flags);
    } catch (const Fail& f) {
        t->last.reset();
        return mh_detail_set_err(f.code, f.msg.c_str());
    } catch (const std::out_of_range&) {
        t->last.reset();
        return mh_detail_set_err(MH_E_INVALID, "malformed term store (index out of range)");
    } catch (const std::bad_alloc&) {
        t->last.reset();
        return mh_detail_set_err(MH_E_NOMEM, "mh_query_build");
    }
    mh_query* r = q.release();
    *info = mh_query_info{};
    info->nodes = r->nodes.data();
    info->tape_off = r->tape_off.data();
    info->n_tapes = (uint32_t)r->tape_off.size() - 1;
    info->consts = r->consts.data();
    info->n_consts = (uint32_t)(r->consts.size() / 8);
    info->columns = r->columns.data();
    info->n_columns = (uint32_t)r->columns.size();
    info->names = r->names.data();
    info->names_len = (uint32_t)r->names.size();
    info->key_limbs = r->key_limbs.data();
    info->group_cols = r->group_cols.data();
    info->group_off = r->group_off.data();
    info->n_groups = (uint32_t)r->group_off.size() - 1;
    info->tables = r->tables.data();
    info->n_tables = (uint32_t)r->tables.size();
    info->table_limbs = r->table_limbs.data();
    info->flags = flags;
    info->n_keys = (uint32_t)(r->key_limbs.size() / NL);
    info->n_table_entries = (uint32_t)(r->table_limbs.size() / NL);
    info->n_defs = (uint32_t)r->def_cols.size();
    info->def_cols = r->def_cols.data();
    info->parent_len = r->parent_len;
    info->root_ends = r->root_ends.data();
    info->n_root_ends = (uint32_t)r->root_ends.size();
    *out = r;
    return MH_OK;
}

int32_t mh_query_free(mh_query* q) {
    if (!q) return mh_detail_set_err(MH_E_INVALID, "null query");
    delete q;
    return MH_OK;
}

}  // extern "C"
