// Candidate guide harvest on the host (mh_guide_harvest): what the sieve's guided rows try for
// one query.  The algorithm is mythril_amd/candidates.py's (documented there and restated here
// step for step, so the two produce the same mh_guide arrays -- tests/test_harvest.py): every
// conjunct of the lowered path condition inverted toward its columns (concat / extract / zext /
// and-mask / ite / +c / -c / xor c / *odd c / not / neg), Or as alternatives, ordered compares as
// boundary values, overflow predicates as extreme operands; symbolic equalities as bit copies or
// tried with the query's constants; ite conditions as soft hints (dominated single-column hints
// pruned); the parent query's witness first; per-column pools.  It runs on the query's lowered
// tape (VAR imm0 = column, CONST imm0 = index into the query's constants), so a LASER query's
// guide costs microseconds instead of the Python harvester's milliseconds.
//
// Values are bit-vectors of up to 1088 bits (tape.MAX_WIDTH), held in a fixed 1152-bit word with
// Python's wrap-then-mask arithmetic.  Alternatives keep Python dict order (insertion order,
// update keeps a key's position), because pool order -- and so the generated rows -- follows it.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <iterator>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/mythril_hip.h"

namespace {

constexpr int NL = 36;  // 1152-bit values
constexpr int kMaxAlts = 16, kMaxSets = 1024, kMaxPool = 64, kMaxEqConsts = 24;
constexpr int kProbDefault = 208, kProbParent = 192, kProbHint = 64, kHintsPerColumn = 2;
constexpr uint32_t kCopyFlag = 0x80000000u;

// op codes of include/mythril_hip.h (enum mh_op) / mythril_amd/tape.py Op
enum : uint8_t {
    CONST = MH_OP_CONST, VAR = MH_OP_VAR, TRUE_ = MH_OP_TRUE, FALSE_ = MH_OP_FALSE,
    BVADD = MH_OP_BVADD, BVSUB = MH_OP_BVSUB, BVMUL = MH_OP_BVMUL, BVNEG = MH_OP_BVNEG,
    BVNOT = MH_OP_BVNOT, BVAND = MH_OP_BVAND, BVOR = MH_OP_BVOR, BVXOR = MH_OP_BVXOR,
    BVSHL = MH_OP_BVSHL,
    BVLSHR = MH_OP_BVLSHR, EQ = MH_OP_EQ, BVULT = MH_OP_BVULT, BVULE = MH_OP_BVULE,
    BVUGT = MH_OP_BVUGT, BVUGE = MH_OP_BVUGE, BVSLT = MH_OP_BVSLT, BVSLE = MH_OP_BVSLE,
    BVSGT = MH_OP_BVSGT, BVSGE = MH_OP_BVSGE, AND = MH_OP_AND, OR = MH_OP_OR, NOT = MH_OP_NOT,
    ITE = MH_OP_ITE, EXTRACT = MH_OP_EXTRACT, CONCAT = MH_OP_CONCAT, ZEXT = MH_OP_ZEXT,
    SEXT = MH_OP_SEXT, KECCAK = MH_OP_KECCAK, ADD_NOOVFL_U = MH_OP_BVADD_NOOVFL_U,
    MUL_NOOVFL_U = MH_OP_BVMUL_NOOVFL_U, SUB_NOUDFL_U = MH_OP_BVSUB_NOUDFL_U,
};

struct U {  // unsigned 1152-bit integer, arithmetic mod 2^1152
    uint32_t w[NL];
    U() { memset(w, 0, sizeof w); }
    static U of(uint64_t x) { U r; r.w[0] = (uint32_t)x; r.w[1] = (uint32_t)(x >> 32); return r; }
    bool zero() const { for (uint32_t x : w) if (x) return false; return true; }
    bool operator==(const U& o) const { return memcmp(w, o.w, sizeof w) == 0; }
    bool operator!=(const U& o) const { return !(*this == o); }
    bool operator<(const U& o) const {
        for (int i = NL - 1; i >= 0; --i)
            if (w[i] != o.w[i]) return w[i] < o.w[i];
        return false;
    }
    int bitlen() const {
        for (int i = NL - 1; i >= 0; --i)
            if (w[i]) return 32 * i + 32 - __builtin_clz(w[i]);
        return 0;
    }
    bool bit(int i) const { return (w[i >> 5] >> (i & 31)) & 1u; }
};
U operator&(U a, const U& b) { for (int i = 0; i < NL; ++i) a.w[i] &= b.w[i]; return a; }
U operator|(U a, const U& b) { for (int i = 0; i < NL; ++i) a.w[i] |= b.w[i]; return a; }
U operator^(U a, const U& b) { for (int i = 0; i < NL; ++i) a.w[i] ^= b.w[i]; return a; }
U operator~(U a) { for (uint32_t& x : a.w) x = ~x; return a; }
U operator+(const U& a, const U& b) {
    U r;
    uint64_t c = 0;
    for (int i = 0; i < NL; ++i) { c += (uint64_t)a.w[i] + b.w[i]; r.w[i] = (uint32_t)c; c >>= 32; }
    return r;
}
U operator-(const U& a, const U& b) { return a + (~b + U::of(1)); }
U neg(const U& a) { return ~a + U::of(1); }
U operator*(const U& a, const U& b) {
    U r;
    for (int i = 0; i < NL; ++i) {
        if (!a.w[i]) continue;
        uint64_t c = 0;
        for (int j = 0; i + j < NL; ++j) {
            c += (uint64_t)a.w[i] * b.w[j] + r.w[i + j];
            r.w[i + j] = (uint32_t)c;
            c >>= 32;
        }
    }
    return r;
}
U shl(const U& a, int s) {
    U r;
    if (s >= 32 * NL) return r;
    const int q = s >> 5, b = s & 31;
    for (int i = NL - 1; i >= q; --i) {
        uint32_t v = a.w[i - q] << b;
        if (b && i - q - 1 >= 0) v |= a.w[i - q - 1] >> (32 - b);
        r.w[i] = v;
    }
    return r;
}
U shr(const U& a, int s) {
    U r;
    if (s >= 32 * NL) return r;
    const int q = s >> 5, b = s & 31;
    for (int i = 0; i + q < NL; ++i) {
        uint32_t v = a.w[i + q] >> b;
        if (b && i + q + 1 < NL) v |= a.w[i + q + 1] << (32 - b);
        r.w[i] = v;
    }
    return r;
}
// 2^w - 1 for w in 0..1088 (< 1152), built once
const U& mask(int w) {
    static const std::vector<U> table = [] {
        std::vector<U> t(1089);
        for (int i = 1; i <= 1088; ++i) t[i] = shl(U::of(1), i) - U::of(1);
        return t;
    }();
    return table[w];
}

// a column value (columns are 1..256 bits wide): what alternatives and pools hold
struct V {
    uint32_t w[8];
    bool operator==(const V& o) const { return memcmp(w, o.w, sizeof w) == 0; }
    bool operator!=(const V& o) const { return !(*this == o); }
    bool operator<(const V& o) const {
        for (int i = 7; i >= 0; --i)
            if (w[i] != o.w[i]) return w[i] < o.w[i];
        return false;
    }
};
V lo256(const U& u) { V v; memcpy(v.w, u.w, sizeof v.w); return v; }

// the inverse of an odd k mod 2^w (Newton: x <- x (2 - k x), 5 correct bits doubling)
U inverse_mod(const U& k, int w) {
    U x = k;  // k * k = 1 mod 8 for odd k
    for (int i = 0; i < 12; ++i) x = x * (U::of(2) - k * x);
    return x & mask(w);
}

// One harvest allocates thousands of small vectors (alternatives, memo entries) and frees them
// all at the end: they come from a bump arena -- per thread, reset by mh_guide_harvest, or a
// harvester session's own, kept while its memo is (mh_harvester).
struct Arena {
    std::vector<std::unique_ptr<char[]>> blocks;
    std::vector<size_t> sizes;
    size_t cur = 0, off = 0;
    void* alloc(size_t n, size_t align) {
        for (;;) {
            if (cur < blocks.size()) {
                const size_t o = (off + align - 1) & ~(align - 1);
                if (o + n <= sizes[cur]) {
                    off = o + n;
                    return blocks[cur].get() + o;
                }
                ++cur;
                off = 0;
                continue;
            }
            const size_t sz = std::max<size_t>(n + align, (size_t)1 << 20);
            blocks.emplace_back(new char[sz]);
            sizes.push_back(sz);
        }
    }
    void reset() {
        cur = off = 0;
        while (blocks.size() > 16) {  // keep at most 16 MB between harvests
            blocks.pop_back();
            sizes.pop_back();
        }
    }
    size_t used() const {
        size_t n = off;
        for (size_t i = 0; i < cur && i < sizes.size(); ++i) n += sizes[i];
        return n;
    }
};
thread_local Arena g_arena;
thread_local Arena* g_cur = &g_arena;  // the arena ArenaAlloc draws from

template <class T>
struct ArenaAlloc {
    using value_type = T;
    ArenaAlloc() = default;
    template <class O>
    ArenaAlloc(const ArenaAlloc<O>&) {}
    T* allocate(size_t n) { return static_cast<T*>(g_cur->alloc(n * sizeof(T), alignof(T))); }
    void deallocate(T*, size_t) {}
    template <class O>
    bool operator==(const ArenaAlloc<O>&) const { return true; }
    template <class O>
    bool operator!=(const ArenaAlloc<O>&) const { return false; }
};
template <class T>
using AVec = std::vector<T, ArenaAlloc<T>>;

struct Node {
    uint8_t op;
    uint16_t width;
    uint32_t a, b, c, imm0, imm1;
};

using Alt = AVec<std::pair<uint32_t, V>>;  // (column, value) in dict insertion order
using Alts = AVec<Alt>;
// an inversion's result, shared by the memo and its callers; none = "don't know" (Python None)
struct Res {
    bool none = true;
    std::shared_ptr<const Alts> p;
    const Alts& alts() const {
        static const Alts kEmpty;
        return p ? *p : kEmpty;
    }
};

Res none_() { return Res(); }
Res of(Alts a) {
    Res r;
    r.none = false;
    r.p = std::allocate_shared<const Alts>(ArenaAlloc<Alts>(), std::move(a));
    return r;
}
Res one_empty() { return of(Alts{Alt{}}); }  // [{}]

const V* find(const Alt& a, uint32_t k) {
    for (const auto& kv : a)
        if (kv.first == k) return &kv.second;
    return nullptr;
}
// dict(y).update(x)
Alt updated(const Alt& y, const Alt& x) {
    Alt z = y;
    for (const auto& kv : x) {
        bool hit = false;
        for (auto& zz : z)
            if (zz.first == kv.first) { zz.second = kv.second; hit = true; break; }
        if (!hit) z.push_back(kv);
    }
    return z;
}
bool is_only_empty(const Alts& a) { return a.size() == 1 && a[0].empty(); }
Alts head(const Alts& a, size_t n) { return Alts(a.begin(), a.begin() + std::min(n, a.size())); }

// candidates.py _merge
Alts merge(const Alts& xs, const Alts& ys) {
    if (is_only_empty(ys)) return head(xs, kMaxAlts);
    if (is_only_empty(xs)) return head(ys, kMaxAlts);
    if (xs.size() == 1 && ys.size() == 1) {
        const Alt* x = &xs[0];
        const Alt* y = &ys[0];
        if (y->size() < x->size()) std::swap(x, y);
        for (const auto& kv : *x) {
            const V* v = find(*y, kv.first);
            if (v && *v != kv.second) return {};
        }
        return {updated(*y, *x)};
    }
    Alts out;
    for (const Alt& x : xs)
        for (const Alt& y : ys) {
            bool clash = false;
            for (const auto& kv : y) {
                const V* v = find(x, kv.first);
                if (v && *v != kv.second) { clash = true; break; }
            }
            if (clash) continue;
            out.push_back(updated(x, y));
            if ((int)out.size() >= kMaxAlts) return out;
        }
    return out;
}

struct Seg { int lo, n; uint32_t col; int col_lo; };
struct Copy { uint32_t dst, src; int dlo, slo, nb; };

struct Harvester {
    std::vector<Node> nd;
    std::vector<U> pool;              // the query's constants
    std::vector<int> cv_state;        // const_value memo: 0 unknown, 1 constant, 2 not
    AVec<U> cv;
    uint32_t n_cols = 0;
    std::vector<uint16_t> widths;
    // inversion memo: key -> (result, hints produced, transitively)
    // (kind, node, value, mask) with values interned; hints by id (one per distinct hint)
    struct Key {
        uint32_t kind, n, v, m;
        uint32_t g = 0;  // the node's generation (set by memoised / memo_hints from gen[n])
        bool operator==(const Key& o) const {
            return kind == o.kind && n == o.n && v == o.v && m == o.m && g == o.g;
        }
    };
    struct KeyHash {
        size_t operator()(const Key& k) const {
            uint64_t h = ((uint64_t)k.n << 32 | k.v) * 0x9E3779B97F4A7C15ull;
            h ^= ((uint64_t)k.m << 1 | k.kind) * 0xC2B2AE3D27D4EB4Full;
            h ^= (uint64_t)k.g * 0x94D049BB133111EBull;
            return (size_t)(h ^ (h >> 31));
        }
    };
    struct UHash {
        size_t operator()(const U& u) const {
            uint64_t h = 1469598103934665603ull;
            for (int i = 0; i < NL; ++i) h = (h ^ u.w[i]) * 1099511628211ull;
            return (size_t)h;
        }
    };
    struct Memo { Res r; AVec<uint32_t> hints; };
    std::unordered_map<U, uint32_t, UHash, std::equal_to<U>, ArenaAlloc<std::pair<const U, uint32_t>>>
        interned;
    std::unordered_map<Key, Memo, KeyHash, std::equal_to<Key>, ArenaAlloc<std::pair<const Key, Memo>>>
        memo;
    AVec<AVec<uint32_t>> cap;
    AVec<std::pair<int, std::shared_ptr<const Alts>>> sets;
    AVec<uint32_t> hints;      // hint ids in the order they became hint sets
    std::vector<uint64_t> pool_digest;  // harvest(): digests of pools[c] at [c * kMaxPool ...)
    std::map<AVec<uint32_t>, uint32_t, std::less<AVec<uint32_t>>,
             ArenaAlloc<std::pair<const AVec<uint32_t>, uint32_t>>> hint_ids;
    AVec<Alts> hint_alts;      // by id: the alternatives a hint set holds
    AVec<char> hint_done;      // by id: already a hint of this query
    // by id, for prune_hints: the one column every alternative sets (-1: not a single-column
    // set) and the largest / smallest value it proposes (a hint set never changes once made)
    AVec<int32_t> hint_col;
    AVec<V> hint_hi, hint_lo;
    std::unordered_map<const Alts*, uint32_t, std::hash<const Alts*>, std::equal_to<const Alts*>,
                       ArenaAlloc<std::pair<const Alts* const, uint32_t>>> hint_of_result;
    AVec<std::shared_ptr<const Alts>> hint_results;
    int n_hints = 0;
    std::vector<std::vector<std::vector<Copy>>> copy_sets;
    std::vector<U> query_consts;
    // the last query's conjuncts and constants (sorted, unique), kept across a session's queries
    std::vector<uint32_t> last_conj;
    std::vector<U> last_qc;
    std::map<int, std::vector<U>> consts_by_width;
    std::map<int, std::vector<uint32_t>> const_ids_by_width;  // their interned ids
    // eq_nodes per conjunct (a function of the tape prefix: kept across a session's queries)
    std::unordered_map<uint64_t, std::vector<uint32_t>> eq_nodes_of;  // by nk(conjunct)
    // What a conjunct and an equality node contribute to a query, kept across a session's
    // queries (functions of the tape prefix, like the memo): the set pushed (null: none) and
    // the hint ids the inversions emit, replayed in order -- exactly what the memo's hits would
    // do, without copying the alternatives again (a 400-constraint path re-read every earlier
    // conjunct's sets and every (equality, constant) pair per query)
    struct Contribution {
        std::shared_ptr<const Alts> set;
        std::vector<uint32_t> hints;
    };
    std::unordered_map<uint64_t, Contribution> conj_done;  // by nk(conjunct)
    struct EqPlan {
        bool skip = false;        // a Bool, a constant side, or both sides equal once stripped
        uint32_t x = 0, y = 0;
        std::vector<std::vector<Copy>> copies;  // copy alternatives (then no value pairs)
        std::unordered_map<uint32_t, Contribution> by_const;  // by the constant's interned id
    };
    std::unordered_map<uint64_t, EqPlan> eq_plan;  // by nk(equality node)
    // Node generations: a session whose next tape shares only a prefix of p nodes with the last
    // one (a JUMPI's other branch, the next state a BFS pops: the same path, another condition)
    // keeps every memo of the nodes below p and gives the indices from p on a new generation,
    // so entries of the nodes the new tape replaces are never found again (truncate)
    std::vector<uint32_t> gen;
    uint32_t cur_gen = 0;
    uint64_t nk(uint32_t n) const { return (uint64_t)gen[n] << 32 | n; }
    void truncate(uint32_t p, uint32_t pc) {
        ++cur_gen;
        nd.resize(p);
        gen.resize(p);
        cv_state.resize(p);
        cv.resize(p);
        pool.resize(pc);
        last_conj.clear();  // its constants are recounted from the query's conjuncts
        last_qc.clear();
    }
    std::vector<uint32_t> memo_hints(Key k) const {
        k.g = gen[k.n];
        auto it = memo.find(k);
        if (it == memo.end()) return {};
        return std::vector<uint32_t>(it->second.hints.begin(), it->second.hints.end());
    }

    // a kept harvester's next query (its tape extends the last one's): the memo, interned values
    // and hint ids stay, the query's own sets and hints start empty
    void begin_query() {
        sets.clear();
        hints.clear();
        std::fill(hint_done.begin(), hint_done.end(), 0);
        n_hints = 0;
        copy_sets.clear();
        query_consts.clear();
        consts_by_width.clear();
        const_ids_by_width.clear();
    }

    static int arity(uint8_t op) {  // tape.py ARITY (lowered tapes hold no host-only ops)
        switch (op) {
            case CONST: case VAR: case TRUE_: case FALSE_: return 0;
            case BVNEG: case BVNOT: case NOT: case EXTRACT: case ZEXT: case SEXT: case KECCAK:
                return 1;
            case ITE: case MH_OP_EVM_ADDMOD: case MH_OP_EVM_MULMOD: return 3;
            default: return 2;
        }
    }
    // mh_guide_harvest_inc: an operand whose value the parent witness fixes (every column it
    // reads has a parent value, every op is one of the bit-layout / linear ops below) counts as
    // known when the other side of an arithmetic op, an equality or a comparison must be
    // solved for -- the incremental round's guide then moves one side and keeps the other where
    // the parent had it (candidates.Harvester parent_eval, the same rule)
    bool peval = false;
    std::unordered_map<uint32_t, U> parent_of;  // column -> parent value
    std::vector<uint8_t> pv_state;                // 0 unknown, 1 known, 2 not
    std::vector<U> pv;
    const U* parent_value(uint32_t root) {
        if (!peval) return nullptr;
        if (pv_state.size() < nd.size()) {
            pv_state.resize(nd.size(), 0);
            pv.resize(nd.size());
        }
        std::vector<std::pair<uint32_t, bool>> st{{root, false}};
        while (!st.empty()) {
            const auto [n, done] = st.back();
            st.pop_back();
            if (pv_state[n]) continue;
            const Node x = nd[n];
            if (const U* c = const_value(n)) {
                pv[n] = *c;
                pv_state[n] = 1;
                continue;
            }
            const bool un = x.op == BVNOT || x.op == BVNEG || x.op == ZEXT || x.op == EXTRACT;
            const bool bin = x.op == BVADD || x.op == BVSUB || x.op == BVXOR || x.op == BVAND ||
                             x.op == BVOR || x.op == BVMUL || x.op == CONCAT;
            if (x.op == VAR) {
                auto it = x.imm0 < n_cols ? parent_of.find(x.imm0) : parent_of.end();
                pv_state[n] = it == parent_of.end() ? 2 : 1;
                if (it != parent_of.end()) pv[n] = it->second & mask(x.width);
                continue;
            }
            if (!un && !bin) {
                pv_state[n] = 2;
                continue;
            }
            if (!done) {
                st.push_back({n, true});
                st.push_back({x.a, false});
                if (bin) st.push_back({x.b, false});
                continue;
            }
            if (pv_state[x.a] != 1 || (bin && pv_state[x.b] != 1)) {
                pv_state[n] = 2;
                continue;
            }
            const U& a = pv[x.a];
            const U m = mask(x.width);
            U v;
            switch (x.op) {
                case BVNOT: v = ~a & m; break;
                case BVNEG: v = neg(a) & m; break;
                case ZEXT: v = a; break;
                case EXTRACT: v = shr(a, (int)x.imm1) & m; break;
                case BVADD: v = (a + pv[x.b]) & m; break;
                case BVSUB: v = (a - pv[x.b]) & m; break;
                case BVXOR: v = (a ^ pv[x.b]) & m; break;
                case BVAND: v = a & pv[x.b]; break;
                case BVOR: v = a | pv[x.b]; break;
                case BVMUL: v = (a * pv[x.b]) & m; break;
                default: v = shl(a, nd[x.b].width) | pv[x.b]; break;  // CONCAT
            }
            pv[n] = v;
            pv_state[n] = 1;
        }
        return pv_state[root] == 1 ? &pv[root] : nullptr;
    }
    // the operand to solve for and the other side's value: a constant first (either side), then
    // (peval) a side the parent fixes, b before a
    // (a_first: a constant a before a constant b, the comparisons' order)
    bool pick(uint32_t a, uint32_t b, uint32_t& t, U& k, bool a_first = false) {
        if (a_first)
            if (const U* ka = const_value(a)) { t = b; k = *ka; return true; }
        if (const U* kb = const_value(b)) { t = a; k = *kb; return true; }
        if (const U* ka = const_value(a)) { t = b; k = *ka; return true; }
        if (const U* pb = parent_value(b)) { t = a; k = *pb; return true; }
        if (const U* pa = parent_value(a)) { t = b; k = *pa; return true; }
        return false;
    }

    const U* const_value(uint32_t n) {
        if (cv_state[n] == 0) {
            const Node& x = nd[n];
            bool ok = false;
            U v;
            if (x.op == CONST) { v = pool[x.imm0]; ok = true; }
            else if (x.op == TRUE_) { v = U::of(1); ok = true; }
            else if (x.op == FALSE_) { ok = true; }
            else if (x.op == CONCAT) {
                const U* hi = const_value(x.a);
                const U* lo = hi ? const_value(x.b) : nullptr;
                if (hi && lo) { v = shl(*hi, nd[x.b].width) | *lo; ok = true; }
            } else if (x.op == EXTRACT || x.op == ZEXT || x.op == SEXT) {
                const U* a = const_value(x.a);
                if (a) {
                    ok = true;
                    if (x.op == EXTRACT) v = shr(*a, (int)x.imm1) & mask((int)(x.imm0 - x.imm1 + 1));
                    else if (x.op == SEXT && a->bit(nd[x.a].width - 1))
                        v = *a | shl(mask((int)x.imm0), nd[x.a].width);
                    else v = *a;
                }
            }
            cv_state[n] = ok ? 1 : 2;
            cv[n] = v;
        }
        return cv_state[n] == 1 ? &cv[n] : nullptr;
    }

    template <class F>
    Res memoised(Key key, F compute) {
        key.g = gen[key.n];
        auto it = memo.find(key);
        if (it == memo.end()) {
            cap.emplace_back();
            Res r = compute();
            AVec<uint32_t> hs = std::move(cap.back());
            cap.pop_back();
            if (!cap.empty()) cap.back().insert(cap.back().end(), hs.begin(), hs.end());
            memo.emplace(key, Memo{r, std::move(hs)});
            return r;
        }
        const Memo& m = it->second;
        for (uint32_t id : m.hints) emit_hint(id);
        return m.r;
    }
    uint32_t intern(const U& u) {
        auto it = interned.find(u);
        if (it != interned.end()) return it->second;
        return interned.emplace(u, (uint32_t)interned.size()).first->second;
    }
    static void push_u(std::vector<uint32_t>& k, const U& v) {
        int top = NL;
        while (top > 0 && !v.w[top - 1]) --top;
        k.push_back((uint32_t)top);
        k.insert(k.end(), v.w, v.w + top);
    }

    Res invert_bits(uint32_t n, const U& value, const U& msk, int depth = 0) {
        return invert_bits_ids(n, intern(value), intern(msk), value, msk, depth);
    }
    // the same with the value and mask already interned (the eq loop's constants)
    Res invert_bits_ids(uint32_t n, uint32_t vid, uint32_t mid, const U& value, const U& msk,
                        int depth = 0) {
        return memoised(Key{0u, n, vid, mid}, [&]() {
            return depth < 64 ? invert_bits_(n, value & msk, msk, depth) : none_();
        });
    }
    Res invert_bits_(uint32_t n, const U& value, const U& msk, int depth) {
        const Node x = nd[n];
        const bool full = msk == mask(x.width);
        if (const U* c = const_value(n)) return (*c & msk) == value ? one_empty() : of({});
        if (x.op == VAR) {
            if (x.imm0 >= n_cols) return none_();
            return of({Alt{{x.imm0, lo256(value)}}});
        }
        if (x.op == CONCAT) {
            Alts acc{Alt{}};
            for (const auto& leaf : concat_leaves(n)) {
                const U m = shr(msk, leaf.second) & mask(nd[leaf.first].width);
                if (m.zero()) continue;
                Res r = invert_bits(leaf.first, shr(value, leaf.second) & m, m, depth + 1);
                if (r.none || is_only_empty(r.alts())) continue;
                const Alts& ra = r.alts();
                if (acc.size() == 1 && ra.size() == 1 && ra[0].size() < acc[0].size()) {
                    // _merge's one-pair case with the accumulated alternative the larger: it
                    // keeps its order and gains r's new columns at the end -- in place
                    bool clash = false;
                    for (const auto& kv : ra[0]) {
                        const V* v = find(acc[0], kv.first);
                        if (v) { clash |= *v != kv.second; continue; }
                        acc[0].push_back(kv);
                    }
                    if (clash) return of({});
                    continue;
                }
                acc = merge(acc, ra);
                if (acc.empty()) return of(acc);
            }
            return of(std::move(acc));
        }
        if (x.op == EXTRACT) return invert_bits(x.a, shl(value, x.imm1), shl(msk, x.imm1), depth + 1);
        if (x.op == BVAND) {
            const uint32_t pr[2][2] = {{x.a, x.b}, {x.b, x.a}};
            for (const auto& p : pr) {
                if (const U* m = const_value(p[1])) {
                    if (!(value & ~*m & msk).zero()) return of({});
                    return invert_bits(p[0], value & *m, msk & *m, depth + 1);
                }
            }
            return none_();
        }
        if (x.op == ZEXT || x.op == SEXT) {
            const int wa = nd[x.a].width;
            if (x.op == ZEXT && !shr(value, wa).zero()) return of({});
            return invert_bits(x.a, value & mask(wa), msk & mask(wa), depth + 1);
        }
        if (x.op == ITE) {
            Alts out;
            const std::pair<uint32_t, bool> br[2] = {{x.b, true}, {x.c, false}};
            for (const auto& p : br) {
                Res r = invert_bits(p.first, value, msk, depth + 1);
                if (r.none || r.alts().empty()) continue;
                Res cond = invert_bool(x.a, p.second, depth + 1);
                if (!cond.none && !cond.alts().empty() && !is_only_empty(cond.alts())) hint(cond);
                out.insert(out.end(), r.alts().begin(), r.alts().end());
            }
            bool has_empty = false;
            for (const Alt& a : out) has_empty |= a.empty();
            if (out.size() > 1 && has_empty) {
                Alts kept;
                for (const Alt& a : out) if (!a.empty()) kept.push_back(a);
                out.swap(kept);
            }
            return of(head(out, kMaxAlts));
        }
        if (!full) return none_();
        const U m = mask(x.width);
        if (x.op == BVADD || x.op == BVSUB || x.op == BVXOR || x.op == BVMUL) {
            uint32_t t;
            U k;
            if (!pick(x.a, x.b, t, k)) return none_();
            U v;
            if (x.op == BVADD) v = value - k;
            else if (x.op == BVSUB) v = t == x.a ? value + k : k - value;
            else if (x.op == BVXOR) v = value ^ k;
            else {
                if (!k.bit(0)) return none_();
                v = value * inverse_mod(k, x.width);
            }
            return invert_bits(t, v & m, m, depth + 1);
        }
        if (x.op == BVNOT) return invert_bits(x.a, ~value & m, m, depth + 1);
        if (x.op == BVNEG) return invert_bits(x.a, neg(value) & m, m, depth + 1);
        return none_();
    }

    std::unordered_map<uint64_t, std::vector<std::pair<uint32_t, int>>> leaves_memo;
    const std::vector<std::pair<uint32_t, int>>& concat_leaves(uint32_t n) {
        auto it = leaves_memo.find(nk(n));
        if (it != leaves_memo.end()) return it->second;
        std::vector<std::pair<uint32_t, int>> got;
        std::vector<std::pair<uint32_t, int>> st{{n, 0}};
        while (!st.empty()) {
            auto [x, lo] = st.back();
            st.pop_back();
            if (nd[x].op == CONCAT) {
                st.push_back({nd[x].a, lo + nd[nd[x].b].width});
                st.push_back({nd[x].b, lo});
            } else {
                got.push_back({x, lo});
            }
        }
        return leaves_memo[nk(n)] = std::move(got);
    }

    Res invert_bool(uint32_t n, bool truth, int depth = 0) {
        if (depth > 64) return none_();
        return memoised(Key{1u, n, truth ? 1u : 0u, 0u}, [&]() { return invert_bool_(n, truth, depth); });
    }
    Res invert_bool_(uint32_t n, bool truth, int depth) {
        const Node x = nd[n];
        if (const U* c = const_value(n)) return (!c->zero()) == truth ? one_empty() : of({});
        if (x.op == NOT) return invert_bool(x.a, !truth, depth + 1);
        if (x.op == AND || x.op == OR) {
            const bool conj = (x.op == AND) == truth;
            Res a = invert_bool(x.a, truth, depth + 1);
            Res b = invert_bool(x.b, truth, depth + 1);
            if (conj) return of(merge(a.none ? Alts{Alt{}} : a.alts(), b.none ? Alts{Alt{}} : b.alts()));
            Alts out;
            if (!a.none) out = a.alts();
            if (!b.none) out.insert(out.end(), b.alts().begin(), b.alts().end());
            if (a.none && b.none) return none_();
            return of(head(out, kMaxAlts));
        }
        if (x.op == EQ) {
            if (nd[x.a].width == 0) return none_();
            uint32_t t;
            U k;
            if (!pick(x.a, x.b, t, k)) return none_();
            if (truth) return invert_bits(t, k, mask(nd[t].width));
            return one_empty();
        }
        if (x.op == ADD_NOOVFL_U || x.op == MUL_NOOVFL_U || x.op == SUB_NOUDFL_U) {
            const int wt = nd[x.a].width;
            const U M = mask(wt);
            std::vector<std::pair<U, U>> pairs;
            if (x.op == SUB_NOUDFL_U) {
                if (truth) pairs = {{U::of(0), U::of(0)}, {U::of(1), U::of(0)}};
                else pairs = {{U::of(0), U::of(1)}, {U::of(1), U::of(2)}};
            } else if (truth) {
                pairs = {{U::of(0), U::of(0)}, {U::of(1), U::of(1)}};
            } else {
                pairs = {{M, U::of(2)}, {M, M}};
            }
            Alts out;
            for (const auto& p : pairs) {
                Res ra = invert_bits(x.a, p.first, M);
                Res rb = invert_bits(x.b, p.second, M);
                if (ra.none && rb.none) continue;
                Alts mg = merge(ra.none ? Alts{Alt{}} : ra.alts(), rb.none ? Alts{Alt{}} : rb.alts());
                out.insert(out.end(), mg.begin(), mg.end());
            }
            if (out.empty()) return none_();
            return of(head(out, kMaxAlts));
        }
        if (x.op >= BVULT && x.op <= BVSGE) {
            const int wt = nd[x.a].width;
            uint32_t t;
            U k;
            if (!pick(x.a, x.b, t, k, true)) return none_();
            Alts out;
            for (const U& v : boundary(x.op, k, t == x.a, truth, wt)) {
                Res r = invert_bits(t, v, mask(wt));
                if (!r.none && !r.alts().empty()) out.insert(out.end(), r.alts().begin(), r.alts().end());
            }
            return of(head(out, kMaxAlts));
        }
        return none_();
    }

    static std::vector<U> boundary(uint8_t op, const U& k, bool var_left, bool truth, int w) {
        const U m = mask(w);
        const bool less = op == BVULT || op == BVULE || op == BVSLT || op == BVSLE;
        bool strict = op == BVULT || op == BVUGT || op == BVSLT || op == BVSGT;
        bool want_below = less == var_left;
        if (!truth) { want_below = !want_below; strict = !strict; }
        std::vector<U> vals;
        if (want_below) {
            if (strict) vals = {k - U::of(1), shr(k, 1), U::of(0)};
            else vals = {k, k - U::of(1), U::of(0)};
        } else {
            if (strict) vals = {k + U::of(1), k + U::of(2), shl(k, 1) + U::of(1)};
            else vals = {k, k + U::of(1)};
        }
        for (U& v : vals) v = v & m;
        return vals;
    }

    // bits of term n that are bits of a column: (lo, nbits, column, column_lo); false = computes
    bool segments(uint32_t n, std::vector<Seg>& out, int depth = 0) {
        out.clear();
        if (depth > 64) return false;
        const Node x = nd[n];
        if (const_value(n)) return true;
        if (x.op == VAR) {
            if (x.imm0 >= n_cols) return false;
            out.push_back({0, (int)x.width, x.imm0, 0});
            return true;
        }
        if (x.op == CONCAT) {
            std::vector<Seg> hi, lo;
            if (!segments(x.a, hi, depth + 1) || !segments(x.b, lo, depth + 1)) return false;
            const int wb = nd[x.b].width;
            out = lo;
            for (const Seg& s : hi) out.push_back({s.lo + wb, s.n, s.col, s.col_lo});
            return true;
        }
        if (x.op == EXTRACT) {
            std::vector<Seg> inner;
            if (!segments(x.a, inner, depth + 1)) return false;
            for (const Seg& s : inner) {
                const int s0 = std::max(s.lo, (int)x.imm1), s1 = std::min(s.lo + s.n, (int)x.imm0 + 1);
                if (s0 < s1) out.push_back({s0 - (int)x.imm1, s1 - s0, s.col, s.col_lo + (s0 - s.lo)});
            }
            return true;
        }
        if (x.op == ZEXT) return segments(x.a, out, depth + 1);
        if (x.op == BVAND) {
            const uint32_t pr[2][2] = {{x.a, x.b}, {x.b, x.a}};
            for (const auto& p : pr) {
                const U* m = const_value(p[1]);
                if (m && ((*m) & ((*m) + U::of(1))).zero()) {
                    std::vector<Seg> inner;
                    if (!segments(p[0], inner, depth + 1)) return false;
                    const int k = m->bitlen();
                    for (const Seg& s : inner)
                        if (s.lo < k) out.push_back({s.lo, std::min(s.n, k - s.lo), s.col, s.col_lo});
                    return true;
                }
            }
            return false;
        }
        if (x.op == ITE) {
            if (const_value(x.c)) return segments(x.b, out, depth + 1);
            if (const_value(x.b)) return segments(x.c, out, depth + 1);
        }
        return false;
    }

    std::vector<std::vector<Copy>> copy_alternatives(uint32_t x, uint32_t y) {
        std::vector<Seg> sx, sy;
        const bool okx = segments(x, sx), oky = segments(y, sy);
        if (!okx || !oky || sx.empty() || sy.empty()) return {};
        std::vector<std::vector<Copy>> alts;
        const std::vector<Seg>* sides[2][2] = {{&sx, &sy}, {&sy, &sx}};
        for (auto& sd : sides) {
            std::vector<Copy> copies;
            for (const Seg& d : *sd[0])
                for (const Seg& s : *sd[1]) {
                    const int s0 = std::max(d.lo, s.lo), s1 = std::min(d.lo + d.n, s.lo + s.n);
                    if (s0 < s1 && d.col != s.col)
                        copies.push_back({d.col, s.col, d.col_lo + (s0 - d.lo), s.col_lo + (s0 - s.lo), s1 - s0});
                }
            if (!copies.empty()) {
                if (copies.size() > 256) copies.resize(256);
                alts.push_back(std::move(copies));
            }
        }
        return alts;
    }

    // candidates.py Harvester._hint: a hint is identified by its alternatives' items (each
    // alternative's sorted by column); the first MAX_SETS/4 distinct ones become hint sets
    void hint(const Res& r) {
        // the same (memoised) inversion result is the same hint: look it up by identity first
        auto known = hint_of_result.find(r.p.get());
        if (known != hint_of_result.end()) return emit_hint(known->second);
        const Alts& alts = r.alts();
        AVec<uint32_t> key;
        for (const Alt& a : alts) {
            Alt s = a;
            std::sort(s.begin(), s.end(), [](const auto& p, const auto& q) { return p.first < q.first; });
            key.push_back(0xFFFFFFFFu);
            for (const auto& kv : s) {
                key.push_back(kv.first);
                key.insert(key.end(), kv.second.w, kv.second.w + 8);
            }
        }
        auto got = hint_ids.emplace(std::move(key), (uint32_t)hint_alts.size());
        if (got.second) {
            Alts kept;
            for (const Alt& a : alts) if (!a.empty()) kept.push_back(a);
            hint_alts.push_back(head(kept, kMaxAlts));
            hint_done.push_back(0);
            const Alts& ha = hint_alts.back();
            int32_t col = ha.empty() ? -1 : (int32_t)ha[0][0].first;
            for (const Alt& a : ha)
                if (a.size() != 1 || (int32_t)a[0].first != col) { col = -1; break; }
            V mx{}, mn{};
            if (col >= 0) {
                mx = mn = ha[0][0].second;
                for (const Alt& a : ha) { mx = std::max(mx, a[0].second); mn = std::min(mn, a[0].second); }
            }
            hint_col.push_back(col);
            hint_hi.push_back(mx);
            hint_lo.push_back(mn);
        }
        hint_results.push_back(r.p);  // keeps the identity valid
        hint_of_result.emplace(r.p.get(), got.first->second);
        emit_hint(got.first->second);
    }
    void emit_hint(uint32_t id) {
        if (!cap.empty()) cap.back().push_back(id);
        if (!hint_done[id] && n_hints < kMaxSets / 4) {
            hint_done[id] = 1;
            ++n_hints;
            hints.push_back(id);
        }
    }

    std::vector<uint32_t> conjuncts(uint32_t root) {
        std::vector<uint32_t> out, st{root};
        while (!st.empty()) {
            const uint32_t n = st.back();
            st.pop_back();
            if (nd[n].op == AND) { st.push_back(nd[n].b); st.push_back(nd[n].a); }
            else out.push_back(n);
        }
        return out;
    }

    std::vector<uint32_t> eq_seen;
    uint32_t eq_epoch = 0;
    std::vector<uint32_t> eq_nodes(uint32_t root, size_t limit = 4096) {
        std::vector<uint32_t> out, st{root};
        ++eq_epoch;  // seen = stamped with this walk's epoch
        if (eq_seen.size() != nd.size()) eq_seen.assign(nd.size(), 0);
        size_t n_seen = 0;
        while (!st.empty() && n_seen < limit) {
            const uint32_t n = st.back();
            st.pop_back();
            if (eq_seen[n] == eq_epoch) continue;
            eq_seen[n] = eq_epoch;
            ++n_seen;
            if (nd[n].op == EQ) out.push_back(n);
            const int k = arity(nd[n].op);
            if (k >= 1) st.push_back(nd[n].a);
            if (k >= 2) st.push_back(nd[n].b);
            if (k >= 3) st.push_back(nd[n].c);
        }
        return out;
    }

    std::pair<uint32_t, uint32_t> strip_common(uint32_t x, uint32_t y) {
        for (int i = 0; i < 64; ++i) {
            const Node ox = nd[x], oy = nd[y];
            if (ox.op != oy.op || ox.width != oy.width) break;
            const uint8_t op = ox.op;
            if (op == KECCAK || op == BVNOT || op == BVNEG ||
                ((op == ZEXT || op == SEXT) && ox.imm0 == oy.imm0)) {
                x = ox.a; y = oy.a;
                continue;
            }
            if (op == BVADD || op == BVSUB || op == BVXOR || op == BVSHL || op == BVLSHR ||
                op == BVMUL || op == CONCAT) {
                const U* bx = const_value(ox.b);
                const U* by = const_value(oy.b);
                if (ox.b == oy.b || (bx && by && *bx == *by)) { x = ox.a; y = oy.a; continue; }
                const U* ax = const_value(ox.a);
                const U* ay = const_value(oy.a);
                if (ox.a == oy.a || (ax && ay && *ax == *ay)) { x = ox.b; y = oy.b; continue; }
            }
            break;
        }
        return {x, y};
    }

    const std::vector<U>& consts_of_width(int w) {
        auto it = consts_by_width.find(w);
        if (it != consts_by_width.end()) return it->second;
        const U m = mask(w);
        std::vector<U> vals;
        for (const U& v : query_consts) vals.push_back(v & m);
        std::sort(vals.begin(), vals.end());
        vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
        std::stable_sort(vals.begin(), vals.end(), [](const U& p, const U& q) {
            const int bp = p.bitlen(), bq = q.bitlen();
            const int gp = bp > 8, gq = bq > 8;
            if (gp != gq) return gp > gq;
            if (bp != bq) return bp > bq;
            return p < q;
        });
        if ((int)vals.size() > kMaxEqConsts) vals.resize(kMaxEqConsts);
        return consts_by_width[w] = std::move(vals);
    }

    const std::vector<uint32_t>& const_ids_of_width(int w) {
        auto it = const_ids_by_width.find(w);
        if (it != const_ids_by_width.end()) return it->second;
        std::vector<uint32_t> ids;
        const U m = mask(w);
        for (const U& k : consts_of_width(w)) ids.push_back(intern(k & m));
        return const_ids_by_width[w] = std::move(ids);
    }

    void harvest(uint32_t root, const Alt* parent, std::vector<std::vector<V>>& pools,
                 std::vector<std::pair<int, const Alts*>>& out_sets,
                 std::vector<std::vector<std::vector<Copy>>>& out_copies) {
        const std::vector<uint32_t> conj = conjuncts(root);
        {   // the query's constants; a query whose conjuncts extend the last one's (LASER order)
            // adds only its new conjuncts' constants to the last set (the same sorted union)
            const bool extends = conj.size() >= last_conj.size() &&
                                 std::equal(last_conj.begin(), last_conj.end(), conj.begin());
            const size_t from = extends ? last_conj.size() : 0;
            std::vector<char> seen(nd.size(), 0);
            std::vector<uint32_t> st(conj.begin() + (long)from, conj.end());
            std::vector<U> qc;
            while (!st.empty()) {
                const uint32_t n = st.back();
                st.pop_back();
                if (seen[n]) continue;
                seen[n] = 1;
                if (nd[n].op == CONST) qc.push_back(pool[nd[n].imm0]);
                const int k = arity(nd[n].op);
                if (k >= 1) st.push_back(nd[n].a);
                if (k >= 2) st.push_back(nd[n].b);
                if (k >= 3) st.push_back(nd[n].c);
            }
            std::sort(qc.begin(), qc.end());
            qc.erase(std::unique(qc.begin(), qc.end()), qc.end());
            if (extends && !last_qc.empty()) {
                std::vector<U> all;
                all.reserve(last_qc.size() + qc.size());
                std::merge(last_qc.begin(), last_qc.end(), qc.begin(), qc.end(),
                           std::back_inserter(all));
                all.erase(std::unique(all.begin(), all.end()), all.end());
                qc.swap(all);
            }
            query_consts = qc;
            last_qc.swap(qc);
            last_conj = conj;
        }
        if (parent && !parent->empty())
            sets.push_back({kProbParent, std::make_shared<const Alts>(Alts{*parent})});
        std::vector<char> seen_eq(nd.size(), 0);
        std::unordered_map<uint32_t, std::tuple<bool, uint32_t, uint32_t,
                                                std::vector<std::vector<Copy>>>> eq_pairs;
        auto replay = [&](const Contribution& c, int prob) {
            for (uint32_t id : c.hints) emit_hint(id);
            if (c.set) sets.push_back({prob, c.set});
        };
        for (uint32_t cj : conj) {
            auto cd = conj_done.find(nk(cj));
            if (cd != conj_done.end()) {
                replay(cd->second, kProbDefault);
            } else {
                Res alts = invert_bool(cj, true);
                Contribution c;
                c.hints = memo_hints(Key{1u, cj, 1u, 0u});
                if (!alts.none && !alts.alts().empty() && !is_only_empty(alts.alts())) {
                    Alts kept;
                    for (const Alt& a : alts.alts()) if (!a.empty()) kept.push_back(a);
                    c.set = std::make_shared<const Alts>(head(kept, kMaxAlts));
                    sets.push_back({kProbDefault, c.set});
                }
                conj_done.emplace(nk(cj), std::move(c));
            }
            auto eqn = eq_nodes_of.find(nk(cj));
            if (eqn == eq_nodes_of.end()) eqn = eq_nodes_of.emplace(nk(cj), eq_nodes(cj)).first;
            for (uint32_t n : eqn->second) {
                if (seen_eq[n]) continue;
                seen_eq[n] = 1;
                auto pit = eq_plan.find(nk(n));
                if (pit == eq_plan.end()) {
                    EqPlan pl;
                    uint32_t x = nd[n].a, y = nd[n].b;
                    if (nd[x].width == 0 || const_value(x) || const_value(y)) {
                        pl.skip = true;
                    } else {
                        std::tie(x, y) = strip_common(x, y);
                        pl.skip = x == y;
                        pl.x = x;
                        pl.y = y;
                        if (!pl.skip) pl.copies = copy_alternatives(x, y);
                    }
                    pit = eq_plan.emplace(nk(n), std::move(pl)).first;
                }
                EqPlan& pl = pit->second;
                if (pl.skip) continue;
                if (!pl.copies.empty()) {
                    if ((int)copy_sets.size() < kMaxSets / 4) copy_sets.push_back(pl.copies);
                    continue;
                }
                const uint32_t x = pl.x, y = pl.y;
                const int w = nd[x].width;
                const std::vector<U>& ks = consts_of_width(w);
                const std::vector<uint32_t>& kids = const_ids_of_width(w);
                const U mw = mask(w);
                const uint32_t mid = intern(mw);
                for (size_t ki = 0; ki < ks.size(); ++ki) {
                    auto bc = pl.by_const.find(kids[ki]);
                    if (bc != pl.by_const.end()) {
                        replay(bc->second, kProbDefault / 2);
                        continue;
                    }
                    const U& k = ks[ki];
                    Res rx = invert_bits_ids(x, kids[ki], mid, k, mw);
                    Res ry = invert_bits_ids(y, kids[ki], mid, k, mw);
                    Contribution c;
                    c.hints = memo_hints(Key{0u, x, kids[ki], mid});
                    const std::vector<uint32_t> hy = memo_hints(Key{0u, y, kids[ki], mid});
                    c.hints.insert(c.hints.end(), hy.begin(), hy.end());
                    if (!rx.none && !rx.alts().empty() && !ry.none && !ry.alts().empty()) {
                        Alts both = merge(rx.alts(), ry.alts());
                        if (!both.empty() && !is_only_empty(both)) {
                            c.set = std::make_shared<const Alts>(head(both, kMaxAlts));
                            sets.push_back({kProbDefault / 2, c.set});
                        }
                    }
                    pl.by_const.emplace(kids[ki], std::move(c));
                }
                if ((int)sets.size() >= kMaxSets) break;
            }
            if ((int)sets.size() >= kMaxSets) break;
        }
        // bounds on one term from several conjuncts (calldatasize guards, argument range
        // checks): values inside their intersection, last, so they override the single-bound
        // boundary values (candidates.py harvest, _intervals / _interval_values)
        for (const Interval& iv : intervals(conj)) {
            if (iv.n < 2 || iv.empty || (int)sets.size() >= kMaxSets) continue;
            const int w = nd[iv.t].width;
            Alts out;
            for (const U& v : interval_values(iv.lo, iv.hi)) {
                Res r = invert_bits(iv.t, v, mask(w));
                if (!r.none && !r.alts().empty())
                    for (const Alt& a : r.alts()) if (!a.empty()) out.push_back(a);
            }
            if (!out.empty())
                sets.push_back({kProbDefault, std::make_shared<const Alts>(head(out, kMaxAlts))});
        }
        out_sets.clear();
        const bool first_parent = parent && !parent->empty() && !sets.empty();
        if (first_parent) out_sets.push_back({sets[0].first, sets[0].second.get()});
        for (uint32_t id : prune_hints()) out_sets.push_back({kProbHint, &hint_alts[id]});
        for (size_t i = first_parent ? 1 : 0; i < sets.size(); ++i)
            out_sets.push_back({sets[i].first, sets[i].second.get()});
        pools.assign(n_cols, {});
        // first occurrences in order, at most kMaxPool per column; the duplicate test compares
        // a 64-bit digest of each value before the value itself (a long path's sets repeat values)
        pool_digest.assign((size_t)n_cols * kMaxPool, 0);
        auto add_pool = [&](uint32_t c, const V& v) {
            auto& p = pools[c];
            const size_t n = p.size();
            if ((int)n >= kMaxPool) return;
            uint64_t h = 0x9E3779B97F4A7C15ull;
            for (int k = 0; k < 8; ++k) h = (h ^ v.w[k]) * 0x100000001B3ull;
            uint64_t* dg = pool_digest.data() + (size_t)c * kMaxPool;
            for (size_t i = 0; i < n; ++i)
                if (dg[i] == h && p[i] == v) return;
            dg[n] = h;
            p.push_back(v);
        };
        for (const auto& s : out_sets)
            for (const Alt& a : *s.second)
                for (const auto& kv : a) add_pool(kv.first, kv.second);
        for (uint32_t c = 0; c < n_cols; ++c) {
            const int w = widths[c];
            for (const U& v : {U::of(0), U::of(1), mask(w), shl(U::of(1), w - 1)}) add_pool(c, lo256(v));
        }
        if ((int)out_sets.size() > kMaxSets) out_sets.resize(kMaxSets);
        out_copies = copy_sets;
        if ((int)out_copies.size() > kMaxSets / 4) out_copies.resize(kMaxSets / 4);
    }

    // candidates.py _bound_of: conjunct n bounds a symbolic term to [lo, hi] (unsigned,
    // inclusive) against a constant -- ULT / ULE / UGT / UGE either way round, their negations,
    // and Or(x < k, x == k) (smt.ULE / smt.UGE); false otherwise
    struct Interval { uint32_t t; U lo, hi; int n; bool empty; };
    bool bound_of(uint32_t n, uint32_t& t, U& lo, U& hi, bool& empty) {
        uint8_t op = nd[n].op;
        uint32_t a = nd[n].a, b = nd[n].b;
        bool truth = true;
        if (op == NOT) {
            truth = false;
            op = nd[a].op;
            b = nd[a].b;
            a = nd[a].a;
        }
        if (op == OR) {  // Or(cmp(x, k), x == k): the non-strict comparison
            const Node& l = nd[a];
            const Node& r = nd[b];
            if (r.op != EQ || (l.op != BVULT && l.op != BVUGT) || l.a != r.a || l.b != r.b)
                return false;
            op = l.op == BVULT ? BVULE : BVUGE;
            a = l.a;
            b = l.b;
        }
        if (op != BVULT && op != BVULE && op != BVUGT && op != BVUGE) return false;
        const U* ka = const_value(a);
        const U* kb = const_value(b);
        if ((ka == nullptr) == (kb == nullptr)) return false;
        bool less = op == BVULT || op == BVULE;
        bool strict = op == BVULT || op == BVUGT;
        t = kb ? a : b;
        const U k = kb ? *kb : *ka;
        if (!kb) less = !less;
        if (!truth) { less = !less; strict = !strict; }
        const U m = mask(nd[t].width);
        empty = false;
        if (less) {
            lo = U::of(0);
            if (strict && k == U::of(0)) empty = true;
            hi = strict ? k - U::of(1) : k;
        } else {
            if (strict && k == m) empty = true;
            lo = strict ? k + U::of(1) : k;
            hi = m;
        }
        return true;
    }
    std::vector<Interval> intervals(const std::vector<uint32_t>& conj) {
        std::vector<Interval> out;
        std::unordered_map<uint32_t, size_t> at;
        for (uint32_t cj : conj) {
            uint32_t t;
            U lo, hi;
            bool empty;
            if (!bound_of(cj, t, lo, hi, empty)) continue;
            auto it = at.find(t);
            if (it == at.end()) {
                at.emplace(t, out.size());
                out.push_back(Interval{t, lo, hi, 1, empty});
            } else {
                Interval& iv = out[it->second];
                if (iv.lo < lo) iv.lo = lo;
                if (hi < iv.hi) iv.hi = hi;
                iv.empty = iv.empty || empty;
                ++iv.n;
            }
        }
        for (Interval& iv : out) if (iv.hi < iv.lo) iv.empty = true;
        return out;
    }
    // candidates.py _interval_values: both ends, the middle, lo + 1 (distinct, in order)
    static std::vector<U> interval_values(const U& lo, const U& hi) {
        std::vector<U> out;
        const U cand[4] = {lo, hi, lo + shr(hi - lo, 1), lo + U::of(1)};
        for (const U& v : cand) {
            if (v < lo || hi < v) continue;
            bool dup = false;
            for (const U& x : out) dup = dup || x == v;
            if (!dup) out.push_back(v);
        }
        return out;
    }

    // candidates.py _prune_hints: per column, of the single-column hint sets only the
    // kHintsPerColumn with the largest and with the smallest values stay (in their order)
    std::vector<uint32_t> prune_hints() const {
        std::map<uint32_t, std::vector<size_t>> by_col;
        for (size_t i = 0; i < hints.size(); ++i)
            if (hint_col[hints[i]] >= 0) by_col[(uint32_t)hint_col[hints[i]]].push_back(i);
        std::vector<char> drop(hints.size(), 0);
        for (auto& kv : by_col) {
            const std::vector<size_t>& idx = kv.second;
            if ((int)idx.size() <= 2 * kHintsPerColumn) continue;
            // extremes per hint, indexed by position in idx (not by hint: one column's hints)
            std::vector<V> hi_v(idx.size()), lo_v(idx.size());
            for (size_t j = 0; j < idx.size(); ++j) {
                hi_v[j] = hint_hi[hints[idx[j]]];
                lo_v[j] = hint_lo[hints[idx[j]]];
            }
            std::vector<size_t> hi(idx.size()), lo(idx.size());
            for (size_t j = 0; j < idx.size(); ++j) hi[j] = lo[j] = j;
            std::stable_sort(hi.begin(), hi.end(), [&](size_t p, size_t q) { return hi_v[q] < hi_v[p]; });
            std::stable_sort(lo.begin(), lo.end(), [&](size_t p, size_t q) { return lo_v[p] < lo_v[q]; });
            for (size_t i : idx) drop[i] = 1;
            for (int j = 0; j < kHintsPerColumn; ++j) drop[idx[hi[j]]] = drop[idx[lo[j]]] = 0;
        }
        std::vector<uint32_t> out;
        for (size_t i = 0; i < hints.size(); ++i) if (!drop[i]) out.push_back(hints[i]);
        return out;
    }
};

}  // namespace

struct mh_harvest {  // owns the arrays an mh_guide from mh_guide_harvest points into
    std::vector<uint32_t> pool_off, pool, set_off, alt_off, entry_col, entry_val;
    std::vector<uint8_t> set_prob;
    std::vector<uint16_t> width16;
};

int32_t mh_detail_set_err(int32_t code, const char* msg);  // capi.cpp

namespace {

// Append the tape nodes, constants and column widths beyond what h holds (a fresh harvester holds
// none), harvest, and fill *out / *guide.
int32_t harvest_into(Harvester& h, const mh_node* nodes, uint32_t n_nodes, const uint32_t* consts,
                     uint32_t n_consts, const uint16_t* col_width, uint32_t n_cols,
                     const uint32_t* parent_cols, const uint32_t* parent_vals, uint32_t n_parent,
                     mh_harvest** out, mh_guide* guide) {
    const uint32_t n0 = (uint32_t)h.nd.size();
    h.nd.resize(n_nodes);
    h.gen.resize(n_nodes, h.cur_gen);
    for (uint32_t i = n0; i < n_nodes; ++i) {
        const mh_node& s = nodes[i];
        Node& d = h.nd[i];
        d.op = s.op; d.width = s.width; d.a = s.a; d.b = s.b; d.c = s.c;
        d.imm0 = s.imm0; d.imm1 = s.imm1;
        const int k = Harvester::arity(s.op);
        if (s.width > 1088 || (k >= 1 && s.a >= i) || (k >= 2 && s.b >= i) ||
            (k >= 3 && s.c >= i) || (s.op == CONST && s.imm0 >= n_consts) ||
            (s.op == EXTRACT && (s.imm1 > s.imm0 || s.imm0 >= 1088)) ||
            ((s.op == ZEXT || s.op == SEXT) && s.imm0 > 1088))
            return mh_detail_set_err(MH_E_INVALID, "malformed tape node");
        // bit-layout operands are bit-vectors (the harvest reads their top bit / width)
        if ((s.op == EXTRACT || s.op == ZEXT || s.op == SEXT || s.op == CONCAT) &&
            (h.nd[s.a].width == 0 || (s.op == CONCAT && h.nd[s.b].width == 0)))
            return mh_detail_set_err(MH_E_INVALID, "bit-layout op over a Bool operand");
    }
    const uint32_t c0 = (uint32_t)h.pool.size();
    h.pool.resize(n_consts);
    for (uint32_t i = c0; i < n_consts; ++i)
        for (int k = 0; k < 8; ++k) h.pool[i].w[k] = consts[8ull * i + k];
    h.cv_state.resize(n_nodes, 0);
    h.cv.resize(n_nodes);
    h.n_cols = n_cols;
    h.widths.assign(col_width, col_width + n_cols);
    for (uint16_t w : h.widths)
        if (w < 1 || w > 256) return mh_detail_set_err(MH_E_INVALID, "column width not 1..256");
    Alt parent;
    for (uint32_t i = 0; i < n_parent; ++i) {
        if (parent_cols[i] >= n_cols)
            return mh_detail_set_err(MH_E_INVALID, "parent column out of range");
        V v;
        for (int k = 0; k < 8; ++k) v.w[k] = parent_vals[8ull * i + k];
        parent.push_back({parent_cols[i], v});
        if (h.peval) {  // a later pair of one column wins, as in the parent set
            U u = U::of(0);
            for (int k = 0; k < 8; ++k) u.w[k] = v.w[k];
            h.parent_of[parent_cols[i]] = u;
        }
    }
    std::vector<std::vector<V>> pools;
    std::vector<std::pair<int, const Alts*>> sets;
    std::vector<std::vector<std::vector<Copy>>> copies;
    h.harvest(n_nodes - 1, n_parent ? &parent : nullptr, pools, sets, copies);
    auto r = std::make_unique<mh_harvest>();
    r->width16.assign(h.widths.begin(), h.widths.end());
    // sized exactly first (a long path's guide holds thousands of entries), then written in place
    size_t n_pool = 0, n_alt = 0, n_ent = 0;
    for (const auto& p : pools) n_pool += p.size();
    for (const auto& s : sets) {
        n_alt += s.second->size();
        for (const Alt& a : *s.second) n_ent += a.size();
    }
    for (const auto& alts : copies) {
        n_alt += alts.size();
        for (const auto& alt : alts) n_ent += alt.size();
    }
    r->pool_off.resize(pools.size() + 1);
    r->pool.resize(8 * n_pool);
    r->set_off.resize(sets.size() + copies.size() + 1);
    r->set_prob.resize(sets.size() + copies.size());
    r->alt_off.resize(n_alt + 1);
    r->entry_col.resize(n_ent);
    r->entry_val.resize(8 * n_ent);
    uint32_t* pv = r->pool.data();
    r->pool_off[0] = 0;
    for (size_t c = 0; c < pools.size(); ++c) {
        for (const V& v : pools[c]) { memcpy(pv, v.w, sizeof v.w); pv += 8; }
        r->pool_off[c + 1] = (uint32_t)((pv - r->pool.data()) / 8);
    }
    uint32_t* ec = r->entry_col.data();
    uint32_t* ev = r->entry_val.data();
    uint32_t* ao = r->alt_off.data();
    uint32_t ne = 0, na = 0, ns = 0;
    *ao++ = 0;
    r->set_off[0] = 0;
    for (const auto& s : sets) {
        r->set_prob[ns] = (uint8_t)s.first;
        for (const Alt& a : *s.second) {
            for (const auto& kv : a) {
                ec[ne] = kv.first;
                memcpy(ev + 8ull * ne, kv.second.w, sizeof kv.second.w);
                ++ne;
            }
            *ao++ = ne;
            ++na;
        }
        r->set_off[++ns] = na;
    }
    for (const auto& alts : copies) {
        r->set_prob[ns] = (uint8_t)kProbDefault;
        for (const auto& alt : alts) {
            for (const Copy& c : alt) {
                ec[ne] = c.dst | kCopyFlag;
                const uint32_t w[8] = {c.src, (uint32_t)c.dlo, (uint32_t)c.slo, (uint32_t)c.nb,
                                       0, 0, 0, 0};
                memcpy(ev + 8ull * ne, w, sizeof w);
                ++ne;
            }
            *ao++ = ne;
            ++na;
        }
        r->set_off[++ns] = na;
    }
    const uint32_t n_sets = (uint32_t)r->set_prob.size();
    // never-empty arrays, as candidates.Guide.arrays() gives them (one zero entry)
    if (r->pool.empty()) r->pool.assign(8, 0);
    if (r->set_prob.empty()) r->set_prob.push_back(0);
    if (r->entry_col.empty()) r->entry_col.push_back(0);
    if (r->entry_val.empty()) r->entry_val.assign(8, 0);
    guide->n_cols = n_cols;
    guide->col_width = r->width16.data();
    guide->pool_off = r->pool_off.data();
    guide->pool = r->pool.data();
    guide->n_sets = n_sets;
    guide->set_prob = r->set_prob.data();
    guide->set_off = r->set_off.data();
    guide->alt_off = r->alt_off.data();
    guide->entry_col = r->entry_col.data();
    guide->entry_val = r->entry_val.data();
    *out = r.release();
    return MH_OK;
}

bool check_args(const mh_node* nodes, uint32_t n_nodes, const uint32_t* consts, uint32_t n_consts,
                const uint16_t* col_width, uint32_t n_cols, const uint32_t* parent_cols,
                const uint32_t* parent_vals, uint32_t n_parent) {
    return nodes && n_nodes && (!n_consts || consts) && (!n_cols || col_width) &&
           (!n_parent || (parent_cols && parent_vals));
}

}  // namespace

// A harvester kept across the queries of a path: when a query's tape, constants and column widths
// extend the last query's (a child of a LASER state whose constraint left its parent's lowering
// as it was, query.cpp), the memoised inversions, interned values and hint ids of the earlier
// queries stay valid (they are functions of the tape prefix) and only the new conjuncts are
// inverted afresh; the guide is the one mh_guide_harvest gives (tests/test_harvest.py).
struct mh_harvester {
    Arena arena;
    std::unique_ptr<Harvester> h;
    std::vector<mh_node> nodes;
    std::vector<uint32_t> consts;
    std::vector<uint16_t> widths;
    uint64_t reused = 0, fresh = 0;
};

namespace {
constexpr size_t kSessionArenaBytes = (size_t)256 << 20;  // start afresh beyond this
struct UseArena {  // ArenaAlloc draws from `a` while in scope
    Arena* prev;
    explicit UseArena(Arena* a) : prev(g_cur) { g_cur = a; }
    ~UseArena() { g_cur = prev; }
};
}  // namespace

extern "C" int32_t mh_guide_harvest(const mh_node* nodes, uint32_t n_nodes, const uint32_t* consts,
                                    uint32_t n_consts, const uint16_t* col_width, uint32_t n_cols,
                                    const uint32_t* parent_cols, const uint32_t* parent_vals,
                                    uint32_t n_parent, mh_harvest** out, mh_guide* guide) {
    if (!out || !guide) return mh_detail_set_err(MH_E_INVALID, "null out pointer");
    *out = nullptr;
    if (!check_args(nodes, n_nodes, consts, n_consts, col_width, n_cols, parent_cols, parent_vals,
                    n_parent))
        return mh_detail_set_err(MH_E_INVALID, "null or empty argument");
    try {
        UseArena use(&g_arena);
        struct ArenaReset {  // declared first: runs after every arena-backed local is gone
            ~ArenaReset() { g_arena.reset(); }
        } arena_reset;
        Harvester h;
        return harvest_into(h, nodes, n_nodes, consts, n_consts, col_width, n_cols, parent_cols,
                            parent_vals, n_parent, out, guide);
    } catch (const std::bad_alloc&) {
        return mh_detail_set_err(MH_E_NOMEM, "host allocation failed");
    }
}

// mh_guide_harvest with the parent witness fixing what it can evaluate (Harvester::peval): the
// incremental round's guide (sieve.newest_tape), stateless like mh_guide_harvest.
extern "C" int32_t mh_guide_harvest_inc(const mh_node* nodes, uint32_t n_nodes,
                                        const uint32_t* consts, uint32_t n_consts,
                                        const uint16_t* col_width, uint32_t n_cols,
                                        const uint32_t* parent_cols, const uint32_t* parent_vals,
                                        uint32_t n_parent, mh_harvest** out, mh_guide* guide) {
    if (!out || !guide) return mh_detail_set_err(MH_E_INVALID, "null out pointer");
    *out = nullptr;
    if (!check_args(nodes, n_nodes, consts, n_consts, col_width, n_cols, parent_cols, parent_vals,
                    n_parent))
        return mh_detail_set_err(MH_E_INVALID, "null or empty argument");
    try {
        UseArena use(&g_arena);
        struct ArenaReset {
            ~ArenaReset() { g_arena.reset(); }
        } arena_reset;
        Harvester h;
        h.peval = true;
        return harvest_into(h, nodes, n_nodes, consts, n_consts, col_width, n_cols, parent_cols,
                            parent_vals, n_parent, out, guide);
    } catch (const std::bad_alloc&) {
        return mh_detail_set_err(MH_E_NOMEM, "host allocation failed");
    }
}

extern "C" int32_t mh_harvester_create(mh_harvester** out) {
    if (!out) return mh_detail_set_err(MH_E_INVALID, "null out pointer");
    *out = new (std::nothrow) mh_harvester();
    return *out ? MH_OK : mh_detail_set_err(MH_E_NOMEM, "mh_harvester_create");
}

extern "C" int32_t mh_harvester_destroy(mh_harvester* s) {
    if (!s) return mh_detail_set_err(MH_E_INVALID, "null harvester");
    {
        UseArena use(&s->arena);
        s->h.reset();
    }
    delete s;
    return MH_OK;
}

extern "C" int32_t mh_harvester_stats(const mh_harvester* s, uint64_t* out /* [3] */) {
    if (!s || !out) return mh_detail_set_err(MH_E_INVALID, "null argument");
    out[0] = s->reused;
    out[1] = s->fresh;
    out[2] = s->arena.used();
    return MH_OK;
}

extern "C" int32_t mh_guide_harvest_with(mh_harvester* s, const mh_node* nodes, uint32_t n_nodes,
                                         const uint32_t* consts, uint32_t n_consts,
                                         const uint16_t* col_width, uint32_t n_cols,
                                         const uint32_t* parent_cols, const uint32_t* parent_vals,
                                         uint32_t n_parent, mh_harvest** out, mh_guide* guide) {
    if (!s || !out || !guide) return mh_detail_set_err(MH_E_INVALID, "null argument");
    *out = nullptr;
    if (!check_args(nodes, n_nodes, consts, n_consts, col_width, n_cols, parent_cols, parent_vals,
                    n_parent))
        return mh_detail_set_err(MH_E_INVALID, "null or empty argument");
    UseArena use(&s->arena);
    try {
        const size_t pn = s->nodes.size(), pc = s->consts.size() / 8, pw = s->widths.size();
        const bool extends = s->h && n_nodes >= pn && n_consts >= pc && n_cols >= pw &&
                             s->arena.used() < kSessionArenaBytes &&
                             memcmp(nodes, s->nodes.data(), pn * sizeof(mh_node)) == 0 &&
                             memcmp(consts, s->consts.data(), pc * 32) == 0 &&
                             memcmp(col_width, s->widths.data(), pw * sizeof(uint16_t)) == 0;
        // otherwise the longest prefix of nodes the two tapes share whose constants and columns
        // are in the prefixes of constants and column widths they share (the other branch of a
        // JUMPI: the path's tape, then other nodes): kept when it is most of the new tape
        uint32_t keep = 0, keep_c = 0;
        if (!extends && s->h && s->arena.used() < kSessionArenaBytes) {
            const size_t mn = std::min<size_t>(pn, n_nodes);
            size_t p = 0;
            while (p < mn && memcmp(&nodes[p], &s->nodes[p], sizeof(mh_node)) == 0) ++p;
            const size_t mc = std::min<size_t>(pc, n_consts), mw = std::min<size_t>(pw, n_cols);
            size_t qc = 0, qw = 0;
            while (qc < mc && memcmp(consts + 8 * qc, s->consts.data() + 8 * qc, 32) == 0) ++qc;
            while (qw < mw && col_width[qw] == s->widths[qw]) ++qw;
            for (size_t i = 0; i < p; ++i)
                if ((nodes[i].op == CONST && nodes[i].imm0 >= qc) ||
                    (nodes[i].op == VAR && nodes[i].imm0 >= qw)) {
                    p = i;
                    break;
                }
            if (p >= 16 && 2 * p >= n_nodes) {
                keep = (uint32_t)p;
                keep_c = (uint32_t)qc;
            }
        }
        if (extends) {
            s->h->begin_query();
            ++s->reused;
        } else if (keep) {
            s->h->truncate(keep, keep_c);
            s->h->begin_query();
            ++s->reused;
        } else {
            s->h.reset();
            s->arena.reset();
            s->h.reset(new Harvester());
            ++s->fresh;
        }
        s->nodes.assign(nodes, nodes + n_nodes);
        s->consts.assign(consts, consts + 8ull * n_consts);
        s->widths.assign(col_width, col_width + n_cols);
        const int32_t r = harvest_into(*s->h, nodes, n_nodes, consts, n_consts, col_width, n_cols,
                                       parent_cols, parent_vals, n_parent, out, guide);
        if (r != MH_OK) {  // a malformed tape leaves nothing to extend
            s->h.reset();
            s->nodes.clear();
        }
        return r;
    } catch (const std::bad_alloc&) {
        s->h.reset();
        s->nodes.clear();
        return mh_detail_set_err(MH_E_NOMEM, "host allocation failed");
    }
}

extern "C" int32_t mh_harvest_free(mh_harvest* h) {
    delete h;
    return MH_OK;
}
