// SMT-LIB2 reader session behind the C-ABI (mh_smtlib_*): the import stage of the product path.
//
// Under the plugin every constraint LASER hands get_model (mythril/support/model.py:37-57,
// laser/smt/solver/solver.py:28-37) is a z3 term, imported through z3's Solver.sexpr() text into
// the sieve's term store (mythril_amd/smtlib.py Z3Importer).  Reading that text in Python cost
// 0.1-3.4 ms per new constraint (the tokenizer plus one hash-consing builder call per
// token occurrence, shared sub-terms included).  This reader parses the same fragment as
// smtlib.Reader and hash-conses against a mirror of the nodes it has already handed to the host:
// a read returns only the nodes the host does not have yet (records, operands either host ids or
// earlier records of the same read), and the host answers with the ids its builder gave them
// (mh_smtlib_commit).  A constraint that extends its parent's shares almost all nodes with it, so
// the host side touches only the few new ones.
//
// Semantics are the Python reader's, rule for rule (tests/test_smtlib_native.py compares the two
// on every LASER-shaped query and the z3-style texts): n-ary and/or/=/distinct folded left, `=>`
// as (or (not a) b), bvcomp as ite, rotates / repeat as extract + concat, z3's BVAddNoOverflow
// expansion recognised back into BVADD_NOOVFL_U, Bool constants as (= v #b1), constants over 256
// bits as CONCATs of 256-bit pool entries.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "../../include/mythril_hip.h"

int32_t mh_detail_set_err(int32_t code, const char* msg);  // capi.cpp

namespace {

enum : uint8_t {
    OP_CONST = 0, OP_VAR = 1, OP_TRUE = 2, OP_FALSE = 3,
    OP_BVADD = 10, OP_BVSUB = 11, OP_BVMUL = 12, OP_BVUDIV = 13, OP_BVUREM = 14, OP_BVSDIV = 15,
    OP_BVSREM = 16, OP_BVSMOD = 17, OP_BVNEG = 18, OP_BVNOT = 19, OP_BVAND = 20, OP_BVOR = 21,
    OP_BVXOR = 22, OP_BVSHL = 23, OP_BVLSHR = 24, OP_BVASHR = 25,
    OP_EQ = 30, OP_BVULT = 31, OP_BVULE = 32, OP_BVUGT = 33, OP_BVUGE = 34, OP_BVSLT = 35,
    OP_BVSLE = 36, OP_BVSGT = 37, OP_BVSGE = 38,
    OP_AND = 40, OP_OR = 41, OP_XOR = 42, OP_NOT = 43, OP_ITE = 45,
    OP_EXTRACT = 50, OP_CONCAT = 51, OP_ZEXT = 52, OP_SEXT = 53,
    OP_ADD_NOOVFL = 61, OP_MUL_NOOVFL = 62,
    OP_ARRAY = 80, OP_CONST_ARRAY = 81, OP_STORE = 82, OP_SELECT = 83, OP_UF = 84,
};
constexpr uint32_t MAX_WIDTH = 1088;

struct Fail {
    std::string msg;
};
[[noreturn]] void fail(const std::string& m) { throw Fail{m}; }

// ---- tokens -------------------------------------------------------------------------------
// The text is tokenized once into a flat array; a '(' token records the index of its ')', so a
// list is a token range and the parser walks indices (no tree, no per-atom allocation).
enum : uint8_t { T_LP, T_RP, T_ATOM, T_QATOM, T_STR };
struct Tok {
    uint8_t type;
    uint32_t off, len;
    uint32_t match;  // T_LP: index of the matching T_RP
};

void tokenize(const char* p, size_t n, std::vector<Tok>& out) {
    out.clear();
    std::vector<uint32_t> open;
    size_t i = 0;
    while (i < n) {
        const char c = p[i];
        if (c == ';') {
            while (i < n && p[i] != '\n') ++i;
            continue;
        }
        if (c == ' ' || c == '\t' || c == '\n' || c == '\r') { ++i; continue; }
        if (c == '(') {
            open.push_back((uint32_t)out.size());
            out.push_back(Tok{T_LP, (uint32_t)i, 1, 0});
            ++i;
            continue;
        }
        if (c == ')') {
            if (open.empty()) fail("unbalanced ')'");
            out[open.back()].match = (uint32_t)out.size();
            open.pop_back();
            out.push_back(Tok{T_RP, (uint32_t)i, 1, 0});
            ++i;
            continue;
        }
        if (c == '|') {
            const char* q = static_cast<const char*>(memchr(p + i + 1, '|', n - i - 1));
            if (!q) fail("unterminated |symbol|");
            const size_t e = (size_t)(q - p);
            out.push_back(Tok{T_QATOM, (uint32_t)(i + 1), (uint32_t)(e - i - 1), 0});
            i = e + 1;
            continue;
        }
        if (c == '"') {
            size_t q = i + 1;
            for (;;) {
                if (q >= n) fail("unterminated string");
                if (p[q] == '"') {
                    if (q + 1 < n && p[q + 1] == '"') { q += 2; continue; }
                    break;
                }
                ++q;
            }
            out.push_back(Tok{T_STR, (uint32_t)i, (uint32_t)(q + 1 - i), 0});
            i = q + 1;
            continue;
        }
        size_t q = i;
        while (q < n && p[q] != ' ' && p[q] != '\t' && p[q] != '\n' && p[q] != '\r' &&
               p[q] != '(' && p[q] != ')' && p[q] != '|' && p[q] != '"' && p[q] != ';')
            ++q;
        out.push_back(Tok{T_ATOM, (uint32_t)i, (uint32_t)(q - i), 0});
        i = q;
    }
    if (!open.empty()) fail("unbalanced '('");
}

// ---- nodes --------------------------------------------------------------------------------
struct Node {
    uint8_t op;
    uint8_t is_array;
    uint32_t width;  // 0 = Bool; array: range width
    int32_t a, b, c;
    uint32_t imm0, imm1;  // array: imm1 = domain
    int32_t sym;          // VAR / ARRAY / UF: symbol string index
    int32_t cidx;         // CONST: value index
    int64_t host;         // the host builder's id, -1 until committed
};

struct Key {
    uint8_t op;
    uint32_t width, imm0, imm1;
    int32_t a, b, c, sym, cidx;
    bool operator==(const Key& o) const {
        return op == o.op && width == o.width && imm0 == o.imm0 && imm1 == o.imm1 && a == o.a &&
               b == o.b && c == o.c && sym == o.sym && cidx == o.cidx;
    }
};
struct KeyHash {
    size_t operator()(const Key& k) const {
        uint64_t h = 0x9E3779B97F4A7C15ull ^ k.op;
        auto mix = [&](uint64_t v) { h ^= v + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2); };
        mix(k.width); mix(k.imm0); mix(k.imm1); mix((uint32_t)k.a); mix((uint32_t)k.b);
        mix((uint32_t)k.c); mix((uint32_t)k.sym); mix((uint32_t)k.cidx);
        return (size_t)h;
    }
};

struct Sort {
    char kind = 'b';  // 'B' Bool, 'b' bit-vector, 'a' array
    uint32_t width = 0, domain = 0;
};

struct Decl {
    bool fun;
    Sort sort, dom;
    int32_t node = -1;  // a constant's term, once built (cleared when a failed read rolls back)
};

struct ConstVal {  // little-endian u32 limbs, width <= 256
    uint32_t l[8];
    uint32_t width;
    bool operator==(const ConstVal& o) const {
        return width == o.width && std::memcmp(l, o.l, sizeof l) == 0;
    }
};
struct ConstHash {
    size_t operator()(const ConstVal& v) const {
        uint64_t h = 1469598103934665603ull ^ v.width;
        for (uint32_t x : v.l) h = (h ^ x) * 1099511628211ull;
        return (size_t)h;
    }
};

}  // namespace

struct mh_smtlib {
    std::vector<Node> nodes;
    std::unordered_map<Key, int32_t, KeyHash> memo;
    // names live in `names_store` (stable addresses); the maps key string_views into it, so a
    // lookup with a view into the text allocates nothing
    std::deque<std::string> names_store;
    std::vector<std::string_view> syms;
    std::unordered_map<std::string_view, int32_t> sym_index;
    std::vector<ConstVal> consts;
    std::unordered_map<ConstVal, int32_t, ConstHash> const_index;
    std::unordered_map<std::string_view, Decl> decls;
    std::unordered_map<std::string_view, int32_t> defs;
    std::unordered_map<std::string_view, int32_t> literals;  // literal text -> its CONST term

    std::string_view own(std::string_view v) {
        names_store.emplace_back(v);
        return names_store.back();
    }
    // the last read: records (nodes new to the host) and command results, owned until next read
    size_t first_new = 0;
    std::vector<mh_smt_record> recs;
    std::vector<uint32_t> rec_consts;
    std::string rec_names;
    std::vector<mh_smt_result> results;
    std::vector<Tok> toks;
    bool pending = false;
    // undo log of the current read: (is_def, name, had_old, old decl / def)
    struct Undo { bool def; std::string_view name; bool had; Decl decl; int32_t node; };
    std::vector<Undo> undo;

    void set_decl(std::string_view name, const Decl& d) {
        auto it = decls.find(name);
        if (it == decls.end()) {
            const std::string_view k = own(name);
            undo.push_back(Undo{false, k, false, Decl{}, 0});
            decls.emplace(k, d);
        } else {
            undo.push_back(Undo{false, it->first, true, it->second, 0});
            it->second = d;
        }
    }
    void set_def(std::string_view name, int32_t n) {
        auto it = defs.find(name);
        if (it == defs.end()) {
            const std::string_view k = own(name);
            undo.push_back(Undo{true, k, false, Decl{}, 0});
            defs.emplace(k, n);
        } else {
            undo.push_back(Undo{true, it->first, true, Decl{}, it->second});
            it->second = n;
        }
    }
    // after a rollback: no cached term may name a node that is gone
    void drop_caches() {
        literals.clear();
        for (auto& kv : decls) kv.second.node = -1;
    }
    void undo_all() {
        for (size_t i = undo.size(); i-- > 0;) {
            const Undo& u = undo[i];
            if (u.def) {
                if (u.had) defs[u.name] = u.node; else defs.erase(u.name);
            } else {
                if (u.had) decls[u.name] = u.decl; else decls.erase(u.name);
            }
        }
        undo.clear();
    }

    int32_t sym(std::string_view s) {
        auto it = sym_index.find(s);
        if (it != sym_index.end()) return it->second;
        const int32_t i = (int32_t)syms.size();
        const std::string_view k = own(s);
        syms.push_back(k);
        sym_index.emplace(k, i);
        return i;
    }

    int32_t add(uint8_t op, uint32_t width, int32_t a = -1, int32_t b = -1, int32_t c = -1,
                uint32_t imm0 = 0, uint32_t imm1 = 0, int32_t sy = -1, int32_t ci = -1,
                bool arr = false) {
        const Key k{op, width, imm0, imm1, a, b, c, sy, ci};
        auto it = memo.find(k);
        if (it != memo.end()) return it->second;
        const int32_t i = (int32_t)nodes.size();
        nodes.push_back(Node{op, (uint8_t)arr, width, a, b, c, imm0, imm1, sy, ci, -1});
        memo.emplace(k, i);
        return i;
    }

    bool is_bool(int32_t n) const { return nodes[n].width == 0 && !nodes[n].is_array; }
    bool is_arr(int32_t n) const { return nodes[n].is_array != 0; }
    uint32_t w(int32_t n) const { return nodes[n].width; }

    // -- constructors with the host builder's sort rules (tape.py TapeBuilder.op) --
    int32_t konst(const uint32_t* limbs, uint32_t width) {
        if (width < 1 || width > MAX_WIDTH) fail("constants are 1..1088 bits wide");
        if (width > 256) {  // CONCAT(const(value >> 256, width - 256), const(low 256 bits))
            const int32_t lo = konst(limbs, 256);
            const int32_t hi = konst(limbs + 8, width - 256);
            return op2(OP_CONCAT, hi, lo);
        }
        ConstVal v{};
        for (uint32_t k = 0; k < 8; ++k) v.l[k] = k * 32 < width ? limbs[k] : 0u;
        if (width % 32) v.l[width / 32] &= (1u << (width % 32)) - 1u;
        v.width = width;
        int32_t ci;
        auto it = const_index.find(v);
        if (it != const_index.end()) {
            ci = it->second;
        } else {
            ci = (int32_t)consts.size();
            consts.push_back(v);
            const_index.emplace(v, ci);
        }
        return add(OP_CONST, width, -1, -1, -1, 0, 0, -1, ci);
    }
    int32_t konst_u(uint64_t v, uint32_t width) {
        uint32_t l[34] = {};
        l[0] = (uint32_t)v;
        l[1] = (uint32_t)(v >> 32);
        return konst(l, width);
    }
    int32_t tru() { return add(OP_TRUE, 0); }
    int32_t fals() { return add(OP_FALSE, 0); }
    int32_t var(std::string_view name, uint32_t width) {
        if (width < 1 || width > 256) fail("variables are 1..256 bits wide");
        return add(OP_VAR, width, -1, -1, -1, 0, 0, sym(name));
    }
    int32_t array(std::string_view name, uint32_t dom, uint32_t rng) {
        return add(OP_ARRAY, rng, -1, -1, -1, 0, dom, sym(name), -1, true);
    }
    int32_t const_array(uint32_t dom, int32_t dflt) {
        if (is_arr(dflt) || is_bool(dflt)) fail("K needs a bit-vector default");
        return add(OP_CONST_ARRAY, w(dflt), dflt, -1, -1, 0, dom, -1, -1, true);
    }
    int32_t store(int32_t arr, int32_t key, int32_t val) {
        if (!is_arr(arr)) fail("store into a non-array");
        const uint32_t dom = nodes[arr].imm1, rng = w(arr);
        if (is_arr(key) || is_arr(val) || w(key) != dom || w(val) != rng || is_bool(key) ||
            is_bool(val))
            fail("store sort mismatch");
        return add(OP_STORE, rng, arr, key, val, 0, dom, -1, -1, true);
    }
    int32_t select(int32_t arr, int32_t idx) {
        if (!is_arr(arr)) fail("select from a non-array");
        if (is_arr(idx) || w(idx) != nodes[arr].imm1) fail("select index width mismatch");
        return add(OP_SELECT, w(arr), arr, idx);
    }
    int32_t apply(std::string_view name, uint32_t dom, uint32_t rng, int32_t arg) {
        if (is_arr(arg) || w(arg) != dom) fail(std::string(name) + ": argument width mismatch");
        return add(OP_UF, rng, arg, -1, -1, 0, dom, sym(name));
    }
    void no_arrays(std::initializer_list<int32_t> xs) {
        for (int32_t x : xs)
            if (is_arr(x)) fail("array operand of a bit-vector / Bool operator");
    }
    int32_t op1(uint8_t op, int32_t a) {
        no_arrays({a});
        if (op == OP_NOT) {
            if (!is_bool(a)) fail("not needs a Bool");
            return add(op, 0, a);
        }
        if (is_bool(a)) fail("bvneg / bvnot need a bit-vector");
        return add(op, w(a), a);
    }
    int32_t op2(uint8_t op, int32_t a, int32_t b) {
        no_arrays({a, b});
        switch (op) {
            case OP_EQ:
                if (w(a) != w(b)) fail("= needs equal sorts");
                return add(op, 0, a, b);
            case OP_AND: case OP_OR: case OP_XOR:
                if (!is_bool(a) || !is_bool(b)) fail("Bool connective over bit-vectors");
                return add(op, 0, a, b);
            case OP_CONCAT:
                if (is_bool(a) || is_bool(b)) fail("concat needs bit-vectors");
                if (w(a) + w(b) > MAX_WIDTH) fail("width exceeds 1088");
                return add(op, w(a) + w(b), a, b);
            default:
                break;
        }
        if (is_bool(a) || w(a) != w(b)) fail("bit-vector operator needs equal widths");
        const bool cmp = (op >= OP_BVULT && op <= OP_BVSGE) || op == OP_ADD_NOOVFL ||
                         op == OP_MUL_NOOVFL;
        return add(op, cmp ? 0 : w(a), a, b);
    }
    int32_t ite(int32_t c, int32_t t, int32_t e) {
        no_arrays({c, t, e});
        if (!is_bool(c) || w(t) != w(e)) fail("ite needs (Bool, s, s)");
        return add(OP_ITE, w(t), c, t, e);
    }
    int32_t extract(int32_t x, uint32_t hi, uint32_t lo) {
        no_arrays({x});
        if (is_bool(x) || lo > hi || hi >= w(x)) fail("bad extract");
        return add(OP_EXTRACT, hi - lo + 1, x, -1, -1, hi, lo);
    }
    int32_t ext(uint8_t op, int32_t x, uint32_t k) {
        no_arrays({x});
        if (is_bool(x)) fail("extension of a Bool");
        if (w(x) + k > MAX_WIDTH) fail("width exceeds 1088");
        return add(op, w(x) + k, x, -1, -1, k);
    }
    int32_t fold(uint8_t op, const std::vector<int32_t>& a) {
        int32_t acc = a[0];
        for (size_t i = 1; i < a.size(); ++i) acc = op2(op, acc, a[i]);
        return acc;
    }
    // z3's BVAddNoOverflow(x, y, False): (= ((_ extract w w) (bvadd ((_ zero_extend 1) x)
    // ((_ zero_extend 1) y))) #b0)
    int32_t add_noovfl(int32_t e, int32_t z) {
        const Node& Z = nodes[z];
        if (Z.op != OP_CONST || Z.width != 1 || (consts[Z.cidx].l[0] & 1)) return -1;
        const Node& E = nodes[e];
        if (E.op != OP_EXTRACT || E.imm0 != E.imm1 || E.width != 1) return -1;
        const Node& S = nodes[E.a];
        if (S.op != OP_BVADD || S.width != E.imm0 + 1) return -1;
        int32_t inner[2];
        const int32_t kids[2] = {S.a, S.b};
        for (int i = 0; i < 2; ++i) {
            const Node& K = nodes[kids[i]];
            if (K.op != OP_ZEXT || K.imm0 != 1 || nodes[K.a].width != E.imm0) return -1;
            inner[i] = K.a;
        }
        return op2(OP_ADD_NOOVFL, inner[0], inner[1]);
    }
};

namespace {

bool starts(std::string_view s, const char* p) { return s.substr(0, strlen(p)) == p; }

class Reader {
public:
    Reader(mh_smtlib& s, const char* text, const std::vector<Tok>& toks)
        : S(s), txt_(text), tk_(toks) {}

    // the top-level commands, in order
    void run() {
        size_t i = 0;
        while (i < tk_.size()) {
            if (tk_[i].type != T_LP) fail("not a command");
            command(i);
            i = tk_[i].match + 1;
        }
    }

private:
    mh_smtlib& S;
    const char* txt_;
    const std::vector<Tok>& tk_;
    // let scopes: the bindings in force per name (innermost last) and the names each open
    // scope bound, so a lookup is one hash probe however deep z3 nests its lets
    std::unordered_map<std::string_view, std::vector<int32_t>> env_;
    std::vector<std::string_view> bound_;

    std::string_view sv(size_t i) const { return std::string_view(txt_ + tk_[i].off, tk_[i].len); }
    bool is_atom(size_t i) const { return tk_[i].type == T_ATOM || tk_[i].type == T_QATOM; }
    bool is_list(size_t i) const { return tk_[i].type == T_LP; }
    size_t next(size_t i) const { return tk_[i].type == T_LP ? tk_[i].match + 1 : i + 1; }
    // the items of the list at token i
    void items(size_t i, std::vector<size_t>& out) const {
        out.clear();
        for (size_t j = i + 1; j < tk_[i].match; j = next(j)) out.push_back(j);
    }
    bool atom_is(size_t i, const char* s) const { return tk_[i].type == T_ATOM && sv(i) == s; }

    uint32_t to_u32(size_t i) const {
        if (tk_[i].type != T_ATOM || tk_[i].len == 0 || tk_[i].len > 9) fail("expected a small numeral");
        uint32_t v = 0;
        for (char c : sv(i)) {
            if (c < '0' || c > '9') fail("expected a numeral: " + std::string(sv(i)));
            v = v * 10 + (uint32_t)(c - '0');
        }
        return v;
    }

    Sort sort_of(size_t i) const {
        Sort r;
        if (is_atom(i)) {
            if (sv(i) == "Bool") { r.kind = 'B'; return r; }
            fail("unsupported sort " + std::string(sv(i)));
        }
        if (!is_list(i)) fail("unsupported sort");
        std::vector<size_t> it;
        items(i, it);
        if (it.size() == 3 && atom_is(it[0], "_") && atom_is(it[1], "BitVec")) {
            r.kind = 'b';
            r.width = to_u32(it[2]);
            return r;
        }
        if (it.size() == 3 && atom_is(it[0], "Array")) {
            const Sort d = sort_of(it[1]), v = sort_of(it[2]);
            if (d.kind != 'b' || v.kind != 'b') fail("arrays map bit-vectors to bit-vectors");
            r.kind = 'a';
            r.domain = d.width;
            r.width = v.width;
            return r;
        }
        fail("unsupported sort");
    }

    static void parse_radix(std::string_view digits, uint32_t radix, uint32_t* limbs) {
        for (int i = 0; i < 34; ++i) limbs[i] = 0;
        if (radix == 16 || radix == 2) {  // digit i from the right: bits [i * b, i * b + b)
            const uint32_t bits = radix == 16 ? 4u : 1u;
            const size_t n = digits.size();
            if (n * bits > 34 * 32) fail("numeral wider than 1088 bits");
            for (size_t i = 0; i < n; ++i) {
                const char ch = digits[n - 1 - i];
                uint32_t d;
                if (ch >= '0' && ch <= '9') d = (uint32_t)(ch - '0');
                else if (ch >= 'a' && ch <= 'f') d = 10u + (uint32_t)(ch - 'a');
                else if (ch >= 'A' && ch <= 'F') d = 10u + (uint32_t)(ch - 'A');
                else fail("bad numeral digit");
                if (d >= radix) fail("bad numeral digit");
                const size_t bit = i * bits;
                limbs[bit / 32] |= d << (bit % 32);
            }
            return;
        }
        for (char ch : digits) {
            uint32_t d;
            if (ch >= '0' && ch <= '9') d = (uint32_t)(ch - '0');
            else if (ch >= 'a' && ch <= 'f') d = 10u + (uint32_t)(ch - 'a');
            else if (ch >= 'A' && ch <= 'F') d = 10u + (uint32_t)(ch - 'A');
            else fail("bad numeral digit");
            if (d >= radix) fail("bad numeral digit");
            uint64_t carry = d;
            for (int k = 0; k < 34; ++k) {
                const uint64_t t = (uint64_t)limbs[k] * radix + carry;
                limbs[k] = (uint32_t)t;
                carry = t >> 32;
            }
            if (carry) fail("numeral wider than 1088 bits");
        }
    }

    void command(size_t ci) {
        std::vector<size_t> it;
        items(ci, it);
        if (it.empty() || tk_[it[0]].type != T_ATOM) fail("not a command");
        const std::string_view h = sv(it[0]);
        if (h == "set-option" || h == "set-info" || h == "set-logic" || h == "check-sat" ||
            h == "get-model" || h == "exit" || h == "get-objectives" || h == "push" ||
            h == "pop" || h == "echo")
            return;
        if (h == "declare-fun") {
            if (it.size() != 4 || !is_list(it[2]) || !is_atom(it[1])) fail("malformed declare-fun");
            std::vector<size_t> args;
            items(it[2], args);
            if (!args.empty()) {
                if (args.size() != 1)
                    fail("only unary functions are supported: " + std::string(sv(it[1])));
                S.set_decl(sv(it[1]), Decl{true, sort_of(it[3]), sort_of(args[0])});
            } else {
                S.set_decl(sv(it[1]), Decl{false, sort_of(it[3]), Sort{}});
            }
            return;
        }
        if (h == "declare-const") {
            if (it.size() != 3 || !is_atom(it[1])) fail("malformed declare-const");
            S.set_decl(sv(it[1]), Decl{false, sort_of(it[2]), Sort{}});
            return;
        }
        if (h == "define-fun") {
            if (it.size() != 5 || !is_list(it[2]) || !is_atom(it[1])) fail("malformed define-fun");
            if (tk_[it[2]].match != it[2] + 1)
                fail("define-fun with arguments is not supported: " + std::string(sv(it[1])));
            S.set_def(sv(it[1]), term(it[4]));
            return;
        }
        if (h == "assert") {
            if (it.size() != 2) fail("malformed assert");
            const int32_t n = term(it[1]);
            if (!S.is_bool(n)) fail("assert of a non-Bool term");
            S.results.push_back(mh_smt_result{MH_SMT_ASSERT, 0, (int64_t)n});
            return;
        }
        if (h == "minimize" || h == "maximize") {
            if (it.size() != 2) fail("malformed objective");
            const int32_t n = term(it[1]);
            S.results.push_back(mh_smt_result{
                h == "minimize" ? (uint32_t)MH_SMT_MINIMIZE : (uint32_t)MH_SMT_MAXIMIZE, 0,
                (int64_t)n});
            return;
        }
        fail("unsupported command " + std::string(h));
    }

    int32_t atom(size_t i) {
        const std::string_view s = sv(i);
        if (tk_[i].type == T_STR) fail("string literal in a term");
        if (tk_[i].type == T_ATOM) {
            if (s.size() > 2 && s[0] == '#' && (s[1] == 'x' || s[1] == 'b')) {
                auto lit = S.literals.find(s);
                if (lit != S.literals.end()) return lit->second;
                uint32_t l[34];
                int32_t n;
                if (s[1] == 'x') {
                    parse_radix(s.substr(2), 16, l);
                    n = S.konst(l, 4u * (uint32_t)(s.size() - 2));
                } else {
                    parse_radix(s.substr(2), 2, l);
                    n = S.konst(l, (uint32_t)(s.size() - 2));
                }
                S.literals.emplace(S.own(s), n);
                return n;
            }
            if (s == "true") return S.tru();
            if (s == "false") return S.fals();
        }
        if (!env_.empty()) {
            auto e = env_.find(s);
            if (e != env_.end() && !e->second.empty()) return e->second.back();
        }
        auto d = S.defs.find(s);
        if (d != S.defs.end()) return d->second;
        auto it = S.decls.find(s);
        if (it == S.decls.end()) fail("undeclared symbol '" + std::string(s) + "'");
        Decl& dc = it->second;
        if (dc.node >= 0) return dc.node;
        if (dc.fun) fail("function '" + std::string(s) + "' used as a constant");
        if (dc.sort.kind == 'B') dc.node = S.op2(OP_EQ, S.var(s, 1), S.konst_u(1, 1));
        else if (dc.sort.kind == 'b') dc.node = S.var(s, dc.sort.width);
        else dc.node = S.array(s, dc.sort.domain, dc.sort.width);
        return dc.node;
    }

    int32_t indexed(size_t head, int32_t x) {
        std::vector<size_t> it;
        items(head, it);
        if (it.size() >= 3 && atom_is(it[0], "as") && atom_is(it[1], "const")) {
            const Sort st = sort_of(it[2]);
            if (st.kind != 'a') fail("(as const ..) of a non-array sort");
            return S.const_array(st.domain, x);
        }
        if (it.size() < 3 || !atom_is(it[0], "_") || !is_atom(it[1]))
            fail("unsupported application head");
        const std::string_view name = sv(it[1]);
        uint32_t idx[2] = {0, 0};
        for (size_t k = 2; k < it.size() && k < 4; ++k) idx[k - 2] = to_u32(it[k]);
        if (name == "extract") {
            if (it.size() != 4) fail("extract takes 2 indices");
            return S.extract(x, idx[0], idx[1]);
        }
        if (it.size() != 3) fail("indexed operator takes 1 index");
        if (name == "zero_extend") return idx[0] == 0 ? x : S.ext(OP_ZEXT, x, idx[0]);
        if (name == "sign_extend") return idx[0] == 0 ? x : S.ext(OP_SEXT, x, idx[0]);
        if (name == "repeat") {
            if (idx[0] == 0) fail("repeat 0");
            int32_t acc = x;
            for (uint32_t k = 1; k < idx[0]; ++k) acc = S.op2(OP_CONCAT, acc, x);
            return acc;
        }
        if (name == "rotate_left" || name == "rotate_right") {
            if (S.is_bool(x) || S.is_arr(x)) fail("rotate of a non-bit-vector");
            const uint32_t w = S.w(x);
            uint32_t k = idx[0] % w;
            if (name == "rotate_right") k = (w - k) % w;
            if (k == 0) return x;
            const int32_t hi = S.extract(x, w - k - 1, 0);
            const int32_t lo = S.extract(x, w - 1, w - k);
            return S.op2(OP_CONCAT, hi, lo);
        }
        fail("unsupported indexed operator " + std::string(name));
    }

    // operator names -> (kind, op), looked up once per application
    enum AKind : uint8_t { A_BIN, A_NARY, A_CMP, A_NEG, A_NOT_BV, A_NOTX, A_COMP, A_CONCAT, A_AND,
                           A_OR, A_XOR, A_NOT, A_IMPL, A_EQ, A_DISTINCT, A_ITE, A_SELECT,
                           A_STORE };
    struct AOp { AKind kind; uint8_t op; };
    static const std::unordered_map<std::string_view, AOp>& ops_table() {
        static const std::unordered_map<std::string_view, AOp> t = {
            {"bvadd", {A_NARY, OP_BVADD}}, {"bvsub", {A_NARY, OP_BVSUB}},
            {"bvmul", {A_NARY, OP_BVMUL}}, {"bvand", {A_NARY, OP_BVAND}},
            {"bvor", {A_NARY, OP_BVOR}}, {"bvxor", {A_NARY, OP_BVXOR}},
            {"bvudiv", {A_BIN, OP_BVUDIV}}, {"bvudiv_i", {A_BIN, OP_BVUDIV}},
            {"bvurem", {A_BIN, OP_BVUREM}}, {"bvurem_i", {A_BIN, OP_BVUREM}},
            {"bvsdiv", {A_BIN, OP_BVSDIV}}, {"bvsdiv_i", {A_BIN, OP_BVSDIV}},
            {"bvsrem", {A_BIN, OP_BVSREM}}, {"bvsrem_i", {A_BIN, OP_BVSREM}},
            {"bvsmod", {A_BIN, OP_BVSMOD}}, {"bvsmod_i", {A_BIN, OP_BVSMOD}},
            {"bvshl", {A_BIN, OP_BVSHL}}, {"bvlshr", {A_BIN, OP_BVLSHR}},
            {"bvashr", {A_BIN, OP_BVASHR}},
            {"bvult", {A_CMP, OP_BVULT}}, {"bvule", {A_CMP, OP_BVULE}},
            {"bvugt", {A_CMP, OP_BVUGT}}, {"bvuge", {A_CMP, OP_BVUGE}},
            {"bvslt", {A_CMP, OP_BVSLT}}, {"bvsle", {A_CMP, OP_BVSLE}},
            {"bvsgt", {A_CMP, OP_BVSGT}}, {"bvsge", {A_CMP, OP_BVSGE}},
            {"bvumul_noovfl", {A_CMP, OP_MUL_NOOVFL}},
            {"bvneg", {A_NEG, OP_BVNEG}}, {"bvnot", {A_NOT_BV, OP_BVNOT}},
            {"bvnand", {A_NOTX, OP_BVAND}}, {"bvnor", {A_NOTX, OP_BVOR}},
            {"bvxnor", {A_NOTX, OP_BVXOR}}, {"bvcomp", {A_COMP, 0}},
            {"concat", {A_CONCAT, 0}}, {"and", {A_AND, 0}}, {"or", {A_OR, 0}},
            {"xor", {A_XOR, 0}}, {"not", {A_NOT, 0}}, {"=>", {A_IMPL, 0}}, {"=", {A_EQ, 0}},
            {"distinct", {A_DISTINCT, 0}}, {"ite", {A_ITE, 0}}, {"select", {A_SELECT, 0}},
            {"store", {A_STORE, 0}}};
        return t;
    }

    int32_t apply(std::string_view h, const int32_t* a, size_t na) {
        auto need = [&](size_t n) {
            if (na != n) fail(std::string(h) + " takes " + std::to_string(n) + " arguments");
        };
        auto fold = [&](uint8_t op) {
            int32_t acc = a[0];
            for (size_t k = 1; k < na; ++k) acc = S.op2(op, acc, a[k]);
            return acc;
        };
        const auto& tab = ops_table();
        const auto found = tab.find(h);
        if (found != tab.end()) {
            const AOp o = found->second;
            switch (o.kind) {
                case A_NARY:
                case A_BIN:
                    if (na < 2 || (na > 2 && o.kind != A_NARY))
                        fail(std::string(h) + " takes 2 arguments");
                    return fold(o.op);
                case A_CMP: need(2); return S.op2(o.op, a[0], a[1]);
                case A_NEG: need(1); return S.op1(OP_BVNEG, a[0]);
                case A_NOT_BV: need(1); return S.op1(OP_BVNOT, a[0]);
                case A_NOTX: need(2); return S.op1(OP_BVNOT, S.op2(o.op, a[0], a[1]));
                case A_COMP:
                    need(2);
                    return S.ite(S.op2(OP_EQ, a[0], a[1]), S.konst_u(1, 1), S.konst_u(0, 1));
                case A_CONCAT: if (!na) fail("concat of nothing"); return fold(OP_CONCAT);
                case A_AND: return na ? fold(OP_AND) : S.tru();
                case A_OR: return na ? fold(OP_OR) : S.fals();
                case A_XOR: if (!na) fail("xor of nothing"); return fold(OP_XOR);
                case A_NOT: need(1); return S.op1(OP_NOT, a[0]);
                case A_IMPL: need(2); return S.op2(OP_OR, S.op1(OP_NOT, a[0]), a[1]);
                case A_EQ: {
                    if (na < 2) fail("= takes 2 or more arguments");
                    for (size_t k = 0; k < na; ++k)
                        if (S.is_arr(a[k])) fail("equality between arrays is not supported");
                    if (na == 2) {
                        int32_t nov = S.add_noovfl(a[0], a[1]);
                        if (nov < 0) nov = S.add_noovfl(a[1], a[0]);
                        if (nov >= 0) return nov;
                    }
                    int32_t acc = S.op2(OP_EQ, a[0], a[1]);
                    for (size_t k = 1; k + 1 < na; ++k)
                        acc = S.op2(OP_AND, acc, S.op2(OP_EQ, a[k], a[k + 1]));
                    return acc;
                }
                case A_DISTINCT: {
                    if (na < 2) fail("distinct takes 2 or more arguments");
                    int32_t acc = -1;
                    for (size_t i = 0; i < na; ++i)
                        for (size_t j = i + 1; j < na; ++j) {
                            const int32_t ne = S.op1(OP_NOT, S.op2(OP_EQ, a[i], a[j]));
                            acc = acc < 0 ? ne : S.op2(OP_AND, acc, ne);
                        }
                    return acc;
                }
                case A_ITE:
                    need(3);
                    if (S.is_arr(a[1])) fail("ite over arrays is not supported");
                    return S.ite(a[0], a[1], a[2]);
                case A_SELECT: need(2); return S.select(a[0], a[1]);
                case A_STORE: need(3); return S.store(a[0], a[1], a[2]);
            }
        }
        auto it = S.decls.find(h);
        if (it != S.decls.end() && it->second.fun) {
            need(1);
            const Decl& d = it->second;
            if (d.sort.kind != 'b' || d.dom.kind != 'b')
                fail("function " + std::string(h) + " must map bit-vectors to bit-vectors");
            return S.apply(it->first, d.dom.width, d.sort.width, a[0]);
        }
        fail("unsupported operator '" + std::string(h) + "'");
    }

public:
    // explicit work stack (no recursion): terms nest thousands deep
    int32_t term(size_t root) {
        enum { EVAL, LET_BODY, APPLY, INDEXED, POP_SCOPE };
        struct Item {
            uint8_t kind;
            uint32_t tok;  // the term's token (EVAL), the let / application / head list
            uint32_t n;    // LET_BODY: bindings; APPLY: arguments
        };
        std::vector<int32_t> vals;
        std::vector<Item> work{{EVAL, (uint32_t)root, 0}};
        std::vector<size_t> marks;
        while (!work.empty()) {
            const Item itm = work.back();
            work.pop_back();
            const size_t t = itm.tok;
            switch (itm.kind) {
                case EVAL: {
                    if (!is_list(t)) { vals.push_back(atom(t)); break; }
                    const size_t h = t + 1;
                    if (h == tk_[t].match) fail("empty application");
                    if (atom_is(h, "let")) {
                        const size_t binds = next(h);
                        if (binds >= tk_[t].match || !is_list(binds)) fail("malformed let");
                        const size_t body = next(binds);
                        if (body >= tk_[t].match || next(body) != tk_[t].match) fail("malformed let");
                        const size_t mark = work.size();
                        work.push_back({LET_BODY, (uint32_t)t, 0});
                        // bound values (outer scope) pushed in order, then reversed in place so
                        // they evaluate first to last
                        for (size_t j = binds + 1; j < tk_[binds].match; j = next(j)) {
                            if (!is_list(j) || !is_atom(j + 1) || next(j + 1) >= tk_[j].match ||
                                next(next(j + 1)) != tk_[j].match)
                                fail("malformed let binding");
                            work.push_back({EVAL, (uint32_t)next(j + 1), 0});
                        }
                        work[mark].n = (uint32_t)(work.size() - mark - 1);
                        std::reverse(work.begin() + (long)mark + 1, work.end());
                        break;
                    }
                    if (is_list(h)) {  // ((_ extract i j) x), ((as const S) v)
                        const size_t arg = next(h);
                        if (arg >= tk_[t].match || next(arg) != tk_[t].match)
                            fail("indexed application takes 1 argument");
                        work.push_back({INDEXED, (uint32_t)h, 0});
                        work.push_back({EVAL, (uint32_t)arg, 0});
                        break;
                    }
                    if (atom_is(h, "_")) {  // (_ bvN w)
                        const size_t lit = next(h);
                        if (lit < tk_[t].match && tk_[lit].type == T_ATOM && starts(sv(lit), "bv") &&
                            next(lit) < tk_[t].match && next(next(lit)) == tk_[t].match) {
                            uint32_t l[34];
                            parse_radix(sv(lit).substr(2), 10, l);
                            vals.push_back(S.konst(l, to_u32(next(lit))));
                            break;
                        }
                        fail("unsupported indexed term");
                    }
                    if (!is_atom(h)) fail("bad application head");
                    const size_t mark = work.size();
                    work.push_back({APPLY, (uint32_t)t, 0});
                    for (size_t j = next(h); j < tk_[t].match; j = next(j))
                        work.push_back({EVAL, (uint32_t)j, 0});
                    work[mark].n = (uint32_t)(work.size() - mark - 1);
                    std::reverse(work.begin() + (long)mark + 1, work.end());
                    break;
                }
                case LET_BODY: {
                    const size_t binds = next(t + 1);
                    const size_t k = itm.n;
                    marks.push_back(bound_.size());
                    size_t i = 0;
                    for (size_t j = binds + 1; j < tk_[binds].match; j = next(j), ++i) {
                        env_[sv(j + 1)].push_back(vals[vals.size() - k + i]);
                        bound_.push_back(sv(j + 1));
                    }
                    vals.resize(vals.size() - k);
                    work.push_back({POP_SCOPE, 0, 0});
                    work.push_back({EVAL, (uint32_t)next(binds), 0});
                    break;
                }
                case APPLY: {
                    const size_t n = itm.n;
                    const int32_t r = apply(sv(t + 1), vals.data() + vals.size() - n, n);
                    vals.resize(vals.size() - n);
                    vals.push_back(r);
                    break;
                }
                case INDEXED: {
                    const int32_t x = vals.back();
                    vals.pop_back();
                    vals.push_back(indexed(t, x));
                    break;
                }
                default:
                    while (bound_.size() > marks.back()) {
                        auto e = env_.find(bound_.back());
                        e->second.pop_back();
                        if (e->second.empty()) env_.erase(e);
                        bound_.pop_back();
                    }
                    marks.pop_back();
            }
        }
        if (vals.size() != 1) fail("malformed term");
        return vals[0];
    }
};

}  // namespace

extern "C" {

int32_t mh_smtlib_create(mh_smtlib** out) {
    if (!out) return mh_detail_set_err(MH_E_INVALID, "null out");
    *out = new (std::nothrow) mh_smtlib();
    return *out ? MH_OK : mh_detail_set_err(MH_E_NOMEM, "mh_smtlib_create");
}

int32_t mh_smtlib_destroy(mh_smtlib* s) {
    if (!s) return mh_detail_set_err(MH_E_INVALID, "null session");
    delete s;
    return MH_OK;
}

int32_t mh_smtlib_read(mh_smtlib* s, const char* text, uint64_t len, mh_smt_batch* out) {
    if (!s || !out || (!text && len)) return mh_detail_set_err(MH_E_INVALID, "null argument");
    if (s->pending) return mh_detail_set_err(MH_E_INVALID, "previous read not committed");
    const size_t n0 = s->nodes.size();
    s->undo.clear();  // what a failed read must undo (decls / defs it wrote)
    s->results.clear();
    try {
        tokenize(text, (size_t)len, s->toks);
        Reader rd(*s, text, s->toks);
        rd.run();
    } catch (const Fail& f) {
        for (size_t i = n0; i < s->nodes.size(); ++i) {
            const Node& nd = s->nodes[i];
            s->memo.erase(Key{nd.op, nd.width, nd.imm0, nd.imm1, nd.a, nd.b, nd.c, nd.sym, nd.cidx});
        }
        s->nodes.resize(n0);
        s->undo_all();
        s->drop_caches();
        s->results.clear();
        return mh_detail_set_err(MH_E_INVALID, ("SMT-LIB: " + f.msg).c_str());
    } catch (const std::bad_alloc&) {
        return mh_detail_set_err(MH_E_NOMEM, "mh_smtlib_read");
    }
    // records: every node the host does not have yet, operands as host ids (>= 0) or -(k + 1)
    // for record k of this batch
    s->recs.clear();
    s->rec_consts.clear();
    s->rec_names.clear();
    s->first_new = n0;
    auto ref = [&](int32_t x) -> int64_t {
        if (x < 0) return 0;
        const Node& nd = s->nodes[x];
        return nd.host >= 0 ? nd.host : -(int64_t)(x - n0) - 1;
    };
    for (size_t i = n0; i < s->nodes.size(); ++i) {
        const Node& nd = s->nodes[i];
        mh_smt_record r{};
        r.op = nd.op;
        r.width = nd.width;
        r.a = ref(nd.a);
        r.b = ref(nd.b);
        r.c = ref(nd.c);
        r.imm0 = nd.imm0;
        r.imm1 = nd.imm1;
        if (nd.sym >= 0) {
            r.name_off = (uint32_t)s->rec_names.size();
            r.name_len = (uint32_t)s->syms[nd.sym].size();
            s->rec_names.append(s->syms[nd.sym].data(), s->syms[nd.sym].size());
        }
        if (nd.op == OP_CONST) {
            r.const_off = (uint32_t)s->rec_consts.size();
            s->rec_consts.insert(s->rec_consts.end(), s->consts[nd.cidx].l, s->consts[nd.cidx].l + 8);
        }
        s->recs.push_back(r);
    }
    for (mh_smt_result& r : s->results) r.node = ref((int32_t)r.node);
    out->records = s->recs.data();
    out->n_records = s->recs.size();
    out->const_limbs = s->rec_consts.data();
    out->names = s->rec_names.data();
    out->results = s->results.data();
    out->n_results = s->results.size();
    s->pending = !s->recs.empty();
    if (!s->pending) s->recs.clear();
    return MH_OK;
}

int32_t mh_smtlib_commit(mh_smtlib* s, const int64_t* host_ids, uint64_t n) {
    if (!s) return mh_detail_set_err(MH_E_INVALID, "null session");
    if (!s->pending) return n ? mh_detail_set_err(MH_E_INVALID, "nothing to commit") : MH_OK;
    if (n != s->recs.size() || !host_ids)
        return mh_detail_set_err(MH_E_INVALID, "commit needs one host id per record");
    for (uint64_t k = 0; k < n; ++k) {
        if (host_ids[k] < 0) return mh_detail_set_err(MH_E_INVALID, "negative host id");
        s->nodes[s->first_new + k].host = host_ids[k];
    }
    s->pending = false;
    return MH_OK;
}

int32_t mh_smtlib_rollback(mh_smtlib* s) {
    // the host could not build the last read's records: forget them (they were never committed)
    if (!s) return mh_detail_set_err(MH_E_INVALID, "null session");
    if (!s->pending) return MH_OK;
    for (size_t i = s->first_new; i < s->nodes.size(); ++i) {
        const Node& nd = s->nodes[i];
        s->memo.erase(Key{nd.op, nd.width, nd.imm0, nd.imm1, nd.a, nd.b, nd.c, nd.sym, nd.cidx});
    }
    s->nodes.resize(s->first_new);
    s->undo_all();  // the read's declarations and definitions may name the dropped nodes
    s->drop_caches();
    s->pending = false;
    return MH_OK;
}

uint64_t mh_smtlib_size(const mh_smtlib* s) { return s ? s->nodes.size() : 0; }

}  // extern "C"
