// Replays a recording of the query path's host-only native calls (tests/tools/host_record.py)
// against csrc/query.cpp + harvest.cpp + smtlib.cpp built into this executable, for
// AddressSanitizer / UBSan runs (tests/test_host_sanitized.py; test infrastructure, no device).
// Every call must return what it returned under Python (MH_OK; a read of malformed text its
// recorded MH_E_INVALID); each query's, guide's and read batch's arrays are read end to end (a
// checksum), so an array shorter than its stated size is an out-of-bounds read the sanitizer
// reports.
//
//   host_replay RECORDING     -> prints "calls=N queries=Q guides=G checksum=X", exit 0
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/mythril_hip.h"

static thread_local std::string g_err;
int32_t mh_detail_set_err(int32_t code, const char* msg) {  // capi.cpp's, for this build
    g_err = msg ? msg : "";
    return code;
}

namespace {

struct Reader {
    const std::vector<uint8_t>& b;
    size_t at = 0;
    bool ok = true;
    template <class T>
    T get() {
        T v{};
        if (at + sizeof(T) > b.size()) { ok = false; return v; }
        std::memcpy(&v, b.data() + at, sizeof(T));
        at += sizeof(T);
        return v;
    }
    const uint8_t* take(size_t n) {
        if (at + n > b.size()) { ok = false; return nullptr; }
        const uint8_t* p = b.data() + at;
        at += n;
        return p;
    }
};

uint64_t mix(uint64_t h, const void* p, size_t n) {
    const uint8_t* c = static_cast<const uint8_t*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 0x100000001B3ull;
    return h;
}

// aligned copies of recorded arrays (the recording's byte stream has no alignment)
template <class T>
std::vector<T> copy_of(const uint8_t* p, size_t n) {
    std::vector<T> v(n ? n : 1);
    if (n) std::memcpy(v.data(), p, n * sizeof(T));
    return v;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 2) {
        std::fprintf(stderr, "usage: host_replay RECORDING\n");
        return 2;
    }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) { std::perror("open"); return 2; }
    std::vector<uint8_t> all;
    uint8_t buf[1 << 16];
    for (size_t n; (n = std::fread(buf, 1, sizeof buf, f)) > 0;) all.insert(all.end(), buf, buf + n);
    std::fclose(f);

    std::unordered_map<uint64_t, mh_terms*> terms;
    std::unordered_map<uint64_t, mh_harvester*> harvesters;
    std::unordered_map<uint64_t, mh_smtlib*> readers;
    uint64_t calls = 0, queries = 0, guides = 0, sum = 0xCBF29CE484222325ull;
    Reader top{all};
    auto fail = [&](const char* what) {
        std::fprintf(stderr, "call %llu (%s): %s\n", (unsigned long long)calls, what, g_err.c_str());
        return 1;
    };
    while (top.at < all.size()) {
        const char kind = top.get<char>();
        const uint64_t sid = top.get<uint64_t>();
        const uint64_t len = top.get<uint64_t>();
        const uint8_t* payload = top.take(len);
        if (!top.ok) { std::fprintf(stderr, "truncated recording\n"); return 2; }
        std::vector<uint8_t> pb(payload, payload + len);
        Reader r{pb};
        ++calls;
        switch (kind) {
        case 'C': {
            mh_terms* t = nullptr;
            if (mh_terms_create(&t) != MH_OK || terms.count(sid)) return fail("terms_create");
            terms[sid] = t;
            break;
        }
        case 'D': {
            auto it = terms.find(sid);
            if (it == terms.end() || mh_terms_destroy(it->second) != MH_OK) return fail("terms_destroy");
            terms.erase(it);
            break;
        }
        case 'O': {
            auto it = terms.find(sid);
            const uint32_t opts = r.get<uint32_t>();
            if (it == terms.end() || !r.ok || mh_terms_set_options(it->second, opts) != MH_OK)
                return fail("terms_set_options");
            break;
        }
        case 'A': {
            auto it = terms.find(sid);
            if (it == terms.end()) return fail("append: unknown session");
            const uint64_t nn = r.get<uint64_t>();
            auto nodes = copy_of<mh_node>(r.take(nn * sizeof(mh_node)), nn);
            const uint64_t nc = r.get<uint64_t>();
            auto consts = copy_of<uint32_t>(r.take(nc * 32), nc * 8);
            std::string names[3];
            uint64_t counts[3];
            for (int k = 0; k < 3; ++k) {
                counts[k] = r.get<uint64_t>();
                const uint64_t bl = r.get<uint64_t>();
                const uint8_t* p = r.take(bl);
                if (p) names[k].assign(reinterpret_cast<const char*>(p), bl);
            }
            if (!r.ok) return fail("append: short record");
            if (mh_terms_append(it->second, nodes.data(), nn, consts.data(), nc, names[0].c_str(),
                                counts[0], names[1].c_str(), counts[1], names[2].c_str(),
                                counts[2]) != MH_OK)
                return fail("terms_append");
            break;
        }
        case 'Q': {
            auto it = terms.find(sid);
            if (it == terms.end()) return fail("query: unknown session");
            const uint32_t n = r.get<uint32_t>();
            auto roots = copy_of<uint32_t>(r.take(4ull * n), n);
            mh_query* q = nullptr;
            mh_query_info info{};
            if (!r.ok || mh_query_build(it->second, roots.data(), n, &q, &info) != MH_OK)
                return fail("query_build");
            ++queries;
            // every array end to end, at the sizes the info states
            const uint64_t n_nodes = info.n_tapes ? info.tape_off[info.n_tapes] : 0;
            sum = mix(sum, info.tape_off, (info.n_tapes + 1) * sizeof(uint64_t));
            sum = mix(sum, info.nodes, n_nodes * sizeof(mh_node));
            sum = mix(sum, info.consts, (size_t)info.n_consts * 32);
            sum = mix(sum, info.columns, (size_t)info.n_columns * sizeof(mh_query_column));
            sum = mix(sum, info.names, info.names_len);
            sum = mix(sum, info.key_limbs, (size_t)info.n_keys * MH_QUERY_KEY_LIMBS * 4);
            sum = mix(sum, info.group_off, (info.n_groups + 1) * sizeof(uint32_t));
            if (info.n_groups) sum = mix(sum, info.group_cols, info.group_off[info.n_groups] * 4ull);
            sum = mix(sum, info.tables, (size_t)info.n_tables * sizeof(mh_query_table));
            sum = mix(sum, info.table_limbs, (size_t)info.n_table_entries * MH_QUERY_KEY_LIMBS * 4);
            for (uint32_t i = 0; i < info.n_columns; ++i) {  // names inside the name buffer
                const mh_query_column& c = info.columns[i];
                if ((uint64_t)c.name_off + c.name_len > info.names_len) return fail("column name range");
            }
            sum = mix(sum, &info.flags, sizeof info.flags);
            // the root boundaries: one per proper prefix, ascending, inside the root tape
            sum = mix(sum, info.root_ends, (size_t)info.n_root_ends * 4);
            const uint64_t root_len = info.n_tapes ? info.tape_off[1] : 0;
            for (uint32_t i = 0; i < info.n_root_ends; ++i)
                if (info.root_ends[i] == 0 || info.root_ends[i] >= root_len ||
                    (i && info.root_ends[i] < info.root_ends[i - 1]))
                    return fail("root_ends");
            if (info.n_root_ends && info.parent_len != info.root_ends[info.n_root_ends - 1])
                return fail("parent_len");
            if (info.n_root_ends && info.n_root_ends + 1 != n) return fail("n_root_ends");
            if (mh_query_free(q) != MH_OK) return fail("query_free");
            break;
        }
        case 'H': {
            mh_harvester* s = nullptr;
            if (mh_harvester_create(&s) != MH_OK || harvesters.count(sid)) return fail("harvester_create");
            harvesters[sid] = s;
            break;
        }
        case 'X': {
            auto it = harvesters.find(sid);
            if (it == harvesters.end() || mh_harvester_destroy(it->second) != MH_OK)
                return fail("harvester_destroy");
            harvesters.erase(it);
            break;
        }
        case 'G':
        case 'g':
        case 'i': {
            const uint32_t nn = r.get<uint32_t>();
            auto nodes = copy_of<mh_node>(r.take((size_t)nn * sizeof(mh_node)), nn);
            const uint32_t nc = r.get<uint32_t>();
            auto consts = copy_of<uint32_t>(r.take((size_t)nc * 32), (size_t)nc * 8);
            const uint32_t ncol = r.get<uint32_t>();
            auto widths = copy_of<uint16_t>(r.take(2ull * ncol), ncol);
            const uint32_t np = r.get<uint32_t>();
            auto pcols = copy_of<uint32_t>(r.take(4ull * np), np);
            auto pvals = copy_of<uint32_t>(r.take(32ull * np), 8ull * np);
            if (!r.ok) return fail("guide: short record");
            mh_harvest* h = nullptr;
            mh_guide g{};
            int32_t rc;
            if (kind == 'G') {
                auto it = harvesters.find(sid);
                if (it == harvesters.end()) return fail("guide: unknown session");
                rc = mh_guide_harvest_with(it->second, nodes.data(), nn, consts.data(), nc,
                                           widths.data(), ncol, pcols.data(), pvals.data(), np, &h, &g);
            } else if (kind == 'i') {  // the incremental round's parent-evaluating harvest
                rc = mh_guide_harvest_inc(nodes.data(), nn, consts.data(), nc, widths.data(), ncol,
                                          pcols.data(), pvals.data(), np, &h, &g);
            } else {
                rc = mh_guide_harvest(nodes.data(), nn, consts.data(), nc, widths.data(), ncol,
                                      pcols.data(), pvals.data(), np, &h, &g);
            }
            if (rc != MH_OK) return fail("guide_harvest");
            ++guides;
            sum = mix(sum, g.col_width, g.n_cols * 2ull);
            sum = mix(sum, g.pool_off, (g.n_cols + 1) * 4ull);
            sum = mix(sum, g.pool, g.pool_off[g.n_cols] * 32ull);
            sum = mix(sum, g.set_prob, g.n_sets);
            sum = mix(sum, g.set_off, (g.n_sets + 1) * 4ull);
            const uint32_t n_alts = g.set_off[g.n_sets];
            sum = mix(sum, g.alt_off, (n_alts + 1) * 4ull);
            const uint32_t n_ent = g.alt_off[n_alts];
            sum = mix(sum, g.entry_col, n_ent * 4ull);
            sum = mix(sum, g.entry_val, n_ent * 32ull);
            if (mh_harvest_free(h) != MH_OK) return fail("harvest_free");
            break;
        }
        case 'S': {
            mh_smtlib* s = nullptr;
            if (mh_smtlib_create(&s) != MH_OK || readers.count(sid)) return fail("smtlib_create");
            readers[sid] = s;
            break;
        }
        case 'Z': {
            auto it = readers.find(sid);
            if (it == readers.end() || mh_smtlib_destroy(it->second) != MH_OK)
                return fail("smtlib_destroy");
            readers.erase(it);
            break;
        }
        case 'R': {  // the recorded return code must come back (malformed text: MH_E_INVALID)
            auto it = readers.find(sid);
            if (it == readers.end()) return fail("read: unknown session");
            const int32_t want = r.get<int32_t>();
            const std::string text(reinterpret_cast<const char*>(pb.data() + r.at), pb.size() - r.at);
            mh_smt_batch bt{};
            const int32_t rc = mh_smtlib_read(it->second, text.data(), text.size(), &bt);
            if (rc != want) return fail("smtlib_read: return code differs");
            if (rc == MH_OK) {
                ++queries;
                uint64_t names_len = 0, limbs = 0;
                for (uint64_t i = 0; i < bt.n_records; ++i) {
                    const mh_smt_record& x = bt.records[i];
                    names_len = std::max<uint64_t>(names_len, (uint64_t)x.name_off + x.name_len);
                    if (x.op == MH_OP_CONST) limbs = std::max<uint64_t>(limbs, x.const_off + 8ull);
                }
                sum = mix(sum, bt.records, bt.n_records * sizeof(mh_smt_record));
                sum = mix(sum, bt.results, bt.n_results * sizeof(mh_smt_result));
                sum = mix(sum, bt.names, names_len);
                sum = mix(sum, bt.const_limbs, limbs * 4);
            }
            break;
        }
        case 'M': {
            auto it = readers.find(sid);
            if (it == readers.end()) return fail("commit: unknown session");
            const uint64_t n = r.get<uint64_t>();
            auto ids = copy_of<int64_t>(r.take(8 * n), n);
            if (!r.ok || mh_smtlib_commit(it->second, ids.data(), n) != MH_OK) return fail("smtlib_commit");
            break;
        }
        case 'B': {
            auto it = readers.find(sid);
            if (it == readers.end() || mh_smtlib_rollback(it->second) != MH_OK) return fail("smtlib_rollback");
            break;
        }
        default:
            std::fprintf(stderr, "unknown record kind %d\n", kind);
            return 2;
        }
    }
    for (auto& kv : terms) mh_terms_destroy(kv.second);
    for (auto& kv : harvesters) mh_harvester_destroy(kv.second);
    for (auto& kv : readers) mh_smtlib_destroy(kv.second);
    std::printf("calls=%llu queries=%llu guides=%llu checksum=%016llx\n",
                (unsigned long long)calls, (unsigned long long)queries,
                (unsigned long long)guides, (unsigned long long)sum);
    return 0;
}
