// Replays the corpus of tests/tools/jit_corpus.py through the tape compiler's interpreter
// lowering (emu_eval: csrc/compile.cpp) and the JIT (emu_jit_eval: csrc/jit.cpp's SSA lowering,
// conjunct ordering, register allocation and emission, run by the host wave emulator), and
// emits each set's module text (emu_jit_module: build_module), all built into this executable
// for AddressSanitizer / UBSan runs (tests/test_host_sanitized.py; test infrastructure, no
// device).  Every return code and every output word must equal the corpus's (the unsanitized
// build's).
//
//   jit_replay CORPUS     -> prints "sets=S tapes=T jitted=J", exit 0
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mythril_hip.h"

extern "C" int32_t emu_eval(const mh_node* nodes, const uint64_t* offs, uint32_t n_tapes,
                            const uint32_t* consts, uint32_t n_consts, uint32_t n_vars,
                            uint32_t tape, const uint32_t* assign, uint64_t rows, uint32_t* out,
                            uint32_t* n_regs_out, char* err, int errlen);
extern "C" int32_t emu_jit_eval(const mh_node* nodes, const uint64_t* offs, uint32_t n_tapes,
                                const uint32_t* consts, uint32_t n_consts, uint32_t n_vars,
                                uint32_t tape, const uint32_t* assign, uint64_t rows,
                                uint32_t* out, uint32_t max_vgpr, uint32_t* info, char* err,
                                int errlen);
extern "C" int64_t emu_jit_module(const mh_node* nodes, const uint64_t* offs, uint32_t n_tapes,
                                  const uint32_t* consts, uint32_t n_consts, uint32_t n_vars,
                                  uint32_t values, uint32_t max_vgpr, int32_t assemble_it,
                                  char* text, uint64_t cap, uint64_t* hsaco_size,
                                  uint32_t* n_jitted, char* err, int errlen);

namespace {

struct In {
    FILE* f;
    bool ok = true;
    template <class T>
    T get() {
        T v{};
        ok = ok && std::fread(&v, sizeof v, 1, f) == 1;
        return v;
    }
    template <class T>
    std::vector<T> arr(size_t n) {
        std::vector<T> v(n ? n : 1);
        ok = ok && (n == 0 || std::fread(v.data(), sizeof(T), n, f) == n);
        return v;
    }
};

}  // namespace

int main(int argc, char** argv) {
    if (argc != 2) {
        std::fprintf(stderr, "usage: jit_replay CORPUS\n");
        return 2;
    }
    In in{std::fopen(argv[1], "rb")};
    if (!in.f) { std::perror("open"); return 2; }
    const uint32_t n_sets = in.get<uint32_t>();
    uint64_t tapes = 0, jitted = 0;
    char err[512];
    for (uint32_t s = 0; s < n_sets && in.ok; ++s) {
        const uint32_t n_tapes = in.get<uint32_t>(), n_vars = in.get<uint32_t>(),
                       n_consts = in.get<uint32_t>(), rows = in.get<uint32_t>();
        auto offs = in.arr<uint64_t>(n_tapes + 1ull);
        auto nodes = in.arr<mh_node>(offs[n_tapes]);
        auto consts = in.arr<uint32_t>(8ull * n_consts);
        auto soa = in.arr<uint32_t>(8ull * n_vars * rows);
        if (!in.ok) { std::fprintf(stderr, "truncated corpus\n"); return 2; }
        for (uint32_t t = 0; t < n_tapes; ++t) {
            const int32_t want_i = in.get<int32_t>();
            auto want_iv = in.arr<uint32_t>(8ull * rows);
            const int32_t want_j = in.get<int32_t>();
            const uint32_t want_jitted = in.get<uint32_t>();
            auto want_jv = in.arr<uint32_t>(8ull * rows);
            if (!in.ok) { std::fprintf(stderr, "truncated corpus\n"); return 2; }
            std::vector<uint32_t> out(8ull * rows);
            uint32_t nregs = 0;
            const int32_t ri = emu_eval(nodes.data(), offs.data(), n_tapes, consts.data(), n_consts,
                                        n_vars, t, soa.data(), rows, out.data(), &nregs, err,
                                        sizeof err);
            if (ri != want_i || (ri == 0 && out != std::vector<uint32_t>(want_iv.begin(),
                                                                        want_iv.begin() + out.size()))) {
                std::fprintf(stderr, "set %u tape %u: interpreter lowering differs (rc %d vs %d)\n", s,
                             t, ri, want_i);
                return 1;
            }
            std::vector<uint32_t> out2(8ull * rows);
            uint32_t info[16] = {};
            const int32_t rj = emu_jit_eval(nodes.data(), offs.data(), n_tapes, consts.data(),
                                            n_consts, n_vars, t, soa.data(), rows, out2.data(), 128,
                                            info, err, sizeof err);
            if (rj != want_j || info[0] != want_jitted ||
                (rj == 0 && info[0] && out2 != std::vector<uint32_t>(want_jv.begin(),
                                                                     want_jv.begin() + out2.size()))) {
                std::fprintf(stderr, "set %u tape %u: native code differs (rc %d vs %d, jitted %u vs %u)\n",
                             s, t, rj, want_j, info[0], want_jitted);
                return 1;
            }
            ++tapes;
            jitted += info[0] != 0;
        }
        // the whole set's module text, both modes (no assembly: comgr is not under test)
        for (uint32_t values = 0; values < 2; ++values) {
            std::vector<char> text(1 << 22);
            uint64_t hsaco = 0;
            uint32_t nj = 0;
            const int64_t len = emu_jit_module(nodes.data(), offs.data(), n_tapes, consts.data(),
                                               n_consts, n_vars, values, 128, 0, text.data(),
                                               text.size(), &hsaco, &nj, err, sizeof err);
            if (len <= 0 || nj == 0) {
                std::fprintf(stderr, "set %u: module emission failed (%lld)\n", s, (long long)len);
                return 1;
            }
        }
    }
    std::fclose(in.f);
    if (!in.ok) { std::fprintf(stderr, "truncated corpus\n"); return 2; }
    std::printf("sets=%u tapes=%llu jitted=%llu\n", n_sets, (unsigned long long)tapes,
                (unsigned long long)jitted);
    return 0;
}
