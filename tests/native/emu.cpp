// TEST-ONLY host emulator of the device interpreter (not part of libmythril_hip).
//
// Runs the tape compiler (mythril_amd/csrc/compile.cpp) and then the device instruction stream
// on the host CPU, using the same limb routines the kernel uses (mythril_amd/csrc/u256_ops.h).
// It lets tests/test_emulator.py check the compiler (lowering, accumulator scheduling, register
// allocation, encoding) and the 256-bit algorithms (division, shifts, signed ops, keccak-f)
// against the Python oracle without a GPU.  The instruction semantics are exec.h's step(), the
// very code the kernel runs.
#include <stdint.h>
#include <string.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "compile.h"
#include "exec.h"
#include "u256_ops.h"

using namespace mh;

// Host machine for exec.h's step(): the same instruction semantics the kernel compiles.
struct HostMachine {
    u32 R[MH_NR_MAX + 1][8];
    u32 nrx_;
    const u32* slots;  // the tape's slot words (w0, w1 pairs)
    const u32* assign;
    u64 cap, row;
    u32 nrx() const { return nrx_; }
    void read(u32 r, u32* v) const { memcpy(v, R[r], 32); }
    u32 read0(u32 r) const { return R[r][0]; }
    void write(u32 r, const u32* v) { memcpy(R[r], v, 32); }
    void iconst(u32 slot, u32* v) const { memcpy(v, slots + 2ull * slot, 32); }
    void var(u32 col, u32* v) const {
        for (int k = 0; k < 8; ++k) v[k] = assign[((u64)col * 8 + k) * cap + row];
    }
};

extern "C" int32_t emu_eval(const mh_node* nodes, const uint64_t* offs, uint32_t n_tapes,
                            const uint32_t* consts, uint32_t n_consts, uint32_t n_vars,
                            uint32_t tape, const uint32_t* assign, uint64_t rows, uint32_t* out,
                            uint32_t* n_regs_out, char* err, int errlen) {
    std::vector<uint32_t> dconsts, words;
    mh::ConstIndex dindex;
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
    const u32* ip = words.data() + 2ull * sel_off;
    const u32 nrx = mh_nrx_of(sel.n_regs);
    for (uint64_t row = 0; row < rows; ++row) {
        HostMachine m;
        memset(m.R, 0xCD, sizeof(m.R));  // poison: reads of never-written registers show up
        m.nrx_ = nrx;
        m.slots = ip;
        m.assign = assign;
        m.cap = rows;
        m.row = row;
        for (uint32_t v = 0; v < n_pre; ++v)
            for (int k = 0; k < 8; ++k) m.R[v][k] = assign[((u64)v * 8 + k) * rows + row];
        u32 s = 0;
        for (;;) {
            if (s >= sel.n_insns) {
                snprintf(err, errlen, "tape ran past its slots");
                return MH_E_INVALID;
            }
            const u32 w0 = ip[2 * s], w1 = ip[2 * s + 1];
            const u32 op = w1 & 0xFFu;
            if (op == D_END) break;
            if (op == D_WINDOW) {
                s = (s / MH_WINDOW + 1) * MH_WINDOW;
                continue;
            }
            s += step<F_DIV | F_KECCAK | F_EVM, true>(m, w0, w1, s);
            // the device leaves the tape at a D_BANDZ whose conjunction is 0 in every lane of a
            // wave; here in the lane alone (stricter: the root must then be 0 for this row)
            if (op == D_BANDZ && (m.R[nrx][0] & 1u) == 0) break;
            if (mh_produces_bool(op) && m.R[nrx][0] > 1u) {
                // the device's Bool handlers assume canonical operands (dev_isa.h): a
                // producer that breaks it must fail here, not only on the GPU
                snprintf(err, errlen, "non-canonical Bool from op %u at slot %u", op, s);
                return MH_E_INVALID;
            }
        }
        u32 res[8];
        memcpy(res, m.R[nrx], 32);
        if (sel.root_bool) {
            res[0] &= 1u;
            for (int k = 1; k < 8; ++k) res[k] = 0;
        }
        for (int k = 0; k < 8; ++k) out[(u64)k * rows + row] = res[k];
    }
    return MH_OK;
}

// Compile every tape and return the concatenated slot words (test-only: instruction-mix
// analysis, scripts/isa_mix.py).  *n_words_out is set to the number of u32 words needed; the
// words are copied when it fits in cap.
extern "C" int32_t emu_compile_words(const mh_node* nodes, const uint64_t* offs, uint32_t n_tapes,
                                     const uint32_t* consts, uint32_t n_consts, uint32_t n_vars,
                                     uint32_t* out, uint64_t cap, uint64_t* n_words_out,
                                     uint32_t* nrx_out, char* err, int errlen) {
    std::vector<uint32_t> dconsts, words;
    mh::ConstIndex dindex;
    for (uint32_t t = 0; t < n_tapes; ++t) {
        CompiledTape ct;
        std::string e;
        int32_t r = compile_tape(nodes + offs[t], (size_t)(offs[t + 1] - offs[t]), consts,
                                 n_consts, n_vars, dconsts, dindex, words, ct, e);
        if (r != MH_OK) {
            snprintf(err, errlen, "tape %u: %s", t, e.c_str());
            return r;
        }
        if (nrx_out) nrx_out[t] = mh_nrx_of(ct.n_regs);
    }
    *n_words_out = words.size();
    if (words.size() <= cap) memcpy(out, words.data(), words.size() * 4);
    return MH_OK;
}

// compile.h split_conjunction, for tests/test_split.py: the parts back to back in `out` (cap
// nodes), part p = out[offs[p] .. offs[p + 1]).  Returns the parts (0: not split), -1 when `out`
// is too small.
extern "C" int32_t emu_split(const mh_node* nodes, uint32_t n, uint32_t want, mh_node* out,
                             uint64_t cap, uint64_t* offs) {
    std::vector<std::vector<mh_node>> parts;
    if (!mh::split_conjunction(nodes, n, want, parts)) return 0;
    uint64_t at = 0;
    offs[0] = 0;
    for (size_t p = 0; p < parts.size(); ++p) {
        if (at + parts[p].size() > cap) return -1;
        memcpy(out + at, parts[p].data(), parts[p].size() * sizeof(mh_node));
        at += parts[p].size();
        offs[p + 1] = at;
    }
    return (int32_t)parts.size();
}
