// Tape compiler interface (host side of libmythril_hip).
#pragma once
#include <stdint.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/mythril_hip.h"
#include "dev_isa.h"

namespace mh {

struct CompiledTape {
    uint32_t n_nodes = 0;
    uint32_t n_insns = 0;
    uint32_t n_regs = 0;
    uint32_t root_bool = 0;
    uint32_t features = 0;
    uint64_t alg_ops = 0;
};

// One instruction of a lowered tape in SSA form (before the interpreter's accumulator pass and
// register allocation): device op (dev_isa.h; the *_R form of an asm pair, the inline constant
// in `cidx`), destination and operand virtual registers (-1 = none).  D_ITE here is the generic
// select (a = cond, b = then, c = else).  Shared by the interpreter's encoder (compile.cpp) and
// the native-code JIT (jit.cpp).
struct SsaInsn {
    uint8_t op;
    int d, a, b, c;
    uint32_t width;   // 1..256
    uint32_t aux;     // immediate (shift amount, SEXT source width, LOADVAR column)
    int cidx;         // inline constant y (index into the 8-limb constant pool), -1 = none
    uint32_t w1raw;   // D_KECCAK second word (lengths)
};

struct SsaTape {
    std::vector<SsaInsn> code;
    int root = -1;        // the root's virtual register
    int n_vregs = 0;      // virtual registers 0..n_pinned-1 are the pinned assignment columns
    int n_pinned = 0;
    uint32_t features = 0;
    bool root_bool = false;
    uint64_t alg_ops = 0;
};

// Deduplicating index of the 8-limb constant pool (limbs -> pool row)
struct ConstKey {
    uint32_t w[8];
    bool operator==(const ConstKey& o) const {
        for (int k = 0; k < 8; ++k)
            if (w[k] != o.w[k]) return false;
        return true;
    }
};
struct ConstKeyHash {
    size_t operator()(const ConstKey& k) const {
        uint64_t h = 1469598103934665603ull;
        for (uint32_t x : k.w) h = (h ^ x) * 1099511628211ull;
        return (size_t)(h ^ (h >> 29));
    }
};
using ConstIndex = std::unordered_map<ConstKey, uint32_t, ConstKeyHash>;

// Lower one tape to SSA, fold constants and drop dead code (compile_tape's first half).
// value_numbering merges identical instructions (the native code's register file has room for
// the longer live ranges; the interpreter's does not); kVnNoLoads merges all but the column loads
// (D_LOADVAR: every use loads again, the native code's fallback under register pressure).
// jit_forms restates the complex ops the
// native code has no machine code for (EVM SIGNEXTEND / BYTE / ADDMOD, EXP by a constant, the
// overflow predicates) on ops it has; the columns of a tape set over MH_MAX_PRELOAD columns stay
// D_LOADVAR (the native code loads the limbs each use demands).
int32_t lower_tape_ssa(const mh_node* nodes, size_t n_nodes, const uint32_t* consts,
                       uint32_t n_consts, uint32_t n_vars, std::vector<uint32_t>& dconsts,
                       ConstIndex& dconst_index, SsaTape& out,
                       std::string& err, int value_numbering = 0, bool jit_forms = false,
                       bool hold_vars = false);
constexpr int kVnAll = 1, kVnNoLoads = 2;

// Bool values of the SSA registers `want` on n_rows sample rows (each pinned column a uniform
// 256-bit value from a splitmix64 stream seeded by `seed`), by the device's own instruction
// semantics (exec.h step).  out[i][r] = value of want[i] on row r.  For ordering conjuncts
// (jit.cpp schedule_conjuncts); never part of a result.
void sample_bools(const SsaTape& st, const std::vector<uint32_t>& pool, uint32_t n_rows,
                  uint64_t seed, const std::vector<int>& want,
                  std::vector<std::vector<uint8_t>>& out);

// Lower one tape.  Appends its instruction words (2 per instruction) to `words` and any new
// constants to the shared device pool `dconsts` (8 limbs each, deduplicated via dconst_index).
int32_t compile_tape(const mh_node* nodes, size_t n_nodes, const uint32_t* consts,
                     uint32_t n_consts, uint32_t n_vars, std::vector<uint32_t>& dconsts,
                     ConstIndex& dconst_index,
                     std::vector<uint32_t>& words, CompiledTape& out, std::string& err);

// A tape whose root is a conjunction, cut into at most `want` parts of consecutive conjuncts of
// about equal cone size: each part the nodes its conjuncts reach, in tape order and re-indexed,
// then the AND of its conjuncts, so a row satisfies the tape iff it satisfies every part (the
// conjunct-parallel short runs of mh_run_async).  False when the root has fewer than two
// conjuncts or `want` < 2.
bool split_conjunction(const mh_node* nodes, uint32_t n_nodes, uint32_t want,
                       std::vector<std::vector<mh_node>>& out);

}  // namespace mh
