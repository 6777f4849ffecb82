// Native-code path for throughput launches (no reference counterpart: it replaces the
// interpreter's per-instruction dispatch for mh_run over a resident tape set).
//
// Each tape is compiled from its SSA form (compile.h lower_tape_ssa) into straight-line gfx950
// machine code with fixed registers: every 256-bit value is 8 limbs, each limb either a
// compile-time constant (no register, no instruction) or one VGPR; Bool values are 64-bit lane
// masks in SGPR pairs (compares leave their result in VCC, the conjunction at the root is
// s_and_b64).  Only the limbs a consumer demands are computed (an AND with a 160-bit mask never
// computes the top three limbs of its operand), shifts by constants are register renaming plus
// at most one v_alignbit per limb, and the division family runs in one shared subroutine.
//
// The machine code of a whole tape set is one code object: a single kernel whose workgroups
// are a 2-D grid (x = block of rows, y = group of tapes).  A group is a run of consecutive tapes
// whose code fits the instruction cache; each wave loads its rows' assignment columns into VGPRs
// once per 64-row chunk and runs every tape of its group over them, so the tape code is fetched
// from the instruction cache rather than decoded per instruction as the interpreter does.
//
// Text is assembled in-process by comgr (jit_comgr.cpp) and loaded with hipModuleLoadData
// (capi.cpp).  The instruction list (MI) is also what the test-only host emulator runs
// (tests/native/jit_emu.cpp), so the emitted code is checked against the oracle without a GPU.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "compile.h"

namespace mh {
namespace jit {

// ---- machine instructions ---------------------------------------------------------------
enum OKind : uint8_t { O_NONE, O_V, O_S, O_VCC, O_IMM, O_LABEL, O_EXEC, O_FONE /* f64 1.0 */ };

struct Opnd {
    uint8_t k = O_NONE;
    uint8_t n = 1;        // registers in the range (1, 2 = pair)
    uint8_t neg = 0;      // f64 source negation modifier
    uint32_t v = 0;       // register number / immediate bits / label id
};

inline Opnd V(uint32_t r, uint8_t n = 1) { Opnd o; o.k = O_V; o.v = r; o.n = n; return o; }
inline Opnd S(uint32_t r, uint8_t n = 1) { Opnd o; o.k = O_S; o.v = r; o.n = n; return o; }
inline Opnd VCC() { Opnd o; o.k = O_VCC; o.n = 2; return o; }
inline Opnd EXEC() { Opnd o; o.k = O_EXEC; o.n = 2; return o; }
inline Opnd IMM(uint32_t x) { Opnd o; o.k = O_IMM; o.v = x; return o; }
inline Opnd LBL(uint32_t id) { Opnd o; o.k = O_LABEL; o.v = id; return o; }
inline Opnd FONE() { Opnd o; o.k = O_FONE; return o; }
inline Opnd NEG(Opnd o) { o.neg = 1; return o; }

// inline constants of 32-bit integer operands (no literal dword, no constant-bus use)
inline bool is_inline(uint32_t x) { return x <= 64u || x >= 0xFFFFFFF0u; }

enum Op : uint16_t {
    // VALU (e64 flag selects the VOP3 encoding where both exist)
    M_V_MOV, M_V_ADD_U32, M_V_SUB_U32, M_V_SUBREV_U32,
    M_V_ADD_CO, M_V_ADDC_CO, M_V_SUB_CO, M_V_SUBB_CO, M_V_SUBREV_CO, M_V_SUBBREV_CO,
    M_V_AND, M_V_OR, M_V_XOR, M_V_NOT, M_V_OR3, M_V_XNOR,
    M_V_ALIGNBIT, M_V_LSHLREV, M_V_LSHRREV, M_V_ASHRREV,
    M_V_CNDMASK,   // d = mask ? src1 : src0
    M_V_CMP_EQ, M_V_CMP_NE, M_V_CMP_LT, M_V_CMP_LE, M_V_CMP_GT, M_V_CMP_GE,  // u32
    M_V_CMP_LT_I32, M_V_CMP_GT_I32,
    M_V_MAD_U64_U32,
    M_V_LSHL_ADD,    // d = (s0 << s1) + s2
    M_V_PERM,        // v_perm_b32 d, s0, s1, sel (byte select from {s0, s1})
    M_V_BFI,         // d = (s0 & s1) | (~s0 & s2)
    M_V_BITOP3,      // gfx950: d = bit i of table o[4] at index s0 << 2 | s1 << 1 | s2 (per bit)
    // f32 (the division's small-quotient estimate)
    M_V_CVT_F32_U32, M_V_FMA_F32, M_V_RCP_F32, M_V_MUL_F32, M_V_CVT_U32_F32, M_V_FRACT_F32,
    M_V_CMP_GT_F32, M_V_CMP_LE_F32,  // VCC / SGPR pair = s0 > s1 / s0 <= s1
    M_V_CVT_F64_U32, M_V_FMA_F64, M_V_RCP_F64, M_V_MUL_F64, M_V_MIN_F64, M_V_CVT_U32_F64,
    M_V_FRACT_F64,
    M_V_CMP_LE_F64,
    // SALU
    M_S_MOV_B32, M_S_MOV_B64, M_S_AND_B64, M_S_OR_B64, M_S_XOR_B64, M_S_XNOR_B64,
    M_S_ANDN2_B64, M_S_ORN2_B64, M_S_NOT_B64, M_S_CMP_EQ_U64, M_S_CMP_LG_U64, M_S_CMP_EQ_U32,
    M_S_CMP_LT_U32,
    // control
    M_S_CBRANCH_SCC0, M_S_CBRANCH_SCC1, M_S_BRANCH, M_LABEL, M_S_NOP,
    M_CALL_DIV,    // s_getpc / s_add / s_swappc into the division subroutine
    M_RET,         // s_setpc_b64 of the return address (end of the subroutine)
    M_CALL_KEC,    // the same into the Keccak-f[1600] subroutine
    // LDS (the variable-shift window, see R_LDS)
    M_DS_WRITE2ST64,  // addr, data0, data1, IMM offset0, IMM offset1 (units of 256 B)
    M_DS_READ2ST64,   // dst pair, addr, IMM offset0, IMM offset1 (units of 256 B)
    M_DS_READ_B32,    // dst, addr, IMM offset (bytes)
    M_S_WAITCNT_LGKM, // IMM count
    // assignment columns that are not pinned (tape sets over 4 columns): limb j of this lane's
    // row, loaded on use -- s[28:29] = assign + j * stride, global_load_dword dst, v2, s[28:29]
    M_LOADCOL,        // dst, IMM j (= 8 * column + limb)
    M_S_WAITCNT_VM,   // IMM count
    M_NUM_OPS
};

struct MI {
    uint16_t op;
    uint8_t e64 = 0;
    uint8_t tag = 0xFF;   // SSA op kind that emitted it (diagnostics; 0xFF = none)
    Opnd o[5];
};

// Assignment columns held in v[R_COL0..] for a whole chunk: every column of a tape set of at most
// this many columns; none above it (the tape code loads the limbs it demands, M_LOADCOL).
constexpr uint32_t kMaxPinnedCols = 4;
inline uint32_t pinned_cols(uint32_t n_vars) { return n_vars <= kMaxPinnedCols ? n_vars : 0u; }

// ---- register map of the generated kernel (documented in jit.cpp) ----------------------
enum : uint32_t {
    R_LDS = 7,           // this lane's LDS byte address of word 0 of its shift window
    R_COL0 = 8,          // assignment column v limb k is v[R_COL0 + 8 v + k]
    R_DIV0 = 40,         // division subroutine registers v[40..79]
    R_DY = 40, R_DR = 48, R_DQ = 56, R_FY = 64, R_FR = 66, R_FC = 68, R_FT = 70,
    R_CARRY = 72, R_MAD = 74, R_C = 76, R_T1 = 77, R_SX = 78, R_SY = 79,
    R_TEMP0 = 80,        // first free VGPR of a tape that can call the division subroutine
    R_TEMP_NODIV = 40,   // ... and of one that cannot
    R_KEC0 = 40,         // Keccak-f[1600] subroutine: lane i of the state in v[40 + 2i] (low
    N_KEC_REGS = 62,     // half), v[41 + 2i] (high) on entry; 12 spare registers up to v101
    R_TEMP_KEC = 102,    // first free VGPR of a tape that hashes
    // SGPRs
    S_VALID = 30,        // valid-lane mask of the current 64-row chunk
    S_RES = 32,          // the tape's root mask
    S_SCRATCH = 34,      // s[34:35]: scratch between tapes (short-circuit tests inside one)
    S_BOOL0 = 40, N_BOOL_PAIRS = 16,   // Bool lane masks s[40:71]
    S_KSTAGE = 72, N_KSTAGE = 4,       // constant staging s72..s75
    S_DIV_RA = 76, S_DIV_TGT = 78, S_DIV_KIND = 80, S_DIV_YNZ = 82, S_DIV_DUMMY = 84,
    S_DIV_MSK = 86, S_DIV_TM = 88, S_DIV_F64K = 90,
    S_PERM_SEL = 92,     // v_perm_b32 byte-swap selector
    S_NEXT_FREE = 93,
};

// Variable shifts go through LDS: each lane owns a window of LDS_WORDS 32-bit words, word w of
// lane l of wave i at byte i * LDS_WAVE_BYTES + w * 256 + 4 l (consecutive lanes, consecutive
// banks).  Words [0, LDS_D) and [LDS_D + 8, LDS_WORDS) stay zero (written once by the kernel
// prologue); a shift writes its operand's 8 limbs at [LDS_D, LDS_D + 8) and reads 9 words from
// a per-lane base moved by the limb part of the amount.
enum : uint32_t {
    LDS_D = 8, LDS_WORDS = 25, LDS_WAVE_BYTES = LDS_WORDS * 256, LDS_WG_BYTES = 4 * LDS_WAVE_BYTES,
};

struct TapeCode {
    bool ok = false;
    std::string why;            // reason the tape stays on the interpreter
    std::vector<MI> code;       // body: root mask in s[S_RES:S_RES+1] (or the root value)
    uint32_t max_vgpr = 0;      // highest VGPR used + 1
    bool calls_div = false;
    bool uses_lds = false;      // variable shifts (the kernel then reserves LDS_WG_BYTES)
    bool calls_kec = false;
    bool root_bool = true;
    uint32_t root_limbs[8];     // values mode: VGPR of each root limb, or ~0u (then constant)
    uint32_t root_const[8];
    uint32_t n_valu = 0, n_valu_wide = 0, n_salu = 0;  // static counts (wide = 4-cycle class)
    uint64_t alg_ops = 0;
};

struct Options {
    uint32_t max_vgpr = 128;    // VGPR budget of the kernel (occupancy: 512 / max_vgpr waves per
                                // SIMD, at most 8; 96..256 -- gfx950 has 256 architectural VGPRs)
    uint32_t max_vgpr_keccak = 168;  // ... of tapes that hash (the state holds 62 VGPRs)
    // Short-circuit conjunctions: a root AND chain is evaluated conjunct by conjunct (cheapest
    // and most selective first, schedule_conjuncts) and the wave leaves the tape as soon as no
    // valid lane (s[30:31]) satisfies the conjuncts so far; its root mask is then 0, the value
    // every skipped row has, so counts, first hits and Bool root values are unchanged.
    bool short_circuit = true;
    // Conjunct order: pass rates measured on this many sample rows (uniform 256-bit columns,
    // compile.h sample_bools); 0 = static guesses only.
    uint32_t sample_rows = 256;
    // Producers of division operands write the subroutine's input registers directly where the
    // copy at the call site would be the value's last use (coalesce_div_moves).
    bool coalesce = true;
    // Assemble the module texts (comgr).  false: emission and module text only -- enough for the
    // code id (Built::text_hash), with no assembler and no device.
    bool assemble = true;
};

// The SSA of `st` reordered for short-circuit evaluation of its root conjunction (insn_cost: VALU
// per SSA instruction from a source-order emission; null = a static per-op table).  Returns false
// (out untouched) when the root is not an AND of at least two conjuncts.  check[v] = 1 marks the
// virtual registers (the first conjunct, then each partial conjunction) after which the emitter
// tests the running mask.
bool schedule_conjuncts(const SsaTape& st, const std::vector<uint32_t>& pool,
                        uint32_t sample_rows, const std::vector<double>* insn_cost, SsaTape& out,
                        std::vector<uint8_t>& check);

// Emit one tape (SSA after folding) with constants from `pool` (8 limbs per entry).
TapeCode emit_tape(const SsaTape& st, const std::vector<uint32_t>& pool, uint32_t n_vars,
                   const Options& opt);
TapeCode emit_tape_body(const SsaTape& st, const std::vector<uint32_t>& pool, uint32_t n_vars,
                        const Options& opt);  // emit_tape without the copy coalescing

// The division subroutine (x in v[R_DR..], y in v[R_DY..], kind in S_DIV_KIND: 0 udiv, 1 urem,
// 2 sdiv, 3 srem, 4 smod; result in v[R_DQ..]).
std::vector<MI> div_routine();

// The Keccak-f[1600] subroutine (fully unrolled, registers renamed from round to round): state
// on entry as R_KEC0 says; on return lane i half h is in v[out[2 i + h]] for the first 4 lanes.
struct KecCode {
    std::vector<MI> code;
    uint32_t out[8];
};
const KecCode& kec_routine();

// Assembly text of one instruction / a list (labels get `prefix`).
std::string print(const MI& m, const std::string& prefix);
void print_list(const std::vector<MI>& code, const std::string& prefix, std::string& out);

// The whole code object source for tapes `codes` (only the ok ones are included), grouped by
// instruction bytes; tape_ids[i] is the result slot of codes[i].
struct Module {
    std::string text;
    std::vector<uint32_t> group_first;   // index into the jitted list of each group's first tape
    std::vector<uint32_t> group_count;
    uint32_t max_vgpr = 0;
    uint32_t n_sgpr = 0;
};
// values = true: every tape stores its root value (8 limbs per row, the parity path) instead of
// counting hits.
uint32_t default_group_bytes();  // 96 KB, or MH_JIT_GROUP_KB
Module build_module(const std::vector<const TapeCode*>& codes,
                    const std::vector<uint32_t>& tape_ids, uint32_t n_vars, bool values,
                    uint32_t group_bytes);

// Diagnostics: tapes whose short-circuit order ran out of registers and kept the source order
// (since the last reset).
uint64_t sc_fallbacks(bool reset);

// Diagnostics: static VALU (and 4-cycle VALU) emitted per SSA op kind since the last reset
// (not thread safe; tests / scripts only).
void op_stats(uint64_t* valu, uint64_t* wide, uint64_t* count, bool reset);

// Estimated machine-code bytes of a tape body.
uint32_t code_bytes(const TapeCode& tc);

// comgr: assemble + link `text` into a gfx950 code object (jit_comgr.cpp).
bool assemble(const std::string& text, std::vector<char>& hsaco, std::string& log);

// A whole tape set to code objects: tapes are lowered and emitted over `threads` contiguous
// slices, binned into occupancy classes by the VGPRs their code object needs
// (occupancy_classes), and each class cut into pieces of about n_tapes / threads tapes; each
// piece becomes one code object (count kernel, and the values kernel when asked), assembled on
// `threads` threads.  No HIP calls: capi.cpp loads the results.
struct Built {
    std::vector<char> hsaco, hsaco_values;
    uint32_t n_groups = 0;
    uint32_t max_vgpr = 0;
    std::vector<uint32_t> tape_ids;    // jitted tapes of this slice
    uint64_t text_hash = 0;            // FNV-1a 64 of the count kernel's module text
    std::string err;
};
struct BuildStats {
    std::vector<uint8_t> jitted;       // per tape
    std::vector<std::string> why;      // per tape: reason when not jitted
    uint64_t code_bytes = 0, valu_static = 0, valu_wide_static = 0;
};
uint32_t module_vgprs(const TapeCode& tc, uint32_t n_vars);
std::vector<uint32_t> occupancy_classes(uint32_t budget);  // ascending ceilings, last = budget
bool build_tapeset(const mh_node* nodes, const uint64_t* offs, uint32_t n_tapes,
                   const uint32_t* consts, uint32_t n_consts, uint32_t n_vars, bool values,
                   const Options& opt, uint32_t threads, std::vector<Built>& out,
                   BuildStats& stats, std::string& err);
// Build threads mh_tapes_jit uses (code objects per occupancy class): min(4, hardware threads),
// or MH_JIT_THREADS.  The cut into code objects, hence the code id, depends on it.
uint32_t default_threads();
// Identifier of the emitted code of a build: FNV-1a 64 over the code objects' module texts in
// order (what the GPU executes, independent of the host sources around it).
uint64_t code_id(const std::vector<Built>& built);

// Kernel arguments (the kernarg layout build_module's prologue reads).
struct KernArgs {
    uint64_t assign;       // 0x00
    uint64_t capacity;     // 0x08
    uint64_t row_first;    // 0x10
    uint64_t row_count;    // 0x18
    uint64_t index_base;   // 0x20
    uint64_t first_hit;    // 0x28 (u64 per tape id, already offset by -result_base)
    uint64_t hit_count;    // 0x30
    uint32_t n_rowblocks;  // 0x38
    uint32_t rows_per_wg;  // 0x3c (multiple of 256)
    uint64_t values_out;   // 0x40 (0: count mode)
    uint32_t group_first;  // 0x48
    uint32_t mode;         // 0x4c (0 count all, 1 first hit)
};
static_assert(sizeof(KernArgs) == 0x50, "kernarg layout");

}  // namespace jit
}  // namespace mh
