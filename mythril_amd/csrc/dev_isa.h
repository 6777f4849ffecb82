// Device instruction set of the sieve interpreter (internal; the public IR is mh_node in
// include/mythril_hip.h).  mh_tapes_compile() lowers each IR tape to this form: a register
// machine over MH_NUM_REGS registers of 8 x u32 limbs (least significant limb first), with
// assignment columns pinned in the first registers.
//
// Encoding: two u32 words per instruction.
//   w0 = op | d << 8 | a << 16 | b << 24
//   w1 = flags | width << 2 | aux << 11      (flags bit 0: operand a is constant aux,
//                                              bit 1: operand b is constant aux; width 1..256)
//   D_ITE: aux = c (else register).  D_LOADC: aux = constant index.
//   D_KECCAK: w1 = c | n0 << 8 | n1 << 14 | n2 << 20 | npieces << 26 (n_i = bytes of piece i).
// Constant operands are read by the scalar unit straight from the constant pool: no register,
// no load instruction, no register-file traffic for them.
#pragma once
#include <stdint.h>

#ifndef MH_NUM_REGS
#define MH_NUM_REGS 12
#endif
#define MH_MAX_PRELOAD 4   // assignment columns kept resident in R0..R3 for the whole launch

enum mh_dop : uint8_t {
    D_NOP = 0,
    // bv x bv -> bv
    D_ADD, D_SUB, D_MUL, D_AND, D_OR, D_XOR, D_SHL, D_LSHR, D_ASHR,
    D_UDIV, D_UREM, D_SDIV, D_SREM, D_SMOD, D_EXP, D_SIGNEXT, D_BYTE,
    D_CONCAT,                       // a = high, b = low, aux = width of b
    // bv -> bv
    D_NEG, D_NOT, D_MOV, D_SHLI, D_LSHRI, D_ASHRI, D_EXTRACT, D_SEXT,
    // bv x bv -> Bool (0/1 in limb 0)
    D_EQ, D_ULT, D_ULE, D_SLT, D_SLE, D_UADD_NOOVFL, D_UMUL_NOOVFL,
    // Bool
    D_BAND, D_BOR, D_BXOR, D_BEQ, D_BNOT, D_TRUE, D_FALSE,
    // others
    D_ITE,                          // a = Bool cond, b = then, aux = else register
    D_BITE,                         // Bool-valued ite, aux = else register
    D_LOADC,                        // aux = constant index
    D_LOADVAR,                      // aux = column
    D_KECCAK,                       // message = concat of up to 3 byte-aligned pieces a, b, c
    D_NUM_OPS
};

static_assert(D_NUM_OPS <= 64, "operand masks are 64-bit");

#define MH_BIT(op) (1ull << (op))
// ops that read operand a / operand b as a full 8-limb value
#define MH_READS_A                                                                             \
    (MH_BIT(D_ADD) | MH_BIT(D_SUB) | MH_BIT(D_MUL) | MH_BIT(D_AND) | MH_BIT(D_OR) |          \
     MH_BIT(D_XOR) | MH_BIT(D_SHL) | MH_BIT(D_LSHR) | MH_BIT(D_ASHR) | MH_BIT(D_UDIV) |      \
     MH_BIT(D_UREM) | MH_BIT(D_SDIV) | MH_BIT(D_SREM) | MH_BIT(D_SMOD) | MH_BIT(D_EXP) |     \
     MH_BIT(D_SIGNEXT) | MH_BIT(D_BYTE) | MH_BIT(D_CONCAT) | MH_BIT(D_NEG) | MH_BIT(D_NOT) | \
     MH_BIT(D_MOV) | MH_BIT(D_SHLI) | MH_BIT(D_LSHRI) | MH_BIT(D_ASHRI) | MH_BIT(D_EXTRACT) | \
     MH_BIT(D_SEXT) | MH_BIT(D_EQ) | MH_BIT(D_ULT) | MH_BIT(D_ULE) | MH_BIT(D_SLT) |         \
     MH_BIT(D_SLE) | MH_BIT(D_UADD_NOOVFL) | MH_BIT(D_UMUL_NOOVFL) | MH_BIT(D_KECCAK))
#define MH_READS_B                                                                             \
    (MH_BIT(D_ADD) | MH_BIT(D_SUB) | MH_BIT(D_MUL) | MH_BIT(D_AND) | MH_BIT(D_OR) |          \
     MH_BIT(D_XOR) | MH_BIT(D_SHL) | MH_BIT(D_LSHR) | MH_BIT(D_ASHR) | MH_BIT(D_UDIV) |      \
     MH_BIT(D_UREM) | MH_BIT(D_SDIV) | MH_BIT(D_SREM) | MH_BIT(D_SMOD) | MH_BIT(D_EXP) |     \
     MH_BIT(D_SIGNEXT) | MH_BIT(D_BYTE) | MH_BIT(D_CONCAT) | MH_BIT(D_EQ) | MH_BIT(D_ULT) |  \
     MH_BIT(D_ULE) | MH_BIT(D_SLT) | MH_BIT(D_SLE) | MH_BIT(D_UADD_NOOVFL) |                 \
     MH_BIT(D_UMUL_NOOVFL) | MH_BIT(D_ITE) | MH_BIT(D_KECCAK))
// ops whose operands are Bools (limb 0 only)
#define MH_BOOL_IN                                                                             \
    (MH_BIT(D_BAND) | MH_BIT(D_BOR) | MH_BIT(D_BXOR) | MH_BIT(D_BEQ) | MH_BIT(D_BNOT) |      \
     MH_BIT(D_ITE) | MH_BIT(D_BITE))
// ops that may take a constant operand (flags) — binary ops without other uses of aux
#define MH_CONST_OPERAND_OK                                                                    \
    (MH_BIT(D_ADD) | MH_BIT(D_SUB) | MH_BIT(D_MUL) | MH_BIT(D_AND) | MH_BIT(D_OR) |          \
     MH_BIT(D_XOR) | MH_BIT(D_SHL) | MH_BIT(D_LSHR) | MH_BIT(D_ASHR) | MH_BIT(D_UDIV) |      \
     MH_BIT(D_UREM) | MH_BIT(D_SDIV) | MH_BIT(D_SREM) | MH_BIT(D_SMOD) | MH_BIT(D_EXP) |     \
     MH_BIT(D_SIGNEXT) | MH_BIT(D_BYTE) | MH_BIT(D_EQ) | MH_BIT(D_ULT) | MH_BIT(D_ULE) |     \
     MH_BIT(D_SLT) | MH_BIT(D_SLE) | MH_BIT(D_UADD_NOOVFL) | MH_BIT(D_UMUL_NOOVFL))

enum { F_ACONST = 1, F_BCONST = 2 };
#define MH_AUX_MAX ((1u << 21) - 1)

// Feature bits (mh_tape_info.features) — select the kernel variant.
enum { F_DIV = 1, F_KECCAK = 2, F_EVM = 4 };

// Per-tape header in the device tape table.
struct mh_dev_tape {
    uint32_t insn_off;   // first instruction (in instructions, not words)
    uint32_t n_insns;
    uint32_t root_reg;
    uint32_t root_bool;  // 1 if the root is Bool
};
