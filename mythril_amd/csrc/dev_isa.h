// Device instruction set of the sieve interpreter (internal; the public IR is mh_node in
// include/mythril_hip.h).  mh_tapes_compile() lowers each IR tape to this form: a register
// machine over MH_NUM_REGS registers of 8 x u32 limbs (least significant limb first), with
// assignment columns pinned in the first registers.
//
// Encoding: two u32 words per instruction.
//   w0 = op | d << 8 | a << 16 | b << 24
//   w1 = c | width << 8 | aux << 17        (width 1..256; aux 15 bits)
//   D_LOADC uses all of w1 as the constant-pool index.
// Op ranges select the operand class the interpreter reads/writes:
//   [1,32)   bv x bv -> bv        reads R[a], R[b]; writes 8 limbs of R[d]
//   [32,48)  bv -> bv             reads R[a]
//   [48,64)  bv x bv -> Bool      writes limb 0 of R[d] (0/1); Bool registers only use limb 0
//   [64,80)  Bool ops             read/write limb 0
//   [80,96)  others (ite, loads, keccak)
#pragma once
#include <stdint.h>

#ifndef MH_NUM_REGS
#define MH_NUM_REGS 16
#endif
#define MH_MAX_PRELOAD 4   // assignment columns kept resident in R0..R3 for the whole launch

enum mh_dop : uint8_t {
    D_NOP = 0,
    // bv x bv -> bv
    D_ADD = 1, D_SUB, D_MUL, D_AND, D_OR, D_XOR, D_SHL, D_LSHR, D_ASHR,
    D_UDIV, D_UREM, D_SDIV, D_SREM, D_SMOD, D_EXP, D_SIGNEXT, D_BYTE,
    D_CONCAT,                       // a = high, b = low, aux = width of b
    // bv -> bv
    D_NEG = 32, D_NOT, D_MOV, D_SHLI, D_LSHRI, D_ASHRI, D_EXTRACT, D_SEXT,
    // bv x bv -> Bool
    D_EQ = 48, D_ULT, D_ULE, D_SLT, D_SLE, D_UADD_NOOVFL, D_UMUL_NOOVFL,
    // Bool
    D_BAND = 64, D_BOR, D_BXOR, D_BEQ, D_BNOT, D_TRUE, D_FALSE,
    // others
    D_ITE = 80,                     // a = Bool cond, b = then, c = else (bv)
    D_BITE,                         // Bool-valued ite
    D_LOADC,                        // w1 = const index
    D_LOADVAR,                      // aux = column
    D_KECCAK                        // message = concat of up to 3 byte-aligned pieces a,b,c;
                                    // w1: c | n0 << 8 | n1 << 14 | n2 << 20 | npieces << 26
                                    //     (n_i = bytes of piece i, 1..32)
};

enum { D_CLASS_VVV = 0, D_CLASS_VV = 1, D_CLASS_VVB = 2, D_CLASS_BOOL = 3, D_CLASS_MISC = 4 };

static inline int mh_dop_class(uint32_t op) {
    return op < 32 ? D_CLASS_VVV : op < 48 ? D_CLASS_VV : op < 64 ? D_CLASS_VVB
         : op < 80 ? D_CLASS_BOOL : D_CLASS_MISC;
}

// Feature bits (mh_tape_info.features) — select the kernel variant.
enum { F_DIV = 1, F_KECCAK = 2, F_EVM = 4 };

// Per-tape header in the device tape table.
struct mh_dev_tape {
    uint32_t insn_off;   // first instruction (in instructions, not words)
    uint32_t n_insns;
    uint32_t root_reg;
    uint32_t root_bool;  // 1 if the root is Bool
};
