// Device instruction set of the sieve interpreter (internal; the public IR is mh_node in
// include/mythril_hip.h).  mh_tapes_compile() lowers each IR tape to this form.
//
// Machine model.  A register file R[0..NRX] of 256-bit values held in VGPRs as 8 "limb planes"
// (plane k = limb k of every register, NRX+1 consecutive VGPRs), indexed by a wave-uniform
// register number through the GPR-index mode (s_set_gpr_idx_on).  The LAST register of every
// plane, R[NRX], is the ACCUMULATOR X.  Every instruction computes
//     X = f(R[a'], y, ...)        then      R[d'] = X
// where a' = NRX means "X itself" (the previous result, no load) and d' = NRX means "no write-back"
// (the copy X -> X is harmless), so operand load and write-back need no branch: the host picks
// the indices.  y is R[b] (the *_R forms) or a 256-bit constant stored INLINE in the instruction
// stream (the *_C forms: the 4 slots after the instruction hold limbs 0..7), read with v_readlane
// like the instruction itself, so no instruction waits on memory.  Assignment columns 0..3 are
// pinned in R0..R3.  NRX depends on the kernel variant (kernels.h) and is fixed at compile time.
//
// Encoding: a slot is two u32 words (w0, w1); an instruction is one slot (+4 constant slots).
//   w0 = a' | b << 8 | d' << 16 | c << 24       (c: ITE else register, KECCAK third piece)
//   w1 = op | width << 8 | aux << 17 | F_YC << 31
//        width 1..256 (9 bits); aux 14 bits: shift amount, SEXT source width, LOADVAR column
//        F_YC (complex ops only): y is the inline constant rather than R[b]
//   D_KECCAK: w1 = op | nw << 8 | full << 10: message = nw (1..3) left-aligned 32-byte words
//             X, R[b], R[c] (big-endian bytes, 0x01 pad already in place unless full = 1)
// Ops below D_FIRST_COMPLEX run in the hand-written assembly core (asm_core.inc, threaded
// code: one computed jump per instruction); the others in C++ (exec.h).  Narrow signed
// compares, sign extension and arithmetic shifts are lowered by the host onto asm ops
// (x ^ 2^(w-1) biasing), so only division, the overflow predicates, keccak and the EVM helpers
// need the C++ path.  Tapes are cut into
// windows of 64 slots (what one wave holds in two VGPRs); D_WINDOW ends a window that is not the
// tape's last, D_END ends the tape.  No instruction straddles a window.
// Bool values are 0/1 in limb 0 (other limbs undefined).  Values narrower than 256 bits are kept
// canonical (zero above the width); the host inserts AND_C masks where an op could overflow.
#pragma once
#include <stdint.h>

// the opcode helpers below are shared by the host (compiler, emulators) and the device's C++
// step() path (exec.h; the MH_ASM_CORE=0 build)
#if defined(__HIPCC__)
#define MH_ISA_FN static inline __host__ __device__
#else
#define MH_ISA_FN static inline
#endif

#define MH_MAX_PRELOAD 4   // assignment columns kept resident in R0..R3 for the whole launch
#define MH_NR_SMALL 7      // register-file sizes of the kernel variants (tapes bucketed by need);
#define MH_NR_MID 9
#define MH_NR_MAX 15       // the accumulator is register NR, so planes are NR+1 VGPRs (even:
                           // VGPR tuples are even-aligned on gfx950)
#define MH_WINDOW 64       // instruction slots per window

enum mh_dop : uint8_t {
    // ---- assembly core (threaded dispatch)
    D_EXIT = 0,  // leave the asm core (never emitted; table slot for every op >= D_FIRST_COMPLEX)
    D_NOP,       // X = R[a'], R[d'] = X   (loads, copies, root)
    D_ADD_R, D_ADD_C, D_SUB_R, D_SUB_C, D_RSUB_R, D_RSUB_C,  // mod 2^256 (host masks)
    D_AND_R, D_AND_C, D_OR_R, D_OR_C, D_XOR_R, D_XOR_C,
    D_EQ_R, D_EQ_C, D_ULT_R, D_ULT_C, D_UGT_R, D_UGT_C, D_ULE_R, D_ULE_C, D_UGE_R, D_UGE_C,
    D_SLT_R, D_SLT_C, D_SGT_R, D_SGT_C, D_SLE_R, D_SLE_C, D_SGE_R, D_SGE_C,  // 256-bit signed
    D_BAND, D_BOR, D_BXOR, D_BEQ, D_BNOT, D_TRUE, D_FALSE,   // y0 = R[b] limb 0
    D_ITE,    // X = R[a'] (then), cond = R[b] limb 0, else = R[c]
    D_ITEC,   // cond = R[a'] limb 0, then = R[b], else = R[c]
    D_BITE,   // Bool select: cond = R[a'], then = R[b] limb 0, else = R[c] limb 0
    D_LOADC,  // X = inline constant
    D_MUL_R, D_MUL_C,  // X = R[a'] * y mod 2^256 (host masks)
    D_SHL_V, D_LSHR_V, D_ASHR_V,  // 256-bit shifts by y (per lane; >= 256 saturates to 0 / fill)
    // 256-bit division family, SMT-LIB semantics (x / 0 = 2^256 - 1, x % 0 = x, signed forms by
    // the bvsdiv/bvsrem/bvsmod sign rules); narrower widths are sign-extended / masked by the host
    D_UDIV_R, D_UDIV_C, D_UREM_R, D_UREM_C, D_SDIV_R, D_SDIV_C, D_SREM_R, D_SREM_C,
    D_SMOD_R, D_SMOD_C,
    // X forms: the first operand is already in the accumulator and the result stays there
    // (a' = d' = X).  Same semantics as the base op; the handlers read y = R[b] directly through
    // the SRC1 index instead of copying it, and skip the write-back (mh_xform / mh_base_op).
    D_ADD_RX, D_ADD_CX, D_SUB_RX, D_SUB_CX, D_RSUB_RX, D_RSUB_CX,
    D_AND_RX, D_AND_CX, D_OR_RX, D_OR_CX, D_XOR_RX, D_XOR_CX,
    D_EQ_RX, D_EQ_CX, D_ULT_RX, D_ULT_CX, D_UGT_RX, D_UGT_CX, D_ULE_RX, D_ULE_CX,
    D_UGE_RX, D_UGE_CX, D_SLT_RX, D_SLT_CX, D_SGT_RX, D_SGT_CX, D_SLE_RX, D_SLE_CX,
    D_SGE_RX, D_SGE_CX,
    D_MUL_RX, D_MUL_CX, D_LOADC_X,
    // immediate shifts, one op per limb count (the limb offsets are static in the handler; the
    // result is always written back, d' = X being the harmless X -> X):
    //   D_SHR0 + q: X = R[a'] >> (32 q + aux)                        aux < 32
    //   D_SHL0 + p: X = R[a'] << (aux ? 32 p + 32 - aux : 32 (p + 1)) mod 2^256, aux < 32
    D_SHR0, D_SHR1, D_SHR2, D_SHR3, D_SHR4, D_SHR5, D_SHR6, D_SHR7,
    D_SHL0, D_SHL1, D_SHL2, D_SHL3, D_SHL4, D_SHL5, D_SHL6, D_SHL7,
    // short-circuit AND of a tape's root conjunction (compile.cpp short_circuit): X = R[a'] &
    // R[b] limb 0 like D_BAND, and when X is 0 in every lane the tape's root is 0 in every lane,
    // so the asm core leaves at this op and the driver ends the tape (X = 0 is the root)
    D_BANDZ,
    D_NUM_ASM,
    // ---- C++ (exec.h); y = R[b] or the inline constant (F_YC)
    D_FIRST_COMPLEX = 112,
    D_UADD_NOOVFL = D_FIRST_COMPLEX,  // z3 BVAddNoOverflow (unsigned) -> Bool
    D_UMUL_NOOVFL,                    // z3 BVMulNoOverflow (unsigned) -> Bool
    D_EXP, D_SIGNEXT, D_BYTE,        // EVM word ops (256-bit)
    D_KECCAK,
    D_LOADVAR,                     // X = assignment column aux (columns beyond the pinned ones)
    D_END,                         // end of tape: X holds the root
    D_WINDOW,                      // end of a 64-slot window: continue with the next one
    D_ADDMOD, D_MULMOD,            // EVM ADDMOD / MULMOD: (X op y) mod R[c], exact; aux bit 0:
                                   // R[c] == 0 gives the low 256 bits of X op y (else 0)
    D_NUM_OPS
};

static_assert(D_NUM_ASM <= D_FIRST_COMPLEX, "asm opcode space");

// the base op of an X form (identity for every other op)
MH_ISA_FN unsigned mh_base_op(unsigned op) {
    if (op >= D_ADD_RX && op <= D_SGE_CX) return D_ADD_R + (op - D_ADD_RX);
    switch (op) {
        case D_MUL_RX: return D_MUL_R;
        case D_MUL_CX: return D_MUL_C;
        case D_LOADC_X: return D_LOADC;
        default: return op;
    }
}

// the X form of a (final, R- or C-form) asm op, or 0 when it has none
MH_ISA_FN unsigned mh_xform(unsigned op) {
    if (op >= D_ADD_R && op <= D_SGE_C) return D_ADD_RX + (op - D_ADD_R);
    switch (op) {
        case D_MUL_R: return D_MUL_RX;
        case D_MUL_C: return D_MUL_CX;
        case D_LOADC: return D_LOADC_X;
        default: return 0;
    }
}

// ops whose result is a Bool (0/1 in limb 0)
MH_ISA_FN bool mh_produces_bool(unsigned op) {
    op = mh_base_op(op);
    return (op >= D_EQ_R && op <= D_SGE_C) || (op >= D_BAND && op <= D_FALSE) || op == D_BITE || op == D_BANDZ ||
           op == D_UADD_NOOVFL || op == D_UMUL_NOOVFL;
}

// *_R / *_C pairs (y from a register / inline constant): 1 = R form, 2 = C form, 0 = neither
MH_ISA_FN int mh_pair_form(unsigned op) {
    op = mh_base_op(op);
    if (op >= D_ADD_R && op <= D_SGE_C) return 1 + ((op - D_ADD_R) & 1);
    if (op == D_MUL_R || op == D_MUL_C) return 1 + (op - D_MUL_R);
    if (op >= D_UDIV_R && op <= D_SMOD_C) return 1 + ((op - D_UDIV_R) & 1);
    return 0;
}

// accumulator index (last register of the planes) of the kernel variant a tape needs
MH_ISA_FN unsigned mh_nrx_of(unsigned n_regs) {
    return n_regs <= MH_NR_SMALL ? MH_NR_SMALL : n_regs <= MH_NR_MID ? MH_NR_MID : MH_NR_MAX;
}
static_assert(D_NUM_OPS <= 128, "opcode space");

enum { F_YC = 1u << 31 };
#define MH_AUX_MAX ((1u << 14) - 1)

// Feature bits (mh_tape_info.features) — select the kernel variant.  A tape without F_CPLX,
// F_KECCAK or F_EVM runs entirely in the asm core (a kernel without the C++ path: fewer VGPRs,
// more waves).  F_DIV is informational (division runs in the asm core).
enum { F_DIV = 1, F_KECCAK = 2, F_EVM = 4, F_CPLX = 8 /* other C++ ops */ };

// Per-tape header in the device tape table.
struct mh_dev_tape {
    uint32_t insn_off;   // first slot of the tape in the slot array
    uint32_t n_insns;    // slots (windows are MH_WINDOW slots apart)
    uint32_t root_bool;  // 1 if the root (X at D_END) is Bool
    uint32_t n_regs;     // registers the tape uses (pinned columns included, X excluded)
};
