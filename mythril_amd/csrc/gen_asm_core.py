#!/usr/bin/env python3
"""Generate asm_core.inc: the threaded-code interpreter core of the sieve kernel (gfx950).

One inline-asm statement per register-file size NR runs the asm-core ops of dev_isa.h back to
back with ONE computed jump per instruction (s_setpc_b64 into a table of 256-byte handler
slots), instead of the binary-search branch tree a C++ switch compiles to: on CDNA every taken
branch stalls the wave on instruction fetch, and that stall, not the arithmetic, bounded the C++
interpreter (rocprofv3: 11.6 branches and ~260 parked cycles per interpreted instruction).

Register model (dev_isa.h): plane k of the register file is VGPRs [k*(NR+1), (k+1)*(NR+1)),
R[r] limb k is v[k*(NR+1) + r], the accumulator X is R[NR]; operands are read and written through
the GPR-index mode, so a' = NR (X itself) and d' = NR (no write-back) need no branch.  Scratch
S0..S16 follows the planes (S0..S7 doubles as y).  Constants ride in the instruction stream and
arrive by v_readlane, like the instructions.  The statement returns with ip at the first
instruction it does not handle (a complex op, D_WINDOW, D_END); the C++ driver
(sieve_kernels.hip) executes that one and re-enters.

Hazards (CDNA3/4 manually-inserted wait states): no VALU-written SGPR is used as a readlane lane
select or a VMEM operand inside the core; VCC is only used as carry/mask (no alias mixing); the
statement opens with s_nop so the VGPRs the compiler wrote just before are safe to readlane.
Every handler ends with s_set_gpr_idx_off before the next dispatch.

GPR-index rule (measured on MI355X, tests/test_asm_core.py checks the static half): an index taken
from the instruction word (S_W0 / S_B / S_D) enables ONE operand slot, and every enabled slot
holds a VGPR.  Handlers that read two indexed sources at static limb offsets under an S_W0 index
(SRC0|SRC1), or that put a constant in an enabled slot, returned wrong values, memory faults or
hangs -- but only at >= 2 waves per SIMD (1024+ workgroups), never in small parity runs, so any
new handler is also checked at full occupancy (scripts/diag_modes.py against a known-good build).

    python3 gen_asm_core.py > asm_core.inc      (run by the Makefile)
"""
import os
import sys

SLOT = 256          # bytes per handler slot
# inline constants by one s_load_dwordx8 from the tape's global copy instead of 8 v_readlane
# (MH_GEN_SMEM=0 restores the readlane form, for A/B builds)
SMEM_CONSTS = os.environ.get("MH_GEN_SMEM", "1") != "0"
# instruction words likewise by s_load_dwordx2 in the dispatch (MH_GEN_SMEM_INSN=0: v_readlane)
SMEM_INSNS = os.environ.get("MH_GEN_SMEM_INSN", "1") != "0"
# and the next instruction's words loaded at the top of the handler (after its constants), so the
# scalar-cache latency overlaps the handler's VALU body (MH_GEN_PREFETCH=0: load in the dispatch)
PREFETCH = SMEM_INSNS and os.environ.get("MH_GEN_PREFETCH", "1") != "0"
# the prefetch covers 8 slots from the next instruction (s_load_dwordx16): its words AND its inline
# constants, so a constant-operand handler copies them from the bank instead of loading
# (MH_GEN_PREFETCH_CONSTS=0: constants by their own s_load_dwordx8)
PREFETCH_CONSTS = PREFETCH and SMEM_CONSTS and os.environ.get("MH_GEN_PREFETCH_CONSTS", "1") != "0"
WINDOW = 64         # dev_isa.h MH_WINDOW
NSLOTS = 128        # op byte < 128 (dev_isa.h static_assert)
# D_LOADVAR (a column beyond the preloaded ones) in the core, as 8 global loads, instead of an
# exit to the C++ driver (~1 us of a wave's time per exit); only in the
# run_lv form the complex-op kernel variants use (MH_GEN_LOADVAR=0: every LOADVAR exits)
LOADVAR = os.environ.get("MH_GEN_LOADVAR", "1") != "0"
D_LOADVAR = 118     # dev_isa.h (static_assert in the .inc)
# likewise z3's unsigned BVAddNoOverflow (D_UADD_NOOVFL, exec.h's rule: no carry out of 256 bits
# and no bit at or above the width), in run_lv only
D_UADD_NOOVFL = 112
CORE_COMPLEX = {D_LOADVAR: "LOADVAR", D_UADD_NOOVFL: "UADD_NOOVFL"}
# D_LOADVAR prefetches the NEXT column the tape loads (its number in the word's b / c fields,
# compile.cpp; 0xffff: none) into 8 spare VGPRs without waiting, so the column load of the next
# LOADVAR overlaps the instructions between the two (MH_GEN_LV_PREFETCH=0: no prefetch).  The
# prefetch lives within one run of the core: every exit drains it (s_waitcnt vmcnt(0)) and an
# entry starts with none in flight.
LV_PREFETCH = LOADVAR and os.environ.get("MH_GEN_LV_PREFETCH", "1") != "0"
# D_WINDOW inside the core (round 5): ip counts slots from the tape's first one and gwin is the
# tape's base, so a window change is ip = next multiple of 64 and the next words' scalar load --
# not an exit to the C++ driver, which reloaded its lane-held window from memory and re-entered
# the core (a round trip per 64 slots: 70 on EtherThief-400's tape).  Needs the words and
# constants by scalar loads (the lane-held window is then only the C++ driver's).
CORE_WINDOW = SMEM_INSNS and SMEM_CONSTS and os.environ.get("MH_GEN_CORE_WINDOW", "1") != "0"
D_WINDOW = 120      # dev_isa.h (static_assert in the .inc)
# ... and the window after the one the core enters is pulled into the caches by one vector load
# of its 64 slots (8 B per lane, into 2 VGPRs nobody reads), issued at the window change and at
# entry: the slots' scalar loads then hit L2 instead of each 64-byte line missing in turn (the
# C++ driver's window reload did this by accident; without it the in-core change was slower)
WIN_PREFETCH = CORE_WINDOW and os.environ.get("MH_GEN_WIN_PREFETCH", "1") != "0"
LV_NONE = 0xFFFF

# opcode numbers: must match enum mh_dop in dev_isa.h (checked by a static_assert in the .inc)
OPS = ["EXIT", "NOP",
       "ADD_R", "ADD_C", "SUB_R", "SUB_C", "RSUB_R", "RSUB_C",
       "AND_R", "AND_C", "OR_R", "OR_C", "XOR_R", "XOR_C",
       "EQ_R", "EQ_C", "ULT_R", "ULT_C", "UGT_R", "UGT_C", "ULE_R", "ULE_C", "UGE_R", "UGE_C",
       "SLT_R", "SLT_C", "SGT_R", "SGT_C", "SLE_R", "SLE_C", "SGE_R", "SGE_C",
       "BAND", "BOR", "BXOR", "BEQ", "BNOT", "TRUE", "FALSE",
       "ITE", "ITEC", "BITE", "LOADC",
       "MUL_R", "MUL_C", "SHL_V", "LSHR_V", "ASHR_V",
       "UDIV_R", "UDIV_C", "UREM_R", "UREM_C", "SDIV_R", "SDIV_C", "SREM_R", "SREM_C",
       "SMOD_R", "SMOD_C",
       # X forms (dev_isa.h): a' = d' = X
       "ADD_RX", "ADD_CX", "SUB_RX", "SUB_CX", "RSUB_RX", "RSUB_CX",
       "AND_RX", "AND_CX", "OR_RX", "OR_CX", "XOR_RX", "XOR_CX",
       "EQ_RX", "EQ_CX", "ULT_RX", "ULT_CX", "UGT_RX", "UGT_CX", "ULE_RX", "ULE_CX",
       "UGE_RX", "UGE_CX", "SLT_RX", "SLT_CX", "SGT_RX", "SGT_CX", "SLE_RX", "SLE_CX",
       "SGE_RX", "SGE_CX",
       "MUL_RX", "MUL_CX", "LOADC_X"] + \
      ["SHR%d" % q for q in range(8)] + ["SHL%d" % q for q in range(8)] + ["BANDZ"]
DIV_KIND = {"UDIV_R": 0, "UDIV_C": 0, "UREM_R": 1, "UREM_C": 1, "SDIV_R": 2, "SDIV_C": 2,
            "SREM_R": 3, "SREM_C": 3, "SMOD_R": 4, "SMOD_C": 4}
OPNUM = {n: i for i, n in enumerate(OPS)}
# handlers longer than a slot live after the table (one extra jump)
OUT_OF_LINE = {"MUL_R", "MUL_C", "SHL_V", "LSHR_V", "ASHR_V", "MUL_RX", "MUL_CX"}

# scalar registers the core owns (declared clobbered)
S_TAB, S_TAB_HI = "s40", "s41"   # handler table base
S_W0, S_W1 = "s42", "s43"        # current instruction words
S_T = "s44"                      # temp
S_PC, S_PC_HI = "s46", "s47"     # jump target
S_B, S_D, S_C = "s48", "s49", "s50"  # register operands (low byte = index)
S_L = "s51"                      # readlane lane
S_Q, S_R = "s52", "s53"          # shift: limb part, bit part
S_K = ["s%d" % (56 + k) for k in range(8)]  # inline constant limbs (s_load_dwordx8 needs s[4n])
S_LANE2 = "s[54:55]"             # lane masks: shift saturation, division y != 0
S_KIND, S_ADV = "s70", "s71"   # division: kind (0 udiv .. 4 smod), slot advance
S_F64N = (68, 69)                # f64 constant pair (2^32, thresholds)
S_F64 = ("s68", "s69")
# prefetched next instruction words (+ with PREFETCH_CONSTS, its constant slots: bank s[72:87])
S_NW0, S_NW1 = ("s72", "s73") if PREFETCH_CONSTS else ("s64", "s65")
S_BANK = "s[72:87]"
S_NT = "s66"                     # prefetch address temp
S_PFC = "s45"                    # LOADVAR prefetch: the column in flight to the PF registers
DISPATCH_MARK = "@@dispatch_words"   # replaced per handler (prefetched or loaded in the dispatch)
SGPR_CLOBBERS = ["s%d" % i for i in range(40, 88 if PREFETCH_CONSTS else 72)]


class Core:
    def __init__(self, nr: int, loadvar: bool = False):
        self.nr = nr
        self.loadvar = loadvar
        self.nr1 = nr + 1
        self.sb = 8 * self.nr1  # scratch base
        self.no_wb = False

    def P(self, k, r=0):
        return "v%d" % (k * self.nr1 + r)

    def X(self, k):
        return self.P(k, self.nr)

    def S(self, j):
        assert 0 <= j <= 31
        return "v%d" % (self.sb + j)

    def Y(self, k):
        return self.S(k)

    def PF(self, k):  # run_lv: the column LOADVAR prefetched (8 VGPRs after the scratch)
        assert 0 <= k < 8
        return "v%d" % (self.sb + N_SCRATCH + k)

    def WP(self):  # the window prefetch's destination pair (after PF; never read)
        r = self.sb + N_SCRATCH + N_PF
        return "v[{}:{}]".format(r, r + 1)

    def win_prefetch(self):
        """One vector load of the 64 slots from slot S_T on (lane j: slot min(S_T + j, n - 1), so
        nothing past the tape's last slot is read), when S_T is inside the tape; no wait."""
        if not WIN_PREFETCH:
            return []
        t = self.S(0)
        return ["s_cmp_lt_u32 {}, %[nsl]".format(S_T),
                "s_cbranch_scc0 L_wpf_%=_{}".format(self._wpf),
                "v_mbcnt_lo_u32_b32 {}, -1, 0".format(t),
                "v_mbcnt_hi_u32_b32 {0}, -1, {0}".format(t),
                "v_add_u32 {0}, {1}, {0}".format(t, S_T),
                "s_sub_u32 {}, %[nsl], 1".format(S_T),
                "v_min_u32 {0}, {1}, {0}".format(t, S_T),
                "v_lshlrev_b32 {0}, 3, {0}".format(t),
                "global_load_dwordx2 {}, {}, %[gwin]".format(self.WP(), t),
                "L_wpf_%=_{}:".format(self._wpf)]

    def lv_address(self, col_sgpr):
        """s[56:57] = address of limb 0 of column `col_sgpr` (SoA planes: vbase + 8 col cap4); the
        row's byte offset is the VGPR voff.  SALU only: no VALU-written SGPR reaches the loads."""
        lo, hi = S_K[0], S_K[1]
        return ["s_lshl_b32 {}, {}, 3".format(S_T, col_sgpr),
                "s_mul_i32 {}, {}, %[cap4]".format(lo, S_T),
                "s_mul_hi_u32 {}, {}, %[cap4]".format(hi, S_T),
                "s_add_u32 {0}, {0}, %[vlo]".format(lo),
                "s_addc_u32 {0}, {0}, %[vhi]".format(hi)]

    def lv_loads(self, dst):
        """8 global loads of the column at s[56:57] into dst(0..7), no wait."""
        lo, hi = S_K[0], S_K[1]
        body = []
        for k in range(8):
            if k:
                body += ["s_add_u32 {0}, {0}, %[cap4]".format(lo),
                         "s_addc_u32 {0}, {0}, 0".format(hi)]
            body.append("global_load_dword {}, %[voff], s[{}:{}]".format(dst(k), lo[1:], hi[1:]))
        return body

    # ---- building blocks
    def dispatch(self, adv):
        out = []
        if adv:
            out.append("s_add_u32 %[ip], %[ip], {}".format(adv))
        if SMEM_INSNS:  # the instruction words by one scalar load (no VALU in the dispatch)
            out.append(DISPATCH_MARK)
        else:
            out += ["v_readlane_b32 {}, %[ic0], %[ip]".format(S_W0),
                    "v_readlane_b32 {}, %[ic1], %[ip]".format(S_W1)]
        out += [
            "s_and_b32 {}, {}, 0x7f".format(S_T, S_W1),
            "s_lshl_b32 {}, {}, 8".format(S_T, S_T),
            "s_add_u32 {}, {}, {}".format(S_PC, S_TAB, S_T),
            "s_addc_u32 {}, {}, 0".format(S_PC_HI, S_TAB_HI),
            "s_setpc_b64 s[46:47]",
        ]
        return out

    @staticmethod
    def load_words():
        if PREFETCH_CONSTS:  # every handler entry finds slots ip..ip+7 in the bank
            return ["s_lshl_b32 {}, %[ip], 3".format(S_T),
                    "s_load_dwordx16 {}, %[gwin], {}".format(S_BANK, S_T),
                    "s_waitcnt lgkmcnt(0)",
                    "s_mov_b64 s[{}:{}], s[{}:{}]".format(S_W0[1:], S_W1[1:], S_NW0[1:], S_NW1[1:])]
        return ["s_lshl_b32 {}, %[ip], 3".format(S_T),
                "s_load_dwordx2 s[{}:{}], %[gwin], {}".format(S_W0[1:], S_W1[1:], S_T),
                "s_waitcnt lgkmcnt(0)"]

    def resolve(self, lines):
        """Replace the dispatch marks of one handler.  A handler with a single static advance
        prefetches the next instruction's words right after its constants' load (or at its top):
        the next slot always exists (every tape ends in D_END, and this op is not the end), so
        the address is the one the dispatch would load.  Other handlers (the division body's
        register advance, entry) load in the dispatch."""
        import re
        marks = [i for i, l in enumerate(lines) if l == DISPATCH_MARK]
        if not marks:
            return lines
        advs = set()
        for i in marks:
            m = re.match(r"s_add_u32 %\[ip\], %\[ip\], (\d+)$", lines[i - 1]) if i else None
            advs.add(int(m.group(1)) if m else None)
        if not PREFETCH or len(advs) != 1 or None in advs:
            out = []
            for l in lines:
                out += self.load_words() if l == DISPATCH_MARK else [l]
            return out
        adv = advs.pop()
        pre = ["s_lshl3_add_u32 {}, %[ip], {}".format(S_NT, 8 * adv),  # (ip << 3) + 8 adv
               ("s_load_dwordx16 {}, %[gwin], {}".format(S_BANK, S_NT) if PREFETCH_CONSTS else
                "s_load_dwordx2 s[{}:{}], %[gwin], {}".format(S_NW0[1:], S_NW1[1:], S_NT))]
        at = 0
        for i, l in enumerate(lines):  # after the constants' wait / copy, if the handler has any
            if l.startswith("s_load_dwordx8"):
                at = i + 2
                assert lines[i + 1] == "s_waitcnt lgkmcnt(0)", lines[i + 1]
                break
            if l.startswith("s_mov_b64 s[56:57]"):
                at = i + 4
                assert all(x.startswith("s_mov_b64 s[") for x in lines[i:at]), lines[i:at]
                break
        assert at < marks[0]
        out = lines[:at] + pre
        for l in lines[at:]:
            out += ["s_waitcnt lgkmcnt(0)",
                    "s_mov_b64 s[{}:{}], s[{}:{}]".format(S_W0[1:], S_W1[1:], S_NW0[1:], S_NW1[1:])] \
                if l == DISPATCH_MARK else [l]
        return out

    def idx_on(self, sreg, modes):
        return ["s_set_gpr_idx_on {}, gpr_idx({})".format(sreg, ",".join(modes))]

    def idx_off(self):
        return ["s_set_gpr_idx_off"]

    def field(self, dst, shift):
        return ["s_lshr_b32 {}, {}, {}".format(dst, S_W0, shift)]

    def y_reg(self, limbs=8):  # Y <- R[b]
        out = self.field(S_B, 8) + self.idx_on(S_B, ["SRC0"])
        out += ["v_mov_b32 {}, {}".format(self.Y(k), self.P(k)) for k in range(limbs)]
        return out + self.idx_off()

    def consts(self, to_y=(), flip7=False):  # S_K <- inline constant; Y[k] <- S_K[k] for k in to_y
        out = []
        if PREFETCH_CONSTS:  # the 4 constant slots after ip arrived with this op's words
            out += ["s_mov_b64 s[{}:{}], s[{}:{}]".format(56 + 2 * i, 57 + 2 * i, 74 + 2 * i,
                                                          75 + 2 * i) for i in range(4)]
        elif SMEM_CONSTS:  # one scalar load of the 4 constant slots after ip (window base gwin)
            out += ["s_lshl_b32 {}, %[ip], 3".format(S_T),
                    "s_add_u32 {0}, {0}, 8".format(S_T),
                    "s_load_dwordx8 s[{}:{}], %[gwin], {}".format(S_K[0][1:], S_K[7][1:], S_T),
                    "s_waitcnt lgkmcnt(0)"]
        else:
            for i in range(4):
                out.append("s_add_u32 {}, %[ip], {}".format(S_L, i + 1))
                out.append("v_readlane_b32 {}, %[ic0], {}".format(S_K[2 * i], S_L))
                out.append("v_readlane_b32 {}, %[ic1], {}".format(S_K[2 * i + 1], S_L))
        if flip7:
            out.append("s_xor_b32 {}, {}, 0x80000000".format(S_K[7], S_K[7]))
        out += ["v_mov_b32 {}, {}".format(self.Y(k), S_K[k]) for k in to_y]
        return out

    def wb(self, limbs=8):  # R[d'] <- X (nothing in an X form)
        if self.no_wb:
            return []
        out = self.field(S_D, 16) + self.idx_on(S_D, ["DST"])
        out += ["v_mov_b32 {}, {}".format(self.P(k), self.X(k)) for k in range(limbs)]
        return out + self.idx_off()

    def bool_out(self, true_if_vcc=True):
        a, b = ("0", "1") if true_if_vcc else ("1", "0")
        return ["v_cndmask_b32_e64 {}, {}, {}, vcc".format(self.X(0), a, b)]

    # ---- X forms: a' = d' = X (dev_isa.h).  The base handler verbatim minus its write-back
    # (R[d'] <- X is X <- X when d' = X): the operand reads keep the base forms' GPR-index
    # patterns (a' = NR reads X through the same indexed src0/src1 as any register).  Forms that
    # read the first operand from X as a plain VGPR beside an indexed operand faulted on gfx950
    # under full occupancy (illegal memory accesses, bisected on MI355X), so none are used.
    def handler_x(self, name):
        base = name[:-2] if name.endswith("_X") else name[:-1]
        self.no_wb = True
        try:
            return self.handler(base)
        finally:
            self.no_wb = False

    # ---- handlers: list of instruction lines, ending in a dispatch (or the exit branch)
    def handler(self, name):
        return self.resolve(self.handler_raw(name))

    def handler_raw(self, name):
        if name.endswith("X") and name != "EXIT":
            return self.handler_x(name)
        X, P, Y, S = self.X, self.P, self.Y, self.S
        a_src0 = self.idx_on(S_W0, ["SRC0"])
        a_src1 = self.idx_on(S_W0, ["SRC1"])
        off = self.idx_off()
        if name == "EXIT":
            return ["s_branch L_out_%="]
        if name == "WINDOW":
            # the next window starts at the next multiple of 64 slots; its words are loaded by
            # the dispatch (no static advance: resolve() must not prefetch from the old ip);
            # the window after it is prefetched
            self._wpf = "w"
            return (["s_add_u32 %[ip], %[ip], {}".format(WINDOW),
                     "s_andn2_b32 %[ip], %[ip], {}".format(WINDOW - 1),
                     "s_add_u32 {}, %[ip], {}".format(S_T, WINDOW)] + self.win_prefetch() +
                    self.dispatch(0))
        if name == "LOADVAR":
            # X = column aux of this lane's row: limb k at vbase + ((8 col + k) cap4) + voff
            # (SoA planes, KParams::assign); the address is SALU arithmetic in s[56:57] (no
            # VALU-written SGPR reaches the loads), the row's byte offset the VGPR voff
            body = ["s_lshr_b32 {}, {}, 17".format(S_R, S_W1),
                    "s_and_b32 {0}, {0}, 0x3fff".format(S_R)]
            if not LV_PREFETCH:
                body += self.lv_address(S_R) + self.lv_loads(X) + ["s_waitcnt vmcnt(0)"]
                return body + self.wb() + self.dispatch(1)
            # the column prefetched by the previous LOADVAR: wait for it and copy; otherwise
            # load it now
            body += ["s_cmp_eq_u32 {}, {}".format(S_R, S_PFC),
                     "s_cbranch_scc0 L_lv_ld_%=",
                     "s_waitcnt vmcnt(0)"]
            body += ["v_mov_b32 {}, {}".format(X(k), self.PF(k)) for k in range(8)]
            body += ["s_branch L_lv_pf_%=", "L_lv_ld_%=:"]
            body += self.lv_address(S_R) + self.lv_loads(X) + ["s_waitcnt vmcnt(0)"]
            # the next column this tape loads (w0 bits 8..15 | 24..31 << 8): in flight to PF
            # while the instructions up to its LOADVAR run
            body += ["L_lv_pf_%=:",
                     "s_bfe_u32 {}, {}, 0x80008".format(S_R, S_W0),
                     "s_lshr_b32 {}, {}, 24".format(S_Q, S_W0),
                     "s_lshl_b32 {0}, {0}, 8".format(S_Q),
                     "s_or_b32 {}, {}, {}".format(S_PFC, S_R, S_Q),
                     "s_cmpk_eq_u32 {}, 0x{:x}".format(S_PFC, LV_NONE),
                     "s_cbranch_scc1 L_lv_wb_%="]
            body += self.lv_address(S_PFC) + self.lv_loads(self.PF)
            body += ["L_lv_wb_%=:"]
            return body + self.wb() + self.dispatch(1)
        if name == "UADD_NOOVFL":
            # y = inline constant (F_YC, 4 slots follow) or R[b]; t = R[a'] + y in S8..15;
            # h = carry | OR_k (t[k] & ~mask_k(w)), with ~mask_k = ~((1 << clamp(w - 32k, 0, 32))
            # - 1) built in SALU (w is wave-uniform); X = (h == 0), Bool in limb 0
            body = self.consts()
            body += ["s_bitcmp1_b32 {}, 31".format(S_W1), "s_cbranch_scc0 L_uno_r_%="]
            body += ["v_mov_b32 {}, {}".format(Y(k), S_K[k]) for k in range(8)]
            body += ["s_branch L_uno_y_%=", "L_uno_r_%=:"] + self.y_reg() + ["L_uno_y_%=:"]
            body += a_src0
            body.append("v_add_co_u32 {}, vcc, {}, {}".format(S(8), P(0), Y(0)))
            body += ["v_addc_co_u32 {}, vcc, {}, {}, vcc".format(S(8 + k), P(k), Y(k))
                     for k in range(1, 8)]
            body += off
            body += ["v_cndmask_b32_e64 {}, 0, 1, vcc".format(S(16)),
                     "s_lshr_b32 {}, {}, 8".format(S_T, S_W1),
                     "s_and_b32 {0}, {0}, 0x1ff".format(S_T)]
            for k in range(8):
                body += ["s_sub_i32 {}, {}, {}".format(S_R, S_T, 32 * k),
                         "s_max_i32 {0}, {0}, 0".format(S_R),
                         "s_min_i32 {0}, {0}, 32".format(S_R),
                         "s_bfm_b64 s[{}:{}], {}, 0".format(S_Q[1:], S_R[1:], S_R),
                         "s_not_b32 {0}, {0}".format(S_Q),
                         "v_and_or_b32 {0}, {1}, {2}, {0}".format(S(16), S_Q, S(8 + k))]
            body += ["v_cmp_eq_u32 vcc, 0, {}".format(S(16))] + self.bool_out(True) + self.wb(1)
            body += ["s_bitcmp1_b32 {}, 31".format(S_W1),
                     "s_cselect_b32 {}, 5, 1".format(S_T),
                     "s_add_u32 %[ip], %[ip], {}".format(S_T)]
            return body + self.dispatch(0)
        if name == "NOP":
            body = a_src0 + ["v_mov_b32 {}, {}".format(X(k), P(k)) for k in range(8)] + off
            return body + self.wb() + self.dispatch(1)
        arith = {"ADD": ("v_add_co_u32", "v_addc_co_u32"), "SUB": ("v_sub_co_u32", "v_subb_co_u32"),
                 "RSUB": ("v_subrev_co_u32", "v_subbrev_co_u32")}
        if name in ("ADD_R", "SUB_R", "RSUB_R"):
            first, rest = arith[name[:-2]]
            body = self.y_reg() + a_src0
            body.append("{} {}, vcc, {}, {}".format(first, X(0), P(0), Y(0)))
            body += ["{} {}, vcc, {}, {}, vcc".format(rest, X(k), P(k), Y(k)) for k in range(1, 8)]
            return body + off + self.wb() + self.dispatch(1)
        if name in ("ADD_C", "SUB_C", "RSUB_C"):
            # y is SGPR src0 for limb 0; VGPR for the carry chain (one scalar operand per VALU)
            first, rest = {"ADD_C": ("v_add_co_u32", "v_addc_co_u32"),
                           "SUB_C": ("v_subrev_co_u32", "v_subbrev_co_u32"),  # R - c
                           "RSUB_C": ("v_sub_co_u32", "v_subb_co_u32")}[name]  # c - R
            body = self.consts(to_y=range(1, 8)) + a_src1
            body.append("{} {}, vcc, {}, {}".format(first, X(0), S_K[0], P(0)))
            body += ["{} {}, vcc, {}, {}, vcc".format(rest, X(k), Y(k), P(k)) for k in range(1, 8)]
            return body + off + self.wb() + self.dispatch(5)
        logic = {"AND": "v_and_b32", "OR": "v_or_b32", "XOR": "v_xor_b32"}
        if name in ("AND_R", "OR_R", "XOR_R"):
            ins = logic[name[:-2]]
            body = self.y_reg() + a_src0
            body += ["{} {}, {}, {}".format(ins, X(k), P(k), Y(k)) for k in range(8)]
            return body + off + self.wb() + self.dispatch(1)
        if name in ("AND_C", "OR_C", "XOR_C"):
            ins = logic[name[:-2]]
            body = self.consts() + a_src1
            body += ["{} {}, {}, {}".format(ins, X(k), S_K[k], P(k)) for k in range(8)]
            return body + off + self.wb() + self.dispatch(5)
        if name in ("EQ_R", "EQ_C"):
            if name == "EQ_R":
                body = self.y_reg() + a_src0
                body += ["v_xor_b32 {}, {}, {}".format(S(8 + k), P(k), Y(k)) for k in range(8)]
            else:
                body = self.consts() + a_src1
                body += ["v_xor_b32 {}, {}, {}".format(S(8 + k), S_K[k], P(k)) for k in range(8)]
            body += off
            body += ["v_or3_b32 {0}, {0}, {1}, {2}".format(S(8), S(9), S(10)),
                     "v_or3_b32 {0}, {0}, {1}, {2}".format(S(8), S(11), S(12)),
                     "v_or3_b32 {0}, {0}, {1}, {2}".format(S(8), S(13), S(14)),
                     "v_or_b32 {0}, {0}, {1}".format(S(8), S(15)),
                     "v_cmp_eq_u32 vcc, 0, {}".format(S(8))]
            body += self.bool_out(True) + self.wb(1)
            return body + self.dispatch(1 if name == "EQ_R" else 5)
        cmp_kind = name[:-2]
        if cmp_kind in ("ULT", "UGT", "ULE", "UGE", "SLT", "SGT", "SLE", "SGE"):
            signed = cmp_kind[0] == "S"
            # borrow chain: R - y (lt) or y - R (gt); le = not gt, ge = not lt
            r_minus_y = cmp_kind[1:] in ("LT", "GE")
            truth = cmp_kind[1:] in ("LT", "GT")
            reg = name.endswith("_R")
            t8 = S(8)
            body = []
            if reg:
                body += self.y_reg()
                if signed:
                    body += a_src1 + ["v_xor_b32 {}, 0x80000000, {}".format(S(9), P(7))] + off
                    body += ["v_xor_b32 {0}, 0x80000000, {0}".format(Y(7))]
                body += a_src0
                if r_minus_y:  # P - Y
                    body.append("v_sub_co_u32 {}, vcc, {}, {}".format(t8, P(0), Y(0)))
                    body += ["v_subb_co_u32 {}, vcc, {}, {}, vcc".format(t8, P(k), Y(k))
                             for k in range(1, 7)]
                    if signed:
                        body += off + ["v_subb_co_u32 {}, vcc, {}, {}, vcc".format(t8, S(9), Y(7))]
                    else:
                        body += ["v_subb_co_u32 {}, vcc, {}, {}, vcc".format(t8, P(7), Y(7))] + off
                else:  # Y - P
                    body.append("v_subrev_co_u32 {}, vcc, {}, {}".format(t8, P(0), Y(0)))
                    body += ["v_subbrev_co_u32 {}, vcc, {}, {}, vcc".format(t8, P(k), Y(k))
                             for k in range(1, 7)]
                    if signed:
                        body += off + ["v_subbrev_co_u32 {}, vcc, {}, {}, vcc".format(t8, S(9), Y(7))]
                    else:
                        body += ["v_subbrev_co_u32 {}, vcc, {}, {}, vcc".format(t8, P(7), Y(7))] + off
            else:
                body += self.consts(to_y=range(1, 8), flip7=signed)
                if signed:
                    body += a_src1 + ["v_xor_b32 {}, 0x80000000, {}".format(S(9), P(7))] + off
                body += a_src1
                if r_minus_y:  # P - c
                    body.append("v_subrev_co_u32 {}, vcc, {}, {}".format(t8, S_K[0], P(0)))
                    body += ["v_subbrev_co_u32 {}, vcc, {}, {}, vcc".format(t8, Y(k), P(k))
                             for k in range(1, 7)]
                    if signed:
                        body += off + ["v_subbrev_co_u32 {}, vcc, {}, {}, vcc".format(t8, Y(7), S(9))]
                    else:
                        body += ["v_subbrev_co_u32 {}, vcc, {}, {}, vcc".format(t8, Y(7), P(7))] + off
                else:  # c - P
                    body.append("v_sub_co_u32 {}, vcc, {}, {}".format(t8, S_K[0], P(0)))
                    body += ["v_subb_co_u32 {}, vcc, {}, {}, vcc".format(t8, Y(k), P(k))
                             for k in range(1, 7)]
                    if signed:
                        body += off + ["v_subb_co_u32 {}, vcc, {}, {}, vcc".format(t8, Y(7), S(9))]
                    else:
                        body += ["v_subb_co_u32 {}, vcc, {}, {}, vcc".format(t8, Y(7), P(7))] + off
            body += self.bool_out(truth) + self.wb(1)
            return body + self.dispatch(1 if reg else 5)
        if name in ("BAND", "BOR", "BXOR", "BEQ"):
            ins = {"BAND": "v_and_b32", "BOR": "v_or_b32", "BXOR": "v_xor_b32",
                   "BEQ": "v_xor_b32"}[name]
            # Bool operands are 0/1 in limb 0 (dev_isa.h), so and/or/xor need no mask and
            # BEQ is 1 ^ a ^ b
            body = self.y_reg(1) + a_src0 + ["{} {}, {}, {}".format(ins, X(0), P(0), Y(0))] + off
            if name == "BEQ":
                body.append("v_xor_b32 {0}, 1, {0}".format(X(0)))
            return body + self.wb(1) + self.dispatch(1)
        if name == "BANDZ":
            # BAND, then the short-circuit test: no lane true -> leave the core at this op (the
            # driver ends the tape; X = 0 is its root).  The next words' prefetch is waited for
            # before leaving (its SGPRs are the compiler's again after the asm block).
            body = self.y_reg(1) + a_src0 + ["v_and_b32 {}, {}, {}".format(X(0), P(0), Y(0))] + off
            body += self.wb(1) + ["v_cmp_ne_u32 vcc, 0, {}".format(X(0)),
                                  "s_cmp_eq_u64 vcc, 0",
                                  "s_cbranch_scc1 L_bz_%="]
            return body + self.dispatch(1) + ["L_bz_%=:", "s_waitcnt lgkmcnt(0)",
                                              "s_branch L_out_%="]
        if name == "BNOT":
            body = a_src1 + ["v_xor_b32 {}, 1, {}".format(X(0), P(0))] + off  # R[a'] in src1
            return body + self.wb(1) + self.dispatch(1)
        if name in ("TRUE", "FALSE"):
            body = ["v_mov_b32 {}, {}".format(X(0), 1 if name == "TRUE" else 0)]
            return body + self.wb(1) + self.dispatch(1)
        if name in ("ITE", "ITEC", "BITE"):
            limbs = 1 if name == "BITE" else 8
            body = self.field(S_B, 8) + self.field(S_C, 24)
            cond_reg = S_B if name == "ITE" else S_W0
            then_reg = S_W0 if name == "ITE" else S_B
            body += self.idx_on(cond_reg, ["SRC1"]) + ["v_and_b32 {}, 1, {}".format(S(16), P(0))]
            body += off + ["v_cmp_ne_u32 vcc, 0, {}".format(S(16))]
            body += self.idx_on(S_C, ["SRC0"])
            body += ["v_mov_b32 {}, {}".format(Y(k), P(k)) for k in range(limbs)] + off
            body += self.idx_on(then_reg, ["SRC1"])
            body += ["v_cndmask_b32 {}, {}, {}, vcc".format(X(k), Y(k), P(k)) for k in range(limbs)]
            body += off
            if name == "BITE":
                body.append("v_and_b32 {0}, 1, {0}".format(X(0)))
            return body + self.wb(limbs) + self.dispatch(1)
        if name == "LOADC":
            body = self.consts() + ["v_mov_b32 {}, {}".format(X(k), S_K[k]) for k in range(8)]
            return body + self.wb() + self.dispatch(5)
        if name[:3] in ("SHR", "SHL") and name[3:].isdigit():
            # immediate shift by q limbs + the alignbit field aux (dev_isa.h D_SHR0 / D_SHL0):
            # the limbs that reach the result are copied out of R[a'] under the SRC0 index (the
            # same single-mode pattern as every other handler), then combined with static limb
            # offsets, no index
            q = int(name[3:])
            body = ["s_lshr_b32 {}, {}, 17".format(S_R, S_W1)]
            body += a_src0
            if name.startswith("SHR"):  # S(j) = limb j for j >= q, S(8) = 0
                body += ["v_mov_b32 {}, {}".format(S(j), P(j)) for j in range(q, 8)] + off
                body.append("v_mov_b32 {}, 0".format(S(8)))
                for k in range(0, 8 - q):
                    body.append("v_alignbit_b32 {}, {}, {}, {}".format(X(k), S(k + q + 1), S(k + q), S_R))
                body += ["v_mov_b32 {}, 0".format(X(k)) for k in range(8 - q, 8)]
            else:  # S(j + 1) = limb j for j <= 7 - q, S(0) = 0
                body += ["v_mov_b32 {}, {}".format(S(j + 1), P(j)) for j in range(0, 8 - q)] + off
                body.append("v_mov_b32 {}, 0".format(S(0)))
                for k in range(q, 8):  # X(k) = alignbit(limb(k - q), limb(k - q - 1), field)
                    body.append("v_alignbit_b32 {}, {}, {}, {}".format(X(k), S(k - q + 1), S(k - q), S_R))
                body += ["v_mov_b32 {}, 0".format(X(k)) for k in range(0, q)]
            return body + self.wb() + self.dispatch(1)
        if name in ("MUL_R", "MUL_C"):
            # product scanning: column k of x*y accumulated by v_mad_u64_u32 into a 64-bit pair
            # that alternates between A = S16:S17 and B = S18:S19; the carry-outs of column k
            # (VCC) are counted straight into the OTHER pair's high word, which the column's first
            # v_addc initialises, so the next column starts as (carries : this column's high word)
            # with one move.  x is copied to S8..S15 so the result can go straight to X even
            # when x is X.
            reg = name == "MUL_R"
            body = self.y_reg() if reg else self.consts()
            yv = (lambda j: Y(j)) if reg else (lambda j: S_K[j])
            body += a_src0 + ["v_mov_b32 {}, {}".format(S(8 + k), P(k)) for k in range(8)] + off
            pair = ["v[{}:{}]".format(self.sb + 16, self.sb + 17),
                    "v[{}:{}]".format(self.sb + 18, self.sb + 19)]
            lo, hi = [S(16), S(18)], [S(17), S(19)]
            for k in range(8):
                cur, nxt = k & 1, 1 - (k & 1)
                for i in range(k + 1):
                    addend = "0" if k == 0 else pair[cur]
                    body.append("v_mad_u64_u32 {}, vcc, {}, {}, {}".format(
                        pair[cur], S(8 + i), yv(k - i), addend))
                    if 0 < k < 7:
                        if i == 0:
                            body.append("v_addc_co_u32 {}, vcc, 0, 0, vcc".format(hi[nxt]))
                        else:
                            body.append("v_addc_co_u32 {0}, vcc, 0, {0}, vcc".format(hi[nxt]))
                body.append("v_mov_b32 {}, {}".format(X(k), lo[cur]))
                if k < 7:
                    body.append("v_mov_b32 {}, {}".format(lo[nxt], hi[cur]))
                if k == 0:
                    body.append("v_mov_b32 {}, 0".format(hi[nxt]))
            return body + self.wb() + self.dispatch(1 if reg else 5)
        if name in ("LSHR_V", "ASHR_V", "SHL_V"):
            # per-lane amount s = y (>= 256 saturates); t = x in S8..S15; 3-stage limb select
            # network on bits 7..5 of s, then v_alignbit by the bit part
            right = name != "SHL_V"
            body = self.y_reg()
            body += a_src0 + ["v_mov_b32 {}, {}".format(S(8 + k), P(k)) for k in range(8)] + off
            big = S_LANE2
            body += ["v_or3_b32 {}, {}, {}, {}".format(S(16), Y(1), Y(2), Y(3)),
                     "v_or3_b32 {0}, {0}, {1}, {2}".format(S(16), Y(4), Y(5)),
                     "v_or3_b32 {0}, {0}, {1}, {2}".format(S(16), Y(6), Y(7)),
                     "v_cmp_ne_u32_e64 {}, 0, {}".format(big, S(16)),
                     "v_cmp_lt_u32_e32 vcc, 0xff, {}".format(Y(0)),
                     "s_or_b64 {0}, {0}, vcc".format(big),
                     "v_lshrrev_b32 {}, 5, {}".format(S(18), Y(0)),   # q (limbs)
                     "v_and_b32 {}, 31, {}".format(S(19), Y(0))]      # r (bits)
            fill = "0"
            if name == "ASHR_V":
                body.append("v_ashrrev_i32 {}, 31, {}".format(S(17), S(15)))
                fill = S(17)
            t = [S(8 + k) for k in range(8)]
            for st in (4, 2, 1):
                body += ["v_and_b32 {}, {}, {}".format(S(20), st, S(18)),
                         "v_cmp_ne_u32_e32 vcc, 0, {}".format(S(20))]
                if right:
                    for k in range(8):
                        src = t[k + st] if k + st < 8 else fill
                        body.append("v_cndmask_b32_e64 {0}, {0}, {1}, vcc".format(t[k], src))
                else:
                    for k in range(7, -1, -1):
                        src = t[k - st] if k - st >= 0 else "0"
                        body.append("v_cndmask_b32_e64 {0}, {0}, {1}, vcc".format(t[k], src))
            if right:
                for k in range(8):
                    hi = t[k + 1] if k < 7 else fill
                    body.append("v_alignbit_b32 {}, {}, {}, {}".format(X(k), hi, t[k], S(19)))
                fillv = fill
            else:
                body += ["v_sub_u32 {}, 32, {}".format(S(20), S(19)),
                         "v_cmp_eq_u32_e32 vcc, 0, {}".format(S(19))]
                for k in range(8):
                    lo = t[k - 1] if k > 0 else "0"
                    body.append("v_alignbit_b32 {}, {}, {}, {}".format(X(k), t[k], lo, S(20)))
                    body.append("v_cndmask_b32_e64 {0}, {0}, {1}, vcc".format(X(k), t[k]))
                fillv = "0"
            body += ["v_cndmask_b32_e64 {0}, {0}, {1}, {2}".format(X(k), fillv, big) for k in range(8)]
            return body + self.wb() + self.dispatch(1)
        if name in DIV_KIND:
            # y into Y, the kind and the slot advance into SGPRs, then the shared body
            reg = name.endswith("_R")
            body = self.y_reg() if reg else self.consts(to_y=range(8))
            body += ["s_mov_b32 {}, {}".format(S_KIND, DIV_KIND[name]),
                     "s_mov_b32 {}, {}".format(S_ADV, 1 if reg else 5),
                     "s_branch L_div_%="]
            return body
        raise KeyError(name)

    def to_f64(self, dst, limbs, tmp):
        """dst (f64 pair) = the 256-bit value limbs[0..7] (Horner with fma, rel. error < 2^-50)."""
        out = ["s_mov_b32 {}, 0".format(S_F64[0]), "s_mov_b32 {}, 0x41f00000".format(S_F64[1]),
               "v_cvt_f64_u32 {}, {}".format(dst, limbs[7])]
        for k in range(6, -1, -1):
            out += ["v_cvt_f64_u32 {}, {}".format(tmp, limbs[k]),
                    "v_fma_f64 {0}, {0}, s[{1}:{2}], {3}".format(dst, S_F64N[0], S_F64N[1], tmp)]
        return out

    def div_body(self):
        """256-bit division by f64 digit estimates over 32-bit digits, no normalisation shifts.
        Step j (7..0, entered at the highest j any lane needs): c = trunc(R / (y 2^(32j))) from
        f64 (relative error ~2^-48, so c is the digit or off by one), R -= c*y*2^(32j) (8 mads),
        then one add-back if R went negative, one subtract if R >= y 2^(32j).  Lanes with y = 0
        keep R = |x| and get q = 2^256 - 1 (SMT-LIB); signed kinds divide |x| by |y| and fix the
        signs by the bvsdiv / bvsrem / bvsmod rules.  Y = S0..7 = y, R = S8..15."""
        X, S = self.X, self.S
        Y = [S(k) for k in range(8)]
        R = [S(8 + k) for k in range(8)]
        FY, FR, FC, FT = ("v[{}:{}]".format(self.sb + i, self.sb + i + 1) for i in (16, 18, 20, 22))
        CARRY = "v[{}:{}]".format(self.sb + 24, self.sb + 25)   # {carry, 0}
        MAD = "v[{}:{}]".format(self.sb + 26, self.sb + 27)     # {lo, hi}
        C, T1, SX, SY = S(28), S(29), S(30), S(31)
        YNZ, DUMMY, MSK, TM = S_LANE2, "s[64:65]", "s[66:67]", "s[44:45]"
        out = ["L_div_%=:"]
        out += self.idx_on(S_W0, ["SRC0"]) + ["v_mov_b32 {}, {}".format(R[k], self.P(k)) for k in range(8)]
        out += self.idx_off()
        # signed kinds: |x|, |y| as (v ^ m) - m with m = sign mask
        out += ["s_cmp_lt_u32 {}, 2".format(S_KIND), "s_cbranch_scc1 L_div_uns_%="]
        for v, m in ((R, SX), (Y, SY)):
            out.append("v_ashrrev_i32 {}, 31, {}".format(m, v[7]))
            out += ["v_xor_b32 {0}, {0}, {1}".format(v[k], m) for k in range(8)]
            out.append("v_sub_co_u32 {0}, vcc, {0}, {1}".format(v[0], m))
            out += ["v_subb_co_u32 {0}, vcc, {0}, {1}, vcc".format(v[k], m) for k in range(1, 8)]
        out.append("L_div_uns_%=:")
        out += ["v_mov_b32 {}, 0".format(X(k)) for k in range(8)]
        # y != 0 lanes; skip everything when no such lane has R >= y
        out += ["v_or3_b32 {}, {}, {}, {}".format(T1, Y[0], Y[1], Y[2]),
                "v_or3_b32 {0}, {0}, {1}, {2}".format(T1, Y[3], Y[4]),
                "v_or3_b32 {0}, {0}, {1}, {2}".format(T1, Y[5], Y[6]),
                "v_or_b32 {0}, {0}, {1}".format(T1, Y[7]),
                "v_cmp_ne_u32_e64 {}, 0, {}".format(YNZ, T1),
                "v_sub_co_u32 {}, vcc, {}, {}".format(T1, R[0], Y[0])]
        out += ["v_subb_co_u32 {}, vcc, {}, {}, vcc".format(T1, R[k], Y[k]) for k in range(1, 8)]
        out += ["s_andn2_b64 {}, {}, vcc".format(MSK, YNZ),
                "s_cmp_eq_u64 {}, 0".format(MSK), "s_cbranch_scc1 L_div_done_%="]
        # 1/yd, qd = R/y for the start digit
        out += self.to_f64(FY, Y, FT)
        out += ["v_rcp_f64 {}, {}".format(FC, FY),
                "s_nop 1",  # trans result -> non-trans VALU use needs a wait state (CDNA3/4)
                "v_fma_f64 {}, -{}, {}, 1.0".format(FT, FY, FC),
                "v_fma_f64 {}, {}, {}, {}".format(FY, FC, FT, FC)]
        out += self.to_f64(FR, R, FT)
        out.append("v_mul_f64 {}, {}, {}".format(FC, FR, FY))
        for j in range(7, 0, -1):  # start at the highest j with qd >= 2^(32j - 1) in some lane
            hi = (1023 + 32 * j - 1) << 20
            out += ["s_mov_b32 {}, 0".format(S_F64[0]), "s_mov_b32 {}, 0x{:x}".format(S_F64[1], hi),
                    "v_cmp_le_f64_e32 vcc, s[{}:{}], {}".format(S_F64N[0], S_F64N[1], FC),
                    "s_and_b64 {}, vcc, {}".format(TM, MSK),
                    "s_cmp_lg_u64 {}, 0".format(TM),
                    "s_cbranch_scc1 L_step{}_%=".format(j)]
        out.append("s_branch L_step0_%=")
        for j in range(7, -1, -1):
            out.append("L_step{}_%=:".format(j))
            out += self.to_f64(FR, R, FT)
            out.append("v_mul_f64 {}, {}, {}".format(FC, FR, FY))
            if j:  # * 2^-32j as an f64 constant (v_ldexp_f64 with an SGPR exponent left FC unscaled on gfx950)
                out += ["s_mov_b32 {}, 0".format(S_F64[0]),
                        "s_mov_b32 {}, 0x{:x}".format(S_F64[1], (1023 - 32 * j) << 20),
                        "v_mul_f64 {0}, {0}, s[{1}:{2}]".format(FC, S_F64N[0], S_F64N[1])]
            # clamp to 2^32 - 1 before the conversion (the estimate may exceed the digit range
            # by the last ulp; NaN from y = 0 lanes becomes the clamp and is zeroed below)
            out += ["s_mov_b32 {}, 0xffe00000".format(S_F64[0]),
                    "s_mov_b32 {}, 0x41efffff".format(S_F64[1]),
                    "v_min_f64 {0}, {0}, s[{1}:{2}]".format(FC, S_F64N[0], S_F64N[1]),
                    "v_cvt_u32_f64 {}, {}".format(C, FC),
                    "v_cndmask_b32_e64 {0}, 0, {0}, {1}".format(C, YNZ)]
            # R[j..] -= c * y  (the product's limbs above limb 7 only feed the borrow)
            out += ["v_mov_b32 {}, 0".format(S(24)), "v_mov_b32 {}, 0".format(S(25))]
            for k in range(8):
                out.append("v_mad_u64_u32 {}, {}, {}, {}, {}".format(MAD, DUMMY, C, Y[k], CARRY))
                out.append("v_mov_b32 {}, {}".format(S(24), S(27)))
                limb = j + k
                if limb <= 7:
                    ins = "v_sub_co_u32 {0}, vcc, {0}, {1}" if k == 0 else "v_subb_co_u32 {0}, vcc, {0}, {1}, vcc"
                    out.append(ins.format(R[limb], S(26)))
                else:
                    out.append("v_subb_co_u32 {}, vcc, 0, {}, vcc".format(T1, S(26)))
            out.append("v_subb_co_u32 {}, vcc, 0, {}, vcc".format(T1, S(24)))  # limb j + 8 > 7
            # negative: add y << 32j back, c - 1
            out += ["s_mov_b64 {}, vcc".format(MSK), "s_cmp_eq_u64 {}, 0".format(MSK),
                    "s_cbranch_scc1 L_noneg{}_%=".format(j)]
            for k in range(8 - j):
                out.append("v_cndmask_b32_e64 {}, 0, {}, {}".format(T1, Y[k], MSK))
                ins = "v_add_co_u32 {0}, vcc, {0}, {1}" if k == 0 else "v_addc_co_u32 {0}, vcc, {0}, {1}, vcc"
                out.append(ins.format(R[j + k], T1))
            out += ["v_cndmask_b32_e64 {}, 0, 1, {}".format(T1, MSK),
                    "v_sub_u32 {0}, {0}, {1}".format(C, T1),
                    "L_noneg{}_%=:".format(j)]
            # R >= y << 32j (y = 0 lanes excluded): subtract once more, c + 1
            out.append("v_sub_co_u32 {}, vcc, {}, {}".format(T1, R[j], Y[0]))
            out += ["v_subb_co_u32 {}, vcc, {}, {}, vcc".format(T1, R[j + k], Y[k]) for k in range(1, 8 - j)]
            out += ["v_subb_co_u32 {}, vcc, 0, {}, vcc".format(T1, Y[k]) for k in range(8 - j, 8)]
            out += ["s_andn2_b64 {}, {}, vcc".format(MSK, YNZ), "s_cmp_eq_u64 {}, 0".format(MSK),
                    "s_cbranch_scc1 L_noge{}_%=".format(j)]
            for k in range(8 - j):
                out.append("v_cndmask_b32_e64 {}, 0, {}, {}".format(T1, Y[k], MSK))
                ins = "v_sub_co_u32 {0}, vcc, {0}, {1}" if k == 0 else "v_subb_co_u32 {0}, vcc, {0}, {1}, vcc"
                out.append(ins.format(R[j + k], T1))
            out += ["v_cndmask_b32_e64 {}, 0, 1, {}".format(T1, MSK),
                    "v_add_u32 {0}, {0}, {1}".format(C, T1),
                    "L_noge{}_%=:".format(j),
                    "v_mov_b32 {}, {}".format(X(j), C)]
        out.append("L_div_done_%=:")
        # y = 0: q = 2^256 - 1 (R already holds |x|)
        out += ["v_cndmask_b32_e64 {0}, -1, {0}, {1}".format(X(k), YNZ) for k in range(8)]

        def cneg(dst, src, m):  # dst = (src ^ m) - m
            o = ["v_xor_b32 {}, {}, {}".format(dst[k], src[k], m) for k in range(8)]
            o.append("v_sub_co_u32 {0}, vcc, {0}, {1}".format(dst[0], m))
            o += ["v_subb_co_u32 {0}, vcc, {0}, {1}, vcc".format(dst[k], m) for k in range(1, 8)]
            return o
        XS = [X(k) for k in range(8)]
        out += ["s_cmp_eq_u32 {}, 0".format(S_KIND), "s_cbranch_scc1 L_div_wb_%=",
                "s_cmp_eq_u32 {}, 2".format(S_KIND), "s_cbranch_scc1 L_div_sdiv_%=",
                "s_cmp_eq_u32 {}, 4".format(S_KIND), "s_cbranch_scc1 L_div_smod_%=",
                "s_cmp_eq_u32 {}, 3".format(S_KIND), "s_cbranch_scc1 L_div_srem_%="]
        # UREM
        out += ["v_mov_b32 {}, {}".format(X(k), R[k]) for k in range(8)] + ["s_branch L_div_wb_%="]
        out.append("L_div_sdiv_%=:")  # q negated when the signs differ
        out += ["v_xor_b32 {}, {}, {}".format(T1, SX, SY)] + cneg(XS, XS, T1) + ["s_branch L_div_wb_%="]
        out.append("L_div_srem_%=:")  # r takes the sign of x
        out += cneg(XS, R, SX) + ["s_branch L_div_wb_%="]
        out.append("L_div_smod_%=:")  # u = |x| % |y|: (x<0 ? -u : u) + (signs differ && u ? +-|y| : 0)
        out += cneg(XS, R, SX)
        out += ["v_or3_b32 {}, {}, {}, {}".format(T1, R[0], R[1], R[2]),
                "v_or3_b32 {0}, {0}, {1}, {2}".format(T1, R[3], R[4]),
                "v_or3_b32 {0}, {0}, {1}, {2}".format(T1, R[5], R[6]),
                "v_or_b32 {0}, {0}, {1}".format(T1, R[7]),
                "v_cmp_ne_u32_e64 {}, 0, {}".format(MSK, T1),
                "v_xor_b32 {}, {}, {}".format(T1, SX, SY),
                "v_cmp_ne_u32_e32 vcc, 0, {}".format(T1),
                "s_and_b64 {0}, {0}, vcc".format(MSK)]
        out += cneg(Y, Y, SY)  # t = +-|y| (the original y)
        for k in range(8):
            out.append("v_cndmask_b32_e64 {}, 0, {}, {}".format(T1, Y[k], MSK))
            ins = "v_add_co_u32 {0}, vcc, {0}, {1}" if k == 0 else "v_addc_co_u32 {0}, vcc, {0}, {1}, vcc"
            out.append(ins.format(X(k), T1))
        out.append("L_div_wb_%=:")
        out += self.wb()
        out += ["s_add_u32 %[ip], %[ip], {}".format(S_ADV)] + self.dispatch(0)
        return out

    def fetch_text(self):
        """Operands of a complex op into S0..7 (x = R[a']), S8..15 (y = R[b] or the inline
        constant), S16..23 (R[c])."""
        S, P = self.S, self.P
        out = ["s_nop 1"]
        out += ["s_set_gpr_idx_on %[w0], gpr_idx(SRC0)"]
        out += ["v_mov_b32 {}, {}".format(S(k), P(k)) for k in range(8)] + ["s_set_gpr_idx_off"]
        out += ["s_lshr_b32 {}, %[w0], 24".format(S_C), "s_set_gpr_idx_on {}, gpr_idx(SRC0)".format(S_C)]
        out += ["v_mov_b32 {}, {}".format(S(16 + k), P(k)) for k in range(8)]
        out += ["s_set_gpr_idx_off", "s_bitcmp1_b32 %[w1], 31", "s_cbranch_scc1 L_yc_%="]
        out += ["s_lshr_b32 {}, %[w0], 8".format(S_B), "s_set_gpr_idx_on {}, gpr_idx(SRC0)".format(S_B)]
        out += ["v_mov_b32 {}, {}".format(S(8 + k), P(k)) for k in range(8)]
        out += ["s_set_gpr_idx_off", "s_branch L_done_%=", "L_yc_%=:"]
        for i in range(4):
            out.append("s_add_u32 {}, %[ip], {}".format(S_L, i + 1))
            out.append("v_readlane_b32 {}, %[ic0], {}".format(S_K[2 * i], S_L))
            out.append("v_readlane_b32 {}, %[ic1], {}".format(S_K[2 * i + 1], S_L))
        out += ["v_mov_b32 {}, {}".format(S(8 + k), S_K[k]) for k in range(8)]
        out += ["L_done_%=:"]
        return out

    def commit_text(self):
        """X = z (S0..7), then R[d'] = X."""
        S, X = self.S, self.X
        out = ["v_mov_b32 {}, {}".format(X(k), S(k)) for k in range(8)]
        out += ["s_lshr_b32 {}, %[w0], 16".format(S_D)]
        out += ["s_set_gpr_idx_on {}, gpr_idx(DST)".format(S_D)]
        out += ["v_mov_b32 {}, {}".format(self.P(k), X(k)) for k in range(8)]
        out += ["s_set_gpr_idx_off"]
        return out

    def asm_text(self):
        lines = ["s_nop 1",
                 "s_getpc_b64 s[40:41]",
                 "L_pc_%=:",
                 "s_add_u32 {0}, {0}, (L_tab_%= - L_pc_%=)".format(S_TAB),
                 "s_addc_u32 {0}, {0}, 0".format(S_TAB_HI)]
        if self.loadvar and LV_PREFETCH:  # nothing in flight on entry
            lines.append("s_mov_b32 {}, 0x{:x}".format(S_PFC, LV_NONE))
        if WIN_PREFETCH:  # the window after the one the core starts in
            self._wpf = "e"
            lines += ["s_andn2_b32 {}, %[ip], {}".format(S_T, WINDOW - 1),
                      "s_add_u32 {0}, {0}, {1}".format(S_T, WINDOW)] + self.win_prefetch()
        lines += self.resolve(self.dispatch(0))
        lines += [".p2align 8", "L_tab_%=:"]
        bodies = []
        for i in range(NSLOTS):
            lines.append(".org L_tab_%= + {}".format(i * SLOT))
            name = OPS[i] if i < len(OPS) else "EXIT"
            if CORE_WINDOW and i == D_WINDOW:
                name = "WINDOW"
            if self.loadvar and i in CORE_COMPLEX:
                name = CORE_COMPLEX[i]
            h = self.handler(name)
            if name in OUT_OF_LINE or name in CORE_COMPLEX.values():  # too long for a slot: jump to a body after the table
                lines.append("s_branch L_body_{}_%=".format(name))
                bodies += ["L_body_{}_%=:".format(name)] + h
            else:
                lines += h
        lines += [".org L_tab_%= + {}".format(NSLOTS * SLOT)] + bodies + self.resolve(self.div_body())
        lines += ["L_out_%=:"]
        if (self.loadvar and LV_PREFETCH) or WIN_PREFETCH:  # prefetches land before the exit
            lines.append("s_waitcnt vmcnt(0)")
        return lines


N_SCRATCH = 32  # S0..S31, declared clobbered by the core (division uses all 32)
N_PF = 8        # run_lv with LV_PREFETCH: the prefetched column, after the scratch


def n_scratch(core):
    """VGPRs after the planes a core's asm text may name: the scratch, the LOADVAR prefetch's 8
    (run_lv), the window prefetch's pair (after them)."""
    if WIN_PREFETCH:
        return N_SCRATCH + N_PF + 2
    return N_SCRATCH + (N_PF if core.loadvar and LV_PREFETCH else 0)


def check_registers(core, lines, n_scratch):
    """Every register the asm names must be a plane register, a declared scratch VGPR or a
    declared SGPR clobber: anything else could hold a live compiler value (an address...)."""
    import re
    hi_plane = 8 * core.nr1
    ok_v = set(range(hi_plane)) | set(range(core.sb, core.sb + n_scratch))
    ok_s = {int(x[1:]) for x in SGPR_CLOBBERS}
    for line in lines:
        for a, b in re.findall(r"\bv\[(\d+):(\d+)\]", line):
            for r in range(int(a), int(b) + 1):
                assert r in ok_v, (line, r)
        for r in re.findall(r"\bv(\d+)\b", line):
            assert int(r) in ok_v, (line, r)
        for a, b in re.findall(r"\bs\[(\d+):(\d+)\]", line):
            for r in range(int(a), int(b) + 1):
                assert r in ok_s, (line, r)
        for r in re.findall(r"\bs(\d+)\b", line):
            assert int(r) in ok_s, (line, r)


def emit(out):
    w = out.write
    w("// GENERATED by gen_asm_core.py -- do not edit.  Threaded-code asm core of the sieve\n")
    w("// interpreter (see the generator's docstring and dev_isa.h for the machine model).\n")
    w("#pragma once\n\n")
    for name, num in OPNUM.items():
        w("static_assert(D_{} == {}, \"asm core opcode numbering\");\n".format(name, num))
    w("static_assert(D_NUM_ASM == {}, \"asm core covers every asm op\");\n".format(len(OPS)))
    w("static_assert(D_LOADVAR == {}, \"asm core LOADVAR slot\");\n".format(D_LOADVAR))
    w("static_assert(D_UADD_NOOVFL == {}, \"asm core UADD_NOOVFL slot\");\n".format(D_UADD_NOOVFL))
    w("static_assert(D_WINDOW == {} && MH_WINDOW == {}, \"asm core WINDOW slot\");\n".format(D_WINDOW, WINDOW))
    # ip of the run functions: slot index from the tape's first slot (1) or in the window (0)
    w("#define MH_ASM_CORE_WINDOW {}\n".format(int(CORE_WINDOW)))
    w("#define MH_ASM_LOADVAR {}\n\n".format(int(LOADVAR)))
    w("template <int NR> struct AsmCore;\n\n")
    for nr in (7, 9, 15):
        c = Core(nr)
        nr1 = nr + 1
        w("template <> struct AsmCore<{}> {{\n".format(nr))
        w("    typedef u32 plane_t __attribute__((ext_vector_type({})));\n".format(nr1))
        cons = []
        for k in range(8):
            cons.append("\"+{{v[{}:{}]}}\"(p{})".format(k * nr1, k * nr1 + nr, k))
        clob = ["\"v{}\"".format(c.sb + j) for j in range(N_SCRATCH)] + \
               ["\"{}\"".format(s) for s in SGPR_CLOBBERS] + ["\"vcc\"", "\"scc\"", "\"m0\""]
        forms = [(c, "run", "")]
        if LOADVAR:
            forms.append((Core(nr, loadvar=True), "run_lv",
                          ", u32 vlo, u32 vhi, u32 cap4, u32 voff"))
        for core, fname, extra in forms:
            n_scr = n_scratch(core)
            clob = ["\"v{}\"".format(c.sb + j) for j in range(n_scr)] + \
                   ["\"{}\"".format(s) for s in SGPR_CLOBBERS] + ["\"vcc\"", "\"scc\"", "\"m0\""]
            w("    // runs asm-core instructions from slot ip of the window (ic0, ic1); returns the\n")
            w("    // slot of the first instruction it does not handle\n")
            if extra:
                w("    // (run_lv also runs D_LOADVAR: columns at vhi:vlo, cap4 bytes per limb plane,\n")
                w("    // this lane's row at byte offset voff)\n")
            w("    __device__ __forceinline__ static u32 {}(plane_t& p0, plane_t& p1, plane_t& p2,\n".format(fname))
            w("            plane_t& p3, plane_t& p4, plane_t& p5, plane_t& p6, plane_t& p7, u32 ic0,\n")
            w("            u32 ic1, u32 ip, const void* gwin, u32 nsl{}) {{\n".format(extra))
            w("        asm volatile(\n")
            for line in core.asm_text():
                w("            \"{}\\n\"\n".format(line))
            w("            : {}, [ip] \"+s\"(ip)\n".format(", ".join(cons)))
            ins = "[ic0] \"v\"(ic0), [ic1] \"v\"(ic1), [gwin] \"s\"(gwin), [nsl] \"s\"(nsl)"
            if extra:
                ins += (", [vlo] \"s\"(vlo), [vhi] \"s\"(vhi), [cap4] \"s\"(cap4), "
                        "[voff] \"v\"(voff)")
            w("            : {}\n".format(ins))
            check_registers(core, core.asm_text(), n_scr)
            w("            : {});\n".format(", ".join(clob)))
            w("        return ip;\n")
            w("    }\n")
        check_registers(c, c.fetch_text(), N_SCRATCH)
        check_registers(c, c.commit_text(), N_SCRATCH)
        sb = c.sb
        vec = "typedef u32 v8_t __attribute__((ext_vector_type(8)));\n"
        w("    " + vec)
        w("    // operands of the complex op at slot ip: x = R[a'], y = R[b] / inline const, c = R[c]\n")
        w("    __device__ __forceinline__ static void fetch(plane_t& p0, plane_t& p1, plane_t& p2,\n")
        w("            plane_t& p3, plane_t& p4, plane_t& p5, plane_t& p6, plane_t& p7, u32 ic0,\n")
        w("            u32 ic1, u32 ip, u32 w0, u32 w1, v8_t& x, v8_t& y, v8_t& c) {\n")
        w("        asm volatile(\n")
        for line in c.fetch_text():
            w("            \"{}\\n\"\n".format(line))
        w("            : {}, \"={{v[{}:{}]}}\"(x), \"={{v[{}:{}]}}\"(y), \"={{v[{}:{}]}}\"(c)\n".format(
            ", ".join(cons), sb, sb + 7, sb + 8, sb + 15, sb + 16, sb + 23))
        w("            : [ic0] \"v\"(ic0), [ic1] \"v\"(ic1), [ip] \"s\"(ip), [w0] \"s\"(w0), [w1] \"s\"(w1)\n")
        w("            : {});\n".format(", ".join("\"{}\"".format(x) for x in
                                          [S_B, S_C, S_L] + S_K + ["scc", "m0"])))
        w("    }\n")
        w("    // X = z, then R[d'] = X\n")
        w("    __device__ __forceinline__ static void commit(plane_t& p0, plane_t& p1, plane_t& p2,\n")
        w("            plane_t& p3, plane_t& p4, plane_t& p5, plane_t& p6, plane_t& p7, u32 w0,\n")
        w("            v8_t z) {\n")
        w("        asm volatile(\n")
        for line in c.commit_text():
            w("            \"{}\\n\"\n".format(line))
        w("            : {}\n".format(", ".join(cons)))
        w("            : [w0] \"s\"(w0), \"{{v[{}:{}]}}\"(z)\n".format(sb, sb + 7))
        w("            : \"{}\", \"scc\", \"m0\");\n".format(S_D))
        w("    }\n")
        w("};\n\n")


if __name__ == "__main__":
    emit(sys.stdout)
