"""Static checks of the generated threaded-code asm core (mythril_amd/csrc/gen_asm_core.py).

* every handler fits its 256-byte dispatch slot (assembled with llvm-mc for gfx950);
* the GPR-index mode is balanced: never left on across a jump or at a handler's end (a stale
  index would redirect the next handler's plain VGPR operands);
* every register the core names is a plane register, a declared scratch VGPR or a declared SGPR
  clobber (checked by the generator itself, exercised here for all three register-file sizes);
* the opcode table of the generator matches dev_isa.h.
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mythril_amd",
                    "csrc")
sys.path.insert(0, CSRC)

import gen_asm_core as G  # noqa: E402

LLVM_MC = "/opt/rocm/lib/llvm/bin/llvm-mc"


def _asm_lines(lines):
    out = []
    for ln in lines:
        ln = (ln.replace("%[ip]", "s39").replace("%[ic0]", "v200").replace("%[ic1]", "v201")
              .replace("%[gwin]", "s[80:81]").replace("%[voff]", "v202")
              .replace("%[vlo]", "s36").replace("%[vhi]", "s37").replace("%[cap4]", "s38").replace("%[nsl]", "s34")
              .replace("%=", "0"))
        if ln.endswith(":"):
            continue
        if ln.startswith(("s_branch L_", "s_cbranch")):
            ln = ln.split()[0] + " 0"
        out.append(ln)
    return out


@pytest.mark.skipif(not os.path.exists(LLVM_MC), reason="llvm-mc not installed")
@pytest.mark.parametrize("nr", [7, 9, 15])
def test_handlers_fit_their_slots(nr):
    core = G.Core(nr)
    for name in G.OPS:
        if name in G.OUT_OF_LINE:
            continue
        src = "\n".join(_asm_lines(core.handler(name))) + "\n"
        p = subprocess.run([LLVM_MC, "-arch=amdgcn", "-mcpu=gfx950", "-show-encoding"],
                           input=src, capture_output=True, text=True)
        assert p.returncode == 0, (name, p.stderr[:400])
        size = sum(len(re.findall(r"0x[0-9a-f]{2}", m))
                   for m in re.findall(r"encoding: \[(.*?)\]", p.stdout))
        assert 0 < size <= G.SLOT, (nr, name, size)


@pytest.mark.parametrize("nr", [7, 9, 15])
def test_gpr_index_mode_is_balanced(nr):
    core = G.Core(nr)
    bodies = [(n, core.handler(n)) for n in G.OPS] + [("div", core.div_body())]
    bodies += [(n, G.Core(nr, loadvar=True).handler(n)) for n in G.CORE_COMPLEX.values()]

    for name, lines in bodies:
        on = False
        for ln in lines:
            if ln.startswith("s_set_gpr_idx_on"):
                assert not on, (name, "nested")
                on = True
            elif ln.startswith("s_set_gpr_idx_off"):
                on = False
            elif ln.startswith(("s_setpc", "s_branch", "s_cbranch")):
                assert not on, (name, ln)
        assert not on, name


@pytest.mark.parametrize("nr", [7, 9, 15])
def test_registers_are_declared(nr):
    core = G.Core(nr)
    G.check_registers(core, core.asm_text(), G.n_scratch(core))


def test_opcode_table_matches_isa_header():
    src = open(os.path.join(CSRC, "dev_isa.h")).read()
    body = src[src.index("enum mh_dop"):src.index("D_NUM_ASM")]
    body = "\n".join(line.split("//")[0] for line in body.splitlines())
    names = re.findall(r"\b(D_[A-Z0-9_]+)", body)
    assert [n[2:] for n in names] == G.OPS


@pytest.mark.parametrize("nr", [7, 9, 15])
def test_indexed_slots_hold_vgprs(nr):
    """While the GPR-index mode is on, every operand slot it enables (SRC0/SRC1/SRC2/DST) holds
    a VGPR: the index is defined for VGPR operands only, and an SGPR or constant in an enabled
    slot is a pattern no handler relies on (memory faults on MI355X were traced to such
    mixtures)."""
    core = G.Core(nr)
    bodies = [(n, core.handler(n)) for n in G.OPS] + [("div", core.div_body())]
    bodies += [(n, G.Core(nr, loadvar=True).handler(n)) for n in G.CORE_COMPLEX.values()]
    bodies += [("fetch", core.fetch_text()), ("commit", core.commit_text())]
    vgpr = re.compile(r"^v(\d+|\[\d+:\d+\])$")
    for name, lines in bodies:
        modes = None
        for ln in lines:
            if ln.startswith("s_set_gpr_idx_on"):
                modes = set(re.search(r"gpr_idx\((.*)\)", ln).group(1).split(","))
                continue
            if ln.startswith("s_set_gpr_idx_off"):
                modes = None
                continue
            if modes is None or not ln.startswith("v_"):
                continue
            mnem, _, rest = ln.partition(" ")
            ops = [o.strip() for o in rest.split(",")]
            dst, srcs = ops[0], ops[1:]
            if srcs and srcs[0] in ("vcc", "s[62:63]", "s[64:65]") and "_co_" in mnem:
                srcs = srcs[1:]  # carry-out destination
            if "DST" in modes:
                assert vgpr.match(dst), (name, ln)
            for slot, op in zip(("SRC0", "SRC1", "SRC2"), srcs):
                if slot in modes:
                    assert vgpr.match(op.lstrip("-")), (name, ln)


@pytest.mark.parametrize("nr", [7, 9, 15])
def test_next_instruction_prefetch(nr):
    """Every dispatch that takes prefetched words (s_mov from S_NW) is preceded, in straight-line
    code from the handler's top, by exactly one load of S_NW at the address the dispatch's own ip
    advance gives; nothing in between writes S_NW / S_NT or leaves the handler; every other
    dispatch loads its words itself.  With PREFETCH_CONSTS the load fills the bank (the next
    instruction's words and its constant slots) and no handler reads the bank's constants after
    issuing it.  No unresolved dispatch mark reaches the asm text."""
    core = G.Core(nr)
    nw = "s[{}:{}]".format(G.S_NW0[1:], G.S_NW1[1:])
    take = "s_mov_b64 s[{}:{}], {}".format(G.S_W0[1:], G.S_W1[1:], nw)
    assert G.DISPATCH_MARK not in core.asm_text()
    n_pre = 0
    for name in G.OPS:
        lines = core.handler(name)
        takes = [i for i, ln in enumerate(lines) if ln == take]
        loads = [i for i, ln in enumerate(lines)
                 if ln.startswith(("s_load_dwordx2 " + nw, "s_load_dwordx16 " + G.S_BANK))
                 and G.S_NT in ln]
        if not takes:
            assert not loads, name
            continue
        n_pre += 1
        assert len(loads) == 1 and loads[0] < takes[0], name
        head = lines[:loads[0]]
        assert not any(ln.endswith(":") for ln in head), (name, "label before the prefetch")
        adv = {int(m.group(1)) for m in (re.match(r"s_add_u32 %\[ip\], %\[ip\], (\d+)$", ln)
                                          for ln in lines) if m}
        assert len(adv) == 1, (name, adv)
        assert lines[loads[0] - 1] == "s_lshl3_add_u32 {}, %[ip], {}".format(G.S_NT, 8 * adv.pop()), name
        for ln in lines[loads[0] + 1:takes[-1]]:
            dst = ln.split(" ", 1)[1].split(",")[0] if " " in ln else ""
            assert dst not in (G.S_NW0, G.S_NW1, G.S_NT, nw, G.S_BANK), (name, ln)
            if G.PREFETCH_CONSTS:  # the constants were copied out of the bank before the load
                assert not any("s[%d:" % r in ln for r in (74, 76, 78, 80)), (name, ln)
            assert not ln.startswith(("s_setpc", "s_branch L_out")), (name, ln)
        for i in takes:
            assert lines[i - 1] == "s_waitcnt lgkmcnt(0)", name
    assert n_pre > len(G.OPS) // 2


@pytest.mark.parametrize("nr", [7, 9, 15])
def test_indexed_operands_stay_in_the_register_file(nr):
    """Every operand the GPR-index mode relocates lands inside the wave's register-file planes
    for every index the host can encode (register operands are 0..NR, dev_isa.h), so an indexed
    access can never reach the scratch VGPRs, the driver's values or past the wave's allocation
    (a co-resident wave's registers).  This rules out an out-of-range index as the cause of the
    full-occupancy faults of the two-source indexed handlers."""
    core = G.Core(nr)
    planes = 8 * (nr + 1)
    bodies = [(n, core.handler(n)) for n in G.OPS] + [("div", core.div_body())]
    bodies += [(n, G.Core(nr, loadvar=True).handler(n)) for n in G.CORE_COMPLEX.values()]
    bodies += [("fetch", core.fetch_text()), ("commit", core.commit_text())]
    vreg = re.compile(r"^v(?:(\d+)|\[(\d+):(\d+)\])$")
    checked = 0
    for name, lines in bodies:
        modes = None
        for ln in lines:
            if ln.startswith("s_set_gpr_idx_on"):
                modes = set(re.search(r"gpr_idx\((.*)\)", ln).group(1).split(","))
                continue
            if ln.startswith("s_set_gpr_idx_off"):
                modes = None
                continue
            if modes is None or not ln.startswith("v_"):
                continue
            mnem, _, rest = ln.partition(" ")
            ops = [o.strip().lstrip("-") for o in rest.split(",")]
            dst, srcs = ops[0], ops[1:]
            if srcs and srcs[0] in ("vcc", "s[62:63]", "s[64:65]") and "_co_" in mnem:
                srcs = srcs[1:]
            slots = [("DST", dst)] + list(zip(("SRC0", "SRC1", "SRC2"), srcs))
            for slot, op in slots:
                if slot not in modes:
                    continue
                m = vreg.match(op)
                assert m, (name, ln)
                hi = int(m.group(1) or m.group(3))
                assert hi + nr < planes, (name, ln, "index reaches v%d" % (hi + nr))
                checked += 1
    assert checked > 100


@pytest.mark.skipif(not os.path.exists(LLVM_MC), reason="llvm-mc not installed")
@pytest.mark.parametrize("nr", [7, 9, 15])
def test_loadvar_handler(nr):
    """The in-core D_LOADVAR (run_lv): assembles for gfx950; its table slot jumps to the body
    only in the run_lv form (run keeps the exit, the asm-only variants never see a LOADVAR);
    limb k lands in X's plane k from the address vbase + (8 col + k) cap4 + voff; the loads
    complete before the write-back; the prefetched next words are taken as in every handler."""
    core = G.Core(nr, loadvar=True)
    lines = core.handler("LOADVAR")
    src = "\n".join(_asm_lines(lines)) + "\n"
    p = subprocess.run([LLVM_MC, "-arch=amdgcn", "-mcpu=gfx950", "-show-encoding"],
                       input=src, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr[:400]
    loads = [ln for ln in lines if ln.startswith("global_load_dword")]
    own = ["global_load_dword {}, %[voff], s[56:57]".format(core.X(k)) for k in range(8)]
    pf = ["global_load_dword {}, %[voff], s[56:57]".format(core.PF(k)) for k in range(8)]
    if G.LV_PREFETCH:
        # its own column into X (unless the previous LOADVAR prefetched it: then a wait and a
        # copy from PF), then the next column into PF, not waited for
        assert loads == own + pf
        waits = [i for i, ln in enumerate(lines) if ln == "s_waitcnt vmcnt(0)"]
        assert len(waits) == 2
        copy = [i for i, ln in enumerate(lines) if ln.startswith("v_mov_b32") and "v%d" % (
            core.sb + G.N_SCRATCH) in ln]
        assert waits[0] < copy[0]  # the prefetched column has landed before it is copied
        assert lines.index(own[-1]) < waits[1] < lines.index(pf[0])
        assert lines.index(pf[-1]) < next(i for i, ln in enumerate(lines)
                                          if ln.startswith("s_set_gpr_idx_on"))
        assert sum(ln == "s_add_u32 s56, s56, %[cap4]" for ln in lines) == 14
        text = core.asm_text()
        # every run starts with nothing in flight and drains the prefetch before it exits
        assert text[text.index("L_out_%=:") + 1] == "s_waitcnt vmcnt(0)"
        assert "s_mov_b32 {}, 0x{:x}".format(G.S_PFC, G.LV_NONE) in text[:8]
        G.check_registers(core, text, G.n_scratch(core))
    else:
        assert loads == own
        assert lines.index("s_waitcnt vmcnt(0)") > lines.index(loads[-1])
        assert lines.index("s_waitcnt vmcnt(0)") < next(i for i, ln in enumerate(lines)
                                                         if ln.startswith("s_set_gpr_idx_on"))
        assert sum(ln == "s_add_u32 s56, s56, %[cap4]" for ln in lines) == 7
    text = core.asm_text()
    slot = text.index(".org L_tab_%= + {}".format(G.D_LOADVAR * G.SLOT))
    assert text[slot + 1] == "s_branch L_body_LOADVAR_%="
    plain = G.Core(nr).asm_text()
    slot = plain.index(".org L_tab_%= + {}".format(G.D_LOADVAR * G.SLOT))
    assert plain[slot + 1] == "s_branch L_out_%=" and not any("%[voff]" in ln for ln in plain)
    if not G.LV_PREFETCH:
        G.check_registers(core, text, G.n_scratch(core))


@pytest.mark.skipif(not os.path.exists(LLVM_MC), reason="llvm-mc not installed")
@pytest.mark.parametrize("nr", [7, 9, 15])
def test_uadd_noovfl_handler(nr):
    """The in-core D_UADD_NOOVFL (run_lv only): assembles; y from the constant bank when F_YC
    (advance 5) else R[b] (advance 1); the 8-limb carry chain reads R[a'] through one SRC0 index;
    one SALU-built mask per limb; a Bool written back in limb 0; the next words loaded in the
    dispatch (the advance is not static)."""
    core = G.Core(nr, loadvar=True)
    lines = core.handler("UADD_NOOVFL")
    src = "\n".join(_asm_lines(lines)) + "\n"
    p = subprocess.run([LLVM_MC, "-arch=amdgcn", "-mcpu=gfx950", "-show-encoding"],
                       input=src, capture_output=True, text=True)
    assert p.returncode == 0, p.stderr[:400]
    assert sum(ln.startswith("v_addc_co_u32") for ln in lines) == 7
    assert sum(ln.startswith("v_and_or_b32") for ln in lines) == 8
    assert sum(ln.startswith("s_bfm_b64") for ln in lines) == 8
    assert "s_cselect_b32 {}, 5, 1".format(G.S_T) in lines
    assert lines[-9:-7] == ["s_lshl_b32 {}, %[ip], 3".format(G.S_T),
                            "s_load_dwordx16 {}, %[gwin], {}".format(G.S_BANK, G.S_T)] \
        or not G.PREFETCH_CONSTS
    text = core.asm_text()
    slot = text.index(".org L_tab_%= + {}".format(G.D_UADD_NOOVFL * G.SLOT))
    assert text[slot + 1] == "s_branch L_body_UADD_NOOVFL_%="
    plain = G.Core(nr).asm_text()
    slot = plain.index(".org L_tab_%= + {}".format(G.D_UADD_NOOVFL * G.SLOT))
    assert plain[slot + 1] == "s_branch L_out_%="


def test_loadvar_slot_matches_isa_header():
    src = open(os.path.join(CSRC, "dev_isa.h")).read()
    body = src[src.index("enum mh_dop"):src.index("D_NUM_OPS")]
    body = "\n".join(line.split("//")[0] for line in body.splitlines())
    body = body[body.index("D_FIRST_COMPLEX = 112,") + len("D_FIRST_COMPLEX = 112,"):]
    after = re.findall(r"\b(D_[A-Z0-9_]+)\b", body.replace("= D_FIRST_COMPLEX", ""))
    assert 112 + after.index("D_LOADVAR") == G.D_LOADVAR
    assert 112 + after.index("D_UADD_NOOVFL") == G.D_UADD_NOOVFL


@pytest.mark.parametrize("nr", [7, 9, 15])
def test_window_change_stays_in_the_core(nr):
    """With CORE_WINDOW the D_WINDOW slot of the table holds a handler that moves ip to the next
    multiple of 64 slots (ip counts from the tape's first slot) and dispatches there -- the C++
    driver sees a window change only when the core leaves for another reason."""
    if not G.CORE_WINDOW:
        pytest.skip("generator built without CORE_WINDOW")
    core = G.Core(nr)
    h = core.handler("WINDOW")
    assert h[:2] == ["s_add_u32 %[ip], %[ip], 64", "s_andn2_b32 %[ip], %[ip], 63"]
    assert h[-1] == "s_setpc_b64 s[46:47]" and not any("L_out" in ln for ln in h)
    # the words are loaded at the new ip, after it is set (no prefetch from the old one)
    loads = [i for i, ln in enumerate(h) if ln.startswith("s_load_dword")]
    assert len(loads) == 1 and loads[0] > 1 and h[loads[0] - 1] == "s_lshl_b32 s44, %[ip], 3"
    text = core.asm_text()
    at = text.index(".org L_tab_%= + {}".format(G.D_WINDOW * G.SLOT))
    assert text[at + 1:at + 1 + len(h)] == h
    if os.path.exists(LLVM_MC):
        src = "\n".join(_asm_lines(h)) + "\n"
        p = subprocess.run([LLVM_MC, "-arch=amdgcn", "-mcpu=gfx950", "-show-encoding"],
                           input=src, capture_output=True, text=True)
        assert p.returncode == 0, p.stderr[:400]
        size = sum(len(re.findall(r"0x[0-9a-f]{2}", m))
                   for m in re.findall(r"encoding: \[(.*?)\]", p.stdout))
        assert 0 < size <= G.SLOT
