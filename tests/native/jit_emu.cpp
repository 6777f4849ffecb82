// TEST-ONLY host emulator of the JIT's machine code (mythril_amd/csrc/jit.h MI lists).
//
// Executes the instruction list the JIT emits for one tape (and the shared division subroutine)
// on a host model of one gfx950 wave: 64 lanes of VGPRs, SGPRs, VCC, SCC.  Every instruction
// kind the emitter uses has its ISA semantics restated here (carry chains, v_mad_u64_u32,
// v_alignbit, v_cndmask, compares, the f64 digit estimates of the division), so
// tests/test_jit.py checks the emitted code -- register allocation, limb specialisation,
// encodings -- against the oracle without a GPU.  Registers nobody wrote are poisoned.
// v_rcp_f64 is modelled as the reciprocal with its mantissa cut to 22 bits (relative error up to
// 2^-22): the hardware instruction is an approximation (LLVM refines it twice for an f64 divide),
// and a model better than the hardware hid a defect once -- one refinement step left digit
// estimates up to ~2^-12 off, which the division's skipped-correction test assumed below 2^-19
// (found on MI355X at 2^24 rows, scripts/diag_find_row.py; the emulator then returned the right
// value because its reciprocal was exact).  v_rcp_f32 is modelled 1 ulp off the rounded
// reciprocal (up or down by the input's low mantissa bits), the hardware's documented bound.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "compile.h"
#include "jit.h"

using namespace mh;
using namespace mh::jit;

namespace {

struct Wave {
    uint32_t v[512][64];
    uint32_t lds[16384];  // this wave's LDS (64 KiB, byte-addressed by the DS ops)
    uint32_t s[128];
    uint64_t vcc = 0;
    bool scc = false;

    uint32_t r32(const Opnd& o, int l) const {
        switch (o.k) {
            case O_V: return v[o.v][l];
            case O_S: return s[o.v];
            case O_IMM: return o.v;
            case O_VCC: return (uint32_t)vcc;
            default: return 0;
        }
    }
    uint64_t mask(const Opnd& o) const {
        switch (o.k) {
            case O_VCC: return vcc;
            case O_S: return (uint64_t)s[o.v] | ((uint64_t)s[o.v + 1] << 32);
            case O_IMM: return (uint64_t)(int64_t)(int32_t)o.v;
            case O_EXEC: return ~0ull;
            default: return 0;
        }
    }
    void set_mask(const Opnd& o, uint64_t m) {
        if (o.k == O_VCC) vcc = m;
        else if (o.k == O_S) { s[o.v] = (uint32_t)m; s[o.v + 1] = (uint32_t)(m >> 32); }
    }
    uint64_t r64(const Opnd& o, int l) const {
        if (o.k == O_V) return (uint64_t)v[o.v][l] | ((uint64_t)v[o.v + 1][l] << 32);
        if (o.k == O_S) return (uint64_t)s[o.v] | ((uint64_t)s[o.v + 1] << 32);
        if (o.k == O_IMM) return (uint64_t)(int64_t)(int32_t)o.v;
        return 0;
    }
    double f64(const Opnd& o, int l) const {
        double d;
        if (o.k == O_FONE) d = 1.0;
        else {
            const uint64_t b = r64(o, l);
            memcpy(&d, &b, 8);
        }
        return o.neg ? -d : d;
    }
    float f32(const Opnd& o, int l) const {
        const uint32_t b = r32(o, l);
        float f;
        memcpy(&f, &b, 4);
        return f;
    }
    void wf32(const Opnd& o, int l, float f) {
        uint32_t b;
        memcpy(&b, &f, 4);
        v[o.v][l] = b;
    }
    void wf64(const Opnd& o, int l, double d) {
        uint64_t b;
        memcpy(&b, &d, 8);
        v[o.v][l] = (uint32_t)b;
        v[o.v + 1][l] = (uint32_t)(b >> 32);
    }
};

struct Err {
    std::string m;
};

uint64_t g_chunk_valu0 = 0;
// executed-instruction counters (per wave): VALU, of them 4-cycle class, SALU, and the part
// inside the division subroutine
struct Counts {
    uint64_t valu = 0, wide = 0, salu = 0, div_valu = 0, div_wide = 0, f64 = 0;
    double alive_valu = 0;  // VALU weighted by the fraction of lanes still alive (compaction bound)
} g_counts;
uint64_t g_alive = ~0ull;  // lanes that satisfy every conjunct tested so far (short circuit)
// compaction study: VALU before the chunk's first short-circuit test, and the live lanes then
uint64_t g_valu_head = 0, g_head_done = 0, g_alive_hist[65];
// compaction study, per segment: (chunk, VALU executed since the chunk began, live lanes after the
// segment's short-circuit test); the chunk's end is a segment with mask ~0 tagged end
struct Seg { uint32_t chunk, valu; uint64_t alive; };
std::vector<Seg> g_segs;
uint32_t g_chunk_id = 0;
const uint32_t* g_mem = nullptr;  // "global memory": the SoA assignment buffer at address 0
uint64_t g_mem_words = 0;
uint64_t g_div_hist[32];  // division calls by executed VALU (buckets of 32)
// executed VALU by the SSA op kind that emitted it: [tag] body, [256 + tag] inside the division
// subroutine called by that op (tag 255 = prologue / untagged)
uint64_t g_tag_valu[512];
uint64_t g_opc_valu[2][256];  // executed VALU by machine opcode (tape body / division subroutine)
uint64_t g_mov_tag[256];      // executed v_mov in tape bodies by the SSA op that emitted them
uint64_t g_tag_op[256][128];  // executed tape-body VALU by (SSA op, machine opcode)
uint64_t g_div_label[128];  // division subroutine: executions of each label (path statistics)

bool is_wide(const MI& m) {
    const uint16_t op = m.op;
    return m.e64 || op == M_V_ADD_CO || op == M_V_ADDC_CO || op == M_V_SUB_CO ||
           op == M_V_SUBB_CO || op == M_V_SUBREV_CO || op == M_V_SUBBREV_CO || op == M_V_OR3 ||
           op == M_V_ALIGNBIT || op == M_V_MAD_U64_U32 || op == M_V_LSHL_ADD ||
           op == M_V_PERM || op == M_V_BFI ||
           (op >= M_V_CMP_EQ && op <= M_V_CMP_GT_I32) ||
           op == M_V_LSHLREV || op == M_V_LSHRREV || op == M_V_ASHRREV ||
           op >= M_V_CVT_F64_U32 || op == M_V_RCP_F32 || op == M_V_CMP_GT_F32 ||
           op == M_V_CMP_LE_F32;
}

void run(Wave& w, const std::vector<MI>& code, const std::vector<MI>& div, int depth = 0,
         uint8_t caller_tag = 0xFF) {
    std::unordered_map<uint32_t, size_t> lab;
    for (size_t i = 0; i < code.size(); ++i)
        if (code[i].op == M_LABEL) lab[code[i].o[0].v] = i;
    size_t pc = 0, steps = 0;
    while (pc < code.size()) {
        if (++steps > 10000000) throw Err{"emulator: runaway"};
        const MI& m = code[pc++];
        const Opnd* o = m.o;
        if (m.op <= M_V_CMP_LE_F64) {
            const bool wd = is_wide(m);
            ++g_counts.valu;
            g_counts.alive_valu += __builtin_popcountll(g_alive) / 64.0;
            g_counts.wide += wd;
            g_counts.f64 += m.op >= M_V_CVT_F64_U32;
            if (depth) { ++g_counts.div_valu; g_counts.div_wide += wd; }
            ++g_tag_valu[depth ? 256 + caller_tag : m.tag];
            ++g_opc_valu[depth ? 1 : 0][m.op & 255];
            if (!depth && m.op == M_V_MOV) ++g_mov_tag[m.tag];
            if (!depth) ++g_tag_op[m.tag][m.op & 127];
        } else if (m.op <= M_S_CMP_LT_U32) {
            ++g_counts.salu;
        }
        auto each = [&](auto f) { for (int l = 0; l < 64; ++l) f(l); };
        auto carry_op = [&](auto f) {  // d = f(l, &carry); sdst = o[1]
            uint64_t cm = 0;
            uint32_t res[64];
            for (int l = 0; l < 64; ++l) {
                bool c = false;
                res[l] = f(l, &c);
                if (c) cm |= 1ull << l;
            }
            for (int l = 0; l < 64; ++l) w.v[o[0].v][l] = res[l];
            w.set_mask(o[1], cm);
        };
        auto bit = [&](const Opnd& mo, int l) { return (w.mask(mo) >> l) & 1ull; };
        switch (m.op) {
            case M_V_MOV: each([&](int l) { w.v[o[0].v][l] = w.r32(o[1], l); }); break;
            case M_V_ADD_U32: each([&](int l) { w.v[o[0].v][l] = w.r32(o[1], l) + w.r32(o[2], l); }); break;
            case M_V_SUB_U32: each([&](int l) { w.v[o[0].v][l] = w.r32(o[1], l) - w.r32(o[2], l); }); break;
            case M_V_SUBREV_U32: each([&](int l) { w.v[o[0].v][l] = w.r32(o[2], l) - w.r32(o[1], l); }); break;
            case M_V_ADD_CO:
                carry_op([&](int l, bool* c) {
                    const uint64_t r = (uint64_t)w.r32(o[2], l) + w.r32(o[3], l);
                    *c = r >> 32;
                    return (uint32_t)r;
                });
                break;
            case M_V_ADDC_CO: {
                const uint64_t cin = w.mask(o[4]);
                carry_op([&](int l, bool* c) {
                    const uint64_t r = (uint64_t)w.r32(o[2], l) + w.r32(o[3], l) + ((cin >> l) & 1);
                    *c = r >> 32;
                    return (uint32_t)r;
                });
                break;
            }
            case M_V_SUB_CO: case M_V_SUBREV_CO: {
                const bool rev = m.op == M_V_SUBREV_CO;
                carry_op([&](int l, bool* c) {
                    const uint64_t a = w.r32(o[rev ? 3 : 2], l), b = w.r32(o[rev ? 2 : 3], l);
                    *c = a < b;
                    return (uint32_t)(a - b);
                });
                break;
            }
            case M_V_SUBB_CO: case M_V_SUBBREV_CO: {
                const bool rev = m.op == M_V_SUBBREV_CO;
                const uint64_t bin = w.mask(o[4]);
                carry_op([&](int l, bool* c) {
                    const uint64_t a = w.r32(o[rev ? 3 : 2], l), b = w.r32(o[rev ? 2 : 3], l);
                    const uint64_t bb = b + ((bin >> l) & 1);
                    *c = a < bb;
                    return (uint32_t)(a - bb);
                });
                break;
            }
            case M_V_AND: each([&](int l) { w.v[o[0].v][l] = w.r32(o[1], l) & w.r32(o[2], l); }); break;
            case M_V_OR: each([&](int l) { w.v[o[0].v][l] = w.r32(o[1], l) | w.r32(o[2], l); }); break;
            case M_V_XOR: each([&](int l) { w.v[o[0].v][l] = w.r32(o[1], l) ^ w.r32(o[2], l); }); break;
            case M_V_NOT: each([&](int l) { w.v[o[0].v][l] = ~w.r32(o[1], l); }); break;
            case M_V_XNOR: each([&](int l) { w.v[o[0].v][l] = ~(w.r32(o[1], l) ^ w.r32(o[2], l)); }); break;
            case M_V_OR3:
                each([&](int l) { w.v[o[0].v][l] = w.r32(o[1], l) | w.r32(o[2], l) | w.r32(o[3], l); });
                break;
            case M_V_ALIGNBIT:
                each([&](int l) {
                    const uint64_t x = ((uint64_t)w.r32(o[1], l) << 32) | w.r32(o[2], l);
                    w.v[o[0].v][l] = (uint32_t)(x >> (w.r32(o[3], l) & 31));
                });
                break;
            case M_V_LSHLREV: each([&](int l) { w.v[o[0].v][l] = w.r32(o[2], l) << (w.r32(o[1], l) & 31); }); break;
            case M_V_LSHRREV: each([&](int l) { w.v[o[0].v][l] = w.r32(o[2], l) >> (w.r32(o[1], l) & 31); }); break;
            case M_V_ASHRREV:
                each([&](int l) { w.v[o[0].v][l] = (uint32_t)((int32_t)w.r32(o[2], l) >> (w.r32(o[1], l) & 31)); });
                break;
            case M_V_CNDMASK: {
                uint32_t res[64];
                for (int l = 0; l < 64; ++l) res[l] = bit(o[3], l) ? w.r32(o[2], l) : w.r32(o[1], l);
                for (int l = 0; l < 64; ++l) w.v[o[0].v][l] = res[l];
                break;
            }
            case M_V_CMP_EQ: case M_V_CMP_NE: case M_V_CMP_LT: case M_V_CMP_LE: case M_V_CMP_GT:
            case M_V_CMP_GE: case M_V_CMP_LT_I32: case M_V_CMP_GT_I32: {
                uint64_t cm = 0;
                for (int l = 0; l < 64; ++l) {
                    const uint32_t a = w.r32(o[1], l), b = w.r32(o[2], l);
                    bool r = false;
                    switch (m.op) {
                        case M_V_CMP_EQ: r = a == b; break;
                        case M_V_CMP_NE: r = a != b; break;
                        case M_V_CMP_LT: r = a < b; break;
                        case M_V_CMP_LE: r = a <= b; break;
                        case M_V_CMP_GT: r = a > b; break;
                        case M_V_CMP_LT_I32: r = (int32_t)a < (int32_t)b; break;
                        case M_V_CMP_GT_I32: r = (int32_t)a > (int32_t)b; break;
                        default: r = a >= b; break;
                    }
                    if (r) cm |= 1ull << l;
                }
                w.set_mask(o[0], cm);
                break;
            }
            case M_V_MAD_U64_U32: {
                uint64_t cm = 0;
                uint64_t res[64];
                for (int l = 0; l < 64; ++l) {
                    const unsigned __int128 r = (unsigned __int128)((uint64_t)w.r32(o[2], l) * w.r32(o[3], l)) +
                                                w.r64(o[4], l);
                    res[l] = (uint64_t)r;
                    if (r >> 64) cm |= 1ull << l;
                }
                for (int l = 0; l < 64; ++l) {
                    w.v[o[0].v][l] = (uint32_t)res[l];
                    w.v[o[0].v + 1][l] = (uint32_t)(res[l] >> 32);
                }
                w.set_mask(o[1], cm);
                break;
            }
            case M_V_LSHL_ADD:
                each([&](int l) {
                    w.v[o[0].v][l] = (w.r32(o[1], l) << (w.r32(o[2], l) & 31)) + w.r32(o[3], l);
                });
                break;
            case M_V_PERM:
                each([&](int l) {
                    const uint64_t src = ((uint64_t)w.r32(o[1], l) << 32) | w.r32(o[2], l);
                    const uint32_t sel = w.r32(o[3], l);
                    uint32_t r = 0;
                    for (int b = 0; b < 4; ++b) {
                        const uint32_t s8 = (sel >> (8 * b)) & 0xFF;
                        uint32_t byte;
                        if (s8 < 8) byte = (uint32_t)(src >> (8 * s8)) & 0xFF;
                        else if (s8 == 12) byte = 0;
                        else if (s8 > 12) byte = 0xFF;
                        else throw Err{"emulator: v_perm sign-extension selector"};
                        r |= byte << (8 * b);
                    }
                    w.v[o[0].v][l] = r;
                });
                break;
            case M_V_BFI:
                each([&](int l) {
                    const uint32_t m = w.r32(o[1], l);
                    w.v[o[0].v][l] = (m & w.r32(o[2], l)) | (~m & w.r32(o[3], l));
                });
                break;
            case M_V_BITOP3:  // bit i = table bit (s0_i << 2 | s1_i << 1 | s2_i)
                each([&](int l) {
                    const uint32_t a = w.r32(o[1], l), b = w.r32(o[2], l), c = w.r32(o[3], l);
                    uint32_t r = 0;
                    for (int t = 0; t < 8; ++t)
                        if ((o[4].v >> t) & 1u)
                            r |= ((t & 4) ? a : ~a) & ((t & 2) ? b : ~b) & ((t & 1) ? c : ~c);
                    w.v[o[0].v][l] = r;
                });
                break;
            case M_V_CVT_F32_U32: each([&](int l) { w.wf32(o[0], l, (float)w.r32(o[1], l)); }); break;
            case M_V_FMA_F32:
                each([&](int l) { w.wf32(o[0], l, fmaf(w.f32(o[1], l), w.f32(o[2], l), w.f32(o[3], l))); });
                break;
            case M_V_MUL_F32: each([&](int l) { w.wf32(o[0], l, w.f32(o[1], l) * w.f32(o[2], l)); }); break;
            case M_V_RCP_F32:
                each([&](int l) {
                    const float x = w.f32(o[1], l);
                    float r = (float)(1.0 / (double)x);
                    uint32_t xb;
                    memcpy(&xb, &x, 4);
                    if (isfinite(r) && r != 0.0f) {
                        if (xb & 1u) r = nextafterf(r, INFINITY);
                        else if (xb & 2u) r = nextafterf(r, 0.0f);
                    }
                    w.wf32(o[0], l, r);
                });
                break;
            case M_V_CVT_U32_F32:
                each([&](int l) {
                    const float d = w.f32(o[1], l);
                    uint32_t r;
                    if (isnan(d) || d <= 0) r = 0;
                    else if (d >= 4294967295.0f) r = 0xFFFFFFFFu;
                    else r = (uint32_t)d;
                    w.v[o[0].v][l] = r;
                });
                break;
            case M_V_FRACT_F32:
                each([&](int l) {
                    const float x = w.f32(o[1], l);
                    w.wf32(o[0], l, isfinite(x) ? fminf(x - floorf(x), 0.99999994f) : NAN);
                });
                break;
            case M_V_CMP_GT_F32: case M_V_CMP_LE_F32: {
                uint64_t cm = 0;
                for (int l = 0; l < 64; ++l) {
                    const float a = w.f32(o[1], l), b = w.f32(o[2], l);
                    if (m.op == M_V_CMP_GT_F32 ? a > b : a <= b) cm |= 1ull << l;
                }
                w.set_mask(o[0], cm);
                break;
            }
            case M_V_CVT_F64_U32: each([&](int l) { w.wf64(o[0], l, (double)w.r32(o[1], l)); }); break;
            case M_V_FMA_F64:
                each([&](int l) { w.wf64(o[0], l, fma(w.f64(o[1], l), w.f64(o[2], l), w.f64(o[3], l))); });
                break;
            case M_V_RCP_F64:
                each([&](int l) {
                    double r = 1.0 / w.f64(o[1], l);
                    uint64_t b;
                    memcpy(&b, &r, 8);
                    if (isfinite(r) && r != 0.0) b &= ~((1ull << 30) - 1);  // 22-bit mantissa
                    memcpy(&r, &b, 8);
                    w.wf64(o[0], l, r);
                });
                break;
            case M_V_MUL_F64: each([&](int l) { w.wf64(o[0], l, w.f64(o[1], l) * w.f64(o[2], l)); }); break;
            case M_V_MIN_F64: each([&](int l) { w.wf64(o[0], l, fmin(w.f64(o[1], l), w.f64(o[2], l))); }); break;
            case M_V_CVT_U32_F64:
                each([&](int l) {
                    const double d = w.f64(o[1], l);
                    uint32_t r;
                    if (isnan(d) || d <= 0) r = 0;
                    else if (d >= 4294967295.0) r = 0xFFFFFFFFu;
                    else r = (uint32_t)d;
                    w.v[o[0].v][l] = r;
                });
                break;
            case M_V_FRACT_F64:
                each([&](int l) {
                    const double x = w.f64(o[1], l);
                    double r;
                    if (!isfinite(x)) r = NAN;
                    else r = fmin(x - floor(x), 0.99999999999999989);
                    w.wf64(o[0], l, r);
                });
                break;
            case M_V_CMP_LE_F64: {
                uint64_t cm = 0;
                for (int l = 0; l < 64; ++l)
                    if (w.f64(o[1], l) <= w.f64(o[2], l)) cm |= 1ull << l;
                w.set_mask(o[0], cm);
                break;
            }
            case M_S_MOV_B32: w.s[o[0].v] = w.r32(o[1], 0); break;
            case M_S_MOV_B64: w.set_mask(o[0], w.mask(o[1])); break;
            case M_S_AND_B64: case M_S_OR_B64: case M_S_XOR_B64: case M_S_XNOR_B64:
            case M_S_ANDN2_B64: case M_S_ORN2_B64: {
                const uint64_t a = w.mask(o[1]), b = w.mask(o[2]);
                uint64_t r = m.op == M_S_AND_B64 ? a & b : m.op == M_S_OR_B64 ? a | b :
                             m.op == M_S_XOR_B64 ? a ^ b : m.op == M_S_XNOR_B64 ? ~(a ^ b) :
                             m.op == M_S_ANDN2_B64 ? a & ~b : a | ~b;
                if (m.op == M_S_AND_B64 && o[0].k == O_S && o[0].v == S_SCRATCH) {
                    g_alive = r;
                    if (!depth)
                        g_segs.push_back({g_chunk_id, (uint32_t)(g_counts.valu - g_chunk_valu0), r});
                    if (!g_head_done && !depth) {
                        g_head_done = 1;
                        g_valu_head += g_counts.valu - g_chunk_valu0;
                        ++g_alive_hist[__builtin_popcountll(r)];
                    }
                }
                w.set_mask(o[0], r);
                w.scc = r != 0;
                break;
            }
            case M_S_NOT_B64: {
                const uint64_t r = ~w.mask(o[1]);
                w.set_mask(o[0], r);
                w.scc = r != 0;
                break;
            }
            case M_S_CMP_EQ_U64: w.scc = w.mask(o[0]) == w.mask(o[1]); break;
            case M_S_CMP_LG_U64: w.scc = w.mask(o[0]) != w.mask(o[1]); break;
            case M_S_CMP_EQ_U32: w.scc = w.r32(o[0], 0) == w.r32(o[1], 0); break;
            case M_S_CMP_LT_U32: w.scc = w.r32(o[0], 0) < w.r32(o[1], 0); break;
            case M_S_CBRANCH_SCC0: case M_S_CBRANCH_SCC1: case M_S_BRANCH: {
                const bool take = m.op == M_S_BRANCH || (m.op == M_S_CBRANCH_SCC1) == w.scc;
                if (take) {
                    auto it = lab.find(o[0].v);
                    if (it == lab.end()) throw Err{"emulator: missing label"};
                    pc = it->second;
                }
                break;
            }
            case M_LABEL:
                if (depth && o[0].v < 128) ++g_div_label[o[0].v];
                break;
            case M_S_NOP: break;
            case M_CALL_DIV: {
                if (depth) throw Err{"emulator: nested call"};
                const uint64_t before = g_counts.div_valu;
                run(w, div, div, depth + 1, m.tag);
                const uint64_t n = (g_counts.div_valu - before) / 32;
                ++g_div_hist[n < 31 ? n : 31];
                break;
            }
            case M_CALL_KEC:
                if (depth) throw Err{"emulator: nested call"};
                run(w, kec_routine().code, div, depth + 1, m.tag);
                break;
            case M_RET: return;
            case M_DS_WRITE2ST64: case M_DS_READ2ST64: case M_DS_READ_B32: {
                auto word = [&](uint32_t byte) -> uint32_t& {
                    if ((byte & 3) || byte / 4 >= 16384) throw Err{"emulator: LDS address"};
                    return w.lds[byte / 4];
                };
                for (int l = 0; l < 64; ++l) {
                    if (m.op == M_DS_WRITE2ST64) {
                        const uint32_t a = w.v[o[0].v][l];
                        word(a + o[3].v * 256) = w.v[o[1].v][l];
                        word(a + o[4].v * 256) = w.v[o[2].v][l];
                    } else if (m.op == M_DS_READ2ST64) {
                        const uint32_t a = w.v[o[1].v][l];
                        w.v[o[0].v][l] = word(a + o[2].v * 256);
                        w.v[o[0].v + 1][l] = word(a + o[3].v * 256);
                    } else {
                        w.v[o[0].v][l] = word(w.v[o[1].v][l] + o[2].v);
                    }
                }
                break;
            }
            case M_S_WAITCNT_LGKM: case M_S_WAITCNT_VM: break;
            case M_LOADCOL: {
                // the kernel's address arithmetic: s[28:29] = s[4:5] + j * s27, then
                // global_load_dword dst, v2, s[28:29] (v2 = the lane's row * 4)
                const uint64_t base = (uint64_t)w.s[4] | ((uint64_t)w.s[5] << 32);
                const uint64_t addr = base + (uint64_t)o[1].v * w.s[27];
                w.s[28] = (uint32_t)addr;
                w.s[29] = (uint32_t)(addr >> 32);
                for (int l = 0; l < 64; ++l) {
                    const uint64_t byte = addr + w.v[2][l];
                    if ((byte & 3) || byte / 4 >= g_mem_words) throw Err{"emulator: global address"};
                    w.v[o[0].v][l] = g_mem[byte / 4];
                }
                break;
            }
            default: throw Err{"emulator: unknown op " + std::to_string(m.op)};
        }
    }
}

bool g_short_circuit = true;  // Options::short_circuit of the emulated builds
int g_vn = kVnAll;            // value numbering of the emulated lowering (build_tapeset's retry)
uint32_t g_sample_rows = Options().sample_rows;

bool lower_and_emit(const mh_node* nodes, const uint64_t* offs, uint32_t n_tapes,
                    const uint32_t* consts, uint32_t n_consts, uint32_t n_vars, uint32_t tape,
                    uint32_t max_vgpr, std::vector<uint32_t>& pool, TapeCode& tc, std::string& e) {
    mh::ConstIndex index;
    SsaTape st;
    std::string err;
    if (tape >= n_tapes) { e = "tape index"; return false; }
    if (lower_tape_ssa(nodes + offs[tape], (size_t)(offs[tape + 1] - offs[tape]), consts,
                       n_consts, n_vars, pool, index, st, err, g_vn, true) != MH_OK) {
        e = "lowering: " + err;
        return false;
    }
    Options opt;
    opt.max_vgpr = max_vgpr;
    opt.short_circuit = g_short_circuit;
    opt.sample_rows = g_sample_rows;
    tc = emit_tape(st, pool, n_vars, opt);
    return true;
}

}  // namespace

// info[0] = 1 if jitted, [1] max_vgpr, [2] n_valu, [3] n_valu_wide, [4] n_salu, [5] calls_div,
// [6] root_bool, [7] code bytes; executed per 64-row chunk: [8] VALU, [9] 4-cycle VALU, [10] SALU,
// [11] VALU inside the division subroutine, [12] 4-cycle VALU inside it.  Returns 0 (evaluated or not jittable: see info[0] / err),
// < 0 on an emulator / lowering error.
extern "C" int32_t emu_jit_eval(const mh_node* nodes, const uint64_t* offs, uint32_t n_tapes,
                                const uint32_t* consts, uint32_t n_consts, uint32_t n_vars,
                                uint32_t tape, const uint32_t* assign, uint64_t rows,
                                uint32_t* out, uint32_t max_vgpr, uint32_t* info, char* err,
                                int errlen) {
    std::vector<uint32_t> pool;
    TapeCode tc;
    std::string e;
    if (!lower_and_emit(nodes, offs, n_tapes, consts, n_consts, n_vars, tape, max_vgpr, pool, tc,
                        e)) {
        snprintf(err, errlen, "%s", e.c_str());
        return -1;
    }
    info[0] = tc.ok;
    info[1] = tc.max_vgpr;
    info[2] = tc.n_valu;
    info[3] = tc.n_valu_wide;
    info[4] = tc.n_salu;
    info[5] = tc.calls_div;
    info[6] = tc.root_bool;
    info[7] = code_bytes(tc);
    if (!tc.ok) {
        snprintf(err, errlen, "%s", tc.why.c_str());
        return 0;
    }
    static const std::vector<MI> div = div_routine();
    static Wave w;
    g_counts = Counts();
    uint64_t chunks = 0;
    try {
        for (uint64_t base = 0; base < rows; base += 64) {
            for (int r = 0; r < 512; ++r)
                for (int l = 0; l < 64; ++l) w.v[r][l] = 0xDEAD0000u + (uint32_t)r;
            for (int r = 0; r < 128; ++r) w.s[r] = 0xBEEF0000u + (uint32_t)r;
            {  // the kernel's valid-lane mask of this chunk (short-circuit tests read it)
                const uint64_t left = rows - base;
                const uint64_t valid = left >= 64 ? ~0ull : ((1ull << left) - 1ull);
                w.s[S_VALID] = (uint32_t)valid;
                w.s[S_VALID + 1] = (uint32_t)(valid >> 32);
            }
            w.vcc = 0x5555AAAA5555AAAAull;
            // the kernel prologue's shift windows: lane l of wave 0, zero words outside [D, D+8)
            for (int l = 0; l < 64; ++l) w.v[R_LDS][l] = 4u * (uint32_t)l;
            for (uint32_t i = 0; i < 16384; ++i) w.lds[i] = 0xBAD0000u + i;
            for (uint32_t wd = 0; wd < LDS_WORDS; ++wd)
                if (wd < LDS_D || wd >= LDS_D + 8)
                    for (int l = 0; l < 64; ++l) w.lds[wd * 64 + l] = 0;
            for (uint32_t c = 0; c < pinned_cols(n_vars); ++c)
                for (int k = 0; k < 8; ++k)
                    for (int l = 0; l < 64; ++l) {
                        const uint64_t row = base + (uint64_t)l < rows ? base + (uint64_t)l : 0;
                        w.v[R_COL0 + 8 * c + k][l] = assign[((uint64_t)c * 8 + k) * rows + row];
                    }
            // the chunk loop's state the tape code reads: v2 = clamped row * 4, s[4:5] = the
            // buffer (address 0 here), s27 = column stride in bytes
            for (int l = 0; l < 64; ++l)
                w.v[2][l] = 4u * (uint32_t)std::min<uint64_t>(base + (uint64_t)l, rows - 1);
            w.s[4] = w.s[5] = 0;
            w.s[27] = (uint32_t)(4 * rows);
            g_mem = assign;
            g_mem_words = (uint64_t)n_vars * 8 * rows;
            g_alive = (uint64_t)w.s[S_VALID] | ((uint64_t)w.s[S_VALID + 1] << 32);
            g_head_done = 0;
            g_chunk_valu0 = g_counts.valu;
            run(w, tc.code, div);
            g_segs.push_back({g_chunk_id | 0x80000000u, (uint32_t)(g_counts.valu - g_chunk_valu0),
                              g_alive});
            ++g_chunk_id;
            if (!g_head_done) ++g_alive_hist[64];  // no test: the whole tape is the head
            ++chunks;
            const uint64_t res = (uint64_t)w.s[S_RES] | ((uint64_t)w.s[S_RES + 1] << 32);
            for (int l = 0; l < 64 && base + (uint64_t)l < rows; ++l) {
                const uint64_t row = base + (uint64_t)l;
                for (int k = 0; k < 8; ++k) {
                    uint32_t x;
                    if (tc.root_bool) x = k == 0 ? (uint32_t)((res >> l) & 1) : 0u;
                    else x = tc.root_limbs[k] != ~0u ? w.v[tc.root_limbs[k]][l] : tc.root_const[k];
                    out[(uint64_t)k * rows + row] = x;
                }
            }
        }
    } catch (const Err& x) {
        snprintf(err, errlen, "%s", x.m.c_str());
        return -2;
    }
    // dynamic counts per 64-row chunk (one wave evaluation of the tape)
    info[8] = (uint32_t)(g_counts.valu / chunks);
    info[9] = (uint32_t)(g_counts.wide / chunks);
    info[10] = (uint32_t)(g_counts.salu / chunks);
    info[11] = (uint32_t)(g_counts.div_valu / chunks);
    info[12] = (uint32_t)(g_counts.div_wide / chunks);
    info[13] = (uint32_t)(g_counts.f64 / chunks);
    info[14] = (uint32_t)(g_counts.alive_valu * 16.0 / (double)chunks);  // x16 fixed point
    return 0;
}

// The module source of a whole tape set (values / count mode); assemble != 0 also runs comgr.
// Returns the text length (and the code object size in *hsaco_size), < 0 on error.
extern "C" int64_t emu_jit_module(const mh_node* nodes, const uint64_t* offs, uint32_t n_tapes,
                                  const uint32_t* consts, uint32_t n_consts, uint32_t n_vars,
                                  uint32_t values, uint32_t max_vgpr, int32_t assemble_it,
                                  char* text, uint64_t cap, uint64_t* hsaco_size,
                                  uint32_t* n_jitted, char* err, int errlen) {
    std::vector<uint32_t> pool;
    mh::ConstIndex index;
    std::vector<TapeCode> codes(n_tapes);
    std::vector<const TapeCode*> ok;
    std::vector<uint32_t> ids;
    Options opt;
    opt.max_vgpr = max_vgpr;
    opt.short_circuit = g_short_circuit;
    opt.sample_rows = g_sample_rows;
    for (uint32_t t = 0; t < n_tapes; ++t) {
        SsaTape st;
        std::string e;
        if (lower_tape_ssa(nodes + offs[t], (size_t)(offs[t + 1] - offs[t]), consts, n_consts,
                           n_vars, pool, index, st, e, true, true) != MH_OK)
            continue;
        codes[t] = emit_tape(st, pool, n_vars, opt);
        if (codes[t].ok) {
            ok.push_back(&codes[t]);
            ids.push_back(t);
        }
    }
    *n_jitted = (uint32_t)ok.size();
    Module m = build_module(ok, ids, n_vars, values != 0, default_group_bytes());
    if (text && cap) {
        const size_t n = std::min<size_t>(cap - 1, m.text.size());
        memcpy(text, m.text.data(), n);
        text[n] = 0;
    }
    *hsaco_size = 0;
    if (assemble_it) {
        std::vector<char> bin;
        std::string log;
        if (!assemble(m.text, bin, log)) {
            snprintf(err, errlen, "%s", log.substr(0, (size_t)errlen - 1).c_str());
            return -1;
        }
        *hsaco_size = bin.size();
    }
    return (int64_t)m.text.size();
}

extern "C" void emu_jit_set_short_circuit(int on) { g_short_circuit = on != 0; }
extern "C" void emu_jit_set_vn(int vn) { g_vn = vn; }
extern "C" void emu_jit_set_sample_rows(uint32_t n) { g_sample_rows = n; }

extern "C" void emu_jit_op_stats(uint64_t* valu, uint64_t* wide, uint64_t* count, int reset) {
    op_stats(valu, wide, count, reset != 0);
}

extern "C" void emu_jit_div_labels(uint64_t* out, int reset) {
    for (int i = 0; i < 128; ++i) {
        out[i] = g_div_label[i];
        if (reset) g_div_label[i] = 0;
    }
}

extern "C" void emu_jit_tag_valu(uint64_t* out, int reset) {
    for (int i = 0; i < 512; ++i) {
        out[i] = g_tag_valu[i];
        if (reset) g_tag_valu[i] = 0;
    }
}

extern "C" void emu_jit_div_hist(uint64_t* out, int reset) {
    for (int i = 0; i < 32; ++i) {
        out[i] = g_div_hist[i];
        if (reset) g_div_hist[i] = 0;
    }
}

// build_tapeset as mh_tapes_jit runs it (no device): per code object, its max VGPR count and
// tape count into objs[2 i], objs[2 i + 1] (at most max_objs), and each tape's object index
// (or -1: not jitted) into tape_obj.  Returns the number of code objects, < 0 on error.
extern "C" int32_t emu_jit_build(const mh_node* nodes, const uint64_t* offs, uint32_t n_tapes,
                                 const uint32_t* consts, uint32_t n_consts, uint32_t n_vars,
                                 uint32_t max_vgpr, uint32_t threads, uint32_t* objs,
                                 uint32_t max_objs, int32_t* tape_obj, char* err, int errlen) {
    Options opt;
    opt.max_vgpr = max_vgpr;
    opt.short_circuit = g_short_circuit;
    opt.sample_rows = g_sample_rows;
    std::vector<Built> built;
    BuildStats stats;
    std::string e;
    if (!build_tapeset(nodes, offs, n_tapes, consts, n_consts, n_vars, false, opt, threads, built,
                       stats, e)) {
        snprintf(err, errlen, "%s", e.c_str());
        return -1;
    }
    for (uint32_t t = 0; t < n_tapes; ++t) tape_obj[t] = -1;
    for (uint32_t i = 0; i < built.size(); ++i) {
        if (i < max_objs) {
            objs[2 * i] = built[i].max_vgpr;
            objs[2 * i + 1] = (uint32_t)built[i].tape_ids.size();
        }
        for (uint32_t t : built[i].tape_ids) tape_obj[t] = (int32_t)i;
    }
    return (int32_t)built.size();
}

extern "C" void emu_jit_opcode_valu(uint64_t* out, int reset) {
    for (int d = 0; d < 2; ++d)
        for (int i = 0; i < 256; ++i) {
            out[256 * d + i] = g_opc_valu[d][i];
            if (reset) g_opc_valu[d][i] = 0;
        }
}

extern "C" void emu_jit_mov_tags(uint64_t* out, int reset) {
    for (int i = 0; i < 256; ++i) {
        out[i] = g_mov_tag[i];
        if (reset) g_mov_tag[i] = 0;
    }
}

extern "C" void emu_jit_tag_op(uint64_t* out, int reset) {
    for (int t = 0; t < 256; ++t)
        for (int o = 0; o < 128; ++o) {
            out[128 * t + o] = g_tag_op[t][o];
            if (reset) g_tag_op[t][o] = 0;
        }
}

extern "C" uint64_t emu_jit_sc_fallbacks(int reset) { return sc_fallbacks(reset != 0); }

// compaction study: [0] VALU before the first short-circuit test (all chunks), [1..65] chunks by
// live lanes at that test (64 = no test)
extern "C" void emu_jit_head_stats(uint64_t* out, int reset) {
    out[0] = g_valu_head;
    for (int i = 0; i <= 64; ++i) out[1 + i] = g_alive_hist[i];
    if (reset) {
        g_valu_head = 0;
        for (int i = 0; i <= 64; ++i) g_alive_hist[i] = 0;
    }
}

// compaction study: the segments recorded since the last reset, as (chunk | end flag, VALU since
// the chunk began, live-lane mask lo, hi) quadruples; returns the count (copies at most cap)
extern "C" uint64_t emu_jit_segments(uint32_t* out, uint64_t cap, int reset) {
    const uint64_t n = g_segs.size();
    for (uint64_t i = 0; i < n && i < cap; ++i) {
        out[4 * i] = g_segs[i].chunk;
        out[4 * i + 1] = g_segs[i].valu;
        out[4 * i + 2] = (uint32_t)g_segs[i].alive;
        out[4 * i + 3] = (uint32_t)(g_segs[i].alive >> 32);
    }
    if (reset) { g_segs.clear(); g_chunk_id = 0; }
    return n;
}
