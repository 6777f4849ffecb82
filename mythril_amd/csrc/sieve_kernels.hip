// Sieve kernels for gfx950: the tape interpreter, the assignment generator and VALU
// micro-benchmarks.  (Throughput runs over a whole tape set use the per-tape native code of
// jit.cpp instead; the interpreter serves queries and the tapes the native code does not cover.)
//
// Mapping: one lane = one candidate assignment (row); a 256-thread workgroup = 256 consecutive
// rows; every wave walks the launch's whole tape list, so the tape stream (instruction words,
// constants) is wave-uniform.  The asm core (asm_core.inc, gen_asm_core.py) takes each
// instruction's two words, and the next instruction's words plus inline constants, by scalar loads
// (s_load_dwordx16 into an SGPR bank) from the tape's global copy, issued one handler ahead, and
// dispatches with one s_setpc_b64 into 256-byte handler slots; the C++ driver below keeps a
// 64-instruction window in two VGPRs (lane j = instruction j, read with v_readlane) for the
// complex ops it executes itself.  Per-lane 256-bit values live in VGPRs: the accumulator X and
// the register file as 8 "limb planes" indexed by the wave-uniform register number
// (s_set_gpr_idx_on, no scratch).  Assignment columns 0..3 are loaded once per launch into
// R0..R3 and stay resident for every tape.  Per-tape results are reduced per workgroup in LDS and
// flushed with one atomic per tape per workgroup.
//
// Kernel variants (kernels.h variant_of): NR in {7, 9, 15} x {asm only, + C++ overflow
// predicates / unpinned columns, + keccak, + keccak/EVM};
// mh_run launches one variant per non-empty bucket of tapes, so a tape set's simple tapes run
// with the register budget (and occupancy) they need rather than the worst tape's.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "dev_isa.h"
#include "exec.h"
#include "kernels.h"
#include "u256_ops.h"

using namespace mh;

#ifndef MH_ASM_CORE
#define MH_ASM_CORE 1  // 0: every op through the C++ step() (reference / A-B builds)
#endif

namespace {

#include "asm_core.inc"

constexpr int kBlock = 256;
#ifndef MH_SIEVE_BLOCK
#define MH_SIEVE_BLOCK 256
#endif
// sieve workgroup size.  A/B on MI355X (config 5): 512 rows per workgroup cut the PMC traffic per
// launch from 9.4 to 5.5 GB (each staged tape chunk read once per 8 waves, half the result
// flushes) but ran 7 % slower (1.92e10 vs 2.07e10 evals/s: longer barriers around the LDS
// staging); the kernel is VALU-bound at ~2 GB/s of HBM, so 256 stays.
constexpr int kSieveBlock = MH_SIEVE_BLOCK;
// A short run (a query's guided first round: 4096 rows, 64 waves) is latency-bound, one wave per
// SIMD walking the whole tape; its workgroups are one wave each, so each wave gets a CU of its
// own (the CU's scalar unit, scalar and instruction caches): EtherThief-400's rounds 123 -> 112
// us (NR 15), 151 -> 136 us (NR 9 with complex ops) (profiles/r05zb; two waves per SIMD instead
// were slower, profiles/r05za).  Longer runs keep 256-thread workgroups, whose waves share one
// LDS instruction stage.  MH_SIEVE_SHORT_BLOCK=256 for A/B.
constexpr u64 kShortRows = 4096;
inline int short_block() {
    static const int b = [] {
        const char* e = std::getenv("MH_SIEVE_SHORT_BLOCK");
        return e && atoi(e) == 256 ? 256 : 64;
    }();
    return b;
}
inline int sieve_block(u64 rows) { return rows <= kShortRows ? short_block() : kSieveBlock; }
#ifndef MH_SIEVE_WAVES9
#define MH_SIEVE_WAVES9 1  // 0: every sieve variant at its natural register allocation
#endif
constexpr int kChunk = 64;  // tapes per LDS result chunk

// Register file: 8 limb planes of NR+1 VGPRs; R[NR] is the accumulator X (dev_isa.h).
template <int NR>
struct RegFile {
    typedef u32 plane_t __attribute__((ext_vector_type(NR + 1)));
    plane_t p0, p1, p2, p3, p4, p5, p6, p7;

    __device__ __forceinline__ void read(u32 r, u32* x) const {
        x[0] = p0[r]; x[1] = p1[r]; x[2] = p2[r]; x[3] = p3[r];
        x[4] = p4[r]; x[5] = p5[r]; x[6] = p6[r]; x[7] = p7[r];
    }
    __device__ __forceinline__ void write(u32 r, const u32* x) {
        p0[r] = x[0]; p1[r] = x[1]; p2[r] = x[2]; p3[r] = x[3];
        p4[r] = x[4]; p5[r] = x[5]; p6[r] = x[6]; p7[r] = x[7];
    }
    __device__ __forceinline__ u32 read0(u32 r) const { return p0[r]; }
};

// Instruction window: lane j of the wave holds slot (window base + j) of the tape in two VGPRs.
struct InsnCache {
    u32 w0, w1;
};

// The machine interface of exec.h's step() on the device (the complex ops).
template <int NR>
struct DevMachine {
    RegFile<NR> R;
    const KParams* p;
    u64 lrow;
    InsnCache ic;

    __device__ __forceinline__ u32 nrx() const { return NR; }
    __device__ __forceinline__ void read(u32 r, u32* v) const { R.read(r, v); }
    __device__ __forceinline__ u32 read0(u32 r) const { return R.read0(r); }
    __device__ __forceinline__ void write(u32 r, const u32* v) { R.write(r, v); }
    __device__ __forceinline__ void iconst(u32 slot, u32* v) const {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            v[2 * k] = __builtin_amdgcn_readlane(ic.w0, slot + k);
            v[2 * k + 1] = __builtin_amdgcn_readlane(ic.w1, slot + k);
        }
    }
    __device__ __forceinline__ void var(u32 col, u32* v) const {
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = p->assign[((u64)col * 8 + k) * p->capacity + lrow];
    }
};

__device__ __forceinline__ u64 splitmix64(u64 x) {
    x += 0x9E3779B97F4A7C15ull;
    u64 z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Run one tape from its first window ic: on return X (= R[NR]) holds the root.  The asm core
// runs the simple ops; each complex op, window change and the end come back here.  LDS holds the
// tape's slots (or global memory when the tape alone exceeds the LDS chunk).
template <int NR, int FEAT>
__device__ __forceinline__ void exec_tape(DevMachine<NR>& m, const uint2* src, InsnCache ic,
                                          u32 n, const uint2* gsrc) {
    u32 win = 0, ip = 0;
    for (;;) {
#if MH_ASM_CORE
        // MH_ASM_CORE_WINDOW: the core takes the slot from the tape's first one and changes
        // windows itself; the lane-held window ic is reloaded here only when it came back in
        // another window than it left
        const u32 at = MH_ASM_CORE_WINDOW ? win + ip : ip;
        const uint2* base = MH_ASM_CORE_WINDOW ? gsrc : gsrc + win;
        u32 back;
        if constexpr (FEAT != 0 && MH_ASM_LOADVAR) {
            // columns beyond the preloaded ones load inside the core (no exit per LOADVAR);
            // launch_sieve keeps capacity * 4 within 32 bits
            const u64 a = (u64)(uintptr_t)m.p->assign;
            back = AsmCore<NR>::run_lv(m.R.p0, m.R.p1, m.R.p2, m.R.p3, m.R.p4, m.R.p5, m.R.p6,
                                       m.R.p7, ic.w0, ic.w1, at, base, n, (u32)a,
                                       (u32)(a >> 32), (u32)(m.p->capacity * 4u),
                                       (u32)m.lrow * 4u);
        } else {
            back = AsmCore<NR>::run(m.R.p0, m.R.p1, m.R.p2, m.R.p3, m.R.p4, m.R.p5, m.R.p6,
                                    m.R.p7, ic.w0, ic.w1, at, base, n);
        }
        if (MH_ASM_CORE_WINDOW) {
            const u32 w = back & ~(u32)(MH_WINDOW - 1);
            if (w != win) {
                win = w;
                const u32 j = win + (threadIdx.x & 63u);
                ic.w0 = ic.w1 = 0u;
                if (j < n) {
                    const uint2 v = src[j];
                    ic.w0 = v.x;
                    ic.w1 = v.y;
                }
            }
            ip = back - win;
        } else {
            ip = back;
        }
#endif
        const u32 w0 = __builtin_amdgcn_readlane(ic.w0, ip);
        const u32 w1 = __builtin_amdgcn_readlane(ic.w1, ip);
        const u32 op = w1 & 0xFFu;
#if MH_ASM_CORE
        // D_BANDZ: the asm core left there because the conjunction is 0 in every lane (X = 0)
        if (op == D_END || op == D_BANDZ) break;
#else
        if (op == D_END) break;
#endif
        if (op == D_WINDOW) {
            win += MH_WINDOW;
            const u32 j = win + (threadIdx.x & 63u);
            ic.w0 = ic.w1 = 0u;
            if (j < n) {
                const uint2 v = src[j];
                ic.w0 = v.x;
                ic.w1 = v.y;
            }
            ip = 0;
            continue;
        }
#if MH_ASM_CORE
        if constexpr (FEAT == 0) {
            break;  // asm-only variant: the host never buckets a complex op here
        } else {
            // complex op: operands out of the register file by asm, the op in C++, the result
            // back by asm -- the C++ code never touches the planes, so they stay in their VGPRs
            typedef typename AsmCore<NR>::v8_t v8_t;
            u32 z[8];
            if (op == D_LOADVAR) {
                // a column beyond the preloaded ones (wide query schemas): no operands to fetch
                m.var((w1 >> 17) & MH_AUX_MAX, z);
            } else {
                v8_t xv, yv, cv;
                AsmCore<NR>::fetch(m.R.p0, m.R.p1, m.R.p2, m.R.p3, m.R.p4, m.R.p5, m.R.p6,
                                   m.R.p7, ic.w0, ic.w1, ip, w0, w1, xv, yv, cv);
                u32 x[8], y[8], c3[8];
#pragma unroll
                for (int k = 0; k < 8; ++k) { x[k] = xv[k]; y[k] = yv[k]; c3[k] = cv[k]; }
                complex_op<FEAT>(m, w1, x, y, c3, z);
            }
            v8_t zv;
#pragma unroll
            for (int k = 0; k < 8; ++k) zv[k] = z[k];
            AsmCore<NR>::commit(m.R.p0, m.R.p1, m.R.p2, m.R.p3, m.R.p4, m.R.p5, m.R.p6, m.R.p7,
                                w0, zv);
            ip += (w1 & F_YC) ? 5u : 1u;
        }
#else
        m.ic = ic;
        ip += step<FEAT, true>(m, w0, w1, ip);
        // D_BANDZ runs like D_BAND; the tape ends only when no lane's conjunction is left true
        // (X = 0 in every lane, the root of every row the wave holds), as the asm core's exit
        if (op == D_BANDZ && __builtin_amdgcn_ballot_w64((m.read0(m.nrx()) & 1u) != 0u) == 0ull)
            break;
#endif
    }
}

template <int NR>
__device__ __forceinline__ void preload(DevMachine<NR>& m, const KParams& p) {
#pragma unroll
    for (u32 v = 0; v < MH_MAX_PRELOAD; ++v) {
        if (v < p.n_pre) {
            u32 x[8];
            m.var(v, x);
            m.R.write(v, x);
        }
    }
}

// LDS-staged instruction chunk: up to kChunk tapes whose instruction words fit in kLdsInsns.
constexpr u32 kLdsInsns = 2048;  // 16 KB

__device__ __forceinline__ InsnCache lds_insns(const uint2* s_insn, u32 off, u32 n, u32 first) {
    const u32 j = first + (threadIdx.x & 63u);
    InsnCache c{0u, 0u};
    if (j < n) {
        const uint2 v = s_insn[off + j];
        c.w0 = v.x;
        c.w1 = v.y;
    }
    return c;
}

template <int NR, int FEAT, int BLOCK>
__device__ __forceinline__ void sieve_body(const KParams& p) {
    __shared__ uint2 s_insn[kLdsInsns];
    __shared__ u32 s_off[kChunk], s_n[kChunk], s_rb[kChunk], s_tid[kChunk];
    __shared__ u32 s_meta[4];  // tapes in chunk, first word index, words, streaming flag
    __shared__ unsigned long long s_min[kChunk];
    __shared__ unsigned long long s_cnt[kChunk];
    const u32 tid = threadIdx.x;
    const u64 row = p.row_first + (u64)blockIdx.x * BLOCK + tid;
    const bool valid = row < p.row_first + p.row_count;
    DevMachine<NR> m;
    m.p = &p;
    m.lrow = valid ? row : p.row_first;
    preload<NR>(m, p);
    const u64 block_first = p.index_base + p.row_first + (u64)blockIdx.x * BLOCK;
    const u64 wave_first = block_first + (tid & ~63u);
    // grid y splits the tape list (a short run -- a query's 256-row first round is one
    // workgroup -- spreads its tapes over CUs instead of running them all on one)
    const u32 id_lo = (u32)((u64)p.n_ids * blockIdx.y / gridDim.y);
    const u32 n_ids = (u32)((u64)p.n_ids * (blockIdx.y + 1) / gridDim.y) - id_lo;
    const u32* tape_ids = p.tape_ids + id_lo;
    for (u32 cb = 0; cb < n_ids;) {
        __syncthreads();  // previous chunk's LDS fully consumed
        if (tid < (u32)kChunk) {
            // chunk formation by wave 0: the bucket's tapes are contiguous in the word array,
            // so the chunk is the longest prefix of the next kChunk tapes within kLdsInsns
            const u32 i = cb + tid;
            const bool in = i < n_ids;
            const u32 t = in ? tape_ids[i] : 0u;
            const mh_dev_tape h = p.tapes[t];
            const u32 base = __builtin_amdgcn_readfirstlane(h.insn_off);
            const u32 end = h.insn_off + h.n_insns - base;
            const unsigned long long fit = __builtin_amdgcn_ballot_w64(in && end <= kLdsInsns);
            u32 nt = (u32)__builtin_popcountll(fit);
            const u32 stream = nt == 0 ? 1u : 0u;  // a single tape larger than the LDS chunk
            nt = stream ? 1u : nt;
            s_off[tid] = stream ? h.insn_off : h.insn_off - base;
            s_n[tid] = h.n_insns;
            s_rb[tid] = h.root_bool;
            s_tid[tid] = t;
            s_min[tid] = (p.mode == MH_MODE_FIRST_HIT && in && p.first_hit)
                             ? p.first_hit[t - p.result_base] : ~0ull;
            s_cnt[tid] = 0;
            if (tid == nt - 1) {
                s_meta[0] = nt;
                s_meta[1] = base;
                s_meta[2] = stream ? 0u : end;
                s_meta[3] = stream;
            }
        }
        __syncthreads();
        const u32 nt = __builtin_amdgcn_readfirstlane(s_meta[0]);
        const u32 wbase = __builtin_amdgcn_readfirstlane(s_meta[1]);
        const u32 nwords = __builtin_amdgcn_readfirstlane(s_meta[2]);
        const bool stream = __builtin_amdgcn_readfirstlane(s_meta[3]) != 0;
        for (u32 k = tid; k < nwords; k += BLOCK) s_insn[k] = p.insns[wbase + k];
        __syncthreads();
        u32 off = __builtin_amdgcn_readfirstlane(s_off[0]);
        u32 n = __builtin_amdgcn_readfirstlane(s_n[0]);
        InsnCache ic = stream ? lds_insns(p.insns, off, n, 0) : lds_insns(s_insn, off, n, 0);
        for (u32 j = 0; j < nt; ++j) {
            const u32 jn = j + 1 < nt ? j + 1 : j;
            const u32 off_next = __builtin_amdgcn_readfirstlane(s_off[jn]);
            const u32 n_next = __builtin_amdgcn_readfirstlane(s_n[jn]);
            InsnCache ic_next{0u, 0u};
            if (!stream) ic_next = lds_insns(s_insn, off_next, n_next, 0);
            bool skip = false;
            if (p.mode == MH_MODE_FIRST_HIT) {
                // early exit: a smaller witness is already known for this tape
                const u64 km = s_min[j];
                const u64 known = ((u64)__builtin_amdgcn_readfirstlane((u32)(km >> 32)) << 32) |
                                  __builtin_amdgcn_readfirstlane((u32)km);
                skip = known < wave_first;
            }
            if (!skip) {
                exec_tape<NR, FEAT>(m, stream ? p.insns + off : s_insn + off, ic, n,
                                    p.insns + (stream ? off : wbase + off));
                u32 X[8];
                m.R.read(NR, X);
                const u32 rb = __builtin_amdgcn_readfirstlane(s_rb[j]);
                if (p.values_out) {  // parity path: the root value of (tape, row)
                    if (rb) {
                        X[0] &= 1u;
#pragma unroll
                        for (int k = 1; k < 8; ++k) X[k] = 0;
                    }
                    if (valid) {
                        const u64 r = row - p.row_first;
#pragma unroll
                        for (int k = 0; k < 8; ++k)
                            p.values_out[((u64)(id_lo + cb + j) * 8 + k) * p.row_count + r] =
                                X[k];
                    }
                }
                const u32 res = rb ? (X[0] & 1u) : (is_zero256(X) ? 0u : 1u);
                const unsigned long long mask = __builtin_amdgcn_ballot_w64(valid && res);
                if (p.masks) {  // a part of a split tape: its wave mask, combined later
                    if ((tid & 63u) == 0) {
                        const u32 t = __builtin_amdgcn_readfirstlane(s_tid[j]);
                        const u64 w = ((u64)blockIdx.x * BLOCK + (tid & ~63u)) / 64u;
                        p.masks[(u64)(t - p.mask_base) * p.mask_stride + w] = mask;
                    }
                } else if (mask && (tid & 63u) == 0) {
                    atomicAdd(&s_cnt[j], (unsigned long long)__builtin_popcountll(mask));
                    atomicMin(&s_min[j], (unsigned long long)(wave_first + __builtin_ctzll(mask)));
                }
            }
            off = off_next;
            n = n_next;
            ic = ic_next;
        }
        __syncthreads();
        if (tid < nt) {
            const u32 ti = s_tid[tid] - p.result_base;
            if (s_cnt[tid] && p.hit_count) atomicAdd(&p.hit_count[ti], s_cnt[tid]);
            if (s_min[tid] != ~0ull && p.first_hit) atomicMin(&p.first_hit[ti], s_min[tid]);
        }
        cb += nt;
    }
}

__global__ void __launch_bounds__(kBlock) generate_kernel(u32* assign, u64 stride, u64 rows,
                                                          u32 n_vars, u64 seed, u64 base) {
    const u64 row = (u64)blockIdx.x * kBlock + threadIdx.x;
    if (row >= rows) return;
    for (u32 v = 0; v < n_vars; ++v) {
#pragma unroll
        for (u32 k = 0; k < 8; ++k) {
            const u64 key = splitmix64(seed ^ (((u64)v * 8 + k) * 0xD1B54A32D192ED03ull));
            assign[((u64)v * 8 + k) * stride + row] = (u32)splitmix64(key ^ (base + row));
        }
    }
}

// Integer VALU issue-rate probe: 32 wave-instructions of ONE kind per loop iteration, written in
// asm so the compiler can neither fuse nor drop them (round 1's C++ kind 2 could compile
// xor + add into one v_xad_u32).  Eight independent accumulators per lane (dependency distance
// 8), the launch's occupancy set by `blocks` (256 threads = 4 waves each).  Kinds (dev_isa.h
// mh_mb_kind): 0 v_add_co/v_addc 256-bit carry chains (4 chains, each its own SGPR carry pair);
// 1 v_mad_u64_u32; 2 v_add_u32; 3 v_xor_b32; 4 v_alignbit_b32; 5 v_cndmask_b32 (SGPR mask);
// 6 v_or3_b32; 7 v_readlane_b32 (VALU -> SGPR); 8 v_mov_b32; 9 v_add_co_u32 with a VCC carry-out
// but no carry-in (independent); 10 v_sub_co_u32 chains through VCC (one chain, dependent).
#define MB8(op) op op op op op op op op
template <int KIND>
__global__ void __launch_bounds__(kBlock) microbench_kernel(u32 iters, u32* sink) {
    u32 a0 = threadIdx.x * 2654435761u, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
        a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    const u32 y = blockIdx.x | 1u;
    for (u32 i = 0; i < iters; ++i) {
        if constexpr (KIND == 0) {
            // 4 independent 8-limb chains = 32 instructions
            asm volatile(
                MB8("v_add_co_u32 %0, s[20:21], %0, %8\n v_addc_co_u32 %1, s[20:21], %1, %8, s[20:21]\n"
                    "v_addc_co_u32 %2, s[20:21], %2, %8, s[20:21]\n v_addc_co_u32 %3, s[20:21], %3, %8, s[20:21]\n")
                : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                : "v"(y) : "s20", "s21");
        } else if constexpr (KIND == 1) {
            u64 m0 = ((u64)a1 << 32) | a0, m1 = ((u64)a3 << 32) | a2, m2 = ((u64)a5 << 32) | a4,
                m3 = ((u64)a7 << 32) | a6;
            asm volatile(MB8("v_mad_u64_u32 %0, s[20:21], %4, %5, %0\n v_mad_u64_u32 %1, s[22:23], %4, %5, %1\n"
                             "v_mad_u64_u32 %2, s[24:25], %4, %5, %2\n v_mad_u64_u32 %3, s[26:27], %4, %5, %3\n")
                         : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3) : "v"(y ^ 0x9E3779B9u), "v"(y)
                         : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27");
            a0 = (u32)m0; a1 = (u32)(m0 >> 32); a2 = (u32)m1; a3 = (u32)(m1 >> 32);
            a4 = (u32)m2; a5 = (u32)(m2 >> 32); a6 = (u32)m3; a7 = (u32)(m3 >> 32);
        } else if constexpr (KIND == 7) {
            u32 acc = 0;
            asm volatile(MB8("v_readlane_b32 s20, %1, 1\n v_readlane_b32 s21, %1, 2\n"
                             "v_readlane_b32 s22, %1, 3\n v_readlane_b32 s23, %1, 4\n")
                         "s_add_u32 %0, s20, s23\n"
                         : "+s"(acc) : "v"(a0) : "s20", "s21", "s22", "s23");
            a1 += acc;
        } else if constexpr (KIND == 10) {
            asm volatile(MB8("v_sub_co_u32 %0, vcc, %0, %8\n v_subb_co_u32 %1, vcc, %1, %8, vcc\n"
                             "v_subb_co_u32 %2, vcc, %2, %8, vcc\n v_subb_co_u32 %3, vcc, %3, %8, vcc\n")
                         : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                         : "v"(y) : "vcc");
        } else {
#define MB_ONE(ins) asm volatile(MB8(ins " %0, %0, %8\n " ins " %1, %1, %8\n " ins " %2, %2, %8\n " ins " %3, %3, %8\n") \
    : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(y))
            if constexpr (KIND == 2) MB_ONE("v_add_u32");
            if constexpr (KIND == 3) MB_ONE("v_xor_b32");
            if constexpr (KIND == 4)
                asm volatile(MB8("v_alignbit_b32 %0, %0, %1, 7\n v_alignbit_b32 %1, %1, %2, 9\n"
                                 "v_alignbit_b32 %2, %2, %3, 11\n v_alignbit_b32 %3, %3, %4, 13\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
            if constexpr (KIND == 5)
                asm volatile("s_mov_b64 s[20:21], 0x5555\n"
                             MB8("v_cndmask_b32_e64 %0, %0, %8, s[20:21]\n v_cndmask_b32_e64 %1, %1, %8, s[20:21]\n"
                                 "v_cndmask_b32_e64 %2, %2, %8, s[20:21]\n v_cndmask_b32_e64 %3, %3, %8, s[20:21]\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(y) : "s20", "s21");
            if constexpr (KIND == 6)
                asm volatile(MB8("v_or3_b32 %0, %0, %8, %4\n v_or3_b32 %1, %1, %8, %5\n"
                                 "v_or3_b32 %2, %2, %8, %6\n v_or3_b32 %3, %3, %8, %7\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(y));
            if constexpr (KIND == 8)
                asm volatile(MB8("v_mov_b32 %0, %4\n v_mov_b32 %1, %5\n v_mov_b32 %2, %6\n v_mov_b32 %3, %7\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
            if constexpr (KIND == 9)
                asm volatile(MB8("v_add_co_u32 %0, vcc, %0, %8\n v_add_co_u32 %1, vcc, %1, %8\n"
                                 "v_add_co_u32 %2, vcc, %2, %8\n v_add_co_u32 %3, vcc, %3, %8\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(y) : "vcc");
            if constexpr (KIND == 11)  // v_cndmask_b32_e32: mask in VCC (implicit)
                asm volatile("s_mov_b64 vcc, 0x5555\n"
                             MB8("v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n"
                                 "v_cndmask_b32 %2, %2, %8, vcc\n v_cndmask_b32 %3, %3, %8, vcc\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(y) : "vcc");
            if constexpr (KIND == 12)  // v_cmp_eq_u32_e32 (VCC written), results folded by s_and
                asm volatile(MB8("v_cmp_eq_u32 vcc, %0, %8\n v_cmp_eq_u32 vcc, %1, %8\n"
                                 "v_cmp_eq_u32 vcc, %2, %8\n v_cmp_eq_u32 vcc, %3, %8\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(y) : "vcc");
            if constexpr (KIND == 13)  // VOP2 with a 32-bit literal (8-byte instruction)
                asm volatile(MB8("v_xor_b32 %0, 0x12345678, %0\n v_xor_b32 %1, 0x2345678a, %1\n"
                                 "v_xor_b32 %2, 0x345678ab, %2\n v_xor_b32 %3, 0x45678abc, %3\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
            if constexpr (KIND == 14) MB_ONE("v_lshlrev_b32");
            if constexpr (KIND == 15)  // VOP3 without an SGPR write or constant
                asm volatile(MB8("v_add3_u32 %0, %0, %8, %4\n v_add3_u32 %1, %1, %8, %5\n"
                                 "v_add3_u32 %2, %2, %8, %6\n v_add3_u32 %3, %3, %8, %7\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(y));
            if constexpr (KIND == 16) {  // v_fma_f64 (4 independent pairs)
                double d0 = a0, d1 = a1, d2 = a2, d3 = a3;
                const double e = 1.0000001;
                asm volatile(MB8("v_fma_f64 %0, %0, %4, %4\n v_fma_f64 %1, %1, %4, %4\n"
                                 "v_fma_f64 %2, %2, %4, %4\n v_fma_f64 %3, %3, %4, %4\n")
                             : "+v"(d0), "+v"(d1), "+v"(d2), "+v"(d3) : "v"(e));
                a0 = (u32)d0 ^ (u32)d1 ^ (u32)d2 ^ (u32)d3;
            }
            if constexpr (KIND == 17) MB_ONE("v_xnor_b32");
            if constexpr (KIND == 18) MB_ONE("v_and_b32");
            if constexpr (KIND == 19) MB_ONE("v_or_b32");
            if constexpr (KIND == 20)
                asm volatile(MB8("v_not_b32 %0, %0\n v_not_b32 %1, %1\n v_not_b32 %2, %2\n v_not_b32 %3, %3\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
            // dependent chains (latency at one wave per SIMD, not throughput): one accumulator
            if constexpr (KIND == 25) {  // v_mad_u64_u32 into one 64-bit accumulator
                u64 m0 = ((u64)a1 << 32) | a0;
                asm volatile(MB8("v_mad_u64_u32 %0, s[20:21], %1, %2, %0\n v_mad_u64_u32 %0, s[20:21], %1, %2, %0\n"
                                 "v_mad_u64_u32 %0, s[20:21], %1, %2, %0\n v_mad_u64_u32 %0, s[20:21], %1, %2, %0\n")
                             : "+v"(m0) : "v"(a2), "v"(y) : "s20", "s21");
                a0 = (u32)m0; a1 = (u32)(m0 >> 32);
            }
            if constexpr (KIND == 26)  // v_add_u32 into one register
                asm volatile(MB8("v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
                                 "v_add_u32 %0, %0, %1\n") : "+v"(a0) : "v"(y));
            if constexpr (KIND == 27)  // v_addc_co_u32 through VCC and one register
                asm volatile("v_add_co_u32 %0, vcc, %0, %1\n"
                             MB8("v_addc_co_u32 %0, vcc, %0, %1, vcc\n v_addc_co_u32 %0, vcc, %0, %1, vcc\n"
                                 "v_addc_co_u32 %0, vcc, %0, %1, vcc\n v_addc_co_u32 %0, vcc, %0, %1, vcc\n")
                             : "+v"(a0) : "v"(y) : "vcc");
            if constexpr (KIND == 28) {  // two v_mad_u64_u32 accumulators interleaved
                u64 m0 = ((u64)a1 << 32) | a0, m1 = ((u64)a3 << 32) | a2;
                asm volatile(MB8("v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n v_mad_u64_u32 %1, s[22:23], %2, %3, %1\n"
                                 "v_mad_u64_u32 %0, s[20:21], %2, %3, %0\n v_mad_u64_u32 %1, s[22:23], %2, %3, %1\n")
                             : "+v"(m0), "+v"(m1) : "v"(a4), "v"(y) : "s20", "s21", "s22", "s23");
                a0 = (u32)m0 ^ (u32)m1; a1 = (u32)(m0 >> 32) ^ (u32)(m1 >> 32);
            }
            if constexpr (KIND == 29) {  // product scanning: mad into the accumulator, carry count
                u64 m0 = ((u64)a1 << 32) | a0;
                asm volatile(MB8("v_mad_u64_u32 %0, vcc, %2, %3, %0\n v_addc_co_u32 %1, vcc, 0, %1, vcc\n")
                             MB8("v_mad_u64_u32 %0, vcc, %2, %3, %0\n v_addc_co_u32 %1, vcc, 0, %1, vcc\n")
                             : "+v"(m0), "+v"(a3) : "v"(a4), "v"(y) : "vcc");
                a0 = (u32)m0; a1 = (u32)(m0 >> 32);
            }
            if constexpr (KIND == 30)  // v_cmp into VCC, then v_cndmask reading it (compare chains)
                asm volatile(MB8("v_cmp_lt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc\n")
                             MB8("v_cmp_lt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc\n")
                             : "+v"(a0) : "v"(y) : "vcc");
            // mixed classes (independent): do quarter-rate and full-rate issue costs add?
            if constexpr (KIND == 31) {  // v_mad_u64_u32 / v_add_u32 alternating
                u64 m0 = ((u64)a1 << 32) | a0, m1 = ((u64)a3 << 32) | a2;
                asm volatile(MB8("v_mad_u64_u32 %0, s[20:21], %4, %5, %0\n v_add_u32 %2, %2, %5\n"
                                 "v_mad_u64_u32 %1, s[22:23], %4, %5, %1\n v_add_u32 %3, %3, %5\n")
                             : "+v"(m0), "+v"(m1), "+v"(a4), "+v"(a5) : "v"(a6), "v"(y)
                             : "s20", "s21", "s22", "s23");
                a0 = (u32)m0 ^ (u32)m1; a1 = (u32)(m0 >> 32) ^ (u32)(m1 >> 32);
            }
            if constexpr (KIND == 32)  // v_addc_co_u32 chain / v_xor_b32 alternating
                asm volatile("v_add_co_u32 %0, vcc, %0, %4\n"
                             MB8("v_addc_co_u32 %0, vcc, %0, %4, vcc\n v_xor_b32 %2, %2, %4\n"
                                 "v_addc_co_u32 %1, vcc, %1, %4, vcc\n v_xor_b32 %3, %3, %4\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(y) : "vcc");
            if constexpr (KIND == 33)  // two v_mad_u64_u32 per v_add_u32 (the multiply's mix)
                asm volatile(MB8("v_mad_u64_u32 v[40:41], s[20:21], %4, %5, v[40:41]\n"
                                 "v_mad_u64_u32 v[42:43], s[22:23], %4, %5, v[42:43]\n"
                                 "v_add_u32 %0, %0, %5\n v_add_u32 %1, %1, %5\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(a6), "v"(y)
                             : "s20", "s21", "s22", "s23", "v40", "v41", "v42", "v43");
            // gfx950's 3-input bitwise op (truth table 0xd2: x ^ (~y & z), Keccak's chi)
            if constexpr (KIND == 34)
                asm volatile(MB8("v_bitop3_b32 %0, %0, %8, %4 bitop3:0xd2\n v_bitop3_b32 %1, %1, %8, %5 bitop3:0xd2\n"
                                 "v_bitop3_b32 %2, %2, %8, %6 bitop3:0xd2\n v_bitop3_b32 %3, %3, %8, %7 bitop3:0xd2\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(y));
            if constexpr (KIND == 35)  // v_bitop3_b32 / v_alignbit_b32 alternating (theta + rho)
                asm volatile(MB8("v_bitop3_b32 %0, %0, %8, %4 bitop3:0x96\n v_alignbit_b32 %1, %1, %5, 7\n"
                                 "v_bitop3_b32 %2, %2, %8, %6 bitop3:0x96\n v_alignbit_b32 %3, %3, %7, 9\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(y));
            // round 6: 64-bit compares and the other candidates for the
            // 4-cycle class -- v_cmp_{lt,eq}_u64 into SGPR pairs, v_lshl_add_u64, the 32-bit
            // multiplies, a VOP3 v_sub_co into an SGPR pair, v_cmp_lt_u32 into an SGPR pair, and
            // the lexicographic 256-bit `<` as 64-bit compares (4 lt + 3 eq + SALU folds)
            if constexpr (KIND == 36 || KIND == 37) {
                u64 m0 = ((u64)a1 << 32) | a0, m1 = ((u64)a3 << 32) | a2, m2 = ((u64)a5 << 32) | a4,
                    m3 = ((u64)a7 << 32) | a6, yy = ((u64)y << 32) | (y ^ 0x9E3779B9u);
                if constexpr (KIND == 36)
                    asm volatile(MB8("v_cmp_lt_u64_e64 s[20:21], %0, %4\n v_cmp_lt_u64_e64 s[22:23], %1, %4\n"
                                     "v_cmp_lt_u64_e64 s[24:25], %2, %4\n v_cmp_lt_u64_e64 s[26:27], %3, %4\n")
                                 : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3) : "v"(yy)
                                 : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27");
                else
                    asm volatile(MB8("v_cmp_eq_u64_e64 s[20:21], %0, %4\n v_cmp_eq_u64_e64 s[22:23], %1, %4\n"
                                     "v_cmp_eq_u64_e64 s[24:25], %2, %4\n v_cmp_eq_u64_e64 s[26:27], %3, %4\n")
                                 : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3) : "v"(yy)
                                 : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27");
                a0 ^= (u32)m0 ^ (u32)m1; a1 ^= (u32)m2 ^ (u32)m3;
            }
            if constexpr (KIND == 38) {
                u64 m0 = ((u64)a1 << 32) | a0, m1 = ((u64)a3 << 32) | a2, m2 = ((u64)a5 << 32) | a4,
                    m3 = ((u64)a7 << 32) | a6, yy = ((u64)y << 32) | (y ^ 0x9E3779B9u);
                asm volatile(MB8("v_lshl_add_u64 %0, %0, 0, %4\n v_lshl_add_u64 %1, %1, 0, %4\n"
                                 "v_lshl_add_u64 %2, %2, 0, %4\n v_lshl_add_u64 %3, %3, 0, %4\n")
                             : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3) : "v"(yy));
                a0 = (u32)m0; a1 = (u32)(m0 >> 32); a2 = (u32)m1; a3 = (u32)(m1 >> 32);
                a4 = (u32)m2; a5 = (u32)(m2 >> 32); a6 = (u32)m3; a7 = (u32)(m3 >> 32);
            }
            if constexpr (KIND == 39) MB_ONE("v_mul_lo_u32");
            if constexpr (KIND == 40) MB_ONE("v_mul_hi_u32");
            if constexpr (KIND == 41) MB_ONE("v_mul_u32_u24");
            if constexpr (KIND == 42)
                asm volatile(MB8("v_sub_co_u32_e64 %0, s[20:21], %0, %8\n v_sub_co_u32_e64 %1, s[22:23], %1, %8\n"
                                 "v_sub_co_u32_e64 %2, s[24:25], %2, %8\n v_sub_co_u32_e64 %3, s[26:27], %3, %8\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(y) : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27");
            if constexpr (KIND == 43)
                asm volatile(MB8("v_cmp_lt_u32_e64 s[20:21], %0, %8\n v_cmp_lt_u32_e64 s[22:23], %1, %8\n"
                                 "v_cmp_lt_u32_e64 s[24:25], %2, %8\n v_cmp_lt_u32_e64 s[26:27], %3, %8\n")
                             : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                             : "v"(y) : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27");
            if constexpr (KIND == 44) {
                // a 256-bit unsigned `<` as 64-bit compares: lt3 | eq3 & (lt2 | eq2 & (lt1 | eq1 &
                // lt0)), 7 VALU compares (+ 1 filler compare, so 4 of them are the 32 VALU of an
                // iteration) and the folds on the scalar unit
                u64 m0 = ((u64)a1 << 32) | a0, m1 = ((u64)a3 << 32) | a2, m2 = ((u64)a5 << 32) | a4,
                    m3 = ((u64)a7 << 32) | a6, yy = ((u64)y << 32) | (y ^ 0x9E3779B9u);
#define LT256 "v_cmp_lt_u64_e64 s[20:21], %0, %4\n v_cmp_lt_u64_e64 s[22:23], %1, %4\n" \
              "v_cmp_eq_u64_e64 s[24:25], %1, %4\n v_cmp_lt_u64_e64 s[26:27], %2, %4\n" \
              "s_and_b64 s[20:21], s[24:25], s[20:21]\n s_or_b64 s[20:21], s[22:23], s[20:21]\n" \
              "v_cmp_eq_u64_e64 s[24:25], %2, %4\n v_cmp_lt_u64_e64 s[22:23], %3, %4\n" \
              "s_and_b64 s[20:21], s[24:25], s[20:21]\n s_or_b64 s[20:21], s[26:27], s[20:21]\n" \
              "v_cmp_eq_u64_e64 s[24:25], %3, %4\n v_cmp_eq_u64_e64 s[26:27], %0, %4\n" \
              "s_and_b64 s[20:21], s[24:25], s[20:21]\n s_or_b64 s[20:21], s[22:23], s[20:21]\n"
                asm volatile(LT256 LT256 LT256 LT256
                             : "+v"(m0), "+v"(m1), "+v"(m2), "+v"(m3) : "v"(yy)
                             : "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27");
#undef LT256
                a0 ^= (u32)m0 ^ (u32)m1; a1 ^= (u32)m2 ^ (u32)m3;
            }
            // partial EXEC masks: does the SIMD skip lane groups that are all inactive?
            if constexpr (KIND >= 21 && KIND <= 24) {
                constexpr uint64_t kExec = KIND == 21 || KIND == 22 ? 0x00000000FFFFFFFFull
                                         : KIND == 23 ? 0x000000000000FFFFull
                                                      : 0x5555555555555555ull;
                if constexpr (KIND == 22)
                    asm volatile("s_mov_b64 s[22:23], exec\n s_mov_b64 exec, %9\n"
                                 MB8("v_alignbit_b32 %0, %0, %1, 7\n v_alignbit_b32 %1, %1, %2, 9\n"
                                     "v_alignbit_b32 %2, %2, %3, 11\n v_alignbit_b32 %3, %3, %4, 13\n")
                                 "s_mov_b64 exec, s[22:23]\n"
                                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                                 : "v"(y), "s"(kExec) : "s22", "s23");
                else
                    asm volatile("s_mov_b64 s[22:23], exec\n s_mov_b64 exec, %9\n"
                                 MB8("v_xor_b32 %0, %0, %8\n v_xor_b32 %1, %1, %8\n"
                                     "v_xor_b32 %2, %2, %8\n v_xor_b32 %3, %3, %8\n")
                                 "s_mov_b64 exec, s[22:23]\n"
                                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                                 : "v"(y), "s"(kExec) : "s22", "s23");
            }
#undef MB_ONE
        }
    }
    const u32 r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
    if (r == 0x12345678u) sink[0] = r;
}
#undef MB8

// Minimum waves per SIMD a variant is compiled for (amdgpu_waves_per_eu; 1 = the natural register
// allocation).  Occupancy decides this latency-bound interpreter's issue rate, so variants whose
// natural allocation lands just above a wave boundary are held below it, at the price of a few
// spilled values outside the asm core: NR 9 asm-only 136 -> 128 VGPRs (four waves, was three);
// NR 9 keccak / keccak+EVM 256 + 2 AGPRs -> 256 (two waves, was one).
constexpr int sieve_min_waves(int nr, int feat) {
    return MH_SIEVE_WAVES9 == 0 ? 1 : nr == 9 && feat == 0 ? 4 : nr == 9 && feat >= 8 ? 2 : 1;
}

template <int NR, int FEAT, int BLOCK>
__global__ void __launch_bounds__(BLOCK)
__attribute__((amdgpu_waves_per_eu(sieve_min_waves(NR, FEAT), 8))) sieve_kernel(const KParams p) {
    sieve_body<NR, FEAT, BLOCK>(p);
}

// one workgroup per split tape: the AND of its parts' wave masks (kernels.h launch_combine)
__global__ void __launch_bounds__(256)
    combine_kernel(const unsigned long long* masks, u64 stride, const u32* split, u32 mask_base,
                   u32 result_base, u64 index0, unsigned long long* first_hit,
                   unsigned long long* hit_count) {
    const u32 t = split[3 * blockIdx.x], s0 = split[3 * blockIdx.x + 1] - mask_base,
              k = split[3 * blockIdx.x + 2];
    u64 first = ~0ull, cnt = 0;
    for (u64 w = threadIdx.x; w < stride; w += 256) {
        unsigned long long m = ~0ull;
        for (u32 i = 0; i < k; ++i) m &= masks[(u64)(s0 + i) * stride + w];
        if (m) {
            cnt += (u64)__builtin_popcountll(m);
            if (first == ~0ull) first = index0 + 64 * w + (u64)__builtin_ctzll(m);
        }
    }
    if (first != ~0ull && first_hit) atomicMin(&first_hit[t - result_base], first);
    if (cnt && hit_count) atomicAdd(&hit_count[t - result_base], cnt);
}

template <int NR, int FEAT, int BLOCK>
hipError_t launch_block(const KParams& p, hipStream_t stream) {
    const u64 blocks = (p.row_count + BLOCK - 1) / BLOCK;
    // fewer row blocks than CUs: split the tapes over grid y until the chip has ~256 workgroups
    u64 gy = 1;
    if (blocks < 256) gy = std::min<u64>(p.n_ids, (256 + blocks - 1) / blocks);
    // the parts of split tapes (conjunct-parallel short runs) each get their own workgroups up
    // to 4096 in all: a part walked after another on the same workgroup gains no latency
    if (p.masks && blocks < 4096) gy = std::max<u64>(gy, std::min<u64>(p.n_ids, 4096 / blocks));
    hipLaunchKernelGGL((sieve_kernel<NR, FEAT, BLOCK>), dim3((unsigned)blocks, (unsigned)gy),
                       dim3(BLOCK), 0, stream, p);
    return hipGetLastError();
}

template <int NR, int FEAT>
hipError_t launch_variant(const KParams& p, hipStream_t stream) {
    return sieve_block(p.row_count) == 64 ? launch_block<NR, FEAT, 64>(p, stream)
                                          : launch_block<NR, FEAT, kSieveBlock>(p, stream);
}

}  // namespace

namespace mh {

uint64_t sieve_mask_stride(uint64_t row_count) {  // the waves of the run's workgroups
    const u64 b = (u64)sieve_block(row_count);
    return (row_count + b - 1) / b * (b / 64);
}

hipError_t launch_combine(const unsigned long long* masks, uint64_t stride, const uint32_t* split,
                          uint32_t n_split, uint32_t mask_base, uint32_t result_base,
                          uint64_t index0, unsigned long long* first_hit,
                          unsigned long long* hit_count, hipStream_t stream) {
    if (n_split == 0) return hipSuccess;
    hipLaunchKernelGGL(combine_kernel, dim3(n_split), dim3(256), 0, stream, masks, stride, split,
                       mask_base, result_base, index0, first_hit, hit_count);
    return hipGetLastError();
}

hipError_t launch_sieve(const KParams& p, uint32_t variant, hipStream_t stream) {
    if (p.row_count == 0 || p.n_ids == 0) return hipSuccess;
    // the complex-op variants' LOADVAR addresses a limb plane with a 32-bit byte stride (the
    // C-ABI refuses such runs first, with MH_E_UNSUPPORTED and a message)
    if (!variant_fits(variant, p.capacity)) return hipErrorInvalidValue;
    constexpr int kCplx = F_CPLX, kKec = F_CPLX | F_KECCAK, kAll = F_CPLX | F_KECCAK | F_EVM;
    switch (variant) {
        case 0: return launch_variant<MH_NR_SMALL, 0>(p, stream);
        case 1: return launch_variant<MH_NR_SMALL, kCplx>(p, stream);
        case 2: return launch_variant<MH_NR_SMALL, kKec>(p, stream);
        case 3: return launch_variant<MH_NR_SMALL, kAll>(p, stream);
        case 4: return launch_variant<MH_NR_MID, 0>(p, stream);
        case 5: return launch_variant<MH_NR_MID, kCplx>(p, stream);
        case 6: return launch_variant<MH_NR_MID, kKec>(p, stream);
        case 7: return launch_variant<MH_NR_MID, kAll>(p, stream);
        case 8: return launch_variant<MH_NR_MAX, 0>(p, stream);
        case 9: return launch_variant<MH_NR_MAX, kCplx>(p, stream);
        case 10: return launch_variant<MH_NR_MAX, kKec>(p, stream);
        default: return launch_variant<MH_NR_MAX, kAll>(p, stream);
    }
}

hipError_t launch_generate(uint32_t* assign, uint64_t stride, uint64_t rows, uint32_t n_vars,
                           uint64_t seed, uint64_t base, hipStream_t stream) {
    const u64 blocks = (rows + kBlock - 1) / kBlock;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(generate_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, assign,
                       stride, rows, n_vars, seed, base);
    return hipGetLastError();
}

hipError_t launch_microbench(uint32_t kind, uint32_t iters, uint32_t blocks, uint32_t* sink,
                             hipStream_t stream) {
    switch (kind) {
#define MB_CASE(k) \
    case k: hipLaunchKernelGGL(microbench_kernel<k>, dim3(blocks), dim3(kBlock), 0, stream, iters, sink); break;
        MB_CASE(0) MB_CASE(1) MB_CASE(2) MB_CASE(3) MB_CASE(4) MB_CASE(5) MB_CASE(6) MB_CASE(7)
        MB_CASE(8) MB_CASE(9) MB_CASE(10) MB_CASE(11) MB_CASE(12) MB_CASE(13) MB_CASE(14)
        MB_CASE(15) MB_CASE(16) MB_CASE(17) MB_CASE(18) MB_CASE(19) MB_CASE(20)
        MB_CASE(21) MB_CASE(22) MB_CASE(23) MB_CASE(24) MB_CASE(25) MB_CASE(26) MB_CASE(27)
        MB_CASE(28) MB_CASE(29) MB_CASE(30) MB_CASE(31) MB_CASE(32) MB_CASE(33) MB_CASE(34)
        MB_CASE(35) MB_CASE(36) MB_CASE(37) MB_CASE(38) MB_CASE(39) MB_CASE(40) MB_CASE(41)
        MB_CASE(42) MB_CASE(43) MB_CASE(44)
#undef MB_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace mh
