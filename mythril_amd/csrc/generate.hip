// Guided candidate generator (mh_assign_generate_guided): one thread per assignment row, SoA
// writes (column v limb k of row r at word (v*8 + k)*stride + r), so a wave's 64 lanes store
// 256 contiguous bytes per limb.  The semantics are stated in include/mythril_hip.h and restated
// bit for bit in oracle/guided_gen.py; the harvest that fills the guide is
// mythril_amd/candidates.py.  Off the hot path: written once per query, before the sieve reads it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels.h"

namespace {

using u32 = uint32_t;
using u64 = uint64_t;

constexpr int kBlock = 256;
constexpr u64 kSaltMode = 0x6A09E667F3BCC909ull;
constexpr u64 kSaltSet = 0xBB67AE8584CAA73Bull;
constexpr u32 kCopy = 0x80000000u;

__device__ __forceinline__ u64 splitmix64(u64 x) {
    x += 0x9E3779B97F4A7C15ull;
    u64 z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// mh_gen_limb on the device
__device__ __forceinline__ u32 gen_limb(u64 seed, u32 var, u64 index, u32 limb) {
    const u64 key = splitmix64(seed ^ (((u64)var * 8 + limb) * 0xD1B54A32D192ED03ull));
    return (u32)splitmix64(key ^ index);
}

__device__ __forceinline__ u32 limb_mask(u32 width, u32 k) {
    const u32 lo = 32 * k;
    if (width >= lo + 32) return 0xFFFFFFFFu;
    if (width <= lo) return 0u;
    return (1u << (width - lo)) - 1u;
}

// bits [lo, lo + n) of an 8-limb value, as a (right-aligned) 8-limb value
__device__ void extract_bits(const u32* v, u32 lo, u32 n, u32* out) {
    const u32 q = lo >> 5, r = lo & 31;
#pragma unroll
    for (u32 k = 0; k < 8; ++k) {
        const u32 a = (q + k < 8) ? v[q + k] : 0u;
        const u32 b = (q + k + 1 < 8) ? v[q + k + 1] : 0u;
        out[k] = r ? ((a >> r) | (b << (32 - r))) : a;
    }
#pragma unroll
    for (u32 k = 0; k < 8; ++k) out[k] &= limb_mask(n, k);
}

// the column's generated value before any set applies: a small value, uniform limbs, or a draw
// from the column's pool
__device__ __forceinline__ void base_value(const mh::KGuide& g, u32 v, u64 seed, u64 gidx, u32* val) {
    const u32 m0 = gen_limb(seed ^ kSaltMode, v, gidx, 0);
    const u32 mode = m0 & 0xFFu;
    const u32 plo = g.pool_off[v], phi = g.pool_off[v + 1];
    if (mode < 64) {
        val[0] = (m0 >> 8) & 0xFFu;
#pragma unroll
        for (u32 k = 1; k < 8; ++k) val[k] = 0;
    } else if (mode < 128 || phi == plo) {
#pragma unroll
        for (u32 k = 0; k < 8; ++k) val[k] = gen_limb(seed, v, gidx, k);
    } else {
        const u32 m1 = gen_limb(seed ^ kSaltMode, v, gidx, 1);
        const u32* src = g.pool + (u64)(plo + m1 % (phi - plo)) * 8;
#pragma unroll
        for (u32 k = 0; k < 8; ++k) val[k] = src[k];
    }
}

// the alternative set j applies to this row, or ~0u (a per-row draw against the set's probability)
__device__ __forceinline__ u32 chosen_alt(const mh::KGuide& g, u32 j, u64 seed, u64 gidx) {
    const u32 s = gen_limb(seed ^ kSaltSet, j, gidx, 0);
    const u32 a0 = g.set_off[j], n_alt = g.set_off[j + 1] - a0;
    if ((s & 0xFFu) >= g.set_prob[j] || n_alt == 0) return ~0u;
    return a0 + (s >> 8) % n_alt;
}

// one entry applied to the row in memory: a value, or bits copied from another column
__device__ void apply_entry(u32* assign, u64 stride, u64 row, const mh::KGuide& g, u32 e) {
    const u32 c = g.entry_col[e];
    const u32* ev = g.entry_val + (u64)e * 8;
    if (c & kCopy) {
        const u32 dst = c & ~kCopy, src = ev[0], dlo = ev[1], slo = ev[2], nb = ev[3];
        u32 sv[8], bits[8], dv[8], m[8], one[8];
#pragma unroll
        for (u32 k = 0; k < 8; ++k) {
            sv[k] = assign[((u64)src * 8 + k) * stride + row];
            dv[k] = assign[((u64)dst * 8 + k) * stride + row];
        }
        extract_bits(sv, slo, nb, bits);
        // shift bits and an nb-wide mask left by dlo
#pragma unroll
        for (u32 k = 0; k < 8; ++k) one[k] = limb_mask(nb, k);
        const u32 q = dlo >> 5, r = dlo & 31;
#pragma unroll
        for (int k = 7; k >= 0; --k) {
            const int s0 = k - (int)q, s1 = k - (int)q - 1;
            const u32 ba = s0 >= 0 ? bits[s0] : 0u, bb = s1 >= 0 ? bits[s1] : 0u;
            const u32 ma = s0 >= 0 ? one[s0] : 0u, mb = s1 >= 0 ? one[s1] : 0u;
            sv[k] = r ? ((ba << r) | (bb >> (32 - r))) : ba;
            m[k] = r ? ((ma << r) | (mb >> (32 - r))) : ma;
        }
        const u32 w = g.width[dst];
#pragma unroll
        for (u32 k = 0; k < 8; ++k)
            assign[((u64)dst * 8 + k) * stride + row] =
                ((dv[k] & ~m[k]) | (sv[k] & m[k])) & limb_mask(w, k);
    } else {
        const u32 w = g.width[c];
#pragma unroll
        for (u32 k = 0; k < 8; ++k)
            assign[((u64)c * 8 + k) * stride + row] = ev[k] & limb_mask(w, k);
    }
}

// Every column's base value written, then every set applied in order, in memory.
__global__ void __launch_bounds__(kBlock)
    guided_kernel(u32* assign, u64 stride, u64 first, u64 count, u64 seed, u64 base,
                  mh::KGuide g) {
    const u64 i = (u64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= count) return;
    const u64 row = first + i;
    const u64 gidx = base + row;
    for (u32 v = 0; v < g.n_cols; ++v) {
        u32 val[8];
        base_value(g, v, seed, gidx, val);
        const u32 w = g.width[v];
#pragma unroll
        for (u32 k = 0; k < 8; ++k)
            assign[((u64)v * 8 + k) * stride + row] = val[k] & limb_mask(w, k);
    }
    for (u32 j = 0; j < g.n_sets; ++j) {
        const u32 alt = chosen_alt(g, j, seed, gidx);
        if (alt == ~0u) continue;
        for (u32 e = g.alt_off[alt]; e < g.alt_off[alt + 1]; ++e) apply_entry(assign, stride, row, g, e);
    }
}

// The same rows, spread over kWaves waves per 64 rows, with the leading value-only sets
// resolved in LDS: a value entry only decides which value a column ends with -- the last one
// applied, i.e. the largest entry index, since entries are laid out in set order -- so the waves
// split the sets, each lane drawing its row's alternative of a set and keeping the largest
// entry per column with an LDS atomic max ([column][row] slots); then the waves split the
// columns and write each column of each row once (the base value, or the winning entry's).  The
// sets from the first one with a copy entry on run in memory, in order, on wave 0.  The one-lane-
// per-row form stored 8 limbs per applied entry, lane-divergently, and left a 256-row launch
// four waves: 0.20 ms per launch on average, up to 0.58 (profiles/r03h).
// STAGED (round 5): the guide's set / alternative / entry-column arrays are copied into LDS
// first, so a set's chain of dependent reads (its probability and alternatives, the chosen
// alternative's entries, each entry's column) costs LDS latency instead of a global load's
// (ET-400's 256-row launch: 304 sets, 16 waves each walking 19 of them, 70 us of mostly load
// latency, profiles/r05f/pprof).
constexpr u32 kLdsRows = 64;
constexpr u32 kWaves = 16;  // a 256-row launch: 4 workgroups of 16 waves, 4 waves per SIMD
constexpr size_t kGenLds = 64 * 1024;  // LDS of one generator workgroup at most

template <bool STAGED>
__global__ void __launch_bounds__(kLdsRows * kWaves)
    guided_lds_kernel(u32* assign, u64 stride, u64 first, u64 count, u64 seed, u64 base,
                      mh::KGuide g) {
    extern __shared__ u32 s_last[];  // [n_cols][kLdsRows]: 1 + the winning entry, 0 = none
    const u32 lane = threadIdx.x % kLdsRows, wave = threadIdx.x / kLdsRows;
    for (u32 k = threadIdx.x; k < g.n_cols * kLdsRows; k += kLdsRows * kWaves) s_last[k] = 0;
    if constexpr (STAGED) {  // the span after the last-entry slots; the pointers rebased on it
        u32* s_span = s_last + g.n_cols * kLdsRows;
        for (u32 k = threadIdx.x; k < g.span_words; k += kLdsRows * kWaves) s_span[k] = g.set_prob[k];
        g.set_off = s_span + (g.set_off - g.set_prob);
        g.alt_off = s_span + (g.alt_off - g.set_prob);
        g.entry_col = s_span + (g.entry_col - g.set_prob);
        g.set_prob = s_span;
    }
    __syncthreads();
    const u64 i = (u64)blockIdx.x * kLdsRows + lane;
    const bool live = i < count;
    const u64 row = first + (live ? i : 0);
    const u64 gidx = base + row;
    if (live) {
        for (u32 j = wave; j < g.n_value_sets; j += kWaves) {
            const u32 alt = chosen_alt(g, j, seed, gidx);
            if (alt == ~0u) continue;
            for (u32 e = g.alt_off[alt]; e < g.alt_off[alt + 1]; ++e)
                atomicMax(&s_last[g.entry_col[e] * kLdsRows + lane], e + 1);
        }
    }
    __syncthreads();
    if (live) {
        for (u32 v = wave; v < g.n_cols; v += kWaves) {
            const u32 e = s_last[v * kLdsRows + lane];
            u32 val[8];
            if (e == 0) {
                base_value(g, v, seed, gidx, val);
            } else {
#pragma unroll
                for (u32 k = 0; k < 8; ++k) val[k] = g.entry_val[(u64)(e - 1) * 8 + k];
            }
            const u32 w = g.width[v];
#pragma unroll
            for (u32 k = 0; k < 8; ++k)
                assign[((u64)v * 8 + k) * stride + row] = val[k] & limb_mask(w, k);
        }
    }
    if (g.n_value_sets == g.n_sets) return;
    __syncthreads();  // every column written (and visible to the workgroup) before the copies
    if (!live || wave != 0) return;
    for (u32 j = g.n_value_sets; j < g.n_sets; ++j) {
        const u32 alt = chosen_alt(g, j, seed, gidx);
        if (alt == ~0u) continue;
        for (u32 e = g.alt_off[alt]; e < g.alt_off[alt + 1]; ++e) apply_entry(assign, stride, row, g, e);
    }
}

__global__ void __launch_bounds__(kBlock)
    results_reset_kernel(u64* first_hit, u64* hit_count, u32 n) {
    const u32 i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (first_hit) first_hit[i] = ~0ull;
    if (hit_count) hit_count[i] = 0;
}

// one workgroup per tape: the words of its witness row (a row outside the buffer reads as none)
__global__ void __launch_bounds__(kBlock)
    witness_rows_kernel(const u32* assign, u64 stride, const u64* first_hit, u64 index_base,
                        u32 n_cols, u32* out) {
    const u64 h = first_hit[blockIdx.x];
    const u64 row = h - index_base;
    const bool hit = h != ~0ull && h >= index_base && row < stride;
    const u32 words = n_cols * 8;
    u32* o = out + (u64)blockIdx.x * words;
    for (u32 w = threadIdx.x; w < words; w += kBlock) o[w] = hit ? assign[(u64)w * stride + row] : 0u;
}

}  // namespace

namespace mh {

hipError_t launch_results_reset(uint64_t* first_hit, uint64_t* hit_count, uint32_t n,
                                hipStream_t stream) {
    if (n == 0 || (!first_hit && !hit_count)) return hipSuccess;
    hipLaunchKernelGGL(results_reset_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, stream,
                       first_hit, hit_count, n);
    return hipGetLastError();
}

hipError_t launch_witness_rows(const uint32_t* assign, uint64_t stride, const uint64_t* first_hit,
                               uint32_t n_tapes, uint64_t index_base, uint32_t n_cols,
                               uint32_t* out, hipStream_t stream) {
    if (n_tapes == 0 || n_cols == 0) return hipSuccess;
    hipLaunchKernelGGL(witness_rows_kernel, dim3(n_tapes), dim3(kBlock), 0, stream, assign, stride,
                       first_hit, index_base, n_cols, out);
    return hipGetLastError();
}

hipError_t launch_generate_guided(uint32_t* assign, uint64_t stride, uint64_t first,
                                  uint64_t count, uint64_t seed, uint64_t base, const KGuide& g,
                                  hipStream_t stream) {
    if (count == 0) return hipSuccess;
    // LDS form while the last-entry slots (256 B per column) fit 48 KB per workgroup
    const size_t lds = (size_t)g.n_cols * kLdsRows * sizeof(u32);
    const size_t staged = lds + (size_t)g.span_words * sizeof(u32);
    const u64 blocks = (count + kLdsRows - 1) / kLdsRows;
    if (g.n_cols && staged <= kGenLds) {
        hipLaunchKernelGGL(guided_lds_kernel<true>, dim3((unsigned)blocks), dim3(kLdsRows * kWaves),
                           staged, stream, assign, stride, first, count, seed, base, g);
    } else if (g.n_cols && lds <= 48 * 1024) {
        hipLaunchKernelGGL(guided_lds_kernel<false>, dim3((unsigned)blocks), dim3(kLdsRows * kWaves),
                           lds, stream, assign, stride, first, count, seed, base, g);
    } else {
        const u64 blocks = (count + kBlock - 1) / kBlock;
        hipLaunchKernelGGL(guided_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, assign,
                           stride, first, count, seed, base, g);
    }
    return hipGetLastError();
}

}  // namespace mh
