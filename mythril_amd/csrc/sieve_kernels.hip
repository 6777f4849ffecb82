// Sieve kernels for gfx950: the tape interpreter, the assignment generator and a VALU
// micro-benchmark.
//
// Mapping: one lane = one candidate assignment (row); a 256-thread workgroup = 256 consecutive
// rows; every wave walks the whole tape batch, so the tape stream (instruction words, constants)
// is wave-uniform and comes through the scalar unit (s_load), while the per-lane 256-bit values
// live in VGPRs.  The register file is 8 "limb planes", each an ext_vector of MH_NUM_REGS u32,
// indexed by the wave-uniform register number (s_set_gpr_idx_on / v_mov), so no per-lane
// scratch is touched.  Assignment columns 0..3 are loaded once per launch into R0..R3 and stay
// resident for every tape: HBM traffic is 32 B x columns per row per launch, independent of the
// number of tapes.  Results are reduced per workgroup in LDS (64-tape chunks) and flushed with
// one atomic per tape per workgroup.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dev_isa.h"
#include "kernels.h"
#include "u256_ops.h"

using namespace mh;

namespace {

constexpr int kBlock = 256;
constexpr int kChunk = 64;  // tapes per LDS result chunk

template <int NR>
struct RegFile {
    typedef u32 plane_t __attribute__((ext_vector_type(NR)));
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
    __device__ __forceinline__ void write0(u32 r, u32 v) { p0[r] = v; }
};

__device__ __forceinline__ u64 splitmix64(u64 x) {
    x += 0x9E3779B97F4A7C15ull;
    u64 z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Keccak-256 of up to three byte-aligned pieces (big-endian byte order within each piece).
__device__ __forceinline__ void keccak_pieces(const u32* P0, const u32* P1, const u32* P2,
                                              u32 n0, u32 n1, u32 n2, u32* z) {
    typedef u32 v32_t __attribute__((ext_vector_type(32)));
    v32_t pv;
#pragma unroll
    for (int k = 0; k < 8; ++k) { pv[k] = P0[k]; pv[8 + k] = P1[k]; pv[16 + k] = P2[k]; }
    const u32 len = n0 + n1 + n2;
    u64 st[25];
#pragma unroll
    for (int i = 0; i < 25; ++i) st[i] = 0;
#pragma unroll
    for (int wd = 0; wd < 34; ++wd) {
        u32 word = 0;
#pragma unroll
        for (int bi = 0; bi < 4; ++bi) {
            const u32 m = 4u * wd + bi;
            u32 byte = 0;
            if (m < len) {  // wave-uniform
                const u32 p = m < n0 ? 0u : (m < n0 + n1 ? 1u : 2u);
                const u32 off = p == 0 ? 0u : (p == 1 ? n0 : n0 + n1);
                const u32 np = p == 0 ? n0 : (p == 1 ? n1 : n2);
                const u32 e = np - 1u - (m - off);  // little-endian byte index in the piece
                const u32 limb = pv[p * 8u + (e >> 2)];
                byte = (limb >> (8u * (e & 3u))) & 0xFFu;
            }
            if (m == len) byte |= 0x01u;
            if (m == 135u) byte |= 0x80u;
            word |= byte << (8 * bi);
        }
        st[wd >> 1] |= (u64)word << (32 * (wd & 1));
    }
    keccak_f1600(st);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int i = 7 - k;  // u32 word i of the output bytes
        const u32 wv = (i & 1) ? (u32)(st[i >> 1] >> 32) : (u32)st[i >> 1];
        z[k] = bswap32(wv);
    }
}

typedef const __attribute__((address_space(4))) u32* cu32_ptr;  // scalar-cache path

struct TapeHead {
    u32 insn_off, n_insns, root_reg, root_bool;
};

__device__ __forceinline__ TapeHead tape_head(const KParams& p, u32 t) {
    const cu32_ptr tp = (cu32_ptr)p.tapes + 4ull * t;
    return TapeHead{tp[0], tp[1], tp[2], tp[3]};
}

// Instruction stream: lane j of the wave holds instruction (64*chunk + j) of the current tape
// in two VGPRs (one coalesced 512-B load per 64 instructions, prefetched one tape ahead); the
// interpreter extracts instruction i with v_readlane into SGPRs, so fetching costs no memory
// round trip per instruction.
struct InsnCache {
    u32 w0, w1;
};

__device__ __forceinline__ InsnCache load_insns(const KParams& p, u32 insn_off, u32 n, u32 first) {
    const u32 lane = threadIdx.x & 63u;
    const u32 j = first + lane;
    InsnCache c{0u, 0u};
    if (j < n) {
        const uint2 v = p.insns[insn_off + j];
        c.w0 = v.x;
        c.w1 = v.y;
    }
    return c;
}

__device__ __forceinline__ void load_const(const KParams& p, u32 idx, u32* z) {
    const cu32_ptr cp = (cu32_ptr)p.consts + 8ull * idx;
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = cp[k];
}

// One instruction = operand reads (register file or scalar constant), one compute, one write of
// R[d]: a single definition of the register-file vectors per step keeps the compiler from
// materialising copies of the whole file on every control-flow merge.
template <int NR, int FEAT>
__device__ __forceinline__ void exec_tape(RegFile<NR>& R, const KParams& p, InsnCache ic,
                                          u32 insn_off, u32 n, u64 lrow) {
    for (u32 i = 0; i < n; ++i) {
        if ((i & 63u) == 0 && i) ic = load_insns(p, insn_off, n, i);  // tapes > 64 insns
        const u32 w0 = __builtin_amdgcn_readlane(ic.w0, i & 63u);
        const u32 w1 = __builtin_amdgcn_readlane(ic.w1, i & 63u);
        const u32 op = w0 & 0xFFu, d = (w0 >> 8) & 0xFFu, a = (w0 >> 16) & 0xFFu, b = w0 >> 24;
        const u32 w = (w1 >> 2) & 0x1FFu, aux = w1 >> 11;
        u32 x[8], y[8], z[8];
        // unconditional register reads (no control-flow merge of operand values); a constant
        // operand b overwrites y from the scalar constant pool
        R.read(a, x);
        R.read(b, y);
        if (((MH_CONST_OPERAND_OK >> op) & 1u) && (w1 & F_BCONST)) load_const(p, aux, y);
        switch (op) {
            // ---- bv x bv -> bv
            case D_ADD: add256(x, y, z); mask_w(z, w); break;
            case D_SUB: sub256(x, y, z); mask_w(z, w); break;
            case D_MUL: mul_lo256(x, y, z); mask_w(z, w); break;
            case D_AND:
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = x[k] & y[k];
                break;
            case D_OR:
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = x[k] | y[k];
                break;
            case D_XOR:
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = x[k] ^ y[k];
                break;
            case D_SHL: bvshl_v(x, shift_amount(y), z, w); break;
            case D_LSHR: bvlshr_v(x, shift_amount(y), z, w); break;
            case D_ASHR: bvashr_v(x, shift_amount(y), z, w); break;
            case D_CONCAT: {
                u32 t[8];
                shl256(x, aux, t);
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = t[k] | y[k];
                break;
            }
            case D_UDIV: case D_UREM: case D_SDIV: case D_SREM: case D_SMOD:
                if constexpr ((FEAT & F_DIV) != 0) divmod_family(op - D_UDIV, x, y, z, w);
                break;
            case D_EXP:
                if constexpr ((FEAT & F_EVM) != 0) evm_exp(x, y, z, w);
                break;
            case D_SIGNEXT:
                if constexpr ((FEAT & F_EVM) != 0) evm_signextend(x, y, z);
                break;
            case D_BYTE:
                if constexpr ((FEAT & F_EVM) != 0) evm_byte(x, y, z);
                break;
            // ---- bv -> bv
            case D_NEG: neg256(x, z); mask_w(z, w); break;
            case D_NOT:
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = ~x[k];
                mask_w(z, w);
                break;
            case D_SHLI:
                if (aux < w) {
                    shl256(x, aux, z);
                    mask_w(z, w);
                } else {
#pragma unroll
                    for (int k = 0; k < 8; ++k) z[k] = 0;
                }
                break;
            case D_LSHRI:
                if (aux < w) {
                    shr256(x, aux, z, 0u);
                } else {
#pragma unroll
                    for (int k = 0; k < 8; ++k) z[k] = 0;
                }
                break;
            case D_ASHRI: bvashr_v(x, aux, z, w); break;
            case D_EXTRACT: shr256(x, aux, z, 0u); mask_w(z, w); break;
            case D_SEXT: sext_to256(x, aux, z); mask_w(z, w); break;
            case D_MOV:
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = x[k];
                break;
            // ---- bv x bv -> Bool (0/1 in limb 0)
            case D_EQ: z[0] = eq256(x, y); break;
            case D_ULT: z[0] = ult256(x, y); break;
            case D_ULE: z[0] = !ult256(y, x); break;
            case D_SLT: z[0] = slt_w(x, y, w); break;
            case D_SLE: z[0] = !slt_w(y, x, w); break;
            case D_UADD_NOOVFL: {
                u32 t[8];
                const u32 cy = add256(x, y, t);
                u32 hi = 0;
                if (w < 256) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) hi |= t[k] & ~width_mask(k, w);
                }
                z[0] = !(cy || hi);
                break;
            }
            case D_UMUL_NOOVFL: {
                u32 t[16];
                mul_full256(x, y, t);
                u32 hi = 0;
#pragma unroll
                for (int k = 8; k < 16; ++k) hi |= t[k];
                if (w < 256) {
#pragma unroll
                    for (int k = 0; k < 8; ++k) hi |= t[k] & ~width_mask(k, w);
                }
                z[0] = hi == 0;
                break;
            }
            // ---- Bool (limb 0)
            case D_BAND: z[0] = x[0] & y[0] & 1u; break;
            case D_BOR: z[0] = (x[0] | y[0]) & 1u; break;
            case D_BXOR: z[0] = (x[0] ^ y[0]) & 1u; break;
            case D_BEQ: z[0] = ((x[0] ^ y[0]) & 1u) ^ 1u; break;
            case D_BNOT: z[0] = (x[0] & 1u) ^ 1u; break;
            case D_TRUE: z[0] = 1u; break;
            case D_FALSE: z[0] = 0u; break;
            // ---- others
            case D_ITE: {  // x[0] = cond, y = then, R[aux] = else
                u32 e[8];
                R.read(aux, e);
                const bool cnd = (x[0] & 1u) != 0;
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = cnd ? y[k] : e[k];
                break;
            }
            case D_BITE: {
                const bool cnd = (x[0] & 1u) != 0;
                z[0] = cnd ? (y[0] & 1u) : (R.read0(aux) & 1u);
                break;
            }
            case D_LOADC: load_const(p, aux, z); break;
            case D_LOADVAR:
#pragma unroll
                for (int k = 0; k < 8; ++k) z[k] = p.assign[((u64)aux * 8 + k) * p.capacity + lrow];
                break;
            case D_KECCAK:
                if constexpr ((FEAT & F_KECCAK) != 0) {
                    const u32 np = (w1 >> 26) & 3u;
                    const u32 n0 = (w1 >> 8) & 63u, n1 = (w1 >> 14) & 63u, n2 = (w1 >> 20) & 63u;
                    u32 P2[8];
                    R.read(w1 & 0xFFu, P2);
                    keccak_pieces(x, y, P2, n0, np > 1 ? n1 : 0u, np > 2 ? n2 : 0u, z);
                }
                break;
            default:
                break;
        }
        R.write(d, z);
    }
}

template <int NR>
__device__ __forceinline__ void preload(RegFile<NR>& R, const KParams& p, u64 lrow) {
#pragma unroll
    for (u32 v = 0; v < MH_MAX_PRELOAD; ++v) {
        if (v < p.n_pre) {
            u32 x[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = p.assign[((u64)v * 8 + k) * p.capacity + lrow];
            R.write(v, x);
        }
    }
}

template <int NR, int FEAT>
__global__ void __launch_bounds__(kBlock) sieve_kernel(const KParams p) {
    __shared__ unsigned long long s_min[kChunk];
    __shared__ unsigned long long s_cnt[kChunk];
    RegFile<NR> R;
    const u32 tid = threadIdx.x;
    const u64 row = p.row_first + (u64)blockIdx.x * kBlock + tid;
    const u64 row_end = p.row_first + p.row_count;
    const bool valid = row < row_end;
    const u64 lrow = valid ? row : p.row_first;
    preload<NR>(R, p, lrow);
    const u64 block_first = p.index_base + p.row_first + (u64)blockIdx.x * kBlock;
    const u64 wave_first = block_first + (tid & ~63u);
    const u32 t_end = p.tape_first + p.tape_count;
    for (u32 cb = p.tape_first; cb < t_end; cb += kChunk) {
        const u32 nt = (t_end - cb) < (u32)kChunk ? (t_end - cb) : (u32)kChunk;
        __syncthreads();
        if (tid < (u32)kChunk) {
            s_min[tid] = (p.mode == MH_MODE_FIRST_HIT && tid < nt && p.first_hit)
                             ? p.first_hit[cb - p.tape_first + tid] : ~0ull;
            s_cnt[tid] = 0;
        }
        __syncthreads();
        TapeHead th = tape_head(p, cb);
        InsnCache ic = load_insns(p, th.insn_off, th.n_insns, 0);
        for (u32 j = 0; j < nt; ++j) {
            const u32 t = cb + j;
            // prefetch the next tape's header and first 64 instructions
            const TapeHead th_next = tape_head(p, j + 1 < nt ? t + 1 : t);
            const InsnCache ic_next = load_insns(p, th_next.insn_off, th_next.n_insns, 0);
            if (p.mode == MH_MODE_FIRST_HIT) {
                // early exit: a smaller witness is already known for this tape
                const u64 km = s_min[j];
                const u64 known = ((u64)__builtin_amdgcn_readfirstlane((u32)(km >> 32)) << 32) |
                                  __builtin_amdgcn_readfirstlane((u32)km);
                if (known < wave_first) {
                    th = th_next;
                    ic = ic_next;
                    continue;
                }
            }
            exec_tape<NR, FEAT>(R, p, ic, th.insn_off, th.n_insns, lrow);
            u32 res;
            if (th.root_bool) {
                res = R.read0(th.root_reg) & 1u;
            } else {
                u32 x[8];
                R.read(th.root_reg, x);
                res = is_zero256(x) ? 0u : 1u;
            }
            const unsigned long long mask = __builtin_amdgcn_ballot_w64(valid && res);
            if (mask && (tid & 63u) == 0) {
                atomicAdd(&s_cnt[j], (unsigned long long)__builtin_popcountll(mask));
                atomicMin(&s_min[j], (unsigned long long)(wave_first + __builtin_ctzll(mask)));
            }
            th = th_next;
            ic = ic_next;
        }
        __syncthreads();
        if (tid < nt) {
            const u32 ti = cb - p.tape_first + tid;
            if (s_cnt[tid] && p.hit_count) atomicAdd(&p.hit_count[ti], s_cnt[tid]);
            if (s_min[tid] != ~0ull && p.first_hit) atomicMin(&p.first_hit[ti], s_min[tid]);
        }
    }
}

// Root value of one tape per row (parity path).
template <int NR>
__global__ void __launch_bounds__(kBlock) values_kernel(const KParams p, u32 tape, u32* out) {
    RegFile<NR> R;
    const u64 r = (u64)blockIdx.x * kBlock + threadIdx.x;
    const bool valid = r < p.row_count;
    const u64 lrow = p.row_first + (valid ? r : 0);
    preload<NR>(R, p, lrow);
    const TapeHead th = tape_head(p, tape);
    exec_tape<NR, F_DIV | F_KECCAK | F_EVM>(R, p, load_insns(p, th.insn_off, th.n_insns, 0),
                                            th.insn_off, th.n_insns, lrow);
    u32 x[8];
    R.read(th.root_reg, x);
    if (th.root_bool) {
        x[0] &= 1u;
#pragma unroll
        for (int k = 1; k < 8; ++k) x[k] = 0;
    }
    if (valid) {
#pragma unroll
        for (int k = 0; k < 8; ++k) out[(u64)k * p.row_count + r] = x[k];
    }
}

__global__ void __launch_bounds__(kBlock) generate_kernel(u32* assign, u64 capacity, u32 n_vars,
                                                          u64 seed, u64 base) {
    const u64 row = (u64)blockIdx.x * kBlock + threadIdx.x;
    if (row >= capacity) return;
    for (u32 v = 0; v < n_vars; ++v) {
#pragma unroll
        for (u32 k = 0; k < 8; ++k) {
            const u64 key = splitmix64(seed ^ (((u64)v * 8 + k) * 0xD1B54A32D192ED03ull));
            assign[((u64)v * 8 + k) * capacity + row] = (u32)splitmix64(key ^ (base + row));
        }
    }
}

// Integer VALU throughput probe: independent dependency chains per lane (enough ILP that the
// measured rate is issue-bound, not latency-bound).
__global__ void __launch_bounds__(kBlock) microbench_kernel(u32 kind, u32 iters, u32* sink) {
    u32 s[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 8; ++k) s[j][k] = threadIdx.x * 2654435761u + 8 * j + k;
    const u32 y = blockIdx.x | 1u;
    if (kind == 0) {  // 4 independent 256-bit add-with-carry chains: 32 ops / iteration
        for (u32 i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                u64 c = y;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    c = (u64)s[j][k] + s[(j + 1) & 3][k] + (c >> 32);
                    s[j][k] = (u32)c;
                }
            }
        }
    } else if (kind == 1) {  // v_mad_u64_u32: 8 independent chains, 8 mads / iteration
        u64 acc[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = s[0][k];
        for (u32 i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k) acc[k] = (u64)(u32)acc[k] * (y + k) + (acc[k] >> 32);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s[0][k] = (u32)acc[k] ^ (u32)(acc[k] >> 32);
    } else {  // xor/add mix: 32 independent ops / iteration
        for (u32 i = 0; i < iters; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int k = 0; k < 8; ++k) s[j][k] = (s[j][k] ^ y) + k;
        }
    }
    u32 r = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int k = 0; k < 8; ++k) r ^= s[j][k];
    if (r == 0x12345678u) sink[0] = r;
}

}  // namespace

namespace mh {

hipError_t launch_sieve(const KParams& p, uint32_t feat, hipStream_t stream) {
    const u64 blocks = (p.row_count + kBlock - 1) / kBlock;
    if (blocks == 0 || p.tape_count == 0) return hipSuccess;
    dim3 grid((unsigned)blocks), block(kBlock);
    if (feat & (F_KECCAK | F_EVM))
        hipLaunchKernelGGL((sieve_kernel<MH_NUM_REGS, F_DIV | F_KECCAK | F_EVM>), grid, block, 0,
                           stream, p);
    else if (feat & F_DIV)
        hipLaunchKernelGGL((sieve_kernel<MH_NUM_REGS, F_DIV>), grid, block, 0, stream, p);
    else
        hipLaunchKernelGGL((sieve_kernel<MH_NUM_REGS, 0>), grid, block, 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_values(const KParams& p, uint32_t tape, uint32_t* out, hipStream_t stream) {
    const u64 blocks = (p.row_count + kBlock - 1) / kBlock;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL((values_kernel<MH_NUM_REGS>), dim3((unsigned)blocks), dim3(kBlock), 0,
                       stream, p, tape, out);
    return hipGetLastError();
}

hipError_t launch_generate(uint32_t* assign, uint64_t capacity, uint32_t n_vars, uint64_t seed,
                           uint64_t base, hipStream_t stream) {
    const u64 blocks = (capacity + kBlock - 1) / kBlock;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(generate_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, stream, assign,
                       capacity, n_vars, seed, base);
    return hipGetLastError();
}

hipError_t launch_microbench(uint32_t kind, uint32_t iters, uint32_t blocks, uint32_t* sink,
                             hipStream_t stream) {
    hipLaunchKernelGGL(microbench_kernel, dim3(blocks), dim3(kBlock), 0, stream, kind, iters,
                       sink);
    return hipGetLastError();
}

}  // namespace mh
