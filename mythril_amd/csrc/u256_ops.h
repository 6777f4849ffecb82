// 256-bit word arithmetic on 8 x u32 limbs (limb 0 least significant), one word per lane.
//
// Written for gfx950 VALU: add/sub as v_add_co/v_addc (v_sub_co/v_subb) carry chains, products
// as v_mad_u64_u32 schoolbook columns, funnel shifts as v_alignbit_b32, selects as v_cndmask.
// Every routine is branch-free per lane except where a wave-uniform skip is marked (MH_ANY):
// lanes of a wave evaluate the same tape on different assignments, so data-dependent control
// flow would serialise the wave.
//
// The functions are __host__ __device__ so tests/native/emu.cpp can run the same code on the
// host CPU: the test emulator, and the tape compiler's constant folding (compile.cpp), which
// evaluates constant-only instructions with the device's own semantics.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MH_FN __host__ __device__ __forceinline__
#else
#define MH_FN static inline
#endif

namespace mh {

typedef uint32_t u32;
typedef uint64_t u64;

// ---- target primitives -------------------------------------------------------------------------
MH_FN u32 alignbit(u32 hi, u32 lo, u32 s) {  // ((hi:lo) >> (s & 31)) & 0xffffffff
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, s);
#else
    return (u32)((((u64)hi << 32) | lo) >> (s & 31));
#endif
}

MH_FN u32 clz32(u32 x) {  // 32 for x == 0
#if defined(__HIP_DEVICE_COMPILE__)
    return x ? (u32)__builtin_clz(x) : 32u;
#else
    return x ? (u32)__builtin_clz(x) : 32u;
#endif
}

MH_FN u32 bswap32(u32 x) { return __builtin_bswap32(x); }

// True if the predicate holds for any lane of the wave (wave-uniform result).  Used only to
// skip work no lane needs; every caller is correct if it returns true unconditionally.
MH_FN bool any_lane(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ballot_w64(p) != 0;
#else
    return p;
#endif
}

// add / subtract with carry: v_add_co_u32 / v_addc_co_u32 (v_sub_co / v_subb_co) on gfx950
MH_FN u32 addc32(u32 x, u32 y, u32 cin, u32* cout) {
#if defined(__clang__)
    return __builtin_addc(x, y, cin, cout);
#else
    const u64 t = (u64)x + y + cin;
    *cout = (u32)(t >> 32);
    return (u32)t;
#endif
}

MH_FN u32 subc32(u32 x, u32 y, u32 bin, u32* bout) {
#if defined(__clang__)
    return __builtin_subc(x, y, bin, bout);
#else
    const u64 t = (u64)x - y - bin;
    *bout = (u32)(t >> 63);
    return (u32)t;
#endif
}

// ---- basic ops ---------------------------------------------------------------------------------
MH_FN u32 add256(const u32* x, const u32* y, u32* z) {  // returns carry out
    u32 c = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = addc32(x[k], y[k], c, &c);
    return c;
}

MH_FN u32 sub256(const u32* x, const u32* y, u32* z) {  // returns borrow out
    u32 br = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = subc32(x[k], y[k], br, &br);
    return br;
}

MH_FN void neg256(const u32* x, u32* z) {
    u32 zero[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    sub256(zero, x, z);
}

MH_FN bool ult256(const u32* x, const u32* y) {
    u32 br = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) (void)subc32(x[k], y[k], br, &br);
    return br != 0;
}

MH_FN bool eq256(const u32* x, const u32* y) {
    u32 d = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) d |= x[k] ^ y[k];
    return d == 0;
}

MH_FN bool is_zero256(const u32* x) {
    u32 d = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) d |= x[k];
    return d == 0;
}

// mask limb k of a `w`-bit value (w in 1..256)
MH_FN u32 width_mask(int k, u32 w) {
    int rem = (int)w - 32 * k;
    return rem >= 32 ? 0xFFFFFFFFu : rem <= 0 ? 0u : ((1u << rem) - 1u);
}

MH_FN void mask_w(u32* x, u32 w) {
    if (w < 256) {
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] &= width_mask(k, w);
    }
}

// bit w-1 of x
MH_FN u32 sign_bit(const u32* x, u32 w) {
    u32 b = 0, lk = (w - 1) >> 5, sh = (w - 1) & 31;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if ((u32)k == lk) b = (x[k] >> sh) & 1u;
    return b;
}

MH_FN void negw(const u32* x, u32* z, u32 w) {
    neg256(x, z);
    mask_w(z, w);
}

// (a * b) mod 2^256, schoolbook on v_mad_u64_u32
MH_FN void mul_lo256(const u32* x, const u32* y, u32* z) {
    u32 r[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u32 carry = 0;
#pragma unroll
        for (int j = 0; j < 8 - i; ++j) {
            // t = x*y + carry (v_mad_u64_u32), r += lo(t), carry = hi(t) + c
            const u64 t = (u64)x[i] * y[j] + carry;
            u32 c;
            r[i + j] = addc32(r[i + j], (u32)t, 0u, &c);
            carry = (u32)(t >> 32) + c;
        }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = r[k];
}

// full 512-bit product (z[16])
MH_FN void mul_full256(const u32* x, const u32* y, u32* z) {
    u32 r[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) r[k] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u64 carry = 0;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            u64 t = (u64)x[i] * y[j] + r[i + j] + carry;
            r[i + j] = (u32)t;
            carry = t >> 32;
        }
        r[i + 8] = (u32)carry;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) z[k] = r[k];
}

// ---- shifts ------------------------------------------------------------------------------------
// Shift amounts are < 256 here (callers saturate).  The limb part goes through a 3-stage
// select network (4, 2, 1 limbs), the bit part through v_alignbit funnel shifts.
MH_FN void shl256(const u32* x, u32 s, u32* z) {
    u32 t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = x[k];
    const u32 q = s >> 5, r = s & 31;
#pragma unroll
    for (int st = 4; st >= 1; st >>= 1) {
        const bool c = (q & (u32)st) != 0;
#pragma unroll
        for (int k = 7; k >= 0; --k) t[k] = c ? (k >= st ? t[k - st] : 0u) : t[k];
    }
#pragma unroll
    for (int k = 7; k >= 0; --k) {
        const u32 lo = k ? t[k - 1] : 0u;
        const u32 v = alignbit(t[k], lo, 32u - r);
        z[k] = r ? v : t[k];
    }
}

MH_FN void shr256(const u32* x, u32 s, u32* z, u32 fill) {  // fill = 0 or 0xffffffff
    u32 t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = x[k];
    const u32 q = s >> 5, r = s & 31;
#pragma unroll
    for (int st = 4; st >= 1; st >>= 1) {
        const bool c = (q & (u32)st) != 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) t[k] = c ? (k + st < 8 ? t[k + st] : fill) : t[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u32 hi = k < 7 ? t[k + 1] : fill;
        z[k] = alignbit(hi, t[k], r);
    }
}

// Shifts by a WAVE-UNIFORM amount s < 256 (tape immediates): the limb offset q is uniform, so
// the limb move is an indexed register read (s_set_gpr_idx / v_movrels, no select network) and
// the bit part one v_alignbit per limb.
MH_FN void shr256_u(const u32* x, u32 s, u32* z, u32 fill) {
    u32 t[17];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = x[k];
#pragma unroll
    for (int k = 8; k < 17; ++k) t[k] = fill;
    const u32 q = s >> 5, r = s & 31;
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = alignbit(t[k + q + 1], t[k + q], r);
}

MH_FN void shl256_u(const u32* x, u32 s, u32* z) {
    u32 t[17];
#pragma unroll
    for (int k = 0; k < 9; ++k) t[k] = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) t[9 + k] = x[k];
    const u32 q = s >> 5, r = s & 31;
    if (r == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) z[k] = t[9 + k - q];
    } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) z[k] = alignbit(t[9 + k - q], t[8 + k - q], 32u - r);
    }
}

// shift amount as a 256-bit value, saturated to 256 (any high limb set => >= 256)
MH_FN u32 shift_amount(const u32* y) {
    u32 hi = 0;
#pragma unroll
    for (int k = 1; k < 8; ++k) hi |= y[k];
    return (hi || y[0] > 256u) ? 256u : y[0];
}

// width-w SMT-LIB shifts on canonical operands
MH_FN void bvshl(const u32* x, u32 s, u32* z, u32 w) {
    if (s >= w) {
#pragma unroll
        for (int k = 0; k < 8; ++k) z[k] = 0;
        return;
    }
    shl256(x, s, z);
    mask_w(z, w);
}

MH_FN void bvshl_v(const u32* x, u32 s, u32* z, u32 w) {  // per-lane amount
    const bool big = s >= w;
    shl256(x, big ? 0u : s, z);
    mask_w(z, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = big ? 0u : z[k];
}

MH_FN void bvlshr_v(const u32* x, u32 s, u32* z, u32 w) {
    const bool big = s >= w;
    shr256(x, big ? 0u : s, z, 0u);
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = big ? 0u : z[k];
}

// sign-extend a canonical w-bit value to 256 bits
MH_FN void sext_to256(const u32* x, u32 w, u32* z) {
    const u32 sb = sign_bit(x, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = sb ? (x[k] | ~width_mask(k, w)) : x[k];
}

MH_FN void bvashr_v(const u32* x, u32 s, u32* z, u32 w) {
    u32 t[8];
    sext_to256(x, w, t);
    const u32 fill = t[7] >> 31 ? 0xFFFFFFFFu : 0u;
    shr256(t, s >= w ? 255u : s, z, fill);
    if (s >= w) {
#pragma unroll
        for (int k = 0; k < 8; ++k) z[k] = fill;
    }
    mask_w(z, w);
}

// ---- division ----------------------------------------------------------------------------------
// floor((uh:um) / d) for d >= 2^31 and uh < d (quotient < 2^32); f64 estimate + exact fix-up.
MH_FN u32 div64by32(u32 uh, u32 um, u32 d, double dinv, u32* rem) {
    const u64 num = ((u64)uh << 32) | um;
    double qd = ((double)uh * 4294967296.0 + (double)um) * dinv;
    qd = qd > 4294967295.0 ? 4294967295.0 : qd;
    u32 q = (u32)qd;
    int64_t r = (int64_t)(num - (u64)q * d);
    if (r < 0) { q -= 1; r += d; }
    if (r < 0) { q -= 1; r += d; }
    if ((u64)r >= d) { q += 1; r -= d; }
    if ((u64)r >= d) { q += 1; r -= d; }
    *rem = (u32)r;
    return q;
}

// One Knuth-D step at digit position J (u[J..J+8] -= qhat * v, with estimate correction).
template <int J>
MH_FN u32 knuth_step(u32* u, const u32* v, double vinv) {
    const u32 uh = u[J + 8], um = u[J + 7], ul = u[J + 6];
    u32 qh, rh;
    bool rbig;  // rhat >= 2^32
    if (uh >= v[7]) {  // uh == v7: qhat = b - 1, rhat = um + v7
        qh = 0xFFFFFFFFu;
        const u64 rr = (u64)um + v[7];
        rh = (u32)rr;
        rbig = (rr >> 32) != 0;
    } else {
        qh = div64by32(uh, um, v[7], vinv, &rh);
        rbig = false;
    }
    // D3: refine with the next divisor digit (at most twice)
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const bool over = !rbig && ((u64)qh * v[6] > (((u64)rh << 32) | ul));
        if (over) {
            qh -= 1;
            const u64 rr = (u64)rh + v[7];
            rh = (u32)rr;
            rbig = (rr >> 32) != 0;
        }
    }
    // D4: multiply and subtract
    u64 carry = 0;
    u32 br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const u64 p = (u64)qh * v[i] + carry;
        carry = p >> 32;
        const u64 t = (u64)u[J + i] - (u32)p - br;
        u[J + i] = (u32)t;
        br = (u32)(t >> 63);
    }
    {
        const u64 t = (u64)u[J + 8] - (u32)carry - br;
        u[J + 8] = (u32)t;
        br = (u32)(t >> 63);
    }
    // D6: add back (probability ~2^-31 per digit): skip unless some lane needs it
    if (any_lane(br != 0)) {
        u64 c = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            c = (u64)u[J + i] + (br ? v[i] : 0u) + c;
            u[J + i] = (u32)c;
            c >>= 32;
        }
        u[J + 8] = u[J + 8] + (br ? (u32)c : 0u);
        qh -= br;
    }
    return qh;
}

// 1/d to f64 rounding: the hardware reciprocal is an approximation (LLVM refines it twice for
// an f64 divide), so two Newton steps on the device -- one left the native code's digit
// estimates ~2^-12 off on MI355X, and the fast path below needs 2^-49.  Only feeds an estimate
// that udivrem256 corrects exactly, so host and device may round differently.
MH_FN double recip_f64(double d) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    return __builtin_fma(r, e, r);
#else
    return 1.0 / d;
#endif
}

// 256-bit value as a double (relative error < 2^-50: Horner over the limbs with fma)
MH_FN double to_f64(const u32* x) {
    double d = (double)x[7];
#pragma unroll
    for (int k = 6; k >= 0; --k) d = __builtin_fma(d, 4294967296.0, (double)x[k]);
    return d;
}

// q = x / y, r = x % y (256-bit unsigned, SMT-LIB: y == 0 gives q = 2^256 - 1, r = x)
//
// Fast path: when every lane's quotient is below 2^47 (the common case: random operands give
// 0- or 1-digit quotients), q is estimated as x/y in f64 (relative error ~2^-49, so the
// truncated estimate is the quotient or off by one), then made exact with one 9-limb product,
// one subtraction and a +-1 correction.  Otherwise (some lane has a long quotient): Knuth
// algorithm D on 32-bit digits with f64 digit estimates.
MH_FN void udivrem256(const u32* x, const u32* y, u32* q, u32* r) {
    // s = leading zeros of y (normalisation shift)
    u32 s = 0;
    bool nz = false;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        if (y[k]) {
            s = 32u * (7 - k) + clz32(y[k]);
            nz = true;
        }
    }
    // fast path for the whole wave: x < y everywhere => q = 0, r = x
    const bool small = nz && ult256(x, y);
    if (!any_lane(!small)) {
#pragma unroll
        for (int k = 0; k < 8; ++k) { q[k] = 0; r[k] = x[k]; }
        return;
    }
    {
        const double qd = to_f64(x) * recip_f64(to_f64(y));
        const bool est_ok = qd < 140737488355328.0;  // 2^47 (false for y == 0: inf / NaN)
        if (!any_lane(nz && !est_ok)) {
            const u64 qi = est_ok ? (u64)qd : 0ull;
            const u32 q0 = (u32)qi, q1 = (u32)(qi >> 32);
            // p = qi * y, 9 limbs (qi <= quotient + 1, so p < x + y < 2^257)
            u32 p[9];
            u64 c = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const u64 t = (u64)q0 * y[k] + c;
                p[k] = (u32)t;
                c = t >> 32;
            }
            p[8] = (u32)c;
            c = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {  // + (q1 * y) << 32
                const u64 t = (u64)q1 * y[k] + p[k + 1] + c;
                p[k + 1] = (u32)t;
                c = t >> 32;
            }
            // rr = x - p over 9 limbs; a borrow means the estimate was one too large
            u32 rr[9], br = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) rr[k] = subc32(x[k], p[k], br, &br);
            rr[8] = subc32(0u, p[8], br, &br);
            const bool neg = br != 0;
            // neg: rr += y (and q - 1); then rr >= y: rr -= y (and q + 1)
            u32 ca = 0, t9[9];
#pragma unroll
            for (int k = 0; k < 8; ++k) t9[k] = addc32(rr[k], neg ? y[k] : 0u, ca, &ca);
            t9[8] = rr[8] + (neg ? ca : 0u);
            u32 d9[9], bd = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) d9[k] = subc32(t9[k], y[k], bd, &bd);
            d9[8] = subc32(t9[8], 0u, bd, &bd);
            const bool ge = bd == 0;  // t9 >= y
            const u64 qf = qi - (neg ? 1ull : 0ull) + (ge ? 1ull : 0ull);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const u32 rk = ge ? d9[k] : t9[k];
                q[k] = nz ? (k == 0 ? (u32)qf : k == 1 ? (u32)(qf >> 32) : 0u) : 0xFFFFFFFFu;
                r[k] = nz ? rk : x[k];
            }
            return;
        }
    }
    u32 v[8];
    shl256(y, s, v);
    // u = x << s as 512 bits (u[16]), built from two 256-bit shifts
    u32 u[17];
    shl256(x, s, u);
    {
        u32 hi[8];
        // x >> (256 - s): for s == 0 this is 0
        const u32 rs = 256u - s;
        shr256(x, rs >= 256u ? 0u : rs, hi, 0u);
#pragma unroll
        for (int k = 0; k < 8; ++k) u[8 + k] = s ? hi[k] : 0u;
    }
    u[16] = 0;
    const double vinv = recip_f64((double)(v[7] ? v[7] : 1u));
    const u32 jmax = s >> 5;  // quotient digits above jmax are zero
    u32 qd[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define MH_KSTEP(J) \
    if (any_lane(nz && (u32)(J) <= jmax)) qd[J] = knuth_step<J>(u, v, vinv);
    MH_KSTEP(7) MH_KSTEP(6) MH_KSTEP(5) MH_KSTEP(4) MH_KSTEP(3) MH_KSTEP(2) MH_KSTEP(1)
    MH_KSTEP(0)
#undef MH_KSTEP
    u32 rr[8];
    shr256(u, s, rr, 0u);  // remainder = u[0..7] >> s
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        q[k] = nz ? ((u32)k <= jmax ? qd[k] : 0u) : 0xFFFFFFFFu;
        r[k] = nz ? rr[k] : x[k];
    }
}

// SMT-LIB signed division family at width w (canonical operands)
MH_FN void bvsdiv(const u32* x, const u32* y, u32* z, u32 w) {
    const u32 ms = sign_bit(x, w), mt = sign_bit(y, w);
    u32 ax[8], ay[8], nx[8], ny[8], q[8], r[8];
    negw(x, nx, w);
    negw(y, ny, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) { ax[k] = ms ? nx[k] : x[k]; ay[k] = mt ? ny[k] : y[k]; }
    udivrem256(ax, ay, q, r);
    mask_w(q, w);
    u32 nq[8];
    negw(q, nq, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = (ms != mt) ? nq[k] : q[k];
}

MH_FN void bvsrem(const u32* x, const u32* y, u32* z, u32 w) {
    const u32 ms = sign_bit(x, w), mt = sign_bit(y, w);
    u32 ax[8], ay[8], nx[8], ny[8], q[8], r[8];
    negw(x, nx, w);
    negw(y, ny, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) { ax[k] = ms ? nx[k] : x[k]; ay[k] = mt ? ny[k] : y[k]; }
    udivrem256(ax, ay, q, r);
    u32 nr[8];
    negw(r, nr, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = ms ? nr[k] : r[k];
}

MH_FN void bvsmod(const u32* x, const u32* y, u32* z, u32 w) {
    const u32 ms = sign_bit(x, w), mt = sign_bit(y, w);
    u32 ax[8], ay[8], nx[8], ny[8], q[8], u[8];
    negw(x, nx, w);
    negw(y, ny, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) { ax[k] = ms ? nx[k] : x[k]; ay[k] = mt ? ny[k] : y[k]; }
    udivrem256(ax, ay, q, u);
    const bool uz = is_zero256(u);
    u32 nu[8], a1[8], a2[8];
    negw(u, nu, w);
    add256(nu, y, a1);  // -u + t
    mask_w(a1, w);
    add256(u, y, a2);   //  u + t
    mask_w(a2, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        u32 v = (!ms && !mt) ? u[k] : (ms && !mt) ? a1[k] : (!ms && mt) ? a2[k] : nu[k];
        z[k] = uz ? 0u : v;
    }
}

// signed compare at width w: flip bit w-1 and compare unsigned
MH_FN bool slt_w(const u32* x, const u32* y, u32 w) {
    u32 xf[8], yf[8];
    const u32 lk = (w - 1) >> 5, bit = 1u << ((w - 1) & 31);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const u32 f = (u32)k == lk ? bit : 0u;
        xf[k] = x[k] ^ f;
        yf[k] = y[k] ^ f;
    }
    return ult256(xf, yf);
}

// The whole division family through ONE udivrem256 site (SMT-LIB sign rules around it), so
// the long division is instantiated once per kernel.  kind: 0 udiv, 1 urem, 2 sdiv, 3 srem,
// 4 smod.
MH_FN void divmod_family(u32 kind, const u32* x, const u32* y, u32* z, u32 w) {
    const bool sgn = kind >= 2;
    const u32 ms = sgn ? sign_bit(x, w) : 0u, mt = sgn ? sign_bit(y, w) : 0u;
    u32 ax[8], ay[8], t[8], q[8], r[8];
    negw(x, t, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) ax[k] = ms ? t[k] : x[k];
    negw(y, t, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) ay[k] = mt ? t[k] : y[k];
    udivrem256(ax, ay, q, r);
    mask_w(q, w);
    if (kind == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) z[k] = q[k];
    } else if (kind == 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) z[k] = r[k];
    } else if (kind == 2) {
        negw(q, t, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) z[k] = (ms != mt) ? t[k] : q[k];
    } else if (kind == 3) {
        negw(r, t, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) z[k] = ms ? t[k] : r[k];
    } else {  // D_SMOD: sign of the divisor
        const bool uz = is_zero256(r);
        u32 s1[8];
        negw(r, t, w);
        if (ms && !mt) add256(t, y, s1);       // -u + t
        else if (!ms && mt) add256(r, y, s1);  //  u + t
        else if (ms && mt) {
#pragma unroll
            for (int k = 0; k < 8; ++k) s1[k] = t[k];  // -u
        } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) s1[k] = r[k];  //  u
        }
        mask_w(s1, w);
#pragma unroll
        for (int k = 0; k < 8; ++k) z[k] = uz ? 0u : s1[k];
    }
}

// ---- EVM ADDMOD / MULMOD: a 512-bit intermediate ------------------------------------------------
// r = u mod y for u < 2^512 (u16: 16 limbs) and y != 0: Knuth algorithm D over 32-bit digits,
// udivrem256's long path with eight more digit positions.  u << s spans 24 limbs (s < 256 is the
// normalisation shift); the top digit position is 8 + s / 32 <= 15, and a lane whose divisor
// needs fewer positions gets zero digits at the extra ones (its window is below v there), so all
// lanes run the same steps.
MH_FN void urem512(const u32* u16, const u32* y, u32* r) {
    u32 s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (y[k]) s = 32u * (7 - k) + clz32(y[k]);
    u32 v[8];
    shl256(y, s, v);
    u32 u[25];
    {
        u32 lo[8], hi[8], t[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { lo[k] = u16[k]; hi[k] = u16[8 + k]; }
        const u32 rs = 256u - s;  // bits of each half shifted into the next (none for s = 0)
        shl256(lo, s, t);
#pragma unroll
        for (int k = 0; k < 8; ++k) u[k] = t[k];
        shl256(hi, s, t);
#pragma unroll
        for (int k = 0; k < 8; ++k) u[8 + k] = t[k];
        shr256(lo, rs >= 256u ? 0u : rs, t, 0u);
#pragma unroll
        for (int k = 0; k < 8; ++k) u[8 + k] |= s ? t[k] : 0u;
        shr256(hi, rs >= 256u ? 0u : rs, t, 0u);
#pragma unroll
        for (int k = 0; k < 8; ++k) u[16 + k] = s ? t[k] : 0u;
        u[24] = 0;
    }
    const double vinv = recip_f64((double)(v[7] ? v[7] : 1u));
#define MH_RSTEP(J) (void)knuth_step<J>(u, v, vinv);
    MH_RSTEP(15) MH_RSTEP(14) MH_RSTEP(13) MH_RSTEP(12) MH_RSTEP(11) MH_RSTEP(10) MH_RSTEP(9)
    MH_RSTEP(8) MH_RSTEP(7) MH_RSTEP(6) MH_RSTEP(5) MH_RSTEP(4) MH_RSTEP(3) MH_RSTEP(2)
    MH_RSTEP(1) MH_RSTEP(0)
#undef MH_RSTEP
    shr256(u, s, r, 0u);  // the remainder is u[0..7] >> s
}

// Yellow-paper ADDMOD (mul = false) / MULMOD (mul = true) of 256-bit words: (x op y) mod n with
// the exact sum / product; n == 0 gives 0, or with zero_low the low 256 bits of x op y (z3's
// extract[255:0](bvurem(zext x op zext y, zext n)), SMT-LIB's x % 0 = x).
MH_FN void evm_modop(bool mul, const u32* x, const u32* y, const u32* n, u32* z, bool zero_low) {
    u32 u[16];
    if (mul) {
        mul_full256(x, y, u);
    } else {
        u[8] = add256(x, y, u);
#pragma unroll
        for (int k = 9; k < 16; ++k) u[k] = 0;
    }
    const bool nz = !is_zero256(n);
    u32 r[8];
    urem512(u, n, r);
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = nz ? r[k] : (zero_low ? u[k] : 0u);
}

// ---- EVM word helpers (256-bit only) -----------------------------------------------------------
MH_FN void evm_exp(const u32* base, const u32* e, u32* z, u32 w) {
    u32 res[8] = {1, 0, 0, 0, 0, 0, 0, 0};
    u32 b[8], ee[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { b[k] = base[k]; ee[k] = e[k]; }
    for (int i = 0; i < 256; ++i) {
        if (!any_lane(!is_zero256(ee))) break;
        const bool bit = ee[0] & 1u;
        u32 t[8];
        mul_lo256(res, b, t);
#pragma unroll
        for (int k = 0; k < 8; ++k) res[k] = bit ? t[k] : res[k];
        mul_lo256(b, b, t);
#pragma unroll
        for (int k = 0; k < 8; ++k) b[k] = t[k];
        shr256(ee, 1, ee, 0u);
    }
    mask_w(res, w);
#pragma unroll
    for (int k = 0; k < 8; ++k) z[k] = res[k];
}

MH_FN void evm_signextend(const u32* kk, const u32* x, u32* z) {
    u32 hi = 0;
#pragma unroll
    for (int k = 1; k < 8; ++k) hi |= kk[k];
    const bool keep = hi || kk[0] > 30u;
    const u32 tb = keep ? 0u : kk[0] * 8u + 7u;  // < 255
    const u32 lk = tb >> 5, sh = tb & 31;
    u32 bit = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if ((u32)k == lk) bit = (x[k] >> sh) & 1u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int rem = (int)tb + 1 - 32 * k;  // bits of this limb at or below tb
        const u32 m = rem >= 32 ? 0xFFFFFFFFu : rem <= 0 ? 0u : ((1u << rem) - 1u);
        const u32 v = bit ? (x[k] | ~m) : (x[k] & m);
        z[k] = keep ? x[k] : v;
    }
}

MH_FN void evm_byte(const u32* ii, const u32* x, u32* z) {
    u32 hi = 0;
#pragma unroll
    for (int k = 1; k < 8; ++k) hi |= ii[k];
    const bool zero = hi || ii[0] > 31u;
    const u32 bi = zero ? 0u : 31u - ii[0];  // byte index from the least significant end
    const u32 lk = bi >> 2, sh = 8u * (bi & 3u);
    u32 limb = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if ((u32)k == lk) limb = x[k];
    z[0] = zero ? 0u : ((limb >> sh) & 0xFFu);
#pragma unroll
    for (int k = 1; k < 8; ++k) z[k] = 0;
}

// ---- Keccak-f[1600] ----------------------------------------------------------------------------
MH_FN u64 rotl64(u64 x, int n) { return n ? ((x << n) | (x >> (64 - n))) : x; }

// Keccak-f[1600] round constants.  On the device a __constant__ table read with a wave-uniform
// index (scalar loads); a local array indexed by the loop counter lived in scratch memory.
#define MH_KECCAK_RC                                                                              \
    {0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull, \
     0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull, \
     0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull, \
     0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull, \
     0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull, \
     0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull}
#if defined(__HIPCC__)
__constant__ static const u64 kKeccakRCDev[24] = MH_KECCAK_RC;
#endif
static const u64 kKeccakRCHost[24] = MH_KECCAK_RC;

MH_FN u64 keccak_rc(int round) {
#if defined(__HIP_DEVICE_COMPILE__)
    return kKeccakRCDev[round];
#else
    return kKeccakRCHost[round];
#endif
}

MH_FN void keccak_f1600(u64* a) {
#pragma unroll 1
    for (int round = 0; round < 24; ++round) {
        u64 c[5], d[5];
#pragma unroll
        for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
#pragma unroll
        for (int x = 0; x < 5; ++x) d[x] = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
#pragma unroll
        for (int i = 0; i < 25; ++i) a[i] ^= d[i % 5];
        // rho + pi, in place along the pi cycle starting at lane 1
        u64 cur = a[1];
#define MH_RP(dst, rot) { u64 t = a[dst]; a[dst] = rotl64(cur, rot); cur = t; }
        MH_RP(10, 1) MH_RP(7, 3) MH_RP(11, 6) MH_RP(17, 10) MH_RP(18, 15) MH_RP(3, 21)
        MH_RP(5, 28) MH_RP(16, 36) MH_RP(8, 45) MH_RP(21, 55) MH_RP(24, 2) MH_RP(4, 14)
        MH_RP(15, 27) MH_RP(23, 41) MH_RP(19, 56) MH_RP(13, 8) MH_RP(12, 25) MH_RP(2, 43)
        MH_RP(20, 62) MH_RP(14, 18) MH_RP(22, 39) MH_RP(9, 61) MH_RP(6, 20) MH_RP(1, 44)
#undef MH_RP
        // chi
#pragma unroll
        for (int y = 0; y < 25; y += 5) {
            const u64 b0 = a[y], b1 = a[y + 1], b2 = a[y + 2], b3 = a[y + 3], b4 = a[y + 4];
            a[y] = b0 ^ (~b1 & b2);
            a[y + 1] = b1 ^ (~b2 & b3);
            a[y + 2] = b2 ^ (~b3 & b4);
            a[y + 3] = b3 ^ (~b4 & b0);
            a[y + 4] = b4 ^ (~b0 & b1);
        }
        a[0] ^= keccak_rc(round);
    }
}

}  // namespace mh
