/*
 * ORACLE (test infrastructure only — never linked into the product library).
 *
 * Plain-C restatement of the tape semantics in oracle/smt_eval.py, for parity checks at sizes
 * the Python oracle cannot reach and for bench.py's cpu_baseline ("port").  Values are held as
 * 34 x u32 little-endian limbs (every IR width up to 1088 bits), each op masked to its width.
 * Semantics are SMT-LIB QF_BV as z3's model evaluator applies them to mythril's terms (see the
 * citation table in oracle/smt_eval.py):
 *   bvudiv x 0 = 2^w-1, bvurem x 0 = x, bvsdiv/bvsrem/bvsmod by the SMT-LIB sign rules,
 *   shifts >= w give 0 / sign fill, keccak = Keccak-256 of the big-endian input bytes
 *   (keccak_function_manager.py:43-57).
 * Division is Knuth's Algorithm D on 32-bit digits (TAOCP vol. 2, 4.3.1), written out here.
 * Node layout and op numbers follow include/mythril_hip.h (mh_node, enum mh_op).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NL 34 /* limbs: 1088 bits (Keccak inputs up to one 136-byte block) */

typedef struct {
    uint8_t op, flags;
    uint16_t width;
    uint32_t a, b, c, imm0, imm1;
} node_t;

typedef struct {
    uint32_t v[NL];
} val_t;

enum {
    CONST = 0, VAR = 1, TRUE_ = 2, FALSE_ = 3,
    BVADD = 10, BVSUB, BVMUL, BVUDIV, BVUREM, BVSDIV, BVSREM, BVSMOD, BVNEG, BVNOT,
    BVAND = 20, BVOR, BVXOR, BVSHL, BVLSHR, BVASHR,
    EQ = 30, BVULT, BVULE, BVUGT, BVUGE, BVSLT, BVSLE, BVSGT, BVSGE,
    AND = 40, OR, XOR, NOT, ITE = 45,
    EXTRACT = 50, CONCAT, ZEXT, SEXT,
    KECCAK = 60, ADD_NOOVFL = 61, MUL_NOOVFL = 62, SUB_NOUDFL = 63,
    EVM_EXP = 70, EVM_SIGNEXTEND = 71, EVM_BYTE = 72, EVM_ADDMOD = 73, EVM_MULMOD = 74
};

static void vmask(val_t* x, int w) {
    for (int k = 0; k < NL; ++k) {
        int rem = w - 32 * k;
        if (rem <= 0) x->v[k] = 0;
        else if (rem < 32) x->v[k] &= (1u << rem) - 1u;
    }
}

static int vbit(const val_t* x, int i) { return (x->v[i >> 5] >> (i & 31)) & 1; }

static int vcmp(const val_t* x, const val_t* y) {
    for (int k = NL - 1; k >= 0; --k)
        if (x->v[k] != y->v[k]) return x->v[k] < y->v[k] ? -1 : 1;
    return 0;
}

static int viszero(const val_t* x) {
    for (int k = 0; k < NL; ++k)
        if (x->v[k]) return 0;
    return 1;
}

static __thread int g_nl = NL; /* limbs covering the current op's width (set per node) */

static void vadd(const val_t* x, const val_t* y, val_t* z) {
    uint64_t c = 0;
    for (int k = 0; k < g_nl; ++k) {
        c += (uint64_t)x->v[k] + y->v[k];
        z->v[k] = (uint32_t)c;
        c >>= 32;
    }
}

static void vsub(const val_t* x, const val_t* y, val_t* z) {
    int64_t br = 0;
    for (int k = 0; k < g_nl; ++k) {
        int64_t t = (int64_t)x->v[k] - y->v[k] - br;
        z->v[k] = (uint32_t)t;
        br = t < 0;
    }
}

static void vmul(const val_t* x, const val_t* y, val_t* z) {
    uint32_t r[NL] = {0};
    for (int i = 0; i < g_nl; ++i) {
        if (!x->v[i]) continue;
        uint64_t c = 0;
        for (int j = 0; i + j < g_nl; ++j) {
            uint64_t t = (uint64_t)x->v[i] * y->v[j] + r[i + j] + c;
            r[i + j] = (uint32_t)t;
            c = t >> 32;
        }
    }
    memcpy(z->v, r, sizeof(r));
}

static void vshl(const val_t* x, unsigned s, val_t* z) { /* s < 512 */
    val_t r;
    memset(&r, 0, sizeof(r));
    unsigned q = s >> 5, b = s & 31;
    for (int k = NL - 1; k >= (int)q; --k) {
        uint32_t hi = x->v[k - q];
        uint32_t lo = (k - (int)q - 1 >= 0) ? x->v[k - q - 1] : 0;
        r.v[k] = b ? (hi << b) | (lo >> (32 - b)) : hi;
    }
    *z = r;
}

static void vshr(const val_t* x, unsigned s, val_t* z) { /* logical, s < 512 */
    val_t r;
    memset(&r, 0, sizeof(r));
    unsigned q = s >> 5, b = s & 31;
    for (int k = 0; k + (int)q < NL; ++k) {
        uint32_t lo = x->v[k + q];
        uint32_t hi = (k + q + 1 < NL) ? x->v[k + q + 1] : 0;
        r.v[k] = b ? (lo >> b) | (hi << (32 - b)) : lo;
    }
    *z = r;
}

static void vneg(const val_t* x, val_t* z, int w) {
    val_t zero;
    memset(&zero, 0, sizeof(zero));
    vsub(&zero, x, z);
    vmask(z, w);
}

static int nlimbs(const val_t* x) {
    int n = NL;
    while (n > 0 && x->v[n - 1] == 0) --n;
    return n;
}

static int clz32(uint32_t x) {
    int n = 0;
    if (!x) return 32;
    while (!(x & 0x80000000u)) { x <<= 1; ++n; }
    return n;
}

/* Knuth Algorithm D: q = u / v, r = u % v (v != 0) */
static void vdivmod(const val_t* u, const val_t* v, val_t* q, val_t* r) {
    memset(q, 0, sizeof(*q));
    memset(r, 0, sizeof(*r));
    int m = nlimbs(u), n = nlimbs(v);
    if (m < n) { *r = *u; return; }
    if (n == 1) {
        uint64_t rem = 0;
        for (int j = m - 1; j >= 0; --j) {
            uint64_t cur = (rem << 32) | u->v[j];
            q->v[j] = (uint32_t)(cur / v->v[0]);
            rem = cur % v->v[0];
        }
        r->v[0] = (uint32_t)rem;
        return;
    }
    int s = clz32(v->v[n - 1]);
    uint32_t vn[NL], un[NL + 1];
    for (int i = n - 1; i > 0; --i)
        vn[i] = (v->v[i] << s) | (s ? (uint32_t)((uint64_t)v->v[i - 1] >> (32 - s)) : 0);
    vn[0] = v->v[0] << s;
    un[m] = s ? (uint32_t)((uint64_t)u->v[m - 1] >> (32 - s)) : 0;
    for (int i = m - 1; i > 0; --i)
        un[i] = (u->v[i] << s) | (s ? (uint32_t)((uint64_t)u->v[i - 1] >> (32 - s)) : 0);
    un[0] = u->v[0] << s;
    for (int j = m - n; j >= 0; --j) {
        uint64_t num = ((uint64_t)un[j + n] << 32) | un[j + n - 1];
        uint64_t qhat = num / vn[n - 1], rhat = num % vn[n - 1];
        while (qhat >= (1ull << 32) ||
               qhat * vn[n - 2] > ((rhat << 32) | un[j + n - 2])) {
            --qhat;
            rhat += vn[n - 1];
            if (rhat >= (1ull << 32)) break;
        }
        int64_t t, k = 0;
        for (int i = 0; i < n; ++i) {
            uint64_t p = qhat * vn[i];
            t = (int64_t)un[i + j] - k - (int64_t)(p & 0xFFFFFFFFu);
            un[i + j] = (uint32_t)t;
            k = (int64_t)(p >> 32) - (t >> 32);
        }
        t = (int64_t)un[j + n] - k;
        un[j + n] = (uint32_t)t;
        q->v[j] = (uint32_t)qhat;
        if (t < 0) {
            q->v[j] -= 1;
            uint64_t c = 0;
            for (int i = 0; i < n; ++i) {
                c += (uint64_t)un[i + j] + vn[i];
                un[i + j] = (uint32_t)c;
                c >>= 32;
            }
            un[j + n] += (uint32_t)c;
        }
    }
    for (int i = 0; i < n; ++i)
        r->v[i] = (un[i] >> s) | (s ? (uint32_t)((uint64_t)un[i + 1] << (32 - s)) : 0);
}

static void bvudivrem(const val_t* x, const val_t* y, val_t* q, val_t* r, int w) {
    if (viszero(y)) {
        memset(q, 0xFF, sizeof(*q));
        vmask(q, w);
        *r = *x;
        return;
    }
    vdivmod(x, y, q, r);
}

/* ---- Keccak-256 ------------------------------------------------------------------------------ */
static const uint64_t RC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
    0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
    0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
static const int ROT[5][5] = {{0, 36, 3, 41, 18}, {1, 44, 10, 45, 2}, {62, 6, 43, 15, 61},
                              {28, 55, 25, 21, 56}, {27, 20, 39, 8, 14}};

static uint64_t rol(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

static void keccakf(uint64_t a[25]) {
    for (int round = 0; round < 24; ++round) {
        uint64_t c[5], b[25];
        for (int x = 0; x < 5; ++x) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
        for (int x = 0; x < 5; ++x) {
            uint64_t d = c[(x + 4) % 5] ^ rol(c[(x + 1) % 5], 1);
            for (int y = 0; y < 5; ++y) a[x + 5 * y] ^= d;
        }
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y) b[y + 5 * ((2 * x + 3 * y) % 5)] = rol(a[x + 5 * y], ROT[x][y]);
        for (int x = 0; x < 5; ++x)
            for (int y = 0; y < 5; ++y)
                a[x + 5 * y] = b[x + 5 * y] ^ (~b[(x + 1) % 5 + 5 * y] & b[(x + 2) % 5 + 5 * y]);
        a[0] ^= RC[round];
    }
}

static void keccak256(const uint8_t* msg, size_t len, uint8_t out[32]) {
    uint64_t a[25];
    memset(a, 0, sizeof(a));
    uint8_t block[136];
    size_t off = 0;
    for (;;) {
        size_t take = len - off < 136 ? len - off : 136;
        memset(block, 0, sizeof(block));
        memcpy(block, msg + off, take);
        int last = take < 136;
        if (last) {
            block[take] |= 0x01;
            block[135] |= 0x80;
        }
        for (int i = 0; i < 17; ++i) {
            uint64_t v = 0;
            for (int b = 0; b < 8; ++b) v |= (uint64_t)block[8 * i + b] << (8 * b);
            a[i] ^= v;
        }
        keccakf(a);
        off += take;
        if (last) break;
    }
    for (int i = 0; i < 4; ++i)
        for (int b = 0; b < 8; ++b) out[8 * i + b] = (uint8_t)(a[i] >> (8 * b));
}

static int vsigned_lt(const val_t* x, const val_t* y, int w) {
    int sx = vbit(x, w - 1), sy = vbit(y, w - 1);
    if (sx != sy) return sx > sy;
    return vcmp(x, y) < 0;
}

/* Value of node i from the values V[] of its operands.  Returns 0, or -1 on a malformed node. */
static int node_value(const node_t* nd, uint64_t i, const uint32_t* consts, uint32_t n_consts,
                      const uint32_t* assign, uint32_t n_vars, val_t* V) {
    {
        const node_t* t = &nd[i];
        const int w = t->width;
        val_t z;
        memset(&z, 0, sizeof(z));
        /* results never exceed their width, and MUL_NOOVFL needs the double-width product */
        g_nl = (t->op == MUL_NOOVFL || t->op == ADD_NOOVFL || t->op == EVM_ADDMOD ||
                t->op == EVM_MULMOD) ? NL : (w + 31) / 32 + 1;
        if (g_nl > NL || w == 0) g_nl = NL;
        const val_t *x = t->a < i ? &V[t->a] : NULL, *y = t->b < i ? &V[t->b] : NULL;
        switch (t->op) {
            case CONST:
                if (t->imm0 >= n_consts) goto bad;
                memcpy(z.v, consts + 8ull * t->imm0, 32);
                vmask(&z, w);
                break;
            case VAR:
                if (t->imm0 >= n_vars) goto bad;
                memcpy(z.v, assign + 8ull * t->imm0, 32);
                vmask(&z, w);
                break;
            case TRUE_: z.v[0] = 1; break;
            case FALSE_: break;
            case BVADD: vadd(x, y, &z); vmask(&z, w); break;
            case BVSUB: vsub(x, y, &z); vmask(&z, w); break;
            case BVMUL: vmul(x, y, &z); vmask(&z, w); break;
            case BVUDIV: case BVUREM: {
                val_t q, r;
                bvudivrem(x, y, &q, &r, w);
                z = t->op == BVUDIV ? q : r;
                break;
            }
            case BVSDIV: case BVSREM: case BVSMOD: {
                int ms = vbit(x, w - 1), mt = vbit(y, w - 1);
                val_t ax = *x, ay = *y, q, r, u;
                if (ms) vneg(x, &ax, w);
                if (mt) vneg(y, &ay, w);
                bvudivrem(&ax, &ay, &q, &r, w);
                if (t->op == BVSDIV) {
                    if (ms != mt) vneg(&q, &z, w); else z = q;
                } else if (t->op == BVSREM) {
                    if (ms) vneg(&r, &z, w); else z = r;
                } else {
                    u = r;
                    if (viszero(&u)) break;
                    if (!ms && !mt) z = u;
                    else if (ms && !mt) { val_t nu; vneg(&u, &nu, w); vadd(&nu, y, &z); vmask(&z, w); }
                    else if (!ms && mt) { vadd(&u, y, &z); vmask(&z, w); }
                    else vneg(&u, &z, w);
                }
                break;
            }
            case BVNEG: vneg(x, &z, w); break;
            case BVNOT: for (int k = 0; k < NL; ++k) z.v[k] = ~x->v[k]; vmask(&z, w); break;
            case BVAND: for (int k = 0; k < NL; ++k) z.v[k] = x->v[k] & y->v[k]; break;
            case BVOR: for (int k = 0; k < NL; ++k) z.v[k] = x->v[k] | y->v[k]; break;
            case BVXOR: for (int k = 0; k < NL; ++k) z.v[k] = x->v[k] ^ y->v[k]; break;
            case BVSHL: case BVLSHR: case BVASHR: {
                val_t wv;
                memset(&wv, 0, sizeof(wv));
                wv.v[0] = (uint32_t)w;
                int big = vcmp(y, &wv) >= 0;
                unsigned s = big ? 0 : y->v[0];
                if (t->op == BVSHL) {
                    if (!big) { vshl(x, s, &z); vmask(&z, w); }
                } else if (t->op == BVLSHR) {
                    if (!big) vshr(x, s, &z);
                } else {
                    int sg = vbit(x, w - 1);
                    if (big) {
                        if (sg) { memset(&z, 0xFF, sizeof(z)); vmask(&z, w); }
                    } else {
                        vshr(x, s, &z);
                        if (sg)
                            for (int i = w - (int)s; i < w; ++i) z.v[i >> 5] |= 1u << (i & 31);
                    }
                }
                break;
            }
            case EQ: z.v[0] = vcmp(x, y) == 0; break;
            case BVULT: z.v[0] = vcmp(x, y) < 0; break;
            case BVULE: z.v[0] = vcmp(x, y) <= 0; break;
            case BVUGT: z.v[0] = vcmp(x, y) > 0; break;
            case BVUGE: z.v[0] = vcmp(x, y) >= 0; break;
            case BVSLT: z.v[0] = vsigned_lt(x, y, nd[t->a].width); break;
            case BVSLE: z.v[0] = !vsigned_lt(y, x, nd[t->a].width); break;
            case BVSGT: z.v[0] = vsigned_lt(y, x, nd[t->a].width); break;
            case BVSGE: z.v[0] = !vsigned_lt(x, y, nd[t->a].width); break;
            case ADD_NOOVFL: {
                val_t s;
                vadd(x, y, &s);
                val_t m = s;
                vmask(&m, nd[t->a].width);
                z.v[0] = vcmp(&m, &s) == 0;
                break;
            }
            case MUL_NOOVFL: {
                /* operands <= 256 bits: the 512-bit product is exact */
                val_t p;
                vmul(x, y, &p);
                val_t m = p;
                vmask(&m, nd[t->a].width);
                z.v[0] = vcmp(&m, &p) == 0;
                break;
            }
            case SUB_NOUDFL: z.v[0] = vcmp(y, x) <= 0; break;
            case AND: z.v[0] = (x->v[0] & y->v[0]) & 1; break;
            case OR: z.v[0] = (x->v[0] | y->v[0]) & 1; break;
            case XOR: z.v[0] = (x->v[0] ^ y->v[0]) & 1; break;
            case NOT: z.v[0] = !(x->v[0] & 1); break;
            case ITE: {
                if (t->c >= i) goto bad;
                z = (x->v[0] & 1) ? *y : V[t->c];
                break;
            }
            case EXTRACT: vshr(x, t->imm1, &z); vmask(&z, t->imm0 - t->imm1 + 1); break;
            case CONCAT: vshl(x, nd[t->b].width, &z); for (int k = 0; k < NL; ++k) z.v[k] |= y->v[k]; break;
            case ZEXT: z = *x; break;
            case SEXT: {
                int wa = nd[t->a].width;
                z = *x;
                if (vbit(x, wa - 1))
                    for (int i2 = wa; i2 < w; ++i2) z.v[i2 >> 5] |= 1u << (i2 & 31);
                break;
            }
            case KECCAK: {
                int nb = nd[t->a].width / 8;
                uint8_t msg[136], h[32];
                for (int j = 0; j < nb; ++j) {
                    int e = nb - 1 - j;
                    msg[j] = (uint8_t)(x->v[e >> 2] >> (8 * (e & 3)));
                }
                keccak256(msg, (size_t)nb, h);
                for (int k = 0; k < 8; ++k)
                    z.v[k] = ((uint32_t)h[31 - 4 * k]) | ((uint32_t)h[30 - 4 * k] << 8) |
                             ((uint32_t)h[29 - 4 * k] << 16) | ((uint32_t)h[28 - 4 * k] << 24);
                break;
            }
            case EVM_EXP: {
                val_t res, b = *x, e = *y;
                memset(&res, 0, sizeof(res));
                res.v[0] = 1;
                while (!viszero(&e)) {
                    if (e.v[0] & 1) { vmul(&res, &b, &res); vmask(&res, w); }
                    vmul(&b, &b, &b);
                    vmask(&b, w);
                    vshr(&e, 1, &e);
                }
                z = res;
                break;
            }
            case EVM_ADDMOD: case EVM_MULMOD: {
                /* yellow-paper ADDMOD / MULMOD: the exact sum / product (<= 512 bits) mod c;
                 * c == 0 gives 0, or with imm0 = 1 the low 256 bits (bvurem's x % 0 = x) */
                if (t->c >= i) goto bad;
                val_t u, q, r;
                memset(&u, 0, sizeof(u));
                if (t->op == EVM_ADDMOD) vadd(x, y, &u);
                else vmul(x, y, &u);
                if (viszero(&V[t->c])) {
                    if (t->imm0 == 1) { z = u; vmask(&z, 256); }
                    break;
                }
                vdivmod(&u, &V[t->c], &q, &r);
                z = r;
                break;
            }
            case EVM_SIGNEXTEND: {
                val_t lim;
                memset(&lim, 0, sizeof(lim));
                lim.v[0] = 31;
                z = *y;
                if (vcmp(x, &lim) <= 0) {
                    int tb = (int)x->v[0] * 8 + 7;
                    if (tb < w) {
                        if (vbit(y, tb)) {
                            for (int i2 = tb + 1; i2 < w; ++i2) z.v[i2 >> 5] |= 1u << (i2 & 31);
                        } else {
                            for (int i2 = tb + 1; i2 < NL * 32; ++i2) z.v[i2 >> 5] &= ~(1u << (i2 & 31));
                        }
                    }
                }
                break;
            }
            case EVM_BYTE: {
                val_t lim;
                memset(&lim, 0, sizeof(lim));
                lim.v[0] = (uint32_t)(w / 8);
                if (vcmp(x, &lim) < 0) {
                    int bi = w / 8 - 1 - (int)x->v[0];
                    z.v[0] = (y->v[bi >> 2] >> (8 * (bi & 3))) & 0xFF;
                }
                break;
            }
            default:
                goto bad;
        }
        V[i] = z;
    }
    return 0;
bad:
    return -1;
}

static __thread val_t* g_V = NULL;  /* per-thread scratch, grown on demand */
static __thread uint8_t* g_done = NULL;
static __thread uint64_t g_cap = 0;

static int scratch(uint64_t n) {
    if (n <= g_cap) return 0;
    free(g_V);
    free(g_done);
    g_cap = n < 256 ? 256 : n;
    g_V = (val_t*)malloc(sizeof(val_t) * g_cap);
    g_done = (uint8_t*)malloc(g_cap);
    if (!g_V || !g_done) { g_cap = 0; return -1; }
    return 0;
}

/* Evaluate one tape; out receives the root (16 limbs).  Returns 0, or -1 on a malformed tape. */
int ct_eval(const node_t* nd, uint64_t n, const uint32_t* consts, uint32_t n_consts,
            const uint32_t* assign /* [n_vars][8] */, uint32_t n_vars, uint32_t* out) {
    if (scratch(n)) return -1;
    for (uint64_t i = 0; i < n; ++i)
        if (node_value(nd, i, consts, n_consts, assign, n_vars, g_V)) return -1;
    memcpy(out, g_V[n - 1].v, sizeof(uint32_t) * NL);
    return 0;
}

/* Short-circuit evaluation of node i: operands on demand (memoised in g_done), the second
 * operand of a Bool AND only when the first holds -- what a scalar evaluator does for a path
 * condition, so the CPU baseline skips the same work the GPU's wave-level short circuit does. */
static int lazy(const node_t* nd, uint64_t i, const uint32_t* consts, uint32_t n_consts,
                const uint32_t* assign, uint32_t n_vars) {
    if (g_done[i]) return 0;
    const node_t* t = &nd[i];
    if (t->op == AND) {
        if (t->a >= i || t->b >= i) return -1;
        if (lazy(nd, t->a, consts, n_consts, assign, n_vars)) return -1;
        if (!(g_V[t->a].v[0] & 1)) {
            memset(&g_V[i], 0, sizeof(val_t));
        } else {
            if (lazy(nd, t->b, consts, n_consts, assign, n_vars)) return -1;
            memset(&g_V[i], 0, sizeof(val_t));
            g_V[i].v[0] = g_V[t->b].v[0] & 1;
        }
        g_done[i] = 1;
        return 0;
    }
    const uint64_t ops[3] = {t->a, t->b, t->c};
    const int ar = t->op <= FALSE_ ? 0 : (t->op == ITE || t->op == EVM_ADDMOD ||
                                         t->op == EVM_MULMOD) ? 3 :
                   (t->op == BVNEG || t->op == BVNOT || t->op == NOT || t->op == EXTRACT ||
                    t->op == ZEXT || t->op == SEXT || t->op == KECCAK) ? 1 : 2;
    for (int k = 0; k < ar; ++k) {
        if (ops[k] >= i) return -1;
        if (lazy(nd, ops[k], consts, n_consts, assign, n_vars)) return -1;
    }
    if (node_value(nd, i, consts, n_consts, assign, n_vars, g_V)) return -1;
    g_done[i] = 1;
    return 0;
}

int ct_eval_lazy(const node_t* nd, uint64_t n, const uint32_t* consts, uint32_t n_consts,
                 const uint32_t* assign, uint32_t n_vars, uint32_t* out) {
    if (n == 0 || scratch(n)) return -1;
    memset(g_done, 0, n);
    if (lazy(nd, n - 1, consts, n_consts, assign, n_vars)) return -1;
    memcpy(out, g_V[n - 1].v, sizeof(uint32_t) * NL);
    return 0;
}

/* ---- counter-based assignment generator (restated from mh_gen_limb) ------------------------- */
static uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static void gen_row(uint64_t seed, uint32_t n_vars, uint64_t index, uint32_t* a) {
    for (uint32_t v = 0; v < n_vars; ++v)
        for (uint32_t k = 0; k < 8; ++k) {
            uint64_t key = splitmix64(seed ^ (((uint64_t)v * 8 + k) * 0xD1B54A32D192ED03ull));
            a[v * 8 + k] = (uint32_t)splitmix64(key ^ index);
        }
}

/* Per-tape hit counts and first witnesses over generated rows [row_first, row_first+rows),
 * evaluated on `threads` OpenMP threads.  Returns 0 or -1. */
static int count_rows(const node_t* nodes, const uint64_t* offs, uint32_t n_tapes,
                      const uint32_t* consts, uint32_t n_consts, uint32_t n_vars, uint64_t seed,
                      uint64_t row_first, uint64_t rows, int threads, uint64_t* count,
                      uint64_t* first, int short_circuit) {
    int err = 0;
    for (uint32_t t = 0; t < n_tapes; ++t) { count[t] = 0; first[t] = ~0ull; }
#pragma omp parallel num_threads(threads)
    {
        uint32_t* a = (uint32_t*)malloc(sizeof(uint32_t) * 8 * (n_vars ? n_vars : 1));
        uint64_t* lc = (uint64_t*)calloc(n_tapes ? n_tapes : 1, sizeof(uint64_t));
        uint64_t* lf = (uint64_t*)malloc(sizeof(uint64_t) * (n_tapes ? n_tapes : 1));
        for (uint32_t t = 0; t < n_tapes; ++t) lf[t] = ~0ull;
        uint32_t out[NL];
#pragma omp for schedule(dynamic, 64)
        for (int64_t r = 0; r < (int64_t)rows; ++r) {
            const uint64_t idx = row_first + (uint64_t)r;
            gen_row(seed, n_vars, idx, a);
            for (uint32_t t = 0; t < n_tapes; ++t) {
                const int rc = short_circuit
                    ? ct_eval_lazy(nodes + offs[t], offs[t + 1] - offs[t], consts, n_consts, a,
                                   n_vars, out)
                    : ct_eval(nodes + offs[t], offs[t + 1] - offs[t], consts, n_consts, a, n_vars,
                              out);
                if (rc != 0) {
                    err = 1;
                    continue;
                }
                int nz = 0;
                for (int k = 0; k < NL; ++k) nz |= out[k] != 0;
                if (nz) {
                    lc[t]++;
                    if (idx < lf[t]) lf[t] = idx;
                }
            }
        }
#pragma omp critical
        for (uint32_t t = 0; t < n_tapes; ++t) {
            count[t] += lc[t];
            if (lf[t] < first[t]) first[t] = lf[t];
        }
        free(a);
        free(lc);
        free(lf);
    }
    return err ? -1 : 0;
}

int ct_count(const node_t* nodes, const uint64_t* offs, uint32_t n_tapes, const uint32_t* consts,
             uint32_t n_consts, uint32_t n_vars, uint64_t seed, uint64_t row_first,
             uint64_t rows, int threads, uint64_t* count, uint64_t* first) {
    return count_rows(nodes, offs, n_tapes, consts, n_consts, n_vars, seed, row_first, rows,
                      threads, count, first, 0);
}

/* The same counts with short-circuit evaluation of Bool ANDs (ct_eval_lazy). */
int ct_count_lazy(const node_t* nodes, const uint64_t* offs, uint32_t n_tapes,
                  const uint32_t* consts, uint32_t n_consts, uint32_t n_vars, uint64_t seed,
                  uint64_t row_first, uint64_t rows, int threads, uint64_t* count,
                  uint64_t* first) {
    return count_rows(nodes, offs, n_tapes, consts, n_consts, n_vars, seed, row_first, rows,
                      threads, count, first, 1);
}

int ct_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
