/*
 * mythril_hip.h — C-ABI of libmythril_hip, the MI355X constraint sieve for Mythril's LASER engine.
 *
 * The sieve evaluates path-constraint "tapes" (flattened z3 QF_BV/Bool terms, see §Tape IR) against
 * millions of candidate assignments resident in HBM and reports, per tape, the smallest satisfying
 * assignment index (a witness) and/or the number of satisfying assignments.  It replaces, for the
 * SAT-by-witness case only, the z3 round trip behind
 *     mythril/support/model.py:15-62            get_model(constraints, minimize=(), maximize=(), ...)
 *     mythril/laser/smt/model.py:45-59          Model.eval(expression, model_completion=True)
 *     mythril/laser/smt/solver/solver.py:47-64  BaseSolver.check / BaseSolver.model
 * (reference = terasum/mythril v0.22.9).  Every entry point below is what a Python ctypes binding in
 * the reference would bind.  Conventions:
 *   - C linkage, plain pointers and sizes, no exceptions cross the ABI, the library never aborts;
 *   - every function returns int32: MH_OK (0) or a negative MH_E_* code; mh_last_error() gives text;
 *   - the caller owns host buffers; the library owns device memory behind opaque handles;
 *   - entry points are re-entrant per handle (one ctx per thread / per GPU).
 */
#ifndef MYTHRIL_HIP_H
#define MYTHRIL_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MH_VERSION_MAJOR 0
#define MH_VERSION_MINOR 1
#define MH_VERSION_PATCH 0

/* ---- error codes ------------------------------------------------------------------------------ */
enum {
    MH_OK = 0,
    MH_E_INVALID = -1,      /* bad argument / malformed tape                                     */
    MH_E_UNSUPPORTED = -2,  /* tape uses a feature the device path does not cover (fall back to z3) */
    MH_E_DEVICE = -3,       /* HIP runtime error                                                 */
    MH_E_NOMEM = -4,        /* host or device allocation failed                                  */
    MH_E_NODEVICE = -5      /* no gfx950 device visible                                          */
};

/* ---- Tape IR ----------------------------------------------------------------------------------
 * A tape is a topologically ordered list of nodes (each node's operands are earlier nodes of the
 * same tape, by tape-local index); the last node is the root.  Sort: width == 0 means Bool, width
 * in 1..512 means a bit-vector of that many bits.  Node semantics are SMT-LIB QF_BV (as z3's
 * model_completion evaluator implements them), plus three EVM-word helpers (MH_OP_EVM_*) and the
 * Keccak-256 hash.  The op -> reference-construction map is in DESIGN.md §Tape IR.             */
enum mh_op {
    MH_OP_CONST = 0,   /* imm0 = const-pool index                   (symbol_factory.BitVecVal)   */
    MH_OP_VAR = 1,     /* imm0 = assignment column; low `width` bits (symbol_factory.BitVecSym)  */
    MH_OP_TRUE = 2,    /* Bool true                                  (symbol_factory.Bool)       */
    MH_OP_FALSE = 3,   /* Bool false                                                            */
    MH_OP_BVADD = 10, MH_OP_BVSUB = 11, MH_OP_BVMUL = 12,
    MH_OP_BVUDIV = 13, MH_OP_BVUREM = 14, MH_OP_BVSDIV = 15, MH_OP_BVSREM = 16, MH_OP_BVSMOD = 17,
    MH_OP_BVNEG = 18, MH_OP_BVNOT = 19,
    MH_OP_BVAND = 20, MH_OP_BVOR = 21, MH_OP_BVXOR = 22,
    MH_OP_BVSHL = 23, MH_OP_BVLSHR = 24, MH_OP_BVASHR = 25,    /* a = value, b = shift amount    */
    MH_OP_EQ = 30,                                               /* bv or Bool operands -> Bool   */
    MH_OP_BVULT = 31, MH_OP_BVULE = 32, MH_OP_BVUGT = 33, MH_OP_BVUGE = 34,
    MH_OP_BVSLT = 35, MH_OP_BVSLE = 36, MH_OP_BVSGT = 37, MH_OP_BVSGE = 38,
    MH_OP_AND = 40, MH_OP_OR = 41, MH_OP_XOR = 42, MH_OP_NOT = 43,
    MH_OP_ITE = 45,                                              /* a = Bool cond, b = then, c = else */
    MH_OP_EXTRACT = 50,                                          /* imm0 = hi, imm1 = lo          */
    MH_OP_CONCAT = 51,                                           /* a = high part, b = low part   */
    MH_OP_ZEXT = 52, MH_OP_SEXT = 53,                            /* imm0 = extra bits             */
    MH_OP_KECCAK = 60,        /* Keccak-256 of the big-endian bytes of a (width % 8 == 0) -> 256 */
    MH_OP_BVADD_NOOVFL_U = 61,  /* z3.BVAddNoOverflow(a, b, False) -> Bool                        */
    MH_OP_BVMUL_NOOVFL_U = 62,  /* z3.BVMulNoOverflow(a, b, False) -> Bool                        */
    MH_OP_BVSUB_NOUDFL_U = 63,  /* z3.BVSubNoUnderflow(a, b, False) -> Bool  (b <=u a)            */
    MH_OP_EVM_EXP = 70,       /* a ** b mod 2^width                                               */
    MH_OP_EVM_SIGNEXTEND = 71,/* a = byte index k, b = x (yellow-paper SIGNEXTEND)                 */
    MH_OP_EVM_BYTE = 72,      /* a = byte index i, b = x (yellow-paper BYTE)                       */
    MH_OP_EVM_ADDMOD = 73,    /* (a + b) mod c, exact sum (yellow-paper ADDMOD); c == 0 gives 0, or */
    MH_OP_EVM_MULMOD = 74     /* (a * b) mod c ...  with imm0 = 1 the low 256 bits of a op b: the
                                 value of z3's extract[255:0](bvurem(zext a op zext b, zext c)),
                                 a shape mh_tapes_compile also recognises and rewrites to these */
};

typedef struct mh_node {
    uint8_t op;      /* enum mh_op                                   */
    uint8_t flags;   /* reserved, must be 0                          */
    uint16_t width;  /* 0 = Bool, else bit-vector width 1..512       */
    uint32_t a, b, c;        /* operand node indices (tape-local)    */
    uint32_t imm0, imm1;     /* op immediates                        */
} mh_node;                   /* 24 bytes, little-endian              */

/* Evaluation modes for mh_run*. */
enum {
    MH_MODE_FIRST_HIT = 0,   /* per tape: smallest satisfying assignment index (early exit allowed) */
    MH_MODE_COUNT_ALL = 1    /* per tape: number of satisfying assignments AND smallest index;       */
                             /*           every (tape, assignment) pair's Bool is determined: no   */
                             /*           early exit across assignments (the native code may stop  */
                             /*           a wave's evaluation once every row of it has a false     */
                             /*           conjunct -- counts and indices are the same)              */
};
#define MH_NO_HIT 0xFFFFFFFFFFFFFFFFull

typedef struct mh_ctx mh_ctx;           /* one device + one stream                                */
typedef struct mh_tapeset mh_tapeset;   /* compiled tapes + const pool, resident on the device    */
typedef struct mh_assign mh_assign;     /* assignments, SoA u32 limbs, resident on the device     */

/* Per-tape compile statistics returned by mh_tapes_info. */
typedef struct mh_tape_info {
    uint32_t n_nodes;        /* IR nodes                                                          */
    uint32_t n_insns;        /* device instructions after legalisation                            */
    uint32_t n_regs;         /* peak registers used (of MH_NUM_REGS)                              */
    uint32_t features;       /* bit 0: division family, bit 1: keccak, bit 2: EVM_EXP             */
    uint64_t alg_ops;        /* SURVEY.md §8(d)'s op-cost table summed over the tape (1100 per
                                division, ...): a reporting figure, not a work count -- the
                                roofline prices a code-independent minimum     */
} mh_tape_info;

/* ---- library / device ------------------------------------------------------------------------ */
int32_t mh_version(uint32_t* major, uint32_t* minor, uint32_t* patch);
const char* mh_last_error(void);                       /* thread-local; never NULL               */
int32_t mh_device_count(int32_t* n);                   /* gfx950 devices visible                 */

int32_t mh_ctx_create(int32_t device, mh_ctx** out);
/* Releases the handle.  Tape sets and assignment buffers created from it keep it alive: its
 * device memory, stream and communicator are freed when the last of them is destroyed (so the
 * destroy order of handles never matters).  Destroying a ctx twice is MH_E_INVALID.             */
int32_t mh_ctx_destroy(mh_ctx* ctx);
/* Launch on an external HIP stream (e.g. torch.cuda.current_stream().cuda_stream; 0/NULL is the
 * null stream).  The ctx starts on a stream of its own.                                          */
int32_t mh_ctx_set_stream(mh_ctx* ctx, void* hip_stream);
int32_t mh_ctx_synchronize(mh_ctx* ctx);
/* mh_tapes_compile keeps each compiled tape by content (nodes, constant values, column count)
 * for the ctx's later compiles, up to 16M instruction words (MH_COMPILE_CACHE=0: off).  This drops
 * them (memory, or a measurement that must not reuse an earlier query's code).                   */
int32_t mh_ctx_clear_cache(mh_ctx* ctx);

/* ---- tapes ----------------------------------------------------------------------------------- */
/* nodes: all tapes concatenated; tape_offsets[n_tapes+1] delimit them (node indices).
 * consts: n_consts x 8 u32 limbs (little-endian limb order, 256-bit entries).
 * n_vars: number of assignment columns the tapes may reference.                                 */
int32_t mh_tapes_compile(mh_ctx* ctx, const mh_node* nodes, const uint64_t* tape_offsets,
                         uint32_t n_tapes, const uint32_t* consts, uint32_t n_consts,
                         uint32_t n_vars, mh_tapeset** out);
/* The same on a worker thread of the context, so the caller's other host work (the guide harvest,
 * mh_guide_harvest_with) runs meanwhile: returns at once; mh_tapes_compile_wait gives what
 * mh_tapes_compile would have.  The arrays must stay valid, and the caller makes no other call on
 * this context, until the wait; one compile at a time per context.                               */
int32_t mh_tapes_compile_async(mh_ctx* ctx, const mh_node* nodes, const uint64_t* tape_offsets,
                               uint32_t n_tapes, const uint32_t* consts, uint32_t n_consts,
                               uint32_t n_vars);
int32_t mh_tapes_compile_wait(mh_ctx* ctx, mh_tapeset** out,
                              double* compile_s /* the compile's own seconds, or NULL */);
int32_t mh_tapes_destroy(mh_tapeset* ts);
int32_t mh_tapes_info(const mh_tapeset* ts, mh_tape_info* info /* [n_tapes] */, uint32_t n_tapes);

/* ---- assignments ----------------------------------------------------------------------------- */
/* Layout in HBM: column v, limb k (0 = least significant) of assignment i is word
 * ((v * 8 + k) * stride + i), stride = capacity + a few padding rows (library-internal: the
 * device memory is only reached through these calls).  Every column is a 256-bit word.          */
int32_t mh_assign_create(mh_ctx* ctx, uint32_t n_vars, uint64_t capacity, mh_assign** out);
int32_t mh_assign_destroy(mh_assign* as);
/* host_soa has the same layout with `count` in place of capacity; fills [first, first+count).   */
int32_t mh_assign_upload(mh_assign* as, const uint32_t* host_soa, uint64_t first, uint64_t count);
int32_t mh_assign_download(const mh_assign* as, uint32_t* host_soa, uint64_t first, uint64_t count);
/* Fill all `capacity` rows from the counter-based generator: row i of this buffer gets the value
 * mh_gen_word(seed, v, global_base + i) (see mh_gen_limb).                                       */
int32_t mh_assign_generate(mh_assign* as, uint64_t seed, uint64_t global_base);
/* Host reference of the generator (same bits as the device kernel).                             */
uint32_t mh_gen_limb(uint64_t seed, uint32_t var, uint64_t index, uint32_t limb);

/* Guided candidates for one query (mythril_amd/candidates.py harvests the guide from the query's
 * terms; SURVEY.md §8f "candidate generation").  Row r in [first, first+count) gets global index
 * g = global_base + r and, for column v < n_cols (width w_v, value pool P_v):
 *     m0 = mh_gen_limb(seed ^ 0x6A09E667F3BCC909, v, g, 0), m1 = the same with limb 1;
 *     (m0 & 0xff) <  64               -> (m0 >> 8) & 0xff                        small
 *     (m0 & 0xff) < 128 or P_v empty  -> limbs mh_gen_limb(seed, v, g, k)        uniform
 *     otherwise                       -> P_v[m1 % |P_v|]                         pool
 * masked to w_v bits.  Then, for each set j in order, with s = mh_gen_limb(seed ^
 * 0xBB67AE8584CAA73B, j, g, 0): if (s & 0xff) < set_prob[j] and the set has alternatives,
 * alternative set_off[j] + (s >> 8) % n_alt is applied: each of its entries writes its value
 * (masked) into column entry_col, or, when entry_col has bit 31 set (MH_GUIDE_COPY), copies bits
 * [src_lo, src_lo + nbits) of column src into bits [dst_lo, dst_lo + nbits) of the destination,
 * with entry_val limbs = {src, dst_lo, src_lo, nbits, 0, 0, 0, 0}.  Later sets override earlier
 * ones.  Columns n_cols.. of the buffer are left untouched.                                     */
#define MH_GUIDE_COPY 0x80000000u
typedef struct mh_guide {
    uint32_t n_cols;             /* columns generated (<= the buffer's n_vars)                   */
    const uint16_t* col_width;   /* [n_cols] 1..256                                              */
    const uint32_t* pool_off;    /* [n_cols + 1] value ranges of `pool`                          */
    const uint32_t* pool;        /* [pool_off[n_cols]] x 8 limbs                                 */
    uint32_t n_sets;
    const uint8_t* set_prob;     /* [n_sets] probability in 1/256                                */
    const uint32_t* set_off;     /* [n_sets + 1] alternative ranges                              */
    const uint32_t* alt_off;     /* [set_off[n_sets] + 1] entry ranges                           */
    const uint32_t* entry_col;   /* [alt_off[set_off[n_sets]]] column, or MH_GUIDE_COPY | dst    */
    const uint32_t* entry_val;   /* x 8 limbs                                                    */
} mh_guide;
int32_t mh_assign_generate_guided(mh_assign* as, uint64_t seed, uint64_t global_base,
                                  uint64_t first, uint64_t count, const mh_guide* guide);

/* Host-only: harvest the guide of one query from its lowered tape (the algorithm of
 * mythril_amd/candidates.py, same arrays; no device is touched).  `nodes` is ONE tape whose root
 * (last node) is the query's Bool path condition, VAR imm0 = column 0..n_cols-1, CONST imm0 =
 * index into `consts` (n_consts x 8 limbs).  The parent query's witness (svm.py:257-262) is
 * n_parent (column, value) pairs, value = 8 limbs, in the witness's order; n_parent = 0 for none.
 * On MH_OK *guide points into *out, which owns the arrays until mh_harvest_free(*out).
 * Replaces the Python harvest behind mythril_amd/candidates.build_guide for Sieve.solve.         */
typedef struct mh_harvest mh_harvest;
int32_t mh_guide_harvest(const mh_node* nodes, uint32_t n_nodes, const uint32_t* consts,
                         uint32_t n_consts, const uint16_t* col_width, uint32_t n_cols,
                         const uint32_t* parent_cols, const uint32_t* parent_vals,
                         uint32_t n_parent, mh_harvest** out, mh_guide* guide);
/* mh_guide_harvest for the incremental round (sieve.newest_tape: the conjuncts a query adds to its
 * parent's): an operand every column of which the parent witness fixes, built from the bit-layout
 * and linear ops, counts as known beside constants when the other side of an arithmetic op, an
 * equality or a comparison is solved for -- so `x + y == k` proposes x = k - y(parent) where the
 * plain harvest proposes nothing.  Stateless; the same arrays as candidates.build_guide(...,
 * parent_eval=True).                                                                           */
int32_t mh_guide_harvest_inc(const mh_node* nodes, uint32_t n_nodes, const uint32_t* consts,
                             uint32_t n_consts, const uint16_t* col_width, uint32_t n_cols,
                             const uint32_t* parent_cols, const uint32_t* parent_vals,
                             uint32_t n_parent, mh_harvest** out, mh_guide* guide);
int32_t mh_harvest_free(mh_harvest* h);
/* The same harvest by a session kept across a path's queries: when the tape, the constants and
 * the column widths extend the last call's (a LASER child whose new constraint left its parent's
 * lowering unchanged: mh_query_build then emits the parent's tape as a prefix), the memoised
 * inversions of the earlier conjuncts are reused and only the new ones are computed; otherwise the
 * session starts afresh.  The guide is the one mh_guide_harvest gives for the same arguments.
 * mh_harvester_stats: [calls that extended, calls that started afresh, arena bytes held].         */
typedef struct mh_harvester mh_harvester;
int32_t mh_harvester_create(mh_harvester** out);
int32_t mh_harvester_destroy(mh_harvester* s);
int32_t mh_harvester_stats(const mh_harvester* s, uint64_t* out /* [3] */);
int32_t mh_guide_harvest_with(mh_harvester* s, const mh_node* nodes, uint32_t n_nodes,
                              const uint32_t* consts, uint32_t n_consts, const uint16_t* col_width,
                              uint32_t n_cols, const uint32_t* parent_cols,
                              const uint32_t* parent_vals, uint32_t n_parent, mh_harvest** out,
                              mh_guide* guide);

/* ---- SMT-LIB import (the product path's first stage) -----------------------------------------
 * Replaces the Python SMT-LIB reader behind mythril_amd/smtlib.Z3Importer, which imports every
 * constraint LASER hands get_model (mythril/support/model.py:37-57; laser/smt/solver/solver.py:
 * 28-37) from z3's Solver.sexpr() text.  A session reads SMT-LIB2 commands (declare-fun,
 * declare-const, define-fun, assert, minimize, maximize; let, n-ary connectives, indexed
 * operators, select / store / (as const ..), unary uninterpreted functions) and hash-conses the
 * terms against the nodes it has already handed to the host.  mh_smtlib_read returns only the
 * nodes the host does not have yet, in creation order (operands: a host id >= 0, or -(k + 1) for
 * record k of the same batch), and one result per assert / minimize / maximize (the same
 * reference form).  The host builds each record in its own term store and must answer with
 * mh_smtlib_commit (the host id of every record) or mh_smtlib_rollback before the next read.
 * Batch arrays stay valid until the next read.  Malformed text: MH_E_INVALID, nothing changes.    */
typedef struct mh_smtlib mh_smtlib;
typedef struct {
    uint8_t op;           /* mh_op, or the host-only kinds 80..84 (ARRAY, CONST_ARRAY, STORE,
                             SELECT, UF: imm1 = domain width, width = range width)               */
    uint8_t pad0;
    uint16_t pad1;
    uint32_t width;       /* 0 = Bool                                                            */
    int64_t a, b, c;      /* operands (only the op's arity is meaningful)                         */
    uint32_t imm0, imm1;  /* EXTRACT hi / lo, ZEXT / SEXT bits; arrays / UFs: imm1 = domain       */
    uint32_t name_off, name_len;  /* VAR / ARRAY / UF: symbol name in batch.names                */
    uint32_t const_off;   /* CONST: 8 little-endian u32 limbs at batch.const_limbs[const_off]    */
    uint32_t pad2;
} mh_smt_record;
enum { MH_SMT_ASSERT = 0, MH_SMT_MINIMIZE = 1, MH_SMT_MAXIMIZE = 2 };
typedef struct {
    uint32_t kind;        /* MH_SMT_ASSERT / MINIMIZE / MAXIMIZE                                 */
    uint32_t pad;
    int64_t node;         /* host id, or -(k + 1) for record k                                    */
} mh_smt_result;
typedef struct {
    const mh_smt_record* records;
    uint64_t n_records;
    const uint32_t* const_limbs;
    const char* names;
    const mh_smt_result* results;
    uint64_t n_results;
} mh_smt_batch;
int32_t mh_smtlib_create(mh_smtlib** out);
int32_t mh_smtlib_destroy(mh_smtlib* s);
int32_t mh_smtlib_read(mh_smtlib* s, const char* text, uint64_t len, mh_smt_batch* out);
int32_t mh_smtlib_commit(mh_smtlib* s, const int64_t* host_ids, uint64_t n);
int32_t mh_smtlib_rollback(mh_smtlib* s);
uint64_t mh_smtlib_size(const mh_smtlib* s);  /* nodes the session mirrors                      */

/* ---- query compiler (the host stages of one get_model query) ---------------------------------
 * Replaces the Python stages behind mythril_amd/sieve.py Sieve.solve for a query: lower_query
 * (mythril_amd/lower.py: arrays, store chains, keccak and other uninterpreted functions onto
 * scalar columns), Sieve.bucket_roots (the DependenceMap of laser/smt/solver/
 * independence_solver.py:38-83 over the lowered columns) and local_tapeset (one device tape per
 * group over the query's own columns and constants).  An mh_terms session mirrors the host's
 * hash-consed term store (tape.py TapeBuilder); mh_terms_append hands it the nodes (flags
 * included: F_ARRAY 1, F_HOST 2; host-only kinds 80..84 as in mh_smt_record), the constant pool
 * entries (8 limbs each) and the variable / array / function names (NUL-terminated, back to back,
 * numbered in order) the host made since the last call.  mh_query_build compiles the conjunction
 * of `roots`: tape 0 is the root (the guide's input, mh_guide_harvest); with n_groups > 1 tapes
 * 1..n_groups are the column-disjoint groups in order of their first conjunct, with n_groups == 1
 * tape 0 is the one group's.  VAR imm0 = column (0..n_columns-1), CONST imm0 = constant
 * (0..n_consts-1).  A ground query has one Bool column "__ground__" no tape reads.  flags
 * MH_QUERY_DEFINITIONS: conjuncts of the shape variable == computed term over other columns were
 * eliminated (sieve.py eliminate_definitions): the defined variables are substituted away, the
 * root and group tapes are the remaining conjunction's, and one more tape per definition (the
 * last n_defs) computes the defined column's value from the witness row.  Constructs the
 * lowering does not model are MH_E_UNSUPPORTED
 * (the query goes to z3).  A session is used by one thread at a time.                            */
typedef struct mh_terms mh_terms;
typedef struct mh_query mh_query;
/* column kinds; a read (MH_COL_READ / MH_COL_UFREAD: an array's / a tabled function's value at a
 * symbolic index term, Ackermann's reduction; MH_COL_KREAD: a keccak application's value, made
 * only under MH_TERMS_KECCAK_READS) carries the index term's node id as its key                 */
enum { MH_COL_VAR = 0, MH_COL_CELL = 1, MH_COL_ELSE = 2, MH_COL_UFCELL = 3, MH_COL_UFELSE = 4,
       MH_COL_READ = 5, MH_COL_UFREAD = 6, MH_COL_KREAD = 7 };
enum { MH_TABLE_CELLS = 0, MH_TABLE_UF_CELLS = 1, MH_TABLE_KECCAK = 2 };
#define MH_QUERY_DEFINITIONS 1u
#define MH_QUERY_REFUTED 2u     /* the conjunction contradicts itself syntactically (a FALSE
                                   conjunct, a conjunct and its negation, a term pinned to an
                                   empty range by equalities / disequalities / unsigned bounds
                                   against constants): no witness exists                       */
#define MH_QUERY_INCREMENTAL 4u /* diagnostic: built from the session's state (taken back to the
                                   common prefix of the roots and extended by the rest) rather
                                   than afresh; the result is the same either way               */
#define MH_QUERY_KEY_LIMBS 36  /* limbs of a table entry / cell key (1152 bits; keccak arguments are
                                   up to 1088 bits wide)                                        */
typedef struct {
    uint32_t name_off, name_len;      /* column name in info.names ("x", "A[0x4]", "A[*]")         */
    uint32_t symbol_off, symbol_len;  /* variable / array / function name                          */
    uint32_t width;
    uint32_t kind;                    /* MH_COL_*                                                  */
    uint32_t key_off;                 /* cells: key = MH_QUERY_KEY_LIMBS limbs at key_limbs[
                                         MH_QUERY_KEY_LIMBS * key_off]; else ~0u                  */
    uint32_t pad;
} mh_query_column;                    /* 32 bytes                                                  */
typedef struct {
    uint32_t kind;                    /* MH_TABLE_*                                                */
    uint32_t name_off, name_len;      /* array / function name in info.names                       */
    uint32_t limb_off;                /* first entry in table_limbs (MH_QUERY_KEY_LIMBS limbs each)  */
    uint32_t n_items;                 /* CELLS: n_items keys (ascending, every harvested key);
                                         KECCAK: the interval base, then n_items (argument, hash)
                                         pairs                                                     */
    uint32_t pad;
} mh_query_table;                     /* 24 bytes                                                  */
typedef struct {
    const mh_node* nodes;             /* every tape, back to back                                  */
    const uint64_t* tape_off;         /* [n_tapes + 1]                                             */
    const uint32_t* consts;           /* [n_consts][8]                                             */
    const mh_query_column* columns;
    const char* names;
    const uint32_t* key_limbs;
    const uint32_t* group_cols;       /* the columns of group g: group_cols[group_off[g] ..        */
    const uint32_t* group_off;        /*   group_off[g + 1]), ascending; [n_groups + 1]            */
    const mh_query_table* tables;
    const uint32_t* table_limbs;
    uint32_t n_tapes, n_consts, n_columns, names_len, n_groups, n_tables, flags;
    uint32_t n_keys;                  /* entries of key_limbs                                      */
    uint32_t n_table_entries;         /* entries of table_limbs                                    */
    uint32_t n_defs;                  /* MH_QUERY_DEFINITIONS: definitions eliminated; the last
                                         n_defs tapes are their terms, the root and group tapes
                                         come first (n_tapes - n_defs of them)                     */
    const uint32_t* def_cols;         /* [n_defs]: the column each definition tape's value gives   */
    uint32_t parent_len;              /* nodes of the root tape that are the tape of the query
                                         without its last root (it is linearised root by root, so
                                         they come first; 0 with one root or definitions): the
                                         nodes at or past it are the newest root's conjuncts    */
    const uint32_t* root_ends;        /* [n_root_ends]: entry d - 1 = nodes of the root tape that are
                                         the tape of the first d roots (d < n_roots; none with
                                         definitions); the last entry is parent_len               */
    uint32_t n_root_ends;
} mh_query_info;
int32_t mh_terms_create(mh_terms** out);
int32_t mh_terms_destroy(mh_terms* t);
/* Session options (lower.py lower_query's keyword arguments; the session's query state is dropped).
 * MH_TERMS_KECCAK_READS: every keccak256_N application is a read column of its own (MH_COL_KREAD)
 * under the stated pairs' ite chain instead of the fixed H(x) = base + ((keccak(x) >> 139) << 6),
 * kept a function and injective by conjuncts (lower.py Lowering._keccak_read / congruence): the
 * sieve's second chance for a query whose keccak values the query pins elsewhere than H.
 * Replaces the reference's keccak_function_manager.py:80-113 hash model for that query.        */
#define MH_TERMS_KECCAK_READS 1u
int32_t mh_terms_set_options(mh_terms* t, uint32_t options);
int32_t mh_terms_append(mh_terms* t, const mh_node* nodes, uint64_t n_nodes,
                        const uint32_t* consts, uint64_t n_consts, const char* var_names,
                        uint64_t n_vars, const char* array_names, uint64_t n_arrays,
                        const char* fn_names, uint64_t n_fns);
/* nodes, constants, variables, arrays, functions the session holds                                */
int32_t mh_terms_sizes(const mh_terms* t, uint64_t* out /* [5] */);
/* On MH_OK *info points into *out, which owns the arrays until mh_query_free(*out).              */
int32_t mh_query_build(mh_terms* t, const uint32_t* roots, uint32_t n_roots, mh_query** out,
                       mh_query_info* info);
int32_t mh_query_free(mh_query* q);

/* ---- evaluation ------------------------------------------------------------------------------ */
/* Evaluate tapes [tape_first, tape_first+tape_count) over assignment rows [row_first,
 * row_first+row_count) of `as`.  Results are indexed by tape - tape_first and hold GLOBAL indices
 * (index_base + row).  Host-pointer form: blocks until done.                                      */
int32_t mh_run(mh_ctx* ctx, const mh_tapeset* ts, uint32_t tape_first, uint32_t tape_count,
               const mh_assign* as, uint64_t row_first, uint64_t row_count, uint64_t index_base,
               uint32_t mode, uint64_t* first_hit /* [tape_count] or NULL */,
               uint64_t* hit_count /* [tape_count] or NULL */);
/* mh_run plus each tape's witness row: rows_out [tape_count][n_cols][8] u32 receives columns
 * 0..n_cols-1 (n_cols <= the buffer's columns) of the row first_hit names, all zero for a tape
 * without a hit -- the model get_model returns (support/model.py:15-62) read back in the same
 * device-to-host copy as the results instead of one mh_assign_download per distinct row.        */
int32_t mh_run_rows(mh_ctx* ctx, const mh_tapeset* ts, uint32_t tape_first, uint32_t tape_count,
                    const mh_assign* as, uint64_t row_first, uint64_t row_count,
                    uint64_t index_base, uint32_t mode, uint64_t* first_hit, uint64_t* hit_count,
                    uint32_t n_cols, uint32_t* rows_out);
/* One guided round of a query in one call: mh_assign_generate_guided of rows [0, count) of `as`
 * (global indices global_base + row) then mh_run_rows over them with index_base = global_base --
 * the sieve's round (Sieve.solve) without a host round trip between the generator and the run.   */
int32_t mh_query_round(mh_ctx* ctx, const mh_tapeset* ts, mh_assign* as, const mh_guide* guide,
                       uint64_t seed, uint64_t global_base, uint64_t count, uint32_t tape_first,
                       uint32_t tape_count, uint32_t mode, uint64_t* first_hit,
                       uint64_t* hit_count, uint32_t n_cols, uint32_t* rows_out);
/* Device-pointer form: enqueues on the ctx stream and returns.  d_first_hit / d_hit_count are
 * device buffers of tape_count u64; they are NOT reset (callers initialise them to MH_NO_HIT / 0
 * with mh_results_reset), so several launches can accumulate into them.                          */
int32_t mh_results_reset(mh_ctx* ctx, uint64_t* d_first_hit, uint64_t* d_hit_count, uint32_t n);
int32_t mh_run_async(mh_ctx* ctx, const mh_tapeset* ts, uint32_t tape_first, uint32_t tape_count,
                     const mh_assign* as, uint64_t row_first, uint64_t row_count,
                     uint64_t index_base, uint32_t mode, uint64_t* d_first_hit,
                     uint64_t* d_hit_count);
/* Parity path: the root value of tape `tape` for rows [row_first, row_first+row_count):
 * out[(k * row_count) + r] = limb k of the root value (Bool roots: 0/1 in limb 0).  Roots wider
 * than 256 bits are MH_E_UNSUPPORTED.  Blocks until done.                                         */
int32_t mh_eval_values(mh_ctx* ctx, const mh_tapeset* ts, uint32_t tape, const mh_assign* as,
                       uint64_t row_first, uint64_t row_count, uint32_t* out /* [8*row_count] */);

/* Batched parity path (Model.eval, laser/smt/model.py:45-59, read in loops by the reference:
 * calldata.py:240-245 evaluates one byte term per call): the root values of the `n` listed tapes
 * at ONE row of `as`, out[8 * i + k] = limb k of tapes[i]'s root.  One kernel launch per
 * register-class variant among the listed tapes (usually one), one copy back, one sync.       */
int32_t mh_eval_values_many(mh_ctx* ctx, const mh_tapeset* ts, const uint32_t* tapes, uint32_t n,
                            const mh_assign* as, uint64_t row, uint32_t* out /* [8*n] */);
/* Kernel launches mh_eval_values_many has made on this context (a test / latency counter).     */
int32_t mh_ctx_eval_launches(const mh_ctx* ctx, uint64_t* launches);

/* ---- measurement ----------------------------------------------------------------------------- */
/* ---- native-code path (no reference counterpart: replaces the interpreter for throughput runs)
 * mh_tapes_jit compiles every tape of the set that the JIT covers to gfx950 machine code -- one
 * code object per slice of tape groups, assembled in-process by comgr and loaded with
 * hipModuleLoadData (mythril_amd/csrc/jit.cpp).  Covered: every op of the IR (the EVM word ops,
 * ADDMOD / MULMOD and the overflow predicates are restated on native operations; EXP and
 * MULMOD by a per-lane operand run as loops), any number of assignment columns (up to 4 are held
 * in registers for a whole 64-row chunk, above that each tape loads the limbs it uses); a tape is
 * refused only when its code exceeds 96 KB or its registers 168 VGPRs (mh_tapes_jitted tells).
 * Afterwards mh_run / mh_run_async over the whole tape set run the jitted tapes through that code
 * and the rest through the interpreter; results are identical.  flags: MH_JIT_VALUES also builds
 * the values kernel behind mh_jit_eval_all; MH_JIT_FULL_EVAL turns off short-circuit evaluation
 * of root conjunctions (by default a wave leaves a tape once no row of its 64 satisfies the
 * conjuncts evaluated so far -- the results are the same either way; the environment variable
 * MH_JIT_SC=0 does the same).  max_vgpr: register budget per wave, 96..256 (occupancy =
 * min(8, 512 / max_vgpr) waves per SIMD), 0 = default 128.  Cost: a few seconds per thousand
 * tapes, once per tape set, outside any timed region.                                            */
#define MH_JIT_VALUES 1u
#define MH_JIT_FULL_EVAL 2u
typedef struct mh_jit_info {
    uint32_t n_jitted;         /* tapes on the native path                                        */
    uint32_t n_groups;         /* tape groups (grid rows of the JIT kernels)                      */
    uint32_t n_modules;        /* code objects                                                    */
    uint32_t max_vgpr;         /* VGPRs per wave of the JIT kernels                               */
    uint64_t code_bytes;       /* machine code, all code objects                                  */
    uint64_t valu_static;      /* static VALU instructions over the jitted tapes (division calls
                                  not expanded)                                                   */
    uint64_t valu_wide_static; /* ... of them in the 4-cycle class (VOP3, carry / compare writes) */
    double build_ms;           /* emission + assembly + load                                      */
} mh_jit_info;
int32_t mh_tapes_jit(mh_tapeset* ts, uint32_t flags, uint32_t max_vgpr);
int32_t mh_tapes_jit_info(const mh_tapeset* ts, mh_jit_info* out);
/* Identifier of the native code mh_tapes_jit built: FNV-1a 64 over its code objects' module texts
 * (count kernels, in launch order).  Profiles of the emitted code are keyed by it, so a host-only
 * change (capi.cpp, the query path) keeps them valid.  mh_jit_code_id computes the same value
 * WITHOUT a device or the assembler (emission only), from the arguments mh_tapes_compile takes and
 * mh_tapes_jit's flags / max_vgpr (the tapes are validated as mh_tapes_compile does).             */
int32_t mh_tapes_jit_code_id(const mh_tapeset* ts, uint64_t* out);
int32_t mh_jit_code_id(const mh_node* nodes, const uint64_t* tape_offsets, uint32_t n_tapes,
                       const uint32_t* consts, uint32_t n_consts, uint32_t n_vars,
                       uint32_t flags, uint32_t max_vgpr, uint64_t* out);
/* 1 if tape t runs on the native path.                                                           */
int32_t mh_tapes_jitted(const mh_tapeset* ts, uint8_t* out /* [n_tapes] */, uint32_t n_tapes);
/* Parity path of the native code: root values of every jitted tape over rows
 * [row_first, row_first + row_count), out = [n_tapes][8][row_count] u32 (slots of tapes not on
 * the native path are left untouched).  Needs mh_tapes_jit(ts, MH_JIT_VALUES, ...).              */
int32_t mh_jit_eval_all(mh_ctx* ctx, const mh_tapeset* ts, const mh_assign* as,
                        uint64_t row_first, uint64_t row_count, uint32_t* out);

/* ---- multi-GPU (no reference counterpart): rows shard across GPUs, one process
 * per GPU, one RCCL communicator per handle.  The only exchange is one all-reduce per batch:
 * MIN of the per-tape smallest witness index (MH_NO_HIT = UINT64_MAX is MIN's identity) and SUM
 * of the hit counts, in place in device buffers, on the ctx stream, so the result is identical
 * for any number of GPUs.  Rank 0 creates the id (mh_comm_unique_id) and the caller distributes
 * it (torch.distributed, a file, ...).  RCCL is dlopen'ed on first use: the path in MH_RCCL_LIB    *
 * when set (tests/test_comm_stub.py points it at a recording stub), else the ROCm install's.     */
#define MH_COMM_ID_BYTES 128
int32_t mh_comm_unique_id(uint8_t* out /* [MH_COMM_ID_BYTES] */);
int32_t mh_comm_init(mh_ctx* ctx, const uint8_t* unique_id, int32_t rank, int32_t world);
int32_t mh_comm_allreduce_results(mh_ctx* ctx, uint64_t* d_first_hit, uint64_t* d_hit_count,
                                  uint32_t n);
int32_t mh_comm_destroy(mh_ctx* ctx);

/* Integer VALU issue-rate micro-benchmark (no reference counterpart: it settles the roofline peak
 * of SURVEY.md §8d).  Runs 32 wave-instructions of one kind per loop iteration, written in asm,
 * at `waves_per_simd` (1..8) waves on every SIMD of the chip, and returns the sustained lane-ops/s
 * (wave-instructions/s x 64).  Kinds: 0 v_add_co/v_addc 256-bit carry chains; 1 v_mad_u64_u32;
 * 2 v_add_u32; 3 v_xor_b32; 4 v_alignbit_b32; 5 v_cndmask_b32; 6 v_or3_b32; 7 v_readlane_b32;
 * 8 v_mov_b32; 9 v_add_co_u32 (carry-out only); 10 v_sub_co/v_subb through VCC;
 * 11 v_cndmask_b32_e32 (VCC mask); 12 v_cmp_eq_u32_e32 (VCC write); 13 v_xor_b32 with a literal;
 * 14 v_lshlrev_b32; 15 v_add3_u32; 16 v_fma_f64; 17 v_xnor_b32; 18 v_and_b32; 19 v_or_b32;
 * 20 v_not_b32; with a partial EXEC mask: 21 v_xor_b32 (low 32 lanes), 22 v_alignbit_b32 (low 32),
 * 23 v_xor_b32 (low 16), 24 v_xor_b32 (every other lane); dependent chains (each instruction
 * reads the previous one's result: latency, at 1 wave per SIMD): 25 v_mad_u64_u32 into one
 * accumulator, 26 v_add_u32, 27 v_addc_co_u32 through VCC, 28 two v_mad_u64_u32 accumulators
 * interleaved, 29 v_mad_u64_u32 + v_addc carry count (product scanning), 30 v_cmp + v_cndmask;
 * mixed classes (independent): 31 v_mad_u64_u32 / v_add_u32 alternating, 32 v_addc_co_u32
 * chains / v_xor_b32 alternating, 33 two v_mad_u64_u32 per two v_add_u32; gfx950's
 * v_bitop3_b32: 34 alone (x ^ (~y & z)), 35 alternating with v_alignbit_b32; round 6:
 * 36 v_cmp_lt_u64 and 37 v_cmp_eq_u64 into SGPR pairs, 38 v_lshl_add_u64, 39 v_mul_lo_u32,
 * 40 v_mul_hi_u32, 41 v_mul_u32_u24, 42 v_sub_co_u32_e64 into SGPR pairs, 43 v_cmp_lt_u32_e64,
 * 44 a 256-bit `<` as 4 lt + 3 eq 64-bit compares with SALU folds (+1 filler compare).    */
#define MH_MB_NUM_KINDS 45
int32_t mh_microbench_issue(mh_ctx* ctx, uint32_t kind, uint32_t waves_per_simd,
                            double* lane_ops_per_s);
/* Survivor-gather micro-benchmark (the memory side of the lane compaction costed in DESIGN.md
 * §5.1): 2^log2_rows rows x 128 B of columns, the rows a hash keeps at permille / 1000 listed in
 * ascending order, each survivor's 128 B read per launch -- layout 0 the sieve's SoA columns
 * (32 scattered 4-byte loads), 1 row-major (8 contiguous 16-byte loads), 2 the SoA streaming read
 * of every row.  Median launch ms over `reps`, useful GB/s (survivors, or rows, x 128 B).        */
int32_t mh_microbench_gather(int32_t device, uint32_t log2_rows, uint32_t permille,
                             uint32_t layout, uint32_t reps, double* ms, double* gbps,
                             uint64_t* survivors);
/* Round-1 form: kinds 0..2 of mh_microbench_issue at 8 waves per SIMD.                           */
int32_t mh_microbench_valu(mh_ctx* ctx, uint32_t kind, double* ops_per_s);
/* Kernel timing on the ctx stream.  While enabled, every sieve launch (mh_run / mh_run_async) is
 * bracketed by HIP events recorded on the ctx stream itself, so the measured span is exactly the
 * launch's device time whatever stream the caller uses.  mh_ctx_kernel_time synchronises, returns
 * the summed milliseconds and the number of launches since the previous call, and resets both.   */
int32_t mh_ctx_enable_timing(mh_ctx* ctx, int32_t enable);
int32_t mh_ctx_kernel_time(mh_ctx* ctx, double* total_ms, uint64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* MYTHRIL_HIP_H */
