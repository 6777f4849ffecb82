// Launch interface between the C-ABI layer (capi.cpp) and the kernels (sieve_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mythril_hip.h"
#include "dev_isa.h"

namespace mh {

struct KParams {
    const uint2* insns;          // instruction words (2 x u32 per instruction)
    const mh_dev_tape* tapes;    // per-tape headers
    const uint32_t* consts;      // device constant pool, 8 limbs per entry
    const uint32_t* assign;      // SoA assignment buffer
    const uint32_t* tape_ids;    // the tapes this launch evaluates (one kernel-variant bucket)
    uint64_t capacity;           // column stride in words (>= rows allocated per column)
    uint32_t n_pre;              // columns preloaded into R0..R(n_pre-1)
    uint32_t n_ids;              // entries of tape_ids
    uint32_t result_base;        // results are indexed by tape id - result_base
    uint32_t pad;
    uint64_t row_first, row_count, index_base;
    uint32_t mode;
    unsigned long long* first_hit;  // [tapes of the run]
    unsigned long long* hit_count;  // [tapes of the run]
    uint32_t* values_out;           // parity path: [n_ids][8][row_count] root values, or null
    // conjunct-parallel short runs (capi.cpp mh_run_async): each wave of a part-tape writes its
    // 64-row Bool mask to masks[(tape id - mask_base) * mask_stride + wave of the run] instead
    // of first hits / counts, which the combine kernel then ANDs per split tape
    unsigned long long* masks;
    uint32_t mask_base;
    uint32_t pad2;
    uint64_t mask_stride;           // waves of the run's grid (sieve_mask_stride)
};

// Kernel variants: register-file size class (NR 7 / 9 / 15) x feature set (asm only / + C++
// complex ops / + keccak / + keccak and the EVM helpers).  Keccak tapes get a kernel without the
// EVM helpers' register footprint.
inline uint32_t nr_class(uint32_t n_regs) {
    return n_regs <= MH_NR_SMALL ? 0u : n_regs <= MH_NR_MID ? 1u : 2u;
}
inline uint32_t variant_of(uint32_t n_regs, uint32_t features) {
    const uint32_t fc = (features & F_EVM) ? 3u : (features & F_KECCAK) ? 2u
                        : (features & F_CPLX) ? 1u : 0u;
    return nr_class(n_regs) * 4 + fc;  // 0..11
}
constexpr uint32_t kNumVariants = 12;
// The complex-op variants (feature class != 0) load columns inside the asm core (run_lv) with a
// 32-bit byte stride per limb plane: their buffers hold fewer than 2^30 rows per column.  The
// asm-only variants index columns with 64-bit arithmetic and take any capacity.
constexpr uint64_t kLoadvarMaxCapacity = 1ull << 30;
inline bool variant_fits(uint32_t variant, uint64_t capacity) {
    return (variant & 3u) == 0 || capacity < kLoadvarMaxCapacity;
}

hipError_t launch_sieve(const KParams& p, uint32_t variant, hipStream_t stream);
hipError_t launch_generate(uint32_t* assign, uint64_t stride, uint64_t rows, uint32_t n_vars,
                           uint64_t seed, uint64_t base, hipStream_t stream);
// Device form of mh_guide (pointers into one device buffer owned by the mh_assign).
struct KGuide {
    uint32_t n_cols, n_sets;
    uint32_t n_value_sets;      // sets [0, n_value_sets) hold no copy entry
    const uint32_t* width;      // [n_cols]
    const uint32_t* pool_off;   // [n_cols + 1]
    const uint32_t* pool;       // x 8 limbs
    const uint32_t* set_prob;   // [n_sets]
    const uint32_t* set_off;    // [n_sets + 1]
    const uint32_t* alt_off;    // [n_alts + 1]
    const uint32_t* entry_col;  // [n_entries]
    const uint32_t* entry_val;  // x 8 limbs
    // set_prob | set_off | alt_off | entry_col lie back to back from set_prob (span_words
    // words): the generator stages them in LDS when they fit
    uint32_t span_words;
};
hipError_t launch_generate_guided(uint32_t* assign, uint64_t stride, uint64_t first,
                                  uint64_t count, uint64_t seed, uint64_t base, const KGuide& g,
                                  hipStream_t stream);
// first_hit[0..n) = MH_NO_HIT, hit_count[0..n) = 0 in one launch (either may be null)
hipError_t launch_results_reset(uint64_t* first_hit, uint64_t* hit_count, uint32_t n,
                                hipStream_t stream);
// each tape's witness row (mh_run_rows): out[t][w] = column word w (column w / 8, limb w % 8) of
// the buffer row first_hit[t] - index_base, zero for a tape without a hit
hipError_t launch_witness_rows(const uint32_t* assign, uint64_t stride, const uint64_t* first_hit,
                               uint32_t n_tapes, uint64_t index_base, uint32_t n_cols,
                               uint32_t* out, hipStream_t stream);
// waves a run of row_count rows launches (the masks' row stride of a conjunct-parallel run)
uint64_t sieve_mask_stride(uint64_t row_count);
// per split tape i (split[3i] = tape id, split[3i+1] = its first part's id, whose masks are
// row id - mask_base, split[3i+2] = parts): the AND of its parts' masks per wave -> atomicMin of
// the first row (index0 + 64 w + lane) into first_hit[tape - result_base] and the count into
// hit_count (either may be null)
hipError_t launch_combine(const unsigned long long* masks, uint64_t stride, const uint32_t* split,
                          uint32_t n_split, uint32_t mask_base, uint32_t result_base,
                          uint64_t index0, unsigned long long* first_hit,
                          unsigned long long* hit_count, hipStream_t stream);
hipError_t launch_microbench(uint32_t kind, uint32_t iters, uint32_t blocks, uint32_t* sink,
                             hipStream_t stream);

}  // namespace mh
