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
    uint64_t capacity;           // rows allocated per column
    uint32_t n_pre;              // columns preloaded into R0..R(n_pre-1)
    uint32_t tape_first, tape_count;
    uint64_t row_first, row_count, index_base;
    uint32_t mode;
    unsigned long long* first_hit;  // [tape_count]
    unsigned long long* hit_count;  // [tape_count]
};

hipError_t launch_sieve(const KParams& p, uint32_t feat, hipStream_t stream);
hipError_t launch_values(const KParams& p, uint32_t tape, uint32_t* out, hipStream_t stream);
hipError_t launch_generate(uint32_t* assign, uint64_t capacity, uint32_t n_vars, uint64_t seed,
                           uint64_t base, hipStream_t stream);
hipError_t launch_microbench(uint32_t kind, uint32_t iters, uint32_t blocks, uint32_t* sink,
                             hipStream_t stream);

}  // namespace mh
