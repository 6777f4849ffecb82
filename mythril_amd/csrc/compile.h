// Tape compiler interface (host side of libmythril_hip).
#pragma once
#include <stdint.h>

#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/mythril_hip.h"
#include "dev_isa.h"

namespace mh {

struct CompiledTape {
    uint32_t n_nodes = 0;
    uint32_t n_insns = 0;
    uint32_t n_regs = 0;
    uint32_t root_bool = 0;
    uint32_t features = 0;
    uint64_t alg_ops = 0;
};

// Lower one tape.  Appends its instruction words (2 per instruction) to `words` and any new
// constants to the shared device pool `dconsts` (8 limbs each, deduplicated via dconst_index).
int32_t compile_tape(const mh_node* nodes, size_t n_nodes, const uint32_t* consts,
                     uint32_t n_consts, uint32_t n_vars, std::vector<uint32_t>& dconsts,
                     std::unordered_map<std::string, uint32_t>& dconst_index,
                     std::vector<uint32_t>& words, CompiledTape& out, std::string& err);

}  // namespace mh
