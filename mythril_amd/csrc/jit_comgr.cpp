// In-process assembler for the sieve JIT: comgr (ROCm's code object manager, the library hiprtc
// is built on) assembles the generated gfx950 source into a relocatable object and links it
// into a loadable code object.  No subprocess, no temporary files.
#include <string.h>

#include <amd_comgr/amd_comgr.h>

#include "jit.h"

namespace mh {
namespace jit {

namespace {

struct Guard {
    amd_comgr_data_set_t in{}, rel{}, exe{};
    amd_comgr_action_info_t info{};
    amd_comgr_data_t src{};
    bool has_in = false, has_rel = false, has_exe = false, has_info = false, has_src = false;
    ~Guard() {
        if (has_src) amd_comgr_release_data(src);
        if (has_info) amd_comgr_destroy_action_info(info);
        if (has_exe) amd_comgr_destroy_data_set(exe);
        if (has_rel) amd_comgr_destroy_data_set(rel);
        if (has_in) amd_comgr_destroy_data_set(in);
    }
};

bool ok(amd_comgr_status_t s, const char* what, std::string& log) {
    if (s == AMD_COMGR_STATUS_SUCCESS) return true;
    const char* msg = nullptr;
    amd_comgr_status_string(s, &msg);
    log += std::string(what) + ": " + (msg ? msg : "comgr error") + "\n";
    return false;
}

void append_logs(amd_comgr_data_set_t set, std::string& log) {
    size_t n = 0;
    if (amd_comgr_action_data_count(set, AMD_COMGR_DATA_KIND_LOG, &n) != AMD_COMGR_STATUS_SUCCESS)
        return;
    for (size_t i = 0; i < n; ++i) {
        amd_comgr_data_t d;
        if (amd_comgr_action_data_get_data(set, AMD_COMGR_DATA_KIND_LOG, i, &d) !=
            AMD_COMGR_STATUS_SUCCESS)
            continue;
        size_t sz = 0;
        amd_comgr_get_data(d, &sz, nullptr);
        std::string b(sz, '\0');
        amd_comgr_get_data(d, &sz, &b[0]);
        log += b;
        amd_comgr_release_data(d);
    }
}

}  // namespace

bool assemble(const std::string& text, std::vector<char>& hsaco, std::string& log) {
    Guard g;
    if (!ok(amd_comgr_create_data_set(&g.in), "create_data_set", log)) return false;
    g.has_in = true;
    if (!ok(amd_comgr_create_data(AMD_COMGR_DATA_KIND_SOURCE, &g.src), "create_data", log))
        return false;
    g.has_src = true;
    if (!ok(amd_comgr_set_data(g.src, text.size(), text.data()), "set_data", log)) return false;
    if (!ok(amd_comgr_set_data_name(g.src, "mh_jit.s"), "set_data_name", log)) return false;
    if (!ok(amd_comgr_data_set_add(g.in, g.src), "data_set_add", log)) return false;
    if (!ok(amd_comgr_create_action_info(&g.info), "create_action_info", log)) return false;
    g.has_info = true;
    if (!ok(amd_comgr_action_info_set_isa_name(g.info, "amdgcn-amd-amdhsa--gfx950"), "isa", log))
        return false;
    amd_comgr_action_info_set_logging(g.info, true);
    if (!ok(amd_comgr_create_data_set(&g.rel), "create_data_set", log)) return false;
    g.has_rel = true;
    const bool a = ok(amd_comgr_do_action(AMD_COMGR_ACTION_ASSEMBLE_SOURCE_TO_RELOCATABLE, g.info,
                                          g.in, g.rel), "assemble", log);
    append_logs(g.rel, log);
    if (!a) return false;
    if (!ok(amd_comgr_create_data_set(&g.exe), "create_data_set", log)) return false;
    g.has_exe = true;
    const bool l = ok(amd_comgr_do_action(AMD_COMGR_ACTION_LINK_RELOCATABLE_TO_EXECUTABLE, g.info,
                                          g.rel, g.exe), "link", log);
    append_logs(g.exe, log);
    if (!l) return false;
    amd_comgr_data_t out;
    if (!ok(amd_comgr_action_data_get_data(g.exe, AMD_COMGR_DATA_KIND_EXECUTABLE, 0, &out),
            "get executable", log))
        return false;
    size_t sz = 0;
    amd_comgr_get_data(out, &sz, nullptr);
    hsaco.resize(sz);
    amd_comgr_get_data(out, &sz, hsaco.data());
    amd_comgr_release_data(out);
    return true;
}

}  // namespace jit
}  // namespace mh
