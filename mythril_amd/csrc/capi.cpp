// C-ABI of libmythril_hip (include/mythril_hip.h): handles, error reporting, device buffers,
// launch orchestration.  No exception crosses the ABI and nothing here aborts the process:
// every failure is an MH_E_* code plus a thread-local message, so the Python front end can fall
// back to z3 (SURVEY.md §5 "fail closed").
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/mythril_hip.h"
#include "compile.h"
#include "dev_isa.h"
#include "jit.h"
#include "kernels.h"

constexpr uint32_t kSideStreams = 3;  // with the ctx stream: GPU_MAX_HW_QUEUES (4) queues

// MH_FANOUT=0 turns the short-run fan-out over side streams off (read once per process)
static bool fanout_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("MH_FANOUT");
        return !(e && e[0] == '0');
    }();
    return on;
}

struct AsyncCompile;  // mh_tapes_compile_async's worker (below)

struct mh_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    uint32_t* scratch = nullptr;  // microbench sink
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> spans;  // one per timed sieve launch
    // per-query latency path (mh_run / mh_eval_values / mh_assign_download): grow-only device
    // result buffer and pinned host staging, so a query allocates nothing
    void* d_buf = nullptr;
    size_t d_buf_bytes = 0;
    void* h_buf = nullptr;
    size_t h_buf_bytes = 0;
    // multi-GPU: one RCCL communicator per handle (mh_comm_init)
    ncclComm_t comm = nullptr;
    int32_t rank = 0, world = 1;
    // device blocks of destroyed tape sets, by power-of-two size class: a query's tape set
    // reuses them instead of calling hipMalloc (a new size class costs milliseconds)
    std::unordered_map<size_t, std::vector<void*>> pool;
    std::unordered_map<void*, size_t> pool_class;
    size_t pool_bytes = 0;
    // tape sets and assignment buffers hold the context: mh_ctx_destroy before them only marks
    // it released, and the last child's destroy frees it
    int32_t children = 0;
    bool released = false;
    // pinned staging of tape-set uploads (one async copy per compile; the next compile waits on
    // the event before it refills the buffer)
    void* h_stage = nullptr;
    size_t h_stage_bytes = 0;
    hipEvent_t stage_ev = nullptr;
    bool stage_pending = false;
    // compiled tapes by content (the tape's nodes, the values of the constants it reads, the
    // column count): a LASER query's groups mostly repeat its parent's (svm.py:257-262), and a
    // tape's instruction words are self-contained (constants inline), so a repeated tape reuses
    // its words; cleared beyond kCacheWords words (mh_tapes_compile) or by mh_ctx_clear_cache
    std::unordered_map<std::string, std::pair<std::vector<uint32_t>, mh::CompiledTape>> compile_cache;
    size_t compile_cache_words = 0;
    // a short run's launches (one per register class) are a few waves each walking a long tape:
    // latency-bound, so they overlap on side streams (forked from and joined back into `stream`
    // by events) instead of queueing behind each other; created on first use
    hipStream_t side[kSideStreams] = {};
    hipEvent_t fork_ev = nullptr, join_ev[kSideStreams] = {};
    // the wave masks of a conjunct-parallel short run (grow-only)
    unsigned long long* d_masks = nullptr;
    size_t masks_bytes = 0;
    // mh_tapes_compile_async: one worker thread, started on first use, joined by ctx_free
    AsyncCompile* acomp = nullptr;
    // kernel launches of mh_eval_values_many (Model.eval batching is measured by it)
    uint64_t eval_launches = 0;
};

// One compile at a time, handed to a worker thread that waits on a condition variable (a thread
// per call would cost its creation; a Python thread costs GIL hand-offs around the native call)
struct AsyncCompile {
    std::mutex m;
    std::condition_variable cv;
    std::thread th;
    bool stop = false, job = false, done = false;
    const mh_node* nodes = nullptr;
    const uint64_t* offs = nullptr;
    uint32_t n_tapes = 0, n_consts = 0, n_vars = 0;
    const uint32_t* consts = nullptr;
    int32_t rc = MH_OK;
    std::string err;
    mh_tapeset* out = nullptr;
    double seconds = 0;
};

namespace {
// RCCL is opened on first use (dlopen), not linked: a process that never shards never loads it.
// The ROCm install's copy comes first, opened by path with its own symbol scope (DEEPBIND): it
// binds to the same libamdhip64.so.7 this library runs on, whereas a Python wheel's bundled
// librccl (torch's) binds to the wheel's own HIP runtime -- on the box that copy fails with
// "no ROCm-capable device" when this library initialised HIP first.
struct Rccl {
    void* h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                               hipStream_t) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};
const Rccl* rccl() {
    static Rccl r;
    static bool tried = false;
    if (!tried) {
        tried = true;
        // MH_RCCL_LIB names another copy first (a recording stub in tests/test_comm_stub.py)
        const char* env = std::getenv("MH_RCCL_LIB");
        for (const char* name : {env, "/opt/rocm/lib/librccl.so.1", "librccl.so.1"}) {
            if (!name || !*name) continue;
            r.h = dlopen(name, RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
            if (r.h || name == env) break;  // a named copy that fails is not replaced
        }
        if (r.h) {
            r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.h, "ncclGetUniqueId");
            r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.h, "ncclCommInitRank");
            r.all_reduce = (decltype(r.all_reduce))dlsym(r.h, "ncclAllReduce");
            r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.h, "ncclCommDestroy");
            r.error_string = (decltype(r.error_string))dlsym(r.h, "ncclGetErrorString");
        }
    }
    if (!r.get_unique_id || !r.comm_init_rank || !r.all_reduce || !r.comm_destroy) return nullptr;
    return &r;
}
}  // namespace

namespace {
hipError_t ctx_dbuf(mh_ctx* c, size_t bytes, void** out) {
    if (bytes > c->d_buf_bytes) {
        if (c->d_buf) (void)hipFree(c->d_buf);
        c->d_buf = nullptr;
        c->d_buf_bytes = 0;
        size_t n = 1 << 16;
        while (n < bytes) n <<= 1;
        hipError_t e = hipMalloc(&c->d_buf, n);
        if (e != hipSuccess) return e;
        c->d_buf_bytes = n;
    }
    *out = c->d_buf;
    return hipSuccess;
}
// smallest class 256 KiB: a query's whole tape set fits one block, so after the first query every
// compile reuses a block (a hipMalloc of a size the process has not seen costs milliseconds)
size_t pool_size_class(size_t bytes) {
    size_t n = 256u << 10;
    while (n < bytes) n <<= 1;
    return n;
}
template <class T>
hipError_t pool_alloc(mh_ctx* c, T** out, size_t bytes) {
    const size_t k = pool_size_class(bytes);
    auto& fl = c->pool[k];
    if (!fl.empty()) {
        *out = static_cast<T*>(fl.back());
        fl.pop_back();
        c->pool_bytes -= k;
        return hipSuccess;
    }
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, k);
    if (e != hipSuccess) return e;
    c->pool_class[p] = k;
    *out = static_cast<T*>(p);
    return hipSuccess;
}
void pool_free(mh_ctx* c, void* p) {
    if (!p) return;
    auto it = c->pool_class.find(p);
    if (it == c->pool_class.end()) {
        (void)hipFree(p);
        return;
    }
    if (c->pool_bytes + it->second > (256u << 20)) {  // keep at most 256 MiB cached
        (void)hipFree(p);
        c->pool_class.erase(it);
        return;
    }
    c->pool[it->second].push_back(p);
    c->pool_bytes += it->second;
}
hipError_t ctx_hbuf(mh_ctx* c, size_t bytes, void** out) {
    if (bytes > c->h_buf_bytes) {
        if (c->h_buf) (void)hipHostFree(c->h_buf);
        c->h_buf = nullptr;
        c->h_buf_bytes = 0;
        size_t n = 1 << 16;
        while (n < bytes) n <<= 1;
        hipError_t e = hipHostMalloc(&c->h_buf, n, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        c->h_buf_bytes = n;
    }
    *out = c->h_buf;
    return hipSuccess;
}
}  // namespace

struct mh_tapeset {
    mh_ctx* ctx = nullptr;
    uint32_t n_tapes = 0;
    uint32_t n_vars = 0;
    void* d_block = nullptr;  // one pool block: insns | ids | tapes | consts
    uint2* d_insns = nullptr;
    mh_dev_tape* d_tapes = nullptr;
    uint32_t* d_consts = nullptr;
    std::vector<mh_tape_info> info;
    // tapes bucketed by kernel variant (kernels.h variant_of): ascending tape ids per bucket,
    // concatenated in d_ids; bucket v is [bucket_off[v], bucket_off[v+1])
    uint32_t* d_ids = nullptr;
    std::vector<uint32_t> ids;
    uint32_t bucket_off[mh::kNumVariants + 1] = {};
    // host copy of the IR, for mh_tapes_jit
    std::vector<mh_node> h_nodes;
    std::vector<uint64_t> h_offs;
    std::vector<uint32_t> h_consts;
    // native-code path (mh_tapes_jit): one module per slice of tape groups; the interpreter's
    // buckets restricted to the tapes the JIT does not take
    struct JitMod {
        hipModule_t mod = nullptr, vmod = nullptr;
        hipFunction_t fn = nullptr, vfn = nullptr;
        uint32_t n_groups = 0;
        // the code object images stay alive as long as the modules: the HIP runtime may read
        // an image after hipModuleLoadData returns (lazy loading)
        std::vector<char> image, vimage;
    };
    std::vector<JitMod> jit;
    std::vector<uint8_t> jitted;
    bool has_jit = false;
    uint32_t* d_ids_rest = nullptr;
    std::vector<uint32_t> ids_rest;
    uint32_t bucket_off_rest[mh::kNumVariants + 1] = {};
    mh_jit_info jinfo{};
    uint64_t code_id = 0;   // mh::jit::code_id of the count kernels' module texts
    // conjunct-parallel short runs (mh_run_async): a long tape's root conjunction cut into parts
    // of consecutive conjuncts, each compiled as a tape of its own (ids n_tapes, n_tapes + 1, ..,
    // in the order of their tapes) and bucketed like the tapes; the buckets without the split
    // tapes; per split tape, ascending: (tape, first part id, parts)
    uint32_t n_parts = 0;
    std::vector<uint32_t> ids_unsplit, part_ids, part_parent, split_tab;
    uint32_t bucket_off_unsplit[mh::kNumVariants + 1] = {};
    uint32_t bucket_off_parts[mh::kNumVariants + 1] = {};
    uint32_t *d_ids_unsplit = nullptr, *d_part_ids = nullptr, *d_split = nullptr;
};

struct mh_assign {
    mh_ctx* ctx = nullptr;
    uint32_t n_vars = 0;
    uint64_t capacity = 0;
    uint64_t stride = 0;           // words between column-limbs (capacity + assign_pad_rows)
    uint32_t* d = nullptr;
    uint32_t* d_guide = nullptr;   // packed mh_guide (grow-only)
    size_t guide_words = 0;
    std::vector<uint32_t> h_guide; // host packing of the guide
    uint32_t* h_pinned = nullptr;  // pinned staging of the packed guide (grow-only)
    size_t pinned_words = 0;
    hipEvent_t staged = nullptr;   // recorded after the staging copy; reuse waits on it
    bool staged_pending = false;
};

namespace {

thread_local std::string g_err;

int32_t set_err(int32_t code, const std::string& msg) {
    g_err = msg;
    return code;
}
}  // namespace

// mh_last_error text for the host-only entry points of other translation units (harvest.cpp)
int32_t mh_detail_set_err(int32_t code, const char* msg) { return set_err(code, msg); }

namespace {

#define MH_HIP(call)                                                                      \
    do {                                                                                  \
        hipError_t e_ = (call);                                                           \
        if (e_ != hipSuccess)                                                             \
            return set_err(MH_E_DEVICE, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

bool is_gfx950(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

// The compile worker thread (mh_tapes_compile_async) sets this: its own calls into the ctx do not
// wait for themselves.
thread_local bool t_compile_worker = false;

// Every entry point that uses a ctx's state (device buffers, the compiled-tape cache, the staging
// buffer, the pool, the stream) passes here: while the ctx's worker thread runs a compile, the
// call waits for that compile to finish (its result stays for mh_tapes_compile_wait), so no two
// threads touch the ctx at once.  The host-only harvest the caller overlaps with the
// compile never enters a ctx.
void settle(const mh_ctx* ctx) {
    AsyncCompile* a = ctx->acomp;
    if (!a || t_compile_worker) return;
    std::unique_lock<std::mutex> lk(a->m);
    a->cv.wait(lk, [&] { return !a->job || a->done; });
}

int32_t use_device(const mh_ctx* ctx) {
    settle(ctx);
    MH_HIP(hipSetDevice(ctx->device));
    return MH_OK;
}

uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int32_t check_run_args(const mh_ctx* ctx, const mh_tapeset* ts, uint32_t tape_first,
                       uint32_t tape_count, const mh_assign* as, uint64_t row_first,
                       uint64_t row_count, uint32_t mode) {
    if (!ctx || !ts || !as) return set_err(MH_E_INVALID, "null handle");
    if (ts->ctx != ctx || as->ctx != ctx) return set_err(MH_E_INVALID, "handles of another ctx");
    if ((uint64_t)tape_first + tape_count > ts->n_tapes)
        return set_err(MH_E_INVALID, "tape range out of bounds");
    if (row_first > as->capacity || row_count > as->capacity - row_first)
        return set_err(MH_E_INVALID, "row range out of bounds");
    if (as->n_vars < ts->n_vars)
        return set_err(MH_E_INVALID, "assignment buffer has fewer columns than the tapes use");
    if (mode != MH_MODE_FIRST_HIT && mode != MH_MODE_COUNT_ALL)
        return set_err(MH_E_INVALID, "bad mode");
    return MH_OK;
}

mh::KParams make_params(const mh_tapeset* ts, uint32_t tape_first, const mh_assign* as,
                        uint64_t row_first, uint64_t row_count, uint64_t index_base,
                        uint32_t mode) {
    mh::KParams p{};
    p.insns = ts->d_insns;
    p.tapes = ts->d_tapes;
    p.consts = ts->d_consts;
    p.assign = as->d;
    p.capacity = as->stride;
    p.n_pre = ts->n_vars <= MH_MAX_PRELOAD ? ts->n_vars : 0;
    p.result_base = tape_first;
    p.row_first = row_first;
    p.row_count = row_count;
    p.index_base = index_base;
    p.mode = mode;
    return p;
}

// Rows per workgroup of the JIT kernels: 4 waves, each over a contiguous run of 64-row chunks.
uint32_t jit_rows_per_wg(uint64_t row_count) {
    static const uint32_t forced = [] {  // diagnostic: MH_JIT_ROWS_PER_WG (multiple of 256)
        const char* e = std::getenv("MH_JIT_ROWS_PER_WG");
        const uint32_t v = e ? (uint32_t)atoi(e) : 0u;
        return (v >= 256 && v % 256 == 0) ? v : 0u;
    }();
    if (forced) return forced;
    uint64_t r = 256;
    while (r < 16384 && r * 2048 < row_count) r *= 2;  // >= ~2048 row blocks before growing
    return (uint32_t)r;
}

int32_t launch_jit(mh_ctx* ctx, const mh_tapeset* ts, const mh_assign* as, uint64_t row_first,
                   uint64_t row_count, uint64_t index_base, uint32_t mode, uint64_t* d_first_hit,
                   uint64_t* d_hit_count, uint32_t* d_values) {
    mh::jit::KernArgs a{};
    a.assign = (uint64_t)(uintptr_t)as->d;
    a.capacity = as->stride;
    a.row_first = row_first;
    a.row_count = row_count;
    a.index_base = index_base;
    a.first_hit = (uint64_t)(uintptr_t)d_first_hit;
    a.hit_count = (uint64_t)(uintptr_t)d_hit_count;
    a.rows_per_wg = jit_rows_per_wg(row_count);
    a.n_rowblocks = (uint32_t)((row_count + a.rows_per_wg - 1) / a.rows_per_wg);
    a.values_out = (uint64_t)(uintptr_t)d_values;
    a.mode = mode;
    if (as->stride >= (1ull << 30) || row_first + row_count > (1ull << 31))
        return set_err(MH_E_UNSUPPORTED, "JIT kernels address < 2^30 rows per column");
    for (const auto& j : ts->jit) {
        hipFunction_t fn = d_values ? j.vfn : j.fn;
        if (!fn || !j.n_groups) continue;
        for (uint32_t g0 = 0; g0 < j.n_groups; g0 += 65535) {
            a.group_first = g0;
            const uint32_t gy = std::min<uint32_t>(65535, j.n_groups - g0);
            size_t sz = sizeof(a);
            void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &sz,
                           HIP_LAUNCH_PARAM_END};
            MH_HIP(hipModuleLaunchKernel(fn, a.n_rowblocks, gy, 1, 256, 1, 1, 0, ctx->stream,
                                         nullptr, cfg));
        }
    }
    return MH_OK;
}

}  // namespace

extern "C" {

int32_t mh_version(uint32_t* major, uint32_t* minor, uint32_t* patch) {
    if (major) *major = MH_VERSION_MAJOR;
    if (minor) *minor = MH_VERSION_MINOR;
    if (patch) *patch = MH_VERSION_PATCH;
    return MH_OK;
}

const char* mh_last_error(void) { return g_err.c_str(); }

int32_t mh_device_count(int32_t* n) {
    if (!n) return set_err(MH_E_INVALID, "null out pointer");
    *n = 0;
    int total = 0;
    if (hipGetDeviceCount(&total) != hipSuccess) {
        (void)hipGetLastError();
        return MH_OK;
    }
    for (int d = 0; d < total; ++d) *n += is_gfx950(d) ? 1 : 0;
    return MH_OK;
}

namespace {
void ctx_free(mh_ctx* ctx);
}

int32_t mh_ctx_create(int32_t device, mh_ctx** out) {
    if (!out) return set_err(MH_E_INVALID, "null out pointer");
    *out = nullptr;
    int total = 0;
    if (hipGetDeviceCount(&total) != hipSuccess || device < 0 || device >= total) {
        (void)hipGetLastError();
        return set_err(MH_E_NODEVICE, "no HIP device " + std::to_string(device));
    }
    if (!is_gfx950(device)) return set_err(MH_E_NODEVICE, "device is not gfx950 (MI355X)");
    mh_ctx* c = new (std::nothrow) mh_ctx();
    if (!c) return set_err(MH_E_NOMEM, "ctx allocation");
    c->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    c->own_stream = c->stream != nullptr;
    // the short-run fan-out's side streams and events up front, when the fan-out is on: a stream
    // created on first use took 14.4 ms inside the query that first needed it (profiles/r04x).
    // With MH_FANOUT=0 a ctx holds its one stream (hardware queues are few per process)
    for (uint32_t i = 0; i < kSideStreams && e == hipSuccess && fanout_enabled(); ++i) {
        e = hipStreamCreateWithFlags(&c->side[i], hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&c->join_ev[i], hipEventDisableTiming);
    }
    if (e == hipSuccess && fanout_enabled())
        e = hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming);
    if (e == hipSuccess) e = hipMalloc(&c->scratch, 64);
    if (e == hipSuccess) {
        // one block of the smallest class ready for the first query, and the pinned upload
        // staging; one round trip through them initialises the runtime's copy path for sizes a
        // query's first large tape set would otherwise pay for (~30 ms once per process)
        void* blk = nullptr;
        const size_t warm = 256u << 10;
        e = pool_alloc(c, (char**)&blk, warm);
        if (e == hipSuccess) e = hipHostMalloc(&c->h_stage, 1u << 20, hipHostMallocDefault);
        if (e == hipSuccess) {
            c->h_stage_bytes = 1u << 20;
            std::memset(c->h_stage, 0, warm);
            e = hipMemcpyAsync(blk, c->h_stage, warm, hipMemcpyHostToDevice, c->stream);
        }
        if (e == hipSuccess)
            e = hipMemcpyAsync(c->h_stage, blk, warm, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (blk) pool_free(c, blk);
    }
    if (e != hipSuccess) {
        ctx_free(c);
        return set_err(MH_E_DEVICE, std::string("ctx init: ") + hipGetErrorString(e));
    }
    *out = c;
    return MH_OK;
}

namespace {
void ctx_free(mh_ctx* ctx) {
    if (AsyncCompile* a = ctx->acomp) {
        {
            std::unique_lock<std::mutex> lk(a->m);
            a->cv.wait(lk, [&] { return !a->job || a->done; });  // a pending compile finishes
            a->stop = true;
        }
        a->cv.notify_all();
        if (a->th.joinable()) a->th.join();
        delete a;
        ctx->acomp = nullptr;
    }
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto& sp : ctx->spans) {
        (void)hipEventDestroy(sp.first);
        (void)hipEventDestroy(sp.second);
    }
    if (ctx->own_stream && ctx->stream) (void)hipStreamDestroy(ctx->stream);
    for (uint32_t i = 0; i < kSideStreams; ++i) {
        if (ctx->side[i]) {
            (void)hipStreamSynchronize(ctx->side[i]);
            (void)hipStreamDestroy(ctx->side[i]);
        }
        if (ctx->join_ev[i]) (void)hipEventDestroy(ctx->join_ev[i]);
    }
    if (ctx->fork_ev) (void)hipEventDestroy(ctx->fork_ev);
    if (ctx->d_masks) (void)hipFree(ctx->d_masks);
    if (ctx->scratch) (void)hipFree(ctx->scratch);
    if (ctx->d_buf) (void)hipFree(ctx->d_buf);
    if (ctx->h_buf) (void)hipHostFree(ctx->h_buf);
    if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
    if (ctx->stage_ev) (void)hipEventDestroy(ctx->stage_ev);
    if (ctx->comm && rccl()) (void)rccl()->comm_destroy(ctx->comm);
    for (auto& kv : ctx->pool_class) (void)hipFree(kv.first);
    delete ctx;
}
// a child (tape set / assignment buffer) of `ctx` is gone
void ctx_unref(mh_ctx* ctx) {
    if (--ctx->children == 0 && ctx->released) ctx_free(ctx);
}
}  // namespace

int32_t mh_ctx_destroy(mh_ctx* ctx) {
    if (!ctx) return MH_OK;
    if (ctx->released) return set_err(MH_E_INVALID, "context already destroyed");
    if (AsyncCompile* a = ctx->acomp) {  // a compile nobody collected: finish and drop it
        mh_tapeset* left = nullptr;
        {
            std::unique_lock<std::mutex> lk(a->m);
            a->cv.wait(lk, [&] { return !a->job || a->done; });
            if (a->job) {
                left = a->out;
                a->out = nullptr;
                a->job = false;
            }
        }
        if (left) (void)mh_tapes_destroy(left);
    }
    if (ctx->children > 0) {
        ctx->released = true;
        return MH_OK;
    }
    ctx_free(ctx);
    return MH_OK;
}

int32_t mh_ctx_clear_cache(mh_ctx* ctx) {
    if (!ctx) return set_err(MH_E_INVALID, "null ctx");
    settle(ctx);
    ctx->compile_cache.clear();
    ctx->compile_cache_words = 0;
    return MH_OK;
}

int32_t mh_ctx_set_stream(mh_ctx* ctx, void* hip_stream) {
    if (!ctx) return set_err(MH_E_INVALID, "null ctx");
    if (int32_t r = use_device(ctx)) return r;
    // uploads queued on the current stream (tape sets, guides: asynchronous copies from pinned
    // staging) must land before anything on the new stream reads them
    MH_HIP(hipStreamSynchronize(ctx->stream));
    if (ctx->own_stream && ctx->stream) MH_HIP(hipStreamDestroy(ctx->stream));
    ctx->stream = (hipStream_t)hip_stream;  // NULL = the device's null stream
    ctx->own_stream = false;
    return MH_OK;
}

int32_t mh_ctx_synchronize(mh_ctx* ctx) {
    if (!ctx) return set_err(MH_E_INVALID, "null ctx");
    if (int32_t r = use_device(ctx)) return r;
    MH_HIP(hipStreamSynchronize(ctx->stream));
    return MH_OK;
}

int32_t mh_tapes_compile_async(mh_ctx* ctx, const mh_node* nodes, const uint64_t* tape_offsets,
                               uint32_t n_tapes, const uint32_t* consts, uint32_t n_consts,
                               uint32_t n_vars) {
    if (!ctx) return set_err(MH_E_INVALID, "null ctx");
    try {
        if (!ctx->acomp) {
            AsyncCompile* a = new AsyncCompile();
            a->th = std::thread([ctx, a] {
                t_compile_worker = true;
                std::unique_lock<std::mutex> lk(a->m);
                for (;;) {
                    a->cv.wait(lk, [&] { return a->stop || (a->job && !a->done); });
                    if (a->stop) return;
                    lk.unlock();
                    mh_tapeset* out = nullptr;
                    const auto t0 = std::chrono::steady_clock::now();
                    const int32_t rc = mh_tapes_compile(ctx, a->nodes, a->offs, a->n_tapes,
                                                        a->consts, a->n_consts, a->n_vars, &out);
                    const double dt = std::chrono::duration<double>(
                                          std::chrono::steady_clock::now() - t0).count();
                    const std::string err = rc == MH_OK ? std::string() : mh_last_error();
                    lk.lock();
                    a->rc = rc;
                    a->err = err;
                    a->out = out;
                    a->seconds = dt;
                    a->done = true;
                    a->cv.notify_all();
                }
            });
            ctx->acomp = a;
        }
    } catch (const std::exception&) {
        return set_err(MH_E_NOMEM, "compile worker thread");
    }
    AsyncCompile* a = ctx->acomp;
    {
        std::lock_guard<std::mutex> lk(a->m);
        if (a->job) return set_err(MH_E_INVALID, "a compile is already pending on this ctx");
        a->nodes = nodes;
        a->offs = tape_offsets;
        a->n_tapes = n_tapes;
        a->consts = consts;
        a->n_consts = n_consts;
        a->n_vars = n_vars;
        a->out = nullptr;
        a->rc = MH_OK;
        a->done = false;
        a->job = true;
    }
    a->cv.notify_all();
    return MH_OK;
}

int32_t mh_tapes_compile_wait(mh_ctx* ctx, mh_tapeset** out, double* compile_s) {
    if (!ctx || !out) return set_err(MH_E_INVALID, "null argument");
    *out = nullptr;
    AsyncCompile* a = ctx->acomp;
    if (!a) return set_err(MH_E_INVALID, "no compile pending on this ctx");
    std::unique_lock<std::mutex> lk(a->m);
    if (!a->job) return set_err(MH_E_INVALID, "no compile pending on this ctx");
    a->cv.wait(lk, [&] { return a->done; });
    a->job = false;
    *out = a->out;
    a->out = nullptr;
    if (compile_s) *compile_s = a->seconds;
    if (a->rc != MH_OK) return set_err(a->rc, a->err);
    return MH_OK;
}

int32_t mh_tapes_compile(mh_ctx* ctx, const mh_node* nodes, const uint64_t* tape_offsets,
                         uint32_t n_tapes, const uint32_t* consts, uint32_t n_consts,
                         uint32_t n_vars, mh_tapeset** out) {
    static const bool trace = std::getenv("MH_TRACE_COMPILE") != nullptr;
    auto tnow = [] { return std::chrono::steady_clock::now(); };
    const auto t_start = tnow();
    if (!ctx || !out || (!nodes && n_tapes) || !tape_offsets || (!consts && n_consts))
        return set_err(MH_E_INVALID, "null argument");
    *out = nullptr;
    settle(ctx);  // the compile cache, staging buffer and pool are the ctx's
    std::vector<uint32_t> words, dconsts;
    mh::ConstIndex dindex;
    std::vector<mh_dev_tape> heads(n_tapes);
    std::vector<mh_tape_info> info(n_tapes);
    std::vector<uint32_t> ids, bucket_off(mh::kNumVariants + 1, 0);
    // conjunct-parallel parts (mh_tapeset): heads n_tapes.. and their buckets
    std::vector<uint32_t> ids_unsplit, part_ids, part_parent, split_tab;
    uint32_t off_unsplit[mh::kNumVariants + 1] = {}, off_parts[mh::kNumVariants + 1] = {};
    try {
        std::vector<std::vector<uint32_t>> tw(n_tapes);
        static const bool use_cache = [] {
            const char* e = std::getenv("MH_COMPILE_CACHE");
            return !(e && e[0] == '0');
        }();
        constexpr size_t kCacheWords = (size_t)16 << 20;  // 128 MB of instruction words
        std::string key;
        // one tape's words and summary, from the cache when its content was compiled before
        auto compile_one = [&](const mh_node* tn, size_t nn, std::vector<uint32_t>& w,
                               mh::CompiledTape& ct, std::string& err) -> int32_t {
            if (use_cache) {  // the tape's content: nodes, constant values, column count
                key.assign(reinterpret_cast<const char*>(&n_vars), sizeof n_vars);
                key.append(reinterpret_cast<const char*>(tn), nn * sizeof(mh_node));
                for (size_t i = 0; i < nn; ++i)
                    if (tn[i].op == MH_OP_CONST && tn[i].imm0 < n_consts)
                        key.append(reinterpret_cast<const char*>(consts + 8ull * tn[i].imm0), 32);
                auto hit = ctx->compile_cache.find(key);
                if (hit != ctx->compile_cache.end()) {
                    w = hit->second.first;
                    ct = hit->second.second;
                    return MH_OK;
                }
            }
            const int32_t r = mh::compile_tape(tn, nn, consts, n_consts, n_vars, dconsts, dindex,
                                               w, ct, err);
            if (r == MH_OK && use_cache) {
                if (ctx->compile_cache_words + w.size() > kCacheWords) {
                    ctx->compile_cache.clear();
                    ctx->compile_cache_words = 0;
                }
                ctx->compile_cache_words += w.size();
                ctx->compile_cache.emplace(key, std::make_pair(w, ct));
            }
            return r;
        };
        for (uint32_t t = 0; t < n_tapes; ++t) {
            const uint64_t b = tape_offsets[t], e = tape_offsets[t + 1];
            if (e <= b) return set_err(MH_E_INVALID, "tape " + std::to_string(t) + " is empty");
            mh::CompiledTape ct;
            std::string err;
            const int32_t r = compile_one(nodes + b, (size_t)(e - b), tw[t], ct, err);
            if (r != MH_OK) return set_err(r, "tape " + std::to_string(t) + ": " + err);
            heads[t] = mh_dev_tape{0, ct.n_insns, ct.root_bool, ct.n_regs};
            info[t] = mh_tape_info{ct.n_nodes, ct.n_insns, ct.n_regs, ct.features, ct.alg_ops};
        }
        // conjunct-parallel parts of the long tapes (a query round's latency is its longest
        // tape walked by one wave per SIMD: parts walk in parallel, mh_run_async); MH_SPLIT_INSNS
        // = the instruction slots from which a tape is cut, one part per that many.  Off by
        // default: measured on the LASER-shaped queries and paths, the parts' compile
        // costs a LASER child about what the parallel walk saves, and the 2^16-row miss round
        // pays the parts' duplicated sub-terms
        const char* se = std::getenv("MH_SPLIT_INSNS");
        const uint32_t split_min = se ? (uint32_t)std::strtoul(se, nullptr, 10) : 0u;
        constexpr uint32_t kMaxParts = 8;
        std::vector<std::vector<uint32_t>> pw;
        std::vector<mh_tape_info> pinfo;
        std::vector<mh_dev_tape> pheads;
        for (uint32_t t = 0; split_min && t < n_tapes; ++t) {
            if (info[t].n_insns < split_min || !heads[t].root_bool) continue;
            const uint64_t b = tape_offsets[t], e = tape_offsets[t + 1];
            const uint32_t want = std::min<uint32_t>(kMaxParts, (info[t].n_insns + split_min - 1) / split_min);
            std::vector<std::vector<mh_node>> parts;
            if (!mh::split_conjunction(nodes + b, (uint32_t)(e - b), std::max<uint32_t>(want, 2), parts))
                continue;
            const size_t p0 = pw.size();
            bool ok = true;
            for (const auto& tp : parts) {
                std::vector<uint32_t> w;
                mh::CompiledTape ct;
                std::string err;
                if (compile_one(tp.data(), tp.size(), w, ct, err) != MH_OK || !ct.root_bool) {
                    ok = false;  // (register pressure of a part, say): the tape runs whole
                    break;
                }
                pw.push_back(std::move(w));
                pinfo.push_back(mh_tape_info{ct.n_nodes, ct.n_insns, ct.n_regs, ct.features, ct.alg_ops});
                pheads.push_back(mh_dev_tape{0, ct.n_insns, ct.root_bool, ct.n_regs});
            }
            if (!ok) {
                pw.resize(p0);
                pinfo.resize(p0);
                pheads.resize(p0);
                continue;
            }
            split_tab.insert(split_tab.end(), {t, n_tapes + (uint32_t)p0, (uint32_t)parts.size()});
            for (size_t i = p0; i < pw.size(); ++i) part_parent.push_back(t);
        }
        // bucket by kernel variant; instruction words laid out bucket by bucket (ascending tape
        // id inside a bucket) so that any run of consecutive bucket entries is one contiguous
        // range of words, which the kernel stages into LDS with one coalesced copy; the parts
        // after the tapes, likewise
        std::vector<char> is_split(n_tapes, 0);
        for (size_t i = 0; i < split_tab.size(); i += 3) is_split[split_tab[i]] = 1;
        std::vector<std::vector<uint32_t>> bucket(mh::kNumVariants);
        for (uint32_t t = 0; t < n_tapes; ++t)
            bucket[mh::variant_of(info[t].n_regs, info[t].features)].push_back(t);
        for (uint32_t v = 0; v < mh::kNumVariants; ++v) {
            bucket_off[v] = (uint32_t)ids.size();
            off_unsplit[v] = (uint32_t)ids_unsplit.size();
            for (uint32_t t : bucket[v]) {
                heads[t].insn_off = (uint32_t)(words.size() / 2);
                words.insert(words.end(), tw[t].begin(), tw[t].end());
                ids.push_back(t);
                if (!is_split[t]) ids_unsplit.push_back(t);
            }
        }
        bucket_off[mh::kNumVariants] = (uint32_t)ids.size();
        off_unsplit[mh::kNumVariants] = (uint32_t)ids_unsplit.size();
        std::vector<std::vector<uint32_t>> pbucket(mh::kNumVariants);
        for (uint32_t i = 0; i < (uint32_t)pw.size(); ++i)
            pbucket[mh::variant_of(pinfo[i].n_regs, pinfo[i].features)].push_back(i);
        heads.resize(n_tapes + pw.size());
        for (uint32_t v = 0; v < mh::kNumVariants; ++v) {
            off_parts[v] = (uint32_t)part_ids.size();
            for (uint32_t i : pbucket[v]) {
                heads[n_tapes + i] = pheads[i];
                heads[n_tapes + i].insn_off = (uint32_t)(words.size() / 2);
                words.insert(words.end(), pw[i].begin(), pw[i].end());
                part_ids.push_back(n_tapes + i);
            }
        }
        off_parts[mh::kNumVariants] = (uint32_t)part_ids.size();
    } catch (const std::bad_alloc&) {
        return set_err(MH_E_NOMEM, "host allocation during compile");
    }
    const auto t_compiled = tnow();
    if (dconsts.empty()) dconsts.assign(8, 0);
    if (words.empty()) words.assign(2, 0);
    // the asm core's scalar prefetch reads the 8 slots from the next instruction on (its words and
    // its inline constants): zero slots after the last tape keep those loads inside the buffer
    words.resize(words.size() + 2 * 8, 0u);
    if (int32_t r = use_device(ctx)) return r;
    mh_tapeset* ts = new (std::nothrow) mh_tapeset();
    if (!ts) return set_err(MH_E_NOMEM, "tapeset allocation");
    ts->ctx = ctx;
    ++ctx->children;
    ts->n_tapes = n_tapes;
    ts->n_vars = n_vars;
    try {
        ts->h_nodes.assign(nodes, nodes + (n_tapes ? tape_offsets[n_tapes] : 0));
        ts->h_offs.assign(tape_offsets, tape_offsets + n_tapes + 1);
        ts->h_consts.assign(consts, consts + (size_t)n_consts * 8);
    } catch (const std::bad_alloc&) {
        mh_tapes_destroy(ts);
        return set_err(MH_E_NOMEM, "host copy of the tapes");
    }
    ts->ids = std::move(ids);
    for (uint32_t v = 0; v <= mh::kNumVariants; ++v) {
        ts->bucket_off[v] = bucket_off[v];
        ts->bucket_off_unsplit[v] = off_unsplit[v];
        ts->bucket_off_parts[v] = off_parts[v];
    }
    ts->info = std::move(info);
    ts->n_parts = (uint32_t)part_parent.size();
    ts->ids_unsplit = std::move(ids_unsplit);
    ts->part_ids = std::move(part_ids);
    ts->part_parent = std::move(part_parent);
    ts->split_tab = std::move(split_tab);
    // one device block and one async copy from pinned staging (a query compiles a tape set per
    // call: four synchronous pageable copies cost more than the kernels they feed)
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    auto b_u32 = [](const std::vector<uint32_t>& v) { return std::max<size_t>(1, v.size()) * 4; };
    const size_t b_insns = words.size() * sizeof(uint32_t), b_ids = b_u32(ts->ids),
                 b_tapes = std::max<size_t>(1, heads.size()) * sizeof(mh_dev_tape),
                 b_consts = dconsts.size() * sizeof(uint32_t);
    const size_t o_ids = al(b_insns), o_tapes = o_ids + al(b_ids), o_consts = o_tapes + al(b_tapes),
                 o_unsplit = o_consts + al(b_consts), o_parts = o_unsplit + al(b_u32(ts->ids_unsplit)),
                 o_split = o_parts + al(b_u32(ts->part_ids)),
                 total = o_split + al(b_u32(ts->split_tab));
    hipError_t e = pool_alloc(ctx, (char**)&ts->d_block, total);
    if (e == hipSuccess && ctx->stage_pending) {
        e = hipEventSynchronize(ctx->stage_ev);
        ctx->stage_pending = false;
    }
    if (e == hipSuccess && total > ctx->h_stage_bytes) {
        const size_t n = std::max<size_t>({total, 2 * ctx->h_stage_bytes, (size_t)1 << 20});
        if (ctx->h_stage) (void)hipHostFree(ctx->h_stage);
        ctx->h_stage = nullptr;
        ctx->h_stage_bytes = 0;
        e = hipHostMalloc(&ctx->h_stage, n, hipHostMallocDefault);
        if (e == hipSuccess) ctx->h_stage_bytes = n;
    }
    if (e == hipSuccess && !ctx->stage_ev)
        e = hipEventCreateWithFlags(&ctx->stage_ev, hipEventDisableTiming);
    if (e == hipSuccess) {
        char* h = (char*)ctx->h_stage;
        std::memcpy(h, words.data(), b_insns);
        if (!ts->ids.empty()) std::memcpy(h + o_ids, ts->ids.data(), ts->ids.size() * sizeof(uint32_t));
        if (!heads.empty()) std::memcpy(h + o_tapes, heads.data(), heads.size() * sizeof(mh_dev_tape));
        std::memcpy(h + o_consts, dconsts.data(), b_consts);
        auto put = [&](size_t o, const std::vector<uint32_t>& v) {
            if (!v.empty()) std::memcpy(h + o, v.data(), v.size() * sizeof(uint32_t));
        };
        put(o_unsplit, ts->ids_unsplit);
        put(o_parts, ts->part_ids);
        put(o_split, ts->split_tab);
        char* d = (char*)ts->d_block;
        ts->d_insns = (uint2*)d;
        ts->d_ids = (uint32_t*)(d + o_ids);
        ts->d_tapes = (mh_dev_tape*)(d + o_tapes);
        ts->d_consts = (uint32_t*)(d + o_consts);
        ts->d_ids_unsplit = (uint32_t*)(d + o_unsplit);
        ts->d_part_ids = (uint32_t*)(d + o_parts);
        ts->d_split = (uint32_t*)(d + o_split);
        e = hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, ctx->stream);
        if (e == hipSuccess) e = hipEventRecord(ctx->stage_ev, ctx->stream);
        if (e == hipSuccess) ctx->stage_pending = true;
    }
    if (e != hipSuccess) {
        mh_tapes_destroy(ts);
        return set_err(MH_E_DEVICE, std::string("tapeset upload: ") + hipGetErrorString(e));
    }
    if (trace) {
        auto us = [](auto a, auto b) {
            return std::chrono::duration<double, std::micro>(b - a).count();
        };
        fprintf(stderr, "mh_tapes_compile: %u tapes, %zu words, compile %.1f us, upload %.1f us\n",
                n_tapes, words.size(), us(t_start, t_compiled), us(t_compiled, tnow()));
    }
    *out = ts;
    return MH_OK;
}

int32_t mh_tapes_destroy(mh_tapeset* ts) {
    if (!ts) return MH_OK;
    settle(ts->ctx);
    (void)hipSetDevice(ts->ctx->device);
    // kernels of this set may still run on the ctx stream: finish them before the blocks go back
    if (ts->ctx->stream) (void)hipStreamSynchronize(ts->ctx->stream);
    pool_free(ts->ctx, ts->d_block);
    if (ts->d_ids_rest) (void)hipFree(ts->d_ids_rest);
    for (auto& j : ts->jit) {
        if (j.mod) (void)hipModuleUnload(j.mod);
        if (j.vmod) (void)hipModuleUnload(j.vmod);
    }
    mh_ctx* ctx = ts->ctx;
    delete ts;
    ctx_unref(ctx);
    return MH_OK;
}

int32_t mh_tapes_info(const mh_tapeset* ts, mh_tape_info* info, uint32_t n_tapes) {
    if (!ts || !info) return set_err(MH_E_INVALID, "null argument");
    if (n_tapes > ts->n_tapes) return set_err(MH_E_INVALID, "n_tapes exceeds the tape set");
    std::copy(ts->info.begin(), ts->info.begin() + n_tapes, info);
    return MH_OK;
}

// Rows of padding after each column-limb.  The limbs of one row lie `stride` words apart; with
// a power-of-two stride (2^26 rows = 256 MiB) the 32 limbs a chunk loads alias in the address
// bits that pick the HBM channel.  MH_ASSIGN_PAD_ROWS overrides (A/B).
uint64_t assign_pad_rows(uint64_t capacity) {
    static const long long forced = [] {
        const char* e = std::getenv("MH_ASSIGN_PAD_ROWS");
        return e ? atoll(e) : -1ll;
    }();
    if (forced >= 0) return (uint64_t)forced;
    (void)capacity;
    return 0;
}

int32_t mh_assign_create(mh_ctx* ctx, uint32_t n_vars, uint64_t capacity, mh_assign** out) {
    if (!ctx || !out) return set_err(MH_E_INVALID, "null argument");
    *out = nullptr;
    if (n_vars == 0 || capacity == 0) return set_err(MH_E_INVALID, "empty assignment buffer");
    if (int32_t r = use_device(ctx)) return r;
    mh_assign* as = new (std::nothrow) mh_assign();
    if (!as) return set_err(MH_E_NOMEM, "assign allocation");
    as->ctx = ctx;
    ++ctx->children;
    as->n_vars = n_vars;
    as->capacity = capacity;
    as->stride = capacity + assign_pad_rows(capacity);
    hipError_t e = hipMalloc(&as->d, (size_t)n_vars * 8 * as->stride * sizeof(uint32_t));
    if (e != hipSuccess) {
        mh_assign_destroy(as);
        return set_err(MH_E_NOMEM, std::string("assignment buffer: ") + hipGetErrorString(e));
    }
    *out = as;
    return MH_OK;
}

int32_t mh_assign_destroy(mh_assign* as) {
    if (!as) return MH_OK;
    settle(as->ctx);
    (void)hipSetDevice(as->ctx->device);
    if (as->staged_pending) (void)hipEventSynchronize(as->staged);
    if (as->staged) (void)hipEventDestroy(as->staged);
    if (as->h_pinned) (void)hipHostFree(as->h_pinned);
    if (as->d) (void)hipFree(as->d);
    if (as->d_guide) (void)hipFree(as->d_guide);
    mh_ctx* ctx = as->ctx;
    delete as;
    ctx_unref(ctx);
    return MH_OK;
}

int32_t mh_assign_upload(mh_assign* as, const uint32_t* host_soa, uint64_t first, uint64_t count) {
    if (!as || (!host_soa && count)) return set_err(MH_E_INVALID, "null argument");
    if (first > as->capacity || count > as->capacity - first)
        return set_err(MH_E_INVALID, "row range out of bounds");
    if (int32_t r = use_device(as->ctx)) return r;
    if (count == 0) return MH_OK;
    // one strided copy into every column-limb's [first, first + count) slice: a definitions
    // evaluation uploads one row, which one copy per column-limb made 0.15 ms (profiles/r04z)
    MH_HIP(hipMemcpy2DAsync(as->d + first, as->stride * sizeof(uint32_t), host_soa,
                            count * sizeof(uint32_t), count * sizeof(uint32_t),
                            (size_t)as->n_vars * 8, hipMemcpyHostToDevice, as->ctx->stream));
    MH_HIP(hipStreamSynchronize(as->ctx->stream));
    return MH_OK;
}

int32_t mh_assign_download(const mh_assign* as, uint32_t* host_soa, uint64_t first,
                           uint64_t count) {
    if (!as || (!host_soa && count)) return set_err(MH_E_INVALID, "null argument");
    if (first > as->capacity || count > as->capacity - first)
        return set_err(MH_E_INVALID, "row range out of bounds");
    if (int32_t r = use_device(as->ctx)) return r;
    if (count == 0) return MH_OK;
    // one strided copy of every column-limb's [first, first + count) slice (a query reads one
    // witness row: one call instead of one per column-limb)
    MH_HIP(hipMemcpy2DAsync(host_soa, count * sizeof(uint32_t), as->d + first,
                            as->stride * sizeof(uint32_t), count * sizeof(uint32_t),
                            (size_t)as->n_vars * 8, hipMemcpyDeviceToHost, as->ctx->stream));
    MH_HIP(hipStreamSynchronize(as->ctx->stream));
    return MH_OK;
}

int32_t mh_assign_generate(mh_assign* as, uint64_t seed, uint64_t global_base) {
    if (!as) return set_err(MH_E_INVALID, "null handle");
    if (int32_t r = use_device(as->ctx)) return r;
    MH_HIP(mh::launch_generate(as->d, as->stride, as->capacity, as->n_vars, seed, global_base,
                               as->ctx->stream));
    return MH_OK;
}

int32_t mh_assign_generate_guided(mh_assign* as, uint64_t seed, uint64_t global_base,
                                  uint64_t first, uint64_t count, const mh_guide* g) {
    if (!as || !g) return set_err(MH_E_INVALID, "null argument");
    if (first > as->capacity || count > as->capacity - first)
        return set_err(MH_E_INVALID, "row range out of bounds");
    if (g->n_cols > as->n_vars) return set_err(MH_E_INVALID, "guide has more columns than the buffer");
    if (g->n_cols && (!g->col_width || !g->pool_off))
        return set_err(MH_E_INVALID, "guide: null column arrays");
    if (g->n_sets && (!g->set_prob || !g->set_off || !g->alt_off))
        return set_err(MH_E_INVALID, "guide: null set arrays");
    // validate every offset and entry on the host: the kernel trusts them
    const uint32_t nc = g->n_cols, ns = g->n_sets;
    if (nc && g->pool_off[0] != 0) return set_err(MH_E_INVALID, "guide: pool_off[0] != 0");
    for (uint32_t v = 0; v < nc; ++v) {
        if (g->col_width[v] < 1 || g->col_width[v] > 256)
            return set_err(MH_E_INVALID, "guide: column width outside 1..256");
        if (g->pool_off[v + 1] < g->pool_off[v])
            return set_err(MH_E_INVALID, "guide: pool_off not monotone");
    }
    const uint32_t n_pool = nc ? g->pool_off[nc] : 0;
    if (n_pool && !g->pool) return set_err(MH_E_INVALID, "guide: null pool");
    const uint32_t n_alts = ns ? g->set_off[ns] : 0;
    if (ns && g->set_off[0] != 0) return set_err(MH_E_INVALID, "guide: set_off[0] != 0");
    for (uint32_t j = 0; j < ns; ++j)
        if (g->set_off[j + 1] < g->set_off[j])
            return set_err(MH_E_INVALID, "guide: set_off not monotone");
    if (ns && g->alt_off[0] != 0) return set_err(MH_E_INVALID, "guide: alt_off[0] != 0");
    for (uint32_t a = 0; a < n_alts; ++a)
        if (g->alt_off[a + 1] < g->alt_off[a])
            return set_err(MH_E_INVALID, "guide: alt_off not monotone");
    const uint32_t n_ent = ns ? g->alt_off[n_alts] : 0;
    if (n_ent && (!g->entry_col || !g->entry_val))
        return set_err(MH_E_INVALID, "guide: null entry arrays");
    // the leading sets without a copy entry (the kernel resolves their writes in LDS)
    uint32_t n_value_sets = 0;
    for (bool copy = false; n_value_sets < ns && !copy; ) {
        for (uint32_t e = g->alt_off[g->set_off[n_value_sets]];
             e < g->alt_off[g->set_off[n_value_sets + 1]] && !copy; ++e)
            copy = (g->entry_col[e] & MH_GUIDE_COPY) != 0;
        if (!copy) ++n_value_sets;
    }
    for (uint32_t e = 0; e < n_ent; ++e) {
        const uint32_t c = g->entry_col[e];
        const uint32_t dst = c & ~MH_GUIDE_COPY;
        if (dst >= nc) return set_err(MH_E_INVALID, "guide: entry column out of range");
        if (c & MH_GUIDE_COPY) {
            const uint32_t* ev = g->entry_val + (size_t)e * 8;
            if (ev[0] >= nc || ev[3] < 1 || ev[3] > 256 || ev[1] >= 256 || ev[2] >= 256)
                return set_err(MH_E_INVALID, "guide: malformed copy entry");
        }
    }
    if (int32_t r = use_device(as->ctx)) return r;
    // pack: width | pool_off | pool | set_prob | set_off | alt_off | entry_col | entry_val
    const size_t o_width = 0, o_poff = o_width + nc, o_pool = o_poff + nc + 1,
                 o_prob = o_pool + (size_t)n_pool * 8, o_soff = o_prob + ns,
                 o_aoff = o_soff + ns + 1, o_ecol = o_aoff + n_alts + 1,
                 o_eval = o_ecol + n_ent, words = o_eval + (size_t)n_ent * 8;
    std::vector<uint32_t>& h = as->h_guide;
    h.assign(words, 0);
    for (uint32_t v = 0; v < nc; ++v) h[o_width + v] = g->col_width[v];
    if (nc) std::copy(g->pool_off, g->pool_off + nc + 1, h.begin() + o_poff);
    if (n_pool) std::copy(g->pool, g->pool + (size_t)n_pool * 8, h.begin() + o_pool);
    for (uint32_t j = 0; j < ns; ++j) h[o_prob + j] = g->set_prob[j];
    if (ns) {
        std::copy(g->set_off, g->set_off + ns + 1, h.begin() + o_soff);
        std::copy(g->alt_off, g->alt_off + n_alts + 1, h.begin() + o_aoff);
    }
    if (n_ent) {
        std::copy(g->entry_col, g->entry_col + n_ent, h.begin() + o_ecol);
        std::copy(g->entry_val, g->entry_val + (size_t)n_ent * 8, h.begin() + o_eval);
    }
    // both buffers grow geometrically: a LASER child's guide is a little larger than its
    // parent's, and a pinned reallocation per query cost ~0.24 ms (hipHostFree 0.19 +
    // hipHostMalloc 0.05, EtherThief-400, profiles/r05o/htrace)
    const size_t grow = std::max<size_t>({words, 2 * as->guide_words, (size_t)1 << 14});
    if (words > as->guide_words) {
        if (as->d_guide) MH_HIP(hipFree(as->d_guide));
        as->d_guide = nullptr;
        as->guide_words = 0;
        MH_HIP(hipMalloc(&as->d_guide, grow * sizeof(uint32_t)));
        as->guide_words = grow;
    }
    // pinned staging: the async copy needs no stream sync; the next call's packing waits on
    // the event of this copy before it overwrites the staging buffer
    if (as->staged_pending) {
        MH_HIP(hipEventSynchronize(as->staged));
        as->staged_pending = false;
    }
    if (words > as->pinned_words) {
        const size_t pgrow = std::max<size_t>({words, 2 * as->pinned_words, (size_t)1 << 14});
        if (as->h_pinned) MH_HIP(hipHostFree(as->h_pinned));
        as->h_pinned = nullptr;
        as->pinned_words = 0;
        MH_HIP(hipHostMalloc(&as->h_pinned, pgrow * sizeof(uint32_t), hipHostMallocDefault));
        as->pinned_words = pgrow;
    }
    if (!as->staged) MH_HIP(hipEventCreateWithFlags(&as->staged, hipEventDisableTiming));
    std::memcpy(as->h_pinned, h.data(), words * sizeof(uint32_t));
    MH_HIP(hipMemcpyAsync(as->d_guide, as->h_pinned, words * sizeof(uint32_t),
                          hipMemcpyHostToDevice, as->ctx->stream));
    MH_HIP(hipEventRecord(as->staged, as->ctx->stream));
    as->staged_pending = true;
    mh::KGuide k;
    k.n_cols = nc;
    k.n_sets = ns;
    k.n_value_sets = n_value_sets;
    k.width = as->d_guide + o_width;
    k.pool_off = as->d_guide + o_poff;
    k.pool = as->d_guide + o_pool;
    k.set_prob = as->d_guide + o_prob;
    k.set_off = as->d_guide + o_soff;
    k.alt_off = as->d_guide + o_aoff;
    k.entry_col = as->d_guide + o_ecol;
    k.entry_val = as->d_guide + o_eval;
    k.span_words = (uint32_t)(o_eval - o_prob);
    MH_HIP(mh::launch_generate_guided(as->d, as->stride, first, count, seed, global_base, k,
                                      as->ctx->stream));
    return MH_OK;
}

uint32_t mh_gen_limb(uint64_t seed, uint32_t var, uint64_t index, uint32_t limb) {
    const uint64_t key = splitmix64(seed ^ (((uint64_t)var * 8 + limb) * 0xD1B54A32D192ED03ull));
    return (uint32_t)splitmix64(key ^ index);
}

int32_t mh_results_reset(mh_ctx* ctx, uint64_t* d_first_hit, uint64_t* d_hit_count, uint32_t n) {
    if (!ctx) return set_err(MH_E_INVALID, "null ctx");
    if (int32_t r = use_device(ctx)) return r;
    // one small kernel for both arrays (two hipMemsetAsync were two fill launches per run)
    MH_HIP(mh::launch_results_reset(d_first_hit, d_hit_count, n, ctx->stream));
    return MH_OK;
}

// A complex-op interpreter tape over a buffer of 2^30 rows per column or more (kernels.h).
static int32_t refuse_capacity(uint64_t capacity) {
    return set_err(MH_E_UNSUPPORTED,
                   "interpreter tapes with complex ops (keccak, EVM helpers, overflow predicates, "
                   "loaded columns) address < 2^30 rows per column; this buffer's stride is " +
                   std::to_string(capacity) + " rows");
}

int32_t mh_run_async(mh_ctx* ctx, const mh_tapeset* ts, uint32_t tape_first, uint32_t tape_count,
                     const mh_assign* as, uint64_t row_first, uint64_t row_count,
                     uint64_t index_base, uint32_t mode, uint64_t* d_first_hit,
                     uint64_t* d_hit_count) {
    if (int32_t r = check_run_args(ctx, ts, tape_first, tape_count, as, row_first, row_count, mode))
        return r;
    if (int32_t r = use_device(ctx)) return r;
    mh::KParams p = make_params(ts, tape_first, as, row_first, row_count, index_base, mode);
    p.first_hit = reinterpret_cast<unsigned long long*>(d_first_hit);
    p.hit_count = reinterpret_cast<unsigned long long*>(d_hit_count);
    // the native code takes the jitted tapes of a whole-set run; the interpreter the rest
    const bool use_jit = ts->has_jit && tape_first == 0 && tape_count == ts->n_tapes;
    // a short interpreter run over a set with split tapes runs their parts instead (conjunct-
    // parallel: each part is a tape of its own, its waves write Bool masks, the combine kernel
    // ANDs them per split tape); MH_SPLIT_ROWS = the largest such run
    static const uint64_t split_rows = [] {
        const char* e = std::getenv("MH_SPLIT_ROWS");
        return e ? std::strtoull(e, nullptr, 10) : 65536ull;
    }();
    const bool split = !use_jit && ts->n_parts && row_count <= split_rows;
    const std::vector<uint32_t>& ids = use_jit ? ts->ids_rest : split ? ts->ids_unsplit : ts->ids;
    const uint32_t* boff = use_jit ? ts->bucket_off_rest
                                   : split ? ts->bucket_off_unsplit : ts->bucket_off;
    uint32_t* d_ids = use_jit ? ts->d_ids_rest : split ? ts->d_ids_unsplit : ts->d_ids;
    // the interpreter's tapes of each kernel-variant bucket inside the requested range
    const uint32_t *lo[mh::kNumVariants], *hi[mh::kNumVariants];
    for (uint32_t v = 0; v < mh::kNumVariants; ++v) {
        const uint32_t* b = ids.data() + boff[v];
        const uint32_t* e = ids.data() + boff[v + 1];
        lo[v] = std::lower_bound(b, e, tape_first);
        hi[v] = std::lower_bound(lo[v], e, tape_first + tape_count);
        // refused before anything is launched
        if (hi[v] != lo[v] && !mh::variant_fits(v, p.capacity)) return refuse_capacity(p.capacity);
    }
    // the split tapes inside the range (split_tab ascends by tape, part ids with it) and their
    // parts per bucket
    uint32_t s_lo = 0, s_hi = 0, part_lo = 0, part_hi = 0;
    const uint32_t *plo[mh::kNumVariants] = {}, *phi[mh::kNumVariants] = {};
    if (split) {
        const uint32_t n_split = (uint32_t)ts->split_tab.size() / 3;
        while (s_lo < n_split && ts->split_tab[3 * s_lo] < tape_first) ++s_lo;
        s_hi = s_lo;
        while (s_hi < n_split && ts->split_tab[3 * s_hi] < tape_first + tape_count) ++s_hi;
        if (s_hi > s_lo) {
            part_lo = ts->split_tab[3 * s_lo + 1];
            part_hi = ts->split_tab[3 * (s_hi - 1) + 1] + ts->split_tab[3 * (s_hi - 1) + 2];
        }
        for (uint32_t v = 0; v < mh::kNumVariants; ++v) {
            const uint32_t* b = ts->part_ids.data() + ts->bucket_off_parts[v];
            const uint32_t* e = ts->part_ids.data() + ts->bucket_off_parts[v + 1];
            plo[v] = std::lower_bound(b, e, part_lo);
            phi[v] = std::lower_bound(plo[v], e, part_hi);
            if (phi[v] != plo[v] && !mh::variant_fits(v, p.capacity)) return refuse_capacity(p.capacity);
        }
    }
    const uint64_t mask_stride = mh::sieve_mask_stride(row_count);
    if (part_hi > part_lo) {
        const size_t need = (size_t)(part_hi - part_lo) * mask_stride * sizeof(unsigned long long);
        if (need > ctx->masks_bytes) {
            if (ctx->d_masks) MH_HIP(hipFree(ctx->d_masks));
            ctx->d_masks = nullptr;
            ctx->masks_bytes = 0;
            size_t n = 1 << 16;
            while (n < need) n <<= 1;
            MH_HIP(hipMalloc(&ctx->d_masks, n));
            ctx->masks_bytes = n;
        }
    }
    std::pair<hipEvent_t, hipEvent_t> sp{nullptr, nullptr};
    if (ctx->timing) {
        MH_HIP(hipEventCreate(&sp.first));
        MH_HIP(hipEventCreate(&sp.second));
        ctx->spans.push_back(sp);
        MH_HIP(hipEventRecord(sp.first, ctx->stream));
    }
    if (use_jit && row_count) {
        if (int32_t r = launch_jit(ctx, ts, as, row_first, row_count, index_base, mode,
                                   d_first_hit, d_hit_count, nullptr))
            return r;
    }
    // one launch per kernel-variant bucket; a short run (a query's guided first round) is one
    // launch per register class instead: the feature sets nest (kernels.h variant_of: a kernel
    // with more handlers runs a tape that needs fewer), the register classes do not (a tape's
    // instruction words address its class's registers), and a class's buckets are consecutive
    // in the id list, which is laid out in the order of the tapes' words
    static const uint64_t merge_rows = [] {
        const char* e = std::getenv("MH_MERGE_ROWS");
        return e ? std::strtoull(e, nullptr, 10) : 4096ull;
    }();
    // (over the whole set only: every bucket is then whole, so a class's buckets are one range)
    const bool merge = !use_jit && row_count <= merge_rows && tape_first == 0 &&
                       tape_count == ts->n_tapes;
    struct Launch { const uint32_t *b, *e; uint32_t variant; bool part; };
    Launch launches[2 * mh::kNumVariants];
    uint32_t n_launch = 0;
    for (int part = 0; part < 2; ++part) {
        const uint32_t* const* L = part ? plo : lo;
        const uint32_t* const* H = part ? phi : hi;
        if (part && !split) break;
        for (uint32_t v = 0; v < mh::kNumVariants; ++v) {
            if (H[v] == L[v]) continue;
            uint32_t last = v;  // with merging: the class's last nonempty bucket, L[v]..H[last]
            if (merge)
                for (uint32_t u = v + 1; u < (v / 4 + 1) * 4; ++u)
                    if (H[u] != L[u]) last = u;
            launches[n_launch++] = Launch{L[v], H[last], last, part != 0};
            v = last;
        }
    }
    // a short run's launches overlap on the side streams (made with the ctx when the fan-out
    // is on); the results they write are disjoint (per tape / per part), and the join puts
    // everything after them back in `stream`'s order
    const uint32_t n_side = fanout_enabled() && (merge || split)
                                ? std::min(n_launch - (n_launch > 0), kSideStreams) : 0;
    if (n_side) {
        MH_HIP(hipEventRecord(ctx->fork_ev, ctx->stream));
        for (uint32_t i = 0; i < n_side; ++i) MH_HIP(hipStreamWaitEvent(ctx->side[i], ctx->fork_ev, 0));
    }
    for (uint32_t i = 0; i < n_launch; ++i) {
        mh::KParams q = p;
        if (launches[i].part) {  // wave masks instead of results
            q.tape_ids = ts->d_part_ids + (launches[i].b - ts->part_ids.data());
            q.masks = ctx->d_masks;
            q.mask_base = part_lo;
            q.mask_stride = mask_stride;
            q.first_hit = nullptr;
            q.hit_count = nullptr;
        } else {
            q.tape_ids = d_ids + (launches[i].b - ids.data());
        }
        q.n_ids = (uint32_t)(launches[i].e - launches[i].b);
        // launch 0 on the ctx stream, the others round-robin over the side streams
        hipStream_t s = n_side && i ? ctx->side[(i - 1) % n_side] : ctx->stream;
        MH_HIP(mh::launch_sieve(q, launches[i].variant, s));
    }
    for (uint32_t i = 0; i < n_side; ++i) {
        MH_HIP(hipEventRecord(ctx->join_ev[i], ctx->side[i]));
        MH_HIP(hipStreamWaitEvent(ctx->stream, ctx->join_ev[i], 0));
    }
    if (s_hi > s_lo)  // every part's masks written: the split tapes' results
        MH_HIP(mh::launch_combine(ctx->d_masks, mask_stride, ts->d_split + 3 * s_lo, s_hi - s_lo,
                                  part_lo, tape_first, index_base + row_first, p.first_hit,
                                  p.hit_count, ctx->stream));
    if (ctx->timing) MH_HIP(hipEventRecord(sp.second, ctx->stream));
    return MH_OK;
}

int32_t mh_run_rows(mh_ctx* ctx, const mh_tapeset* ts, uint32_t tape_first, uint32_t tape_count,
                    const mh_assign* as, uint64_t row_first, uint64_t row_count,
                    uint64_t index_base, uint32_t mode, uint64_t* first_hit, uint64_t* hit_count,
                    uint32_t n_cols, uint32_t* rows_out) {
    if (int32_t r = check_run_args(ctx, ts, tape_first, tape_count, as, row_first, row_count, mode))
        return r;
    if (n_cols && (!rows_out || n_cols > as->n_vars))
        return set_err(MH_E_INVALID, "mh_run_rows: rows_out null or n_cols beyond the buffer's columns");
    if (int32_t r = use_device(ctx)) return r;
    const size_t n = std::max<uint32_t>(tape_count, 1);
    const size_t res_bytes = 2 * n * sizeof(uint64_t);
    const size_t row_bytes = (size_t)tape_count * n_cols * 8 * sizeof(uint32_t);
    void* dv = nullptr;
    void* hv = nullptr;
    MH_HIP(ctx_dbuf(ctx, res_bytes + row_bytes, &dv));
    MH_HIP(ctx_hbuf(ctx, res_bytes + row_bytes, &hv));
    uint64_t* d = static_cast<uint64_t*>(dv);
    uint64_t* h = static_cast<uint64_t*>(hv);
    int32_t r = mh_results_reset(ctx, d, d + n, (uint32_t)n);
    if (r == MH_OK)
        r = mh_run_async(ctx, ts, tape_first, tape_count, as, row_first, row_count, index_base,
                         mode, d, d + n);
    hipError_t e = hipSuccess;
    if (r == MH_OK && row_bytes)
        e = mh::launch_witness_rows(as->d, as->stride, d, tape_count, index_base, n_cols,
                                    reinterpret_cast<uint32_t*>(d + 2 * n), ctx->stream);
    if (r == MH_OK && e == hipSuccess)  // results and rows in one copy into pinned memory
        e = hipMemcpyAsync(h, d, res_bytes + row_bytes, hipMemcpyDeviceToHost, ctx->stream);
    if (r == MH_OK && e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (r == MH_OK && e == hipSuccess && first_hit && tape_count)
        std::memcpy(first_hit, h, tape_count * sizeof(uint64_t));
    if (r == MH_OK && e == hipSuccess && hit_count && tape_count)
        std::memcpy(hit_count, h + n, tape_count * sizeof(uint64_t));
    if (r == MH_OK && e == hipSuccess && row_bytes) std::memcpy(rows_out, h + 2 * n, row_bytes);
    if (r != MH_OK) return r;
    if (e != hipSuccess) return set_err(MH_E_DEVICE, std::string("mh_run: ") + hipGetErrorString(e));
    return MH_OK;
}

int32_t mh_run(mh_ctx* ctx, const mh_tapeset* ts, uint32_t tape_first, uint32_t tape_count,
               const mh_assign* as, uint64_t row_first, uint64_t row_count, uint64_t index_base,
               uint32_t mode, uint64_t* first_hit, uint64_t* hit_count) {
    return mh_run_rows(ctx, ts, tape_first, tape_count, as, row_first, row_count, index_base, mode,
                       first_hit, hit_count, 0, nullptr);
}

int32_t mh_query_round(mh_ctx* ctx, const mh_tapeset* ts, mh_assign* as, const mh_guide* guide,
                       uint64_t seed, uint64_t global_base, uint64_t count, uint32_t tape_first,
                       uint32_t tape_count, uint32_t mode, uint64_t* first_hit,
                       uint64_t* hit_count, uint32_t n_cols, uint32_t* rows_out) {
    if (!ctx || !as || as->ctx != ctx) return set_err(MH_E_INVALID, "null or foreign assignment buffer");
    if (int32_t r = check_run_args(ctx, ts, tape_first, tape_count, as, 0, count, mode)) return r;
    // the generator, the run and the copy queue back to back on the ctx stream: one host sync
    if (int32_t r = mh_assign_generate_guided(as, seed, global_base, 0, count, guide)) return r;
    return mh_run_rows(ctx, ts, tape_first, tape_count, as, 0, count, global_base, mode, first_hit,
                       hit_count, n_cols, rows_out);
}

int32_t mh_eval_values(mh_ctx* ctx, const mh_tapeset* ts, uint32_t tape, const mh_assign* as,
                       uint64_t row_first, uint64_t row_count, uint32_t* out) {
    if (int32_t r = check_run_args(ctx, ts, tape, 1, as, row_first, row_count, MH_MODE_COUNT_ALL))
        return r;
    if (!out && row_count) return set_err(MH_E_INVALID, "null out");
    if (row_count == 0) return MH_OK;
    if (int32_t r = use_device(ctx)) return r;
    const uint32_t variant = mh::variant_of(ts->info[tape].n_regs, ts->info[tape].features);
    if (!mh::variant_fits(variant, as->stride)) return refuse_capacity(as->stride);
    // the production sieve kernel in values mode, over a one-tape list
    uint32_t* d = nullptr;
    MH_HIP(hipMalloc(&d, (8 * row_count + 8) * sizeof(uint32_t)));
    uint32_t* d_id = d + 8 * row_count;  // [0]: tape id, [2..5]: first_hit / hit_count
    mh::KParams p = make_params(ts, tape, as, row_first, row_count, 0, MH_MODE_COUNT_ALL);
    p.tape_ids = d_id;
    p.n_ids = 1;
    p.first_hit = reinterpret_cast<unsigned long long*>(d_id + 2);
    p.hit_count = reinterpret_cast<unsigned long long*>(d_id + 4);
    p.values_out = d;
    // copies on the ctx stream: the first use of the null stream creates a hardware queue
    // (20.6 ms, profiles/r04x), which a query's first definitions evaluation paid
    const uint32_t ids[8] = {tape, 0, 0xFFFFFFFFu, 0xFFFFFFFFu, 0, 0, 0, 0};
    hipError_t e = hipMemcpyAsync(d_id, ids, sizeof(ids), hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess)
        e = mh::launch_sieve(p, variant, ctx->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(out, d, 8 * row_count * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    (void)hipFree(d);
    if (e != hipSuccess)
        return set_err(MH_E_DEVICE, std::string("mh_eval_values: ") + hipGetErrorString(e));
    return MH_OK;
}

int32_t mh_eval_values_many(mh_ctx* ctx, const mh_tapeset* ts, const uint32_t* tapes,
                            uint32_t n, const mh_assign* as, uint64_t row, uint32_t* out) {
    if (int32_t r = check_run_args(ctx, ts, 0, 0, as, row, 1, MH_MODE_COUNT_ALL)) return r;
    if (n == 0) return MH_OK;
    if (!tapes || !out) return set_err(MH_E_INVALID, "null tapes / out");
    uint32_t top = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (tapes[i] >= ts->n_tapes) return set_err(MH_E_INVALID, "tape id out of bounds");
        top = std::max(top, tapes[i]);
    }
    if (int32_t r = use_device(ctx)) return r;
    // one launch of the production sieve kernel in values mode per register-class variant: the
    // listed tapes of a variant are its id list, their values land at [position][8] (one row)
    std::vector<std::pair<uint32_t, uint32_t>> by_var;  // (variant, position in `tapes`)
    by_var.reserve(n);
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t v = mh::variant_of(ts->info[tapes[i]].n_regs, ts->info[tapes[i]].features);
        if (!mh::variant_fits(v, as->stride)) return refuse_capacity(as->stride);
        by_var.push_back({v, i});
    }
    std::stable_sort(by_var.begin(), by_var.end(),
                     [](const auto& a, const auto& b) { return a.first < b.first; });
    // device block: values [n][8], ids [n], first_hit / hit_count [top + 1] each (scratch: the
    // kernel's count-mode bookkeeping, indexed by tape id)
    const size_t n_words = (size_t)8 * n + n + 4 * ((size_t)top + 1) + 2;
    std::vector<uint32_t> h(n + 4 * ((size_t)top + 1) + 2, 0u);
    for (uint32_t i = 0; i < n; ++i) h[i] = tapes[by_var[i].second];
    // the ctx's grow-only result buffer (stream-ordered after any earlier use of it)
    void* dv = nullptr;
    MH_HIP(ctx_dbuf(ctx, n_words * sizeof(uint32_t), &dv));
    uint32_t* d = static_cast<uint32_t*>(dv);
    uint32_t* d_ids = d + 8 * (size_t)n;
    uint32_t* d_res = d_ids + n + ((n & 1) ? 1 : 0);  // 8-byte aligned
    hipError_t e = hipMemcpyAsync(d_ids, h.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice,
                                  ctx->stream);
    if (e == hipSuccess)
        e = hipMemsetAsync(d_res, 0xFF, 2 * ((size_t)top + 1) * sizeof(uint32_t), ctx->stream);
    if (e == hipSuccess)
        e = hipMemsetAsync(d_res + 2 * ((size_t)top + 1), 0, 2 * ((size_t)top + 1) * sizeof(uint32_t),
                           ctx->stream);
    uint32_t launches = 0;
    for (uint32_t i = 0; i < n && e == hipSuccess;) {
        uint32_t j = i;
        while (j < n && by_var[j].first == by_var[i].first) ++j;
        mh::KParams p = make_params(ts, 0, as, row, 1, 0, MH_MODE_COUNT_ALL);
        p.tape_ids = d_ids + i;
        p.n_ids = j - i;
        p.first_hit = reinterpret_cast<unsigned long long*>(d_res);
        p.hit_count = reinterpret_cast<unsigned long long*>(d_res + 2 * ((size_t)top + 1));
        p.values_out = d + 8 * (size_t)i;
        e = mh::launch_sieve(p, by_var[i].first, ctx->stream);
        ++launches;
        i = j;
    }
    std::vector<uint32_t> vals((size_t)8 * n);
    if (e == hipSuccess)
        e = hipMemcpyAsync(vals.data(), d, vals.size() * sizeof(uint32_t), hipMemcpyDeviceToHost,
                           ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess)
        return set_err(MH_E_DEVICE, std::string("mh_eval_values_many: ") + hipGetErrorString(e));
    for (uint32_t i = 0; i < n; ++i)
        std::memcpy(out + 8 * (size_t)by_var[i].second, vals.data() + 8 * (size_t)i,
                    8 * sizeof(uint32_t));
    ctx->eval_launches += launches;
    return MH_OK;
}

int32_t mh_ctx_eval_launches(const mh_ctx* ctx, uint64_t* launches) {
    if (!ctx || !launches) return set_err(MH_E_INVALID, "null argument");
    *launches = ctx->eval_launches;
    return MH_OK;
}

int32_t mh_tapes_jit(mh_tapeset* ts, uint32_t flags, uint32_t max_vgpr) {
    if (!ts) return set_err(MH_E_INVALID, "null tapeset");
    if (ts->has_jit) return set_err(MH_E_INVALID, "tapeset already has native code");
    if (int32_t r = use_device(ts->ctx)) return r;
    const auto t0 = std::chrono::steady_clock::now();
    mh::jit::Options opt;
    opt.max_vgpr = max_vgpr ? max_vgpr : 128;
    opt.short_circuit = (flags & MH_JIT_FULL_EVAL) == 0;
    if (const char* e = std::getenv("MH_JIT_SC")) opt.short_circuit = opt.short_circuit && atoi(e) != 0;
    // gfx950 has 256 architectural VGPRs per wave (an allocation above it would only fail later,
    // in the assembler)
    if (opt.max_vgpr > 256 || opt.max_vgpr < 96) return set_err(MH_E_INVALID, "max_vgpr outside 96..256");
    // build threads = code objects per occupancy class = launches per run: 4 (MI355X, config 5,
    // profiles/r02y: 16 objects 3.195e11 evals/s, 4 3.222e11, 1 3.226e11 -- each launch drains
    // its tail before the next starts; 4 keeps the emission and assembly parallel)
    const uint32_t threads = mh::jit::default_threads();
    std::vector<mh::jit::Built> built;
    mh::jit::BuildStats stats;
    std::string err;
    bool ok;
    try {
        ok = mh::jit::build_tapeset(ts->h_nodes.data(), ts->h_offs.data(), ts->n_tapes,
                                    ts->h_consts.data(), (uint32_t)(ts->h_consts.size() / 8),
                                    ts->n_vars, (flags & MH_JIT_VALUES) != 0, opt, threads, built,
                                    stats, err);
    } catch (const std::bad_alloc&) {
        return set_err(MH_E_NOMEM, "host allocation during JIT build");
    }
    if (!ok) return set_err(MH_E_UNSUPPORTED, "JIT: " + err);
    const uint64_t code_id = mh::jit::code_id(built);
    std::vector<mh_tapeset::JitMod> mods;
    mods.reserve(built.size());
    auto unload = [&]() {
        for (auto& j : mods) {
            if (j.mod) (void)hipModuleUnload(j.mod);
            if (j.vmod) (void)hipModuleUnload(j.vmod);
        }
    };
    uint32_t maxv = 0;
    for (auto& b : built) {
        if (b.hsaco.empty()) continue;
        mods.emplace_back();
        mh_tapeset::JitMod& j = mods.back();
        j.n_groups = b.n_groups;
        j.image.swap(b.hsaco);
        j.vimage.swap(b.hsaco_values);
        hipError_t e = hipModuleLoadData(&j.mod, j.image.data());
        if (e == hipSuccess) e = hipModuleGetFunction(&j.fn, j.mod, "mh_jit");
        if (e == hipSuccess && !j.vimage.empty()) {
            e = hipModuleLoadData(&j.vmod, j.vimage.data());
            if (e == hipSuccess) e = hipModuleGetFunction(&j.vfn, j.vmod, "mh_jit");
        }
        if (e != hipSuccess) {
            unload();
            return set_err(MH_E_DEVICE, std::string("JIT module load: ") + hipGetErrorString(e));
        }
        maxv = std::max(maxv, b.max_vgpr);
    }
    // the interpreter's buckets without the jitted tapes
    std::vector<uint32_t> rest;
    uint32_t boff[mh::kNumVariants + 1];
    for (uint32_t v = 0; v < mh::kNumVariants; ++v) {
        boff[v] = (uint32_t)rest.size();
        for (uint32_t i = ts->bucket_off[v]; i < ts->bucket_off[v + 1]; ++i)
            if (!stats.jitted[ts->ids[i]]) rest.push_back(ts->ids[i]);
    }
    boff[mh::kNumVariants] = (uint32_t)rest.size();
    uint32_t* d_rest = nullptr;
    hipError_t e = hipMalloc(&d_rest, std::max<size_t>(1, rest.size()) * sizeof(uint32_t));
    if (e == hipSuccess && !rest.empty())
        e = hipMemcpy(d_rest, rest.data(), rest.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        if (d_rest) (void)hipFree(d_rest);
        unload();
        return set_err(MH_E_DEVICE, std::string("JIT bucket upload: ") + hipGetErrorString(e));
    }
    ts->jit = std::move(mods);
    ts->jitted = stats.jitted;
    ts->ids_rest = std::move(rest);
    std::copy(boff, boff + mh::kNumVariants + 1, ts->bucket_off_rest);
    ts->d_ids_rest = d_rest;
    ts->has_jit = true;
    ts->code_id = code_id;
    mh_jit_info& ji = ts->jinfo;
    ji = mh_jit_info{};
    for (uint8_t x : stats.jitted) ji.n_jitted += x;
    for (const auto& j : ts->jit) ji.n_groups += j.n_groups;
    ji.n_modules = (uint32_t)ts->jit.size();
    ji.max_vgpr = maxv;
    ji.code_bytes = stats.code_bytes;
    ji.valu_static = stats.valu_static;
    ji.valu_wide_static = stats.valu_wide_static;
    ji.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return MH_OK;
}

int32_t mh_tapes_jit_code_id(const mh_tapeset* ts, uint64_t* out) {
    if (!ts || !out) return set_err(MH_E_INVALID, "null argument");
    if (!ts->has_jit) return set_err(MH_E_INVALID, "no native code (mh_tapes_jit first)");
    *out = ts->code_id;
    return MH_OK;
}

int32_t mh_jit_code_id(const mh_node* nodes, const uint64_t* tape_offsets, uint32_t n_tapes,
                       const uint32_t* consts, uint32_t n_consts, uint32_t n_vars,
                       uint32_t flags, uint32_t max_vgpr, uint64_t* out) {
    if (!out || (n_tapes && (!nodes || !tape_offsets)) || (n_consts && !consts))
        return set_err(MH_E_INVALID, "null argument");
    // the same validation mh_tapes_compile gives a tape set (the JIT reads only checked IR)
    try {
        std::vector<uint32_t> dconsts, w;
        mh::ConstIndex dindex;
        for (uint32_t t = 0; t < n_tapes; ++t) {
            const uint64_t b = tape_offsets[t], e = tape_offsets[t + 1];
            if (e <= b) return set_err(MH_E_INVALID, "tape " + std::to_string(t) + " is empty");
            mh::CompiledTape ct;
            std::string err;
            w.clear();
            const int32_t r = mh::compile_tape(nodes + b, (size_t)(e - b), consts, n_consts,
                                               n_vars, dconsts, dindex, w, ct, err);
            if (r != MH_OK) return set_err(r, "tape " + std::to_string(t) + ": " + err);
        }
    } catch (const std::bad_alloc&) {
        return set_err(MH_E_NOMEM, "host allocation during validation");
    }
    mh::jit::Options opt;
    opt.max_vgpr = max_vgpr ? max_vgpr : 128;
    if (opt.max_vgpr > 256 || opt.max_vgpr < 96) return set_err(MH_E_INVALID, "max_vgpr outside 96..256");
    opt.short_circuit = (flags & MH_JIT_FULL_EVAL) == 0;
    if (const char* e = std::getenv("MH_JIT_SC")) opt.short_circuit = opt.short_circuit && atoi(e) != 0;
    opt.assemble = false;
    std::vector<mh::jit::Built> built;
    mh::jit::BuildStats stats;
    std::string err;
    try {
        if (!mh::jit::build_tapeset(nodes, tape_offsets, n_tapes, consts, n_consts, n_vars, false,
                                    opt, mh::jit::default_threads(), built, stats, err))
            return set_err(MH_E_UNSUPPORTED, "JIT: " + err);
    } catch (const std::bad_alloc&) {
        return set_err(MH_E_NOMEM, "host allocation during JIT build");
    }
    *out = mh::jit::code_id(built);
    return MH_OK;
}

int32_t mh_tapes_jit_info(const mh_tapeset* ts, mh_jit_info* out) {
    if (!ts || !out) return set_err(MH_E_INVALID, "null argument");
    *out = ts->jinfo;
    return MH_OK;
}

int32_t mh_tapes_jitted(const mh_tapeset* ts, uint8_t* out, uint32_t n_tapes) {
    if (!ts || (!out && n_tapes)) return set_err(MH_E_INVALID, "null argument");
    if (n_tapes > ts->n_tapes) return set_err(MH_E_INVALID, "n_tapes exceeds the tape set");
    for (uint32_t t = 0; t < n_tapes; ++t) out[t] = ts->has_jit ? ts->jitted[t] : 0;
    return MH_OK;
}

int32_t mh_jit_eval_all(mh_ctx* ctx, const mh_tapeset* ts, const mh_assign* as,
                        uint64_t row_first, uint64_t row_count, uint32_t* out) {
    if (int32_t r = check_run_args(ctx, ts, 0, ts ? ts->n_tapes : 0, as, row_first, row_count,
                                   MH_MODE_COUNT_ALL))
        return r;
    if (!ts->has_jit) return set_err(MH_E_INVALID, "no native code (mh_tapes_jit first)");
    for (const auto& j : ts->jit)
        if (j.n_groups && !j.vfn) return set_err(MH_E_INVALID, "built without MH_JIT_VALUES");
    if (!out && row_count) return set_err(MH_E_INVALID, "null out");
    if (row_count == 0) return MH_OK;
    if (int32_t r = use_device(ctx)) return r;
    const size_t n = (size_t)ts->n_tapes * 8 * row_count;
    uint32_t* d = nullptr;
    MH_HIP(hipMalloc(&d, n * sizeof(uint32_t)));
    hipError_t e = hipMemcpy(d, out, n * sizeof(uint32_t), hipMemcpyHostToDevice);
    int32_t r = MH_OK;
    if (e == hipSuccess)
        r = launch_jit(ctx, ts, as, row_first, row_count, 0, MH_MODE_COUNT_ALL, nullptr, nullptr, d);
    if (e == hipSuccess && r == MH_OK) e = hipStreamSynchronize(ctx->stream);
    if (e == hipSuccess && r == MH_OK) e = hipMemcpy(out, d, n * sizeof(uint32_t), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (r != MH_OK) return r;
    if (e != hipSuccess) return set_err(MH_E_DEVICE, std::string("mh_jit_eval_all: ") + hipGetErrorString(e));
    return MH_OK;
}

int32_t mh_comm_unique_id(uint8_t* out) {
    if (!out) return set_err(MH_E_INVALID, "null out");
    const Rccl* r = rccl();
    if (!r) return set_err(MH_E_UNSUPPORTED, "RCCL (librccl.so) not loadable");
    ncclUniqueId id;
    const ncclResult_t e = r->get_unique_id(&id);
    if (e != ncclSuccess)
        return set_err(MH_E_DEVICE, std::string("ncclGetUniqueId: ") +
                                        (r->error_string ? r->error_string(e) : "error"));
    static_assert(sizeof(id) == MH_COMM_ID_BYTES, "RCCL unique id size");
    std::memcpy(out, &id, sizeof(id));
    return MH_OK;
}

int32_t mh_comm_init(mh_ctx* ctx, const uint8_t* unique_id, int32_t rank, int32_t world) {
    if (!ctx || !unique_id) return set_err(MH_E_INVALID, "null argument");
    if (world < 1 || rank < 0 || rank >= world) return set_err(MH_E_INVALID, "bad rank / world");
    if (ctx->comm) return set_err(MH_E_INVALID, "ctx already has a communicator");
    const Rccl* r = rccl();
    if (!r) return set_err(MH_E_UNSUPPORTED, "RCCL (librccl.so) not loadable");
    if (int32_t rc = use_device(ctx)) return rc;
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    const ncclResult_t e = r->comm_init_rank(&ctx->comm, world, id, rank);
    if (e != ncclSuccess) {
        ctx->comm = nullptr;
        return set_err(MH_E_DEVICE, std::string("ncclCommInitRank: ") +
                                        (r->error_string ? r->error_string(e) : "error"));
    }
    ctx->rank = rank;
    ctx->world = world;
    return MH_OK;
}

int32_t mh_comm_allreduce_results(mh_ctx* ctx, uint64_t* d_first_hit, uint64_t* d_hit_count,
                                  uint32_t n) {
    if (!ctx) return set_err(MH_E_INVALID, "null ctx");
    if (!ctx->comm) return set_err(MH_E_INVALID, "no communicator (mh_comm_init)");
    const Rccl* r = rccl();
    if (int32_t rc = use_device(ctx)) return rc;
    // the one exchange of a sharded run: smallest witness index (NO_HIT = UINT64_MAX is the
    // identity of MIN) and summed hit counts, in place on the ctx stream
    ncclResult_t e = ncclSuccess;
    if (d_first_hit && n)
        e = r->all_reduce(d_first_hit, d_first_hit, n, ncclUint64, ncclMin, ctx->comm, ctx->stream);
    if (e == ncclSuccess && d_hit_count && n)
        e = r->all_reduce(d_hit_count, d_hit_count, n, ncclUint64, ncclSum, ctx->comm, ctx->stream);
    if (e != ncclSuccess)
        return set_err(MH_E_DEVICE, std::string("ncclAllReduce: ") +
                                        (r->error_string ? r->error_string(e) : "error"));
    return MH_OK;
}

int32_t mh_comm_destroy(mh_ctx* ctx) {
    if (!ctx) return set_err(MH_E_INVALID, "null ctx");
    if (ctx->comm && rccl()) (void)rccl()->comm_destroy(ctx->comm);
    ctx->comm = nullptr;
    ctx->rank = 0;
    ctx->world = 1;
    return MH_OK;
}

int32_t mh_microbench_issue(mh_ctx* ctx, uint32_t kind, uint32_t waves_per_simd,
                            double* lane_ops_per_s) {
    if (!ctx || !lane_ops_per_s || kind >= MH_MB_NUM_KINDS || waves_per_simd == 0 ||
        waves_per_simd > 8)
        return set_err(MH_E_INVALID, "bad argument");
    if (int32_t r = use_device(ctx)) return r;
    // 256 CUs x 4 SIMDs; a 256-thread workgroup is 4 waves, one per SIMD of its CU
    const uint32_t blocks = 256u * waves_per_simd, iters = 8192;
    hipEvent_t e0, e1;
    MH_HIP(hipEventCreate(&e0));
    MH_HIP(hipEventCreate(&e1));
    MH_HIP(mh::launch_microbench(kind, 64, blocks, ctx->scratch, ctx->stream));  // warm-up
    MH_HIP(hipEventRecord(e0, ctx->stream));
    MH_HIP(mh::launch_microbench(kind, iters, blocks, ctx->scratch, ctx->stream));
    MH_HIP(hipEventRecord(e1, ctx->stream));
    MH_HIP(hipEventSynchronize(e1));
    float ms = 0;
    MH_HIP(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    // 32 wave-instructions of the measured kind per iteration (kind 7: 32 readlanes + 1 SALU)
    const double lanes = (double)blocks * 256.0;
    *lane_ops_per_s = lanes * iters * 32.0 / (ms * 1e-3);
    return MH_OK;
}

int32_t mh_microbench_valu(mh_ctx* ctx, uint32_t kind, double* ops_per_s) {
    // round-1 entry point: kind 0 add/addc chains, 1 v_mad_u64_u32, 2 v_add_u32 (no carry),
    // each at 8 waves per SIMD
    if (kind > 2) return set_err(MH_E_INVALID, "bad argument");
    return mh_microbench_issue(ctx, kind, 8, ops_per_s);
}

int32_t mh_ctx_enable_timing(mh_ctx* ctx, int32_t enable) {
    if (!ctx) return set_err(MH_E_INVALID, "null ctx");
    ctx->timing = enable != 0;
    return MH_OK;
}

int32_t mh_ctx_kernel_time(mh_ctx* ctx, double* total_ms, uint64_t* launches) {
    if (!ctx || !total_ms || !launches) return set_err(MH_E_INVALID, "null argument");
    if (int32_t r = use_device(ctx)) return r;
    double sum = 0.0;
    hipError_t err = hipSuccess;
    for (auto& sp : ctx->spans) {
        float ms = 0.f;
        if (err == hipSuccess) err = hipEventSynchronize(sp.second);
        if (err == hipSuccess) err = hipEventElapsedTime(&ms, sp.first, sp.second);
        sum += ms;
        (void)hipEventDestroy(sp.first);
        (void)hipEventDestroy(sp.second);
    }
    *launches = ctx->spans.size();
    ctx->spans.clear();
    *total_ms = sum;
    if (err != hipSuccess)
        return set_err(MH_E_DEVICE, std::string("kernel timing: ") + hipGetErrorString(err));
    return MH_OK;
}

}  // extern "C"
