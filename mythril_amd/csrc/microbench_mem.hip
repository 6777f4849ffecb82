// Survivor-gather micro-benchmark (mh_microbench_gather; no reference counterpart): what the
// lane compaction of DESIGN §5.1 / §10 would pay to reload a survivor row's columns from HBM.
//
// A buffer of 2^log2_rows rows x 4 columns x 8 limbs (config 5's 128 B of columns per row) is
// filled on the device; the survivor rows are the rows whose splitmix hash falls under
// permille / 1000 (the head test's survival rate), listed in ascending row order (the most
// favourable order a per-workgroup queue could hand them out in).  One launch reads every
// survivor's 128 B and folds it into one word per survivor (so nothing is optimised away):
//   layout 0: the sieve's SoA layout ([column][limb][row]): 32 scattered 4-byte loads per row;
//   layout 1: a row-major (AoS) layout ([row][32 words]): 8 contiguous 16-byte loads per row;
//   layout 2: the SoA streaming read the kernel does today (every row, coalesced), for scale.
// Reported: the median launch time over `reps` launches and the useful bytes per second
// (survivors x 128 B, or rows x 128 B for layout 2).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <vector>

#include "../../include/mythril_hip.h"

int32_t mh_detail_set_err(int32_t code, const char* msg);  // capi.cpp

namespace {

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void fill_kernel(uint32_t* buf, uint64_t n_words) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t j = i; j < n_words; j += step) buf[j] = (uint32_t)mix(j);
}

// survivors: one flag per row, then an exclusive scan on the host side is avoided by a per-block
// compaction into a row list with one atomic per wave (order inside a wave kept, waves in any
// order: the list is sorted afterwards by a second pass on the host copy)
__global__ void mark_kernel(uint32_t* list, uint32_t* count, uint64_t rows, uint32_t permille) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const bool s = r < rows && (mix(r ^ 0x5EEDull) % 1000u) < permille;
    const uint64_t m = __ballot(s);
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t base = 0;
    if (lane == 0 && m) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __shfl(base, 0);
    if (s) list[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint32_t)r;
}

__global__ void gather_soa(const uint32_t* __restrict__ col, uint64_t stride,
                           const uint32_t* __restrict__ list, uint32_t n, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t r = list[i];
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t w = 0; w < 32; ++w) acc ^= col[(uint64_t)w * stride + r] * (w + 1);
    out[i] = acc;
}

__global__ void gather_aos(const uint4* __restrict__ rows, const uint32_t* __restrict__ list,
                           uint32_t n, uint32_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4* p = rows + (uint64_t)list[i] * 8;
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t q = 0; q < 8; ++q) {
        const uint4 v = p[q];
        acc ^= (v.x + v.y * 3u + v.z * 5u + v.w * 7u) * (q + 1);
    }
    out[i] = acc;
}

__global__ void stream_soa(const uint32_t* __restrict__ col, uint64_t stride, uint64_t rows,
                           uint32_t* out) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= rows) return;
    uint32_t acc = 0;
#pragma unroll
    for (uint32_t w = 0; w < 32; ++w) acc ^= col[(uint64_t)w * stride + r] * (w + 1);
    if (acc == 0x12345678u) out[0] = acc;  // practically never: keeps the loads live
}

}  // namespace

extern "C" int32_t mh_microbench_gather(int32_t device, uint32_t log2_rows, uint32_t permille,
                                        uint32_t layout, uint32_t reps, double* ms_out,
                                        double* gbps_out, uint64_t* survivors_out) {
    if (!ms_out || !gbps_out || log2_rows < 10 || log2_rows > 28 || permille > 1000 ||
        layout > 2 || reps == 0 || reps > 1000)
        return mh_detail_set_err(MH_E_INVALID, "mh_microbench_gather: bad argument");
    if (hipSetDevice(device) != hipSuccess)
        return mh_detail_set_err(MH_E_NODEVICE, "mh_microbench_gather: no such device");
    const uint64_t rows = 1ull << log2_rows, words = rows * 32;
    uint32_t *buf = nullptr, *list = nullptr, *count = nullptr, *out = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    std::vector<float> times;
    uint32_t n = 0;
    hipError_t e = hipMalloc(&buf, words * 4);
    if (e == hipSuccess) e = hipMalloc(&list, rows * 4);
    if (e == hipSuccess) e = hipMalloc(&count, 4);
    if (e == hipSuccess) e = hipMalloc(&out, rows * 4);
    if (e == hipSuccess) e = hipMemset(count, 0, 4);
    if (e == hipSuccess) {
        fill_kernel<<<4096, 256>>>(buf, words);
        mark_kernel<<<(unsigned)((rows + 255) / 256), 256>>>(list, count, rows, permille);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(&n, count, 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && n) {  // ascending row order
        std::vector<uint32_t> h(n);
        e = hipMemcpy(h.data(), list, (size_t)n * 4, hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        if (e == hipSuccess) e = hipMemcpy(list, h.data(), (size_t)n * 4, hipMemcpyHostToDevice);
    }
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    for (uint32_t it = 0; e == hipSuccess && it <= reps; ++it) {  // launch 0 warms up
        e = hipEventRecord(e0, nullptr);
        if (layout == 0 && n)
            gather_soa<<<(n + 255) / 256, 256>>>(buf, rows, list, n, out);
        else if (layout == 1 && n)
            gather_aos<<<(n + 255) / 256, 256>>>(reinterpret_cast<const uint4*>(buf), list, n, out);
        else if (layout == 2)
            stream_soa<<<(unsigned)((rows + 255) / 256), 256>>>(buf, rows, rows, out);
        if (e == hipSuccess) e = hipGetLastError();
        if (e == hipSuccess) e = hipEventRecord(e1, nullptr);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        float ms = 0.f;
        if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
        if (e == hipSuccess && it) times.push_back(ms);
    }
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (buf) (void)hipFree(buf);
    if (list) (void)hipFree(list);
    if (count) (void)hipFree(count);
    if (out) (void)hipFree(out);
    if (e != hipSuccess)
        return mh_detail_set_err(MH_E_DEVICE, hipGetErrorString(e));
    std::sort(times.begin(), times.end());
    const double ms = times[times.size() / 2];
    const double useful = (layout == 2 ? (double)rows : (double)n) * 128.0;
    *ms_out = ms;
    *gbps_out = ms > 0 ? useful / (ms * 1e-3) / 1e9 : 0.0;
    if (survivors_out) *survivors_out = n;
    return MH_OK;
}
