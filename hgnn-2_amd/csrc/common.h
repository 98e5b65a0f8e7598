// Shared device helpers for the gfx950 kernels of hgnn_amd.
//
// Conventions used by every kernel in this directory:
//  * wave = 64 lanes (CDNA4); block sizes are multiples of 64;
//  * feature matrices are row-major [rows][C] fp32, one row per node or per
//    line-graph edge slot, rows of a batch packed graph after graph;
//  * sizes that depend on the batch content (packed row totals) live in device
//    memory and are read by the kernels, so a forward needs no host sync; grids
//    are sized from the dense padded capacities (bs*Nmax, bs*Emax) and blocks
//    past the device total exit at once.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hgnn_amd.h"

#define HGNN_WAVE 64

#define HGNN_HOST_CHECK(expr)                                       \
    do {                                                            \
        hipError_t _e = (expr);                                     \
        if (_e != hipSuccess) return HGNN_ERR_HIP;                  \
    } while (0)

#define HGNN_LAUNCH_CHECK()                                         \
    do {                                                            \
        hipError_t _e = hipGetLastError();                          \
        if (_e != hipSuccess) return HGNN_ERR_HIP;                  \
    } while (0)

namespace hgnn {

// Per-dispatch kernel clock (bench.py's per-class timer, net.hip Timer): while t_clock is set on the
// enqueuing thread, HGNN_KLAUNCH launches through hipExtLaunchKernel with a start / stop event pair that
// the runtime binds to the kernel's own dispatch (its begin / end timestamps, as rocprofv3's kernel trace
// reports them) -- no marker packets between the kernels of the stream, so timing changes neither the
// stream's dispatch order nor what the kernel overlaps with.
//
// Stamp mode (st != nullptr): no events at all.  The kernels of the timed classes take a stamp slot
// (clock_stamps, a null pointer otherwise) and every wave of the launch writes s_memrealtime (100 MHz,
// chip-wide) at entry and at exit (WaveStamp): the launch's duration is max(exit) - min(entry), read after
// the timed region.  Event timing -- markers or dispatch-bound pairs -- changes the timed kernel itself
// (every timed dispatch gets a completion signal with a system-scope release: the aggregation backward ran
// 19 -> 30 us per launch inside rocprofv3's own trace while bench.py timed it), stamps do not.
struct LaunchClock {
    hipEvent_t* ev;  // pairs: start, stop (event modes)
    int* cls;        // class of each launch
    int cap;         // launches available
    int* used;       // launches taken
    int k;           // class of the launches being enqueued
    uint64_t* st = nullptr;  // stamp mode: device stamp buffer
    int* st_off = nullptr;   // per launch: first word of its slot
    int* st_n = nullptr;     // per launch: words of its slot (2 per wave)
    long long st_cap = 0;    // words available
    long long* st_used = nullptr;
    uintptr_t strm = 0;          // the stream the launches go to
    uintptr_t* st_strm = nullptr;  // per launch: its stream
};
inline thread_local LaunchClock* t_clock = nullptr;
// Stamp slot of a launch of `waves` waves (stamp mode), else nullptr.
inline uint64_t* clock_stamps(long long waves) {
    LaunchClock* c = t_clock;
    if (!c || !c->st || *c->used >= c->cap || *c->st_used + 2 * waves > c->st_cap) return nullptr;
    const int i = (*c->used)++;
    c->cls[i] = c->k;
    c->st_off[i] = (int)*c->st_used;
    c->st_n[i] = (int)(2 * waves);
    if (c->st_strm) c->st_strm[i] = c->strm;
    *c->st_used += 2 * waves;
    return c->st + c->st_off[i];
}
#ifdef __HIP_DEVICE_COMPILE__
#define HGNN_REALTIME() __builtin_amdgcn_s_memrealtime()
#else
#define HGNN_REALTIME() 0ull
#endif
// Entry / exit stamps of one wave (wave id = linear block id x waves per block + wave in block), written
// by lane 0 with a plain vector store; the destructor covers every return path of the kernel.
struct WaveStamp {
    uint64_t* p;
    __device__ __forceinline__ explicit WaveStamp(uint64_t* slot) : p(nullptr) {
        if (!slot) return;
        const long long b = blockIdx.x + (long long)gridDim.x * (blockIdx.y + (long long)gridDim.y * blockIdx.z);
        p = slot + 2 * (b * (blockDim.x >> 6) + (threadIdx.x >> 6));
        if ((threadIdx.x & 63) == 0) p[0] = HGNN_REALTIME();
    }
    __device__ __forceinline__ ~WaveStamp() {
        if (p && (threadIdx.x & 63) == 0) p[1] = HGNN_REALTIME();
    }
};
inline bool clock_pair(hipEvent_t* a, hipEvent_t* b) {
    LaunchClock* c = t_clock;
    if (!c || !c->ev || *c->used >= c->cap) return false;
    const int i = (*c->used)++;
    c->cls[i] = c->k;
    *a = c->ev[2 * i];
    *b = c->ev[2 * i + 1];
    return true;
}

// Every kernel launch of the library: hipLaunchKernelGGL, or, under a LaunchClock, the same launch with a
// dispatch-bound event pair.  (Variadic so a template kernel's commas need no parentheses.)
template <typename F, typename... Args>
inline void klaunch(F kernel, const dim3& grid, const dim3& block, uint32_t lds, hipStream_t s, Args... args) {
    hipEvent_t a, b;
    if (clock_pair(&a, &b)) hipExtLaunchKernelGGL(kernel, grid, block, lds, s, a, b, 0u, args...);
    else hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
}
#define HGNN_KLAUNCH(...) hgnn::klaunch(__VA_ARGS__)

// Device-side error bits (OR-ed into a workspace word; see include/hgnn_amd.h).
enum : uint32_t {
    ERR_PAD_NONZERO = 1u << 0,   // operator entry outside the graph's real block
    ERR_MASK = 1u << 1,          // mask[:, :, 0] disagrees with N_batch / E_batch
    ERR_SIZES = 1u << 2,         // N_b > Nmax, E_b > Emax or negative count
    ERR_CCN_SELFLOOP = 1u << 3,  // CCN adjacency without self loop (chi_ii absent)
    ERR_CCN_DEGREE = 1u << 4,    // CCN degree above the compiled bound
    ERR_CCN_ASYM = 1u << 5,      // CCN adjacency pattern not symmetric
    ERR_DIAG_ID = 1u << 6,       // operator slice 0 or 1 (I, D) with an off-diagonal entry (diagonal I / D mode)
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// The same total on DPP moves (no LDS round trip), returned uniform (lane 63's value).  Every lane
// of the wave must be active.  quad_perm [1,0,3,2] / [2,3,0,1] sum quads, row_half_mirror and
// row_mirror finish each 16-lane row, row_bcast:15 / :31 carry rows 0 -> 1, 2 -> 3 and 1 -> 2, 3.
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_moved(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROWS, 0xF, false));
}
__device__ __forceinline__ float wave_total(float v) {
    v += dpp_moved<0xB1, 0xF>(v);
    v += dpp_moved<0x4E, 0xF>(v);
    v += dpp_moved<0x141, 0xF>(v);
    v += dpp_moved<0x140, 0xF>(v);
    v += dpp_moved<0x142, 0xA>(v);
    v += dpp_moved<0x143, 0xC>(v);
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}
// wave_total's tree for a double (the two halves moved by the same DPP controls), uniform result
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_moved_d(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, ROWS, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, ROWS, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_total_d(double v) {
    v += dpp_moved_d<0xB1, 0xF>(v);
    v += dpp_moved_d<0x4E, 0xF>(v);
    v += dpp_moved_d<0x141, 0xF>(v);
    v += dpp_moved_d<0x140, 0xF>(v);
    v += dpp_moved_d<0x142, 0xA>(v);
    v += dpp_moved_d<0x143, 0xC>(v);
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), 63);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// value of v in lane l (l wave-uniform)
__device__ __forceinline__ float lane_value(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

template <typename T>
__host__ __device__ __forceinline__ T ceil_div(T a, T b) { return (a + b - 1) / b; }

// Entry of a per-row sparse operator list: packed column index and up to
// three coefficients (J_TOT = 3 slices for J = 1, or {Pm, Pd}).  16 bytes so a
// wave-uniform entry is one dwordx4 load.
struct __align__(16) Entry3 {
    int col;
    float v0, v1, v2;
};

// Row descriptor: entries of row r live at [start, start + count) in the
// structure's entry array (rows own fixed-capacity slots: no prefix sum, so
// the extraction is a single pass with no inter-graph scan).
struct __align__(8) RowInfo {
    int start;
    int count;
};

}  // namespace hgnn
