// Device helpers shared by the general CCN-2D kernels (ccn.hip) and the one-workgroup-per-graph CCN-2D
// kernels (ccn2_small.hip): the combined contraction weights, the wave-uniform neighbour walk and the
// parameter-partial layout.  One definition, so both paths do the same arithmetic in the same order.
#pragma once
#include "kernels.h"

namespace hgnn {
namespace {

enum { WA, WB, WQ1, WQ2, WQ3, WQ4, WQ15, WQ16, WQ17, NWC };

// combined weights of output channels [o0, o0 + hc): wc[k][o][c]
template <int HC, int CM>
__device__ __forceinline__ void c2_weights(float (*wc)[HC][CM], const float* __restrict__ W, int cin, int o0, int hc) {
    const int K = 18 * cin;
    for (int t = threadIdx.x; t < HC * CM; t += blockDim.x) {
        const int o = t / CM, c = t % CM;
        const bool ok = o < hc && c < cin;
        const float* w = W + (long long)(o0 + (ok ? o : 0)) * K;
        float r[18];
#pragma unroll
        for (int q = 0; q < 18; ++q) r[q] = ok ? w[q * cin + c] : 0.f;
        float a = r[0];
#pragma unroll
        for (int q = 6; q < 15; ++q) a += r[q];
        wc[WA][o][c] = a;
        wc[WB][o][c] = r[5];
        wc[WQ1][o][c] = r[1];
        wc[WQ2][o][c] = r[2];
        wc[WQ3][o][c] = r[3];
        wc[WQ4][o][c] = r[4];
        wc[WQ15][o][c] = r[15];
        wc[WQ16][o][c] = r[16];
        wc[WQ17][o][c] = r[17];
    }
}

// next NB set bits of a 64-bit wave-uniform set, ascending (-1 past the end)
template <int NB>
__device__ __forceinline__ void c2_take(unsigned long long& s, int (&aa)[NB]) {
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        aa[u] = s ? __ffsll((long long)s) - 1 : -1;
        s &= s ? s - 1ull : 0ull;
    }
}

// 64-bit wave-uniform value of lane l
__device__ __forceinline__ unsigned long long lane_value_u64(unsigned long long v, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)v, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ int lane_value_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// t[u][c] = T[a_u][b][lane] for a batch of NB neighbours (0 where lane is not in C_a or a_u < 0); lane a of
// my_mask holds neighbour a's common-neighbourhood mask, lane a of my_row the row p_a(b) of F_{j_a}
__device__ __forceinline__ const float* lane_value_ptr(const float* p, int l) {
    const unsigned long long v = lane_value_u64((unsigned long long)(uintptr_t)p, l);
    return reinterpret_cast<const float*>((uintptr_t)v);
}
template <int CM, int NB>
__device__ __forceinline__ void c2_load_rows(int cin, int n, const int (&aa)[NB], const short* sp,
                                             unsigned long long my_mask, const float* my_row, float (&t)[NB][CM]) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int u = 0; u < NB; ++u) {
        const int a = aa[u] >= 0 ? aa[u] : 0;
        const bool vz = aa[u] >= 0 && ((lane_value_u64(my_mask, a) >> lane) & 1ull);
        const int pz = vz ? (int)sp[a * n + lane] : 0;
        const float* q = lane_value_ptr(my_row, a) + pz * cin;
#pragma unroll
        for (int c = 0; c < CM; ++c) t[u][c] = c < cin ? q[c] : 0.f;
#pragma unroll
        for (int c = 0; c < CM; ++c) t[u][c] = vz ? t[u][c] : 0.f;
    }
}
// lane a's row p_a(b) of F_{j_a} (a in A_b; any valid row otherwise)
__device__ __forceinline__ const float* c2_row_of(const float* fin, int cin, const short* sp, int n, int b, bool in,
                                                  int my_oj, int my_dj) {
    const int lane = threadIdx.x & 63;
    const int pb = in ? (int)sp[lane * n + b] : 0;
    return fin + ((long long)my_oj + (long long)pb * my_dj) * cin;
}

// dW_q[o][c] of the 18 contraction blocks from the distinct sums (see k_c2_bwd)
__device__ __forceinline__ void c2_write_partials(float* row, int cin, int c, float nf, float p0, float p1, float p2,
                                                  float p3, float p15, float p16, float p4, float p17) {
    row[0 * cin + c] = nf * p0;
    row[1 * cin + c] = p1;
    row[2 * cin + c] = nf * p2;
    row[3 * cin + c] = p3;
    row[4 * cin + c] = p4;
    row[5 * cin + c] = p0;
    for (int q = 6; q < 15; ++q) row[q * cin + c] = nf * p0;
    row[15 * cin + c] = p15;
    row[16 * cin + c] = p16;
    row[17 * cin + c] = p17;
}

constexpr int C2_NACC = 6;  // P0, P1, P2, P3, P15, P16
}  // namespace
}  // namespace hgnn
