// Sparse operator x feature aggregation (the graph_oper / P_multi hot loops).
//
// Forward (models/layers/layers_mnb.py:391-434): for one packed output row r
//   out[r, j*Cg + c]          = sum_{e in G(r)} v_j(e) * Xg[col(e), c]   j < J+2
//   out[r, J*Cg + c]          = sum_{e in P(r)} Pm(e)  * Xp[col(e), c]
//   out[r, J*Cg + Cp + c]     = sum_{e in P(r)} Pd(e)  * Xp[col(e), c]
// i.e. the reference's cat(graph_oper(W, X), P_multi(Pm, Y), P_multi(Pd, Y)) of
// one layer, built row by row.  One wave per row; the row's entry list is
// wave-uniform (scalar loads); each gathered feature row is one coalesced
// vector load of 64 lanes x CPL channels and feeds all J+2 (or both P)
// coefficients.  Variable degree = a loop of wave-uniform trip count, so the
// segmented reduction needs no cross-lane traffic at all.
//
// Backward: the transposed lists (S_WT, S_PE/S_PN) gather the upstream
// gradient blocks:  out[r, c] (+)= sum_e sum_j v_j * dA[col, j*C + c]
//                                + sum_e Pm * dA[col, m_off + c] + Pd * dA[col, d_off + c].
#include "kernels.h"

namespace hgnn {

template <int CPL>
__device__ __forceinline__ void load_row(const float* __restrict__ p, int C, int lane, float (&x)[CPL]) {
    const int c0 = lane * CPL;
    constexpr uintptr_t AL = (CPL >= 4 ? 16 : 4 * CPL) - 1;
    if (C == 64 * CPL && (reinterpret_cast<uintptr_t>(p) & AL) == 0) {
        if constexpr (CPL == 1) {
            x[0] = p[c0];
        } else if constexpr (CPL == 2) {
            const float2 v = *reinterpret_cast<const float2*>(p + c0);
            x[0] = v.x;
            x[1] = v.y;
        } else if constexpr (CPL == 4) {
            const float4 v = *reinterpret_cast<const float4*>(p + c0);
            x[0] = v.x;
            x[1] = v.y;
            x[2] = v.z;
            x[3] = v.w;
        } else {
#pragma unroll
            for (int i = 0; i < CPL; i += 4) {
                const float4 v = *reinterpret_cast<const float4*>(p + c0 + i);
                x[i] = v.x;
                x[i + 1] = v.y;
                x[i + 2] = v.z;
                x[i + 3] = v.w;
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < CPL; ++i) x[i] = (c0 + i < C) ? p[c0 + i] : 0.f;
    }
}

template <int CPL>
__device__ __forceinline__ void store_row(float* __restrict__ p, int C, int lane, const float (&x)[CPL]) {
    const int c0 = lane * CPL;
    constexpr uintptr_t AL = (CPL >= 4 ? 16 : 4 * CPL) - 1;
    if (C == 64 * CPL && (reinterpret_cast<uintptr_t>(p) & AL) == 0) {
        if constexpr (CPL == 1) {
            p[c0] = x[0];
        } else if constexpr (CPL == 2) {
            *reinterpret_cast<float2*>(p + c0) = make_float2(x[0], x[1]);
        } else {
#pragma unroll
            for (int i = 0; i < CPL; i += 4)
                *reinterpret_cast<float4*>(p + c0 + i) = make_float4(x[i], x[i + 1], x[i + 2], x[i + 3]);
        }
    } else {
#pragma unroll
        for (int i = 0; i < CPL; ++i)
            if (c0 + i < C) p[c0 + i] = x[i];
    }
}

// Entry lists are fetched lane-parallel (lane e holds entry e of a 64-entry chunk)
// and broadcast with readlane, and U feature rows are loaded before any is used,
// so a row of n entries costs ~n/U dependent memory round trips instead of 2n.
constexpr int AGG_U = 4;

__device__ __forceinline__ float4 lane_entry(const float* __restrict__ entries, int stride, int start, int n, int lane) {
    // W / WL entries: (col, v_0..v_{J-1}) padded to `stride` floats; P entries: (col, pm, pd, -)
    if (lane < n) return *reinterpret_cast<const float4*>(entries + (long long)(start + lane) * stride);
    return make_float4(__int_as_float(0), 0.f, 0.f, 0.f);
}

__device__ __forceinline__ float bcast(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Per-lane BN constants of the CPL channels a lane owns (lane * CPL + i).
template <int CPL>
struct LaneBn {
    float mu[CPL], sd[CPL], w, b;
    bool on;
    __device__ __forceinline__ void init(const BnView& v, int C, int lane) {
        on = v.mean != nullptr;
        w = b = 0.f;
#pragma unroll
        for (int i = 0; i < CPL; ++i) mu[i] = 0.f, sd[i] = 1.f;
        if (!on) return;
        w = *v.w;
        b = *v.b;
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
            const int c = lane * CPL + i;
            if (c < C) mu[i] = v.mean[c], sd[i] = v.std[c];
        }
    }
    __device__ __forceinline__ void apply(float (&x)[CPL]) const {
        if (!on) return;
#pragma unroll
        for (int i = 0; i < CPL; ++i) x[i] = bn_z(x[i], mu[i], sd[i], w, b);
    }
};

template <int JT, int CG, int CP>
__global__ void __launch_bounds__(256) k_agg_fwd(AggFwdArgs a) {
    const int r = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    if (r >= *a.total_rows) return;
    float* o = a.out + (long long)r * a.ldo;
    if constexpr (CG > 0) {
        float acc[JT][CG];
#pragma unroll
        for (int j = 0; j < JT; ++j)
#pragma unroll
            for (int i = 0; i < CG; ++i) acc[j][i] = 0.f;
        const RowInfo ri = a.g.rows[r];
        const int stride = a.g.stride;
        LaneBn<CG> bn;
        bn.init(a.gbn, a.cg, lane);
        for (int e0 = 0; e0 < ri.count; e0 += 64) {
            const int n = min(64, ri.count - e0);
            // JT <= 3: one float4 per entry; larger JT reads the extra coefficients below
            const float4 me = lane_entry(a.g.entries, stride, ri.start + e0, n, lane);
            float mx[JT > 3 ? JT - 3 : 1];
            if constexpr (JT > 3) {
#pragma unroll
                for (int j = 3; j < JT; ++j)
                    mx[j - 3] = lane < n ? a.g.entries[(long long)(ri.start + e0 + lane) * stride + 1 + j] : 0.f;
            }
            for (int e = 0; e < n; e += AGG_U) {
                float x[AGG_U][CG];
                float v[AGG_U][JT];
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) {
                    const int eu = min(e + u, n - 1);
                    const int col = __builtin_amdgcn_readlane(__float_as_int(me.x), eu);
                    const bool live = e + u < n;
                    v[u][0] = live ? bcast(me.y, eu) : 0.f;
                    if constexpr (JT > 1) v[u][1] = live ? bcast(me.z, eu) : 0.f;
                    if constexpr (JT > 2) v[u][2] = live ? bcast(me.w, eu) : 0.f;
#pragma unroll
                    for (int j = 3; j < JT; ++j) v[u][j] = live ? bcast(mx[j - 3], eu) : 0.f;
                    load_row<CG>(a.xg + (long long)col * a.cg, a.cg, lane, x[u]);
                }
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) bn.apply(x[u]);
#pragma unroll
                for (int u = 0; u < AGG_U; ++u)
#pragma unroll
                    for (int j = 0; j < JT; ++j)
#pragma unroll
                        for (int i = 0; i < CG; ++i) acc[j][i] = fmaf(v[u][j], x[u][i], acc[j][i]);
            }
        }
#pragma unroll
        for (int j = 0; j < JT; ++j) store_row<CG>(o + j * a.cg, a.cg, lane, acc[j]);
    }
    if constexpr (CP > 0) {
        float am[CP], ad[CP];
#pragma unroll
        for (int i = 0; i < CP; ++i) am[i] = ad[i] = 0.f;
        const RowInfo ri = a.p.rows[r];
        LaneBn<CP> bn;
        bn.init(a.pbn, a.cp, lane);
        for (int e0 = 0; e0 < ri.count; e0 += 64) {
            const int n = min(64, ri.count - e0);
            const float4 me = lane_entry(a.p.entries, 4, ri.start + e0, n, lane);
            for (int e = 0; e < n; e += AGG_U) {
                float x[AGG_U][CP], vm[AGG_U], vd[AGG_U];
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) {
                    const int eu = min(e + u, n - 1);
                    const int col = __builtin_amdgcn_readlane(__float_as_int(me.x), eu);
                    const bool live = e + u < n;
                    vm[u] = live ? bcast(me.y, eu) : 0.f;
                    vd[u] = live ? bcast(me.z, eu) : 0.f;
                    load_row<CP>(a.xp + (long long)col * a.cp, a.cp, lane, x[u]);
                }
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) bn.apply(x[u]);
#pragma unroll
                for (int u = 0; u < AGG_U; ++u)
#pragma unroll
                    for (int i = 0; i < CP; ++i) {
                        am[i] = fmaf(vm[u], x[u][i], am[i]);
                        ad[i] = fmaf(vd[u], x[u][i], ad[i]);
                    }
            }
        }
        const int base = JT * a.cg;
        store_row<CP>(o + base, a.cp, lane, am);
        store_row<CP>(o + base + a.cp, a.cp, lane, ad);
    }
    // zero the row padding [K, ldo): the GEMMs run over the padded width
    const int kk = JT * a.cg + (CP > 0 ? 2 * a.cp : 0);
    if (lane < a.ldo - kk) o[kk + lane] = 0.f;
}

static int cpl_of(int c) {
    if (c <= 0) return 0;
    if (c <= 64) return 1;
    if (c <= 128) return 2;
    if (c <= 256) return 4;
    if (c <= 512) return 8;
    return -1;
}

template <int JT, int CG>
static int agg_fwd_cp(const AggFwdArgs& a, dim3 g, hipStream_t s) {
    switch (cpl_of(a.xp ? a.cp : 0)) {
        case 0: hipLaunchKernelGGL((k_agg_fwd<JT, CG, 0>), g, dim3(256), 0, s, a); break;
        case 1: hipLaunchKernelGGL((k_agg_fwd<JT, CG, 1>), g, dim3(256), 0, s, a); break;
        case 2: hipLaunchKernelGGL((k_agg_fwd<JT, CG, 2>), g, dim3(256), 0, s, a); break;
        case 4: hipLaunchKernelGGL((k_agg_fwd<JT, CG, 4>), g, dim3(256), 0, s, a); break;
        case 8: hipLaunchKernelGGL((k_agg_fwd<JT, CG, 8>), g, dim3(256), 0, s, a); break;
        default: return 2;
    }
    HGNN_LAUNCH_CHECK();
    return 0;
}

template <int JT>
static int agg_fwd_cg(const AggFwdArgs& a, dim3 g, hipStream_t s) {
    switch (cpl_of(a.xg ? a.cg : 0)) {
        case 1: return agg_fwd_cp<JT, 1>(a, g, s);
        case 2: return agg_fwd_cp<JT, 2>(a, g, s);
        case 4: return agg_fwd_cp<JT, 4>(a, g, s);
        case 8: return agg_fwd_cp<JT, 8>(a, g, s);
        default: return 2;
    }
}

int launch_agg_fwd(const AggFwdArgs& a, hipStream_t s) {
    if (a.cap_rows <= 0) return 0;
    const dim3 g(ceil_div(a.cap_rows, 4));
    switch (a.jtot) {
        case 3: return agg_fwd_cg<3>(a, g, s);
        case 4: return agg_fwd_cg<4>(a, g, s);
        case 5: return agg_fwd_cg<5>(a, g, s);
        default: return 2;
    }
}

template <int JT, int C, bool HG, bool HP>
__global__ void __launch_bounds__(256) k_agg_bwd(AggBwdArgs a) {
    const int r = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    if (r >= *a.total_rows) return;
    float acc[C];
    float* o = a.out + (long long)r * a.ldo;
    if (a.accumulate) {
        load_row<C>(o, a.c, lane, acc);
    } else {
#pragma unroll
        for (int i = 0; i < C; ++i) acc[i] = 0.f;
    }
    if constexpr (HG) {
        const RowInfo ri = a.g.rows[r];
        const int stride = a.g.stride;
        constexpr int UB = 4;  // entries in flight (x the slices with a nonzero coefficient)
        for (int e0 = 0; e0 < ri.count; e0 += 64) {
            const int n = min(64, ri.count - e0);
            const float4 me = lane_entry(a.g.entries, stride, ri.start + e0, n, lane);
            float mx[JT > 3 ? JT - 3 : 1];
            if constexpr (JT > 3) {
#pragma unroll
                for (int j = 3; j < JT; ++j)
                    mx[j - 3] = lane < n ? a.g.entries[(long long)(ri.start + e0 + lane) * stride + 1 + j] : 0.f;
            }
            for (int e = 0; e < n; e += UB) {
                float x[UB][JT][C], v[UB][JT];
#pragma unroll
                for (int u = 0; u < UB; ++u) {
                    const int eu = min(e + u, n - 1);
                    const int col = __builtin_amdgcn_readlane(__float_as_int(me.x), eu);
                    const bool live = e + u < n;
                    v[u][0] = live ? bcast(me.y, eu) : 0.f;
                    if constexpr (JT > 1) v[u][1] = live ? bcast(me.z, eu) : 0.f;
                    if constexpr (JT > 2) v[u][2] = live ? bcast(me.w, eu) : 0.f;
#pragma unroll
                    for (int j = 3; j < JT; ++j) v[u][j] = live ? bcast(mx[j - 3], eu) : 0.f;
                    const float* src = a.ing + (long long)col * a.ldg + a.gofs;
                    // slices with a zero coefficient are skipped (wave-uniform): I and D live on the
                    // diagonal entry only and A^k has no diagonal in general, so an entry needs 1-2
                    // of its J+2 gradient blocks -- about half the gathered bytes
#pragma unroll
                    for (int j = 0; j < JT; ++j) {
                        if (v[u][j] != 0.f) {
                            load_row<C>(src + j * a.c, a.c, lane, x[u][j]);
                        } else {
#pragma unroll
                            for (int i = 0; i < C; ++i) x[u][j][i] = 0.f;
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < UB; ++u)
#pragma unroll
                    for (int j = 0; j < JT; ++j)
#pragma unroll
                        for (int i = 0; i < C; ++i) acc[i] = fmaf(v[u][j], x[u][j][i], acc[i]);
            }
        }
    }
    if constexpr (HP) {
        const RowInfo ri = a.p.rows[r];
        for (int e0 = 0; e0 < ri.count; e0 += 64) {
            const int n = min(64, ri.count - e0);
            const float4 me = lane_entry(a.p.entries, 4, ri.start + e0, n, lane);
            for (int e = 0; e < n; e += AGG_U) {
                float xm[AGG_U][C], xd[AGG_U][C], vm[AGG_U], vd[AGG_U];
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) {
                    const int eu = min(e + u, n - 1);
                    const int col = __builtin_amdgcn_readlane(__float_as_int(me.x), eu);
                    const bool live = e + u < n;
                    vm[u] = live ? bcast(me.y, eu) : 0.f;
                    vd[u] = live ? bcast(me.z, eu) : 0.f;
                    const float* src = a.inp + (long long)col * a.ldp;
                    load_row<C>(src + a.pofs_m, a.c, lane, xm[u]);
                    load_row<C>(src + a.pofs_d, a.c, lane, xd[u]);
                }
#pragma unroll
                for (int u = 0; u < AGG_U; ++u)
#pragma unroll
                    for (int i = 0; i < C; ++i) acc[i] = fmaf(vd[u], xd[u][i], fmaf(vm[u], xm[u][i], acc[i]));
            }
        }
    }
    store_row<C>(o, a.c, lane, acc);
}

template <int JT, int C>
static int agg_bwd_parts(const AggBwdArgs& a, dim3 g, hipStream_t s) {
    const bool hg = a.ing != nullptr, hp = a.inp != nullptr;
    if (hg && hp) hipLaunchKernelGGL((k_agg_bwd<JT, C, true, true>), g, dim3(256), 0, s, a);
    else if (hg) hipLaunchKernelGGL((k_agg_bwd<JT, C, true, false>), g, dim3(256), 0, s, a);
    else if (hp) hipLaunchKernelGGL((k_agg_bwd<JT, C, false, true>), g, dim3(256), 0, s, a);
    else return 1;
    HGNN_LAUNCH_CHECK();
    return 0;
}

template <int JT>
static int agg_bwd_c(const AggBwdArgs& a, dim3 g, hipStream_t s) {
    switch (cpl_of(a.c)) {
        case 1: return agg_bwd_parts<JT, 1>(a, g, s);
        case 2: return agg_bwd_parts<JT, 2>(a, g, s);
        case 4: return agg_bwd_parts<JT, 4>(a, g, s);
        case 8: return agg_bwd_parts<JT, 8>(a, g, s);
        default: return 2;
    }
}

int launch_agg_bwd(const AggBwdArgs& a, hipStream_t s) {
    if (a.cap_rows <= 0) return 0;
    const dim3 g(ceil_div(a.cap_rows, 4));
    switch (a.jtot) {
        case 3: return agg_bwd_c<3>(a, g, s);
        case 4: return agg_bwd_c<4>(a, g, s);
        case 5: return agg_bwd_c<5>(a, g, s);
        default: return 2;
    }
}

}  // namespace hgnn
