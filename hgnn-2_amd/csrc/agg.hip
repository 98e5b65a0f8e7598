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

#include <initializer_list>

namespace hgnn {

// Row loads / stores of one wave (lane owns channels lane*CPL ..).  V = the host checked that
// C == 64*CPL and every row address is aligned for the vector width (the executor's layouts
// always are), so the vector form is straight-line code; otherwise a guarded scalar form.
template <int CPL, bool V>
__device__ __forceinline__ void load_row(const float* __restrict__ p, int C, int lane, float (&x)[CPL]) {
    const int c0 = lane * CPL;
    if constexpr (V) {
        if constexpr (CPL == 1) {
            x[0] = p[c0];
        } else if constexpr (CPL == 2) {
            const float2 v = *reinterpret_cast<const float2*>(p + c0);
            x[0] = v.x;
            x[1] = v.y;
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

template <int CPL, bool V>
__device__ __forceinline__ void store_row(float* __restrict__ p, int C, int lane, const float (&x)[CPL]) {
    const int c0 = lane * CPL;
    if constexpr (V) {
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

// Host side of V: channel count fills the lanes exactly, base pointers and every offset /
// leading dimension keep the vector alignment.
static bool vec_ok(int cpl, int c, const void* base, std::initializer_list<long long> offs) {
    if (c != 64 * cpl) return false;
    const int w = cpl >= 4 ? 4 : cpl;  // floats per vector access
    if (reinterpret_cast<uintptr_t>(base) % (4 * w)) return false;
    for (long long o : offs)
        if (o % w) return false;
    return true;
}

// Entry lists are fetched lane-parallel (lane e holds entry e of a 64-entry chunk)
// and broadcast with readlane, and U feature rows are loaded before any is used,
// so a row of n entries costs ~n/U dependent memory round trips instead of 2n.
#ifndef AGG_UNROLL
#define AGG_UNROLL 4
#endif
constexpr int AGG_U = AGG_UNROLL;
// rows (waves) per block of the aggregation kernels; AGG_BLOCK_WAVES at build time (A/B)
#ifndef AGG_BLOCK_WAVES
#define AGG_BLOCK_WAVES 4
#endif
constexpr int AGG_WV = AGG_BLOCK_WAVES, AGG_NT = 64 * AGG_WV;

__device__ __forceinline__ float4 lane_entry(const float* __restrict__ entries, int stride, int start, int n, int lane) {
    // W / WL entries: (col, v_0..v_{J-1}) padded to `stride` floats; P entries: (col, pm, pd, -)
    if (lane < n) return *reinterpret_cast<const float4*>(entries + (long long)(start + lane) * stride);
    return make_float4(__int_as_float(0), 0.f, 0.f, 0.f);
}

// Row info through the constant address space: a wave-uniform index then becomes one scalar
// load (lgkmcnt, not the vector counter the gathers wait on) and the row's counts live in SGPRs.
// The lists are written by an earlier launch and only read here.
__device__ __forceinline__ RowInfo row_info(const RowInfo* rows, int r) {
    typedef const __attribute__((address_space(4))) int* ConstInts;
    const ConstInts q = (ConstInts)(reinterpret_cast<const int*>(rows) + 2 * (long long)r);
    RowInfo v;
    v.start = q[0];
    v.count = q[1];
    return v;
}

__device__ __forceinline__ float bcast(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Per-lane BN constants of the CPL channels a lane owns (lane * CPL + i).
template <int CPL>
struct LaneBn {
    float mu[CPL], sc[CPL], w, b;  // sc = w / std per channel
    bool on;
    __device__ __forceinline__ void init(const BnView& v, int C, int lane) {
        on = v.mean != nullptr;
        w = b = 0.f;
#pragma unroll
        for (int i = 0; i < CPL; ++i) mu[i] = 0.f, sc[i] = 1.f;
        if (!on) return;
        w = *v.w;
        b = *v.b;
#pragma unroll
        for (int i = 0; i < CPL; ++i) {
            const int c = lane * CPL + i;
            if (c < C) mu[i] = v.mean[c], sc[i] = bn_scale(w, v.std[c]);
        }
    }
    __device__ __forceinline__ void apply(float (&x)[CPL]) const {
        if (!on) return;
#pragma unroll
        for (int i = 0; i < CPL; ++i) x[i] = bn_z_s(x[i], mu[i], sc[i], b);
    }
};

// Diagonal I / D mode (AggFwdArgs::j0 = 2): the row's entries of one 64-entry chunk (lane e: entry e, m = (col,
// v_0, v_1, ..)) -- the diagonal entry's (v_0, v_1) go to diag[r]; an off-diagonal entry with v_0 or v_1 nonzero
// is an operator the GEMMs' diagonal form cannot take (ERR_DIAG_ID).  found: a diagonal entry was met (uniform).
__device__ __forceinline__ void diag_scan(const AggFwdArgs& a, int r, float4 m, int n, int lane, bool& found) {
    const bool live = lane < n;
    const int col = __float_as_int(m.x);
    const bool on = live && col == r;
    if (on) a.diag[r] = make_float2(m.y, m.z);
    if (__ballot(on)) found = true;
    const bool bad = live && col != r && (m.y != 0.f || m.z != 0.f);
    if (__ballot(bad) && lane == 0) atomicOr(a.err, ERR_DIAG_ID);
}

template <int JT, int CG, int CP, bool V, int J0>
__global__ void __launch_bounds__(AGG_NT) k_agg_fwd(AggFwdArgs a) {
    WaveStamp stamp(a.stamps);
    const int r = __builtin_amdgcn_readfirstlane(blockIdx.x * AGG_WV + (threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    if (r >= *a.total_rows) return;
    float* o = a.out + (long long)r * a.ldo;
    constexpr int CGx = CG > 0 ? CG : 1, CPx = CP > 0 ? CP : 1;
    float acc[JT][CGx], am[CPx], ad[CPx];
#pragma unroll
    for (int j = 0; j < JT; ++j)
#pragma unroll
        for (int i = 0; i < CGx; ++i) acc[j][i] = 0.f;
#pragma unroll
    for (int i = 0; i < CPx; ++i) am[i] = ad[i] = 0.f;
    // The G and P chains (row info -> entry chunk -> feature gathers) run interleaved: both
    // row infos, then both entry chunks, then the gathers of both lists in one batch, so a
    // row costs ~3 dependent memory round trips instead of 6.
    RowInfo rg{0, 0}, rp{0, 0};
    if constexpr (CG > 0) rg = row_info(a.g.rows, r);
    if constexpr (CP > 0) rp = row_info(a.p.rows, r);
    LaneBn<CGx> bng;
    LaneBn<CPx> bnp;
    if constexpr (CG > 0) bng.init(a.gbn, a.cg, lane);
    if constexpr (CP > 0) bnp.init(a.pbn, a.cp, lane);
    const int stride = a.g.stride;
    const int nmax = max(rg.count, rp.count);
    bool dfound = false;
    for (int e0 = 0; e0 < nmax; e0 += 64) {
        const int ng = min(64, max(0, rg.count - e0)), np = min(64, max(0, rp.count - e0));
        float4 mg = make_float4(0.f, 0.f, 0.f, 0.f), mp = mg;
        float mx[JT > 3 ? JT - 3 : 1];
        if constexpr (CG > 0) {
            // JT <= 3: one float4 per entry; larger JT reads the extra coefficients below
            mg = lane_entry(a.g.entries, stride, rg.start + e0, ng, lane);
            if constexpr (JT > 3) {
#pragma unroll
                for (int j = 3; j < JT; ++j)
                    mx[j - 3] = lane < ng ? a.g.entries[(long long)(rg.start + e0 + lane) * stride + 1 + j] : 0.f;
            }
            if constexpr (J0 > 0)
                if (a.diag) diag_scan(a, r, mg, ng, lane, dfound);
        }
        if constexpr (CP > 0) mp = lane_entry(a.p.entries, 4, rp.start + e0, np, lane);
        const int nn = max(ng, np);
        for (int e = 0; e < nn; e += AGG_U) {
            float xg[AGG_U][CGx], v[AGG_U][JT], xp[AGG_U][CPx], vm[AGG_U], vd[AGG_U];
            if constexpr (CG > 0) {
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) {
                    // dead slots re-read the last live row with zero coefficients (no branch)
                    const int eu = max(0, min(e + u, ng - 1));
                    const int col = __builtin_amdgcn_readlane(__float_as_int(mg.x), eu);
                    const bool live = e + u < ng;
                    v[u][0] = live ? bcast(mg.y, eu) : 0.f;
                    if constexpr (JT > 1) v[u][1] = live ? bcast(mg.z, eu) : 0.f;
                    if constexpr (JT > 2) v[u][2] = live ? bcast(mg.w, eu) : 0.f;
#pragma unroll
                    for (int j = 3; j < JT; ++j) v[u][j] = live ? bcast(mx[j - 3], eu) : 0.f;
                    if (ng > 0) load_row<CG, V>(a.xg + (long long)col * a.cg, a.cg, lane, xg[u]);
                    else
#pragma unroll
                        for (int i = 0; i < CG; ++i) xg[u][i] = 0.f;
                }
            }
            if constexpr (CP > 0) {
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) {
                    const int eu = max(0, min(e + u, np - 1));
                    const int col = __builtin_amdgcn_readlane(__float_as_int(mp.x), eu);
                    const bool live = e + u < np;
                    vm[u] = live ? bcast(mp.y, eu) : 0.f;
                    vd[u] = live ? bcast(mp.z, eu) : 0.f;
                    if (np > 0) load_row<CP, V>(a.xp + (long long)col * a.cp, a.cp, lane, xp[u]);
                    else
#pragma unroll
                        for (int i = 0; i < CP; ++i) xp[u][i] = 0.f;
                }
            }
            if constexpr (CG > 0) {
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) bng.apply(xg[u]);
#pragma unroll
                for (int u = 0; u < AGG_U; ++u)
#pragma unroll
                    for (int j = J0; j < JT; ++j)
#pragma unroll
                        for (int i = 0; i < CG; ++i) acc[j][i] = fmaf(v[u][j], xg[u][i], acc[j][i]);
            }
            if constexpr (CP > 0) {
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) bnp.apply(xp[u]);
#pragma unroll
                for (int u = 0; u < AGG_U; ++u)
#pragma unroll
                    for (int i = 0; i < CP; ++i) {
                        am[i] = fmaf(vm[u], xp[u][i], am[i]);
                        ad[i] = fmaf(vd[u], xp[u][i], ad[i]);
                    }
            }
        }
    }
    if constexpr (CG > 0) {
#pragma unroll
        for (int j = J0; j < JT; ++j) store_row<CG, V>(o + (j - J0) * a.cg, a.cg, lane, acc[j]);
        if constexpr (J0 > 0)
            if (a.diag && !dfound && lane == 0) a.diag[r] = make_float2(0.f, 0.f);
    }
    if constexpr (CP > 0) {
        const int base = (JT - J0) * a.cg;
        store_row<CP, V>(o + base, a.cp, lane, am);
        store_row<CP, V>(o + base + a.cp, a.cp, lane, ad);
    }
    // zero the row padding [K, ldo): the GEMMs run over the padded width
    if (a.pad_from >= 0) {
        const int kk = a.pad_from > 0 ? a.pad_from : (JT - J0) * a.cg + (CP > 0 ? 2 * a.cp : 0);
        if (lane < a.ldo - kk) o[kk + lane] = 0.f;
    }
}

// k_agg_fwd with RPW rows per wave (rows RPW w .. RPW w + RPW - 1): the row infos of all of them, then the first entry
// chunk of all of them, are fetched before the first row's gathers, so RPW rows cost RPW + 2 dependent round
// trips instead of 3 RPW.
template <int JT, int CG, int CP, bool V, int RPW, int J0>
__global__ void __launch_bounds__(AGG_NT) k_agg_fwd_rpw(AggFwdArgs a) {
    WaveStamp stamp(a.stamps);
    const int r0 = __builtin_amdgcn_readfirstlane((blockIdx.x * AGG_WV + (threadIdx.x >> 6)) * RPW);
    const int lane = threadIdx.x & 63;
    const int total = *a.total_rows;
    if (r0 >= total) return;
    constexpr int CGx = CG > 0 ? CG : 1, CPx = CP > 0 ? CP : 1, MX = JT > 3 ? JT - 3 : 1;
    // The G and P chains (row info -> entry chunk -> feature gathers) run interleaved: both
    // row infos, then both entry chunks, then the gathers of both lists in one batch, so a
    // row costs ~3 dependent memory round trips instead of 6.
    RowInfo rgk[RPW], rpk[RPW];
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
        const int r = min(r0 + k, total - 1);  // (rows past the total: a live row, never stored)
        rgk[k] = RowInfo{0, 0};
        rpk[k] = RowInfo{0, 0};
        if constexpr (CG > 0) rgk[k] = row_info(a.g.rows, r);
        if constexpr (CP > 0) rpk[k] = row_info(a.p.rows, r);
    }
    LaneBn<CGx> bng;
    LaneBn<CPx> bnp;
    if constexpr (CG > 0) bng.init(a.gbn, a.cg, lane);
    if constexpr (CP > 0) bnp.init(a.pbn, a.cp, lane);
    const int stride = a.g.stride;
    // the first 64-entry chunk of every row's lists
    float4 mgk[RPW], mpk[RPW];
    float mxk[RPW][MX];
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
        mgk[k] = mpk[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        const int ng = min(64, rgk[k].count), np = min(64, rpk[k].count);
        if constexpr (CG > 0) {
            mgk[k] = lane_entry(a.g.entries, stride, rgk[k].start, ng, lane);
            if constexpr (JT > 3) {
#pragma unroll
                for (int j = 3; j < JT; ++j)
                    mxk[k][j - 3] = lane < ng ? a.g.entries[(long long)(rgk[k].start + lane) * stride + 1 + j] : 0.f;
            }
        }
        if constexpr (CP > 0) mpk[k] = lane_entry(a.p.entries, 4, rpk[k].start, np, lane);
    }
#pragma unroll
    for (int k = 0; k < RPW; ++k) {
    const int r = r0 + k;
    if (r >= total) break;
    const RowInfo rg = rgk[k], rp = rpk[k];
    float* o = a.out + (long long)r * a.ldo;
    float acc[JT][CGx], am[CPx], ad[CPx];
#pragma unroll
    for (int j = 0; j < JT; ++j)
#pragma unroll
        for (int i = 0; i < CGx; ++i) acc[j][i] = 0.f;
#pragma unroll
    for (int i = 0; i < CPx; ++i) am[i] = ad[i] = 0.f;
    const int nmax = max(rg.count, rp.count);
    bool dfound = false;
    for (int e0 = 0; e0 < nmax; e0 += 64) {
        const int ng = min(64, max(0, rg.count - e0)), np = min(64, max(0, rp.count - e0));
        float4 mg = mgk[k], mp = mpk[k];
        float mx[MX];
#pragma unroll
        for (int j = 0; j < MX; ++j) mx[j] = mxk[k][j];
        if (e0 > 0) {
            if constexpr (CG > 0) {
                // JT <= 3: one float4 per entry; larger JT reads the extra coefficients below
                mg = lane_entry(a.g.entries, stride, rg.start + e0, ng, lane);
                if constexpr (JT > 3) {
#pragma unroll
                    for (int j = 3; j < JT; ++j)
                        mx[j - 3] = lane < ng ? a.g.entries[(long long)(rg.start + e0 + lane) * stride + 1 + j] : 0.f;
                }
            }
            if constexpr (CP > 0) mp = lane_entry(a.p.entries, 4, rp.start + e0, np, lane);
        }
        if constexpr (J0 > 0 && CG > 0)
            if (a.diag) diag_scan(a, r, mg, ng, lane, dfound);
        const int nn = max(ng, np);
        for (int e = 0; e < nn; e += AGG_U) {
            float xg[AGG_U][CGx], v[AGG_U][JT], xp[AGG_U][CPx], vm[AGG_U], vd[AGG_U];
            if constexpr (CG > 0) {
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) {
                    // dead slots re-read the last live row with zero coefficients (no branch)
                    const int eu = max(0, min(e + u, ng - 1));
                    const int col = __builtin_amdgcn_readlane(__float_as_int(mg.x), eu);
                    const bool live = e + u < ng;
                    v[u][0] = live ? bcast(mg.y, eu) : 0.f;
                    if constexpr (JT > 1) v[u][1] = live ? bcast(mg.z, eu) : 0.f;
                    if constexpr (JT > 2) v[u][2] = live ? bcast(mg.w, eu) : 0.f;
#pragma unroll
                    for (int j = 3; j < JT; ++j) v[u][j] = live ? bcast(mx[j - 3], eu) : 0.f;
                    if (ng > 0) load_row<CG, V>(a.xg + (long long)col * a.cg, a.cg, lane, xg[u]);
                    else
#pragma unroll
                        for (int i = 0; i < CG; ++i) xg[u][i] = 0.f;
                }
            }
            if constexpr (CP > 0) {
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) {
                    const int eu = max(0, min(e + u, np - 1));
                    const int col = __builtin_amdgcn_readlane(__float_as_int(mp.x), eu);
                    const bool live = e + u < np;
                    vm[u] = live ? bcast(mp.y, eu) : 0.f;
                    vd[u] = live ? bcast(mp.z, eu) : 0.f;
                    if (np > 0) load_row<CP, V>(a.xp + (long long)col * a.cp, a.cp, lane, xp[u]);
                    else
#pragma unroll
                        for (int i = 0; i < CP; ++i) xp[u][i] = 0.f;
                }
            }
            if constexpr (CG > 0) {
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) bng.apply(xg[u]);
#pragma unroll
                for (int u = 0; u < AGG_U; ++u)
#pragma unroll
                    for (int j = J0; j < JT; ++j)
#pragma unroll
                        for (int i = 0; i < CG; ++i) acc[j][i] = fmaf(v[u][j], xg[u][i], acc[j][i]);
            }
            if constexpr (CP > 0) {
#pragma unroll
                for (int u = 0; u < AGG_U; ++u) bnp.apply(xp[u]);
#pragma unroll
                for (int u = 0; u < AGG_U; ++u)
#pragma unroll
                    for (int i = 0; i < CP; ++i) {
                        am[i] = fmaf(vm[u], xp[u][i], am[i]);
                        ad[i] = fmaf(vd[u], xp[u][i], ad[i]);
                    }
            }
        }
    }
    if constexpr (CG > 0) {
#pragma unroll
        for (int j = J0; j < JT; ++j) store_row<CG, V>(o + (j - J0) * a.cg, a.cg, lane, acc[j]);
        if constexpr (J0 > 0)
            if (a.diag && !dfound && lane == 0) a.diag[r] = make_float2(0.f, 0.f);
    }
    if constexpr (CP > 0) {
        const int base = (JT - J0) * a.cg;
        store_row<CP, V>(o + base, a.cp, lane, am);
        store_row<CP, V>(o + base + a.cp, a.cp, lane, ad);
    }
    // zero the row padding [K, ldo): the GEMMs run over the padded width
    if (a.pad_from >= 0) {
        const int kk = a.pad_from > 0 ? a.pad_from : (JT - J0) * a.cg + (CP > 0 ? 2 * a.cp : 0);
        if (lane < a.ldo - kk) o[kk + lane] = 0.f;
    }
    }
}

static int cpl_of(int c) {
    if (c <= 0) return 0;
    if (c <= 64) return 1;
    if (c <= 128) return 2;
    if (c <= 256) return 4;
    if (c <= 512) return 8;
    return -1;
}

template <int JT, int CG, int CP, int J0>
static void agg_fwd_v(const AggFwdArgs& a0, dim3 g, hipStream_t s) {
    AggFwdArgs a = a0;
    const int kk = (JT - J0) * a.cg + (CP > 0 ? 2 * a.cp : 0);
    const bool v = (CG == 0 || vec_ok(CG, a.cg, a.xg, {})) && (CP == 0 || vec_ok(CP, a.cp, a.xp, {})) &&
                   (CG == 0 || vec_ok(CG, a.cg, a.out, {a.ldo, (long long)kk})) &&
                   (CP == 0 || vec_ok(CP, a.cp, a.out, {a.ldo, (long long)(JT - J0) * a.cg, (long long)a.cp}));
    static const int rpw = [] {  // rows per wave: 1 (k_agg_fwd), 2 or 4 (k_agg_fwd_rpw; J_tot = 3 only)
        const char* e = getenv("HGNN_AGG_RPW");
        const int r = e ? atoi(e) : 2;
        return r == 4 ? 4 : (r == 1 ? 1 : 2);
    }();
    if constexpr (JT == 3) {
        if (rpw > 1) {
            const dim3 g2(ceil_div(a.cap_rows, rpw * AGG_WV));
            a.stamps = clock_stamps((long long)g2.x * AGG_WV);
            if (rpw == 4) {
                if (v) HGNN_KLAUNCH((k_agg_fwd_rpw<JT, CG, CP, true, 4, J0>), g2, dim3(AGG_NT), 0, s, a);
                else HGNN_KLAUNCH((k_agg_fwd_rpw<JT, CG, CP, false, 4, J0>), g2, dim3(AGG_NT), 0, s, a);
            } else {
                if (v) HGNN_KLAUNCH((k_agg_fwd_rpw<JT, CG, CP, true, 2, J0>), g2, dim3(AGG_NT), 0, s, a);
                else HGNN_KLAUNCH((k_agg_fwd_rpw<JT, CG, CP, false, 2, J0>), g2, dim3(AGG_NT), 0, s, a);
            }
            return;
        }
    }
    a.stamps = clock_stamps((long long)g.x * AGG_WV);
    if (v) HGNN_KLAUNCH((k_agg_fwd<JT, CG, CP, true, J0>), g, dim3(AGG_NT), 0, s, a);
    else HGNN_KLAUNCH((k_agg_fwd<JT, CG, CP, false, J0>), g, dim3(AGG_NT), 0, s, a);
}

template <int JT, int CG, int CP>
static int agg_fwd_j0(const AggFwdArgs& a, dim3 g, hipStream_t s) {
    // the diagonal I / D form is built for the layer widths the executor gives it: G and P inputs of the
    // same 2d <= 256 channels (or no P part, GNN_simple)
    if (a.j0 == 2) {
        if constexpr (CG > 0 && CG <= 4 && (CP == 0 || CP == CG)) {
            agg_fwd_v<JT, CG, CP, 2>(a, g, s);
            return 0;
        }
        return 2;
    }
    agg_fwd_v<JT, CG, CP, 0>(a, g, s);
    return 0;
}

template <int JT, int CG>
static int agg_fwd_cp(const AggFwdArgs& a, dim3 g, hipStream_t s) {
    int r = 0;
    switch (cpl_of(a.xp ? a.cp : 0)) {
        case 0: r = agg_fwd_j0<JT, CG, 0>(a, g, s); break;
        case 1: r = agg_fwd_j0<JT, CG, 1>(a, g, s); break;
        case 2: r = agg_fwd_j0<JT, CG, 2>(a, g, s); break;
        case 4: r = agg_fwd_j0<JT, CG, 4>(a, g, s); break;
        case 8: r = agg_fwd_j0<JT, CG, 8>(a, g, s); break;
        default: return 2;
    }
    if (r) return r;
    HGNN_LAUNCH_CHECK();
    return 0;
}

template <int JT>
static int agg_fwd_cg(const AggFwdArgs& a, dim3 g, hipStream_t s) {
    switch (cpl_of(a.xg ? a.cg : 0)) {
        case 0:  // P part only (its columns still start at jtot * cg)
            if (!a.xp) return 2;
            return agg_fwd_cp<JT, 0>(a, g, s);
        case 1: return agg_fwd_cp<JT, 1>(a, g, s);
        case 2: return agg_fwd_cp<JT, 2>(a, g, s);
        case 4: return agg_fwd_cp<JT, 4>(a, g, s);
        case 8: return agg_fwd_cp<JT, 8>(a, g, s);
        default: return 2;
    }
}

int launch_agg_fwd(const AggFwdArgs& a, hipStream_t s) {
    if (a.cap_rows <= 0) return 0;
    if (a.j0 != 0 && (a.j0 != 2 || !a.xg || (a.diag && !a.err))) return HGNN_ERR_ARG;
    const dim3 g(ceil_div(a.cap_rows, AGG_WV));
    switch (a.jtot) {
        case 3: return agg_fwd_cg<3>(a, g, s);
        case 4: return agg_fwd_cg<4>(a, g, s);
        case 5: return agg_fwd_cg<5>(a, g, s);
        case 6: return agg_fwd_cg<6>(a, g, s);
        case 7: return agg_fwd_cg<7>(a, g, s);
        default: return 2;
    }
}

// Backward gathers.  The G gather (transposed operator lists, output = the gradient of the
// half's own features) and the P gather (transposed Pm/Pd lists, output = the other kind's
// features) write different tensors; launch_agg_bwd_pair runs both in one grid (blocks
// [0, gb) gather G, the rest P), so neither runs alone on a partly filled chip.
// Entries [0, n) of one 64-entry chunk of a G row, UB entries in flight (x the slices with a
// nonzero coefficient).
template <int JT, int C, bool V, int UB>
__device__ __forceinline__ void agg_bwd_g_chunk(const AggBwdArgs& a, float4 me, const float (&mx)[JT > 3 ? JT - 3 : 1],
                                                int n, int lane, float (&acc)[C]) {
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
                    load_row<C, V>(src + j * a.c, a.c, lane, x[u][j]);
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

// Long rows (the transposed line-graph lists hold rows of up to ~35 entries: 8 % of the rows,
// 59 % of the entries at config 2) take 8 entries per round trip instead of 4 (serial trace:
// 127.9 -> 122.6 us per step).
constexpr int AGG_LONG = 8;

template <int JT, int C, bool V>
__device__ __forceinline__ void agg_bwd_g(const AggBwdArgs& a, int r, int lane) {
    float acc[C];
    float* o = a.out + (long long)r * a.ldo;
    if (a.accumulate) {
        load_row<C, V>(o, a.c, lane, acc);
    } else {
#pragma unroll
        for (int i = 0; i < C; ++i) acc[i] = 0.f;
    }
    const RowInfo ri = row_info(a.g.rows, r);
    const int stride = a.g.stride;
    for (int e0 = 0; e0 < ri.count; e0 += 64) {
        const int n = min(64, ri.count - e0);
        const float4 me = lane_entry(a.g.entries, stride, ri.start + e0, n, lane);
        float mx[JT > 3 ? JT - 3 : 1];
        mx[0] = 0.f;
        if constexpr (JT > 3) {
#pragma unroll
            for (int j = 3; j < JT; ++j)
                mx[j - 3] = lane < n ? a.g.entries[(long long)(ri.start + e0 + lane) * stride + 1 + j] : 0.f;
        }
        if (n > AGG_LONG) agg_bwd_g_chunk<JT, C, V, AGG_LONG>(a, me, mx, n, lane, acc);
        else agg_bwd_g_chunk<JT, C, V, 4>(a, me, mx, n, lane, acc);
    }
    store_row<C, V>(o, a.c, lane, acc);
}

template <int C, bool V>
__device__ __forceinline__ void agg_bwd_p(const AggBwdArgs& a, int r, int lane) {
    float acc[C];
    float* o = a.out + (long long)r * a.ldo;
    if (a.accumulate) {
        load_row<C, V>(o, a.c, lane, acc);
    } else {
#pragma unroll
        for (int i = 0; i < C; ++i) acc[i] = 0.f;
    }
    const RowInfo ri = row_info(a.p.rows, r);
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
                load_row<C, V>(src + a.pofs_m, a.c, lane, xm[u]);
                load_row<C, V>(src + a.pofs_d, a.c, lane, xd[u]);
            }
#pragma unroll
            for (int u = 0; u < AGG_U; ++u)
#pragma unroll
                for (int i = 0; i < C; ++i) acc[i] = fmaf(vd[u], xd[u][i], fmaf(vm[u], xm[u][i], acc[i]));
        }
    }
    store_row<C, V>(o, a.c, lane, acc);
}

// MODE 1: G only (ga); 2: P only (pa); 3: blocks [0, gb) G on ga, the rest P on pa.
template <int JT, int CG, int CP, bool V, int MODE>
__global__ void __launch_bounds__(AGG_NT) k_agg_bwd(AggBwdArgs ga, AggBwdArgs pa, int gb) {
    WaveStamp stamp(ga.stamps);
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    if (MODE == 1 || (MODE == 3 && (int)blockIdx.x < gb)) {
        if constexpr (MODE != 2) {
            const int r = __builtin_amdgcn_readfirstlane((int)blockIdx.x * AGG_WV + wv);
            if (r >= *ga.total_rows) return;
            agg_bwd_g<JT, CG, V>(ga, r, lane);
        }
    } else {
        if constexpr (MODE != 1) {
            const int r = __builtin_amdgcn_readfirstlane(((int)blockIdx.x - (MODE == 3 ? gb : 0)) * AGG_WV + wv);
            if (r >= *pa.total_rows) return;
            agg_bwd_p<CP, V>(pa, r, lane);
        }
    }
}

static bool bwd_vec_g(int cpl, const AggBwdArgs& a) {
    return vec_ok(cpl, a.c, a.ing, {a.ldg, a.gofs}) && vec_ok(cpl, a.c, a.out, {a.ldo});
}
static bool bwd_vec_p(int cpl, const AggBwdArgs& a) {
    return vec_ok(cpl, a.c, a.inp, {a.ldp, a.pofs_m, a.pofs_d}) && vec_ok(cpl, a.c, a.out, {a.ldo});
}

template <int JT, int C>
static int agg_bwd_single(const AggBwdArgs& a0, hipStream_t s) {
    const dim3 g(ceil_div(a0.cap_rows, AGG_WV));
    AggBwdArgs a = a0;
    a.stamps = clock_stamps((long long)g.x * AGG_WV);
    if (a.ing) {
        if (bwd_vec_g(C, a)) HGNN_KLAUNCH((k_agg_bwd<JT, C, C, true, 1>), g, dim3(AGG_NT), 0, s, a, a, 0);
        else HGNN_KLAUNCH((k_agg_bwd<JT, C, C, false, 1>), g, dim3(AGG_NT), 0, s, a, a, 0);
    } else {
        if (bwd_vec_p(C, a)) HGNN_KLAUNCH((k_agg_bwd<3, C, C, true, 2>), g, dim3(AGG_NT), 0, s, a, a, 0);
        else HGNN_KLAUNCH((k_agg_bwd<3, C, C, false, 2>), g, dim3(AGG_NT), 0, s, a, a, 0);
    }
    HGNN_LAUNCH_CHECK();
    return 0;
}

template <int JT>
static int agg_bwd_c(const AggBwdArgs& a, hipStream_t s) {
    switch (cpl_of(a.c)) {
        case 1: return agg_bwd_single<JT, 1>(a, s);
        case 2: return agg_bwd_single<JT, 2>(a, s);
        case 4: return agg_bwd_single<JT, 4>(a, s);
        case 8: return agg_bwd_single<JT, 8>(a, s);
        default: return 2;
    }
}

int launch_agg_bwd(const AggBwdArgs& a, hipStream_t s) {
    if (a.cap_rows <= 0) return 0;
    if ((a.ing != nullptr) == (a.inp != nullptr)) return 1;  // exactly one of the two gathers
    switch (a.jtot) {
        case 3: return agg_bwd_c<3>(a, s);
        case 4: return agg_bwd_c<4>(a, s);
        case 5: return agg_bwd_c<5>(a, s);
        case 6: return agg_bwd_c<6>(a, s);
        case 7: return agg_bwd_c<7>(a, s);
        default: return 2;
    }
}

template <int JT, int C>
static int agg_bwd_pair_c(const AggBwdArgs& ga0, const AggBwdArgs& pa, hipStream_t s) {
    const int gb = ceil_div(ga0.cap_rows, AGG_WV), pb = ceil_div(pa.cap_rows, AGG_WV);
    AggBwdArgs ga = ga0;
    ga.stamps = clock_stamps((long long)(gb + pb) * AGG_WV);
    HGNN_KLAUNCH((k_agg_bwd<JT, C, C, true, 3>), dim3(gb + pb), dim3(AGG_NT), 0, s, ga, pa, gb);
    HGNN_LAUNCH_CHECK();
    return 0;
}

template <int JT>
static int agg_bwd_pair_j(const AggBwdArgs& ga, const AggBwdArgs& pa, hipStream_t s) {
    switch (cpl_of(ga.c)) {
        case 1: return agg_bwd_pair_c<JT, 1>(ga, pa, s);
        case 2: return agg_bwd_pair_c<JT, 2>(ga, pa, s);
        case 4: return agg_bwd_pair_c<JT, 4>(ga, pa, s);
        case 8: return agg_bwd_pair_c<JT, 8>(ga, pa, s);
        default: return 2;
    }
}

int launch_agg_bwd_pair(const AggBwdArgs& ga, const AggBwdArgs& pa, hipStream_t s) {
    // one grid for both gathers when they share the lane layout and the vector path;
    // otherwise two launches
    const int cpl = cpl_of(ga.c);
    const bool pair = ga.ing && !ga.inp && pa.inp && !pa.ing && ga.cap_rows > 0 && pa.cap_rows > 0 &&
                      cpl > 0 && cpl == cpl_of(pa.c) && ga.jtot == pa.jtot && bwd_vec_g(cpl, ga) &&
                      bwd_vec_p(cpl, pa);
    if (!pair) {
        int r = launch_agg_bwd(ga, s);
        if (r) return r;
        return launch_agg_bwd(pa, s);
    }
    switch (ga.jtot) {
        case 3: return agg_bwd_pair_j<3>(ga, pa, s);
        case 4: return agg_bwd_pair_j<4>(ga, pa, s);
        case 5: return agg_bwd_pair_j<5>(ga, pa, s);
        case 6: return agg_bwd_pair_j<6>(ga, pa, s);
        case 7: return agg_bwd_pair_j<7>(ga, pa, s);
        default: return 2;
    }
}

}  // namespace hgnn
