// Dense gradient of the graph operators W (bs, Nmax, Nmax, J+2).
//
// scripts/train_mnb.py:56-57 sets W.requires_grad, so the reference's backward
// materialises W.grad through every graph_oper(W, X_l) (layers_mnb.py:401-409):
//   dW[b, n, m, j] = sum_l sum_f dG_l[b, j F_l + f, n] * X_l[b, f, m]
// over all Nmax x Nmax positions.  Padded positions are not zero in general:
//  * X_l at a padded node m is the previous BN's output there,
//    w * ((0 - mean_c) / std_c) + b (batch_normalization.py:43, 76), a per-channel
//    constant; for l = 0 it is the dense input X itself;
//  * dG_l at a padded node n is 0 for the middle layers (the BN mask) but, for the
//    readout, the same vector sum_o dy[b, o] fc.w[o, :] at every position
//    (layers_mnb.py:386 sums fc over all Nmax positions).
// Per graph and slice j this is a small GEMM  G_j (Nmax x F) . X (Nmax x F)^T,
// done with v_mfma_f32_32x32x2_f32 on 32x32 tiles of (n, m): one workgroup per
// graph stages the graph's G and X rows in LDS (F in chunks), each wave owns a
// few (n-tile, m-tile, j) items.
#include <algorithm>
#include <type_traits>

#include "kernels.h"

namespace hgnn {

typedef float f32x16 __attribute__((ext_vector_type(16)));
// where only 3 items exist, left one wave per SIMD)
// Staging of one FC-wide chunk: every load is an unconditional buffer load (out-of-range
// elements get an out-of-bounds offset and read 0), the padded-row values (readout vector, BN of
// zero) come from per-chunk LDS constants afterwards.  Loads under per-lane conditions made hipcc
// wait vmcnt(0) after each one: 132 full waits per launch, ~20 us per launch for ~4 us of work.
// Slices [j0, j0 + J) of the G rows are staged (J = a.jt, or 1 for a per-slice block).
template <int FC, int V>
__device__ __forceinline__ void dw_stage(const DwDenseArgs& a, int b, int off, int nb, int npad, int f0, int fc,
                                         int j0, int J, float* Gs, float* Xs, int GP, const float* Rs,
                                         const float* Bmu, const float* Bsc, const float* Bz) {
    typedef typename std::conditional<V == 4, float4, float>::type vt;
    constexpr unsigned OOB = 0x7ffffff0u;
    constexpr int XP = FC + 1;
    constexpr int FV = FC / V;
    const int F = a.f, nmax = a.nmax;
    // wave-uniform descriptor inputs (readfirstlane): a descriptor the compiler cannot prove uniform
    // becomes a waterfall loop around every buffer load
    const int total = __builtin_amdgcn_readfirstlane(a.node_off[a.bs]);
    const auto rg = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.dA), 0,
        __builtin_amdgcn_readfirstlane((int)min((long long)total * a.lda * 4, (long long)OOB)), 0x00020000);
    const uintptr_t xs = reinterpret_cast<uintptr_t>(a.xdense ? a.xdense : a.xp);
    const uintptr_t xsu = ((uintptr_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(xs >> 32)) << 32) |
                          (unsigned)__builtin_amdgcn_readfirstlane((int)(xs & 0xffffffffu));
    const long long xbytes = a.xdense ? (long long)a.bs * F * nmax * 4 : (long long)total * F * 4;
    const auto rx = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<float*>(xsu), 0,
                                                      __builtin_amdgcn_readfirstlane((int)min(xbytes, (long long)OOB)),
                                                      0x00020000);
    auto ld = [&](__amdgpu_buffer_rsrc_t r, unsigned o) -> vt {
        if constexpr (V == 4) return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)o, 0, 0));
        else return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (int)o, 0, 0));
    };
    auto el = [](vt& v, int q) -> float& { return reinterpret_cast<float*>(&v)[q]; };
    const int JFV = J * FV, g_n = npad * JFV, x_n = npad * FV;
    constexpr int U = 8;
    // element i = (row n, column c) of the G image walked by carries: i advances by 256 per load, so (n, c)
    // advances by (dn, dc) plus a carry -- the per-element division by the runtime J FV cost ~20 VALU each
    const int dn = 256 / JFV, dc = 256 - dn * JFV;
    int cn = (int)threadIdx.x / JFV, cc = (int)threadIdx.x - cn * JFV;
    // G rows (the dA slices): all U loads of a round issued before any is used, offsets by select
    for (int base = 0; base < g_n; base += 256 * U) {
        vt v[U];
        int nn[U], ccs[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            nn[u] = cn;
            ccs[u] = cc;
            cc += dc;
            cn += dn;
            if (cc >= JFV) {
                cc -= JFV;
                ++cn;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * 256 + threadIdx.x;
            const int n = nn[u], rem = ccs[u], j = rem / FV, f = (rem % FV) * V;
            const bool live = i < g_n && n < nb && f < fc;
            v[u] = ld(rg, live ? (unsigned)((long long)(off + n) * a.lda + (j0 + j) * F + f0 + f) * 4u : OOB);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * 256 + threadIdx.x;
            const int n = nn[u], rem = ccs[u], j = rem / FV, f = (rem % FV) * V;
            if (i < g_n) {
                const bool pad_row = Rs != nullptr && n >= nb && n < nmax;
                float* d = Gs + n * GP + j * FC + f;
#pragma unroll
                for (int q = 0; q < V; ++q) {
                    const float rv = (pad_row && f + q < fc) ? Rs[j * FC + f + q] : 0.f;
                    d[q] = pad_row ? rv : el(v[u], q);
                }
            }
        }
    }
    // X rows (the layer input): BN on load, the BN of 0 at padded rows
    for (int base = 0; base < x_n; base += 256 * U) {
        vt v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int ix = base + u * 256 + threadIdx.x;
            const int m = ix / FV, f = (ix % FV) * V;
            unsigned o = OOB;
            if (a.xdense) o = (ix < x_n && f < fc && m < nmax) ? (unsigned)(((long long)b * F + f0 + f) * nmax + m) * 4u : OOB;
            else o = (ix < x_n && f < fc && m < nb) ? (unsigned)((long long)(off + m) * F + f0 + f) * 4u : OOB;
            v[u] = ld(rx, o);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int ix = base + u * 256 + threadIdx.x;
            const int m = ix / FV, f = (ix % FV) * V;
            if (ix < x_n) {
                float* d = Xs + m * XP + f;
#pragma unroll
                for (int q = 0; q < V; ++q) {
                    float x = el(v[u], q);
                    if (Bmu != nullptr && !a.xdense && f + q < fc)
                        x = m < nb ? bn_z_s(x, Bmu[f + q], Bsc[f + q], *a.pb) : (m < nmax ? Bz[f + q] : 0.f);
                    d[q] = x;
                }
            }
        }
    }
}

// MAXI = (n-tile, m-tile, slice) items per wave kept in registers: sized to the
// graph so the accumulators do not cap occupancy (5 x 16 AGPRs at Nmax <= 32,
// where only 3 items exist, left one wave per SIMD)
// (A per-(graph, slice) block split -- a third of the loads per block, 3x the blocks -- was measured
// at 350 K vs 366 K graphs/s: on the side stream the extra blocks crowd the main stream's backward
// more than the shorter kernel saves; retired in round 4.)
template <int FC, int MAXI>
__global__ void __launch_bounds__(256) k_dw_dense(DwDenseArgs a) {
    WaveStamp stamp(a.stamps);
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int nmax = a.nmax, F = a.f;
    const int J = a.jt, j0 = 0, JA = a.jt;
    const int npad = (nmax + 31) / 32 * 32;
    const int tiles = npad / 32;
    const int nitems = tiles * tiles * J;
    constexpr int XP = FC + 1;
    const int GP = J * FC + 1;
    float* Gs = smem;               // [npad][GP]
    float* Xs = smem + npad * GP;   // [npad][XP]
    float* Rs = Xs + npad * XP;     // [J * FC] readout vector of the chunk
    float* Bmu = Rs + J * FC;       // [FC] BN mean, scale, and the BN of 0 (padded rows)
    float* Bsc = Bmu + FC;
    float* Bz = Bsc + FC;
    // the input BN's per-channel constants do not depend on the graph: with one channel chunk (F <= FC),
    // staged once per block instead of once per graph (one dependent round trip per graph saved)
    const bool bn_once = a.pmean && F <= FC;
    auto bn_consts = [&](int f0, int fc) {
        for (int t = threadIdx.x; t < FC; t += 256) {
            const int c = f0 + min(t, fc - 1);
            Bmu[t] = a.pmean[c];
            Bsc[t] = bn_scale(*a.pw, a.pstd[c]);
            Bz[t] = bn_z(0.f, a.pmean[c], a.pstd[c], *a.pw, *a.pb);
        }
    };
    if (bn_once) bn_consts(0, F);
    // graphs b, b + gridDim.x, ...: the grid may be smaller than the batch (launch_fc), so the kernel holds
    // fewer of the side stream's CUs beside the main stream's backward
    for (int b = blockIdx.x; b < a.bs; b += gridDim.x) {
    const int off = a.node_off[b];
    const int nb = a.node_off[b + 1] - off;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int h = lane >> 5, l31 = lane & 31;
    // float4 staging needs 16-byte aligned rows and slices
    const bool vec = !a.xdense && F % 4 == 0 && a.lda % 4 == 0 &&
                     ((reinterpret_cast<uintptr_t>(a.dA) | reinterpret_cast<uintptr_t>(a.xp)) & 15) == 0;

    float* dWb = a.dW + (long long)b * nmax * nmax * JA;
    // block-uniform passes over the items; gridDim.y blocks of a graph share them
    const int ystart = blockIdx.y, ystep = gridDim.y;
    for (int base = ystart * 4 * MAXI; base < nitems; base += ystep * 4 * MAXI) {
    f32x16 acc[MAXI];
#pragma unroll
    for (int q = 0; q < MAXI; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;

    for (int f0 = 0; f0 < F; f0 += FC) {
        const int fc = min(FC, F - f0);
        __syncthreads();
        // per-chunk constants: readout vector sum_o dout[b, o] fcw[o, j F + f0 + f], BN of the input
        if (a.dout)
            for (int t = threadIdx.x; t < J * FC; t += 256) {
                const int j = t / FC, f = t % FC;
                float r = 0.f;
                if (f < fc)
                    for (int o = 0; o < a.dim_out; ++o)
                        r = fmaf(a.dout[b * a.dim_out + o], a.fcw[(long long)o * a.kfc + (j0 + j) * F + f0 + f], r);
                Rs[t] = r;
            }
        if (a.pmean && !bn_once) bn_consts(f0, fc);
        __syncthreads();
        if (vec)
            dw_stage<FC, 4>(a, b, off, nb, npad, f0, fc, j0, J, Gs, Xs, GP, a.dout ? Rs : nullptr,
                            a.pmean ? Bmu : nullptr, Bsc, Bz);
        else
            dw_stage<FC, 1>(a, b, off, nb, npad, f0, fc, j0, J, Gs, Xs, GP, a.dout ? Rs : nullptr,
                            a.pmean ? Bmu : nullptr, Bsc, Bz);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < MAXI; ++q) {
            const int it = base + wv + 4 * q;
            if (it < nitems) {
                const int j = it % J, tm = (it / J) % tiles, tn = it / (J * tiles);
                const float* ga = Gs + (tn * 32 + l31) * GP + j * FC + h;
                const float* xb = Xs + (tm * 32 + l31) * XP + h;
#pragma unroll 4
                for (int kk = 0; kk < FC; kk += 2)
                    acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(ga[kk], xb[kk], acc[q], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < MAXI; ++q) {
        const int it = base + wv + 4 * q;
        if (it >= nitems) continue;
        const int j = it % J, tm = (it / J) % tiles, tn = it / (J * tiles);
        const int jo = j0 + j;
        const int m = tm * 32 + l31;
        // read all 16 previous values before any store: a load-add-store per element
        // is serialised by the compiler (possible aliasing) into 16 memory round trips
        // (clamped unconditional loads, selected after: see dw_stage)
        float old[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int n = min(tn * 32 + (r & 3) + 8 * (r >> 2) + 4 * h, nmax - 1);
            old[r] = dWb[((long long)n * nmax + min(m, nmax - 1)) * JA + jo];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r)
            if (!a.accumulate) old[r] = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int n = tn * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (n < nmax && m < nmax) dWb[((long long)n * nmax + m) * JA + jo] = old[r] + acc[q][r];
        }
    }
    }
    __syncthreads();  // the next graph's staging overwrites the LDS images
    }
}

template <int FC, int MAXI>
static void allow_lds(size_t lds) {
    // dynamic LDS beyond 64 KB must be allowed per kernel (gfx950: 160 KB per CU)
    // (the whole 160 KB once: a first call with a smaller size must not cap a later, larger one)
    static bool done = false;
    if (!done && lds > 64 * 1024) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_dw_dense<FC, MAXI>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        done = true;
    }
}

// Blocks of the dense dW (x): one per graph when HGNN_DWD_GRID=0; else at most this many, each walking
// graphs b, b + grid, ...  The kernel runs on the side stream at two waves per SIMD (~225 registers): one
// block per graph (512 at config 2) holds every SIMD's wave slots and blocks the main stream's BN-backward
// statistics kernel until it ends (round-5 stamp timeline: 7-14 us of main-stream idle per node half).
static int dwd_grid(int bs) {
    static const int g = [] {
        const char* e = getenv("HGNN_DWD_GRID");
        return e ? atoi(e) : 256;
    }();
    return g <= 0 ? bs : std::min(bs, g);
}

template <int FC>
static void launch_fc(const DwDenseArgs& a0, int maxi, int gy, size_t lds, hipStream_t s) {
    DwDenseArgs a = a0;
    const int gx = dwd_grid(a0.bs);
    a.stamps = clock_stamps((long long)gx * gy * 4);
    allow_lds<FC, 1>(lds);
    allow_lds<FC, 3>(lds);
    allow_lds<FC, 5>(lds);
    if (maxi <= 1) HGNN_KLAUNCH((k_dw_dense<FC, 1>), dim3(gx, gy), dim3(256), lds, s, a);
    else if (maxi <= 3) HGNN_KLAUNCH((k_dw_dense<FC, 3>), dim3(gx, gy), dim3(256), lds, s, a);
    else HGNN_KLAUNCH((k_dw_dense<FC, 5>), dim3(gx, gy), dim3(256), lds, s, a);
}

// Narrow inputs (F <= 16: layer 0's node features, the GNN_simple layers of config 1): the outer
// products are a handful of FMAs per output, so one block per graph computes them straight from
// LDS copies of G and X -- no 32-wide MFMA tiles padded from F = 4 or 5 to 32 channels.  Same
// padded-position values as k_dw_dense (dG = 0 at padded n outside the readout, the BN of 0 at
// padded m); f summed in order.
__global__ void __launch_bounds__(256) k_dw_dense_narrow(DwDenseArgs a) {
    WaveStamp stamp(a.stamps);
    extern __shared__ float sm[];
    const int b = blockIdx.x;
    const int nmax = a.nmax, J = a.jt, F = a.f, JF = J * F;
    float* G = sm;               // [nmax][J F]
    float* X = sm + nmax * JF;   // [nmax][F]
    const int off = a.node_off[b], nb = a.node_off[b + 1] - off;
    const float pw = a.pmean ? *a.pw : 0.f, pb = a.pmean ? *a.pb : 0.f;
    for (int i = threadIdx.x; i < nmax * JF; i += 256) {
        const int n = i / JF, q = i - n * JF;
        G[i] = n < nb ? a.dA[(long long)(off + n) * a.lda + q] : 0.f;
    }
    for (int i = threadIdx.x; i < nmax * F; i += 256) {
        const int m = i / F, f = i - m * F;
        float x;
        if (a.xdense) x = a.xdense[((long long)b * F + f) * nmax + m];
        else if (m < nb) {
            x = a.xp[(long long)(off + m) * F + f];
            if (a.pmean) x = bn_z_s(x, a.pmean[f], bn_scale(pw, a.pstd[f]), pb);
        } else {
            x = a.pmean ? bn_z(0.f, a.pmean[f], a.pstd[f], pw, pb) : 0.f;
        }
        X[i] = x;
    }
    __syncthreads();
    float* dWb = a.dW + (long long)b * nmax * nmax * J;
    const int tot = nmax * nmax * J;
    // gridDim.y blocks of a graph split its outputs (few graphs: cfg1's 32 would be 32 blocks)
    for (int i = blockIdx.y * 256 + threadIdx.x; i < tot; i += 256 * gridDim.y) {
        const int n = i / (nmax * J), m = (i / J) % nmax, j = i % J;
        const float* g = G + n * JF + j * F;
        const float* x = X + m * F;
        float v = 0.f;
        for (int f = 0; f < F; ++f) v = fmaf(g[f], x[f], v);
        dWb[i] = a.accumulate ? dWb[i] + v : v;
    }
}

int launch_dw_dense(const DwDenseArgs& a, hipStream_t s) {
    static const bool narrow_ok = [] {
        const char* e = getenv("HGNN_DW_NARROW");
        return !e || e[0] != '0';
    }();
    if (narrow_ok && a.f <= 16 && !a.dout) {
        const size_t lds = sizeof(float) * (size_t)a.nmax * (a.jt * a.f + a.f);
        if (lds <= 64 * 1024) {
            const int gy = std::max(1, std::min(16, 512 / std::max(1, a.bs)));
            DwDenseArgs as = a;
            as.stamps = clock_stamps((long long)a.bs * gy * 4);
            HGNN_KLAUNCH(k_dw_dense_narrow, dim3(a.bs, gy), dim3(256), lds, s, as);
            HGNN_LAUNCH_CHECK();
            return 0;
        }
    }
    const int npad = (a.nmax + 31) / 32 * 32;
    // one F chunk when it fits (F = 2d = 128 at config 2): 19.1 -> 18.3 us per launch
    int fc = npad <= 32 ? (a.f > 64 ? 128 : 64) : (npad <= 64 ? 32 : 16);
    const int tiles = npad / 32;
    // few graphs (cfg1: 32): the items' passes of a graph spread over blocks, so the grid is not a
    // handful of long blocks
    const int J = a.jt;
    auto lds_of = [&](int c) {
        return sizeof(float) * ((size_t)npad * ((J * c + 1) + (c + 1)) + (size_t)J * c + 3 * c);
    };
    // the graph's G and X rows stay in LDS (up to the CU's 160 KB): SBM graphs of several hundred
    // nodes take 8-channel chunks (Nmax <= ~1200 at J + 2 = 3 slices)
    if (lds_of(fc) > 160 * 1024) fc = 8;
    const size_t lds = lds_of(fc);
    if (lds > 160 * 1024) return HGNN_ERR_UNSUPPORTED;
    const int nitems = tiles * tiles * J;
    int maxi = ceil_div(nitems, 4), gy = 1;
    if (a.bs < 256 && nitems > 4) {
        maxi = 1;
        gy = ceil_div(nitems, 4);
    }
    if (fc == 128) launch_fc<128>(a, maxi, gy, lds, s);
    else if (fc == 64) launch_fc<64>(a, maxi, gy, lds, s);
    else if (fc == 32) launch_fc<32>(a, maxi, gy, lds, s);
    else if (fc == 16) launch_fc<16>(a, maxi, gy, lds, s);
    else launch_fc<8>(a, maxi, gy, lds, s);
    HGNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace hgnn
