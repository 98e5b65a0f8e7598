// CCN-2D on small graphs (nmax <= 32): one workgroup per graph, every level of a call in one dispatch.
//
// The reference's driver runs CCN_2D one graph per step (scripts/train_ccn.py:31-73: net(X, A + I), loss,
// backward, an optimizer step), and a QM9 graph has at most 29 nodes of degree ~2-6.  The general path
// (ccn.hip) spends such a call on dispatches: 3 plan kernels, pack, a level kernel per layer, two readout
// kernels forward; the readout backward, per level a node pass, a parameter reduction and a gather, and an
// unpack backward.  Here one 512-thread workgroup per graph
//   * builds the receptive fields in LDS (row bit sets of the adjacency, utils_ccn.py:159-163; degrees,
//     self positions, the exclusive prefixes of d and d^2; every chi position by popcount, 66-106),
//   * runs each level node by node, one wave per node: the promotion, the closed-form collapse6to3 and the
//     Linear + ReLU of k_c2_fwd (utils_ccn.py:281-300, contraction.py:106-121), then the readout
//     (model_ccn.py:102-105) -- forward: one dispatch;
//   * backward: the readout backward, then per level the node pass of k_c2_bwd (dp format, parameter
//     partials), the gather of k_c2_gather (levels >= 1) or the level-0 sum of k_ccn2_dx0 -- one dispatch
//     (+ one reduction over the graphs when bs > 1).
// Same arithmetic in the same order as the general kernels, so outputs, dX and (bs = 1) the parameter
// gradients are those of the general path bit for bit: where k_c2_fwd / k_c2_bwd give the receptive-field
// rows b to four waves (b = w, w + 4, ...) and add the four waves' partials, the node's one wave walks the
// same four row classes one after the other and adds their partials in the same order; where a general
// kernel spreads n^2 entries over 256 threads (e = t, t + 256, ...), the wave walks the four 64-entry
// classes of t likewise.  The helpers the two paths share are in ccn2_shared.h.
//
// Levels F_l, the dp format and the level-0 terms live in a per-graph global workspace region (the rows of
// a graph's levels: sum_i d_i^2 <= nmax^3); plan, weights and per-node scratch in LDS.
#include <cstdint>

#include "ccn2_shared.h"

namespace hgnn {
namespace {

constexpr int Q_NT = 512, Q_NW = Q_NT / 64;  // one wave per node: QM9's <= 29 nodes in <= 4 rounds
constexpr int Q_N = 32;                      // nmax bound (a row of the pattern in one ballot word)
constexpr int Q_CF = 8;                      // f_in bound: the general path's CM = 8 level-0 instantiation
constexpr int Q_H = 2;                       // hidden bound: one HC = 2 output pass, CM = 2 at levels >= 1
constexpr int Q_HC = 2;
constexpr int Q_LMAX = 15;
constexpr int Q_NF = 64;                     // readout width bound (f + L h <= 8 + 15 * 2)
constexpr int Q_RT = 256;                    // threads of the general readout / reduction kernels

struct QArgs {
    const float* adj;          // (bs, nmax, nmax) with self loops
    const int64_t* n_batch;    // (bs,) or null
    const float* X;            // (bs, nmax, f)
    int bs, nmax, f, h, L, n_out;
    long long r1, r2;          // per-graph row bounds: sum d <= nmax^2, sum d^2 <= nmax^3
    long long gstride;         // floats of one graph's workspace region
    const float* W[Q_LMAX];
    const float* B[Q_LMAX];
    const float* fcw;
    const float* fcb;
    float* feat;               // [bs][nf] readout features (forward writes, backward reads)
    float* ppart[Q_LMAX];      // per level [bs nmax][h K_l + h] node partials at the packed node index
    float* gws;                // graph regions
    float* out;                // forward
    int* err;
    int tag;
    const float* dout;         // backward
    float* gW[Q_LMAX];
    float* gB[Q_LMAX];
    float* gfcw;
    float* gfcb;
    float* dX;
};

struct QGraph {
    unsigned long long bits[Q_N];     // row bit sets
    int deg[Q_N], selfpos[Q_N];
    int off1[Q_N + 4], off2[Q_N + 4];  // exclusive prefixes of d and d^2 (graph-local row offsets)
    unsigned char nbr[Q_N * Q_N];     // ascending neighbour ids
    float Xs[Q_N * Q_CF];             // [n][f]
    float wc[NWC * Q_HC * Q_CF];      // the level's combined weights (c2_weights)
    float nsum[Q_LMAX][Q_N][Q_H];     // per-node sums of F_l (the readout's per-level features)
    float vec[Q_NF];                  // readout features (forward) / dsum (backward)
    double dred[4][Q_CF];
    int base;                         // packed index of the graph's first node
};

struct QWave {
    unsigned long long vmask[Q_N];
    int oj[Q_N], dj[Q_N], o1[Q_N], ii[Q_N], aj[Q_N];
    float xs[Q_N][Q_CF];
    float qw[4][Q_N][Q_HC];
    float q3p[Q_N][Q_HC];
    float q3s[Q_N][Q_HC];
    float d3s[Q_N][Q_HC];
    float rdpL[Q_N][Q_HC];
    float rs[Q_N][4][Q_HC];
    float gs[Q_N][Q_CF];
    float red[4][C2_NACC][Q_HC][Q_HC];
    float redt[4][2][Q_HC];
    float redb[4][Q_HC];
    float trL[Q_HC], s_diag[Q_HC];
};

__host__ __device__ inline size_t q_al16(size_t x) { return (x + 15) / 16 * 16; }
__host__ __device__ inline size_t q_sp_bytes(int nmax) { return q_al16(2 * (size_t)nmax * nmax); }
__host__ __device__ inline size_t q_p_bytes(int nmax) { return q_al16(4 * (size_t)nmax * nmax * Q_HC); }
__host__ __device__ inline size_t q_wave_bytes(int nmax) {
    return q_al16(sizeof(QWave)) + q_sp_bytes(nmax) + q_p_bytes(nmax);
}
__host__ __device__ inline size_t q_lds_bytes(int nmax) { return q_al16(sizeof(QGraph)) + Q_NW * q_wave_bytes(nmax); }
constexpr size_t Q_LDS_MAX = 160 * 1024;

// LDS accesses of one wave's lanes to each other's entries: the LDS executes a wave's operations in order,
// so a compiler barrier is all that is needed between a store and another lane's load
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int q_nodes(const QArgs& a, int b, uint32_t& bad) {
    int n = a.n_batch ? (int)a.n_batch[b] : a.nmax;
    if (n < 0 || n > a.nmax) {
        bad |= ERR_SIZES;
        n = n < 0 ? 0 : a.nmax;
    }
    return n;
}

// Graph b's receptive fields, offsets, packed base index and node features in LDS; returns this lane's
// validation bits (the general plan's ERR_CCN_SELFLOOP / ERR_CCN_ASYM)
__device__ uint32_t q_plan(const QArgs& a, int b, int n, QGraph& g) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float* A = a.adj + (long long)b * a.nmax * a.nmax;
    uint32_t bad = 0;
    for (int r = wv; r < n; r += Q_NW) {
        const bool nz = lane < n && A[(long long)r * a.nmax + lane] > 0.f;  // utils_ccn.py:195 (A > 0)
        const unsigned long long m = __ballot(nz);
        if (nz) g.nbr[r * Q_N + __popcll(m & ((1ull << lane) - 1ull))] = (unsigned char)lane;
        const bool self = (m >> r) & 1ull;
        if (lane == 0) {
            g.bits[r] = m;
            g.deg[r] = __popcll(m);
            g.selfpos[r] = self ? __popcll(m & ((1ull << r) - 1ull)) : -1;
        }
        if (!self) bad |= ERR_CCN_SELFLOOP;
    }
    for (int e = threadIdx.x; e < n * a.f; e += Q_NT) g.Xs[e] = a.X[(long long)b * a.nmax * a.f + e];
    __syncthreads();
    if (wv == 0) {
        const int d = lane < n ? g.deg[lane] : 0;
        int x1 = d, x2 = d * d;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t1 = __shfl_up(x1, o, 64), t2 = __shfl_up(x2, o, 64);
            if (lane >= o) {
                x1 += t1;
                x2 += t2;
            }
        }
        if (lane <= Q_N) {
            g.off1[lane] = x1 - d;
            g.off2[lane] = x2 - d * d;
        }
    } else if (wv == 1) {
        int s = 0;
        if (a.n_batch) {
            for (int q = lane; q < b; q += 64) {
                const long long v = a.n_batch[q];
                s += v < 0 ? 0 : (v > a.nmax ? a.nmax : (int)v);
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        } else {
            s = b * a.nmax;
        }
        if (lane == 0) g.base = s;
    }
    // every neighbour j of r must list r (the gathers walk N(j) for the readers of F_j)
    for (int r = wv; r < n; r += Q_NW) {
        const unsigned long long m = g.bits[r];
        if (lane < n && ((m >> lane) & 1ull) && !((g.bits[lane] >> r) & 1ull)) bad |= ERR_CCN_ASYM;
    }
    __syncthreads();
    return bad;
}

// node i's position maps (int16, the general kernels' sp), its neighbours' row offsets / degrees / level-0
// features and the common-neighbourhood masks (c2_prologue)
template <int CM>
__device__ __forceinline__ void q_prologue(const QGraph& g, QWave& w, short* sp, int i, int n, bool level0, int cin,
                                           int f) {
    const int lane = threadIdx.x & 63;
    for (int e = lane; e < n * n; e += 64) {
        const int ai = e / n, x = e - ai * n;
        const int j = g.nbr[i * Q_N + ai], u = g.nbr[i * Q_N + x];
        const unsigned long long m = g.bits[j];
        sp[e] = ((m >> u) & 1ull) ? (short)__popcll(m & ((1ull << u) - 1ull)) : (short)-1;
    }
    if (lane < n) {
        const int j = g.nbr[i * Q_N + lane];
        w.oj[lane] = g.off2[j];
        w.dj[lane] = g.deg[j];
#pragma unroll
        for (int c = 0; c < CM; ++c) w.xs[lane][c] = (level0 && c < cin) ? g.Xs[j * f + c] : 0.f;
    }
    wsync();
    for (int ai = 0; ai < n; ++ai) {
        const unsigned long long m = __ballot(lane < n && sp[ai * n + lane] >= 0);
        if (lane == 0) w.vmask[ai] = m;
    }
    wsync();
}

// One node of a forward level: k_c2_fwd's arithmetic (one output pass: h <= HC)
template <int CM, int NB, bool L0>
__device__ void q_node_fwd(const QArgs& a, QGraph& g, QWave& w, short* sp, float* P, int i, int l, const float* fin,
                           int cin, float* fout) {
    constexpr int HC = Q_HC;
    const int lane = threadIdx.x & 63;
    const int h = a.h, hc = h, o0 = 0;
    const float* bias = a.B[l];
    const float(*wc)[HC][CM] = reinterpret_cast<const float(*)[HC][CM]>(g.wc);
    const int n = g.deg[i];
    q_prologue<CM>(g, w, sp, i, n, L0, cin, a.f);
    const long long o2 = g.off2[i];
    const float nf = (float)n;
    const bool la = lane < n;
    const unsigned long long my_mask = la ? w.vmask[lane] : 0ull;
    const int my_oj = la ? w.oj[lane] : 0, my_dj = la ? w.dj[lane] : 0;
    for (int e = lane; e < n * n * HC; e += 64) P[e] = 0.f;
    wsync();
    if constexpr (L0) {
        float vacc[HC];
#pragma unroll
        for (int o = 0; o < HC; ++o) vacc[o] = 0.f;
        const float mf = (float)__popcll(my_mask);
        const bool va = la && ((my_mask >> lane) & 1ull);
        float u[HC], dl[HC], bx[HC], q3a[HC];
#pragma unroll
        for (int o = 0; o < HC; ++o) {
            u[o] = dl[o] = bx[o] = q3a[o] = 0.f;
#pragma unroll
            for (int c = 0; c < CM; ++c) {
                if (c >= cin) break;
                const float x = la ? w.xs[lane][c] : 0.f;
                u[o] = fmaf(fmaf(fmaf(nf, wc[WA][o][c], wc[WB][o][c]), mf, wc[WQ15][o][c]), x, u[o]);
                dl[o] = fmaf(wc[WQ16][o][c], x, dl[o]);
                bx[o] = fmaf(nf * wc[WQ2][o][c], x, bx[o]);
                vacc[o] = fmaf(wc[WQ1][o][c], x, vacc[o]);
                q3a[o] = fmaf(wc[WQ3][o][c], x, q3a[o]);
            }
            dl[o] = va ? dl[o] : 0.f;
            vacc[o] *= mf * mf;
            q3a[o] *= mf;
        }
        {  // k_c2_fwd's wave 0: [x = y](W4 tot + W17 d3)
            float dg[HC];
#pragma unroll
            for (int o = 0; o < HC; ++o) dg[o] = 0.f;
#pragma unroll
            for (int c = 0; c < CM; ++c) {
                if (c >= cin) break;
                const float x = la ? w.xs[lane][c] : 0.f;
                const float tt = wave_total(mf * mf * x), dd = wave_total(va ? x : 0.f);
#pragma unroll
                for (int o = 0; o < HC; ++o) dg[o] = fmaf(wc[WQ4][o][c], tt, fmaf(wc[WQ17][o][c], dd, dg[o]));
            }
            if (lane == 0)
#pragma unroll
                for (int o = 0; o < HC; ++o) w.s_diag[o] = dg[o];
        }
        for (int b = 0; b < n; ++b) {
            const unsigned long long ab = __ballot(la && ((my_mask >> b) & 1ull));
            const bool in = (ab >> lane) & 1ull;
            float s[HC];
#pragma unroll
            for (int o = 0; o < HC; ++o) {
                if (in && o < hc) P[(lane * n + b) * HC + o] += u[o];
                s[o] = in ? dl[o] : 0.f;
                const float q = wave_total(in ? q3a[o] : 0.f);
                if (lane == 0) w.q3p[b][o] = q;
            }
            unsigned long long as = ab;
            while (as) {
                const int aa = __ffsll((long long)as) - 1;
                as &= as - 1ull;
                const bool vz = (lane_value_u64(my_mask, aa) >> lane) & 1ull;
#pragma unroll
                for (int o = 0; o < HC; ++o) {
                    const float bxa = lane_value(bx[o], aa);
                    s[o] += vz ? bxa : 0.f;
                }
            }
            if (la)
#pragma unroll
                for (int o = 0; o < HC; ++o)
                    if (o < hc) P[(b * n + lane) * HC + o] += s[o];
            wsync();
        }
        // W1 q1[a] once (k_c2_fwd keeps wave 0's copy, the other waves add zeros)
        if (la)
#pragma unroll
            for (int o = 0; o < HC; ++o) {
                w.qw[0][lane][o] = vacc[o];
                w.qw[1][lane][o] = w.qw[2][lane][o] = w.qw[3][lane][o] = 0.f;
            }
    } else {
        static_assert(CM == Q_HC, "levels >= 1 have cin = hidden <= 2 channels");
        for (int cls = 0; cls < 4; ++cls) {  // k_c2_fwd's wave cls: rows b = cls, cls + 4, ...
            float vacc[HC];
#pragma unroll
            for (int o = 0; o < HC; ++o) vacc[o] = 0.f;
            for (int b = cls; b < n; b += 4) {
                float sa[CM], sck[CM], d1k[CM], d2k[CM];
#pragma unroll
                for (int c = 0; c < CM; ++c) sa[c] = sck[c] = d1k[c] = d2k[c] = 0.f;
                if (lane == 0)
#pragma unroll
                    for (int c = 0; c < CM; ++c) w.d3s[b][c] = 0.f;
                const unsigned long long ab = __ballot(la && ((my_mask >> b) & 1ull));
                const bool in = (ab >> lane) & 1ull;
                const float* my_row = c2_row_of(fin, cin, sp, n, b, in, my_oj, my_dj);
                unsigned long long as = ab;
                while (as) {
                    int aa[NB];
                    c2_take<NB>(as, aa);
                    float t[NB][CM];
                    c2_load_rows<CM, NB>(cin, n, aa, sp, my_mask, my_row, t);
#pragma unroll
                    for (int u = 0; u < NB; ++u) {
                        const int av = aa[u];
                        if (av < 0) break;
                        const bool me = lane == av;
#pragma unroll
                        for (int c = 0; c < CM; ++c) {
                            if (c >= cin) break;
                            const float sc = wave_total(t[u][c]);
                            const float d1 = lane_value(t[u][c], b);
                            sck[c] = me ? sc : sck[c];
                            d1k[c] = me ? d1 : d1k[c];
                            d2k[c] = me ? t[u][c] : d2k[c];
                            sa[c] += t[u][c];
                        }
                        if (av == b && lane == b)
#pragma unroll
                            for (int c = 0; c < CM; ++c) w.d3s[b][c] = t[u][c];
                    }
                }
                float q3[CM];
#pragma unroll
                for (int c = 0; c < CM; ++c) q3[c] = c < cin ? wave_total(sa[c]) : 0.f;
#pragma unroll
                for (int o = 0; o < HC; ++o) {
                    if (o >= hc) break;
                    float U = 0.f, V = 0.f, S = 0.f;
#pragma unroll
                    for (int c = 0; c < CM; ++c) {
                        if (c >= cin) break;
                        U = fmaf(fmaf(nf, wc[WA][o][c], wc[WB][o][c]), sck[c], U);
                        U = fmaf(wc[WQ15][o][c], d1k[c], U);
                        V = fmaf(wc[WQ1][o][c], sck[c], V);
                        S = fmaf(nf * wc[WQ2][o][c], sa[c], S);
                        S = fmaf(wc[WQ16][o][c], d2k[c], S);
                    }
                    if (in) P[(lane * n + b) * HC + o] += U;
                    vacc[o] += in ? V : 0.f;
                    if (la) P[(b * n + lane) * HC + o] += S;
                    if (lane == 0) {
                        float q = 0.f;
#pragma unroll
                        for (int c = 0; c < CM; ++c) q = fmaf(wc[WQ3][o][c], q3[c], q);
                        w.q3p[b][o] = q;
                    }
                }
                if (lane == 0)
#pragma unroll
                    for (int c = 0; c < CM; ++c) w.q3s[b][c] = q3[c];
                wsync();
            }
            if (la)
#pragma unroll
                for (int o = 0; o < HC; ++o) w.qw[cls][lane][o] = vacc[o];
        }
        wsync();
        if (lane < hc) {  // [x = y](W4 tot + W17 d3), sums over b in a fixed order
            const int o = lane;
            float dg = 0.f;
            for (int c = 0; c < cin; ++c) {
                float tt = 0.f, dd = 0.f;
                for (int b = 0; b < n; ++b) {
                    tt += w.q3s[b][c];
                    dd += w.d3s[b][c];
                }
                dg = fmaf(wc[WQ4][o][c], tt, dg);
                dg = fmaf(wc[WQ17][o][c], dd, dg);
            }
            w.s_diag[o] = dg;
        }
    }
    wsync();
    // F_out entries and the node's sum of them (k_c2_fwd's 256 threads: the four 64-entry classes)
    float nsw[4][HC];
#pragma unroll
    for (int vw = 0; vw < 4; ++vw) {
        float ns[HC];
#pragma unroll
        for (int o = 0; o < HC; ++o) ns[o] = 0.f;
        for (int e = vw * 64 + lane; e < n * n; e += 256) {
            const int x = e / n, y = e - x * n;
#pragma unroll
            for (int o = 0; o < HC; ++o) {
                if (o >= hc) break;
                float s = bias[o0 + o] + P[e * HC + o];
                s += (w.qw[0][x][o] + w.qw[1][x][o]) + (w.qw[2][x][o] + w.qw[3][x][o]);
                s += w.q3p[x][o];
                if (x == y) s += w.s_diag[o];
                s = s < 0.f ? 0.f : s;
                fout[(o2 + e) * h + o0 + o] = s;
                ns[o] += s;
            }
        }
#pragma unroll
        for (int o = 0; o < HC; ++o) nsw[vw][o] = wave_total(ns[o]);
    }
    if (lane < hc) {
        const int o = lane;
        g.nsum[l][i][o0 + o] = (nsw[0][o] + nsw[1][o]) + (nsw[2][o] + nsw[3][o]);
    }
    wsync();
}

// Readout column sums in fp64 (k_ccn_readout_part's order for a one-chunk graph, k_ccn_readout's feat):
// vec[col0 + c] = (float)(0 + sum over rows r of val(r, c)), rows over the first 256 threads, then their 4 waves
template <typename V>
__device__ void q_colsum(QGraph& g, int rows, int nc, int col0, V val) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double acc[Q_CF];
#pragma unroll
    for (int c = 0; c < Q_CF; ++c) acc[c] = 0.0;
    if ((int)threadIdx.x < Q_RT)
        for (int r = threadIdx.x; r < rows; r += Q_RT)
            for (int c = 0; c < nc; ++c) val(r, c, acc[c]);
    for (int c = 0; c < nc; ++c) {
        const double t = wave_sum_d(acc[c]);
        if (lane == 0 && wv < 4) g.dred[wv][c] = t;
    }
    __syncthreads();
    if ((int)threadIdx.x < nc) {
        const int c = threadIdx.x;
        const double pb = g.dred[0][c] + g.dred[1][c] + g.dred[2][c] + g.dred[3][c];
        double t = 0.0;
        t += pb;
        g.vec[col0 + c] = (float)t;
    }
    __syncthreads();
}

template <int CF>
__global__ void __launch_bounds__(Q_NT) k_ccn2_small_fwd(QArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    __shared__ uint32_t sbad;
    __shared__ double sred[4];
    QGraph& g = *reinterpret_cast<QGraph*>(lds);
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    char* wbase = lds + q_al16(sizeof(QGraph)) + (size_t)wv * q_wave_bytes(a.nmax);
    QWave& w = *reinterpret_cast<QWave*>(wbase);
    short* sp = reinterpret_cast<short*>(wbase + q_al16(sizeof(QWave)));
    float* P = reinterpret_cast<float*>(wbase + q_al16(sizeof(QWave)) + q_sp_bytes(a.nmax));
    if (threadIdx.x == 0) sbad = 0;
    uint32_t bad = 0;
    const int n = q_nodes(a, b, bad);
    bad |= q_plan(a, b, n, g);
    const int f = a.f, h = a.h, nf = f + a.L * h;
    float* G = a.gws + (long long)b * a.gstride;
    // level 0 of the readout: sum_i d_i^2 X[i] (utils_ccn.py:167-172 tile X[i] d_i x d_i times)
    q_colsum(g, n, f, 0, [&](int r, int c, double& acc) {
        const double d = g.deg[r];
        const double wgt = d * d;
        acc += wgt * (double)g.Xs[r * f + c];
    });
    for (int l = 0; l < a.L; ++l) {
        const int cin = l == 0 ? f : h;
        float* fout = G + (long long)l * a.r2 * h;
        const float* fin = l == 0 ? nullptr : G + (long long)(l - 1) * a.r2 * h;
        if (l == 0) c2_weights<Q_HC, CF>(reinterpret_cast<float(*)[Q_HC][CF]>(g.wc), a.W[l], cin, 0, h);
        else c2_weights<Q_HC, Q_HC>(reinterpret_cast<float(*)[Q_HC][Q_HC]>(g.wc), a.W[l], cin, 0, h);
        __syncthreads();
        for (int i = wv; i < n; i += Q_NW) {
            if (l == 0) q_node_fwd<CF, 1, true>(a, g, w, sp, P, i, l, fin, cin, fout);
            else q_node_fwd<Q_HC, 8, false>(a, g, w, sp, P, i, l, fin, cin, fout);
        }
        __syncthreads();
        q_colsum(g, n, h, f + l * h, [&](int r, int c, double& acc) { acc += (double)g.nsum[l][r][c]; });
    }
    for (int k = threadIdx.x; k < nf; k += Q_NT) a.feat[(long long)b * nf + k] = g.vec[k];
    // out = fc(feat) in fp64 (k_ccn_readout's order)
    for (int o = 0; o < a.n_out; ++o) {
        double s = 0.0;
        if ((int)threadIdx.x < Q_RT)
            for (int k = threadIdx.x; k < nf; k += Q_RT) s += (double)a.fcw[o * nf + k] * (double)g.vec[k];
        s = wave_sum_d(s);
        __syncthreads();
        if (lane == 0 && wv < 4) sred[wv] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            const double t = sred[0] + sred[1] + sred[2] + sred[3];
            a.out[(long long)b * a.n_out + o] = (float)(t + (double)a.fcb[o]);
        }
    }
    for (int o = 32; o > 0; o >>= 1) bad |= (uint32_t)__shfl_xor((int)bad, o, 64);
    if (lane == 0 && bad) atomicOr(&sbad, bad);
    __syncthreads();
    if (threadIdx.x == 0 && sbad) a.err[0] = a.tag * 256 + (int)sbad;  // vector store (host-mapped word)
}

// One node of a backward level: k_c2_bwd's arithmetic.  dF: this level's dF (read, then overwritten by dp;
// the top level reads dtop instead); pp: the node's partial row; g0: level 0's per-neighbour terms.
template <int CM, int NB, bool L0>
__device__ void q_node_bwd(const QArgs& a, QGraph& g, QWave& w, short* sp, float* dpL, int i, float* dF,
                           const float* dtop, const float* F, const float* fin, int cin, float* rdp_g, float* trd_g,
                           float* pp, float* g0) {
    constexpr int HC = Q_HC;
    const int lane = threadIdx.x & 63;
    const int h = a.h, hc = h, o0 = 0;
    const float(*wc)[HC][CM] = reinterpret_cast<const float(*)[HC][CM]>(g.wc);
    const int n = g.deg[i];
    q_prologue<CM>(g, w, sp, i, n, L0, cin, a.f);
    const long long o2 = g.off2[i], o1 = g.off1[i];
    const bool la = lane < n;
    const unsigned long long my_mask = la ? w.vmask[lane] : 0ull;
    const int my_oj = la ? w.oj[lane] : 0, my_dj = la ? w.dj[lane] : 0;
    const float nf = (float)n;
    const int K = 18 * cin;
    if (L0)
        for (int e = lane; e < n * CM; e += 64) (&w.gs[0][0])[(e / CM) * Q_CF + e % CM] = 0.f;
    // dp = dF relu'(F_out), its per-class column sums (the bias partial)
#pragma unroll
    for (int vw = 0; vw < 4; ++vw) {
        float sb[HC];
#pragma unroll
        for (int o = 0; o < HC; ++o) sb[o] = 0.f;
        for (int e = vw * 64 + lane; e < n * n; e += 256) {
#pragma unroll
            for (int o = 0; o < HC; ++o) {
                float d = 0.f;
                if (o < hc) {
                    const long long r = (o2 + e) * h + o0 + o;
                    d = F[r] > 0.f ? (dtop ? dtop[o0 + o] : dF[r]) : 0.f;
                    dF[r] = d;
                }
                dpL[e * HC + o] = d;
                sb[o] += d;
            }
        }
#pragma unroll
        for (int o = 0; o < HC; ++o) {
            const float t = wave_total(sb[o]);
            if (lane == 0) w.redb[vw][o] = t;
        }
    }
    wsync();
    // row sums and trace of dp
    for (int x = 0; x < n; ++x)
#pragma unroll
        for (int o = 0; o < HC; ++o) {
            const float r = wave_total(lane < n ? dpL[(x * n + lane) * HC + o] : 0.f);
            if (lane == 0) {
                w.rdpL[x][o] = r;
                if (o < hc) rdp_g[(o1 + x) * h + o0 + o] = r;
            }
        }
#pragma unroll
    for (int o = 0; o < HC; ++o) {
        const float r = wave_total(lane < n ? dpL[(lane * n + lane) * HC + o] : 0.f);
        if (lane == 0) {
            w.trL[o] = r;
            if (o < hc) trd_g[(long long)i * h + o0 + o] = r;
        }
    }
    wsync();
    if constexpr (L0) {
        for (int av = 0; av < n; ++av) {
            const unsigned long long ma = w.vmask[av];
            const bool vb = lane < n && ((ma >> lane) & 1ull);
#pragma unroll
            for (int o = 0; o < HC; ++o) {
                const float r1 = wave_total(vb ? dpL[(av * n + lane) * HC + o] : 0.f);
                const float r2 = wave_total(vb ? dpL[(lane * n + av) * HC + o] : 0.f);
                const float r3 = wave_total(vb ? w.rdpL[lane][o] : 0.f);
                float s = 0.f;
                unsigned long long zs = ma;
                while (zs) {
                    const int z = __ffsll((long long)zs) - 1;
                    zs &= zs - 1ull;
                    s += vb ? dpL[(lane * n + z) * HC + o] : 0.f;
                }
                const float bs = wave_total(s);
                if (lane == 0) {
                    w.rs[av][0][o] = r1;
                    w.rs[av][1][o] = r2;
                    w.rs[av][2][o] = r3;
                    w.rs[av][3][o] = bs;
                }
            }
        }
        wsync();
        for (int p = 0; p < hc * cin; ++p) {
            const int o = p / cin, c = p % cin;
            const float mf = (float)__popcll(my_mask);
            const bool va = la && ((my_mask >> lane) & 1ull);
            const float x = la ? w.xs[lane][c] : 0.f;
            const float r1 = la ? w.rs[lane][0][o] : 0.f, r2 = la ? w.rs[lane][1][o] : 0.f;
            const float r3 = la ? w.rs[lane][2][o] : 0.f, bs = la ? w.rs[lane][3][o] : 0.f;
            const float ra = la ? w.rdpL[lane][o] : 0.f;
            const float s0 = wave_total(mf * x * r1), s1 = wave_total(mf * mf * x * ra);
            const float s2 = wave_total(x * bs), s3 = wave_total(mf * x * r3);
            const float s15 = wave_total(x * r1), s16 = wave_total(va ? x * r2 : 0.f);
            const float tt = wave_total(mf * mf * x), dd = wave_total(va ? x : 0.f);
            if (lane == 0)
                c2_write_partials(pp + (long long)(o0 + o) * K, cin, c, nf, s0, s1, s2, s3, s15, s16, w.trL[o] * tt,
                                  w.trL[o] * dd);
        }
        for (int t = lane; t < n * cin; t += 64) {
            const int av = t / cin, c = t % cin;
            const unsigned long long ma = w.vmask[av];
            const float mf = (float)__popcll(ma);
            const bool va = (ma >> av) & 1ull;
            float gg = 0.f;
            for (int o = 0; o < hc; ++o) {
                const float r1 = w.rs[av][0][o], r2 = w.rs[av][1][o], r3 = w.rs[av][2][o], bs = w.rs[av][3][o];
                float s = mf * fmaf(fmaf(nf, wc[WA][o][c], wc[WB][o][c]), r1, mf * wc[WQ1][o][c] * w.rdpL[av][o]);
                s = fmaf(nf * wc[WQ2][o][c], bs, s);
                s = fmaf(mf * wc[WQ3][o][c], r3, s);
                s = fmaf(mf * mf * wc[WQ4][o][c], w.trL[o], s);
                s = fmaf(wc[WQ15][o][c], r1, s);
                if (va) s = fmaf(wc[WQ16][o][c], r2, fmaf(wc[WQ17][o][c], w.trL[o], s));
                gg += s;
            }
            w.gs[av][c] += gg;
        }
    } else {
        static_assert(CM == Q_HC, "levels >= 1 have cin = hidden <= 2 channels");
        for (int cls = 0; cls < 4; ++cls) {  // k_c2_bwd's wave cls
            float acc[C2_NACC][HC][CM], tot[CM], d3[CM];
#pragma unroll
            for (int k = 0; k < C2_NACC; ++k)
#pragma unroll
                for (int o = 0; o < HC; ++o)
#pragma unroll
                    for (int c = 0; c < CM; ++c) acc[k][o][c] = 0.f;
#pragma unroll
            for (int c = 0; c < CM; ++c) tot[c] = d3[c] = 0.f;
            for (int b = cls; b < n; b += 4) {
                float sa[CM];
#pragma unroll
                for (int c = 0; c < CM; ++c) sa[c] = 0.f;
                unsigned long long as = __ballot(la && ((my_mask >> b) & 1ull));
                const float* my_row = c2_row_of(fin, cin, sp, n, b, (as >> lane) & 1ull, my_oj, my_dj);
                float my_ab[HC], my_ba[HC], my_ra[HC];
#pragma unroll
                for (int o = 0; o < HC; ++o) {
                    my_ab[o] = la ? dpL[(lane * n + b) * HC + o] : 0.f;
                    my_ba[o] = la ? dpL[(b * n + lane) * HC + o] : 0.f;
                    my_ra[o] = la ? w.rdpL[lane][o] : 0.f;
                }
                while (as) {
                    int aa[NB];
                    c2_take<NB>(as, aa);
                    float t[NB][CM];
                    c2_load_rows<CM, NB>(cin, n, aa, sp, my_mask, my_row, t);
#pragma unroll
                    for (int u = 0; u < NB; ++u) {
                        const int av = aa[u];
                        if (av < 0) break;
#pragma unroll
                        for (int o = 0; o < HC; ++o) {
                            const float dab = lane_value(my_ab[o], av), dba = lane_value(my_ba[o], av);
                            const float ra = lane_value(my_ra[o], av);
                            const float d15 = lane == b ? dab : 0.f, d16 = lane == av ? dba : 0.f;
#pragma unroll
                            for (int c = 0; c < CM; ++c) {
                                acc[0][o][c] = fmaf(dab, t[u][c], acc[0][o][c]);
                                acc[1][o][c] = fmaf(ra, t[u][c], acc[1][o][c]);
                                acc[4][o][c] = fmaf(d15, t[u][c], acc[4][o][c]);
                                acc[5][o][c] = fmaf(d16, t[u][c], acc[5][o][c]);
                            }
                        }
                        if (av == b && lane == b)
#pragma unroll
                            for (int c = 0; c < CM; ++c) d3[c] += t[u][c];
#pragma unroll
                        for (int c = 0; c < CM; ++c) sa[c] += t[u][c];
                    }
                }
#pragma unroll
                for (int o = 0; o < HC; ++o) {
                    const float dbz = lane < n ? dpL[(b * n + lane) * HC + o] : 0.f;
#pragma unroll
                    for (int c = 0; c < CM; ++c) acc[2][o][c] = fmaf(dbz, sa[c], acc[2][o][c]);
                }
#pragma unroll
                for (int c = 0; c < CM; ++c) {
                    if (c >= cin) break;
                    const float q3 = wave_total(sa[c]);
                    if (lane == 0) {
#pragma unroll
                        for (int o = 0; o < HC; ++o) acc[3][o][c] = fmaf(w.rdpL[b][o], q3, acc[3][o][c]);
                        tot[c] += q3;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < C2_NACC; ++k) {
                if (k == 3) continue;
#pragma unroll
                for (int o = 0; o < HC; ++o)
#pragma unroll
                    for (int c = 0; c < CM; ++c) {
                        if (c >= cin) break;
                        acc[k][o][c] = wave_total(acc[k][o][c]);
                    }
            }
#pragma unroll
            for (int c = 0; c < CM; ++c) {
                if (c >= cin) break;
                d3[c] = wave_total(d3[c]);
            }
            if (lane == 0) {
#pragma unroll
                for (int k = 0; k < C2_NACC; ++k)
#pragma unroll
                    for (int o = 0; o < HC; ++o)
#pragma unroll
                        for (int c = 0; c < CM; ++c) w.red[cls][k][o][c] = acc[k][o][c];
#pragma unroll
                for (int c = 0; c < CM; ++c) {
                    w.redt[cls][0][c] = tot[c];
                    w.redt[cls][1][c] = d3[c];
                }
            }
        }
        wsync();
        for (int t = lane; t < hc * cin; t += 64) {
            const int o = t / cin, c = t % cin;
            float s[C2_NACC];
#pragma unroll
            for (int k = 0; k < C2_NACC; ++k)
                s[k] = (w.red[0][k][o][c] + w.red[1][k][o][c]) + (w.red[2][k][o][c] + w.red[3][k][o][c]);
            const float tt = (w.redt[0][0][c] + w.redt[1][0][c]) + (w.redt[2][0][c] + w.redt[3][0][c]);
            const float dd = (w.redt[0][1][c] + w.redt[1][1][c]) + (w.redt[2][1][c] + w.redt[3][1][c]);
            c2_write_partials(pp + (long long)(o0 + o) * K, cin, c, nf, s[0], s[1], s[2], s[3], s[4], s[5],
                              w.trL[o] * tt, w.trL[o] * dd);
        }
    }
    if (lane < hc)
        pp[(long long)h * K + o0 + lane] = (w.redb[0][lane] + w.redb[1][lane]) + (w.redb[2][lane] + w.redb[3][lane]);
    wsync();
    if (L0 && g0)
        for (int t = lane; t < n * cin; t += 64) g0[(o1 + t / cin) * cin + t % cin] = w.gs[t / cin][t % cin];
    wsync();
}

// Gather of node j's input gradient of level l >= 1 from the dp format: k_c2_gather<2, 8>'s arithmetic
__device__ void q_node_gather(const QArgs& a, QGraph& g, QWave& w, short* sp, int j, const float* dp,
                              const float* rdp, const float* trd, const float* rdv, float* dout) {
    constexpr int H = Q_HC, NB = 8;
    const int lane = threadIdx.x & 63;
    const int h = a.h;
    const float(*wc)[H][H] = reinterpret_cast<const float(*)[H][H]>(g.wc);
    const int n = g.deg[j];
    const long long o2 = g.off2[j];
    const int sj = g.selfpos[j];
    for (int e = lane; e < n * n; e += 64) {
        const int ai = e / n, x = e - ai * n;
        const int jj = g.nbr[j * Q_N + ai], u = g.nbr[j * Q_N + x];
        const unsigned long long m = g.bits[jj];
        sp[e] = ((m >> u) & 1ull) ? (short)__popcll(m & ((1ull << u) - 1ull)) : (short)-1;
    }
    if (lane < n) {
        const int i = g.nbr[j * Q_N + lane];
        w.ii[lane] = i;
        w.dj[lane] = g.deg[i];
        w.oj[lane] = g.off2[i];
        w.o1[lane] = g.off1[i];
    }
    wsync();
    for (int av = 0; av < n; ++av) {
        const unsigned long long m = __ballot(lane < n && sp[av * n + lane] >= 0);
        if (lane == 0) {
            w.vmask[av] = m;
            w.aj[av] = sp[av * n + sj];  // position of j in N(i_a)
        }
    }
    wsync();
    float rd[H];
#pragma unroll
    for (int c = 0; c < H; ++c) rd[c] = (rdv && c < h) ? rdv[c] : 0.f;
    const bool la = lane < n;
    const unsigned long long my_mask = la ? w.vmask[lane] : 0ull;
    const int my_i = la ? w.ii[lane] : 0, my_di = la ? w.dj[lane] : 0, my_oi = la ? w.oj[lane] : 0;
    const int my_o1 = la ? w.o1[lane] : 0, my_aj = la ? w.aj[lane] : 0;
    float my_ra[H], my_tr[H];
#pragma unroll
    for (int o = 0; o < H; ++o) {
        my_ra[o] = (la && o < h) ? rdp[((long long)my_o1 + my_aj) * h + o] : 0.f;
        my_tr[o] = (la && o < h) ? trd[(long long)my_i * h + o] : 0.f;
    }
    for (int u = 0; u < n; ++u) {
        float acc[H];
#pragma unroll
        for (int c = 0; c < H; ++c) acc[c] = 0.f;
        const unsigned long long au = __ballot(la && ((my_mask >> u) & 1ull));
        const bool in = (au >> lane) & 1ull;
        const int my_b = in ? (int)sp[lane * n + u] : 0;
        const float nfi = (float)my_di;
        float base[H], e1[H], e2[H], e3[H];
        {
            const float* pab = dp + ((long long)my_oi + (long long)my_aj * my_di + my_b) * h;
            const float* pba = dp + ((long long)my_oi + (long long)my_b * my_di + my_aj) * h;
            const float* prb = rdp + ((long long)my_o1 + my_b) * h;
            float vab[H], vba[H], vrb[H];
#pragma unroll
            for (int o = 0; o < H; ++o) {
                vab[o] = (in && o < h) ? pab[o] : 0.f;
                vba[o] = (in && o < h) ? pba[o] : 0.f;
                vrb[o] = (in && o < h) ? prb[o] : 0.f;
            }
#pragma unroll
            for (int c = 0; c < H; ++c) {
                float b0 = 0.f, x1 = 0.f, x2 = 0.f, x3 = 0.f;
#pragma unroll
                for (int o = 0; o < H; ++o) {
                    if (o >= h) break;
                    b0 = fmaf(fmaf(nfi, wc[WA][o][c], wc[WB][o][c]), vab[o], b0);
                    b0 = fmaf(wc[WQ1][o][c], my_ra[o], b0);
                    b0 = fmaf(wc[WQ3][o][c], vrb[o], b0);
                    b0 = fmaf(wc[WQ4][o][c], my_tr[o], b0);
                    x1 = fmaf(wc[WQ15][o][c], vab[o], x1);
                    x2 = fmaf(wc[WQ16][o][c], vba[o], x2);
                    x3 = fmaf(wc[WQ17][o][c], my_tr[o], x3);
                }
                base[c] = b0;
                e1[c] = x1;
                e2[c] = x2;
                e3[c] = x3;
            }
        }
        const float* my_row = dp + ((long long)my_oi + (long long)my_b * my_di) * h;
        unsigned long long as = au;
        while (as) {
            int aa[NB];
            c2_take<NB>(as, aa);
            float dz[NB][H];
            int zz[NB];
            bool vz[NB];
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                const int av = aa[q] >= 0 ? aa[q] : 0;
                vz[q] = aa[q] >= 0 && ((lane_value_u64(my_mask, av) >> lane) & 1ull);
                zz[q] = vz[q] ? (int)sp[av * n + lane] : 0;
                const float* pz = lane_value_ptr(my_row, av) + zz[q] * h;
#pragma unroll
                for (int o = 0; o < H; ++o) dz[q][o] = o < h ? pz[o] : 0.f;
            }
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                const int av = aa[q];
                if (av < 0) break;
                const int bb = lane_value_i(my_b, av), ajv = lane_value_i(my_aj, av);
                const float nfa = lane_value(nfi, av);
                const bool f1 = zz[q] == bb, f2 = zz[q] == ajv, f3 = f1 && ajv == bb;
#pragma unroll
                for (int c = 0; c < H; ++c) {
                    if (c >= h) break;
                    float w2 = 0.f;
#pragma unroll
                    for (int o = 0; o < H; ++o) {
                        if (o >= h) break;
                        w2 = fmaf(wc[WQ2][o][c], dz[q][o], w2);
                    }
                    const float x1 = lane_value(e1[c], av), x2 = lane_value(e2[c], av), x3 = lane_value(e3[c], av);
                    float t = fmaf(nfa, w2, lane_value(base[c], av));
                    t += f1 ? x1 : 0.f;
                    t += f2 ? x2 : 0.f;
                    t += f3 ? x3 : 0.f;
                    acc[c] += vz[q] ? t : 0.f;
                }
            }
        }
        if (lane < n)
#pragma unroll
            for (int c = 0; c < H; ++c) {
                if (c >= h) break;
                dout[(o2 + (long long)u * n + lane) * h + c] = acc[c] + rd[c];
            }
    }
    wsync();
}

template <int CF>
__global__ void __launch_bounds__(Q_NT) k_ccn2_small_bwd(QArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    QGraph& g = *reinterpret_cast<QGraph*>(lds);
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    char* wbase = lds + q_al16(sizeof(QGraph)) + (size_t)wv * q_wave_bytes(a.nmax);
    QWave& w = *reinterpret_cast<QWave*>(wbase);
    short* sp = reinterpret_cast<short*>(wbase + q_al16(sizeof(QWave)));
    float* dpL = reinterpret_cast<float*>(wbase + q_al16(sizeof(QWave)) + q_sp_bytes(a.nmax));
    uint32_t bad = 0;
    const int n = q_nodes(a, b, bad);
    (void)q_plan(a, b, n, g);  // the forward reported the batch's validation bits
    const int f = a.f, h = a.h, L = a.L, nf = f + L * h;
    float* G = a.gws + (long long)b * a.gstride;
    float* dA = G + (long long)L * a.r2 * h;
    float* dB = dA + a.r2 * h;
    float* rdp = dB + a.r2 * h;
    float* trd = rdp + a.r1 * h;
    float* g0 = trd + (long long)a.nmax * h;
    // dsum[k] = sum_o dout[b][o] fcw[o][k] (k_ccn_readout_bwd's order)
    const float* dob = a.dout + (long long)b * a.n_out;
    for (int k = threadIdx.x; k < nf; k += Q_NT) {
        float s = 0.f;
        for (int o = 0; o < a.n_out; ++o) s = fmaf(dob[o], a.fcw[o * nf + k], s);
        g.vec[k] = s;
    }
    if (a.bs == 1)  // fc gradients: k_ccn_readout_bwd's wave per output over one graph
        for (int q = wv; q < a.n_out * nf + a.n_out; q += Q_NW) {
            double s = 0.0;
            if (q < a.n_out * nf) {
                const int o = q / nf, k = q % nf;
                if (lane < 1) s += (double)dob[o] * (double)a.feat[k];
            } else if (lane < 1) {
                s += (double)dob[q - a.n_out * nf];
            }
            s = wave_sum_d(s);
            if (lane == 0) {
                if (q < a.n_out * nf) a.gfcw[q] = (float)s;
                else a.gfcb[q - a.n_out * nf] = (float)s;
            }
        }
    __syncthreads();
    float* dcur = dA;
    float* dnext = dB;
    for (int l = L - 1; l >= 0; --l) {
        const int cin = l == 0 ? f : h;
        const int K = 18 * cin, stride = h * K + h;
        float* pl = a.ppart[l];
        const float* Fl = G + (long long)l * a.r2 * h;
        const float* fin = l == 0 ? nullptr : G + (long long)(l - 1) * a.r2 * h;
        const float* dtop = l == L - 1 ? g.vec + f + (L - 1) * h : nullptr;
        if (l == 0) c2_weights<Q_HC, CF>(reinterpret_cast<float(*)[Q_HC][CF]>(g.wc), a.W[l], cin, 0, h);
        else c2_weights<Q_HC, Q_HC>(reinterpret_cast<float(*)[Q_HC][Q_HC]>(g.wc), a.W[l], cin, 0, h);
        __syncthreads();
        for (int i = wv; i < n; i += Q_NW) {
            float* pp = pl + (long long)(g.base + i) * stride;
            if (l == 0) q_node_bwd<CF, 1, true>(a, g, w, sp, dpL, i, dcur, dtop, Fl, fin, cin, rdp, trd, pp, g0);
            else q_node_bwd<Q_HC, 8, false>(a, g, w, sp, dpL, i, dcur, dtop, Fl, fin, cin, rdp, trd, pp, nullptr);
        }
        __syncthreads();
        if (a.bs == 1)  // parameter gradients: k_ccn_param_reduce's order over the graph's nodes
            for (int k = wv; k < stride; k += Q_NW) {
                double s = 0.0;
                if (lane < n) s += (double)pl[(long long)lane * stride + k];
                s = wave_sum_d(s);
                if (lane == 0) {
                    const double z = 0.0, t = ((s + z) + z) + z;
                    if (k < h * K) a.gW[l][k] = (float)t;
                    else a.gB[l][k - h * K] = (float)t;
                }
            }
        if (l > 0) {  // dF_{l-1} (the combined weights in g.wc are this level's: c2_dT_weights' values)
            for (int j = wv; j < n; j += Q_NW)
                q_node_gather(a, g, w, sp, j, dcur, rdp, trd, g.vec + f + (l - 1) * h, dnext);
        } else {  // dX[j] = sum over neighbours i of G_i[a_j] + d_j^2 dsum0 (k_ccn2_dx0)
            for (int j = wv; j < n; j += Q_NW) {
                const int nj = g.deg[j];
                float t[Q_CF];
#pragma unroll
                for (int c = 0; c < Q_CF; ++c) t[c] = 0.f;
                for (int x = lane; x < nj; x += 64) {
                    const int i = g.nbr[j * Q_N + x];
                    const unsigned long long mi = g.bits[i];
                    const int aj = __popcll(mi & ((1ull << j) - 1ull));  // position of j in N(i)
                    const float* gi = g0 + ((long long)g.off1[i] + aj) * cin;
#pragma unroll
                    for (int c = 0; c < Q_CF; ++c)
                        if (c < cin) t[c] += gi[c];
                }
#pragma unroll
                for (int c = 0; c < Q_CF; ++c) {
                    if (c >= cin) break;
                    const float s = wave_sum(t[c]);
                    if (lane == 0) {
                        const float rd = g.vec[c];
                        a.dX[((long long)b * a.nmax + j) * f + c] = s + (float)(nj * nj) * rd;
                    }
                }
            }
        }
        __syncthreads();
        float* t = dcur;
        dcur = dnext;
        dnext = t;
    }
    for (int e = threadIdx.x; e < (a.nmax - n) * f; e += Q_NT) a.dX[((long long)b * a.nmax + n) * f + e] = 0.f;
}

// Batches: the parameter gradients summed over the batch's nodes in k_ccn_param_reduce's order (blocks
// [0, np)), the fc gradients over the graphs in k_ccn_readout_bwd's order (the remaining blocks, a wave each)
__global__ void __launch_bounds__(256) k_ccn2_small_reduce(QArgs a, int np) {
    __shared__ double red[4];
    __shared__ int s_tot;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int h = a.h, f = a.f, L = a.L, nf = f + L * h;
    if ((int)blockIdx.x < np) {
        int k = blockIdx.x, l = 0;
        for (; l < L; ++l) {
            const int K = 18 * (l == 0 ? f : h), st = h * K + h;
            if (k < st) break;
            k -= st;
        }
        const int K = 18 * (l == 0 ? f : h), stride = h * K + h;
        if (threadIdx.x < 64) {  // total nodes of the batch (the packed index range)
            int s = 0;
            for (int q = lane; q < a.bs; q += 64) {
                const long long v = a.n_batch ? a.n_batch[q] : a.nmax;
                s += v < 0 ? 0 : (v > a.nmax ? a.nmax : (int)v);
            }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
            if (lane == 0) s_tot = s;
        }
        __syncthreads();
        const int n = s_tot;
        double s = 0.0;
        for (int i = threadIdx.x; i < n; i += 256) s += (double)a.ppart[l][(long long)i * stride + k];
        s = wave_sum_d(s);
        if (lane == 0) red[wv] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            const double t = red[0] + red[1] + red[2] + red[3];
            if (k < h * K) a.gW[l][k] = (float)t;
            else a.gB[l][k - h * K] = (float)t;
        }
        return;
    }
    const int q = ((int)blockIdx.x - np) * 4 + wv;
    if (q >= a.n_out * nf + a.n_out) return;
    double s = 0.0;
    if (q < a.n_out * nf) {
        const int o = q / nf, k = q % nf;
        for (int b = lane; b < a.bs; b += 64) s += (double)a.dout[b * a.n_out + o] * (double)a.feat[(long long)b * nf + k];
    } else {
        const int o = q - a.n_out * nf;
        for (int b = lane; b < a.bs; b += 64) s += (double)a.dout[b * a.n_out + o];
    }
    s = wave_sum_d(s);
    if (lane == 0) {
        if (q < a.n_out * nf) a.gfcw[q] = (float)s;
        else a.gfcb[q - a.n_out * nf] = (float)s;
    }
}

int q_nf(const hgnn_ccn_config* c) { return c->f_in + c->layers * c->hidden; }
long long q_prow(const hgnn_ccn_config* c, int l) {
    const int K = 18 * (l == 0 ? c->f_in : c->hidden);
    return (long long)c->hidden * K + c->hidden;
}
long long q_gstride(const hgnn_ccn_config* c) {
    const long long n = c->nmax, r1 = n * n, r2 = n * n * n;
    const long long fl = (long long)c->layers * r2 * c->hidden + 2 * r2 * c->hidden + r1 * c->hidden +
                         n * c->hidden + r1 * c->f_in;
    return (fl + 63) / 64 * 64;
}
size_t q_al256(size_t x) { return (x + 255) / 256 * 256; }

// workspace: feat, the per-level partial rows, the graph regions
QArgs q_args(const hgnn_ccn_config* c, const float* X, const float* adj, const int64_t* nb, const float* const* params,
             void* ws) {
    QArgs a{};
    a.adj = adj;
    a.n_batch = nb;
    a.X = X;
    a.bs = c->bs;
    a.nmax = c->nmax;
    a.f = c->f_in;
    a.h = c->hidden;
    a.L = c->layers;
    a.n_out = c->n_out;
    a.r1 = (long long)c->nmax * c->nmax;
    a.r2 = a.r1 * c->nmax;
    a.gstride = q_gstride(c);
    for (int l = 0; l < c->layers; ++l) {
        a.W[l] = params[2 * l];
        a.B[l] = params[2 * l + 1];
    }
    a.fcw = params[2 * c->layers];
    a.fcb = params[2 * c->layers + 1];
    char* p = static_cast<char*>(ws);
    a.feat = reinterpret_cast<float*>(p);
    p += q_al256(4 * (size_t)c->bs * q_nf(c));
    for (int l = 0; l < c->layers; ++l) {
        a.ppart[l] = reinterpret_cast<float*>(p);
        p += q_al256(4 * (size_t)c->bs * c->nmax * q_prow(c, l));
    }
    a.gws = reinterpret_cast<float*>(p);
    return a;
}

template <typename K>
void q_lds_attr(K kernel, bool& done) {
    if (!done) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)Q_LDS_MAX);
        (void)hipGetLastError();  // a refused opt-in shows at the launch, not here
        done = true;
    }
}

}  // namespace

bool ccn2_small_ok(const hgnn_ccn_config* c) {
    return c && c->order == 2 && c->bs > 0 && c->nmax > 0 && c->nmax <= Q_N && c->f_in > 0 && c->f_in <= Q_CF &&
           c->hidden > 0 && c->hidden <= Q_H && c->layers >= 1 && c->layers <= Q_LMAX && c->n_out > 0 &&
           q_nf(c) <= Q_NF && q_lds_bytes(c->nmax) <= Q_LDS_MAX;
}

size_t ccn2_small_workspace_bytes(const hgnn_ccn_config* c) {
    if (!ccn2_small_ok(c)) return 0;
    size_t t = q_al256(4 * (size_t)c->bs * q_nf(c));
    for (int l = 0; l < c->layers; ++l) t += q_al256(4 * (size_t)c->bs * c->nmax * q_prow(c, l));
    return t + 4 * (size_t)c->bs * q_gstride(c);
}

int ccn2_small_forward(const hgnn_ccn_config* c, const float* X, const float* adj, const int64_t* nb,
                       const float* const* params, void* ws, int32_t* err, int32_t tag, float* out, hipStream_t s) {
    QArgs a = q_args(c, X, adj, nb, params, ws);
    a.out = out;
    a.err = err;
    a.tag = tag;
    static bool attr = false;
    q_lds_attr(&k_ccn2_small_fwd<Q_CF>, attr);
    HGNN_KLAUNCH(k_ccn2_small_fwd<Q_CF>, dim3(c->bs), dim3(Q_NT), q_lds_bytes(c->nmax), s, a);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int ccn2_small_backward(const hgnn_ccn_config* c, const float* X, const float* adj, const int64_t* nb,
                        const float* const* params, void* ws, const float* dout, float* const* grads, float* dX,
                        hipStream_t s) {
    QArgs a = q_args(c, X, adj, nb, params, ws);
    a.dout = dout;
    a.dX = dX;
    for (int l = 0; l < c->layers; ++l) {
        a.gW[l] = grads[2 * l];
        a.gB[l] = grads[2 * l + 1];
    }
    a.gfcw = grads[2 * c->layers];
    a.gfcb = grads[2 * c->layers + 1];
    static bool attr = false;
    q_lds_attr(&k_ccn2_small_bwd<Q_CF>, attr);
    HGNN_KLAUNCH(k_ccn2_small_bwd<Q_CF>, dim3(c->bs), dim3(Q_NT), q_lds_bytes(c->nmax), s, a);
    HGNN_LAUNCH_CHECK();
    if (c->bs > 1) {
        int np = 0;
        for (int l = 0; l < c->layers; ++l) np += (int)q_prow(c, l);
        const int nf = q_nf(c);
        HGNN_KLAUNCH(k_ccn2_small_reduce, dim3(np + (c->n_out * nf + c->n_out + 3) / 4), dim3(256), 0, s, a, np);
        HGNN_LAUNCH_CHECK();
    }
    return HGNN_OK;
}

}  // namespace hgnn
