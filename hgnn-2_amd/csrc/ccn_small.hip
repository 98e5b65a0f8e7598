// CCN-1D on small graphs (n <= 64 nodes): one workgroup per graph, the whole call in LDS.
//
// The reference's driver calls the network one graph at a time (scripts/train_ccn.py:31-73: net(X, A + I),
// loss, backward and an optimizer step per graph), and QM9 graphs have at most 29 nodes: there the general
// path (ccn.hip) spends the call on dispatches, not arithmetic (5 plan + 5 forward + 9 backward launches,
// ~0.18 ms of GPU time and more of host time per graph).  Here one workgroup per graph
//   * builds the receptive fields in LDS: row bit sets over the graph's nodes (utils_ccn.py:195-199,
//     nbr_i = ascending nonzero(adj[i])), degrees, row offsets, and reads every chi position by popcount
//     (index of u in N(j) = bits below u in j's row, utils_ccn.py:66-106),
//   * runs every level (promotion + the two contractions + Linear + ReLU, utils_ccn.py:281-324) and the
//     readout (model_ccn.py:50-64) -- forward: one dispatch,
//   * backward: rebuilds the plan and the levels in LDS, then walks them back (one dispatch for one
//     graph; a batch adds one reduction of the per-graph parameter partials).
// Per level the arithmetic is the one-chunk path of k_ccn1_fwd / k_ccn1_bwd_node / k_ccn1_bwd_gather in
// the same order, so forward values and input gradients are those of the general path; the weight
// gradients are summed per lane over a wave's nodes, then over lanes and waves (fp32), where the general
// path sums per node and then over nodes in fp64.
#include <cstdio>
#include <cstdlib>

#include "kernels.h"

namespace hgnn {
namespace {

constexpr int CS_NT = 512, CS_NW = CS_NT / 64;   // 8 waves (~4 nodes of a QM9 graph each; 256 VGPRs a lane)
constexpr int CS_RT = 256;                         // threads of the fp64 readout sums (the general path's order)
constexpr int CS_CF = 8;                              // f_in and hidden bound
constexpr int CS_LMAX = 15;
constexpr int CS_NFMAX = CS_CF + CS_LMAX * CS_CF;     // readout width bound
constexpr int CS_PMAX = CS_CF * 2 * CS_CF + CS_CF;    // one level's weight + bias entries
constexpr int CS_XMAX = 64 * CS_CF;                 // staged node features
constexpr int CS_WMAX = CS_LMAX * CS_PMAX;            // staged level weights and biases
constexpr size_t CS_FIXED = 512 + 256 + 272 + 4096 + 4 * CS_NW * CS_PMAX + 4 * CS_NFMAX + 8 * CS_NW * CS_CF +
                            4 * CS_XMAX + 4 * CS_WMAX;
constexpr size_t CS_LDS_MAX = 150 * 1024;  // dynamic LDS opt-in (the forward also has a static word)

struct CsArgs {
    const float* adj;        // (bs, nmax, nmax) with self loops
    const int64_t* n_batch;  // (bs,) or null: every graph has nmax nodes
    const float* X;          // (bs, nmax, f)
    int bs, nmax, f, h, L, n_out, rcap;  // rcap = nmax^2 bounds sum_i d_i of any graph
    const float* W[CS_LMAX];
    const float* B[CS_LMAX];
    const float* fcw;
    const float* fcb;
    float* feat;             // [bs][nf] readout features (forward writes, backward reads)
    float* out;              // (bs, n_out)
    int* err;                // forward: graphs with validation bits store tag * 256 + bits
    int tag;
    const float* dout;       // backward
    float* ppart;            // backward, bs > 1: [bs][ptot] level weight / bias partials, levels ascending
    float* gW[CS_LMAX];      // backward, bs == 1: gradients written directly
    float* gB[CS_LMAX];
    float* gfcw;
    float* gfcb;
    float* dX;               // (bs, nmax, f), padding rows zeroed
    unsigned long long* prof;  // diagnostic phase stamps of graph 0 (HGNN_CCN_SMALL_PROF), or null
};

// phase stamp k of graph 0 (s_memtime core cycles), diagnostic builds of the timing only
#define CS_STAMP(k)                                                          \
    do {                                                                     \
        if (a.prof && blockIdx.x == 0 && threadIdx.x == 0) a.prof[k] = clock64(); \
    } while (0)

struct CsLds {
    unsigned long long* bits;  // [64] row bit sets
    int* deg;                  // [64]
    int* off1;                 // [65] exclusive prefix of deg
    unsigned char* nbr;        // [64][64] ascending neighbour ids
    float* red;                // [CS_NW][CS_PMAX]
    float* vec;                // [CS_NFMAX] readout features (forward) / dsum (backward)
    double* dred;              // [CS_NW][CS_CF]
    float* Xs;                 // [n][f] the graph's node features
    float* Ws;                 // level l: W_l [h][2 cin] then b_l [h], levels ascending
    float* F;                  // forward: 2 levels (ping-pong); backward: all L levels, [rcap][h] each
    float* dcoll;              // backward: [rcap][2 cmax]
    float* dF0;                // backward: [rcap][h] x 2
    float* dF1;
};

// The level walks read CF channels of a row unconditionally and drop the ones past the row's width by
// selects: up to CF - 1 floats past the last region (F's second ping-pong buffer forward, dF1 backward),
// so the request carries CS_CF floats of padding and every such read stays inside the allocation.
__host__ __device__ inline size_t cs_lds_bytes(int rcap, int f, int h, int L, bool bwd) {
    const int cmax = f > h ? f : h;
    return CS_FIXED + 4 * (size_t)rcap * (bwd ? (size_t)h * L + 2 * cmax + 2 * h : 2 * (size_t)h) + 4 * CS_CF;
}

__device__ inline CsLds cs_carve(char* base, const CsArgs& a, bool bwd) {
    CsLds s;
    size_t o = 0;
    s.bits = reinterpret_cast<unsigned long long*>(base + o);
    o += 512;
    s.deg = reinterpret_cast<int*>(base + o);
    o += 256;
    s.off1 = reinterpret_cast<int*>(base + o);
    o += 272;
    s.nbr = reinterpret_cast<unsigned char*>(base + o);
    o += 4096;
    s.red = reinterpret_cast<float*>(base + o);
    o += 4 * CS_NW * CS_PMAX;
    s.vec = reinterpret_cast<float*>(base + o);
    o += 4 * CS_NFMAX;
    s.dred = reinterpret_cast<double*>(base + o);
    o += 8 * CS_NW * CS_CF;
    s.Xs = reinterpret_cast<float*>(base + o);
    o += 4 * CS_XMAX;
    s.Ws = reinterpret_cast<float*>(base + o);
    o += 4 * CS_WMAX;
    s.F = reinterpret_cast<float*>(base + o);
    o += 4 * (size_t)a.rcap * a.h * (bwd ? a.L : 2);
    s.dcoll = s.dF0 = s.dF1 = nullptr;
    if (bwd) {
        const int cmax = a.f > a.h ? a.f : a.h;
        s.dcoll = reinterpret_cast<float*>(base + o);
        o += 4 * (size_t)a.rcap * 2 * cmax;
        s.dF0 = reinterpret_cast<float*>(base + o);
        o += 4 * (size_t)a.rcap * a.h;
        s.dF1 = reinterpret_cast<float*>(base + o);
    }
    return s;
}

__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v |= (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}

// offset of level l's weights in Ws
__device__ __forceinline__ int cs_woff(int l, int f, int h) {
    return l == 0 ? 0 : (h * 2 * f + h) + (l - 1) * (h * 2 * h + h);
}

// One round of loads for the whole call: the graph's adjacency block (into As, stride n), its node
// features and every level's weights; every later access is to LDS (the dependent global round trips
// of a per-node walk were most of a QM9 graph's time).
__device__ void cs_stage(const CsArgs& a, int b, int n, const CsLds& s, float* As) {
    const float* A = a.adj + (long long)b * a.nmax * a.nmax;
    const float* Xg = a.X + (long long)b * a.nmax * a.f;
    const int na = n * n, nx = n * a.f, nw = cs_woff(a.L, a.f, a.h);
    const int total = na + nx + nw;
    constexpr int U = 4;
    for (int e0 = threadIdx.x; e0 < total; e0 += CS_NT * U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = e0 + u * CS_NT;
            v[u] = 0.f;
            if (e < na) {
                const int r = e / n;
                v[u] = A[(long long)r * a.nmax + (e - r * n)];
            } else if (e < na + nx) {
                v[u] = Xg[e - na];
            } else if (e < total) {
                int p = e - na - nx, l = 0;
                while (l + 1 < a.L && p >= cs_woff(l + 1, a.f, a.h)) ++l;
                const int q = p - cs_woff(l, a.f, a.h), hk = a.h * 2 * (l == 0 ? a.f : a.h);
                v[u] = q < hk ? a.W[l][q] : a.B[l][q - hk];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = e0 + u * CS_NT;
            if (e < na) As[e] = v[u];
            else if (e < na + nx) s.Xs[e - na] = v[u];
            else if (e < total) s.Ws[e - na - nx] = v[u];
        }
    }
    __syncthreads();
}

// Graph b's receptive fields from the staged adjacency: nbr, bits, deg, off1 in LDS.  Returns this lane's
// validation bits (self loop missing, pattern not symmetric -- the general plan's ERR_CCN_SELFLOOP /
// ERR_CCN_ASYM).
__device__ uint32_t cs_plan(int n, const CsLds& s, const float* As) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t bad = 0;
    // row 0's first entry is what an idle lane (past the graph) reads as its neighbour id: defined even
    // for an empty slot (n = 0), so its bits / off1 reads stay inside the arrays
    if (n == 0 && threadIdx.x == 0) s.nbr[0] = 0;
    for (int r = wv; r < n; r += CS_NW) {
        const bool nz = lane < n && As[r * n + lane] > 0.f;  // utils_ccn.py:195 (A > 0)
        const unsigned long long m = __ballot(nz);
        if (nz) s.nbr[r * 64 + __popcll(m & ((1ull << lane) - 1ull))] = (unsigned char)lane;
        if (lane == 0) {
            s.bits[r] = m;
            s.deg[r] = __popcll(m);
        }
        if (!((m >> r) & 1ull)) bad |= ERR_CCN_SELFLOOP;
    }
    __syncthreads();
    if (wv == 0) {
        const int d = lane < n ? s.deg[lane] : 0;
        int x = d;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int t = __shfl_up(x, o, 64);
            if (lane >= o) x += t;
        }
        s.off1[lane] = x - d;
        if (lane == 63) s.off1[64] = x;
        // lanes per node of the level walks: the power of two >= the largest receptive field
        int dm = d;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) dm = max(dm, __shfl_xor(dm, o, 64));
        int g = 1;
        while (g < dm) g <<= 1;
        if (lane == 0) s.off1[66] = g;
    }
    // every neighbour j of r must list r (the backward gathers node j's readers from N(j))
    for (int r = wv; r < n; r += CS_NW) {
        const unsigned long long m = s.bits[r];
        if (lane < n && ((m >> lane) & 1ull) && !((s.bits[lane] >> r) & 1ull)) bad |= ERR_CCN_ASYM;
    }
    __syncthreads();
    return bad;
}

// Level walks pack several nodes into a wave: G lanes per node (G = the power of two >= the graph's largest
// receptive field, off1[66]), lane p of group g serves position / neighbour p of node i = base + wv * 64/G + g
// (-1 past the graph).  A QM9 graph (d <= 5, G = 8) takes 8 nodes per wave: one pass of the 8 waves.
struct CsSlot {
    int i, p;
};
__device__ __forceinline__ CsSlot cs_slot(int base, int G, int n) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int i = base + wv * (64 / G) + lane / G;
    return CsSlot{i < n ? i : -1, lane & (G - 1)};
}

// Node i, lane p < d_i (w = nbr_i[p]):  rs[c] = sum_a T[a][p][c] (p as the position x: w read from N(j_a), a
// ascending) and colv[c] = sum_x T[p][x][c] (p as the neighbour a: every u_x read from N(w), x ascending),
// T[a][x] = F_{j_a}[pos(u_x in N(j_a))] (level 0: X[j_a] when present).  Lane-local loops over the node's
// neighbours -- no cross-lane reduction -- in the order of k_ccn1_fwd's one-chunk path.  Branch-free: the
// four neighbours' ids, their rows and offsets, then every channel of both reads go out as one batch of LDS
// loads each (reads past a row are discarded by the selects; cs_lds_bytes pads the allocation for them).
template <int CF>
__device__ __forceinline__ void cs_collect(const CsLds& s, CsSlot sl, int G, const float* __restrict__ Xg,
                                           const float* Fin, int cin, float (&rs)[CF], float (&colv)[CF]) {
    const int ib = (sl.i >= 0 ? sl.i : 0) * 64;
    const int d = sl.i >= 0 ? s.deg[sl.i] : 0;
    const bool v = sl.p < d;
    const bool lv0 = Fin == nullptr;
    const float* B = lv0 ? Xg : Fin;
    const int wl = s.nbr[ib + (v ? sl.p : 0)];
    const unsigned long long ml = s.bits[wl];
    const unsigned long long bl = (1ull << wl) - 1ull;
    const int ol = s.off1[wl];
    const int dl = d > 0 ? d - 1 : 0;
#pragma unroll
    for (int c = 0; c < CF; ++c) rs[c] = colv[c] = 0.f;
    for (int k0 = 0; k0 < G; k0 += 4) {
        int jk[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) jk[q] = s.nbr[ib + min(k0 + q, dl)];
        unsigned long long mk[4];
        int ok_[4], a1[4], a2[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            mk[q] = s.bits[jk[q]];
            ok_[q] = s.off1[jk[q]];
        }
        bool g1[4], g2[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const bool live = v && k0 + q < d;
            g1[q] = live && ((mk[q] >> wl) & 1ull);
            g2[q] = live && ((ml >> jk[q]) & 1ull);
            a1[q] = lv0 ? jk[q] * cin : (ok_[q] + __popcll(mk[q] & bl)) * cin;
            a2[q] = lv0 ? wl * cin : (ol + __popcll(ml & ((1ull << jk[q]) - 1ull))) * cin;
        }
        float t1[4][CF], t2[4][CF];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int c = 0; c < CF; ++c) {
                t1[q][c] = B[a1[q] + c];
                t2[q][c] = B[a2[q] + c];
            }
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int c = 0; c < CF; ++c) {
                rs[c] += (c < cin && g1[q]) ? t1[q][c] : 0.f;
                colv[c] += (c < cin && g2[q]) ? t2[q][c] : 0.f;
            }
    }
}

// F_l rows of node i: relu(b + W [rs | colv]) in k_ccn1_fwd's order
template <int CF>
__device__ __forceinline__ void cs_update(const CsLds& s, CsSlot sl, const float (&rs)[CF], const float (&colv)[CF],
                                          int cin, const float* __restrict__ W, const float* __restrict__ bias, int h,
                                          float* Fout) {
    if (sl.i < 0 || sl.p >= s.deg[sl.i]) return;
    const int k2 = 2 * cin;
    const int row = s.off1[sl.i] + sl.p;
    for (int o = 0; o < h; ++o) {
        float v = bias[o];
#pragma unroll
        for (int c = 0; c < CF; ++c)
            if (c < cin) v = fmaf(W[o * k2 + c], rs[c], v);
#pragma unroll
        for (int c = 0; c < CF; ++c)
            if (c < cin) v = fmaf(W[o * k2 + cin + c], colv[c], v);
        Fout[row * h + o] = v < 0.f ? 0.f : v;
    }
}

// One level of the forward walk: F_l of every node (CF = the level's channel bound)
template <int CF>
__device__ __forceinline__ void cs_fwd_level(const CsLds& s, int n, int G, const float* Xg, const float* fin, int cin,
                                             const float* Wl, int h, float* fout) {
    for (int base = 0; base < n; base += CS_NW * (64 / G)) {
        const CsSlot sl = cs_slot(base, G, n);
        float rs[CF], colv[CF];
        cs_collect<CF>(s, sl, G, Xg, fin, cin, rs, colv);
        cs_update<CF>(s, sl, rs, colv, cin, Wl, Wl + h * 2 * cin, h, fout);
    }
}

// Readout column sums in fp64 (k_ccn_readout_part's order for a one-chunk graph): vec[col0 + c] =
// sum over rows r of val(r, c), rows over the first 256 threads, then their 4 waves.
template <int CF, typename V>
__device__ __forceinline__ void cs_colsum(const CsLds& s, int rows, int C, int col0, V val) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double acc[CF];
#pragma unroll
    for (int c = 0; c < CF; ++c) acc[c] = 0.0;
    if (threadIdx.x < CS_RT)
        for (int r = threadIdx.x; r < rows; r += CS_RT)
#pragma unroll
            for (int c = 0; c < CF; ++c)
                if (c < C) acc[c] += val(r, c);
#pragma unroll
    for (int c = 0; c < CF; ++c) {
        if (c >= C) break;
        const double t = wave_sum_d(acc[c]);
        if (lane == 0) s.dred[wv * CS_CF + c] = t;
    }
    __syncthreads();
    if ((int)threadIdx.x < C) {
        const int c = threadIdx.x;
        s.vec[col0 + c] = (float)(s.dred[c] + s.dred[CS_CF + c] + s.dred[2 * CS_CF + c] + s.dred[3 * CS_CF + c]);
    }
    __syncthreads();
}

__device__ __forceinline__ int cs_nodes(const CsArgs& a, int b, uint32_t& bad) {
    int n = a.n_batch ? (int)a.n_batch[b] : a.nmax;
    if (n < 0 || n > a.nmax) {
        bad |= ERR_SIZES;
        n = n < 0 ? 0 : a.nmax;
    }
    return n;
}

template <int CF>
__global__ void __launch_bounds__(CS_NT) k_ccn1_small_fwd(CsArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    __shared__ uint32_t sbad;
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const CsLds s = cs_carve(lds, a, false);
    CS_STAMP(0);
    if (threadIdx.x == 0) sbad = 0;
    uint32_t bad = 0;
    const int n = cs_nodes(a, b, bad);
    cs_stage(a, b, n, s, s.F);
    CS_STAMP(1);
    bad |= cs_plan(n, s, s.F);
    CS_STAMP(2);
    const float* Xg = s.Xs;
    const int h = a.h, f = a.f, nf = f + a.L * h;
    const int G = s.off1[66];
    // level 0 of the readout: sum_i d_i X[i]  (utils_ccn.py:212-216 tiles X[i] d_i times)
    cs_colsum<CF>(s, n, f, 0, [&](int r, int c) { return (double)s.deg[r] * (double)Xg[r * f + c]; });
    CS_STAMP(3);
    const int rows = s.off1[n];
    const float* fin = nullptr;
    for (int l = 0; l < a.L; ++l) {
        const int cin = l == 0 ? f : h;
        float* fout = s.F + (size_t)(l & 1) * a.rcap * h;
        const float* Wl = s.Ws + cs_woff(l, f, h);
        if (cin <= 2) cs_fwd_level<2>(s, n, G, Xg, fin, cin, Wl, h, fout);
        else cs_fwd_level<CF>(s, n, G, Xg, fin, cin, Wl, h, fout);
        __syncthreads();
        CS_STAMP(4 + 2 * l);
        cs_colsum<CF>(s, rows, h, f + l * h, [&](int r, int c) { return (double)fout[r * h + c]; });
        CS_STAMP(5 + 2 * l);
        fin = fout;
    }
    for (int k = threadIdx.x; k < nf; k += CS_NT) a.feat[(long long)b * nf + k] = s.vec[k];
    // out = fc(feat) in fp64 (k_ccn_readout's order)
    for (int o = 0; o < a.n_out; ++o) {
        double acc = 0.0;
        if (threadIdx.x < CS_RT)
            for (int k = threadIdx.x; k < nf; k += CS_RT) acc += (double)a.fcw[o * nf + k] * (double)s.vec[k];
        acc = wave_sum_d(acc);
        __syncthreads();
        if (lane == 0) s.dred[wv] = acc;
        __syncthreads();
        if (threadIdx.x == 0)
            a.out[(long long)b * a.n_out + o] = (float)(s.dred[0] + s.dred[1] + s.dred[2] + s.dred[3] + (double)a.fcb[o]);
    }
    CS_STAMP(30);
    bad = wave_or(bad);
    if (lane == 0 && bad) atomicOr(&sbad, bad);
    __syncthreads();
    if (threadIdx.x == 0 && sbad) a.err[0] = a.tag * 256 + (int)sbad;  // vector store (host-mapped word)
    CS_STAMP(31);
}

// One level of the backward walk (node pass, parameter gradients, gather), CF = this level's channel
// bound (levels of hidden <= 2 take CF = 2: a quarter of the loads and selects of the 8-channel form).
template <int CF, int CH>
__device__ void cs_bwd_level(const CsArgs& a, const CsLds& s, int b, int l, int n, int G, const float* Xg,
                             const float* dFc, float* dFn) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    (void)wv;
    const int h = a.h, f = a.f, L = a.L;
    (void)L;
    const int p0 = h * 2 * f + h, p1 = h * 2 * h + h;
    const int cin = l == 0 ? f : h, k2 = 2 * cin;
    const float* W = s.Ws + cs_woff(l, f, h);
    const float* Fl = s.F + (size_t)l * a.rcap * h;
    const float* fin = l == 0 ? nullptr : s.F + (size_t)(l - 1) * a.rcap * h;
    const bool top = l == L - 1;
    const float* dtop = s.vec + f + (L - 1) * h;
    // node pass: dpre = dF relu', per-lane parameter sums, dcoll = W^T dpre (k_ccn1_bwd_node's order)
    float aw[CH][CF], ac[CH][CF], ab[CH];
#pragma unroll
    for (int o = 0; o < CH; ++o) {
        ab[o] = 0.f;
#pragma unroll
        for (int c = 0; c < CF; ++c) aw[o][c] = ac[o][c] = 0.f;
    }
    for (int base = 0; base < n; base += CS_NW * (64 / G)) {
        const CsSlot sl = cs_slot(base, G, n);
        float rs[CF], colv[CF];
        cs_collect<CF>(s, sl, G, Xg, fin, cin, rs, colv);
        const int ii = sl.i >= 0 ? sl.i : 0;
        const bool vx = sl.i >= 0 && sl.p < s.deg[ii];
        const int row = s.off1[ii] + sl.p;
        float dp[CH];
#pragma unroll
        for (int o = 0; o < CH; ++o) {
            const float g = top ? dtop[o] : dFc[row * h + o];  // unconditional LDS reads
            dp[o] = (vx && o < h && Fl[row * h + o] > 0.f) ? g : 0.f;
            ab[o] += dp[o];
#pragma unroll
            for (int c = 0; c < CF; ++c) {
                aw[o][c] = fmaf(dp[o], rs[c], aw[o][c]);
                ac[o][c] = fmaf(dp[o], colv[c], ac[o][c]);
            }
        }
        if (vx)
            for (int k = 0; k < k2; ++k) {
                float t = 0.f;
#pragma unroll
                for (int o = 0; o < CH; ++o)
                    if (o < h) t = fmaf(W[o * k2 + k], dp[o], t);
                s.dcoll[row * k2 + k] = t;
            }
    }
    // level parameter gradients: lanes, then the waves in order
#pragma unroll
    for (int o = 0; o < CH; ++o) {
        if (o >= h) break;
#pragma unroll
        for (int c = 0; c < CF; ++c) {
            if (c >= cin) break;
            const float tw = wave_total(aw[o][c]);
            const float tc = wave_total(ac[o][c]);
            if (lane == 0) {
                s.red[wv * CS_PMAX + o * k2 + c] = tw;
                s.red[wv * CS_PMAX + o * k2 + cin + c] = tc;
            }
        }
        const float tb = wave_total(ab[o]);
        if (lane == 0) s.red[wv * CS_PMAX + h * k2 + o] = tb;
    }
    __syncthreads();
    const int P = h * k2 + h;
    for (int p = threadIdx.x; p < P; p += CS_NT) {
        float v = s.red[p];
#pragma unroll
        for (int w = 1; w < CS_NW; ++w) v += s.red[w * CS_PMAX + p];
        if (a.bs == 1) {
            if (p < h * k2) a.gW[l][p] = v;
            else a.gB[l][p - h * k2] = v;
        } else {
            const int poff = l == 0 ? 0 : p0 + (l - 1) * p1;
            a.ppart[(long long)b * (p0 + (L - 1) * p1) + poff + p] = v;
        }
    }
    // gather: dF_{l-1}[j][u] = sum_{i in N(j)} [q valid] (drow_i[q] + dcol_i[pos of j]) + readout term;
    // level 0: dX[j] = the sum over u + d_j dsum  (k_ccn1_bwd_gather's order)
    for (int base = 0; base < n; base += CS_NW * (64 / G)) {
        const CsSlot sl = cs_slot(base, G, n);
        const int j = sl.i >= 0 ? sl.i : 0;
        const int d = sl.i >= 0 ? s.deg[j] : 0;
        const bool vu = sl.p < d;
        const int uu = s.nbr[j * 64 + (vu ? sl.p : 0)];
        const unsigned long long bu = (1ull << uu) - 1ull, bj = (1ull << j) - 1ull;
        const int dl = d > 0 ? d - 1 : 0;
        float acc[CF];
#pragma unroll
        for (int c = 0; c < CF; ++c) acc[c] = 0.f;
        for (int a0 = 0; a0 < G; a0 += 4) {
            int ik[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) ik[q] = s.nbr[j * 64 + min(a0 + q, dl)];
            unsigned long long m[4];
            int ri[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                m[q] = s.bits[ik[q]];
                ri[q] = s.off1[ik[q]];
            }
            float t1[4][CF], t2[4][CF];
            bool ok[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                ok[q] = vu && ((m[q] >> uu) & 1ull) && a0 + q < d;
                const float* s1 = s.dcoll + (ri[q] + __popcll(m[q] & bu)) * k2;
                const float* s2 = s.dcoll + (ri[q] + __popcll(m[q] & bj)) * k2 + cin;
#pragma unroll
                for (int c = 0; c < CF; ++c) {  // unconditional LDS reads, discarded by the selects
                    t1[q][c] = s1[c];
                    t2[q][c] = s2[c];
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int c = 0; c < CF; ++c)
                    acc[c] += (c < cin && ok[q]) ? t1[q][c] + t2[q][c] : 0.f;
        }
        if (l > 0) {
            if (vu)
#pragma unroll
                for (int c = 0; c < CF; ++c)
                    if (c < cin) dFn[(s.off1[j] + sl.p) * cin + c] = acc[c] + s.vec[f + (l - 1) * h + c];
        } else {
            // the node's G lanes summed by an xor tree: with zeros past d this is wave_total's association
#pragma unroll
            for (int c = 0; c < CF; ++c) {
                if (c >= cin) break;
                float tot = vu ? acc[c] : 0.f;
                for (int o = 1; o < G; o <<= 1) tot += __shfl_xor(tot, o, 64);
                if (sl.i >= 0 && sl.p == 0) a.dX[((long long)b * a.nmax + j) * f + c] = tot + (float)d * s.vec[c];
            }
        }
    }
    __syncthreads();
}

template <int CF, int CH>
__global__ void __launch_bounds__(CS_NT) k_ccn1_small_bwd(CsArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int b = blockIdx.x;
    const CsLds s = cs_carve(lds, a, true);
    uint32_t bad = 0;
    const int n = cs_nodes(a, b, bad);
    cs_stage(a, b, n, s, s.F);
    (void)cs_plan(n, s, s.F);  // the forward reported the batch's validation bits
    const float* Xg = s.Xs;
    const int h = a.h, f = a.f, L = a.L, nf = f + L * h;
    const int G = s.off1[66];
    // the levels again, all kept
    for (int l = 0; l < L; ++l) {
        const int cin = l == 0 ? f : h;
        const float* fin = l == 0 ? nullptr : s.F + (size_t)(l - 1) * a.rcap * h;
        float* fout = s.F + (size_t)l * a.rcap * h;
        const float* Wl = s.Ws + cs_woff(l, f, h);
        if (cin <= 2) cs_fwd_level<2>(s, n, G, Xg, fin, cin, Wl, h, fout);
        else cs_fwd_level<CF>(s, n, G, Xg, fin, cin, Wl, h, fout);
        __syncthreads();
    }
    // dsum[k] = sum_o dout[b][o] fcw[o][k] (k_ccn_readout_bwd's order); one graph: the fc gradients here
    const float* dob = a.dout + (long long)b * a.n_out;
    for (int k = threadIdx.x; k < nf; k += CS_NT) {
        float t = 0.f;
        for (int o = 0; o < a.n_out; ++o) t = fmaf(dob[o], a.fcw[o * nf + k], t);
        s.vec[k] = t;
    }
    if (a.bs == 1)
        for (int w = threadIdx.x; w < a.n_out * nf + a.n_out; w += CS_NT) {
            if (w < a.n_out * nf) a.gfcw[w] = (float)((double)dob[w / nf] * (double)a.feat[w % nf]);
            else a.gfcb[w - a.n_out * nf] = (float)(double)dob[w - a.n_out * nf];
        }
    __syncthreads();
    float* dFc = s.dF0;
    float* dFn = s.dF1;
    for (int l = L - 1; l >= 0; --l) {
        if ((l == 0 ? f : h) <= 2) cs_bwd_level<2, CH>(a, s, b, l, n, G, Xg, dFc, dFn);
        else cs_bwd_level<CF, CH>(a, s, b, l, n, G, Xg, dFc, dFn);
        float* t = dFc;
        dFc = dFn;
        dFn = t;
    }
    for (int e = threadIdx.x; e < (a.nmax - n) * f; e += CS_NT) a.dX[((long long)b * a.nmax + n) * f + e] = 0.f;
}

// Batches: parameter gradient = sum over graphs in fp64, one wave per entry (the level entries, then fc
// weight and bias from dout and the readout features, k_ccn_readout_bwd's order).
__global__ void __launch_bounds__(256) k_ccn1_small_reduce(CsArgs a) {
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int h = a.h, f = a.f, L = a.L, nf = f + L * h;
    const int p0 = h * 2 * f + h, p1 = h * 2 * h + h, ptot = p0 + (L - 1) * p1;
    if (w >= ptot + a.n_out * nf + a.n_out) return;
    double s = 0.0;
    if (w < ptot) {
        for (int b = lane; b < a.bs; b += 64) s += (double)a.ppart[(long long)b * ptot + w];
    } else if (w < ptot + a.n_out * nf) {
        const int o = (w - ptot) / nf, k = (w - ptot) % nf;
        for (int b = lane; b < a.bs; b += 64) s += (double)a.dout[b * a.n_out + o] * (double)a.feat[(long long)b * nf + k];
    } else {
        const int o = w - ptot - a.n_out * nf;
        for (int b = lane; b < a.bs; b += 64) s += (double)a.dout[b * a.n_out + o];
    }
    s = wave_sum_d(s);
    if (lane != 0) return;
    if (w < ptot) {
        const int l = w < p0 ? 0 : 1 + (w - p0) / p1;
        const int p = l == 0 ? w : (w - p0) % p1;
        const int k2 = 2 * (l == 0 ? f : h);
        if (p < h * k2) a.gW[l][p] = (float)s;
        else a.gB[l][p - h * k2] = (float)s;
    } else if (w < ptot + a.n_out * nf) {
        a.gfcw[w - ptot] = (float)s;
    } else {
        a.gfcb[w - ptot - a.n_out * nf] = (float)s;
    }
}

bool cs_ok(const hgnn_ccn_config* c) {
    return c && c->order == 1 && c->bs > 0 && c->nmax > 0 && c->nmax <= 64 && c->f_in > 0 && c->f_in <= CS_CF &&
           c->hidden > 0 && c->hidden <= CS_CF && c->layers >= 1 && c->layers <= CS_LMAX && c->n_out > 0 &&
           cs_lds_bytes(c->nmax * c->nmax, c->f_in, c->hidden, c->layers, true) <= CS_LDS_MAX;
}

size_t cs_ptot(const hgnn_ccn_config* c) {
    const int h = c->hidden, f = c->f_in;
    return (size_t)(h * 2 * f + h) + (size_t)(c->layers - 1) * (h * 2 * h + h);
}

CsArgs cs_args(const hgnn_ccn_config* c, const float* X, const float* adj, const int64_t* nb,
               const float* const* params, void* ws) {
    CsArgs a{};
    a.adj = adj;
    a.n_batch = nb;
    a.X = X;
    a.bs = c->bs;
    a.nmax = c->nmax;
    a.f = c->f_in;
    a.h = c->hidden;
    a.L = c->layers;
    a.n_out = c->n_out;
    a.rcap = c->nmax * c->nmax;
    for (int l = 0; l < c->layers; ++l) {
        a.W[l] = params[2 * l];
        a.B[l] = params[2 * l + 1];
    }
    a.fcw = params[2 * c->layers];
    a.fcb = params[2 * c->layers + 1];
    const int nf = c->f_in + c->layers * c->hidden;
    a.feat = static_cast<float*>(ws);
    a.ppart = reinterpret_cast<float*>(static_cast<char*>(ws) + (4 * (size_t)c->bs * nf + 255) / 256 * 256);
    return a;
}

template <typename K>
void cs_lds_attr(K kernel, bool& done) {
    if (!done) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)CS_LDS_MAX);
        (void)hipGetLastError();  // a refused opt-in shows at the launch, not here
        done = true;
    }
}

}  // namespace
}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_ccn_small_supported(const hgnn_ccn_config* cfg) {
    if (cfg && cfg->order == 2) return ccn2_small_ok(cfg) ? 1 : 0;
    return cs_ok(cfg) ? 1 : 0;
}

int hgnn_host_word_alloc(void** host_ptr, void** dev_ptr) {
    if (!host_ptr || !dev_ptr) return HGNN_ERR_ARG;
    void* h = nullptr;
    HGNN_HOST_CHECK(hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent));
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipHostFree(h);
        return HGNN_ERR_HIP;
    }
    static_cast<int32_t*>(h)[0] = 0;
    *host_ptr = h;
    *dev_ptr = d;
    return HGNN_OK;
}

size_t hgnn_ccn_small_workspace_bytes(const hgnn_ccn_config* cfg) {
    if (cfg && cfg->order == 2) return ccn2_small_workspace_bytes(cfg);
    if (!cs_ok(cfg)) return 0;
    const int nf = cfg->f_in + cfg->layers * cfg->hidden;
    return (4 * (size_t)cfg->bs * nf + 255) / 256 * 256 + (cfg->bs > 1 ? 4 * (size_t)cfg->bs * cs_ptot(cfg) : 0);
}

int hgnn_ccn_small_forward(const hgnn_ccn_config* cfg, const float* d_X, const float* d_adj,
                           const int64_t* d_n_batch, const float* const* params, void* workspace, int32_t* d_err,
                           int32_t tag, float* d_out, void* stream) {
    const bool two = cfg && cfg->order == 2;
    if (two ? !ccn2_small_ok(cfg) : !cs_ok(cfg)) return HGNN_ERR_UNSUPPORTED;
    if (!d_X || !d_adj || !params || !workspace || !d_err || !d_out || tag <= 0 || tag >= (1 << 23))
        return HGNN_ERR_ARG;
    if (two)
        return ccn2_small_forward(cfg, d_X, d_adj, d_n_batch, params, workspace, d_err, tag, d_out,
                                  (hipStream_t)stream);
    CsArgs a = cs_args(cfg, d_X, d_adj, d_n_batch, params, workspace);
    a.out = d_out;
    a.err = d_err;
    a.tag = tag;
    const size_t lds = cs_lds_bytes(a.rcap, a.f, a.h, a.L, false);
    static bool attr = false;
    cs_lds_attr(&k_ccn1_small_fwd<CS_CF>, attr);
    static const bool prof = getenv("HGNN_CCN_SMALL_PROF") != nullptr;
    static unsigned long long* dprof = nullptr;
    if (prof) {
        if (!dprof) HGNN_HOST_CHECK(hipMalloc(&dprof, 32 * 8));
        HGNN_HOST_CHECK(hipMemsetAsync(dprof, 0, 32 * 8, (hipStream_t)stream));
        a.prof = dprof;
    }
    HGNN_KLAUNCH(k_ccn1_small_fwd<CS_CF>, dim3(cfg->bs), dim3(CS_NT), lds, (hipStream_t)stream, a);
    HGNN_LAUNCH_CHECK();
    if (prof) {  // diagnostic: phase cycles of graph 0 (synchronises)
        unsigned long long hp[32];
        HGNN_HOST_CHECK(hipMemcpyAsync(hp, dprof, sizeof(hp), hipMemcpyDeviceToHost, (hipStream_t)stream));
        HGNN_HOST_CHECK(hipStreamSynchronize((hipStream_t)stream));
        fprintf(stderr, "ccn_small_fwd cycles:");
        for (int k = 1; k < 32; ++k)
            if (hp[k]) fprintf(stderr, " %d:%llu", k, hp[k] - hp[0]);
        fprintf(stderr, "\n");
    }
    return HGNN_OK;
}

int hgnn_ccn_small_backward(const hgnn_ccn_config* cfg, const float* d_X, const float* d_adj,
                            const int64_t* d_n_batch, const float* const* params, void* workspace,
                            const float* d_dout, float* const* grads, float* d_dX, void* stream) {
    const bool two = cfg && cfg->order == 2;
    if (two ? !ccn2_small_ok(cfg) : !cs_ok(cfg)) return HGNN_ERR_UNSUPPORTED;
    if (!d_X || !d_adj || !params || !workspace || !d_dout || !grads || !d_dX) return HGNN_ERR_ARG;
    if (two)
        return ccn2_small_backward(cfg, d_X, d_adj, d_n_batch, params, workspace, d_dout, grads, d_dX,
                                   (hipStream_t)stream);
    hipStream_t s = (hipStream_t)stream;
    CsArgs a = cs_args(cfg, d_X, d_adj, d_n_batch, params, workspace);
    a.dout = d_dout;
    a.dX = d_dX;
    for (int l = 0; l < cfg->layers; ++l) {
        a.gW[l] = grads[2 * l];
        a.gB[l] = grads[2 * l + 1];
    }
    a.gfcw = grads[2 * cfg->layers];
    a.gfcb = grads[2 * cfg->layers + 1];
    const size_t lds = cs_lds_bytes(a.rcap, a.f, a.h, a.L, true);
    if (cfg->hidden <= 2) {
        static bool attr = false;
        cs_lds_attr(&k_ccn1_small_bwd<CS_CF, 2>, attr);
        HGNN_KLAUNCH((k_ccn1_small_bwd<CS_CF, 2>), dim3(cfg->bs), dim3(CS_NT), lds, s, a);
    } else {
        static bool attr = false;
        cs_lds_attr(&k_ccn1_small_bwd<CS_CF, CS_CF>, attr);
        HGNN_KLAUNCH((k_ccn1_small_bwd<CS_CF, CS_CF>), dim3(cfg->bs), dim3(CS_NT), lds, s, a);
    }
    HGNN_LAUNCH_CHECK();
    if (cfg->bs > 1) {
        const int nf = cfg->f_in + cfg->layers * cfg->hidden;
        const int outs = (int)cs_ptot(cfg) + cfg->n_out * nf + cfg->n_out;
        HGNN_KLAUNCH(k_ccn1_small_reduce, dim3((outs + 3) / 4), dim3(256), 0, s, a);
        HGNN_LAUNCH_CHECK();
    }
    return HGNN_OK;
}

}  // extern "C"
