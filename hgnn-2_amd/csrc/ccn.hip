// Covariant compositional networks (CCN_1D / CCN_2D) on gfx950.
//
// Reference: models/compnets/model_ccn.py (CCN_1D 18-64, CCN_2D 68-105) over
// functions/utils_ccn.py (receptive fields and chi matrices 66-145, base
// features 148-222, promotions 225-278, updates 281-324) and
// functions/contraction.py (collapse6to3, 106-121).
//
// Index construction (bit-exact with the reference's int semantics):
//   nbr_i = ascending nonzero(adj[i])  (utils_ccn.py:195-199), d_i = |nbr_i| (incl. self loop)
//   pos[i][a][x] = index of nbr_i[x] in nbr_{j_a} or -1, j_a = nbr_i[a]  == the chi_{i j_a}
//   matrices (utils_ccn.py:66-106) as position maps.
// CCN-1D layer, node i (n = d_i):  T[a][x] = F_{j_a}[pos(x)] ;  row[x] = sum_a T, col[a] = sum_x T;
//   F'_i[x] = relu(W [row[x] | col[x]] + b)                        (utils_ccn.py:303-324)
// CCN-2D layer: T[a][b][z] = F_{j_a}[pos(b)][pos(z)] (chi F chi^T), H = T (x) chi_ii = T (x) I, and
//   the 18 contractions of collapse6to3 reduce to (re-derived in DESIGN.md):
//     q0 = n Sc, q1 = q1[x], q2 = n Sa, q3 = q3[x], q4 = d_xy tot, q5 = Sc, q6..14 = n Sc,
//     q15 = T[x][y][y], q16 = T[y][x][y], q17 = d_xy sum_k T[k][k][k]
//   with Sc[a][b] = sum_z T, Sa[b][z] = sum_a T, q1[a] = sum_bz T, q3[b] = sum_az T.
//   O(n^3 C) per node instead of the reference's materialised n^5 C tensor.
// Backward is a gather over the transposed position maps (no atomics): node j collects,
// for every neighbour i, the gradient of the entries of T_i that read F_j.
#include <vector>

#include "ccn2_shared.h"

namespace hgnn {
namespace {

constexpr int CCN_MAXD = 64;     // CCN-2D fast-path degree bound (one wave per receptive-field row, 64-bit ballots)
constexpr int CCN_BIGD = 256;    // CCN-2D degree bound: degrees 65..256 take the _big kernels (rows in 64-lane
                                 // chunks, membership as 4 x 64-bit words, position maps read from L2)
constexpr int CCN_BW = CCN_BIGD / 64;

// bit x of a multi-word set (CCN-2D common neighbourhoods of the large-degree kernels)
__device__ __forceinline__ bool mbit(const unsigned long long* m, int x) { return (m[x >> 6] >> (x & 63)) & 1ull; }
constexpr int CCN1_MAXD = 1024;  // CCN-1D degree bound (rows walked in 64-lane chunks; per-wave LDS row sums)
constexpr int C1F = 8, C1H = 8;  // CCN-1D one-chunk fast path: channels (f_in / hidden) and outputs

struct CcnPlanView {
    const int* node_off;   // (bs + 1)
    const int* deg;        // per node
    const int* nbr;        // per node: slot of nmax global node ids
    const int* selfpos;    // index of i in nbr_i
    const int* graph;      // node -> graph
    const int* off1;       // exclusive prefix of deg      (row offsets of 1D features)
    const int* off2;       // exclusive prefix of deg^2    (row offsets of 2D features, pos maps)
    const int* pos;        // [sum deg^2] position maps
    int nmax;
};

// ------------------------------------------------------------------ plan
// Row r of graph b (wave per row, CCN_NB_ROWS rows per block): the neighbour list (ascending), degree and
// self position, and the row's pattern as a bit set over the graph's local node ids (64-bit words) with
// the exclusive prefix count of each word, from which k_ccn_pos reads positions by popcount.
constexpr int CCN_NB_ROWS = 16;
__global__ void __launch_bounds__(256) k_ccn_nbrs(const float* __restrict__ adj, int nmax, const int* node_off,
                                                  int* deg, int* nbr, int* selfpos, int* graph,
                                                  unsigned long long* bits, int* bcnt, uint32_t* err, int maxd) {
    const int b = blockIdx.x;
    const int n0 = node_off[b];
    const int nb = node_off[b + 1] - n0;
    const int nw = (nmax + 63) >> 6;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float* A = adj + (long long)b * nmax * nmax;
    const int r1 = min(nb, (int)(blockIdx.y + 1) * CCN_NB_ROWS);
    for (int r = blockIdx.y * CCN_NB_ROWS + wv; r < r1; r += 4) {
        const int gi = n0 + r;
        int cnt = 0, sp = -1;
        for (int c0 = 0; c0 < nb; c0 += 64) {
            const int c = c0 + lane;
            const bool nz = c < nb && A[(long long)r * nmax + c] > 0.f;   // utils_ccn.py:195 (A > 0)
            const unsigned long long m = __ballot(nz);
            const int p = __popcll(m & ((1ull << lane) - 1ull));
            if (nz) {
                nbr[(long long)gi * nmax + cnt + p] = n0 + c;
                if (c == r) sp = cnt + p;
            }
            if (lane == 0) {
                bits[(long long)gi * nw + (c0 >> 6)] = m;
                bcnt[(long long)gi * nw + (c0 >> 6)] = cnt;
            }
            cnt += __popcll(m);
        }
        // self position: the lane that saw c == r holds it
        const unsigned long long hs = __ballot(sp >= 0);
        if (lane == 0) {
            deg[gi] = cnt;
            graph[gi] = b;
            if (cnt > maxd) atomicOr(err, (uint32_t)ERR_CCN_DEGREE);
        }
        if (hs == 0ull) {
            if (lane == 0) {
                selfpos[gi] = -1;
                atomicOr(err, (uint32_t)ERR_CCN_SELFLOOP);
            }
        } else if (sp >= 0) {
            selfpos[gi] = sp;
        }
    }
}

// exclusive scans of deg and deg^2 over all nodes (single block of 1024: a serial run of consecutive
// nodes per thread, then a scan of the 1024 run totals); totals[0..1] = the sums, totals[2] = max degree
__global__ void __launch_bounds__(1024) k_ccn_scan(const int* deg, const int* total_nodes, int* off1, int* off2,
                                                   int* totals) {
    __shared__ int s1[1024], s2[1024];
    const int t = threadIdx.x;
    const int n = *total_nodes;
    const int per = (n + 1023) / 1024;
    const int i0 = min(n, t * per), i1 = min(n, i0 + per);
    __shared__ int smax[16];
    int a1 = 0, a2 = 0, dm = 0;
    for (int i = i0; i < i1; ++i) {
        const int d = deg[i];
        a1 += d;
        a2 += d * d;
        dm = max(dm, d);
    }
    s1[t] = a1;
    s2[t] = a2;
    for (int o = 32; o > 0; o >>= 1) dm = max(dm, __shfl_xor(dm, o, 64));
    if ((t & 63) == 0) smax[t >> 6] = dm;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const int b1 = t >= o ? s1[t - o] : 0, b2 = t >= o ? s2[t - o] : 0;
        __syncthreads();
        s1[t] += b1;
        s2[t] += b2;
        __syncthreads();
    }
    int c1 = s1[t] - a1, c2 = s2[t] - a2;
    for (int i = i0; i < i1; ++i) {
        const int d = deg[i];
        off1[i] = c1;
        off2[i] = c2;
        c1 += d;
        c2 += d * d;
    }
    if (t == 1023) {
        off1[n] = s1[1023];
        off2[n] = s2[1023];
        totals[0] = s1[1023];
        totals[1] = s2[1023];
        int m = 0;
        for (int w = 0; w < 16; ++w) m = max(m, smax[w]);
        totals[2] = m;  // largest receptive field
    }
}

// pos[off2[i] + a*d_i + x] = index of nbr_i[x] in nbr_{nbr_i[a]}, or -1: the count of j's neighbours
// below u = nbr_i[x] in j's row bit set (prefix count of u's word + popcount of the bits below u).
// The position of i itself in N(j) must exist for every j in N(i): the gather-form backward walks
// N(j) for the readers of F_j, so the pattern has to be symmetric.
__global__ void __launch_bounds__(256) k_ccn_pos(CcnPlanView v, const int* total_nodes,
                                                 const unsigned long long* __restrict__ bits,
                                                 const int* __restrict__ bcnt, int* pos, long long pos_cap,
                                                 uint32_t* err) {
    const int i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    if (i >= *total_nodes) return;
    // an asynchronous plan sized pos by a bound: a batch beyond it is refused, never overrun
    if ((long long)v.off2[*total_nodes] > pos_cap) {
        if (i == 0 && lane == 0) atomicOr(err, (uint32_t)ERR_SIZES);
        return;
    }
    const int n = v.deg[i];
    if (n > CCN1_MAXD) return;
    const int nw = (v.nmax + 63) >> 6;
    const int n0 = v.node_off[v.graph[i]];
    const int si = v.selfpos[i];
    const int* ni = v.nbr + (long long)i * v.nmax;
    const long long pb = v.off2[i];
    for (int x0 = 0; x0 < n; x0 += 64) {
        const int x = x0 + lane;
        const int u = x < n ? ni[x] - n0 : 0;
        const int uw = u >> 6;
        const unsigned long long below = (1ull << (u & 63)) - 1ull;
        for (int a = 0; a < n; a += 4) {
            unsigned long long w[4];
            int c[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int j = ni[a + q < n ? a + q : a];
                w[q] = bits[(long long)j * nw + uw];
                c[q] = bcnt[(long long)j * nw + uw];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (a + q >= n) break;
                if (x < n) {
                    const bool in = (w[q] >> (u & 63)) & 1ull;
                    const int p = in ? c[q] + __popcll(w[q] & below) : -1;
                    pos[pb + (long long)(a + q) * n + x] = p;
                    if (x == si && p < 0) atomicOr(err, (uint32_t)ERR_CCN_ASYM);
                }
            }
        }
    }
}

// ------------------------------------------------------------------ CCN-1D
// One wave per node; lane x = receptive-field position, in 64-lane chunks for degrees above 64
// (SBM-1000 nodes reach d ~ 200).  Level-0 input is X tiled (utils_ccn.py:212-216): F_0[j][p] = X[j].
// Row sums (over a) accumulate per position in the wave's LDS row, column sums (over x) are wave
// sums of the chunks; for d <= 64 the summation order is the single-chunk one.
__global__ void __launch_bounds__(256) k_ccn1_fwd(CcnPlanView v, const int* total_nodes, const float* __restrict__ fin,
                                                  int level0, const float* __restrict__ X, int cin,
                                                  const float* __restrict__ W, const float* __restrict__ bias, int h,
                                                  float* __restrict__ coll, float* __restrict__ fout) {
    __shared__ float srow[4][CCN1_MAXD];
    const int wv = threadIdx.x >> 6;
    const int i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wv);
    const int lane = threadIdx.x & 63;
    if (i >= *total_nodes) return;
    const int n = v.deg[i];
    if (n > CCN1_MAXD) return;
    const int* ni = v.nbr + (long long)i * v.nmax;
    const int* pi = v.pos + v.off2[i];
    const long long r0 = v.off1[i];
    const int k2 = 2 * cin;
    if (n <= 64 && cin <= C1F) {
        // one chunk, no cross-lane reduction: lane l keeps the row sum of position x = l (a ascending) and
        // the column sum of neighbour a = l (x ascending), four neighbours per round, every channel at once
        const int l = lane;
        const bool vl = l < n;
        const int jl = ni[vl ? l : 0];
        const float* fl = level0 ? X + (long long)jl * cin : fin + (long long)v.off1[jl] * cin;
        float rs[C1F], colv[C1F];
#pragma unroll
        for (int c = 0; c < C1F; ++c) rs[c] = colv[c] = 0.f;
        for (int k0 = 0; k0 < n; k0 += 4) {
            float t1[4][C1F], t2[4][C1F];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int k = min(k0 + q, n - 1);
                const int j = ni[k];
                const int p1 = vl ? pi[(long long)k * n + l] : -1;  // position x = l in N(j_k)
                const int p2 = vl ? pi[(long long)l * n + k] : -1;  // position x = k in N(j_l)
                const bool ok1 = p1 >= 0 && k0 + q < n, ok2 = p2 >= 0 && k0 + q < n;
                const float* s1 = level0 ? X + (long long)j * cin : fin + ((long long)v.off1[j] + max(p1, 0)) * cin;
                const float* s2 = level0 ? fl : fl + (long long)max(p2, 0) * cin;
#pragma unroll
                for (int c = 0; c < C1F; ++c) {
                    t1[q][c] = (c < cin && ok1) ? s1[c] : 0.f;
                    t2[q][c] = (c < cin && ok2) ? s2[c] : 0.f;
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int c = 0; c < C1F; ++c) {
                    rs[c] += t1[q][c];
                    colv[c] += t2[q][c];
                }
        }
        if (vl) {
            const long long row = r0 + l;
#pragma unroll
            for (int c = 0; c < C1F; ++c)
                if (c < cin) {
                    coll[row * k2 + c] = rs[c];
                    coll[row * k2 + cin + c] = colv[c];
                }
            for (int o = 0; o < h; ++o) {
                float s = bias[o];
#pragma unroll
                for (int c = 0; c < C1F; ++c)
                    if (c < cin) s = fmaf(W[o * k2 + c], rs[c], s);
#pragma unroll
                for (int c = 0; c < C1F; ++c)
                    if (c < cin) s = fmaf(W[o * k2 + cin + c], colv[c], s);
                fout[row * h + o] = s < 0.f ? 0.f : s;
            }
        }
        return;
    }
    float* rs = srow[wv];  // wave-private; each position owned by one lane
    for (int c = 0; c < cin; ++c) {
        for (int x = lane; x < n; x += 64) rs[x] = 0.f;
        for (int a = 0; a < n; ++a) {
            const int j = ni[a];
            const long long rj = v.off1[j];
            float cs = 0.f;
            for (int x0 = 0; x0 < n; x0 += 64) {
                const int x = x0 + lane;
                float t = 0.f;
                if (x < n) {
                    const int p = pi[(long long)a * n + x];
                    if (p >= 0) t = level0 ? X[(long long)j * cin + c] : fin[(rj + p) * cin + c];
                    rs[x] += t;
                }
                cs += wave_sum(t);
            }
            if (lane == 0) coll[(r0 + a) * k2 + cin + c] = cs;
        }
        for (int x = lane; x < n; x += 64) coll[(r0 + x) * k2 + c] = rs[x];
    }
    for (int x = lane; x < n; x += 64) {
        const long long row = r0 + x;
        for (int o = 0; o < h; ++o) {
            float s = bias[o];
            for (int k = 0; k < k2; ++k) s = fmaf(W[o * k2 + k], coll[row * k2 + k], s);
            fout[row * h + o] = s < 0.f ? 0.f : s;
        }
    }
}

// dpre = dF * relu'; param partials per node; dcoll = W^T dpre  -> [drow | dcol]
__global__ void __launch_bounds__(256) k_ccn1_bwd_node(CcnPlanView v, const int* total_nodes,
                                                       const float* __restrict__ dF, const float* __restrict__ F,
                                                       const float* __restrict__ coll, int cin,
                                                       const float* __restrict__ W, int h, float* __restrict__ dcoll,
                                                       float* __restrict__ ppart) {
    const int i = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    if (i >= *total_nodes) return;
    int n = v.deg[i];
    if (n > CCN1_MAXD) n = 0;  // flagged by the plan; partials written as zeros
    const int k2 = 2 * cin;
    const long long r0 = v.off1[i];
    float* pp = ppart + (long long)i * (h * k2 + h);
    auto dpre = [&](long long row, int o) { return F[row * h + o] > 0.f ? dF[row * h + o] : 0.f; };
    if (n <= 64 && cin <= C1F && h <= C1H) {  // one chunk: every value of lane x's row loaded once
        const int x = lane;
        const bool vx = x < n;
        const long long row = r0 + x;
        float dp[C1H], cl[2 * C1F];
#pragma unroll
        for (int o = 0; o < C1H; ++o) dp[o] = (vx && o < h) ? dpre(row, o) : 0.f;
#pragma unroll
        for (int k = 0; k < 2 * C1F; ++k) cl[k] = (vx && k < k2) ? coll[row * k2 + k] : 0.f;
#pragma unroll
        for (int o = 0; o < C1H; ++o) {
            if (o >= h) break;
#pragma unroll
            for (int k = 0; k < 2 * C1F; ++k) {
                if (k >= k2) break;
                const float t = wave_total(dp[o] * cl[k]);
                if (lane == 0) pp[o * k2 + k] = t;
            }
            const float sb = wave_total(dp[o]);
            if (lane == 0) pp[h * k2 + o] = sb;
        }
        if (vx)
#pragma unroll
            for (int k = 0; k < 2 * C1F; ++k) {
                if (k >= k2) break;
                float t = 0.f;
#pragma unroll
                for (int o = 0; o < C1H; ++o)
                    if (o < h) t = fmaf(W[o * k2 + k], dp[o], t);
                dcoll[row * k2 + k] = t;
            }
        return;
    }
    for (int o = 0; o < h; ++o) {
        for (int k = 0; k < k2; ++k) {
            float acc = 0.f;
            for (int x = lane; x < n; x += 64) acc += dpre(r0 + x, o) * coll[(r0 + x) * k2 + k];
            const float s = wave_sum(acc);
            if (lane == 0) pp[o * k2 + k] = s;
        }
        float accb = 0.f;
        for (int x = lane; x < n; x += 64) accb += dpre(r0 + x, o);
        const float sb = wave_sum(accb);
        if (lane == 0) pp[h * k2 + o] = sb;
    }
    for (int x = lane; x < n; x += 64) {
        const long long row = r0 + x;
        for (int k = 0; k < k2; ++k) {
            float s = 0.f;
            for (int o = 0; o < h; ++o) s = fmaf(W[o * k2 + k], dpre(row, o), s);
            dcoll[row * k2 + k] = s;
        }
    }
}

// dF_prev[j][u] = sum_{i in N(j)} [q(u) valid] (drow_i[q(u)] + dcol_i[aj]) (+ readout term);
// level 0: dX[j] = sum_u of it + d_j * dsum0
__global__ void __launch_bounds__(256) k_ccn1_bwd_gather(CcnPlanView v, const int* total_nodes,
                                                         const float* __restrict__ dcoll, int cin,
                                                         const float* __restrict__ dsum, int dsum_ld, int dsum_off,
                                                         int level0, float* __restrict__ dout) {
    const int j = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    if (j >= *total_nodes) return;
    const int n = v.deg[j];
    if (n > CCN1_MAXD) return;
    const int* nj = v.nbr + (long long)j * v.nmax;
    const int* pj = v.pos + v.off2[j];
    const int sj = v.selfpos[j];
    const int g = v.graph[j];
    const int k2 = 2 * cin;
    if (n <= 64 && cin <= C1F) {  // one chunk: the indices of a neighbour once for every channel
        const int u = lane;
        const bool vu = u < n;
        float acc[C1F];
#pragma unroll
        for (int c = 0; c < C1F; ++c) acc[c] = 0.f;
        for (int a0 = 0; a0 < n; a0 += 4) {
            float t1[4][C1F], t2[4][C1F];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int a = min(a0 + q, n - 1);
                const int i = nj[a];
                const int aj = pj[(long long)a * n + sj];
                const int qq = vu ? pj[(long long)a * n + u] : -1;
                const bool ok = qq >= 0 && a0 + q < n;
                const long long ri = v.off1[i];
                const float* s1 = dcoll + (ri + max(qq, 0)) * k2;
                const float* s2 = dcoll + (ri + aj) * k2 + cin;
#pragma unroll
                for (int c = 0; c < C1F; ++c) {
                    t1[q][c] = (c < cin && ok) ? s1[c] : 0.f;
                    t2[q][c] = (c < cin && ok) ? s2[c] : 0.f;
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int c = 0; c < C1F; ++c) acc[c] += t1[q][c] + t2[q][c];
        }
#pragma unroll
        for (int c = 0; c < C1F; ++c) {
            if (c >= cin) break;
            const float rd = dsum ? dsum[(long long)g * dsum_ld + dsum_off + c] : 0.f;
            if (level0) {
                const float tot = wave_total(vu ? acc[c] : 0.f);
                if (lane == 0) dout[(long long)j * cin + c] = tot + (float)n * rd;
            } else if (vu) {
                dout[((long long)v.off1[j] + u) * cin + c] = acc[c] + rd;
            }
        }
        return;
    }
    for (int c = 0; c < cin; ++c) {
        const float rd = dsum ? dsum[(long long)g * dsum_ld + dsum_off + c] : 0.f;
        float tot = 0.f;
        for (int u = lane; u < n; u += 64) {
            float acc = 0.f;
            for (int a = 0; a < n; ++a) {
                const int i = nj[a];
                const int q = pj[(long long)a * n + u];
                if (q < 0) continue;
                const int aj = pj[(long long)a * n + sj];
                const long long ri = v.off1[i];
                acc += dcoll[(ri + q) * k2 + c] + dcoll[(ri + aj) * k2 + cin + c];
            }
            if (level0) tot += acc;
            else dout[((long long)v.off1[j] + u) * cin + c] = acc + rd;
        }
        if (level0) {
            const float s = wave_sum(tot);
            if (lane == 0) dout[(long long)j * cin + c] = s + (float)n * rd;
        }
    }
}

// ------------------------------------------------------------------ CCN-2D
struct C2Save {
    float* Sc;   // [sum d^2][C]  Sc[a][b]
    float* Sa;   // [sum d^2][C]  Sa[b][z]
    float* D1;   // [sum d^2][C]  T[a][b][b]
    float* D2;   // [sum d^2][C]  T[a][b][a]
    float* q1;   // [sum d][C]
    float* q3;   // [sum d][C]
    float* tot;  // [nodes][C]
    float* d3;   // [nodes][C]
};

constexpr int C2_CMAX = 8;  // channels of a CCN-2D level (f_in or hidden) handled per pass (narrow kernels)
constexpr int C2_HMAX = 8;  // hidden size bound of the fused output stage (narrow kernels)
constexpr int C2_CMAX_WIDE = 16;  // the wide instantiations: f_in, hidden <= 16
constexpr int C2_HMAX_WIDE = 16;

// CCN-2D layer, receptive fields of degree <= 64 (SBM-200: d ~ 20-60; QM9: d <= 6).
//
// Block per node i (n = d_i), one wave per receptive-field row b.  The wave walks the neighbours a
// with b in C_a (C_a = {x : p_a(x) >= 0}, the common neighbourhood N(i) n N(j_a), ascending) and
// loads the row segment t[z] = T[a][b][z] = F_{j_a}[p_a(b)][p_a(z)] (lane z, z in C_a: one
// coalesced piece of a row of F_{j_a}).  Every contraction statistic comes from that one load:
//   Sa[b][z] += t                         lane z; the wave owns row b of Sa
//   Sc[a][b]  = sum_z t                   wave total (DPP)           -> entry (a, b)
//   D1[a][b]  = t[b]                      lane b's value             -> entry (a, b)
//   D2[a][b]  = t[a]                      lane a's value (a in C_a)  -> entry (b, a), lane a here
//   q1[a]    += Sc[a][b] (W1-projected, per-wave LDS partials), d3 = sum_b t[b] at a == b
// The Linear of the 18 blocks (q0 = n Sc, q1, q2 = n Sa, q3, q4 = [x=y] tot, q5 = Sc,
// q6..14 = n Sc, q15 = D1, q16 = D2^T, q17 = [x=y] d3) is applied with combined weights
// (A = W0 + W6 + ... + W14: alpha = n A + W5 multiplies Sc) and assembled in LDS:
//   pre[x][y] = P[x][y] + W1 q1[x] + W3 q3[x] + [x = y](W4 tot + W17 d3) + bias,
// where P[x][y] receives at most two additions onto zero -- the row wave's part (n W2 Sa + W16 D2^T)
// and the column wave's (alpha Sc + W15 D1) -- so its value does not depend on their order.
// Nothing but F_out is written: the backward (k_c2_bwd) recomputes these sums instead of reading
// saved n^2 C arrays.  Level 0 (F_0[j] = X[j] tiled, utils_ccn.py:167-172): t = X[j_a] on C_a,
// Sc = m_a X[j_a], D1 = X[j_a], no gather and no reduction.
// Output channels are processed HC at a time (one pass each; h = 2 -- the reference's default --
// is one pass).  Dynamic LDS: P [ncap^2][HC] floats, then the position map [ncap^2] int16.
constexpr int C2_NCAP = 64;
size_t c2_dyn_lds(int ncap, int hc_max) { return (size_t)ncap * ncap * (4 * hc_max + 2); }

// node i's position maps into LDS as int16, all loads of a thread in flight before the stores
__device__ __forceinline__ void c2_copy_pos(const int* __restrict__ pos, int nn, short* sp) {
    for (int e0 = threadIdx.x; e0 < nn; e0 += 256 * 8) {
        int t[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) t[k] = e0 + k * 256 < nn ? pos[e0 + k * 256] : 0;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (e0 + k * 256 < nn) sp[e0 + k * 256] = (short)t[k];
    }
}

// node prologue shared by k_c2_fwd / k_c2_bwd: position map (int16) and neighbour data in LDS,
// then the common-neighbourhood masks
template <int CM>
__device__ __forceinline__ void c2_prologue(const CcnPlanView& v, int i, int n, int level0, const float* __restrict__ X,
                                            int cin, short* sp, unsigned long long* vmask, int* s_oj, int* s_dj,
                                            float (*s_x)[CM]) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int* ni = v.nbr + (long long)i * v.nmax;
    const long long o2 = v.off2[i];
    c2_copy_pos(v.pos + o2, n * n, sp);
    if ((int)threadIdx.x < n) {
        const int j = ni[threadIdx.x];
        s_oj[threadIdx.x] = v.off2[j];
        s_dj[threadIdx.x] = v.deg[j];
#pragma unroll
        for (int c = 0; c < CM; ++c) s_x[threadIdx.x][c] = (level0 && c < cin) ? X[(long long)j * cin + c] : 0.f;
    }
    __syncthreads();
    for (int a = wv; a < n; a += 4) {
        const unsigned long long m = __ballot(lane < n && sp[a * n + lane] >= 0);
        if (lane == 0) vmask[a] = m;
    }
    __syncthreads();
}

template <int CM, int HC, int NB, bool L0>
__global__ void __launch_bounds__(256) k_c2_fwd(CcnPlanView v, const int* total_nodes, const float* __restrict__ fin,
                                                const float* __restrict__ X, int cin, const float* __restrict__ W,
                                                const float* __restrict__ bias, int h, int ncap,
                                                float* __restrict__ fout, float* __restrict__ nsum) {
    extern __shared__ float c2_dyn[];
    __shared__ unsigned long long vmask[C2_NCAP];
    __shared__ int s_oj[C2_NCAP], s_dj[C2_NCAP];
    __shared__ float s_x[C2_NCAP][CM];
    __shared__ float wc[NWC][HC][CM];
    __shared__ float qw[4][C2_NCAP][HC];  // per-wave sums of W1 Sc[a][b] over the wave's rows b (W1 q1[a])
    __shared__ float q3p[C2_NCAP][HC];    // W3 q3[b]
    __shared__ float q3s[C2_NCAP][CM];    // q3[b] (tot = sum_b q3[b])
    __shared__ float d3s[C2_NCAP][CM];    // T[b][b][b]
    __shared__ float s_diag[HC];
    __shared__ float s_ns[4][HC];
    const int i = blockIdx.x;
    if (i >= *total_nodes) return;
    const int n = v.deg[i];
    if (n > C2_NCAP || n > ncap || cin > CM) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float* P = c2_dyn;
    short* sp = reinterpret_cast<short*>(c2_dyn + ncap * ncap * HC);
    c2_prologue<CM>(v, i, n, L0 ? 1 : 0, X, cin, sp, vmask, s_oj, s_dj, s_x);
    const long long o2 = v.off2[i];
    const float nf = (float)n;
    // lane a holds neighbour a's mask, row offset and degree (read by the walks with readlane)
    const bool la = lane < n;
    const unsigned long long my_mask = la ? vmask[lane] : 0ull;
    const int my_oj = la ? s_oj[lane] : 0, my_dj = la ? s_dj[lane] : 0;
    for (int o0 = 0; o0 < h; o0 += HC) {
        const int hc = min(HC, h - o0);
        c2_weights<HC, CM>(wc, W, cin, o0, hc);
        for (int e = threadIdx.x; e < n * n * HC; e += 256) P[e] = 0.f;
        __syncthreads();
        float vacc[HC];  // lane a: sum over this wave's rows b of W1 Sc[a][b]
#pragma unroll
        for (int o = 0; o < HC; ++o) vacc[o] = 0.f;
        if constexpr (L0) {
            // T = X[j_a] on C_a x C_a: every block of the Linear is a per-neighbour vector (lane a)
            //   Sc[a][b] = m_a X_a, D1[a][b] = X_a, D2[a][b] = [a in C_a] X_a (b in C_a),
            //   Sa[b][z] = sum_{a: b,z in C_a} X_a, q1[a] = m_a^2 X_a, q3[b] = sum_{a: b in C_a} m_a X_a,
            //   tot = sum_a m_a^2 X_a, d3 = sum_a [a in C_a] X_a
            const float mf = (float)__popcll(my_mask);
            const bool va = la && ((my_mask >> lane) & 1ull);
            float u[HC], dl[HC], bx[HC], q3a[HC];
#pragma unroll
            for (int o = 0; o < HC; ++o) {
                u[o] = dl[o] = bx[o] = q3a[o] = 0.f;
#pragma unroll
                for (int c = 0; c < CM; ++c) {
                    if (c >= cin) break;
                    const float x = la ? s_x[lane][c] : 0.f;
                    u[o] = fmaf(fmaf(fmaf(nf, wc[WA][o][c], wc[WB][o][c]), mf, wc[WQ15][o][c]), x, u[o]);
                    dl[o] = fmaf(wc[WQ16][o][c], x, dl[o]);
                    bx[o] = fmaf(nf * wc[WQ2][o][c], x, bx[o]);
                    vacc[o] = fmaf(wc[WQ1][o][c], x, vacc[o]);
                    q3a[o] = fmaf(wc[WQ3][o][c], x, q3a[o]);
                }
                dl[o] = va ? dl[o] : 0.f;
                vacc[o] *= mf * mf;  // W1 q1[a]
                q3a[o] *= mf;
            }
            if (wv == 0) {
                float dg[HC];
#pragma unroll
                for (int o = 0; o < HC; ++o) dg[o] = 0.f;
#pragma unroll
                for (int c = 0; c < CM; ++c) {
                    if (c >= cin) break;
                    const float x = la ? s_x[lane][c] : 0.f;
                    const float tt = wave_total(mf * mf * x), dd = wave_total(va ? x : 0.f);
#pragma unroll
                    for (int o = 0; o < HC; ++o) dg[o] = fmaf(wc[WQ4][o][c], tt, fmaf(wc[WQ17][o][c], dd, dg[o]));
                }
                if (lane < HC) {
#pragma unroll
                    for (int o = 0; o < HC; ++o)
                        if (lane == o) s_diag[o] = dg[o];
                }
            }
            for (int b = wv; b < n; b += 4) {
                const unsigned long long ab = __ballot(la && ((my_mask >> b) & 1ull));  // a with b in C_a
                const bool in = (ab >> lane) & 1ull;
                float s[HC];
#pragma unroll
                for (int o = 0; o < HC; ++o) {
                    if (in && o < hc) atomicAdd(&P[(lane * n + b) * HC + o], u[o]);  // entry (a, b): alpha Sc + W15 D1
                    s[o] = in ? dl[o] : 0.f;                                            // entry (b, a): W16 D2[a][b]
                    const float q = wave_total(in ? q3a[o] : 0.f);
                    if (lane == 0) q3p[b][o] = q;
                }
                unsigned long long as = ab;
                while (as) {
                    const int a = __ffsll((long long)as) - 1;
                    as &= as - 1ull;
                    const bool vz = (lane_value_u64(my_mask, a) >> lane) & 1ull;
#pragma unroll
                    for (int o = 0; o < HC; ++o) {
                        const float bxa = lane_value(bx[o], a);  // readlane outside any lane-dependent branch
                        s[o] += vz ? bxa : 0.f;                  // n W2 Sa[b][z]
                    }
                }
                if (la)
#pragma unroll
                    for (int o = 0; o < HC; ++o)
                        if (o < hc) atomicAdd(&P[(b * n + lane) * HC + o], s[o]);
            }
            if (wv != 0)
#pragma unroll
                for (int o = 0; o < HC; ++o) vacc[o] = 0.f;  // W1 q1[a] once (wave 0's copy)
        } else {
            for (int b = wv; b < n; b += 4) {
                // lane a (a in A_b) keeps Sc[a][b], D1[a][b] = T[a][b][b] and D2[a][b] = T[a][b][a]; the
                // projections through the weights follow once per row
                float sa[CM], sck[CM], d1k[CM], d2k[CM];
#pragma unroll
                for (int c = 0; c < CM; ++c) sa[c] = sck[c] = d1k[c] = d2k[c] = 0.f;
                if (lane == 0)
#pragma unroll
                    for (int c = 0; c < CM; ++c) d3s[b][c] = 0.f;
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
                        const int a = aa[u];
                        if (a < 0) break;
                        const bool me = lane == a;
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
                        if (a == b && lane == b)
#pragma unroll
                            for (int c = 0; c < CM; ++c) d3s[b][c] = t[u][c];
                    }
                }
                // row b done: the column part of P[a][b] (lanes a in A_b), the row part of P[b][z], q3[b]
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
                        S = fmaf(wc[WQ16][o][c], d2k[c], S);  // entry (b, a): W16 D2[a][b], lane a
                    }
                    if (in) atomicAdd(&P[(lane * n + b) * HC + o], U);  // entry (a, b): alpha Sc + W15 D1
                    vacc[o] += in ? V : 0.f;                            // q1[a]
                    if (la) atomicAdd(&P[(b * n + lane) * HC + o], S);
                    if (lane == 0) {
                        float q = 0.f;
#pragma unroll
                        for (int c = 0; c < CM; ++c) q = fmaf(wc[WQ3][o][c], q3[c], q);
                        q3p[b][o] = q;
                    }
                }
                if (lane == 0)
#pragma unroll
                    for (int c = 0; c < CM; ++c) q3s[b][c] = q3[c];
            }
            __syncthreads();
            if ((int)threadIdx.x < hc) {  // [x = y](W4 tot + W17 d3), sums over b in a fixed order
                const int o = threadIdx.x;
                float dg = 0.f;
                for (int c = 0; c < cin; ++c) {
                    float tt = 0.f, dd = 0.f;
                    for (int b = 0; b < n; ++b) {
                        tt += q3s[b][c];
                        dd += d3s[b][c];
                    }
                    dg = fmaf(wc[WQ4][o][c], tt, dg);
                    dg = fmaf(wc[WQ17][o][c], dd, dg);
                }
                s_diag[o] = dg;
            }
        }
        if (la)
#pragma unroll
            for (int o = 0; o < HC; ++o) qw[wv][lane][o] = vacc[o];
        __syncthreads();
        float ns[HC];  // this node's sum of F_out (the readout's per-level feature, model_ccn.py:102)
#pragma unroll
        for (int o = 0; o < HC; ++o) ns[o] = 0.f;
        for (int e = threadIdx.x; e < n * n; e += 256) {
            const int x = e / n, y = e - x * n;
#pragma unroll
            for (int o = 0; o < HC; ++o) {
                if (o >= hc) break;
                float s = bias[o0 + o] + P[e * HC + o];
                s += (qw[0][x][o] + qw[1][x][o]) + (qw[2][x][o] + qw[3][x][o]);
                s += q3p[x][o];
                if (x == y) s += s_diag[o];
                s = s < 0.f ? 0.f : s;
                fout[(o2 + e) * h + o0 + o] = s;
                ns[o] += s;
            }
        }
#pragma unroll
        for (int o = 0; o < HC; ++o) {
            const float t = wave_total(ns[o]);
            if (lane == 0) s_ns[wv][o] = t;
        }
        __syncthreads();
        if ((int)threadIdx.x < hc)
            nsum[(long long)i * h + o0 + threadIdx.x] =
                (s_ns[0][threadIdx.x] + s_ns[1][threadIdx.x]) + (s_ns[2][threadIdx.x] + s_ns[3][threadIdx.x]);
        __syncthreads();
    }
}

struct C2Grad {
    float* dSc;  // [sum d^2][C]  (dSc + dq1 folded)
    float* dSa;  // [sum d^2][C]  (dSa + dq3 + dtot folded)
    float* dD1;  // [sum d^2][C]
    float* dD2;  // [sum d^2][C]  indexed [a][b]
    float* dd3;  // [nodes][C]
};

// Backward node pass of the degrees 65..256 (their forward: k_ccn2_fwd_big, which saves the
// contraction statistics C2Save): parameter partials from the saved statistics, the gradient
// matrices of the contraction blocks (C2Grad, this node only) and, at level 0, the per-neighbour
// sums G[a] for k_ccn2_dx0; the dp format for the gather kernels follows in k_c2_dp_big.
// One sweep over the n^2 entries per output o for the parameter partials (the 9 distinct
// contraction blocks x cin accumulate in registers, then one wave-sum + LDS combine each), and one
// sweep for the input-side gradients (every channel of an entry from one read of dpre); the level-0
// reduction walks 64-lane chunks and multi-word common-neighbour sets.
template <int CM, int HM>
__global__ void __launch_bounds__(256) k_ccn2_bwd_node_big(CcnPlanView v, const int* total_nodes,
                                                       const float* __restrict__ dF, const float* __restrict__ F,
                                                       C2Save sv, int cin, const float* __restrict__ W, int h,
                                                       C2Grad gd, float* __restrict__ ppart,
                                                       float* __restrict__ g0) {
    constexpr int MAXN = CCN_BIGD;
    __shared__ float sdq1[MAXN * CM], sdq3[MAXN * CM], sdtot[CM], sdd3[CM];
    __shared__ float red[4][10 * CM];
    __shared__ float sw[HM * 18 * CM];
    const int i = blockIdx.x;
    if (i >= *total_nodes) return;
    const int n = v.deg[i];
    if (n <= CCN_MAXD || n > CCN_BIGD || cin > CM || h > HM) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long o2 = v.off2[i], o1 = v.off1[i];
    const float nf = (float)n;
    const int K = 18 * cin;
    float* pp = ppart + (long long)i * (h * K + h);
    for (int t = threadIdx.x; t < h * K; t += 256) sw[t] = W[t];
    for (int t = threadIdx.x; t < n * CM; t += 256) sdq1[t] = sdq3[t] = 0.f;
    if (threadIdx.x < cin) sdtot[threadIdx.x] = sdd3[threadIdx.x] = 0.f;
    // parameter partials: dW[o][q*C + c] = sum_xy dpre[x][y][o] * block_q[x][y][c]
    // distinct blocks: 0 (n Sc; also 6..14), 1 q1, 2 n Sa, 3 q3, 4 tot (diag), 5 Sc, 15 D1, 16 D2^T, 17 d3 (diag)
    for (int o = 0; o < h; ++o) {
        float acc[9][CM];
        float sb = 0.f;
#pragma unroll
        for (int q = 0; q < 9; ++q)
#pragma unroll
            for (int c = 0; c < CM; ++c) acc[q][c] = 0.f;
        for (int e = threadIdx.x; e < n * n; e += 256) {
            const int x = e / n, y = e % n;
            const long long r = o2 + e;
            const float dp = F[r * h + o] > 0.f ? dF[r * h + o] : 0.f;
            sb += dp;
#pragma unroll
            for (int c = 0; c < CM; ++c) {
                if (c >= cin) break;
                const float sc = sv.Sc[r * cin + c];
                acc[0][c] = fmaf(dp, nf * sc, acc[0][c]);
                acc[1][c] = fmaf(dp, sv.q1[(o1 + x) * cin + c], acc[1][c]);
                acc[2][c] = fmaf(dp, nf * sv.Sa[r * cin + c], acc[2][c]);
                acc[3][c] = fmaf(dp, sv.q3[(o1 + x) * cin + c], acc[3][c]);
                if (x == y) {
                    acc[4][c] = fmaf(dp, sv.tot[(long long)i * cin + c], acc[4][c]);
                    acc[8][c] = fmaf(dp, sv.d3[(long long)i * cin + c], acc[8][c]);
                }
                acc[5][c] = fmaf(dp, sc, acc[5][c]);
                acc[6][c] = fmaf(dp, sv.D1[r * cin + c], acc[6][c]);
                acc[7][c] = fmaf(dp, sv.D2[(o2 + y * n + x) * cin + c], acc[7][c]);
            }
        }
#pragma unroll
        for (int q = 0; q < 9; ++q)
#pragma unroll
            for (int c = 0; c < CM; ++c) {
                if (c >= cin) break;
                const float t = wave_sum(acc[q][c]);
                if (lane == 0) red[wv][q * CM + c] = t;
            }
        sb = wave_sum(sb);
        if (lane == 0) red[wv][9 * CM] = sb;
        __syncthreads();
        for (int t = threadIdx.x; t < 18 * cin; t += 256) {
            const int q = t / cin, c = t % cin;
            const int d = q < 6 ? q : (q < 15 ? 0 : q - 9);  // distinct-block index of q
            pp[o * K + q * cin + c] = red[0][d * CM + c] + red[1][d * CM + c] + red[2][d * CM + c] +
                                      red[3][d * CM + c];
        }
        if (threadIdx.x == 0) pp[h * K + o] = red[0][9 * CM] + red[1][9 * CM] + red[2][9 * CM] +
                                              red[3][9 * CM];
        __syncthreads();
    }
    // input-side gradients of the contraction blocks: g_q = W_q^T dpre
    for (int e = threadIdx.x; e < n * n; e += 256) {
        const int x = e / n, y = e % n;
        const long long r = o2 + e;
        float dp[HM];
#pragma unroll
        for (int o = 0; o < HM; ++o) dp[o] = (o < h && F[r * h + o] > 0.f) ? dF[r * h + o] : 0.f;
        for (int c = 0; c < cin; ++c) {
            float g[18];
#pragma unroll
            for (int q = 0; q < 18; ++q) g[q] = 0.f;
#pragma unroll
            for (int o = 0; o < HM; ++o) {
                if (o >= h) break;
                const float* w = sw + o * K;
#pragma unroll
                for (int q = 0; q < 18; ++q) g[q] = fmaf(w[q * cin + c], dp[o], g[q]);
            }
            float s9 = 0.f;
#pragma unroll
            for (int q = 6; q < 15; ++q) s9 += g[q];
            gd.dSc[r * cin + c] = nf * (g[0] + s9) + g[5];
            gd.dSa[r * cin + c] = nf * g[2];
            gd.dD1[r * cin + c] = g[15];
            gd.dD2[(o2 + y * n + x) * cin + c] = g[16];
            atomicAdd(&sdq1[x * CM + c], g[1]);
            atomicAdd(&sdq3[x * CM + c], g[3]);
            if (x == y) {
                atomicAdd(&sdtot[c], g[4]);
                atomicAdd(&sdd3[c], g[17]);
            }
        }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < n * n; e += 256) {
        const int a = e / n;
        const long long r = o2 + e;
        for (int c = 0; c < cin; ++c) {
            gd.dSc[r * cin + c] += sdq1[a * CM + c];                 // q1[a] = sum_b Sc[a][b]
            gd.dSa[r * cin + c] += sdq3[a * CM + c] + sdtot[c];      // q3[b] = sum_z Sa[b][z]; tot: every entry
        }
    }
    if (threadIdx.x < cin) gd.dd3[(long long)i * cin + threadIdx.x] = sdd3[threadIdx.x];
    if (!g0) return;
    // Level 0 (F_0[j] = X[j] tiled): dX[j] needs only the sum of dT_i[a_j][b][z] over the valid (b, z),
    // so node i reduces its own gradient matrices per neighbour a (coalesced, L2-hot) instead of
    // every j gathering them:  G[a] = m_a sum_{b in C_a} dSc[a][b] + sum_{b,z in C_a} dSa[b][z]
    //   + sum_{b in C_a} dD1[a][b] + [a in C_a] (sum_{b in C_a} dD2[a][b] + dd3),  C_a = {x: pos_a(x) >= 0}
    // dSa of one channel is staged in LDS so the masked row sums read LDS, not scattered HBM rows
    __shared__ unsigned long long vmb[CCN_BIGD][CCN_BW];
    __shared__ int smc[CCN_BIGD];
    const int nw = (n + 63) >> 6;
    __syncthreads();
    for (int a = wv; a < n; a += 4) {
        int cnt = 0;
        for (int w = 0; w < nw; ++w) {
            const int x = w * 64 + lane;
            const unsigned long long m = __ballot(x < n && v.pos[o2 + (long long)a * n + x] >= 0);
            if (lane == 0) vmb[a][w] = m;
            cnt += __popcll(m);
        }
        if (lane == 0) smc[a] = cnt;
    }
    __syncthreads();
    for (int c = 0; c < cin; ++c)
        for (int a = wv; a < n; a += 4) {
            const bool va = mbit(vmb[a], a);
            const float mf = (float)smc[a];
            float t = 0.f;
            for (int b = lane; b < n; b += 64) {
                if (!mbit(vmb[a], b)) continue;
                const long long rab = (o2 + (long long)a * n + b) * cin + c;
                t += mf * gd.dSc[rab] + gd.dD1[rab] + (va ? gd.dD2[rab] : 0.f);
                for (int w = 0; w < nw; ++w) {
                    unsigned long long zs = vmb[a][w];
                    while (zs) {
                        const int z = w * 64 + __ffsll((long long)zs) - 1;
                        zs &= zs - 1ull;
                        t += gd.dSa[(o2 + (long long)b * n + z) * cin + c];
                    }
                }
            }
            t = wave_sum(t);
            if (lane == 0) g0[(o1 + a) * cin + c] = t + (va ? sdd3[c] : 0.f);
        }
}

// dX[j] (level 0) = sum over neighbours i of G_i[a_j] (k_ccn2_bwd_node) + d_j^2 dsum0.
__global__ void __launch_bounds__(256) k_ccn2_dx0(CcnPlanView v, const int* total_nodes, const float* __restrict__ g0,
                                                  int cin, const float* __restrict__ dsum, int dsum_ld,
                                                  float* __restrict__ dout) {
    const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (j >= *total_nodes) return;
    const int n = v.deg[j];
    if (n > CCN_BIGD) return;
    const long long o2 = v.off2[j];
    const int* nj = v.nbr + (long long)j * v.nmax;
    const int sj = v.selfpos[j];
    const int g = v.graph[j];
    float t[C2_CMAX_WIDE];
#pragma unroll
    for (int c = 0; c < C2_CMAX_WIDE; ++c) t[c] = 0.f;
    for (int x = lane; x < n; x += 64) {  // one chunk for d <= 64; the indices once for every channel
        const int i = nj[x];
        const int aj = v.pos[o2 + (long long)x * n + sj];  // position of j in N(i)
        const float* gi = g0 + ((long long)v.off1[i] + aj) * cin;
#pragma unroll
        for (int c = 0; c < C2_CMAX_WIDE; ++c)
            if (c < cin) t[c] += gi[c];
    }
#pragma unroll
    for (int c = 0; c < C2_CMAX_WIDE; ++c) {
        if (c >= cin) break;
        const float s = wave_sum(t[c]);
        if (lane == 0) {
            const float rd = dsum ? dsum[(long long)g * dsum_ld + c] : 0.f;
            dout[(long long)j * cin + c] = s + (float)(n * n) * rd;
        }
    }
}

// Backward of one CCN-2D level for the nodes of degree <= 64, block per node i:
//   dp = dF * relu'(F_out) (written back in place of dF; dF of the top level read straight from the readout's
//   per-graph slice dtop when given), rdp[x] = sum_y dp[x][y], tr = sum_x dp[x][x]
//   -- the "dp format" the gather kernels rebuild dT from (k_c2_gather);
//   parameter partials  dW_q[o][c] = sum_xy dp[x][y][o] block_q[x][y][c], db[o] = sum dp, with
//     P0 = sum dp Sc, P1 = sum_x rdp[x] q1[x], P2 = sum dp Sa, P3 = sum_x rdp[x] q3[x],
//     P15 = sum dp D1, P16 = sum dp[x][y] D2[y][x], tot, d3:
//     dW_{0,6..14} = n P0, dW_5 = P0, dW_1 = P1, dW_2 = n P2, dW_3 = P3, dW_4 = tr tot, dW_15 = P15,
//     dW_16 = P16, dW_17 = tr d3.
// Level >= 1: the forward's row walk again (same loads), every sum lane-level (dp[a][b] . t summed
// over the walk, wave totals once at the end).  Level 0 (T = X[j_a] on C_a) in closed form from the
// per-neighbour masked sums R1[a] = sum_{b in C_a} dp[a][b], R2[a] = sum_{b in C_a} dp[b][a],
// R3[a] = sum_{b in C_a} rdp[b], BS[a] = sum_{b,z in C_a} dp[b][z], which also give dX's per-node
// terms  G[a] = sum_{b,z in C_a} dT[a][b][z]  (k_ccn2_dx0 adds them up per input node).
template <int CM, int HC, int NB, bool L0>
__global__ void __launch_bounds__(256) k_c2_bwd(CcnPlanView v, const int* total_nodes, float* __restrict__ dF,
                                                const float* __restrict__ dtop, int dtop_ld,
                                                const float* __restrict__ F, const float* __restrict__ fin,
                                                const float* __restrict__ X, int cin,
                                                const float* __restrict__ W, int h, int ncap,
                                                float* __restrict__ rdp_g, float* __restrict__ trd_g,
                                                float* __restrict__ ppart, float* __restrict__ g0) {
    extern __shared__ float c2_dyn[];
    __shared__ unsigned long long vmask[C2_NCAP];
    __shared__ int s_oj[C2_NCAP], s_dj[C2_NCAP];
    __shared__ float s_x[C2_NCAP][CM];
    __shared__ float wc[NWC][HC][CM];
    __shared__ float rdpL[C2_NCAP][HC];
    __shared__ float trL[HC];
    __shared__ float red[4][C2_NACC][HC][CM];
    __shared__ float redt[4][2][CM];  // tot, d3
    __shared__ float redb[4][HC];
    __shared__ float gs[C2_NCAP][CM];
    __shared__ float rs[C2_NCAP][4][HC];  // level 0: R1, R2, R3, BS per neighbour
    const int i = blockIdx.x;
    if (i >= *total_nodes) return;
    const int n = v.deg[i];
    if (n > C2_NCAP || n > ncap || cin > CM) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    float* dpL = c2_dyn;
    short* sp = reinterpret_cast<short*>(c2_dyn + ncap * ncap * HC);
    c2_prologue<CM>(v, i, n, L0 ? 1 : 0, X, cin, sp, vmask, s_oj, s_dj, s_x);
    const long long o2 = v.off2[i], o1 = v.off1[i];
    const int gi = v.graph[i];
    const bool la = lane < n;
    const unsigned long long my_mask = la ? vmask[lane] : 0ull;
    const int my_oj = la ? s_oj[lane] : 0, my_dj = la ? s_dj[lane] : 0;
    const float nf = (float)n;
    const int K = 18 * cin;
    float* pp = ppart + (long long)i * (h * K + h);
    for (int e = threadIdx.x; e < C2_NCAP * CM; e += 256) (&gs[0][0])[e] = 0.f;
    for (int o0 = 0; o0 < h; o0 += HC) {
        const int hc = min(HC, h - o0);
        c2_weights<HC, CM>(wc, W, cin, o0, hc);
        float sb[HC];
#pragma unroll
        for (int o = 0; o < HC; ++o) sb[o] = 0.f;
        for (int e = threadIdx.x; e < n * n; e += 256) {
#pragma unroll
            for (int o = 0; o < HC; ++o) {
                float d = 0.f;
                if (o < hc) {
                    const long long r = (o2 + e) * h + o0 + o;
                    d = F[r] > 0.f ? (dtop ? dtop[(long long)gi * dtop_ld + o0 + o] : dF[r]) : 0.f;
                    dF[r] = d;
                }
                dpL[e * HC + o] = d;
                sb[o] += d;
            }
        }
#pragma unroll
        for (int o = 0; o < HC; ++o) {
            const float t = wave_total(sb[o]);
            if (lane == 0) redb[wv][o] = t;
        }
        __syncthreads();
        // row sums and trace of dp
        for (int x = wv; x < n; x += 4)
#pragma unroll
            for (int o = 0; o < HC; ++o) {
                const float r = wave_total(lane < n ? dpL[(x * n + lane) * HC + o] : 0.f);
                if (lane == 0) {
                    rdpL[x][o] = r;
                    if (o < hc) rdp_g[(o1 + x) * h + o0 + o] = r;
                }
            }
        if (wv == 0)
#pragma unroll
            for (int o = 0; o < HC; ++o) {
                const float r = wave_total(lane < n ? dpL[(lane * n + lane) * HC + o] : 0.f);
                if (lane == 0) {
                    trL[o] = r;
                    if (o < hc) trd_g[(long long)i * h + o0 + o] = r;
                }
            }
        __syncthreads();
        if constexpr (L0) {
            // per neighbour a (wave per a): the masked sums of dp the closed forms need
            for (int a = wv; a < n; a += 4) {
                const unsigned long long ma = vmask[a];
                const bool vb = lane < n && ((ma >> lane) & 1ull);
#pragma unroll
                for (int o = 0; o < HC; ++o) {
                    const float r1 = wave_total(vb ? dpL[(a * n + lane) * HC + o] : 0.f);
                    const float r2 = wave_total(vb ? dpL[(lane * n + a) * HC + o] : 0.f);
                    const float r3 = wave_total(vb ? rdpL[lane][o] : 0.f);
                    float s = 0.f;
                    unsigned long long zs = ma;
                    while (zs) {
                        const int z = __ffsll((long long)zs) - 1;
                        zs &= zs - 1ull;
                        s += vb ? dpL[(lane * n + z) * HC + o] : 0.f;
                    }
                    const float bs = wave_total(s);
                    if (lane == 0) {
                        rs[a][0][o] = r1;
                        rs[a][1][o] = r2;
                        rs[a][2][o] = r3;
                        rs[a][3][o] = bs;
                    }
                }
            }
            __syncthreads();
            // parameter partials: (o, c) pairs over the waves, lanes over the neighbours a, wave totals
            for (int p = wv; p < hc * cin; p += 4) {
                const int o = p / cin, c = p % cin;
                const float mf = (float)__popcll(my_mask);
                const bool va = la && ((my_mask >> lane) & 1ull);
                const float x = la ? s_x[lane][c] : 0.f;
                const float r1 = la ? rs[lane][0][o] : 0.f, r2 = la ? rs[lane][1][o] : 0.f;
                const float r3 = la ? rs[lane][2][o] : 0.f, bs = la ? rs[lane][3][o] : 0.f;
                const float ra = la ? rdpL[lane][o] : 0.f;
                const float s0 = wave_total(mf * x * r1), s1 = wave_total(mf * mf * x * ra);
                const float s2 = wave_total(x * bs), s3 = wave_total(mf * x * r3);
                const float s15 = wave_total(x * r1), s16 = wave_total(va ? x * r2 : 0.f);
                const float tt = wave_total(mf * mf * x), dd = wave_total(va ? x : 0.f);
                if (lane == 0)
                    c2_write_partials(pp + (long long)(o0 + o) * K, cin, c, nf, s0, s1, s2, s3, s15, s16, trL[o] * tt,
                                      trL[o] * dd);
            }
            // G[a] = m_a sum dSc[a][.] + sum dSa + sum dD1[a][.] + [a in C_a](sum dD2[a][.] + dd3), this chunk's o
            for (int t = threadIdx.x; t < n * cin; t += 256) {
                const int a = t / cin, c = t % cin;
                const unsigned long long ma = vmask[a];
                const float mf = (float)__popcll(ma);
                const bool va = (ma >> a) & 1ull;
                float g = 0.f;
                for (int o = 0; o < hc; ++o) {
                    const float r1 = rs[a][0][o], r2 = rs[a][1][o], r3 = rs[a][2][o], bs = rs[a][3][o];
                    float s = mf * fmaf(fmaf(nf, wc[WA][o][c], wc[WB][o][c]), r1, mf * wc[WQ1][o][c] * rdpL[a][o]);
                    s = fmaf(nf * wc[WQ2][o][c], bs, s);
                    s = fmaf(mf * wc[WQ3][o][c], r3, s);
                    s = fmaf(mf * mf * wc[WQ4][o][c], trL[o], s);
                    s = fmaf(wc[WQ15][o][c], r1, s);
                    if (va) s = fmaf(wc[WQ16][o][c], r2, fmaf(wc[WQ17][o][c], trL[o], s));
                    g += s;
                }
                gs[a][c] += g;
            }
        } else {
            float acc[C2_NACC][HC][CM], tot[CM], d3[CM];
#pragma unroll
            for (int k = 0; k < C2_NACC; ++k)
#pragma unroll
                for (int o = 0; o < HC; ++o)
#pragma unroll
                    for (int c = 0; c < CM; ++c) acc[k][o][c] = 0.f;
#pragma unroll
            for (int c = 0; c < CM; ++c) tot[c] = d3[c] = 0.f;
            for (int b = wv; b < n; b += 4) {
                float sa[CM];
#pragma unroll
                for (int c = 0; c < CM; ++c) sa[c] = 0.f;
                unsigned long long as = __ballot(la && ((my_mask >> b) & 1ull));
                const float* my_row = c2_row_of(fin, cin, sp, n, b, (as >> lane) & 1ull, my_oj, my_dj);
                // lane a: dp[a][b], dp[b][a], rdp[a] of this row (read once, then by readlane)
                float my_ab[HC], my_ba[HC], my_ra[HC];
#pragma unroll
                for (int o = 0; o < HC; ++o) {
                    my_ab[o] = la ? dpL[(lane * n + b) * HC + o] : 0.f;
                    my_ba[o] = la ? dpL[(b * n + lane) * HC + o] : 0.f;
                    my_ra[o] = la ? rdpL[lane][o] : 0.f;
                }
                while (as) {
                    int aa[NB];
                    c2_take<NB>(as, aa);
                    float t[NB][CM];
                    c2_load_rows<CM, NB>(cin, n, aa, sp, my_mask, my_row, t);
#pragma unroll
                    for (int u = 0; u < NB; ++u) {
                        const int a = aa[u];
                        if (a < 0) break;
#pragma unroll
                        for (int o = 0; o < HC; ++o) {
                            const float dab = lane_value(my_ab[o], a), dba = lane_value(my_ba[o], a);
                            const float ra = lane_value(my_ra[o], a);
                            const float d15 = lane == b ? dab : 0.f, d16 = lane == a ? dba : 0.f;
#pragma unroll
                            for (int c = 0; c < CM; ++c) {
                                acc[0][o][c] = fmaf(dab, t[u][c], acc[0][o][c]);
                                acc[1][o][c] = fmaf(ra, t[u][c], acc[1][o][c]);
                                acc[4][o][c] = fmaf(d15, t[u][c], acc[4][o][c]);
                                acc[5][o][c] = fmaf(d16, t[u][c], acc[5][o][c]);
                            }
                        }
                        if (a == b && lane == b)
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
                    const float q3 = wave_total(sa[c]);  // uniform: P3 and tot kept in lane 0 only
                    if (lane == 0) {
#pragma unroll
                        for (int o = 0; o < HC; ++o) acc[3][o][c] = fmaf(rdpL[b][o], q3, acc[3][o][c]);
                        tot[c] += q3;
                    }
                }
            }
            // lane-level sums -> wave totals (P3 and tot are lane 0's)
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
                        for (int c = 0; c < CM; ++c) red[wv][k][o][c] = acc[k][o][c];
#pragma unroll
                for (int c = 0; c < CM; ++c) {
                    redt[wv][0][c] = tot[c];
                    redt[wv][1][c] = d3[c];
                }
            }
            __syncthreads();
            for (int t = threadIdx.x; t < hc * cin; t += 256) {
                const int o = t / cin, c = t % cin;
                float s[C2_NACC];
#pragma unroll
                for (int k = 0; k < C2_NACC; ++k)
                    s[k] = (red[0][k][o][c] + red[1][k][o][c]) + (red[2][k][o][c] + red[3][k][o][c]);
                const float tt = (redt[0][0][c] + redt[1][0][c]) + (redt[2][0][c] + redt[3][0][c]);
                const float dd = (redt[0][1][c] + redt[1][1][c]) + (redt[2][1][c] + redt[3][1][c]);
                c2_write_partials(pp + (long long)(o0 + o) * K, cin, c, nf, s[0], s[1], s[2], s[3], s[4], s[5],
                                  trL[o] * tt, trL[o] * dd);
            }
        }
        if ((int)threadIdx.x < hc)
            pp[(long long)h * K + o0 + threadIdx.x] = (redb[0][threadIdx.x] + redb[1][threadIdx.x]) +
                                                      (redb[2][threadIdx.x] + redb[3][threadIdx.x]);
        __syncthreads();
    }
    if (L0 && g0) {
        __syncthreads();
        for (int t = threadIdx.x; t < n * cin; t += 256) g0[(o1 + t / cin) * cin + t % cin] = gs[t / cin][t % cin];
    }
}

// Gather of one CCN-2D level's input gradient from the dp format (no atomics): node j collects, for
// every neighbour i = i_a with u, w in C_a, the gradient of the entry of T_i that read F_j[u][w]:
//   dF_{l-1}[j][u][w] = sum_a dT_i[aj][b][z] (+ readout),  b = p_a(u), z = p_a(w), aj = position of j in N(i),
//   dT[a][b][z] = dSc[a][b] + dSa[b][z] + [z = b] dD1[a][b] + [z = a] dD2[a][b] + [a = b = z] dd3,
//   dSc[a][b] = (n_i A + W5)^T dp[a][b] + W1^T rdp[a],   dSa[b][z] = n_i W2^T dp[b][z] + W3^T rdp[b] + W4^T tr,
//   dD1[a][b] = W15^T dp[a][b],   dD2[a][b] = W16^T dp[b][a],   dd3 = W17^T tr      (A = W0 + W6 + ... + W14).
// Per (u, a) the wave-uniform part is five h-vectors of node i, the lane part one row piece dp[b][z].
// The level's input has cin = h channels (levels >= 1 only: level 0 goes through k_ccn2_dx0).
template <int H>
__device__ __forceinline__ void c2_dT_weights(float (*wc)[H][H], const float* __restrict__ W, int h) {
    const int K = 18 * h;
    for (int t = threadIdx.x; t < H * H; t += blockDim.x) {
        const int o = t / H, c = t % H;
        const bool ok = o < h && c < h;
        const float* w = W + (long long)(ok ? o : 0) * K;
        float r[18];
#pragma unroll
        for (int q = 0; q < 18; ++q) r[q] = ok ? w[q * h + c] : 0.f;
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

struct C2Dp {
    const float* dp;   // [sum d^2][h]
    const float* rdp;  // [sum d][h]
    const float* trd;  // [nodes][h]
};

// loads of one (i, a) pair: ld[0] dp[aj][b], ld[1] dp[b][aj], ld[2] rdp[aj], ld[3] rdp[b], ld[4] tr, ld[5] dp[b][z]
template <int H>
__device__ __forceinline__ void c2_dT_load(const C2Dp& g, int h, long long oi, long long o1i, int i, int di, int aj,
                                           int b, int z, float (&ld)[6][H]) {
    const float* pab = g.dp + (oi + (long long)aj * di + b) * h;
    const float* pba = g.dp + (oi + (long long)b * di + aj) * h;
    const float* pbz = g.dp + (oi + (long long)b * di + z) * h;
#pragma unroll
    for (int o = 0; o < H; ++o) {
        const bool ok = o < h;
        ld[0][o] = ok ? pab[o] : 0.f;
        ld[1][o] = ok ? pba[o] : 0.f;
        ld[2][o] = ok ? g.rdp[(o1i + aj) * h + o] : 0.f;
        ld[3][o] = ok ? g.rdp[(o1i + b) * h + o] : 0.f;
        ld[4][o] = ok ? g.trd[(long long)i * h + o] : 0.f;
        ld[5][o] = ok ? pbz[o] : 0.f;
    }
}

template <int H>
__device__ __forceinline__ void c2_dT_add(const float (*wc)[H][H], const float (&ld)[6][H], int h, float nfi, int aj,
                                          int b, int z, float (&acc)[H]) {
    const bool e1 = z == b, e2 = z == aj, e3 = aj == b && b == z;
#pragma unroll
    for (int c = 0; c < H; ++c) {
        if (c >= h) break;
        float s = 0.f;
#pragma unroll
        for (int o = 0; o < H; ++o) {
            if (o >= h) break;
            s = fmaf(fmaf(nfi, wc[WA][o][c], wc[WB][o][c]), ld[0][o], s);
            s = fmaf(wc[WQ1][o][c], ld[2][o], s);
            s = fmaf(wc[WQ3][o][c], ld[3][o], s);
            s = fmaf(wc[WQ4][o][c], ld[4][o], s);
            s = fmaf(nfi * wc[WQ2][o][c], ld[5][o], s);
            if (e1) s = fmaf(wc[WQ15][o][c], ld[0][o], s);
            if (e2) s = fmaf(wc[WQ16][o][c], ld[1][o], s);
            if (e3) s = fmaf(wc[WQ17][o][c], ld[4][o], s);
        }
        acc[c] += s;
    }
}

template <int H, int NB>
__global__ void __launch_bounds__(256) k_c2_gather(CcnPlanView v, const int* total_nodes, C2Dp g,
                                                   const float* __restrict__ W, int h, const float* __restrict__ dsum,
                                                   int dsum_ld, int dsum_off, float* __restrict__ dout) {
    __shared__ short sp[C2_NCAP * C2_NCAP];
    __shared__ unsigned long long vmask[C2_NCAP];
    __shared__ int s_i[C2_NCAP], s_di[C2_NCAP], s_oi[C2_NCAP], s_o1[C2_NCAP], s_aj[C2_NCAP];
    __shared__ float wc[NWC][H][H];
    const int j = blockIdx.x;
    if (j >= *total_nodes) return;
    const int n = v.deg[j];
    if (n > C2_NCAP || h > H) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long o2 = v.off2[j];
    const int* nj = v.nbr + (long long)j * v.nmax;
    const int sj = v.selfpos[j];
    const int gr = v.graph[j];
    c2_dT_weights<H>(wc, W, h);
    c2_copy_pos(v.pos + o2, n * n, sp);
    if ((int)threadIdx.x < n) {
        const int i = nj[threadIdx.x];
        s_i[threadIdx.x] = i;
        s_di[threadIdx.x] = v.deg[i];
        s_oi[threadIdx.x] = v.off2[i];
        s_o1[threadIdx.x] = v.off1[i];
    }
    __syncthreads();
    for (int a = wv; a < n; a += 4) {
        const unsigned long long m = __ballot(lane < n && sp[a * n + lane] >= 0);
        if (lane == 0) {
            vmask[a] = m;
            s_aj[a] = sp[a * n + sj];  // position of j in N(i_a)
        }
    }
    __syncthreads();
    float rd[H];
#pragma unroll
    for (int c = 0; c < H; ++c) rd[c] = (dsum && c < h) ? dsum[(long long)gr * dsum_ld + dsum_off + c] : 0.f;
    // lane a holds neighbour i_a's mask, node, degree, offsets, the position aj of j in N(i_a), and the
    // row-independent parts of its dp format (rdp_i[aj], tr_i)
    const bool la = lane < n;
    const unsigned long long my_mask = la ? vmask[lane] : 0ull;
    const int my_i = la ? s_i[lane] : 0, my_di = la ? s_di[lane] : 0, my_oi = la ? s_oi[lane] : 0;
    const int my_o1 = la ? s_o1[lane] : 0, my_aj = la ? s_aj[lane] : 0;
    float my_ra[H], my_tr[H];
#pragma unroll
    for (int o = 0; o < H; ++o) {
        my_ra[o] = (la && o < h) ? g.rdp[((long long)my_o1 + my_aj) * h + o] : 0.f;
        my_tr[o] = (la && o < h) ? g.trd[(long long)my_i * h + o] : 0.f;
    }
    for (int u = wv; u < n; u += 4) {
        float acc[H];
#pragma unroll
        for (int c = 0; c < H; ++c) acc[c] = 0.f;
        // lanes a with u in C_a: b = p_a(u), and every part of dT_i[aj][b][.] that does not depend on z,
        // projected through the weights once per row:
        //   base = (n_i A + W5)^T dp[aj][b] + W1^T rdp[aj] + W3^T rdp[b] + W4^T tr,
        //   e1 = W15^T dp[aj][b] (z = b), e2 = W16^T dp[b][aj] (z = aj), e3 = W17^T tr (aj = b = z);
        // the walk then adds n_i W2^T dp[b][z] per lane
        const unsigned long long au = __ballot(la && ((my_mask >> u) & 1ull));
        const bool in = (au >> lane) & 1ull;
        const int my_b = in ? (int)sp[lane * n + u] : 0;
        const float nfi = (float)my_di;
        float base[H], e1[H], e2[H], e3[H];
        {
            const float* pab = g.dp + ((long long)my_oi + (long long)my_aj * my_di + my_b) * h;
            const float* pba = g.dp + ((long long)my_oi + (long long)my_b * my_di + my_aj) * h;
            const float* prb = g.rdp + ((long long)my_o1 + my_b) * h;
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
        const float* my_row = g.dp + ((long long)my_oi + (long long)my_b * my_di) * h;  // row b of dp_i
        // the neighbours a with u in C_a, ascending, NB at a time: one row piece dp_i[b][z] per lane each
        unsigned long long as = au;
        while (as) {
            int aa[NB];
            c2_take<NB>(as, aa);
            float dz[NB][H];
            int zz[NB];
            bool vz[NB];
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                const int a = aa[q] >= 0 ? aa[q] : 0;
                vz[q] = aa[q] >= 0 && ((lane_value_u64(my_mask, a) >> lane) & 1ull);
                zz[q] = vz[q] ? (int)sp[a * n + lane] : 0;
                const float* pz = lane_value_ptr(my_row, a) + zz[q] * h;
#pragma unroll
                for (int o = 0; o < H; ++o) dz[q][o] = o < h ? pz[o] : 0.f;
            }
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                const int a = aa[q];
                if (a < 0) break;
                const int b = lane_value_i(my_b, a), aj = lane_value_i(my_aj, a);
                const float nfa = lane_value(nfi, a);
                const bool f1 = zz[q] == b, f2 = zz[q] == aj, f3 = f1 && aj == b;
#pragma unroll
                for (int c = 0; c < H; ++c) {
                    if (c >= h) break;
                    float w2 = 0.f;
#pragma unroll
                    for (int o = 0; o < H; ++o) {
                        if (o >= h) break;
                        w2 = fmaf(wc[WQ2][o][c], dz[q][o], w2);
                    }
                    const float x1 = lane_value(e1[c], a), x2 = lane_value(e2[c], a), x3 = lane_value(e3[c], a);
                    float t = fmaf(nfa, w2, lane_value(base[c], a));
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
}

// dp format for the nodes of degree 65..256 (their parameter partials and level-0 terms come from
// k_ccn2_bwd_node_big, which reads the raw dF): dp in place, row sums, trace
__global__ void __launch_bounds__(256) k_c2_dp_big(CcnPlanView v, const int* total_nodes, float* __restrict__ dF,
                                                   const float* __restrict__ F, int h, float* __restrict__ rdp_g,
                                                   float* __restrict__ trd_g) {
    const int i = blockIdx.x;
    if (i >= *total_nodes) return;
    const int n = v.deg[i];
    if (n <= C2_NCAP || n > CCN_BIGD) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long o2 = v.off2[i], o1 = v.off1[i];
    __shared__ float trp[4];
    for (int o = 0; o < h; ++o) {
        float tr = 0.f;
        for (int x = wv; x < n; x += 4) {
            float s = 0.f;
            for (int y = lane; y < n; y += 64) {
                const long long r = (o2 + (long long)x * n + y) * h + o;
                const float d = F[r] > 0.f ? dF[r] : 0.f;
                dF[r] = d;
                s += d;
                if (y == x) tr += d;
            }
            s = wave_total(s);
            if (lane == 0) rdp_g[(o1 + x) * h + o] = s;
        }
        tr = wave_total(tr);
        if (lane == 0) trp[wv] = tr;
        __syncthreads();
        if (threadIdx.x == 0) trd_g[(long long)i * h + o] = (trp[0] + trp[1]) + (trp[2] + trp[3]);
        __syncthreads();
    }
}


// ------------------------------------------------------------------ CCN-2D, degrees 65..256
// The same passes as k_ccn2_fwd / k_ccn2_bwd_node / k_ccn2_bwd_gather for the nodes whose receptive
// field exceeds one wave (SBM graphs of several hundred nodes: d ~ 70-210): the lane index walks its
// range in 64-lane chunks, the common-neighbour sets C_a are CCN_BW 64-bit words per row (LDS), and
// the position maps are read from global memory (n^2 ints per node, L2-resident) instead of LDS.
// Launched only when a batch can hold such degrees (nmax > 64); nodes with d <= 64 exit at once
// (they are the fast kernels'), so every node is computed by exactly one of the two.
template <int CM, int HM>
__global__ void __launch_bounds__(256) k_ccn2_fwd_big(CcnPlanView v, const int* total_nodes,
                                                      const float* __restrict__ fin, int level0,
                                                      const float* __restrict__ X, int cin,
                                                      const float* __restrict__ W, const float* __restrict__ bias,
                                                      int h, C2Save sv, float* __restrict__ fout,
                                                      float* __restrict__ nsum) {
    __shared__ unsigned long long vmask[CCN_BIGD][CCN_BW];  // bit x of row a: x in C_a
    __shared__ int s_j[CCN_BIGD], s_dj[CCN_BIGD], s_oj[CCN_BIGD], s_mc[CCN_BIGD];
    __shared__ float sred[2][4][CM];
    const int i = blockIdx.x;
    if (i >= *total_nodes) return;
    const int n = v.deg[i];
    if (n <= CCN_MAXD || n > CCN_BIGD || cin > CM || h > HM) return;
    const int nw = (n + 63) >> 6;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int* ni = v.nbr + (long long)i * v.nmax;
    const long long o2 = v.off2[i], o1 = v.off1[i];
    const int* sp = v.pos + o2;  // sp[a n + x]
    for (int t = threadIdx.x; t < n; t += 256) {
        const int j = ni[t];
        s_j[t] = j;
        s_dj[t] = v.deg[j];
        s_oj[t] = v.off2[j];
    }
    for (int a = wv; a < n; a += 4) {
        int cnt = 0;
        for (int w = 0; w < nw; ++w) {
            const int x = w * 64 + lane;
            const unsigned long long m = __ballot(x < n && sp[(long long)a * n + x] >= 0);
            if (lane == 0) vmask[a][w] = m;
            cnt += __popcll(m);
        }
        if (lane == 0) s_mc[a] = cnt;
    }
    __syncthreads();

    // ---- pass A: wave per neighbour a, lane b (64-lane chunks)
    float tq[CM], td3[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c) tq[c] = td3[c] = 0.f;
    for (int a = wv; a < n; a += 4) {
        const int j = s_j[a], dj = s_dj[a];
        const bool va = mbit(vmask[a], a);
        float qa[CM];
#pragma unroll
        for (int c = 0; c < CM; ++c) qa[c] = 0.f;
        for (int b0 = 0; b0 < n; b0 += 64) {
            const int b = b0 + lane;
            const int pb = b < n ? sp[(long long)a * n + b] : -1;
            const bool vb = pb >= 0;
            float sc[CM], d1[CM], d2[CM];
#pragma unroll
            for (int c = 0; c < CM; ++c) sc[c] = d1[c] = d2[c] = 0.f;
            if (level0) {
                const float mf = (float)s_mc[a];
#pragma unroll
                for (int c = 0; c < CM; ++c) {
                    if (c >= cin) break;
                    const float xj = X[(long long)j * cin + c];
                    sc[c] = vb ? mf * xj : 0.f;
                    d1[c] = vb ? xj : 0.f;
                    d2[c] = (vb && va) ? xj : 0.f;
                }
            } else {
                const float* row = fin + ((long long)s_oj[a] + (long long)(vb ? pb : 0) * dj) * cin;
                for (int w = 0; w < nw; ++w) {
                    unsigned long long zs = vmask[a][w];
                    while (zs) {
                        int zz[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            zz[u] = zs ? w * 64 + __ffsll((long long)zs) - 1 : -1;
                            zs &= zs ? zs - 1ull : 0ull;
                        }
                        float t[4][CM];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int pz = zz[u] >= 0 ? sp[(long long)a * n + zz[u]] : 0;
#pragma unroll
                            for (int c = 0; c < CM; ++c) t[u][c] = c < cin ? row[(long long)pz * cin + c] : 0.f;
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int z = zz[u];
                            if (z < 0) break;
                            if (vb) {
#pragma unroll
                                for (int c = 0; c < CM; ++c) {
                                    if (c >= cin) break;
                                    sc[c] += t[u][c];
                                    if (z == b) d1[c] = t[u][c];
                                    if (z == a) d2[c] = t[u][c];
                                }
                            }
                        }
                    }
                }
            }
            if (b < n) {
                const long long r = (o2 + (long long)a * n + b) * cin;
#pragma unroll
                for (int c = 0; c < CM; ++c) {
                    if (c >= cin) break;
                    sv.Sc[r + c] = sc[c];
                    sv.D1[r + c] = d1[c];
                    sv.D2[r + c] = d2[c];
                }
            }
#pragma unroll
            for (int c = 0; c < CM; ++c) {
                if (c >= cin) break;
                qa[c] += wave_sum(sc[c]);
                if (b == a) td3[c] += d1[c];  // T[a][a][a]
            }
        }
#pragma unroll
        for (int c = 0; c < CM; ++c) {
            if (c >= cin) break;
            if (lane == 0) sv.q1[(o1 + a) * cin + c] = qa[c];
            tq[c] += qa[c];
        }
    }
#pragma unroll
    for (int c = 0; c < CM; ++c) {
        if (c >= cin) break;
        const float t3 = wave_sum(td3[c]);
        if (lane == 0) {
            sred[0][wv][c] = tq[c];
            sred[1][wv][c] = t3;
        }
    }

    // ---- pass B: wave per receptive-field row b, lane z (chunks); the a with b in C_a ascending
    for (int b = wv; b < n; b += 4) {
        float q3[CM];
#pragma unroll
        for (int c = 0; c < CM; ++c) q3[c] = 0.f;
        for (int z0 = 0; z0 < n; z0 += 64) {
            const int z = z0 + lane;
            float sa[CM];
#pragma unroll
            for (int c = 0; c < CM; ++c) sa[c] = 0.f;
            for (int a0 = 0; a0 < n; a0 += 64) {
                const int al = a0 + lane < n ? a0 + lane : 0;
                unsigned long long as = __ballot(a0 + lane < n && mbit(vmask[al], b));
                while (as) {
                    int aa[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        aa[u] = as ? a0 + __ffsll((long long)as) - 1 : -1;
                        as &= as ? as - 1ull : 0ull;
                    }
                    float t[4][CM];
                    bool vz[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int a = aa[u] >= 0 ? aa[u] : 0;
                        vz[u] = aa[u] >= 0 && z < n && mbit(vmask[a], z);
                        const float* q;
                        if (level0) {
                            q = X + (long long)s_j[a] * cin;
                        } else {
                            const int pb = max(sp[(long long)a * n + b], 0), pz = vz[u] ? sp[(long long)a * n + z] : 0;
                            q = fin + ((long long)s_oj[a] + (long long)pb * s_dj[a] + pz) * cin;
                        }
#pragma unroll
                        for (int c = 0; c < CM; ++c) t[u][c] = c < cin ? q[c] : 0.f;
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        if (aa[u] < 0) break;
                        if (vz[u]) {
#pragma unroll
                            for (int c = 0; c < CM; ++c) {
                                if (c >= cin) break;
                                sa[c] += t[u][c];
                            }
                        }
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < CM; ++c) {
                if (c >= cin) break;
                if (z < n) sv.Sa[(o2 + (long long)b * n + z) * cin + c] = sa[c];
                q3[c] += wave_sum(sa[c]);
            }
        }
#pragma unroll
        for (int c = 0; c < CM; ++c) {
            if (c >= cin) break;
            if (lane == 0) sv.q3[(o1 + b) * cin + c] = q3[c];
        }
    }
    __syncthreads();
    if (threadIdx.x < cin) {
        const int c = threadIdx.x;
        float t = 0.f, t3 = 0.f;
        for (int w = 0; w < 4; ++w) {
            t += sred[0][w][c];
            t3 += sred[1][w][c];
        }
        sv.tot[(long long)i * cin + c] = t;
        sv.d3[(long long)i * cin + c] = t3;
    }
    __syncthreads();
    // output stage: as k_ccn2_fwd
    const float nf = (float)n;
    const int K = 18 * cin;
    __shared__ float sw[HM * 18 * CM];
    for (int t = threadIdx.x; t < h * K; t += 256) sw[t] = W[t];
    __syncthreads();
    float ns[HM];  // this node's sum of F_out (readout)
#pragma unroll
    for (int o = 0; o < HM; ++o) ns[o] = 0.f;
    for (int e = threadIdx.x; e < n * n; e += 256) {
        const int x = e / n, y = e % n;
        float s[HM];
#pragma unroll
        for (int o = 0; o < HM; ++o) s[o] = o < h ? bias[o] : 0.f;
        for (int c = 0; c < cin; ++c) {
            const float sc = sv.Sc[(o2 + e) * cin + c];
            const float sa = sv.Sa[(o2 + e) * cin + c];
            float blk[18];
            blk[0] = nf * sc;
            blk[1] = sv.q1[(o1 + x) * cin + c];
            blk[2] = nf * sa;
            blk[3] = sv.q3[(o1 + x) * cin + c];
            blk[4] = x == y ? sv.tot[(long long)i * cin + c] : 0.f;
            blk[5] = sc;
#pragma unroll
            for (int q = 6; q < 15; ++q) blk[q] = nf * sc;
            blk[15] = sv.D1[(o2 + e) * cin + c];
            blk[16] = sv.D2[(o2 + (long long)y * n + x) * cin + c];
            blk[17] = x == y ? sv.d3[(long long)i * cin + c] : 0.f;
#pragma unroll
            for (int o = 0; o < HM; ++o) {
                if (o >= h) break;
                const float* w = sw + o * K;
#pragma unroll
                for (int q = 0; q < 18; ++q) s[o] = fmaf(w[q * cin + c], blk[q], s[o]);
            }
        }
#pragma unroll
        for (int o = 0; o < HM; ++o) {
            if (o >= h) break;
            s[o] = s[o] < 0.f ? 0.f : s[o];
            fout[(o2 + e) * h + o] = s[o];
            ns[o] += s[o];
        }
    }
    __shared__ float s_ns[4][HM];
#pragma unroll
    for (int o = 0; o < HM; ++o) {
        const float t = wave_total(ns[o]);
        if (lane == 0) s_ns[wv][o] = t;
    }
    __syncthreads();
    if ((int)threadIdx.x < h)
        nsum[(long long)i * h + threadIdx.x] =
            (s_ns[0][threadIdx.x] + s_ns[1][threadIdx.x]) + (s_ns[2][threadIdx.x] + s_ns[3][threadIdx.x]);
}

// k_c2_gather for degrees 65..256: lane w of row u in 64-lane chunks, the neighbours a with u in C_a
// in 64-wide ballot chunks (ascending), position maps read from global memory (L2-resident)
template <int H, int NB>
__global__ void __launch_bounds__(256) k_c2_gather_big(CcnPlanView v, const int* total_nodes, C2Dp g,
                                                       const float* __restrict__ W, int h,
                                                       const float* __restrict__ dsum, int dsum_ld, int dsum_off,
                                                       float* __restrict__ dout) {
    __shared__ unsigned long long vmask[CCN_BIGD][CCN_BW];
    __shared__ int s_i[CCN_BIGD], s_di[CCN_BIGD], s_oi[CCN_BIGD], s_o1[CCN_BIGD], s_aj[CCN_BIGD];
    __shared__ float wc[NWC][H][H];
    const int j = blockIdx.x;
    if (j >= *total_nodes) return;
    const int n = v.deg[j];
    if (n <= C2_NCAP || n > CCN_BIGD || h > H) return;
    const int nw = (n + 63) >> 6;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long o2 = v.off2[j];
    const int* sp = v.pos + o2;
    const int* nj = v.nbr + (long long)j * v.nmax;
    const int sj = v.selfpos[j];
    const int gr = v.graph[j];
    c2_dT_weights<H>(wc, W, h);
    for (int t = threadIdx.x; t < n; t += 256) {
        const int i = nj[t];
        s_i[t] = i;
        s_di[t] = v.deg[i];
        s_oi[t] = v.off2[i];
        s_o1[t] = v.off1[i];
        s_aj[t] = sp[(long long)t * n + sj];  // position of j in N(i_a)
    }
    for (int a = wv; a < n; a += 4)
        for (int w = 0; w < nw; ++w) {
            const int x = w * 64 + lane;
            const unsigned long long m = __ballot(x < n && sp[(long long)a * n + x] >= 0);
            if (lane == 0) vmask[a][w] = m;
        }
    __syncthreads();
    float rd[H];
#pragma unroll
    for (int c = 0; c < H; ++c) rd[c] = (dsum && c < h) ? dsum[(long long)gr * dsum_ld + dsum_off + c] : 0.f;
    for (int u = wv; u < n; u += 4) {
        for (int w0 = 0; w0 < n; w0 += 64) {
            const int wl = w0 + lane;
            float acc[H];
#pragma unroll
            for (int c = 0; c < H; ++c) acc[c] = 0.f;
            for (int a0 = 0; a0 < n; a0 += 64) {
                const int al = a0 + lane < n ? a0 + lane : 0;
                unsigned long long as = __ballot(a0 + lane < n && mbit(vmask[al], u));
                while (as) {
                    int aa[NB];
                    c2_take<NB>(as, aa);
                    float ld[NB][6][H];
                    int zb[NB], zz[NB];
                    bool vz[NB];
#pragma unroll
                    for (int q = 0; q < NB; ++q) {
                        const int a = aa[q] >= 0 ? a0 + aa[q] : 0;
                        vz[q] = aa[q] >= 0 && wl < n && mbit(vmask[a], wl);
                        zb[q] = max(sp[(long long)a * n + u], 0);
                        zz[q] = vz[q] ? sp[(long long)a * n + wl] : 0;
                        c2_dT_load<H>(g, h, s_oi[a], s_o1[a], s_i[a], s_di[a], s_aj[a], zb[q], zz[q], ld[q]);
                    }
#pragma unroll
                    for (int q = 0; q < NB; ++q) {
                        if (aa[q] < 0) break;
                        if (!vz[q]) continue;
                        const int a = a0 + aa[q];
                        c2_dT_add<H>(wc, ld[q], h, (float)s_di[a], s_aj[a], zb[q], zz[q], acc);
                    }
                }
            }
            if (wl < n)
#pragma unroll
                for (int c = 0; c < H; ++c) {
                    if (c >= h) break;
                    dout[(o2 + (long long)u * n + wl) * h + c] = acc[c] + rd[c];
                }
        }
    }
}

// ------------------------------------------------------------------ readout
// feat[b] = cat_l (sum over the graph's rows of F_l); level 0: sum_i d_i^order X[i]
struct ReadoutArgs {
    int nch;              // chunks per graph of k_ccn_readout_part
    int per_node;         // F[l] holds per-node sums ([nodes][h], CCN-2D) instead of feature rows
    CcnPlanView v;
    int order, L, f, h, n_out, bs;
    const float* X;
    const float* F[16];   // levels 1..L (packed)
    const float* fcw;
    const float* fcb;
    float* feat;          // [bs][f + L h]
    float* out;           // [bs][n_out]
};

// Two stages so a graph's rows (Σd² of them per level on SBM-200: 261 K) are summed by many blocks:
// part[b][k][col] over row chunk k of graph b (fp64, fixed order), then one block per graph adds
// the chunks and applies fc.  Chunks per graph (gridDim.y of the first stage) from the rows per graph:
// up to RO_CH for SBM-200-size levels, one for QM9-size graphs (a few hundred rows).
constexpr int RO_CH = 32;
int ro_chunks(long long rows, int bs) {
    const long long per = bs > 0 ? rows / bs : rows;
    const long long c = per / 4096 + 1;
    return (int)(c < RO_CH ? c : RO_CH);
}

__global__ void __launch_bounds__(256) k_ccn_readout_part(ReadoutArgs r, double* __restrict__ part) {
    __shared__ double red[4][C2_CMAX];
    const int b = blockIdx.x, k = blockIdx.y;
    const int n0 = r.v.node_off[b], n1 = r.v.node_off[b + 1];
    const int* off = r.order == 1 ? r.v.off1 : r.v.off2;
    const int nf = r.f + r.L * r.h;
    const int nch = gridDim.y;
    double* pb = part + ((long long)b * nch + k) * nf;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    auto flush = [&](double (&acc)[C2_CMAX], int nc, int col0) {
        for (int c = 0; c < nc; ++c) {
            const double t = wave_sum_d(acc[c]);
            if (lane == 0) red[wv][c] = t;
        }
        __syncthreads();
        if ((int)threadIdx.x < nc)
            pb[col0 + threadIdx.x] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] +
                                     red[3][threadIdx.x];
        __syncthreads();
    };
    // level 0: sum_i d_i^order X[i]  (utils_ccn.py:212-216 / 167-172 tile X[i] d_i or d_i^2 times)
    for (int c0 = 0; c0 < r.f; c0 += C2_CMAX) {
        const int nc = min(C2_CMAX, r.f - c0);
        double acc[C2_CMAX];
        for (int c = 0; c < C2_CMAX; ++c) acc[c] = 0.0;
        const int len = n1 - n0, per = (len + nch - 1) / nch;
        const int i0 = n0 + k * per, i1 = min(n1, i0 + per);
        for (int i = i0 + (int)threadIdx.x; i < i1; i += 256) {
            const double d = r.v.deg[i];
            const double wgt = r.order == 1 ? d : d * d;
            for (int c = 0; c < nc; ++c) acc[c] += wgt * (double)r.X[(long long)i * r.f + c0 + c];
        }
        flush(acc, nc, c0);
    }
    for (int l = 0; l < r.L; ++l) {
        const long long r0 = r.per_node ? n0 : off[n0], r1 = r.per_node ? n1 : off[n1];
        const long long len = r1 - r0, per = (len + nch - 1) / nch;
        const long long q0 = r0 + k * per, q1 = min(r1, q0 + per);
        for (int c0 = 0; c0 < r.h; c0 += C2_CMAX) {
            const int nc = min(C2_CMAX, r.h - c0);
            double acc[C2_CMAX];
            for (int c = 0; c < C2_CMAX; ++c) acc[c] = 0.0;
            for (long long q = q0 + threadIdx.x; q < q1; q += 256)
                for (int c = 0; c < nc; ++c) acc[c] += (double)r.F[l][q * r.h + c0 + c];
            flush(acc, nc, r.f + l * r.h + c0);
        }
    }
}

__global__ void __launch_bounds__(256) k_ccn_readout(ReadoutArgs r, const double* __restrict__ part) {
    __shared__ double red[4];
    const int b = blockIdx.x;
    const int nf = r.f + r.L * r.h;
    float* feat = r.feat + (long long)b * nf;
    auto bsum = [&](double x) {
        x = wave_sum_d(x);
        __syncthreads();
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = x;
        __syncthreads();
        return red[0] + red[1] + red[2] + red[3];
    };
    for (int col = threadIdx.x; col < nf; col += 256) {
        double t = 0.0;
        for (int k = 0; k < r.nch; ++k) t += part[((long long)b * r.nch + k) * nf + col];
        feat[col] = (float)t;
    }
    __syncthreads();
    for (int o = 0; o < r.n_out; ++o) {
        double s = 0.0;
        for (int k = threadIdx.x; k < nf; k += 256) s += (double)r.fcw[o * nf + k] * (double)feat[k];
        const double t = bsum(s);
        if (threadIdx.x == 0) r.out[(long long)b * r.n_out + o] = (float)(t + (double)r.fcb[o]);
    }
}

// dsum[b][k] = sum_o dout[b][o] fcw[o][k] (blocks [0, nd)); dfcw[o][k], dfcb[o] summed over the graphs in
// fp64, one wave per output (the remaining blocks; was one block doing all of it serially)
__global__ void __launch_bounds__(256) k_ccn_readout_bwd(const float* __restrict__ dout, const float* __restrict__ feat,
                                                         const float* __restrict__ fcw, int bs, int n_out, int nf,
                                                         float* __restrict__ dsum, float* __restrict__ dfcw,
                                                         float* __restrict__ dfcb) {
    const int nd = (bs * nf + 255) / 256;
    if ((int)blockIdx.x < nd) {
        const int e = blockIdx.x * 256 + threadIdx.x;
        if (e < bs * nf) {
            const int b = e / nf, k = e % nf;
            float s = 0.f;
            for (int o = 0; o < n_out; ++o) s = fmaf(dout[b * n_out + o], fcw[o * nf + k], s);
            dsum[e] = s;
        }
        return;
    }
    const int w = ((int)blockIdx.x - nd) * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (w >= n_out * nf + n_out) return;
    double s = 0.0;
    if (w < n_out * nf) {
        const int o = w / nf, k = w % nf;
        for (int b = lane; b < bs; b += 64) s += (double)dout[b * n_out + o] * (double)feat[(long long)b * nf + k];
    } else {
        const int o = w - n_out * nf;
        for (int b = lane; b < bs; b += 64) s += (double)dout[b * n_out + o];
    }
    s = wave_sum_d(s);
    if (lane == 0) {
        if (w < n_out * nf) dfcw[w] = (float)s;
        else dfcb[w - n_out * nf] = (float)s;
    }
}

// sum the per-node parameter partials: out[k] = sum_i part[i][k]  (k < kw: weight, then bias)
__global__ void __launch_bounds__(256) k_ccn_param_reduce(const float* __restrict__ part, const int* total_nodes,
                                                          int kw, int kb, float* __restrict__ dw, float* __restrict__ db) {
    __shared__ double red[4];
    const int k = blockIdx.x;
    const int n = *total_nodes;
    const int stride = kw + kb;
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) s += (double)part[(long long)i * stride + k];
    s = wave_sum_d(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double t = red[0] + red[1] + red[2] + red[3];
        if (k < kw) dw[k] = (float)t;
        else db[k - kw] = (float)t;
    }
}

// dF[row][c] = dsum[graph][off + c] for every feature row of the node (top level)
__global__ void k_ccn_bcast(CcnPlanView v, const int* total_nodes, int order, const float* __restrict__ dsum, int ld,
                            int off, int h, float* __restrict__ dF) {
    const int i = blockIdx.x;
    if (i >= *total_nodes) return;
    const int g = v.graph[i];
    const long long r0 = order == 1 ? v.off1[i] : v.off2[i];
    const long long r1 = order == 1 ? v.off1[i + 1] : v.off2[i + 1];
    for (long long q = r0 * h + threadIdx.x; q < r1 * h; q += blockDim.x) dF[q] = dsum[(long long)g * ld + off + (int)(q % h)];
}

// X (bs, nmax, f) padded -> packed [nodes][f]; and the inverse for dX (zero padding)
__global__ void k_ccn_pack_x(const float* __restrict__ X, const int* node_off, int nmax, int f, float* __restrict__ Xp) {
    const int b = blockIdx.x;
    const int n0 = node_off[b], nb = node_off[b + 1] - n0;
    for (int e = threadIdx.x; e < nb * f; e += blockDim.x) Xp[(long long)n0 * f + e] = X[(long long)b * nmax * f + e];
}

__global__ void k_ccn_unpack_dx(const float* __restrict__ dXp, const int* node_off, int nmax, int f,
                                float* __restrict__ dX) {
    const int b = blockIdx.x;
    const int n0 = node_off[b], nb = node_off[b + 1] - n0;
    for (int e = threadIdx.x; e < nmax * f; e += blockDim.x)
        dX[(long long)b * nmax * f + e] = e < nb * f ? dXp[(long long)n0 * f + e] : 0.f;
}

// collapse6to3 on a general F (C, n, n, n, n, n): out[x][y][q*C + ch]
// (functions/contraction.py: _c6to2_111 44-61, _c6to2_12 64-85, _c6to2_3 88-103)
__global__ void k_collapse6to3(const float* __restrict__ F, float* __restrict__ out, int C, int n) {
    const long long tot = (long long)n * n * 18 * C;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= tot) return;
    const int ch = (int)(idx % C), q = (int)((idx / C) % 18);
    const int y = (int)((idx / (18LL * C)) % n), x = (int)(idx / (18LL * C * n));
    auto G = [&](int a, int b, int c, int d, int e) {
        return F[(((((long long)ch * n + a) * n + b) * n + c) * n + d) * n + e];
    };
    float s = 0.f;
    if (q == 0) {
        for (int c = 0; c < n; ++c) for (int d = 0; d < n; ++d) for (int e = 0; e < n; ++e) s += G(x, y, c, d, e);
    } else if (q == 1) {
        for (int b = 0; b < n; ++b) for (int c = 0; c < n; ++c) for (int e = 0; e < n; ++e) s += G(x, b, c, y, e);
    } else if (q == 2) {
        for (int a = 0; a < n; ++a) for (int d = 0; d < n; ++d) for (int e = 0; e < n; ++e) s += G(a, x, y, d, e);
    } else if (q == 3) {
        for (int a = 0; a < n; ++a) for (int c = 0; c < n; ++c) for (int e = 0; e < n; ++e) s += G(a, x, c, y, e);
    } else if (q == 4) {
        for (int a = 0; a < n; ++a) for (int b = 0; b < n; ++b) for (int c = 0; c < n; ++c) s += G(a, b, c, x, y);
    } else if (q == 5) {
        for (int e = 0; e < n; ++e) for (int c = 0; c < n; ++c) s += G(x, y, c, c, e);
    } else if (q < 15) {
        for (int c = 0; c < n; ++c) for (int d = 0; d < n; ++d) s += G(x, y, c, d, d);
    } else if (q == 15) {
        for (int b = 0; b < n; ++b) s += G(x, b, b, y, b);
    } else if (q == 16) {
        for (int a = 0; a < n; ++a) s += G(a, x, a, y, a);
    } else {
        for (int a = 0; a < n; ++a) s += G(a, a, a, x, y);
    }
    out[idx] = s;
}

// adjoint of k_collapse6to3: dF[ch][a][b][c][d][e] from dOut[x][y][q*C + ch]
__global__ void k_collapse6to3_bwd(const float* __restrict__ dO, float* __restrict__ dF, int C, int n) {
    const long long tot = (long long)C * n * n * n * n * n;
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= tot) return;
    long long t = idx;
    const int e = (int)(t % n); t /= n;
    const int d = (int)(t % n); t /= n;
    const int c = (int)(t % n); t /= n;
    const int b = (int)(t % n); t /= n;
    const int a = (int)(t % n); t /= n;
    const int ch = (int)t;
    auto g = [&](int x, int y, int q) { return dO[((long long)x * n + y) * 18 * C + q * C + ch]; };
    float s = g(a, b, 0) + g(a, d, 1) + g(b, c, 2) + g(b, d, 3) + g(d, e, 4);
    if (c == d) s += g(a, b, 5);
    if (d == e)
        for (int q = 6; q < 15; ++q) s += g(a, b, q);
    if (b == c && c == e) s += g(a, d, 15);
    if (a == c && c == e) s += g(b, d, 16);
    if (a == b && b == c) s += g(d, e, 17);
    dF[idx] = s;
}

// ------------------------------------------------------------------ executor
struct CcnLayout {
    size_t node_off, deg, nbr, selfpos, graph, off1, off2, totals, err, bits, bcnt, pos;
    size_t plan_bytes;
    // feature workspace (needs sums)
    std::vector<size_t> F, coll, nsum;  // per level 1..L
    std::vector<C2Save> dummy;
    size_t sc[16], sa[16], d1[16], d2[16], q1[16], q3[16], tot[16], d3[16];
    size_t feat, rpart, g0, dsum, ppart, dF[2], dcoll, g_sc, g_sa, g_d1, g_d2, g_d3, xp, dxp, rdp, trd;
    size_t bytes;
};

size_t al(size_t x) { return (x + 255) / 256 * 256; }

bool ccn_ok(const hgnn_ccn_config* c) {
    return c && (c->order == 1 || c->order == 2) && c->bs > 0 && c->nmax > 0 && c->f_in > 0 && c->hidden > 0 &&
           c->layers >= 1 && c->layers <= 15 && c->n_out > 0 &&
           (c->order == 1 || (c->f_in <= C2_CMAX_WIDE && c->hidden <= C2_CMAX_WIDE && c->hidden <= C2_HMAX_WIDE));
}

CcnLayout ccn_layout(const hgnn_ccn_config* c, long long sum_d, long long sum_d2) {
    CcnLayout L{};
    const long long nodes = (long long)c->bs * c->nmax;
    size_t t = 0;
    auto take = [&](size_t n) {
        const size_t o = t;
        t += al(n);
        return o;
    };
    L.node_off = take(4 * (c->bs + 1));
    L.deg = take(4 * nodes);
    L.nbr = take(4 * nodes * c->nmax);
    L.selfpos = take(4 * nodes);
    L.graph = take(4 * nodes);
    L.off1 = take(4 * (nodes + 1));
    L.off2 = take(4 * (nodes + 1));
    L.totals = take(32);
    L.err = take(16);
    const int nw = (c->nmax + 63) / 64;
    L.bits = take(8 * nodes * nw);
    L.bcnt = take(4 * nodes * nw);
    L.pos = take(4 * (size_t)(sum_d2 > 0 ? sum_d2 : 1));
    L.plan_bytes = t;
    const long long rows = c->order == 1 ? sum_d : sum_d2;
    const int Lv = c->layers;
    const int h = c->hidden, f = c->f_in;
    L.F.resize(Lv);
    L.coll.resize(Lv);
    L.nsum.resize(Lv);
    int cmax = f > h ? f : h;
    const bool big = c->order == 2 && c->nmax > CCN_MAXD;  // degrees above 64 possible
    for (int l = 0; l < Lv; ++l) {
        const int cin = l == 0 ? f : h;
        L.F[l] = take(4 * (size_t)rows * h);
        if (c->order == 2) L.nsum[l] = take(4 * (size_t)nodes * h);
        if (c->order == 1) {
            L.coll[l] = take(4 * (size_t)rows * 2 * cin);
        } else if (big) {  // C2Save: only the large-degree kernels keep contraction statistics
            L.sc[l] = take(4 * (size_t)sum_d2 * cin);
            L.sa[l] = take(4 * (size_t)sum_d2 * cin);
            L.d1[l] = take(4 * (size_t)sum_d2 * cin);
            L.d2[l] = take(4 * (size_t)sum_d2 * cin);
            L.q1[l] = take(4 * (size_t)sum_d * cin);
            L.q3[l] = take(4 * (size_t)sum_d * cin);
            L.tot[l] = take(4 * (size_t)nodes * cin);
            L.d3[l] = take(4 * (size_t)nodes * cin);
        }
    }
    const int nf = f + Lv * h;
    L.feat = take(4 * (size_t)c->bs * nf);
    L.rpart = take(8 * (size_t)c->bs * RO_CH * nf);
    L.g0 = take(4 * (size_t)(sum_d > 0 ? sum_d : 1) * c->f_in);
    L.dsum = take(4 * (size_t)c->bs * nf);
    const int kmax = (c->order == 1 ? 2 : 18) * cmax;
    L.ppart = take(4 * (size_t)nodes * (h * kmax + h));
    L.dF[0] = take(4 * (size_t)rows * cmax);
    L.dF[1] = take(4 * (size_t)rows * cmax);
    if (c->order == 1) {
        L.dcoll = take(4 * (size_t)rows * 2 * cmax);
    } else {
        L.rdp = take(4 * (size_t)(sum_d > 0 ? sum_d : 1) * h);  // dp format: row sums and trace of dp
        L.trd = take(4 * (size_t)nodes * h);
        if (big) {  // C2Grad of the large-degree backward node pass
            L.g_sc = take(4 * (size_t)sum_d2 * cmax);
            L.g_sa = take(4 * (size_t)sum_d2 * cmax);
            L.g_d1 = take(4 * (size_t)sum_d2 * cmax);
            L.g_d2 = take(4 * (size_t)sum_d2 * cmax);
            L.g_d3 = take(4 * (size_t)nodes * cmax);
        }
    }
    L.xp = take(4 * (size_t)nodes * f);
    L.dxp = take(4 * (size_t)nodes * f);
    L.bytes = t;
    return L;
}

template <typename T>
T* P(void* base, size_t off) {
    return reinterpret_cast<T*>(static_cast<char*>(base) + off);
}

CcnPlanView plan_view(const hgnn_ccn_config* c, const CcnLayout& L, void* ws) {
    CcnPlanView v;
    v.node_off = P<int>(ws, L.node_off);
    v.deg = P<int>(ws, L.deg);
    v.nbr = P<int>(ws, L.nbr);
    v.selfpos = P<int>(ws, L.selfpos);
    v.graph = P<int>(ws, L.graph);
    v.off1 = P<int>(ws, L.off1);
    v.off2 = P<int>(ws, L.off2);
    v.pos = P<int>(ws, L.pos);
    v.nmax = c->nmax;
    return v;
}

C2Save save_of(const CcnLayout& L, void* ws, int l) {
    C2Save s;
    s.Sc = P<float>(ws, L.sc[l]);
    s.Sa = P<float>(ws, L.sa[l]);
    s.D1 = P<float>(ws, L.d1[l]);
    s.D2 = P<float>(ws, L.d2[l]);
    s.q1 = P<float>(ws, L.q1[l]);
    s.q3 = P<float>(ws, L.q3[l]);
    s.tot = P<float>(ws, L.tot[l]);
    s.d3 = P<float>(ws, L.d3[l]);
    return s;
}

// The CCN-2D kernels of degrees <= 64 take the receptive-field bound ncap = min(max degree, 64) for their
// dynamic LDS (P or dp [ncap^2][HC] fp32 + the int16 position map): 40 KB at ncap = 64.
// Instantiations by channel count: cin <= 2 (the reference's hidden_size = 2 levels), <= 8, <= 16.
int c2_ncap(long long dmax) { return dmax < C2_NCAP ? (int)(dmax > 1 ? dmax : 1) : C2_NCAP; }

template <int CM, int HC, int NB, bool L0>
int launch_c2_fwd_t(const CcnPlanView& v, const int* tot, const float* fin, const float* X, int cin, const float* W,
                    const float* b, int h, int ncap, int nodes, float* fout, float* nsum, hipStream_t s) {
    const size_t lds = c2_dyn_lds(ncap, HC);
    HGNN_KLAUNCH((k_c2_fwd<CM, HC, NB, L0>), dim3(nodes > 0 ? nodes : 1), dim3(256), lds, s, v, tot, fin, X, cin,
                       W, b, h, ncap, fout, nsum);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int launch_c2_fwd(const CcnPlanView& v, const int* tot, const float* fin, int level0, const float* X, int cin,
                  const float* W, const float* b, int h, long long dmax, int nodes, float* fout, float* nsum,
                  hipStream_t s) {
    const int ncap = c2_ncap(dmax);
    if (level0) {
        if (cin <= 8) return launch_c2_fwd_t<8, 2, 1, true>(v, tot, fin, X, cin, W, b, h, ncap, nodes, fout, nsum, s);
        return launch_c2_fwd_t<16, 2, 1, true>(v, tot, fin, X, cin, W, b, h, ncap, nodes, fout, nsum, s);
    }
    if (cin <= 2) return launch_c2_fwd_t<2, 2, 8, false>(v, tot, fin, X, cin, W, b, h, ncap, nodes, fout, nsum, s);
    if (cin <= 8) return launch_c2_fwd_t<8, 2, 4, false>(v, tot, fin, X, cin, W, b, h, ncap, nodes, fout, nsum, s);
    return launch_c2_fwd_t<16, 2, 2, false>(v, tot, fin, X, cin, W, b, h, ncap, nodes, fout, nsum, s);
}

template <int CM, int HC, int NB, bool L0>
int launch_c2_bwd_t(const CcnPlanView& v, const int* tot, float* dF, const float* dtop, int dtop_ld, const float* F,
                    const float* fin, const float* X, int cin, const float* W, int h, int ncap, int nodes, float* rdp,
                    float* trd, float* ppart, float* g0, hipStream_t s) {
    const size_t lds = c2_dyn_lds(ncap, HC);
    HGNN_KLAUNCH((k_c2_bwd<CM, HC, NB, L0>), dim3(nodes > 0 ? nodes : 1), dim3(256), lds, s, v, tot, dF, dtop,
                       dtop_ld, F, fin, X, cin, W, h, ncap, rdp, trd, ppart, g0);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int launch_c2_bwd(const CcnPlanView& v, const int* tot, float* dF, const float* dtop, int dtop_ld, const float* F,
                  const float* fin, int level0,
                  const float* X, int cin, const float* W, int h, long long dmax, int nodes, float* rdp, float* trd,
                  float* ppart, float* g0, hipStream_t s) {
    const int ncap = c2_ncap(dmax);
    if (level0) {
        if (cin <= 8)
            return launch_c2_bwd_t<8, 2, 1, true>(v, tot, dF, dtop, dtop_ld, F, fin, X, cin, W, h, ncap, nodes, rdp, trd, ppart, g0, s);
        return launch_c2_bwd_t<16, 2, 1, true>(v, tot, dF, dtop, dtop_ld, F, fin, X, cin, W, h, ncap, nodes, rdp, trd, ppart, g0, s);
    }
    if (cin <= 2)
        return launch_c2_bwd_t<2, 2, 8, false>(v, tot, dF, dtop, dtop_ld, F, fin, X, cin, W, h, ncap, nodes, rdp, trd, ppart, g0, s);
    if (cin <= 8)
        return launch_c2_bwd_t<8, 2, 4, false>(v, tot, dF, dtop, dtop_ld, F, fin, X, cin, W, h, ncap, nodes, rdp, trd, ppart, g0, s);
    return launch_c2_bwd_t<16, 1, 2, false>(v, tot, dF, dtop, dtop_ld, F, fin, X, cin, W, h, ncap, nodes, rdp, trd, ppart, g0, s);
}

int launch_c2_gather(const CcnPlanView& v, const int* tot, const C2Dp& g, const float* W, int h, const float* dsum,
                     int dsum_ld, int dsum_off, long long dmax, int nodes, float* dout, hipStream_t s) {
    const dim3 grid(nodes > 0 ? nodes : 1);
    if (h <= 2)
        HGNN_KLAUNCH((k_c2_gather<2, 8>), grid, dim3(256), 0, s, v, tot, g, W, h, dsum, dsum_ld, dsum_off, dout);
    else if (h <= 8)
        HGNN_KLAUNCH((k_c2_gather<8, 1>), grid, dim3(256), 0, s, v, tot, g, W, h, dsum, dsum_ld, dsum_off, dout);
    else
        HGNN_KLAUNCH((k_c2_gather<16, 1>), grid, dim3(256), 0, s, v, tot, g, W, h, dsum, dsum_ld, dsum_off, dout);
    HGNN_LAUNCH_CHECK();
    if (dmax > C2_NCAP) {
        if (h <= 2)
            HGNN_KLAUNCH((k_c2_gather_big<2, 4>), grid, dim3(256), 0, s, v, tot, g, W, h, dsum, dsum_ld,
                               dsum_off, dout);
        else if (h <= 8)
            HGNN_KLAUNCH((k_c2_gather_big<8, 1>), grid, dim3(256), 0, s, v, tot, g, W, h, dsum, dsum_ld,
                               dsum_off, dout);
        else
            HGNN_KLAUNCH((k_c2_gather_big<16, 1>), grid, dim3(256), 0, s, v, tot, g, W, h, dsum, dsum_ld,
                               dsum_off, dout);
        HGNN_LAUNCH_CHECK();
    }
    return HGNN_OK;
}

}  // namespace
}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_collapse6to3(const float* d_F, float* d_out, int c, int n, void* stream) {
    if (!d_F || !d_out || c <= 0 || n <= 0) return HGNN_ERR_ARG;
    const long long tot = (long long)n * n * 18 * c;
    HGNN_KLAUNCH(k_collapse6to3, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_F,
                       d_out, c, n);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int hgnn_collapse6to3_backward(const float* d_dout, float* d_dF, int c, int n, void* stream) {
    if (!d_dout || !d_dF || c <= 0 || n <= 0) return HGNN_ERR_ARG;
    const long long tot = (long long)c * n * n * n * n * n;
    HGNN_KLAUNCH(k_collapse6to3_bwd, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       d_dout, d_dF, c, n);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int hgnn_ccn_plan_offsets(const hgnn_ccn_config* cfg, long long max_sum_d2, size_t* offs) {
    if (!ccn_ok(cfg) || !offs) return HGNN_ERR_ARG;
    const CcnLayout L = ccn_layout(cfg, 0, max_sum_d2);
    const size_t o[9] = {L.node_off, L.deg, L.nbr, L.selfpos, L.graph, L.off1, L.off2, L.pos, L.err};
    for (int i = 0; i < 9; ++i) offs[i] = o[i];
    return HGNN_OK;
}

size_t hgnn_ccn_plan_bytes(const hgnn_ccn_config* cfg, long long max_sum_d2) {
    if (!ccn_ok(cfg)) return 0;
    return ccn_layout(cfg, 0, max_sum_d2).plan_bytes;
}

static int ccn_plan(const hgnn_ccn_config* cfg, const float* d_adj, const int64_t* d_n_batch, void* plan_ws,
                    long long max_sum_d2, long long* h_sums, hipStream_t s, bool sync) {
    if (!ccn_ok(cfg) || !d_adj || !d_n_batch || !plan_ws || !h_sums) return HGNN_ERR_ARG;
    const CcnLayout L = ccn_layout(cfg, 0, max_sum_d2);
    BatchMeta m;
    m.node_off = P<int>(plan_ws, L.node_off);
    m.edge_off = P<int>(plan_ws, L.off1);  // scratch, overwritten by the scan
    m.totals = P<int>(plan_ws, L.totals);
    m.err = P<uint32_t>(plan_ws, L.err);
    HGNN_HOST_CHECK(hipMemsetAsync(m.err, 0, 4, s));
    int r = launch_plan(d_n_batch, nullptr, cfg->bs, cfg->nmax, 0, m, s);
    if (r) return r;
    CcnPlanView v = plan_view(cfg, L, plan_ws);
    HGNN_KLAUNCH(k_ccn_nbrs, dim3(cfg->bs, (cfg->nmax + CCN_NB_ROWS - 1) / CCN_NB_ROWS), dim3(256), 0, s, d_adj,
                       cfg->nmax, v.node_off, P<int>(plan_ws, L.deg), P<int>(plan_ws, L.nbr),
                       P<int>(plan_ws, L.selfpos), P<int>(plan_ws, L.graph), P<unsigned long long>(plan_ws, L.bits),
                       P<int>(plan_ws, L.bcnt), m.err, cfg->order == 1 ? CCN1_MAXD : CCN_BIGD);
    HGNN_LAUNCH_CHECK();
    HGNN_KLAUNCH(k_ccn_scan, dim3(1), dim3(1024), 0, s, P<int>(plan_ws, L.deg), m.totals,
                       P<int>(plan_ws, L.off1), P<int>(plan_ws, L.off2), m.totals + 2);
    HGNN_LAUNCH_CHECK();
    long long nodes = (long long)cfg->bs * cfg->nmax;
    if (sync) {
        int hbuf[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        HGNN_HOST_CHECK(hipMemcpyAsync(hbuf, m.totals, 32, hipMemcpyDeviceToHost, s));
        HGNN_HOST_CHECK(hipStreamSynchronize(s));
        nodes = hbuf[0];
        h_sums[0] = hbuf[2];
        h_sums[1] = hbuf[3];
        h_sums[2] = nodes;
        h_sums[3] = hbuf[4];
        if (h_sums[1] > max_sum_d2) return HGNN_ERR_ARG;  // caller re-plans with a larger bound
    } else {
        // bounds, no host sync: every graph's d_i <= n_b <= nmax; the kernels read the device totals
        h_sums[0] = nodes * cfg->nmax;
        h_sums[1] = max_sum_d2;
        h_sums[2] = nodes;
        h_sums[3] = cfg->nmax;
    }
    HGNN_KLAUNCH(k_ccn_pos, dim3((unsigned)((nodes + 3) / 4 > 0 ? (nodes + 3) / 4 : 1)), dim3(256), 0, s, v,
                       m.totals, P<unsigned long long>(plan_ws, L.bits), P<int>(plan_ws, L.bcnt),
                       P<int>(plan_ws, L.pos), max_sum_d2, m.err);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int hgnn_ccn_plan(const hgnn_ccn_config* cfg, const float* d_adj, const int64_t* d_n_batch, void* plan_ws,
                  long long max_sum_d2, long long* h_sums, void* stream) {
    return ccn_plan(cfg, d_adj, d_n_batch, plan_ws, max_sum_d2, h_sums, (hipStream_t)stream, true);
}

int hgnn_ccn_plan_async(const hgnn_ccn_config* cfg, const float* d_adj, const int64_t* d_n_batch, void* plan_ws,
                        long long max_sum_d2, long long* h_sums_bound, void* stream) {
    // the bound must hold for any content, so no later kernel can meet an unplanned position map
    if (!cfg || max_sum_d2 < (long long)cfg->bs * cfg->nmax * cfg->nmax * cfg->nmax) return HGNN_ERR_ARG;
    return ccn_plan(cfg, d_adj, d_n_batch, plan_ws, max_sum_d2, h_sums_bound, (hipStream_t)stream, false);
}

uint32_t* hgnn_ccn_error_word(const hgnn_ccn_config* cfg, void* plan_ws, long long max_sum_d2) {
    if (!ccn_ok(cfg) || !plan_ws) return nullptr;
    return P<uint32_t>(plan_ws, ccn_layout(cfg, 0, max_sum_d2).err);
}

size_t hgnn_ccn_workspace_bytes(const hgnn_ccn_config* cfg, const long long* sums) {
    if (!ccn_ok(cfg) || !sums) return 0;
    const CcnLayout L = ccn_layout(cfg, sums[0], sums[1]);
    return L.bytes - L.plan_bytes;
}

static void* feat_ws(void* ws, const CcnLayout& L) { return static_cast<char*>(ws) - L.plan_bytes; }

int hgnn_ccn_forward(const hgnn_ccn_config* cfg, const long long* sums, const float* d_X, const float* const* params,
                     void* plan_ws, long long max_sum_d2, void* workspace, float* d_out, void* stream) {
    if (!ccn_ok(cfg) || !sums || !d_X || !params || !plan_ws || !workspace || !d_out) return HGNN_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    const CcnLayout Lp = ccn_layout(cfg, 0, max_sum_d2);
    const CcnLayout L = ccn_layout(cfg, sums[0], sums[1]);
    CcnPlanView v = plan_view(cfg, Lp, plan_ws);
    void* W = feat_ws(workspace, L);
    const int* tot = P<int>(plan_ws, Lp.totals);
    const int nodes = (int)sums[2];
    const int h = cfg->hidden, f = cfg->f_in;
    float* Xp = P<float>(W, L.xp);
    HGNN_KLAUNCH(k_ccn_pack_x, dim3(cfg->bs), dim3(256), 0, s, d_X, v.node_off, cfg->nmax, f, Xp);
    HGNN_LAUNCH_CHECK();
    d_X = Xp;
    for (int l = 0; l < cfg->layers; ++l) {
        const int cin = l == 0 ? f : h;
        const float* fin = l == 0 ? nullptr : P<float>(W, L.F[l - 1]);
        const float* w = params[2 * l];
        const float* b = params[2 * l + 1];
        if (cfg->order == 1) {
            HGNN_KLAUNCH(k_ccn1_fwd, dim3(nodes > 0 ? (nodes + 3) / 4 : 1), dim3(256), 0, s, v, tot, fin,
                               l == 0 ? 1 : 0, d_X, cin, w, b, h, P<float>(W, L.coll[l]), P<float>(W, L.F[l]));
        } else {
            const bool narrow = cin <= C2_CMAX && h <= C2_HMAX;
            const int r = launch_c2_fwd(v, tot, fin, l == 0 ? 1 : 0, d_X, cin, w, b, h, sums[3], nodes,
                                        P<float>(W, L.F[l]), P<float>(W, L.nsum[l]), s);
            if (r) return r;
            if (sums[3] > CCN_MAXD) {  // degrees 65..256 present (or possible): their nodes in the large-degree kernel
                if (narrow)
                    HGNN_KLAUNCH((k_ccn2_fwd_big<C2_CMAX, C2_HMAX>), dim3(nodes > 0 ? nodes : 1), dim3(256), 0, s,
                                       v, tot, fin, l == 0 ? 1 : 0, d_X, cin, w, b, h, save_of(L, W, l),
                                       P<float>(W, L.F[l]), P<float>(W, L.nsum[l]));
                else
                    HGNN_KLAUNCH((k_ccn2_fwd_big<C2_CMAX_WIDE, C2_HMAX_WIDE>), dim3(nodes > 0 ? nodes : 1),
                                       dim3(256), 0, s, v, tot, fin, l == 0 ? 1 : 0, d_X, cin, w, b, h,
                                       save_of(L, W, l), P<float>(W, L.F[l]), P<float>(W, L.nsum[l]));
            }
        }
        HGNN_LAUNCH_CHECK();
    }
    ReadoutArgs ra{};
    ra.v = v;
    ra.order = cfg->order;
    ra.L = cfg->layers;
    ra.f = f;
    ra.h = h;
    ra.n_out = cfg->n_out;
    ra.bs = cfg->bs;
    ra.X = d_X;
    ra.per_node = cfg->order == 2;  // CCN-2D: the forward kernels left each node's row sum
    for (int l = 0; l < cfg->layers; ++l) ra.F[l] = P<float>(W, cfg->order == 2 ? L.nsum[l] : L.F[l]);
    ra.fcw = params[2 * cfg->layers];
    ra.fcb = params[2 * cfg->layers + 1];
    ra.feat = P<float>(W, L.feat);
    ra.out = d_out;
    ra.nch = ro_chunks(cfg->order == 2 ? nodes : sums[0], cfg->bs);
    HGNN_KLAUNCH(k_ccn_readout_part, dim3(cfg->bs, ra.nch), dim3(256), 0, s, ra, P<double>(W, L.rpart));
    HGNN_LAUNCH_CHECK();
    HGNN_KLAUNCH(k_ccn_readout, dim3(cfg->bs), dim3(256), 0, s, ra, P<double>(W, L.rpart));
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int hgnn_ccn_backward(const hgnn_ccn_config* cfg, const long long* sums, const float* const* params, void* plan_ws,
                      long long max_sum_d2, void* workspace, const float* d_dout, float* const* grads, float* d_dX,
                      void* stream) {
    if (!ccn_ok(cfg) || !sums || !params || !plan_ws || !workspace || !d_dout || !grads || !d_dX) return HGNN_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    const CcnLayout Lp = ccn_layout(cfg, 0, max_sum_d2);
    const CcnLayout L = ccn_layout(cfg, sums[0], sums[1]);
    CcnPlanView v = plan_view(cfg, Lp, plan_ws);
    void* W = feat_ws(workspace, L);
    const int* tot = P<int>(plan_ws, Lp.totals);
    const int nodes = (int)sums[2];
    const int h = cfg->hidden, f = cfg->f_in, Lv = cfg->layers;
    const int nf = f + Lv * h;
    float* dsum = P<float>(W, L.dsum);
    HGNN_KLAUNCH(k_ccn_readout_bwd,
                       dim3((cfg->bs * nf + 255) / 256 + (cfg->n_out * nf + cfg->n_out + 3) / 4), dim3(256), 0, s,
                       d_dout, P<float>(W, L.feat), params[2 * Lv], cfg->bs, cfg->n_out, nf, dsum, grads[2 * Lv],
                       grads[2 * Lv + 1]);
    HGNN_LAUNCH_CHECK();
    const unsigned nb4 = nodes > 0 ? (unsigned)(nodes + 3) / 4 : 1u;
    const unsigned nb1 = nodes > 0 ? (unsigned)nodes : 1u;
    const long long rows = cfg->order == 1 ? sums[0] : sums[1];
    // dF of the top level = readout broadcast of its slice of dsum
    float* dF = P<float>(W, L.dF[0]);
    float* dFn = P<float>(W, L.dF[1]);
    // CCN-2D without large-degree nodes: the top level's backward reads the broadcast slice of dsum itself
    const bool bigd = cfg->order == 2 && sums[3] > CCN_MAXD;
    const bool top_direct = cfg->order == 2 && !bigd;
    if (!top_direct) {
        HGNN_KLAUNCH(k_ccn_bcast, dim3(nb1), dim3(64), 0, s, v, tot, cfg->order, dsum, nf, f + (Lv - 1) * h, h,
                           dF);
        HGNN_LAUNCH_CHECK();
    }
    for (int l = Lv - 1; l >= 0; --l) {
        const int cin = l == 0 ? f : h;
        const float* w = params[2 * l];
        const int K = (cfg->order == 1 ? 2 : 18) * cin;
        float* ppart = P<float>(W, L.ppart);
        if (cfg->order == 1) {
            HGNN_KLAUNCH(k_ccn1_bwd_node, dim3(nb4), dim3(256), 0, s, v, tot, dF, P<float>(W, L.F[l]),
                               P<float>(W, L.coll[l]), cin, w, h, P<float>(W, L.dcoll), ppart);
        } else {
            const bool narrow = cin <= C2_CMAX && h <= C2_HMAX;
            float* g0p = l == 0 ? P<float>(W, L.g0) : nullptr;
            const float* fin = l == 0 ? nullptr : P<float>(W, L.F[l - 1]);
            if (bigd) {  // the large-degree nodes read the raw dF: before the dp rewrite
                C2Grad gd{P<float>(W, L.g_sc), P<float>(W, L.g_sa), P<float>(W, L.g_d1), P<float>(W, L.g_d2),
                          P<float>(W, L.g_d3)};
                if (narrow)
                    HGNN_KLAUNCH((k_ccn2_bwd_node_big<C2_CMAX, C2_HMAX>), dim3(nb1), dim3(256), 0, s, v, tot, dF,
                                       P<float>(W, L.F[l]), save_of(L, W, l), cin, w, h, gd, ppart, g0p);
                else
                    HGNN_KLAUNCH((k_ccn2_bwd_node_big<C2_CMAX_WIDE, C2_HMAX_WIDE>), dim3(nb1), dim3(256), 0, s, v,
                                       tot, dF, P<float>(W, L.F[l]), save_of(L, W, l), cin, w, h, gd, ppart, g0p);
                HGNN_LAUNCH_CHECK();
                HGNN_KLAUNCH(k_c2_dp_big, dim3(nb1), dim3(256), 0, s, v, tot, dF, P<float>(W, L.F[l]), h,
                                   P<float>(W, L.rdp), P<float>(W, L.trd));
                HGNN_LAUNCH_CHECK();
            }
            const float* dtop = top_direct && l == Lv - 1 ? dsum + f + (Lv - 1) * h : nullptr;
            const int r = launch_c2_bwd(v, tot, dF, dtop, nf, P<float>(W, L.F[l]), fin, l == 0 ? 1 : 0,
                                        P<float>(W, L.xp), cin, w, h, sums[3], nodes, P<float>(W, L.rdp),
                                        P<float>(W, L.trd), ppart, g0p, s);
            if (r) return r;
        }
        HGNN_LAUNCH_CHECK();
        HGNN_KLAUNCH(k_ccn_param_reduce, dim3(h * K + h), dim3(256), 0, s, ppart, tot, h * K, h, grads[2 * l],
                           grads[2 * l + 1]);
        HGNN_LAUNCH_CHECK();
        const int lvl0 = l == 0 ? 1 : 0;
        float* dst = lvl0 ? P<float>(W, L.dxp) : dFn;
        const int doff = lvl0 ? 0 : f + (l - 1) * h;
        if (cfg->order == 1) {
            HGNN_KLAUNCH(k_ccn1_bwd_gather, dim3(nb4), dim3(256), 0, s, v, tot, P<float>(W, L.dcoll), cin, dsum,
                               nf, doff, lvl0, dst);
        } else {
            if (lvl0) {
                HGNN_KLAUNCH(k_ccn2_dx0, dim3(nb4), dim3(256), 0, s, v, tot, P<float>(W, L.g0), cin, dsum, nf,
                                   dst);
            } else {
                const C2Dp g{dF, P<float>(W, L.rdp), P<float>(W, L.trd)};
                const int r = launch_c2_gather(v, tot, g, w, h, dsum, nf, doff, sums[3], nodes, dst, s);
                if (r) return r;
            }
        }
        HGNN_LAUNCH_CHECK();
        float* t = dF;
        dF = dFn;
        dFn = t;
    }
    (void)rows;
    HGNN_KLAUNCH(k_ccn_unpack_dx, dim3(cfg->bs), dim3(256), 0, s, P<float>(W, L.dxp), v.node_off, cfg->nmax, f,
                       d_dX);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

}  // extern "C"
