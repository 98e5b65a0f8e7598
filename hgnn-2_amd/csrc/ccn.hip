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

#include "kernels.h"

namespace hgnn {
namespace {

constexpr int CCN_MAXD = 64;     // CCN-2D fast-path degree bound (one wave per receptive-field row, 64-bit ballots)
constexpr int CCN_BIGD = 256;    // CCN-2D degree bound: degrees 65..256 take the _big kernels (rows in 64-lane
                                 // chunks, membership as 4 x 64-bit words, position maps read from L2)
constexpr int CCN_BW = CCN_BIGD / 64;

// bit x of a multi-word set (CCN-2D common neighbourhoods of the large-degree kernels)
__device__ __forceinline__ bool mbit(const unsigned long long* m, int x) { return (m[x >> 6] >> (x & 63)) & 1ull; }
constexpr int CCN1_MAXD = 1024;  // CCN-1D degree bound (rows walked in 64-lane chunks; per-wave LDS row sums)

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
__global__ void __launch_bounds__(256) k_ccn_nbrs(const float* __restrict__ adj, int nmax, const int* node_off,
                                                  int* deg, int* nbr, int* selfpos, int* graph, uint32_t* err,
                                                  int maxd) {
    const int b = blockIdx.x;
    const int n0 = node_off[b];
    const int nb = node_off[b + 1] - n0;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const float* A = adj + (long long)b * nmax * nmax;
    for (int r = wv; r < nb; r += 4) {
        const int gi = n0 + r;
        int cnt = 0, sp = -1;
        for (int c0 = 0; c0 < nb; c0 += 64) {
            const int c = c0 + lane;
            const bool nz = c < nb && A[(long long)r * nmax + c] > 0.f;   // utils_ccn.py:195 (A > 0)
            // the gather-form backward walks N(j) for the readers of F_j: needs a symmetric pattern
            if (c < nb && nz != (A[(long long)c * nmax + r] > 0.f)) atomicOr(err, (uint32_t)ERR_CCN_ASYM);
            const unsigned long long m = __ballot(nz);
            const int p = __popcll(m & ((1ull << lane) - 1ull));
            if (nz) {
                nbr[(long long)gi * nmax + cnt + p] = n0 + c;
                if (c == r) sp = cnt + p;
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

// exclusive scans of deg and deg^2 over all nodes (single block); totals[0..1]
__global__ void __launch_bounds__(256) k_ccn_scan(const int* deg, const int* total_nodes, int* off1, int* off2,
                                                  int* totals) {
    __shared__ int s1[256], s2[256], carry[2];
    const int t = threadIdx.x;
    const int n = *total_nodes;
    if (t == 0) carry[0] = carry[1] = 0;
    __syncthreads();
    for (int base = 0; base < n; base += 256) {
        const int i = base + t;
        const int d = i < n ? deg[i] : 0;
        s1[t] = d;
        s2[t] = d * d;
        __syncthreads();
        for (int o = 1; o < 256; o <<= 1) {
            const int a1 = t >= o ? s1[t - o] : 0, a2 = t >= o ? s2[t - o] : 0;
            __syncthreads();
            s1[t] += a1;
            s2[t] += a2;
            __syncthreads();
        }
        if (i < n) {
            off1[i] = carry[0] + s1[t] - d;
            off2[i] = carry[1] + s2[t] - d * d;
        }
        __syncthreads();
        if (t == 255) {
            carry[0] += s1[255];
            carry[1] += s2[255];
        }
        __syncthreads();
    }
    if (t == 0) {
        off1[n] = carry[0];
        off2[n] = carry[1];
        totals[0] = carry[0];
        totals[1] = carry[1];
    }
}

// pos[off2[i] + a*d_i + x] = index of nbr_i[x] in nbr_{nbr_i[a]} (binary search), or -1
__global__ void __launch_bounds__(256) k_ccn_pos(CcnPlanView v, const int* total_nodes, int* pos, long long pos_cap,
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
    const int* ni = v.nbr + (long long)i * v.nmax;
    for (int x0 = 0; x0 < n; x0 += 64) {
        const int x = x0 + lane;
        const int me = x < n ? ni[x] : -1;
        for (int a = 0; a < n; ++a) {
            const int j = ni[a];
            const int dj = v.deg[j];
            const int* nj = v.nbr + (long long)j * v.nmax;
            int p = -1;
            if (x < n) {
                int lo = 0, hi = dj - 1;
                while (lo <= hi) {
                    const int mid = (lo + hi) >> 1;
                    const int val = nj[mid];
                    if (val == me) {
                        p = mid;
                        break;
                    }
                    if (val < me) lo = mid + 1;
                    else hi = mid - 1;
                }
                pos[v.off2[i] + (long long)a * n + x] = p;
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

// Block per node i (n = d_i).  T[a][b][z] = F_{j_a}[p_a(b)][p_a(z)] is nonzero only where both
// positions exist, i.e. b, z in the common neighbourhood C_a = N(i) n N(j_a) (|C_a| = m_a, 10.9 on
// average on SBM-200 against d = 36), so the contraction statistics are gathered over C_a x C_a
// only: sum_a m_a^2 instead of d^3 (9x less on config 5).  Zero terms are skipped, not added, so
// the sums are those of the dense loops.  Two wave-parallel passes, no atomics (deterministic):
//   pass A, wave per a, lane b:  Sc[a][b] = sum_{z in C_a} T, D1[a][b] = T[a][b][b],
//           D2[a][b] = T[a][b][a], q1[a] = sum_b Sc (wave sum), d3 += T[a][a][a]
//   pass B, wave per b, lane z:  Sa[b][z] = sum_{a: b in C_a} T, q3[b] = sum_z Sa (wave sum)
// The validity of the loop index (z in pass A, a in pass B) is wave-uniform, so each wave walks
// the set bits of a ballot.  Level 0 (F_0[j] = X[j] tiled, utils_ccn.py:167-172) needs no gather.
constexpr int C2_CMAX = 8;  // channels of a CCN-2D level (f_in or hidden) handled per pass (narrow kernels)
constexpr int C2_HMAX = 8;  // hidden size bound of the fused output stage (narrow kernels)
constexpr int C2_CMAX_WIDE = 16;  // the wide instantiations: f_in, hidden <= 16
constexpr int C2_HMAX_WIDE = 16;

template <int CM, int HM>
__global__ void __launch_bounds__(256) k_ccn2_fwd(CcnPlanView v, const int* total_nodes, const float* __restrict__ fin,
                                                  int level0, const float* __restrict__ X, int cin,
                                                  const float* __restrict__ W, const float* __restrict__ bias, int h,
                                                  C2Save sv, float* __restrict__ fout) {
    __shared__ int sp[CCN_MAXD * CCN_MAXD];
    __shared__ unsigned long long vmask[CCN_MAXD];  // bit x of vmask[a]: x in C_a
    __shared__ float sred[2][4][CM];           // per-wave partial q1-total and d3
    __shared__ int s_j[CCN_MAXD], s_dj[CCN_MAXD], s_oj[CCN_MAXD];  // neighbour a: node, degree, 2D row offset
    const int i = blockIdx.x;
    if (i >= *total_nodes) return;
    const int n = v.deg[i];
    if (n > CCN_MAXD || cin > CM || h > HM) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int* ni = v.nbr + (long long)i * v.nmax;
    const long long o2 = v.off2[i], o1 = v.off1[i];
    for (int e = threadIdx.x; e < n * n; e += 256) sp[e] = v.pos[o2 + e];
    if (threadIdx.x < n) {
        const int j = ni[threadIdx.x];
        s_j[threadIdx.x] = j;
        s_dj[threadIdx.x] = v.deg[j];
        s_oj[threadIdx.x] = v.off2[j];
    }
    __syncthreads();
    for (int a = wv; a < n; a += 4) {
        const unsigned long long m = __ballot(lane < n && sp[a * n + lane] >= 0);
        if (lane == 0) vmask[a] = m;
    }
    __syncthreads();

    // ---- pass A: wave per neighbour a, lane b
    float tq[CM], td3[CM];
#pragma unroll
    for (int c = 0; c < CM; ++c) tq[c] = td3[c] = 0.f;
    for (int a = wv; a < n; a += 4) {
        const int j = ni[a];
        const unsigned long long ma = vmask[a];
        const int pb = lane < n ? sp[a * n + lane] : -1;
        const bool vb = pb >= 0;
        float sc[CM], d1[CM], d2[CM];
#pragma unroll
        for (int c = 0; c < CM; ++c) sc[c] = d1[c] = d2[c] = 0.f;
        if (level0) {
            const float mf = (float)__popcll(ma);
            const bool va = (ma >> a) & 1ull;
#pragma unroll
            for (int c = 0; c < CM; ++c) {
                if (c >= cin) break;
                const float xj = X[(long long)j * cin + c];
                sc[c] = vb ? mf * xj : 0.f;
                d1[c] = vb ? xj : 0.f;
                d2[c] = (vb && va) ? xj : 0.f;
            }
        } else {
            const int dj = s_dj[a];
            const float* row = fin + ((long long)s_oj[a] + (long long)(vb ? pb : 0) * dj) * cin;
            // the common neighbours z (wave-uniform) in batches of 4: all loads of a batch in flight
            // before any is used (a one-at-a-time walk paid one memory latency per z); same order of
            // summation
            unsigned long long zs = ma;
            while (zs) {
                int zz[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    zz[u] = zs ? __ffsll((long long)zs) - 1 : -1;
                    zs &= zs ? zs - 1ull : 0ull;
                }
                float t[4][CM];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int pz = zz[u] >= 0 ? sp[a * n + zz[u]] : 0;  // valid row: loads need no mask
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
                            if (z == lane) d1[c] = t[u][c];
                            if (z == a) d2[c] = t[u][c];
                        }
                    }
                }
            }
        }
        if (lane < n) {
            const long long r = (o2 + (long long)a * n + lane) * cin;
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
            const float q = wave_sum(sc[c]);           // q1[a] = sum_b Sc[a][b]
            if (lane == 0) sv.q1[(o1 + a) * cin + c] = q;
            tq[c] += q;
            if (lane == a) td3[c] += d1[c];            // T[a][a][a]
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

    // ---- pass B: wave per receptive-field row b, lane z
    for (int b = wv; b < n; b += 4) {
        float sa[CM];
#pragma unroll
        for (int c = 0; c < CM; ++c) sa[c] = 0.f;
        // the neighbours a with b in C_a, ascending, in batches of 4 (loads first, then the sums)
        unsigned long long as = __ballot(lane < n && ((vmask[lane < n ? lane : 0] >> b) & 1ull));
        while (as) {
            int aa[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                aa[u] = as ? __ffsll((long long)as) - 1 : -1;
                as &= as ? as - 1ull : 0ull;
            }
            float t[4][CM];
            bool vz[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int a = aa[u] >= 0 ? aa[u] : 0;
                const unsigned long long ma = vmask[a];
                vz[u] = aa[u] >= 0 && lane < n && ((ma >> lane) & 1ull);
                const float* q;
                if (level0) {
                    q = X + (long long)s_j[a] * cin;
                } else {
                    const int pb = max(sp[a * n + b], 0), pz = vz[u] ? sp[a * n + lane] : 0;
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
#pragma unroll
        for (int c = 0; c < CM; ++c) {
            if (c >= cin) break;
            if (lane < n) sv.Sa[(o2 + (long long)b * n + lane) * cin + c] = sa[c];
            const float q3 = wave_sum(sa[c]);
            if (lane == 0) sv.q3[(o1 + b) * cin + c] = q3;
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
    // output: out[x][y][o] = relu(sum_q W_q . block_q[x][y] + b)   (W: h x 18 C, block q at cols q*C..)
    // the statistics of an entry are read once per channel and feed every output o (weights in LDS)
    const float nf = (float)n;
    const int K = 18 * cin;
    __shared__ float sw[HM * 18 * CM];
    for (int t = threadIdx.x; t < h * K; t += 256) sw[t] = W[t];
    __syncthreads();
    for (int e = threadIdx.x; e < n * n; e += 256) {
        const int x = e / n, y = e % n;
        float s[HM];
#pragma unroll
        for (int o = 0; o < HM; ++o) s[o] = o < h ? bias[o] : 0.f;
        for (int c = 0; c < cin; ++c) {
            const float sc = sv.Sc[(o2 + x * n + y) * cin + c];
            const float sa = sv.Sa[(o2 + x * n + y) * cin + c];
            float blk[18];
            blk[0] = nf * sc;
            blk[1] = sv.q1[(o1 + x) * cin + c];
            blk[2] = nf * sa;
            blk[3] = sv.q3[(o1 + x) * cin + c];
            blk[4] = x == y ? sv.tot[(long long)i * cin + c] : 0.f;
            blk[5] = sc;
#pragma unroll
            for (int q = 6; q < 15; ++q) blk[q] = nf * sc;
            blk[15] = sv.D1[(o2 + x * n + y) * cin + c];
            blk[16] = sv.D2[(o2 + y * n + x) * cin + c];
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
            fout[(o2 + e) * h + o] = s[o] < 0.f ? 0.f : s[o];
        }
    }
}

struct C2Grad {
    float* dSc;  // [sum d^2][C]  (dSc + dq1 folded)
    float* dSa;  // [sum d^2][C]  (dSa + dq3 + dtot folded)
    float* dD1;  // [sum d^2][C]
    float* dD2;  // [sum d^2][C]  indexed [a][b]
    float* dd3;  // [nodes][C]
};

// Block per node: dpre = dF * relu'(F); param partials; node-level gradient matrices.
// One sweep over the n^2 entries per output o for the parameter partials (the 9 distinct
// contraction blocks x cin accumulate in registers, then one wave-sum + LDS combine each), and one
// sweep for the input-side gradients (every channel of an entry from one read of dpre).
// BIG: the instantiation for degrees 65..256 (the level-0 reduction walks 64-lane chunks and
// multi-word common-neighbour sets, dSa read from L2 instead of an n x n LDS copy).
template <int CM, int HM, bool BIG = false>
__global__ void __launch_bounds__(256) k_ccn2_bwd_node(CcnPlanView v, const int* total_nodes,
                                                       const float* __restrict__ dF, const float* __restrict__ F,
                                                       C2Save sv, int cin, const float* __restrict__ W, int h,
                                                       C2Grad gd, float* __restrict__ ppart,
                                                       float* __restrict__ g0) {
    constexpr int MAXN = BIG ? CCN_BIGD : CCN_MAXD;
    __shared__ float sdq1[MAXN * CM], sdq3[MAXN * CM], sdtot[CM], sdd3[CM];
    __shared__ float red[4][10 * CM];
    __shared__ float sw[HM * 18 * CM];
    const int i = blockIdx.x;
    if (i >= *total_nodes) return;
    const int n = v.deg[i];
    if ((BIG ? (n <= CCN_MAXD || n > CCN_BIGD) : n > CCN_MAXD) || cin > CM || h > HM) return;
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
    if constexpr (BIG) {
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
        return;
    }
    __shared__ unsigned long long vm[CCN_MAXD];
    __shared__ float sa_l[CCN_MAXD * CCN_MAXD];
    __syncthreads();
    for (int a = wv; a < n; a += 4) {
        const unsigned long long m = __ballot(lane < n && v.pos[o2 + a * n + lane] >= 0);
        if (lane == 0) vm[a] = m;
    }
    for (int c = 0; c < cin; ++c) {
        __syncthreads();
        for (int e = threadIdx.x; e < n * n; e += 256) sa_l[e] = gd.dSa[(o2 + e) * cin + c];
        __syncthreads();
        for (int a = wv; a < n; a += 4) {
            const unsigned long long ma = vm[a];
            const bool vb = lane < n && ((ma >> lane) & 1ull);
            const bool va = (ma >> a) & 1ull;
            const float mf = (float)__popcll(ma);
            float t = 0.f;
            if (vb) {
                const long long rab = (o2 + (long long)a * n + lane) * cin + c;
                t = mf * gd.dSc[rab] + gd.dD1[rab] + (va ? gd.dD2[rab] : 0.f);
                unsigned long long zs = ma;
                while (zs) {
                    const int z = __ffsll((long long)zs) - 1;
                    zs &= zs - 1ull;
                    t += sa_l[lane * n + z];
                }
            }
            t = wave_sum(t);
            if (lane == 0) g0[(o1 + a) * cin + c] = t + (va ? sdd3[c] : 0.f);
        }
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
    for (int c = 0; c < cin; ++c) {
        float t = 0.f;
        for (int x = lane; x < n; x += 64) {  // one chunk for d <= 64
            const int i = nj[x];
            const int aj = v.pos[o2 + (long long)x * n + sj];  // position of j in N(i)
            t += g0[((long long)v.off1[i] + aj) * cin + c];
        }
        t = wave_sum(t);
        if (lane == 0) {
            const float rd = dsum ? dsum[(long long)v.graph[j] * dsum_ld + c] : 0.f;
            dout[(long long)j * cin + c] = t + (float)(n * n) * rd;
        }
    }
}

// Block per node j: dF_prev[j][u][w] = sum over neighbours i of the gradient of the entry of T_i that
// read F_j[u][w] (+ readout); level 0: dX[j] = sum over (u, w) (+ d_j^2 dsum0).  As in the forward,
// F_j[u][w] is read by T_i only where u, w are both common neighbours of i and j: wave per row u,
// lane w, walking the neighbours a with u in C_a (wave-uniform), lanes gathering where w in C_a.
template <int C, int NB>
__global__ void __launch_bounds__(256) k_ccn2_bwd_gather(CcnPlanView v, const int* total_nodes, C2Grad gd, int cin,
                                                         const float* __restrict__ dsum, int dsum_ld, int dsum_off,
                                                         int level0, float* __restrict__ dout) {
    // C: channel bound of this instantiation (cin <= C); NB: neighbours gathered per batch
    __shared__ int sp[CCN_MAXD * CCN_MAXD];
    __shared__ unsigned long long vmask[CCN_MAXD];
    __shared__ float red[4][C];
    __shared__ int s_i[CCN_MAXD], s_di[CCN_MAXD], s_oi[CCN_MAXD], s_aj[CCN_MAXD];  // neighbour a of j
    const int j = blockIdx.x;
    if (j >= *total_nodes) return;
    const int n = v.deg[j];
    if (n > CCN_MAXD || cin > C) return;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long o2 = v.off2[j];
    const int* nj = v.nbr + (long long)j * v.nmax;
    const int sj = v.selfpos[j];
    const int g = v.graph[j];
    for (int e = threadIdx.x; e < n * n; e += 256) sp[e] = v.pos[o2 + e];
    if (threadIdx.x < n) {
        const int i = nj[threadIdx.x];
        s_i[threadIdx.x] = i;
        s_di[threadIdx.x] = v.deg[i];
        s_oi[threadIdx.x] = v.off2[i];
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
    float rd[C], part[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        rd[c] = (dsum && c < cin) ? dsum[(long long)g * dsum_ld + dsum_off + c] : 0.f;
        part[c] = 0.f;
    }
    for (int u = wv; u < n; u += 4) {
        float acc[C];
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] = 0.f;
        // the neighbours a with u in C_a, ascending, NB at a time: every load of a batch is in flight
        // before the sums (the per-a walk paid ~3 dependent memory latencies per a: 2.2 -> 0.7 ms per
        // launch at config 5)
        unsigned long long as = __ballot(lane < n && ((vmask[lane < n ? lane : 0] >> u) & 1ull));
        while (as) {
            int aa[NB];
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                aa[q] = as ? __ffsll((long long)as) - 1 : -1;
                as &= as ? as - 1ull : 0ull;
            }
            float tsc[NB][C], tsa[NB][C], td1[NB][C], td2[NB][C], td3[NB][C];
            int zb[NB], zz[NB], zaj[NB];
            bool vz[NB];
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                const int a = aa[q] >= 0 ? aa[q] : 0;
                vz[q] = aa[q] >= 0 && lane < n && ((vmask[a] >> lane) & 1ull);
                const int b = max(sp[a * n + u], 0), z = vz[q] ? sp[a * n + lane] : 0;
                const int aj = s_aj[a], di = s_di[a], i = s_i[a];
                const long long oi = s_oi[a];
                const long long rab = (oi + (long long)aj * di + b) * cin, rbz = (oi + (long long)b * di + z) * cin;
                zb[q] = b;
                zz[q] = z;
                zaj[q] = aj;
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const bool ok = c < cin;
                    tsc[q][c] = ok ? gd.dSc[rab + c] : 0.f;
                    tsa[q][c] = ok ? gd.dSa[rbz + c] : 0.f;
                    td1[q][c] = ok ? gd.dD1[rab + c] : 0.f;
                    td2[q][c] = ok ? gd.dD2[rab + c] : 0.f;
                    td3[q][c] = ok ? gd.dd3[(long long)i * cin + c] : 0.f;
                }
            }
#pragma unroll
            for (int q = 0; q < NB; ++q) {
                if (aa[q] < 0) break;
                if (!vz[q]) continue;
                const int b = zb[q], z = zz[q], aj = zaj[q];
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    if (c >= cin) break;
                    float t = tsc[q][c] + tsa[q][c];
                    if (z == b) t += td1[q][c];
                    if (z == aj) t += td2[q][c];
                    if (aj == b && b == z) t += td3[q][c];
                    acc[c] += t;
                }
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if (c >= cin) break;
            if (level0) part[c] += acc[c];
            else if (lane < n) dout[(o2 + (long long)u * n + lane) * cin + c] = acc[c] + rd[c];
        }
    }
    if (level0) {
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if (c >= cin) break;
            const float t = wave_sum(part[c]);
            if (lane == 0) red[wv][c] = t;
        }
        __syncthreads();
        if (threadIdx.x < cin) {
            const int c = threadIdx.x;
            dout[(long long)j * cin + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c] + (float)(n * n) * rd[c];
        }
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
                                                      int h, C2Save sv, float* __restrict__ fout) {
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
            fout[(o2 + e) * h + o] = s[o] < 0.f ? 0.f : s[o];
        }
    }
}

// k_ccn2_bwd_gather for degrees 65..256: lane w of row u in 64-lane chunks, the neighbours a with
// u in C_a in 64-wide ballot chunks (ascending: the summation order of the fast kernel's walk).
template <int C, int NB>
__global__ void __launch_bounds__(256) k_ccn2_bwd_gather_big(CcnPlanView v, const int* total_nodes, C2Grad gd,
                                                             int cin, const float* __restrict__ dsum, int dsum_ld,
                                                             int dsum_off, int level0, float* __restrict__ dout) {
    __shared__ unsigned long long vmask[CCN_BIGD][CCN_BW];
    __shared__ float red[4][C];
    __shared__ int s_i[CCN_BIGD], s_di[CCN_BIGD], s_oi[CCN_BIGD], s_aj[CCN_BIGD];
    const int j = blockIdx.x;
    if (j >= *total_nodes) return;
    const int n = v.deg[j];
    if (n <= CCN_MAXD || n > CCN_BIGD || cin > C) return;
    const int nw = (n + 63) >> 6;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const long long o2 = v.off2[j];
    const int* sp = v.pos + o2;
    const int* nj = v.nbr + (long long)j * v.nmax;
    const int sj = v.selfpos[j];
    const int g = v.graph[j];
    for (int t = threadIdx.x; t < n; t += 256) {
        const int i = nj[t];
        s_i[t] = i;
        s_di[t] = v.deg[i];
        s_oi[t] = v.off2[i];
        s_aj[t] = sp[(long long)t * n + sj];  // position of j in N(i_a)
    }
    for (int a = wv; a < n; a += 4)
        for (int w = 0; w < nw; ++w) {
            const int x = w * 64 + lane;
            const unsigned long long m = __ballot(x < n && sp[(long long)a * n + x] >= 0);
            if (lane == 0) vmask[a][w] = m;
        }
    __syncthreads();
    float rd[C], part[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        rd[c] = (dsum && c < cin) ? dsum[(long long)g * dsum_ld + dsum_off + c] : 0.f;
        part[c] = 0.f;
    }
    for (int u = wv; u < n; u += 4) {
        for (int w0 = 0; w0 < n; w0 += 64) {
            const int wl = w0 + lane;
            float acc[C];
#pragma unroll
            for (int c = 0; c < C; ++c) acc[c] = 0.f;
            for (int a0 = 0; a0 < n; a0 += 64) {
                const int al = a0 + lane < n ? a0 + lane : 0;
                unsigned long long as = __ballot(a0 + lane < n && mbit(vmask[al], u));
                while (as) {
                    int aa[NB];
#pragma unroll
                    for (int q = 0; q < NB; ++q) {
                        aa[q] = as ? a0 + __ffsll((long long)as) - 1 : -1;
                        as &= as ? as - 1ull : 0ull;
                    }
                    float tsc[NB][C], tsa[NB][C], td1[NB][C], td2[NB][C], td3[NB][C];
                    int zb[NB], zz[NB], zaj[NB];
                    bool vz[NB];
#pragma unroll
                    for (int q = 0; q < NB; ++q) {
                        const int a = aa[q] >= 0 ? aa[q] : 0;
                        vz[q] = aa[q] >= 0 && wl < n && mbit(vmask[a], wl);
                        const int b = max(sp[(long long)a * n + u], 0), z = vz[q] ? sp[(long long)a * n + wl] : 0;
                        const int aj = s_aj[a], di = s_di[a], i = s_i[a];
                        const long long oi = s_oi[a];
                        const long long rab = (oi + (long long)aj * di + b) * cin, rbz = (oi + (long long)b * di + z) * cin;
                        zb[q] = b;
                        zz[q] = z;
                        zaj[q] = aj;
#pragma unroll
                        for (int c = 0; c < C; ++c) {
                            const bool ok = c < cin;
                            tsc[q][c] = ok ? gd.dSc[rab + c] : 0.f;
                            tsa[q][c] = ok ? gd.dSa[rbz + c] : 0.f;
                            td1[q][c] = ok ? gd.dD1[rab + c] : 0.f;
                            td2[q][c] = ok ? gd.dD2[rab + c] : 0.f;
                            td3[q][c] = ok ? gd.dd3[(long long)i * cin + c] : 0.f;
                        }
                    }
#pragma unroll
                    for (int q = 0; q < NB; ++q) {
                        if (aa[q] < 0) break;
                        if (!vz[q]) continue;
                        const int b = zb[q], z = zz[q], aj = zaj[q];
#pragma unroll
                        for (int c = 0; c < C; ++c) {
                            if (c >= cin) break;
                            float t = tsc[q][c] + tsa[q][c];
                            if (z == b) t += td1[q][c];
                            if (z == aj) t += td2[q][c];
                            if (aj == b && b == z) t += td3[q][c];
                            acc[c] += t;
                        }
                    }
                }
            }
#pragma unroll
            for (int c = 0; c < C; ++c) {
                if (c >= cin) break;
                if (level0) part[c] += acc[c];
                else if (wl < n) dout[(o2 + (long long)u * n + wl) * cin + c] = acc[c] + rd[c];
            }
        }
    }
    if (level0) {
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if (c >= cin) break;
            const float t = wave_sum(part[c]);
            if (lane == 0) red[wv][c] = t;
        }
        __syncthreads();
        if (threadIdx.x < cin) {
            const int c = threadIdx.x;
            dout[(long long)j * cin + c] = red[0][c] + red[1][c] + red[2][c] + red[3][c] + (float)(n * n) * rd[c];
        }
    }
}

// ------------------------------------------------------------------ readout
// feat[b] = cat_l (sum over the graph's rows of F_l); level 0: sum_i d_i^order X[i]
struct ReadoutArgs {
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
// the RO_CH chunks and applies fc.
constexpr int RO_CH = 32;

__global__ void __launch_bounds__(256) k_ccn_readout_part(ReadoutArgs r, double* __restrict__ part) {
    __shared__ double red[4][C2_CMAX];
    const int b = blockIdx.x, k = blockIdx.y;
    const int n0 = r.v.node_off[b], n1 = r.v.node_off[b + 1];
    const int* off = r.order == 1 ? r.v.off1 : r.v.off2;
    const int nf = r.f + r.L * r.h;
    double* pb = part + ((long long)b * RO_CH + k) * nf;
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
        const int len = n1 - n0, per = (len + RO_CH - 1) / RO_CH;
        const int i0 = n0 + k * per, i1 = min(n1, i0 + per);
        for (int i = i0 + (int)threadIdx.x; i < i1; i += 256) {
            const double d = r.v.deg[i];
            const double wgt = r.order == 1 ? d : d * d;
            for (int c = 0; c < nc; ++c) acc[c] += wgt * (double)r.X[(long long)i * r.f + c0 + c];
        }
        flush(acc, nc, c0);
    }
    for (int l = 0; l < r.L; ++l) {
        const long long r0 = off[n0], r1 = off[n1];
        const long long len = r1 - r0, per = (len + RO_CH - 1) / RO_CH;
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
        for (int k = 0; k < RO_CH; ++k) t += part[((long long)b * RO_CH + k) * nf + col];
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

// dsum[b][k] = sum_o dout[b][o] fcw[o][k];  dfcw, dfcb summed over graphs (one block)
__global__ void __launch_bounds__(256) k_ccn_readout_bwd(const float* __restrict__ dout, const float* __restrict__ feat,
                                                         const float* __restrict__ fcw, int bs, int n_out, int nf,
                                                         float* __restrict__ dsum, float* __restrict__ dfcw,
                                                         float* __restrict__ dfcb) {
    for (int e = threadIdx.x; e < bs * nf; e += 256) {
        const int b = e / nf, k = e % nf;
        float s = 0.f;
        for (int o = 0; o < n_out; ++o) s = fmaf(dout[b * n_out + o], fcw[o * nf + k], s);
        dsum[e] = s;
    }
    for (int e = threadIdx.x; e < n_out * nf; e += 256) {
        const int o = e / nf, k = e % nf;
        double s = 0.0;
        for (int b = 0; b < bs; ++b) s += (double)dout[b * n_out + o] * (double)feat[(long long)b * nf + k];
        dfcw[e] = (float)s;
    }
    for (int o = threadIdx.x; o < n_out; o += 256) {
        double s = 0.0;
        for (int b = 0; b < bs; ++b) s += (double)dout[b * n_out + o];
        dfcb[o] = (float)s;
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
    size_t node_off, deg, nbr, selfpos, graph, off1, off2, totals, err, pos;
    size_t plan_bytes;
    // feature workspace (needs sums)
    std::vector<size_t> F, coll;    // per level 1..L
    std::vector<C2Save> dummy;
    size_t sc[16], sa[16], d1[16], d2[16], q1[16], q3[16], tot[16], d3[16];
    size_t feat, rpart, g0, dsum, ppart, dF[2], dcoll, g_sc, g_sa, g_d1, g_d2, g_d3, xp, dxp;
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
    L.totals = take(16);
    L.err = take(16);
    L.pos = take(4 * (size_t)(sum_d2 > 0 ? sum_d2 : 1));
    L.plan_bytes = t;
    const long long rows = c->order == 1 ? sum_d : sum_d2;
    const int Lv = c->layers;
    const int h = c->hidden, f = c->f_in;
    L.F.resize(Lv);
    L.coll.resize(Lv);
    int cmax = f > h ? f : h;
    for (int l = 0; l < Lv; ++l) {
        const int cin = l == 0 ? f : h;
        L.F[l] = take(4 * (size_t)rows * h);
        if (c->order == 1) {
            L.coll[l] = take(4 * (size_t)rows * 2 * cin);
        } else {
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
        L.g_sc = take(4 * (size_t)sum_d2 * cmax);
        L.g_sa = take(4 * (size_t)sum_d2 * cmax);
        L.g_d1 = take(4 * (size_t)sum_d2 * cmax);
        L.g_d2 = take(4 * (size_t)sum_d2 * cmax);
        L.g_d3 = take(4 * (size_t)nodes * cmax);
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

}  // namespace
}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_collapse6to3(const float* d_F, float* d_out, int c, int n, void* stream) {
    if (!d_F || !d_out || c <= 0 || n <= 0) return HGNN_ERR_ARG;
    const long long tot = (long long)n * n * 18 * c;
    hipLaunchKernelGGL(k_collapse6to3, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream, d_F,
                       d_out, c, n);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int hgnn_collapse6to3_backward(const float* d_dout, float* d_dF, int c, int n, void* stream) {
    if (!d_dout || !d_dF || c <= 0 || n <= 0) return HGNN_ERR_ARG;
    const long long tot = (long long)c * n * n * n * n * n;
    hipLaunchKernelGGL(k_collapse6to3_bwd, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
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
    hipLaunchKernelGGL(k_ccn_nbrs, dim3(cfg->bs), dim3(256), 0, s, d_adj, cfg->nmax, v.node_off,
                       P<int>(plan_ws, L.deg), P<int>(plan_ws, L.nbr), P<int>(plan_ws, L.selfpos),
                       P<int>(plan_ws, L.graph), m.err, cfg->order == 1 ? CCN1_MAXD : CCN_BIGD);
    HGNN_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_ccn_scan, dim3(1), dim3(256), 0, s, P<int>(plan_ws, L.deg), m.totals,
                       P<int>(plan_ws, L.off1), P<int>(plan_ws, L.off2), m.totals + 2);
    HGNN_LAUNCH_CHECK();
    long long nodes = (long long)cfg->bs * cfg->nmax;
    if (sync) {
        int hbuf[4] = {0, 0, 0, 0};
        HGNN_HOST_CHECK(hipMemcpyAsync(hbuf, m.totals, 16, hipMemcpyDeviceToHost, s));
        HGNN_HOST_CHECK(hipStreamSynchronize(s));
        nodes = hbuf[0];
        h_sums[0] = hbuf[2];
        h_sums[1] = hbuf[3];
        h_sums[2] = nodes;
        if (h_sums[1] > max_sum_d2) return HGNN_ERR_ARG;  // caller re-plans with a larger bound
    } else {
        // bounds, no host sync: every graph's d_i <= n_b <= nmax; the kernels read the device totals
        h_sums[0] = nodes * cfg->nmax;
        h_sums[1] = max_sum_d2;
        h_sums[2] = nodes;
    }
    hipLaunchKernelGGL(k_ccn_pos, dim3((unsigned)((nodes + 3) / 4 > 0 ? (nodes + 3) / 4 : 1)), dim3(256), 0, s, v,
                       m.totals, P<int>(plan_ws, L.pos), max_sum_d2, m.err);
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
    hipLaunchKernelGGL(k_ccn_pack_x, dim3(cfg->bs), dim3(256), 0, s, d_X, v.node_off, cfg->nmax, f, Xp);
    HGNN_LAUNCH_CHECK();
    d_X = Xp;
    for (int l = 0; l < cfg->layers; ++l) {
        const int cin = l == 0 ? f : h;
        const float* fin = l == 0 ? nullptr : P<float>(W, L.F[l - 1]);
        const float* w = params[2 * l];
        const float* b = params[2 * l + 1];
        if (cfg->order == 1) {
            hipLaunchKernelGGL(k_ccn1_fwd, dim3(nodes > 0 ? (nodes + 3) / 4 : 1), dim3(256), 0, s, v, tot, fin,
                               l == 0 ? 1 : 0, d_X, cin, w, b, h, P<float>(W, L.coll[l]), P<float>(W, L.F[l]));
        } else {
            const bool narrow = cin <= C2_CMAX && h <= C2_HMAX;
            if (narrow)
                hipLaunchKernelGGL((k_ccn2_fwd<C2_CMAX, C2_HMAX>), dim3(nodes > 0 ? nodes : 1), dim3(256), 0, s, v, tot,
                                   fin, l == 0 ? 1 : 0, d_X, cin, w, b, h, save_of(L, W, l), P<float>(W, L.F[l]));
            else
                hipLaunchKernelGGL((k_ccn2_fwd<C2_CMAX_WIDE, C2_HMAX_WIDE>), dim3(nodes > 0 ? nodes : 1), dim3(256), 0,
                                   s, v, tot, fin, l == 0 ? 1 : 0, d_X, cin, w, b, h, save_of(L, W, l),
                                   P<float>(W, L.F[l]));
            HGNN_LAUNCH_CHECK();
            if (cfg->nmax > CCN_MAXD) {  // degrees 65..256 possible: their nodes in the large-degree kernel
                if (narrow)
                    hipLaunchKernelGGL((k_ccn2_fwd_big<C2_CMAX, C2_HMAX>), dim3(nodes > 0 ? nodes : 1), dim3(256), 0, s,
                                       v, tot, fin, l == 0 ? 1 : 0, d_X, cin, w, b, h, save_of(L, W, l),
                                       P<float>(W, L.F[l]));
                else
                    hipLaunchKernelGGL((k_ccn2_fwd_big<C2_CMAX_WIDE, C2_HMAX_WIDE>), dim3(nodes > 0 ? nodes : 1),
                                       dim3(256), 0, s, v, tot, fin, l == 0 ? 1 : 0, d_X, cin, w, b, h,
                                       save_of(L, W, l), P<float>(W, L.F[l]));
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
    for (int l = 0; l < cfg->layers; ++l) ra.F[l] = P<float>(W, L.F[l]);
    ra.fcw = params[2 * cfg->layers];
    ra.fcb = params[2 * cfg->layers + 1];
    ra.feat = P<float>(W, L.feat);
    ra.out = d_out;
    hipLaunchKernelGGL(k_ccn_readout_part, dim3(cfg->bs, RO_CH), dim3(256), 0, s, ra, P<double>(W, L.rpart));
    HGNN_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_ccn_readout, dim3(cfg->bs), dim3(256), 0, s, ra, P<double>(W, L.rpart));
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
    hipLaunchKernelGGL(k_ccn_readout_bwd, dim3(1), dim3(256), 0, s, d_dout, P<float>(W, L.feat), params[2 * Lv],
                       cfg->bs, cfg->n_out, nf, dsum, grads[2 * Lv], grads[2 * Lv + 1]);
    HGNN_LAUNCH_CHECK();
    const unsigned nb4 = nodes > 0 ? (unsigned)(nodes + 3) / 4 : 1u;
    const unsigned nb1 = nodes > 0 ? (unsigned)nodes : 1u;
    const long long rows = cfg->order == 1 ? sums[0] : sums[1];
    // dF of the top level = readout broadcast of its slice of dsum
    float* dF = P<float>(W, L.dF[0]);
    float* dFn = P<float>(W, L.dF[1]);
    hipLaunchKernelGGL(k_ccn_bcast, dim3(nb1), dim3(64), 0, s, v, tot, cfg->order, dsum, nf, f + (Lv - 1) * h, h, dF);
    HGNN_LAUNCH_CHECK();
    for (int l = Lv - 1; l >= 0; --l) {
        const int cin = l == 0 ? f : h;
        const float* w = params[2 * l];
        const int K = (cfg->order == 1 ? 2 : 18) * cin;
        float* ppart = P<float>(W, L.ppart);
        if (cfg->order == 1) {
            hipLaunchKernelGGL(k_ccn1_bwd_node, dim3(nb4), dim3(256), 0, s, v, tot, dF, P<float>(W, L.F[l]),
                               P<float>(W, L.coll[l]), cin, w, h, P<float>(W, L.dcoll), ppart);
        } else {
            C2Grad gd{P<float>(W, L.g_sc), P<float>(W, L.g_sa), P<float>(W, L.g_d1), P<float>(W, L.g_d2),
                      P<float>(W, L.g_d3)};
            const bool narrow = cin <= C2_CMAX && h <= C2_HMAX;
            float* g0p = l == 0 ? P<float>(W, L.g0) : nullptr;
            if (narrow)
                hipLaunchKernelGGL((k_ccn2_bwd_node<C2_CMAX, C2_HMAX>), dim3(nb1), dim3(256), 0, s, v, tot, dF,
                                   P<float>(W, L.F[l]), save_of(L, W, l), cin, w, h, gd, ppart, g0p);
            else
                hipLaunchKernelGGL((k_ccn2_bwd_node<C2_CMAX_WIDE, C2_HMAX_WIDE>), dim3(nb1), dim3(256), 0, s, v, tot,
                                   dF, P<float>(W, L.F[l]), save_of(L, W, l), cin, w, h, gd, ppart, g0p);
            HGNN_LAUNCH_CHECK();
            if (cfg->nmax > CCN_MAXD) {
                if (narrow)
                    hipLaunchKernelGGL((k_ccn2_bwd_node<C2_CMAX, C2_HMAX, true>), dim3(nb1), dim3(256), 0, s, v, tot,
                                       dF, P<float>(W, L.F[l]), save_of(L, W, l), cin, w, h, gd, ppart, g0p);
                else
                    hipLaunchKernelGGL((k_ccn2_bwd_node<C2_CMAX_WIDE, C2_HMAX_WIDE, true>), dim3(nb1), dim3(256), 0, s,
                                       v, tot, dF, P<float>(W, L.F[l]), save_of(L, W, l), cin, w, h, gd, ppart, g0p);
            }
        }
        HGNN_LAUNCH_CHECK();
        hipLaunchKernelGGL(k_ccn_param_reduce, dim3(h * K + h), dim3(256), 0, s, ppart, tot, h * K, h, grads[2 * l],
                           grads[2 * l + 1]);
        HGNN_LAUNCH_CHECK();
        const int lvl0 = l == 0 ? 1 : 0;
        float* dst = lvl0 ? P<float>(W, L.dxp) : dFn;
        const int doff = lvl0 ? 0 : f + (l - 1) * h;
        if (cfg->order == 1) {
            hipLaunchKernelGGL(k_ccn1_bwd_gather, dim3(nb4), dim3(256), 0, s, v, tot, P<float>(W, L.dcoll), cin, dsum,
                               nf, doff, lvl0, dst);
        } else {
            C2Grad gd{P<float>(W, L.g_sc), P<float>(W, L.g_sa), P<float>(W, L.g_d1), P<float>(W, L.g_d2),
                      P<float>(W, L.g_d3)};
            if (lvl0)
                hipLaunchKernelGGL(k_ccn2_dx0, dim3(nb4), dim3(256), 0, s, v, tot, P<float>(W, L.g0), cin, dsum, nf,
                                   dst);
            else {
                if (cin <= 2)
                    hipLaunchKernelGGL((k_ccn2_bwd_gather<2, 4>), dim3(nb1), dim3(256), 0, s, v, tot, gd, cin, dsum,
                                       nf, doff, lvl0, dst);
                else if (cin <= C2_CMAX)
                    hipLaunchKernelGGL((k_ccn2_bwd_gather<C2_CMAX, 1>), dim3(nb1), dim3(256), 0, s, v, tot, gd, cin,
                                       dsum, nf, doff, lvl0, dst);
                else
                    hipLaunchKernelGGL((k_ccn2_bwd_gather<C2_CMAX_WIDE, 1>), dim3(nb1), dim3(256), 0, s, v, tot, gd,
                                       cin, dsum, nf, doff, lvl0, dst);
                HGNN_LAUNCH_CHECK();
                if (cfg->nmax > CCN_MAXD) {
                    if (cin <= 2)
                        hipLaunchKernelGGL((k_ccn2_bwd_gather_big<2, 4>), dim3(nb1), dim3(256), 0, s, v, tot, gd, cin,
                                           dsum, nf, doff, lvl0, dst);
                    else if (cin <= C2_CMAX)
                        hipLaunchKernelGGL((k_ccn2_bwd_gather_big<C2_CMAX, 1>), dim3(nb1), dim3(256), 0, s, v, tot, gd,
                                           cin, dsum, nf, doff, lvl0, dst);
                    else
                        hipLaunchKernelGGL((k_ccn2_bwd_gather_big<C2_CMAX_WIDE, 1>), dim3(nb1), dim3(256), 0, s, v, tot,
                                           gd, cin, dsum, nf, doff, lvl0, dst);
                }
            }
        }
        HGNN_LAUNCH_CHECK();
        float* t = dF;
        dF = dFn;
        dFn = t;
    }
    (void)rows;
    hipLaunchKernelGGL(k_ccn_unpack_dx, dim3(cfg->bs), dim3(256), 0, s, P<float>(W, L.dxp), v.node_off, cfg->nmax, f,
                       d_dX);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

}  // extern "C"
