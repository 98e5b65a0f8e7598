// Internal launch wrappers shared by the executor and the C-ABI layer.
#pragma once

#include "common.h"

namespace hgnn {

// ---------------------------------------------------------------- structure
// Kinds of per-row operator lists built from the dense padded inputs.
enum StructKind : int {
    S_W = 0,    // node rows n, cols m:  W[b, n, m, :]           (graph_oper(W, X))
    S_WT = 1,   // node rows m, cols n:  W[b, n, m, :]           (its transpose)
    S_WL = 2,   // edge rows, WL[b, e, e', :]                    (graph_oper(WL, XL))
    S_WLT = 3,  // transpose of WL
    S_PN = 4,   // node rows n, edge cols m: {Pm, Pd}[b, n, m]    (P_multi(Pm, .))
    S_PE = 5,   // edge rows m, node cols n: {Pm, Pd}[b, n, m]    (P_multi(Pm^T, .))
    S_COUNT = 6
};

struct StructView {
    const RowInfo* rows;   // per packed row: [start, start + count) in entries
    const float* entries;  // (1 + ncoef) floats per entry, padded to 4 or 8 floats
    int stride;            // floats per entry (4 or 8)
};

struct BatchMeta {
    int* node_off;   // (bs + 1) packed node row offsets
    int* edge_off;   // (bs + 1) packed edge row offsets
    int* totals;     // [0] = total nodes, [1] = total edge slots
    uint32_t* err;   // validation bits (ERR_*)
    double* zero64 = nullptr;  // optional: a region the first kernel of the forward zeroes (k_plan block 0)
    int zero64_n = 0;          //   (the BN-backward statistics accumulators, BnBwdArgs::acc64)
};

struct RepackTable;
// rt (optional): a weight repack table done by extra blocks of the same launch
int launch_plan(const int64_t* nb, const int64_t* eb, int bs, int nmax, int emax, BatchMeta m,
                hipStream_t s, const RepackTable* rt = nullptr);

struct ExtractArgs {
    const float* W;
    const float* WL;
    const float* Pm;
    const float* Pd;
    const float* mask;
    const float* mask_lg;
    int bs, nmax, emax, jtot;
    BatchMeta meta;
    RowInfo* rows[S_COUNT];
    float* entries[S_COUNT];
    int entry_stride_w;   // floats per W/WL entry
    int validate;
    int dual;             // 0: GNN_simple (only S_W / S_WT)
    int kind0;            // first block slot of the launch (blockIdx.y + kind0, struct.hip)
    // optional: pack the inputs in the same launch (X (bs, f, nmax) -> xo [nodes][f];
    // XL (bs, 1, emax) -> xlo [edges])
    const float* X;
    const float* XL;
    int f;
    float* xo;
    float* xlo;
    uint64_t* stamps;  // the launch's stamp slot under a stamp-mode clock (common.h WaveStamp), else null
    int dbg;           // diagnostics (HGNN_XR_DBG, k_extract_reg): 1 = stop after the loads, 2 = after the marks
};
int launch_extract(const ExtractArgs& a, hipStream_t s);

// Pack X (bs, f, nmax) -> [nodes][f];  XL (bs, 1, emax) -> [edges][1].
int launch_pack_nodes(const float* X, int bs, int f, int nmax, BatchMeta m, float* out, hipStream_t s);
int launch_pack_edges(const float* XL, int bs, int emax, BatchMeta m, float* out, hipStream_t s);
// Unpack [nodes][f] -> dense (bs, f, nmax), zero padding.
int launch_unpack_nodes(const float* in, int bs, int f, int nmax, BatchMeta m, float* X, hipStream_t s);

// ---------------------------------------------------------------- aggregation
// BN of a layer output applied where it is read: z = w ((y - mean_c) / std_c) + b
// (batch_normalization.py:43, 76), bit-identical to a separate apply pass.
// mean == nullptr: the features are read as stored.
struct BnView {
    const float* mean;
    const float* std;
    const float* w;
    const float* b;
};

// BN output z = w (y - mean) / std + b, evaluated as (y - mean) * (w / std) + b with the
// scale rounded once per channel: every reader (aggregation, dense dW) uses these two
// functions, so all consumers see the same z.  The reference's operation order
// (sub, div, mul, add) differs by a few ulp; an exact __fdiv_rn per gathered element cost
// the aggregation forward ~15 % (measured: 0.198 -> 0.167 ms per step).
__device__ __forceinline__ float bn_scale(float w, float sd) { return w / sd; }
__device__ __forceinline__ float bn_z_s(float y, float mu, float scale, float b) { return fmaf(y - mu, scale, b); }
__device__ __forceinline__ float bn_z(float y, float mu, float sd, float w, float b) {
    return bn_z_s(y, mu, bn_scale(w, sd), b);
}

struct AggFwdArgs {
    const int* total_rows;  // device
    int cap_rows;
    // G part: out[:, j*Cg + c] = sum_e v_j * Xg[col, c]
    StructView g;
    const float* xg;
    int cg, jtot;
    BnView gbn;             // xg holds pre-BN y (mean != null) or the features themselves
    // P part: out[:, jtot*Cg + c] = sum pm * Xp[col, c];  [.. + Cp + c] = sum pd * Xp[col, c]
    StructView p;
    const float* xp;
    int cp;
    BnView pbn;
    float* out;
    int ldo;
    // the row's zero padding [pad_from, ldo): 0 = after the parts this launch writes, -1 = none
    // (a G-only launch beside a P-only one, which writes the padding)
    int pad_from;
    // j0 = 2 ("diagonal I / D"): slices 0 and 1 of G (graph_operators' I and D, functions/operators.py:19-23)
    // are not aggregated -- the Conv1d GEMMs read x itself and scale it per row (gemm_bf3.hip) -- so the G part
    // holds slices 2 .. jtot - 1 at (j - 2) * cg and P starts at (jtot - 2) * cg.  diag (optional): per row
    // the diagonal entry's (v_0, v_1), (0, 0) for a row without one; an entry off the diagonal with v_0 or v_1
    // nonzero ORs ERR_DIAG_ID into err
    int j0;
    float2* diag;
    uint32_t* err;
    uint64_t* stamps;  // set by the launch under a stamp-mode clock (common.h WaveStamp), else null
};
int launch_agg_fwd(const AggFwdArgs& a, hipStream_t s);

struct AggBwdArgs {
    const int* total_rows;
    int cap_rows;
    // G part: out[r, c] += sum_e sum_j v_j * ing[col, gofs + j*C + c]
    StructView g;
    const float* ing;
    int ldg, gofs, jtot;
    // P part: out[r, c] += sum_e pm * inp[col, pofs_m + c] + pd * inp[col, pofs_d + c]
    StructView p;
    const float* inp;
    int ldp, pofs_m, pofs_d;
    int c;
    float* out;
    int ldo;
    int accumulate;
    uint64_t* stamps;  // the launch's stamp slot (common.h WaveStamp), else null
};
int launch_agg_bwd(const AggBwdArgs& a, hipStream_t s);  // exactly one of ing / inp
// the G gather of ga and the P gather of pa (different outputs) in one grid when they
// share the lane layout, else two launches
int launch_agg_bwd_pair(const AggBwdArgs& ga, const AggBwdArgs& pa, hipStream_t s);

// ---------------------------------------------------------------- GEMM (gemm3.hip, gemm_bf3.hip, repack.hip)
// fp32 x as three bf16 parts x1 + x2 + x3 (residual below 2^-26 |x|): the operand form of the split-bf16
// GEMM (gemm_bf3.hip).  Non-finite inputs: x = +-Inf (or |x| above the bf16 maximum, which rounds x1 to Inf)
// gives x2 = Inf - Inf = NaN, so a split-bf16 GEMM (the forward at 2d % 64 == 0, the dA at 2d <= 128, every
// dW GEMM) returns NaN where an fp32 GEMM returns Inf; finite inputs below the bf16 maximum (~3.4e38) are
// unaffected.  Not guarded in the split: a select per element costs ~3 VALU in the staging loop these GEMMs
// are bound by (round 5: 32 v_cmp + 110 v_cndmask per 24 MFMAs); HGNN_FWD_BF3=0 / HGNN_DA_BF3=0 /
// HGNN_DW_BF3=0 select the fp32 GEMMs.
__device__ __forceinline__ void split3(float x, __bf16& a, __bf16& b, __bf16& c) {
    a = (__bf16)x;
    const float r = x - (float)a;
    b = (__bf16)r;
    c = (__bf16)(r - (float)b);
}
__host__ __device__ inline int bf3_ld(int k) { return (k + 15) / 16 * 16; }  // plane row length (bf16)
// The forward Conv1d-pair GEMM on bf16 MFMA (three-way split, fp32 accuracy): Y = A . B^T + bias, ReLU
// from column relu_from, BN partials per 64-row tile (as launch_gemm3_fwd); A fp32 [M][lda] (k < kp),
// B three bf16 planes b + p pb [N][ldb] (ldb >= bf3_ld(k), zero beyond k)
// The dA GEMM on bf16 MFMA (three-way split): Y[M][n] = A[M][k] . B^T for k <= 128 (A = dY fp32 [M][lda],
// B = WT's three bf16 planes b + p pb [n][ldb], ldb >= bf3_ld(k), zero beyond k); HGNN_ERR_UNSUPPORTED otherwise
// The diagonal I / D operand columns of the Conv1d GEMMs (AggFwdArgs::j0 = 2): the logical operand of a half is
// [v_0(r) x̂_r | v_1(r) x̂_r | aggregate of slices 2.. and P], x̂ = BN(x) of the half's G input applied on load --
// the values the full aggregation stores in its I and D columns, bit for bit (fmaf(v, x̂, 0) per element, as
// the aggregation's first live FMA), so the GEMMs see the same operand.  kx = 2c leading logical columns come
// from x; the rest from the aggregate (its column k - kx).  kx = 0: no such columns (the operand is the
// aggregate alone).
struct DiagIdArgs {
    const float* x;        // the G input of the half, pre-BN y [rows][ldx]
    int ldx, c;            // c channels: kx = 2c (a multiple of 32 and c <= 256 where set)
    const float2* diag;    // per row (v_0, v_1) of the diagonal entry (AggFwdArgs::diag)
    BnView bn;             // BN of the producer of x (mean != null)
};
int launch_gemm_bf3_da(const float* a, int lda, const int* m_valid, int m_cap, int k, const __bf16* b, long long pb,
                       int ldb, int n, float* y, int ldy, hipStream_t s);
// (id: the diagonal I / D columns, k counts them; null = none)
// The BN finalize done by the forward GEMM's last block (ticket; zero on entry, left zero): mean / std of the 2d
// channels from the fp64 sums and the running statistics update, as k_bn_finalize's atomic form computes them
struct FwdBnFin {
    float* mean;
    float* std;
    float* run_mean;
    float* run_std;
    float momentum;
    unsigned* ticket;
};
// (bn_acc: the BN statistics as fp64 atomic sums [BN_ACC_COPIES][2][n] (sum y, sum y^2, zero on entry) instead of the
// per-tile partials bn_part; fin (with bn_acc): the finalize in the GEMM's last block, no k_bn_finalize)
int launch_gemm_bf3_fwd(const float* a, int lda, const int* m_valid, int m_cap, int k, const __bf16* b, long long pb,
                        int ldb, int n, const float* bias, int relu_from, float* y, int ldy, float* bn_part,
                        hipStream_t s, const DiagIdArgs* id = nullptr, double* bn_acc = nullptr,
                        const FwdBnFin* fin = nullptr);
// The dW GEMM (launch_gemm3_dw's contract) on bf16 MFMA through the same three-way split (id: as the forward's,
// for the aggregate operand)
int launch_gemm_bf3_dw(const float* dy, int lddy, const float* a, int lda, const int* r_valid, int r_cap, int o,
                       int k, int nz, float* slabs, int xcd, hipStream_t s, const DiagIdArgs* id = nullptr);

struct RepackItem {
    const float* wl;   // linear conv weight (d, K)
    const float* wr;   // ReLU conv weight (d, K)
    const float* bl;
    const float* br;
    float* wt;         // out: [K][ldt], columns [2d, ldt) zero
    float* wc;         // out: [2d][kp]
    float* bc;         // out: [2d]
    int k, kp, ldt;
    __bf16* wc3;       // optional out: Wcat as three bf16 planes [3][2d][ldc3] (split3), zero beyond K
    int ldc3;
    __bf16* wt3;       // optional out: WT as three bf16 planes [3][K][ldt3] (split3; the split-bf16 dA GEMM's B),
    int ldt3;          // zero beyond 2d
};
constexpr int REPACK_MAX = 24;
struct RepackTable {
    RepackItem it[REPACK_MAX];
    int n, d;
    int y;  // blocks per item (repack_y)
    uint64_t* stamps;  // the launch's stamp slot under a stamp-mode clock (common.h WaveStamp), else null
};
int launch_repack(const RepackTable& t, hipStream_t s);
// blocks per repack item: ~4 elements per thread of the largest item, 8..256 blocks (d = 64: 80
// transpose tiles; d = 128: 320 -- 96 blocks left 44 us of sequential tiles at d = 128)
inline int repack_y(const RepackTable& t) {
    long long mx = 1;
    for (int i = 0; i < t.n; ++i) mx = mx > (long long)t.it[i].k * t.it[i].ldt ? mx : (long long)t.it[i].k * t.it[i].ldt;
    const long long y = (mx + 1023) / 1024;
    return (int)(y < 8 ? 8 : (y > 256 ? 256 : y));
}
// one repack item's share of block yb of t.y (256 threads):
// WT[k][n] = Wcat[n][k] (dA B), WC[n][k < kp] = Wcat[n][k] zero-padded to kp (forward B),
// bc = cat(b_lin, b_relu)
__device__ __forceinline__ void repack_part(const RepackTable& t, int item, int yb) {
    const RepackItem& it = t.it[item];
    const int d = t.d, c2 = 2 * d, K = it.k, kp = it.kp, ldt = it.ldt;
    auto W = [&](int n, int k) { return n < d ? it.wl[(long long)n * K + k] : it.wr[(long long)(n - d) * K + k]; };
    // WT through 32 x 33 LDS tiles: reads along k and writes along n both coalesced (the direct
    // transpose wrote 4-byte scattered stores: 8 us at d = 64, 44 us at d = 128); the columns
    // [2d, ldt) -- the zero padding of an odd 2d to the dA GEMM's float4 k -- are written as zeros
    __shared__ float tile[32][33];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 8 row groups
    const int nkt = (K + 31) / 32, ntiles = ((ldt + 31) / 32) * nkt;
    for (int tl = yb; tl < ntiles; tl += t.y) {
        const int n0 = (tl / nkt) * 32, k0 = (tl % nkt) * 32;
        for (int rr = ty; rr < 32; rr += 8) {
            const int n = n0 + rr, k = k0 + tx;
            tile[rr][tx] = (n < c2 && k < K) ? W(n, k) : 0.f;
        }
        __syncthreads();
        for (int rr = ty; rr < 32; rr += 8) {
            const int k = k0 + rr, n = n0 + tx;
            if (k < K && n < ldt) it.wt[(long long)k * ldt + n] = tile[tx][rr];
            if (it.wt3 && k < K && n < it.ldt3) {  // (ldt3 = bf3_ld(ldt) <= the tiles' 32-column cover)
                const long long e = (long long)k * it.ldt3 + n, pl = (long long)K * it.ldt3;
                __bf16 a, b, c;
                split3(tile[tx][rr], a, b, c);
                it.wt3[e] = a;
                it.wt3[pl + e] = b;
                it.wt3[2 * pl + e] = c;
            }
        }
        __syncthreads();
    }
    // WC as three bf16 planes (the split-bf16 forward GEMM's B operand), coalesced along k
    // (32-bit element indices: 2d <= 1024 rows of at most a few thousand k; the 64-bit division per element
    // these loops had was most of the launch's VALU)
    // 4 elements per thread per round, every load issued (clamped, unconditional) before the first store: one
    // load per iteration made each block a chain of dependent round trips (~7 us per wave in the step)
    auto Wc = [&](int n, int k) {  // W(n, k) with n, k clamped into range (a live address, masked after)
        n = min(n, c2 - 1);
        k = min(k, K - 1);
        return n < d ? it.wl[(long long)n * K + k] : it.wr[(long long)(n - d) * K + k];
    };
    constexpr int RU = 4;
    const int step = t.y * 256;
    if (it.wc3) {
        const int n3 = c2 * it.ldc3;
        for (int e0 = yb * 256 + (int)threadIdx.x; e0 < n3; e0 += RU * step) {
            float v[RU];
#pragma unroll
            for (int u = 0; u < RU; ++u) {
                const int e = min(e0 + u * step, n3 - 1), n = e / it.ldc3, k = e - n * it.ldc3;
                v[u] = Wc(n, k);
            }
#pragma unroll
            for (int u = 0; u < RU; ++u) {
                const int e = e0 + u * step;
                if (e >= n3) break;
                const int n = e / it.ldc3, k = e - n * it.ldc3;
                __bf16 a, b, c;
                split3(k < K ? v[u] : 0.f, a, b, c);
                it.wc3[e] = a;
                it.wc3[n3 + e] = b;
                it.wc3[2 * n3 + e] = c;
            }
        }
    }
    // WC (zero-padded to kp) and bc: coalesced along k
    const int nc = c2 * kp;
    for (int e0 = yb * 256 + (int)threadIdx.x; e0 < nc; e0 += RU * step) {
        float v[RU];
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            const int e = min(e0 + u * step, nc - 1), n = e / kp, k = e - n * kp;
            v[u] = Wc(n, k);
        }
#pragma unroll
        for (int u = 0; u < RU; ++u) {
            const int e = e0 + u * step;
            if (e >= nc) break;
            const int n = e / kp, k = e - n * kp;
            it.wc[e] = k < K ? v[u] : 0.f;
        }
    }
    for (int n = yb * 256 + (int)threadIdx.x; n < c2; n += step) it.bc[n] = n < d ? it.bl[n] : it.br[n - d];
}

// GEMM v3 (gemm3.hip): both operands k-contiguous ("NT"), used for the forward and dA.
int gemm_fwd_tiles_m(int m_cap);  // 64-row tiles of the forward GEMM's BN partials
bool gemm3_ok(int lda, int ldb, int ldc, const void* a, const void* b);
// mfma16: the 16x16x4-MFMA kernel may take the imbalanced (small-grid) shapes; its k-order differs
// from the 32x32x2 kernel's by rounding (line-graph networks; GNN_simple keeps the 32x32 order)
int launch_gemm3_fwd(const float* a, int lda, const int* m_valid, int m_cap, int k, const float* wc, int ldw, int n,
                     const float* bias, int relu_from, float* y, int ldy, float* bn_part, hipStream_t s,
                     int mfma16 = 0);
int launch_gemm3_da(const float* dy, int lddy, const int* m_valid, int m_cap, int o, const float* wt, int ldw,
                    int kout, float* da, int ldda, hipStream_t s);
// dW split-K: the host fixes the number of row chunks nz (a multiple of 8, ~dw3_target_blocks() blocks with
// the output tiles); the kernels derive the chunk length from the device row count, so every chunk
// holds rows whatever the batch's fill of its capacity
int dw3_chunks(int r_cap, int o, int k);
bool dw_bf3_enabled();  // the dW GEMM on split-bf16 MFMA (HGNN_DW_BF3 != 0)
__host__ __device__ inline int dw3_kc(int rows, int nz) {
    int kc = (rows + nz - 1) / nz;
    kc = (kc + 31) / 32 * 32;
    return kc < 64 ? 64 : kc;
}
size_t dw3_slab_floats(int r_cap, int o, int k);
int launch_gemm3_dw(const float* dy, int lddy, const float* a, int lda, const int* r_valid, int r_cap, int o, int k,
                    int nz, float* slabs, hipStream_t s, const DiagIdArgs* id = nullptr);
// slabs [z][o][k] -> dW (rows [0, split) -> dw0, [split, o_real) -> dw1; rows >= o_real are the
// zero padding of an odd 2d); bias grads from the BN-backward per-tile column sums of dY
// (dbpart [tiles][o_real])
int launch_dw_reduce2(const float* slabs, const int* r_valid, int nz, int o, int o_real, int k, int split,
                      float* dw0, float* dw1, const float* dbpart, float* db0, float* db1, hipStream_t s);

// ---------------------------------------------------------------- BN
struct BnFwdArgs {
    const double* acc;     // optional: the forward GEMM's fp64 atomic sums [BN_ACC_COPIES][2][c] (sum y, sum y^2); else
                           // part
    const float* part;     // [tiles][c][3]
    int tiles, c;
    const int* count;      // device: total real rows (sum N_batch / E_batch)
    const float* w;        // scalar
    const float* b;        // scalar
    float* mean;           // (c,) batch or running (eval) statistics in use
    float* std;            // (c,)
    float* run_mean;       // running stats (may be null)
    float* run_std;
    int training;
    float momentum;
    uint64_t* stamps;  // the launch's stamp slot under a stamp-mode clock (common.h WaveStamp), else null
};
int launch_bn_finalize(const BnFwdArgs& a, hipStream_t s);

int launch_bn_apply(const float* y, const int* total_rows, int cap_rows, int c,
                    const float* mean, const float* std, const float* w, const float* b,
                    float* z, hipStream_t s);

// BN backward: dY = relu'(Y) * (w / std) * (dZ - mean(dZ.w) - H * mean(dZ.w . H)) (training)
struct BnBwdArgs {
    const float* y;        // pre-BN activations [rows][c]
    const float* dz;       // gradient wrt BN output [rows][c]
    const int* total_rows;
    int cap_rows, c;
    const float* mean;
    const float* std;
    const float* w;
    int relu_from;
    int training;
    float* part;           // scratch [tiles][c][2]
    float* sums;           // scratch [c][2] + [2]
    float* dy;             // out [rows][ldy] (ldy = 0: c; ldy > c only on the scalar path, c % 4 != 0)
    int ldy;
    float* dw;             // scalar out
    float* db;             // scalar out
    float* dbpart;         // optional out: per-64-row-tile column sums of dy [tiles][c]
    // optional (the float4 part4 / apply4 path): the statistics go by fp64 atomics into acc64 (BN_ACC_COPIES copies
    // [copy][4][c], zero on entry; copy = tile % BN_ACC_COPIES spreads the adders) instead of per-tile partials
    // summed by k_bn_bwd_fin -- apply4 reads the copies in a fixed order -- and apply4 zeroes acc64_zero (the next
    // half's region) for the call after it.  Other paths zero acc64_zero with a memset.
    double* acc64;
    double* acc64_zero;
    uint64_t* stamps;  // the launch's stamp slot under a stamp-mode clock (common.h WaveStamp), else null
};
constexpr int BN_ACC_COPIES = 8, BN_ACC_STATS = 4;
__host__ __device__ inline long long bn_acc_doubles(int c) { return (long long)BN_ACC_COPIES * BN_ACC_STATS * c; }
// apply = 0: only the statistics (part + fin)
int launch_bn_backward(const BnBwdArgs& a, hipStream_t s, int apply = 1);
__host__ __device__ inline int bn_bwd_tiles(int cap_rows) { return (cap_rows + 63) / 64; }
// k_bn_bwd_part / part4 -> k_bn_bwd_fin partials: float4 {sum g, sum g h, sum dz h, sum dz} per (channel,
// 64-row tile), channel-major [c][tiles] so the fin's per-channel loads are contiguous over the tiles
__host__ __device__ inline long long bn_bwd_part_index(int ch, int tile, int tiles) {
    return ((long long)ch * tiles + tile) * 4;
}

// dY of BN backward + ReLU for one element (batch_normalization.py:65-77 autograd):
// g = w dz, h = (y - mean) / std, train: (g - m1 - h m2) / std with m1 = mean(g),
// m2 = mean(g h) over the real rows; eval: g / std; ReLU branch masked where y <= 0.
__device__ __forceinline__ float bn_bwd_dy(float yv, float dzv, float mu, float sd, float wv, float m1, float m2,
                                           bool training, bool relu) {
    const float g = wv * dzv;
    float d;
    if (training) {
        const float h = __fdiv_rn(__fsub_rn(yv, mu), sd);
        d = (g - m1 - h * m2) / sd;
    } else {
        d = g / sd;
    }
    if (relu && !(yv > 0.f)) d = 0.f;
    return d;
}

// Same with the reciprocal of std rounded once per channel (the float4 BN-backward kernels):
// multiplications instead of two correctly rounded divisions per element.
__device__ __forceinline__ float bn_bwd_dy_inv(float yv, float dzv, float mu, float isd, float wv, float m1, float m2,
                                               bool training, bool relu) {
    const float g = wv * dzv;
    float d;
    if (training) {
        const float h = (yv - mu) * isd;
        d = (g - m1 - h * m2) * isd;
    } else {
        d = g * isd;
    }
    if (relu && !(yv > 0.f)) d = 0.f;
    return d;
}

// ---------------------------------------------------------------- dense dW of the operators
struct DwDenseArgs {
    const float* dA;       // node-half aggregate gradient [rows][lda]; G block = cols [0, jt*f)
    int lda;
    int f, jt;
    const float* xp;       // packed layer input [rows][f]  (unless xdense); pre-BN y when pmean != null
    const float* xdense;   // dense (bs, f, nmax) layer input (layer 0), or null
    const float* pmean;    // BN stats of the producer of xp (applied on load; padded value), or null -> 0
    const float* pstd;
    const float* pw;
    const float* pb;
    const float* dout;     // readout: dG at padded rows = dout[b] . fcw[:, k] ; null otherwise
    const float* fcw;
    int dim_out, kfc;
    const int* node_off;
    int bs, nmax;
    float* dW;             // (bs, nmax, nmax, jt)
    int accumulate;
    uint64_t* stamps;  // the launch's stamp slot under a stamp-mode clock (common.h WaveStamp), else null
};
int launch_dw_dense(const DwDenseArgs& a, hipStream_t s);

// ---------------------------------------------------------------- readout
int launch_readout_fwd(const float* a, int k, const int* node_off, int bs, int nmax,
                       const float* fcw, const float* fcb, int dim_out,
                       float* colsum, float* out, hipStream_t s);
int launch_readout_bwd_da(const float* dout, const int* node_off, int bs, int cap_rows,
                          const int* total_rows, const float* fcw, int dim_out, int k,
                          float* da, hipStream_t s);
int launch_readout_bwd_params(const float* dout, const float* colsum, int bs, int nmax,
                              int dim_out, int k, float* dfcw, float* dfcb, void* scratch, hipStream_t s);
size_t readout_bwd_scratch_bytes(int dim_out, int k);
// The last layer's transposed gathers straight from the readout gradient row R_b = dout[b] . fcw
// (no [rows][K] gradient buffer): G rows -> g_out (node features), P rows -> p_out (edge features).
struct ReadoutAggArgs {
    const float* dout;
    const float* fcw;
    int dim_out, k;          // k = fc input width (jt * cg + 2 * cp)
    int jt, cg, cp, bs;
    const int* node_off;
    const int* edge_off;
    StructView g;            // S_WT (node rows)
    const int* g_total;
    int g_cap;
    float* g_out;            // null: no G gather
    int g_acc;
    StructView p;            // S_PE (edge rows)
    const int* p_total;
    int p_cap;
    float* p_out;            // null: no P gather
    int p_acc;
    uint64_t* stamps;  // the launch's stamp slot under a stamp-mode clock (common.h WaveStamp), else null
};
int launch_readout_agg_bwd(const ReadoutAggArgs& a, hipStream_t s);
// whether the readout-row backward (launch_readout_agg_bwd and, with dw, launch_dw_readout) fits its
// LDS; the executor falls back to the materialised [rows][K] readout gradient otherwise
struct DwDenseArgs;
bool readout_row_fits(const ReadoutAggArgs& ra, const DwDenseArgs* dw);
// dW of the readout layer's graph_oper: dW[b, n, m, j] (+)= sum_f R_b[j F + f] X[m, f], every n
int launch_dw_readout(const DwDenseArgs& a, hipStream_t s);

// CCN-2D one-workgroup-per-graph path (ccn2_small.hip) behind hgnn_ccn_small_* for order 2
bool ccn2_small_ok(const hgnn_ccn_config* c);
size_t ccn2_small_workspace_bytes(const hgnn_ccn_config* c);
int ccn2_small_forward(const hgnn_ccn_config* c, const float* X, const float* adj, const int64_t* nb,
                       const float* const* params, void* ws, int32_t* err, int32_t tag, float* out, hipStream_t s);
int ccn2_small_backward(const hgnn_ccn_config* c, const float* X, const float* adj, const int64_t* nb,
                        const float* const* params, void* ws, const float* dout, float* const* grads, float* dX,
                        hipStream_t s);

}  // namespace hgnn
