// fp32 GEMM on bf16 MFMA through a three-way operand split (the forward Conv1d-pair GEMM).
//
// An fp32 operand x is used as three bf16 parts, x = x1 + x2 + x3 (split3: x1 = bf16(x), x2 = bf16(x - x1),
// x3 = bf16(x - x1 - x2); the residual is below 2^-26 |x|).  A product is the six bf16 x bf16 terms with
// i + j <= 4, each exact in fp32, accumulated in fp32 by v_mfma_f32_32x32x16_bf16; the three dropped
// terms are below 2^-26 of the product, so the result carries the error of an fp32 GEMM (one rounding per
// accumulation).  Six bf16 MFMAs (6 x 32 cycles per 32x32x16) replace eight fp32 ones (8 x 64 cycles per
// 32x32x16 of v_mfma_f32_32x32x2_f32): 2.7x fewer MFMA cycles, which the forward GEMM (K = 640 at
// config 2, bound by the fp32 MFMA issue rate) turns into time.
//
// Y[M][N] = A[M][K] . B[N][K]^T (+ bias, ReLU from column relu_from, BN partials per 64-row tile) with A
// the fp32 aggregate (split at staging) and B the weights as three bf16 planes [3][N][ldb] (split once by
// the repack, zero beyond K).  Block 64 x 64, 2 x 2 waves of 32 x 32, k stages of 32 staged global ->
// registers -> LDS (double buffer); LDS plane rows of 64 B with the 16-B chunks XOR-swizzled by
// (row >> 2) & 3, so the fragment reads (ds_read_b128: 8 k of one row per lane) are conflict-free.
#include "kernels.h"

namespace hgnn {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int G_BM = 64, G_BN = 64, G_BK = 32, G_NT = 256;
constexpr int G_ROWB = G_BK * 2;                      // bytes of one plane row in a stage
constexpr int G_PLANE = G_BM * G_ROWB;                // bytes of one plane of one operand (BM == BN)
constexpr int G_STAGE = 6 * G_PLANE;                  // A planes, then B planes

__device__ __forceinline__ int swz(int row, int ch) { return row * G_ROWB + 16 * (ch ^ ((row >> 2) & 3)); }

// The staging loads of the forward and dA GEMMs through buffer descriptors: A's records end at row M, B's at the
// third plane's row N; a masked load (column past K or past the plane row, weight row past N) takes the lane
// offset 2^31, past both record counts, and the range check returns zeros -- no exec branch around a load and
// no select at the split.  The launchers keep (m_cap + 64) lda and 3 pb below 2^29 elements.
struct BufOps {
    __amdgpu_buffer_rsrc_t sa, sb;
    unsigned arow_off;  // bytes of the thread's A row
    int ldb, N, n0;
    long long pb;
    __device__ BufOps(const float* A, int lda, int M, int gm, const __bf16* B, long long pb_, int ldb_, int N_, int n0_)
        : ldb(ldb_), N(N_), n0(n0_), pb(pb_) {
        sa = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), 0, M * lda * 4, 0x00020000);
        sb = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(B), 0, (int)((2 * pb_ + (long long)N_ * ldb_) * 2),
                                               0x00020000);
        arow_off = (unsigned)(gm * lda) * 4u;
    }
    // four floats of the thread's A row from column k (a multiple of 4)
    __device__ __forceinline__ float4 a4(int k, bool ok) const {
        const unsigned o = ok ? arow_off + 4u * (unsigned)k : 0x80000000u;
        return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(sa, (int)o, 0, 0));
    }
    // element e of the stage's B image (plane e >> 8, row (e & 255) >> 2, chunk e & 3) of the stage at k0
    __device__ __forceinline__ u32x4 b8(int e, int k0) const {
        const int pl = e >> 8, row = (e & 255) >> 2, kb = k0 + 8 * (e & 3), gn = n0 + row;
        const unsigned o = (gn < N && kb < ldb) ? (unsigned)((pl * pb + (long long)gn * ldb + kb) * 2) : 0x80000000u;
        return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(sb, (int)o, 0, 0));
    }
};

template <bool ID>
__global__ void __launch_bounds__(G_NT) k_gemm_bf3_fwd(const float* __restrict__ A, int lda,
                                                       const __bf16* __restrict__ B, long long pb, int ldb,
                                                       const int* __restrict__ m_valid, int m_cap, int N, int K,
                                                       float* __restrict__ Y, int ldy, const float* __restrict__ bias,
                                                       int relu_from, float* __restrict__ bn_part,
                                                       uint64_t* stamps, DiagIdArgs id, double* __restrict__ bn_acc,
                                                       FwdBnFin fin) {
    WaveStamp stamp(stamps);
    __shared__ __attribute__((aligned(16))) char lds[2 * G_STAGE];
    __shared__ float bn_mu[256], bn_sc[256];  // diagonal I / D columns: BN of x per channel
    const int M = m_valid ? *m_valid : m_cap;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv >> 1, wn = wv & 1;
    // the column tiles of a row tile on one XCD (blocks b and b + 8 share an XCD's L2): gridDim.x % 8 == 0,
    // so the row tile's aggregate rows come from HBM once
    const int L = blockIdx.x + gridDim.x * blockIdx.y, jj = L >> 3;
    const int by = jj % gridDim.y, bx = (L & 7) + 8 * (jj / gridDim.y);
    const int m0 = bx * G_BM, n0 = by * G_BN;
    if (M <= 0 && fin.ticket && bn_acc && L == 0) {  // no rows: the finalize of empty statistics (k_bn_finalize's)
        const float sf = (float)sqrt(1e-5);
        for (int ch = threadIdx.x; ch < N; ch += G_NT) {
            fin.mean[ch] = 0.f;
            fin.std[ch] = sf;
            if (fin.run_mean) {
                const float m1 = 1.0f - fin.momentum;
                fin.run_mean[ch] = __fadd_rn(__fmul_rn(m1, 0.f), __fmul_rn(fin.momentum, fin.run_mean[ch]));
                fin.run_std[ch] = __fadd_rn(__fmul_rn(m1, sf), __fmul_rn(fin.momentum, fin.run_std[ch]));
            }
        }
    }
    if (m0 >= M) return;
    // staging: A -- 64 rows x 4 chunks of 8 k, one chunk (two float4) per thread, split into the three
    // planes; B -- 3 planes x 64 rows x 4 chunks of 16 B, three per thread
    const int arow = tid >> 2, ach = tid & 3;
    // diagonal I / D columns (DiagIdArgs): logical k < kx read x (BN applied at the store, times the row's v_0 /
    // v_1); kx is a multiple of G_BK, so a stage is wholly of one kind
    const int kx = ID ? 2 * id.c : 0;
    float2 dg = make_float2(0.f, 0.f);
    float bnb = 0.f;
    if constexpr (ID) {
        for (int c = tid; c < id.c; c += G_NT) {
            const float w = *id.bn.w;
            bn_mu[c] = id.bn.mean[c];
            bn_sc[c] = bn_scale(w, id.bn.std[c]);
        }
        bnb = *id.bn.b;
        if (m0 + arow < M) dg = id.diag[m0 + arow];  // rows past M: coefficient 0, the operand 0
    }
    float4 ra[2];
    u32x4 rb[3];
    const BufOps bo(A, lda, M, m0 + arow, B, pb, ldb, N, n0);
    auto load = [&](int k0) {
        const int k = k0 + 8 * ach, gm = m0 + arow;
        if (ID && k0 < kx) {
            const int ch = k - (k >= id.c ? id.c : 0);
            const float* xp = id.x + (long long)gm * id.ldx + ch;
            ra[0] = gm < M ? *reinterpret_cast<const float4*>(xp) : make_float4(0.f, 0.f, 0.f, 0.f);
            ra[1] = gm < M ? *reinterpret_cast<const float4*>(xp + 4) : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
            ra[0] = bo.a4(k - kx, k < K);
            ra[1] = bo.a4(k - kx + 4, k + 4 < K);
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) rb[i] = bo.b8(tid + G_NT * i, k0);
    };
    auto store = [&](int buf, int k0) {
        char* st = lds + buf * G_STAGE;
        float xv[8] = {ra[0].x, ra[0].y, ra[0].z, ra[0].w, ra[1].x, ra[1].y, ra[1].z, ra[1].w};
        if (ID && k0 < kx) {  // v_j(r) * BN(x): the aggregation's fmaf(v_j, x̂, 0) of the diagonal entry
            const int k = k0 + 8 * ach, hi = k >= id.c, ch = k - (hi ? id.c : 0);
            const float v = hi ? dg.y : dg.x;
#pragma unroll
            for (int e = 0; e < 8; ++e) xv[e] = fmaf(v, bn_z_s(xv[e], bn_mu[ch + e], bn_sc[ch + e], bnb), 0.f);
        }
        bf16x8 p0, p1, p2;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            __bf16 a, b, c;
            split3(xv[e], a, b, c);
            p0[e] = a;
            p1[e] = b;
            p2[e] = c;
        }
        *reinterpret_cast<bf16x8*>(st + swz(arow, ach)) = p0;
        *reinterpret_cast<bf16x8*>(st + G_PLANE + swz(arow, ach)) = p1;
        *reinterpret_cast<bf16x8*>(st + 2 * G_PLANE + swz(arow, ach)) = p2;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int e = tid + G_NT * i, pl = e >> 8, row = (e & 255) >> 2, ch = e & 3;
            *reinterpret_cast<u32x4*>(st + (3 + pl) * G_PLANE + swz(row, ch)) = rb[i];
        }
    };
    f32x16 acc, tacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const int nt = (K + G_BK - 1) / G_BK;
    const int r31 = lane & 31, h = lane >> 5;
    const int frow = wm * 32 + r31, fcol = wn * 32 + r31;
    if constexpr (ID) __syncthreads();  // the BN table
    auto mma = [&](int t) {
        const char* st = lds + (t & 1) * G_STAGE;
#pragma unroll
        for (int r = 0; r < 16; ++r) tacc[r] = 0.f;
#pragma unroll
        for (int s = 0; s < G_BK / 16; ++s) {
            const int ch = 2 * s + h;
            bf16x8 a[3], b[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                a[p] = *reinterpret_cast<const bf16x8*>(st + p * G_PLANE + swz(frow, ch));
                b[p] = *reinterpret_cast<const bf16x8*>(st + (3 + p) * G_PLANE + swz(fcol, ch));
            }
            // the six terms with i + j <= 4, the small ones first
            tacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], tacc, 0, 0, 0);
            tacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], tacc, 0, 0, 0);
            tacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], tacc, 0, 0, 0);
            tacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], tacc, 0, 0, 0);
            tacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], tacc, 0, 0, 0);
            tacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], tacc, 0, 0, 0);
        }
    };
    load(0);
    store(0, 0);
    __syncthreads();
    load(G_BK);  // (past K: zeros, unused)
    // a branch-free body (the loads past K read zeros through the range check), so the split of stage t + 1 and the
    // MFMAs of stage t share one scheduling region; the last stage after the loop
    for (int t = 0; t + 1 < nt; ++t) {
        mma(t);
        store((t + 1) & 1, (t + 1) * G_BK);
        load((t + 2) * G_BK);
        acc += tacc;  // per-stage partial sums added to acc (fma chains of G_BK terms, as the fp32 GEMMs)
        __syncthreads();
    }
    mma(nt - 1);
    acc += tacc;
    // epilogue (k_gemm3 E3_FWD's): bias, ReLU, store, BN partials (count, mean, M2) per 64-row tile.
    // C/D layout of the 32x32 MFMA: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    float* red = reinterpret_cast<float*>(lds);  // free: the main loop ended with a barrier
    const int col = wn * 32 + r31, gn = n0 + col;
    const float bv = gn < N ? bias[gn] : 0.f;
    const bool relu = gn >= relu_from;
    float sm = 0.f;
    int cnt = 0;
    double s1 = 0.0, s2 = 0.0;  // bn_acc: fp64 sums of y and y^2 (each y^2 exact in fp64)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int gm = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        float v = acc[r] + bv;
        if (relu) v = v < 0.f ? 0.f : v;
        acc[r] = v;
        if (gm < M) {
            if (gn < N) Y[(long long)gm * ldy + gn] = v;
            sm += v;
            ++cnt;
            if (bn_acc) {
                s1 += (double)v;
                s2 = fma((double)v, (double)v, s2);
            }
        }
    }
    if (bn_acc) {
        // the tile's column sums: the two 32-lane halves (shuffle), the two row halves of the block (LDS), then one
        // no-return fp64 atomic per column and statistic into copy bx % BN_ACC_COPIES (spreads the adders)
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        double* redd = reinterpret_cast<double*>(lds);  // free: the main loop ended with a barrier
        if (lane < 32 && wm == 1) {
            redd[col] = s1;
            redd[G_BN + col] = s2;
        }
        __syncthreads();
        if (!fin.ticket) {
            if (lane < 32 && wm == 0 && gn < N) {
                double* dst = bn_acc + (long long)(bx % BN_ACC_COPIES) * 2 * N + gn;
                atomicAdd(dst, s1 + redd[col]);
                atomicAdd(dst + N, s2 + redd[G_BN + col]);
            }
            return;
        }
        // the finalize in the last block: returning atomics (performed before this block's ticket), the ticket, then the
        // last block reads the sums back with returning atomics (never a stale cache line) and finishes every channel
        __shared__ int last;
        __shared__ double sink[G_NT];
        double chk = 0.0;
        if (lane < 32 && wm == 0 && gn < N) {
            double* dst = bn_acc + (long long)(bx % BN_ACC_COPIES) * 2 * N + gn;
            chk += atomicAdd(dst, s1 + redd[col]);
            chk += atomicAdd(dst + N, s2 + redd[G_BN + col]);
        }
        sink[tid] = chk;
        __syncthreads();
        if (tid == 0) last = atomicAdd(fin.ticket, 1u) == (unsigned)(ceil_div(M, G_BM) * gridDim.y - 1);
        __syncthreads();
        if (!last) return;
        for (int ch = tid; ch < N; ch += G_NT) {
            double S = 0.0, Q = 0.0;
#pragma unroll
            for (int q = 0; q < BN_ACC_COPIES; ++q) {
                S += atomicAdd(bn_acc + ((long long)q * 2 + 0) * N + ch, 0.0);
                Q += atomicAdd(bn_acc + ((long long)q * 2 + 1) * N + ch, 0.0);
            }
            // k_bn_finalize's atomic form, bit for bit
            const double Nr = (double)M;
            const double mean = Nr > 0.0 ? S / Nr : 0.0;
            const double var = 1e-5 + (Nr > 0.0 ? fmax(Q / Nr - mean * mean, 0.0) : 0.0);
            const float mf = (float)mean;
            const float sf = (float)sqrt(var);
            fin.mean[ch] = mf;
            fin.std[ch] = sf;
            if (fin.run_mean) {
                const float m1 = 1.0f - fin.momentum;
                fin.run_mean[ch] = __fadd_rn(__fmul_rn(m1, mf), __fmul_rn(fin.momentum, fin.run_mean[ch]));
                fin.run_std[ch] = __fadd_rn(__fmul_rn(m1, sf), __fmul_rn(fin.momentum, fin.run_std[ch]));
            }
        }
        if (tid == 0) *fin.ticket = 0u;  // for the next half's GEMM (it follows this kernel's end)
        return;
    }
    if (!bn_part) return;
    sm += __shfl_xor(sm, 32, 64);
    cnt += __shfl_xor(cnt, 32, 64);
    if (lane < 32) {
        red[wm * G_BN + col] = sm;
        red[2 * G_BN + wm * G_BN + col] = (float)cnt;
    }
    __syncthreads();
    const float S = red[col] + red[G_BN + col];
    const float Cn = red[2 * G_BN + col] + red[3 * G_BN + col];
    const float mean = Cn > 0.f ? S / Cn : 0.f;
    __syncthreads();
    float q = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int gm = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (gm < M) {
            const float dl = acc[r] - mean;
            q = fmaf(dl, dl, q);
        }
    }
    q += __shfl_xor(q, 32, 64);
    if (lane < 32) red[wm * G_BN + col] = q;
    __syncthreads();
    if (wm == 0 && lane < 32 && gn < N) {
        float* pp = bn_part + ((long long)bx * N + gn) * 3;
        pp[0] = Cn;
        pp[1] = mean;
        pp[2] = red[col] + red[G_BN + col];
    }
}

// ---- dA on bf16 MFMA: Y[M][N] = A[M][K] . B[N][K]^T for a short reduction (K <= 32 NST: the 2d outputs of a
// Conv1d pair, 128 at d = 64), A = dY (fp32, split at staging), B = WT's three bf16 planes (the repack's wt3).
// k_gemm_bf3_fwd's tiles, LDS image and product order, but every stage's global loads are issued before the
// first is used (clamped addresses, zeroed after, so no exec branch splits them): four stages of 12 MFMAs
// per wave cannot hide a load round trip each, as the forward's one-stage-ahead prefetch asks.  Plain store.
template <int NST>
__global__ void __launch_bounds__(G_NT) k_gemm_bf3_da(const float* __restrict__ A, int lda,
                                                      const __bf16* __restrict__ B, long long pb, int ldb,
                                                      const int* __restrict__ m_valid, int m_cap, int N, int K,
                                                      float* __restrict__ Y, int ldy, uint64_t* stamps) {
    WaveStamp stamp(stamps);
    __shared__ __attribute__((aligned(16))) char lds[2 * G_STAGE];
    const int M = m_valid ? *m_valid : m_cap;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv >> 1, wn = wv & 1;
    const int L = blockIdx.x + gridDim.x * blockIdx.y, jj = L >> 3;  // (k_gemm_bf3_fwd's XCD mapping)
    const int by = jj % gridDim.y, bx = (L & 7) + 8 * (jj / gridDim.y);
    const int m0 = bx * G_BM, n0 = by * G_BN;
    if (m0 >= M) return;
    const int arow = tid >> 2, ach = tid & 3;
    const BufOps bo(A, lda, M, m0 + arow, B, pb, ldb, N, n0);
    float4 ra[NST][2];
    u32x4 rb[NST][3];
#pragma unroll
    for (int t = 0; t < NST; ++t) {
        const int k = t * G_BK + 8 * ach;
        ra[t][0] = bo.a4(k, k < K);
        ra[t][1] = bo.a4(k + 4, k + 4 < K);
#pragma unroll
        for (int i = 0; i < 3; ++i) rb[t][i] = bo.b8(tid + G_NT * i, t * G_BK);
    }
    auto store = [&](int buf, int t) {
        char* st = lds + buf * G_STAGE;
        const float xv[8] = {ra[t][0].x, ra[t][0].y, ra[t][0].z, ra[t][0].w,
                             ra[t][1].x, ra[t][1].y, ra[t][1].z, ra[t][1].w};
        bf16x8 p0, p1, p2;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            __bf16 a, b, c;
            split3(xv[e], a, b, c);
            p0[e] = a;
            p1[e] = b;
            p2[e] = c;
        }
        *reinterpret_cast<bf16x8*>(st + swz(arow, ach)) = p0;
        *reinterpret_cast<bf16x8*>(st + G_PLANE + swz(arow, ach)) = p1;
        *reinterpret_cast<bf16x8*>(st + 2 * G_PLANE + swz(arow, ach)) = p2;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const int e = tid + G_NT * i, pl = e >> 8, row = (e & 255) >> 2, ch = e & 3;
            *reinterpret_cast<u32x4*>(st + (3 + pl) * G_PLANE + swz(row, ch)) = rb[t][i];
        }
    };
    f32x16 acc, tacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    const int r31 = lane & 31, h = lane >> 5;
    const int frow = wm * 32 + r31, fcol = wn * 32 + r31;
    store(0, 0);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < NST; ++t) {
        const char* st = lds + (t & 1) * G_STAGE;
#pragma unroll
        for (int r = 0; r < 16; ++r) tacc[r] = 0.f;
#pragma unroll
        for (int s = 0; s < G_BK / 16; ++s) {
            const int ch = 2 * s + h;
            bf16x8 a[3], b[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                a[p] = *reinterpret_cast<const bf16x8*>(st + p * G_PLANE + swz(frow, ch));
                b[p] = *reinterpret_cast<const bf16x8*>(st + (3 + p) * G_PLANE + swz(fcol, ch));
            }
            tacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], tacc, 0, 0, 0);
            tacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], tacc, 0, 0, 0);
            tacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], tacc, 0, 0, 0);
            tacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], tacc, 0, 0, 0);
            tacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], tacc, 0, 0, 0);
            tacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], tacc, 0, 0, 0);
        }
        acc += tacc;
        if (t + 1 < NST) store((t + 1) & 1, t + 1);
        __syncthreads();
    }
    const int gn = n0 + wn * 32 + r31;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M && gn < N) Y[(long long)m * ldy + gn] = acc[r];
    }
}

// ---- dW on bf16 MFMA: slabs[z][m][n] = sum_{r in chunk z} A[r][m] B[r][n] (k_gemm3_tn's contract: A = dY
// [R][lda], m < M = 2d; B = the saved aggregate [R][ldb], n < N = kp; chunk z of dw3_kc(R, nz) rows), each
// operand split into three bf16 planes at staging and the six products with i + j <= 4 summed on
// v_mfma_f32_32x32x16_bf16 -- the fp32 version is bound by its MFMA issue (8 x 64 cycles per 32x32x16 step
// of a wave against 6 x 32 here).  Block 128 x 128, 8 waves of 32 x 64; stages of 16 rows.  The reduction
// index is the row r, so the LDS planes hold the transposed image [m][16 r] (32 B per m, the two 16-B halves
// swapped by bit 3 of m: conflict-free ds_read_b128 fragments); a thread stages one column and four rows of
// each operand (scalar loads, 256 B per wave instruction).  A stage is short (12 MFMAs per wave), so the
// global loads run PD - 1 stages ahead in a register ring.
constexpr int D_BK = 16, D_NT = 512, D_ROWB = D_BK * 2, D_PLANE = 128 * D_ROWB, D_STAGE = 6 * D_PLANE;

__device__ __forceinline__ int dswz(int m, int ch) { return m * D_ROWB + 16 * (ch ^ ((m >> 3) & 1)); }

// The ring (round 5; the first form, k_gemm_bf3_tn, was retired in round 6): the loads unconditional (clamped row and column, the
// out-of-range values zeroed at the split), no branch inside the unrolled stage group (the stages past the
// chunk's last run on zeroed planes and add nothing), and each group of loads pinned where it is issued --
// the conditional loads and the in-loop breaks of the first form left a vmcnt(0) before every stage, so its
// ring never had a load in flight across a stage.
// VIRT: the block's 128 output columns are diagonal I / D columns (DiagIdArgs; n0 < kx, kx a multiple of 128):
// the B operand is v_j(r) * BN(x[r][ch]) built at the split from x and the row's diag coefficient, loaded by the
// same ring; otherwise B is the aggregate's column n - kx.
template <int PD, bool VIRT>
__device__ __forceinline__ void dw_ring_body(char* lds, const float* __restrict__ A, int lda, const float* __restrict__ B,
                                             int ldb, float* __restrict__ slabs, int M, int N, int m0, int n0, int bz,
                                             int kbeg, int kend, const DiagIdArgs& id, int kx) {
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv >> 1, wn = wv & 1;
    const int col = tid & 127, rq = tid >> 7;
    const int n = n0 + col;
    const bool am = m0 + col < M, bn = n < N;
    const float* ap = A + min(m0 + col, M - 1);
    const float* bp;
    const float* cp = nullptr;  // VIRT: the row's coefficient (v_0 or v_1 of diag[r])
    long long ldbb = ldb;
    float mu = 0.f, sc = 1.f, bb = 0.f;
    if constexpr (VIRT) {
        const int hi = n >= id.c, ch = n - (hi ? id.c : 0);
        bp = id.x + ch;
        ldbb = id.ldx;
        cp = reinterpret_cast<const float*>(id.diag) + hi;
        mu = id.bn.mean[ch];
        sc = bn_scale(*id.bn.w, id.bn.std[ch]);
        bb = *id.bn.b;
    } else {
        bp = B + min(n, N - 1) - kx;
    }
    constexpr int NC = VIRT ? 4 : 1;
    float ra[PD][4], rb[PD][4], rc[PD][NC];
    // the aggregate columns (not VIRT): buffer loads through a descriptor re-based on the stage's first row, whose
    // record count ends at the chunk's last row -- the range check returns 0 for rows past kend and for the
    // out-of-range columns (their lane offset is 2^31, past any record count), so the per-lane offsets are
    // loop-invariant and neither a row clamp nor the masks at the split are needed (the clamped form spent 25 of
    // its ~100 VALU instructions per stage on 64-bit row addresses)
    unsigned voa[4], vob[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        voa[i] = am ? (unsigned)(((4 * rq + i) * lda + m0 + col) * 4) : 0x80000000u;
        vob[i] = bn ? (unsigned)(((4 * rq + i) * ldb + n - kx) * 4) : 0x80000000u;
    }
    auto load = [&](float (&xa)[4], float (&xb)[4], float (&xc)[NC], int k0) {
        if constexpr (VIRT) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const long long gk = min(k0 + 4 * rq + i, kend - 1);
                xa[i] = ap[gk * lda];
                xb[i] = bp[gk * ldbb];
                xc[i] = cp[2 * gk];
            }
        } else {
            const int rows = max(kend - k0, 0);
            const auto sa = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A) + (long long)k0 * lda, 0,
                                                              rows * lda * 4, 0x00020000);
            const auto sb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(B) + (long long)k0 * ldb, 0,
                                                              rows * ldb * 4, 0x00020000);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                xa[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(sa, (int)voa[i], 0, 0));
                xb[i] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(sb, (int)vob[i], 0, 0));
            }
        }
    };
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    auto store = [&](const float (&xa)[4], const float (&xb)[4], const float (&xc)[NC], int buf, int k0) {
        char* st = lds + buf * D_STAGE;
        const int off = dswz(col, rq >> 1) + (rq & 1) * 8;
        bf16x4 p[3], q[3];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const bool in = !VIRT || (k0 + 4 * rq + i < kend);  // VIRT: clamped loads, masked here
            __bf16 x, y, z;
            split3(in && (!VIRT || am) ? xa[i] : 0.f, x, y, z);
            p[0][i] = x;
            p[1][i] = y;
            p[2][i] = z;
            float bv = xb[i];
            if constexpr (VIRT) bv = fmaf(xc[i], bn_z_s(bv, mu, sc, bb), 0.f);  // the aggregation's value
            split3(in && (!VIRT || bn) ? bv : 0.f, x, y, z);
            q[0][i] = x;
            q[1][i] = y;
            q[2][i] = z;
        }
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
            *reinterpret_cast<bf16x4*>(st + pl * D_PLANE + off) = p[pl];
            *reinterpret_cast<bf16x4*>(st + (3 + pl) * D_PLANE + off) = q[pl];
        }
    };
    f32x16 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    const int nt = (kend - kbeg + D_BK - 1) / D_BK;
    const int r31 = lane & 31, h = lane >> 5;
#pragma unroll
    for (int u = 0; u < PD; ++u) load(ra[u], rb[u], rc[u], kbeg + u * D_BK);
    __builtin_amdgcn_sched_barrier(0);
    store(ra[0], rb[0], rc[0], 0, kbeg);
    __syncthreads();
    for (int t0 = 0; t0 < nt; t0 += PD) {
#pragma unroll
        for (int u = 0; u < PD; ++u) {
            const int t = t0 + u;
            const char* st = lds + (t & 1) * D_STAGE;
            bf16x8 a[3], b[2][3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
                a[pl] = *reinterpret_cast<const bf16x8*>(st + pl * D_PLANE + dswz(wm * 32 + r31, h));
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    b[j][pl] = *reinterpret_cast<const bf16x8*>(st + (3 + pl) * D_PLANE + dswz(wn * 64 + j * 32 + r31, h));
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[j][1], acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[j][2], acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[j][0], acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[j][1], acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[j][0], acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[j][0], acc[j], 0, 0, 0);
            }
            const int un = (u + 1) % PD;  // the slot holding stage t + 1
            store(ra[un], rb[un], rc[un], (t + 1) & 1, kbeg + (t + 1) * D_BK);
            load(ra[u], rb[u], rc[u], kbeg + (t + PD) * D_BK);  // slot u (stage t, staged) takes stage t + PD
            __builtin_amdgcn_sched_barrier(0);
            __syncthreads();
        }
    }
    float* out = slabs + (long long)bz * M * N;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int gn = n0 + wn * 64 + j * 32 + r31;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int gm = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (gm < M && gn < N) out[(long long)gm * N + gn] = acc[j][r];
        }
    }
}

template <int PD, bool ID>
__global__ void __launch_bounds__(D_NT) k_gemm_bf3_tn_ring(const float* __restrict__ A, int lda,
                                                           const float* __restrict__ B, int ldb,
                                                           float* __restrict__ slabs, int M, int N,
                                                           const int* __restrict__ r_valid, int nz, int xcd_remap,
                                                           uint64_t* stamps, DiagIdArgs id) {
    WaveStamp stamp(stamps);
    static_assert(PD >= 2, "a ring of at least two stages");
    __shared__ __attribute__((aligned(16))) char lds[2 * D_STAGE];
    int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if (xcd_remap) {
        const int T = gridDim.x * gridDim.y;
        const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        const int j = L >> 3, t = j % T;
        bz = (L & 7) + 8 * (j / T);
        bx = t % gridDim.x;
        by = t / gridDim.x;
    }
    const int m0 = bx * 128, n0 = by * 128;
    const int R = *r_valid;
    const int kchunk = dw3_kc(R, nz);
    const int kbeg = bz * kchunk, kend = min(R, kbeg + kchunk);
    if (kbeg >= kend) return;
    const int kx = ID ? 2 * id.c : 0;
    if constexpr (ID) {
        if (n0 < kx) {
            dw_ring_body<(PD > 3 ? PD - 1 : PD), true>(lds, A, lda, B, ldb, slabs, M, N, m0, n0, bz, kbeg, kend, id, kx);
            return;
        }
    }
    dw_ring_body<PD, false>(lds, A, lda, B, ldb, slabs, M, N, m0, n0, bz, kbeg, kend, id, kx);
}

// BufOps' 32-bit byte offsets: the rows a block can name (m_cap + 64) and the three weight planes below 2^29 elements
bool bufops_ok(int m_cap, int lda, long long pb, int ldb, int n) {
    return (long long)(m_cap + G_BM) * lda < (1ll << 29) && 3 * pb < (1ll << 29) && (long long)n * ldb <= pb;
}

// the diagonal I / D columns' contract (DiagIdArgs): 2c a multiple of 32, c <= 256, float4-aligned x rows
bool diag_id_ok(const DiagIdArgs* id, int k) {
    return id->x && id->diag && id->bn.mean && id->bn.std && id->bn.w && id->bn.b && id->c > 0 && id->c <= 256 &&
           (2 * id->c) % 32 == 0 && id->ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(id->x) & 15) == 0 &&
           2 * id->c < k;
}

}  // namespace

int launch_gemm_bf3_dw(const float* dy, int lddy, const float* a, int lda, const int* r_valid, int r_cap, int o,
                       int k, int nz, float* slabs, int xcd, hipStream_t s, const DiagIdArgs* id) {
    if (r_cap <= 0) return 0;
    if (nz <= 0) return HGNN_ERR_ARG;
    // the ring's buffer descriptors hold a chunk's bytes in a 31-bit record count
    if ((long long)r_cap * (lda > lddy ? lda : lddy) >= (1ll << 29)) return HGNN_ERR_UNSUPPORTED;
    // diagonal I / D columns: whole 128-column output tiles (kx a multiple of 128), the ring kernel
    if (id && (!diag_id_ok(id, k) || (2 * id->c) % 128 || (long long)r_cap * id->ldx >= (1ll << 31)))
        return HGNN_ERR_UNSUPPORTED;
    const DiagIdArgs none{};
    const DiagIdArgs ida = id ? *id : none;
    // ring depth 4 (k_gemm_bf3_tn_ring<4>, round 5: 1.1038 vs 1.1146 ms median over eight alternating pairs against
    // the retired unringed form; depth 3 bimodal, depth 2 slower -- DESIGN.md §8 round 5)
    const dim3 g(ceil_div(o, 128), ceil_div(k, 128), nz);
    static const int ring = [] {  // HGNN_DW_RING: 2..4 = k_gemm_bf3_tn_ring<depth>
        const char* e = getenv("HGNN_DW_RING");
        const int v = e ? atoi(e) : 4;
        return v < 2 ? 2 : (v > 4 ? 4 : v);
    }();
    uint64_t* st = clock_stamps((long long)g.x * g.y * g.z * (D_NT / 64));
    const int xr = xcd && nz % 8 == 0 ? 1 : 0;
#define HGNN_DW_RING_LAUNCH(D, I) \
    HGNN_KLAUNCH((k_gemm_bf3_tn_ring<D, I>), g, dim3(D_NT), 0, s, dy, lddy, a, lda, slabs, o, k, r_valid, nz, xr, st, ida)
    switch (ring * 2 + (id ? 1 : 0)) {
        case 4: HGNN_DW_RING_LAUNCH(2, false); break;
        case 5: HGNN_DW_RING_LAUNCH(2, true); break;
        case 6: HGNN_DW_RING_LAUNCH(3, false); break;
        case 7: HGNN_DW_RING_LAUNCH(3, true); break;
        case 9: HGNN_DW_RING_LAUNCH(4, true); break;
        default: HGNN_DW_RING_LAUNCH(4, false); break;
    }
#undef HGNN_DW_RING_LAUNCH
    HGNN_LAUNCH_CHECK();
    return 0;
}

int launch_gemm_bf3_da(const float* a, int lda, const int* m_valid, int m_cap, int k, const __bf16* b, long long pb,
                       int ldb, int n, float* y, int ldy, hipStream_t s) {
    if (m_cap <= 0 || n <= 0) return 0;
    if (k < 4 || k > 4 * G_BK || lda % 4 || k % 4 || ldb % 8 || pb % 8 || k > lda || bf3_ld(k) > ldb ||
        (reinterpret_cast<uintptr_t>(a) & 15) || (reinterpret_cast<uintptr_t>(b) & 15))
        return HGNN_ERR_UNSUPPORTED;
    if (!bufops_ok(m_cap, lda, pb, ldb, n)) return HGNN_ERR_UNSUPPORTED;
    const int gx = ceil_div(ceil_div(m_cap, G_BM), 8) * 8;
    const dim3 g(gx, ceil_div(n, G_BN));
    uint64_t* st = clock_stamps((long long)g.x * g.y * (G_NT / 64));
    switch (ceil_div(k, G_BK)) {
        case 1: HGNN_KLAUNCH(k_gemm_bf3_da<1>, g, dim3(G_NT), 0, s, a, lda, b, pb, ldb, m_valid, m_cap, n, k, y, ldy, st); break;
        case 2: HGNN_KLAUNCH(k_gemm_bf3_da<2>, g, dim3(G_NT), 0, s, a, lda, b, pb, ldb, m_valid, m_cap, n, k, y, ldy, st); break;
        case 3: HGNN_KLAUNCH(k_gemm_bf3_da<3>, g, dim3(G_NT), 0, s, a, lda, b, pb, ldb, m_valid, m_cap, n, k, y, ldy, st); break;
        default: HGNN_KLAUNCH(k_gemm_bf3_da<4>, g, dim3(G_NT), 0, s, a, lda, b, pb, ldb, m_valid, m_cap, n, k, y, ldy, st); break;
    }
    HGNN_LAUNCH_CHECK();
    return 0;
}

int launch_gemm_bf3_fwd(const float* a, int lda, const int* m_valid, int m_cap, int k, const __bf16* b, long long pb,
                        int ldb, int n, const float* bias, int relu_from, float* y, int ldy, float* bn_part,
                        hipStream_t s, const DiagIdArgs* id, double* bn_acc, const FwdBnFin* fin) {
    if (m_cap <= 0 || n <= 0) return 0;
    if (fin && (!bn_acc || !fin->mean || !fin->std || !fin->ticket)) return HGNN_ERR_ARG;
    const int kx = id ? 2 * id->c : 0;
    if (id && !diag_id_ok(id, k)) return HGNN_ERR_UNSUPPORTED;
    if (lda % 4 || k % 4 || ldb % 8 || pb % 8 || k - kx > lda || bf3_ld(k) > ldb ||
        (reinterpret_cast<uintptr_t>(a) & 15) || (reinterpret_cast<uintptr_t>(b) & 15))
        return HGNN_ERR_UNSUPPORTED;
    if (!bufops_ok(m_cap, lda, pb, ldb, n)) return HGNN_ERR_UNSUPPORTED;
    if (id && (long long)m_cap * id->ldx * 4 >= (1ll << 31)) return HGNN_ERR_UNSUPPORTED;
    const int gx = ceil_div(ceil_div(m_cap, G_BM), 8) * 8;
    const dim3 g(gx, ceil_div(n, G_BN));
    const DiagIdArgs none{};
    const FwdBnFin nofin{};
    const FwdBnFin& fb = fin ? *fin : nofin;
    if (id)
        HGNN_KLAUNCH(k_gemm_bf3_fwd<true>, g, dim3(G_NT), 0, s, a, lda, b, pb, ldb, m_valid, m_cap, n, k, y, ldy, bias,
                     relu_from, bn_part, clock_stamps((long long)g.x * g.y * (G_NT / 64)), *id, bn_acc, fb);
    else
        HGNN_KLAUNCH(k_gemm_bf3_fwd<false>, g, dim3(G_NT), 0, s, a, lda, b, pb, ldb, m_valid, m_cap, n, k, y, ldy, bias,
                     relu_from, bn_part, clock_stamps((long long)g.x * g.y * (G_NT / 64)), none, bn_acc, fb);
    HGNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace hgnn
