// GEMM v3 ("NT"): C[M][N] = A[M][K] . B[N][K]^T with both operands k-contiguous,
// fp32 MFMA v_mfma_f32_32x32x2_f32.
//
// Forward:  Y[rows][2d]  = Agg[rows][kp] . Wcat[2d][kp]^T  (+ bias, ReLU half, BN partials)
// dA:       dA[rows][K]  = dY[rows][2d]  . WT[K][2d]^T
// Both operands are staged global -> registers -> LDS with float4 loads into
// k-contiguous LDS rows (stride BK + 4 floats: conflict-free ds_read_b128), so
// no transpose happens anywhere.  The k order inside a BK tile is permuted:
// MFMA step s contracts k = s (lanes 0-31) and k = BK/2 + s (lanes 32-63); the
// same permutation on A and B leaves the sum unchanged, and one ds_read_b128
// per operand then feeds 4 consecutive MFMA steps.  Measured on the box
// (the round-1 GEMM lab; tools/gemm4_lab.hip is the current one) against v2 on the config-2 shapes: node fwd 57 -> 30 us,
// edge fwd 79 -> 51 us, edge dA 64 -> 48 us.
#include <stdlib.h>

#include <algorithm>

#include "kernels.h"

namespace hgnn {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---- Diagnostic build only (make EXTRA=-DHGNN_CLOCK_DIAG into its own BUILD / OUT, tools/clock_diag.py):
// wave 0 of every block stamps the shader clock (s_memtime, shader cycles) and the constant 100 MHz
// clock (s_memrealtime) around the GEMM main loop, so clock = d(memtime) / d(memrealtime) x 100 MHz
// (MI355X_MICROARCH.md, DVFS give-back item 6).  In the normal build no stamp exists.
#ifdef HGNN_CLOCK_DIAG
constexpr unsigned CLOCK_SLOTS = 1u << 16;
struct ClockStamp {
    unsigned long long dt, dr;
    unsigned kid, pad;
};
__device__ ClockStamp g_clock[CLOCK_SLOTS];
__device__ unsigned g_clock_n;
#define CLK_BEGIN()                                  \
    unsigned long long _clk_t0 = 0, _clk_r0 = 0;     \
    if (threadIdx.x == 0) {                          \
        _clk_t0 = __builtin_amdgcn_s_memtime();      \
        _clk_r0 = __builtin_amdgcn_s_memrealtime();  \
    }
#define CLK_END(KID_)                                                       \
    if (threadIdx.x == 0) {                                                 \
        const unsigned long long _t1 = __builtin_amdgcn_s_memtime();        \
        const unsigned long long _r1 = __builtin_amdgcn_s_memrealtime();    \
        const unsigned _i = atomicAdd(&g_clock_n, 1u);                      \
        if (_i < CLOCK_SLOTS) {                                             \
            g_clock[_i].dt = _t1 - _clk_t0;                                 \
            g_clock[_i].dr = _r1 - _clk_r0;                                 \
            g_clock[_i].kid = (KID_);                                       \
        }                                                                   \
    }
// Phase stamps of the dW GEMM (same diagnostic build, tools/dw_phases.py): thread 0 of every block records
// s_memrealtime (100 MHz, chip-wide) at entry, loop start, loop end and exit, plus the CU it ran on (HW_ID,
// XCC_ID), so a launch's span splits into block start-up, main loop, epilogue and late (second-round or
// CU-waiting) blocks.  Stored with vector stores from thread 0.
constexpr unsigned PHASE_SLOTS = 1u << 17;
struct PhaseStamp {
    unsigned long long t[4];
    unsigned hw, xcc, blk, rows;
};
__device__ PhaseStamp g_phase[PHASE_SLOTS];
__device__ unsigned g_phase_n;
#define PH_DECL() unsigned long long _ph[4] = {0ull, 0ull, 0ull, 0ull};
#define PH_MARK(I_)                                                     \
    if (threadIdx.x == 0) _ph[I_] = __builtin_amdgcn_s_memrealtime();
#define PH_FLUSH(ROWS_)                                                                               \
    if (threadIdx.x == 0) {                                                                           \
        _ph[3] = __builtin_amdgcn_s_memrealtime();                                                    \
        const unsigned _i = atomicAdd(&g_phase_n, 1u);                                                \
        if (_i < PHASE_SLOTS) {                                                                       \
            PhaseStamp& _s = g_phase[_i];                                                             \
            _s.t[0] = _ph[0];                                                                         \
            _s.t[1] = _ph[1];                                                                         \
            _s.t[2] = _ph[2];                                                                         \
            _s.t[3] = _ph[3];                                                                         \
            _s.hw = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);                              \
            _s.xcc = (unsigned)__builtin_amdgcn_s_getreg((15 << 11) | 20);                            \
            _s.blk = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);                  \
            _s.rows = (unsigned)(ROWS_);                                                              \
        }                                                                                             \
    }
#else
#define CLK_BEGIN()
#define CLK_END(KID_)
#define PH_DECL()
#define PH_MARK(I_)
#define PH_FLUSH(ROWS_)
#endif

namespace {

enum { E3_FWD = 0, E3_STORE = 1 };

struct G3 {
    const float* a;
    int lda;
    const float* b;
    int ldb;
    int m_cap;
    const int* m_valid;
    int k;
    int n;
    float* c;
    int ldc;
    const float* bias;
    int relu_from;
    float* bn_part;  // [ceil(m_cap / 64)][n][3] (count, mean, M2)
    int xcd;            // E3_FWD: the column tiles of a row tile on one XCD (gridDim.x % 8 == 0)
};

template <int BM, int BN, int BK, int WGM, int WGN, int EPI>
__global__ void __launch_bounds__(64 * WGM * WGN) k_gemm3(G3 p) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int TM = BM / WGM, TN = BN / WGN, AM = TM / 32, AN = TN / 32;
    constexpr int LDK = BK + 4;
    constexpr int AF4 = BM * BK / 4 / NT, BF4 = BN * BK / 4 / NT;
    static_assert(AF4 >= 1 && BF4 >= 1 && AM >= 1 && AN >= 1, "tile shape");
    static_assert(EPI != E3_FWD || (BM == 64 && WGM == 2), "BN partials are per 64-row tile");
    __shared__ __attribute__((aligned(16))) float As[2][BM * LDK];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDK];

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv / WGN, wn = wv % WGN;
    int bx = blockIdx.x, by = blockIdx.y;
    if (EPI == E3_FWD && p.xcd) {
        // blocks b and b + 8 share an XCD's L2 (MI355X_MICROARCH.md): the gridDim.y column tiles
        // of one row tile get equal b % 8, so its A rows (the wide aggregate) come from HBM once
        const int L = blockIdx.x + gridDim.x * blockIdx.y, j = L >> 3;
        by = j % gridDim.y;
        bx = (L & 7) + 8 * (j / gridDim.y);
    }
    const int m0 = bx * BM, n0 = by * BN;
    const int Mv = p.m_valid ? *p.m_valid : p.m_cap;
    if (m0 >= Mv) return;
    const int K = p.k, N = p.n;

    // K % 4 == 0 (host-checked): a float4 is wholly inside or outside the k range, so the
    // loads' range checks are the only masking (the forward GEMM runs over the padded width kp,
    // whose padding columns are zero in both operands).  A per-element tail select in the
    // staging doubled the k-loop's instruction count (321 vs 204 per k-step) and cost ~5 us
    // per launch (round-1 GEMM lab).
    float4 ra[AF4], rb[BF4];
    // Loads are unconditional buffer loads: an out-of-range float4 gets an out-of-bounds offset
    // and reads 0 in hardware.  A conditional load made the compiler merge the loaded and the
    // zero value with register moves straight after the load, i.e. a vmcnt(0) in the middle of
    // the prefetch (seen in the .s of the forward variant); a select at the LDS store moved the
    // staging arrays to scratch; a pointer select with a zero constant became flat loads.
    // buffer resources over the valid rows: an out-of-range float4 gets offset OOB and reads 0
    constexpr unsigned OOB = 0x7ffffff0u;
    const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.a), 0, Mv * p.lda * 4, 0x00020000);
    const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.b), 0, N * p.ldb * 4, 0x00020000);
    auto ld4 = [](__amdgpu_buffer_rsrc_t r, unsigned off) {
        return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
    };
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            const int gm = m0 + row, gk = k0 + kq;
            const unsigned off = (gm < Mv && gk < K) ? (unsigned)(gm * p.lda + gk) * 4u : OOB;
            ra[i] = ld4(rs_a, off);
        }
#pragma unroll
        for (int i = 0; i < BF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            const int gn = n0 + row, gk = k0 + kq;
            const unsigned off = (gn < N && gk < K) ? (unsigned)(gn * p.ldb + gk) * 4u : OOB;
            rb[i] = ld4(rs_b, off);
        }
    };
    auto store = [&](int buf, int k0) {
        (void)k0;
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            *reinterpret_cast<float4*>(&As[buf][row * LDK + kq]) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < BF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            *reinterpret_cast<float4*>(&Bs[buf][row * LDK + kq]) = rb[i];
        }
    };

    // Each BK-deep k tile is summed by the MFMAs into a fresh accumulator (tacc) and added to
    // acc afterwards: fma chains of BK instead of K (640) terms.  Measured on the box: the
    // one-chain version's outputs were 1.0-1.5x twice the reference fp32 error against fp64
    // (SURVEY §8 c second leg) on the bs=128 / bs=512 d=128 tests; the split costs 16 VALU adds
    // per 16 MFMAs.
    f32x16 acc[AM][AN], tacc[AM][AN];
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nt = ceil_div(K, BK);
    const int h = lane >> 5, l31 = lane & 31;
    CLK_BEGIN()
    load(0);
    store(0, 0);
    __syncthreads();
    if (nt > 1) load(BK);
    for (int t = 0; t < nt; ++t) {
        const int buf = t & 1;
        const float* as = &As[buf][(wm * TM + l31) * LDK + h * (BK / 2)];
        const float* bs = &Bs[buf][(wn * TN + l31) * LDK + h * (BK / 2)];
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
            for (int j = 0; j < AN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) tacc[i][j][r] = 0.f;
#pragma unroll
        for (int g = 0; g < BK / 8; ++g) {
            float4 a[AM], b[AN];
#pragma unroll
            for (int i = 0; i < AM; ++i) a[i] = *reinterpret_cast<const float4*>(as + i * 32 * LDK + 4 * g);
#pragma unroll
            for (int j = 0; j < AN; ++j) b[j] = *reinterpret_cast<const float4*>(bs + j * 32 * LDK + 4 * g);
#pragma unroll
            for (int i = 0; i < AM; ++i)
#pragma unroll
                for (int j = 0; j < AN; ++j) {
                    tacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, tacc[i][j], 0, 0, 0);
                    tacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, tacc[i][j], 0, 0, 0);
                    tacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, tacc[i][j], 0, 0, 0);
                    tacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, tacc[i][j], 0, 0, 0);
                }
        }
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
            for (int j = 0; j < AN; ++j) acc[i][j] += tacc[i][j];
        if (t + 1 < nt) {
            store(buf ^ 1, (t + 1) * BK);
            if (t + 2 < nt) load((t + 2) * BK);
        }
        __syncthreads();
    }
    CLK_END(EPI == E3_FWD ? 0u : 1u)

    // C/D layout of the 32x32 MFMA: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    if constexpr (EPI == E3_FWD) {
        float* red = &As[0][0];  // [2][BN] sums + [2][BN] counts, then [2][BN] M2
        float s[AN];
        int cnt[AN];
#pragma unroll
        for (int j = 0; j < AN; ++j) {
            const int gn = n0 + wn * TN + j * 32 + l31;
            const float bias = gn < N ? p.bias[gn] : 0.f;
            const bool relu = gn >= p.relu_from;
            s[j] = 0.f;
            cnt[j] = 0;
#pragma unroll
            for (int i = 0; i < AM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int gm = m0 + wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    float v = acc[i][j][r] + bias;
                    if (relu) v = v < 0.f ? 0.f : v;
                    acc[i][j][r] = v;
                    if (gm < Mv) {
                        if (gn < N) p.c[(long long)gm * p.ldc + gn] = v;
                        s[j] += v;
                        ++cnt[j];
                    }
                }
        }
        if (p.bn_part) {
            float mean[AN];
#pragma unroll
            for (int j = 0; j < AN; ++j) {
                s[j] += __shfl_xor(s[j], 32, 64);
                cnt[j] += __shfl_xor(cnt[j], 32, 64);
                const int col = wn * TN + j * 32 + l31;
                if (lane < 32) {
                    red[wm * BN + col] = s[j];
                    red[2 * BN + wm * BN + col] = (float)cnt[j];
                }
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < AN; ++j) {
                const int col = wn * TN + j * 32 + l31;
                const float S = red[col] + red[BN + col];
                const float C = red[2 * BN + col] + red[3 * BN + col];
                mean[j] = C > 0.f ? S / C : 0.f;
                cnt[j] = (int)C;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < AN; ++j) {
                float q = 0.f;
#pragma unroll
                for (int i = 0; i < AM; ++i)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int gm = m0 + wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                        if (gm < Mv) {
                            const float dl = acc[i][j][r] - mean[j];
                            q = fmaf(dl, dl, q);
                        }
                    }
                q += __shfl_xor(q, 32, 64);
                const int col = wn * TN + j * 32 + l31;
                if (lane < 32) red[wm * BN + col] = q;
            }
            __syncthreads();
            if (wm == 0 && lane < 32) {
#pragma unroll
                for (int j = 0; j < AN; ++j) {
                    const int col = wn * TN + j * 32 + l31;
                    const int gn = n0 + col;
                    if (gn < N) {
                        float* pp = p.bn_part + ((long long)bx * N + gn) * 3;
                        pp[0] = (float)cnt[j];
                        pp[1] = mean[j];
                        pp[2] = red[col] + red[BN + col];
                    }
                }
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
            for (int j = 0; j < AN; ++j) {
                const int gn = n0 + wn * TN + j * 32 + l31;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int gm = m0 + wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (gm < Mv && gn < N) p.c[(long long)gm * p.ldc + gn] = acc[i][j][r];
                }
            }
    }
}

// dW ("TN"): slabs[z][m][n] = sum_{r in chunk z} A[r][m] B[r][n], with A = dY [R][2d] and
// B = the saved aggregate [R][kp].  Both operands are reduction-major, so LDS keeps
// the natural [k][m] image (float4 copies) and fragments are ds_read_b32, with the
// same k permutation and a one-step register prefetch of the next fragments.
// Measured (round-1 GEMM lab, config-2 shapes): edge 78 -> 41 us, node 37.5 -> 21 us vs v2.
template <int BM, int BN, int BK, int WGM, int WGN>
__global__ void __launch_bounds__(64 * WGM * WGN) k_gemm3_tn(const float* __restrict__ A, int lda,
                                                             const float* __restrict__ B, int ldb,
                                                             float* __restrict__ slabs, int M, int N,
                                                             const int* __restrict__ r_valid, int nz,
                                                             int xcd_remap) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int TM = BM / WGM, TN = BN / WGN, AM = TM / 32, AN = TN / 32;
    constexpr int PA = BM + 4, PB = BN + 4;
    constexpr int AF4 = BM * BK / 4 / NT, BF4 = BN * BK / 4 / NT;
    static_assert(AF4 >= 1 && BF4 >= 1 && AM >= 1 && AN >= 1, "tile shape");
    static_assert(AF4 * 4 * NT == BM * BK && BF4 * 4 * NT == BN * BK, "staging must cover the tile");
    __shared__ __attribute__((aligned(16))) float As[2][BK * PA];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK * PB];
    PH_DECL()
    PH_MARK(0)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv / WGN, wn = wv % WGN;
    int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if (xcd_remap) {
        // the output tiles of one row chunk on one XCD (blocks b and b + 8 share an XCD's L2,
        // MI355X_MICROARCH.md), so the chunk's dY rows are fetched from HBM once, not once per
        // tile; gridDim.z is a multiple of 8 here
        const int T = gridDim.x * gridDim.y;
        const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        const int j = L >> 3, t = j % T;
        bz = (L & 7) + 8 * (j / T);
        bx = t % gridDim.x;
        by = t / gridDim.x;
    }
    const int m0 = bx * BM, n0 = by * BN;
    const int R = *r_valid;
    const int kchunk = dw3_kc(R, nz);
    const int kbeg = bz * kchunk, kend = min(R, kbeg + kchunk);
    if (kbeg >= kend) {  // the reduce only sums the chunks that hold rows
        PH_FLUSH(0)
        return;
    }
    float4 ra[AF4], rb[BF4];
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int e = tid + i * NT, kr = e / (BM / 4), mq = (e % (BM / 4)) * 4;
            const int gk = k0 + kr, gm = m0 + mq;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (gk < kend && gm < M) v = *reinterpret_cast<const float4*>(A + (long long)gk * lda + gm);
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < BF4; ++i) {
            const int e = tid + i * NT, kr = e / (BN / 4), nq = (e % (BN / 4)) * 4;
            const int gk = k0 + kr, gn = n0 + nq;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (gk < kend && gn < N) v = *reinterpret_cast<const float4*>(B + (long long)gk * ldb + gn);
            rb[i] = v;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int e = tid + i * NT, kr = e / (BM / 4), mq = (e % (BM / 4)) * 4;
            *reinterpret_cast<float4*>(&As[buf][kr * PA + mq]) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < BF4; ++i) {
            const int e = tid + i * NT, kr = e / (BN / 4), nq = (e % (BN / 4)) * 4;
            *reinterpret_cast<float4*>(&Bs[buf][kr * PB + nq]) = rb[i];
        }
    };
    f32x16 acc[AM][AN];
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nt = ceil_div(kend - kbeg, BK);
    const int h = lane >> 5, l31 = lane & 31;
    CLK_BEGIN()
    PH_MARK(1)
    load(kbeg);
    store(0);
    __syncthreads();
    if (nt > 1) load(kbeg + BK);
    for (int t = 0; t < nt; ++t) {
        const int buf = t & 1;
        const float* as = &As[buf][h * (BK / 2) * PA + wm * TM + l31];
        const float* bs = &Bs[buf][h * (BK / 2) * PB + wn * TN + l31];
        float fa[2][AM], fb[2][AN];
#pragma unroll
        for (int i = 0; i < AM; ++i) fa[0][i] = as[i * 32];
#pragma unroll
        for (int j = 0; j < AN; ++j) fb[0][j] = bs[j * 32];
#pragma unroll
        for (int st = 0; st < BK / 2; ++st) {
            const int cur = st & 1, nxt = cur ^ 1;
            if (st + 1 < BK / 2) {
#pragma unroll
                for (int i = 0; i < AM; ++i) fa[nxt][i] = as[(st + 1) * PA + i * 32];
#pragma unroll
                for (int j = 0; j < AN; ++j) fb[nxt][j] = bs[(st + 1) * PB + j * 32];
            }
#pragma unroll
            for (int i = 0; i < AM; ++i)
#pragma unroll
                for (int j = 0; j < AN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[cur][i], fb[cur][j], acc[i][j], 0, 0, 0);
        }
        if (t + 1 < nt) {
            store(buf ^ 1);
            if (t + 2 < nt) load(kbeg + (t + 2) * BK);
        }
        __syncthreads();
    }
    CLK_END(2u)
    PH_MARK(2)
    float* out = slabs + (long long)bz * M * N;
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j) {
            const int gn = n0 + wn * TN + j * 32 + l31;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gm = m0 + wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (gm < M && gn < N) out[(long long)gm * N + gn] = acc[i][j][r];
            }
        }
    PH_FLUSH(kend - kbeg)
}

// ---- dA on v_mfma_f32_16x16x4_f32 with LDS-DMA staging (tools/gemm4_lab.hip, "g5")
// C[M][N] = A[M][K] . B[N][K]^T, both k-contiguous, plain store.  Each stage of BK = 32 k is
// filled by buffer_load ... lds (16 B per lane, 1 KB per wave instruction, rows of 128 B with the
// 16-B slots XOR-swizzled by (row >> 1) & 7 so the fragment reads are conflict-free) and consumed
// after a counted vmcnt + s_barrier; lane (l15, g) reads 4 consecutive k of its row and step s of
// half hh contracts k = 16 hh + 4 g + s (same permutation on A and B).  Measured on the config-2
// dA shapes: edge 50.2 -> 47.5 us, node 23.8 -> 21.1 us against k_gemm3<64,128,...,E3_STORE>; step
// 338-339 K -> 342-345 K graphs/s.  Not used for the forward: the 16x16 MFMA's different k order
// put GNN_simple's 20-layer fixture output 1.2e-5 relative from the reference (bound 1e-5), against
// k_gemm3's inside it, for ~10 us per step.
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4 rsrc4(const void* p, int bytes) {
    const unsigned long long a = (unsigned long long)(uintptr_t)p;
    i32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
    r.y = __builtin_amdgcn_readfirstlane((int)(a >> 32) & 0xffff);
    r.z = __builtin_amdgcn_readfirstlane(bytes);
    r.w = 0x00020000;
    return r;
}

// 16 B per lane, global -> LDS at the wave-uniform LDS byte address + lane * 16.  Inline asm keeps
// the load out of hipcc's waitcnt bookkeeping (a builtin form made it wait vmcnt(0) before every
// LDS read); the kernel counts it with its own vmcnt.
__device__ __forceinline__ void dma16(i32x4 r, unsigned voff, unsigned lds_addr) {
    int keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(r), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
        : "memory");
}

// vmcnt(n) + lgkmcnt(0) + s_barrier in one statement (a compiler memory barrier too)
template <int N>
__device__ __forceinline__ void stage_barrier() {
    static_assert(N >= 0 && N < 16, "vmcnt");
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// FWD: the forward GEMM's epilogue (k_gemm3 E3_FWD: bias, ReLU from column relu_from, BN partials
// (count, mean, M2) per 64-row tile); used with 32 x 16 wave tiles for the node halves, whose
// 32 x 32-wave k_gemm3 grid (1 216 waves on 1 024 SIMDs) left most SIMDs with one wave and some
// with two.
template <int BM, int BN, int WGM, int WGN, bool FWD = false>
__global__ void __launch_bounds__(64 * WGM * WGN) k_gemm5(const float* __restrict__ A, int lda,
                                                          const float* __restrict__ B, int ldb,
                                                          const int* __restrict__ m_valid, int m_cap, int N, int K,
                                                          float* __restrict__ C, int ldc, int xcd,
                                                          const float* __restrict__ bias = nullptr,
                                                          int relu_from = 0, float* __restrict__ bn_part = nullptr,
                                                          uint64_t* stamps = nullptr) {
    WaveStamp stamp(stamps);
    constexpr int BK = 32, NW = WGM * WGN, ST = 2;
    constexpr int TM = BM / WGM, TN = BN / WGN, AM = TM / 16, AN = TN / 16;
    constexpr int AI = BM * BK * 4 / 1024, BI = BN * BK * 4 / 1024;  // 1-KB wave instructions per stage
    static_assert(AI % NW == 0 && BI % NW == 0, "staging split");
    constexpr int APW = AI / NW, BPW = BI / NW;
    constexpr int SF = (BM + BN) * BK;  // floats per stage
    __shared__ __attribute__((aligned(1024))) float lds[ST * SF];
    const int M = __builtin_amdgcn_readfirstlane(m_valid ? *m_valid : m_cap);
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wv / WGN, wn = wv % WGN;
    int bx = blockIdx.x, by = blockIdx.y;
    if (xcd) {  // the column tiles of a row tile on one XCD (see k_gemm3); gridDim.x % 8 == 0
        const int L = blockIdx.x + gridDim.x * blockIdx.y, j = L >> 3;
        by = j % gridDim.y;
        bx = (L & 7) + 8 * (j / gridDim.y);
    }
    const int m0 = bx * BM, n0 = by * BN;
    if (m0 >= M) return;
    constexpr unsigned OOB = 0x7ffffff0u;
    const i32x4 ra = rsrc4(A, M * lda * 4), rb = rsrc4(B, N * ldb * 4);
    const int lrow = lane >> 3, lslot = lane & 7;
    const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)lds;
    auto issue = [&](int st, int k0) {
        const unsigned base = lds0 + st * SF * 4;
#pragma unroll
        for (int i = 0; i < APW; ++i) {
            const int inst = wv * APW + i, row = inst * 8 + lrow;
            const int sl = lslot ^ ((row >> 1) & 7), gm = m0 + row, gk = k0 + 4 * sl;
            dma16(ra, (gm < M && gk < K) ? (unsigned)(gm * lda + gk) * 4u : OOB, base + inst * 1024);
        }
#pragma unroll
        for (int i = 0; i < BPW; ++i) {
            const int inst = wv * BPW + i, row = inst * 8 + lrow;
            const int sl = lslot ^ ((row >> 1) & 7), gn = n0 + row, gk = k0 + 4 * sl;
            dma16(rb, (gn < N && gk < K) ? (unsigned)(gn * ldb + gk) * 4u : OOB, base + BM * BK * 4 + inst * 1024);
        }
    };
    // per-k-tile accumulators added to acc (parity: fma chains of BK terms, as k_gemm3)
    f32x4 acc[AM][AN], tacc[AM][AN];
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;
    const int nt = (K + BK - 1) / BK;
    const int g = lane >> 4, l15 = lane & 15;
    CLK_BEGIN()
    issue(0, 0);
    stage_barrier<0>();
    for (int t = 0; t < nt; ++t) {
        if (t + 1 < nt) issue((t + 1) & 1, (t + 1) * BK);
        const float* as = lds + (t & 1) * SF;
        const float* bs = as + BM * BK;
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
            for (int j = 0; j < AN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) tacc[i][j][r] = 0.f;
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            float4 a[AM], b[AN];
#pragma unroll
            for (int i = 0; i < AM; ++i) {
                const int row = wm * TM + i * 16 + l15;
                a[i] = *reinterpret_cast<const float4*>(as + row * BK + 4 * ((hh * 4 + g) ^ ((row >> 1) & 7)));
            }
#pragma unroll
            for (int j = 0; j < AN; ++j) {
                const int row = wn * TN + j * 16 + l15;
                b[j] = *reinterpret_cast<const float4*>(bs + row * BK + 4 * ((hh * 4 + g) ^ ((row >> 1) & 7)));
            }
#pragma unroll
            for (int i = 0; i < AM; ++i)
#pragma unroll
                for (int j = 0; j < AN; ++j) {
                    tacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].x, b[j].x, tacc[i][j], 0, 0, 0);
                    tacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].y, b[j].y, tacc[i][j], 0, 0, 0);
                    tacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].z, b[j].z, tacc[i][j], 0, 0, 0);
                    tacc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].w, b[j].w, tacc[i][j], 0, 0, 0);
                }
        }
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
            for (int j = 0; j < AN; ++j) acc[i][j] += tacc[i][j];
        stage_barrier<0>();  // tile t + 1 landed; every wave is done with tile t's buffer
    }
    CLK_END(FWD ? 3u : 4u)
    // C layout of the 16x16 MFMA: col = lane & 15, row = 4 (lane >> 4) + r
    if constexpr (FWD) {
        static_assert(BM == 64 && WGM == 2 && AN == 1, "BN partials per 64-row tile, one column per lane");
        float* red = lds;  // the stage buffers are free: the main loop ended with a barrier
        const int col = wn * TN + l15, gn = n0 + col;
        const float bv = gn < N ? bias[gn] : 0.f;
        const bool relu = gn >= relu_from;
        float sm = 0.f;
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gm = m0 + wm * TM + i * 16 + 4 * g + r;
                float v = acc[i][0][r] + bv;
                if (relu) v = v < 0.f ? 0.f : v;
                acc[i][0][r] = v;
                if (gm < M) {
                    if (gn < N) C[(long long)gm * ldc + gn] = v;
                    sm += v;
                    ++cnt;
                }
            }
        if (bn_part) {
            sm += __shfl_xor(sm, 16, 64);
            sm += __shfl_xor(sm, 32, 64);
            cnt += __shfl_xor(cnt, 16, 64);
            cnt += __shfl_xor(cnt, 32, 64);
            if (lane < 16) {
                red[wm * BN + col] = sm;
                red[2 * BN + wm * BN + col] = (float)cnt;
            }
            __syncthreads();
            const float S = red[col] + red[BN + col];
            const float Cn = red[2 * BN + col] + red[3 * BN + col];
            const float mean = Cn > 0.f ? S / Cn : 0.f;
            __syncthreads();
            float q = 0.f;
#pragma unroll
            for (int i = 0; i < AM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int gm = m0 + wm * TM + i * 16 + 4 * g + r;
                    if (gm < M) {
                        const float dl = acc[i][0][r] - mean;
                        q = fmaf(dl, dl, q);
                    }
                }
            q += __shfl_xor(q, 16, 64);
            q += __shfl_xor(q, 32, 64);
            if (lane < 16) red[wm * BN + col] = q;
            __syncthreads();
            if (wm == 0 && lane < 16 && gn < N) {
                float* pp = bn_part + ((long long)bx * N + gn) * 3;
                pp[0] = Cn;
                pp[1] = mean;
                pp[2] = red[col] + red[BN + col];
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j) {
            const int gn = n0 + wn * TN + j * 16 + l15;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int gm = m0 + wm * TM + i * 16 + 4 * g + r;
                if (gm < M && gn < N) C[(long long)gm * ldc + gn] = acc[i][j][r];
            }
        }
}

}  // namespace

// Target block count of the dW GEMM (split-K chunks x output tiles).  Every launched block has rows
// (dw3_kc): at config 2, 256 blocks (one per CU) measured 1.340 / 1.344 ms per step against 1.377 /
// 1.378 for 512 and 1.401 / 1.404 for 1024 (same box, alternating runs) -- the dW kernel runs on the
// side stream beside the main stream's backward, and more of its blocks crowd the main stream's
// kernels off the CUs; HGNN_DW_BLOCKS overrides.
static int dw3_target_blocks() {
    static const int t = [] {
        const char* e = getenv("HGNN_DW_BLOCKS");
        const int v = e ? atoi(e) : 256;
        return v >= 16 && v <= 4096 ? v : 256;
    }();
    return t;
}

int dw3_chunks(int r_cap, int o, int k) {
    const int tiles = ceil_div(o, 128) * ceil_div(k, 128);
    // 256 blocks at config 2 (5 output tiles); twice that for the wide networks (config 4, d = 128: 20
    // tiles, 3.39 -> 3.32 ms per step), whose main-stream kernels are long enough to leave room
    const int target = getenv("HGNN_DW_BLOCKS") || tiles < 16 ? dw3_target_blocks() : 2 * dw3_target_blocks();
    int chunks = target / (tiles > 0 ? tiles : 1);
    // never more chunks than 64-row pieces of the capacity; a multiple of 8 (XCD-aware order),
    // rounded DOWN so the grid stays within the target: standalone on the config-2 edge dW shape
    // (tools/dw_lab.hip) 48 chunks x 5 tiles = 240 blocks ran 41.5 us (0.58 of the fp32 MFMA peak),
    // 56 x 5 = 280 blocks (a second partial round on 24 CUs) 55 us
    chunks = std::min(chunks, ceil_div(r_cap > 0 ? r_cap : 1, 64));
    // a multiple of 8 keeps the XCD-aware order (launch_gemm3_dw); when rounding down would idle more
    // than a fifth of the target (config 4: 20 output tiles, 12 -> 8 chunks = 160 blocks on 256 CUs)
    // the exact count runs in the linear order instead
    const int c8 = chunks / 8 * 8;
    if (c8 >= 8 && 5 * c8 >= 4 * chunks) return c8;
    return chunks < 1 ? 1 : chunks;
}

size_t dw3_slab_floats(int r_cap, int o, int k) { return (size_t)dw3_chunks(r_cap, o, k) * o * k; }

bool dw_bf3_enabled() {
    static const bool on = [] {
        const char* e = getenv("HGNN_DW_BF3");
        return !e || e[0] != '0';
    }();
    return on;
}

// slabs[z][o][k] = sum_{r in chunk z} dY[r, o] A[r, k]
int launch_gemm3_dw(const float* dy, int lddy, const float* a, int lda, const int* r_valid, int r_cap, int o, int k,
                    int nz, float* slabs, hipStream_t s, const DiagIdArgs* id) {
    if (r_cap <= 0) return 0;
    if (nz <= 0) return HGNN_ERR_ARG;
    static const bool xcd = [] {
        const char* e = getenv("HGNN_DW_XCD");
        return !e || e[0] != '0';
    }();
    const bool bf3 = dw_bf3_enabled();
    if (bf3) return launch_gemm_bf3_dw(dy, lddy, a, lda, r_valid, r_cap, o, k, nz, slabs, xcd, s, id);
    if (id) return HGNN_ERR_UNSUPPORTED;  // the diagonal I / D columns: the split-bf16 kernel only
    HGNN_KLAUNCH((k_gemm3_tn<128, 128, 32, 4, 2>), dim3(ceil_div(o, 128), ceil_div(k, 128), nz), dim3(512), 0, s,
                       dy, lddy, a, lda, slabs, o, k, r_valid, nz, xcd && nz % 8 == 0 ? 1 : 0);
    HGNN_LAUNCH_CHECK();
    return 0;
}

int gemm_fwd_tiles_m(int m_cap) { return ceil_div(m_cap, 64); }

bool gemm3_ok(int lda, int ldb, int ldc, const void* a, const void* b) {
    auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    return lda % 4 == 0 && ldb % 4 == 0 && ldc % 4 == 0 && al(a) && al(b);
}

// Y[r, n] = A[r, :k] . Wc[n, :k] + bias[n]; ReLU on n >= relu_from; BN partials per 64-row tile.
int launch_gemm3_fwd(const float* a, int lda, const int* m_valid, int m_cap, int k, const float* wc, int ldw, int n,
                     const float* bias, int relu_from, float* y, int ldy, float* bn_part, hipStream_t s,
                     int mfma16) {
    if (m_cap <= 0) return 0;
    if (k % 4 != 0) return HGNN_ERR_UNSUPPORTED;  // pass the padded width (zero padding in both operands)
    if ((long long)m_cap * lda * 4 >= (1ll << 31) || (long long)n * ldw * 4 >= (1ll << 31)) return HGNN_ERR_UNSUPPORTED;
    // 32 x 16 wave tiles (v_mfma_f32_16x16x4_f32, LDS-DMA staging) when the 32 x 32-wave grid would
    // leave the SIMDs unevenly loaded (under 2 waves per SIMD): the node halves.  Default (3): 64 x 32
    // block tiles of 4 waves -- config 2's 9.7 K node rows make 608 blocks, 2-3 per CU, instead of
    // 304 64 x 64 blocks of 8 waves that left 48 CUs with two blocks and the rest with one (22.2 vs
    // 24.4 us per launch, same results bit for bit); HGNN_FWD_G5=1 the 64 x 64 tiles, 0 never, 2 always
    static const int g5 = [] {
        const char* e = getenv("HGNN_FWD_G5");
        return e ? atoi(e) : 3;
    }();
    const long long waves32 = (long long)ceil_div(m_cap, 64) * ceil_div(n, 64) * 4;
    if (mfma16 && g5 > 0 && n % 64 == 0 && n <= 512 && (g5 == 2 || waves32 < 2 * 1024)) {
        const int gx = ceil_div(ceil_div(m_cap, 64), 8) * 8;
        if (g5 == 3)  // 64 x 32 tiles of 4 waves: twice the blocks, finer per-CU balance
            HGNN_KLAUNCH((k_gemm5<64, 32, 2, 2, true>), dim3(gx, n / 32), dim3(256), 0, s, a, lda, wc, ldw,
                         m_valid, m_cap, n, k, y, ldy, 1, bias, relu_from, bn_part,
                         clock_stamps((long long)gx * (n / 32) * 4));
        else
            HGNN_KLAUNCH((k_gemm5<64, 64, 2, 4, true>), dim3(gx, n / 64), dim3(512), 0, s, a, lda, wc, ldw,
                         m_valid, m_cap, n, k, y, ldy, 1, bias, relu_from, bn_part,
                         clock_stamps((long long)gx * (n / 64) * 8));
        HGNN_LAUNCH_CHECK();
        return 0;
    }
    G3 p{};
    p.a = a;
    p.lda = lda;
    p.b = wc;
    p.ldb = ldw;
    p.m_cap = m_cap;
    p.m_valid = m_valid;
    p.k = k;
    p.n = n;
    p.c = y;
    p.ldc = ldy;
    p.bias = bias;
    p.relu_from = relu_from;
    p.bn_part = bn_part;
    static const bool xcd = [] {
        const char* e = getenv("HGNN_FWD_XCD");
        return !e || e[0] != '0';
    }();
    const int bn = n <= 128 ? 64 : 128;
    p.xcd = xcd && ceil_div(n, bn) > 1;
    const int gx = p.xcd ? ceil_div(ceil_div(m_cap, 64), 8) * 8 : ceil_div(m_cap, 64);  // padded tiles exit
    if (n <= 128) {
        // 64-column tiles up to 2d = 128: twice the blocks of 64 x 128 tiles, measured (round-1 GEMM lab)
        // edge forward 47.7 -> 40.7 us, node forward 34 -> 28 us
        HGNN_KLAUNCH((k_gemm3<64, 64, 32, 2, 2, E3_FWD>), dim3(gx, ceil_div(n, 64)), dim3(256), 0, s, p);
    } else {
        HGNN_KLAUNCH((k_gemm3<64, 128, 32, 2, 2, E3_FWD>), dim3(gx, ceil_div(n, 128)), dim3(256), 0, s, p);
    }
    HGNN_LAUNCH_CHECK();
    return 0;
}

// dA[r, j] = sum_o dY[r, o] WT[j, o]   (j < kout)
int launch_gemm3_da(const float* dy, int lddy, const int* m_valid, int m_cap, int o, const float* wt, int ldw,
                    int kout, float* da, int ldda, hipStream_t s) {
    if (m_cap <= 0) return 0;
    if (o % 4 != 0) return HGNN_ERR_UNSUPPORTED;
    if ((long long)m_cap * lddy * 4 >= (1ll << 31) || (long long)kout * ldw * 4 >= (1ll << 31)) return HGNN_ERR_UNSUPPORTED;
    static const bool dma = [] {
        const char* e = getenv("HGNN_GEMM_DMA");
        return !(e && e[0] == '0');
    }();
    auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    if (dma && lddy % 4 == 0 && ldw % 4 == 0 && al(dy) && al(wt)) {
        static const bool xcd = [] {
            const char* e = getenv("HGNN_DA_XCD");
            return !e || e[0] != '0';
        }();
        const int gx = xcd ? ceil_div(ceil_div(m_cap, 64), 8) * 8 : ceil_div(m_cap, 64);
        const dim3 g(gx, ceil_div(kout, 64));
        HGNN_KLAUNCH((k_gemm5<64, 64, 2, 2>), g, dim3(256), 0, s, dy, lddy, wt, ldw, m_valid, m_cap, kout, o, da, ldda,
                     xcd ? 1 : 0, static_cast<const float*>(nullptr), 0, static_cast<float*>(nullptr),
                     clock_stamps((long long)g.x * g.y * 4));
        HGNN_LAUNCH_CHECK();
        return 0;
    }
    G3 p{};
    p.a = dy;
    p.lda = lddy;
    p.b = wt;
    p.ldb = ldw;
    p.m_cap = m_cap;
    p.m_valid = m_valid;
    p.k = o;
    p.n = kout;
    p.c = da;
    p.ldc = ldda;
    HGNN_KLAUNCH((k_gemm3<64, 128, 32, 2, 2, E3_STORE>), dim3(ceil_div(m_cap, 64), ceil_div(kout, 128)),
                       dim3(256), 0, s, p);
    HGNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace hgnn

#ifdef HGNN_CLOCK_DIAG
// Diagnostic build: copy out (and with reset != 0 clear) the clock stamps; returns the count.
extern "C" int hgnn_diag_clock_read(void* out, int max_n, int reset) {
    unsigned n = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(hgnn::g_clock_n), sizeof(n)) != hipSuccess) return -1;
    if (n > hgnn::CLOCK_SLOTS) n = hgnn::CLOCK_SLOTS;
    const unsigned k = n < (unsigned)max_n ? n : (unsigned)max_n;
    if (k && hipMemcpyFromSymbol(out, HIP_SYMBOL(hgnn::g_clock), k * sizeof(hgnn::ClockStamp)) != hipSuccess)
        return -1;
    if (reset) {
        const unsigned z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(hgnn::g_clock_n), &z, sizeof(z)) != hipSuccess) return -1;
    }
    return (int)k;
}

// Diagnostic build: the dW GEMM's phase stamps (48 B each), as above.
extern "C" int hgnn_diag_phase_read(void* out, int max_n, int reset) {
    unsigned n = 0;
    if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(hgnn::g_phase_n), sizeof(n)) != hipSuccess) return -1;
    if (n > hgnn::PHASE_SLOTS) n = hgnn::PHASE_SLOTS;
    const unsigned k = n < (unsigned)max_n ? n : (unsigned)max_n;
    if (k && hipMemcpyFromSymbol(out, HIP_SYMBOL(hgnn::g_phase), k * sizeof(hgnn::PhaseStamp)) != hipSuccess)
        return -1;
    if (reset) {
        const unsigned z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(hgnn::g_phase_n), &z, sizeof(z)) != hipSuccess) return -1;
    }
    return (int)k;
}
#endif
