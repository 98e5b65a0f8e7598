// fp32 MFMA GEMMs for the 1x1 Conv1d feature mixes of every layer
// (models/layers/layers_mnb.py:36-37, 172-177, 239-244, 305-310) and their
// backward.  gfx950 has no xf32, so the exact-f32 `v_mfma_f32_32x32x2_f32`
// (64 FLOP/clk/SIMD, the fp32 peak) carries the dense per-node/per-edge mix:
//   forward : Y[r, n]  = A[r, :] . W(n)[:] + b(n);  relu on n >= relu_from;
//             plus per-tile BN partials (count, mean, M2) of Y over valid rows
//   dA      : dA[r, k] = sum_o dY[r, o] Wcat[o, k]
//   dW      : dWcat[o, k] = sum_r dY[r, o] A[r, k]  (split-K over rows into slabs,
//             the extra column k = K carries the bias gradient sum_r dY[r, o])
// The two Conv1d of a layer half (linear cv2/cv4 and ReLU cv1/cv3, concatenated
// as cat(linear, relu) by the reference) are one GEMM with N = 2d: W rows
// [0, split) come from the linear conv, [split, 2d) from the ReLU conv.
//
// Tile 64x64x32, 256 threads = 4 waves in 2x2, each wave one 32x32 MFMA tile.
// Operand tiles are staged [k][m] / [k][n] in LDS with a +1 pad, so the MFMA
// operand reads (32 consecutive rows per half-wave) and the transposing
// stores are bank-conflict free; the next K-tile is prefetched into registers
// while the current one is multiplied.
#include "kernels.h"

namespace hgnn {

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {
constexpr int BM = 64, BN = 64, BK = 32;
constexpr int PADA = BM + 1, PADB = BN + 1;

enum { AM_MK = 0, AM_KM = 1 };
enum { BMODE_NK2 = 0, BMODE_KN2 = 1, BMODE_KN1 = 2 };
enum { EPI_FWD = 0, EPI_STORE = 1, EPI_SLAB = 2 };

struct GP {
    const float* a;
    int lda;
    const float* b0;
    const float* b1;
    int ldb, bsplit, nones;
    int m_cap;
    const int* m_valid;
    int kdim;
    const int* k_valid;
    int n;
    int kchunk;
    float* c;
    int ldc;
    const float* bias0;
    const float* bias1;
    int relu_from;
    float* bn_part;
};
}  // namespace

template <int AMODE, int BMODE, int EPI>
__global__ void __launch_bounds__(256) k_gemm(GP p) {
    __shared__ float As[BK][PADA];
    __shared__ float Bs[BK][PADB];
    __shared__ float red_s[2][BN];
    __shared__ int red_c[2][BN];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    const int m0 = blockIdx.x * BM;
    const int n0 = blockIdx.y * BN;
    const int Mv = p.m_valid ? *p.m_valid : p.m_cap;
    if (m0 >= Mv) return;
    const int Kv = p.k_valid ? *p.k_valid : p.kdim;
    int kbeg = 0, kend = Kv;
    if constexpr (EPI == EPI_SLAB) {
        kbeg = blockIdx.z * p.kchunk;
        kend = min(Kv, kbeg + p.kchunk);
        if (kbeg >= kend) return;
    }
    const int N = p.n;

    float ra[8], rb[8];
    auto load_tile = [&](int k0) {
        if constexpr (AMODE == AM_MK) {
            const int mm = tid >> 2, kc = (tid & 3) * 8;
            const int gm = m0 + mm;
            const float* row = p.a + (long long)gm * p.lda;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int gk = k0 + kc + i;
                ra[i] = (gm < Mv && gk < kend) ? row[gk] : 0.f;
            }
        } else {
            const int kk = tid >> 3, mc = (tid & 7) * 8;
            const int gk = k0 + kk;
            const float* row = p.a + (long long)gk * p.lda;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int gm = m0 + mc + i;
                ra[i] = (gk < kend && gm < Mv) ? row[gm] : 0.f;
            }
        }
        if constexpr (BMODE == BMODE_NK2) {
            const int nn = tid >> 2, kc = (tid & 3) * 8;
            const int gn = n0 + nn;
            const float* row = gn < p.bsplit ? p.b0 + (long long)gn * p.ldb
                                             : p.b1 + (long long)(gn - p.bsplit) * p.ldb;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int gk = k0 + kc + i;
                rb[i] = (gn < N && gk < kend) ? row[gk] : 0.f;
            }
        } else {
            const int kk = tid >> 3, nc = (tid & 7) * 8;
            const int gk = k0 + kk;
            const float* row;
            if constexpr (BMODE == BMODE_KN2)
                row = gk < p.bsplit ? p.b0 + (long long)gk * p.ldb : p.b1 + (long long)(gk - p.bsplit) * p.ldb;
            else
                row = p.b0 + (long long)gk * p.ldb;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int gn = n0 + nc + i;
                float v = 0.f;
                if (gk < kend) {
                    if constexpr (BMODE == BMODE_KN1) v = gn < p.nones ? row[gn] : (gn == p.nones ? 1.f : 0.f);
                    else v = gn < N ? row[gn] : 0.f;
                }
                rb[i] = v;
            }
        }
    };
    auto store_tile = [&]() {
        if constexpr (AMODE == AM_MK) {
            const int mm = tid >> 2, kc = (tid & 3) * 8;
#pragma unroll
            for (int i = 0; i < 8; ++i) As[kc + i][mm] = ra[i];
        } else {
            const int kk = tid >> 3, mc = (tid & 7) * 8;
#pragma unroll
            for (int i = 0; i < 8; ++i) As[kk][mc + i] = ra[i];
        }
        if constexpr (BMODE == BMODE_NK2) {
            const int nn = tid >> 2, kc = (tid & 3) * 8;
#pragma unroll
            for (int i = 0; i < 8; ++i) Bs[kc + i][nn] = rb[i];
        } else {
            const int kk = tid >> 3, nc = (tid & 7) * 8;
#pragma unroll
            for (int i = 0; i < 8; ++i) Bs[kk][nc + i] = rb[i];
        }
    };

    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;

    load_tile(kbeg);
    for (int k0 = kbeg; k0 < kend; k0 += BK) {
        __syncthreads();
        store_tile();
        __syncthreads();
        if (k0 + BK < kend) load_tile(k0 + BK);
        const int ar = wr * 32 + (lane & 31);
        const int bc = wc * 32 + (lane & 31);
        const int kh = lane >> 5;
#pragma unroll
        for (int kk = 0; kk < BK; kk += 2) {
            const float av = As[kk + kh][ar];
            const float bv = Bs[kk + kh][bc];
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
        }
    }

    // C/D layout of 32x32 MFMA: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
    const int col = wc * 32 + (lane & 31);
    const int gn = n0 + col;
    if constexpr (EPI == EPI_FWD) {
        float bias = 0.f;
        if (gn < N) bias = gn < p.bsplit ? p.bias0[gn] : p.bias1[gn - p.bsplit];
        const bool relu = gn >= p.relu_from;
        float y[16];
        float s = 0.f;
        int cnt = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const int gm = m0 + row;
            float v = acc[r] + bias;
            if (relu) v = v < 0.f ? 0.f : v;
            y[r] = v;
            if (gm < Mv) {
                if (gn < N) p.c[(long long)gm * p.ldc + gn] = v;
                s += v;
                ++cnt;
            }
        }
        if (p.bn_part) {
            s += __shfl_xor(s, 32, 64);
            cnt += __shfl_xor(cnt, 32, 64);
            if (lane < 32) {
                red_s[wr][col] = s;
                red_c[wr][col] = cnt;
            }
            __syncthreads();
            const float S = red_s[0][col] + red_s[1][col];
            const int C = red_c[0][col] + red_c[1][col];
            const float mean = C > 0 ? S / (float)C : 0.f;
            float q = 0.f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                if (m0 + row < Mv) {
                    const float dlt = y[r] - mean;
                    q = fmaf(dlt, dlt, q);
                }
            }
            q += __shfl_xor(q, 32, 64);
            __syncthreads();
            if (lane < 32) red_s[wr][col] = q;
            __syncthreads();
            if (wr == 0 && lane < 32 && gn < N) {
                float* pp = p.bn_part + ((long long)blockIdx.x * N + gn) * 3;
                pp[0] = (float)C;
                pp[1] = mean;
                pp[2] = red_s[0][col] + red_s[1][col];
            }
        }
    } else if constexpr (EPI == EPI_STORE) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const int gm = m0 + row;
            if (gm < Mv && gn < N) p.c[(long long)gm * p.ldc + gn] = acc[r];
        }
    } else {
        float* slab = p.c + (long long)blockIdx.z * p.m_cap * N;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int row = wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const int gm = m0 + row;
            if (gm < p.m_cap && gn < N) slab[(long long)gm * N + gn] = acc[r];
        }
    }
}

int gemm_fwd_tiles_m(int m_cap) { return ceil_div(m_cap, BM); }

int launch_gemm_fwd(const GemmFwdArgs& g, hipStream_t s) {
    if (g.m_cap <= 0) return 0;
    GP p{};
    p.a = g.a;
    p.lda = g.lda;
    p.b0 = g.w0;
    p.b1 = g.w1;
    p.ldb = g.k;
    p.bsplit = g.split;
    p.m_cap = g.m_cap;
    p.m_valid = g.m_valid;
    p.kdim = g.k;
    p.n = g.n;
    p.c = g.y;
    p.ldc = g.ldy;
    p.bias0 = g.b0;
    p.bias1 = g.b1;
    p.relu_from = g.relu_from;
    p.bn_part = g.bn_part;
    const dim3 grid(ceil_div(g.m_cap, BM), ceil_div(g.n, BN));
    hipLaunchKernelGGL((k_gemm<AM_MK, BMODE_NK2, EPI_FWD>), grid, dim3(256), 0, s, p);
    HGNN_LAUNCH_CHECK();
    return 0;
}

int launch_gemm_da(const GemmDaArgs& g, hipStream_t s) {
    if (g.m_cap <= 0) return 0;
    GP p{};
    p.a = g.dy;
    p.lda = g.lddy;
    p.b0 = g.w0;
    p.b1 = g.w1;
    p.ldb = g.k;
    p.bsplit = g.split;
    p.m_cap = g.m_cap;
    p.m_valid = g.m_valid;
    p.kdim = g.o;
    p.n = g.k;
    p.c = g.da;
    p.ldc = g.ldda;
    const dim3 grid(ceil_div(g.m_cap, BM), ceil_div(g.k, BN));
    hipLaunchKernelGGL((k_gemm<AM_MK, BMODE_KN2, EPI_STORE>), grid, dim3(256), 0, s, p);
    HGNN_LAUNCH_CHECK();
    return 0;
}

namespace {
int dw_kchunk(int r_cap, int o, int k) {
    const int tiles = ceil_div(o, BM) * ceil_div(k + 1, BN);
    int chunks = 640 / (tiles > 0 ? tiles : 1);
    if (chunks < 1) chunks = 1;
    int kc = ceil_div(r_cap > 0 ? r_cap : 1, chunks);
    kc = ceil_div(kc, BK) * BK;
    if (kc < 4 * BK) kc = 4 * BK;
    return kc;
}
}  // namespace

size_t gemm_dw_slab_floats(int r_cap, int o, int k) {
    const int kc = dw_kchunk(r_cap, o, k);
    const int z = ceil_div(r_cap > 0 ? r_cap : 1, kc);
    return (size_t)z * o * (k + 1);
}

__global__ void k_dw_reduce(const float* __restrict__ slabs, const int* k_valid, int kchunk,
                            int M, int N, int split, int kreal, float* dw0, float* dw1,
                            float* db0, float* db1) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= M * N) return;
    const int zv = ceil_div(*k_valid, kchunk);
    float s = 0.f;
    for (int z = 0; z < zv; ++z) s += slabs[(long long)z * M * N + idx];
    const int o = idx / N, c = idx % N;
    if (c < kreal) {
        if (o < split) dw0[(long long)o * kreal + c] = s;
        else dw1[(long long)(o - split) * kreal + c] = s;
    } else {
        if (o < split) db0[o] = s;
        else db1[o - split] = s;
    }
}

int launch_gemm_dw(const GemmDwArgs& g, hipStream_t s) {
    const int kc = dw_kchunk(g.r_cap, g.o, g.k);
    const int z = ceil_div(g.r_cap > 0 ? g.r_cap : 1, kc);
    GP p{};
    p.a = g.dy;
    p.lda = g.lddy;
    p.b0 = g.a;
    p.ldb = g.lda;
    p.nones = g.k;
    p.m_cap = g.o;
    p.m_valid = nullptr;
    p.kdim = g.r_cap;
    p.k_valid = g.r_valid;
    p.n = g.k + 1;
    p.kchunk = kc;
    p.c = g.slabs;
    const dim3 grid(ceil_div(g.o, BM), ceil_div(g.k + 1, BN), z);
    hipLaunchKernelGGL((k_gemm<AM_KM, BMODE_KN1, EPI_SLAB>), grid, dim3(256), 0, s, p);
    HGNN_LAUNCH_CHECK();
    const int total = g.o * (g.k + 1);
    hipLaunchKernelGGL(k_dw_reduce, dim3(ceil_div(total, 256)), dim3(256), 0, s, g.slabs, g.r_valid,
                       kc, g.o, g.k + 1, g.split, g.k, g.dw0, g.dw1, g.db0, g.db1);
    HGNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace hgnn
