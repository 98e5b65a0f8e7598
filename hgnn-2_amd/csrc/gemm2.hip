// GEMM v2: fp32 MFMA (v_mfma_f32_32x32x2_f32) with full-line vector staging.
//
// Used whenever every leading dimension is a multiple of 4 floats (the
// executor pads its own buffers so this holds at d even); gemm.hip remains
// the general fallback.  Differences from v1, each aimed at what the first
// rocprof run showed (GEMMs at 12-15 % of the fp32 MFMA peak):
//  * global -> register staging with float4 loads, 8 consecutive lanes per
//    128-B row segment (v1's scalar, fragment-shaped loads kept the texture
//    path busy -- cdna_hip_programming.md §5 "Projection GEMM", item 3);
//  * B is always N-major (n contiguous): the forward weights are repacked once
//    per forward into Wcat^T [K][2d], dA reads Wcat [2d][K] as is, dW reads
//    the saved aggregate [rows][K] -> B tiles go to LDS with ds_write_b128;
//  * LDS double buffer, one barrier per K-tile, next tile prefetched into
//    registers while the current one is multiplied;
//  * 2x2 waves, each wave (BM/2)x(BN/2) = up to 2x2 MFMA 32x32 accumulators.
#include "kernels.h"

namespace hgnn {

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

enum { A_MK = 0, A_KM = 1 };
enum { E_FWD = 0, E_STORE = 1, E_SLAB = 2 };

struct G2 {
    const float* a;
    int lda;
    const float* b0;
    const float* b1;
    int ldb, bsplit;
    int m_cap;
    const int* m_valid;
    int kdim;
    const int* k_valid;
    int n;
    int kchunk;
    float* c;
    int ldc;
    const float* bias;
    int relu_from;
    float* bn_part;
    long long slab_stride;
};

template <int BM, int BN, int BK, int AMODE, int EPI>
__global__ void __launch_bounds__(256) k_gemm2(G2 p) {
    constexpr int WM = BM / 2, WN = BN / 2;
    constexpr int AM = WM / 32, AN = WN / 32;
    constexpr int PA = (AMODE == A_MK) ? BM + 1 : BM + 4;
    constexpr int PB = BN + 4;
    // A staging: MK -> rows of BK floats, KM -> k-rows of BM floats
    constexpr int A_F4 = BM * BK / 4 / 256;  // float4 per thread
    constexpr int B_F4 = BN * BK / 4 / 256;
    static_assert(A_F4 >= 1 && B_F4 >= 1, "tile too small for 256 threads");
    __shared__ __attribute__((aligned(16))) float As[2][BK][PA];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK][PB];

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wr = wv >> 1, wc = wv & 1;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const int Mv = p.m_valid ? *p.m_valid : p.m_cap;
    if (m0 >= Mv) return;
    const int Kv = p.k_valid ? *p.k_valid : p.kdim;
    int kbeg = 0, kend = Kv;
    if constexpr (EPI == E_SLAB) {
        kbeg = blockIdx.z * p.kchunk;
        kend = min(Kv, kbeg + p.kchunk);
        if (kbeg >= kend) return;
    }
    const int N = p.n;

    float4 ra[A_F4], rb[B_F4];
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            const int e = tid + i * 256;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (AMODE == A_MK) {
                const int row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
                const int gm = m0 + row, gk = k0 + kq;
                if (gm < Mv && gk < kend) {
                    v = *reinterpret_cast<const float4*>(p.a + (long long)gm * p.lda + gk);
                    if (gk + 3 >= kend) {
                        if (gk + 1 >= kend) v.y = 0.f;
                        if (gk + 2 >= kend) v.z = 0.f;
                        v.w = 0.f;
                    }
                }
            } else {
                const int kr = e / (BM / 4), mq = (e % (BM / 4)) * 4;
                const int gk = k0 + kr, gm = m0 + mq;
                if (gk < kend && gm < Mv) {
                    v = *reinterpret_cast<const float4*>(p.a + (long long)gk * p.lda + gm);
                    if (gm + 3 >= Mv) {
                        if (gm + 1 >= Mv) v.y = 0.f;
                        if (gm + 2 >= Mv) v.z = 0.f;
                        v.w = 0.f;
                    }
                }
            }
            ra[i] = v;
        }
#pragma unroll
        for (int i = 0; i < B_F4; ++i) {
            const int e = tid + i * 256;
            const int kr = e / (BN / 4), nq = (e % (BN / 4)) * 4;
            const int gk = k0 + kr, gn = n0 + nq;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (gk < kend && gn < N) {
                const float* row = gk < p.bsplit ? p.b0 + (long long)gk * p.ldb
                                                 : p.b1 + (long long)(gk - p.bsplit) * p.ldb;
                v = *reinterpret_cast<const float4*>(row + gn);
                if (gn + 3 >= N) {
                    if (gn + 1 >= N) v.y = 0.f;
                    if (gn + 2 >= N) v.z = 0.f;
                    v.w = 0.f;
                }
            }
            rb[i] = v;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < A_F4; ++i) {
            const int e = tid + i * 256;
            if constexpr (AMODE == A_MK) {
                const int row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
                As[buf][kq + 0][row] = ra[i].x;
                As[buf][kq + 1][row] = ra[i].y;
                As[buf][kq + 2][row] = ra[i].z;
                As[buf][kq + 3][row] = ra[i].w;
            } else {
                const int kr = e / (BM / 4), mq = (e % (BM / 4)) * 4;
                *reinterpret_cast<float4*>(&As[buf][kr][mq]) = ra[i];
            }
        }
#pragma unroll
        for (int i = 0; i < B_F4; ++i) {
            const int e = tid + i * 256;
            const int kr = e / (BN / 4), nq = (e % (BN / 4)) * 4;
            *reinterpret_cast<float4*>(&Bs[buf][kr][nq]) = rb[i];
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
    load(kbeg);
    store(0);
    __syncthreads();
    if (nt > 1) load(kbeg + BK);
    const int h = lane >> 5, l31 = lane & 31;
    for (int t = 0; t < nt; ++t) {
        const int buf = t & 1;
#pragma unroll
        for (int kk = 0; kk < BK; kk += 2) {
            float av[AM], bv[AN];
#pragma unroll
            for (int i = 0; i < AM; ++i) av[i] = As[buf][kk + h][wr * WM + i * 32 + l31];
#pragma unroll
            for (int j = 0; j < AN; ++j) bv[j] = Bs[buf][kk + h][wc * WN + j * 32 + l31];
#pragma unroll
            for (int i = 0; i < AM; ++i)
#pragma unroll
                for (int j = 0; j < AN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i], bv[j], acc[i][j], 0, 0, 0);
        }
        if (t + 1 < nt) {
            store(buf ^ 1);
            if (t + 2 < nt) load(kbeg + (t + 2) * BK);
        }
        __syncthreads();
    }

    // C/D layout of the 32x32 MFMA: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    if constexpr (EPI == E_FWD) {
        float* red = &As[0][0][0];  // reuse LDS: [2][BN] sums + [2][BN] counts
        float s[AN];
        int cnt[AN];
#pragma unroll
        for (int j = 0; j < AN; ++j) {
            const int gn = n0 + wc * WN + j * 32 + l31;
            const float bias = gn < N ? p.bias[gn] : 0.f;
            const bool relu = gn >= p.relu_from;
            s[j] = 0.f;
            cnt[j] = 0;
#pragma unroll
            for (int i = 0; i < AM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int gm = m0 + wr * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
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
                const int col = wc * WN + j * 32 + l31;
                if (lane < 32) {
                    red[wr * BN + col] = s[j];
                    red[2 * BN + wr * BN + col] = (float)cnt[j];
                }
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < AN; ++j) {
                const int col = wc * WN + j * 32 + l31;
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
                        const int gm = m0 + wr * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                        if (gm < Mv) {
                            const float dl = acc[i][j][r] - mean[j];
                            q = fmaf(dl, dl, q);
                        }
                    }
                q += __shfl_xor(q, 32, 64);
                const int col = wc * WN + j * 32 + l31;
                if (lane < 32) red[wr * BN + col] = q;
            }
            __syncthreads();
            if (wr == 0 && lane < 32) {
#pragma unroll
                for (int j = 0; j < AN; ++j) {
                    const int col = wc * WN + j * 32 + l31;
                    const int gn = n0 + col;
                    if (gn < N) {
                        float* pp = p.bn_part + ((long long)blockIdx.x * N + gn) * 3;
                        pp[0] = (float)cnt[j];
                        pp[1] = mean[j];
                        pp[2] = red[col] + red[BN + col];
                    }
                }
            }
        }
    } else {
        float* out = p.c;
        int mlim = Mv;
        if constexpr (EPI == E_SLAB) {
            out += (long long)blockIdx.z * p.slab_stride;
            mlim = p.m_cap;
        }
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
            for (int j = 0; j < AN; ++j) {
                const int gn = n0 + wc * WN + j * 32 + l31;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int gm = m0 + wr * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (gm < mlim && gn < N) out[(long long)gm * p.ldc + gn] = acc[i][j][r];
                }
            }
    }
}

}  // namespace

// Weight repack for GEMM v2: WT[k][n] = Wcat[n][k] (forward B, N-major), WC[n][k < kp]
// = Wcat[n][k] zero-padded to kp columns (dA B), bc = cat(b_lin, b_relu).
__global__ void __launch_bounds__(256) k_repack(RepackTable t) {
    const RepackItem& it = t.it[blockIdx.x];
    const int d = t.d, c2 = 2 * d, K = it.k, kp = it.kp;
    const long long nt = (long long)K * c2, nc = (long long)c2 * kp;
    for (long long e = (long long)blockIdx.y * blockDim.x + threadIdx.x; e < nt + nc + c2;
         e += (long long)gridDim.y * blockDim.x) {
        if (e < nt) {
            // coalesced reads along k, scattered 4-byte writes (the L2 merges them)
            const int n = (int)(e / K), k = (int)(e % K);
            it.wt[(long long)k * c2 + n] = n < d ? it.wl[(long long)n * K + k] : it.wr[(long long)(n - d) * K + k];
        } else if (e < nt + nc) {
            const long long f = e - nt;
            const int n = (int)(f / kp), k = (int)(f % kp);
            float v = 0.f;
            if (k < K) v = n < d ? it.wl[(long long)n * K + k] : it.wr[(long long)(n - d) * K + k];
            it.wc[f] = v;
        } else {
            const int n = (int)(e - nt - nc);
            it.bc[n] = n < d ? it.bl[n] : it.br[n - d];
        }
    }
}

int launch_repack(const RepackTable& t, hipStream_t s) {
    if (t.n <= 0) return 0;
    hipLaunchKernelGGL(k_repack, dim3(t.n, 96), dim3(256), 0, s, t);
    HGNN_LAUNCH_CHECK();
    return 0;
}

bool gemm2_ok(int lda, int ldb, int ldc, const void* a, const void* b0, const void* b1) {
    auto al = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    return lda % 4 == 0 && ldb % 4 == 0 && ldc % 4 == 0 && al(a) && al(b0) && (b1 == nullptr || al(b1));
}

// Y[r, n] = A[r, :] . WT[:, n] + bias[n]; relu on n >= relu_from; BN partials.
int launch_gemm2_fwd(const float* a, int lda, const int* m_valid, int m_cap, int k, const float* wt, int n,
                     const float* bias, int relu_from, float* y, int ldy, float* bn_part, hipStream_t s) {
    if (m_cap <= 0) return 0;
    G2 p{};
    p.a = a;
    p.lda = lda;
    p.b0 = wt;
    p.b1 = wt;
    p.ldb = n;
    p.bsplit = 1 << 30;
    p.m_cap = m_cap;
    p.m_valid = m_valid;
    p.kdim = k;
    p.n = n;
    p.c = y;
    p.ldc = ldy;
    p.bias = bias;
    p.relu_from = relu_from;
    p.bn_part = bn_part;
    if (n <= 64) {
        const dim3 g(ceil_div(m_cap, 32), ceil_div(n, 64));
        // 32-row tiles: 2x2 waves of 16 rows are not possible with 32x32 MFMA; use BM = 64 instead
        const dim3 g2(ceil_div(m_cap, 64), ceil_div(n, 64));
        (void)g;
        hipLaunchKernelGGL((k_gemm2<64, 64, 32, A_MK, E_FWD>), g2, dim3(256), 0, s, p);
    } else {
        const dim3 g(ceil_div(m_cap, 64), ceil_div(n, 128));
        hipLaunchKernelGGL((k_gemm2<64, 128, 32, A_MK, E_FWD>), g, dim3(256), 0, s, p);
    }
    HGNN_LAUNCH_CHECK();
    return 0;
}

int gemm2_fwd_tile_m(int n) { return 64; }

// dA[r, k] = sum_o dY[r, o] Wcat[o, k]  (Wcat rows split at `split` between w0 and w1)
int launch_gemm2_da(const float* dy, int lddy, const int* m_valid, int m_cap, int o, const float* w0,
                    const float* w1, int split, int ldw, int k, float* da, int ldda, hipStream_t s) {
    if (m_cap <= 0) return 0;
    G2 p{};
    p.a = dy;
    p.lda = lddy;
    p.b0 = w0;
    p.b1 = w1;
    p.ldb = ldw;
    p.bsplit = split;
    p.m_cap = m_cap;
    p.m_valid = m_valid;
    p.kdim = o;
    p.n = k;
    p.c = da;
    p.ldc = ldda;
    const dim3 g(ceil_div(m_cap, 64), ceil_div(k, 128));
    hipLaunchKernelGGL((k_gemm2<64, 128, 32, A_MK, E_STORE>), g, dim3(256), 0, s, p);
    HGNN_LAUNCH_CHECK();
    return 0;
}

int dw2_kchunk(int r_cap, int o, int k) {
    const int tiles = ceil_div(o, o > 64 ? 128 : 64) * ceil_div(k, 128);
    int chunks = 320 / (tiles > 0 ? tiles : 1);
    if (chunks < 1) chunks = 1;
    int kc = ceil_div(r_cap > 0 ? r_cap : 1, chunks);
    kc = ceil_div(kc, 32) * 32;
    return kc < 128 ? 128 : kc;
}

size_t dw2_slab_floats(int r_cap, int o, int k) {
    const int kc = dw2_kchunk(r_cap, o, k);
    return (size_t)ceil_div(r_cap > 0 ? r_cap : 1, kc) * o * k;
}

__global__ void __launch_bounds__(256) k_dw_reduce2(const float* __restrict__ slabs, const int* r_valid,
                                                    int kchunk, int M, int N, int split, float* dw0, float* dw1,
                                                    const float* __restrict__ dbpart, float* db0, float* db1) {
    const int nwb = (M * N + 255) / 256;
    if ((int)blockIdx.x >= nwb) {
        // trailing blocks: the bias gradient of output channel o (k_db_reduce's work, same order)
        __shared__ double red[4];
        const int o = blockIdx.x - nwb;
        const int tv = ceil_div(*r_valid, 64);
        double s = 0.0;
        for (int t = threadIdx.x; t < tv; t += 256) s += (double)dbpart[(long long)t * M + o];
        s = wave_sum_d(s);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            const double t = red[0] + red[1] + red[2] + red[3];
            if (o < split) db0[o] = (float)t;
            else db1[o - split] = (float)t;
        }
        return;
    }
    const int idx = blockIdx.x * 256 + threadIdx.x;
    const int rows = *r_valid;
    if (idx < M * N) {
        const int zv = ceil_div(rows, kchunk);
        const long long st = (long long)M * N;
        float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
        int z = 0;
        for (; z + 4 <= zv; z += 4) {
            s0 += slabs[z * st + idx];
            s1 += slabs[(z + 1) * st + idx];
            s2 += slabs[(z + 2) * st + idx];
            s3 += slabs[(z + 3) * st + idx];
        }
        for (; z < zv; ++z) s0 += slabs[z * st + idx];
        const float s = (s0 + s1) + (s2 + s3);
        const int o = idx / N, c = idx % N;
        if (o < split) dw0[(long long)o * N + c] = s;
        else dw1[(long long)(o - split) * N + c] = s;
    }
}

int launch_dw_reduce2(const float* slabs, const int* r_valid, int kchunk, int o, int k, int split, float* dw0,
                      float* dw1, const float* dbpart, float* db0, float* db1, hipStream_t s) {
    const int total = o * k;
    // one launch: ceil(o k / 256) blocks of slab sums, then o blocks of bias sums
    hipLaunchKernelGGL(k_dw_reduce2, dim3(ceil_div(total, 256) + (dbpart ? o : 0)), dim3(256), 0, s, slabs, r_valid,
                       kchunk, o, k, split, dw0, dw1, dbpart, db0, db1);
    HGNN_LAUNCH_CHECK();
    return 0;
}

// slabs[z][o][k] = sum_{r in chunk z} dY[r, o] A[r, k]
int launch_gemm2_dw(const float* dy, int lddy, const float* a, int lda, const int* r_valid, int r_cap, int o,
                    int k, int kchunk, float* slabs, hipStream_t s) {
    G2 p{};
    p.a = dy;
    p.lda = lddy;
    p.b0 = a;
    p.b1 = a;
    p.ldb = lda;
    p.bsplit = 1 << 30;
    p.m_cap = o;
    p.m_valid = nullptr;
    p.kdim = r_cap;
    p.k_valid = r_valid;
    p.n = k;
    p.kchunk = kchunk;
    p.c = slabs;
    p.ldc = k;
    p.slab_stride = (long long)o * k;
    const int z = ceil_div(r_cap > 0 ? r_cap : 1, kchunk);
    if (o > 64) {
        const dim3 g(ceil_div(o, 128), ceil_div(k, 128), z);
        hipLaunchKernelGGL((k_gemm2<128, 128, 16, A_KM, E_SLAB>), g, dim3(256), 0, s, p);
    } else {
        const dim3 g(ceil_div(o, 64), ceil_div(k, 128), z);
        hipLaunchKernelGGL((k_gemm2<64, 128, 32, A_KM, E_SLAB>), g, dim3(256), 0, s, p);
    }
    HGNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace hgnn
