// GEMM tuning lab (not part of the library): times candidate fp32 MFMA GEMM
// shapes of the LG-GNN step on the box and checks them against a naive kernel.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include tools/gemm_lab.hip -o /tmp/gemm_lab
#include "../hgnn-2_amd/csrc/gemm2.hip"
#include "../hgnn-2_amd/csrc/gemm3.hip"
#include "../hgnn-2_amd/csrc/dwdense.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace hgnn;

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

// C[M][N] = A[M][K] . B[N][K]^T   (both operands k-contiguous), K % 4 == 0.
// k-permuted fragments: MFMA step s of a BK tile contracts k = s and k = BK/2 + s
// (lane half h picks which), so one ds_read_b128 feeds 4 consecutive steps.
template <int BM, int BN, int BK, int WGM, int WGN, int PIPE = 0>
__global__ void __launch_bounds__(64 * WGM * WGN) k_nt(const float* __restrict__ A, int lda,
                                                       const float* __restrict__ B, int ldb, float* __restrict__ C,
                                                       int ldc, int M, int N, int K, int kchunk, long long slab) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int TM = BM / WGM, TN = BN / WGN, AM = TM / 32, AN = TN / 32;
    constexpr int LDK = BK + 4;
    constexpr int AF4 = BM * BK / 4 / NT, BF4 = BN * BK / 4 / NT;
    static_assert(AF4 >= 1 && BF4 >= 1 && AM >= 1 && AN >= 1, "shape");
    __shared__ __attribute__((aligned(16))) float As[2][BM * LDK];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDK];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv / WGN, wn = wv % WGN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const int kbeg = blockIdx.z * kchunk, kend = min(K, kbeg + kchunk);
    float4 ra[AF4], rb[BF4];
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            const int gm = m0 + row, gk = k0 + kq;
            ra[i] = (gm < M && gk < kend) ? *reinterpret_cast<const float4*>(A + (long long)gm * lda + gk)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < BF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            const int gn = n0 + row, gk = k0 + kq;
            rb[i] = (gn < N && gk < kend) ? *reinterpret_cast<const float4*>(B + (long long)gn * ldb + gk)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store = [&](int buf) {
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
    f32x16 acc[AM][AN];
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nt = (kend - kbeg + BK - 1) / BK;
    const int h = lane >> 5, l31 = lane & 31;
    if (nt > 0) {
        load(kbeg);
        store(0);
        __syncthreads();
        if (nt > 1) load(kbeg + BK);
    }
    for (int t = 0; t < nt; ++t) {
        const int buf = t & 1;
        const float* as = &As[buf][(wm * TM + l31) * LDK + h * (BK / 2)];
        const float* bs = &Bs[buf][(wn * TN + l31) * LDK + h * (BK / 2)];
        if constexpr (PIPE == 0) {
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
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
                }
        }
        } else {
            // fragments of group g+1 are read while group g's MFMAs run; MFMA order
            // step-major so consecutive MFMAs hit different accumulators
            float4 fa[2][AM], fb[2][AN];
#pragma unroll
            for (int i = 0; i < AM; ++i) fa[0][i] = *reinterpret_cast<const float4*>(as + i * 32 * LDK);
#pragma unroll
            for (int j = 0; j < AN; ++j) fb[0][j] = *reinterpret_cast<const float4*>(bs + j * 32 * LDK);
#pragma unroll
            for (int g = 0; g < BK / 8; ++g) {
                const int cur = g & 1, nxt = cur ^ 1;
                if (g + 1 < BK / 8) {
#pragma unroll
                    for (int i = 0; i < AM; ++i)
                        fa[nxt][i] = *reinterpret_cast<const float4*>(as + i * 32 * LDK + 4 * (g + 1));
#pragma unroll
                    for (int j = 0; j < AN; ++j)
                        fb[nxt][j] = *reinterpret_cast<const float4*>(bs + j * 32 * LDK + 4 * (g + 1));
                }
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int i = 0; i < AM; ++i)
#pragma unroll
                        for (int j = 0; j < AN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[cur][i][q], fb[cur][j][q], acc[i][j],
                                                                             0, 0, 0);
            }
        }
        if (t + 1 < nt) {
            store(buf ^ 1);
            if (t + 2 < nt) load(kbeg + (t + 2) * BK);
        }
        __syncthreads();
    }
    float* out = C + blockIdx.z * slab;
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j) {
            const int gn = n0 + wn * TN + j * 32 + l31;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gm = m0 + wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (gm < M && gn < N) out[(long long)gm * ldc + gn] = acc[i][j][r];
            }
        }
}

__global__ void k_naive(const float* A, const float* B, float* C, int M, int N, int K) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)M * N) return;
    const int m = idx / N, n = idx % N;
    double s = 0;
    for (int k = 0; k < K; ++k) s += (double)A[(long long)m * K + k] * B[(long long)n * K + k];
    C[idx] = (float)s;
}

__global__ void k_sum_slabs(const float* S, float* C, long long MN, int z) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= MN) return;
    float s = 0.f;
    for (int i = 0; i < z; ++i) s += S[i * MN + idx];
    C[idx] = s;
}

__global__ void k_transpose(const float* B, float* BT, int N, int K) {  // B [N][K] -> BT [K][N]
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)N * K) return;
    const int n = idx / K, k = idx % K;
    BT[(long long)k * N + n] = B[idx];
}

struct Shape {
    const char* name;
    int M, N, K;
};

// Distance-D register prefetch: D register stage sets, so the global loads of k-tile t+D
// are issued while tile t computes (k_nt: D = 1).  LDS stays double-buffered.
template <int BM, int BN, int BK, int WGM, int WGN, int D, int ORD = 0, int MID = 0, int PROBE = 0>
__global__ void __launch_bounds__(64 * WGM * WGN) k_ntd(const float* __restrict__ A, int lda,
                                                        const float* __restrict__ B, int ldb, float* __restrict__ C,
                                                        int ldc, int M, int N, int K) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int TM = BM / WGM, TN = BN / WGN, AM = TM / 32, AN = TN / 32;
    constexpr int LDK = BK + 4;
    constexpr int AF4 = BM * BK / 4 / NT, BF4 = BN * BK / 4 / NT;
    __shared__ __attribute__((aligned(16))) float As[2][BM * LDK];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDK];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv / WGN, wn = wv % WGN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    constexpr unsigned OOB = 0x7ffffff0u;
    const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), 0, M * lda * 4, 0x00020000);
    const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(B), 0, N * ldb * 4, 0x00020000);
    auto ld4 = [](__amdgpu_buffer_rsrc_t r, unsigned off) {
        return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
    };
    float4 ra[D][AF4], rb[D][BF4];
    auto load = [&](int st, int k0) {
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            const int gm = m0 + row, gk = k0 + kq;
            ra[st][i] = ld4(rs_a, (gm < M && gk < K) ? (unsigned)(gm * lda + gk) * 4u : OOB);
        }
#pragma unroll
        for (int i = 0; i < BF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            const int gn = n0 + row, gk = k0 + kq;
            rb[st][i] = ld4(rs_b, (gn < N && gk < K) ? (unsigned)(gn * ldb + gk) * 4u : OOB);
        }
    };
    auto store = [&](int st, int buf) {
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            *reinterpret_cast<float4*>(&As[buf][row * LDK + kq]) = ra[st][i];
        }
#pragma unroll
        for (int i = 0; i < BF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            *reinterpret_cast<float4*>(&Bs[buf][row * LDK + kq]) = rb[st][i];
        }
    };
    f32x16 acc[AM][AN];
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nt = (K + BK - 1) / BK;
    const int h = lane >> 5, l31 = lane & 31;
    // prologue: tiles 0..D loaded, tile 0 stored
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (d < nt) load(d, d * BK);
    store(0, 0);
    __syncthreads();
    if (D < nt) load(0, D * BK);
    // tile t+1 lives in stage (t+1) % D; tile t+D+1 is loaded into the stage freed by the store
    for (int t = 0; t < nt; ++t) {
        const int buf = t & 1;
        const float* as = &As[buf][(wm * TM + l31) * LDK + h * (BK / 2)];
        const float* bs = &Bs[buf][(wn * TN + l31) * LDK + h * (BK / 2)];
        auto next = [&]() {
            if (t + 1 < nt) {
                // stage index must be compile-time for register arrays: unrolled switch over D
#pragma unroll
                for (int d = 0; d < D; ++d)
                    if ((t + 1) % D == d) {
                        if (PROBE != 2) {
                            store(d, buf ^ 1);
                            if (t + 1 + D < nt) load(d, (t + 1 + D) * BK);
                        }
                    }
            }
        };
#pragma unroll
        for (int g = 0; g < BK / 8; ++g) {
            if (MID && g == BK / 16) next();  // next tile's LDS store in the middle of the MFMAs
            float4 a[AM], b[AN];
#pragma unroll
            for (int i = 0; i < AM; ++i) a[i] = *reinterpret_cast<const float4*>(as + i * 32 * LDK + 4 * g);
#pragma unroll
            for (int j = 0; j < AN; ++j) b[j] = *reinterpret_cast<const float4*>(bs + j * 32 * LDK + 4 * g);
            if constexpr (PROBE == 1) {
#pragma unroll
                for (int i = 0; i < AM; ++i)
#pragma unroll
                    for (int j = 0; j < AN; ++j) acc[i][j][0] += a[i].x * b[j].y + a[i].z * b[j].w;
            } else if constexpr (ORD == 0) {
#pragma unroll
                for (int i = 0; i < AM; ++i)
#pragma unroll
                    for (int j = 0; j < AN; ++j) {
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].x, b[j].x, acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].y, b[j].y, acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].z, b[j].z, acc[i][j], 0, 0, 0);
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i].w, b[j].w, acc[i][j], 0, 0, 0);
                    }
            } else {
                // step-major: consecutive MFMAs on different accumulators
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int i = 0; i < AM; ++i)
#pragma unroll
                        for (int j = 0; j < AN; ++j)
                            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i][q], b[j][q], acc[i][j], 0, 0, 0);
            }
        }
        if (!MID) next();
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j) {
            const int gn = n0 + wn * TN + j * 32 + l31;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gm = m0 + wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (gm < M && gn < N) C[(long long)gm * ldc + gn] = acc[i][j][r];
            }
        }
}

template <int BM, int BN, int BK, int WGM, int WGN, int D, int ORD = 0, int MID = 0, int PROBE = 0>
void run_ntd(const char* tag, const Shape& sh, const float* A, const float* B, float* C, const float* ref,
             hipStream_t s) {
    const dim3 g((sh.M + BM - 1) / BM, (sh.N + BN - 1) / BN);
    const long long MN = (long long)sh.M * sh.N;
    auto launch = [&]() {
        hipLaunchKernelGGL((k_ntd<BM, BN, BK, WGM, WGN, D, ORD, MID, PROBE>), g, dim3(64 * WGM * WGN), 0, s, A, sh.K, B, sh.K, C, sh.N,
                           sh.M, sh.N, sh.K);
    };
    launch();
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20;
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<float> hc(MN), hr(MN);
    CK(hipMemcpy(hc.data(), C, MN * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hr.data(), ref, MN * 4, hipMemcpyDeviceToHost));
    double err = 0, mx = 0;
    for (long long i = 0; i < MN; ++i) {
        err = fmax(err, fabs(hc[i] - hr[i]));
        mx = fmax(mx, fabs(hr[i]));
    }
    const double us = ms * 1e3 / reps;
    printf("%-10s %-28s blocks=%6d  %8.1f us  %6.1f TF/s  err=%.2e\n", sh.name, tag, g.x * g.y, us,
           2.0 * sh.M * sh.N * sh.K / (us * 1e-6) / 1e12, err);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

// ---- fp32 GEMM on bf16 MFMA with a 3-way operand split ("bf16x6"): x = hi + mid + lo
// (each bf16 round-to-nearest of the remainder, exact to ~2^-24), product terms
// hh + hm + mh + hl + lh + mm (the dropped ones are <= 2^-23 relative), accumulated in fp32.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3(float4 v, bf16x4_t& h, bf16x4_t& m, bf16x4_t& l) {
    const float x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const __bf16 hi = (__bf16)x[i];
        const float r1 = x[i] - (float)hi;
        const __bf16 mi = (__bf16)r1;
        const float r2 = r1 - (float)mi;
        h[i] = hi;
        m[i] = mi;
        l[i] = (__bf16)r2;
    }
}

template <int BM, int BN, int WGM, int WGN>
__global__ void __launch_bounds__(64 * WGM * WGN) k_x6(const float* __restrict__ A, int lda, const float* __restrict__ B,
                                                       int ldb, float* __restrict__ C, int ldc, int M, int N, int K) {
    constexpr int BK = 32, BKP = BK + 8;  // 80-B LDS rows: conflict-free ds_read_b128
    constexpr int NT = 64 * WGM * WGN;
    constexpr int TM = BM / WGM, TN = BN / WGN, AM = TM / 32, AN = TN / 32;
    constexpr int AF4 = BM * BK / 4 / NT, BF4 = BN * BK / 4 / NT;
    static_assert(AF4 >= 1 && BF4 >= 1 && AM >= 1 && AN >= 1, "shape");
    __shared__ __attribute__((aligned(16))) __bf16 As[2][3][BM * BKP];
    __shared__ __attribute__((aligned(16))) __bf16 Bs[2][3][BN * BKP];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv / WGN, wn = wv % WGN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    constexpr unsigned OOB = 0x7ffffff0u;
    const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), 0, M * lda * 4, 0x00020000);
    const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(B), 0, N * ldb * 4, 0x00020000);
    auto ld4 = [](__amdgpu_buffer_rsrc_t r, unsigned off) {
        return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
    };
    float4 ra[AF4], rb[BF4];
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            const int gm = m0 + row, gk = k0 + kq;
            ra[i] = ld4(rs_a, (gm < M && gk < K) ? (unsigned)(gm * lda + gk) * 4u : OOB);
        }
#pragma unroll
        for (int i = 0; i < BF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            const int gn = n0 + row, gk = k0 + kq;
            rb[i] = ld4(rs_b, (gn < N && gk < K) ? (unsigned)(gn * ldb + gk) * 4u : OOB);
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            bf16x4_t h, m, l;
            split3(ra[i], h, m, l);
            *reinterpret_cast<bf16x4_t*>(&As[buf][0][row * BKP + kq]) = h;
            *reinterpret_cast<bf16x4_t*>(&As[buf][1][row * BKP + kq]) = m;
            *reinterpret_cast<bf16x4_t*>(&As[buf][2][row * BKP + kq]) = l;
        }
#pragma unroll
        for (int i = 0; i < BF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            bf16x4_t h, m, l;
            split3(rb[i], h, m, l);
            *reinterpret_cast<bf16x4_t*>(&Bs[buf][0][row * BKP + kq]) = h;
            *reinterpret_cast<bf16x4_t*>(&Bs[buf][1][row * BKP + kq]) = m;
            *reinterpret_cast<bf16x4_t*>(&Bs[buf][2][row * BKP + kq]) = l;
        }
    };
    f32x16 acc[AM][AN];
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nt = (K + BK - 1) / BK;
    const int h = lane >> 5, l31 = lane & 31;
    load(0);
    store(0);
    __syncthreads();
    if (nt > 1) load(BK);
    for (int t = 0; t < nt; ++t) {
        const int buf = t & 1;
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
            bf16x8_t fa[3][AM], fb[3][AN];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
#pragma unroll
                for (int i = 0; i < AM; ++i)
                    fa[p][i] = *reinterpret_cast<const bf16x8_t*>(&As[buf][p][(wm * TM + i * 32 + l31) * BKP + ks * 16 + 8 * h]);
#pragma unroll
                for (int j = 0; j < AN; ++j)
                    fb[p][j] = *reinterpret_cast<const bf16x8_t*>(&Bs[buf][p][(wn * TN + j * 32 + l31) * BKP + ks * 16 + 8 * h]);
            }
#pragma unroll
            for (int i = 0; i < AM; ++i)
#pragma unroll
                for (int j = 0; j < AN; ++j) {
                    // small terms first
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[1][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[2][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2][i], fb[0][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[1][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[0][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
                }
        }
        if (t + 1 < nt) {
            store(buf ^ 1);
            if (t + 2 < nt) load((t + 2) * BK);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j) {
            const int gn = n0 + wn * TN + j * 32 + l31;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gm = m0 + wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (gm < M && gn < N) C[(long long)gm * ldc + gn] = acc[i][j][r];
            }
        }
}

template <int BM, int BN, int WGM, int WGN>
void run_x6(const char* tag, const Shape& sh, const float* A, const float* B, float* C, const float* ref,
            hipStream_t s) {
    const dim3 g((sh.M + BM - 1) / BM, (sh.N + BN - 1) / BN);
    const long long MN = (long long)sh.M * sh.N;
    auto launch = [&]() {
        hipLaunchKernelGGL((k_x6<BM, BN, WGM, WGN>), g, dim3(64 * WGM * WGN), 0, s, A, sh.K, B, sh.K, C, sh.N, sh.M,
                           sh.N, sh.K);
    };
    launch();
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20;
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<float> hc(MN), hr(MN);
    CK(hipMemcpy(hc.data(), C, MN * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hr.data(), ref, MN * 4, hipMemcpyDeviceToHost));
    double err = 0, mx = 0;
    for (long long i = 0; i < MN; ++i) {
        err = fmax(err, fabs(hc[i] - hr[i]));
        mx = fmax(mx, fabs(hr[i]));
    }
    const double us = ms * 1e3 / reps;
    printf("%-10s %-28s blocks=%6d  %8.1f us  %6.1f TF/s(fp32-eq)  err=%.2e (max|ref| %.1f)\n", sh.name, tag, g.x * g.y,
           us, 2.0 * sh.M * sh.N * sh.K / (us * 1e-6) / 1e12, err, mx);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

// v2: BK templated, register prefetch distance D, B optionally pre-split in global
// (3 bf16 planes [3][N][K], written once per weight update), LDS double-buffered.
__global__ void k_split_planes(const float* __restrict__ x, __bf16* __restrict__ planes, long long n) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float v = x[i];
    const __bf16 hi = (__bf16)v;
    const float r1 = v - (float)hi;
    const __bf16 mi = (__bf16)r1;
    planes[i] = hi;
    planes[n + i] = mi;
    planes[2 * n + i] = (__bf16)(r1 - (float)mi);
}

template <int BM, int BN, int BK, int WGM, int WGN, int D, bool PREB>
__global__ void __launch_bounds__(64 * WGM * WGN) k_x6b(const float* __restrict__ A, int lda, const float* __restrict__ B,
                                                        const __bf16* __restrict__ Bp, int ldb, float* __restrict__ C,
                                                        int ldc, int M, int N, int K) {
    constexpr int BKP = BK + 8;
    constexpr int NT = 64 * WGM * WGN;
    constexpr int TM = BM / WGM, TN = BN / WGN, AM = TM / 32, AN = TN / 32;
    constexpr int AF4 = BM * BK / 4 / NT, BF4 = BN * BK / 4 / NT;
    static_assert(AF4 >= 1 && BF4 >= 1 && AM >= 1 && AN >= 1, "shape");
    __shared__ __attribute__((aligned(16))) __bf16 As[2][3][BM * BKP];
    __shared__ __attribute__((aligned(16))) __bf16 Bs[2][3][BN * BKP];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv / WGN, wn = wv % WGN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    constexpr unsigned OOB = 0x7ffffff0u;
    const auto rs_a = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A), 0, M * lda * 4, 0x00020000);
    const auto rs_b = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(B), 0, N * ldb * 4, 0x00020000);
    const long long np = (long long)N * ldb;  // plane size (elements)
    const auto rs_p = __builtin_amdgcn_make_buffer_rsrc(const_cast<__bf16*>(Bp), 0, (int)(3 * np * 2), 0x00020000);
    auto ld4 = [](__amdgpu_buffer_rsrc_t r, unsigned off) {
        return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
    };
    auto ld2 = [](__amdgpu_buffer_rsrc_t r, unsigned off) {
        return __builtin_bit_cast(bf16x4_t, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
    };
    float4 ra[D][AF4], rb[D][PREB ? 1 : BF4];
    bf16x4_t rp[D][PREB ? 3 : 1][PREB ? BF4 : 1];
    auto load = [&](int st, int k0) {
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            const int gm = m0 + row, gk = k0 + kq;
            ra[st][i] = ld4(rs_a, (gm < M && gk < K) ? (unsigned)(gm * lda + gk) * 4u : OOB);
        }
#pragma unroll
        for (int i = 0; i < BF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            const int gn = n0 + row, gk = k0 + kq;
            const bool ok = gn < N && gk < K;
            if constexpr (PREB) {
#pragma unroll
                for (int q = 0; q < 3; ++q)
                    rp[st][q][i] = ld2(rs_p, ok ? (unsigned)(q * np + gn * ldb + gk) * 2u : OOB);
            } else {
                rb[st][i] = ld4(rs_b, ok ? (unsigned)(gn * ldb + gk) * 4u : OOB);
            }
        }
    };
    auto store = [&](int st, int buf) {
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            bf16x4_t h, m, l;
            split3(ra[st][i], h, m, l);
            *reinterpret_cast<bf16x4_t*>(&As[buf][0][row * BKP + kq]) = h;
            *reinterpret_cast<bf16x4_t*>(&As[buf][1][row * BKP + kq]) = m;
            *reinterpret_cast<bf16x4_t*>(&As[buf][2][row * BKP + kq]) = l;
        }
#pragma unroll
        for (int i = 0; i < BF4; ++i) {
            const int e = tid + i * NT, row = e / (BK / 4), kq = (e % (BK / 4)) * 4;
            if constexpr (PREB) {
#pragma unroll
                for (int q = 0; q < 3; ++q) *reinterpret_cast<bf16x4_t*>(&Bs[buf][q][row * BKP + kq]) = rp[st][q][i];
            } else {
                bf16x4_t h, m, l;
                split3(rb[st][i], h, m, l);
                *reinterpret_cast<bf16x4_t*>(&Bs[buf][0][row * BKP + kq]) = h;
                *reinterpret_cast<bf16x4_t*>(&Bs[buf][1][row * BKP + kq]) = m;
                *reinterpret_cast<bf16x4_t*>(&Bs[buf][2][row * BKP + kq]) = l;
            }
        }
    };
    f32x16 acc[AM][AN];
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nt = (K + BK - 1) / BK;
    const int h = lane >> 5, l31 = lane & 31;
#pragma unroll
    for (int d = 0; d < D; ++d)
        if (d < nt) load(d, d * BK);
    store(0, 0);
    __syncthreads();
    if (D < nt) load(0, D * BK);
    for (int t = 0; t < nt; ++t) {
        const int buf = t & 1;
#pragma unroll
        for (int ks = 0; ks < BK / 16; ++ks) {
            bf16x8_t fa[3][AM], fb[3][AN];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
#pragma unroll
                for (int i = 0; i < AM; ++i)
                    fa[p][i] = *reinterpret_cast<const bf16x8_t*>(&As[buf][p][(wm * TM + i * 32 + l31) * BKP + ks * 16 + 8 * h]);
#pragma unroll
                for (int j = 0; j < AN; ++j)
                    fb[p][j] = *reinterpret_cast<const bf16x8_t*>(&Bs[buf][p][(wn * TN + j * 32 + l31) * BKP + ks * 16 + 8 * h]);
            }
#pragma unroll
            for (int i = 0; i < AM; ++i)
#pragma unroll
                for (int j = 0; j < AN; ++j) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[1][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[2][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2][i], fb[0][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[1][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][i], fb[0][j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][i], fb[0][j], acc[i][j], 0, 0, 0);
                }
        }
        if (t + 1 < nt) {
#pragma unroll
            for (int d = 0; d < D; ++d)
                if ((t + 1) % D == d) {
                    store(d, buf ^ 1);
                    if (t + 1 + D < nt) load(d, (t + 1 + D) * BK);
                }
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j) {
            const int gn = n0 + wn * TN + j * 32 + l31;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gm = m0 + wm * TM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (gm < M && gn < N) C[(long long)gm * ldc + gn] = acc[i][j][r];
            }
        }
}

template <int BM, int BN, int BK, int WGM, int WGN, int D, bool PREB>
void run_x6b(const char* tag, const Shape& sh, const float* A, const float* B, float* C, const float* ref,
             hipStream_t s) {
    const dim3 g((sh.M + BM - 1) / BM, (sh.N + BN - 1) / BN);
    const long long MN = (long long)sh.M * sh.N, NB = (long long)sh.N * sh.K;
    __bf16* Bp;
    CK(hipMalloc(&Bp, 3 * NB * 2));
    hipLaunchKernelGGL(k_split_planes, dim3((NB + 255) / 256), dim3(256), 0, s, B, Bp, NB);
    auto launch = [&]() {
        hipLaunchKernelGGL((k_x6b<BM, BN, BK, WGM, WGN, D, PREB>), g, dim3(64 * WGM * WGN), 0, s, A, sh.K, B, Bp, sh.K,
                           C, sh.N, sh.M, sh.N, sh.K);
    };
    launch();
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20;
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<float> hc(MN), hr(MN);
    CK(hipMemcpy(hc.data(), C, MN * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hr.data(), ref, MN * 4, hipMemcpyDeviceToHost));
    double err = 0;
    for (long long i = 0; i < MN; ++i) err = fmax(err, fabs(hc[i] - hr[i]));
    const double us = ms * 1e3 / reps;
    printf("%-10s %-32s blocks=%6d  %8.1f us  %6.1f TF/s(fp32-eq)  err=%.2e\n", sh.name, tag, g.x * g.y, us,
           2.0 * sh.M * sh.N * sh.K / (us * 1e-6) / 1e12, err);
    CK(hipFree(Bp));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

template <int BM, int BN, int BK, int WGM, int WGN, int PIPE = 0>
void run_nt(const char* tag, const Shape& sh, const float* A, const float* B, float* C, float* slabs, const float* ref,
            int splits, hipStream_t s) {
    const int kchunk = ((sh.K + splits - 1) / splits + BK - 1) / BK * BK;
    const int z = (sh.K + kchunk - 1) / kchunk;
    const dim3 g((sh.M + BM - 1) / BM, (sh.N + BN - 1) / BN, z);
    const long long MN = (long long)sh.M * sh.N;
    float* dst = z > 1 ? slabs : C;
    auto launch = [&]() {
        hipLaunchKernelGGL((k_nt<BM, BN, BK, WGM, WGN, PIPE>), g, dim3(64 * WGM * WGN), 0, s, A, sh.K, B, sh.K, dst, sh.N,
                           sh.M, sh.N, sh.K, kchunk, MN);
        if (z > 1) hipLaunchKernelGGL(k_sum_slabs, dim3((MN + 255) / 256), dim3(256), 0, s, slabs, C, MN, z);
    };
    launch();
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20;
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<float> hc(MN), hr(MN);
    CK(hipMemcpy(hc.data(), C, MN * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hr.data(), ref, MN * 4, hipMemcpyDeviceToHost));
    double err = 0, mx = 0;
    for (long long i = 0; i < MN; ++i) {
        err = fmax(err, fabs(hc[i] - hr[i]));
        mx = fmax(mx, fabs(hr[i]));
    }
    const double us = ms * 1e3 / reps;
    const double tf = 2.0 * sh.M * sh.N * sh.K / (us * 1e-6) / 1e12;
    printf("%-10s %-28s split=%d blocks=%6d  %8.1f us  %6.1f TF/s  err=%.2e (max|ref| %.1f)\n", sh.name, tag, z,
           g.x * g.y * g.z, us, tf, err, mx);
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
}

// dW-style "TN": C[z][M][N] = sum_{r in chunk z} A[r][m] B[r][n]; A = dY [R][M], B = Agg [R][N].
// LDS keeps the natural [k][m] layout (float4 copies); fragments by ds_read_b32
// with the same k permutation (step s contracts rows s and BK/2 + s).
template <int BM, int BN, int BK, int WGM, int WGN>
__global__ void __launch_bounds__(64 * WGM * WGN) k_tn(const float* __restrict__ A, int lda,
                                                       const float* __restrict__ B, int ldb, float* __restrict__ C,
                                                       int M, int N, int R, int kchunk) {
    constexpr int NT = 64 * WGM * WGN;
    constexpr int TM = BM / WGM, TN = BN / WGN, AM = TM / 32, AN = TN / 32;
    constexpr int PA = BM + 4, PB = BN + 4;
    constexpr int AF4 = BM * BK / 4 / NT, BF4 = BN * BK / 4 / NT;
    static_assert(AF4 >= 1 && BF4 >= 1 && AM >= 1 && AN >= 1, "shape");
    __shared__ __attribute__((aligned(16))) float As[2][BK * PA];
    __shared__ __attribute__((aligned(16))) float Bs[2][BK * PB];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv / WGN, wn = wv % WGN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const int kbeg = blockIdx.z * kchunk, kend = min(R, kbeg + kchunk);
    float4 ra[AF4], rb[BF4];
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < AF4; ++i) {
            const int e = tid + i * NT, kr = e / (BM / 4), mq = (e % (BM / 4)) * 4;
            const int gk = k0 + kr, gm = m0 + mq;
            ra[i] = (gk < kend && gm < M) ? *reinterpret_cast<const float4*>(A + (long long)gk * lda + gm)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int i = 0; i < BF4; ++i) {
            const int e = tid + i * NT, kr = e / (BN / 4), nq = (e % (BN / 4)) * 4;
            const int gk = k0 + kr, gn = n0 + nq;
            rb[i] = (gk < kend && gn < N) ? *reinterpret_cast<const float4*>(B + (long long)gk * ldb + gn)
                                          : make_float4(0.f, 0.f, 0.f, 0.f);
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
    const int nt = (kend - kbeg + BK - 1) / BK;
    const int h = lane >> 5, l31 = lane & 31;
    if (nt > 0) {
        load(kbeg);
        store(0);
        __syncthreads();
        if (nt > 1) load(kbeg + BK);
    }
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
    float* out = C + (long long)blockIdx.z * M * N;
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
}

__global__ void k_naive_tn(const float* A, const float* B, float* C, int M, int N, int R) {
    const long long idx = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long long)M * N) return;
    const int m = idx / N, n = idx % N;
    double s = 0;
    for (int r = 0; r < R; ++r) s += (double)A[(long long)r * M + m] * B[(long long)r * N + n];
    C[idx] = (float)s;
}

template <int BM, int BN, int BK, int WGM, int WGN>
void run_tn(const char* tag, int M, int N, int R, const float* A, const float* B, float* C, float* slabs,
            const float* ref, int target_blocks, hipStream_t s) {
    const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    int z = target_blocks / tiles;
    if (z < 1) z = 1;
    int kchunk = (R + z - 1) / z;
    kchunk = (kchunk + BK - 1) / BK * BK;
    z = (R + kchunk - 1) / kchunk;
    const dim3 g((M + BM - 1) / BM, (N + BN - 1) / BN, z);
    const long long MN = (long long)M * N;
    auto launch = [&]() {
        hipLaunchKernelGGL((k_tn<BM, BN, BK, WGM, WGN>), g, dim3(64 * WGM * WGN), 0, s, A, M, B, N, slabs, M, N, R,
                           kchunk);
    };
    auto reduce = [&]() {
        hipLaunchKernelGGL(k_sum_slabs, dim3((MN + 255) / 256), dim3(256), 0, s, slabs, C, MN, z);
    };
    launch();
    reduce();
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    const int reps = 20;
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1, s));
    for (int r = 0; r < reps; ++r) reduce();
    CK(hipEventRecord(e2, s));
    CK(hipEventSynchronize(e2));
    float ms, ms2;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventElapsedTime(&ms2, e1, e2));
    std::vector<float> hc(MN), hr(MN);
    CK(hipMemcpy(hc.data(), C, MN * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hr.data(), ref, MN * 4, hipMemcpyDeviceToHost));
    double err = 0, mx = 0;
    for (long long i = 0; i < MN; ++i) {
        err = fmax(err, fabs(hc[i] - hr[i]));
        mx = fmax(mx, fabs(hr[i]));
    }
    const double us = ms * 1e3 / reps, us2 = ms2 * 1e3 / reps;
    printf("dW R=%-6d %-30s z=%3d blocks=%5d gemm %7.1f us (%6.1f TF/s) + reduce %5.1f us  err=%.2e (max %.1f)\n", R, tag,
           z, g.x * g.y * g.z, us, 2.0 * M * N * R / (us * 1e-6) / 1e12, us2, err, mx);
}

void dw_lab(hipStream_t s) {
    const int M = 128, N = 640;
    for (int R : {9728, 23296}) {
        std::vector<float> ha((size_t)R * M), hb((size_t)R * N);
        srand(2);
        for (auto& v : ha) v = (float)rand() / (float)RAND_MAX - 0.5f;
        for (auto& v : hb) v = (float)rand() / (float)RAND_MAX - 0.5f;
        float *A, *B, *C, *Rf, *S;
        CK(hipMalloc(&A, ha.size() * 4));
        CK(hipMalloc(&B, hb.size() * 4));
        CK(hipMalloc(&C, (size_t)M * N * 4));
        CK(hipMalloc(&Rf, (size_t)M * N * 4));
        CK(hipMalloc(&S, (size_t)M * N * 4 * 512));
        CK(hipMemcpy(A, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(B, hb.data(), hb.size() * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_naive_tn, dim3((M * N + 255) / 256), dim3(256), 0, s, A, B, Rf, M, N, R);
        CK(hipStreamSynchronize(s));
        {  // current library path (v2 slab GEMM, reduce not included)
            const int kc = dw2_kchunk(R, M, N);
            auto launch = [&]() { launch_gemm2_dw(A, M, B, N, nullptr, R, M, N, kc, S, s); };
            launch();
            CK(hipStreamSynchronize(s));
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < 20; ++r) launch();
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("dW R=%-6d %-30s gemm %7.1f us\n", R, "v2 launch_gemm2_dw", ms * 1e3 / 20);
        }
        for (int tb : {256, 512, 1024}) {
            run_tn<128, 128, 32, 2, 2>("tn<128,128,32,2x2>", M, N, R, A, B, C, S, Rf, tb, s);
            run_tn<128, 128, 16, 2, 2>("tn<128,128,16,2x2>", M, N, R, A, B, C, S, Rf, tb, s);
            run_tn<64, 128, 32, 2, 2>("tn<64,128,32,2x2>", M, N, R, A, B, C, S, Rf, tb, s);
            run_tn<128, 64, 32, 2, 2>("tn<128,64,32,2x2>", M, N, R, A, B, C, S, Rf, tb, s);
            run_tn<128, 128, 32, 4, 2>("tn<128,128,32,4x2> 512", M, N, R, A, B, C, S, Rf, tb, s);
        }
        CK(hipFree(A));
        CK(hipFree(B));
        CK(hipFree(C));
        CK(hipFree(Rf));
        CK(hipFree(S));
    }
}

void dwdense_lab(hipStream_t s) {
    const int bs = 512, nmax = 29, F = 128, J = 3, lda = 640;
    std::vector<int> off(bs + 1);
    srand(3);
    off[0] = 0;
    for (int b = 0; b < bs; ++b) off[b + 1] = off[b] + 9 + rand() % 21;
    const int rows = off[bs];
    float *dA, *xp, *dW, *mean, *stdv, *pw, *pb;
    int* noff;
    CK(hipMalloc(&dA, (size_t)rows * lda * 4));
    CK(hipMalloc(&xp, (size_t)rows * F * 4));
    CK(hipMalloc(&dW, (size_t)bs * nmax * nmax * J * 4));
    CK(hipMalloc(&mean, F * 4));
    CK(hipMalloc(&stdv, F * 4));
    CK(hipMalloc(&pw, 4));
    CK(hipMalloc(&pb, 4));
    CK(hipMalloc(&noff, (bs + 1) * 4));
    CK(hipMemcpy(noff, off.data(), (bs + 1) * 4, hipMemcpyHostToDevice));
    CK(hipMemset(dA, 0, (size_t)rows * lda * 4));
    CK(hipMemset(xp, 0, (size_t)rows * F * 4));
    CK(hipMemset(dW, 0, (size_t)bs * nmax * nmax * J * 4));
    std::vector<float> ones(F, 1.f);
    CK(hipMemcpy(stdv, ones.data(), F * 4, hipMemcpyHostToDevice));
    CK(hipMemset(mean, 0, F * 4));
    CK(hipMemset(pw, 0, 4));
    CK(hipMemset(pb, 0, 4));
    for (int acc = 0; acc < 2; ++acc) {
        DwDenseArgs a{};
        a.dA = dA;
        a.lda = lda;
        a.f = F;
        a.jt = J;
        a.xp = xp;
        a.pmean = mean;
        a.pstd = stdv;
        a.pw = pw;
        a.pb = pb;
        a.node_off = noff;
        a.bs = bs;
        a.nmax = nmax;
        a.dW = dW;
        a.accumulate = acc;
        launch_dw_dense(a, s);
        CK(hipStreamSynchronize(s));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < 20; ++r) launch_dw_dense(a, s);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("dw_dense bs=%d nmax=%d F=%d accumulate=%d: %.1f us\n", bs, nmax, F, acc, ms * 1e3 / 20);
    }
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    if (getenv("LAB_DWDENSE")) {
        dwdense_lab(s);
        return 0;
    }
    if (getenv("LAB_DW")) {
        dw_lab(s);
        return 0;
    }
    const Shape shapes[] = {
        {"node_fwd", 9728, 128, 640},
        {"edge_fwd", 23296, 128, 640},
        {"edge_dA", 23296, 640, 128},
        {"node_dA", 9728, 640, 128},
        {"bal256_fwd", 16384, 128, 640},  // exactly 256 tiles of 64 rows: no tail imbalance
        {"bal512_fwd", 32768, 128, 640},  // 512 tiles: two per CU
    };
    for (const Shape& sh : shapes) {
        const long long na = (long long)sh.M * sh.K, nb = (long long)sh.N * sh.K, nc = (long long)sh.M * sh.N;
        std::vector<float> ha(na), hb(nb);
        srand(1);
        for (auto& v : ha) v = (float)rand() / RAND_MAX - 0.5f;
        for (auto& v : hb) v = (float)rand() / RAND_MAX - 0.5f;
        float *A, *B, *BT, *C, *R, *S, *bias;
        CK(hipMalloc(&A, na * 4));
        CK(hipMalloc(&B, nb * 4));
        CK(hipMalloc(&BT, nb * 4));
        CK(hipMalloc(&C, nc * 4));
        CK(hipMalloc(&R, nc * 4));
        CK(hipMalloc(&S, nc * 4 * 8));
        CK(hipMalloc(&bias, sh.N * 4));
        CK(hipMemset(bias, 0, sh.N * 4));
        CK(hipMemcpy(A, ha.data(), na * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(B, hb.data(), nb * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_naive, dim3((nc + 255) / 256), dim3(256), 0, s, A, B, R, sh.M, sh.N, sh.K);
        hipLaunchKernelGGL(k_transpose, dim3((nb + 255) / 256), dim3(256), 0, s, B, BT, sh.N, sh.K);
        CK(hipStreamSynchronize(s));
        // current library kernel (v2) for reference
        {
            auto launch = [&]() {
                launch_gemm2_fwd(A, sh.K, nullptr, sh.M, sh.K, BT, sh.N, bias, 1 << 30, C, sh.N, nullptr, s);
            };
            launch();
            CK(hipStreamSynchronize(s));
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < 20; ++r) launch();
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / 20;
            printf("%-10s %-28s                       %8.1f us  %6.1f TF/s\n", sh.name, "v2 k_gemm2<64,128,32>", us,
                   2.0 * sh.M * sh.N * sh.K / (us * 1e-6) / 1e12);
        }
        {
            int* mv;
            float* part;
            const int cap = sh.M * 3 / 2;
            CK(hipMalloc(&mv, 4));
            CK(hipMemcpy(mv, &sh.M, 4, hipMemcpyHostToDevice));
            CK(hipMalloc(&part, (size_t)(cap / 64 + 1) * sh.N * 3 * 4));
            float* Abig;
            CK(hipMalloc(&Abig, (size_t)cap * sh.K * 4));
            CK(hipMemcpy(Abig, A, na * 4, hipMemcpyDeviceToDevice));
            auto timeit = [&](const char* tag, auto&& launch, int reps) {
                launch();
                CK(hipStreamSynchronize(s));
                hipEvent_t e0, e1;
                CK(hipEventCreate(&e0));
                CK(hipEventCreate(&e1));
                CK(hipEventRecord(e0, s));
                for (int r = 0; r < reps; ++r) launch();
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double us = ms * 1e3 / reps;
                printf("%-10s %-40s reps=%5d %8.1f us  %6.1f TF/s\n", sh.name, tag, reps, us,
                       2.0 * sh.M * sh.N * sh.K / (us * 1e-6) / 1e12);
            };
            auto lib_fwd = [&]() {
                launch_gemm3_fwd(Abig, sh.K, mv, cap, sh.K, B, sh.K, sh.N, bias, sh.N / 2, C, sh.N, part, s);
            };
            auto lib_nopart = [&]() {
                launch_gemm3_fwd(Abig, sh.K, mv, cap, sh.K, B, sh.K, sh.N, bias, sh.N / 2, C, sh.N, nullptr, s);
            };
            auto lib_da = [&]() { launch_gemm3_da(Abig, sh.K, mv, cap, sh.K, B, sh.K, sh.N, C, sh.N, s); };
            auto lib_exact = [&]() {
                launch_gemm3_fwd(Abig, sh.K, nullptr, sh.M, sh.K, B, sh.K, sh.N, bias, sh.N / 2, C, sh.N, nullptr, s);
            };
            auto lib_exact_part = [&]() {
                launch_gemm3_fwd(Abig, sh.K, nullptr, sh.M, sh.K, B, sh.K, sh.N, bias, sh.N / 2, C, sh.N, part, s);
            };
            timeit("lib gemm3_fwd (exact M, no m_valid, no part)", lib_exact, 20);
            timeit("lib gemm3_fwd (exact M, no m_valid, part)", lib_exact_part, 20);
            timeit("lib gemm3_fwd (m_valid, bn_part)", lib_fwd, 20);
            timeit("lib gemm3_fwd (m_valid, no part)", lib_nopart, 20);
            timeit("lib gemm3_da  (m_valid)", lib_da, 20);
            timeit("lib gemm3_fwd x2000 (heat)", lib_fwd, 2000);
            timeit("lib gemm3_fwd after heat", lib_fwd, 20);
            CK(hipFree(mv));
            CK(hipFree(part));
            CK(hipFree(Abig));
        }
        if (getenv("LAB_SPLIT")) {
            // split-K with a separate slab-sum kernel: does finer work granularity pay at these M?
            run_ntd<64, 64, 32, 2, 2, 1>("ntd<64,64,32,2x2> D1", sh, A, B, C, R, s);
            run_ntd<64, 64, 32, 2, 2, 1, 0, 0, 1>("ntd<64,64> PROBE staging-only", sh, A, B, C, R, s);
            run_ntd<64, 64, 32, 2, 2, 1, 0, 0, 2>("ntd<64,64> PROBE mfma+lds-only", sh, A, B, C, R, s);
            run_x6<64, 64, 2, 2>("x6<64,64,2x2>", sh, A, B, C, R, s);
            for (int sp : {1}) {
                run_nt<64, 128, 32, 2, 2>("nt<64,128,32,2x2>", sh, A, B, C, S, R, sp, s);
                run_nt<64, 64, 32, 2, 2>("nt<64,64,32,2x2>", sh, A, B, C, S, R, sp, s);
                run_nt<32, 128, 32, 1, 4>("nt<32,128,32,1x4>", sh, A, B, C, S, R, sp, s);
            }
            CK(hipFree(A));
            CK(hipFree(B));
            CK(hipFree(BT));
            CK(hipFree(C));
            CK(hipFree(R));
            CK(hipFree(S));
            CK(hipFree(bias));
            continue;
        }
        for (int sp : {1}) {
            run_nt<64, 128, 32, 2, 2>("nt<64,128,32,2x2>", sh, A, B, C, S, R, sp, s);
            run_nt<64, 128, 32, 2, 2, 1>("nt<64,128,32,2x2> pipe", sh, A, B, C, S, R, sp, s);
            run_nt<64, 128, 64, 2, 2, 1>("nt<64,128,64,2x2> pipe", sh, A, B, C, S, R, sp, s);
            run_nt<64, 64, 32, 2, 2, 1>("nt<64,64,32,2x2> pipe", sh, A, B, C, S, R, sp, s);
            run_nt<64, 64, 64, 2, 2, 1>("nt<64,64,64,2x2> pipe", sh, A, B, C, S, R, sp, s);
            run_nt<128, 128, 32, 2, 2, 1>("nt<128,128,32,2x2> pipe", sh, A, B, C, S, R, sp, s);
            run_nt<128, 128, 32, 4, 2, 1>("nt<128,128,32,4x2> pipe 512", sh, A, B, C, S, R, sp, s);
            run_nt<64, 128, 32, 2, 4, 1>("nt<64,128,32,2x4> pipe 512", sh, A, B, C, S, R, sp, s);
            run_nt<128, 64, 32, 4, 2, 1>("nt<128,64,32,4x2> pipe 512", sh, A, B, C, S, R, sp, s);
            run_nt<32, 128, 32, 1, 4, 1>("nt<32,128,32,1x4> pipe", sh, A, B, C, S, R, sp, s);
        }
        CK(hipFree(A));
        CK(hipFree(B));
        CK(hipFree(BT));
        CK(hipFree(C));
        CK(hipFree(R));
        CK(hipFree(S));
        CK(hipFree(bias));
    }
    return 0;
}
