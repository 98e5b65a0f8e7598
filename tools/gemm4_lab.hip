// GEMM staging lab: the library's NT GEMM (k_gemm3, register-staged, 2 LDS buffers) against an
// LDS-DMA pipeline (buffer_load ... lds, 3 stages, XOR-swizzled 128-B rows, raw s_barrier with a
// counted vmcnt) on the config-2 shapes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/gemm4_lab.hip -o tools/gemm4_lab
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../hgnn-2_amd/csrc/gemm3.hip"

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

using namespace hgnn;

typedef float f32x16 __attribute__((ext_vector_type(16)));


typedef int i32x4 __attribute__((ext_vector_type(4)));

// buffer descriptor in SGPRs: base, stride 0, num_records = bytes (offsets past it read 0)
__device__ __forceinline__ i32x4 rsrc(const void* p, int bytes) {
    const unsigned long long a = (unsigned long long)(uintptr_t)p;
    i32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
    r.y = __builtin_amdgcn_readfirstlane((int)(a >> 32) & 0xffff);
    r.z = __builtin_amdgcn_readfirstlane(bytes);
    r.w = 0x00020000;
    return r;
}

// 16 B per lane, global -> LDS (wave-uniform LDS byte address + lane * 16).  Inline asm keeps the
// load out of hipcc's waitcnt bookkeeping: the kernel counts it with its own vmcnt waits.
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

// PR: 0 = the kernel; 1 = no staging in the loop (MFMA + LDS reads on stale tiles); 2 = staging only
template <int BM, int BN, int WGM, int WGN, int ST, int PR = 0>
__global__ void __launch_bounds__(64 * WGM * WGN) k_g4(const float* __restrict__ A, int lda,
                                                       const float* __restrict__ B, int ldb, int M, int N, int K,
                                                       float* __restrict__ C, int ldc) {
    constexpr int BK = 32, NW = WGM * WGN;
    constexpr int TM = BM / WGM, TN = BN / WGN, AM = TM / 32, AN = TN / 32;
    constexpr int AI = BM * BK * 4 / 1024, BI = BN * BK * 4 / 1024;  // 1-KB wave instructions per stage
    static_assert(AI % NW == 0 && BI % NW == 0, "staging split");
    constexpr int APW = AI / NW, BPW = BI / NW, PER = APW + BPW;
    constexpr int SF = (BM + BN) * BK;  // floats per stage
    __shared__ __attribute__((aligned(1024))) float lds[ST * SF];

    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wv / WGN, wn = wv % WGN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    if (m0 >= M) return;
    constexpr unsigned OOB = 0x7ffffff0u;
    const i32x4 ra = rsrc(A, M * lda * 4), rb = rsrc(B, N * ldb * 4);
    const int lrow = lane >> 3, lslot = lane & 7;
    const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)lds;
    auto issue = [&](int st, int k0) {
        const unsigned base = lds0 + st * SF * 4;
#pragma unroll
        for (int i = 0; i < APW; ++i) {
            const int inst = wv * APW + i, row = inst * 8 + lrow;
            const int s = lslot ^ ((row >> 1) & 7), gm = m0 + row, gk = k0 + 4 * s;
            const unsigned off = (gm < M && gk < K) ? (unsigned)(gm * lda + gk) * 4u : OOB;
            dma16(ra, off, base + inst * 1024);
        }
#pragma unroll
        for (int i = 0; i < BPW; ++i) {
            const int inst = wv * BPW + i, row = inst * 8 + lrow;
            const int s = lslot ^ ((row >> 1) & 7), gn = n0 + row, gk = k0 + 4 * s;
            const unsigned off = (gn < N && gk < K) ? (unsigned)(gn * ldb + gk) * 4u : OOB;
            dma16(rb, off, base + BM * BK * 4 + inst * 1024);
        }
    };
    f32x16 acc[AM][AN], tacc[AM][AN];
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nt = (K + BK - 1) / BK;
    const int h = lane >> 5, l31 = lane & 31, sw = (l31 >> 1) & 7;
#pragma unroll
    for (int p = 0; p < ST - 1; ++p)
        if (p < nt) issue(p, p * BK);
    if (nt > 1) stage_barrier<(ST - 2) * PER>();
    else stage_barrier<0>();
    for (int t = 0; t < nt; ++t) {
        if (PR != 1 && t + ST - 1 < nt) issue((t + ST - 1) % ST, (t + ST - 1) * BK);
        const float* as = lds + (t % ST) * SF + (wm * TM + l31) * BK;
        const float* bs = lds + (t % ST) * SF + BM * BK + (wn * TN + l31) * BK;
#pragma unroll
        for (int i = 0; i < AM; ++i)
#pragma unroll
            for (int j = 0; j < AN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) tacc[i][j][r] = 0.f;
#pragma unroll
        for (int g = 0; g < (PR == 2 ? 1 : BK / 8); ++g) {
            const int slot = (h * 4 + g) ^ sw;
            float4 a[AM], b[AN];
#pragma unroll
            for (int i = 0; i < AM; ++i) a[i] = *reinterpret_cast<const float4*>(as + i * 32 * BK + 4 * slot);
#pragma unroll
            for (int j = 0; j < AN; ++j) b[j] = *reinterpret_cast<const float4*>(bs + j * 32 * BK + 4 * slot);
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
        // tile t + 1 landed (this wave's part): later tiles may stay in flight
        if constexpr (ST >= 3) {
            if (t + ST - 1 < nt) stage_barrier<(ST - 2) * PER>();
            else stage_barrier<0>();
        } else {
            stage_barrier<0>();
        }
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

typedef float f32x4 __attribute__((ext_vector_type(4)));

// The same pipeline on v_mfma_f32_16x16x4_f32: MI355X_MICROARCH.md (DVFS give-back, item 7) measures
// the 16x16 MFMA shape holding a higher clock than the 32x32 one at equal cycles per FLOP.
// Wave tile 32x32 = 2 x 2 tiles of 16x16; lane (l15, g = lane >> 4) reads 4 consecutive k of its
// row (16-B slot hh * 4 + g of the 128-B row) and feeds element s to MFMA step s, so step s of half
// hh contracts k = 16 hh + 4 g + s over the 4 lane groups -- the same permutation on A and B.
template <int BM, int BN, int WGM, int WGN, int ST>
__global__ void __launch_bounds__(64 * WGM * WGN) k_g5(const float* __restrict__ A, int lda,
                                                       const float* __restrict__ B, int ldb, int M, int N, int K,
                                                       float* __restrict__ C, int ldc) {
    constexpr int BK = 32, NW = WGM * WGN;
    constexpr int TM = BM / WGM, TN = BN / WGN, AM = TM / 16, AN = TN / 16;
    constexpr int AI = BM * BK * 4 / 1024, BI = BN * BK * 4 / 1024;
    static_assert(AI % NW == 0 && BI % NW == 0, "staging split");
    constexpr int APW = AI / NW, BPW = BI / NW, PER = APW + BPW;
    constexpr int SF = (BM + BN) * BK;
    __shared__ __attribute__((aligned(1024))) float lds[ST * SF];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wv / WGN, wn = wv % WGN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    if (m0 >= M) return;
    constexpr unsigned OOB = 0x7ffffff0u;
    const i32x4 ra = rsrc(A, M * lda * 4), rb = rsrc(B, N * ldb * 4);
    const int lrow = lane >> 3, lslot = lane & 7;
    const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) float*)lds;
    auto issue = [&](int st, int k0) {
        const unsigned base = lds0 + st * SF * 4;
#pragma unroll
        for (int i = 0; i < APW; ++i) {
            const int inst = wv * APW + i, row = inst * 8 + lrow;
            const int s = lslot ^ ((row >> 1) & 7), gm = m0 + row, gk = k0 + 4 * s;
            const unsigned off = (gm < M && gk < K) ? (unsigned)(gm * lda + gk) * 4u : OOB;
            dma16(ra, off, base + inst * 1024);
        }
#pragma unroll
        for (int i = 0; i < BPW; ++i) {
            const int inst = wv * BPW + i, row = inst * 8 + lrow;
            const int s = lslot ^ ((row >> 1) & 7), gn = n0 + row, gk = k0 + 4 * s;
            const unsigned off = (gn < N && gk < K) ? (unsigned)(gn * ldb + gk) * 4u : OOB;
            dma16(rb, off, base + BM * BK * 4 + inst * 1024);
        }
    };
    f32x4 acc[AM][AN], tacc[AM][AN];
#pragma unroll
    for (int i = 0; i < AM; ++i)
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][j][r] = 0.f;
    const int nt = (K + BK - 1) / BK;
    const int g = lane >> 4, l15 = lane & 15;
#pragma unroll
    for (int p = 0; p < ST - 1; ++p)
        if (p < nt) issue(p, p * BK);
    if (nt > 1) stage_barrier<(ST - 2) * PER>();
    else stage_barrier<0>();
    for (int t = 0; t < nt; ++t) {
        if (t + ST - 1 < nt) issue((t + ST - 1) % ST, (t + ST - 1) * BK);
        const float* as = lds + (t % ST) * SF;
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
                const int slot = (hh * 4 + g) ^ ((row >> 1) & 7);
                a[i] = *reinterpret_cast<const float4*>(as + row * BK + 4 * slot);
            }
#pragma unroll
            for (int j = 0; j < AN; ++j) {
                const int row = wn * TN + j * 16 + l15;
                const int slot = (hh * 4 + g) ^ ((row >> 1) & 7);
                b[j] = *reinterpret_cast<const float4*>(bs + row * BK + 4 * slot);
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
        if constexpr (ST >= 3) {
            if (t + ST - 1 < nt) stage_barrier<(ST - 2) * PER>();
            else stage_barrier<0>();
        } else {
            stage_barrier<0>();
        }
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

__global__ void k_ref(const float* A, const float* B, float* C, int M, int N, int K) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)M * N) return;
    const int m = (int)(i / N), n = (int)(i % N);
    double s = 0.0;
    for (int k = 0; k < K; ++k) s += (double)A[(long long)m * K + k] * (double)B[(long long)n * K + k];
    C[i] = (float)s;
}

struct Shape {
    const char* name;
    int M, N, K;
};

template <typename F>
static double timeit(F&& f, hipStream_t s, int reps = 50) {
    f();
    CK(hipStreamSynchronize(s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) f();
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1e3 / reps;
}

static double maxerr(const float* d, const float* r, long long n) {
    std::vector<float> a(n), b(n);
    CK(hipMemcpy(a.data(), d, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), r, n * 4, hipMemcpyDeviceToHost));
    double e = 0.0;
    for (long long i = 0; i < n; ++i) e = std::max(e, (double)std::fabs(a[i] - b[i]));
    return e;
}

template <int BM, int BN, int WGM, int WGN, int ST, int PR = 0>
static void run_g4(const char* tag, const Shape& sh, const float* A, const float* B, float* C, const float* R,
                   hipStream_t s) {
    CK(hipMemset(C, 0, (size_t)sh.M * sh.N * 4));
    const dim3 g((sh.M + BM - 1) / BM, (sh.N + BN - 1) / BN);
    auto f = [&]() {
        hipLaunchKernelGGL((k_g4<BM, BN, WGM, WGN, ST, PR>), g, dim3(64 * WGM * WGN), 0, s, A, sh.K, B, sh.K, sh.M, sh.N,
                           sh.K, C, sh.N);
    };
    const double us = timeit(f, s);
    printf("%-9s %-34s blocks=%5d %7.1f us %6.1f TF/s err=%.2e\n", sh.name, tag, g.x * g.y, us,
           2.0 * sh.M * sh.N * sh.K / (us * 1e-6) / 1e12, maxerr(C, R, (long long)sh.M * sh.N));
}

template <int BM, int BN, int WGM, int WGN, int ST>
static void run_g5(const char* tag, const Shape& sh, const float* A, const float* B, float* C, const float* R,
                   hipStream_t s) {
    CK(hipMemset(C, 0, (size_t)sh.M * sh.N * 4));
    const dim3 g((sh.M + BM - 1) / BM, (sh.N + BN - 1) / BN);
    auto f = [&]() {
        hipLaunchKernelGGL((k_g5<BM, BN, WGM, WGN, ST>), g, dim3(64 * WGM * WGN), 0, s, A, sh.K, B, sh.K, sh.M, sh.N,
                           sh.K, C, sh.N);
    };
    const double us = timeit(f, s);
    printf("%-9s %-34s blocks=%5d %7.1f us %6.1f TF/s err=%.2e\n", sh.name, tag, g.x * g.y, us,
           2.0 * sh.M * sh.N * sh.K / (us * 1e-6) / 1e12, maxerr(C, R, (long long)sh.M * sh.N));
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const Shape shapes[] = {
        {"edge_fwd", 23296, 128, 640},
        {"node_fwd", 9728, 128, 640},
        {"edge_dA", 23296, 640, 128},
        {"node_dA", 9728, 640, 128},
        {"node0_fwd", 9728, 128, 272},
    };
    for (const Shape& sh : shapes) {
        const long long na = (long long)sh.M * sh.K, nb = (long long)sh.N * sh.K, nc = (long long)sh.M * sh.N;
        std::vector<float> ha(na), hb(nb);
        srand(1);
        for (auto& v : ha) v = (float)rand() / RAND_MAX - 0.5f;
        for (auto& v : hb) v = (float)rand() / RAND_MAX - 0.5f;
        float *A, *B, *C, *R, *bias;
        int* mv;
        CK(hipMalloc(&A, na * 4));
        CK(hipMalloc(&B, nb * 4));
        CK(hipMalloc(&C, nc * 4));
        CK(hipMalloc(&R, nc * 4));
        CK(hipMalloc(&bias, sh.N * 4));
        CK(hipMalloc(&mv, 4));
        CK(hipMemcpy(mv, &sh.M, 4, hipMemcpyHostToDevice));
        CK(hipMemset(bias, 0, sh.N * 4));
        CK(hipMemcpy(A, ha.data(), na * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(B, hb.data(), nb * 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_ref, dim3((nc + 255) / 256), dim3(256), 0, s, A, B, R, sh.M, sh.N, sh.K);
        CK(hipStreamSynchronize(s));
        {
            CK(hipMemset(C, 0, nc * 4));
            auto f = [&]() {
                if (sh.N <= 128)
                    launch_gemm3_fwd(A, sh.K, mv, sh.M, sh.K, B, sh.K, sh.N, bias, 1 << 30, C, sh.N, nullptr, s);
                else
                    launch_gemm3_da(A, sh.K, mv, sh.M, sh.K, B, sh.K, sh.N, C, sh.N, s);
            };
            const double us = timeit(f, s);
            printf("%-9s %-34s              %7.1f us %6.1f TF/s err=%.2e\n", sh.name, "lib k_gemm3", us,
                   2.0 * sh.M * sh.N * sh.K / (us * 1e-6) / 1e12, maxerr(C, R, nc));
        }
        run_g4<64, 64, 2, 2, 2>("g4<64,64,2x2> 2st", sh, A, B, C, R, s);
        run_g4<64, 64, 2, 2, 2, 1>("g4<64,64,2x2> 2st PROBE mfma+lds", sh, A, B, C, R, s);
        run_g4<64, 64, 2, 2, 2, 2>("g4<64,64,2x2> 2st PROBE staging", sh, A, B, C, R, s);
        if (sh.N > 128) {  // the library's dA kernel on 64 x 64 tiles
            CK(hipMemset(C, 0, nc * 4));
            G3 p{};
            p.a = A; p.lda = sh.K; p.b = B; p.ldb = sh.K; p.m_cap = sh.M; p.m_valid = mv; p.k = sh.K; p.n = sh.N;
            p.c = C; p.ldc = sh.N;
            auto f = [&]() {
                hipLaunchKernelGGL((k_gemm3<64, 64, 32, 2, 2, E3_STORE>), dim3((sh.M + 63) / 64, (sh.N + 63) / 64),
                                   dim3(256), 0, s, p);
            };
            const double us = timeit(f, s);
            printf("%-9s %-34s              %7.1f us %6.1f TF/s err=%.2e\n", sh.name, "lib k_gemm3<64,64> E3_STORE", us,
                   2.0 * sh.M * sh.N * sh.K / (us * 1e-6) / 1e12, maxerr(C, R, nc));
        }
        run_g5<64, 64, 2, 2, 2>("g5 16x16x4 <64,64,2x2> 2st", sh, A, B, C, R, s);
        run_g5<64, 64, 2, 2, 3>("g5 16x16x4 <64,64,2x2> 3st", sh, A, B, C, R, s);
        run_g5<32, 64, 1, 2, 2>("g5 16x16x4 <32,64,1x2> 2st", sh, A, B, C, R, s);
        run_g5<64, 128, 2, 2, 2>("g5 16x16x4 <64,128,2x2> 2st", sh, A, B, C, R, s);
        run_g4<64, 128, 2, 2, 2>("g4<64,128,2x2> 2st", sh, A, B, C, R, s);

        CK(hipFree(A));
        CK(hipFree(B));
        CK(hipFree(C));
        CK(hipFree(R));
        CK(hipFree(bias));
        CK(hipFree(mv));
    }
    return 0;
}
