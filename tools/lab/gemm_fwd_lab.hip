// Forward-GEMM lab (round 5): the production split-bf16 forward GEMM (k_gemm_bf3_fwd, csrc/gemm_bf3.hip) and
// experimental variants, standalone on the step's shapes (M = 9 728 node / 23 296 edge rows, K = 640, N = 128)
// and on large shapes, timed with HIP events over back-to-back launches; TF/s of fp32-equivalent algorithmic
// FLOPs against the split-bf16 peak (2516.8 / 6 = 419.5 TF/s); every variant checked against a fp64 reference.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/lab/gemm_fwd_lab.hip -o tools/lab/gemm_fwd_lab
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../hgnn-2_amd/csrc/gemm_bf3.hip"


#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

using namespace hgnn;

#include "gemm_fwd_exp.h"

__global__ void k_split_b(const float* w, __bf16* b, long long pb, int ldb, int N, int K) {
    const int n = blockIdx.y, k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= ldb) return;
    const float x = k < K ? w[(long long)n * K + k] : 0.f;
    __bf16 a0, a1, a2;
    split3(x, a0, a1, a2);
    b[(long long)n * ldb + k] = a0;
    b[pb + (long long)n * ldb + k] = a1;
    b[2 * pb + (long long)n * ldb + k] = a2;
}

__global__ void k_ref(const float* A, const float* W, float* Y, int M, int N, int K, int lda) {
    const int m = blockIdx.y, n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    double s = 0.0;
    for (int k = 0; k < K; ++k) s += (double)A[(long long)m * lda + k] * W[(long long)n * K + k];
    Y[(long long)m * N + n] = (float)s;
}

struct Shape {
    int M, K, N;
};

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 50;
    std::vector<Shape> shapes = {{9728, 640, 128}, {23296, 640, 128}, {65536, 640, 128}, {262144, 640, 128},
                                 {23296, 1280, 256}, {8192, 4096, 4096}};
    for (const Shape& sh : shapes) {
        const int M = sh.M, K = sh.K, N = sh.N, lda = K, ldb = bf3_ld(K);
        const long long pb = (long long)N * ldb;
        float *A, *W, *Y, *Yr, *part;
        __bf16* B;
        int* mv;
        CK(hipMalloc(&A, (size_t)M * lda * 4));
        CK(hipMalloc(&W, (size_t)N * K * 4));
        CK(hipMalloc(&Y, (size_t)M * N * 4));
        CK(hipMalloc(&Yr, (size_t)M * N * 4));
        CK(hipMalloc(&part, (size_t)ceil_div(M, 64) * N * 3 * 4));
        CK(hipMalloc(&B, (size_t)3 * pb * 2));
        CK(hipMalloc(&mv, 4));
        std::vector<float> h((size_t)M * lda);
        srand(1);
        for (auto& x : h) x = (float)rand() / RAND_MAX * 2.f - 1.f;
        CK(hipMemcpy(A, h.data(), h.size() * 4, hipMemcpyHostToDevice));
        std::vector<float> hw((size_t)N * K);
        for (auto& x : hw) x = ((float)rand() / RAND_MAX * 2.f - 1.f) * 0.1f;
        CK(hipMemcpy(W, hw.data(), hw.size() * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(mv, &M, 4, hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_split_b, dim3(ceil_div(ldb, 256), N), dim3(256), 0, 0, W, B, pb, ldb, N, K);
        const bool check = (long long)M * N * K <= 4ll << 30;
        if (check) hipLaunchKernelGGL(k_ref, dim3(ceil_div(N, 256), M), dim3(256), 0, 0, A, W, Yr, M, N, K, lda);
        std::vector<float> ref((size_t)M * N), got((size_t)M * N);
        if (check) CK(hipMemcpy(ref.data(), Yr, ref.size() * 4, hipMemcpyDeviceToHost));
        auto bench = [&](const char* name, auto&& go) {
            CK(hipMemset(Y, 0, (size_t)M * N * 4));
            go();
            CK(hipDeviceSynchronize());
            double err = 0.0;
            if (check) {
                CK(hipMemcpy(got.data(), Y, got.size() * 4, hipMemcpyDeviceToHost));
                for (size_t i = 0; i < got.size(); ++i) err = fmax(err, fabs((double)got[i] - ref[i]));
            }
            for (int i = 0; i < 3; ++i) go();
            hipEvent_t e0, e1;
            CK(hipEventCreate(&e0));
            CK(hipEventCreate(&e1));
            CK(hipEventRecord(e0, 0));
            for (int i = 0; i < reps; ++i) go();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / reps;
            const double tf = 2.0 * M * N * K / (us * 1e-6) / 1e12;
            const double gbs = ((double)M * lda * 4 + (double)M * N * 4) / (us * 1e-6) / 1e9;
            printf("%-22s M=%6d K=%5d N=%5d  %9.2f us  %7.1f TF  %.3f of 419.5  %6.0f GB/s  max|err| %.2e\n", name, M, K, N,
                   us, tf, tf / 419.5, gbs, err);
            fflush(stdout);
            CK(hipEventDestroy(e0));
            CK(hipEventDestroy(e1));
        };
        float* zb;
        CK(hipMalloc(&zb, (size_t)N * 4));
        CK(hipMemset(zb, 0, (size_t)N * 4));
        bench("prod k_gemm_bf3_fwd", [&] {
            launch_gemm_bf3_fwd(A, lda, mv, M, K, B, pb, ldb, N, zb, N, Y, N, part, 0);
        });
        exp_variants(bench, A, lda, mv, M, K, B, pb, ldb, N, Y, part);
        CK(hipFree(A));
        CK(hipFree(W));
        CK(hipFree(Y));
        CK(hipFree(Yr));
        CK(hipFree(part));
        CK(hipFree(B));
        CK(hipFree(mv));
        CK(hipFree(zb));
    }
    return 0;
}
