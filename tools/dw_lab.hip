// dW GEMM lab: k_gemm3_tn tile / wave shapes and split-K chunk counts on the config-2 dW shapes
// (slabs[z][128][640] = sum over the chunk's rows of dY[r][128] x A[r][640]), standalone, timed with
// HIP events over many launches; checked against a naive reference on one shape.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/dw_lab.hip -o tools/dw_lab_bin
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../hgnn-2_amd/csrc/gemm3.hip"

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

using namespace hgnn;

__global__ void k_ref(const float* dy, const float* a, float* out, int R, int M, int N) {
    const int m = blockIdx.y, n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    double s = 0.0;
    for (int r = 0; r < R; ++r) s += (double)dy[(long long)r * M + m] * a[(long long)r * N + n];
    out[(long long)m * N + n] = (float)s;
}

__global__ void k_sum(const float* slabs, float* out, int Z, int MN) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= MN) return;
    float s = 0.f;
    for (int z = 0; z < Z; ++z) s += slabs[(long long)z * MN + i];
    out[i] = s;
}

template <int BM, int BN, int BK, int WGM, int WGN>
float run(const char* name, const float* dy, const float* a, float* slabs, const int* rv, int R, int M, int N, int nz,
          int reps, float* check) {
    const dim3 grid(ceil_div(M, BM), ceil_div(N, BN), nz);
    auto go = [&] {
        hipLaunchKernelGGL((k_gemm3_tn<BM, BN, BK, WGM, WGN>), grid, dim3(64 * WGM * WGN), 0, 0, dy, M, a, N, slabs, M,
                           N, rv, nz, 1);
    };
    for (int i = 0; i < 5; ++i) go();
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) go();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const float us = ms * 1e3f / reps;
    const double tf = 2.0 * R * M * N / (us * 1e-6) / 1e12;
    printf("%-28s R=%6d nz=%4d blocks=%5d  %7.2f us  %6.1f TF  %.3f of 157.3\n", name, R, nz,
           grid.x * grid.y * grid.z, us, tf, tf / 157.3);
    if (check) {
        float* out;
        CK(hipMalloc(&out, sizeof(float) * M * N));
        hipLaunchKernelGGL(k_sum, dim3(ceil_div(M * N, 256)), dim3(256), 0, 0, slabs, out, nz, M * N);
        std::vector<float> h(M * N), r(M * N);
        CK(hipMemcpy(h.data(), out, sizeof(float) * M * N, hipMemcpyDeviceToHost));
        CK(hipMemcpy(r.data(), check, sizeof(float) * M * N, hipMemcpyDeviceToHost));
        double err = 0.0, mx = 0.0;
        for (int i = 0; i < M * N; ++i) {
            err = std::max(err, (double)std::fabs(h[i] - r[i]));
            mx = std::max(mx, (double)std::fabs(r[i]));
        }
        printf("    max |err| %.3g (max |ref| %.3g)\n", err, mx);
        CK(hipFree(out));
    }
    return us;
}

int main() {
    const int M = 128, N = 640;
    const int rows[2] = {23296, 9728};
    const int Rmax = 23296;
    std::vector<float> hdy((size_t)Rmax * M), ha((size_t)Rmax * N);
    srand(1);
    for (auto& v : hdy) v = (float)rand() / RAND_MAX - 0.5f;
    for (auto& v : ha) v = (float)rand() / RAND_MAX - 0.5f;
    float *dy, *a, *slabs, *ref;
    int* rv;
    CK(hipMalloc(&dy, sizeof(float) * hdy.size()));
    CK(hipMalloc(&a, sizeof(float) * ha.size()));
    CK(hipMalloc(&slabs, sizeof(float) * 1024 * M * N));
    CK(hipMalloc(&ref, sizeof(float) * M * N));
    CK(hipMalloc(&rv, sizeof(int)));
    CK(hipMemcpy(dy, hdy.data(), sizeof(float) * hdy.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(a, ha.data(), sizeof(float) * ha.size(), hipMemcpyHostToDevice));
    for (int R : rows) {
        CK(hipMemcpy(rv, &R, sizeof(int), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(k_ref, dim3(ceil_div(N, 256), M), dim3(256), 0, 0, dy, a, ref, R, M, N);
        CK(hipDeviceSynchronize());
        const int reps = 200;
        for (int nz : {32, 48, 64, 96, 128}) {
            run<128, 128, 32, 4, 2>("tn<128,128,32,4,2> (cur)", dy, a, slabs, rv, R, M, N, nz, reps,
                                    nz == 48 ? ref : nullptr);
            run<128, 128, 32, 2, 2>("tn<128,128,32,2,2> 64x64w", dy, a, slabs, rv, R, M, N, nz, reps,
                                    nz == 48 ? ref : nullptr);
            run<128, 64, 32, 2, 2>("tn<128,64,32,2,2> 64x32w", dy, a, slabs, rv, R, M, N, nz, reps, nullptr);
            run<128, 128, 32, 2, 4>("tn<128,128,32,2,4> 64x32w", dy, a, slabs, rv, R, M, N, nz, reps, nullptr);
        }
    }
    return 0;
}
