// Standalone 1x1 Conv1d on the reference's channel-major (bs, C, N) layout,
// for the layer-level modules (models/layers/layers_mnb.py layer_* classes used
// one at a time).  Transposes to row-major [bs*N][C], runs the same fp32 MFMA
// GEMM as the network executor, transposes back.
#include "kernels.h"

namespace hgnn {
namespace {

// out[(b*n + p) * c + ch] = in[(b*c + ch) * n + p]   (and the inverse)
__global__ void k_to_rows(const float* __restrict__ in, float* __restrict__ out, int bs, int c, int n) {
    const long long tot = (long long)bs * c * n;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot;
         i += (long long)gridDim.x * blockDim.x) {
        const int p = (int)(i % n), ch = (int)((i / n) % c), b = (int)(i / ((long long)c * n));
        out[((long long)b * n + p) * c + ch] = in[i];
    }
}

__global__ void k_from_rows(const float* __restrict__ in, float* __restrict__ out, int bs, int c, int n,
                            int relu) {
    const long long tot = (long long)bs * c * n;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot;
         i += (long long)gridDim.x * blockDim.x) {
        const int p = (int)(i % n), ch = (int)((i / n) % c), b = (int)(i / ((long long)c * n));
        float v = in[((long long)b * n + p) * c + ch];
        if (relu) v = v < 0.f ? 0.f : v;
        out[i] = v;
    }
}

int grid_for(long long n) {
    long long b = (n + 255) / 256;
    return (int)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

struct ConvWs {
    size_t xt, yt, slabs, cnt, bytes;
};

ConvWs conv_ws(int bs, int cin, int cout, int n) {
    ConvWs w;
    const size_t rows = (size_t)bs * n;
    auto up = [](size_t x) { return (x + 255) / 256 * 256; };
    w.xt = 0;
    w.yt = up(rows * cin * 4);
    w.slabs = w.yt + up(rows * (cin > cout ? cin : cout) * 4);
    w.cnt = w.slabs + up(gemm_dw_slab_floats((int)rows, cout, cin) * 4);
    w.bytes = w.cnt + 256;
    return w;
}

}  // namespace
}  // namespace hgnn

using namespace hgnn;

extern "C" {

size_t hgnn_conv1x1_workspace_bytes(int bs, int cin, int cout, int n) {
    if (bs <= 0 || cin <= 0 || cout <= 0 || n <= 0) return 0;
    return conv_ws(bs, cin, cout, n).bytes;
}

int hgnn_conv1x1_forward(const float* d_x, const float* d_w, const float* d_b, float* d_y, int bs, int cin,
                         int cout, int n, int relu, void* workspace, void* stream) {
    if (!d_x || !d_w || !d_b || !d_y || !workspace || bs <= 0 || cin <= 0 || cout <= 0 || n <= 0)
        return HGNN_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    const ConvWs w = conv_ws(bs, cin, cout, n);
    char* ws = (char*)workspace;
    float* xt = (float*)(ws + w.xt);
    float* yt = (float*)(ws + w.yt);
    const long long rows = (long long)bs * n;
    hipLaunchKernelGGL(k_to_rows, dim3(grid_for(rows * cin)), dim3(256), 0, s, d_x, xt, bs, cin, n);
    HGNN_LAUNCH_CHECK();
    GemmFwdArgs g{};
    g.a = xt;
    g.lda = cin;
    g.m_valid = nullptr;
    g.m_cap = (int)rows;
    g.k = cin;
    g.w0 = d_w;
    g.w1 = d_w;
    g.b0 = d_b;
    g.b1 = d_b;
    g.n = cout;
    g.split = cout;
    g.relu_from = cout;
    g.y = yt;
    g.ldy = cout;
    g.bn_part = nullptr;
    int r = launch_gemm_fwd(g, s);
    if (r) return r;
    hipLaunchKernelGGL(k_from_rows, dim3(grid_for(rows * cout)), dim3(256), 0, s, yt, d_y, bs, cout, n, relu);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

// dy is the gradient wrt the conv OUTPUT before any ReLU (the caller applies the ReLU mask).
int hgnn_conv1x1_backward(const float* d_x, const float* d_w, const float* d_dy, float* d_dx, float* d_dw,
                          float* d_db, int bs, int cin, int cout, int n, void* workspace, void* stream) {
    if (!d_x || !d_w || !d_dy || !d_dw || !d_db || !workspace || bs <= 0 || cin <= 0 || cout <= 0 || n <= 0)
        return HGNN_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    const ConvWs w = conv_ws(bs, cin, cout, n);
    char* ws = (char*)workspace;
    float* xt = (float*)(ws + w.xt);
    float* yt = (float*)(ws + w.yt);
    float* slabs = (float*)(ws + w.slabs);
    int* cnt = (int*)(ws + w.cnt);
    const long long rows = (long long)bs * n;
    HGNN_HOST_CHECK(hipMemsetD32Async((hipDeviceptr_t)cnt, (int)rows, 1, s));
    hipLaunchKernelGGL(k_to_rows, dim3(grid_for(rows * cin)), dim3(256), 0, s, d_x, xt, bs, cin, n);
    HGNN_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_to_rows, dim3(grid_for(rows * cout)), dim3(256), 0, s, d_dy, yt, bs, cout, n);
    HGNN_LAUNCH_CHECK();
    GemmDwArgs gw{};
    gw.dy = yt;
    gw.lddy = cout;
    gw.a = xt;
    gw.lda = cin;
    gw.r_valid = cnt;
    gw.r_cap = (int)rows;
    gw.o = cout;
    gw.k = cin;
    gw.split = cout;
    gw.slabs = slabs;
    gw.dw0 = d_dw;
    gw.dw1 = d_dw;
    gw.db0 = d_db;
    gw.db1 = d_db;
    int r = launch_gemm_dw(gw, s);
    if (r) return r;
    if (d_dx) {
        // dxt reuses the xt region (x no longer needed)
        GemmDaArgs gd{};
        gd.dy = yt;
        gd.lddy = cout;
        gd.m_valid = nullptr;
        gd.m_cap = (int)rows;
        gd.o = cout;
        gd.w0 = d_w;
        gd.w1 = d_w;
        gd.split = cout;
        gd.k = cin;
        gd.da = xt;
        gd.ldda = cin;
        r = launch_gemm_da(gd, s);
        if (r) return r;
        hipLaunchKernelGGL(k_from_rows, dim3(grid_for(rows * cin)), dim3(256), 0, s, xt, d_dx, bs, cin, n, 0);
        HGNN_LAUNCH_CHECK();
    }
    return HGNN_OK;
}

}  // extern "C"
