// Standalone 1x1 Conv1d on the reference's channel-major (bs, C, N) layout,
// for the layer-level modules (models/layers/layers_mnb.py layer_* classes used
// one at a time).  Transposes to row-major [bs*N][C] (rows padded to a multiple of 4
// floats), runs the network executor's fp32 MFMA GEMMs (gemm3.hip: forward, dA, dW),
// transposes back.
#include "kernels.h"

namespace hgnn {
namespace {

// out[(b*n + p) * ld + ch] = in[(b*c + ch) * n + p]; columns [c, ld) of every row zeroed
__global__ void k_to_rows(const float* __restrict__ in, float* __restrict__ out, int bs, int c, int n, int ld) {
    const long long tot = (long long)bs * ld * n;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot;
         i += (long long)gridDim.x * blockDim.x) {
        const int p = (int)(i % n), ch = (int)((i / n) % ld), b = (int)(i / ((long long)ld * n));
        out[((long long)b * n + p) * ld + ch] = ch < c ? in[((long long)b * c + ch) * n + p] : 0.f;
    }
}

__global__ void k_from_rows(const float* __restrict__ in, float* __restrict__ out, int bs, int c, int n, int ld,
                            int relu) {
    const long long tot = (long long)bs * c * n;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot;
         i += (long long)gridDim.x * blockDim.x) {
        const int p = (int)(i % n), ch = (int)((i / n) % c), b = (int)(i / ((long long)c * n));
        float v = in[((long long)b * n + p) * ld + ch];
        if (relu) v = v < 0.f ? 0.f : v;
        out[i] = v;
    }
}

// wc[o][k] = w[o][k] (k < cin, zero to ldk);  wt[k][o] = w[o][k] (o < cout, zero to ldo)
__global__ void k_pad_weights(const float* __restrict__ w, int cout, int cin, float* __restrict__ wc, int ldk,
                              float* __restrict__ wt, int ldo) {
    const int nc = cout * ldk, nt = cin * ldo;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nc + nt; i += gridDim.x * blockDim.x) {
        if (i < nc) {
            const int o = i / ldk, k = i % ldk;
            wc[i] = k < cin ? w[(long long)o * cin + k] : 0.f;
        } else {
            const int j = i - nc, k = j / ldo, o = j % ldo;
            wt[j] = o < cout ? w[(long long)o * cin + k] : 0.f;
        }
    }
}

// db[o] = sum_b sum_p dy[b, o, p]  (one block per channel, fixed order)
__global__ void __launch_bounds__(256) k_bias_grad(const float* __restrict__ dy, int bs, int cout, int n,
                                                   float* __restrict__ db) {
    __shared__ double red[4];
    const int o = blockIdx.x;
    double acc = 0.0;
    const long long tot = (long long)bs * n;
    for (long long i = threadIdx.x; i < tot; i += 256) {
        const long long b = i / n, p = i % n;
        acc += (double)dy[(b * cout + o) * n + p];
    }
    acc = wave_sum_d(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) db[o] = (float)(red[0] + red[1] + red[2] + red[3]);
}

int grid_for(long long n) {
    long long b = (n + 255) / 256;
    return (int)(b > 4096 ? 4096 : (b < 1 ? 1 : b));
}

int pad4(int x) { return (x + 3) / 4 * 4; }

struct ConvWs {
    size_t xt, yt, wc, wt, slabs, cnt, bytes;
};

ConvWs conv_ws(int bs, int cin, int cout, int n) {
    ConvWs w;
    const size_t rows = (size_t)bs * n;
    const int cinp = pad4(cin), coutp = pad4(cout);
    auto up = [](size_t x) { return (x + 255) / 256 * 256; };
    w.xt = 0;
    w.yt = up(rows * cinp * 4);
    w.wc = w.yt + up(rows * (cinp > coutp ? cinp : coutp) * 4);
    w.wt = w.wc + up((size_t)cout * cinp * 4);
    w.slabs = w.wt + up((size_t)cin * coutp * 4);
    w.cnt = w.slabs + up(dw3_slab_floats((int)rows, cout, cin) * 4);
    w.bytes = w.cnt + 256;
    return w;
}

bool conv_fits(int bs, int cin, int cout, int n) {
    const long long rows = (long long)bs * n, lim = (1ll << 31) - 1;
    const long long w = pad4(cin) > pad4(cout) ? pad4(cin) : pad4(cout);
    return rows * w * 4 <= lim && (long long)cout * pad4(cin) * 4 <= lim && (long long)cin * pad4(cout) * 4 <= lim;
}

}  // namespace
}  // namespace hgnn

using namespace hgnn;

extern "C" {

size_t hgnn_conv1x1_workspace_bytes(int bs, int cin, int cout, int n) {
    if (bs <= 0 || cin <= 0 || cout <= 0 || n <= 0 || !conv_fits(bs, cin, cout, n)) return 0;
    return conv_ws(bs, cin, cout, n).bytes;
}

int hgnn_conv1x1_forward(const float* d_x, const float* d_w, const float* d_b, float* d_y, int bs, int cin,
                         int cout, int n, int relu, void* workspace, void* stream) {
    if (!d_x || !d_w || !d_b || !d_y || !workspace || bs <= 0 || cin <= 0 || cout <= 0 || n <= 0)
        return HGNN_ERR_ARG;
    if (!conv_fits(bs, cin, cout, n)) return HGNN_ERR_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    const ConvWs w = conv_ws(bs, cin, cout, n);
    char* ws = (char*)workspace;
    float* xt = (float*)(ws + w.xt);
    float* yt = (float*)(ws + w.yt);
    float* wc = (float*)(ws + w.wc);
    float* wt = (float*)(ws + w.wt);
    const int cinp = pad4(cin), coutp = pad4(cout);
    const long long rows = (long long)bs * n;
    HGNN_KLAUNCH(k_to_rows, dim3(grid_for(rows * cinp)), dim3(256), 0, s, d_x, xt, bs, cin, n, cinp);
    HGNN_LAUNCH_CHECK();
    HGNN_KLAUNCH(k_pad_weights, dim3(grid_for((long long)cout * cinp + (long long)cin * coutp)), dim3(256), 0, s,
                       d_w, cout, cin, wc, cinp, wt, coutp);
    HGNN_LAUNCH_CHECK();
    // the executor's fp32 MFMA GEMM (gemm3.hip, NT): Y = Xrows . Wc^T + b, ReLU applied on the way back
    int r = launch_gemm3_fwd(xt, cinp, nullptr, (int)rows, cinp, wc, cinp, cout, d_b, cout, yt, cout, nullptr, s);
    if (r) return r;
    HGNN_KLAUNCH(k_from_rows, dim3(grid_for(rows * cout)), dim3(256), 0, s, yt, d_y, bs, cout, n, cout, relu);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

// dy is the gradient wrt the conv OUTPUT before any ReLU (the caller applies the ReLU mask).
int hgnn_conv1x1_backward(const float* d_x, const float* d_w, const float* d_dy, float* d_dx, float* d_dw,
                          float* d_db, int bs, int cin, int cout, int n, void* workspace, void* stream) {
    if (!d_x || !d_w || !d_dy || !d_dw || !d_db || !workspace || bs <= 0 || cin <= 0 || cout <= 0 || n <= 0)
        return HGNN_ERR_ARG;
    if (!conv_fits(bs, cin, cout, n)) return HGNN_ERR_UNSUPPORTED;
    hipStream_t s = (hipStream_t)stream;
    const ConvWs w = conv_ws(bs, cin, cout, n);
    char* ws = (char*)workspace;
    float* xt = (float*)(ws + w.xt);
    float* yt = (float*)(ws + w.yt);
    float* wc = (float*)(ws + w.wc);
    float* wt = (float*)(ws + w.wt);
    float* slabs = (float*)(ws + w.slabs);
    int* cnt = (int*)(ws + w.cnt);
    const int cinp = pad4(cin), coutp = pad4(cout);
    const long long rows = (long long)bs * n;
    HGNN_HOST_CHECK(hipMemsetD32Async((hipDeviceptr_t)cnt, (int)rows, 1, s));
    HGNN_KLAUNCH(k_to_rows, dim3(grid_for(rows * cinp)), dim3(256), 0, s, d_x, xt, bs, cin, n, cinp);
    HGNN_LAUNCH_CHECK();
    HGNN_KLAUNCH(k_to_rows, dim3(grid_for(rows * coutp)), dim3(256), 0, s, d_dy, yt, bs, cout, n, coutp);
    HGNN_LAUNCH_CHECK();
    HGNN_KLAUNCH(k_pad_weights, dim3(grid_for((long long)cout * cinp + (long long)cin * coutp)), dim3(256), 0, s,
                       d_w, cout, cin, wc, cinp, wt, coutp);
    HGNN_LAUNCH_CHECK();
    // dW = dYrows^T . Xrows (TN, row-chunk slabs) -> reduce; db = column sums of dY
    const int nz = dw3_chunks((int)rows, cout, cin);
    int r = launch_gemm3_dw(yt, coutp, xt, cinp, cnt, (int)rows, cout, cin, nz, slabs, s);
    if (r) return r;
    r = launch_dw_reduce2(slabs, cnt, nz, cout, cout, cin, cout, d_dw, d_dw, nullptr, nullptr, nullptr, s);
    if (r) return r;
    HGNN_KLAUNCH(k_bias_grad, dim3(cout), dim3(256), 0, s, d_dy, bs, cout, n, d_db);
    HGNN_LAUNCH_CHECK();
    if (d_dx) {
        // dX = dYrows . Wt^T (NT); written over xt (x no longer needed)
        r = launch_gemm3_da(yt, coutp, nullptr, (int)rows, coutp, wt, coutp, cin, xt, cinp, s);
        if (r) return r;
        HGNN_KLAUNCH(k_from_rows, dim3(grid_for(rows * cin)), dim3(256), 0, s, xt, d_dx, bs, cin, n, cinp, 0);
        HGNN_LAUNCH_CHECK();
    }
    return HGNN_OK;
}

}  // extern "C"
