// Layer-level drop-ins on the reference's dense padded tensors:
//   graph_oper / graph_op  (models/layers/layers_mnb.py:391-411, functions/utils.py:24-52)
//   P_multi / Pmul         (models/layers/layers_mnb.py:414-434, functions/utils.py:55-81)
//   BN                     (models/layers/batch_normalization.py:23-108)
// These serve callers that use the ops one at a time on dense inputs (the
// reference's layer-level API).  The network path (net.hip) never calls them:
// it walks the extracted sparse lists instead.  One workgroup per graph, the
// graph's operator slice and features staged in LDS when they fit.
#include "../../include/hgnn_amd.h"
#include "kernels.h"

namespace hgnn {
namespace {

// out[b, j*F + f, n] = sum_m A[b, n, m, j] X[b, f, m]
__global__ void __launch_bounds__(256) k_gop_fwd(const float* __restrict__ A, const float* __restrict__ X,
                                                 float* __restrict__ out, int N, int J, int F) {
    const int b = blockIdx.x, j = blockIdx.y;
    const float* Ab = A + (long long)b * N * N * J;
    const float* Xb = X + (long long)b * F * N;
    float* ob = out + (long long)b * J * F * N + (long long)j * F * N;
    for (int i = threadIdx.x; i < F * N; i += blockDim.x) {
        const int f = i / N, n = i % N;
        float s = 0.f;
        for (int m = 0; m < N; ++m) s = fmaf(Ab[((long long)n * N + m) * J + j], Xb[(long long)f * N + m], s);
        ob[i] = s;
    }
}

// dX[b, f, m] = sum_j sum_n A[b, n, m, j] dO[b, jF + f, n]
__global__ void __launch_bounds__(256) k_gop_bwd_x(const float* __restrict__ A, const float* __restrict__ dO,
                                                   float* __restrict__ dX, int N, int J, int F) {
    const int b = blockIdx.x;
    const float* Ab = A + (long long)b * N * N * J;
    const float* db = dO + (long long)b * J * F * N;
    for (int i = threadIdx.x; i < F * N; i += blockDim.x) {
        const int f = i / N, m = i % N;
        float s = 0.f;
        for (int j = 0; j < J; ++j)
            for (int n = 0; n < N; ++n)
                s = fmaf(Ab[((long long)n * N + m) * J + j], db[((long long)j * F + f) * N + n], s);
        dX[(long long)b * F * N + i] = s;
    }
}

// dA[b, n, m, j] = sum_f dO[b, jF + f, n] X[b, f, m]
__global__ void __launch_bounds__(256) k_gop_bwd_a(const float* __restrict__ X, const float* __restrict__ dO,
                                                   float* __restrict__ dA, int N, int J, int F) {
    const int b = blockIdx.x;
    const float* Xb = X + (long long)b * F * N;
    const float* db = dO + (long long)b * J * F * N;
    for (int i = threadIdx.x; i < N * N * J; i += blockDim.x) {
        const int j = i % J, m = (i / J) % N, n = i / (J * N);
        float s = 0.f;
        for (int f = 0; f < F; ++f) s = fmaf(db[((long long)j * F + f) * N + n], Xb[(long long)f * N + m], s);
        dA[(long long)b * N * N * J + i] = s;
    }
}

// out[b, f, n] = sum_m P[b, n, m] X[b, f, m], P with explicit strides
__global__ void __launch_bounds__(256) k_pm_fwd(const float* __restrict__ P, long sb, long sn, long sm,
                                                const float* __restrict__ X, float* __restrict__ out, int N,
                                                int M, int F) {
    const int b = blockIdx.x;
    const float* Pb = P + b * sb;
    const float* Xb = X + (long long)b * F * M;
    for (int i = threadIdx.x; i < F * N; i += blockDim.x) {
        const int f = i / N, n = i % N;
        float s = 0.f;
        for (int m = 0; m < M; ++m) s = fmaf(Pb[n * sn + m * sm], Xb[(long long)f * M + m], s);
        out[(long long)b * F * N + i] = s;
    }
}

// dX[b, f, m] = sum_n P[b, n, m] dO[b, f, n];  dP[b, n, m] = sum_f dO[b, f, n] X[b, f, m] (dense (bs, N, M))
__global__ void __launch_bounds__(256) k_pm_bwd(const float* __restrict__ P, long sb, long sn, long sm,
                                                const float* __restrict__ X, const float* __restrict__ dO,
                                                float* __restrict__ dX, float* __restrict__ dP, int N, int M,
                                                int F) {
    const int b = blockIdx.x;
    const float* Pb = P + b * sb;
    const float* Xb = X + (long long)b * F * M;
    const float* db = dO + (long long)b * F * N;
    for (int i = threadIdx.x; i < F * M; i += blockDim.x) {
        const int f = i / M, m = i % M;
        float s = 0.f;
        for (int n = 0; n < N; ++n) s = fmaf(Pb[n * sn + m * sm], db[(long long)f * N + n], s);
        dX[(long long)b * F * M + i] = s;
    }
    if (dP) {
        for (int i = threadIdx.x; i < N * M; i += blockDim.x) {
            const int n = i / M, m = i % M;
            float s = 0.f;
            for (int f = 0; f < F; ++f) s = fmaf(db[(long long)f * N + n], Xb[(long long)f * M + m], s);
            dP[(long long)b * N * M + i] = s;
        }
    }
}

__device__ __forceinline__ double bsum(double v, double* red) {
    v = wave_sum_d(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
    return t;
}

// BN statistics, one block per channel.  H = mask[b, n, 0] * X.
__global__ void __launch_bounds__(256) k_bnd_stats(const float* __restrict__ X, const int64_t* __restrict__ nb,
                                                   const float* __restrict__ mask, float* mean, float* stdv,
                                                   int bs, int C, int N) {
    __shared__ double red[4];
    const int c = blockIdx.x;
    double cnt = 0.0;
    for (int b = threadIdx.x; b < bs; b += blockDim.x) cnt += (double)nb[b];
    const double n = bsum(cnt, red);
    double s = 0.0;
    for (long long i = threadIdx.x; i < (long long)bs * N; i += blockDim.x) {
        const int b = (int)(i / N), p = (int)(i % N);
        s += (double)(mask[((long long)b * N + p) * N] * X[((long long)b * C + c) * N + p]);
    }
    const double mu = bsum(s, red) / n;
    double q = 0.0;
    for (long long i = threadIdx.x; i < (long long)bs * N; i += blockDim.x) {
        const int b = (int)(i / N), p = (int)(i % N);
        const double mk = mask[((long long)b * N + p) * N];
        const double h = mk * X[((long long)b * C + c) * N + p];
        q += mk * (h - mu) * (h - mu);
    }
    const double var = 1e-5 + bsum(q, red) / n;
    if (threadIdx.x == 0) {
        mean[c] = (float)mu;
        stdv[c] = (float)sqrt(var);
    }
}

__global__ void __launch_bounds__(256) k_bnd_apply(const float* __restrict__ X, const float* __restrict__ mask,
                                                   const float* mean, const float* stdv, const float* w,
                                                   const float* bb, float* out, int bs, int C, int N) {
    const long long tot = (long long)bs * C * N;
    const float wv = *w, bv = *bb;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot;
         i += (long long)gridDim.x * blockDim.x) {
        const int p = (int)(i % N), c = (int)((i / N) % C), b = (int)(i / ((long long)C * N));
        const float h = mask[((long long)b * N + p) * N] * X[i];
        out[i] = __fadd_rn(__fmul_rn(wv, __fdiv_rn(__fsub_rn(h, mean[c]), stdv[c])), bv);
    }
}

// Per channel sums over ALL positions: S1 = sum dO, S2 = sum dO * Hhat (padded positions included:
// their output w * (-mean/std) + b still depends on the statistics).
__global__ void __launch_bounds__(256) k_bnd_bwd_stats(const float* __restrict__ X, const float* __restrict__ mask,
                                                       const float* mean, const float* stdv,
                                                       const float* __restrict__ dO, float* sums, int bs, int C,
                                                       int N) {
    __shared__ double red[4];
    const int c = blockIdx.x;
    double s1 = 0.0, s2 = 0.0;
    for (long long i = threadIdx.x; i < (long long)bs * N; i += blockDim.x) {
        const int b = (int)(i / N), p = (int)(i % N);
        const long long idx = ((long long)b * C + c) * N + p;
        const double h = ((double)(mask[((long long)b * N + p) * N] * X[idx]) - mean[c]) / stdv[c];
        s1 += dO[idx];
        s2 += (double)dO[idx] * h;
    }
    const double S1 = bsum(s1, red);
    const double S2 = bsum(s2, red);
    if (threadIdx.x == 0) {
        sums[2 * c] = (float)S1;
        sums[2 * c + 1] = (float)S2;
    }
}

__global__ void __launch_bounds__(256) k_bnd_bwd_apply(const float* __restrict__ X, const int64_t* __restrict__ nb,
                                                       const float* __restrict__ mask, const float* mean,
                                                       const float* stdv, const float* w,
                                                       const float* __restrict__ dO, const float* sums,
                                                       float* __restrict__ dX, float* dw, float* db, int bs,
                                                       int C, int N, int training) {
    __shared__ double red[4];
    const float wv = *w;
    double cnt = 0.0;
    for (int b = threadIdx.x; b < bs; b += blockDim.x) cnt += (double)nb[b];
    const double n = bsum(cnt, red);
    if (blockIdx.x == 0) {
        double a = 0.0, d = 0.0;
        for (int c = threadIdx.x; c < C; c += blockDim.x) {
            a += sums[2 * c + 1];
            d += sums[2 * c];
        }
        const double A = bsum(a, red), D = bsum(d, red);
        if (threadIdx.x == 0) {
            *dw = (float)A;
            *db = (float)D;
        }
    }
    const long long tot = (long long)bs * C * N;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < tot;
         i += (long long)gridDim.x * blockDim.x) {
        const int p = (int)(i % N), c = (int)((i / N) % C), b = (int)(i / ((long long)C * N));
        const float mk = mask[((long long)b * N + p) * N];
        float g;
        if (training) {
            const float h = (mk * X[i] - mean[c]) / stdv[c];
            g = wv / stdv[c] * (dO[i] - (float)(sums[2 * c] / n) - h * (float)(sums[2 * c + 1] / n));
        } else {
            g = wv * dO[i] / stdv[c];
        }
        dX[i] = mk * g;
    }
}

int blocks_for(long long n) {
    long long b = (n + 255) / 256;
    if (b > 4096) b = 4096;
    if (b < 1) b = 1;
    return (int)b;
}

}  // namespace
}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_graph_oper_forward(const float* d_A, const float* d_X, float* d_out, int bs, int n, int j, int f,
                            void* stream) {
    if (!d_A || !d_X || !d_out || bs < 0 || n < 0 || j <= 0 || f < 0) return HGNN_ERR_ARG;
    if (bs == 0 || n == 0 || f == 0) return HGNN_OK;
    HGNN_KLAUNCH(k_gop_fwd, dim3(bs, j), dim3(256), 0, (hipStream_t)stream, d_A, d_X, d_out, n, j, f);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int hgnn_graph_oper_backward(const float* d_A, const float* d_X, const float* d_dout, float* d_dX, float* d_dA,
                             int bs, int n, int j, int f, void* stream) {
    if (!d_A || !d_X || !d_dout || bs < 0 || n < 0 || j <= 0 || f < 0) return HGNN_ERR_ARG;
    if (bs == 0 || n == 0) return HGNN_OK;
    if (d_dX && f > 0) {
        HGNN_KLAUNCH(k_gop_bwd_x, dim3(bs), dim3(256), 0, (hipStream_t)stream, d_A, d_dout, d_dX, n, j, f);
        HGNN_LAUNCH_CHECK();
    }
    if (d_dA) {
        HGNN_KLAUNCH(k_gop_bwd_a, dim3(bs), dim3(256), 0, (hipStream_t)stream, d_X, d_dout, d_dA, n, j, f);
        HGNN_LAUNCH_CHECK();
    }
    return HGNN_OK;
}

int hgnn_p_multi_forward(const float* d_P, long sb, long sn, long sm, const float* d_X, float* d_out, int bs,
                         int n, int m, int f, void* stream) {
    if (!d_P || !d_X || !d_out || bs < 0 || n < 0 || m < 0 || f < 0) return HGNN_ERR_ARG;
    if (bs == 0 || n == 0 || f == 0) return HGNN_OK;
    HGNN_KLAUNCH(k_pm_fwd, dim3(bs), dim3(256), 0, (hipStream_t)stream, d_P, sb, sn, sm, d_X, d_out, n, m, f);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int hgnn_p_multi_backward(const float* d_P, long sb, long sn, long sm, const float* d_X, const float* d_dout,
                          float* d_dX, float* d_dP, int bs, int n, int m, int f, void* stream) {
    if (!d_P || !d_X || !d_dout || !d_dX || bs < 0 || n < 0 || m < 0 || f < 0) return HGNN_ERR_ARG;
    if (bs == 0 || m == 0) return HGNN_OK;
    HGNN_KLAUNCH(k_pm_bwd, dim3(bs), dim3(256), 0, (hipStream_t)stream, d_P, sb, sn, sm, d_X, d_dout, d_dX,
                       d_dP, n, m, f);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int hgnn_bn_forward(const float* d_X, const int64_t* d_nb, const float* d_mask, const float* d_w, const float* d_b,
                    float* d_mean, float* d_std, float* d_out, int bs, int c, int n, int training, void* stream) {
    if (!d_X || !d_nb || !d_mask || !d_w || !d_b || !d_mean || !d_std || !d_out || bs <= 0 || c <= 0 || n <= 0)
        return HGNN_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    if (training) {
        HGNN_KLAUNCH(k_bnd_stats, dim3(c), dim3(256), 0, s, d_X, d_nb, d_mask, d_mean, d_std, bs, c, n);
        HGNN_LAUNCH_CHECK();
    }
    HGNN_KLAUNCH(k_bnd_apply, dim3(blocks_for((long long)bs * c * n)), dim3(256), 0, s, d_X, d_mask, d_mean,
                       d_std, d_w, d_b, d_out, bs, c, n);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int hgnn_bn_backward(const float* d_X, const int64_t* d_nb, const float* d_mask, const float* d_w,
                     const float* d_mean, const float* d_std, const float* d_dout, float* d_dX, float* d_dw,
                     float* d_db, float* d_scratch, int bs, int c, int n, int training, void* stream) {
    if (!d_X || !d_nb || !d_mask || !d_w || !d_mean || !d_std || !d_dout || !d_dX || !d_dw || !d_db || !d_scratch)
        return HGNN_ERR_ARG;
    if (bs <= 0 || c <= 0 || n <= 0) return HGNN_ERR_ARG;
    hipStream_t s = (hipStream_t)stream;
    float* sums = d_scratch;
    HGNN_KLAUNCH(k_bnd_bwd_stats, dim3(c), dim3(256), 0, s, d_X, d_mask, d_mean, d_std, d_dout, sums, bs, c, n);
    HGNN_LAUNCH_CHECK();
    HGNN_KLAUNCH(k_bnd_bwd_apply, dim3(blocks_for((long long)bs * c * n)), dim3(256), 0, s, d_X, d_nb, d_mask,
                       d_mean, d_std, d_w, d_dout, sums, d_dX, d_dw, d_db, bs, c, n, training);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

}  // extern "C"
