// Device-resident training step pieces: the loss and the
// optimizer of scripts/train_mnb.py:41-91 without host round trips.
//
//  * hgnn_mse_loss: T' = normalize_data(T, mean, std) (functions/utils.py:84-95,
//    mean only when std < 1e-5, Q14), loss = mean((out - T')^2) (nn.MSELoss,
//    scripts/train_mnb.py:76), the seed gradient dout = 2 (out - T') / n, the MAE
//    of utils.evaluation (functions/utils.py:98-102) and the RunningAverage
//    updates of both (functions/utils.py:134-146) -- one block, no host sync
//    (the reference calls .item() twice per batch).
//  * hgnn_adamax_step: torch.optim.Adamax (scripts/main_gnn_qm9.py:185) over every
//    parameter tensor in one launch (multi-tensor apply): per element
//      g += wd p;  m = lerp(m, g, 1 - b1);  u = max(b2 u, |g| + eps);
//      p -= lr / (1 - b1^t) * m / u
//    in torch's operation order (lerp as a + w (b - a) for w < 0.5).
#include "kernels.h"

namespace hgnn {
namespace {

__global__ void __launch_bounds__(256) k_mse_loss(const float* __restrict__ out, const float* __restrict__ t, int n,
                                                  float t_mean, float t_std, float* __restrict__ stats,
                                                  float* __restrict__ dout) {
    __shared__ double red[2][4];
    double se = 0.0, ae = 0.0;
    const bool scale = !(t_std < 1e-5f);
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        float tn = t[i] - t_mean;
        if (scale) tn = tn / t_std;
        const float d = out[i] - tn;
        se += (double)d * d;
        ae += fabs((double)d);
        if (dout) dout[i] = 2.0f * d / (float)n;
    }
    se = wave_sum_d(se);
    ae = wave_sum_d(ae);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        red[0][w] = se;
        red[1][w] = ae;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double S = 0.0, A = 0.0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
            S += red[0][i];
            A += red[1][i];
        }
        const float loss = n > 0 ? (float)(S / n) : 0.f;
        const float mae = n > 0 ? (float)(A / n) : 0.f;
        stats[0] = loss;
        stats[1] = mae;
        // RunningAverage(momentum = 0.1): first value taken as is, then 0.9 new + 0.1 old
        stats[2] = stats[2] == 0.f ? loss : 0.9f * loss + 0.1f * stats[2];
        stats[3] = stats[3] == 0.f ? mae : 0.9f * mae + 0.1f * stats[3];
    }
}

// Classification branch of the reference step (scripts/train_mnb.py:50-51: mean == 0 ->
// T = T.squeeze().long(); the drivers pass nn.CrossEntropyLoss, scripts/main_generate.py:147):
// loss = mean_i (logsumexp(out_i) - out_i[t_i]), dout = (softmax(out_i) - onehot(t_i)) / n,
// the running loss as in k_mse_loss; the MAE meters are not updated (train_mnb.py:81-82).
// One block; a thread per row, classes in a serial loop (C is the model's dim_output).
__global__ void __launch_bounds__(256) k_xent_loss(const float* __restrict__ out, const float* __restrict__ t, int n,
                                                   int c, float* __restrict__ stats, float* __restrict__ dout,
                                                   uint32_t* __restrict__ err) {
    __shared__ double red[4];
    double se = 0.0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float* x = out + (long long)i * c;
        const int ti = (int)t[i];  // LongTensor cast truncates toward zero
        if (ti < 0 || ti >= c || (float)ti != t[i]) {
            // a rejected row contributes nothing: its dout row is zero, never uninitialised memory
            atomicOr(err, 1u);
            if (dout)
                for (int k = 0; k < c; ++k) dout[(long long)i * c + k] = 0.f;
            continue;
        }
        float m = x[0];
        for (int k = 1; k < c; ++k) m = fmaxf(m, x[k]);
        float s = 0.f;
        for (int k = 0; k < c; ++k) s += expf(x[k] - m);
        const float lse = m + logf(s);
        se += (double)(lse - x[ti]);
        if (dout) {
            const float inv = 1.0f / (float)n;
            for (int k = 0; k < c; ++k) dout[(long long)i * c + k] = (expf(x[k] - lse) - (k == ti ? 1.f : 0.f)) * inv;
        }
    }
    se = wave_sum_d(se);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = se;
    __syncthreads();
    if (threadIdx.x == 0) {
        double S = 0.0;
        for (int i = 0; i < (int)(blockDim.x >> 6); ++i) S += red[i];
        const float loss = n > 0 ? (float)(S / n) : 0.f;
        stats[0] = loss;
        stats[2] = stats[2] == 0.f ? loss : 0.9f * loss + 0.1f * stats[2];
    }
}

constexpr int ADAMAX_MAX = 64;

struct AdamaxTable {
    float* p[ADAMAX_MAX];
    const float* g[ADAMAX_MAX];
    float* m[ADAMAX_MAX];
    float* u[ADAMAX_MAX];
    int n[ADAMAX_MAX];
    int start[ADAMAX_MAX + 1];  // prefix of per-tensor block counts
    int count;
};

__global__ void __launch_bounds__(256) k_adamax(AdamaxTable tab, float lr_c, float w, float beta2, float eps,
                                                float wd) {
    // block -> tensor by the block prefix (uniform scan over <= 64 entries)
    int t = 0;
    while (t + 1 < tab.count && (int)blockIdx.x >= tab.start[t + 1]) ++t;
    const int i = ((int)blockIdx.x - tab.start[t]) * 256 + threadIdx.x;
    if (i >= tab.n[t]) return;
    float g = tab.g[t][i];
    const float p = tab.p[t][i];
    if (wd != 0.f) g = g + wd * p;
    const float m0 = tab.m[t][i];
    const float m = m0 + w * (g - m0);  // torch lerp, weight < 0.5
    const float u = fmaxf(tab.u[t][i] * beta2, fabsf(g) + eps);
    tab.m[t][i] = m;
    tab.u[t][i] = u;
    tab.p[t][i] = p + (-lr_c) * (m / u);  // addcdiv_(m, u, value = -clr)
}

}  // namespace
}  // namespace hgnn

using namespace hgnn;

extern "C" {

int hgnn_mse_loss(const float* d_out, const float* d_t, int n, float t_mean, float t_std, float* d_stats,
                  float* d_dout, void* stream) {
    if (!d_out || !d_t || !d_stats || n < 0) return HGNN_ERR_ARG;
    HGNN_KLAUNCH(k_mse_loss, dim3(1), dim3(256), 0, static_cast<hipStream_t>(stream), d_out, d_t, n, t_mean,
                       t_std, d_stats, d_dout);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int hgnn_xent_loss(const float* d_out, const float* d_t, int n, int c, float* d_stats, float* d_dout,
                   uint32_t* d_err, void* stream) {
    if (!d_out || !d_t || !d_stats || !d_err || n < 0 || c < 1) return HGNN_ERR_ARG;
    HGNN_KLAUNCH(k_xent_loss, dim3(1), dim3(256), 0, static_cast<hipStream_t>(stream), d_out, d_t, n, c,
                       d_stats, d_dout, d_err);
    HGNN_LAUNCH_CHECK();
    return HGNN_OK;
}

int hgnn_adamax_step(int n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                     float* const* exp_inf, const int64_t* numel, double lr, double beta1, double beta2,
                     double eps, double weight_decay, long long step, void* stream) {
    if (n_tensors < 0 || (n_tensors > 0 && (!params || !grads || !exp_avg || !exp_inf || !numel)) || step < 1)
        return HGNN_ERR_ARG;
    // hyper-parameters combine in double (Python floats) and reach the kernel as fp32
    // scalars, as torch's scalar arguments do: clr = lr / (1 - beta1^step), w = 1 - beta1
    const double bc = 1.0 - pow(beta1, (double)step);
    const float lr_c = (float)(lr / bc);
    const float w = (float)(1.0 - beta1);
    hipStream_t s = static_cast<hipStream_t>(stream);
    for (int base = 0; base < n_tensors; base += ADAMAX_MAX) {
        AdamaxTable tab{};
        tab.count = 0;
        int blocks = 0;
        for (int k = base; k < n_tensors && tab.count < ADAMAX_MAX; ++k) {
            if (numel[k] < 0 || numel[k] > (1ll << 30)) return HGNN_ERR_ARG;
            const int c = tab.count++;
            tab.p[c] = params[k];
            tab.g[c] = grads[k];
            tab.m[c] = exp_avg[k];
            tab.u[c] = exp_inf[k];
            tab.n[c] = (int)numel[k];
            tab.start[c] = blocks;
            blocks += (int)ceil_div<long long>(numel[k], 256);
        }
        tab.start[tab.count] = blocks;
        if (blocks == 0) continue;
        HGNN_KLAUNCH(k_adamax, dim3(blocks), dim3(256), 0, s, tab, lr_c, w, (float)beta2, (float)eps,
                           (float)weight_decay);
        HGNN_LAUNCH_CHECK();
    }
    return HGNN_OK;
}

}  // extern "C"
