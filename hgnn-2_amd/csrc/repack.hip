// Weight repack of the Conv1d pairs and the dW slab reduction of the fp32 MFMA GEMMs
// (gemm3.hip).  Each half-layer's two 1x1 convolutions (linear branch cv2/cv4, ReLU
// branch cv1/cv3; models/layers/layers_mnb.py:239-244, 272-288) run as one GEMM over
// Wcat = [W_lin; W_relu] (2d rows):
//  * forward B operand: Wcat zero-padded to kp columns, [2d][kp] (k-contiguous, NT GEMM);
//  * dA B operand: Wcat^T, [K][2d];
//  * bias cat(b_lin, b_relu).
// The dW GEMM (k_gemm3_tn) writes one [2d][K] slab per row chunk; k_dw_reduce2 sums them
// into the two weight gradients and the bias gradients from the BN backward's per-tile
// column sums of dY.
#include "kernels.h"

namespace hgnn {

// WT[k][n] = Wcat[n][k] (forward B, N-major), WC[n][k < kp]
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

}  // namespace hgnn
