// Dense gradient of the graph operators W (bs, Nmax, Nmax, J+2).
//
// scripts/train_mnb.py:56-57 sets W.requires_grad, so the reference's backward
// materialises W.grad through every graph_oper(W, X_l) (layers_mnb.py:401-409):
//   dW[b, n, m, j] = sum_l sum_f dG_l[b, j F_l + f, n] * X_l[b, f, m]
// over all Nmax x Nmax positions.  Padded positions are not zero in general:
//  * X_l at a padded node m is the previous BN's output there,
//    w * ((0 - mean_c) / std_c) + b (batch_normalization.py:43, 76), a per-channel
//    constant; for l = 0 it is the dense input X itself;
//  * dG_l at a padded node n is 0 for the middle layers (the BN mask) but, for the
//    readout, the same vector sum_o dy[b, o] fc.w[o, :] at every position
//    (layers_mnb.py:386 sums fc over all Nmax positions).
// One workgroup per graph; the graph's dG_l and X_l rows are staged through LDS
// in channel chunks, every thread keeps up to 16 outputs in registers.
#include "kernels.h"

namespace hgnn {

namespace {
constexpr int FC = 64;   // channels per LDS chunk
constexpr int FP = FC + 1;  // padded row: rows of one wave hit distinct banks
constexpr int R = 16;    // outputs per thread per pass
}

__global__ void __launch_bounds__(256) k_dw_dense(DwDenseArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int b = blockIdx.x;
    const int nmax = a.nmax, J = a.jt, F = a.f;
    const int off = a.node_off[b];
    const int nb = a.node_off[b + 1] - off;
    float* G = smem;                     // [nmax][J][FP]
    float* Xs = smem + nmax * J * FP;    // [nmax][FP]
    const int total = nmax * nmax * J;
    float* dWb = a.dW + (long long)b * total;
    for (int base = 0; base < total; base += 256 * R) {
        float acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = 0.f;
        for (int f0 = 0; f0 < F; f0 += FC) {
            const int fc = min(FC, F - f0);
            __syncthreads();
            for (int i = threadIdx.x; i < nmax * J * FC; i += blockDim.x) {
                const int n = i / (J * FC), j = (i / FC) % J, f = i % FC;
                const int li = (n * J + j) * FP + f;
                float v = 0.f;
                if (f < fc) {
                    const int k = j * F + f0 + f;
                    if (n < nb) {
                        v = a.dA[(long long)(off + n) * a.lda + k];
                    } else if (a.dout) {
                        for (int o = 0; o < a.dim_out; ++o)
                            v = fmaf(a.dout[b * a.dim_out + o], a.fcw[(long long)o * a.kfc + k], v);
                    }
                }
                G[li] = v;
            }
            for (int i = threadIdx.x; i < nmax * FC; i += blockDim.x) {
                const int m = i / FC, f = i % FC;
                float v = 0.f;
                if (f < fc) {
                    const int c = f0 + f;
                    if (a.xdense) {
                        v = a.xdense[((long long)b * F + c) * nmax + m];
                    } else if (m < nb) {
                        v = a.xp[(long long)(off + m) * F + c];
                    } else if (a.pmean) {
                        const float h = __fdiv_rn(__fsub_rn(0.f, a.pmean[c]), a.pstd[c]);
                        v = __fadd_rn(__fmul_rn(*a.pw, h), *a.pb);
                    }
                }
                Xs[m * FP + f] = v;
            }
            __syncthreads();
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int o = base + r * 256 + threadIdx.x;
                if (o < total) {
                    const int j = o % J, m = (o / J) % nmax, n = o / (J * nmax);
                    const float* g = G + (n * J + j) * FP;
                    const float* x = Xs + m * FP;
                    float s = acc[r];
                    for (int f = 0; f < fc; ++f) s = fmaf(g[f], x[f], s);
                    acc[r] = s;
                }
            }
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int o = base + r * 256 + threadIdx.x;
            if (o < total) dWb[o] = a.accumulate ? dWb[o] + acc[r] : acc[r];
        }
    }
}

int launch_dw_dense(const DwDenseArgs& a, hipStream_t s) {
    const size_t lds = sizeof(float) * (size_t)a.nmax * (a.jt + 1) * FP;
    if (lds > 160 * 1024) return 2;
    hipLaunchKernelGGL(k_dw_dense, dim3(a.bs), dim3(256), lds, s, a);
    HGNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace hgnn
