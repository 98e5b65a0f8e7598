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
// Per graph and slice j this is a small GEMM  G_j (Nmax x F) . X (Nmax x F)^T,
// done with v_mfma_f32_32x32x2_f32 on 32x32 tiles of (n, m): one workgroup per
// graph stages the graph's G and X rows in LDS (F in chunks), each wave owns a
// few (n-tile, m-tile, j) items.
#include "kernels.h"

namespace hgnn {

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {
constexpr int MAXI = 5;  // items per wave kept in registers
}

template <int FC>
__global__ void __launch_bounds__(256) k_dw_dense(DwDenseArgs a) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int b = blockIdx.x;
    const int nmax = a.nmax, J = a.jt, F = a.f;
    const int npad = (nmax + 31) / 32 * 32;
    const int tiles = npad / 32;
    const int nitems = tiles * tiles * J;
    constexpr int XP = FC + 1;
    const int GP = J * FC + 1;
    float* Gs = smem;               // [npad][GP]
    float* Xs = smem + npad * GP;   // [npad][XP]
    const int off = a.node_off[b];
    const int nb = a.node_off[b + 1] - off;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int h = lane >> 5, l31 = lane & 31;

    float* dWb = a.dW + (long long)b * nmax * nmax * J;
    for (int base = 0; base < nitems; base += 4 * MAXI) {  // block-uniform passes over the items
    f32x16 acc[MAXI];
#pragma unroll
    for (int q = 0; q < MAXI; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;

    for (int f0 = 0; f0 < F; f0 += FC) {
        const int fc = min(FC, F - f0);
        __syncthreads();
        for (int i = threadIdx.x; i < npad * J * FC; i += blockDim.x) {
            const int n = i / (J * FC), j = (i / FC) % J, f = i % FC;
            float v = 0.f;
            if (f < fc && n < nmax) {
                const int k = j * F + f0 + f;
                if (n < nb) {
                    v = a.dA[(long long)(off + n) * a.lda + k];
                } else if (a.dout) {
                    for (int o = 0; o < a.dim_out; ++o)
                        v = fmaf(a.dout[b * a.dim_out + o], a.fcw[(long long)o * a.kfc + k], v);
                }
            }
            Gs[n * GP + j * FC + f] = v;
        }
        for (int i = threadIdx.x; i < npad * FC; i += blockDim.x) {
            const int m = i / FC, f = i % FC;
            float v = 0.f;
            if (f < fc && m < nmax) {
                const int c = f0 + f;
                if (a.xdense) {
                    v = a.xdense[((long long)b * F + c) * nmax + m];
                } else if (m < nb) {
                    v = a.xp[(long long)(off + m) * F + c];
                } else if (a.pmean) {
                    const float hh = __fdiv_rn(__fsub_rn(0.f, a.pmean[c]), a.pstd[c]);
                    v = __fadd_rn(__fmul_rn(*a.pw, hh), *a.pb);
                }
            }
            Xs[m * XP + f] = v;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < MAXI; ++q) {
            const int it = base + wv + 4 * q;
            if (it < nitems) {
                const int j = it % J, tm = (it / J) % tiles, tn = it / (J * tiles);
                const float* ga = Gs + (tn * 32 + l31) * GP + j * FC + h;
                const float* xb = Xs + (tm * 32 + l31) * XP + h;
#pragma unroll 4
                for (int kk = 0; kk < FC; kk += 2)
                    acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(ga[kk], xb[kk], acc[q], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < MAXI; ++q) {
        const int it = base + wv + 4 * q;
        if (it >= nitems) continue;
        const int j = it % J, tm = (it / J) % tiles, tn = it / (J * tiles);
        const int m = tm * 32 + l31;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int n = tn * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (n < nmax && m < nmax) {
                float* p = dWb + ((long long)n * nmax + m) * J + j;
                *p = a.accumulate ? *p + acc[q][r] : acc[q][r];
            }
        }
    }
    }
}

int launch_dw_dense(const DwDenseArgs& a, hipStream_t s) {
    const int npad = (a.nmax + 31) / 32 * 32;
    const int fc = npad <= 32 ? 64 : (npad <= 64 ? 32 : 16);
    const size_t lds = sizeof(float) * (size_t)npad * ((a.jt * fc + 1) + (fc + 1));
    if (lds > 64 * 1024) return 2;
    if (fc == 64) hipLaunchKernelGGL(k_dw_dense<64>, dim3(a.bs), dim3(256), lds, s, a);
    else if (fc == 32) hipLaunchKernelGGL(k_dw_dense<32>, dim3(a.bs), dim3(256), lds, s, a);
    else hipLaunchKernelGGL(k_dw_dense<16>, dim3(a.bs), dim3(256), lds, s, a);
    HGNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace hgnn
