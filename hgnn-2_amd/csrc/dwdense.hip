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

// MAXI = (n-tile, m-tile, slice) items per wave kept in registers: sized to the
// graph so the accumulators do not cap occupancy (5 x 16 AGPRs at Nmax <= 32,
// where only 3 items exist, left one wave per SIMD)
template <int FC, int MAXI>
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
    // float4 staging needs 16-byte aligned rows and slices
    const bool vec = !a.xdense && F % 4 == 0 && a.lda % 4 == 0 &&
                     ((reinterpret_cast<uintptr_t>(a.dA) | reinterpret_cast<uintptr_t>(a.xp)) & 15) == 0;

    float* dWb = a.dW + (long long)b * nmax * nmax * J;
    // block-uniform passes over the items; gridDim.y blocks of a graph share them
    for (int base = blockIdx.y * 4 * MAXI; base < nitems; base += gridDim.y * 4 * MAXI) {
    f32x16 acc[MAXI];
#pragma unroll
    for (int q = 0; q < MAXI; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;

    for (int f0 = 0; f0 < F; f0 += FC) {
        const int fc = min(FC, F - f0);
        __syncthreads();
        // Staging issues U independent loads per thread before touching LDS: the
        // element-at-a-time loop was bound by one load latency per element.
        constexpr int U = 8;
        if (vec) {
            // G rows (dA slices) and X rows share one index space, so every load of the
            // chunk is in flight before the first LDS write
            constexpr int F4 = FC / 4;
            const int g4 = npad * J * F4;
            const int t4 = g4 + npad * F4;
            for (int base = 0; base < t4; base += 256 * U) {
                float4 v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int i = base + u * 256 + threadIdx.x;
                    v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (i < g4) {
                        const int n = i / (J * F4), j = (i / F4) % J, f = (i % F4) * 4;
                        if (f < fc && n < nmax) {
                            const int k = j * F + f0 + f;
                            if (n < nb) {
                                v[u] = *reinterpret_cast<const float4*>(a.dA + (long long)(off + n) * a.lda + k);
                            } else if (a.dout) {
                                for (int o = 0; o < a.dim_out; ++o) {
                                    const float d = a.dout[b * a.dim_out + o];
                                    const float* w = a.fcw + (long long)o * a.kfc + k;
                                    v[u].x = fmaf(d, w[0], v[u].x);
                                    v[u].y = fmaf(d, w[1], v[u].y);
                                    v[u].z = fmaf(d, w[2], v[u].z);
                                    v[u].w = fmaf(d, w[3], v[u].w);
                                }
                            }
                        }
                    } else if (i < t4) {
                        const int ix = i - g4;
                        const int m = ix / F4, f = (ix % F4) * 4;
                        if (f < fc && m < nmax) {
                            const int c = f0 + f;
                            if (m < nb) {
                                v[u] = *reinterpret_cast<const float4*>(a.xp + (long long)(off + m) * F + c);
                                if (a.pmean) {
                                    v[u].x = bn_z(v[u].x, a.pmean[c], a.pstd[c], *a.pw, *a.pb);
                                    v[u].y = bn_z(v[u].y, a.pmean[c + 1], a.pstd[c + 1], *a.pw, *a.pb);
                                    v[u].z = bn_z(v[u].z, a.pmean[c + 2], a.pstd[c + 2], *a.pw, *a.pb);
                                    v[u].w = bn_z(v[u].w, a.pmean[c + 3], a.pstd[c + 3], *a.pw, *a.pb);
                                }
                            } else if (a.pmean) {
                                float t[4];
#pragma unroll
                                for (int q = 0; q < 4; ++q) {
                                    t[q] = bn_z(0.f, a.pmean[c + q], a.pstd[c + q], *a.pw, *a.pb);
                                }
                                v[u] = make_float4(t[0], t[1], t[2], t[3]);
                            }
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int i = base + u * 256 + threadIdx.x;
                    float* d = nullptr;
                    if (i < g4) {
                        const int n = i / (J * F4), j = (i / F4) % J, f = (i % F4) * 4;
                        d = Gs + n * GP + j * FC + f;
                    } else if (i < t4) {
                        const int ix = i - g4;
                        d = Xs + (ix / F4) * XP + (ix % F4) * 4;
                    }
                    if (d) {
                        d[0] = v[u].x;
                        d[1] = v[u].y;
                        d[2] = v[u].z;
                        d[3] = v[u].w;
                    }
                }
            }
        } else {
            const int gn = npad * J * FC;
            for (int base = 0; base < gn; base += 256 * U) {
                float v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int i = base + u * 256 + threadIdx.x;
                    v[u] = 0.f;
                    const int n = i / (J * FC), j = (i / FC) % J, f = i % FC;
                    if (i < gn && f < fc && n < nmax) {
                        const int k = j * F + f0 + f;
                        if (n < nb) {
                            v[u] = a.dA[(long long)(off + n) * a.lda + k];
                        } else if (a.dout) {
                            for (int o = 0; o < a.dim_out; ++o)
                                v[u] = fmaf(a.dout[b * a.dim_out + o], a.fcw[(long long)o * a.kfc + k], v[u]);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int i = base + u * 256 + threadIdx.x;
                    if (i < gn) Gs[(i / (J * FC)) * GP + ((i / FC) % J) * FC + i % FC] = v[u];
                }
            }
            const int xn = npad * FC;
            for (int base = 0; base < xn; base += 256 * U) {
                float v[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int i = base + u * 256 + threadIdx.x;
                    v[u] = 0.f;
                    const int m = i / FC, f = i % FC;
                    if (i < xn && f < fc && m < nmax) {
                        const int c = f0 + f;
                        if (a.xdense) {
                            v[u] = a.xdense[((long long)b * F + c) * nmax + m];
                        } else if (m < nb) {
                            v[u] = a.xp[(long long)(off + m) * F + c];
                            if (a.pmean) v[u] = bn_z(v[u], a.pmean[c], a.pstd[c], *a.pw, *a.pb);
                        } else if (a.pmean) {
                            v[u] = bn_z(0.f, a.pmean[c], a.pstd[c], *a.pw, *a.pb);
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int i = base + u * 256 + threadIdx.x;
                    if (i < xn) Xs[(i / FC) * XP + i % FC] = v[u];
                }
            }
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
        // read all 16 previous values before any store: a load-add-store per element
        // is serialised by the compiler (possible aliasing) into 16 memory round trips
        float old[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int n = tn * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            old[r] = (a.accumulate && n < nmax && m < nmax) ? dWb[((long long)n * nmax + m) * J + j] : 0.f;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int n = tn * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (n < nmax && m < nmax) dWb[((long long)n * nmax + m) * J + j] = old[r] + acc[q][r];
        }
    }
    }
}

template <int FC>
static void launch_fc(const DwDenseArgs& a, int maxi, int gy, size_t lds, hipStream_t s) {
    if (maxi <= 1) hipLaunchKernelGGL((k_dw_dense<FC, 1>), dim3(a.bs, gy), dim3(256), lds, s, a);
    else if (maxi <= 3) hipLaunchKernelGGL((k_dw_dense<FC, 3>), dim3(a.bs, gy), dim3(256), lds, s, a);
    else hipLaunchKernelGGL((k_dw_dense<FC, 5>), dim3(a.bs, gy), dim3(256), lds, s, a);
}

int launch_dw_dense(const DwDenseArgs& a, hipStream_t s) {
    const int npad = (a.nmax + 31) / 32 * 32;
    const int fc = npad <= 32 ? 64 : (npad <= 64 ? 32 : 16);
    const size_t lds = sizeof(float) * (size_t)npad * ((a.jt * fc + 1) + (fc + 1));
    if (lds > 64 * 1024) return 2;
    const int tiles = npad / 32;
    const int nitems = tiles * tiles * a.jt;
    int maxi = ceil_div(nitems, 4), gy = 1;
    if (a.bs < 256 && nitems > 4) {
        // few graphs (cfg1: 32): one item per wave and the items' passes spread over blocks, so the
        // grid is not a handful of long blocks (17 -> a few us per launch)
        maxi = 1;
        gy = ceil_div(nitems, 4);
    }
    if (fc == 64) launch_fc<64>(a, maxi, gy, lds, s);
    else if (fc == 32) launch_fc<32>(a, maxi, gy, lds, s);
    else launch_fc<16>(a, maxi, gy, lds, s);
    HGNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace hgnn
