// Masked batch normalisation with scalar affine parameters
// (models/layers/batch_normalization.py:23-108) and the readout of the last
// layer (models/layers/layers_mnb.py:88-95, 379-388).
//
// BN statistics are over the REAL rows of the whole batch (mean_with_padding:
// sum over (b, n) of the masked tensor / sum(N_batch)), var = 1e-5 + mean of
// squared deviations, std = sqrt(var).  Rows are packed, so "real" = every
// packed row.  The GEMM epilogue already produced per-64-row-tile (count,
// mean, M2); they are combined in fp64 (Chan) per channel, which keeps the
// two-pass accuracy of the reference without a second pass over Y.
#include <algorithm>

#include "kernels.h"

namespace hgnn {

__device__ __forceinline__ double block_sum_d(double v, double* red) {
    v = wave_sum_d(v);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double t = 0.0;
    const int nw = blockDim.x >> 6;
    for (int i = 0; i < nw; ++i) t += red[i];
    return t;
}

// One wave per channel (4 channels per block): the tile partials of a channel in batches of 8 per
// lane (all loads in flight, clamped and selected after), wave sums only -- no block barriers.
// (A block per channel with three block-wide fp64 reductions took ~5.3 us per launch.)
__global__ void __launch_bounds__(256) k_bn_finalize(BnFwdArgs a) {
    WaveStamp stamp(a.stamps);
    const int lane = threadIdx.x & 63;
    const int ch = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ch >= a.c) return;
    if (!a.training) {
        if (lane == 0) {
            a.mean[ch] = a.run_mean[ch];
            a.std[ch] = a.run_std[ch];
        }
        return;
    }
    const int rows = *a.count;
    if (a.acc) {
        // the forward GEMM's fp64 atomic sums (copies summed in copy order): mean = S / N, var = Q / N - mean^2 in fp64
        // (every y^2 exact in fp64, the sums carry ~1e-16 relative), then the same rounding to float as below
        if (lane == 0) {
            double S = 0.0, Q = 0.0;
#pragma unroll
            for (int q = 0; q < BN_ACC_COPIES; ++q) {
                S += a.acc[((long long)q * 2 + 0) * a.c + ch];
                Q += a.acc[((long long)q * 2 + 1) * a.c + ch];
            }
            const double N = (double)rows;
            const double mean = N > 0.0 ? S / N : 0.0;
            const double var = 1e-5 + (N > 0.0 ? fmax(Q / N - mean * mean, 0.0) : 0.0);
            const float mf = (float)mean;
            const float sf = (float)sqrt(var);
            a.mean[ch] = mf;
            a.std[ch] = sf;
            if (a.run_mean) {
                const float m1 = 1.0f - a.momentum;
                a.run_mean[ch] = __fadd_rn(__fmul_rn(m1, mf), __fmul_rn(a.momentum, a.run_mean[ch]));
                a.run_std[ch] = __fadd_rn(__fmul_rn(m1, sf), __fmul_rn(a.momentum, a.run_std[ch]));
            }
        }
        return;
    }
    const int tiles = ceil_div(rows, 64);
    constexpr int U = 8;
    // two passes over the tile partials (count, mean, M2) held in registers (one load round up to 512 tiles;
    // beyond, the second pass reads them again): N and sum n m, then M2 = sum (q + n (m - mean)^2), all in
    // fp64 with DPP wave totals (wave_total_d: no LDS round trips) -- the per-lane and per-wave Chan merges
    // this replaced spent ~1.5 us in fp64 divisions and 36 ds_bpermute shuffles per wave
    float pn[U], pm[U], pq[U];
    auto load = [&](int t0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = min(t0 + u * 64 + lane, max(tiles - 1, 0));
            const float* p = a.part + ((long long)t * a.c + ch) * 3;
            const bool in = t0 + u * 64 + lane < tiles;
            pn[u] = in ? p[0] : 0.f;
            pm[u] = in ? p[1] : 0.f;
            pq[u] = in ? p[2] : 0.f;
        }
    };
    double n = 0.0, sm = 0.0;
    for (int t0 = 0; t0 < tiles; t0 += 64 * U) {
        load(t0);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            n += (double)pn[u];
            sm = fma((double)pn[u], (double)pm[u], sm);
        }
    }
    const double N = wave_total_d(n);
    const double mean = N > 0.0 ? wave_total_d(sm) / N : 0.0;
    double q = 0.0;
    for (int t0 = 0; t0 < tiles; t0 += 64 * U) {
        if (tiles > 64 * U) load(t0);  // one batch: still in registers
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double d = (double)pm[u] - mean;
            q += (double)pq[u] + (double)pn[u] * d * d;
        }
    }
    const double M2 = wave_total_d(q);
    if (lane == 0) {
        const double var = 1e-5 + (N > 0.0 ? M2 / N : 0.0);
        const float mf = (float)mean;
        const float sf = (float)sqrt(var);
        a.mean[ch] = mf;
        a.std[ch] = sf;
        if (a.run_mean) {
            // running = (1 - momentum) * batch + momentum * running (batch_normalization.py:37-38)
            const float m1 = 1.0f - a.momentum;
            a.run_mean[ch] = __fadd_rn(__fmul_rn(m1, mf), __fmul_rn(a.momentum, a.run_mean[ch]));
            a.run_std[ch] = __fadd_rn(__fmul_rn(m1, sf), __fmul_rn(a.momentum, a.run_std[ch]));
        }
    }
}

int launch_bn_finalize(const BnFwdArgs& a, hipStream_t s) {
    BnFwdArgs b = a;
    b.stamps = clock_stamps((long long)ceil_div(a.c, 4) * 4);
    HGNN_KLAUNCH(k_bn_finalize, dim3(ceil_div(a.c, 4)), dim3(256), 0, s, b);
    HGNN_LAUNCH_CHECK();
    return 0;
}

// z = w * ((y - mean) / std) + b   (batch_normalization.py:43, 76)
__global__ void __launch_bounds__(256) k_bn_apply(const float* __restrict__ y, const int* total_rows,
                                                  int c, const float* __restrict__ mean,
                                                  const float* __restrict__ stdv, const float* w,
                                                  const float* b, float* __restrict__ z) {
    const long long n = (long long)(*total_rows) * c;
    const float wv = *w, bv = *b;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (long long)gridDim.x * blockDim.x) {
        const int ch = (int)(i % c);
        const float h = __fdiv_rn(__fsub_rn(y[i], mean[ch]), stdv[ch]);
        z[i] = __fadd_rn(__fmul_rn(wv, h), bv);
    }
}

int launch_bn_apply(const float* y, const int* total_rows, int cap_rows, int c, const float* mean,
                    const float* std, const float* w, const float* b, float* z, hipStream_t s) {
    const long long n = (long long)cap_rows * c;
    int blocks = (int)ceil_div<long long>(n, 256);
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    HGNN_KLAUNCH(k_bn_apply, dim3(blocks), dim3(256), 0, s, y, total_rows, c, mean, std, w, b, z);
    HGNN_LAUNCH_CHECK();
    return 0;
}

// ---------------------------------------------------------------- BN backward

// Per 64-row tile and channel: {sum g, sum g h, sum dz h, sum dz}, g = w dz, h = (y - mean) / std.
__global__ void __launch_bounds__(256) k_bn_bwd_part(BnBwdArgs a) {
    const int tile = blockIdx.x;
    const int total = *a.total_rows;
    const int r0 = tile * 64;
    if (r0 >= total) return;
    const int r1 = min(total, r0 + 64);
    const float wv = *a.w;
    // all 256 threads busy: rgn row groups x cw channels; 4 independent loads in flight per thread
    __shared__ float red[4][256];
    const int cw = a.c < 256 ? a.c : 256;
    const int rgn = 256 / cw;
    const int tch = threadIdx.x % cw, rg = threadIdx.x / cw;
    for (int ch0 = 0; ch0 < a.c; ch0 += cw) {
        const int ch = ch0 + tch;
        float s1 = 0.f, s2 = 0.f, t1 = 0.f, t2 = 0.f;
        if (rg < rgn && ch < a.c) {
            const float mu = a.mean[ch], sd = a.std[ch];
            int r = r0 + rg;
            for (; r + 3 * rgn < r1; r += 4 * rgn) {
                float dz[4], yv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const long long i = (long long)(r + u * rgn) * a.c + ch;
                    dz[u] = a.dz[i];
                    yv[u] = a.y[i];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float h = __fdiv_rn(__fsub_rn(yv[u], mu), sd);
                    const float g = wv * dz[u];
                    s1 += g;
                    s2 = fmaf(g, h, s2);
                    t1 = fmaf(dz[u], h, t1);
                    t2 += dz[u];
                }
            }
            for (; r < r1; r += rgn) {
                const long long i = (long long)r * a.c + ch;
                const float dz = a.dz[i];
                const float h = __fdiv_rn(__fsub_rn(a.y[i], mu), sd);
                const float g = wv * dz;
                s1 += g;
                s2 = fmaf(g, h, s2);
                t1 = fmaf(dz, h, t1);
                t2 += dz;
            }
        }
        red[0][threadIdx.x] = s1;
        red[1][threadIdx.x] = s2;
        red[2][threadIdx.x] = t1;
        red[3][threadIdx.x] = t2;
        __syncthreads();
        if (rg == 0 && ch < a.c) {
            float* p = a.part + bn_bwd_part_index(ch, tile, bn_bwd_tiles(a.cap_rows));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float t = 0.f;
                for (int q = 0; q < rgn; ++q) t += red[j][q * cw + tch];
                p[j] = t;
            }
        }
        __syncthreads();
    }
}

// float4 form of k_bn_bwd_part / k_bn_bwd_apply for c % 4 == 0, c <= 1024 (the executor's
// halves: c = 2d): c/4 lanes per row, 256/(c/4) row groups, every thread keeps four rows'
// float4 loads of y and dz in flight (the scalar forms above ran at ~1 TB/s: two 4-B loads
// per lane per row and 1.2 blocks per CU).
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float& f4c(float4& v, int i) { return reinterpret_cast<float*>(&v)[i]; }

__global__ void __launch_bounds__(256) k_bn_bwd_part4(BnBwdArgs a) {
    WaveStamp stamp(a.stamps);
    const int tile = blockIdx.x;
    const int total = *a.total_rows;
    const int r0 = tile * 64;
    if (r0 >= total) return;
    const int r1 = min(total, r0 + 64);
    const float wv = *a.w;
    // row groups: at most the tile's 64 rows (narrow C: more groups would only lengthen the serial
    // per-channel combine below -- 256 of them made this kernel 16 us at C = 4, cfg1)
    const int L = a.c >> 2, RG = min(256 / L, 64);
    const int lane = threadIdx.x % L, rg = threadIdx.x / L;
    __shared__ float4 red[4][256];
    float4 s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rg < RG) {
        float mu[4], isd[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            mu[i] = a.mean[4 * lane + i];
            isd[i] = 1.0f / a.std[4 * lane + i];
        }
        auto acc = [&](float4 dz, float4 yv) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float h = (f4c(yv, i) - mu[i]) * isd[i];
                const float d = f4c(dz, i);
                const float g = wv * d;
                f4c(s[0], i) += g;
                f4c(s[1], i) = fmaf(g, h, f4c(s[1], i));
                f4c(s[2], i) = fmaf(d, h, f4c(s[2], i));
                f4c(s[3], i) += d;
            }
        };
        int r = r0 + rg;
        for (; r + 3 * RG < r1; r += 4 * RG) {
            float4 dz[4], yv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const long long i = (long long)(r + u * RG) * a.c + 4 * lane;
                dz[u] = ld4(a.dz + i);
                yv[u] = ld4(a.y + i);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) acc(dz[u], yv[u]);
        }
        for (; r < r1; r += RG) {
            const long long i = (long long)r * a.c + 4 * lane;
            acc(ld4(a.dz + i), ld4(a.y + i));
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) red[j][threadIdx.x] = s[j];
    __syncthreads();
    for (int ch = threadIdx.x; ch < a.c; ch += 256) {
        const int l = ch >> 2, comp = ch & 3;
        float4 t4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float t = 0.f;
            for (int q = 0; q < RG; ++q) t += f4c(red[j][q * L + l], comp);
            f4c(t4, j) = t;
        }
        if (a.acc64) {
            // the tile's four sums into copy tile % BN_ACC_COPIES, [copy][j][c]: a wave's lanes add 64 consecutive
            // doubles (no-return atomics, performed at the memory side; the kernel boundary orders them for apply4)
            double* dst = a.acc64 + (long long)(tile % BN_ACC_COPIES) * BN_ACC_STATS * a.c + ch;
#pragma unroll
            for (int j = 0; j < 4; ++j) atomicAdd(dst + (long long)j * a.c, (double)f4c(t4, j));
        } else {
            *reinterpret_cast<float4*>(a.part + bn_bwd_part_index(ch, tile, bn_bwd_tiles(a.cap_rows))) = t4;
        }
    }
}

// The per-channel statistics of the atomic path: the BN_ACC_COPIES copies of stat j summed in copy order (fixed), as
// k_bn_bwd_fin rounds its fp64 total to the float it stores
__device__ __forceinline__ float bn_acc_stat(const double* acc, int c, int j, int ch) {
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < BN_ACC_COPIES; ++q) v += acc[((long long)q * BN_ACC_STATS + j) * c + ch];
    return (float)v;
}

__global__ void __launch_bounds__(256) k_bn_bwd_apply4(BnBwdArgs a) {
    WaveStamp stamp(a.stamps);
    const int total = *a.total_rows;
    const float wv = *a.w;
    const float inv_n = total > 0 ? 1.0f / (float)total : 0.f;
    // atomic path: the statistics m1 / m2 of every channel from the accumulator copies, once per block into LDS
    __shared__ float sm12[2][1024];
    if (a.acc64) {
        for (int ch = threadIdx.x; ch < a.c; ch += blockDim.x) {
            sm12[0][ch] = bn_acc_stat(a.acc64, a.c, 0, ch);
            sm12[1][ch] = bn_acc_stat(a.acc64, a.c, 1, ch);
        }
        // the next half's accumulators (its part4 runs after this kernel): zeroed for it
        if (a.acc64_zero)
            for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < bn_acc_doubles(a.c);
                 i += (long long)gridDim.x * blockDim.x)
                a.acc64_zero[i] = 0.0;
        __syncthreads();
    }
    if (blockIdx.x == 0) {
        __shared__ double redd[4];
        double t1 = 0.0, t2 = 0.0;
        for (int ch = threadIdx.x; ch < a.c; ch += blockDim.x) {
            t1 += (double)(a.acc64 ? bn_acc_stat(a.acc64, a.c, 2, ch) : a.sums[ch * 4 + 2]);
            t2 += (double)(a.acc64 ? bn_acc_stat(a.acc64, a.c, 3, ch) : a.sums[ch * 4 + 3]);
        }
        const double T1 = block_sum_d(t1, redd);
        const double T2 = block_sum_d(t2, redd);
        if (threadIdx.x == 0) {
            *a.dw = (float)T1;
            *a.db = (float)T2;
        }
    }
    const int r0 = blockIdx.x * 64;
    if (r0 >= total) return;
    const int r1 = min(total, r0 + 64);
    const int L = a.c >> 2, RG = min(256 / L, 64);  // see k_bn_bwd_part4
    const int lane = threadIdx.x % L, rg = threadIdx.x / L;
    __shared__ float4 red[256];
    float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
    if (rg < RG) {
        float mu[4], isd[4], m1[4], m2[4];
        bool relu[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int ch = 4 * lane + i;
            mu[i] = a.mean[ch];
            isd[i] = 1.0f / a.std[ch];
            m1[i] = (a.acc64 ? sm12[0][ch] : a.sums[ch * 4 + 0]) * inv_n;
            m2[i] = (a.acc64 ? sm12[1][ch] : a.sums[ch * 4 + 1]) * inv_n;
            relu[i] = ch >= a.relu_from;
        }
        auto one = [&](long long i, float4 yv, float4 dz) {
            float4 d;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                f4c(d, k) = bn_bwd_dy_inv(f4c(yv, k), f4c(dz, k), mu[k], isd[k], wv, m1[k], m2[k], a.training != 0,
                                          relu[k]);
                f4c(cs, k) += f4c(d, k);
            }
            *reinterpret_cast<float4*>(a.dy + i) = d;
        };
        int r = r0 + rg;
        for (; r + 7 * RG < r1; r += 8 * RG) {
            float4 dz[8], yv[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const long long i = (long long)(r + u * RG) * a.c + 4 * lane;
                dz[u] = ld4(a.dz + i);
                yv[u] = ld4(a.y + i);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) one((long long)(r + u * RG) * a.c + 4 * lane, yv[u], dz[u]);
        }
        for (; r + 3 * RG < r1; r += 4 * RG) {
            float4 dz[4], yv[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const long long i = (long long)(r + u * RG) * a.c + 4 * lane;
                dz[u] = ld4(a.dz + i);
                yv[u] = ld4(a.y + i);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) one((long long)(r + u * RG) * a.c + 4 * lane, yv[u], dz[u]);
        }
        for (; r < r1; r += RG) {
            const long long i = (long long)r * a.c + 4 * lane;
            one(i, ld4(a.y + i), ld4(a.dz + i));
        }
    }
    if (a.dbpart) {
        red[threadIdx.x] = cs;
        __syncthreads();
        for (int ch = threadIdx.x; ch < a.c; ch += 256) {
            const int l = ch >> 2, comp = ch & 3;
            float t = 0.f;
            for (int q = 0; q < RG; ++q) t += f4c(red[q * L + l], comp);
            a.dbpart[(long long)blockIdx.x * a.c + ch] = t;
        }
    }
}

static bool bn_vec4(const BnBwdArgs& a) {
    const uintptr_t al = reinterpret_cast<uintptr_t>(a.y) | reinterpret_cast<uintptr_t>(a.dz) |
                         reinterpret_cast<uintptr_t>(a.dy);
    return a.c > 0 && a.c % 4 == 0 && a.c <= 1024 && (al & 15) == 0;
}

// One wave per channel, as k_bn_finalize: the 4 statistics of a channel over the tile partials.
__global__ void __launch_bounds__(256) k_bn_bwd_fin(BnBwdArgs a) {
    WaveStamp stamp(a.stamps);
    const int lane = threadIdx.x & 63;
    const int ch = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (ch >= a.c) return;
    const int tiles = ceil_div(*a.total_rows, 64);
    const int ntl = bn_bwd_tiles(a.cap_rows);  // the partials' tile stride
    constexpr int U = 8;
    double v[4] = {0.0, 0.0, 0.0, 0.0};
    for (int t0 = 0; t0 < tiles; t0 += 64 * U) {
        float4 pv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = min(t0 + u * 64 + lane, max(tiles - 1, 0));
            pv[u] = *reinterpret_cast<const float4*>(a.part + bn_bwd_part_index(ch, t, ntl));
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (t0 + u * 64 + lane < tiles) {
                v[0] += (double)pv[u].x;
                v[1] += (double)pv[u].y;
                v[2] += (double)pv[u].z;
                v[3] += (double)pv[u].w;
            }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = wave_total_d(v[j]);  // DPP tree, no LDS round trips
    if (lane == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) a.sums[ch * 4 + j] = (float)v[j];
    }
}

__global__ void __launch_bounds__(256) k_bn_bwd_apply(BnBwdArgs a) {
    const int total = *a.total_rows;
    const long long n = (long long)total * a.c;
    const float wv = *a.w;
    const float inv_n = total > 0 ? 1.0f / (float)total : 0.f;
    if (blockIdx.x == 0) {
        __shared__ double red[4];
        double t1 = 0.0, t2 = 0.0;
        for (int ch = threadIdx.x; ch < a.c; ch += blockDim.x) {
            t1 += (double)a.sums[ch * 4 + 2];
            t2 += (double)a.sums[ch * 4 + 3];
        }
        const double T1 = block_sum_d(t1, red);
        const double T2 = block_sum_d(t2, red);
        if (threadIdx.x == 0) {
            *a.dw = (float)T1;
            *a.db = (float)T2;
        }
    }
    (void)n;
    // one 64-row tile per block; per-channel column sums of dY -> dbpart (the conv bias grads)
    __shared__ float red[256];
    const int r0 = blockIdx.x * 64;
    if (r0 >= total) return;
    const int r1 = min(total, r0 + 64);
    // dY rows of stride ldy > c (an odd 2d padded for the dA GEMM's float4 k): the padding columns
    // are zeroed here, so the GEMM's zero weight columns never meet uninitialised workspace
    const int ldy = a.ldy > 0 ? a.ldy : a.c;
    for (int e = threadIdx.x; e < (r1 - r0) * (ldy - a.c); e += blockDim.x)
        a.dy[(long long)(r0 + e / (ldy - a.c)) * ldy + a.c + e % (ldy - a.c)] = 0.f;
    const int cw = a.c < 256 ? a.c : 256;
    const int rgn = 256 / cw;
    const int tch = threadIdx.x % cw, rg = threadIdx.x / cw;
    for (int ch0 = 0; ch0 < a.c; ch0 += cw) {
        const int ch = ch0 + tch;
        float cs = 0.f;
        if (rg < rgn && ch < a.c) {
            const float sd = a.std[ch];
            const float mu = a.mean[ch];
            const float m1 = a.sums[ch * 4 + 0] * inv_n;
            const float m2 = a.sums[ch * 4 + 1] * inv_n;
            auto one = [&](float yv, float dzv) {
                return bn_bwd_dy(yv, dzv, mu, sd, wv, m1, m2, a.training != 0, ch >= a.relu_from);
            };
            int r = r0 + rg;
            for (; r + 3 * rgn < r1; r += 4 * rgn) {
                float yv[4], dzv[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const long long i = (long long)(r + u * rgn) * a.c + ch;
                    yv[u] = a.y[i];
                    dzv[u] = a.dz[i];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float d = one(yv[u], dzv[u]);
                    a.dy[(long long)(r + u * rgn) * ldy + ch] = d;
                    cs += d;
                }
            }
            for (; r < r1; r += rgn) {
                const long long i = (long long)r * a.c + ch;
                const float d = one(a.y[i], a.dz[i]);
                a.dy[(long long)r * ldy + ch] = d;
                cs += d;
            }
        }
        if (a.dbpart) {
            red[threadIdx.x] = cs;
            __syncthreads();
            if (rg == 0 && ch < a.c) {
                float t = 0.f;
                for (int q = 0; q < rgn; ++q) t += red[q * cw + tch];
                a.dbpart[(long long)blockIdx.x * a.c + ch] = t;
            }
            __syncthreads();
        }
    }
}

// ---- Two-launch BN backward (c = 4L, L in {16, 32, 64}: 2d = 64 / 128 / 256).  The three-launch
// form above spends ~6 us of a ~20 us half on k_bn_bwd_fin, a launch that only sums the tile
// partials.  Here the statistics pass uses 256-row tiles (1024 threads, 8-16 rows in flight per
// thread), so there are few enough partials (91 at config 2's edge half) that every block of the
// apply pass sums them itself in its prologue (same fixed order in every block: identical sums,
// deterministic), and k_bn_bwd_fin disappears.  dbpart keeps its 64-row tiles.
constexpr int BN2_THREADS = 1024, BN2_ROWS = 256;

// sum over the 64 / L lane groups of a wave that hold the same channels (lanes t, t + L, ...): the
// result is complete in lanes [0, L)
template <int L>
__device__ __forceinline__ float4 wave_groups_sum4(float4 v) {
#pragma unroll
    for (int o = L; o < 64; o <<= 1) {
        v.x += __shfl_xor(v.x, o, 64);
        v.y += __shfl_xor(v.y, o, 64);
        v.z += __shfl_xor(v.z, o, 64);
        v.w += __shfl_xor(v.w, o, 64);
    }
    return v;
}

__device__ __forceinline__ float4 f4_zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

// LS: the row width in float4 (LS = L, or 2 L when a tile's channels are split over blockIdx.y: the
// 256-channel layers of d = 128 read 512 KB per 256-row tile, too much for one CU's load pipeline --
// two blocks per tile, each C = 4 L channels, write the same per-tile partials)
template <int L, int LS = L>
__global__ void __launch_bounds__(BN2_THREADS) k_bn_bwd_part2(BnBwdArgs a) {
    constexpr int RG = BN2_THREADS / L, RPT = BN2_ROWS / RG, C = 4 * LS;
    const int tile = blockIdx.x;
    const int total = *a.total_rows;
    const int r0 = tile * BN2_ROWS;
    if (r0 >= total) return;
    const int r1 = min(total, r0 + BN2_ROWS);
    const float wv = *a.w;
    const int c0 = blockIdx.y * 4 * L;  // first channel of this block
    const int lane = threadIdx.x % L, rg = threadIdx.x / L;
    float mu[4], isd[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        mu[i] = a.mean[c0 + 4 * lane + i];
        isd[i] = 1.0f / a.std[c0 + 4 * lane + i];
    }
    float4 st[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) st[j] = f4_zero();
    constexpr int U = RPT < 8 ? RPT : 8;
#pragma unroll
    for (int i0 = 0; i0 < RPT; i0 += U) {
        float4 dz[U], yv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long r = min(r0 + rg + RG * (i0 + u), r1 - 1);  // clamped: unconditional loads
            dz[u] = ld4(a.dz + r * C + c0 + 4 * lane);
            yv[u] = ld4(a.y + r * C + c0 + 4 * lane);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (r0 + rg + RG * (i0 + u) >= r1) continue;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float h = (f4c(yv[u], k) - mu[k]) * isd[k];
                const float d = f4c(dz[u], k);
                const float g = wv * d;
                f4c(st[0], k) += g;
                f4c(st[1], k) = fmaf(g, h, f4c(st[1], k));
                f4c(st[2], k) = fmaf(d, h, f4c(st[2], k));
                f4c(st[3], k) += d;
            }
        }
    }
    // over the RG row groups, in a fixed order: the 64 / L groups of a wave by shuffles, then the 16
    // wave partials of all four statistics through LDS in one round (was four rounds of a 32-deep
    // serial LDS walk)
    constexpr int SR = L <= 32 ? 4 : 2;  // statistics per LDS round (32 KB)
    __shared__ float4 red[SR][BN2_THREADS / 64][L];
    const int wid = threadIdx.x >> 6;
    const int ch = threadIdx.x;  // < 4 L: the channel (of this block's slice) this thread finishes
    float out[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) st[j] = wave_groups_sum4<L>(st[j]);
#pragma unroll
    for (int j0 = 0; j0 < 4; j0 += SR) {
        if (j0 > 0) __syncthreads();
#pragma unroll
        for (int j = 0; j < SR; ++j)
            if ((threadIdx.x & 63) < L) red[j][wid][lane] = st[j0 + j];
        __syncthreads();
        if (ch < 4 * L) {
#pragma unroll
            for (int j = 0; j < SR; ++j) {
                float t = 0.f;
#pragma unroll
                for (int w = 0; w < BN2_THREADS / 64; ++w) t += f4c(red[j][w][ch >> 2], ch & 3);
                out[j0 + j] = t;
            }
        }
    }
    if (ch < 4 * L)
        *reinterpret_cast<float4*>(a.part + ((long long)tile * C + c0 + ch) * 4) =
            make_float4(out[0], out[1], out[2], out[3]);
}

template <int L>
__global__ void __launch_bounds__(BN2_THREADS) k_bn_bwd_apply2(BnBwdArgs a) {
    constexpr int RG = BN2_THREADS / L, RPT = BN2_ROWS / RG, C = 4 * L, SUB = BN2_THREADS / C;
    constexpr int RPQ = 64 / RG;  // rows of a thread per 64-row dbpart tile
    const int total = *a.total_rows;
    const int r0 = blockIdx.x * BN2_ROWS;
    const bool first = blockIdx.x == 0;
    if (r0 >= total && !first) return;
    const int tiles = ceil_div(total, BN2_ROWS);
    // prologue: the per-channel sums over all tile partials, fp64, fixed order (thread (ch, sub)
    // sums tiles sub, sub + SUB, ...; then the SUB sub-sums in order)
    __shared__ __attribute__((aligned(16))) double2 sbuf[2 * BN2_THREADS];  // prologue sums, then the dbpart reduction
    double2* pr = sbuf;
    double2* pt = sbuf + BN2_THREADS;
    __shared__ float sm1[C], sm2[C];
    {
        const int ch = threadIdx.x % C, sub = threadIdx.x / C;
        double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
        int t = sub;
        for (; t + 3 * SUB < tiles; t += 4 * SUB) {
            float4 q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) q[u] = ld4(a.part + ((long long)(t + u * SUB) * C + ch) * 4);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                v0 += (double)q[u].x;
                v1 += (double)q[u].y;
                v2 += (double)q[u].z;
                v3 += (double)q[u].w;
            }
        }
        for (; t < tiles; t += SUB) {
            const float4 q = ld4(a.part + ((long long)t * C + ch) * 4);
            v0 += (double)q.x;
            v1 += (double)q.y;
            v2 += (double)q.z;
            v3 += (double)q.w;
        }
        pr[threadIdx.x] = make_double2(v0, v1);
        pt[threadIdx.x] = make_double2(v2, v3);
    }
    __syncthreads();
    const float inv_n = total > 0 ? 1.0f / (float)total : 0.f;
    if (threadIdx.x < C) {
        double s1 = 0.0, s2 = 0.0;
        for (int q = 0; q < SUB; ++q) {
            s1 += pr[q * C + threadIdx.x].x;
            s2 += pr[q * C + threadIdx.x].y;
        }
        sm1[threadIdx.x] = (float)s1 * inv_n;
        sm2[threadIdx.x] = (float)s2 * inv_n;
        if (first) {  // BN scalar grads: dw = sum_c sum dz h, db = sum_c sum dz (per channel rounded, as k_bn_bwd_fin)
            double t1 = 0.0, t2 = 0.0;
            for (int q = 0; q < SUB; ++q) {
                t1 += pt[q * C + threadIdx.x].x;
                t2 += pt[q * C + threadIdx.x].y;
            }
            pt[threadIdx.x] = make_double2((double)(float)t1, (double)(float)t2);
        }
    }
    __syncthreads();
    if (first && threadIdx.x == 0) {
        double T1 = 0.0, T2 = 0.0;
        for (int c = 0; c < C; ++c) {
            T1 += pt[c].x;
            T2 += pt[c].y;
        }
        *a.dw = (float)T1;
        *a.db = (float)T2;
    }
    if (r0 >= total) return;
    const int r1 = min(total, r0 + BN2_ROWS);
    const float wv = *a.w;
    const int lane = threadIdx.x % L, rg = threadIdx.x / L;
    float mu[4], isd[4], m1[4], m2[4];
    bool relu[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int ch = 4 * lane + i;
        mu[i] = a.mean[ch];
        isd[i] = 1.0f / a.std[ch];
        m1[i] = sm1[ch];
        m2[i] = sm2[ch];
        relu[i] = ch >= a.relu_from;
    }
    float4 cs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) cs[q] = f4_zero();
    constexpr int U = RPT < 8 ? RPT : 8;
#pragma unroll
    for (int i0 = 0; i0 < RPT; i0 += U) {
        float4 dz[U], yv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long r = min(r0 + rg + RG * (i0 + u), r1 - 1);
            dz[u] = ld4(a.dz + r * C + 4 * lane);
            yv[u] = ld4(a.y + r * C + 4 * lane);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int r = r0 + rg + RG * (i0 + u);
            if (r >= r1) continue;
            float4 d;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                f4c(d, k) = bn_bwd_dy_inv(f4c(yv[u], k), f4c(dz[u], k), mu[k], isd[k], wv, m1[k], m2[k],
                                          a.training != 0, relu[k]);
                f4c(cs[(i0 + u) / RPQ], k) += f4c(d, k);
            }
            *reinterpret_cast<float4*>(a.dy + (long long)r * C + 4 * lane) = d;
        }
    }
    if (!a.dbpart) return;
    // per-64-row-tile column sums of dY (the conv bias gradients): every thread holds its rows' sums for
    // the block's four tiles; over the row groups in a fixed order -- the lane groups of a wave by
    // shuffles, then the 16 wave partials of all four tiles through LDS in one round
    constexpr int NWV = BN2_THREADS / 64, QR = L <= 32 ? 4 : 2;  // tiles per LDS round (32 KB)
    float4 (*red)[NWV][L] = reinterpret_cast<float4 (*)[NWV][L]>(sbuf);
    const int wid = threadIdx.x >> 6;
    const int t64 = ceil_div(total, 64);
#pragma unroll
    for (int q = 0; q < 4; ++q) cs[q] = wave_groups_sum4<L>(cs[q]);
#pragma unroll
    for (int q0 = 0; q0 < 4; q0 += QR) {
        __syncthreads();  // the prologue's (or the previous round's) readers of sbuf are done
#pragma unroll
        for (int q = 0; q < QR; ++q)
            if ((threadIdx.x & 63) < L) red[q][wid][lane] = cs[q0 + q];
        __syncthreads();
        if (threadIdx.x < C) {
#pragma unroll
            for (int q = 0; q < QR; ++q) {
                const int tq = blockIdx.x * 4 + q0 + q;
                float t = 0.f;
#pragma unroll
                for (int w = 0; w < NWV; ++w) t += f4c(red[q][w][threadIdx.x >> 2], threadIdx.x & 3);
                if (tq < t64) a.dbpart[(long long)tq * C + threadIdx.x] = t;
            }
        }
    }
}


// ---- The same two-launch BN backward for narrow channel counts (c = 4L, L in {1, 2, 4}: the
// GNN_simple layers of config 1).  256 rows per block, one row per lane group (256 L threads),
// and the row-group sums as wave shuffles + a sum over the block's waves instead of a serial walk
// over 256 row groups.  Replaces the single-block k_bn_bwd_small (18.6 us per launch at config 1:
// one CU does all the work).
template <int L>
__device__ __forceinline__ float4 wave_rows_sum4(float4 v) {
    // sum over the lanes of a wave holding the same channel group (lanes t, t + L, t + 2L, ...)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int o = 32; o >= L; o >>= 1) f4c(v, k) += __shfl_xor(f4c(v, k), o, 64);
    return v;
}

template <int L>
__global__ void __launch_bounds__(256 * L) k_bn_bwd_part2s(BnBwdArgs a) {
    constexpr int NT = 256 * L, C = 4 * L, NW = NT / 64;
    const int total = *a.total_rows;
    const int r0 = blockIdx.x * BN2_ROWS;
    if (r0 >= total) return;
    const float wv = *a.w;
    const int lane = threadIdx.x % L, r = r0 + threadIdx.x / L;
    float4 st[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) st[j] = f4_zero();
    if (r < total) {
        float4 dz = ld4(a.dz + (long long)r * C + 4 * lane), yv = ld4(a.y + (long long)r * C + 4 * lane);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float mu = a.mean[4 * lane + k], isd = 1.0f / a.std[4 * lane + k];
            const float h = (f4c(yv, k) - mu) * isd;
            const float d = f4c(dz, k);
            const float g = wv * d;
            f4c(st[0], k) = g;
            f4c(st[1], k) = g * h;
            f4c(st[2], k) = d * h;
            f4c(st[3], k) = d;
        }
    }
    __shared__ float4 wp[4][NW][L];
    const int w = threadIdx.x >> 6, wl = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float4 t = wave_rows_sum4<L>(st[j]);
        if (wl < L) wp[j][w][wl] = t;
    }
    __syncthreads();
    if ((int)threadIdx.x < C) {
        const int ch = threadIdx.x;
        float out[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float t = 0.f;
            for (int q = 0; q < NW; ++q) t += f4c(wp[j][q][ch >> 2], ch & 3);
            out[j] = t;
        }
        *reinterpret_cast<float4*>(a.part + ((long long)blockIdx.x * C + ch) * 4) =
            make_float4(out[0], out[1], out[2], out[3]);
    }
}

template <int L>
__global__ void __launch_bounds__(256 * L) k_bn_bwd_apply2s(BnBwdArgs a) {
    constexpr int NT = 256 * L, C = 4 * L, NW = NT / 64, SUB = NT / C;
    const int total = *a.total_rows;
    const int r0 = blockIdx.x * BN2_ROWS;
    const bool first = blockIdx.x == 0;
    if (r0 >= total && !first) return;
    const int tiles = ceil_div(total, BN2_ROWS);
    __shared__ double2 pr[NT];
    __shared__ double2 pt[NT];
    __shared__ float sm1[C], sm2[C];
    {
        const int ch = threadIdx.x % C, sub = threadIdx.x / C;
        double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
        for (int t = sub; t < tiles; t += SUB) {
            const float4 q = ld4(a.part + ((long long)t * C + ch) * 4);
            v0 += (double)q.x;
            v1 += (double)q.y;
            v2 += (double)q.z;
            v3 += (double)q.w;
        }
        pr[threadIdx.x] = make_double2(v0, v1);
        pt[threadIdx.x] = make_double2(v2, v3);
    }
    __syncthreads();
    const float inv_n = total > 0 ? 1.0f / (float)total : 0.f;
    if ((int)threadIdx.x < C) {
        double s1 = 0.0, s2 = 0.0, t1 = 0.0, t2 = 0.0;
        for (int q = 0; q < SUB; ++q) {
            s1 += pr[q * C + threadIdx.x].x;
            s2 += pr[q * C + threadIdx.x].y;
            t1 += pt[q * C + threadIdx.x].x;
            t2 += pt[q * C + threadIdx.x].y;
        }
        sm1[threadIdx.x] = (float)s1 * inv_n;
        sm2[threadIdx.x] = (float)s2 * inv_n;
        if (first) pt[threadIdx.x] = make_double2((double)(float)t1, (double)(float)t2);
    }
    __syncthreads();
    if (first && threadIdx.x == 0) {
        double T1 = 0.0, T2 = 0.0;
        for (int c = 0; c < C; ++c) {
            T1 += pt[c].x;
            T2 += pt[c].y;
        }
        *a.dw = (float)T1;
        *a.db = (float)T2;
    }
    if (r0 >= total) return;
    const float wv = *a.w;
    const int lane = threadIdx.x % L, r = r0 + threadIdx.x / L;
    float4 d = f4_zero();
    if (r < total) {
        float4 dz = ld4(a.dz + (long long)r * C + 4 * lane), yv = ld4(a.y + (long long)r * C + 4 * lane);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int ch = 4 * lane + k;
            f4c(d, k) = bn_bwd_dy_inv(f4c(yv, k), f4c(dz, k), a.mean[ch], 1.0f / a.std[ch], wv, sm1[ch], sm2[ch],
                                      a.training != 0, ch >= a.relu_from);
        }
        *reinterpret_cast<float4*>(a.dy + (long long)r * C + 4 * lane) = d;
    }
    if (!a.dbpart) return;
    // per-64-row-tile column sums of dY: a tile is L consecutive waves
    __shared__ float4 wd[NW][L];
    const int w = threadIdx.x >> 6, wl = threadIdx.x & 63;
    const float4 t = wave_rows_sum4<L>(d);
    if (wl < L) wd[w][wl] = t;
    __syncthreads();
    const int t64 = ceil_div(total, 64);
    if ((int)threadIdx.x < 4 * C) {
        const int q = threadIdx.x / C, ch = threadIdx.x % C, tq = blockIdx.x * 4 + q;
        if (tq < t64) {
            float acc = 0.f;
            for (int u = 0; u < L; ++u) acc += f4c(wd[q * L + u][ch >> 2], ch & 3);
            a.dbpart[(long long)tq * C + ch] = acc;
        }
    }
}

template <int L>
static void bn2s_launch(const BnBwdArgs& a, hipStream_t s) {
    const int t2 = ceil_div(a.cap_rows, BN2_ROWS);
    HGNN_KLAUNCH(k_bn_bwd_part2s<L>, dim3(t2), dim3(256 * L), 0, s, a);
    HGNN_KLAUNCH(k_bn_bwd_apply2s<L>, dim3(t2), dim3(256 * L), 0, s, a);
}

static bool bn2_enabled() {
    static const bool on = [] {
        const char* e = getenv("HGNN_BN_BWD2");
        return !e || e[0] != '0';
    }();
    return on;
}

// The wide two-launch form (c = 64 / 128 / 256) is off by default since round 4: with the dW GEMM on bf16 MFMA
// beside it, the three-launch form's 64-row tiles (many 256-thread blocks instead of ~91 of 1024 threads)
// measured 1.254-1.265 vs 1.282-1.313 ms per step in five alternating pairs (config 2); HGNN_BN_BWD2=1
// turns it back on
static bool bn2_wide_enabled() {
    static const bool on = [] {
        const char* e = getenv("HGNN_BN_BWD2");
        return e && e[0] == '1';
    }();
    return on;
}

template <int L>
static void bn2_launch(const BnBwdArgs& a, hipStream_t s) {
    const int t2 = ceil_div(a.cap_rows, BN2_ROWS);
    if constexpr (L == 64)  // 256 channels: two blocks of 128 per tile
        HGNN_KLAUNCH((k_bn_bwd_part2<32, 64>), dim3(t2, 2), dim3(BN2_THREADS), 0, s, a);
    else
        HGNN_KLAUNCH(k_bn_bwd_part2<L>, dim3(t2), dim3(BN2_THREADS), 0, s, a);
    HGNN_KLAUNCH(k_bn_bwd_apply2<L>, dim3(t2), dim3(BN2_THREADS), 0, s, a);
}

int launch_bn_backward(const BnBwdArgs& a, hipStream_t s, int apply) {
    const int tiles = bn_bwd_tiles(a.cap_rows);
    // the paths without the atomic statistics still hand the next half a zeroed accumulator region
    const bool acc_path =
        a.acc64 && bn_vec4(a) && (a.ldy == 0 || a.ldy == a.c) && apply && a.c <= 1024 &&
        !(bn2_enabled() && ceil_div(a.cap_rows, BN2_ROWS) <= 192 && (a.c == 4 || a.c == 8 || a.c == 16)) &&
        !(bn2_wide_enabled() && ceil_div(a.cap_rows, BN2_ROWS) <= 192 && (a.c == 64 || a.c == 128 || a.c == 256));
    if (a.acc64_zero && !acc_path)
        HGNN_HOST_CHECK(hipMemsetAsync(a.acc64_zero, 0, (size_t)bn_acc_doubles(a.c) * sizeof(double), s));
    if (a.ldy != 0 && a.ldy < a.c) return HGNN_ERR_ARG;
    // a padded dY stride is written by the scalar apply only
    const bool v4 = bn_vec4(a) && (a.ldy == 0 || a.ldy == a.c);
    // (c / 4 a power of two: the per-wave shuffle reduction pairs the lanes of one channel group)
    // the two-launch forms sum every statistics partial in each apply block's prologue (O(tiles^2 C)
    // L2 reads): only up to 192 row tiles of capacity (49 K rows; config 2's edge half is 140 with 91
    // live); larger inputs take part4 + fin + apply4
    const bool few = ceil_div(a.cap_rows, BN2_ROWS) <= 192;
    if (apply && v4 && bn2_enabled() && few && tiles > 0 && (a.c == 4 || a.c == 8 || a.c == 16)) {
        if (a.c == 4) bn2s_launch<1>(a, s);
        else if (a.c == 8) bn2s_launch<2>(a, s);
        else bn2s_launch<4>(a, s);
        HGNN_LAUNCH_CHECK();
        return 0;
    }
    if (apply && v4 && tiles > 0 && bn2_wide_enabled() && few && (a.c == 64 || a.c == 128 || a.c == 256)) {
        if (a.c == 64) bn2_launch<16>(a, s);
        else if (a.c == 128) bn2_launch<32>(a, s);
        else bn2_launch<64>(a, s);
        HGNN_LAUNCH_CHECK();
        return 0;
    }
    BnBwdArgs as = a;  // a stamp slot per launch (stamp-mode clock only)
    // the atomic statistics (acc64): part4 -> apply4, no k_bn_bwd_fin
    const bool acc = a.acc64 && v4 && apply && a.c <= 1024;
    if (!acc) {
        as.acc64 = nullptr;
        as.acc64_zero = nullptr;
    }
    if (tiles > 0) {
        as.stamps = v4 ? clock_stamps((long long)tiles * 4) : nullptr;
        if (v4) HGNN_KLAUNCH(k_bn_bwd_part4, dim3(tiles), dim3(256), 0, s, as);
        else HGNN_KLAUNCH(k_bn_bwd_part, dim3(tiles), dim3(256), 0, s, a);
    }
    HGNN_LAUNCH_CHECK();
    if (!acc) {
        as.stamps = clock_stamps((long long)ceil_div(a.c, 4) * 4);
        HGNN_KLAUNCH(k_bn_bwd_fin, dim3(ceil_div(a.c, 4)), dim3(256), 0, s, as);
        HGNN_LAUNCH_CHECK();
    }
    if (!apply) return 0;
    as.stamps = v4 ? clock_stamps((long long)(tiles > 0 ? tiles : 1) * 4) : nullptr;
    if (v4) HGNN_KLAUNCH(k_bn_bwd_apply4, dim3(tiles > 0 ? tiles : 1), dim3(256), 0, s, as);
    else HGNN_KLAUNCH(k_bn_bwd_apply, dim3(tiles > 0 ? tiles : 1), dim3(256), 0, s, a);
    HGNN_LAUNCH_CHECK();
    return 0;
}

// ---------------------------------------------------------------- readout
// y[b, o] = sum_{n < N_b} sum_k A[n, k] fcw[o, k] + Nmax * fcb[o]
// The reference sums fc(x1) over all Nmax padded positions; padded positions
// have x1 = 0, so each contributes exactly fc.bias (layers_mnb.py:92, 386).
// One 1024-thread block per graph, a thread per column; the row loop issues 8
// independent loads per round (the serial walk was latency-bound: 27 us / step).
constexpr int RO_THREADS = 1024;

__global__ void __launch_bounds__(RO_THREADS) k_readout_fwd(const float* __restrict__ A, int k,
                                                            const int* __restrict__ node_off, int nmax,
                                                            const float* __restrict__ fcw,
                                                            const float* __restrict__ fcb, int dim_out,
                                                            float* __restrict__ colsum,
                                                            float* __restrict__ out, uint64_t* stamps) {
    WaveStamp stamp(stamps);
    __shared__ double red[RO_THREADS / 64];
    const int b = blockIdx.x;
    const int r0 = node_off[b], r1 = node_off[b + 1];
    // fp64 column sums: the reference sums per-position dot products with
    // torch.sum (pairwise); a plain fp32 running sum would be less accurate
    double part0 = 0.0;
    for (int kk = threadIdx.x; kk < k; kk += RO_THREADS) {
        const float* col = A + kk;
        double c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int r = r0;
        for (; r + 8 <= r1; r += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = col[(long long)(r + u) * k];
#pragma unroll
            for (int u = 0; u < 8; ++u) c[u] += (double)v[u];
        }
        for (int u = 0; r < r1; ++r, ++u) c[u] += (double)col[(long long)r * k];
        const double cs = ((c[0] + c[1]) + (c[2] + c[3])) + ((c[4] + c[5]) + (c[6] + c[7]));
        colsum[(long long)b * k + kk] = (float)cs;
        if (dim_out > 0) part0 += cs * (double)fcw[kk];
    }
    __syncthreads();
    for (int o = 0; o < dim_out; ++o) {
        double part = 0.0;
        if (o == 0) {
            part = part0;
        } else {
            for (int kk = threadIdx.x; kk < k; kk += RO_THREADS)
                part += (double)colsum[(long long)b * k + kk] * (double)fcw[(long long)o * k + kk];
        }
        part = wave_sum_d(part);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = part;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0.0;
            for (int w = 0; w < RO_THREADS / 64; ++w) t += red[w];
            out[b * dim_out + o] = (float)(t + (double)nmax * (double)fcb[o]);
        }
        __syncthreads();
    }
}

int launch_readout_fwd(const float* a, int k, const int* node_off, int bs, int nmax, const float* fcw,
                       const float* fcb, int dim_out, float* colsum, float* out, hipStream_t s) {
    HGNN_KLAUNCH(k_readout_fwd, dim3(bs), dim3(RO_THREADS), 0, s, a, k, node_off, nmax, fcw, fcb, dim_out,
                 colsum, out, clock_stamps((long long)bs * (RO_THREADS / 64)));
    HGNN_LAUNCH_CHECK();
    return 0;
}

// dA[r, k] = sum_o dout[b(r), o] fcw[o, k]
__global__ void __launch_bounds__(256) k_readout_bwd_da(const float* __restrict__ dout,
                                                        const int* __restrict__ node_off,
                                                        const float* __restrict__ fcw, int dim_out,
                                                        int k, float* __restrict__ da) {
    const int b = blockIdx.x;
    const int r0 = node_off[b], r1 = node_off[b + 1];
    for (int kk = threadIdx.x; kk < k; kk += blockDim.x) {
        float v = 0.f;
        for (int o = 0; o < dim_out; ++o) v = fmaf(dout[b * dim_out + o], fcw[(long long)o * k + kk], v);
        for (int r = r0; r < r1; ++r) da[(long long)r * k + kk] = v;
    }
}

int launch_readout_bwd_da(const float* dout, const int* node_off, int bs, int cap_rows, const int* total_rows,
                          const float* fcw, int dim_out, int k, float* da, hipStream_t s) {
    (void)cap_rows;
    (void)total_rows;
    HGNN_KLAUNCH(k_readout_bwd_da, dim3(bs), dim3(256), 0, s, dout, node_off, fcw, dim_out, k, da);
    HGNN_LAUNCH_CHECK();
    return 0;
}

// ---- Readout backward without the [rows][K] gradient buffer.  The readout sums fc(x1) over the
// nodes of a graph (layers_mnb.py:385-386), so the gradient of x1 at every node n of graph b is
// the same row R_b = dout[b] . fcw.  The transposed gathers of the last layer therefore reduce
// to the row's coefficient sums times R_b:
//   G rows (graph_oper(W, X)^T):  dX[r, c] (+)= sum_j (sum_e v_j(e)) R_b[j C + c]
//   P rows (P_multi(Pm/Pd, XL)^T): dXL[r, c] (+)= (sum_e pm) R_b[Kg + c] + (sum_e pd) R_b[Kg + Cp + c]
// (entries of a row only reference columns of the same graph), and the dense operator gradient
// of the readout is dW[b, n, m, j] = sum_f R_b[j F + f] X[m, f] for every n < Nmax.  The
// coefficient sums are exact for the reference's operators (small dyadic values), so only the
// order of the final products differs from the gather form.
__device__ __forceinline__ float readout_row(const float* __restrict__ dout, const float* __restrict__ fcw,
                                             int dim_out, int k, int b, int col) {
    float v = 0.f;
    for (int o = 0; o < dim_out; ++o) v = fmaf(dout[b * dim_out + o], fcw[(long long)o * k + col], v);
    return v;
}

// One block per (graph, kind): blockIdx.y = 0 -> the graph's node rows (G), 1 -> its edge rows (P).
// A thread per row sums the row's coefficients (4 entries in flight), then the block writes the
// rows coalesced over (row, channel).
constexpr int RA_THREADS = 256;

__global__ void __launch_bounds__(RA_THREADS) k_readout_agg_bwd(ReadoutAggArgs a) {
    WaveStamp stamp(a.stamps);
    const int b = blockIdx.x;
    const bool g = blockIdx.y == 0;
    float* out = g ? a.g_out : a.p_out;
    if (!out) return;
    extern __shared__ float sh[];
    const int ns = g ? a.jt : 2;
    const int C = g ? a.cg : a.cp;
    const int* off = g ? a.node_off : a.edge_off;
    const int r0 = off[b], nr = off[b + 1] - r0;
    float* R = sh;                // [ns C]: R_b over the gathered columns
    float* CS = sh + ns * C;      // [rows][ns]
    const int kb = g ? 0 : a.jt * a.cg;
    for (int t = threadIdx.x; t < ns * C; t += RA_THREADS)
        R[t] = readout_row(a.dout, a.fcw, a.dim_out, a.k, b, kb + t);
    const StructView L = g ? a.g : a.p;
    for (int i = threadIdx.x; i < nr; i += RA_THREADS) {
        const RowInfo ri = L.rows[r0 + i];
        float cs[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) cs[j] = 0.f;
        int e = 0;
        for (; e + 4 <= ri.count; e += 4) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(L.entries + (long long)(ri.start + e + u) * L.stride);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                cs[0] += v[u].y;
                cs[1] += v[u].z;
                cs[2] += v[u].w;
                for (int j = 3; j < ns; ++j) cs[j] += L.entries[(long long)(ri.start + e + u) * L.stride + 1 + j];
            }
        }
        for (; e < ri.count; ++e) {
            const float* en = L.entries + (long long)(ri.start + e) * L.stride;
            for (int j = 0; j < ns; ++j) cs[j] += en[1 + j];
        }
        for (int j = 0; j < ns; ++j) CS[i * ns + j] = cs[j];
    }
    __syncthreads();
    // a wave per row, lanes along the channels (float4 where C % 4 == 0: the row-major [rows][C] output of
    // the executor always is); the flat (row, channel) loop's two integer divisions per element were most
    // of this kernel's VALU
    const int acc = g ? a.g_acc : a.p_acc;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = RA_THREADS / 64;
    if ((C & 3) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
        for (int r = wv; r < nr; r += nw) {
            float4* orow = reinterpret_cast<float4*>(out + (long long)(r0 + r) * C);
            for (int c4 = lane; c4 < (C >> 2); c4 += 64) {
                float4 v = acc ? orow[c4] : make_float4(0.f, 0.f, 0.f, 0.f);
                for (int j = 0; j < ns; ++j) {
                    const float w = CS[r * ns + j];
                    const float4 q = *reinterpret_cast<const float4*>(R + j * C + 4 * c4);
                    v.x = fmaf(w, q.x, v.x);
                    v.y = fmaf(w, q.y, v.y);
                    v.z = fmaf(w, q.z, v.z);
                    v.w = fmaf(w, q.w, v.w);
                }
                orow[c4] = v;
            }
        }
        return;
    }
    for (int r = wv; r < nr; r += nw)
        for (int c = lane; c < C; c += 64) {
            float v = acc ? out[(long long)(r0 + r) * C + c] : 0.f;
            for (int j = 0; j < ns; ++j) v = fmaf(CS[r * ns + j], R[j * C + c], v);
            out[(long long)(r0 + r) * C + c] = v;
        }
}

// dynamic LDS of the two readout-row kernels (beyond 64 KB allowed per kernel, up to the CU's 160 KB)
constexpr size_t RO_LDS_CAP = 160 * 1024;

static size_t readout_agg_bwd_lds(const ReadoutAggArgs& a) {
    const int maxrows = a.p_out ? (a.p_cap + a.bs - 1) / a.bs : 0;  // rows per graph <= emax
    const int grow = (a.g_cap + a.bs - 1) / a.bs;
    return sizeof(float) * (size_t)std::max(a.jt * a.cg + grow * a.jt, 2 * a.cp + maxrows * 2);
}

static size_t dw_readout_lds(const DwDenseArgs& a) {
    return sizeof(float) * ((size_t)a.jt * a.f + (size_t)a.nmax * (a.f + 1) + (size_t)a.nmax * a.jt);
}

template <typename K>
static void allow_ro_lds(K* kernel, size_t lds) {
    if (lds > 64 * 1024)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)RO_LDS_CAP);
}

bool readout_row_fits(const ReadoutAggArgs& ra, const DwDenseArgs* dw) {
    if (ra.jt > 8) return false;
    if ((ra.g_out || ra.p_out) && readout_agg_bwd_lds(ra) > RO_LDS_CAP) return false;
    return !dw || dw_readout_lds(*dw) <= RO_LDS_CAP;
}

int launch_readout_agg_bwd(const ReadoutAggArgs& a, hipStream_t s) {
    if (a.jt > 8 || (!a.g_out && !a.p_out)) return a.jt > 8 ? HGNN_ERR_UNSUPPORTED : 0;
    const size_t lds = readout_agg_bwd_lds(a);
    if (lds > RO_LDS_CAP) return HGNN_ERR_UNSUPPORTED;
    allow_ro_lds(k_readout_agg_bwd, lds);
    ReadoutAggArgs as = a;
    as.stamps = clock_stamps((long long)a.bs * (a.p_out ? 2 : 1) * (RA_THREADS / 64));
    HGNN_KLAUNCH(k_readout_agg_bwd, dim3(a.bs, a.p_out ? 2 : 1), dim3(RA_THREADS), lds, s, as);
    HGNN_LAUNCH_CHECK();
    return 0;
}

// dW[b, n, m, j] (+)= u_b[m, j] = sum_f R_b[j F + f] X[m, f] for all n < Nmax: one block per graph,
// u in LDS, then written to every row n.  X: BN of the producer applied on load, the BN of 0 at
// padded m (as k_dw_dense); the dense layer input (xdense) as stored.
__global__ void __launch_bounds__(256) k_dw_readout(DwDenseArgs a) {
    WaveStamp stamp(a.stamps);
    extern __shared__ float sh[];
    const int b = blockIdx.x;
    const int nmax = a.nmax, J = a.jt, F = a.f, FP = F + 1;
    float* R = sh;              // [J F]
    float* X = sh + J * F;      // [nmax][F + 1]
    float* U = X + nmax * FP;   // [nmax J]
    const int off = a.node_off[b], nb = a.node_off[b + 1] - off;
    const float wv = a.pw ? *a.pw : 0.f, bv = a.pb ? *a.pb : 0.f;
    for (int t = threadIdx.x; t < J * F; t += 256)
        R[t] = readout_row(a.dout, a.fcw, a.dim_out, a.kfc, b, t);
    for (int t = threadIdx.x; t < nmax * F; t += 256) {  // coalesced over f
        const int m = t / F, f = t % F;
        float x;
        if (a.xdense) {
            x = a.xdense[((long long)b * F + f) * nmax + m];
        } else if (m < nb) {
            x = a.xp[(long long)(off + m) * F + f];
            if (a.pmean) x = bn_z_s(x, a.pmean[f], bn_scale(wv, a.pstd[f]), bv);
        } else {
            x = a.pmean ? bn_z(0.f, a.pmean[f], a.pstd[f], wv, bv) : 0.f;
        }
        X[m * FP + f] = x;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < nmax * J; t += 256) {
        const int m = t / J, j = t % J;
        float u = 0.f;
        for (int f = 0; f < F; ++f) u = fmaf(R[j * F + f], X[m * FP + f], u);
        U[t] = u;
    }
    __syncthreads();
    float* dWb = a.dW + (long long)b * nmax * nmax * J;
    const int per = nmax * J;
    // the same row u for every n: a thread per column t of the [n][per] block, walking the rows (no 64-bit
    // modulo per element)
    for (int t = threadIdx.x; t < per; t += 256) {
        const float u = U[t];
        for (int n = 0; n < nmax; ++n) {
            float* q = dWb + (long long)n * per + t;
            *q = a.accumulate ? *q + u : u;
        }
    }
}

int launch_dw_readout(const DwDenseArgs& a, hipStream_t s) {
    const size_t lds = dw_readout_lds(a);
    if (lds > RO_LDS_CAP || !a.dout) return HGNN_ERR_UNSUPPORTED;
    allow_ro_lds(k_dw_readout, lds);
    DwDenseArgs as = a;
    as.stamps = clock_stamps((long long)a.bs * 4);
    HGNN_KLAUNCH(k_dw_readout, dim3(a.bs), dim3(256), lds, s, as);
    HGNN_LAUNCH_CHECK();
    return 0;
}

// dfcw[o, k] = sum_b dout[b, o] colsum[b, k];  dfcb[o] = Nmax sum_b dout[b, o]
// Stage 1: block (k-chunk of 64, graph chunk) -> fp64 partials; stage 2 sums the chunks in order.
constexpr int RB_CHUNKS = 16;

__global__ void __launch_bounds__(256) k_readout_bwd_part(const float* __restrict__ dout,
                                                          const float* __restrict__ colsum, int bs,
                                                          int dim_out, int k, double* __restrict__ part,
                                                          uint64_t* stamps) {
    WaveStamp stamp(stamps);
    __shared__ double red[4][64];
    const int kk = blockIdx.x * 64 + (threadIdx.x & 63);
    const int g = threadIdx.x >> 6;
    const int per = ceil_div(bs, RB_CHUNKS);
    const int b0 = blockIdx.y * per, b1 = min(bs, b0 + per);
    for (int o = 0; o < dim_out; ++o) {
        double s = 0.0;
        if (kk < k)
            for (int b = b0 + g; b < b1; b += 4)
                s += (double)dout[b * dim_out + o] * (double)colsum[(long long)b * k + kk];
        red[g][threadIdx.x & 63] = s;
        __syncthreads();
        if (g == 0 && kk < k) {
            const int t = threadIdx.x & 63;
            part[((long long)blockIdx.y * dim_out + o) * k + kk] = red[0][t] + red[1][t] + red[2][t] + red[3][t];
        }
        __syncthreads();
        if (blockIdx.x == 0) {  // this chunk's sum of dout (bias gradient partial)
            double sb = 0.0;
            for (int b = b0 + (int)threadIdx.x; b < b1; b += 256) sb += (double)dout[b * dim_out + o];
            red[g][threadIdx.x & 63] = wave_sum_d(sb);
            __syncthreads();
            if (threadIdx.x == 0)
                part[(long long)RB_CHUNKS * dim_out * k + blockIdx.y * dim_out + o] =
                    red[0][0] + red[1][0] + red[2][0] + red[3][0];
            __syncthreads();
        }
    }
}

__global__ void __launch_bounds__(256) k_readout_bwd_params(const float* __restrict__ dout,
                                                            const double* __restrict__ part, int bs,
                                                            int nmax, int dim_out, int k,
                                                            float* __restrict__ dfcw,
                                                            float* __restrict__ dfcb, uint64_t* stamps) {
    WaveStamp stamp(stamps);
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx < dim_out * k) {
        double s = 0.0;
        for (int c = 0; c < RB_CHUNKS; ++c) s += part[(long long)c * dim_out * k + idx];
        dfcw[idx] = (float)s;
    }
    if (idx < dim_out) {
        double s = 0.0;
        for (int c = 0; c < RB_CHUNKS; ++c) s += part[(long long)RB_CHUNKS * dim_out * k + c * dim_out + idx];
        dfcb[idx] = (float)(s * (double)nmax);
    }
    (void)dout;
    (void)bs;
}

size_t readout_bwd_scratch_bytes(int dim_out, int k) {
    return sizeof(double) * RB_CHUNKS * dim_out * ((size_t)k + 1);
}

int launch_readout_bwd_params(const float* dout, const float* colsum, int bs, int nmax, int dim_out, int k,
                              float* dfcw, float* dfcb, void* scratch, hipStream_t s) {
    double* part = static_cast<double*>(scratch);
    HGNN_KLAUNCH(k_readout_bwd_part, dim3(ceil_div(k, 64), RB_CHUNKS), dim3(256), 0, s, dout, colsum, bs,
                 dim_out, k, part, clock_stamps((long long)ceil_div(k, 64) * RB_CHUNKS * 4));
    HGNN_LAUNCH_CHECK();
    const int n = dim_out * k > dim_out ? dim_out * k : dim_out;
    HGNN_KLAUNCH(k_readout_bwd_params, dim3(ceil_div(n, 256)), dim3(256), 0, s, dout, part, bs, nmax,
                 dim_out, k, dfcw, dfcb, clock_stamps((long long)ceil_div(n, 256) * 4));
    HGNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace hgnn
