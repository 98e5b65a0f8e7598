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
__global__ void __launch_bounds__(256) k_repack(RepackTable t) { repack_part(t, blockIdx.x, blockIdx.y); }

int launch_repack(const RepackTable& t, hipStream_t s) {
    if (t.n <= 0) return 0;
    RepackTable u = t;
    u.y = repack_y(t);
    HGNN_KLAUNCH(k_repack, dim3(u.n, u.y), dim3(256), 0, s, u);
    HGNN_LAUNCH_CHECK();
    return 0;
}

// Slab sums: SG groups of slabs per output, each summed by one thread (4 accumulators), the SG
// partials combined in order through LDS -- many slabs (the narrow-K layer-0 halves cut their rows
// into ~374 chunks) no longer mean one long serial chain per output.  Trailing blocks: the bias
// gradient of output channel o from the BN-backward tile sums (k_db_reduce's work, same order).
template <int SG>
__global__ void __launch_bounds__(256) k_dw_reduce2(const float* __restrict__ slabs, const int* r_valid,
                                                    int nz, int M, int MR, int N, int split, float* dw0,
                                                    float* dw1, const float* __restrict__ dbpart, float* db0,
                                                    float* db1) {
    constexpr int OUT = 256 / SG;
    const int nwb = (MR * N + OUT - 1) / OUT;
    if ((int)blockIdx.x >= nwb) {
        __shared__ double red[4];
        const int o = blockIdx.x - nwb;
        const int tv = ceil_div(*r_valid, 64);
        double s = 0.0;
        for (int t = threadIdx.x; t < tv; t += 256) s += (double)dbpart[(long long)t * MR + o];
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
    __shared__ float part[SG][OUT];
    const int ol = threadIdx.x % OUT, g = threadIdx.x / OUT;
    const int idx = blockIdx.x * OUT + ol;
    const int rows = *r_valid;
    const int zv = rows > 0 ? ceil_div(rows, dw3_kc(rows, nz)) : 0;  // the chunks k_gemm3_tn filled
    const long long st = (long long)M * N;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (idx < MR * N) {
        int z = g;
        for (; z + 3 * SG < zv; z += 4 * SG) {
            s0 += slabs[z * st + idx];
            s1 += slabs[(z + SG) * st + idx];
            s2 += slabs[(z + 2 * SG) * st + idx];
            s3 += slabs[(z + 3 * SG) * st + idx];
        }
        for (; z < zv; z += SG) s0 += slabs[z * st + idx];
    }
    part[g][ol] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (g == 0 && idx < MR * N) {
        float s = 0.f;
#pragma unroll
        for (int q = 0; q < SG; ++q) s += part[q][ol];
        const int o = idx / N, c = idx % N;
        if (o < split) dw0[(long long)o * N + c] = s;
        else dw1[(long long)(o - split) * N + c] = s;
    }
}

// Slab sums with float4 columns (the default when the shapes allow): a wave sums 256 consecutive outputs of its
// slab group (1 KB per slab row, coalesced), the NW waves of a block take interleaved slab groups and
// are combined in order through LDS; the bias gradients as in k_dw_reduce2.  NW = 16 for small outputs (the
// narrow layer-0 dW: 2 048 outputs, 8 blocks, each wave 64 slabs deep at NW = 4 -- a latency chain at the end
// of the backward's side stream), else 4.
template <int NW>
__global__ void __launch_bounds__(64 * NW) k_dw_reduce4(const float* __restrict__ slabs, const int* r_valid, int nz, int M,
                                                    int MR, int N, int split, float* dw0, float* dw1,
                                                    const float* __restrict__ dbpart, float* db0, float* db1,
                                                    uint64_t* stamps) {
    WaveStamp stamp(stamps);
    const int total = MR * N, nwb = (total + 255) / 256;
    if ((int)blockIdx.x >= nwb) {
        __shared__ double red[NW];
        const int o = blockIdx.x - nwb;
        const int tv = ceil_div(*r_valid, 64);
        double s = 0.0;
        for (int t = threadIdx.x; t < tv; t += 64 * NW) s += (double)dbpart[(long long)t * MR + o];
        s = wave_sum_d(s);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) {
            double t = 0.0;
            for (int q = 0; q < NW; ++q) t += red[q];
            if (o < split) db0[o] = (float)t;
            else db1[o - split] = (float)t;
        }
        return;
    }
    __shared__ float4 part[NW][64];
    const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
    const int idx = blockIdx.x * 256 + 4 * lane;  // first of this lane's four outputs (total % 4 == 0)
    const int rows = *r_valid;
    const int zv = rows > 0 ? ceil_div(rows, dw3_kc(rows, nz)) : 0;
    const long long st = (long long)M * N;
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
    if (idx < total) {
        int z = g;
        for (; z + NW < zv; z += 2 * NW) {
            const float4 a = *reinterpret_cast<const float4*>(slabs + z * st + idx);
            const float4 b = *reinterpret_cast<const float4*>(slabs + (z + NW) * st + idx);
            s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
            s1.x += b.x; s1.y += b.y; s1.z += b.z; s1.w += b.w;
        }
        for (; z < zv; z += NW) {
            const float4 a = *reinterpret_cast<const float4*>(slabs + z * st + idx);
            s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
        }
    }
    part[g][lane] = make_float4(s0.x + s1.x, s0.y + s1.y, s0.z + s1.z, s0.w + s1.w);
    __syncthreads();
    if (g == 0 && idx < total) {
        float4 t = part[0][lane];
#pragma unroll
        for (int q = 1; q < NW; ++q) {
            const float4 v = part[q][lane];
            t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
        }
        const float tv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int o = (idx + q) / N, c = (idx + q) % N;
            if (o < split) dw0[(long long)o * N + c] = tv[q];
            else dw1[(long long)(o - split) * N + c] = tv[q];
        }
    }
}

int launch_dw_reduce2(const float* slabs, const int* r_valid, int nz, int o, int o_real, int k, int split,
                      float* dw0, float* dw1, const float* dbpart, float* db0, float* db1, hipStream_t s) {
    if (o_real <= 0 || o_real > o || nz <= 0) return HGNN_ERR_ARG;
    const int total = o_real * k;
    // slab groups by the slab count: more groups when there are many slabs per output
    const int nb = dbpart ? o_real : 0;
    if (total % 4 == 0 && ((long long)o * k) % 4 == 0 && ((uintptr_t)slabs & 15) == 0) {
        const int nwb = ceil_div(total, 256);
        if (nwb <= 64)
            HGNN_KLAUNCH(k_dw_reduce4<16>, dim3(nwb + nb), dim3(1024), 0, s, slabs, r_valid, nz, o, o_real, k, split,
                         dw0, dw1, dbpart, db0, db1, clock_stamps((long long)(nwb + nb) * 16));
        else
            HGNN_KLAUNCH(k_dw_reduce4<4>, dim3(nwb + nb), dim3(256), 0, s, slabs, r_valid, nz, o, o_real, k, split,
                         dw0, dw1, dbpart, db0, db1, clock_stamps((long long)(nwb + nb) * 4));
    } else if (nz > 32) {
        HGNN_KLAUNCH(k_dw_reduce2<16>, dim3(ceil_div(total, 16) + nb), dim3(256), 0, s, slabs, r_valid, nz,
                           o, o_real, k, split, dw0, dw1, dbpart, db0, db1);
    } else {
        HGNN_KLAUNCH(k_dw_reduce2<4>, dim3(ceil_div(total, 64) + nb), dim3(256), 0, s, slabs, r_valid, nz,
                           o, o_real, k, split, dw0, dw1, dbpart, db0, db1);
    }
    HGNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace hgnn
