// Batch plan + dense padded operators -> per-row sparse operator lists.
//
// The reference keeps every operator as a dense zero-padded tensor and walks it
// with one torch.mm per graph and slice (models/layers/layers_mnb.py:403-409,
// 426-432).  Here the dense inputs of one batch are read once, on device, and
// turned into per-row neighbour lists that the aggregation kernels walk:
//   W  (bs, Nmax, Nmax, J+2)  -> S_W (rows n) and S_WT (rows m)
//   WL (bs, Emax, Emax, J+2)  -> S_WL, S_WLT
//   Pm, Pd (bs, Nmax, Emax)   -> S_PN (node rows) and S_PE (edge rows)
// Each packed row owns a fixed slot of `cap` entries (cap = the dense row
// length) so the build is one pass with no prefix sum across graphs; a ballot
// compacts the nonzeros of each 64-column chunk.  The union of the J+2 slices
// (or of Pm and Pd) is stored once per (row, col), so one gathered feature row
// feeds every slice.
#include "kernels.h"

namespace hgnn {

__global__ void __launch_bounds__(256) k_plan(const int64_t* __restrict__ nb,
                                              const int64_t* __restrict__ eb, int bs,
                                              int nmax, int emax, BatchMeta m) {
    __shared__ int sn[256];
    __shared__ int se[256];
    __shared__ int carry[2];
    const int t = threadIdx.x;
    if (t == 0) {
        carry[0] = 0;
        carry[1] = 0;
    }
    __syncthreads();
    for (int base = 0; base < bs; base += 256) {
        const int i = base + t;
        int vn = 0, ve = 0;
        if (i < bs) {
            long long n = nb[i];
            long long e = eb ? eb[i] : 0;
            if (n < 0 || n > nmax || e < 0 || e > emax) {
                atomicOr(m.err, (uint32_t)ERR_SIZES);
                n = n < 0 ? 0 : (n > nmax ? nmax : n);
                e = e < 0 ? 0 : (e > emax ? emax : e);
            }
            vn = (int)n;
            ve = (int)e;
        }
        sn[t] = vn;
        se[t] = ve;
        __syncthreads();
        // Hillis-Steele inclusive scan (bs is small: one pass per 256 graphs)
        for (int o = 1; o < 256; o <<= 1) {
            int an = t >= o ? sn[t - o] : 0;
            int ae = t >= o ? se[t - o] : 0;
            __syncthreads();
            sn[t] += an;
            se[t] += ae;
            __syncthreads();
        }
        if (i < bs) {
            m.node_off[i] = carry[0] + sn[t] - vn;
            m.edge_off[i] = carry[1] + se[t] - ve;
        }
        __syncthreads();
        if (t == 255) {
            carry[0] += sn[255];
            carry[1] += se[255];
        }
        __syncthreads();
    }
    if (t == 0) {
        m.node_off[bs] = carry[0];
        m.edge_off[bs] = carry[1];
        m.totals[0] = carry[0];
        m.totals[1] = carry[1];
    }
}

int launch_plan(const int64_t* nb, const int64_t* eb, int bs, int nmax, int emax, BatchMeta m,
                hipStream_t s) {
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(256), 0, s, nb, eb, bs, nmax, emax, m);
    HGNN_LAUNCH_CHECK();
    return 0;
}

// One workgroup per (graph, structure kind).  NC = number of coefficients per
// entry (J+2 for W/WL, 2 for Pm/Pd).
template <int NC>
__device__ void extract_rows(int rows, int cols, int row_packed0, int col_packed0,
                             long long slot0, int cap, const float* __restrict__ s0,
                             const float* __restrict__ s1, long long rs, long long cs,
                             long long js, RowInfo* __restrict__ out_rows,
                             float* __restrict__ entries, int stride) {
    const int lane = threadIdx.x & 63;
    const int wv = threadIdx.x >> 6;
    for (int r = wv; r < rows; r += 4) {
        const long long slot = slot0 + (long long)r * cap;
        int cnt = 0;
        for (int c0 = 0; c0 < cols; c0 += 64) {
            const int c = c0 + lane;
            float v[NC];
            bool nz = false;
#pragma unroll
            for (int j = 0; j < NC; ++j) v[j] = 0.f;
            if (c < cols) {
                if (s1 == nullptr) {
                    const float* p = s0 + r * rs + c * cs;
#pragma unroll
                    for (int j = 0; j < NC; ++j) v[j] = p[j * js];
                } else {
                    v[0] = s0[r * rs + c * cs];
                    v[1] = s1[r * rs + c * cs];
                }
#pragma unroll
                for (int j = 0; j < NC; ++j) nz |= (v[j] != 0.f);
            }
            const unsigned long long mask = __ballot(nz);
            const int pos = __popcll(mask & ((1ull << lane) - 1ull));
            if (nz) {
                float* e = entries + (slot + cnt + pos) * stride;
                e[0] = __int_as_float(col_packed0 + c);
#pragma unroll
                for (int j = 0; j < NC; ++j) e[1 + j] = v[j];
            }
            cnt += __popcll(mask);
        }
        if (lane == 0) {
            RowInfo ri;
            ri.start = (int)slot;
            ri.count = cnt;
            out_rows[row_packed0 + r] = ri;
        }
    }
}

// Flags any nonzero of a dense (R, C, NC) block outside [0, rr) x [0, rc).
__device__ void validate_block(const float* __restrict__ blk, int R, int C, int NC, int rr,
                               int rc, uint32_t* err) {
    const long long total = (long long)R * C * NC;
    bool bad = false;
    for (long long i = threadIdx.x; i < total; i += blockDim.x) {
        const int r = (int)(i / ((long long)C * NC));
        const int c = (int)((i / NC) % C);
        if ((r >= rr || c >= rc) && blk[i] != 0.f) bad = true;
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(err, (uint32_t)ERR_PAD_NONZERO);
}

__device__ void validate_mask(const float* __restrict__ mask, int n, int real, uint32_t* err) {
    // mask[b, i, 0] must be 1 for i < real and 0 beyond (functions/batching.py:182-183)
    bool bad = false;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const float v = mask[(long long)i * n];
        const float want = (i < real && real > 0) ? 1.f : 0.f;
        if (v != want) bad = true;
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(err, (uint32_t)ERR_MASK);
}

template <int JT>
__global__ void __launch_bounds__(256) k_extract(ExtractArgs a) {
    const int b = blockIdx.x;
    const int kind = blockIdx.y;
    const int n0 = a.meta.node_off[b];
    const int nb = a.meta.node_off[b + 1] - n0;
    const int nmax = a.nmax;
    const long long wblk = (long long)nmax * nmax * JT;
    switch (kind) {
        case S_W: {
            const float* src = a.W + b * wblk;
            extract_rows<JT>(nb, nb, n0, n0, (long long)b * nmax * nmax, nmax, src, nullptr,
                             (long long)nmax * JT, JT, 1, a.rows[S_W], a.entries[S_W],
                             a.entry_stride_w);
            if (a.validate) {
                validate_block(src, nmax, nmax, JT, nb, nb, a.meta.err);
                validate_mask(a.mask + (long long)b * nmax * nmax, nmax, nb, a.meta.err);
            }
            break;
        }
        case S_WT: {
            const float* src = a.W + b * wblk;
            extract_rows<JT>(nb, nb, n0, n0, (long long)b * nmax * nmax, nmax, src, nullptr, JT,
                             (long long)nmax * JT, 1, a.rows[S_WT], a.entries[S_WT],
                             a.entry_stride_w);
            break;
        }
        default: {
            const int emax = a.emax;
            const int e0 = a.meta.edge_off[b];
            const int eb = a.meta.edge_off[b + 1] - e0;
            const long long lblk = (long long)emax * emax * JT;
            const long long pblk = (long long)nmax * emax;
            if (kind == S_WL) {
                const float* src = a.WL + b * lblk;
                extract_rows<JT>(eb, eb, e0, e0, (long long)b * emax * emax, emax, src, nullptr,
                                 (long long)emax * JT, JT, 1, a.rows[S_WL], a.entries[S_WL],
                                 a.entry_stride_w);
                if (a.validate) {
                    validate_block(src, emax, emax, JT, eb, eb, a.meta.err);
                    validate_mask(a.mask_lg + (long long)b * emax * emax, emax, eb, a.meta.err);
                }
            } else if (kind == S_WLT) {
                const float* src = a.WL + b * lblk;
                extract_rows<JT>(eb, eb, e0, e0, (long long)b * emax * emax, emax, src, nullptr,
                                 JT, (long long)emax * JT, 1, a.rows[S_WLT], a.entries[S_WLT],
                                 a.entry_stride_w);
            } else if (kind == S_PN) {
                const float* pm = a.Pm + b * pblk;
                const float* pd = a.Pd + b * pblk;
                extract_rows<2>(nb, eb, n0, e0, (long long)b * nmax * emax, emax, pm, pd, emax,
                                1, 0, a.rows[S_PN], a.entries[S_PN], 4);
                if (a.validate) {
                    validate_block(pm, nmax, emax, 1, nb, eb, a.meta.err);
                    validate_block(pd, nmax, emax, 1, nb, eb, a.meta.err);
                }
            } else {  // S_PE
                const float* pm = a.Pm + b * pblk;
                const float* pd = a.Pd + b * pblk;
                extract_rows<2>(eb, nb, e0, n0, (long long)b * emax * nmax, nmax, pm, pd, 1,
                                emax, 0, a.rows[S_PE], a.entries[S_PE], 4);
            }
        }
    }
}

int launch_extract(const ExtractArgs& a, hipStream_t s) {
    const dim3 grid(a.bs, a.dual ? S_COUNT : 2);
    switch (a.jtot) {
        case 3: hipLaunchKernelGGL(k_extract<3>, grid, dim3(256), 0, s, a); break;
        case 4: hipLaunchKernelGGL(k_extract<4>, grid, dim3(256), 0, s, a); break;
        case 5: hipLaunchKernelGGL(k_extract<5>, grid, dim3(256), 0, s, a); break;
        default: return 2;
    }
    HGNN_LAUNCH_CHECK();
    return 0;
}

__global__ void k_pack_nodes(const float* __restrict__ X, int f, int nmax, BatchMeta m,
                             float* __restrict__ out) {
    const int b = blockIdx.x;
    const int n0 = m.node_off[b];
    const int nb = m.node_off[b + 1] - n0;
    const float* xb = X + (long long)b * f * nmax;
    for (int i = threadIdx.x; i < nb * f; i += blockDim.x) {
        const int n = i / f, c = i % f;
        out[(long long)(n0 + n) * f + c] = xb[(long long)c * nmax + n];
    }
}

int launch_pack_nodes(const float* X, int bs, int f, int nmax, BatchMeta m, float* out,
                      hipStream_t s) {
    hipLaunchKernelGGL(k_pack_nodes, dim3(bs), dim3(128), 0, s, X, f, nmax, m, out);
    HGNN_LAUNCH_CHECK();
    return 0;
}

__global__ void k_pack_edges(const float* __restrict__ XL, int emax, BatchMeta m,
                             float* __restrict__ out) {
    const int b = blockIdx.x;
    const int e0 = m.edge_off[b];
    const int eb = m.edge_off[b + 1] - e0;
    for (int i = threadIdx.x; i < eb; i += blockDim.x) out[e0 + i] = XL[(long long)b * emax + i];
}

int launch_pack_edges(const float* XL, int bs, int emax, BatchMeta m, float* out, hipStream_t s) {
    hipLaunchKernelGGL(k_pack_edges, dim3(bs), dim3(128), 0, s, XL, emax, m, out);
    HGNN_LAUNCH_CHECK();
    return 0;
}

__global__ void k_unpack_nodes(const float* __restrict__ in, int f, int nmax, BatchMeta m,
                               float* __restrict__ X) {
    const int b = blockIdx.x;
    const int n0 = m.node_off[b];
    const int nb = m.node_off[b + 1] - n0;
    float* xb = X + (long long)b * f * nmax;
    for (int i = threadIdx.x; i < nmax * f; i += blockDim.x) {
        const int c = i / nmax, n = i % nmax;
        xb[i] = n < nb ? in[(long long)(n0 + n) * f + c] : 0.f;
    }
}

int launch_unpack_nodes(const float* in, int bs, int f, int nmax, BatchMeta m, float* X,
                        hipStream_t s) {
    hipLaunchKernelGGL(k_unpack_nodes, dim3(bs), dim3(128), 0, s, in, f, nmax, m, X);
    HGNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace hgnn
