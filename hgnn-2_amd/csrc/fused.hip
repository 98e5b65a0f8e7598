// Fused aggregation + 1x1-conv GEMM: the aggregate A = cat(graph_oper(W, Xg), P_multi(Pm, Xp),
// P_multi(Pd, Xp)) of a half-layer (models/layers/layers_mnb.py:266-290, 391-434) is produced
// tile by tile in LDS from the CSR row lists and consumed there by fp32 MFMAs
// (v_mfma_f32_32x32x2_f32): the [rows][K] aggregate never has to round-trip through HBM
// for the GEMM.
//
// One kernel serves two products of the same shape "gather-then-multiply":
//  * forward:   Y[r, n]  = bias[n] + sum_{s, c} A_s[r, c] Wcat[n, off_s + c]
//               A_s[r, c] = sum_{e in list(r)} v_s(e) BN(X)[col(e), c]
//    epilogue: ReLU on n >= relu_from, store Y, per-64-row-tile BN partials (count, mean, M2);
//    optionally the aggregate is also stored (the dW GEMM reads it).
//  * backward dX (the transposed aggregation reformulated, no dA buffer):
//               dX[m, c] (+)= sum_{s, o} G_s[m, o] Wcat[o, off_s + c]
//               G_s[m, o] = sum_{e in list^T(m)} v_s(e) dY[col(e), o]
//    i.e. dX = (W^T dY) Wcat_s instead of W^T (dY Wcat_s): the same sums, gathered over the
//    128-wide dY rows instead of the 640-wide dA rows.
//
// Block: 64 output rows x BN columns, 256 threads = 2 x 2 waves (32 x BN/2 each).  The K loop
// runs over chunks = (segment, 16 input channels): a chunk holds all ns slices of those 16
// channels (ns = J+2 for the operator list, 2 for {Pm, Pd}), so every gathered 64-B feature
// piece feeds all ns slices at once.  Producer thread = (row tid/4, channels 4 (tid%4) ..+3):
// its row's first FEU entries are kept in registers for the whole segment, the feature loads
// of chunk i+1 are issued before the MFMAs of chunk i and consumed after them (LDS double
// buffer, one barrier per chunk).  MFMA operand order follows gemm3.hip (k permuted inside a
// chunk identically for A and B, ds_read_b128 fragments); each chunk is summed into a fresh
// accumulator and added (fp32 chains of <= 80 terms).
#include <algorithm>

#include "kernels.h"

namespace hgnn {

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int FBM = 64;   // output rows per block
constexpr int FCW = 16;   // input channels per chunk
constexpr int FEU = 6;    // entries per row held in registers (the rest are streamed)

__device__ __forceinline__ float4 f4fma(float v, float4 x, float4 a) {
    return make_float4(fmaf(v, x.x, a.x), fmaf(v, x.y, a.y), fmaf(v, x.z, a.z), fmaf(v, x.w, a.w));
}

template <int BN, int NSM, int EPI>
__global__ void __launch_bounds__(256, 2) k_fused(FusedArgs fa) {
    constexpr int KCM = NSM * FCW, LDK = KCM + 4;
    constexpr int TN = BN / 2, AN = TN / 32;
    static_assert(AN >= 1, "tile");
    __shared__ __attribute__((aligned(16))) float As[2][FBM * LDK];
    __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDK];

    int bid = blockIdx.x;
    const bool j1 = bid >= fa.job[0].blocks;
    if (j1) bid -= fa.job[0].blocks;
    const FusedJob& J = j1 ? fa.job[1] : fa.job[0];

    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int wm = wv >> 1, wn = wv & 1;
    const int m0 = bid * FBM, n0 = blockIdx.y * BN;
    const int Mv = *J.total_rows;
    if (m0 >= Mv) return;
    const int N = J.n;
    if (n0 >= N) return;

    // ---- producer state: thread -> (row rr, channel quad q)
    const int rr = tid >> 2, q = tid & 3;
    const int grow = m0 + rr;
    const bool rvalid = grow < Mv;
    int cnt[2] = {0, 0}, st[2] = {0, 0};
    float4 ent[2][FEU];
    float2 ent2[2][NSM > 3 ? FEU : 1];
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
        if (sg < J.nseg && rvalid) {
            const RowInfo ri = J.seg[sg].list.rows[grow];
            cnt[sg] = ri.count;
            st[sg] = ri.start;
        }
#pragma unroll
        for (int u = 0; u < FEU; ++u) {
            ent[sg][u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (NSM > 3) ent2[sg][u] = make_float2(0.f, 0.f);
            if (u < cnt[sg]) {
                const float* e = J.seg[sg].list.entries + (long long)(st[sg] + u) * J.seg[sg].list.stride;
                ent[sg][u] = *reinterpret_cast<const float4*>(e);
                if constexpr (NSM > 3)
                    if (J.seg[sg].ns > 3) ent2[sg][u] = *reinterpret_cast<const float2*>(e + 4);
            }
        }
    }
    const int nch0 = J.seg[0].cs / FCW;
    const int nch = nch0 + (J.nseg > 1 ? J.seg[1].cs / FCW : 0);

    // ---- chunk staging registers
    float4 xg[FEU];     // gathered feature pieces of the chunk being prepared
    float4 mu, sc;      // BN constants of those 4 channels
    float bnb = 0.f;
    constexpr int BF4 = BN * KCM / 4 / 256;  // B float4 per thread (at the widest chunk)
    static_assert(BF4 * 256 * 4 == BN * KCM, "B staging");
    float4 rb[BF4];

    auto seg_of = [&](int i, int& cc) {
        if (i < nch0) {
            cc = i;
            return 0;
        }
        cc = i - nch0;
        return 1;
    };
    // issue the loads of chunk i (features of the cached entries, BN constants, B tile)
    auto load = [&](int i) {
        int cc;
        const int sg = seg_of(i, cc);
        const FusedSeg& S = J.seg[sg];
        const int c0 = cc * FCW + q * 4;
#pragma unroll
        for (int u = 0; u < FEU; ++u) {
            const int col = __float_as_int(ent[sg][u].x);
            xg[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (u < cnt[sg]) xg[u] = *reinterpret_cast<const float4*>(S.src + (long long)col * S.ld + c0);
        }
        if (S.bn.mean) {
            mu = *reinterpret_cast<const float4*>(S.bn.mean + c0);
            sc = *reinterpret_cast<const float4*>(S.bn.std + c0);
            bnb = *S.bn.b;
            const float w = *S.bn.w;
            sc = make_float4(bn_scale(w, sc.x), bn_scale(w, sc.y), bn_scale(w, sc.z), bn_scale(w, sc.w));
        }
        const int ns = S.ns, kc4 = ns * (FCW / 4);
#pragma unroll
        for (int f = 0; f < BF4; ++f) {
            const int e = tid + f * 256;
            const int n = e / kc4, rem = e % kc4, s = rem / (FCW / 4), cq = rem % (FCW / 4);
            const int gn = n0 + n;
            rb[f] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (n < BN && gn < N)
                rb[f] = *reinterpret_cast<const float4*>(S.b + (long long)gn * S.b_n + (long long)s * S.b_s + cc * FCW +
                                                         cq * 4);
        }
    };
    // finish chunk i into LDS buffer buf: aggregate (BN on load), entries beyond FEU streamed
    auto store = [&](int i, int buf) {
        int cc;
        const int sg = seg_of(i, cc);
        const FusedSeg& S = J.seg[sg];
        const int ns = S.ns, c0 = cc * FCW + q * 4;
        const bool bn = S.bn.mean != nullptr;
        float4 acc[NSM];
#pragma unroll
        for (int s = 0; s < NSM; ++s) acc[s] = make_float4(0.f, 0.f, 0.f, 0.f);
        auto bnx = [&](float4 x) {
            if (!bn) return x;
            return make_float4(bn_z_s(x.x, mu.x, sc.x, bnb), bn_z_s(x.y, mu.y, sc.y, bnb), bn_z_s(x.z, mu.z, sc.z, bnb),
                               bn_z_s(x.w, mu.w, sc.w, bnb));
        };
        auto add = [&](const float4& e4, const float2& e2, float4 x) {
            acc[0] = f4fma(e4.y, x, acc[0]);
            if (NSM > 1 && ns > 1) acc[1] = f4fma(e4.z, x, acc[1]);
            if (NSM > 2 && ns > 2) acc[2] = f4fma(e4.w, x, acc[2]);
            if constexpr (NSM > 3) {
                if (ns > 3) acc[3] = f4fma(e2.x, x, acc[3]);
                if (NSM > 4 && ns > 4) acc[4] = f4fma(e2.y, x, acc[4]);
            }
        };
#pragma unroll
        for (int u = 0; u < FEU; ++u) {
            if (u < cnt[sg]) {
                float2 e2 = make_float2(0.f, 0.f);
                if constexpr (NSM > 3) e2 = ent2[sg][u];
                add(ent[sg][u], e2, bnx(xg[u]));
            }
        }
        // rows with more entries than fit in registers (phantom-slot rows, SBM degrees)
        for (int u = FEU; u < cnt[sg]; ++u) {
            const float* e = S.list.entries + (long long)(st[sg] + u) * S.list.stride;
            const float4 e4 = *reinterpret_cast<const float4*>(e);
            float2 e2 = make_float2(0.f, 0.f);
            if constexpr (NSM > 3)
                if (ns > 3) e2 = *reinterpret_cast<const float2*>(e + 4);
            const float4 x = *reinterpret_cast<const float4*>(S.src + (long long)__float_as_int(e4.x) * S.ld + c0);
            add(e4, e2, bnx(x));
        }
        float* as = &As[buf][rr * LDK + q * 4];
#pragma unroll
        for (int s = 0; s < NSM; ++s)
            if (s < ns) *reinterpret_cast<float4*>(as + s * FCW) = acc[s];
        if (J.a_out && blockIdx.y == 0 && rvalid) {
            // the aggregate in the reference's column order (slice-major), for the dW GEMM
            float* ao = J.a_out + (long long)grow * J.lda_out + (sg == 0 ? 0 : J.seg[0].ns * J.seg[0].cs) + c0;
#pragma unroll
            for (int s = 0; s < NSM; ++s)
                if (s < ns) *reinterpret_cast<float4*>(ao + (long long)s * S.cs) = acc[s];
        }
        const int kc4 = ns * (FCW / 4);
#pragma unroll
        for (int f = 0; f < BF4; ++f) {
            const int e = tid + f * 256;
            const int n = e / kc4, rem = e % kc4, s = rem / (FCW / 4), cq = rem % (FCW / 4);
            if (n < BN) *reinterpret_cast<float4*>(&Bs[buf][n * LDK + s * FCW + cq * 4]) = rb[f];
        }
    };

    f32x16 acc[AN], tacc[AN];
#pragma unroll
    for (int j = 0; j < AN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

    const int h = lane >> 5, l31 = lane & 31;
    load(0);
    store(0, 0);
    __syncthreads();
    for (int t = 0; t < nch; ++t) {
        const int buf = t & 1;
        if (t + 1 < nch) load(t + 1);
        int cc;
        const int ns = J.seg[seg_of(t, cc)].ns;
        const int kh = ns * (FCW / 2);  // half of this chunk's k range
        const float* as = &As[buf][(wm * 32 + l31) * LDK + h * kh];
        const float* bs = &Bs[buf][(wn * TN + l31) * LDK + h * kh];
#pragma unroll
        for (int j = 0; j < AN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) tacc[j][r] = 0.f;
        for (int g = 0; g < kh / 4; ++g) {
            const float4 a = *reinterpret_cast<const float4*>(as + 4 * g);
            float4 b[AN];
#pragma unroll
            for (int j = 0; j < AN; ++j) b[j] = *reinterpret_cast<const float4*>(bs + j * 32 * LDK + 4 * g);
#pragma unroll
            for (int j = 0; j < AN; ++j) {
                tacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, b[j].x, tacc[j], 0, 0, 0);
                tacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, b[j].y, tacc[j], 0, 0, 0);
                tacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, b[j].z, tacc[j], 0, 0, 0);
                tacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, b[j].w, tacc[j], 0, 0, 0);
            }
        }
#pragma unroll
        for (int j = 0; j < AN; ++j) acc[j] += tacc[j];
        if (t + 1 < nch) store(t + 1, buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue.  C/D layout of the 32x32 MFMA: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    if constexpr (EPI == FEPI_FWD) {
        if (J.a_out && blockIdx.y == 0 && rvalid && tid < 4 * FBM) {
            // zero the aggregate's row padding [K, lda_out): the dW GEMM runs over the padded width
            const int kk = J.seg[0].ns * J.seg[0].cs + (J.nseg > 1 ? J.seg[1].ns * J.seg[1].cs : 0);
            if (q < J.lda_out - kk) J.a_out[(long long)grow * J.lda_out + kk + q] = 0.f;
        }
        float* red = &As[0][0];  // [2][BN] sums + [2][BN] counts, then [2][BN] M2
        float s[AN];
        int cn[AN];
#pragma unroll
        for (int j = 0; j < AN; ++j) {
            const int gn = n0 + wn * TN + j * 32 + l31;
            const float bias = gn < N ? J.bias[gn] : 0.f;
            const bool relu = gn >= J.relu_from;
            s[j] = 0.f;
            cn[j] = 0;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gm = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                float v = acc[j][r] + bias;
                if (relu) v = v < 0.f ? 0.f : v;
                acc[j][r] = v;
                if (gm < Mv) {
                    if (gn < N) J.out[(long long)gm * J.ldo + gn] = v;
                    s[j] += v;
                    ++cn[j];
                }
            }
        }
        if (J.bn_part) {
            float mean[AN];
#pragma unroll
            for (int j = 0; j < AN; ++j) {
                s[j] += __shfl_xor(s[j], 32, 64);
                cn[j] += __shfl_xor(cn[j], 32, 64);
                const int col = wn * TN + j * 32 + l31;
                if (lane < 32) {
                    red[wm * BN + col] = s[j];
                    red[2 * BN + wm * BN + col] = (float)cn[j];
                }
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < AN; ++j) {
                const int col = wn * TN + j * 32 + l31;
                const float S = red[col] + red[BN + col];
                const float C = red[2 * BN + col] + red[3 * BN + col];
                mean[j] = C > 0.f ? S / C : 0.f;
                cn[j] = (int)C;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < AN; ++j) {
                float qq = 0.f;
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int gm = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (gm < Mv) {
                        const float dl = acc[j][r] - mean[j];
                        qq = fmaf(dl, dl, qq);
                    }
                }
                qq += __shfl_xor(qq, 32, 64);
                const int col = wn * TN + j * 32 + l31;
                if (lane < 32) red[wm * BN + col] = qq;
            }
            __syncthreads();
            if (wm == 0 && lane < 32) {
#pragma unroll
                for (int j = 0; j < AN; ++j) {
                    const int col = wn * TN + j * 32 + l31;
                    const int gn = n0 + col;
                    if (gn < N) {
                        float* pp = J.bn_part + ((long long)bid * N + gn) * 3;
                        pp[0] = (float)cn[j];
                        pp[1] = mean[j];
                        pp[2] = red[col] + red[BN + col];
                    }
                }
            }
        }
    } else {
#pragma unroll
        for (int j = 0; j < AN; ++j) {
            const int gn = n0 + wn * TN + j * 32 + l31;
            if (gn >= N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int gm = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (gm < Mv) {
                    float* o = J.out + (long long)gm * J.ldo + gn;
                    *o = J.accumulate ? *o + acc[j][r] : acc[j][r];
                }
            }
        }
    }
}

bool seg_ok(const FusedSeg& s) {
    auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    if (s.cs <= 0 || s.cs % FCW != 0 || s.ns < 1 || s.ns > 5) return false;
    if (!al(s.src) || s.ld % 4 != 0 || !al(s.b) || s.b_n % 4 != 0 || s.b_s % 4 != 0) return false;
    if (s.list.stride % 4 != 0 || (s.ns > 3 && s.list.stride < 8)) return false;
    if (s.bn.mean && (!al(s.bn.mean) || !al(s.bn.std))) return false;
    return true;
}

template <int BN, int NSM>
int launch_bn(const FusedArgs& a, int epi, int grid_y, hipStream_t s) {
    const dim3 g(a.job[0].blocks + a.job[1].blocks, grid_y);
    if (epi == FEPI_FWD) hipLaunchKernelGGL((k_fused<BN, NSM, FEPI_FWD>), g, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_fused<BN, NSM, FEPI_ACC>), g, dim3(256), 0, s, a);
    HGNN_LAUNCH_CHECK();
    return 0;
}

}  // namespace

int fused_blocks(int cap_rows) { return ceil_div(cap_rows, FBM); }

bool fused_ok(const FusedJob& j) {
    if (j.nseg < 1 || j.nseg > 2 || !j.total_rows || !j.out || j.n <= 0) return false;
    for (int i = 0; i < j.nseg; ++i)
        if (!seg_ok(j.seg[i])) return false;
    if (j.a_out && (j.lda_out % 4 != 0 || (reinterpret_cast<uintptr_t>(j.a_out) & 15))) return false;
    return true;
}

int launch_fused(FusedArgs a, int epi, hipStream_t s) {
    int nsm = 0, nmax = 0;
    for (int i = 0; i < 2; ++i) {
        FusedJob& j = a.job[i];
        if (i == 1 && j.nseg == 0) {
            j.blocks = 0;
            continue;
        }
        if (!fused_ok(j)) return HGNN_ERR_UNSUPPORTED;
        if (epi == FEPI_FWD && (i == 1 || !j.bias)) return HGNN_ERR_ARG;
        j.blocks = fused_blocks(j.cap_rows);
        for (int k = 0; k < j.nseg; ++k) nsm = std::max(nsm, j.seg[k].ns);
        nmax = std::max(nmax, j.n);
    }
    if (a.job[0].blocks + a.job[1].blocks == 0) return 0;
    // 64-column tiles up to N = 64 (d <= 32), else 128-column tiles (grid.y = ceil(N / 128))
    if (nmax <= 64) return nsm <= 3 ? launch_bn<64, 3>(a, epi, 1, s) : launch_bn<64, 5>(a, epi, 1, s);
    const int gy = ceil_div(nmax, 128);
    return nsm <= 3 ? launch_bn<128, 3>(a, epi, gy, s) : launch_bn<128, 5>(a, epi, gy, s);
}

}  // namespace hgnn
