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
#include <type_traits>

#include "kernels.h"

namespace hgnn {

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int FBM = 64;   // output rows per block
constexpr int FCW = 16;   // input channels per chunk
constexpr int FEU = 6;    // entries per row held in registers (the rest are streamed)
constexpr unsigned OOB = 0x7ffffff0u;  // buffer-load offset past every range: reads 0

__device__ __forceinline__ float4 f4fma(float v, float4 x, float4 a) {
    return make_float4(fmaf(v, x.x, a.x), fmaf(v, x.y, a.y), fmaf(v, x.z, a.z), fmaf(v, x.w, a.w));
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p, long long bytes) {
    // descriptor inputs made provably wave-uniform (no waterfall loops around the loads)
    const unsigned long long a = reinterpret_cast<unsigned long long>(p);
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
    const unsigned n = __builtin_amdgcn_readfirstlane((unsigned)(bytes > 0x7fffffffll ? 0x7fffffffll : bytes));
    float* q = reinterpret_cast<float*>(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(q, 0, n, 0x00020000);
}

__device__ __forceinline__ float4 ld4(__amdgpu_buffer_rsrc_t r, unsigned off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
}

template <int BN, int JT, int EPI>
__global__ void __launch_bounds__(256, JT == 3 ? 2 : 1) k_fused(FusedArgs fa) {
    constexpr int KCM = JT * FCW, LDK = KCM + 4;
    constexpr int TN = BN / 2, AN = TN / 32;
    static_assert(AN >= 1 && JT >= 3, "tile");
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

    // producer thread -> (row rr, channel quad q of the 16-channel chunk)
    const int rr = tid >> 2, q = tid & 3;
    const int grow = m0 + rr;
    const bool rvalid = grow < Mv;
    const int h = lane >> 5, l31 = lane & 31;

    f32x16 acc[AN], tacc[AN];
#pragma unroll
    for (int j = 0; j < AN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

    int buf = 0;
    // one K segment: NS slices per gathered piece, cs / 16 chunks, pipelined one chunk deep
    auto run_seg = [&](auto nsc, const FusedSeg& S, int koff) {
        constexpr int NS = decltype(nsc)::value;
        constexpr int KC4 = NS * (FCW / 4);                  // float4 per B row of a chunk
        constexpr int BF4 = (BN * KC4 + 255) / 256;          // B float4 per thread
        constexpr int KH = NS * (FCW / 2);                   // half of the chunk's k range
        const auto rs_x = rsrc(S.src, S.src_bytes);
        const auto rs_b = rsrc(S.b, S.b_bytes);
        const int ld = S.ld, nch = S.cs / FCW, stride = S.list.stride;
        const bool bn = S.bn.mean != nullptr;
        // this thread's row: the first FEU entries in registers (dead slots: zero coefficients,
        // out-of-range feature offsets -> the loads return 0)
        int cnt = 0, st = 0;
        if (rvalid) {
            const RowInfo ri = S.list.rows[grow];
            cnt = ri.count;
            st = ri.start;
        }
        float4 ent[FEU];
        float2 ent2[NS > 3 ? FEU : 1];
#pragma unroll
        for (int u = 0; u < FEU; ++u) {
            ent[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (NS > 3) ent2[u] = make_float2(0.f, 0.f);
            if (u < cnt) {
                const float* e = S.list.entries + (long long)(st + u) * stride;
                ent[u] = *reinterpret_cast<const float4*>(e);
                if constexpr (NS > 3) ent2[u] = *reinterpret_cast<const float2*>(e + 4);
            }
        }
        unsigned xoff[FEU];
#pragma unroll
        for (int u = 0; u < FEU; ++u)
            xoff[u] = u < cnt ? (unsigned)((long long)__float_as_int(ent[u].x) * ld + q * 4) * 4u : OOB;
        float4 xg[FEU], rb[BF4], mu = make_float4(0.f, 0.f, 0.f, 0.f), sc = mu;
        float bnb = 0.f, bnw = 0.f;
        if (bn) {
            bnb = *S.bn.b;
            bnw = *S.bn.w;
        }
        auto load = [&](int cc) {
#pragma unroll
            for (int u = 0; u < FEU; ++u) xg[u] = ld4(rs_x, xoff[u] == OOB ? OOB : xoff[u] + cc * FCW * 4);
            if (bn) {
                mu = *reinterpret_cast<const float4*>(S.bn.mean + cc * FCW + q * 4);
                sc = *reinterpret_cast<const float4*>(S.bn.std + cc * FCW + q * 4);
            }
#pragma unroll
            for (int f = 0; f < BF4; ++f) {
                const int e = tid + f * 256;
                const int n = e / KC4, rem = e % KC4, sl = rem / (FCW / 4), cq = rem % (FCW / 4);
                const int gn = n0 + n;
                const bool ok = n < BN && gn < N && e < BN * KC4;
                const long long o = (long long)gn * S.b_n + (long long)sl * S.b_s + cc * FCW + cq * 4;
                rb[f] = ld4(rs_b, ok ? (unsigned)(o * 4) : OOB);
            }
        };
        auto store = [&](int cc, int bf) {
            float4 a[NS];
#pragma unroll
            for (int sl = 0; sl < NS; ++sl) a[sl] = make_float4(0.f, 0.f, 0.f, 0.f);
            float4 s4 = sc;
            if (bn) s4 = make_float4(bn_scale(bnw, sc.x), bn_scale(bnw, sc.y), bn_scale(bnw, sc.z), bn_scale(bnw, sc.w));
            auto bnx = [&](float4 x) {
                if (!bn) return x;
                return make_float4(bn_z_s(x.x, mu.x, s4.x, bnb), bn_z_s(x.y, mu.y, s4.y, bnb),
                                   bn_z_s(x.z, mu.z, s4.z, bnb), bn_z_s(x.w, mu.w, s4.w, bnb));
            };
            auto add = [&](const float4& e4, const float2& e2, float4 x) {
                a[0] = f4fma(e4.y, x, a[0]);
                a[1] = f4fma(e4.z, x, a[1]);
                if constexpr (NS > 2) a[2] = f4fma(e4.w, x, a[2]);
                if constexpr (NS > 3) a[3] = f4fma(e2.x, x, a[3]);
                if constexpr (NS > 4) a[4] = f4fma(e2.y, x, a[4]);
            };
#pragma unroll
            for (int u = 0; u < FEU; ++u) {
                float2 e2 = make_float2(0.f, 0.f);
                if constexpr (NS > 3) e2 = ent2[u];
                // a dead slot read 0 and has zero coefficients: BN must not turn it into b
                const float4 x = xoff[u] == OOB ? xg[u] : bnx(xg[u]);
                add(ent[u], e2, x);
            }
            // rows with more entries than registers (phantom-slot rows, high degrees): streamed
            for (int u = FEU; u < cnt; ++u) {
                const float* e = S.list.entries + (long long)(st + u) * stride;
                const float4 e4 = *reinterpret_cast<const float4*>(e);
                float2 e2 = make_float2(0.f, 0.f);
                if constexpr (NS > 3) e2 = *reinterpret_cast<const float2*>(e + 4);
                const unsigned o = (unsigned)((long long)__float_as_int(e4.x) * ld + cc * FCW + q * 4) * 4u;
                add(e4, e2, bnx(ld4(rs_x, o)));
            }
            float* as = &As[bf][rr * LDK + q * 4];
#pragma unroll
            for (int sl = 0; sl < NS; ++sl) *reinterpret_cast<float4*>(as + sl * FCW) = a[sl];
            if (EPI == FEPI_FWD && J.a_out && blockIdx.y == 0 && rvalid) {
                // the aggregate in the reference's column order (slice-major), for the dW GEMM
                float* ao = J.a_out + (long long)grow * J.lda_out + koff + cc * FCW + q * 4;
#pragma unroll
                for (int sl = 0; sl < NS; ++sl) *reinterpret_cast<float4*>(ao + (long long)sl * S.cs) = a[sl];
            }
#pragma unroll
            for (int f = 0; f < BF4; ++f) {
                const int e = tid + f * 256;
                const int n = e / KC4, rem = e % KC4, sl = rem / (FCW / 4), cq = rem % (FCW / 4);
                if (n < BN && e < BN * KC4) *reinterpret_cast<float4*>(&Bs[bf][n * LDK + sl * FCW + cq * 4]) = rb[f];
            }
        };
        auto mfma = [&](int bf) {
            const float* as = &As[bf][(wm * 32 + l31) * LDK + h * KH];
            const float* bs = &Bs[bf][(wn * TN + l31) * LDK + h * KH];
#pragma unroll
            for (int j = 0; j < AN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) tacc[j][r] = 0.f;
#pragma unroll
            for (int g = 0; g < KH / 4; ++g) {
                const float4 av = *reinterpret_cast<const float4*>(as + 4 * g);
                float4 bv[AN];
#pragma unroll
                for (int j = 0; j < AN; ++j) bv[j] = *reinterpret_cast<const float4*>(bs + j * 32 * LDK + 4 * g);
#pragma unroll
                for (int j = 0; j < AN; ++j) {
                    tacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv[j].x, tacc[j], 0, 0, 0);
                    tacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv[j].y, tacc[j], 0, 0, 0);
                    tacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv[j].z, tacc[j], 0, 0, 0);
                    tacc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv[j].w, tacc[j], 0, 0, 0);
                }
            }
#pragma unroll
            for (int j = 0; j < AN; ++j) acc[j] += tacc[j];
        };
        load(0);
        store(0, buf);
        __syncthreads();
        for (int cc = 0; cc < nch; ++cc) {
            if (cc + 1 < nch) load(cc + 1);
            mfma(buf);
            if (cc + 1 < nch) store(cc + 1, buf ^ 1);
            __syncthreads();
            buf ^= 1;
        }
    };
    using I2 = std::integral_constant<int, 2>;
    using IJ = std::integral_constant<int, JT>;
    // segment 0 is the operator list (J + 2 slices) unless this job gathers only {Pm, Pd}
    if (J.seg[0].ns == 2) run_seg(I2{}, J.seg[0], 0);
    else run_seg(IJ{}, J.seg[0], 0);
    if (J.nseg > 1) run_seg(I2{}, J.seg[1], J.seg[0].ns * J.seg[0].cs);

    // ---- epilogue.  C/D layout of the 32x32 MFMA: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
    if constexpr (EPI == FEPI_FWD) {
        if (J.a_out && blockIdx.y == 0 && rvalid) {
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
    if (s.src_bytes <= 0 || s.src_bytes > 0x7fffffffll || s.b_bytes <= 0 || s.b_bytes > 0x7fffffffll) return false;
    return true;
}

template <int BN, int JT>
int launch_bn(const FusedArgs& a, int epi, int grid_y, hipStream_t s) {
    const dim3 g(a.job[0].blocks + a.job[1].blocks, grid_y);
    if (epi == FEPI_FWD) hipLaunchKernelGGL((k_fused<BN, JT, FEPI_FWD>), g, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_fused<BN, JT, FEPI_ACC>), g, dim3(256), 0, s, a);
    HGNN_LAUNCH_CHECK();
    return 0;
}

template <int BN>
int launch_jt(const FusedArgs& a, int epi, int jt, int grid_y, hipStream_t s) {
    switch (jt) {
        case 3: return launch_bn<BN, 3>(a, epi, grid_y, s);
        case 4: return launch_bn<BN, 4>(a, epi, grid_y, s);
        case 5: return launch_bn<BN, 5>(a, epi, grid_y, s);
        default: return HGNN_ERR_UNSUPPORTED;
    }
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
    int jt = 3, nmax = 0;
    for (int i = 0; i < 2; ++i) {
        FusedJob& j = a.job[i];
        if (i == 1 && j.nseg == 0) {
            j.blocks = 0;
            continue;
        }
        if (!fused_ok(j)) return HGNN_ERR_UNSUPPORTED;
        if (epi == FEPI_FWD && (i == 1 || !j.bias)) return HGNN_ERR_ARG;
        // segment 0: the operator list (J + 2 slices) or a {Pm, Pd} list; segment 1: {Pm, Pd}
        if (j.seg[0].ns != 2) jt = j.seg[0].ns;
        if (j.nseg > 1 && j.seg[1].ns != 2) return HGNN_ERR_UNSUPPORTED;
        j.blocks = fused_blocks(j.cap_rows);
        nmax = std::max(nmax, j.n);
    }
    for (int i = 0; i < 2; ++i)
        if (a.job[i].nseg && a.job[i].seg[0].ns != 2 && a.job[i].seg[0].ns != jt) return HGNN_ERR_UNSUPPORTED;
    if (jt < 3) return HGNN_ERR_UNSUPPORTED;
    if (a.job[0].blocks + a.job[1].blocks == 0) return 0;
    // 64-column tiles up to N = 64 (d <= 32), else 128-column tiles (grid.y = ceil(N / 128))
    if (nmax <= 64) return launch_jt<64>(a, epi, jt, 1, s);
    return launch_jt<128>(a, epi, jt, ceil_div(nmax, 128), s);
}

}  // namespace hgnn
