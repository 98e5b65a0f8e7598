// Experimental forward-GEMM variants for tools/lab/gemm_fwd_lab.hip (round 5).
//
// k_fwd_x: both operands copied global -> LDS by LDS-DMA (buffer_load ... lds, no VGPR staging, no ds_write)
// in a ring of ST stages of 32 k; A stays fp32 in LDS and each wave splits its own A fragment after the LDS read
// (v_mfma_f32_32x32x16_bf16 operand: 8 consecutive k of one row per lane = two ds_read_b128), B arrives as the
// repack's three bf16 planes.  Block 64 x BN, 4 waves of 32 x (BN / 2): a wave's A split feeds BN / 32 MFMA
// column subtiles.  Epilogue = k_gemm_bf3_fwd's (bias, ReLU, BN partials per 64-row tile).
namespace xlab {

typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4 rsrc(const void* p, unsigned bytes) {
    const unsigned long long a = (unsigned long long)(uintptr_t)p;
    i32x4 r;
    r.x = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
    r.y = __builtin_amdgcn_readfirstlane((int)(a >> 32) & 0xffff);
    r.z = __builtin_amdgcn_readfirstlane((int)bytes);
    r.w = 0x00020000;
    return r;
}

__device__ __forceinline__ void dma16(i32x4 r, unsigned voff, unsigned lds_addr) {
    int keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "buffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(r), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
        : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm_barrier() {
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

__device__ __forceinline__ void split8(const float4& x0, const float4& x1, bf16x8& p0, bf16x8& p1, bf16x8& p2) {
    const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        __bf16 a, b, c;
        split3(xv[e], a, b, c);
        p0[e] = a;
        p1[e] = b;
        p2[e] = c;
    }
}

template <int BN, int ST>
__global__ void __launch_bounds__(256) k_fwd_x(const float* __restrict__ A, int lda, const __bf16* __restrict__ B,
                                               long long pb, int ldb, const int* __restrict__ m_valid, int m_cap,
                                               int N, int K, float* __restrict__ Y, int ldy,
                                               const float* __restrict__ bias, int relu_from,
                                               float* __restrict__ bn_part) {
    constexpr int BM = 64, BK = 32, NJ = BN / 64;  // column subtiles of 32 per wave
    constexpr int A_BYTES = BM * BK * 4;            // 8 KB: rows of 128 B
    constexpr int B_PLANE = BN * BK * 2;            // rows of 64 B
    constexpr int S_BYTES = A_BYTES + 3 * B_PLANE;
    constexpr int A_INST = A_BYTES / 1024 / 4, B_INST = 3 * B_PLANE / 1024 / 4;  // DMA instructions per wave per stage
    constexpr int PER = A_INST + B_INST;
    __shared__ __attribute__((aligned(1024))) char lds[ST * S_BYTES];
    const int M = __builtin_amdgcn_readfirstlane(m_valid ? *m_valid : m_cap);
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wv >> 1, wn = wv & 1;
    const int L = blockIdx.x + gridDim.x * blockIdx.y, jj = L >> 3;
    const int by = jj % gridDim.y, bx = (L & 7) + 8 * (jj / gridDim.y);
    const int m0 = bx * BM, n0 = by * BN;
    if (m0 >= M) return;
    constexpr unsigned OOB = 0x7ffffff0u;
    const i32x4 ra = rsrc(A, (unsigned)M * lda * 4), rb = rsrc(B, (unsigned)(3 * pb * 2));
    const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
    auto issue = [&](int slot, int k0) {
        const unsigned base = lds0 + slot * S_BYTES;
#pragma unroll
        for (int i = 0; i < A_INST; ++i) {  // 8 rows of 128 B per instruction
            const int inst = wv * A_INST + i, row = inst * 8 + (lane >> 3), ps = lane & 7;
            const int ls = ps ^ ((row >> 1) & 7), gm = m0 + row, gk = k0 + 4 * ls;
            dma16(ra, (gm < M && gk < K) ? (unsigned)(gm * lda + gk) * 4u : OOB, base + inst * 1024);
        }
#pragma unroll
        for (int i = 0; i < B_INST; ++i) {  // 16 rows of 64 B per instruction; plane-major
            const int inst = wv * B_INST + i, pl = inst / (B_PLANE / 1024), pi = inst % (B_PLANE / 1024);
            const int row = pi * 16 + (lane >> 2), ps = lane & 3;
            const int ls = ps ^ ((row >> 2) & 3), gn = n0 + row, gk = k0 + 8 * ls;
            dma16(rb, (gn < N && gk < ldb) ? (unsigned)((pl * pb + (long long)gn * ldb + gk) * 2) : OOB,
                  base + A_BYTES + pl * B_PLANE + pi * 1024);
        }
    };
    f32x16 acc[NJ], tacc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    const int nt = (K + BK - 1) / BK;
    const int r31 = lane & 31, h = lane >> 5;
    const int arow = wm * 32 + r31;
#pragma unroll
    for (int s = 0; s < ST - 1; ++s)
        if (s < nt) issue(s, s * BK);
    for (int t = 0; t < nt; ++t) {
        // stage t landed (this wave's part), then every wave's part and every wave done with stage t - 1
        if (t + ST - 2 < nt) wait_vm_barrier<PER * (ST - 2)>();
        else wait_vm_barrier<0>();
        if (t + ST - 1 < nt) issue((t + ST - 1) % ST, (t + ST - 1) * BK);
        const char* st = lds + (t % ST) * S_BYTES;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) tacc[j][r] = 0.f;
#pragma unroll
        for (int s = 0; s < BK / 16; ++s) {
            const int c0 = 4 * s + 2 * h;  // logical 16-B chunk of this lane's 8 k
            const float4 x0 = *reinterpret_cast<const float4*>(st + arow * 128 + 16 * (c0 ^ ((arow >> 1) & 7)));
            const float4 x1 = *reinterpret_cast<const float4*>(st + arow * 128 + 16 * ((c0 + 1) ^ ((arow >> 1) & 7)));
            bf16x8 b[NJ][3];
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int brow = wn * (BN / 2) + j * 32 + r31, cb = 2 * s + h;
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    b[j][p] = *reinterpret_cast<const bf16x8*>(st + A_BYTES + p * B_PLANE + brow * 64 +
                                                              16 * (cb ^ ((brow >> 2) & 3)));
            }
            bf16x8 a[3];
            split8(x0, x1, a[0], a[1], a[2]);
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[j][1], tacc[j], 0, 0, 0);
                tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[j][2], tacc[j], 0, 0, 0);
                tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[j][0], tacc[j], 0, 0, 0);
                tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[j][1], tacc[j], 0, 0, 0);
                tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[j][0], tacc[j], 0, 0, 0);
                tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[j][0], tacc[j], 0, 0, 0);
            }
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[j] += tacc[j];
    }
    __syncthreads();
    // epilogue: bias, ReLU, store, BN partials (count, mean, M2) per 64-row tile, per column
    float* red = reinterpret_cast<float*>(lds);
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int col = wn * (BN / 2) + j * 32 + r31, gn = n0 + col;
        const float bv = gn < N ? bias[gn] : 0.f;
        const bool relu = gn >= relu_from;
        float sm = 0.f;
        int cnt = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int gm = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            float v = acc[j][r] + bv;
            if (relu) v = v < 0.f ? 0.f : v;
            acc[j][r] = v;
            if (gm < M) {
                if (gn < N) Y[(long long)gm * ldy + gn] = v;
                sm += v;
                ++cnt;
            }
        }
        sm += __shfl_xor(sm, 32, 64);
        cnt += __shfl_xor(cnt, 32, 64);
        if (lane < 32) {
            red[wm * BN + col] = sm;
            red[2 * BN + wm * BN + col] = (float)cnt;
        }
    }
    if (!bn_part) return;
    __syncthreads();
    float mean[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int col = wn * (BN / 2) + j * 32 + r31;
        const float S = red[col] + red[BN + col];
        const float Cn = red[2 * BN + col] + red[3 * BN + col];
        mean[j] = Cn > 0.f ? S / Cn : 0.f;
        if (wm == 0 && lane < 32 && n0 + col < N) bn_part[((long long)bx * N + n0 + col) * 3] = Cn;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int col = wn * (BN / 2) + j * 32 + r31;
        float q = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int gm = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (gm < M) {
                const float dl = acc[j][r] - mean[j];
                q = fmaf(dl, dl, q);
            }
        }
        q += __shfl_xor(q, 32, 64);
        if (lane < 32) red[wm * BN + col] = q;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int col = wn * (BN / 2) + j * 32 + r31, gn = n0 + col;
        if (wm == 0 && lane < 32 && gn < N) {
            float* pp = bn_part + ((long long)bx * N + gn) * 3;
            pp[1] = mean[j];
            pp[2] = red[col] + red[BN + col];
        }
    }
}

template <int BN, int ST>
void launch_x(const float* a, int lda, const int* mv, int m_cap, int k, const __bf16* b, long long pb, int ldb, int n,
              float* y, float* part, const float* bias) {
    const int gx = ceil_div(ceil_div(m_cap, 64), 8) * 8;
    hipLaunchKernelGGL((k_fwd_x<BN, ST>), dim3(gx, ceil_div(n, BN)), dim3(256), 0, 0, a, lda, b, pb, ldb, mv, m_cap, n,
                       k, y, n, bias, n, part);
}

}  // namespace xlab

template <typename Bench>
void exp_variants_x(Bench& bench, const float* A, int lda, const int* mv, int M, int K, const __bf16* B, long long pb,
                    int ldb, int N, float* Y, float* part, float*& zb) {
    bench("x 64x64 ST2", [&] { xlab::launch_x<64, 2>(A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb); });
    bench("x 64x64 ST3", [&] { xlab::launch_x<64, 3>(A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb); });
    bench("x 64x64 ST4", [&] { xlab::launch_x<64, 4>(A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb); });
    if (N % 128 == 0) {
        bench("x 64x128 ST2", [&] { xlab::launch_x<128, 2>(A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb); });
        bench("x 64x128 ST3", [&] { xlab::launch_x<128, 3>(A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb); });
    }
}

// ---- k_fwd_r: A fragments straight from global memory into registers (no LDS for A), B planes through an
// LDS-DMA ring.  Wave tile 32 rows x BN/WC columns; block WR x WC waves (64 * WR * WC threads), tile
// 32 WR x BN.  A is prefetched PD sub-steps (16 k each) ahead in a register ring (8 fp32 per lane per sub-step:
// the MFMA's 8 consecutive k of one row), split into the three bf16 planes right before its MFMAs.  Every
// load is issued unconditionally (out-of-range offsets return zeros through the buffer resource), so each
// stage issues the same number of vector-memory operations and the explicit vmcnt of the B ring is exact.
namespace xlab {

typedef float f32x4v __attribute__((ext_vector_type(4)));
// 16 B per lane into registers, opaque to the compiler's waitcnt pass: the kernel waits for it with its own
// counted vmcnt (the pass, not knowing the LDS-DMA ops, would otherwise wait for them too)
__device__ __forceinline__ f32x4v aload16(i32x4 r, unsigned voff) {
    f32x4v v;
    asm volatile("buffer_load_dwordx4 %0, %1, %2, 0 offen" : "=v"(v) : "v"(voff), "s"(r) : "memory");
    return v;
}

template <int WR, int WC, int BN, int PD, int ST>
__global__ void __launch_bounds__(64 * WR * WC) k_fwd_r(const float* __restrict__ A, int lda,
                                                        const __bf16* __restrict__ B, long long pb, int ldb,
                                                        const int* __restrict__ m_valid, int m_cap, int N, int K,
                                                        float* __restrict__ Y, int ldy, const float* __restrict__ bias,
                                                        int relu_from, float* __restrict__ bn_part) {
    constexpr int NW = WR * WC, BM = 32 * WR, BK = 32, NJ = BN / WC / 32;
    static_assert(NJ >= 1 && BN % (32 * WC) == 0, "wave columns");
    constexpr int B_PLANE = BN * BK * 2, S_BYTES = 3 * B_PLANE;
    constexpr int B_INST = 3 * B_PLANE / 1024;
    static_assert(B_INST % NW == 0, "B DMA split");
    constexpr int BPW = B_INST / NW;
    static_assert(PD % 2 == 0, "a stage is two sub-steps");
    __shared__ __attribute__((aligned(1024))) char lds[ST * S_BYTES > WR * 4 * BN * 4 ? ST * S_BYTES : WR * 4 * BN * 4];
    const int M = __builtin_amdgcn_readfirstlane(m_valid ? *m_valid : m_cap);
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wr = wv / WC, wc = wv % WC;
    const int L = blockIdx.x + gridDim.x * blockIdx.y, jj = L >> 3;
    const int by = jj % gridDim.y, bx = (L & 7) + 8 * (jj / gridDim.y);
    const int m0 = bx * BM, n0 = by * BN;
    if (m0 >= M) return;
    constexpr unsigned OOB = 0x7ffffff0u;
    const i32x4 ra = rsrc(A, (unsigned)M * lda * 4), rb = rsrc(B, (unsigned)(3 * pb * 2));
    const unsigned lds0 = (unsigned)(uintptr_t)(__attribute__((address_space(3))) char*)lds;
    const int r31 = lane & 31, h = lane >> 5;
    const int arow = m0 + wr * 32 + r31;
    const bool arow_ok = arow < M;
    const unsigned abase = (unsigned)arow * lda * 4;
    const int nsub = (K + 15) / 16;
    auto aload = [&](f32x4v (&x)[2], int sub) {
        const int k = sub * 16 + 8 * h;
        const bool ok = arow_ok && k < K;
        x[0] = aload16(ra, ok ? abase + k * 4 : OOB);
        x[1] = aload16(ra, ok && k + 4 < K ? abase + (k + 4) * 4 : OOB);
    };
    auto bissue = [&](int slot, int k0) {
        const unsigned base = lds0 + slot * S_BYTES;
#pragma unroll
        for (int i = 0; i < BPW; ++i) {
            const int inst = wv * BPW + i, pl = inst / (B_PLANE / 1024), pi = inst % (B_PLANE / 1024);
            const int row = pi * 16 + (lane >> 2), ps = lane & 3;
            const int ls = ps ^ ((row >> 2) & 3), gn = n0 + row, gk = k0 + 8 * ls;
            dma16(rb, (gn < N && gk < ldb) ? (unsigned)((pl * pb + (long long)gn * ldb + gk) * 2) : OOB,
                  base + pl * B_PLANE + pi * 1024);
        }
    };
    f32x16 acc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    const int nst = (nsub + 1) / 2;
    // prologue: B stages 0 .. ST-2, A sub-steps 0 .. PD-1
#pragma unroll
    for (int s = 0; s < ST - 1; ++s) bissue(s, s * BK);
    f32x4v ring[PD][2];
#pragma unroll
    for (int u = 0; u < PD; ++u) aload(ring[u], u);
    // per stage this wave issues BPW DMA + 4 A loads; B of stage s was issued ST - 1 stages ahead, and after it
    // came the A loads of PD sub-steps ... (all unconditional): younger ops at the top of stage s
    // steady state: B(s) was issued at the top of stage s - ST + 1, followed by that stage's 4 A loads and
    // ST - 2 full stages (BPW + 4 each); in the first stages more ops are younger, so the wait is conservative
    constexpr int YOUNG = 4 + (ST - 2) * (BPW + 4);
    static_assert(2 * PD >= 4 * (ST - 1) - 4 + 4, "prologue: at least YOUNG younger ops");
    // nsub % PD == 0 (the host checks): a loop without early exits keeps every ring slot in the registers it
    // was loaded into (a conditional break made the compiler copy in-flight ring registers at the back-edge)
    for (int s0 = 0; s0 < nst; s0 += PD / 2) {
#pragma unroll
        for (int us = 0; us < PD / 2; ++us) {
            const int s = s0 + us;
            asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(YOUNG) : "memory");
            bissue((s + ST - 1) % ST, (s + ST - 1) * BK);
            const char* st = lds + (s % ST) * S_BYTES;
            f32x16 tacc[NJ];
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) tacc[j][r] = 0.f;
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
                const int u = 2 * us + ss;
                bf16x8 b[NJ][3];
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    const int brow = wc * (BN / WC) + j * 32 + r31, cb = 2 * ss + h;
#pragma unroll
                    for (int p = 0; p < 3; ++p)
                        b[j][p] = *reinterpret_cast<const bf16x8*>(st + p * B_PLANE + brow * 64 +
                                                                  16 * (cb ^ ((brow >> 2) & 3)));
                }
                // A of this sub-step: younger than its two loads are the A loads of the next PD - 1 sub-steps and
                // the B DMA of the stage tops since (u / 2 + 1 of them counted: exact in the first pass, a
                // slightly early wait later)
                asm volatile("s_waitcnt vmcnt(%2)"
                             : "+v"(ring[u][0]), "+v"(ring[u][1])
                             : "n"(2 * (PD - 1) + (u / 2 + 1) * BPW)
                             : "memory");
                bf16x8 a[3];
                const f32x4v x0 = ring[u][0], x1 = ring[u][1];
                split8(make_float4(x0.x, x0.y, x0.z, x0.w), make_float4(x1.x, x1.y, x1.z, x1.w), a[0], a[1], a[2]);
                aload(ring[u], 2 * s + ss + PD);
#pragma unroll
                for (int j = 0; j < NJ; ++j) {
                    tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[j][1], tacc[j], 0, 0, 0);
                    tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[j][2], tacc[j], 0, 0, 0);
                    tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[j][0], tacc[j], 0, 0, 0);
                    tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[j][1], tacc[j], 0, 0, 0);
                    tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[j][0], tacc[j], 0, 0, 0);
                    tacc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[j][0], tacc[j], 0, 0, 0);
                }
            }
#pragma unroll
            for (int j = 0; j < NJ; ++j) acc[j] += tacc[j];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    // epilogue: bias, ReLU, store; BN partials (count, mean, M2) per 64-row tile (pairs of row waves)
    float* red = reinterpret_cast<float*>(lds);  // [WR][4][BN]: sum, count, M2 per row wave
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int col = wc * (BN / WC) + j * 32 + r31, gn = n0 + col;
        const float bv = gn < N ? bias[gn] : 0.f;
        const bool relu = gn >= relu_from;
        float sm = 0.f;
        int cnt = 0;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int gm = m0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            float v = acc[j][r] + bv;
            if (relu) v = v < 0.f ? 0.f : v;
            acc[j][r] = v;
            if (gm < M) {
                if (gn < N) Y[(long long)gm * ldy + gn] = v;
                sm += v;
                ++cnt;
            }
        }
        sm += __shfl_xor(sm, 32, 64);
        cnt += __shfl_xor(cnt, 32, 64);
        if (lane < 32) {
            red[(wr * 4 + 0) * BN + col] = sm;
            red[(wr * 4 + 1) * BN + col] = (float)cnt;
        }
    }
    if (!bn_part) return;
    __syncthreads();
    const int pair = wr & ~1;  // the 64-row tile of this row wave: row waves pair, pair + 1
    float mean[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int col = wc * (BN / WC) + j * 32 + r31;
        float S = red[(pair * 4) * BN + col], Cn = red[(pair * 4 + 1) * BN + col];
        if (pair + 1 < WR) {
            S += red[((pair + 1) * 4) * BN + col];
            Cn += red[((pair + 1) * 4 + 1) * BN + col];
        }
        mean[j] = Cn > 0.f ? S / Cn : 0.f;
        if ((wr & 1) == 0 && lane < 32 && n0 + col < N)
            bn_part[((long long)(m0 / 64 + wr / 2) * N + n0 + col) * 3] = Cn;
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int col = wc * (BN / WC) + j * 32 + r31;
        float q = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int gm = m0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
            if (gm < M) {
                const float dl = acc[j][r] - mean[j];
                q = fmaf(dl, dl, q);
            }
        }
        q += __shfl_xor(q, 32, 64);
        if (lane < 32) red[(wr * 4 + 2) * BN + col] = q;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const int col = wc * (BN / WC) + j * 32 + r31, gn = n0 + col;
        if ((wr & 1) == 0 && lane < 32 && gn < N) {
            float* pp = bn_part + ((long long)(m0 / 64 + wr / 2) * N + gn) * 3;
            pp[1] = mean[j];
            pp[2] = red[(pair * 4 + 2) * BN + col] + (pair + 1 < WR ? red[((pair + 1) * 4 + 2) * BN + col] : 0.f);
        }
    }
}

template <int WR, int WC, int BN, int PD, int ST>
void launch_r(const float* a, int lda, const int* mv, int m_cap, int k, const __bf16* b, long long pb, int ldb, int n,
              float* y, float* part, const float* bias) {
    constexpr int BM = 32 * WR;
    const int gx = ceil_div(ceil_div(m_cap, BM), 8) * 8;
    hipLaunchKernelGGL((k_fwd_r<WR, WC, BN, PD, ST>), dim3(gx, ceil_div(n, BN)), dim3(64 * WR * WC), 0, 0, a, lda, b,
                       pb, ldb, mv, m_cap, n, k, y, n, bias, n, part);
}

}  // namespace xlab

template <typename Bench>
void exp_variants_r(Bench& bench, const float* A, int lda, const int* mv, int M, int K, const __bf16* B, long long pb,
                    int ldb, int N, float* Y, float* part, const float* zb) {
    if (N % 128 || (K / 16) % 8 || K % 16) return;
    bench("r 2x1 BN128 PD4 ST2", [&] { xlab::launch_r<2, 1, 128, 4, 2>(A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb); });
    bench("r 2x1 BN128 PD8 ST3", [&] { xlab::launch_r<2, 1, 128, 8, 3>(A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb); });
    bench("r 4x1 BN128 PD4 ST2", [&] { xlab::launch_r<4, 1, 128, 4, 2>(A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb); });
    bench("r 4x1 BN128 PD8 ST3", [&] { xlab::launch_r<4, 1, 128, 8, 3>(A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb); });
    bench("r 2x2 BN128 PD4 ST2", [&] { xlab::launch_r<2, 2, 128, 4, 2>(A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb); });
    bench("r 2x2 BN128 PD8 ST3", [&] { xlab::launch_r<2, 2, 128, 8, 3>(A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb); });
}

template <typename Bench>
void exp_variants(Bench& bench, const float* A, int lda, const int* mv, int M, int K, const __bf16* B, long long pb,
                  int ldb, int N, float* Y, float* part) {
    static float* zb = nullptr;
    if (!zb) {
        hipMalloc(&zb, 4096 * 4);
        hipMemset(zb, 0, 4096 * 4);
    }
    if (getenv("LAB_X")) exp_variants_x(bench, A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb);
    exp_variants_r(bench, A, lda, mv, M, K, B, pb, ldb, N, Y, part, zb);
}
