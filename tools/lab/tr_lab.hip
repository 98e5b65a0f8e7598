// Lab: the semantics of ds_read_b64_tr_b16 as the dW GEMM uses it (row-major [k][col] LDS image with a 320-B row
// stride; an MFMA 32x32x16 operand fragment of 32 columns from two transposed reads).  Fills LDS with element value
// (k << 8) | col, reads the fragment for every lane and checks lane l got column base + (l & 31), k = 8 (l >> 5) + e.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
constexpr int ROWB = 320;  // bytes per k row (128 columns + 32 elements of padding)
__global__ void k_tr(int* out, int cbase) {
    __shared__ __attribute__((aligned(16))) char lds[16 * ROWB];
    for (int i = threadIdx.x; i < 16 * 160; i += 64) {
        const int k = i / 160, c = i % 160;
        reinterpret_cast<short*>(lds)[i] = (short)((k << 8) | c);
    }
    __syncthreads();
    const int l = threadIdx.x, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3, h = g >> 1;
    const int m0 = cbase + 16 * (g & 1);
    short r[8];
    for (int j = 0; j < 2; ++j) {
        const int k0 = 8 * h + 4 * j;
        const char* a = lds + (k0 + q) * ROWB + (m0 + 4 * p) * 2;
        v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)a);
        for (int e = 0; e < 4; ++e) r[4 * j + e] = v[e];
    }
    int bad = 0;
    for (int e = 0; e < 8; ++e) {
        const int want = ((8 * h + e) << 8) | (cbase + (l & 31));
        if (r[e] != want) ++bad;
    }
    out[l] = bad;
    if (bad && l < 8) printf("lane %d: got %x %x %x %x %x %x %x %x\n", l, r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7]);
}
int main() {
    int* d;
    hipMalloc(&d, 64 * sizeof(int));
    int tot = 0;
    for (int cb = 0; cb <= 96; cb += 32) {
        k_tr<<<1, 64>>>(d, cb);
        int h[64];
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        int b = 0;
        for (int i = 0; i < 64; ++i) b += h[i];
        printf("cbase %d: %d wrong elements\n", cb, b);
        tot += b;
    }
    printf(tot ? "TR_LAB FAIL\n" : "TR_LAB OK\n");
    return tot ? 1 : 0;
}
