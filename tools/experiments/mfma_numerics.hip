// Probe: how v_mfma_f32_32x32x16_bf16 rounds its sum (products + C).
// Each case fills A row 0 / B column 0 (k = 0..15) and C[0][0]; prints D[0][0]
// next to the exactly-rounded (RNE) and truncated (RTZ) results.
// hipcc --offload-arch=gfx950 -O2 mfma_numerics.hip -o mfma_numerics
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

// a[16], b[16] bf16 bit patterns for row 0 / col 0; c = C[0][0]
__global__ void probe(const unsigned short* a, const unsigned short* b, float c, float* out, float* out32) {
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    bf16x8 av, bv;
    for (int j = 0; j < 8; ++j) {
        unsigned short za = 0, zb = 0;
        unsigned short ua = r == 0 ? a[8 * h + j] : za;
        unsigned short ub = r == 0 ? b[8 * h + j] : zb;
        av[j] = __builtin_bit_cast(__bf16, ua);
        bv[j] = __builtin_bit_cast(__bf16, ub);
    }
    floatx16 acc;
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    if (l == 0) acc[0] = c;   // row 0 col 0 lives in lane 0 reg 0
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
    if (l == 0) out[0] = acc[0];
    // the same sum as an f32 fmaf chain on the f32 MFMA (k order 0..15)
    floatx16 a2;
    for (int i = 0; i < 16; ++i) a2[i] = 0.f;
    if (l == 0) a2[0] = c;
    for (int k = 0; k < 16; k += 2) {
        float fa = 0.f, fb = 0.f;
        if (r == 0) {
            unsigned ua = ((unsigned)a[k + h]) << 16, ub = ((unsigned)b[k + h]) << 16;
            fa = __builtin_bit_cast(float, ua);
            fb = __builtin_bit_cast(float, ub);
        }
        a2 = __builtin_amdgcn_mfma_f32_32x32x2f32(fa, fb, a2, 0, 0, 0);
    }
    if (l == 0) out32[0] = a2[0];
}

static unsigned short bf(float f) {
    unsigned u;
    memcpy(&u, &f, 4);
    return (unsigned short)(u >> 16);   // exact for the values used here
}

static void run(const char* name, const float* av, const float* bv, float c) {
    unsigned short ha[16], hb[16];
    long double exact = c;
    for (int k = 0; k < 16; ++k) {
        ha[k] = bf(av[k]);
        hb[k] = bf(bv[k]);
        exact += (long double)av[k] * bv[k];
    }
    unsigned short *da, *db;
    float *dout, *dout32;
    hipMalloc(&da, 32);
    hipMalloc(&db, 32);
    hipMalloc(&dout, 4);
    hipMalloc(&dout32, 4);
    hipMemcpy(da, ha, 32, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, 32, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, da, db, c, dout, dout32);
    float o = 0, o32 = 0;
    hipMemcpy(&o, dout, 4, hipMemcpyDeviceToHost);
    hipMemcpy(&o32, dout32, 4, hipMemcpyDeviceToHost);
    const float rne = (float)exact;
    const float rtz = (float)(exact > 0 ? std::nextafter((float)exact, 0.f) : 0.f);
    printf("%-34s bf16-mfma %.9e  f32-chain %.9e  exact-RNE %.9e  (RTZ-ish %.9e)  exact %.12Le\n", name, o, o32, rne,
           ((long double)rne > exact && exact > 0) ? rtz : rne, exact);
    hipFree(da);
    hipFree(db);
    hipFree(dout);
    hipFree(dout32);
}

int main() {
    float a[16], b[16];
    const float u = ldexpf(1.f, -23);   // ulp(1.0)
    // 1: c = 1, one product = 0.75 ulp -> RNE 1+ulp, RTZ 1
    for (int k = 0; k < 16; ++k) a[k] = b[k] = 0.f;
    a[0] = 1.f; b[0] = 0.75f * u;
    run("c=1 + 0.75ulp", a, b, 1.f);
    // 2: c = 1, 16 products of 0.25 ulp each -> exact 1 + 4 ulp
    for (int k = 0; k < 16; ++k) { a[k] = 1.f; b[k] = 0.25f * u; }
    run("c=1 + 16 x 0.25ulp", a, b, 1.f);
    // 3: c = 1, 16 products of 0.0625 ulp -> exact 1 + 1 ulp
    for (int k = 0; k < 16; ++k) { a[k] = 1.f; b[k] = 0.0625f * u; }
    run("c=1 + 16 x 1/16ulp", a, b, 1.f);
    // 4: c = 0, big cancellation: 2^10 - 2^10 + 16 small
    for (int k = 0; k < 16; ++k) { a[k] = 1.f; b[k] = ldexpf(1.f, -20); }
    b[0] = 1024.f; b[1] = -1024.f;
    run("c=0, 1024-1024+14*2^-20", a, b, 0.f);
    // 5: c = -1, one product = -0.75 ulp (negative side)
    for (int k = 0; k < 16; ++k) a[k] = b[k] = 0.f;
    a[0] = 1.f; b[0] = -0.75f * u;
    run("c=-1 - 0.75ulp", a, b, -1.f);
    // 6: c = 1, product 0.5 ulp + tiny (tie breaker)
    for (int k = 0; k < 16; ++k) a[k] = b[k] = 0.f;
    a[0] = 1.f; b[0] = 0.5f * u; a[1] = 1.f; b[1] = ldexpf(1.f, -40);
    run("c=1 + 0.5ulp + 2^-40", a, b, 1.f);
    // 7: c = 1, product 0.5 ulp exactly (tie -> even = 1)
    for (int k = 0; k < 16; ++k) a[k] = b[k] = 0.f;
    a[0] = 1.f; b[0] = 0.5f * u;
    run("c=1 + 0.5ulp (tie)", a, b, 1.f);
    // 8: c = 1+ulp, product 0.5 ulp exactly (tie -> even = 1+2ulp)
    for (int k = 0; k < 16; ++k) a[k] = b[k] = 0.f;
    a[0] = 1.f; b[0] = 0.5f * u;
    run("c=1+ulp + 0.5ulp (tie)", a, b, 1.f + u);
    // 9: c = 2^-10, products ~1 (c small vs products)
    for (int k = 0; k < 16; ++k) { a[k] = 1.f; b[k] = 1.f + k * ldexpf(1.f, -7); }
    run("c=2^-30 + sum(1+k/128)", a, b, ldexpf(1.f, -30));
    // 10: c = 0, products 1 and 16 x 2^-26 (products below the big one's ulp)
    for (int k = 0; k < 16; ++k) { a[k] = 1.f; b[k] = ldexpf(1.f, -26); }
    b[0] = 1.f;
    run("c=0, 1 + 15 x 2^-26", a, b, 0.f);
    return 0;
}
