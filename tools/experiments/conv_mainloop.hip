// Microbenchmark of the 3x3 forward-conv main loop (conv.hip conv_fwd_kernel,
// KS=3, PRO, 128x128 tile, BK=16) with parts switched off, to see which part
// keeps the MFMA pipe from saturating.  Not part of the product; results are
// garbage for the ablated variants, only the timings matter.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 conv_mainloop.hip -o conv_mainloop && ./conv_mainloop
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float floatx16 __attribute__((ext_vector_type(16)));
constexpr int NT = 256, BK = 16, BM = 128, BN = 128, KS = 3, MAXC = 256;

template <bool LOAD, bool STORE, bool SYNC, bool PRO, bool T14 = false>
__global__ void __launch_bounds__(NT, 4) k3(const float* __restrict__ x, const float* __restrict__ w,
                                            const float* __restrict__ ps, const float* __restrict__ ph, float* y,
                                            int B, int Cin, int H, int W, int Cout) {
    constexpr int TM = 2, TN = 2, ALD = BM + 2, BLD = BN + 4, A_PER = 8, B_PER = 8, T = 9;
    __shared__ float As[2][BK][ALD];
    __shared__ float Bs[2][BK][BLD];
    __shared__ float2 s_ss[MAXC];
    const int Ho = H, Wo = W, P = Ho * Wo, HWin = H * W;
    const int64_t N = (int64_t)B * P;
    const int Ktot = Cin * 9;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * (BN / 2);
    const int m0 = blockIdx.y * BM;
    const int64_t n0 = (int64_t)blockIdx.x * BN;
    for (int c = tid; c < Cin; c += NT) s_ss[c] = make_float2(ps[c], ph[c]);
    const int am = tid % BM, ak0 = (tid / BM) * A_PER;
    const int bnl = tid % BN, bk0 = tid / BN;
    const int64_t ncol = n0 + bnl;
    const int cb = (int)(ncol / P), p = (int)(ncol - (int64_t)cb * P);
    const int coh = p / Wo, cow = p - coh * Wo;
    const float* xb = x + (int64_t)cb * Cin * HWin;
    const float* wrow = w + (int64_t)(m0 + am) * Ktot;
    float ra[A_PER], rb[B_PER];
    bool b_inb = true;
    auto load = [&](int kt) {
        const float4* src = reinterpret_cast<const float4*>(wrow);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const float4 v = src[min(kt + ak0 + 4 * j, Ktot - 4) >> 2];
            ra[4 * j] = v.x; ra[4 * j + 1] = v.y; ra[4 * j + 2] = v.z; ra[4 * j + 3] = v.w;
        }
        const int kg = kt / BK, tap = kg % T, ci0 = (kg / T) * BK;
        const int kh = tap / KS, kw = tap - kh * KS;
        const int ih = coh - 1 + kh, iw = cow - 1 + kw;
        b_inb = ih >= 0 && ih < H && iw >= 0 && iw < W;
        const float* s = xb + (b_inb ? ih * W + iw : 0);
#pragma unroll
        for (int j = 0; j < B_PER; ++j) rb[j] = s[(int64_t)(ci0 + bk0 + 2 * j) * HWin];
    };
    auto store = [&](int buf, int kt) {
#pragma unroll
        for (int j = 0; j < A_PER; ++j) As[buf][ak0 + j][am] = ra[j];
        const int ci0 = ((kt / BK) / T) * BK;
#pragma unroll
        for (int j = 0; j < B_PER; ++j) {
            const int r = bk0 + 2 * j;
            float v = rb[j];
            if (PRO) { const float2 ss = s_ss[ci0 + r]; v = fmaxf(fmaf(v, ss.x, ss.y), 0.f); }
            Bs[buf][r][bnl] = b_inb ? v : 0.f;
        }
    };
    floatx16 acc[TM][TN];
    for (int i = 0; i < TM; ++i) for (int j = 0; j < TN; ++j) for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    __syncthreads();
    const int nkt = Ktot / BK;
    load(0);
    store(0, 0);
    store(1, 0);
    __syncthreads();
    const int li = lane & 31, lk = lane >> 5;
    if (T14) {
        // tile 0 is in LDS[0]; registers hold tile 1
        if (nkt > 1) load(BK);
        for (int t = 0; t < nkt; ++t) {
            const int cur = t & 1;
            if (t > 0) __syncthreads();                       // reads of t-1 done, writes of t visible
            if (t + 1 < nkt) {
                store(cur ^ 1, (t + 1) * BK);                   // tile t+1 -> LDS[(t+1)&1]
                if (t + 2 < nkt) load((t + 2) * BK);            // re-issue immediately
            }
#pragma unroll
            for (int s = 0; s < BK / 2; ++s) {
                float af[TM], bf[TN];
#pragma unroll
                for (int i = 0; i < TM; ++i) af[i] = As[cur][2 * s + lk][wm + 32 * i + li];
#pragma unroll
                for (int j = 0; j < TN; ++j) bf[j] = Bs[cur][2 * s + lk][wn + 32 * j + li];
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
            }
        }
    } else
    for (int t = 0; t < nkt; ++t) {
        const int cur = t & 1;
        if (LOAD && t + 1 < nkt) load((t + 1) * BK);
#pragma unroll
        for (int s = 0; s < BK / 2; ++s) {
            float af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = As[cur][2 * s + lk][wm + 32 * i + li];
#pragma unroll
            for (int j = 0; j < TN; ++j) bf[j] = Bs[cur][2 * s + lk][wn + 32 * j + li];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        if (t + 1 < nkt) {
            if (STORE) store(cur ^ 1, (t + 1) * BK);
            if (SYNC) __syncthreads();
        }
    }
    float s = 0.f;
    for (int i = 0; i < TM; ++i) for (int j = 0; j < TN; ++j) for (int r = 0; r < 16; ++r) s += acc[i][j][r];
    y[(int64_t)blockIdx.x * NT + tid + (int64_t)blockIdx.y * gridDim.x * NT] = s;
}

template <bool L, bool S, bool Y, bool PRO, bool T14 = false>
void run(const char* name, const float* x, const float* w, const float* ps, const float* ph, float* y) {
    const int B = 32, C = 128, H = 64;
    dim3 grid(B * H * H / BN, C / BM);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((k3<L, S, Y, PRO, T14>), grid, dim3(NT), 0, 0, x, w, ps, ph, y, B, C, H, H, C);
    hipEventRecord(e0);
    const int reps = 20;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL((k3<L, S, Y, PRO, T14>), grid, dim3(NT), 0, 0, x, w, ps, ph, y, B, C, H, H, C);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    const double fl = 2.0 * B * C * C * 9 * H * H;
    printf("%-34s %8.1f us  %6.1f TF\n", name, us, fl / us / 1e6);
}


__device__ float g_zero4[4] = {0.f, 0.f, 0.f, 0.f};

// All-glds variant: no prologue (activation materialised), weights [K][Cout].
// A: 16 rows x 512 B per K step, 2 x dwordx4 DMA per wave; B: per-lane im2col,
// 8 x dword DMA per wave (halo lanes read a zero word).
__global__ void __launch_bounds__(NT, 4) k4(const float* __restrict__ x, const float* __restrict__ wT, float* y,
                                            int B, int Cin, int H, int W, int Cout) {
    constexpr int TM = 2, TN = 2, T = 9;
    constexpr int ASZ = BK * BM, BSZ = BK * BN, BUF = ASZ + BSZ;
    __shared__ float lds[2 * BUF];
    const int P = H * W, HW = H * W;
    const int Ktot = Cin * 9;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * (BN / 2);
    const int m0 = blockIdx.y * BM;
    const int64_t n0 = (int64_t)blockIdx.x * BN;
    // B: this lane's two columns (halves h = 0, 1)
    const float* xb[2];
    int oh[2], ow[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int64_t n = n0 + h * 64 + lane;
        const int b = (int)(n / P), p = (int)(n - (int64_t)b * P);
        oh[h] = p / W;
        ow[h] = p - oh[h] * W;
        xb[h] = x + (int64_t)b * Cin * HW;
    }
    auto issue = [&](int kt, int buf) {
        float* A = lds + buf * BUF;
        float* Bb = A + ASZ;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int row = 4 * wid + 2 * j + (lane >> 5);
            const float* src = wT + (int64_t)(kt + row) * Cout + m0 + 4 * (lane & 31);
            __builtin_amdgcn_global_load_lds(src, A + (4 * wid + 2 * j) * BM, 16, 0, 0);
        }
        const int kg = kt / BK, tap = kg % T, ci0 = (kg / T) * BK;
        const int dh = tap / 3 - 1, dw = tap % 3 - 1;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int ih = oh[h] + dh, iw = ow[h] + dw;
            const bool inb = ih >= 0 && ih < H && iw >= 0 && iw < W;
            const float* base = xb[h] + ih * W + iw;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * wid + r;
                const float* src = inb ? base + (int64_t)(ci0 + row) * HW : g_zero4;
                __builtin_amdgcn_global_load_lds(src, Bb + row * BN + h * 64, 4, 0, 0);
            }
        }
    };
    floatx16 acc[TM][TN];
    for (int i = 0; i < TM; ++i) for (int j = 0; j < TN; ++j) for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const int nkt = Ktot / BK;
    issue(0, 0);
    const int li = lane & 31, lk = lane >> 5;
    for (int t = 0; t < nkt; ++t) {
        const int cur = t & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t + 1 < nkt) issue((t + 1) * BK, cur ^ 1);
        const float* A = lds + cur * BUF;
        const float* Bb = A + ASZ;
#pragma unroll
        for (int s = 0; s < BK / 2; ++s) {
            float af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = A[(2 * s + lk) * BM + wm + 32 * i + li];
#pragma unroll
            for (int j = 0; j < TN; ++j) bf[j] = Bb[(2 * s + lk) * BN + wn + 32 * j + li];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
    }
    float sum = 0.f;
    for (int i = 0; i < TM; ++i) for (int j = 0; j < TN; ++j) for (int r = 0; r < 16; ++r) sum += acc[i][j][r];
    y[(int64_t)blockIdx.x * NT + tid + (int64_t)blockIdx.y * gridDim.x * NT] = sum;
}

void run4(const char* name, const float* x, const float* w, float* y) {
    const int B = 32, C = 128, H = 64;
    dim3 grid(B * H * H / BN, C / BM);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k4, grid, dim3(NT), 0, 0, x, w, y, B, C, H, H, C);
    hipEventRecord(e0);
    const int reps = 20;
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k4, grid, dim3(NT), 0, 0, x, w, y, B, C, H, H, C);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    const double fl = 2.0 * B * C * C * 9 * H * H;
    printf("%-34s %8.1f us  %6.1f TF\n", name, us, fl / us / 1e6);
}

int main() {
    const int B = 32, C = 128, H = 64;
    float *x, *w, *ps, *ph, *y;
    hipMalloc(&x, sizeof(float) * B * C * H * H);
    hipMalloc(&w, sizeof(float) * C * C * 9);
    hipMalloc(&ps, sizeof(float) * C);
    hipMalloc(&ph, sizeof(float) * C);
    hipMalloc(&y, sizeof(float) * B * C * H * H);
    hipMemset(x, 0, sizeof(float) * B * C * H * H);
    hipMemset(w, 0, sizeof(float) * C * C * 9);
    hipMemset(ps, 0, sizeof(float) * C);
    hipMemset(ph, 0, sizeof(float) * C);
    run<true, true, true, true>("full (loads+stores+sync, PRO)", x, w, ps, ph, y);
    run<true, true, true, true, true>("T14 order, PRO", x, w, ps, ph, y);
    run4("all-glds, no PRO", x, w, y);
    run<true, true, true, false, true>("T14 order, no PRO", x, w, ps, ph, y);
    run<true, true, true, false>("full, no PRO", x, w, ps, ph, y);
    run<false, true, true, true>("no global loads", x, w, ps, ph, y);
    run<true, false, true, true>("no LDS stores", x, w, ps, ph, y);
    run<true, true, false, true>("no barrier (racy)", x, w, ps, ph, y);
    run<false, false, true, true>("LDS reads+MFMA+barrier only", x, w, ps, ph, y);
    run<false, false, false, true>("LDS reads+MFMA only", x, w, ps, ph, y);
    hipDeviceSynchronize();
    return 0;
}
