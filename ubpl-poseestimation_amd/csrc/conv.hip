// Convolutions of the stacked hourglass as implicit GEMMs on the CDNA4 matrix
// cores: the Conv wrapper (models/base/layers.py:31-50) in its three shapes —
// 1x1 stride 1 (Residual conv1/conv3/skip, features, heads, merges), 3x3
// stride 1 pad 1 (Residual conv2) and the 7x7 stride 2 pad 3 stem
// (models/pose/hourglass.py:22).
//
// GEMM view, NCHW, n = b*P + p (P = Ho*Wo, contiguous in memory):
//   forward  Y[b,m,p] = sum_k W[m,k] * X~[b,k,p] + bias[m] (+ R[b,m,p])
//            k = ci*KS*KS + kh*KS + kw, X~ = im2col of relu(x*scale + shift)
//            (the pre-activation BN+ReLU of Residual is applied while the
//            operand is staged: bn(x) is never written to HBM);
//   dgrad    = forward with the weights transposed/flipped (stride 1 only);
//   wgrad    dW[m,n] = sum_k dY[m,k] * X~[k,n] over k = (b, p), split over
//            workgroups along k into a slab, reduced deterministically; the
//            n-tile-0 workgroups also sum dY rows -> the bias gradient.
//
// Matrix core: v_mfma_f32_32x32x2_f32 (exact f32 fmaf chains, the fp32 path
// the parity tests hold to 1e-4).  Lane maps (cdna_hip_programming.md §3):
// A[i=l&31][k=l>>5], B[k=l>>5][j=l&31], C/D col = l&31,
// row = (r&3) + 8*(r>>2) + 4*(l>>5).  Block = 4 waves in a 2x2 grid; both
// operands staged k-major in LDS (As[k][m], Bs[k][n]) so a wave's fragment
// read is 32 consecutive floats per half-wave; register-staged double buffer
// (global loads of tile t+1 issued before the MFMAs of tile t).
#include "common.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int NT = 256;

// ------------------------------------------------------------------ forward
template <int BM, int BN, int BK, int KS, int ST, bool PRO, bool VECB>
struct FwdCfg {
    static constexpr int PADK = (KS - 1) / 2;
    static constexpr int TM = BM / 64, TN = BN / 64;  // 32x32 MFMA tiles per wave
    static constexpr int ALD = BM + 2, BLD = BN + 4;  // LDS row lengths (floats)
    static constexpr int A_PER = BM * BK / NT, B_PER = BK * BN / NT;
};

template <int BM, int BN, int BK, int KS, int ST, bool PRO, bool VECB>
__global__ void __launch_bounds__(NT) conv_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ bias,
                                                     const float* __restrict__ pscale,
                                                     const float* __restrict__ pshift, const float* res,
                                                     float* y, int B, int Cin, int H, int W, int Cout, int Ho,
                                                     int Wo) {
    using C = FwdCfg<BM, BN, BK, KS, ST, PRO, VECB>;
    __shared__ float As[2][BK][C::ALD];
    __shared__ float Bs[2][BK][C::BLD];

    const int P = Ho * Wo;
    const int64_t N = (int64_t)B * P;
    const int Ktot = Cin * KS * KS;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * (BN / 2);
    const int m0 = blockIdx.y * BM;
    const int64_t n0 = (int64_t)blockIdx.x * BN;

    // ---- A loader: thread owns row am, k chunk ak0 .. ak0+A_PER-1
    const int am = tid % BM;
    const int ak0 = (tid / BM) * C::A_PER;
    // ---- B loader (scalar): thread owns column bnl, rows bk0 + j*(NT/BN)
    const int bnl = tid % BN;
    const int bk0 = tid / BN;
    // ---- B loader (vector 1x1): thread owns 4 columns 4*(tid % (BN/4)), rows
    const int vn4 = tid % (BN / 4);
    const int vk0 = tid / (BN / 4);
    constexpr int VROWS = NT / (BN / 4);  // rows covered per pass

    // Column decomposition for the scalar loader (fixed per thread per tile)
    int cb = 0, coh = 0, cow = 0;
    bool cvalid;
    {
        const int64_t n = n0 + (VECB ? 4 * vn4 : bnl);
        cvalid = n < N;
        if (cvalid) {
            cb = (int)(n / P);
            const int p = (int)(n - (int64_t)cb * P);
            coh = p / Wo;
            cow = p - coh * Wo;
        }
    }

    float ra[C::A_PER];
    float rb[VECB ? 4 * (BK / VROWS) : C::B_PER];

    auto load_a = [&](int kt) {
#pragma unroll
        for (int j = 0; j < C::A_PER; ++j) {
            const int k = kt + ak0 + j;
            const int m = m0 + am;
            ra[j] = (m < Cout && k < Ktot) ? w[(int64_t)m * Ktot + k] : 0.f;
        }
    };
    auto load_b = [&](int kt) {
        if constexpr (VECB) {
            // 1x1 stride 1: X~[k][n..n+3] = x[b, k, p..p+3] (P % 4 == 0)
#pragma unroll
            for (int j = 0; j < BK / VROWS; ++j) {
                const int k = kt + vk0 + j * VROWS;
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (cvalid && k < Ktot) {
                    const int p = coh * Wo + cow;
                    v = *reinterpret_cast<const float4*>(x + ((int64_t)cb * Cin + k) * P + p);
                    if (PRO) {
                        const float sc = pscale[k], sh = pshift[k];
                        v.x = fmaxf(fmaf(v.x, sc, sh), 0.f);
                        v.y = fmaxf(fmaf(v.y, sc, sh), 0.f);
                        v.z = fmaxf(fmaf(v.z, sc, sh), 0.f);
                        v.w = fmaxf(fmaf(v.w, sc, sh), 0.f);
                    }
                }
                rb[4 * j + 0] = v.x;
                rb[4 * j + 1] = v.y;
                rb[4 * j + 2] = v.z;
                rb[4 * j + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < C::B_PER; ++j) {
                const int k = kt + bk0 + j * (NT / BN);
                float v = 0.f;
                if (cvalid && k < Ktot) {
                    const int ci = k / (KS * KS);
                    const int r = k - ci * (KS * KS);
                    const int kh = r / KS, kw = r - kh * KS;
                    const int ih = coh * ST - C::PADK + kh, iw = cow * ST - C::PADK + kw;
                    if (ih >= 0 && ih < H && iw >= 0 && iw < W) {
                        v = x[(((int64_t)cb * Cin + ci) * H + ih) * W + iw];
                        if (PRO) v = fmaxf(fmaf(v, pscale[ci], pshift[ci]), 0.f);
                    }
                }
                rb[j] = v;
            }
        }
    };
    auto store_ab = [&](int buf) {
#pragma unroll
        for (int j = 0; j < C::A_PER; ++j) As[buf][ak0 + j][am] = ra[j];
        if constexpr (VECB) {
#pragma unroll
            for (int j = 0; j < BK / VROWS; ++j)
                *reinterpret_cast<float4*>(&Bs[buf][vk0 + j * VROWS][4 * vn4]) =
                    make_float4(rb[4 * j], rb[4 * j + 1], rb[4 * j + 2], rb[4 * j + 3]);
        } else {
#pragma unroll
            for (int j = 0; j < C::B_PER; ++j) Bs[buf][bk0 + j * (NT / BN)][bnl] = rb[j];
        }
    };

    floatx16 acc[C::TM][C::TN];
#pragma unroll
    for (int i = 0; i < C::TM; ++i)
#pragma unroll
        for (int j = 0; j < C::TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nkt = (Ktot + BK - 1) / BK;
    load_a(0);
    load_b(0);
    store_ab(0);
    __syncthreads();
    const int li = lane & 31, lk = lane >> 5;
    for (int t = 0; t < nkt; ++t) {
        const int cur = t & 1;
        if (t + 1 < nkt) {
            load_a((t + 1) * BK);
            load_b((t + 1) * BK);
        }
#pragma unroll
        for (int s = 0; s < BK / 2; ++s) {
            float af[C::TM], bf[C::TN];
#pragma unroll
            for (int i = 0; i < C::TM; ++i) af[i] = As[cur][2 * s + lk][wm + 32 * i + li];
#pragma unroll
            for (int j = 0; j < C::TN; ++j) bf[j] = Bs[cur][2 * s + lk][wn + 32 * j + li];
#pragma unroll
            for (int i = 0; i < C::TM; ++i)
#pragma unroll
                for (int j = 0; j < C::TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        if (t + 1 < nkt) {
            store_ab(cur ^ 1);
            __syncthreads();
        }
    }

    // ---- epilogue: + bias (+ residual), coalesced along n
#pragma unroll
    for (int j = 0; j < C::TN; ++j) {
        const int64_t n = n0 + wn + 32 * j + li;
        if (n >= N) continue;
        const int b = (int)(n / P);
        const int p = (int)(n - (int64_t)b * P);
#pragma unroll
        for (int i = 0; i < C::TM; ++i) {
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
                if (m < Cout) {
                    const int64_t o = ((int64_t)b * Cout + m) * P + p;
                    float v = acc[i][j][r];
                    if (bias) v += bias[m];
                    if (res) v += res[o];
                    y[o] = v;
                }
            }
        }
    }
}

// ------------------------------------------------------------------ wgrad
template <int BM, int BN, int BK, int KS, int ST, bool PRO>
__global__ void __launch_bounds__(NT) conv_wgrad_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                       const float* __restrict__ pscale,
                                                       const float* __restrict__ pshift, int B, int Cin, int H,
                                                       int W, int Cout, int Ho, int Wo, int kchunk,
                                                       float* __restrict__ slab, int with_bias) {
    constexpr int PADK = (KS - 1) / 2;
    constexpr int TM = BM / 64, TN = BN / 64;
    constexpr int ALD = BM + 1, BLD = BN + 1;
    constexpr int KL = 32;                 // lanes along k in the loaders
    constexpr int RSTEP = NT / KL;         // rows per loader pass
    constexpr int A_PER = BM / RSTEP, B_PER = BN / RSTEP;
    static_assert(BK == KL, "loader assumes BK == 32");
    __shared__ float As[2][BK][ALD];
    __shared__ float Bs[2][BK][BLD];

    const int P = Ho * Wo;
    const int64_t Kall = (int64_t)B * P;
    const int Ntot = Cin * KS * KS;
    const int Nt = Ntot + 1;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * (BN / 2);
    const int m0 = blockIdx.y * BM;
    const int nb0 = blockIdx.x * BN;
    const int64_t k_begin = (int64_t)blockIdx.z * kchunk;
    const int64_t k_end = min(Kall, k_begin + kchunk);

    const int lk_ld = tid % KL;    // loader: k within tile
    const int lr_ld = tid / KL;    // loader: first row
    const bool bias_blk = with_bias && blockIdx.x == 0;

    float ra[A_PER], rb[B_PER];
    auto load = [&](int64_t kt) {
        const int64_t k = kt + lk_ld;
        const bool kv = k < k_end;
        int b = 0, p = 0, oh = 0, ow = 0;
        if (kv) {
            b = (int)(k / P);
            p = (int)(k - (int64_t)b * P);
            oh = p / Wo;
            ow = p - oh * Wo;
        }
#pragma unroll
        for (int j = 0; j < A_PER; ++j) {
            const int m = m0 + lr_ld + j * RSTEP;
            ra[j] = (kv && m < Cout) ? dy[((int64_t)b * Cout + m) * P + p] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < B_PER; ++j) {
            const int n = nb0 + lr_ld + j * RSTEP;
            float v = 0.f;
            if (kv && n < Ntot) {
                const int ci = n / (KS * KS);
                const int r = n - ci * (KS * KS);
                const int kh = r / KS, kw = r - kh * KS;
                const int ih = oh * ST - PADK + kh, iw = ow * ST - PADK + kw;
                if (ih >= 0 && ih < H && iw >= 0 && iw < W) {
                    v = x[(((int64_t)b * Cin + ci) * H + ih) * W + iw];
                    if (PRO) v = fmaxf(fmaf(v, pscale[ci], pshift[ci]), 0.f);
                }
            }
            rb[j] = v;
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int j = 0; j < A_PER; ++j) As[buf][lk_ld][lr_ld + j * RSTEP] = ra[j];
#pragma unroll
        for (int j = 0; j < B_PER; ++j) Bs[buf][lk_ld][lr_ld + j * RSTEP] = rb[j];
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    float bsum = 0.f;  // bias-gradient row sum (threads < BM of n-tile-0 blocks)

    const int nkt = (int)((k_end - k_begin + BK - 1) / BK);
    if (nkt > 0) {
        load(k_begin);
        store(0);
    }
    __syncthreads();
    const int li = lane & 31, lk = lane >> 5;
    for (int t = 0; t < nkt; ++t) {
        const int cur = t & 1;
        if (t + 1 < nkt) load(k_begin + (int64_t)(t + 1) * BK);
        if (bias_blk && tid < BM) {
#pragma unroll 8
            for (int kk = 0; kk < BK; ++kk) bsum += As[cur][kk][tid];
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
        if (t + 1 < nkt) {
            store(cur ^ 1);
            __syncthreads();
        }
    }

    float* sl = slab + (int64_t)blockIdx.z * Cout * Nt;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = nb0 + wn + 32 * j + li;
        if (n >= Ntot) continue;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
                if (m < Cout) sl[(int64_t)m * Nt + n] = acc[i][j][r];
            }
    }
    if (bias_blk && tid < BM && m0 + tid < Cout) sl[(int64_t)(m0 + tid) * Nt + Ntot] = bsum;
}

__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int Cout,
                                                          int Ntot, int with_bias, float* __restrict__ dw,
                                                          float* __restrict__ db, int accumulate) {
    const int Nt = Ntot + 1;
    const int64_t total = (int64_t)Cout * Nt;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int m = (int)(i / Nt), n = (int)(i - (int64_t)m * Nt);
        if (n == Ntot && !with_bias) continue;
        float s = 0.f;
        for (int z = 0; z < splits; ++z) s += slab[(int64_t)z * total + i];
        if (n < Ntot) {
            float* d = dw + (int64_t)m * Ntot + n;
            *d = accumulate ? *d + s : s;
        } else if (db) {
            db[m] = accumulate ? db[m] + s : s;
        }
    }
}

// wt[ci][co][kh][kw] = w[co][ci][KS-1-kh][KS-1-kw]
__global__ void weight_flip_kernel(const float* __restrict__ w, int Cout, int Cin, int KS, float* __restrict__ wt) {
    const int64_t total = (int64_t)Cout * Cin * KS * KS;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int kw = (int)(i % KS);
        int64_t t = i / KS;
        const int kh = (int)(t % KS);
        t /= KS;
        const int co = (int)(t % Cout);
        const int ci = (int)(t / Cout);
        wt[i] = w[(((int64_t)co * Cin + ci) * KS + (KS - 1 - kh)) * KS + (KS - 1 - kw)];
    }
}

template <int BM, int BN, int KS, int ST, bool PRO, bool VECB>
int launch_fwd(const float* x, const float* w, const float* bias, const float* ps, const float* sh, const float* res,
               float* y, int B, int Cin, int H, int W, int Cout, int Ho, int Wo, hipStream_t st) {
    const int64_t N = (int64_t)B * Ho * Wo;
    dim3 grid((unsigned)((N + BN - 1) / BN), (unsigned)((Cout + BM - 1) / BM));
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, 16, KS, ST, PRO, VECB>), grid, dim3(NT), 0, st, x, w, bias, ps, sh,
                       res, y, B, Cin, H, W, Cout, Ho, Wo);
    UBPL_LAUNCH_CHECK();
    return 0;
}

template <int BM, int BN, int KS, int ST, bool PRO, bool VECB>
int fwd_bm(bool big, const float* x, const float* w, const float* bias, const float* ps, const float* sh,
           const float* res, float* y, int B, int Cin, int H, int W, int Cout, int Ho, int Wo, hipStream_t st) {
    if (big) return launch_fwd<128, BN, KS, ST, PRO, VECB>(x, w, bias, ps, sh, res, y, B, Cin, H, W, Cout, Ho, Wo, st);
    return launch_fwd<64, BN, KS, ST, PRO, VECB>(x, w, bias, ps, sh, res, y, B, Cin, H, W, Cout, Ho, Wo, st);
}

template <int KS, int ST, bool PRO>
int wgrad_launch(const float* dy, const float* x, const float* ps, const float* sh, int B, int Cin, int H, int W,
                 int Cout, int Ho, int Wo, int splits, int kchunk, float* slab, int with_bias, hipStream_t st) {
    constexpr int BM = 64, BN = 64;
    const int Ntot = Cin * KS * KS;
    dim3 grid((unsigned)((Ntot + BN - 1) / BN), (unsigned)((Cout + BM - 1) / BM), (unsigned)splits);
    hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, 32, KS, ST, PRO>), grid, dim3(NT), 0, st, dy, x, ps, sh, B, Cin, H,
                       W, Cout, Ho, Wo, kchunk, slab, with_bias);
    UBPL_LAUNCH_CHECK();
    return 0;
}

void wgrad_plan(int B, int Cin, int Cout, int KS, int Ho, int Wo, int* splits, int* kchunk) {
    const int64_t K = (int64_t)B * Ho * Wo;
    const int64_t tiles = (int64_t)((Cin * KS * KS + 63) / 64) * ((Cout + 63) / 64);
    int64_t want = (1024 + tiles - 1) / tiles;            // ~1024 workgroups
    int64_t maxs = (K + 255) / 256;                       // >= 256 k per split
    if (want > maxs) want = maxs;
    if (want < 1) want = 1;
    int64_t chunk = (K + want - 1) / want;
    chunk = (chunk + 31) / 32 * 32;
    *kchunk = (int)chunk;
    *splits = (int)((K + chunk - 1) / chunk);
}

}  // namespace

// y[B,Cout,Ho,Wo] = conv(relu(x*pscale + pshift) or x, w[Cout,Cin,KS,KS], pad=(KS-1)/2) + bias (+ res).
// Supported (KS, stride): (1,1), (3,1), (7,2).  res may alias y (in-place add).
UBPL_API int ubpl_conv2d_forward(const float* x, int B, int Cin, int H, int W, const float* w, const float* bias,
                                 int Cout, int KS, int stride, const float* pscale, const float* pshift,
                                 const float* res, float* y, int Ho, int Wo, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const bool pro = pscale != nullptr;
    const bool big = Cout >= 128;
    if (KS == 1 && stride == 1) {
        const bool vec = ((Ho * Wo) % 4 == 0) && (((uintptr_t)x & 15) == 0);
        if (vec) {
            if (pro) return fwd_bm<128, 128, 1, 1, true, true>(big, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, st);
            return fwd_bm<128, 128, 1, 1, false, true>(big, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, st);
        }
        if (pro) return fwd_bm<128, 128, 1, 1, true, false>(big, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, st);
        return fwd_bm<128, 128, 1, 1, false, false>(big, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, st);
    }
    if (KS == 3 && stride == 1) {
        if (pro) return fwd_bm<128, 128, 3, 1, true, false>(big, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, st);
        return fwd_bm<128, 128, 3, 1, false, false>(big, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, st);
    }
    if (KS == 7 && stride == 2) {
        if (pro) return fwd_bm<64, 128, 7, 2, true, false>(false, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, st);
        return fwd_bm<64, 128, 7, 2, false, false>(false, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, st);
    }
    return (int)hipErrorInvalidValue;
}

// Floats of slab workspace ubpl_conv2d_wgrad needs.
UBPL_API int64_t ubpl_conv2d_wgrad_workspace(int B, int Cin, int Cout, int KS, int Ho, int Wo) {
    int splits, kchunk;
    wgrad_plan(B, Cin, Cout, KS, Ho, Wo, &splits, &kchunk);
    return (int64_t)splits * Cout * (Cin * KS * KS + 1);
}

// dw[Cout,Cin,KS,KS] (+)= sum over (b,p) dy * im2col(relu(x*pscale+pshift) or x);
// db[Cout] (+)= sum over (b,p) dy (db nullable).  slab: workspace floats.
UBPL_API int ubpl_conv2d_wgrad(const float* dy, const float* x, int B, int Cin, int H, int W, int Cout, int KS,
                               int stride, const float* pscale, const float* pshift, int Ho, int Wo, float* slab,
                               float* dw, float* db, int accumulate, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    int splits, kchunk;
    wgrad_plan(B, Cin, Cout, KS, Ho, Wo, &splits, &kchunk);
    const bool pro = pscale != nullptr;
    const int wb = db != nullptr;
    int rc;
    if (KS == 1 && stride == 1)
        rc = pro ? wgrad_launch<1, 1, true>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st)
                 : wgrad_launch<1, 1, false>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st);
    else if (KS == 3 && stride == 1)
        rc = pro ? wgrad_launch<3, 1, true>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st)
                 : wgrad_launch<3, 1, false>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st);
    else if (KS == 7 && stride == 2)
        rc = pro ? wgrad_launch<7, 2, true>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st)
                 : wgrad_launch<7, 2, false>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st);
    else
        return (int)hipErrorInvalidValue;
    if (rc) return rc;
    const int Ntot = Cin * KS * KS;
    const int64_t total = (int64_t)Cout * (Ntot + 1);
    int grid = (int)((total + 255) / 256);
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid), dim3(256), 0, st, slab, splits, Cout, Ntot, wb, dw, db,
                       accumulate);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// wt = transpose(flip(w)) so that dgrad(stride 1) = conv(dy, wt).
UBPL_API int ubpl_conv_weight_flip(const float* w, int Cout, int Cin, int KS, float* wt, void* stream) {
    const int64_t total = (int64_t)Cout * Cin * KS * KS;
    int grid = (int)((total + 255) / 256);
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(weight_flip_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, KS, wt);
    UBPL_LAUNCH_CHECK();
    return 0;
}
