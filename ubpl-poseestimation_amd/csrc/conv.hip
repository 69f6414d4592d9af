// Convolutions of the stacked hourglass as implicit GEMMs on the CDNA4 matrix
// cores: the Conv wrapper (models/base/layers.py:31-50) in its three shapes —
// 1x1 stride 1 (Residual conv1/conv3/skip, features, heads, merges), 3x3
// stride 1 pad 1 (Residual conv2) and the 7x7 stride 2 pad 3 stem
// (models/pose/hourglass.py:22).
//
// GEMM view, NCHW, n = b*P + p (P = Ho*Wo, contiguous in memory):
//   forward  Y[b,m,p] = sum_k W~[m,k] * X~[b,k,p] + bias[m] (+ R[b,m,p])
//            GROUPED TAP-MAJOR k = (ci/16)*16T + tap*16 + ci%16 (tap = kh*KS+kw,
//            T = KS*KS), W~ = the weights re-laid out [Cout][Cin/16][T][16]
//            (ubpl_conv_weight_tapmajor), so a K tile of BK = 16 channels
//            shares one tap (input coordinates once per tile, not per element)
//            and the T taps of one 16-channel group follow each other: the
//            re-reads of an input row stay inside the L2 working set.  X~ = im2col of
//            relu(x*scale + shift): the pre-activation BN+ReLU of Residual is
//            applied while the operand is staged (bn(x) never touches HBM;
//            scale/shift sit in LDS for the whole workgroup);
//   dgrad    = forward with the weights flipped/transposed (stride 1 only);
//   wgrad    dW[m,n] = sum_k dY[m,k] * X~[k,n] over k = (b, p), n tap-major,
//            split along k over workgroups into a slab and reduced
//            deterministically (the reduce writes the reference layout);
//            the n-tile-0 workgroups also sum dY rows = the bias gradient.
// Small grids (deep hourglass levels: 32x32 .. 4x4 planes, K = 1152) split K
// over workgroups too (slab + reduce-epilogue), so every level fills the chip.
//
// Matrix core: v_mfma_f32_32x32x2_f32 (exact f32 fmaf chains).  Lane maps
// (cdna_hip_programming.md §3): A[i=l&31][k=l>>5], B[k=l>>5][j=l&31],
// C/D col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5).  4 waves in a 2x2 grid;
// operands staged k-major in LDS (As[k][m], Bs[k][n]) so a fragment read is
// 32 consecutive floats per half-wave; register-staged double buffer with one
// barrier per K step.
#include "common.h"
#include <cstdlib>
using ubpl::conv_kgroup;
using ubpl::xcd_remap;

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int NT = 256;
constexpr int BK = 16;
constexpr int MAXC = 256;  // largest Cin with a fused BN prologue

// component-wise select (a float4 ternary can be lowered to a pointer select through scratch)
__device__ __forceinline__ float4 sel4(bool ok, float4 v) {
    return make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
}


// ------------------------------------------------------------------ forward
// TAPK: k tiles never straddle a tap (Cin % BK == 0 or KS == 1).
// AVEC: Ktot % 4 == 0 and 16-B aligned weights: float4 weight loads only.
template <int BM, int BN, int KS, int ST, bool PRO, bool VECB, bool TAPK, bool AVEC>
__global__ void __launch_bounds__(NT, 4) conv_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                     const float* __restrict__ bias,
                                                     const float* __restrict__ pscale,
                                                     const float* __restrict__ pshift, const float* res, float* y,
                                                     int B, int Cin, int H, int W, int Cout, int Ho, int Wo,
                                                     int kchunk, float* __restrict__ slab) {
    constexpr int PADK = (KS - 1) / 2;
    constexpr int TM = BM / 64, TN = BN / 64;
    constexpr int ALD = BM + 2, BLD = BN + 4;
    constexpr int A_PER = BM * BK / NT;          // 8 (BM=128) or 4 (BM=64)
    constexpr int B_PER = BK * BN / NT;          // 8
    constexpr int VROWS = NT / (BN / 4);         // vector loader rows per pass
    __shared__ float As[2][BK][ALD];
    __shared__ float Bs[2][BK][BLD];
    __shared__ float2 s_ss[PRO ? MAXC : 1];   // (scale, shift) per input channel

    const int P = Ho * Wo, HWin = H * W;
    const int64_t N = (int64_t)B * P;
    const int Ktot = Cin * KS * KS;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // (wave-uniform: SGPR)
    const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * (BN / 2);
    // XCD-aware tile order: the m tiles of one n tile, then neighbouring n
    // tiles (shared halo rows), share an L2; split-K slowest.
    const int lam = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                              gridDim.x * gridDim.y * gridDim.z);
    const int by = lam % gridDim.y, bx = (lam / gridDim.y) % gridDim.x, bz = lam / (gridDim.y * gridDim.x);
    const int m0 = by * BM;
    const int64_t n0 = (int64_t)bx * BN;
    const int k_begin = bz * kchunk;
    const int k_end = min(Ktot, k_begin + kchunk);
    constexpr int T = KS * KS;
    const int G = conv_kgroup(Cin);

    if (PRO) {
        for (int c = tid; c < Cin; c += NT) s_ss[c] = make_float2(pscale[c], pshift[c]);
    }

    // A loader: row am, k chunk ak0 .. ak0 + A_PER - 1 (vectorised when aligned)
    const int am = tid % BM;
    const int ak0 = (tid / BM) * A_PER;
    // B loader column(s)
    const int bnl = VECB ? 4 * (tid % (BN / 4)) : tid % BN;
    const int bk0 = VECB ? tid / (BN / 4) : tid / BN;
    int cb = 0, coh = 0, cow = 0;
    const int64_t ncol = n0 + bnl;
    const bool cvalid = ncol < N;
    if (cvalid) {
        cb = (int)(ncol / P);
        const int p = (int)(ncol - (int64_t)cb * P);
        coh = p / Wo;
        cow = p - coh * Wo;
    }
    const float* xb = x + (int64_t)cb * Cin * HWin;

    float ra[A_PER];
    float rb[B_PER];
    bool b_inb = false;

    // Loads are unconditional at a clamped (always valid) address and stay raw
    // in registers while the K step's MFMAs run; masks and the BN prologue are
    // applied when the values are stored to LDS.  (A load under a per-element
    // branch, or a select right after it, makes hipcc wait vmcnt(0) on the spot:
    // cdna_hip_programming.md §5 'Three .s-level traps' (c).)
    const int am_c = min(m0 + am, Cout - 1);
    const bool am_ok = m0 + am < Cout;
    const float* wrow = w + (int64_t)am_c * Ktot;
    auto load_a = [&](int kt) {
        const int k = kt + ak0;
        if constexpr (AVEC) {
            // clamped to the last aligned 4-vector; the tail is masked at store time
            const float4* src = reinterpret_cast<const float4*>(wrow);
#pragma unroll
            for (int j = 0; j < A_PER / 4; ++j) {
                const float4 v = src[min(k + 4 * j, Ktot - 4) >> 2];
                ra[4 * j] = v.x;
                ra[4 * j + 1] = v.y;
                ra[4 * j + 2] = v.z;
                ra[4 * j + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int j = 0; j < A_PER; ++j) ra[j] = wrow[min(k + j, Ktot - 1)];
        }
    };
    auto load_b = [&](int kt) {
        if constexpr (VECB) {
            // 1x1 stride 1: X~[ci][n..n+3] = x[b, ci, p..p+3] (P % 4 == 0)
            const int p = coh * Wo + cow;
#pragma unroll
            for (int j = 0; j < BK / VROWS; ++j) {
                const int kc = min(kt + bk0 + j * VROWS, Cin - 1);
                const float4 v = *reinterpret_cast<const float4*>(xb + (int64_t)kc * P + p);
                rb[4 * j] = v.x;
                rb[4 * j + 1] = v.y;
                rb[4 * j + 2] = v.z;
                rb[4 * j + 3] = v.w;
            }
        } else if constexpr (TAPK) {
            // one (channel group, tap) per K tile (G == BK): input coordinates once per tile
            const int kg = kt / BK;
            const int tap = kg % T, ci0 = (kg / T) * BK;
            const int kh = tap / KS, kw = tap - kh * KS;
            const int ih = coh * ST - PADK + kh, iw = cow * ST - PADK + kw;
            b_inb = cvalid && ih >= 0 && ih < H && iw >= 0 && iw < W;
            const float* src = xb + (b_inb ? ih * W + iw : 0);
#pragma unroll
            for (int j = 0; j < B_PER; ++j) rb[j] = src[(int64_t)min(ci0 + bk0 + j * (NT / BN), Cin - 1) * HWin];
        } else {
            // generic (stem, Cin = 3): tap and channel per element
#pragma unroll
            for (int j = 0; j < B_PER; ++j) {
                const int k = kt + bk0 + j * (NT / BN);
                float v = 0.f;
                if (cvalid && k < k_end) {
                    const int cb = k / (G * T), rem = k - cb * G * T;
                    const int tap = rem / G, ci = cb * G + (rem - (rem / G) * G);
                    const int kh = tap / KS, kw = tap - kh * KS;
                    const int ih = coh * ST - PADK + kh, iw = cow * ST - PADK + kw;
                    if (ih >= 0 && ih < H && iw >= 0 && iw < W) {
                        v = xb[(int64_t)ci * HWin + ih * W + iw];
                        if (PRO) v = fmaxf(fmaf(v, s_ss[ci].x, s_ss[ci].y), 0.f);
                    }
                }
                rb[j] = v;
            }
        }
    };
    // prologue evaluated unconditionally, then selected (a conditional LDS read
    // becomes an exec-mask branch with its own lgkmcnt wait)
    auto store_ab = [&](int buf, int kt) {
        {
            const int k = kt + ak0;
#pragma unroll
            for (int j = 0; j < A_PER; ++j) As[buf][ak0 + j][am] = (am_ok && k + j < k_end) ? ra[j] : 0.f;
        }
        if constexpr (VECB) {
#pragma unroll
            for (int j = 0; j < BK / VROWS; ++j) {
                const int k = kt + bk0 + j * VROWS;
                const bool ok = cvalid && k < k_end;
                float4 v = make_float4(rb[4 * j], rb[4 * j + 1], rb[4 * j + 2], rb[4 * j + 3]);
                if (PRO) {
                    const float2 ss = s_ss[min(k, Cin - 1)];
                    v.x = fmaxf(fmaf(v.x, ss.x, ss.y), 0.f);
                    v.y = fmaxf(fmaf(v.y, ss.x, ss.y), 0.f);
                    v.z = fmaxf(fmaf(v.z, ss.x, ss.y), 0.f);
                    v.w = fmaxf(fmaf(v.w, ss.x, ss.y), 0.f);
                }
                *reinterpret_cast<float4*>(&Bs[buf][bk0 + j * VROWS][bnl]) = sel4(ok, v);
            }
        } else if constexpr (TAPK) {
            const int ci0 = ((kt / BK) / T) * BK;
#pragma unroll
            for (int j = 0; j < B_PER; ++j) {
                const int r = bk0 + j * (NT / BN);
                const bool ok = b_inb && kt + r < k_end;
                float v = rb[j];
                if (PRO) {
                    const float2 ss = s_ss[min(ci0 + r, Cin - 1)];
                    v = fmaxf(fmaf(v, ss.x, ss.y), 0.f);
                }
                Bs[buf][r][bnl] = ok ? v : 0.f;
            }
        } else {
#pragma unroll
            for (int j = 0; j < B_PER; ++j) Bs[buf][bk0 + j * (NT / BN)][bnl] = rb[j];
        }
    };

    // Accumulators start at bias (+ residual): those loads overlap the operand
    // prologue instead of trailing the main loop, and the epilogue only stores.
    // An element is read and written by the same thread, so res may alias y.
    const int li = lane & 31, lk = lane >> 5;
    int64_t obase[TN];
    bool nok[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int64_t n = n0 + wn + 32 * j + li;
        nok[j] = n < N;
        const int64_t nc = nok[j] ? n : N - 1;
        const int b = (int)(nc / P);
        const int p = (int)(nc - (int64_t)b * P);
        obase[j] = (int64_t)b * Cout * P + p;
    }
    floatx16 acc[TM][TN];
    const bool direct = slab == nullptr;
    ubpl::seed_acc<TM, TN>(acc, direct ? bias : nullptr, direct ? res : nullptr, obase, m0 + wm, Cout, P);

    if (PRO) __syncthreads();  // s_sc / s_sh ready
    const int nkt = (k_end - k_begin + BK - 1) / BK;
    // T14 order (cdna_hip_programming.md §5 'glds vs register staging'): tile
    // t+1 is written to LDS right AFTER the barrier that ends tile t-1's reads,
    // and tile t+2's loads are issued at once, so every load has a whole K step
    // of MFMAs to land in.
    if (nkt > 0) {
        load_a(k_begin);
        load_b(k_begin);
        store_ab(0, k_begin);
    }
    if (nkt > 1) {
        load_a(k_begin + BK);
        load_b(k_begin + BK);
    }
    for (int t = 0; t < nkt; ++t) {
        const int cur = t & 1;
        __syncthreads();   // tile t visible; tile t-1's reads of buffer cur^1 done
        if (t + 1 < nkt) {
            store_ab(cur ^ 1, k_begin + (t + 1) * BK);
            if (t + 2 < nkt) {
                load_a(k_begin + (t + 2) * BK);
                load_b(k_begin + (t + 2) * BK);
            }
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

    if (slab != nullptr) {
        // split-K partial tile: slab[z][m][n]
        float* sl = slab + (int64_t)bz * Cout * N;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t n = n0 + wn + 32 * j + li;
            if (n >= N) continue;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
                    if (m < Cout) sl[(int64_t)m * N + n] = acc[i][j][r];
                }
        }
        return;
    }
    // ---- epilogue: stores, coalesced along n (bias / residual are in acc)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        if (!nok[j]) continue;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
                if (m < Cout) y[obase[j] + (int64_t)m * P] = acc[i][j][r];
            }
    }
}

// ------------------------------------------------------------------ 1x1, LDS-DMA fed
// 1x1 stride-1 conv as Y[m, n] = sum_k Wk[k][m] * X[b, k, p] (n = b*P + p)
// with the weights k-major ([Cin][Cout]: the data-gradient re-layout of a 1x1
// conv, or the reference layout itself for a data gradient).  Both operand
// tiles are k-rows of contiguous floats — BN (128) pixels of one input channel
// (NCHW as it lies) and BM output channels — so they go global -> LDS by
// LDS-DMA (global_load_lds_dwordx4, 1 KB per wave instruction), no staging
// registers.  The fused pre-activation relu(x*scale + shift) is applied to the
// B fragment after its LDS read (2 VALU per 2 MFMAs).  3-stage ring with
// counted vmcnt and a raw s_barrier, as conv_split.hip's conv_psa_kernel.
// Fragment reads are ds_read_b32 of 32 consecutive floats per half-wave
// (conflict-free, no swizzle).
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int BM, bool PRO>
__global__ void __launch_bounds__(NT, 2) conv1x1_dma_kernel(const float* __restrict__ x, const float* __restrict__ wk,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ pscale,
                                                          const float* __restrict__ pshift, const float* res,
                                                          float* y, int B, int K, int P, int M, int kchunk,
                                                          float* __restrict__ slab, float* __restrict__ stat_part) {
    constexpr int BN1 = 128;
    constexpr int TM = BM / 64, TN = BN1 / 64;
    constexpr int NS = 3;
    constexpr int AB = BK * BM * 4, BB = BK * BN1 * 4;       // bytes per stage
    constexpr int A_INS = AB / 1024, B_INS = BB / 1024;     // DMA instructions per stage
    constexpr int A_PW = A_INS / 4, B_PW = B_INS / 4;       // per wave
    constexpr int A_RPI = 1024 / (BM * 4);                  // rows per A instruction
    __shared__ __attribute__((aligned(16))) char lds[NS * (AB + BB)];

    const int64_t N = (int64_t)B * P;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // (wave-uniform: SGPR)
    const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * (BN1 / 2);
    const int lam = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                              gridDim.x * gridDim.y * gridDim.z);
    const int by = lam % gridDim.y, bx = (lam / gridDim.y) % gridDim.x, bz = lam / (gridDim.y * gridDim.x);
    const int m0 = by * BM;
    const int64_t n0 = (int64_t)bx * BN1;
    const int k_begin = bz * kchunk;
    const int k_end = min(K, k_begin + kchunk);

    // DMA sources (per lane, k-independent part).  A instruction q (of A_INS)
    // covers k rows q*A_RPI .. +A_RPI-1; lane L: row q*A_RPI + L / (BM/4),
    // columns 4*(L % (BM/4)) .. +3.  B instruction q: rows 2q, 2q+1; lane L:
    // row 2q + (L >> 5), pixels 4*(L & 31) .. +3 of the tile.
    const int a_row = lane / (BM / 4);
    const int a_col = min(m0 + 4 * (lane % (BM / 4)), M - 4);
    const int b_row = lane >> 5;
    // per-lane 32-bit byte offsets over wave-uniform bases (scalar + vector
    // addressing).  K % 16 == 0 (checked by the entry point): every DMA row is
    // a real k row.
    const uint32_t a_lane = (uint32_t)((a_row * M + a_col) * 4);
    uint32_t b_lane;
    {
        int64_t n = n0 + 4 * (lane & 31);
        n = n < N ? n : N - 4;
        const int64_t b = n / P;
        b_lane = (uint32_t)((b * K * P + (n - b * P) + (int64_t)b_row * P) * 4);
    }
    auto stage = [&](int buf, int kt) {
        char* base = lds + buf * (AB + BB);
#pragma unroll
        for (int i = 0; i < A_PW; ++i) {
            const int q = wid * A_PW + i;
            const int k0 = min(kt + q * A_RPI, K - A_RPI);
            const char* ab = reinterpret_cast<const char*>(wk + (int64_t)k0 * M);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(ab + a_lane), (lds_ptr_t)(base + q * 1024), 16, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < B_PW; ++i) {
            const int q = wid * B_PW + i;
            const int k0 = min(kt + 2 * q, K - 2);
            const char* bb = reinterpret_cast<const char*>(x + (int64_t)k0 * P);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bb + b_lane), (lds_ptr_t)(base + AB + q * 1024), 16, 0, 0);
        }
    };

    // accumulators start at bias (+ residual), as conv_fwd_kernel
    const int li = lane & 31, lk = lane >> 5;
    int64_t obase[TN];
    bool nok[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int64_t n = n0 + wn + 32 * j + li;
        nok[j] = n < N;
        const int64_t nc = nok[j] ? n : N - 1;
        const int b = (int)(nc / P);
        const int p = (int)(nc - (int64_t)b * P);
        obase[j] = (int64_t)b * M * P + p;
    }
    floatx16 acc[TM][TN];
    const bool direct = slab == nullptr;
    ubpl::seed_acc<TM, TN>(acc, direct ? bias : nullptr, direct ? res : nullptr, obase, m0 + wm, M, P);

    const int nkt = (k_end - k_begin + BK - 1) / BK;
    if (nkt > 0) stage(0, k_begin);
    if (nkt > 1) stage(1, k_begin + BK);
    for (int t = 0; t < nkt; ++t) {
        if (t + 1 < nkt) vm_wait<A_PW + B_PW>();
        else vm_wait<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (t + 2 < nkt) stage((t + 2) % NS, k_begin + (t + 2) * BK);
        const int kt = k_begin + t * BK;
        const float* As = reinterpret_cast<const float*>(lds + (t % NS) * (AB + BB));
        const float* Bs = reinterpret_cast<const float*>(lds + (t % NS) * (AB + BB) + AB);
        // the K step's 16 (scale, shift) pairs by scalar loads (kt is uniform;
        // an LDS table would alias the DMA images and cost a vmcnt(0) per step)
        float scs[BK], shs[BK];
        if (PRO) {
            const int kb = __builtin_amdgcn_readfirstlane(min(kt, K - BK));
#pragma unroll
            for (int q = 0; q < BK; ++q) {
                scs[q] = pscale[kb + q];
                shs[q] = pshift[kb + q];
            }
        }
#pragma unroll
        for (int s = 0; s < BK / 2; ++s) {
            const int kr = 2 * s + lk;
            const bool kok = kt + kr < k_end;        // K tail: zero the B fragment
            float af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = As[kr * BM + wm + 32 * i + li];
            float sc = 1.f, sh = 0.f;
            if (PRO) {
                sc = lk ? scs[2 * s + 1] : scs[2 * s];
                sh = lk ? shs[2 * s + 1] : shs[2 * s];
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                float v = Bs[kr * BN1 + wn + 32 * j + li];
                if (PRO) v = fmaxf(fmaf(v, sc, sh), 0.f);
                bf[j] = kok ? v : 0.f;
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    if (slab != nullptr) {
        float* sl = slab + (int64_t)bz * M * N;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t n = n0 + wn + 32 * j + li;
            if (n >= N) continue;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
                    if (m < M) sl[(int64_t)m * N + n] = acc[i][j][r];
                }
        }
        return;
    }
    if (stat_part) ubpl::tile_bn_partials<TM, TN>(acc, nok, m0 + wm, M, n0 + wn, N, stat_part);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        if (!nok[j]) continue;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * lk;
                if (m < M) y[obase[j] + (int64_t)m * P] = acc[i][j][r];
            }
    }
}

// y[b,m,p] = sum_z slab[z][m][b*P+p] + bias[m] (+ res)
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ slab, int splits, int Cout,
                                                           int P, int64_t N, const float* __restrict__ bias,
                                                           const float* res, float* y) {
    const int64_t total = (int64_t)Cout * N;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        // i enumerates the output in NCHW order: i = (b*Cout + m)*P + p
        const int p = (int)(i % P);
        const int64_t t = i / P;
        const int m = (int)(t % Cout);
        const int64_t b = t / Cout;
        const int64_t n = b * P + p;
        float s = 0.f;
        for (int z = 0; z < splits; ++z) s += slab[((int64_t)z * Cout + m) * N + n];
        if (bias) s += bias[m];
        if (res) s += res[i];
        y[i] = s;
    }
}

// ------------------------------------------------------------------ wgrad
// n tap-major: n = tap*Cin + ci; TAPN: a BN-wide n tile lies in one tap.
template <int BM, int BN, int KS, int ST, bool PRO, bool TAPN>
__global__ void __launch_bounds__(NT) conv_wgrad_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                       const float* __restrict__ pscale,
                                                       const float* __restrict__ pshift, int B, int Cin, int H,
                                                       int W, int Cout, int Ho, int Wo, int kchunk,
                                                       float* __restrict__ slab, int with_bias) {
    constexpr int PADK = (KS - 1) / 2;
    constexpr int TM = BM / 64, TN = BN / 64;
    constexpr int WBK = 32;
    constexpr int ALD = BM + 1, BLD = BN + 1;
    constexpr int RSTEP = NT / WBK;
    constexpr int A_PER = BM / RSTEP, B_PER = BN / RSTEP;
    __shared__ float As[2][WBK][ALD];
    __shared__ float Bs[2][WBK][BLD];
    __shared__ float s_sc[PRO ? MAXC : 1], s_sh[PRO ? MAXC : 1];

    const int P = Ho * Wo, HWin = H * W;
    const int64_t Kall = (int64_t)B * P;
    const int Ntot = Cin * KS * KS;
    const int Nt = Ntot + 1;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // (wave-uniform: SGPR)
    const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * (BN / 2);
    const int m0 = blockIdx.y * BM;
    const int nb0 = blockIdx.x * BN;
    const int64_t k_begin = (int64_t)blockIdx.z * kchunk;
    const int64_t k_end = min(Kall, k_begin + kchunk);
    const int lk_ld = tid % WBK;
    const int lr_ld = tid / WBK;
    const bool bias_blk = with_bias && blockIdx.x == 0;
    // tap of this workgroup's n tile (TAPN)
    const int tap_blk = nb0 / Cin, ci_blk = nb0 - tap_blk * Cin;
    const int kh_blk = tap_blk / KS, kw_blk = tap_blk - kh_blk * KS;

    if (PRO) {
        for (int c = tid; c < Cin; c += NT) {
            s_sc[c] = pscale[c];
            s_sh[c] = pshift[c];
        }
        __syncthreads();
    }

    float ra[A_PER], rb[B_PER];
    auto load = [&](int64_t kt) {
        const int64_t k = kt + lk_ld;
        const bool kv = k < k_end;
        const int64_t kc = kv ? k : k_begin;        // clamped, always valid
        const int b = (int)(kc / P);
        const int p = (int)(kc - (int64_t)b * P);
        const int oh = p / Wo, ow = p - oh * Wo;
        const float* dyb = dy + (int64_t)b * Cout * P + p;
#pragma unroll
        for (int j = 0; j < A_PER; ++j) {
            const int m = m0 + lr_ld + j * RSTEP;
            const float v = dyb[(int64_t)min(m, Cout - 1) * P];
            ra[j] = (kv && m < Cout) ? v : 0.f;
        }
        const float* xb = x + (int64_t)b * Cin * HWin;
        if constexpr (TAPN) {
            const int ih = oh * ST - PADK + kh_blk, iw = ow * ST - PADK + kw_blk;
            const bool inb = kv && ih >= 0 && ih < H && iw >= 0 && iw < W;
            const float* src = xb + (inb ? ih * W + iw : 0);
#pragma unroll
            for (int j = 0; j < B_PER; ++j) {
                const int r = lr_ld + j * RSTEP;
                const bool ok = inb && nb0 + r < Ntot;
                const int ci = min(ci_blk + r, Cin - 1);
                float v = src[(int64_t)ci * HWin];
                if (PRO) v = fmaxf(fmaf(v, s_sc[ci], s_sh[ci]), 0.f);
                rb[j] = ok ? v : 0.f;
            }
        } else {
#pragma unroll
            for (int j = 0; j < B_PER; ++j) {
                const int n = nb0 + lr_ld + j * RSTEP;
                float v = 0.f;
                if (kv && n < Ntot) {
                    const int tap = n / Cin, ci = n - tap * Cin;
                    const int kh = tap / KS, kw = tap - kh * KS;
                    const int ih = oh * ST - PADK + kh, iw = ow * ST - PADK + kw;
                    if (ih >= 0 && ih < H && iw >= 0 && iw < W) {
                        v = xb[(int64_t)ci * HWin + ih * W + iw];
                        if (PRO) v = fmaxf(fmaf(v, s_sc[ci], s_sh[ci]), 0.f);
                    }
                }
                rb[j] = v;
            }
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
    float bsum = 0.f;

    const int nkt = (int)((k_end - k_begin + WBK - 1) / WBK);
    if (nkt > 0) {
        load(k_begin);
        store(0);
    }
    __syncthreads();
    const int li = lane & 31, lk = lane >> 5;
    for (int t = 0; t < nkt; ++t) {
        const int cur = t & 1;
        if (t + 1 < nkt) load(k_begin + (int64_t)(t + 1) * WBK);
        if (bias_blk && tid < BM) {
#pragma unroll 8
            for (int kk = 0; kk < WBK; ++kk) bsum += As[cur][kk][tid];
        }
#pragma unroll
        for (int s = 0; s < WBK / 2; ++s) {
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

// ------------------------------------------------------------------ wgrad v2
// Both operands run along k = b*P + p in memory (dY[b][m][p], x[b][ci][p']),
// so they are staged k-contiguous: float4 global loads, As[m][16] / Bs[n][16]
// (64-B rows of four 16-B slots, slot XOR-swizzled by (row>>2)&3: conflict-free
// ds_write_b128 and ds_read_b128, no padding, 32 KB double-buffered).  Inside
// a 16-k step the reduction order is permuted: lane half h = l>>5 takes
// k = 8h + 4q + e at MFMA (q, e), so one ds_read_b128 carries the operands of
// four MFMAs.  n is tap-major (n = tap*Cin + ci) with the tap decoded per
// staged row once, so any Cin (64, the stem's 3) works; the n-tile-0
// workgroups sum their dY rows from registers (bias gradient).
template <int BM, int BN, int KS, int ST, bool PRO, bool VEC1>
__global__ void __launch_bounds__(NT, 4) conv_wgrad2_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                           const float* __restrict__ pscale,
                                                           const float* __restrict__ pshift, int B, int Cin, int H,
                                                           int W, int Cout, int Ho, int Wo, int kchunk,
                                                           float* __restrict__ slab, int with_bias) {
    constexpr int PADK = (KS - 1) / 2;
    constexpr int TM = BM / 64, TN = BN / 64;
    constexpr int AR = BM / 64, BR = BN / 64;   // staged rows per thread
    __shared__ float4 As[2][BM * 4];
    __shared__ float4 Bs[2][BN * 4];
    __shared__ float s_sc[PRO ? MAXC : 1], s_sh[PRO ? MAXC : 1];

    const int P = Ho * Wo, HWin = H * W;
    const int Kall = B * P;
    const int Ntot = Cin * KS * KS, Nt = Ntot + 1;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // (wave-uniform: SGPR)
    const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * (BN / 2);
    // XCD-aware tile order: the n tiles (taps) and m tiles of one k split read
    // the same dy / x rows and share an L2.
    const int lam = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                              gridDim.x * gridDim.y * gridDim.z);
    const int bx = lam % gridDim.x, by = (lam / gridDim.x) % gridDim.y, bz = lam / (gridDim.x * gridDim.y);
    const int m0 = by * BM, nb0 = bx * BN;
    const int k_begin = bz * kchunk;
    const int k_end = min(Kall, k_begin + kchunk);
    const int q = tid & 3, r0 = tid >> 2;
    const bool bias_blk = with_bias && bx == 0;

    if (PRO) {
        for (int c = tid; c < Cin; c += NT) {
            s_sc[c] = pscale[c];
            s_sh[c] = pshift[c];
        }
        __syncthreads();
    }
    int am[AR];
    bool aok[AR];
#pragma unroll
    for (int j = 0; j < AR; ++j) {
        const int m = m0 + r0 + 64 * j;
        aok[j] = m < Cout;
        am[j] = min(m, Cout - 1);
    }
    int bci[BR], bdh[BR], bdw[BR];
    bool bok[BR];
#pragma unroll
    for (int j = 0; j < BR; ++j) {
        const int n = nb0 + r0 + 64 * j;
        bok[j] = n < Ntot;
        const int nn = min(n, Ntot - 1);
        const int tap = nn / Cin, ci = nn - tap * Cin;
        const int kh = tap / KS, kw = tap - kh * KS;
        bci[j] = ci;
        bdh[j] = kh - PADK;
        bdw[j] = kw - PADK;
    }

    // raw loads stay in registers across the MFMAs; masks / prologue at store
    float4 ra[AR], rb[BR];
    float bsum[AR];
    bool kv_st = false;
    unsigned bmask = 0;          // generic B path: 4 in-bounds bits per staged row
#pragma unroll
    for (int j = 0; j < AR; ++j) bsum[j] = 0.f;
    auto load = [&](int kt) {
        const int k = kt + 4 * q;
        kv_st = k < k_end;                          // k_end % 4 == 0: all four or none
        const int kc = kv_st ? k : k_begin;
        const int b = kc / P, p = kc - b * P;
#pragma unroll
        for (int j = 0; j < AR; ++j)
            ra[j] = *reinterpret_cast<const float4*>(dy + ((int64_t)b * Cout + am[j]) * P + p);
        if constexpr (VEC1) {
#pragma unroll
            for (int j = 0; j < BR; ++j)
                rb[j] = *reinterpret_cast<const float4*>(x + ((int64_t)b * Cin + bci[j]) * HWin + p);
        } else {
            const int oh = p / Wo, ow = p - oh * Wo;   // Wo % 4 == 0: one output row
            bmask = 0;
#pragma unroll
            for (int j = 0; j < BR; ++j) {
                const int ih = oh * ST + bdh[j];
                const bool rok = bok[j] && ih >= 0 && ih < H;
                const float* src = x + ((int64_t)b * Cin + bci[j]) * HWin + (rok ? ih * W : 0);
                float e4[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int iw = (ow + e) * ST + bdw[j];
                    const bool ok = rok && iw >= 0 && iw < W;
                    e4[e] = src[ok ? iw : 0];
                    bmask |= (ok ? 1u : 0u) << (4 * j + e);
                }
                rb[j] = make_float4(e4[0], e4[1], e4[2], e4[3]);
            }
        }
    };
    auto store = [&](int buf) {
#pragma unroll
        for (int j = 0; j < AR; ++j) {
            const int row = r0 + 64 * j;
            const float4 v = sel4(kv_st && aok[j], ra[j]);
            As[buf][row * 4 + (q ^ ((row >> 2) & 3))] = v;
            if (bias_blk) bsum[j] += (v.x + v.y) + (v.z + v.w);
        }
#pragma unroll
        for (int j = 0; j < BR; ++j) {
            const int row = r0 + 64 * j;
            float4 v = rb[j];
            if (PRO) {
                const float sc = s_sc[bci[j]], sh = s_sh[bci[j]];
                v.x = fmaxf(fmaf(v.x, sc, sh), 0.f);
                v.y = fmaxf(fmaf(v.y, sc, sh), 0.f);
                v.z = fmaxf(fmaf(v.z, sc, sh), 0.f);
                v.w = fmaxf(fmaf(v.w, sc, sh), 0.f);
            }
            if constexpr (VEC1) {
                v = sel4(kv_st && bok[j], v);
            } else {
                const unsigned mj = kv_st ? (bmask >> (4 * j)) : 0u;
                v = make_float4((mj & 1) ? v.x : 0.f, (mj & 2) ? v.y : 0.f, (mj & 4) ? v.z : 0.f,
                                (mj & 8) ? v.w : 0.f);
            }
            Bs[buf][row * 4 + (q ^ ((row >> 2) & 3))] = v;
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nkt = (k_end - k_begin + 15) / 16;
    // T14 order, as in conv_fwd_kernel
    if (nkt > 0) {
        load(k_begin);
        store(0);
    }
    if (nkt > 1) load(k_begin + 16);
    const int li = lane & 31, h = lane >> 5;
    for (int t = 0; t < nkt; ++t) {
        const int cur = t & 1;
        __syncthreads();
        if (t + 1 < nkt) {
            store(cur ^ 1);
            if (t + 2 < nkt) load(k_begin + (t + 2) * 16);
        }
#pragma unroll
        for (int q2 = 0; q2 < 2; ++q2) {
            const int sl = 2 * h + q2;
            float4 af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = wm + 32 * i + li;
                af[i] = As[cur][row * 4 + (sl ^ ((row >> 2) & 3))];
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int row = wn + 32 * j + li;
                bf[j] = Bs[cur][row * 4 + (sl ^ ((row >> 2) & 3))];
            }
#pragma unroll
            for (int e = 0; e < 4; ++e)
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i][e], bf[j][e], acc[i][j], 0, 0, 0);
        }
    }

    float* sl = slab + (int64_t)bz * Cout * Nt;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = nb0 + wn + 32 * j + li;
        if (n >= Ntot) continue;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < Cout) sl[(int64_t)m * Nt + n] = acc[i][j][r];
            }
    }
    if (bias_blk) {
#pragma unroll
        for (int j = 0; j < AR; ++j) {
            float v = bsum[j];
            v += __shfl_xor(v, 1, 64);
            v += __shfl_xor(v, 2, 64);
            if (q == 0 && aok[j]) sl[(int64_t)(m0 + r0 + 64 * j) * Nt + Ntot] = v;
        }
    }
}

// slab columns are tap-major (n = tap*Cin + ci); dw is the reference layout
// [Cout][Cin][KS][KS] (ci*KS*KS + tap).  R split-lanes per output element
// (256/R elements per block) sum interleaved splits with two accumulators;
// the R partials are combined in a fixed order (deterministic).  The sums are
// f64, rounded once: with hundreds of splits (the 1x1 weight gradients over
// 128x128 planes: K = B*16384 pixels in 8-step slices) an f32 sum of the
// partials would add more rounding than the slices themselves carry.
template <int R>
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ slab, int splits, int Cout,
                                                          int Cin, int T, int with_bias, float* __restrict__ dw,
                                                          float* __restrict__ db, int accumulate) {
    constexpr int C = 256 / R;
    __shared__ double red[R][C];
    const int Ntot = Cin * T;
    const int Nt = Ntot + 1;
    const int64_t total = (int64_t)Cout * Nt;
    const int c = threadIdx.x % C, r = threadIdx.x / C;
    for (int64_t i0 = (int64_t)blockIdx.x * C; i0 < total; i0 += (int64_t)gridDim.x * C) {
        const int64_t i = i0 + c;
        const int64_t ic = i < total ? i : total - 1;
        double s0 = 0.0, s1 = 0.0;
        int z = r;
        for (; z + R < splits; z += 2 * R) {
            s0 += (double)slab[(int64_t)z * total + ic];
            s1 += (double)slab[(int64_t)(z + R) * total + ic];
        }
        if (z < splits) s0 += (double)slab[(int64_t)z * total + ic];
        double sd = s0 + s1;
        if (R > 1) {
            red[r][c] = sd;
            __syncthreads();
            if (r == 0) {
                sd = red[0][c];
#pragma unroll
                for (int q = 1; q < R; ++q) sd += red[q][c];
            }
            __syncthreads();
        }
        const float s = (float)sd;
        if (r != 0 || i >= total) continue;
        const int m = (int)(i / Nt), n = (int)(i - (int64_t)m * Nt);
        if (n < Ntot) {
            const int tap = n / Cin, ci = n - tap * Cin;
            float* d = dw + (int64_t)m * Ntot + (int64_t)ci * T + tap;
            *d = accumulate ? *d + s : s;
        } else if (with_bias && db) {
            db[m] = accumulate ? db[m] + s : s;
        }
    }
}

int launch_wgrad_reduce(const float* slab, int splits, int Cout, int Cin, int T, int wb, float* dw, float* db,
                        int accumulate, hipStream_t st) {
    const int64_t total = (int64_t)Cout * (Cin * T + 1);
    int R = 1;
    while (R < 16 && R * 32 < splits) R *= 2;           // <= ~32 loads per thread
    const int C = 256 / R;
    int64_t g = (total + C - 1) / C;
    if (g > 8192) g = 8192;
    switch (R) {
#define UBPL_RED(R_)                                                                                                 \
    case R_:                                                                                                         \
        hipLaunchKernelGGL(wgrad_reduce_kernel<R_>, dim3((unsigned)g), dim3(256), 0, st, slab, splits, Cout, Cin, T, \
                           wb, dw, db, accumulate);                                                                  \
        break;
        UBPL_RED(1) UBPL_RED(2) UBPL_RED(4) UBPL_RED(8) UBPL_RED(16)
#undef UBPL_RED
    }
    UBPL_LAUNCH_CHECK();
    return 0;
}

// Forward weight layout (grouped tap-major): wt[co][ci/G][tap][ci%G] = w[co][ci][tap].
__device__ __forceinline__ int64_t fwd_layout_src(int64_t i, int Cout, int Cin, int T) {
    const int G = conv_kgroup(Cin);
    const int gi = (int)(i % G);
    const int64_t t1 = i / G;
    const int tap = (int)(t1 % T);
    const int64_t t2 = t1 / T;
    const int cb = (int)(t2 % (Cin / G));
    const int co = (int)(t2 / (Cin / G));
    return ((int64_t)co * Cin + cb * G + gi) * T + tap;
}

// dgrad weights = the forward layout of the flipped, transposed kernel:
// wd[ci][co/G][tap][co%G] = w[co][ci][T-1-tap]  (G = conv_kgroup(Cout)).
__device__ __forceinline__ int64_t dgrad_layout_src(int64_t i, int Cout, int Cin, int T) {
    const int G = conv_kgroup(Cout);
    const int gi = (int)(i % G);
    const int64_t t1 = i / G;
    const int tap = (int)(t1 % T);
    const int64_t t2 = t1 / T;
    const int cb = (int)(t2 % (Cout / G));
    const int ci = (int)(t2 / (Cout / G));
    return ((int64_t)(cb * G + gi) * Cin + ci) * T + (T - 1 - tap);
}

__global__ void tapmajor_kernel(const float* __restrict__ w, int Cout, int Cin, int T, float* __restrict__ wt) {
    const int64_t total = (int64_t)Cout * Cin * T;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
        wt[i] = w[fwd_layout_src(i, Cout, Cin, T)];
}

__global__ void flip_tapmajor_kernel(const float* __restrict__ w, int Cout, int Cin, int T, float* __restrict__ wd) {
    const int64_t total = (int64_t)Cout * Cin * T;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
        wd[i] = w[dgrad_layout_src(i, Cout, Cin, T)];
}

// Batched weight re-layout over a segment table (int64 [nseg][5]:
// src_off, dst_off, Cout, Cin, T), one segment per blockIdx.y.
// mode 0: forward layout, mode 1: dgrad layout (above).
__global__ void __launch_bounds__(256) relayout_kernel(const float* __restrict__ src, float* __restrict__ dst,
                                                      const int64_t* __restrict__ table, int mode) {
    const int64_t* e = table + (int64_t)blockIdx.y * 5;
    const int64_t so = e[0], dof = e[1];
    const int Cout = (int)e[2], Cin = (int)e[3], T = (int)e[4];
    const int64_t total = (int64_t)Cout * Cin * T;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x)
        dst[dof + i] = src[so + (mode == 0 ? fwd_layout_src(i, Cout, Cin, T) : dgrad_layout_src(i, Cout, Cin, T))];
}

struct Plan {
    int bm, splits, kchunk;
};

// ---- grid planning: a cost model over whole CU rounds.
// Blocks spread evenly over the CUs; a CU with c blocks (r = min(c, occ)
// resident) runs them in c * (steps + 2) K steps at a rate that needs ~3
// resident blocks to hide latency.  Split-K adds the slab written by the
// main kernel and re-read by the reduce, plus one launch.
struct Device {
    int ncu = 256;
    int occ_fwd128 = 4, occ_fwd64 = 5, occ_wgrad = 4;
    int occ_dma128 = 2, occ_dma64 = 2;
    int occ_w2[2][2] = {{8, 5}, {5, 4}};   // [bm == 128][bn == 128]
};

const Device& device_info();

double split_cost(int64_t tiles, int s, int64_t nsteps, int occ, int ncu, double step_flops, double slab_bytes_per_split) {
    const int64_t blocks = tiles * s;
    const int64_t per_cu = (blocks + ncu - 1) / ncu;
    const int64_t r = per_cu < occ ? per_cu : occ;
    const double eff = r >= 3 ? 1.0 : (r + 1) / 4.0;
    const int64_t steps = (nsteps + s - 1) / s;
    const double rate = 0.6e12 * 0.8;             // f32 MFMA flop/s per CU, sustained
    double t = (double)per_cu * (double)(steps + 2) * step_flops / (rate * eff);
    if (s > 1) t += 2.0 * s * slab_bytes_per_split / 5e12 + 4e-6;
    return t;
}

int best_split(int64_t tiles, int64_t nsteps, int maxs, int occ, int ncu, double step_flops,
               double slab_bytes_per_split) {
    int best = 1;
    double bc = split_cost(tiles, 1, nsteps, occ, ncu, step_flops, slab_bytes_per_split);
    for (int s = 2; s <= maxs; ++s) {
        const double c = split_cost(tiles, s, nsteps, occ, ncu, step_flops, slab_bytes_per_split);
        if (c < bc * 0.97) {      // a split must pay for itself clearly
            bc = c;
            best = s;
        }
    }
    return best;
}

// Tile height + split-K for the forward (BN = 128, BK = 16).
Plan fwd_plan(int Cout, int64_t N, int Ktot, int bn, bool dma = false) {
    const Device& d = device_info();
    // tuning hook: UBPL_DMA_BM=64|128 pins the 1x1 DMA kernel's tile height
    static const int force_bm = [] {
        const char* e = getenv("UBPL_DMA_BM");
        return e ? atoi(e) : 0;
    }();
    const int nkt = (Ktot + BK - 1) / BK;
    const int maxs = nkt / 2 > 0 ? nkt / 2 : 1;            // >= 2 K steps per split
    Plan best{64, 1, 0};
    double bc = 1e30;
    for (int bm : {128, 64}) {
        if (bm == 128 && Cout <= 64) continue;
        if (dma && force_bm && bm != force_bm && !(force_bm == 128 && Cout <= 64)) continue;
        const int64_t tiles = ((Cout + bm - 1) / bm) * ((N + bn - 1) / bn);
        const int occ = dma ? (bm == 128 ? d.occ_dma128 : d.occ_dma64) : (bm == 128 ? d.occ_fwd128 : d.occ_fwd64);
        const double sf = 2.0 * bm * bn * BK;
        const int s = best_split(tiles, nkt, maxs, occ, d.ncu, sf, 4.0 * Cout * N);
        // 64-row tiles re-read the B operand twice as often: ~15% slower per flop (measured)
        const double c = split_cost(tiles, s, nkt, occ, d.ncu, sf, 4.0 * Cout * N) / (bm == 128 ? 1.0 : 0.85);
        if (c < bc) {
            bc = c;
            best.bm = bm;
            best.splits = s;
        }
    }
    const int steps = (nkt + best.splits - 1) / best.splits;
    best.kchunk = steps * BK;
    best.splits = (nkt + steps - 1) / steps;
    return best;
}

template <int BM, int BN, int KS, int ST, bool PRO, bool VECB, bool TAPK, bool AVEC>
int launch_fwd(const float* x, const float* w, const float* bias, const float* ps, const float* sh, const float* res,
               float* y, int B, int Cin, int H, int W, int Cout, int Ho, int Wo, const Plan& pl, float* slab,
               hipStream_t st) {
    const int64_t N = (int64_t)B * Ho * Wo;
    dim3 grid((unsigned)((N + BN - 1) / BN), (unsigned)((Cout + BM - 1) / BM), (unsigned)pl.splits);
    const bool split = pl.splits > 1;
    hipLaunchKernelGGL((conv_fwd_kernel<BM, BN, KS, ST, PRO, VECB, TAPK, AVEC>), grid, dim3(NT), 0, st, x, w, bias, ps, sh,
                       split ? nullptr : res, y, B, Cin, H, W, Cout, Ho, Wo, pl.kchunk, split ? slab : nullptr);
    UBPL_LAUNCH_CHECK();
    if (split) {
        const int64_t total = (int64_t)Cout * N;
        int g = (int)((total + 255) / 256);
        if (g > 8192) g = 8192;
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3(g), dim3(256), 0, st, slab, pl.splits, Cout, Ho * Wo, N, bias,
                           res, y);
        UBPL_LAUNCH_CHECK();
    }
    return 0;
}

template <int KS, int ST, bool PRO, bool VECB, bool TAPK, bool AVEC>
int fwd_bm2(const Plan& pl, const float* x, const float* w, const float* bias, const float* ps, const float* sh,
            const float* res, float* y, int B, int Cin, int H, int W, int Cout, int Ho, int Wo, float* slab,
            hipStream_t st) {
    if (pl.bm == 128)
        return launch_fwd<128, 128, KS, ST, PRO, VECB, TAPK, AVEC>(x, w, bias, ps, sh, res, y, B, Cin, H, W, Cout,
                                                                  Ho, Wo, pl, slab, st);
    return launch_fwd<64, 128, KS, ST, PRO, VECB, TAPK, AVEC>(x, w, bias, ps, sh, res, y, B, Cin, H, W, Cout, Ho, Wo,
                                                             pl, slab, st);
}

// AVEC (float4 weight rows) when Ktot % 4 == 0 and w is 16-B aligned; KS = 3
// (Cin % 16 == 0) always qualifies, the stem (Cin = 3) never does.
template <int KS, int ST, bool PRO, bool VECB, bool TAPK>
int fwd_bm(const Plan& pl, const float* x, const float* w, const float* bias, const float* ps, const float* sh,
           const float* res, float* y, int B, int Cin, int H, int W, int Cout, int Ho, int Wo, float* slab,
           hipStream_t st) {
    const bool avec = ((Cin * KS * KS) % 4 == 0) && (((uintptr_t)w & 15) == 0);
    if constexpr (KS == 7) {
        return fwd_bm2<KS, ST, PRO, VECB, TAPK, false>(pl, x, w, bias, ps, sh, res, y, B, Cin, H, W, Cout, Ho, Wo, slab, st);
    } else {
        if (avec)
            return fwd_bm2<KS, ST, PRO, VECB, TAPK, true>(pl, x, w, bias, ps, sh, res, y, B, Cin, H, W, Cout, Ho, Wo, slab, st);
        if constexpr (KS == 3) return (int)hipErrorInvalidValue;
        else return fwd_bm2<KS, ST, PRO, VECB, TAPK, false>(pl, x, w, bias, ps, sh, res, y, B, Cin, H, W, Cout, Ho, Wo, slab, st);
    }
}

template <int BM, int BN, int KS, int ST, bool PRO, bool VEC1>
int wgrad2_launch(const float* dy, const float* x, const float* ps, const float* sh, int B, int Cin, int H, int W,
                  int Cout, int Ho, int Wo, int splits, int kchunk, float* slab, int with_bias, hipStream_t st) {
    const int Ntot = Cin * KS * KS;
    dim3 grid((unsigned)((Ntot + BN - 1) / BN), (unsigned)((Cout + BM - 1) / BM), (unsigned)splits);
    hipLaunchKernelGGL((conv_wgrad2_kernel<BM, BN, KS, ST, PRO, VEC1>), grid, dim3(NT), 0, st, dy, x, ps, sh, B, Cin,
                       H, W, Cout, Ho, Wo, kchunk, slab, with_bias);
    UBPL_LAUNCH_CHECK();
    return 0;
}

template <int KS, int ST, bool PRO, bool VEC1>
int wgrad2_tile(int bm, int bn, const float* dy, const float* x, const float* ps, const float* sh, int B, int Cin,
                int H, int W, int Cout, int Ho, int Wo, int splits, int kchunk, float* slab, int wb, hipStream_t st) {
    if (bm == 128 && bn == 128)
        return wgrad2_launch<128, 128, KS, ST, PRO, VEC1>(dy, x, ps, sh, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st);
    if (bm == 128)
        return wgrad2_launch<128, 64, KS, ST, PRO, VEC1>(dy, x, ps, sh, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st);
    if (bn == 128)
        return wgrad2_launch<64, 128, KS, ST, PRO, VEC1>(dy, x, ps, sh, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st);
    return wgrad2_launch<64, 64, KS, ST, PRO, VEC1>(dy, x, ps, sh, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st);
}

template <int KS, int ST, bool PRO, bool TAPN>
int wgrad_launch(const float* dy, const float* x, const float* ps, const float* sh, int B, int Cin, int H, int W,
                 int Cout, int Ho, int Wo, int splits, int kchunk, float* slab, int with_bias, hipStream_t st) {
    constexpr int BM = 64, BN = 64;
    const int Ntot = Cin * KS * KS;
    dim3 grid((unsigned)((Ntot + BN - 1) / BN), (unsigned)((Cout + BM - 1) / BM), (unsigned)splits);
    hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, KS, ST, PRO, TAPN>), grid, dim3(NT), 0, st, dy, x, ps, sh, B, Cin,
                       H, W, Cout, Ho, Wo, kchunk, slab, with_bias);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// k-contiguous float4 staging (conv_wgrad2_kernel) needs P % 4 == 0 and, for a
// spatial kernel, whole float4 groups inside one output row.
bool wgrad_v2_shape(int KS, int Ho, int Wo) { return (Ho * Wo) % 4 == 0 && (KS == 1 || Wo % 4 == 0); }

struct WPlan {
    int splits, kchunk, bm, bn;
};

// Split of the k = b*P + p reduction over workgroups for the weight gradient.
// v2: BM x BN tiles in {64,128}^2, 16-k steps, chosen by the cost model with a
// per-flop efficiency for the smaller tiles; v1: 64x64, 32-k steps.
WPlan wgrad_plan(int B, int Cin, int Cout, int KS, int Ho, int Wo, bool v2) {
    const Device& d = device_info();
    const int64_t K = (int64_t)B * Ho * Wo;
    const int64_t Ntot = (int64_t)Cin * KS * KS;
    // keep the slab (splits * Cout * (Ntot+1) floats, written + re-read) no larger
    // than the operands it is computed from (dy and x: K * (Cout + Cin) floats)
    // (slabs up to 8 MB are allowed regardless: small levels need the splits)
    int64_t cap = (K * (Cout + Cin)) / ((int64_t)Cout * (Ntot + 1));
    const int64_t cap_small = (int64_t)(8 << 20) / (4 * (int64_t)Cout * (Ntot + 1));
    if (cap < cap_small) cap = cap_small;
    WPlan best{1, 0, 64, 64};
    double bc = 1e30;
    for (int bm : {128, 64})
        for (int bn : {128, 64}) {
            if (!v2 && (bm != 64 || bn != 64)) continue;
            if (bm == 128 && Cout <= 64) continue;
            if (bn == 128 && Ntot <= 64) continue;
            const int kb = v2 ? 16 : 32;
            const int64_t tiles = ((Ntot + bn - 1) / bn) * ((Cout + bm - 1) / bm);
            const int64_t nsteps = (K + kb - 1) / kb;
            int64_t maxs = (K + 4 * kb - 1) / (4 * kb);     // every split >= 4 k steps
            if (maxs > cap) maxs = cap;
            if (maxs > 512) maxs = 512;
            if (maxs < 1) maxs = 1;
            const int occ = v2 ? d.occ_w2[bm == 128][bn == 128] : d.occ_wgrad;
            const double sf = 2.0 * bm * bn * kb, sb = 4.0 * Cout * (Ntot + 1);
            const int s = best_split(tiles, nsteps, (int)maxs, occ, d.ncu, sf, sb);
            const double eff = (bm * bn == 16384) ? 1.0 : (bm * bn == 8192 ? 0.85 : 0.7);
            const double c = split_cost(tiles, s, nsteps, occ, d.ncu, sf, sb) / eff;
            if (c < bc) {
                bc = c;
                int64_t chunk = (K + s - 1) / s;
                chunk = (chunk + kb - 1) / kb * kb;
                best.kchunk = (int)chunk;
                best.splits = (int)((K + chunk - 1) / chunk);
                best.bm = bm;
                best.bn = bn;
            }
        }
    return best;
}

const Device& device_info() {
    static Device d = [] {
        Device r;
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            r.ncu = v;
        int o = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, conv_fwd_kernel<128, 128, 3, 1, true, false, true, true>, NT,
                                                         0) == hipSuccess && o > 0)
            r.occ_fwd128 = o;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, conv_fwd_kernel<64, 128, 3, 1, true, false, true, true>, NT,
                                                         0) == hipSuccess && o > 0)
            r.occ_fwd64 = o;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, conv_wgrad_kernel<64, 64, 3, 1, true, true>, NT, 0) ==
                hipSuccess && o > 0)
            r.occ_wgrad = o;
        auto q = [&](const void* f, int& dst) {
            int v2 = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&v2, f, NT, 0) == hipSuccess && v2 > 0) dst = v2;
        };
        q((const void*)conv1x1_dma_kernel<128, true>, r.occ_dma128);
        q((const void*)conv1x1_dma_kernel<64, true>, r.occ_dma64);
        q((const void*)conv_wgrad2_kernel<64, 64, 3, 1, true, false>, r.occ_w2[0][0]);
        q((const void*)conv_wgrad2_kernel<64, 128, 3, 1, true, false>, r.occ_w2[0][1]);
        q((const void*)conv_wgrad2_kernel<128, 64, 3, 1, true, false>, r.occ_w2[1][0]);
        q((const void*)conv_wgrad2_kernel<128, 128, 3, 1, true, false>, r.occ_w2[1][1]);
        (void)hipGetLastError();
        return r;
    }();
    return d;
}

}  // namespace

namespace {
template <int BM, bool PRO>
int launch_1x1_dma(const float* x, const float* wk, const float* bias, const float* ps, const float* sh,
                   const float* res, float* y, int B, int K, int P, int M, const Plan& pl, float* slab,
                   float* stat_part, hipStream_t st) {
    const int64_t N = (int64_t)B * P;
    dim3 grid((unsigned)((N + 127) / 128), (unsigned)((M + BM - 1) / BM), (unsigned)pl.splits);
    const bool split = pl.splits > 1;
    hipLaunchKernelGGL((conv1x1_dma_kernel<BM, PRO>), grid, dim3(NT), 0, st, x, wk, bias, ps, sh,
                       split ? nullptr : res, y, B, K, P, M, pl.kchunk, split ? slab : nullptr,
                       split ? nullptr : stat_part);
    UBPL_LAUNCH_CHECK();
    if (split) {
        const int64_t total = (int64_t)M * N;
        int g = (int)((total + 255) / 256);
        if (g > 8192) g = 8192;
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3(g), dim3(256), 0, st, slab, pl.splits, M, P, N, bias, res, y);
        UBPL_LAUNCH_CHECK();
        if (stat_part) return ubpl_bn_partials(y, B, M, P, stat_part, st);
    }
    return 0;
}
}  // namespace

UBPL_API int64_t ubpl_conv1x1_kmajor_workspace(int B, int Cin, int Cout, int P) {
    const Plan pl = fwd_plan(Cout, (int64_t)B * P, Cin, 128, true);
    return pl.splits > 1 ? (int64_t)pl.splits * Cout * B * P : 0;
}

// 1x1 stride-1 conv with k-major weights wk [Cin][Cout] (the data-gradient
// re-layout of a 1x1 conv; for a data gradient, the reference weights
// themselves): y[B,Cout,P] = conv(relu(x*pscale + pshift) or x) + bias (+ res,
// may alias y).  Needs Cin % 16 == 0, Cout % 4 == 0, P % 4 == 0, Cin <= 256 with a prologue,
// 16-B aligned x / wk.  slab: ubpl_conv1x1_kmajor_workspace floats (nullable at 0).
// stat_part (nullable): BatchNorm partials of y (ubpl_bn_partials layout).
UBPL_API int ubpl_conv1x1_forward_kmajor(const float* x, int B, int Cin, int P, const float* wk, const float* bias,
                                         int Cout, const float* pscale, const float* pshift, const float* res,
                                         float* y, float* slab, float* stat_part, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const bool pro = pscale != nullptr;
    if ((pro && Cin > MAXC) || Cin % BK != 0 || Cout % 4 != 0 || P % 4 != 0 || (((uintptr_t)x) & 15) ||
        (((uintptr_t)wk) & 15))
        return (int)hipErrorInvalidValue;
    const Plan pl = fwd_plan(Cout, (int64_t)B * P, Cin, 128, true);
    if (pl.splits > 1 && slab == nullptr) return (int)hipErrorInvalidValue;
    if (pl.bm == 128)
        return pro ? launch_1x1_dma<128, true>(x, wk, bias, pscale, pshift, res, y, B, Cin, P, Cout, pl, slab, stat_part, st)
                   : launch_1x1_dma<128, false>(x, wk, bias, pscale, pshift, res, y, B, Cin, P, Cout, pl, slab, stat_part, st);
    return pro ? launch_1x1_dma<64, true>(x, wk, bias, pscale, pshift, res, y, B, Cin, P, Cout, pl, slab, stat_part, st)
               : launch_1x1_dma<64, false>(x, wk, bias, pscale, pshift, res, y, B, Cin, P, Cout, pl, slab, stat_part, st);
}

// Floats of workspace ubpl_conv2d_forward needs (split-K slab); 0 = none.
// w must be in the layout of ubpl_conv_weight_tapmajor for KS > 1.
UBPL_API int64_t ubpl_conv2d_forward_workspace(int B, int Cin, int Cout, int KS, int Ho, int Wo) {
    const int64_t N = (int64_t)B * Ho * Wo;
    const Plan pl = fwd_plan(Cout, N, Cin * KS * KS, 128);
    return pl.splits > 1 ? (int64_t)pl.splits * Cout * N : 0;
}

// y[B,Cout,Ho,Wo] = conv(relu(x*pscale + pshift) or x, w~, pad=(KS-1)/2) + bias (+ res).
// w~: [Cout][Cin] for KS == 1, tap-major [Cout][KS*KS][Cin] otherwise.
// Supported (KS, stride): (1,1), (3,1), (7,2).  res may alias y.  slab: the
// workspace of ubpl_conv2d_forward_workspace (nullable when that is 0).
UBPL_API int ubpl_conv2d_forward(const float* x, int B, int Cin, int H, int W, const float* w, const float* bias,
                                 int Cout, int KS, int stride, const float* pscale, const float* pshift,
                                 const float* res, float* y, int Ho, int Wo, float* slab, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const bool pro = pscale != nullptr;
    if (pro && Cin > MAXC) return (int)hipErrorInvalidValue;
    const int64_t N = (int64_t)B * Ho * Wo;
    const Plan pl = fwd_plan(Cout, N, Cin * KS * KS, 128);
    if (pl.splits > 1 && slab == nullptr) return (int)hipErrorInvalidValue;
    if (KS == 1 && stride == 1) {
        const bool vec = ((Ho * Wo) % 4 == 0) && (((uintptr_t)x & 15) == 0);
        if (vec)
            return pro ? fwd_bm<1, 1, true, true, true>(pl, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, slab, st)
                       : fwd_bm<1, 1, false, true, true>(pl, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, slab, st);
        return pro ? fwd_bm<1, 1, true, false, true>(pl, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, slab, st)
                   : fwd_bm<1, 1, false, false, true>(pl, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, slab, st);
    }
    if (KS == 3 && stride == 1) {
        if (Cin % BK != 0) return (int)hipErrorInvalidValue;
        return pro ? fwd_bm<3, 1, true, false, true>(pl, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, slab, st)
                   : fwd_bm<3, 1, false, false, true>(pl, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, slab, st);
    }
    if (KS == 7 && stride == 2) {
        return pro ? fwd_bm<7, 2, true, false, false>(pl, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, slab, st)
                   : fwd_bm<7, 2, false, false, false>(pl, x, w, bias, pscale, pshift, res, y, B, Cin, H, W, Cout, Ho, Wo, slab, st);
    }
    return (int)hipErrorInvalidValue;
}

// Floats of slab workspace ubpl_conv2d_wgrad needs.
UBPL_API int64_t ubpl_conv2d_wgrad_workspace(int B, int Cin, int Cout, int KS, int Ho, int Wo) {
    int64_t s = wgrad_plan(B, Cin, Cout, KS, Ho, Wo, false).splits;
    if (wgrad_v2_shape(KS, Ho, Wo)) {
        const int64_t s2 = wgrad_plan(B, Cin, Cout, KS, Ho, Wo, true).splits;
        if (s2 > s) s = s2;
    }
    return s * Cout * (Cin * KS * KS + 1);
}

// dw[Cout,Cin,KS,KS] (+)= sum over (b,p) dy * im2col(relu(x*pscale+pshift) or x);
// db[Cout] (+)= sum over (b,p) dy (db nullable).  slab: workspace floats.
UBPL_API int ubpl_conv2d_wgrad(const float* dy, const float* x, int B, int Cin, int H, int W, int Cout, int KS,
                               int stride, const float* pscale, const float* pshift, int Ho, int Wo, float* slab,
                               float* dw, float* db, int accumulate, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (pscale != nullptr && Cin > MAXC) return (int)hipErrorInvalidValue;
    const bool pro = pscale != nullptr;
    const int wb = db != nullptr;
    const bool v2 = wgrad_v2_shape(KS, Ho, Wo) && (((uintptr_t)dy & 15) == 0);
    const WPlan pl = wgrad_plan(B, Cin, Cout, KS, Ho, Wo, v2);
    const int splits = pl.splits, kchunk = pl.kchunk;
    int rc;
    if (v2) {
        const bool vec1 = KS == 1 && stride == 1 && (((uintptr_t)x & 15) == 0) && ((H * W) % 4 == 0);
#define UBPL_W2(KS_, ST_, VEC_)                                                                                     \
    (pro ? wgrad2_tile<KS_, ST_, true, VEC_>(pl.bm, pl.bn, dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits,  \
                                             kchunk, slab, wb, st)                                                    \
         : wgrad2_tile<KS_, ST_, false, VEC_>(pl.bm, pl.bn, dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, \
                                              kchunk, slab, wb, st))
        if (KS == 1 && stride == 1)
            rc = vec1 ? UBPL_W2(1, 1, true) : UBPL_W2(1, 1, false);
        else if (KS == 3 && stride == 1)
            rc = UBPL_W2(3, 1, false);
        else if (KS == 7 && stride == 2)
            rc = UBPL_W2(7, 2, false);
        else
            return (int)hipErrorInvalidValue;
#undef UBPL_W2
    } else {
        const bool tapn = (KS == 1) || (Cin % 64 == 0);
        if (KS == 1 && stride == 1)
            rc = pro ? wgrad_launch<1, 1, true, true>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st)
                     : wgrad_launch<1, 1, false, true>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st);
        else if (KS == 3 && stride == 1 && tapn)
            rc = pro ? wgrad_launch<3, 1, true, true>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st)
                     : wgrad_launch<3, 1, false, true>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st);
        else if (KS == 3 && stride == 1)
            rc = pro ? wgrad_launch<3, 1, true, false>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st)
                     : wgrad_launch<3, 1, false, false>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st);
        else if (KS == 7 && stride == 2)
            rc = pro ? wgrad_launch<7, 2, true, false>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st)
                     : wgrad_launch<7, 2, false, false>(dy, x, pscale, pshift, B, Cin, H, W, Cout, Ho, Wo, splits, kchunk, slab, wb, st);
        else
            return (int)hipErrorInvalidValue;
    }
    if (rc) return rc;
    return launch_wgrad_reduce(slab, splits, Cout, Cin, KS * KS, wb, dw, db, accumulate, st);
}

// Reduce a weight-gradient slab [splits][Cout][Cin*T + 1] (columns tap-major
// n = tap*Cin + ci, the last = bias) into dw (reference layout) and db (nullable).
UBPL_API int ubpl_wgrad_slab_reduce(const float* slab, int splits, int Cout, int Cin, int T, int with_bias, float* dw,
                                    float* db, int accumulate, void* stream) {
    return launch_wgrad_reduce(slab, splits, Cout, Cin, T, with_bias, dw, db, accumulate, (hipStream_t)stream);
}

// Forward weight layout: wt[co][ci/G][tap][ci%G] = w[co][ci][tap], G = 16 if it
// divides Cin, else Cin (plain tap-major); for KS == 1 it is w itself.
UBPL_API int ubpl_conv_weight_tapmajor(const float* w, int Cout, int Cin, int KS, float* wt, void* stream) {
    const int64_t total = (int64_t)Cout * Cin * KS * KS;
    int grid = (int)((total + 255) / 256);
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(tapmajor_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, KS * KS, wt);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// dgrad weights (stride 1): the forward layout of the flipped, transposed
// kernel, wd[ci][co/G][tap][co%G] = w[co][ci][KS*KS-1-tap]: dx = conv(dy, wd).
UBPL_API int ubpl_conv_weight_flip(const float* w, int Cout, int Cin, int KS, float* wt, void* stream) {
    const int64_t total = (int64_t)Cout * Cin * KS * KS;
    int grid = (int)((total + 255) / 256);
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(flip_tapmajor_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, w, Cout, Cin, KS * KS,
                       wt);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// All conv weights of a model re-laid out in one launch (see relayout_kernel).
UBPL_API int ubpl_conv_weights_relayout(const float* src, float* dst, const int64_t* table, int nseg, int mode,
                                        void* stream) {
    if (nseg <= 0) return 0;
    hipLaunchKernelGGL(relayout_kernel, dim3(64, nseg), dim3(256), 0, (hipStream_t)stream, src, dst, table, mode);
    UBPL_LAUNCH_CHECK();
    return 0;
}
