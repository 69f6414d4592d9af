// Convolutions on the bf16 matrix cores with fp32 operands carried as sums of
// bf16 pieces ("split-bf16"): v = v0 + v1 (+ v2), v0 = bf16(v), v1 = bf16(v - v0),
// v2 = bf16(v - v0 - v1).  A product a*b is the sum of the piece products with
// pa + pb < NP (the dropped ones are below the fp32-relevant range for NP = 3,
// ~2^-16 relative for NP = 2), each exact in f32, summed by
// v_mfma_f32_32x32x16_bf16 into an f32 accumulator:
//   NP = 2: 3 MFMAs per 32x32x16 step (16/3 = 5.3x the v_mfma_f32_32x32x2_f32 rate);
//   NP = 3: 6 MFMAs (2.7x), rounding error at the level of an f32 fmaf chain.
// Same GEMM views, K order and epilogues as conv.hip (the Conv wrapper,
// models/base/layers.py:31-50): grouped tap-major k = (ci/16)*16T + tap*16 + ci%16.
//
// Operand images in LDS: [piece][row][4 x 16 B] with the row's 32 k of one
// K step in four 16-B chunks (chunk c = 2s + h holds k = 16s + 8h .. +7, the
// 8 bf16 lane (r, h) of MFMA k-step s reads) — A rows = output channels, B rows
// = output pixels n, both k-contiguous, chunk XOR-swizzled by (row >> 2) & 3
// (conflict-free ds_read_b128 for the 16-lane groups of a 32-row fragment read).
// Weights are split once per pass (ubpl_conv_weights_split, a batched
// re-layout into NP bf16 planes); activations are split while they are staged,
// after the fused BN+ReLU prologue.
#include <atomic>
#include "common.h"
#include <cstdlib>
using ubpl::xcd_remap;

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short short8 __attribute__((ext_vector_type(8)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

namespace {

// the unguarded epilogues' stores non-temporal (UBPL_NT_EPI, below); the 1x1 split-load kernel's
// transposed residual epilogue (UBPL_SOL_TEPI); its launch-bounds occupancy (UBPL_SOL_LB); the
// one-buffer halo kernel's deepest A ring (UBPL_PSAH_NA_MAX) — build-time knobs, defaults measured
// (DESIGN.md §4, §6).  Round 6: the timing-only diagnostic builds and the variants that measured
// slower (the warp-specialized 1x1 and 3x3 kernels, the 16x16x32 halo forms, fair arbitration,
// clock stamps) were removed from the product source; they stay in the git history.
#ifndef UBPL_SOL_TEPI
#define UBPL_SOL_TEPI 1
#endif
#ifndef UBPL_PSAH_NA_MAX
#define UBPL_PSAH_NA_MAX 3
#endif
#ifndef UBPL_SOL_LB
#define UBPL_SOL_LB 2
#endif

constexpr int NT = 256;
constexpr int PSA_KSUB1 = 2;     // conv_psa_kernel on the bf16 path: 16-k steps per stage (measured)
constexpr int SOL_PRO_K = 512;   // conv1x1_sol_kernel: largest input channel count with a prologue
constexpr int BK = 32;
constexpr int BN = 128;

using ubpl::split2;

__device__ __forceinline__ int swz(int row, int c) { return c ^ ((row >> 2) & 3); }

// One 32x32x16 piece product: bf16 pieces (NP = 1, 3) or fp16 pieces (NP = 2, the
// 2xfp16 path: common.h split2); the fragments travel as 16-bit lanes either way.
template <int NP>
__device__ __forceinline__ floatx16 mfma_piece(const bf16x8 a, const bf16x8 b, const floatx16 c) {
    if constexpr (NP == 2)
        return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, a), __builtin_bit_cast(half8, b), c,
                                                      0, 0, 0);
    else
        return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// element e of a piece fragment as f32 (fp16 pieces for NP = 2, bf16 otherwise)
template <int NP>
__device__ __forceinline__ float piece_elem(const bf16x8 v, int e) {
    if constexpr (NP == 2) return (float)__builtin_bit_cast(half8, v)[e];
    else return (float)v[e];
}

// acc += sum over piece pairs (pa, pb), pa + pb < NP, smallest terms first
template <int NP>
__device__ __forceinline__ void mfma_split(floatx16& acc, const bf16x8 (&a)[NP], const bf16x8 (&b)[NP]) {
#pragma unroll
    for (int d = NP - 1; d >= 0; --d)
#pragma unroll
        for (int pa = d; pa >= 0; --pa) acc = mfma_piece<NP>(a[pa], b[d - pa], acc);
}

// acc += t one element at a time.  The floatx16 `+=` lowers to v_pk_add_f32,
// which beside MFMAs costs ~13 cycles more per instruction than the two scalar
// adds it replaces (MI355X_MICROARCH.md, 'price of one filler beside MFMAs':
// packed f32 VALU is an anti-lever there); scalar v_add_f32 hide in the MFMA
// gaps.  Same rounding: one f32 add per element.  The empty asm on each sum
// keeps the SLP vectorizer from re-packing the adds (it emits no instruction).
__device__ __forceinline__ void drain(floatx16& acc, const floatx16 t) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        float v = acc[r] + t[r];
        asm("" : "+v"(v));
        acc[r] = v;
    }
}

// Ping-pong schedule of one chunk chain (its NP(NP+1)/2 MFMAs) with the previous
// tile's 16 drain adds spread over the MFMA gaps (6 x (1 MFMA : 3 VALU) for the
// 6-product chain, 3 x (1 : 6) for the 3-product one)
template <int NP>
__device__ __forceinline__ void pp_schedule() {
    constexpr int NMF = NP * (NP + 1) / 2;
    constexpr int NV = (16 + NMF - 1) / NMF;
#pragma unroll
    for (int g = 0; g < NMF; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
}

// the same sum started from zero (one 16-k chunk of the chunked accumulation):
// the first MFMA takes C = 0 as an inline constant, no zeroed registers
template <int NP>
__device__ __forceinline__ floatx16 mfma_split0(const bf16x8 (&a)[NP], const bf16x8 (&b)[NP]) {
    const floatx16 zero = {};
    floatx16 t = mfma_piece<NP>(a[NP - 1], b[0], zero);
#pragma unroll
    for (int d = NP - 1; d >= 0; --d)
#pragma unroll
        for (int pa = d; pa >= 0; --pa)
            if (!(d == NP - 1 && pa == NP - 1)) t = mfma_piece<NP>(a[pa], b[d - pa], t);
    return t;
}


// The scalar epilogue of a TM x TN tile of 32 x 32 MFMA blocks (rows mrow0 + ..,
// output offsets obase[j] + m * P): when the whole tile is in range (`full`,
// wave-uniform) the stores go out unguarded — each guarded store had been a
// compare, an exec-mask branch and a restore.
// the unguarded epilogue's stores non-temporal (streamed past the caches: the output is
// read next by another kernel, far more than L2 holds): 207.5 vs 212.7 us on the 128-ch
// 64x64 halo conv, 238 vs 252 at 64 ch 128x128, 1x1 1-3 %, the step within noise
// (profiles/r04_psa_diag.txt); UBPL_NT_EPI=0 at build time: plain stores
#ifndef UBPL_NT_EPI
#define UBPL_NT_EPI 1
#endif
// inv: 1 / the accumulators' scale (seed_acc), applied exactly (a power of two)
template <int TM, int TN>
__device__ __forceinline__ void store_tile(const floatx16 (&acc)[TM][TN], const bool (&nok)[TN],
                                           const int64_t (&obase)[TN], int mrow0, int M, int P, float* y,
                                           bool full, float inv = 1.f) {
    const int h = (threadIdx.x & 63) >> 5;
    if (full) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    float* d = y + obase[j] + (int64_t)(mrow0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h) * P;
                    if (UBPL_NT_EPI) __builtin_nontemporal_store(acc[i][j][r] * inv, d);
                    else *d = acc[i][j][r] * inv;
                }
        return;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        if (!nok[j]) continue;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = mrow0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < M) y[obase[j] + (int64_t)m * P] = acc[i][j][r] * inv;
            }
    }
}

// ------------------------------------------------------------------ forward
// x NCHW f32; wp: NP planes (stride wplane elements) of the grouped tap-major
// weights [Cout][Ktot] as bf16; Cin % 16 == 0.  Epilogue / split-K slab as
// conv.hip's conv_fwd_kernel.
template <int BM, int KS, int ST, bool PRO, int NP>
__global__ void __launch_bounds__(NT, 2) conv_fwd_split_kernel(
    const float* __restrict__ x, const uint16_t* __restrict__ wp, int64_t wplane, const float* __restrict__ bias,
    const float* __restrict__ pscale, const float* __restrict__ pshift, const float* res, float* y, int B, int Cin,
    int H, int W, int Cout, int Ho, int Wo, int kchunk, float* __restrict__ slab) {
    constexpr int PADK = (KS - 1) / 2;
    constexpr int T = KS * KS;
    constexpr int TM = BM / 64, TN = BN / 64;
    constexpr int ACH = BM == 128 ? 2 : 1;   // 16-B weight chunks per thread per piece
    __shared__ uint4 lds[2 * NP * (BM + BN) * 4];
    uint4* As = lds;
    uint4* Bs = lds + 2 * NP * BM * 4;

    const int P = Ho * Wo, HWin = H * W;
    const int64_t N = (int64_t)B * P;
    const int Ktot = Cin * T;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // (wave-uniform: SGPR)
    const int wm = (wid >> 1) * (BM / 2), wn = (wid & 1) * (BN / 2);
    const int lam = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                              gridDim.x * gridDim.y * gridDim.z);
    const int by = lam % gridDim.y, bx = (lam / gridDim.y) % gridDim.x, bz = lam / (gridDim.y * gridDim.x);
    const int m0 = by * BM;
    const int64_t n0 = (int64_t)bx * BN;
    const int k_begin = bz * kchunk;
    const int k_end = min(Ktot, k_begin + kchunk);

    // ---- A (weights) loader: row am, chunks ac0 .. ac0 + ACH - 1
    const int am = tid % BM;
    const int ac0 = (tid / BM) * ACH;
    const bool am_ok = m0 + am < Cout;
    const uint16_t* wrow = wp + (int64_t)min(m0 + am, Cout - 1) * Ktot;
    // ---- B (activations) loader: column bn, k half g (16 k = one (group, tap))
    const int bnl = tid & (BN - 1);
    const int g = __builtin_amdgcn_readfirstlane(tid >> 7);
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

    uint4 ra[NP][ACH];
    float rb[16];
    bool b_inb = false;

    auto load = [&](int kt) {
        {
            const int k = min(kt + 8 * ac0, Ktot - 8 * ACH);
#pragma unroll
            for (int p = 0; p < NP; ++p)
#pragma unroll
                for (int c = 0; c < ACH; ++c)
                    ra[p][c] = *reinterpret_cast<const uint4*>(wrow + (int64_t)p * wplane + k + 8 * c);
        }
        const int kk = kt + 16 * g;
        const int kg = kk >> 4;
        const int tap = kg % T;
        const int ci0 = min((kg / T) * 16, Cin - 16);
        const int kh = tap / KS, kw = tap - kh * KS;
        const int ih = coh * ST - PADK + kh, iw = cow * ST - PADK + kw;
        b_inb = cvalid && kk < k_end && ih >= 0 && ih < H && iw >= 0 && iw < W;
        const float* src = xb + (int64_t)ci0 * HWin + (b_inb ? ih * W + iw : 0);
#pragma unroll
        for (int j = 0; j < 16; ++j) rb[j] = src[(int64_t)j * HWin];
    };
    auto store = [&](int buf, int kt) {
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int c = 0; c < ACH; ++c) {
                const int ch = ac0 + c;
                const bool ok = am_ok && kt + 8 * ch < k_end;
                As[((buf * NP + p) * BM + am) * 4 + swz(am, ch)] = ok ? ra[p][c] : make_uint4(0, 0, 0, 0);
            }
        // prologue on every element (unconditional scalar loads of the 16
        // channels' coefficients), then a select: a load or an LDS read under
        // the in-bounds condition becomes a branch with its own vmcnt(0)
        float v[16];
        if (PRO) {
            const int kg = (kt + 16 * g) >> 4;
            const int ci0 = __builtin_amdgcn_readfirstlane(min((kg / T) * 16, Cin - 16));
            float sc[16], sh[16];
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                sc[j] = pscale[ci0 + j];
                sh[j] = pshift[ci0 + j];
            }
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = fmaxf(fmaf(rb[j], sc[j], sh[j]), 0.f);
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = rb[j];
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = b_inb ? v[j] : 0.f;
        uint32_t pk[NP][8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            uint32_t o[NP];
            split2<NP>(v[2 * i], v[2 * i + 1], o);
#pragma unroll
            for (int p = 0; p < NP; ++p) pk[p][i] = o[p];
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            uint4* rowp = Bs + ((buf * NP + p) * BN + bnl) * 4;
            rowp[swz(bnl, 2 * g)] = make_uint4(pk[p][0], pk[p][1], pk[p][2], pk[p][3]);
            rowp[swz(bnl, 2 * g + 1)] = make_uint4(pk[p][4], pk[p][5], pk[p][6], pk[p][7]);
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    const int nkt = (k_end - k_begin + BK - 1) / BK;
    if (nkt > 0) {
        load(k_begin);
        store(0, k_begin);
    }
    if (nkt > 1) load(k_begin + BK);
    const int li = lane & 31, h = lane >> 5;
    for (int t = 0; t < nkt; ++t) {
        const int cur = t & 1;
        __syncthreads();
        if (t + 1 < nkt) {
            store(cur ^ 1, k_begin + (t + 1) * BK);
            if (t + 2 < nkt) load(k_begin + (t + 2) * BK);
        }
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int c = 2 * s + h;
            bf16x8 af[TM][NP], bfr[TN][NP];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = wm + 32 * i + li;
#pragma unroll
                for (int p = 0; p < NP; ++p)
                    af[i][p] = __builtin_bit_cast(bf16x8, As[((cur * NP + p) * BM + row) * 4 + swz(row, c)]);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const int row = wn + 32 * j + li;
#pragma unroll
                for (int p = 0; p < NP; ++p)
                    bfr[j][p] = __builtin_bit_cast(bf16x8, Bs[((cur * NP + p) * BN + row) * 4 + swz(row, c)]);
            }
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    if constexpr (NP == 3) {
                        // the bf16 MFMA aligns its 17 addends to the largest and
                        // truncates below ~2^-26 of it (tools/experiments/mfma_numerics):
                        // against a large running sum that bias grows with K.  Each
                        // 16-k chunk starts from 0 and is added with a rounded f32 add.
                        floatx16 tmp;
#pragma unroll
                        for (int r = 0; r < 16; ++r) tmp[r] = 0.f;
                        mfma_split<NP>(tmp, af[i], bfr[j]);
                        drain(acc[i][j], tmp);
                    } else {
                        mfma_split<NP>(acc[i][j], af[i], bfr[j]);
                    }
                }
        }
    }

    if (slab != nullptr) {
        float* sl = slab + (int64_t)bz * Cout * N;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t n = n0 + wn + 32 * j + li;
            if (n >= N) continue;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (m < Cout) sl[(int64_t)m * N + n] = acc[i][j][r];
                }
        }
        return;
    }
    // epilogue: + bias (+ residual; res may alias y: all loads before any store)
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
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = min(m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h, Cout - 1);
                if (bias) acc[i][j][r] += bias[m];
                if (res) acc[i][j][r] += res[obase[j] + (int64_t)m * P];
            }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        if (!nok[j]) continue;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < Cout) y[obase[j] + (int64_t)m * P] = acc[i][j][r];
            }
    }
}

// ------------------------------------------------------------------ pre-split activations
// PSA layout: NP bf16 planes (`plane` elements apart) of [B][C/16][Hp][Wp][16],
// Hp = H + 2*pad, Wp = W + 2*pad, the border zero: a pixel's 16 channels of one
// group are 32 contiguous bytes = the two 16-B chunks of one B-operand row of
// a K step, and a 3x3 tap is a constant offset (no bounds checks in the conv).
// v = relu(x*scale + shift) (PRO) or x, then split; the border stays 0 (the
// reference pads the BN+ReLU output: models/base/layers.py:45-50).
// NP = 2 (2xfp16): the pieces of v * asc.  DUAL: also the 3-piece 6xbf16 image of v into dst3
// (the 2xfp16 forward's conv input, kept for the 6xbf16 weight gradient: one read, two images).
template <int NP, bool PRO, bool DUAL = false>
__global__ void __launch_bounds__(256) split_act_kernel(const float* __restrict__ x, int C, int H, int W,
                                                       const float* __restrict__ pscale,
                                                       const float* __restrict__ pshift, int pad,
                                                       uint16_t* __restrict__ dst, int64_t plane, float asc,
                                                       uint16_t* __restrict__ dst3, int64_t plane3) {
    const int Hp = H + 2 * pad, Wp = W + 2 * pad, G = C >> 4;
    const int b = blockIdx.z, g = blockIdx.y;
    const int pix = blockIdx.x * 256 + threadIdx.x;
    if (pix >= Hp * Wp) return;
    const int hp = pix / Wp, wq = pix - hp * Wp;
    const int h = hp - pad, w = wq - pad;
    const bool in = h >= 0 && h < H && w >= 0 && w < W;
    const int64_t HW = (int64_t)H * W;
    const float* src = x + ((int64_t)b * C + 16 * g) * HW + (in ? h * W + w : 0);
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = src[j * HW];
    if (PRO) {
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = fmaxf(fmaf(v[j], pscale[16 * g + j], pshift[16 * g + j]), 0.f);
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = in ? v[j] : 0.f;
    const int64_t o = (((int64_t)(b * G + g) * Hp + hp) * Wp + wq) * 16;
    ubpl::store_psa_row<NP>(v, dst + o, plane, NP == 2 ? asc : 1.f);
    if constexpr (DUAL) ubpl::store_psa_row<3>(v, dst3 + o, plane3);
}

// ------------------------------------------------------------------ the stem on the split path
// Space-to-depth: the 7x7 stride-2 pad-3 stem conv (models/pose/hourglass.py
// pre.0, models/base/layers.py:31-50) = a stride-1 4x4 conv over the 4 phase
// images x'[c*4 + 2ph + pw][i][j] = x[c][2i + ph][2j + pw] with taps
// (a, b) in 0..3 at offsets (a - 2, b - 2) and the kernel
// w'[o][c*4 + 2ph + pw][a][b] = w[o][c][2(a - 2) + ph + 3][2(b - 2) + pw + 3]
// (zero outside the 7x7 window): K = 16 channels x 16 taps on the split path
// instead of 147 on the exact-f32 kernel.  The phase image goes straight to the
// PSA layout (C*4 <= 16 channels, the rest zero) with a `pad` border.
template <int NP>
__global__ void __launch_bounds__(256) stem_s2d_split_kernel(const float* __restrict__ x, int C, int H, int W,
                                                            int pad, uint16_t* __restrict__ dst, int64_t plane) {
    const int Ho = H / 2, Wo = W / 2;
    const int Hp = Ho + 2 * pad, Wp = Wo + 2 * pad;
    const int b = blockIdx.y;
    const int pix = blockIdx.x * 256 + threadIdx.x;
    if (pix >= Hp * Wp) return;
    const int hp = pix / Wp, wq = pix - hp * Wp;
    const int i = hp - pad, j = wq - pad;
    const bool in = i >= 0 && i < Ho && j >= 0 && j < Wo;
    float v[16];
#pragma unroll
    for (int ch = 0; ch < 16; ++ch) {
        const int c = ch >> 2, ph = (ch >> 1) & 1, pw = ch & 1;
        const bool ok = in && c < C;
        const int64_t off = (((int64_t)b * C + (ok ? c : 0)) * H + (ok ? 2 * i + ph : 0)) * W + (ok ? 2 * j + pw : 0);
        const float t = x[off];
        v[ch] = ok ? t : 0.f;
    }
    ubpl::store_psa_row<NP>(v, dst + (((int64_t)b * Hp + hp) * Wp + wq) * 16, plane);
}

// w [Cout][C][KS][KS] (KS odd, stride 2, pad KS/2) -> the split, grouped
// tap-major weights of the s2d conv: [piece][Cout][KT*KT taps][16 channels]
// (KT = 4 for KS = 7): tap (a, b) of phase (ph, pw) is w[.][.][2(a - KT/2) +
// ph + KS/2][2(b - KT/2) + pw + KS/2], zero outside the KSxKS window.
template <int NP>
__global__ void __launch_bounds__(256) stem_weight_s2d_split_kernel(const float* __restrict__ w, int Cout, int C,
                                                                   int KS, int KT, uint16_t* __restrict__ dst,
                                                                   int64_t plane) {
    const int64_t total = (int64_t)Cout * KT * KT * 16;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= total) return;
    const int ch = (int)(idx % 16);
    const int tap = (int)((idx / 16) % (KT * KT));
    const int o = (int)(idx / (16 * KT * KT));
    const int a = tap / KT, bb = tap - a * KT;
    const int c = ch >> 2, ph = (ch >> 1) & 1, pw = ch & 1;
    const int kh = 2 * (a - KT / 2) + ph + KS / 2, kw = 2 * (bb - KT / 2) + pw + KS / 2;
    const bool ok = c < C && kh >= 0 && kh < KS && kw >= 0 && kw < KS;
    float v = ok ? w[(((int64_t)o * C + c) * KS + kh) * KS + kw] : 0.f;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const __bf16 hv = (__bf16)v;
        dst[(int64_t)p * plane + idx] = __builtin_bit_cast(uint16_t, hv);
        v -= (float)hv;
    }
}

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

// Forward conv (stride 1) over PSA activations and split weights, both staged
// global -> LDS by LDS-DMA (global_load_lds_dwordx4: no staging registers, no
// VALU), BK = 16 = one (channel group, tap) per K step.  LDS stage image:
// [piece][row][2 x 16 B] for A (BM rows) then B (128 rows); a DMA instruction
// fills 32 rows lane-linearly (lane L: row L>>1, slot L&1), so the chunk
// swizzle c ^ ((row >> 3) & 1) (conflict-free ds_read_b128 of a 32-row
// fragment) is applied on the SOURCE address and again on the read.  Wave w
// moves rows 32w..32w+31 of both operands.  3-stage ring: stage t+2 is issued
// right after the barrier that retires stage t (each wave's counted vmcnt
// leaves stage t+1's DMA in flight; raw s_barrier, never __syncthreads, whose
// fence would drain it: cdna_hip_programming.md §5 'Pipelining across barriers').
template <int N>
__device__ __forceinline__ void vm_wait() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// EPI: the opt-in BatchNorm-partials epilogues (UBPL_FWD_EPI / UBPL_BWD_EPI)
// are compiled in; without them the kernel needs no scratch (the epilogue's
// register pressure spilled ~190 VGPRs to scratch in every launch).
// KSUB: 16-k steps per stage and barrier (1; 2-4 on the one-piece bf16 path,
// whose single MFMA per tile per 16-k step left the loop bound by the ring's
// barriers and waits: KSUB steps of MFMAs between two barriers)
template <int BM, int KS, int NP, int BNT = 128, int WGM = 2, bool EPI = false, int KSUB = 1>
__global__ void __launch_bounds__(NT, 2) conv_psa_kernel(const uint16_t* __restrict__ xs, int64_t xplane,
                                                        const uint16_t* __restrict__ wp, int64_t wplane,
                                                        const float* __restrict__ bias, const float* res, float* y,
                                                        int B, int Cin, int H, int W, int pad, int Cout, int kchunk,
                                                        float* __restrict__ slab, float* __restrict__ stat_part,
                                                        ubpl::BnBwdEpi bwd, float osc,
                                                        const float* __restrict__ ascp) {
    // osc: the accumulators' scale (2xfp16: weight scale x activation scale, the latter
    // read from *ascp when the image's scale lives on the device — a data gradient's,
    // bn.hip fp16_scale_for; 1 on the other paths)
    if (ascp != nullptr) osc *= *ascp;
    constexpr int PADK = KS / 2;   // odd KS: centred; even KS (the stem, 4x4): taps -KS/2 .. KS/2 - 1
    constexpr int T = KS * KS;
    // waves: WGM along the output channels x 4/WGM along the pixels (64-row
    // tiles on 256 pixels: 1 x 4, wave tile 64 x 64)
    constexpr int WGN = 4 / WGM;
    constexpr int TM = BM / WGM / 32, TN = BNT / WGN / 32;
    constexpr int AB = NP * BM * 32, BB = NP * BNT * 32;   // bytes per stage
    // 128-pixel tiles: 3-stage ring; 256-pixel tiles (wave tile 64 x 128, twice
    // the MFMAs per barrier and per fragment byte): 2 stages, 2 workgroups per CU
    constexpr int NS = BNT == 256 ? 2 : 3;
    constexpr int BQ = BNT / 128;                          // B DMA instructions per wave per piece
    constexpr int SB = AB + BB;                            // one 16-k step's image
    __shared__ __attribute__((aligned(16))) char lds[NS * KSUB * SB];

    const int P = H * W, Hp = H + 2 * pad, Wp = W + 2 * pad, G = Cin >> 4;
    const int64_t N = (int64_t)B * P;
    const int Ktot = Cin * T;
    // (wid wave-uniform in an SGPR: the DMA index math stays scalar)
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int dw = wid;                                    // the wave's share of the DMA pieces
    const int wm = (wid / WGN) * (BM / WGM), wn = (wid % WGN) * (BNT / WGN);
    const int lam = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                              gridDim.x * gridDim.y * gridDim.z);
    const int by = lam % gridDim.y, bx = (lam / gridDim.y) % gridDim.x, bz = lam / (gridDim.y * gridDim.x);
    const int m0 = by * BM;
    const int64_t n0 = (int64_t)bx * BNT;
    const int k_begin = bz * kchunk;
    const int k_end = min(Ktot, k_begin + kchunk);

    // DMA lane geometry
    const int lr = lane >> 1;
    const int lchunk = (lane & 1) ^ ((lr >> 3) & 1);
    const bool a_issue = BM / 32 >= NT / 64 || dw < BM / 32;   // every wave when BM >= 128
    // per-lane 32-bit byte offsets over wave-uniform bases (scalar + vector
    // addressing: no 64-bit VALU per DMA instruction)
    const uint32_t a_lane = (uint32_t)(((int64_t)min(m0 + 32 * dw + lr, Cout - 1) * Ktot + 8 * lchunk) * 2);
    uint32_t b_lane[BQ];   // wave w moves pixel rows 32*(BQ*w + q) .. +31
#pragma unroll
    for (int q = 0; q < BQ; ++q) {
        int64_t n = n0 + 32 * (BQ * dw + q) + lr;
        n = n < N ? n : N - 1;
        const int b = (int)(n / P);
        const int p = (int)(n - (int64_t)b * P);
        const int oh = p / W, ow = p - oh * W;
        b_lane[q] =
            (uint32_t)(((((int64_t)b * G * Hp + oh + pad - PADK) * Wp + ow + pad - PADK) * 16 + 8 * lchunk) * 2);
    }
    // DMA piece d (0 .. NP*(1+BQ)-1) of stage (buf, kt): d = p*(1+BQ) + 0 -> A piece p,
    // d = p*(1+BQ) + 1 + q -> B piece p, row block q
    constexpr int NDMA = NP * (1 + BQ);
    // buf: the 16-k step's image slot (stage * KSUB + sub-step)
    auto stage_piece = [&](int buf, int kt, int d) {
        const int kg = kt >> 4;
        const int tap = kg % T, cg = kg / T;
        const int kh = tap / KS, kw = tap - kh * KS;
        const int64_t boff = ((int64_t)cg * Hp + kh) * Wp * 16 + kw * 16;
        char* base = lds + buf * SB;
        const int p = d / (1 + BQ), r = d % (1 + BQ);
        if (r == 0) {
            const char* ab = reinterpret_cast<const char*>(wp + p * wplane + kt);
            if (a_issue)
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)(ab + a_lane),
                                                 (lds_ptr_t)(base + p * BM * 32 + dw * 1024), 16, 0, 0);
        } else {
            const int q = r - 1;
            const char* bb = reinterpret_cast<const char*>(xs + p * xplane + boff);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bb + b_lane[q]),
                                             (lds_ptr_t)(base + AB + p * BNT * 32 + (BQ * dw + q) * 1024), 16, 0,
                                             0);
        }
    };
    // stage sb: its KSUB 16-k steps (those before k_end)
    auto stage = [&](int buf, int sb) {
#pragma unroll
        for (int u = 0; u < KSUB; ++u) {
            const int kt = k_begin + (sb * KSUB + u) * 16;
            if (KSUB == 1 || kt < k_end) {
#pragma unroll
                for (int d = 0; d < NDMA; ++d) stage_piece(buf * KSUB + u, kt, d);
            }
        }
    };

    const int nk16 = (k_end - k_begin) >> 4;               // 16-k steps
    const int nkt = (nk16 + KSUB - 1) / KSUB;              // stages

    // accumulators start at bias (+ residual): see conv.hip conv_fwd_kernel
    const int li = lane & 31, h = lane >> 5;
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
    ubpl::seed_acc<TM, TN, true>(acc, direct ? bias : nullptr, direct ? res : nullptr, obase, m0 + wm, Cout, P, osc);
    const float inv = 1.f / osc;

    if (nkt > 0) stage(0, 0);
    if (NS == 3 && nkt > 1) stage(1, 1);
    for (int t = 0; t < nkt; ++t) {
        // retire stage t (this wave's DMA), then the barrier: every wave's
        // stage t has landed and every wave is done reading stage t-1
        if (NS == 3 && t + 1 < nkt && (KSUB == 1 || (t + 2) * KSUB <= nk16)) {
            if (a_issue) vm_wait<KSUB * (NP + BQ * NP)>();
            else vm_wait<KSUB * BQ * NP>();
        } else {
            vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (t + NS - 1 < nkt) stage((t + NS - 1) % NS, t + NS - 1);
#pragma unroll
        for (int u = 0; u < KSUB; ++u) {
        if (KSUB > 1 && (t * KSUB + u) >= nk16) break;
        const int cur = t % NS;
        const char* base = lds + (cur * KSUB + u) * SB;
        bf16x8 af[TM][NP], bfr[TN][NP];
        auto read_b = [&](int j) {
            const int row = wn + 32 * j + li;
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                bfr[j][p] = *reinterpret_cast<const bf16x8*>(base + AB + p * BNT * 32 + row * 32 +
                                                            16 * (h ^ ((row >> 3) & 1)));
            }
        };
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int row = wm + 32 * i + li;
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                af[i][p] = *reinterpret_cast<const bf16x8*>(base + p * BM * 32 + row * 32 + 16 * (h ^ ((row >> 3) & 1)));
            }
        }
        if constexpr (NP >= 2 && TN > 2) {
            // ping-pong chunks: tile q's 6-MFMA chain is issued with tile q-1's
            // 16 drain adds between its MFMAs (3 VALU slots per MFMA gap), so the
            // adds hide in the matrix pipe's gaps instead of trailing each chain
#pragma unroll
            for (int j = 0; j < TN / 2; ++j) read_b(j);
            __builtin_amdgcn_sched_barrier(0);
            floatx16 prev = mfma_split0<NP>(af[0], bfr[0]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = TN / 2; j < TN; ++j) read_b(j);
#pragma unroll
            for (int q = 1; q < TM * TN; ++q) {
                const int j = q / TM, i = q % TM, pj = (q - 1) / TM, pi = (q - 1) % TM;
                const floatx16 cur = mfma_split0<NP>(af[i], bfr[j]);
                drain(acc[pi][pj], prev);
                pp_schedule<NP>();
                prev = cur;
            }
            drain(acc[TM - 1][TN - 1], prev);
        } else if constexpr (NP >= 2) {
#pragma unroll
            for (int j = 0; j < TN; ++j) read_b(j);
            // every tile's chunk chain first, the f32 adds after them (behind a
            // scheduling barrier): an add right behind its own chain waits out
            // the MFMA latency (s_nop) with the other tiles' chains not issued
            floatx16 tmp[TM][TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    tmp[i][j] = mfma_split0<NP>(af[i], bfr[j]);
                }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) drain(acc[i][j], tmp[i][j]);
        } else {
#pragma unroll
            for (int j = 0; j < TN; ++j) read_b(j);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) mfma_split<NP>(acc[i][j], af[i], bfr[j]);
        }
        }   // sub-steps
        // fragments consumed (the MFMAs waited on them) before the next barrier
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    if (slab != nullptr) {
        float* sl = slab + (int64_t)bz * Cout * N;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t n = n0 + wn + 32 * j + li;
            if (n >= N) continue;
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                    if (m < Cout) sl[(int64_t)m * N + n] = acc[i][j][r] * inv;
                }
        }
        return;
    }
    if (EPI && stat_part) ubpl::tile_bn_partials<TM, TN>(acc, nok, m0 + wm, Cout, n0 + wn, N, stat_part);
    if (EPI && bwd.part) ubpl::tile_bn_bwd_partials<TM, TN>(acc, nok, obase, m0 + wm, Cout, P, n0 + wn, N, bwd);
    store_tile<TM, TN>(acc, nok, obase, m0 + wm, Cout, P, y, m0 + BM <= Cout && n0 + BNT <= N, inv);
}

// ------------------------------------------------------------------ 3x3, input halo staged once per channel group
// The 3x3 stride-1 conv over PSA activations (pad 1: the PSA image's own zero
// border is the conv padding) with the B operand staged ONCE per 16-channel
// group instead of once per (group, tap): a workgroup's 256-pixel tile is
// R = 256 / W whole output rows of one image, whose 3x3 receptive field is
// PSA rows oh0 .. oh0 + R + 1 x all W + 2 columns — one contiguous
// (R + 2) (W + 2) x 32 B run per piece, copied by LDS-DMA as it lies.  The
// nine taps then read their B fragments from that halo image at a per-tap
// pixel offset (kh (W + 2) + kw).  conv_psa_kernel moves 9 x 256 pixels per
// group; this kernel (R + 2)(W + 2) (396 at W = 64: 5.8x fewer B bytes through
// the CU's L2 -> LDS path, 2.2x fewer bytes per K step in all, the weights
// included).  Weights: the A ring of conv_psa_kernel (3 stages, one per K step
// = (group, tap)); halo images double-buffered per group: the next group's
// halo is issued at the group's tap 0 and retired by tap 3 (counted vmcnt).
// One workgroup per CU (LDS 85-160 KB); BM 128: wave tile 64 x 128 (as
// conv_psa_kernel<128, 3, NP, 256, 2>), BM 64: 64 x 64 (4 waves along the
// pixels, as conv_psa_kernel<64, 3, NP, 256, 1>); the same ping-pong drains.
// Halo chunk swizzle as conv_psa_kernel's rows: pixel q's two 16-B halves
// swapped when (q >> 3) & 1 (applied on the DMA source and on the read).
// NHB = 1 (6xbf16, one team): ONE halo buffer and two workgroups per CU (<= 80 KB
// each): the next group's halo is loaded after every wave finished the group's last
// tap (a second barrier then), the partner workgroup's MFMAs covering that bubble.
// BNT1: pixels per team tile — 256, or 192 for the 96-wide planes (two rows; 128-row
// tiles only: wave tile 64 x 96, three 32-pixel fragments)
template <int WW, int NP, int BM, int TEAMS = 1, int NHB = 2, int BNT1 = 256>
__global__ void __launch_bounds__(NT * TEAMS, (NHB == 1 || (NP == 2 && TEAMS == 1)) ? 2 : 1) conv_psah_kernel(const uint16_t* __restrict__ xs, int64_t xplane,
                                                        const uint16_t* __restrict__ wp, int64_t wplane,
                                                        const float* __restrict__ bias, const float* res, float* y,
                                                        int B, int Cin, int H, int Cout, float osc,
                                                        const float* __restrict__ ascp) {
    if (ascp != nullptr) osc *= *ascp;   // (see conv_psa_kernel)
    constexpr int BNT = BNT1 * TEAMS, R = BNT / WW, W2 = WW + 2;
    static_assert(BNT1 == 256 || (BNT1 == 192 && BM == 128), "192-pixel tiles: 128 rows");
    constexpr int NW = 4 * TEAMS;              // waves (TEAMS 4-wave teams, one 256-pixel tile each)
    constexpr int HPX = (R + 2) * W2;          // halo pixels
    constexpr int HI = (HPX + 31) / 32;        // DMA instructions per piece (32 pixels each)
    constexpr int HB = HPX * 32;               // halo image bytes per piece (exact: the last chunk of a
                                               // piece starts at HPX - 32, rewriting pixels it overlaps)
    constexpr int HTOT = NP * HI;
    constexpr int NH = (HTOT + NW - 1) / NW;   // halo DMA instructions per wave (spares repeat the last one)
    constexpr int AB = NP * BM * 32;           // A bytes per K step
    constexpr int AI = AB / 1024;              // A DMA instructions per K step (1 KB each)
    constexpr int NAW = (AI + NW - 1) / NW;    // per wave (spares repeat the last one)
    // GS (the one-piece path): a stage is a whole channel group — its halo and the
    // nine taps' A images (one barrier per 9 K steps; 8 MFMAs per wave per K step
    // left the per-step ring bound by its barriers); NS_G slots.  Otherwise A per
    // K step in an NA-stage ring, halos double-buffered (NHB = 2) or one buffer
    // reloaded at each group boundary (NHB = 1).
    constexpr bool GS = NP == 1;
    constexpr int NS_G = 3 * (NP * HB + 9 * AB) <= 160 * 1024 ? 3 : 2;
    static_assert(NHB == 2 || (!GS && TEAMS == 1), "one halo buffer: split pieces, one team");
    // (one halo buffer: as many A stages, 2 .. UBPL_PSAH_NA_MAX, as fit two workgroups per CU)
    constexpr int NA1 = UBPL_PSAH_NA_MAX * AB + NP * HB <= 80 * 1024 ? UBPL_PSAH_NA_MAX
                        : (3 * AB + NP * HB <= 80 * 1024 ? 3 : 2);
    constexpr int NA = GS ? 9 * NS_G : (NHB == 1 ? NA1 : 3);   // A images
    constexpr int WGM = BM / 64, WGN = 4 / WGM;
    constexpr int TM = 2, TN = BNT1 / WGN / 32;
    static_assert(BM == 64 || BM == 128, "64- or 128-row tiles");
    constexpr int OFF_H = NA * AB, LDS_BYTES = OFF_H + (GS ? NS_G : NHB) * NP * HB;
    static_assert(LDS_BYTES <= 160 * 1024, "LDS");
    static_assert(BNT % WW == 0 && WW % 32 == 0, "whole rows of 32-pixel fragments");
    __shared__ __attribute__((aligned(16))) char lds[LDS_BYTES];

    const int P = H * WW, Hp = H + 2, G = Cin >> 4;
    const int64_t N = (int64_t)B * P;
    const int Ktot = Cin * 9;
    // (wid wave-uniform in an SGPR: the DMA index math below stays scalar)
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = ((wid & 3) / WGN) * 64, wn = (wid >> 2) * BNT1 + ((wid & 3) % WGN) * (BNT1 / WGN);
    const int lam = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
    const int by = lam % gridDim.y, bx = lam / gridDim.y;
    const int m0 = by * BM;
    const int64_t n0 = (int64_t)bx * BNT;
    const int tpi = H / R;                     // tiles per image
    const int b = bx / tpi, oh0 = (bx - b * tpi) * R;

    const int lr = lane >> 1;
    const int lchunk = (lane & 1) ^ ((lr >> 3) & 1);
    // A instruction i = u * NW + wid: piece i / (BM / 32), rows 32 (i % (BM / 32)) .. —
    // the row block depends on the wave only (NW % (BM / 32) == 0): one lane offset
    static_assert(NW % (BM / 32) == 0, "row block per wave");
    const uint32_t a_lane = (uint32_t)(((int64_t)min(m0 + 32 * (wid % (BM / 32)) + lr, Cout - 1) * Ktot +
                                        8 * lchunk) * 2);
    auto stage_a = [&](int slot, int s) {
        const char* base = reinterpret_cast<const char*>(wp + s * 16);
#pragma unroll
        for (int u = 0; u < NAW; ++u) {
            // (a spare repeats the last piece's instruction for the same row block: same bytes)
            const int i = u * NW + wid < AI ? u * NW + wid : (NP - 1) * (BM / 32) + wid % (BM / 32);
            const int p = i / (BM / 32), rb = i % (BM / 32);
            char* dst = lds + slot * AB + p * BM * 32 + rb * 1024;
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(base + (int64_t)p * wplane * 2 + a_lane),
                                             (lds_ptr_t)dst, 16, 0, 0);
        }
    };
    // halo of group cg: instruction i = wid * NH + u (piece i / HI, 32-pixel chunk i % HI)
    auto stage_h = [&](int buf, int cg) {
        const int64_t gpx = (((int64_t)b * G + cg) * Hp + oh0) * W2;   // first halo pixel (PSA pixel index)
        // (the lane terms made opaque here: otherwise the compiler keeps all NH per-lane
        // source offsets live across the K loop, ~20 VGPRs, and spills the tile)
        int lr = lane >> 1, lo = lane & 1;
        asm volatile("" : "+v"(lr), "+v"(lo));
#pragma unroll
        for (int u = 0; u < NH; ++u) {
            const int i = min(wid * NH + u, HTOT - 1);  // (a spare repeats the last: same bytes)
            const int p = i / HI, c0 = min((i - p * HI) * 32, HPX - 32);
            const int q = c0 + lr;
            const int ch = lo ^ ((q >> 3) & 1);
            const char* src = reinterpret_cast<const char*>(xs + p * xplane + (gpx + q) * 16) + ch * 16;
            char* dst = lds + OFF_H + (buf * NP + p) * HB + c0 * 32;
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)src, (lds_ptr_t)dst, 16, 0, 0);
        }
    };

    const int li = lane & 31, h = lane >> 5;
    // output offsets: computed for the seed and again for the stores (not live
    // across the K loop: register budget of the two-team variant)
    auto out_base = [&](int64_t (&obase)[TN], bool (&nok)[TN]) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t n = n0 + wn + 32 * j + li;
            nok[j] = n < N;
            const int64_t nc = nok[j] ? n : N - 1;
            const int bb = (int)(nc / P);
            const int pp = (int)(nc - (int64_t)bb * P);
            obase[j] = (int64_t)bb * Cout * P + pp;
        }
    };
    // halo pixel of tap (0, 0) for tile-local output pixel nt: row nt / WW, column nt % WW
    const int nt0 = wn + li;
    floatx16 acc[TM][TN];
    {
        int64_t obase[TN];
        bool nok[TN];
        out_base(obase, nok);
        ubpl::seed_acc<TM, TN, true>(acc, bias, res, obase, m0 + wm, Cout, P, osc);
    }

    // one K step (group cg's tap at pixel offset toff): fragments from the A image
    // at abase and the halo image at hbase
    auto step = [&](const char* abase, const char* hbase, int toff) {
        bf16x8 af[TM][NP], bfr[TN][NP];
        auto read_b = [&](int j) {
            const int nt = nt0 + 32 * j;
            const int q = nt + (nt / WW) * 2 + toff;
            const char* rp = hbase + q * 32 + 16 * (h ^ ((q >> 3) & 1));
#pragma unroll
            for (int p = 0; p < NP; ++p) bfr[j][p] = *reinterpret_cast<const bf16x8*>(rp + p * HB);
        };
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int row = wm + 32 * i + li;
#pragma unroll
            for (int p = 0; p < NP; ++p)
                af[i][p] = *reinterpret_cast<const bf16x8*>(abase + p * BM * 32 + row * 32 + 16 * (h ^ ((row >> 3) & 1)));
        }
        if constexpr (NP == 1) {
            // one MFMA per tile, accumulated directly (conv_psa_kernel's one-piece path)
#pragma unroll
            for (int j = 0; j < TN; ++j) read_b(j);
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) mfma_split<NP>(acc[i][j], af[i], bfr[j]);
        } else {
            // ping-pong chunks (conv_psa_kernel): tile q's chain with tile q-1's drain adds in its gaps
#pragma unroll
            for (int j = 0; j < TN / 2; ++j) read_b(j);
            __builtin_amdgcn_sched_barrier(0);
            floatx16 prev = mfma_split0<NP>(af[0], bfr[0]);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int j = TN / 2; j < TN; ++j) read_b(j);
#pragma unroll
            for (int q = 1; q < TM * TN; ++q) {
                const int j = q / TM, i = q % TM, pj = (q - 1) / TM, pi = (q - 1) % TM;
                const floatx16 cur = mfma_split0<NP>(af[i], bfr[j]);
                drain(acc[pi][pj], prev);
                pp_schedule<NP>();
                prev = cur;
            }
            drain(acc[TM - 1][TN - 1], prev);
        }
    };

    if constexpr (GS) {
        // one stage per channel group (halo + the nine taps' A images), NS_G-slot
        // ring, one barrier per group
        auto stage_g = [&](int slot, int cg) {
            stage_h(slot, cg);
#pragma unroll
            for (int tp = 0; tp < 9; ++tp) stage_a(slot * 9 + tp, cg * 9 + tp);
        };
        for (int c = 0; c < NS_G - 1 && c < G; ++c) stage_g(c, c);
        for (int cg = 0; cg < G; ++cg) {
            // group cg landed; (3 slots) group cg+1 may stay in flight
            if (NS_G == 3 && cg + 1 < G) vm_wait<NH + 9 * NAW>();
            else vm_wait<0>();
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (cg + NS_G - 1 < G) stage_g((cg + NS_G - 1) % NS_G, cg + NS_G - 1);
            const int slot = cg % NS_G;
            const char* hbase = lds + OFF_H + slot * NP * HB;
#pragma unroll 1
            for (int tp = 0; tp < 9; ++tp) {
                const int kh = tp / 3;
                step(lds + (slot * 9 + tp) * AB, hbase, kh * W2 + (tp - 3 * kh));
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    } else {
        const int nk = G * 9;
        stage_h(0, 0);
        for (int a = 0; a < NA - 1 && a < nk; ++a) stage_a(a, a);
        for (int s = 0; s < nk; ++s) {
            const int cg = s / 9, tap = s - cg * 9;
            if (NHB == 1 && tap == 0 && cg > 0) {
                // every wave done with group cg - 1: reload the one halo buffer, wait for it
                vm_wait<(NA - 2) * NAW>();
                __builtin_amdgcn_s_barrier();
                asm volatile("" ::: "memory");
                stage_h(0, cg);
                vm_wait<0>();
            } else if (NHB == 1) {
                if (s + 1 < nk) vm_wait<(NA - 2) * NAW>();
                else vm_wait<0>();
            } else if (s + 1 < nk) {
                // A(s) and (tap 0) halo(cg) landed; the A images issued after A(s) (NA - 2
                // of them) and the next group's halo, when issued after A(s), may stay in flight
                if (tap >= 1 && tap <= NA - 1 && cg + 1 < G) vm_wait<(NA - 2) * NAW + NH>();
                else vm_wait<(NA - 2) * NAW>();
            } else {
                vm_wait<0>();
            }
            __builtin_amdgcn_s_barrier();
            asm volatile("" ::: "memory");
            if (s + NA - 1 < nk) stage_a((s + NA - 1) % NA, s + NA - 1);
            if (NHB == 2 && tap == 0 && cg + 1 < G) stage_h((cg + 1) & 1, cg + 1);
            const int kh = tap / 3;
            step(lds + (s % NA) * AB, lds + OFF_H + (NHB == 2 ? (cg & 1) : 0) * NP * HB, kh * W2 + (tap - 3 * kh));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
    }

    int64_t obase[TN];
    bool nok[TN];
    out_base(obase, nok);
    store_tile<TM, TN>(acc, nok, obase, m0 + wm, Cout, P, y, m0 + BM <= Cout && n0 + BNT <= N, 1.f / osc);
}

// ------------------------------------------------------------------ 1x1, split on load
// y[b,m,p] = sum_k w[m][k] v[b,k,p] + bias[m] (+ res), v = relu(x*pscale +
// pshift) (PRO) or x, on the 6xbf16 path without a pre-split operand: the f32
// activations (NCHW) go global -> LDS by LDS-DMA as the 16 k rows of a
// 256-pixel tile (1 KB each; rows 8-15 shifted 128 B so the two 32-lane halves
// of a fragment read sit in opposite bank halves), and each wave reads its own
// pixels' B fragments from that f32 image (lane (n, h): k = 8h..8h+7 of pixel
// n, 8 ds_read_b32), applies the prologue and splits into 3 bf16 pieces in
// registers.  Waves split the tile along pixels (wave w: all BM rows x pixels
// 64w..64w+63), so each value is split once per workgroup.  Weights: 3 bf16
// planes of [M][K] (ubpl_conv_weights_split with KS = 1), staged as in
// conv_psa_kernel.  2-stage ring, 2 workgroups per CU.  The activation read is
// the f32 tensor itself: no split pass, no 6-byte/element PSA image.
// BNT: pixels per tile, 256 (wave w: pixels 64w..64w+63) or 128 (32 per wave: half the
// LDS and accumulators, three workgroups per CU, so one workgroup's epilogue stores run
// beside the others' K loops)
template <int BM, bool PRO, bool EPI = false, int NP = 3, int NS = 2, int BNT = 256, int NSB = NS>
__global__ void __launch_bounds__(NT, BNT == 128 ? 3 : UBPL_SOL_LB) conv1x1_sol_kernel(const float* __restrict__ x,
                                                           const uint16_t* __restrict__ wp, int64_t wplane,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ pscale,
                                                           const float* __restrict__ pshift, const float* res,
                                                           float* y, int B, int K, int P, int M,
                                                           float* __restrict__ stat_part, ubpl::BnBwdEpi bwd,
                                                           float asc, float osc) {
    // NP = 3: 6xbf16 (f32-equivalent); NP = 2: 2xfp16 (activations scaled by asc after the
    // prologue, accumulators by osc = weight scale x asc, undone at the stores); NP = 1: the
    // "bf16" precision (operands rounded to bf16, one MFMA per product, accumulated in f32)
    // NS: stages in the LDS ring (2, or 3 with 64-row tiles: two K steps' DMA in flight);
    // NSB = 3 with NS = 2: a deeper ring for the activation stream alone (HBM: two K
    // steps of it in flight per workgroup) beside the weights' two stages (L2-resident)
    static_assert(BNT == 256 || BNT == 128, "256- or 128-pixel tiles");
    static_assert(NSB == NS || (NS == 2 && NSB == 3), "B ring: as deep as A's, or 3 beside A's 2");
    constexpr int TM = BM / 32, TN = BNT / 128;
    constexpr int BQ = BNT / 64;             // B DMA instructions per wave per K step (1 KB each)
    constexpr int AB = NP * BM * 32;         // A stage bytes: [piece][BM rows][32 B]
    constexpr int BH = 8 * BNT * 4 + 128;    // one 8-row half of the B image (+ bank shift)
    constexpr int BB = 2 * BH;
    __shared__ __attribute__((aligned(16))) char lds[NS * AB + NSB * BB];   // A slots, then B slots
    // the prologue's (scale, shift) per input channel (K <= SOL_PRO_K), staged once:
    // a lane's 8 channels of a K step are 2 ds_read_b128 each, instead of scalar
    // loads of both 8-channel halves and 16 per-lane selects (48 VALU per K step)
    __shared__ __attribute__((aligned(16))) float lds_sc[PRO ? SOL_PRO_K : 4], lds_sh[PRO ? SOL_PRO_K : 4];

    const int64_t N = (int64_t)B * P;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // (wave-uniform: SGPR)
    const int wn = (BNT / 4) * wid;
    if (PRO) {
        for (int k = tid; k < K; k += NT) {
            lds_sc[k] = pscale[k];
            lds_sh[k] = pshift[k];
        }
        // a full barrier (waits for the LDS stores): the K loop's raw s_barrier does
        // not, and without it a wave could read another wave's coefficients of the
        // first K step before they land (before any DMA is issued: costs no overlap)
        __syncthreads();
    }
    const int lam = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
    const int by = lam % gridDim.y, bx = lam / gridDim.y;
    const int m0 = by * BM;
    const int64_t n0 = (int64_t)bx * BNT;

    // A DMA (as conv_psa_kernel): wave w < BM/32 moves rows 32w..32w+31 of each piece
    const int lr = lane >> 1;
    const int lchunk = (lane & 1) ^ ((lr >> 3) & 1);
    const bool a_issue = BM / 32 >= NT / 64 || wid < BM / 32;   // every wave when BM >= 128
    const uint32_t a_lane = (uint32_t)(((int64_t)min(m0 + 32 * wid + lr, M - 1) * K + 8 * lchunk) * 2);
    // B DMA: wave w moves k rows 4w..4w+3; 256-pixel tiles: one row per instruction,
    // lane L pixels n0 + 4L .. +3; 128-pixel tiles: two rows per instruction, lanes
    // 32-63 the second (P % 4 == 0)
    uint32_t b_lane;
    {
        const int pl = BNT == 256 ? lane : (lane & 31);
        int64_t n = n0 + 4 * pl;
        n = n < N ? n : N - 4;
        const int64_t b = n / P;
        b_lane = (uint32_t)((b * K * P + (n - b * P) + (BNT == 256 ? 0 : (int64_t)(lane >> 5) * P)) * 4);
    }
    auto stage_a = [&](int buf, int kt) {
        char* base = lds + buf * AB;
        if (a_issue) {
#pragma unroll
            for (int p = 0; p < NP; ++p) {
                const char* ab = reinterpret_cast<const char*>(wp + p * wplane + kt);
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)(ab + a_lane),
                                                 (lds_ptr_t)(base + p * BM * 32 + wid * 1024), 16, 0, 0);
            }
        }
    };
    auto stage_b = [&](int buf, int kt) {
        char* base = lds + NS * AB + buf * BB;
#pragma unroll
        for (int q = 0; q < BQ; ++q) {
            const int r = 4 * wid + q * (4 / BQ);
            const char* bb = reinterpret_cast<const char*>(x + (int64_t)(kt + r) * P);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bb + b_lane),
                                             (lds_ptr_t)(base + (r >> 3) * BH + (r & 7) * (BNT * 4)), 16, 0, 0);
        }
    };
    auto stage = [&](int buf, int kt) {
        stage_a(buf, kt);
        stage_b(buf, kt);
    };

    // accumulators start at bias (+ residual): see conv_psa_kernel
    const int li = lane & 31, h = lane >> 5;
    // output offsets: computed for the seed and again for the epilogue (not live
    // across the K loop: the tile spilled ~30 VGPRs to scratch with them)
    auto out_base = [&](int64_t (&ob)[TN], bool (&ok)[TN]) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int64_t n = n0 + wn + 32 * j + li;
            ok[j] = n < N;
            const int64_t nc = ok[j] ? n : N - 1;
            const int b = (int)(nc / P);
            const int p = (int)(nc - (int64_t)b * P);
            ob[j] = (int64_t)b * M * P + p;
        }
    };
    int64_t obase[TN];
    bool nok[TN];
    out_base(obase, nok);
    floatx16 acc[TM][TN];
    // UBPL_SOL_TEPI (with a residual): the output tile leaves through LDS as
    // float4 rows (8 stores per lane per 32-row block instead of 32 scalar
    // stores) with the residual added there by float4 loads issued ahead of
    // the stores, instead of seeding the accumulators with 128 scalar loads per
    // lane before the K loop (128->256 + skip at 64x64 B=32: 101 -> 91 us);
    // without a residual the scalar epilogue measured faster
    const bool tepi = UBPL_SOL_TEPI && BNT == 256 && !EPI && res != nullptr &&
                      ((((uintptr_t)y) | (uintptr_t)res) & 15) == 0;
    ubpl::seed_acc<TM, TN>(acc, bias, tepi ? nullptr : res, obase, m0, M, P, osc);
    const float inv = 1.f / osc;

    const int nkt = K >> 4;
    constexpr bool deepb = NSB != NS;
    // this lane's k half of K step kt: 8 (scale, shift) pairs of the prologue
    auto load_coef = [&](int kt, float (&sc)[8], float (&sh)[8]) {
        if (PRO) {
            const float4* qs = reinterpret_cast<const float4*>(lds_sc + kt + 8 * h);
            const float4* qh = reinterpret_cast<const float4*>(lds_sh + kt + 8 * h);
            const float4 s0 = qs[0], s1 = qs[1], h0 = qh[0], h1 = qh[1];
            sc[0] = s0.x; sc[1] = s0.y; sc[2] = s0.z; sc[3] = s0.w;
            sc[4] = s1.x; sc[5] = s1.y; sc[6] = s1.z; sc[7] = s1.w;
            sh[0] = h0.x; sh[1] = h0.y; sh[2] = h0.z; sh[3] = h0.w;
            sh[4] = h1.x; sh[5] = h1.y; sh[6] = h1.z; sh[7] = h1.w;
        }
    };
    // this wave's B fragment of pixel column j (32 pixels) from a B stage: 8 f32 per lane,
    // prologue, split into NP bf16 pieces
    auto split_col = [&](const char* bbase, int j, const float (&sc)[8], const float (&sh)[8], bf16x8 (&out)[NP]) {
        const float* bs = reinterpret_cast<const float*>(bbase + h * BH) + wn + li;
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            v[e] = bs[e * BNT + 32 * j];
            if (PRO) v[e] = fmaxf(fmaf(v[e], sc[e], sh[e]), 0.f);
            if constexpr (NP == 2) v[e] *= asc;
        }
        uint32_t pk[NP][4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            uint32_t o[NP];
            split2<NP>(v[2 * e], v[2 * e + 1], o);
#pragma unroll
            for (int p = 0; p < NP; ++p) pk[p][e] = o[p];
        }
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const uint4 u = make_uint4(pk[p][0], pk[p][1], pk[p][2], pk[p][3]);
            out[p] = __builtin_bit_cast(bf16x8, u);
        }
    };
    stage(0, 0);
    if (NS == 3 && nkt > 1) stage(1, 16);
    if (deepb && nkt > 1) stage_b(1, 16);
    for (int t = 0; t < nkt; ++t) {
        // stage t landed for every wave (NS = 3: this wave's stage t+1 DMA may stay in
        // flight; deepb: B(t+1), issued after A(t), may stay in flight), every wave
        // done with stage t-1
        if (NS == 3 && t + 1 < nkt) {
            if (a_issue) vm_wait<NP + BQ>();
            else vm_wait<BQ>();
        } else if (deepb && t + 1 < nkt) {
            vm_wait<BQ>();
        } else {
            vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (deepb) {
            // A(t+1) first, then B(t+2): the next wait leaves only B(t+2) in flight
            if (t + 1 < nkt) stage_a((t + 1) % NS, (t + 1) * 16);
            if (t + 2 < nkt) stage_b((t + 2) % NSB, (t + 2) * 16);
        } else if (t + NS - 1 < nkt) {
            stage((t + NS - 1) % NS, (t + NS - 1) * 16);
        }
        const int kt = t * 16;
        const char* base = lds + (t % NS) * AB;                       // A of stage t
        const char* bbase = lds + NS * AB + (t % NSB) * BB;           // B of stage t
        float sc[8], sh[8];
        load_coef(kt, sc, sh);
        bf16x8 bfr[TN][NP];
#pragma unroll
        for (int j = 0; j < TN; ++j) split_col(bbase, j, sc, sh, bfr[j]);
        if constexpr (NP == 1) {
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int row = 32 * i + li;
                bf16x8 af[NP];
                af[0] = *reinterpret_cast<const bf16x8*>(base + row * 32 + 16 * (h ^ ((row >> 3) & 1)));
#pragma unroll
                for (int j = 0; j < TN; ++j) mfma_split<NP>(acc[i][j], af, bfr[j]);
            }
        } else {
        auto lda = [&](int i, bf16x8 (&o)[NP]) {
            const int row = 32 * i + li;
#pragma unroll
            for (int p = 0; p < NP; ++p)
                o[p] = *reinterpret_cast<const bf16x8*>(base + p * BM * 32 + row * 32 + 16 * (h ^ ((row >> 3) & 1)));
        };
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            bf16x8 af[NP];
            lda(i, af);
#pragma unroll
            for (int j = 0; j < TN; ++j) drain(acc[i][j], mfma_split0<NP>(af, bfr[j]));   // per-chunk accumulation
            // (register budget: one row block's A fragments live at a time)
            __builtin_amdgcn_sched_barrier(0);
        }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    out_base(obase, nok);
    if constexpr (EPI) {
        if (stat_part) ubpl::tile_bn_partials<TM, TN>(acc, nok, m0, M, n0 + wn, N, stat_part);
        if (bwd.part) ubpl::tile_bn_bwd_partials<TM, TN>(acc, nok, obase, m0, M, P, n0 + wn, N, bwd);
    }
    if constexpr (BNT == 256) if (tepi) {
        // every wave is done with the ring (its last reads waited on above); a
        // wave-private [32 rows][64 + 4 pixels] f32 image per 32-row block
        __syncthreads();
        constexpr int RS = 68;
        static_assert(NS * AB + NSB * BB >= 4 * 32 * RS * 4, "transposed epilogue image exceeds the ring");
        float* img = reinterpret_cast<float*>(lds) + wid * 32 * RS;
        const int rr = lane >> 4, c4 = (lane & 15) * 4;
        const int64_t n = n0 + wn + c4;   // 4 pixels of one image (P % 4 == 0)
        const bool ok = n < N;
        const int64_t b = ok ? n / P : 0;
        const int64_t ob = b * M * P + (n - b * P);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            // this block's residual rows first (8 loads in flight, ahead of the
            // stores, which may alias them)
            float4 q[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int m = m0 + 32 * i + rr + 4 * k;
                q[k] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (res != nullptr && ok && m < M) q[k] = *reinterpret_cast<const float4*>(res + ob + (int64_t)m * P);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) img[((r & 3) + 8 * (r >> 2) + 4 * h) * RS + 32 * j + li] = acc[i][j][r];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int row = rr + 4 * k;
                const int m = m0 + 32 * i + row;
                float4 v = *reinterpret_cast<const float4*>(img + row * RS + c4);
                if (ok && m < M) {
                    v.x = fmaf(v.x, inv, q[k].x); v.y = fmaf(v.y, inv, q[k].y);
                    v.z = fmaf(v.z, inv, q[k].z); v.w = fmaf(v.w, inv, q[k].w);
                    *reinterpret_cast<float4*>(y + ob + (int64_t)m * P) = v;
                }
            }
        }
        return;
    }
    store_tile<TM, TN>(acc, nok, obase, m0, M, P, y, m0 + BM <= M && n0 + BNT <= N, inv);
}

// ------------------------------------------------------------------ 3x3 weight gradient
// dW[co][tap][ci] = sum over (b, oh, ow) of dy[b,co,oh,ow] * x[b,ci,oh+kh-1,ow+kw-1]
// on the split path, both operands in the PSA layout with a 1-pixel border
// (dy: the data gradient's own pre-split operand; x: the forward's pre-split
// conv input = relu(bn(t1)), kept for the backward).  GEMM: M = co, N = (tap,
// ci) tap-major (n-tile = one tap x 128 channels), K = pixels, K step = 16
// consecutive pixels of one output row (W % 16 == 0), split over workgroups
// into a slab [z][Cout][9*Cin + 1] reduced by conv.hip's wgrad_reduce_kernel
// (last column: the bias gradient, summed by the tap-0 workgroups).
// The MFMA wants 8 consecutive pixels of one channel per lane, the PSA image
// holds 16 channels per pixel: fragments come from LDS by
// ds_read_b64_tr_b16 (a 16-lane group reads a 4-pixel x 16-channel block,
// lane i gets channel i's 4 pixels), two per 8-bf16 fragment.  LDS stage
// image [piece][16-channel group][16 pixel rows][32 B]; odd groups store
// pixel rows 0-3 <-> 4-7 swapped (pre-permuted DMA source) so the two groups a
// 32-lane half reads sit in opposite 128-B bank halves.
template <int NP, int CB = 128>
__global__ void __launch_bounds__(NT, 2) wgrad3_psa_kernel(const uint16_t* __restrict__ dys, int64_t dplane,
                                                          const uint16_t* __restrict__ xs, int64_t xplane, int B,
                                                          int Cin, int Cout, int H, int W, int steps_per_split,
                                                          float* __restrict__ slab, const float* __restrict__ dscale) {
    // NP = 2 (2xfp16): dys are the fp16 pieces of dy * (*dscale) (bn.hip fp16_scale_for), xs of
    // x * FP16_ACT_SCALE (the forward's image): the slab gets the products unscaled exactly.
    // CB = channel block of both tile sides (128, or 64 for the 64-channel convs:
    // wave tile 32 x 32, waves 0-1 move the operands)
    constexpr int BM = CB, TM = CB / 64, TN = CB / 64, NS = 3;
    constexpr int GR = CB / 16;                            // channel groups per operand tile
    constexpr int PI = GR * 512;                           // piece image: GR groups x 16 px x 32 B
    constexpr int AB = NP * PI, BB = NP * PI;              // bytes per 16-pixel step
    // 64-channel tiles carry two 16-pixel steps per stage (one barrier per 12 MFMA
    // chains instead of 6)
    constexpr int KS2 = CB == 64 ? 2 : 1;
    constexpr int SUB = AB + BB;
    __shared__ __attribute__((aligned(16))) char lds[NS * KS2 * SUB];
    typedef short v4i16 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) v4i16* tr_ptr_t;

    const int Hp = H + 2, Wp = W + 2;
    const int Gci = Cin >> 4, Gco = Cout >> 4;
    const int Ntot = 9 * Cin, Nt = Ntot + 1;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // (wave-uniform: SGPR)
    const int wm = (wid >> 1) * (CB / 2), wn = (wid & 1) * (CB / 2);
    // tile order: n tiles (tap, ci) fastest so the 9 taps of one K split share an L2
    const int lam = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                              gridDim.x * gridDim.y * gridDim.z);
    const int bx = lam % gridDim.x, by = (lam / gridDim.x) % gridDim.y, bz = lam / (gridDim.x * gridDim.y);
    const int m0 = by * BM;
    const int ntile_per_tap = Cin / CB;
    const int tap = bx / ntile_per_tap, ci0 = (bx - tap * ntile_per_tap) * CB;
    const int kh = tap / 3, kw = tap - 3 * (tap / 3);
    const int wsteps = W >> 4;
    const int total_steps = B * H * wsteps;
    const int s_begin = bz * steps_per_split;
    const int s_end = min(total_steps, s_begin + steps_per_split);
    const int nkt = max(0, s_end - s_begin);

    // DMA lane geometry: wave w < GR/2 moves channel groups 2w, 2w+1 of both operands
    const bool d_issue = wid < GR / 2;
    const int gl = 2 * wid + (lane >> 5);
    const int rphys = (lane & 31) >> 1;
    const int rlog = rphys ^ (4 * (gl & 1));
    const int64_t HWp = (int64_t)Hp * Wp;
    // per-lane 32-bit byte offsets; the rest of each DMA address is wave-uniform
    // (scalar base + vector offset addressing, no 64-bit VALU per instruction)
    const uint32_t a_lane = (uint32_t)(((gl * HWp + rlog) * 16 + 8 * (lane & 1)) * 2);
    const uint32_t b_lane = a_lane;
    const char* dys_m = reinterpret_cast<const char*>(dys + (int64_t)(m0 >> 4) * HWp * 16);
    const char* xs_c = reinterpret_cast<const char*>(xs + (int64_t)(ci0 >> 4) * HWp * 16);
    auto stage1 = [&](char* base, int s) {
        const int b = s / (H * wsteps);
        const int rem = s - b * (H * wsteps);
        const int oh = rem / wsteps, ow0 = (rem - oh * wsteps) * 16;
        const int64_t aoff = (int64_t)b * Gco * HWp * 16 + ((int64_t)(oh + 1) * Wp + ow0 + 1) * 16;
        const int64_t boff = (int64_t)b * Gci * HWp * 16 + ((int64_t)(oh + kh) * Wp + ow0 + kw) * 16;
        if (!d_issue) return;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            const char* ab = dys_m + 2 * (p * dplane + aoff);
            const char* bb = xs_c + 2 * (p * xplane + boff);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(ab + a_lane), (lds_ptr_t)(base + p * PI + wid * 1024), 16,
                                             0, 0);
            __builtin_amdgcn_global_load_lds((gbl_ptr_t)(bb + b_lane), (lds_ptr_t)(base + AB + p * PI + wid * 1024),
                                             16, 0, 0);
        }
    };
    auto stage = [&](int buf, int s) {   // steps s .. s + KS2 - 1 (those before s_end)
#pragma unroll
        for (int u = 0; u < KS2; ++u)
            if (s + u < s_end) stage1(lds + (buf * KS2 + u) * SUB, s + u);
    };

    // transposed-read geometry: 16-lane group g reads channel group (tile base
    // + (g & 1)), pixel rows 8*(g >> 1) + 4t + q (q = i16 >> 2), columns 4*(i16 & 3)
    const int g16 = lane >> 4, i16 = lane & 15;
    const int qrow = i16 >> 2, pcol = i16 & 3;
    auto tr_off = [&](int grp, int t) {   // byte offset inside a piece image
        const int row = (8 * (g16 >> 1) + 4 * t + qrow) ^ (4 * (grp & 1));
        return grp * 512 + row * 32 + 8 * pcol;
    };
    int aoffs[TM][2], boffs[TN][2];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int t = 0; t < 2; ++t) aoffs[i][t] = tr_off((wm + 32 * i) / 16 + (g16 & 1), t);
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int t = 0; t < 2; ++t) boffs[j][t] = tr_off((wn + 32 * j) / 16 + (g16 & 1), t);

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    // the bias gradient of split z is summed by the tap (z % 9) workgroups (their
    // first 128 input channels), spreading that VALU work over the taps
    const bool bias_wave = tap == bz % 9 && ci0 == 0 && wn == 0;
    float bsum[TM] = {};

    const int iters = (nkt + KS2 - 1) / KS2;
    if (iters > 0) stage(0, s_begin);
    if (iters > 1) stage(1, s_begin + KS2);
    for (int t = 0; t < iters; ++t) {
        // counted wait only when the newer stage in flight is a full one
        if (t + 1 < iters && s_begin + (t + 2) * KS2 <= s_end) vm_wait<2 * NP * KS2>();
        else vm_wait<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (t + 2 < iters) stage((t + 2) % NS, s_begin + (t + 2) * KS2);
#pragma unroll
        for (int u = 0; u < KS2; ++u) {
            if (s_begin + t * KS2 + u >= s_end) break;
            char* base = lds + ((t % NS) * KS2 + u) * SUB;
            bf16x8 af[TM][NP], bfr[TN][NP];
#pragma unroll
            for (int p = 0; p < NP; ++p) {
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const v4i16 lo =
                        __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(base + p * PI + aoffs[i][0]));
                    const v4i16 hi =
                        __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(base + p * PI + aoffs[i][1]));
                    const short8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    af[i][p] = __builtin_bit_cast(bf16x8, v);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const v4i16 lo =
                        __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(base + AB + p * PI + boffs[j][0]));
                    const v4i16 hi =
                        __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(base + AB + p * PI + boffs[j][1]));
                    const short8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    bfr[j][p] = __builtin_bit_cast(bf16x8, v);
                }
            }
            if (bias_wave) {
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int p = 0; p < NP; ++p)
#pragma unroll
                        for (int e = 0; e < 8; ++e) bsum[i] += piece_elem<NP>(af[i][p], e);
            }
            floatx16 tmp[TM][TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) tmp[i][j] = mfma_split0<NP>(af[i], bfr[j]);
            __builtin_amdgcn_sched_barrier(0);   // chains first, adds after (see conv_psa_kernel)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) drain(acc[i][j], tmp[i][j]);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    float* sl = slab + (int64_t)bz * Cout * Nt;
    const int li = lane & 31, h = lane >> 5;
    float inv = 1.f, binv = 1.f;
    if constexpr (NP == 2) {
        binv = 1.f / *dscale;
        inv = binv / ubpl::FP16_ACT_SCALE;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = tap * Cin + ci0 + wn + 32 * j + li;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                sl[(int64_t)m * Nt + n] = acc[i][j][r] * inv;
            }
    }
    if (bias_wave) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            // lane (r, h) summed channel wm + 32i + r over pixels 8h..8h+7 of each step
            const float v = bsum[i] + __shfl_xor(bsum[i], 32, 64);
            if (h == 0) sl[(int64_t)(m0 + wm + 32 * i + li) * Nt + Ntot] = v * binv;
        }
    }
}

// 64-channel 3x3 weight gradient (wgrad3_psa_kernel's operands and slab): an
// n-tile is one kernel ROW — the 3 taps (kh, 0..2) x 64 input channels — so a
// wave's tile is 32 output channels x 96 (3 taps x 32 channels): 18 MFMA
// chains per barrier instead of 6 with 64 x 64 one-tap tiles.  Stage image: A
// [piece][4 groups][16 px][32 B], then B per tap kw [piece][4 groups][16 px][32 B]
// (the three taps' shifted pixel windows DMA'd separately); wave 0 moves A,
// wave 1 + kw moves tap kw of B (6 DMA instructions each per stage).
template <int NP>
__global__ void __launch_bounds__(NT, 2) wgrad3_psa64_kernel(const uint16_t* __restrict__ dys, int64_t dplane,
                                                            const uint16_t* __restrict__ xs, int64_t xplane, int B,
                                                            int Cin, int Cout, int H, int W, int steps_per_split,
                                                            float* __restrict__ slab, const float* __restrict__ dscale) {
    // NP = 2: the scales of wgrad3_psa_kernel
    constexpr int TN = 3, NS = 3;
    constexpr int PI = 4 * 512;               // piece image: 4 groups x 16 px x 32 B
    constexpr int OB = NP * PI;               // one operand image (A, or one tap of B)
    constexpr int SB = 4 * OB;                // stage: A + 3 taps of B
    __shared__ __attribute__((aligned(16))) char lds[NS * SB];
    typedef short v4i16 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) v4i16* tr_ptr_t;

    const int Hp = H + 2, Wp = W + 2;
    const int Gci = Cin >> 4, Gco = Cout >> 4;
    const int Ntot = 9 * Cin, Nt = Ntot + 1;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // (wave-uniform: SGPR)
    const int wm = (wid >> 1) * 32, wn = (wid & 1) * 96;
    const int lam = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                              gridDim.x * gridDim.y * gridDim.z);
    const int bx = lam % gridDim.x, by = (lam / gridDim.x) % gridDim.y, bz = lam / (gridDim.x * gridDim.y);
    const int m0 = by * 64;
    const int nci = Cin / 64;
    const int kh = bx / nci, ci0 = (bx - kh * nci) * 64;
    const int wsteps = W >> 4;
    const int total_steps = B * H * wsteps;
    const int s_begin = bz * steps_per_split;
    const int s_end = min(total_steps, s_begin + steps_per_split);
    const int nkt = max(0, s_end - s_begin);

    // DMA: group pair gp (2 groups, one per half-wave), the swizzled pixel row
    const int64_t HWp = (int64_t)Hp * Wp;
    const int rphys = (lane & 31) >> 1;
    uint32_t lane_off[2];
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) {
        const int gl = 2 * gp + (lane >> 5);
        const int rlog = rphys ^ (4 * (gl & 1));
        lane_off[gp] = (uint32_t)(((gl * HWp + rlog) * 16 + 8 * (lane & 1)) * 2);
    }
    const char* dys_m = reinterpret_cast<const char*>(dys + (int64_t)(m0 >> 4) * HWp * 16);
    const char* xs_c = reinterpret_cast<const char*>(xs + (int64_t)(ci0 >> 4) * HWp * 16);
    const int kw_w = wid - 1;   // the B tap this wave moves (waves 1..3)
    auto stage = [&](int buf, int s) {
        const int b = s / (H * wsteps);
        const int rem = s - b * (H * wsteps);
        const int oh = rem / wsteps, ow0 = (rem - oh * wsteps) * 16;
        char* base = lds + buf * SB;
        const char* src;
        int64_t plane;
        if (wid == 0) {
            src = dys_m + 2 * ((int64_t)b * Gco * HWp * 16 + ((int64_t)(oh + 1) * Wp + ow0 + 1) * 16);
            plane = dplane;
        } else {
            src = xs_c + 2 * ((int64_t)b * Gci * HWp * 16 + ((int64_t)(oh + kh) * Wp + ow0 + kw_w) * 16);
            plane = xplane;
            base += OB * (1 + kw_w);
        }
#pragma unroll
        for (int p = 0; p < NP; ++p)
#pragma unroll
            for (int gp = 0; gp < 2; ++gp)
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src + 2 * p * plane + lane_off[gp]),
                                                 (lds_ptr_t)(base + p * PI + gp * 1024), 16, 0, 0);
    };

    // transposed-read geometry (as wgrad3_psa_kernel)
    const int g16 = lane >> 4, i16 = lane & 15;
    const int qrow = i16 >> 2, pcol = i16 & 3;
    auto tr_off = [&](int grp, int t) {
        const int row = (8 * (g16 >> 1) + 4 * t + qrow) ^ (4 * (grp & 1));
        return grp * 512 + row * 32 + 8 * pcol;
    };
    int aoffs[2], boffs[TN][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) aoffs[t] = tr_off(wm / 16 + (g16 & 1), t);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int nb = wn / 32 + j;   // 32-column block: tap nb/2, channels 32*(nb&1) ..
#pragma unroll
        for (int t = 0; t < 2; ++t) boffs[j][t] = OB * (1 + (nb >> 1)) + tr_off(2 * (nb & 1) + (g16 & 1), t);
    }

    floatx16 acc[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
    const bool bias_wave = kh == bz % 3 && ci0 == 0 && wn == 0;
    float bsum = 0.f;

    if (nkt > 0) stage(0, s_begin);
    if (nkt > 1) stage(1, s_begin + 1);
    for (int t = 0; t < nkt; ++t) {
        if (t + 1 < nkt) vm_wait<2 * NP>();
        else vm_wait<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (t + 2 < nkt) stage((t + 2) % NS, s_begin + t + 2);
        const char* base = lds + (t % NS) * SB;
        bf16x8 af[NP], bfr[TN][NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            {
                const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(base + p * PI + aoffs[0]));
                const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(base + p * PI + aoffs[1]));
                const short8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                af[p] = __builtin_bit_cast(bf16x8, v);
            }
#pragma unroll
            for (int j = 0; j < TN; ++j) {
                const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(base + p * PI + boffs[j][0]));
                const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(base + p * PI + boffs[j][1]));
                const short8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                bfr[j][p] = __builtin_bit_cast(bf16x8, v);
            }
        }
        if (bias_wave) {
#pragma unroll
            for (int p = 0; p < NP; ++p)
#pragma unroll
                for (int e = 0; e < 8; ++e) bsum += piece_elem<NP>(af[p], e);
        }
        floatx16 tmp[TN];
#pragma unroll
        for (int j = 0; j < TN; ++j) tmp[j] = mfma_split0<NP>(af, bfr[j]);
        __builtin_amdgcn_sched_barrier(0);   // chains first, adds after (see conv_psa_kernel)
#pragma unroll
        for (int j = 0; j < TN; ++j) drain(acc[j], tmp[j]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    float* sl = slab + (int64_t)bz * Cout * Nt;
    const int li = lane & 31, h = lane >> 5;
    float inv = 1.f, binv = 1.f;
    if constexpr (NP == 2) {
        binv = 1.f / *dscale;
        inv = binv / ubpl::FP16_ACT_SCALE;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int nb = wn / 32 + j;
        const int n = (kh * 3 + (nb >> 1)) * Cin + ci0 + 32 * (nb & 1) + li;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int m = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * h;
            sl[(int64_t)m * Nt + n] = acc[j][r] * inv;
        }
    }
    if (bias_wave) {
        const float v = bsum + __shfl_xor(bsum, 32, 64);
        if (h == 0) sl[(int64_t)(m0 + wm + li) * Nt + Ntot] = v * binv;
    }
}

// ------------------------------------------------------------------ the stem's weight gradient (space-to-depth)
// The 7x7 stride-2 stem's weight gradient as the weight gradient of its
// space-to-depth form (stem_s2d_split_kernel / stem_weight_s2d_split_kernel): a
// stride-1 4x4 conv of the 16-channel phase image, so
//   dW'[co][tap (a, b)][ci] = sum over (n, oh, ow) of dy[n, co, oh, ow] * x'[n, ci, oh + a - 2, ow + b - 2]
// on the split path, both operands PSA images: dys = split(dy) with a 1-pixel
// border (the BN backward emits it), xs = the forward's phase image with its
// 2-pixel border (kept for the backward).  GEMM: M = Cout (64-row blocks), N =
// 16 taps x 16 channels (all of it per workgroup), K = pixels, K step = 16
// consecutive pixels of one output row; split over workgroups into a slab
// [z][Cout][257] reduced by wgrad_reduce_kernel (T = 16, Cin = 16; last column:
// the bias gradient, from wave 0's A fragments).  Wave w takes kernel row a = w
// (4 taps x 16 channels = 64 columns) x the 64 rows: wave tile 64 x 64.
// Stage: A [piece][4 channel groups][16 px][32 B] (odd groups' pixel rows 0-3
// <-> 4-7 swapped, as wgrad3_psa_kernel), B the 4-row x 19-pixel halo of the
// step's receptive field [piece][4 rows][19 px][32 B] (a tap is a pixel offset);
// fragments by ds_read_b64_tr_b16.  3-stage ring.
template <int NP>
__global__ void __launch_bounds__(NT, 2) wgrad_stem_psa_kernel(const uint16_t* __restrict__ dys, int64_t dplane,
                                                              const uint16_t* __restrict__ xs, int64_t xplane,
                                                              int B, int Cout, int H, int W, int steps_per_split,
                                                              float* __restrict__ slab) {
    constexpr int NS = 3, HXP = 19, BROWS = 4 * HXP;       // halo: 4 rows x 19 pixels
    constexpr int API = 4 * 16 * 32;                       // A piece image: 4 groups x 16 px x 32 B
    constexpr int BPI = BROWS * 32;                        // B piece image
    constexpr int AB = NP * API, SUB = AB + NP * BPI;
    constexpr int AI = NP * 2, BI = NP * 3, NI = AI + BI;  // DMA instructions per stage (1 KB each)
    constexpr int NPW = (NI + 3) / 4;                      // per wave
    __shared__ __attribute__((aligned(16))) char lds[NS * SUB];
    typedef short v4i16 __attribute__((ext_vector_type(4)));
    typedef __attribute__((address_space(3))) v4i16* tr_ptr_t;

    const int Hp = H + 2, Wp = W + 2, Hx = H + 4, Wx = W + 4;
    const int Go = Cout >> 4;
    constexpr int Ntot = 256, Nt = Ntot + 1;
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    // grid (Cout / 64, splits): the row blocks of one split side by side (same L2)
    const int lam = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
    const int by = lam % gridDim.x, bz = lam / gridDim.x;
    const int m0 = by * 64;
    const int wsteps = W >> 4;
    const int total_steps = B * H * wsteps;
    const int s_begin = bz * steps_per_split;
    const int s_end = min(total_steps, s_begin + steps_per_split);
    const int nkt = max(0, s_end - s_begin);

    // per-instruction lane offsets (bytes, relative to the step's base): instruction i
    // of a stage, i = u * 4 + wid: A piece i / 2 (groups 2 (i % 2), +1), B piece
    // (i - AI) / 3, 32-pixel chunk (i - AI) % 3 (the last one overlapping: starts at 76 - 32)
    uint32_t loff[NPW];
    int lpiece[NPW];
    bool lisa[NPW], lon[NPW];
    const int lrow = lane >> 1, lhalf = lane & 1;
#pragma unroll
    for (int u = 0; u < NPW; ++u) {
        const int i = u * 4 + wid;
        lon[u] = i < NI;
        lisa[u] = i < AI;
        if (i < AI) {
            const int gl = 2 * (i % 2) + (lrow >> 4);
            const int rphys = lrow & 15, rlog = rphys ^ (4 * (gl & 1));
            lpiece[u] = i / 2;
            loff[u] = (uint32_t)((((int64_t)gl * Hp * Wp) + rlog) * 16 + 8 * lhalf) * 2;
        } else {
            const int j = i - AI, c = j % 3;
            const int q = min(c * 32, BROWS - 32) + lrow;
            const int a = q / HXP, px = q - a * HXP;
            lpiece[u] = j / 3;
            loff[u] = (uint32_t)(((int64_t)a * Wx + px) * 16 + 8 * lhalf) * 2;
        }
    }
    const char* dys_m = reinterpret_cast<const char*>(dys + (int64_t)(m0 >> 4) * Hp * Wp * 16);
    auto stage = [&](int buf, int s) {
        if (s >= s_end) return;
        const int b = s / (H * wsteps);
        const int rem = s - b * (H * wsteps);
        const int oh = rem / wsteps, ow0 = (rem - oh * wsteps) * 16;
        const int64_t aoff = ((int64_t)b * Go * Hp * Wp + (int64_t)(oh + 1) * Wp + ow0 + 1) * 16;
        const int64_t boff = (((int64_t)b * Hx + oh) * Wx + ow0) * 16;
        char* base = lds + buf * SUB;
#pragma unroll
        for (int u = 0; u < NPW; ++u) {
            if (!lon[u]) continue;
            const int i = u * 4 + wid;
            if (lisa[u]) {
                const char* src = dys_m + 2 * (lpiece[u] * dplane + aoff);
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src + loff[u]),
                                                 (lds_ptr_t)(base + lpiece[u] * API + (i % 2) * 1024), 16, 0, 0);
            } else {
                const int j = i - AI, c = j % 3;
                const char* src = reinterpret_cast<const char*>(xs) + 2 * (lpiece[u] * xplane + boff);
                __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src + loff[u]),
                                                 (lds_ptr_t)(base + AB + lpiece[u] * BPI + min(c * 32, BROWS - 32) * 32),
                                                 16, 0, 0);
            }
        }
    };
    // this wave's DMA instructions per stage (the counted waits below)
    const int mine = (NI - wid + 3) / 4;

    // transposed reads: 16-lane group g16 = lane >> 4; lane i16 = (qrow, pcol)
    const int g16 = lane >> 4, i16 = lane & 15;
    const int qrow = i16 >> 2, pcol = i16 & 3;
    int aoffs[2][2], boffs[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int grp = 2 * i + (g16 & 1);
            const int row = (8 * (g16 >> 1) + 4 * t + qrow) ^ (4 * (grp & 1));
            aoffs[i][t] = grp * 512 + row * 32 + 8 * pcol;
        }
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int px = 8 * (g16 >> 1) + 4 * t + qrow + 2 * j + (g16 & 1);   // tap b = 2j + (g16 & 1)
            boffs[j][t] = (wid * HXP + px) * 32 + 8 * pcol;
        }

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
    const bool bias_wave = wid == 0;
    float bsum[2] = {0.f, 0.f};

    stage(0, s_begin);
    stage(1, s_begin + 1);
    for (int t = 0; t < nkt; ++t) {
        // stage t landed (this wave's stage t+1 DMA may stay in flight)
        if (t + 1 < nkt) {
            // NP = 3: 15 instructions per stage (4 / 4 / 4 / 3 per wave); NP = 1: 5 (2 / 1 / 1 / 1)
            if (mine == 4) vm_wait<4>();
            else if (mine == 3) vm_wait<3>();
            else if (mine == 2) vm_wait<2>();
            else vm_wait<1>();
        } else {
            vm_wait<0>();
        }
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (t + 2 < nkt) stage((t + 2) % NS, s_begin + t + 2);
        char* base = lds + (t % NS) * SUB;
        bf16x8 af[2][NP], bfr[2][NP];
#pragma unroll
        for (int p = 0; p < NP; ++p) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(base + p * API + aoffs[i][0]));
                const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(base + p * API + aoffs[i][1]));
                const short8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                af[i][p] = __builtin_bit_cast(bf16x8, v);
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(base + AB + p * BPI + boffs[j][0]));
                const v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tr_ptr_t)(base + AB + p * BPI + boffs[j][1]));
                const short8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                bfr[j][p] = __builtin_bit_cast(bf16x8, v);
            }
        }
        if (bias_wave) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int p = 0; p < NP; ++p)
#pragma unroll
                    for (int e = 0; e < 8; ++e) bsum[i] += (float)af[i][p][e];
        }
        floatx16 tmp[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) tmp[i][j] = mfma_split0<NP>(af[i], bfr[j]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) drain(acc[i][j], tmp[i][j]);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }

    float* sl = slab + (int64_t)bz * Cout * Nt;
    const int li = lane & 31, h = lane >> 5;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = 64 * wid + 32 * j + li;                   // tap 4 wid + 2 j + li / 16, channel li % 16
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = m0 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
                sl[(int64_t)m * Nt + n] = acc[i][j][r];
            }
    }
    if (bias_wave) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            // lane (r, h) summed channel 32i + r over pixels 8h..8h+7 of each step
            const float v = bsum[i] + __shfl_xor(bsum[i], 32, 64);
            if (h == 0) sl[(int64_t)(m0 + 32 * i + li) * Nt + Ntot] = v;
        }
    }
}

// the space-to-depth weight gradient dws [Cout][16 ci][16 taps] + its bias column dbs
// [Cout] (wgrad_reduce_kernel's layout for Cin = 16, T = 16) -> the 7x7 gradient dw
// [Cout][C][7][7] (+)= and db (+)=: tap (a, b), channel c*4 + 2 ph + pw of the phase
// image holds w[.][c][2 (a - 2) + ph + 3][2 (b - 2) + pw + 3], i.e. kh -> (ph, a) =
// ((kh + 1) & 1, (kh + 1 - ph) / 2)
__global__ void __launch_bounds__(256) stem_wgrad_map_kernel(const float* __restrict__ dws,
                                                             const float* __restrict__ dbs, int Cout, int C,
                                                             float* __restrict__ dw, float* __restrict__ db,
                                                             int accumulate) {
    constexpr int KS = 7;
    const int64_t total = (int64_t)Cout * C * KS * KS;
    const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (db != nullptr && idx < Cout) db[idx] = accumulate ? db[idx] + dbs[idx] : dbs[idx];
    if (idx >= total) return;
    const int kw = (int)(idx % KS), kh = (int)((idx / KS) % KS);
    const int c = (int)((idx / (KS * KS)) % C), o = (int)(idx / (KS * KS * C));
    const int ph = (kh + 1) & 1, a = (kh + 1 - ph) / 2;
    const int pw = (kw + 1) & 1, bb = (kw + 1 - pw) / 2;
    const float v = dws[(int64_t)o * 256 + (c * 4 + 2 * ph + pw) * 16 + a * 4 + bb];
    dw[idx] = accumulate ? dw[idx] + v : v;
}

// ------------------------------------------------------------------ 1x1 weight gradient, split on load
// dW[m][k] = sum over pixels n of dy[m][n] * v[k][n], v = relu(x*pscale + pshift)
// (PRO) or x; db[m] = sum dy[m][n].  GEMM: M = Cout, N = Cin, K = pixels, both
// operands pixel-contiguous in NCHW (no transposes).  K step = 16 pixels of one
// image (P % 16 == 0), split over workgroups into a slab [z][Cout][Cin + 1] (last
// column: the bias gradient, from the Cin-tile-0 workgroups) reduced by
// conv.hip's wgrad_reduce_kernel.  The f32 operands come global -> registers
// (two steps ahead), each element is split ONCE per workgroup by the thread
// that loaded it (thread t: row t/2 of both operands, pixels 8(t&1)..+7), and
// the pieces go to a double-buffered LDS image [operand][piece][128 rows][32 B]
// (chunk swizzle c ^ ((row >> 3) & 1), conflict-free ds_read_b128 fragments,
// conv_psa_kernel's layout).  Tile CM x CN (128 or 64 channels of dy / of x:
// the 64-channel convs of the first residual at 128x128), wave tile CM/2 x CN/2.
// With 64 rows an operand row is loaded by 4 threads (4 pixels each).
template <bool PRO, int NP = 3, int CM = 128, int CN = 128>
__global__ void __launch_bounds__(NT, 2) wgrad1_sol_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                          const float* __restrict__ pscale,
                                                          const float* __restrict__ pshift, int B, int Cin, int Cout,
                                                          int P, int steps_per_split, float* __restrict__ slab) {
    // NP = 3: 6xbf16; NP = 1: bf16 operands, f32 accumulation (the "bf16" precision)
    constexpr int TM = CM / 64, TN = CN / 64;
    constexpr int PIA = CM * 32, PIB = CN * 32;   // one piece image: rows x 16 pixels x 2 B
    constexpr int OA = NP * PIA;                  // dy pieces, then x pieces
    constexpr int SB = OA + NP * PIB;             // one stage
    constexpr int TPA = NT / CM, TPB = NT / CN;   // loader threads per row
    constexpr int PPA = 16 / TPA, PPB = 16 / TPB; // pixels per loader thread (8 or 4)
    constexpr int FA = PPA / 4, FB = PPB / 4;     // float4s per loader thread
    __shared__ __attribute__((aligned(16))) char lds[2 * SB];

    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // (wave-uniform: SGPR)
    const int wm = (wid >> 1) * (CM / 2), wn = (wid & 1) * (CN / 2);
    const int lam = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                              gridDim.x * gridDim.y * gridDim.z);
    const int bx = lam % gridDim.x, by = (lam / gridDim.x) % gridDim.y, bz = lam / (gridDim.x * gridDim.y);
    const int m0 = by * CM, c0 = bx * CN;
    const int psteps = P >> 4;
    const int total = B * psteps;
    const int s_begin = bz * steps_per_split;
    const int s_end = min(total, s_begin + steps_per_split);
    const int nkt = max(0, s_end - s_begin);

    // loader / splitter: dy row ra, pixels PPA*qa .. +PPA-1 of the step; x row rb likewise
    const int ra = tid / TPA, qa = tid % TPA, rb = tid / TPB, qb = tid % TPB;
    const float* arow = dy + (int64_t)(m0 + ra) * P + PPA * qa;
    const float* brow = x + (int64_t)(c0 + rb) * P + PPB * qb;
    float sc = 1.f, sh = 0.f;
    if (PRO) {
        sc = pscale[c0 + rb];
        sh = pshift[c0 + rb];
    }
    // 16-B chunk (pixels 8c .. 8c+7) swizzled by row, then the 8-B half for 4-pixel loaders
    const int wofa = ra * 32 + 16 * (((PPA * qa) >> 3) ^ ((ra >> 3) & 1)) + 2 * ((PPA * qa) & 7);
    const int wofb = rb * 32 + 16 * (((PPB * qb) >> 3) ^ ((rb >> 3) & 1)) + 2 * ((PPB * qb) & 7);
    auto gload = [&](float4 (&a)[FA], float4 (&b)[FB], int s) {
        const int bb = s / psteps;
        const int p0 = (s - bb * psteps) * 16;
        const float4* a4 = reinterpret_cast<const float4*>(arow + (int64_t)bb * Cout * P + p0);
        const float4* b4 = reinterpret_cast<const float4*>(brow + (int64_t)bb * Cin * P + p0);
#pragma unroll
        for (int f = 0; f < FA; ++f) a[f] = a4[f];
#pragma unroll
        for (int f = 0; f < FB; ++f) b[f] = b4[f];
    };
    float bsum = 0.f;
    auto split_store = [&](int buf, const float4 (&a)[FA], const float4 (&b)[FB]) {
        float va[PPA], vb[PPB];
#pragma unroll
        for (int f = 0; f < FA; ++f) {
            va[4 * f] = a[f].x, va[4 * f + 1] = a[f].y, va[4 * f + 2] = a[f].z, va[4 * f + 3] = a[f].w;
        }
#pragma unroll
        for (int f = 0; f < FB; ++f) {
            vb[4 * f] = b[f].x, vb[4 * f + 1] = b[f].y, vb[4 * f + 2] = b[f].z, vb[4 * f + 3] = b[f].w;
        }
        if constexpr (PPA == 8)
            bsum += ((va[0] + va[1]) + (va[2] + va[3])) + ((va[4] + va[5]) + (va[6] + va[7]));
        else
            bsum += (va[0] + va[1]) + (va[2] + va[3]);
        if (PRO) {
#pragma unroll
            for (int e = 0; e < PPB; ++e) vb[e] = fmaxf(fmaf(vb[e], sc, sh), 0.f);
        }
        uint32_t pa[NP][PPA / 2], pb[NP][PPB / 2];
#pragma unroll
        for (int e = 0; e < PPA / 2; ++e) {
            uint32_t o[NP];
            split2<NP>(va[2 * e], va[2 * e + 1], o);
#pragma unroll
            for (int p = 0; p < NP; ++p) pa[p][e] = o[p];
        }
#pragma unroll
        for (int e = 0; e < PPB / 2; ++e) {
            uint32_t o[NP];
            split2<NP>(vb[2 * e], vb[2 * e + 1], o);
#pragma unroll
            for (int p = 0; p < NP; ++p) pb[p][e] = o[p];
        }
        char* base = lds + buf * SB;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
            if constexpr (PPA == 8)
                *reinterpret_cast<uint4*>(base + p * PIA + wofa) = make_uint4(pa[p][0], pa[p][1], pa[p][2], pa[p][3]);
            else
                *reinterpret_cast<uint2*>(base + p * PIA + wofa) = make_uint2(pa[p][0], pa[p][1]);
            if constexpr (PPB == 8)
                *reinterpret_cast<uint4*>(base + OA + p * PIB + wofb) =
                    make_uint4(pb[p][0], pb[p][1], pb[p][2], pb[p][3]);
            else
                *reinterpret_cast<uint2*>(base + OA + p * PIB + wofb) = make_uint2(pb[p][0], pb[p][1]);
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;
    const int li = lane & 31, h = lane >> 5;

    float4 cA[FA], cB[FB], nA[FA], nB[FB];
    if (nkt > 0) gload(cA, cB, s_begin);
    if (nkt > 1) gload(nA, nB, s_begin + 1);
    for (int t = 0; t < nkt; ++t) {
        // buffer t&1 was last read in step t-2, before every wave's step t-1 barrier
        split_store(t & 1, cA, cB);
#pragma unroll
        for (int f = 0; f < FA; ++f) cA[f] = nA[f];
#pragma unroll
        for (int f = 0; f < FB; ++f) cB[f] = nB[f];
        if (t + 2 < nkt) gload(nA, nB, s_begin + t + 2);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        const char* base = lds + (t & 1) * SB;
        bf16x8 af[TM][NP], bfr[TN][NP];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
            const int row = wm + 32 * i + li;
#pragma unroll
            for (int p = 0; p < NP; ++p)
                af[i][p] = *reinterpret_cast<const bf16x8*>(base + p * PIA + row * 32 + 16 * (h ^ ((row >> 3) & 1)));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int row = wn + 32 * j + li;
#pragma unroll
            for (int p = 0; p < NP; ++p)
                bfr[j][p] =
                    *reinterpret_cast<const bf16x8*>(base + OA + p * PIB + row * 32 + 16 * (h ^ ((row >> 3) & 1)));
        }
        if constexpr (NP == 1) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) mfma_split<NP>(acc[i][j], af[i], bfr[j]);
        } else {
            floatx16 tmp[TM][TN];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    tmp[i][j] = mfma_split0<NP>(af[i], bfr[j]);
                }
            __builtin_amdgcn_sched_barrier(0);   // chains first, adds after (see conv_psa_kernel)
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j) drain(acc[i][j], tmp[i][j]);
        }
    }

    const int Nt = Cin + 1;
    float* sl = slab + (int64_t)bz * Cout * Nt;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
        const int n = c0 + wn + 32 * j + li;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int m = m0 + wm + 32 * i + (q & 3) + 8 * (q >> 2) + 4 * h;
                sl[(int64_t)m * Nt + n] = acc[i][j][q];
            }
    }
    // bias gradient: the TPA threads of a row (adjacent lanes) hold its pixel chunks
    float bt = bsum + __shfl_xor(bsum, 1, 64);
    if constexpr (TPA == 4) bt += __shfl_xor(bt, 2, 64);
    if (bx == 0 && qa == 0) sl[(int64_t)(m0 + ra) * Nt + Cin] = bt;
}

// y[b,m,p] = sum_z slab[z][m][b*P+p] + bias[m] (+ res)
__global__ void __launch_bounds__(256) split_reduce_kernel(const float* __restrict__ slab, int splits, int Cout, int P,
                                                          int64_t N, const float* __restrict__ bias, const float* res,
                                                          float* y) {
    const int64_t total = (int64_t)Cout * N;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
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

// ------------------------------------------------------------------ weights
// Batched split re-layout over a segment table (int64 [nseg][5]: src_off,
// dst_off, Cout, Cin, T), one segment per blockIdx.y; NP bf16 planes of
// `plane` elements.  mode 0: forward layout wt[co][ci/G][tap][ci%G] =
// w[co][ci][tap]; mode 1: data-gradient layout wd[ci][co/G][tap][co%G] =
// w[co][ci][T-1-tap] (G = 16 when it divides the contraction channels).
__global__ void __launch_bounds__(256) split_relayout_kernel(const float* __restrict__ src,
                                                            uint16_t* __restrict__ dst, int64_t plane,
                                                            const int64_t* __restrict__ table, int mode, int np) {
    const int64_t* e = table + (int64_t)blockIdx.y * 5;
    const int64_t so = e[0], dof = e[1];
    const int Cout = (int)e[2], Cin = (int)e[3], T = (int)e[4];
    const int64_t total = (int64_t)Cout * Cin * T;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        int64_t s;
        if (mode == 0) {
            const int G = ubpl::conv_kgroup(Cin);
            const int gi = (int)(i % G);
            const int64_t t1 = i / G;
            const int tap = (int)(t1 % T);
            const int64_t t2 = t1 / T;
            const int cbk = (int)(t2 % (Cin / G));
            const int co = (int)(t2 / (Cin / G));
            s = ((int64_t)co * Cin + cbk * G + gi) * T + tap;
        } else {
            const int G = ubpl::conv_kgroup(Cout);
            const int gi = (int)(i % G);
            const int64_t t1 = i / G;
            const int tap = (int)(t1 % T);
            const int64_t t2 = t1 / T;
            const int cbk = (int)(t2 % (Cout / G));
            const int ci = (int)(t2 / (Cout / G));
            s = ((int64_t)(cbk * G + gi) * Cin + ci) * T + (T - 1 - tap);
        }
        float v = src[so + s];
        if (np == 2) {
            // 2xfp16: the fp16 pieces of w * fp16_wscale(contraction length) (common.h split2)
            v *= ubpl::fp16_wscale((mode == 0 ? Cin : Cout) * T);
            const _Float16 hv = (_Float16)v;
            dst[dof + i] = __builtin_bit_cast(uint16_t, hv);
            dst[plane + dof + i] = __builtin_bit_cast(uint16_t, (_Float16)(v - (float)hv));
            continue;
        }
        for (int p = 0; p < np; ++p) {
            const __bf16 hv = (__bf16)v;
            dst[(int64_t)p * plane + dof + i] = __builtin_bit_cast(uint16_t, hv);
            v -= (float)hv;
        }
    }
}

// ------------------------------------------------------------------ planning
struct Plan {
    int bm, splits, kchunk;
};

struct Occ {
    int ncu = 256;
    int f128[2] = {2, 1}, f64[2] = {3, 2};   // register-staged kernel [NP == 3]
    int p128[2] = {2, 2}, p64[2] = {3, 2};   // conv_psa_kernel [NP == 3]
};

const Occ& occ_info();

// Blocks spread evenly over the CUs; a CU with c blocks (r = min(c, occ)
// resident) runs them in c * (steps + 2) K steps at a rate that needs ~2
// resident blocks to hide latency.  Split-K adds the slab round trip + a launch.
double plan_cost(int64_t tiles, int s, int64_t nsteps, int occ, int ncu, double step_flops, double slab_bytes) {
    const int64_t blocks = tiles * s;
    const int64_t per_cu = (blocks + ncu - 1) / ncu;
    const int64_t r = per_cu < occ ? per_cu : occ;
    const double eff = r >= 2 ? 1.0 : 0.6;
    const int64_t steps = (nsteps + s - 1) / s;
    const double rate = 2.0e12;   // split-bf16 flop/s per CU, sustained (model only)
    double t = (double)((per_cu + r - 1) / r) * r * (double)(steps + 2) * step_flops / (rate * eff);
    if (s > 1) t += 2.0 * s * slab_bytes / 5e12 + 4e-6;
    return t;
}

Plan fwd_plan(int Cout, int64_t N, int Ktot, int np, bool psa = false) {
    const Occ& d = occ_info();
    const int bk = psa ? 16 : BK;
    const int nkt = (Ktot + bk - 1) / bk;
    // UBPL_NO_SPLITK=1 (diagnostic): never split K (no slab, no reduce launch)
    static const bool no_splitk = [] {
        const char* e = std::getenv("UBPL_NO_SPLITK");
        return e != nullptr && e[0] == '1';
    }();
    const int maxs = no_splitk ? 1 : (nkt / 2 > 0 ? nkt / 2 : 1);
    Plan best{64, 1, 0};
    double bc = 1e30;
    for (int bm : {128, 64}) {
        if (bm == 128 && Cout <= 64) continue;
        const int64_t tiles = ((Cout + bm - 1) / bm) * ((N + BN - 1) / BN);
        const int occ = psa ? (bm == 128 ? d.p128[np == 3] : d.p64[np == 3])
                            : (bm == 128 ? d.f128[np == 3] : d.f64[np == 3]);
        const double sf = 2.0 * bm * BN * bk;
        int s_best = 1;
        double c_best = plan_cost(tiles, 1, nkt, occ, d.ncu, sf, 4.0 * Cout * N);
        for (int s = 2; s <= maxs; ++s) {
            const double c = plan_cost(tiles, s, nkt, occ, d.ncu, sf, 4.0 * Cout * N);
            if (c < c_best * 0.97) {
                c_best = c;
                s_best = s;
            }
        }
        const double c = c_best / (bm == 128 ? 1.0 : 0.85);
        if (c < bc) {
            bc = c;
            best.bm = bm;
            best.splits = s_best;
        }
    }
    const int steps = (nkt + best.splits - 1) / best.splits;
    best.kchunk = steps * bk;
    best.splits = (nkt + steps - 1) / steps;
    return best;
}

void launch_split_reduce(const float* slab, int splits, int Cout, int P, int64_t N, const float* bias,
                         const float* res, float* y, hipStream_t st);

// the accumulators' scale of a split conv: 2xfp16 (NP = 2) the weight scale of its contraction
// length x the activation scale (common.h split2), else 1
// (dev_act: the activation scale is read on the device, *ascp; the host part is the weight scale)
inline float psa_osc(int np, int ktot, bool dev_act = false) {
    return np == 2 ? ubpl::fp16_wscale(ktot) * (dev_act ? 1.f : ubpl::FP16_ACT_SCALE) : 1.f;
}

template <int BM, int KS, int NP, int BNT, int WGM = 2, int KSUB = 1>
int launch_psa(const uint16_t* xs, int64_t xplane, const uint16_t* wp, int64_t wplane, const float* bias,
               const float* res, float* y, int B, int Cin, int H, int W, int pad, int Cout, const Plan& pl,
               float* slab, float* stat_part, const ubpl::BnBwdEpi& bwd, hipStream_t st,
               const float* ascp = nullptr) {
    const int64_t N = (int64_t)B * H * W;
    dim3 grid((unsigned)((N + BNT - 1) / BNT), (unsigned)((Cout + BM - 1) / BM), (unsigned)pl.splits);
    const bool split = pl.splits > 1;
    const ubpl::BnBwdEpi off{nullptr, nullptr, 0, nullptr};
    const float osc = psa_osc(NP, Cin * KS * KS, ascp != nullptr);
    if constexpr (NP != 2) {   // (epilogue partials: not on the scaled 2xfp16 accumulators)
        if (!split && (stat_part || bwd.part)) {
            hipLaunchKernelGGL((conv_psa_kernel<BM, KS, NP, BNT, WGM, true, KSUB>), grid, dim3(NT), 0, st, xs, xplane,
                               wp, wplane, bias, res, y, B, Cin, H, W, pad, Cout, pl.kchunk, nullptr, stat_part, bwd,
                               osc, ascp);
            UBPL_LAUNCH_CHECK();
            return 0;
        }
    }
    hipLaunchKernelGGL((conv_psa_kernel<BM, KS, NP, BNT, WGM, false, KSUB>), grid,
                       dim3(NT), 0, st, xs, xplane, wp, wplane,
                       bias, split ? nullptr : res, y, B, Cin, H, W, pad, Cout, pl.kchunk, split ? slab : nullptr,
                       nullptr, off, osc, ascp);
    UBPL_LAUNCH_CHECK();
    if (split) {
        launch_split_reduce(slab, pl.splits, Cout, H * W, N, bias, res, y, st);
        UBPL_LAUNCH_CHECK();
        if (stat_part) {
            const int e = ubpl_bn_partials(y, B, Cout, H * W, stat_part, st);
            if (e) return e;
        }
        if (bwd.part)
            return ubpl_bn_backward_partials(y, bwd.x, B, Cout, H * W, bwd.coef, bwd.coef + Cout,
                                             bwd.coef + 2 * Cout, bwd.relu, bwd.part, st);
    }
    return 0;
}

template <int BM, int KS, int ST, bool PRO, int NP>
int launch_fwd(const float* x, const uint16_t* wp, int64_t plane, const float* bias, const float* ps, const float* sh,
               const float* res, float* y, int B, int Cin, int H, int W, int Cout, int Ho, int Wo, const Plan& pl,
               float* slab, hipStream_t st) {
    const int64_t N = (int64_t)B * Ho * Wo;
    dim3 grid((unsigned)((N + BN - 1) / BN), (unsigned)((Cout + BM - 1) / BM), (unsigned)pl.splits);
    const bool split = pl.splits > 1;
    hipLaunchKernelGGL((conv_fwd_split_kernel<BM, KS, ST, PRO, NP>), grid, dim3(NT), 0, st, x, wp, plane, bias, ps, sh,
                       split ? nullptr : res, y, B, Cin, H, W, Cout, Ho, Wo, pl.kchunk, split ? slab : nullptr);
    UBPL_LAUNCH_CHECK();
    if (split) {
        launch_split_reduce(slab, pl.splits, Cout, Ho * Wo, N, bias, res, y, st);
        UBPL_LAUNCH_CHECK();
    }
    return 0;
}

void launch_split_reduce(const float* slab, int splits, int Cout, int P, int64_t N, const float* bias,
                         const float* res, float* y, hipStream_t st) {
    const int64_t total = (int64_t)Cout * N;
    int gsz = (int)((total + 255) / 256);
    if (gsz > 8192) gsz = 8192;
    hipLaunchKernelGGL(split_reduce_kernel, dim3(gsz), dim3(256), 0, st, slab, splits, Cout, P, N, bias, res, y);
}

template <int KS, int ST, int NP>
int fwd_dispatch(const Plan& pl, bool pro, const float* x, const uint16_t* wp, int64_t plane, const float* bias,
                 const float* ps, const float* sh, const float* res, float* y, int B, int Cin, int H, int W, int Cout,
                 int Ho, int Wo, float* slab, hipStream_t st) {
#define UBPL_FS(BM_, PRO_)                                                                                        \
    return launch_fwd<BM_, KS, ST, PRO_, NP>(x, wp, plane, bias, ps, sh, res, y, B, Cin, H, W, Cout, Ho, Wo, pl, \
                                             slab, st)
    if (pl.bm == 128) {
        if (pro) UBPL_FS(128, true);
        UBPL_FS(128, false);
    }
    if (pro) UBPL_FS(64, true);
    UBPL_FS(64, false);
#undef UBPL_FS
}

const Occ& occ_info() {
    static Occ d = [] {
        Occ r;
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
            r.ncu = v;
        auto q = [&](const void* f, int& dst) {
            int o = 0;
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, f, NT, 0) == hipSuccess && o > 0) dst = o;
        };
        q((const void*)conv_fwd_split_kernel<128, 3, 1, true, 2>, r.f128[0]);
        q((const void*)conv_fwd_split_kernel<128, 3, 1, true, 3>, r.f128[1]);
        q((const void*)conv_fwd_split_kernel<64, 3, 1, true, 2>, r.f64[0]);
        q((const void*)conv_fwd_split_kernel<64, 3, 1, true, 3>, r.f64[1]);
        q((const void*)conv_psa_kernel<128, 3, 2>, r.p128[0]);
        q((const void*)conv_psa_kernel<128, 3, 3>, r.p128[1]);
        q((const void*)conv_psa_kernel<64, 3, 2>, r.p64[0]);
        q((const void*)conv_psa_kernel<64, 3, 3>, r.p64[1]);
        (void)hipGetLastError();
        return r;
    }();
    return d;
}

}  // namespace

// Floats of split-K workspace ubpl_conv2d_forward_split needs; 0 = none.
UBPL_API int64_t ubpl_conv2d_forward_split_workspace(int B, int Cin, int Cout, int KS, int Ho, int Wo, int npieces) {
    const int64_t N = (int64_t)B * Ho * Wo;
    const Plan pl = fwd_plan(Cout, N, Cin * KS * KS, npieces);
    return pl.splits > 1 ? (int64_t)pl.splits * Cout * N : 0;
}

// y = conv(relu(x*pscale + pshift) or x, w, pad (KS-1)/2) + bias (+ res) on the
// split-bf16 MFMA path.  wsplit: npieces (2 or 3) bf16 planes, `plane`
// elements apart, of the weights in ubpl_conv_weights_split's layout.
// (KS, stride) in {(1,1), (3,1)}; Cin % 16 == 0; res may alias y.
UBPL_API int ubpl_conv2d_forward_split(const float* x, int B, int Cin, int H, int W, const uint16_t* wsplit,
                                       int64_t plane, const float* bias, int Cout, int KS, int stride,
                                       const float* pscale, const float* pshift, const float* res, float* y, int Ho,
                                       int Wo, float* slab, int npieces, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (Cin % 16 != 0 || stride != 1 || npieces != 3) return (int)hipErrorInvalidValue;
    if ((((uintptr_t)wsplit) & 15) != 0 || (plane % 8) != 0) return (int)hipErrorInvalidValue;
    const bool pro = pscale != nullptr;
    const int64_t N = (int64_t)B * Ho * Wo;
    const Plan pl = fwd_plan(Cout, N, Cin * KS * KS, npieces);
    if (pl.splits > 1 && slab == nullptr) return (int)hipErrorInvalidValue;
#define UBPL_FD(KS_, NP_)                                                                                     \
    return fwd_dispatch<KS_, 1, NP_>(pl, pro, x, wsplit, plane, bias, pscale, pshift, res, y, B, Cin, H, W, \
                                     Cout, Ho, Wo, slab, st)
    if (KS == 1) UBPL_FD(1, 3);
    if (KS == 3) UBPL_FD(3, 3);
#undef UBPL_FD
    return (int)hipErrorInvalidValue;
}

// Split re-layout of many convs in one launch (table as ubpl_conv_weights_relayout;
// dst_off multiples of 8).  dst: npieces planes of `plane` bf16 elements.
UBPL_API int ubpl_conv_weights_split(const float* src, uint16_t* dst, int64_t plane, const int64_t* table, int nseg,
                                     int mode, int npieces, void* stream) {
    if (nseg <= 0) return 0;
    if (npieces < 1 || npieces > 3) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(split_relayout_kernel, dim3(64, nseg), dim3(256), 0, (hipStream_t)stream, src, dst, plane,
                       table, mode, npieces);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// Pre-split activations (PSA layout, see split_act_kernel): dst = npieces bf16
// planes `plane` elements apart of [B][C/16][H+2pad][W+2pad][16];
// v = relu(x*pscale + pshift) when pscale != nullptr, else x.  C % 16 == 0.
UBPL_API int ubpl_split_activation(const float* x, int B, int C, int H, int W, const float* pscale,
                                   const float* pshift, int pad, int npieces, uint16_t* dst, int64_t plane,
                                   uint16_t* dst3, int64_t plane3, void* stream) {
    if (C % 16 != 0 || npieces < 1 || npieces > 3 || pad < 0 || (plane % 8) != 0) return (int)hipErrorInvalidValue;
    if (dst3 != nullptr && (npieces != 2 || (plane3 % 8) != 0)) return (int)hipErrorInvalidValue;
    const int Hp = H + 2 * pad, Wp = W + 2 * pad;
    dim3 grid((unsigned)((Hp * Wp + 255) / 256), (unsigned)(C / 16), (unsigned)B);
    hipStream_t st = (hipStream_t)stream;
    const bool pro = pscale != nullptr;
#define UBPL_SA(NP_, PRO_, ...)                                                                                \
    hipLaunchKernelGGL((split_act_kernel<NP_, PRO_, ##__VA_ARGS__>), grid, dim3(256), 0, st, x, C, H, W, pscale,  \
                       pshift, pad, dst, plane, ubpl::FP16_ACT_SCALE, dst3, plane3)
    if (npieces == 1) {   // the "bf16" precision: one piece = bf16(v)
        if (pro) UBPL_SA(1, true);
        else UBPL_SA(1, false);
    } else if (npieces == 2 && dst3 != nullptr) {   // 2xfp16 (scaled) + the 6xbf16 image
        if (pro) UBPL_SA(2, true, true);
        else UBPL_SA(2, false, true);
    } else if (npieces == 2) {
        if (pro) UBPL_SA(2, true);
        else UBPL_SA(2, false);
    } else {
        if (pro) UBPL_SA(3, true);
        else UBPL_SA(3, false);
    }
#undef UBPL_SA
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int64_t ubpl_conv2d_forward_psa_workspace(int B, int Cin, int Cout, int KS, int H, int W, int npieces) {
    const int64_t N = (int64_t)B * H * W;
    const Plan pl = fwd_plan(Cout, N, Cin * KS * KS, npieces, true);
    return pl.splits > 1 ? (int64_t)pl.splits * Cout * N : 0;
}

// y = conv(xs, w, stride 1, pad (KS-1)/2) + bias (+ res) with xs in the PSA
// layout (border pad >= (KS-1)/2) and w from ubpl_conv_weights_split (same
// npieces).  KS in {1, 3}; Cin % 16 == 0; res may alias y.
namespace {
// dispatch knobs of the 3x3 halo kernel: from the environment once (UBPL_PSA_HALO = 0 / 1,
// UBPL_PSA_TEAMS = 1 / 2; diagnostics), overridden by ubpl_set_psa_dispatch (tests)
struct PsaDispatch {
    int halo, teams;
};
std::atomic<int> g_psa_halo{-2}, g_psa_teams{-2};
PsaDispatch psa_dispatch() {
    if (g_psa_halo.load(std::memory_order_relaxed) == -2) {
        const char* h = getenv("UBPL_PSA_HALO");
        const char* t = getenv("UBPL_PSA_TEAMS");
        const int hv = h ? atoi(h) : -1;
        int expect = -2;
        g_psa_halo.compare_exchange_strong(expect, hv == 0 || hv == 1 ? hv : -1);
        expect = -2;
        g_psa_teams.compare_exchange_strong(expect, t ? atoi(t) : -1);
    }
    return {g_psa_halo.load(std::memory_order_relaxed), g_psa_teams.load(std::memory_order_relaxed)};
}
}  // namespace


UBPL_API int ubpl_set_psa_dispatch(int halo_mode, int teams) {
    if (halo_mode == -2 && teams == -2) {   // back to the environment's values (read again at the next launch)
        g_psa_halo.store(-2);
        g_psa_teams.store(-2);
        return 0;
    }
    if (halo_mode < -1 || halo_mode > 3 || teams < -1 || teams > 2) return (int)hipErrorInvalidValue;
    psa_dispatch();                       // the environment's values are read first, then replaced
    g_psa_halo.store(halo_mode);
    g_psa_teams.store(teams);
    return 0;
}

UBPL_API int ubpl_conv2d_forward_psa(const uint16_t* xs, int64_t xplane, int B, int Cin, int H, int W, int pad,
                                     const uint16_t* wsplit, int64_t wplane, const float* bias, int Cout, int KS,
                                     const float* res, float* y, float* slab, int npieces, float* stat_part,
                                     const float* bn_x, const float* bn_coef, int bn_relu, float* bn_part,
                                     const float* act_scale, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (Cin % 16 != 0 || npieces < 1 || npieces > 3 || pad < KS / 2 || (KS != 1 && KS != 3 && KS != 4))
        return (int)hipErrorInvalidValue;
    const ubpl::BnBwdEpi bwd{bn_part ? bn_x : nullptr, bn_coef, bn_relu, bn_part};
    if ((((uintptr_t)wsplit) & 15) != 0 || (((uintptr_t)xs) & 15) != 0 || (wplane % 8) != 0 || (xplane % 8) != 0)
        return (int)hipErrorInvalidValue;
    const int64_t N = (int64_t)B * H * W;
    const Plan pl = fwd_plan(Cout, N, Cin * KS * KS, npieces, true);
    if (pl.splits > 1 && slab == nullptr) return (int)hipErrorInvalidValue;
    // unsplit 128-row launches run on 256-pixel tiles (+12 % on the 64x64-level
    // 3x3 conv); tuning hook: UBPL_PSA_BN=128 keeps 128-pixel tiles everywhere
    static const bool bn256 = [] {
        const char* e = getenv("UBPL_PSA_BN");
        return !(e && atoi(e) == 128);
    }();
    // unsplit 64-row 3x3 launches run on 256-pixel tiles with a 1 x 4 wave
    // layout (wave tile 64 x 64: +14-19 % on the 128x128 64-channel and the
    // 32x32 128-channel convs); UBPL_PSA_BM64W=0 keeps 64 x 128 tiles
    static const bool bm64w = [] {
        const char* e = getenv("UBPL_PSA_BM64W");
        return !(e && atoi(e) == 0);
    }();
    if (npieces == 2 && (stat_part || bwd.part)) return (int)hipErrorInvalidValue;   // (6xbf16 / bf16 only)
    if (npieces != 2 && act_scale != nullptr) return (int)hipErrorInvalidValue;
    if (KS == 4) {   // the space-to-depth stem (ubpl_stem_s2d_split): 64-row tiles on 256 pixels
        if (pl.bm != 64 || pl.splits != 1 || (npieces != 3 && npieces != 1) || N % 256 != 0)
            return (int)hipErrorInvalidValue;
        if (npieces == 1)
            return launch_psa<64, 4, 1, 256, 1>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin, H, W, pad, Cout,
                                                pl, slab, stat_part, bwd, st, act_scale);
        return launch_psa<64, 4, 3, 256, 1>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin, H, W, pad, Cout, pl,
                                            slab, stat_part, bwd, st, act_scale);
    }
    // the one-piece (bf16) path: KSUB 16-k steps per stage and barrier (UBPL_PSA_KSUB1 in 1..4)
    static const int ksub1 = [] {
        const char* e = getenv("UBPL_PSA_KSUB1");
        const int v = e ? atoi(e) : PSA_KSUB1;
        return v >= 1 && v <= 4 ? v : PSA_KSUB1;
    }();
#define UBPL_PSA1(BM_, KS_, WGM_)                                                                                  \
    do {                                                                                                           \
        switch (ksub1) {                                                                                           \
            case 2: return launch_psa<BM_, KS_, 1, 256, WGM_, 2>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin, \
                                                                   H, W, pad, Cout, pl, slab, stat_part, bwd, st, act_scale); \
            case 3: return launch_psa<BM_, KS_, 1, 256, WGM_, 3>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin, \
                                                                   H, W, pad, Cout, pl, slab, stat_part, bwd, st, act_scale); \
            case 4: return launch_psa<BM_, KS_, 1, 256, WGM_, 4>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin, \
                                                                   H, W, pad, Cout, pl, slab, stat_part, bwd, st, act_scale); \
            default: return launch_psa<BM_, KS_, 1, 256, WGM_, 1>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin,\
                                                                    H, W, pad, Cout, pl, slab, stat_part, bwd, st, act_scale);\
        }                                                                                                          \
    } while (0)
    // 3x3 stride-1 pad-1 on the split / bf16 paths, 128- or 64-row tiles, whole-row 256-pixel
    // tiles: the input halo staged once per channel group (conv_psah_kernel).  Default
    // (measured, tools/psa_bench.py, profiles/r04_psa_diag.txt): the split paths (6xbf16, 2xfp16)
    // on the one-halo-buffer, two-workgroups-per-CU variant (6xbf16: 212 vs 221 us at 128 ch
    // 64x64, 750 vs 786 at 256 ch, 250 vs 295 at 64 ch 128x128, 69 vs 75 at 128 ch 32x32); the
    // bf16 path at W <= 64 (54.6 vs 59.4 us at 128 ch 64x64, 184 vs 206 at 256 ch, 22.0 vs 27.0
    // at 128 ch 32x32; 104 vs 87 at 128x128: not there).
    // halo dispatch (psa_dispatch(), read once): -1 default; 0: none (conv_psa_kernel); 1:
    // every eligible launch on the double-buffered halo (two teams where the grid fills the
    // chip); test-only through ubpl_set_psa_dispatch: 2: as 1, required (a 3x3 launch the
    // kernel cannot take is an error); 3: the one-buffer variant for every eligible split-piece
    // launch, required.  The tests compare the kernels in one process; the modes compute in
    // the same order, bit for bit.
    const int halo_mode = psa_dispatch().halo;
    const bool split_np = npieces == 3 || npieces == 2;
    // (2xfp16 on double-buffered halos at two workgroups per CU — they fit 80 KB at W <= 64 —
    // measured slower than the one buffer: 122.4 vs 116.2 us, 426.5 vs 433.0 img/s, round 6)
    const bool one_buf = split_np && (halo_mode >= 3 || halo_mode < 0);
    // the 96-wide planes: 192-pixel tiles on 128 rows whatever the plan's row block (its
    // cost model is conv_psa_kernel's), the one-buffer variant only
    const bool w96 = W == 96 && Cout % 128 == 0 && H % 2 == 0 &&
                     ((split_np && one_buf) || (npieces == 1 && halo_mode > 0));   // (bf16: opt-in, slower)
    const bool halo_ok = KS == 3 && pad == 1 && pl.splits == 1 && !stat_part && !bwd.part &&
                         (((pl.bm == 128 || bm64w) && (W == 32 || W == 64 || W == 128) && H % (256 / W) == 0) ||
                          w96);
    if ((halo_mode >= 2) && KS == 3 && !halo_ok) return (int)hipErrorInvalidValue;
    const bool halo = halo_mode < 0 ? ((npieces == 1 && W <= 64) || one_buf) : halo_mode != 0;
    const float osc = psa_osc(npieces, Cin * KS * KS, act_scale != nullptr);
    if (halo && halo_ok) {
        // two 4-wave teams per workgroup (512 pixels: one halo, one A ring for both,
        // two waves per SIMD) where the grid still fills the chip; UBPL_PSA_TEAMS=1 / 2
        const int te = psa_dispatch().teams;
        const int mt = (Cout + pl.bm - 1) / pl.bm;
        const bool teams2 = !one_buf && (te > 0 ? te == 2 : (N / 512) * mt >= 256) && W <= 64 &&
                            H % (512 / W) == 0;
        if (teams2) {
            const dim3 grid2((unsigned)(N / 512), (unsigned)mt);
#define UBPL_PSAH2(W_, BM_)                                                                                         \
    do {                                                                                                            \
        if (npieces == 3)                                                                                           \
            hipLaunchKernelGGL((conv_psah_kernel<W_, 3, BM_, 2>), grid2, dim3(2 * NT), 0, st, xs, xplane, wsplit,   \
                               wplane, bias, res, y, B, Cin, H, Cout, osc, act_scale);                                         \
        else if (npieces == 2)                                                                                      \
            hipLaunchKernelGGL((conv_psah_kernel<W_, 2, BM_, 2>), grid2, dim3(2 * NT), 0, st, xs, xplane, wsplit,   \
                               wplane, bias, res, y, B, Cin, H, Cout, osc, act_scale);                                         \
        else                                                                                                        \
            hipLaunchKernelGGL((conv_psah_kernel<W_, 1, BM_, 2>), grid2, dim3(2 * NT), 0, st, xs, xplane, wsplit,   \
                               wplane, bias, res, y, B, Cin, H, Cout, osc, act_scale);                                         \
    } while (0)
            if (pl.bm == 128) {
                if (W == 64) UBPL_PSAH2(64, 128);
                else UBPL_PSAH2(32, 128);
            } else {
                if (W == 64) UBPL_PSAH2(64, 64);
                else UBPL_PSAH2(32, 64);
            }
#undef UBPL_PSAH2
            UBPL_LAUNCH_CHECK();
            return 0;
        }
        if (w96) {
            const dim3 g96((unsigned)(N / 192), (unsigned)(Cout / 128));
            if (npieces == 3)
                hipLaunchKernelGGL((conv_psah_kernel<96, 3, 128, 1, 1, 192>), g96, dim3(NT), 0, st, xs, xplane, wsplit,
                                   wplane, bias, res, y, B, Cin, H, Cout, osc, act_scale);
            else if (npieces == 2)
                hipLaunchKernelGGL((conv_psah_kernel<96, 2, 128, 1, 1, 192>), g96, dim3(NT), 0, st, xs, xplane, wsplit,
                                   wplane, bias, res, y, B, Cin, H, Cout, osc, act_scale);
            else
                hipLaunchKernelGGL((conv_psah_kernel<96, 1, 128, 1, 2, 192>), g96, dim3(NT), 0, st, xs, xplane, wsplit,
                                   wplane, bias, res, y, B, Cin, H, Cout, osc, act_scale);
            UBPL_LAUNCH_CHECK();
            return 0;
        }
        const dim3 grid((unsigned)(N / 256), (unsigned)mt);
        // one halo buffer, two workgroups per CU (split pieces), or double-buffered halos
#define UBPL_PSAH(W_, BM_)                                                                                           \
    do {                                                                                                             \
        if (npieces == 3 && one_buf)                                                                                 \
            hipLaunchKernelGGL((conv_psah_kernel<W_, 3, BM_, 1, 1>), grid, dim3(NT), 0, st, xs, xplane, wsplit,      \
                               wplane, bias, res, y, B, Cin, H, Cout, osc, act_scale);                                          \
        else if (npieces == 2 && one_buf)                                                                            \
            hipLaunchKernelGGL((conv_psah_kernel<W_, 2, BM_, 1, 1>), grid, dim3(NT), 0, st, xs, xplane, wsplit,      \
                               wplane, bias, res, y, B, Cin, H, Cout, osc, act_scale);                                          \
        else if (npieces == 3)                                                                                       \
            hipLaunchKernelGGL((conv_psah_kernel<W_, 3, BM_>), grid, dim3(NT), 0, st, xs, xplane, wsplit, wplane,    \
                               bias, res, y, B, Cin, H, Cout, osc, act_scale);                                                  \
        else if (npieces == 2)                                                                                       \
            hipLaunchKernelGGL((conv_psah_kernel<W_, 2, BM_>), grid, dim3(NT), 0, st, xs, xplane, wsplit, wplane,    \
                               bias, res, y, B, Cin, H, Cout, osc, act_scale);                                                  \
        else                                                                                                         \
            hipLaunchKernelGGL((conv_psah_kernel<W_, 1, BM_>), grid, dim3(NT), 0, st, xs, xplane, wsplit, wplane,    \
                               bias, res, y, B, Cin, H, Cout, osc, act_scale);                                                  \
    } while (0)
        if (pl.bm == 128) {
            if (W == 64) UBPL_PSAH(64, 128);
            else if (W == 128) UBPL_PSAH(128, 128);
            else UBPL_PSAH(32, 128);
        } else {
            if (W == 64) UBPL_PSAH(64, 64);
            else if (W == 128) UBPL_PSAH(128, 64);
            else UBPL_PSAH(32, 64);
        }
#undef UBPL_PSAH
        UBPL_LAUNCH_CHECK();
        return 0;
    }
    if (bm64w && pl.bm == 64 && pl.splits == 1 && N % 256 == 0 && (KS == 3 || npieces == 1)) {
        if (npieces == 3)
            return launch_psa<64, 3, 3, 256, 1>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin, H, W, pad, Cout, pl,
                                                slab, stat_part, bwd, st, act_scale);
        if (npieces == 2)
            return launch_psa<64, 3, 2, 256, 1>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin, H, W, pad, Cout, pl,
                                                slab, stat_part, bwd, st, act_scale);
        if (KS == 3) UBPL_PSA1(64, 3, 1);
        UBPL_PSA1(64, 1, 1);
    }
    if (bn256 && pl.bm == 128 && pl.splits == 1 && N % 256 == 0) {
        if (npieces == 1) {
            if (KS == 3) UBPL_PSA1(128, 3, 2);
            UBPL_PSA1(128, 1, 2);
        }
        if (npieces == 2) {
            if (KS == 3)
                return launch_psa<128, 3, 2, 256>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin, H, W, pad, Cout,
                                                  pl, slab, stat_part, bwd, st, act_scale);
            return launch_psa<128, 1, 2, 256>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin, H, W, pad, Cout, pl,
                                              slab, stat_part, bwd, st, act_scale);
        }
        if (KS == 3) {
            return launch_psa<128, 3, 3, 256>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin, H, W, pad, Cout, pl,
                                              slab, stat_part, bwd, st, act_scale);
        }
        return launch_psa<128, 1, 3, 256>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin, H, W, pad, Cout, pl,
                                          slab, stat_part, bwd, st, act_scale);
    }
#define UBPL_PS(BM_, KS_, NP_) \
    return launch_psa<BM_, KS_, NP_, 128>(xs, xplane, wsplit, wplane, bias, res, y, B, Cin, H, W, pad, Cout, pl, \
                                          slab, stat_part, bwd, st, act_scale)
#define UBPL_PS_BM(KS_, NP_)          \
    if (pl.bm == 128) UBPL_PS(128, KS_, NP_); \
    UBPL_PS(64, KS_, NP_)
    if (KS == 1) {
        if (npieces == 1) { UBPL_PS_BM(1, 1); }
        if (npieces == 2) { UBPL_PS_BM(1, 2); }
        UBPL_PS_BM(1, 3);
    }
    if (KS == 3) {
        if (npieces == 1) { UBPL_PS_BM(3, 1); }
        if (npieces == 2) { UBPL_PS_BM(3, 2); }
        UBPL_PS_BM(3, 3);
    }
#undef UBPL_PS_BM
#undef UBPL_PS
#undef UBPL_PSA1
    return (int)hipErrorInvalidValue;
}

// ---- 1x1 with the split on load
namespace {
bool sol_supported(int B, int Cin, int Cout, int P) {
    // Cout % 64 != 0 (the 16-channel heatmap projection, preds.*.conv): one
    // 64-row tile with the rows past Cout clamped on load and never stored
    return B > 0 && P > 0 && Cin % 16 == 0 && Cin > 0 && Cout % 16 == 0 && P % 4 == 0 && (int64_t)B * P >= 4 &&
           (int64_t)B * Cin * P * 4 < (1LL << 32) && (int64_t)Cout * Cin * 2 < (1LL << 31);
}
}  // namespace

// 1 when ubpl_conv1x1_forward_split_load takes this shape and fills the chip
// (>= one 256-pixel workgroup per CU); 0: use the f32 1x1 kernel (split-K plans).
// Output-channel block: 128 rows (each pixel tile split once per 128 channels)
// unless that leaves CUs idle; then 64 (the 32x32-plane 256->128 convs at B=32:
// 128 -> 256 workgroups).
// UBPL_SOL_BM=64: 64-row tiles everywhere (A/B knob); UBPL_SOL_NS=3: 3-stage ring on 64-row tiles
static int sol_env(const char* name, int dflt) {
    const char* e = getenv(name);
    return e ? atoi(e) : dflt;
}
static int sol_bm(int64_t N, int Cout) {
    static const int force = sol_env("UBPL_SOL_BM", 0);
    if (Cout % 128 != 0 || force == 64) return 64;
    return ((N + 255) / 256) * (Cout / 128) >= occ_info().ncu ? 128 : 64;
}

UBPL_API int ubpl_conv1x1_split_load_preferred(int B, int Cin, int Cout, int P) {
    if (!sol_supported(B, Cin, Cout, P)) return 0;
    const int64_t N = (int64_t)B * P;
    const int bm = sol_bm(N, Cout);
    const int64_t wgs = ((N + 255) / 256) * ((Cout + bm - 1) / bm);
    return wgs >= occ_info().ncu ? 1 : 0;
}

// y = conv1x1(relu(x*pscale + pshift) or x) + bias (+ res, may alias y) on the
// 6xbf16 path, x NCHW f32 split while it is staged (conv1x1_sol_kernel).
// wsplit: 3 bf16 planes (`wplane` elements apart) of [Cout][Cin] from
// ubpl_conv_weights_split (mode 0 of a 1x1 conv; mode 1 = its data gradient,
// then x = dy and Cin/Cout swap).  Cin % 16 == 0, Cout % 64 == 0, P % 4 == 0,
// x / wsplit 16-B aligned.  stat_part (nullable): BatchNorm partials of y.
UBPL_API int ubpl_conv1x1_forward_split_load(const float* x, int B, int Cin, int P, const uint16_t* wsplit,
                                             int64_t wplane, const float* bias, int Cout, const float* pscale,
                                             const float* pshift, const float* res, float* y, float* stat_part,
                                             const float* bn_x, const float* bn_coef, int bn_relu, float* bn_part,
                                             int npieces, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (!sol_supported(B, Cin, Cout, P) || (((uintptr_t)x) & 15) || (((uintptr_t)wsplit) & 15) || (wplane % 8) ||
        npieces < 1 || npieces > 3)
        return (int)hipErrorInvalidValue;
    const bool pro = pscale != nullptr;
    if (pro && Cin > SOL_PRO_K) return (int)hipErrorInvalidValue;
    const int64_t N = (int64_t)B * P;
    const int bm = sol_bm(N, Cout);
    const ubpl::BnBwdEpi bwd{bn_part ? bn_x : nullptr, bn_coef, bn_relu, bn_part};
    dim3 grid((unsigned)((N + 255) / 256), (unsigned)((Cout + bm - 1) / bm));
    const bool epi = stat_part != nullptr || bn_part != nullptr;
    if (epi && (npieces != 3 || Cout % 64 != 0)) return (int)hipErrorInvalidValue;   // (epilogue partials: 6xbf16, whole tiles)
    const float asc = ubpl::FP16_ACT_SCALE, osc = psa_osc(npieces, Cin);
    static const bool ns3 = sol_env("UBPL_SOL_NS", 2) == 3;
    // the activation ring 3 stages deep beside the weights' 2 (two K steps of the HBM
    // stream in flight per workgroup; the default since round 5, measured even with the
    // 2-stage ring, profiles/r05_v1_sol_nsb.txt); UBPL_SOL_NSB=2: one ring of 2 stages
    static const bool nsb3 = sol_env("UBPL_SOL_NSB", 3) == 3;
#define UBPL_SOL(BM_, PRO_)                                                                                       \
    do {                                                                                                          \
        if (npieces == 1 && nsb3)                                                                                 \
            hipLaunchKernelGGL((conv1x1_sol_kernel<BM_, PRO_, false, 1, 2, 256, 3>), grid, dim3(NT), 0, st, x,    \
                               wsplit, wplane, bias, pscale, pshift, res, y, B, Cin, P, Cout, nullptr, bwd, asc, osc); \
        else if (npieces == 1)                                                                                    \
            hipLaunchKernelGGL((conv1x1_sol_kernel<BM_, PRO_, false, 1>), grid, dim3(NT), 0, st, x, wsplit,       \
                               wplane, bias, pscale, pshift, res, y, B, Cin, P, Cout, nullptr, bwd, asc, osc);    \
        else if (npieces == 2 && nsb3)                                                                            \
            hipLaunchKernelGGL((conv1x1_sol_kernel<BM_, PRO_, false, 2, 2, 256, 3>), grid, dim3(NT), 0, st, x,    \
                               wsplit, wplane, bias, pscale, pshift, res, y, B, Cin, P, Cout, nullptr, bwd, asc, osc); \
        else if (npieces == 2)                                                                                    \
            hipLaunchKernelGGL((conv1x1_sol_kernel<BM_, PRO_, false, 2>), grid, dim3(NT), 0, st, x, wsplit,       \
                               wplane, bias, pscale, pshift, res, y, B, Cin, P, Cout, nullptr, bwd, asc, osc);    \
        else if (BM_ == 64 && ns3 && !epi)                                                                        \
            hipLaunchKernelGGL((conv1x1_sol_kernel<64, PRO_, false, 3, 3>), grid, dim3(NT), 0, st, x, wsplit,     \
                               wplane, bias, pscale, pshift, res, y, B, Cin, P, Cout, nullptr, bwd, asc, osc);    \
        else if (epi)                                                                                             \
            hipLaunchKernelGGL((conv1x1_sol_kernel<BM_, PRO_, true>), grid, dim3(NT), 0, st, x, wsplit, wplane,   \
                               bias, pscale, pshift, res, y, B, Cin, P, Cout, stat_part, bwd, asc, osc);          \
        else if (nsb3)                                                                                            \
            hipLaunchKernelGGL((conv1x1_sol_kernel<BM_, PRO_, false, 3, 2, 256, 3>), grid, dim3(NT), 0, st, x,    \
                               wsplit, wplane, bias, pscale, pshift, res, y, B, Cin, P, Cout, nullptr, bwd, asc, osc); \
        else                                                                                                      \
            hipLaunchKernelGGL((conv1x1_sol_kernel<BM_, PRO_>), grid, dim3(NT), 0, st, x, wsplit, wplane, bias,   \
                               pscale, pshift, res, y, B, Cin, P, Cout, nullptr, bwd, asc, osc);                  \
    } while (0)
    if (bm == 128) {
        if (pro) UBPL_SOL(128, true);
        else UBPL_SOL(128, false);
    } else {
        if (pro) UBPL_SOL(64, true);
        else UBPL_SOL(64, false);
    }
#undef UBPL_SOL
    UBPL_LAUNCH_CHECK();
    return 0;
}

// ---- 3x3 weight gradient on the split path
namespace {
int wgrad3_cb(int Cin, int Cout) { return (Cin % 128 == 0 && Cout % 128 == 0) ? 128 : 64; }

int wgrad3_splits(int B, int Cin, int Cout, int H, int W) {
    const int cb = wgrad3_cb(Cin, Cout);
    // 128: one tap x 128 channels per n-tile; 64: one kernel row (3 taps) x 64 channels
    const int tiles = cb == 128 ? 9 * (Cin / cb) * (Cout / cb) : 3 * (Cin / 64) * (Cout / 64);
    const int steps = B * H * (W / 16);
    static const int wgs = sol_env("UBPL_WGRAD3_WGS", 512);   // two workgroups per CU (256: even within noise, round 6)
    int s = wgs / tiles;                               // whole rounds of the CUs, not one over
    if (s < 1) s = 1;
    if (s > steps / 8) s = steps / 8 > 0 ? steps / 8 : 1;   // >= 8 K steps per split
    const int per = (steps + s - 1) / s;
    return (steps + per - 1) / per;
}
}  // namespace

UBPL_API int64_t ubpl_wgrad3_psa_workspace(int B, int Cin, int Cout, int H, int W) {
    if (Cin % 64 || Cout % 64 || W % 16) return 0;
    return (int64_t)wgrad3_splits(B, Cin, Cout, H, W) * Cout * (9 * Cin + 1);
}

// dw[Cout,Cin,3,3] (+)= 3x3 weight gradient, db[Cout] (+)= sum dy (nullable), from
// PSA operands with a 1-pixel border: dys = split(dy) [B][Cout/16][H+2][W+2][16],
// xs = split(conv input) [B][Cin/16][H+2][W+2][16], npieces = 3.  Needs
// Cin % 64 == 0, Cout % 64 == 0 (128-channel tiles when both are multiples of 128), W % 16 == 0.
// slab: ubpl_wgrad3_psa_workspace floats.
UBPL_API int ubpl_wgrad3_psa(const uint16_t* dys, int64_t dplane, const uint16_t* xs, int64_t xplane, int B, int Cin,
                             int Cout, int H, int W, float* slab, float* dw, float* db, int accumulate, int npieces,
                             const float* dscale, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (Cin % 64 || Cout % 64 || W % 16 || npieces < 1 || npieces > 3 || slab == nullptr ||
        (npieces == 2) != (dscale != nullptr))
        return (int)hipErrorInvalidValue;
    if ((((uintptr_t)dys) & 15) || (((uintptr_t)xs) & 15) || (dplane % 8) || (xplane % 8)) return (int)hipErrorInvalidValue;
    const int splits = wgrad3_splits(B, Cin, Cout, H, W);
    const int steps = B * H * (W / 16);
    const int per = (steps + splits - 1) / splits;
    const int cb = wgrad3_cb(Cin, Cout);
    if (cb == 128) {
        dim3 grid((unsigned)(9 * (Cin / cb)), (unsigned)(Cout / cb), (unsigned)splits);
        if (npieces == 1)
            hipLaunchKernelGGL((wgrad3_psa_kernel<1, 128>), grid, dim3(NT), 0, st, dys, dplane, xs, xplane, B, Cin,
                               Cout, H, W, per, slab, dscale);
        else if (npieces == 2)
            hipLaunchKernelGGL((wgrad3_psa_kernel<2, 128>), grid, dim3(NT), 0, st, dys, dplane, xs, xplane, B, Cin,
                               Cout, H, W, per, slab, dscale);
        else
            hipLaunchKernelGGL((wgrad3_psa_kernel<3, 128>), grid, dim3(NT), 0, st, dys, dplane, xs, xplane, B, Cin,
                               Cout, H, W, per, slab, dscale);
    } else {
        dim3 grid((unsigned)(3 * (Cin / 64)), (unsigned)(Cout / 64), (unsigned)splits);
        if (npieces == 1)
            hipLaunchKernelGGL((wgrad3_psa64_kernel<1>), grid, dim3(NT), 0, st, dys, dplane, xs, xplane, B, Cin, Cout,
                               H, W, per, slab, dscale);
        else if (npieces == 2)
            hipLaunchKernelGGL((wgrad3_psa64_kernel<2>), grid, dim3(NT), 0, st, dys, dplane, xs, xplane, B, Cin, Cout,
                               H, W, per, slab, dscale);
        else
            hipLaunchKernelGGL((wgrad3_psa64_kernel<3>), grid, dim3(NT), 0, st, dys, dplane, xs, xplane, B, Cin, Cout,
                               H, W, per, slab, dscale);
    }
    UBPL_LAUNCH_CHECK();
    return ubpl_wgrad_slab_reduce(slab, splits, Cout, Cin, 9, db != nullptr, dw, db, accumulate, stream);
}

// ---- the stem's weight gradient on the split path (space-to-depth)
namespace {
int wgrad_stem_splits(int B, int Cout, int H, int W) {
    const int steps = B * H * (W / 16);
    int s = 512 / (Cout / 64);                          // one round of 2 workgroups per CU
    if (s < 1) s = 1;
    if (s > steps / 8) s = steps / 8 > 0 ? steps / 8 : 1;
    const int per = (steps + s - 1) / s;
    return (steps + per - 1) / per;
}
}  // namespace

UBPL_API int64_t ubpl_wgrad_stem_psa_workspace(int B, int Cout, int H, int W) {
    if (B < 1 || Cout % 64 || W % 16 || H < 1) return 0;
    return (int64_t)wgrad_stem_splits(B, Cout, H, W) * Cout * 257 + (int64_t)Cout * 257;
}

UBPL_API int ubpl_wgrad_stem_psa(const uint16_t* dys, int64_t dplane, const uint16_t* xs, int64_t xplane, int B,
                                 int C, int Cout, int H, int W, int KS, float* slab, float* dw, float* db,
                                 int accumulate, int npieces, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if ((npieces != 3 && npieces != 1) || KS != 7 || C < 1 || C > 4 || Cout % 64 || W % 16 || H < 1 || B < 1 ||
        slab == nullptr)
        return (int)hipErrorInvalidValue;
    if ((((uintptr_t)dys) & 15) || (((uintptr_t)xs) & 15) || (dplane % 8) || (xplane % 8))
        return (int)hipErrorInvalidValue;
    const int splits = wgrad_stem_splits(B, Cout, H, W);
    const int steps = B * H * (W / 16);
    const int per = (steps + splits - 1) / splits;
    if (npieces == 1)
        hipLaunchKernelGGL((wgrad_stem_psa_kernel<1>), dim3((unsigned)(Cout / 64), (unsigned)splits), dim3(NT), 0,
                           st, dys, dplane, xs, xplane, B, Cout, H, W, per, slab);
    else
        hipLaunchKernelGGL((wgrad_stem_psa_kernel<3>), dim3((unsigned)(Cout / 64), (unsigned)splits), dim3(NT), 0,
                           st, dys, dplane, xs, xplane, B, Cout, H, W, per, slab);
    UBPL_LAUNCH_CHECK();
    float* dws = slab + (int64_t)splits * Cout * 257;
    const int e = ubpl_wgrad_slab_reduce(slab, splits, Cout, 16, 16, 1, dws, dws + (int64_t)Cout * 256, 0, stream);
    if (e) return e;
    const int64_t total = (int64_t)Cout * C * KS * KS;
    hipLaunchKernelGGL(stem_wgrad_map_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, dws,
                       dws + (int64_t)Cout * 256, Cout, C, dw, db, accumulate);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// ---- 1x1 weight gradient with the split on load
namespace {
int wgrad1_cb(int C) { return C % 128 == 0 ? 128 : 64; }

bool wgrad1_sol_supported(int B, int Cin, int Cout, int P) {
    return B > 0 && Cin % 64 == 0 && Cout % 64 == 0 && P % 16 == 0 && P > 0 &&
           (int64_t)B * Cin * P < (1LL << 31) && (int64_t)B * Cout * P < (1LL << 31);
}

int wgrad1_sol_splits(int B, int Cin, int Cout, int P) {
    const int tiles = (Cin / wgrad1_cb(Cin)) * (Cout / wgrad1_cb(Cout));
    const int steps = B * (P / 16);
    static const int wgs = sol_env("UBPL_WGRAD1_WGS", 256);   // one workgroup per CU (profiles/r06_v10_wgrad_wgs_ab.txt)
    int s = wgs / tiles;                                    // whole rounds of the CUs
    if (s < 1) s = 1;
    if (s > steps / 8) s = steps / 8 > 0 ? steps / 8 : 1;   // >= 8 K steps per split
    const int per = (steps + s - 1) / s;
    return (steps + per - 1) / per;
}
}  // namespace

// Floats of slab ubpl_wgrad1x1_split_load needs; 0 = shape not supported
// (Cin % 64, Cout % 64, P % 16): use ubpl_conv2d_wgrad.
UBPL_API int64_t ubpl_wgrad1x1_split_load_workspace(int B, int Cin, int Cout, int P) {
    if (!wgrad1_sol_supported(B, Cin, Cout, P)) return 0;
    return (int64_t)wgrad1_sol_splits(B, Cin, Cout, P) * Cout * (Cin + 1);
}

// dw[Cout,Cin,1,1] (+)= 1x1 weight gradient, db[Cout] (+)= sum dy (nullable),
// on the 6xbf16 path with both f32 operands split while they are staged
// (wgrad1_sol_kernel): dy [B,Cout,P], x [B,Cin,P], v = relu(x*pscale + pshift)
// when pscale != nullptr.  16-B aligned dy / x.
UBPL_API int ubpl_wgrad1x1_split_load(const float* dy, const float* x, int B, int Cin, int Cout, int P,
                                      const float* pscale, const float* pshift, float* slab, float* dw, float* db,
                                      int accumulate, int npieces, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    if (!wgrad1_sol_supported(B, Cin, Cout, P) || slab == nullptr || (((uintptr_t)dy) & 15) ||
        (((uintptr_t)x) & 15) || (npieces != 1 && npieces != 3))
        return (int)hipErrorInvalidValue;
    const int splits = wgrad1_sol_splits(B, Cin, Cout, P);
    const int steps = B * (P / 16);
    const int per = (steps + splits - 1) / splits;
    const int cm = wgrad1_cb(Cout), cn = wgrad1_cb(Cin);
    dim3 grid((unsigned)(Cin / cn), (unsigned)(Cout / cm), (unsigned)splits);
#define UBPL_W1(CM_, CN_)                                                                                          \
    do {                                                                                                           \
        if (pscale != nullptr && npieces == 3)                                                                     \
            hipLaunchKernelGGL((wgrad1_sol_kernel<true, 3, CM_, CN_>), grid, dim3(NT), 0, st, dy, x, pscale,       \
                               pshift, B, Cin, Cout, P, per, slab);                                                \
        else if (npieces == 3)                                                                                     \
            hipLaunchKernelGGL((wgrad1_sol_kernel<false, 3, CM_, CN_>), grid, dim3(NT), 0, st, dy, x, pscale,      \
                               pshift, B, Cin, Cout, P, per, slab);                                                \
        else if (pscale != nullptr)                                                                                \
            hipLaunchKernelGGL((wgrad1_sol_kernel<true, 1, CM_, CN_>), grid, dim3(NT), 0, st, dy, x, pscale,       \
                               pshift, B, Cin, Cout, P, per, slab);                                                \
        else                                                                                                       \
            hipLaunchKernelGGL((wgrad1_sol_kernel<false, 1, CM_, CN_>), grid, dim3(NT), 0, st, dy, x, pscale,      \
                               pshift, B, Cin, Cout, P, per, slab);                                                \
    } while (0)
    if (cm == 128 && cn == 128) UBPL_W1(128, 128);
    else if (cm == 128) UBPL_W1(128, 64);
    else if (cn == 128) UBPL_W1(64, 128);
    else UBPL_W1(64, 64);
#undef UBPL_W1
    UBPL_LAUNCH_CHECK();
    return ubpl_wgrad_slab_reduce(slab, splits, Cout, Cin, 1, db != nullptr, dw, db, accumulate, stream);
}

// ---- the stem on the split path (space-to-depth, see stem_s2d_split_kernel)
// x [B][C][H][W] (C <= 4, H, W even) -> PSA planes [B][1][H/2 + 2pad][W/2 + 2pad][16]
// of the 4 phase images per channel; pad >= 2 for the 7x7 stem.
UBPL_API int ubpl_stem_s2d_split(const float* x, int B, int C, int H, int W, int pad, int npieces, uint16_t* dst,
                                 int64_t plane, void* stream) {
    if (C < 1 || C > 4 || (H & 1) || (W & 1) || (npieces != 3 && npieces != 1) || pad < 0 || (plane % 8) != 0)
        return (int)hipErrorInvalidValue;
    const int Hp = H / 2 + 2 * pad, Wp = W / 2 + 2 * pad;
    dim3 grid((unsigned)((Hp * Wp + 255) / 256), (unsigned)B);
    if (npieces == 1)
        hipLaunchKernelGGL(stem_s2d_split_kernel<1>, grid, dim3(256), 0, (hipStream_t)stream, x, C, H, W, pad, dst,
                           plane);
    else
        hipLaunchKernelGGL(stem_s2d_split_kernel<3>, grid, dim3(256), 0, (hipStream_t)stream, x, C, H, W, pad, dst,
                           plane);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// w [Cout][C][KS][KS] (KS odd, C <= 4) -> split weights of the s2d conv for
// ubpl_conv2d_forward_psa (Cin = 16, KS' = (KS + 1) / 2 rounded up to even = 4
// for the 7x7 stem): npieces planes of Cout * KS'^2 * 16 bf16.
UBPL_API int ubpl_stem_weight_s2d_split(const float* w, int Cout, int C, int KS, int npieces, uint16_t* dst,
                                        int64_t plane, void* stream) {
    const int KT = ((KS + 1) / 2 + 1) & ~1;
    if (C < 1 || C > 4 || !(KS & 1) || (npieces != 3 && npieces != 1) || KT != 4 || (plane % 8) != 0)
        return (int)hipErrorInvalidValue;
    const int64_t total = (int64_t)Cout * KT * KT * 16;
    if (npieces == 1)
        hipLaunchKernelGGL(stem_weight_s2d_split_kernel<1>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, w, Cout, C, KS, KT, dst, plane);
    else
        hipLaunchKernelGGL(stem_weight_s2d_split_kernel<3>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                           (hipStream_t)stream, w, Cout, C, KS, KT, dst, plane);
    UBPL_LAUNCH_CHECK();
    return 0;
}
