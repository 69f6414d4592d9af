// BatchNorm2d (train-mode batch statistics, eval-mode running statistics) for
// the hourglass (models/base/layers.py:41,57-61; nn.BatchNorm2d momentum 0.1,
// eps 1e-5).  NCHW: a channel is B contiguous HW planes.
//
// Forward never materialises bn(x) for the residual branches: the statistics
// kernels produce per-channel (scale, shift) = (g*invstd, b - mean*g*invstd)
// — PyTorch's own transform form — and the consuming convolution applies
// relu(x*scale + shift) while staging its operand (conv.hip prologue).
//
// Statistics: each (channel, batch-slice) workgroup accumulates sum and sum of
// squares of (x - x0) — x0 a sample of the channel, which removes the
// cancellation of E[x^2] - E[x]^2 — then reduces in f64.  Partials go to a
// slab; the channel's last-arriving workgroup (ticket counter) combines them
// in slice order: deterministic, one launch.
//
// Backward: dyp = dz * [x*scale + shift > 0] (ReLU mask recomputed bit-for-bit
// as the forward prologue computed it); per channel S1 = sum dyp,
// S2 = sum dyp*(x - mean); dbeta += S1, dgamma += S2*invstd;
// dx = a*dyp + b*(x - mean) + c with a = g*invstd, b = -g*invstd^3*S2/N,
// c = -g*invstd*S1/N, plus up to two addends (residual-gradient sums).
#include "common.h"
#include <cstdlib>

namespace {

// Last-arriver hand-off (cdna_hip_programming.md §6 Guideline 16, split-K
// counter form with write-through payload): thread 0 of every (channel,
// slice) block stores its two partials with agent-scope atomic stores (sc1,
// write-through: no release fence, which would write back the whole L2),
// drains them, and takes a ticket; the block drawing the last ticket reads the
// channel's partials with agent-scope atomic loads (sc1: past any stale L1
// line), one slice per lane, sums them in a fixed order (deterministic) and
// resets the counter.
__device__ __forceinline__ void publish2(double* p, double a, double b) {
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(a),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p + 1), (unsigned long long)__double_as_longlong(b),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double consume(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// UBPL_BN_ACQREL=1 (diagnostic): the ticket RMW with agent-scope acq_rel ordering
// (release: the partials' stores complete and the L2 is written back before it;
// acquire in the last arriver: its L2 lines invalidated before the partials are read)
#ifndef UBPL_BN_ACQREL
#define UBPL_BN_ACQREL 0
#endif
__device__ __forceinline__ bool last_arriver(unsigned* cnt, unsigned n) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(cnt, 1u, UBPL_BN_ACQREL ? __ATOMIC_ACQ_REL : __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    if (old != n - 1) return false;
    __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// Wave 0 of every (channel, slice) block publishes the slice's two sums and
// takes a ticket; in the channel's last block the 64 lanes read the slices in
// parallel (one round trip, not one per slice: a serial read chain here was
// ~10 % of the training step) and sum them in a fixed tree order
// (deterministic).  Returns true in lane 0 of that block, with the totals.
// Doubles between two channels' slice partials: 2 per slice, rounded up to
// 256 B, so no two channels' partials share a cache line (their publishers
// and last arrivers may sit on different XCDs, each with its own L2).
__host__ __device__ __forceinline__ int64_t chan_stride(int nsp) { return ((int64_t)2 * nsp + 31) / 32 * 32; }

__device__ __forceinline__ bool combine_slices(double* pc, int sp, int nsp, unsigned* cnt, double d1, double d2,
                                               double& t1, double& t2) {
    if (threadIdx.x >= 64) return false;
    const int lane = threadIdx.x;
    int last = 0;
    if (lane == 0) {
        publish2(pc + sp * 2, d1, d2);
        last = last_arriver(cnt, nsp) ? 1 : 0;
    }
    if (!__shfl(last, 0, 64)) return false;
    t1 = 0.0;
    t2 = 0.0;
    for (int q = lane; q < nsp; q += 64) {
        t1 += consume(pc + q * 2);
        t2 += consume(pc + q * 2 + 1);
    }
    t1 = ubpl::wave_sum(t1);
    t2 = ubpl::wave_sum(t2);
    return lane == 0;
}

// The same hand-off with 4 values per slice: (S1, S2) summed in a fixed order and
// (Mg, Mx) maxima (order-free): the bounded backward statistics (bwd_stats_kernel
// BOUND).  Channel stride chan_stride(2 * nsp).  Returns true in EVERY lane of wave 0
// of the channel's last block (wave-uniform), the totals in lane 0.
__device__ __forceinline__ bool combine_slices4(double* pc, int sp, int nsp, unsigned* cnt, double d1, double d2,
                                                float m1, float m2, double& t1, double& t2, float& u1, float& u2) {
    if (threadIdx.x >= 64) return false;
    const int lane = threadIdx.x;
    int last = 0;
    if (lane == 0) {
        publish2(pc + sp * 4, d1, d2);
        publish2(pc + sp * 4 + 2, (double)m1, (double)m2);
        last = last_arriver(cnt, nsp) ? 1 : 0;
    }
    if (!__shfl(last, 0, 64)) return false;
    t1 = 0.0;
    t2 = 0.0;
    double a1 = 0.0, a2 = 0.0;
    for (int q = lane; q < nsp; q += 64) {
        t1 += consume(pc + q * 4);
        t2 += consume(pc + q * 4 + 1);
        a1 = fmax(a1, consume(pc + q * 4 + 2));
        a2 = fmax(a2, consume(pc + q * 4 + 3));
    }
    t1 = ubpl::wave_sum(t1);
    t2 = ubpl::wave_sum(t2);
    u1 = ubpl::wave_max((float)a1);
    u2 = ubpl::wave_max((float)a2);
    return true;
}

// Power-of-two scale that puts a tensor whose |values| <= bound at <= 2^14 (the
// 2xfp16 split's operand range: common.h split2); 1 for an all-zero tensor.
__device__ __forceinline__ float fp16_scale_for(float bound) {
    if (!(bound > 0.f) || !isfinite(bound)) return 1.f;
    int e;
    frexpf(bound, &e);                     // bound < 2^e
    e = min(max(14 - e, -60), 60);
    return ldexpf(1.f, e);
}

struct StatsOut {
    const float* gamma;
    const float* beta;
    float eps, momentum;
    float *rmean, *rvar, *mean_out, *invstd_out, *scale, *shift;
};

// One (channel c, batch slice) per block over the flattened (b, pixel) range:
// sum and sum of squares of (x - x0), x0 = x[0, c, 0]; f32 per thread, f64
// across the block and the slices.  The last block of channel c finalizes it.
// Visits the float4 offsets of channel c over images [b0, b1) of an NCHW
// tensor (hw4 float4s per plane, 256-thread blocks), calling f(slot, offset)
// (slot = the position in a group of U).  When every plane is whole
// 256-float4 rows (hw4 = 256 * 2^k: the 32x32 planes and up) each thread walks
// the same elements in the same order as the flattened (image, offset) loop,
// with no index division and U independent loads in flight; otherwise that loop.
template <int U, typename F>
__device__ __forceinline__ void visit_chan4(int b0, int b1, int C, int c, int hw4, F&& f) {
    const int kq = hw4 >> 8;
    if (kq > 0 && (hw4 & 255) == 0 && (kq & (kq - 1)) == 0) {
        const int ksh = __builtin_ctz(kq);
        const int nj = (b1 - b0) << ksh;
        const int64_t bstride = (int64_t)C * hw4;
        const int64_t base = ((int64_t)b0 * C + c) * hw4 + threadIdx.x;
        int j = 0;
        for (; j + U <= nj; j += U) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int jj = j + u;
                f(u, base + (int64_t)(jj >> ksh) * bstride + ((int64_t)(jj & (kq - 1)) << 8));
            }
        }
        for (; j < nj; ++j) f(0, base + (int64_t)(j >> ksh) * bstride + ((int64_t)(j & (kq - 1)) << 8));
        return;
    }
    // (the small planes: U iterations' loads issued together — the loop was one
    // dependent load round trip per iteration, ~10 us per launch at 16x16 / B=32;
    // same elements, same order)
    const int n4 = (b1 - b0) * hw4;
    const int st = blockDim.x;
    int i = threadIdx.x;
    for (; i + (U - 1) * st < n4; i += U * st) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int ii = i + u * st;
            const int bb = ii / hw4, o4 = ii - bb * hw4;
            f(u, ((int64_t)(b0 + bb) * C + c) * hw4 + o4);
        }
    }
    for (; i < n4; i += st) {
        const int bb = i / hw4, o4 = i - bb * hw4;
        f(0, ((int64_t)(b0 + bb) * C + c) * hw4 + o4);
    }
}

template <bool VEC, int U = 4>
__global__ void __launch_bounds__(256) stats_kernel(const float* __restrict__ x, int B, int C, int HW, int bper,
                                                   double* __restrict__ part, unsigned* __restrict__ cnt,
                                                   StatsOut o) {
    __shared__ double red[16];
    const int c = blockIdx.x, sp = blockIdx.y;
    const int b0 = sp * bper, b1 = min(B, b0 + bper);
    const float x0 = x[(int64_t)c * HW];
    float s1 = 0.f, s2 = 0.f;
    if (VEC) {
        // one accumulator, elements in the flattened loop's order (bit-identical
        // statistics); only the loads run ahead
        const float4* x4 = reinterpret_cast<const float4*>(x);
        visit_chan4<U>(b0, b1, C, c, HW >> 2, [&](int, int64_t off) {
            const float4 v = x4[off];
            const float a = v.x - x0, q = v.y - x0, r = v.z - x0, d = v.w - x0;
            s1 += (a + q) + (r + d);
            s2 = fmaf(a, a, fmaf(q, q, fmaf(r, r, fmaf(d, d, s2))));
        });
    } else {
        const int n = (b1 - b0) * HW;
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const int bb = i / HW, o1 = i - bb * HW;
            const float a = x[((int64_t)(b0 + bb) * C + c) * HW + o1] - x0;
            s1 += a;
            s2 = fmaf(a, a, s2);
        }
    }
    const double d1 = ubpl::block_sum((double)s1, red);
    const double d2 = ubpl::block_sum((double)s2, red);
    double t1, t2;
    if (!combine_slices(part + (int64_t)c * chan_stride(gridDim.y), sp, gridDim.y, cnt + c, d1, d2, t1, t2)) return;
    const int64_t N = (int64_t)B * HW;
    const double m1 = t1 / (double)N;
    double var = t2 / (double)N - m1 * m1;
    if (var < 0) var = 0;
    const double mean = (double)x0 + m1;
    const float invstd = (float)(1.0 / sqrt(var + (double)o.eps));
    const float sc = invstd * o.gamma[c];
    o.mean_out[c] = (float)mean;
    o.invstd_out[c] = invstd;
    o.scale[c] = sc;
    o.shift[c] = o.beta[c] - (float)mean * sc;
    if (o.rmean) {
        const double unb = N > 1 ? var * (double)N / (double)(N - 1) : var;
        o.rmean[c] = (float)((double)o.momentum * mean + (1.0 - (double)o.momentum) * (double)o.rmean[c]);
        o.rvar[c] = (float)((double)o.momentum * unb + (1.0 - (double)o.momentum) * (double)o.rvar[c]);
    }
}

__global__ void eval_coeff_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                  const float* __restrict__ rmean, const float* __restrict__ rvar, float eps, int C,
                                  float* __restrict__ scale, float* __restrict__ shift) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float invstd = (float)(1.0 / sqrt((double)rvar[c] + (double)eps));
    const float sc = invstd * gamma[c];
    scale[c] = sc;
    shift[c] = beta[c] - rmean[c] * sc;
}

__global__ void __launch_bounds__(256) apply_kernel(const float* __restrict__ x, const float* __restrict__ scale,
                                                   const float* __restrict__ shift, int C, int HW, int64_t total4,
                                                   int relu, float* __restrict__ y) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int hw4 = HW >> 2;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += stride) {
        const int c = (int)((i / hw4) % C);
        const float sc = scale[c], sh = shift[c];
        float4 v = reinterpret_cast<const float4*>(x)[i];
        v.x = fmaf(v.x, sc, sh);
        v.y = fmaf(v.y, sc, sh);
        v.z = fmaf(v.z, sc, sh);
        v.w = fmaf(v.w, sc, sh);
        if (relu) {
            v.x = fmaxf(v.x, 0.f);
            v.y = fmaxf(v.y, 0.f);
            v.z = fmaxf(v.z, 0.f);
            v.w = fmaxf(v.w, 0.f);
        }
        reinterpret_cast<float4*>(y)[i] = v;
    }
}

// Finalize kernels: one 1024-thread block per channel, NPT independent slice
// loads per thread before any add (a dependent load-add chain made each
// finalize launch latency-bound, ~15 us on the training step's critical path).
constexpr int FT = 1024, NPT = 8;

struct BwdOut {
    const float* gamma;
    const float* invstd;
    float *dgamma, *dbeta, *ca, *cb, *cc;
    // BOUND: per channel a bound of |dx| (|a| max|g| + |b| max|x - mean| + |c|) into bnd[c],
    // and from the tensor's last channel the 2xfp16 scale of dx (fp16_scale_for) into *dxscale
    float* bnd;
    unsigned* tcnt;
    float* dxscale;
};

// Per (channel, slice): S1 = sum dyp, S2 = sum dyp*(x - mean) with the ReLU
// mask recomputed; the channel's last block produces dgamma/dbeta and the
// coefficients of dx = a*dyp + b*(x - mean) + c.
template <bool VEC, bool BOUND = false>
__global__ void __launch_bounds__(256) bwd_stats_kernel(const float* __restrict__ dz, const float* __restrict__ x,
                                                       int B, int C, int HW, int bper,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const float* __restrict__ mean, int relu,
                                                       double* __restrict__ part, unsigned* __restrict__ cnt,
                                                       BwdOut o) {
    __shared__ double red[16];
    __shared__ float redf[16];
    const int c = blockIdx.x, sp = blockIdx.y;
    const int b0 = sp * bper, b1 = min(B, b0 + bper);
    const float sc = scale[c], sh = shift[c], mu = mean[c];
    float s1 = 0.f, s2 = 0.f;
    float mg = 0.f, mx = 0.f;   // BOUND: max |g|, max |x - mean| of the slice
    if (VEC) {
        // (visit_chan4 here measured 7 % slower: the flattened loop stays; on the small
        // planes — <= 8 iterations per thread — all of them load first, then accumulate
        // in the same order)
        const int hw4 = HW >> 2;
        const int n4 = (b1 - b0) * hw4;
        const float4* x4 = reinterpret_cast<const float4*>(x);
        const float4* d4 = reinterpret_cast<const float4*>(dz);
        auto acc1 = [&](float4 xv, float4 g) {
            if (relu) {
                g.x = fmaf(xv.x, sc, sh) > 0.f ? g.x : 0.f;
                g.y = fmaf(xv.y, sc, sh) > 0.f ? g.y : 0.f;
                g.z = fmaf(xv.z, sc, sh) > 0.f ? g.z : 0.f;
                g.w = fmaf(xv.w, sc, sh) > 0.f ? g.w : 0.f;
            }
            s1 += (g.x + g.y) + (g.z + g.w);
            s2 = fmaf(g.x, xv.x - mu, fmaf(g.y, xv.y - mu, fmaf(g.z, xv.z - mu, fmaf(g.w, xv.w - mu, s2))));
            if (BOUND) {
                mg = fmaxf(mg, fmaxf(fmaxf(fabsf(g.x), fabsf(g.y)), fmaxf(fabsf(g.z), fabsf(g.w))));
                mx = fmaxf(mx, fmaxf(fmaxf(fabsf(xv.x - mu), fabsf(xv.y - mu)),
                                     fmaxf(fabsf(xv.z - mu), fabsf(xv.w - mu))));
            }
        };
        auto off_of = [&](int i) {
            const int bb = i / hw4, o4 = i - bb * hw4;
            return ((int64_t)(b0 + bb) * C + c) * hw4 + o4;
        };
        const int st = blockDim.x;
        if (n4 <= 8 * st) {
            float4 xv[8], g[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = threadIdx.x + u * st;
                if (i < n4) {
                    const int64_t off = off_of(i);
                    xv[u] = x4[off];
                    g[u] = d4[off];
                }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (threadIdx.x + u * st < n4) acc1(xv[u], g[u]);
        } else {
            for (int i = threadIdx.x; i < n4; i += st) {
                const int64_t off = off_of(i);
                acc1(x4[off], d4[off]);
            }
        }
    } else {
        const int n = (b1 - b0) * HW;
        for (int i = threadIdx.x; i < n; i += blockDim.x) {
            const int bb = i / HW, o1 = i - bb * HW;
            const int64_t off = ((int64_t)(b0 + bb) * C + c) * HW + o1;
            const float xv = x[off];
            float g = dz[off];
            if (relu && !(fmaf(xv, sc, sh) > 0.f)) g = 0.f;
            s1 += g;
            s2 = fmaf(g, xv - mu, s2);
            if (BOUND) {
                mg = fmaxf(mg, fabsf(g));
                mx = fmaxf(mx, fabsf(xv - mu));
            }
        }
    }
    const double d1 = ubpl::block_sum((double)s1, red);
    const double d2 = ubpl::block_sum((double)s2, red);
    double t1, t2;
    if constexpr (!BOUND) {
        if (!combine_slices(part + (int64_t)c * chan_stride(gridDim.y), sp, gridDim.y, cnt + c, d1, d2, t1, t2))
            return;
        const double N = (double)((int64_t)B * HW);
        const double is = o.invstd[c], g = o.gamma[c];
        if (o.dgamma) o.dgamma[c] += (float)(t2 * is);
        if (o.dbeta) o.dbeta[c] += (float)t1;
        o.ca[c] = (float)(g * is);
        o.cb[c] = (float)(-g * is * is * is * t2 / N);
        o.cc[c] = (float)(-g * is * t1 / N);
    } else {
        const float bmg = ubpl::block_max(mg, redf);
        const float bmx = ubpl::block_max(mx, redf);
        float ug, ux;
        if (!combine_slices4(part + (int64_t)c * chan_stride(2 * gridDim.y), sp, gridDim.y, cnt + c, d1, d2, bmg,
                             bmx, t1, t2, ug, ux))
            return;
        // wave 0 of the channel's last block (converged); lane 0 holds the totals
        const int lane = threadIdx.x;
        int tlast = 0;
        if (lane == 0) {
            const double N = (double)((int64_t)B * HW);
            const double is = o.invstd[c], g = o.gamma[c];
            if (o.dgamma) o.dgamma[c] += (float)(t2 * is);
            if (o.dbeta) o.dbeta[c] += (float)t1;
            const float a = (float)(g * is), bq = (float)(-g * is * is * is * t2 / N), cq = (float)(-g * is * t1 / N);
            o.ca[c] = a;
            o.cb[c] = bq;
            o.cc[c] = cq;
            // |dx| <= |a| max|g| + |b| max|x - mean| + |c|, 1 % over for the f32 rounding of dx
            const float bound = 1.01f * (fabsf(a) * ug + fabsf(bq) * ux + fabsf(cq));
            __hip_atomic_store(reinterpret_cast<unsigned*>(o.bnd + c), __float_as_uint(bound), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            tlast = last_arriver(o.tcnt, C) ? 1 : 0;
        }
        if (!__shfl(tlast, 0, 64)) return;
        // the tensor's last channel: max over every channel's bound -> the scale of dx
        float m = 0.f;
        for (int q = lane; q < C; q += 64)
            m = fmaxf(m, __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(o.bnd + q),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
        m = ubpl::wave_max(m);
        if (lane == 0) *o.dxscale = fp16_scale_for(m);
    }
}

// Backward statistics partials, per (channel c, 64-pixel slice q of the flat
// (b, p) range): part[(c*np + q)*2 + {0,1}] = (S1, S2) = (sum g, sum g*(x -
// mean)), the layout the conv epilogues write (common.h tile_bn_bwd_partials),
// combined by bn_bwd_finalize_kernel.  One wave per 4 x IT slices of one
// channel: lane l takes pixels 4l..4l+3 of a 256-pixel chunk (float4; P % 4 ==
// 0), a 16-lane row is one slice (DPP row sums).  (The default statistics path
// is bwd_stats_kernel above — one launch; a partials pass + finalize launch
// measured 0.7 % slower on the training step.)
template <bool VEC>
__global__ void __launch_bounds__(256) bn_bwd_partials_kernel(const float* __restrict__ dz,
                                                             const float* __restrict__ x, int C, int P, int64_t N,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ mean, int relu,
                                                             float* __restrict__ part) {
    constexpr int IT = 4;   // 256-pixel chunks (4 slices each) per wave
    const int64_t np = (N + 63) / 64, nw = (np + 4 * IT - 1) / (4 * IT);
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (w >= (int64_t)C * nw) return;
    const int lane = threadIdx.x & 63;
    const int c = (int)(w / nw);
    const int64_t u0 = (w - (int64_t)c * nw) * IT;
    const float sc = scale[c], sh = shift[c], mu = mean[c];
    float g[IT][4], xv[IT][4];
#pragma unroll
    for (int it = 0; it < IT; ++it) {   // all loads first
        const int64_t n0 = (u0 + it) * 256 + 4 * lane;
        if (VEC) {   // P % 4 == 0, 16-B aligned: the lane's 4 pixels are one float4 of one image
            const int64_t nc = n0 < N ? n0 : 0;
            const int64_t b = nc / P;
            const int64_t off = (b * C + c) * P + (nc - b * P);
            const float4 gv = *reinterpret_cast<const float4*>(dz + off);
            const float4 xq = *reinterpret_cast<const float4*>(x + off);
            g[it][0] = gv.x, g[it][1] = gv.y, g[it][2] = gv.z, g[it][3] = gv.w;
            xv[it][0] = xq.x, xv[it][1] = xq.y, xv[it][2] = xq.z, xv[it][3] = xq.w;
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t nc = n0 + e < N ? n0 + e : 0;
                const int64_t b = nc / P;
                const int64_t off = (b * C + c) * P + (nc - b * P);
                g[it][e] = dz[off];
                xv[it][e] = x[off];
            }
        }
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int64_t n0 = (u0 + it) * 256 + 4 * lane;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float ge = n0 + e < N ? g[it][e] : 0.f;
            if (relu && !(fmaf(xv[it][e], sc, sh) > 0.f)) ge = 0.f;
            s1 += ge;
            s2 = fmaf(ge, xv[it][e] - mu, s2);
        }
        s1 = ubpl::row_sum16(s1);
        s2 = ubpl::row_sum16(s2);
        const int64_t q = (u0 + it) * 4 + (lane >> 4);
        if ((lane & 15) == 15 && q < np) {
            part[((int64_t)c * np + q) * 2] = s1;
            part[((int64_t)c * np + q) * 2 + 1] = s2;
        }
    }
}

// Channel totals of the backward partials in f64 (fixed order): dgamma +=
// S2*invstd, dbeta += S1, and the coefficients of dx = a*g + b*(x - mean) + c.
__global__ void __launch_bounds__(FT) bn_bwd_finalize_kernel(const float* __restrict__ part, int64_t np, int64_t N,
                                                            BwdOut o) {
    __shared__ double red[16];
    const int c = blockIdx.x;
    const float2* pc = reinterpret_cast<const float2*>(part) + (int64_t)c * np;
    double t1 = 0.0, t2 = 0.0;
    for (int64_t q0 = 0; q0 < np; q0 += (int64_t)FT * NPT) {
        float2 v[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {   // independent loads first
            const int64_t q = q0 + threadIdx.x + (int64_t)k * FT;
            v[k] = q < np ? pc[q] : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            t1 += (double)v[k].x;
            t2 += (double)v[k].y;
        }
    }
    t1 = ubpl::block_sum(t1, red);
    t2 = ubpl::block_sum(t2, red);
    if (threadIdx.x != 0) return;
    const double is = o.invstd[c], g = o.gamma[c];
    if (o.dgamma) o.dgamma[c] += (float)(t2 * is);
    if (o.dbeta) o.dbeta[c] += (float)t1;
    o.ca[c] = (float)(g * is);
    o.cb[c] = (float)(-g * is * is * is * t2 / (double)N);
    o.cc[c] = (float)(-g * is * t1 / (double)N);
}

__device__ __forceinline__ float bwd_one(float g, float xv, float sc, float sh, float mu, float a, float b, float c,
                                         int relu) {
    if (relu && !(fmaf(xv, sc, sh) > 0.f)) g = 0.f;
    return fmaf(a, g, fmaf(b, xv - mu, c));
}

// HW % 4 == 0: float4 lanes, one channel per 4-vector.  total4 = B*C*HW/4.
__global__ void __launch_bounds__(256) bwd_apply_vec_kernel(const float* dz, const float* __restrict__ x, int C,
                                                           int HW4, int64_t total4, const float* __restrict__ scale,
                                                           const float* __restrict__ shift,
                                                           const float* __restrict__ mean, int relu,
                                                           const float* __restrict__ ca,
                                                           const float* __restrict__ cb,
                                                           const float* __restrict__ cc, const float* add1,
                                                           const float* add2, float* dx) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total4; i += stride) {
        const int c = (int)((i / HW4) % C);
        const float sc = scale[c], sh = shift[c], mu = mean[c], a = ca[c], b = cb[c], cx = cc[c];
        const float4 xv = reinterpret_cast<const float4*>(x)[i];
        const float4 g = reinterpret_cast<const float4*>(dz)[i];
        float4 v;
        v.x = bwd_one(g.x, xv.x, sc, sh, mu, a, b, cx, relu);
        v.y = bwd_one(g.y, xv.y, sc, sh, mu, a, b, cx, relu);
        v.z = bwd_one(g.z, xv.z, sc, sh, mu, a, b, cx, relu);
        v.w = bwd_one(g.w, xv.w, sc, sh, mu, a, b, cx, relu);
        if (add1) {
            const float4 q = reinterpret_cast<const float4*>(add1)[i];
            v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
        }
        if (add2) {
            const float4 q = reinterpret_cast<const float4*>(add2)[i];
            v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
        }
        reinterpret_cast<float4*>(dx)[i] = v;
    }
}

// The same per (image, channel) plane (HW4 % 256 == 0: planes of 32x32 and up): grid
// (HW4 / (256 U), B*C), so the channel and its six coefficients are block-uniform (scalar
// loads, no per-element 64-bit index division) and each thread issues its U float4s of
// every operand before computing (dx may alias dz / add1 / add2: same elements).
template <int U>
__global__ void __launch_bounds__(256) bwd_apply_plane_kernel(const float* dz, const float* __restrict__ x, int C,
                                                             int HW4, const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ mean, int relu,
                                                             const float* __restrict__ ca,
                                                             const float* __restrict__ cb,
                                                             const float* __restrict__ cc, const float* add1,
                                                             const float* add2, float* dx) {
    const int pl = blockIdx.y;
    const int c = pl % C;
    const float sc = scale[c], sh = shift[c], mu = mean[c], a = ca[c], b = cb[c], cx = cc[c];
    const int64_t base = (int64_t)pl * HW4 + blockIdx.x * (256 * U) + threadIdx.x;
    const float4* x4 = reinterpret_cast<const float4*>(x) + base;
    const float4* d4 = reinterpret_cast<const float4*>(dz) + base;
    float4 xv[U], g[U], q1[U], q2[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        xv[u] = x4[u * 256];
        g[u] = d4[u * 256];
        if (add1) q1[u] = reinterpret_cast<const float4*>(add1)[base + u * 256];
        if (add2) q2[u] = reinterpret_cast<const float4*>(add2)[base + u * 256];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        float4 v;
        v.x = bwd_one(g[u].x, xv[u].x, sc, sh, mu, a, b, cx, relu);
        v.y = bwd_one(g[u].y, xv[u].y, sc, sh, mu, a, b, cx, relu);
        v.z = bwd_one(g[u].z, xv[u].z, sc, sh, mu, a, b, cx, relu);
        v.w = bwd_one(g[u].w, xv[u].w, sc, sh, mu, a, b, cx, relu);
        if (add1) { v.x += q1[u].x; v.y += q1[u].y; v.z += q1[u].z; v.w += q1[u].w; }
        if (add2) { v.x += q2[u].x; v.y += q2[u].y; v.z += q2[u].z; v.w += q2[u].w; }
        reinterpret_cast<float4*>(dx)[base + u * 256] = v;
    }
}

__global__ void __launch_bounds__(256) bwd_apply_kernel(const float* dz, const float* __restrict__ x, int C, int HW,
                                                       int64_t total, const float* __restrict__ scale,
                                                       const float* __restrict__ shift,
                                                       const float* __restrict__ mean, int relu,
                                                       const float* __restrict__ ca, const float* __restrict__ cb,
                                                       const float* __restrict__ cc, const float* add1,
                                                       const float* add2, float* dx) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
        const int c = (int)((i / HW) % C);
        float v = bwd_one(dz[i], x[i], scale[c], shift[c], mean[c], ca[c], cb[c], cc[c], relu);
        if (add1) v += add1[i];
        if (add2) v += add2[i];
        dx[i] = v;
    }
}

int splits_for(int B, int C) {
    int s = (2048 + C - 1) / C;
    if (s > B) s = B;
    if (s < 1) s = 1;
    return s;
}

// The batch slices a statistics launch actually uses: splits_for's bound, and
// at least ~8k elements per (channel, slice) block — small planes get one
// block per channel (at 4x4 / B=32, 2048 blocks of 32 elements each were pure
// launch and ticket overhead).
int bn_env(const char* name, int dflt) {
    const char* e = getenv(name);
    return e != nullptr ? atoi(e) : dflt;
}

int splits_for(int B, int C, int HW) {
    int s = splits_for(B, C);
    // (tuning hook: UBPL_BN_MINSLICE elements per (channel, slice) block, default 8192)
    static const int64_t minslice = bn_env("UBPL_BN_MINSLICE", 8192) > 0 ? bn_env("UBPL_BN_MINSLICE", 8192) : 8192;
    const int64_t per_slice = (int64_t)B * HW / minslice;
    if (s > per_slice) s = per_slice > 1 ? (int)per_slice : 1;
    return s;
}

int grid_ew(int64_t n) {
    int64_t g = (n + 255) / 256;
    if (g > 4096) g = 4096;
    if (g < 1) g = 1;
    return (int)g;
}

}  // namespace

// Scratch: part must hold ubpl_bn_part_doubles(B, C) doubles, ZEROED before
// first use: MAXBN arrival counters at its head (a fixed place, whatever C a
// call has; every call leaves them at zero again), then per channel the
// 2 * splits partial sums, channels chan_stride(splits) doubles apart.
constexpr int MAXBN = 512;
constexpr int CNT_DOUBLES = MAXBN / 2;
constexpr int MAX_SPLITS = 2048 / 64 + 1;   // splits_for's bound for C >= 64 (and B)
// ---- statistics from 64-pixel partials (conv-epilogue fused: common.h
// tile_bn_partials; or bn_partials_kernel below).  part [C][np][2] f32 =
// (S, M2) per slice, Chan's parallel form.
// One wave per (channel, 64-pixel slice): lane = pixel (coalesced along p),
// S and M2 by wave reductions.  4 waves per block.
__global__ void __launch_bounds__(256) bn_partials_kernel(const float* __restrict__ y, int C, int P, int64_t N,
                                                         float* __restrict__ part) {
    const int64_t np = (N + 63) / 64;
    const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);   // (c, q)
    if (w >= (int64_t)C * np) return;
    const int lane = threadIdx.x & 63;
    const int c = (int)(w / np);
    const int64_t q = w - (int64_t)c * np;
    const int64_t n = q * 64 + lane;
    const bool ok = n < N;
    const int64_t nc = ok ? n : N - 1;
    const int64_t b = nc / P;
    const float v = y[(b * C + c) * P + (nc - b * P)];
    const float cnt = (float)(N - q * 64 < 64 ? N - q * 64 : 64);
    const float s = ubpl::wave_sum(ok ? v : 0.f);
    const float d = ok ? v - s / cnt : 0.f;
    const float m2 = ubpl::wave_sum(d * d);
    if (lane == 0) {
        part[w * 2] = s;
        part[w * 2 + 1] = m2;
    }
}

// mean = sum S / N; M2 = sum M2_q + sum n_q (S_q/n_q - mean)^2, in f64.
__global__ void __launch_bounds__(FT) bn_finalize_partials_kernel(const float* __restrict__ part, int64_t np,
                                                                 int64_t N, StatsOut o) {
    __shared__ double red[16];
    const int c = blockIdx.x;
    const float2* pc = reinterpret_cast<const float2*>(part) + (int64_t)c * np;
    auto nq_of = [&](int64_t q) { return (double)(N - q * 64 < 64 ? N - q * 64 : 64); };
    double t1 = 0.0;
    float2 v[NPT];   // the first FT*NPT slices stay in registers for the second pass
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int64_t q = threadIdx.x + (int64_t)k * FT;
        v[k] = q < np ? pc[q] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int k = 0; k < NPT; ++k) t1 += (double)v[k].x;
    for (int64_t q0 = (int64_t)FT * NPT; q0 < np; q0 += (int64_t)FT * NPT) {
        float w[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const int64_t q = q0 + threadIdx.x + (int64_t)k * FT;
            w[k] = q < np ? pc[q].x : 0.f;
        }
#pragma unroll
        for (int k = 0; k < NPT; ++k) t1 += (double)w[k];
    }
    t1 = ubpl::block_sum(t1, red);
    const double mean = t1 / (double)N;
    double t2 = 0.0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int64_t q = threadIdx.x + (int64_t)k * FT;
        if (q < np) {
            const double nq = nq_of(q);
            const double dm = (double)v[k].x / nq - mean;
            t2 += (double)v[k].y + nq * dm * dm;
        }
    }
    for (int64_t q0 = (int64_t)FT * NPT; q0 < np; q0 += (int64_t)FT * NPT) {
        float2 w[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const int64_t q = q0 + threadIdx.x + (int64_t)k * FT;
            w[k] = q < np ? pc[q] : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const int64_t q = q0 + threadIdx.x + (int64_t)k * FT;
            if (q < np) {
                const double nq = nq_of(q);
                const double dm = (double)w[k].x / nq - mean;
                t2 += (double)w[k].y + nq * dm * dm;
            }
        }
    }
    t2 = ubpl::block_sum(t2, red);
    if (threadIdx.x != 0) return;
    const double var = t2 / (double)N;
    const float invstd = (float)(1.0 / sqrt(var + (double)o.eps));
    const float sc = invstd * o.gamma[c];
    o.mean_out[c] = (float)mean;
    o.invstd_out[c] = invstd;
    o.scale[c] = sc;
    o.shift[c] = o.beta[c] - (float)mean * sc;
    if (o.rmean) {
        const double unb = N > 1 ? var * (double)N / (double)(N - 1) : var;
        o.rmean[c] = (float)((double)o.momentum * mean + (1.0 - (double)o.momentum) * (double)o.rmean[c]);
        o.rvar[c] = (float)((double)o.momentum * unb + (1.0 - (double)o.momentum) * (double)o.rvar[c]);
    }
}

UBPL_API int ubpl_bn_splits(int B, int C) { return splits_for(B, C); }

// Floats of a partial-statistics buffer for C channels over N = B*P pixels.
UBPL_API int64_t ubpl_bn_partial_floats(int C, int64_t N) { return 2 * (int64_t)C * ((N + 63) / 64); }

// part [C][ceil(N/64)][2] = per 64-pixel slice (S, M2) of y [B,C,P]: the layout
// conv epilogues produce themselves.
UBPL_API int ubpl_bn_partials(const float* y, int B, int C, int P, float* part, void* stream) {
    const int64_t N = (int64_t)B * P;
    const int64_t n = (int64_t)C * ((N + 63) / 64);
    hipLaunchKernelGGL(bn_partials_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, y, C,
                       P, N, part);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// Train-mode BatchNorm statistics from partials (outputs as ubpl_bn_forward_stats).
UBPL_API int ubpl_bn_stats_from_partials(const float* part, int C, int64_t N, const float* gamma,
                                         const float* beta, float eps, float momentum, float* rmean, float* rvar,
                                         float* mean_out, float* invstd_out, float* scale, float* shift_out,
                                         void* stream) {
    StatsOut o{gamma, beta, eps, momentum, rmean, rvar, mean_out, invstd_out, scale, shift_out};
    hipLaunchKernelGGL(bn_finalize_partials_kernel, dim3(C), dim3(FT), 0, (hipStream_t)stream, part,
                       (N + 63) / 64, N, o);
    UBPL_LAUNCH_CHECK();
    return 0;
}
// (+ the bounded backward statistics' area: 4 doubles per slice of up to MAXBN channels, then a
// tensor ticket and MAXBN per-channel bounds; the tickets return to zero after every launch)
UBPL_API int64_t ubpl_bn_part_doubles(int B, int C) {
    (void)B;
    (void)C;
    return CNT_DOUBLES + (int64_t)MAXBN * chan_stride(2 * MAX_SPLITS) + 32 + MAXBN / 2;
}

// Train-mode statistics of x [B,C,H,W] -> mean, invstd, (scale, shift) and the
// running-stat update (rmean/rvar nullable: track_running_stats off).
UBPL_API int ubpl_bn_forward_stats(const float* x, int B, int C, int HW, const float* gamma, const float* beta,
                                   float eps, float momentum, float* rmean, float* rvar, double* part,
                                   float* mean_out, float* invstd_out, float* scale, float* shift, void* stream) {
    const int splits = splits_for(B, C, HW);
    const int bper = (B + splits - 1) / splits;
    const int gs = (B + bper - 1) / bper;
    if (C > MAXBN) return (int)hipErrorInvalidValue;
    unsigned* cnt = reinterpret_cast<unsigned*>(part);
    part += CNT_DOUBLES;
    const StatsOut o{gamma, beta, eps, momentum, rmean, rvar, mean_out, invstd_out, scale, shift};
    const bool vec = (HW % 4 == 0) && (((uintptr_t)x & 15) == 0);
    // (tuning hook: UBPL_BN_U=8: eight float4 loads in flight per thread instead of four)
    static const bool u8 = bn_env("UBPL_BN_U", 4) == 8;
    if (vec && u8)
        hipLaunchKernelGGL((stats_kernel<true, 8>), dim3(C, gs), dim3(256), 0, (hipStream_t)stream, x, B, C, HW, bper,
                           part, cnt, o);
    else if (vec)
        hipLaunchKernelGGL(stats_kernel<true>, dim3(C, gs), dim3(256), 0, (hipStream_t)stream, x, B, C, HW, bper, part,
                           cnt, o);
    else
        hipLaunchKernelGGL(stats_kernel<false>, dim3(C, gs), dim3(256), 0, (hipStream_t)stream, x, B, C, HW, bper,
                           part, cnt, o);
    UBPL_LAUNCH_CHECK();
    return 0;
}

UBPL_API int ubpl_bn_eval_coeffs(const float* gamma, const float* beta, const float* rmean, const float* rvar,
                                 float eps, int C, float* scale, float* shift, void* stream) {
    hipLaunchKernelGGL(eval_coeff_kernel, dim3(ubpl::cdiv(C, 64)), dim3(64), 0, (hipStream_t)stream, gamma, beta,
                       rmean, rvar, eps, C, scale, shift);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// y = [relu](x*scale + shift); HW must be a multiple of 4, x/y 16-B aligned.
UBPL_API int ubpl_bn_apply(const float* x, int B, int C, int HW, const float* scale, const float* shift, int relu,
                           float* y, void* stream) {
    if ((HW & 3) || (((uintptr_t)x | (uintptr_t)y) & 15)) return (int)hipErrorInvalidValue;
    const int64_t total4 = (int64_t)B * C * HW / 4;
    hipLaunchKernelGGL(apply_kernel, dim3(grid_ew(total4)), dim3(256), 0, (hipStream_t)stream, x, scale, shift, C, HW,
                       total4, relu, y);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// Backward of y = [relu](bn(x)) given dz = dL/dy.  dgamma/dbeta are
// ACCUMULATED (+=).  dx = add1 + add2 + dL/dx (add1/add2 nullable; dx may
// alias dz, add1 or add2).  coef: scratch of 3*C floats.
// dx of the BN backward written straight into the PSA layout (conv_split.hip
// split_act_kernel's [B][C/16][H+2pad][W+2pad][16] bf16 planes, zero border):
// one thread per padded pixel of one 16-channel group, like split_act.
template <int NP>
__global__ void __launch_bounds__(256) bwd_apply_split_kernel(const float* __restrict__ dz,
                                                             const float* __restrict__ x, int C, int H, int W,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift,
                                                             const float* __restrict__ mean, int relu,
                                                             const float* __restrict__ ca,
                                                             const float* __restrict__ cb,
                                                             const float* __restrict__ cc, int pad,
                                                             uint16_t* __restrict__ dst, int64_t plane,
                                                             const float* __restrict__ dxscale) {
    // NP = 2 (2xfp16): the pieces of dx * (*dxscale), the power of two the statistics chose
    const int Hp = H + 2 * pad, Wp = W + 2 * pad, G = C >> 4;
    const int b = blockIdx.z, g = blockIdx.y;
    const int pix = blockIdx.x * 256 + threadIdx.x;
    if (pix >= Hp * Wp) return;
    const int hp = pix / Wp, wq = pix - hp * Wp;
    const int h = hp - pad, w = wq - pad;
    const bool in = h >= 0 && h < H && w >= 0 && w < W;
    const int64_t HW = (int64_t)H * W;
    const int64_t o = ((int64_t)b * C + 16 * g) * HW + (in ? h * W + w : 0);
    float v[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int c = 16 * g + j;
        const float r = bwd_one(dz[o + j * HW], x[o + j * HW], scale[c], shift[c], mean[c], ca[c], cb[c], cc[c], relu);
        v[j] = in ? r : 0.f;
    }
    ubpl::store_psa_row<NP>(v, dst + (((int64_t)(b * G + g) * Hp + hp) * Wp + wq) * 16, plane,
                            NP == 2 ? *dxscale : 1.f);
}

namespace {
// statistics -> coefficients: one bwd_stats_kernel launch, or (part != nullptr:
// the producer's epilogue wrote the partials) the f64 finalize
int bwd_stats(const float* dz, const float* x, int B, int C, int HW, const float* gamma, const float* mean,
              const float* invstd, const float* scale, const float* shift, int relu, double* scratch,
              const float* part, float* coef, float* dgamma, float* dbeta, hipStream_t st, bool bound = false) {
    // bound: also the 2xfp16 scale of dx at coef[3C] (bwd_stats_kernel BOUND; coef: 3C + 1 floats, the
    // per-channel bounds and the tensor ticket in the scratch's tail)
    unsigned* cnt = reinterpret_cast<unsigned*>(scratch);
    BwdOut o{gamma, invstd, dgamma, dbeta, coef, coef + C, coef + 2 * C, nullptr, nullptr, nullptr};
    if (bound) {
        if (part != nullptr || C > MAXBN || scratch == nullptr) return (int)hipErrorInvalidValue;
        const int splits = splits_for(B, C, HW);
        const int bper = (B + splits - 1) / splits;
        const int gs = (B + bper - 1) / bper;
        double* sl = scratch + CNT_DOUBLES;
        double* tail = sl + (int64_t)MAXBN * chan_stride(2 * MAX_SPLITS);
        o.tcnt = reinterpret_cast<unsigned*>(tail);
        o.bnd = reinterpret_cast<float*>(tail + 32);
        o.dxscale = coef + 3 * C;
        const bool vec = (HW % 4 == 0) && ((((uintptr_t)dz | (uintptr_t)x) & 15) == 0);
        if (vec)
            hipLaunchKernelGGL((bwd_stats_kernel<true, true>), dim3(C, gs), dim3(256), 0, st, dz, x, B, C, HW, bper,
                               scale, shift, mean, relu, sl, cnt, o);
        else
            hipLaunchKernelGGL((bwd_stats_kernel<false, true>), dim3(C, gs), dim3(256), 0, st, dz, x, B, C, HW, bper,
                               scale, shift, mean, relu, sl, cnt, o);
        UBPL_LAUNCH_CHECK();
        return 0;
    }
    if (part == nullptr) {   // one launch: slices + last-arriver combine
        if (C > MAXBN || scratch == nullptr) return (int)hipErrorInvalidValue;
        const int splits = splits_for(B, C, HW);
        const int bper = (B + splits - 1) / splits;
        const int gs = (B + bper - 1) / bper;
        const bool vec = (HW % 4 == 0) && ((((uintptr_t)dz | (uintptr_t)x) & 15) == 0);
        double* sl = scratch + CNT_DOUBLES;
        if (vec)
            hipLaunchKernelGGL(bwd_stats_kernel<true>, dim3(C, gs), dim3(256), 0, st, dz, x, B, C, HW, bper, scale,
                               shift, mean, relu, sl, cnt, o);
        else
            hipLaunchKernelGGL(bwd_stats_kernel<false>, dim3(C, gs), dim3(256), 0, st, dz, x, B, C, HW, bper, scale,
                               shift, mean, relu, sl, cnt, o);
        UBPL_LAUNCH_CHECK();
        return 0;
    }
    const int64_t N = (int64_t)B * HW;
    const int64_t np = (N + 63) / 64;
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(FT), 0, st, part, np, N, o);
    UBPL_LAUNCH_CHECK();
    return 0;
}
}  // namespace

// Backward statistics partials of dz (ReLU mask from x's BN) alone: the layout
// ubpl_bn_backward's `part` takes; part: ubpl_bn_partial_floats(C, B*HW) floats.
UBPL_API int ubpl_bn_backward_partials(const float* dz, const float* x, int B, int C, int HW, const float* scale,
                                       const float* shift, const float* mean, int relu, float* part, void* stream) {
    const int64_t N = (int64_t)B * HW;
    const int64_t np = (N + 63) / 64;
    const bool vec = (HW % 4 == 0) && ((((uintptr_t)dz | (uintptr_t)x) & 15) == 0);
    const int64_t waves = (int64_t)C * ((np + 15) / 16);
    const dim3 grid((unsigned)((waves + 3) / 4));
    if (vec)
        hipLaunchKernelGGL(bn_bwd_partials_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, dz, x, C, HW, N,
                           scale, shift, mean, relu, part);
    else
        hipLaunchKernelGGL(bn_bwd_partials_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, dz, x, C, HW, N,
                           scale, shift, mean, relu, part);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// ubpl_bn_backward with dx delivered as PSA planes only (no f32 dx, no
// addends): statistics, then bwd_apply_split_kernel.  C % 16 == 0.
UBPL_API int ubpl_bn_backward_split(const float* dz, const float* x, int B, int C, int H, int W, const float* gamma,
                                    const float* mean, const float* invstd, const float* scale, const float* shift,
                                    int relu, double* scratch, const float* part, float* coef, float* dgamma,
                                    float* dbeta, int pad, int npieces, uint16_t* dst, int64_t plane, void* stream) {
    const int HW = H * W;
    if (C % 16 != 0 || npieces < 1 || npieces > 3 || pad < 0) return (int)hipErrorInvalidValue;
    hipStream_t st = (hipStream_t)stream;
    // npieces 2 (2xfp16): dx scaled by the power of two its bound asks for (coef[3C]: coef holds 3C + 1 floats)
    const int e = bwd_stats(dz, x, B, C, HW, gamma, mean, invstd, scale, shift, relu, scratch, part, coef, dgamma,
                            dbeta, st, npieces == 2);
    if (e) return e;
    const float* dxs = coef + 3 * C;
    const float *ca = coef, *cb = coef + C, *cc = coef + 2 * C;
    const int Hp = H + 2 * pad, Wp = W + 2 * pad;
    dim3 grid((unsigned)((Hp * Wp + 255) / 256), (unsigned)(C / 16), (unsigned)B);
    if (npieces == 3)
        hipLaunchKernelGGL(bwd_apply_split_kernel<3>, grid, dim3(256), 0, st, dz, x, C, H, W, scale, shift, mean,
                           relu, ca, cb, cc, pad, dst, plane, dxs);
    else if (npieces == 1)
        hipLaunchKernelGGL(bwd_apply_split_kernel<1>, grid, dim3(256), 0, st, dz, x, C, H, W, scale, shift, mean,
                           relu, ca, cb, cc, pad, dst, plane, dxs);
    else
        hipLaunchKernelGGL(bwd_apply_split_kernel<2>, grid, dim3(256), 0, st, dz, x, C, H, W, scale, shift, mean,
                           relu, ca, cb, cc, pad, dst, plane, dxs);
    UBPL_LAUNCH_CHECK();
    return 0;
}

// dx = BatchNorm(+ReLU) backward of dz (+ add1 + add2), dgamma/dbeta (+)= ;
// statistics by one bwd_stats_kernel launch over `scratch` (ubpl_bn_part_doubles,
// zeroed before first use), or — part != nullptr — from the backward partials
// dz's producer wrote (then only the f64 finalize runs); coef: 3*C floats.
UBPL_API int ubpl_bn_backward(const float* dz, const float* x, int B, int C, int HW, const float* gamma,
                              const float* mean, const float* invstd, const float* scale, const float* shift,
                              int relu, double* scratch, const float* part, float* coef, float* dgamma,
                              float* dbeta, const float* add1, const float* add2, float* dx, void* stream) {
    hipStream_t st = (hipStream_t)stream;
    const int e = bwd_stats(dz, x, B, C, HW, gamma, mean, invstd, scale, shift, relu, scratch, part, coef, dgamma,
                            dbeta, st);
    if (e) return e;
    const uintptr_t al = (uintptr_t)dz | (uintptr_t)x | (uintptr_t)dx | (uintptr_t)add1 | (uintptr_t)add2;
    const bool vec = (HW % 4 == 0) && ((al & 15) == 0);
    const float *ca = coef, *cb = coef + C, *cc = coef + 2 * C;
    const int64_t total = (int64_t)B * C * HW;
    // (UBPL_BN_PLANE=0: the round-4 grid-stride kernel everywhere)
    static const bool plane_env = [] {
        const char* e = getenv("UBPL_BN_PLANE");
        return !(e && atoi(e) == 0);
    }();
    const int hw4 = HW / 4;
    if (vec && plane_env && hw4 % 256 == 0 && (int64_t)B * C < 65536) {
        const int u = hw4 % 1024 == 0 ? 4 : (hw4 % 512 == 0 ? 2 : 1);
        const dim3 grid((unsigned)(hw4 / (256 * u)), (unsigned)(B * C));
        if (u == 4)
            hipLaunchKernelGGL(bwd_apply_plane_kernel<4>, grid, dim3(256), 0, st, dz, x, C, hw4, scale, shift, mean,
                               relu, ca, cb, cc, add1, add2, dx);
        else if (u == 2)
            hipLaunchKernelGGL(bwd_apply_plane_kernel<2>, grid, dim3(256), 0, st, dz, x, C, hw4, scale, shift, mean,
                               relu, ca, cb, cc, add1, add2, dx);
        else
            hipLaunchKernelGGL(bwd_apply_plane_kernel<1>, grid, dim3(256), 0, st, dz, x, C, hw4, scale, shift, mean,
                               relu, ca, cb, cc, add1, add2, dx);
    } else if (vec)
        hipLaunchKernelGGL(bwd_apply_vec_kernel, dim3(grid_ew(total / 4)), dim3(256), 0, st, dz, x, C, HW / 4,
                           total / 4, scale, shift, mean, relu, ca, cb, cc, add1, add2, dx);
    else
        hipLaunchKernelGGL(bwd_apply_kernel, dim3(grid_ew(total)), dim3(256), 0, st, dz, x, C, HW, total, scale,
                           shift, mean, relu, ca, cb, cc, add1, add2, dx);
    UBPL_LAUNCH_CHECK();
    return 0;
}
