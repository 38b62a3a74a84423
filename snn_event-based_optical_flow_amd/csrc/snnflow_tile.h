// Shared tile machinery of the conv-layer kernels (LIFFireNet cells, ConvLIF cells):
// halo staging, 3x3 conv / transposed conv of one pixel from LDS, block reductions into
// sharded fp64 accumulators.  Device code only; included by the .hip translation units.
#pragma once

#include <type_traits>

#include "snnflow_dev.h"

#ifndef SNNFLOW_PIN_PF
#define SNNFLOW_PIN_PF 1  // C = 16 / 32 conv MFMA loops: pin the fragment prefetch one k-step ahead (sched_barrier)
#endif

namespace snnflow {

// ---------------------------------------------------------------------------
// LDS staging of a halo tile
// ---------------------------------------------------------------------------

// Strided input (e.g. event_cnt NCHW, or an NHWC spike tensor) -> tile[p][ci]
template <int CIN, int NTH = NT>
__device__ void stage_strided(const float* __restrict__ x, int64_t sb, int64_t sc, int64_t sh, int64_t sw,
                              const Tile& tl, int H, int W, float* tile) {
    constexpr int P = Pad<CIN>::v;
    const int tid = threadIdx.x;
    const float* xb = x + (int64_t)tl.b * sb;
    if (sc == 1) {
        for (int e = tid; e < HN * CIN; e += NTH) {
            const int p = e / CIN, ci = e - p * CIN;
            const int r = p / HWD, cc = p - r * HWD;
            const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
            tile[p * P + ci] = in_image(h, w, H, W) ? xb[h * sh + w * sw + ci] : 0.0f;
        }
    } else {
        for (int e = tid; e < HN * CIN; e += NTH) {
            const int ci = e / HN, p = e - ci * HN;
            const int r = p / HWD, cc = p - r * HWD;
            const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
            tile[p * P + ci] = in_image(h, w, H, W) ? xb[ci * sc + h * sh + w * sw] : 0.0f;
        }
    }
}

// Contiguous NHWC [B][H][W][C] (C % 4 == 0) -> tile
template <int C, int NTH = NT>
__device__ void stage_nhwc(const float* __restrict__ x, const Tile& tl, int H, int W, float* tile) {
    static_assert(C % 4 == 0, "vector staging");
    constexpr int P = Pad<C>::v, Q = C / 4;
    const int tid = threadIdx.x;
    for (int e = tid; e < HN * Q; e += NTH) {
        const int p = e / Q, q = e - p * Q;
        const int r = p / HWD, cc = p - r * HWD;
        const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (in_image(h, w, H, W))
            v = *reinterpret_cast<const float4*>(x + (((int64_t)tl.b * H + h) * W + w) * C + 4 * q);
        *reinterpret_cast<float4*>(tile + p * P + 4 * q) = v;
    }
}

// The same from a spike bit plane (ABI 39): exact 0/1 floats
template <int C, int NTH = NT>
__device__ void stage_nhwc_bits(const uint8_t* __restrict__ bits, const Tile& tl, int H, int W, float* tile) {
    constexpr int P = Pad<C>::v, Q = C / 4;
    for (int e = threadIdx.x; e < HN * Q; e += NTH) {
        const int p = e / Q, q = e - p * Q;
        const int r = p / HWD, cc = p - r * HWD;
        const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
        const unsigned wb = in_image(h, w, H, W) ? spk_load_bits<C>(bits, ((int64_t)tl.b * H + h) * W + w) : 0u;
        *reinterpret_cast<float4*>(tile + p * P + 4 * q) = spk_quad<C>(wb, q);
    }
}

// ---------------------------------------------------------------------------
// 3x3 convolution of one output pixel (outputs [co0, co0+CO)) from an LDS halo tile.
// wt: [3][3][CIN][C]; co0 must be wave-uniform (scalar weight loads).
// acc += sum_{ky,kx,ci} w * x.
// ---------------------------------------------------------------------------
template <int CIN, int C, int CO = C>
__device__ inline void conv_acc(const float* tile, const float* __restrict__ wt, int ty, int tx, int co0,
                                float (&acc)[CO]) {
    constexpr int P = Pad<CIN>::v, VW = VecW<CIN>::v;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const float* xp = tile + ((ty + ky) * HWD + (tx + kx)) * P;
            const cfloat_ptr wk = as_const(wt) + (ky * 3 + kx) * CIN * C + co0;
            constexpr int UR = CIN <= 8 ? CIN : 1;
#pragma unroll UR
            for (int ci = 0; ci < CIN; ci += VW) {
                float xs[VW];
                if constexpr (VW == 4) {
                    const float4 v = *reinterpret_cast<const float4*>(xp + ci);
                    xs[0] = v.x; xs[1] = v.y; xs[2] = v.z; xs[3] = v.w;
                } else if constexpr (VW == 2) {
                    const float2 v = *reinterpret_cast<const float2*>(xp + ci);
                    xs[0] = v.x; xs[1] = v.y;
                } else {
                    xs[0] = xp[ci];
                }
#pragma unroll
                for (int j = 0; j < VW; ++j) {
#pragma unroll
                    for (int co = 0; co < CO; ++co) acc[co] = fmaf(wk[(ci + j) * C + co], xs[j], acc[co]);
                }
            }
        }
    }
}

// Transposed 3x3 (input gradient, inputs [ci0, ci0+CI)) of one pixel from an LDS tile of
// output gradients.  wd: [3][3][C][CIN]; ci0 wave-uniform.
// gx[ci] += sum_{ky,kx,co} w[co][ci][ky][kx] * g[h+1-ky][w+1-kx][co]
template <int C, int CIN, int CI = CIN>
__device__ inline void dgrad_acc(const float* gtile, const float* __restrict__ wd, int ty, int tx, int ci0,
                                 float (&gx)[CI]) {
    constexpr int P = Pad<C>::v;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const float* gp = gtile + ((ty + 2 - ky) * HWD + (tx + 2 - kx)) * P;
            const cfloat_ptr wk = as_const(wd) + (ky * 3 + kx) * C * CIN + ci0;
            constexpr int UR = C <= 8 ? C : 1;
#pragma unroll UR
            for (int co = 0; co < C; co += 4) {
                const float4 v = *reinterpret_cast<const float4*>(gp + co);
                const float gs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
#pragma unroll
                    for (int ci = 0; ci < CI; ++ci) gx[ci] = fmaf(wk[(co + j) * CIN + ci], gs[j], gx[ci]);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Implicit-GEMM 3x3 convolution of a block's NT output pixels on the matrix cores
// (v_mfma_f32_16x16x4_f32: f32 operands, f32 accumulation, bit-for-bit a k-ordered fmaf
// chain -- the same arithmetic as the vector path, in a different summation order).
//
//   out[p][n] = sum_{tap, k} src[halo(p, tap)][k] * wB[tap][n][k]
//
// M = pixels: 16 M-tiles of 16 consecutive pixels of one tile row (TW = 32), split over
// the block's NW waves.  N = output channels in 16-wide tiles (NOUT = 8 pads with zero
// weights).  K = 9 taps x KIN channels; in the MFMA of step j of a 16-channel block, lane
// group g = lane >> 4 supplies channel 16 kb + E g + j for both operands (a permutation of
// k, so each lane reads E consecutive channels with one LDS / global vector load).
// src: LDS halo tile [HN][Pad<KIN>]; wB: global, [9][NOUT][KIN] (k fastest).
// FLIP = false: halo(p, tap) = p + (ky, kx) (forward conv); true: p + (2 - ky, 2 - kx)
// (input gradient of the conv: wB then holds the forward weights in [tap][cin][c] order).
// ---------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int KIN, int NOUT>
struct MfmaGeo {
    static_assert(KIN % 4 == 0 && (KIN < 16 || KIN % 16 == 0), "MFMA conv: KIN in {4, 8, 16, 32, ...}");
    static constexpr int E = KIN >= 16 ? 4 : KIN / 4;    // channels per lane per 16-channel block
    static constexpr int NKB = KIN >= 16 ? KIN / 16 : 1;  // 16-channel blocks of K per tap
    static constexpr int NNT = (NOUT + 15) / 16;          // 16-wide output-channel tiles
    static constexpr int BPT = NNT * NKB * E;             // B operand floats per lane per tap
};

template <int E>
__device__ inline void ld_vec(const float* p, float* v) {
    if constexpr (E == 4) {
        const float4 t = *reinterpret_cast<const float4*>(p);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else if constexpr (E == 2) {
        const float2 t = *reinterpret_cast<const float2*>(p);
        v[0] = t.x; v[1] = t.y;
    } else {
        v[0] = p[0];
    }
}

// B fragments of one tap for n-tiles [ntb, ntb + WNT) (zeros for padded channels n >= NOUT).
template <int KIN, int NOUT, int WNT = MfmaGeo<KIN, NOUT>::NNT>
__device__ inline void mfma_load_b(const float* __restrict__ wB, int tap, int ntb,
                                   float (&b)[WNT * MfmaGeo<KIN, NOUT>::NKB * MfmaGeo<KIN, NOUT>::E]) {
    using G = MfmaGeo<KIN, NOUT>;
    const int lane = threadIdx.x & 63, m = lane & 15, g = lane >> 4;
#pragma unroll
    for (int nt = 0; nt < WNT; ++nt) {
        const int n = (ntb + nt) * 16 + m;
        const bool ok = n < NOUT;
        const float* p = wB + (int64_t)(tap * NOUT + (ok ? n : 0)) * KIN + g * G::E;
#pragma unroll
        for (int kb = 0; kb < G::NKB; ++kb) {
            float v[G::E];
            ld_vec<G::E>(p + kb * 16, v);
#pragma unroll
            for (int j = 0; j < G::E; ++j) b[(nt * G::NKB + kb) * G::E + j] = ok ? v[j] : 0.0f;
        }
    }
}

// Accumulators of one wave.  The 16 M-tiles x NNT N-tiles of a block are split over its NW
// waves in NG n-groups: wave wv owns M-tiles [mt0, mt0 + MT) and N-tiles [nt0, nt0 + WNT).
// NG = 1: every wave all N-tiles (fewest A reads); NG = 2 at C = 32: half the B operand per
// wave (the weight fragments every wave streams from L2 halve).
template <int KIN, int NOUT, int NW, int NG = 1>
struct MfmaAcc {
    static constexpr int NNT = MfmaGeo<KIN, NOUT>::NNT;
    static_assert(NNT % NG == 0 && NW % NG == 0 && (16 * NG) % NW == 0, "wave tiling");
    static constexpr int MT = 16 * NG / NW;  // M-tiles per wave
    static constexpr int WNT = NNT / NG;     // N-tiles per wave
    f32x4 v[MT][WNT];
    __device__ static inline int mt0(int wv) { return (wv / NG) * MT; }
    __device__ static inline int nt0(int wv) { return (wv % NG) * WNT; }
    __device__ inline void zero() {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < WNT; ++j) v[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
};

template <int KIN, int NOUT, bool FLIP, int NW, int NG = 1>
__device__ void mfma_conv3x3(const float* src, const float* __restrict__ wB, MfmaAcc<KIN, NOUT, NW, NG>& acc) {
    using G = MfmaGeo<KIN, NOUT>;
    using A = MfmaAcc<KIN, NOUT, NW, NG>;
    static_assert(NT == 256 && TW == 32 && 16 % NW == 0, "MFMA conv: 8x32 tiles, NW | 16");
    constexpr int P = Pad<KIN>::v, MT = A::MT, WNT = A::WNT, BPW = WNT * G::NKB * G::E;
    const int lane = threadIdx.x & 63, m = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int mtb = A::mt0(wv), ntb = A::nt0(wv);
    float bc[BPW], bn[BPW];
    mfma_load_b<KIN, NOUT, WNT>(wB, 0, ntb, bc);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
        if (tap + 1 < 9) mfma_load_b<KIN, NOUT, WNT>(wB, tap + 1, ntb, bn);  // next tap's weights in flight
        const int ky = tap / 3, kx = tap - 3 * (tap / 3);
        const int oy = FLIP ? 2 - ky : ky, ox = FLIP ? 2 - kx : kx;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int T = mtb + mt, row = T >> 1, c0 = (T & 1) * 16;
            const float* ap = src + ((row + oy) * HWD + c0 + m + ox) * P + g * G::E;
#pragma unroll
            for (int kb = 0; kb < G::NKB; ++kb) {
                float a[G::E];
                ld_vec<G::E>(ap + kb * 16, a);
#pragma unroll
                for (int j = 0; j < G::E; ++j)
#pragma unroll
                    for (int nt = 0; nt < WNT; ++nt)
                        acc.v[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[j], bc[(nt * G::NKB + kb) * G::E + j],
                                                                             acc.v[mt][nt], 0, 0, 0);
            }
        }
        if (tap + 1 < 9) {
#pragma unroll
            for (int i = 0; i < BPW; ++i) bc[i] = bn[i];
        }
    }
}

// ---------------------------------------------------------------------------
// The same implicit GEMM on the bf16 matrix cores (v_mfma_f32_16x16x32_bf16, 16x the f32
// rate) for inputs that are exact in bf16 -- spikes (0/1) -- with the f32 weights split
// w = hi + mid + lo into three bf16 parts (round-to-nearest; the residuals are exact in
// f32, so the parts carry all 24 mantissa bits).  Every product x*part is exact in f32 and
// accumulates in f32: the result equals the f32 conv up to summation order.
// K = (tap, channel) in chunks of 32: lane group g = lane >> 4 supplies 8 consecutive
// channels of one tap (A: 8 floats of its pixel from LDS; B: 8 weights [tap][n][c0..c0+7]).
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int KIN, int NOUT>
struct Bf3Geo {
    static_assert(KIN % 8 == 0 && (KIN <= 32 ? 32 % KIN == 0 : KIN % 32 == 0), "bf16 conv: KIN 8, 16, 32, 64..");
    static constexpr int GPT = KIN / 8;                   // lane groups per tap
    static constexpr int TPI = GPT >= 4 ? 1 : 4 / GPT;    // taps per instruction
    static constexpr int IPT = GPT >= 4 ? GPT / 4 : 1;    // instructions per tap
    static constexpr int NI = ((9 + TPI - 1) / TPI) * IPT;  // K chunks of 32
    static constexpr int NNT = (NOUT + 15) / 16;
};

// tap and first channel of lane group g in K chunk i (tap >= 9: padding)
template <int KIN>
__device__ inline void bf3_k(int i, int g, int& tap, int& c0) {
    using G = Bf3Geo<KIN, 16>;
    if constexpr (G::GPT >= 4) {
        tap = i / G::IPT;
        c0 = ((i % G::IPT) * 4 + g) * 8;
    } else {
        tap = i * G::TPI + g / G::GPT;
        c0 = (g % G::GPT) * 8;
    }
}

__device__ inline bool exact_bf16(float v) { return v == (float)(__bf16)v; }

template <int KIN, int NOUT, int WNT = Bf3Geo<KIN, NOUT>::NNT>
__device__ inline void bf3_load_b(const float* __restrict__ wB, int i, int ntb, float (&w)[WNT][8]) {
    const int lane = threadIdx.x & 63, m = lane & 15, g = lane >> 4;
    int tap, c0;
    bf3_k<KIN>(i, g, tap, c0);
#pragma unroll
    for (int nt = 0; nt < WNT; ++nt) {
        const int n = (ntb + nt) * 16 + m;
        if (tap < 9 && n < NOUT) {
            const float* p = wB + (int64_t)(tap * NOUT + n) * KIN + c0;
            const float4 u = *reinterpret_cast<const float4*>(p), v = *reinterpret_cast<const float4*>(p + 4);
            w[nt][0] = u.x; w[nt][1] = u.y; w[nt][2] = u.z; w[nt][3] = u.w;
            w[nt][4] = v.x; w[nt][5] = v.y; w[nt][6] = v.z; w[nt][7] = v.w;
        } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) w[nt][j] = 0.0f;
        }
    }
}

template <int KIN, int NOUT, int NW, typename AT = float, int NG = 1>
__device__ void mfma_conv3x3_bf3(const AT* src, const float* __restrict__ wB, MfmaAcc<KIN, NOUT, NW, NG>& acc) {
    using G = Bf3Geo<KIN, NOUT>;
    using A = MfmaAcc<KIN, NOUT, NW, NG>;
    static_assert(NT == 256 && TW == 32 && 16 % NW == 0, "MFMA conv: 8x32 tiles, NW | 16");
    static_assert(G::NNT == MfmaGeo<KIN, NOUT>::NNT, "accumulator tiling");
    constexpr bool ABF = std::is_same<AT, __bf16>::value;  // A: bf16 tile [HN][KIN] of exact values
    constexpr int P = ABF ? KIN : Pad<KIN>::v, MT = A::MT, WNT = A::WNT;
    const int lane = threadIdx.x & 63, m = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int mtb = A::mt0(wv), ntb = A::nt0(wv);
    float wc[WNT][8], wn[WNT][8];
    bf3_load_b<KIN, NOUT, WNT>(wB, 0, ntb, wc);
#pragma unroll
    for (int i = 0; i < G::NI; ++i) {
        if (i + 1 < G::NI) bf3_load_b<KIN, NOUT, WNT>(wB, i + 1, ntb, wn);  // next chunk's weights in flight
        bf16x8 bh[WNT], bm[WNT], bl[WNT];
#pragma unroll
        for (int nt = 0; nt < WNT; ++nt)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float w = wc[nt][j];
                const __bf16 h = (__bf16)w;
                const float r1 = w - (float)h;
                const __bf16 md = (__bf16)r1;
                bh[nt][j] = h;
                bm[nt][j] = md;
                bl[nt][j] = (__bf16)(r1 - (float)md);
            }
        int tap, c0;
        bf3_k<KIN>(i, g, tap, c0);
        const int ky = tap / 3, kx = tap - 3 * (tap / 3);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int T = mtb + mt, row = T >> 1, cb = (T & 1) * 16;
            bf16x8 a;
            if (tap < 9) {
                const AT* ap = src + ((row + ky) * HWD + cb + m + kx) * P + c0;
                if constexpr (ABF) {
                    a = *reinterpret_cast<const bf16x8*>(ap);
                } else {
                    const float4 u = *reinterpret_cast<const float4*>(ap), v = *reinterpret_cast<const float4*>(ap + 4);
                    a[0] = (__bf16)u.x; a[1] = (__bf16)u.y; a[2] = (__bf16)u.z; a[3] = (__bf16)u.w;
                    a[4] = (__bf16)v.x; a[5] = (__bf16)v.y; a[6] = (__bf16)v.z; a[7] = (__bf16)v.w;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) a[j] = (__bf16)0.0f;
            }
#pragma unroll
            for (int nt = 0; nt < WNT; ++nt) {
                acc.v[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bl[nt], acc.v[mt][nt], 0, 0, 0);
                acc.v[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bm[nt], acc.v[mt][nt], 0, 0, 0);
                acc.v[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bh[nt], acc.v[mt][nt], 0, 0, 0);
            }
        }
        if (i + 1 < G::NI) {
#pragma unroll
            for (int nt = 0; nt < WNT; ++nt)
#pragma unroll
                for (int j = 0; j < 8; ++j) wc[nt][j] = wn[nt][j];
        }
    }
}

// The B operand of mfma_conv3x3_bf3 split ONCE per block: weights [tap][NOUT][KIN] (f32,
// global) -> LDS fragments [chunk i][n-tile][part hi/mid/lo][lane][8] bf16, exactly what a
// lane feeds v_mfma_f32_16x16x32_bf16 (same round-to-nearest split as the in-loop form, so
// results are bit-identical).  load() issues the global reads at kernel start; store()
// splits and writes before a later barrier.
template <int KIN, int NOUT, int NTH>
struct FragStage {
    using G = Bf3Geo<KIN, NOUT>;
    static constexpr int E = G::NI * G::NNT * 64 * 8;  // elements per part
    static constexpr int R = (E + NTH - 1) / NTH;
    static constexpr int HALFS = 3 * E;                // bf16 entries in LDS
    float r[R];
    __device__ inline void load(const float* __restrict__ wB) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int e = (int)threadIdx.x + i * NTH;
            const int j = e & 7, lane = (e >> 3) & 63, rest = e >> 9;
            const int nt = rest % G::NNT, ch = rest / G::NNT, n = nt * 16 + (lane & 15);
            int tap, c0;
            bf3_k<KIN>(ch, lane >> 4, tap, c0);
            // unconditional load (index 0 where the element is padding), selected after: a conditional
            // load made the compiler wait before issuing the next one
            const bool ok = e < E && tap < 9 && n < NOUT;
            const float v = wB[ok ? (tap * NOUT + n) * KIN + c0 + j : 0];
            r[i] = ok ? v : 0.0f;
        }
    }
    // Two convs sharing the A operand in one B operand (NOUT <= 8, one n-tile): columns n < 8 from wB0,
    // columns 8 <= n < 8 + NOUT from wB1 (the recurrent input gradient packed beside the ff one)
    __device__ inline void load2(const float* __restrict__ wB0, const float* __restrict__ wB1) {
        static_assert(NOUT <= 8 && G::NNT == 1, "packed fragments: two convs of <= 8 outputs");
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int e = (int)threadIdx.x + i * NTH;
            const int j = e & 7, lane = (e >> 3) & 63, ch = e >> 9, n = lane & 15;
            int tap, c0;
            bf3_k<KIN>(ch, lane >> 4, tap, c0);
            const float* w = n < 8 ? wB0 : wB1;
            const int nn = n & 7;
            const bool ok = e < E && tap < 9 && nn < NOUT;
            const float v = w[ok ? (tap * NOUT + nn) * KIN + c0 + j : 0];
            r[i] = ok ? v : 0.0f;
        }
    }
    __device__ inline void store(__bf16* lds) const {
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int e = (int)threadIdx.x + i * NTH;
            if (e < E) {
                const int low = e & 511, frag = e >> 9;  // (lane, j) and (chunk, n-tile)
                const float w = r[i];
                const __bf16 h = (__bf16)w;
                const float r1 = w - (float)h;
                const __bf16 md = (__bf16)r1;
                __bf16* f = lds + frag * 3 * 512 + low;
                f[0] = h;
                f[512] = md;
                f[1024] = (__bf16)(r1 - (float)md);
            }
        }
    }
};

// mfma_conv3x3_bf3 with the B operand from FragStage fragments in LDS (no per-wave split).
// A from an f32 halo tile [HN][Pad<KIN>], or (AT = __bf16) from a bf16 tile [HN][KIN] of
// exact values (spikes): one 16-B LDS read is the lane's A operand.
template <int KIN, int NOUT, int NW, typename AT = float>
__device__ void mfma_conv3x3_bf3f(const AT* src, const __bf16* frag, MfmaAcc<KIN, NOUT, NW>& acc) {
    using G = Bf3Geo<KIN, NOUT>;
    static_assert(NT == 256 && TW == 32 && 16 % NW == 0, "MFMA conv: 8x32 tiles, NW | 16");
    static_assert(G::NNT == MfmaGeo<KIN, NOUT>::NNT, "accumulator tiling");
    constexpr bool ABF = std::is_same<AT, __bf16>::value;
    constexpr int P = ABF ? KIN : Pad<KIN>::v, MT = 16 / NW;
    const int lane = threadIdx.x & 63, m = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const bf16x8* fv = reinterpret_cast<const bf16x8*>(frag);
#pragma unroll
    for (int i = 0; i < G::NI; ++i) {
        bf16x8 bh[G::NNT], bm[G::NNT], bl[G::NNT];
#pragma unroll
        for (int nt = 0; nt < G::NNT; ++nt) {
            const bf16x8* f = fv + (i * G::NNT + nt) * 3 * 64 + lane;
            bh[nt] = f[0];
            bm[nt] = f[64];
            bl[nt] = f[128];
        }
        int tap, c0;
        bf3_k<KIN>(i, g, tap, c0);
        const int ky = tap / 3, kx = tap - 3 * (tap / 3);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int T = wv * MT + mt, row = T >> 1, cb = (T & 1) * 16;
            bf16x8 a;
            if (tap < 9) {
                const AT* ap = src + ((row + ky) * HWD + cb + m + kx) * P + c0;
                if constexpr (ABF) {
                    a = *reinterpret_cast<const bf16x8*>(ap);
                } else {
                    const float4 u = *reinterpret_cast<const float4*>(ap), v = *reinterpret_cast<const float4*>(ap + 4);
                    a[0] = (__bf16)u.x; a[1] = (__bf16)u.y; a[2] = (__bf16)u.z; a[3] = (__bf16)u.w;
                    a[4] = (__bf16)v.x; a[5] = (__bf16)v.y; a[6] = (__bf16)v.z; a[7] = (__bf16)v.w;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) a[j] = (__bf16)0.0f;
            }
#pragma unroll
            for (int nt = 0; nt < G::NNT; ++nt) {
                acc.v[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bl[nt], acc.v[mt][nt], 0, 0, 0);
                acc.v[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bm[nt], acc.v[mt][nt], 0, 0, 0);
                acc.v[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bh[nt], acc.v[mt][nt], 0, 0, 0);
            }
        }
    }
}

// mfma_conv3x3_bf3f with the fragments in global memory (snnflow_prep_desc.frag_fwd, L2-resident:
// every block reads the same few KB), the next chunk's fragments in flight during this chunk's
// products.  C = 16 / 32, where the fragments do not fit beside the tiles in LDS.
template <int KIN, int NOUT, int NW, typename AT = float, int NG = 1>
__device__ void mfma_conv3x3_bf3g(const AT* src, const __bf16* __restrict__ frag, MfmaAcc<KIN, NOUT, NW, NG>& acc) {
    using G = Bf3Geo<KIN, NOUT>;
    using A = MfmaAcc<KIN, NOUT, NW, NG>;
    static_assert(NT == 256 && TW == 32 && 16 % NW == 0, "MFMA conv: 8x32 tiles, NW | 16");
    static_assert(G::NNT == MfmaGeo<KIN, NOUT>::NNT, "accumulator tiling");
    constexpr bool ABF = std::is_same<AT, __bf16>::value;
    constexpr int P = ABF ? KIN : Pad<KIN>::v, MT = A::MT, WNT = A::WNT;
    const int lane = threadIdx.x & 63, m = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int mtb = A::mt0(wv), ntb = A::nt0(wv);
    const bf16x8* fv = reinterpret_cast<const bf16x8*>(frag) + lane;
    bf16x8 cur[WNT][3], nxt[WNT][3];
#pragma unroll
    for (int nt = 0; nt < WNT; ++nt)
#pragma unroll
        for (int q = 0; q < 3; ++q) cur[nt][q] = fv[((ntb + nt) * 3 + q) * 64];
#pragma unroll
    for (int i = 0; i < G::NI; ++i) {
        if (i + 1 < G::NI) {
#pragma unroll
            for (int nt = 0; nt < WNT; ++nt)
#pragma unroll
                for (int q = 0; q < 3; ++q) nxt[nt][q] = fv[(((i + 1) * G::NNT + ntb + nt) * 3 + q) * 64];
        }
        // keep the next k-step's fragment loads here, a whole k-step of MFMAs ahead of their use (the
        // scheduler otherwise sinks them next to their first MFMA under register pressure: an L2 round
        // trip exposed every few MFMAs)
        if constexpr (SNNFLOW_PIN_PF) __builtin_amdgcn_sched_barrier(0);
        int tap, c0;
        bf3_k<KIN>(i, g, tap, c0);
        const int ky = tap / 3, kx = tap - 3 * (tap / 3);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int T = mtb + mt, row = T >> 1, cb = (T & 1) * 16;
            bf16x8 a;
            if (tap < 9) {
                const AT* ap = src + ((row + ky) * HWD + cb + m + kx) * P + c0;
                if constexpr (ABF) {
                    a = *reinterpret_cast<const bf16x8*>(ap);
                } else {
                    const float4 u = *reinterpret_cast<const float4*>(ap), v = *reinterpret_cast<const float4*>(ap + 4);
                    a[0] = (__bf16)u.x; a[1] = (__bf16)u.y; a[2] = (__bf16)u.z; a[3] = (__bf16)u.w;
                    a[4] = (__bf16)v.x; a[5] = (__bf16)v.y; a[6] = (__bf16)v.z; a[7] = (__bf16)v.w;
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) a[j] = (__bf16)0.0f;
            }
#pragma unroll
            for (int nt = 0; nt < WNT; ++nt) {
                acc.v[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, cur[nt][2], acc.v[mt][nt], 0, 0, 0);
                acc.v[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, cur[nt][1], acc.v[mt][nt], 0, 0, 0);
                acc.v[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, cur[nt][0], acc.v[mt][nt], 0, 0, 0);
            }
        }
        if (i + 1 < G::NI) {
#pragma unroll
            for (int nt = 0; nt < WNT; ++nt)
#pragma unroll
                for (int q = 0; q < 3; ++q) cur[nt][q] = nxt[nt][q];
        }
    }
}

// The transposed 3x3 conv (input gradient: A = dL/dy at the flipped tap offset, as
// mfma_conv3x3<..., FLIP = true>) with BOTH operands split into three bf16 parts: A from a
// three-part bf16 tile [3][HN][KIN] (src3, hi / mid / lo of the f32 gradient), B from FragStage
// fragments.  Six products per K chunk (mid*mid, lo*hi, hi*lo, mid*hi, hi*mid, hi*hi, small
// to large; the dropped ones are below 2^-24 relative), each on v_mfma_f32_16x16x32_bf16 at
// 16 cycles against 8 x 32 for the same K on the f32 matrix cores; f32 accumulation.
template <int KIN, int NOUT, int NW>
__device__ void mfma_dgrad_bf6(const __bf16* src3, const __bf16* frag, MfmaAcc<KIN, NOUT, NW>& acc) {
    using G = Bf3Geo<KIN, NOUT>;
    static_assert(NT == 256 && TW == 32 && 16 % NW == 0, "MFMA conv: 8x32 tiles, NW | 16");
    static_assert(G::NNT == MfmaGeo<KIN, NOUT>::NNT, "accumulator tiling");
    constexpr int MT = 16 / NW, PART = HN * KIN;
    const int lane = threadIdx.x & 63, m = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const bf16x8* fv = reinterpret_cast<const bf16x8*>(frag);
#pragma unroll
    for (int i = 0; i < G::NI; ++i) {
        bf16x8 bh[G::NNT], bm[G::NNT], bl[G::NNT];
#pragma unroll
        for (int nt = 0; nt < G::NNT; ++nt) {
            const bf16x8* f = fv + (i * G::NNT + nt) * 3 * 64 + lane;
            bh[nt] = f[0];
            bm[nt] = f[64];
            bl[nt] = f[128];
        }
        int tap, c0;
        bf3_k<KIN>(i, g, tap, c0);
        const int ky = tap / 3, kx = tap - 3 * (tap / 3);
        const int oy = 2 - ky, ox = 2 - kx;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int T = wv * MT + mt, row = T >> 1, cb = (T & 1) * 16;
            bf16x8 ah, am, al;
            if (tap < 9) {
                const __bf16* ap = src3 + ((row + oy) * HWD + cb + m + ox) * KIN + c0;
                ah = *reinterpret_cast<const bf16x8*>(ap);
                am = *reinterpret_cast<const bf16x8*>(ap + PART);
                al = *reinterpret_cast<const bf16x8*>(ap + 2 * PART);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) ah[j] = am[j] = al[j] = (__bf16)0.0f;
            }
#pragma unroll
            for (int nt = 0; nt < G::NNT; ++nt) {
                f32x4 c = acc.v[mt][nt];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm[nt], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh[nt], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl[nt], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh[nt], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm[nt], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh[nt], c, 0, 0, 0);
                acc.v[mt][nt] = c;
            }
        }
    }
}

// mfma_dgrad_bf6 with the weight fragments in global memory (snnflow_prep_desc.frag_bwd,
// L2-resident), the next chunk's in flight during this chunk's products (C = 16 / 32).
template <int KIN, int NOUT, int NW, int NG = 1>
__device__ void mfma_dgrad_bf6g(const __bf16* src3, const __bf16* __restrict__ frag, MfmaAcc<KIN, NOUT, NW, NG>& acc) {
    using G = Bf3Geo<KIN, NOUT>;
    using A = MfmaAcc<KIN, NOUT, NW, NG>;
    static_assert(NT == 256 && TW == 32 && 16 % NW == 0, "MFMA conv: 8x32 tiles, NW | 16");
    static_assert(G::NNT == MfmaGeo<KIN, NOUT>::NNT, "accumulator tiling");
    constexpr int MT = A::MT, WNT = A::WNT, PART = HN * KIN;
    const int lane = threadIdx.x & 63, m = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int mtb = A::mt0(wv), ntb = A::nt0(wv);
    const bf16x8* fv = reinterpret_cast<const bf16x8*>(frag) + lane;
    bf16x8 cur[WNT][3], nxt[WNT][3];
#pragma unroll
    for (int nt = 0; nt < WNT; ++nt)
#pragma unroll
        for (int q = 0; q < 3; ++q) cur[nt][q] = fv[((ntb + nt) * 3 + q) * 64];
#pragma unroll
    for (int i = 0; i < G::NI; ++i) {
        if (i + 1 < G::NI) {
#pragma unroll
            for (int nt = 0; nt < WNT; ++nt)
#pragma unroll
                for (int q = 0; q < 3; ++q) nxt[nt][q] = fv[(((i + 1) * G::NNT + ntb + nt) * 3 + q) * 64];
        }
        // keep the next k-step's fragment loads here, a whole k-step of MFMAs ahead of their use (the
        // scheduler otherwise sinks them next to their first MFMA under register pressure: an L2 round
        // trip exposed every few MFMAs)
        if constexpr (SNNFLOW_PIN_PF) __builtin_amdgcn_sched_barrier(0);
        int tap, c0;
        bf3_k<KIN>(i, g, tap, c0);
        const int ky = tap / 3, kx = tap - 3 * (tap / 3);
        const int oy = 2 - ky, ox = 2 - kx;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int T = mtb + mt, row = T >> 1, cb = (T & 1) * 16;
            bf16x8 ah, am, al;
            if (tap < 9) {
                const __bf16* ap = src3 + ((row + oy) * HWD + cb + m + ox) * KIN + c0;
                ah = *reinterpret_cast<const bf16x8*>(ap);
                am = *reinterpret_cast<const bf16x8*>(ap + PART);
                al = *reinterpret_cast<const bf16x8*>(ap + 2 * PART);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) ah[j] = am[j] = al[j] = (__bf16)0.0f;
            }
#pragma unroll
            for (int nt = 0; nt < WNT; ++nt) {
                f32x4 c = acc.v[mt][nt];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, cur[nt][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, cur[nt][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, cur[nt][2], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, cur[nt][0], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, cur[nt][1], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, cur[nt][0], c, 0, 0, 0);
                acc.v[mt][nt] = c;
            }
        }
        if (i + 1 < G::NI) {
#pragma unroll
            for (int nt = 0; nt < WNT; ++nt)
#pragma unroll
                for (int q = 0; q < 3; ++q) cur[nt][q] = nxt[nt][q];
        }
    }
}

// hi / mid / lo bf16 parts of four floats into three bf16 tiles (part stride `part`).
__device__ inline void split3_store4(__bf16* d, int part, const float4& v) {
    typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
    const float x[4] = {v.x, v.y, v.z, v.w};
    bf16x4 h, md, lo;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const __bf16 a = (__bf16)x[j];
        const float r1 = x[j] - (float)a;
        const __bf16 b = (__bf16)r1;
        h[j] = a;
        md[j] = b;
        lo[j] = (__bf16)(r1 - (float)b);
    }
    *reinterpret_cast<bf16x4*>(d) = h;
    *reinterpret_cast<bf16x4*>(d + part) = md;
    *reinterpret_cast<bf16x4*>(d + 2 * part) = lo;
}

// A weight tensor of N floats staged into LDS by the whole block: the loads are issued into
// registers at kernel start (load) and written to LDS before a later barrier (store), so
// the matrix-core loops read their B operands from LDS and never wait on global memory.
template <int N, int NTH>
struct WStage {
    static constexpr int R = (N + NTH - 1) / NTH;
    float r[R];
    __device__ inline void load(const float* __restrict__ w) {
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int e = (int)threadIdx.x + i * NTH;
            r[i] = (e < N) ? w[e] : 0.0f;
        }
    }
    __device__ inline void store(float* lds) const {
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int e = (int)threadIdx.x + i * NTH;
            if (e < N) lds[e] = r[i];
        }
    }
};

// Accumulators (C/D layout: lane holds pixels 4g..4g+3 of its M-tile, channel n = lane & 15)
// [+ a second set added element-wise when SUM: ff + rec] -> LDS out[NT][Pad<NOUT>].
template <bool SUM, int KIN, int NOUT, int NW, int KIN2, int NG>
__device__ void mfma_store(const MfmaAcc<KIN, NOUT, NW, NG>& acc, const MfmaAcc<KIN2, NOUT, NW, NG>& acc2, float* out) {
    using A = MfmaAcc<KIN, NOUT, NW, NG>;
    constexpr int PO = Pad<NOUT>::v, MT = A::MT, WNT = A::WNT;
    const int lane = threadIdx.x & 63, m = lane & 15, g = lane >> 4;
    const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int mtb = A::mt0(wv), ntb = A::nt0(wv);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int T = mtb + mt, row = T >> 1, c0 = (T & 1) * 16;
#pragma unroll
        for (int nt = 0; nt < WNT; ++nt) {
            const int n = (ntb + nt) * 16 + m;
            if (n < NOUT) {
                f32x4 v = acc.v[mt][nt];
                if constexpr (SUM) v = v + acc2.v[mt][nt];
#pragma unroll
                for (int r = 0; r < 4; ++r) out[(row * TW + c0 + g * 4 + r) * PO + n] = v[r];
            }
        }
    }
}

// Opaque use of a register array: stops LLVM from sinking its computation into a
// following conditional block (where the scalar-weight schedule no longer fits).
template <int N>
__device__ inline void pin(float (&v)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(v[i]));
}

// Block-level sums of per-thread floats, then one fp64 atomic add per sum.  The block's
// threads form PARTS groups of NT consecutive threads (whole waves); each group sums
// its own NV values and dst(part, j) is the accumulator address of sum j of group part.
// One LDS scratch for the block sums of every kernel variant (a __shared__ array in the templated
// function would be allocated once per instantiation, all of them in a wavefront launch).
constexpr int kSumScratch = 8 * 4 * 48;  // waves x rows x sums (C = 32 backward: 3 * 16)
__device__ inline float* sum_scratch() {
    __shared__ float buf[kSumScratch];
    return buf;
}

template <int NV, int PARTS, typename Dst>
__device__ void block_atomic_sum_parts(const float (&v)[NV], Dst dst) {
    constexpr int WPP = NT / 64, NW = WPP * PARTS;
    if constexpr (NW * 4 * NV > kSumScratch) {  // many sums (C = 32 top LIF backward): wave totals
        __shared__ float wred[NW][NV];
        const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
        for (int j = 0; j < NV; ++j) {
            const float s = wave_total(v[j]);
            if (lane == 0) wred[wv][j] = s;
        }
        __syncthreads();
        for (int t = threadIdx.x; t < PARTS * NV; t += NT * PARTS) {
            const int part = t / NV, j = t - part * NV;
            double s = 0.0;
#pragma unroll
            for (int w = 0; w < WPP; ++w) s += (double)wred[part * WPP + w][j];
            atomicAdd(dst(part, j), s);
        }
        return;
    }
    // 16-lane row totals by DPP (four chains at a time, no readlane round trips), the four row
    // totals of every wave through LDS, then the per-part sum in fp64
    float* red = sum_scratch();  // [NW * 4][NV]
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int j0 = 0; j0 < NV; j0 += 4) {
        constexpr int G = 4;
        float r[G];
#pragma unroll
        for (int j = 0; j < G; ++j) r[j] = j0 + j < NV ? v[j0 + j] + dppf<0xB1>(v[j0 + j]) : 0.0f;
#pragma unroll
        for (int j = 0; j < G; ++j) r[j] += dppf<0x4E>(r[j]);
#pragma unroll
        for (int j = 0; j < G; ++j) r[j] += dppf<0x141>(r[j]);
#pragma unroll
        for (int j = 0; j < G; ++j) r[j] += dppf<0x140>(r[j]);
        if ((lane & 15) == 0) {
#pragma unroll
            for (int j = 0; j < G; ++j)
                if (j0 + j < NV) red[(wv * 4 + (lane >> 4)) * NV + j0 + j] = r[j];
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < PARTS * NV; t += NT * PARTS) {
        const int part = t / NV, j = t - part * NV;
        double s = 0.0;
#pragma unroll
        for (int w = 0; w < 4 * WPP; ++w) s += (double)red[(part * 4 * WPP + w) * NV + j];
        atomicAdd(dst(part, j), s);
    }
}

template <int NV>
__device__ void block_atomic_sum(const float (&v)[NV], double* acc) {
    block_atomic_sum_parts<NV, 1>(v, [acc](int, int j) { return acc + j; });
}

// Accumulators already consumed by an earlier kernel of the chain are zeroed here
// (grid-stride over all threads of the launch).
__device__ inline void zero_consumed(double* z0, double* z1, int n, const Grid& g) {
    for (int j = g.bid * (int)blockDim.x + threadIdx.x; j < n; j += g.nb * (int)blockDim.x) {
        if (z0) z0[j] = 0.0;
        if (z1) z1[j] = 0.0;
    }
}
__device__ inline void zero_consumed(double* z0, double* z1, int n) { zero_consumed(z0, z1, n, hw_grid()); }

// Totals of the M sums of a sharded accumulator (n sums per replica, M <= n, M <= NT)
// into LDS out[M]: TPJ = NT/M threads per sum each add a strided subset of the
// replicas (all their loads in flight at once), then one LDS pass.  One global round
// trip; called by every thread of the block (contains barriers).
// Split form: acc_gather_load issues the replica loads into registers (call it before the
// kernel's other loads, so that the coefficient math after acc_gather_reduce overlaps their
// latency instead of waiting behind them: vmcnt retires loads in order).
template <int M>
struct AccGather {
    static_assert(M >= 1 && M <= NT, "acc_gather: M sums");
    static constexpr int TPJ = NT / M;
    static constexpr int PER = (kAccShards + TPJ - 1) / TPJ;
    double v[PER];
};

template <int M, bool SC1 = false>
__device__ inline void acc_gather_load(const double* acc, int n, AccGather<M>& r) {
    using A = AccGather<M>;
    const int tid = threadIdx.x, st = acc_stride(n);
    const int j = tid % M, g = tid / M;
#pragma unroll
    for (int k = 0; k < A::PER; ++k) {
        const int sh = g + k * A::TPJ;
        const bool ok = tid < A::TPJ * M && sh < kAccShards;
        const double v = ld_f64<SC1>(acc + (ok ? sh * st + j : 0));  // unconditional (see FragStage::load)
        r.v[k] = ok ? v : 0.0;
    }
}

template <int M>
__device__ void acc_gather_reduce(const AccGather<M>& r, double* out) {
    using A = AccGather<M>;
    constexpr int TPJ = A::TPJ, PER = A::PER;
    __shared__ double red[TPJ * M];
    const int tid = threadIdx.x;
    if (tid < TPJ * M) {
        const int j = tid % M, g = tid / M;
        double sum = 0.0;
#pragma unroll
        for (int k = 0; k < PER; ++k) sum += r.v[k];
        red[g * M + j] = sum;
    }
    __syncthreads();
    if (tid < M) {
        double sum = 0.0;
        for (int g = 0; g < TPJ; ++g) sum += red[g * M + tid];
        out[tid] = sum;
    }
    __syncthreads();
}

template <int M>
__device__ void acc_gather(const double* acc, int n, double* out) {
    static_assert(M >= 1 && M <= NT, "acc_gather: M sums");
    constexpr int TPJ = NT / M;
    constexpr int PER = (kAccShards + TPJ - 1) / TPJ;
    __shared__ double red[TPJ * M];
    const int tid = threadIdx.x, st = acc_stride(n);
    if (tid < TPJ * M) {
        const int j = tid % M, g = tid / M;
        double v[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int sh = g + k * TPJ;
            v[k] = sh < kAccShards ? acc[sh * st + j] : 0.0;
        }
        double sum = 0.0;
#pragma unroll
        for (int k = 0; k < PER; ++k) sum += v[k];
        red[g * M + j] = sum;
    }
    __syncthreads();
    if (tid < M) {
        double sum = 0.0;
        for (int g = 0; g < TPJ; ++g) sum += red[g * M + tid];
        out[tid] = sum;
    }
    __syncthreads();
}

// The same over NTH threads with the reduction scratch supplied by the caller (a region of the
// block's LDS pool that is not live yet): no static LDS of its own, and TPJ = NTH / M threads per sum,
// each summing PER = 32 / TPJ shards (C = 32 backward: 2C = 64 sums x 8 threads, 4 loads each,
// instead of 162 x 1 thread with 32 loads in flight and 32 dependent fp64 adds).
template <int M, int NTH>
__device__ void acc_gather_pool(const double* acc, int n, double* out, double* red) {
    static_assert(M >= 1 && M <= NTH, "acc_gather_pool: M sums");
    constexpr int TPJ = NTH / M;
    constexpr int PER = (kAccShards + TPJ - 1) / TPJ;
    const int tid = threadIdx.x, st = acc_stride(n);
    if (tid < TPJ * M) {
        const int j = tid % M, g = tid / M;
        double v[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int sh = g + k * TPJ;
            v[k] = sh < kAccShards ? acc[sh * st + j] : 0.0;
        }
        double sum = 0.0;
#pragma unroll
        for (int k = 0; k < PER; ++k) sum += v[k];
        red[g * M + j] = sum;
    }
    __syncthreads();
    if (tid < M) {
        double sum = 0.0;
        for (int g = 0; g < TPJ; ++g) sum += red[g * M + tid];
        out[tid] = sum;
    }
    __syncthreads();
}

__device__ inline void zero4(float4* r, int n) {
    for (int i = 0; i < n; ++i) r[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Register-prefetch budget: halo tiles of up to 16 channels are held in registers
// (<= 6 float4 per thread each); wider layers stage straight into LDS.
template <int CH, int NTH = NT>
struct Prefetch { static constexpr bool on = (CH % 4 == 0) && Halo4<CH, NTH>::R <= 6; };

// Conv-layer kernels run SPLIT threads per output pixel (SPLIT groups of NT threads, whole
// waves): group `part` owns output channels [part*C/SPLIT, ...) in the forward and input
// channels [part*CIN/SPLIT, ...) in the backward.  SPLIT = 2 doubles the waves per SIMD
// (the launch has only 2 blocks per CU at cfg2) so one wave's loads and barriers overlap
// another's arithmetic.  The group index is wave-uniform (readfirstlane): weight
// addresses stay scalar.
__device__ inline int thread_part() { return __builtin_amdgcn_readfirstlane((int)threadIdx.x / NT); }


}  // namespace snnflow
