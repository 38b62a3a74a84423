// Device-side building blocks shared by the snnflow HIP kernels (gfx950 / CDNA4).
//
// Numerics: the library is compiled with -ffp-contract=off so elementwise code
// keeps the reference's separate multiply / add roundings; convolution
// accumulations use explicit fmaf.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "snnflow.h"

namespace snnflow {

constexpr int TH = SNNFLOW_TILE_H;
constexpr int TW = SNNFLOW_TILE_W;
constexpr int NT = TH * TW;             // 256 threads = 4 waves, one output pixel each
constexpr int HH = TH + 2;              // halo tile rows
constexpr int HWD = TW + 2;             // halo tile cols
constexpr int HN = HH * HWD;            // halo pixels (340)
constexpr float kPiF = 3.14159265358979323846f;

// LDS pixel stride (floats) for a C-channel pixel: conflict-free ds_read_b128 when
// consecutive lanes read consecutive pixels (C=8 -> 12, 16 -> 20, 32 -> 36 dwords).
template <int C> struct Pad { static constexpr int v = (C <= 4 || C % 4 != 0) ? C : C + 4; };

// Channel-block width for vector LDS access of a C-channel pixel.
template <int C> struct VecW { static constexpr int v = (C % 4 == 0) ? 4 : ((C % 2 == 0) ? 2 : 1); };

// Weights are read with wave-uniform indices; reading them through the constant
// address space (4) lets the compiler use scalar loads (s_load_dwordx8/x16) whose
// results feed v_fma as SGPR operands, instead of one vector load per lane.
typedef const __attribute__((address_space(4))) float* cfloat_ptr;
__device__ inline cfloat_ptr as_const(const float* p) { return (cfloat_ptr)(p); }

struct Tile { int b, h0, w0; };

__host__ __device__ inline int tiles_per_image(int H, int W) {
    return ((H + TH - 1) / TH) * ((W + TW - 1) / TW);
}

// Block -> tile.  Blocks b and b+8 share an XCD under round-robin dispatch; give each
// XCD group a contiguous range of tiles so neighbouring tiles (shared halo rows) hit
// the same L2.  Bijective for any grid size.  Speed only, never correctness.
// A kernel body's view of its grid: the hardware grid for a plain launch, or one task's
// range of blocks inside a wavefront launch (several independent layer-steps per launch).
struct Grid { int bid, nb; };
__device__ inline Grid hw_grid() { return Grid{(int)blockIdx.x, (int)gridDim.x}; }

__device__ inline Tile block_tile(int H, int W, const Grid& g) {
    const int nb = g.nb, bid = g.bid;
    const int q = nb / 8, r = nb % 8, x = bid % 8;
    int t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
    const int tw = (W + TW - 1) / TW, th = (H + TH - 1) / TH;
    Tile tl;
    tl.w0 = (t % tw) * TW; t /= tw;
    tl.h0 = (t % th) * TH;
    tl.b = t / th;
    return tl;
}
__device__ inline Tile block_tile(int H, int W) { return block_tile(H, W, hw_grid()); }

__device__ inline float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// DPP lane exchange (GFX9 encodings): quad_perm [1,0,3,2] = 0xB1, [2,3,0,1] = 0x4E,
// row_half_mirror = 0x141, row_mirror = 0x140.
template <int CTRL>
__device__ inline float dppf(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// Sum over the 64 lanes of a wave, result wave-uniform (all lanes must be active).
// Rows of 16 reduce through DPP (no LDS traffic); the four row totals via readlane.
__device__ inline float wave_total(float v) {
    v += dppf<0xB1>(v);
    v += dppf<0x4E>(v);
    v += dppf<0x141>(v);
    v += dppf<0x140>(v);
    const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
    const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
    const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
    const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
    return ((r0 + r1) + r2) + r3;
}

// Sharded batch-sum accumulators (include/snnflow.h): [shard][acc_stride(n)] doubles.
constexpr int kAccShards = SNNFLOW_ACC_SHARDS;
__host__ __device__ constexpr int acc_stride(int n) { return SNNFLOW_ACC_STRIDE(n); }

// This block's replica of an accumulator of n sums.
__device__ inline double* acc_shard(double* acc, int n, int bid) { return acc + (bid % kAccShards) * acc_stride(n); }
__device__ inline double* acc_shard(double* acc, int n) { return acc_shard(acc, n, (int)blockIdx.x); }

// p[i] as one unconditional 16-B load, or zeros when p is NULL (the load then reads
// fallback[i], which must be valid).  A `p ? p[i] : 0` select makes the compiler split
// the load into four dword loads.
__device__ inline float4 ld4_or_zero(const float4* p, const float4* fallback, int64_t i) {
    const float4 t = (p ? p : fallback)[i];
    return p ? t : make_float4(0.f, 0.f, 0.f, 0.f);
}

// Output stores of the layer kernels (states, pre-BN currents, gradients): write-through
// (sc1 buffer stores) so the kernel does not end with megabytes of dirty L2 lines to write
// back at the boundary (MI355X_MICROARCH.md price list, row 'boundary').  0: plain stores.
#ifndef SNNFLOW_WT_STORES
#define SNNFLOW_WT_STORES 0  // measured: sc1 stores cost 2.48 -> 3.32 ms per cfg2 step (the next kernel loses its L2 hits)
#endif
typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ inline void st_out4(float4* base, int64_t i, const float4& v) {
#if SNNFLOW_WT_STORES
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
    const i32x4 d = {__builtin_bit_cast(int, v.x), __builtin_bit_cast(int, v.y), __builtin_bit_cast(int, v.z),
                     __builtin_bit_cast(int, v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(d, r, (int)(i * 16), 0, 16);  // aux 16 = sc1
#else
    base[i] = v;
#endif
}

// Stores of data no kernel reads before the next time step (the cell states written by the
// conv kernels): write-through when SNNFLOW_WT_STATE, so they do not sit dirty in L2 at the
// kernel boundary.  Measured per call site: faster in k_conv_fwd, slower in the streaming
// k_lif_fwd and for the state gradients of k_layer_bwd (plain stores there).
#ifndef SNNFLOW_WT_STATE
#define SNNFLOW_WT_STATE 1
#endif
__device__ inline void st_state4(float4* base, int64_t i, const float4& v) {
#if SNNFLOW_WT_STATE
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
    const i32x4 d = {__builtin_bit_cast(int, v.x), __builtin_bit_cast(int, v.y), __builtin_bit_cast(int, v.z),
                     __builtin_bit_cast(int, v.w)};
    __builtin_amdgcn_raw_buffer_store_b128(d, r, (int)(i * 16), 0, 16);  // aux 16 = sc1
#else
    base[i] = v;
#endif
}

__device__ inline bool in_image(int h, int w, int H, int W) { return h >= 0 && h < H && w >= 0 && w < W; }

// Loads of bytes another workgroup of the SAME launch wrote (the persistent dataflow kernels,
// snnflow_fwd_seq): SC1 = `sc1` loads, which bypass this CU's vector L1 and are served by the XCD's
// L2 (MI355X_MICROARCH.md, inter-workgroup visibility): never a stale L1 copy.  Producer and
// consumer of such bytes run on the same XCD there (XCD-affine work queues), so the L2 is shared;
// the base pointer must be wave-uniform (buffer descriptor in SGPRs).  SC1 = false: plain loads.
// (the b128 result must be taken as an unsigned vector: read through an int vector and
// __builtin_bit_cast per element, ROCm 7.2 narrows the load to one dword and broadcasts it)
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ inline float4 u4f(const u32x4& v) {
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
template <bool SC1>
__device__ inline float4 ld4(const float4* base, int64_t i) {
    if constexpr (SC1) {
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(base), (short)0, 0x7fffffff, 0x00020000);
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(i * 16), 0, 16);  // aux 16 = sc1
        return u4f(v);
    } else {
        return base[i];
    }
}
template <bool SC1>
__device__ inline float ld1(const float* p) {
    if constexpr (SC1) {
        return __builtin_bit_cast(float, __hip_atomic_load(reinterpret_cast<const unsigned*>(p), __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT));
    } else {
        return *p;
    }
}
template <bool SC1>
__device__ inline double ld_f64(const double* p) {
    if constexpr (SC1) {
        return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    } else {
        return *p;
    }
}
template <bool SC1>
__device__ inline float4 ld4_or_zero_sc(const float4* p, const float4* fallback, int64_t i) {
    const float4 t = ld4<SC1>(p ? p : fallback, i);
    return p ? t : make_float4(0.f, 0.f, 0.f, 0.f);
}

// A C-channel NHWC halo tile as float4 elements e = pixel * (C/4) + quad, distributed
// round-robin over the block's NTH threads (element e -> thread e % NTH, slot e / NTH),
// so a thread issues all R of its loads before using any (register prefetch).
template <int CH, int NTH = NT>
struct Halo4 {
    static constexpr int Q = CH / 4;  // meaningful for CH % 4 == 0 only
    static constexpr int E = HN * Q;
    static constexpr int R = (E + NTH - 1) / NTH;
};

// float4 index of halo element e in an NHWC tensor with CH channels; -1 outside the tile/image.
template <int CH>
__device__ inline int64_t halo_idx4(int e, const Tile& tl, int H, int W) {
    constexpr int Q = CH / 4;
    if (e >= HN * Q) return -1;
    const int p = e / Q, q = e - p * Q;
    const int r = p / HWD, cc = p - r * HWD;
    const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
    if (!in_image(h, w, H, W)) return -1;
    return (((int64_t)tl.b * H + h) * W + w) * Q + q;
}

// BASE: the halo's origin (pixel (h0 - 1, w0 - 1) of image b) is block-uniform, so its 64-bit offset
// is scalar math once per call and each element adds a 32-bit (row, column, quad) offset to it
// (measured at C = 8: forward slot 20.8 -> 20.5 us, backward slot 24.4 -> 25.0 us; at C = 32 the
// forward slot 87 -> 110 us: used for the C = 8 forward halos only).
template <int CH, int NTH = NT, bool BASE = false, bool SC1 = false>
__device__ inline void halo_load(const float* __restrict__ src, const Tile& tl, int H, int W,
                                 float4 (&r)[Halo4<CH, NTH>::R]) {
    if constexpr (SC1) {  // BASE addressing through one sc1 buffer descriptor at the halo origin
        constexpr int Q = CH / 4;
        const float4* base = reinterpret_cast<const float4*>(src) +
                             (((int64_t)tl.b * H + (tl.h0 - 1)) * W + (tl.w0 - 1)) * Q;
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(base), (short)0, 0x7fffffff, 0x00020000);
#pragma unroll
        for (int i = 0; i < Halo4<CH, NTH>::R; ++i) {
            const int e = threadIdx.x + i * NTH;
            const int p = e / Q, q = e - p * Q;
            const int rr = p / HWD, cc = p - rr * HWD;
            const bool ok = e < Halo4<CH, NTH>::E && in_image(tl.h0 + rr - 1, tl.w0 + cc - 1, H, W);
            // outside the image: an offset past num_records, which the range check turns into zeros
            // without a memory access (the descriptor base itself may lie before the tensor)
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, ok ? ((rr * W + cc) * Q + q) * 16 : (int)0x7ffffff0,
                                                                  0, 16);
            r[i] = ok ? u4f(v) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    } else if constexpr (BASE) {
        constexpr int Q = CH / 4;
        const float4* base = reinterpret_cast<const float4*>(src) +
                             (((int64_t)tl.b * H + (tl.h0 - 1)) * W + (tl.w0 - 1)) * Q;
#pragma unroll
        for (int i = 0; i < Halo4<CH, NTH>::R; ++i) {
            const int e = threadIdx.x + i * NTH;
            const int p = e / Q, q = e - p * Q;
            const int rr = p / HWD, cc = p - rr * HWD;
            const bool ok = e < Halo4<CH, NTH>::E && in_image(tl.h0 + rr - 1, tl.w0 + cc - 1, H, W);
            r[i] = ok ? base[(rr * W + cc) * Q + q] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    } else {
#pragma unroll
        for (int i = 0; i < Halo4<CH, NTH>::R; ++i) {
            const int64_t k = halo_idx4<CH>(threadIdx.x + i * NTH, tl, H, W);
            r[i] = (k >= 0) ? reinterpret_cast<const float4*>(src)[k] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    }
}

template <int CH, int NTH = NT>
__device__ inline void halo_store(float* tile, const float4 (&r)[Halo4<CH, NTH>::R]) {
    constexpr int Q = CH / 4;
#pragma unroll
    for (int i = 0; i < Halo4<CH, NTH>::R; ++i) {
        const int e = threadIdx.x + i * NTH;
        if (e < Halo4<CH, NTH>::E) {
            const int p = e / Q, q = e - p * Q;
            *reinterpret_cast<float4*>(tile + p * Pad<CH>::v + 4 * q) = r[i];
        }
    }
}

// ---- spike bit planes (ABI 39): a pixel's CH spikes in one CH-bit word, channel ch at bit
// (ch % 4) * (CH / 4) + ch / 4 (SNNFLOW_SPK_BIT): in the quad-per-lane halo loops (element e = pixel *
// Q + quad, the Q = CH / 4 lanes of a pixel consecutive in the wave) spike j of every quad is one
// ballot, and the pixel's word is Q-bit slices of the four ballots.
template <int CH>
__device__ inline unsigned spk_load_bits(const uint8_t* __restrict__ p, int64_t pix) {
    static_assert(CH == 8 || CH == 16 || CH == 32, "bit-plane widths");
    if constexpr (CH == 8) return p[pix];
    else if constexpr (CH == 16) return reinterpret_cast<const uint16_t*>(p)[pix];
    else return reinterpret_cast<const uint32_t*>(p)[pix];
}
template <int CH>
__device__ inline void spk_store_bits(uint8_t* __restrict__ p, int64_t pix, unsigned w) {
    if constexpr (CH == 8) p[pix] = (uint8_t)w;
    else if constexpr (CH == 16) reinterpret_cast<uint16_t*>(p)[pix] = (uint16_t)w;
    else reinterpret_cast<uint32_t*>(p)[pix] = w;
}
// channels 4q .. 4q+3 of a pixel word as exact 0/1 floats
template <int CH>
__device__ inline float4 spk_quad(unsigned w, int q) {
    constexpr int Q = CH / 4;
    return make_float4((float)((w >> q) & 1u), (float)((w >> (Q + q)) & 1u), (float)((w >> (2 * Q + q)) & 1u),
                       (float)((w >> (3 * Q + q)) & 1u));
}
// The word of this lane's pixel from the spikes s of the wave's quad-per-lane elements (every lane of
// the wave that holds an element calls it; the result is meaningful in every lane of the pixel).
template <int CH>
__device__ inline unsigned spk_pack_wave(const float4& s, int lane) {
    constexpr int Q = CH / 4;
    const unsigned long long b0 = __builtin_amdgcn_ballot_w64(s.x != 0.f), b1 = __builtin_amdgcn_ballot_w64(s.y != 0.f);
    const unsigned long long b2 = __builtin_amdgcn_ballot_w64(s.z != 0.f), b3 = __builtin_amdgcn_ballot_w64(s.w != 0.f);
    const int sh = lane & ~(Q - 1);
    constexpr unsigned m = (1u << Q) - 1u;
    return ((unsigned)(b0 >> sh) & m) | (((unsigned)(b1 >> sh) & m) << Q) | (((unsigned)(b2 >> sh) & m) << (2 * Q)) |
           (((unsigned)(b3 >> sh) & m) << (3 * Q));
}
// halo words of a bit plane in halo_load's element order (element e = pixel * (CH/4) + quad; 0 outside
// the image): one word per element, expanded with spk_quad(w, e % (CH/4)) where it is used
template <int CH, int NTH = NT>
__device__ inline void halo_load_bits(const uint8_t* __restrict__ src, const Tile& tl, int H, int W,
                                      unsigned (&r)[Halo4<CH, NTH>::R]) {
    constexpr int Q = CH / 4;
#pragma unroll
    for (int i = 0; i < Halo4<CH, NTH>::R; ++i) {
        const int64_t k = halo_idx4<CH>(threadIdx.x + i * NTH, tl, H, W);
        r[i] = (k >= 0) ? spk_load_bits<CH>(src, k / Q) : 0u;
    }
}

// Per-channel LIF coefficients: I = y*alpha + shift (torch CPU BN transform order:
// alpha = invstd*gamma, shift = bias - mean*alpha), beta clamped to [0,1].
struct LifCoef { float alpha, shift, beta, theta; };

__device__ inline LifCoef lif_coef(const snnflow_neuron& n, const float* stats, int C, int c) {
    LifCoef k;
    const float mean = stats[c], invstd = stats[C + c];
    k.alpha = invstd * n.bn_weight[c];
    k.shift = n.bn_bias[c] - mean * k.alpha;
    k.beta = fminf(fmaxf(n.beta[c], 0.0f), 1.0f);
    k.theta = n.threshold[c];
    return k;
}

// snn.Leaky (0.9.4, restated: oracle/lif_ref.py LeakyRef), reset_delay=False.
struct LifOut { float s, mout, v, mprime, I; };

__device__ inline LifOut lif_step(float y, float m, const LifCoef& k, bool zero_reset) {
    LifOut o;
    o.I = y * k.alpha + k.shift;
    const float r = (m - k.theta > 0.0f) ? 1.0f : 0.0f;
    if (zero_reset) {
        o.mprime = (1.0f - r) * m;
        o.v = k.beta * o.mprime + o.I;
    } else {
        o.mprime = m;
        o.v = (k.beta * m + o.I) - r * k.theta;
    }
    o.s = (o.v - k.theta > 0.0f) ? 1.0f : 0.0f;
    const float dr = o.s - r;
    o.mout = zero_reset ? o.v - dr * o.v : o.v - dr * k.theta;
    return o;
}

// snntorch ATan surrogate (alpha = 2): alpha/2 / (1 + (pi/2*alpha*x)^2)
__device__ inline float atan_sg(float x) {
    const float u = kPiF * x;
    return __frcp_rn(1.0f + u * u);
}

}  // namespace snnflow
