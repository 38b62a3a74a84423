// Event warping, bilinear IWE splatting and the contrast-maximisation loss (fwd + bwd)
// for gfx950.  Reference: utils/iwe.py:4-93 (purge_unfeasible, get_interpolation,
// interpolate) and loss/flow.py:58-121, 178-303 (EventWarping); restated in
// oracle/iwe_ref.py.
//
// Bit-exactness contract for the corner indices:
//   w = pos + ((tref - ts_k) * f) * s    ts_k = ts + k (f32), no FMA (-ffp-contract=off)
//   y0 = floor(wy), y1 = floor(wy + 1)    (not floor(wy) + 1)
//   idx = (cy*inb)*W + cx*inb computed in f32
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <cstdlib>

#include "snnflow_dev.h"
#include "snnflow_warp.h"

using namespace snnflow;

int snnflow_set_error(int code, const char* msg);
#define SNN_FAIL(code, msg) return snnflow_set_error((code), (msg))
#define SNN_CHECK_LAUNCH()                                                        \
    do {                                                                          \
        hipError_t e_ = hipGetLastError();                                        \
        if (e_ != hipSuccess) return snnflow_set_error((int)e_, hipGetErrorString(e_)); \
    } while (0)

namespace {

// Bijective XCD-aware block order: consecutive logical blocks land on one XCD (blocks b and b+8
// share an XCD under round-robin dispatch), so the neighbouring rows one block reads that the
// next block owns, or a sample's events and images, stay in that XCD's L2.
__device__ inline int xcd_block() {
    const int bid = blockIdx.x, nb = gridDim.x;
    const int x = bid % 8, q = nb / 8, r = nb % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}


// d/dz of max(0, z) as torch.maximum(zeros, z) backward: 1 above, 1/2 on the tie, 0 below.
__device__ inline float relu_tie(float z) { return z > 0.0f ? 1.0f : (z == 0.0f ? 0.5f : 0.0f); }
__device__ inline float sgnf(float d) { return d > 0.0f ? 1.0f : (d < 0.0f ? -1.0f : 0.0f); }

// Event e = (sample b, concatenated index i) of window k: its 4 floats and 2 pol floats.
struct EventRef { const float* ev; const float* pol; int k; };

// The window tables of the argument block (pass offsets; event, polarity and flow pointers), copied
// once per block into LDS: the per-event lookups index them with a per-lane window index, which on
// the argument block itself is a chain of dependent scalar-memory-missing vector loads (the pass
// search alone up to T of them) ahead of every event load.  n0: events per window and sample when
// every window holds the same count (the pass is then one division), else 0.
struct WinTab {
    int32_t off[SNNFLOW_MAX_WINDOWS + 1];
    const float* ev[SNNFLOW_MAX_WINDOWS];
    const float* pol[SNNFLOW_MAX_WINDOWS];
    const float* fl[SNNFLOW_MAX_WINDOWS];
    int n0;
};

// Called by every thread of the block before its first lookup (contains a barrier).
__device__ inline void wintab_load(const snnflow_iwe_loss_args& a, WinTab& w) {
    const int t = threadIdx.x;
    if (t <= a.T) w.off[t] = a.off[t];
    if (t < a.T) {
        w.ev[t] = a.events[t];
        w.pol[t] = a.pol[t];
    }
    if (t < a.tf) w.fl[t] = a.flows[t];
    if (t == 0) {
        int n0 = a.off[1] - a.off[0];
        if (a.off[0] != 0 || n0 <= 0) n0 = 0;
        for (int k = 1; k < a.T && n0 > 0; ++k)
            if (a.off[k + 1] - a.off[k] != n0) n0 = 0;
        w.n0 = n0;
    }
    __syncthreads();
}

__device__ inline int pass_of(const WinTab& w, int T, int i) {
    if (w.n0 > 0) {
        const int k = i / w.n0;
        return k < T ? k : T - 1;
    }
    int k = 0;
    while (k + 1 < T && i >= w.off[k + 1]) ++k;
    return k;
}

__device__ inline EventRef event_ref(const WinTab& w, int T, int b, int i) {
    const int k = pass_of(w, T, i);
    const int o = w.off[k];
    const int64_t nk = w.off[k + 1] - o, j = (int64_t)b * nk + (i - o);
    EventRef r;
    r.ev = w.ev[k] + j * 4;
    r.pol = w.pol[k] + j * 2;
    r.k = k;
    return r;
}


__device__ inline const float* flow_of(const snnflow_iwe_loss_args& a, int b, int t) {
    return a.flows[t] + (int64_t)b * 2 * a.H * a.W;
}
__device__ inline const float* mask_of(const snnflow_iwe_loss_args& a, int b, int t) {
    return a.masks[t] + (int64_t)b * a.H * a.W;
}

// IWE splat with LDS-privatised images over events binned by the band of their warped corners.
// k_iwe_wbin, one block per (sample b, event window k): gathers every event's flow at its pixel,
// warps it to both reference times (warp4: tref = T for direction 0, 0 for direction 1) and files one
// record per (event, direction, band of SB_BAND pixels touched by a corner of non-zero weight) --
// rec = (ts + k, y, x, pol mask 0 | flow y, flow x, pol mask 1, 0), 32 B -- into the (b, k) region of
// the record scratch, direction-major and band by band (a band histogram in LDS, a wave-0 prefix scan,
// the placement; bins [B][T][2 nbands + 1]: each (direction, band)'s start in the region).
// k_iwe_splat, one block per (sample, direction, band): owns the four images (cnt+, cnt-, ts+, ts-) of
// its band in LDS, reads the band's records of the T windows (contiguous, no rescan of the event
// lists: every record is read once), re-warps them (the same warp4 on the same inputs: the same
// corners and weights) and adds the corners inside the band, then writes the band once (no memset, no
// global atomics).  images layout: [dir 2][img 4][B][HW].
// Deterministic accumulation (SNNFLOW_SPLAT_FIXED, default): every corner contribution v is split
// exactly into two 64-bit fixed-point integers, v = H 2^-32 + L 2^-75 (H = rint(v 2^32) in double,
// L = rint((v - H 2^-32) 2^75): exact for |v| >= 2^-51), and the two are added with integer LDS
// atomics.  Integer addition is associative, so the band totals -- the whole IWE -- are the same
// bits on every run whatever order the records' atomics land in, and they are the exact sums of the
// fp32 contributions (rounded once to fp32 at the end).  Two words because the loss reads ratios
// (ts image / count image, loss/flow.py:219-233) that do not shrink with the weights: a pixel hit
// only by a 1e-7 corner still contributes ts^2 to the loss, so the fraction needs relative, not
// absolute, precision.  Range: |sum| < 2^31 per pixel and image.  (0: fp32 LDS atomics,
// order-dependent rounding.)
#ifndef SNNFLOW_SPLAT_FIXED
#define SNNFLOW_SPLAT_FIXED 1
#endif
constexpr bool kSplatFixed = SNNFLOW_SPLAT_FIXED != 0;
constexpr int SPLAT_NT = 1024, SB_BAND = 1024, WB_NT = 1024, WB_U = 2, kMaxSBands = 2048;  // H W <= 2^21 pixels
// the loss backward's bins (k_iwe_bin / k_iwe_wbin, k_iwe_bwd_band): bands of GB_BAND pixels
#ifndef SNNFLOW_GB_BAND
#define SNNFLOW_GB_BAND 512
#endif
#ifndef SNNFLOW_GB_NT
#define SNNFLOW_GB_NT 256
#endif
constexpr int GB_NT = SNNFLOW_GB_NT, BIN_NT = 1024, GB_BAND = SNNFLOW_GB_BAND, kMaxBands = (1 << 21) / GB_BAND;  // H W <= 2^21 pixels

struct SplatLdsF {  // fp32 images
    float v[4][SB_BAND];
    __device__ void zero(int tid) { for (int j = tid; j < 4 * SB_BAND; j += SPLAT_NT) (&v[0][0])[j] = 0.0f; }
    __device__ void add(int q, int i, float x) { atomicAdd(&v[q][i], x); }
    __device__ float get(int q, int i) const { return v[q][i]; }
};
struct SplatLdsX {  // exact two-word fixed point
    unsigned long long hi[4][SB_BAND], lo[4][SB_BAND];
    __device__ void zero(int tid) {
        for (int j = tid; j < 4 * SB_BAND; j += SPLAT_NT) (&hi[0][0])[j] = 0, (&lo[0][0])[j] = 0;
    }
    __device__ void add(int q, int i, float x) {
        // corner weights (x ts) lie in [0, 1]; the clamp keeps any input inside the fixed-point range
        // (|d| < 2^30: rint(d 2^32) fits a 64-bit word with room for 2^31 additions)
        const double d = fmin(fmax((double)x, -0x1p30), 0x1p30);
        const double h = rint(d * 0x1p32);               // exact: x has 24 significant bits
        const double r = d - h * 0x1p-32;                // exact, |r| <= 2^-33
        const long long l = (long long)rint(r * 0x1p75);
        atomicAdd(&hi[q][i], (unsigned long long)(long long)h);
        if (l != 0) atomicAdd(&lo[q][i], (unsigned long long)l);  // zero for every |x| >= 2^-9
    }
    __device__ float get(int q, int i) const {
        return (float)((double)(long long)hi[q][i] * 0x1p-32 + (double)(long long)lo[q][i] * 0x1p-75);
    }
};
typedef std::conditional_t<kSplatFixed, SplatLdsX, SplatLdsF> SplatLds;

// Records per (event, direction) at most: the non-zero corners of a warp lie within 2 W + 2 pixels
// (y1 = floor(wy + 1) may exceed floor(wy) + 1 by one under rounding, likewise x1).
__host__ __device__ inline int splat_rec_per_event(int W) { return (2 * W + 2) / SB_BAND + 2; }
__host__ __device__ inline int splat_bands(int64_t HWp) { return (int)((HWp + SB_BAND - 1) / SB_BAND); }

// The record scratch after the images: [B M R 2] records of 32 B ((b, k) region at R 2 (b M + off[k]))
// and the bin table [B][T][2 nbands + 1] ints.
__host__ __device__ inline int64_t splat_img_floats(int B, int64_t HWp) { return 8 * (int64_t)B * HWp; }
__host__ __device__ inline int64_t splat_rec_floats(int B, int M, int W) { return (int64_t)B * M * splat_rec_per_event(W) * 2 * 8; }

// The loss scratch (snnflow_iwe_scratch_floats), float offsets, each region 16-B aligned: the IWEs, the
// forward's records and bin table, the backward's records (rec4 = (ts + window, y, x, pol mask 0),
// rec1 = pol mask 1) and bin table [B][tf][nbands_g + 1].
struct LossScratch {
    int64_t rec, bins, rec4, rec1, gbins, total;
    __host__ __device__ LossScratch(int B, int M, int T, int tf, int H, int W) {
        const int64_t HWp = (int64_t)H * W;
        auto up4 = [](int64_t x) { return (x + 3) / 4 * 4; };
        rec = splat_img_floats(B, HWp);
        bins = rec + splat_rec_floats(B, M, W);
        rec4 = up4(bins + (int64_t)B * T * (2 * ((HWp + SB_BAND - 1) / SB_BAND) + 1));
        rec1 = rec4 + 4 * (int64_t)B * M;
        gbins = rec1 + (int64_t)B * M;
        total = gbins + (int64_t)B * tf * ((HWp + GB_BAND - 1) / GB_BAND + 1);
    }
};

// The bands (ascending, distinct) that the non-zero corners of one warp touch, as a count and the
// first band; corners are idx-ordered (c0 <= c1 <= c2 <= c3 for in-image corners).
template <typename F>
__device__ inline void corner_bands(const Corner (&c)[4], F&& visit) {
    int prev = -1;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (c[q].wt == 0.0f) continue;
        const int band = c[q].idx / SB_BAND;
        if (band != prev) visit(band);
        prev = band;
    }
}

__global__ __launch_bounds__(WB_NT) void k_iwe_wbin(snnflow_iwe_loss_args a, int nbands, float4* rec, int* bins, int nbg,
                                                     float4* rec4, float* rec1, int* gbins) {
    __shared__ int cnt[2 * kMaxSBands], cur[2 * kMaxSBands];
    __shared__ int gcnt[kMaxBands], gcur[kMaxBands];  // the backward's bins (own-pixel bands; tf == T)
    __shared__ WinTab wt;
    const int tid = threadIdx.x;
    wintab_load(a, wt);
    const int k = blockIdx.x % a.T, b = blockIdx.x / a.T;
    const int i0 = a.off[k], i1 = a.off[k + 1];
    const int64_t HWp = (int64_t)a.H * a.W;
    const int R = splat_rec_per_event(a.W), nb2 = 2 * nbands;
    // with one flow per event window the backward's (sample, flow window) regions are this block's:
    // its bins by the band of the event's own pixel are formed here too (else k_iwe_bin, in the backward)
    const bool gb = a.tf == a.T;
    for (int j = tid; j < nb2; j += WB_NT) cnt[j] = 0;
    if (gb)
        for (int j = tid; j < nbg; j += WB_NT) gcnt[j] = 0;
    __syncthreads();
    const float* fl = wt.fl[a.tf == 1 ? 0 : k] + (int64_t)b * 2 * HWp;
    auto gband = [&](const float4& r0) {
        const int pix = (int)(r0.y * (float)a.W + r0.z);
        const int q = pix / GB_BAND;
        return q < 0 ? 0 : (q >= nbg ? nbg - 1 : q);
    };
    // one event: its record halves and the corners of both warps
    auto warp_event = [&](int i, float4& r0, float4& r1, Corner (&c0)[4], Corner (&c1)[4]) {
        const EventRef r = event_ref(wt, a.T, b, i);
        const float4 ev = *reinterpret_cast<const float4*>(r.ev);
        const float2 pm = *reinterpret_cast<const float2*>(r.pol);
        const int pix = (int)(ev.y * (float)a.W + ev.z);
        const float fy = fl[HWp + pix], fx = fl[pix];
        const float ts = ev.x + (float)k;
        r0 = make_float4(ts, ev.y, ev.z, pm.x);
        r1 = make_float4(fy, fx, pm.y, 0.0f);
        float wy, wx;
        warp4(ts, ev.y, ev.z, fy, fx, (float)a.T, a.flow_scaling, a.H, a.W, c0, wy, wx);
        warp4(ts, ev.y, ev.z, fy, fx, 0.0f, a.flow_scaling, a.H, a.W, c1, wy, wx);
    };
    // the window's first WB_U * WB_NT events stay in registers between the histogram and the placement
    // (their loads and flow gathers issued together: one chain of dependent loads per thread); any
    // further events are loaded again for the placement
    float4 kr0[WB_U], kr1[WB_U];
#pragma unroll
    for (int u = 0; u < WB_U; ++u) {
        const int i = i0 + tid + u * WB_NT;
        kr0[u] = kr1[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (i < i1) {
            const EventRef r = event_ref(wt, a.T, b, i);
            const float4 ev = *reinterpret_cast<const float4*>(r.ev);
            const float2 pm = *reinterpret_cast<const float2*>(r.pol);
            kr0[u] = make_float4(ev.x + (float)k, ev.y, ev.z, pm.x);
            kr1[u] = make_float4(0.f, 0.f, pm.y, 0.f);
        }
    }
#pragma unroll
    for (int u = 0; u < WB_U; ++u) {
        const int i = i0 + tid + u * WB_NT;
        if (i < i1) {
            const int pix = (int)(kr0[u].y * (float)a.W + kr0[u].z);
            kr1[u].x = fl[HWp + pix];
            kr1[u].y = fl[pix];
        }
    }
    auto warps = [&](const float4& r0, const float4& r1, Corner (&c0)[4], Corner (&c1)[4]) {
        float wy, wx;
        warp4(r0.x, r0.y, r0.z, r1.x, r1.y, (float)a.T, a.flow_scaling, a.H, a.W, c0, wy, wx);
        warp4(r0.x, r0.y, r0.z, r1.x, r1.y, 0.0f, a.flow_scaling, a.H, a.W, c1, wy, wx);
    };
#pragma unroll
    for (int u = 0; u < WB_U; ++u) {
        if (i0 + tid + u * WB_NT >= i1) continue;
        Corner c0[4], c1[4];
        warps(kr0[u], kr1[u], c0, c1);
        corner_bands(c0, [&](int band) { atomicAdd(&cnt[band], 1); });
        corner_bands(c1, [&](int band) { atomicAdd(&cnt[nbands + band], 1); });
        if (gb) atomicAdd(&gcnt[gband(kr0[u])], 1);
    }
    for (int i = i0 + tid + WB_U * WB_NT; i < i1; i += WB_NT) {
        float4 r0, r1;
        Corner c0[4], c1[4];
        warp_event(i, r0, r1, c0, c1);
        corner_bands(c0, [&](int band) { atomicAdd(&cnt[band], 1); });
        corner_bands(c1, [&](int band) { atomicAdd(&cnt[nbands + band], 1); });
        if (gb) atomicAdd(&gcnt[gband(r0)], 1);
    }
    __syncthreads();
    int* bo = bins + ((int64_t)b * a.T + k) * (nb2 + 1);
    if (tid < 64) {  // exclusive prefix over (direction, band), 64 at a time
        int carry = 0;
        for (int j0 = 0; j0 < nb2; j0 += 64) {
            const int j = j0 + tid;
            const int c = j < nb2 ? cnt[j] : 0;
            int x = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(x, o, 64);
                if (tid >= o) x += y;
            }
            if (j < nb2) {
                cur[j] = carry + x - c;
                bo[j] = carry + x - c;
            }
            carry += __shfl(x, 63, 64);
        }
        if (tid == 0) bo[nb2] = carry;
    } else if (gb && tid < 128) {  // (wave 1) the same over the own-pixel bands
        const int l = tid - 64;
        int* go = gbins + ((int64_t)b * a.tf + k) * (nbg + 1);
        int carry = 0;
        for (int j0 = 0; j0 < nbg; j0 += 64) {
            const int j = j0 + l;
            const int c = j < nbg ? gcnt[j] : 0;
            int x = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(x, o, 64);
                if (l >= o) x += y;
            }
            if (j < nbg) {
                gcur[j] = carry + x - c;
                go[j] = carry + x - c;
            }
            carry += __shfl(x, 63, 64);
        }
        if (l == 0) go[nbg] = carry;
    }
    __syncthreads();
    float4* rg = rec + (int64_t)R * 2 * ((int64_t)b * a.M + i0) * 2;  // (two float4 per record)
    const int64_t gbase = (int64_t)b * a.M + i0;
    auto gplace = [&](const float4& r0, const float4& r1) {
        if (!gb) return;
        const int slot = atomicAdd(&gcur[gband(r0)], 1);
        rec4[gbase + slot] = r0;
        rec1[gbase + slot] = r1.z;
    };
    auto place = [&](const float4& r0, const float4& r1, const Corner (&c0)[4], const Corner (&c1)[4]) {
        auto put = [&](int j) {
            const int slot = atomicAdd(&cur[j], 1);
            rg[2 * slot] = r0;
            rg[2 * slot + 1] = r1;
        };
        corner_bands(c0, [&](int band) { put(band); });
        corner_bands(c1, [&](int band) { put(nbands + band); });
    };
#pragma unroll
    for (int u = 0; u < WB_U; ++u) {
        if (i0 + tid + u * WB_NT >= i1) continue;
        Corner c0[4], c1[4];
        warps(kr0[u], kr1[u], c0, c1);
        place(kr0[u], kr1[u], c0, c1);
        gplace(kr0[u], kr1[u]);
    }
    for (int i = i0 + tid + WB_U * WB_NT; i < i1; i += WB_NT) {
        float4 r0, r1;
        Corner c0[4], c1[4];
        warp_event(i, r0, r1, c0, c1);
        place(r0, r1, c0, c1);
        gplace(r0, r1);
    }
}

// Device-side argument faults of the loss kernels (snnflow_device_errors): a bin table whose segment
// lies outside its window's record region (a corrupted or stale scratch) is skipped and flagged here
// instead of being read out of bounds.  Bit 1: k_iwe_splat, bit 2: k_iwe_bwd_band.
__device__ unsigned int g_snnflow_dev_err = 0u;

// Test hook (SNNFLOW_FAULT_INJECT=1|2 at library load): overwrite one entry of the forward's (1) or the
// backward's (2) bin table after it is formed, so the checks above can be exercised on the GPU.
__global__ void k_iwe_corrupt_bins(int* bins, int n) {
    if (threadIdx.x == 0 && n > 1) bins[1] = 1 << 28;
}

__global__ __launch_bounds__(SPLAT_NT) void k_iwe_splat(snnflow_iwe_loss_args a, int nbands, const float4* __restrict__ rec,
                                                        const int* __restrict__ bins) {
    __shared__ SplatLds img;
    __shared__ int64_t seg0[SNNFLOW_MAX_WINDOWS];
    __shared__ int pre[SNNFLOW_MAX_WINDOWS + 1];
    const int tid = threadIdx.x;
    const int blk = xcd_block();
    const int band = blk % nbands, d = (blk / nbands) % 2, b = blk / (2 * nbands);
    const int64_t HWp = (int64_t)a.H * a.W, imgsz = (int64_t)a.B * HWp;
    const int p0 = band * SB_BAND;
    const int np = (int)((HWp - p0) < SB_BAND ? (HWp - p0) : SB_BAND);
    const int R = splat_rec_per_event(a.W), nb2 = 2 * nbands, j = d * nbands + band;
    if (tid < 64) {  // the band's segment in every window's region, and their prefix
        int len = 0;
        if (tid < a.T) {
            const int* bo = bins + ((int64_t)b * a.T + tid) * (nb2 + 1);
            int s0 = bo[j];
            len = bo[j + 1] - s0;
            // the segment must lie in the window's region of R * 2 records per event
            const int64_t cap = (int64_t)R * 2 * (a.off[tid + 1] - a.off[tid]);
            if (s0 < 0 || len < 0 || (int64_t)s0 + len > cap) {
                atomicOr(&g_snnflow_dev_err, 1u);
                s0 = 0;
                len = 0;
            }
            seg0[tid] = (int64_t)R * 2 * ((int64_t)b * a.M + a.off[tid]) + s0;  // record index of the segment's start
        }
        int x = len;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (tid >= o) x += y;
        }
        if (tid < a.T) pre[tid + 1] = x;
        if (tid == 0) pre[0] = 0;
    }
    img.zero(tid);
    __syncthreads();
    const int total = pre[a.T];
    const float tref = d == 0 ? (float)a.T : 0.0f;
    for (int f = tid; f < total; f += SPLAT_NT) {
        int lo = 0, hi = a.T - 1;  // the window holding flat record f: last k with pre[k] <= f
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (pre[mid] <= f) lo = mid;
            else hi = mid - 1;
        }
        const int64_t ri = (int64_t)seg0[lo] + (f - pre[lo]);
        const float4 r0 = rec[2 * ri], r1 = rec[2 * ri + 1];
        const float ts = r0.x, pm0 = r0.w, pm1 = r1.z;
        const float tsw = d == 0 ? ts : (float)a.T - ts;
        Corner c[4];
        float wy, wx;
        warp4(ts, r0.y, r0.z, r1.x, r1.y, tref, a.flow_scaling, a.H, a.W, c, wy, wx);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float w = c[q].wt;
            const int li = c[q].idx - p0;
            if (w == 0.0f || li < 0 || li >= np) continue;
            const float wts = w * tsw;
            if (pm0 != 0.0f) {
                img.add(0, li, w * pm0);
                img.add(2, li, wts * pm0);
            }
            if (pm1 != 0.0f) {
                img.add(1, li, w * pm1);
                img.add(3, li, wts * pm1);
            }
        }
    }
    __syncthreads();
    float* out = a.images + (int64_t)d * 4 * imgsz + (int64_t)b * HWp + p0;
#pragma unroll
    for (int q = 0; q < 4; ++q)
        for (int jj = tid; jj < np; jj += SPLAT_NT) out[(int64_t)q * imgsz + jj] = img.get(q, jj);
}

__device__ inline float charb(float d) { return sqrtf(d * d + 1e-6f); }

// Per (sample, range of windows, chunk of NT pixels): IWE loss terms of both directions
// (first-range blocks) + the smoothness terms of the range's windows, reduced per block and
// stored as one row of partial sums acc[block][LOSS_NV] (no atomics; k_iwe_finalize sums rows
// in fixed order).  Row: {S+, S-, nz} x {fw, bw}, then the five smoothness sums.
// The window loop carries the centre pixel of window t+1 (needed by the dt term) into the next
// iteration, so every flow / mask map is read once per pixel instead of twice.
constexpr int LOSS_NV = 11;
#ifndef SNNFLOW_LOSS_MIN_BLOCKS
#define SNNFLOW_LOSS_MIN_BLOCKS 1024  // (2048: +1.7 us over the three kernels, 4096 / 8192: slower still)
#endif
constexpr int LOSS_MIN_BLOCKS = SNNFLOW_LOSS_MIN_BLOCKS;  // split the window loop until the grid has this many blocks

__host__ __device__ inline int loss_chunks(int64_t HWp) { return (int)((HWp + NT - 1) / NT); }
__host__ __device__ inline int loss_tsplit(int B, int64_t HWp, int tf) {
    const int64_t base = (int64_t)B * loss_chunks(HWp);
    const int64_t s = (LOSS_MIN_BLOCKS + base - 1) / base;
    return s < 1 ? 1 : (s > tf ? tf : (int)s);
}

__global__ __launch_bounds__(NT) void k_iwe_loss(snnflow_iwe_loss_args a, int chunks, int tsplit) {
    __shared__ float red[NT / 64][LOSS_NV];
    const int blk = xcd_block();
    const int tid = threadIdx.x, chunk = blk % chunks, tg = (blk / chunks) % tsplit, b = blk / (chunks * tsplit);
    const int64_t HWp = (int64_t)a.H * a.W, img = (int64_t)a.B * HWp;
    float v[LOSS_NV];
#pragma unroll
    for (int j = 0; j < LOSS_NV; ++j) v[j] = 0.0f;
    const int p = chunk * NT + tid;
    if (p < HWp) {
        const int h = p / a.W, w = p - h * a.W;
        const bool right = w + 1 < a.W, down = h + 1 < a.H, up = h >= 1, sm = a.smoothing_mask != 0;
        const int t0 = tg * a.tf / tsplit, t1 = (tg + 1) * a.tf / tsplit;
        // neighbours right, down, down-right, up-right (a neighbour outside the image reads this pixel:
        // address always valid, term skipped), loaded a window ahead of their use
        const int Wd = a.W;
        const int off[4] = {1, Wd, Wd + 1, -Wd + 1};
        const bool ok[4] = {right, down, down && right, up && right};
        auto load_nb = [&](int t, float (&X)[4], float (&Y)[4], float (&M)[4]) {
            const float* fx = flow_of(a, b, t);
            const float* m = mask_of(a, b, t);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int pq = ok[q] ? p + off[q] : p;
                X[q] = fx[pq];
                Y[q] = fx[HWp + pq];
                M[q] = m[pq];
            }
        };
        float X[4], Y[4], M[4];
        load_nb(t0, X, Y, M);
        const float* f0 = flow_of(a, b, t0);
        float cx = f0[p], cy = f0[HWp + p], cm = mask_of(a, b, t0)[p];
        // (the images after the first window's loads are issued: their in-place stores would
        // otherwise hold those loads back)
        if (tg == 0) {
            const float T = (float)a.T;
#pragma unroll
            for (int d = 0; d < 2; ++d) {
                const float* base = a.images + (int64_t)d * 4 * img + (int64_t)b * HWp + p;
                float q4[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) q4[q] = base[q * img];
                const float cp = q4[0], cn = q4[1], tp = q4[2], tn = q4[3];
                const float A = (tp / (cp + 1e-9f)) / T;
                const float Bv = (tn / (cn + 1e-9f)) / T;
                v[3 * d + 0] += A * A;
                v[3 * d + 1] += Bv * Bv;
                v[3 * d + 2] += (cp + cn > 0.0f) ? 1.0f : 0.0f;
            }
        }
        for (int t = t0; t < t1; ++t) {
            float nX[4], nY[4], nM[4];
            const bool more = t + 1 < t1;
            if (more) load_nb(t + 1, nX, nY, nM);
            float nx = 0.0f, ny = 0.0f, nm = 0.0f;
            if (t + 1 < a.tf) {
                const float* f2 = flow_of(a, b, t + 1);
                nx = f2[p];
                ny = f2[HWp + p];
                nm = mask_of(a, b, t + 1)[p];
            }
            // pair ('a' = centre of window t, 'b' = (bx, by, bm)): masked Charbonnier term
            auto term = [&](float bx, float by, float bm) {
                const float dd = (cx - bx) + (cy - by);
                const float c = charb(dd);
                return sm ? (cm * bm) * c : c;
            };
#pragma unroll
            for (int q = 0; q < 4; ++q)  // dx, dy, dxdy_dr, dxdy_ur
                if (ok[q]) v[6 + q] += term(X[q], Y[q], M[q]);
            if (t + 1 < a.tf) {
                if (!a.overwrite_intermediate) v[10] += term(nx, ny, nm);  // dt
                cx = nx;
                cy = ny;
                cm = nm;
            }
            if (more) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    X[q] = nX[q];
                    Y[q] = nY[q];
                    M[q] = nM[q];
                }
            }
        }
    }
    const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
    for (int j = 0; j < LOSS_NV; ++j) {
        const float s = wave_total(v[j]);
        if (lane == 0) red[wv][j] = s;
    }
    __syncthreads();
    if (tid < LOSS_NV) {
        double s = 0.0;
#pragma unroll
        for (int w2 = 0; w2 < NT / 64; ++w2) s += (double)red[w2][tid];
        a.acc[(int64_t)blk * LOSS_NV + tid] = s;
    }
}

// Fixed-order fp64 reduction of the partial rows, then loss = sum_b (S+ + S-)_fw / nz_fw
// + ... (loss/flow.py:219-261) + weight * smoothness.  One block: wave w reduces the rows
// of samples w, w + 16, ... (all 11 columns), then the smoothness sums add up over samples.
constexpr int FIN_NT = 1024;

__global__ __launch_bounds__(FIN_NT) void k_iwe_finalize(snnflow_iwe_loss_args a, int rows_b) {
    __shared__ double outv[6 * 64 + 5];    // B <= 64 (checked by the host)
    __shared__ double smp[64][5];          // per-sample smoothness sums
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // wave w reduces samples w, w + 16, ...: lane-strided rows, all 11 columns at once
    for (int b = wv; b < a.B; b += FIN_NT / 64) {
        double s[LOSS_NV];
#pragma unroll
        for (int j = 0; j < LOSS_NV; ++j) s[j] = 0.0;
        const double* r = a.acc + (int64_t)b * rows_b * LOSS_NV;
#pragma unroll 4
        for (int c = lane; c < rows_b; c += 64) {
#pragma unroll
            for (int j = 0; j < LOSS_NV; ++j) s[j] += r[(int64_t)c * LOSS_NV + j];
        }
#pragma unroll
        for (int j = 0; j < LOSS_NV; ++j) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) s[j] += __shfl_xor(s[j], off, 64);
        }
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < 6; ++j) outv[6 * b + j] = s[j];
#pragma unroll
            for (int j = 0; j < 5; ++j) smp[b][j] = s[6 + j];
        }
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        double t = 0.0;
        for (int b = 0; b < a.B; ++b) t += smp[b][threadIdx.x];
        outv[6 * a.B + threadIdx.x] = t;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    float total = 0.0f;
    for (int d = 0; d < 2; ++d) {
        float dir = 0.0f;
        for (int bb = 0; bb < a.B; ++bb) {
            const float sp = (float)outv[6 * bb + 3 * d], sn = (float)outv[6 * bb + 3 * d + 1];
            const float nz = (float)outv[6 * bb + 3 * d + 2];
            float lb = sp + sn;
            if (a.loss_scaling) lb = lb / nz;
            float* ps = a.persample + ((int64_t)d * a.B + bb) * 4;
            ps[0] = sp; ps[1] = sn; ps[2] = nz; ps[3] = lb;
            dir += lb;
        }
        total += dir;
    }
    const int comps = a.overwrite_intermediate ? 4 : 5;
    float sm = (float)outv[6 * a.B + 0];
    for (int j = 1; j < comps; ++j) sm += (float)outv[6 * a.B + j];
    sm = sm / (float)comps / (float)a.tf;
    for (int j = 0; j < 5; ++j) a.smooth[j] = (float)outv[6 * a.B + j];
    a.smooth[5] = sm;
    a.loss[0] = total + a.weight * sm;
}

// dL/d(images) at one pixel of one direction (loss/flow.py:219-261 differentiated): (d/dcnt+, d/dcnt-,
// d/dts+, d/dts-) from the pixel's four IWE values, its sample's loss row (nz, loss_b) and the loss
// gradient g.  Formed where it is gathered (k_iwe_bwd_band: at the events' warped corners), so no
// per-pixel image-gradient pass and no buffer.
__device__ inline float4 img_grad(const float* __restrict__ im, int64_t img, int64_t id, float g, float gS, float nz,
                                  float lb, float T, bool loss_scaling) {
    const float cp = im[id], cn = im[img + id], tp = im[2 * img + id], tn = im[3 * img + id];
    const float dp = cp + 1e-9f, dn = cn + 1e-9f;
    const float qp = tp / dp, qn = tn / dn;
    const float Ap = qp / T, An = qn / T;
    const float gqp = ((2.0f * Ap) * gS) / T, gqn = ((2.0f * An) * gS) / T;
    float gcp = -gqp * (qp / dp), gcn = -gqn * (qn / dn);
    if (loss_scaling && !(cp + cn > 0.0f)) {
        const float gz = -(lb / nz) * g;  // d(sum/nz)/dnz on pixels the nonzero mask did not overwrite
        gcp += gz;
        gcn += gz;
    }
    return make_float4(gcp, gcn, gqp / dp, gqn / dn);
}

// Eight lanes per event in the per-event backward (k_iwe_bwd_band), one per (direction d, corner q): the
// event / flow loads are shared (same addresses), each lane gathers its corner's four image gradients,
// the corners are summed by lane exchange before the (flow_scaling, dt) factor of their direction, the
// directions after it.  (One thread per event left ~5 waves per CU with a chain of 2 x 16
// dependent-address gathers each: latency-bound.)
constexpr int kBwdLanes = 8;

// The events of every (sample, flow window) binned by the pixel band (GB_BAND pixels) of the event's own
// pixel -- the pixel its flow gradient lands in.  The binning depends on the event lists only.  Each
// event is copied into its bin as a record: rec4 = (ts + window, y, x, polarity mask 0) and rec1 =
// polarity mask 1, so that a band's block reads its events contiguously with no index indirection.
// The region of flow window t (events [i0, i1) of the concatenation: window t, or all of them when
// tf == 1) is [b M + i0, b M + i1) of rec4 / rec1, band by band; bins [B][tf][nbands + 1]: each band's
// start in that region (the last entry: the window's count).  The order inside a band follows the LDS
// atomics (it does not matter: the consumer sums in exact fixed point).  One block per (sample, flow
// window): a band histogram, a wave-0 prefix scan, the placement.

__device__ inline void flow_window_events(const snnflow_iwe_loss_args& a, int t, int& i0, int& i1) {
    i0 = a.tf == 1 ? 0 : a.off[t];
    i1 = a.tf == 1 ? a.M : a.off[t + 1];
}

__global__ __launch_bounds__(BIN_NT) void k_iwe_bin(snnflow_iwe_loss_args a, int nbands, float4* rec4, float* rec1,
                                                    int* bins) {
    __shared__ int cnt[kMaxBands], cur[kMaxBands];
    __shared__ WinTab wt;
    const int tid = threadIdx.x;
    wintab_load(a, wt);
    const int t = blockIdx.x % a.tf, b = blockIdx.x / a.tf;
    int i0, i1;
    flow_window_events(a, t, i0, i1);
    for (int k = tid; k < nbands; k += BIN_NT) cnt[k] = 0;
    __syncthreads();
    auto band_of = [&](const float* ev) {
        const int pix = (int)(ev[1] * (float)a.W + ev[2]);
        const int k = pix / GB_BAND;
        return k < 0 ? 0 : (k >= nbands ? nbands - 1 : k);
    };
    for (int i = i0 + tid; i < i1; i += BIN_NT) atomicAdd(&cnt[band_of(event_ref(wt, a.T, b, i).ev)], 1);
    __syncthreads();
    int* bo = bins + ((int64_t)b * a.tf + t) * (nbands + 1);
    if (tid < 64) {  // exclusive prefix over the bands, 64 at a time
        int carry = 0;
        for (int k0 = 0; k0 < nbands; k0 += 64) {
            const int k = k0 + tid;
            const int c = k < nbands ? cnt[k] : 0;
            int x = c;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(x, o, 64);
                if (tid >= o) x += y;
            }
            if (k < nbands) {
                cur[k] = carry + x - c;
                bo[k] = carry + x - c;
            }
            carry += __shfl(x, 63, 64);
        }
        if (tid == 0) bo[nbands] = carry;
    }
    __syncthreads();
    const int64_t base = (int64_t)b * a.M + i0;
    for (int i = i0 + tid; i < i1; i += BIN_NT) {
        const EventRef r = event_ref(wt, a.T, b, i);
        const float4 ev = *reinterpret_cast<const float4*>(r.ev);
        const float2 pm = *reinterpret_cast<const float2*>(r.pol);
        const int slot = atomicAdd(&cur[band_of(r.ev)], 1);
        rec4[base + slot] = make_float4(ev.x + (float)r.k, ev.y, ev.z, pm.x);
        rec1[base + slot] = pm.y;
    }
}

// dL/dflow of one (sample, flow window t, band of GB_BAND pixels), written once:
//  * the smoothness part (loss/flow.py:263-303 differentiated): per pixel the 8 neighbour pairs of
//    window t (the flow / mask values of the band and its neighbour rows, [p0 - W - 1, p0 + GB_BAND + W
//    + 1), staged in LDS by coalesced loads) and the dt pairs (t-1, t), (t, t+1) (centres straight from
//    memory; each pair's term is the one its other window computes, the same floats);
//  * the events' part: each event of the band's bin (events binned by the band of their own pixel --
//    the pixel their flow gradient lands in) forms dL/d(images) at the 4 corners of both warps from the
//    IWE values there (img_grad) and
//    chains them through the bilinear weights to its flow (eight lanes per event, kBwdLanes); the
//    band's per-pixel sums of those are formed in LDS in exact two-word fixed point (integer adds: the
//    sums do not depend on the order of the events; SplatLdsX's split).  No block reads an event
//    outside its bin.
//  g_flows = smoothness + the event sum (where a pixel has events), the same floats as a separate
//  smoothness pass followed by adding the sums.  Dynamic LDS: 3 (GB_BAND + 2 W + 2) floats.
struct GevLds {
    unsigned long long hi[2][GB_BAND], lo[2][GB_BAND];
};
__host__ __device__ inline int gb_stage_floats(int W) { return 3 * (GB_BAND + 2 * W + 2); }

__global__ __launch_bounds__(GB_NT) void k_iwe_bwd_band(snnflow_iwe_loss_args a, const float* g_loss, float* g_flows,
                                                        const float4* __restrict__ rec4, const float* __restrict__ rec1,
                                                        const int* __restrict__ bins, int nbands, int has_events) {
    __shared__ GevLds acc;
    extern __shared__ float nbs[];  // [3][S]: flow x, flow y, mask of window t around the band
    const int tid = threadIdx.x;
    const int blk = xcd_block();  // a sample's windows and bands on one XCD: its flows / image gradients in one L2
    const int band = blk % nbands, rest = blk / nbands, t = rest % a.tf, b = rest / a.tf;
    const int64_t HWp = (int64_t)a.H * a.W, img = (int64_t)a.B * HWp;
    const int p0 = band * GB_BAND;
    const int np = (int)((HWp - p0) < GB_BAND ? (HWp - p0) : GB_BAND);
    const int S = GB_BAND + 2 * a.W + 2, lo = p0 - a.W - 1;
    float* const sx = nbs;
    float* const sy = nbs + S;
    float* const smk = nbs + 2 * S;
    // smoothness inputs: window t around the band (LDS), the centres of windows t-1 and t+1 (registers)
    constexpr int PPT = GB_BAND / GB_NT;  // band pixels per thread
    const bool sm = a.smoothing_mask != 0, dt_terms = !a.overwrite_intermediate;
    const float* f1 = flow_of(a, b, t);
    const float* m1 = mask_of(a, b, t);
    for (int e = tid; e < S; e += GB_NT) {
        const int64_t q = (int64_t)lo + e;
        const bool in = q >= 0 && q < HWp;
        sx[e] = in ? f1[q] : 0.0f;
        sy[e] = in ? f1[HWp + q] : 0.0f;
        smk[e] = in ? m1[q] : 0.0f;
    }
    float px_[PPT], py_[PPT], pm_[PPT], nx_[PPT], ny_[PPT], nm_[PPT];
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
        const int j = tid + k * GB_NT;
        const int64_t p = p0 + j;
        px_[k] = py_[k] = pm_[k] = nx_[k] = ny_[k] = nm_[k] = 0.0f;
        if (j < np && dt_terms && t >= 1) {
            const float* fp = flow_of(a, b, t - 1);
            px_[k] = fp[p];
            py_[k] = fp[HWp + p];
            pm_[k] = mask_of(a, b, t - 1)[p];
        }
        if (j < np && dt_terms && t + 1 < a.tf) {
            const float* fn = flow_of(a, b, t + 1);
            nx_[k] = fn[p];
            ny_[k] = fn[HWp + p];
            nm_[k] = mask_of(a, b, t + 1)[p];
        }
    }
    int e0 = 0, e1 = 0;
    int64_t base = 0;
    if (has_events) {
        const int* bo = bins + ((int64_t)b * a.tf + t) * (nbands + 1);
        int i0, i1;
        flow_window_events(a, t, i0, i1);
        e0 = bo[band];
        e1 = bo[band + 1];
        base = (int64_t)b * a.M + i0;
        if (e0 < 0 || e1 < e0 || e1 > i1 - i0) {  // the bin must lie in the window's records
            if (tid == 0) atomicOr(&g_snnflow_dev_err, 2u);
            e0 = e1 = 0;
        }
    }
    for (int j = tid; j < 2 * GB_BAND; j += GB_NT) (&acc.hi[0][0])[j] = 0, (&acc.lo[0][0])[j] = 0;
    const float* fl = a.flows[a.tf == 1 ? 0 : t] + (int64_t)b * 2 * HWp;
    __syncthreads();
    // the smoothness gradient of this thread's pixels (the sum order of the per-pixel form: the 8
    // neighbours -- right, left, down, up, down-right, up-left, up-right, down-left; odd q: this pixel
    // is the pair's 'b' -- then +(t, t+1), then -(t-1, t))
    float smooth[PPT];
    {
        const float g = g_loss[0];
        const int comps = a.overwrite_intermediate ? 4 : 5;
        const float gsm = ((g * a.weight) / (float)comps) / (float)a.tf;
        // d(term)/d(flow of 'a') for the pair ('a', 'b'); 'b' receives the negative
        auto pg = [&](float ax, float ay, float am, float bx, float by, float bm) {
            const float dd = (ax - bx) + (ay - by);
            const float c = charb(dd);
            const float mk = sm ? am * bm : 1.0f;
            return ((mk * gsm) / (2.0f * c)) * (2.0f * dd);
        };
        const int Wd = a.W;
        const int off[8] = {1, -1, Wd, -Wd, Wd + 1, -Wd - 1, -Wd + 1, Wd - 1};
#pragma unroll
        for (int k = 0; k < PPT; ++k) {
            const int j = tid + k * GB_NT;
            const int p = p0 + (j < np ? j : 0);
            const int h = p / a.W, w = p - h * a.W;
            const bool vr = w + 1 < a.W, vl = w >= 1, vd = h + 1 < a.H, vu = h >= 1;
            const bool ok[8] = {vr, vl, vd, vu, vd && vr, vu && vl, vu && vr, vd && vl};
            const int c0 = p - lo;
            const float cx = sx[c0], cy = sy[c0], cm = smk[c0];
            float v = 0.0f;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                if (!ok[q]) continue;
                const int e = c0 + off[q];
                if (q % 2 == 0) v += pg(cx, cy, cm, sx[e], sy[e], smk[e]);
                else v -= pg(sx[e], sy[e], smk[e], cx, cy, cm);
            }
            if (t + 1 < a.tf && dt_terms) v += pg(cx, cy, cm, nx_[k], ny_[k], nm_[k]);
            if (dt_terms && t >= 1) v -= pg(px_[k], py_[k], pm_[k], cx, cy, cm);
            smooth[k] = v;
        }
    }
    const int sub = tid & (kBwdLanes - 1), d = sub >> 2, qc = sub & 3;
    const float tref = d == 0 ? (float)a.T : 0.0f;
    const float* im = a.images + (int64_t)d * 4 * img + (int64_t)b * HWp;
    const float gl = g_loss[0];
    const float* ps = a.persample + ((int64_t)d * a.B + b) * 4;
    const float nz = ps[2], lb = ps[3];
    const float gS = a.loss_scaling ? gl / nz : gl;
    const bool lsc = a.loss_scaling != 0;
    // every lane runs every round (the lane exchanges need the whole 8-lane group): a slot past the bin
    // contributes zeros
    for (int s0 = e0; s0 < e1; s0 += GB_NT / kBwdLanes) {
        const int slot = s0 + tid / kBwdLanes;
        const bool on = slot < e1;
        float gwy = 0.0f, gwx = 0.0f, dt = 0.0f;
        int q = -1;
        if (on) {
            const float4 ev = rec4[base + slot];
            const float pm1 = rec1[base + slot];
            const float ts = ev.x, y = ev.y, x = ev.z, pm0 = ev.w;
            const int pix = (int)(y * (float)a.W + x);
            q = pix - p0;
            const float fy = fl[HWp + pix], fx = fl[pix];
            const float tsw = d == 0 ? ts : (float)a.T - ts;
            Corner c[4];
            float wy, wx;
            warp4(ts, y, x, fy, fx, tref, a.flow_scaling, a.H, a.W, c, wy, wx);
            Corner cq = c[0];
#pragma unroll
            for (int k = 1; k < 4; ++k)
                if (qc == k) cq = c[k];
            if (cq.inb) {
                const float4 G = img_grad(im, img, cq.idx, gl, gS, nz, lb, (float)a.T, lsc);
                const float gwt = (G.x * pm0 + G.y * pm1) + (G.z * (tsw * pm0) + G.w * (tsw * pm1));
                // wt = ay * ax * mask: d/day = ax, d/dax = ay; ay = max(0, 1 - |dy|)
                const float gay = gwt * cq.ax, gax = gwt * cq.ay;
                gwy = -(gay * relu_tie(1.0f - fabsf(cq.dy))) * sgnf(cq.dy);
                gwx = -(gax * relu_tie(1.0f - fabsf(cq.dx))) * sgnf(cq.dx);
            }
            dt = tref - ts;
        }
        gwy += __shfl_xor(gwy, 1, 64);
        gwx += __shfl_xor(gwx, 1, 64);
        gwy += __shfl_xor(gwy, 2, 64);
        gwx += __shfl_xor(gwx, 2, 64);
        float gfy = (gwy * a.flow_scaling) * dt, gfx = (gwx * a.flow_scaling) * dt;
        gfy += __shfl_xor(gfy, 4, 64);
        gfx += __shfl_xor(gfx, 4, 64);
        if (on && sub < 2 && q >= 0 && q < np) {  // lane 0: the x component, lane 1: y
            // clamped to |v| <= 2^30 (a per-event flow gradient beyond that is not a number this sum can
            // carry exactly in 64 bits: rint(v 2^32) must leave room for the pixel's other events)
            const double v = fmin(fmax((double)(sub == 0 ? gfx : gfy), -0x1p30), 0x1p30);
            if (v != 0.0) {
                const double h = rint(v * 0x1p32);
                const long long l = (long long)rint((v - h * 0x1p-32) * 0x1p75);
                atomicAdd(&acc.hi[sub][q], (unsigned long long)(long long)h);
                if (l != 0) atomicAdd(&acc.lo[sub][q], (unsigned long long)l);
            }
        }
    }
    __syncthreads();
    float* gf = g_flows + (((int64_t)b * a.tf + t) * 2) * HWp + p0;
#pragma unroll
    for (int k = 0; k < PPT; ++k) {
        const int q = tid + k * GB_NT;
        if (q >= np) continue;
#pragma unroll
        for (int c = 0; c < 2; ++c) {  // plane 0: x, 1: y
            const unsigned long long h = acc.hi[c][q], l = acc.lo[c][q];
            gf[c * HWp + q] =
                (h | l) ? smooth[k] + (float)((double)(long long)h * 0x1p-32 + (double)(long long)l * 0x1p-75) : smooth[k];
        }
    }
}

__global__ void k_iwe_corners(const float* __restrict__ events, const float* __restrict__ flow_ev, int B, int M,
                              float tref, int H, int W, float s, int round_idx, int32_t* idx, float* wout) {
    const int64_t n = (int64_t)B * M;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        const int b = (int)(e / M), i = (int)(e - (int64_t)b * M);
        const float* ev = events + e * 4;
        const float fy = flow_ev[e * 2], fx = flow_ev[e * 2 + 1];
        if (round_idx) {
            const float dt = tref - ev[0];
            const float wy = ev[1] + (dt * fy) * s, wx = ev[2] + (dt * fx) * s;
            const float cy = rintf(wy), cx = rintf(wx);
            const bool inb = cy >= 0.0f && cy < (float)H && cx >= 0.0f && cx < (float)W;
            const float m = inb ? 1.0f : 0.0f;
            idx[(int64_t)b * M + i] = (int)((cy * m) * (float)W + cx * m);
            wout[(int64_t)b * M + i] = 1.0f * m;
        } else {
            Corner c[4];
            float wy, wx;
            warp4(ev[0], ev[1], ev[2], fy, fx, tref, s, H, W, c, wy, wx);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                idx[(int64_t)b * 4 * M + (int64_t)q * M + i] = c[q].idx;
                wout[(int64_t)b * 4 * M + (int64_t)q * M + i] = c[q].wt;
            }
        }
    }
}

__global__ void k_iwe_interpolate(const int32_t* __restrict__ idx, const float* __restrict__ w,
                                  const float* __restrict__ pol, int64_t pol_sb, int B, int K, int HW, float* img) {
    const int64_t n = (int64_t)B * K;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        const int b = (int)(e / K), i = (int)(e - (int64_t)b * K);
        float v = w[e];
        if (pol) v = v * pol[(int64_t)b * pol_sb + i];
        if (v != 0.0f) atomicAdd(img + (int64_t)b * HW + idx[e], v);
    }
}

// Backward of get_interpolation (utils/iwe.py:37-65) w.r.t. the per-event flow: the gradients
// of the 4 corner weights [B][4][M] -> dL/dflow_ev [B][M][2] (y, x).  weights = prod(max(0,
// 1 - |w - c|), -1) * mask, w = pos + ((tref - ts) * f) * s: the same chain as k_iwe_bwd_band.
__global__ void k_iwe_corners_bwd(const float* __restrict__ events, const float* __restrict__ flow_ev, int B, int M,
                                  float tref, int H, int W, float s, const float* __restrict__ g_w,
                                  float* __restrict__ g_flow_ev) {
    const int64_t n = (int64_t)B * M;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        const int b = (int)(e / M), i = (int)(e - (int64_t)b * M);
        const float* ev = events + e * 4;
        Corner c[4];
        float wy, wx;
        warp4(ev[0], ev[1], ev[2], flow_ev[e * 2], flow_ev[e * 2 + 1], tref, s, H, W, c, wy, wx);
        float gwy = 0.0f, gwx = 0.0f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const float gwt = c[q].inb ? g_w[(int64_t)b * 4 * M + (int64_t)q * M + i] : 0.0f;
            const float gay = gwt * c[q].ax, gax = gwt * c[q].ay;
            gwy += -(gay * relu_tie(1.0f - fabsf(c[q].dy))) * sgnf(c[q].dy);
            gwx += -(gax * relu_tie(1.0f - fabsf(c[q].dx))) * sgnf(c[q].dx);
        }
        const float dt = tref - ev[0];
        g_flow_ev[e * 2] = (gwy * s) * dt;
        g_flow_ev[e * 2 + 1] = (gwx * s) * dt;
    }
}

// Backward of interpolate (utils/iwe.py:84-92): scatter_add_ backward is a gather,
// dL/dweights[e] = dL/dimg[b, idx[e]] * polarity_mask[e].
__global__ void k_iwe_interpolate_bwd(const int32_t* __restrict__ idx, const float* __restrict__ pol, int64_t pol_sb,
                                      int B, int K, int HW, const float* __restrict__ g_img, float* __restrict__ g_w) {
    const int64_t n = (int64_t)B * K;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
        const int b = (int)(e / K), i = (int)(e - (int64_t)b * K);
        const float g = g_img[(int64_t)b * HW + idx[e]];
        g_w[e] = pol ? g * pol[(int64_t)b * pol_sb + i] : g;
    }
}

int grid_for(int64_t n, int per_block, int cap) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

int check_loss_args(const snnflow_iwe_loss_args* a) {
    if (!a || a->B <= 0 || a->B > 64 || a->M < 0 || a->T <= 0 || a->T > SNNFLOW_MAX_WINDOWS || a->H <= 0 ||
        a->W <= 0 || !(a->tf == 1 || a->tf == a->T))
        SNN_FAIL(SNNFLOW_E_ARG, "iwe_loss: bad shape (B <= 64, T <= 64, tf in {1, T})");
    if (!a->images || !a->acc || !a->persample || !a->smooth || !a->loss)
        SNN_FAIL(SNNFLOW_E_ARG, "iwe_loss: missing buffer");
    for (int k = 0; k < a->T; ++k)
        if (!a->events[k] || !a->pol[k]) SNN_FAIL(SNNFLOW_E_ARG, "iwe_loss: missing event window");
    for (int t = 0; t < a->tf; ++t)
        if (!a->flows[t] || !a->masks[t]) SNN_FAIL(SNNFLOW_E_ARG, "iwe_loss: missing flow / mask window");
    if (a->off[0] != 0 || a->off[a->T] != a->M) SNN_FAIL(SNNFLOW_E_ARG, "iwe_loss: offsets must span [0, M]");
    for (int k = 0; k < a->T; ++k)
        if (a->off[k + 1] < a->off[k]) SNN_FAIL(SNNFLOW_E_ARG, "iwe_loss: offsets must be non-decreasing");
    return 0;
}

}  // namespace

extern "C" {

int64_t snnflow_iwe_scratch_floats(int B, int M, int T, int tf, int H, int W) {
    return LossScratch(B, M, T, tf, H, W).total;
}

static int fault_inject_env() {
    const char* v = getenv("SNNFLOW_FAULT_INJECT");
    return v ? atoi(v) : 0;
}
static const int g_fault_inject = fault_inject_env();

int snnflow_device_errors(int clear) {
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return snnflow_set_error((int)e, hipGetErrorString(e));
    unsigned v = 0u;
    e = hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_snnflow_dev_err), sizeof(v), 0, hipMemcpyDeviceToHost);
    if (e == hipSuccess && clear) {
        const unsigned z = 0u;
        e = hipMemcpyToSymbol(HIP_SYMBOL(g_snnflow_dev_err), &z, sizeof(z), 0, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) return snnflow_set_error((int)e, hipGetErrorString(e));
    return (int)v;
}

int snnflow_iwe_acc_doubles(int B, int H, int W, int tf) {
    const int64_t HWp = (int64_t)H * W;
    return (int)((int64_t)B * loss_tsplit(B, HWp, tf) * loss_chunks(HWp) * LOSS_NV);
}

int snnflow_iwe_loss_fwd(const snnflow_iwe_loss_args* a, void* stream) {
    if (int rc = check_loss_args(a)) return rc;
    const hipStream_t s = (hipStream_t)stream;
    const int64_t HWp = (int64_t)a->H * a->W;
    const int nbands = splat_bands(HWp), nbg = (int)((HWp + GB_BAND - 1) / GB_BAND);
    if (nbands > kMaxSBands || nbg > kMaxBands) SNN_FAIL(SNNFLOW_E_ARG, "iwe_loss: H * W above 2^21 pixels");
    if ((reinterpret_cast<uintptr_t>(a->images) & 15) != 0) SNN_FAIL(SNNFLOW_E_ARG, "iwe_loss: images scratch not 16-B aligned");
    const LossScratch ls(a->B, a->M, a->T, a->tf, a->H, a->W);
    float4* rec = reinterpret_cast<float4*>(a->images + ls.rec);
    int* bins = reinterpret_cast<int*>(a->images + ls.bins);
    hipLaunchKernelGGL(k_iwe_wbin, dim3(a->B * a->T), dim3(WB_NT), 0, s, *a, nbands, rec, bins, nbg,
                       reinterpret_cast<float4*>(a->images + ls.rec4), a->images + ls.rec1,
                       reinterpret_cast<int*>(a->images + ls.gbins));
    if (g_fault_inject == 1) hipLaunchKernelGGL(k_iwe_corrupt_bins, dim3(1), dim3(64), 0, s, bins, 2 * nbands + 1);
    hipLaunchKernelGGL(k_iwe_splat, dim3(a->B * 2 * nbands), dim3(SPLAT_NT), 0, s, *a, nbands, rec, bins);
    const int chunks = loss_chunks(HWp), tsplit = loss_tsplit(a->B, HWp, a->tf);
    hipLaunchKernelGGL(k_iwe_loss, dim3(a->B * tsplit * chunks), dim3(NT), 0, s, *a, chunks, tsplit);
    hipLaunchKernelGGL(k_iwe_finalize, dim3(1), dim3(FIN_NT), 0, s, *a, tsplit * chunks);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_iwe_loss_bwd(const snnflow_iwe_loss_args* a, const float* g_loss, float* g_flows, void* stream) {
    if (int rc = check_loss_args(a)) return rc;
    if (!g_loss || !g_flows) SNN_FAIL(SNNFLOW_E_ARG, "iwe_loss_bwd: missing buffer");
    const hipStream_t s = (hipStream_t)stream;
    const int64_t HWp = (int64_t)a->H * a->W;
    // the events binned by own-pixel band (tf == T: the forward's k_iwe_wbin formed these bins), then per
    // band: the smoothness gradient + the events' gradients summed per pixel in exact fixed point
    const int nbands = (int)((HWp + GB_BAND - 1) / GB_BAND);
    if (nbands > kMaxBands) SNN_FAIL(SNNFLOW_E_ARG, "iwe_loss_bwd: H * W above 2^21 pixels");
    const size_t gb_lds = (size_t)gb_stage_floats(a->W) * sizeof(float);
    if (gb_lds > 48 * 1024) SNN_FAIL(SNNFLOW_E_ARG, "iwe_loss_bwd: W above 1791 pixels");
    const LossScratch ls(a->B, a->M, a->T, a->tf, a->H, a->W);
    float4* rec4 = reinterpret_cast<float4*>(a->images + ls.rec4);
    float* rec1 = a->images + ls.rec1;
    int* bins = reinterpret_cast<int*>(a->images + ls.gbins);
    if (a->M > 0 && a->tf != a->T)
        hipLaunchKernelGGL(k_iwe_bin, dim3(a->B * a->tf), dim3(BIN_NT), 0, s, *a, nbands, rec4, rec1, bins);
    if (g_fault_inject == 2 && a->M > 0) hipLaunchKernelGGL(k_iwe_corrupt_bins, dim3(1), dim3(64), 0, s, bins, nbands + 1);
    hipLaunchKernelGGL(k_iwe_bwd_band, dim3(a->B * a->tf * nbands), dim3(GB_NT), gb_lds, s, *a, g_loss, g_flows,
                       rec4, rec1, bins, nbands, a->M > 0 ? 1 : 0);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_iwe_corners(const float* events, const float* flow_ev, int B, int M, float tref, int H, int W,
                        float flow_scaling, int round_idx, int32_t* idx, float* w, void* stream) {
    if (!events || !flow_ev || !idx || !w || B <= 0 || M < 0 || H <= 0 || W <= 0)
        SNN_FAIL(SNNFLOW_E_ARG, "iwe_corners: bad args");
    if (M == 0) return 0;
    hipLaunchKernelGGL(k_iwe_corners, dim3(grid_for((int64_t)B * M, 256, 4096)), dim3(256), 0, (hipStream_t)stream,
                       events, flow_ev, B, M, tref, H, W, flow_scaling, round_idx, idx, w);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_iwe_interpolate(const int32_t* idx, const float* w, const float* pol, int64_t pol_sb, int B, int K, int H,
                            int W, float* img, void* stream) {
    if (!idx || !w || !img || B <= 0 || K < 0 || H <= 0 || W <= 0) SNN_FAIL(SNNFLOW_E_ARG, "iwe_interpolate: bad args");
    const hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(img, 0, sizeof(float) * (size_t)B * H * W, s);
    if (e != hipSuccess) SNN_FAIL((int)e, hipGetErrorString(e));
    if (K == 0) return 0;
    hipLaunchKernelGGL(k_iwe_interpolate, dim3(grid_for((int64_t)B * K, 256, 4096)), dim3(256), 0, s, idx, w, pol,
                       pol_sb, B, K, H * W, img);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_iwe_corners_bwd(const float* events, const float* flow_ev, int B, int M, float tref, int H, int W,
                            float flow_scaling, const float* g_w, float* g_flow_ev, void* stream) {
    if (!events || !flow_ev || !g_w || !g_flow_ev || B <= 0 || M < 0 || H <= 0 || W <= 0)
        SNN_FAIL(SNNFLOW_E_ARG, "iwe_corners_bwd: bad args");
    if (M == 0) return 0;
    hipLaunchKernelGGL(k_iwe_corners_bwd, dim3(grid_for((int64_t)B * M, 256, 4096)), dim3(256), 0,
                       (hipStream_t)stream, events, flow_ev, B, M, tref, H, W, flow_scaling, g_w, g_flow_ev);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_iwe_interpolate_bwd(const int32_t* idx, const float* pol, int64_t pol_sb, int B, int K, int H, int W,
                                const float* g_img, float* g_w, void* stream) {
    if (!idx || !g_img || !g_w || B <= 0 || K < 0 || H <= 0 || W <= 0)
        SNN_FAIL(SNNFLOW_E_ARG, "iwe_interpolate_bwd: bad args");
    if (K == 0) return 0;
    hipLaunchKernelGGL(k_iwe_interpolate_bwd, dim3(grid_for((int64_t)B * K, 256, 4096)), dim3(256), 0,
                       (hipStream_t)stream, idx, pol, pol_sb, B, K, H * W, g_img, g_w);
    SNN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
