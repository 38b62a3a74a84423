// ConvLIF / ConvLIFRecurrent cells (the U-Net neuron flavour) for gfx950: one kernel per
// cell and time step in each direction.
//
// Reference semantics (restated in oracle/lif_ref.py SpikingCellRef, pinned by the
// reference-generated tests/golden/spiking_cells_case.npz):
//   models/spiking_submodules.py:121-151  ConvLIF.forward (stride 1, no norm)
//   models/spiking_submodules.py:265-300  ConvLIFRecurrent.forward (rec conv of z before detach)
//   models/spiking_util.py:82-109         ArctanSpike: fwd (x > 0), bwd g / (1 + width*x*x)
//
// Forward: conv of the input halo (+ conv of the previous spikes) from LDS, then the
// membrane update and spike per pixel; writes state (v_out, z_out), the spikes (+ residual)
// and the current I = ff (+ rec) for the backward pass.
// Backward: dL/dI on the halo from (g_out, g_state, v_out) -> dgrad of both convolutions,
// dL/dv_prev per pixel, threshold / leak sums (fp64 atomics, sharded), dL/dI written for the
// deferred weight gradient (snnflow_wgrad with stats = NULL).
#include <cmath>

#include "snnflow_dev.h"
#include "snnflow_tile.h"

using namespace snnflow;

int snnflow_set_error(int code, const char* msg);
#define SNN_FAIL(code, msg) return snnflow_set_error((code), (msg))
#define SNN_CHECK_LAUNCH()                                                        \
    do {                                                                          \
        hipError_t e_ = hipGetLastError();                                        \
        if (e_ != hipSuccess) return snnflow_set_error((int)e_, hipGetErrorString(e_)); \
    } while (0)

namespace {

// Per-channel constants: leak = sigmoid(leak_raw) (torch: 1 / (1 + exp(-x))),
// th = clamp_min(thresh, 0.01).
struct CellCoef { float leak, th; };

__device__ inline CellCoef cell_coef(const snnflow_convlif_params& p, int c) {
    CellCoef k;
    k.leak = 1.0f / (1.0f + expf(-p.leak[c]));
    const float t = p.thresh[c];
    k.th = t < 0.01f ? 0.01f : t;
    return k;
}

// v_out of one element (evaluation order of the reference expression)
__device__ inline float membrane(float v, float z, float I, const CellCoef& k, bool hard) {
    if (hard) return ((v * k.leak) * (1.0f - z)) + ((1.0f - k.leak) * I);
    return ((v * k.leak) + ((1.0f - k.leak) * I)) - (z * k.th);
}

template <int CIN, int C, bool REC, int SPLIT>
__global__ __launch_bounds__(NT * SPLIT) void k_convlif_fwd(snnflow_convlif_fwd_args a) {
    constexpr int NTB = NT * SPLIT, CO = C / SPLIT;
    constexpr int PI_ = Pad<CIN>::v, PC = Pad<C>::v;
    __shared__ __attribute__((aligned(16))) float tile[HN * PI_];
    __shared__ __attribute__((aligned(16))) float rtile[REC ? HN * PC : 4];
    __shared__ CellCoef coef[C];

    const int tid = threadIdx.x, pt = tid % NT, ty = pt / TW, tx = pt - ty * TW;
    const int part = thread_part(), co0 = part * CO;
    const int H = a.H, W = a.W;
    const Tile tl = block_tile(H, W);
    const int64_t plane = (int64_t)a.B * H * W * C;
    if (tid < C) coef[tid] = cell_coef(a.p, tid);
    stage_strided<CIN, NTB>(a.x, a.xs_b, a.xs_c, a.xs_h, a.xs_w, tl, H, W, tile);
    const bool has_rec = REC && a.prev_state != nullptr;
    if constexpr (REC) {
        if (has_rec) stage_nhwc<C, NTB>(a.prev_state + plane, tl, H, W, rtile);
    }
    __syncthreads();

    float I[CO];
#pragma unroll
    for (int co = 0; co < CO; ++co) I[co] = 0.0f;
    conv_acc<CIN, C, CO>(tile, a.wt_ff, ty, tx, co0, I);
    if constexpr (REC) {
        if (has_rec) {
            float r[CO];
#pragma unroll
            for (int co = 0; co < CO; ++co) r[co] = 0.0f;
            conv_acc<C, C, CO>(rtile, a.wt_rec, ty, tx, co0, r);
#pragma unroll
            for (int co = 0; co < CO; ++co) I[co] = I[co] + r[co];  // ff + rec (:282-289)
        }
    }

    const int h = tl.h0 + ty, w = tl.w0 + tx;
    if (h >= H || w >= W) return;
    const int64_t pix = ((int64_t)tl.b * H + h) * W + w;
    const bool hard = a.p.hard_reset != 0;
    const float* vp = a.prev_state ? a.prev_state + pix * C + co0 : nullptr;
    const float* rs = a.residual ? a.residual + tl.b * a.rs_b + h * a.rs_h + w * a.rs_w : nullptr;
    float* st = a.state + pix * C + co0;
    float* out = a.out + pix * C + co0;
    float* cur = a.current + pix * C + co0;
#pragma unroll
    for (int q = 0; q < CO; q += 4) {
        float vo[4], zo[4], oo[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int c = co0 + q + j;
            const float v = vp ? vp[q + j] : 0.0f;
            const float z = vp ? vp[plane + q + j] : 0.0f;
            vo[j] = membrane(v, z, I[q + j], coef[c], hard);
            zo[j] = (vo[j] - coef[c].th > 0.0f) ? 1.0f : 0.0f;
            oo[j] = rs ? zo[j] + rs[(int64_t)c * a.rs_c] : zo[j];
        }
        *reinterpret_cast<float4*>(st + q) = make_float4(vo[0], vo[1], vo[2], vo[3]);
        *reinterpret_cast<float4*>(st + plane + q) = make_float4(zo[0], zo[1], zo[2], zo[3]);
        *reinterpret_cast<float4*>(out + q) = make_float4(oo[0], oo[1], oo[2], oo[3]);
        *reinterpret_cast<float4*>(cur + q) = make_float4(I[q], I[q + 1], I[q + 2], I[q + 3]);
    }
}

// dL/dv_out of one element: g_state_v + (g_out + g_state_z) * sg(v_out - th)
struct Gv { float gv, gxs; };

__device__ inline Gv grad_vout(float gout, float gsv, float gsz, float vout, const CellCoef& k, float width) {
    const float x = vout - k.th;
    const float sg = 1.0f / (1.0f + (width * x) * x);
    Gv r;
    r.gxs = (gout + gsz) * sg;  // dL/d(v_out - th) through the spike
    r.gv = gsv + r.gxs;
    return r;
}

template <int CIN, int C, bool REC, int SPLIT>
__global__ __launch_bounds__(NT * SPLIT) void k_convlif_bwd(snnflow_convlif_bwd_args a) {
    constexpr int NTB = NT * SPLIT, CI = CIN / SPLIT, CR = C / SPLIT, CO = C / SPLIT;
    static_assert(CI * SPLIT == CIN && CR * SPLIT == C, "channel split");
    constexpr int PC = Pad<C>::v;
    __shared__ __attribute__((aligned(16))) float G[HN * PC];
    __shared__ CellCoef coef[C];

    const int tid = threadIdx.x, pt = tid % NT, ty = pt / TW, tx = pt - ty * TW;
    const int part = thread_part(), ci0 = part * CI, cr0 = part * CR, co0 = part * CO;
    const int H = a.H, W = a.W;
    const Tile tl = block_tile(H, W);
    const int64_t plane = (int64_t)a.B * H * W * C;
    const bool hard = a.p.hard_reset != 0;
    const float width = a.p.act_width;
    if (tid < C) coef[tid] = cell_coef(a.p, tid);
    __syncthreads();

    // dL/dI = dL/dv_out * (1 - leak) on the halo
    for (int e = tid; e < HN * C; e += NTB) {
        const int p = e / C, c = e - p * C;
        const int r = p / HWD, cc = p - r * HWD;
        const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
        float gI = 0.0f;
        if (in_image(h, w, H, W)) {
            const int64_t px = ((int64_t)tl.b * H + h) * W + w;
            const float go = a.g_out ? a.g_out[tl.b * a.gs_b + c * a.gs_c + h * a.gs_h + w * a.gs_w] : 0.0f;
            const float gsv = a.g_state ? a.g_state[px * C + c] : 0.0f;
            const float gsz = a.g_state ? a.g_state[plane + px * C + c] : 0.0f;
            const Gv g = grad_vout(go, gsv, gsz, a.state[px * C + c], coef[c], width);
            gI = g.gv * (1.0f - coef[c].leak);
        }
        G[p * PC + c] = gI;
    }
    __syncthreads();

    const int h = tl.h0 + ty, w = tl.w0 + tx;
    const bool in = h < H && w < W;
    const int64_t pix = ((int64_t)tl.b * H + h) * W + w;

    // input gradient of the ff conv; spike-half gradient of the previous state via the rec conv
    if (a.g_x && a.wt_bwd_ff) {
        float gx[CI];
#pragma unroll
        for (int ci = 0; ci < CI; ++ci) gx[ci] = 0.0f;
        dgrad_acc<C, CIN, CI>(G, a.wt_bwd_ff, ty, tx, ci0, gx);
        if (in) {
            float* gb = a.g_x + tl.b * a.gxs_b + h * a.gxs_h + w * a.gxs_w;
#pragma unroll
            for (int ci = 0; ci < CI; ++ci) gb[(int64_t)(ci0 + ci) * a.gxs_c] = gx[ci];
        }
    }
    float gz[CR];
#pragma unroll
    for (int c = 0; c < CR; ++c) gz[c] = 0.0f;
    if constexpr (REC) {
        if (a.g_prev && a.wt_bwd_rec) dgrad_acc<C, C, CR>(G, a.wt_bwd_rec, ty, tx, cr0, gz);
    }
    pin(gz);

    // per pixel: dL/dv_prev, dL/dI for the weight gradient, threshold / leak sums
    float vsum[2 * CO];
#pragma unroll
    for (int j = 0; j < 2 * CO; ++j) vsum[j] = 0.0f;
    if (in) {
        const float* vp = a.prev_state ? a.prev_state + pix * C : nullptr;
#pragma unroll
        for (int q = 0; q < CO; q += 4) {
            float gvp[4], gIo[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = co0 + q + j;
                const float go = a.g_out ? a.g_out[tl.b * a.gs_b + c * a.gs_c + h * a.gs_h + w * a.gs_w] : 0.0f;
                const float gsv = a.g_state ? a.g_state[pix * C + c] : 0.0f;
                const float gsz = a.g_state ? a.g_state[plane + pix * C + c] : 0.0f;
                const CellCoef k = coef[c];
                const Gv g = grad_vout(go, gsv, gsz, a.state[pix * C + c], k, width);
                const float v = vp ? vp[c] : 0.0f, z = vp ? vp[plane + c] : 0.0f;
                const float I = a.current[pix * C + c];
                gIo[j] = g.gv * (1.0f - k.leak);
                // hard: v_out = (v*leak)*(1-z) + (1-leak)*I ; soft: (v*leak + (1-leak)*I) - z*th
                gvp[j] = hard ? (g.gv * (1.0f - z)) * k.leak : g.gv * k.leak;
                const float dleak = hard ? (v * (1.0f - z)) - I : v - I;
                vsum[q + j] += -g.gxs + (hard ? 0.0f : -(g.gv * z));  // dL/dth
                vsum[CO + q + j] += g.gv * dleak;                      // dL/dleak (before sigmoid')
            }
            *reinterpret_cast<float4*>(a.g_current + pix * C + co0 + q) = make_float4(gIo[0], gIo[1], gIo[2], gIo[3]);
            if (a.g_prev)
                *reinterpret_cast<float4*>(a.g_prev + pix * C + co0 + q) = make_float4(gvp[0], gvp[1], gvp[2], gvp[3]);
        }
        if (a.g_prev) {
            // spike half: rec-conv gradient (ConvLIFRecurrent) or zero (z detached in ConvLIF)
            float* gzp = a.g_prev + plane + pix * C + cr0;
#pragma unroll
            for (int c = 0; c < CR; c += 4)
                *reinterpret_cast<float4*>(gzp + c) = make_float4(gz[c], gz[c + 1], gz[c + 2], gz[c + 3]);
        }
    }
    double* acc = acc_shard(a.acc, 2 * C);
    block_atomic_sum_parts<2 * CO, SPLIT>(vsum, [acc](int pp, int j) {
        return acc + (j < CO ? pp * CO + j : C + pp * CO + (j - CO));
    });
}

__global__ void k_convlif_param_grads(const double* acc, const float* leak, const float* thresh, int c,
                                      int accumulate, float* g_leak, float* g_thresh) {
    const int j = threadIdx.x;
    if (j >= c) return;
    const int st = acc_stride(2 * c);
    double sth = 0.0, slk = 0.0;
#pragma unroll
    for (int k = 0; k < kAccShards; ++k) {  // fixed order over the replicas
        sth += acc[k * st + j];
        slk += acc[k * st + c + j];
    }
    const float s = 1.0f / (1.0f + expf(-leak[j]));
    const float gth = thresh[j] >= 0.01f ? (float)sth : 0.0f;
    const float glk = ((float)slk * (1.0f - s)) * s;
    g_thresh[j] = accumulate ? g_thresh[j] + gth : gth;
    g_leak[j] = accumulate ? g_leak[j] + glk : glk;
}

template <int C, int SP>
int convlif_fwd_c(const snnflow_convlif_fwd_args& a, hipStream_t s) {
    const dim3 grid(snnflow_conv_blocks(a.B, a.H, a.W)), block(NT * SP);
#define CLF(CI_)                                                                                         \
    if (a.wt_rec) hipLaunchKernelGGL((k_convlif_fwd<CI_, C, true, SP>), grid, block, 0, s, a);          \
    else hipLaunchKernelGGL((k_convlif_fwd<CI_, C, false, SP>), grid, block, 0, s, a);
    if (a.cin == C) { CLF(C) }
    else if (a.cin == 1) { CLF(1) }
    else if (a.cin == 2) { CLF(2) }
    else if (a.cin == 3) { CLF(3) }
    else if (a.cin == 4) { CLF(4) }
    else if (a.cin == 5) { CLF(5) }
    else SNN_FAIL(SNNFLOW_E_CHANNELS, "convlif_fwd: unsupported cin");
#undef CLF
    SNN_CHECK_LAUNCH();
    return 0;
}

template <int C, int SP>
int convlif_bwd_c(const snnflow_convlif_bwd_args& a, hipStream_t s) {
    const dim3 grid(snnflow_conv_blocks(a.B, a.H, a.W)), block(NT * SP), block1(NT);
    // the input-channel split of the dgrad needs cin % SP == 0
#define CLB(CI_, SPX, BLK)                                                                                  \
    if (a.wt_bwd_rec) hipLaunchKernelGGL((k_convlif_bwd<CI_, C, true, SPX>), grid, BLK, 0, s, a);          \
    else hipLaunchKernelGGL((k_convlif_bwd<CI_, C, false, SPX>), grid, BLK, 0, s, a);
    if (a.cin == C) { CLB(C, SP, block) }
    else if (a.cin == 1) { CLB(1, 1, block1) }
    else if (a.cin == 2) { CLB(2, 1, block1) }
    else if (a.cin == 3) { CLB(3, 1, block1) }
    else if (a.cin == 4) { CLB(4, 1, block1) }
    else if (a.cin == 5) { CLB(5, 1, block1) }
    else SNN_FAIL(SNNFLOW_E_CHANNELS, "convlif_bwd: unsupported cin");
#undef CLB
    SNN_CHECK_LAUNCH();
    return 0;
}

}  // namespace

extern "C" {

int snnflow_convlif_fwd(const snnflow_convlif_fwd_args* a, void* stream) {
    if (!a || a->B <= 0 || a->H <= 0 || a->W <= 0 || !a->x || !a->wt_ff || !a->p.leak || !a->p.thresh || !a->out ||
        !a->state || !a->current)
        SNN_FAIL(SNNFLOW_E_ARG, "convlif_fwd: bad args");
    const hipStream_t s = (hipStream_t)stream;
    switch (a->c) {
        case 4: return convlif_fwd_c<4, 1>(*a, s);
        case 8: return convlif_fwd_c<8, 2>(*a, s);
        case 16: return convlif_fwd_c<16, 2>(*a, s);
        case 32: return convlif_fwd_c<32, 1>(*a, s);
        default: SNN_FAIL(SNNFLOW_E_CHANNELS, "convlif_fwd: c must be 4, 8, 16 or 32");
    }
}

int snnflow_convlif_bwd(const snnflow_convlif_bwd_args* a, void* stream) {
    if (!a || a->B <= 0 || a->H <= 0 || a->W <= 0 || !a->state || !a->current || !a->g_current || !a->acc ||
        !a->p.leak || !a->p.thresh)
        SNN_FAIL(SNNFLOW_E_ARG, "convlif_bwd: bad args");
    if (a->g_x && !a->wt_bwd_ff) SNN_FAIL(SNNFLOW_E_ARG, "convlif_bwd: input gradient needs wt_bwd_ff");
    const hipStream_t s = (hipStream_t)stream;
    switch (a->c) {
        case 4: return convlif_bwd_c<4, 1>(*a, s);
        case 8: return convlif_bwd_c<8, 2>(*a, s);
        case 16: return convlif_bwd_c<16, 2>(*a, s);
        case 32: return convlif_bwd_c<32, 1>(*a, s);
        default: SNN_FAIL(SNNFLOW_E_CHANNELS, "convlif_bwd: c must be 4, 8, 16 or 32");
    }
}

int snnflow_convlif_param_grads(const double* acc, const float* leak, const float* thresh, int c, int accumulate,
                                float* g_leak, float* g_thresh, void* stream) {
    if (!acc || !leak || !thresh || !g_leak || !g_thresh || c <= 0 || c > NT)
        SNN_FAIL(SNNFLOW_E_ARG, "convlif_param_grads: bad args");
    hipLaunchKernelGGL(k_convlif_param_grads, dim3(1), dim3(NT), 0, (hipStream_t)stream, acc, leak, thresh, c,
                       accumulate, g_leak, g_thresh);
    SNN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
