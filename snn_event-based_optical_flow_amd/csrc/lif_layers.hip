// LIFFireNet cell kernels for gfx950: fused [LIF(l) on a halo tile] + conv3x3(l+1) + BN
// statistics forward, LIF(+pred) forward, and the matching backward kernels.
//
// Reference semantics (restated, see oracle/lif_ref.py):
//   cell   SNNtorch_ConvLIF(Recurrent).forward  models/SNNtorch_spiking_submodules.py:283-322, 515-567
//   neuron snntorch.Leaky (0.9.4), reset_delay=False, ATan surrogate (third-party, restated)
//   BN     torch BatchNorm2d train/eval (batch stats over B,H,W; running stats momentum update)
//   pred   models/submodules.py:ConvLayer (1x1 conv + bias, tanh)
//
// Layout: NHWC activations, state [2][B][H][W][C].  One 256-thread block owns an
// 8x32 pixel tile; halo rows are recomputed by neighbouring blocks (never stored).
#include <cmath>
#include <string>

#include "snnflow_dev.h"

using namespace snnflow;

namespace {
thread_local std::string g_err;
}

int snnflow_set_error(int code, const char* msg) {
    g_err = msg;
    return code;
}

#define SNN_FAIL(code, msg) return snnflow_set_error((code), (msg))
#define SNN_CHECK_LAUNCH()                                                        \
    do {                                                                          \
        hipError_t e_ = hipGetLastError();                                        \
        if (e_ != hipSuccess) return snnflow_set_error((int)e_, hipGetErrorString(e_)); \
    } while (0)

namespace {

// ---------------------------------------------------------------------------
// LDS staging of a halo tile
// ---------------------------------------------------------------------------
__device__ inline bool in_image(int h, int w, int H, int W) { return h >= 0 && h < H && w >= 0 && w < W; }

// Strided input (e.g. event_cnt NCHW, or an NHWC spike tensor) -> tile[p][ci]
template <int CIN>
__device__ void stage_strided(const float* __restrict__ x, int64_t sb, int64_t sc, int64_t sh, int64_t sw,
                              const Tile& tl, int H, int W, float* tile) {
    constexpr int P = Pad<CIN>::v;
    const int tid = threadIdx.x;
    const float* xb = x + (int64_t)tl.b * sb;
    if (sc == 1) {
        for (int e = tid; e < HN * CIN; e += NT) {
            const int p = e / CIN, ci = e - p * CIN;
            const int r = p / HWD, cc = p - r * HWD;
            const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
            tile[p * P + ci] = in_image(h, w, H, W) ? xb[h * sh + w * sw + ci] : 0.0f;
        }
    } else {
        for (int e = tid; e < HN * CIN; e += NT) {
            const int ci = e / HN, p = e - ci * HN;
            const int r = p / HWD, cc = p - r * HWD;
            const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
            tile[p * P + ci] = in_image(h, w, H, W) ? xb[ci * sc + h * sh + w * sw] : 0.0f;
        }
    }
}

// Contiguous NHWC [B][H][W][C] (C % 4 == 0) -> tile
template <int C>
__device__ void stage_nhwc(const float* __restrict__ x, const Tile& tl, int H, int W, float* tile) {
    static_assert(C % 4 == 0, "vector staging");
    constexpr int P = Pad<C>::v, Q = C / 4;
    const int tid = threadIdx.x;
    for (int e = tid; e < HN * Q; e += NT) {
        const int p = e / Q, q = e - p * Q;
        const int r = p / HWD, cc = p - r * HWD;
        const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (in_image(h, w, H, W))
            v = *reinterpret_cast<const float4*>(x + (((int64_t)tl.b * H + h) * W + w) * C + 4 * q);
        *reinterpret_cast<float4*>(tile + p * P + 4 * q) = v;
    }
}

// ---------------------------------------------------------------------------
// 3x3 convolution of one output pixel (all C outputs) from an LDS halo tile.
// wt: [3][3][CIN][C] (uniform -> scalar loads).  acc += sum_{ky,kx,ci} w * x.
// ---------------------------------------------------------------------------
template <int CIN, int C>
__device__ inline void conv_acc(const float* tile, const float* __restrict__ wt, int ty, int tx, float (&acc)[C]) {
    constexpr int P = Pad<CIN>::v, VW = VecW<CIN>::v;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const float* xp = tile + ((ty + ky) * HWD + (tx + kx)) * P;
            const cfloat_ptr wk = as_const(wt) + (ky * 3 + kx) * CIN * C;
#pragma unroll(CIN <= 8 ? CIN : 1)
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
                    for (int co = 0; co < C; ++co) acc[co] = fmaf(wk[(ci + j) * C + co], xs[j], acc[co]);
                }
            }
        }
    }
}

// Transposed 3x3 (input gradient) of one pixel from an LDS tile of output gradients.
// wd: [3][3][C][CIN].  gx[ci] += sum_{ky,kx,co} w[co][ci][ky][kx] * g[h+1-ky][w+1-kx][co]
template <int C, int CIN>
__device__ inline void dgrad_acc(const float* gtile, const float* __restrict__ wd, int ty, int tx, float (&gx)[CIN]) {
    constexpr int P = Pad<C>::v;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const float* gp = gtile + ((ty + 2 - ky) * HWD + (tx + 2 - kx)) * P;
            const cfloat_ptr wk = as_const(wd) + (ky * 3 + kx) * C * CIN;
#pragma unroll(C <= 8 ? C : 1)
            for (int co = 0; co < C; co += 4) {
                const float4 v = *reinterpret_cast<const float4*>(gp + co);
                const float gs[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
#pragma unroll
                    for (int ci = 0; ci < CIN; ++ci) gx[ci] = fmaf(wk[(co + j) * CIN + ci], gs[j], gx[ci]);
                }
            }
        }
    }
}

// Per-block weight-gradient partial of one 3x3 conv:
//   dW[co][ci][ky][kx] = sum_{tile pixels p} g[p][co] * x[p + (ky-1, kx-1)][ci]
// G: LDS g tile (halo layout, C channels), X: LDS input halo tile (CIN channels).
// Items (k, co-block of 4, ci-block of VW) x pixel groups; groups reduced in fixed order.
template <int CIN, int C>
struct WgradShape {
    static constexpr int VW = VecW<CIN>::v;
    static constexpr int NCB = CIN / VW;
    static constexpr int Q = 9 * (C / 4) * NCB;
    static constexpr int GR = (Q >= NT) ? 1 : NT / Q;
    static constexpr int SCRATCH = (GR > 1) ? GR * Q * 4 * VW : 1;
};

template <int CIN, int C>
__device__ void wgrad_tile(const float* G, const float* X, float* __restrict__ slab, int accumulate, float* scratch) {
    using S = WgradShape<CIN, C>;
    constexpr int VW = S::VW, Q = S::Q, GR = S::GR, PC = Pad<C>::v, PX = Pad<CIN>::v;
    const int tid = threadIdx.x;
    for (int q0 = 0; q0 < Q; q0 += (GR > 1 ? Q : NT)) {
        const int q = (GR > 1) ? tid % Q : q0 + tid;
        const int g = (GR > 1) ? tid / Q : 0;
        const bool active = (GR > 1) ? (g < GR) : (q < Q);
        float acc[4][VW];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < VW; ++j) acc[i][j] = 0.f;
        int kidx = 0, cob = 0, cib = 0;
        if (active) {
            kidx = q % 9;
            const int rest = q / 9;
            cob = rest % (C / 4);
            cib = rest / (C / 4);
            const int ky = kidx / 3, kx = kidx % 3;
            for (int p = g; p < NT; p += GR) {
                const int ty = p / TW, tx = p - ty * TW;
                const float4 gv4 = *reinterpret_cast<const float4*>(G + ((ty + 1) * HWD + tx + 1) * PC + cob * 4);
                const float gv[4] = {gv4.x, gv4.y, gv4.z, gv4.w};
                const float* xp = X + ((ty + ky) * HWD + tx + kx) * PX + cib * VW;
                float xv[VW];
                if constexpr (VW == 4) {
                    const float4 v = *reinterpret_cast<const float4*>(xp);
                    xv[0] = v.x; xv[1] = v.y; xv[2] = v.z; xv[3] = v.w;
                } else if constexpr (VW == 2) {
                    const float2 v = *reinterpret_cast<const float2*>(xp);
                    xv[0] = v.x; xv[1] = v.y;
                } else {
                    xv[0] = xp[0];
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < VW; ++j) acc[i][j] = fmaf(gv[i], xv[j], acc[i][j]);
            }
        }
        if constexpr (GR > 1) {
            if (active) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < VW; ++j) scratch[((g * Q + q) * 4 + i) * VW + j] = acc[i][j];
            }
            __syncthreads();
            for (int e = tid; e < Q * 4 * VW; e += NT) {
                float s = 0.f;
                for (int gg = 0; gg < GR; ++gg) s += scratch[gg * Q * 4 * VW + e];
                const int qq = e / (4 * VW), ij = e - qq * 4 * VW, i = ij / VW, j = ij - i * VW;
                const int kk = qq % 9, rest = qq / 9, cb = rest % (C / 4), ib = rest / (C / 4);
                const int widx = ((cb * 4 + i) * CIN + ib * VW + j) * 9 + kk;
                slab[widx] = accumulate ? slab[widx] + s : s;
            }
            __syncthreads();
        } else {
            if (active) {
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < VW; ++j) {
                        const int widx = ((cob * 4 + i) * CIN + cib * VW + j) * 9 + kidx;
                        slab[widx] = accumulate ? slab[widx] + acc[i][j] : acc[i][j];
                    }
            }
        }
    }
}

// dL/dm of the membrane input: v = beta*((1-r)*m) + I (zero reset) or beta*m + I - r*theta;
// r = H(m - theta) is detached (snntorch mem_reset).
__device__ inline float mem_grad(float gv, float m, const LifCoef& k, bool zero_reset) {
    const float gmp = gv * k.beta;
    if (!zero_reset) return gmp;
    const float r = (m - k.theta > 0.0f) ? 1.0f : 0.0f;
    return gmp * (1.0f - r);
}

// Block-level sum of NV per-thread floats, then one fp64 atomic add per value into
// acc (the block's partial; NV <= NT values issued by consecutive lanes).
template <int NV>
__device__ void block_atomic_sum(const float (&v)[NV], double* acc) {
    __shared__ float red[4][NV];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const float s = wave_sum(v[j]);
        if (lane == 0) red[wv][j] = s;
    }
    __syncthreads();
    for (int j = threadIdx.x; j < NV; j += NT)
        atomicAdd(acc + j, (((double)red[0][j] + (double)red[1][j]) + (double)red[2][j]) + (double)red[3][j]);
}

// Block 0 zeroes accumulators already consumed by an earlier kernel of the chain.
__device__ inline void zero_consumed(double* z0, double* z1, int n) {
    if (blockIdx.x != 0) return;
    for (int j = threadIdx.x; j < n; j += NT) {
        if (z0) z0[j] = 0.0;
        if (z1) z1[j] = 0.0;
    }
}

// BatchNorm statistics of channel c from batch sums (train) or running stats (eval):
// mean = S/N, var = SS/N - mean^2 (biased), invstd = 1/sqrt(var + eps) in fp64.
struct BnStat { float mean, invstd; double dmean, dvar; };

__device__ inline BnStat bn_stat(const snnflow_neuron& n, const double* acc, int C, int c, double N) {
    BnStat st;
    if (n.bn_train) {
        st.dmean = acc[c] / N;
        st.dvar = acc[C + c] / N - st.dmean * st.dmean;
        if (st.dvar < 0.0) st.dvar = 0.0;
        st.mean = (float)st.dmean;
        st.invstd = (float)(1.0 / sqrt(st.dvar + n.eps));
    } else {
        st.dmean = n.running_mean[c];
        st.dvar = n.running_var[c];
        st.mean = n.running_mean[c];
        st.invstd = (float)(1.0 / sqrt((double)n.running_var[c] + n.eps));
    }
    return st;
}

// Prologue of a LIF consumer: per-channel coefficients in LDS; block 0 also stores
// (mean, invstd) for the backward pass and performs the running-stat update
// (momentum, unbiased variance) and num_batches_tracked += 1 of torch's BatchNorm2d.
__device__ void lif_prologue(const snnflow_neuron& n, const double* acc, int C, double N, float* stats_out,
                             LifCoef* coef, float* mean_out) {
    const int c = threadIdx.x;
    if (c < C) {
        const BnStat st = bn_stat(n, acc, C, c, N);
        LifCoef k;
        k.alpha = st.invstd * n.bn_weight[c];
        k.shift = n.bn_bias[c] - st.mean * k.alpha;
        k.beta = fminf(fmaxf(n.beta[c], 0.0f), 1.0f);
        k.theta = n.threshold[c];
        coef[c] = k;
        if (mean_out) mean_out[c] = st.mean;
        if (blockIdx.x == 0) {
            if (stats_out) {
                stats_out[c] = st.mean;
                stats_out[C + c] = st.invstd;
            }
            if (n.bn_train && n.running_mean) {
                const double unb = N > 1.0 ? st.dvar * N / (N - 1.0) : st.dvar;
                n.running_mean[c] = (float)(n.momentum * st.dmean + (1.0 - n.momentum) * (double)n.running_mean[c]);
                n.running_var[c] = (float)(n.momentum * unb + (1.0 - n.momentum) * (double)n.running_var[c]);
            }
        }
    }
    if (c == 0 && blockIdx.x == 0 && n.bn_train && n.num_batches_tracked) n.num_batches_tracked[0] += 1;
}

// Layer-l gradients of (gamma, bn bias, beta, threshold) [and pred] from the LIF-backward
// sums: gamma = dotp*invstd, bias = sum g, theta = -sum g, beta = sum g*m' (0 <= beta <= 1)
// (torch batch_norm_cpu_backward; snntorch Leaky; clamp backward passes on [0,1]).
__device__ void neuron_grads(const snnflow_neuron& n, const float* stats, const double* acc, int C,
                             const snnflow_neuron_grad& ng, int accumulate, int has_pred, float* g_pred_w,
                             float* g_pred_b) {
    if (blockIdx.x != 0) return;
    const int c = threadIdx.x;
    if (c < C) {
        const double gsum = acc[c], dotp = acc[C + c], gbm = acc[2 * C + c];
        const float gw = (float)(dotp * (double)stats[C + c]);
        const float gb = (float)gsum;
        const float gth = -(float)gsum;
        const float be = n.beta[c];
        const float gbe = (be >= 0.0f && be <= 1.0f) ? (float)gbm : 0.0f;
        if (accumulate) {
            ng.bn_weight[c] += gw; ng.bn_bias[c] += gb; ng.threshold[c] += gth; ng.beta[c] += gbe;
        } else {
            ng.bn_weight[c] = gw; ng.bn_bias[c] = gb; ng.threshold[c] = gth; ng.beta[c] = gbe;
        }
    }
    if (has_pred) {
        for (int j = threadIdx.x; j < 2 * C + 2; j += NT) {
            const float g = (float)acc[3 * C + j];
            float* dst = (j < 2 * C) ? g_pred_w + j : g_pred_b + (j - 2 * C);
            *dst = accumulate ? *dst + g : g;
        }
    }
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------
__global__ void k_prep_weights(const float* __restrict__ w, int c, int cin, float* __restrict__ wt_fwd,
                               float* __restrict__ wt_bwd, float* thr) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = c * cin * 9;
    if (w && e < n) {
        const int k = e % 9, ci = (e / 9) % cin, co = e / (9 * cin);
        const float v = w[e];
        wt_fwd[(k * cin + ci) * c + co] = v;
        wt_bwd[(k * c + co) * cin + ci] = v;
    }
    if (thr && e < c) {
        const float t = thr[e];
        thr[e] = (t < 0.01f) ? 0.01f : t;
    }
}

template <int CIN, int C, bool LIF_IN, bool REC>
__global__ __launch_bounds__(NT) void k_conv_fwd(snnflow_conv_fwd_args a) {
    constexpr int PI_ = Pad<CIN>::v, PC = Pad<C>::v;
    constexpr int PMAX = (REC && PC > PI_) ? PC : PI_;
    __shared__ __attribute__((aligned(16))) float tile[HN * PMAX];
    __shared__ LifCoef coef[LIF_IN ? CIN : 1];

    const int tid = threadIdx.x, ty = tid / TW, tx = tid - ty * TW;
    const int H = a.H, W = a.W;
    const Tile tl = block_tile(H, W);
    zero_consumed(a.zero0, a.zero1, a.zero_n);

    if constexpr (LIF_IN) {
        lif_prologue(a.prev, a.prev_acc, CIN, (double)a.B * H * W, a.prev_stats, coef, nullptr);
        __syncthreads();
        // LIF of the previous layer over the halo tile; interior pixels also write its state.
        const bool zr = a.prev.zero_reset != 0;
        const int64_t plane = (int64_t)a.B * H * W * CIN;
        for (int p = tid; p < HN; p += NT) {
            const int r = p / HWD, cc = p - r * HWD;
            const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
            float* dst = tile + p * PI_;
            if (in_image(h, w, H, W)) {
                const int64_t pix = ((int64_t)tl.b * H + h) * W + w;
                const bool interior = (r >= 1 && r <= TH && cc >= 1 && cc <= TW);
#pragma unroll
                for (int ci = 0; ci < CIN; ci += 4) {
                    const float4 yv = *reinterpret_cast<const float4*>(a.prev_y + pix * CIN + ci);
                    const float4 mv = a.prev_mem ? *reinterpret_cast<const float4*>(a.prev_mem + pix * CIN + ci)
                                                 : make_float4(0.f, 0.f, 0.f, 0.f);
                    const LifOut o0 = lif_step(yv.x, mv.x, coef[ci + 0], zr);
                    const LifOut o1 = lif_step(yv.y, mv.y, coef[ci + 1], zr);
                    const LifOut o2 = lif_step(yv.z, mv.z, coef[ci + 2], zr);
                    const LifOut o3 = lif_step(yv.w, mv.w, coef[ci + 3], zr);
                    const float4 sv = make_float4(o0.s, o1.s, o2.s, o3.s);
                    *reinterpret_cast<float4*>(dst + ci) = sv;
                    if (interior) {
                        *reinterpret_cast<float4*>(a.prev_state + pix * CIN + ci) =
                            make_float4(o0.mout, o1.mout, o2.mout, o3.mout);
                        *reinterpret_cast<float4*>(a.prev_state + plane + pix * CIN + ci) = sv;
                    }
                }
            } else {
#pragma unroll
                for (int ci = 0; ci < CIN; ++ci) dst[ci] = 0.0f;
            }
        }
    } else {
        stage_strided<CIN>(a.x, a.xs_b, a.xs_c, a.xs_h, a.xs_w, tl, H, W, tile);
    }
    __syncthreads();

    float y[C];
#pragma unroll
    for (int co = 0; co < C; ++co) y[co] = 0.0f;
    conv_acc<CIN, C>(tile, a.wt_ff, ty, tx, y);

    if constexpr (REC) {
        if (a.s_prev) {
            __syncthreads();
            stage_nhwc<C>(a.s_prev, tl, H, W, tile);
            __syncthreads();
            float r[C];
#pragma unroll
            for (int co = 0; co < C; ++co) r[co] = 0.0f;
            conv_acc<C, C>(tile, a.wt_rec, ty, tx, r);
#pragma unroll
            for (int co = 0; co < C; ++co) y[co] = y[co] + r[co];  // ff + rec (:540)
        }
    }

    const int h = tl.h0 + ty, w = tl.w0 + tx;
    const bool in = (h < H) && (w < W);
    if (in) {
        float* yp = a.y + (((int64_t)tl.b * H + h) * W + w) * C;
#pragma unroll
        for (int co = 0; co < C; co += 4)
            *reinterpret_cast<float4*>(yp + co) = make_float4(y[co], y[co + 1], y[co + 2], y[co + 3]);
    }
    if (a.acc) {
        float v[2 * C];
#pragma unroll
        for (int co = 0; co < C; ++co) {
            const float yy = in ? y[co] : 0.0f;
            v[co] = yy;
            v[C + co] = yy * yy;
        }
        block_atomic_sum<2 * C>(v, a.acc);
    }
}

template <int C, bool PRED>
__global__ __launch_bounds__(NT) void k_lif_fwd(snnflow_lif_fwd_args a) {
    __shared__ LifCoef coef[C];
    const int tid = threadIdx.x;
    zero_consumed(a.zero0, a.zero1, a.zero_n);
    lif_prologue(a.n, a.acc, C, (double)a.B * a.H * a.W, a.stats, coef, nullptr);
    __syncthreads();
    const bool zr = a.n.zero_reset != 0;
    const int64_t HWp = (int64_t)a.H * a.W, npix = (int64_t)a.B * HWp, plane = npix * C;
    for (int64_t p = (int64_t)blockIdx.x * NT + tid; p < npix; p += (int64_t)gridDim.x * NT) {
        float s[C];
#pragma unroll
        for (int c = 0; c < C; c += 4) {
            const float4 yv = *reinterpret_cast<const float4*>(a.y + p * C + c);
            const float4 mv = a.mem ? *reinterpret_cast<const float4*>(a.mem + p * C + c) : make_float4(0.f, 0.f, 0.f, 0.f);
            const LifOut o0 = lif_step(yv.x, mv.x, coef[c + 0], zr);
            const LifOut o1 = lif_step(yv.y, mv.y, coef[c + 1], zr);
            const LifOut o2 = lif_step(yv.z, mv.z, coef[c + 2], zr);
            const LifOut o3 = lif_step(yv.w, mv.w, coef[c + 3], zr);
            s[c] = o0.s; s[c + 1] = o1.s; s[c + 2] = o2.s; s[c + 3] = o3.s;
            *reinterpret_cast<float4*>(a.state + p * C + c) = make_float4(o0.mout, o1.mout, o2.mout, o3.mout);
            *reinterpret_cast<float4*>(a.state + plane + p * C + c) = make_float4(o0.s, o1.s, o2.s, o3.s);
        }
        if constexpr (PRED) {
            const int64_t b = p / HWp, hw = p - b * HWp;
#pragma unroll
            for (int o = 0; o < 2; ++o) {
                float acc = 0.0f;
#pragma unroll
                for (int c = 0; c < C; ++c) acc = fmaf(a.pred_w[o * C + c], s[c], acc);
                a.flow[(b * 2 + o) * HWp + hw] = tanhf(acc + a.pred_b[o]);
            }
        }
    }
}

template <int C, bool PRED>
__global__ __launch_bounds__(NT) void k_lif_bwd(snnflow_lif_bwd_args a) {
    constexpr int NV = 3 * C + (PRED ? 2 * C + 2 : 0);
    __shared__ LifCoef coef[C];
    __shared__ float meanv[C];
    const int tid = threadIdx.x;
    zero_consumed(a.zero0, a.zero1, a.zero_n);
    if (tid < C) {
        coef[tid] = lif_coef(a.n, a.stats, C, tid);
        meanv[tid] = a.stats[tid];
    }
    __syncthreads();
    const bool zr = a.n.zero_reset != 0;
    const int64_t HWp = (int64_t)a.H * a.W, npix = (int64_t)a.B * HWp, plane = npix * C;
    float v[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) v[j] = 0.0f;
    for (int64_t p = (int64_t)blockIdx.x * NT + tid; p < npix; p += (int64_t)gridDim.x * NT) {
        float gs[C];
#pragma unroll
        for (int c = 0; c < C; ++c) gs[c] = 0.0f;
        if (a.g_out) {
#pragma unroll
            for (int c = 0; c < C; ++c) gs[c] = a.g_out[p * C + c];
        }
        if (a.g_state) {
#pragma unroll
            for (int c = 0; c < C; ++c) gs[c] = gs[c] + a.g_state[plane + p * C + c];
        }
        float gpre[2] = {0.0f, 0.0f};
        if constexpr (PRED) {
            if (a.g_flow) {
                const int64_t b = p / HWp, hw = p - b * HWp;
#pragma unroll
                for (int o = 0; o < 2; ++o) {
                    const float f = a.flow[(b * 2 + o) * HWp + hw];
                    const float g = a.g_flow[b * a.gflow_sb + o * a.gflow_sc + hw];
                    gpre[o] = g * (1.0f - f * f);  // tanh backward
                }
#pragma unroll
                for (int c = 0; c < C; ++c)
                    gs[c] = gs[c] + (a.pred_w[c] * gpre[0] + a.pred_w[C + c] * gpre[1]);
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const float yy = a.y[p * C + c];
            const float mm = a.mem ? a.mem[p * C + c] : 0.0f;
            const LifOut o = lif_step(yy, mm, coef[c], zr);
            const float gv = atan_sg(o.v - coef[c].theta) * gs[c];
            a.g_cur[p * C + c] = gv;
            if (a.g_mem) a.g_mem[p * C + c] = mem_grad(gv, mm, coef[c], zr);
            v[c] += gv;
            v[C + c] += (yy - meanv[c]) * gv;
            v[2 * C + c] += gv * o.mprime;
            if constexpr (PRED) {
                v[3 * C + c] += gpre[0] * o.s;
                v[4 * C + c] += gpre[1] * o.s;
            }
        }
        if constexpr (PRED) {
            v[5 * C] += gpre[0];
            v[5 * C + 1] += gpre[1];
        }
    }
    block_atomic_sum<NV>(v, a.acc);
}

template <int CIN, int C, bool LIF_IN, bool REC>
__global__ __launch_bounds__(NT) void k_layer_bwd(snnflow_layer_bwd_args a) {
    using WS = WgradShape<CIN, C>;
    using WR = WgradShape<C, C>;
    constexpr int PI_ = Pad<CIN>::v, PC = Pad<C>::v;
    constexpr int PX = (REC && PC > PI_) ? PC : PI_;
    constexpr int SCR = (WS::SCRATCH > WR::SCRATCH) ? WS::SCRATCH : WR::SCRATCH;
    __shared__ __attribute__((aligned(16))) float G[HN * PC];
    __shared__ __attribute__((aligned(16))) float X[HN * PX];
    __shared__ __attribute__((aligned(16))) float scratch[SCR];
    __shared__ float bn_mean[C], bn_inv[C], bn_gm[C], bn_k[C], bn_w[C];
    __shared__ LifCoef pcoef[LIF_IN ? CIN : 1];
    __shared__ float pmean[LIF_IN ? CIN : 1];
    constexpr int NVP = LIF_IN ? 3 * CIN : 1;

    const int tid = threadIdx.x, ty = tid / TW, tx = tid - ty * TW;
    const int H = a.H, W = a.W;
    const Tile tl = block_tile(H, W);
    const double N = (double)a.B * H * W;
    const float nf = (float)N;
    zero_consumed(a.zero0, a.zero1, a.zero_n);
    neuron_grads(a.n, a.stats, a.acc_in, C, a.ng, a.accumulate, a.has_pred, a.g_pred_w, a.g_pred_b);

    if (tid < C) {
        const float mean = a.stats[tid], inv = a.stats[C + tid];
        bn_mean[tid] = mean;
        bn_inv[tid] = inv;
        bn_w[tid] = a.n.bn_weight[tid];
        if (a.n.bn_train) {
            // torch batch_norm_cpu_backward: k = dotp*invstd*invstd/n, grad_mean = sum/n
            bn_k[tid] = (float)a.acc_in[C + tid] * inv * inv / nf;
            bn_gm[tid] = (float)(a.acc_in[tid] / N);
        } else {
            bn_k[tid] = 0.0f;
            bn_gm[tid] = 0.0f;
        }
    }
    if constexpr (LIF_IN) {
        if (tid < CIN) {
            pcoef[tid] = lif_coef(a.prev, a.prev_stats, CIN, tid);
            pmean[tid] = a.prev_stats[tid];
        }
    }
    __syncthreads();

    // Stage A: BN backward on the halo -> G = dL/dy (pre-BN conv output of layer l)
    for (int e = tid; e < HN * (C / 4); e += NT) {
        const int p = e / (C / 4), q = e - p * (C / 4);
        const int r = p / HWD, cc = p - r * HWD;
        const int h = tl.h0 + r - 1, w = tl.w0 + cc - 1;
        float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
        if (in_image(h, w, H, W)) {
            const int64_t off = (((int64_t)tl.b * H + h) * W + w) * C + 4 * q;
            const float4 g = *reinterpret_cast<const float4*>(a.g_cur + off);
            const float4 yv = *reinterpret_cast<const float4*>(a.y + off);
            const float gi[4] = {g.x, g.y, g.z, g.w}, yi[4] = {yv.x, yv.y, yv.z, yv.w};
            float o[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = 4 * q + j;
                const float dx = (yi[j] - bn_mean[c]) * bn_k[c];
                o[j] = (((gi[j] - bn_gm[c]) - dx) * bn_inv[c]) * bn_w[c];
            }
            out = make_float4(o[0], o[1], o[2], o[3]);
        }
        *reinterpret_cast<float4*>(G + p * PC + 4 * q) = out;
    }
    __syncthreads();

    const int h = tl.h0 + ty, w = tl.w0 + tx;
    const bool in = (h < H) && (w < W);
    const int64_t pix = ((int64_t)tl.b * H + h) * W + w;

    // Stage B: input gradient (dgrad) of ff and rec convolutions
    float gx[CIN];
#pragma unroll
    for (int ci = 0; ci < CIN; ++ci) gx[ci] = 0.0f;
    if (a.wt_bwd_ff) dgrad_acc<C, CIN>(G, a.wt_bwd_ff, ty, tx, gx);
    if constexpr (REC) {
        if (a.g_state_prev) {
            float gr[C];
#pragma unroll
            for (int c = 0; c < C; ++c) gr[c] = 0.0f;
            dgrad_acc<C, C>(G, a.wt_bwd_rec, ty, tx, gr);
            if (in) {
                const int64_t plane = (int64_t)a.B * H * W * C;
#pragma unroll
                for (int c = 0; c < C; c += 4) {
                    if (a.zero_mem_half)
                        *reinterpret_cast<float4*>(a.g_state_prev + pix * C + c) = make_float4(0.f, 0.f, 0.f, 0.f);
                    *reinterpret_cast<float4*>(a.g_state_prev + plane + pix * C + c) =
                        make_float4(gr[c], gr[c + 1], gr[c + 2], gr[c + 3]);
                }
            }
        }
    }

    // Stage C: weight gradients (per-block slabs)
    const int64_t blk = blockIdx.x;
    bool dense = false;
    if constexpr (CIN % 4 == 0)
        dense = a.xs_c == 1 && a.xs_w == CIN && a.xs_h == (int64_t)W * CIN && a.xs_b == (int64_t)H * W * CIN;
    if constexpr (CIN % 4 == 0) {
        if (dense) stage_nhwc<CIN>(a.x, tl, H, W, X);
    }
    if (!dense) stage_strided<CIN>(a.x, a.xs_b, a.xs_c, a.xs_h, a.xs_w, tl, H, W, X);
    __syncthreads();
    wgrad_tile<CIN, C>(G, X, a.slab_ff + blk * (C * CIN * 9), a.accumulate, scratch);
    if constexpr (REC) {
        float* slab = a.slab_rec + blk * (C * C * 9);
        if (a.s_prev) {
            __syncthreads();
            stage_nhwc<C>(a.s_prev, tl, H, W, X);
            __syncthreads();
            wgrad_tile<C, C>(G, X, slab, a.accumulate, scratch);
        } else if (!a.accumulate) {
            for (int e = tid; e < C * C * 9; e += NT) slab[e] = 0.0f;
        }
    }

    // Stage D: LIF backward of layer l-1 on the dgrad result, or the plain input gradient
    if constexpr (LIF_IN) {
        float v[NVP];
#pragma unroll
        for (int j = 0; j < NVP; ++j) v[j] = 0.0f;
        if (in) {
            const bool zr = a.prev.zero_reset != 0;
            const int64_t plane = (int64_t)a.B * H * W * CIN;
#pragma unroll
            for (int ci = 0; ci < CIN; ++ci) {
                float gs = gx[ci];
                if (a.prev_g_state) gs = gs + a.prev_g_state[plane + pix * CIN + ci];
                const float yy = a.prev_y[pix * CIN + ci];
                const float mm = a.prev_mem ? a.prev_mem[pix * CIN + ci] : 0.0f;
                const LifOut o = lif_step(yy, mm, pcoef[ci], zr);
                const float gv = atan_sg(o.v - pcoef[ci].theta) * gs;
                a.prev_g_cur[pix * CIN + ci] = gv;
                if (a.prev_g_mem) a.prev_g_mem[pix * CIN + ci] = mem_grad(gv, mm, pcoef[ci], zr);
                v[ci] = gv;
                v[CIN + ci] = (yy - pmean[ci]) * gv;
                v[2 * CIN + ci] = gv * o.mprime;
            }
        }
        block_atomic_sum<NVP>(v, a.acc_out);
    } else {
        if (a.g_x && a.wt_bwd_ff && in) {
            float* gb = a.g_x + (int64_t)tl.b * a.gxs_b + h * a.gxs_h + w * a.gxs_w;
#pragma unroll
            for (int ci = 0; ci < CIN; ++ci) gb[ci * a.gxs_c] = gx[ci];
        }
    }
}

__global__ void k_slab_reduce(snnflow_slab_desc d0, snnflow_slab_desc d1, snnflow_slab_desc d2, snnflow_slab_desc d3,
                              snnflow_slab_desc d4, snnflow_slab_desc d5, snnflow_slab_desc d6, snnflow_slab_desc d7,
                              snnflow_slab_desc d8, snnflow_slab_desc d9, snnflow_slab_desc d10, snnflow_slab_desc d11,
                              snnflow_slab_desc d12, snnflow_slab_desc d13, snnflow_slab_desc d14, snnflow_slab_desc d15,
                              int nblk) {
    const snnflow_slab_desc ds[16] = {d0, d1, d2, d3, d4, d5, d6, d7, d8, d9, d10, d11, d12, d13, d14, d15};
    const snnflow_slab_desc d = ds[blockIdx.y];
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= d.elems) return;
    double s = 0.0;
    for (int b = 0; b < nblk; ++b) s += d.slab[(int64_t)b * d.elems + e];
    d.out[e] = (float)s;
}

__global__ void k_lif_export(const float* __restrict__ x, const float* __restrict__ mem, const float* __restrict__ beta,
                             const float* __restrict__ thr, int64_t total, int C, int HW, float* spk, float* mout) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)((i / HW) % C);
        const float m = beta[c] * mem[i] + x[i];
        const bool s = m >= thr[c];
        spk[i] = s ? 1.0f : 0.0f;
        mout[i] = s ? 0.0f : m;
    }
}

// ---------------------------------------------------------------------------
// Host dispatch
// ---------------------------------------------------------------------------
bool valid_c(int c) { return c == 4 || c == 8 || c == 16 || c == 32; }

template <int C>
int conv_fwd_c(const snnflow_conv_fwd_args& a, hipStream_t s) {
    const dim3 grid(snnflow_conv_blocks(a.B, a.H, a.W)), block(NT);
    if (a.lif_in) {
        if (a.cin != C) SNN_FAIL(SNNFLOW_E_CHANNELS, "conv_fwd: lif_in requires cin == c");
        if (a.wt_rec) hipLaunchKernelGGL((k_conv_fwd<C, C, true, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((k_conv_fwd<C, C, true, false>), grid, block, 0, s, a);
    } else if (a.wt_rec) {
        if (a.cin != C) SNN_FAIL(SNNFLOW_E_CHANNELS, "conv_fwd: recurrent cell requires cin == c");
        hipLaunchKernelGGL((k_conv_fwd<C, C, false, true>), grid, block, 0, s, a);
    } else {
        if (a.cin == 1) hipLaunchKernelGGL((k_conv_fwd<1, C, false, false>), grid, block, 0, s, a);
        else if (a.cin == 2) hipLaunchKernelGGL((k_conv_fwd<2, C, false, false>), grid, block, 0, s, a);
        else if (a.cin == 4) hipLaunchKernelGGL((k_conv_fwd<4, C, false, false>), grid, block, 0, s, a);
        else if (a.cin == 5) hipLaunchKernelGGL((k_conv_fwd<5, C, false, false>), grid, block, 0, s, a);
        else if (a.cin == C) hipLaunchKernelGGL((k_conv_fwd<C, C, false, false>), grid, block, 0, s, a);
        else SNN_FAIL(SNNFLOW_E_CHANNELS, "conv_fwd: unsupported cin");
    }
    SNN_CHECK_LAUNCH();
    return 0;
}

template <int C>
int layer_bwd_c(const snnflow_layer_bwd_args& a, hipStream_t s) {
    const dim3 grid(snnflow_conv_blocks(a.B, a.H, a.W)), block(NT);
    if (a.lif_in) {
        if (a.cin != C) SNN_FAIL(SNNFLOW_E_CHANNELS, "layer_bwd: lif_in requires cin == c");
        if (a.wt_bwd_rec) hipLaunchKernelGGL((k_layer_bwd<C, C, true, true>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((k_layer_bwd<C, C, true, false>), grid, block, 0, s, a);
    } else if (a.wt_bwd_rec) {
        if (a.cin != C) SNN_FAIL(SNNFLOW_E_CHANNELS, "layer_bwd: recurrent cell requires cin == c");
        hipLaunchKernelGGL((k_layer_bwd<C, C, false, true>), grid, block, 0, s, a);
    } else {
        if (a.cin == 1) hipLaunchKernelGGL((k_layer_bwd<1, C, false, false>), grid, block, 0, s, a);
        else if (a.cin == 2) hipLaunchKernelGGL((k_layer_bwd<2, C, false, false>), grid, block, 0, s, a);
        else if (a.cin == 4) hipLaunchKernelGGL((k_layer_bwd<4, C, false, false>), grid, block, 0, s, a);
        else if (a.cin == 5) hipLaunchKernelGGL((k_layer_bwd<5, C, false, false>), grid, block, 0, s, a);
        else if (a.cin == C) hipLaunchKernelGGL((k_layer_bwd<C, C, false, false>), grid, block, 0, s, a);
        else SNN_FAIL(SNNFLOW_E_CHANNELS, "layer_bwd: unsupported cin");
    }
    SNN_CHECK_LAUNCH();
    return 0;
}

int elem_grid(int64_t n) {
    int64_t g = (n + NT - 1) / NT;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" {

int snnflow_abi_version(void) { return SNNFLOW_ABI_VERSION; }
const char* snnflow_last_error(void) { return g_err.c_str(); }

int snnflow_conv_blocks(int B, int H, int W) { return B * tiles_per_image(H, W); }

int snnflow_prep_weights(const float* w, int c, int cin, float* wt_fwd, float* wt_bwd, float* threshold,
                         void* stream) {
    if (c <= 0 || cin <= 0 || (w && (!wt_fwd || !wt_bwd)) || (!w && !threshold))
        SNN_FAIL(SNNFLOW_E_ARG, "prep_weights: bad args");
    const int n = c * cin * 9;
    hipLaunchKernelGGL(k_prep_weights, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, w, c, cin, wt_fwd,
                       wt_bwd, threshold);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_conv_fwd(const snnflow_conv_fwd_args* a, void* stream) {
    if (!a || a->B <= 0 || a->H <= 0 || a->W <= 0 || !a->wt_ff || !a->y)
        SNN_FAIL(SNNFLOW_E_ARG, "conv_fwd: bad args");
    if (a->lif_in ? (!a->prev_y || !a->prev_state || (a->prev.bn_train && !a->prev_acc)) : !a->x)
        SNN_FAIL(SNNFLOW_E_ARG, "conv_fwd: missing input");
    const hipStream_t s = (hipStream_t)stream;
    switch (a->c) {
        case 4: return conv_fwd_c<4>(*a, s);
        case 8: return conv_fwd_c<8>(*a, s);
        case 16: return conv_fwd_c<16>(*a, s);
        case 32: return conv_fwd_c<32>(*a, s);
        default: SNN_FAIL(SNNFLOW_E_CHANNELS, "conv_fwd: c must be 4, 8, 16 or 32");
    }
}

int snnflow_lif_fwd(const snnflow_lif_fwd_args* a, void* stream) {
    if (!a || !a->y || !a->state || a->B <= 0 || a->H <= 0 || a->W <= 0 || (a->n.bn_train && !a->acc))
        SNN_FAIL(SNNFLOW_E_ARG, "lif_fwd: bad args");
    if (a->pred_w && (!a->pred_b || !a->flow)) SNN_FAIL(SNNFLOW_E_ARG, "lif_fwd: pred needs bias and flow");
    const hipStream_t s = (hipStream_t)stream;
    const dim3 grid(elem_grid((int64_t)a->B * a->H * a->W)), block(NT);
    const bool pred = a->pred_w != nullptr;
    switch (a->c) {
#define LIF_FWD_CASE(CC)                                                                     \
    case CC:                                                                                 \
        if (pred) hipLaunchKernelGGL((k_lif_fwd<CC, true>), grid, block, 0, s, *a);          \
        else hipLaunchKernelGGL((k_lif_fwd<CC, false>), grid, block, 0, s, *a);              \
        break;
        LIF_FWD_CASE(4) LIF_FWD_CASE(8) LIF_FWD_CASE(16) LIF_FWD_CASE(32)
#undef LIF_FWD_CASE
        default: SNN_FAIL(SNNFLOW_E_CHANNELS, "lif_fwd: c must be 4, 8, 16 or 32");
    }
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_lif_bwd(const snnflow_lif_bwd_args* a, void* stream) {
    if (!a || !a->y || !a->stats || !a->g_cur || !a->acc) SNN_FAIL(SNNFLOW_E_ARG, "lif_bwd: bad args");
    const bool pred = a->pred_w != nullptr;
    if (pred && !a->flow) SNN_FAIL(SNNFLOW_E_ARG, "lif_bwd: pred needs flow");
    const hipStream_t s = (hipStream_t)stream;
    const dim3 grid(elem_grid((int64_t)a->B * a->H * a->W)), block(NT);
    switch (a->c) {
#define LIF_BWD_CASE(CC)                                                                     \
    case CC:                                                                                 \
        if (pred) hipLaunchKernelGGL((k_lif_bwd<CC, true>), grid, block, 0, s, *a);          \
        else hipLaunchKernelGGL((k_lif_bwd<CC, false>), grid, block, 0, s, *a);              \
        break;
        LIF_BWD_CASE(4) LIF_BWD_CASE(8) LIF_BWD_CASE(16) LIF_BWD_CASE(32)
#undef LIF_BWD_CASE
        default: SNN_FAIL(SNNFLOW_E_CHANNELS, "lif_bwd: c must be 4, 8, 16 or 32");
    }
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_layer_bwd(const snnflow_layer_bwd_args* a, void* stream) {
    if (!a || !a->y || !a->stats || !a->g_cur || !a->acc_in || !a->x || !a->slab_ff)
        SNN_FAIL(SNNFLOW_E_ARG, "layer_bwd: bad args");
    if (!a->ng.bn_weight || !a->ng.bn_bias || !a->ng.beta || !a->ng.threshold)
        SNN_FAIL(SNNFLOW_E_ARG, "layer_bwd: missing parameter-gradient buffers");
    if (a->has_pred && (!a->g_pred_w || !a->g_pred_b)) SNN_FAIL(SNNFLOW_E_ARG, "layer_bwd: pred gradients");
    if (a->wt_bwd_rec && !a->slab_rec) SNN_FAIL(SNNFLOW_E_ARG, "layer_bwd: recurrent layer needs slab_rec");
    if (a->lif_in && (!a->wt_bwd_ff || !a->prev_y || !a->prev_stats || !a->prev_g_cur || !a->acc_out))
        SNN_FAIL(SNNFLOW_E_ARG, "layer_bwd: lif_in needs previous-layer buffers");
    const hipStream_t s = (hipStream_t)stream;
    switch (a->c) {
        case 4: return layer_bwd_c<4>(*a, s);
        case 8: return layer_bwd_c<8>(*a, s);
        case 16: return layer_bwd_c<16>(*a, s);
        case 32: return layer_bwd_c<32>(*a, s);
        default: SNN_FAIL(SNNFLOW_E_CHANNELS, "layer_bwd: c must be 4, 8, 16 or 32");
    }
}

int snnflow_slab_reduce(const snnflow_slab_desc* d, int n, int nblk, void* stream) {
    if (!d || n <= 0 || n > SNNFLOW_MAX_SLABS || nblk <= 0) SNN_FAIL(SNNFLOW_E_ARG, "slab_reduce: bad args");
    snnflow_slab_desc ds[16] = {};
    int maxe = 0;
    for (int i = 0; i < n; ++i) {
        ds[i] = d[i];
        if (!d[i].slab || !d[i].out || d[i].elems <= 0) SNN_FAIL(SNNFLOW_E_ARG, "slab_reduce: bad descriptor");
        maxe = d[i].elems > maxe ? d[i].elems : maxe;
    }
    hipLaunchKernelGGL(k_slab_reduce, dim3((maxe + 255) / 256, n), dim3(256), 0, (hipStream_t)stream, ds[0], ds[1],
                       ds[2], ds[3], ds[4], ds[5], ds[6], ds[7], ds[8], ds[9], ds[10], ds[11], ds[12], ds[13], ds[14],
                       ds[15], nblk);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_lif_export(const float* x, const float* mem, const float* beta, const float* thr, int N, int C, int HW,
                       float* spk, float* mem_out, void* stream) {
    if (!x || !mem || !beta || !thr || !spk || !mem_out || N < 0 || C <= 0 || HW <= 0)
        SNN_FAIL(SNNFLOW_E_ARG, "lif_export: bad args");
    const int64_t total = (int64_t)N * C * HW;
    if (total == 0) return 0;
    int g = elem_grid(total);
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_lif_export, dim3(g), dim3(NT), 0, (hipStream_t)stream, x, mem, beta, thr, total, C, HW, spk,
                       mem_out);
    SNN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
