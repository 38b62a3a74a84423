// Standalone normalisation and pointwise-conv kernels (gfx950) for the cell-by-cell path of the
// LIFFireNet family: MPBN / TEBN cells and the prediction ConvLayer called as modules.
//
// Reference semantics:
//   models/SNNtorch_spiking_submodules.py:66-121  MPBN = BatchNorm2d of the membrane after the
//                                                 (detached) LIF update, state = stack([MPBN(mem), spk])
//   models/SNNtorch_spiking_submodules.py:18-63   TEBN = BatchNorm2d(x) * p[t] (p.mean(0) without t)
//   torch.nn.BatchNorm2d (train: biased batch variance to normalise, unbiased into running_var,
//                         momentum update; eval: running statistics)
//   models/submodules.py:16-113                   ConvLayer (1x1 conv + bias + activation)
//
// Layout: BatchNorm works on [P][C] channel-fastest rows (the NHWC state halves of the cells);
// batch sums are fp64, per-block partials summed in a fixed order (deterministic).
#include <cmath>

#include "snnflow_dev.h"

int snnflow_set_error(int code, const char* msg);
#define SNN_FAIL(code, msg) return snnflow_set_error((code), (msg))
#define SNN_CHECK_LAUNCH()                                                        \
    do {                                                                          \
        hipError_t e_ = hipGetLastError();                                        \
        if (e_ != hipSuccess) return snnflow_set_error((int)e_, hipGetErrorString(e_)); \
    } while (0)

namespace {

constexpr int BN_NT = 256;

inline int bn_blocks(int64_t P, int C) {
    const int64_t ppb = BN_NT / C;                  // pixels per block iteration
    int64_t nb = (P + ppb * 4 - 1) / (ppb * 4);     // >= 4 pixels per thread
    if (nb > SNNFLOW_BN_PARTS) nb = SNNFLOW_BN_PARTS;
    return nb < 1 ? 1 : (int)nb;
}

// Per-block fp64 partial sums over the block's pixels: part[blk][0][c] = sum a, part[blk][1][c] = sum b.
// MODE 0: a = x, b = x^2.  MODE 1: a = g, b = g * (x - mean) * invstd.
template <int MODE>
__global__ __launch_bounds__(BN_NT) void k_bn_partial(const float* __restrict__ x, const float* __restrict__ g,
                                                      int64_t P, int C, const float* __restrict__ mean,
                                                      const float* __restrict__ invstd, double* part) {
    __shared__ double sa[BN_NT], sb[BN_NT];
    const int t = threadIdx.x, c = t % C, pl = t / C, ppb = BN_NT / C;
    double a = 0.0, b = 0.0;
    float m = 0.f, is = 0.f;
    if (MODE == 1) {
        m = mean[c];
        is = invstd[c];
    }
    for (int64_t p = (int64_t)blockIdx.x * ppb + pl; p < P; p += (int64_t)gridDim.x * ppb) {
        const float v = x[p * C + c];
        if (MODE == 0) {
            a += (double)v;
            b += (double)v * (double)v;
        } else {
            const float gv = g[p * C + c];
            a += (double)gv;
            b += (double)gv * (double)((v - m) * is);
        }
    }
    sa[t] = a;
    sb[t] = b;
    __syncthreads();
    if (t < C) {
        double ra = 0.0, rb = 0.0;
        for (int k = 0; k < ppb; ++k) {
            ra += sa[k * C + t];
            rb += sb[k * C + t];
        }
        part[(int64_t)blockIdx.x * 2 * C + t] = ra;
        part[(int64_t)blockIdx.x * 2 * C + C + t] = rb;
    }
}

// One block: statistics of the batch (train) or of the running buffers (eval) -> save_mean/invstd,
// running-statistics update (torch: unbiased variance, momentum).
__global__ void k_bn_stats(const double* part, int nb, int64_t P, int C, int train, float eps, float momentum,
                           float* running_mean, float* running_var, int64_t* nbt, float* save_mean,
                           float* save_invstd) {
    const int c = threadIdx.x;
    if (c >= C) return;
    if (!train) {
        save_mean[c] = running_mean[c];
        save_invstd[c] = 1.0f / sqrtf(running_var[c] + eps);
        return;
    }
    double s = 0.0, q = 0.0;
    for (int b = 0; b < nb; ++b) {
        s += part[(int64_t)b * 2 * C + c];
        q += part[(int64_t)b * 2 * C + C + c];
    }
    const double mean = s / (double)P;
    double var = q / (double)P - mean * mean;
    if (var < 0.0) var = 0.0;
    save_mean[c] = (float)mean;
    save_invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
    if (running_mean) {
        const double unb = P > 1 ? var * (double)P / (double)(P - 1) : var;
        running_mean[c] = (1.0f - momentum) * running_mean[c] + momentum * (float)mean;
        running_var[c] = (1.0f - momentum) * running_var[c] + momentum * (float)unb;
    }
    if (nbt && c == 0) nbt[0] += 1;
}

__global__ __launch_bounds__(BN_NT) void k_bn_apply(const float* __restrict__ x, int64_t P, int C,
                                                    const float* __restrict__ mean, const float* __restrict__ invstd,
                                                    const float* __restrict__ w, const float* __restrict__ b,
                                                    float* __restrict__ y) {
    const int64_t n = P * C;
    for (int64_t i = (int64_t)blockIdx.x * BN_NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * BN_NT) {
        const int c = (int)(i % C);
        float v = (x[i] - mean[c]) * invstd[c];
        if (w) v = v * w[c];
        if (b) v = v + b[c];
        y[i] = v;
    }
}

// Backward finish: g_weight = sum g*xhat, g_bias = sum g; coefficients for the input gradient into coef
// [3][C] = (w*invstd, mean g, mean g*xhat).
__global__ void k_bn_bwd_sums(const double* part, int nb, int64_t P, int C, const float* w, const float* invstd,
                              int train, float* g_weight, float* g_bias, float* coef) {
    const int c = threadIdx.x;
    if (c >= C) return;
    double s = 0.0, q = 0.0;
    for (int b = 0; b < nb; ++b) {
        s += part[(int64_t)b * 2 * C + c];
        q += part[(int64_t)b * 2 * C + C + c];
    }
    if (g_weight) g_weight[c] = (float)q;
    if (g_bias) g_bias[c] = (float)s;
    coef[c] = (w ? w[c] : 1.0f) * invstd[c];
    coef[C + c] = train ? (float)(s / (double)P) : 0.0f;
    coef[2 * C + c] = train ? (float)(q / (double)P) : 0.0f;
}

__global__ __launch_bounds__(BN_NT) void k_bn_dx(const float* __restrict__ x, const float* __restrict__ g, int64_t P,
                                                 int C, const float* __restrict__ mean,
                                                 const float* __restrict__ invstd, const float* __restrict__ coef,
                                                 float* __restrict__ gx) {
    const int64_t n = P * C;
    for (int64_t i = (int64_t)blockIdx.x * BN_NT + threadIdx.x; i < n; i += (int64_t)gridDim.x * BN_NT) {
        const int c = (int)(i % C);
        const float xh = (x[i] - mean[c]) * invstd[c];
        gx[i] = coef[c] * (g[i] - coef[C + c] - xh * coef[2 * C + c]);
    }
}

inline int grid_for(int64_t n) {
    int64_t gs = (n + BN_NT - 1) / BN_NT;
    if (gs > 8192) gs = 8192;
    return gs < 1 ? 1 : (int)gs;
}

// ---------------------------------------------------------------------------------------------
// 1x1 convolution + bias + activation (ConvLayer as the prediction layer)
// ---------------------------------------------------------------------------------------------
__device__ inline float act_fwd(float v, int act) {
    switch (act) {
        case SNNFLOW_ACT_TANH: return tanhf(v);
        case SNNFLOW_ACT_RELU: return v > 0.f ? v : 0.f;
        case SNNFLOW_ACT_SIGMOID: return 1.0f / (1.0f + expf(-v));
        default: return v;
    }
}

__device__ inline float act_bwd(float out, float pre_pos, int act) {  // d act / d pre from the output
    switch (act) {
        case SNNFLOW_ACT_TANH: return 1.0f - out * out;
        case SNNFLOW_ACT_RELU: return pre_pos;
        case SNNFLOW_ACT_SIGMOID: return out * (1.0f - out);
        default: return 1.0f;
    }
}

__global__ __launch_bounds__(BN_NT) void k_pw_fwd(snnflow_pointwise_args a) {
    const int64_t HW = (int64_t)a.H * a.W, P = (int64_t)a.B * HW;
    const int64_t p = (int64_t)blockIdx.x * BN_NT + threadIdx.x;
    if (p >= P) return;
    const int64_t bi = p / HW, hw = p % HW, h = hw / a.W, w = hw % a.W;
    const float* xp = a.x + bi * a.xs[0] + h * a.xs[2] + w * a.xs[3];
    float acc[SNNFLOW_PW_MAX_COUT];
#pragma unroll
    for (int o = 0; o < SNNFLOW_PW_MAX_COUT; ++o) acc[o] = 0.f;
    for (int ci = 0; ci < a.cin; ++ci) {
        const float v = xp[(int64_t)ci * a.xs[1]];
#pragma unroll
        for (int o = 0; o < SNNFLOW_PW_MAX_COUT; ++o)
            if (o < a.cout) acc[o] = fmaf(a.w[o * a.cin + ci], v, acc[o]);
    }
#pragma unroll
    for (int o = 0; o < SNNFLOW_PW_MAX_COUT; ++o)
        if (o < a.cout) a.out[(bi * a.cout + o) * HW + hw] = act_fwd(acc[o] + (a.b ? a.b[o] : 0.f), a.act);
}

// g_pre = g_out * act'(out); g_x (if any) = W^T g_pre; per-block fp64 partials of dW (cout x cin) and db.
__global__ __launch_bounds__(BN_NT) void k_pw_bwd(snnflow_pointwise_args a, const float* __restrict__ g_out,
                                                  int64_t gs_b, int64_t gs_c, double* part) {
    __shared__ float red[BN_NT / 64][SNNFLOW_PW_MAX_COUT * (SNNFLOW_PW_MAX_CIN + 1)];
    const int64_t HW = (int64_t)a.H * a.W, P = (int64_t)a.B * HW;
    const int nk = a.cout * (a.cin + 1);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int NJ = (SNNFLOW_PW_MAX_COUT * (SNNFLOW_PW_MAX_CIN + 1) + 63) / 64;
    double tot[NJ];  // this thread's share of the block's nk sums (k = lane + 64 j)
#pragma unroll
    for (int j = 0; j < NJ; ++j) tot[j] = 0.0;
    for (int64_t base = (int64_t)blockIdx.x * BN_NT; base < P; base += (int64_t)gridDim.x * BN_NT) {
        const int64_t p = base + threadIdx.x;
        float gp[SNNFLOW_PW_MAX_COUT];
        const float* xp = nullptr;
        int64_t bi = 0, hw = 0;
        if (p < P) {
            bi = p / HW;
            hw = p % HW;
            const int64_t h = hw / a.W, w = hw % a.W;
            xp = a.x + bi * a.xs[0] + h * a.xs[2] + w * a.xs[3];
        }
#pragma unroll
        for (int o = 0; o < SNNFLOW_PW_MAX_COUT; ++o) {
            gp[o] = 0.f;
            if (p < P && o < a.cout) {
                const float out = a.out[(bi * a.cout + o) * HW + hw];
                float pre_pos = 1.f;
                if (a.act == SNNFLOW_ACT_RELU) pre_pos = out > 0.f ? 1.f : 0.f;
                gp[o] = g_out[bi * gs_b + o * gs_c + hw] * act_bwd(out, pre_pos, a.act);
            }
        }
        if (p < P && a.g_x) {
            const int64_t h = hw / a.W, w = hw % a.W;
            float* gxp = a.g_x + bi * a.gxs[0] + h * a.gxs[2] + w * a.gxs[3];
            for (int ci = 0; ci < a.cin; ++ci) {
                float s = 0.f;
#pragma unroll
                for (int o = 0; o < SNNFLOW_PW_MAX_COUT; ++o)
                    if (o < a.cout) s = fmaf(a.w[o * a.cin + ci], gp[o], s);
                gxp[(int64_t)ci * a.gxs[1]] = s;
            }
        }
        // wave sums of gp * x (dW) and gp (db), then the block's waves in a fixed order
        for (int k = 0; k < nk; ++k) {
            const int o = k / (a.cin + 1), ci = k % (a.cin + 1);
            float v = 0.f;
            if (p < P) {
                float go = 0.f;
#pragma unroll
                for (int oo = 0; oo < SNNFLOW_PW_MAX_COUT; ++oo)
                    if (oo == o) go = gp[oo];
                v = ci < a.cin ? go * xp[(int64_t)ci * a.xs[1]] : go;
            }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
            if (lane == 0) red[wv][k] = v;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int k = lane + 64 * j;
            if (wv == 0 && k < nk) {
                double s = 0.0;
                for (int q = 0; q < BN_NT / 64; ++q) s += (double)red[q][k];
                tot[j] += s;
            }
        }
        __syncthreads();
    }
    if (wv == 0)
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int k = lane + 64 * j;
            if (k < nk) part[(int64_t)blockIdx.x * nk + k] = tot[j];
        }
}

__global__ void k_pw_param_grads(const double* part, int nb, int cout, int cin, float* g_w, float* g_b) {
    const int nk = cout * (cin + 1);
    for (int k = threadIdx.x; k < nk; k += blockDim.x) {
        double s = 0.0;
        for (int b = 0; b < nb; ++b) s += part[(int64_t)b * nk + k];
        const int o = k / (cin + 1), ci = k % (cin + 1);
        if (ci < cin) {
            if (g_w) g_w[o * cin + ci] = (float)s;
        } else if (g_b) {
            g_b[o] = (float)s;
        }
    }
}

}  // namespace

extern "C" {

int snnflow_bn_fwd(const snnflow_bn_fwd_args* a, void* stream) {
    if (!a || !a->x || !a->y || a->P <= 0 || a->C <= 0 || a->C > BN_NT || (BN_NT % a->C) != 0 ||
        !a->save_mean || !a->save_invstd)
        SNN_FAIL(SNNFLOW_E_ARG, "bn_fwd: bad arguments (C must divide 256)");
    if (!a->train && (!a->running_mean || !a->running_var)) SNN_FAIL(SNNFLOW_E_ARG, "bn_fwd: eval needs running stats");
    if (a->train && !a->scratch) SNN_FAIL(SNNFLOW_E_ARG, "bn_fwd: scratch missing");
    const hipStream_t s = (hipStream_t)stream;
    const int nb = bn_blocks(a->P, a->C);
    if (a->train)
        hipLaunchKernelGGL(k_bn_partial<0>, dim3(nb), dim3(BN_NT), 0, s, a->x, nullptr, a->P, a->C, nullptr, nullptr,
                           a->scratch);
    hipLaunchKernelGGL(k_bn_stats, dim3(1), dim3(BN_NT), 0, s, a->scratch, nb, a->P, a->C, a->train, a->eps,
                       a->momentum, a->running_mean, a->running_var, a->num_batches_tracked, a->save_mean,
                       a->save_invstd);
    hipLaunchKernelGGL(k_bn_apply, dim3(grid_for(a->P * a->C)), dim3(BN_NT), 0, s, a->x, a->P, a->C, a->save_mean,
                       a->save_invstd, a->weight, a->bias, a->y);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_bn_bwd(const snnflow_bn_bwd_args* a, void* stream) {
    if (!a || !a->x || !a->g || a->P <= 0 || a->C <= 0 || a->C > BN_NT || (BN_NT % a->C) != 0 || !a->save_mean ||
        !a->save_invstd || !a->scratch)
        SNN_FAIL(SNNFLOW_E_ARG, "bn_bwd: bad arguments (C must divide 256)");
    const hipStream_t s = (hipStream_t)stream;
    const int nb = bn_blocks(a->P, a->C);
    float* coef = reinterpret_cast<float*>(a->scratch + (int64_t)SNNFLOW_BN_PARTS * 2 * a->C);
    hipLaunchKernelGGL(k_bn_partial<1>, dim3(nb), dim3(BN_NT), 0, s, a->x, a->g, a->P, a->C, a->save_mean,
                       a->save_invstd, a->scratch);
    hipLaunchKernelGGL(k_bn_bwd_sums, dim3(1), dim3(BN_NT), 0, s, a->scratch, nb, a->P, a->C, a->weight,
                       a->save_invstd, a->train, a->g_weight, a->g_bias, coef);
    if (a->g_x)
        hipLaunchKernelGGL(k_bn_dx, dim3(grid_for(a->P * a->C)), dim3(BN_NT), 0, s, a->x, a->g, a->P, a->C,
                           a->save_mean, a->save_invstd, coef, a->g_x);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_bn_scratch_doubles(int C) { return SNNFLOW_BN_PARTS * 2 * C + (3 * C + 1) / 2 + 1; }

int snnflow_pointwise_fwd(const snnflow_pointwise_args* a, void* stream) {
    if (!a || !a->x || !a->w || !a->out || a->B <= 0 || a->H <= 0 || a->W <= 0 || a->cin <= 0 ||
        a->cin > SNNFLOW_PW_MAX_CIN || a->cout <= 0 || a->cout > SNNFLOW_PW_MAX_COUT || a->act < 0 || a->act > 3)
        SNN_FAIL(SNNFLOW_E_ARG, "pointwise_fwd: bad arguments");
    const int64_t P = (int64_t)a->B * a->H * a->W;
    hipLaunchKernelGGL(k_pw_fwd, dim3((unsigned)((P + BN_NT - 1) / BN_NT)), dim3(BN_NT), 0, (hipStream_t)stream, *a);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_pointwise_bwd(const snnflow_pointwise_args* a, const float* g_out, int64_t gs_b, int64_t gs_c,
                          float* g_w, float* g_b, double* scratch, void* stream) {
    if (!a || !a->x || !a->w || !a->out || !g_out || !scratch || a->B <= 0 || a->H <= 0 || a->W <= 0 ||
        a->cin <= 0 || a->cin > SNNFLOW_PW_MAX_CIN || a->cout <= 0 || a->cout > SNNFLOW_PW_MAX_COUT)
        SNN_FAIL(SNNFLOW_E_ARG, "pointwise_bwd: bad arguments");
    const hipStream_t s = (hipStream_t)stream;
    const int64_t P = (int64_t)a->B * a->H * a->W;
    int64_t nb = (P + BN_NT * 8 - 1) / (BN_NT * 8);
    if (nb > SNNFLOW_BN_PARTS) nb = SNNFLOW_BN_PARTS;
    if (nb < 1) nb = 1;
    hipLaunchKernelGGL(k_pw_bwd, dim3((unsigned)nb), dim3(BN_NT), 0, s, *a, g_out, gs_b, gs_c, scratch);
    hipLaunchKernelGGL(k_pw_param_grads, dim3(1), dim3(BN_NT), 0, s, scratch, (int)nb, a->cout, a->cin, g_w, g_b);
    SNN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
