// Evaluation-path kernels for gfx950: images of warped events for visualisation /
// deblurring (utils/iwe.py:96-150 deblur_events, compute_pol_iwe; called per window by
// eval_flow.py:220-230) and the average endpoint error (loss/flow.py:597-649 AEE).
#include <cmath>

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

__global__ __launch_bounds__(NT) void k_pol_iwe(const float* __restrict__ events, const float* __restrict__ flow,
                                               const float* __restrict__ pol, int64_t pol_stride, int nimg, int B,
                                               int N, int H, int W, float tref, float s, int round_idx,
                                               float* out) {
    const int64_t n = (int64_t)B * N, HWp = (int64_t)H * W;
    for (int64_t e = (int64_t)blockIdx.x * NT + threadIdx.x; e < n; e += (int64_t)gridDim.x * NT) {
        const int b = (int)(e / N);
        const float* ev = events + e * 4;
        const float ts = ev[0], y = ev[1], x = ev[2];
        const int64_t fpix = (int64_t)(y * (float)W + x);  // deblur_events: flow_idx.long()
        const float* fl = flow + (int64_t)b * 2 * HWp;
        const float fy = fl[HWp + fpix], fx = fl[fpix];
        float* img = out + (int64_t)b * nimg * HWp;
        float m[2] = {1.0f, 1.0f};
        if (pol)
            for (int k = 0; k < nimg; ++k) m[k] = pol[e * pol_stride + k];
        if (round_idx) {
            const float dt = tref - ts;
            const float wy = y + (dt * fy) * s, wx = x + (dt * fx) * s;
            const float cy = rintf(wy), cx = rintf(wx);  // torch.round: half to even
            const bool inb = cy >= 0.0f && cy < (float)H && cx >= 0.0f && cx < (float)W;
            const float mk = inb ? 1.0f : 0.0f;
            const int idx = (int)((cy * mk) * (float)W + cx * mk);
            for (int k = 0; k < nimg; ++k) {
                const float v = mk * m[k];
                if (v != 0.0f) atomicAdd(img + k * HWp + idx, v);
            }
        } else {
            Corner c[4];
            float wy, wx;
            warp4(ts, y, x, fy, fx, tref, s, H, W, c, wy, wx);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                for (int k = 0; k < nimg; ++k) {
                    const float v = c[q].wt * m[k];
                    if (v != 0.0f) atomicAdd(img + k * HWp + c[q].idx, v);
                }
        }
    }
}

// per pixel: endpoint error and validity; per-sample sums (fp64 atomics): acc[2b] = sum err,
// acc[2b+1] = sum valid, acc[2B] = outliers over the batch.  blocks: B * chunks.
__global__ __launch_bounds__(NT) void k_aee(snnflow_aee_args a, int chunks) {
    __shared__ float red[NT / 64][3];
    const int tid = threadIdx.x, b = blockIdx.x / chunks, chunk = blockIdx.x - b * chunks;
    const int64_t HWp = (int64_t)a.H * a.W;
    const int64_t p = (int64_t)chunk * NT + tid;
    float err = 0.0f, val = 0.0f, out = 0.0f;
    if (p < HWp) {
        const float r = a.dt_ratio[b];
        const float* f = a.flow + (int64_t)b * 2 * HWp + p;
        const float* g = a.gtflow + (int64_t)b * 2 * HWp + p;
        const float fx = (f[0] * a.flow_scaling) * r, fy = (f[HWp] * a.flow_scaling) * r;
        const float mag = sqrtf(fx * fx + fy * fy);
        const float dx = fx - g[0], dy = fy - g[HWp];
        const float e = sqrtf(dx * dx + dy * dy);
        const bool valid = a.event_mask[(int64_t)b * HWp + p] != 0.0f && !(g[0] == 0.0f && g[HWp] == 0.0f);
        const float mk = valid ? 1.0f : 0.0f;
        err = e * mk;
        val = mk;
        out = (err > 3.0f && err > 0.05f * (mag * mk)) ? 1.0f : 0.0f;
    }
    const float s0 = wave_total(err), s1 = wave_total(val), s2 = wave_total(out);
    if ((tid & 63) == 0) {
        red[tid >> 6][0] = s0;
        red[tid >> 6][1] = s1;
        red[tid >> 6][2] = s2;
    }
    __syncthreads();
    if (tid < 3) {
        double t = 0.0;
        for (int w = 0; w < NT / 64; ++w) t += (double)red[w][tid];
        atomicAdd(tid < 2 ? a.acc + 2 * b + tid : a.acc + 2 * a.B, t);
    }
}

__global__ void k_aee_finalize(snnflow_aee_args a) {
    const int b = threadIdx.x;
    if (b >= a.B) return;
    const float nvalid = (float)a.acc[2 * b + 1];
    a.aee[b] = (float)a.acc[2 * b] / (nvalid + 1e-9f);
    a.percent[b] = (float)a.acc[2 * a.B] / (nvalid + 1e-9f);
}

__global__ void k_zero_f64(double* p, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) p[i] = 0.0;
}

}  // namespace

extern "C" {

int snnflow_pol_iwe(const float* events, const float* flow, const float* pol, int64_t pol_stride, int nimg, int B,
                    int N, int H, int W, float tref, float flow_scaling, int round_idx, float* out, void* stream) {
    if (!events || !flow || !out || B <= 0 || N < 0 || H <= 0 || W <= 0 || nimg < 1 || nimg > 2 ||
        (nimg == 2 && !pol))
        SNN_FAIL(SNNFLOW_E_ARG, "pol_iwe: bad args");
    const hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(out, 0, sizeof(float) * (size_t)B * nimg * H * W, s);
    if (e != hipSuccess) SNN_FAIL((int)e, hipGetErrorString(e));
    const int64_t n = (int64_t)B * N;
    if (n == 0) return 0;
    int64_t g = (n + NT - 1) / NT;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_pol_iwe, dim3((unsigned)g), dim3(NT), 0, s, events, flow, pol, pol_stride, nimg, B, N, H, W,
                       tref, flow_scaling, round_idx, out);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_aee(const snnflow_aee_args* a, void* stream) {
    if (!a || a->B <= 0 || a->B > NT || a->H <= 0 || a->W <= 0 || !a->flow || !a->gtflow || !a->event_mask ||
        !a->dt_ratio || !a->acc || !a->aee || !a->percent)
        SNN_FAIL(SNNFLOW_E_ARG, "aee: bad args");
    const hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_zero_f64, dim3(1), dim3(NT), 0, s, a->acc, 2 * a->B + 1);
    const int chunks = (int)(((int64_t)a->H * a->W + NT - 1) / NT);
    hipLaunchKernelGGL(k_aee, dim3(a->B * chunks), dim3(NT), 0, s, *a, chunks);
    hipLaunchKernelGGL(k_aee_finalize, dim3(1), dim3(NT), 0, s, *a);
    SNN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
