// On-device event encodings for gfx950: the loader step in front of the network
// (reference dataloader/encodings.py:30-85 events_to_image / events_to_voxel /
// events_to_channels, dataloader/base.py create_mask_encoding / create_polarity_mask),
// batched over samples, one thread per event.  Counts, masks and polarity masks are
// exact (integer-valued fp32 sums); voxel sums follow the atomic arrival order.
#include <cmath>

#include "snnflow_dev.h"

using namespace snnflow;

int snnflow_set_error(int code, const char* msg);
#define SNN_FAIL(code, msg) return snnflow_set_error((code), (msg))
#define SNN_CHECK_LAUNCH()                                                        \
    do {                                                                          \
        hipError_t e_ = hipGetLastError();                                        \
        if (e_ != hipSuccess) return snnflow_set_error((int)e_, hipGetErrorString(e_)); \
    } while (0)

namespace {

__global__ __launch_bounds__(NT) void k_encode(snnflow_encode_args a) {
    const int64_t n = (int64_t)a.B * a.N;
    const int64_t HWp = (int64_t)a.H * a.W;
    for (int64_t e = (int64_t)blockIdx.x * NT + threadIdx.x; e < n; e += (int64_t)gridDim.x * NT) {
        const int b = (int)(e / a.N), i = (int)(e - (int64_t)b * a.N);
        const int64_t o = (int64_t)b * a.batch_stride + (int64_t)i * a.ev_stride;
        const float p = a.ps[o];
        if (a.pol_mask) {
            a.pol_mask[e * 2] = p < 0.0f ? 0.0f : p;
            a.pol_mask[e * 2 + 1] = (p > 0.0f ? 0.0f : p) * -1.0f;
        }
        const float yf = a.ys[o], xf = a.xs[o];
        const int64_t yi = (int64_t)yf, xi = (int64_t)xf;  // .long(): truncation toward zero
        if (yi < 0 || yi >= a.H || xi < 0 || xi >= a.W) continue;
        const int64_t pix = yi * a.W + xi;
        if (a.cnt) {
            float* c = a.cnt + (int64_t)b * 2 * HWp + pix;
            const float pos = p * (p < 0.0f ? 0.0f : p), neg = p * (p > 0.0f ? 0.0f : p);
            if (pos != 0.0f) atomicAdd(c, pos);
            if (neg != 0.0f) atomicAdd(c + HWp, neg);
        }
        if (a.mask) a.mask[(int64_t)b * HWp + pix] = fabsf(p);
        if (a.image) {
            float* im = a.image + (int64_t)b * HWp + pix;
            if (a.accumulate) atomicAdd(im, p);
            else *im = p;
        }
        if (a.voxel) {
            float t = a.ts[o] * (float)(a.num_bins - 1);
            if (a.round_ts) t = rintf(t);  // torch.round: half to even
            float* v = a.voxel + (int64_t)b * a.num_bins * HWp + pix;
            for (int k = 0; k < a.num_bins; ++k) {
                const float w = fmaxf(0.0f, 1.0f - fabsf(t - (float)k));
                if (w != 0.0f) atomicAdd(v + k * HWp, p * w);
            }
        }
    }
}

}  // namespace

extern "C" int snnflow_encode_events(const snnflow_encode_args* a, void* stream) {
    if (!a || a->B <= 0 || a->N < 0 || a->H <= 0 || a->W <= 0 || !a->ps || !a->ys || !a->xs ||
        (a->voxel && (!a->ts || a->num_bins < 1)))
        SNN_FAIL(SNNFLOW_E_ARG, "encode_events: bad args");
    const hipStream_t s = (hipStream_t)stream;
    const size_t HWp = (size_t)a->H * a->W;
    hipError_t e = hipSuccess;
    if (a->cnt && e == hipSuccess) e = hipMemsetAsync(a->cnt, 0, sizeof(float) * a->B * 2 * HWp, s);
    if (a->voxel && e == hipSuccess) e = hipMemsetAsync(a->voxel, 0, sizeof(float) * a->B * a->num_bins * HWp, s);
    if (a->image && e == hipSuccess) e = hipMemsetAsync(a->image, 0, sizeof(float) * a->B * HWp, s);
    if (a->mask && e == hipSuccess) e = hipMemsetAsync(a->mask, 0, sizeof(float) * a->B * HWp, s);
    if (e != hipSuccess) SNN_FAIL((int)e, hipGetErrorString(e));
    const int64_t n = (int64_t)a->B * a->N;
    if (n == 0) return 0;
    int64_t g = (n + NT - 1) / NT;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_encode, dim3((unsigned)g), dim3(NT), 0, s, *a);
    SNN_CHECK_LAUNCH();
    return 0;
}
