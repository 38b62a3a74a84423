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

// Banded form (snnflow_pol_iwe): one block per (sample, band of POLB_BAND pixels) holds the band's
// nimg images in LDS, scans the sample's events, adds the contributions that land in the band with
// LDS atomics, and writes the whole band once -- no memset launch, no global atomics.  Rounded
// warps with 0/1 masks add exact integers (order-free); bilinear weights add in LDS-atomic order,
// as the global atomics of k_pol_iwe did.
constexpr int POLB_NT = 1024, POLB_BAND = 4096;  // ~1 event per thread at 1000-event windows: one load chain

__global__ __launch_bounds__(POLB_NT) void k_pol_iwe_band(const float* __restrict__ events, const float* __restrict__ flow,
                                                         const float* __restrict__ pol, int64_t pol_stride, int nimg,
                                                         int N, int H, int W, float tref, float s, int round_idx,
                                                         int nbands, float* out) {
    __shared__ float img[2][POLB_BAND];
    const int tid = threadIdx.x, band = blockIdx.x % nbands, b = blockIdx.x / nbands;
    const int64_t HWp = (int64_t)H * W;
    const int p0 = band * POLB_BAND;
    const int np = (int)(HWp - p0 < POLB_BAND ? HWp - p0 : POLB_BAND);
    for (int j = tid; j < 2 * POLB_BAND; j += POLB_NT) (&img[0][0])[j] = 0.0f;
    __syncthreads();
    const float* fl = flow + (int64_t)b * 2 * HWp;
    for (int i = tid; i < N; i += POLB_NT) {
        const int64_t e = (int64_t)b * N + i;
        const float* ev = events + e * 4;  // (event views need not be 16-B aligned)
        const float ts = ev[0], y = ev[1], x = ev[2];
        const int64_t fpix = (int64_t)(y * (float)W + x);  // deblur_events: flow_idx.long()
        const float fy = fl[HWp + fpix], fx = fl[fpix];
        float m[2] = {1.0f, 1.0f};
        if (pol)
            for (int k = 0; k < nimg; ++k) m[k] = pol[e * pol_stride + k];
        if (round_idx) {
            const float dt = tref - ts;
            const float wy = y + (dt * fy) * s, wx = x + (dt * fx) * s;
            const float cy = rintf(wy), cx = rintf(wx);  // torch.round: half to even
            const bool inb = cy >= 0.0f && cy < (float)H && cx >= 0.0f && cx < (float)W;
            const float mk = inb ? 1.0f : 0.0f;
            const int li = (int)((cy * mk) * (float)W + cx * mk) - p0;
            if (li >= 0 && li < np)
                for (int k = 0; k < nimg; ++k) {
                    const float v = mk * m[k];
                    if (v != 0.0f) atomicAdd(&img[k][li], v);
                }
        } else {
            Corner c[4];
            float wy, wx;
            warp4(ts, y, x, fy, fx, tref, s, H, W, c, wy, wx);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int li = c[q].idx - p0;
                if (li < 0 || li >= np) continue;
                for (int k = 0; k < nimg; ++k) {
                    const float v = c[q].wt * m[k];
                    if (v != 0.0f) atomicAdd(&img[k][li], v);
                }
            }
        }
    }
    __syncthreads();
    for (int k = 0; k < nimg; ++k)
        for (int j = tid; j < np; j += POLB_NT) out[((int64_t)b * nimg + k) * HWp + p0 + j] = img[k][j];
}

// AEE in one launch.  Per pixel: endpoint error, validity, outlier; per (sample, slice of
// AEE_NT * AEE_PPT pixels) block one fp64 row {sum err, sum valid, outliers} at acc[1 + 3 blk]; the
// last block to finish (completion counter acc[0]) sums every sample's rows in slice order, writes
// aee / percent (the outliers counted over the whole batch, loss/flow.py:647) and resets the
// counter: deterministic, no zero / finalize launches.  Few large blocks: each block's release
// fence writes its XCD's L2 back, so the block count is kept near one per sample.
constexpr int AEE_NT = 1024, AEE_PPT = 4;

__host__ __device__ inline int aee_slices(int64_t HWp) {
    return (int)((HWp + (int64_t)AEE_NT * AEE_PPT - 1) / ((int64_t)AEE_NT * AEE_PPT));
}

__global__ __launch_bounds__(AEE_NT) void k_aee(snnflow_aee_args a, int slices) {
    __shared__ double red[AEE_NT / 64][3];
    __shared__ double smp[AEE_NT][3];  // B <= AEE_NT (host check)
    __shared__ int last;
    const int tid = threadIdx.x, b = blockIdx.x / slices, sl = blockIdx.x - b * slices;
    const int64_t HWp = (int64_t)a.H * a.W;
    const int64_t p0 = (int64_t)sl * AEE_NT * AEE_PPT + tid;
    const float r = a.dt_ratio ? a.dt_ratio[b] : a.dt_gt[a.dt_gt_n == 1 ? 0 : b] / a.dt_input[a.dt_input_n == 1 ? 0 : b];
    const float* f = a.flow + (int64_t)b * 2 * HWp;
    const float* g = a.gtflow + (int64_t)b * 2 * HWp;
    const float* em = a.event_mask + (int64_t)b * HWp;
    // every load of the thread's AEE_PPT pixels first (one memory latency), then the math
    float fx_[AEE_PPT], fy_[AEE_PPT], gx_[AEE_PPT], gy_[AEE_PPT], m_[AEE_PPT];
#pragma unroll
    for (int u = 0; u < AEE_PPT; ++u) {
        const int64_t p = p0 + (int64_t)u * AEE_NT;
        const bool ok = p < HWp;
        fx_[u] = ok ? f[p] : 0.0f;
        fy_[u] = ok ? f[HWp + p] : 0.0f;
        gx_[u] = ok ? g[p] : 0.0f;
        gy_[u] = ok ? g[HWp + p] : 0.0f;
        m_[u] = ok ? em[p] : 0.0f;
    }
    float err = 0.0f, val = 0.0f, out = 0.0f;
#pragma unroll
    for (int u = 0; u < AEE_PPT; ++u) {
        const float fx = (fx_[u] * a.flow_scaling) * r, fy = (fy_[u] * a.flow_scaling) * r;
        const float gx = gx_[u], gy = gy_[u];
        const float mag = sqrtf(fx * fx + fy * fy);
        const float dx = fx - gx, dy = fy - gy;
        const float e = sqrtf(dx * dx + dy * dy);
        const bool valid = m_[u] != 0.0f && !(gx == 0.0f && gy == 0.0f);  // (m_ = 0 past the image)
        const float mk = valid ? 1.0f : 0.0f;
        const float ae = e * mk;
        err += ae;
        val += mk;
        out += (ae > 3.0f && ae > 0.05f * (mag * mk)) ? 1.0f : 0.0f;
    }
    // per-thread sums of <= AEE_PPT pixels in fp32 (counts exact), across threads in fp64
    double s0 = err, s1 = val, s2 = out;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        s0 += __shfl_xor(s0, off, 64);
        s1 += __shfl_xor(s1, off, 64);
        s2 += __shfl_xor(s2, off, 64);
    }
    if ((tid & 63) == 0) {
        red[tid >> 6][0] = s0;
        red[tid >> 6][1] = s1;
        red[tid >> 6][2] = s2;
    }
    __syncthreads();
    // wave 0 writes the block's row, fences it device-wide (one wave per block: a fence is an L2
    // write-back + invalidate, and every wave of every block fencing cost ~15 us here), then counts
    // the block as done; the last block's wave 0 fences again (acquire) before the rows are read
    if (tid < 64) {
        if (tid < 3) {
            double t = 0.0;
            for (int w = 0; w < AEE_NT / 64; ++w) t += red[w][tid];
            a.acc[1 + 3 * (int64_t)blockIdx.x + tid] = t;
        }
        __threadfence();
        if (tid == 0) {
            const unsigned long long done = atomicAdd(reinterpret_cast<unsigned long long*>(a.acc), 1ull);
            last = done == (unsigned long long)gridDim.x - 1;
            if (last) __threadfence();
        }
    }
    __syncthreads();
    if (!last) return;
    if (tid < a.B) {
        double e = 0.0, v = 0.0, o = 0.0;
        const double* rr = a.acc + 1 + 3 * (int64_t)tid * slices;
        for (int c = 0; c < slices; ++c) {
            e += rr[3 * c];
            v += rr[3 * c + 1];
            o += rr[3 * c + 2];
        }
        smp[tid][0] = e;
        smp[tid][1] = v;
        smp[tid][2] = o;
    }
    __syncthreads();
    if (tid < a.B) {
        double outl = 0.0;
        for (int bb = 0; bb < a.B; ++bb) outl += smp[bb][2];
        const float nvalid = (float)smp[tid][1];
        a.aee[tid] = (float)smp[tid][0] / (nvalid + 1e-9f);
        a.percent[tid] = (float)outl / (nvalid + 1e-9f);
    }
    if (tid == 0) *reinterpret_cast<unsigned long long*>(a.acc) = 0ull;
}

// All flow metrics (snnflow.h, snnflow_flow_metrics): one row of FM_NV per-block sums per
// (sample, chunk of NT pixels):
//   0 nvalid  1 aee  2 aee outliers  3 nee  4 nee outliers  5 aae  6 aae outliers  7 naae
//   8..11 masked sums of f'x, f'y, gx, gy   12 ang*|f'| (all pixels)  13 |f'|*valid
//   14 ang * (valid && |f'| >= thr)  15 (valid && |f'| >= thr)
constexpr int FM_NV = 16;
constexpr float kClampLo = -1.0f + 1e-5f, kClampHi = 1.0f - 1e-5f;

__global__ __launch_bounds__(NT) void k_flow_metrics(snnflow_flow_metrics_args a, int chunks) {
    __shared__ float red[NT / 64][FM_NV];
    const int tid = threadIdx.x, b = blockIdx.x / chunks, chunk = blockIdx.x - b * chunks;
    const int64_t HWp = (int64_t)a.H * a.W;
    const int64_t p = (int64_t)chunk * NT + tid;
    float v[FM_NV];
#pragma unroll
    for (int j = 0; j < FM_NV; ++j) v[j] = 0.0f;
    if (p < HWp) {
        const float r = a.dt_ratio[b];
        const float* f = a.flow + (int64_t)b * 2 * HWp + p;
        const float* g = a.gtflow + (int64_t)b * 2 * HWp + p;
        const float fx = (f[0] * a.flow_scaling) * r, fy = (f[HWp] * a.flow_scaling) * r;
        const float gx = g[0], gy = g[HWp];
        const float fn = sqrtf(fx * fx + fy * fy), gn = sqrtf(gx * gx + gy * gy);
        const float dx = fx - gx, dy = fy - gy;
        const float e = sqrtf(dx * dx + dy * dy);
        const bool valid = a.event_mask[(int64_t)b * HWp + p] != 0.0f && !(gx == 0.0f && gy == 0.0f);
        const float mk = valid ? 1.0f : 0.0f;
        const float dot = fx * gx + fy * gy;
        // AEE (:609-649)
        const float ae = e * mk;
        v[0] = mk;
        v[1] = ae;
        v[2] = (ae > 3.0f && ae > 0.05f * (fn * mk)) ? 1.0f : 0.0f;
        // NEE (:663-701)
        const float ne = (e / (fminf(fn, gn) + 0.01f)) * mk;
        v[3] = ne;
        v[4] = ne > 0.5f ? 1.0f : 0.0f;
        // AAE (:715-762), the reference's cosine formula
        const float aa = acosf(fminf(fmaxf((fn * gn) / (dot + 0.01f), kClampLo), kClampHi)) * mk;
        v[5] = aa;
        v[6] = aa > (float)(3.14159265358979323846 / 6.0) ? 1.0f : 0.0f;
        // angular error with the normalised cosine (NAAE, AAE_Weighted, AAE_Filtered)
        const float ang = acosf(fminf(fmaxf(dot / (fn * gn + 1e-9f), kClampLo), kClampHi));
        v[7] = (ang / (fn + 1e-9f)) * mk;
        // AE_ofMeans (:835-883)
        v[8] = fx * mk;
        v[9] = fy * mk;
        v[10] = gx * mk;
        v[11] = gy * mk;
        // AAE_Weighted (:888-909): numerator over every pixel
        v[12] = ang * fn;
        v[13] = fn * mk;
        // AAE_Filtered (:917-937)
        const float mf = (valid && fn >= a.mag_threshold) ? 1.0f : 0.0f;
        v[14] = ang * mf;
        v[15] = mf;
    }
    const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
    for (int j = 0; j < FM_NV; ++j) {
        const float s = wave_total(v[j]);
        if (lane == 0) red[wv][j] = s;
    }
    __syncthreads();
    if (tid < FM_NV) {
        double t = 0.0;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) t += (double)red[w][tid];
        a.rows[(int64_t)blockIdx.x * FM_NV + tid] = t;
    }
}

// Fixed-order reduction of the rows: wave w owns samples w, w + 4, ...; then the metrics.
__global__ __launch_bounds__(NT) void k_flow_metrics_finalize(snnflow_flow_metrics_args a, int chunks) {
    __shared__ double sums[NT][FM_NV];  // B <= NT (host check)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int b = wv; b < a.B; b += NT / 64) {
        double s[FM_NV];
#pragma unroll
        for (int j = 0; j < FM_NV; ++j) s[j] = 0.0;
        const double* r = a.rows + (int64_t)b * chunks * FM_NV;
#pragma unroll 2
        for (int c = lane; c < chunks; c += 64) {
#pragma unroll
            for (int j = 0; j < FM_NV; ++j) s[j] += r[(int64_t)c * FM_NV + j];
        }
#pragma unroll
        for (int j = 0; j < FM_NV; ++j) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) s[j] += __shfl_xor(s[j], off, 64);
        }
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < FM_NV; ++j) sums[b][j] = s[j];
        }
    }
    __syncthreads();
    const int b = threadIdx.x;
    if (b >= a.B) return;
    double aee_out = 0.0, nee_out = 0.0;  // the reference counts these over the whole batch
    for (int bb = 0; bb < a.B; ++bb) {
        aee_out += sums[bb][2];
        nee_out += sums[bb][4];
    }
    const double* s = sums[b];
    const float nv = (float)s[0], den = nv + 1e-9f;
    float* o = a.out + (int64_t)b * SNNFLOW_NUM_METRICS;
    o[SNNFLOW_M_AEE] = (float)s[1] / den;
    o[SNNFLOW_M_AEE_PCT] = (float)aee_out / den;
    o[SNNFLOW_M_NEE] = (float)s[3] / den;
    o[SNNFLOW_M_NEE_PCT] = (float)nee_out / den;
    o[SNNFLOW_M_AAE] = (float)s[5] / den;
    o[SNNFLOW_M_AAE_PCT] = (float)s[6] / den;
    o[SNNFLOW_M_NAAE] = (float)s[7] / den;
    const float mfx = (float)s[8] / den, mfy = (float)s[9] / den, mgx = (float)s[10] / den, mgy = (float)s[11] / den;
    const float mfn = sqrtf(mfx * mfx + mfy * mfy), mgn = sqrtf(mgx * mgx + mgy * mgy);
    o[SNNFLOW_M_AE_OF_MEANS] = acosf(fminf(fmaxf((mfx * mgx + mfy * mgy) / (mfn * mgn + 1e-9f), kClampLo), kClampHi));
    o[SNNFLOW_M_AAE_WEIGHTED] = (float)s[12] / ((float)s[13] + 1e-9f);
    o[SNNFLOW_M_AAE_FILTERED] = (float)s[14] / ((float)s[15] + 1e-9f);
}

}  // namespace

extern "C" {

int snnflow_pol_iwe(const float* events, const float* flow, const float* pol, int64_t pol_stride, int nimg, int B,
                    int N, int H, int W, float tref, float flow_scaling, int round_idx, float* out, void* stream) {
    if (!events || !flow || !out || B <= 0 || N < 0 || H <= 0 || W <= 0 || nimg < 1 || nimg > 2 ||
        (nimg == 2 && !pol))
        SNN_FAIL(SNNFLOW_E_ARG, "pol_iwe: bad args");
    const hipStream_t s = (hipStream_t)stream;
    const int64_t HWp = (int64_t)H * W, nbands = (HWp + POLB_BAND - 1) / POLB_BAND;
    if ((int64_t)B * nbands <= 65535 * 64 && N <= 65536) {  // banded: every block scans its sample's events
        hipLaunchKernelGGL(k_pol_iwe_band, dim3((unsigned)(B * nbands)), dim3(POLB_NT), 0, s, events, flow, pol, pol_stride,
                           nimg, N, H, W, tref, flow_scaling, round_idx, (int)nbands, out);
        SNN_CHECK_LAUNCH();
        return 0;
    }
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
    if (!a || a->B <= 0 || a->B > AEE_NT || a->H <= 0 || a->W <= 0 || !a->flow || !a->gtflow || !a->event_mask ||
        !a->acc || !a->aee || !a->percent)
        SNN_FAIL(SNNFLOW_E_ARG, "aee: bad args");
    if (!a->dt_ratio && (!a->dt_gt || !a->dt_input || (a->dt_gt_n != 1 && a->dt_gt_n != a->B) ||
                         (a->dt_input_n != 1 && a->dt_input_n != a->B)))
        SNN_FAIL(SNNFLOW_E_ARG, "aee: dt_ratio, or dt_gt / dt_input of 1 or B entries");
    const hipStream_t s = (hipStream_t)stream;
    const int slices = aee_slices((int64_t)a->H * a->W);
    hipLaunchKernelGGL(k_aee, dim3(a->B * slices), dim3(AEE_NT), 0, s, *a, slices);
    SNN_CHECK_LAUNCH();
    return 0;
}

int snnflow_aee_acc_doubles(int B, int H, int W) {
    return (int)(1 + 3 * (int64_t)B * aee_slices((int64_t)H * W));
}

int snnflow_flow_metrics_rows(int B, int H, int W) {
    return (int)((int64_t)B * (((int64_t)H * W + NT - 1) / NT) * FM_NV);
}

int snnflow_flow_metrics(const snnflow_flow_metrics_args* a, void* stream) {
    if (!a || a->B <= 0 || a->B > NT || a->H <= 0 || a->W <= 0 || !a->flow || !a->gtflow || !a->event_mask ||
        !a->dt_ratio || !a->rows || !a->out)
        SNN_FAIL(SNNFLOW_E_ARG, "flow_metrics: bad args");
    const hipStream_t s = (hipStream_t)stream;
    const int chunks = (int)(((int64_t)a->H * a->W + NT - 1) / NT);
    hipLaunchKernelGGL(k_flow_metrics, dim3(a->B * chunks), dim3(NT), 0, s, *a, chunks);
    hipLaunchKernelGGL(k_flow_metrics_finalize, dim3(1), dim3(NT), 0, s, *a, chunks);
    SNN_CHECK_LAUNCH();
    return 0;
}

}  // extern "C"
