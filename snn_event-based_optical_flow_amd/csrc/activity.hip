// Spike-activity log for gfx950: the `log=True` branch of LIFFireNet.forward
// (reference models/model.py:188-205), which reduces every layer's output to
// `l.detach().ne(0).float().mean().item()` -- nine reductions and nine host syncs per
// step in the reference.  Here: one launch over all tensors of the step (blockIdx.y picks
// the tensor), each wave tests 64 x 4 elements per iteration with four wavefront ballots
// whose popcounts are wave-uniform, the block sums its waves in LDS and adds one integer
// per block; the caller reads the counts back once.  Integer counts are exact and
// independent of the order of the additions.
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

constexpr int kWaves = NT / 64;
constexpr int kMaxBlocksPerTensor = 1024;  // 4 per CU: one streaming round per tensor

struct CountArgs {
    const float* ptr[SNNFLOW_MAX_COUNT_TENSORS];
    int64_t size[SNNFLOW_MAX_COUNT_TENSORS];
    unsigned long long* counts;
};

// Number of lanes of this wave whose predicate holds (wave-uniform result).
__device__ inline unsigned wave_count(bool p) { return (unsigned)__popcll(__ballot(p)); }

__global__ __launch_bounds__(NT) void k_count_nonzero(CountArgs a) {
    const int i = blockIdx.y;
    const float* __restrict__ p = a.ptr[i];
    const int64_t n = a.size[i];
    const int64_t stride = (int64_t)gridDim.x * NT;
    unsigned long long c = 0;  // wave-uniform
    if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
        const int64_t n4 = n >> 2;
        const float4* __restrict__ p4 = reinterpret_cast<const float4*>(p);
        for (int64_t base = (int64_t)blockIdx.x * NT; base < n4; base += stride) {
            const int64_t j = base + threadIdx.x;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (j < n4) v = p4[j];
            c += wave_count(v.x != 0.f) + wave_count(v.y != 0.f) + wave_count(v.z != 0.f) +
                 wave_count(v.w != 0.f);
        }
        // ragged tail (< 4 elements) by block 0's first wave
        if (blockIdx.x == 0 && threadIdx.x < 64) {
            const int64_t j = (n4 << 2) + threadIdx.x;
            c += wave_count(j < n && p[j] != 0.f);
        }
    } else {
        for (int64_t base = (int64_t)blockIdx.x * NT; base < n; base += stride) {
            const int64_t j = base + threadIdx.x;
            c += wave_count(j < n && p[j] != 0.f);
        }
    }
    __shared__ unsigned long long part[kWaves];
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) part[wave] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) t += part[w];
        if (t) atomicAdd(a.counts + i, t);
    }
}

}  // namespace

extern "C" int snnflow_count_nonzero(const float* const* ptrs, const int64_t* sizes, int n, uint64_t* counts,
                                     void* stream) {
    if (!ptrs || !sizes || !counts || n <= 0 || n > SNNFLOW_MAX_COUNT_TENSORS)
        SNN_FAIL(SNNFLOW_E_ARG, "count_nonzero: bad args");
    CountArgs a = {};
    int64_t most = 0;
    for (int i = 0; i < n; ++i) {
        if (sizes[i] < 0 || (sizes[i] > 0 && !ptrs[i])) SNN_FAIL(SNNFLOW_E_ARG, "count_nonzero: bad tensor");
        a.ptr[i] = ptrs[i];
        a.size[i] = sizes[i];
        const int64_t v = (sizes[i] + 3) / 4;
        if (v > most) most = v;
    }
    a.counts = reinterpret_cast<unsigned long long*>(counts);
    const hipStream_t s = (hipStream_t)stream;
    hipError_t e = hipMemsetAsync(counts, 0, sizeof(uint64_t) * (size_t)n, s);
    if (e != hipSuccess) return snnflow_set_error((int)e, hipGetErrorString(e));
    int64_t gx = (most + NT - 1) / NT;
    if (gx < 1) gx = 1;
    if (gx > kMaxBlocksPerTensor) gx = kMaxBlocksPerTensor;
    hipLaunchKernelGGL(k_count_nonzero, dim3((unsigned)gx, (unsigned)n), dim3(NT), 0, s, a);
    SNN_CHECK_LAUNCH();
    return 0;
}
