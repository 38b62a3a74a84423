// Workgroup dispatch probe: how fast does the chip fill with resident blocks, and what does a launch of
// N blocks of T threads cost when every block just waits ~W us?  Each block's wave 0 stamps its start
// and end (s_memrealtime, 100 MHz) into a per-block array; the host prints the launch time (hipEvent),
// the spread of block starts and the residency timeline.  Timing only; every block writes its own slot.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

__global__ void k_wait(unsigned long long* stamps, int wait_ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long t = t0;
    while (t - t0 < (unsigned long long)wait_ticks) {  // bounded: wait_ticks of the 100 MHz clock
        __builtin_amdgcn_s_sleep(2);
        t = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = t0;
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

int main(int argc, char** argv) {
    const int wait_us = argc > 1 ? atoi(argv[1]) : 10;
    const int cfgs[][2] = {{256, 512}, {768, 512}, {1024, 512}, {1536, 512}, {2048, 512}, {3072, 256},
                           {1536, 1024}, {6144, 128}, {4096, 256}};
    unsigned long long* d;
    hipMalloc(&d, 2 * 8192 * sizeof(unsigned long long));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (auto& c : cfgs) {
        const int nb = c[0], nt = c[1];
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0, 0);
            hipLaunchKernelGGL(k_wait, dim3(nb), dim3(nt), 0, 0, d, wait_us * 100);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
        }
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        std::vector<unsigned long long> h(2 * nb);
        hipMemcpy(h.data(), d, 2 * nb * sizeof(unsigned long long), hipMemcpyDeviceToHost);
        unsigned long long s0 = ~0ull, s1 = 0, en = 0;
        std::vector<double> starts(nb);
        for (int b = 0; b < nb; ++b) {
            s0 = std::min(s0, h[2 * b]);
            s1 = std::max(s1, h[2 * b]);
            en = std::max(en, h[2 * b + 1]);
        }
        for (int b = 0; b < nb; ++b) starts[b] = (h[2 * b] - s0) * 0.01;
        std::sort(starts.begin(), starts.end());
        auto pct = [&](double q) { return starts[std::min(nb - 1, (int)(q * nb))]; };
        printf("blocks %5d x %4d threads (%6d waves): launch %7.2f us, block starts p10/50/90/100 %6.2f %6.2f %6.2f %6.2f us, span %7.2f us\n",
               nb, nt, nb * nt / 64, ms * 1000.0, pct(0.1), pct(0.5), pct(0.9), (s1 - s0) * 0.01, (en - s0) * 0.01);
    }
    hipFree(d);
    return 0;
}
