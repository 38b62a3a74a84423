// Probe (not product code): an explicit HIP graph of a wavefront of kernel nodes with the LIFFireNet
// dependency shape ((k-1, t), (k, t-1), (k+1, t-1)); instantiate + launch + check the order; then
// whether launching that graph while a stream captures (as a torch graph capture would) is accepted.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_task(int* order, int* clock_, int id, int spin) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const long long t0 = clock64();
        while (clock64() - t0 < spin) {}
        order[id] = atomicAdd(clock_, 1);
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int build(hipGraph_t* g, int* order, int* clk, int K, int T, int spin) {
    CK(hipGraphCreate(g, 0));
    std::vector<hipGraphNode_t> node(K * T);
    std::vector<int> ids(K * T);
    for (int d = 0; d < K + 2 * (T - 1); ++d)
        for (int k = 0; k < K; ++k) {
            if ((d - k) % 2 || (d - k) < 0 || (d - k) / 2 >= T) continue;
            const int t = (d - k) / 2, id = t * K + k;
            ids[id] = id;
            std::vector<hipGraphNode_t> deps;
            if (k > 0) deps.push_back(node[t * K + k - 1]);
            if (t > 0) deps.push_back(node[(t - 1) * K + k]);
            if (t > 0 && k + 1 < K) deps.push_back(node[(t - 1) * K + k + 1]);
            void* args[] = {&order, &clk, &ids[id], &spin};
            hipKernelNodeParams p = {};
            p.func = (void*)k_task;
            p.gridDim = dim3(64);
            p.blockDim = dim3(64);
            p.kernelParams = args;
            CK(hipGraphAddKernelNode(&node[id], *g, deps.data(), deps.size(), &p));
        }
    return 0;
}

int main() {
    const int K = 8, T = 6;
    int *order, *clk;
    CK(hipMalloc(&order, K * T * sizeof(int)));
    CK(hipMalloc(&clk, sizeof(int)));
    CK(hipMemset(clk, 0, sizeof(int)));
    hipGraph_t g;
    if (build(&g, order, clk, K, T, 20000)) return 1;
    hipGraphExec_t ge;
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    std::vector<int> h(K * T);
    CK(hipMemcpy(h.data(), order, K * T * sizeof(int), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int t = 0; t < T; ++t)
        for (int k = 0; k < K; ++k) {
            const int o = h[t * K + k];
            if (k > 0 && h[t * K + k - 1] > o) ++bad;
            if (t > 0 && h[(t - 1) * K + k] > o) ++bad;
            if (t > 0 && k + 1 < K && h[(t - 1) * K + k + 1] > o) ++bad;
        }
    printf("explicit graph: %d nodes, dependency violations %d\n", K * T, bad);
    // concurrency: a 2-node graph of independent long tasks vs one task
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a, s));
        CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("wavefront graph replay %.3f ms (%d levels x spin; serial would be %d x spin)\n", ms, K + 2 * (T - 1), K * T);
    }
    // serial baseline: the same 48 tasks back to back on one stream
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(a, s));
        for (int i = 0; i < K * T; ++i) hipLaunchKernelGGL(k_task, dim3(64), dim3(64), 0, s, order, clk, i, 20000);
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("serial stream %.3f ms\n", ms);
    }
    // the wavefront by stream capture: 4 side streams forked from the origin, tasks on stream
    // (k / 2) % 4, cross-stream dependencies through events (the pattern of the torch probe that crashed)
    {
        hipStream_t o, ss[4];
        CK(hipStreamCreate(&o));
        for (int i = 0; i < 4; ++i) CK(hipStreamCreate(&ss[i]));
        std::vector<hipEvent_t> ev(K * T);
        for (auto& x : ev) CK(hipEventCreateWithFlags(&x, hipEventDisableTiming));
        hipEvent_t fork, join[4];
        CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
        for (int i = 0; i < 4; ++i) CK(hipEventCreateWithFlags(&join[i], hipEventDisableTiming));
        CK(hipStreamBeginCapture(o, hipStreamCaptureModeGlobal));
        CK(hipEventRecord(fork, o));
        for (int i = 0; i < 4; ++i) CK(hipStreamWaitEvent(ss[i], fork, 0));
        for (int d = 0; d < K + 2 * (T - 1); ++d)
            for (int k = 0; k < K; ++k) {
                if ((d - k) % 2 || (d - k) < 0 || (d - k) / 2 >= T) continue;
                const int t = (d - k) / 2, id = t * K + k;
                hipStream_t st = ss[(k / 2) % 4];
                int dd[3][2] = {{k - 1, t}, {k, t - 1}, {k + 1, t - 1}};
                for (auto& q : dd) {
                    if (q[0] < 0 || q[0] >= K || q[1] < 0) continue;
                    if (ss[(q[0] / 2) % 4] != st) CK(hipStreamWaitEvent(st, ev[q[1] * K + q[0]], 0));
                }
                hipLaunchKernelGGL(k_task, dim3(64), dim3(64), 0, st, order, clk, id, 20000);
                CK(hipEventRecord(ev[id], st));
            }
        for (int i = 0; i < 4; ++i) {
            CK(hipEventRecord(join[i], ss[i]));
            CK(hipStreamWaitEvent(o, join[i], 0));
        }
        hipGraph_t cg = nullptr;
        hipError_t e2 = hipStreamEndCapture(o, &cg);
        printf("multi-stream capture end -> %s\n", hipGetErrorString(e2));
        if (e2 == hipSuccess) {
            hipGraphExec_t cge;
            e2 = hipGraphInstantiate(&cge, cg, nullptr, nullptr, 0);
            printf("multi-stream instantiate -> %s\n", hipGetErrorString(e2));
            if (e2 == hipSuccess) {
                for (int rep = 0; rep < 2; ++rep) {
                    CK(hipEventRecord(a, s));
                    CK(hipGraphLaunch(cge, s));
                    CK(hipEventRecord(b, s));
                    CK(hipEventSynchronize(b));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, a, b));
                    printf("multi-stream captured graph %.3f ms\n", ms);
                }
            }
        }
    }
    // the graph launched while another stream captures (a child graph in the captured graph?)
    hipStream_t c;
    CK(hipStreamCreate(&c));
    CK(hipStreamBeginCapture(c, hipStreamCaptureModeGlobal));
    hipError_t e = hipGraphLaunch(ge, c);
    printf("hipGraphLaunch during capture -> %s\n", hipGetErrorString(e));
    hipGraph_t outer = nullptr;
    e = hipStreamEndCapture(c, &outer);
    printf("end capture -> %s\n", hipGetErrorString(e));
    if (e == hipSuccess && outer) {
        size_t n = 0;
        hipGraphGetNodes(outer, nullptr, &n);
        printf("captured graph nodes: %zu\n", n);
        hipGraphExec_t oe;
        e = hipGraphInstantiate(&oe, outer, nullptr, nullptr, 0);
        printf("instantiate -> %s\n", hipGetErrorString(e));
        if (e == hipSuccess) {
            e = hipGraphLaunch(oe, s);
            printf("launch outer -> %s\n", hipGetErrorString(e));
            CK(hipStreamSynchronize(s));
        }
    }
    // alternative: add the wavefront graph as a child node of a graph we build ourselves
    hipGraph_t par;
    CK(hipGraphCreate(&par, 0));
    hipGraphNode_t ch;
    e = hipGraphAddChildGraphNode(&ch, par, nullptr, 0, g);
    printf("child graph node -> %s\n", hipGetErrorString(e));
    printf("done\n");
    return 0;
}
