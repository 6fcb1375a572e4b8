// Launch-path microbenchmark for the C5 frame's stage shape: a dependent chain of K small kernels
// (about the size of the area / index / tick launches) on one stream, then one stream sync.
//   eager   : K hipLaunchKernelGGL per iteration
//   replay  : the chain captured once, hipGraphLaunch per iteration (fixed arguments)
//   update  : the chain re-captured every iteration (arguments may change), hipGraphExecUpdate
//             into the instantiated graph, hipGraphLaunch -- what a per-frame capture costs
//   setp    : hipGraphExecKernelNodeSetParams on every node of the instantiated graph, launch
// Prints one JSON line per mode: us per iteration (host wall, sync included).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mb/graph_launch tools/mb/graph_launch.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

__global__ void k_step(float *__restrict__ a, int n, int iters, float s) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = a[i];
    for (int t = 0; t < iters; ++t) v = v * 0.999f + s;
    a[i] = v;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 25;          // kernels per chain
    const int blocks = argc > 2 ? atoi(argv[2]) : 64;     // blocks per kernel
    const int iters = argc > 3 ? atoi(argv[3]) : 200;     // work per thread
    const int reps = argc > 4 ? atoi(argv[4]) : 200;
    const int n = blocks * 256;
    float *a;
    CK(hipMalloc(&a, (size_t)n * sizeof(float)));
    CK(hipMemset(a, 0, (size_t)n * sizeof(float)));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    auto chain = [&](int frame) {
        for (int k = 0; k < K; ++k)
            hipLaunchKernelGGL(k_step, dim3(blocks + (frame & 1)), dim3(256), 0, st, a, n, iters,
                               0.001f * (float)(k + frame));
    };
    auto timed = [&](const char *mode, auto body) {
        for (int r = 0; r < 20; ++r) body(r);
        CK(hipStreamSynchronize(st));
        std::vector<double> t(reps);
        for (int r = 0; r < reps; ++r) {
            const double t0 = now_us();
            body(r);
            CK(hipStreamSynchronize(st));
            t[r] = now_us() - t0;
        }
        std::sort(t.begin(), t.end());
        printf("{\"mode\": \"%s\", \"kernels\": %d, \"blocks\": %d, \"iters\": %d, \"p50_us\": %.1f, "
               "\"p10_us\": %.1f, \"p90_us\": %.1f}\n",
               mode, K, blocks, iters, t[reps / 2], t[reps / 10], t[reps * 9 / 10]);
        fflush(stdout);
    };
    // device time of one chain (events around an eager chain)
    {
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        chain(0);
        CK(hipEventRecord(e0, st));
        chain(0);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"mode\": \"eager_device\", \"kernels\": %d, \"us\": %.1f}\n", K, ms * 1e3);
    }
    timed("eager", [&](int r) { chain(r); });
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
    chain(0);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    timed("replay", [&](int) { CK(hipGraphLaunch(ge, st)); });
    timed("update", [&](int r) {
        hipGraph_t g2;
        CK(hipStreamBeginCapture(st, hipStreamCaptureModeRelaxed));
        chain(r);
        CK(hipStreamEndCapture(st, &g2));
        hipGraphExecUpdateResult res;
        hipGraphNode_t err;
        CK(hipGraphExecUpdate(ge, g2, &err, &res));
        CK(hipGraphLaunch(ge, st));
        CK(hipGraphDestroy(g2));
    });
    {
        size_t nn = 0;
        CK(hipGraphGetNodes(g, nullptr, &nn));
        std::vector<hipGraphNode_t> nodes(nn);
        CK(hipGraphGetNodes(g, nodes.data(), &nn));
        std::vector<hipKernelNodeParams> kp(nn);
        for (size_t i = 0; i < nn; ++i) CK(hipGraphKernelNodeGetParams(nodes[i], &kp[i]));
        std::vector<float> sv(nn);
        timed("setp", [&](int r) {
            for (size_t i = 0; i < nn; ++i) {
                hipKernelNodeParams p = kp[i];
                p.gridDim = dim3(blocks + (r & 1));
                sv[i] = 0.001f * (float)(i + r);
                void *args[4] = {&a, (void *)&n, (void *)&iters, &sv[i]};
                p.kernelParams = args;
                CK(hipGraphExecKernelNodeSetParams(ge, nodes[i], &p));
            }
            CK(hipGraphLaunch(ge, st));
        });
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipStreamDestroy(st));
    CK(hipFree(a));
    return 0;
}
