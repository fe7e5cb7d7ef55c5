// Micro-benchmark: the sample sort of a nearly sorted key array (Evrard -n 100 size) launched kernel by kernel vs
// replayed as one captured hipGraph. Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../sphexa_amd/csrc/include
//   -I../../sphexa_amd/csrc/hip sort_graph.hip ../../sphexa_amd/csrc/hip/sample_sort.hip -o sort_graph
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "hip_api.h"

#define CK(x)                                                                                                          \
    do                                                                                                                 \
    {                                                                                                                  \
        hipError_t e_ = (x);                                                                                           \
        if (e_ != hipSuccess)                                                                                          \
        {                                                                                                              \
            std::printf("%s failed: %s\n", #x, hipGetErrorString(e_));                                                 \
            std::exit(1);                                                                                              \
        }                                                                                                              \
    } while (0)

int main(int argc, char** argv)
{
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : 463277;
    const int reps  = 200;
    std::mt19937_64 rng(1);
    std::vector<uint64_t> k(n);
    for (int64_t i = 0; i < n; ++i)
        k[i] = uint64_t(i) << 20 | (rng() & 0xFFFFF);
    for (int64_t i = 0; i + 8 < n; i += 97)
        std::swap(k[i], k[i + 7]);
    uint64_t *dIn, *dOut;
    uint32_t* dV;
    void* tmp;
    const size_t tb = sphx::hip::sampleSortTempBytes(n);
    CK(hipMalloc(&dIn, n * 8));
    CK(hipMalloc(&dOut, n * 8));
    CK(hipMalloc(&dV, n * 4));
    CK(hipMalloc(&tmp, tb));
    CK(hipMemcpy(dIn, k.data(), n * 8, hipMemcpyHostToDevice));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 10; ++w)
        sphx::hip::sampleSortPairs(n, dIn, nullptr, dOut, dV, tmp, tb, s);
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r)
        sphx::hip::sampleSortPairs(n, dIn, nullptr, dOut, dV, tmp, tb, s);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float msDirect;
    CK(hipEventElapsedTime(&msDirect, a, b));

    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    sphx::hip::sampleSortPairs(n, dIn, nullptr, dOut, dV, tmp, tb, s);
    CK(hipStreamEndCapture(s, &g));
    size_t nodes = 0;
    CK(hipGraphGetNodes(g, nullptr, &nodes));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int w = 0; w < 10; ++w)
        CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < reps; ++r)
        CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float msGraph;
    CK(hipEventElapsedTime(&msGraph, a, b));
    std::vector<uint64_t> o(n);
    CK(hipMemcpy(o.data(), dOut, n * 8, hipMemcpyDeviceToHost));
    std::sort(k.begin(), k.end());
    const bool ok = o == k;
    std::printf("n %lld: direct %.1f us/sort, graph %.1f us/sort (%zu nodes), sorted %s\n", (long long)n,
                1000.0 * msDirect / reps, 1000.0 * msGraph / reps, nodes, ok ? "ok" : "WRONG");
    return ok ? 0 : 1;
}
