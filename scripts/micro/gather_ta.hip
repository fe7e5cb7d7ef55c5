// Texture-address cost of wave64 gathers on gfx950: time per wave-instruction of float4 / float2 gathers by access
// pattern and address form (global_load with 64-bit lane addresses vs buffer_load with 32-bit offsets). Every wave
// reads inside one of 8 windows of 256 KiB (2 MiB: L2 resident, like the pair loops' neighbor records).
//   hipcc -O3 --offload-arch=gfx950 -o gather_ta gather_ta.hip && ./gather_ta
#include <cstdio>
#include <cstdint>
#include <vector>

#include <hip/hip_runtime.h>

#define CK(x)                                                                                                         \
    do                                                                                                                \
    {                                                                                                                 \
        hipError_t e = (x);                                                                                           \
        if (e != hipSuccess)                                                                                          \
        {                                                                                                             \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                                           \
            return 1;                                                                                                 \
        }                                                                                                             \
    } while (0)

constexpr int kSteps  = 256;   // gathers per lane
constexpr int kWindow = 16384; // float4 records per wave window (256 KiB)
constexpr int kWindows = 8;    // windows in use: 2 MiB, resident in every XCD's L2

// lane l at step k reads record (l * laneMul + k * stepMul) mod window; laneMul sets the spread within one instruction
template<bool kBuffer, int W>
__global__ __launch_bounds__(256) void gather(const float4* __restrict__ src, float* __restrict__ out, int laneMul,
                                              int stepMul, int64_t nrec)
{
    const int lane  = threadIdx.x & 63;
    const int64_t w = (int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6)) % kWindows;
    const float4* base = src + w * kWindow;
    float acc = 0.f;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, kWindow * 16, 0x00020000);
#pragma unroll 8
    for (int k = 0; k < kSteps; ++k)
    {
        // laneMul < 0: cooperative records of -laneMul float4 chunks (lanes of one record fetch its consecutive
        // chunks), records `stepMul` float4 apart and scattered (hash of lane group and step)
        unsigned r;
        if (laneMul < 0)
        {
            const int C = -laneMul, g = lane / C;
            const unsigned h = (unsigned(g) * 2654435761u) ^ (unsigned(k) * 40503u);
            r = ((h % unsigned(kWindow / stepMul)) * stepMul + unsigned(lane % C)) & (kWindow - 1);
        }
        else r = unsigned(lane * laneMul + k * stepMul) & (kWindow - 1);
        if constexpr (W == 4)
        {
            float4 v;
            if constexpr (kBuffer)
            {
                auto t = __builtin_amdgcn_raw_buffer_load_b128(rs, r * 16, 0, 0);
                v      = *reinterpret_cast<float4*>(&t);
            }
            else v = base[r];
            acc += v.x + v.y + v.z + v.w;
        }
        else
        {
            float2 v;
            if constexpr (kBuffer)
            {
                auto t = __builtin_amdgcn_raw_buffer_load_b64(rs, r * 16, 0, 0);
                v      = *reinterpret_cast<float2*>(&t);
            }
            else v = *reinterpret_cast<const float2*>(base + r);
            acc += v.x + v.y;
        }
    }
    if (acc == 12345.f) out[threadIdx.x] = acc;
}

int main()
{
    const int64_t nrec = int64_t(kWindow) * 4096; // 1 GiB
    float4* src;
    float* out;
    CK(hipMalloc(&src, nrec * 16));
    CK(hipMalloc(&out, 4096));
    CK(hipMemset(src, 0, nrec * 16));
    const int blocks = 256 * 64; // 64 blocks of 4 waves per CU
    struct P
    {
        const char* name;
        int laneMul, stepMul;
    } pats[] = {
        {"coalesced (lane = record)", 1, 64},           // 16 segments / instruction
        {"4 lanes per 64-B segment, 2 records apart", 2, 128}, // 32 segments
        {"1 lane per 64-B segment", 4, 256},           // 64 segments
        {"1 lane per 128-B line", 8, 512},             // 64 lines
        {"scattered (odd stride 37)", 37, 1},          // 64 segments, 1 record step
        {"same record for all lanes", 0, 1},           // 1 segment
        {"coop 64-B records at 64-B stride (16 records)", -4, 4},
        {"coop 64-B records at 128-B stride (16 records)", -4, 8},
        {"coop 128-B records at 128-B stride (8 records)", -8, 8},
        {"coop 32-B records at 32-B stride (32 records)", -2, 2},
        {"coop 80-B records at 80-B stride (12.8 records)", -5, 5},
        {"per-lane 16-B records scattered", -1, 1},
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    printf("| pattern | form | width | ns/launch | cycles per wave-instruction per CU (2.1 GHz) |\n|---|---|---|---|---|\n");
    for (auto& p : pats)
        for (int form = 0; form < 2; ++form)
            for (int wd : {4, 2})
            {
                auto run = [&]()
                {
                    if (form == 0 && wd == 4) gather<false, 4><<<blocks, 256>>>(src, out, p.laneMul, p.stepMul, nrec);
                    if (form == 1 && wd == 4) gather<true, 4><<<blocks, 256>>>(src, out, p.laneMul, p.stepMul, nrec);
                    if (form == 0 && wd == 2) gather<false, 2><<<blocks, 256>>>(src, out, p.laneMul, p.stepMul, nrec);
                    if (form == 1 && wd == 2) gather<true, 2><<<blocks, 256>>>(src, out, p.laneMul, p.stepMul, nrec);
                };
                run();
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(a));
                for (int it = 0; it < 5; ++it)
                    run();
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                const double ns      = ms * 1e6 / 5;
                const double winstr  = double(blocks) * 4 * kSteps / 256.0; // wave-instructions per CU
                printf("| %s | %s | dwordx%d | %.0f | %.1f |\n", p.name, form ? "buffer" : "global", wd, ns,
                       ns * 2.1 / winstr);
            }
    return 0;
}
