// VALU issue rate of gfx950 per SIMD: how many wave64 VALU instructions a SIMD retires per cycle for independent
// v_fma_f32 / v_pk_fma_f32 / v_exp_f32 streams at 1..8 waves per SIMD. Decides whether a pair loop whose counters
// show ~4 cycles per VALU instruction per SIMD is at the VALU limit (design data of the round-6 pair loops).
//   hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 -o valu_rate valu_rate.hip && ./valu_rate
#include <cstdio>
#include <cstdint>

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

typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int kIters = 4096;

// kind 0: 8 independent v_fma_f32 chains; 1: 8 independent v_pk_fma_f32 chains; 2: 4 fma + 4 v_exp_f32;
// 3: 8 independent v_add_u32 chains; 4: 8 v_and_b32/v_lshl_or chains (bit ops); 5: v_cndmask_b32 chains
template<int kind>
__global__ __launch_bounds__(64) void valuKernel(float* out, float s, long long* clk)
{
    float a[8];
    f2 p[8];
    unsigned ia[8];
    for (int k = 0; k < 8; ++k)
    {
        a[k] = float(threadIdx.x + k);
        p[k] = f2{a[k], a[k] + 1.f};
        ia[k] = threadIdx.x * 7u + k;
    }
    const f2 s2 = f2{s, s};
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; ++it)
    {
#pragma unroll
        for (int k = 0; k < 8; ++k)
        {
            if constexpr (kind == 0) a[k] = __builtin_fmaf(a[k], s, 0.5f);
            else if constexpr (kind == 1) p[k] = __builtin_elementwise_fma(p[k], s2, f2{0.5f, 0.25f});
            else if constexpr (kind == 2)
            {
                if (k & 1) a[k] = __builtin_amdgcn_exp2f(a[k]);
                else a[k] = __builtin_fmaf(a[k], s, 0.5f);
            }
            else if constexpr (kind == 3)
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(ia[k]) : "v"(ia[(k + 1) & 7]));
            else if constexpr (kind == 4)
                asm volatile("v_lshl_or_b32 %0, %0, 1, %1" : "+v"(ia[k]) : "v"(ia[(k + 3) & 7]));
            else
                asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(ia[k]) : "v"(ia[(k + 5) & 7]));
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    float r = 0.f;
    for (int k = 0; k < 8; ++k)
        r += a[k] + p[k].x + p[k].y + float(ia[k]);
    out[blockIdx.x * 64 + threadIdx.x] = r;
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template<int kind>
int run(const char* name, float* out, long long* clk, long long* hclk)
{
    // waves per SIMD: 256 CUs x 4 SIMDs x w waves (one-wave blocks; the dispatcher spreads them)
    for (int w : {1, 2, 4, 8})
    {
        const int blocks = 256 * 4 * w;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        valuKernel<kind><<<blocks, 64>>>(out, 0.999f, clk);
        CK(hipEventRecord(e0));
        valuKernel<kind><<<blocks, 64>>>(out, 0.999f, clk);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipMemcpy(hclk, clk, sizeof(long long) * blocks, hipMemcpyDeviceToHost));
        double avg = 0;
        for (int b = 0; b < blocks; ++b)
            avg += double(hclk[b]);
        avg /= blocks;
        const double instr = double(kIters) * 8; // VALU instructions of the timed loop per wave
        // per SIMD: w waves x instr in (cycles of one wave's loop) -> instructions per cycle per SIMD
        printf("%-10s waves/SIMD %d: %.3f ms, %.0f cycles per wave loop, %.2f cycles per instr per wave, "
               "SIMD issue %.3f instr/cycle\n",
               name, w, ms, avg, avg / instr, w * instr / avg);
    }
    return 0;
}

int main()
{
    float* out;
    long long *clk, *hclk;
    CK(hipMalloc(&out, sizeof(float) * 256 * 4 * 8 * 64));
    CK(hipMalloc(&clk, sizeof(long long) * 256 * 4 * 8));
    hclk = new long long[256 * 4 * 8];
    if (run<0>("v_fma_f32", out, clk, hclk)) return 1;
    if (run<1>("v_pk_fma", out, clk, hclk)) return 1;
    if (run<2>("fma+exp", out, clk, hclk)) return 1;
    if (run<3>("v_add_u32", out, clk, hclk)) return 1;
    if (run<4>("v_lshl_or", out, clk, hclk)) return 1;
    if (run<5>("v_cndmask", out, clk, hclk)) return 1;
    return 0;
}
