// Issue cost of single VALU instructions on gfx950 at full occupancy (8 waves per SIMD, 8 independent chains per
// wave): the time of N instructions relative to the same number of v_fma_f32 (4 cycles per wave64 instruction).
// Design data of the round-6 pair loops: which operations (address arithmetic, moves, conversions, packed fp32,
// transcendentals) cost a full VALU slot.
//   hipcc -O3 -fno-slp-vectorize --offload-arch=gfx950 -o valu_cost valu_cost.hip && ./valu_cost
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

constexpr int kIters = 2048;

// one instruction per chain and step: v = op(v, w); 8 chains. OP is the asm text with %0 (in/out) and %1 (other)
#define DEF_K(NAME, OP, C1, C2)                                                                                       \
    __global__ __launch_bounds__(64) void NAME(unsigned* out)                                                         \
    {                                                                                                                 \
        C1 a[8];                                                                                                      \
        C2 b[8];                                                                                                      \
        for (int k = 0; k < 8; ++k)                                                                                   \
        {                                                                                                             \
            a[k] = C1(threadIdx.x + k + 1);                                                                           \
            b[k] = C2(threadIdx.x * 3 + k + 1);                                                                       \
        }                                                                                                             \
        for (int it = 0; it < kIters; ++it)                                                                           \
        {                                                                                                             \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) asm volatile(OP : "+v"(a[k]) : "v"(b[k]));                \
        }                                                                                                             \
        unsigned r = 0;                                                                                               \
        for (int k = 0; k < 8; ++k)                                                                                   \
        {                                                                                                             \
            unsigned u;                                                                                               \
            __builtin_memcpy(&u, &a[k], 4);                                                                           \
            r += u;                                                                                                   \
        }                                                                                                             \
        out[blockIdx.x * 64 + threadIdx.x] = r;                                                                       \
    }

typedef float f2 __attribute__((ext_vector_type(2)));

// as DEF_K with an SGPR operand %1 (a kernel argument)
#define DEF_S(NAME, OP)                                                                                               \
    __global__ __launch_bounds__(64) void NAME(unsigned* out, float sv)                                               \
    {                                                                                                                 \
        float a[8];                                                                                                   \
        for (int k = 0; k < 8; ++k)                                                                                   \
            a[k] = float(threadIdx.x + k + 1);                                                                        \
        for (int it = 0; it < kIters; ++it)                                                                           \
        {                                                                                                             \
            _Pragma("unroll") for (int k = 0; k < 8; ++k) asm volatile(OP : "+v"(a[k]) : "s"(sv));                   \
        }                                                                                                             \
        float r = 0;                                                                                                  \
        for (int k = 0; k < 8; ++k)                                                                                   \
            r += a[k];                                                                                                \
        out[blockIdx.x * 64 + threadIdx.x] = unsigned(r);                                                             \
    }

DEF_K(kFma, "v_fma_f32 %0, %0, %1, 1.0", float, float)
DEF_K(kMul, "v_mul_f32 %0, %0, %1", float, float)
DEF_K(kAddU, "v_add_u32 %0, %0, %1", unsigned, unsigned)
DEF_K(kSubU, "v_sub_u32 %0, %0, %1", unsigned, unsigned)
DEF_K(kMov, "v_mov_b32 %0, %1", unsigned, unsigned)
DEF_K(kAnd, "v_and_b32 %0, %0, %1", unsigned, unsigned)
DEF_K(kLsh, "v_lshlrev_b32 %0, 1, %0", unsigned, unsigned)
DEF_K(kBfe, "v_bfe_u32 %0, %0, 3, 6", unsigned, unsigned)
DEF_K(kCvt, "v_cvt_f32_i32 %0, %1", float, unsigned)
DEF_K(kRcp, "v_rcp_f32 %0, %0", float, float)
DEF_K(kSqrt, "v_sqrt_f32 %0, %0", float, float)
DEF_K(kSin, "v_sin_f32 %0, %0", float, float)
DEF_K(kRsq, "v_rsq_f32 %0, %0", float, float)
DEF_K(kCmpCnd, "v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc", float, float)
DEF_K(kPkMul, "v_pk_mul_f32 %0, %0, %1", f2, f2)
DEF_K(kPkFma, "v_pk_fma_f32 %0, %0, %1, %1", f2, f2)
DEF_K(kLshAdd64, "v_lshl_add_u64 %0, %0, 2, %1", uint64_t, uint64_t)
DEF_K(kMax, "v_max_f32 %0, %0, %1", float, float)
DEF_K(kAddF, "v_add_f32 %0, %0, %1", float, float)
DEF_K(kSubF, "v_sub_f32 %0, %0, %1", float, float)
DEF_K(kFmac, "v_fmac_f32 %0, %0, %1", float, float)
DEF_K(kOr, "v_or_b32 %0, %0, %1", unsigned, unsigned)
DEF_K(kLshV, "v_lshlrev_b32 %0, %1, %0", unsigned, unsigned)
DEF_K(kLshlOr, "v_lshl_or_b32 %0, %0, 1, %1", unsigned, unsigned)
DEF_K(kMin, "v_min_f32 %0, %0, %1", float, float)
DEF_K(kCvtU, "v_cvt_f32_u32 %0, %1", float, unsigned)
DEF_K(kExp, "v_exp_f32 %0, %0", float, float)
DEF_K(kCmpOnly, "v_cmp_gt_f32 vcc, %0, %1", float, float)
DEF_K(kMad24, "v_mad_u32_u24 %0, %0, %1, 3", unsigned, unsigned)
DEF_K(kMulLit, "v_mul_f32 %0, 0x3f9df3b6, %0", float, float)
DEF_K(kMulInl, "v_mul_f32 %0, 2.0, %0", float, float)
DEF_K(kCnd, "v_cndmask_b32 %0, %0, %1, s[0:1]", float, float)
DEF_S(kFmaS, "v_fma_f32 %0, %0, %1, 1.0")
DEF_S(kMulS, "v_mul_f32 %0, %1, %0")
DEF_S(kAddS, "v_add_f32 %0, %1, %0")

template<class K, class... A>
int run(const char* name, K kern, unsigned* out, float& fmaMs, int instrPer, A... args)
{
    const int blocks = 256 * 4 * 8;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    kern<<<blocks, 64>>>(out, args...);
    CK(hipEventRecord(e0));
    for (int r = 0; r < 4; ++r)
        kern<<<blocks, 64>>>(out, args...);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 4;
    if (fmaMs == 0.f) fmaMs = ms;
    // cycles per instruction per SIMD, relative to v_fma_f32 = 4
    printf("%-22s %.3f ms  %.2f cycles per instruction (fma = 4)\n", name, ms, 4.0 * ms / fmaMs / instrPer);
    return 0;
}

int main()
{
    unsigned* out;
    CK(hipMalloc(&out, sizeof(unsigned) * 256 * 4 * 8 * 64));
    float f = 0.f;
    run("v_fma_f32", kFma, out, f, 1);
    run("v_mul_f32", kMul, out, f, 1);
    run("v_max_f32", kMax, out, f, 1);
    run("v_add_u32", kAddU, out, f, 1);
    run("v_sub_u32", kSubU, out, f, 1);
    run("v_mov_b32", kMov, out, f, 1);
    run("v_and_b32", kAnd, out, f, 1);
    run("v_lshlrev_b32", kLsh, out, f, 1);
    run("v_bfe_u32", kBfe, out, f, 1);
    run("v_cvt_f32_i32", kCvt, out, f, 1);
    run("v_rcp_f32", kRcp, out, f, 1);
    run("v_sqrt_f32", kSqrt, out, f, 1);
    run("v_sin_f32", kSin, out, f, 1);
    run("v_rsq_f32", kRsq, out, f, 1);
    run("v_cmp+v_cndmask (per pair)", kCmpCnd, out, f, 1);
    run("v_pk_mul_f32", kPkMul, out, f, 1);
    run("v_pk_fma_f32", kPkFma, out, f, 1);
    run("v_lshl_add_u64", kLshAdd64, out, f, 1);
    run("v_add_f32", kAddF, out, f, 1);
    run("v_sub_f32", kSubF, out, f, 1);
    run("v_fmac_f32", kFmac, out, f, 1);
    run("v_or_b32", kOr, out, f, 1);
    run("v_lshlrev_b32 (vgpr)", kLshV, out, f, 1);
    run("v_lshl_or_b32", kLshlOr, out, f, 1);
    run("v_min_f32", kMin, out, f, 1);
    run("v_cvt_f32_u32", kCvtU, out, f, 1);
    run("v_exp_f32", kExp, out, f, 1);
    run("v_cmp_gt_f32 (vcc)", kCmpOnly, out, f, 1);
    run("v_mad_u32_u24", kMad24, out, f, 1);
    run("v_mul_f32 literal", kMulLit, out, f, 1);
    run("v_mul_f32 inline 2.0", kMulInl, out, f, 1);
    run("v_cndmask_b32 s[0:1]", kCnd, out, f, 1);
    run("v_fma_f32 sgpr", kFmaS, out, f, 1, 0.999f);
    run("v_mul_f32 sgpr", kMulS, out, f, 1, 0.999f);
    run("v_add_f32 sgpr", kAddS, out, f, 1, 0.5f);
    return 0;
}
