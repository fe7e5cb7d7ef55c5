/*! SPH math shared by the OpenMP reference path and the gfx950 kernels.
 *
 * Behavioural parity with the reference (cited per function):
 *   sph/include/sph/kernels.hpp            updateH, tsKCourant, artificial_viscosity, symv
 *   sph/include/sph/table_lookup.hpp       linear-interpolated kernel table over [0,2], 20000 points
 *   sph/include/sph/eos.hpp                ideal gas cv / EOS
 *   sph/include/sph/hydro_ve/(xmass|ve_def_gradh|iad|divv_curlv|av_switches|momentum_energy)_kern.hpp  VE j-loops
 *   sph/include/sph/hydro_std/(iad|momentum_energy)_kern.hpp                                          STD j-loops
 *   sph/include/sph/positions.hpp          Press position update, AB2 energy update
 *
 * Data access is decoupled from the math: every j-loop reads source particles through a *loader* returning a
 * small record (SrcPos, SrcIad, ...). The OpenMP path assembles records from the SoA fields; the gfx950 path reads
 * 16-byte aligned array-of-records buffers packed once per loop, so one neighbor costs 2-8 dwordx4 loads from one
 * or two cache lines instead of up to 21 scattered 4-byte gathers. Fields that the reference derives per pair
 * (xm/kx, kx*m/xm) are packed already derived — bit-identical because the same fp32 operations are applied.
 * The neighbor list accessor is (nbr, stride): neighbor k is nbr[k*stride] with stride 1 on the CPU; on the GPU
 * nbr is the lane's PackedLane (16-bit delta-coded lists in per-group rows, packed_list.hpp).
 */
#pragma once

#include <cmath>
#include <cstddef>
#include <cstdint>

#include "annotation.hpp"
#include "box.hpp"
#include "packed_list.hpp"

namespace sphx
{

#ifndef SPHX_HYDRO_TYPE
#define SPHX_HYDRO_TYPE float
#endif
// hydro precision (reference sph/types.hpp:39-46). Production builds use float; the golden-value module
// (csrc/golden, tests/test_golden.py) instantiates the same j-loops with double, as the reference's sph/test does.
using HT = SPHX_HYDRO_TYPE;
constexpr bool kHydroF32 = sizeof(HT) == 4;
using CT = double;  // coordinate precision

constexpr int kTableSize = 20000;

struct SphConsts
{
    double K;           // kernel normalization
    double Kcour;
    double Krho;
    double gamma;
    double muiConst;
    float alphamin;
    float alphamax;
    float decayConstant;
    float Atmin;
    float Atmax;
    float ramp;
    unsigned ng0;
    unsigned ngmax;
    float sincIndex;  // exponent n of the sinc^n kernel
    int kernelChoice; // 0: sinc^n, 1: 0.9 sinc^4 + 0.1 sinc^9
    int fixedPoint;   // GPU pair loops may read fixed-point (QFrame) records: nonzero when the coordinate quantum
                      // is <= 2^-22 of the smallest h; bits 1.. hold the frame shifts (qframeOf, ops/hydro.py:
                      // fixed_point_code), else fp64-coordinate records
};

//! @brief linear interpolation in a table sampled on [0, 2]
template<class T>
SPHX_HD T tableLookup(const T* table, T v)
{
    constexpr int nInt = kTableSize - 1;
    constexpr T dx     = T(2.0) / nInt;
    constexpr T invDx  = T(1) / dx;
    int idx            = int(v * invDx);
#ifndef SPHX_SELECT_TABLE
    // a (wave-uniformly) skipped branch is cheaper than always loading + selecting (measured, profiles/)
    if (idx >= nInt) return T(0);
    T d = (table[idx + 1] - table[idx]) * invDx;
    return table[idx] + d * (v - T(idx) * dx);
#else
    bool inside = idx < nInt;
    idx         = inside ? idx : nInt - 1;
    T t0 = table[idx], t1 = table[idx + 1];
    T r  = t0 + (t1 - t0) * invDx * (v - T(idx) * dx);
    return inside ? r : T(0);
#endif
}

/*! @brief SPH kernel W(v) and dW/dv on [0, 2) (reference sph_kernel_tables.hpp: sinc^n of (pi/2) v, or the
 *         0.9 sinc^4 + 0.1 sinc^9 mix, tabulated at 20000 points and interpolated by lt::lookup).
 *
 * The OpenMP path interpolates the same 20000-point tables as the reference. On the GPU the tables (80 kB each)
 * do not fit the 32 kB vector L1, so every lookup pair became an L2 round trip inside the pair loop; there the
 * kernel is evaluated analytically from one sin/cos pair instead (the table's interpolation error, ~1e-8
 * relative, is below fp32 rounding). Build with -DSPHX_TABLE_KERNEL to use the tables on the GPU as well.
 */
template<int kN = 0>
struct KernelFnT
{
    const HT* wh;
    const HT* whd;
    HT n;
    int choice;
    // kN = 6: the default kernel (choice 0, sinc^6) fixed at compile time, so the pair loops carry no per-neighbor
    // scalar branches on choice and n (KernelFnSinc6, selected per launch by withKernelFn); kN = 0: runtime n, choice

#if defined(__HIP_DEVICE_COMPILE__) && !defined(SPHX_TABLE_KERNEL)
    //! s^k for a compile-time k as powN forms it (the same products; inlined, the surrounding FMA contraction may differ)
    template<int k>
    SPHX_HD static HT powC(HT s)
    {
        static_assert(k == 5 || k == 6, "the sinc^6 kernel and its derivative");
        if constexpr (k == 6)
        {
            HT s3 = s * s * s;
            return s3 * s3;
        }
        else
        {
            HT p = s * s;
            p *= p;
            return s * p;
        }
    }
    SPHX_HD bool generic() const { return kN == 0 && choice != 0; }
    SPHX_HD HT nVal() const { return kN ? HT(kN) : n; }
    //! sinc(x) and d sinc/dv for x = (pi/2) v
    SPHX_HD void sinc(HT v, HT& s, HT& ds) const
    {
        constexpr HT halfPi = HT(1.5707963267948966);
        HT x  = halfPi * v;
        HT sn = __sinf(x), cs = __cosf(x);
        HT ix = rcpF(x);
        s     = v > HT(0) ? sn * ix : HT(1);
        ds    = v > HT(0) ? halfPi * (cs - s) * ix : HT(0);
    }
    //! s^n: integer exponents up to 15 (the kernel's n = 6 and the derivative's n - 1 = 5) by multiplication (n is
    //! uniform: scalar branches), others through exp2/log2 (two quarter-rate transcendentals and range handling)
    SPHX_HD static HT powN(HT s, HT n)
    {
        if (n == HT(6))
        {
            HT s3 = s * s * s;
            return s3 * s3;
        }
#ifndef SPHX_POW_EXP2 // (A/B variant: every exponent but 6 through exp2/log2)
        const int k = int(n);
        if (HT(k) == n && k >= 1 && k <= 15)
        {
            HT r = (k & 1) ? s : HT(1);
            HT p = s * s;
            if (k & 2) r *= p;
            p *= p;
            if (k & 4) r *= p;
            p *= p;
            if (k & 8) r *= p;
            return r;
        }
#endif
        return s > HT(0) ? exp2(n * log2(s)) : HT(0);
    }
    SPHX_HD HT w(HT v) const
    {
        if (v >= HT(2)) return HT(0);
        HT s, ds;
        sinc(v, s, ds);
        if (choice == 0) return powN(s, n);
        HT s2 = s * s, s4 = s2 * s2;
        return HT(0.9) * s4 + HT(0.1) * s4 * s4 * s;
    }
    SPHX_HD HT dw(HT v) const
    {
        if (v >= HT(2)) return HT(0);
        HT s, ds;
        sinc(v, s, ds);
        if (choice == 0) return n * powN(s, n - HT(1)) * ds;
        HT s2 = s * s, s3 = s2 * s, s8 = (s2 * s2) * (s2 * s2);
        return (HT(0.9) * HT(4) * s3 + HT(0.1) * HT(9) * s8) * ds;
    }
    /* Quarter-argument forms of the pair loops: u = v / 4, so the hardware sine (v_sin_f32 takes revolutions,
     * sin(2 pi u) = sin(pi v / 2)) needs no argument scaling and sinc * 2 pi = sin(2 pi u) / u needs no division by
     * pi/2. For choice 0 the constant (2 pi)^n is left in every term: wq(u) = S w(4u), S = wqScale(), and the loops
     * divide their sums by S once per target (every term of a sum carries exactly one kernel value). v dW/dv needs no
     * division either: v d(sinc^n)/dv = n sinc^(n-1) (cos x - sinc). Choice 1 (the sinc^4 / sinc^9 mix): S = 1. */
    SPHX_HD HT wqScale() const
    {
        // (in double: once per target, and the fp32 exp2 would add its ulp to every sum)
        constexpr double log2TwoPi = 2.651496129472318798043279295;
        return (kN || choice == 0) ? HT(exp2(double(nVal()) * log2TwoPi)) : HT(1);
    }
    SPHX_HD HT wq(HT u) const
    {
        if (generic()) return w(HT(4) * u);
        constexpr HT twoPi = HT(6.283185307179586);
        HT sq = __builtin_amdgcn_sinf(u) * rcpF(u);
        sq    = u > HT(0) ? sq : twoPi; // (r = 0: sinc = 1)
        HT r;
        if constexpr (kN != 0) r = powC<kN>(sq);
        else r = powN(sq, n);
        return u < HT(0.5) ? r : HT(0);
    }
    /*! @brief wq for a neighbor of the list of the target whose h defines u: the search's exact fp64 test put it
     *         inside 2h, so u < 1/2 up to the fp32 rounding of u. No support test: at u = 1/2 (1 + eps) the sine is
     *         ~1e-7 and its n-th power below 1e-40, which is the kernel value there. (u = 0 keeps sinc = 1.) */
    SPHX_HD HT wqIn(HT u) const
    {
        if (generic()) return w(HT(4) * u);
        constexpr HT twoPi = HT(6.283185307179586);
        HT sq = __builtin_amdgcn_sinf(u) * rcpF(u);
        sq    = u > HT(0) ? sq : twoPi;
        if constexpr (kN != 0) return powC<kN>(sq);
        else return powN(sq, n);
    }
    //! @brief S w(4u) and S v dW/dv at v = 4u for a list neighbor (see wq, wqIn: no support test)
    SPHX_HD void wdq(HT u, HT& wS, HT& vdwS) const
    {
        if (generic())
        {
            wS   = w(HT(4) * u);
            vdwS = HT(4) * u * dw(HT(4) * u);
            return;
        }
        constexpr HT twoPi = HT(6.283185307179586);
        HT sq = __builtin_amdgcn_sinf(u) * rcpF(u);
        sq    = u > HT(0) ? sq : twoPi;
        const HT cs = __builtin_amdgcn_cosf(u);
        HT p;
        if constexpr (kN != 0) p = powC<kN - 1>(sq);
        else p = powN(sq, n - HT(1));
        wS   = p * sq;
        vdwS = nVal() * p * (twoPi * cs - sq);
    }
#else
    SPHX_HD HT w(HT v) const { return tableLookup(wh, v); }
    SPHX_HD HT dw(HT v) const { return tableLookup(whd, v); }
    //! host forms of the quarter-argument interface (no scaling: S = 1)
    SPHX_HD HT wqScale() const { return HT(1); }
    SPHX_HD HT wq(HT u) const { return w(HT(4) * u); }
    SPHX_HD HT wqIn(HT u) const { return w(HT(4) * u); }
    SPHX_HD void wdq(HT u, HT& wS, HT& vdwS) const
    {
        wS   = w(HT(4) * u);
        vdwS = HT(4) * u * dw(HT(4) * u);
    }
#endif
};
using KernelFn      = KernelFnT<0>;
using KernelFnSinc6 = KernelFnT<6>;

//! @brief smoothing length update targeting ng0 neighbors (reference kernels.hpp updateH)
template<class T>
SPHX_HD T updateH(unsigned ng0, unsigned nc, T h)
{
    constexpr T c0 = T(1023.0);
    constexpr T ex = T(1.0 / 10.0);
    return h * T(0.5) * pow(T(1) + c0 * T(ng0) / T(nc), ex);
}

template<class T>
SPHX_HD T tsKCourant(T maxvsignal, T h, T c, T Kcour)
{
    T v = maxvsignal > T(0) ? maxvsignal : c;
    return Kcour * h / v;
}

SPHX_HD double idealGasCv(double mui, double gamma)
{
    constexpr double R = 8.317e7;
    return R / mui / (gamma - 1.0);
}

//! @brief ideal gas EOS from temperature: returns p, c
SPHX_HD void idealGasEOS(double temp, double rho, double mui, double gamma, double& p, double& c)
{
    double tmp = idealGasCv(mui, gamma) * temp * (gamma - 1.0);
    p          = rho * tmp;
    c          = sqrt(tmp);
}

/*! @brief polytropic EOS p = K rho^gamma (gamma = 3) of a 1.4 M_sun, 12.8 km neutron star (K fixed for that star,
 *         reference sph/include/sph/eos.hpp:50-85 polytropicEOS / computeEOS_Polytropic); returns p, c
 */
SPHX_HD void polytropicEOS(double rho, double& p, double& c)
{
    constexpr double Kpol = 2.246341237993810232e-10, gammaPol = 3.0;
    p                     = Kpol * rho * rho * rho;
    c                     = sqrt(gammaPol * p / rho);
}

//! @brief ideal gas EOS from internal energy: returns p, c
SPHX_HD void idealGasEOSu(double u, double rho, double gamma, double& p, double& c)
{
    double tmp = u * (gamma - 1.0);
    p          = rho * tmp;
    c          = sqrt(tmp);
}

template<class T>
SPHX_HD T artificialViscosity(T alpha_i, T alpha_j, T c_i, T c_j, T w_ij)
{
    constexpr T beta = T(2.0);
    T visc           = T(0);
    if (w_ij < T(0))
    {
        T vsig = (alpha_i + alpha_j) / T(4) * (c_i + c_j) - beta * w_ij;
        visc   = -vsig * w_ij;
    }
    return visc;
}

//! @brief Adams-Bashforth 2 energy update (reference positions.hpp energyUpdate)
SPHX_HD double energyUpdate(double u_old, double dt, double dt_m1, double du, double du_m1)
{
    double deltaA = 0.5 * dt * dt / dt_m1;
    double deltaB = dt + deltaA;
    double u_new  = u_old + du * deltaB - du_m1 * deltaA;
    if (u_new < 0.) { u_new = u_old * exp(u_new * dt / u_old); }
    return u_new;
}

// ---------------------------------------------------------------------------------------------------------
// source records
// ---------------------------------------------------------------------------------------------------------

//! @brief position + mass (xmass, kx/gradh): 32 B
struct alignas(16) SrcPos
{
    CT x, y, z;
    HT m;
    HT xm;
};

//! @brief IAD + divv/curlv + AV switches: 48 B (three 16-B chunks); vol = xm/kx (VE) or m/rho (STD). The IAD and
//!        divv/curlv loops read xm, the AV-switch loop reads c (and divv): they share one slot, filled by the pack
//!        for the loop that follows.
struct alignas(16) SrcIad
{
    CT x, y, z;
    HT vol;
    HT vx, vy, vz;
    union
    {
        HT xm;
        HT c;
    };
    HT divv;
};
static_assert(!kHydroF32 || sizeof(SrcIad) == 48, "SrcIad is three 16-byte chunks");

//! @brief VE momentum/energy: 96 B (+ velocity gradient for AV cleaning: 128 B). Per-particle factors of the pair
//!        terms are precomputed at pack time (1/h, m/rho) so the pair loop has no divisions.
struct alignas(16) SrcMom
{
    CT x, y, z;
    HT vx, vy, vz;
    HT ih;
    HT c11, c12, c13, c22, c23, c33;
    HT m, c, xm, rho;
    HT prho, alpha, mrho;
};

struct alignas(16) SrcGradV
{
    HT dV[6];
    HT pad[2];
};

//! @brief STD momentum/energy: 80 B
struct alignas(16) SrcStd
{
    CT x, y, z;
    HT vx, vy, vz, ih;
    HT c11, c12, c13, c22, c23, c33;
    HT m, rho, p, c;
};

//! @brief fixed-point (QFrame) variants of the gfx950 records: XMass 16 B, Gradh with uniform mass 16 B (the mass
//!        comes from the launch), IAD + divv/curlv 32 B, VE momentum 80 B
struct alignas(16) SrcPosQ
{
    uint32_t x, y, z;
    HT m;
};

struct alignas(16) SrcXmQ
{
    uint32_t x, y, z;
    HT xm;
};

struct alignas(16) SrcIadQ
{
    uint32_t x, y, z;
    HT vol;
    HT vx, vy, vz;
    HT xm;
};
static_assert(!kHydroF32 || sizeof(SrcIadQ) == 32, "SrcIadQ is two 16-byte chunks");

struct alignas(16) SrcMomQ
{
    uint32_t x, y, z;
    HT vx, vy, vz;
    HT ih;
    HT c11, c12, c13, c22, c23, c33;
    HT m, c, xm, rho;
    HT prho, alpha, mrho;
};
static_assert(!kHydroF32 || sizeof(SrcMomQ) == 80, "SrcMomQ is five 16-byte chunks");

/*! @brief VE momentum records of the fixed-point, uniform-mass path: a 64-B main record plus an 8-B side record.
 *
 * The pair loops are bound by the texture addresser, which spends one cycle per 64-B cache segment a wave
 * instruction touches (profiles/r5: TA_BUSY ~= TCP_TOTAL_CACHE_ACCESSES, 28.6 accesses per cooperative SrcMomQ load =
 * 13 records x 2.25 segments). A 64-B record in a 64-B aligned array is exactly one segment: the cooperative gather
 * of a step then touches 64 segments instead of 143. With the mass uniform (taken from the launch) and m/rho derived
 * from rho, the momentum loop's 18 source dwords are these 16 + {rho, alpha} in the side array (one dwordx2 gather).
 */
struct alignas(64) SrcMomQ64
{
    uint32_t x, y, z;
    HT vx, vy, vz;
    HT ih;
    HT c11, c12, c13, c22, c23, c33;
    HT c, xm, prho;
};
static_assert(!kHydroF32 || sizeof(SrcMomQ64) == 64, "SrcMomQ64 is one 64-byte segment");

struct alignas(8) SrcMomSide
{
    HT rho, alpha;
};

//! @brief the momentum loop's record from the split form (m uniform, m/rho derived)
SPHX_HD SrcMomQ momOfSplit(const SrcMomQ64& a, const SrcMomSide& s, HT m)
{
    SrcMomQ r;
    r.x     = a.x;
    r.y     = a.y;
    r.z     = a.z;
    r.vx    = a.vx;
    r.vy    = a.vy;
    r.vz    = a.vz;
    r.ih    = a.ih;
    r.c11   = a.c11;
    r.c12   = a.c12;
    r.c13   = a.c13;
    r.c22   = a.c22;
    r.c23   = a.c23;
    r.c33   = a.c33;
    r.m     = m;
    r.c     = a.c;
    r.xm    = a.xm;
    r.rho   = s.rho;
    r.prho  = a.prho;
    r.alpha = s.alpha;
    r.mrho  = m * rcpF(s.rho);
    return r;
}

//! @brief source mass of a Gradh record: stored, or the uniform mass of the launch (SrcXmQ)
SPHX_HD HT massOf(const SrcPos& p, HT) { return p.m; }
SPHX_HD HT massOf(const SrcXmQ&, HT mUniform) { return mUniform; }

//! @brief pair separation (i - j) in hydro precision with the j-loop periodic fold at 2h_i
SPHX_HD void pairDelta(CT xi, CT yi, CT zi, CT xj, CT yj, CT zj, HT hi, const Box& box, HT& rx, HT& ry, HT& rz)
{
    rx = HT(xi - xj);
    ry = HT(yi - yj);
    rz = HT(zi - zj);
    foldPbc(box, HT(2) * hi, rx, ry, rz);
}

/*! @brief fixed-point coordinate frame of the gfx950 source records: coordinates become 32-bit offsets in the box.
 *         Periodic dimensions span the full 2^32 range, so the wrapping int32 difference of two offsets IS the
 *         minimum image (no fold); open dimensions use 2^31 per box length: the box is the bounding box of the
 *         particles (Domain.update_box), so offsets lie in [0, 2^31] and a difference of two of them never wraps to a
 *         small value (|dx| <= L -> |int32 difference| <= 2^31; only a difference of exactly 2^31 flips its sign and
 *         stays far). Quantizing the positions costs at most one quantum q (L/2^32 periodic, L/2^31 open) per separation component; the
 *         integer difference is then exact and rounds once to fp32. The host admits this path only while
 *         q <= 2^-22 h_min (ops/hydro.py FIXED_POINT_REL_QUANTUM), i.e. within 2-4x of the reference's fp32 rounding
 *         of its fp64 difference at the kernel support of the smallest particle, and below it for h >= 4 h_min;
 *         otherwise the loops read fp64-coordinate records. Records shrink by 12 B, which is what lets XMass,
 *         Gradh (uniform mass), IAD and momentum drop one 16-B gather chunk per neighbor.
 */
struct QFrame
{
    double lo[3], s[3]; // offset = rint((x - lo) * s) mod 2^32
    float inv[3];       // separation = int32(offset_i - offset_j) * inv
};

/*! @brief frame of the pair loops: SphConsts::fixedPoint = 1 | shift_x << 1 | shift_y << 6 | shift_z << 11 (0: fp64
 *         records). A shift of k multiplies the scale by 2^k: offsets then wrap with period P = L / 2^k (periodic) or
 *         2L / 2^k (open). The wrapping int32 difference is still the exact separation of every pair closer than P/2,
 *         and the pair loops only evaluate pairs within 2 h_i: the host picks the largest shifts with P/2 > 2 h_max
 *         (ops/hydro.py fixed_point_code), so a box whose smallest h is far below its extent (a collapsing cloud)
 *         keeps 32-bit records with quanta of P/2^32 instead of L/2^31. Periodic images move an offset by a multiple
 *         of 2^32 (L is 2^k periods), so the wrapped difference stays the minimum image. The neighbor search needs
 *         the unwrapped box frame (candidates lie farther than 2h) and always uses shift 0 (code 1).
 */
inline QFrame qframeOf(const Box& b, int code = 1)
{
    QFrame q;
    for (int d = 0; d < 3; ++d)
    {
        const double L   = b.len(d) > 0 ? b.len(d) : 1.0;
        const int shift  = (code >> (1 + 5 * d)) & 31;
        q.lo[d]          = b.lo[d];
        q.s[d]           = std::ldexp(1.0, (b.periodic(d) ? 32 : 31) + shift) / L;
        q.inv[d]         = float(1.0 / q.s[d]);
    }
    return q;
}

//! offset modulo 2^32 ((v - lo) * s stays below 2^52 for shifts <= 20, ops/hydro.py MAX_FRAME_SHIFT)
SPHX_HD uint32_t quantize(double v, double lo, double s)
{
    return uint32_t((unsigned long long)(long long)rint((v - lo) * s));
}

//! @brief pair separation of two records with fp64 coordinates (minimum image folded at 2h_i)
template<class R>
SPHX_HD void pairSep(const Box& box, const R& pi, const R& pj, HT hi, HT& rx, HT& ry, HT& rz)
{
    pairDelta(pi.x, pi.y, pi.z, pj.x, pj.y, pj.z, hi, box, rx, ry, rz);
}

//! @brief pair separation of two fixed-point records (QFrame): wrapping integer difference, one fp32 rounding (plus the
//!        position quantization of the records, see QFrame)
template<class R>
SPHX_HD void pairSep(const QFrame& q, const R& pi, const R& pj, HT, HT& rx, HT& ry, HT& rz)
{
    rx = HT(int32_t(pi.x - pj.x)) * q.inv[0];
    ry = HT(int32_t(pi.y - pj.y)) * q.inv[1];
    rz = HT(int32_t(pi.z - pj.z)) * q.inv[2];
}

/*! @brief v held in a vector register from here on (GPU). On gfx950 VALU instructions that read an SGPR operand issue
 *         at ~60 % of the rate of their all-VGPR forms (fma/mul/add: ~1.7x slower, scripts/micro/valu_cost.hip), so
 *         the pair loops copy their loop-invariant uniform constants to VGPRs once. Host: identity. */
template<class T>
SPHX_HD T inVgpr(T v)
{
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(v));
#endif
    return v;
}

//! @brief the frame of a pair loop with its inverse quanta in VGPRs (inVgpr); fp64 boxes unchanged
SPHX_HD QFrame vgprFrame(QFrame q)
{
    for (int k = 0; k < 3; ++k)
        q.inv[k] = inVgpr(q.inv[k]);
    return q;
}
SPHX_HD const Box& vgprFrame(const Box& b) { return b; }

//! @brief 1/sqrt(x) in hydro precision (annotation.hpp rsqrtF)
SPHX_HD HT rsqrtH(HT x) { return rsqrtF(x); }

// ---------------------------------------------------------------------------------------------------------
// VE formulation
// ---------------------------------------------------------------------------------------------------------


// gathers in flight per lane and loop kind (tuned on MI355X; see profiles/)
#ifndef SPHX_BATCH_POS
#define SPHX_BATCH_POS 4
#endif
#ifndef SPHX_BATCH_IAD
#define SPHX_BATCH_IAD 2
#endif
#ifndef SPHX_BATCH_MOM
#define SPHX_BATCH_MOM 1
#endif

#if defined(__HIP_DEVICE_COMPILE__)
constexpr bool kDeviceBatching = true;
#else
constexpr bool kDeviceBatching = false;
#endif

/*! @brief neighbor loop with memory-level parallelism: on the GPU, B indices and then B source records are loaded
 *         before the B pair evaluations run, so every wave keeps B independent gathers in flight (the pair loops
 *         are latency bound otherwise: one dependent index->record->math chain per iteration). The OpenMP build
 *         evaluates one neighbor at a time. Evaluation order (and hence the floating-point sums) is unchanged.
 */
//! @brief list stride value of the GPU layout: 4-entry blocks per lane, blocks of one group 256 entries apart
constexpr int kBlockedList = -4;

//! @brief neighbor k of a list (see the file comment for the two layouts)
template<class Idx>
SPHX_HD Idx listAt(const Idx* nbr, int stride, unsigned k)
{
    return stride == kBlockedList ? nbr[size_t(k >> 2) * 256 + (k & 3)] : nbr[size_t(k) * size_t(stride)];
}

template<int B, class Idx, class Ld, class F>
SPHX_HD void forEachNeighbor(const Idx* nbr, int stride, unsigned nc, const Ld& ld, F&& f)
{
    using Rec  = decltype(ld(0u));
    unsigned k = 0;
    if constexpr (kDeviceBatching && B > 1)
    {
        for (; k + B <= nc; k += B)
        {
            unsigned j[B];
            Rec r[B];
#pragma unroll
            for (int u = 0; u < B; ++u)
                j[u] = unsigned(listAt(nbr, stride, k + u));
#pragma unroll
            for (int u = 0; u < B; ++u)
                r[u] = ld(j[u]);
#pragma unroll
            for (int u = 0; u < B; ++u)
                f(j[u], r[u]);
        }
    }
#pragma nounroll
    for (; k < nc; ++k)
    {
        unsigned j = unsigned(listAt(nbr, stride, k));
        f(j, ld(j));
    }
}

#ifndef SPHX_COOP_MIN_CHUNKS
#define SPHX_COOP_MIN_CHUNKS 3 // records of fewer 16-byte chunks use per-lane gathers (A/B measured, profiles/)
#endif

#if defined(__HIPCC__)
//! @brief double from the two 32-bit halves of a staged chunk
__device__ __forceinline__ double chunkDouble(float lo, float hi)
{
    return __hiloint2double(__float_as_int(hi), __float_as_int(lo));
}

/*! @brief record from its staged 16-byte chunks, field by field in registers. A memcpy/bit-cast of the chunk array
 *         into the record would leave a private array that the compiler promotes to LDS (per-lane ds_write_b64 /
 *         ds_read_b32..b128 round trips with 2-4 way bank conflicts on every neighbor).
 */
template<class R>
__device__ R coopUnpack(const float4* o);

template<>
__device__ __forceinline__ SrcPos coopUnpack<SrcPos>(const float4* o)
{
    static_assert(offsetof(SrcPos, m) == 24 && sizeof(SrcPos) == 32, "SrcPos layout");
    SrcPos r;
    r.x  = chunkDouble(o[0].x, o[0].y);
    r.y  = chunkDouble(o[0].z, o[0].w);
    r.z  = chunkDouble(o[1].x, o[1].y);
    r.m  = o[1].z;
    r.xm = o[1].w;
    return r;
}

template<>
__device__ __forceinline__ SrcIad coopUnpack<SrcIad>(const float4* o)
{
    static_assert(offsetof(SrcIad, vol) == 24 && offsetof(SrcIad, divv) == 44, "SrcIad layout");
    SrcIad r;
    r.x    = chunkDouble(o[0].x, o[0].y);
    r.y    = chunkDouble(o[0].z, o[0].w);
    r.z    = chunkDouble(o[1].x, o[1].y);
    r.vol  = o[1].z;
    r.vx   = o[1].w;
    r.vy   = o[2].x;
    r.vz   = o[2].y;
    r.xm   = o[2].z;
    r.divv = o[2].w;
    return r;
}

template<>
__device__ __forceinline__ SrcMom coopUnpack<SrcMom>(const float4* o)
{
    static_assert(offsetof(SrcMom, vx) == 24 && offsetof(SrcMom, c11) == 40 && offsetof(SrcMom, m) == 64 &&
                      offsetof(SrcMom, mrho) == 88 && sizeof(SrcMom) == 96,
                  "SrcMom layout");
    SrcMom r;
    r.x     = chunkDouble(o[0].x, o[0].y);
    r.y     = chunkDouble(o[0].z, o[0].w);
    r.z     = chunkDouble(o[1].x, o[1].y);
    r.vx    = o[1].z;
    r.vy    = o[1].w;
    r.vz    = o[2].x;
    r.ih    = o[2].y;
    r.c11   = o[2].z;
    r.c12   = o[2].w;
    r.c13   = o[3].x;
    r.c22   = o[3].y;
    r.c23   = o[3].z;
    r.c33   = o[3].w;
    r.m     = o[4].x;
    r.c     = o[4].y;
    r.xm    = o[4].z;
    r.rho   = o[4].w;
    r.prho  = o[5].x;
    r.alpha = o[5].y;
    r.mrho  = o[5].z;
    return r;
}

template<>
__device__ __forceinline__ SrcMomQ coopUnpack<SrcMomQ>(const float4* o)
{
    static_assert(offsetof(SrcMomQ, vx) == 12 && offsetof(SrcMomQ, c11) == 28 && offsetof(SrcMomQ, m) == 52 &&
                      offsetof(SrcMomQ, mrho) == 76,
                  "SrcMomQ layout");
    SrcMomQ r;
    r.x     = __float_as_uint(o[0].x);
    r.y     = __float_as_uint(o[0].y);
    r.z     = __float_as_uint(o[0].z);
    r.vx    = o[0].w;
    r.vy    = o[1].x;
    r.vz    = o[1].y;
    r.ih    = o[1].z;
    r.c11   = o[1].w;
    r.c12   = o[2].x;
    r.c13   = o[2].y;
    r.c22   = o[2].z;
    r.c23   = o[2].w;
    r.c33   = o[3].x;
    r.m     = o[3].y;
    r.c     = o[3].z;
    r.xm    = o[3].w;
    r.rho   = o[4].x;
    r.prho  = o[4].y;
    r.alpha = o[4].z;
    r.mrho  = o[4].w;
    return r;
}

template<>
__device__ __forceinline__ SrcMomQ64 coopUnpack<SrcMomQ64>(const float4* o)
{
    static_assert(offsetof(SrcMomQ64, vx) == 12 && offsetof(SrcMomQ64, c11) == 28 && offsetof(SrcMomQ64, c) == 52,
                  "SrcMomQ64 layout");
    SrcMomQ64 r;
    r.x    = __float_as_uint(o[0].x);
    r.y    = __float_as_uint(o[0].y);
    r.z    = __float_as_uint(o[0].z);
    r.vx   = o[0].w;
    r.vy   = o[1].x;
    r.vz   = o[1].y;
    r.ih   = o[1].z;
    r.c11  = o[1].w;
    r.c12  = o[2].x;
    r.c13  = o[2].y;
    r.c22  = o[2].z;
    r.c23  = o[2].w;
    r.c33  = o[3].x;
    r.c    = o[3].y;
    r.xm   = o[3].z;
    r.prho = o[3].w;
    return r;
}

template<>
__device__ __forceinline__ SrcIadQ coopUnpack<SrcIadQ>(const float4* o)
{
    SrcIadQ r;
    r.x   = __float_as_uint(o[0].x);
    r.y   = __float_as_uint(o[0].y);
    r.z   = __float_as_uint(o[0].z);
    r.vol = o[0].w;
    r.vx  = o[1].x;
    r.vy  = o[1].y;
    r.vz  = o[1].z;
    r.xm  = o[1].w;
    return r;
}

template<>
__device__ __forceinline__ SrcStd coopUnpack<SrcStd>(const float4* o)
{
    static_assert(offsetof(SrcStd, vx) == 24 && offsetof(SrcStd, c11) == 40 && offsetof(SrcStd, m) == 64 &&
                      sizeof(SrcStd) == 80,
                  "SrcStd layout");
    SrcStd r;
    r.x   = chunkDouble(o[0].x, o[0].y);
    r.y   = chunkDouble(o[0].z, o[0].w);
    r.z   = chunkDouble(o[1].x, o[1].y);
    r.vx  = o[1].z;
    r.vy  = o[1].w;
    r.vz  = o[2].x;
    r.ih  = o[2].y;
    r.c11 = o[2].z;
    r.c12 = o[2].w;
    r.c13 = o[3].x;
    r.c22 = o[3].y;
    r.c23 = o[3].z;
    r.c33 = o[3].w;
    r.m   = o[4].x;
    r.rho = o[4].y;
    r.p   = o[4].z;
    r.c   = o[4].w;
    return r;
}

/*! @brief record loader of the gfx950 pair loops: cooperative, cache-line-coalesced gathers staged through LDS.
 *
 * At neighbor step k every lane needs the C x 16-byte record of its own neighbor j. Loading it directly costs C
 * wave-wide gathers in which all 64 lanes touch different cache lines (64 L1 tag lookups per instruction, the
 * bottleneck of the pair loops). Here the wave loads the 64 records as 64*C consecutive 16-byte chunks: in
 * instruction q lane l fetches chunk p of record r, q*64 + l = r*C + p, so a record's chunks come from adjacent lanes
 * and one instruction touches ~64/C records' lines instead of 64. The chunks are written to a per-wave LDS tile
 * (record stride C|1 float4: conflict-free 16-lane groups) and every lane reads back its own record. The
 * neighbor index of record r comes from lane r (ds_bpermute). Indices are read two steps ahead and the gathers of
 * step k+1 are in flight while step k is evaluated. Lanes past their own neighbor count fetch @p self (valid
 * address) and skip the evaluation; all 64 lanes must call the loop (uniform trip count = wave max of nc).
 */
template<class R>
struct CoopLoader
{
    const R* r;
    float4* tile; // 64 * (C | 1) float4 of LDS per wave
    unsigned self; // the target's own record: stands in for list entries past the lane's count
    static constexpr int C = int(sizeof(R) / 16);
    static constexpr int S = C | 1;
    static_assert(sizeof(R) % 16 == 0, "records are whole float4s");

    __device__ R operator()(unsigned j) const { return r[j]; }

    //! @brief index of the record whose chunk this lane fetches in instruction q, from the owning lane's index j
    __device__ __forceinline__ unsigned spread(unsigned j, int q) const
    {
        const int rr = (q * 64 + int(threadIdx.x & 63)) / C;
        return unsigned(__shfl(int(j), rr));
    }

    //! @brief chunk q of the cooperative gather: this lane's 16 bytes of record rr = (q*64 + lane) / C
    __device__ __forceinline__ float4 issue(unsigned jr, int q) const
    {
        const int c  = q * 64 + (threadIdx.x & 63);
        const int rr = c / C;
        return reinterpret_cast<const float4*>(r)[size_t(jr) * C + (c - rr * C)];
    }

    __device__ __forceinline__ void stage(float4 v, int q) const
    {
        const int c  = q * 64 + (threadIdx.x & 63);
        const int rr = c / C;
        tile[rr * S + (c - rr * C)] = v;
    }

    __device__ __forceinline__ float4 own(int p) const { return tile[(threadIdx.x & 63) * S + p]; }
};

/*! @brief keep a loaded record in registers at this point. The packed-list loops skip entries equal to the target
 *         (jump/padding slots); a record whose fields are only used under that test would have its load sunk into
 *         the branch behind a full vmcnt(0) wait, serializing the batched gathers (measured on the AV loop). */
template<class T>
__device__ __forceinline__ void pinRegs(T& v)
{
    static_assert(sizeof(T) % 4 == 0, "records are whole dwords");
    uint32_t w[sizeof(T) / 4];
    __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
    for (unsigned k = 0; k < sizeof(T) / 4; ++k)
        asm volatile("" : "+v"(w[k]));
    __builtin_memcpy(&v, w, sizeof(T));
}

/*! @brief per-lane gather loop of the small records (any loader returning a record by value) over a packed list:
 *         one list block (8 entries) decoded per row, its records gathered 4 at a time */
template<class Ld, class F>
__device__ void forEachNeighborDirect(const PackedLane& pl, const Ld& ld, F&& f)
{
    // small records (cooperative path measured slower for 32 B): per-lane gathers, four records in flight (a
    // deeper software pipeline measured slower: more VGPRs, same texture work); the next list block is prefetched
    const unsigned nblk = pl.nblk;
    if (nblk == 0) return;
    int4 w     = pl.block(0);
    auto batch = [&](int w0, int w1)
    {
        unsigned j[4];
        pl.decode(w0, j[0], j[1]);
        pl.decode(w1, j[2], j[3]);
        decltype(ld(0u)) rr[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            rr[u] = ld(j[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
        {
            pinRegs(rr[u]);
            if (j[u] != pl.self) f(j[u], rr[u]);
        }
    };
    for (unsigned b = 0; b < nblk; ++b)
    {
        const int4 wn = pl.block(b + 1);
        batch(w.x, w.y);
        batch(w.z, w.w);
        w = wn;
    }
}

/*! @brief AV-switch source records on the fixed-point frame: 32 B stored (coordinates, vol, v, c) + divv read from
 *         its own field, i.e. two dwordx4 gathers and one dword gather per neighbor instead of three chunks of the
 *         48-B SrcIad (the six fields of the AV loop do not fit the 20 B left next to the coordinates) */
struct alignas(16) SrcAvQ
{
    uint32_t x, y, z;
    HT vol;
    HT vx, vy, vz;
    HT c;
};

struct SrcAvQd
{
    uint32_t x, y, z;
    HT vol, vx, vy, vz, c, divv;
};

struct AvQLoader
{
    const SrcAvQ* r;
    const HT* divv;
    __device__ SrcAvQd operator()(unsigned j) const
    {
        const SrcAvQ a = r[j];
        return SrcAvQd{a.x, a.y, a.z, a.vol, a.vx, a.vy, a.vz, a.c, divv[j]};
    }
};

template<int B, class F>
__device__ void forEachNeighbor(const PackedLane* pl, int, unsigned, const AvQLoader& ld, F&& f)
{
    forEachNeighborDirect(*pl, ld, f);
}

template<int B, class R, class F>
__device__ void forEachNeighbor(const PackedLane* plp, int, unsigned, const CoopLoader<R>& ld, F&& f)
{
    constexpr int C = CoopLoader<R>::C;
    constexpr bool direct = C < SPHX_COOP_MIN_CHUNKS;
    const PackedLane& pl = *plp;
    if constexpr (direct)
    {
        forEachNeighborDirect(pl, ld, f);
        return;
    }
    const unsigned nblk = pl.nblk;
    if (nblk == 0) return;
    // Neighbor indices come in 8-entry list blocks (one coalesced 1 KiB load per eight steps, one block ahead,
    // decoded through the group's chunk table in LDS), are spread to the chunk lanes with ds_bpermute two steps
    // ahead, and the chunk data is gathered one step ahead of the evaluation. Unrolled by eight with ping-pong
    // buffers (A/B data, I1/I2 indices): no register rotation. Padding codes and the target's own entry decode to
    // the target itself: gathered, not evaluated.
    auto consume = [&](const float4 (&raw)[C], unsigned j)
    {
        float4 o[C];
#pragma unroll
        for (int q = 0; q < C; ++q)
            ld.stage(raw[q], q);
#pragma unroll
        for (int p = 0; p < C; ++p)
            o[p] = ld.own(p);
#ifndef SPHX_COOP_NARROW
        // keep every chunk live as a whole: otherwise the fields a loop leaves unused split the 16-byte LDS reads
        // into ds_read_b32/b64/read2 pieces whose bank groups conflict 2-4 ways at the odd record strides
#pragma unroll
        for (int p = 0; p < C; ++p)
            asm volatile("" : "+v"(o[p].x), "+v"(o[p].y), "+v"(o[p].z), "+v"(o[p].w));
#endif
        const R rec = coopUnpack<R>(o);
        if (j != pl.self) f(j, rec);
    };
    unsigned D[8];
    // (the block decoded after the last one lies past the list and is never used: not checked)
    auto decodeChecked = [&](int4 w, bool used)
    {
        decodeBlock(w, pl.ctab, D);
#ifdef SPHX_DEVICE_CHECKS
#pragma unroll
        for (int u = 0; u < 8; ++u)
            D[u] = used ? pl.checked(D[u]) : D[u];
#endif
    };
    decodeChecked(pl.block(0), true);
    unsigned I1[C], I2[C];
    float4 A[C], Bf[C];
#pragma unroll
    for (int q = 0; q < C; ++q)
    {
        A[q]  = ld.issue(ld.spread(D[0], q), q);
        I1[q] = ld.spread(D[1], q);
    }
    for (unsigned b = 0; b < nblk; ++b)
    {
        const int4 W = pl.block(b + 1); // past the list: row 0 (valid memory), entries replaced below
        const bool more = b + 1 < nblk;
#pragma unroll
        for (int u = 0; u < 8; u += 2)
        {
            unsigned jA, jB;
            if (u < 6)
            {
                jA = D[u + 2];
                jB = D[u + 3];
            }
            else
            {
                // steps 6, 7 spread the first two entries of the next block (the target's own record past the list)
                decodeWord(W.x, pl.ctab, jA, jB);
                jA = more ? pl.checked(jA) : pl.self;
                jB = more ? pl.checked(jB) : pl.self;
            }
#pragma unroll
            for (int q = 0; q < C; ++q)
            {
                I2[q] = ld.spread(jA, q);
                Bf[q] = ld.issue(I1[q], q);
            }
            consume(A, D[u]);
#pragma unroll
            for (int q = 0; q < C; ++q)
            {
                I1[q] = ld.spread(jB, q);
                A[q]  = ld.issue(I2[q], q);
            }
            consume(Bf, D[u + 1]);
        }
        decodeChecked(W, more);
    }
}

/*! @brief loader of the split momentum records (SrcMomQ64 cooperative + SrcMomSide per lane, uniform mass): returns
 *         the assembled SrcMomQ, so momentumEnergyJLoop runs unchanged on it */
template<bool kBuf = false>
struct MomSplitLoaderT
{
    CoopLoader<SrcMomQ64> main;
    const SrcMomSide* side;
    HT m;
    // kBuf: the neighbor gathers as raw buffer loads with 32-bit byte offsets (both arrays < 4 GiB; the launcher
    // checks): one 32-bit shift-or per load instead of the two 64-bit address instructions of a global load
    // (v_lshlrev_b64 + v_lshl_add_u64, ~6.5 cycles each per wave on gfx950, profiles/r6/valu_cost_micro.txt) and the
    // moves that build their register pairs: 2055 -> 1984 VALU per 8-neighbor iteration. Measured on the 16/32-B
    // direct-gather loops (XMass, Gradh, IAD, AV) the same change was neutral or slower (profiles/r6/buffer_loads.md).
    __amdgpu_buffer_rsrc_t rsMain, rsSide;

    __device__ SrcMomQ operator()(unsigned j) const { return momOfSplit(main.r[j], side[j], m); }

    //! @brief chunk q of the cooperative gather (CoopLoader::issue)
    __device__ __forceinline__ float4 issue(unsigned jr, int q) const
    {
        if constexpr (!kBuf) return main.issue(jr, q);
        else
        {
            // chunk of this lane: (q * 64 + lane) mod 4 = lane mod 4 (64-B records, 4 chunks)
            static_assert(sizeof(SrcMomQ64) == 64, "four 16-B chunks");
            const unsigned off = (jr << 6) | ((threadIdx.x & 3u) << 4);
            typedef float f4v __attribute__((ext_vector_type(4)));
            const f4v v = __builtin_amdgcn_raw_buffer_load_b128(rsMain, off, 0, 0);
            return make_float4(v.x, v.y, v.z, v.w);
        }
    }
    __device__ __forceinline__ SrcMomSide sideAt(unsigned j) const
    {
        if constexpr (!kBuf) return side[j];
        else
        {
            static_assert(sizeof(SrcMomSide) == 8, "one 8-B load");
            typedef float f2v __attribute__((ext_vector_type(2)));
            const f2v v = __builtin_amdgcn_raw_buffer_load_b64(rsSide, j << 3, 0, 0);
            SrcMomSide r;
            __builtin_memcpy(&r, &v, 8);
            return r;
        }
    }
};
using MomSplitLoader = MomSplitLoaderT<false>;

/*! @brief the cooperative loop of forEachNeighbor(CoopLoader) for the split momentum records: the 64-B main records
 *         move as 4 chunks per record (16 records per wave instruction, one 64-B segment each), and each lane gathers
 *         its own 8-B side record with the same one-step-ahead schedule */
template<int B, bool kBuf, class F>
__device__ void forEachNeighbor(const PackedLane* plp, int, unsigned, const MomSplitLoaderT<kBuf>& ldm, F&& f)
{
    using R            = SrcMomQ64;
    const auto& ld     = ldm.main;
    constexpr int C    = CoopLoader<R>::C;
    const PackedLane& pl = *plp;
    const unsigned nblk  = pl.nblk;
    if (nblk == 0) return;
    auto consume = [&](const float4 (&raw)[C], const SrcMomSide& sd, unsigned j)
    {
        float4 o[C];
#pragma unroll
        for (int q = 0; q < C; ++q)
            ld.stage(raw[q], q);
#pragma unroll
        for (int p = 0; p < C; ++p)
            o[p] = ld.own(p);
#pragma unroll
        for (int p = 0; p < C; ++p)
            asm volatile("" : "+v"(o[p].x), "+v"(o[p].y), "+v"(o[p].z), "+v"(o[p].w));
        const SrcMomQ rec = momOfSplit(coopUnpack<R>(o), sd, ldm.m);
        if (j != pl.self) f(j, rec);
    };
    unsigned D[8];
    auto decodeChecked = [&](int4 w, bool used)
    {
        decodeBlock(w, pl.ctab, D);
#ifdef SPHX_DEVICE_CHECKS
#pragma unroll
        for (int u = 0; u < 8; ++u)
            D[u] = used ? pl.checked(D[u]) : D[u];
#endif
    };
    decodeChecked(pl.block(0), true);
    unsigned I1[C], I2[C];
    float4 A[C], Bf[C];
    SrcMomSide As, Bs;
#pragma unroll
    for (int q = 0; q < C; ++q)
    {
        A[q]  = ldm.issue(ld.spread(D[0], q), q);
        I1[q] = ld.spread(D[1], q);
    }
    As = ldm.sideAt(D[0]);
    for (unsigned b = 0; b < nblk; ++b)
    {
        const int4 W    = pl.block(b + 1);
        const bool more = b + 1 < nblk;
#pragma unroll
        for (int u = 0; u < 8; u += 2)
        {
            unsigned jA, jB;
            if (u < 6)
            {
                jA = D[u + 2];
                jB = D[u + 3];
            }
            else
            {
                decodeWord(W.x, pl.ctab, jA, jB);
                jA = more ? pl.checked(jA) : pl.self;
                jB = more ? pl.checked(jB) : pl.self;
            }
#pragma unroll
            for (int q = 0; q < C; ++q)
            {
                I2[q] = ld.spread(jA, q);
                Bf[q] = ldm.issue(I1[q], q);
            }
            Bs = ldm.sideAt(D[u + 1]);
            consume(A, As, D[u]);
#pragma unroll
            for (int q = 0; q < C; ++q)
            {
                I1[q] = ld.spread(jB, q);
                A[q]  = ldm.issue(I2[q], q);
            }
            As = ldm.sideAt(jA);
            consume(Bf, Bs, D[u + 1]);
        }
        decodeChecked(W, more);
    }
}
#endif

/*! @brief cross-wave reductions of the LDS-staged loops (csrc/hip/staged.h: W waves split one group's neighbor
 *         lists and add their partial sums after the loop). Every other loader: nothing to do. The J-loops start
 *         their sums at zero and add the target's own term after the reduction, so it is counted once. */
template<class Ld, class... T>
SPHX_HD void reduceAcross(const Ld&, T&...)
{
}
template<class Ld, class... T>
SPHX_HD void reduceAcrossMax(const Ld&, T&...)
{
}
template<class Ld>
SPHX_HD void reduceAcrossN(const Ld&, HT*, int)
{
}

//! @brief xm_i = m_i / rho0_i, rho0_i = K h^-3 sum_j W_ij m_j including self (reference xmass_kern.hpp)
template<class Idx, class Ld, class KF>
SPHX_HD HT xmassJLoop(unsigned i, double K, const Box& box, const Idx* nbr, int stride, unsigned nc, HT hi,
                      const Ld& ld, const KF& kf)
{
    SrcPos pi = ld(i);
    HT hInv = HT(1) / hi, h3Inv = hInv * hInv * hInv, hq = HT(0.25) * hInv;
    HT rho0 = 0;
    forEachNeighbor<SPHX_BATCH_POS>(nbr, stride, nc, ld, [&](unsigned j, const SrcPos& pj) {
        HT rx, ry, rz;
        pairDelta(pi.x, pi.y, pi.z, pj.x, pj.y, pj.z, hi, box, rx, ry, rz);
        HT dist = sqrtF(rx * rx + ry * ry + rz * rz);
        rho0 += kf.wqIn(dist * hq) * pj.m;
    });
    rho0 = pi.m + rho0 / kf.wqScale(); // (kernel scale, KernelFn::wq; the target's own term W(0) m_i)
    return pi.m / (rho0 * HT(K) * h3Inv);
}

//! @brief kx (VE normalization) and grad-h term (reference ve_def_gradh_kern.hpp)
template<class G, class Idx, class Ld, class KF>
SPHX_HD void veDefGradhJLoop(unsigned i, double K, const G& box, const Idx* nbr, int stride, unsigned nc, HT hi,
                             const Ld& ld, const KF& kf, HT& kxOut, HT& gradhOut,
                             HT mUniform = HT(0))
{
    const auto pi = ld(i);
    HT mi = massOf(pi, mUniform), xmi = pi.xm;
    HT hInv = HT(1) / hi, h3Inv = hInv * hInv * hInv, hq = HT(0.25) * hInv;

    HT kxi      = 0;
    HT whomegai = 0;
    HT wrho0i   = 0;
    const auto bx = vgprFrame(box);
    forEachNeighbor<SPHX_BATCH_POS>(nbr, stride, nc, ld, [&](unsigned j, const auto& pj) {
        HT rx, ry, rz;
        pairSep(bx, pi, pj, hi, rx, ry, rz);
        HT dist  = sqrtF(rx * rx + ry * ry + rz * rz);
        HT w, vdw; // (S-scaled, KernelFn::wdq)
        kf.wdq(dist * hq, w, vdw);
        HT dterh = -(HT(3) * w + vdw);
        HT xmj   = pj.xm;
        kxi += w * xmj;
        whomegai += dterh * xmj;
        wrho0i += dterh * massOf(pj, mUniform);
    });
    reduceAcross(ld, kxi, whomegai, wrho0i);
    // the kernel scale, then the target's own terms: W(0) = 1, dW(0) = 0
    const HT invS = HT(1) / kf.wqScale();
    kxi      = xmi + kxi * invS;
    whomegai = -HT(3) * xmi + whomegai * invS;
    wrho0i   = -HT(3) * mi + wrho0i * invS;
    HT Kf = HT(K);
    kxi *= Kf * h3Inv;
    whomegai *= Kf * h3Inv * hInv;
    wrho0i *= Kf * h3Inv * hInv;

    whomegai  = whomegai * mi / xmi + (kxi - Kf * xmi * h3Inv) * wrho0i;
    HT rhoi   = kxi * mi / xmi;
    HT dhdrho = -hi / (rhoi * HT(3));
    kxOut     = kxi;
    gradhOut  = HT(1) - dhdrho * whomegai;
}

//! @brief invert the IAD tau matrix into c11..c33 with exponent normalization (reference iad_kern.hpp)
SPHX_HD void invertTau(HT tau[6], HT hi, double K, HT c[6])
{
    auto getExp = [](HT v) { return v == HT(0) ? 0 : ilogb(v); };
    int expSum  = getExp(tau[0]) + getExp(tau[1]) + getExp(tau[2]) + getExp(tau[3]) + getExp(tau[4]) + getExp(tau[5]);
    HT norm     = ldexp(HT(1), -expSum / 6);
    for (int k = 0; k < 6; ++k)
        tau[k] *= norm;
    HT t11 = tau[0], t12 = tau[1], t13 = tau[2], t22 = tau[3], t23 = tau[4], t33 = tau[5];
    HT det = t11 * t22 * t33 + HT(2) * t12 * t23 * t13 - t11 * t23 * t23 - t22 * t13 * t13 - t33 * t12 * t12;
    HT factor = norm * (hi * hi * hi) / (det * HT(K));
    c[0]      = (t22 * t33 - t23 * t23) * factor;
    c[1]      = (t13 * t23 - t33 * t12) * factor;
    c[2]      = (t12 * t23 - t22 * t13) * factor;
    c[3]      = (t11 * t33 - t13 * t13) * factor;
    c[4]      = (t13 * t12 - t11 * t23) * factor;
    c[5]      = (t11 * t22 - t12 * t12) * factor;
}

//! @brief IAD matrix with volumes vol_j (VE: xm/kx, STD: m/rho) (reference hydro_ve/iad_kern.hpp, hydro_std)
template<class Idx, class Ld>
SPHX_HD void iadJLoop(unsigned i, double K, const Box& box, const Idx* nbr, int stride, unsigned nc, HT hi,
                      const Ld& ld, const KernelFn& kf, HT c[6])
{
    HT tau[6] = {0, 0, 0, 0, 0, 0};
    SrcIad pi = ld(i);
    HT hq     = HT(0.25) / hi;
    forEachNeighbor<SPHX_BATCH_IAD>(nbr, stride, nc, ld, [&](unsigned j, const SrcIad& pj) {
        HT rx, ry, rz;
        pairDelta(pi.x, pi.y, pi.z, pj.x, pj.y, pj.z, hi, box, rx, ry, rz);
        HT dist = sqrtF(rx * rx + ry * ry + rz * rz);
        HT w    = kf.wqIn(dist * hq);
        HT vw   = pj.vol * w;
        tau[0] += rx * rx * vw;
        tau[1] += rx * ry * vw;
        tau[2] += rx * rz * vw;
        tau[3] += ry * ry * vw;
        tau[4] += ry * rz * vw;
        tau[5] += rz * rz * vw;
    });
    const HT invS = HT(1) / kf.wqScale();
    for (int k = 0; k < 6; ++k)
        tau[k] *= invS;
    invertTau(tau, hi, K, c);
}

//! @brief velocity divergence, |curl|, optional symmetric velocity gradient (reference divv_curlv_kern.hpp)
template<class Idx, class Ld>
SPHX_HD void divvCurlvJLoop(unsigned i, double K, const Box& box, const Idx* nbr, int stride, unsigned nc, HT hi,
                            HT kxi, const HT ci[6], const Ld& ld, const KernelFn& kf, HT& divvOut, HT& curlvOut, HT* dV)
{
    SrcIad pi = ld(i);
    HT hInv = HT(1) / hi, hInv3 = hInv * hInv * hInv, hq = HT(0.25) * hInv;
    HT c11 = ci[0], c12 = ci[1], c13 = ci[2], c22 = ci[3], c23 = ci[4], c33 = ci[5];
    HT dVx[3] = {0, 0, 0}, dVy[3] = {0, 0, 0}, dVz[3] = {0, 0, 0};
    forEachNeighbor<SPHX_BATCH_IAD>(nbr, stride, nc, ld, [&](unsigned j, const SrcIad& pj) {
        HT rx, ry, rz;
        pairDelta(pi.x, pi.y, pi.z, pj.x, pj.y, pj.z, hi, box, rx, ry, rz);
        HT dist = sqrtF(rx * rx + ry * ry + rz * rz);
        HT vxji = pj.vx - pi.vx, vyji = pj.vy - pi.vy, vzji = pj.vz - pi.vz;
        HT W    = kf.wqIn(dist * hq);
        HT tA0  = -(c11 * rx + c12 * ry + c13 * rz) * W;
        HT tA1  = -(c12 * rx + c22 * ry + c23 * rz) * W;
        HT tA2  = -(c13 * rx + c23 * ry + c33 * rz) * W;
        HT xmj  = pj.xm;
        HT ax = vxji * xmj, ay = vyji * xmj, az = vzji * xmj;
        dVx[0] += ax * tA0;
        dVx[1] += ax * tA1;
        dVx[2] += ax * tA2;
        dVy[0] += ay * tA0;
        dVy[1] += ay * tA1;
        dVy[2] += ay * tA2;
        dVz[0] += az * tA0;
        dVz[1] += az * tA1;
        dVz[2] += az * tA2;
    });
    HT nk   = HT(K) * hInv3 / (kxi * kf.wqScale());
    divvOut = nk * (dVx[0] + dVy[1] + dVz[2]);
    HT cx = dVz[1] - dVy[2], cy = dVx[2] - dVz[0], cz = dVy[0] - dVx[1];
    curlvOut = nk * sqrt(cx * cx + cy * cy + cz * cz);
    if (dV)
    {
        dV[0] = nk * dVx[0];
        dV[1] = nk * (dVx[1] + dVy[0]);
        dV[2] = nk * (dVx[2] + dVz[0]);
        dV[3] = nk * dVy[1];
        dV[4] = nk * (dVy[2] + dVz[1]);
        dV[5] = nk * dVz[2];
    }
}

/*! @brief IAD matrix and velocity divergence/curl in ONE pass over the neighbors
 *
 * The reference (iad_divv_curlv_gpu.cu) runs the IAD loop, inverts tau into c_i, then runs a second loop where every
 * term is -(c_i . r_ij) W_ij v_ji xm_j. Because c_i is constant over j, the second loop equals -c_i . M with
 * M[a][b] = sum_j v_ji[a] xm_j W_ij r_ij[b], so M is accumulated together with tau and the neighbor data is read
 * once. Mathematically identical; rounding differs from the two-pass form at the 1e-7 relative level.
 */
template<bool kAvS = false, class G, class Idx, class Ld, class KF>
SPHX_HD void iadDivvCurlvJLoop(unsigned i, double K, const G& box, const Idx* nbr, int stride, unsigned nc, HT hi,
                               HT kxi, const Ld& ld, const KF& kf, HT c[6], HT& divvOut, HT& curlvOut, HT* dV,
                               HT* avS = nullptr)
{
    HT tau[6]  = {0, 0, 0, 0, 0, 0};
    HT M[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    HT S[3]    = {0, 0, 0};
    const auto pi = ld(i);
    HT hInv = HT(1) / hi, hInv3 = hInv * hInv * hInv, hq = HT(0.25) * hInv;
    const auto bx = vgprFrame(box);
    forEachNeighbor<SPHX_BATCH_IAD>(nbr, stride, nc, ld, [&](unsigned j, const auto& pj) {
        HT rx, ry, rz;
        pairSep(bx, pi, pj, hi, rx, ry, rz);
        HT dist = sqrtF(rx * rx + ry * ry + rz * rz);
        HT w    = kf.wqIn(dist * hq);
        HT vw   = pj.vol * w;
        tau[0] += rx * rx * vw;
        tau[1] += rx * ry * vw;
        tau[2] += rx * rz * vw;
        tau[3] += ry * ry * vw;
        tau[4] += ry * rz * vw;
        tau[5] += rz * rz * vw;
        if constexpr (kAvS)
        {
            S[0] += vw * rx;
            S[1] += vw * ry;
            S[2] += vw * rz;
        }
        HT xw = pj.xm * w;
        HT ax = (pj.vx - pi.vx) * xw, ay = (pj.vy - pi.vy) * xw, az = (pj.vz - pi.vz) * xw;
        M[0][0] += ax * rx;
        M[0][1] += ax * ry;
        M[0][2] += ax * rz;
        M[1][0] += ay * rx;
        M[1][1] += ay * ry;
        M[1][2] += ay * rz;
        M[2][0] += az * rx;
        M[2][1] += az * ry;
        M[2][2] += az * rz;
    });
    reduceAcrossN(ld, tau, 6);
    reduceAcrossN(ld, &M[0][0], 9);
    if constexpr (kAvS) reduceAcrossN(ld, S, 3);
    {
        // the kernel scale (KernelFn::wq)
        const HT invS = HT(1) / kf.wqScale();
        for (int k = 0; k < 6; ++k)
            tau[k] *= invS;
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b)
                M[a][b] *= invS;
        if constexpr (kAvS)
            for (int k = 0; k < 3; ++k)
                S[k] *= invS;
    }
    invertTau(tau, hi, K, c);
    if constexpr (kAvS)
    {
        avS[0] = S[0];
        avS[1] = S[1];
        avS[2] = S[2];
    }
    // dV_a[k] = -sum_b c[k][b] M[a][b], c symmetric (c11 c12 c13 c22 c23 c33)
    HT dVv[3][3];
    for (int a = 0; a < 3; ++a)
    {
        dVv[a][0] = -(c[0] * M[a][0] + c[1] * M[a][1] + c[2] * M[a][2]);
        dVv[a][1] = -(c[1] * M[a][0] + c[3] * M[a][1] + c[4] * M[a][2]);
        dVv[a][2] = -(c[2] * M[a][0] + c[4] * M[a][1] + c[5] * M[a][2]);
    }
    HT nk   = HT(K) * hInv3 / kxi;
    divvOut = nk * (dVv[0][0] + dVv[1][1] + dVv[2][2]);
    HT cx = dVv[2][1] - dVv[1][2], cy = dVv[0][2] - dVv[2][0], cz = dVv[1][0] - dVv[0][1];
    curlvOut = nk * sqrt(cx * cx + cy * cy + cz * cz);
    if (dV)
    {
        dV[0] = nk * dVv[0][0];
        dV[1] = nk * (dVv[0][1] + dVv[1][0]);
        dV[2] = nk * (dVv[0][2] + dVv[2][0]);
        dV[3] = nk * dVv[1][1];
        dV[4] = nk * (dVv[1][2] + dVv[2][1]);
        dV[5] = nk * dVv[2][2];
    }
}

//! @brief Cullen-Dehnen style AV switch (reference av_switches_kern.hpp)
template<class G, class Idx, class Ld>
SPHX_HD HT avSwitchesJLoop(unsigned i, double K, const G& box, const Idx* nbr, int stride, unsigned nc, HT hi,
                           const HT ci6[6], const Ld& ld, const KernelFn& kf, double dt, HT alphamin, HT alphamax,
                           HT decayConstant, HT alpha_i)
{
    const auto pi = ld(i);
    HT ci     = pi.c;
    HT c11 = ci6[0], c12 = ci6[1], c13 = ci6[2], c22 = ci6[3], c23 = ci6[4], c33 = ci6[5];
    HT vsig  = HT(1.e-40) * ci;
    HT hInv  = HT(1) / hi, hInv3 = hInv * hInv * hInv, hq = HT(0.25) * hInv;
    HT divvi = pi.divv;
    HT gx = 0, gy = 0, gz = 0;
    const HT KhS = HT(K) * hInv3 / kf.wqScale();
    forEachNeighbor<SPHX_BATCH_IAD>(nbr, stride, nc, ld, [&](unsigned j, const auto& pj) {
        HT rx, ry, rz;
        pairSep(box, pi, pj, hi, rx, ry, rz);
        HT r2      = rx * rx + ry * ry + rz * rz;
        HT invDist = rsqrtH(r2);
        HT dist    = r2 * invDist;
        HT vxij = pi.vx - pj.vx, vyij = pi.vy - pj.vy, vzij = pi.vz - pj.vz;
        HT rv   = rx * vxij + ry * vyij + rz * vzij;
        // branch-free: a branch here lets the compiler sink the load of pj.c into it, behind a full vmcnt(0) that
        // serializes the batched gathers (AV 36 % slower than IAD before, profiles/r2_perf_log.md)
        HT vst  = ci + pj.c - HT(3) * rv * invDist;
        HT vsij = rv < HT(0) ? vst : HT(0);
        vsig   = smax(vsig, vsij);
        HT W   = KhS * kf.wqIn(dist * hq);
        HT tA0 = -(c11 * rx + c12 * ry + c13 * rz) * W;
        HT tA1 = -(c12 * rx + c22 * ry + c23 * rz) * W;
        HT tA2 = -(c13 * rx + c23 * ry + c33 * rz) * W;
        HT f   = pj.vol * (divvi - pj.divv);
        gx += f * tA0;
        gy += f * tA1;
        gz += f * tA2;
    });
    HT graddivv = sqrt(gx * gx + gy * gy + gz * gz);
    HT alphaloc = 0;
    if (divvi < HT(0))
    {
        HT a     = hi * hi * graddivv;
        alphaloc = alphamax * a / (a + hi * fabs(divvi) + HT(0.05) * ci);
    }
    if (alphaloc >= alpha_i) { alpha_i = alphaloc; }
    else
    {
        HT decay    = hi / (decayConstant * vsig);
        HT alphadot = (alphaloc >= alphamin) ? (alphaloc - alpha_i) / decay : (alphamin - alpha_i) / decay;
        alpha_i += alphadot * HT(dt);
    }
    return alpha_i;
}

/*! @brief AV-switch source record with the volume-weighted divergence vd = vol divv: 32 B on the fixed-point frame,
 *         i.e. two dwordx4 gathers per neighbor and no separate divv gather.
 *
 * The AV loop's gradient sum  g_i = sum_j vol_j (divv_i - divv_j) tA_ij,  tA_ij = -C_i r_ij K h_i^-3 w_ij,
 * is linear in the j terms, so  g_i = -K h_i^-3 C_i (divv_i S_i - T_i)  with  S_i = sum_j vol_j w_ij r_ij  (the IAD
 * loop accumulates it next to tau: same neighbors, same w_ij) and  T_i = sum_j vd_j w_ij r_ij. vol_j and divv_j then
 * only enter as their product. Mathematically identical to avSwitchesJLoop; rounding differs at the fp32 level.
 */
struct alignas(16) SrcAvV
{
    uint32_t x, y, z;
    HT vd;
    HT vx, vy, vz;
    HT c;
};
static_assert(!kHydroF32 || sizeof(SrcAvV) == 32, "SrcAvV is two 16-byte chunks");

#if defined(__HIPCC__)
template<>
__device__ __forceinline__ SrcAvV coopUnpack<SrcAvV>(const float4* o)
{
    SrcAvV r;
    r.x  = __float_as_uint(o[0].x);
    r.y  = __float_as_uint(o[0].y);
    r.z  = __float_as_uint(o[0].z);
    r.vd = o[0].w;
    r.vx = o[1].x;
    r.vy = o[1].y;
    r.vz = o[1].z;
    r.c  = o[1].w;
    return r;
}
#endif

template<class G, class Idx, class Ld, class KF>
SPHX_HD HT avSwitchesVJLoop(unsigned i, double K, const G& box, const Idx* nbr, int stride, unsigned nc, HT hi,
                            const HT ci6[6], HT divvi, const HT Si[3], const Ld& ld, const KF& kf, double dt,
                            HT alphamin, HT alphamax, HT decayConstant, HT alpha_i)
{
    const auto pi = ld(i);
    HT ci    = pi.c;
    HT vsig  = HT(1.e-40) * ci;
    HT hInv  = HT(1) / hi, hInv3 = hInv * hInv * hInv, hq = HT(0.25) * hInv;
    HT T[3]  = {0, 0, 0};
    const auto bx = vgprFrame(box);
    forEachNeighbor<SPHX_BATCH_IAD>(nbr, stride, nc, ld, [&](unsigned j, const auto& pj) {
        HT rx, ry, rz;
        pairSep(bx, pi, pj, hi, rx, ry, rz);
        HT r2      = rx * rx + ry * ry + rz * rz;
        HT invDist = rsqrtH(r2);
        HT dist    = r2 * invDist;
        HT vxij = pi.vx - pj.vx, vyij = pi.vy - pj.vy, vzij = pi.vz - pj.vz;
        HT rv   = rx * vxij + ry * vyij + rz * vzij;
        // branch-free: a branch here lets the compiler sink the load of pj.c into it, behind a full vmcnt(0) that
        // serializes the batched gathers (AV 36 % slower than IAD before, profiles/r2_perf_log.md)
        HT vst  = ci + pj.c - HT(3) * rv * invDist;
        HT vsij = rv < HT(0) ? vst : HT(0);
        vsig  = smax(vsig, vsij);
        HT wd = kf.wqIn(dist * hq) * pj.vd;
        T[0] += wd * rx;
        T[1] += wd * ry;
        T[2] += wd * rz;
    });
    reduceAcross(ld, T[0], T[1], T[2]);
    reduceAcrossMax(ld, vsig);
    {
        const HT invS = HT(1) / kf.wqScale(); // (KernelFn::wq)
        T[0] *= invS;
        T[1] *= invS;
        T[2] *= invS;
    }
    const HT D[3] = {divvi * Si[0] - T[0], divvi * Si[1] - T[1], divvi * Si[2] - T[2]};
    const HT s    = -HT(K) * hInv3;
    HT gx = s * (ci6[0] * D[0] + ci6[1] * D[1] + ci6[2] * D[2]);
    HT gy = s * (ci6[1] * D[0] + ci6[3] * D[1] + ci6[4] * D[2]);
    HT gz = s * (ci6[2] * D[0] + ci6[4] * D[1] + ci6[5] * D[2]);
    HT graddivv = sqrt(gx * gx + gy * gy + gz * gz);
    HT alphaloc = 0;
    if (divvi < HT(0))
    {
        HT a     = hi * hi * graddivv;
        alphaloc = alphamax * a / (a + hi * fabs(divvi) + HT(0.05) * ci);
    }
    if (alphaloc >= alpha_i) { alpha_i = alphaloc; }
    else
    {
        HT decay    = hi / (decayConstant * vsig);
        HT alphadot = (alphaloc >= alphamin) ? (alphaloc - alpha_i) / decay : (alphamin - alpha_i) / decay;
        alpha_i += alphadot * HT(dt);
    }
    return alpha_i;
}

//! @brief additive AV-cleaning correction to r.v (reference momentum_energy_kern.hpp avRvCorrection)
SPHX_HD HT avRvCorrection(HT rx, HT ry, HT rz, HT eta_ab, HT eta_crit, const HT gi[6], const HT gj[6])
{
    auto quad = [rx, ry, rz](const HT g[6])
    {
        HT s0 = g[0] * rx + g[1] * ry + g[2] * rz;
        HT s1 = g[3] * ry + g[4] * rz;
        HT s2 = g[5] * rz;
        return rx * s0 + ry * s1 + rz * s2;
    };
    HT d1 = quad(gi);
    HT d2 = quad(gj);
    HT d3 = HT(1);
    if (eta_ab < eta_crit)
    {
        HT e = HT(5) * (eta_ab - eta_crit);
        d3   = exp(-e * e);
    }
    HT A   = (d2 != HT(0)) ? d1 / d2 : HT(0);
    HT Ap1 = HT(1) + A;
    HT phi = HT(0.5) * d3 * smax(HT(0), smin(HT(1), HT(4) * A / (Ap1 * Ap1)));
    return -phi * (d1 + d2);
}

//! @brief VE momentum and energy equations (reference hydro_ve/momentum_energy_kern.hpp)
template<bool avClean, class G, class Idx, class Ld, class LdG, class KF>
SPHX_HD void momentumEnergyJLoop(unsigned i, const SphConsts& sc, const G& box, const Idx* nbr, int stride,
                                 unsigned nc, const Ld& ld, const LdG& ldg, const KF& kf, HT& axOut, HT& ayOut,
                                 HT& azOut, double& duOut, HT& maxvsignalOut)
{
    const auto pi = ld(i);
    HT hInv = pi.ih, hi = HT(1) / hInv, ci = pi.c, alphai = pi.alpha, xmi = pi.xm;
    HT rhoi = pi.rho, prhoi = pi.prho, invRhoi = HT(1) / rhoi, log2xmi = log2(xmi);
    HT hInv3 = hInv * hInv * hInv;
    HT gVi[6] = {0, 0, 0, 0, 0, 0};
    if (avClean)
    {
        SrcGradV g = ldg(i);
        for (int k = 0; k < 6; ++k)
            gVi[k] = g.dV[k];
    }
    HT etaCrit = cbrt(HT(32) * HT(M_PI) / HT(3) / HT(nc + 1));

    // Sums with the kernel weights folded into per-pair coefficients (same terms as the reference's
    // tA_i = -C_i r W_i, tA_j = -C_j r W_j form, regrouped):
    //   a_i = -K sum_j (m_j prho_i a_mom W_i + av/2 W_i) (C_i r) + (m_j prho_j b_mom W_j + bv/2 W_j) (C_j r)
    //   du_i = K (prho_i sum -m_j a_mom W_i v.(C_i r) + 1/2 max(0, -1/2 sum av W_i v.(C_i r) + bv W_j v.(C_j r)))
    // so the six tA components are never formed (profiles/r3_perf_log.md: 144 -> ~100 VALU per pair)
    HT maxvs = 0, mx = 0, my = 0, mz = 0, e1 = 0, e2 = 0;
    const HT Atmin = inVgpr(HT(sc.Atmin)), Atmax = inVgpr(HT(sc.Atmax)), ramp = inVgpr(HT(sc.ramp));
    const HT xmi2 = xmi * xmi;
    const auto bx = vgprFrame(box);

    forEachNeighbor<SPHX_BATCH_MOM>(nbr, stride, nc, ld, [&](unsigned j, const auto& pj) {
        HT rx, ry, rz;
        pairSep(bx, pi, pj, hi, rx, ry, rz);
        HT r2      = rx * rx + ry * ry + rz * rz;
        HT invDist = rsqrtH(r2);
        HT dist    = r2 * invDist;
        HT vxij = pi.vx - pj.vx, vyij = pi.vy - pj.vy, vzij = pi.vz - pj.vz;
        HT hjInv = pj.ih;
        // quarter arguments and S-scaled kernel values (KernelFn::wq; the sums are rescaled once after the loop)
        HT dq = HT(0.25) * dist;
        HT u1 = dq * hInv, u2 = dq * hjInv;
        HT Wi = hInv3 * kf.wqIn(u1); // (u1 from the target's h: inside the support, KernelFn::wqIn)
        HT Wj = hjInv * hjInv * hjInv * kf.wq(u2);

        // u = C r for the target and the neighbor
        HT uix = pi.c11 * rx + pi.c12 * ry + pi.c13 * rz;
        HT uiy = pi.c12 * rx + pi.c22 * ry + pi.c23 * rz;
        HT uiz = pi.c13 * rx + pi.c23 * ry + pi.c33 * rz;
        HT ujx = pj.c11 * rx + pj.c12 * ry + pj.c13 * rz;
        HT ujy = pj.c12 * rx + pj.c22 * ry + pj.c23 * rz;
        HT ujz = pj.c13 * rx + pj.c23 * ry + pj.c33 * rz;

        HT mj = pj.m, cj = pj.c, xmj = pj.xm, rhoj = pj.rho;

        HT rv = rx * vxij + ry * vyij + rz * vzij;
        if (avClean)
        {
            SrcGradV gj = ldg(j);
            rv += avRvCorrection(rx, ry, rz, HT(4) * smin(u1, u2), etaCrit, gVi, gj.dV);
        }
        HT wij  = rv * invDist;
        HT visc = artificialViscosity(alphai, pj.alpha, ci, cj, wij);
        HT vs   = HT(0.5) * (ci + cj) - HT(2) * wij;
        maxvs   = vs > maxvs ? vs : maxvs;

        // generalized volume elements with the Atwood ramp; Atwood = |rho_i - rho_j| / (rho_i + rho_j)
        HT a_mom, b_mom;
        HT dRho = fabs(rhoi - rhoj), sRho = rhoi + rhoj;
        if (dRho < Atmin * sRho)
        {
            a_mom = xmi2;
            b_mom = xmj * xmj;
        }
        else if (dRho > Atmax * sRho)
        {
            a_mom = xmi * xmj;
            b_mom = a_mom;
        }
        else
        {
            // xmi^(2-s) xmj^s = xmi^2 (xmj/xmi)^s and xmj^(2-s) xmi^s = xmj^2 (xmj/xmi)^-s
            HT sigma = ramp * (dRho * rcpF(sRho) - Atmin);
            HT e     = sigma * (log2(xmj) - log2xmi);
            a_mom    = xmi2 * exp2(e);
            b_mom    = xmj * xmj * exp2(-e);
        }

        HT av  = mj * invRhoi * visc;
        HT bv  = pj.mrho * visc;
        HT vui = vxij * uix + vyij * uiy + vzij * uiz;
        HT vuj = vxij * ujx + vyij * ujy + vzij * ujz;
        HT mja = mj * a_mom;
        HT Ai  = (mja * prhoi + HT(0.5) * av) * Wi;
        HT Aj  = (mj * pj.prho * b_mom + HT(0.5) * bv) * Wj;
        mx += Ai * uix + Aj * ujx;
        my += Ai * uiy + Aj * ujy;
        mz += Ai * uiz + Aj * ujz;
        e1 += mja * Wi * vui;
        e2 += av * Wi * vui + bv * Wj * vuj;
    });
    reduceAcross(ld, mx, my, mz, e1, e2);
    reduceAcrossMax(ld, maxvs);
    HT aviscE     = smax(HT(0), HT(-0.5) * e2);
    HT Kf         = HT(sc.K) / kf.wqScale(); // (every summed term carries one S-scaled kernel value)
    duOut         = double(Kf * (-prhoi * e1 + HT(0.5) * aviscE));
    axOut         = Kf * mx;
    ayOut         = Kf * my;
    azOut         = Kf * mz;
    maxvsignalOut = maxvs;
}

//! @brief standard SPH momentum and energy, constant alpha=1 AV (reference hydro_std/momentum_energy_kern.hpp)
template<class Idx, class Ld>
SPHX_HD void momentumEnergyStdJLoop(unsigned i, double K, const Box& box, const Idx* nbr, int stride, unsigned nc,
                                    const Ld& ld, const KernelFn& kf, HT& axOut, HT& ayOut, HT& azOut, double& duOut,
                                    HT& maxvsignalOut)
{
    SrcStd pi = ld(i);
    HT hInv = pi.ih, hi = HT(1) / hInv, roi = pi.rho, pri = pi.p, ci = pi.c;
    HT mi_roi = pi.m / roi;
    HT hInv3 = hInv * hInv * hInv;
    HT maxvs = 0, mx = 0, my = 0, mz = 0, energy = 0;
    forEachNeighbor<SPHX_BATCH_MOM>(nbr, stride, nc, ld, [&](unsigned j, const SrcStd& pj) {
        HT rx, ry, rz;
        pairDelta(pi.x, pi.y, pi.z, pj.x, pj.y, pj.z, hi, box, rx, ry, rz);
        HT r2      = rx * rx + ry * ry + rz * rz;
        HT invDist = rsqrtH(r2);
        HT dist    = r2 * invDist;
        HT vxij = pi.vx - pj.vx, vyij = pi.vy - pj.vy, vzij = pi.vz - pj.vz;
        HT hjInv = pj.ih;
        HT dq = HT(0.25) * dist;
        HT u1 = dq * hInv, u2 = dq * hjInv;
        HT rv = rx * vxij + ry * vyij + rz * vzij;
        HT Wi = hInv3 * kf.wqIn(u1); // (S-scaled: KernelFn::wq; inside the support: wqIn)
        HT Wj = hjInv * hjInv * hjInv * kf.wq(u2);
        HT tAi0 = pi.c11 * rx + pi.c12 * ry + pi.c13 * rz;
        HT tAi1 = pi.c12 * rx + pi.c22 * ry + pi.c23 * rz;
        HT tAi2 = pi.c13 * rx + pi.c23 * ry + pi.c33 * rz;
        HT tAj0 = pj.c11 * rx + pj.c12 * ry + pj.c13 * rz;
        HT tAj1 = pj.c12 * rx + pj.c22 * ry + pj.c23 * rz;
        HT tAj2 = pj.c13 * rx + pj.c23 * ry + pj.c33 * rz;
        HT roj = pj.rho, cj = pj.c;
        HT wij  = rv * invDist;
        HT visc = HT(0.5) * artificialViscosity(HT(1), HT(1), ci, cj, wij);
        HT vs   = ci + cj - HT(3) * wij;
        maxvs   = vs > maxvs ? vs : maxvs;
        HT mj      = pj.m;
        HT mjrojWj = mj / roj * Wj;
        HT mjproi  = mj * pri / (roi * roi);
        {
            HT a = Wi * (mjproi + visc * mi_roi);
            HT b = mjrojWj * (pj.p / roj + visc);
            mx += a * tAi0 + b * tAj0;
            my += a * tAi1 + b * tAj1;
            mz += a * tAi2 + b * tAj2;
        }
        {
            HT a = Wi * (HT(2) * mjproi + visc * mi_roi);
            HT b = visc * mjrojWj;
            energy += vxij * (a * tAi0 + b * tAj0) + vyij * (a * tAi1 + b * tAj1) + vzij * (a * tAi2 + b * tAj2);
        }
    });
    HT Kf         = HT(K) / kf.wqScale();
    duOut         = double(-Kf * HT(0.5) * energy);
    axOut         = Kf * mx;
    ayOut         = Kf * my;
    azOut         = Kf * mz;
    maxvsignalOut = maxvs;
}

// ---------------------------------------------------------------------------------------------------------
// record loaders
// ---------------------------------------------------------------------------------------------------------

//! @brief loader from a packed array of records (gfx950 path)
template<class R>
struct RecLoader
{
    const R* r;
    SPHX_HD R operator()(unsigned j) const { return r[j]; }
};

//! @brief SoA loaders (OpenMP path): assemble the record from separate fields
struct SoaPos
{
    const CT *x, *y, *z;
    const HT *m, *xm;
    SPHX_HD SrcPos operator()(unsigned j) const { return {x[j], y[j], z[j], m[j], xm ? xm[j] : HT(0)}; }
};

struct SoaIad
{
    const CT *x, *y, *z;
    const HT *numer, *denom, *vx, *vy, *vz, *xm, *c, *divv;
    SPHX_HD SrcIad operator()(unsigned j) const
    {
        SrcIad r;
        r.x    = x[j];
        r.y    = y[j];
        r.z    = z[j];
        r.vol  = numer ? numer[j] / denom[j] : HT(0);
        r.vx   = vx ? vx[j] : HT(0);
        r.vy   = vy ? vy[j] : HT(0);
        r.vz   = vz ? vz[j] : HT(0);
        if (c) r.c = c[j];
        else r.xm = xm ? xm[j] : HT(0);
        r.divv = divv ? divv[j] : HT(0);
        return r;
    }
};

struct SoaMom
{
    const CT *x, *y, *z;
    const HT *vx, *vy, *vz, *h, *c11, *c12, *c13, *c22, *c23, *c33, *m, *c, *xm, *kx, *prho, *alpha;
    SPHX_HD SrcMom operator()(unsigned j) const
    {
        SrcMom r;
        r.x = x[j];
        r.y = y[j];
        r.z = z[j];
        r.vx = vx[j];
        r.vy = vy[j];
        r.vz = vz[j];
        r.ih = HT(1) / h[j];
        r.c11 = c11[j];
        r.c12 = c12[j];
        r.c13 = c13[j];
        r.c22 = c22[j];
        r.c23 = c23[j];
        r.c33 = c33[j];
        r.m = m[j];
        r.c = c[j];
        r.xm = xm[j];
        r.rho = kx[j] * m[j] / xm[j];
        r.prho = prho[j];
        r.alpha = alpha[j];
        r.mrho = m[j] / r.rho;
        return r;
    }
};

struct SoaGradV
{
    const HT* dV[6];
    SPHX_HD SrcGradV operator()(unsigned j) const
    {
        SrcGradV g;
        for (int k = 0; k < 6; ++k)
            g.dV[k] = dV[k] ? dV[k][j] : HT(0);
        g.pad[0] = g.pad[1] = 0;
        return g;
    }
};

struct SoaStd
{
    const CT *x, *y, *z;
    const HT *vx, *vy, *vz, *h, *c11, *c12, *c13, *c22, *c23, *c33, *m, *rho, *p, *c;
    SPHX_HD SrcStd operator()(unsigned j) const
    {
        SrcStd r;
        r.x = x[j];
        r.y = y[j];
        r.z = z[j];
        r.vx = vx[j];
        r.vy = vy[j];
        r.vz = vz[j];
        r.ih = HT(1) / h[j];
        r.c11 = c11[j];
        r.c12 = c12[j];
        r.c13 = c13[j];
        r.c22 = c22[j];
        r.c23 = c23[j];
        r.c33 = c33[j];
        r.m = m[j];
        r.rho = rho[j];
        r.p = p[j];
        r.c = c[j];
        return r;
    }
};

} // namespace sphx
