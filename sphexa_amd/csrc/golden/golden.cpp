/*! Golden-value harness: the SPH j-loops of sph_math.hpp instantiated in double precision (-DSPHX_HYDRO_TYPE=double),
 *  as the reference pins its kernels with T = double in sph/test/ve.cpp:112-232 and sph/test/std.cpp:98-123.
 *
 *  Every entry point evaluates particle 0 of the given arrays against the neighbor list 1..n-1 (the reference
 *  fixture layout) through the same SoA loaders the OpenMP path uses, and returns the loop outputs. The production
 *  fp32 paths (OpenMP and gfx950) are pinned to the same fixture through the regular operators (tests/test_golden.py).
 */
#include <numeric>
#include <vector>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "sphx/sph_math.hpp"

namespace py = pybind11;
using namespace sphx;

static_assert(sizeof(HT) == 8, "the golden harness is built with -DSPHX_HYDRO_TYPE=double");

using Arr = py::array_t<double, py::array::c_style | py::array::forcecast>;

namespace
{

const double* ptr(const Arr& a) { return a.data(); }

struct Fixture
{
    std::vector<int32_t> nbr;
    unsigned nc;
    explicit Fixture(size_t n)
        : nbr(n - 1)
        , nc(unsigned(n - 1))
    {
        std::iota(nbr.begin(), nbr.end(), 1);
    }
};

Box openBox(double lo, double hi)
{
    Box b;
    for (int d = 0; d < 3; ++d)
    {
        b.lo[d] = lo;
        b.hi[d] = hi;
        b.bc[d] = 0;
    }
    return b;
}

KernelFn kernel(const Arr& wh, const Arr& whd, double sincIndex) { return KernelFn{ptr(wh), ptr(whd), sincIndex, 0}; }

} // namespace

PYBIND11_MODULE(_sphx_golden, m)
{
    m.doc() = "fp64 instantiation of the SPH j-loops for golden-value tests";

    m.def("xmass", [](double K, double lo, double hi, Arr x, Arr y, Arr z, Arr h, Arr mass, Arr wh, Arr whd,
                      double n) {
        Fixture f(x.size());
        SoaPos ld{ptr(x), ptr(y), ptr(z), ptr(mass), nullptr};
        return xmassJLoop(0, K, openBox(lo, hi), f.nbr.data(), 1, f.nc, ptr(h)[0], ld, kernel(wh, whd, n));
    });

    m.def("ve_def_gradh", [](double K, double lo, double hi, Arr x, Arr y, Arr z, Arr h, Arr mass, Arr xm, Arr wh,
                             Arr whd, double n) {
        Fixture f(x.size());
        SoaPos ld{ptr(x), ptr(y), ptr(z), ptr(mass), ptr(xm)};
        HT kx, gradh;
        veDefGradhJLoop(0, K, openBox(lo, hi), f.nbr.data(), 1, f.nc, ptr(h)[0], ld, kernel(wh, whd, n), kx, gradh);
        return py::make_tuple(kx, gradh);
    });

    m.def("iad", [](double K, double lo, double hi, Arr x, Arr y, Arr z, Arr h, Arr numer, Arr denom, Arr wh, Arr whd,
                    double n) {
        Fixture f(x.size());
        SoaIad ld{ptr(x), ptr(y), ptr(z), ptr(numer), ptr(denom), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
        HT c[6];
        iadJLoop(0, K, openBox(lo, hi), f.nbr.data(), 1, f.nc, ptr(h)[0], ld, kernel(wh, whd, n), c);
        return std::vector<double>(c, c + 6);
    });

    m.def("divv_curlv", [](double K, double lo, double hi, Arr x, Arr y, Arr z, Arr vx, Arr vy, Arr vz, Arr h,
                           std::vector<double> ci, Arr kx, Arr xm, Arr wh, Arr whd, double n) {
        Fixture f(x.size());
        SoaIad ld{ptr(x), ptr(y), ptr(z), nullptr, nullptr, ptr(vx), ptr(vy), ptr(vz), ptr(xm), nullptr, nullptr};
        HT divv, curlv, dV[6];
        divvCurlvJLoop(0, K, openBox(lo, hi), f.nbr.data(), 1, f.nc, ptr(h)[0], ptr(kx)[0], ci.data(), ld,
                       kernel(wh, whd, n), divv, curlv, dV);
        return py::make_tuple(divv, curlv, std::vector<double>(dV, dV + 6));
    });

    m.def("av_switches", [](double K, double lo, double hi, Arr x, Arr y, Arr z, Arr vx, Arr vy, Arr vz, Arr h, Arr c,
                            std::vector<double> ci, Arr kx, Arr xm, Arr divv, Arr wh, Arr whd, double n, double dt,
                            double alphamin, double alphamax, double decay, double alpha0) {
        Fixture f(x.size());
        SoaIad ld{ptr(x), ptr(y), ptr(z), ptr(xm), ptr(kx), ptr(vx), ptr(vy), ptr(vz), nullptr, ptr(c), ptr(divv)};
        return avSwitchesJLoop(0, K, openBox(lo, hi), f.nbr.data(), 1, f.nc, ptr(h)[0], ci.data(), ld,
                               kernel(wh, whd, n), dt, alphamin, alphamax, decay, alpha0);
    });

    m.def("momentum_energy", [](bool avClean, double K, double Atmin, double Atmax, double lo, double hi, Arr x, Arr y,
                                Arr z, Arr vx, Arr vy, Arr vz, Arr h, Arr c11, Arr c12, Arr c13, Arr c22, Arr c23,
                                Arr c33, Arr mass, Arr c, Arr xm, Arr kx, Arr prho, Arr alpha, std::vector<Arr> dV,
                                Arr wh, Arr whd, double n) {
        Fixture f(x.size());
        SphConsts sc{};
        sc.K     = K;
        sc.Atmin = float(Atmin);
        sc.Atmax = float(Atmax);
        sc.ramp  = float(1.0 / (Atmax - Atmin));
        SoaMom ld{ptr(x),   ptr(y),   ptr(z),   ptr(vx),  ptr(vy),   ptr(vz), ptr(h),  ptr(c11), ptr(c12), ptr(c13),
                  ptr(c22), ptr(c23), ptr(c33), ptr(mass), ptr(c),   ptr(xm), ptr(kx), ptr(prho), ptr(alpha)};
        SoaGradV ldg{{ptr(dV[0]), ptr(dV[1]), ptr(dV[2]), ptr(dV[3]), ptr(dV[4]), ptr(dV[5])}};
        HT ax, ay, az, maxvs;
        double du;
        Box box = openBox(lo, hi);
        KernelFn kf = kernel(wh, whd, n);
        if (avClean)
            momentumEnergyJLoop<true>(0, sc, box, f.nbr.data(), 1, f.nc, ld, ldg, kf, ax, ay, az, du, maxvs);
        else
            momentumEnergyJLoop<false>(0, sc, box, f.nbr.data(), 1, f.nc, ld, ldg, kf, ax, ay, az, du, maxvs);
        return py::make_tuple(ax, ay, az, du, maxvs);
    });

    m.def("momentum_energy_std", [](double K, double lo, double hi, Arr x, Arr y, Arr z, Arr vx, Arr vy, Arr vz, Arr h,
                                    Arr c11, Arr c12, Arr c13, Arr c22, Arr c23, Arr c33, Arr mass, Arr rho, Arr p,
                                    Arr c, Arr wh, Arr whd, double n) {
        Fixture f(x.size());
        SoaStd ld{ptr(x),   ptr(y),   ptr(z),   ptr(vx),   ptr(vy),  ptr(vz), ptr(h), ptr(c11), ptr(c12),
                  ptr(c13), ptr(c22), ptr(c23), ptr(c33), ptr(mass), ptr(rho), ptr(p), ptr(c)};
        HT ax, ay, az, maxvs;
        double du;
        momentumEnergyStdJLoop(0, K, openBox(lo, hi), f.nbr.data(), 1, f.nc, ld, kernel(wh, whd, n), ax, ay, az, du,
                               maxvs);
        return py::make_tuple(ax, ay, az, du, maxvs);
    });
}
