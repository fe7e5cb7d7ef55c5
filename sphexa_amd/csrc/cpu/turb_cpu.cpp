// Turbulence stirring force, OpenMP reference path (reference sph/include/sph/hydro_turb/stirring.hpp:40-100).
#include <cmath>

#include "cpu_api.hpp"

namespace sphx::cpu
{

void computeStirring(int64_t first, int64_t last, const double* x, const double* y, const double* z, float* ax,
                     float* ay, float* az, int64_t numModes, const double* modes, const double* phaseRe,
                     const double* phaseIm, const double* amplitudes, double norm)
{
#pragma omp parallel for schedule(static)
    for (int64_t i = first; i < last; ++i)
    {
        double a[3] = {0, 0, 0};
        for (int64_t m = 0; m < numModes; ++m)
        {
            // cos/sin of k.x: the real and imaginary part of exp(i k.x)
            double ph = modes[3 * m] * x[i] + modes[3 * m + 1] * y[i] + modes[3 * m + 2] * z[i];
            double re = std::cos(ph), im = std::sin(ph);
            for (int d = 0; d < 3; ++d)
                a[d] += amplitudes[m] * (phaseRe[3 * m + d] * re - phaseIm[3 * m + d] * im);
        }
        ax[i] += float(norm * a[0]);
        ay[i] += float(norm * a[1]);
        az[i] += float(norm * a[2]);
    }
}

} // namespace sphx::cpu
