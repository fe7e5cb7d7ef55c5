// Declarations of the OpenMP reference path (module _sphx_cpu).
#pragma once

#include <cstdint>
#include <vector>

#include "sphx/box.hpp"
#include "sphx/sph_math.hpp"

namespace sphx::cpu
{

//! @brief SoA field pointers of the VE momentum loop (assembled into SrcMom records by SoaMom)
struct VeMomentumPtrs
{
    const CT *x, *y, *z;
    const HT *vx, *vy, *vz, *h, *m, *prho, *c;
    const HT* cij[6];
    const HT *kx, *xm, *alpha;
    const HT* dV[6];
    const HT* wh;
};

struct StdMomentumPtrs
{
    const CT *x, *y, *z;
    const HT *vx, *vy, *vz, *h, *m, *rho, *p, *c;
    const HT* cij[6];
    const HT* wh;
};

struct LinkedOctree
{
    int64_t numNodes{0};
    int64_t numLeaves{0};
    std::vector<KeyT> prefixes;        // placeholder codes, level-major, key-minor
    std::vector<int32_t> childOffsets; // 0 for leaves
    std::vector<int32_t> parents;      // per sibling group
    std::vector<int32_t> nodeToLeaf;   // -1 for internal nodes
    std::vector<int32_t> leafToNode;
    std::vector<int64_t> levelRange;   // first node index of each level, size kMaxLevel+2
};

void computeKeys(int64_t n, const double* x, const double* y, const double* z, const Box& box, int kind, KeyT* keys);
void sortKeys(int64_t n, KeyT* keys, int32_t* perm);
void gatherBytes(int64_t n, const int32_t* perm, const char* src, char* dst, int elemSize);
void nodeCounts(const KeyT* tree, int64_t L, const KeyT* keys, int64_t n, uint32_t* counts);
bool rebalance(std::vector<KeyT>& tree, const uint32_t* counts, uint32_t bucket);
std::vector<KeyT> buildTree(std::vector<KeyT> tree, const KeyT* keys, int64_t n, uint32_t bucket,
                            std::vector<uint32_t>& counts, int maxIter);
LinkedOctree linkOctree(const KeyT* tree, int64_t L);
void nodeRanges(const LinkedOctree& o, const KeyT* keys, int64_t n, int64_t offset, int32_t* nodeStart,
                int32_t* nodeEnd);
void tightBoxes(const LinkedOctree& o, const int32_t* nodeStart, const int32_t* nodeEnd, const double* x,
                const double* y, const double* z, double* center, double* half);

void boxesWithRadius(int64_t N, const int32_t* childOffsets, const int32_t* nodeToLeaf, const int64_t* levelRange,
                     const int32_t* nodeStart, const int32_t* nodeEnd, const double* x, const double* y,
                     const double* z, const float* h, double factor, double* center, double* half);

//! @brief flat view of a linked octree with tight node boxes, as used by the traversals
struct TreeView
{
    int64_t numNodes;
    const int32_t* childOffsets;
    const int32_t* nodeToLeaf;
    const int32_t* nodeStart;
    const int32_t* nodeEnd;
    const double* center;
    const double* half;
};

void markInBoxes(int64_t numBoxes, const double* bc, const double* bh, const TreeView& t, const double* x,
                 const double* y, const double* z, const Box& box, uint8_t* flags);

} // namespace sphx::cpu

#include "sphx/gravity.hpp"

namespace sphx::cpu
{

void gravityUpsweep(int64_t N, const int32_t* child, const int32_t* n2l, const int64_t* levelRange,
                    const KeyT* prefixes, const int32_t* ns, const int32_t* ne, const double* x, const double* y,
                    const double* z, const float* m, const Box& box, int kind, double invTheta, double* centers,
                    Quadrupole* mp, bool leavesGiven = false);
double computeGravity(int64_t first, int64_t last, const int32_t* child, const int32_t* n2l, const int32_t* ns,
                      const int32_t* ne, const double* centers, const Quadrupole* mp, const double* x,
                      const double* y, const double* z, const float* h, const float* m, double G, float* ax,
                      float* ay, float* az, double* ugrav, int64_t* stats = nullptr);
double directSum(int64_t first, int64_t last, int64_t n, const double* x, const double* y, const double* z,
                 const float* h, const float* m, double G, float* ax, float* ay, float* az, double* ugrav);
void markLet(int64_t nb, const double* bc, const double* bh, const int32_t* child, const int32_t* n2l,
             const double* tcenter, const double* thalf, const double* gcenters, const Box& box, uint8_t* failed);
double m2pFlat(int64_t first, int64_t last, const double* x, const double* y, const double* z, const float* m,
               int64_t M, const double* mc, const Quadrupole* mp, double G, float* ax, float* ay, float* az,
               double* ugrav);

} // namespace sphx::cpu

namespace sphx::cpu
{

//! turbulence stirring: a_i += norm * sum_m amp_m (Re_m cos(k_m.x_i) - Im_m sin(k_m.x_i)), modes as (kx,ky,kz)
void computeStirring(int64_t first, int64_t last, const double* x, const double* y, const double* z, float* ax,
                     float* ay, float* az, int64_t numModes, const double* modes, const double* phaseRe,
                     const double* phaseIm, const double* amplitudes, double norm);

} // namespace sphx::cpu
