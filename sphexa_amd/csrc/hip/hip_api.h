// Host-side API of the gfx950 module (_sphx_hip): argument structs and launcher declarations.
#pragma once

#include <cstdint>
#include <vector>

#include <hip/hip_runtime.h>

#include "sphx/box.hpp"
#include "sphx/cooling.hpp"
#include "sphx/sph_math.hpp"

namespace sphx::hip
{

struct NsTree
{
    const int32_t* child;
    const int32_t* n2l;
    const int32_t* ns;
    const int32_t* ne;
    const double* center;
    const double* half;
};

struct NbrArgs
{
    int64_t first, last;
    const int32_t* nidx;
    const int32_t* nc;
    unsigned ngmax;
    unsigned ntot = 0; // number of source records (set by the launchers; clamps the cooperative gathers)
};

struct PosArgs
{
    double *x, *y, *z;
    float *vx, *vy, *vz, *xm1, *ym1, *zm1;
    const float *ax, *ay, *az, *h;
    double *temp, *u;
    const double* du;
    float* dum1;
};

// sfc_sort.hip
void computeKeys(int64_t n, const double* x, const double* y, const double* z, const Box& box, int kind, KeyT* keys,
                 hipStream_t s);
//! the bit-serial reference form of computeKeys (sfc.hpp hilbertKey; computeKeys walks a table: identical keys)
void computeKeysSerial(int64_t n, const double* x, const double* y, const double* z, const Box& box, int kind,
                       KeyT* keys, hipStream_t s);
//! states of the Hilbert key table (built on first use; a consistency failure throws)
int hilbertTableStates();
void computeKeysDevBox(int64_t n, const double* x, const double* y, const double* z, const Box& box, const double* ext,
                       int kind, KeyT* keys, hipStream_t s, int layout = 0);
size_t sortPairsTempBytes(int64_t n);
void sortPairs(int64_t n, const KeyT* keysIn, KeyT* keysOut, const int32_t* valsIn, int32_t* valsOut, void* tmp,
               size_t tmpBytes, int beginBit, int endBit, hipStream_t s);
void sortKeys(int64_t n, const KeyT* keysIn, KeyT* keysOut, int32_t* perm, void* tmp, size_t tmpBytes, hipStream_t s);
//! non-empty sorted runs a merge handles (mergeSortedRuns); more runs: sort
constexpr int kMergeRuns = 16;
//! stable merge of the sorted runs [runOffsets[b], runOffsets[b + 1]) of keys (host offsets): out = merged keys,
//! perm = source index of each output position
void mergeSortedRuns(int64_t n, const KeyT* keys, const int64_t* runOffsets, int numRuns, KeyT* out, int32_t* perm,
                     hipStream_t s);
void gather(int64_t n, const int32_t* perm, const void* src, void* dst, int elemSize, hipStream_t s);
void gatherMerged(int64_t n, const int32_t* pm, int64_t nLo, int64_t nStay, const int32_t* permStay,
                  const std::vector<uintptr_t>& own, const std::vector<uintptr_t>& recv,
                  const std::vector<uintptr_t>& dst, int elemSize, hipStream_t s);
// halo_discovery.hip: every destination rank in one launch per stage
void markHalosMulti(int nDest, int nbPer, const double* boxes, const uint8_t* enabled, const int32_t* child,
                    const int32_t* n2l, const int32_t* ns, const int32_t* ne, const double* center, const double* half,
                    const double* x, const double* y, const double* z, int64_t n, const Box& box, uint8_t* flags,
                    hipStream_t s);
void remoteTreeScatter(int64_t M, const int32_t* nodes, const double* rc, const float* rq, double* centers, float* mp,
                       int forceAccept, double value, hipStream_t s);
void markLetMulti(int nDest, int nbPer, const double* boxes, const uint8_t* enabled, const int32_t* child,
                  const int32_t* n2l, const double* tc, const double* th, const double* gc, int64_t N, const Box& box,
                  uint8_t* failed, hipStream_t s);
void letSelectMulti(int nDest, int64_t N, int64_t L, int64_t np, const uint8_t* enabled, const uint8_t* failed,
                    const uint8_t* outside, const int32_t* leafToNode, const int32_t* ns, const int32_t* ne,
                    int64_t offset, const void* mp, const int32_t* parents, uint8_t* pflags, uint8_t* send,
                    hipStream_t s);
void flagWords(int nRows, int64_t n, const uint8_t* flags, int64_t* wcnt, int64_t* count, int countStride,
               hipStream_t s);
void scatterFlagIndices(int nRows, int64_t n, const uint8_t* flags, const int64_t* wpos, int64_t* out, hipStream_t s,
                        int64_t offset = 0);
void splitMultipoleRows(int64_t n, const double* rows, double* centers, float* quads, int64_t* codes, hipStream_t s);
void rangeCounts(int64_t n, const uint64_t* keys, const uint64_t* bounds, int nRanks, int64_t* out, int outStride,
                 hipStream_t s);
void coarseCut(int64_t N, const int64_t* levelRange, int maxDepth, const int32_t* n2l, const double* center,
               const double* half, int maxBoxes, double* out, hipStream_t s);
void packMultipoleRows(int64_t n, const int64_t* idx, const double* gc, const void* mp, const uint64_t* prefixes,
                       double* rows, hipStream_t s);
void haloOwnerCheck(int64_t nLo, int64_t nHalo, int64_t end, const uint64_t* keys, const uint64_t* bounds, int nBounds,
                    const int64_t* recvStart, const int32_t* senders, int nSenders, int self, double* bad,
                    hipStream_t s);
void leavingIndices(int64_t nSend, const int32_t* perm, int64_t eSelf, int64_t nStay, int64_t* out, hipStream_t s);
void gatherMulti(int64_t n, const int32_t* perm, const std::vector<uintptr_t>& src, const std::vector<uintptr_t>& dst,
                 int elemSize, hipStream_t s);
//! halo message rows of several fields (8-byte fields first, rows padded to 8 bytes); idx == nullptr: rows 0..n-1
int rowBytes(const std::vector<int>& sizes);
void packRows(int64_t n, const int64_t* idx, const std::vector<uintptr_t>& src, const std::vector<int>& sizes,
              void* rows, hipStream_t s);
void unpackRows(int64_t n, const void* rows, const std::vector<uintptr_t>& dst, const std::vector<int>& sizes,
                int64_t dstOffset, hipStream_t s);
size_t scanTempBytes(int64_t n);
// hand-written sample sort and tile scans (sample_sort.hip)
size_t sampleSortTempBytes(int64_t n);
void sampleSortPairs(int64_t n, const uint64_t* keysIn, const uint32_t* valsIn, uint64_t* keysOut, uint32_t* valsOut,
                     void* tmp, size_t tmpBytes, hipStream_t s);
size_t exclusiveScanTempBytes(int64_t n);
void exclusiveScanI64Hip(const int64_t* in, int64_t* out, int64_t n, void* tmp, size_t tmpBytes, hipStream_t s);
void exclusiveScanI64(const int64_t* in, int64_t* out, int64_t n, void* tmp, size_t tmpBytes, hipStream_t s);

// reduce.hip: device reductions in two launches (block partials + one fold kernel; workspace: reduceWorkBytes() of
// partials, one per concurrently reducing stream)
size_t reduceWorkBytes();
void multiMinMax(int64_t n, const std::vector<uintptr_t>& ptrs, const std::vector<int>& isDouble, double* out,
                 void* work, hipStream_t s, int layout = 0);
void maxNorm2(int64_t first, int64_t last, const float* ax, const float* ay, const float* az, double* out, void* work,
              hipStream_t s);
void timestepReduce(int64_t first, int64_t last, const float* ax, const float* ay, const float* az,
                    const float* courantDev, double courantHost, const float* divvMax, double rhoHost, double Krho,
                    double etaAcc, double eps, double others, double prevDt, double* out, void* work, hipStream_t s);
//! *out = max of f over [first, last) (float32 device scalar; two launches)
void fieldMax(int64_t first, int64_t last, const float* f, float* out, void* work, hipStream_t s);
//! n 32-bit words at p set to value (hipMemsetD32Async: e.g. +inf for a min-reduced scalar), stream-ordered
void fill32(void* p, uint32_t value, int64_t n, hipStream_t s);
void add3(int64_t first, int64_t last, const float* bx, const float* by, const float* bz, float* ax, float* ay,
          float* az, hipStream_t s);
//! 0/1 byte flags -> bitmask (bit k of byte b = flag 8 b + k); *count (int64, may be null) += number of set flags
void packBits(int64_t n, const uint8_t* flags, uint8_t* bits, int64_t* count, hipStream_t s);
void unpackBits(int64_t n, const uint8_t* bits, uint8_t* flags, hipStream_t s);
//! bytes at p set to value (hipMemsetAsync), stream-ordered
void memsetAsync(void* p, int value, size_t bytes, hipStream_t s);

// octree.hip
void nodeCounts(const KeyT* tree, int64_t L, const KeyT* keys, int64_t n, int32_t* counts, hipStream_t s);
void nodeCounts64(const KeyT* tree, int64_t L, const KeyT* keys, int64_t n, int64_t* counts, hipStream_t s);
void rebalanceOps(const KeyT* tree, const int32_t* counts, int64_t L, uint32_t bucket, int64_t* ops, int* changed,
                  hipStream_t s);
void emitLeavesLaunch(const KeyT* tree, const int64_t* ops, int64_t L, KeyT* out, int64_t newL, hipStream_t s);
void internalCounts(const KeyT* tree, int64_t L, int64_t* icount, hipStream_t s);
void makeCodes(const KeyT* tree, int64_t L, const int64_t* ioff, int64_t Ni, KeyT* codes, int32_t* vals,
               hipStream_t s);
void linkNodes(const KeyT* codes, const int32_t* vals, int64_t N, int32_t* child, int32_t* parents,
               int32_t* leafToNode, int64_t* levelRange, hipStream_t s);
void nodeRanges(const KeyT* codes, int64_t N, const KeyT* keys, int64_t n, int64_t offset, int32_t* ns, int32_t* ne,
                hipStream_t s);
void leafBoxesFused(const int32_t* n2l, int64_t N, const int32_t* ns, const int32_t* ne, const double* x,
                    const double* y, const double* z, const int32_t* child, const int32_t* parents, double* center,
                    double* half, unsigned* cnt, hipStream_t s);
void leafBoxes(const int32_t* n2l, int64_t N, const int32_t* ns, const int32_t* ne, const double* x,
               const double* y, const double* z, const float* h, double factor, double* center, double* half,
               hipStream_t s);
void upsweepBoxes(int64_t a, int64_t b, const int32_t* n2l, const int32_t* child, double* center, double* half,
                  hipStream_t s);
void markInBoxes(int64_t nb, const double* bc, const double* bh, const int32_t* child, const int32_t* n2l,
                 const int32_t* ns, const int32_t* ne, const double* center, const double* half, const double* x,
                 const double* y, const double* z, const Box& box, uint8_t* flags, hipStream_t s);

// neighbors.hip
// stats: [0] h-iteration failures, [1] groups overflowing even the spill storage, [2] spilled groups, [3]/[4] rounds /
// touched leaves (opt-in), [6] groups over the chunk-table capacity | groups that recovered from it by halving h << 32,
// [8 + 32 k] overflow-row stripe counters
size_t neighborScratchBytes(int64_t n, unsigned ngmax);
//! overflow prediction of the neighbor search (neighbors.hip PredOut / predMarkKernel); all null: off
struct SplitPredict
{
    const uint64_t* keys = nullptr;              // SFC keys, index = particle index
    const unsigned long long* predIn = nullptr;  // [count, key pairs] recorded by the previous search
    unsigned long long* predOut = nullptr;       // this search's record (for the next one)
    int32_t* flags = nullptr;                    // per-group stamps (>= groups entries)
    int stamp = 0;
    int cap = 0;                                 // key pairs per record
    unsigned long long* listCount = nullptr;     // predicted groups: count + list (>= 3 cap entries)
    int32_t* list = nullptr;
    int mark = 1; // 0: predIn is known to be empty (the previous search split no group): record only
};
void findNeighbors(int64_t first, int64_t last, const double* x, const double* y, const double* z, float* h,
                   const NsTree& t, const Box& box, unsigned ng0, unsigned ngmax, int32_t* nidx, int home,
                   int ovStride, int32_t* nc, int iterateH, unsigned long long* stats, void* scratch,
                   int testFrontCap, const float* m, int64_t ntot, void* rec, hipStream_t s, const SplitPredict& sp = SplitPredict{});
//! threads per block of the production pair loops (256 or 512, hydro.hip withPairBlock)
void setPairBlock(int block);
//! pair-loop instances: compile-time sinc^6 kernel function, 32-bit buffer gathers of the momentum loop (both default on)
void setPairPaths(bool kernelFixed, bool momBuf);
//! pair loops that run LDS-staged (hydro.hip g_staged: bit 0 XMass, 1 Gradh, 2 IAD, 3 AV, 4 momentum)
void setStaged(unsigned mask);
unsigned stagedMask();
//! the search stores its per-slot staged-source masks (packed_list.hpp) also when no staged loop is enabled (tests)
void setListMasks(bool on);
bool listMasksForced();
//! fixed-point {x, y, z, m} records (QFrame of the box) of particles [0, n): the search and the XMass loop read them
void packPosQ(int64_t n, const double* x, const double* y, const double* z, const float* m, const QFrame& q,
              SrcPosQ* out, hipStream_t s);
//! overflow-row stripes of the packed-list pool; stats must hold 8 + 32 * stripes counters
int neighborRowStripes();
//! list-row demand of the next search's five pool candidates per overflow stripe (zeroed over[5 * stripes], += )
void rowPlan(int64_t groups, unsigned ngmax, const int32_t* tab, int home, unsigned long long* over, hipStream_t s);

// hydro.hip
struct MomFields
{
    const double *x, *y, *z;
    const float *vx, *vy, *vz, *h, *m, *prho, *c;
    const float* cij[6];
    const float *kx, *xm, *alpha;
    const float* dV[6];
};

struct StdFields
{
    const double *x, *y, *z;
    const float *vx, *vy, *vz, *h, *m, *rho, *p, *c;
    const float* cij[6];
};

// Record hand-offs of the fixed-point VE loops (hydro.hip packRanges): inDone = 0 pack all source records, 1 the own
// range was written by the previous loop's epilogue, 2 all are written (the search's SrcPosQ); the *Out pointers are
// the next loop's record arrays the epilogue fills for the own targets (null: none).
void xmass(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const double* x, const double* y,
           const double* z, const float* h, const float* m, const float* wh, void* rec, float* xm, hipStream_t s,
           int inDone = 0, void* xmOut = nullptr);
void veDefGradh(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const double* x,
                const double* y, const double* z, const float* h, const float* m, const float* wh, const float* whd,
                const float* xm, void* rec, float* kx, float* gradh, float mUniform, hipStream_t s, int inDone = 0,
                void* iadOut = nullptr, const float* vx = nullptr, const float* vy = nullptr,
                const float* vz = nullptr, const double* eosTemp = nullptr, float* eosPrho = nullptr,
                float* eosC = nullptr, float* eosRho = nullptr, float* eosP = nullptr);
void eosPolytropic(int64_t first, int64_t last, const float* kx, const float* xm, const float* m, float* p, float* c,
                   hipStream_t s);
void eosVe(int64_t first, int64_t last, const SphConsts& sc, const double* temp, const float* m, const float* kx,
           const float* xm, const float* gradh, float* prho, float* c, float* rho, float* p, hipStream_t s);
void eosStd(int64_t first, int64_t last, const SphConsts& sc, const double* temp, const float* m, float* rho,
            float* p, float* c, hipStream_t s);
void iad(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const double* x, const double* y,
         const double* z, const float* h, const float* wh, const float* numer, const float* denom, void* rec,
         float* const cij[6], hipStream_t s);
void iadDivvCurlv(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const double* x,
                  const double* y, const double* z, const float* vx, const float* vy, const float* vz, const float* h,
                  const float* wh, const float* kx, const float* xm, void* rec, float* const cij[6], float* divv,
                  float* curlv, float* const dV[6], void* avS, hipStream_t s, int inDone = 0, void* avOut = nullptr,
                  void* momOut = nullptr, const float* cs = nullptr, const float* m = nullptr,
                  const float* prho = nullptr, int momSplit = 0);
void avSwitches(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const double* x,
                const double* y, const double* z, const float* vx, const float* vy, const float* vz, const float* h,
                const float* c, float* const cij[6], const float* wh, const float* kx, const float* xm,
                const float* divv, double dt, void* rec, const void* avS, float* alpha, hipStream_t s, int inDone = 0,
                void* momOut = nullptr, float* alphaOut = nullptr, const double* dtDev = nullptr, int momSplit = 0);
void momentumEnergyVe(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const MomFields& f,
                      bool avClean, const float* wh, void* rec, void* recGradV, float* ax, float* ay, float* az,
                      double* du, float* minDt, hipStream_t s, int inDone = 0, float mUniform = 0.f);
void momentumEnergyStd(const NbrArgs& a, const SphConsts& sc, const Box& box, int64_t ntot, const StdFields& f,
                       const float* wh, void* rec, float* ax, float* ay, float* az, double* du, float* minDt,
                       hipStream_t s);
void updatePositions(int64_t first, int64_t last, double dt, double dt_m1, const PosArgs& p, double cv,
                     const Box& box, hipStream_t s, const double* dtDev = nullptr);
void updateH(int64_t first, int64_t last, unsigned ng0, const int32_t* nc, float* h, hipStream_t s);
//! updatePositions + updateH (+ conservedQuantities into cons when given, over the updated values) in one pass
void updateStep(int64_t first, int64_t last, double dt, double dt_m1, const PosArgs& p, double cv, const Box& box,
                hipStream_t s, const double* dtDev, unsigned ng0, const int32_t* nc, float* h, const float* m,
                double* cons, const double* eg0, const double* eg1);
void conservedQuantities(int64_t first, int64_t last, const double* x, const double* y, const double* z,
                         const float* vx, const float* vy, const float* vz, const float* m, const double* temp,
                         const double* u, const int32_t* nc, double cv, double* out, hipStream_t s,
                         const double* eg0 = nullptr, const double* eg1 = nullptr);

// cooling.hip (physics: sphx/cooling.hpp); coolingTimestep min-reduces into *out (initialize to 1e300)
void coolParticles(int64_t first, int64_t last, double dt, const float* rho, const double* u, double* du,
                   const CoolingParams& p, hipStream_t s);
void coolingTimestep(int64_t first, int64_t last, const float* rho, const double* u, const CoolingParams& p,
                     double* out, hipStream_t s);
void coolingEos(int64_t first, int64_t last, double gamma, const float* rho, const double* u, float* pr, float* c,
                hipStream_t s);

// multipole.hip (order-P Cartesian multipoles, P in [1, 6]; math: sphx/multipole.hpp)
void multipoleUpsweep(int order, int64_t N, const int32_t* n2l, const int32_t* child, const int64_t* levelRange,
                      const int32_t* ns, const int32_t* ne, const double* x, const double* y, const double* z,
                      const float* m, const double* centers, float* Q, hipStream_t s);
void computeGravityMultipole(int order, int64_t first, int64_t last, const int32_t* child, const int32_t* n2l,
                             const int32_t* ns, const int32_t* ne, const double* centers, const float* Q,
                             const double* x, const double* y, const double* z, const float* h, const float* m,
                             double G, float* ax, float* ay, float* az, double* ugrav, double* esum, int* overflow,
                             hipStream_t s);

// gravity.hip
void gravityUpsweepFused(const int32_t* n2l, int64_t N, const int32_t* ns, const int32_t* ne, const double* x,
                         const double* y, const double* z, const float* m, const int32_t* child,
                         const int32_t* parents, const KeyT* prefixes, const Box& box, int kind, double invTheta,
                         double* centers, void* mp, unsigned* cnt, hipStream_t s);
void gravityLeaves(const int32_t* n2l, int64_t N, const int32_t* ns, const int32_t* ne, const double* x,
                   const double* y, const double* z, const float* m, double* centers, void* mp, hipStream_t s);
void gravityUpsweepLevel(int64_t a, int64_t b, const int32_t* n2l, const int32_t* child, double* centers, void* mp,
                         hipStream_t s);
void gravitySetMac(int64_t N, const KeyT* prefixes, const Box& box, int kind, double invTheta, double* centers,
                   hipStream_t s);
// Barnes-Hut in two phases: interaction lists (per 64-target group, tagged with the target halves they apply to),
// then evaluation (M2P kernel, P2P kernel, combine, fused fallback for groups that overflowed the slabs)
size_t gravityScratchBytes(int64_t n, int capM, int capL);

// device-check build (common.h SPHX_DCHECK): read and clear the failed-check bits of each translation unit
unsigned dcheckHydro();
unsigned dcheckSfc();
unsigned dcheckGravity();
bool deviceChecksEnabled();
void computeGravityLists(int64_t first, int64_t last, const int32_t* child, const int32_t* n2l, const int32_t* ns,
                         const int32_t* ne, const double* centers, const void* mp, const double* x, const double* y,
                         const double* z, unsigned long long* stats, void* scratch, int testFrontCap, int capM,
                         int capL, hipStream_t s);
void computeGravityEval(int64_t first, int64_t last, const int32_t* child, const int32_t* n2l, const int32_t* ns,
                        const int32_t* ne, const double* centers, const void* mp, const double* x, const double* y,
                        const double* z, const float* h, const float* m, float G, float* ax, float* ay, float* az,
                        double* ugrav, double* out, unsigned long long* stats, void* scratch, int capM, int capL,
                        void* pacc, int64_t nsrc, int64_t numNodes, void* rec, const double* mm, hipStream_t s, int phase = 0);
//! bytes of the record buffer of computeGravityEval (16 B per source particle, 40 B per tree node)
inline size_t gravityRecordBytes(int64_t nsrc, int64_t numNodes) { return size_t(16 * nsrc + 40 * numNodes); }
void directSum(int64_t first, int64_t last, int64_t n, const double* x, const double* y, const double* z,
               const float* h, const float* m, float G, float* ax, float* ay, float* az, double* ugrav, double* out,
               hipStream_t s);

void markLet(int64_t nb, const double* bc, const double* bh, const int32_t* child, const int32_t* n2l,
             const double* tc, const double* th, const double* gc, const Box& box, uint8_t* failed, hipStream_t s);
void markOutsideRange(int64_t N, const KeyT* prefixes, KeyT lo, KeyT hi, uint8_t* failed, hipStream_t s);
//! LET selection from the open flags (failed | outside, outside may be null): particle flags (over the tree's particles
//! starting at offset) of opened leaves, send flags of the first unopened non-empty nodes below opened ones
void letSelect(int64_t N, int64_t L, int64_t np, const uint8_t* failed, const uint8_t* outside,
               const int32_t* leafToNode, const int32_t* ns, const int32_t* ne, int64_t offset, const void* mp,
               const int32_t* parents, uint8_t* pflags, uint8_t* send, hipStream_t s);
// let_tree.hip: the remote LET tree on the device (plan in the sync, build at the gravity phase)
size_t remoteLetWorkBytes(int64_t M);
//! plan words (uint64, kLetPlanWords = 24): [0] leaf-array entries L + 1, [1] overlapping nodes, [2 + l] leaves at level l
void remoteLetPlan(int64_t M, const KeyT* codes, void* work, uint64_t* plan, hipStream_t s);
void remoteLetEmit(int64_t M, const KeyT* codes, const void* work, KeyT* tree, hipStream_t s);
void remoteLetScatter(int64_t M, const void* work, const int32_t* leafToNode, const double* rc, const float* rq,
                      double* centers, float* mp, int mode, double value, hipStream_t s);
void remoteLetUpsweep(const int64_t* levelRange, const int32_t* n2l, const int32_t* child, double* centers, void* mp,
                      hipStream_t s);
void m2pFlat(int64_t first, int64_t last, const double* x, const double* y, const double* z, const float* m,
             int64_t M, const double* mc, const void* mp, float G, float* ax, float* ay, float* az, double* ugrav,
             double* out, hipStream_t s);

// turbulence.hip: modes = numModes records of 10 floats {kx, ky, kz, pad, amp*Re[3], amp*Im[3]}
void computeStirring(int64_t first, int64_t last, const double* x, const double* y, const double* z, float* ax,
                     float* ay, float* az, int numModes, const void* modes, float norm, hipStream_t s);
//! OU update of the phases (6 per mode, fp64, dt from the device) and the stirring table rows, one launch
void turbulencePhases(int numModes, double* phases, const double* noise, const double* kvec, const double* amps,
                      const double* dtDev, double decayTime, double variance, double solWeight, void* table,
                      hipStream_t s);

} // namespace sphx::hip
