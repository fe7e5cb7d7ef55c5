/*! Packed neighbor lists of the GPU path: 16-bit delta-coded entries in 1-KiB list rows allocated per target group.
 *
 * The reference keeps no neighbor lists on the GPU (each of its five SPH kernels re-traverses the tree,
 * sph/hydro_ve/*_gpu.cu); here the search stores them once per step and every pair loop streams them. Stored as
 * int32 at a fixed ngmax stride they cost 608 B/particle (ngmax 150), two thirds of the whole footprint. Entries of a
 * lane's list are ascending SFC indices of a compact neighborhood, so consecutive entries are close: on the Sedov
 * lattice (64 M particles) 99.46 % of the steps between consecutive entries (the first one measured from the target)
 * fit 15 bits (profiles/r2_list_stats.md).
 *
 * Slot (16 bit): bit 0 = emit flag, bits 1..15 = signed d.
 *   emit: prev += d, the entry is prev                  (|step| <= 16383: one slot)
 *   jump: prev += d * 2^14, no entry                    (larger steps: jump slots, then one emit slot)
 *   0x0000 is a jump by 0: padding. A jump can move by +-2^28, so any 31-bit index step is a few slots.
 * A decoded jump or padding slot yields the target's own index, which is never one of its neighbors: the pair loops
 * skip an entry equal to the target.
 *
 * Layout of one search's list buffer (int32):
 *   [ group tables: G x kTab ints, padded to 256 ints ][ rows: 1 KiB each = 64 lanes x int4 (8 slots per lane) ]
 *   group table: [0] = number of list rows of the group (wave-uniform trip count of the pair loops),
 *                [1 + b] = row of list block b; entries past the group's rows name row 0 (valid memory: the pair
 *                loops prefetch two blocks ahead).
 * Rows: group g owns `home` rows (g*home ..), chosen by the host from the previous search's row counts; rows past
 * those come from one of 64 overflow stripes through an atomic counter per stripe (neighbors.hip PackedOut). The
 * host reads the counters, and repeats the search with more overflow rows if a stripe ran out.
 */
#pragma once

#include <cstddef>
#include <cstdint>

#include "annotation.hpp"

namespace sphx
{

//! slots per lane a list may use beyond ngmax entries (jump slots); a lane needing more re-iterates h
constexpr unsigned kListJumpSlack = 32;
//! list rows (8 slots per lane) a group may use
SPHX_HD constexpr unsigned packedRowsMax(unsigned ngmax) { return (ngmax + kListJumpSlack + 7) / 8; }
//! ints per group table: row count + rows + 2 prefetch entries, rounded to 4 (16-B aligned tables)
SPHX_HD constexpr unsigned packedTableInts(unsigned ngmax) { return (packedRowsMax(ngmax) + 3 + 3) & ~3u; }
//! ints of the table region of a list buffer for `groups` target groups (rows start 1-KiB aligned)
SPHX_HD constexpr int64_t packedTableRegion(int64_t groups, unsigned ngmax)
{
    return (groups * int64_t(packedTableInts(ngmax)) + 255) / 256 * 256;
}

constexpr int kSlotFine = 16383; // largest |d| of an emit slot
constexpr int kJumpShift = 14;

//! number of slots that encode a step of `delta` (1 emit slot + jump slots)
SPHX_HD unsigned slotsFor(int delta)
{
    unsigned n = 1;
    while (delta < -kSlotFine - 1 || delta > kSlotFine)
    {
        int J = (delta + (1 << (kJumpShift - 1))) >> kJumpShift;
        J     = J < -kSlotFine - 1 ? -kSlotFine - 1 : (J > kSlotFine ? kSlotFine : J);
        delta -= J * (1 << kJumpShift);
        ++n;
    }
    return n;
}

//! emit the slots of one step (jumps first, then the emit slot) through put(uint16 slot)
template<class Put>
SPHX_HD void encodeStep(int delta, Put&& put)
{
    while (delta < -kSlotFine - 1 || delta > kSlotFine)
    {
        int J = (delta + (1 << (kJumpShift - 1))) >> kJumpShift;
        J     = J < -kSlotFine - 1 ? -kSlotFine - 1 : (J > kSlotFine ? kSlotFine : J);
        put(unsigned(J * 2) & 0xFFFFu);
        delta -= J * (1 << kJumpShift);
    }
    put((unsigned(delta * 2) | 1u) & 0xFFFFu);
}

#if defined(__HIPCC__)
//! @brief slot -> entry (or `self` for jumps/padding); `prev` carries the running index
__device__ __forceinline__ unsigned decodeSlot(int d, unsigned e, unsigned& prev, unsigned self)
{
    prev += unsigned(e ? d : d * (1 << kJumpShift));
    return e ? prev : self;
}

//! @brief the 2 entries of one word of a list block (slot 2q in the low half of word q)
__device__ __forceinline__ void decodeWord(int w, unsigned& prev, unsigned self, unsigned& j0, unsigned& j1)
{
    j0 = decodeSlot(__builtin_amdgcn_sbfe(w, 1, 15), unsigned(w) & 1u, prev, self);
    j1 = decodeSlot(w >> 17, (unsigned(w) >> 16) & 1u, prev, self);
}

//! @brief the 8 entries of one list block (int4 = 8 slots)
__device__ __forceinline__ void decodeBlock(int4 w, unsigned& prev, unsigned self, unsigned (&j)[8])
{
    decodeWord(w.x, prev, self, j[0], j[1]);
    decodeWord(w.y, prev, self, j[2], j[3]);
    decodeWord(w.z, prev, self, j[4], j[5]);
    decodeWord(w.w, prev, self, j[6], j[7]);
}

#ifndef SPHX_DCHECK // translation units without the kernels' common.h (host bindings): checks compile to nothing
#define SPHX_DCHECK(cond, bit) ((void)0)
#endif

//! @brief one lane's view of its group's packed list (see the file comment)
struct PackedLane
{
    const int32_t* tab; // group table (wave-uniform address: scalar loads)
    const int4* rows;   // first row + lane
    unsigned self;      // target index: decoded jump/padding slots, skipped by the loops
    unsigned nblk;      // list rows of the group (wave-uniform)
#ifdef SPHX_DEVICE_CHECKS
    unsigned ntot; // source records (device-check build: decoded indices are checked against it)
#endif

    //! the decoded index j, or the target itself if j is out of range (device-check build: reported, bit 0)
    __device__ __forceinline__ unsigned checked(unsigned j) const
    {
#ifdef SPHX_DEVICE_CHECKS
        SPHX_DCHECK(j < ntot, 0);
        return j < ntot ? j : self;
#else
        return j;
#endif
    }

    __device__ __forceinline__ int4 block(unsigned b) const
    {
        const int32_t r = *(const __attribute__((address_space(4))) int32_t*)(tab + 1 + b);
        return rows[size_t(r) * 64];
    }
};
#endif

} // namespace sphx
