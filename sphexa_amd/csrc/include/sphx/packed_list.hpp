/*! Chunk-coded neighbor lists of the GPU path: one 16-bit code per entry, 8 per 16-byte block, in 1-KiB rows
 *  allocated per 64-particle target group.
 *
 * The reference keeps no neighbor lists on the GPU (each of its five SPH kernels re-traverses the tree,
 * sph/hydro_ve/ *_gpu.cu); here the search stores them once per step and every pair loop streams them. Stored as
 * int32 at a fixed ngmax stride they cost 608 B/particle (ngmax 150).
 *
 * The search of a group tests the sources of its candidate leaves in chunks of at most 64 consecutive particles
 * (one chunk = one wave-wide coalesced load, lane k holds particle c0 + k). Every chunk that holds a candidate gets a
 * slot s in the group's chunk table (table[s] = c0); a neighbor is then the 16-bit code
 *     code = s | k << 10        (s < kChunkCap <= 1024, k < 64)   ->   j = table[s] + k.
 * Slot 0 is the group's own first particle, so code (lane << 10) decodes to the target itself: that is the padding
 * code of a lane's last block, and the lists also hold the target itself (the search counts it, as the reference's
 * nc does, instead of excluding it per candidate). The pair loops skip entries equal to the target. Lanes past the
 * last particle of a partial group pad with the last particle (the loops clamp them to it: a valid record).
 * A code is final when the candidate test finds the hit: the search writes list blocks straight from its hit ring,
 * without raw index lists, read-back or a delta-encoding pass; entries are independent (no prefix chain to decode).
 *
 * Layout of one search's list buffer (int32):
 *   [ group tables: G x packedTableInts ints, padded to 256 ints ][ rows: 1 KiB each = 64 lanes x int4 ]
 *   group table: [0] = list blocks nblk (wave-uniform trip count of the pair loops), [1] = nch | Tc << 10 | T << 16
 *                (tableWord) with nch the chunk-table entries, Tc the rows of chunk bases and T all table rows,
 *                [2 + r] = row of ordinal r. Ordinals 0 .. Tc-1 hold the chunk bases (256 ints per row), ordinals
 *                Tc .. T-1 the chunk masks (bit k of slot s: source c0 + k was staged for the group, i.e. lies in the
 *                group's search box; 128 {lo, hi} int pairs per row; the search reserves Tc and T from an upper bound
 *                of nch; written only while an LDS-staged pair loop is enabled, else T = Tc), ordinals T .. T+nblk-1 the list blocks (row of 64 lanes x 8 codes). Entries past them name
 *                row 0 (valid memory: the pair loops prefetch a block ahead). Every code (s, k) of a list has bit k of
 *                mask s set (s >= 1), so the union of a group's sources is known from the table alone: the LDS-staged
 *                pair loops (hydro.hip StagedGroup) load it once per group.
 * Rows: group g owns `home` rows (g*home ..), chosen by the host from the previous search's row counts; rows past
 * those come from one of 64 overflow stripes through an atomic counter per stripe (neighbors.hip). The host reads
 * the counters and repeats the search with more overflow rows if a stripe ran out.
 */
#pragma once

#include <cstddef>
#include <cstdint>

#include "annotation.hpp"

namespace sphx
{

//! chunk-table capacity per target group (the pair loops keep the table in LDS: 4 B per slot and wave)
constexpr unsigned kChunkCap = 512;
constexpr unsigned kChunkSlotBits = 10;
constexpr unsigned kChunkSlotMask = (1u << kChunkSlotBits) - 1;
//! rows of a chunk table at capacity
constexpr unsigned kChunkTabRowsMax = (kChunkCap + 255) / 256;
//! rows of the chunk masks at capacity (64-bit mask of the staged sources per slot, 128 per row)
constexpr unsigned kMaskTabRowsMax = (kChunkCap + 127) / 128;
//! table rows (chunk bases + masks) at capacity
constexpr unsigned kTableRowsMax = kChunkTabRowsMax + kMaskTabRowsMax;
//! list blocks a lane may fill: ngmax neighbors + the target itself
SPHX_HD constexpr unsigned listBlocksMax(unsigned ngmax) { return (ngmax + 1 + 7) / 8; }
//! rows a group may use (chunk table + masks + list blocks)
SPHX_HD constexpr unsigned packedRowsMax(unsigned ngmax) { return listBlocksMax(ngmax) + kTableRowsMax; }
//! ints per group table: counts + rows + 2 prefetch entries, rounded to 4 (16-B aligned tables)
SPHX_HD constexpr unsigned packedTableInts(unsigned ngmax) { return (2 + packedRowsMax(ngmax) + 2 + 3) & ~3u; }
//! ints of the table region of a list buffer for `groups` target groups (rows start 1-KiB aligned)
SPHX_HD constexpr int64_t packedTableRegion(int64_t groups, unsigned ngmax)
{
    return (groups * int64_t(packedTableInts(ngmax)) + 255) / 256 * 256;
}
//! rows of a chunk table with nch entries
SPHX_HD constexpr unsigned chunkTabRows(unsigned nch) { return (nch + 255) / 256; }
//! rows of the chunk masks of nch entries
SPHX_HD constexpr unsigned maskTabRows(unsigned nch) { return (nch + 127) / 128; }
//! group-table word 1: chunk-table entries | chunk-base rows << 10 | table rows << 16
SPHX_HD constexpr uint32_t tableWord(unsigned nch, unsigned Tc, unsigned T) { return nch | Tc << 10 | T << 16; }
SPHX_HD constexpr unsigned tableWordNch(uint32_t w) { return w & 0x3FFu; }
SPHX_HD constexpr unsigned tableWordTc(uint32_t w) { return (w >> 10) & 0x3Fu; }
SPHX_HD constexpr unsigned tableWordT(uint32_t w) { return w >> 16; }
//! code of particle c0 + k of chunk slot s
SPHX_HD constexpr uint32_t chunkCode(unsigned s, unsigned k) { return s | (k << kChunkSlotBits); }

#if defined(__HIPCC__)

#ifndef SPHX_DCHECK // translation units without the kernels' common.h (host bindings): checks compile to nothing
#define SPHX_DCHECK(cond, bit) ((void)0)
#endif

//! @brief the 2 entries of one word of a list block (code 2q in the low half of word q). The slot is masked to the
//!        table capacity, so a corrupted code stays inside the LDS table (device-check builds then flag the index).
__device__ __forceinline__ void decodeWord(int w, const uint32_t* ctab, unsigned& j0, unsigned& j1)
{
    static_assert((kChunkCap & (kChunkCap - 1)) == 0 && kChunkCap <= (1u << kChunkSlotBits), "table capacity");
    j0 = ctab[unsigned(w) & (kChunkCap - 1)] + __builtin_amdgcn_ubfe(unsigned(w), kChunkSlotBits, 6);
    j1 = ctab[__builtin_amdgcn_ubfe(unsigned(w), 16, kChunkSlotBits) & (kChunkCap - 1)] +
         (unsigned(w) >> (16 + kChunkSlotBits));
}

//! @brief the 8 entries of one list block (int4 = 8 codes)
__device__ __forceinline__ void decodeBlock(int4 w, const uint32_t* ctab, unsigned (&j)[8])
{
    decodeWord(w.x, ctab, j[0], j[1]);
    decodeWord(w.y, ctab, j[2], j[3]);
    decodeWord(w.z, ctab, j[4], j[5]);
    decodeWord(w.w, ctab, j[6], j[7]);
}

//! @brief one lane's view of its group's list (see the file comment)
struct PackedLane
{
    const int32_t* tab;   // row ordinals of the list blocks (group table + 2 + T; wave-uniform: scalar loads)
    const int4* rows;     // first row + lane
    const uint32_t* ctab; // the group's chunk table in this wave's LDS
    unsigned self;        // target index: padding codes decode to it, the loops skip it
    unsigned nblk;        // list blocks of the group (wave-uniform)
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
        const int32_t r = *(const __attribute__((address_space(4))) int32_t*)(tab + b);
        return rows[size_t(r) * 64];
    }

    __device__ __forceinline__ void decode(int w, unsigned& j0, unsigned& j1) const
    {
        decodeWord(w, ctab, j0, j1);
        j0 = checked(j0);
        j1 = checked(j1);
    }
};
#endif

} // namespace sphx
