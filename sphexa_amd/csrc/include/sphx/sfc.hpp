// Space-filling-curve keys and cornerstone key algebra.
//
// Parity (behaviour, not code): reference domain/include/cstone/sfc/{hilbert,morton,sfc,common}.hpp.
//   - 64-bit keys, 21 bits per dimension, 63 bits used           (sfc/common.hpp:47-120)
//   - Hilbert is the default curve; Morton available             (sfc/sfc.hpp:44-54)
//   - node ranges are powers of 8, level 0 = root = [0, 2^63)    (sfc/common.hpp nodeRange/treeLevel)
//   - Warren-Salmon placeholder-bit encoding of (key, level)     (sfc/common.hpp:300-360)
// The Hilbert curve is computed with Skilling's transposed-axes algorithm ("Programming the Hilbert curve",
// AIP Conf. Proc. 707, 2004): inverse-undo + Gray encode on the three 21-bit integer coordinates, then bit
// interleave. Any key prefix of length 3*l addresses exactly one level-l octree cell (property checked in
// tests/test_sfc.py), which is all the cornerstone octree needs.
#pragma once

#include "annotation.hpp"

namespace sphx
{

using KeyT = uint64_t;

constexpr int kMaxLevel     = 21;
constexpr uint32_t kGridMax = 1u << kMaxLevel; // integer grid resolution per dimension
constexpr KeyT kKeyEnd      = KeyT(1) << 63;   // one past the last key

//! @brief number of keys covered by an octree node at @p level
SPHX_HD KeyT nodeRange(int level) { return KeyT(1) << (3 * (kMaxLevel - level)); }

//! @brief level of a node with key range @p range (must be a power of 8)
SPHX_HD int treeLevel(KeyT range) { return kMaxLevel - (63 - clz64(range)) / 3; }

//! @brief coarsest level at which @p key is a node start (0 for key 0)
SPHX_HD int alignmentLevel(KeyT key)
{
    if (key == 0) return 0;
    int tz = ctz64(key) / 3;
    int l  = kMaxLevel - tz;
    return l < 0 ? 0 : l;
}

//! @brief Warren-Salmon placeholder-bit code: sorting these gives level-major, key-minor node order
SPHX_HD KeyT placeholderCode(KeyT key, int level)
{
    return (KeyT(1) << (3 * level)) | (key >> (3 * (kMaxLevel - level)));
}

SPHX_HD int placeholderLevel(KeyT code) { return (63 - clz64(code)) / 3; }

SPHX_HD KeyT placeholderKey(KeyT code)
{
    int l = placeholderLevel(code);
    return (code ^ (KeyT(1) << (3 * l))) << (3 * (kMaxLevel - l));
}

//! @brief spread the lower 21 bits of v so that bit b lands at bit 3b
SPHX_HD KeyT spreadBits3(uint32_t v)
{
    KeyT x = v & 0x1fffff;
    x      = (x | x << 32) & 0x1f00000000ffffULL;
    x      = (x | x << 16) & 0x1f0000ff0000ffULL;
    x      = (x | x << 8) & 0x100f00f00f00f00fULL;
    x      = (x | x << 4) & 0x10c30c30c30c30c3ULL;
    x      = (x | x << 2) & 0x1249249249249249ULL;
    return x;
}

//! @brief inverse of spreadBits3
SPHX_HD uint32_t compactBits3(KeyT x)
{
    x &= 0x1249249249249249ULL;
    x = (x ^ (x >> 2)) & 0x10c30c30c30c30c3ULL;
    x = (x ^ (x >> 4)) & 0x100f00f00f00f00fULL;
    x = (x ^ (x >> 8)) & 0x1f0000ff0000ffULL;
    x = (x ^ (x >> 16)) & 0x1f00000000ffffULL;
    x = (x ^ (x >> 32)) & 0x1fffff;
    return uint32_t(x);
}

SPHX_HD KeyT mortonKey(uint32_t ix, uint32_t iy, uint32_t iz)
{
    return (spreadBits3(ix) << 2) | (spreadBits3(iy) << 1) | spreadBits3(iz);
}

SPHX_HD void decodeMorton(KeyT k, uint32_t& ix, uint32_t& iy, uint32_t& iz)
{
    ix = compactBits3(k >> 2);
    iy = compactBits3(k >> 1);
    iz = compactBits3(k);
}

//! @brief 3D Hilbert key of integer coordinates in [0, 2^21)
SPHX_HD KeyT hilbertKey(uint32_t ix, uint32_t iy, uint32_t iz)
{
    uint32_t X0 = ix, X1 = iy, X2 = iz;
    // inverse undo of the excess work
    for (uint32_t Q = 1u << (kMaxLevel - 1); Q > 1; Q >>= 1)
    {
        uint32_t P = Q - 1;
        // i = 0
        if (X0 & Q) { X0 ^= P; }
        // i = 1
        if (X1 & Q) { X0 ^= P; }
        else
        {
            uint32_t t = (X0 ^ X1) & P;
            X0 ^= t;
            X1 ^= t;
        }
        // i = 2
        if (X2 & Q) { X0 ^= P; }
        else
        {
            uint32_t t = (X0 ^ X2) & P;
            X0 ^= t;
            X2 ^= t;
        }
    }
    // Gray encode
    X1 ^= X0;
    X2 ^= X1;
    uint32_t t = 0;
    for (uint32_t Q = 1u << (kMaxLevel - 1); Q > 1; Q >>= 1)
    {
        if (X2 & Q) { t ^= Q - 1; }
    }
    X0 ^= t;
    X1 ^= t;
    X2 ^= t;
    return (spreadBits3(X0) << 2) | (spreadBits3(X1) << 1) | spreadBits3(X2);
}

//! @brief inverse of hilbertKey
SPHX_HD void decodeHilbert(KeyT key, uint32_t& ix, uint32_t& iy, uint32_t& iz)
{
    uint32_t X0 = compactBits3(key >> 2);
    uint32_t X1 = compactBits3(key >> 1);
    uint32_t X2 = compactBits3(key);
    // Gray decode
    uint32_t t = X2 >> 1;
    X2 ^= X1;
    X1 ^= X0;
    X0 ^= t;
    // undo excess work
    for (uint32_t Q = 2; Q != kGridMax; Q <<= 1)
    {
        uint32_t P = Q - 1;
        // i = 2
        if (X2 & Q) { X0 ^= P; }
        else
        {
            uint32_t s = (X0 ^ X2) & P;
            X0 ^= s;
            X2 ^= s;
        }
        // i = 1
        if (X1 & Q) { X0 ^= P; }
        else
        {
            uint32_t s = (X0 ^ X1) & P;
            X0 ^= s;
            X1 ^= s;
        }
        // i = 0
        if (X0 & Q) { X0 ^= P; }
    }
    ix = X0;
    iy = X1;
    iz = X2;
}

enum SfcKind : int
{
    kHilbert = 0,
    kMorton  = 1,
};

SPHX_HD KeyT sfcKey(int kind, uint32_t ix, uint32_t iy, uint32_t iz)
{
    return kind == kMorton ? mortonKey(ix, iy, iz) : hilbertKey(ix, iy, iz);
}

SPHX_HD void sfcDecode(int kind, KeyT k, uint32_t& ix, uint32_t& iy, uint32_t& iz)
{
    if (kind == kMorton) { decodeMorton(k, ix, iy, iz); }
    else { decodeHilbert(k, ix, iy, iz); }
}

//! @brief integer lower corner of the level-@p level node containing @p key
SPHX_HD void nodeIntCorner(int kind, KeyT key, int level, uint32_t& ix, uint32_t& iy, uint32_t& iz)
{
    sfcDecode(kind, key, ix, iy, iz);
    uint32_t mask = ~((1u << (kMaxLevel - level)) - 1u);
    ix &= mask;
    iy &= mask;
    iz &= mask;
}

} // namespace sphx
