/*! Hilbert keys as a finite-state machine (host construction). The curve of sfc.hpp hilbertKey seen level by level:
 *  a cell's state (orientation) maps the octant of each child to its key digit and to the child's state. The machine
 *  is derived from hilbertKey itself: the octant -> digit permutation of a cell identifies its state, and every
 *  transition is checked against hilbertKey on cells deeper in the tree. Used by the GPU key kernel
 *  (csrc/hip/sfc_sort.hip, tables in LDS, two levels per lookup) and checked on the CPU (cpu/bind_cpu.cpp
 *  hilbert_fsm_check, tests/test_sfc.py).
 */
#pragma once

#include <array>
#include <cstdint>
#include <map>
#include <stdexcept>
#include <vector>

#include "sfc.hpp"

namespace sphx
{

struct HilbertFsm
{
    int nStates = 0;
    std::vector<uint8_t> t1;  // [state][octant] = digit | next << 3   (next < 32)
    std::vector<uint16_t> t2; // [state][o1 * 8 + o2] = d1 << 3 | d2 | next << 6
};

//! octant of child o of a cell: (x bit, y bit, z bit) = (o >> 2, o >> 1, o) & 1 (the Morton / key digit order)
inline std::array<uint8_t, 8> hilbertPerm(uint32_t cx, uint32_t cy, uint32_t cz, int level)
{
    std::array<uint8_t, 8> p{};
    const uint32_t half = 1u << (kMaxLevel - level - 1);
    for (int o = 0; o < 8; ++o)
    {
        const KeyT k = hilbertKey(cx + ((o >> 2) & 1) * half, cy + ((o >> 1) & 1) * half, cz + (o & 1) * half);
        p[o]         = uint8_t((k >> (3 * (kMaxLevel - level - 1))) & 7);
    }
    return p;
}

inline HilbertFsm buildHilbertFsm()
{
    struct Cell
    {
        uint32_t x, y, z;
        int level;
    };
    std::map<std::array<uint8_t, 8>, int> ids;
    std::vector<std::array<uint8_t, 8>> perms;
    std::vector<std::array<int, 8>> next;
    std::vector<Cell> rep, queue{{0, 0, 0, 0}};
    auto idOf = [&](const Cell& c) -> int
    {
        const auto p = hilbertPerm(c.x, c.y, c.z, c.level);
        auto it      = ids.find(p);
        if (it != ids.end()) return it->second;
        const int id = int(perms.size());
        ids[p]       = id;
        perms.push_back(p);
        next.push_back({});
        rep.push_back(c);
        return id;
    };
    idOf(queue[0]);
    // breadth-first over the states' representative cells (the shallowest cell of each state)
    for (size_t s = 0; s < rep.size(); ++s)
    {
        const Cell c       = rep[s];
        const uint32_t half = 1u << (kMaxLevel - c.level - 1);
        if (c.level + 2 > kMaxLevel) throw std::runtime_error("Hilbert table: a state first seen too deep");
        for (int o = 0; o < 8; ++o)
            next[s][o] = idOf(Cell{c.x + ((o >> 2) & 1) * half, c.y + ((o >> 1) & 1) * half, c.z + (o & 1) * half,
                                   c.level + 1});
        if (rep.size() > size_t(32)) throw std::runtime_error("Hilbert table: more states than expected");
    }
    // every transition on a second cell of each state (a deeper one, same permutation) against hilbertKey
    std::vector<Cell> check;
    for (uint32_t probe = 0; probe < 4096; ++probe)
    {
        const int level     = 2 + int(probe % 17);
        const uint32_t span = 1u << (kMaxLevel - level);
        const uint32_t m    = (1u << level) - 1u;
        const uint32_t h    = probe * 2654435761u;
        check.push_back(Cell{((h >> 3) & m) * span, ((h >> 11) & m) * span, ((h >> 19) & m) * span, level});
    }
    for (const Cell& c : check)
    {
        auto it = ids.find(hilbertPerm(c.x, c.y, c.z, c.level));
        if (it == ids.end()) throw std::runtime_error("Hilbert table: unseen state");
        const uint32_t half = 1u << (kMaxLevel - c.level - 1);
        for (int o = 0; o < 8; ++o)
        {
            const auto pc = hilbertPerm(c.x + ((o >> 2) & 1) * half, c.y + ((o >> 1) & 1) * half,
                                        c.z + (o & 1) * half, c.level + 1);
            if (perms[next[it->second][o]] != pc) throw std::runtime_error("Hilbert table: inconsistent transition");
        }
    }
    HilbertFsm f;
    f.nStates = int(perms.size());
    f.t1.resize(size_t(f.nStates) * 8);
    f.t2.resize(size_t(f.nStates) * 64);
    for (int s = 0; s < f.nStates; ++s)
        for (int o1 = 0; o1 < 8; ++o1)
        {
            const int s1          = next[s][o1];
            f.t1[s * 8 + o1]      = uint8_t(perms[s][o1] | (s1 << 3));
            for (int o2 = 0; o2 < 8; ++o2)
                f.t2[s * 64 + o1 * 8 + o2] =
                    uint16_t((perms[s][o1] << 3) | perms[s1][o2] | (next[s1][o2] << 6));
        }
    return f;
}

//! @brief the Hilbert key of integer coordinates walked through the machine's two-level table (host form of the GPU
//!        kernel's loop)
inline KeyT hilbertKeyFsm(const HilbertFsm& f, uint32_t ix, uint32_t iy, uint32_t iz)
{
    auto oct = [&](int b) { return (((ix >> b) & 1u) << 2) | (((iy >> b) & 1u) << 1) | ((iz >> b) & 1u); };
    uint32_t e  = f.t1[oct(kMaxLevel - 1)];
    KeyT key    = e & 7u;
    uint32_t st = e >> 3;
    for (int b = kMaxLevel - 2; b >= 1; b -= 2)
    {
        const uint32_t v = f.t2[st * 64 + ((oct(b) << 3) | oct(b - 1))];
        key              = (key << 6) | (v & 63u);
        st               = v >> 6;
    }
    return key;
}

} // namespace sphx
