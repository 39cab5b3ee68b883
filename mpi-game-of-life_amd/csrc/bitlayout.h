// bitlayout.h -- the engine's in-HBM word formats (host + device).
//
// The public format (gol.h, the oracle, data.txt) is canonical: bit j of word q
// is column 64q+j.  Inside the engine every word is stored column-split: the low
// dword holds the 32 even columns (64q+2j -> bit j) and the high dword the 32 odd
// columns (64q+2j+1 -> bit 32+j).  Then the left neighbour of every odd column and
// the right neighbour of every even column sit at the same bit index in the other
// half, and only the two remaining neighbour planes need a funnel shift
// (2 v_alignbit per word instead of 4; see life_kernels.hip).  Conversion happens
// only at load/store, random init and digest.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GOL_HD __host__ __device__ __forceinline__
#else
#define GOL_HD inline
#endif

// gather the bits at even positions of x into the low 32 bits
GOL_HD uint64_t gol_compress_even(uint64_t x)
{
    x &= 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x >> 4)) & 0x00FF00FF00FF00FFull;
    x = (x | (x >> 8)) & 0x0000FFFF0000FFFFull;
    x = (x | (x >> 16)) & 0x00000000FFFFFFFFull;
    return x;
}

// spread the low 32 bits of x to the even positions
GOL_HD uint64_t gol_spread_even(uint64_t x)
{
    x &= 0x00000000FFFFFFFFull;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x;
}

// canonical -> column-split
GOL_HD uint64_t gol_split64(uint64_t c)
{
    return gol_compress_even(c) | (gol_compress_even(c >> 1) << 32);
}

// column-split -> canonical
GOL_HD uint64_t gol_join64(uint64_t v)
{
    return gol_spread_even(v) | (gol_spread_even(v >> 32) << 1);
}

// bit index inside a column-split word of column j (0..63) of that word
GOL_HD unsigned gol_split_bit(unsigned j) { return ((j & 1u) << 5) | (j >> 1); }

// ---- lane groups of 4 planes (two words, 128 columns) ----
// The stencil kernel works on lane groups of NP 32-bit planes: NP/2 words, 32*NP
// columns, column 32*NP*g + NP*j + k at bit j of plane k (plane 2i in the low and
// plane 2i+1 in the high dword of the group's word i).  NP = 2 is the column
// split above.  With NP = 4 the neighbours of planes 1 and 2 are other planes at
// the same bit; only plane 0's left and plane 3's right neighbours need a funnel
// shift, so the 2 lane moves + 2 v_alignbit are paid per 128 columns, not per 64.

// gather the bits at positions = 0 mod 4 of x into the low 16 bits
GOL_HD uint64_t gol_compress4(uint64_t x)
{
    x &= 0x1111111111111111ull;
    x = (x | (x >> 3)) & 0x0303030303030303ull;
    x = (x | (x >> 6)) & 0x000F000F000F000Full;
    x = (x | (x >> 12)) & 0x000000FF000000FFull;
    x = (x | (x >> 24)) & 0x000000000000FFFFull;
    return x;
}

// spread the low 16 bits of x to the positions = 0 mod 4
GOL_HD uint64_t gol_spread4(uint64_t x)
{
    x &= 0x000000000000FFFFull;
    x = (x | (x << 24)) & 0x000000FF000000FFull;
    x = (x | (x << 12)) & 0x000F000F000F000Full;
    x = (x | (x << 6)) & 0x0303030303030303ull;
    x = (x | (x << 3)) & 0x1111111111111111ull;
    return x;
}

// canonical words c[0..np/2-1] of one lane group -> stored words s[0..np/2-1]
GOL_HD void gol_split_group(const uint64_t* c, uint64_t* s, int np)
{
    if (np == 2) {
        s[0] = gol_split64(c[0]);
        return;
    }
    uint64_t p[4];
    for (int k = 0; k < 4; ++k)
        p[k] = gol_compress4(c[0] >> k) | (gol_compress4(c[1] >> k) << 16);
    s[0] = p[0] | (p[1] << 32);
    s[1] = p[2] | (p[3] << 32);
}

// stored words s[0..np/2-1] of one lane group -> canonical words c[0..np/2-1]
GOL_HD void gol_join_group(const uint64_t* s, uint64_t* c, int np)
{
    if (np == 2) {
        c[0] = gol_join64(s[0]);
        return;
    }
    const uint64_t p[4] = {s[0] & 0xFFFFFFFFull, s[0] >> 32, s[1] & 0xFFFFFFFFull, s[1] >> 32};
    uint64_t c0 = 0, c1 = 0;
    for (int k = 0; k < 4; ++k) {
        c0 |= gol_spread4(p[k]) << k;
        c1 |= gol_spread4(p[k] >> 16) << k;
    }
    c[0] = c0;
    c[1] = c1;
}
