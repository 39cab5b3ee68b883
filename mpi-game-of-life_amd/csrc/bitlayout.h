// bitlayout.h -- the engine's in-HBM word format (host + device).
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
