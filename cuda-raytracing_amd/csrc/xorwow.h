// xorwow.h -- curand-compatible XORWOW seeding shared by host and device code.
#pragma once

#include <stdint.h>

#include "rt_math.h"

// Jump matrices kept: 4^k * 2^67 for k < 32 covers any 64-bit subsequence.
#define RT_XORWOW_JUMPS 32

// Flat [RT_XORWOW_JUMPS][800] table of A^(4^k * 2^67) (host memory, built once).
const uint32_t* rt_xorwow_jump_table();

// curand_init step 1 (seed salting) for a 32-bit seed as passed by init_rng
// (Random.cu:10 takes `unsigned int seed`, widened to unsigned long long): st = {d, v0..v4}.
RT_HD void rt_xorwow_seed(uint32_t seed, uint32_t st[6]) {
    const uint32_t s0 = seed ^ 0xaad26b49u;
    const uint32_t s1 = 0u ^ 0xf7dcefddu;  // upper 32 bits of the widened seed are 0
    const uint32_t t0 = 1099087573u * s0;
    const uint32_t t1 = 2591861531u * s1;
    st[0] = 6615241u + t1 + t0;
    st[1] = 123456789u + t0;
    st[2] = 362436069u ^ t0;
    st[3] = 521288629u + t1;
    st[4] = 88675123u ^ t1;
    st[5] = 5783321u + t0;
}
