// host_sim.h -- the handful of HIP device intrinsics minigrid-rl_amd/csrc/mgx_device.h uses, for a host
// (g++) build of its generator: TEST INFRASTRUCTURE (tests/test_generator_host.py), never the product.
#pragma once
#include <cstdint>
#include <cstring>

#define __device__
#define __host__
#define __forceinline__ inline
#define __noinline__ __attribute__((noinline))
#define __align__(n) alignas(n)
#define __restrict__ __restrict

struct uint4 { uint32_t x, y, z, w; };

static inline int __ffsll(long long v) { return __builtin_ffsll(v); }
static inline int __ffs(int v) { return __builtin_ffs(v); }
static inline int __popc(unsigned v) { return __builtin_popcount(v); }
static inline int __clz(int v) { return v ? __builtin_clz((unsigned)v) : 32; }
static inline unsigned __umul24(unsigned a, unsigned b) { return (a & 0xFFFFFFu) * (b & 0xFFFFFFu); }
static inline int __mul24(int a, int b) {
    const int a24 = (int)((unsigned)a << 8) >> 8, b24 = (int)((unsigned)b << 8) >> 8;
    return a24 * b24;
}
static inline uint64_t __umul64hi(uint64_t a, uint64_t b) { return (uint64_t)(((unsigned __int128)a * b) >> 64); }
static inline double __dmul_rn(double a, double b) { return a * b; }      // built with -ffp-contract=off
static inline double __dsub_rn(double a, double b) { return a - b; }
static inline int min(int a, int b) { return a < b ? a : b; }
static inline int max(int a, int b) { return a > b ? a : b; }
