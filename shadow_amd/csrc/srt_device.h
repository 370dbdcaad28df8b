/*
 * srt_device.h -- shared device-side definitions for the gfx950 kernels.
 */
#ifndef SRT_DEVICE_H
#define SRT_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "srt_internal.h"

#define SRT_HIPCHK(expr)                                                                   \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess) {                                                            \
            srt_set_error("HIP error %s at %s:%d (%s)", hipGetErrorString(e_), __FILE__,   \
                          __LINE__, #expr);                                                \
            return SRT_E_DEVICE;                                                           \
        }                                                                                  \
    } while (0)

/* pivot-block edge of the blocked Floyd-Warshall and the output-tile edge of its kernels */
#define SRT_FW_B 64
/* LDS row stride (u32) of a 64-wide tile: +4 keeps 16-byte alignment for ds_read_b128 */
#define SRT_FW_LDT (SRT_FW_B + 4)

/* counter-based generator hash (shadow_amd/graphs.py restates it bit for bit) */
__host__ __device__ static inline uint64_t srt_splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__host__ __device__ static inline uint64_t srt_hash(uint64_t seed, uint64_t stream, uint32_t i,
                                                    uint32_t j) {
    return srt_splitmix64(srt_splitmix64(seed * 4ull + stream) ^ (((uint64_t)i << 32) | j));
}

static inline int srt_ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

/* internal (C++ linkage) entry points shared between translation units */
int srt_dense_post_device(int32_t n, int32_t ld, int32_t directed, const uint32_t* w,
                          const double* r, uint32_t* d, double* rel, hipStream_t st,
                          srt_build_stats* stats);

#endif
