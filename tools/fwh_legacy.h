/* fwh_legacy.h -- the 4-wave FW update kernel (fwh_update_kernel, 256 threads of 8 x 8) and its
 * staging helpers, moved out of the product (shadow_amd/csrc/fw16.hip) in round 4: the 8-wave
 * fwq_update_kernel replaced it in round 2 (C4 FW 362.9 -> 339.9 ms). Kept for the A/B harnesses
 * tools/fwh_variants.hip and tools/fw16_ablate.hip, which include fw16.hip and then this file. */
#pragma once

struct fwh_stage_regs {
    uint4 a[2], b[2];
};

static __device__ __forceinline__ void fwh_gload(fwh_stage_regs& g, const u16* __restrict__ A,
                                                 const u16* __restrict__ B, size_t ld, int tid) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int ia = tid + q * 256, ra = ia & 127, ca = (ia >> 7) * 8; /* 128 rows x 32 pivots */
        const int ib = tid + q * 256, rb = ib >> 4, cb = (ib & 15) * 8;  /* 32 pivots x 128 cols */
        g.a[q] = *reinterpret_cast<const uint4*>(A + (size_t)ra * ld + ca);
        g.b[q] = *reinterpret_cast<const uint4*>(B + (size_t)rb * ld + cb);
    }
}

static __device__ __forceinline__ void fwh_swrite(const fwh_stage_regs& g, uint32_t* __restrict__ sA,
                                                  u16* __restrict__ sB, int tid) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int ia = tid + q * 256, ra = ia & 127, ca = (ia >> 7) * 8;
        const int ib = tid + q * 256, rb = ib >> 4, cb = (ib & 15) * 8;
        const uint4 v = g.a[q];
        uint32_t* d = sA + ((ca >> 1) * 128 + ra) * 2; /* pairs ca/2 .. ca/2+3 of row ra */
        *reinterpret_cast<uint2*>(d) = make_uint2(splat(v.x & 0xFFFFu), splat(v.x >> 16));
        *reinterpret_cast<uint2*>(d + 256) = make_uint2(splat(v.y & 0xFFFFu), splat(v.y >> 16));
        *reinterpret_cast<uint2*>(d + 512) = make_uint2(splat(v.z & 0xFFFFu), splat(v.z >> 16));
        *reinterpret_cast<uint2*>(d + 768) = make_uint2(splat(v.w & 0xFFFFu), splat(v.w >> 16));
        *reinterpret_cast<uint4*>(sB + rb * UBS + cb) = g.b[q];
    }
}

/* SYM: the A slice of tile row I is the pivot panel transposed, A[r][m] = P[m][I0 + r]; a thread
 * loads 8 rows of pivots 2p and 2p+1 (two coalesced 16-B pieces) and writes them pair-major */
static __device__ __forceinline__ void fwh_gload_sym(fwh_stage_regs& g, const u16* __restrict__ Ph,
                                                     int I0, const u16* __restrict__ B, size_t ld,
                                                     int tid) {
    const int p = tid >> 4, rg = tid & 15;
    g.a[0] = *reinterpret_cast<const uint4*>(Ph + (size_t)(2 * p) * ld + I0 + rg * 8);
    g.a[1] = *reinterpret_cast<const uint4*>(Ph + (size_t)(2 * p + 1) * ld + I0 + rg * 8);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int ib = tid + q * 256, rb = ib >> 4, cb = (ib & 15) * 8;
        g.b[q] = *reinterpret_cast<const uint4*>(B + (size_t)rb * ld + cb);
    }
}

static __device__ __forceinline__ void fwh_swrite_sym(const fwh_stage_regs& g,
                                                      uint32_t* __restrict__ sA,
                                                      u16* __restrict__ sB, int tid) {
    const int p = tid >> 4, rg = tid & 15;
    const uint32_t a0[4] = {g.a[0].x, g.a[0].y, g.a[0].z, g.a[0].w}; /* pivot 2p, rows 2i, 2i+1 */
    const uint32_t a1[4] = {g.a[1].x, g.a[1].y, g.a[1].z, g.a[1].w}; /* pivot 2p+1 */
#pragma unroll
    for (int i = 0; i < 4; ++i)
        *reinterpret_cast<uint4*>(sA + ((p * 128) + rg * 8 + 2 * i) * 2) =
            make_uint4(splat(a0[i] & 0xFFFFu), splat(a1[i] & 0xFFFFu), splat(a0[i] >> 16),
                       splat(a1[i] >> 16));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int ib = tid + q * 256, rb = ib >> 4, cb = (ib & 15) * 8;
        *reinterpret_cast<uint4*>(sB + rb * UBS + cb) = g.b[q];
    }
}

/* LDS operand reads: B rows m, m+1 at the thread's 8 columns; A (splat pivots m, m+1) of 4 rows */
/* rows r0..r0+3 of the thread's block, pivots m, m+1: 32 v_add_u32 + 16 v_pk_minimum3_f16 */
template <int R0>
static __device__ __forceinline__ void fwh_rows(uint32_t (&acc)[8][4], const uint2 (&a)[4],
                                                const uint4 (&b)[2]) {
    const uint32_t b0[4] = {b[0].x, b[0].y, b[0].z, b[0].w};
    const uint32_t b1[4] = {b[1].x, b[1].y, b[1].z, b[1].w};
#pragma unroll
    for (int r = 0; r < 4; ++r) relax_row4(acc[R0 + r], a[r].x, a[r].y, b0, b1);
}

#define FWH_PHASE __builtin_amdgcn_sched_barrier(0)
static __device__ __forceinline__ void fwh_stage(uint32_t (&acc)[8][4], const uint32_t* __restrict__ sA,
                                                 const u16* __restrict__ sB, int tx, int ty) {
    const uint32_t* pa0 = sA + ty * 8 * 2; /* rows 0-3 of the thread's block (pair 0) */
    const uint32_t* pa1 = pa0 + 4 * 2;     /* rows 4-7 */
    const u16* pb = sB + tx * 8;
    uint4 B0[2], B1[2];
    uint2 A0[4], A1[4];
    fwh_readB(B0, pb, 0);
    fwh_readA(A0, pa0, 0);
#pragma unroll 1
    for (int m = 0; m < UKC; m += 4) {
        /* every phase issues the reads the next phase needs, then computes on registers that
         * were read one phase earlier (the clamped last reads are harmless re-reads) */
        const int m2 = m + 2, m4 = min(m + 4, UKC - 2);
        fwh_readA(A1, pa1, m);
        FWH_PHASE;
        fwh_rows<0>(acc, A0, B0);
        FWH_PHASE;
        fwh_readB(B1, pb, m2);
        fwh_readA(A0, pa0, m2);
        FWH_PHASE;
        fwh_rows<4>(acc, A1, B0);
        FWH_PHASE;
        fwh_readA(A1, pa1, m2);
        FWH_PHASE;
        fwh_rows<0>(acc, A0, B1);
        FWH_PHASE;
        fwh_readB(B0, pb, m4);
        fwh_readA(A0, pa0, m4);
        FWH_PHASE;
        fwh_rows<4>(acc, A1, B1);
        FWH_PHASE;
    }
}

template <bool SYM, int XM = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void fwh_update_kernel(
    u16* __restrict__ D, int ld, const u16* __restrict__ P, int k0, int ncol_tiles, int i0, int skip,
    const uint32_t* __restrict__ tl, int te) {
    __shared__ __attribute__((aligned(16))) uint32_t sA[UKC / 2 * 128 * 2];
    __shared__ __attribute__((aligned(16))) u16 sB[UKC * UBS];
    if constexpr (XM == 3 || XM == 6 || XM == 7 || XM == 8) FW_CHAIN_PRIO(); /* next-row tiles */
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    int I, J, Iloc;
    if (!fw_tile_of<SYM, XM>(ncol_tiles, i0, skip, tl, te, I, J, Iloc)) return;
    u16* C = D + (size_t)Iloc * 128 * ld + J * 128;
    const u16* Ag = D + (size_t)I * 128 * ld + k0;
    const u16* Bg = P + J * 128;
    fwh_stage_regs g;
    if (SYM)
        fwh_gload_sym(g, P, I * 128, Bg, ld, tid);
    else
        fwh_gload(g, Ag, Bg, ld, tid);
    uint32_t acc[8][4];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const uint4 v = *reinterpret_cast<const uint4*>(C + (size_t)(ty * 8 + r) * ld + tx * 8);
        acc[r][0] = v.x;
        acc[r][1] = v.y;
        acc[r][2] = v.z;
        acc[r][3] = v.w;
    }
    /* unchanged-row test without a 32-VGPR copy of C or a second HBM read of it: values only
     * decrease, so a row changed iff the sum of its eight u16 values decreased (v_dot2_u32_u16) */
    uint32_t sum0[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) sum0[r] = rowsum16(acc[r]);
    if (SYM)
        fwh_swrite_sym(g, sA, sB, tid);
    else
        fwh_swrite(g, sA, sB, tid);
    __syncthreads();
    if (SYM) /* in flight during stage 0 */
        fwh_gload_sym(g, P + (size_t)UKC * ld, I * 128, Bg + (size_t)UKC * ld, ld, tid);
    else
        fwh_gload(g, Ag + UKC, Bg + (size_t)UKC * ld, ld, tid);
    fwh_stage(acc, sA, sB, tx, ty);
    __syncthreads();
    if (SYM)
        fwh_swrite_sym(g, sA, sB, tid);
    else
        fwh_swrite(g, sA, sB, tid);
    __syncthreads();
    fwh_stage(acc, sA, sB, tx, ty);
    /* store only the rows that changed */
#pragma unroll
    for (int r = 0; r < 8; ++r)
        if (rowsum16(acc[r]) != sum0[r])
            *reinterpret_cast<uint4*>(C + (size_t)(ty * 8 + r) * ld + tx * 8) =
                make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
}
