/*
 * fw16.hip -- packed 16-bit blocked Floyd-Warshall for gfx950.
 *
 * Distances are held as u16 quanta, two per 32-bit register, capped at CAP. Two instruction
 * mixes implement the min-plus step (issue costs measured by tools/valu_rate*.hip, 4 waves/SIMD):
 *
 *   FM (f16-compare) path, CAP = 0x3DFF: two pivots per step. One plain v_add_u32 adds a pair of
 *     halves (both <= CAP, so each half-sum <= 0x7BFE: no carry crosses the half boundary), and
 *     one v_pk_minimum3_f16 takes min(acc, t_m, t_m+1) per half. The half-sums are bit patterns
 *     of non-negative finite f16 values (< 0x7C00 = +inf), whose f16 order is their integer
 *     order, denormals included (checked exhaustively-by-sample on the device: 0 mismatches of
 *     4M triples, profiles/r01_valu_issue_rates2.txt). 4 relaxations = 2 adds + 1 min3:
 *     2.48 cycles per relaxation per wave64, against 3.80 for the U path.
 *   U path, CAP = 0x7FFF: one v_add_u32 + one v_pk_min_u16 per 2 relaxations.
 *
 * Both are exact where the true distance is below CAP: every stored value is min(candidate,
 * previous) <= CAP, and min(a,CAP) + min(b,CAP) >= min(a+b, CAP), so the table computed is
 * min(D, CAP) element-wise. If any real pair reaches CAP the build reports inexact and the caller
 * reruns with the next wider path (FM -> U -> u32 kernels) -- the table is never approximate.
 * The A operand is staged pre-splatted, (a, a) per 32-bit LDS word, so the add needs no
 * per-half operand select.
 *
 * Kernels (pivot block KB = 64 rows/cols per round):
 *   fw16_diag    closure of the 64x64 diagonal tile in LDS (64 dependent steps; u16 pk_min, valid
 *                for either CAP since sums of two values <= 0x7FFF fit 16 bits)
 *   fw16_panel   pivot-row panel tiles Dkk* (x) X and pivot-column tiles X (x) Dkk* (64x64)
 *   fw16_update  every 128x128 tile: C <- min(C, A (x) B), A = D[I][k-block], B = P[:, J]
 * The 128x128 update tile gives each of 256 threads an 8x8 block: per pivot step 2 LDS reads
 * (8 B of A, 16 B of B) feed 64 relaxations (0.5 B/relax, vs 2 B/relax for the u32 4x4 tile).
 */
#include "srt_device.h"

typedef unsigned short u16;
typedef u16 u16x2 __attribute__((ext_vector_type(2)));

#define KB 64
#define CAP_U 0x7FFFu /* cap of the U path (v_pk_min_u16) */
/* kernels on the round-to-round critical chain (next pivot block's tiles, diagonal closure,
 * panel, panel assembly) raise their waves' issue priority above the bulk update's, which
 * shares every SIMD with them; stream priority alone only orders dispatch */
#define FW_CHAIN_PRIO() __builtin_amdgcn_s_setprio(3)
#define CAP_F 0x3DFFu /* cap of the FM path: 2 * CAP_F < 0x7C00 (f16 +inf) */
#define LDA16 (KB + 8) /* u16 stride of an A row in LDS: 144 B, 16-byte aligned */
#define UKC 32          /* pivots per LDS stage in the update kernel (two stages per launch) */

static __device__ __forceinline__ u16x2 as2(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
static __device__ __forceinline__ uint32_t as32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
static __device__ __forceinline__ uint32_t splat(uint32_t h) { return h | (h << 16); }
/* per half: min(acc, x, y) on u16 bit patterns in [0, 0x7BFF] -> one v_pk_minimum3_f16.
 * Inline asm: written with the generic minimum builtins, LLVM re-associates the chain across
 * pivot pairs into two-input minimum3s with a duplicated operand (1.5x the min instructions). */
/* (the plain-C row step's instruction mix of the A/B builds in tools/) */
__attribute__((unused)) static __device__ __forceinline__ uint32_t min3h(uint32_t acc, uint32_t x,
                                                                         uint32_t y) {
    uint32_t r;
    asm("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(acc), "v"(x), "v"(y));
    return r;
}
/* acc = min(acc, a0 + b0, a1 + b1) per half as one fixed add, add, s_nop 0, min3 group. A packed
 * (VOP3P) instruction issued right after the VALU write of its operand is held by the hardware
 * interlock, which stalls the SIMD; one s_nop 0 in that wave lets the other waves issue instead:
 * the update's instruction stream runs at 85.7% of the issue model with it against 67.6% without
 * (tools/valu_banks.hip, 8 waves per SIMD; VGPR bank placement measured no effect). Left to the
 * scheduler, the adds of a row pair are also hoisted ahead of their mins (5% slower). */
static __device__ __forceinline__ uint32_t relax2h(uint32_t acc, uint32_t a0, uint32_t b0, uint32_t a1,
                                                   uint32_t b1) {
    uint32_t t0, t1;
    asm("v_add_u32 %1, %3, %4\n\tv_add_u32 %2, %5, %6\n\ts_nop 0\n\tv_pk_minimum3_f16 %0, %0, %1, %2"
        : "+v"(acc), "=&v"(t0), "=&v"(t1)
        : "v"(a0), "v"(b0), "v"(a1), "v"(b1));
    return acc;
}
/* acc = min(acc, a + b) per half on the U path (v_pk_min_u16), with the same s_nop 0 before the
 * packed min */
static __device__ __forceinline__ uint32_t relax1u(uint32_t acc, uint32_t a, uint32_t b) {
    uint32_t t;
    asm("v_add_u32 %1, %2, %3\n\ts_nop 0\n\tv_pk_min_u16 %0, %0, %1" : "+v"(acc), "=&v"(t) : "v"(a), "v"(b));
    return acc;
}
/* relax2h over a thread-row of four words in one block, each triple with its own temporaries (no
 * false dependence between consecutive triples through reused registers) */
static __device__ __forceinline__ void relax_row4(uint32_t (&acc)[4], uint32_t a0, uint32_t a1,
                                                  const uint32_t (&b0)[4], const uint32_t (&b1)[4]) {
    uint32_t t0, t1, t2, t3, t4, t5, t6, t7;
    asm("v_add_u32 %4, %12, %14\n\tv_add_u32 %5, %13, %18\n\ts_nop 0\n\tv_pk_minimum3_f16 %0, %0, %4, %5\n\t"
        "v_add_u32 %6, %12, %15\n\tv_add_u32 %7, %13, %19\n\ts_nop 0\n\tv_pk_minimum3_f16 %1, %1, %6, %7\n\t"
        "v_add_u32 %8, %12, %16\n\tv_add_u32 %9, %13, %20\n\ts_nop 0\n\tv_pk_minimum3_f16 %2, %2, %8, %9\n\t"
        "v_add_u32 %10, %12, %17\n\tv_add_u32 %11, %13, %21\n\ts_nop 0\n\tv_pk_minimum3_f16 %3, %3, %10, %11"
        : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "=&v"(t0), "=&v"(t1), "=&v"(t2),
          "=&v"(t3), "=&v"(t4), "=&v"(t5), "=&v"(t6), "=&v"(t7)
        : "v"(a0), "v"(a1), "v"(b0[0]), "v"(b0[1]), "v"(b0[2]), "v"(b0[3]), "v"(b1[0]), "v"(b1[1]),
          "v"(b1[2]), "v"(b1[3]));
}
template <int I>
static __device__ __forceinline__ uint32_t lane4(const uint4& v) {
    if constexpr (I == 0) return v.x;
    else if constexpr (I == 1) return v.y;
    else if constexpr (I == 2) return v.z;
    else return v.w;
}

/* ---- staging ------------------------------------------------------------------------------ */
/* A (TM rows x KC pivots) into LDS as (a, a) words: row r, pivot m at sA[r * (KC + 4) + m]
 * (row stride 16-byte aligned, offset by 4 banks per row) */
template <int TM, int KC>
__device__ __forceinline__ void stage_A(uint32_t* __restrict__ sA, const u16* __restrict__ g,
                                        size_t ldg, int tid) {
    constexpr int PER = KC / 8; /* uint4 per row */
    for (int idx = tid; idx < TM * PER; idx += 256) {
        const int row = idx / PER, c8 = (idx % PER) * 8;
        const uint4 v = *reinterpret_cast<const uint4*>(g + (size_t)row * ldg + c8);
        uint32_t* d = sA + row * (KC + 4) + c8;
        *reinterpret_cast<uint4*>(d) = make_uint4(splat(v.x & 0xFFFFu), splat(v.x >> 16),
                                                  splat(v.y & 0xFFFFu), splat(v.y >> 16));
        *reinterpret_cast<uint4*>(d + 4) = make_uint4(splat(v.z & 0xFFFFu), splat(v.z >> 16),
                                                      splat(v.w & 0xFFFFu), splat(v.w >> 16));
    }
}

/* B (KC pivot rows x TN columns) into LDS as packed u16 pairs */
template <int TN, int KC>
__device__ __forceinline__ void stage_B(u16* __restrict__ sB, const u16* __restrict__ g, size_t ldg,
                                        int tid) {
    constexpr int LDB = TN + 8;
    constexpr int PER = TN / 8;
    for (int idx = tid; idx < KC * PER; idx += 256) {
        const int row = idx / PER, c8 = (idx % PER) * 8;
        *reinterpret_cast<uint4*>(sB + row * LDB + c8) =
            *reinterpret_cast<const uint4*>(g + (size_t)row * ldg + c8);
    }
}

/* ---- register-blocked min-plus over KC staged pivots ---------------------------------------- */
template <bool FM, int MM, int RN>
__device__ __forceinline__ void step_rows(u16x2 (&acc)[RN / 2], u16x2 (&acc1)[RN / 2], const uint4& a0,
                                          const uint4& a1, const uint32_t (&bv)[4][RN / 2]) {
    if constexpr (FM) {
        /* pivots MM, MM+1: two adds per column pair and row, one 3-input min */
#pragma unroll
        for (int c = 0; c < RN / 2; ++c) {
            acc[c] = as2(relax2h(as32(acc[c]), lane4<MM>(a0), bv[MM][c], lane4<MM + 1>(a0), bv[MM + 1][c]));
            acc1[c] = as2(relax2h(as32(acc1[c]), lane4<MM>(a1), bv[MM][c], lane4<MM + 1>(a1), bv[MM + 1][c]));
        }
    } else {
        /* one pivot at a time, two rows: RN independent adds, then RN mins */
#pragma unroll
        for (int mm = MM; mm < MM + 2; ++mm) {
            const uint32_t s0 = mm == MM ? lane4<MM>(a0) : lane4<MM + 1>(a0);
            const uint32_t s1 = mm == MM ? lane4<MM>(a1) : lane4<MM + 1>(a1);
#pragma unroll
            for (int c = 0; c < RN / 2; ++c) {
                acc[c] = as2(relax1u(as32(acc[c]), s0, bv[mm][c]));
                acc1[c] = as2(relax1u(as32(acc1[c]), s1, bv[mm][c]));
            }
        }
    }
}

template <bool FM, int TN, int RM, int RN, int KC>
__device__ __forceinline__ void mp16(u16x2 (&acc)[RM][RN / 2], const uint32_t* __restrict__ sA,
                                     const u16* __restrict__ sB, int tx, int ty) {
    constexpr int LDB = TN + 8, LDA = KC + 4;
    const uint32_t* pa = sA + ty * RM * LDA;
    const u16* pb = sB + tx * RN;
#pragma unroll 1
    for (int m = 0; m < KC; m += 4) {
        uint32_t bv[4][RN / 2]; /* packed B pairs of pivots m..m+3 */
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
            if constexpr (RN == 8) {
                uint4 v = *reinterpret_cast<const uint4*>(pb + (m + mm) * LDB);
                bv[mm][0] = v.x;
                bv[mm][1] = v.y;
                bv[mm][2] = v.z;
                bv[mm][3] = v.w;
            } else {
                uint2 v = *reinterpret_cast<const uint2*>(pb + (m + mm) * LDB);
                bv[mm][0] = v.x;
                bv[mm][1] = v.y;
            }
        }
        /* rows in groups of four: (a, a) words of pivots m..m+3, one b128 read per row */
#pragma unroll
        for (int rg = 0; rg < RM; rg += 4) {
            uint4 av[4];
#pragma unroll
            for (int r = 0; r < 4; ++r)
                av[r] = *reinterpret_cast<const uint4*>(pa + (rg + r) * LDA + m);
#pragma unroll
            for (int r = 0; r < 4; r += 2) {
                step_rows<FM, 0, RN>(acc[rg + r], acc[rg + r + 1], av[r], av[r + 1], bv);
                step_rows<FM, 2, RN>(acc[rg + r], acc[rg + r + 1], av[r], av[r + 1], bv);
            }
        }
    }
}

template <int RM, int RN>
__device__ __forceinline__ void load_acc16(u16x2 (&acc)[RM][RN / 2], const u16* __restrict__ C,
                                           size_t ldc, int tx, int ty) {
#pragma unroll
    for (int r = 0; r < RM; ++r) {
        const u16* p = C + (size_t)(ty * RM + r) * ldc + tx * RN;
        if constexpr (RN == 8) {
            uint4 v = *reinterpret_cast<const uint4*>(p);
            acc[r][0] = as2(v.x);
            acc[r][1] = as2(v.y);
            acc[r][2] = as2(v.z);
            acc[r][3] = as2(v.w);
        } else {
            uint2 v = *reinterpret_cast<const uint2*>(p);
            acc[r][0] = as2(v.x);
            acc[r][1] = as2(v.y);
        }
    }
}

/* store only the rows of the thread block that changed (unchanged tiles cost no HBM write) */
template <int RM, int RN>
__device__ __forceinline__ void store_acc16(const u16x2 (&acc)[RM][RN / 2],
                                            const u16x2 (&old)[RM][RN / 2], u16* __restrict__ C,
                                            size_t ldc, int tx, int ty) {
#pragma unroll
    for (int r = 0; r < RM; ++r) {
        bool ch = false;
#pragma unroll
        for (int c = 0; c < RN / 2; ++c) ch |= as32(acc[r][c]) != as32(old[r][c]);
        if (!ch) continue;
        u16* p = C + (size_t)(ty * RM + r) * ldc + tx * RN;
        if constexpr (RN == 8)
            *reinterpret_cast<uint4*>(p) =
                make_uint4(as32(acc[r][0]), as32(acc[r][1]), as32(acc[r][2]), as32(acc[r][3]));
        else
            *reinterpret_cast<uint2*>(p) = make_uint2(as32(acc[r][0]), as32(acc[r][1]));
    }
}

/* ---- kernels --------------------------------------------------------------------------------- */
/* 8 columns per thread (ld is a multiple of 128): two 16-B loads of w, one 16-B store of d */
__global__ void fw16_init_kernel(int n, int ld, int row0, const uint32_t* __restrict__ w,
                                 u16* __restrict__ d, uint32_t cap) {
    const int j8 = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
    const int i = row0 + blockIdx.y;
    if (j8 >= ld) return;
    const size_t ix = (size_t)blockIdx.y * ld + j8;
    uint32_t x[8];
    if (i < n && j8 + 8 <= n) {
        const uint4 a = *reinterpret_cast<const uint4*>(w + ix);
        const uint4 b = *reinterpret_cast<const uint4*>(w + ix + 4);
        x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
        x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
    } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] = (i < n && j8 + q < n) ? w[ix + q] : cap;
    }
    uint32_t o[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t lo = (i == j8 + 2 * q) ? 0u : min(x[2 * q], cap);
        const uint32_t hi = (i == j8 + 2 * q + 1) ? 0u : min(x[2 * q + 1], cap);
        o[q] = lo | (hi << 16);
    }
    *reinterpret_cast<uint4*>(d + ix) = make_uint4(o[0], o[1], o[2], o[3]);
}

/* Closure of the 64x64 block in LDS (stride LDA16, zero diagonal) by in-place min-plus squaring,
 * D <- min(D, D (x) D), until a pass changes nothing -- at most 6 passes (a simple path inside
 * the block has <= 63 hops; after pass t every path of <= 2^t hops is covered). Every value read
 * or written is the length of a real path inside the block (u16 sums of two values <= CAP never
 * carry across halves), so entries read while a neighbour writes its new (smaller) values only
 * speed convergence; a pass that changes nothing leaves D = min(D, D (x) D), which with the zero
 * diagonal is the closure -- the same matrix as 64 dependent FW steps, in ~3-4 barriers instead
 * of 64 (the block's shortest paths have few hops: C4's trees are <= 5 deep). 4x4 per thread. */
template <bool FM>
static __device__ __forceinline__ void close64(u16* __restrict__ s, int tid) {
    const int tx = tid & 15, ty = tid >> 4;
#pragma unroll 1
    for (int pass = 0; pass < 6; ++pass) {
        uint2 acc[4], old[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) old[r] = acc[r] = *reinterpret_cast<const uint2*>(s + (4 * ty + r) * LDA16 + 4 * tx);
#pragma unroll 2
        for (int m = 0; m < KB; m += 4) {
            uint2 a[4], b[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] = *reinterpret_cast<const uint2*>(s + (4 * ty + r) * LDA16 + m);
#pragma unroll
            for (int q = 0; q < 4; ++q) b[q] = *reinterpret_cast<const uint2*>(s + (m + q) * LDA16 + 4 * tx);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t p[4] = {splat(a[r].x & 0xFFFFu), splat(a[r].x >> 16),
                                       splat(a[r].y & 0xFFFFu), splat(a[r].y >> 16)};
                if constexpr (FM) {
#pragma unroll
                    for (int q = 0; q < 4; q += 2) {
                        acc[r].x = relax2h(acc[r].x, p[q], b[q].x, p[q + 1], b[q + 1].x);
                        acc[r].y = relax2h(acc[r].y, p[q], b[q].y, p[q + 1], b[q + 1].y);
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        acc[r].x = relax1u(acc[r].x, p[q], b[q].x);
                        acc[r].y = relax1u(acc[r].y, p[q], b[q].y);
                    }
                }
            }
        }
        int ch = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (acc[r].x != old[r].x || acc[r].y != old[r].y) {
                ch = 1;
                *reinterpret_cast<uint2*>(s + (4 * ty + r) * LDA16 + 4 * tx) = acc[r];
            }
        if (!__syncthreads_or(ch)) break;
    }
}

/* closure of the diagonal tile in LDS (close64) */
template <bool FM>
__global__ __launch_bounds__(256) void fw16_diag_kernel(u16* __restrict__ P, int ld, int k0) {
    __shared__ __attribute__((aligned(16))) u16 s[KB * LDA16];
    FW_CHAIN_PRIO();
    const int tid = threadIdx.x;
    u16* T = P + k0;
    for (int idx = tid; idx < KB * 8; idx += 256) {
        const int row = idx >> 3, c8 = (idx & 7) * 8;
        *reinterpret_cast<uint4*>(s + row * LDA16 + c8) =
            *reinterpret_cast<const uint4*>(T + (size_t)row * ld + c8);
    }
    __syncthreads();
    close64<FM>(s, tid);
    for (int idx = tid; idx < KB * 8; idx += 256) {
        const int row = idx >> 3, c8 = (idx & 7) * 8;
        *reinterpret_cast<uint4*>(T + (size_t)row * ld + c8) =
            *reinterpret_cast<const uint4*>(s + row * LDA16 + c8);
    }
}

/* pivot-row panel tiles (k, j): X <- Dkk* (x) X ; pivot-column tiles (i, k): X <- X (x) Dkk* */
/* SYM (undirected graphs, one shard): only upper-triangle panel tiles -- row tiles right of the
 * pivot block and column tiles above it -- are kept; fw16_refresh_kernel mirrors the column tiles
 * into the lower part of the pivot rows so P is a full panel. */
template <bool FM, bool SYM>
__global__ __launch_bounds__(256) void fw16_panel_kernel(u16* __restrict__ D, int ld, int row0,
                                                         int nrow_tiles, u16* __restrict__ P, int k0,
                                                         int ncol_tiles, int do_row, int do_col) {
    __shared__ __attribute__((aligned(16))) uint32_t sA[KB * (KB + 4)];
    __shared__ __attribute__((aligned(16))) u16 sB[KB * (KB + 8)];
    FW_CHAIN_PRIO();
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    int bid = blockIdx.x;
    u16* C;
    if (bid < ncol_tiles) {
        if (!do_row || bid * KB == k0 || (SYM && bid * KB < k0)) return;
        C = P + bid * KB;
        stage_A<KB, KB>(sA, P + k0, ld, tid);
        stage_B<KB, KB>(sB, C, ld, tid);
    } else {
        bid -= ncol_tiles;
        if (!do_col || bid >= nrow_tiles || row0 + bid * KB == k0 || (SYM && row0 + bid * KB > k0))
            return;
        C = D + (size_t)bid * KB * ld + k0;
        stage_A<KB, KB>(sA, C, ld, tid);
        stage_B<KB, KB>(sB, P + k0, ld, tid);
    }
    u16x2 old[4][2], acc[4][2];
    load_acc16<4, 4>(old, C, ld, tx, ty);
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 2; ++c) acc[r][c] = old[r][c];
    mp16<FM, KB, 4, 4, KB>(acc, sA, sB, tx, ty);
    store_acc16<4, 4>(acc, old, C, ld, tx, ty);
}

/* SYM: pivot rows' lower part from the (upper) column tiles: D[k0+m][j0+c] = D[j0+c][k0+m] */
__global__ __launch_bounds__(256) void fw16_refresh_kernel(u16* __restrict__ D, int ld, int k0) {
    __shared__ u16 t[KB][KB + 2];
    FW_CHAIN_PRIO();
    const int j0 = blockIdx.x * KB, tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    u16 v[KB / 4]; /* all loads in flight before the LDS stores */
#pragma unroll
    for (int q = 0; q < KB / 4; ++q) v[q] = D[(size_t)(j0 + ty + 4 * q) * ld + k0 + tx];
#pragma unroll
    for (int q = 0; q < KB / 4; ++q) t[ty + 4 * q][tx] = v[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < KB / 4; ++q) D[(size_t)(k0 + ty + 4 * q) * ld + j0 + tx] = t[tx][ty + 4 * q];
}

/* SYM, after the last round: lower triangle from the upper, 64x64 tiles (I > J) */
__global__ __launch_bounds__(256) void fw16_mirror_kernel(u16* __restrict__ D, int ld) {
    __shared__ u16 t[KB][KB + 2];
    const int I = blockIdx.y, J = blockIdx.x;
    if (I <= J) return;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    u16 v[KB / 4];
#pragma unroll
    for (int q = 0; q < KB / 4; ++q) v[q] = D[(size_t)(J * KB + ty + 4 * q) * ld + I * KB + tx];
#pragma unroll
    for (int q = 0; q < KB / 4; ++q) t[ty + 4 * q][tx] = v[q];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < KB / 4; ++q) D[(size_t)(I * KB + ty + 4 * q) * ld + J * KB + tx] = t[tx][ty + 4 * q];
}

/* every 128x128 tile of the local rows: D_IJ <- min(D_IJ, D_I,k (x) P_k,J) */
/* Tile rows: I = i0 + bid / ncol_tiles, skipping tile row `skip` (-1: none) -- the lookahead
 * schedule updates the next pivot block's tile row first and the others after it. */
static __device__ __forceinline__ int tile_row(int bid, int ncol_tiles, int i0, int skip) {
    const int I = i0 + bid / ncol_tiles;
    return (skip >= 0 && I >= skip) ? I + 1 : I;
}

template <bool FM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void fw16_update_kernel(u16* __restrict__ D, int ld,
                                                          const u16* __restrict__ P, int k0,
                                                          int ncol_tiles, int i0, int skip,
                                                          const uint32_t* __restrict__ /*tl*/,
                                                          int /*te*/) {
    __shared__ __attribute__((aligned(16))) uint32_t sA[128 * (UKC + 4)];
    __shared__ __attribute__((aligned(16))) u16 sB[UKC * (128 + 8)];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    /* XCD-aware order: consecutive blocks land on different XCDs; give each XCD a contiguous run
     * of tiles in a row band so its L2 keeps the band's A slice and the panel columns. */
    const int nb = gridDim.x;
    const int per = nb >> 3;
    const int bid = (nb & 7) == 0 ? (blockIdx.x & 7) * per + (blockIdx.x >> 3) : blockIdx.x;
    const int I = tile_row(bid, ncol_tiles, i0, skip), J = bid % ncol_tiles;
    u16* C = D + (size_t)I * 128 * ld + J * 128;
    u16x2 old[8][4], acc[8][4];
    load_acc16<8, 8>(old, C, ld, tx, ty); /* HBM reads in flight during the staging */
#pragma unroll
    for (int h = 0; h < KB; h += UKC) {
        /* two 32-pivot stages keep LDS at 27 KB per block (4 blocks per CU) */
        if (h) __syncthreads();
        stage_A<128, UKC>(sA, D + (size_t)I * 128 * ld + k0 + h, ld, tid);
        stage_B<128, UKC>(sB, P + (size_t)h * ld + J * 128, ld, tid);
        __syncthreads();
        if (!h) {
#pragma unroll
            for (int r = 0; r < 8; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[r][c] = old[r][c];
        }
        mp16<FM, 128, 8, 8, UKC>(acc, sA, sB, tx, ty);
    }
    store_acc16<8, 8>(acc, old, C, ld, tx, ty);
}

/* ---- f16-compare update, software-pipelined ------------------------------------------------ *
 * Same tile as fw16_update_kernel<true> (128x128 outputs, 8x8 per thread, two 32-pivot stages)
 * with the latencies taken off the critical path:
 *   - the next stage's A/B slices are loaded into registers while the current stage computes;
 *   - LDS operands of pivot pair p+1 are read while pair p computes (double-buffered registers);
 *   - the unchanged-row test compares per-row sums of the u16 values (8 VGPRs) instead of
 *     holding a copy of C in 32 VGPRs or reading it again from HBM.
 * Per pivot pair and thread: 2 ds_read_b128 (B, 8 columns x 2 pivots) + 4 ds_read_b128 (A, 8 rows
 * x 2 splatted pivots) feed 64 v_add_u32 + 32 v_pk_minimum3_f16 = 128 relaxations.
 * A is laid out pivot-pair-major in LDS: word pair (splat A[r][2p], splat A[r][2p+1]) at
 * sA[(p * 128 + r) * 2], so a thread's 4 consecutive rows are one 32-byte run (two full-rate
 * ds_read_b128; a row-major A makes the compiler pair the reads into half-rate ds_read2_b64). */
#define UBS (128 + 8) /* B row stride in LDS u16 */

typedef unsigned short us2 __attribute__((ext_vector_type(2)));
/* sum of the eight u16 values of a thread-row (four packed words): 4 x v_dot2_u32_u16 */
static __device__ __forceinline__ uint32_t rowsum16(const uint32_t (&w)[4]) {
    const us2 one = {1, 1};
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) s = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, w[c]), one, s, false);
    return s;
}


/* upper-triangle tile (I <= J) of linear index x among T tile rows: row I holds T - I tiles */
static __device__ __forceinline__ void tri_decode(int x, int T, int* I, int* J) {
    auto off = [T](int i) { return i * T - (i * (i - 1)) / 2; };
    const double tt = T + 0.5;
    int i = (int)(tt - sqrt(tt * tt - 2.0 * x));
    i = max(0, min(i, T - 1));
    while (i > 0 && off(i) > x) --i;
    while (i + 1 < T && off(i + 1) <= x) ++i;
    *I = i;
    *J = i + (x - off(i));
}



/* Row-sharded symmetric rounds: of the tile pair (I, J) / (J, I), I != J, the rank owning row I
 * keeps (I, J) when I < J and I + J is even, or I > J and I + J is odd; the other one is its
 * transpose, filled in at the end. Every rank then holds about half of its row block's tiles,
 * whatever its position. */
static __host__ __device__ __forceinline__ bool sym_kept(int I, int J) {
    return I == J || ((I < J) == (((I + J) & 1) == 0));
}

/* SYM: only upper-triangle tiles (I <= J, grid T(T+1)/2) -- an undirected graph's distance
 * matrix stays symmetric through every round, so the lower triangle is the transpose and half the
 * relaxations are skipped; A comes from the pivot panel transposed.
 * XM (row-sharded SYM, D = the rank's rows from tile row i0 = tb, te = end tile row, skip = the
 * tile row K1 of the next pivot block or -1): 3 = the kept tiles of tile row K1 (block b < T: J =
 * b) and of tile column K1 in the rank's rows (b >= T: I = tb + b - T), which the next pivot
 * panel is assembled from; 4 = the rank's kept-tile list tl minus those; 5 = the whole list;
 * 6 = (one GPU, two update streams) the upper-triangle tiles of tile row / column K1 whose
 * I + J has the parity i0; 7 / 8 = mode 3 restricted to even / odd J (the sharded rounds' two
 * update streams). */
/* The tile (I, J) the calling block of a mode-XM launch updates and its local tile row Iloc;
 * false when the block has nothing to do (the modes: the comment above). */
template <bool SYM, int XM>
static __device__ __forceinline__ bool fw_tile_of(int ncol_tiles, int i0, int skip,
                                                  const uint32_t* __restrict__ tl, int te, int& I,
                                                  int& J, int& Iloc) {
    const int nb = gridDim.x;
    const int per = nb >> 3;
    const int bid = (nb & 7) == 0 ? (blockIdx.x & 7) * per + (blockIdx.x >> 3) : blockIdx.x;
    if (XM == 3 || XM == 7 || XM == 8) {
        if (blockIdx.x < ncol_tiles) {
            J = blockIdx.x;
            I = skip;
            if (I < i0 || I >= te || !sym_kept(I, J)) return false;
        } else {
            I = i0 + (int)blockIdx.x - ncol_tiles;
            J = skip;
            if (I >= te || I == skip || !sym_kept(I, J)) return false;
        }
        if (XM != 3 && (J & 1) != XM - 7) return false; /* two update streams: tile set J mod 2 */
        Iloc = I - i0;
    } else if (XM == 6) { /* one GPU, upper triangle: the cross of K1 restricted to I + J = i0 mod 2 */
        I = min((int)blockIdx.x, skip);
        J = max((int)blockIdx.x, skip);
        if (((I + J) & 1) != i0) return false;
        Iloc = I;
    } else if (XM == 4 || XM == 5) {
        const uint32_t t = tl[bid];
        I = (int)(t >> 16);
        J = (int)(t & 0xFFFFu);
        if (XM == 4 && (I == skip || J == skip)) return false;
        Iloc = I - i0;
    } else if (SYM) {
        tri_decode(bid, ncol_tiles, &I, &J);
        Iloc = I;
    } else {
        I = tile_row(bid, ncol_tiles, i0, skip);
        J = bid % ncol_tiles;
        Iloc = I;
    }
    return true;
}


/* LDS operand reads of the update tile (A: 4 x u16 pairs, B: 2 x 8 u16) */
static __device__ __forceinline__ void fwh_readB(uint4 (&b)[2], const u16* __restrict__ pb, int m) {
    b[0] = *reinterpret_cast<const uint4*>(pb + m * UBS);
    b[1] = *reinterpret_cast<const uint4*>(pb + (m + 1) * UBS);
}
static __device__ __forceinline__ void fwh_readA(uint2 (&a)[4], const uint32_t* __restrict__ pa, int m) {
    const uint4 q0 = *reinterpret_cast<const uint4*>(pa + (m >> 1) * 256);
    const uint4 q1 = *reinterpret_cast<const uint4*>(pa + (m >> 1) * 256 + 4);
    a[0] = make_uint2(q0.x, q0.y);
    a[1] = make_uint2(q0.z, q0.w);
    a[2] = make_uint2(q1.x, q1.y);
    a[3] = make_uint2(q1.z, q1.w);
}

/* ---- the same update at 8 waves per SIMD --------------------------------------------------- *
 * 512 threads per 128x128 tile, 4 rows x 8 columns per thread: 16 accumulator VGPRs, <= 64 in
 * all, so 8 waves share each SIMD (4 for fwh_update_kernel's 8x8 blocks at 119 VGPRs). The
 * f16-compare mix issues at 2.29 cycles per relaxation with 8 waves against 2.48 with 4
 * (profiles/r01_valu_issue_rates2.txt), and the tile's C load, staging and stores are spread
 * over twice the waves. Per pivot pair and thread: 2 ds_read_b128 of B + 2 of A feed 32 v_add_u32
 * + 16 v_pk_minimum3_f16 (LDS: 4 ds_read_b128 per 64 relaxations, 44% of the array's rate at
 * the VALU issue rate). Same LDS image, modes and results as fwh_update_kernel
 * (tools/fwh_variants.hip: 67.3% vs 64.2% of the issue model on a full 32k update). */
struct fwq_stage_regs {
    uint4 a, b; /* SYM: a = (pivot 2p rows 4g..4g+3, pivot 2p+1 rows 4g..4g+3) */
};

static __device__ __forceinline__ void fwq_gload(fwq_stage_regs& g, const u16* __restrict__ A,
                                                 const u16* __restrict__ B, size_t ld, int tid) {
    const int ra = tid & 127, ca = (tid >> 7) * 8; /* 128 rows x 32 pivots */
    const int rb = tid >> 4, cb = (tid & 15) * 8;  /* 32 pivots x 128 columns */
    g.a = *reinterpret_cast<const uint4*>(A + (size_t)ra * ld + ca);
    g.b = *reinterpret_cast<const uint4*>(B + (size_t)rb * ld + cb);
}

static __device__ __forceinline__ void fwq_gload_sym(fwq_stage_regs& g, const u16* __restrict__ Ph,
                                                     int I0, const u16* __restrict__ B, size_t ld,
                                                     int tid) {
    const int p = tid >> 5, rg = tid & 31;
    const uint2 a0 = *reinterpret_cast<const uint2*>(Ph + (size_t)(2 * p) * ld + I0 + rg * 4);
    const uint2 a1 = *reinterpret_cast<const uint2*>(Ph + (size_t)(2 * p + 1) * ld + I0 + rg * 4);
    g.a = make_uint4(a0.x, a0.y, a1.x, a1.y);
    const int rb = tid >> 4, cb = (tid & 15) * 8;
    g.b = *reinterpret_cast<const uint4*>(B + (size_t)rb * ld + cb);
}

template <bool SYM>
static __device__ __forceinline__ void fwq_swrite(const fwq_stage_regs& g, uint32_t* __restrict__ sA,
                                                  u16* __restrict__ sB, int tid) {
    if constexpr (SYM) {
        const int p = tid >> 5, rg = tid & 31;
        const uint32_t a0[2] = {g.a.x, g.a.y}, a1[2] = {g.a.z, g.a.w};
#pragma unroll
        for (int i = 0; i < 2; ++i) /* rows 4rg + 2i (low halves) and 4rg + 2i + 1 (high) */
            *reinterpret_cast<uint4*>(sA + ((p * 128) + rg * 4 + 2 * i) * 2) =
                make_uint4(splat(a0[i] & 0xFFFFu), splat(a1[i] & 0xFFFFu), splat(a0[i] >> 16),
                           splat(a1[i] >> 16));
    } else {
        const int ra = tid & 127, ca = (tid >> 7) * 8;
        const uint4 v = g.a;
        uint32_t* d = sA + ((ca >> 1) * 128 + ra) * 2; /* pairs ca/2 .. ca/2+3 of row ra */
        *reinterpret_cast<uint2*>(d) = make_uint2(splat(v.x & 0xFFFFu), splat(v.x >> 16));
        *reinterpret_cast<uint2*>(d + 256) = make_uint2(splat(v.y & 0xFFFFu), splat(v.y >> 16));
        *reinterpret_cast<uint2*>(d + 512) = make_uint2(splat(v.z & 0xFFFFu), splat(v.z >> 16));
        *reinterpret_cast<uint2*>(d + 768) = make_uint2(splat(v.w & 0xFFFFu), splat(v.w >> 16));
    }
    const int rb = tid >> 4, cb = (tid & 15) * 8;
    *reinterpret_cast<uint4*>(sB + rb * UBS + cb) = g.b;
}

/* rows 0..3 of the thread's 4x8 block, pivots m, m+1: 32 v_add_u32 + 16 v_pk_minimum3_f16, one
 * asm block per row (relax_row4; the fixed-triple and plain-C forms measured slower, §5.1) */
static __device__ __forceinline__ void fwq_rows(uint32_t (&acc)[4][4], const uint2 (&a)[4],
                                                const uint4 (&b)[2]) {
    const uint32_t b0[4] = {b[0].x, b[0].y, b[0].z, b[0].w};
    const uint32_t b1[4] = {b[1].x, b[1].y, b[1].z, b[1].w};
#pragma unroll
    for (int r = 0; r < 4; ++r) relax_row4(acc[r], a[r].x, a[r].y, b0, b1);
}

static __device__ __forceinline__ void fwq_stage(uint32_t (&acc)[4][4], const uint32_t* __restrict__ sA,
                                                 const u16* __restrict__ sB, int tx, int ty) {
    const uint32_t* pa = sA + ty * 4 * 2;
    const u16* pb = sB + tx * 8;
    /* no register double-buffering (it spills at 64 VGPRs): the other 7 waves of the SIMD hide the
     * LDS latency */
#pragma unroll 2
    for (int m = 0; m < UKC; m += 2) {
        uint4 b[2];
        uint2 a[4];
        fwh_readB(b, pb, m);
        fwh_readA(a, pa, m);
        fwq_rows(acc, a, b);
    }
}

/* NST stages of UKC pivots per C-tile residency: 2 (a 64-pivot round), 4 (the 128-row panel
 * P = P_a over P_b) or 8 (256 rows, P_a..P_d). prev >= 0: the cross tiles the chain stream updated
 * while closing the round's later panels start past them -- 128-pivot rounds: the cross of prev
 * holds P_a; 256-pivot rounds: the cross of prev + 1 holds P_a..P_c, the rest of the cross of prev
 * holds P_a. (Applying a panel a tile already took is harmless -- min-plus with the same operands
 * is idempotent -- so the small cross launches do not track it.)
 * XM 9: the cross of tile `skip` (tile row and column, upper triangle), every tile.
 * XM 13: the cross of tiles skip and skip + 1 whose I + J has the parity i0 (256-pivot rounds:
 * the next round's two pivot tile rows). XM 4 with NST 8 leaves out both crosses. */
template <bool SYM, int XM = 0, int NST = 2>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8, 8))) void fwq_update_kernel(
    u16* __restrict__ D, int ld, const u16* __restrict__ P, int k0, int ncol_tiles, int i0, int skip,
    const uint32_t* __restrict__ tl, int te, int prev = -1, u16* __restrict__ outq = nullptr) {
    __shared__ __attribute__((aligned(16))) uint32_t sA[UKC / 2 * 128 * 2];
    __shared__ __attribute__((aligned(16))) u16 sB[UKC * UBS];
    if constexpr (XM == 3 || XM == 6 || XM == 7 || XM == 8 || XM == 9 || XM == 13)
        FW_CHAIN_PRIO(); /* next-row tiles */
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    int I, J, Iloc;
    int q20 = 0;
    if constexpr (XM == 20) {
        /* split-k squaring (ld <= 2048): tile (I, J) x pivot block q of NST * UKC pivots from
         * k0, C read from D, min(C, A (x) B) written whole to outq's slice q */
        const int tiles = ncol_tiles * ncol_tiles;
        const int bid = (int)blockIdx.x % tiles;
        q20 = (int)blockIdx.x / tiles;
        I = bid / ncol_tiles;
        J = bid % ncol_tiles;
        Iloc = I;
        k0 += q20 * NST * UKC;
        P = D + (size_t)k0 * ld;
    } else if constexpr (XM == 9) {
        I = min((int)blockIdx.x, skip);
        J = max((int)blockIdx.x, skip);
        Iloc = I;
    } else if constexpr (XM == 13) {
        const int b = (int)blockIdx.x, second = b >= ncol_tiles;
        const int c = second ? b - ncol_tiles : b, k = skip + second;
        if (second && c == skip) return; /* (skip, skip + 1) is in the first set */
        I = min(c, k);
        J = max(c, k);
        if (((I + J) & 1) != i0) return;
        Iloc = I;
    } else if (!fw_tile_of<SYM, XM>(ncol_tiles, i0, skip, tl, te, I, J, Iloc)) {
        return;
    }
    if constexpr (XM == 4 && NST == 8)
        if (I == skip + 1 || J == skip + 1) return;
    /* wave-uniform first stage */
    int s0 = 0;
    if (NST == 4 && prev >= 0 && (I == prev || J == prev)) s0 = NST / 2;
    if (NST == 8 && prev >= 0)
        s0 = (I == prev + 1 || J == prev + 1) ? 6 : (I == prev || J == prev) ? 2 : 0;
    u16* C = D + (size_t)Iloc * 128 * ld + J * 128;
    const u16* Ag = D + (size_t)I * 128 * ld + k0;
    const u16* Bg = P + J * 128;
    fwq_stage_regs g;
    if (SYM)
        fwq_gload_sym(g, P + (size_t)s0 * UKC * ld, I * 128, Bg + (size_t)s0 * UKC * ld, ld, tid);
    else
        fwq_gload(g, Ag + s0 * UKC, Bg + (size_t)s0 * UKC * ld, ld, tid);
    uint32_t acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint4 v = *reinterpret_cast<const uint4*>(C + (size_t)(ty * 4 + r) * ld + tx * 8);
        acc[r][0] = v.x;
        acc[r][1] = v.y;
        acc[r][2] = v.z;
        acc[r][3] = v.w;
    }
    uint32_t sum0[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        sum0[r] = rowsum16(acc[r]);
        /* keep the four sums live, not the sixteen loaded words they came from (the compiler
         * otherwise sinks the sums to the stores and spills the rows) */
        asm volatile("" : "+v"(sum0[r]));
    }
#pragma unroll 1
    for (int s = s0; s < NST; ++s) {
        if (s > s0) __syncthreads(); /* the previous stage's LDS reads are done */
        fwq_swrite<SYM>(g, sA, sB, tid);
        __syncthreads();
        if (s + 1 < NST) { /* in flight during this stage */
            if (SYM)
                fwq_gload_sym(g, P + (size_t)(s + 1) * UKC * ld, I * 128,
                              Bg + (size_t)(s + 1) * UKC * ld, ld, tid);
            else
                fwq_gload(g, Ag + (s + 1) * UKC, Bg + (size_t)(s + 1) * UKC * ld, ld, tid);
        }
        fwq_stage(acc, sA, sB, tx, ty);
    }
    /* the store addresses are formed again here (an opaque copy of the thread index): kept from
     * the C load, the four 64-bit row addresses spill across the loop */
    int tq = tid;
    asm volatile("" : "+v"(tq));
    if constexpr (XM == 20) {
        u16* Oq = outq + (size_t)q20 * ld * ld + (size_t)Iloc * 128 * ld + J * 128 +
                  (size_t)((tq >> 4) * 4) * ld + (tq & 15) * 8;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            *reinterpret_cast<uint4*>(Oq + (size_t)r * ld) =
                make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
        (void)sum0;
        return;
    }
    u16* Cq = C + (size_t)((tq >> 4) * 4) * ld + (tq & 15) * 8;
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (rowsum16(acc[r]) != sum0[r])
            *reinterpret_cast<uint4*>(Cq + (size_t)r * ld) =
                make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
}

/* widen to the u32 table and flag saturation of a real pair (i, j < n) */
/* flags[0]: a real pair reached the cap (inexact); flags[1]: a real distance exceeds 254 quanta
 * (the post pass can read the distances as u8 otherwise) -- one atomic per wave at most, and none
 * once the flag is seen set */
__global__ void fw16_finish_kernel(int n, int ld, int row0, const u16* __restrict__ d16,
                                   uint32_t* __restrict__ lat, int* __restrict__ flags,
                                   uint32_t cap) {
    /* 8 columns per thread (ld is a multiple of 128): one 16-B load, two 16-B stores */
    const int j8 = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
    const int i = row0 + blockIdx.y;
    bool big = false, sat = false;
    if (j8 < ld) {
        const size_t ix = (size_t)blockIdx.y * ld + j8;
        const uint4 v = *reinterpret_cast<const uint4*>(d16 + ix);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
        uint32_t o[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const uint32_t x = (w4[q >> 1] >> (16 * (q & 1))) & 0xFFFFu;
            const bool real = i < n && j8 + q < n;
            o[q] = (x == cap) ? SRT_INF : x;
            sat |= real && x == cap;
            big |= real && x > 254u;
        }
        *reinterpret_cast<uint4*>(lat + ix) = make_uint4(o[0], o[1], o[2], o[3]);
        *reinterpret_cast<uint4*>(lat + ix + 4) = make_uint4(o[4], o[5], o[6], o[7]);
    }
    if (sat) atomicOr(flags, 1);
    if (__ballot(big) && (threadIdx.x & 63) == 0 &&
        !__hip_atomic_load(flags + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicOr(flags + 1, 1);
}

/* ---- row-sharded symmetric rounds: pivot panel from every rank, final transpose fill -------- */
/* Pivot panel of block k (tile row K) as R broadcasts: column block J comes from its contributor
 * (K's owner when it keeps (K, J), else the owner of row J, as (J, K)^T); blocks are staged in
 * (contributor, J) order, so each contributor's blocks are one contiguous broadcast. */
static __device__ __forceinline__ int sym_contrib(int K, int J, const int* __restrict__ own) {
    return sym_kept(K, J) ? own[K] : own[J];
}
/* position of column block J in the staged panel: blocks in (contributor, J) order. The owner
 * table is staged in LDS and the count spread over the workgroup (T <= SYM_TMAX tile columns). */
#define SYM_TMAX 1024
static __device__ int sym_contrib_pos(int K, int J, int T, const int* __restrict__ own, int* s_own,
                                      int* s_cnt) {
    for (int q = threadIdx.x; q < T; q += blockDim.x) s_own[q] = own[q];
    if (threadIdx.x == 0) *s_cnt = 0;
    __syncthreads();
    const int c = sym_contrib(K, J, s_own);
    int mine = 0;
    for (int q = threadIdx.x; q < T; q += blockDim.x) {
        const int cq = sym_contrib(K, q, s_own);
        mine += cq < c || (cq == c && q < J);
    }
    if (mine) atomicAdd(s_cnt, mine);
    __syncthreads();
    return *s_cnt;
}

/* rows of the staged-panel chain kernels per thread (sym_panel_stage_kernel, sym_cross_stage_kernel:
 * 1024 / SYM_RM threads per workgroup) */
#define SYM_RM 2

/* this rank's blocks of panel k into the staging buffer (64 x 128 each); with stage_b, a grid of
 * 2T also packs the band's second half (rows k0 + 64..) into stage_b (128-pivot rounds: one launch) */
__global__ __launch_bounds__(256) void sym_contrib_pack_kernel(const u16* __restrict__ D, int ld,
                                                               int row0, int tb, int K, int k0,
                                                               int T, const int* __restrict__ own,
                                                               int me, u16* __restrict__ stage,
                                                               u16* __restrict__ stage_b = nullptr) {
    __shared__ u16 t[128][KB + 8];
    __shared__ int s_own[SYM_TMAX], s_cnt;
    FW_CHAIN_PRIO();
    int J = (int)blockIdx.x;
    const int tid = threadIdx.x;
    if (J >= T) { /* the second half (uniform per workgroup) */
        J -= T;
        k0 += KB;
        stage = stage_b;
    }
    if (J >= T || sym_contrib(K, J, own) != me) return;
    u16* dst = stage + (size_t)sym_contrib_pos(K, J, T, own, s_own, &s_cnt) * (KB * 128);
    if (sym_kept(K, J)) { /* this rank owns the pivot rows: straight copy, 16 B per access */
        const u16* src = D + (size_t)(k0 - row0) * ld + (size_t)J * 128;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = tid + q * 256, row = i >> 4, c8 = (i & 15) * 8;
            *reinterpret_cast<uint4*>(dst + row * 128 + c8) =
                *reinterpret_cast<const uint4*>(src + (size_t)row * ld + c8);
        }
        return;
    }
    /* tile (J, K): rows r of block J, pivot columns m -> staged [m][r] */
    const u16* src = D + (size_t)(J - tb) * 128 * ld + k0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int i = tid + q * 256, r = i >> 3, m8 = (i & 7) * 8;
        *reinterpret_cast<uint4*>(&t[r][m8]) = *reinterpret_cast<const uint4*>(src + (size_t)r * ld + m8);
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int i = tid + q * 256, m = i >> 4, r8 = (i & 15) * 8;
        u16 v[8];
#pragma unroll
        for (int x = 0; x < 8; ++x) v[x] = t[r8 + x][m];
        uint4 o;
        o.x = v[0] | ((uint32_t)v[1] << 16);
        o.y = v[2] | ((uint32_t)v[3] << 16);
        o.z = v[4] | ((uint32_t)v[5] << 16);
        o.w = v[6] | ((uint32_t)v[7] << 16);
        *reinterpret_cast<uint4*>(dst + m * 128 + r8) = o;
    }
}

/* Panel of block k from the staged blocks in two launches (replacing unpack + diagonal + panel +
 * the owner's copy). Staged position of tile column J: blocks in (contributor, J) order. */
static __device__ int sym_stage_pos(int K, int J, int T, const int* __restrict__ own, int* s_own,
                                    int* s_cnt) {
    return sym_contrib_pos(K, J, T, own, s_own, s_cnt);
}

/* one workgroup: the diagonal block from its staged tile column, closed in LDS (64 dependent
 * steps, as fw16_diag_kernel), into P and, on the owner (prow != NULL), its pivot rows */
__global__ __launch_bounds__(256) void sym_diag_stage_kernel(u16* __restrict__ P, int ld, int K,
                                                             int k0, int T,
                                                             const int* __restrict__ own,
                                                             const u16* __restrict__ stage,
                                                             u16* __restrict__ prow) {
    __shared__ __attribute__((aligned(16))) u16 s[KB * LDA16];
    __shared__ int s_own[SYM_TMAX], s_cnt;
    FW_CHAIN_PRIO();
    const int tid = threadIdx.x;
    const u16* src = stage + (size_t)sym_stage_pos(K, K, T, own, s_own, &s_cnt) * (KB * 128) + (k0 & 127);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int i = tid + q * 256, row = i >> 3, c8 = (i & 7) * 8;
        *reinterpret_cast<uint4*>(s + row * LDA16 + c8) = *reinterpret_cast<const uint4*>(src + row * 128 + c8);
    }
    __syncthreads();
    close64<true>(s, tid);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int i = tid + q * 256, row = i >> 3, c8 = (i & 7) * 8;
        const uint4 v = *reinterpret_cast<const uint4*>(s + row * LDA16 + c8);
        *reinterpret_cast<uint4*>(P + (size_t)row * ld + k0 + c8) = v;
        if (prow) *reinterpret_cast<uint4*>(prow + (size_t)row * ld + k0 + c8) = v;
    }
}

/* P[:, j0..j0+63] = min(X, Dkk* (x) X) for every 64-column block j0 != k0, from the staged block X
 * and the closed diagonal block in P (as fw16_panel_kernel), into P and the owner's rows.
 * Workgroup J: the 64 x 128 staged block of tile column J (both 64-column halves; the half holding
 * the diagonal block is not written), RM rows x 8 columns per thread (1024 / RM threads). The
 * chain kernels run one workgroup per CU beside the bulk update, so fewer rows per thread (RM = 2)
 * put twice the waves on the latency-bound pivot loop. */
template <int RM>
__global__ __launch_bounds__(1024 / RM) void sym_panel_stage_kernel(u16* __restrict__ P, int ld, int K,
                                                                   int k0, int T,
                                                                   const int* __restrict__ own,
                                                                   const u16* __restrict__ stage,
                                                                   u16* __restrict__ prow) {
    constexpr int NT = 1024 / RM;
    __shared__ __attribute__((aligned(16))) u16 s[KB * LDA16];       /* Dkk* */
    __shared__ __attribute__((aligned(16))) u16 x[KB * (128 + 8)];   /* this workgroup's block */
    __shared__ int s_own[SYM_TMAX], s_cnt;
    FW_CHAIN_PRIO();
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int J = (int)blockIdx.x;
    const u16* xsrc = stage + (size_t)sym_stage_pos(K, J, T, own, s_own, &s_cnt) * (KB * 128);
#pragma unroll
    for (int q = 0; q < 512 / NT; ++q) {
        const int i = tid + q * NT, row = i >> 3, c8 = (i & 7) * 8;
        *reinterpret_cast<uint4*>(s + row * LDA16 + c8) =
            *reinterpret_cast<const uint4*>(P + (size_t)row * ld + k0 + c8);
    }
#pragma unroll
    for (int q = 0; q < 1024 / NT; ++q) {
        const int i = tid + q * NT, row = i >> 4, c8 = (i & 15) * 8;
        *reinterpret_cast<uint4*>(x + row * (128 + 8) + c8) =
            *reinterpret_cast<const uint4*>(xsrc + row * 128 + c8);
    }
    __syncthreads();
    uint32_t acc[RM][4];
#pragma unroll
    for (int r = 0; r < RM; ++r) {
        const uint4 v = *reinterpret_cast<const uint4*>(x + (RM * ty + r) * (128 + 8) + 8 * tx);
        acc[r][0] = v.x;
        acc[r][1] = v.y;
        acc[r][2] = v.z;
        acc[r][3] = v.w;
    }
#pragma unroll 2
    for (int m = 0; m < KB; m += 4) {
        uint2 a[RM];
        uint4 b[4];
#pragma unroll
        for (int r = 0; r < RM; ++r) a[r] = *reinterpret_cast<const uint2*>(s + (RM * ty + r) * LDA16 + m);
#pragma unroll
        for (int q = 0; q < 4; ++q) b[q] = *reinterpret_cast<const uint4*>(x + (m + q) * (128 + 8) + 8 * tx);
#pragma unroll
        for (int r = 0; r < RM; ++r) {
            const uint32_t p[4] = {splat(a[r].x & 0xFFFFu), splat(a[r].x >> 16),
                                   splat(a[r].y & 0xFFFFu), splat(a[r].y >> 16)};
#pragma unroll
            for (int q = 0; q < 4; q += 2) {
                const uint32_t b0[4] = {b[q].x, b[q].y, b[q].z, b[q].w};
                const uint32_t b1[4] = {b[q + 1].x, b[q + 1].y, b[q + 1].z, b[q + 1].w};
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[r][c] = relax2h(acc[r][c], p[q], b0[c], p[q + 1], b1[c]);
            }
        }
    }
    const int j0 = J * 128 + 8 * tx;
    if ((j0 & ~(KB - 1)) == k0) return; /* the diagonal block: sym_diag_stage_kernel's */
#pragma unroll
    for (int r = 0; r < RM; ++r) {
        const size_t o = (size_t)(RM * ty + r) * ld + j0;
        const uint4 v = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
        *reinterpret_cast<uint4*>(P + o) = v;
        if (prow) *reinterpret_cast<uint4*>(prow + o) = v;
    }
}

/* 128/256-pivot sharded rounds: the staged blocks of a later 64-row quarter y of the band (tile
 * row Ky, 64 x 128 per tile column J, in Ky's staging order) take a closed earlier pivot block x
 * (tile column Kx, columns cx..cx+63 of it) before P_y is closed:
 * X[J] = min(X[J], X_Kx[:, cx:cx+64] (x) P_x[:, J]), where X_Kx[:, cx:cx+64] = D[y][x] is the staged
 * block of tile column Kx and P_x the closed row panel x. The workgroup of J = Kx rewrites the
 * D[y][x] the others read: either value is a valid operand (P_x is closed, so old and updated
 * D[y][x] give the same minimum), as in blocked FW's column-panel/rest split. */
template <int RM>
__global__ __launch_bounds__(1024 / RM) void sym_cross_stage_kernel(const u16* __restrict__ Pa, int ld,
                                                                   int K, int T,
                                                                   const int* __restrict__ own,
                                                                   u16* __restrict__ stage, int Kx,
                                                                   int cx) {
    constexpr int NT = 1024 / RM;
    __shared__ __attribute__((aligned(16))) u16 s[KB * LDA16];     /* D[y][x] */
    __shared__ __attribute__((aligned(16))) u16 x[KB * (128 + 8)]; /* P_x[:, J] */
    __shared__ int s_own[SYM_TMAX], s_cnt;
    FW_CHAIN_PRIO();
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int J = (int)blockIdx.x;
    const u16* ak = stage + (size_t)sym_stage_pos(K, Kx, T, own, s_own, &s_cnt) * (KB * 128) + cx;
    __syncthreads(); /* s_cnt is reused by the second position */
    u16* xj = stage + (size_t)sym_stage_pos(K, J, T, own, s_own, &s_cnt) * (KB * 128);
#pragma unroll
    for (int q = 0; q < 512 / NT; ++q) {
        const int i = tid + q * NT, row = i >> 3, c8 = (i & 7) * 8;
        *reinterpret_cast<uint4*>(s + row * LDA16 + c8) =
            *reinterpret_cast<const uint4*>(ak + row * 128 + c8);
    }
#pragma unroll
    for (int q = 0; q < 1024 / NT; ++q) {
        const int i = tid + q * NT, row = i >> 4, c8 = (i & 15) * 8;
        *reinterpret_cast<uint4*>(x + row * (128 + 8) + c8) =
            *reinterpret_cast<const uint4*>(Pa + (size_t)row * ld + (size_t)J * 128 + c8);
    }
    uint32_t acc[RM][4];
#pragma unroll
    for (int r = 0; r < RM; ++r) {
        const uint4 v = *reinterpret_cast<const uint4*>(xj + (RM * ty + r) * 128 + 8 * tx);
        acc[r][0] = v.x;
        acc[r][1] = v.y;
        acc[r][2] = v.z;
        acc[r][3] = v.w;
    }
    __syncthreads();
#pragma unroll 2
    for (int m = 0; m < KB; m += 4) {
        uint2 a[RM];
        uint4 b[4];
#pragma unroll
        for (int r = 0; r < RM; ++r) a[r] = *reinterpret_cast<const uint2*>(s + (RM * ty + r) * LDA16 + m);
#pragma unroll
        for (int q = 0; q < 4; ++q) b[q] = *reinterpret_cast<const uint4*>(x + (m + q) * (128 + 8) + 8 * tx);
#pragma unroll
        for (int r = 0; r < RM; ++r) {
            const uint32_t p[4] = {splat(a[r].x & 0xFFFFu), splat(a[r].x >> 16),
                                   splat(a[r].y & 0xFFFFu), splat(a[r].y >> 16)};
#pragma unroll
            for (int q = 0; q < 4; q += 2) {
                const uint32_t b0[4] = {b[q].x, b[q].y, b[q].z, b[q].w};
                const uint32_t b1[4] = {b[q + 1].x, b[q + 1].y, b[q + 1].z, b[q + 1].w};
#pragma unroll
                for (int c = 0; c < 4; ++c) acc[r][c] = relax2h(acc[r][c], p[q], b0[c], p[q + 1], b1[c]);
            }
        }
    }
#pragma unroll
    for (int r = 0; r < RM; ++r)
        *reinterpret_cast<uint4*>(xj + (RM * ty + r) * 128 + 8 * tx) =
            make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
}

/* Two-deep sharded rounds (fw16_build_sym_sharded, deep): a closed 128-row panel P (rows P_a over
 * P_b, 128 x ld) applied to a band that was staged early -- the two 64-row halves sa / sb of tile
 * row Kb, 64 x 128 per tile column J in Kb's staging order. In symmetric rounds the A operand of a
 * row-Kb tile is P's own columns at Kb (D[i][k] = D[k][i] = P[k][i]), so the band needs nothing but
 * P: X[:, J] = min(X[:, J], P[:, Kb]^T (x) P[:, J]), the fwq_update_kernel<true> tile with C in the
 * staging buffer (row stride 128). One workgroup per tile column, 128 pivots in four stages. */
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(8, 8))) void fwq_band_kernel(
    const u16* __restrict__ P, int ld, int Kb, int T, const int* __restrict__ own,
    u16* __restrict__ sa, u16* __restrict__ sb) {
    __shared__ __attribute__((aligned(16))) uint32_t sA[UKC / 2 * 128 * 2];
    __shared__ __attribute__((aligned(16))) u16 sB[UKC * UBS];
    __shared__ int s_own[SYM_TMAX], s_cnt;
    FW_CHAIN_PRIO();
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int J = (int)blockIdx.x;
    const size_t pos = (size_t)sym_stage_pos(Kb, J, T, own, s_own, &s_cnt) * (KB * 128);
    /* rows 4 ty .. 4 ty + 3 of the 128-row tile: the a half below 64, the b half above */
    u16* C = (ty < 16 ? sa + pos + (size_t)(ty * 4) * 128 : sb + pos + (size_t)(ty * 4 - 64) * 128) +
             tx * 8;
    const u16* Bg = P + J * 128;
    fwq_stage_regs g;
    fwq_gload_sym(g, P, Kb * 128, Bg, ld, tid);
    uint32_t acc[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint4 v = *reinterpret_cast<const uint4*>(C + r * 128);
        acc[r][0] = v.x;
        acc[r][1] = v.y;
        acc[r][2] = v.z;
        acc[r][3] = v.w;
    }
#pragma unroll 1
    for (int s = 0; s < 4; ++s) {
        if (s > 0) __syncthreads();
        fwq_swrite<true>(g, sA, sB, tid);
        __syncthreads();
        if (s + 1 < 4)
            fwq_gload_sym(g, P + (size_t)(s + 1) * UKC * ld, Kb * 128, Bg + (size_t)(s + 1) * UKC * ld,
                          ld, tid);
        fwq_stage(acc, sA, sB, tx, ty);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
        *reinterpret_cast<uint4*>(C + r * 128) = make_uint4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
}

/* final fill: kept tile (I, J) of the sender, transposed into a contiguous 128 x 128 block */
__global__ __launch_bounds__(256) void sym_fill_pack_kernel(const u16* __restrict__ D, int ld, int tb,
                                                            const uint32_t* __restrict__ pairs,
                                                            u16* __restrict__ out) {
    __shared__ u16 t[128][128 + 2];
    const uint32_t p = pairs[blockIdx.x];
    const int I = (int)(p >> 16), J = (int)(p & 0xFFFFu);
    const u16* src = D + (size_t)(I - tb) * 128 * ld + (size_t)J * 128;
    for (int i = threadIdx.x; i < 128 * 128; i += 256) t[i / 128][i % 128] = src[(size_t)(i / 128) * ld + i % 128];
    __syncthreads();
    u16* dst = out + (size_t)blockIdx.x * (128 * 128);
    for (int i = threadIdx.x; i < 128 * 128; i += 256) dst[i] = t[i % 128][i / 128];
}

/* receiver: block b (the sender's pair (I, J), J in this rank's rows) becomes tile (J, I) */
__global__ __launch_bounds__(256) void sym_fill_unpack_kernel(u16* __restrict__ D, int ld, int tb,
                                                              const uint32_t* __restrict__ pairs,
                                                              const u16* __restrict__ in) {
    const uint32_t p = pairs[blockIdx.x];
    const int I = (int)(p >> 16), J = (int)(p & 0xFFFFu);
    const u16* src = in + (size_t)blockIdx.x * (128 * 128);
    u16* dst = D + (size_t)(J - tb) * 128 * ld + (size_t)I * 128;
    for (int i = threadIdx.x; i < 128 * 128; i += 256) dst[(size_t)(i / 128) * ld + i % 128] = src[i];
}

/* both tiles in this rank's rows: kept (I, J) transposed into (J, I) */
__global__ __launch_bounds__(256) void sym_fill_local_kernel(u16* __restrict__ D, int ld, int tb,
                                                             const uint32_t* __restrict__ pairs) {
    __shared__ u16 t[128][128 + 2];
    const uint32_t p = pairs[blockIdx.x];
    const int I = (int)(p >> 16), J = (int)(p & 0xFFFFu);
    const u16* src = D + (size_t)(I - tb) * 128 * ld + (size_t)J * 128;
    for (int i = threadIdx.x; i < 128 * 128; i += 256) t[i / 128][i % 128] = src[(size_t)(i / 128) * ld + i % 128];
    __syncthreads();
    u16* dst = D + (size_t)(J - tb) * 128 * ld + (size_t)I * 128;
    for (int i = threadIdx.x; i < 128 * 128; i += 256) dst[(size_t)(i / 128) * ld + i % 128] = t[i % 128][i / 128];
}

#ifndef SRT_FW16_DEVICE_ONLY
#define FW_UPDATE(SYMV, XMV, GRID, STREAM, ...) \
    fwq_update_kernel<SYMV, XMV><<<(GRID), 512, 0, (STREAM)>>>(__VA_ARGS__)
/* ---- orchestration --------------------------------------------------------------------------- *
 * Lookahead schedule (one row shard per rank; a single GPU is the 1-rank case). Round k uses the
 * 64-row pivot panel P_k (owner: in place in its rows; others: a double-buffered receive panel).
 * Main stream st:      wait P_k ready -> pivot-column tiles of k -> update k
 * Critical stream cs:  diagonal closure + pivot-row panel of k+1 -> broadcast P_k+1 -> P_k+1 ready
 * On the owner of k+1 the update of round k is split: the 128-row tile row holding block k+1 goes
 * first, cs starts the k+1 panel as soon as it is done, and the remaining tile rows of round k
 * overlap the panel work and the RCCL broadcast. A receive panel is overwritten only after the
 * update that last read it (round k-1) has finished.
 * Without a broadcast to hide (one GPU) the split and the cross-stream events cost more than the
 * overlap returns (C2: 1.01 -> 1.34 ms), so the single-GPU build runs the same rounds on one stream
 * in order; SRT_FORM lookahead=1 forces the two-stream schedule (tests exercise it on one GPU). */
/* per-device u16 working matrix of the last build (rows of the shard, ld columns); the dense
 * post pass reads it transposed for the predecessor search (half the bytes of the u32 table) */
static u16* fw16_bufs[SRT_STATE_SLOTS];
static size_t fw16_caps[SRT_STATE_SLOTS]; /* elements allocated in fw16_bufs (shared by both build forms) */
static int* fw16_flags[SRT_STATE_SLOTS];
static int fw16_small[SRT_STATE_SLOTS]; /* last build: every real distance <= 254 quanta */
int srt_fw16_small(void) { return fw16_small[srt_state_slot()]; }
static thread_local int g_sharded_rp = 64; /* pivots per round of this thread's last sharded build */
const uint16_t* srt_fw16_matrix(void) { return fw16_bufs[srt_state_slot()]; }

typedef struct {
    hipStream_t cs;
    hipEvent_t ready[2], row_done, upd_done[2], init_done;
    /* one-GPU symmetric rounds on two update streams (st, xs) */
    hipStream_t xs;
    hipEvent_t e_set[2][2]; /* [round & 1][tile set]: the set's next-row tiles are done */
    hipEvent_t xs_done[2];  /* sharded symmetric rounds: stream xs finished round k's update */
    /* two-deep sharded rounds: the band stream (pack + broadcast) and its staged-band arrivals */
    hipStream_t ms;
    hipEvent_t arr[3], applied[3];
    uint32_t* tl2;
    size_t tl2_cap;
    int ok;
} fw16_sched;

static int sched_get(fw16_sched** out, int dev) {
    static fw16_sched sc[SRT_STATE_SLOTS];
    fw16_sched* x = &sc[dev % SRT_STATE_SLOTS];
    if (!x->ok) {
        int lo = 0, hi = 0;
        SRT_HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        SRT_HIPCHK(hipStreamCreateWithPriority(&x->cs, hipStreamNonBlocking, hi));
        for (int i = 0; i < 2; ++i) {
            SRT_HIPCHK(hipEventCreateWithFlags(&x->ready[i], hipEventDisableTiming));
            SRT_HIPCHK(hipEventCreateWithFlags(&x->upd_done[i], hipEventDisableTiming));
        }
        SRT_HIPCHK(hipEventCreateWithFlags(&x->row_done, hipEventDisableTiming));
        SRT_HIPCHK(hipEventCreateWithFlags(&x->init_done, hipEventDisableTiming));
        SRT_HIPCHK(hipStreamCreateWithFlags(&x->xs, hipStreamNonBlocking));
        for (int i = 0; i < 4; ++i)
            SRT_HIPCHK(hipEventCreateWithFlags(&x->e_set[i / 2][i % 2], hipEventDisableTiming));
        for (int i = 0; i < 2; ++i)
            SRT_HIPCHK(hipEventCreateWithFlags(&x->xs_done[i], hipEventDisableTiming));
        SRT_HIPCHK(hipStreamCreateWithPriority(&x->ms, hipStreamNonBlocking, hi));
        for (int i = 0; i < 3; ++i) {
            SRT_HIPCHK(hipEventCreateWithFlags(&x->arr[i], hipEventDisableTiming));
            SRT_HIPCHK(hipEventCreateWithFlags(&x->applied[i], hipEventDisableTiming));
        }
        x->ok = 1;
    }
    *out = x;
    return SRT_OK;
}

/* Upper-triangle blocked FW for an undirected graph on one GPU (f16-compare kernels). */
/* Upper-triangle blocked FW for an undirected graph on one GPU (f16-compare kernels).
 * two: the upper-triangle tiles are split by the parity of I + J into two static sets, each
 * updated by its own stream (st, xs) every round, while the high-priority stream cs closes the
 * next diagonal block, builds the next panel and refreshes it as soon as both streams have
 * updated their tiles of the next pivot block's tile row and column (launched first). A stream
 * depends only on its own previous launches and on the panel, so one stream's next round starts
 * in the other's tail and the panel work overlaps the update. A stream may then read pivot rows
 * that the other stream has already relaxed in the next round: those values are still lengths
 * of real paths, no larger than the round requires, so the result is the same exact matrix. */
static int fw16_build_sym(int n, int ld, const uint32_t* w, uint32_t* lat, hipStream_t st,
                          evpool_t* evp, int* exact, bool two, int round_pivots) {
    const bool r128 = round_pivots == 128, r256 = round_pivots == 256;
    const int dev = srt_state_slot(); /* the device, or this virtual rank's slot */
    size_t* caps = fw16_caps;
    int** flags = fw16_flags;
    const size_t need = (size_t)ld * ld;
    if (caps[dev] < need || !fw16_bufs[dev]) {
        if (fw16_bufs[dev]) SRT_HIPCHK(hipFree(fw16_bufs[dev]));
        fw16_bufs[dev] = NULL;
        caps[dev] = 0;
        SRT_HIPCHK(hipMalloc(&fw16_bufs[dev], need * sizeof(u16)));
        caps[dev] = need;
    }
    if (!flags[dev]) SRT_HIPCHK(hipMalloc(&flags[dev], 2 * sizeof(int)));
    u16* d = fw16_bufs[dev];
    fw16_init_kernel<<<dim3(srt_ceil_div(ld, 2048), ld), 256, 0, st>>>(n, ld, 0, w, d, CAP_F);
    SRT_HIPCHK(hipGetLastError());
    const int nb = ld / KB, T = ld / 128;
    const int ntri = T * (T + 1) / 2;
    if (!two) {
        for (int k0 = 0; k0 < ld; k0 += KB) {
            u16* P = d + (size_t)k0 * ld;
            fw16_diag_kernel<true><<<1, 256, 0, st>>>(P, ld, k0);
            fw16_panel_kernel<true, true><<<2 * nb, 256, 0, st>>>(d, ld, 0, nb, P, k0, nb, 1, 1);
            if (k0 > 0) fw16_refresh_kernel<<<k0 / KB, 256, 0, st>>>(d, ld, k0);
            if (evp) SRT_HIPCHK(hipEventRecord(evp->ev[evp->used++], st));
            FW_UPDATE(true, 0, ntri, st, d, ld, P, k0, T, 0, -1, nullptr, 0);
            if (evp) SRT_HIPCHK(hipEventRecord(evp->ev[evp->used++], st));
            SRT_HIPCHK(hipGetLastError());
        }
    } else {
        fw16_sched* sc;
        int rc = sched_get(&sc, dev);
        if (rc) return rc;
        hipStream_t cs = sc->cs, xs = sc->xs;
        /* the two tile sets, row-major, as device lists */
        uint32_t* h = (uint32_t*)malloc((size_t)ntri * sizeof(uint32_t));
        if (!h) return SRT_E_NOMEM;
        int nset[2] = {0, 0};
        for (int p = 0, o = 0; p < 2; p++)
            for (int I = 0; I < T; I++)
                for (int J = I; J < T; J++)
                    if (((I + J) & 1) == p) {
                        h[o++] = ((uint32_t)I << 16) | (uint32_t)J;
                        nset[p]++;
                    }
        if (!sc->tl2 || sc->tl2_cap < (size_t)ntri) {
            if (sc->tl2) SRT_HIPCHK(hipFree(sc->tl2));
            sc->tl2 = NULL;
            SRT_HIPCHK(hipMalloc(&sc->tl2, (size_t)ntri * sizeof(uint32_t)));
            sc->tl2_cap = (size_t)ntri;
        }
        const hipError_t ce = hipMemcpyAsync(sc->tl2, h, (size_t)ntri * sizeof(uint32_t),
                                             hipMemcpyHostToDevice, st);
        const hipError_t se = ce == hipSuccess ? hipStreamSynchronize(st) : ce;
        free(h);
        SRT_HIPCHK(se);
        const uint32_t* tls[2] = {sc->tl2, sc->tl2 + nset[0]};
        hipStream_t ss[2] = {st, xs};
        auto produce = [&](int k) -> int {
            const int k0 = k * KB;
            u16* P = d + (size_t)k0 * ld;
            fw16_diag_kernel<true><<<1, 256, 0, cs>>>(P, ld, k0);
            fw16_panel_kernel<true, true><<<2 * nb, 256, 0, cs>>>(d, ld, 0, nb, P, k0, nb, 1, 1);
            if (k0 > 0) fw16_refresh_kernel<<<k0 / KB, 256, 0, cs>>>(d, ld, k0);
            SRT_HIPCHK(hipGetLastError());
            SRT_HIPCHK(hipEventRecord(sc->ready[k & 1], cs));
            return SRT_OK;
        };
        SRT_HIPCHK(hipEventRecord(sc->init_done, st));
        SRT_HIPCHK(hipStreamWaitEvent(cs, sc->init_done, 0));
        SRT_HIPCHK(hipStreamWaitEvent(xs, sc->init_done, 0));
        if (r256) {
            /* 256-pivot rounds (pivot blocks a..d = 4j..4j+3: tile rows R0 = 2j, R1 = 2j + 1):
             * every C tile stays resident for four panels (eight 32-pivot stages). Chain stream cs,
             * per round j: close P_a, apply it to the cross of R0; close P_b, apply P_a and P_b to
             * the cross of R1; close P_c, apply it to the cross of R1; close P_d -> ready[j].
             * Update stream p, per round j (after ready[j]): the crosses of the next round's tile
             * rows with all four panels, then the rest, whose tiles in the crosses of R0 / R1 start
             * past the panels the chain already applied (fwq_update_kernel prev). */
            auto closep = [&](int k0) -> int {
                u16* P = d + (size_t)k0 * ld;
                fw16_diag_kernel<true><<<1, 256, 0, cs>>>(P, ld, k0);
                fw16_panel_kernel<true, true><<<2 * nb, 256, 0, cs>>>(d, ld, 0, nb, P, k0, nb, 1, 1);
                if (k0 > 0) fw16_refresh_kernel<<<k0 / KB, 256, 0, cs>>>(d, ld, k0);
                SRT_HIPCHK(hipGetLastError());
                return SRT_OK;
            };
            auto produce4 = [&](int j) -> int {
                const int ka = 4 * j * KB, R0 = 2 * j;
                int rc2;
                if ((rc2 = closep(ka))) return rc2;
                fwq_update_kernel<true, 9, 2><<<T, 512, 0, cs>>>(d, ld, d + (size_t)ka * ld, ka, T, 0,
                                                               R0, nullptr, 0, -1);
                if ((rc2 = closep(ka + KB))) return rc2;
                fwq_update_kernel<true, 9, 4><<<T, 512, 0, cs>>>(d, ld, d + (size_t)ka * ld, ka, T, 0,
                                                               R0 + 1, nullptr, 0, -1);
                if ((rc2 = closep(ka + 2 * KB))) return rc2;
                fwq_update_kernel<true, 9, 2><<<T, 512, 0, cs>>>(
                    d, ld, d + (size_t)(ka + 2 * KB) * ld, ka + 2 * KB, T, 0, R0 + 1, nullptr, 0, -1);
                if ((rc2 = closep(ka + 3 * KB))) return rc2;
                SRT_HIPCHK(hipGetLastError());
                SRT_HIPCHK(hipEventRecord(sc->ready[j & 1], cs));
                return SRT_OK;
            };
            const int R = T / 2;
            if ((rc = produce4(0))) return rc;
            for (int j = 0; j < R; ++j) {
                const int ka = 4 * j * KB;
                u16* Pa = d + (size_t)ka * ld;
                const bool next = j + 1 < R;
                for (int p = 0; p < 2; p++) {
                    SRT_HIPCHK(hipStreamWaitEvent(ss[p], sc->ready[j & 1], 0));
                    if (next) {
                        fwq_update_kernel<true, 13, 8><<<2 * T, 512, 0, ss[p]>>>(
                            d, ld, Pa, ka, T, p, 2 * j + 2, nullptr, 0, -1);
                        SRT_HIPCHK(hipEventRecord(sc->e_set[j & 1][p], ss[p]));
                    }
                }
                if (next) {
                    SRT_HIPCHK(hipStreamWaitEvent(cs, sc->e_set[j & 1][0], 0));
                    SRT_HIPCHK(hipStreamWaitEvent(cs, sc->e_set[j & 1][1], 0));
                    if ((rc = produce4(j + 1))) return rc;
                }
                const int e0 = evp ? evp->used : 0;
                if (evp && next) {
                    evp->group = 4;
                    evp->used += 4;
                }
                for (int p = 0; p < 2; p++) {
                    if (evp && next) SRT_HIPCHK(hipEventRecord(evp->ev[e0 + p], ss[p]));
                    if (next)
                        fwq_update_kernel<true, 4, 8><<<(unsigned)nset[p], 512, 0, ss[p]>>>(
                            d, ld, Pa, ka, T, 0, 2 * j + 2, tls[p], T, 2 * j);
                    else
                        fwq_update_kernel<true, 5, 8><<<(unsigned)nset[p], 512, 0, ss[p]>>>(
                            d, ld, Pa, ka, T, 0, -1, tls[p], T, 2 * j);
                    if (evp && next) SRT_HIPCHK(hipEventRecord(evp->ev[e0 + 2 + p], ss[p]));
                }
                SRT_HIPCHK(hipGetLastError());
            }
        } else if (r128) {
            /* 128-pivot rounds (pivot blocks a = 2j, b = 2j + 1: tile row j): every C tile stays
             * resident for both panels (four 32-pivot stages), which halves the per-pivot C loads,
             * row sums and stores and the bulk launches. Chain stream cs, per round j:
             * close P_a, apply it to the cross of tile j (its row and column, XM 9), close P_b ->
             * ready[j]. Update stream p, per round j: (after ready[j]) the cross of tile j + 1
             * with P_a and P_b, then the rest with both, where the cross of j takes P_b only (it
             * has P_a). The cross of j + 1 is excluded from round j's rest and updated first, so
             * cs can close P_a' of round j + 1 under the rest; cs's cross updates touch no tile
             * of the rest launch still running (round j - 1 excludes the cross of j). */
            auto produce2 = [&](int j) -> int {
                const int ka = 2 * j * KB;
                u16* Pa = d + (size_t)ka * ld;
                fw16_diag_kernel<true><<<1, 256, 0, cs>>>(Pa, ld, ka);
                fw16_panel_kernel<true, true><<<2 * nb, 256, 0, cs>>>(d, ld, 0, nb, Pa, ka, nb, 1, 1);
                if (ka > 0) fw16_refresh_kernel<<<ka / KB, 256, 0, cs>>>(d, ld, ka);
                fwq_update_kernel<true, 9, 2><<<T, 512, 0, cs>>>(d, ld, Pa, ka, T, 0, j, nullptr, 0, -1);
                const int kb = ka + KB;
                u16* Pb = d + (size_t)kb * ld;
                fw16_diag_kernel<true><<<1, 256, 0, cs>>>(Pb, ld, kb);
                fw16_panel_kernel<true, true><<<2 * nb, 256, 0, cs>>>(d, ld, 0, nb, Pb, kb, nb, 1, 1);
                fw16_refresh_kernel<<<kb / KB, 256, 0, cs>>>(d, ld, kb);
                SRT_HIPCHK(hipGetLastError());
                SRT_HIPCHK(hipEventRecord(sc->ready[j & 1], cs));
                return SRT_OK;
            };
            if ((rc = produce2(0))) return rc;
            for (int j = 0; j < T; ++j) {
                const int ka = 2 * j * KB;
                u16* Pa = d + (size_t)ka * ld;
                const bool next = j + 1 < T;
                for (int p = 0; p < 2; p++) {
                    SRT_HIPCHK(hipStreamWaitEvent(ss[p], sc->ready[j & 1], 0));
                    if (next) {
                        fwq_update_kernel<true, 6, 4><<<T, 512, 0, ss[p]>>>(d, ld, Pa, ka, T, p, j + 1,
                                                                          nullptr, 0, -1);
                        SRT_HIPCHK(hipEventRecord(sc->e_set[j & 1][p], ss[p]));
                    }
                }
                if (next) {
                    SRT_HIPCHK(hipStreamWaitEvent(cs, sc->e_set[j & 1][0], 0));
                    SRT_HIPCHK(hipStreamWaitEvent(cs, sc->e_set[j & 1][1], 0));
                    if ((rc = produce2(j + 1))) return rc;
                }
                const int e0 = evp ? evp->used : 0;
                if (evp && next) {
                    evp->group = 4;
                    evp->used += 4;
                }
                for (int p = 0; p < 2; p++) {
                    if (evp && next) SRT_HIPCHK(hipEventRecord(evp->ev[e0 + p], ss[p]));
                    if (next)
                        fwq_update_kernel<true, 4, 4><<<(unsigned)nset[p], 512, 0, ss[p]>>>(
                            d, ld, Pa, ka, T, 0, j + 1, tls[p], T, j);
                    else
                        fwq_update_kernel<true, 5, 4><<<(unsigned)nset[p], 512, 0, ss[p]>>>(
                            d, ld, Pa, ka, T, 0, -1, tls[p], T, j);
                    if (evp && next) SRT_HIPCHK(hipEventRecord(evp->ev[e0 + 2 + p], ss[p]));
                }
                SRT_HIPCHK(hipGetLastError());
            }
        } else {
        if ((rc = produce(0))) return rc;
        for (int k = 0; k < nb; ++k) {
            const int k0 = k * KB;
            u16* P = d + (size_t)k0 * ld;
            const bool next = k + 1 < nb;
            const int K1 = next ? ((k + 1) * KB) / 128 : -1;
            for (int p = 0; p < 2; p++) {
                SRT_HIPCHK(hipStreamWaitEvent(ss[p], sc->ready[k & 1], 0));
                if (next) {
                    FW_UPDATE(true, 6, T, ss[p], d, ld, P, k0, T, p, K1, nullptr, 0);
                    SRT_HIPCHK(hipEventRecord(sc->e_set[k & 1][p], ss[p]));
                }
            }
            if (next) {
                SRT_HIPCHK(hipStreamWaitEvent(cs, sc->e_set[k & 1][0], 0));
                SRT_HIPCHK(hipStreamWaitEvent(cs, sc->e_set[k & 1][1], 0));
                if ((rc = produce(k + 1))) return rc;
            }
            /* timed as one unit: the two rest-of-round launches, from the first start to the
             * last end (evpool group 4: start A, start B, end A, end B) */
            const int e0 = evp ? evp->used : 0;
            if (evp && next) {
                evp->group = 4;
                evp->used += 4;
            }
            for (int p = 0; p < 2; p++) {
                if (evp && next) SRT_HIPCHK(hipEventRecord(evp->ev[e0 + p], ss[p]));
                if (next)
                    FW_UPDATE(true, 4, (unsigned)nset[p], ss[p],
                        d, ld, P, k0, T, 0, K1, tls[p], T);
                else
                    FW_UPDATE(true, 5, (unsigned)nset[p], ss[p],
                        d, ld, P, k0, T, 0, -1, tls[p], T);
                if (evp && next) SRT_HIPCHK(hipEventRecord(evp->ev[e0 + 2 + p], ss[p]));
            }
            SRT_HIPCHK(hipGetLastError());
        }
        }
        SRT_HIPCHK(hipEventRecord(sc->row_done, xs));
        SRT_HIPCHK(hipStreamWaitEvent(st, sc->row_done, 0));
    }
    fw16_mirror_kernel<<<dim3(nb, nb), 256, 0, st>>>(d, ld);
    SRT_HIPCHK(hipMemsetAsync(flags[dev], 0, 2 * sizeof(int), st));
    fw16_finish_kernel<<<dim3(srt_ceil_div(ld, 2048), ld), 256, 0, st>>>(n, ld, 0, d, lat, flags[dev],
                                                                        CAP_F);
    SRT_HIPCHK(hipGetLastError());
    int hf[2] = {0, 0};
    SRT_HIPCHK(hipMemcpyAsync(hf, flags[dev], 2 * sizeof(int), hipMemcpyDeviceToHost, st));
    SRT_HIPCHK(hipStreamSynchronize(st));
    *exact = hf[0] ? 0 : 1;
    fw16_small[dev] = hf[1] ? 0 : 1;
    return SRT_OK;
}

/* Row-sharded symmetric FW (undirected graph, f16-compare path, R > 1 ranks; SURVEY §8e with the
 * one-GPU upper-triangle saving). Rows stay in the srt_shard_rows blocks; of each tile pair
 * (I, J) / (J, I) one rank keeps and updates one orientation (sym_kept), so every rank updates
 * about half of its row block whatever its position. Round k needs the full pivot panel P_k (64 x
 * ld): column block J is in the kept tile (K, J) at the owner of tile row K, or is (J, K)^T at
 * the owner of row J. Every rank stages the blocks it holds (transposing the latter) and
 * broadcasts them, one grouped broadcast per round (4 MiB in all at C4); each rank then closes
 * the diagonal block and updates the row panel itself (24 us, instead of a second collective
 * in the chain), and the owner writes the result back into its pivot rows. Every rank updates
 * its kept tiles with A = P^T (column block I) and B = P (column block J), as on one GPU.
 * Lookahead as in srt_fw16_build: each round first updates the kept tiles of the next pivot
 * block's tile row and column (XM 3), the high-priority stream cs assembles and closes the next
 * panel under the rest of the round (XM 4). After the last round each rank receives the
 * transposes of the tiles it does not keep (point-to-point) and fills them in locally. */
static int fw16_build_sym_sharded(const srt_comm* comm, int n, int ld, int row0, int nrows,
                                  const uint32_t* w_rows, uint32_t* lat_rows, hipStream_t st,
                                  evpool_t* evp, int* exact, int kbr) {
    const int dev = srt_state_slot();
    const int R = srt_comm_size(comm), me = srt_comm_rank(comm);
    /* kbr = 128: 128-pivot rounds (pivot block = tile row K, panels P_a over P_b, four 32-pivot
     * stages per C-tile residency); kbr = 64: 64-pivot rounds */
    const bool r128 = kbr == 128;
    const int T = ld / 128, nb = ld / kbr;
    const int tb = row0 / 128, te = (row0 + nrows) / 128;
    size_t* caps = fw16_caps;
    int** flags = fw16_flags;
    const size_t need = (size_t)nrows * ld + 2 * (size_t)kbr * ld;
    if (caps[dev] < need || !fw16_bufs[dev]) {
        if (fw16_bufs[dev]) SRT_HIPCHK(hipFree(fw16_bufs[dev]));
        fw16_bufs[dev] = NULL;
        caps[dev] = 0;
        SRT_HIPCHK(hipMalloc(&fw16_bufs[dev], need * sizeof(u16)));
        caps[dev] = need;
    }
    if (!flags[dev]) SRT_HIPCHK(hipMalloc(&flags[dev], 2 * sizeof(int)));
    fw16_sched* sc;
    int rc = sched_get(&sc, dev);
    if (rc) return rc;
    hipStream_t cs = sc->cs;
    u16* d = fw16_bufs[dev];
    u16* pbuf[2] = {d + (size_t)nrows * ld, d + (size_t)nrows * ld + (size_t)kbr * ld};
    /* tile-row ranges of every rank, the owner of each tile row, this rank's kept tiles */
    int* qtb = (int*)malloc((size_t)R * sizeof(int));
    int* qte = (int*)malloc((size_t)R * sizeof(int));
    int* own = (int*)malloc((size_t)T * sizeof(int));
    const size_t maxkept = (size_t)(te - tb) * T + 1;
    uint32_t* hkept = (uint32_t*)malloc(maxkept * sizeof(uint32_t));
    if (!qtb || !qte || !own || !hkept) {
        free(qtb);
        free(qte);
        free(own);
        free(hkept);
        return SRT_E_NOMEM;
    }
    for (int q = 0; q < R; q++) {
        int32_t qb, qe;
        srt_shard_rows(ld, SRT_SHARD_ALIGN, R, q, &qb, &qe);
        qtb[q] = qb / 128;
        qte[q] = qe / 128;
        for (int K = qtb[q]; K < qte[q] && K < T; K++) own[K] = q;
    }
    /* kept tiles, even J first, then odd J: the lists of the two update streams */
    size_t nkept = 0, nset[2] = {0, 0};
    for (int p = 0; p < 2; p++)
        for (int I = tb; I < te; I++)
            for (int J = p; J < T; J += 2)
                if (sym_kept(I, J)) {
                    hkept[nkept++] = ((uint32_t)I << 16) | (uint32_t)J;
                    nset[p]++;
                }
    /* device scratch: kept-tile list, gather send (this rank's rows) and receive (a panel) */
    uint32_t* tl = NULL;
    int* down = NULL; /* owner of each tile row, on the device */
    u16* grecv = NULL; /* staged panel blocks in (contributor, J) order (r128: rows a, then b) */
    int* cnt = (int*)calloc(2 * (size_t)R, sizeof(int)); /* per contributor (256: two tile rows) */
    const size_t blk = (size_t)KB * 128;
    /* two-deep 128-pivot rounds (N > 1 with two or more tile rows): band k + 3 is staged
     * and broadcast on its own stream right after round k's update, three rounds ahead, and each
     * rank applies the two panels it missed to the staged band itself (fwq_band_kernel) */
    const bool deep = r128 && R > 1 && T >= 2;
    const size_t nstage = (size_t)(kbr / KB) * ((size_t)T + 1) * blk * (deep ? 3 : 1);
    bool ok = cnt && hipMalloc(&tl, (nkept + 1) * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&down, (size_t)T * sizeof(int)) == hipSuccess &&
              hipMalloc(&grecv, nstage * sizeof(u16)) == hipSuccess;
    if (ok)
        ok = hipMemcpyAsync(down, own, (size_t)T * sizeof(int), hipMemcpyHostToDevice, st) ==
                 hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess;
    /* timing-only communicator: the blocks other ranks would send stay a small constant, so the
     * arithmetic keeps the u16 tier and the u8 post pass (the tables are not correct) */
    if (ok && srt_comm_is_solo(comm))
        ok = hipMemsetD16Async((hipDeviceptr_t)grecv, 3, nstage, st) == hipSuccess;
    void** sp = (void**)calloc((size_t)R, sizeof(void*));
    void** rp = (void**)calloc((size_t)R, sizeof(void*));
    size_t* sbytes = (size_t*)calloc((size_t)R, sizeof(size_t));
    size_t* rbytes = (size_t*)calloc((size_t)R, sizeof(size_t));
    ok = ok && sp && rp && sbytes && rbytes;
    if (ok && nkept) /* pageable source: finished before the host list can change */
        ok = hipMemcpyAsync(tl, hkept, nkept * sizeof(uint32_t), hipMemcpyHostToDevice, st) ==
                 hipSuccess &&
             hipStreamSynchronize(st) == hipSuccess;
#define SYM_FAIL(code)                                                                             \
    do {                                                                                           \
        rc = (code);                                                                               \
        goto out;                                                                                  \
    } while (0)
#define SYM_HIP(expr)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            srt_set_error("HIP error %s at %s:%d (%s)", hipGetErrorString(e_), __FILE__,           \
                          __LINE__, #expr);                                                        \
            SYM_FAIL(SRT_E_DEVICE);                                                                \
        }                                                                                          \
    } while (0)
    {
        if (!ok) {
            srt_set_error("sharded symmetric FW: scratch allocation failed");
            SYM_FAIL(SRT_E_NOMEM);
        }
        if (nrows > 0)
            fw16_init_kernel<<<dim3(srt_ceil_div(ld, 2048), nrows), 256, 0, st>>>(n, ld, row0, w_rows,
                                                                               d, CAP_F);
        SYM_HIP(hipGetLastError());
        SYM_HIP(hipEventRecord(sc->init_done, st));
        SYM_HIP(hipStreamWaitEvent(cs, sc->init_done, 0));
        auto panel_of = [&](int k) -> u16* { return pbuf[k & 1]; };
        /* on cs: assemble P_k from every rank's blocks (its tiles' round k-1 values are final),
         * then every rank closes the diagonal block and updates the row panel itself; the owner
         * also writes the result back into its pivot rows */
        auto produce = [&](int k) -> int {
            const int k0 = k * KB, K = k0 / 128, o = own[K];
            /* P was last read by round k-2's rest launches, which precede round k-1's next-row
             * launches on both update streams; cs waited for those (e_set), so it is free */
            u16* P = pbuf[k & 1];
            for (int q = 0; q < R; q++) cnt[q] = 0;
            for (int J = 0; J < T; J++) cnt[sym_kept(K, J) ? o : own[J]]++;
            if (cnt[me])
                sym_contrib_pack_kernel<<<T, 256, 0, cs>>>(d, ld, row0, tb, K, k0, T, down, me, grecv);
            SRT_HIPCHK(hipGetLastError());
            int r = srt_coll_group_begin(comm);
            size_t off = 0;
            for (int q = 0; q < R && !r; q++) {
                if (cnt[q])
                    r = srt_coll_bcast(comm, grecv + off * blk, (size_t)cnt[q] * blk * sizeof(u16), q, cs);
                off += (size_t)cnt[q];
            }
            const int r2 = srt_coll_group_end(comm);
            if (r || r2) return r ? r : r2;
            /* straight from the staged blocks: closure, then row panel (+ the owner's rows) */
            u16* prow = me == o ? d + (size_t)(k0 - row0) * ld : nullptr;
            sym_diag_stage_kernel<<<1, 256, 0, cs>>>(P, ld, K, k0, T, down, grecv, prow);
            sym_panel_stage_kernel<SYM_RM><<<T, 1024 / SYM_RM, 0, cs>>>(P, ld, K, k0, T, down, grecv, prow);
            SRT_HIPCHK(hipGetLastError());
            SRT_HIPCHK(hipEventRecord(sc->ready[k & 1], cs));
            return SRT_OK;
        };
        /* 128-pivot rounds: the band of tile row K (rows a, then b) is staged and broadcast as
         * two half-panels; every rank closes P_a, applies it to the staged b rows
         * (sym_cross_stage_kernel), then closes P_b -- P = P_a over P_b, 128 x ld */
        auto produce128 = [&](int k) -> int {
            const int k0 = k * 128, K = k, o = own[K];
            u16* P = pbuf[k & 1];
            u16* sa = grecv;
            u16* sb = grecv + ((size_t)T + 1) * blk;
            for (int q = 0; q < R; q++) cnt[q] = 0;
            for (int J = 0; J < T; J++) cnt[sym_kept(K, J) ? o : own[J]]++;
            if (cnt[me]) /* both halves in one launch */
                sym_contrib_pack_kernel<<<2 * T, 256, 0, cs>>>(d, ld, row0, tb, K, k0, T, down, me, sa,
                                                               sb);
            SRT_HIPCHK(hipGetLastError());
            int r = srt_coll_group_begin(comm);
            size_t off = 0;
            for (int q = 0; q < R && !r; q++) {
                if (cnt[q]) {
                    const size_t bytes = (size_t)cnt[q] * blk * sizeof(u16);
                    r = srt_coll_bcast(comm, sa + off * blk, bytes, q, cs);
                    if (!r) r = srt_coll_bcast(comm, sb + off * blk, bytes, q, cs);
                }
                off += (size_t)cnt[q];
            }
            const int r2 = srt_coll_group_end(comm);
            if (r || r2) return r ? r : r2;
            u16* prow_a = me == o ? d + (size_t)(k0 - row0) * ld : nullptr;
            u16* prow_b = prow_a ? prow_a + (size_t)KB * ld : nullptr;
            u16* Pb = P + (size_t)KB * ld;
            sym_diag_stage_kernel<<<1, 256, 0, cs>>>(P, ld, K, k0, T, down, sa, prow_a);
            sym_panel_stage_kernel<SYM_RM><<<T, 1024 / SYM_RM, 0, cs>>>(P, ld, K, k0, T, down, sa, prow_a);
            sym_cross_stage_kernel<SYM_RM><<<T, 1024 / SYM_RM, 0, cs>>>(P, ld, K, T, down, sb, K, 0);
            sym_diag_stage_kernel<<<1, 256, 0, cs>>>(Pb, ld, K, k0 + KB, T, down, sb, prow_b);
            sym_panel_stage_kernel<SYM_RM><<<T, 1024 / SYM_RM, 0, cs>>>(Pb, ld, K, k0 + KB, T, down, sb, prow_b);
            SRT_HIPCHK(hipGetLastError());
            SRT_HIPCHK(hipEventRecord(sc->ready[k & 1], cs));
            return SRT_OK;
        };
        auto make = [&](int k) -> int { return r128 ? produce128(k) : produce(k); };
        /* two update streams (st: even J, xs: odd J), as on one GPU (fw16_build_sym): each
         * depends on its own launches and the panel, so their rounds overlap */
        hipStream_t ss[2] = {st, sc->xs};
        const uint32_t* tls[2] = {tl, tl + nset[0]};
        SYM_HIP(hipStreamWaitEvent(sc->xs, sc->init_done, 0));
        if (deep) {
            /* Two-deep rounds. Band j (tile row j, rows a then b) is packed from the real tiles
             * after round j - 3's update (panels <= j - 3; the update of round j - 2 may already
             * be writing them -- every value read is a real path length no larger than what the
             * round needs, as with the two update streams), broadcast on the band stream ms, and
             * takes P_{j-2} and P_{j-1} on arrival (fwq_band_kernel, on cs) before it is closed
             * into P_j. The broadcast then has a whole round of the update to hide under, and the
             * chain from P_k to P_{k+1} is one band apply plus the closures. The update launches
             * cover every kept tile (no cross exclusions): the pivot rows take their own closed
             * panel there (min-plus with a closed panel is idempotent), so the closures write no
             * pivot rows. */
            hipStream_t ms = sc->ms;
            auto sa_of = [&](int j) { return grecv + (size_t)(j % 3) * 2 * ((size_t)T + 1) * blk; };
            auto sb_of = [&](int j) { return sa_of(j) + ((size_t)T + 1) * blk; };
            auto send = [&](int j) -> int { /* on ms: pack band j, broadcast, mark its arrival */
                const int o = own[j];
                u16* sa = sa_of(j);
                u16* sb = sb_of(j);
                for (int q = 0; q < R; q++) cnt[q] = 0;
                for (int J = 0; J < T; J++) cnt[sym_kept(j, J) ? o : own[J]]++;
                if (cnt[me])
                    sym_contrib_pack_kernel<<<2 * T, 256, 0, ms>>>(d, ld, row0, tb, j, j * 128, T, down,
                                                                   me, sa, sb);
                SRT_HIPCHK(hipGetLastError());
                int r = srt_coll_group_begin(comm);
                size_t off = 0;
                for (int q = 0; q < R && !r; q++) {
                    if (cnt[q]) {
                        const size_t bytes = (size_t)cnt[q] * blk * sizeof(u16);
                        r = srt_coll_bcast(comm, sa + off * blk, bytes, q, ms);
                        if (!r) r = srt_coll_bcast(comm, sb + off * blk, bytes, q, ms);
                    }
                    off += (size_t)cnt[q];
                }
                const int r2 = srt_coll_group_end(comm);
                if (r || r2) return r ? r : r2;
                SRT_HIPCHK(hipEventRecord(sc->arr[j % 3], ms));
                return SRT_OK;
            };
            auto close = [&](int j) -> int { /* on cs: the staged band j (complete) -> P_j */
                const int j0 = j * 128;
                u16* P = pbuf[j & 1];
                u16* Pb = P + (size_t)KB * ld;
                u16* sa = sa_of(j);
                u16* sb = sb_of(j);
                sym_diag_stage_kernel<<<1, 256, 0, cs>>>(P, ld, j, j0, T, down, sa, nullptr);
                sym_panel_stage_kernel<SYM_RM><<<T, 1024 / SYM_RM, 0, cs>>>(P, ld, j, j0, T, down, sa, nullptr);
                sym_cross_stage_kernel<SYM_RM><<<T, 1024 / SYM_RM, 0, cs>>>(P, ld, j, T, down, sb, j, 0);
                sym_diag_stage_kernel<<<1, 256, 0, cs>>>(Pb, ld, j, j0 + KB, T, down, sb, nullptr);
                sym_panel_stage_kernel<SYM_RM><<<T, 1024 / SYM_RM, 0, cs>>>(Pb, ld, j, j0 + KB, T, down, sb, nullptr);
                SRT_HIPCHK(hipGetLastError());
                SRT_HIPCHK(hipEventRecord(sc->ready[j & 1], cs));
                return SRT_OK;
            };
            /* P_k into the staged band j: the band's last panel (j = k + 1) on cs, on the chain from
             * P_k to P_{k+1}; its first (j = k + 2) on the band stream ms, which has broadcast the
             * band and then idles until round k's update ends (its next send): off the chain, and
             * no fifth stream (four hardware queues per process: a fifth would share one, and a
             * wait there stalls an update stream). The last apply of band j waits for it
             * (applied[j]). */
            auto apply = [&](int k, int j) -> int {
                hipStream_t as = j == k + 1 ? cs : ms;
                if (j == k + 1) {
                    SRT_HIPCHK(hipStreamWaitEvent(cs, sc->arr[j % 3], 0));
                    if (j >= 2) SRT_HIPCHK(hipStreamWaitEvent(cs, sc->applied[j % 3], 0));
                } else {
                    SRT_HIPCHK(hipStreamWaitEvent(ms, sc->ready[k & 1], 0));
                }
                fwq_band_kernel<<<T, 512, 0, as>>>(pbuf[k & 1], ld, j, T, down, sa_of(j), sb_of(j));
                SRT_HIPCHK(hipGetLastError());
                if (j == k + 2) SRT_HIPCHK(hipEventRecord(sc->applied[j % 3], ms));
                return SRT_OK;
            };
            SYM_HIP(hipStreamWaitEvent(ms, sc->init_done, 0));
            for (int j = 0; j < 3 && j < nb; j++)
                if ((rc = send(j))) goto out;
            SYM_HIP(hipStreamWaitEvent(cs, sc->arr[0], 0));
            if ((rc = close(0))) goto out;
            int timed = 0;
            for (int k = 0; k < nb; ++k) {
                u16* P = panel_of(k);
                const bool next = k + 1 < nb;
                const bool t_first = evp && next && timed == 0, t_last = evp && k + 2 == nb;
                if (evp && next) {
                    evp->group = 4;
                    evp->used = 4 * ++timed;
                }
                for (int p = 0; p < 2; p++) {
                    SYM_HIP(hipStreamWaitEvent(ss[p], sc->ready[k & 1], 0));
                    if (t_first) SYM_HIP(hipEventRecord(evp->ev[p], ss[p]));
                    if (nset[p])
                        fwq_update_kernel<true, 5, 4><<<(unsigned)nset[p], 512, 0, ss[p]>>>(
                            d, ld, P, k * 128, T, tb, -1, tls[p], te);
                    if (t_last) SYM_HIP(hipEventRecord(evp->ev[evp->used - 2 + p], ss[p]));
                    SYM_HIP(hipEventRecord(sc->e_set[k & 1][p], ss[p]));
                }
                SYM_HIP(hipGetLastError());
                /* band stream: P_k into band k + 2 (arrived), then band k + 3 once round k's
                 * update has (at least) passed over its tiles */
                if (k + 2 < nb && (rc = apply(k, k + 2))) goto out;
                if (k + 3 < nb) {
                    SYM_HIP(hipStreamWaitEvent(ms, sc->e_set[k & 1][0], 0));
                    SYM_HIP(hipStreamWaitEvent(ms, sc->e_set[k & 1][1], 0));
                    if ((rc = send(k + 3))) goto out;
                }
                if (!next) continue;
                if ((rc = apply(k, k + 1))) goto out;
                if (k >= 1) { /* P_{k+1} overwrites P_{k-1}: its update launches are done */
                    SYM_HIP(hipStreamWaitEvent(cs, sc->e_set[(k - 1) & 1][0], 0));
                    SYM_HIP(hipStreamWaitEvent(cs, sc->e_set[(k - 1) & 1][1], 0));
                }
                if ((rc = close(k + 1))) goto out;
            }
        } else {
        if ((rc = make(0))) goto out;
        /* Host enqueue order per round: next-row launches, the rest launches, then the next
         * panel on cs. At N ranks a round is ~100 us of GPU work and ~20 HIP calls, so the host
         * is the bottleneck if the bulk update waits behind the chain's calls; the chain kernels
         * run at raised wave priority wherever they land (FW_CHAIN_PRIO). */
        int timed = 0; /* rounds timed as one unit: the first start and the last end (evpool) */
        /* The next pivot row's cross runs on the chain stream (after both streams' rest of the
         * round before, whose tiles it follows), so the update streams run their rest launches
         * back to back instead of NR -> rest with two launch gaps a round: one rank of N = 8
         * 49.2 -> 46.0 ms, N = 4 unchanged (83.5 ms). (retired one-GPU NRCS form) keeps NR on the update
         * streams. */
        for (int k = 0; k < nb; ++k) {
            const int k0 = k * kbr;
            u16* P = panel_of(k);
            const bool next = k + 1 < nb;
            const int K1 = next ? (k + 1) * kbr / 128 : -1;
            for (int p = 0; p < 2; p++) SYM_HIP(hipStreamWaitEvent(ss[p], sc->ready[k & 1], 0));
            /* the unit's period only needs the first round's starts and the last round's ends
             * (evpool_sum, group 4): two records per round fewer on the host's critical path */
            const bool t_first = evp && next && timed == 0, t_last = evp && k + 2 == nb;
            if (evp && next) {
                evp->group = 4;
                evp->used = 4 * ++timed;
            }
            for (int p = 0; p < 2; p++) {
                if (t_first) SYM_HIP(hipEventRecord(evp->ev[p], ss[p]));
                if (nset[p] && r128) {
                    if (next)
                        fwq_update_kernel<true, 4, 4><<<(unsigned)nset[p], 512, 0, ss[p]>>>(
                            d, ld, P, k0, T, tb, K1, tls[p], te);
                    else
                        fwq_update_kernel<true, 5, 4><<<(unsigned)nset[p], 512, 0, ss[p]>>>(
                            d, ld, P, k0, T, tb, -1, tls[p], te);
                } else if (nset[p]) {
                    if (next)
                        FW_UPDATE(true, 4, (unsigned)nset[p], ss[p],
                            d, ld, P, k0, T, tb, K1, tls[p], te);
                    else
                        FW_UPDATE(true, 5, (unsigned)nset[p], ss[p],
                            d, ld, P, k0, T, tb, -1, tls[p], te);
                }
                if (t_last) SYM_HIP(hipEventRecord(evp->ev[evp->used - 2 + p], ss[p]));
            }
            SYM_HIP(hipGetLastError());
            /* rest(k) done: round k + 1's cross follows it on the chain stream */
            for (int p = 0; p < 2; p++) SYM_HIP(hipEventRecord(sc->e_set[k & 1][p], ss[p]));
            if (next) {
                /* the cross of K1 was last updated by rest(k - 1); P of round k + 1's buffer was
                 * last read by rest(k - 1) and the cross of round k - 1 (on cs) */
                if (k >= 1) {
                    SYM_HIP(hipStreamWaitEvent(cs, sc->e_set[(k - 1) & 1][0], 0));
                    SYM_HIP(hipStreamWaitEvent(cs, sc->e_set[(k - 1) & 1][1], 0));
                }
                if (r128)
                    fwq_update_kernel<true, 3, 4><<<T + (te - tb), 512, 0, cs>>>(d, ld, P, k0, T, tb,
                                                                                K1, nullptr, te);
                else
                    FW_UPDATE(true, 3, T + (te - tb), cs, d, ld, P, k0, T, tb, K1, nullptr, te);
                SYM_HIP(hipGetLastError());
                if ((rc = make(k + 1))) goto out;
            }
        }
        } /* one-deep rounds */
        SYM_HIP(hipEventRecord(sc->xs_done[0], sc->xs));
        SYM_HIP(hipStreamWaitEvent(st, sc->xs_done[0], 0));
        /* fill the tiles this rank does not keep: transposes from their keepers */
        {
            size_t nloc = 0;
            size_t* scount = (size_t*)calloc((size_t)R, sizeof(size_t));
            size_t* rcount = (size_t*)calloc((size_t)R, sizeof(size_t));
            if (!scount || !rcount) {
                free(scount);
                free(rcount);
                SYM_FAIL(SRT_E_NOMEM);
            }
            for (int q = 0; q < R; q++) {
                for (int I = tb; I < te; I++) /* this rank keeps (I, J), J in q's rows */
                    for (int J = qtb[q]; J < qte[q]; J++)
                        if (I != J && sym_kept(I, J)) (q == me ? nloc : scount[q])++;
                if (q != me)
                    for (int I = qtb[q]; I < qte[q]; I++) /* q keeps (I, J), J in this rank's rows */
                        for (int J = tb; J < te; J++)
                            if (sym_kept(I, J)) rcount[q]++;
            }
            size_t stot = 0, rtot = 0;
            for (int q = 0; q < R; q++) {
                stot += scount[q];
                rtot += rcount[q];
            }
            const size_t npairs = nloc + stot + rtot;
            uint32_t* hp = (uint32_t*)malloc((npairs + 1) * sizeof(uint32_t));
            uint32_t* dp = NULL;
            u16* fsend = NULL;
            u16* frecv = NULL;
            const size_t tile = 128 * 128;
            bool fok = hp && hipMalloc(&dp, (npairs + 1) * sizeof(uint32_t)) == hipSuccess &&
                       hipMalloc(&fsend, (stot + 1) * tile * sizeof(u16)) == hipSuccess &&
                       hipMalloc(&frecv, (rtot + 1) * tile * sizeof(u16)) == hipSuccess;
            if (fok) {
                /* layout of hp: local pairs, then send pairs by peer, then receive pairs by peer */
                size_t o = 0;
                for (int I = tb; I < te; I++)
                    for (int J = tb; J < te; J++)
                        if (I != J && sym_kept(I, J)) hp[o++] = ((uint32_t)I << 16) | (uint32_t)J;
                for (int q = 0; q < R; q++)
                    if (q != me)
                        for (int I = tb; I < te; I++)
                            for (int J = qtb[q]; J < qte[q]; J++)
                                if (sym_kept(I, J)) hp[o++] = ((uint32_t)I << 16) | (uint32_t)J;
                for (int q = 0; q < R; q++)
                    if (q != me)
                        for (int I = qtb[q]; I < qte[q]; I++)
                            for (int J = tb; J < te; J++)
                                if (sym_kept(I, J)) hp[o++] = ((uint32_t)I << 16) | (uint32_t)J;
                fok = hipMemcpyAsync(dp, hp, npairs * sizeof(uint32_t), hipMemcpyHostToDevice, st) ==
                      hipSuccess;
                /* the copy reads pageable host memory: finish it before hp is freed */
                fok = fok && hipStreamSynchronize(st) == hipSuccess;
            }
            if (fok) {
                if (nloc) sym_fill_local_kernel<<<(unsigned)nloc, 256, 0, st>>>(d, ld, tb, dp);
                if (stot)
                    sym_fill_pack_kernel<<<(unsigned)stot, 256, 0, st>>>(d, ld, tb, dp + nloc, fsend);
                size_t so = 0, ro = 0;
                for (int q = 0; q < R; q++) {
                    sp[q] = fsend + so * tile;
                    sbytes[q] = q == me ? 0 : scount[q] * tile * sizeof(u16);
                    rp[q] = frecv + ro * tile;
                    rbytes[q] = q == me ? 0 : rcount[q] * tile * sizeof(u16);
                    so += q == me ? 0 : scount[q];
                    ro += q == me ? 0 : rcount[q];
                }
                fok = hipGetLastError() == hipSuccess;
                if (fok && srt_comm_is_solo(comm)) /* timing only: see grecv */
                    fok = hipMemsetD16Async((hipDeviceptr_t)frecv, 3, (rtot + 1) * tile, st) ==
                          hipSuccess;
                if (fok && (rc = srt_coll_exchange(comm, sp, sbytes, rp, rbytes, st))) fok = false;
                if (fok && rtot)
                    sym_fill_unpack_kernel<<<(unsigned)rtot, 256, 0, st>>>(d, ld, tb,
                                                                          dp + nloc + stot, frecv);
                fok = fok && hipGetLastError() == hipSuccess &&
                      hipStreamSynchronize(st) == hipSuccess;
            }
            if (dp) (void)hipFree(dp);
            if (fsend) (void)hipFree(fsend);
            if (frecv) (void)hipFree(frecv);
            free(hp);
            free(scount);
            free(rcount);
            if (!fok) {
                if (!rc) {
                    srt_set_error("sharded symmetric FW: final fill failed");
                    rc = SRT_E_DEVICE;
                }
                goto out;
            }
        }
        SYM_HIP(hipMemsetAsync(flags[dev], 0, 2 * sizeof(int), st));
        if (nrows > 0)
            fw16_finish_kernel<<<dim3(srt_ceil_div(ld, 2048), nrows), 256, 0, st>>>(
                n, ld, row0, d, lat_rows, flags[dev], CAP_F);
        SYM_HIP(hipGetLastError());
        int hf[2] = {0, 0};
        SYM_HIP(hipMemcpyAsync(hf, flags[dev], 2 * sizeof(int), hipMemcpyDeviceToHost, st));
        SYM_HIP(hipStreamSynchronize(st));
        *exact = hf[0] ? 0 : 1;
        fw16_small[dev] = hf[1] ? 0 : 1;
    }
out:
#undef SYM_HIP
#undef SYM_FAIL
    (void)hipStreamSynchronize(cs);
    (void)hipStreamSynchronize(sc->ms);
    (void)hipStreamSynchronize(st);
    if (tl) (void)hipFree(tl);
    if (down) (void)hipFree(down);
    if (grecv) (void)hipFree(grecv);
    free(cnt);
    free(sp);
    free(rp);
    free(sbytes);
    free(rbytes);
    free(qtb);
    free(qte);
    free(own);
    free(hkept);
    return rc;
}

int srt_fw16_build_sym_sharded(const srt_comm* comm, int n, int ld, int row0, int nrows,
                               const uint32_t* w_rows, uint32_t* lat_rows, hipStream_t st,
                               evpool_t* evp, int* exact) {
    if (ld % 128 || nrows % 128 || row0 % 128 || srt_comm_size(comm) < 2 || ld / 128 > SYM_TMAX) {
        srt_set_error("sharded symmetric FW needs 128-aligned shards, two or more ranks and at "
                      "most %d tile columns", SYM_TMAX);
        return SRT_E_ARG;
    }
    /* 128-pivot rounds with the 8-wave update (a 256-pivot form measured slower at N = 8: 57.6
     * vs 45.9 ms for one rank; 64-pivot rounds slower still) */
    const int rp = 128;
    g_sharded_rp = rp;
    return fw16_build_sym_sharded(comm, n, ld, row0, nrows, w_rows, lat_rows, st, evp, exact, rp);
}
int srt_fw16_sharded_round_pivots(void) { return g_sharded_rp; }

static int fw16_square(int n, int ld, const uint32_t* w, uint32_t* lat, hipStream_t st,
                       evpool_t* evp, int* exact);

/* Distances by bit-parallel Dial levels (levels.hip) into the u32 rows (and the level build's own
 * u8 rows) -- exact and small by construction. *nlev = the level that settled every pair, or 0
 * when the levels do not apply or miss their budget -- the caller then runs the FW. */
int srt_fw16_levels(const srt_comm* comm, int n, int ld, int row0, int nrows, int directed,
                    const uint32_t* w_rows, const double* r_rows, uint32_t* lat_rows,
                    hipStream_t st, evpool_t* evp, double fw_ms, int* nlev, int64_t* bytes) {
    *nlev = 0;
    *bytes = 0;
    /* the level post pass reads the build's own u8 rows, not the u16 FW matrix: none written */
    return srt_levels_build(comm, n, ld, row0, nrows, directed, w_rows, r_rows, lat_rows, fw_ms, st,
                            evp, nlev, bytes);
}

int srt_fw16_build(int n, int ld, int row0, int nrows, const uint32_t* w_rows, uint32_t* lat_rows,
                   hipStream_t st, evpool_t* evp, srt_owner_fn owner_of, srt_panel_bcast_fn bcast,
                   void* ctx, int rank, int fm, int* sym, int* exact) {
    if (ld % 128 || nrows % 128 || row0 % 128) {
        srt_set_error("u16 FW needs ld and the row shard to be multiples of 128");
        return SRT_E_ARG;
    }
    /* small matrices on one GPU (ld <= 2048, C2's 1,000 vertices): min-plus squaring to a fixed
     * point instead of ld / 64 latency-bound FW rounds; SRT_FORM square=0 keeps the rounds */
    if (fm && !bcast && !owner_of && row0 == 0 && nrows == ld && ld <= 2048 &&
        srt_form_int("square", 1) != 0) {
        if (sym) *sym = 5;
        return fw16_square(n, ld, w_rows, lat_rows, st, evp, exact);
    }
    u16** bufs = fw16_bufs;
    size_t* caps = fw16_caps;
    int** flags = fw16_flags;
    const int dev = srt_state_slot(); /* the device, or this virtual rank's slot */
    const size_t need = (size_t)nrows * ld + 2 * (size_t)KB * ld;
    if (caps[dev] < need) {
        if (bufs[dev]) SRT_HIPCHK(hipFree(bufs[dev]));
        SRT_HIPCHK(hipMalloc(&bufs[dev], need * sizeof(u16)));
        caps[dev] = need;
    }
    if (!flags[dev]) SRT_HIPCHK(hipMalloc(&flags[dev], 2 * sizeof(int)));
    fw16_sched* sc;
    int rc = sched_get(&sc, dev);
    if (rc) return rc;
    const bool lookahead = bcast != NULL;
    /* upper-triangle rounds: undirected graph, f16-compare path, the whole matrix on one GPU */
    const bool want_sym = sym && *sym && srt_form_int("sym", 1) != 0;
    if (sym) *sym = 0;
    if (want_sym && fm && !bcast && !owner_of && row0 == 0 && nrows == ld) {
        /* two update streams once the rounds are long enough to hide their event waits, with
         * 256-pivot rounds (128 where ld is not a multiple of 256): with the update's compute loop
         * at ~85% of the issue model, the per-tile C load, row sums, staging and store are what is
         * left to amortize, so the longest rounds measured fastest */
        const bool two = ld >= 8192;
        const int rp = two ? (ld % 256 == 0 ? 256 : 128) : 64;
        *sym = rp == 256 ? 4 : rp == 128 ? 3 : two ? 2 : 1;
        return fw16_build_sym(n, ld, w_rows, lat_rows, st, evp, exact, two, rp);
    }
    hipStream_t cs = lookahead ? sc->cs : st;
    u16* d = bufs[dev];
    u16* pbuf[2] = {bufs[dev] + (size_t)nrows * ld, bufs[dev] + (size_t)nrows * ld + (size_t)KB * ld};
    const uint32_t cap = fm ? CAP_F : CAP_U;
    auto panel = fm ? fw16_panel_kernel<true, false> : fw16_panel_kernel<false, false>;
    /* the update of round k0 on this shard's tile rows (i0, skip as in tile_row) */
    auto update = [&](unsigned grid, const u16* P, int k0, int ncol, int i0, int skip) {
        if (!fm)
            fw16_update_kernel<false><<<grid, 256, 0, st>>>(d, ld, P, k0, ncol, i0, skip, nullptr, 0);
        else
            fwq_update_kernel<false><<<grid, 512, 0, st>>>(d, ld, P, k0, ncol, i0, skip, nullptr, 0);
    };
    if (nrows > 0) {
        fw16_init_kernel<<<dim3(srt_ceil_div(ld, 2048), nrows), 256, 0, st>>>(n, ld, row0, w_rows, d,
                                                                           cap);
        SRT_HIPCHK(hipGetLastError());
    }
    const int nb = ld / KB, nrb = nrows / KB, ncol128 = ld / 128, nrow128 = nrows / 128;
    const int rounds = ld / KB;
    auto owner = [&](int k) { return owner_of ? owner_of(ctx, k * KB) : rank; };
    auto panel_of = [&](int k) -> u16* {
        return owner(k) == rank ? d + (size_t)(k * KB - row0) * ld : pbuf[k & 1];
    };
    /* critical-stream part of round k: owner closes the diagonal tile and the pivot-row panel,
     * then every rank takes part in the broadcast; P_k ready is signalled on cs */
    auto produce = [&](int k) -> int {
        u16* P = panel_of(k);
        if (owner(k) == rank) {
            (fm ? fw16_diag_kernel<true> : fw16_diag_kernel<false>)<<<1, 256, 0, cs>>>(P, ld, k * KB);
            panel<<<nb, 256, 0, cs>>>(d, ld, row0, nrb, P, k * KB, nb, 1, 0);
            SRT_HIPCHK(hipGetLastError());
        } else if (k >= 2 && lookahead) {
            SRT_HIPCHK(hipStreamWaitEvent(cs, sc->upd_done[k & 1], 0)); /* round k-2 read it */
        }
        if (bcast) {
            int r = bcast(ctx, P, (size_t)KB * ld * sizeof(u16), owner(k), cs);
            if (r) return r;
        }
        if (lookahead) SRT_HIPCHK(hipEventRecord(sc->ready[k & 1], cs));
        return SRT_OK;
    };
    if (lookahead) {
        SRT_HIPCHK(hipEventRecord(sc->init_done, st));
        SRT_HIPCHK(hipStreamWaitEvent(cs, sc->init_done, 0));
    }
    if ((rc = produce(0))) return rc;
    for (int k = 0; k < rounds; ++k) {
        const int k0 = k * KB;
        u16* P = panel_of(k);
        if (lookahead) SRT_HIPCHK(hipStreamWaitEvent(st, sc->ready[k & 1], 0));
        const bool next = k + 1 < rounds;
        const int skip =
            (lookahead && next && owner(k + 1) == rank) ? ((k + 1) * KB - row0) / 128 : -1;
        if (nrb > 0) {
            panel<<<nb + nrb, 256, 0, st>>>(d, ld, row0, nrb, P, k0, nb, 0, 1);
            if (evp) SRT_HIPCHK(hipEventRecord(evp->ev[evp->used++], st));
            if (skip >= 0) {
                update(ncol128, P, k0, ncol128, skip, -1);
                SRT_HIPCHK(hipEventRecord(sc->row_done, st));
                SRT_HIPCHK(hipStreamWaitEvent(cs, sc->row_done, 0));
                if ((rc = produce(k + 1))) return rc;
                if (nrow128 > 1)
                    update(ncol128 * (nrow128 - 1), P, k0, ncol128, 0, skip);
            } else {
                update(ncol128 * nrow128, P, k0, ncol128, 0, -1);
            }
            if (evp) SRT_HIPCHK(hipEventRecord(evp->ev[evp->used++], st));
            SRT_HIPCHK(hipGetLastError());
        }
        if (lookahead) SRT_HIPCHK(hipEventRecord(sc->upd_done[k & 1], st));
        if (next && skip < 0 && (rc = produce(k + 1))) return rc;
    }
    SRT_HIPCHK(hipMemsetAsync(flags[dev], 0, 2 * sizeof(int), st));
    if (nrows > 0)
        fw16_finish_kernel<<<dim3(srt_ceil_div(ld, 2048), nrows), 256, 0, st>>>(
            n, ld, row0, d, lat_rows, flags[dev], cap);
    SRT_HIPCHK(hipGetLastError());
    int hf[2] = {0, 0};
    SRT_HIPCHK(hipMemcpyAsync(hf, flags[dev], 2 * sizeof(int), hipMemcpyDeviceToHost, st));
    SRT_HIPCHK(hipStreamSynchronize(st));
    *exact = hf[0] ? 0 : 1;
    fw16_small[dev] = hf[1] ? 0 : 1;
    return SRT_OK;
}

/* ---- distance rows of a few sources on a dense graph (no all-pairs FW) -------------------- */
/* w16 = min(w, cap) (the B operand: every arc, the self-loop on the diagonal) */
__global__ void rows_w16_kernel(int ld, const uint32_t* __restrict__ w, u16* __restrict__ w16,
                                uint32_t cap) {
    const size_t i8 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (i8 >= (size_t)ld * ld) return;
    const uint4 a = *reinterpret_cast<const uint4*>(w + i8);
    const uint4 b = *reinterpret_cast<const uint4*>(w + i8 + 4);
    auto c = [&](uint32_t x) { return x < cap ? x : cap; };
    *reinterpret_cast<uint4*>(w16 + i8) = make_uint4(c(a.x) | (c(a.y) << 16), c(a.z) | (c(a.w) << 16),
                                                     c(b.x) | (c(b.y) << 16), c(b.z) | (c(b.w) << 16));
}

/* D_S row i = the arcs of source verts[i] (capped), 0 at the source; padding rows stay at cap */
__global__ void rows_init_kernel(int ld, int nsub, const int32_t* __restrict__ verts,
                                 const u16* __restrict__ w16, u16* __restrict__ ds, uint32_t cap) {
    const int i = blockIdx.y;
    const int j8 = (blockIdx.x * blockDim.x + threadIdx.x) * 8;
    if (j8 >= ld) return;
    uint4 v = make_uint4(cap | (cap << 16), cap | (cap << 16), cap | (cap << 16), cap | (cap << 16));
    int s = -1;
    if (i < nsub) {
        s = verts[i];
        v = *reinterpret_cast<const uint4*>(w16 + (size_t)s * ld + j8);
    }
    *reinterpret_cast<uint4*>(ds + (size_t)i * ld + j8) = v;
    if (s >= j8 && s < j8 + 8) ds[(size_t)i * ld + s] = 0;
}

/* sum of the rows (values only decrease: an unchanged sum is a fixed point) */
__global__ void rows_sum_kernel(size_t count, const u16* __restrict__ ds,
                                unsigned long long* __restrict__ sum) {
    unsigned long long acc = 0;
    for (size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; i < count;
         i += (size_t)gridDim.x * blockDim.x * 8) {
        const uint4 v = *reinterpret_cast<const uint4*>(ds + i);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) acc += (w4[q] & 0xFFFFu) + (w4[q] >> 16);
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0) atomicAdd(sum, acc);
}

/* Shortest-distance rows of nsub sources (device list dverts) on a dense graph with n vertices:
 * Bellman-Ford on u16 quanta, D_S <- min(D_S, D_S (x) W), in place (the update kernel of the FW,
 * fwq_update_kernel<false>, with A = the rows' own columns and B = the rows of W), until a pass
 * changes nothing. Each pass extends every path by at least one arc in pivot order, so it ends
 * after (fewest hops of a shortest path) + 1 passes; a complete graph's shortest paths have a few
 * hops. Cost nsub * n^2 per pass, against the FW's n^3: it wins for few sources (the attached
 * vertices, topology.c:1604-1656). ds: nsp x ld (nsp = nsub rounded up to 128); lat_rows: nsub x
 * ld u32 quanta. *exact = 0 when a real distance reached the cap (the caller runs the FW). */
int srt_fw16_rows(int n, int ld, int nsub, const int32_t* dverts, const uint32_t* w, u16* w16,
                  u16* ds, uint32_t* lat_rows, hipStream_t st, int* exact, int* small, int* passes) {
    if (ld % 128 || nsub < 1 || n > ld) {
        srt_set_error("srt_fw16_rows: bad arguments");
        return SRT_E_ARG;
    }
    const int dev = srt_state_slot();
    const int nsp = srt_ceil_div(nsub, 128) * 128, T = ld / 128;
    const size_t ll = (size_t)ld * ld;
    rows_w16_kernel<<<(unsigned)srt_ceil_div((long long)(ll / 8), 256), 256, 0, st>>>(ld, w, w16, CAP_F);
    rows_init_kernel<<<dim3(srt_ceil_div(ld, 2048), nsp), 256, 0, st>>>(ld, nsub, dverts, w16, ds, CAP_F);
    SRT_HIPCHK(hipGetLastError());
    unsigned long long* dsum = nullptr;
    SRT_HIPCHK(srt_malloc_async((void**)&dsum, sizeof(unsigned long long), st));
    struct freer {
        unsigned long long* p;
        hipStream_t s;
        ~freer() { (void)hipFreeAsync(p, s); }
    } fr{dsum, st};
    unsigned long long prev = ~0ull;
    int it = 0;
    for (; it < n + 1; ++it) {
        for (int k0 = 0; k0 < ld; k0 += 256) {
            if (k0 + 256 <= ld)
                fwq_update_kernel<false, 0, 8><<<(unsigned)(nsp / 128 * T), 512, 0, st>>>(
                    ds, ld, w16 + (size_t)k0 * ld, k0, T, 0, -1, nullptr, 0);
            else
                fwq_update_kernel<false, 0, 4><<<(unsigned)(nsp / 128 * T), 512, 0, st>>>(
                    ds, ld, w16 + (size_t)k0 * ld, k0, T, 0, -1, nullptr, 0);
        }
        SRT_HIPCHK(hipMemsetAsync(dsum, 0, sizeof(unsigned long long), st));
        rows_sum_kernel<<<256, 256, 0, st>>>((size_t)nsp * ld, ds, dsum);
        SRT_HIPCHK(hipGetLastError());
        unsigned long long cur = 0;
        SRT_HIPCHK(hipMemcpyAsync(&cur, dsum, sizeof(cur), hipMemcpyDeviceToHost, st));
        SRT_HIPCHK(hipStreamSynchronize(st));
        if (cur == prev) break;
        prev = cur;
    }
    if (passes) *passes = it + 1;
    int* flags = fw16_flags[dev];
    if (!flags) {
        SRT_HIPCHK(hipMalloc(&fw16_flags[dev], 2 * sizeof(int)));
        flags = fw16_flags[dev];
    }
    SRT_HIPCHK(hipMemsetAsync(flags, 0, 2 * sizeof(int), st));
    fw16_finish_kernel<<<dim3(srt_ceil_div(ld, 2048), nsub), 256, 0, st>>>(n, ld, 0, ds, lat_rows, flags,
                                                                          CAP_F);
    SRT_HIPCHK(hipGetLastError());
    int hf[2] = {0, 0};
    SRT_HIPCHK(hipMemcpyAsync(hf, flags, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
    SRT_HIPCHK(hipStreamSynchronize(st));
    *exact = hf[0] ? 0 : 1;
    if (small) *small = hf[1] ? 0 : 1;
    return SRT_OK;
}

/* Min-plus squaring to a fixed point on one GPU: D <- min(D, D (x) D) in place, every tile and
 * every pivot per pass (the update kernel with A and B both from D), until a pass changes
 * nothing. Values only decrease and are always lengths of real paths, so the concurrent in-place
 * reads are harmless (as in the FW rounds); a pass that changes nothing leaves D = min(D, D (x) D)
 * with a zero diagonal, which is the closure. Pass p covers every path of up to 2^p arcs (more,
 * with the in-place updates), so a graph whose shortest paths have h arcs takes about
 * log2(h) + 2 passes of four launches: for small n that replaces ld / 64 FW rounds, each a chain
 * of dependent launches (C2: 16 rounds). */
static __device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    return min(a & 0xFFFFu, b & 0xFFFFu) | (min(a >> 16, b >> 16) << 16);
}

/* D = min over q < nq of the split-k partials (each already <= D); flag: any entry changed.
 * NQ > 0: the partial count is a compile-time constant and all loads issue together */
template <int NQ>
__global__ void sq_reduce_kernel(size_t count, int nq, const u16* __restrict__ part,
                                 u16* __restrict__ d, int* __restrict__ flag) {
    if (NQ > 0) nq = NQ;
    bool ch = false;
    for (size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 8; i < count;
         i += (size_t)gridDim.x * blockDim.x * 8) {
        uint4 m = *reinterpret_cast<const uint4*>(part + i);
#pragma unroll
        for (int q = 1; q < (NQ > 0 ? NQ : nq); ++q) {
            const uint4 x = *reinterpret_cast<const uint4*>(part + (size_t)q * count + i);
            m.x = pk_min_u16(m.x, x.x);
            m.y = pk_min_u16(m.y, x.y);
            m.z = pk_min_u16(m.z, x.z);
            m.w = pk_min_u16(m.w, x.w);
        }
        const uint4 o = *reinterpret_cast<const uint4*>(d + i);
        if (m.x != o.x || m.y != o.y || m.z != o.z || m.w != o.w) {
            *reinterpret_cast<uint4*>(d + i) = m;
            ch = true;
        }
    }
    /* one flag write per workgroup: same-address atomics serialise in L2 (one per wave over
     * 2048 waves cost 12 us of a 20 us pass at C2) */
    if (__syncthreads_or(ch) && threadIdx.x == 0) atomicOr(flag, 1);
}

static int fw16_square(int n, int ld, const uint32_t* w, uint32_t* lat, hipStream_t st,
                       evpool_t* evp, int* exact) {
    const int dev = srt_state_slot();
    const size_t need = (size_t)ld * ld + 2 * (size_t)KB * ld;
    if (fw16_caps[dev] < need) {
        if (fw16_bufs[dev]) SRT_HIPCHK(hipFree(fw16_bufs[dev]));
        SRT_HIPCHK(hipMalloc(&fw16_bufs[dev], need * sizeof(u16)));
        fw16_caps[dev] = need;
    }
    if (!fw16_flags[dev]) SRT_HIPCHK(hipMalloc(&fw16_flags[dev], 2 * sizeof(int)));
    u16* d = fw16_bufs[dev];
    int* flags = fw16_flags[dev];
    const int T = ld / 128;
    fw16_init_kernel<<<dim3(srt_ceil_div(ld, 2048), ld), 256, 0, st>>>(n, ld, 0, w, d, CAP_F);
    SRT_HIPCHK(hipGetLastError());
    unsigned long long* dsum = nullptr;
    SRT_HIPCHK(srt_malloc_async((void**)&dsum, 2 * sizeof(unsigned long long), st));
    struct freer {
        unsigned long long* p;
        hipStream_t s;
        ~freer() { (void)hipFreeAsync(p, s); }
    } fr{dsum, st};
    /* split-k: one launch per squaring over every (tile, 256-pivot block) -- T^2 ld / 256
     * workgroups, every CU busy at C2's T = 8 -- into per-block partials, then one reduce pass
     * that also says whether anything changed (an in-place form, one launch per 256-pivot block and
     * one workgroup per tile, used 64 workgroups on C2 and was retired in round 4) */
    const int nq8 = ld / 256, tail = (ld % 256) ? 1 : 0;
    int* sflag = reinterpret_cast<int*>(dsum); /* four change flags (dsum holds 16 bytes) */
    u16* part = nullptr;
    SRT_HIPCHK(srt_malloc_async((void**)&part, (size_t)(nq8 + tail) * ld * ld * 2, st));
    struct freer2 {
        u16* p;
        hipStream_t s;
        ~freer2() {
            if (p) (void)hipFreeAsync(p, s);
        }
    } fr2{part, st};
    /* timing (bench): the passes as one span, the first start to the end of the last checked
     * pass (evpool group 4, one unit per pass) -- no event records between passes */
    if (evp) {
        int rc = evpool_reserve(evp, 4 * 64);
        if (rc) return rc;
        evp->group = 4;
        evp->used = 0;
        SRT_HIPCHK(hipEventRecord(evp->ev[0], st));
        SRT_HIPCHK(hipEventRecord(evp->ev[1], st));
    }
    int hf[2] = {0, 0};
    bool finished = false;
    for (int it = 0; it < 64; ++it) {
        if (nq8)
            fwq_update_kernel<false, 20, 8><<<(unsigned)(T * T * nq8), 512, 0, st>>>(
                d, ld, d, 0, T, 0, 0, nullptr, 0, -1, part);
        if (tail)
            fwq_update_kernel<false, 20, 4><<<(unsigned)(T * T), 512, 0, st>>>(
                d, ld, d, nq8 * 256, T, 0, 0, nullptr, 0, -1, part + (size_t)nq8 * ld * ld);
        if (!(it & 3)) SRT_HIPCHK(hipMemsetAsync(sflag, 0, 4 * sizeof(int), st));
        const size_t cnt = (size_t)ld * ld;
        const unsigned rg = (unsigned)std::min<size_t>(256, srt_ceil_div((long long)(cnt / 8), 256));
        if (nq8 + tail == 4)
            sq_reduce_kernel<4><<<rg, 256, 0, st>>>(cnt, 4, part, d, sflag + (it & 3));
        else
            sq_reduce_kernel<0><<<rg, 256, 0, st>>>(cnt, nq8 + tail, part, d, sflag + (it & 3));
        SRT_HIPCHK(hipGetLastError());
        /* the change flags are read every fourth pass (one host round trip per four passes;
         * complete graphs converge in 3-4): a pass after the fixed point changes nothing and
         * costs only its time. The finish pass (u32 table, exactness and small-distance flags) is
         * enqueued with the check, so a converged squaring needs no second round trip; otherwise
         * its output is overwritten later. */
        if ((it & 3) != 3) continue;
        if (evp) {
            evp->used = 4 * (it + 1);
            SRT_HIPCHK(hipEventRecord(evp->ev[evp->used - 2], st));
            SRT_HIPCHK(hipEventRecord(evp->ev[evp->used - 1], st));
        }
        SRT_HIPCHK(hipMemsetAsync(flags, 0, 2 * sizeof(int), st));
        fw16_finish_kernel<<<dim3(srt_ceil_div(ld, 2048), ld), 256, 0, st>>>(n, ld, 0, d, lat,
                                                                            flags, CAP_F);
        SRT_HIPCHK(hipGetLastError());
        int ch[4] = {0, 0, 0, 0};
        SRT_HIPCHK(hipMemcpyAsync(ch, sflag, 4 * sizeof(int), hipMemcpyDeviceToHost, st));
        SRT_HIPCHK(hipMemcpyAsync(hf, flags, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
        SRT_HIPCHK(hipStreamSynchronize(st));
        if (!ch[0] || !ch[1] || !ch[2] || !ch[3]) {
            finished = true;
            break;
        }
    }
    if (!finished) {
        SRT_HIPCHK(hipMemsetAsync(flags, 0, 2 * sizeof(int), st));
        fw16_finish_kernel<<<dim3(srt_ceil_div(ld, 2048), ld), 256, 0, st>>>(n, ld, 0, d, lat, flags, CAP_F);
        SRT_HIPCHK(hipGetLastError());
        SRT_HIPCHK(hipMemcpyAsync(hf, flags, 2 * sizeof(int), hipMemcpyDeviceToHost, st));
        SRT_HIPCHK(hipStreamSynchronize(st));
    }
    *exact = hf[0] ? 0 : 1;
    fw16_small[dev] = hf[1] ? 0 : 1;
    return SRT_OK;
}
#endif /* SRT_FW16_DEVICE_ONLY */
