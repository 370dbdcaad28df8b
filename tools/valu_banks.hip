// Issue rate of the FW update's inner instruction stream (one pivot pair of fwq_rows: 16 add, add,
// pk_minimum3 triples over a 4x8 thread block) with hand-placed VGPRs, to see what VGPR bank
// placement costs: A = the compiler's placement in fwq_update_kernel (operand and temporary
// banks collide), B = operands and temporaries placed so no instruction reads two VGPRs of one
// bank (bank = register index mod 4). 8 or 4 waves per SIMD, as valu_rate2.hip.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 2048

#define CLOB "v0","v1","v2","v3","v4","v5","v6","v7","v8","v9","v10","v11","v12","v13","v14","v15", \
             "v16","v17","v18","v19","v20","v21","v22","v23","v24","v25","v26","v27","v28","v29","v30","v31", \
             "v32","v33","v34","v35","v36","v37","v38","v39","v40","v41","v42","v43","v44","v45","v46","v47", \
             "v48","v49","v50","v51","v52","v53","v54","v55"

#define T(acc, a, b, c, d, t0, t1) \
    "v_add_u32 v" #t0 ", v" #a ", v" #b "\n\tv_add_u32 v" #t1 ", v" #c ", v" #d \
    "\n\tv_pk_minimum3_f16 v" #acc ", v" #acc ", v" #t0 ", v" #t1 "\n\t"

/* A: acc v0-15 (row r: v4r..v4r+3), a[r] = (v16+2r, v17+2r), b0 = v24-27, b1 = v28-31, temps v32/v33 */
#define ROWA(r, acc0, ax, ay)                                   \
    T(acc0, ax, 24, ay, 28, 32, 33) T(acc0##1, ax, 25, ay, 29, 32, 33)
#define BODY_A \
    T(0, 16, 24, 17, 28, 32, 33) T(1, 16, 25, 17, 29, 32, 33) T(2, 16, 26, 17, 30, 32, 33) T(3, 16, 27, 17, 31, 32, 33) \
    T(4, 18, 24, 19, 28, 32, 33) T(5, 18, 25, 19, 29, 32, 33) T(6, 18, 26, 19, 30, 32, 33) T(7, 18, 27, 19, 31, 32, 33) \
    T(8, 20, 24, 21, 28, 32, 33) T(9, 20, 25, 21, 29, 32, 33) T(10, 20, 26, 21, 30, 32, 33) T(11, 20, 27, 21, 31, 32, 33) \
    T(12, 22, 24, 23, 28, 32, 33) T(13, 22, 25, 23, 29, 32, 33) T(14, 22, 26, 23, 30, 32, 33) T(15, 22, 27, 23, 31, 32, 33)
/* B: a[r].x in bank 0 (v32+4r), a[r].y in bank 1 (v33+4r); b0 = v26 v27 v30 v31, b1 = v18 v19 v22 v23
 * (banks 2/3); temps for an accumulator of bank k from banks k+1, k+2 (v48..v51) */
#define TB0(acc, ax, b, ay, d) T(acc, ax, b, ay, d, 49, 50)
#define TB1(acc, ax, b, ay, d) T(acc, ax, b, ay, d, 50, 51)
#define TB2(acc, ax, b, ay, d) T(acc, ax, b, ay, d, 51, 48)
#define TB3(acc, ax, b, ay, d) T(acc, ax, b, ay, d, 48, 49)
#define BODY_B \
    TB0(0, 32, 26, 33, 18) TB1(1, 32, 27, 33, 19) TB2(2, 32, 30, 33, 22) TB3(3, 32, 31, 33, 23) \
    TB0(4, 36, 26, 37, 18) TB1(5, 36, 27, 37, 19) TB2(6, 36, 30, 37, 22) TB3(7, 36, 31, 37, 23) \
    TB0(8, 40, 26, 41, 18) TB1(9, 40, 27, 41, 19) TB2(10, 40, 30, 41, 22) TB3(11, 40, 31, 41, 23) \
    TB0(12, 44, 26, 45, 18) TB1(13, 44, 27, 45, 19) TB2(14, 44, 30, 45, 22) TB3(15, 44, 31, 45, 23)
/* C: as B but the temporaries rotate over 8 registers (v48..v55), banks still apart */
#define BODY_C \
    T(0, 32, 26, 33, 18, 49, 50) T(1, 32, 27, 33, 19, 54, 55) T(2, 32, 30, 33, 22, 51, 48) T(3, 32, 31, 33, 23, 52, 53) \
    T(4, 36, 26, 37, 18, 49, 50) T(5, 36, 27, 37, 19, 54, 55) T(6, 36, 30, 37, 22, 51, 48) T(7, 36, 31, 37, 23, 52, 53) \
    T(8, 40, 26, 41, 18, 49, 50) T(9, 40, 27, 41, 19, 54, 55) T(10, 40, 30, 41, 22, 51, 48) T(11, 40, 31, 41, 23, 52, 53) \
    T(12, 44, 26, 45, 18, 49, 50) T(13, 44, 27, 45, 19, 54, 55) T(14, 44, 30, 45, 22, 51, 48) T(15, 44, 31, 45, 23, 52, 53)

/* D: C with s_nop 0 between the second add and the min3 (the compiler's separate-statement form) */
#define TN(acc, a, b, c, d, t0, t1) \
    "v_add_u32 v" #t0 ", v" #a ", v" #b "\n\tv_add_u32 v" #t1 ", v" #c ", v" #d \
    "\n\ts_nop 0\n\tv_pk_minimum3_f16 v" #acc ", v" #acc ", v" #t0 ", v" #t1 "\n\t"
#define BODY_D \
    TN(0, 32, 26, 33, 18, 49, 50) TN(1, 32, 27, 33, 19, 54, 55) TN(2, 32, 30, 33, 22, 51, 48) TN(3, 32, 31, 33, 23, 52, 53) \
    TN(4, 36, 26, 37, 18, 49, 50) TN(5, 36, 27, 37, 19, 54, 55) TN(6, 36, 30, 37, 22, 51, 48) TN(7, 36, 31, 37, 23, 52, 53) \
    TN(8, 40, 26, 41, 18, 49, 50) TN(9, 40, 27, 41, 19, 54, 55) TN(10, 40, 30, 41, 22, 51, 48) TN(11, 40, 31, 41, 23, 52, 53) \
    TN(12, 44, 26, 45, 18, 49, 50) TN(13, 44, 27, 45, 19, 54, 55) TN(14, 44, 30, 45, 22, 51, 48) TN(15, 44, 31, 45, 23, 52, 53)
/* E: two triples interleaved (4 adds, then the 2 min3s), temps of the pair in four banks */
#define TE(acc, a, b, c, d, t0, t1, acc2, a2, b2, c2, d2, t2, t3) \
    "v_add_u32 v" #t0 ", v" #a ", v" #b "\n\tv_add_u32 v" #t1 ", v" #c ", v" #d "\n\t" \
    "v_add_u32 v" #t2 ", v" #a2 ", v" #b2 "\n\tv_add_u32 v" #t3 ", v" #c2 ", v" #d2 "\n\t" \
    "v_pk_minimum3_f16 v" #acc ", v" #acc ", v" #t0 ", v" #t1 "\n\t" \
    "v_pk_minimum3_f16 v" #acc2 ", v" #acc2 ", v" #t2 ", v" #t3 "\n\t"
#define BODY_E \
    TE(0, 32, 26, 33, 18, 49, 50, 1, 32, 27, 33, 19, 54, 55) TE(2, 32, 30, 33, 22, 51, 48, 3, 32, 31, 33, 23, 52, 53) \
    TE(4, 36, 26, 37, 18, 49, 50, 5, 36, 27, 37, 19, 54, 55) TE(6, 36, 30, 37, 22, 51, 48, 7, 36, 31, 37, 23, 52, 53) \
    TE(8, 40, 26, 41, 18, 49, 50, 9, 40, 27, 41, 19, 54, 55) TE(10, 40, 30, 41, 22, 51, 48, 11, 40, 31, 41, 23, 52, 53) \
    TE(12, 44, 26, 45, 18, 49, 50, 13, 44, 27, 45, 19, 54, 55) TE(14, 44, 30, 45, 22, 51, 48, 15, 44, 31, 45, 23, 52, 53)
/* F: the pure-mix form of valu_rate2 (adds read the accumulator itself), in one block */
#define TF(acc, t0, t1) \
    "v_add_u32 v" #t0 ", v" #acc ", v26\n\tv_add_u32 v" #t1 ", v" #acc ", v18\n\t" \
    "v_pk_minimum3_f16 v" #acc ", v" #acc ", v" #t0 ", v" #t1 "\n\t"
#define BODY_F \
    TF(0, 49, 50) TF(1, 54, 55) TF(2, 51, 48) TF(3, 52, 53) TF(4, 49, 50) TF(5, 54, 55) TF(6, 51, 48) TF(7, 52, 53) \
    TF(8, 49, 50) TF(9, 54, 55) TF(10, 51, 48) TF(11, 52, 53) TF(12, 49, 50) TF(13, 54, 55) TF(14, 51, 48) TF(15, 52, 53)
#define BODY_FN \
    TF(0, 49, 50) "s_nop 0\n\t" TF(1, 54, 55) "s_nop 0\n\t" TF(2, 51, 48) "s_nop 0\n\t" TF(3, 52, 53) "s_nop 0\n\t" \
    TF(4, 49, 50) "s_nop 0\n\t" TF(5, 54, 55) "s_nop 0\n\t" TF(6, 51, 48) "s_nop 0\n\t" TF(7, 52, 53) "s_nop 0\n\t" \
    TF(8, 49, 50) "s_nop 0\n\t" TF(9, 54, 55) "s_nop 0\n\t" TF(10, 51, 48) "s_nop 0\n\t" TF(11, 52, 53) "s_nop 0\n\t" \
    TF(12, 49, 50) "s_nop 0\n\t" TF(13, 54, 55) "s_nop 0\n\t" TF(14, 51, 48) "s_nop 0\n\t" TF(15, 52, 53) "s_nop 0\n\t"

/* D1 / D2: s_nop 1 / s_nop 2 (two / three wait states) instead of s_nop 0 */
#define TN1(acc, a, b, c, d, t0, t1) \
    "v_add_u32 v" #t0 ", v" #a ", v" #b "\n\tv_add_u32 v" #t1 ", v" #c ", v" #d \
    "\n\ts_nop 1\n\tv_pk_minimum3_f16 v" #acc ", v" #acc ", v" #t0 ", v" #t1 "\n\t"
#define TN2(acc, a, b, c, d, t0, t1) \
    "v_add_u32 v" #t0 ", v" #a ", v" #b "\n\tv_add_u32 v" #t1 ", v" #c ", v" #d \
    "\n\ts_nop 2\n\tv_pk_minimum3_f16 v" #acc ", v" #acc ", v" #t0 ", v" #t1 "\n\t"
#define BODY_X(TT) \
    TT(0, 32, 26, 33, 18, 49, 50) TT(1, 32, 27, 33, 19, 54, 55) TT(2, 32, 30, 33, 22, 51, 48) TT(3, 32, 31, 33, 23, 52, 53) \
    TT(4, 36, 26, 37, 18, 49, 50) TT(5, 36, 27, 37, 19, 54, 55) TT(6, 36, 30, 37, 22, 51, 48) TT(7, 36, 31, 37, 23, 52, 53) \
    TT(8, 40, 26, 41, 18, 49, 50) TT(9, 40, 27, 41, 19, 54, 55) TT(10, 40, 30, 41, 22, 51, 48) TT(11, 40, 31, 41, 23, 52, 53) \
    TT(12, 44, 26, 45, 18, 49, 50) TT(13, 44, 27, 45, 19, 54, 55) TT(14, 44, 30, 45, 22, 51, 48) TT(15, 44, 31, 45, 23, 52, 53)
/* J: four groups' adds (8), then their four min3s: the nearest operand is written 4 slots back */
#define TJ(a0, ax, b0, ay, c0, t0, t1, a1, b1, c1, t2, t3, a2, b2, c2, t4, t5, a3, b3, c3, t6, t7, ax2, ay2) \
    "v_add_u32 v" #t0 ", v" #ax ", v" #b0 "\n\tv_add_u32 v" #t1 ", v" #ay ", v" #c0 "\n\t" \
    "v_add_u32 v" #t2 ", v" #ax ", v" #b1 "\n\tv_add_u32 v" #t3 ", v" #ay ", v" #c1 "\n\t" \
    "v_add_u32 v" #t4 ", v" #ax ", v" #b2 "\n\tv_add_u32 v" #t5 ", v" #ay ", v" #c2 "\n\t" \
    "v_add_u32 v" #t6 ", v" #ax ", v" #b3 "\n\tv_add_u32 v" #t7 ", v" #ay ", v" #c3 "\n\t" \
    "v_pk_minimum3_f16 v" #a0 ", v" #a0 ", v" #t0 ", v" #t1 "\n\t" \
    "v_pk_minimum3_f16 v" #a1 ", v" #a1 ", v" #t2 ", v" #t3 "\n\t" \
    "v_pk_minimum3_f16 v" #a2 ", v" #a2 ", v" #t4 ", v" #t5 "\n\t" \
    "v_pk_minimum3_f16 v" #a3 ", v" #a3 ", v" #t6 ", v" #t7 "\n\t"
#define BODY_J \
    TJ(0, 32, 26, 33, 18, 48, 49, 1, 27, 19, 50, 51, 2, 30, 22, 52, 53, 3, 31, 23, 54, 55, 0, 0) \
    TJ(4, 36, 26, 37, 18, 48, 49, 5, 27, 19, 50, 51, 6, 30, 22, 52, 53, 7, 31, 23, 54, 55, 0, 0) \
    TJ(8, 40, 26, 41, 18, 48, 49, 9, 27, 19, 50, 51, 10, 30, 22, 52, 53, 11, 31, 23, 54, 55, 0, 0) \
    TJ(12, 44, 26, 45, 18, 48, 49, 13, 27, 19, 50, 51, 14, 30, 22, 52, 53, 15, 31, 23, 54, 55, 0, 0)

#define INIT "v_mov_b32 v0, 0x30003000\n\tv_mov_b32 v1, v0\n\tv_mov_b32 v2, v0\n\tv_mov_b32 v3, v0\n\t" \
    "v_mov_b32 v4, v0\n\tv_mov_b32 v5, v0\n\tv_mov_b32 v6, v0\n\tv_mov_b32 v7, v0\n\t"              \
    "v_mov_b32 v8, v0\n\tv_mov_b32 v9, v0\n\tv_mov_b32 v10, v0\n\tv_mov_b32 v11, v0\n\t"             \
    "v_mov_b32 v12, v0\n\tv_mov_b32 v13, v0\n\tv_mov_b32 v14, v0\n\tv_mov_b32 v15, v0\n\t"
#define KERNEL(NAME, BODY)                                                                         \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned long long* clk) {         \
        unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
        asm volatile(INIT ::: CLOB);                                                               \
        for (int it = 0; it < ITERS; ++it) asm volatile(BODY ::: CLOB);                            \
        unsigned x;                                                                                \
        asm volatile("v_xor_b32 %0, v0, v15" : "=v"(x) :: CLOB);                                   \
        unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
        if (x == 0x9e3779b9u) out[threadIdx.x] = x;                                                \
        if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = c1 - c0; clk[1] = r1 - r0; }           \
    }
KERNEL(k_a, BODY_A)
KERNEL(k_b, BODY_B)
KERNEL(k_c, BODY_C)
KERNEL(k_d, BODY_D)
KERNEL(k_e, BODY_E)
KERNEL(k_f, BODY_F)
KERNEL(k_fn, BODY_FN)
KERNEL(k_d1, BODY_X(TN1))
KERNEL(k_d2, BODY_X(TN2))
KERNEL(k_j, BODY_J)

typedef void (*kfn)(unsigned*, unsigned long long*);
static void run(const char* name, kfn f, int w, unsigned* out, unsigned long long* clk) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = 256 * w;
    f<<<grid, 256>>>(out, clk);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) f<<<grid, 256>>>(out, clk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long c[2];
    hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / (double)c[1] * 0.1;
    /* per SIMD: 5 launches x w waves x ITERS x 16 triples x 4 relaxations (wave-level) */
    const double relax = 5.0 * w * ITERS * 16 * 4;
    printf("%-40s waves/SIMD %d: %.3f ms, s_memtime clock %.2f GHz, %.3f cycles/relax at 2.4 GHz "
           "(%.1f%% of the 2.0 model)\n", name, w, ms / 5, ghz, ms * 1e-3 * 2.4e9 / relax,
           100.0 * 2.0 / (ms * 1e-3 * 2.4e9 / relax));
}
int main() {
    unsigned* out;
    unsigned long long* clk;
    hipMalloc(&out, 4096);
    hipMalloc(&clk, 16);
    for (int w : {8, 4}) {
        run("A compiler placement (bank collisions)", k_a, w, out, clk);
        run("B bank-free operands and temps", k_b, w, out, clk);
        run("C bank-free, rotating temps", k_c, w, out, clk);
        run("D = C + s_nop 0 before each min3", k_d, w, out, clk);
        run("D1 = C + s_nop 1 before each min3", k_d1, w, out, clk);
        run("D2 = C + s_nop 2 before each min3", k_d2, w, out, clk);
        run("J = 8 adds then 4 min3s (4 back)", k_j, w, out, clk);
        run("E = C, two triples interleaved", k_e, w, out, clk);
        run("F adds read the accumulator (valu_rate2)", k_f, w, out, clk);
        run("F + s_nop 0 after each triple", k_fn, w, out, clk);
    }
    return 0;
}
