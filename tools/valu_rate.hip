// Issue rate of single VALU instructions on gfx950: 16 independent registers, inline asm, full
// occupancy (8 waves/SIMD), no other VALU in the loop. Reports cycles per wave64 instruction per
// SIMD at the clock measured with s_memtime/s_memrealtime inside the kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#define ITERS 4096

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define R16P(X, Y) X(0) Y(8) X(1) Y(9) X(2) Y(10) X(3) Y(11) X(4) Y(12) X(5) Y(13) X(6) Y(14) X(7) Y(15) \
    X(8) Y(0) X(9) Y(1) X(10) Y(2) X(11) Y(3) X(12) Y(4) X(13) Y(5) X(14) Y(6) X(15) Y(7)
#define KERNEL(NAME, ASM)                                                                    \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned long long* clk, unsigned s) { \
        unsigned x0 = s ^ threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,     \
                 x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7, x8 = x0 + 8, x9 = x0 + 9, x10 = x0 + 10, \
                 x11 = x0 + 11, x12 = x0 + 12, x13 = x0 + 13, x14 = x0 + 14, x15 = x0 + 15;     \
        unsigned y = s * 7 + threadIdx.x, z = s * 13 + threadIdx.x;                             \
        unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
        for (int it = 0; it < ITERS; it++) {                                                   \
            _Pragma("unroll") for (int q = 0; q < 1; q++) {                                    \
                R16(ASM)                                                                       \
            }                                                                                  \
        }                                                                                      \
        unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
        unsigned a = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ x8 ^ x9 ^ x10 ^ x11 ^ x12 ^ x13 ^ x14 ^ x15; \
        if (a == 0x9e3779b9u) out[threadIdx.x] = a;                                             \
        if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }       \
    }

#define A_PKADD(i) asm volatile("v_pk_add_u16 %0, %0, %1 clamp" : "+v"(x##i) : "v"(y));
#define A_PKMIN(i) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_ADD(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_MIN(i) asm volatile("v_min_u32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_MIN3(i) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define A_ADD3(i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define A_FMA(i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define A_PKFADD(i) asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_PKFMIN(i) asm volatile("v_pk_min_f16 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_ADDMIN(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x##i) : "v"(y)); asm volatile("v_min_u32 %0, %0, %1" : "+v"(x##i) : "v"(z));

#define A_SUB(i) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_MIN16(i) asm volatile("v_min_u16 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_MAX(i) asm volatile("v_max_u32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_MINF(i) asm volatile("v_min_f32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_ADDF(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_AND(i) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_MINI(i) asm volatile("v_min_i32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_PKMAXI(i) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_MED3(i) asm volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define A_LSHL(i) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(x##i));
#define A_PKFMA(i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(xx##i) : "v"(yy), "v"(zz));
#define A_MIN16HI(i) asm volatile("v_min_u16_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(x##i) : "v"(y));
#define A_ADD16(i) asm volatile("v_add_u16 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_MINF16(i) asm volatile("v_min_f16 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_MAX16(i) asm volatile("v_max_u16 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_CND(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x##i) : "v"(y) : "vcc");
#define A_MUL24(i) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_OR(i) asm volatile("v_or_b32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_XOR(i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_MAXF(i) asm volatile("v_max_f32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_MULF(i) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_SUBREV(i) asm volatile("v_subrev_u32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define A_MOV(i) asm volatile("v_mov_b32 %0, %1" : "=v"(x##i) : "v"(y));
#define KERNEL2(NAME, A1, A2)                                                                  \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned long long* clk, unsigned s) { \
        unsigned x0 = s ^ threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,     \
                 x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7, x8 = x0 + 8, x9 = x0 + 9, x10 = x0 + 10, \
                 x11 = x0 + 11, x12 = x0 + 12, x13 = x0 + 13, x14 = x0 + 14, x15 = x0 + 15;     \
        unsigned y = s * 7 + threadIdx.x, z = s * 13 + threadIdx.x;                             \
        unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
        for (int it = 0; it < ITERS / 2; it++) {                                               \
            R16P(A1, A2)                                                                       \
        }                                                                                      \
        unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
        unsigned a = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ x8 ^ x9 ^ x10 ^ x11 ^ x12 ^ x13 ^ x14 ^ x15; \
        if (a == 0x9e3779b9u) out[threadIdx.x] = a;                                             \
        if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }       \
    }
KERNEL2(m_add_pkmin, A_ADD, A_PKMIN)
KERNEL2(m_pkadd_pkmin, A_PKADD, A_PKMIN)
KERNEL2(m_add_min16, A_ADD, A_MIN16)
KERNEL2(m_min16_min16hi, A_MIN16, A_MIN16HI)
KERNEL2(m_add_min, A_ADD, A_MIN)
KERNEL2(m_add_add, A_ADD, A_SUB)
KERNEL(k_min16hi, A_MIN16HI)
KERNEL(k_add16, A_ADD16)
KERNEL(k_minf16, A_MINF16)
KERNEL(k_max16, A_MAX16)
KERNEL(k_cnd, A_CND)
KERNEL(k_mul24, A_MUL24)
KERNEL(k_or, A_OR)
KERNEL(k_xor, A_XOR)
KERNEL(k_maxf, A_MAXF)
KERNEL(k_mulf, A_MULF)
KERNEL(k_subrev, A_SUBREV)
KERNEL(k_sub, A_SUB)
KERNEL(k_min16, A_MIN16)
KERNEL(k_max, A_MAX)
KERNEL(k_minf, A_MINF)
KERNEL(k_addf, A_ADDF)
KERNEL(k_and, A_AND)
KERNEL(k_mini, A_MINI)
KERNEL(k_pkmaxi, A_PKMAXI)
KERNEL(k_med3, A_MED3)
KERNEL(k_lshl, A_LSHL)
KERNEL(k_pkadd, A_PKADD)
KERNEL(k_pkmin, A_PKMIN)
KERNEL(k_add, A_ADD)
KERNEL(k_min, A_MIN)
KERNEL(k_min3, A_MIN3)
KERNEL(k_add3, A_ADD3)
KERNEL(k_fma, A_FMA)
KERNEL(k_pkfadd, A_PKFADD)
KERNEL(k_pkfmin, A_PKFMIN)

typedef void (*kfn)(unsigned*, unsigned long long*, unsigned);
void run(const char* name, kfn f, int waves_per_simd, unsigned* out, unsigned long long* clk) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    int grid = 256 * waves_per_simd;  // 4-wave WGs, one wave per SIMD each
    f<<<grid, 256>>>(out, clk, 3);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) f<<<grid, 256>>>(out, clk, 3 + r);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    unsigned long long c[2]; hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    double ghz = (double)c[0] / (double)c[1] * 0.1;  // s_memrealtime ticks at 100 MHz
    double instr_per_simd = 5.0 * waves_per_simd * (double)ITERS * 16;
    double cyc = ms * 1e-3 * ghz * 1e9 / instr_per_simd;
    printf("%-14s waves/SIMD %d: %.3f ms, clock %.2f GHz, %.2f cycles per wave64 instr per SIMD\n",
           name, waves_per_simd, ms / 5, ghz, cyc);
}

int main() {
    unsigned* out; unsigned long long* clk;
    hipMalloc(&out, 4096); hipMalloc(&clk, 16);
    for (int w : {8, 4}) {
        run("v_add_u32", k_add, w, out, clk);
        run("v_pk_min_u16", k_pkmin, w, out, clk);
        run("v_min_u16", k_min16, w, out, clk);
        run("v_min_u16 sdwa hi", k_min16hi, w, out, clk);
        run("v_add_u16", k_add16, w, out, clk);
        run("v_max_u16", k_max16, w, out, clk);
        run("v_min_f16", k_minf16, w, out, clk);
        run("v_cndmask_b32", k_cnd, w, out, clk);
        run("v_mul_u32_u24", k_mul24, w, out, clk);
        run("v_or_b32", k_or, w, out, clk);
        run("v_xor_b32", k_xor, w, out, clk);
        run("v_max_f32", k_maxf, w, out, clk);
        run("v_mul_f32", k_mulf, w, out, clk);
        run("v_subrev_u32", k_subrev, w, out, clk);
        run("v_min_u32", k_min, w, out, clk);
        run("mix add+pkmin", m_add_pkmin, w, out, clk);
        run("mix pkadd+pkmin", m_pkadd_pkmin, w, out, clk);
        run("mix add+min16", m_add_min16, w, out, clk);
        run("mix min16+min16hi", m_min16_min16hi, w, out, clk);
        run("mix add+min", m_add_min, w, out, clk);
        run("mix add+sub", m_add_add, w, out, clk);
    }
    return 0;
}
