// Issue rates of the candidate min-plus instruction mixes on gfx950 (same method as valu_rate.hip:
// 16 independent register chains, inline asm, 4 or 8 waves per SIMD, cycles from s_memtime), plus
// an exactness check of v_pk_minimum3_f16 used as an unsigned min on u16 bit patterns in
// [0, 0x7BFF] (non-negative finite f16 values order like their bit patterns; denormals included).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define ITERS 4096

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define PROLOGUE                                                                                \
    unsigned x0 = s ^ threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,          \
             x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7, x8 = x0 + 8, x9 = x0 + 9, x10 = x0 + 10,      \
             x11 = x0 + 11, x12 = x0 + 12, x13 = x0 + 13, x14 = x0 + 14, x15 = x0 + 15;          \
    unsigned y = (s * 7 + threadIdx.x) & 0x3DFF3DFFu, z = (s * 13 + threadIdx.x) & 0x3DFF3DFFu;  \
    unsigned t0 = y, t1 = z;                                                                     \
    unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#define EPILOGUE                                                                                 \
    unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime(); \
    unsigned a = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ x8 ^ x9 ^ x10 ^ x11 ^ x12 ^ x13 ^ x14 ^ \
                 x15 ^ t0 ^ t1;                                                                  \
    if (a == 0x9e3779b9u) out[threadIdx.x] = a;                                                  \
    if (threadIdx.x == 0 && blockIdx.x == 0) {                                                   \
        clk[0] = c1 - c0;                                                                        \
        clk[1] = r1 - r0;                                                                        \
    }
/* one instruction per chain per iteration */
#define KERNEL1(NAME, OP)                                                                        \
    __global__ __launch_bounds__(256) void NAME(unsigned* out, unsigned long long* clk, unsigned s) { \
        PROLOGUE for (int it = 0; it < ITERS; it++) { R16(OP) } EPILOGUE                        \
    }

#define O_PKMIN3F(i) asm volatile("v_pk_minimum3_f16 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define O_PKADDF(i) asm volatile("v_pk_add_f16 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define O_PKMINF(i) asm volatile("v_pk_min_f16 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define O_MIN3U32(i) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define O_MIN3U16(i) asm volatile("v_min3_u16 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define O_PKMINU16(i) asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define O_ADD(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x##i) : "v"(y));
/* min-plus step as the update kernel would issue it: two adds into temporaries, one 3-input min */
#define O_ADD2_PKMIN3F(i)                                                                  \
    asm volatile("v_add_u32 %0, %1, %2" : "=v"(t0) : "v"(x##i), "v"(y));                   \
    asm volatile("v_add_u32 %0, %1, %2" : "=v"(t1) : "v"(x##i), "v"(z));                   \
    asm volatile("v_pk_minimum3_f16 %0, %0, %1, %2" : "+v"(x##i) : "v"(t0), "v"(t1));
#define O_ADD2_MIN3U32(i)                                                                  \
    asm volatile("v_add_u32 %0, %1, %2" : "=v"(t0) : "v"(x##i), "v"(y));                   \
    asm volatile("v_add_u32 %0, %1, %2" : "=v"(t1) : "v"(x##i), "v"(z));                   \
    asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(x##i) : "v"(t0), "v"(t1));
#define O_ADD_PKMINU16(i)                                                                  \
    asm volatile("v_add_u32 %0, %1, %2" : "=v"(t0) : "v"(x##i), "v"(y));                   \
    asm volatile("v_pk_min_u16 %0, %0, %1" : "+v"(x##i) : "v"(t0));
#define O_PKADDF2_PKMIN3F(i)                                                               \
    asm volatile("v_pk_add_f16 %0, %1, %2" : "=v"(t0) : "v"(x##i), "v"(y));                \
    asm volatile("v_pk_add_f16 %0, %1, %2" : "=v"(t1) : "v"(x##i), "v"(z));                \
    asm volatile("v_pk_minimum3_f16 %0, %0, %1, %2" : "+v"(x##i) : "v"(t0), "v"(t1));

KERNEL1(k_pkmin3f, O_PKMIN3F)
KERNEL1(k_pkaddf, O_PKADDF)
KERNEL1(k_pkminf, O_PKMINF)
KERNEL1(k_min3u32, O_MIN3U32)
KERNEL1(k_min3u16, O_MIN3U16)
KERNEL1(k_pkminu16, O_PKMINU16)
KERNEL1(k_add, O_ADD)
KERNEL1(k_add2_pkmin3f, O_ADD2_PKMIN3F)
KERNEL1(k_add2_min3u32, O_ADD2_MIN3U32)
KERNEL1(k_add_pkminu16, O_ADD_PKMINU16)
KERNEL1(k_pkaddf2_pkmin3f, O_PKADDF2_PKMIN3F)

/* exactness of pk_minimum3_f16 as an unsigned u16 min over [0, 0x7BFF] (bit patterns) */
__global__ void check_min3(const unsigned* a, const unsigned* b, const unsigned* c, int n,
                           unsigned* bad) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    unsigned r;
    asm volatile("v_pk_minimum3_f16 %0, %1, %2, %3" : "=v"(r) : "v"(a[i]), "v"(b[i]), "v"(c[i]));
    unsigned lo = min(min(a[i] & 0xFFFF, b[i] & 0xFFFF), c[i] & 0xFFFF);
    unsigned hi = min(min(a[i] >> 16, b[i] >> 16), c[i] >> 16);
    if (r != (lo | (hi << 16))) atomicAdd(bad, 1u);
}

typedef void (*kfn)(unsigned*, unsigned long long*, unsigned);
static void run(const char* name, kfn f, int waves_per_simd, int instr_per_chain_iter,
                int relax_per_chain_iter, unsigned* out, unsigned long long* clk) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    int grid = 256 * waves_per_simd;
    f<<<grid, 256>>>(out, clk, 3);
    hipEventRecord(a);
    for (int r = 0; r < 5; r++) f<<<grid, 256>>>(out, clk, 3 + r);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    unsigned long long c[2];
    hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    double ghz = (double)c[0] / (double)c[1] * 0.1;
    double chains = 5.0 * waves_per_simd * (double)ITERS * 16;
    double cyc_instr = ms * 1e-3 * ghz * 1e9 / (chains * instr_per_chain_iter);
    double cyc_relax = relax_per_chain_iter ? ms * 1e-3 * ghz * 1e9 / (chains * relax_per_chain_iter) : 0;
    printf("%-22s waves/SIMD %d: %.3f ms, clock %.2f GHz, %.2f cycles/instr", name, waves_per_simd,
           ms / 5, ghz, cyc_instr);
    if (relax_per_chain_iter) printf(", %.2f cycles/relax", cyc_relax);
    printf("\n");
}

int main() {
    unsigned* out;
    unsigned long long* clk;
    hipMalloc(&out, 4096);
    hipMalloc(&clk, 16);
    for (int w : {8, 4}) {
        run("v_pk_minimum3_f16", k_pkmin3f, w, 1, 0, out, clk);
        run("v_pk_add_f16", k_pkaddf, w, 1, 0, out, clk);
        run("v_pk_min_f16", k_pkminf, w, 1, 0, out, clk);
        run("v_min3_u32", k_min3u32, w, 1, 0, out, clk);
        run("v_min3_u16", k_min3u16, w, 1, 0, out, clk);
        run("v_pk_min_u16", k_pkminu16, w, 1, 0, out, clk);
        run("v_add_u32", k_add, w, 1, 0, out, clk);
        run("add,add,pk_minimum3", k_add2_pkmin3f, w, 3, 4, out, clk);
        run("add,add,min3_u32", k_add2_min3u32, w, 3, 2, out, clk);
        run("add,pk_min_u16", k_add_pkminu16, w, 2, 2, out, clk);
        run("pkaddf,pkaddf,pkmin3", k_pkaddf2_pkmin3f, w, 3, 4, out, clk);
    }
    /* exactness: random triples + every small value against a few others */
    const int n = 1 << 22;
    unsigned *ha = (unsigned*)malloc(n * 4), *hb = (unsigned*)malloc(n * 4), *hc = (unsigned*)malloc(n * 4);
    srand(7);
    for (int i = 0; i < n; i++) {
        unsigned r = (unsigned)rand() ^ ((unsigned)rand() << 15);
        unsigned lo = i < 65536 ? (unsigned)(i % 0x7C00) : (r % 0x7C00);
        unsigned hi = (unsigned)(rand() % 0x7C00);
        ha[i] = lo | (hi << 16);
        hb[i] = ((unsigned)(rand() % 0x7C00)) | ((unsigned)(i < 4096 ? i : rand() % 0x7C00) << 16);
        hc[i] = ((unsigned)(rand() % 64)) | ((unsigned)(rand() % 0x7C00) << 16);
    }
    unsigned *da, *db, *dc, *dbad, bad = 0;
    hipMalloc(&da, n * 4);
    hipMalloc(&db, n * 4);
    hipMalloc(&dc, n * 4);
    hipMalloc(&dbad, 4);
    hipMemcpy(da, ha, n * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, hb, n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dc, hc, n * 4, hipMemcpyHostToDevice);
    hipMemset(dbad, 0, 4);
    check_min3<<<n / 256, 256>>>(da, db, dc, n, dbad);
    hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
    printf("pk_minimum3_f16 as u16 min over [0,0x7BFF]: %u mismatches of %d\n", bad, n);
    return 0;
}
