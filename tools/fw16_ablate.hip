// Ablation microbenchmark of the packed-u16 FW update tile (one process, interleaved rounds).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ishadow_amd/csrc tools/fw16_ablate.hip
#define SRT_FW16_DEVICE_ONLY
#include "../shadow_amd/csrc/fw16.hip"
#include "fwh_legacy.h"
#include <cstdio>
#include <vector>
#include <algorithm>

template <bool FM, bool IO, bool STAGE, bool COMPUTE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void abl_kernel(u16* __restrict__ D, int ld, const u16* __restrict__ P,
                                                  int k0, int ncol_tiles, unsigned* sink) {
    __shared__ __attribute__((aligned(16))) uint32_t sA[128 * (UKC + 4)];
    __shared__ __attribute__((aligned(16))) u16 sB[UKC * (128 + 8)];
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int nb = gridDim.x, per = nb >> 3;
    const int bid = (nb & 7) == 0 ? (blockIdx.x & 7) * per + (blockIdx.x >> 3) : blockIdx.x;
    const int I = bid / ncol_tiles, J = bid % ncol_tiles;
    u16* C = D + (size_t)I * 128 * ld + J * 128;
    u16x2 old[8][4];
    if (IO) load_acc16<8, 8>(old, C, ld, tx, ty);
    else for (int r = 0; r < 8; ++r) for (int c = 0; c < 4; ++c) old[r][c] = as2(0x10001000u + r + c + tid);
    u16x2 acc[8][4];
    for (int r = 0; r < 8; ++r) for (int c = 0; c < 4; ++c) acc[r][c] = old[r][c];
    for (int h = 0; h < KB; h += UKC) {
        if (STAGE) {
            if (h) __syncthreads();
            stage_A<128, UKC>(sA, D + (size_t)I * 128 * ld + k0 + h, ld, tid);
            stage_B<128, UKC>(sB, P + (size_t)h * ld + J * 128, ld, tid);
            __syncthreads();
        }
        if (COMPUTE) mp16<FM, 128, 8, 8, UKC>(acc, sA, sB, tx, ty);
    }
    if (IO) store_acc16<8, 8>(acc, old, C, ld, tx, ty);
    else {
        unsigned x = 0;
        for (int r = 0; r < 8; ++r) for (int c = 0; c < 4; ++c) x ^= as32(acc[r][c]);
        if (x == 0x12345678u) sink[tid] = x;
    }
}

template <bool FM, bool IO, bool ST, bool CO>
float run(u16* D, int ld, unsigned* sink, int rounds) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int nct = ld / 128, grid = nct * nct;
    hipEventRecord(a);
    for (int k = 0; k < rounds; ++k) {
        const int k0 = (k * 64) % ld;
        abl_kernel<FM, IO, ST, CO><<<grid, 256>>>(D, ld, D + (size_t)k0 * ld, k0, nct, sink);
    }
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms / rounds;
}

float run_fwh(u16* D, int ld, int rounds) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int nct = ld / 128, grid = nct * nct;
    hipEventRecord(a);
    for (int k = 0; k < rounds; ++k) {
        const int k0 = (k * 64) % ld;
        fwh_update_kernel<false><<<grid, 256>>>(D, ld, D + (size_t)k0 * ld, k0, nct, 0, -1, nullptr, 0);
    }
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms / rounds;
}

int main(int argc, char** argv) {
    const int ld = argc > 1 ? atoi(argv[1]) : 32768;
    const int rounds = 20;
    u16* D; unsigned* sink;
    hipMalloc(&D, (size_t)ld * ld * 2); hipMalloc(&sink, 4096);
    hipMemset(D, 0x11, (size_t)ld * ld * 2);
    {
        std::vector<float> t;
        for (int it = 0; it < 5; ++it) t.push_back(run_fwh(D, ld, rounds));
        std::sort(t.begin(), t.end());
        printf("FWH pipelined full median %.4f ms  min %.4f ms\n", t[2], t[0]);
    }
    if (argc > 2 && argv[2][0] == 'f') return 0; /* profiling runs: the pipelined kernel only */
    const char* names[] = {"full", "no-io", "no-stage", "compute-only", "io-only", "io+stage", "stage-only"};
    for (int fm = 1; fm >= 0; --fm) {
        std::vector<std::vector<float>> t(7);
        for (int it = 0; it < 5; ++it) {
            if (fm) {
                t[0].push_back(run<true, true, true, true>(D, ld, sink, rounds));
                t[1].push_back(run<true, false, true, true>(D, ld, sink, rounds));
                t[2].push_back(run<true, true, false, true>(D, ld, sink, rounds));
                t[3].push_back(run<true, false, false, true>(D, ld, sink, rounds));
            } else {
                t[0].push_back(run<false, true, true, true>(D, ld, sink, rounds));
                t[1].push_back(run<false, false, true, true>(D, ld, sink, rounds));
                t[2].push_back(run<false, true, false, true>(D, ld, sink, rounds));
                t[3].push_back(run<false, false, false, true>(D, ld, sink, rounds));
            }
            t[4].push_back(run<false, true, false, false>(D, ld, sink, rounds));
            t[5].push_back(run<false, true, true, false>(D, ld, sink, rounds));
            t[6].push_back(run<false, false, true, false>(D, ld, sink, rounds));
        }
        for (int v = 0; v < 7; ++v) {
            std::sort(t[v].begin(), t[v].end());
            printf("%s %-14s median %.4f ms  min %.4f ms\n", fm ? "FM" : "U ", names[v], t[v][2], t[v][0]);
        }
    }
    return 0;
}
