/*
 * shadow_compat.c -- weak fallbacks for the Shadow symbols the drop-in layer calls.
 *
 * Inside Shadow these are Shadow's own strong definitions (address.c, random.c:39-43,
 * worker.c:627-629) and the linker picks those. Standalone (tests, bench) the layouts below are
 * the reference's: struct _Address starts with the network-order IP (address.c:23-25), struct
 * _Random is {seedState, initialSeed} driven by glibc rand_r (random.c:15-43).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>

struct _Address;
struct _Random;

__attribute__((weak)) uint32_t address_toNetworkIP(struct _Address* address) {
    return address ? *(const uint32_t*)address : 0;
}

__attribute__((weak)) double random_nextDouble(struct _Random* random) {
    unsigned int* seedState = (unsigned int*)random;
    int v = rand_r(seedState);
    return (double)v / (double)RAND_MAX;
}

__attribute__((weak)) void worker_updateMinTimeJump(double minPathLatency) { (void)minPathLatency; }
