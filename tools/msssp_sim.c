/*
 * msssp_sim.c -- CPU model of the multi-source shared-frontier SSSP (shadow_amd/csrc/msssp.hip),
 * used to size the design (pulls per vertex, passes per batch) and to check that its fixed point is
 * the canonical table (tools/msssp_sim.py compares it with oracle/ on the same graphs).
 *
 * 64 sources (lanes) share one frontier. A vertex's state is (D, R) per lane; a pull recomputes it
 * from all of its in-arcs: D = min (D[u] + w), ties by (D[u], u) (the canonical predecessor of
 * SURVEY §8a-4), R = R[pred] * r(pred, v). A changed vertex propagates (its out-neighbours become
 * candidates of the next pass) once some lane of it is below the bucket bound T; otherwise it waits
 * in the pending set until T passes it (delta-stepping over the lane minimum).
 * jacobi = 1 computes each pass from the previous pass's states (the GPU's worst case), 0 in place.
 * Built as a shared library: gcc -O2 -shared -fPIC tools/msssp_sim.c -o /tmp/libmsssp_sim.so
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define L 64
#define INF 0xFFFFFFFFu

typedef struct {
    int64_t pulls, passes, buckets, arcs, hub_arcs, hub_pulls;
} sim_counts;

int msssp_sim_batch(int n, const int32_t* irp, const int32_t* icol, const uint32_t* iw,
                    const double* ir, const int32_t* orp, const int32_t* ocol, int nl,
                    const int32_t* srcs, uint32_t delta, int jacobi, uint32_t* Dout, double* Rout,
                    sim_counts* cnt) {
    uint32_t* D = (uint32_t*)malloc((size_t)n * L * 4);
    double* R = (double*)malloc((size_t)n * L * 8);
    uint32_t* D2 = (uint32_t*)malloc((size_t)n * L * 4);
    double* R2 = (double*)malloc((size_t)n * L * 8);
    int32_t* F = (int32_t*)malloc((size_t)n * 4);
    int32_t* NF = (int32_t*)malloc((size_t)n * 4);
    int32_t* C = (int32_t*)malloc((size_t)n * 4);
    uint8_t* cand = (uint8_t*)calloc((size_t)n, 1);
    uint8_t* pend = (uint8_t*)calloc((size_t)n, 1);
    uint32_t* mind = (uint32_t*)malloc((size_t)n * 4);
    int8_t* srclane = (int8_t*)malloc((size_t)n * L);
    if (!D || !R || !D2 || !R2 || !F || !NF || !C || !cand || !pend || !mind || !srclane) return -1;
    for (size_t i = 0; i < (size_t)n * L; i++) {
        D[i] = INF;
        R[i] = 0.0;
        srclane[i] = 0;
    }
    for (int v = 0; v < n; v++) mind[v] = INF;
    int nf = 0;
    for (int l = 0; l < nl; l++) {
        D[(size_t)srcs[l] * L + l] = 0;
        R[(size_t)srcs[l] * L + l] = 1.0;
        srclane[(size_t)srcs[l] * L + l] = 1;
        if (mind[srcs[l]] == INF) F[nf++] = srcs[l];
        mind[srcs[l]] = 0;
    }
    memset(cnt, 0, sizeof(*cnt));
    uint32_t T = delta;
    for (;;) {
        while (nf > 0) {
            int nc = 0;
            for (int i = 0; i < nf; i++) {
                const int u = F[i];
                for (int k = orp[u]; k < orp[u + 1]; k++)
                    if (!cand[ocol[k]]) {
                        cand[ocol[k]] = 1;
                        C[nc++] = ocol[k];
                    }
            }
            cnt->passes++;
            cnt->pulls += nc;
            const uint32_t* Ds = D;
            const double* Rs = R;
            if (jacobi) {
                memcpy(D2, D, (size_t)n * L * 4);
                memcpy(R2, R, (size_t)n * L * 8);
                Ds = D2;
                Rs = R2;
            }
            int nn = 0;
            for (int i = 0; i < nc; i++) {
                const int v = C[i];
                cand[v] = 0;
                cnt->arcs += irp[v + 1] - irp[v];
                if (irp[v + 1] - irp[v] > 64) {
                    cnt->hub_arcs += irp[v + 1] - irp[v];
                    cnt->hub_pulls++;
                }
                int changed = 0;
                uint32_t mn = INF;
                for (int l = 0; l < L; l++) {
                    uint32_t bd = INF, bdu = INF;
                    int bk = -1;
                    for (int k = irp[v]; k < irp[v + 1]; k++) {
                        const uint32_t du = Ds[(size_t)icol[k] * L + l];
                        if (du == INF) continue;
                        const uint32_t c = du + iw[k];
                        if (c < bd || (c == bd && (du < bdu || (du == bdu && icol[k] < icol[bk])))) {
                            bd = c;
                            bdu = du;
                            bk = k;
                        }
                    }
                    uint32_t nd;
                    double nr;
                    if (srclane[(size_t)v * L + l]) {
                        nd = 0;
                        nr = 1.0;
                    } else if (bk < 0) {
                        nd = INF;
                        nr = 0.0;
                    } else {
                        nd = bd;
                        nr = Rs[(size_t)icol[bk] * L + l] * ir[bk];
                    }
                    const size_t o = (size_t)v * L + l;
                    if (nd != D[o] || memcmp(&nr, &R[o], 8)) changed = 1;
                    D[o] = nd;
                    R[o] = nr;
                    if (nd < mn) mn = nd;
                }
                mind[v] = mn;
                if (changed) {
                    if (mn < T) {
                        NF[nn++] = v;
                        pend[v] = 0;
                    } else {
                        pend[v] = 1;
                    }
                }
            }
            int32_t* t = F;
            F = NF;
            NF = t;
            nf = nn;
        }
        uint32_t pm = INF;
        for (int v = 0; v < n; v++)
            if (pend[v] && mind[v] < pm) pm = mind[v];
        if (pm == INF) break;
        T = (pm / delta + 1) * delta;
        cnt->buckets++;
        for (int v = 0; v < n; v++)
            if (pend[v] && mind[v] < T) {
                pend[v] = 0;
                F[nf++] = v;
            }
    }
    for (int l = 0; l < nl; l++)
        for (int v = 0; v < n; v++) {
            Dout[(size_t)l * n + v] = D[(size_t)v * L + l];
            Rout[(size_t)l * n + v] = R[(size_t)v * L + l];
        }
    free(D);
    free(R);
    free(D2);
    free(R2);
    free(F);
    free(NF);
    free(C);
    free(cand);
    free(pend);
    free(mind);
    free(srclane);
    return 0;
}
