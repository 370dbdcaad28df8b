/* Test driver (tests/test_gml_parallel.py): parses one GML file with gml_parse_ex on one thread
 * and in pieces on several threads (par_min = 0) and compares every output field, or the error
 * message when the parse fails. Prints "same <n> <m> <pieces-path>" or the first difference. */
#include <math.h>
#include <time.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gml.h"

static int same_attr(const gml_attr* a, const gml_attr* b, int64_t count) {
    if (strcmp(a->name, b->name) || a->is_string != b->is_string) return 0;
    for (int64_t i = 0; i < count; i++) {
        if (a->is_string) {
            if (strcmp(a->str[i], b->str[i])) return 0;
        } else {
            const double x = a->num[i], y = b->num[i];
            if (!(x == y || (isnan(x) && isnan(y)))) return 0;
        }
    }
    return 1;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    fseek(f, 0, SEEK_END);
    long len = ftell(f);
    fseek(f, 0, SEEK_SET);
    char* text = (char*)malloc((size_t)len + 1);
    if (fread(text, 1, (size_t)len, f) != (size_t)len) return 2;
    fclose(f);
    const int nt = atoi(argv[2]);
    gml_graph a, b;
    char ea[512], eb[512];
    struct timespec t0, t1, t2;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    const int ra = gml_parse_ex(text, (size_t)len, &a, ea, sizeof(ea), 1, 0);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const int rb = gml_parse_ex(text, (size_t)len, &b, eb, sizeof(eb), nt, 0);
    clock_gettime(CLOCK_MONOTONIC, &t2);
    if (argc > 3) /* timing: the one-thread and the pieces parse, ms */
        fprintf(stderr, "{\"bytes\": %ld, \"threads\": %d, \"ms_one\": %.1f, \"ms_pieces\": %.1f}\n", len, nt,
                (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) / 1e6,
                (t2.tv_sec - t1.tv_sec) * 1e3 + (t2.tv_nsec - t1.tv_nsec) / 1e6);
    if (ra || rb) {
        if (ra != rb || strcmp(ea, eb)) {
            printf("error differs: [%s] vs [%s]\n", ra ? ea : "ok", rb ? eb : "ok");
            return 1;
        }
        printf("same-error %s\n", ea);
        return 0;
    }
    if (a.n != b.n || a.m != b.m || a.directed != b.directed || a.nva != b.nva || a.nea != b.nea) {
        printf("shape differs: n %d/%d m %lld/%lld dir %d/%d nva %d/%d nea %d/%d\n", a.n, b.n,
               (long long)a.m, (long long)b.m, a.directed, b.directed, a.nva, b.nva, a.nea, b.nea);
        return 1;
    }
    for (int64_t e = 0; e < a.m; e++)
        if (a.esrc[e] != b.esrc[e] || a.edst[e] != b.edst[e]) {
            printf("edge %lld differs\n", (long long)e);
            return 1;
        }
    for (int i = 0; i < a.nva; i++)
        if (!same_attr(&a.va[i], &b.va[i], a.n)) {
            printf("vertex attribute %s differs\n", a.va[i].name);
            return 1;
        }
    for (int i = 0; i < a.nea; i++)
        if (!same_attr(&a.ea[i], &b.ea[i], a.m)) {
            printf("edge attribute %s differs\n", a.ea[i].name);
            return 1;
        }
    printf("same %d %lld %d\n", a.n, (long long)a.m, b.pieces);
    gml_free(&a);
    gml_free(&b);
    free(text);
    return 0;
}
