// Host cost of the level build's reliability-table union (levels.hip): the concatenation of R
// blocks of ~500 values (C4 at N = 8: every rank holds the same ~500 loss values) sorted and
// deduplicated, against an open-addressing set then a sort of the distinct values.
// g++ -O2 tools/union_bench.cpp -o /tmp/union_bench && /tmp/union_bench
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
int main() {
    std::mt19937_64 g(1);
    for (int R : {2, 4, 8}) {
        std::vector<unsigned long long> base(501);
        for (auto& x : base) x = 0x3FE0000000000000ull | (g() & 0xFFFFFFFFFFFFull);
        double t_sort = 1e9, t_set = 1e9;
        for (int rep = 0; rep < 50; rep++) {
            std::vector<std::vector<unsigned long long>> blocks(R, base);
            for (auto& b : blocks) std::shuffle(b.begin(), b.end(), g);
            auto t0 = std::chrono::steady_clock::now();
            std::vector<unsigned long long> u;
            for (auto& b : blocks) u.insert(u.end(), b.begin(), b.end());
            std::sort(u.begin(), u.end());
            u.erase(std::unique(u.begin(), u.end()), u.end());
            auto t1 = std::chrono::steady_clock::now();
            size_t all = 0;
            for (auto& b : blocks) all += b.size();
            size_t cap = 64;
            while (cap < 2 * all) cap <<= 1;
            int shift = 64;
            for (size_t c = cap; c > 1; c >>= 1) --shift;
            std::vector<unsigned long long> set(cap, ~0ull), v;
            for (auto& b : blocks)
                for (unsigned long long x : b) {
                    size_t h = (size_t)((x * 0x9E3779B97F4A7C15ull) >> shift);
                    while (set[h] != ~0ull && set[h] != x) h = (h + 1) & (cap - 1);
                    if (set[h] == ~0ull) {
                        set[h] = x;
                        v.push_back(x);
                    }
                }
            std::sort(v.begin(), v.end());
            auto t2 = std::chrono::steady_clock::now();
            if (v != u) { printf("mismatch\n"); return 1; }
            t_sort = std::min(t_sort, std::chrono::duration<double, std::micro>(t1 - t0).count());
            t_set = std::min(t_set, std::chrono::duration<double, std::micro>(t2 - t1).count());
        }
        printf("{\"ranks\": %d, \"values_per_rank\": 501, \"us_sort_all\": %.1f, \"us_set_then_sort\": %.1f}\n", R, t_sort, t_set);
    }
    return 0;
}
