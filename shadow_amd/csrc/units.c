/*
 * units.c -- latency / bandwidth grammar of Shadow's graph attributes, restated in C.
 *
 * Reference: /root/reference/src/main/core/support/units.rs
 *   FromStr regex ^([+-]?[0-9\.]*)\s*(.*)$, value/unit trimmed          :404-437
 *   value parsed as u64 (optional '+', digits only: "10.5", "-10" fail) :434
 *   time units (ns|us|μs|ms|s|sec|...|min|h|...), no unit = seconds     :232-251, :226-230
 *   SI-upper prefixes for bits (K|Ki|M|Mi|G|Gi|T|Ti + long forms)       :150-170
 *   Time suffixes [""], BitsPerSec suffixes ["bit","bits"]               :547, :577
 *   parse_time_nanosec / parse_bandwidth: convert().unwrap(), i64 check  :776-837
 * The reference panics where `convert()` overflows u64 (the unwrap); this port returns -2 so the
 * caller can fail validation loudly instead of aborting the process.
 */
#include <stdint.h>
#include <string.h>

#include "shadow_routing.h"

/* Unicode White_Space (Rust char::is_whitespace / regex \s) for one UTF-8 sequence at p.
 * Returns the byte length of the whitespace character, 0 if none. */
static size_t utf8_space(const unsigned char* p, const unsigned char* end) {
    if (p >= end) return 0;
    unsigned char c = p[0];
    if (c == ' ' || (c >= 0x09 && c <= 0x0d)) return 1;
    if (c == 0xC2 && p + 1 < end && (p[1] == 0x85 || p[1] == 0xA0)) return 2;
    if (c == 0xE1 && p + 2 < end && p[1] == 0x9A && p[2] == 0x80) return 3; /* U+1680 */
    if (c == 0xE2 && p + 2 < end) {
        if (p[1] == 0x80 && ((p[2] >= 0x80 && p[2] <= 0x8A) || p[2] == 0xA8 || p[2] == 0xA9 ||
                             p[2] == 0xAF))
            return 3; /* U+2000..200A, 2028, 2029, 202F */
        if (p[1] == 0x81 && p[2] == 0x9F) return 3; /* U+205F */
    }
    if (c == 0xE3 && p + 2 < end && p[1] == 0x80 && p[2] == 0x80) return 3; /* U+3000 */
    return 0;
}

/* Length in bytes of a trailing Unicode whitespace character ending at end (0 if none). */
static size_t utf8_space_back(const unsigned char* begin, const unsigned char* end) {
    for (size_t k = 1; k <= 3 && end - k >= begin; k++)
        if (utf8_space(end - k, end) == k) return k;
    return 0;
}

typedef struct {
    const char* v;
    size_t vl;
    const char* u;
    size_t ul;
} vu_t;

/* Applies ^([+-]?[0-9\.]*)\s*(.*)$ and trims both groups. Returns 0 on a match. */
static int split_value_unit(const char* s, vu_t* out) {
    const unsigned char* p = (const unsigned char*)s;
    const unsigned char* end = p + strlen(s);
    const unsigned char* vb = p;
    if (p < end && (*p == '+' || *p == '-')) p++;
    while (p < end && ((*p >= '0' && *p <= '9') || *p == '.')) p++;
    const unsigned char* ve = p;
    size_t k;
    while ((k = utf8_space(p, end)) > 0) p += k;
    /* (.*)$ : '.' matches anything but '\n' */
    for (const unsigned char* q = p; q < end; q++)
        if (*q == '\n') return -1;
    const unsigned char* ub = p;
    const unsigned char* ue = end;
    while ((k = utf8_space(ub, ue)) > 0) ub += k;
    while (ue > ub && (k = utf8_space_back(ub, ue)) > 0) ue -= k;
    out->v = (const char*)vb;
    out->vl = (size_t)(ve - vb);
    out->u = (const char*)ub;
    out->ul = (size_t)(ue - ub);
    return 0;
}

/* Rust u64::from_str: optional '+', then at least one ASCII digit, no overflow. */
static int parse_u64(const char* s, size_t len, uint64_t* out) {
    size_t i = 0;
    if (len > 0 && s[0] == '+') i = 1;
    if (i == len) return -1;
    uint64_t v = 0;
    for (; i < len; i++) {
        if (s[i] < '0' || s[i] > '9') return -1;
        uint64_t d = (uint64_t)(s[i] - '0');
        if (v > (UINT64_MAX - d) / 10) return -1;
        v = v * 10 + d;
    }
    *out = v;
    return 0;
}

static int eq(const char* a, size_t al, const char* lit) {
    return al == strlen(lit) && memcmp(a, lit, al) == 0;
}

/* TimePrefix::from_str (units.rs:232-251) -> nanoseconds per unit; 0 = unknown unit. */
static uint64_t time_factor_ns(const char* u, size_t ul) {
    if (ul == 0) return 1000000000ull; /* default prefix: Sec */
    if (eq(u, ul, "ns") || eq(u, ul, "nanosecond") || eq(u, ul, "nanoseconds")) return 1ull;
    if (eq(u, ul, "us") || eq(u, ul, "\xce\xbcs") || eq(u, ul, "microsecond") ||
        eq(u, ul, "microseconds"))
        return 1000ull;
    if (eq(u, ul, "ms") || eq(u, ul, "millisecond") || eq(u, ul, "milliseconds"))
        return 1000000ull;
    if (eq(u, ul, "s") || eq(u, ul, "sec") || eq(u, ul, "secs") || eq(u, ul, "second") ||
        eq(u, ul, "seconds"))
        return 1000000000ull;
    if (eq(u, ul, "m") || eq(u, ul, "min") || eq(u, ul, "mins") || eq(u, ul, "minute") ||
        eq(u, ul, "minutes"))
        return 60000000000ull;
    if (eq(u, ul, "h") || eq(u, ul, "hr") || eq(u, ul, "hrs") || eq(u, ul, "hour") ||
        eq(u, ul, "hours"))
        return 3600000000000ull;
    return 0;
}

/* SiPrefixUpper::from_str (units.rs:150-170) -> multiplier; 0 = unknown prefix. */
static uint64_t si_upper_factor(const char* u, size_t ul) {
    if (ul == 0) return 1ull;
    if (eq(u, ul, "K") || eq(u, ul, "kilo")) return 1000ull;
    if (eq(u, ul, "Ki") || eq(u, ul, "kibi")) return 1024ull;
    if (eq(u, ul, "M") || eq(u, ul, "mega")) return 1000000ull;
    if (eq(u, ul, "Mi") || eq(u, ul, "mebi")) return 1048576ull;
    if (eq(u, ul, "G") || eq(u, ul, "giga")) return 1000000000ull;
    if (eq(u, ul, "Gi") || eq(u, ul, "gibi")) return 1073741824ull;
    if (eq(u, ul, "T") || eq(u, ul, "tera")) return 1000000000000ull;
    if (eq(u, ul, "Ti") || eq(u, ul, "tebi")) return 1099511627776ull;
    return 0;
}

static int64_t finish(uint64_t value, uint64_t factor) {
    if (factor != 0 && value > UINT64_MAX / factor) return -2; /* reference: unwrap() panics */
    uint64_t x = value * factor;
    if (x > (uint64_t)INT64_MAX) return -1; /* try_into::<i64>() fails -> -1 */
    return (int64_t)x;
}

int64_t srt_parse_time_nanosec(const char* s) {
    if (!s) return -1;
    vu_t vu;
    if (split_value_unit(s, &vu)) return -1;
    /* Time suffixes are [""]: strip_suffix("") always succeeds, the prefix is the whole unit.
     * The unit is resolved before the value is parsed (units.rs:421-434). */
    uint64_t f = time_factor_ns(vu.u, vu.ul);
    if (f == 0) return -1;
    uint64_t v;
    if (parse_u64(vu.v, vu.vl, &v)) return -1;
    return finish(v, f);
}

int64_t srt_parse_bandwidth(const char* s) {
    if (!s) return -1;
    vu_t vu;
    if (split_value_unit(s, &vu)) return -1;
    const char* p = vu.u;
    size_t pl = vu.ul;
    /* suffixes ["bit", "bits"]: the first one that strips wins, else the whole unit */
    if (pl >= 3 && memcmp(p + pl - 3, "bit", 3) == 0)
        pl -= 3;
    else if (pl >= 4 && memcmp(p + pl - 4, "bits", 4) == 0)
        pl -= 4;
    uint64_t f = si_upper_factor(p, pl);
    if (f == 0) return -1;
    uint64_t v;
    if (parse_u64(vu.v, vu.vl, &v)) return -1;
    return finish(v, f);
}
