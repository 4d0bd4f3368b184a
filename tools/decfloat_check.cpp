// Host check of kcp_amd/csrc/decfloat.h (the decimal -> float64 path of
// kernel K0) against glibc's correctly rounded strtod, the host decoder's
// conversion (json.cpp).  Prints "<checked> <accepted> <mismatches>".
#include <locale.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>

#include "../kcp_amd/csrc/decfloat.h"

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    std::mt19937_64 rng(argc > 2 ? atol(argv[2]) : 12345);
    locale_t cloc = newlocale(LC_ALL_MASK, "C", (locale_t)0);
    long accepted = 0, bad = 0;
    char buf[64];
    for (long i = 0; i < n; i++) {
        const int nd = 1 + (int)(rng() % 19);
        uint64_t man = 0;
        for (int k = 0; k < nd; k++) man = man * 10 + (k == 0 ? 1 + rng() % 9 : rng() % 10);
        int e10;
        switch (rng() % 4) {
            case 0: e10 = (int)(rng() % 45) - 22; break;        // common magnitudes
            case 1: e10 = -nd - (int)(rng() % 4); break;         // 0.xxxx style
            case 2: e10 = (int)(rng() % 700) - 350; break;       // full range incl. sub/overflow
            default: e10 = (int)(rng() % 20) - 19; break;
        }
        const bool neg = rng() & 1;
        snprintf(buf, sizeof buf, "%s%llue%d", neg ? "-" : "", (unsigned long long)man, e10);
        uint64_t got;
        if (!gd::decimal_to_double(man, e10, neg, &got)) continue;
        accepted++;
        double want = strtod_l(buf, nullptr, cloc);
        uint64_t wb;
        memcpy(&wb, &want, 8);
        if (wb != got) {
            if (bad < 10) fprintf(stderr, "mismatch %s: got %016llx want %016llx\n", buf, (unsigned long long)got,
                                  (unsigned long long)wb);
            bad++;
        }
    }
    printf("%ld %ld %ld\n", n, accepted, bad);
    return bad ? 1 : 0;
}
