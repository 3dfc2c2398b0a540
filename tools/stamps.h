// Host side of the development phase stamps (kernels_common.h STAMP):
// per-phase median cycle counts over workgroups and tile iterations.
#pragma once
#include <algorithm>
#include <cstdio>
#include <vector>

// stamps[((wg * STAMP_TILES + it) * 2 + w) * 16 + slot]; slot k..k+1 gaps for
// k < nslots - 1, the last gap runs to slot 0 of the next iteration
inline void stamp_report(const std::vector<unsigned long long> &h, int nwg, int tiles, int nslots, const char **names,
                         double kernel_us) {
    for (int w = 0; w < 2; w++) {
        printf("  wave %s:", w ? "last" : "0   ");
        double tot = 0;
        for (int k = 1; k <= nslots; k++) {
            std::vector<double> g;
            for (int wg = 0; wg < nwg; wg++)
                for (int it = 0; it < tiles; it++) {
                    const unsigned long long *s = &h[((size_t)(wg * tiles + it) * 2 + w) * 16];
                    const unsigned long long *sn = &h[((size_t)(wg * tiles + it + 1) * 2 + w) * 16];
                    const unsigned long long a = s[k - 1];
                    const unsigned long long b = k < nslots ? s[k] : (it + 1 < tiles ? sn[0] : 0);
                    if (a && b && b > a) g.push_back((double)(b - a));
                }
            std::sort(g.begin(), g.end());
            const double md = g.empty() ? 0 : g[g.size() / 2];
            tot += md;
            printf("  %s %.0f", names[k - 1], md);
        }
        printf("  | iteration %.0f cyc\n", tot);
    }
    printf("  (kernel %.1f us)\n", kernel_us);
}
