// comb_sim.cpp — CPU experiment for the shuffle engine's speculation: how fast
// does the true Fisher-Yates draw chain (rand 0.8.5 shuffle on ChaCha12 words)
// meet one of M speculative walks started at guesses around an uncertain epoch
// boundary, and how many words do those walks cost when neighbours that reach
// the same (position, range) are merged?  Uses the engine's own walker and
// ChaCha code (shuffle_host.cpp).
//   g++ -O3 -march=native -std=c++17 -I../../burn-ppo_amd/csrc comb_sim.cpp \
//       ../../burn-ppo_amd/csrc/shuffle_host.cpp -o comb_sim
//   ./comb_sim M spread_sigmas e_sigma trials
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#include "shuffle_host.h"

static const uint32_t N = 8388608;
static const uint64_t CK = 1024;

int main(int argc, char **argv) {
    const int M = argc > 1 ? atoi(argv[1]) : 6;
    const double spread = argc > 2 ? atof(argv[2]) : 2.0;
    const double esig = argc > 3 ? atof(argv[3]) : 1.0;    // boundary sd in units of one epoch's sd
    const int trials = argc > 4 ? atoi(argv[4]) : 8;
    double Ew = 0, var = 0;
    for (uint32_t R = N; R >= 2; R--) {
        const double a = (double)(R << __builtin_clz(R)) / 4294967296.0;
        Ew += 1.0 / a;
        var += (1.0 - a) / (a * a);
    }
    const double sig = std::sqrt(var) * esig;
    const uint64_t span = (uint64_t)(2 * spread * sig) + 4 * CK;
    const uint64_t P = span + (uint64_t)(Ew + 8 * sig) + 8 * CK;
    printf("N=%u Ew=%.0f sd=%.0f boundary sd=%.0f M=%d spread=+-%.1f sd words=%llu\n", N, Ew, std::sqrt(var), sig, M,
           spread, (unsigned long long)P);
    std::vector<uint32_t> w(P);
    uint32_t key[8] = {1, 2, 3, 4, 5, 6, 7, 8};
    std::mt19937_64 rng(12345);
    std::normal_distribution<double> nd(0.0, sig);
    double tot_words = 0, tot_meet = 0;
    int misses = 0;
    std::vector<double> meets;
    for (int t = 0; t < trials; t++) {
        key[0] = 100 + t;
        bppo_host::chacha12_words(key, 7, 0, w.data(), P);
        const double centre = (double)span / 2;
        double xt = centre + nd(rng);
        xt = std::min(std::max(xt, 1.0), (double)span - 1);
        const uint64_t x0 = (uint64_t)xt;
        // comb walks
        struct Wk { uint64_t pos; uint32_t r; bool live; };
        std::vector<Wk> ws(M);
        for (int k = 0; k < M; k++) {
            const double g = centre + ((k + 0.5) / M - 0.5) * 2.0 * spread * sig;
            ws[k] = {(uint64_t)std::max(0.0, std::floor(g)), N, true};
        }
        uint64_t tp = x0;
        uint32_t tr = N;
        int64_t meet_at = -1;
        double words = 0;
        // lockstep by checkpoint index
        for (uint64_t q = (std::min(ws[0].pos, x0) / CK + 1) * CK; q < P; q += CK) {
            bool any = false;
            for (int k = 0; k < M; k++) {
                Wk &a = ws[k];
                if (!a.live || a.r < 2 || a.pos >= q) { any |= a.live && a.r >= 2; continue; }
                const uint64_t before = a.pos;
                a.pos += bppo_host::chain_walk_nj(w.data() + a.pos, q - a.pos, &a.r);
                words += (double)(a.pos - before);
                any = true;
            }
            // merge neighbours at q (walks never cross: compare consecutive live ones)
            int prev = -1;
            for (int k = 0; k < M; k++) {
                if (!ws[k].live || ws[k].pos != q) continue;
                if (prev >= 0 && ws[prev].pos == q && ws[prev].r == ws[k].r) ws[k].live = false;
                else prev = k;
            }
            if (meet_at < 0 && tr >= 2 && tp < q) {
                tp += bppo_host::chain_walk_nj(w.data() + tp, q - tp, &tr);
                if (tp == q)
                    for (int k = 0; k < M; k++)
                        if (ws[k].live && ws[k].pos == q && ws[k].r == tr) { meet_at = (int64_t)(q - x0); break; }
            }
            if (!any && (meet_at >= 0 || tr < 2)) break;
        }
        int surv = 0;
        for (auto &a : ws) surv += a.live;
        if (meet_at < 0) misses++; else { tot_meet += meet_at; meets.push_back((double)meet_at); }
        tot_words += words;
        printf("  trial %d: truth %+.2f sd, meet %lld words, comb words %.1fM (%.1f epochs), survivors %d\n", t,
               (xt - centre) / sig, (long long)meet_at, words / 1e6, words / Ew, surv);
    }
    std::sort(meets.begin(), meets.end());
    printf("SUMMARY M=%d spread=%.1f esig=%.2f: miss %d/%d, median meet %.0f words, mean comb cost %.2f epochs\n", M,
           spread, esig, misses, trials, meets.empty() ? -1.0 : meets[meets.size() / 2], tot_words / trials / Ew);
    return 0;
}
