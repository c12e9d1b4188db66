/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Plain-DP restatement of the primer-hit search of the
 * pychopper-style read reorientation (scripts/01_pychopper.sh:45-57: `pychopper -m edlib -b
 * M13_seqs_for_pychopper.fa -c M13_config_for_pychopper.txt -p ...`).  pychopper v2.7.0 and
 * edlib are not vendored in /root/reference and not installed here: PARITY UNPINNED.  The
 * semantics below are the build's definition, restated from edlib's documented
 * HW ("infix") mode; oracle/chopper.py carries the segmentation / classification half.
 *
 * For one label (a primer, or its reverse complement) P of length m and one read R of length n,
 * one edlib call `edlibAlign(P, R, HW, TASK_LOC, k)` (edlib 1.3.x, edlib.cpp edlibAlign: the HW
 * end locations, then one reverse SHW alignment per end location for its start):
 *   match(P[i], R[j])  = R[j] not in ACGT (N matches anything, edlib additionalEqualities
 *                        style), or R[j] in IUPAC(P[i])                (reads upper-cased)
 *   D(j), 1 <= j <= n  = min over s <= j of unit-cost editdist(P, R[s:j))   (HW / infix)
 *   k                  = (int)(cutoff * m)
 *   best               = min over j of D(j) (edlib's editDistance); no hits when best > k
 *   hits               = every stop j with D(j) == best (edlib's endLocations, ascending), each
 *                        with dist = best and start = the SMALLEST s with
 *                        editdist(P, R[s:stop)) == best: edlib takes the last position of the
 *                        reverse SHW alignment ("taking last location as start ensures that
 *                        alignment will not start with insertions if it can start with
 *                        mismatches instead"), i.e. the longest optimal alignment ending there
 * Computed with the textbook O(m n) column DP (no bit vectors), independently of the HIP
 * kernel's Myers scan and warm-up segmentation.  orc_chop_batch runs it over a batch on
 * pthreads (the bench's CPU baseline).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int iupac4(char c) {
    switch (c) {
        case 'A': return 1; case 'C': return 2; case 'G': return 4; case 'T': case 'U': return 8;
        case 'R': return 5; case 'Y': return 10; case 'S': return 6; case 'W': return 9;
        case 'K': return 12; case 'M': return 3; case 'B': return 14; case 'D': return 13;
        case 'H': return 11; case 'V': return 7; case 'N': return 15;
        default: return 0;
    }
}

static int base_bit(uint8_t c) {   /* read byte -> 1/2/4/8, 0 = not ACGT (matches anything) */
    switch (c) {
        case 'A': case 'a': return 1;
        case 'C': case 'c': return 2;
        case 'G': case 'g': return 4;
        case 'T': case 't': return 8;
        default: return 0;
    }
}

static inline int eqc(int pm, int rb) { return rb == 0 || (pm & rb) != 0; }

/* hits: up to cap records of {stop, start, dist}; returns the total number found (may exceed
 * cap), or -1 on a bad pattern. */
int orc_chop_hits(const char* pat, int m, double cutoff, const uint8_t* read, int n,
                  int32_t* out, int cap) {
    if (m < 1 || m > 4096) return -1;
    int* pm = malloc(sizeof(int) * m);
    int* col = malloc(sizeof(int) * (m + 1));
    int* g = malloc(sizeof(int) * (m + 1));
    for (int i = 0; i < m; ++i) {
        pm[i] = iupac4(pat[i]);
        if (!pm[i]) {
            free(pm); free(col); free(g);
            return -1;
        }
    }
    const int k = (int)(cutoff * m);
    int* D = malloc(sizeof(int) * ((size_t)n + 1));
    for (int i = 0; i <= m; ++i) col[i] = i;
    int best = m + 1;
    D[0] = m;
    for (int j = 1; j <= n; ++j) {
        const int rb = base_bit(read[j - 1]);
        int diag = col[0];   /* D(0, j-1) = 0: free start */
        col[0] = 0;
        for (int i = 1; i <= m; ++i) {
            const int up = col[i - 1] + 1, left = col[i] + 1;
            const int dg = diag + (eqc(pm[i - 1], rb) ? 0 : 1);
            diag = col[i];
            int v = dg < up ? dg : up;
            col[i] = v < left ? v : left;
        }
        D[j] = col[m];
        if (D[j] < best) best = D[j];
    }
    int nh = 0;
    for (int j = 1; j <= n && best <= k; ++j) {
        if (D[j] != best) continue;
        /* start: G(i, t) = editdist(P[m-i:], R[stop-t:stop)); last t <= m + best with
         * G(m, t) == best (an alignment of cost best spans at most m + best columns) */
        int start = -1;
        for (int i = 0; i <= m; ++i) g[i] = i;
        const int tmax = j < m + best ? j : m + best;
        for (int t = 1; t <= tmax; ++t) {
            const int rb = base_bit(read[j - t]);
            int diag = g[0];
            g[0] = t;
            for (int i = 1; i <= m; ++i) {
                const int up = g[i - 1] + 1, left = g[i] + 1;
                const int dg = diag + (eqc(pm[m - i], rb) ? 0 : 1);
                diag = g[i];
                int v = dg < up ? dg : up;
                g[i] = v < left ? v : left;
            }
            if (g[m] == best) start = j - t;
        }
        if (nh < cap) {
            out[3 * nh] = j;
            out[3 * nh + 1] = start;
            out[3 * nh + 2] = best;
        }
        ++nh;
    }
    free(D);
    free(pm); free(col); free(g);
    return nh;
}

typedef struct {
    const char* const* pats;
    const int* plens;
    int npat;
    double cutoff;
    const uint8_t* blob;
    const uint64_t* offs;
    const uint32_t* lens;
    size_t lo, hi;
    int32_t* nhits;
} ChopJob;

static void* chop_worker(void* arg) {
    ChopJob* J = (ChopJob*)arg;
    int32_t scratch[3 * 64];
    for (size_t r = J->lo; r < J->hi; ++r) {
        int32_t tot = 0;
        for (int p = 0; p < J->npat; ++p)
            tot += orc_chop_hits(J->pats[p], J->plens[p], J->cutoff, J->blob + J->offs[r],
                                 (int)J->lens[r], scratch, 64);
        J->nhits[r] = tot;
    }
    return NULL;
}

/* Hit counts of every read over every label (the labels given as patterns), on `threads`
 * pthreads. */
int orc_chop_batch(const char* const* pats, const int* plens, int npat, double cutoff,
                   const uint8_t* blob, const uint64_t* offs, const uint32_t* lens, size_t n,
                   int threads, int32_t* nhits) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    ChopJob jobs[256];
    for (int t = 0; t < threads; ++t) {
        ChopJob J = {pats, plens, npat, cutoff, blob, offs, lens, n * t / threads,
                     n * (t + 1) / threads, nhits};
        jobs[t] = J;
        pthread_create(&th[t], NULL, chop_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    return 0;
}
