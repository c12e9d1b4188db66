/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the product
 * path (nanopore-barcoding-orc_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / the timed CPU baseline.
 *
 * CPU restatement of the adapter-matching semantics of cutadapt v4.9.0, the third-party tool that
 * the reference's hot path shells out to (reference README.md:7; call sites
 * scripts/02_cutadapt_loop.sh:64-72 (round 1, -g file:SP5 --rc) and :91-103 (round 2,
 * -a file:SP27rc --rc); scripts/04_cleaning_primers.sh:371-388 (linked -g F...R)).
 *
 * cutadapt is NOT vendored in /root/reference and is not installed here, so this
 * file restates its published algorithm (cutadapt/_align.pyx Aligner.locate, adapters.py
 * Front/Back/LinkedAdapter.match_to, modifiers.py AdapterCutter.best_match / ReverseComplementer)
 * from the specification in SURVEY.md §8a.  The reference holds no tests, golden vectors or
 * fixtures for this path, so:
 *
 *     PARITY UNPINNED — no reference-side fixture pins these semantics; tie-break rules marked
 *     [UNVERIFIED] below are the riskiest items (see DESIGN.md "Parity status").
 *
 * Deliberately literal: the DP keeps ONE column, Ukkonen's `last` cut-off and its stale cells,
 * exactly as _align.pyx does, so that the GPU path (full-column Myers + exact traceback, which
 * never keeps stale cells) is checked against an independent formulation.
 */
#include <ctype.h>
#include <limits.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* EndSkip flags, cutadapt/_align.pyx (REFERENCE_START=1, QUERY_START=2, REFERENCE_END=4,
 * QUERY_STOP=8); adapters.py Where.FRONT / Where.BACK. */
enum { ORC_REF_START = 1, ORC_QUERY_START = 2, ORC_REF_END = 4, ORC_QUERY_STOP = 8 };
enum { ORC_FRONT = ORC_QUERY_START | ORC_QUERY_STOP | ORC_REF_START,
       ORC_BACK = ORC_QUERY_START | ORC_QUERY_STOP | ORC_REF_END };

static uint8_t IUPAC_TABLE[256], ACGT_TABLE[256], COMPLEMENT[256];
static pthread_once_t tables_once = PTHREAD_ONCE_INIT;

static void init_tables(void) {
    /* _align.pyx IUPAC_TABLE / ACGT_TABLE: A=1 C=2 G=4 T=U=8, IUPAC codes are unions,
     * everything else 0 (never matches).  Both cases. */
    static const char* codes[] = {"A1", "C2", "G4", "T8", "U8", "R5", "Y10", "S6", "W9", "K12",
                                  "M3", "B14", "D13", "H11", "V7", "N15"};
    memset(IUPAC_TABLE, 0, 256);
    memset(ACGT_TABLE, 0, 256);
    for (size_t i = 0; i < sizeof(codes) / sizeof(codes[0]); ++i) {
        int c = codes[i][0], v = atoi(codes[i] + 1);
        IUPAC_TABLE[c] = IUPAC_TABLE[tolower(c)] = (uint8_t)v;
        if (v == 1 || v == 2 || v == 4 || v == 8) ACGT_TABLE[c] = ACGT_TABLE[tolower(c)] = (uint8_t)v;
    }
    /* dnaio reverse_complement table: ACGTUMRWSYKVHDBN (+ lowercase); other bytes unchanged. */
    for (int i = 0; i < 256; ++i) COMPLEMENT[i] = (uint8_t)i;
    const char* from = "ACGTUMRWSYKVHDBNacgtumrwsykvhdbn";
    const char* to = "TGCAAKYWSRMBDHVNtgcaakywsrmbdhvn";
    for (int i = 0; from[i]; ++i) COMPLEMENT[(uint8_t)from[i]] = (uint8_t)to[i];
}

void orc_revcomp(const char* in, int n, char* out) {
    pthread_once(&tables_once, init_tables);
    for (int i = 0; i < n; ++i) out[i] = (char)COMPLEMENT[(uint8_t)in[n - 1 - i]];
}

/* ------------------------------------------------------------------------------------------ */
/* Aligner (cutadapt/_align.pyx class Aligner)                                                 */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    int cost, score, origin;
} orc_entry;

typedef struct {
    int m;
    uint8_t ref[256];   /* translated reference */
    int n_counts[257];  /* n_counts[i] = #N in reference[:i]                                  */
    int effective_length;
    double max_error_rate;
    int start_in_ref, start_in_query, stop_in_ref, stop_in_query;
    int wildcard_ref, wildcard_query, min_overlap;
} orc_aligner;

/* Aligner.__cinit__ / _set_reference.  Returns 0, or -1 on bad input. */
static int aligner_init(orc_aligner* al, const char* reference, int m, double max_error_rate,
                        int flags, int wildcard_ref, int wildcard_query, int min_overlap) {
    pthread_once(&tables_once, init_tables);
    if (m <= 0 || m > 255) return -1;
    memset(al, 0, sizeof(*al));
    al->m = m;
    al->max_error_rate = max_error_rate;
    al->start_in_ref = (flags & ORC_REF_START) != 0;
    al->start_in_query = (flags & ORC_QUERY_START) != 0;
    al->stop_in_ref = (flags & ORC_REF_END) != 0;
    al->stop_in_query = (flags & ORC_QUERY_STOP) != 0;
    al->wildcard_ref = wildcard_ref;
    al->wildcard_query = wildcard_query;
    al->min_overlap = min_overlap;
    int nc = 0;
    for (int i = 0; i < m; ++i) {
        al->n_counts[i] = nc;
        if (reference[i] == 'N' || reference[i] == 'n') ++nc;
    }
    al->n_counts[m] = nc;
    al->effective_length = m;
    for (int i = 0; i < m; ++i) al->ref[i] = (uint8_t)reference[i];
    if (wildcard_ref) {
        al->effective_length = m - nc;
        if (al->effective_length == 0) return -1;
        for (int i = 0; i < m; ++i) al->ref[i] = IUPAC_TABLE[(uint8_t)reference[i]];
    } else if (wildcard_query) {
        for (int i = 0; i < m; ++i) al->ref[i] = ACGT_TABLE[(uint8_t)reference[i]];
    }
    return 0;
}

/* Aligner.locate(query) -> (ref_start, ref_stop, query_start, query_stop, score, errors).
 * Returns 1 and fills out[6] when an acceptable alignment exists, else 0. */
static int aligner_locate(const orc_aligner* al, const char* query, int n, int out[6],
                          uint8_t* s2 /* scratch, >= n bytes */, orc_entry* column /* m+1 */) {
    const int m = al->m;
    const uint8_t* s1 = al->ref;
    int compare_ascii = 0;
    if (al->wildcard_query) {
        for (int j = 0; j < n; ++j) s2[j] = IUPAC_TABLE[(uint8_t)query[j]];
    } else if (al->wildcard_ref) {
        for (int j = 0; j < n; ++j) s2[j] = ACGT_TABLE[(uint8_t)query[j]];
    } else {
        for (int j = 0; j < n; ++j) s2[j] = (uint8_t)toupper((unsigned char)query[j]);
        compare_ascii = 1;
    }
    const double max_error_rate = al->max_error_rate;
    const int k = (int)(max_error_rate * m); /* maximum no. of errors */
    int max_n = n, min_n = 0;
    if (!al->start_in_query) max_n = n < m + k ? n : m + k; /* costs only get worse after m */
    if (!al->stop_in_query) min_n = n - m - k > 0 ? n - m - k : 0;

    /* Fill column min_n (four cases). Scores: match +1, mismatch -1, insertion/deletion -2. */
    for (int i = 0; i <= m; ++i) {
        if (!al->start_in_ref && !al->start_in_query) {
            column[i].score = -2 * (i > min_n ? i : min_n);
            column[i].cost = i > min_n ? i : min_n;
            column[i].origin = 0;
        } else if (al->start_in_ref && !al->start_in_query) {
            column[i].score = 0;
            column[i].cost = min_n;
            column[i].origin = min_n - i < 0 ? min_n - i : 0;
        } else if (!al->start_in_ref && al->start_in_query) {
            column[i].score = -2 * i; /* [UNVERIFIED] i * insertion_score */
            column[i].cost = i;
            column[i].origin = min_n - i > 0 ? min_n - i : 0;
        } else {
            column[i].score = 0;
            column[i].cost = i < min_n ? i : min_n;
            column[i].origin = min_n - i;
        }
    }

    int best_ref_stop = m, best_query_stop = n, best_cost = m + n + 1, best_origin = 0;
    /* [UNVERIFIED] the initial best score.  INT_MIN accepts any acceptable cell, also one whose
     * score is <= 0.  If cutadapt's _align.pyx seeds its best match with score 0 (and keeps the
     * "score > best or (equal and cost lower)" update), accepted cells scoring < 0 would be
     * refused there.  Such cells exist only under an absolute -e or a small -O (DESIGN.md §8c
     * finding 1); at the reference's -e 0.1 -O 3 every accepted cell scores > 0, so the two
     * readings agree.  tools/parity_vs_cutadapt.sh case "negscore" separates them. */
    int best_score = INT_MIN;

    /* Ukkonen's trick: index of the last cell that is at most k */
    int last = m < k + 1 ? m : k + 1;
    if (al->start_in_ref) last = m;

    for (int j = min_n + 1; j <= max_n; ++j) {
        orc_entry diag_entry = column[0]; /* remember first entry before overwriting */
        if (al->start_in_query) {
            column[0].origin = j;
        } else {
            column[0].cost = j;
            column[0].score = -2 * j;
        }
        for (int i = 1; i <= last; ++i) {
            int equal = compare_ascii ? (s1[i - 1] == s2[j - 1]) : ((s1[i - 1] & s2[j - 1]) != 0);
            int cost, origin, score;
            if (equal) {
                cost = diag_entry.cost;
                origin = diag_entry.origin;
                score = diag_entry.score + 1;
            } else {
                int cost_diag = diag_entry.cost + 1;
                int cost_deletion = column[i].cost + 1;
                int cost_insertion = column[i - 1].cost + 1;
                if (cost_diag <= cost_deletion && cost_diag <= cost_insertion) { /* MISMATCH */
                    cost = cost_diag;
                    origin = diag_entry.origin;
                    score = diag_entry.score - 1;
                } else if (cost_insertion <= cost_deletion) { /* INSERTION */
                    cost = cost_insertion;
                    origin = column[i - 1].origin;
                    score = column[i - 1].score - 2;
                } else { /* DELETION */
                    cost = cost_deletion;
                    origin = column[i].origin;
                    score = column[i].score - 2;
                }
            }
            diag_entry = column[i];
            column[i].cost = cost;
            column[i].origin = origin;
            column[i].score = score;
        }
        while (last >= 0 && column[last].cost > k) --last;
        if (last < m) {
            ++last;
        } else if (al->stop_in_query) {
            /* Found a match in the last row. */
            int length = m + (column[m].origin < 0 ? column[m].origin : 0);
            int cur_effective_length = length;
            if (al->wildcard_ref) {
                cur_effective_length =
                    length < m ? length - al->n_counts[length] : al->effective_length;
            }
            int cost = column[m].cost, score = column[m].score;
            int acceptable = length >= al->min_overlap &&
                             (double)cost <= (double)cur_effective_length * max_error_rate;
            /* [UNVERIFIED] tie rule: higher score wins; equal score -> lower cost. */
            if (acceptable && (score > best_score || (score == best_score && cost < best_cost))) {
                best_score = score;
                best_cost = cost;
                best_origin = column[m].origin;
                best_ref_stop = m;
                best_query_stop = j;
                if (cost == 0 && score == m) break; /* exact full match: stop early */
            }
        }
    }
    if (max_n == n) {
        int first_i = al->stop_in_ref ? 0 : m;
        for (int i = first_i; i <= m; ++i) { /* search in last column */
            int length = i + (column[i].origin < 0 ? column[i].origin : 0);
            int cur_effective_length = length;
            if (al->wildcard_ref) {
                cur_effective_length =
                    length < m ? length - al->n_counts[length] : al->effective_length;
            }
            int cost = column[i].cost, score = column[i].score;
            int acceptable = length >= al->min_overlap &&
                             (double)cost <= (double)cur_effective_length * max_error_rate;
            if (acceptable && (score > best_score || (score == best_score && cost < best_cost))) {
                best_score = score;
                best_cost = cost;
                best_origin = column[i].origin;
                best_ref_stop = i;
                best_query_stop = n;
            }
        }
    }
    if (best_cost == m + n + 1) return 0;
    int start1, start2;
    if (best_origin >= 0) {
        start1 = 0;
        start2 = best_origin;
    } else {
        start1 = -best_origin;
        start2 = 0;
    }
    out[0] = start1;
    out[1] = best_ref_stop;
    out[2] = start2;
    out[3] = best_query_stop;
    out[4] = best_score;
    out[5] = best_cost;
    return 1;
}

/* Stand-alone locate for tests: ref/query ASCII. */
int orc_locate(const char* ref, int m, const char* query, int n, double max_error_rate, int flags,
               int wildcard_ref, int wildcard_query, int min_overlap, int out[6]) {
    orc_aligner al;
    if (aligner_init(&al, ref, m, max_error_rate, flags, wildcard_ref, wildcard_query,
                     min_overlap) != 0)
        return -1;
    uint8_t* s2 = (uint8_t*)malloc((size_t)n + 1);
    orc_entry column[257];
    int r = aligner_locate(&al, query, n, out, s2, column);
    free(s2);
    return r;
}

/* ------------------------------------------------------------------------------------------ */
/* Panels of adapters (adapters.py FrontAdapter/BackAdapter, modifiers.py AdapterCutter)       */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    int n;
    int where[64]; /* ORC_FRONT / ORC_BACK per adapter */
    orc_aligner al[64];
} orc_panel;

/* Matches the layout of dmx_match in include/dmx.h (kept independent on purpose). */
typedef struct {
    int32_t rstart, rstop;
    int16_t astart, astop;
    int16_t score, errors;
} orc_match;

typedef struct {
    int16_t bin1, bin2;
    uint8_t rc1, rc2, flags, pad;
    orc_match m1, m2;
} orc_result;

/* Build a panel.  seqs[i] must already be uppercased with U->T (parser.py does so).
 * Adapter wildcards are enabled iff the sequence has a non-ACGT character
 * (adapters.py: adapter_wildcards and not set(sequence) <= set("ACGT")).
 * max_errors >= 1 is an absolute error count (converted per adapter to a rate). */
orc_panel* orc_panel_new(int n, const char* const* seqs, const int* lens, const int* where,
                         double max_errors, int min_overlap) {
    pthread_once(&tables_once, init_tables);
    if (n <= 0 || n > 64) return NULL;
    orc_panel* p = (orc_panel*)calloc(1, sizeof(orc_panel));
    p->n = n;
    for (int a = 0; a < n; ++a) {
        int wild = 0;
        for (int i = 0; i < lens[a]; ++i) {
            char c = seqs[a][i];
            if (c != 'A' && c != 'C' && c != 'G' && c != 'T') wild = 1;
        }
        double rate = max_errors >= 1.0 ? max_errors / (double)lens[a] : max_errors;
        p->where[a] = where[a];
        if (aligner_init(&p->al[a], seqs[a], lens[a], rate, where[a], wild, 0, min_overlap) != 0) {
            free(p);
            return NULL;
        }
    }
    return p;
}

void orc_panel_free(orc_panel* p) { free(p); }

typedef struct {
    uint8_t* s2;
    orc_entry column[257];
} orc_scratch;

/* AdapterCutter.best_match over adapters in file order: keep the match with greater score;
 * on equal score the one with fewer errors [UNVERIFIED]; else the earlier adapter.
 * Returns adapter index or -1. */
static int best_match(const orc_panel* p, const char* seq, int n, orc_match* out,
                      orc_scratch* sc) {
    int best = -1;
    orc_match bm;
    memset(&bm, 0, sizeof(bm));
    for (int a = 0; a < p->n; ++a) {
        int r[6];
        if (!aligner_locate(&p->al[a], seq, n, r, sc->s2, sc->column)) continue;
        if (best < 0 || r[4] > bm.score || (r[4] == bm.score && r[5] < bm.errors)) {
            best = a;
            bm.astart = (int16_t)r[0];
            bm.astop = (int16_t)r[1];
            bm.rstart = r[2];
            bm.rstop = r[3];
            bm.score = (int16_t)r[4];
            bm.errors = (int16_t)r[5];
        }
    }
    *out = bm;
    return best;
}

/* One demux round with --rc (modifiers.py ReverseComplementer): best match on the read and on
 * its reverse complement; RC is used iff its score is strictly greater.  Writes the trimmed
 * sequence of the chosen orientation to trimmed[] (FRONT: seq[rstop:], BACK: seq[:rstart];
 * untrimmed forward read when nothing matched).  Returns the adapter index or -1. */
static int demux_round(const orc_panel* p, const char* seq, int n, int use_rc, uint8_t* is_rc,
                       orc_match* m, char* rc_buf, char* trimmed, int* trimmed_len,
                       orc_scratch* sc) {
    orc_match mf, mr;
    int af = best_match(p, seq, n, &mf, sc);
    int ar = -1;
    if (use_rc) {
        orc_revcomp(seq, n, rc_buf);
        ar = best_match(p, rc_buf, n, &mr, sc);
    }
    int fscore = af >= 0 ? mf.score : 0, rscore = ar >= 0 ? mr.score : 0;
    const char* src = seq;
    int a = af;
    *is_rc = 0;
    if (use_rc && rscore > fscore) {
        *is_rc = 1;
        src = rc_buf;
        a = ar;
        *m = mr;
    } else if (af >= 0) {
        *m = mf;
    } else {
        memset(m, 0, sizeof(*m));
    }
    if (a < 0) {
        memcpy(trimmed, seq, (size_t)n);
        *trimmed_len = n;
        return -1;
    }
    if (p->where[a] == ORC_FRONT) {
        *trimmed_len = n - m->rstop;
        memcpy(trimmed, src + m->rstop, (size_t)*trimmed_len);
    } else {
        *trimmed_len = m->rstart;
        memcpy(trimmed, src, (size_t)*trimmed_len);
    }
    return a;
}

/* Single round on one read (what one cutadapt invocation does).  Returns adapter idx or -1. */
int orc_round(const orc_panel* p, const char* seq, int n, int use_rc, orc_result* res,
              char* trimmed, int* trimmed_len) {
    orc_scratch sc;
    sc.s2 = (uint8_t*)malloc((size_t)n + 1);
    char* rc = (char*)malloc((size_t)n + 1);
    memset(res, 0, sizeof(*res));
    res->bin2 = -1;
    int a = demux_round(p, seq, n, use_rc, &res->rc1, &res->m1, rc, trimmed, trimmed_len, &sc);
    res->bin1 = (int16_t)a;
    free(rc);
    free(sc.s2);
    return a;
}

/* Two-round composition of 02_cutadapt_loop.sh: round 1 (panel p1, normally FRONT) on the read;
 * reads with a round-1 match go to round 2 (panel p2, normally BACK) on the round-1-trimmed
 * sequence.  final[] receives the round-2-trimmed sequence (the record written to the
 * SP27_x_SP5_y file).  Returns 0. */
int orc_two_round(const orc_panel* p1, const orc_panel* p2, const char* seq, int n, int use_rc,
                  orc_result* res, char* final_seq, int* final_len) {
    orc_scratch sc;
    sc.s2 = (uint8_t*)malloc((size_t)n + 1);
    char* rc = (char*)malloc((size_t)n + 1);
    char* t1 = (char*)malloc((size_t)n + 1);
    int t1_len = 0;
    memset(res, 0, sizeof(*res));
    res->bin2 = -1;
    int a = demux_round(p1, seq, n, use_rc, &res->rc1, &res->m1, rc, t1, &t1_len, &sc);
    res->bin1 = (int16_t)a;
    *final_len = 0;
    if (a >= 0) {
        int b = demux_round(p2, t1, t1_len, use_rc, &res->rc2, &res->m2, rc, final_seq, final_len,
                            &sc);
        res->bin2 = (int16_t)b;
    }
    free(t1);
    free(rc);
    free(sc.s2);
    return 0;
}

/* Linked adapters -g F...R (adapters.py LinkedAdapter.match_to; both parts required with -g
 * [UNVERIFIED]): front match on the read, back match on read[front.rstop:]; best linked adapter by
 * summed score, ties -> fewer summed errors, then earlier.  No --rc (04_cleaning_primers.sh:377).
 * Coordinates: m1 in read coords, m2 in coords of read[m1.rstop:].  Returns pair index or -1. */
int orc_linked(const orc_panel* fronts, const orc_panel* backs, const char* seq, int n,
               orc_result* res) {
    orc_scratch sc;
    sc.s2 = (uint8_t*)malloc((size_t)n + 1);
    int best = -1, best_score = 0, best_err = 0;
    orc_match bf, bb;
    memset(res, 0, sizeof(*res));
    res->bin1 = res->bin2 = -1;
    for (int a = 0; a < fronts->n; ++a) {
        int rf[6], rb[6];
        if (!aligner_locate(&fronts->al[a], seq, n, rf, sc.s2, sc.column)) continue;
        if (!aligner_locate(&backs->al[a], seq + rf[3], n - rf[3], rb, sc.s2, sc.column)) continue;
        int score = rf[4] + rb[4], err = rf[5] + rb[5];
        if (best < 0 || score > best_score || (score == best_score && err < best_err)) {
            best = a;
            best_score = score;
            best_err = err;
            bf.astart = (int16_t)rf[0];
            bf.astop = (int16_t)rf[1];
            bf.rstart = rf[2];
            bf.rstop = rf[3];
            bf.score = (int16_t)rf[4];
            bf.errors = (int16_t)rf[5];
            bb.astart = (int16_t)rb[0];
            bb.astop = (int16_t)rb[1];
            bb.rstart = rb[2];
            bb.rstop = rb[3];
            bb.score = (int16_t)rb[4];
            bb.errors = (int16_t)rb[5];
        }
    }
    if (best >= 0) {
        res->bin1 = res->bin2 = (int16_t)best;
        res->m1 = bf;
        res->m2 = bb;
    }
    free(sc.s2);
    return best;
}

/* ------------------------------------------------------------------------------------------ */
/* Batch drivers (pthreads) — used by tests for bulk comparison and by bench.py cpu_baseline.  */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    const orc_panel *p1, *p2;
    const char* seqs;
    const uint64_t* offs;
    const uint32_t* lens;
    orc_result* res;
    int use_rc, linked;
    size_t lo, hi;
} batch_job;

static void* batch_worker(void* arg) {
    batch_job* j = (batch_job*)arg;
    size_t maxlen = 0;
    for (size_t r = j->lo; r < j->hi; ++r)
        if (j->lens[r] > maxlen) maxlen = j->lens[r];
    char* fin = (char*)malloc(maxlen + 1);
    for (size_t r = j->lo; r < j->hi; ++r) {
        const char* s = j->seqs + j->offs[r];
        int n = (int)j->lens[r];
        if (j->linked) {
            orc_linked(j->p1, j->p2, s, n, &j->res[r]);
        } else if (j->p2) {
            int fl;
            orc_two_round(j->p1, j->p2, s, n, j->use_rc, &j->res[r], fin, &fl);
        } else {
            int tl;
            orc_round(j->p1, s, n, j->use_rc, &j->res[r], fin, &tl);
        }
    }
    free(fin);
    return NULL;
}

/* mode: 0 = single round (p2 ignored), 1 = two rounds, 2 = linked (p1 fronts, p2 backs). */
int orc_batch(const orc_panel* p1, const orc_panel* p2, int mode, int use_rc, const char* seqs,
              const uint64_t* offs, const uint32_t* lens, size_t n_reads, orc_result* res,
              int n_threads) {
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256];
    batch_job jobs[256];
    size_t per = (n_reads + (size_t)n_threads - 1) / (size_t)n_threads;
    int started = 0;
    for (int t = 0; t < n_threads; ++t) {
        size_t lo = (size_t)t * per, hi = lo + per > n_reads ? n_reads : lo + per;
        if (lo >= hi) break;
        jobs[t] = (batch_job){p1, mode == 0 ? NULL : p2, seqs, offs, lens, res, use_rc, mode == 2,
                              lo, hi};
        pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
        ++started;
    }
    for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
    return 0;
}
