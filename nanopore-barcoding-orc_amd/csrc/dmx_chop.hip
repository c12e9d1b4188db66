// dmx_chop.hip — pychopper-style read reorientation on the GPU, the
// producer of the demultiplexer's input:
//
//   scripts/01_pychopper.sh:45-57   pychopper -b adapters_primers/M13_seqs_for_pychopper.fa
//                                   -c adapters_primers/M13_config_for_pychopper.txt -k LSK114
//                                   -Q 10 -w R -u U -l S -S STATS -p -t 24 -m edlib IN > PASS
//
// pychopper 2.7.10 and its edlib backend are not vendored in /root/reference and not installed
// here: the semantics are the build's restatement (checkers oracle/chop_oracle.c
// and oracle/chopper.py), parity unpinned.  Per read:
//   hits      every label (each primer of the -b FASTA and its reverse complement; IUPAC codes,
//             N = any base; a read N matches anything) is searched like one edlib HW / TASK_LOC
//             call with k = int(cutoff * m) (edlib 1.3.x edlibAlign): D(j) = least edit distance
//             of the label ending at read column j, best = min over the read of D(j); when
//             best <= k every column with D(j) == best is a hit (edlib's end locations) whose
//             start is that of the LONGEST optimal alignment ending there (edlib's reverse SHW
//             alignment, last position);
//   segments  the read's hits sorted by (start, stop, label); consecutive hits (a, b) whose
//             labels form a configuration rule (-c, e.g. "+:SP5,-SP27|-:SP27,-SP5") are a
//             candidate segment on the rule's strand, span [a.start, b.stop) with -p (keep
//             primers), else [a.stop, b.start) (empty if the hits overlap).  The segments are
//             the best path over the candidates: no shared hit, greatest summed length
//             (pychopper's usable length), ties -> the earlier candidate.
// The host (dmx/chop.py) classifies reads by segment count and writes the outputs.
//
// MI355X design — integer/bit work, VALU-bound like the demux filter (no MFMA, no GEMM shape):
//   chop_kernel   a block owns up to 64 consecutive reads.  Its lanes take (512-column segment,
//                 label) tasks, labels fastest, so the lanes of one segment load the same packed
//                 words.  A lane runs the 64-bit Myers/Hyyro step of the demux scans (labels
//                 <= 64 nt) from m + k columns before its segment — exact for every D <= k from
//                 the segment's first column on, as an alignment of cost <= k spans <= m + k
//                 columns — keeps, per run of D <= k inside its segment, the columns at the
//                 run's minimum (first column + a 64-bit offset mask), and at the run's end
//                 appends them to an LDS hit list unless a lower D was already seen for the
//                 (read, label): by this lane, or by any lane through the block's LDS minimum
//                 (atomicMin).  After a barrier the hits above the (read, label) minimum are
//                 dropped and one lane per hit finds its start (an anchored Myers scan of the
//                 reverse-complement label over the reverse-complement view, m + best
//                 columns); the block groups its hits by read (counting scatter), one
//                 lane per read insertion-sorts its few hits and picks its segments, and the block
//                 reserves its ranges of the global hit and segment lists with one atomic each.
//   chop_blkscan_kernel, chop_order_kernel
//                 move every block's ranges into read order (block order = read order), so the
//                 host receives read-ordered hits and segments without a sort.
// A block whose hits overflow its LDS list (reads with hundreds of primer hits) is redone alone
// by chop_big_kernel: hit lists in global memory sized by the count the LDS pass measured
// without the cross-lane pruning (which depends on timing; the redo prunes within lanes only),
// counting scatter by read, parallel rank sort per read; a staging overflow re-runs with larger
// buffers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstring>
#include <string>
#include <vector>

#include "dmx_internal.h"

namespace dmx {

constexpr int kChopMaxLabels = 2 * DMX_CHOP_MAX_PRIMERS;
constexpr int kChopMaxRules = DMX_CHOP_MAX_RULES;
#ifndef DMX_CHOP_SEG
#define DMX_CHOP_SEG 512
#endif
constexpr uint32_t kChopSeg = DMX_CHOP_SEG;   // columns owned by one scan lane
constexpr int kChopBlock = 256;
constexpr uint32_t kChopReads = 64;      // reads per block (first launch)
constexpr uint32_t kChopHitCap = 512;    // LDS hit list per block

struct ChopLabel {
    uint64_t peq[8];   // match vectors by read code | no-match bit << 2 (4..7: read N, all rows)
    int32_t m, k;
};
struct ChopPanel {
    int32_t n_labels, keep, n_rules, pad;
    int8_t rule[kChopMaxLabels * kChopMaxLabels];   // first rule pairing (left, right), or -1
    int8_t rstrand[kChopMaxRules];
    ChopLabel lab[kChopMaxLabels];
};
static_assert(sizeof(dmx_chop_hit) == 16 && sizeof(dmx_chop_seg) == 16, "record layout");
static_assert(sizeof(ChopLabel) % 8 == 0 && offsetof(ChopPanel, lab) % 8 == 0, "panel layout");

struct ChopArgs {
    Packed pk;                 // the resident packed batch (+ bounds in DMX_DEBUG_BOUNDS builds)
    const uint64_t* offs;
    const uint32_t* lens;
    uint32_t n_reads;
    const ChopPanel* panel;
    dmx_chop_hit* hits;        // staging: block ranges in reservation order
    dmx_chop_seg* segs;
    uint64_t hit_cap, seg_cap;
    uint32_t* nhit;            // per read
    uint32_t* nseg;
    uint32_t* blk;             // per block: hit base, hits, segment base, segments
    unsigned long long* ctr;   // [0] hits, [1] segments, [2] flags (bit 0: LDS list overflow),
                               // [3] blocks overflowing their LDS hit list
    uint32_t* ovf;             // (block, exact hit count) of each such block
    uint64_t ovf_cap;
};

struct ChopOrderArgs {
    const uint32_t* blk;
    const uint32_t* off;       // per block: read-order hit offset, segment offset
    uint32_t nb;
    const dmx_chop_hit* hstage;
    dmx_chop_hit* hits;
    const dmx_chop_seg* sstage;
    dmx_chop_seg* segs;
};

// Where a scan lane appends its hits.  nall == nullptr (chop_big_kernel): every hit that passes
// the lane's own minimum is stored (a count the LDS pass measured exactly); otherwise hits are
// stored only if no lower D is known for the (read, label) yet, and nall counts them all.
struct ChopSink {
    uint32_t* nh;          // stored hits (keeps counting past cap)
    uint32_t* nall;        // hits before the cross-lane pruning, or nullptr
    dmx_chop_hit* list;
    uint32_t cap;
    uint32_t* smin;        // the block's least D per (read, label): [read - r0][label]
    uint32_t r0;
};

__device__ __forceinline__ void chop_push(const ChopSink& S, uint32_t read, int lab, int dist,
                                          uint32_t stop) {
    const uint32_t i = atomicAdd(S.nh, 1u);
    if (i < S.cap) {
        dmx_chop_hit h;
        h.read = read;
        h.label = (int16_t)lab;
        h.dist = (int16_t)dist;
        h.start = -1;
        h.stop = (int32_t)stop;
        S.list[i] = h;
    }
}

// The columns at one run's minimum: bstop and bstop + every set bit of `more`.
__device__ __forceinline__ void chop_flush(const ChopSink& S, uint32_t read, int lab, int best,
                                           uint32_t bstop, uint64_t more, int& lmin) {
    if (best > lmin) return;
    lmin = best;
    uint32_t* smin = S.smin + (read - S.r0) * (uint32_t)kChopMaxLabels + (uint32_t)lab;
    bool store = true;
    if (S.nall) {
        atomicAdd(S.nall, 1u + (uint32_t)__popcll(more));
        store = (uint32_t)best <= *smin;
    }
    atomicMin(smin, (uint32_t)best);
    if (!store) return;
    chop_push(S, read, lab, best, bstop);
    while (more) {
        chop_push(S, read, lab, best, bstop + (uint32_t)__builtin_ctzll(more));
        more &= more - 1ull;
    }
}

// One (segment, label) task: D(j) over the owned columns (s0, s0 + kChopSeg] of the read.
// HB: the last row's bit is in the low (0) or high (1) 32-bit half for every label, or -1
// (mixed: selected per step).
template <int HB>
__device__ __forceinline__ void chop_scan(const ChopArgs& A, const ChopLabel& L, int lab,
                                          uint32_t read, uint32_t si, const ChopSink& S) {
    const uint32_t n = A.lens[read];
    const uint64_t off = A.offs[read];
    const int m = L.m, k = L.k;
    const uint32_t hbit = (uint32_t)(m - 1);
    const uint32_t s0 = si * kChopSeg, s1 = s0 + kChopSeg;
    const uint32_t send = min(n, s1);
    // warm-up: starting at ws, the scan's D(m, j) is the true value whenever an optimal
    // alignment starts at or after ws, and never below it.  An alignment of cost c <= k spans
    // at most m + c columns, so from column ws + m + k on every D <= k is exact and every
    // D > k stays > k: D(j) is exact wherever it matters for j > s0.  Runs crossing a segment
    // boundary are split; each piece reports its own minimum columns, a superset of the
    // columns at the (read, label) minimum, which the block keeps.
    const uint32_t wu = (uint32_t)(m + k);
    const uint32_t ws = s0 > wu ? s0 - wu : 0u;
    uint64_t pv = ~0ull, mv = 0ull, more = 0ull;
    int d = m;
    bool run = false;
    int best = 0, lmin = k;
    uint32_t bstop = 0;
    for (uint32_t p = ws; p < send; p += 16) {
        uint32_t codes, nb;
        fetch16(A.pk, off, n, 0u, 0u, p, codes, nb);
        const uint32_t cnt = min(16u, send - p);
        uint64_t eqv[16];
#pragma unroll
        for (int q = 0; q < 16; ++q)
            eqv[q] = L.peq[((codes >> (2 * q)) & 3u) | (((nb >> q) & 1u) << 2)];
#pragma unroll
        for (int h = 0; h < 16; h += 8) {
            // quiet stretch: outside a run with d > k + 8, |D(j) - D(j-1)| <= 1 keeps the next 8
            // columns above k, so when every lane of the wave is quiet and has 8 columns left
            // they take bare steps (no run tracking, no per-column exec masking).
            if (__all(!run && d > k + 8 && cnt >= (uint32_t)h + 8u)) {
#pragma unroll
                for (int q = h; q < h + 8; ++q) myers_step<HB>(eqv[q], pv, mv, d, hbit);
                continue;
            }
#pragma unroll
            for (int q = h; q < h + 8; ++q) {
                if ((uint32_t)q < cnt) {
                    myers_step<HB>(eqv[q], pv, mv, d, hbit);
                    const uint32_t j = p + (uint32_t)q + 1u;
                    if (d <= k && j > s0) {
                        if (!run || d < best) {
                            run = true;
                            best = d;
                            bstop = j;
                            more = 0ull;
                        } else if (d == best) {
                            if (j - bstop < 64u) {
                                more |= 1ull << (j - bstop);
                            } else {   // a long run: report these columns, keep collecting
                                chop_flush(S, read, lab, best, bstop, more, lmin);
                                bstop = j;
                                more = 0ull;
                            }
                        }
                    } else if (run) {
                        run = false;
                        chop_flush(S, read, lab, best, bstop, more, lmin);
                    }
                }
            }
        }
    }
    if (run) chop_flush(S, read, lab, best, bstop, more, lmin);
}

// Start of the longest optimal alignment ending at `stop` (edlib: the last position of the
// reverse SHW alignment): the reverse-complement label R (label ^ 1) anchored at
// reverse-complement view position n - stop (row 0 = t: the text is not free at the anchor),
// last t <= m + best with D'(m, t) == best.  min over t of D'(m, t) is `best`.
__device__ int chop_start(const ChopArgs& A, const ChopLabel& R, uint32_t read, int best,
                          uint32_t stop) {
    const uint32_t n = A.lens[read];
    const uint64_t off = A.offs[read];
    const int m = R.m;
    const uint32_t hb = (uint32_t)(m - 1);
    uint64_t pv = ~0ull, mv = 0ull;
    int d = m;
    const uint32_t tmax = min(stop, (uint32_t)(m + best));
    int start = -1;
    for (uint32_t t0 = 0; t0 < tmax; t0 += 16) {
        uint32_t codes, nb;
        fetch16(A.pk, off, n, 1u, 0u, n - stop + t0, codes, nb);
        const uint32_t cnt = min(16u, tmax - t0);
        for (uint32_t q = 0; q < cnt; ++q) {
            const uint64_t eq = R.peq[((codes >> (2 * q)) & 3u) | (((nb >> q) & 1u) << 2)];
            const uint64_t xv = eq | mv;
            const uint64_t xh = (((eq & pv) + pv) ^ pv) | eq;
            uint64_t ph = mv | ~(xh | pv);
            uint64_t mh = pv & xh;
            d += (int)((ph >> hb) & 1ull) - (int)((mh >> hb) & 1ull);
            ph = (ph << 1) | 1ull;
            mh <<= 1;
            pv = mh | ~(xv | ph);
            mv = ph & xv;
            if (d == best) start = (int)(stop - (t0 + q + 1u));
        }
    }
    return start;
}

__device__ __forceinline__ bool hit_less(const dmx_chop_hit& a, const dmx_chop_hit& b) {
    if (a.start != b.start) return a.start < b.start;
    if (a.stop != b.stop) return a.stop < b.stop;
    return a.label < b.label;
}

__device__ __forceinline__ void chop_load_panel(const ChopPanel* P, ChopLabel* s_lab,
                                                int8_t* s_rule, int8_t* s_rstrand) {
    for (int i = threadIdx.x; i < P->n_labels * (int)(sizeof(ChopLabel) / 8); i += blockDim.x)
        reinterpret_cast<uint64_t*>(s_lab)[i] = reinterpret_cast<const uint64_t*>(P->lab)[i];
    for (int i = threadIdx.x; i < kChopMaxLabels * kChopMaxLabels; i += blockDim.x)
        s_rule[i] = P->rule[i];
    if (threadIdx.x < kChopMaxRules) s_rstrand[threadIdx.x] = P->rstrand[threadIdx.x];
}

// s_pre[t] = first (segment) task of read r0 + t, s_pre[nr] = the block's segments; s_cnt is
// left zeroed.  Every thread must call it.
__device__ __forceinline__ void chop_segment_prefix(const ChopArgs& A, uint32_t r0, uint32_t nr,
                                                    uint32_t* s_cnt, uint32_t* s_pre) {
    if (threadIdx.x < nr)
        s_cnt[threadIdx.x] = (A.lens[r0 + threadIdx.x] + kChopSeg - 1u) / kChopSeg;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (uint32_t t = 0; t < nr; ++t) {
            s_pre[t] = acc;
            acc += s_cnt[t];
            s_cnt[t] = 0u;
        }
        s_pre[nr] = acc;
    }
    __syncthreads();
}

// Last t in [0, nr) with pre[t] <= x.
__device__ __forceinline__ uint32_t chop_last_le(const uint32_t* pre, uint32_t nr, uint32_t x) {
    uint32_t lo = 0, hi = nr - 1u;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1u) >> 1;
        if (pre[mid] <= x) lo = mid;
        else hi = mid - 1u;
    }
    return lo;
}

// Once every read's hits are sorted in srt[s_off[t] .. s_off[t + 1]): one lane per read picks
// the best path over its candidate segments into seg[s_off[t] ...] (seg must not alias srt), the block reserves its output
// ranges (one atomic per list) and writes them.  srt / seg: LDS (chop_kernel) or global scratch
// (chop_big_kernel).  Every thread must call it.
__device__ void chop_pair_write(const ChopArgs& A, uint32_t b, uint32_t r0, uint32_t nr,
                                uint32_t nh, bool keep, const int8_t* s_rule,
                                const int8_t* s_rstrand, const dmx_chop_hit* srt,
                                dmx_chop_seg* seg, const uint32_t* s_off, uint32_t* s_sc,
                                uint32_t* s_soff, uint32_t* s_base) {
    if (threadIdx.x < nr) {
        const uint32_t t = threadIdx.x;
        const uint32_t o = s_off[t], c = s_off[t + 1] - o;
        // Best path, right to left: b1 / b2 = greatest summed length over hits a+1.. / a+2..;
        // candidate a (consecutive hits a, a+1 forming a rule) is taken when it reaches at
        // least b1 (ties -> the earlier candidate).  Decisions go to the first word of seg[o+a]
        // (free until the forward pass writes segment ns <= a over it, after reading it).
        uint32_t* take = reinterpret_cast<uint32_t*>(seg + o);
        uint64_t b1 = 0, b2 = 0;
        for (uint32_t a = c > 1u ? c - 1u : 0u; a-- > 0;) {
            const dmx_chop_hit h1 = srt[o + a], h2 = srt[o + a + 1];
            uint64_t cur = b1;
            uint32_t tk = 0;
            if (s_rule[h1.label * kChopMaxLabels + h2.label] >= 0) {
                const int32_t x0 = keep ? h1.start : h1.stop;
                const int32_t x1 = keep ? h2.stop : h2.start;
                const uint64_t v = (uint64_t)(uint32_t)max(0, x1 - x0) + b2;
                if (v >= b1) {
                    cur = v;
                    tk = 1u;
                }
            }
            take[4 * a] = tk;
            b2 = b1;
            b1 = cur;
        }
        uint32_t ns = 0;
        for (uint32_t a = 0; a + 1 < c;) {
            if (take[4 * a]) {
                const dmx_chop_hit h1 = srt[o + a], h2 = srt[o + a + 1];
                const int ri = s_rule[h1.label * kChopMaxLabels + h2.label];
                dmx_chop_seg sg;
                sg.read = h1.read;
                const int32_t x0 = keep ? h1.start : h1.stop;
                const int32_t x1 = keep ? h2.stop : h2.start;
                sg.start = x0;
                sg.stop = max(x0, x1);
                sg.strand = (int16_t)s_rstrand[ri];
                sg.rule = (int16_t)ri;
                seg[o + ns] = sg;
                ++ns;
                a += 2;
            } else {
                ++a;
            }
        }
        s_sc[t] = ns;
        A.nhit[r0 + t] = c;
        A.nseg[r0 + t] = ns;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (uint32_t t = 0; t < nr; ++t) {
            s_soff[t] = acc;
            acc += s_sc[t];
        }
        s_soff[nr] = acc;
        s_base[0] = (uint32_t)atomicAdd(&A.ctr[0], (unsigned long long)nh);
        s_base[1] = (uint32_t)atomicAdd(&A.ctr[1], (unsigned long long)acc);
        A.blk[4 * b + 0] = s_base[0];
        A.blk[4 * b + 1] = nh;
        A.blk[4 * b + 2] = s_base[1];
        A.blk[4 * b + 3] = acc;
    }
    __syncthreads();
    const uint64_t hb = s_base[0], sb = s_base[1];
    for (uint32_t i = threadIdx.x; i < nh; i += blockDim.x)
        if (hb + i < A.hit_cap) A.hits[hb + i] = srt[i];
    const uint32_t nsg = s_soff[nr];
    for (uint32_t i = threadIdx.x; i < nsg; i += blockDim.x) {
        const uint32_t t = chop_last_le(s_soff, nr, i);
        if (sb + i < A.seg_cap) A.segs[sb + i] = seg[s_off[t] + (i - s_soff[t])];
    }
}

template <int HB>
__global__ __launch_bounds__(kChopBlock) void chop_kernel(ChopArgs A) {
    __shared__ ChopLabel s_lab[kChopMaxLabels];
    __shared__ int8_t s_rule[kChopMaxLabels * kChopMaxLabels];
    __shared__ int8_t s_rstrand[kChopMaxRules];
    __shared__ uint32_t s_pre[kChopReads + 1], s_off[kChopReads + 1], s_soff[kChopReads + 1];
    __shared__ uint32_t s_cnt[kChopReads], s_sc[kChopReads];
    __shared__ dmx_chop_hit s_hit[kChopHitCap];
    __shared__ dmx_chop_hit s_srt[kChopHitCap];
    __shared__ uint32_t s_nh, s_nall, s_base[2];
    // least D per (read, label) during the scans and the filter; s_srt is written only after
    static_assert(kChopReads * kChopMaxLabels * 4 <= sizeof(dmx_chop_hit) * kChopHitCap, "s_min");
    uint32_t* s_min = reinterpret_cast<uint32_t*>(s_srt);
    chop_load_panel(A.panel, s_lab, s_rule, s_rstrand);
    const int NL = A.panel->n_labels;
    const bool keep = A.panel->keep != 0;
    const uint32_t r0 = blockIdx.x * kChopReads;
    const uint32_t nr = min(kChopReads, A.n_reads - r0);
    if (threadIdx.x == 0) s_nh = s_nall = 0u;
    for (uint32_t i = threadIdx.x; i < kChopReads * kChopMaxLabels; i += blockDim.x)
        s_min[i] = ~0u;
    chop_segment_prefix(A, r0, nr, s_cnt, s_pre);

    // 1. scans: (segment, label) tasks, labels fastest
    const ChopSink S{&s_nh, &s_nall, s_hit, kChopHitCap, s_min, r0};
    const uint32_t total = s_pre[nr] * (uint32_t)NL;
    for (uint32_t task = threadIdx.x; task < total; task += blockDim.x) {
        const uint32_t sg = task / (uint32_t)NL;
        const int lab = (int)(task - sg * (uint32_t)NL);
        const uint32_t t = chop_last_le(s_pre, nr, sg);
        chop_scan<HB>(A, s_lab[lab], lab, r0 + t, sg - s_pre[t], S);
    }
    __syncthreads();
    const uint32_t ns = s_nh;
    if (ns > kChopHitCap) {   // block-uniform: redone by chop_big_kernel with the exact count
        if (threadIdx.x == 0) {
            atomicOr(&A.ctr[2], 1ull);
            const unsigned long long i = atomicAdd(&A.ctr[3], 1ull);
            if (i < A.ovf_cap) {
                A.ovf[2 * i] = blockIdx.x;
                A.ovf[2 * i + 1] = s_nall;
            }
        }
        return;
    }

    // 2. drop hits above their (read, label) minimum; starts; group by read (counting scatter)
    for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) {
        dmx_chop_hit h = s_hit[i];
        const uint32_t t = h.read - r0;
        if ((uint32_t)h.dist > s_min[t * kChopMaxLabels + (uint32_t)h.label]) {
            s_hit[i].read = ~0u;
            continue;
        }
        h.start = chop_start(A, s_lab[h.label ^ 1], h.read, h.dist, (uint32_t)h.stop);
        s_hit[i] = h;
        atomicAdd(&s_cnt[t], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (uint32_t t = 0; t < nr; ++t) {
            s_off[t] = acc;
            acc += s_cnt[t];
            s_cnt[t] = 0u;
        }
        s_off[nr] = acc;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) {
        const dmx_chop_hit h = s_hit[i];
        if (h.read == ~0u) continue;
        const uint32_t t = h.read - r0;
        s_srt[s_off[t] + atomicAdd(&s_cnt[t], 1u)] = h;
    }
    __syncthreads();
    const uint32_t nh = s_off[nr];

    // 3. one lane per read: insertion-sort its few hits by (start, stop, label)
    if (threadIdx.x < nr) {
        const uint32_t o = s_off[threadIdx.x], c = s_off[threadIdx.x + 1] - o;
        for (uint32_t a = 1; a < c; ++a) {
            const dmx_chop_hit x = s_srt[o + a];
            uint32_t b = a;
            while (b > 0 && hit_less(x, s_srt[o + b - 1])) {
                s_srt[o + b] = s_srt[o + b - 1];
                --b;
            }
            s_srt[o + b] = x;
        }
    }
    __syncthreads();
    // 4. pair and write; the segments of read t land in s_hit[s_off[t] ...] (free now)
    chop_pair_write(A, blockIdx.x, r0, nr, nh, keep, s_rule, s_rstrand, s_srt,
                    reinterpret_cast<dmx_chop_seg*>(s_hit), s_off, s_sc, s_soff, s_base);
}

// A block of chop_kernel whose hits overflowed its LDS list (reads with hundreds of primer
// hits), redone with the hit lists in global memory: H = scratch[base .. base + count) and
// T = temp[...] of the same size, count = the exact number the LDS pass counted.  Counting
// scatter by read into T, a parallel rank sort of every read's range back into H (the keys
// (start, stop, label) of one read are distinct), then the same pairing and output as
// chop_kernel (one range per 64-read block, so the read-order compaction is unchanged).
__global__ __launch_bounds__(kChopBlock) void chop_big_kernel(ChopArgs A, const uint64_t* base,
                                                              dmx_chop_hit* scratch,
                                                              dmx_chop_hit* temp,
                                                              uint32_t* counter) {
    __shared__ ChopLabel s_lab[kChopMaxLabels];
    __shared__ int8_t s_rule[kChopMaxLabels * kChopMaxLabels];
    __shared__ int8_t s_rstrand[kChopMaxRules];
    __shared__ uint32_t s_pre[kChopReads + 1], s_off[kChopReads + 1], s_soff[kChopReads + 1];
    __shared__ uint32_t s_cnt[kChopReads], s_sc[kChopReads];
    __shared__ uint32_t s_min[kChopReads * kChopMaxLabels];
    __shared__ uint32_t s_base[2];
    for (uint32_t i = threadIdx.x; i < kChopReads * kChopMaxLabels; i += blockDim.x)
        s_min[i] = ~0u;
    chop_load_panel(A.panel, s_lab, s_rule, s_rstrand);
    const int NL = A.panel->n_labels;
    const bool keep = A.panel->keep != 0;
    const uint32_t b = A.ovf[2 * blockIdx.x];
    const uint32_t r0 = b * kChopReads;
    const uint32_t nr = min(kChopReads, A.n_reads - r0);
    const uint32_t cap = (uint32_t)(base[blockIdx.x + 1] - base[blockIdx.x]);
    dmx_chop_hit* H = scratch + base[blockIdx.x];
    dmx_chop_hit* T = temp + base[blockIdx.x];
    uint32_t* cnt = counter + blockIdx.x;
    chop_segment_prefix(A, r0, nr, s_cnt, s_pre);
    const ChopSink S{cnt, nullptr, H, cap, s_min, r0};
    const uint32_t total = s_pre[nr] * (uint32_t)NL;
    for (uint32_t task = threadIdx.x; task < total; task += blockDim.x) {
        const uint32_t sg = task / (uint32_t)NL;
        const int lab = (int)(task - sg * (uint32_t)NL);
        const uint32_t t = chop_last_le(s_pre, nr, sg);
        chop_scan<-1>(A, s_lab[lab], lab, r0 + t, sg - s_pre[t], S);
    }
    __syncthreads();
    const uint32_t ns = min(atomicAdd(cnt, 0u), cap);
    for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) {
        dmx_chop_hit h = H[i];
        const uint32_t t = h.read - r0;
        if ((uint32_t)h.dist > s_min[t * kChopMaxLabels + (uint32_t)h.label]) {
            H[i].read = ~0u;
            continue;
        }
        h.start = chop_start(A, s_lab[h.label ^ 1], h.read, h.dist, (uint32_t)h.stop);
        H[i] = h;
        atomicAdd(&s_cnt[t], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t acc = 0;
        for (uint32_t t = 0; t < nr; ++t) {
            s_off[t] = acc;
            acc += s_cnt[t];
            s_cnt[t] = 0u;
        }
        s_off[nr] = acc;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) {
        const dmx_chop_hit h = H[i];
        if (h.read == ~0u) continue;
        const uint32_t t = h.read - r0;
        T[s_off[t] + atomicAdd(&s_cnt[t], 1u)] = h;
    }
    __syncthreads();
    const uint32_t nh = s_off[nr];
    for (uint32_t t = 0; t < nr; ++t) {   // block-uniform
        const uint32_t o = s_off[t], c = s_off[t + 1] - o;
        for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) {
            const dmx_chop_hit x = T[o + i];
            uint32_t rank = 0;
            for (uint32_t j = 0; j < c; ++j) rank += hit_less(T[o + j], x) ? 1u : 0u;
            H[o + rank] = x;
        }
    }
    __syncthreads();
    chop_pair_write(A, b, r0, nr, nh, keep, s_rule, s_rstrand, H,
                    reinterpret_cast<dmx_chop_seg*>(T), s_off, s_sc, s_soff, s_base);
}

// Exclusive scan of the per-block hit / segment counts (one block; a few 100k entries).
__global__ __launch_bounds__(1024) void chop_blkscan_kernel(const uint32_t* blk, uint32_t nb,
                                                            uint32_t* off) {
    __shared__ uint32_t s_h[1024], s_s[1024];
    const uint32_t per = (nb + 1023u) / 1024u;
    const uint32_t lo = min(nb, threadIdx.x * per), hi = min(nb, lo + per);
    uint32_t h = 0, s = 0;
    for (uint32_t b = lo; b < hi; ++b) {
        h += blk[4 * b + 1];
        s += blk[4 * b + 3];
    }
    s_h[threadIdx.x] = h;
    s_s[threadIdx.x] = s;
    __syncthreads();
    for (uint32_t dlt = 1; dlt < 1024u; dlt <<= 1) {
        const uint32_t xh = threadIdx.x >= dlt ? s_h[threadIdx.x - dlt] : 0u;
        const uint32_t xs = threadIdx.x >= dlt ? s_s[threadIdx.x - dlt] : 0u;
        __syncthreads();
        s_h[threadIdx.x] += xh;
        s_s[threadIdx.x] += xs;
        __syncthreads();
    }
    h = threadIdx.x ? s_h[threadIdx.x - 1] : 0u;
    s = threadIdx.x ? s_s[threadIdx.x - 1] : 0u;
    for (uint32_t b = lo; b < hi; ++b) {
        off[2 * b] = h;
        off[2 * b + 1] = s;
        h += blk[4 * b + 1];
        s += blk[4 * b + 3];
    }
}

__global__ __launch_bounds__(256) void chop_order_kernel(ChopOrderArgs O) {
    for (uint32_t b = blockIdx.x; b < O.nb; b += gridDim.x) {
        const uint32_t hb = O.blk[4 * b], nh = O.blk[4 * b + 1];
        const uint32_t sb = O.blk[4 * b + 2], ns = O.blk[4 * b + 3];
        const uint32_t ho = O.off[2 * b], so = O.off[2 * b + 1];
        for (uint32_t i = threadIdx.x; i < nh; i += blockDim.x) O.hits[ho + i] = O.hstage[hb + i];
        for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) O.segs[so + i] = O.sstage[sb + i];
    }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
struct ChopState {
    ChopPanel host{};
    bool set = false;
    ChopPanel* d_panel = nullptr;
    dmx_chop_hit* d_hstage = nullptr;
    dmx_chop_hit* d_hits = nullptr;
    dmx_chop_seg* d_sstage = nullptr;
    dmx_chop_seg* d_segs = nullptr;
    size_t hit_cap = 0, seg_cap = 0;
    uint32_t* d_nhit = nullptr;
    uint32_t* d_nseg = nullptr;
    size_t read_cap = 0;
    uint32_t* d_blk = nullptr;
    uint32_t* d_blkoff = nullptr;
    size_t blk_cap = 0;
    unsigned long long* d_ctr = nullptr;
    uint32_t* d_ovf = nullptr;            // overflowing blocks (block, count), blk_cap entries
    uint64_t* d_ovf_base = nullptr;       // chop_big_kernel: hit-list bases, scratch, counters
    dmx_chop_hit* d_big = nullptr;
    size_t big_cap = 0;
    uint32_t* d_big_cnt = nullptr;
    size_t big_blocks_cap = 0;
    uint64_t n_hits = 0, n_segs = 0;
    size_t n_reads = 0;
    bool done = false;
    hipEvent_t ev[4] = {};
    float ms[2] = {0.f, 0.f};
    size_t n_big = 0;   // blocks redone by chop_big_kernel in the last exec
    int hb = -1;   // chop_kernel variant: last-row bit in the high (1) / low (0) half, or mixed
};

void chop_release(Ctx* c) {
    ChopState* s = c->chop;
    if (!s) return;
    void* bufs[] = {s->d_panel, s->d_hstage, s->d_hits,    s->d_sstage, s->d_segs,
                    s->d_nhit,  s->d_nseg,   s->d_blk,     s->d_blkoff, s->d_ctr,
                    s->d_ovf,   s->d_ovf_base, s->d_big,   s->d_big_cnt};
    for (void* b : bufs)
        if (b) hipFree(b);
    for (auto& e : s->ev)
        if (e) hipEventDestroy(e);
    delete s;
    c->chop = nullptr;
}

void chop_invalidate(Ctx* c) {
    if (c->chop) c->chop->done = false;   // results belong to the previous resident batch
}

}  // namespace dmx

using namespace dmx;

namespace {

#define CHOP_CK(call)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (call);                                                            \
        if (e_ != hipSuccess) {                                                            \
            c->err = std::string("dmx_chop: ") + #call + ": " + hipGetErrorString(e_);     \
            return DMX_E_HIP;                                                              \
        }                                                                                  \
    } while (0)

template <typename T>
hipError_t dev_realloc(T** p, size_t count) {
    if (*p) {
        hipFree(*p);
        *p = nullptr;
    }
    return hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T));
}

int iupac_bits(char ch) {
    switch (ch) {
        case 'A': return 1;
        case 'C': return 2;
        case 'G': return 4;
        case 'T': return 8;
        case 'R': return 5;
        case 'Y': return 10;
        case 'S': return 6;
        case 'W': return 9;
        case 'K': return 12;
        case 'M': return 3;
        case 'B': return 14;
        case 'D': return 13;
        case 'H': return 11;
        case 'V': return 7;
        case 'N': return 15;
        default: return 0;
    }
}

char iupac_comp(char ch) {
    const char* a = "ACGTRYSWKMBDHVN";
    const char* b = "TGCAYRSWMKVHDBN";
    const char* p = ch ? std::strchr(a, ch) : nullptr;
    return p ? b[p - a] : 'N';
}

void build_label(ChopLabel& L, const std::string& s, double cutoff) {
    std::memset(&L, 0, sizeof(L));
    const int m = (int)s.size();
    L.m = m;
    L.k = (int)(cutoff * m);
    for (int i = 0; i < m; ++i) {
        const int b = iupac_bits(s[i]);
        for (int c = 0; c < 4; ++c)
            if (b & (1 << c)) L.peq[c] |= 1ull << i;
    }
    const uint64_t all = m >= 64 ? ~0ull : ((1ull << m) - 1ull);
    for (int c = 4; c < 8; ++c) L.peq[c] = all;
}

ChopState* chop_state(Ctx* c) {
    if (!c->chop) {
        c->chop = new ChopState();
        for (auto& e : c->chop->ev) hipEventCreate(&e);
    }
    return c->chop;
}

}  // namespace

extern "C" int dmx_chop_set(dmx_ctx* c, const char* const* primers, const int* plens,
                            int n_primers, const int* rule_left, const int* rule_right,
                            const int* rule_strand, int n_rules, double cutoff,
                            int keep_primers) {
    if (!c) return DMX_E_INVALID;
    if (n_primers < 1 || n_primers > DMX_CHOP_MAX_PRIMERS || !primers || !plens) {
        c->err = "dmx_chop_set: 1.." + std::to_string(DMX_CHOP_MAX_PRIMERS) + " primers supported";
        return DMX_E_UNSUPPORTED;
    }
    if (n_rules < 0 || n_rules > DMX_CHOP_MAX_RULES ||
        (n_rules && (!rule_left || !rule_right || !rule_strand))) {
        c->err = "dmx_chop_set: 0.." + std::to_string(DMX_CHOP_MAX_RULES) + " rules supported";
        return DMX_E_UNSUPPORTED;
    }
    if (!(cutoff >= 0.0 && cutoff < 1.0)) {
        c->err = "dmx_chop_set: cutoff must be in [0, 1)";
        return DMX_E_INVALID;
    }
    ChopPanel P;
    std::memset(&P, 0, sizeof(P));
    std::memset(P.rule, -1, sizeof(P.rule));
    P.n_labels = 2 * n_primers;
    P.keep = keep_primers ? 1 : 0;
    P.n_rules = n_rules;
    for (int p = 0; p < n_primers; ++p) {
        const int L = plens[p];
        if (!primers[p] || L < 1 || L > 64) {
            c->err = "dmx_chop_set: primer " + std::to_string(p) + " must have 1..64 nt";
            return DMX_E_UNSUPPORTED;
        }
        std::string fw(primers[p], (size_t)L), rc((size_t)L, 'N');
        for (int i = 0; i < L; ++i) {
            char ch = fw[i];
            if (ch >= 'a' && ch <= 'z') ch = (char)(ch - 32);
            if (ch == 'U') ch = 'T';
            if (!iupac_bits(ch)) {
                c->err = "dmx_chop_set: primer " + std::to_string(p) + " has a non-IUPAC character";
                return DMX_E_INVALID;
            }
            fw[i] = ch;
        }
        for (int i = 0; i < L; ++i) rc[L - 1 - i] = iupac_comp(fw[i]);
        build_label(P.lab[2 * p], fw, cutoff);
        build_label(P.lab[2 * p + 1], rc, cutoff);
    }
    for (int r = 0; r < n_rules; ++r) {
        const int a = rule_left[r], b = rule_right[r], st = rule_strand[r];
        if (a < 0 || a >= P.n_labels || b < 0 || b >= P.n_labels || (st != 0 && st != 1)) {
            c->err = "dmx_chop_set: rule " + std::to_string(r) + " names an unknown label or strand";
            return DMX_E_INVALID;
        }
        if (P.rule[a * kChopMaxLabels + b] < 0) P.rule[a * kChopMaxLabels + b] = (int8_t)r;
        P.rstrand[r] = (int8_t)st;
    }
    CHOP_CK(hipSetDevice(c->device));
    ChopState* s = chop_state(c);
    if (!s->d_panel) CHOP_CK(hipMalloc((void**)&s->d_panel, sizeof(ChopPanel)));
    CHOP_CK(hipMemcpyAsync(s->d_panel, &P, sizeof(ChopPanel), hipMemcpyHostToDevice, c->stream));
    CHOP_CK(hipStreamSynchronize(c->stream));
    bool hi = true, lo = true;
    for (int l = 0; l < P.n_labels; ++l) {
        hi = hi && P.lab[l].m > 32;
        lo = lo && P.lab[l].m <= 32;
    }
    s->hb = hi ? 1 : (lo ? 0 : -1);
    s->host = P;
    s->set = true;
    s->done = false;
    return DMX_OK;
}

extern "C" int dmx_chop_exec(dmx_ctx* c, uint64_t* n_hits, uint64_t* n_segs) {
    if (!c) return DMX_E_INVALID;
    ChopState* s = c->chop;
    if (!s || !s->set) {
        c->err = "dmx_chop_exec before dmx_chop_set";
        return DMX_E_STATE;
    }
    const size_t n = c->n_reads;
    if (n && !c->d_seq) {
        c->err = "dmx_chop_exec before dmx_load";
        return DMX_E_STATE;
    }
    CHOP_CK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    s->done = false;
    if (!s->d_ctr) CHOP_CK(hipMalloc((void**)&s->d_ctr, 4 * sizeof(unsigned long long)));
    if (s->read_cap < n || !s->d_nhit) {
        CHOP_CK(dev_realloc(&s->d_nhit, n));
        CHOP_CK(dev_realloc(&s->d_nseg, n));
        s->read_cap = n;
    }
    if (s->hit_cap < 2 * n + 4096 || !s->d_hstage) {
        const size_t cap = 4 * n + 4096;
        CHOP_CK(dev_realloc(&s->d_hstage, cap));
        CHOP_CK(dev_realloc(&s->d_hits, cap));
        s->hit_cap = cap;
    }
    if (s->seg_cap < n + 4096 || !s->d_sstage) {
        const size_t cap = 2 * n + 4096;
        CHOP_CK(dev_realloc(&s->d_sstage, cap));
        CHOP_CK(dev_realloc(&s->d_segs, cap));
        s->seg_cap = cap;
    }
    unsigned long long ctr[4] = {0, 0, 0, 0};
    const uint32_t nb = (uint32_t)((n + kChopReads - 1) / kChopReads);
    if (s->blk_cap < nb || !s->d_blk) {
        CHOP_CK(dev_realloc(&s->d_blk, 4 * (size_t)nb));
        CHOP_CK(dev_realloc(&s->d_blkoff, 2 * (size_t)nb));
        CHOP_CK(dev_realloc(&s->d_ovf, 2 * (size_t)nb));
        s->blk_cap = nb;
    }
    size_t n_big = 0;
    CHOP_CK(bounds_reset(c, st));
    for (;;) {
        CHOP_CK(hipMemsetAsync(s->d_ctr, 0, 4 * sizeof(unsigned long long), st));
        ChopArgs A;
        A.pk.seq = c->d_seq;
        A.pk.nmask = c->d_nmask;
        A.pk.bd = make_bounds(c, kKerChop);
        A.offs = c->d_offs;
        A.lens = c->d_lens;
        A.n_reads = (uint32_t)n;
        A.panel = s->d_panel;
        A.hits = s->d_hstage;
        A.segs = s->d_sstage;
        A.hit_cap = s->hit_cap;
        A.seg_cap = s->seg_cap;
        A.nhit = s->d_nhit;
        A.nseg = s->d_nseg;
        A.blk = s->d_blk;
        A.ctr = s->d_ctr;
        A.ovf = s->d_ovf;
        A.ovf_cap = nb;
        CHOP_CK(hipEventRecord(s->ev[0], st));
        if (nb) {
            if (s->hb == 1) hipLaunchKernelGGL(chop_kernel<1>, dim3(nb), dim3(kChopBlock), 0, st, A);
            else if (s->hb == 0) hipLaunchKernelGGL(chop_kernel<0>, dim3(nb), dim3(kChopBlock), 0, st, A);
            else hipLaunchKernelGGL(chop_kernel<-1>, dim3(nb), dim3(kChopBlock), 0, st, A);
        }
        CHOP_CK(hipGetLastError());
        CHOP_CK(hipEventRecord(s->ev[1], st));
        CHOP_CK(hipMemcpyAsync(ctr, s->d_ctr, 4 * sizeof(unsigned long long),
                               hipMemcpyDeviceToHost, st));
        CHOP_CK(hipStreamSynchronize(st));
        n_big = 0;
        if (ctr[2] & 1ull) {   // blocks whose hits overflowed the LDS list: redo them alone
            const size_t no = (size_t)std::min<unsigned long long>(ctr[3], nb);
            std::vector<uint32_t> ovf(2 * no);
            CHOP_CK(hipMemcpy(ovf.data(), s->d_ovf, ovf.size() * 4, hipMemcpyDeviceToHost));
            std::vector<uint64_t> base(no + 1, 0);
            for (size_t i = 0; i < no; ++i) base[i + 1] = base[i] + ovf[2 * i + 1];
            if (s->big_cap < base[no] || !s->d_big) {
                CHOP_CK(dev_realloc(&s->d_big, 2 * base[no]));
                s->big_cap = base[no];
            }
            if (s->big_blocks_cap < no + 1 || !s->d_ovf_base) {
                CHOP_CK(dev_realloc(&s->d_ovf_base, no + 1));
                CHOP_CK(dev_realloc(&s->d_big_cnt, no + 1));
                s->big_blocks_cap = no + 1;
            }
            CHOP_CK(hipMemcpyAsync(s->d_ovf_base, base.data(), (no + 1) * 8,
                                   hipMemcpyHostToDevice, st));
            CHOP_CK(hipMemsetAsync(s->d_big_cnt, 0, (no + 1) * 4, st));
            set_kid(A.pk.bd, kKerChopBig);
            hipLaunchKernelGGL(chop_big_kernel, dim3((uint32_t)no), dim3(kChopBlock), 0, st, A,
                               (const uint64_t*)s->d_ovf_base, s->d_big, s->d_big + s->big_cap,
                               s->d_big_cnt);
            CHOP_CK(hipGetLastError());
            CHOP_CK(hipEventRecord(s->ev[1], st));
            CHOP_CK(hipMemcpyAsync(ctr, s->d_ctr, 4 * sizeof(unsigned long long),
                                   hipMemcpyDeviceToHost, st));
            CHOP_CK(hipStreamSynchronize(st));
            n_big = no;
        }
        if (ctr[0] >= (1ull << 32) || ctr[1] >= (1ull << 32)) {
            c->err = "dmx_chop_exec: more than 2^32 hits in one batch";
            return DMX_E_UNSUPPORTED;
        }
        if (ctr[0] > s->hit_cap || ctr[1] > s->seg_cap) {
            if (ctr[0] > s->hit_cap) {
                const size_t cap = ctr[0] + ctr[0] / 4 + 4096;
                CHOP_CK(dev_realloc(&s->d_hstage, cap));
                CHOP_CK(dev_realloc(&s->d_hits, cap));
                s->hit_cap = cap;
            }
            if (ctr[1] > s->seg_cap) {
                const size_t cap = ctr[1] + ctr[1] / 4 + 4096;
                CHOP_CK(dev_realloc(&s->d_sstage, cap));
                CHOP_CK(dev_realloc(&s->d_segs, cap));
                s->seg_cap = cap;
            }
            continue;
        }
        break;
    }
    s->n_big = n_big;
    CHOP_CK(hipEventRecord(s->ev[2], st));
    if (nb) {
        hipLaunchKernelGGL(chop_blkscan_kernel, dim3(1), dim3(1024), 0, st,
                           (const uint32_t*)s->d_blk, nb, s->d_blkoff);
        ChopOrderArgs O{s->d_blk, s->d_blkoff, nb, s->d_hstage, s->d_hits, s->d_sstage,
                        s->d_segs};
        hipLaunchKernelGGL(chop_order_kernel, dim3(std::min<uint32_t>(nb, 8192u)), dim3(256), 0,
                           st, O);
        CHOP_CK(hipGetLastError());
    }
    CHOP_CK(hipEventRecord(s->ev[3], st));
    CHOP_CK(hipEventSynchronize(s->ev[3]));
    if (const int brc = bounds_check(c, "dmx_chop_exec")) return brc;
    hipEventElapsedTime(&s->ms[0], s->ev[0], s->ev[1]);
    hipEventElapsedTime(&s->ms[1], s->ev[2], s->ev[3]);
    s->n_hits = ctr[0];
    s->n_segs = ctr[1];
    s->n_reads = n;
    s->done = true;
    if (n_hits) *n_hits = ctr[0];
    if (n_segs) *n_segs = ctr[1];
    return DMX_OK;
}

extern "C" int dmx_chop_fetch(dmx_ctx* c, uint32_t* n_seg, uint32_t* n_hit, dmx_chop_seg* segs,
                              size_t seg_cap, dmx_chop_hit* hits, size_t hit_cap) {
    if (!c) return DMX_E_INVALID;
    ChopState* s = c->chop;
    if (!s || !s->done) {
        c->err = "dmx_chop_fetch before dmx_chop_exec";
        return DMX_E_STATE;
    }
    CHOP_CK(hipSetDevice(c->device));
    hipStream_t st = c->stream;
    const size_t n = s->n_reads;
    if (n_seg && n)
        CHOP_CK(hipMemcpyAsync(n_seg, s->d_nseg, n * 4, hipMemcpyDeviceToHost, st));
    if (n_hit && n)
        CHOP_CK(hipMemcpyAsync(n_hit, s->d_nhit, n * 4, hipMemcpyDeviceToHost, st));
    const size_t ns = std::min<uint64_t>(s->n_segs, seg_cap);
    const size_t nh = std::min<uint64_t>(s->n_hits, hit_cap);
    if (segs && ns)
        CHOP_CK(hipMemcpyAsync(segs, s->d_segs, ns * sizeof(dmx_chop_seg), hipMemcpyDeviceToHost,
                               st));
    if (hits && nh)
        CHOP_CK(hipMemcpyAsync(hits, s->d_hits, nh * sizeof(dmx_chop_hit), hipMemcpyDeviceToHost,
                               st));
    CHOP_CK(hipStreamSynchronize(st));
    return DMX_OK;
}

extern "C" int dmx_chop_stats(dmx_ctx* c, float* ms, int n_ms) {
    if (!c || (n_ms > 0 && !ms)) return DMX_E_INVALID;
    ChopState* s = c->chop;
    if (!s || !s->done) {
        c->err = "dmx_chop_stats before dmx_chop_exec";
        return DMX_E_STATE;
    }
    for (int i = 0; i < n_ms && i < 2; ++i) ms[i] = s->ms[i];
    return (int)s->n_big;
}
