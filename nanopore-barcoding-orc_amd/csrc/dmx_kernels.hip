// dmx_kernels.hip — gfx950 kernels of the two-round demultiplexer and their launch sequence.
//
// Replaces the per-read hot loop of cutadapt 4.9 as driven by scripts/02_cutadapt_loop.sh:64-72
// (round 1: 5' SP5 adapters, --rc) and :91-103 (round 2: 3' SP27rc adapters, --rc, on every SP5
// bin), and scripts/04_cleaning_primers.sh:371-388 (linked primers).  Semantics restated in
// oracle/cutadapt_oracle.c; design and exactness argument in DESIGN.md §3.
//
// Per round: scan -> resolve -> select -> finalize, all on one HIP stream, no host round trip.
#include <algorithm>
#include <cstring>
#include <memory>
#include <type_traits>
#include <utility>
#include <vector>

#include "dmx_device.h"
#include "dmx_internal.h"

namespace dmx {

// ---------------------------------------------------------------------------------------------
// shared helpers
// ---------------------------------------------------------------------------------------------
struct RoundArgs {
    Packed pk;                   // the resident packed batch (+ bounds in DMX_DEBUG_BOUNDS builds)
    const uint64_t* offs;
    const uint32_t* lens;
    const DevPanel* panel;
    const ItemView* items;       // nullptr: item i = read i, whole read (round 0)
    const uint32_t* n_items_dev; // device count of items (when items != nullptr)
    uint32_t n_items;            // host count / upper bound
    int32_t T;                   // tasks per item
    int32_t per_task_slot;       // linked round 0: one winner slot per (read, pair)
    int32_t slot_div;            // > 0: one slot per (item, orientation), sub / slot_div = o
    Cluster* cl;
    Outcome* outc;
    uint32_t* cl_count;
    uint32_t cl_cap;
    uint32_t* flags;             // bit0 cluster overflow, bit1 window violation
    unsigned long long* winner;  // per slot, ~0 = none
    int32_t* origin;             // per slot
    int32_t* lb;                 // per slot: lower bound of the best accepted score (0 = none)
    Window* win;
    uint32_t* win_count;         // [kShards]: shard s at win + s * win_scap
    uint32_t win_cap;
    uint32_t win_scap;
    Window* win2;                // verified windows (when the panel has a shared prefix)
    uint32_t* win2_count;        // [kShards], per-shard capacity win_scap
    uint32_t* diag;              // [0] resolved clusters, [1] tracebacks
    int32_t band;                // 1: emit candidate cells (band kernels), 0: clusters (ring)
    Cand* cand[2];               // candidate lists: [0] cost <= 3 (band 7), [1] cost 4..7 (15)
    Outcome* cand_out[2];
    uint32_t* cand_count;        // [2][kShards] x kShardStride: list l, shard s at cand[l] + s * cand_scap
    uint32_t cand_cap;
    uint32_t cand_scap;          // per-shard capacity
    int32_t screen;              // 1: the window scan runs the index screen's surviving pairs
    Window* tasks;               // index screen survivors: window pieces of one adapter each
    uint32_t* task_count;        // [kShards]: shard s at tasks + s * task_scap
    uint32_t task_cap;
    uint32_t task_scap;
    const DevPieces* pieces;     // piece screen tables
    FTask* ftask;                // piece screen -> filter tasks
    uint32_t* ftask_count;       // [kShards]: shard s at ftask + s * ftask_scap
    uint32_t ftask_scap;
    uint32_t* stage;             // window code slots (wstage_kernel), stage_cap of them
    uint32_t stage_cap;
    // flat piece scan: cell bitmaps [2 round + strand], kCellGuardWords words before index 0
    uint32_t n_words;
    uint32_t nsb;                // 4096-nt superblocks of the packed batch
    int32_t round;
    uint32_t* cells[4];
};

// DESIGN.md §3.10.  The filter, the prefix verification and the index screen are necessary
// conditions that only compare lower bounds of edit costs with thresholds.  Reading a read's
// non-ACGT bases as the 2-bit code packed for them (A) instead of "matches nothing" can only turn
// a mismatch into a match, so every cost they compute can only go down: they stay necessary
// conditions, and the exact stages (window scan, band DP) still see the no-match mask.  So by
// default those three never use the mask (DMX_MASK_SKIP=0: the round-4 behaviour, for A/B).
#ifndef DMX_MASK_SKIP
#define DMX_MASK_SKIP 1
#endif
constexpr bool kNecessaryMask = !DMX_MASK_SKIP;

struct TaskView {
    uint32_t read, n, strand, start, len;
    uint64_t off;
    int o, a;
    bool clean = false;   // the exact stages may skip the no-match mask (Window kWinClean)
    uint32_t tag = 0;     // window code slot + 1 (0: gather from the packed batch)
    uint32_t sbl = 0;     // the slot's base column + kViewReachPre (bits 0..23), filled columns
};

// A pointer moved into SGPRs (readfirstlane) in the global address space: a per-lane select
// between such pointers stays a select, where the compiler turns a per-lane index into a
// RoundArgs pointer array into a dependent load of the kernel argument.
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* sgpr_ptr(T* p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return reinterpret_cast<__attribute__((address_space(1))) T*>(lo | (hi << 32));
}

// cd into p[i] through a global-address-space pointer (two 16-B and one 8-B store).
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void store_cand(__attribute__((address_space(1))) Cand* p, uint32_t i,
                                           const Cand& cd) {
    static_assert(sizeof(Cand) == 40, "Cand layout");
    u32x4_t a, b;
    u32x2_t c;
    __builtin_memcpy(&a, reinterpret_cast<const char*>(&cd), 16);
    __builtin_memcpy(&b, reinterpret_cast<const char*>(&cd) + 16, 16);
    __builtin_memcpy(&c, reinterpret_cast<const char*>(&cd) + 32, 8);
    auto* d = reinterpret_cast<__attribute__((address_space(1))) char*>(p + i);
    *reinterpret_cast<__attribute__((address_space(1))) u32x4_t*>(d) = a;
    *reinterpret_cast<__attribute__((address_space(1))) u32x4_t*>(d + 16) = b;
    *reinterpret_cast<__attribute__((address_space(1))) u32x2_t*>(d + 32) = c;
}

// A record's `off` field -> the view's first nt and its window code slot (kStageWords).
__device__ __forceinline__ void view_off(const Packed& pk, uint64_t off, TaskView& tv) {
    tv.off = off & kOffMask;
    tv.tag = DMX_STAGE_SLOTS ? (uint32_t)(off >> kOffBits) : 0u;
    tv.sbl = 0;
    if (DMX_STAGE_SLOTS && tv.tag) {
        const uint2 h = *reinterpret_cast<const uint2*>(pk.stage + (size_t)(tv.tag - 1) *
                                                                      kStageWords + 12);
        tv.sbl = (h.x + kViewReachPre) | (h.y << 24);
    }
}

// 16 view positions from p out of the view's window code slot, when it holds them: the same
// codes and no-match bits as the gather (wstage_kernel filled the slot with fetch16s).
__device__ __forceinline__ bool staged16(const Packed& pk, const TaskView& tv, int p, bool mask,
                                         uint32_t& codes, uint32_t& nbits) {
    if (!DMX_STAGE_SLOTS || !tv.tag) return false;
    const int rel = p + kViewReachPre - (int)(tv.sbl & 0xFFFFFFu);
    if (rel < 0 || rel + 16 > (int)(tv.sbl >> 24)) return false;
    const uint32_t* sl = pk.stage + (size_t)(tv.tag - 1) * kStageWords;
    uint64_t c;
    __builtin_memcpy(&c, sl + (rel >> 4), 8);
    codes = (uint32_t)(c >> (2 * (rel & 15)));
    if (mask) {
        uint64_t m;
        __builtin_memcpy(&m, sl + 8 + (rel >> 5), 8);
        nbits = (uint32_t)(m >> (rel & 31)) & 0xFFFFu;
    } else {
        nbits = 0u;
    }
    return true;
}

// fetch16 of a view that may have a window code slot
__device__ __forceinline__ void fetch16t(const Packed& pk, const TaskView& tv, uint32_t p,
                                         uint32_t& codes, uint32_t& nbits, bool load_mask = true) {
    if (staged16(pk, tv, (int)p, load_mask, codes, nbits)) return;
    fetch16(pk, tv.off, tv.n, tv.strand, tv.start, p, codes, nbits, load_mask);
}

// An empty view at the first valid offset (DMX_DEBUG_BOUNDS builds: an item or read index out of
// range; the violation is recorded and the task scans nothing).
__device__ __forceinline__ bool empty_view(TaskView& tv) {
    tv.read = 0;
    tv.n = tv.start = tv.len = tv.strand = 0;
    tv.off = kMinOffset;
    tv.o = tv.a = 0;
    return false;
}

__device__ __forceinline__ bool task_view(const RoundArgs& R, uint32_t item, int sub, int A,
                                          TaskView& tv) {
    if (R.items) {
        if (!DMX_BOUND(R.pk.bd, items, item, kBufItem)) return empty_view(tv);
        const ItemView v = R.items[item];
        tv.read = v.read;
        tv.start = v.start;
        tv.len = v.len;
        tv.strand = v.strand;
        if (v.only_adapter >= 0) {   // linked: exactly one task per item, no RC
            tv.o = 0;
            tv.a = v.only_adapter;
        } else {
            tv.o = sub / A;
            tv.a = sub % A;
        }
    } else {
        tv.read = item;
        tv.start = 0;
        tv.strand = 0;
        tv.len = R.lens[item];
        tv.o = sub / A;
        tv.a = sub % A;
        if (R.per_task_slot) {
            tv.o = 0;
            tv.a = sub;
        }
    }
    if (!DMX_BOUND(R.pk.bd, reads, tv.read, kBufRead)) return empty_view(tv);
    tv.n = R.lens[tv.read];
    tv.off = R.offs[tv.read];
    if (tv.o) {   // reverse complement of the view (strand s, start st, len l) of a read of n nt
        tv.start = tv.n - tv.start - tv.len;
        tv.strand ^= 1u;
    }
    return true;
}

__device__ __forceinline__ uint32_t slot_of(const RoundArgs& R, uint32_t item, int sub) {
    if (R.per_task_slot) return item * (uint32_t)R.T + (uint32_t)sub;
    return R.slot_div ? 2u * item + (uint32_t)(sub >= R.slot_div) : item;
}

// Row stride of the code-major match tables in LDS: lanes of one window read one code row at
// consecutive adapters; windows sharing a wave read other codes' rows, shifted by 24 banks
// (a power-of-two stride put every code's copy of adapter a in the same bank).
constexpr int kPeqStride = kMaxAdapters + 24;
constexpr int kIpeqStride = 9;   // index screen: words per adapter (4 codes + bank padding)

// An adapter's length, k, end and kk (DevAdapter's four bytes m, k, where, kk): what the scans
// need per task, held in LDS by the kernels (a per-lane read of DevAdapter is a global load the
// task's first gather waits behind).
struct AdLite {
    int m, k, kk;
    bool front;
};
__device__ __forceinline__ uint32_t ad_word(const DevAdapter& ad) {
    return (uint32_t)ad.m | ((uint32_t)ad.k << 8) | ((uint32_t)ad.where << 16) |
           ((uint32_t)(uint8_t)ad.kk << 24);
}
__device__ __forceinline__ AdLite ad_lite(uint32_t w) {
    return AdLite{(int)(w & 255u), (int)((w >> 8) & 255u), (int)(int8_t)(w >> 24),
                  ((w >> 16) & 255u) == kFront};
}
__device__ __forceinline__ AdLite ad_lite(const DevAdapter& ad) { return ad_lite(ad_word(ad)); }

__device__ __forceinline__ void load_panel_lds(const DevPanel* P, uint64_t* s_peq, int8_t* s_acc,
                                               int8_t* s_pacc, uint32_t* s_amk) {
    const int A = P->n_adapters;
    for (int a = threadIdx.x; a < A; a += blockDim.x) s_amk[a] = ad_word(P->ad[a]);
    for (int x = threadIdx.x; x < 8 * A; x += blockDim.x) {
        const int c = x / A, a = x % A;   // code-major, power-of-two row stride (no multiply)
        s_peq[c * kPeqStride + a] = P->ad[a].peq[c];   // lanes of one read: consecutive words
    }
    for (int x = threadIdx.x; x < 72 * A; x += blockDim.x) {
        s_acc[x] = P->ad[x / 72].acc[x % 72];
        s_pacc[x] = P->ad[x / 72].pacc[x % 72];
    }
}

// Can last-row cell (m, j) with cost d be accepted at all? (aligned adapter length <= j + d)
__device__ __forceinline__ bool row_candidate(const int8_t* pacc, int m, uint32_t j, int d) {
    const uint32_t L = min((uint32_t)m, j + (uint32_t)d);
    return d <= (int)pacc[L];
}

// ---------------------------------------------------------------------------------------------
// scan: per (item, orientation, adapter) Myers over a column range; emits candidate clusters.
// Besides the clusters each task publishes a lower bound of the slot's final best score (from
// cells that are certainly accepted with the whole adapter aligned: score >= m - 3 * cost), so
// the resolve stage can drop clusters whose score upper bound is below it.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ Cluster make_cluster(uint32_t item, int sub, uint32_t j1, uint32_t j2,
                                                int lastcol, int ub) {
    Cluster c;
    c.item = item;
    c.sub = (uint16_t)sub;
    c.lastcol = (uint8_t)lastcol;
    c.ub = (int8_t)max(-128, min(127, ub));
    c.j1 = j1;
    c.j2 = j2;
    return c;
}

// Lower-bound key: the slot has an accepted cell of orientation o, cost `cost` and score >= lb,
// so the slot's winning key is <= (lb, o, cost) in make_key's order (score desc, forward before
// RC, cost asc).  Max over tasks: higher score, then forward, then lower cost.  A cell of equal
// score bound loses to it only if it is RC against a forward bound, or of the same orientation
// with a higher cost — a forward cell beats an RC cell of equal score whatever the costs
// (ReverseComplementer takes the RC read only on a strictly greater score).
__device__ __forceinline__ int lb_key(int lb, int o, int cost) {
    return lb > 0 ? (lb << 9) | ((1 - o) << 8) | (255 - cost) : 0;
}
__device__ __forceinline__ int lb_score(int lbk) { return lbk ? (lbk >> 9) : -1000; }
// can a cell of orientation o and cost `cost` whose score is at most ub beat the bound?
__device__ __forceinline__ bool beats_lb(int lbk, int ub, int o, int cost) {
    if (!lbk) return true;
    const int lbs = lbk >> 9, lbo = 1 - ((lbk >> 8) & 1), lbc = 255 - (lbk & 255);
    return ub > lbs || (ub == lbs && (o < lbo || (o == lbo && cost <= lbc)));
}

// One task's Myers scan over view columns (js, jhi]; last-row candidates are reported for
// columns in [jlo, jhi] only.  js == 0 with `real` uses cutadapt's column-0 initialisation;
// otherwise the restricted start D'(i, js) = i, exact for every cell of cost <= k at column
// >= js + m + k + 1.  Emits clusters; returns this task's score lower bound.
__device__ __forceinline__ int scan_task(const RoundArgs& R, const Stage<Cluster>& st,
                                         const TaskView& tv, uint32_t item, int sub,
                                         const uint64_t* peq, int A, AdLite ad,
                                         const int8_t* acc, const int8_t* pacc, uint32_t js,
                                         bool real, uint32_t jlo, uint32_t jhi, bool lastcol) {
    const int m = ad.m;
    const int kk = ad.kk;
    const bool front = ad.front;
    const uint32_t hbit = (uint32_t)(m - 1);
    const uint32_t gap = (uint32_t)(m + ad.k + 1);

    uint64_t pv = (front && real) ? 0ull : ~0ull, mv = 0ull;
    int d = (front && real) ? 0 : m;
    bool have = false;
    uint32_t cj1 = 0, cj2 = 0;
    int cub = -128, lbk = 0;   // lbk = lb_key of the best certainly-accepted cell, 0 = none

#define DMX_SCAN_STEP(q)                                                                  \
    {                                                                                     \
        const uint32_t code = ((codes >> (2 * (q))) & 3u) | (((nb >> (q)) & 1u) << 2);    \
        myers_step(peq[code * kPeqStride], pv, mv, d, hbit);                              \
        if (d <= kk) {                                                                    \
            const uint32_t j = p0 + (q) + 1;                                              \
            const int lr = min(m, (int)j + d);                                            \
            if (j >= jlo && d <= (int)pacc[lr]) {                                         \
                const int ubc = lr - 2 * d;                                               \
                {   /* certainly accepted: aligned length >= L0 and acc is monotone */       \
                    const int L0 = min(m, (int)j - d);                                    \
                    if (L0 >= 0 && d <= (int)acc[L0]) lbk = max(lbk, lb_key(L0 - 3 * d, tv.o, d)); \
                }                                                                         \
                if (have && j - cj2 <= gap) {                                             \
                    cj2 = j;                                                              \
                    cub = max(cub, ubc);                                                  \
                } else {                                                                  \
                    if (have) st.push(make_cluster(item, sub, cj1, cj2, 0, cub));         \
                    have = true;                                                          \
                    cj1 = cj2 = j;                                                        \
                    cub = ubc;                                                            \
                }                                                                         \
            }                                                                             \
        }                                                                                 \
    }

    uint32_t p0 = js;
    uint32_t ncodes, nnb, ncodes2 = 0, nnb2 = 0;   // the next two chunks, in flight
    fetch16t(R.pk, tv, p0, ncodes, nnb);
    if (p0 + 16 < jhi)
        fetch16t(R.pk, tv, p0 + 16, ncodes2, nnb2);
    for (; p0 + 16 <= jhi; p0 += 16) {
        const uint32_t codes = ncodes, nb = nnb;
        ncodes = ncodes2;
        nnb = nnb2;
        if (p0 + 32 < jhi)
            fetch16t(R.pk, tv, p0 + 32, ncodes2, nnb2);
#pragma unroll
        for (int q = 0; q < 16; ++q) DMX_SCAN_STEP(q)
    }
    if (p0 < jhi) {
        const uint32_t codes = ncodes, nb = nnb;
        const int cnt = (int)(jhi - p0);
        for (int q = 0; q < cnt; ++q) DMX_SCAN_STEP(q)
    }
#undef DMX_SCAN_STEP

    // 3' adapters: cutadapt also scans the last column (cells (i, n), i <= m: adapter prefix
    // aligned at the read end).  Flag it if any such cell would be accepted.  Cell (m, n) is a
    // last-row cell the column loop reports, except in an empty view (no column): there only the
    // last-column scan sees it (cost m, score -2m: accepted at rates >= 1, e.g. -e 3 and m = 3).
    const uint32_t len = tv.len;
    if (lastcol && !front) {   // an empty view too: cells (i, 0) cost i (rate >= 1 accepts)
        int dd = 0;
        int ubl = -128;
        const int ilast = len == 0 ? m : m - 1;
        for (int i = 1; i <= ilast; ++i) {
            dd += (int)((pv >> (i - 1)) & 1ull) - (int)((mv >> (i - 1)) & 1ull);
            if (dd <= (int)acc[i]) {              // accepted for sure (aligned length is i)
                ubl = max(ubl, i - 2 * dd);
                lbk = max(lbk, lb_key(i - 3 * dd, tv.o, dd));
            }
        }
        if (ubl > -128) {
            if (have && len - cj2 <= gap) {
                st.push(make_cluster(item, sub, cj1, len, 1, max(cub, ubl)));
            } else {
                if (have) st.push(make_cluster(item, sub, cj1, cj2, 0, cub));
                st.push(make_cluster(item, sub, len, len, 1, ubl));
            }
            have = false;
        }
    }
    if (have) st.push(make_cluster(item, sub, cj1, cj2, 0, cub));
    return lbk;
}

// Band mode: the same scan, but candidate END CELLS are emitted (after pruning with this
// task's own score lower bound), each carrying its exact cost; no clusters, no resolve pass.
struct CandSink {
    Stage<Cand, kCandStageCap> st[2];
};

// Per-wave staging: each wave appends to its own LDS slice and flushes it on its own (one
// global atomic per flush, no block barrier), so waves of a block never wait for each other.
template <class Rec, int CAP>
struct WaveStage {
    Rec* buf;              // LDS [CAP], this wave's slice
    uint32_t* cnt;         // LDS, this wave's counter
    Rec* g;
    uint32_t* gcount;
    uint32_t gcap;
    uint32_t* flags;
    uint32_t ovf;

    __device__ __forceinline__ void push(const Rec& r) const {
        const uint32_t i = atomicAdd(cnt, 1u);
        if (i < (uint32_t)CAP) {
            buf[i] = r;
            return;
        }
        const uint32_t gi = atomicAdd(gcount, 1u);   // slice full: direct (rare)
        if (gi < gcap) g[gi] = r;
        else atomicOr(flags, ovf);
    }
    __device__ __forceinline__ uint32_t count() const { return *cnt; }
    // Every lane of the wave calls this at a wave-uniform point.  LDS operations of one wave
    // complete in issue order, so the slice written by the pushes above is visible here.
    __device__ __forceinline__ void flush() const {
        const uint32_t n = min(*cnt, (uint32_t)CAP);
        if (n == 0) return;
        const uint32_t lane = threadIdx.x & 63u;
        uint32_t b = 0;
        if (lane == 0) b = atomicAdd(gcount, n);
        b = __builtin_amdgcn_readfirstlane(b);
        for (uint32_t i = lane; i < n; i += 64) {
            if (b + i < gcap) g[b + i] = buf[i];
            else atomicOr(flags, ovf);
        }
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) *cnt = 0;
        __builtin_amdgcn_wave_barrier();
    }
};

// The shard a wave appends to (waves of a block spread over consecutive shards).
__device__ __forceinline__ uint32_t wave_shard() {
    return (blockIdx.x * (kScanBlock / 64) + (threadIdx.x >> 6)) & (uint32_t)(kShards - 1);
}

// Reader side of a sharded list: the block's prefix over the shards' (clamped) counts in LDS,
// and the dense index -> record index map.  Every thread of the block calls load().
struct ShardMap {
    uint32_t* pre;   // LDS [kShards + 1]
    uint32_t scap;
    __device__ __forceinline__ void load(const uint32_t* counts, uint32_t shard_cap) {
        scap = shard_cap;
        if (threadIdx.x == 0) {
            uint32_t t = 0;
            for (int k = 0; k < kShards; ++k) {
                pre[k] = t;
                t += min(counts[k * kShardStride], shard_cap);
            }
            pre[kShards] = t;
        }
        __syncthreads();
    }
    __device__ __forceinline__ uint32_t total() const { return pre[kShards]; }
    __device__ __forceinline__ uint32_t phys(uint32_t t) const {
        uint32_t s = 0;
#pragma unroll
        for (uint32_t h = kShards / 2; h > 0; h >>= 1)
            if (t >= pre[s + h]) s += h;
        return s * scap + (t - pre[s]);
    }
};

#ifndef DMX_WSCAN_LANE_ROWS   // window-scan per-lane match-vector rows (A/B, off: see wscan_task)
#define DMX_WSCAN_LANE_ROWS 0
#endif
#ifndef DMX_WAVE_CAND_CAP   // rare: cells of earlier 64-column segments (16 with the window
#define DMX_WAVE_CAND_CAP (DMX_WSCAN_LANE_ROWS ? 16 : 32)   // scan's per-lane rows, to make room
#endif   // in LDS; 32 vs 16: 46.51 vs 46.85 ms, profiles/r5_ab_wscan_waves_candcap.txt)
#ifndef DMX_WAVE_CAND_FLUSH
#define DMX_WAVE_CAND_FLUSH (DMX_WAVE_CAND_CAP / 2)
#endif
constexpr int kWaveCandCap = DMX_WAVE_CAND_CAP;
constexpr int kWaveWinCap = 64;   // per-wave window / task staging (filter, verify, screen)

struct WaveCandSink {
    WaveStage<Cand, kWaveCandCap> st[2];
};

__device__ __forceinline__ Cand make_cand(const TaskView& tv, uint32_t item, int sub, int iend,
                                          int cost, uint32_t j) {
    Cand c;
    c.item = item;
    c.sub = (uint16_t)sub;
    c.iend = (uint8_t)iend;
    c.cost = (uint8_t)cost;
    c.j = j;
    c.n = tv.n;
    c.start = tv.start;
    c.len = tv.len;
    c.strand = (uint8_t)tv.strand;
    c.o = (uint8_t)tv.o;
    c.a = (uint8_t)tv.a;
    c.clean = tv.clean ? 1 : 0;
    c.off = tv.off | ((uint64_t)tv.tag << kOffBits);
    return c;
}

// can a cell of orientation o and cost `cost` whose aligned adapter length is <= lr beat the
// lower-bound key?
__device__ __forceinline__ bool viable_lb(int lbk, int lr, int o, int cost) {
    return beats_lb(lbk, lr - 2 * cost, o, cost);
}

// 16 view positions from view position p (may be negative or past the view: pads and guard
// words).  Positions before -kViewReachPre are read at -kViewReachPre, so a gather never starts
// more than kViewReachPre + 15 nt before a view, or ends more than kViewReachPre + 32 nt past
// it on the reverse strand; the host checks per panel that this stays inside the device guard
// for every offset dmx_load / dmx_run accept (dmx_panel_reach).  Callers take columns before the
// view as free-start warm-up only, where any codes are safe (the index screen of a 3' panel at
// -e 0.3 starts up to m + k columns before a short view).  The positions are signed: the seed-46
// fault of round 4 was an unsigned wrap of such a position below the buffer.
// MASK = false: the codes only, no-match bits 0 (one 8-byte gather instead of two).
template <bool MASK = true>
__device__ __forceinline__ void fetch16s(const Packed& pk, const TaskView& tv, int p,
                                         uint32_t& codes, uint32_t& nbits) {
    p = max(p, -kViewReachPre);
    if (staged16(pk, tv, p, MASK && !tv.clean, codes, nbits)) return;
    if (tv.strand == 0) {
        const int64_t g = (int64_t)tv.off + (int64_t)tv.start + p;
        codes = code32(pk, g);
        nbits = (MASK && !tv.clean) ? mask32(pk, g) & 0xFFFFu : 0u;
    } else {
        const int64_t b = (int64_t)tv.off + (int64_t)tv.n - 1 - (int64_t)tv.start - p - 15;
        codes = ~rev_pairs(code32(pk, b));
        nbits = (MASK && !tv.clean) ? __brev(mask32(pk, b)) >> 16 : 0u;
    }
}

// fetch16s in two halves (round 6).  fetch16s branches on the lane's strand and finishes the
// gathered words inside each branch (shift, pair reversal, complement), so the compiler waits
// for the gather right where it is issued (`s_waitcnt vmcnt(0)` in both branches): the loops'
// "next chunks in flight" were never in flight, and every chunk cost a full memory round trip.
// chunk16_load only issues the 8-byte gathers (no branch on the strand, the words unused), and
// chunk16_codes finishes them when the chunk is consumed, one chunk later.  Same positions,
// same clamp, same bits as fetch16s.
struct Chunk16 {
    uint64_t c = 0, m = 0;   // words q, q + 1 of the codes and of the no-match mask
};
// Lowest batch nt of view positions [p, p + 16) (fetch16s' g / b).
__device__ __forceinline__ int64_t chunk16_pos(const TaskView& tv, int p) {
    p = max(p, -kViewReachPre);
    const int64_t f = (int64_t)tv.off + (int64_t)tv.start + p;
    const int64_t b = (int64_t)tv.off + (int64_t)tv.n - 1 - (int64_t)tv.start - p - 15;
    return tv.strand ? b : f;
}
__device__ __forceinline__ uint64_t load8(const uint32_t* __restrict__ w, int64_t q,
                                          const Bounds& bd, uint32_t buf) {
#ifdef DMX_DEBUG_BOUNDS
    if (!bchk(bd, q, bd.lo, bd.hi - 1, buf)) return 0ull;
#else
    (void)bd, (void)buf;
#endif
    uint64_t v;
    __builtin_memcpy(&v, w + q, 8);
    return v;
}
template <bool MASK = true>
__device__ __forceinline__ Chunk16 chunk16_load(const Packed& pk, const TaskView& tv, int p) {
    const int64_t g = chunk16_pos(tv, p);
    Chunk16 r;
    r.c = load8(pk.seq, (2 * g) >> 5, pk.bd, kBufSeq);
    if (MASK && !tv.clean) r.m = load8(pk.nmask, g >> 5, pk.bd, kBufMask);
    return r;
}
template <bool MASK = true>
__device__ __forceinline__ void chunk16_codes(const TaskView& tv, int p, const Chunk16& r,
                                              uint32_t& codes, uint32_t& nbits) {
    // only the low 5 bits of the position matter here: 32-bit arithmetic
    const int pc = max(p, -kViewReachPre);
    const uint32_t f = (uint32_t)tv.off + tv.start + (uint32_t)pc;
    const uint32_t b = (uint32_t)tv.off + tv.n - 1u - tv.start - (uint32_t)pc - 15u;
    const uint32_t g = tv.strand ? b : f;
    const uint32_t c = (uint32_t)(r.c >> ((2u * g) & 31u));
    codes = tv.strand ? ~rev_pairs(c) : c;
    if (MASK) {
        const uint32_t m = (uint32_t)(r.m >> (g & 31u));
        nbits = tv.strand ? __brev(m) >> 16 : m & 0xFFFFu;
    } else {
        nbits = 0u;
    }
}

// The no-match bits of view positions [p, p + 32) (the filter's clean-flag history).
__device__ __forceinline__ uint32_t mask32s(const Packed& pk, const TaskView& tv, int p) {
    if (tv.strand == 0) return mask32(pk, (int64_t)tv.off + (int64_t)tv.start + p);
    return __brev(mask32(pk, (int64_t)tv.off + (int64_t)tv.n - 1 - (int64_t)tv.start - p - 31));
}

template <class Sink>
__device__ __forceinline__ void flush_cands(const Sink& sink, const TaskView& tv, uint32_t item,
                                         int sub, int m, int lbk, uint32_t seg, uint64_t cm,
                                         uint64_t c0, uint64_t c1, uint64_t c2) {
    while (cm) {
        const int bit = __ffsll((unsigned long long)cm) - 1;
        cm &= cm - 1;
        const int cost = (int)((c0 >> bit) & 1ull) | ((int)((c1 >> bit) & 1ull) << 1) |
                         ((int)((c2 >> bit) & 1ull) << 2);
        const uint32_t j = seg + (uint32_t)bit;
        if (!viable_lb(lbk, min(m, (int)j + cost), tv.o, cost)) continue;
        const Cand cd = make_cand(tv, item, sub, m, cost, j);
        if (cost <= 3) sink.st[0].push(cd);
        else sink.st[1].push(cd);
    }
}

// 16 bytes in four registers: byte q <- low byte of v (q a compile-time constant after
// unrolling: one v_perm), and signed byte q for a run-time q (selects; a register array indexed
// at run time would be demoted to LDS or scratch).
struct Bytes16 {
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
    __device__ __forceinline__ void put(int q, uint32_t v) {
        const uint32_t sel = (0x03020100u & ~(0xFFu << (8 * (q & 3)))) | (4u << (8 * (q & 3)));
        if (q < 4) w0 = __builtin_amdgcn_perm(v, w0, sel);
        else if (q < 8) w1 = __builtin_amdgcn_perm(v, w1, sel);
        else if (q < 12) w2 = __builtin_amdgcn_perm(v, w2, sel);
        else w3 = __builtin_amdgcn_perm(v, w3, sel);
    }
    __device__ __forceinline__ int get(int q) const {
        const uint32_t x = q < 8 ? (q < 4 ? w0 : w1) : (q < 12 ? w2 : w3);
        return (int)(int8_t)(uint8_t)(x >> (8 * (q & 3)));
    }
};

// A task's candidate cells held in registers until the wave's next uniform point: its last
// 64-column segment (cells with bits in `cells`, costs in three planes) and its 3' last-column
// rows by list, all already filtered by the task's final lower-bound key.  Cells of earlier
// segments (hit spans over 64 columns: rare) go through the staging sink as before.
struct CandOut {
    uint64_t cells = 0, c0 = 0, c1 = 0, c2 = 0;
    uint64_t rows0 = 0, rows1 = 0;      // rows by list (cost <= 3 / > 3)
    uint64_t pv = 0, mv = 0;            // column `len`: the rows' costs
    uint32_t seg = 0;
    int mlist = -1;                     // cell (m, 0) of an empty 3' view: its list, -1 = none
};

// Sum of v over the wave's 64 lanes, in every lane.  Precondition: wave64 with ALL 64 lanes
// active, i.e. called after reconvergence (both callers, finalize0/1, reach it after block-stride
// loops whose exits every lane takes; an inactive lane would contribute garbage to the xor tree).
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Exclusive prefix sum over the 64 lanes of the wave (every lane calls it), and the total.
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t& total) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, 64);
        if (lane >= (uint32_t)d) x += y;
    }
    total = __shfl(x, 63, 64);
    return x - v;
}

// Write every lane's held candidates: one prefix sum and one global atomic per list for the
// whole wave (per-record or per-flush atomics on the two list counters serialise the scan).
// Called by all lanes of the wave at a wave-uniform point; lanes without a task hold nothing.
__device__ __forceinline__ void emit_cands(const RoundArgs& R, const CandOut& co,
                                           const TaskView& tv, uint32_t item, int sub, int m) {
    const uint32_t n1 = (uint32_t)(__popcll(co.cells & co.c2) + __popcll(co.rows1) +
                                   (co.mlist == 1 ? 1 : 0));
    const uint32_t n0 = (uint32_t)(__popcll(co.cells & ~co.c2) + __popcll(co.rows0) +
                                   (co.mlist == 0 ? 1 : 0));
    uint32_t tot;
    const uint32_t pre = wave_excl_scan(n0 | (n1 << 16), tot);   // <= 64 x 128 per list
    if (tot == 0) return;                                        // wave-uniform
    const uint32_t sh = wave_shard();
    uint32_t b0 = 0, b1 = 0;
    if ((threadIdx.x & 63u) == 0) {
        if (tot & 0xFFFFu) b0 = atomicAdd(R.cand_count + sh * kShardStride, tot & 0xFFFFu);
        if (tot >> 16) b1 = atomicAdd(R.cand_count + (kShards + sh) * kShardStride, tot >> 16);
    }
    b0 = __builtin_amdgcn_readfirstlane(b0) + (pre & 0xFFFFu);
    b1 = __builtin_amdgcn_readfirstlane(b1) + (pre >> 16);
    // the lane's list picks one of two pointers held in SGPRs (R.cand[l] with a per-lane l is a
    // dependent load of the kernel argument before every store)
    __attribute__((address_space(1))) Cand* const cl0 = sgpr_ptr(R.cand[0] + sh * R.cand_scap);
    __attribute__((address_space(1))) Cand* const cl1 = sgpr_ptr(R.cand[1] + sh * R.cand_scap);
    const auto put = [&](int l, const Cand& cd) __attribute__((always_inline)) {
        const uint32_t i = l ? b1++ : b0++;
        if (i < R.cand_scap) store_cand(l ? cl1 : cl0, i, cd);
        else atomicOr(R.flags, 8u);
    };
    uint64_t x = co.cells;
    while (x) {
        const int bit = __ffsll((unsigned long long)x) - 1;
        x &= x - 1;
        const int cost = (int)((co.c0 >> bit) & 1ull) | ((int)((co.c1 >> bit) & 1ull) << 1) |
                         ((int)((co.c2 >> bit) & 1ull) << 2);
        put(cost > 3, make_cand(tv, item, sub, m, cost, co.seg + (uint32_t)bit));
    }
    x = co.rows0 | co.rows1;
    while (x) {
        const int i = __ffsll((unsigned long long)x) - 1;
        x &= x - 1;
        const int cost = col_cost(co.pv, co.mv, i);
        put(cost > 3, make_cand(tv, item, sub, i, cost, tv.len));
    }
    if (co.mlist >= 0)   // (m, 0): a last-row cell, key position t = j = 0 (band kernel)
        put(co.mlist, make_cand(tv, item, sub, m, col_cost(co.pv, co.mv, m), tv.len));
}

// PSTRIDE: u64 between a match vector table's code rows; ZROW: the table has one code row per
// read code 0..3 plus an all-zero row 4 for non-ACGT (the window scan's per-lane rows) instead
// of the panel table's rows 4..7.
template <int HB, class Sink, int PSTRIDE = kPeqStride, bool ZROW = false>
__device__ __forceinline__ int scan_task_cand_hb(const RoundArgs& R, const Sink& sink,
                                                 const TaskView& tv, uint32_t item, int sub,
                                                 const uint64_t* peq, int A, AdLite ad,
                                                 const int8_t* acc, const int8_t* pacc,
                                                 uint32_t js, bool real, uint32_t jlo,
                                                 uint32_t jhi, bool lastcol,
                                                 CandOut* out = nullptr) {
    const int m = ad.m;
    const int kk = ad.kk;   // <= 7 in band mode (three cost planes)
    const bool front = ad.front;
    const uint32_t hbit = (uint32_t)(m - 1);

    uint64_t pv = (front && real) ? 0ull : ~0ull, mv = 0ull;
    int d = (front && real) ? 0 : m;
    int lbk = 0;
    bool segset = false;
    uint32_t seg = 0;
    uint64_t cm = 0, c0 = 0, c1 = 0, c2 = 0;

    // One hit column j (D(m, j) = dv <= kk): the acceptance tests near column 0, the lower-bound
    // key, and the column's cost bits in the current 64-column segment.
    auto hit = [&](uint32_t j, int dv) __attribute__((always_inline)) {
        bool ok = j >= jlo;
        int L0 = m;
        if (ok && (int)j < m + kk) {   // near column 0: the acceptance tables
            ok = dv <= (int)pacc[min(m, (int)j + dv)];
            L0 = min(m, (int)j - dv);
            if (ok && !(L0 >= 0 && dv <= (int)acc[L0])) L0 = -1;
        }
        if (ok) {
            // certainly accepted: aligned length >= L0 and acc is monotone (far from column 0,
            // L0 = m and acc[m] = k >= d)
            if (L0 >= 0) lbk = max(lbk, lb_key(L0 - 3 * dv, tv.o, dv));
            if (!segset) {
                segset = true;
                seg = j;
            }
            const uint64_t bm = 1ull << (j - seg);
            cm |= bm;
            if (dv & 1) c0 |= bm;
            if (dv & 2) c1 |= bm;
            if (dv & 4) c2 |= bm;
        }
    };
    // The 16 steps of a chunk are branch-free: each records the sign of D - kk - 1 (a hit bit,
    // shifted in from the bottom: column q ends at bit 15 - q) and D's low byte; the hit columns
    // of this lane are visited afterwards in column order.  (A per-column branch on D <= kk is
    // taken by some lane of the wave in nearly every column.)
    const int e0 = kk + 1;
    int e = d - e0;                   // D - kk - 1: negative exactly at hit columns
#define DMX_CAND_REC(q)                                                                   \
    {                                                                                     \
        myers_step<HB>(eqv(q), pv, mv, e, hbit);                                          \
        hits = __builtin_amdgcn_alignbit(hits, (uint32_t)e, 31);                          \
        dq.put((q), (uint32_t)e);                                                         \
    }
#define DMX_CAND_VISIT(NQ)                                                                \
    while (hits) {                                                                        \
        const int q = (int)__clz(hits) - (32 - (NQ));                                     \
        hits &= ~(0x80000000u >> __clz(hits));                                            \
        hit(p0 + (uint32_t)q + 1u, dq.get(q) + e0);                                    \
    }
#define DMX_CAND_EQ                                                                       \
    const auto eqv = [&](int q) __attribute__((always_inline)) {                          \
        const uint32_t cq = (codes >> (2 * q)) & 3u, nq = (nb >> q) & 1u;                 \
        return peq[(ZROW ? (nq ? 4u : cq) : (cq | (nq << 2))) * PSTRIDE];                 \
    };

    uint32_t p0 = js;
    // the next chunk in flight (clean windows: codes only, chunk16_load skips the mask)
    Chunk16 nx = chunk16_load(R.pk, tv, (int)p0);
    for (; p0 + 16 <= jhi; p0 += 16) {
        uint32_t codes, nb;
        chunk16_codes(tv, (int)p0, nx, codes, nb);
        if (p0 + 16 < jhi) nx = chunk16_load(R.pk, tv, (int)p0 + 16);
        if (segset && p0 + 16 >= seg + 64) {   // this chunk could overflow the 64-bit segment
            flush_cands(sink, tv, item, sub, m, lbk, seg, cm, c0, c1, c2);
            segset = false;
            cm = c0 = c1 = c2 = 0;
        }
        DMX_CAND_EQ
        uint32_t hits = 0;
        Bytes16 dq;
#pragma unroll
        for (int q = 0; q < 16; ++q) DMX_CAND_REC(q)
        DMX_CAND_VISIT(16)
    }
    if (p0 < jhi) {
        uint32_t codes, nb;
        chunk16_codes(tv, (int)p0, nx, codes, nb);
        if (segset && p0 + 16 >= seg + 64) {
            flush_cands(sink, tv, item, sub, m, lbk, seg, cm, c0, c1, c2);
            segset = false;
            cm = c0 = c1 = c2 = 0;
        }
        DMX_CAND_EQ
        const int cnt = (int)(jhi - p0);
        uint32_t hits = 0;
        Bytes16 dq;
#pragma unroll
        for (int q = 0; q < 16; ++q)
            if (q < cnt) DMX_CAND_REC(q)
        // cnt steps ran: column q's hit bit sits at bit cnt - 1 - q
        while (hits) {
            const int q = (int)__clz(hits) - (32 - cnt);
            hits &= ~(0x80000000u >> __clz(hits));
            hit(p0 + (uint32_t)q + 1u, dq.get(q) + e0);
        }
    }
    d = e + e0;
#undef DMX_CAND_REC
#undef DMX_CAND_VISIT
#undef DMX_CAND_EQ
    // 3' adapters: last-column cells (adapter prefix aligned at the read end); cell (m, 0) of
    // an empty view (no column loop reports it as a last-row cell) in `mrow`
    uint64_t rows = 0;
    bool mrow = false;
    const uint32_t len = tv.len;
    if (lastcol && !front) {   // an empty view too: cells (i, 0) cost i (rate >= 1 accepts)
        int dd = 0;
        const int ilast = len == 0 ? m : m - 1;
        for (int i = 1; i <= ilast; ++i) {
            dd += (int)((pv >> (i - 1)) & 1ull) - (int)((mv >> (i - 1)) & 1ull);
            if (dd <= (int)acc[i]) {              // accepted for sure (aligned length is i)
                if (i < m) rows |= 1ull << i;
                else mrow = true;
                lbk = max(lbk, lb_key(i - 3 * dd, tv.o, dd));
            }
        }
    }
    if (out) {   // hold the cells for the wave's direct emission (emit_cands)
        uint64_t keep = 0, x = cm;
        while (x) {
            const int bit = __ffsll((unsigned long long)x) - 1;
            x &= x - 1;
            const int cost = (int)((c0 >> bit) & 1ull) | ((int)((c1 >> bit) & 1ull) << 1) |
                             ((int)((c2 >> bit) & 1ull) << 2);
            if (viable_lb(lbk, min(m, (int)(seg + (uint32_t)bit) + cost), tv.o, cost))
                keep |= 1ull << bit;
        }
        out->cells = keep;
        out->c0 = c0;
        out->c1 = c1;
        out->c2 = c2;
        out->seg = seg;
        out->pv = pv;
        out->mv = mv;
        out->rows0 = out->rows1 = 0;
        while (rows) {
            const int i = __ffsll((unsigned long long)rows) - 1;
            rows &= rows - 1;
            const int cost = col_cost(pv, mv, i);
            if (!viable_lb(lbk, i, tv.o, cost)) continue;
            if (cost <= 3) out->rows0 |= 1ull << i;
            else out->rows1 |= 1ull << i;
        }
        out->mlist = -1;
        if (mrow) {
            const int cost = col_cost(pv, mv, m);
            if (viable_lb(lbk, m, tv.o, cost)) out->mlist = cost <= 3 ? 0 : 1;
        }
        return lbk;
    }
    if (cm) flush_cands(sink, tv, item, sub, m, lbk, seg, cm, c0, c1, c2);
    while (rows) {                                // scan order: after every last-row cell
        const int i = __ffsll((unsigned long long)rows) - 1;
        rows &= rows - 1;
        const int cost = col_cost(pv, mv, i);
        if (!viable_lb(lbk, i, tv.o, cost)) continue;
        const Cand cd = make_cand(tv, item, sub, i, cost, len);
        if (cost <= 3) sink.st[0].push(cd);
        else sink.st[1].push(cd);
    }
    if (mrow) {
        const int cost = col_cost(pv, mv, m);
        if (viable_lb(lbk, m, tv.o, cost)) {
            const Cand cd = make_cand(tv, item, sub, m, cost, len);
            if (cost <= 3) sink.st[0].push(cd);
            else sink.st[1].push(cd);
        }
    }
    return lbk;
}

// The last adapter row's bit sits in the low or the high word of the 64-bit vectors; both
// variants are compiled so the step needs no per-column select.
template <class Sink, int PSTRIDE = kPeqStride, bool ZROW = false>
__device__ __forceinline__ int scan_task_cand(const RoundArgs& R, const Sink& sink,
                                              const TaskView& tv, uint32_t item, int sub,
                                              const uint64_t* peq, int A, AdLite ad,
                                              const int8_t* acc, const int8_t* pacc,
                                              uint32_t js, bool real, uint32_t jlo,
                                              uint32_t jhi, bool lastcol,
                                              CandOut* out = nullptr) {
    if (ad.m > 32)
        return scan_task_cand_hb<1, Sink, PSTRIDE, ZROW>(R, sink, tv, item, sub, peq, A, ad, acc,
                                                         pacc, js, real, jlo, jhi, lastcol, out);
    return scan_task_cand_hb<0, Sink, PSTRIDE, ZROW>(R, sink, tv, item, sub, peq, A, ad, acc,
                                                     pacc, js, real, jlo, jhi, lastcol, out);
}

#define DMX_CAND_STAGE                                                                    \
    __shared__ Cand s_cand[2][kCandStageCap];                                             \
    __shared__ uint32_t s_ccnt[2], s_cbase[2];                                            \
    if (threadIdx.x < 2) s_ccnt[threadIdx.x] = 0;                                         \
    const uint32_t bsh = blockIdx.x & (uint32_t)(kShards - 1);                           \
    const CandSink sink{{Stage<Cand, kCandStageCap>{s_cand[0], &s_ccnt[0], &s_cbase[0],    \
                                                    R.cand[0] + bsh * R.cand_scap,         \
                                                    R.cand_count + bsh * kShardStride,     \
                                                    R.cand_scap,                           \
                                                    R.flags, 8u},                          \
                         Stage<Cand, kCandStageCap>{s_cand[1], &s_ccnt[1], &s_cbase[1],    \
                                                    R.cand[1] + bsh * R.cand_scap,         \
                                                    R.cand_count +                         \
                                                        (kShards + bsh) * kShardStride,    \
                                                    R.cand_scap, R.flags, 8u}}};

// Both kernels are templated on BAND; only the stage the instantiation uses takes LDS.
#define DMX_STAGES                                                                        \
    __shared__ Cluster s_cl[BAND ? 1 : kStageCap];                                        \
    __shared__ uint32_t s_clcnt, s_clbase;                                                \
    if (threadIdx.x == 0) s_clcnt = 0;                                                    \
    const Stage<Cluster> st{s_cl, &s_clcnt, &s_clbase, R.cl, R.cl_count, R.cl_cap,        \
                            R.flags, 1u};                                                 \
    __shared__ Cand s_cand[2][BAND ? kCandStageCap : 1];                                  \
    __shared__ uint32_t s_ccnt[2], s_cbase[2];                                            \
    if (threadIdx.x < 2) s_ccnt[threadIdx.x] = 0;                                         \
    const uint32_t bsh = blockIdx.x & (uint32_t)(kShards - 1);                           \
    const CandSink sink{{Stage<Cand, kCandStageCap>{s_cand[0], &s_ccnt[0], &s_cbase[0],    \
                                                    R.cand[0] + bsh * R.cand_scap,         \
                                                    R.cand_count + bsh * kShardStride,     \
                                                    R.cand_scap,                           \
                                                    R.flags, 8u},                          \
                         Stage<Cand, kCandStageCap>{s_cand[1], &s_ccnt[1], &s_cbase[1],    \
                                                    R.cand[1] + bsh * R.cand_scap,         \
                                                    R.cand_count +                         \
                                                        (kShards + bsh) * kShardStride,    \
                                                    R.cand_scap, R.flags, 8u}}};

#define DMX_CLUSTER_STAGE                                                                 \
    __shared__ Cluster s_cl[kStageCap];                                                   \
    __shared__ uint32_t s_clcnt, s_clbase;                                                \
    if (threadIdx.x == 0) s_clcnt = 0;                                                    \
    const Stage<Cluster> st{s_cl, &s_clcnt, &s_clbase, R.cl, R.cl_count, R.cl_cap,        \
                            R.flags, 1u};

// Full scan (panels without a usable shared suffix): one lane per (item, orientation, adapter).
template <bool BAND>
__global__ __launch_bounds__(kScanBlock) void scan_kernel(RoundArgs R) {
    __shared__ uint64_t s_peq[8 * kPeqStride];
    __shared__ int8_t s_acc[72 * kMaxAdapters];
    __shared__ int8_t s_pacc[72 * kMaxAdapters];
    __shared__ uint32_t s_amk[kMaxAdapters];
    DMX_STAGES
    load_panel_lds(R.panel, s_peq, s_acc, s_pacc, s_amk);
    __syncthreads();

    const int A = R.panel->n_adapters;
    const int T = R.T;
    const int rpb = kScanBlock / T;
    const int tid = threadIdx.x;
    const uint32_t item = blockIdx.x * (uint32_t)rpb + (uint32_t)(tid / T);
    const int sub = tid % T;
    const uint32_t n_items = R.items ? *R.n_items_dev : R.n_items;
    if (tid < rpb * T && item < n_items) {
        TaskView tv;
        task_view(R, item, sub, A, tv);
        int lb;
        if constexpr (BAND)
            lb = scan_task_cand(R, sink, tv, item, sub, s_peq + tv.a, A, ad_lite(s_amk[tv.a]),
                                s_acc + 72 * tv.a, s_pacc + 72 * tv.a, 0, true, 1, tv.len, true);
        else
            lb = scan_task(R, st, tv, item, sub, s_peq + tv.a, A, ad_lite(s_amk[tv.a]),
                           s_acc + 72 * tv.a, s_pacc + 72 * tv.a, 0, true, 1, tv.len, true);
        const uint32_t slot = slot_of(R, item, sub);
        if (lb > 0 && DMX_BOUND(R.pk.bd, slots, slot, kBufSlot)) atomicMax(&R.lb[slot], lb);
    }
    if constexpr (BAND) {
        sink.st[0].flush();
        sink.st[1].flush();
    } else {
        st.flush();
    }
}

__device__ __forceinline__ uint32_t align32(uint32_t hi, uint32_t lo, uint32_t r) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> r);
}

__device__ __forceinline__ uint32_t bsel(uint32_t mask, uint32_t a, uint32_t b) {
    return (a & mask) | (b & ~mask);      // mask ? a : b, bitwise (stays in registers)
}

// ---------------------------------------------------------------------------------------------
// Consecutive 64-position stretches of a view, read as whole aligned 64-nt blocks of the packed
// read (one 16-B code load + one 8-B mask load per block, instead of two 4-B gathers per 16
// positions): the two blocks holding the current stretch and the next block in flight.  A lane's
// stretches start 64 positions apart, so its bit alignment inside the blocks never changes and the
// extraction is the filter's (seg_extract): word selects + funnel shifts, no indexed registers.
// Strand 1 walks the global blocks downwards and reverses + complements each 16-position chunk.
// MASK = false: the no-match mask is not loaded and every chunk's no-match bits are 0 (a read N
// reads as its packed code, A): for the necessary-condition stages.
// ---------------------------------------------------------------------------------------------
template <bool MASK = true>
struct ViewBlocks {
    uint32_t cw[12], nw[6];      // [0..7]/[0..3]: blocks B, B + 1 (ascending); [8..11]/[4..5]:
                                 // the block in flight (B + 2 on strand 0, B - 1 on strand 1)
    uint32_t m1, m2, r, r2;
    const uint4* sp;
    const uint2* np;
    int64_t nxt;                 // the next block to load
    bool rev;
#ifdef DMX_DEBUG_BOUNDS
    Bounds bd;
#endif

    __device__ __forceinline__ void load(int k, int64_t b) {
#ifdef DMX_DEBUG_BOUNDS
        if (!bchk(bd, 4 * b, bd.lo, bd.hi - 3, kBufSeq) ||
            (MASK && !bchk(bd, 2 * b, bd.lo, bd.hi - 1, kBufMask))) {
            for (int x = 0; x < 4; ++x) cw[4 * k + x] = 0u;
            nw[2 * k] = nw[2 * k + 1] = 0u;
            return;
        }
#endif
        const uint4 c4 = sp[b];
        cw[4 * k + 0] = c4.x;
        cw[4 * k + 1] = c4.y;
        cw[4 * k + 2] = c4.z;
        cw[4 * k + 3] = c4.w;
        if constexpr (MASK) {
            const uint2 n2 = np[b];
            nw[2 * k + 0] = n2.x;
            nw[2 * k + 1] = n2.y;
        } else {
            nw[2 * k + 0] = nw[2 * k + 1] = 0u;
        }
    }
    // view positions [p, p + 64 * n_stretch) of the view (strand, start, n, off) of tv
    __device__ __forceinline__ void init(const RoundArgs& R, const TaskView& tv, int p) {
        rev = tv.strand != 0;
        const int64_t g = rev ? (int64_t)tv.off + (int64_t)tv.n - 1 - tv.start - p - 63
                              : (int64_t)tv.off + tv.start + p;
        const int64_t blk = g >> 6;               // floor: the buffers carry guard words
        const uint32_t sh = (uint32_t)(g & 63);
        sp = reinterpret_cast<const uint4*>(R.pk.seq);
        np = reinterpret_cast<const uint2*>(R.pk.nmask);
#ifdef DMX_DEBUG_BOUNDS
        bd = R.pk.bd;
#endif
        load(0, blk);
        load(1, blk + 1);
        nxt = rev ? blk - 1 : blk + 2;
        load(2, nxt);
        nxt += rev ? -1 : 1;
        m1 = ((sh >> 4) & 1u) ? ~0u : 0u;
        m2 = ((sh >> 5) & 1u) ? ~0u : 0u;
        r = (2u * sh) & 31u;
        r2 = sh & 31u;
    }
    // the current stretch as 4 chunks (view order), then slide by one block; `more`: a later
    // stretch will be needed after the next one (load its block now)
    __device__ __forceinline__ void extract(uint32_t vc[4], uint32_t vn[4], bool more) {
        uint32_t a[7], t[5], asc[4], tn[3];
#pragma unroll
        for (int k = 0; k < 7; ++k) a[k] = bsel(m1, cw[k + 1], cw[k]);
#pragma unroll
        for (int k = 0; k < 5; ++k) t[k] = bsel(m2, a[k + 2], a[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) asc[k] = align32(t[k + 1], t[k], r);
#pragma unroll
        for (int k = 0; k < 3; ++k) tn[k] = bsel(m2, nw[k + 1], nw[k]);
        const uint32_t an[2] = {align32(tn[1], tn[0], r2), align32(tn[2], tn[1], r2)};
        if (!rev) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                vc[c] = asc[c];
                vn[c] = MASK ? (an[c >> 1] >> (16 * (c & 1))) & 0xFFFFu : 0u;
            }
        } else {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int d = 3 - c;
                vc[c] = ~rev_pairs(asc[d]);                        // complement = 3 - code
                vn[c] = MASK ? __brev((an[d >> 1] >> (16 * (d & 1))) & 0xFFFFu) >> 16 : 0u;
            }
        }
        // slide: strand 0 (lo, hi, in flight) -> (hi, in flight, next);
        //        strand 1 (lo, hi, in flight) -> (in flight, lo, next)
        const uint32_t rm = rev ? ~0u : 0u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t lo = cw[k], hi = cw[4 + k], fl = cw[8 + k];
            cw[k] = bsel(rm, fl, hi);
            cw[4 + k] = bsel(rm, lo, fl);
        }
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const uint32_t lo = nw[k], hi = nw[2 + k], fl = nw[4 + k];
            nw[k] = bsel(rm, fl, hi);
            nw[2 + k] = bsel(rm, lo, fl);
        }
        if (more) {
            load(2, nxt);
            nxt += rev ? -1 : 1;
        }
    }
};

// ---------------------------------------------------------------------------------------------
// filter: 32-bit Myers of the panel's shared suffix block (L rows) over every view, cut into
// SEGMENTS of S = kSegSpan - W view positions.  One lane per segment: lanes of a wave take
// consecutive segments of the same view, so their loads cover one contiguous stretch of the
// packed read (each lane streams its positions once, as whole aligned 64-nt blocks).
// A segment after the first starts W = L + kf columns early with the restricted-start column
// D(i) = i: an alignment of the block with cost <= kf spans at most L + kf columns, so every
// hit column of the segment (b(j) <= kf) is computed exactly.  Hit columns
// (b(j) <= min(kf, pf[min(71, j + kf)])) are grouped into windows; a window never crosses a
// segment boundary.  Segments are ordered strand 0 first, then strand 1, so the strand branch is
// wave-uniform except in one wave per block.
// ---------------------------------------------------------------------------------------------
#ifndef DMX_SEG_VIEWS
#define DMX_SEG_VIEWS 512
#endif
constexpr uint32_t kSegViewsPerBlock = DMX_SEG_VIEWS;   // views per filter block (>= 256)
// Segment span A/B with streamed blocks (c2x24, ms per step): 256 -> 52.38, 512 -> 52.41,
// 768 -> 55.99 (the warm-up saved is lost to the longer idle tails of last segments)
#ifndef DMX_SEG_SPAN
#define DMX_SEG_SPAN 256
#endif
constexpr int kSegSpan = DMX_SEG_SPAN;        // view positions per segment (S + W)
// A view's last segment spans at most kSegSpan positions, i.e. ceil(kSegSpan / 64) 64-position
// steps; the block prologue groups last segments into FOUR step buckets (16-bit fields of
// s_tot / s_totl, LB[g][0..4]).  A span-384 A/B build with kStepsPerBucket = kSegSpan / 256 = 1
// put 6-step segments in buckets 5..6: LB[g][5] read past the array, s_lastv written outside
// its region, and the run died with an illegal memory access (round 3).  The bucket width is
// therefore derived from the span so that the invariant below holds for every span; the kernel
// also flags (bit 16) any bucket outside 1..4 instead of indexing with it.
constexpr int kStepsPerBucket = (kSegSpan + 255) / 256;   // 64-position steps per bucket
constexpr int kLastBuckets = 4;
static_assert(kSegSpan >= 128 && kSegSpan <= 1024 && kSegSpan % 64 == 0,
              "segment span: 128..1024 positions, whole 64-position steps");
static_assert(kLastBuckets * kStepsPerBucket * 64 >= kSegSpan,
              "every last segment's step count must fall into one of the four step buckets");

__device__ __forceinline__ Window make_window(uint32_t item, int o, const TaskView& tv,
                                              uint32_t j1, uint32_t j2, int lastcol, int bmin,
                                              bool clean = false) {
    Window w;
    w.item = item;
    w.o = (uint8_t)o;
    w.lastcol = (uint8_t)lastcol;
    w.strand = (uint8_t)(tv.strand | (clean ? kWinClean : 0u));
    w.bmin = (uint8_t)min(bmin, 255);
    w.j1 = j1;
    w.j2 = j2;
    w.n = tv.n;
    w.start = tv.start;
    w.len = tv.len;
    w.info = 0;
    w.off = tv.off;
    return w;
}

struct SegState {
    uint32_t pv, mv;
    int e;          // last-row cost b minus (kf_far + 1): negative exactly where b <= kf_far
    bool have;
    uint32_t w1, w2;
    int wb;
    uint64_t dh;    // clean flags: bit c = a no-match bit in view positions [hb + 16c, +16)
    int hb;
};

// The filter's clean-flag history spans clean_reach (<= 128) positions before the segment and
// the segment itself in 16-position chunks: 64 bits hold it for spans up to 768.
#ifndef DMX_CLEAN_OFF   // A/B: 1 = no clean flags (every window loads the mask, round 4)
#define DMX_CLEAN_OFF 0
#endif
constexpr bool kCleanHist = !DMX_CLEAN_OFF && (kSegSpan + 128) / 16 + 4 <= 64;

// Is the no-match mask zero over the view positions an exact stage reads for window [w1, w2]
// (columns): [w1 - rb, w2 - 1], clipped at the view start?  (Positions outside the view are
// never used by them.)  rb = clean_reach, 0 = off.
__device__ __forceinline__ bool window_clean(const SegState& S, uint32_t w1, uint32_t w2, int rb) {
    if (!kCleanHist || rb == 0) return false;
    const int lo = max(0, (int)w1 - rb), hi = (int)w2 - 1;
    if (hi < lo) return true;                     // nothing of the view is read
    const int cl = (lo - S.hb) >> 4, ch = (hi - S.hb) >> 4;
    if (cl < 0 || ch > 63) return false;          // outside the history: unknown
    const uint64_t m = (ch - cl >= 63 ? ~0ull : ((2ull << (ch - cl)) - 1ull)) << cl;
    return (S.dh & m) == 0;
}

// Myers step of the filter block, stored in the TOP filter_len bits of the word (the rows
// below are all-match padding that stays at cost 0, so they act as row 0): the last row is bit
// 31, and the carries of the two horizontal shifts are its +1 / -1 (one v_add_co each, whose
// carry the cost update consumes) instead of two bit-field extracts.
__device__ __forceinline__ void myers_step_top(uint32_t eq, uint32_t& pv, uint32_t& mv, int& e) {
    const uint32_t xv = eq | mv;
    const uint32_t xh = (((eq & pv) + pv) ^ pv) | eq;
    const uint32_t ph = mv | ~(xh | pv);
    const uint32_t mh = pv & xh;
    // (round 5 A/B: the +1 / -1 as shifts + v_add3 instead of the carries removes the VCC
    // hazard s_nops, 33 -> 3 per 16 columns, but lengthens the dependent chain: filter 11.6 ->
    // 13.9 ms, profiles/r5_ab_filter_cost_shift.txt)
    uint32_t cp, cm;
    const uint32_t ph2 = __builtin_addc(ph, ph, 0u, &cp);
    const uint32_t mh2 = __builtin_addc(mh, mh, 0u, &cm);
    e += (int)cp - (int)cm;
    pv = mh2 | ~(xv | ph2);
    mv = ph2 & xv;
}

// 8 two-bit codes (16 bits) -> 8 nibbles holding code * 4 (an LDS byte offset into a u32
// table): one v_perm spreads the two bytes, two shift-or-mask steps the codes.
__device__ __forceinline__ uint32_t spread_codes(uint32_t codes, uint32_t sel) {
    uint32_t x = __builtin_amdgcn_perm(0u, codes, sel);   // bytes -> bytes 0 and 2
    x = (x | (x << 4)) & 0x0F0F0F0Fu;                      // 4-bit halves -> bytes
    return ((x << 2) | (x << 4)) & 0xCCCCCCCCu;             // 2-bit codes -> nibbles, * 4
}

// One 16-position chunk (view positions p0 .. p0+15) of a filter segment.  All 16 steps always
// run (lanes of a wave stay in lockstep); columns past the segment end (q >= cnt) cannot hit.
// The steps are branch-free: hit columns go into a 16-bit mask (and the chunk's minimum b, a
// lower bound of every hit's b, into cb); windows are formed afterwards.  CAREFUL (the first 64
// positions of every segment): per-column thresholds, -1 in the warm-up (columns <= hit_from)
// and the prefix-max acceptance pf[j + kf] near the view start; beyond them every column's
// threshold is kf_far (the host checks pf[j + kf] >= kf_far for j > 64).
template <bool CAREFUL>
__device__ __forceinline__ void filter_chunk(uint32_t codes, uint32_t nb, uint32_t p0, int cnt,
                                             SegState& S, const uint32_t* s_fpeq,
                                             const int8_t* s_thr, int kf_far, uint32_t gap,
                                             uint32_t hit_from, int rb,
                                             const WaveStage<Window, kWaveWinCap>& st,
                                             uint32_t item, int o,
                                             const TaskView& tv) {
    uint32_t eq[16];
    // N read as A unless kNecessaryMask: the spread path for every chunk
    if (!kNecessaryMask || __builtin_amdgcn_ballot_w64(nb != 0u) == 0) {   // byte offsets
        const uint32_t lo = spread_codes(codes, 0x0c010c00u);
        const uint32_t hi = spread_codes(codes, 0x0c030c02u);
        const char* base = reinterpret_cast<const char*>(s_fpeq);
#pragma unroll
        for (int q = 0; q < 16; ++q)
            eq[q] = *reinterpret_cast<const uint32_t*>(
                base + __builtin_amdgcn_ubfe(q < 8 ? lo : hi, 4 * (q & 7), 4));
    } else {
#pragma unroll
        for (int q = 0; q < 16; ++q)
            eq[q] = s_fpeq[((codes >> (2 * q)) & 3u) | (((nb >> q) & 1u) << 2)];
    }
    uint4 tw = {0u, 0u, 0u, 0u};
    if constexpr (CAREFUL)   // 16 per-position thresholds (s_thr: 16-byte aligned rows)
        tw = *reinterpret_cast<const uint4*>(s_thr + (hit_from == 0 ? p0 : 240u));
    uint32_t hits = 0;       // column q's hit bit is shifted in from the bottom: ends at 15 - q
    int cm = 1 << 20;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        myers_step_top(eq[q], S.pv, S.mv, S.e);
        int sgn = S.e;       // < 0 exactly at a hit column
        if constexpr (CAREFUL) {
            const uint32_t w = q < 4 ? tw.x : q < 8 ? tw.y : q < 12 ? tw.z : tw.w;
            const int t = __builtin_amdgcn_sbfe((int)w, 8 * (q & 3), 8) |
                          ((int)(p0 + (uint32_t)q - hit_from) >> 31);   // -1 in the warm-up
            sgn = S.e + kf_far - t;
        }
        hits = __builtin_amdgcn_alignbit(hits, (uint32_t)sgn, 31);
        cm = min(cm, S.e);
    }
    hits &= cnt >= 16 ? 0xFFFFu : (cnt > 0 ? (0xFFFFu << (16 - cnt)) & 0xFFFFu : 0u);
#ifdef DMX_FILTER_NO_HITS   // timing A/B only (results invalid): the filter without windows.
    asm volatile("" ::"v"(hits), "v"(cm));   // The scan stays live.  Round 5: filter 11.45 /
    hits = 0;                                // 11.69 -> 10.91 / 10.90 ms, i.e. forming windows
#endif                                       // costs ~0.6 ms (profiles/r5_ab_filter_no_hits.txt)
    if constexpr (!CAREFUL) {   // warm-up columns (j <= hit_from) of a later segment never hit
        const int nw = (int)hit_from - (int)p0;
        hits &= nw >= 16 ? 0u : (nw <= 0 ? 0xFFFFu : (0xFFFFu >> nw));
    }
    const int cb = cm + kf_far + 1;   // the chunk's minimum b: a lower bound of every hit's b
    while (hits) {
        const int q = (int)__clz(hits) - 16;
        hits &= ~(0x80000000u >> __clz(hits));
        const uint32_t j = p0 + (uint32_t)q + 1;
        if (S.have && j - S.w2 <= gap) {
            S.w2 = j;
            S.wb = min(S.wb, cb);
        } else {
            if (S.have)
                st.push(make_window(item, o, tv, S.w1, S.w2, 0, S.wb,
                                    window_clean(S, S.w1, S.w2, rb)));
            S.have = true;
            S.w1 = S.w2 = j;
            S.wb = cb;
        }
    }
}

// Process view positions [P0, P1) (P1 - P0 <= kSegSpan) of one view, streaming the packed
// read as whole aligned 64-nt blocks (ViewBlocks: two blocks held, the next one in flight).
__device__ __forceinline__ void filter_segment(const RoundArgs& R, const TaskView& tv,
                                               uint32_t P0, uint32_t P1, SegState& S,
                                               const uint32_t* s_fpeq, const int8_t* s_thr,
                                               int kf_far, uint32_t gap, uint32_t hit_from,
                                               int rb, const WaveStage<Window, kWaveWinCap>& st,
                                               uint32_t item, int o) {
    ViewBlocks<true> B;
    B.init(R, tv, (int)P0);
    // clean-flag history: 16-position chunks from hb = P0 - rb; the rb
    // positions before the segment are read as mask words (none before the view start: the
    // exact stages never read there), the segment's own from its blocks below
    S.hb = (int)P0 - rb;
    S.dh = 0;
    if (kCleanHist && rb) {
        for (int q = 0; q < rb; q += 32) {
            const int p = S.hb + q;
            if (p + 32 <= 0) continue;
            const uint32_t m = mask32s(R.pk, tv, p);   // (a chunk past P0: the segment's own)
            S.dh |= (uint64_t)(((m & 0xFFFFu) ? 1u : 0u) | ((m >> 16) ? 2u : 0u)) << (q >> 4);
        }
    }
    const uint32_t nsteps = (P1 - P0 + 63u) / 64u;
    for (uint32_t s = 0, p0 = P0; p0 < P1; ++s, p0 += 64) {
        uint32_t vc[4], vn[4];
        B.extract(vc, vn, s + 2u < nsteps);
        if (kCleanHist && rb) {
            const uint32_t nz = (vn[0] ? 1u : 0u) | (vn[1] ? 2u : 0u) | (vn[2] ? 4u : 0u) |
                                (vn[3] ? 8u : 0u);
            S.dh |= (uint64_t)nz << ((rb >> 4) + 4 * (int)s);
        }
        // per-column thresholds only near the view start (segment 0, grouped first in the
        // block's task order, so the branch is wave-uniform but for one wave); later segments
        // have threshold kf_far everywhere and mask their warm-up columns
        const bool careful = p0 == P0 && hit_from == 0;
        for (int c = 0; c < 4; ++c) {
            const uint32_t pc = p0 + 16u * (uint32_t)c;
            const int cnt = (int)P1 - (int)pc;
            if (careful)
                filter_chunk<true>(vc[0], vn[0], pc, cnt, S, s_fpeq, s_thr, kf_far, gap,
                                   hit_from, rb, st, item, o, tv);
            else
                filter_chunk<false>(vc[0], vn[0], pc, cnt, S, s_fpeq, s_thr, kf_far, gap,
                                    hit_from, rb, st, item, o, tv);
            vc[0] = vc[1];
            vc[1] = vc[2];
            vc[2] = vc[3];
            vn[0] = vn[1];
            vn[1] = vn[2];
            vn[2] = vn[3];
        }
    }
}

// 5 waves per SIMD (96 VGPRs, one spilled) measured 52.41 -> 52.36 ms per step against 4
#ifndef DMX_FILTER_WAVES
#define DMX_FILTER_WAVES 5
#endif
__global__ __launch_bounds__(kScanBlock) __attribute__((amdgpu_waves_per_eu(DMX_FILTER_WAVES))) void filter_kernel(RoundArgs R) {
    __shared__ uint32_t s_fpeq[8];
    __shared__ int8_t s_pf[72];
    __shared__ __attribute__((aligned(16))) int8_t s_thr[kScanBlock];
    __shared__ Window s_win[kScanBlock / 64][kWaveWinCap];   // per-wave window staging
    __shared__ uint32_t s_wcnt[kScanBlock / 64];
    // Block task order per strand: every view's segment 0; then the middle segments (neither
    // first nor last), view-major; then the views' last segments grouped by their number of
    // 64-position steps (1..4), so the waves of short tails finish early.  s_pre / s_prl: first
    // / middle segments before view v; s_lastv: the views of the last-segment region in order.
    __shared__ uint32_t s_pre[2][kSegViewsPerBlock], s_prl[2][kSegViewsPerBlock];
    __shared__ uint16_t s_lastv[2][kSegViewsPerBlock];
    __shared__ uint32_t s_tot[2][kScanBlock], s_totl[2][kScanBlock];
    const DevPanel* P = R.panel;
    const int no = P->n_orient;
    const uint32_t n_items = R.items ? *R.n_items_dev : R.n_items;
    const uint32_t n_views = n_items * (uint32_t)no;
    const uint32_t vbeg = blockIdx.x * kSegViewsPerBlock;
    if (vbeg >= n_views) return;                       // block-uniform
    const uint32_t nv = min(n_views - vbeg, kSegViewsPerBlock);
    const int A = P->n_adapters;
    const int L = P->scan_len;                         // the block's last L rows (<= filter_len)
    const int kf = P->kf;
    const uint32_t W = (uint32_t)(L + kf);
    const uint32_t SEG = (uint32_t)kSegSpan - W;       // host guarantees W <= 96
    if (threadIdx.x < 8) s_fpeq[threadIdx.x] = P->filter_peq[threadIdx.x];
    if (threadIdx.x < 72) s_pf[threadIdx.x] = P->pf[threadIdx.x];
    if (threadIdx.x < kScanBlock / 64) s_wcnt[threadIdx.x] = 0;
    {   // hit threshold of column j = p + 1 (view position p): the largest cost d <= kf_far that
        // an acceptable last-row cell (m, j) of some adapter can have.  Its aligned adapter length
        // is at most j + d, so d <= pf[min(71, j + d)]; b(j) <= d.  (Near the view start this is
        // much tighter than d <= pf[j + kf]: a column j < min_overlap never hits.)
        const int far0 = min((int)P->kf, (int)P->pf[71]);
        const int j = (int)threadIdx.x + 1;
        int t = -1;
        for (int d = 0; d <= far0; ++d)
            if (d <= (int)P->pf[min(j + d, 71)]) t = d;
        s_thr[threadIdx.x] = (int8_t)t;
    }

    // segment counts per view, grouped by strand; block-wide exclusive scan
    constexpr int VPT = kSegViewsPerBlock / kScanBlock;   // views per thread
    uint32_t cnt[VPT], bk[VPT];
    int grp[VPT];
    uint32_t sum0 = 0, sum1 = 0, suml0 = 0, suml1 = 0;
#pragma unroll
    for (int e = 0; e < VPT; ++e) {
        const uint32_t vl = threadIdx.x * VPT + e;
        cnt[e] = 0;
        bk[e] = 0;
        grp[e] = 0;
        if (vl < nv) {
            const uint32_t v = vbeg + vl;
            TaskView tv;
            task_view(R, v / (uint32_t)no, (int)(v % (uint32_t)no) * A, A, tv);
            // an empty view of a 3' panel still gets its last-column window (one segment)
            cnt[e] = tv.len ? (tv.len + SEG - 1) / SEG : (P->where == kFront ? 0u : 1u);
            grp[e] = (int)tv.strand;
            if (cnt[e] >= 2) {   // last segment: positions [seg0 - W, len), in 64-position
                bk[e] = ((tv.len - (cnt[e] - 1u) * SEG + W + 63u) / 64u + kStepsPerBucket - 1u) /
                        kStepsPerBucket;   // steps, kStepsPerBucket per bucket (1..4)
                if (bk[e] < 1u || bk[e] > (uint32_t)kLastBuckets) {   // excluded statically
                    atomicOr(R.flags, 16u);
                    bk[e] = 0;
                }
            }
        }
        const uint32_t f = cnt[e] ? 1u : 0u, l = cnt[e] >= 2 ? cnt[e] - 2u : 0u;
        if (grp[e]) {
            sum1 += f;
            suml1 += l;
        } else {
            sum0 += f;
            suml0 += l;
        }
    }
    s_tot[0][threadIdx.x] = sum0;
    s_tot[1][threadIdx.x] = sum1;
    s_totl[0][threadIdx.x] = suml0;
    s_totl[1][threadIdx.x] = suml1;
    __syncthreads();
    for (uint32_t d = 1; d < kScanBlock; d <<= 1) {   // inclusive Hillis-Steele scans
        uint32_t x0 = 0, x1 = 0, y0 = 0, y1 = 0;
        if (threadIdx.x >= d) {
            x0 = s_tot[0][threadIdx.x - d];
            x1 = s_tot[1][threadIdx.x - d];
            y0 = s_totl[0][threadIdx.x - d];
            y1 = s_totl[1][threadIdx.x - d];
        }
        __syncthreads();
        s_tot[0][threadIdx.x] += x0;
        s_tot[1][threadIdx.x] += x1;
        s_totl[0][threadIdx.x] += y0;
        s_totl[1][threadIdx.x] += y1;
        __syncthreads();
    }
    {
        uint32_t r0 = s_tot[0][threadIdx.x] - sum0, r1 = s_tot[1][threadIdx.x] - sum1;
        uint32_t q0 = s_totl[0][threadIdx.x] - suml0, q1 = s_totl[1][threadIdx.x] - suml1;
#pragma unroll
        for (int e = 0; e < VPT; ++e) {
            const uint32_t vl = threadIdx.x * VPT + e;
            if (vl < kSegViewsPerBlock) {
                s_pre[0][vl] = r0;
                s_pre[1][vl] = r1;
                s_prl[0][vl] = q0;
                s_prl[1][vl] = q1;
            }
            const uint32_t f = cnt[e] ? 1u : 0u, l = cnt[e] >= 2 ? cnt[e] - 2u : 0u;
            if (grp[e]) {
                r1 += f;
                q1 += l;
            } else {
                r0 += f;
                q0 += l;
            }
        }
    }
    __syncthreads();
    const uint32_t F0 = s_tot[0][kScanBlock - 1], F1 = s_tot[1][kScanBlock - 1];
    const uint32_t M0 = s_totl[0][kScanBlock - 1], M1 = s_totl[1][kScanBlock - 1];
    __syncthreads();
    // last segments per (strand, step bucket): 16-bit fields, buckets 1|2 in s_tot, 3|4 in
    // s_totl (a block has <= 1024 views, so no field overflows)
    uint32_t bl[2] = {0u, 0u}, bh[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < VPT; ++e) {
        if (!bk[e]) continue;
        const uint32_t one = 1u << (16u * ((bk[e] - 1u) & 1u));
        if (bk[e] <= 2) bl[grp[e]] += one;
        else bh[grp[e]] += one;
    }
    s_tot[0][threadIdx.x] = bl[0];
    s_tot[1][threadIdx.x] = bl[1];
    s_totl[0][threadIdx.x] = bh[0];
    s_totl[1][threadIdx.x] = bh[1];
    __syncthreads();
    for (uint32_t d = 1; d < kScanBlock; d <<= 1) {
        uint32_t x0 = 0, x1 = 0, y0 = 0, y1 = 0;
        if (threadIdx.x >= d) {
            x0 = s_tot[0][threadIdx.x - d];
            x1 = s_tot[1][threadIdx.x - d];
            y0 = s_totl[0][threadIdx.x - d];
            y1 = s_totl[1][threadIdx.x - d];
        }
        __syncthreads();
        s_tot[0][threadIdx.x] += x0;
        s_tot[1][threadIdx.x] += x1;
        s_totl[0][threadIdx.x] += y0;
        s_totl[1][threadIdx.x] += y1;
        __syncthreads();
    }
    uint32_t LB[2][5];   // region base of each step bucket, LB[g][4] = the region's size
#pragma unroll
    for (int g = 0; g < 2; ++g) {
        const uint32_t lo = s_tot[g][kScanBlock - 1], hi = s_totl[g][kScanBlock - 1];
        LB[g][0] = 0;
        LB[g][1] = lo & 0xFFFFu;
        LB[g][2] = LB[g][1] + (lo >> 16);
        LB[g][3] = LB[g][2] + (hi & 0xFFFFu);
        LB[g][4] = LB[g][3] + (hi >> 16);
    }
    {
        uint32_t xl[2], xh[2];
#pragma unroll
        for (int g = 0; g < 2; ++g) {
            xl[g] = s_tot[g][threadIdx.x] - bl[g];
            xh[g] = s_totl[g][threadIdx.x] - bh[g];
        }
#pragma unroll
        for (int e = 0; e < VPT; ++e) {
            if (!bk[e]) continue;
            const int g = grp[e];
            const uint32_t b = bk[e] - 1u, sh = 16u * (b & 1u);
            uint32_t& x = b < 2 ? xl[g] : xh[g];
            s_lastv[g][LB[g][b] + ((x >> sh) & 0xFFFFu)] = (uint16_t)(threadIdx.x * VPT + e);
            x += 1u << sh;
        }
    }
    __syncthreads();
    const uint32_t T0 = F0 + M0 + LB[0][4], T1 = F1 + M1 + LB[1][4];
    const uint32_t wv = threadIdx.x >> 6;   // windows staged per wave: no block barriers below
    const uint32_t wsh = wave_shard();
    const WaveStage<Window, kWaveWinCap> st{s_win[wv], &s_wcnt[wv], R.win + wsh * R.win_scap,
                                            R.win_count + wsh * kShardStride, R.win_scap,
                                            R.flags, 4u};

    const bool front = P->where == kFront;
    const int kf_far = min(kf, (int)s_pf[71]);
    const uint32_t gap = (uint32_t)P->max_mk;
    const int rb = kCleanHist ? P->clean_reach : 0;   // clean flags for the exact stages
    // the block's rows sit in the top L bits (filter_peq, host side): rows start at cost i
    const uint32_t pv_rows = L >= 32 ? ~0u : ~0u << (32 - L);

    // With both orientations of every item (--rc) the two strand groups have equal segment
    // counts; then the block's two halves walk them in step (half 0: strand-0 segment tt, half
    // 1: strand-1 segment tt), so both strands of the same reads are loaded together and the
    // second load of each byte hits in L2 (strand-major order re-read it from the fabric:
    // 1.8x the algorithmic bytes).  The strand branch stays wave-uniform.
    const bool paired = T1 == T0 && F1 == F0 && M1 == M0 && LB[0][1] == LB[1][1] &&
                        LB[0][2] == LB[1][2] && LB[0][3] == LB[1][3] && T0 > 0;
    const uint32_t step = paired ? (uint32_t)kScanBlock / 2 : (uint32_t)kScanBlock;
    const uint32_t total = paired ? T0 : T0 + T1;
    for (uint32_t tb = 0; tb < total; tb += step) {
        int g;
        uint32_t tt;
        bool valid;
        if (paired) {
            g = threadIdx.x >= (uint32_t)kScanBlock / 2 ? 1 : 0;
            tt = tb + (threadIdx.x & ((uint32_t)kScanBlock / 2 - 1));
            valid = tt < T0;
        } else {
            const uint32_t t = tb + threadIdx.x;
            valid = t < T0 + T1;
            g = t < T0 ? 0 : 1;
            tt = g ? t - T0 : t;
        }
        if (valid) {
            // tasks [0, F_g): segment 0 of the views in order; then the later segments,
            // view-major.  The view is the last one whose prefix is <= the index (views of the
            // other strand, and views without such segments, add 0).
            const uint32_t Fg = g ? F1 : F0, Mg = g ? M1 : M0;
            uint32_t lo = 0, k;
            if (tt >= Fg + Mg) {                       // last segments, by step bucket
                lo = s_lastv[g][tt - Fg - Mg];
                k = 0xFFFFFFFFu;                       // (set from the view's length below)
            } else {
                const bool first = tt < Fg;
                const uint32_t x = first ? tt : tt - Fg;
                const uint32_t* pre = first ? s_pre[g] : s_prl[g];
                uint32_t hi = nv;                      // answer in [lo, hi)
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (pre[mid] <= x) lo = mid;
                    else hi = mid;
                }
                k = first ? 0u : 1u + (x - pre[lo]);
            }
            const uint32_t v = vbeg + lo;
            const uint32_t item = v / (uint32_t)no;
            const int o = (int)(v % (uint32_t)no);
            TaskView tv;
            task_view(R, item, o * A, A, tv);
            if (k == 0xFFFFFFFFu) k = (tv.len + SEG - 1) / SEG - 1u;
            const uint32_t seg0 = k * SEG;
            const uint32_t P0 = k ? seg0 - W : 0u;
            const uint32_t P1 = min(tv.len, seg0 + SEG);
            SegState S;
            const bool fresh = k == 0;                 // view start: the panel's own column 0
            S.pv = (fresh && front) ? 0u : pv_rows;
            S.mv = 0u;
            S.e = ((fresh && front) ? 0 : L) - (kf_far + 1);
            S.have = false;
            S.w1 = S.w2 = 0;
            S.wb = 255;
            filter_segment(R, tv, P0, P1, S, s_fpeq, s_thr, kf_far, gap, seg0, rb, st, item,
                           o);
            const uint32_t len = tv.len;
            if (!front && P1 == len) {
                // 3' panels: the last column (adapter prefix off the read end) is always checked
                if (S.have && len - S.w2 <= gap) {
                    st.push(make_window(item, o, tv, S.w1, len, 1, S.wb,
                                        window_clean(S, S.w1, len, rb)));
                } else {
                    if (S.have)
                        st.push(make_window(item, o, tv, S.w1, S.w2, 0, S.wb,
                                            window_clean(S, S.w1, S.w2, rb)));
                    st.push(make_window(item, o, tv, len, len, 1, 255,
                                        window_clean(S, len, len, rb)));
                }
                S.have = false;
            }
            if (S.have)
                st.push(make_window(item, o, tv, S.w1, S.w2, 0, S.wb,
                                    window_clean(S, S.w1, S.w2, rb)));
        }
        __builtin_amdgcn_wave_barrier();
        if (st.count() > kWaveWinCap / 2) st.flush();
    }
    __builtin_amdgcn_wave_barrier();
    st.flush();
}

// ---------------------------------------------------------------------------------------------
// Piece screen: one lane per (item, part) of the item's orientation-0 view.  The
// lane samples an 8-mer every S positions of the part's codes (view order) and looks it up in an
// LDS bitmap of the panel's sampled piece 8-mers (both orientations: a piece of orientation 1 is
// stored reverse complemented, so one pass over the read serves both views).  A hit is checked
// against every (piece, offset) entry of its 8-mer on the codes held in registers; an exact copy
// marks the 16-position cells of the view where an alignment containing it can end.  Runs of
// marked cells (gaps of <= 2 cells filled: a restricted start costs W warm-up positions anyway)
// become filter tasks; a 3' view's last-column window is emitted here unless a task reaches the
// view end (the task then emits it, merged with a nearby hit window, as the full filter does).
// A part owns the piece copies that START in it, so each copy is seen by exactly one lane.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kPsItemsPerBlock = 512;   // items per screen block step (2 per thread)
#ifndef DMX_PIECE_GRID
#define DMX_PIECE_GRID (256 * 4)
#endif
constexpr uint32_t kPieceGrid = DMX_PIECE_GRID;   // resident blocks (persistent grids)
#ifndef DMX_SCAN_GRID
#define DMX_SCAN_GRID (256 * 8)
#endif
constexpr uint32_t kScanGrid = DMX_SCAN_GRID;     // the flat scan: 8 waves per SIMD

__device__ __forceinline__ uint32_t ps_view_len(const RoundArgs& R, uint32_t item) {
    if (R.items) {
        if (!DMX_BOUND(R.pk.bd, items, item, kBufItem)) return 0u;
        return R.items[item].len;
    }
    if (!DMX_BOUND(R.pk.bd, reads, item, kBufRead)) return 0u;
    return R.lens[item];
}
// positions per part of a view of n positions (a multiple of 16, <= part_max) and the part count
__device__ __forceinline__ uint32_t ps_part_len(uint32_t n, uint32_t pmax) {
    const uint32_t np = (n + pmax - 1) / pmax;
    return np <= 1 ? ((n + 15u) & ~15u) : (((n + np - 1) / np + 15u) & ~15u);
}
__device__ __forceinline__ uint32_t ps_parts(uint32_t n, uint32_t pmax, bool front) {
    if (n == 0) return front ? 0u : 1u;   // an empty 3' view still gets its last-column window
    const uint32_t pl = ps_part_len(n, pmax);
    return (n + pl - 1) / pl;
}
// v[i] for a lane-varying i in [0, 4] (no indexed registers: a select chain)
__device__ __forceinline__ uint32_t sel5(uint32_t i, uint32_t v0, uint32_t v1, uint32_t v2,
                                         uint32_t v3, uint32_t v4) {
    uint32_t r = i == 4u ? v4 : v3;
    r = i == 2u ? v2 : r;
    r = i == 1u ? v1 : r;
    return i == 0u ? v0 : r;
}
// set cells [clo, chi] in a lane's 64-cell mask based at cell `base` (the host sizes parts so
// that every cell a part can mark fits; a violation sets flag bit 16 and is reported)
__device__ __forceinline__ void ps_mark(uint64_t& m, int base, int clo, int chi, uint32_t* flags) {
    const int d0 = clo - base, d1 = chi - base;
    if (d0 < 0 || d1 > 63) {
        atomicOr(flags, 16u);
        return;
    }
    m |= ((2ull << (d1 - d0)) - 1ull) << d0;   // d1 - d0 = 63: 2 << 63 wraps to 0, all ones
}
// Reserve this lane's `cnt` records of a sharded list with one global atomic per wave (every
// lane of the wave calls it at the same point); returns the lane's first index in the shard.
__device__ __forceinline__ uint32_t wave_reserve(uint32_t* gcount, uint32_t cnt) {
    const int lane = (int)(threadIdx.x & 63u);
    uint32_t x = cnt;   // inclusive scan over the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, (unsigned)d, 64);
        if (lane >= d) x += y;
    }
    const uint32_t total = __shfl(x, 63, 64);
    uint32_t base = 0;
    if (lane == 0 && total) base = atomicAdd(gcount, total);
    base = __shfl(base, 0, 64);
    return base + x - cnt;
}
// The filter tasks of marked cells in view order: runs of 16-position cells (cell u covers view
// positions [16u - delta, 16u - delta + 16), clipped to the view), cut into segments of at most
// kSegSpan positions with the W-position restricted-start warm-up before each (from the view
// start: the panel's own column 0, no warm-up).
struct PsRuns {
    uint64_t m;
    int base, delta, n, W, SEG, s, e;
    __device__ __forceinline__ bool next(FTask& ft, uint32_t item, int o) {
        while (s >= e) {
            if (!m) return false;
            const int u = (int)__builtin_ctzll((unsigned long long)m);
            const uint64_t r = ~(m >> u);
            const int run = r ? (int)__builtin_ctzll((unsigned long long)r) : 64 - u;
            m &= run >= 64 ? 0ull : ~(((1ull << run) - 1ull) << u);
            s = max(0, 16 * (base + u) - delta);
            e = min(n, 16 * (base + u + run) - delta);
        }
        const int ee = min(e, s + SEG);
        ft.item = item;
        if (s < W) {
            ft.p0 = 0;
            ft.span = (uint16_t)ee;
            ft.hoff = 0;
            ft.flags = (uint8_t)(o | 2);
        } else {
            ft.p0 = (uint32_t)(s - W);
            ft.span = (uint16_t)(ee - s + W);
            ft.hoff = (uint8_t)W;
            ft.flags = (uint8_t)o;
        }
        s = ee;
        return true;
    }
};
__device__ __forceinline__ void ftask_view(FTask& ft, const TaskView& tv) {
    ft.flags |= (uint8_t)((tv.strand & 1u) << 2);
    ft.n = tv.n;
    ft.start = tv.start;
    ft.len = tv.len;
    ft.off = tv.off;
}
// Write one view's filter tasks (two passes: count, one wave reservation, write); returns whether
// a task reaches the view end.  Every lane of the wave calls it.
__device__ __forceinline__ bool ps_emit(const RoundArgs& R, FTask* fbuf, uint32_t* fcnt,
                                        PsRuns rr, uint32_t item, int o, const TaskView& tv) {
    uint32_t cnt = 0;
    bool reached = false;
    {
        PsRuns c = rr;
        FTask ft;
        while (c.next(ft, item, o)) {
            ++cnt;
            reached |= (int)(ft.p0 + ft.span) == rr.n;
        }
    }
    uint32_t fi = wave_reserve(fcnt, cnt);
    FTask ft;
    while (rr.next(ft, item, o)) {
        ftask_view(ft, tv);
        if (fi < R.ftask_scap) fbuf[fi] = ft;
        else atomicOr(R.flags, 4u);
        ++fi;
    }
    return reached;
}
// A 3' view's standalone last-column window (no task reaches the view end), clean when the view
// holds no N in [n - rb, n) (what the exact stages read for it).  Every lane of the wave calls it.
__device__ __forceinline__ void ps_lastcol(const RoundArgs& R, Window* wbuf, uint32_t* wcnt,
                                           bool want, uint32_t item, int o, const TaskView& tv,
                                           int rb) {
    Window w;
    if (want) {
        const int n = (int)tv.len;
        bool clean = false;
        if (rb) {
            clean = true;
            for (int p = max(0, n - rb); p < n; p += 32) {
                uint32_t mk = mask32s(R.pk, tv, p);
                if (n - p < 32) mk &= (1u << (n - p)) - 1u;
                clean &= mk == 0u;
            }
        }
        w = make_window(item, o, tv, (uint32_t)n, (uint32_t)n, 1, 255, clean);
    }
    const uint32_t wi = wave_reserve(wcnt, want ? 1u : 0u);
    if (want) {
        if (wi < R.win_scap) wbuf[wi] = w;
        else atomicOr(R.flags, 4u);
    }
}

// The panel's piece tables -> LDS (dynamic: the fixed bitmap + rank base, then the keys and
// entries); returns the entry array.
struct PsTables {
    uint32_t* bm;
    uint16_t* rk;
    uint32_t* key;
    uint64_t* ent;
};
__device__ __forceinline__ PsTables ps_load_tables(const DevPieces* Q, uint8_t* dyn) {
    PsTables t;
    const int nk = Q->n_keys, ne = Q->n_entries;
    t.bm = reinterpret_cast<uint32_t*>(dyn);
    t.rk = reinterpret_cast<uint16_t*>(dyn + 4 * kPieceBitmapWords);
    t.key = reinterpret_cast<uint32_t*>(dyn + kPieceLdsFixed);
    t.ent = reinterpret_cast<uint64_t*>(dyn + kPieceLdsFixed + 8 * ((nk + 1) / 2));
    for (int x = threadIdx.x; x < kPieceBitmapWords; x += blockDim.x) {
        t.bm[x] = Q->bitmap[x];
        t.rk[x] = Q->rank_base[x];
    }
    for (int x = threadIdx.x; x < nk; x += blockDim.x) t.key[x] = Q->key[x];
    for (int x = threadIdx.x; x < ne; x += blockDim.x) t.ent[x] = Q->entry[x];
    return t;
}
// The entries of 8-mer K (which the bitmap holds): [first, first + count) of t.ent
__device__ __forceinline__ uint32_t ps_key(const PsTables& t, uint32_t K) {
    const uint32_t wi = K >> 5;
    const uint32_t rank = (uint32_t)t.rk[wi] + (uint32_t)__popc(t.bm[wi] & ((1u << (K & 31u)) - 1u));
    return t.key[rank];
}
// 8-mer lookups of one 64-position step: w0..w5 = positions [C - 16, C + 80), samples C + qS
template <int S>
__device__ __forceinline__ typename std::conditional<S == 1, uint64_t, uint32_t>::type
ps_lookups(const uint32_t* bm, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, uint32_t w4,
           uint32_t w5) {
    using HitT = typename std::conditional<S == 1, uint64_t, uint32_t>::type;
    HitT hits = 0;
#if defined(DMX_PS_AB) && DMX_PS_AB == 2   // timing A/B only (results invalid): no lookups
    asm volatile("" ::"v"(w0), "v"(w1), "v"(w2), "v"(w3), "v"(w4), "v"(w5));
#else
    const uint32_t wv6[6] = {w0, w1, w2, w3, w4, w5};
#pragma unroll
    for (int q = 0; q < 64 / S; ++q) {
        const int u = q * S + 16;
        const uint32_t K = align32(wv6[(u >> 4) + 1], wv6[u >> 4], 2u * (u & 15));
        const uint32_t word = bm[(K >> 5) & (uint32_t)(kPieceBitmapWords - 1)];
        hits |= (HitT)__builtin_amdgcn_ubfe(word, K & 31u, 1) << q;
    }
#endif
#if defined(DMX_PS_AB) && (DMX_PS_AB == 1 || DMX_PS_AB == 2)   // timing A/B: no checks
    asm volatile("" ::"v"(hits));
    hits = 0;
#endif
    return hits;
}

// ---------------------------------------------------------------------------------------------
// Per-part piece screen (any batch layout; the flat scan below takes sorted, non-overlapping
// batches): one lane per (item, part) of the item's orientation-0 view; the lane streams its
// part's codes, looks up the sampled 8-mers, checks hits against their (piece, offset) entries
// on the codes held in registers, and marks the 16-position cells of the view where an
// alignment containing a verified copy can end.  A part owns the copies that START in it.
// ---------------------------------------------------------------------------------------------
#ifndef DMX_PIECE_WAVES
#define DMX_PIECE_WAVES 1
#endif
template <int S>
__global__ __launch_bounds__(kScanBlock) __attribute__((amdgpu_waves_per_eu(DMX_PIECE_WAVES))) void pscreen_kernel(RoundArgs R) {
    static_assert(S == 1 || S == 2 || S == 4, "sampling stride: 64 positions per step");
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    __shared__ uint32_t s_pre[kPsItemsPerBlock + 1];
    __shared__ uint32_t s_sc[kScanBlock];
    const DevPieces* Q = R.pieces;
    const DevPanel* P = R.panel;
    const uint32_t tid = threadIdx.x;
    const PsTables tb_ = ps_load_tables(Q, s_dyn);
    const uint32_t n_items = R.items ? *R.n_items_dev : R.n_items;
    const bool front = P->where == kFront;
    const uint32_t pmax = (uint32_t)Q->part_max;
    const int A = P->n_adapters;
    const int no = P->n_orient;
    const uint32_t wsh = wave_shard();
    FTask* const fbuf = R.ftask + wsh * R.ftask_scap;
    uint32_t* const fcnt = R.ftask_count + wsh * kShardStride;
    Window* const wbuf = R.win + wsh * R.win_scap;
    uint32_t* const wcnt = R.win_count + wsh * kShardStride;
    const int W = P->scan_len + P->kf;
    const int SEG = kSegSpan - W;
    const int rb = kCleanHist ? P->clean_reach : 0;
    const int lo_off = Q->lo_off, dlo_min = Q->dlo_min;
    const int fcells = (Q->front_reach + 15) >> 4;

    for (uint32_t ib = blockIdx.x * kPsItemsPerBlock; ib < n_items;
         ib += gridDim.x * kPsItemsPerBlock) {            // block-uniform
        const uint32_t ni = min(n_items - ib, kPsItemsPerBlock);
        // parts per item, block-wide exclusive scan (2 items per thread)
        uint32_t c0 = 0, c1 = 0;
        if (2 * tid < ni) c0 = ps_parts(ps_view_len(R, ib + 2 * tid), pmax, front);
        if (2 * tid + 1 < ni) c1 = ps_parts(ps_view_len(R, ib + 2 * tid + 1), pmax, front);
        __syncthreads();   // the previous step's s_pre / s_sc readers (and the table copy)
        s_sc[tid] = c0 + c1;
        __syncthreads();
        for (uint32_t d = 1; d < kScanBlock; d <<= 1) {
            const uint32_t x = tid >= d ? s_sc[tid - d] : 0u;
            __syncthreads();
            s_sc[tid] += x;
            __syncthreads();
        }
        {
            const uint32_t ex = s_sc[tid] - c0 - c1;
            s_pre[2 * tid] = ex;
            s_pre[2 * tid + 1] = ex + c0;
        }
        __syncthreads();
        const uint32_t T = s_sc[kScanBlock - 1];

        for (uint32_t tb = 0; tb < T; tb += kScanBlock) {
            const uint32_t t = tb + tid;
            uint32_t item = 0;
            int n = 0, a = 0, b = 0;
            bool act = false;
            uint64_t m0 = 0, m1 = 0;
            int base0 = 0, base1 = 0;
            TaskView tv;
            if (t < T) {
                uint32_t lo = 0, hi = ni;              // the last item whose prefix is <= t
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (s_pre[mid] <= t) lo = mid;
                    else hi = mid;
                }
                item = ib + lo;
                const uint32_t part = t - s_pre[lo];
                act = task_view(R, item, 0, A, tv);
                n = (int)tv.len;
                const int pl = (int)ps_part_len((uint32_t)n, pmax);
                a = (int)part * pl;
                b = min(n, a + pl);
                base0 = a == 0 ? 0 : (a + lo_off) >> 4;
                base1 = b == n ? 0 : max(0, n - b + dlo_min) >> 4;
            }
            // stream the part: w0..w5 = view positions [a - 16 + 64k, a + 80 + 64k) in step k,
            // which samples x = a + 64k + q S: the 8-mer of positions [x, x + 8)
            const int xe = b + S - 1;                  // copies starting in [a, b) are sampled
            const int nsteps = (act && n > 0) ? (xe - a + 63) / 64 : 0;
            if (nsteps > 0) {
                uint32_t w0, w1, w2, w3, w4, w5, nb;
                fetch16s<false>(R.pk, tv, a - 16, w0, nb);
                fetch16s<false>(R.pk, tv, a, w1, nb);
                ViewBlocks<false> B;
                B.init(R, tv, a + 16);
                for (int k = 0; k < nsteps; ++k) {
                    uint32_t vc[4], vn[4];
                    B.extract(vc, vn, k + 2 < nsteps);
                    w2 = vc[0];
                    w3 = vc[1];
                    w4 = vc[2];
                    w5 = vc[3];
                    auto hits = ps_lookups<S>(tb_.bm, w0, w1, w2, w3, w4, w5);
                    using HitT = decltype(hits);
                    {
                        const int lim = xe - (a + 64 * k);     // sampled positions < xe
                        const int nq = lim >= 64 ? 64 / S : (lim <= 0 ? 0 : (lim + S - 1) / S);
                        if (nq < 64 / S) hits &= (HitT)((((HitT)1) << nq) - (HitT)1);
                    }
                    while (hits) {
                        const int q = (int)__builtin_ctzll((unsigned long long)hits);
                        hits &= hits - (HitT)1;
                        const int u = q * S + 16;
                        const int x = a + 64 * k + q * S;
                        const uint32_t ui = (uint32_t)u >> 4;
                        const uint32_t K = align32(sel5(ui, w1, w2, w3, w4, w5),
                                                   sel5(ui, w0, w1, w2, w3, w4),
                                                   2u * ((uint32_t)u & 15u)) & 0xFFFFu;
                        const uint32_t kr = ps_key(tb_, K);
                        const int e0 = (int)(kr & 0xFFFFu), e1 = e0 + (int)(kr >> 16);
                        for (int e = e0; e < e1; ++e) {
                            const uint64_t ev = tb_.ent[e];
                            const int len = (int)((ev >> 32) & 31u);
                            const int off = (int)((ev >> 38) & 3u);
                            const int g = x - off;
                            if (g < a || g >= b || g + len > n) continue;
                            const int ug = u - off;    // 14 .. 79
                            const uint32_t gi = (uint32_t)ug >> 4;
                            const uint32_t cw = align32(sel5(gi, w1, w2, w3, w4, w5),
                                                        sel5(gi, w0, w1, w2, w3, w4),
                                                        2u * ((uint32_t)ug & 15u));
                            const uint32_t msk = len >= 16 ? ~0u : ((1u << (2 * len)) - 1u);
                            if ((cw & msk) != (uint32_t)ev) continue;
                            const int dlo = (int)((ev >> 40) & 255u) - 128;
                            const int dhi = (int)((ev >> 48) & 255u) - 128;
                            const bool o1 = ((ev >> 37) & 1u) != 0;
                            // orientation 1: the copy sits at view-1 positions [n - g - len,
                            // n - g), so its alignment ends at view-1 column n - g + d
                            const int pe = o1 ? n - g : g + len;
                            const int plo = max(pe + dlo - 1, 0), phi = min(pe + dhi - 1, n - 1);
                            if (plo > phi) continue;
                            if (o1) ps_mark(m1, base1, plo >> 4, phi >> 4, R.flags);
                            else ps_mark(m0, base0, plo >> 4, phi >> 4, R.flags);
                        }
                    }
                    w0 = w4;
                    w1 = w5;
                }
            }
            // filter tasks per orientation; a 3' view's last-column window unless a task of this
            // lane reaches the view end (that task emits it, merged as the full filter does)
            for (int o = 0; o < no; ++o) {
                PsRuns rr{0ull, o ? base1 : base0, 0, n, W, SEG, 0, 0};
                bool last = false;
                TaskView tvo = tv;
                if (act) {
                    uint64_t m = o ? m1 : m0;
                    const bool at_start = o == 0 ? a == 0 : b == n;   // holds view position 0
                    last = !front && (o == 0 ? b == n : a == 0);      // ... the view's end
                    if (front && at_start && n > 0)    // partial alignments from column 0
                        ps_mark(m, rr.base, 0, min(fcells, (n + 15) >> 4) - 1, R.flags);
                    const int ncell = ((n + 15) >> 4) - rr.base;      // cells inside the view
                    if (ncell < 64) m &= ncell <= 0 ? 0ull : ((1ull << ncell) - 1ull);
                    m |= ((m << 1) & (m >> 1)) | ((m << 1) & (m >> 2)) | ((m << 2) & (m >> 1));
                    rr.m = m;
                    if (o) task_view(R, item, A, A, tvo);
                }
                const bool reached = ps_emit(R, fbuf, fcnt, rr, item, o, tvo);
                ps_lastcol(R, wbuf, wcnt, last && !reached, item, o, tvo, rb);
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Flat piece scan: once per exec, waves stride over 4096-nt superblocks of the
// packed batch, lane l takes nt [4096 b + 64 l, + 64) with one 16-B load (neighbours' words by lane
// shuffles), so every lane does the same work and the loads are coalesced.  The table is the
// combined table of every flat round.  The superblock's words are also kept in LDS; its sampled
// 8-mer hits are numbered lane by lane (a wave prefix sum) and checked 64 at a time, one per lane:
// the copy against each entry of the 8-mer (codes from LDS), then the nt where an alignment
// containing the copy can end are marked in the cell bitmap of the entry's round and copy strand
// (global atomics).  A lane's hits take adjacent check lanes, so the pieces of one adapter copy,
// which mark the same cells, sit side by side: a mark its left neighbour already makes is
// dropped.  No read or view is looked up: the marks are positions of the batch, and
// pcompact_kernel reads each view's own range of them.
// ---------------------------------------------------------------------------------------------
constexpr int kSbWords = kSuperNt / 16 + 8;   // LDS copy of a superblock: 4 words before, 4 after

// Check one sampled 8-mer (batch nt X; cw = codes of nt [X - 3, X + 29)) against its entries and
// mark cells.  A copy of a strand-0 piece at nt [x, x + len) ends alignments of a strand-0 view at
// nt x + len - 1 + [dlo, dhi]; a copy of a strand-1 piece (the reverse complement) ends them, in a
// strand-1 view that walks the batch backwards, at nt x - [dlo, dhi].  Every lane of the wave
// calls it (valid: the lane holds a hit).
// The four cell bitmaps' pointers held in scalar registers: readfirstlane keeps the compiler from
// turning a per-lane select between them back into a per-lane load of RoundArgs::cells.
typedef __attribute__((address_space(1))) uint32_t gu32;   // a global-memory word
struct CellPtrs {
    gu32* p[4];   // (global address space: a generic pointer would load through flat)
    __device__ __forceinline__ explicit CellPtrs(const RoundArgs& R) {
#pragma unroll
        for (int i = 0; i < 4; ++i) p[i] = sgpr_ptr(R.cells[i]);
    }
};

__device__ __forceinline__ void flat_check(const RoundArgs& R, const CellPtrs& cp,
                                           const PsTables& tb, uint64_t cw, uint64_t X,
                                           bool valid) {
    gu32* p1 = nullptr;       // the lane's first mark (deduplicated against the left lane's)
    uint32_t b1 = 0;
    if (valid) {
        const uint32_t kr = ps_key(tb, (uint32_t)(cw >> 6) & 0xFFFFu);
        const int64_t last = (int64_t)R.n_words * 16 - 1;
        const int e0 = (int)(kr & 0xFFFFu), e1 = e0 + (int)(kr >> 16);
        for (int e = e0; e < e1; ++e) {
            const uint64_t ev = tb.ent[e];
            const int len = (int)((ev >> 32) & 31u);
            const int off = (int)((ev >> 38) & 3u);
            const uint32_t msk = len >= 16 ? ~0u : ((1u << (2 * len)) - 1u);
            if (((uint32_t)(cw >> (2 * (3 - off))) & msk) != (uint32_t)ev) continue;
            const int tau = (int)((ev >> 37) & 1u);   // 1: the adapter reads reverse complemented
            const int dlo = (int)((ev >> 40) & 255u) - 128;
            const int dhi = (int)((ev >> 48) & 255u) - 128;
            const int64_t x = (int64_t)X - off;       // the copy's first nt
            int64_t nlo = tau ? x - dhi : x + len + dlo - 1;
            int64_t nhi = tau ? x - dlo : x + len + dhi - 1;
            nlo = nlo < 0 ? 0 : nlo;
            nhi = nhi > last ? last : nhi;
            if (nlo > nhi) continue;
            // the entry's round and strand pick one of four uniform pointers (indexing R.cells
            // by a lane's value is a dependent load of the kernel argument)
            const int ci = 2 * (int)((ev >> 56) & 1u) + tau;
            gu32* cells = ci < 2 ? (ci == 0 ? cp.p[0] : cp.p[1]) : (ci == 2 ? cp.p[2] : cp.p[3]);
            for (int64_t c = nlo >> 4; c <= (nhi >> 4);) {   // one atomic per bitmap word
                const int64_t w = c >> 5;
                const int64_t cend = min(nhi >> 4, (w << 5) + 31);
                const uint32_t bits = (uint32_t)((((2ull << (cend - c)) - 1ull)) << (c & 31));
                if (!p1) {
                    p1 = cells + w;
                    b1 = bits;
                } else {
#if defined(DMX_PS_AB) && DMX_PS_AB == 3   // timing A/B only: no marks
                    asm volatile("" ::"v"(bits), "v"(cells + w));
#else
                    __hip_atomic_fetch_or(cells + w, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
                }
                c = cend + 1;
            }
        }
    }
    const uint64_t pa = (uint64_t)p1;
    const uint64_t pl = ((uint64_t)__shfl_up((uint32_t)(pa >> 32), 1u, 64) << 32) |
                        (uint64_t)__shfl_up((uint32_t)pa, 1u, 64);
    const uint32_t bl = __shfl_up(b1, 1u, 64);
    const bool dup = (threadIdx.x & 63u) != 0u && pl == pa && (bl & b1) == b1;
    if (p1 && !dup) {
#if defined(DMX_PS_AB) && DMX_PS_AB == 3
        asm volatile("" ::"v"(b1), "v"(p1));
#else
        __hip_atomic_fetch_or(p1, b1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#endif
    }
}

template <int S>
__global__ __launch_bounds__(kScanBlock) void pscan_kernel(RoundArgs R) {
    static_assert(S == 1 || S == 2 || S == 4, "sampling stride: 64 positions per step");
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    __shared__ __attribute__((aligned(16))) uint32_t s_sb[kScanBlock / 64][kSbWords];
    __shared__ uint16_t s_q[kScanBlock / 64][64];
    const PsTables tb = ps_load_tables(R.pieces, s_dyn);
    __syncthreads();
    const CellPtrs cp(R);
    const int lane = (int)(threadIdx.x & 63u);
    uint32_t* const sbw = s_sb[threadIdx.x >> 6];   // [4 + k]: word k of the superblock
    uint16_t* const q = s_q[threadIdx.x >> 6];
    const uint4* sp = reinterpret_cast<const uint4*>(R.pk.seq);
    const uint32_t nw = gridDim.x * (kScanBlock / 64);
    for (uint32_t sb = blockIdx.x * (kScanBlock / 64) + (threadIdx.x >> 6); sb < R.nsb; sb += nw) {
        const int64_t wd = (int64_t)sb * (kSuperNt / 16) + 4 * lane;   // the lane's first word
        const bool live = wd < (int64_t)R.n_words;
        uint4 c = {0u, 0u, 0u, 0u};
        if (live) c = sp[wd >> 2];
        uint32_t w0 = __shfl_up(c.w, 1u, 64), w5 = __shfl_down(c.x, 1u, 64);
        if (lane == 0) w0 = R.pk.seq[wd - 1];         // (the device guard covers word -1)
        if (lane == 63) w5 = live ? R.pk.seq[wd + 4] : 0u;
        auto hits = ps_lookups<S>(tb.bm, w0, c.x, c.y, c.z, c.w, w5);
        using HitT = decltype(hits);
        if (!live) hits = 0;
        reinterpret_cast<uint4*>(sbw)[1 + lane] = c;
        if (lane == 0) sbw[3] = w0;
        if (lane == 63) {
            sbw[kSbWords - 4] = w5;
            sbw[kSbWords - 3] = 0u;
            sbw[kSbWords - 2] = 0u;
            sbw[kSbWords - 1] = 0u;
        }
        uint32_t total;
        uint32_t idx = wave_excl_scan((uint32_t)__popcll((unsigned long long)hits), total);
        const uint64_t C0 = (uint64_t)sb * kSuperNt;
        for (uint32_t base = 0; base < total; base += 64) {   // wave-uniform
            while (hits && idx < base + 64u) {                 // this lane's hits, in order
                const int qq = (int)__builtin_ctzll((unsigned long long)hits);
                hits &= hits - (HitT)1;
                q[idx - base] = (uint16_t)(lane * 64 + qq * S);
                ++idx;
            }
            __builtin_amdgcn_wave_barrier();
            const bool v = (uint32_t)lane < total - base;
            const uint32_t p = v ? q[lane] : 0u;
            // codes of nt [p - 3, p + 29) of the superblock: LDS words 4 + floor((p - 3) / 16) ..
            const uint32_t t = p + 61u;
            const uint32_t wi = t >> 4, sh = 2u * (t & 15u);
            const uint64_t lo = ((uint64_t)sbw[wi + 1] << 32) | sbw[wi];
            const uint64_t cw = sh ? (lo >> sh) | ((uint64_t)sbw[wi + 2] << (64u - sh)) : lo;
#if defined(DMX_PS_AB) && DMX_PS_AB == 4   // timing A/B only: queue without checks
            asm volatile("" ::"v"(cw));
#else
            flat_check(R, cp, tb, cw, C0 + p, v);
#endif
            __builtin_amdgcn_wave_barrier();
        }
    }
}

// Flat scan -> filter tasks: one lane per item; per orientation the view's cells in view order
// (cell u covers view positions [16u - delta, +16)), plus a FRONT panel's partial-alignment cells
// at the view start; a 3' view's last-column window unless a task reaches the view end.
__global__ __launch_bounds__(kScanBlock) void pcompact_kernel(RoundArgs R) {
    const DevPanel* P = R.panel;
    const DevPieces* Q = R.pieces;
    const uint32_t n_items = R.items ? *R.n_items_dev : R.n_items;
    const bool front = P->where == kFront;
    const int A = P->n_adapters;
    const int no = P->n_orient;
    const int W = P->scan_len + P->kf;
    const int SEG = kSegSpan - W;
    const int rb = kCleanHist ? P->clean_reach : 0;
    const int fr = Q->front_reach;
    const uint32_t wsh = wave_shard();
    FTask* const fbuf = R.ftask + wsh * R.ftask_scap;
    uint32_t* const fcnt = R.ftask_count + wsh * kShardStride;
    Window* const wbuf = R.win + wsh * R.win_scap;
    uint32_t* const wcnt = R.win_count + wsh * kShardStride;
    const uint32_t stride = gridDim.x * blockDim.x;
    // Cells [k0, k0 + 64) of a view in view order come from three bitmap words.  They are
    // loaded with no branch on the strand and finished where they are used, so the loads of
    // both orientations' first 64 cells, and of a view's next 64 cells, are in flight together
    // instead of one round trip each.  The bitmap of the lane's strand is a select between
    // two uniform pointers (indexing R.cells by the lane's strand is a dependent global load).
    const CellPtrs cp(R);
    const gu32* const cb0 = cp.p[2 * R.round];
    const gu32* const cb1 = cp.p[2 * R.round + 1];
    struct View {
        TaskView tv;
        int64_t p0nt = 0;   // nt of view position 0
        int delta = 0, ncell = 0, l = 0;
        uint3 w = {0u, 0u, 0u};
    };
    const auto words = [&](const View& v, int k0, uint3& wv) __attribute__((always_inline)) {
        const int64_t c0 = v.p0nt >> 4;
        const int64_t cs = v.tv.strand ? c0 - k0 - 63 : c0 + k0;   // lowest cell
        const gu32* cb = v.tv.strand ? cb1 : cb0;
        // unconditional (word 0 when the cells are not needed: inside the bitmap's guard), so
        // no merge with a default value waits for the load where it is issued
        const int64_t w = k0 < v.ncell ? cs >> 5 : 0;              // floor
        wv.x = cb[w];
        wv.y = cb[w + 1];
        wv.z = cb[w + 2];
    };
    const auto prep = [&](uint32_t item, bool act, int o, View& v) __attribute__((always_inline)) {
        if (act) {
            task_view(R, item, o * A, A, v.tv);
            v.l = (int)v.tv.len;
        }
        // nt of view position 0 and the walk direction through the cells
        v.p0nt = v.tv.strand ? (int64_t)v.tv.off + v.tv.n - 1 - v.tv.start
                             : (int64_t)v.tv.off + v.tv.start;
        v.delta = act ? (v.tv.strand ? 15 - (int)(v.p0nt & 15) : (int)(v.p0nt & 15)) : 0;
        v.ncell = act && v.l > 0 ? (v.l + v.delta + 15) >> 4 : 0;   // cells of the view
        words(v, 0, v.w);
    };
    const auto run = [&](uint32_t item, bool act, int o, const View& v) __attribute__((always_inline)) {
        bool reached = false;
        uint3 cur = v.w;
        for (int k0 = 0; __ballot(k0 < v.ncell); k0 += 64) {
            uint3 nx = {0u, 0u, 0u};
            words(v, k0 + 64, nx);                                 // the next 64 cells, in flight
            uint64_t m = 0;
            if (k0 < v.ncell) {
                // cells k0 .. k0 + 63 in view order = bitmap cells c0 + u (strand 0) or
                // c0 - u (strand 1), c0 = the cell of view position 0
                const int64_t c0 = v.p0nt >> 4;
                const int64_t cs = v.tv.strand ? c0 - k0 - 63 : c0 + k0;   // lowest cell
                const uint32_t sh = (uint32_t)(cs & 31);
                const uint64_t lo = ((uint64_t)cur.y << 32) | cur.x;
                const uint64_t x = sh ? (lo >> sh) | ((uint64_t)cur.z << (64 - sh)) : lo;
                m = v.tv.strand ? __builtin_bitreverse64(x) : x;
                if (front && k0 == 0)               // partial alignments from column 0
                    m |= (fr + v.delta + 15) >> 4 >= 64 ? ~0ull
                                                        : ((1ull << ((fr + v.delta + 15) >> 4)) - 1ull);
                const int left = v.ncell - k0;
                if (left < 64) m &= (1ull << left) - 1ull;
                m |= ((m << 1) & (m >> 1)) | ((m << 1) & (m >> 2)) | ((m << 2) & (m >> 1));
            }
            PsRuns rr{m, k0, v.delta, v.l, W, SEG, 0, 0};
            reached |= ps_emit(R, fbuf, fcnt, rr, item, o, v.tv);
            cur = nx;
        }
        ps_lastcol(R, wbuf, wcnt, act && !front && !reached, item, o, v.tv, rb);
    };
    for (uint32_t i0 = blockIdx.x * blockDim.x; i0 < n_items; i0 += stride) {   // wave-uniform
        const uint32_t item = i0 + threadIdx.x;
        const bool act = item < n_items;
        View v0, v1;   // (no branch on `no`: a merge there made the first loads wait)
        v0.tv.strand = v1.tv.strand = 0;
        const bool act1 = act && no > 1;
        prep(item, act, 0, v0);
        prep(item, act1, 1, v1);
        run(item, act, 0, v0);
        run(item, act1, 1, v1);
    }
}

// The shared-suffix filter over the piece screen's tasks: one lane per task, the same segment
// scan, windows and last-column rule as filter_kernel (a task is a segment of at most kSegSpan
// positions; tasks of one view never report the same column twice).
__global__ __launch_bounds__(kScanBlock) __attribute__((amdgpu_waves_per_eu(DMX_FILTER_WAVES))) void ftask_kernel(RoundArgs R) {
    __shared__ uint32_t s_fpeq[8];
    __shared__ __attribute__((aligned(16))) int8_t s_thr[kScanBlock];
    __shared__ Window s_win[kScanBlock / 64][kWaveWinCap];
    __shared__ uint32_t s_wcnt[kScanBlock / 64];
    __shared__ uint32_t s_spre[kShards + 1];
    const DevPanel* P = R.panel;
    const int L = P->scan_len;
    const int kf = P->kf;
    if (threadIdx.x < 8) s_fpeq[threadIdx.x] = P->filter_peq[threadIdx.x];
    if (threadIdx.x < kScanBlock / 64) s_wcnt[threadIdx.x] = 0;
    {   // per-column hit thresholds near the view start (filter_kernel)
        const int far0 = min((int)P->kf, (int)P->pf[71]);
        const int j = (int)threadIdx.x + 1;
        int t = -1;
        for (int d = 0; d <= far0; ++d)
            if (d <= (int)P->pf[min(j + d, 71)]) t = d;
        s_thr[threadIdx.x] = (int8_t)t;
    }
    ShardMap sm{s_spre, 0u};
    sm.load(R.ftask_count, R.ftask_scap);              // (its barrier covers the above)
    const uint32_t total = sm.total();
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t wsh = wave_shard();
    const WaveStage<Window, kWaveWinCap> st{s_win[wv], &s_wcnt[wv], R.win + wsh * R.win_scap,
                                            R.win_count + wsh * kShardStride, R.win_scap,
                                            R.flags, 4u};
    const bool front = P->where == kFront;
    const int kf_far = min(kf, (int)P->pf[71]);
    const uint32_t gap = (uint32_t)P->max_mk;
    const int rb = kCleanHist ? P->clean_reach : 0;
    const uint32_t pv_rows = L >= 32 ? ~0u : ~0u << (32 - L);
    for (uint32_t tb = blockIdx.x * kScanBlock; tb < total; tb += gridDim.x * kScanBlock) {
        const uint32_t ti = tb + threadIdx.x;
        if (ti < total) {
            const FTask ft = R.ftask[sm.phys(ti)];
            const int o = ft.flags & 1;
            const bool fresh = (ft.flags & 2) != 0;
            TaskView tv;
            tv.read = 0;
            tv.n = ft.n;
            tv.start = ft.start;
            tv.len = ft.len;
            tv.strand = (ft.flags >> 2) & 1u;
            tv.off = ft.off;
            tv.o = o;
            tv.a = 0;
            const uint32_t P0 = ft.p0;
            const uint32_t P1 = min(tv.len, P0 + (uint32_t)ft.span);
            const uint32_t hit_from = fresh ? 0u : P0 + ft.hoff;
            SegState S;
            S.pv = (fresh && front) ? 0u : pv_rows;
            S.mv = 0u;
            S.e = ((fresh && front) ? 0 : L) - (kf_far + 1);
            S.have = false;
            S.w1 = S.w2 = 0;
            S.wb = 255;
            filter_segment(R, tv, P0, P1, S, s_fpeq, s_thr, kf_far, gap, hit_from, rb, st,
                           ft.item, o);
            const uint32_t len = tv.len;
            if (!front && P1 == len) {   // the last column, merged with a nearby hit window
                if (S.have && len - S.w2 <= gap) {
                    st.push(make_window(ft.item, o, tv, S.w1, len, 1, S.wb,
                                        window_clean(S, S.w1, len, rb)));
                } else {
                    if (S.have)
                        st.push(make_window(ft.item, o, tv, S.w1, S.w2, 0, S.wb,
                                            window_clean(S, S.w1, S.w2, rb)));
                    st.push(make_window(ft.item, o, tv, len, len, 1, 255,
                                        window_clean(S, len, len, rb)));
                }
                S.have = false;
            }
            if (S.have)
                st.push(make_window(ft.item, o, tv, S.w1, S.w2, 0, S.wb,
                                    window_clean(S, S.w1, S.w2, rb)));
        }
        __builtin_amdgcn_wave_barrier();
        if (st.count() > kWaveWinCap / 2) st.flush();
    }
    __builtin_amdgcn_wave_barrier();
    st.flush();
}

// ---------------------------------------------------------------------------------------------
// verify: one lane per filter window; 32-bit Myers of the shared PREFIX block over the columns
// where the prefix of an alignment ending in the window would end.  Keeps the window only if
//   (rows) some full alignment ending in [j1, j2] could cost <= kf: bmin + min D_pre <= kf
//          (FRONT windows near the read start may hold partial alignments: always kept), or
//   (end)  3' last-column cells: an adapter prefix of length i at the read end costs
//          D_pre(i, len) for i < pre_len, or contains the whole prefix block ending within
//          m_max - 1 - pre_len + kf columns of the end.
// Survivors are compacted into the second window list for the window scan.
// ---------------------------------------------------------------------------------------------
#ifndef DMX_SORT_GROUP
#define DMX_SORT_GROUP 2048
#endif
constexpr int kSortGroup = DMX_SORT_GROUP;   // tasks ordered by length per block step
constexpr int kSortBins = 64;                // counting-sort bins of 4 columns (last: >= 252)
constexpr int kSortShift = 2;
static_assert(kSortGroup % kScanBlock == 0, "sort group");

#ifndef DMX_VERIFY_WAVES
#define DMX_VERIFY_WAVES 1   // occupancy floor (1: the compiler's choice, 5 waves at 96 VGPRs)
#endif
__global__ __launch_bounds__(kScanBlock) __attribute__((amdgpu_waves_per_eu(DMX_VERIFY_WAVES))) void verify_kernel(RoundArgs R) {
    __shared__ Window s_w[kStageCap];
    __shared__ uint32_t s_wc, s_wb;
    __shared__ int8_t s_pf[72];
    __shared__ uint32_t s_ppeq[8];
    if (threadIdx.x == 0) s_wc = 0;
    const DevPanel* P = R.panel;
    if (threadIdx.x < 72) s_pf[threadIdx.x] = P->pf[threadIdx.x];
    if (threadIdx.x < 8) s_ppeq[threadIdx.x] = P->pre_peq[threadIdx.x];
    __shared__ uint32_t s_spre[kShards + 1];
    ShardMap sm{s_spre, 0u};
    sm.load(R.win_count, R.win_scap);                  // (its barrier covers the above)
    const uint32_t bsh = blockIdx.x & (uint32_t)(kShards - 1);
    const Stage<Window> st{s_w, &s_wc, &s_wb, R.win2 + bsh * R.win_scap,
                           R.win2_count + bsh * kShardStride,
                           R.win_scap, R.flags, 4u};
    const bool front = P->where == kFront;
    const int L = P->pre_len, kf = P->kf;
    const uint32_t total = sm.total();
    // FRONT panels: a wave costs its widest window (filter windows are ~11 columns wide, a few
    // over 100), so each block takes kSortGroup consecutive windows at a time and runs them in
    // order of their column range, as the screen and the window scan do.
#ifndef DMX_VERIFY_SORT
#define DMX_VERIFY_SORT 1
#endif
#ifndef DMX_VERIFY_PREFETCH
#define DMX_VERIFY_PREFETCH 0
#endif
    const bool sorted = DMX_VERIFY_SORT && front;
    __shared__ uint32_t s_ord[kSortGroup];
    __shared__ uint32_t s_bin[kSortBins];
    for (uint32_t gb = blockIdx.x * kSortGroup; gb < total; gb += gridDim.x * kSortGroup) {
      const uint32_t gn = min((uint32_t)kSortGroup, total - gb);
      if (sorted) {   // block-uniform
        if (threadIdx.x < kSortBins) s_bin[threadIdx.x] = 0;
        __syncthreads();                           // (also: the last group's s_ord)
        constexpr int PER = kSortGroup / kScanBlock;
        uint32_t key[PER], pos[PER];
        // every record's fields first (unconditional loads, clamped index: all in flight at
        // once), then the bin counts
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            const uint32_t li = threadIdx.x + (uint32_t)e * kScanBlock;
            const Window* w = R.win + sm.phys(gb + min(li, gn - 1u));
            const int span = (int)w->j2 - (int)w->j1;   // the rows range grows with it
            key[e] = (uint32_t)min(max(span, 0) >> kSortShift, kSortBins - 1);
        }
#pragma unroll
        for (int e = 0; e < PER; ++e)
            if (threadIdx.x + (uint32_t)e * kScanBlock < gn) pos[e] = atomicAdd(&s_bin[key[e]], 1u);
        __syncthreads();
        if (threadIdx.x == 0) {                    // exclusive scan over the bins
            uint32_t acc = 0;
            for (int b = 0; b < kSortBins; ++b) {
                const uint32_t c = s_bin[b];
                s_bin[b] = acc;
                acc += c;
            }
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            const uint32_t li = threadIdx.x + (uint32_t)e * kScanBlock;
            if (li < gn) s_ord[s_bin[key[e]] + pos[e]] = li;
        }
        __syncthreads();
      }
      // DMX_VERIFY_PREFETCH (A/B, off): the next stride's window record is loaded before this
      // stride's scan.  Measured slower: 108 VGPRs drop verify to 4 waves, and forcing 5 spills
      // (verify 1.39 / 1.44 -> 1.47 / 1.51 ms, profiles/r5_ab_verify_prefetch.txt)
      Window wn{};
      if (DMX_VERIFY_PREFETCH && threadIdx.x < gn)
          wn = R.win[sm.phys(gb + (sorted ? s_ord[threadIdx.x] : threadIdx.x))];
      for (uint32_t sb = 0; sb < gn; sb += kScanBlock) {   // block-uniform
        const uint32_t li = sb + threadIdx.x;
        Window wcur{};
        if (DMX_VERIFY_PREFETCH) {
            wcur = wn;
            const uint32_t ln = li + kScanBlock;
            if (ln < gn) wn = R.win[sm.phys(gb + (sorted ? s_ord[ln] : ln))];
        }
        if (li < gn) {
            Window w = DMX_VERIFY_PREFETCH ? wcur : R.win[sm.phys(gb + (sorted ? s_ord[li] : li))];
            const int len = (int)w.len;
            const bool rows_free = (front && (int)w.j1 <= P->max_mk) || w.bmin == 255;
            // column ranges the prefix block must be evaluated on
            int lo = 1 << 30, hi = -1;
            if (!rows_free) {
                lo = (int)w.j1 - P->off_max - kf;
                hi = (int)w.j2 - P->off_min + kf;
            }
            const int end_lo = len - (P->m_max - 1 - L + kf);
            if (w.lastcol) {
                lo = min(lo, end_lo);
                hi = len;
            }
            bool keep = rows_free && w.bmin != 255;    // near-start FRONT window: keep as is
            uint32_t info = 0;                         // Window.info for the index screen
            if (!keep && hi >= 0) {
                lo = max(lo, 0);
                hi = min(hi, len);
                TaskView tv;
                tv.read = 0;
                tv.n = w.n;
                tv.strand = w.strand & 1u;
                tv.start = w.start;
                tv.len = w.len;
                view_off(R.pk, w.off, tv);
                tv.o = w.o;
                tv.a = 0;
                int js = lo - L - kf - 1;              // restricted start: exact from lo on
                if (js < 0) js = 0;
                uint32_t pv = ~0u, mv = 0u;
                int d = L;
                int dmin_rows = 1 << 20, dmin_end = 1 << 20, dmin_near = 1 << 20;
                // P ending this close to the end: 3' cells holding P and part of an index block
                const int near_lo = len - (P->m_max - P->filter_len - L - 1) - kf;
                const uint32_t hbit = (uint32_t)(L - 1);
                const int rlo = w.bmin == 255 ? (1 << 30) : (int)w.j1 - P->off_max - kf;
                const int rhi = (int)w.j2 - P->off_min + kf;
                if (js == 0) {   // column 0 itself (3' panels: D(L, 0) = L)
                    if (rlo <= 0 && rhi >= 0) dmin_rows = L;
                    if (end_lo <= 0) dmin_end = L;
                    if (near_lo <= 0) dmin_near = L;
                }
                // the columns js + 1 .. hi as 64-position stretches of whole aligned blocks
                // (one lane per window: the block loads are scattered, so few and wide)
                const int nst = (hi - js + 63) >> 6;
                ViewBlocks<kNecessaryMask> vb;   // N read as A: a lower bound of D_pre
                if (nst > 0) vb.init(R, tv, js);
                for (int st_i = 0; st_i < nst; ++st_i) {
                    uint32_t vc[4], vn[4];
                    vb.extract(vc, vn, st_i + 2 < nst);
#pragma unroll
                    for (int ch = 0; ch < 4; ++ch) {
                        const int p0 = js + 64 * st_i + 16 * ch;
                        const int cnt = min(16, hi - p0);
                        if (cnt <= 0) break;
                        const uint32_t codes = vc[ch], nb = vn[ch];
                        for (int q = 0; q < cnt; ++q) {
                            const uint32_t code = ((codes >> (2 * q)) & 3u) |
                                                  (((nb >> q) & 1u) << 2);
                            myers_step32(s_ppeq[code], pv, mv, d, hbit);
                            const int j = p0 + q + 1;
                            if (j >= rlo && j <= rhi) dmin_rows = min(dmin_rows, d);
                            if (j >= end_lo) dmin_end = min(dmin_end, d);
                            if (j >= near_lo) dmin_near = min(dmin_near, d);
                        }
                    }
                }
                if (!rows_free && (int)w.bmin + dmin_rows <= kf) keep = true;
                // Index-screen bounds of the prefix block's cost: the restricted start is exact
                // where D_pre <= kf and never lowers D, so min(dmin, kf + 1) is a lower bound of
                // the true minimum as far as any test against a threshold <= kf can tell.
                if (!rows_free) info = (uint32_t)min(dmin_rows, kf + 1);
                if (w.lastcol) {
                    if (dmin_end <= kf) keep = true;                  // whole prefix block at end
                    info |= (uint32_t)min(dmin_end, kf + 1) << 8;      // P ending near the end
                    info |= (uint32_t)min(dmin_near, kf + 1) << 24;    // ... within l_max + kf
                    int dd = 0;                                       // prefix cells at column len
                    bool pcell = false;
                    for (int i = 1; i <= L; ++i) {
                        dd += (int)((pv >> (i - 1)) & 1u) - (int)((mv >> (i - 1)) & 1u);
                        pcell |= dd <= (int)s_pf[i];
                    }
                    if (pcell || hi == 0) {                           // (hi == 0: empty view)
                        keep = true;
                        info |= 1u << 16;
                    }
                }
            }
            w.info = info;
            if (keep) st.push(w);
        }
        if (stage_count(&s_wc) > kStageCap / 2) st.flush();
      }
    }
    st.flush();
}

// ---------------------------------------------------------------------------------------------
// index screen (between verify and the window scan).  Every adapter of a filtered
// + verified panel is P + I_a + S: the shared prefix P (pre_len rows), its own index block I_a
// (l_a = m_a - pre_len - filter_len rows, 1..32) and the shared suffix S.  Splitting an alignment
// at the block boundaries splits its cost: c_P + c_I + c_S <= d, where the I_a band is an
// alignment of all of I_a ending at some column x2 with |j - x2 - |S|| <= c_S <= kf.
//   last-row cells (m, j): c_S >= bmin (the filter's block cost at every hit column of the
//     window), c_P >= the verify's prefix bound, so D_I(l_a, x2) <= kk_a - bmin - c_P for some
//     x2 in [j1 - |S| - kf, j2 - |S| + kf].  FRONT cells at j < jsplit may skip rows of I_a at
//     column 0: that part of a window (the "near piece") keeps every adapter.
//   3' last-column cells (i, len): i <= pre_len is identical for every adapter (only the first
//     adapter needs it when the acceptance tables agree); otherwise P ends within
//     m_max - 1 - pre_len + kf columns of the end, at cost >= dPe (verify), and
//     pre_len < i < pre_len + l_a needs dPn + D_I(i - pre_len, len) <= acc_a[i] (dPn: P ending
//     within l_max - 1 + kf columns of the end);
//     i >= pre_len + l_a needs dPe + D_I(l_a, x2) <= kk_a for some x2 in [len - |S| + 1 - kf, len].
// D_I is the 32-bit Myers of I_a alone with a free start in the read, started l_a + kk_a + 1
// columns before the first column of interest with D(i) = i: exact wherever D <= kk_a, never
// lower.  One lane per (window, adapter); each survivor becomes one task record (the window
// piece with the adapter in `info`), so the window scan runs full waves of surviving tasks.
// ---------------------------------------------------------------------------------------------

__device__ __forceinline__ Window make_task(Window w, uint32_t jlo, uint32_t jhi, bool lastcol,
                                            int a) {
    w.lastcol = lastcol ? 1 : 0;
    w.j1 = jlo;
    w.j2 = jhi;
    w.info = (uint32_t)a;       // a task is a window piece of one adapter
    return w;
}

__global__ __launch_bounds__(kScanBlock) void iscreen_kernel(RoundArgs R) {
    // adapter-major [a][kIpeqStride], codes 0..3: I_a's rows in the top l_a bits (row pre_len + r
    // at bit 32 - l_a + r), all-match padding below (myers_step_top); 9 words per adapter keep
    // the 24 lanes of one window (same code) on distinct banks
    __shared__ uint32_t s_ipeq[kMaxAdapters * kIpeqStride];
    __shared__ int8_t s_acc[72 * kMaxAdapters];
    __shared__ Window s_task[kScanBlock / 64][kWaveWinCap];   // per-wave task staging
    __shared__ uint32_t s_tc[kScanBlock / 64], s_nend;
    const DevPanel* P = R.panel;
    const int A = P->n_adapters;
    const int pl = P->pre_len, sl = P->filter_len, kf = P->kf;
    for (int x = threadIdx.x; x < 4 * A; x += blockDim.x) {
        const int c = x & 3, a = x >> 2;
        const int l = (int)P->ad[a].m - pl - sl;
        const uint64_t v = P->ad[a].peq[c] >> pl;
        s_ipeq[a * kIpeqStride + c] =
            l >= 32 ? (uint32_t)v
                    : ((uint32_t)(v & ((1ull << l) - 1ull)) << (32 - l)) | ((1u << (32 - l)) - 1u);
    }
    for (int x = threadIdx.x; x < 72 * A; x += blockDim.x) s_acc[x] = P->ad[x / 72].acc[x % 72];
    if (threadIdx.x < kScanBlock / 64) s_tc[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_nend = 0;
    __shared__ uint32_t s_spre[kShards + 1];
    ShardMap sm{s_spre, 0u};
    sm.load(R.win2_count, R.win_scap);                 // (its barrier covers the above)
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t wsh = wave_shard();
    const WaveStage<Window, kWaveWinCap> st{s_task[wv], &s_tc[wv], R.tasks + wsh * R.task_scap,
                                            R.task_count + wsh * kShardStride, R.task_scap,
                                            R.flags, 4u};
    const Window* wl = R.win2;
    const uint32_t nwin = sm.total();
    const uint32_t total = nwin * (uint32_t)A;    // host: win_cap * A < 2^32
    const bool front = P->where == kFront;
    const int jsplit = front ? P->jsplit : 0;
    const bool pshared = P->pshared != 0;

    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t base = blockIdx.x * blockDim.x; base < total; base += stride) {
        const uint32_t t = base + threadIdx.x;
        if (t < total) {
            const uint32_t wi = t / (uint32_t)A;
            const int a = (int)(t - wi * (uint32_t)A);
            const Window w = wl[sm.phys(wi)];
            const DevAdapter& ad = P->ad[a];
            const int len = (int)w.len, j1 = (int)w.j1, j2 = (int)w.j2;
            const int l = (int)ad.m - pl - sl, kk = ad.kk;
            const int bm = w.bmin;
            const int dP = (int)(w.info & 255u), dPe = (int)((w.info >> 8) & 255u);
            const int dPn = (int)(w.info >> 24);
            const bool lastc = !front && w.lastcol;
            // the near piece [j1, min(j2, jsplit - 1)] keeps every adapter
            if (j1 < jsplit) {
                const int jh = min(j2, jsplit - 1);
                st.push(make_task(w, (uint32_t)j1, (uint32_t)jh, false, a));
            }
            const int jr = max(j1, jsplit);               // far piece: last-row cells [jr, j2]
            const int thr = kk - bm - dP;                 // (bm = 255: no hit column, no rows)
            const bool rows = bm != 255 && jr <= j2 && thr >= 0;
            // P-only last-column cells: identical for every adapter, the first one wins ties;
            // an empty view keeps every adapter
            bool pass = lastc && (len == 0 || (((w.info >> 16) & 1u) && (a == 0 || !pshared)));
            bool by_end = true;                           // (diagnostic: no last-row reason)
            const int thr_e = kk - dPe;                   // 3' cells holding all of I_a
            if (!pass && (rows || lastc)) {
                const int xr_lo = jr - sl - kf, xr_hi = j2 - sl + kf;
                const int xe_lo = len - sl + 1 - kf;
                int xs = 1 << 30, xe = -1;
                if (rows) {
                    xs = xr_lo;
                    xe = min(xr_hi, len);
                }
                if (lastc) {
                    xs = min(xs, xe_lo);
                    xe = len;
                }
                // The I_a band starts where the P band ends: at or after x1 = jr - l - |S| - kf
                // (last-row cells) or len - (m - 1 - pre_len) - kf (3' cells).  A restricted
                // start D'(i, x0) = i at any x0 <= x1 gives every such band its cost or less, so
                // the chunk grid (ending exactly at xe) starts at or before that column; columns in
                // front of the view only lower D further.  Every column with D <= threshold thus
                // tests <= threshold.
                int x1 = 1 << 30;
                if (rows) x1 = jr - l - sl - kf;
                if (lastc) x1 = min(x1, len - ((int)ad.m - 1 - pl) - kf);
                const int nch = (xe - x1 + 15) >> 4;
                const int jb = xe - 16 * nch;
                const int xrh = min(xr_hi, len);
                const char* ip = reinterpret_cast<const char*>(s_ipeq + a * kIpeqStride);
                const uint32_t rows_m = l >= 32 ? ~0u : ~0u << (32 - l);   // I_a's rows
                uint32_t pv = rows_m, mv = 0u;
                int d = l;
                TaskView tv;
                tv.read = 0;
                tv.n = w.n;
                tv.strand = w.strand & 1u;
                tv.start = w.start;
                tv.len = w.len;
                view_off(R.pk, w.off, tv);
                tv.o = w.o;
                tv.a = a;
                uint32_t c0 = 0, n0 = 0, c1 = 0, n1 = 0;   // two chunks in flight
                if (nch > 0) fetch16s<kNecessaryMask>(R.pk, tv, jb, c0, n0);
                if (nch > 1) fetch16s<kNecessaryMask>(R.pk, tv, jb + 16, c1, n1);
                for (int k = 0; k < nch && !pass; ++k) {
                    const int p0 = jb + 16 * k;
                    const uint32_t codes = c0, nb = n0;
                    c0 = c1;
                    n0 = n1;
                    if (k + 2 < nch) fetch16s<kNecessaryMask>(R.pk, tv, p0 + 32, c1, n1);
                    // this chunk's columns p0+1 .. p0+16: the threshold of the regions it touches
                    // and the first column counted (earlier ones are warm-up)
                    const bool inR = rows && p0 + 16 >= xr_lo && p0 + 1 <= xrh;
                    const bool inE = lastc && p0 + 16 >= xe_lo;
                    const int tk = max(inR ? thr : -1, inE ? thr_e : -1);
                    const int qlo = min(inR ? xr_lo : (1 << 30), inE ? xe_lo : (1 << 30)) - p0 - 1;
                    uint32_t eq[16];
                    {
                        const uint32_t lo = spread_codes(codes, 0x0c010c00u);
                        const uint32_t hi = spread_codes(codes, 0x0c030c02u);
#pragma unroll
                        for (int q = 0; q < 16; ++q)
                            eq[q] = *reinterpret_cast<const uint32_t*>(
                                ip + __builtin_amdgcn_ubfe(q < 8 ? lo : hi, 4 * (q & 7), 4));
                    }
                    if (__builtin_amdgcn_ballot_w64(nb != 0u)) {   // non-ACGT: no match in I_a
#pragma unroll
                        for (int q = 0; q < 16; ++q)
                            eq[q] &= ~((uint32_t)__builtin_amdgcn_sbfe((int)nb, q, 1) & rows_m);
                    }
                    int cm = 127;
                    if (__builtin_amdgcn_ballot_w64(qlo > 0) == 0) {   // every column counts
#pragma unroll
                        for (int q = 0; q < 16; ++q) {
                            myers_step_top(eq[q], pv, mv, d);
                            cm = min(cm, d);
                        }
                    } else {
#pragma unroll
                        for (int q = 0; q < 16; ++q) {
                            myers_step_top(eq[q], pv, mv, d);
                            cm = min(cm, q >= qlo ? d : 127);
                        }
                    }
                    pass = cm <= tk;
                    by_end = !inR;
                }
                if (lastc && !pass) {   // partial I_a at the read end: cells (pl + r, len)
                    int dd = 0;
                    const int sh = 32 - l;   // row pre_len + r at bit sh + r - 1
                    for (int r = 1; r < l && !pass; ++r) {
                        dd += (int)((pv >> (sh + r - 1)) & 1u) - (int)((mv >> (sh + r - 1)) & 1u);
                        pass = dPn + dd <= (int)s_acc[72 * a + pl + r];
                    }
                }
            }
            if (pass) {
                st.push(make_task(w, (uint32_t)jr, (uint32_t)j2, lastc, a));
                if (by_end) atomicAdd(&s_nend, 1u);
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (st.count() > kWaveWinCap / 2) st.flush();
    }
    __builtin_amdgcn_wave_barrier();
    st.flush();
    __syncthreads();
    if (threadIdx.x == 0 && s_nend) atomicAdd(&R.diag[3], s_nend);     // by 3' cells only
}

// ---------------------------------------------------------------------------------------------
// Window code slots: the index screen, the window scan and the band each read
// the codes around a verified window; without slots each gathers them from the packed batch (a
// few random 64-B lines per window and stage).  One lane per (window, 16-column chunk) gathers
// them once, with the same fetch16s, into the window's slot (kStageWords, dense list order), and
// tags the record's `off` with slot + 1; tasks and candidates inherit the tag.  The slot covers
// columns [base, base + 128), base = max(j1 - back, lo) with back = the panel's largest m + k + 1
// and lo = -min(kViewReachPre, m_max + 7) (no gather reaches further before a view than the
// band's own), chunks starting at or before the view end (later ones keep the gather).
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kScanBlock) void wstage_kernel(RoundArgs R, Window* wl,
                                                            const uint32_t* counts, int back,
                                                            int lo) {
    __shared__ uint32_t s_spre[kShards + 1];
    ShardMap sm{s_spre, 0u};
    sm.load(counts, R.win_scap);
    const uint32_t nwin = min(sm.total(), R.stage_cap);
    const uint32_t k = threadIdx.x & 7u;            // the lane's chunk
    const uint32_t step = (gridDim.x * blockDim.x) >> 3;
    for (uint32_t g = (blockIdx.x * blockDim.x + threadIdx.x) >> 3; g < nwin; g += step) {
        const uint32_t phys = sm.phys(g);
        Window* wp = wl + phys;
        const Window w = *wp;
        TaskView tv;
        tv.read = 0;
        tv.n = w.n;
        tv.strand = w.strand & 1u;
        tv.clean = false;                           // the no-match bits always (exact stages)
        tv.start = w.start;
        tv.len = w.len;
        tv.off = w.off & kOffMask;
        tv.o = w.o;
        tv.a = 0;
        const int base = max((int)w.j1 - back, lo);
        const int nfill = min(max(((int)w.len - base) / 16 + 1, 0), 8);
        uint32_t codes = 0, nb = 0;
        if ((int)k < nfill) fetch16s<true>(R.pk, tv, base + 16 * (int)k, codes, nb);
        uint32_t* sl = R.stage + (size_t)g * kStageWords;
        sl[k] = codes;
        const uint32_t nbn = __shfl_down(nb, 1u, 64);   // (the 8 lanes of a window run together)
        if (!(k & 1u)) sl[8 + (k >> 1)] = nb | (nbn << 16);
        if (k == 0) {
            sl[12] = (uint32_t)base;
            sl[13] = 16u * (uint32_t)nfill;
            if (base + kViewReachPre < (1 << 24))
                wp->off = tv.off | ((uint64_t)(g + 1) << kOffBits);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Packed index screen (the same necessary conditions as iscreen_kernel): one lane
// per (verified window, quad of adapters).  Each adapter's index block runs in a 16-bit half of a
// dword — two adapters per dword, two dwords per lane — with gfx950's packed 16-bit VALU
// (v_pk_add_u16 keeps the halves' carries apart, v_pk_lshlrev_b16 their shifts), so one
// instruction steps two adapters.  A block longer than 16 rows is cut to its LAST 16 rows: with a
// free start in the read, an alignment of all of I_a ending at column x restricted to those rows
// is an alignment of the cut block ending at the same x of no larger cost, so D_cut <= D_I at
// every column (the screen only ever tests D <= threshold: a lower bound keeps it necessary).
// Rows of a 3' partial-I cell above the cut count as cost 0 (again a lower bound).  The block
// sits in the top l' bits of its half with all-match padding below (it stays at cost 0 and acts
// as row 0, as in myers_step_top); non-ACGT codes (table rows 4..7) match only the padding.
// LDS: [code][quad] u64 with 64-B code rows, so the six lanes of a window (24 adapters) read six
// consecutive u64 of one row and windows with other codes read other rows on other banks
// (ds_read_b64, 64 banks: code c at banks 16c .. 16c + 11) — conflict-free.
// ---------------------------------------------------------------------------------------------
typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_pk(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }

// Myers step of two 16-bit blocks (last row = bit 15 of each half); d: per-half last-row cost.
__device__ __forceinline__ void myers_step_pk(uint32_t eq, uint32_t& pv, uint32_t& mv, u16x2& d) {
    const uint32_t xv = eq | mv;
    const uint32_t s = as_u32(as_pk(eq & pv) + as_pk(pv));
    // Xh = (s ^ Pv) | Eq is never formed: Xh | Pv = s | Pv | Eq (one v_or3), and
    // Pv & Xh = Pv & ((s ^ Pv) | Eq) is one v_bitop3
    const uint32_t ph = mv | ~(s | pv | eq);
    const uint32_t mh = pv & ((s ^ pv) | eq);
    d = d + (as_pk(ph) >> (uint16_t)15) - (as_pk(mh) >> (uint16_t)15);
    const uint32_t ph2 = as_u32(as_pk(ph) << (uint16_t)1);
    const uint32_t mh2 = as_u32(as_pk(mh) << (uint16_t)1);
    pv = mh2 | ~(xv | ph2);
    mv = ph2 & xv;
}

// f * 32 as one v_lshl_add with the lane's row base (left to itself the compiler turns the
// bit-field extract + scale into shift + mask + add: three VALU per column instead of two)
__device__ __forceinline__ uint32_t lds_off32(uint32_t f, uint32_t base) {
    uint32_t r;
    asm("v_lshl_add_u32 %0, %1, 5, %2" : "=v"(r) : "v"(f), "v"(base));
    return r;
}

// bit k of b (k < 8) -> bit 4k + 3 (the no-match bit of column k's nibble)
__device__ __forceinline__ uint32_t spread_bits_nib(uint32_t b) {
    uint32_t x = b & 0xFFu;
    x = (x | (x << 12)) & 0x000F000Fu;
    x = (x | (x << 6)) & 0x03030303u;
    x = (x | (x << 3)) & 0x11111111u;
    return x << 3;
}


constexpr int kScreenQuads = 8;             // adapters <= 32 (larger panels: iscreen_kernel)
constexpr int kScreenRow = 8;               // u64 per code row (64 B)
constexpr int kScreenCap = 128;             // per-wave task staging (4 pushes per lane per round)

#ifndef DMX_SCREEN_WAVES
#define DMX_SCREEN_WAVES 4
#endif
__global__ __launch_bounds__(kScanBlock) __attribute__((amdgpu_waves_per_eu(DMX_SCREEN_WAVES))) void iscreen4_kernel(RoundArgs R) {
    __shared__ uint64_t s_q[8 * kScreenRow];
    __shared__ int8_t s_acc[72 * 4 * kScreenQuads];
    __shared__ uint32_t s_par[4 * kScreenQuads];   // per adapter: l | kk << 8 | m << 16 | l' << 24
    __shared__ int8_t s_pimax[4 * kScreenQuads];   // max acc[pre_len + r], r = 1 .. l - 1
    __shared__ Window s_task[kScanBlock / 64][kScreenCap];
    __shared__ uint32_t s_tc[kScanBlock / 64], s_nend;
    const DevPanel* P = R.panel;
    const int A = P->n_adapters;
    const int Q = (A + 3) >> 2;
    const int pl = P->pre_len, sl = P->filter_len, kf = P->kf;
    for (int x = threadIdx.x; x < 8 * kScreenRow; x += blockDim.x) {
        const int c = x / kScreenRow, q = x % kScreenRow;
        uint64_t v = 0;
        for (int h = 0; h < 4; ++h) {
            const int a = 4 * q + h;
            uint32_t half = 0xFFFFu;                  // absent adapter: padding only
            if (a < A) {
                const int l = (int)P->ad[a].m - pl - sl;
                const int lc = min(l, 16);
                const uint32_t pad = (1u << (16 - lc)) - 1u;
                // rows pre_len + (l - lc) .. pre_len + l - 1 of the adapter, top lc bits
                const uint32_t rows = c < 4 ? (uint32_t)((P->ad[a].peq[c] >> (pl + l - lc)) &
                                                         ((1ull << lc) - 1ull))
                                            : 0u;
                half = (rows << (16 - lc)) | pad;
            }
            v |= (uint64_t)half << (16 * h);
        }
        s_q[c * kScreenRow + q] = v;
    }
    for (int x = threadIdx.x; x < 72 * A; x += blockDim.x) s_acc[x] = P->ad[x / 72].acc[x % 72];
    for (int a = threadIdx.x; a < A; a += blockDim.x) {
        const int l = (int)P->ad[a].m - pl - sl;
        s_par[a] = (uint32_t)l | ((uint32_t)(uint8_t)P->ad[a].kk << 8) |
                   ((uint32_t)P->ad[a].m << 16) | ((uint32_t)min(l, 16) << 24);
        int mx = -1;
        for (int r = 1; r < l; ++r) mx = max(mx, (int)P->ad[a].acc[pl + r]);
        s_pimax[a] = (int8_t)mx;
    }
    if (threadIdx.x < kScanBlock / 64) s_tc[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_nend = 0;
    __shared__ uint32_t s_spre[kShards + 1];
    ShardMap sm{s_spre, 0u};
    sm.load(R.win2_count, R.win_scap);                 // (its barrier covers the above)
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t wsh = wave_shard();
    const WaveStage<Window, kScreenCap> st{s_task[wv], &s_tc[wv], R.tasks + wsh * R.task_scap,
                                           R.task_count + wsh * kShardStride, R.task_scap,
                                           R.flags, 4u};
    const Window* wl = R.win2;
    const uint32_t nwin = sm.total();
    const uint32_t total = nwin * (uint32_t)Q;
    const bool front = P->where == kFront;
    const int jsplit = front ? P->jsplit : 0;
    const bool pshared = P->pshared != 0;

    // FRONT panels: a wave costs its longest lane, and near pieces (no scan) and wide windows
    // share the list with the common ~3-chunk windows (tools/screen_stats.py: wave max / mean
    // 1.37 on round 1 of c2x24); each block takes kSortGroup consecutive lanes at a time and runs
    // them in order of their window's scan span.  3' panels' windows are even (1.04): unsorted.
    const bool sorted = front;
    __shared__ uint32_t s_ord[kSortGroup];
    __shared__ uint32_t s_bin[kSortBins];
    for (uint32_t gb = blockIdx.x * kSortGroup; gb < total; gb += gridDim.x * kSortGroup) {
      const uint32_t gn = min((uint32_t)kSortGroup, total - gb);
      if (sorted) {   // block-uniform
        if (threadIdx.x < kSortBins) s_bin[threadIdx.x] = 0;
        __syncthreads();                           // (also: the last group's s_ord)
        constexpr int PER = kSortGroup / kScanBlock;
        uint32_t key[PER], pos[PER];
        // every record's fields first (unconditional loads, clamped index: all in flight at
        // once), then the bin counts
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            const uint32_t li = threadIdx.x + (uint32_t)e * kScanBlock;
            const Window* w = wl + sm.phys((gb + min(li, gn - 1u)) / (uint32_t)Q);
            const int j1 = (int)w->j1, j2 = (int)w->j2;
            const int span = w->bmin != 255 ? j2 - max(j1, jsplit) : -1;
            key[e] = span < 0 ? 0u : 1u + (uint32_t)min(span >> kSortShift, kSortBins - 2);
        }
#pragma unroll
        for (int e = 0; e < PER; ++e)
            if (threadIdx.x + (uint32_t)e * kScanBlock < gn) pos[e] = atomicAdd(&s_bin[key[e]], 1u);
        __syncthreads();
        if (threadIdx.x == 0) {                    // exclusive scan over the bins
            uint32_t acc = 0;
            for (int b = 0; b < kSortBins; ++b) {
                const uint32_t c = s_bin[b];
                s_bin[b] = acc;
                acc += c;
            }
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < PER; ++e) {
            const uint32_t li = threadIdx.x + (uint32_t)e * kScanBlock;
            if (li < gn) s_ord[s_bin[key[e]] + pos[e]] = li;
        }
        __syncthreads();
      }
      for (uint32_t sb = 0; sb < gn; sb += kScanBlock) {   // block-uniform
        const uint32_t li = sb + threadIdx.x;
        const bool live = li < gn;
        const uint32_t t = gb + (live ? (sorted ? s_ord[li] : li) : 0u);
        uint32_t near_m = 0, pass_m = 0, end_m = 0;   // per adapter k of the quad (bits 0..3)
        Window w{};
        int q = 0;
        if (live) {
            const uint32_t wi = t / (uint32_t)Q;
            q = (int)(t - wi * (uint32_t)Q);
            w = wl[sm.phys(wi)];
            const int len = (int)w.len, j1 = (int)w.j1, j2 = (int)w.j2;
            const int bm = w.bmin;
            const int dP = (int)(w.info & 255u), dPe = (int)((w.info >> 8) & 255u);
            const int dPn = (int)(w.info >> 24);
            const bool lastc = !front && w.lastcol;
            const uint32_t valid = A - 4 * q >= 4 ? 0xFu : ((1u << (A - 4 * q)) - 1u);
            if (j1 < jsplit) near_m = valid;                 // the near piece keeps every adapter
            const int jr = max(j1, jsplit);
            const bool rows_base = bm != 255 && jr <= j2;
            // per adapter: thresholds, first column of the band, which tests apply
            int thr[4], thre[4], x1 = 1 << 30;
            uint32_t need = 0, rows_m = 0;
            const bool pinfo = ((w.info >> 16) & 1u) != 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int a = 4 * q + k;
                const uint32_t par = (valid >> k) & 1u ? s_par[a] : 0u;
                const int l = (int)(par & 255u), kk = (int)((par >> 8) & 255u);
                const int m = (int)((par >> 16) & 255u);
                thr[k] = kk - bm - dP;                        // (bm = 255: no hit column)
                thre[k] = kk - dPe;
                const bool rk = ((valid >> k) & 1u) && rows_base && thr[k] >= 0;
                if (!rk) thr[k] = -1;
                if (!lastc) thre[k] = -1;
                // P-only last-column cells: identical for every adapter, the first one wins
                // ties; an empty view keeps every adapter
                if (((valid >> k) & 1u) && lastc && (len == 0 || (pinfo && (a == 0 || !pshared))))
                    pass_m |= 1u << k;
                if (((valid >> k) & 1u) && !((pass_m >> k) & 1u) && (rk || lastc)) {
                    need |= 1u << k;
                    if (rk) x1 = min(x1, jr - l - sl - kf);
                    if (lastc) x1 = min(x1, len - (m - 1 - pl) - kf);
                }
                if (rk) rows_m |= 1u << k;
            }
            end_m = valid;                                   // (diagnostic: no last-row reason)
            if (need) {
                const bool rows = rows_m != 0;
                const int xr_lo = jr - sl - kf, xr_hi = j2 - sl + kf;
                const int xe_lo = len - sl + 1 - kf;
                int xe = -1;
                if (rows) xe = min(xr_hi, len);
                if (lastc) xe = len;
                const int nch = (xe - x1 + 15) >> 4;
                const int jb = xe - 16 * nch;
                const int xrh = min(xr_hi, len);
                uint32_t lp[2];                              // l' of the four halves
                {
                    const uint32_t p0 = s_par[4 * q] >> 24, p1 = s_par[4 * q + 1] >> 24;
                    const uint32_t p2 = s_par[4 * q + 2] >> 24, p3 = s_par[4 * q + 3] >> 24;
                    lp[0] = (valid & 1u ? p0 : 0u) | ((valid & 2u ? p1 : 0u) << 16);
                    lp[1] = (valid & 4u ? p2 : 0u) | ((valid & 8u ? p3 : 0u) << 16);
                }
                // block rows = the top l' bits of each half (D(i, x0) = i there, 0 below)
                uint32_t pv0, pv1, mv0 = 0u, mv1 = 0u;
                {
                    const uint32_t r0 = (0xFFFFu << (16 - (lp[0] & 0xFFFFu))) & 0xFFFFu;
                    const uint32_t r1 = (0xFFFFu << (16 - (lp[0] >> 16))) & 0xFFFFu;
                    const uint32_t r2 = (0xFFFFu << (16 - (lp[1] & 0xFFFFu))) & 0xFFFFu;
                    const uint32_t r3 = (0xFFFFu << (16 - (lp[1] >> 16))) & 0xFFFFu;
                    pv0 = r0 | (r1 << 16);
                    pv1 = r2 | (r3 << 16);
                }
                u16x2 d0 = as_pk(lp[0]), d1 = as_pk(lp[1]);
                TaskView tv;
                tv.read = 0;
                tv.n = w.n;
                tv.strand = w.strand & 1u;
                tv.start = w.start;
                tv.len = w.len;
                view_off(R.pk, w.off, tv);
                tv.o = w.o;
                tv.a = 0;
                const char* qb = reinterpret_cast<const char*>(s_q);
                const uint32_t q8 = 8u * (uint32_t)q;   // the lane's quad within a code row
                Chunk16 nx;                                  // the next chunk, in flight
                if (nch > 0) nx = chunk16_load<kNecessaryMask>(R.pk, tv, jb);
                for (int kc = 0; kc < nch && (need & ~pass_m); ++kc) {
                    const int p0 = jb + 16 * kc;
                    uint32_t codes, nb;
                    chunk16_codes<kNecessaryMask>(tv, p0, nx, codes, nb);
                    if (kc + 1 < nch) nx = chunk16_load<kNecessaryMask>(R.pk, tv, p0 + 16);
                    const bool inR = rows && p0 + 16 >= xr_lo && p0 + 1 <= xrh;
                    const bool inE = lastc && p0 + 16 >= xe_lo;
                    const int qlo = min(inR ? xr_lo : (1 << 30), inE ? xe_lo : (1 << 30)) - p0 - 1;
                    // nibble q of lo/hi: code * 2 + no-match * 8, i.e. the byte offset / 32 of
                    // the column's code row ([code][quad] u64, 64-B rows)
                    uint32_t lo = ((spread_codes(codes, 0x0c010c00u) >> 1));
                    uint32_t hi = ((spread_codes(codes, 0x0c030c02u) >> 1));
                    if (__builtin_amdgcn_ballot_w64(nb != 0u)) {
                        lo |= spread_bits_nib(nb);
                        hi |= spread_bits_nib(nb >> 8);
                    }
                    uint32_t cm0 = 0xFFFFFFFFu, cm1 = 0xFFFFFFFFu;
                    u16x2 m0 = as_pk(cm0), m1 = as_pk(cm1);
                    if (__builtin_amdgcn_ballot_w64(qlo > 0) == 0) {   // every column counts
#pragma unroll
                        for (int c = 0; c < 16; ++c) {
                            const uint64_t e = *reinterpret_cast<const uint64_t*>(
                                qb + lds_off32(__builtin_amdgcn_ubfe(c < 8 ? lo : hi,
                                                                     4 * (c & 7), 4), q8));
                            myers_step_pk((uint32_t)e, pv0, mv0, d0);
                            myers_step_pk((uint32_t)(e >> 32), pv1, mv1, d1);
                            m0 = __builtin_elementwise_min(m0, d0);
                            m1 = __builtin_elementwise_min(m1, d1);
                        }
                    } else {
#pragma unroll
                        for (int c = 0; c < 16; ++c) {
                            const uint64_t e = *reinterpret_cast<const uint64_t*>(
                                qb + lds_off32(__builtin_amdgcn_ubfe(c < 8 ? lo : hi,
                                                                     4 * (c & 7), 4), q8));
                            myers_step_pk((uint32_t)e, pv0, mv0, d0);
                            myers_step_pk((uint32_t)(e >> 32), pv1, mv1, d1);
                            if (c >= qlo) {
                                m0 = __builtin_elementwise_min(m0, d0);
                                m1 = __builtin_elementwise_min(m1, d1);
                            }
                        }
                    }
                    cm0 = as_u32(m0);
                    cm1 = as_u32(m1);
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint32_t cmk = ((k < 2 ? cm0 : cm1) >> (16 * (k & 1))) & 0xFFFFu;
                        const int tk = max(inR ? thr[k] : -1, inE ? thre[k] : -1);
                        if (((need >> k) & 1u) && !((pass_m >> k) & 1u) && (int)cmk <= tk) {
                            pass_m |= 1u << k;
                            if (inR) end_m &= ~(1u << k);
                        }
                    }
                }
                // partial I_a at the read end: cells (pre_len + r, len), r = 1 .. l - 1
                if (lastc) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        if (!((need >> k) & 1u) || ((pass_m >> k) & 1u)) continue;
                        const int a = 4 * q + k;
                        if (dPn > (int)s_pimax[a]) continue;   // no row can pass (D >= 0)
                        const uint32_t par = s_par[a];
                        const int l = (int)(par & 255u), lc = (int)(par >> 24);
                        const uint32_t pvh = ((k < 2 ? pv0 : pv1) >> (16 * (k & 1))) & 0xFFFFu;
                        const uint32_t mvh = ((k < 2 ? mv0 : mv1) >> (16 * (k & 1))) & 0xFFFFu;
                        bool ok = false;
                        int dd = 0;
                        for (int r = 1; r < l && !ok; ++r) {
                            if (r > l - lc) {   // row r of I_a = bit 16 - l + r - 1 of the half
                                const int b = 16 - l + r - 1;
                                dd += (int)((pvh >> b) & 1u) - (int)((mvh >> b) & 1u);
                            }                   // rows above the cut: cost >= 0
                            ok = dPn + dd <= (int)s_acc[72 * a + pl + r];
                        }
                        if (ok) pass_m |= 1u << k;
                    }
                }
            }
            pass_m &= valid;
            end_m &= pass_m;
        }
        // pushes: at most 4 per lane, one wave-uniform round per adapter of the quad; a flush
        // before each round keeps the slice from overflowing (kScreenCap >= 64 + 64)
        const int jr = max((int)w.j1, jsplit);
        const bool lastc = !front && w.lastcol;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            __builtin_amdgcn_wave_barrier();
            if (st.count() > kScreenCap - 64) st.flush();
            if ((near_m >> k) & 1u)
                st.push(make_task(w, w.j1, (uint32_t)min((int)w.j2, jsplit - 1), false, 4 * q + k));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            __builtin_amdgcn_wave_barrier();
            if (st.count() > kScreenCap - 64) st.flush();
            if ((pass_m >> k) & 1u) {
                st.push(make_task(w, (uint32_t)jr, w.j2, lastc, 4 * q + k));
                if ((end_m >> k) & 1u) atomicAdd(&s_nend, 1u);
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (st.count() > kScreenCap / 2) st.flush();
      }
    }
    __builtin_amdgcn_wave_barrier();
    st.flush();
    __syncthreads();
    if (threadIdx.x == 0 && s_nend) atomicAdd(&R.diag[3], s_nend);     // by 3' cells only
}

// Window scan: one lane per (window, adapter) — or, after the index screen, per surviving
// (piece, adapter) — in a block-uniform grid stride over the device-side count, so that the
// block can flush its staged records between strides.
// One (window or piece, adapter) task of the window scan.
// Window-scan match vectors: the 64 lanes of a wave scan random (task,
// adapter, code) triples, and a gather of 64-bit vectors from the panel's [code][adapter] table
// conflicts ~2 extra LDS cycles per read.  DMX_WSCAN_LANE_ROWS=1 (A/B): a lane copies its task's
// adapter vectors into rows of its own (s_lrow[code][thread], plus a zero row 4 for non-ACGT
// codes), so the 32 lanes of a ds_read_b64 group read 32 distinct bank pairs.  Measured (round
// 5, profiles/r5_ab_wscan_lane_rows.txt): conflict cycles per LDS instruction 1.94 / 2.01 ->
// 0.62 / 0.83, window scan time unchanged (3.64 / 2.18 vs 3.62 / 2.16 ms): LDS waits are 0.1 %
// of its wave cycles, it waits on its global gathers.  Off by default (10 KB more LDS).
constexpr int kLaneRows = 5;

template <bool BAND, class ClStage, class Sink>
__device__ __forceinline__ void wscan_task(const RoundArgs& R, const Window& w, int a, int A,
                                           const uint64_t* s_peq, const int8_t* s_acc,
                                           const int8_t* s_pacc, const uint32_t* s_amk,
                                           const ClStage& st, const Sink& sink, CandOut& co,
                                           TaskView& tv, int& sub, uint64_t* lrow) {
    sub = w.o * A + a;
    tv.read = 0;
    tv.n = w.n;
    tv.strand = w.strand & 1u;
    tv.clean = (w.strand & kWinClean) != 0;
    tv.start = w.start;
    tv.len = w.len;
    view_off(R.pk, w.off, tv);
    tv.o = w.o;
    tv.a = a;
    const AdLite ad = ad_lite(s_amk[a]);
    int js = (int)w.j1 - ad.m - ad.k - 1;
    const bool real = js <= 0;
    if (real) js = 0;
    int lb;
    if constexpr (BAND && DMX_WSCAN_LANE_ROWS) {
#pragma unroll
        for (int c = 0; c < 4; ++c) lrow[c * kScanBlock] = s_peq[c * kPeqStride + a];
        lb = scan_task_cand<Sink, kScanBlock, true>(R, sink, tv, w.item, sub, lrow, A, ad,
                                                    s_acc + 72 * a, s_pacc + 72 * a,
                                                    (uint32_t)js, real, w.j1, w.j2,
                                                    w.lastcol != 0, &co);
    } else if constexpr (BAND) {
        lb = scan_task_cand(R, sink, tv, w.item, sub, s_peq + a, A, ad, s_acc + 72 * a,
                            s_pacc + 72 * a, (uint32_t)js, real, w.j1, w.j2,
                            w.lastcol != 0, &co);
    } else
        lb = scan_task(R, st, tv, w.item, sub, s_peq + a, A, ad, s_acc + 72 * a,
                       s_pacc + 72 * a, (uint32_t)js, real, w.j1, w.j2, w.lastcol != 0);
    const uint32_t slot = slot_of(R, w.item, sub);
    if (lb > 0 && DMX_BOUND(R.pk.bd, slots, slot, kBufSlot)) atomicMax(&R.lb[slot], lb);
}

// Occupancy floor for the window scan (register budget 512 / waves): at 129 VGPRs the compiler
// drops to 3 waves per SIMD, measured 7 % slower on the whole step.  Round 5: 4 waves spill 31
// VGPRs, 3 waves need 153 and spill none, and are still slower (window scan 3.62 / 2.16 ->
// 3.85 / 2.38 ms, profiles/r5_ab_wscan_waves_candcap.txt).
#ifndef DMX_WSCAN_WAVES
#define DMX_WSCAN_WAVES 4
#endif
template <bool BAND>
__global__ __launch_bounds__(kScanBlock) __attribute__((amdgpu_waves_per_eu(DMX_WSCAN_WAVES))) void wscan_kernel(RoundArgs R) {
    __shared__ uint64_t s_peq[8 * kPeqStride];
    __shared__ int8_t s_acc[72 * kMaxAdapters];
    __shared__ int8_t s_pacc[72 * kMaxAdapters];
    __shared__ uint32_t s_amk[kMaxAdapters];
    __shared__ Cluster s_cl[BAND ? 1 : kStageCap];
    __shared__ uint32_t s_clcnt, s_clbase;
    __shared__ Cand s_wcand[BAND ? kScanBlock / 64 : 1][2][kWaveCandCap];
    __shared__ uint32_t s_wcn[kScanBlock / 64][2];
    constexpr bool kRows = BAND && DMX_WSCAN_LANE_ROWS;
    __shared__ uint64_t s_lrow[kRows ? kLaneRows * kScanBlock : 1];   // [code][thread]
    if constexpr (kRows) s_lrow[4 * kScanBlock + threadIdx.x] = 0ull;   // non-ACGT: no match
    uint64_t* const lrow = s_lrow + (kRows ? threadIdx.x : 0u);
#ifdef DMX_WSCAN_LDS_PAD   // A/B: occupancy cap through LDS
    __shared__ uint32_t s_pad[DMX_WSCAN_LDS_PAD / 4];
    if (threadIdx.x == 0) s_pad[R.n_items & 7] = 0;
#endif
    if (threadIdx.x == 0) s_clcnt = 0;
    if (threadIdx.x < 2 * (kScanBlock / 64)) (&s_wcn[0][0])[threadIdx.x] = 0;
    const Stage<Cluster> st{s_cl, &s_clcnt, &s_clbase, R.cl, R.cl_count, R.cl_cap, R.flags, 1u};
    const uint32_t wv = BAND ? threadIdx.x >> 6 : 0u;
    const uint32_t wsh = wave_shard();
    const WaveCandSink sink{{WaveStage<Cand, kWaveCandCap>{s_wcand[wv][0], &s_wcn[wv][0],
                                                           R.cand[0] + wsh * R.cand_scap,
                                                           R.cand_count + wsh * kShardStride,
                                                           R.cand_scap,
                                                           R.flags, 8u},
                             WaveStage<Cand, kWaveCandCap>{s_wcand[wv][1], &s_wcn[wv][1],
                                                           R.cand[1] + wsh * R.cand_scap,
                                                           R.cand_count + (kShards + wsh) * kShardStride,
                                                           R.cand_scap, R.flags, 8u}}};
    load_panel_lds(R.panel, s_peq, s_acc, s_pacc, s_amk);
    __shared__ uint32_t s_spre[kShards + 1];
    ShardMap sm{s_spre, 0u};
    const Window* wl = R.panel->pre_len ? R.win2 : R.win;
    if (R.screen) sm.load(R.task_count, R.task_scap);  // (its barrier covers the above)
    else sm.load(R.panel->pre_len ? R.win2_count : R.win_count, R.win_scap);

    const int A = R.panel->n_adapters;
    if (R.screen) {   // the index screen's surviving (window piece, adapter) tasks
      // A wave costs its longest task, and a FRONT panel's list mixes near pieces (a few
      // columns, every adapter) with full windows (m + k + 1 + width columns): each block takes
      // kSortGroup consecutive tasks at a time and runs them in order of their column count,
      // so the 64 tasks of a wave have nearly equal lengths (tools/task_stats.py, round 1 of
      // c2x24: wave max / mean 1.90 -> 1.09; window scan 4.8 -> 4.1 ms).  3' panels' tasks
      // are already even (1.08), and there the sort only costs (2.4 -> 2.6 ms): not sorted.
      const bool sorted = R.panel->where == kFront;
      __shared__ uint16_t s_ord[kSortGroup];   // (indices < kSortGroup: 16 bits halve the LDS)
      static_assert(kSortGroup <= 65536, "sort-group indices are 16-bit");
      __shared__ uint32_t s_bin[kSortBins];
      __shared__ uint8_t s_mk[kMaxAdapters];
      for (int a = threadIdx.x; a < A; a += blockDim.x)
          s_mk[a] = (uint8_t)min(255, (int)R.panel->ad[a].m + (int)R.panel->ad[a].k + 1);
      {
        const Window* tl = R.tasks;
        const uint32_t nt = sm.total();
        for (uint32_t gb = blockIdx.x * kSortGroup; gb < nt; gb += gridDim.x * kSortGroup) {
            const uint32_t gn = min((uint32_t)kSortGroup, nt - gb);
            if (sorted) {   // block-uniform
            if (threadIdx.x < kSortBins) s_bin[threadIdx.x] = 0;
            __syncthreads();                       // (also: s_mk, and the last group's s_ord)
            constexpr int PER = kSortGroup / kScanBlock;
            uint32_t key[PER], pos[PER];
            // every record's fields first (unconditional loads, clamped index: all in flight at
            // once), then the bin counts
#pragma unroll
            for (int e = 0; e < PER; ++e) {
                const uint32_t li = threadIdx.x + (uint32_t)e * kScanBlock;
                const Window* w = tl + sm.phys(gb + min(li, gn - 1u));
                const int j1 = (int)w->j1, j2 = (int)w->j2, a = (int)w->info;
                const int cols = j2 - max(j1 - (int)s_mk[a], 0);
                key[e] = (uint32_t)min(max(cols, 0) >> kSortShift, kSortBins - 1);
            }
#pragma unroll
            for (int e = 0; e < PER; ++e)
                if (threadIdx.x + (uint32_t)e * kScanBlock < gn)
                    pos[e] = atomicAdd(&s_bin[key[e]], 1u);
            __syncthreads();
            if (threadIdx.x == 0) {                // exclusive scan over the bins
                uint32_t acc = 0;
                for (int b = 0; b < kSortBins; ++b) {
                    const uint32_t c = s_bin[b];
                    s_bin[b] = acc;
                    acc += c;
                }
            }
            __syncthreads();
#pragma unroll
            for (int e = 0; e < PER; ++e) {
                const uint32_t li = threadIdx.x + (uint32_t)e * kScanBlock;
                if (li < gn) s_ord[s_bin[key[e]] + pos[e]] = (uint16_t)li;
            }
            __syncthreads();
            }
            for (uint32_t sb = 0; sb < gn; sb += kScanBlock) {   // block-uniform
                const uint32_t li = sb + threadIdx.x;
                CandOut co;
                TaskView tv{};
                int sub = 0;
                uint32_t item = 0;
                if (li < gn) {
                    const Window w = tl[sm.phys(gb + (sorted ? s_ord[li] : li))];
                    item = w.item;
                    wscan_task<BAND>(R, w, (int)w.info, A, s_peq, s_acc, s_pacc, s_amk, st, sink, co,
                                     tv, sub, lrow);
                }
                if constexpr (BAND) {
                    emit_cands(R, co, tv, item, sub, (int)(s_amk[tv.a] & 255u));
                    __builtin_amdgcn_wave_barrier();
                    if (sink.st[0].count() > DMX_WAVE_CAND_FLUSH) sink.st[0].flush();
                    if (sink.st[1].count() > DMX_WAVE_CAND_FLUSH) sink.st[1].flush();
                } else {
                    if (stage_count(&s_clcnt) > kStageCap / 2) st.flush();
                }
            }
        }
      }
        if constexpr (BAND) {
            __builtin_amdgcn_wave_barrier();
            sink.st[0].flush();
            sink.st[1].flush();
        } else {
            st.flush();
        }
        return;
    }
    const uint64_t total = (uint64_t)sm.total() * (uint64_t)A;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x; base < total;
         base += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t t = base + threadIdx.x;
        CandOut co;
        TaskView tv{};
        int sub = 0;
        uint32_t item = 0;
        if (t < total) {
            const Window w = wl[sm.phys((uint32_t)(t / A))];
            const int a = (int)(t % A);
            item = w.item;
            wscan_task<BAND>(R, w, a, A, s_peq, s_acc, s_pacc, s_amk, st, sink, co, tv, sub,
                             lrow);
        }
        if constexpr (BAND) {                        // wave-uniform: no block barrier
            emit_cands(R, co, tv, item, sub, (int)(s_amk[tv.a] & 255u));
            __builtin_amdgcn_wave_barrier();
            if (sink.st[0].count() > DMX_WAVE_CAND_FLUSH) sink.st[0].flush();
            if (sink.st[1].count() > DMX_WAVE_CAND_FLUSH) sink.st[1].flush();
        } else {
            if (stage_count(&s_clcnt) > kStageCap / 2) st.flush();
        }
    }
    if constexpr (BAND) {
        __builtin_amdgcn_wave_barrier();
        sink.st[0].flush();
        sink.st[1].flush();
    } else {
        st.flush();
    }
}

// ---------------------------------------------------------------------------------------------
// resolve: one lane per cluster; restricted Myers window + cutadapt tie-broken traceback.
// The last RING columns of (Pv, Mv) and the read codes live in LDS, lane-interleaved.
// ---------------------------------------------------------------------------------------------
// The adapter's match vectors live in registers: Eq for a read code is a 3-level select.
struct PeqRegs {
    uint64_t p0, p1, p2, p3;
    __device__ __forceinline__ uint64_t eq(uint32_t code) const {
        const uint64_t a = (code & 1u) ? p1 : p0;
        const uint64_t b = (code & 1u) ? p3 : p2;
        const uint64_t e = (code & 2u) ? b : a;
        return (code & 4u) ? 0ull : e;
    }
};

template <int RING>
struct Walker {
    Packed pk;
    uint32_t* flags;
    TaskView tv;
    PeqRegs peq;
    const uint64_t* rp;     // LDS ring (P): rp[slot * 64]
    const uint64_t* rm;
    int js;
    bool real, front;

    // Walk cutadapt's DP pointers from cell (i, j) back to the alignment start; s0 = ring slot
    // of column j.  Pointer rule (_align.pyx locate): equal characters -> diagonal; else
    // mismatch if diag <= deletion and diag <= insertion; else insertion (up) if
    // insertion <= deletion; else deletion (left).  Scores: +1 match, -1 mismatch, -2 indel.
    // Runs of matches only touch registers; the ring is read at the <= k error cells.
    __device__ void trace(int i, int j, int s0, int& origin, int& score) const {
        score = 0;
        int cbase = 1 << 30;          // view position of bit 0 of the cached 16-code chunk
        uint32_t codes = 0, nb = 0;
        while (i > 0) {
            if (j == js) {
                if (real) {
                    if (front) {
                        origin = -i;           // FRONT column 0: origin -i, score 0
                    } else {
                        score -= 2 * i;        // BACK column 0: cost i, score -2i, origin 0
                        origin = 0;
                    }
                } else {
                    atomicOr(flags, 2u);       // unreachable for cost <= k
                    score -= 2 * i;
                    origin = js;
                }
                return;
            }
            const int p = j - 1;              // view position of column j's character
            if (p < cbase) {
                cbase = max(p - 15, 0);
                fetch16t(pk, tv, (uint32_t)cbase, codes, nb);
            }
            const int sh = p - cbase;
            const uint32_t code = ((codes >> (2 * sh)) & 3u) | (((nb >> sh) & 1u) << 2);
            const int s1 = s0 == 0 ? RING - 1 : s0 - 1;
            if ((peq.eq(code) >> (i - 1)) & 1ull) {
                --i;
                --j;
                ++score;
                s0 = s1;
                continue;
            }
            const uint64_t p1 = rp[s1 * 64], m1 = rm[s1 * 64];
            const int cdel = col_cost(p1, m1, i);                                   // D(i, j-1)
            const int cd = cdel - (int)((p1 >> (i - 1)) & 1ull) + (int)((m1 >> (i - 1)) & 1ull);
            const int cins = col_cost(rp[s0 * 64], rm[s0 * 64], i - 1);             // D(i-1, j)
            if (cd <= cdel && cd <= cins) {
                --i;
                --j;
                score -= 1;
                s0 = s1;
            } else if (cins <= cdel) {
                --i;
                score -= 2;
            } else {
                --j;
                score -= 2;
                s0 = s1;
            }
        }
        origin = j;
    }
};

// resolve: one lane per cluster.  The forward pass re-runs Myers over the cluster window and
// keeps the last RING columns of (Pv, Mv) in LDS; candidate cells are only MARKED in a bitmask
// and traced back at sync points every `sync` columns, so that all lanes of a wave walk their
// tracebacks in lockstep (inline tracebacks at per-lane columns serialise the wave).
// Dynamic LDS: ring P [RING*64] u64, ring M [RING*64] u64, acc [72*A], pacc [72*A].
template <int RING>
__global__ __launch_bounds__(kResolveBlock) void resolve_kernel(RoundArgs R) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint64_t* s_rp = (uint64_t*)smem;
    uint64_t* s_rm = s_rp + RING * kResolveBlock;
    int8_t* s_acc = (int8_t*)(s_rm + RING * kResolveBlock);
    const int A = R.panel->n_adapters;
    int8_t* s_pacc = s_acc + 72 * A;
    for (int x = threadIdx.x; x < 72 * A; x += blockDim.x) {
        s_acc[x] = R.panel->ad[x / 72].acc[x % 72];
        s_pacc[x] = R.panel->ad[x / 72].pacc[x % 72];
    }
    __syncthreads();

    const uint32_t total = min(*R.cl_count, R.cl_cap);
    const int lane = threadIdx.x;
    uint32_t n_resolved = 0, n_traces = 0;
    uint64_t* rp = s_rp + lane;
    uint64_t* rm = s_rm + lane;

    for (uint32_t ci = blockIdx.x * kResolveBlock + lane; ci < total;
         ci += gridDim.x * kResolveBlock) {
        const Cluster c = R.cl[ci];
        const uint32_t slot = slot_of(R, c.item, c.sub);
        if (!DMX_BOUND(R.pk.bd, slots, slot, kBufSlot)) continue;
        const int lbk = R.lb[slot];
        const int lbs = lb_score(lbk);                // slot's best score is >= lbs
        Outcome out;
        out.key = ~0ull;
        out.origin = 0;
        out.pad = 0;
        if ((int)c.ub < lbs) {            // cannot reach the slot's guaranteed best score
            R.outc[ci] = out;
            continue;
        }
        TaskView tv;
        task_view(R, c.item, c.sub, A, tv);
        ++n_resolved;
        const DevAdapter& ad = R.panel->ad[tv.a];
        const int m = ad.m, k = ad.k, kk = ad.kk;
        const bool front = ad.where == kFront;
        const PeqRegs peq{ad.peq[0], ad.peq[1], ad.peq[2], ad.peq[3]};
        const uint64_t snapshot = R.winner[slot];
        const int8_t* acc = s_acc + 72 * tv.a;
        const int8_t* pacc = s_pacc + 72 * tv.a;
        const int sync = min(RING - (m + k + 2), 31);   // >= 4 by host-side ring choice

        int js = (int)c.j1 - m - k - 1;
        const bool real = js <= 0;
        if (real) js = 0;
        uint64_t pv = (front && real) ? 0ull : ~0ull, mv = 0ull;
        int d = (front && real) ? 0 : m;
        rp[0] = pv;                       // slot(js) = 0
        rm[0] = mv;

        const Walker<RING> W{R.pk, R.flags, tv, peq, rp, rm, js, real, front};
        bool found = false;
        int bs = 0, bc = 0, bo = 0;
        uint64_t bt = 0;

        // can a cell of cost `cost` whose aligned adapter length is <= lr still win the slot?
        auto viable = [&](int lr, int cost) {
            return beats_lb(lbk, lr - 2 * cost, tv.o, cost);   // score <= lr - 2 cost
        };
        auto consider = [&](int iend, int j, int s, int cost, uint64_t t) {
            const int ub = min(iend, j + cost) - 2 * cost;
            if (!viable(min(iend, j + cost), cost)) return;
            if (found && (ub < bs || (ub == bs && cost >= bc))) return;
            if (make_key(ub, tv.o, cost, tv.a, t) > snapshot) return;
            int origin, score;
            if (cost == 0) {                  // exact: the pointer chain is the pure diagonal
                origin = j - iend;            // (FRONT only when j < iend: reaches column 0)
                score = j >= iend ? iend : j;
            } else {
                W.trace(iend, j, s, origin, score);
                ++n_traces;
            }
            const int lr = iend + (origin < 0 ? origin : 0);
            if (lr < 0 || cost > (int)acc[lr]) return;
            if (!found || score > bs || (score == bs && cost < bc)) {
                found = true;
                bs = score;
                bc = cost;
                bt = t;
                bo = origin;
            }
        };

        const uint32_t hbit = (uint32_t)(m - 1);
        int sl = 0;                       // ring slot of the current column
        uint32_t pending = 0;             // candidate columns since the last sync (bit = age)
        int since = 0;                    // columns since the last sync
        uint32_t curj = (uint32_t)js;     // current column
        // trace the marked cells, oldest first (locate's scan order), all lanes together
        auto drain = [&]() {
            while (pending) {
                const int age = 31 - __clz(pending);          // oldest marked column
                pending &= ~(1u << age);
                const int sidx = sl - age < 0 ? sl - age + RING : sl - age;
                const int j = (int)curj - age;
                const int cost = col_cost(rp[sidx * 64], rm[sidx * 64], m);
                consider(m, j, sidx, cost, (uint64_t)j);
            }
            since = 0;
        };
        uint32_t ncodes, nnb;             // next chunk, prefetched one chunk ahead
        fetch16t(R.pk, tv, (uint32_t)js, ncodes, nnb);
        for (uint32_t p0 = (uint32_t)js; p0 < c.j2; p0 += 16) {
            const uint32_t codes = ncodes, nb = nnb;
            if (p0 + 16 < c.j2)
                fetch16t(R.pk, tv, p0 + 16, ncodes, nnb);
            const uint32_t cnt = min(16u, c.j2 - p0);
            for (uint32_t q = 0; q < cnt; ++q) {
                const uint32_t code = ((codes >> (2 * q)) & 3u) | (((nb >> q) & 1u) << 2);
                myers_step(peq.eq(code), pv, mv, d, hbit);
                const uint32_t j = p0 + q + 1;
                curj = j;
                sl = sl == RING - 1 ? 0 : sl + 1;
                rp[sl * 64] = pv;
                rm[sl * 64] = mv;
                pending <<= 1;
                if (j >= c.j1 && d <= kk) {
                    const int lr = min(m, (int)j + d);
                    if (d <= (int)pacc[lr] && viable(lr, d)) pending |= 1u;
                }
                if (++since == sync) drain();
            }
        }
        drain();
        if (c.lastcol && !front) {   // (m, 0) of an empty view: a last-row cell at t = 0
            int dd = 0;
            const int ilast = tv.len == 0 ? m : m - 1;
            for (int i = 1; i <= ilast; ++i) {
                dd += (int)((pv >> (i - 1)) & 1ull) - (int)((mv >> (i - 1)) & 1ull);
                if (dd <= (int)acc[i])
                    consider(i, (int)tv.len, sl, dd,
                             i == m ? (uint64_t)tv.len : (uint64_t)tv.len + 1 + i);
            }
        }
        if (found) {
            out.key = make_key(bs, tv.o, bc, tv.a, bt);
            out.origin = bo;
            atomicMin(&R.winner[slot], (unsigned long long)out.key);
        }
        R.outc[ci] = out;
    }
    // diagnostics: clusters that survived the lb prune, tracebacks walked (one atomic / lane)
    if (n_resolved) atomicAdd(R.diag, n_resolved);
    if (n_traces) atomicAdd(R.diag + 1, n_traces);
}

// ---------------------------------------------------------------------------------------------
// resolve (banded): no ring.  Every optimal path to an end cell x of cost c stays within c
// diagonals of x's diagonal (each indel moves one diagonal), and every cell that decides the
// tie-broken path (a minimum option of a path cell) lies on such a path, so the full DP
// (cost, origin, score) restricted to the 2H+1 diagonals around x (H >= c), evaluated from row 0
// with cutadapt's initialisation, reproduces cutadapt's origin and score of x exactly
// (DESIGN.md §3.5).  The band lives in registers: no LDS, full occupancy, no traceback.
// ---------------------------------------------------------------------------------------------
// Banded DP, two state words per cell: C = cost and P = origin * 256 + V, V = vertical moves on
// the chosen path.  The score follows from them at the end cell: with A adapter chars aligned,
// score = matches - mismatches - 2 * indels = A - 2 * cost - V (A = ie, or ie - i0 for a FRONT
// path entering at column 0 of row i0).  Cutadapt's pointer rule (_align.pyx) as selects:
//   diagonal if the characters match or cost(diag) <= min(up, left); else up (insertion) if
//   cost(up) <= cost(left); else left.  EDGE: the band reaches column 0 or beyond the view end.
template <int W, bool EDGE>
__device__ __forceinline__ void band_dp2(const uint8_t* rm, const Packed& pk,
                                         const TaskView& tv, bool front,
                                         int ie, int je, int& cost, int& origin, int& score) {
    constexpr int H = W / 2;
    constexpr int INF = 1 << 20;
    const int dx = je - ie;            // diagonal of the end cell; cell k <-> diagonal dx-H+k
    const int n = (int)tv.len;
    int C[W], P[W];
#pragma unroll
    for (int k = 0; k < W; ++k) {      // row 0: free start in the read
        const int jj = dx - H + k;
        C[k] = (EDGE && (jj < 0 || jj > n)) ? INF : 0;
        P[k] = jj * 256;
    }
    // read codes of row i, cell k: view position i - 1 + dx - H + k; a 48-position window of
    // three 16-code words (w0 current, w1 next, w2 prefetched) advancing 16 rows at a time
    int base = dx - H;
    uint32_t w0, n0, w1, n1;
    Chunk16 r2 = chunk16_load(pk, tv, base + 32);   // the third chunk stays in flight
    {
        const Chunk16 r0 = chunk16_load(pk, tv, base), r1 = chunk16_load(pk, tv, base + 16);
        chunk16_codes(tv, base, r0, w0, n0);
        chunk16_codes(tv, base + 16, r1, w1, n1);
    }
    int o = 0;
    uint32_t rnext = rm[0];           // rm[i * kMaxAdapters]: row i's match mask (row-major table)
    for (int i = 1; i <= ie; ++i) {
        if (o == 16) {                 // uniform: every lane advances one row per iteration
            w0 = w1;
            n0 = n1;
            chunk16_codes(tv, base + 32, r2, w1, n1);
            base += 16;
            // the band's last cell reads view position dx - H + ie + W - 2: no fetch past it
            if (base + 32 <= dx - H + ie + W - 2) r2 = chunk16_load(pk, tv, base + 32);
            o = 0;
        }
        const uint32_t codes = o ? __builtin_amdgcn_alignbit(w1, w0, 2 * o) : w0;
        const uint32_t nb = ((n1 << 16) | n0) >> o;
        const uint32_t rmask = rnext;
        rnext = rm[min(i, 63) * kMaxAdapters];
        int lc = INF, lp = 0;          // left neighbour (same row, already updated)
#pragma unroll
        for (int k = 0; k < W; ++k) {
            const int uc = (k + 1 < W) ? C[(k + 1) % W] : INF;
            const int up = (k + 1 < W) ? P[(k + 1) % W] : 0;
            const uint32_t code = (codes >> (2 * k)) & 3u;
            const bool eq = ((rmask >> code) & 1u) > ((nb >> k) & 1u);   // N matches nothing
            const int mn = min(lc, uc);
            const int ip = uc <= lc ? up + 1 : lp;
            const bool td = eq || C[k] <= mn;
            int c = td ? C[k] + (eq ? 0 : 1) : mn + 1;
            int pp = td ? P[k] : ip;
            if constexpr (EDGE) {
                const int jj = i + dx - H + k;
                if (jj == 0) {                         // column 0: cutadapt's initialisation
                    c = front ? 0 : i;
                    pp = front ? -i * 256 : i;
                }
                if (jj < 0 || jj > n) c = INF;
            }
            C[k] = c;
            P[k] = pp;
            lc = c;
            lp = pp;
        }
        ++o;
    }
    cost = C[H];
    origin = P[H] >> 8;
    const int v = P[H] & 255;
    score = ie - max(-origin, 0) - 2 * cost - v;
}

// 16 no-match bits -> the even bits of a word (bit k -> bit 2k), aligned with 2-bit codes.
__device__ __forceinline__ uint32_t spread_even(uint32_t x) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    return (x | (x << 1)) & 0x55555555u;
}

// band_dp2 for a band inside the view (no column 0, no view end) and adapter rows of one code
// each (A/C/G/T; the block checks its panel): every cell is ONE packed word
//   S = cost << 9 | origin index << 3 | V
// (origin index: the row-0 band cell the chosen path starts from; V: its vertical moves).
// cutadapt's pointer rule — diagonal if the characters match or cost(diag) <= min(up, left),
// else up if cost(up) <= cost(left), else left — is the lexicographic minimum of (cost,
// preference) over the three moves with preference diagonal 0 < up 1 < left 2 (a matching
// diagonal costs at most either other move, since neighbouring cells differ by <= 1).  So a cell
// is one v_min3 over S_diag + mismatch << 9, S_up + (1 << 9 | 1 << 7 | 1) (an up move is one V)
// and S_left + (1 << 9 | 2 << 7), with the preference bits cleared afterwards.  The three options
// never tie in (cost, preference), so the low bits never decide.  V <= cost <= 7 on every path
// that can reach the end cell (costs never fall along a path), so on those cells the 3-bit V
// field cannot carry into the origin index; a cell of a larger cost is never chosen by one of a
// smaller cost.  Mismatches for a whole row: the row's code replicated to every 2-bit field,
// XORed with the 16 read codes; a field is nonzero where they differ (read N: never a match).
template <int W>
__device__ __forceinline__ void band_dp_fast(const uint8_t* rm, const Packed& pk,
                                             const TaskView& tv, int ie,
                                             int je, int& cost, int& origin, int& score) {
    static_assert(W <= 15, "origin index: 4 bits");
    constexpr int H = W / 2;
    constexpr uint32_t INF = 1u << 30;
    constexpr uint32_t UP = (1u << 9) | (1u << 7) | 1u, LEFT = (1u << 9) | (2u << 7);
    const int dx = je - ie;
    uint32_t S[W];
#pragma unroll
    for (int k = 0; k < W; ++k) S[k] = (uint32_t)k << 3;   // row 0: free start, cost 0
    int base = dx - H;
    uint32_t w0, n0, w1, n1;
    Chunk16 r2 = chunk16_load(pk, tv, base + 32);   // the third chunk stays in flight
    {
        const Chunk16 r0 = chunk16_load(pk, tv, base), r1 = chunk16_load(pk, tv, base + 16);
        chunk16_codes(tv, base, r0, w0, n0);
        chunk16_codes(tv, base + 16, r1, w1, n1);
    }
    n0 = spread_even(n0);
    n1 = spread_even(n1);
    int o = 0;
    uint32_t rnext = rm[0];
    for (int i = 1; i <= ie; ++i) {
        if (o == 16) {                 // uniform: every lane advances one row per iteration
            w0 = w1;
            n0 = n1;
            uint32_t n2;
            chunk16_codes(tv, base + 32, r2, w1, n2);
            n1 = spread_even(n2);
            base += 16;
            if (base + 32 <= dx - H + ie + W - 2) r2 = chunk16_load(pk, tv, base + 32);
            o = 0;
        }
        const uint32_t codes = o ? __builtin_amdgcn_alignbit(w1, w0, 2 * o) : w0;
        const uint32_t nbs = o ? __builtin_amdgcn_alignbit(n1, n0, 2 * o) : n0;
        const uint32_t rb = rnext;
        rnext = rm[min(i, 63) * kMaxAdapters];
        const uint32_t x = codes ^ (((rb >> 4) & 3u) * 0x55555555u);
        const uint32_t ne = x | (x >> 1) | nbs;   // bit 2k: cell k is a mismatch
        uint32_t left = INF;
#pragma unroll
        for (int k = 0; k < W; ++k) {
            const uint32_t d = S[k] + (__builtin_amdgcn_ubfe(ne, 2 * k, 1) << 9);
            const uint32_t u = (k + 1 < W) ? S[k + 1] + UP : INF;
            const uint32_t v = min(min(d, u), left + LEFT) & ~(3u << 7);
            S[k] = v;
            left = v;
        }
        ++o;
    }
    cost = (int)(S[H] >> 9);
    origin = dx - H + (int)((S[H] >> 3) & 15u);
    score = ie - 2 * cost - (int)(S[H] & 7u);
}

// The DP of one queued cell with the narrowest exact band for the wave: cells are sorted by cost
// before a DP pass, so a wave's cells share a cost (or two neighbouring ones) and the wave runs
// 2c + 1 diagonals for its largest cost c (wave-uniform branch; H >= c keeps the band exact).
template <int C, int CMAX, bool EDGE>
__device__ __forceinline__ void band_dp_cost(int wc, bool fast, const uint8_t* rm,
                                             const Packed& pk,
                                             const TaskView& tv, bool front, int ie, int je,
                                             int& cost, int& origin, int& score) {
    if constexpr (C < CMAX) {
        if (wc > C) {
            band_dp_cost<C + 1, CMAX, EDGE>(wc, fast, rm, pk, tv, front, ie, je, cost,
                                             origin, score);
            return;
        }
    }
    if constexpr (!EDGE) {
        if (fast) {   // block-uniform
            band_dp_fast<2 * C + 1>(rm, pk, tv, ie, je, cost, origin, score);
            return;
        }
    }
    band_dp2<2 * C + 1, EDGE>(rm, pk, tv, front, ie, je, cost, origin, score);
}

// Band kernel over one candidate list (costs CMIN..CMAX; cost-0 cells need no DP).  Every block
// takes 256 candidates at a time through cheap checks first (score upper bound against the slot's
// lower bound and current winner; cost-0 cells are pure diagonals), and appends the survivors to
// one of two LDS queues: band-interior cells, and cells whose band reaches column 0 or the view
// end.  A queue runs a DP pass whenever it holds 256 cells (and once more, partially, at the end),
// so the DP waves are full whatever the prune rate; a pass first sorts its cells by cost, so each
// wave runs the narrowest band its cells allow (band_dp_cost).  The slot's best is the minimum
// key over all its candidates (key order = locate's / best_match's / ReverseComplementer's order).
#ifndef DMX_BAND_SPLIT   // list 1 in two launches, cost 4 then cost 5 (0: one launch)
#define DMX_BAND_SPLIT 1
#endif
constexpr bool kBandSplit = DMX_BAND_SPLIT != 0;
template <int CMIN, int CMAX>
// Occupancy floors of list 0 (costs 1..3) and list 1 with kk <= 5: the DP passes wait on their
// cells' loads, and 8 / 6 waves per SIMD (64 / 80 VGPRs) measured 8.44 -> 8.28 ms
// per step on c2x24 against the compiler's 7 / 5 (list 0 then spills 2 VGPRs).  The kk <= 7
// variant keeps its registers.
#ifndef DMX_BAND_WAVES0
#define DMX_BAND_WAVES0 8
#endif
#ifndef DMX_BAND_WAVES1
#define DMX_BAND_WAVES1 6
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(
    CMAX <= 3 ? DMX_BAND_WAVES0 : (CMAX <= 5 ? DMX_BAND_WAVES1 : 1)))) void band_cand_kernel(
    RoundArgs R, int list, int cmask) {
    // s_rm[i * kMaxAdapters + a]: bit c = adapter a's char i matches read code c.  Row-major, so
    // the lanes of a wave (one row i, different adapters) read neighbouring bytes: no bank
    // conflicts (an adapter-major table put every adapter's row i in one of 4 banks).
    __shared__ uint8_t s_rm[kMaxAdapters * 64];
    __shared__ uint32_t s_q[2][512];                 // queued cells: [0] interior, [1] edge
    __shared__ uint8_t s_qc[2][512];                 // their costs
    __shared__ uint32_t s_sorted[256];
    __shared__ uint8_t s_sc[256];
    __shared__ uint32_t s_hist[8], s_nq[2], s_n;
    __shared__ uint32_t s_amk[kMaxAdapters];         // ad_word per adapter
    __shared__ int8_t s_bacc[72 * kMaxAdapters];     // acc tables
    const DevPanel* P = R.panel;
    const int A = P->n_adapters;
    for (int a = threadIdx.x; a < A; a += blockDim.x) s_amk[a] = ad_word(P->ad[a]);
    for (int x = threadIdx.x; x < 72 * A; x += blockDim.x) s_bacc[x] = P->ad[x / 72].acc[x % 72];
    // bits 0-3: codes adapter char i matches; bits 4-5: that code when it is exactly one
    __shared__ uint32_t s_multi;   // some adapter char matches more or fewer than one code
    if (threadIdx.x == 0) s_multi = 0;
    __syncthreads();
    for (int x = threadIdx.x; x < 64 * A; x += blockDim.x) {
        const int a = x >> 6, i = x & 63;
        const DevAdapter& ad = P->ad[a];
        uint32_t r = 0;
        for (int c = 0; c < 4; ++c) r |= (uint32_t)((ad.peq[c] >> i) & 1ull) << c;
        if (__popc(r) == 1) r |= (uint32_t)(__ffs(r) - 1) << 4;
        else if (i < (int)ad.m) s_multi = 1u;
        s_rm[i * kMaxAdapters + a] = (uint8_t)r;
    }
    if (threadIdx.x == 0) {
        s_nq[0] = 0;
        s_nq[1] = 0;
        s_n = 0;
    }
    __shared__ uint32_t s_spre[kShards + 1];
    ShardMap sm{s_spre, 0u};
    sm.load(R.cand_count + list * kShards * kShardStride, R.cand_scap);   // (barrier: above too)
    const uint32_t total = sm.total();
    const Cand* cl = R.cand[list];
    Outcome* outs = R.cand_out[list];
    const uint32_t wave = threadIdx.x >> 6;
    const bool fast = s_multi == 0;                  // (read after sm.load's barrier)

    // One DP pass over the top `cnt` (<= 256) cells of queue e (block-uniform call).
    auto dp_pass = [&](int e, uint32_t cnt) {
        const uint32_t lo = s_nq[e] - cnt;
        if (threadIdx.x < 8) s_hist[threadIdx.x] = 0;
        __syncthreads();
        uint32_t ci = 0, cost = 0, pos = 0;
        const bool have = threadIdx.x < cnt;
        if (have) {
            ci = s_q[e][lo + threadIdx.x];
            cost = s_qc[e][lo + threadIdx.x];
            pos = atomicAdd(&s_hist[cost], 1u);
        }
        __syncthreads();
        if (have) {
            uint32_t before = 0;
            for (uint32_t c = 0; c < cost; ++c) before += s_hist[c];
            s_sorted[before + pos] = ci;
            s_sc[before + pos] = (uint8_t)cost;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            s_nq[e] = lo;
            s_n += cnt;
        }
        if (64u * wave < cnt) {                      // waves with cells (wave-uniform)
            const uint32_t last = min(64u * wave + 63u, cnt - 1u);
            const int wc = (int)s_sc[last];          // the wave's largest cost (sorted)
            if (threadIdx.x < cnt) {
                const uint32_t cj = s_sorted[threadIdx.x];
                const Cand c = cl[cj];
                const uint32_t slot = slot_of(R, c.item, c.sub);
                const bool slot_in = DMX_BOUND(R.pk.bd, slots, slot, kBufSlot);
                const int cst = c.cost, iend = c.iend;
                const int j = (int)c.j;
                const AdLite ad = ad_lite(s_amk[c.a]);
                const int8_t* const acc = s_bacc + 72 * c.a;
                const uint64_t t = iend == ad.m ? (uint64_t)j : (uint64_t)c.len + 1 + iend;
                TaskView tv;
                tv.read = 0;
                tv.n = c.n;
                tv.strand = c.strand;
                tv.clean = c.clean != 0;
                tv.start = c.start;
                tv.len = c.len;
                view_off(R.pk, c.off, tv);
                tv.o = c.o;
                tv.a = c.a;
                int c2, origin, score;
#ifdef DMX_BAND_SKIP_DP   // timing A/B only (results invalid): the band stage without its DPs
                c2 = cst;
                origin = (int)(c.j) - iend;
                score = (int)wc;
                if (false)
#endif
                if (e == 0)
                    band_dp_cost<CMIN == 0 ? 1 : CMIN, CMAX, false>(
                        wc, fast, s_rm + c.a, R.pk, tv, ad.front, iend, j, c2,
                        origin, score);
                else
                    band_dp_cost<CMIN == 0 ? 1 : CMIN, CMAX, true>(
                        wc, fast, s_rm + c.a, R.pk, tv, ad.front, iend, j, c2,
                        origin, score);
                if (c2 != cst) atomicOr(R.flags, 2u);    // band / scan disagreement: bug
                const int lr = iend + (origin < 0 ? origin : 0);
                if (slot_in && lr >= 0 && cst <= (int)acc[lr]) {
                    Outcome out;
                    out.key = make_key(score, c.o, cst, c.a, t);
                    out.origin = origin;
                    out.pad = (int32_t)slot;             // select_cand needs no Cand reload
                    atomicMin(&R.winner[slot], (unsigned long long)out.key);
                    outs[cj] = out;
                }
            }
        }
        __syncthreads();
    };

    for (uint32_t base = blockIdx.x * blockDim.x; base < total; base += gridDim.x * blockDim.x) {
        const uint32_t ti = base + threadIdx.x;
        const uint32_t ci = ti < total ? sm.phys(ti) : 0u;
        Cand c{};
        if (ti < total) c = cl[ci];
        // cmask != 0: this launch takes the list's cells whose cost has its bit set (the others'
        // outcomes are written by the launch that takes them)
        if (ti < total && (cmask == 0 || ((cmask >> c.cost) & 1))) {
            const uint32_t slot = slot_of(R, c.item, c.sub);
            const bool slot_in = DMX_BOUND(R.pk.bd, slots, slot, kBufSlot);
            const int cost = c.cost, iend = c.iend;
            const int j = (int)c.j;
            const uint64_t t = iend == (int)(s_amk[c.a] & 255u) ? (uint64_t)j
                                                               : (uint64_t)c.len + 1 + iend;
            Outcome out;
            out.key = ~0ull;
            out.origin = 0;
            out.pad = 0;
            const int lrmax = min(iend, j + cost);
            const int ub = lrmax - 2 * cost;
            if (slot_in && viable_lb(R.lb[slot], lrmax, c.o, cost) &&
                make_key(ub, c.o, cost, c.a, t) <= R.winner[slot]) {
                if (cost == 0) {              // exact: the pointer chain is the pure diagonal
                    const int origin = j - iend;
                    const int score = j >= iend ? iend : j;
                    const int lr = iend + (origin < 0 ? origin : 0);
                    if (lr >= 0 && 0 <= (int)s_bacc[72 * c.a + lr]) {
                        out.key = make_key(score, c.o, 0, c.a, t);
                        out.origin = origin;
                        out.pad = (int32_t)slot;
                        atomicMin(&R.winner[slot], (unsigned long long)out.key);
                    }
                } else {
                    const int dx = j - iend;
                    const int H = CMAX;       // the widest band this kernel may run
                    const int e = (dx - H < 0 || j + H > (int)c.len) ? 1 : 0;
                    const uint32_t q = atomicAdd(&s_nq[e], 1u);
                    s_q[e][q] = ci;
                    s_qc[e][q] = (uint8_t)cost;
                }
            }
            outs[ci] = out;
        }
        __syncthreads();
        for (int e = 0; e < 2; ++e)                 // full passes (each queue ends below 256)
            while (s_nq[e] >= 256u) dp_pass(e, 256u);
        // every thread has read the queue counts before any thread pushes again (a fast wave's
        // next-round push would otherwise send a slow wave alone into dp_pass's barriers)
        __syncthreads();
    }
    for (int e = 0; e < 2; ++e)
        if (s_nq[e]) dp_pass(e, s_nq[e]);
    if (threadIdx.x == 0 && s_n) atomicAdd(R.diag + 1, s_n);
}

__global__ void select_cand_kernel(RoundArgs R) {
    __shared__ uint32_t s_spre[kShards + 1];
    for (int list = 0; list < 2; ++list) {
        ShardMap sm{s_spre, 0u};
        __syncthreads();   // the previous list's map is no longer read
        sm.load(R.cand_count + list * kShards * kShardStride, R.cand_scap);
        const uint32_t total = sm.total();
        for (uint32_t ti = blockIdx.x * blockDim.x + threadIdx.x; ti < total;
             ti += gridDim.x * blockDim.x) {
            const uint32_t ci = sm.phys(ti);
            const Outcome o = R.cand_out[list][ci];
            if (o.key == ~0ull) continue;
            const uint32_t slot = (uint32_t)o.pad;   // band_cand_kernel stores the cell's slot
            if (!DMX_BOUND(R.pk.bd, slots, slot, kBufSlot)) continue;
            if (R.winner[slot] == o.key) R.origin[slot] = o.origin;
        }
    }
}

// select: the cluster whose outcome is the slot's winner publishes its origin.
__global__ void select_kernel(RoundArgs R) {
    const uint32_t total = min(*R.cl_count, R.cl_cap);
    for (uint32_t ci = blockIdx.x * blockDim.x + threadIdx.x; ci < total;
         ci += gridDim.x * blockDim.x) {
        const Outcome o = R.outc[ci];
        if (o.key == ~0ull) continue;
        const Cluster c = R.cl[ci];
        const uint32_t slot = slot_of(R, c.item, c.sub);
        if (!DMX_BOUND(R.pk.bd, slots, slot, kBufSlot)) continue;
        if (R.winner[slot] == o.key) R.origin[slot] = o.origin;
    }
}

// ---------------------------------------------------------------------------------------------
// finalize
// ---------------------------------------------------------------------------------------------
// Decode a winning key into a cutadapt Match on a view of length vlen.
__device__ __forceinline__ void decode_match(uint64_t key, int origin, uint32_t vlen,
                                             const DevPanel* P, dmx_match& mt, int& a, int& o) {
    a = key_adapter(key);
    o = key_orient(key);
    const uint64_t t = key_t(key);
    int refstop, qstop;
    if (t <= vlen) {
        qstop = (int)t;
        refstop = P->ad[a].m;
    } else {
        refstop = (int)(t - vlen - 1);
        qstop = (int)vlen;
    }
    mt.rstop = qstop;
    mt.astop = (int16_t)refstop;
    if (origin >= 0) {
        mt.astart = 0;
        mt.rstart = origin;
    } else {
        mt.astart = (int16_t)(-origin);
        mt.rstart = 0;
    }
    mt.score = (int16_t)key_score(key);
    mt.errors = (int16_t)key_cost(key);
}

struct FinalArgs {
    const uint32_t* lens;
    const DevPanel* p0;
    const DevPanel* p1;
    const unsigned long long* winner;
    const int32_t* origin;
    dmx_result* res;
    ItemView* items;            // round-1 item list (out for finalize0, in for finalize1)
    uint32_t* n_items;
    uint32_t n_reads;
    int32_t mode;
    int32_t A0, A1;             // adapters per panel
    int32_t oslot;              // this round keeps one winner slot per (item, orientation)
    unsigned long long* counts; // (A0+1)*(A1+1) + 2
    // linked mode
    const unsigned long long* winner0;   // per (read, pair) front winners
    const int32_t* origin0;
    unsigned long long* linked_best;     // per read: best pair key
    Bounds bd;                           // DMX_DEBUG_BOUNDS: extents of the buffers above
};

// ---------------------------------------------------------------------------------------------
// linked adapters (-g F...R; adapters.py LinkedAdapter.match_to, both parts required):
//   round 0: one winner per (read, pair) = the front primer's own best cell on the read;
//   round 1: each pair with a front match scans its back primer on read[front.rstop:];
//   combine: best pair by summed score, then summed errors, then pair order.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void finalize0_linked_kernel(FinalArgs F) {
    __shared__ uint32_t s_nq, s_qbase;
    if (threadIdx.x == 0) s_nq = 0;
    __syncthreads();
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t nmine = 0, qi = 0;
    uint32_t n = 0;
    if (r < F.n_reads && DMX_BOUND(F.bd, reads, r, kBufRes) &&
        DMX_BOUND(F.bd, linked, r, kBufLinked) &&
        DMX_BOUND(F.bd, slots, (size_t)r * F.A0 + F.A0 - 1, kBufSlot)) {
        dmx_result out;
        out.bin1 = out.bin2 = -1;
        out.rc1 = out.rc2 = 0;
        out.flags = 0;
        out._pad = 0;
        out.m1 = dmx_match{0, 0, 0, 0, 0, 0};
        out.m2 = out.m1;
        F.res[r] = out;
        F.linked_best[r] = ~0ull;
        n = F.lens[r];
        for (int a = 0; a < F.A0; ++a) nmine += F.winner[(size_t)r * F.A0 + a] != ~0ull;
        if (nmine) qi = atomicAdd(&s_nq, nmine);   // LDS; one global atomic per block below
    }
    __syncthreads();
    if (threadIdx.x == 0) s_qbase = s_nq ? atomicAdd(F.n_items, s_nq) : 0u;
    __syncthreads();
    if (nmine) {
        uint32_t idx = s_qbase + qi;
        for (int a = 0; a < F.A0; ++a) {
            const uint64_t key = F.winner[(size_t)r * F.A0 + a];
            if (key == ~0ull) continue;
            dmx_match m;
            int aa, o;
            decode_match(key, F.origin[(size_t)r * F.A0 + a], n, F.p0, m, aa, o);
            ItemView v;
            v.read = r;
            v.strand = 0;
            v.pad = 0;
            v.only_adapter = (int16_t)a;
            v.start = (uint32_t)m.rstop;
            v.len = n - (uint32_t)m.rstop;
            if (DMX_BOUND(F.bd, items, idx, kBufItem)) F.items[idx] = v;
            ++idx;
        }
    }
}

__global__ __launch_bounds__(256) void finalize1_linked_kernel(FinalArgs F) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *F.n_items) return;
    if (!DMX_BOUND(F.bd, items, i, kBufItem) || !DMX_BOUND(F.bd, slots, i, kBufSlot)) return;
    const ItemView v = F.items[i];
    const uint64_t kb = F.winner[i];
    if (kb == ~0ull) return;
    const int a = v.only_adapter;
    if (!DMX_BOUND(F.bd, linked, v.read, kBufLinked)) return;
    const uint64_t kf = F.winner0[(size_t)v.read * F.A0 + a];
    const int sum = key_score(kf) + key_score(kb);
    const int err = key_cost(kf) + key_cost(kb);
    const uint64_t ck = ((uint64_t)(511 - sum) << 54) | ((uint64_t)err << 46) |
                        ((uint64_t)a << 38) | (uint64_t)i;
    atomicMin(&F.linked_best[v.read], (unsigned long long)ck);
}

__global__ __launch_bounds__(256) void finalize2_linked_kernel(FinalArgs F) {
    __shared__ unsigned int s_hist[kMaxAdapters + 1];
    for (int x = threadIdx.x; x <= F.A0; x += blockDim.x) s_hist[x] = 0;
    __syncthreads();
    // block-stride (kFinalGrid blocks): one flush of the pair histogram per block
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < F.n_reads;
         r += gridDim.x * blockDim.x) {
        const uint64_t ck = DMX_BOUND(F.bd, linked, r, kBufLinked) ? F.linked_best[r] : ~0ull;
        int b = -1;
        if (ck != ~0ull) {
            const uint32_t i = (uint32_t)(ck & ((1ull << 38) - 1));
            const int a = (int)((ck >> 38) & 255);
            if (!DMX_BOUND(F.bd, items, i, kBufItem) || !DMX_BOUND(F.bd, slots, i, kBufSlot) ||
                !DMX_BOUND(F.bd, reads, r, kBufRes))
                continue;
            const ItemView v = F.items[i];
            dmx_result& out = F.res[r];
            int aa, o;
            decode_match(F.winner0[(size_t)r * F.A0 + a], F.origin0[(size_t)r * F.A0 + a],
                         F.lens[r], F.p0, out.m1, aa, o);
            decode_match(F.winner[i], F.origin[i], v.len, F.p1, out.m2, aa, o);
            out.bin1 = out.bin2 = (int16_t)a;
            b = a;
        }
        atomicAdd(&s_hist[b + 1], 1u);
    }
    __syncthreads();
    for (int x = threadIdx.x; x <= F.A0; x += blockDim.x)
        if (s_hist[x] && DMX_BOUND(F.bd, counts, x * (F.A0 + 1) + x, kBufCount))
            atomicAdd(&F.counts[x * (F.A0 + 1) + x], (unsigned long long)s_hist[x]);
}

// The winning key of slot base `i` and its orientation.  With one slot per orientation,
// ReverseComplementer's rule: the reverse complement is used iff its best score is strictly
// greater than the forward one, an orientation without a match counting 0 — so the chosen
// orientation may have no match (o = 1, key = none: the read is written reverse-complemented
// and unmatched).  Returns the index of the chosen slot.
__device__ __forceinline__ uint32_t pick_winner(const FinalArgs& F, uint32_t i, uint64_t& key,
                                                int& o) {
    if (!DMX_BOUND(F.bd, slots, F.oslot ? 2 * (uint64_t)i + 1 : i, kBufSlot)) {
        key = ~0ull;
        o = 0;
        return 0;
    }
    if (!F.oslot) {
        key = F.winner[i];
        o = key != ~0ull ? key_orient(key) : 0;
        return i;
    }
    const uint64_t kf = F.winner[2 * i], kr = F.winner[2 * i + 1];
    const int sf = kf != ~0ull ? key_score(kf) : 0, sr = kr != ~0ull ? key_score(kr) : 0;
    o = sr > sf ? 1 : 0;
    key = o ? kr : kf;
    return 2 * i + (uint32_t)o;
}

// Round 0 epilogue (one thread per read): write m1/bin1, build the round-1 view (the
// round-0-trimmed sequence: FRONT -> view[rstop:], BACK -> view[:rstart]) and queue it.
// Block-stride over the reads (kFinalGrid blocks): the bin histogram is flushed once per block,
// not once per 256 reads (one global atomic per bin and block, on a few dozen addresses).
#ifndef DMX_FINAL_GRID
#define DMX_FINAL_GRID 2048
#endif
constexpr uint32_t kFinalGrid = DMX_FINAL_GRID;
__global__ __launch_bounds__(256) void finalize0_kernel(FinalArgs F) {
    __shared__ unsigned int s_hist[2 * (kMaxAdapters + 1) + 1];
    __shared__ uint32_t s_nq, s_qbase;
    const int nh = F.A0 + 1;
    for (int x = threadIdx.x; x < nh + 1; x += blockDim.x) s_hist[x] = 0;
    if (threadIdx.x == 0) s_nq = 0;
    __syncthreads();
    uint32_t n_rc = 0;
    for (uint32_t base = blockIdx.x * 256u; base < F.n_reads; base += gridDim.x * 256u) {
        const uint32_t r = base + threadIdx.x;
        ItemView v;
        uint32_t qi = ~0u;             // this read's slot in the block's share of the item list
        if (r < F.n_reads && DMX_BOUND(F.bd, reads, r, kBufRes)) {
            dmx_result out;
            out.bin1 = -1;
            out.bin2 = -1;
            out.rc1 = out.rc2 = 0;
            out.flags = 0;
            out._pad = 0;
            out.m1 = dmx_match{0, 0, 0, 0, 0, 0};
            out.m2 = out.m1;
            uint64_t key;
            int o;
            const uint32_t ws = pick_winner(F, r, key, o);
            out.rc1 = (uint8_t)o;
            if (key != ~0ull) {
                int a;
                const uint32_t n = F.lens[r];
                decode_match(key, F.origin[ws], n, F.p0, out.m1, a, o);
                out.bin1 = (int16_t)a;
                out.rc1 = (uint8_t)o;
                if (F.mode == DMX_MODE_TWO_ROUND) {
                    v.read = r;
                    v.strand = (uint8_t)o;
                    v.pad = 0;
                    v.only_adapter = -1;
                    if (F.p0->ad[a].where == kFront) {
                        v.start = (uint32_t)out.m1.rstop;
                        v.len = n - (uint32_t)out.m1.rstop;
                    } else {
                        v.start = 0;
                        v.len = (uint32_t)out.m1.rstart;
                    }
                    qi = atomicAdd(&s_nq, 1u);    // LDS; one global atomic per pass below
                } else {
                    atomicAdd(&s_hist[a + 1], 1u);
                }
            } else {
                atomicAdd(&s_hist[0], 1u);
            }
            n_rc += o ? 1u : 0u;
            F.res[r] = out;
        }
        __syncthreads();
        if (threadIdx.x == 0) {   // (the other threads wait at the barrier below)
            s_qbase = s_nq ? atomicAdd(F.n_items, s_nq) : 0u;
            s_nq = 0;
        }
        __syncthreads();
        if (qi != ~0u && DMX_BOUND(F.bd, items, s_qbase + qi, kBufItem)) F.items[s_qbase + qi] = v;
    }
    // reads taken reverse-complemented: one LDS atomic per wave
    n_rc = wave_sum(n_rc);
    if ((threadIdx.x & 63u) == 0 && n_rc) atomicAdd(&s_hist[nh], n_rc);
    __syncthreads();
    const int stride1 = F.mode == DMX_MODE_TWO_ROUND ? F.A1 + 1 : 1;
    const int ncounts = (F.A0 + 1) * stride1;
    for (int x = threadIdx.x; x < nh + 1; x += blockDim.x) {
        const unsigned int v = s_hist[x];
        if (!v) continue;
        const int ix = x == nh ? ncounts : x * stride1;
        if (DMX_BOUND(F.bd, counts, ix, kBufCount))
            atomicAdd(&F.counts[ix], (unsigned long long)v);
    }
}

// Round 1 epilogue (one thread per queued item): m2/bin2 and the (bin1, bin2) histogram.
__global__ __launch_bounds__(256) void finalize1_kernel(FinalArgs F) {
    extern __shared__ unsigned int s_hist2[];
    const int nbins = (F.A0 + 1) * (F.A1 + 1);
    for (int x = threadIdx.x; x < nbins + 1; x += blockDim.x) s_hist2[x] = 0;
    __syncthreads();
    const uint32_t n_items = *F.n_items;
    uint32_t n_rc = 0;
    // block-stride (kFinalGrid blocks): one flush of the (bin1, bin2) histogram per block
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n_items; i += gridDim.x * 256u) {
        if (!DMX_BOUND(F.bd, items, i, kBufItem)) break;
        const ItemView v = F.items[i];
        if (!DMX_BOUND(F.bd, reads, v.read, kBufRes)) continue;
        dmx_result& out = F.res[v.read];
        uint64_t key;
        int o;
        const uint32_t ws = pick_winner(F, i, key, o);
        int b = -1;
        out.rc2 = (uint8_t)o;
        if (key != ~0ull) {
            int a;
            decode_match(key, F.origin[ws], v.len, F.p1, out.m2, a, o);
            out.bin2 = (int16_t)a;
            b = a;
        }
        n_rc += o ? 1u : 0u;
        atomicAdd(&s_hist2[(out.bin1 + 1) * (F.A1 + 1) + (b + 1)], 1u);
    }
    n_rc = wave_sum(n_rc);
    if ((threadIdx.x & 63u) == 0 && n_rc) atomicAdd(&s_hist2[nbins], n_rc);
    __syncthreads();
    for (int x = threadIdx.x; x < nbins + 1; x += blockDim.x) {
        const unsigned int c = s_hist2[x];
        const int ix = x == nbins ? nbins + 1 : x;
        if (c && DMX_BOUND(F.bd, counts, ix, kBufCount))
            atomicAdd(&F.counts[ix], (unsigned long long)c);
    }
}

// ---------------------------------------------------------------------------------------------
// host-side launch sequence
// ---------------------------------------------------------------------------------------------
static int resolve_grid(const Ctx* c) {
    (void)c;
    return 256 * 8;   // grid-stride; one 64-lane block per CU is LDS-limited (ring)
}

// DMX_DEBUG_SYNC=1 (diagnostics): synchronise after every stage and name the one that failed,
// so a device fault is attributed to its kernel instead of to the next API call.
static bool debug_sync() {
    static const bool on = getenv("DMX_DEBUG_SYNC") != nullptr;
    return on;
}
#define DMX_DBG_SYNC(name)                                                                   \
    do {                                                                                      \
        if (debug_sync()) {                                                                   \
            const hipError_t e_ = hipStreamSynchronize(st);                                   \
            if (e_ != hipSuccess) {                                                           \
                fprintf(stderr, "dmx debug: %s (round %d): %s\n", name, round,                \
                        hipGetErrorString(e_));                                               \
                return DMX_E_HIP;                                                             \
            }                                                                                 \
        }                                                                                     \
    } while (0)

Bounds make_bounds(const Ctx* c, int kid) {
    Bounds b;
#ifdef DMX_DEBUG_BOUNDS
    b.lo = -(int64_t)kGuardWords;
    b.hi = (int64_t)c->cap_words + kGuardWords;   // both buffers: cap_words + 2 guards words
    b.slots = c->slot_cap;
    b.items = c->item_alloc;
    b.reads = c->n_reads;
    b.counts = c->n_counts;
    b.linked = c->cap_reads;
    b.rec = c->d_counters;
    b.kid = kid;
#else
    (void)c, (void)kid;
#endif
    return b;
}

hipError_t bounds_reset(Ctx* c, hipStream_t st) {
#ifdef DMX_DEBUG_BOUNDS
    return hipMemsetAsync(c->d_counters + kBoundsRec, 0, 4 * sizeof(uint32_t), st);
#else
    (void)c, (void)st;
    return hipSuccess;
#endif
}

int bounds_check(Ctx* c, const char* where) {
#ifdef DMX_DEBUG_BOUNDS
    static const char* const kKer[] = {
        "?", "filter_kernel", "verify_kernel", "iscreen_kernel", "iscreen4_kernel",
        "wscan_kernel", "scan_kernel", "band_cand_kernel<0,3>", "band_cand_kernel<4,5|7>",
        "select_cand_kernel", "resolve_kernel", "select_kernel", "finalize0_kernel",
        "finalize1_kernel", "finalize0_linked_kernel", "finalize1_linked_kernel",
        "finalize2_linked_kernel", "chop_kernel", "chop_big_kernel", "chop_start",
        "bounds_selftest_kernel", "pscreen_kernel"};
    static const char* const kBuf[] = {"?", "seq", "nmask", "winner slots", "items", "results",
                                       "counts", "reads", "linked keys", "candidates", "chop"};
    uint32_t rec[4];
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess)
        e = hipMemcpy(rec, c->d_counters + kBoundsRec, sizeof(rec), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        c->err = std::string(where) + ": " + hipGetErrorString(e);
        return DMX_E_HIP;
    }
    if (!rec[0]) return DMX_OK;
    const int k = (int)rec[0] - 1;
    const int64_t idx = (int64_t)(((uint64_t)rec[3] << 32) | rec[2]);
    char msg[256];
    snprintf(msg, sizeof msg, "%s: bounds violation in %s: %s index %lld outside its buffer",
             where, k > 0 && k < (int)(sizeof kKer / sizeof *kKer) ? kKer[k] : "?",
             rec[1] < sizeof kBuf / sizeof *kBuf ? kBuf[rec[1]] : "?", (long long)idx);
    c->err = msg;
    return DMX_E_STATE;
#else
    (void)c, (void)where;
    return DMX_OK;
#endif
}

// DMX_DEBUG_BOUNDS builds: one gather below the guard, one slot past the winner array and one
// in range, through the checked accessors (dmx_debug_bounds_selftest).
__global__ void bounds_selftest_kernel(Packed pk, uint64_t slot_probe, uint32_t* out) {
#ifdef DMX_DEBUG_BOUNDS
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    out[0] = code32(pk, (int64_t)(-16 * kGuardWords - 64));       // below the guard: refused
    out[1] = DMX_BOUND(pk.bd, slots, slot_probe, kBufSlot) ? 1u : 0u;
    out[2] = code32(pk, kMinOffset);                               // in range
#else
    (void)pk, (void)slot_probe, (void)out;
#endif
}

int bounds_selftest(Ctx* c, uint32_t* host_out) {
#ifdef DMX_DEBUG_BOUNDS
    if (!c->d_seq || !c->d_winner[0]) {
        c->err = "dmx_debug_bounds_selftest: load and run a batch first";
        return DMX_E_STATE;
    }
    uint32_t* d_out = nullptr;
    if (hipMalloc((void**)&d_out, 3 * sizeof(uint32_t)) != hipSuccess) return DMX_E_HIP;
    Packed pk;
    pk.seq = c->d_seq;
    pk.nmask = c->d_nmask;
    pk.bd = make_bounds(c, kKerSelfTest);
    hipMemsetAsync(c->d_counters + 3, 0, sizeof(uint32_t), c->stream);
    bounds_reset(c, c->stream);
    hipLaunchKernelGGL(bounds_selftest_kernel, dim3(1), dim3(64), 0, c->stream, pk,
                       (uint64_t)c->slot_cap, d_out);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess)
        e = hipMemcpy(host_out, d_out, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost);
    hipFree(d_out);
    if (e != hipSuccess) return DMX_E_HIP;
    return bounds_check(c, "dmx_debug_bounds_selftest");
#else
    (void)host_out;
    c->err = "dmx_debug_bounds_selftest: not a DMX_DEBUG_BOUNDS build";
    return DMX_E_UNSUPPORTED;
#endif
}

// The flat piece scan: which rounds it serves this exec, their combined table
// (rebuilt when a panel or the mode changes: every entry of round r tagged with r, the sampling
// stride the smallest of theirs — a piece's `step` consecutive sampled offsets cover any smaller
// power-of-two stride too) and two cell bitmaps per flat round sized to the batch.  Rounds whose
// tables do not fit together, one-orientation panels and DMX_NO_FLAT=1 take the per-part screen.
int prepare_flat(Ctx* c, hipStream_t st) {
    c->flat_rounds = 0;
    if (c->n_reads == 0 || c->mode == DMX_MODE_LINKED || std::getenv("DMX_NO_FLAT")) return DMX_OK;
    int want = 0;
    for (int r = 0; r < 2; ++r)
        if ((r == 0 || c->mode == DMX_MODE_TWO_ROUND) && c->panel[r].set && c->panel[r].filter &&
            c->panel[r].piece_step && c->panel[r].n_orient == 2)
            want |= 1 << r;
    if (!want) return DMX_OK;
    const size_t nsb = (c->n_words + kSuperNt / 16 - 1) / (kSuperNt / 16);
    if (nsb >= (1ull << 31) || c->n_words >= (1ull << 31)) return DMX_OK;
    if (c->flat_gen != c->panel_gen || c->flat_want != want) {
        c->flat_gen = c->panel_gen;
        c->flat_want = want;
        c->flat_step = 0;
        std::vector<std::pair<uint32_t, uint64_t>> ents;   // (8-mer, tagged entry)
        int step = 4, npc = 0;
        for (int r = 0; r < 2; ++r) {
            if (!(want >> r & 1)) continue;
            const DevPieces& Q = c->panel[r].pieces;
            step = std::min(step, (int)Q.step);
            npc += Q.n_pieces;
            for (int e = 0; e < Q.n_entries; ++e) {
                const uint64_t v = Q.entry[e];
                const int off = (int)((v >> 38) & 3u);
                ents.push_back({(uint32_t)(v >> (2 * off)) & 0xFFFFu, v | ((uint64_t)r << 56)});
            }
        }
        if (ents.empty() || ents.size() > (size_t)kMaxPieceEntries) return DMX_OK;
        std::sort(ents.begin(), ents.end());
        std::unique_ptr<DevPieces> T(new DevPieces());
        memset(T.get(), 0, sizeof(DevPieces));
        int nk = 0;
        for (size_t e = 0; e < ents.size(); ++e) {
            if (e == 0 || ents[e].first != ents[e - 1].first) {
                T->key[nk++] = (uint32_t)e;
                T->bitmap[ents[e].first >> 5] |= 1u << (ents[e].first & 31);
            }
            T->key[nk - 1] += 1u << 16;
            T->entry[e] = ents[e].second;
        }
        for (int w = 0, rk = 0; w < kPieceBitmapWords; ++w) {
            T->rank_base[w] = (uint16_t)rk;
            rk += __builtin_popcount(T->bitmap[w]);
        }
        T->on = 1;
        T->step = step;
        T->n_pieces = npc;
        T->n_keys = nk;
        T->n_entries = (int)ents.size();
        if (!c->d_pieces_flat &&
            hipMalloc((void**)&c->d_pieces_flat, sizeof(DevPieces)) != hipSuccess)
            return DMX_E_NOMEM;
        // the previous exec's scan may still read the old table
        if (hipStreamSynchronize(st) != hipSuccess ||
            hipMemcpy(c->d_pieces_flat, T.get(), sizeof(DevPieces), hipMemcpyHostToDevice) !=
                hipSuccess)
            return DMX_E_HIP;
        c->flat_lds = (size_t)kPieceLdsFixed + 8 * ((size_t)(nk + 1) / 2) + 8 * ents.size();
        c->flat_step = step;
    }
    if (!c->flat_step) return DMX_OK;   // the tables do not fit together: the per-part screen
    const size_t cw = (c->n_words + 31) / 32 + 2 * kCellGuardWords;
    for (int i = 0; i < 4; ++i) {
        if (!(want >> (i >> 1) & 1) || (c->d_cells[i] && c->cells_cap[i] >= cw)) continue;
        if (c->d_cells[i]) hipFree(c->d_cells[i]);
        c->d_cells[i] = nullptr;
        c->cells_cap[i] = 0;
        if (hipMalloc((void**)&c->d_cells[i], cw * 4) != hipSuccess) return DMX_E_NOMEM;
        c->cells_cap[i] = cw;
    }
    c->cells_words = cw;
    c->flat_rounds = want;
    return DMX_OK;
}

int launch_round(Ctx* c, int round, hipStream_t st) {
    RoundArgs R;
    R.pk.seq = c->d_seq;
    R.pk.nmask = c->d_nmask;
    R.pk.bd = make_bounds(c, 0);
    R.offs = c->d_offs;
    R.lens = c->d_lens;
    R.panel = c->d_panel[round];
    const HostPanel& hp = c->panel[round];
    const bool linked = c->mode == DMX_MODE_LINKED;
    R.per_task_slot = (linked && round == 0) ? 1 : 0;
    R.slot_div = c->orient_slot[round] ? hp.n : 0;
    if (round == 0) {
        R.items = nullptr;
        R.n_items_dev = nullptr;
        R.n_items = (uint32_t)c->n_reads;
        R.T = linked ? hp.n : hp.n * hp.n_orient;
    } else {
        R.items = c->d_items;
        R.n_items_dev = c->d_counters + 2;
        R.n_items = (uint32_t)c->item_cap;
        R.T = linked ? 1 : hp.n * hp.n_orient;
    }
    R.cl = c->d_cl[round];
    R.outc = c->d_outc[round];
    R.cl_count = c->d_counters + round;
    R.cl_cap = (uint32_t)c->cl_cap;
    R.flags = c->d_counters + 3;
    R.winner = c->d_winner[round];
    R.origin = c->d_origin[round];
    R.lb = c->d_lb[round];
    if (R.T > kScanBlock) return DMX_E_UNSUPPORTED;
    hipMemsetAsync(R.lb, 0, sizeof(int32_t) * (round == 0 ? c->slot_cap
                                                         : c->item_cap * (R.slot_div ? 2 : 1)),
                   st);

    const uint32_t rpb = kScanBlock / R.T;
    const uint32_t grid = (uint32_t)((R.n_items + rpb - 1) / rpb);
    R.diag = c->d_counters + 16 + 4 * round;
    R.win = c->d_win;
    R.win_count = c->d_shard + (kShWin + round) * kShards * kShardStride;
    R.win2 = c->d_win2;
    R.win2_count = c->d_shard + (kShWin2 + round) * kShards * kShardStride;
    R.win_cap = (uint32_t)c->win_cap;
    R.win_scap = (uint32_t)(c->win_cap / kShards);
    const bool band = c->band_ok[round] && !c->force_ring;
    R.band = band ? 1 : 0;
    for (int l = 0; l < 2; ++l) {
        R.cand[l] = c->d_cand[round][l];
        R.cand_out[l] = c->d_cand_out[round][l];
    }
    R.cand_count = c->d_shard + (kShCand + 2 * round) * kShards * kShardStride;
    R.cand_cap = (uint32_t)c->cand_cap;
    R.cand_scap = (uint32_t)(c->cand_cap / kShards);
    R.screen = (hp.filter && hp.verify && hp.screen && !linked && !c->no_screen &&
                (uint64_t)c->win_cap * (uint64_t)hp.n < (1ull << 32)) ? 1 : 0;
    R.tasks = c->d_tasks;
    R.task_count = c->d_shard + (kShTasks + round) * kShards * kShardStride;
    R.task_cap = (uint32_t)c->task_cap;
    R.task_scap = (uint32_t)(c->task_cap / kShards);
    R.pieces = c->d_pieces[round];
    R.ftask = c->d_ftask;
    R.ftask_count = c->d_shard + (kShFtask + round) * kShards * kShardStride;
    R.ftask_scap = (uint32_t)(c->ftask_cap / kShards);
    // window code slots: band-mode window scans of this pipeline, offsets that leave tag bits
    R.stage = (DMX_STAGE_SLOTS && c->d_stage && !linked && hp.filter && band && c->use_stage &&
               (uint64_t)c->n_words * 16 < (1ull << kOffBits))
                  ? c->d_stage : nullptr;
    R.stage_cap = (uint32_t)c->stage_cap;
    R.pk.stage = c->d_stage;
    R.n_words = (uint32_t)c->n_words;
    R.nsb = (uint32_t)((c->n_words + kSuperNt / 16 - 1) / (kSuperNt / 16));
    R.round = round;
    for (int i = 0; i < 4; ++i)
        R.cells[i] = (c->flat_rounds >> (i >> 1) & 1) ? c->d_cells[i] + kCellGuardWords : nullptr;
    hipEventRecord(c->ev[round * 3 + 0], st);
    if (round == 0 && c->flat_rounds) {   // the flat scan: every flat round's marks at once
        for (int i = 0; i < 4; ++i)
            if (R.cells[i]) hipMemsetAsync(c->d_cells[i], 0, 4 * c->cells_words, st);
        RoundArgs S = R;
        S.pieces = c->d_pieces_flat;
        const uint32_t sgrid = std::min<uint32_t>((R.nsb + 3) / 4, kScanGrid);
        const size_t lds = c->flat_lds;
        set_kid(S.pk.bd, kKerPieces);
        if (sgrid > 0) {
            if (c->flat_step == 4)
                hipLaunchKernelGGL(pscan_kernel<4>, dim3(sgrid), dim3(kScanBlock), lds, st, S);
            else if (c->flat_step == 2)
                hipLaunchKernelGGL(pscan_kernel<2>, dim3(sgrid), dim3(kScanBlock), lds, st, S);
            else
                hipLaunchKernelGGL(pscan_kernel<1>, dim3(sgrid), dim3(kScanBlock), lds, st, S);
        }
        DMX_DBG_SYNC("pscan_kernel");
    }
    if (hp.filter && !linked) {   // linked primers: short, no shared suffix block; plain scan
        if (hp.piece_step) {      // piece screen, then the filter on its tasks
            set_kid(R.pk.bd, kKerPieces);
            if (c->flat_rounds >> round & 1) {   // the flat scan's marks -> filter tasks
                const uint32_t cgrid = std::min<uint32_t>((R.n_items + 255) / 256, 2048u);
                if (cgrid > 0)
                    hipLaunchKernelGGL(pcompact_kernel, dim3(cgrid), dim3(kScanBlock), 0, st, R);
                DMX_DBG_SYNC("pcompact_kernel");
            } else {   // the per-part screen
                const DevPieces& Q = hp.pieces;   // LDS image: bitmap + rank base, keys, entries
                const size_t lds = (size_t)kPieceLdsFixed + 8 * ((Q.n_keys + 1) / 2) +
                                   8 * (size_t)Q.n_entries;
                const uint32_t pgrid =
                    (uint32_t)((R.n_items + kPsItemsPerBlock - 1) / kPsItemsPerBlock);
                const uint32_t grid = std::min<uint32_t>(pgrid, kPieceGrid);
                if (pgrid > 0) {
                    if (hp.piece_step == 4)
                        hipLaunchKernelGGL(pscreen_kernel<4>, dim3(grid), dim3(kScanBlock), lds, st, R);
                    else if (hp.piece_step == 2)
                        hipLaunchKernelGGL(pscreen_kernel<2>, dim3(grid), dim3(kScanBlock), lds, st, R);
                    else
                        hipLaunchKernelGGL(pscreen_kernel<1>, dim3(grid), dim3(kScanBlock), lds, st, R);
                }
                DMX_DBG_SYNC("pscreen_kernel");
            }
            hipEventRecord(c->ev[15 + round], st);
            set_kid(R.pk.bd, kKerFilter);
            hipLaunchKernelGGL(ftask_kernel, dim3(256 * 8), dim3(kScanBlock), 0, st, R);
            DMX_DBG_SYNC("ftask_kernel");
        } else {
            const uint64_t nviews = (uint64_t)R.n_items * (uint64_t)hp.n_orient;
            const uint32_t fgrid =
                (uint32_t)((nviews + kSegViewsPerBlock - 1) / kSegViewsPerBlock);
            set_kid(R.pk.bd, kKerFilter);
            if (fgrid > 0)
                hipLaunchKernelGGL(filter_kernel, dim3(fgrid), dim3(kScanBlock), 0, st, R);
            DMX_DBG_SYNC("filter_kernel");
        }
        hipEventRecord(c->ev[9 + 2 * round], st);
        set_kid(R.pk.bd, kKerVerify);
        if (hp.verify)
            hipLaunchKernelGGL(verify_kernel, dim3(256 * 8), dim3(kScanBlock), 0, st, R);
        DMX_DBG_SYNC("verify_kernel");
        if (R.stage) {   // window code slots for the screen, the window scan and the band
            set_kid(R.pk.bd, kKerVerify);
            const bool v = hp.pre_len != 0;   // the window scan's list (wscan_kernel)
            hipLaunchKernelGGL(wstage_kernel, dim3(256 * 8), dim3(kScanBlock), 0, st, R,
                               v ? c->d_win2 : c->d_win, v ? R.win2_count : R.win_count,
                               hp.stage_back, hp.stage_lo);
            DMX_DBG_SYNC("wstage_kernel");
        }
        hipEventRecord(c->ev[10 + 2 * round], st);
        if (R.screen) {   // packed quads for panels of <= 32 adapters (DMX_SCREEN_V1: A/B)
            if (hp.n <= 4 * kScreenQuads && !c->screen_v1) {
                set_kid(R.pk.bd, kKerScreen4);
                hipLaunchKernelGGL(iscreen4_kernel, dim3(256 * 16), dim3(kScanBlock), 0, st, R);
            } else {
                set_kid(R.pk.bd, kKerScreen);
                hipLaunchKernelGGL(iscreen_kernel, dim3(256 * 16), dim3(kScanBlock), 0, st, R);
            }
        }
        DMX_DBG_SYNC("iscreen");
        hipEventRecord(c->ev[13 + round], st);
        set_kid(R.pk.bd, kKerWscan);
        // (near-start tasks in a second launch, pruned against the slot lower bounds of the
        // first: measured no faster, profiles/r6_ab_wscan_near_phase_*.txt)
        if (band) hipLaunchKernelGGL(wscan_kernel<true>, dim3(256 * 16), dim3(kScanBlock), 0, st, R);
        else hipLaunchKernelGGL(wscan_kernel<false>, dim3(256 * 16), dim3(kScanBlock), 0, st, R);
        DMX_DBG_SYNC("wscan_kernel");
    } else if (grid > 0) {
        hipEventRecord(c->ev[9 + 2 * round], st);
        hipEventRecord(c->ev[10 + 2 * round], st);
        hipEventRecord(c->ev[13 + round], st);
        set_kid(R.pk.bd, kKerScan);
        if (band) hipLaunchKernelGGL(scan_kernel<true>, dim3(grid), dim3(kScanBlock), 0, st, R);
        else hipLaunchKernelGGL(scan_kernel<false>, dim3(grid), dim3(kScanBlock), 0, st, R);
        DMX_DBG_SYNC("scan_kernel");
    }
    hipEventRecord(c->ev[round * 3 + 1], st);
    if (band) {
        set_kid(R.pk.bd, kKerBand0);
        // (list 0 in two launches, costs 0..2 then 3, measured slower: round 2's band 2.15 ->
        // 2.30 ms, profiles/r6_ab_band_list0_split.txt; the exact cost-0 cells first, then costs 1..3,
        // 2.98 -> 3.21 ms, profiles/r6_ab_band_zero_first.txt)
        hipLaunchKernelGGL((band_cand_kernel<0, 3>), dim3(256 * 8), dim3(256), 0, st, R, 0, 0);
        DMX_DBG_SYNC("band_cand_kernel<0, 3>");
        set_kid(R.pk.bd, kKerBand1);
        if (c->band_wide[round] && kBandSplit) {   // costs 4, 5, then 6..7 (as below)
            hipLaunchKernelGGL((band_cand_kernel<4, 7>), dim3(256 * 4), dim3(256), 0, st, R, 1, 16);
            hipLaunchKernelGGL((band_cand_kernel<4, 7>), dim3(256 * 4), dim3(256), 0, st, R, 1, 32);
            hipLaunchKernelGGL((band_cand_kernel<4, 7>), dim3(256 * 4), dim3(256), 0, st, R, 1, 192);
        } else if (c->band_wide[round]) {
            hipLaunchKernelGGL((band_cand_kernel<4, 7>), dim3(256 * 4), dim3(256), 0, st, R, 1, 0);
        } else if (kBandSplit) {
            // every cost in list 1 is <= 5 (a band of 2 * 5 + 1 diagonals is exact).  The cost-4
            // cells first: their exact keys are in the winner slots when the cost-5 launch
            // screens its cells (a cost-5 cell's score is at most 49 of 59, below a cost-4
            // winner's unless that has 2+ deletions), so fewer cost-5 DPs run (band 3.74 / 2.81
            // -> 2.98 / 2.15 ms per round, profiles/r6_ab_band_list1_split.txt).
            hipLaunchKernelGGL((band_cand_kernel<4, 5>), dim3(256 * 4), dim3(256), 0, st, R, 1, 16);
            hipLaunchKernelGGL((band_cand_kernel<4, 5>), dim3(256 * 4), dim3(256), 0, st, R, 1, 32);
        } else {
            hipLaunchKernelGGL((band_cand_kernel<4, 5>), dim3(256 * 4), dim3(256), 0, st, R, 1, 0);
        }
        DMX_DBG_SYNC("band_cand_kernel<4, 5|7>");
        set_kid(R.pk.bd, kKerSelectCand);
        hipLaunchKernelGGL(select_cand_kernel, dim3(1024), dim3(256), 0, st, R);
        DMX_DBG_SYNC("select_cand_kernel");
        hipEventRecord(c->ev[round * 3 + 2], st);
        return hipGetLastError() == hipSuccess ? DMX_OK : DMX_E_HIP;
    }
    const size_t tabs = (size_t)144 * hp.n;
    static bool attr_set = false;
    if (!attr_set) {   // dynamic LDS above 64 KiB must be allowed explicitly
        hipFuncSetAttribute((const void*)resolve_kernel<kRingSmall>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        hipFuncSetAttribute((const void*)resolve_kernel<kRingLarge>,
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    set_kid(R.pk.bd, kKerResolve);
    if (c->ring_small[round])
        hipLaunchKernelGGL(resolve_kernel<kRingSmall>, dim3(resolve_grid(c)), dim3(kResolveBlock),
                           (size_t)kRingSmall * kResolveBlock * 16 + tabs, st, R);
    else
        hipLaunchKernelGGL(resolve_kernel<kRingLarge>, dim3(resolve_grid(c)), dim3(kResolveBlock),
                           (size_t)kRingLarge * kResolveBlock * 16 + tabs, st, R);
    DMX_DBG_SYNC("resolve_kernel");
    set_kid(R.pk.bd, kKerSelect);
    hipLaunchKernelGGL(select_kernel, dim3(1024), dim3(256), 0, st, R);
    DMX_DBG_SYNC("select_kernel");
    hipEventRecord(c->ev[round * 3 + 2], st);
    return hipGetLastError() == hipSuccess ? DMX_OK : DMX_E_HIP;
}

__global__ void mask_scatter_kernel(uint32_t* mask, const uint32_t* exc, uint32_t n,
                                    uint32_t base) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        mask[exc[i] - base] = exc[n + i];
}

__global__ void rebase_offsets_kernel(uint64_t* offs, uint32_t n, uint64_t g0) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        offs[i] -= g0;
}

int launch_rebase_offsets(uint64_t* offs, uint32_t n, uint64_t g0, hipStream_t st) {
    if (!n) return DMX_OK;
    const uint32_t grid = min((n + 255u) / 256u, 2048u);
    hipLaunchKernelGGL(rebase_offsets_kernel, dim3(grid), dim3(256), 0, st, offs, n, g0);
    return hipGetLastError() == hipSuccess ? DMX_OK : DMX_E_HIP;
}

int launch_mask_scatter(uint32_t* mask, const uint32_t* d_exc, uint32_t n, uint32_t base,
                        hipStream_t st) {
    if (!n) return DMX_OK;
    const uint32_t grid = min((n + 255u) / 256u, 1024u);
    hipLaunchKernelGGL(mask_scatter_kernel, dim3(grid), dim3(256), 0, st, mask, d_exc, n, base);
    return hipGetLastError() == hipSuccess ? DMX_OK : DMX_E_HIP;
}

int launch_finalize(Ctx* c, int round, hipStream_t st) {
    FinalArgs F;
    F.lens = c->d_lens;
    F.p0 = c->d_panel[0];
    F.p1 = c->d_panel[1];
    F.winner = c->d_winner[round];
    F.origin = c->d_origin[round];
    F.res = c->d_res;
    F.items = c->d_items;
    F.n_items = c->d_counters + 2;
    F.n_reads = (uint32_t)c->n_reads;
    F.mode = c->mode;
    F.A0 = c->panel[0].n;
    F.A1 = c->mode == DMX_MODE_SINGLE ? 0 : c->panel[1].n;
    F.oslot = c->orient_slot[round] ? 1 : 0;
    F.counts = c->d_counts;
    F.winner0 = c->d_winner[0];
    F.origin0 = c->d_origin[0];
    F.linked_best = c->d_linked;
    F.bd = make_bounds(c, kKerFin0);
    if (c->mode == DMX_MODE_LINKED) {
        const uint32_t gr = (uint32_t)((c->n_reads + 255) / 256);
        if (round == 0) {
            set_kid(F.bd, kKerFin0L);
            if (gr) hipLaunchKernelGGL(finalize0_linked_kernel, dim3(gr), dim3(256), 0, st, F);
        } else {
            const uint32_t gi = (uint32_t)((c->item_cap + 255) / 256);
            set_kid(F.bd, kKerFin1L);
            if (gi) hipLaunchKernelGGL(finalize1_linked_kernel, dim3(gi), dim3(256), 0, st, F);
            set_kid(F.bd, kKerFin2L);
            if (gr)
                hipLaunchKernelGGL(finalize2_linked_kernel, dim3(std::min(gr, kFinalGrid)),
                                   dim3(256), 0, st, F);
        }
        DMX_DBG_SYNC("finalize_linked");
        hipEventRecord(c->ev[6 + round], st);
        return hipGetLastError() == hipSuccess ? DMX_OK : DMX_E_HIP;
    }
    if (round == 0) {
        const uint32_t grid = (uint32_t)std::min<size_t>((c->n_reads + 255) / 256, kFinalGrid);
        if (grid) hipLaunchKernelGGL(finalize0_kernel, dim3(grid), dim3(256), 0, st, F);
    } else {
        const uint32_t grid = (uint32_t)std::min<size_t>((c->item_cap + 255) / 256, kFinalGrid);
        const size_t shm = sizeof(unsigned int) * ((size_t)(F.A0 + 1) * (F.A1 + 1) + 1);
        set_kid(F.bd, kKerFin1);
        if (grid) hipLaunchKernelGGL(finalize1_kernel, dim3(grid), dim3(256), shm, st, F);
    }
    DMX_DBG_SYNC("finalize");
    hipEventRecord(c->ev[6 + round], st);
    return hipGetLastError() == hipSuccess ? DMX_OK : DMX_E_HIP;
}

}  // namespace dmx
