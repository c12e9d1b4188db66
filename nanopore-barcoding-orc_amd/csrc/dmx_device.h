// dmx_device.h — device-side data layout and primitives of the demultiplexer (gfx950 / CDNA4).
//
// What the kernels compute is cutadapt 4.9's Aligner.locate (upstream cutadapt/_align.pyx;
// restated in oracle/cutadapt_oracle.c) for every (read, adapter, orientation) of a round, then
// AdapterCutter.best_match + ReverseComplementer selection.  Reference call sites:
// scripts/02_cutadapt_loop.sh:64-72 (round 1, -g file:SP5 --rc), :91-103 (round 2, -a file:SP27rc
// --rc); scripts/04_cleaning_primers.sh:371-388 (linked primers).
//
// Algorithm:
//   scan    — one lane per (read, orientation, adapter) runs a Myers/Hyyro bit-vector over the
//             whole read: one 64-bit word per adapter (m <= 64), giving the exact unit-cost DP
//             last-row cost D(m, j) of every column.  Columns with D <= k form candidate
//             clusters (plus the final column for 3' adapters).
//   resolve — one lane per cluster re-runs Myers from column j1-m-k-1 (restricted start; exact
//             for every cell of cost <= k, proof in DESIGN.md), keeps the last 128 columns of
//             (Pv, Mv) in LDS, and walks cutadapt's tie-broken pointer chain back from each
//             candidate cell to recover (origin, score) exactly; keeps cutadapt's best cell.
//   select/finalize — 64-bit packed keys make "best over adapters and orientations" one
//             atomicMin per read.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dmx {

constexpr int kMaxAdapters = 64;
constexpr int kMaxLen = 64;       // adapter length limit: one 64-bit Myers word
constexpr int kRingSmall = 74;    // resolve ring when every adapter has m + k + 2 + 4 <= 74
constexpr int kRingLarge = 128;   // otherwise (one 64-lane block per CU)
constexpr int kScanBlock = 256;
constexpr int kResolveBlock = 64;

enum : uint8_t { kFront = 1, kBack = 2 };

// One adapter of a panel as the kernels see it.
struct DevAdapter {
    uint64_t peq[8];    // match bit-vectors per read code: 0..3 = A,C,G,T; 4..7 = non-ACGT (0)
    int8_t acc[72];     // acc[L]: max accepted cost for an alignment covering L adapter chars,
                        // -1 if never (L < min_overlap).  Precomputed on the host in IEEE double
                        // exactly as `cost <= effective_length * max_error_rate` (_align.pyx).
    int8_t pacc[72];    // prefix maximum of acc: a last-row cell (m, j) of cost d can only be
                        // accepted if d <= pacc[min(m, j + d)] (its aligned adapter length is
                        // at most min(m, j + d)); prunes the always-cheap cells near column 0.
    uint8_t m;          // adapter length
    uint8_t k;          // int(max_error_rate * m): band used to size the resolve window
    uint8_t where;      // kFront / kBack
    int8_t kk;          // max_L acc[L]: no cell with a larger cost can ever be accepted
    uint8_t pad[4];
};
static_assert(sizeof(DevAdapter) == 216, "DevAdapter layout");

struct DevPanel {
    int32_t n_adapters;
    int32_t n_orient;    // 2 with --rc, else 1
    int32_t where;       // kFront / kBack when uniform, else 0
    // Shared-suffix filter (0 = disabled): the last `filter_len` (<= 32) characters are common
    // to every adapter of the panel, so any acceptable last-row cell (m, j) of any adapter has a
    // block cost b(j) <= its own cost.  One 32-bit Myers scan per read view
    // finds all columns where some adapter may end; per-adapter scans run only there.
    int32_t filter_len;
    int32_t kf;          // max over adapters of kk
    int32_t max_mk;      // max over adapters of m + k + 1
    // rows the filter kernel scans: the LAST scan_len (<= filter_len) rows of the block.  A
    // suffix of the block ends at the same column and costs no more, so its cost is a lower
    // bound of b(j) and the filter stays a necessary condition (verify / screen keep filter_len)
    int32_t scan_len;
    // reach of the exact stages before a window, in view positions (window scan start m + k + 1,
    // band start m + 7), rounded up to 16; 0 = no clean flags (every window loads the mask).  The
    // filter marks a window `clean` when the no-match mask is zero over [j1 - clean_reach, j2]
    // 
    int32_t clean_reach;
    uint32_t filter_peq[8];
    int8_t pf[72];       // max over adapters of pacc[L]
    // Shared-prefix verification (0 = disabled): the first `pre_len` (<= 32) characters are common
    // to every adapter and pre_len + filter_len <= min m, so a full alignment of cost c ending at
    // column j costs >= b(j) + min D_pre(j') over j' in [j - off_max - c, j - off_min + c]
    // (off = m - pre_len), and a 3' last-column cell needs the prefix near the read end.
    int32_t pre_len;
    int32_t off_min, off_max;
    int32_t m_max;
    // Index screen: every adapter is P + I_a + S with |I_a| in 1..32.
    int32_t jsplit;      // FRONT: a last-row cell at column j >= jsplit contains every row of I_a
    int32_t pshared;     // acceptance tables agree on rows <= pre_len for every adapter, so a
                         // 3' last-column cell inside P is identical for all adapters
    uint32_t pre_peq[8];
    DevAdapter ad[kMaxAdapters];
};

// A column range of one (item, orientation) that the per-adapter window scan must cover.
// info (set by verify, read by the index screen): bits 0-7 = a lower bound of the shared-prefix
// block's cost in every full alignment ending in the window (0 if not computed), bits 8-15 = the
// same for the prefix block ending near the view end (3' last-column cells), bit 16 = some 3'
// last-column cell inside the shared prefix (rows <= pre_len) may be accepted, bits 24-31 = the
// prefix block's bound for 3' cells ending inside an index block (P within l_max - 1 + kf of the
// end).
struct Window {
    uint32_t item;
    uint8_t o;
    uint8_t lastcol;     // 3' panel: window ends at the final column (last-column cells)
    uint8_t strand;      // oriented view of the item (copied so the window scan needs no
    uint8_t bmin;        // dependent loads): strand, start, len, read length n, first nt off;
    uint32_t j1, j2;     // bmin = min suffix-block cost over the hits (255 = no hit).
                         // strand bit 1 (kWinClean): the view's no-match mask is zero over
                         // [j1 - clean_reach, j2], so the exact stages need not load it
    uint32_t n, start, len, info;
    uint64_t off;
};
static_assert(sizeof(Window) == 40 && offsetof(Window, off) == 32, "Window layout");
constexpr uint8_t kWinClean = 2;   // Window.strand bit 1

constexpr int kStageCap = 256;    // LDS staging of emitted records per block
// Appendable lists are split into kShards shards, each with its own counter (a slot of
// Ctx::d_shard) and a fixed capacity: one device-scope counter that every wave of the grid
// appends through serialises them (measured: the window scan ran at the counter's atomic rate).
#ifndef DMX_SHARDS
#define DMX_SHARDS 16
#endif
constexpr int kShards = DMX_SHARDS;
constexpr int kShardStride = 32;   // u32 words between counters: one 128-B line each
enum ShardList { kShWin = 0, kShWin2 = 2, kShTasks = 4, kShCand = 6, kShFtask = 10, kShLists = 12 };

// ---------------------------------------------------------------------------------------------
// Piece screen.  Every adapter a of an ACGT panel is cut into K_a + 1 disjoint
// row pieces, K_a = acc[m_a] (the largest cost of an accepted alignment covering all m_a rows).
// An alignment of all rows with <= K_a edits leaves at least one piece without an edit, i.e. an
// exact copy of that piece in the read, and it ends at column e + (m_a - r1) +- K_a where e is the
// position after the copy and r1 the piece's end row.  The screen finds exact copies of the
// pieces (and of their reverse complements, for the other orientation) and sends the shared-suffix
// filter only to the 16-position cells where such an alignment can end, plus the FRONT
// partial-alignment cells at the view start; a 3' view's last-column window is emitted directly.
// ---------------------------------------------------------------------------------------------
constexpr int kMaxPieces = 1024;         // distinct (piece, orientation) records
constexpr int kMaxPieceEntries = 2048;   // (sampled 8-mer, piece, offset) entries
constexpr int kPieceK = 8;               // sampled k-mer length (a 64 Ki-bit LDS bitmap)
constexpr int kPieceBitmapWords = 1 << (2 * kPieceK - 5);

// An entry of the piece table (one per (piece, sampled offset)), packed in 64 bits: the piece's
// 2-bit codes in view-0 read order (nt i at bits 2i; orientation 1: the reverse complement),
// its length, orientation, the sampled 8-mer's offset inside it, and the range of alignment end
// columns after the copy (dlo, dhi; + 128); the flat scan's combined table tags each entry with
// its round (bit 56).
constexpr int kPieceMaxOff = 3;            // an entry's 8-mer offset in its piece: 2 bits
__host__ __device__ inline uint64_t piece_entry(uint32_t val, int len, int o, int off, int dlo,
                                                int dhi, int round = 0) {
    return (uint64_t)val | ((uint64_t)len << 32) | ((uint64_t)o << 37) | ((uint64_t)off << 38) |
           ((uint64_t)(dlo + 128) << 40) | ((uint64_t)(dhi + 128) << 48) |
           ((uint64_t)round << 56);
}

struct DevPieces {
    int32_t on;            // 1: the piece screen replaces the full filter pass
    int32_t step;          // sampling stride s: an 8-mer every s positions (pieces >= 8 + s - 1)
    int32_t n_pieces, n_keys, n_entries;
    int32_t front_reach;   // FRONT: positions [0, front_reach) hold partial (column-0) alignments
    int32_t part_max;      // view positions per screen lane (multiple of 16)
    int32_t lo_off;        // min over orientation-0 pieces of len + dlo - 1 (>= 0)
    int32_t dlo_min;       // min over orientation-1 pieces of dlo
    int32_t pad[3];
    // the LDS image (pscreen_kernel copies it whole): bitmap, rank base, keys, entries
    uint32_t bitmap[kPieceBitmapWords];       // bit K: some entry samples the 8-mer K
    uint16_t rank_base[kPieceBitmapWords];    // set bits before each word: 8-mer -> key index
    uint32_t key[kMaxPieceEntries];           // key r (increasing 8-mer): first entry | count << 16
    uint64_t entry[kMaxPieceEntries];         // piece_entry(), grouped by key
};
constexpr int kPieceLdsFixed = kPieceBitmapWords * 6;   // bitmap + rank base, bytes

// One filter task of the piece screen: view positions [p0, p0 + span) of (item, o); columns
// p0 + hoff + 1 .. are reported (the positions before are the restricted-start warm-up); fresh:
// p0 = 0 with the panel's own column 0 (careful per-column thresholds, like segment 0).  The
// oriented view travels with the task (the filter needs no dependent loads).
struct FTask {
    uint32_t item;
    uint32_t p0;
    uint16_t span;
    uint8_t hoff;
    uint8_t flags;   // bit 0: orientation, bit 1: fresh, bit 2: the view's strand
    uint32_t n, start, len;   // the read's length; the oriented view
    uint64_t off;             // the read's first nt
};
static_assert(sizeof(FTask) == 32, "FTask layout");

// Flat piece scan: the packed batch is scanned once per exec as one stream of
// 4096-nt superblocks against the combined table of every flat round.  Marks live in batch nt
// coordinates, independent of reads and views: cell bitmap 2 r + t holds one bit per 16 nt for
// the copies of round r's pieces on strand t, and a view of strand t reads bitmap 2 r + t over its
// own nt range (a cell shared with a neighbouring read, or a copy across a read boundary, only
// adds filter work).
constexpr int kSuperNt = 4096;   // nt per wave step: 64 lanes x 64 nt
constexpr int kCellGuardWords = 4;   // zero words before / after each cell bitmap
constexpr int kCandStageCap = 128; // per candidate list

// Block-level staging of appended records: lanes append to LDS (LDS atomics), the block then
// reserves its range of the global list with ONE global atomic.  A single global counter
// hammered by every lane serialises at the memory side (MI355X_MICROARCH.md, 'fanin').
template <typename Rec, int CAP = kStageCap>
struct Stage {
    Rec* buf;              // LDS [CAP]
    uint32_t* cnt;         // LDS
    uint32_t* base;        // LDS scratch
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
        const uint32_t gi = atomicAdd(gcount, 1u);   // LDS full: direct (rare)
        if (gi < gcap) g[gi] = r;
        else atomicOr(flags, ovf);
    }
    // Every thread of the block must call flush().
    __device__ __forceinline__ void flush() const {
        __syncthreads();
        const uint32_t n = min(*cnt, (uint32_t)CAP);
        if (threadIdx.x == 0) *base = n ? atomicAdd(gcount, n) : 0u;
        __syncthreads();
        const uint32_t b = *base;
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
            if (b + i < gcap) g[b + i] = buf[i];
            else atomicOr(flags, ovf);
        }
        __syncthreads();
        if (threadIdx.x == 0) *cnt = 0;
        __syncthreads();
    }
};

// Block-uniform snapshot of LDS staging counters for a flush decision.  Every thread reads them
// between two barriers: without the second one a fast wave could skip the flush, start the next
// round and push (raising a counter) before a slow wave has read it; the slow wave would then
// flush alone and its barriers would pair with the other waves' loop barriers, so the flush would
// copy slots whose pushes had not landed (lost and duplicated records, found at scale by
// tools/determinism.py).
__device__ __forceinline__ uint32_t stage_count(const uint32_t* c) {
    __syncthreads();
    const uint32_t v = *c;
    __syncthreads();
    return v;
}

// A view of a read: strand 0 = the read as given, strand 1 = its reverse complement; the view
// is positions [start, start+len) of that strand.
struct ItemView {
    uint32_t read;
    uint32_t start;
    uint32_t len;
    uint8_t strand;
    uint8_t pad;
    int16_t only_adapter;   // linked mode: the pair index, else -1
};

struct Cluster {      // candidate columns [j1, j2] of one task (item, orientation, adapter)
    uint32_t item;
    uint16_t sub;     // o * A + a (or a in linked mode)
    uint8_t lastcol;  // 3' adapter: final column holds cells with cost <= k
    int8_t ub;        // upper bound of the score of any cell of the cluster
    uint32_t j1, j2;
};

// One candidate end cell (band mode): the window scan knows its exact cost; the band kernel
// recovers cutadapt's origin and score for it.  Carries the oriented view (no dependent loads).
struct Cand {
    uint32_t item;
    uint16_t sub;
    uint8_t iend;        // end row (m for last-row cells, i < m for last-column cells)
    uint8_t cost;
    uint32_t j;          // end column
    uint32_t n, start, len;
    uint8_t strand, o, a, clean;   // clean: the band reads codes only (Window kWinClean)
    uint64_t off;
};
static_assert(sizeof(Cand) == 40 && offsetof(Cand, off) == 32, "Cand layout");

struct Outcome {      // best cell found by the resolve lane of a cluster
    uint64_t key;     // ~0 = none
    int32_t origin;
    int32_t pad;      // band_cand_kernel: the cell's winner slot (read by select_cand_kernel)
};

// 64-bit ordering key, smaller = better, matching cutadapt's selection order:
//   score desc (Aligner.locate / best_match / ReverseComplementer), forward before RC on equal
//   score, fewer errors, earlier adapter (file order), earlier cell in locate's scan order.
// Fields (high to low): 127 - score (8 bits: accepted matches may score <= 0 with high error
// allowances, down to -128), orientation (1), cost (7), adapter (8), scan position (40).
__host__ __device__ inline uint64_t make_key(int score, int o, int cost, int a, uint64_t t) {
    const int s = score < -128 ? -128 : score;
    return ((uint64_t)(127 - s) << 56) | ((uint64_t)o << 55) | ((uint64_t)cost << 48) |
           ((uint64_t)a << 40) | (t & ((1ull << 40) - 1));
}
__host__ __device__ inline int key_score(uint64_t k) { return 127 - (int)(k >> 56); }
__host__ __device__ inline int key_orient(uint64_t k) { return (int)((k >> 55) & 1); }
__host__ __device__ inline int key_cost(uint64_t k) { return (int)((k >> 48) & 127); }
__host__ __device__ inline int key_adapter(uint64_t k) { return (int)((k >> 40) & 255); }
__host__ __device__ inline uint64_t key_t(uint64_t k) { return k & ((1ull << 40) - 1); }

// ---------------------------------------------------------------------------------------------
// Bounds of the device buffers.  Release builds: empty, every check is `true`.
// DMX_DEBUG_BOUNDS builds (dmx/libdmx_bounds.so): every gather of the packed batch and every
// slot / item / result / count access is checked against its buffer's extent, which the host
// passes per launch; a violation is not performed (a read returns 0) but sets flag bit 32 and
// records the first offender (kernel id, buffer id, index) in d_counters[24..27], so the call
// fails naming the kernel instead of faulting.
// ---------------------------------------------------------------------------------------------
enum BoundsBuf : uint32_t {
    kBufSeq = 1, kBufMask = 2, kBufSlot = 3, kBufItem = 4, kBufRes = 5, kBufCount = 6,
    kBufRead = 7, kBufLinked = 8, kBufCand = 9, kBufChop = 10
};
enum BoundsKernel : int32_t {
    kKerFilter = 1, kKerVerify, kKerScreen, kKerScreen4, kKerWscan, kKerScan, kKerBand0,
    kKerBand1, kKerSelectCand, kKerResolve, kKerSelect, kKerFin0, kKerFin1, kKerFin0L, kKerFin1L,
    kKerFin2L, kKerChop, kKerChopBig, kKerChopStart, kKerSelfTest, kKerPieces
};
constexpr int kBoundsRec = 24;     // d_counters[24..27]: kernel id + 1, buffer, index lo / hi

struct Bounds {
#ifdef DMX_DEBUG_BOUNDS
    int64_t lo, hi;                // valid u32 word indices of d_seq / d_nmask (guards included)
    uint64_t slots, items, reads, counts, linked;   // element counts of the other buffers
    uint32_t* rec;                 // d_counters
    int32_t kid;                   // the launch's kernel (BoundsKernel)
#endif
};

// Is index i of buffer `buf` inside [lo, hi)?  Records the first violation.
__device__ __forceinline__ bool bchk(const Bounds& b, int64_t i, int64_t lo, int64_t hi,
                                     uint32_t buf) {
#ifdef DMX_DEBUG_BOUNDS
    if (i >= lo && i < hi) return true;
    atomicOr(b.rec + 3, 32u);
    if (atomicCAS(b.rec + kBoundsRec, 0u, (uint32_t)b.kid + 1u) == 0u) {
        b.rec[kBoundsRec + 1] = buf;
        b.rec[kBoundsRec + 2] = (uint32_t)(uint64_t)i;
        b.rec[kBoundsRec + 3] = (uint32_t)((uint64_t)i >> 32);
    }
    return false;
#else
    (void)b, (void)i, (void)lo, (void)hi, (void)buf;
    return true;
#endif
}
#ifdef DMX_DEBUG_BOUNDS
#define DMX_BOUND(bd, field, i, buf) bchk((bd), (int64_t)(i), 0, (int64_t)(bd).field, (buf))
#else
#define DMX_BOUND(bd, field, i, buf) true
#endif

// ---------------------------------------------------------------------------------------------
// Packed read streams.  seq: 2 bits per nt (16 nt / u32, nt x at bits 2(x%16)); nmask: 1 bit per
// nt (1 = not ACGT, never matches).  dmx_pack puts DMX_PACK_PAD (64) nt of padding at both ends,
// and the device buffers carry kGuardWords (64) zeroed words on both sides (1024 nt of codes).
// Every global position is a SIGNED nt index: a gather before the first read floors to a negative
// word inside the guard (round 4's two faults were unsigned wraps of such positions).  The host
// checks per panel that the deepest reach of any kernel before / after a view stays inside the
// guard for every accepted offset (set_panel_impl, dmx_panel_reach).
// ---------------------------------------------------------------------------------------------
constexpr int kGuardWords = 64;        // zeroed u32 words before/after d_seq and d_nmask
constexpr int kGuardNt = 16 * kGuardWords;   // guard of the codes buffer in nt (the mask's is 2x)
constexpr int kMinOffset = 16;         // smallest read offset dmx_load / dmx_run accept
constexpr int kMinTail = 64;           // nt every read keeps before the end of the packed words
constexpr int kViewReachPre = 64;      // fetch16s: positions before -64 are read at -64

struct Packed {
    const uint32_t* seq;
    const uint32_t* nmask;
    Bounds bd;
    const uint32_t* stage = nullptr;   // window code slots (kStageWords each, wstage_kernel)
};

// Window code slots: the codes and no-match bits of 128 view columns of one
// verified window, gathered once by wstage_kernel for the index screen, the window scan and the
// band.  Words 0..7: codes of columns base + 16 i .. (2 bits each, view orientation), 8..11:
// no-match bits of columns base + 32 i .., 12: base, 13: columns filled (16 per gathered chunk).
// A window, task or candidate names its slot in the top bits of its `off` (slot + 1, 0 = none).
constexpr int kStageWords = 16;
// Window code slots are an A/B build (make variant NAME=stage
// DEFS=-DDMX_STAGE_SLOTS=1, then DMX_STAGE=1 at run time): measured slower, and compiled in they
// cost every gathering stage registers for the slot test (window scan 43 instead of 31 spilled
// VGPRs at 4 waves, index screen 7 instead of 2, band list 0 18 instead of 2).
#ifndef DMX_STAGE_SLOTS
#define DMX_STAGE_SLOTS 0
#endif
constexpr int kOffBits = 36;                              // batch nt offsets < 2^36
constexpr uint64_t kOffMask = (1ull << kOffBits) - 1ull;

__device__ __forceinline__ uint32_t window32(const uint32_t* __restrict__ w, int64_t bitpos,
                                             const Bounds& bd, uint32_t buf) {
    const int64_t q = bitpos >> 5;   // arithmetic shift: floor for negative positions
    const uint32_t sh = (uint32_t)bitpos & 31u;
#ifdef DMX_DEBUG_BOUNDS
    if (!bchk(bd, q, bd.lo, bd.hi - 1, buf)) return 0u;
#else
    (void)bd, (void)buf;
#endif
#ifdef DMX_WINDOW32_SPLIT   // A/B build: two 4-byte loads
    const uint64_t v = ((uint64_t)w[q + 1] << 32) | (uint64_t)w[q];
#else
    uint64_t v;   // words q and q + 1 as ONE 8-byte load (global_load_dwordx2 at a 4-byte
    __builtin_memcpy(&v, w + q, 8);   // aligned address: one request instead of two)
#endif
    return (uint32_t)(v >> sh);
}
// 16 codes (32 bits) and 32 no-match bits from global nt position g
__device__ __forceinline__ uint32_t code32(const Packed& pk, int64_t g) {
    return window32(pk.seq, 2 * g, pk.bd, kBufSeq);
}
__device__ __forceinline__ uint32_t mask32(const Packed& pk, int64_t g) {
    return window32(pk.nmask, g, pk.bd, kBufMask);
}

// Reverse the order of the 16 2-bit fields of w.
__device__ __forceinline__ uint32_t rev_pairs(uint32_t w) {
    const uint32_t v = __brev(w);
    return ((v >> 1) & 0x55555555u) | ((v << 1) & 0xAAAAAAAAu);
}

// 16 consecutive view positions starting at view position p: 2-bit codes (complemented on the
// reverse strand) and the no-match bits.  `off`/`n`: the read's first nt and length; view
// (strand, start).
// load_mask = false (a `clean` view range): the codes only, no-match bits 0.
__device__ __forceinline__ void fetch16(const Packed& pk, uint64_t off, uint32_t n,
                                        uint32_t strand, uint32_t start, uint32_t p,
                                        uint32_t& codes, uint32_t& nbits, bool load_mask = true) {
    if (strand == 0) {
        const int64_t g = (int64_t)off + start + p;
        codes = code32(pk, g);
        nbits = load_mask ? mask32(pk, g) & 0xFFFFu : 0u;
    } else {   // lowest nt of the window
        const int64_t b = (int64_t)off + (int64_t)n - 1 - start - (int64_t)p - 15;
        codes = ~rev_pairs(code32(pk, b));                           // complement = 3 - c
        nbits = load_mask ? __brev(mask32(pk, b)) >> 16 : 0u;
    }
}

// One Myers/Hyyro column step for semi-global matching with a free start in the read
// (D(0, j) = 0 for all j, so the row-0 horizontal delta shifted in is 0).
// Bit i-1 of Pv/Mv: vertical delta D(i, j) - D(i-1, j) is +1 / -1.
// Written on 32-bit halves so gfx950 folds the boolean algebra into v_bitop3 (the 64-bit form
// compiles to separate and/or/xor pairs); one 64-bit add carries between the halves.
// HB: 0 = the last row's bit (hbit) is in the low word, 1 = in the high word, -1 = select.
template <int HB>
__device__ __forceinline__ void myers_step_hw(uint32_t eql, uint32_t eqh, uint32_t& pvl,
                                              uint32_t& pvh, uint32_t& mvl, uint32_t& mvh, int& d,
                                              uint32_t hbit) {
    const uint32_t xvl = eql | mvl, xvh = eqh | mvh;
    uint32_t cy, cy2;
    const uint32_t sl = __builtin_addc(eql & pvl, pvl, 0u, &cy);     // v_add_co / v_addc_co
    const uint32_t sh = __builtin_addc(eqh & pvh, pvh, cy, &cy2);
    const uint32_t xhl = (sl ^ pvl) | eql, xhh = (sh ^ pvh) | eqh;
    const uint32_t phl = mvl | ~(xhl | pvl), phh = mvh | ~(xhh | pvh);
    const uint32_t mhl = pvl & xhl, mhh = pvh & xhh;
    uint32_t ps, ms;
    if constexpr (HB == 0) {
        ps = phl;
        ms = mhl;
    } else if constexpr (HB == 1) {
        ps = phh;
        ms = mhh;
    } else {
        ps = hbit >= 32 ? phh : phl;
        ms = hbit >= 32 ? mhh : mhl;
    }
    d += (int)__builtin_amdgcn_ubfe(ps, hbit & 31u, 1) +
         __builtin_amdgcn_sbfe((int)ms, hbit & 31u, 1);
    const uint32_t phh1 = __builtin_amdgcn_alignbit(phh, phl, 31), phl1 = phl << 1;
    const uint32_t mhh1 = __builtin_amdgcn_alignbit(mhh, mhl, 31), mhl1 = mhl << 1;
    pvl = mhl1 | ~(xvl | phl1);
    pvh = mhh1 | ~(xvh | phh1);
    mvl = phl1 & xvl;
    mvh = phh1 & xvh;
}

template <int HB = -1>
__device__ __forceinline__ void myers_step(uint64_t eq, uint64_t& pv, uint64_t& mv, int& d,
                                           uint32_t hbit) {
    uint32_t pvl = (uint32_t)pv, pvh = (uint32_t)(pv >> 32);
    uint32_t mvl = (uint32_t)mv, mvh = (uint32_t)(mv >> 32);
    myers_step_hw<HB>((uint32_t)eq, (uint32_t)(eq >> 32), pvl, pvh, mvl, mvh, d, hbit);
    pv = ((uint64_t)pvh << 32) | pvl;
    mv = ((uint64_t)mvh << 32) | mvl;
}

// 32-bit variant for the shared-suffix filter block.
__device__ __forceinline__ void myers_step32(uint32_t eq, uint32_t& pv, uint32_t& mv, int& d,
                                             uint32_t hbit) {
    const uint32_t xv = eq | mv;
    const uint32_t xh = (((eq & pv) + pv) ^ pv) | eq;
    uint32_t ph = mv | ~(xh | pv);
    uint32_t mh = pv & xh;
    // +1 / -1 from the last row's horizontal deltas: one v_add3 of an unsigned and a signed
    // one-bit field
    d += (int)__builtin_amdgcn_ubfe(ph, hbit, 1) + __builtin_amdgcn_sbfe((int)mh, hbit, 1);
    ph <<= 1;
    mh <<= 1;
    pv = mh | ~(xv | ph);
    mv = ph & xv;
}

// D(i, j) from column j's vertical-delta vectors (row 0 is 0).
__device__ __forceinline__ int col_cost(uint64_t pv, uint64_t mv, int i) {
    const uint64_t mask = i >= 64 ? ~0ull : ((1ull << i) - 1ull);
    return __popcll(pv & mask) - __popcll(mv & mask);
}

}  // namespace dmx
