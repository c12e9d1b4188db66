/*
 * dmx.h — C-ABI of the MI355X-native two-round barcode demultiplexer (libdmx.so).
 *
 * Drop-in boundary.  In the reference the hot path is a PROCESS boundary: bash calls the
 * `cutadapt` executable (scripts/02_cutadapt_loop.sh:64-72 round 1, :91-103 round 2;
 * scripts/04_cleaning_primers.sh:371-388 linked primers).  Our drop-in `cutadapt` CLI
 * (nanopore-barcoding-orc_amd/bin/cutadapt, Python) keeps that surface and calls this library
 * through ctypes.  Each entry point below names the cutadapt-side interface whose work it
 * replaces (upstream cutadapt 4.9 is not vendored in /root/reference).
 *
 * Conventions: plain pointers and sizes, no torch types.  Host buffers are caller-owned, device
 * buffers library-owned.  Status 0 = OK, negative = error (message via dmx_last_error).
 * One context per device; a context is not thread-safe (one host thread per context).
 */
#ifndef DMX_H
#define DMX_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DMX_ABI_VERSION 4

/* Panel flags (dmx_set_panel.flags). */
#define DMX_FRONT 0x01  /* -g ADAPTER: 5' adapter, Where.FRONT (prefix of adapter may be skipped at read start) */
#define DMX_BACK 0x02   /* -a ADAPTER: 3' adapter, Where.BACK  (suffix may be skipped at read end)          */
#define DMX_RC 0x10     /* --rc: also try the reverse complement; use it iff its score is strictly greater  */

/* Run modes (dmx_set_mode). */
#define DMX_MODE_SINGLE 0    /* one cutadapt invocation: round 0 panel only                                   */
#define DMX_MODE_TWO_ROUND 1 /* 02_cutadapt_loop.sh fused: round 0 on the read, round 1 on the round-0-trimmed */
#define DMX_MODE_LINKED 2    /* -g F...R linked pairs: round 0 = fronts, round 1 = backs (pair i <-> i)        */

/* Error codes. */
#define DMX_OK 0
#define DMX_E_INVALID -1
#define DMX_E_HIP -2
#define DMX_E_NOMEM -3
#define DMX_E_UNSUPPORTED -4
#define DMX_E_STATE -5

/* One adapter match (cutadapt Match: astart/astop on the adapter, rstart/rstop on the read view
 * that round was run on, i.e. already reverse-complemented when rc == 1). */
typedef struct dmx_match {
    int32_t rstart, rstop;
    int16_t astart, astop;
    int16_t score, errors;
} dmx_match;

/* Per-read result (caller-owned array, one entry per read).
 * bin = adapter index in the panel (file order), -1 = no match ("unknown").
 * TWO_ROUND: m2 coordinates are on the round-1 output (trimmed, oriented) sequence.
 * LINKED: bin1 = bin2 = pair index; m1 = front part on the read, m2 = back part on
 *         read[m1.rstop:]. */
typedef struct dmx_result {
    int16_t bin1, bin2;
    uint8_t rc1, rc2;
    uint8_t flags, _pad;
    dmx_match m1, m2;
} dmx_result;

typedef struct dmx_ctx dmx_ctx;

/* Replaces: process start-up of `cutadapt -j N` (cli.main).  Opens HIP device `device`. */
int dmx_open(int device, dmx_ctx** out);
/* Replaces: cutadapt's exit. */
void dmx_close(dmx_ctx* ctx);
/* ctx = NULL: the last failure of a call that takes no context (dmx_comm_unique_id: why RCCL
 * could not be loaded), or "null context". */
const char* dmx_last_error(dmx_ctx* ctx);
int dmx_abi_version(void);

/* Replaces: parser.py adapter parsing of `-g file:` / `-a file:` / `-g F...R` (one call per panel).
 * seqs: uppercase IUPAC (U already mapped to T), lens <= 64.  max_errors: -e value (< 1 rate,
 * >= 1 absolute count).  min_overlap: -O (cutadapt default 3).  Adapter wildcards are enabled for
 * an adapter iff it has a non-ACGT character (cutadapt default). */
int dmx_set_panel(dmx_ctx* ctx, int round, const char* const* seqs, const int* lens,
                  int n_adapters, double max_errors, int min_overlap, int flags);
/* As dmx_set_panel, with a per-adapter DMX_FRONT / DMX_BACK (one cutadapt call mixing -g and -a,
 * scripts/04_cleaning_primers.sh:476-507); rc: 1 for --rc. */
int dmx_set_panel_mixed(dmx_ctx* ctx, int round, const char* const* seqs, const int* lens,
                        const int* wheres, int n_adapters, double max_errors, int min_overlap,
                        int rc);
int dmx_set_mode(dmx_ctx* ctx, int mode);
/* Host only (no GPU; tests): the piece screen dmx_set_panel would build for
 * these arguments: out[0..7] = {sampling stride (0 = off: the full filter pass), pieces, sampled
 * 8-mer keys, entries, FRONT partial-alignment reach, positions per screen lane, min len + dlo - 1
 * of orientation-0 pieces, min dlo of orientation-1 pieces}; entries (up to cap, may be NULL):
 * the packed (piece, offset) entries, grouped by 8-mer (dmx_device.h piece_entry). */
int dmx_panel_pieces(const char* const* seqs, const int* lens, int n_adapters, double max_errors,
                     int min_overlap, int flags, int32_t* out, int n_out, uint64_t* entries,
                     int cap);
/* Host only (no GPU; tests): how far the kernels' gathers reach around a read view for the
 * panel dmx_set_panel (wheres == NULL) or dmx_set_panel_mixed (wheres, flags & DMX_RC) would
 * build from these arguments, in nt: out[0] before view position 0 as the kernels' warm-up
 * formulas ask, out[1] after the clamp at -64 (positions before it are read at -64: warm-up
 * columns, where any codes are safe), out[2] past the view end, out[3] / out[4] the guard
 * needed below / above the packed words for the smallest offset and tail dmx_run accepts, out[5]
 * the guard the device buffers carry.  Returns what dmx_set_panel would return: it refuses a
 * panel with out[3] or out[4] > out[5] (DMX_E_UNSUPPORTED, out still filled). */
int dmx_panel_reach(const char* const* seqs, const int* lens, const int* wheres, int n_adapters,
                    double max_errors, int min_overlap, int flags, int32_t* out, int n_out);

/* Host-side packer (no GPU needed): ASCII reads -> 2-bit codes (A=0,C=1,G=2,T=3, 16 nt per
 * little-endian u32 word) + 1-bit "no-match" mask (any non-ACGT byte, e.g. N).  Reads are laid
 * out back to back starting at nt offset DMX_PACK_PAD; out_offsets[i] is read i's first nt.
 * Required words for both outputs: dmx_pack_words(total_nt). */
#define DMX_PACK_PAD 64
size_t dmx_pack_words(uint64_t total_nt, size_t n_reads);
int dmx_pack(const uint8_t* ascii, const uint64_t* offsets, const uint32_t* lens, size_t n_reads,
             uint32_t* out_seq2b, uint32_t* out_nmask, uint64_t* out_offsets);

/* Replaces: the per-read hot loop of one or more cutadapt runs (ReverseComplementer ->
 * AdapterCutter.best_match -> Adapter.match_to -> Aligner.locate, for every read) for the whole
 * input.  Synchronous: uploads, runs both rounds on the GPU, downloads `out`.  Layout contract
 * (checked; DMX_E_INVALID otherwise): every read has offsets[i] >= 16 and offsets[i] + lens[i]
 * + 64 <= 16 * n_words, lens[i] < 2^30.  Reads may overlap or come in any order.  The device
 * copies carry 1024 nt of zeroed guard on both sides, and every panel is checked to keep the
 * kernels' gathers around a view inside it for such offsets (dmx_panel_reach).  Batches in
 * dmx_pack's layout above 1.5 chunks (DMX_RUN_CHUNK reads, default 2^21) run as overlapped
 * chunks, others in one shot (same results). */
int dmx_run(dmx_ctx* ctx, const uint32_t* seq2b, const uint32_t* nmask, const uint64_t* offsets,
            const uint32_t* lens, size_t n_words, size_t n_reads, dmx_result* out);

/* As dmx_run, with the no-match mask given sparsely: its nonzero 32-bit words (mask word index
 * = nt / 32, as in dmx_pack's nmask) as strictly increasing exc_idx[] with their values
 * exc_val[].  Almost every nt of a read is A/C/G/T, so this uploads ~1% of the dense bitmap's
 * bytes; the device zero-fills the mask and scatters the exceptions.  Same results as dmx_run. */
int dmx_run_sparse(dmx_ctx* ctx, const uint32_t* seq2b, const uint32_t* exc_idx,
                   const uint32_t* exc_val, size_t n_exc, const uint64_t* offsets,
                   const uint32_t* lens, size_t n_words, size_t n_reads, dmx_result* out);
/* Host helper (no GPU): the nonzero words of a dmx_pack no-match mask of n_words words, in
 * increasing index order (first `cap` written); returns their total number. */
size_t dmx_mask_exceptions(const uint32_t* nmask, size_t n_words, uint32_t* out_idx,
                           uint32_t* out_val, size_t cap);
/* Page-lock (pin) / release caller host memory that batches are uploaded from (reused batch
 * buffers): pinned uploads run at the DMA rate instead of through pageable staging. */
int dmx_host_register(void* ptr, size_t bytes);
int dmx_host_unregister(void* ptr);

/* Number of visible HIP devices (0 if none). */
int dmx_device_count(void);

/* Multi-GPU form of dmx_run: the batch (dmx_pack layout) is split into
 * n_ctx contiguous read ranges balanced by total length, each range runs on its own context
 * (one device each) from its own host thread, and results land in `out` in input order.
 * out_counts (optional, n_counts entries) receives the per-bin counts summed over the shards:
 * when the contexts are one dmx_comm_init_all set (in that order), by an RCCL all-reduce of the
 * devices' count arrays over xGMI; otherwise (e.g. several contexts sharing one device) on the
 * host.  Returns the number of count entries (or DMX_OK without out_counts), negative on error
 * (message via dmx_last_error(ctxs[0])).  Contexts must share mode and panels. */
int dmx_run_multi(dmx_ctx* const* ctxs, int n_ctx, const uint32_t* seq2b, const uint32_t* nmask,
                  const uint64_t* offsets, const uint32_t* lens, size_t n_words, size_t n_reads,
                  dmx_result* out, uint64_t* out_counts, size_t n_counts);

/* ---- Multi-GPU count exchange (RCCL over xGMI) -------------------------------
 * Replaces: the per-adapter totals of the reference's single cutadapt process per panel
 * (scripts/02_cutadapt_loop.sh:64-72,91-103, `-j 24` workers on one node, report.py); sharded
 * over GPUs, each shard's (A0+1)(A1+1)+2 counts are summed in HBM by one ncclAllReduce.
 * One process, several GPUs: dmx_comm_init_all over contexts on distinct devices (ncclCommInitAll;
 * rank k = ctxs[k]); dmx_run_multi then reduces its counts with RCCL.
 * One process per GPU: rank 0 calls dmx_comm_unique_id and hands the DMX_COMM_ID_BYTES bytes to
 * every rank (any control plane), each rank calls dmx_comm_init_rank (ncclCommInitRank; blocks
 * until all ranks joined), then after each dmx_exec dmx_allreduce_counts (collective: every rank
 * calls it) sums the ranks' counts in place on the context's stream and copies them to
 * out_counts (optional); dmx_counts then returns the summed counts until the next dmx_exec.
 * dmx_close releases the communicator. */
#define DMX_COMM_ID_BYTES 128
int dmx_comm_unique_id(uint8_t* id);
int dmx_comm_init_rank(dmx_ctx* ctx, const uint8_t* id, int n_ranks, int rank);
int dmx_comm_init_all(dmx_ctx* const* ctxs, int n_ctx);
/* Number of ranks of the context's communicator (0 = none). */
int dmx_comm_size(dmx_ctx* ctx);
/* Returns the number of count entries, negative on error. */
int dmx_allreduce_counts(dmx_ctx* ctx, uint64_t* out_counts, size_t n_out);

/* Device-resident form (benchmarks / pipelined hosts): dmx_load copies a packed batch to HBM
 * once; dmx_exec enqueues the full pipeline on the context's stream (asynchronous); dmx_sync
 * waits; dmx_fetch copies results of the last exec to the host. */
int dmx_load(dmx_ctx* ctx, const uint32_t* seq2b, const uint32_t* nmask, const uint64_t* offsets,
             const uint32_t* lens, size_t n_words, size_t n_reads);
int dmx_exec(dmx_ctx* ctx);
int dmx_sync(dmx_ctx* ctx);
int dmx_fetch(dmx_ctx* ctx, dmx_result* out);

/* Replaces: cutadapt's per-adapter match statistics (report.py).  counts has
 * (A0+1)*(A1+1) entries: index (bin1+1)*(A1+1) + (bin2+1) (A1 = 0 in SINGLE mode), then
 * two more entries: number of reads that used the reverse complement in round 0 / round 1. */
int dmx_counts(dmx_ctx* ctx, uint64_t* out_counts, size_t n_out);

/* Diagnostics of the last dmx_exec: per-stage device time in ms measured with HIP events on the
 * context's stream (order: scan0, resolve0, finalize0, scan1, resolve1, finalize1, total, then
 * the parts of scan0/scan1 spent in the shared-suffix filter and the prefix verification:
 * filter0, verify0, filter1, verify1, then the index screen and the window scan:
 * screen0, wscan0, screen1, wscan1, then the piece screen's part of filter0 / filter1:
 * pieces0, pieces1 — pass n_stage = 17 to receive them all), and
 * counts[n_counts <= 14] = {candidate clusters r0, r1, filter windows kept for the window scan
 * r0, r1, candidate cells (band mode) or clusters resolved after pruning (ring mode) r0, r1,
 * band DPs / tracebacks r0, r1, filter windows before prefix verification r0, r1, (window
 * piece, adapter) tasks passed by the index screen r0, r1, filter tasks of the piece screen
 * r0, r1}, and flags
 * (bit0 cluster overflow, bit1 exactness-check violation, bit2 filter-window / task overflow,
 * bit3 candidate-cell overflow, bit4 a filter invariant (step bucket or piece-screen cell range)
 * violated, bit5 a bounds violation (DMX_DEBUG_BOUNDS builds); must be 0). */
int dmx_stats(dmx_ctx* ctx, float* stage_ms, int n_stage, uint64_t* counts, int n_counts,
              int* flags);

/* Diagnostics (tests and tools only): copy an intermediate list of the last dmx_exec to the host
 * (up to cap_bytes; returns the list's size in bytes, negative on error).  The window and task
 * lists are shared by both rounds, so after a two-round exec only round 1's are resident; the
 * candidate lists are per round.  Records are the library's internal layouts (40-byte windows /
 * tasks / candidates; DMX_DBG_FLAGS: the 4-byte pipeline flags word). */
#define DMX_DBG_WINDOWS 0
#define DMX_DBG_VERIFIED 1
#define DMX_DBG_TASKS 2
#define DMX_DBG_CANDS0 3
#define DMX_DBG_CANDS1 4
#define DMX_DBG_FLAGS 5
int dmx_debug_fetch(dmx_ctx* ctx, int what, int round, void* out, size_t cap_bytes);
/* DMX_DEBUG_BOUNDS builds only (dmx/libdmx_bounds.so; DMX_E_UNSUPPORTED otherwise): every gather
 * of the packed batch and every winner-slot / item / result / count access of every kernel is
 * checked against its buffer; a violation is skipped, and dmx_exec / dmx_run / dmx_chop_exec fail
 * with DMX_E_STATE naming the kernel, buffer and index (dmx_last_error).  This self test launches
 * one gather below the guard, one winner slot past its array and one valid gather; out3 receives
 * {codes read below the guard (0), slot check result (0), a valid gather}; returns DMX_E_STATE
 * with the first violation's message when the checks work. */
int dmx_debug_bounds_selftest(dmx_ctx* ctx, uint32_t* out3);

/* ---- Residual-primer failsafe: exact degenerate-motif location (`seqkit locate -d`) ---------
 * Replaces: `seqkit locate -d --pattern-file PRIMERS ENDS` in the failsafe of
 * scripts/04_cleaning_primers.sh:397-460 (`:422`; seqkit v2, not vendored).  Every occurrence
 * (overlapping ones included) of every IUPAC pattern (1..64 nt, at most 128 patterns) in every
 * record, on the positive strand and — unless DMX_LOC_ONLY_POSITIVE — on the negative strand
 * (the pattern matched against the reverse complement; reported in positive-strand
 * coordinates).  Case-sensitive unless DMX_LOC_IGNORE_CASE (seqkit -i).  Pattern codes admit
 * A/C/G/T(U) as IUPAC says (N = any of them); any other record byte matches nothing.
 * Records are ASCII (caller-owned blob + offsets/lengths).  Writes min(total, cap) hits in
 * unspecified order, *n_hits = total (call again with a larger buffer if total > cap). */
#define DMX_LOC_IGNORE_CASE 0x1
#define DMX_LOC_ONLY_POSITIVE 0x2
typedef struct dmx_hit {
    uint64_t seq;      /* record index                                    */
    int32_t pattern;   /* pattern index                                   */
    int32_t strand;    /* 0 = '+', 1 = '-'                                */
    int32_t start;     /* 1-based first position on the positive strand   */
    int32_t end;       /* 1-based last position (inclusive)               */
} dmx_hit;
int dmx_locate(dmx_ctx* ctx, const char* const* patterns, const int* plens, int n_patterns,
               int flags, const uint8_t* ascii, const uint64_t* offsets, const uint32_t* lens,
               size_t n_seqs, dmx_hit* out, size_t cap, uint64_t* n_hits);

/* ---- Read reorientation, pychopper style (the producer of the demultiplexer's input) ---------
 * Replaces: the primer search and read segmentation of
 *   `pychopper -b M13_seqs_for_pychopper.fa -c M13_config_for_pychopper.txt -p -m edlib`
 * (scripts/01_pychopper.sh:45-57; pychopper 2.7.10 / edlib are not vendored — the semantics are
 * restated in DESIGN.md §8d, parity unpinned).  Runs on the batch made resident by dmx_load.
 * Labels: primer p (file order) is label 2p, its reverse complement label 2p+1 (pychopper's
 * "-NAME").  IUPAC codes in primers (N = any base); a read N matches anything.
 * Hits: per label, as one edlib HW / EDLIB_TASK_LOC call with k = (int)(cutoff * m): when the
 * least infix edit distance over the read, best, is <= k, every read column whose least
 * distance equals best is a hit (stop), with the start of the longest optimal alignment
 * ending there (edlib's reverse SHW alignment, last position).
 * Segments: in a read's hits sorted by (start, stop, label), consecutive hits (a, b) with a
 * rule (rule_left[r], rule_right[r]) are a candidate segment on strand rule_strand[r] (0 '+',
 * 1 '-'; the first rule of a pair wins) spanning [a.start, b.stop) with keep_primers
 * (pychopper -p), else [a.stop, b.start) (empty if the hits overlap).  The read's segments are
 * the best path over its candidates: no two share a hit, greatest summed length (pychopper's
 * usable length), ties -> the earlier candidate. */
#define DMX_CHOP_MAX_PRIMERS 8
#define DMX_CHOP_MAX_RULES 32
typedef struct dmx_chop_hit {
    uint32_t read;
    int16_t label;
    int16_t dist;          /* edit distance                                        */
    int32_t start, stop;   /* [start, stop) on the read as given                   */
} dmx_chop_hit;
typedef struct dmx_chop_seg {
    uint32_t read;
    int32_t start, stop;   /* [start, stop) on the read as given, stop >= start     */
    int16_t strand;        /* 0 = '+', 1 = '-' (the segment is written reverse-complemented) */
    int16_t rule;
} dmx_chop_seg;
/* primers: uppercase IUPAC (U -> T), 1..64 nt each; cutoff in [0, 1). */
int dmx_chop_set(dmx_ctx* ctx, const char* const* primers, const int* plens, int n_primers,
                 const int* rule_left, const int* rule_right, const int* rule_strand, int n_rules,
                 double cutoff, int keep_primers);
/* Hits and segments of every resident read (synchronous); totals in *n_hits / *n_segs. */
int dmx_chop_exec(dmx_ctx* ctx, uint64_t* n_hits, uint64_t* n_segs);
/* Results of the last dmx_chop_exec (any pointer may be NULL): per-read segment and hit counts
 * (n_reads entries each) and the first seg_cap / hit_cap records in read order (within a read:
 * segments left to right, hits by (start, stop, label)). */
int dmx_chop_fetch(dmx_ctx* ctx, uint32_t* n_seg, uint32_t* n_hit, dmx_chop_seg* segs,
                   size_t seg_cap, dmx_chop_hit* hits, size_t hit_cap);
/* Device time (ms) of the last dmx_chop_exec: [0] chop_kernel (and chop_big_kernel when blocks
 * overflowed), [1] the read-order compaction.  Returns the number of 64-read blocks redone with
 * global hit lists (more primer hits than the 512-entry LDS list holds). */
int dmx_chop_stats(dmx_ctx* ctx, float* ms, int n_ms);

#ifdef __cplusplus
}
#endif
#endif /* DMX_H */
