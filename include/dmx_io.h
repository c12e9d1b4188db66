/*
 * dmx_io.h — C-ABI of libdmx_io.so: native FASTQ/FASTA(.gz) ingest fused with the 2-bit
 * packer, and per-bin (demultiplexed) FASTQ/FASTA(.gz) writers.  Host-only (no GPU).
 *
 * Replaces the record I/O around cutadapt's hot loop: dnaio's FASTQ/FASTA
 * parser and xopen's gzip reader/writers for `IN.fastq.gz` and `-o OUT/{name}_X.fastq.gz`
 * (scripts/02_cutadapt_loop.sh:70-71,100-101; scripts/04_cleaning_primers.sh:377-388).
 * dnaio/xopen are not vendored in /root/reference; conventions restated in dmx_io.cpp.
 *
 * Reader: a background thread feeds a pool of `threads` workers that inflate gzip input in
 * parallel (any gzip stream: members in parallel, and a single member by speculative chunked
 * decoding, csrc/dmx_inflate.h), index lines, validate records and pack sequences into the libdmx device
 * layout (include/dmx.h, DMX_PACK_PAD), one batch of about `batch_bytes` of text at a time, up
 * to two batches ahead of the consumer.  Writer ("sink"): dmx_sink_write renders the records of
 * a batch into per-output buffers and compresses them as independent gzip members on
 * `threads` workers, in the background, while the caller moves on to the next batch; records
 * keep input order within every output.
 * Status 0 = OK, negative = error (message via dmx_reader_error / dmx_sink_error).
 */
#ifndef DMX_IO_H
#define DMX_IO_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DMX_IO_ABI_VERSION 1

/* One batch of records (library-owned; valid until dmx_batch_free). Spans are [start, end). */
typedef struct dmx_batch {
    size_t n_reads;
    int32_t fasta;          /* 1: FASTA input (no qualities)                                   */
    int32_t _pad;
    const uint8_t* text;    /* record text as read (after decompression)                        */
    const uint64_t* head;   /* n x {start, end}: name line without '@' / '>' (and without '\r') */
    const uint8_t* seqtext; /* FASTQ: == text; FASTA: the records' sequence lines joined         */
    const uint64_t* seq;    /* n x {start, end} into seqtext                                     */
    const uint64_t* qual;   /* n x {start, end} into text; NULL for FASTA                        */
    const uint32_t* lens;   /* n sequence lengths                                               */
    /* the same reads in the libdmx device layout (dmx_pack output), ready for dmx_run */
    const uint32_t* seq2b;
    const uint32_t* nmask;
    const uint64_t* offsets;
    size_t n_words;
    uint64_t total_nt;
} dmx_batch;

typedef struct dmx_reader dmx_reader;
typedef struct dmx_sink dmx_sink;

int dmx_io_abi_version(void);
/* Process-wide memory budget of the readers' and writers' buffers, in bytes (0 = none, the
 * default): with a budget, the parallel inflate cuts smaller chunks (its working set about
 * budget / 16), the read-ahead blocks shrink, and the pools of recycled batch buffers hold at
 * most budget / 32 each.  Readers opened later use it.  The batch size is the caller's
 * (dmx/nio.py batch_bytes_for_budget).  Returns the previous budget. */
uint64_t dmx_io_set_memory_budget(uint64_t bytes);
/* One gzip member of src[0, n) in the writers' format (RFC 1952 with a "DX" size subfield;
 * level 1 = Huffman-only DEFLATE, levels 2..9 the record-aware encoder (header-line LZ77,
 * sequence lines in blocks of their own; DMX_GZIP_LIBDEFLATE=1: libdeflate at that level), 0 =
 * stored): written to out (cap bytes, at least 2 n + 4096), its length to *out_len.  0 on
 * success, negative if cap is too small. */
int dmx_io_gzip(const uint8_t* src, size_t n, int level, uint8_t* out, size_t cap,
                size_t* out_len);

/* Inflate a gzip stream held in memory (one or more members; tests and tools: the reader's
 * own gzip path, parallel on `threads` unless DMX_SEQ_INFLATE=1) into out (cap bytes).
 * 0 = OK (*out_len bytes), -2 = invalid / truncated stream or CRC mismatch, -3 = cap too small. */
int dmx_io_inflate(const uint8_t* src, size_t n, int threads, uint8_t* out, size_t cap,
                   size_t* out_len);

/* path: a file (gzip detected by its magic bytes) or "-" for stdin. */
int dmx_reader_open(const char* path, size_t batch_bytes, int threads, dmx_reader** out);
/* Next batch in input order; *out = NULL at end of input. */
int dmx_reader_next(dmx_reader* r, dmx_batch** out);
const char* dmx_reader_error(dmx_reader* r);
void dmx_reader_close(dmx_reader* r);
/* Releases the caller's reference (a sink still rendering the batch keeps its own). */
void dmx_batch_free(dmx_batch* b);

/* Open n_out outputs (created / truncated now, like cutadapt's demultiplexed outputs); a path
 * ending in ".gz" is gzip-compressed at `level`.  fasta_out: write FASTA records. */
int dmx_sink_open(const char* const* paths, int n_out, int fasta_out, int level, int threads,
                  dmx_sink** out);
/* Queue the records of batch b: read i goes to output out_idx[i] (-1 = not written) as
 *   name = head + " rc" x n_rc[i],
 *   sequence = orient(seq, rc[i])[start[i]:stop[i]] (orient = reverse complement if rc[i],
 *   qualities reversed with it).
 * Asynchronous: returns once the previous batch has been written; the arrays are copied. */
int dmx_sink_write(dmx_sink* s, dmx_batch* b, const int32_t* out_idx, const int32_t* start,
                   const int32_t* stop, const uint8_t* rc, const uint8_t* n_rc);
/* Wait for pending writes, close every output; n_written / bp_written (n_out entries each,
 * may be NULL) receive the records and bases written per output. */
/* Row form (pychopper-style outputs, several records per read): row r writes read[r] to output
 * out_idx[r] (-1 = nothing) as sequence = read[start[r]:stop[r]] (positions on the read as
 * given), reverse-complemented (qualities reversed) if rc[r]; name = the read's name line when
 * name_mode[r] == 0, or "{start}:{stop}|{id} strand=+|-{comment}" when name_mode[r] == 1 (id = the
 * name up to the first blank, comment = the rest of the line).  Rows of one output keep their
 * order.  Asynchronous like dmx_sink_write. */
int dmx_sink_write_rows(dmx_sink* s, dmx_batch* b, size_t n_rows, const uint32_t* read,
                        const int32_t* out_idx, const int32_t* start, const int32_t* stop,
                        const uint8_t* rc, const uint8_t* name_mode);
/* Rows named as segments with their own " rc" suffixes (the fused 01 -> 02 loop): row r writes
 * read[r][start[r]:stop[r]] (reverse-complemented if rc[r]) named
 * "{name_start}:{name_stop}|{id} strand=+|-{comment}" (strand from name_strand) followed by
 * n_rc[r] x " rc".  Asynchronous like dmx_sink_write. */
int dmx_sink_write_rows2(dmx_sink* s, dmx_batch* b, size_t n_rows, const uint32_t* read,
                         const int32_t* out_idx, const int32_t* start, const int32_t* stop,
                         const uint8_t* rc, const int32_t* name_start, const int32_t* name_stop,
                         const uint8_t* name_strand, const uint8_t* n_rc);
/* Pack views of a batch's reads into the libdmx device layout (include/dmx.h, as dmx_pack
 * lays out reads): view i = read[i][start[i]:stop[i]], reverse-complemented if rc[i] — the
 * records pychopper writes for segments (scripts/01_pychopper.sh) handed to the demultiplexer
 * without rendering or re-reading them.  n_words >= dmx_pack_words(sum of lengths, n_views).
 * 0 = OK, -2 = a view outside its read, -3 = n_words too small. */
int dmx_batch_pack_views(const dmx_batch* b, size_t n_views, const uint32_t* read,
                         const int32_t* start, const int32_t* stop, const uint8_t* rc,
                         int threads, uint32_t* out_seq2b, uint32_t* out_nmask,
                         uint64_t* out_offsets, uint32_t* out_lens, size_t n_words);
int dmx_sink_close(dmx_sink* s, uint64_t* n_written, uint64_t* bp_written);
const char* dmx_sink_error(dmx_sink* s);

/* Mean read quality of a FASTQ batch (pychopper -Q): out[i] = -10 log10 of the mean Phred+33
 * error probability of read i, summed in read order in IEEE double (0 for an empty read).
 * Returns -2 for a FASTA batch. */
int dmx_batch_mean_qual(const dmx_batch* b, double* out);
/* Free a sink after dmx_sink_close (or to abandon it). */
void dmx_sink_free(dmx_sink* s);

/* Round-2 cache of the unchanged 02_cutadapt_loop.sh (a resident process runs its 13 calls):
 * keep the uncompressed text of this sink's gzip outputs in memory (the rendered buffers, not a
 * copy) up to max_bytes retained in the process; call before the first write.  At
 * dmx_sink_close each output is registered under its real path, inode, size, mtime and the
 * CRC-32 of its first 64 KiB; dmx_reader_open of that file, unchanged on disk, then reads the
 * text from memory (no read, no inflate) and drops it.  Replaces: re-reading and inflating each
 * SP5 bin in the round-2 calls (scripts/02_cutadapt_loop.sh:91-103). */
int dmx_sink_retain(dmx_sink* s, uint64_t max_bytes);
/* Per output o: keep = 0 excludes it from retention (an output no later call reads back, e.g.
 * the round-1 `unknown` bin that 02_cutadapt_loop.sh:79 skips); keep = 1 re-includes it before
 * its first write.  Call after dmx_sink_retain. */
int dmx_sink_retain_output(dmx_sink* s, int o, int keep);
/* 1 if this reader takes its text from a retained sink output (no file read), else 0. */
int dmx_reader_in_memory(const dmx_reader* r);
/* Bytes of retained output text held in this process; drop all of it. */
uint64_t dmx_io_retained_bytes(void);
void dmx_io_drop_retained(void);

#ifdef __cplusplus
}
#endif
#endif /* DMX_IO_H */
