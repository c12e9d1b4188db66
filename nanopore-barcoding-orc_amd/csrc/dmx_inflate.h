// dmx_inflate.h — DEFLATE (RFC 1951) decoder for PARALLEL decompression of ordinary gzip
// streams (a single member written by gzip / Python's gzip / zlib, or unsized concatenated
// members), used by libdmx_io's reader (dmx_io.cpp ParGzSource).
//
// The input of 02_cutadapt_loop.sh is `pychopped_<ds>.gz` (scripts/02_cutadapt_loop.sh:15,
// 28-34,71): one gzip member, which zlib can only inflate front to back.  The stream is cut into
// chunks of compressed bytes decoded on separate threads:
//   * chunk 0 starts where the previous round ended (a known block boundary) with the real
//     32 KiB window, and decodes into bytes;
//   * chunk k > 0 first FINDS a dynamic-Huffman block header at or after its nominal start
//     (find_block: header fields in range, complete code-length / literal / distance codes, the
//     block decodes to its end-of-block symbol, and the next header parses), then decodes with
//     an UNKNOWN window: the 32 KiB before the chunk are "markers" 256 + w (w = window index),
//     so the output is 16-bit symbols, and a back-reference into the unknown window copies the
//     marker;
//   * every chunk decodes until the first block header at or after the next chunk's nominal
//     start.  Chunk k's speculative start is accepted only if it equals chunk k-1's actual end;
//     otherwise chunk k is decoded again from that end with the real window.  So a false
//     positive of the block finder can cost time, never correctness.
//   * markers are resolved against the real window (the previous chunk's last 32 KiB, itself
//     resolved first), and every member's CRC-32 and ISIZE are checked.
// The decoder follows zlib's inflate on what it rejects (over-subscribed or incomplete codes
// except a single one-bit code, missing end-of-block code, repeat with no previous length,
// more than 286 / 30 codes, invalid symbols 286-287 / 30-31, distances beyond the data, stored
// LEN/NLEN mismatch), so any stream zlib inflates is decoded to the same bytes.
#pragma once

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <new>
#include <vector>

namespace dmxi {

constexpr int kWin = 32768;   // DEFLATE window
constexpr int kLitBits = 10, kDistBits = 8;   // primary table bits of the two codes

// Growable buffer that leaves its elements uninitialised (outputs are hundreds of MB).
template <typename T>
struct Buf {
    T* p = nullptr;
    size_t n = 0, cap = 0;
    Buf() = default;
    Buf(const Buf&) = delete;
    Buf& operator=(const Buf&) = delete;
    Buf(Buf&& o) noexcept : p(o.p), n(o.n), cap(o.cap) { o.p = nullptr; o.n = o.cap = 0; }
    ~Buf() { std::free(p); }
    void reserve(size_t c) {
        if (c <= cap) return;
        size_t nc = cap ? cap : 1024;
        while (nc < c) nc *= 2;
        T* q = static_cast<T*>(std::realloc(p, nc * sizeof(T)));
        if (!q) throw std::bad_alloc();
        p = q;
        cap = nc;
    }
};

// Huffman decode table: a primary table indexed by the next `pbits` stream bits, and
// subtables for longer codes.  Entry: bits 0-15 symbol (or subtable offset), bits 16-20 code
// length (or subtable index bits), bit 31 subtable link; 0 = invalid code.
struct Huff {
    static constexpr uint32_t kSub = 1u << 31;
    uint32_t t[4096];
    int pbits = 0;
};

inline uint32_t rev_bits(uint32_t c, int n) {
    uint32_t r = 0;
    for (int i = 0; i < n; ++i) r |= ((c >> i) & 1u) << (n - 1 - i);
    return r;
}

enum class Code { kOk, kIncomplete, kOver, kEmpty };

// Kraft check of code lengths (max 15).
inline Code code_shape(const uint8_t* lens, int n, int* count_out = nullptr) {
    int count[16] = {0};
    for (int i = 0; i < n; ++i) count[lens[i]]++;
    if (count_out) std::memcpy(count_out, count, sizeof(count));
    if (count[0] == n) return Code::kEmpty;
    int left = 1;
    for (int l = 1; l <= 15; ++l) {
        left <<= 1;
        left -= count[l];
        if (left < 0) return Code::kOver;
    }
    return left > 0 ? Code::kIncomplete : Code::kOk;
}

// Build a table.  Returns false when the code is over-subscribed, or incomplete other than a
// single code of length 1 (zlib's rule; `code_lengths` tables must always be complete), or when
// the subtables would not fit.  An empty code builds an all-invalid table (decoding fails on use).
inline bool build(Huff& h, int pbits, const uint8_t* lens, int n, bool code_lengths) {
    int count[16];
    const Code shape = code_shape(lens, n, count);
    if (shape == Code::kOver) return false;
    int maxlen = 0;
    for (int l = 15; l >= 1; --l)
        if (count[l]) {
            maxlen = l;
            break;
        }
    if (shape == Code::kIncomplete && (code_lengths || maxlen != 1)) return false;
    h.pbits = pbits;
    const uint32_t psize = 1u << pbits;
    std::memset(h.t, 0, sizeof(uint32_t) * psize);
    if (shape == Code::kEmpty) return true;
    uint32_t next[16];
    uint32_t c = 0;
    count[0] = 0;
    for (int l = 1; l <= 15; ++l) {
        c = (c + (uint32_t)count[l - 1]) << 1;
        next[l] = c;
    }
    // subtable sizes: the longest code under each pbits-bit prefix
    uint8_t submax[1u << 11];
    if (maxlen > pbits) std::memset(submax, 0, psize);
    uint32_t codes[320];
    if (n > 320) return false;
    for (int s = 0; s < n; ++s) {
        const int l = lens[s];
        if (!l) continue;
        codes[s] = next[l]++;
        if (l > pbits) {
            const uint32_t pre = codes[s] >> (l - pbits);
            if (submax[pre] < l) submax[pre] = (uint8_t)l;
        }
    }
    uint32_t used = psize;
    if (maxlen > pbits) {
        for (uint32_t pre = 0; pre < psize; ++pre) {
            if (!submax[pre]) continue;
            const int sb = submax[pre] - pbits;
            if (used + (1u << sb) > 4096) return false;
            h.t[rev_bits(pre, pbits)] = Huff::kSub | (uint32_t)sb << 16 | used;
            std::memset(h.t + used, 0, sizeof(uint32_t) << sb);
            used += 1u << sb;
        }
    }
    for (int s = 0; s < n; ++s) {
        const int l = lens[s];
        if (!l) continue;
        const uint32_t e = (uint32_t)l << 16 | (uint32_t)s;
        if (l <= pbits) {
            const uint32_t r = rev_bits(codes[s], l);
            for (uint32_t i = r; i < psize; i += 1u << l) h.t[i] = e;
        } else {
            const uint32_t pre = codes[s] >> (l - pbits);
            const uint32_t link = h.t[rev_bits(pre, pbits)];
            const int sb = (int)((link >> 16) & 31);
            const uint32_t base = link & 0xFFFFu;
            const int sl = l - pbits;
            const uint32_t r = rev_bits(codes[s] & ((1u << sl) - 1u), sl);
            for (uint32_t i = r; i < (1u << sb); i += 1u << sl) h.t[base + i] = e;
        }
    }
    return true;
}

constexpr uint16_t kLBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
constexpr uint8_t kLExt[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                               2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
constexpr uint16_t kDBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,
                                 33,  49,  65,  97,  129, 193,  257,  385,  513,  769,
                                 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
constexpr uint8_t kDExt[30] = {0, 0, 0, 0, 1, 1, 2, 2,  3,  3,  4,  4,  5,  5,  6,
                               6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
constexpr uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct Tables {
    Huff lit, dist;
};

inline const Tables& fixed_tables() {
    static const Tables* t = [] {
        auto* f = new Tables();
        uint8_t l[288], d[32];   // 32 distance codes of 5 bits (30, 31 decode as invalid)
        for (int i = 0; i < 144; ++i) l[i] = 8;
        for (int i = 144; i < 256; ++i) l[i] = 9;
        for (int i = 256; i < 280; ++i) l[i] = 7;
        for (int i = 280; i < 288; ++i) l[i] = 8;
        for (int i = 0; i < 32; ++i) d[i] = 5;
        build(f->lit, kLitBits, l, 288, false);
        build(f->dist, kDistBits, d, 32, false);
        return f;
    }();
    return *t;
}

// Input: `data` holds `nbytes` valid bytes followed by >= 16 readable padding bytes.  Bit
// positions are absolute within `data`, LSB first.
struct In {
    const uint8_t* data = nullptr;
    uint64_t nbytes = 0;
    bool eof = false;   // nbytes is the end of the stream (else more input may follow)
    inline uint64_t peek(uint64_t pos) const {   // >= 57 valid bits
        uint64_t v;
        std::memcpy(&v, data + (pos >> 3), 8);
        return v >> (pos & 7);
    }
    inline uint64_t end_bits() const { return nbytes * 8; }
};

template <int PB>
inline uint32_t decode_sym(const Huff& h, uint64_t v) {
    uint32_t e = h.t[v & ((1u << PB) - 1u)];
    if (__builtin_expect((e & Huff::kSub) != 0, 0))
        e = h.t[(e & 0xFFFFu) + ((uint32_t)(v >> PB) & ((1u << ((e >> 16) & 31)) - 1u))];
    return e;   // 0: invalid
}

// Dynamic block header at pos (after BFINAL/BTYPE): code lengths -> tables.  strict (block
// finder): the literal/length code must be complete and the distance code complete or a
// single one-bit code.  Returns false on any invalid header; pos advances past it.
inline bool read_dynamic(const In& in, uint64_t& pos, Tables& T, bool strict) {
    uint64_t v = in.peek(pos);
    const int hlit = (int)(v & 31) + 257, hdist = (int)((v >> 5) & 31) + 1,
              hclen = (int)((v >> 10) & 15) + 4;
    if (hlit > 286 || hdist > 30) return false;
    pos += 14;
    uint8_t cl[19] = {0};
    v = in.peek(pos);
    for (int i = 0; i < hclen; ++i) cl[kClOrder[i]] = (uint8_t)((v >> (3 * i)) & 7);
    pos += 3 * (uint64_t)hclen;
    {   // quick Kraft test before building (the block finder calls this at every candidate)
        int k = 0;
        for (int i = 0; i < 19; ++i)
            if (cl[i]) k += 128 >> cl[i];
        if (k != 128) return false;
    }
    Huff clh;
    if (!build(clh, 7, cl, 19, true)) return false;
    uint8_t lens[286 + 30];
    const int total = hlit + hdist;
    for (int i = 0; i < total;) {
        if (pos > in.end_bits()) return false;
        v = in.peek(pos);
        const uint32_t e = clh.t[v & 127];
        if (!e) return false;
        const int l = (int)((e >> 16) & 31);
        const int sym = (int)(e & 0xFFFF);
        v >>= l;
        pos += (uint64_t)l;
        if (sym < 16) {
            lens[i++] = (uint8_t)sym;
            continue;
        }
        int rep;
        uint8_t val = 0;
        if (sym == 16) {
            if (i == 0) return false;
            val = lens[i - 1];
            rep = 3 + (int)(v & 3);
            pos += 2;
        } else if (sym == 17) {
            rep = 3 + (int)(v & 7);
            pos += 3;
        } else {
            rep = 11 + (int)(v & 127);
            pos += 7;
        }
        if (i + rep > total) return false;
        std::memset(lens + i, val, (size_t)rep);
        i += rep;
    }
    if (pos > in.end_bits()) return false;
    if (lens[256] == 0) return false;   // no end-of-block code
    if (strict) {
        if (code_shape(lens, hlit) != Code::kOk) return false;
        const Code ds = code_shape(lens + hlit, hdist);
        if (ds == Code::kOver || ds == Code::kEmpty) return false;
        if (ds == Code::kIncomplete) {
            int nz = 0;
            for (int i = 0; i < hdist; ++i) nz += lens[hlit + i] != 0;
            if (nz != 1) return false;
        }
    }
    if (!build(T.lit, kLitBits, lens, hlit, false)) return false;
    if (!build(T.dist, kDistBits, lens + hlit, hdist, false)) return false;
    return true;
}

// Events of one decode run, at output offsets relative to the run's first output element.
struct Event {
    uint64_t out;        // output offset
    int kind;            // 0: a gzip member starts, 1: a member ends (crc / isize = its trailer)
    uint32_t crc, isize;
};

enum class Stop {
    kBoundary,   // stopped at a block header at or after stop_bit (pos = that header)
    kEnd,        // end of the stream after a member trailer (eof)
    kNeedMore,   // ran past the available input before a stop (more input is needed; at the
                 // end of the stream: truncated input)
    kError,      // invalid stream (or a wrong speculative start)
};

// gzip member header at byte-aligned pos (RFC 1952).  Returns 1 parsed, 0 need more input,
// -1 invalid.
inline int parse_member_header(const In& in, uint64_t& pos) {
    uint64_t b = pos >> 3;
    auto avail = [&](uint64_t need) { return b + need <= in.nbytes; };
    if (!avail(10)) return in.eof ? -1 : 0;
    const uint8_t* h = in.data + b;
    if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8) return -1;
    const uint8_t flg = h[3];
    if (flg & 0xE0) return -1;
    uint64_t q = b + 10;
    if (flg & 4) {
        if (q + 2 > in.nbytes) return in.eof ? -1 : 0;
        const uint64_t xlen = in.data[q] | (uint64_t)in.data[q + 1] << 8;
        q += 2 + xlen;
    }
    for (int f : {8, 16}) {
        if (!(flg & f)) continue;
        while (q < in.nbytes && in.data[q]) ++q;
        if (q >= in.nbytes) return in.eof ? -1 : 0;
        ++q;
    }
    if (flg & 2) q += 2;
    if (q > in.nbytes) return in.eof ? -1 : 0;
    pos = q * 8;
    return 1;
}

// LZ77 copy of `len` elements from `dist` back.  Whole 16-byte words when the distance spans at
// least one (each word reads only elements already written; the last one may write up to 15
// bytes past op + len: callers keep kSlack elements of room), a fill for distance 1 (runs of
// one quality character), elementwise otherwise.
constexpr uint32_t kSlack = 16;
template <typename T>
inline void copy_match(T* op, uint32_t dist, uint32_t len) {
    constexpr uint32_t W = 16 / sizeof(T);
    const T* src = op - dist;
    if (dist >= W) {
        for (uint32_t i = 0; i < len; i += W) std::memcpy(op + i, src + i, 16);
    } else if (dist == 1) {
        const T v = src[0];
        for (uint32_t i = 0; i < len; ++i) op[i] = v;
    } else {
        for (uint32_t i = 0; i < len; ++i) op[i] = src[i];
    }
}

// Decode from `pos` until the first block header at or after stop_bit, the end of the stream,
// or an error.  T = uint8_t: the 32 KiB before out.p[base] hold the real window (out.n starts
// at base = kWin); T = uint16_t: they hold markers 256 + w.  hist0: the first output index a
// back-reference may reach (base - known window bytes; a member start moves it).  at_member:
// pos is at a gzip member header (or the stream's end) rather than at a block header; updated.
template <typename T>
Stop inflate_run(const In& in, uint64_t& pos, bool& at_member, Buf<T>& out, uint64_t hist0,
                 uint64_t stop_bit, std::vector<Event>& ev) {
    const uint64_t base = kWin;
    Tables dyn;
    for (;;) {
        if (at_member) {
            uint64_t b = (pos + 7) >> 3;
            while (b < in.nbytes && in.data[b] == 0) ++b;   // zero padding between members
            pos = b * 8;
            if (b >= in.nbytes) return in.eof ? Stop::kEnd : Stop::kNeedMore;
            const int hr = parse_member_header(in, pos);
            if (hr == 0) return Stop::kNeedMore;
            if (hr < 0) return Stop::kError;
            ev.push_back({out.n - base, 0, 0, 0});
            hist0 = out.n;
            at_member = false;
        }
        if (pos >= stop_bit) return Stop::kBoundary;
        if (pos + 3 > in.end_bits()) return Stop::kNeedMore;
        const uint64_t hv = in.peek(pos);
        const bool final = hv & 1;
        const int type = (int)((hv >> 1) & 3);
        pos += 3;
        if (type == 3) return Stop::kError;
        if (type == 0) {   // stored
            pos = (pos + 7) & ~7ull;
            const uint64_t b = pos >> 3;
            if (b + 4 > in.nbytes) return Stop::kNeedMore;
            const uint32_t len = in.data[b] | (uint32_t)in.data[b + 1] << 8;
            const uint32_t nlen = in.data[b + 2] | (uint32_t)in.data[b + 3] << 8;
            if ((len ^ 0xFFFFu) != nlen) return Stop::kError;
            if (b + 4 + len > in.nbytes) return Stop::kNeedMore;
            out.reserve(out.n + len);
            for (uint32_t i = 0; i < len; ++i) out.p[out.n + i] = in.data[b + 4 + i];
            out.n += len;
            pos = (b + 4 + len) * 8;
        } else {
            const Tables* tb = &fixed_tables();
            if (type == 2) {
                if (!read_dynamic(in, pos, dyn, false))
                    return pos > in.end_bits() ? Stop::kNeedMore : Stop::kError;
                tb = &dyn;
            }
            const Huff& lit = tb->lit;
            const Huff& dst = tb->dist;
            const uint64_t endb = in.end_bits();
            T* op = nullptr;
            size_t cap_left = 0;
            auto room = [&](size_t need) {
                if (cap_left < need) {
                    out.n = (size_t)(op ? op - out.p : out.n);
                    out.reserve(out.n + (size_t)(1u << 20) + need);
                    op = out.p + out.n;
                    cap_left = out.cap - out.n;
                }
            };
            op = out.p + out.n;
            cap_left = out.cap - out.n;
            for (;;) {
                if (pos > endb) {
                    out.n = (size_t)(op - out.p);
                    return Stop::kNeedMore;
                }
                room(258 + kSlack);
                uint64_t v = in.peek(pos);   // >= 57 valid bits
                uint32_t e = decode_sym<kLitBits>(lit, v);
                if (!e) {
                    out.n = (size_t)(op - out.p);
                    return Stop::kError;
                }
                int cl = (int)((e >> 16) & 31);
                uint32_t sym = e & 0xFFFFu;
                // up to three literals per load (codes <= 15 bits; two literals, a length code
                // and its extra bits take <= 50 of the 57 bits)
                if (sym < 256) {
                    *op++ = (T)sym;
                    v >>= cl;
                    pos += (uint64_t)cl;
                    e = decode_sym<kLitBits>(lit, v);
                    if (!e) {
                        --cap_left;
                        continue;   // reported by the next iteration
                    }
                    cl = (int)((e >> 16) & 31);
                    sym = e & 0xFFFFu;
                    if (sym < 256) {
                        *op++ = (T)sym;
                        v >>= cl;
                        pos += (uint64_t)cl;
                        e = decode_sym<kLitBits>(lit, v);
                        if (e && (e & 0xFFFFu) < 256) {
                            *op++ = (T)(e & 0xFFFFu);
                            pos += (e >> 16) & 31;
                            cap_left -= 3;
                            continue;
                        }
                        cap_left -= 2;
                        continue;
                    }
                    --cap_left;
                }
                pos += (uint64_t)cl;
                if (sym == 256) break;
                const uint32_t ls = sym - 257;
                if (ls >= 29) {
                    out.n = (size_t)(op - out.p);
                    return Stop::kError;
                }
                v >>= cl;
                const uint32_t len = kLBase[ls] + ((uint32_t)v & ((1u << kLExt[ls]) - 1u));
                pos += kLExt[ls];
                v = in.peek(pos);
                const uint32_t de = decode_sym<kDistBits>(dst, v);
                if (!de || (de & 0xFFFFu) >= 30) {
                    out.n = (size_t)(op - out.p);
                    return Stop::kError;
                }
                const int dl = (int)((de >> 16) & 31);
                const uint32_t ds = de & 0xFFFFu;
                v >>= dl;
                const uint32_t dist = kDBase[ds] + ((uint32_t)v & ((1u << kDExt[ds]) - 1u));
                pos += (uint64_t)dl + kDExt[ds];
                const uint64_t at = (uint64_t)(op - out.p);
                if (dist > at - hist0) {
                    out.n = (size_t)at;
                    return Stop::kError;
                }
                copy_match(op, dist, len);
                op += len;
                cap_left -= len;
            }
            out.n = (size_t)(op - out.p);
            if (pos > endb) return Stop::kNeedMore;
        }
        if (final) {   // member trailer: CRC-32, ISIZE
            pos = (pos + 7) & ~7ull;
            const uint64_t b = pos >> 3;
            if (b + 8 > in.nbytes) return Stop::kNeedMore;
            const uint8_t* t = in.data + b;
            const uint32_t crc = t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24;
            const uint32_t isz = t[4] | (uint32_t)t[5] << 8 | (uint32_t)t[6] << 16 | (uint32_t)t[7] << 24;
            ev.push_back({out.n - base, 1, crc, isz});
            pos = (b + 8) * 8;
            at_member = true;
        }
    }
}

// First position in [from_bit, to_bit) that starts a non-final dynamic block which decodes to
// its end-of-block symbol (with an unknown window) and is followed by a valid block header.
// scratch: any uint16 buffer (reused).
inline bool find_block(const In& in, uint64_t from_bit, uint64_t to_bit, uint64_t& found,
                       Buf<uint16_t>& scratch) {
    Tables T;
    std::vector<Event> ev;
    const uint64_t lim = std::min<uint64_t>(to_bit, in.end_bits() > 64 ? in.end_bits() - 64 : 0);
    for (uint64_t b = from_bit; b < lim; ++b) {
        const uint64_t v = in.peek(b);
        if ((v & 7) != 4) continue;                            // BFINAL 0, BTYPE 2
        if (((v >> 3) & 31) > 29 || ((v >> 8) & 31) > 29) continue;
        uint64_t p = b + 3;
        if (!read_dynamic(in, p, T, true)) continue;
        // decode this one block (markers for the unknown window)
        scratch.reserve(kWin + (1u << 16));
        for (int i = 0; i < kWin; ++i) scratch.p[i] = (uint16_t)(256 + i);
        scratch.n = kWin;
        uint64_t q = b;
        bool atm = false;
        ev.clear();
        // stop at the first header after b: decode_run stops at block headers >= b + 1
        const Stop st = inflate_run<uint16_t>(in, q, atm, scratch, 0, b + 1, ev);
        if (st != Stop::kBoundary || atm) continue;
        // the next header must parse too
        const uint64_t nv = in.peek(q);
        const int nt = (int)((nv >> 1) & 3);
        if (nt == 3) continue;
        if (nt == 2) {
            uint64_t r = q + 3;
            if (!read_dynamic(in, r, T, true)) continue;
        } else if (nt == 0) {
            const uint64_t bb = (q + 3 + 7) >> 3;
            if (bb + 4 > in.nbytes) continue;
            const uint32_t len = in.data[bb] | (uint32_t)in.data[bb + 1] << 8;
            const uint32_t nlen = in.data[bb + 2] | (uint32_t)in.data[bb + 3] << 8;
            if ((len ^ 0xFFFFu) != nlen) continue;
        }
        found = b;
        return true;
    }
    return false;
}

}  // namespace dmxi
