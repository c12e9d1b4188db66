// dmx_deflate.h — Huffman-only DEFLATE (RFC 1951) encoder for the per-bin gzip writers.
//
// FASTQ is 2-bit-entropy bases plus skewed qualities: LZ77 finds little in it (zlib level 1
// spends most of its time looking), so the writers entropy-code bytes only (zlib's
// Z_HUFFMAN_ONLY strategy, same output class).  zlib's Huffman-only path tallies every byte
// through its general LZ77 machinery (~80 MB/s per core on the build host); this encoder does a
// 4-way histogram and a table-driven bit packer per block (several times faster), emitting
// standard dynamic-Huffman blocks any inflater reads.
//
// Block format (RFC 1951 §3.2.7): BFINAL, BTYPE = 2, HLIT = 0 (257 literal/length codes: bytes
// + end-of-block), HDIST = 1 (two distance codes of length 1, never used — the pkzip rule of at
// least one distance code, as zlib writes it), the code-length code (max length 7) and the 259
// code lengths sent without run-length codes (≈ 130 B per block), then the literals and EOB.
// Literal code lengths are limited to 15 bits by halving the frequencies until the Huffman tree
// fits (rare: only blocks with very rare bytes).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <vector>

namespace dmxz {

struct BitWriter {
    uint8_t* p;
    uint64_t buf = 0;
    int n = 0;
    explicit BitWriter(uint8_t* out) : p(out) {}
    // len <= 16; the caller keeps 8 spare bytes after the output
    inline void put(uint32_t bits, int len) {
        buf |= (uint64_t)bits << n;
        n += len;
        if (n >= 32) {
            std::memcpy(p, &buf, 4);
            p += 4;
            buf >>= 32;
            n -= 32;
        }
    }
    inline void flush() {   // pad the last byte with zero bits
        while (n > 0) {
            *p++ = (uint8_t)buf;
            buf >>= 8;
            n -= 8;
        }
        n = 0;
        buf = 0;
    }
};

// Huffman code lengths (<= maxlen) of nsym symbols; symbols with frequency 0 get length 0.
// Needs >= 2 symbols of nonzero frequency.
inline void huff_lengths(const uint32_t* freq, int nsym, int maxlen, uint8_t* len) {
    std::vector<uint64_t> f(freq, freq + nsym);
    std::vector<int> leaf;   // symbols sorted by (frequency, symbol)
    std::vector<uint64_t> w;
    std::vector<int> parent;
    for (;;) {
        leaf.clear();
        for (int s = 0; s < nsym; ++s)
            if (f[s]) leaf.push_back(s);
        std::sort(leaf.begin(), leaf.end(),
                  [&](int a, int b) { return f[a] != f[b] ? f[a] < f[b] : a < b; });
        const int m = (int)leaf.size();
        std::memset(len, 0, (size_t)nsym);
        if (m == 0) return;
        if (m == 1) {
            len[leaf[0]] = 1;
            return;
        }
        // nodes 0..m-1: leaves in weight order; m..2m-2: internal nodes in creation order
        // (nondecreasing weight, so the two queues merge like a sorted list)
        w.assign((size_t)(2 * m - 1), 0);
        parent.assign((size_t)(2 * m - 1), -1);
        for (int i = 0; i < m; ++i) w[i] = f[leaf[i]];
        int li = 0, ii = m;
        for (int k = m; k < 2 * m - 1; ++k) {
            int pick[2];
            for (int t = 0; t < 2; ++t) {
                if (li < m && (ii >= k || w[li] <= w[ii])) pick[t] = li++;
                else pick[t] = ii++;
            }
            w[k] = w[pick[0]] + w[pick[1]];
            parent[pick[0]] = parent[pick[1]] = k;
        }
        std::vector<int> depth((size_t)(2 * m - 1), 0);
        int dmax = 0;
        for (int k = 2 * m - 3; k >= 0; --k) {   // parents are created after their children
            depth[k] = depth[parent[k]] + 1;
            if (k < m) dmax = std::max(dmax, depth[k]);
        }
        if (dmax <= maxlen) {
            for (int i = 0; i < m; ++i) len[leaf[i]] = (uint8_t)depth[i];
            return;
        }
        for (auto& x : f)
            if (x) x = (x + 1) >> 1;   // flatten the distribution and retry
    }
}

// Canonical codes (RFC 1951 §3.2.2), bit-reversed for the LSB-first stream.
inline void huff_codes(const uint8_t* len, int nsym, uint16_t* code) {
    uint32_t count[16] = {0}, next[16] = {0};
    for (int s = 0; s < nsym; ++s) count[len[s]]++;
    count[0] = 0;
    uint32_t c = 0;
    for (int b = 1; b < 16; ++b) {
        c = (c + count[b - 1]) << 1;
        next[b] = c;
    }
    for (int s = 0; s < nsym; ++s) {
        const int l = len[s];
        if (!l) {
            code[s] = 0;
            continue;
        }
        uint32_t v = next[l]++, r = 0;
        for (int i = 0; i < l; ++i) {
            r = (r << 1) | (v & 1u);
            v >>= 1;
        }
        code[s] = (uint16_t)r;
    }
}

// One dynamic-Huffman block of literals src[0, n) (n >= 1).
inline void huff_block(BitWriter& bw, const uint8_t* src, size_t n, bool final) {
    uint32_t h[4][256];
    std::memset(h, 0, sizeof(h));
    size_t i = 0;
    for (; i + 4 <= n; i += 4) {
        h[0][src[i]]++;
        h[1][src[i + 1]]++;
        h[2][src[i + 2]]++;
        h[3][src[i + 3]]++;
    }
    for (; i < n; ++i) h[0][src[i]]++;
    uint32_t freq[257];
    for (int s = 0; s < 256; ++s) freq[s] = h[0][s] + h[1][s] + h[2][s] + h[3][s];
    freq[256] = 1;   // end of block
    uint8_t len[259];
    huff_lengths(freq, 257, 15, len);
    len[257] = len[258] = 1;   // the two distance codes
    uint16_t code[257];
    huff_codes(len, 257, code);

    // code-length code over the 259 lengths, sent one symbol each (no run-length codes)
    uint32_t cf[19] = {0};
    for (int s = 0; s < 259; ++s) cf[len[s]]++;
    int used = 0;
    for (int s = 0; s < 19; ++s) used += cf[s] ? 1 : 0;
    if (used < 2) cf[cf[0] ? 1 : 0]++;   // a complete code needs two symbols
    uint8_t cl[19];
    huff_lengths(cf, 19, 7, cl);
    uint16_t cc[19];
    huff_codes(cl, 19, cc);
    static const uint8_t kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    int hclen = 19;
    while (hclen > 4 && cl[kOrder[hclen - 1]] == 0) --hclen;

    bw.put(final ? 1u : 0u, 1);
    bw.put(2u, 2);            // dynamic Huffman
    bw.put(0u, 5);            // HLIT: 257 literal/length codes
    bw.put(1u, 5);            // HDIST: 2 distance codes
    bw.put((uint32_t)(hclen - 4), 4);
    for (int k = 0; k < hclen; ++k) bw.put(cl[kOrder[k]], 3);
    for (int s = 0; s < 259; ++s) bw.put(cc[len[s]], cl[len[s]]);

    uint32_t tab[256];
    for (int s = 0; s < 256; ++s) tab[s] = (uint32_t)code[s] | ((uint32_t)len[s] << 16);
    // branch-free packing: three codes (<= 45 bits) on top of <= 7 pending bits, then store 8
    // bytes and advance by the whole bytes written (the output keeps 8 bytes of slack)
    uint64_t buf = bw.buf;
    int nb = bw.n;
    uint8_t* p = bw.p;
    while (nb >= 8) {
        *p++ = (uint8_t)buf;
        buf >>= 8;
        nb -= 8;
    }
    i = 0;
    for (; i + 3 <= n; i += 3) {
        // the three codes are joined off the bit-position dependency chain
        const uint32_t e0 = tab[src[i]], e1 = tab[src[i + 1]], e2 = tab[src[i + 2]];
        const int l0 = (int)(e0 >> 16), l01 = l0 + (int)(e1 >> 16);
        const uint64_t v = (uint64_t)(e0 & 0xFFFFu) | ((uint64_t)(e1 & 0xFFFFu) << l0) |
                           ((uint64_t)(e2 & 0xFFFFu) << l01);
        buf |= v << nb;
        nb += l01 + (int)(e2 >> 16);
        std::memcpy(p, &buf, 8);
        p += nb >> 3;
        buf >>= nb & ~7;
        nb &= 7;
    }
    bw.buf = buf;
    bw.n = nb;
    bw.p = p;
    for (; i < n; ++i) bw.put(code[src[i]], len[src[i]]);
    bw.put(code[256], len[256]);
}

// Output bound of huff_deflate for n input bytes.
inline size_t huff_bound(size_t n) { return 2 * n + 512 * (n / (256u << 10) + 2) + 64; }

// Raw DEFLATE stream of src[0, n) into out (huff_bound(n) bytes); returns its length.
inline size_t huff_deflate(const uint8_t* src, size_t n, uint8_t* out) {
    BitWriter bw(out);
    if (n == 0) {   // one empty stored block
        bw.put(1u, 1);
        bw.put(0u, 2);
        bw.flush();
        const uint8_t st[4] = {0, 0, 0xFF, 0xFF};
        std::memcpy(bw.p, st, 4);
        return (size_t)(bw.p - out) + 4;
    }
    constexpr size_t kBlock = 256u << 10;
    for (size_t o = 0; o < n; o += kBlock) {
        const size_t m = std::min(kBlock, n - o);
        huff_block(bw, src + o, m, o + m == n);
    }
    bw.flush();
    return (size_t)(bw.p - out);
}

// ------------------------------------------------------------------------------------------
// Record-aware LZ77 + Huffman: the writers' levels 2..9 (dmx_io.cpp gzip_member routes every
// level from 2 to 9 here and ignores the level: -2 and -9 give the same stream;
// DMX_GZIP_LIBDEFLATE=1 restores per-level output through libdeflate).
//
// Split by line type, zlib -5 and Huffman-only compare like this on nanopore-style FASTQ
// (MinKNOW headers, autocorrelated qualities; profiles/r5_gzip_levels.json): headers 6.4 MB ->
// 0.99 MB (zlib -5) vs 4.1 MB (Huffman only); sequence 21.9 MB -> 6.6 vs 6.2 MB; qualities
// 21.9 MB -> 13.2 vs 12.6 MB.  All of LZ77's gain is in the header lines (run id, flow cell,
// model, the read id repeated as parent_read_id); in sequence and quality lines its matches
// cost more than they save.  So this encoder searches matches only in header lines — a line
// starting with '@' or '>' that does not follow a lone "+" line (that one is a quality line) —
// against earlier header bytes of the member (one hash probe on 4-byte grams, plus the same
// column of the previous header), and Huffman-codes everything else as literals with the
// table-driven packer above.  The output is ordinary dynamic-Huffman DEFLATE.

struct LzMatch {
    uint32_t pos, len, dist;   // pos relative to the member start
};

struct LzTables {
    uint8_t len_sym[259];      // match length 3..258 -> length symbol - 257
    uint8_t dist_sym[512];     // d - 1 < 256: [d - 1]; else [256 + ((d - 1) >> 7)]
    uint16_t len_base[29];
    uint8_t len_xb[29];
    uint16_t dist_base[30];
    uint8_t dist_xb[30];
    LzTables() {
        static const uint16_t lb[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                        31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
        static const uint8_t lx[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                       2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
        static const uint16_t db[30] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,
                                        33,   49,   65,   97,   129,  193,   257,   385,   513, 769,
                                        1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
        static const uint8_t dx[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3,  3,  4,  4,  5,  5,  6,
                                       6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
        std::memcpy(len_base, lb, sizeof(lb));
        std::memcpy(len_xb, lx, sizeof(lx));
        std::memcpy(dist_base, db, sizeof(db));
        std::memcpy(dist_xb, dx, sizeof(dx));
        std::memset(len_sym, 0, sizeof(len_sym));
        for (int k = 0; k < 28; ++k)
            for (int l = lb[k]; l < (k + 1 < 28 ? lb[k + 1] : 258); ++l) len_sym[l] = (uint8_t)k;
        len_sym[258] = 28;
        for (int s = 0; s < 30; ++s)
            for (uint32_t d = db[s]; d < (uint32_t)db[s] + (1u << dx[s]); ++d) {
                if (d - 1 < 256) dist_sym[d - 1] = (uint8_t)s;
                else dist_sym[256 + ((d - 1) >> 7)] = (uint8_t)s;
            }
    }
    uint32_t dsym(uint32_t d) const { return d - 1 < 256 ? dist_sym[d - 1] : dist_sym[256 + ((d - 1) >> 7)]; }
};
inline const LzTables& lz_tables() {
    static const LzTables t;
    return t;
}

// Equal bytes of a[0..) and b[0..), at most maxl (a < b, both readable for maxl bytes).
inline uint32_t lz_match_len(const uint8_t* a, const uint8_t* b, uint32_t maxl) {
    uint32_t l = 0;
    while (l + 8 <= maxl) {
        uint64_t x, y;
        std::memcpy(&x, a + l, 8);
        std::memcpy(&y, b + l, 8);
        if (x != y) return l + ((uint32_t)__builtin_ctzll(x ^ y) >> 3);
        l += 8;
    }
    while (l < maxl && a[l] == b[l]) ++l;
    return l;
}

constexpr int kLzHashBits = 12;
inline uint32_t lz_hash4(const uint8_t* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return (v * 2654435761u) >> (32 - kLzHashBits);
}

// One pass over the lines of s[0, n): greedy matches (length >= 4; >= 5 beyond 4 KiB) inside the
// header lines, and the sequence lines (the line after a header, without its newline; empty
// ones skipped) as [a, b) ranges.  A match ends at the header's newline at the latest, so it
// never reaches into the sequence line.
inline void fq_scan(const uint8_t* s, size_t n, std::vector<LzMatch>& out,
                    std::vector<std::pair<uint32_t, uint32_t>>& seqs) {
    out.clear();
    seqs.clear();
    int64_t ht[1 << kLzHashBits];
    std::fill(ht, ht + (1 << kLzHashBits), (int64_t)-1);
    bool prev_plus = false, prev_head = false;
    size_t last_head = SIZE_MAX;   // start of the previous header line
    for (size_t ls = 0; ls < n;) {
        const void* nl = std::memchr(s + ls, '\n', n - ls);
        const size_t le = nl ? (size_t)((const uint8_t*)nl - s) : n;
        const bool head = (s[ls] == '@' || s[ls] == '>') && !prev_plus;
        if (prev_head && !head && le > ls) seqs.emplace_back((uint32_t)ls, (uint32_t)le);
        prev_plus = le - ls == 1 && s[ls] == '+';
        prev_head = head;
        if (head) {
            for (size_t i = ls; i + 4 <= le;) {
                const uint32_t h = lz_hash4(s + i);
                const int64_t c = ht[h];
                ht[h] = (int64_t)i;
                const uint32_t maxl = (uint32_t)std::min<size_t>(258, std::min(le + 1, n) - i);
                uint32_t best = 0, bd = 0;
                if (c >= 0 && i - (size_t)c <= 32768) {
                    best = lz_match_len(s + c, s + i, maxl);
                    bd = (uint32_t)(i - (size_t)c);
                }
                if (last_head != SIZE_MAX) {   // the same column of the previous header
                    const size_t a = last_head + (i - ls);
                    if (a < ls && i - a <= 32768 && i - a != bd) {
                        const uint32_t l = lz_match_len(s + a, s + i, maxl);
                        if (l > best) {
                            best = l;
                            bd = (uint32_t)(i - a);
                        }
                    }
                }
                if (best >= 5 || (best == 4 && bd <= 4096)) {
                    out.push_back({(uint32_t)i, best, bd});
                    const size_t e = i + best;
                    for (size_t k = i + 1; k < e && k + 4 <= le; ++k) ht[lz_hash4(s + k)] = (int64_t)k;
                    i = e;
                } else {
                    ++i;
                }
            }
            last_head = ls;
        }
        ls = le + 1;
    }
}

// Run-length coded code lengths (RFC 1951 §3.2.7 symbols 16, 17, 18): (symbol, extra) pairs.
inline size_t rle_lengths(const uint8_t* L, int n, uint8_t* sym, uint8_t* xtra) {
    size_t k = 0;
    for (int i = 0; i < n;) {
        int r = 1;
        while (i + r < n && L[i + r] == L[i]) ++r;
        if (L[i] == 0) {
            int left = r;
            while (left >= 11) {
                const int t = std::min(left, 138);
                sym[k] = 18, xtra[k++] = (uint8_t)(t - 11);
                left -= t;
            }
            if (left >= 3) {
                sym[k] = 17, xtra[k++] = (uint8_t)(left - 3);
                left = 0;
            }
            while (left-- > 0) sym[k] = 0, xtra[k++] = 0;
        } else {
            sym[k] = L[i], xtra[k++] = 0;
            int left = r - 1;
            while (left >= 3) {
                const int t = std::min(left, 6);
                sym[k] = 16, xtra[k++] = (uint8_t)(t - 3);
                left -= t;
            }
            while (left-- > 0) sym[k] = L[i], xtra[k++] = 0;
        }
        i += r;
    }
    return k;
}

// Append `len` (<= 49) bits with at most 7 pending; stores 8 bytes (the output keeps slack).
inline void pack_bits(uint64_t& buf, int& nb, uint8_t*& p, uint64_t v, int len) {
    buf |= v << nb;
    nb += len;
    std::memcpy(p, &buf, 8);
    p += nb >> 3;
    buf >>= nb & ~7;
    nb &= 7;
}

// Literals src[0, n) through the code table tab (code | length << 16), three per store.
inline void pack_lits(uint64_t& buf, int& nb, uint8_t*& p, const uint32_t* tab, const uint8_t* src,
                      size_t n) {
    size_t i = 0;
    for (; i + 3 <= n; i += 3) {
        const uint32_t e0 = tab[src[i]], e1 = tab[src[i + 1]], e2 = tab[src[i + 2]];
        const int l0 = (int)(e0 >> 16), l01 = l0 + (int)(e1 >> 16);
        const uint64_t v = (uint64_t)(e0 & 0xFFFFu) | ((uint64_t)(e1 & 0xFFFFu) << l0) |
                           ((uint64_t)(e2 & 0xFFFFu) << l01);
        pack_bits(buf, nb, p, v, l01 + (int)(e2 >> 16));
    }
    for (; i < n; ++i) pack_bits(buf, nb, p, tab[src[i]] & 0xFFFFu, (int)(tab[src[i]] >> 16));
}

// The codes of one kind of block: literal/length and distance code lengths and codes from the
// symbol frequencies (freq[256] = the end-of-block count), and the block header after BFINAL
// (BTYPE, HLIT, HDIST, HCLEN, the code-length code, the run-length coded lengths) as chunks of
// <= 48 bits, so blocks of one kind can repeat it cheaply.
struct LzCode {
    uint8_t ll[286], dl[30];
    uint16_t code[286], dcode[30];
    uint32_t tab[256];                              // literal code | length << 16
    int nlit = 257, ndist = 2;
    std::vector<std::pair<uint64_t, int>> hdr;
    uint64_t hdr_bits = 0;

    void build(const uint32_t* freq, const uint32_t* dfreq) {
        huff_lengths(freq, 286, 15, ll);
        nlit = 286;
        while (nlit > 257 && ll[nlit - 1] == 0) --nlit;
        huff_lengths(dfreq, 30, 15, dl);
        int used = 0;
        for (int s = 0; s < 30; ++s) used += dl[s] ? 1 : 0;
        if (used < 2) {   // no or one distance code: complete it with length-1 codes 0 / 1
            if (!dl[0]) dl[0] = 1;
            else dl[1] = 1;
            if (used == 0) dl[1] = 1;
        }
        ndist = 30;
        while (ndist > 1 && dl[ndist - 1] == 0) --ndist;
        huff_codes(ll, 286, code);
        huff_codes(dl, 30, dcode);
        for (int s = 0; s < 256; ++s) tab[s] = (uint32_t)code[s] | ((uint32_t)ll[s] << 16);

        uint8_t L[286 + 30];
        std::memcpy(L, ll, (size_t)nlit);
        std::memcpy(L + nlit, dl, (size_t)ndist);
        uint8_t rs[286 + 30], rx[286 + 30];
        const size_t nr = rle_lengths(L, nlit + ndist, rs, rx);
        uint32_t cf[19] = {0};
        for (size_t k = 0; k < nr; ++k) cf[rs[k]]++;
        int cu = 0;
        for (int s = 0; s < 19; ++s) cu += cf[s] ? 1 : 0;
        if (cu < 2) cf[cf[0] ? 1 : 0]++;
        uint8_t cl[19];
        huff_lengths(cf, 19, 7, cl);
        uint16_t cc[19];
        huff_codes(cl, 19, cc);
        static const uint8_t kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
        int hclen = 19;
        while (hclen > 4 && cl[kOrder[hclen - 1]] == 0) --hclen;
        hdr.clear();
        hdr_bits = 0;
        uint64_t acc = 0;
        int an = 0;
        auto put = [&](uint64_t v, int len) {
            if (an + len > 48) {
                hdr.emplace_back(acc, an);
                acc = 0;
                an = 0;
            }
            acc |= v << an;
            an += len;
            hdr_bits += (uint64_t)len;
        };
        put(2u, 2);   // dynamic Huffman
        put((uint64_t)(nlit - 257), 5);
        put((uint64_t)(ndist - 1), 5);
        put((uint64_t)(hclen - 4), 4);
        for (int k = 0; k < hclen; ++k) put(cl[kOrder[k]], 3);
        static const uint8_t kRx[3] = {2, 3, 7};
        for (size_t k = 0; k < nr; ++k) {
            put(cc[rs[k]], cl[rs[k]]);
            if (rs[k] >= 16) put(rx[k], kRx[rs[k] - 16]);
        }
        if (an) hdr.emplace_back(acc, an);
    }
    // Bits of the coded symbols (extra bits not counted: they are the same under any code).
    uint64_t cost(const uint32_t* freq, const uint32_t* dfreq) const {
        uint64_t c = 0;
        for (int s = 0; s < 286; ++s) c += (uint64_t)freq[s] * ll[s];
        for (int s = 0; s < 30; ++s) c += (uint64_t)dfreq[s] * dl[s];
        return c;
    }
};

struct Packer {
    uint64_t buf = 0;
    int nb = 0;   // < 8 between calls
    uint8_t* p;
};

// One block of src[a, b) with the matches m[0, nm) (inside the range) under the codes C.
inline void lz_emit(Packer& k, const LzCode& C, const uint8_t* src, size_t a, size_t b,
                    const LzMatch* m, size_t nm, bool final) {
    const LzTables& T = lz_tables();
    pack_bits(k.buf, k.nb, k.p, final ? 1u : 0u, 1);
    for (const auto& h : C.hdr) pack_bits(k.buf, k.nb, k.p, h.first, h.second);
    size_t cur = a;
    for (size_t j = 0; j < nm; ++j) {
        pack_lits(k.buf, k.nb, k.p, C.tab, src + cur, m[j].pos - cur);
        const uint32_t len = m[j].len, d = m[j].dist;
        const int ls = T.len_sym[len], ds = (int)T.dsym(d);
        const int lc = 257 + ls;
        uint64_t v = C.code[lc];
        int n = C.ll[lc];
        v |= (uint64_t)(len - T.len_base[ls]) << n;
        n += T.len_xb[ls];
        v |= (uint64_t)C.dcode[ds] << n;
        n += C.dl[ds];
        v |= (uint64_t)(d - T.dist_base[ds]) << n;
        n += T.dist_xb[ds];
        pack_bits(k.buf, k.nb, k.p, v, n);
        cur = m[j].pos + len;
    }
    pack_lits(k.buf, k.nb, k.p, C.tab, src + cur, b - cur);
    pack_bits(k.buf, k.nb, k.p, C.code[256], C.ll[256]);
}

// Literal histogram of s[0, n) added into f.
inline void lz_hist(const uint8_t* s, size_t n, uint32_t* f) {
    uint32_t h[4][256];
    std::memset(h, 0, sizeof(h));
    size_t i = 0;
    for (; i + 4 <= n; i += 4) {
        h[0][s[i]]++;
        h[1][s[i + 1]]++;
        h[2][s[i + 2]]++;
        h[3][s[i + 3]]++;
    }
    for (; i < n; ++i) h[0][s[i]]++;
    for (int c = 0; c < 256; ++c) f[c] += h[0][c] + h[1][c] + h[2][c] + h[3][c];
}

// Symbol frequencies of src[a, b) with the matches m[0, nm) added into freq / dfreq.
inline void lz_freq(const uint8_t* src, size_t a, size_t b, const LzMatch* m, size_t nm,
                    uint32_t* freq, uint32_t* dfreq) {
    const LzTables& T = lz_tables();
    size_t cur = a;
    for (size_t j = 0; j < nm; ++j) {
        lz_hist(src + cur, m[j].pos - cur, freq);
        freq[257 + T.len_sym[m[j].len]]++;
        dfreq[T.dsym(m[j].dist)]++;
        cur = m[j].pos + m[j].len;
    }
    lz_hist(src + cur, b - cur, freq);
}

// Raw DEFLATE stream of src[0, n) into out (huff_bound(n) bytes); returns its length.  Two
// layouts, whichever the code lengths price lower for the member:
//  - split: one block per sequence line and one per stretch between them (the "+" line, the
//    quality line, the next header), each kind under its own codes — bases cost ~2.25 bits
//    instead of sharing one table with ~40 quality symbols, for two block headers (~40 B) per
//    record;
//  - mixed: blocks of ~256 KiB, one table each (short reads, FASTA without headers, text that
//    is not FASTQ).
inline size_t fq_deflate(const uint8_t* src, size_t n, uint8_t* out) {
    // positions are 32-bit (the writers' members are <= 1 MiB); a larger single member from
    // dmx_io_gzip gets the Huffman-only stream
    if (n == 0 || n >= ((size_t)1 << 31)) return huff_deflate(src, n, out);
    thread_local std::vector<LzMatch> ms;
    thread_local std::vector<std::pair<uint32_t, uint32_t>> sq;
    fq_scan(src, n, ms, sq);
    Packer k;
    k.p = out;
    thread_local LzCode CS, CQ, CM;
    bool split = false;
    if (!sq.empty()) {
        uint32_t fs[286] = {0}, fq[286] = {0}, ds[30] = {0}, dq[30] = {0};
        size_t cur = 0, j = 0, nq = 0;
        for (const auto& r : sq) {
            size_t j1 = j;
            while (j1 < ms.size() && ms[j1].pos < r.first) ++j1;
            if (r.first > cur) {
                lz_freq(src, cur, r.first, ms.data() + j, j1 - j, fq, dq);
                ++nq;
            }
            lz_hist(src + r.first, r.second - r.first, fs);
            cur = r.second;
            j = j1;
        }
        if (cur < n) {
            lz_freq(src, cur, n, ms.data() + j, ms.size() - j, fq, dq);
            ++nq;
        }
        fs[256] = (uint32_t)sq.size();
        fq[256] = (uint32_t)std::max<size_t>(nq, 1);
        CS.build(fs, ds);
        CQ.build(fq, dq);
        uint32_t fm[286], dm[30];
        const uint32_t nblk = (uint32_t)(n / (256u << 10) + 1);
        for (int s = 0; s < 286; ++s) fm[s] = fs[s] + fq[s];
        for (int s = 0; s < 30; ++s) dm[s] = dq[s];
        fm[256] = nblk;
        CM.build(fm, dm);
        const uint64_t c_split = CS.cost(fs, ds) + CQ.cost(fq, dq) +
                                 (uint64_t)sq.size() * (1 + CS.hdr_bits) + (uint64_t)nq * (1 + CQ.hdr_bits);
        const uint64_t c_mixed = CM.cost(fm, dm) + (uint64_t)nblk * (1 + CM.hdr_bits);
        split = c_split < c_mixed;
    }
    if (split) {
        size_t cur = 0, j = 0;
        for (size_t r = 0; r < sq.size(); ++r) {
            const size_t a = sq[r].first, b = sq[r].second;
            size_t j1 = j;
            while (j1 < ms.size() && ms[j1].pos < a) ++j1;
            if (a > cur) lz_emit(k, CQ, src, cur, a, ms.data() + j, j1 - j, false);
            lz_emit(k, CS, src, a, b, nullptr, 0, b == n);
            cur = b;
            j = j1;
        }
        if (cur < n) lz_emit(k, CQ, src, cur, n, ms.data() + j, ms.size() - j, true);
    } else {
        constexpr size_t kBlock = 256u << 10;
        size_t b0 = 0, j = 0;
        while (b0 < n) {
            size_t b1 = std::min(n, b0 + kBlock), j1 = j;
            while (j1 < ms.size() && ms[j1].pos < b1) {   // a block ends after whole matches
                b1 = std::max(b1, (size_t)ms[j1].pos + ms[j1].len);
                ++j1;
            }
            uint32_t fm[286] = {0}, dm[30] = {0};
            lz_freq(src, b0, b1, ms.data() + j, j1 - j, fm, dm);
            fm[256] = 1;
            CM.build(fm, dm);
            lz_emit(k, CM, src, b0, b1, ms.data() + j, j1 - j, b1 == n);
            b0 = b1;
            j = j1;
        }
    }
    BitWriter bw(k.p);   // pad the last byte
    bw.buf = k.buf;
    bw.n = k.nb;
    bw.flush();
    return (size_t)(bw.p - out);
}

}  // namespace dmxz
