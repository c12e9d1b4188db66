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

}  // namespace dmxz
