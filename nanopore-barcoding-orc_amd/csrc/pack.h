// pack.h — host-side 2-bit packer shared by libdmx (dmx_pack) and libdmx_io (fused
// parse + pack).  Layout (include/dmx.h): A=0 C=1 G=2 T=3, 16 nt per little-endian u32 word;
// a 1-bit "no match" mask per nt for any non-ACGT byte (cutadapt's read wildcard table maps
// N and other characters to nothing); every read starts on a 32-nt boundary
// after DMX_PACK_PAD nt of padding.  Lower-case acgt pack like upper case (reads are matched
// upper-cased).
#pragma once
#include <cstddef>
#include <cstdint>

namespace dmx {

constexpr int kPackAlign = 32;   // every read starts on a 32-nt (one nmask word) boundary

struct PackTables {
    uint8_t code[256];
    uint8_t nflag[256];
    PackTables() {
        for (int i = 0; i < 256; ++i) {
            code[i] = 0;
            nflag[i] = 1;
        }
        const char* s = "ACGT";
        for (int k = 0; k < 4; ++k) {
            code[(uint8_t)s[k]] = code[(uint8_t)(s[k] + 32)] = (uint8_t)k;
            nflag[(uint8_t)s[k]] = nflag[(uint8_t)(s[k] + 32)] = 0;
        }
    }
};
inline const PackTables& pack_tables() {
    static const PackTables t;
    return t;
}

// Pack one read of n nt from src into the word arrays at nt offset g0 (a multiple of 32).
// Every word of the read's ceil(n/32) groups is written (zero tail), and reads are laid out
// back to back on 32-nt boundaries, so only the DMX_PACK_PAD head and the tail after the last
// read need zeroing by the caller.
inline void pack_one(const uint8_t* src, uint32_t n, uint64_t g0, uint32_t* seq, uint32_t* nmask) {
    const PackTables& T = pack_tables();
    uint32_t* sw = seq + g0 / 16;
    uint32_t* nw = nmask + g0 / 32;
    for (uint32_t x = 0; x < n; x += 32) {
        const uint32_t cnt = n - x < 32u ? n - x : 32u;
        uint32_t w0 = 0, w1 = 0, nb = 0;
        for (uint32_t y = 0; y < cnt; ++y) {
            const uint8_t ch = src[x + y];
            const uint32_t cd = T.code[ch];
            if (y < 16) w0 |= cd << (2 * y);
            else w1 |= cd << (2 * (y - 16));
            nb |= (uint32_t)T.nflag[ch] << y;
        }
        sw[x / 16] = w0;
        sw[x / 16 + 1] = w1;   // whole 32-nt groups: no word of a read's span is left unwritten
        nw[x / 32] = nb;
    }
}

// The reverse complement of the n nt at src, packed like pack_one: nt y is the complement of
// src[n - 1 - y] (code ^ 3: A<->T, C<->G); a non-ACGT byte stays no-match (code 0, mask bit),
// exactly what pack_one gives for the reverse-complemented text.
inline void pack_one_rc(const uint8_t* src, uint32_t n, uint64_t g0, uint32_t* seq,
                        uint32_t* nmask) {
    const PackTables& T = pack_tables();
    uint32_t* sw = seq + g0 / 16;
    uint32_t* nw = nmask + g0 / 32;
    for (uint32_t x = 0; x < n; x += 32) {
        const uint32_t cnt = n - x < 32u ? n - x : 32u;
        uint32_t w0 = 0, w1 = 0, nb = 0;
        for (uint32_t y = 0; y < cnt; ++y) {
            const uint8_t ch = src[n - 1 - (x + y)];
            const uint32_t nf = T.nflag[ch];
            const uint32_t cd = nf ? 0u : (T.code[ch] ^ 3u);
            if (y < 16) w0 |= cd << (2 * y);
            else w1 |= cd << (2 * (y - 16));
            nb |= nf << y;
        }
        sw[x / 16] = w0;
        sw[x / 16 + 1] = w1;
        nw[x / 32] = nb;
    }
}

inline void pack_range(const uint8_t* ascii, const uint64_t* offsets, const uint32_t* lens,
                       size_t lo, size_t hi, const uint64_t* out_offsets, uint32_t* seq,
                       uint32_t* nmask) {
    for (size_t r = lo; r < hi; ++r) pack_one(ascii + offsets[r], lens[r], out_offsets[r], seq, nmask);
}

}  // namespace dmx
