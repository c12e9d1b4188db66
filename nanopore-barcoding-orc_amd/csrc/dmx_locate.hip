// dmx_locate.hip — exact degenerate-motif location on the GPU (`seqkit locate -d`), the
// residual-primer failsafe of scripts/04_cleaning_primers.sh:397-460:
//
//   seqkit subseq -r 1:100 / -r -100:-1 trimmed.fasta > ends      (:414-419)
//   seqkit locate -d --pattern-file primers ends > locations      (:422)
//   seqkit grep -v -f ids trimmed.fasta > cleanest                (:436)
//
// seqkit (v2.x, not vendored in /root/reference) turns each degenerate pattern into a regular
// expression of IUPAC character classes and reports every match — overlapping ones included
// (greedy mode restarts one position after each match start) — on the positive strand and,
// by default, on the negative strand (the pattern searched on the reverse complement of the
// sequence, reported in positive-strand coordinates).  Matching is case-sensitive without -i.
//
// MI355X design: the failsafe reads ~200 nt per record (two 100-nt ends) against a handful of
// primers (<= 64 nt) — HBM-bound byte work, no DP.  One lane per (record, pattern): a
// bit-parallel Shift-And over the record's bytes keeps both strands' states in two 64-bit
// words (the negative strand = the reverse-complemented pattern scanned on the positive
// strand: a match of it ending at e is a match of the pattern on the reverse complement, same
// positive-strand interval).  The per-(pattern, strand, character class) match masks sit in
// LDS; lanes of a wave take consecutive patterns of the same record, so a record's bytes are
// fetched once per wave from L2 and broadcast.  Hits (rare: the failsafe fires only on
// residual primers) are appended with one atomic each.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "dmx_internal.h"

namespace dmx {

constexpr int kLocClasses = 9;          // A C G T(U) a c g t(u), other
constexpr int kLocMaxPatterns = 128;    // LDS: 128 x 2 x 9 x 8 B = 18 KB
constexpr int kLocBlock = 256;

struct LocPattern {
    uint64_t B[2][kLocClasses];   // [strand][class]: bit i set iff pattern position i admits it
    uint64_t hit;                 // 1 << (len - 1)
};

struct LocArgs {
    const uint8_t* ascii;
    const uint64_t* offs;
    const uint32_t* lens;
    uint64_t n_seqs;
    const LocPattern* pat;
    int n_pat;
    int both;
    const uint8_t* cls;            // 256-entry byte -> class table
    dmx_hit* hits;
    unsigned long long* n_hits;
    uint64_t cap;
};

__device__ __forceinline__ void loc_emit(const LocArgs& A, uint64_t s, int p, int strand,
                                         uint32_t end) {
    const unsigned long long i = atomicAdd(A.n_hits, 1ull);
    if (i < A.cap) {
        dmx_hit h;
        h.seq = s;
        h.pattern = p;
        h.strand = strand;
        h.end = (int32_t)end;
        h.start = 0;   // host derives start = end - len + 1
        A.hits[i] = h;
    }
}

__global__ __launch_bounds__(kLocBlock) void locate_kernel(LocArgs A) {
    __shared__ LocPattern s_pat[kLocMaxPatterns];
    __shared__ uint8_t s_cls[256];
    for (int i = threadIdx.x; i < A.n_pat * (int)(sizeof(LocPattern) / 8); i += blockDim.x)
        reinterpret_cast<uint64_t*>(s_pat)[i] = reinterpret_cast<const uint64_t*>(A.pat)[i];
    for (int i = threadIdx.x; i < 256; i += blockDim.x) s_cls[i] = A.cls[i];
    __syncthreads();
    const uint64_t total = A.n_seqs * (uint64_t)A.n_pat;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t s = t / (uint64_t)A.n_pat;
        const int p = (int)(t - s * (uint64_t)A.n_pat);
        const LocPattern& P = s_pat[p];
        const uint8_t* src = A.ascii + A.offs[s];
        const uint32_t n = A.lens[s];
        uint64_t dp = 0, dm = 0;
        // aligned 4-byte loads; the first word may start before the record
        const uintptr_t a0 = reinterpret_cast<uintptr_t>(src);
        const uint32_t* w = reinterpret_cast<const uint32_t*>(a0 & ~(uintptr_t)3);
        uint32_t sh = (uint32_t)(a0 & 3u);
        uint32_t pos = 0;
        while (pos < n) {
            const uint32_t word = *w++ >> (8 * sh);
            const uint32_t cnt = min(4u - sh, n - pos);
            sh = 0;
            for (uint32_t b = 0; b < cnt; ++b, ++pos) {
                const int c = s_cls[(word >> (8 * b)) & 0xFFu];
                dp = ((dp << 1) | 1ull) & P.B[0][c];
                dm = ((dm << 1) | 1ull) & P.B[1][c];
                if (dp & P.hit) loc_emit(A, s, p, 0, pos + 1);
                if ((dm & P.hit) && A.both) loc_emit(A, s, p, 1, pos + 1);
            }
        }
    }
}

}  // namespace dmx

using namespace dmx;

namespace {

// IUPAC code -> admitted bases (bit 0 A, 1 C, 2 G, 3 T/U); 0 = not a nucleotide code.
int iupac_bases(char ch) {
    switch (ch) {
        case 'A': return 1;
        case 'C': return 2;
        case 'G': return 4;
        case 'T': case 'U': return 8;
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

int comp_bases(int b) {   // A<->T, C<->G
    return ((b & 1) << 3) | ((b & 8) >> 3) | ((b & 2) << 1) | ((b & 4) >> 1);
}

}  // namespace

extern "C" int dmx_locate(dmx_ctx* c, const char* const* patterns, const int* plens,
                          int n_patterns, int flags, const uint8_t* ascii,
                          const uint64_t* offsets, const uint32_t* lens, size_t n_seqs,
                          dmx_hit* out, size_t cap, uint64_t* n_hits) {
    if (!c || !n_hits || (n_patterns > 0 && (!patterns || !plens)) || (n_seqs && (!offsets || !lens)) ||
        (cap && !out))
        return DMX_E_INVALID;
    if (n_patterns < 0 || n_patterns > kLocMaxPatterns) {
        c->err = "dmx_locate: 0.." + std::to_string(kLocMaxPatterns) + " patterns supported";
        return DMX_E_UNSUPPORTED;
    }
    const bool icase = flags & DMX_LOC_IGNORE_CASE;
    std::vector<LocPattern> pat(std::max(n_patterns, 1));
    for (int p = 0; p < n_patterns; ++p) {
        const int L = plens[p];
        if (L < 1 || L > 64) {
            c->err = "dmx_locate: pattern " + std::to_string(p) + " has length " +
                     std::to_string(L) + " (1..64 supported)";
            return DMX_E_UNSUPPORTED;
        }
        LocPattern& P = pat[p];
        std::memset(&P, 0, sizeof(P));
        P.hit = 1ull << (L - 1);
        for (int i = 0; i < L; ++i) {
            const char raw = patterns[p][i];
            const bool lower = raw >= 'a' && raw <= 'z';
            const char up = lower ? (char)(raw - 32) : raw;
            const int b = iupac_bases(up);
            if (!b) {
                c->err = std::string("dmx_locate: pattern ") + std::to_string(p) +
                         " has a non-IUPAC character '" + raw + "'";
                return DMX_E_INVALID;
            }
            // positive strand: position i; negative strand: reverse complement, position
            // L-1-i of the reverse-complemented pattern
            const int bc = comp_bases(b);
            const int base_cls = (lower && !icase) ? 4 : 0;
            for (int k = 0; k < 4; ++k) {
                if (b & (1 << k)) P.B[0][base_cls + k] |= 1ull << i;
                if (bc & (1 << k)) P.B[1][base_cls + k] |= 1ull << (L - 1 - i);
            }
        }
    }
    uint8_t cls[256];
    for (int i = 0; i < 256; ++i) cls[i] = 8;
    const char* up = "ACGT";
    const char* lo = "acgt";
    for (int k = 0; k < 4; ++k) {
        cls[(uint8_t)up[k]] = (uint8_t)k;
        cls[(uint8_t)lo[k]] = (uint8_t)(icase ? k : 4 + k);
    }
    cls[(uint8_t)'U'] = 3;
    cls[(uint8_t)'u'] = (uint8_t)(icase ? 3 : 7);

    *n_hits = 0;
    if (n_seqs == 0 || n_patterns == 0) return DMX_OK;
    if (hipSetDevice(c->device) != hipSuccess) {
        c->err = "dmx_locate: hipSetDevice failed";
        return DMX_E_HIP;
    }
    uint64_t total = 0;
    for (size_t i = 0; i < n_seqs; ++i) total = std::max(total, offsets[i] + lens[i]);
    uint8_t* d_ascii = nullptr;
    uint64_t* d_offs = nullptr;
    uint32_t* d_lens = nullptr;
    LocPattern* d_pat = nullptr;
    uint8_t* d_cls = nullptr;
    dmx_hit* d_hits = nullptr;
    unsigned long long* d_n = nullptr;
    int rc = DMX_OK;
    auto ck = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && rc == DMX_OK) {
            c->err = std::string("dmx_locate: ") + what + ": " + hipGetErrorString(e);
            rc = DMX_E_HIP;
        }
        return rc == DMX_OK;
    };
    hipStream_t st = c->stream;
    // +4: the kernel's aligned word loads may reach 3 bytes past the last record
    if (ck(hipMalloc((void**)&d_ascii, total + 8), "hipMalloc") &&
        ck(hipMalloc((void**)&d_offs, n_seqs * 8), "hipMalloc") &&
        ck(hipMalloc((void**)&d_lens, n_seqs * 4), "hipMalloc") &&
        ck(hipMalloc((void**)&d_pat, sizeof(LocPattern) * n_patterns), "hipMalloc") &&
        ck(hipMalloc((void**)&d_cls, 256), "hipMalloc") &&
        ck(hipMalloc((void**)&d_hits, sizeof(dmx_hit) * std::max<size_t>(cap, 1)), "hipMalloc") &&
        ck(hipMalloc((void**)&d_n, 8), "hipMalloc") &&
        ck(hipMemsetAsync(d_ascii + total, 0, 8, st), "hipMemset") &&
        ck(hipMemcpyAsync(d_ascii, ascii, total, hipMemcpyHostToDevice, st), "upload") &&
        ck(hipMemcpyAsync(d_offs, offsets, n_seqs * 8, hipMemcpyHostToDevice, st), "upload") &&
        ck(hipMemcpyAsync(d_lens, lens, n_seqs * 4, hipMemcpyHostToDevice, st), "upload") &&
        ck(hipMemcpyAsync(d_pat, pat.data(), sizeof(LocPattern) * n_patterns,
                          hipMemcpyHostToDevice, st), "upload") &&
        ck(hipMemcpyAsync(d_cls, cls, 256, hipMemcpyHostToDevice, st), "upload") &&
        ck(hipMemsetAsync(d_n, 0, 8, st), "hipMemset")) {
        LocArgs A{d_ascii, d_offs, d_lens, (uint64_t)n_seqs, d_pat, n_patterns,
                  (flags & DMX_LOC_ONLY_POSITIVE) ? 0 : 1, d_cls, d_hits, d_n, (uint64_t)cap};
        const uint64_t tasks = (uint64_t)n_seqs * (uint64_t)n_patterns;
        const int grid = (int)std::min<uint64_t>((tasks + kLocBlock - 1) / kLocBlock, 8192);
        hipLaunchKernelGGL(locate_kernel, dim3(grid), dim3(kLocBlock), 0, st, A);
        ck(hipGetLastError(), "locate_kernel launch");
        unsigned long long nh = 0;
        if (ck(hipMemcpyAsync(&nh, d_n, 8, hipMemcpyDeviceToHost, st), "download") &&
            ck(hipStreamSynchronize(st), "sync")) {
            *n_hits = nh;
            const size_t got = (size_t)std::min<unsigned long long>(nh, cap);
            if (got && ck(hipMemcpy(out, d_hits, got * sizeof(dmx_hit), hipMemcpyDeviceToHost),
                          "download")) {
                for (size_t i = 0; i < got; ++i)
                    out[i].start = out[i].end - plens[out[i].pattern] + 1;
            }
        }
    }
    void* bufs[] = {d_ascii, d_offs, d_lens, d_pat, d_cls, d_hits, d_n};
    for (void* b : bufs)
        if (b) hipFree(b);
    return rc;
}
