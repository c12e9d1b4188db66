// dmx_io.cpp — libdmx_io: native FASTQ/FASTA(.gz) ingest fused with the 2-bit packer, and
// per-bin writers with parallel gzip (include/dmx_io.h).
//
// Record conventions restated from dnaio/xopen as cutadapt 4.9 uses them (not vendored in
// /root/reference):
//  * FASTQ: 4 lines per record; line 1 starts with '@' and its remainder is the record name;
//    line 3 starts with '+'; sequence and quality lengths must agree; "\r\n" line ends accepted.
//    Output records are written as "@name\nSEQ\n+\nQUAL\n".
//  * FASTA: '>' name line followed by any number of sequence lines, joined (whitespace at line
//    ends stripped); output records are written on one line, ">name\nSEQ\n".
//  * A reverse-complemented read (--rc) gets " rc" appended to its name, its sequence reverse
//    complemented (IUPAC codes complemented, case kept) and its qualities reversed.
//  * gzip output is written as a series of independent members (a valid gzip file; readers
//    decompress it as one stream); an output that receives no records is still a valid (empty)
//    gzip file, like xopen's.
#include "../../include/dmx_io.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "dmx_deflate.h"
#include "dmx_inflate.h"
#include "pack.h"

// libdeflate (system library of the image; only the runtime .so is installed, so the few
// entry points used are declared here): whole-member raw-DEFLATE decompression and CRC-32.
extern "C" {
struct libdeflate_decompressor;
libdeflate_decompressor* libdeflate_alloc_decompressor(void);
void libdeflate_free_decompressor(libdeflate_decompressor* d);
int libdeflate_deflate_decompress(libdeflate_decompressor* d, const void* in, size_t in_nbytes,
                                  void* out, size_t out_nbytes_avail, size_t* actual_out_nbytes);
uint32_t libdeflate_crc32(uint32_t crc, const void* buffer, size_t len);
struct libdeflate_compressor;
libdeflate_compressor* libdeflate_alloc_compressor(int compression_level);
size_t libdeflate_deflate_compress(libdeflate_compressor* c, const void* in, size_t in_nbytes,
                                   void* out, size_t out_nbytes_avail);
size_t libdeflate_deflate_compress_bound(libdeflate_compressor* c, size_t in_nbytes);
void libdeflate_free_compressor(libdeflate_compressor* c);
}

namespace {

constexpr uint64_t kPad = 64;   // DMX_PACK_PAD (include/dmx.h)

// Large buffers (>= 32 MiB, which glibc maps on their own) are marked MADV_HUGEPAGE before
// their first touch: on the GPU box (THP "madvise") filling 3 GB then takes 0.19 s instead of
// 0.51 s and releasing it at exit 0.1 s less (tools/thp_probe.py, profiles/r5_thp_probe.json).
// DMX_NO_HUGEPAGES=1 leaves them on 4 KiB pages.
const bool kHugePages = [] {
    const char* e = getenv("DMX_NO_HUGEPAGES");
    return !(e && e[0] == '1');
}();

inline void advise_huge(void* p, size_t bytes) {
    if (!kHugePages || bytes < (32u << 20)) return;
    const uintptr_t s = ((uintptr_t)p + 4095) & ~(uintptr_t)4095;
    const uintptr_t e = ((uintptr_t)p + bytes) & ~(uintptr_t)4095;
    if (e > s) madvise((void*)s, e - s, MADV_HUGEPAGE);   // advisory: failure changes nothing
}

// Allocator that leaves trivially constructible elements uninitialised on resize: batch
// buffers are hundreds of MB and every byte is written by read/inflate/pack anyway.
template <typename T>
struct NoInit : std::allocator<T> {
    template <typename U>
    struct rebind {
        using other = NoInit<U>;
    };
    NoInit() = default;
    template <typename U>
    NoInit(const NoInit<U>&) {}
    T* allocate(size_t n) {
        T* p = std::allocator<T>::allocate(n);
        advise_huge(p, n * sizeof(T));
        return p;
    }
    template <typename U>
    void construct(U* p) noexcept {
        ::new (static_cast<void*>(p)) U;
    }
    template <typename U, typename... A>
    void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
using Bytes = std::vector<uint8_t, NoInit<uint8_t>>;
using Words = std::vector<uint32_t, NoInit<uint32_t>>;

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
const bool kIoDebug = getenv("DMX_IO_DEBUG") != nullptr;

// dmx_io_set_memory_budget (0 = none)
std::atomic<uint64_t> g_mem_budget{0};

int clamp_threads(int t) {
    if (t <= 0) t = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(t, 64));
}

// Run f(t) for t in [0, nth) on nth threads (the calling thread takes t = 0).
// Persistent workers for parallel(): the reader and the writer fan out to -j threads several
// times per batch (inflate, newline scan, parse, pack, render, compress), and with batches of a
// few tens of MB (a round-2 call's bin) thread creation per fan-out became a visible cost.
// Workers claim the indices of a fan-out from a shared counter; the caller claims too and then
// waits for the indices the workers took, so concurrent fan-outs (reader and writer threads)
// never wait on each other's queue position.
struct WorkPool {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    std::vector<std::thread> workers;
    bool stop = false;
    ~WorkPool() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : workers) t.join();
    }
    void loop() {
        for (;;) {
            std::function<void()> job;
            {
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return stop || !q.empty(); });
                if (q.empty()) return;
                job = std::move(q.front());
                q.pop_front();
            }
            job();
        }
    }
    void submit(int n, const std::function<void()>& job) {
        {
            std::lock_guard<std::mutex> g(mu);
            while ((int)workers.size() < std::min(n, 255)) workers.emplace_back([this] { loop(); });
            for (int i = 0; i < n; ++i) q.push_back(job);
        }
        if (n == 1) cv.notify_one();
        else cv.notify_all();
    }
};
WorkPool& work_pool() {
    static WorkPool* p = new WorkPool();   // never destroyed: workers may outlive static dtors
    return *p;
}

template <typename F>
void parallel(int nth, F&& f) {
    if (nth <= 1) {
        f(0);
        return;
    }
    struct Group {
        std::atomic<int> next{1};
        int n = 0;
        std::mutex m;
        std::condition_variable cv;
        int done = 0;
        std::function<void(int)>* fn = nullptr;
        void run_claimed() {   // claim and run indices until none is left
            for (int t; (t = next.fetch_add(1)) < n;) {
                (*fn)(t);
                std::lock_guard<std::mutex> g(m);
                if (++done == n - 1) cv.notify_all();
            }
        }
    };
    std::function<void(int)> fn = [&f](int t) { f(t); };
    auto g = std::make_shared<Group>();
    g->n = nth;
    g->fn = &fn;
    work_pool().submit(nth - 1, [g] { g->run_claimed(); });
    f(0);
    g->run_claimed();
    std::unique_lock<std::mutex> l(g->m);
    g->cv.wait(l, [&] { return g->done == nth - 1; });
}

// ------------------------------------------------------------------------------------------
// sources

struct Source {
    virtual ~Source() = default;
    virtual long read(uint8_t* dst, size_t cap) = 0;   // bytes read, 0 = end, < 0 = error
    virtual size_t chunk_hint() const { return 8u << 20; }   // preferred read size
    std::string err;
};

struct FdSource : Source {
    int fd = -1;
    bool own = false;
    int threads = 1;        // regular files: reads of >= 8 MB as parallel preads
    int kind = 0;           // 0 unknown, 1 regular file (preads at `off`), 2 other (read(2))
    int64_t off = 0, size = 0;
    ~FdSource() override {
        if (own && fd >= 0) ::close(fd);
    }
    long read(uint8_t* dst, size_t cap) override {
        if (kind == 0) {
            struct stat st;
            kind = 2;
            if (fstat(fd, &st) == 0 && S_ISREG(st.st_mode)) {
                const off_t at = lseek(fd, 0, SEEK_CUR);
                if (at >= 0) {
                    kind = 1;
                    off = (int64_t)at;
                    size = (int64_t)st.st_size;
                }
            }
        }
        if (kind == 1) {   // the kernel's page-cache copy of a large read on the pool
            if (off >= size) {
                struct stat st;
                if (fstat(fd, &st) == 0) size = (int64_t)st.st_size;
                if (off >= size) return 0;
            }
            const size_t k = (size_t)std::min<int64_t>((int64_t)cap, size - off);
            const int nc = std::max(1, (int)std::min<size_t>((size_t)threads, k >> 22));
            std::atomic<bool> bad{false};
            std::atomic<int> eno{0};
            auto slice = [&](int t) {
                const size_t a = k * (size_t)t / (size_t)nc, b = k * (size_t)(t + 1) / (size_t)nc;
                for (size_t x = a; x < b && !bad;) {
                    const ssize_t n = ::pread(fd, dst + x, b - x, (off_t)(off + (int64_t)x));
                    if (n < 0 && errno == EINTR) continue;
                    if (n <= 0) {   // error, or the file shrank under us
                        eno = n < 0 ? errno : EIO;
                        bad = true;
                        break;
                    }
                    x += (size_t)n;
                }
            };
            if (nc > 1) parallel(nc, slice);
            else slice(0);
            if (bad) {
                err = std::string("read: ") + strerror(eno.load());
                return -1;
            }
            off += (int64_t)k;
            return (long)k;
        }
        size_t got = 0;
        while (got < cap) {
            const ssize_t n = ::read(fd, dst + got, cap - got);
            if (n < 0) {
                if (errno == EINTR) continue;
                err = std::string("read: ") + strerror(errno);
                return -1;
            }
            if (n == 0) break;
            got += (size_t)n;
        }
        return (long)got;
    }
};

// Pushed-back first bytes (format sniffing) in front of another source.
struct PrefixSource : Source {
    std::unique_ptr<Source> inner;
    std::vector<uint8_t> head;
    size_t pos = 0;
    long read(uint8_t* dst, size_t cap) override {
        size_t got = 0;
        if (pos < head.size()) {
            got = std::min(cap, head.size() - pos);
            memcpy(dst, head.data() + pos, got);
            pos += got;
        }
        if (got < cap) {
            const long n = inner->read(dst + got, cap - got);
            if (n < 0) {
                err = inner->err;
                return -1;
            }
            got += (size_t)n;
        }
        return (long)got;
    }
};

// ------------------------------------------------------------------------------------------
// Retained outputs (the round-2 cache of the unchanged 02_cutadapt_loop.sh).
// A sink opened with dmx_sink_retain keeps the uncompressed text it rendered for each gzip output
// (the buffers it compressed: moved, never copied).  At close the file's identity is recorded —
// real path, inode, size, mtime (ns) and the CRC-32 of its first 64 KiB as written — and a later
// dmx_reader_open of the same file, unchanged on disk, reads the text from memory instead of
// reading and inflating the file (then drops it: each bin is read once by the script).  Any
// mismatch reads the file.  Bounded by the caps the sinks were opened with.
struct Retained {
    std::vector<Bytes> pieces;
    uint64_t bytes = 0;
    dev_t dev = 0;
    ino_t ino = 0;
    off_t size = 0;
    int64_t mtime_ns = 0;
    uint32_t head_crc = 0;
};
std::mutex g_ret_mu;
std::map<std::string, Retained> g_retained;
uint64_t g_ret_bytes = 0;

int64_t mtime_ns(const struct stat& st) {
    return (int64_t)st.st_mtim.tv_sec * 1000000000ll + st.st_mtim.tv_nsec;
}

// CRC-32 of the first min(64 KiB, size) bytes of the file; false if unreadable
bool head_crc(const char* path, uint32_t& crc) {
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    uint8_t buf[65536];
    size_t got = 0;
    while (got < sizeof(buf)) {
        const ssize_t n = ::read(fd, buf + got, sizeof(buf) - got);
        if (n < 0 && errno == EINTR) continue;
        if (n <= 0) break;
        got += (size_t)n;
    }
    ::close(fd);
    crc = libdeflate_crc32(0u, buf, got);
    return true;
}

std::string real_path(const char* p) {
    char rp[PATH_MAX];
    return realpath(p, rp) ? std::string(rp) : std::string();
}

// The retained text of `path` if the file on disk is the one that was written (moved out of
// the registry), else false.
bool take_retained(const char* path, Retained& out) {
    const std::string rp = real_path(path);
    if (rp.empty()) return false;
    struct stat st;
    if (::stat(rp.c_str(), &st) != 0) return false;
    Retained r;
    {
        std::lock_guard<std::mutex> g(g_ret_mu);
        auto it = g_retained.find(rp);
        if (it == g_retained.end()) return false;
        r = std::move(it->second);
        g_ret_bytes -= r.bytes;
        g_retained.erase(it);
    }
    uint32_t crc = 0;
    if (r.dev != st.st_dev || r.ino != st.st_ino || r.size != st.st_size ||
        r.mtime_ns != mtime_ns(st) || !head_crc(rp.c_str(), crc) || crc != r.head_crc)
        return false;
    out = std::move(r);
    return true;
}

// The retained text as a source: pieces copied out in order (large reads in parallel).
struct MemSource : Source {
    std::vector<Bytes> pieces;
    size_t pi = 0, off = 0;
    int threads = 1;
    long read(uint8_t* dst, size_t cap) override {
        // the copies of this read: (piece, offset, length, destination)
        struct Cp {
            const uint8_t* s;
            uint8_t* d;
            size_t n;
        };
        std::vector<Cp> cps;
        size_t got = 0;
        const size_t pi0 = pi;
        while (got < cap && pi < pieces.size()) {
            const size_t n = std::min(cap - got, pieces[pi].size() - off);
            cps.push_back({pieces[pi].data() + off, dst + got, n});
            got += n;
            off += n;
            if (off == pieces[pi].size()) {
                ++pi;
                off = 0;
            }
        }
        if (got >= (8u << 20) && threads > 1) {
            // split into ~1 MiB copies over the pool
            std::vector<Cp> parts;
            for (const Cp& c : cps)
                for (size_t a = 0; a < c.n; a += (1u << 20))
                    parts.push_back({c.s + a, c.d + a, std::min<size_t>(1u << 20, c.n - a)});
            std::atomic<size_t> next{0};
            parallel(threads, [&](int) {
                for (size_t k; (k = next.fetch_add(1)) < parts.size();)
                    memcpy(parts[k].d, parts[k].s, parts[k].n);
            });
        } else {
            for (const Cp& c : cps) memcpy(c.d, c.s, c.n);
        }
        for (size_t k = pi0; k < pi; ++k) Bytes().swap(pieces[k]);   // consumed: memory back
        return (long)got;
    }
    size_t chunk_hint() const override { return 64u << 20; }
};

// zlib inflate of a gzip file; concatenated members (pigz / bgzip / our own writer) are read
// as one stream.
struct GzSource : Source {
    std::unique_ptr<Source> raw;
    z_stream zs{};
    std::vector<uint8_t> in;
    bool in_eof = false, ended = false, started = false;
    explicit GzSource(std::unique_ptr<Source> r) : raw(std::move(r)), in(1 << 20) {}
    ~GzSource() override {
        if (started) inflateEnd(&zs);
    }
    bool refill() {
        if (zs.avail_in || in_eof) return true;
        const long n = raw->read(in.data(), in.size());
        if (n < 0) {
            err = raw->err;
            return false;
        }
        if (n == 0) in_eof = true;
        zs.next_in = in.data();
        zs.avail_in = (uInt)n;
        return true;
    }
    long read(uint8_t* dst, size_t cap) override {
        if (!started) {
            if (inflateInit2(&zs, 15 + 16) != Z_OK) {
                err = "inflateInit2 failed";
                return -1;
            }
            started = true;
        }
        size_t got = 0;
        while (got < cap && !ended) {
            if (!refill()) return -1;
            if (zs.avail_in == 0 && in_eof) {
                err = "truncated gzip input";
                return -1;
            }
            const size_t want = std::min<size_t>(cap - got, 1u << 30);
            zs.next_out = dst + got;
            zs.avail_out = (uInt)want;
            const int ret = inflate(&zs, Z_NO_FLUSH);
            got += want - zs.avail_out;
            if (ret == Z_STREAM_END) {
                // another member may follow (skip zero padding some writers append)
                for (;;) {
                    if (!refill()) return -1;
                    while (zs.avail_in && *zs.next_in == 0) {
                        ++zs.next_in;
                        --zs.avail_in;
                    }
                    if (zs.avail_in || in_eof) break;
                }
                if (zs.avail_in == 0) {
                    ended = true;
                } else if (inflateReset(&zs) != Z_OK) {
                    err = "inflateReset failed";
                    return -1;
                }
            } else if (ret != Z_OK && ret != Z_BUF_ERROR) {
                err = std::string("gzip: ") + (zs.msg ? zs.msg : "corrupt input");
                return -1;
            }
        }
        return (long)got;
    }
};

// Any other gzip stream: parallel inflate (ParGzSource below), or zlib's sequential inflate
// with DMX_SEQ_INFLATE=1.
std::unique_ptr<Source> make_gz_source(std::unique_ptr<Source> raw, int threads, bool ahead);

// gzip members that state their own size — our writer's "DX" extra subfield (compressed and
// uncompressed member size) or BGZF's "BC" (bgzip, htslib) — are inflated in parallel, each
// straight into its place in the batch buffer, and checked against the member's CRC-32 and
// ISIZE.  A member without a size field hands the rest of the stream to the sequential
// GzSource.  (A plain single-member file, e.g. Python's gzip output, is always sequential.)
struct MemberGzSource : Source {
    std::unique_ptr<Source> raw;
    std::vector<uint8_t> cbuf;    // compressed bytes not yet consumed start at cpos
    size_t cpos = 0;
    bool raw_eof = false;
    int threads = 1;
    std::unique_ptr<Source> seq;  // sequential fallback
    std::vector<uint8_t> pending; // a member larger than the caller's buffer
    size_t ppos = 0;

    size_t chunk_hint() const override { return 1u << 30; }

    // Drop consumed bytes; only between gathers (gathered members hold offsets into cbuf).
    void compact() {
        if (cpos > (64u << 20) && cpos * 2 > cbuf.size()) {
            cbuf.erase(cbuf.begin(), cbuf.begin() + (ptrdiff_t)cpos);
            cpos = 0;
        }
    }

    bool fill(size_t need) {   // make cbuf hold >= need bytes from cpos (or reach EOF)
        while (!raw_eof && cbuf.size() - cpos < need) {
            const size_t old = cbuf.size();
            const size_t want = std::max<size_t>(need - (old - cpos), 16u << 20);
            cbuf.resize(old + want);
            const long n = raw->read(cbuf.data() + old, want);
            if (n < 0) {
                err = raw->err;
                return false;
            }
            cbuf.resize(old + (size_t)n);
            if (n == 0) raw_eof = true;
        }
        return true;
    }

    struct Member {
        size_t hdr, clen, data, dlen, usize, out;
        uint32_t crc;
    };

    // Parse the member header at cpos: 1 = sized member, 0 = unsized (fallback), -1 = error.
    int parse(Member& m) {
        if (!fill(64)) return -1;
        const size_t avail = cbuf.size() - cpos;
        const uint8_t* h = cbuf.data() + cpos;
        if (avail < 18 || h[0] != 0x1f || h[1] != 0x8b || h[2] != 8) return avail < 18 && avail ? -2 : 0;
        const uint8_t flg = h[3];
        if (!(flg & 4)) return 0;
        const size_t xlen = h[10] | (size_t)h[11] << 8;
        if (!fill(12 + xlen + 1024)) return -1;
        h = cbuf.data() + cpos;
        const size_t av2 = cbuf.size() - cpos;
        if (12 + xlen > av2) return -2;
        uint64_t csize = 0, usize = 0;
        bool have_u = false;
        for (size_t p = 12; p + 4 <= 12 + xlen;) {
            const size_t len = h[p + 2] | (size_t)h[p + 3] << 8;
            if (p + 4 + len > 12 + xlen) break;
            if (h[p] == 'D' && h[p + 1] == 'X' && len == 8) {
                csize = (uint32_t)(h[p + 4] | h[p + 5] << 8 | h[p + 6] << 16 | (uint32_t)h[p + 7] << 24);
                usize = (uint32_t)(h[p + 8] | h[p + 9] << 8 | h[p + 10] << 16 | (uint32_t)h[p + 11] << 24);
                have_u = true;
            } else if (h[p] == 'B' && h[p + 1] == 'C' && len == 2) {
                csize = (size_t)(h[p + 4] | h[p + 5] << 8) + 1;
            }
            p += 4 + len;
        }
        if (!csize) return 0;
        size_t q = 12 + xlen;
        if (flg & 8) {   // FNAME
            while (q < av2 && h[q]) ++q;
            ++q;
        }
        if (flg & 16) {  // FCOMMENT
            while (q < av2 && h[q]) ++q;
            ++q;
        }
        if (flg & 2) q += 2;   // FHCRC
        if (!fill(csize)) return -1;
        if (cbuf.size() - cpos < csize || q + 8 > csize) return -2;
        h = cbuf.data() + cpos;
        const uint8_t* t = h + csize - 8;
        m.crc = (uint32_t)(t[0] | t[1] << 8 | t[2] << 16 | (uint32_t)t[3] << 24);
        const uint32_t isize = (uint32_t)(t[4] | t[5] << 8 | t[6] << 16 | (uint32_t)t[7] << 24);
        if (have_u && (uint32_t)usize != isize) return -2;
        m.hdr = cpos;
        m.clen = csize;
        m.data = cpos + q;
        m.dlen = csize - q - 8;
        m.usize = isize;
        return 1;
    }

    // Whole-member inflate (the member's size is known) with libdeflate, one decompressor per
    // worker thread; checked against the member's ISIZE and CRC-32.
    static bool inflate_member(const uint8_t* src, size_t n, uint8_t* dst, size_t usize,
                               uint32_t crc) {
        struct Dec {
            libdeflate_decompressor* d = libdeflate_alloc_decompressor();
            ~Dec() {
                if (d) libdeflate_free_decompressor(d);
            }
        };
        thread_local Dec dec;
        if (!dec.d) return false;
        size_t got = 0;
        if (libdeflate_deflate_decompress(dec.d, src, n, dst, usize, &got) != 0 || got != usize)
            return false;
        return libdeflate_crc32(0u, dst, usize) == crc;
    }

    void switch_to_sequential() {
        auto pre = std::make_unique<PrefixSource>();
        pre->head.assign(cbuf.begin() + (ptrdiff_t)cpos, cbuf.end());
        pre->inner = std::move(raw);
        cbuf.clear();
        cpos = 0;
        seq = make_gz_source(std::move(pre), threads, false);
    }

    long read(uint8_t* dst, size_t cap) override {
        size_t got = 0;
        if (ppos < pending.size()) {
            got = std::min(cap, pending.size() - ppos);
            memcpy(dst, pending.data() + ppos, got);
            ppos += got;
            if (ppos == pending.size()) {
                pending.clear();
                ppos = 0;
            }
        }
        while (got < cap) {
            if (seq) {
                const long n = seq->read(dst + got, cap - got);
                if (n < 0) {
                    err = seq->err;
                    return -1;
                }
                return (long)(got + (size_t)n);
            }
            compact();
            std::vector<Member> ms;
            size_t plan = got;
            bool stop = false;
            while (ms.size() < 65536) {
                if (!fill(1)) return -1;
                while (cpos < cbuf.size() && cbuf[cpos] == 0) ++cpos;   // zero padding
                if (cpos == cbuf.size()) {
                    if (!fill(1)) return -1;
                    if (cpos == cbuf.size()) {
                        stop = true;   // end of input
                        break;
                    }
                    continue;
                }
                Member m;
                const int pr = parse(m);
                if (pr < 0) {
                    if (err.empty()) err = pr == -2 ? "truncated or corrupt gzip member" : "read error";
                    return -1;
                }
                if (pr == 0) {
                    if (ms.empty() && plan == got) switch_to_sequential();
                    stop = ms.empty();
                    break;
                }
                if (plan + m.usize > cap) {
                    if (ms.empty() && plan == got) {   // does not fit: stage it
                        pending.resize(m.usize);
                        if (!inflate_member(cbuf.data() + m.data, m.dlen, pending.data(), m.usize, m.crc)) {
                            err = "gzip member failed to inflate or CRC mismatch";
                            return -1;
                        }
                        cpos += m.clen;
                        const size_t k = std::min(cap - got, pending.size());
                        memcpy(dst + got, pending.data(), k);
                        ppos = k;
                        if (ppos == pending.size()) {
                            pending.clear();
                            ppos = 0;
                        }
                        got += k;
                    }
                    stop = true;
                    break;
                }
                m.out = plan;
                plan += m.usize;
                cpos += m.clen;
                ms.push_back(m);
            }
            if (!ms.empty()) {
                std::atomic<size_t> next{0};
                std::atomic<bool> bad{false};
                const int nt = (int)std::min<size_t>(threads, ms.size());
                parallel(nt, [&](int) {
                    for (size_t k; (k = next.fetch_add(1)) < ms.size();) {
                        const Member& m = ms[k];
                        if (!inflate_member(cbuf.data() + m.data, m.dlen, dst + m.out, m.usize, m.crc))
                            bad = true;
                    }
                });
                if (bad) {
                    err = "gzip member failed to inflate or CRC mismatch";
                    return -1;
                }
                got = plan;
            }
            if (stop || ms.empty()) {
                if (seq) continue;
                break;
            }
        }
        return (long)got;
    }
};

// Parallel inflate of gzip streams whose members do not state their size — an ordinary
// single-member file such as 02_cutadapt_loop.sh's input `pychopped_<ds>.gz` (:15,28-34,71) —
// on `threads` workers (dmx_inflate.h: speculative chunk decoding with a marker window, each
// speculative start checked against the previous chunk's actual end, markers resolved against
// the real window, CRC-32 / ISIZE of every member checked).  One round decodes up to `threads`
// chunks of `chunk` compressed bytes; its output goes straight into the caller's buffer when
// it fits.  DMX_INFLATE_CHUNK_KB sets the chunk size (tests use small chunks to put many chunk
// edges into small files); DMX_SEQ_INFLATE=1 selects the sequential zlib path instead.
struct ParGzSource : Source {
    std::unique_ptr<Source> raw;
    int threads = 1;
    size_t chunk = 4u << 20;           // compressed bytes per chunk
    size_t margin = 4u << 20;          // input held past the last chunk's nominal end
    size_t compact_at = 64u << 20;     // consumed input bytes dropped beyond this much
    std::vector<uint8_t> cbuf;         // compressed input; cn valid bytes, then >= 64 zero bytes
    size_t cn = 0;
    bool raw_eof = false;
    uint64_t pos = 0;                  // bit position in cbuf of the next decode
    bool at_member = true, done = false;
    std::vector<uint8_t> win;          // the last <= 32 KiB of output
    bool in_member = false;            // CRC-32 / size of the current member's output so far
    uint32_t mcrc = 0;
    uint64_t msize = 0;
    Bytes pend;                        // decoded output not yet delivered
    size_t ppos = 0;
    double ratio = 2.5;                // output / compressed bytes of the last round (FASTQ)

    struct Chunk {
        uint64_t nominal = 0, stop = 0, start = 0, end = 0;
        bool found = false, bytes = false, atm_in = false, atm_out = false;
        dmxi::Stop st = dmxi::Stop::kError;
        dmxi::Buf<uint8_t> b8;
        dmxi::Buf<uint16_t> b16, scratch;
        std::vector<dmxi::Event> ev;
        std::vector<uint8_t> w0;       // the real window before this chunk (resolve)
        uint64_t n = 0, out = 0;       // output elements, offset in the round's output
        std::vector<std::pair<uint64_t, uint32_t>> seg;   // (length, CRC-32) between events
    };
    std::vector<Chunk> ch;

    explicit ParGzSource(std::unique_ptr<Source> r, int nth) : raw(std::move(r)), threads(nth) {
        // with a memory budget: a round's working set (compressed input ~2x, 16-bit outputs of
        // ~3.5x the compressed bytes, the round's output) is about 12 x threads x chunk; keep
        // it near budget / 16
        if (const uint64_t b = g_mem_budget.load())
            chunk = std::min<size_t>(chunk, std::max<size_t>(256u << 10,
                                                             b / (192u * (uint64_t)std::max(1, nth))));
        if (const char* e = getenv("DMX_INFLATE_CHUNK_KB")) {
            const long kb = atol(e);
            if (kb > 0) chunk = (size_t)kb << 10;
        }
        margin = std::max<size_t>(g_mem_budget.load() ? std::min<size_t>(4u << 20, 4 * chunk)
                                                       : (4u << 20), chunk);
        if (const uint64_t b = g_mem_budget.load())
            compact_at = std::min<size_t>(compact_at, std::max<size_t>(4u << 20, b / 64));
    }
    size_t chunk_hint() const override { return 1u << 30; }

    bool fill(size_t need) {   // cbuf holds >= need bytes from pos / 8 (or all of the input)
        const size_t from = (size_t)(pos >> 3);
        if (from > compact_at && from * 2 > cn) {   // drop consumed input
            cbuf.erase(cbuf.begin(), cbuf.begin() + (ptrdiff_t)from);
            cn -= from;
            pos -= (uint64_t)from * 8;
        }
        const size_t at = (size_t)(pos >> 3);
        while (!raw_eof && cn - at < need) {
            const size_t want = std::max<size_t>(need - (cn - at), 16u << 20);
            cbuf.resize(cn + want + 64);
            const long n = raw->read(cbuf.data() + cn, want);
            if (n < 0) {
                err = raw->err;
                return false;
            }
            cn += (size_t)n;
            if (n == 0) raw_eof = true;
        }
        cbuf.resize(cn + 64);
        memset(cbuf.data() + cn, 0, 64);
        return true;
    }

    // Decode chunk c from `from` with the real window `w` into bytes.
    static dmxi::Stop decode_bytes(const dmxi::In& in, Chunk& c, uint64_t from, bool atm,
                                   const std::vector<uint8_t>& w) {
        // output estimate: ~3.5x the compressed bytes up to the stop (FASTQ), grown on demand
        const uint64_t lim = std::min<uint64_t>(c.stop, in.end_bits());
        c.b8.reserve(dmxi::kWin + (size_t)(lim > from ? (lim - from) / 8 * 7 / 2 : 0) + (1u << 16));
        memset(c.b8.p, 0, dmxi::kWin - w.size());
        if (!w.empty()) memcpy(c.b8.p + dmxi::kWin - w.size(), w.data(), w.size());
        c.b8.n = dmxi::kWin;
        c.ev.clear();
        c.start = from;
        c.end = from;
        c.atm_in = atm;
        c.atm_out = atm;
        c.bytes = true;
        c.w0 = w;
        c.st = dmxi::inflate_run<uint8_t>(in, c.end, c.atm_out, c.b8, dmxi::kWin - w.size(), c.stop,
                                          c.ev);
        c.n = c.b8.n - dmxi::kWin;
        return c.st;
    }

    // The last <= 32 KiB of (w followed by chunk c's resolved output).
    static bool tail_after(const std::vector<uint8_t>& w, const Chunk& c, std::vector<uint8_t>& t) {
        const size_t keep = (size_t)std::min<uint64_t>(c.n, dmxi::kWin);
        const size_t from_w = std::min<size_t>(w.size(), (size_t)dmxi::kWin - keep);
        // a member starting inside the chunk resets the history: the window is then the output
        // since that start, but the markers never reach before it, so keeping w is harmless
        t.assign(w.end() - (ptrdiff_t)from_w, w.end());
        const size_t o = t.size();
        t.resize(o + keep);
        if (c.bytes) {
            if (keep) memcpy(t.data() + o, c.b8.p + dmxi::kWin + (c.n - keep), keep);
            return true;
        }
        const uint16_t* s = c.b16.p + dmxi::kWin + (c.n - keep);
        const size_t wmiss = dmxi::kWin - w.size();   // markers below this index are undefined
        for (size_t i = 0; i < keep; ++i) {
            const uint16_t v = s[i];
            if (v < 256) {
                t[o + i] = (uint8_t)v;
            } else {
                const size_t wi = v - 256u;
                if (wi < wmiss) return false;
                t[o + i] = w[wi - wmiss];
            }
        }
        return true;
    }

    // One round; 1 = done (output appended), 0 = retry with more input, -1 = error.
    int round(uint8_t* dst, size_t cap, size_t& wrote) {
        const int nth = std::max(1, threads);
        // a round's output goes straight into the caller's buffer when it fits; otherwise it
        // waits in `pend` and reaches the caller by a serial copy (on the box: ~25 % of a
        // 16-thread round).  So the chunks are sized for the round to fit `cap` at the last
        // round's output ratio (down to chunk / 8).
        size_t chunk_r = chunk;
        if (nth > 1 && cap < ((size_t)1 << 40)) {
            const double fit = (double)cap / ((double)nth * ratio * 1.15);
            chunk_r = std::min(chunk, std::max<size_t>(std::max<size_t>(chunk / 8, 64u << 10),
                                                       (size_t)fit));
        }
        if (!fill((size_t)nth * chunk_r + margin)) return -1;
        const dmxi::In in{cbuf.data(), cn, raw_eof};
        const uint64_t p0 = pos;
        const size_t b0 = (size_t)(p0 >> 3);
        const size_t avail = cn - b0;
        // chunks of chunk_r bytes; at the end of the input the rest is split evenly (chunks of
        // at least chunk_r / 4) so the last round keeps the threads busy too
        size_t nch = 1, cs = chunk_r;
        if (nth > 1) {
            const size_t usable = raw_eof ? avail : (avail > margin ? avail - margin : 0);
            const size_t minc = std::max<size_t>(chunk_r / 4, 64u << 10);
            nch = std::max<size_t>(1, std::min<size_t>((size_t)nth, (usable + minc - 1) / minc));
            if (raw_eof) cs = std::max<size_t>(minc, (usable + nch - 1) / nch);
            nch = std::max<size_t>(1, std::min(nch, usable / std::max<size_t>(cs, 1) +
                                                        (raw_eof ? 1 : 0)));
        }
        if (ch.size() < nch) ch.resize(nch);
        for (size_t k = 0; k < nch; ++k) {
            Chunk& c = ch[k];
            c.nominal = k == 0 ? p0 : (uint64_t)(b0 + k * cs) * 8;
            const uint64_t e = (uint64_t)(b0 + (k + 1) * cs) * 8;
            c.stop = k + 1 < nch ? e : (raw_eof && e >= (uint64_t)cn * 8 ? UINT64_MAX : e);
            c.found = false;
            c.bytes = false;
        }
        const double t0 = kIoDebug ? now_s() : 0;
        std::vector<double> tfind(nch, 0.0), tdec(nch, 0.0);
        std::atomic<size_t> next{1};
        parallel((int)nch, [&](int t) {
            if (t == 0) {
                decode_bytes(in, ch[0], p0, at_member, win);
                ch[0].found = true;
            }
            for (size_t k; (k = next.fetch_add(1)) < nch;) {
                Chunk& c = ch[k];
                uint64_t s = 0;
                const double tf = kIoDebug ? now_s() : 0;
                const bool fnd = dmxi::find_block(in, c.nominal,
                                                  c.stop == UINT64_MAX ? in.end_bits() : c.stop, s,
                                                  c.scratch);
                if (kIoDebug) tfind[k] = now_s() - tf;
                if (!fnd) continue;
                c.found = true;
                c.start = s;
                c.end = s;
                c.atm_in = c.atm_out = false;
                c.ev.clear();
                const uint64_t lim = std::min<uint64_t>(c.stop, in.end_bits());
                c.b16.reserve(dmxi::kWin + (size_t)(lim > s ? (lim - s) / 8 * 7 / 2 : 0) + (1u << 16));
                for (int i = 0; i < dmxi::kWin; ++i) c.b16.p[i] = (uint16_t)(256 + i);
                c.b16.n = dmxi::kWin;
                c.st = dmxi::inflate_run<uint16_t>(in, c.end, c.atm_out, c.b16, 0, c.stop, c.ev);
                c.n = c.b16.n - dmxi::kWin;
                if (kIoDebug) tdec[k] = now_s() - tf - tfind[k];
            }
        });
        const double t1 = kIoDebug ? now_s() : 0;
        // stitch: accept a speculative chunk only where it starts at its predecessor's end,
        // else decode it again from there with the real window
        std::vector<uint8_t> w = win;
        uint64_t total = 0;
        for (size_t k = 0; k < nch; ++k) {
            Chunk& c = ch[k];
            if (k > 0) {
                const Chunk& p = ch[k - 1];
                if (p.st == dmxi::Stop::kEnd) {   // the stream ended before this chunk
                    nch = k;
                    break;
                }
                const bool ok = c.found && !c.bytes && c.start == p.end && !p.atm_out &&
                                (c.st == dmxi::Stop::kBoundary || c.st == dmxi::Stop::kEnd);
                if (!ok) decode_bytes(in, c, p.end, p.atm_out, w);
                else c.w0 = w;
            }
            if (c.st == dmxi::Stop::kNeedMore) {
                if (raw_eof) {
                    err = "truncated gzip input";
                    return -1;
                }
                margin *= 2;
                return 0;
            }
            if (c.st == dmxi::Stop::kError) {   // near the end of the input: truncation
                err = raw_eof && c.end + 512 >= in.end_bits() ? "truncated gzip input"
                                                              : "gzip: invalid compressed data";
                return -1;
            }
            std::vector<uint8_t> t;
            if (!tail_after(w, c, t)) {
                err = "gzip: invalid compressed data (distance too far back)";
                return -1;
            }
            w.swap(t);
            c.out = total;
            total += c.n;
        }
        // resolve / copy into the destination and CRC the pieces between member events
        const double t2 = kIoDebug ? now_s() : 0;
        uint8_t* out = dst;
        if (total > cap) {
            pend.resize(total);
            ppos = 0;
            out = pend.data();
        }
        std::atomic<bool> bad{false};
        std::atomic<size_t> nk{0};
        parallel((int)std::min<size_t>(nch, (size_t)nth), [&](int) {
            for (size_t k; (k = nk.fetch_add(1)) < nch;) {
                Chunk& c = ch[k];
                uint8_t* o = out + c.out;
                if (c.bytes) {
                    if (c.n) memcpy(o, c.b8.p + dmxi::kWin, c.n);
                } else {
                    const uint16_t* s = c.b16.p + dmxi::kWin;
                    const size_t wmiss = dmxi::kWin - c.w0.size();
                    const uint8_t* w0 = c.w0.data();
                    bool fail = false;
                    for (uint64_t i = 0; i < c.n; ++i) {
                        const uint32_t v = s[i];
                        if (v < 256) {
                            o[i] = (uint8_t)v;
                        } else if (v - 256u >= wmiss) {
                            o[i] = w0[v - 256u - wmiss];
                        } else {
                            fail = true;
                            o[i] = 0;
                        }
                    }
                    if (fail) bad = true;
                }
                c.seg.clear();
                uint64_t a = 0;
                for (const auto& e : c.ev) {
                    c.seg.emplace_back(e.out - a, libdeflate_crc32(0u, o + a, e.out - a));
                    a = e.out;
                }
                c.seg.emplace_back(c.n - a, libdeflate_crc32(0u, o + a, c.n - a));
            }
        });
        if (bad) {
            err = "gzip: invalid compressed data (distance too far back)";
            return -1;
        }
        for (size_t k = 0; k < nch; ++k) {
            const Chunk& c = ch[k];
            for (size_t s = 0; s < c.seg.size(); ++s) {
                const uint64_t len = c.seg[s].first;
                if (len) {
                    if (!in_member) {
                        err = "gzip: data outside a member";
                        return -1;
                    }
                    mcrc = (uint32_t)crc32_combine(mcrc, c.seg[s].second, (z_off_t)len);
                    msize += len;
                }
                if (s < c.ev.size()) {
                    const dmxi::Event& e = c.ev[s];
                    if (e.kind == 0) {
                        in_member = true;
                        mcrc = 0;
                        msize = 0;
                    } else {
                        if (!in_member || e.crc != mcrc || e.isize != (uint32_t)msize) {
                            err = "gzip: CRC-32 or length mismatch";
                            return -1;
                        }
                        in_member = false;
                    }
                }
            }
        }
        if (kIoDebug) {
            double mf = 0, md = 0;
            int redo = 0;
            for (size_t k = 0; k < nch; ++k) {
                mf = std::max(mf, tfind[k]);
                md = std::max(md, tdec[k]);
                redo += k > 0 && ch[k].bytes;
            }
            fprintf(stderr, "[pinflate] chunks %zu out %.1f MB: decode %.3f s (max find %.3f, "
                    "max dec %.3f), stitch %.3f s, resolve+crc %.3f s, redone %d\n", nch,
                    total / 1e6, t1 - t0, mf, md, t2 - t1, now_s() - t2, redo);
        }
        const Chunk& last = ch[nch - 1];
        if (last.end > p0 && total > 0)   // output / compressed ratio, for the next round's size
            ratio = std::max(1.0, (double)total / ((double)(last.end - p0) / 8.0));
        pos = last.end;
        at_member = last.atm_out;
        done = last.st == dmxi::Stop::kEnd;
        if (done && in_member) {
            err = "truncated gzip input";
            return -1;
        }
        win.swap(w);
        wrote = total > cap ? cap : (size_t)total;
        if (total > cap) {
            memcpy(dst, pend.data(), cap);
            ppos = cap;
        }
        return 1;
    }

    long read(uint8_t* dst, size_t cap) override {
        size_t got = 0;
        if (ppos < pend.size()) {
            got = std::min(cap, pend.size() - ppos);
            memcpy(dst, pend.data() + ppos, got);
            ppos += got;
            if (ppos == pend.size()) {
                pend.clear();
                ppos = 0;
            }
        }
        // one round per call (a partly filled buffer is a valid read): a second round into the
        // rest of the buffer would be cut small or spill into `pend`
        while (got == 0 && !done) {
            size_t w = 0;
            const int r = round(dst, cap, w);
            if (r < 0) return -1;
            got += w;
        }
        return (long)got;
    }
};

// Read-ahead: a thread of its own pulls blocks from the inner source (the parallel inflate's
// rounds) up to `depth` blocks ahead, so inflating the next text overlaps the reader's newline
// scan, parse and pack of the current batch (both fan out to the same work pool; before, the
// reader thread ran them strictly one after the other).  Consumed blocks go back to the thread
// (no re-faulting of 64 MB buffers).
struct AheadSource : Source {
    struct Blk {
        std::unique_ptr<uint8_t[]> p;   // blk bytes, uninitialised
        size_t n = 0;
    };
    std::unique_ptr<Source> in;
    size_t blk = 64u << 20;
    size_t depth = 2;
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Blk> full, spare;
    bool eof = false, failed = false, stop = false;
    Blk cur;
    size_t cpos = 0;

    int threads = 1;   // the copy into the caller's buffer

    explicit AheadSource(std::unique_ptr<Source> s, int nth) : in(std::move(s)), threads(nth) {
        if (const uint64_t b = g_mem_budget.load())   // two blocks in flight: <= budget / 16
            blk = std::min<size_t>(blk, std::max<size_t>(4u << 20, b / 32));
        if (const char* e = getenv("DMX_INFLATE_AHEAD_KB")) {   // tests: many small blocks
            const long kb = atol(e);
            if (kb > 0) blk = (size_t)kb << 10;
        }
        th = std::thread([this] { run(); });
    }
    ~AheadSource() override {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        th.join();   // a read in progress finishes first (bounded: one inflate round)
    }
    size_t chunk_hint() const override { return 1u << 30; }
    void run() {
        for (;;) {
            Blk b;
            {
                std::unique_lock<std::mutex> l(mu);
                cv.wait(l, [&] { return stop || full.size() < depth; });
                if (stop) return;
                if (!spare.empty()) {
                    b = std::move(spare.front());
                    spare.pop_front();
                }
            }
            long n = -1;
            std::string e;
            try {   // (an exception must not leave this thread: std::terminate)
                if (!b.p) b.p.reset(new uint8_t[blk]);
                n = in->read(b.p.get(), blk);
                if (n < 0) e = in->err;
            } catch (const std::bad_alloc&) {
                e = "out of memory (gzip read-ahead)";
            }
            std::lock_guard<std::mutex> g(mu);
            if (n < 0) {
                err = e;
                failed = true;
            } else if (n == 0) {
                eof = true;
            } else {
                b.n = (size_t)n;
                full.push_back(std::move(b));
            }
            cv.notify_all();
            if (n <= 0) return;
        }
    }
    long read(uint8_t* dst, size_t cap) override {
        size_t got = 0;
        while (got < cap) {
            if (cpos == cur.n) {
                std::unique_lock<std::mutex> l(mu);
                if (cur.p) spare.push_back(std::move(cur));
                cur = Blk();
                cpos = 0;
                cv.notify_all();
                cv.wait(l, [&] { return !full.empty() || eof || failed; });
                if (full.empty()) {
                    if (failed) return -1;
                    break;   // end of input
                }
                cur = std::move(full.front());
                full.pop_front();
                cv.notify_all();
            }
            const size_t k = std::min(cap - got, cur.n - cpos);
            // a round's ~60 MB: the copy into the batch runs on the pool (a serial copy was
            // ~7 ms of every 30 ms inflate round on the box)
            const int nc = (int)std::min<size_t>((size_t)threads, k >> 22);
            uint8_t* d = dst + got;
            const uint8_t* sp = cur.p.get() + cpos;
            if (nc > 1)
                parallel(nc, [&](int t) {
                    const size_t a = k * (size_t)t / (size_t)nc, b = k * (size_t)(t + 1) / (size_t)nc;
                    memcpy(d + a, sp + a, b - a);
                });
            else
                memcpy(d, sp, k);
            cpos += k;
            got += k;
        }
        return (long)got;
    }
};

// The reader's inflating sources run ahead on a thread of their own (DMX_INFLATE_AHEAD=0: A/B,
// inflate on the reader's thread).
std::unique_ptr<Source> read_ahead(std::unique_ptr<Source> p, int threads) {
    const char* a = getenv("DMX_INFLATE_AHEAD");
    if (threads > 1 && !(a && a[0] == '0'))
        return std::make_unique<AheadSource>(std::move(p), threads);
    return p;
}

std::unique_ptr<Source> make_gz_source(std::unique_ptr<Source> raw, int threads, bool ahead) {
    const char* e = getenv("DMX_SEQ_INFLATE");
    if (e && atoi(e)) return std::make_unique<GzSource>(std::move(raw));
    std::unique_ptr<Source> p = std::make_unique<ParGzSource>(std::move(raw), threads);
    return ahead ? read_ahead(std::move(p), threads) : std::move(p);
}

// A memory range as a source (dmx_io_inflate).
struct SpanSource : Source {
    const uint8_t* p = nullptr;
    size_t n = 0, at = 0;
    long read(uint8_t* dst, size_t cap) override {
        const size_t k = std::min(cap, n - at);
        memcpy(dst, p + at, k);
        at += k;
        return (long)k;
    }
};

// ------------------------------------------------------------------------------------------
// batches

// Process-wide cache of large buffers.  glibc serves allocations above 32 MiB by mmap and unmaps
// them on free, so every batch (and every CLI call of the resident server) faulted its ~256 MB
// of text and packed words in again, page by page, from the threads that fill them.  Batches
// hand their big buffers back here and the next batch takes them, pages still mapped.
template <class V>
struct BigPool {
    static constexpr size_t kMinBytes = 32u << 20;
    static constexpr size_t kKeep = 8;
    std::mutex mu;
    std::vector<V> keep;
    // v (empty) gets a pooled buffer of capacity >= n elements, if there is one
    void take(V& v, size_t n) {
        std::lock_guard<std::mutex> g(mu);
        int bi = -1;
        for (int i = 0; i < (int)keep.size(); ++i)
            if (keep[i].capacity() >= n && (bi < 0 || keep[i].capacity() < keep[bi].capacity()))
                bi = i;
        if (bi < 0) return;
        v.swap(keep[bi]);
        keep.erase(keep.begin() + bi);
        v.clear();
    }
    void give(V& v) {
        const size_t b = v.capacity() * sizeof(typename V::value_type);
        if (b < kMinBytes) return;
        const uint64_t budget = g_mem_budget.load();
        std::lock_guard<std::mutex> g(mu);
        size_t held = 0;
        for (const V& k : keep) held += k.capacity() * sizeof(typename V::value_type);
        if (keep.size() < kKeep && (!budget || held + b <= budget / 32)) {
            keep.emplace_back();
            keep.back().swap(v);
        }
    }
    // v grows to n elements (contents kept), from the pool when it has to reallocate
    void grow(V& v, size_t n) {
        if (v.capacity() >= n) return;
        V nv;
        take(nv, n);
        if (nv.capacity() < n) {
            v.reserve(n);
            return;
        }
        nv.assign(v.begin(), v.end());
        v.swap(nv);
        give(nv);
    }
};
BigPool<Bytes> g_bytes_pool;
BigPool<Words> g_words_pool;

struct Batch : dmx_batch {
    std::atomic<int> refs{1};
    Bytes text_v, seqtext_v;
    std::vector<uint64_t> head_v, seq_v, qual_v, offs_v;
    std::vector<uint32_t> lens_v;
    Words seq2b_v, nmask_v;
    ~Batch() {
        g_bytes_pool.give(text_v);
        g_bytes_pool.give(seqtext_v);
        g_words_pool.give(seq2b_v);
        g_words_pool.give(nmask_v);
    }
    void publish() {
        text = text_v.data();
        head = head_v.data();
        seqtext = fasta ? seqtext_v.data() : text_v.data();
        seq = seq_v.data();
        qual = fasta ? nullptr : qual_v.data();
        lens = lens_v.data();
        seq2b = seq2b_v.data();
        nmask = nmask_v.data();
        offsets = offs_v.data();
        n_words = seq2b_v.size();
    }
};

void release(Batch* b) {
    if (b && b->refs.fetch_sub(1) == 1) delete b;
}

// Newline positions of buf[0, n) in order, found by nth threads.
std::vector<uint64_t> newlines(const uint8_t* buf, size_t n, int nth) {
    nth = (int)std::min<size_t>(nth, std::max<size_t>(1, n >> 20));
    std::vector<std::vector<uint64_t>> part(nth);
    parallel(nth, [&](int t) {
        const size_t lo = n * t / nth, hi = n * (t + 1) / nth;
        auto& v = part[t];
        v.reserve((hi - lo) / 64 + 16);
        const uint8_t* p = buf + lo;
        const uint8_t* e = buf + hi;
        while (p < e) {
            const void* q = memchr(p, '\n', (size_t)(e - p));
            if (!q) break;
            v.push_back((uint64_t)((const uint8_t*)q - buf));
            p = (const uint8_t*)q + 1;
        }
    });
    size_t tot = 0;
    for (auto& v : part) tot += v.size();
    std::vector<uint64_t> out;
    out.reserve(tot);
    for (auto& v : part) out.insert(out.end(), v.begin(), v.end());
    return out;
}

inline uint64_t strip_cr(const uint8_t* buf, uint64_t s, uint64_t e) {
    return (e > s && buf[e - 1] == '\r') ? e - 1 : e;
}

size_t pack_words(uint64_t total_nt, size_t n_reads) {   // == dmx_pack_words (dmx_api.cpp)
    const uint64_t nt = 2 * kPad + total_nt + (uint64_t)dmx::kPackAlign * n_reads;
    return (size_t)((nt + 31) / 32 * 2 + 4);
}

// Lay out and pack b's sequences (seqtext spans) in the device layout.
void pack_batch(Batch* b, int nth) {
    const size_t n = b->n_reads;
    b->offs_v.resize(n);
    uint64_t g = kPad, total = 0;
    for (size_t r = 0; r < n; ++r) {
        b->offs_v[r] = g;
        g += ((uint64_t)b->lens_v[r] + dmx::kPackAlign - 1) / dmx::kPackAlign * dmx::kPackAlign;
        total += b->lens_v[r];
    }
    b->total_nt = total;
    const size_t words = pack_words(total, n);
    g_words_pool.grow(b->seq2b_v, words);
    g_words_pool.grow(b->nmask_v, words);
    b->seq2b_v.resize(words);
    b->nmask_v.resize(words);
    // zero the head pad and everything after the last read (reads tile [kPad, g) exactly)
    std::fill(b->seq2b_v.begin(), b->seq2b_v.begin() + kPad / 16, 0u);
    std::fill(b->nmask_v.begin(), b->nmask_v.begin() + kPad / 32, 0u);
    std::fill(b->seq2b_v.begin() + std::min<size_t>(words, g / 16), b->seq2b_v.end(), 0u);
    std::fill(b->nmask_v.begin() + std::min<size_t>(words, g / 32), b->nmask_v.end(), 0u);
    const uint8_t* st = b->fasta ? b->seqtext_v.data() : b->text_v.data();
    nth = (int)std::min<size_t>(nth, std::max<size_t>(1, n / 2048));
    parallel(nth, [&](int t) {
        const size_t lo = n * t / nth, hi = n * (t + 1) / nth;
        for (size_t r = lo; r < hi; ++r)
            dmx::pack_one(st + b->seq_v[2 * r], b->lens_v[r], b->offs_v[r], b->seq2b_v.data(),
                          b->nmask_v.data());
    });
}

// FASTQ records of text[0, cut) whose line ends are nl[0, 4n).
bool parse_fastq(Batch* b, const std::vector<uint64_t>& nl, size_t n, int nth, std::string& err) {
    const uint8_t* buf = b->text_v.data();
    b->head_v.resize(2 * n);
    b->seq_v.resize(2 * n);
    b->qual_v.resize(2 * n);
    b->lens_v.resize(n);
    std::atomic<int64_t> bad{-1};
    std::atomic<int> why{0};
    const int nt = (int)std::min<size_t>(nth, std::max<size_t>(1, n / 4096));
    parallel(nt, [&](int t) {
        const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
        for (size_t r = lo; r < hi; ++r) {
            uint64_t s[4], e[4];
            for (int k = 0; k < 4; ++k) {
                const size_t li = 4 * r + k;
                s[k] = li ? nl[li - 1] + 1 : 0;
                e[k] = strip_cr(buf, s[k], nl[li]);
            }
            int w = 0;
            if (e[0] == s[0] || buf[s[0]] != '@') w = 1;
            else if (e[2] == s[2] || buf[s[2]] != '+') w = 2;
            else if (e[1] - s[1] != e[3] - s[3]) w = 3;
            if (w) {
                int64_t cur = bad.load();
                while ((cur < 0 || (int64_t)r < cur) && !bad.compare_exchange_weak(cur, (int64_t)r)) {}
                if (bad.load() == (int64_t)r) why = w;
                continue;
            }
            b->head_v[2 * r] = s[0] + 1;
            b->head_v[2 * r + 1] = e[0];
            b->seq_v[2 * r] = s[1];
            b->seq_v[2 * r + 1] = e[1];
            b->qual_v[2 * r] = s[3];
            b->qual_v[2 * r + 1] = e[3];
            b->lens_v[r] = (uint32_t)(e[1] - s[1]);
        }
    });
    if (bad.load() >= 0) {
        static const char* msg[] = {"", "FASTQ record does not start with '@'",
                                    "FASTQ record third line does not start with '+'",
                                    "FASTQ sequence and quality lengths differ"};
        err = std::string(msg[why.load()]) + " (record " + std::to_string(bad.load() + 1) +
              " of the batch)";
        return false;
    }
    return true;
}

inline bool is_space(uint8_t c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

// FASTA records of text[0, cut): starts[] are the '>' positions, nl[] the newlines.
bool parse_fasta(Batch* b, const std::vector<uint64_t>& starts, const std::vector<uint64_t>& nl,
                 uint64_t cut, int nth, std::string& err) {
    const uint8_t* buf = b->text_v.data();
    const size_t n = starts.size();
    b->head_v.resize(2 * n);
    b->seq_v.resize(2 * n);
    b->lens_v.resize(n);
    std::vector<uint64_t> slen(n);
    const int nt = (int)std::min<size_t>(nth, std::max<size_t>(1, n / 1024));
    // pass 1: header span and sequence length of each record
    parallel(nt, [&](int t) {
        const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
        for (size_t r = lo; r < hi; ++r) {
            const uint64_t s = starts[r];
            const uint64_t end = r + 1 < n ? starts[r + 1] : cut;
            auto it = std::lower_bound(nl.begin(), nl.end(), s);
            const uint64_t he = (it != nl.end() && *it < end) ? *it : end;
            b->head_v[2 * r] = s + 1;
            b->head_v[2 * r + 1] = strip_cr(buf, s + 1, he);
            uint64_t L = 0, p = he + 1;
            while (p < end) {
                const uint8_t* q = (const uint8_t*)memchr(buf + p, '\n', (size_t)(end - p));
                uint64_t le = q ? (uint64_t)(q - buf) : end;
                uint64_t ls = p, lz = le;
                while (ls < lz && is_space(buf[ls])) ++ls;
                while (lz > ls && is_space(buf[lz - 1])) --lz;
                L += lz - ls;
                p = le + 1;
            }
            slen[r] = L;
        }
    });
    uint64_t tot = 0;
    for (size_t r = 0; r < n; ++r) {
        b->seq_v[2 * r] = tot;
        tot += slen[r];
        b->seq_v[2 * r + 1] = tot;
        if (slen[r] >= (1ull << 31)) {
            err = "FASTA record longer than 2^31 nt";
            return false;
        }
        b->lens_v[r] = (uint32_t)slen[r];
    }
    b->seqtext_v.resize(tot + 1);
    // pass 2: join the sequence lines
    parallel(nt, [&](int t) {
        const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
        for (size_t r = lo; r < hi; ++r) {
            const uint64_t end = r + 1 < n ? starts[r + 1] : cut;
            uint64_t p = b->head_v[2 * r + 1];
            while (p < end && buf[p] != '\n') ++p;
            ++p;
            uint8_t* dst = b->seqtext_v.data() + b->seq_v[2 * r];
            while (p < end) {
                const uint8_t* q = (const uint8_t*)memchr(buf + p, '\n', (size_t)(end - p));
                uint64_t le = q ? (uint64_t)(q - buf) : end;
                uint64_t ls = p, lz = le;
                while (ls < lz && is_space(buf[ls])) ++ls;
                while (lz > ls && is_space(buf[lz - 1])) --lz;
                memcpy(dst, buf + ls, lz - ls);
                dst += lz - ls;
                p = le + 1;
            }
        }
    });
    return true;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// reader

struct dmx_reader {
    std::unique_ptr<Source> src;
    size_t batch_bytes = 256u << 20;
    int threads = 1;
    int format = 0;   // 1 FASTQ, 2 FASTA
    bool in_memory = false;   // the text comes from a retained sink output (no file read)
    Bytes carry;
    bool src_eof = false;

    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<Batch*> q;
    bool done = false, stop = false;
    std::string err;          // producer error (reported in order, after queued batches)
    std::string api_err;

    void produce();
    bool next_batch(Batch** out, std::string& e);
};

bool dmx_reader::next_batch(Batch** out, std::string& e) {
    *out = nullptr;
    Bytes buf;
    buf.swap(carry);
    size_t target = std::max<size_t>(batch_bytes, buf.size() + (1u << 20));
    double t0 = kIoDebug ? now_s() : 0, t1 = 0, t2 = 0;
    for (;;) {
        // fill
        g_bytes_pool.grow(buf, target + 64);
        while (!src_eof && buf.size() < target) {
            const size_t old = buf.size();
            const size_t want = std::min<size_t>(target - old, src->chunk_hint());
            buf.resize(old + want);
            const long n = src->read(buf.data() + old, want);
            if (n < 0) {
                e = src->err;
                return false;
            }
            buf.resize(old + (size_t)n);
            if (n == 0) src_eof = true;
        }
        if (!format) {
            size_t p = 0;
            while (p < buf.size() && (buf[p] == '\n' || buf[p] == '\r' || is_space(buf[p]))) ++p;
            if (p == buf.size()) {
                if (src_eof) return true;   // empty input
                buf.clear();
                continue;
            }
            if (buf[p] == '@') format = 1;
            else if (buf[p] == '>') format = 2;
            else {
                e = "input is neither FASTQ ('@') nor FASTA ('>')";
                return false;
            }
            if (p) buf.erase(buf.begin(), buf.begin() + p);
        }
        if (buf.empty()) return true;
        if (kIoDebug) t1 = now_s();
        std::vector<uint64_t> nl = newlines(buf.data(), buf.size(), threads);
        if (src_eof && buf.back() != '\n') {   // last line without a newline
            buf.push_back('\n');
            nl.push_back(buf.size() - 1);
        }
        auto* b = new Batch();
        b->fasta = format == 2;
        uint64_t cut = 0;
        if (format == 1) {
            size_t nrec = nl.size() / 4;
            if (src_eof && nl.size() % 4) {
                // tolerate trailing blank lines only
                const uint64_t s = nrec ? nl[4 * nrec - 1] + 1 : 0;
                for (uint64_t p = s; p < buf.size(); ++p)
                    if (!(buf[p] == '\n' || buf[p] == '\r' || is_space(buf[p]))) {
                        delete b;
                        e = "truncated FASTQ input (record with fewer than 4 lines)";
                        return false;
                    }
            }
            if (nrec == 0 && !src_eof) {
                delete b;
                target = buf.size() * 2;
                continue;
            }
            cut = nrec ? nl[4 * nrec - 1] + 1 : buf.size();
            if (src_eof && nl.size() % 4) cut = buf.size();
            b->n_reads = nrec;
            carry.assign(buf.begin() + (ptrdiff_t)cut, buf.end());
            buf.resize(cut);
            b->text_v.swap(buf);
            if (!parse_fastq(b, nl, nrec, threads, e)) {
                delete b;
                return false;
            }
        } else {
            // record starts: '>' at the start of the buffer or after a newline
            std::vector<uint64_t> starts;
            if (buf[0] == '>') starts.push_back(0);
            for (uint64_t p : nl)
                if (p + 1 < buf.size() && buf[p + 1] == '>') starts.push_back(p + 1);
            if (starts.empty() || starts[0] != 0) {
                delete b;
                e = "FASTA sequence before the first '>'";
                return false;
            }
            if (!src_eof && starts.size() < 2) {
                delete b;
                target = buf.size() * 2;
                continue;
            }
            if (src_eof) {
                cut = buf.size();
            } else {
                cut = starts.back();
                starts.pop_back();
            }
            b->n_reads = starts.size();
            carry.assign(buf.begin() + (ptrdiff_t)cut, buf.end());
            buf.resize(cut);
            b->text_v.swap(buf);
            nl.erase(std::lower_bound(nl.begin(), nl.end(), cut), nl.end());
            if (!parse_fasta(b, starts, nl, cut, threads, e)) {
                delete b;
                return false;
            }
        }
        if (b->n_reads == 0 && src_eof && carry.empty()) {
            delete b;
            return true;
        }
        if (kIoDebug) t2 = now_s();
        pack_batch(b, threads);
        b->publish();
        if (kIoDebug)
            fprintf(stderr, "dmx_io batch: %zu reads, %.1f MB text: fill %.3f s, parse %.3f s, pack %.3f s\n",
                    b->n_reads, b->text_v.size() / 1e6, t1 - t0, t2 - t1, now_s() - t2);
        *out = b;
        return true;
    }
}

void dmx_reader::produce() {
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || q.size() < 2; });
            if (stop) return;
        }
        Batch* b = nullptr;
        std::string e;
        const bool ok = next_batch(&b, e);
        std::lock_guard<std::mutex> lk(mu);
        if (!ok) {
            err = e.empty() ? "read error" : e;
            done = true;
        } else if (!b) {
            done = true;
        } else {
            q.push_back(b);
        }
        cv.notify_all();
        if (done) return;
    }
}

extern "C" {

int dmx_io_abi_version(void) { return DMX_IO_ABI_VERSION; }

uint64_t dmx_io_set_memory_budget(uint64_t bytes) { return g_mem_budget.exchange(bytes); }

int dmx_reader_open(const char* path, size_t batch_bytes, int threads, dmx_reader** out) {
    if (!path || !out) return -1;
    *out = nullptr;
    if (strcmp(path, "-")) {   // a file this process wrote with dmx_sink_retain, unchanged
        Retained ret;
        if (take_retained(path, ret)) {
            auto* r = new dmx_reader();
            auto m = std::make_unique<MemSource>();
            m->pieces = std::move(ret.pieces);
            m->threads = clamp_threads(threads);
            r->src = std::move(m);
            r->in_memory = true;
            r->batch_bytes = std::max<size_t>(batch_bytes, 1u << 16);
            r->threads = clamp_threads(threads);
            r->th = std::thread([r] { r->produce(); });
            *out = r;
            return 0;
        }
    }
    auto fd = std::make_unique<FdSource>();
    fd->threads = clamp_threads(threads);
    if (!strcmp(path, "-")) {
        fd->fd = 0;
    } else {
        fd->fd = ::open(path, O_RDONLY);
        fd->own = true;
        if (fd->fd < 0) return -2;
    }
    // sniff gzip magic and, for gzip, whether members carry their size (DX / BGZF BC)
    auto pre = std::make_unique<PrefixSource>();
    pre->head.resize(16);
    const long n = fd->read(pre->head.data(), 16);
    if (n < 0) return -2;
    pre->head.resize((size_t)n);
    const bool gz = n >= 2 && pre->head[0] == 0x1f && pre->head[1] == 0x8b;
    const bool sized = gz && n >= 16 && (pre->head[3] & 4) &&
                       ((pre->head[12] == 'D' && pre->head[13] == 'X') ||
                        (pre->head[12] == 'B' && pre->head[13] == 'C'));
    pre->inner = std::move(fd);
    auto* r = new dmx_reader();
    if (sized) {
        auto m = std::make_unique<MemberGzSource>();
        m->raw = std::move(pre);
        m->threads = clamp_threads(threads);
        r->src = read_ahead(std::move(m), clamp_threads(threads));
    } else if (gz) {
        r->src = make_gz_source(std::move(pre), clamp_threads(threads), true);
    } else {
        r->src = std::move(pre);
    }
    r->batch_bytes = std::max<size_t>(batch_bytes, 1u << 16);
    r->threads = clamp_threads(threads);
    r->th = std::thread([r] { r->produce(); });
    *out = r;
    return 0;
}

int dmx_reader_next(dmx_reader* r, dmx_batch** out) {
    if (!r || !out) return -1;
    *out = nullptr;
    std::unique_lock<std::mutex> lk(r->mu);
    r->cv.wait(lk, [&] { return !r->q.empty() || r->done; });
    if (!r->q.empty()) {
        *out = r->q.front();
        r->q.pop_front();
        r->cv.notify_all();
        return 0;
    }
    if (!r->err.empty()) {
        r->api_err = r->err;
        return -3;
    }
    return 0;
}

const char* dmx_reader_error(dmx_reader* r) { return r ? r->api_err.c_str() : "null reader"; }

int dmx_reader_in_memory(const dmx_reader* r) { return r && r->in_memory ? 1 : 0; }

int dmx_io_inflate(const uint8_t* src, size_t n, int threads, uint8_t* out, size_t cap,
                   size_t* out_len) {
    if ((!src && n) || (!out && cap) || !out_len) return -1;
    auto sp = std::make_unique<SpanSource>();
    sp->p = src;
    sp->n = n;
    auto gz = make_gz_source(std::move(sp), clamp_threads(threads), false);
    size_t got = 0;
    for (;;) {
        const long k = gz->read(out + got, cap - got);
        if (k < 0) return -2;
        got += (size_t)k;
        if (k == 0) break;
        if (got == cap) {   // full: is there more?
            uint8_t extra;
            const long m = gz->read(&extra, 1);
            if (m < 0) return -2;
            if (m > 0) return -3;
            break;
        }
    }
    *out_len = got;
    return 0;
}

void dmx_reader_close(dmx_reader* r) {
    if (!r) return;
    {
        std::lock_guard<std::mutex> lk(r->mu);
        r->stop = true;
        r->cv.notify_all();
    }
    if (r->th.joinable()) r->th.join();
    for (Batch* b : r->q) release(b);
    delete r;
}

void dmx_batch_free(dmx_batch* b) { release(static_cast<Batch*>(b)); }

}  // extern "C"

// ------------------------------------------------------------------------------------------
// sink

namespace {

struct Comp {
    uint8_t t[256];
    Comp() {
        for (int i = 0; i < 256; ++i) t[i] = (uint8_t)i;
        const char* a = "ACGTUMRWSYKVHDBNacgtumrwsykvhdbn";
        const char* b = "TGCAAKYWSRMBDHVNtgcaakywsrmbdhvn";
        for (int i = 0; a[i]; ++i) t[(uint8_t)a[i]] = (uint8_t)b[i];
    }
};
const Comp kComp;

struct Out {
    std::string path;
    FILE* fp = nullptr;
    bool gz = false;
    bool any = false;
    uint64_t n = 0, bp = 0;
    std::vector<Bytes> kept;    // dmx_sink_retain: the rendered text, in output order
    uint64_t kept_bytes = 0;
    bool keep = false;          // still retaining (dropped when the cap would be exceeded)
};

struct Job {
    Batch* b = nullptr;
    std::vector<int32_t> idx, start, stop;
    std::vector<uint8_t> rc, nrc;
    // row mode (dmx_sink_write_rows): row r renders read rread[r]; start/stop are positions on
    // the read as given (reverse-complemented after cutting when rc); mode 1 names the record
    // "{start}:{stop}|{id} strand=+|-{comment}"
    bool rows = false;
    std::vector<uint32_t> rread;
    std::vector<uint8_t> mode;
    // mode 2 (dmx_sink_write_rows2): the name is the segment's "{ns}:{ne}|{id} strand=..." of
    // (nstart, nstop, nstrand) followed by nrc " rc" suffixes; start/stop/rc give the sequence
    std::vector<int32_t> nstart, nstop;
    std::vector<uint8_t> nstrand;
};

inline uint32_t ndigits(uint32_t v) {
    uint32_t d = 1;
    while (v >= 10) {
        v /= 10;
        ++d;
    }
    return d;
}

inline uint8_t* put_u32(uint8_t* p, uint32_t v) {
    uint8_t tmp[10];
    int n = 0;
    do {
        tmp[n++] = (uint8_t)('0' + v % 10);
        v /= 10;
    } while (v);
    while (n) *p++ = tmp[--n];
    return p;
}

constexpr size_t kMemberMax = 1u << 20;   // uncompressed bytes per gzip member

inline void put32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

// One gzip member (RFC 1952) whose header carries a "DX" extra subfield with the member's
// compressed and uncompressed size, so that our reader (and any reader that skips unknown
// subfields, i.e. all of them) can find member boundaries and inflate members in parallel.
// Level 1 (`-Z`) is Huffman-only deflate: on FASTQ (2-bit-entropy bases, skewed qualities)
// zlib's level-1 LZ77 finds little and costs most of the time — zlib's Huffman-only strategy
// measured 2.6x faster and 4 % smaller here, and the table-driven encoder of dmx_deflate.h is
// several times faster again (same kind of stream).  Appends to `out`.
// Levels 2..9 use the record-aware encoder of dmx_deflate.h (fq_deflate: LZ77 in header lines
// only, sequence lines and the rest in blocks with codes of their own): on FASTQ its members
// are smaller than zlib's and libdeflate's at any level, at several times libdeflate -5's speed
// (profiles/r5_gzip_levels.json), so every level above 1 gets it.  DMX_GZIP_LIBDEFLATE=1 selects
// libdeflate at the requested level instead.  Level 0: stored blocks (libdeflate).
const bool kLibdeflateLevels = [] {
    const char* e = getenv("DMX_GZIP_LIBDEFLATE");
    return e && *e && strcmp(e, "0") != 0;
}();

bool gzip_member(const uint8_t* src, size_t n, int level, Bytes& out) {
    if (level == 1 || (level >= 2 && !kLibdeflateLevels)) {
        const size_t base = out.size();
        const size_t hdr = 24;
        out.resize(base + hdr + dmxz::huff_bound(n) + 16);
        uint8_t* h = out.data() + base;
        const uint8_t fixed[12] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, (uint8_t)(level == 1 ? 4 : level >= 9 ? 2 : 0), 3, 12, 0};
        memcpy(h, fixed, 12);
        h[12] = 'D';
        h[13] = 'X';
        h[14] = 8;
        h[15] = 0;
        const size_t clen = level == 1 ? dmxz::huff_deflate(src, n, h + hdr)
                                       : dmxz::fq_deflate(src, n, h + hdr);
        const size_t total = hdr + clen + 8;
        put32(h + 16, (uint32_t)total);
        put32(h + 20, (uint32_t)n);
        put32(h + hdr + clen, libdeflate_crc32(0u, src, n));
        put32(h + hdr + clen + 4, (uint32_t)n);
        out.resize(base + total);
        return true;
    }
    // other levels: libdeflate's compressor at the same level (one per thread and level);
    // its output at a zlib level is about zlib's size at that level, at several times zlib's
    // speed.  cutadapt's default is level 5 (dmx/cli.py --compression-level).
    struct Comp {
        libdeflate_compressor* c[13] = {nullptr};
        ~Comp() {
            for (auto* x : c)
                if (x) libdeflate_free_compressor(x);
        }
    };
    thread_local Comp comp;
    if (level < 0 || level > 12) return false;
    if (!comp.c[level]) comp.c[level] = libdeflate_alloc_compressor(level);
    libdeflate_compressor* lc = comp.c[level];
    if (!lc) return false;
    const size_t base = out.size();
    const size_t hdr = 24;
    const size_t bound = libdeflate_deflate_compress_bound(lc, n);
    out.resize(base + hdr + bound + 16);
    uint8_t* h = out.data() + base;
    const uint8_t fixed[12] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, (uint8_t)(level >= 9 ? 2 : 0), 3, 12, 0};
    memcpy(h, fixed, 12);
    h[12] = 'D';
    h[13] = 'X';
    h[14] = 8;
    h[15] = 0;
    const size_t clen = libdeflate_deflate_compress(lc, src, n, h + hdr, bound);
    if (clen == 0) return false;
    const size_t total = hdr + clen + 8;
    put32(h + 16, (uint32_t)total);
    put32(h + 20, (uint32_t)n);
    put32(h + hdr + clen, libdeflate_crc32(0u, src, n));
    put32(h + hdr + clen + 4, (uint32_t)n);
    out.resize(base + total);
    return true;
}

}  // namespace

extern "C" int dmx_io_gzip(const uint8_t* src, size_t n, int level, uint8_t* out, size_t cap,
                           size_t* out_len) {
    if ((!src && n) || !out || !out_len || level < 0 || level > 9) return -1;
    Bytes m;
    if (!gzip_member(src, n, level, m)) return -1;
    if (m.size() > cap) return -2;
    memcpy(out, m.data(), m.size());
    *out_len = m.size();
    return 0;
}

struct dmx_sink {
    std::vector<Out> outs;
    uint64_t retain_cap = 0;    // process-wide retained-bytes cap (0: no retention)
    bool fasta_out = false;
    int level = 1;
    int threads = 1;
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::unique_ptr<Job> pending;
    bool busy = false, stop = false, closed = false;
    std::string err, api_err;

    void worker();
    bool process(Job& j, std::string& e);
};

bool dmx_sink::process(Job& j, std::string& e) {
    Batch* b = j.b;
    const size_t n = j.rows ? j.rread.size() : b->n_reads;
    const int nout = (int)outs.size();
    const int nth = (int)std::min<size_t>(threads, std::max<size_t>(1, n / 1024));
    const bool fq = !fasta_out && !b->fasta;
    // pass 1: bytes per (thread, output)
    std::vector<std::vector<uint64_t>> sz(nth, std::vector<uint64_t>(nout, 0));
    std::vector<std::vector<uint64_t>> cnt(nth, std::vector<uint64_t>(nout, 0));
    std::vector<std::vector<uint64_t>> bps(nth, std::vector<uint64_t>(nout, 0));
    std::atomic<bool> range_bad{false};
    parallel(nth, [&](int t) {
        const size_t lo = n * t / nth, hi = n * (t + 1) / nth;
        for (size_t r = lo; r < hi; ++r) {
            const int o = j.idx[r];
            if (o < 0) continue;
            const size_t ri = j.rows ? j.rread[r] : r;
            if (o >= nout || ri >= b->n_reads || j.start[r] < 0 || j.stop[r] < j.start[r] ||
                (uint32_t)j.stop[r] > b->lens_v[ri]) {
                range_bad = true;
                continue;
            }
            const uint64_t L = (uint64_t)(j.stop[r] - j.start[r]);
            const uint64_t hl = b->head_v[2 * ri + 1] - b->head_v[2 * ri];
            if (j.rows && j.mode[r] == 2 &&
                (j.nstart[r] < 0 || j.nstop[r] < j.nstart[r] ||
                 (uint32_t)j.nstop[r] > b->lens_v[ri])) {
                range_bad = true;
                continue;
            }
            const uint64_t h = (j.rows && j.mode[r] == 1)
                                   ? hl + ndigits((uint32_t)j.start[r]) +
                                         ndigits((uint32_t)j.stop[r]) + 2 + 9
                               : (j.rows && j.mode[r] == 2)
                                   ? hl + ndigits((uint32_t)j.nstart[r]) +
                                         ndigits((uint32_t)j.nstop[r]) + 2 + 9 + 3ull * j.nrc[r]
                                   : hl + 3ull * j.nrc[r];
            sz[t][o] += 1 + h + 1 + L + 1 + (fq ? 2 + L + 1 : 0);
            cnt[t][o] += 1;
            bps[t][o] += L;
        }
    });
    if (range_bad) {
        e = "dmx_sink_write: output index or trim coordinates out of range";
        return false;
    }
    std::vector<std::vector<Bytes>> buf(nth, std::vector<Bytes>(nout));
    // pass 2: render
    parallel(nth, [&](int t) {
        std::vector<uint8_t*> w(nout, nullptr);
        for (int o = 0; o < nout; ++o) {
            buf[t][o].resize(sz[t][o]);
            w[o] = buf[t][o].data();
        }
        const size_t lo = n * t / nth, hi = n * (t + 1) / nth;
        const uint8_t* tx = b->text_v.data();
        const uint8_t* st = b->fasta ? b->seqtext_v.data() : tx;
        for (size_t r = lo; r < hi; ++r) {
            const int o = j.idx[r];
            if (o < 0) continue;
            const size_t ri = j.rows ? j.rread[r] : r;
            uint8_t* p = w[o];
            *p++ = fq ? '@' : '>';
            const uint64_t hs = b->head_v[2 * ri], he = b->head_v[2 * ri + 1];
            if (j.rows && j.mode[r] >= 1) {   // segment of a read: "start:stop|id strand=+ ..."
                const bool m2 = j.mode[r] == 2;
                p = put_u32(p, (uint32_t)(m2 ? j.nstart[r] : j.start[r]));
                *p++ = ':';
                p = put_u32(p, (uint32_t)(m2 ? j.nstop[r] : j.stop[r]));
                *p++ = '|';
                uint64_t cut = hs;
                while (cut < he && tx[cut] != ' ' && tx[cut] != '\t') ++cut;
                memcpy(p, tx + hs, cut - hs);
                p += cut - hs;
                memcpy(p, (m2 ? j.nstrand[r] : j.rc[r]) ? " strand=-" : " strand=+", 9);
                p += 9;
                memcpy(p, tx + cut, he - cut);
                p += he - cut;
                if (m2)
                    for (int k = 0; k < j.nrc[r]; ++k) {
                        memcpy(p, " rc", 3);
                        p += 3;
                    }
            } else {
                memcpy(p, tx + hs, he - hs);
                p += he - hs;
                for (int k = 0; k < j.nrc[r]; ++k) {
                    memcpy(p, " rc", 3);
                    p += 3;
                }
            }
            *p++ = '\n';
            const uint32_t len = b->lens_v[ri];
            uint32_t a = (uint32_t)j.start[r], z = (uint32_t)j.stop[r];
            if (j.rows && j.rc[r]) {   // row coordinates are on the read as given
                a = len - (uint32_t)j.stop[r];
                z = len - (uint32_t)j.start[r];
            }
            const uint8_t* s = st + b->seq_v[2 * ri];
            if (!j.rc[r]) {
                memcpy(p, s + a, z - a);
                p += z - a;
            } else {   // orient = reverse complement: out[k] = comp(s[len-1-k])
                for (uint32_t k = a; k < z; ++k) *p++ = kComp.t[s[len - 1 - k]];
            }
            *p++ = '\n';
            if (fq) {
                *p++ = '+';
                *p++ = '\n';
                const uint8_t* q = tx + b->qual_v[2 * ri];
                if (!j.rc[r]) {
                    memcpy(p, q + a, z - a);
                    p += z - a;
                } else {
                    for (uint32_t k = a; k < z; ++k) *p++ = q[len - 1 - k];
                }
                *p++ = '\n';
            }
            w[o] = p;
        }
    });
    // pass 3: compress (independent gzip members of <= kMemberMax bytes), largest first
    bool any_gz = false;
    for (auto& o : outs) any_gz |= o.gz;
    std::vector<std::vector<std::vector<Bytes>>> part;   // [thread][output] -> members
    if (any_gz) {
        struct Piece {
            int t, o;
            size_t lo, hi, k;
        };
        std::vector<Piece> jobs;
        part.assign(nth, std::vector<std::vector<Bytes>>(nout));
        for (int t = 0; t < nth; ++t)
            for (int o = 0; o < nout; ++o) {
                if (!outs[o].gz || buf[t][o].empty()) continue;
                const size_t sz = buf[t][o].size();
                const size_t np = (sz + kMemberMax - 1) / kMemberMax;
                part[t][o].resize(np);
                for (size_t k = 0; k < np; ++k)
                    jobs.push_back({t, o, sz * k / np, sz * (k + 1) / np, k});
            }
        std::sort(jobs.begin(), jobs.end(),
                  [](const Piece& x, const Piece& y) { return x.hi - x.lo > y.hi - y.lo; });
        std::atomic<size_t> next{0};
        std::atomic<bool> bad{false};
        const int nc = (int)std::min<size_t>(threads, std::max<size_t>(1, jobs.size()));
        parallel(nc, [&](int) {
            for (size_t k; (k = next.fetch_add(1)) < jobs.size();) {
                const Piece& pc = jobs[k];
                if (!gzip_member(buf[pc.t][pc.o].data() + pc.lo, pc.hi - pc.lo, level,
                                 part[pc.t][pc.o][pc.k]))
                    bad = true;
            }
        });
        if (bad) {
            e = "gzip compression failed";
            return false;
        }
    }
    // pass 4: write in input order
    for (int o = 0; o < nout; ++o) {
        Out& f = outs[o];
        for (int t = 0; t < nth; ++t) {
            auto put = [&](const Bytes& v) {
                if (v.empty()) return true;
                f.any = true;
                return fwrite(v.data(), 1, v.size(), f.fp) == v.size();
            };
            bool ok = true;
            if (f.gz) {
                for (const Bytes& pm : part[t][o]) ok = ok && put(pm);
                if (f.keep && !buf[t][o].empty()) {   // retain the text: move, not copy
                    const uint64_t nb = buf[t][o].size();
                    bool fits;
                    {
                        std::lock_guard<std::mutex> g(g_ret_mu);
                        fits = g_ret_bytes + nb <= retain_cap;
                        if (fits) g_ret_bytes += nb;
                    }
                    if (fits) {
                        f.kept_bytes += nb;
                        f.kept.push_back(std::move(buf[t][o]));
                    } else {                          // over the cap: this output goes to disk
                        std::lock_guard<std::mutex> g(g_ret_mu);
                        g_ret_bytes -= f.kept_bytes;
                        f.kept_bytes = 0;
                        f.keep = false;
                        std::vector<Bytes>().swap(f.kept);
                    }
                }
            } else {
                ok = put(buf[t][o]);
            }
            if (!ok) {
                e = "write failed: " + f.path + ": " + strerror(errno);
                return false;
            }
            f.n += cnt[t][o];
            f.bp += bps[t][o];
        }
    }
    return true;
}

void dmx_sink::worker() {
    for (;;) {
        std::unique_ptr<Job> j;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || pending; });
            if (!pending) return;
            j = std::move(pending);
        }
        std::string e;
        const bool ok = err.empty() ? process(*j, e) : true;
        release(j->b);
        std::lock_guard<std::mutex> lk(mu);
        if (!ok && err.empty()) err = e;
        busy = false;
        cv.notify_all();
    }
}

extern "C" {

int dmx_sink_open(const char* const* paths, int n_out, int fasta_out, int level, int threads,
                  dmx_sink** out) {
    if (!paths || n_out <= 0 || !out) return -1;
    *out = nullptr;
    auto* s = new dmx_sink();
    s->fasta_out = fasta_out != 0;
    s->level = std::max(0, std::min(9, level));
    s->threads = clamp_threads(threads);
    s->outs.resize(n_out);
    for (int o = 0; o < n_out; ++o) {
        Out& f = s->outs[o];
        f.path = paths[o] ? paths[o] : "";
        f.gz = f.path.size() > 3 && f.path.compare(f.path.size() - 3, 3, ".gz") == 0;
        f.fp = f.path == "-" ? stdout : fopen(f.path.c_str(), "wb");
        if (!f.fp) {
            s->api_err = "cannot open " + f.path + ": " + strerror(errno);
            for (int k = 0; k < o; ++k)
                if (s->outs[k].fp && s->outs[k].fp != stdout) fclose(s->outs[k].fp);
            for (auto& g : s->outs) g.fp = nullptr;
            *out = s;   // caller reads the message, then frees
            return -2;
        }
        setvbuf(f.fp, nullptr, _IOFBF, 1 << 20);
    }
    s->th = std::thread([s] { s->worker(); });
    *out = s;
    return 0;
}

}  // extern "C"

namespace {

int sink_enqueue(dmx_sink* s, Batch* b, std::unique_ptr<Job> j) {
    std::unique_lock<std::mutex> lk(s->mu);
    s->cv.wait(lk, [&] { return !s->busy; });
    if (!s->err.empty()) {
        s->api_err = s->err;
        return -3;
    }
    b->refs.fetch_add(1);
    j->b = b;
    s->pending = std::move(j);
    s->busy = true;
    s->cv.notify_all();
    return 0;
}

struct QualTable {
    double p[256];
    QualTable() {
        for (int i = 0; i < 256; ++i) p[i] = std::pow(10.0, -((double)i - 33.0) / 10.0);
    }
};

// 32 nt of a packed stream (include/dmx.h layout) from nt position p: their 2-bit codes and
// their no-match bits.  Reads up to two words past the 32 nt, inside a batch's tail pad.
inline uint64_t codes32_at(const uint32_t* w, uint64_t p) {
    const uint64_t i = p / 16;
    const unsigned __int128 v = (unsigned __int128)w[i] | ((unsigned __int128)w[i + 1] << 32) |
                                ((unsigned __int128)w[i + 2] << 64);
    return (uint64_t)(v >> (2 * (unsigned)(p % 16)));
}
inline uint32_t mask32_at(const uint32_t* m, uint64_t p) {
    const uint64_t i = p / 32;
    return (uint32_t)((((uint64_t)m[i + 1] << 32) | (uint64_t)m[i]) >> (p % 32));
}
inline uint64_t rev_fields2(uint64_t x) {   // reverse the order of the 32 2-bit fields
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
    return __builtin_bswap64(x);
}
inline uint32_t rev_bits32(uint32_t x) {
    x = ((x >> 1) & 0x55555555u) | ((x & 0x55555555u) << 1);
    x = ((x >> 2) & 0x33333333u) | ((x & 0x33333333u) << 2);
    x = ((x >> 4) & 0x0F0F0F0Fu) | ((x & 0x0F0F0F0Fu) << 4);
    return __builtin_bswap32(x);
}
inline uint64_t spread2(uint32_t m) {   // bit k -> bits 2k and 2k + 1
    uint64_t x = m;
    x = (x | (x << 16)) & 0x0000FFFF0000FFFFull;
    x = (x | (x << 8)) & 0x00FF00FF00FF00FFull;
    x = (x | (x << 4)) & 0x0F0F0F0F0F0F0F0Full;
    x = (x | (x << 2)) & 0x3333333333333333ull;
    x = (x | (x << 1)) & 0x5555555555555555ull;
    return x | (x << 1);
}

// One view of n nt at nt position p of a batch's packed words, reverse-complemented if rc,
// packed at g0 (a 32-nt boundary) exactly as dmx::pack_one / pack_one_rc would pack its text:
// a word copy per 32 nt instead of a table lookup per nt.  The batch words were packed from the
// same text by pack_one, so a forward copy is that packing; on the reverse strand a code becomes
// code ^ 3 (A<->T, C<->G) and a no-match nt keeps code 0 and its mask bit.  Whole groups are
// written, with the fields past n zero.
inline void pack_view(const uint32_t* seq, const uint32_t* nm, uint64_t p, uint32_t n, bool rc,
                      uint64_t g0, uint32_t* out_seq, uint32_t* out_nm) {
    uint32_t* sw = out_seq + g0 / 16;
    uint32_t* nw = out_nm + g0 / 32;
    for (uint32_t x = 0; x < n; x += 32) {
        const uint32_t cnt = n - x < 32u ? n - x : 32u;
        uint64_t c;
        uint32_t m;
        if (!rc) {
            c = codes32_at(seq, p + x);
            m = mask32_at(nm, p + x);
        } else {   // output nt y = complement of view nt n - 1 - (x + y): the block ending there
            const uint64_t q = p + n - x - 32;   // >= p - 31 >= kPad - 31 > 0
            m = rev_bits32(mask32_at(nm, q));
            c = (~rev_fields2(codes32_at(seq, q))) & ~spread2(m);
        }
        if (cnt < 32) {
            c &= (1ull << (2 * cnt)) - 1ull;
            m &= (1u << cnt) - 1u;
        }
        sw[x / 16] = (uint32_t)c;
        sw[x / 16 + 1] = (uint32_t)(c >> 32);
        nw[x / 32] = m;
    }
}

// Mean qualities of reads [lo, hi): each read's sum runs in read order from 0.0 (bit-exact with
// a plain loop, oracle/chopper.py mean_qual), but four reads' chains are interleaved, so each
// add's latency hides behind the other chains' adds.  A chain whose read ends takes the next.
void mean_qual_range(const Batch* b, const double* tab, size_t lo, size_t hi, double* out) {
    constexpr int K = 4;
    const uint8_t* qp[K];
    uint32_t left[K];
    double sum[K];
    size_t rid[K];
    size_t next = lo;
    const auto finish = [&](size_t r, double s) {
        out[r] = -10.0 * std::log10(s / (double)b->lens_v[r]);
    };
    const auto refill = [&](int j) {
        while (next < hi) {
            const size_t r = next++;
            if (!b->lens_v[r]) {
                out[r] = 0.0;
                continue;
            }
            qp[j] = b->text_v.data() + b->qual_v[2 * r];
            left[j] = b->lens_v[r];
            sum[j] = 0.0;
            rid[j] = r;
            return true;
        }
        return false;
    };
    int act = 0;
    while (act < K && refill(act)) ++act;
    while (act == K) {
        const uint32_t step = std::min(std::min(left[0], left[1]), std::min(left[2], left[3]));
        double s0 = sum[0], s1 = sum[1], s2 = sum[2], s3 = sum[3];
        const uint8_t *a0 = qp[0], *a1 = qp[1], *a2 = qp[2], *a3 = qp[3];
        for (uint32_t k = 0; k < step; ++k) {
            s0 += tab[a0[k]];
            s1 += tab[a1[k]];
            s2 += tab[a2[k]];
            s3 += tab[a3[k]];
        }
        sum[0] = s0, sum[1] = s1, sum[2] = s2, sum[3] = s3;
        for (int j = K - 1; j >= 0; --j) {
            qp[j] += step;
            left[j] -= step;
            if (left[j]) continue;
            finish(rid[j], sum[j]);
            if (!refill(j)) {   // the range is drained: keep the chains compact
                --act;
                qp[j] = qp[act], left[j] = left[act], sum[j] = sum[act], rid[j] = rid[act];
            }
        }
    }
    for (int j = 0; j < act; ++j) {
        double s = sum[j];
        for (uint32_t k = 0; k < left[j]; ++k) s += tab[qp[j][k]];
        finish(rid[j], s);
    }
}

}  // namespace

extern "C" {

int dmx_sink_write(dmx_sink* s, dmx_batch* bp, const int32_t* out_idx, const int32_t* start,
                   const int32_t* stop, const uint8_t* rc, const uint8_t* n_rc) {
    if (!s || !bp || s->closed || !s->th.joinable()) return -1;
    Batch* b = static_cast<Batch*>(bp);
    const size_t n = b->n_reads;
    if (n && (!out_idx || !start || !stop || !rc || !n_rc)) return -1;
    auto j = std::make_unique<Job>();
    j->idx.assign(out_idx, out_idx + n);
    j->start.assign(start, start + n);
    j->stop.assign(stop, stop + n);
    j->rc.assign(rc, rc + n);
    j->nrc.assign(n_rc, n_rc + n);
    return sink_enqueue(s, b, std::move(j));
}

int dmx_sink_write_rows(dmx_sink* s, dmx_batch* bp, size_t n_rows, const uint32_t* read,
                        const int32_t* out_idx, const int32_t* start, const int32_t* stop,
                        const uint8_t* rc, const uint8_t* name_mode) {
    if (!s || !bp || s->closed || !s->th.joinable()) return -1;
    if (n_rows && (!read || !out_idx || !start || !stop || !rc || !name_mode)) return -1;
    Batch* b = static_cast<Batch*>(bp);
    auto j = std::make_unique<Job>();
    j->rows = true;
    j->rread.assign(read, read + n_rows);
    j->idx.assign(out_idx, out_idx + n_rows);
    j->start.assign(start, start + n_rows);
    j->stop.assign(stop, stop + n_rows);
    j->rc.assign(rc, rc + n_rows);
    j->mode.assign(name_mode, name_mode + n_rows);
    for (uint8_t m : j->mode)
        if (m > 1) return -1;   // mode 2 needs the segment names (dmx_sink_write_rows2)
    j->nrc.assign(n_rows, 0);
    return sink_enqueue(s, b, std::move(j));
}

int dmx_sink_write_rows2(dmx_sink* s, dmx_batch* bp, size_t n_rows, const uint32_t* read,
                         const int32_t* out_idx, const int32_t* start, const int32_t* stop,
                         const uint8_t* rc, const int32_t* name_start, const int32_t* name_stop,
                         const uint8_t* name_strand, const uint8_t* n_rc) {
    if (!s || !bp || s->closed || !s->th.joinable()) return -1;
    if (n_rows && (!read || !out_idx || !start || !stop || !rc || !name_start || !name_stop ||
                   !name_strand || !n_rc))
        return -1;
    Batch* b = static_cast<Batch*>(bp);
    auto j = std::make_unique<Job>();
    j->rows = true;
    j->rread.assign(read, read + n_rows);
    j->idx.assign(out_idx, out_idx + n_rows);
    j->start.assign(start, start + n_rows);
    j->stop.assign(stop, stop + n_rows);
    j->rc.assign(rc, rc + n_rows);
    j->mode.assign(n_rows, 2);
    j->nstart.assign(name_start, name_start + n_rows);
    j->nstop.assign(name_stop, name_stop + n_rows);
    j->nstrand.assign(name_strand, name_strand + n_rows);
    j->nrc.assign(n_rc, n_rc + n_rows);
    return sink_enqueue(s, b, std::move(j));
}

int dmx_batch_pack_views(const dmx_batch* bp, size_t n_views, const uint32_t* read,
                         const int32_t* start, const int32_t* stop, const uint8_t* rc,
                         int threads, uint32_t* out_seq2b, uint32_t* out_nmask,
                         uint64_t* out_offsets, uint32_t* out_lens, size_t n_words) {
    if (!bp || (n_views && (!read || !start || !stop || !rc || !out_offsets || !out_lens)) ||
        !out_seq2b || !out_nmask)
        return -1;
    const Batch* b = static_cast<const Batch*>(bp);
    uint64_t g = kPad, total = 0;
    for (size_t i = 0; i < n_views; ++i) {
        if (read[i] >= b->n_reads || start[i] < 0 || stop[i] < start[i] ||
            (uint32_t)stop[i] > b->lens_v[read[i]])
            return -2;
        out_offsets[i] = g;
        out_lens[i] = (uint32_t)(stop[i] - start[i]);
        g += ((uint64_t)out_lens[i] + dmx::kPackAlign - 1) / dmx::kPackAlign * dmx::kPackAlign;
        total += out_lens[i];
    }
    // the same word count as dmx_pack_words(total, n_views) (include/dmx.h)
    const uint64_t nt = 2 * kPad + total + (uint64_t)dmx::kPackAlign * n_views;
    if (n_words < (size_t)((nt + 31) / 32 * 2 + 4)) return -3;
    // views tile [kPad, g) in whole 32-nt groups, each written below: zero the rest only
    std::fill(out_seq2b, out_seq2b + kPad / 16, 0u);
    std::fill(out_nmask, out_nmask + kPad / 32, 0u);
    std::fill(out_seq2b + std::min<size_t>(n_words, g / 16), out_seq2b + n_words, 0u);
    std::fill(out_nmask + std::min<size_t>(n_words, g / 32), out_nmask + n_words, 0u);
    const int nth = (int)std::min<size_t>(clamp_threads(threads), std::max<size_t>(1, n_views / 1024));
    parallel(nth, [&](int t) {
        const size_t lo = n_views * t / nth, hi = n_views * (t + 1) / nth;
        for (size_t i = lo; i < hi; ++i)
            pack_view(b->seq2b_v.data(), b->nmask_v.data(), b->offs_v[read[i]] + (uint64_t)start[i],
                      out_lens[i], rc[i] != 0, out_offsets[i], out_seq2b, out_nmask);
    });
    return 0;
}

int dmx_batch_mean_qual(const dmx_batch* bp, double* out) {
    if (!bp) return -1;
    const Batch* b = static_cast<const Batch*>(bp);
    if (b->fasta) return -2;
    const size_t n = b->n_reads;
    if (n && !out) return -1;
    static const QualTable qt;
    const int nth = (int)std::min<size_t>(std::min(clamp_threads(0), 16),
                                          std::max<size_t>(1, n / 4096));
    parallel(nth, [&](int t) {
        mean_qual_range(b, qt.p, n * t / nth, n * (t + 1) / nth, out);
    });
    return 0;
}

int dmx_sink_close(dmx_sink* s, uint64_t* n_written, uint64_t* bp_written) {
    if (!s) return -1;
    if (s->th.joinable()) {
        {
            std::unique_lock<std::mutex> lk(s->mu);
            s->cv.wait(lk, [&] { return !s->busy; });
            s->stop = true;
            s->cv.notify_all();
        }
        s->th.join();
    }
    int rc = 0;
    if (!s->err.empty()) {
        s->api_err = s->err;
        rc = -3;
    }
    for (size_t o = 0; o < s->outs.size(); ++o) {
        Out& f = s->outs[o];
        if (!f.fp) continue;
        if (f.gz && !f.any) {   // empty output: still a valid gzip file
            Bytes m;
            if (!gzip_member(nullptr, 0, s->level, m) || fwrite(m.data(), 1, m.size(), f.fp) != m.size()) {
                s->api_err = "write failed: " + f.path;
                rc = -3;
            }
        }
        const bool is_std = f.fp == stdout;
        if (is_std ? fflush(f.fp) != 0 : fclose(f.fp) != 0) {
            s->api_err = "close failed: " + f.path + ": " + strerror(errno);
            rc = -3;
        }
        f.fp = nullptr;
        if (f.keep) {   // register the retained text under the file's identity as written
            Retained r;
            struct stat st;
            const std::string rp = is_std ? std::string() : real_path(f.path.c_str());
            if (rc == 0 && !rp.empty() && ::stat(rp.c_str(), &st) == 0 &&
                head_crc(rp.c_str(), r.head_crc)) {
                r.pieces = std::move(f.kept);
                r.bytes = f.kept_bytes;
                r.dev = st.st_dev;
                r.ino = st.st_ino;
                r.size = st.st_size;
                r.mtime_ns = mtime_ns(st);
                std::lock_guard<std::mutex> g(g_ret_mu);
                auto it = g_retained.find(rp);
                if (it != g_retained.end()) {   // an older retained copy of the same path
                    g_ret_bytes -= it->second.bytes;
                    g_retained.erase(it);
                }
                g_retained.emplace(rp, std::move(r));
            } else {
                std::lock_guard<std::mutex> g(g_ret_mu);
                g_ret_bytes -= f.kept_bytes;
            }
            f.kept_bytes = 0;
            f.keep = false;
            std::vector<Bytes>().swap(f.kept);
        }
        if (n_written) n_written[o] = f.n;
        if (bp_written) bp_written[o] = f.bp;
    }
    s->closed = true;
    return rc;
}

const char* dmx_sink_error(dmx_sink* s) { return s ? s->api_err.c_str() : "null sink"; }

int dmx_sink_retain(dmx_sink* s, uint64_t max_bytes) {
    if (!s) return -1;
    std::unique_lock<std::mutex> lk(s->mu);
    s->cv.wait(lk, [&] { return !s->busy; });
    s->retain_cap = max_bytes;
    for (auto& f : s->outs) f.keep = max_bytes > 0 && f.gz && f.path != "-" && f.n == 0;
    return 0;
}

int dmx_sink_retain_output(dmx_sink* s, int o, int keep) {
    if (!s || o < 0 || o >= (int)s->outs.size()) return -1;
    std::unique_lock<std::mutex> lk(s->mu);
    s->cv.wait(lk, [&] { return !s->busy; });
    Out& f = s->outs[o];
    if (!keep) {   // never retained from here on; release what it already holds
        if (f.kept_bytes) {
            std::lock_guard<std::mutex> g(g_ret_mu);
            g_ret_bytes -= f.kept_bytes;
        }
        f.kept_bytes = 0;
        f.keep = false;
        std::vector<Bytes>().swap(f.kept);
    } else if (f.n == 0) {
        f.keep = s->retain_cap > 0 && f.gz && f.path != "-";
    }
    return 0;
}

uint64_t dmx_io_retained_bytes(void) {
    std::lock_guard<std::mutex> g(g_ret_mu);
    return g_ret_bytes;
}

void dmx_io_drop_retained(void) {
    std::lock_guard<std::mutex> g(g_ret_mu);
    for (const auto& kv : g_retained) g_ret_bytes -= kv.second.bytes;   // (open sinks' bytes
    g_retained.clear();                                                 //  stay counted)
}

void dmx_sink_free(dmx_sink* s) {
    if (!s) return;
    if (!s->closed) dmx_sink_close(s, nullptr, nullptr);
    delete s;
}

}  // extern "C"
