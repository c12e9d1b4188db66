// Single-thread decode speed of csrc/dmx_inflate.h against zlib on one gzip file (CPU only).
//   g++ -O3 -march=native -I nanopore-barcoding-orc_amd/csrc tools/microbench/inflate_speed.cpp \
//       -lz -o tools/microbench/inflate_speed && tools/microbench/inflate_speed FILE.gz
// Prints MB/s of output for: zlib inflate; inflate_run<uint8_t> (the reader's chunk 0, real
// window); inflate_run<uint16_t> (a speculative chunk's 16-bit output, here from the start).
#include <zlib.h>

#include <chrono>
#include <cstdio>
#include <vector>

#include "dmx_inflate.h"

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

template <typename T>
static double run_dmx(const std::vector<uint8_t>& gz, size_t& n_out) {
    dmxi::In in{gz.data(), gz.size() - 64, true};
    dmxi::Buf<T> out;
    out.reserve(dmxi::kWin + (gz.size() * 4));
    for (int i = 0; i < dmxi::kWin; ++i) out.p[i] = (T)(sizeof(T) == 1 ? 0 : 256 + i);
    out.n = dmxi::kWin;
    std::vector<dmxi::Event> ev;
    uint64_t pos = 0;
    bool atm = true;
    const double t = now();
    const dmxi::Stop st = dmxi::inflate_run<T>(in, pos, atm, out, dmxi::kWin, UINT64_MAX, ev);
    const double dt = now() - t;
    if (st != dmxi::Stop::kEnd) fprintf(stderr, "dmx decode stopped with %d\n", (int)st);
    n_out = out.n - dmxi::kWin;
    return dt;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    std::vector<uint8_t> gz;
    uint8_t buf[1 << 16];
    for (size_t k; (k = fread(buf, 1, sizeof buf, f)) > 0;) gz.insert(gz.end(), buf, buf + k);
    fclose(f);
    const size_t clen = gz.size();
    gz.resize(clen + 64, 0);

    std::vector<uint8_t> out(clen * 4);
    z_stream zs{};
    inflateInit2(&zs, 31);
    zs.next_in = gz.data();
    zs.avail_in = (uInt)clen;
    size_t zn = 0;
    const double t = now();
    for (;;) {
        zs.next_out = out.data() + zn;
        zs.avail_out = (uInt)std::min<size_t>(out.size() - zn, 1u << 30);
        const int r = inflate(&zs, Z_NO_FLUSH);
        zn = out.size() - zn - zs.avail_out + zn;
        zn = (size_t)(zs.next_out - out.data());
        if (r == Z_STREAM_END) break;
        if (r != Z_OK) {
            fprintf(stderr, "zlib %d\n", r);
            return 1;
        }
    }
    const double tz = now() - t;
    inflateEnd(&zs);
    size_t n8 = 0, n16 = 0;
    const double t8 = run_dmx<uint8_t>(gz, n8);
    const double t16 = run_dmx<uint16_t>(gz, n16);
    printf("{\"out_mb\": %.1f, \"zlib_mb_s\": %.1f, \"dmx_u8_mb_s\": %.1f, \"dmx_u16_mb_s\": %.1f, "
           "\"same_size\": %s}\n", zn / 1e6, zn / 1e6 / tz, n8 / 1e6 / t8, n16 / 1e6 / t16,
           (n8 == zn && n16 == zn) ? "true" : "false");
    return 0;
}
