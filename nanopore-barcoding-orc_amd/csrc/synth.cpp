// synth.cpp — seeded synthetic nanopore amplicon reads for tests and benchmarks (host C++,
// no GPU).  Workload shapes follow SURVEY.md §8d (configs 1-4): read = [flank] SP5_i + insert +
// SP27rc_j [flank] (pychopper orientation, 01_pychopper.sh config "+:SP5,-SP27"), adapter
// regions mutated at rate e (sub:ins:del = 60:20:20), a fraction reverse-complemented and a
// fraction without adapters.  Every read is a pure function of (seed, read index), so shards
// generated on different ranks are identical to one big generation.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {   // splitmix64
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
    uint32_t below(uint32_t n) { return (uint32_t)(uni() * n); }
    double normal() {
        double u1 = uni(), u2 = uni();
        if (u1 < 1e-300) u1 = 1e-300;
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
    }
};

const char kBases[4] = {'A', 'C', 'G', 'T'};

inline char comp(char c) {
    switch (c) {
        case 'A': return 'T';
        case 'C': return 'G';
        case 'G': return 'C';
        case 'T': return 'A';
        default: return 'N';
    }
}

}  // namespace

extern "C" {

// Parameters of one synthetic workload.
struct SynthParams {
    int32_t length_model;      // 0 fixed total length, 1 lognormal, 2 COI/rRNA mixture
    double len_mean;           // model 0: fixed length; model 1: mean of the lognormal
    double len_sigma_log;      // model 1
    int32_t len_min, len_max;  // clip
    double adapter_error;      // per adapter base
    double rc_fraction;
    double adapterless_fraction;
    double n_fraction;         // per insert base: an 'N'
    int32_t n1_used, n2_used;  // adapters drawn from the first n*_used of each panel
    int32_t flank_max;         // random flank length U[0, flank_max] on both ends
    int32_t linked;            // 1: pair i of both panels (linked primers, config 5)
    double missing_fraction;   // linked: one primer (front or back, equally) left out
};

static uint32_t draw_length(const SynthParams& p, Rng& g) {
    double L;
    if (p.length_model == 0) {
        L = p.len_mean;
    } else if (p.length_model == 1) {
        const double mu = std::log(p.len_mean) - 0.5 * p.len_sigma_log * p.len_sigma_log;
        L = std::exp(mu + p.len_sigma_log * g.normal());
    } else if (p.length_model == 2) {   // 70% COI insert U[300,900], 30% rRNA N(3000,150)
        if (g.uni() < 0.7) L = 300 + g.uni() * 600 + 116;   // + ~116 nt of adapters
        else L = 3000 + 150 * g.normal() + 116;
    } else {   // 3: COI amplicon consensus: insert U[300,900] + two ~26-nt primers
        L = 300 + g.uni() * 600 + 52;
    }
    if (L < p.len_min) L = p.len_min;
    if (L > p.len_max) L = p.len_max;
    return (uint32_t)L;
}

static inline uint64_t read_seed(uint64_t seed, uint64_t idx) {
    Rng g(seed ^ (idx * 0xD1B54A32D192ED03ull));
    return g.next();
}

// Upper bound of the generated length of each read (mutations may add a few bases).
void synth_lengths(const SynthParams* p, uint64_t seed, uint64_t first, size_t n,
                   uint32_t* out_cap) {
    for (size_t r = 0; r < n; ++r) {
        Rng g(read_seed(seed, first + r));
        out_cap[r] = draw_length(*p, g) + 2 * (uint32_t)p->flank_max + 64;
    }
}

// One base of an IUPAC code (degenerate primer positions are instantiated at random).
static char instantiate(char c, Rng& g) {
    const char* set;
    switch (c) {
        case 'A': case 'C': case 'G': case 'T': return c;
        case 'R': set = "AG"; break;
        case 'Y': set = "CT"; break;
        case 'S': set = "CG"; break;
        case 'W': set = "AT"; break;
        case 'K': set = "GT"; break;
        case 'M': set = "AC"; break;
        case 'B': set = "CGT"; break;
        case 'D': set = "AGT"; break;
        case 'H': set = "ACT"; break;
        case 'V': set = "ACG"; break;
        default: set = "ACGT"; break;
    }
    return set[g.below((uint32_t)strlen(set))];
}

static void mutate_into(const char* a, int m, double e, Rng& g, std::vector<char>& out) {
    for (int i = 0; i < m; ++i) {
        const char ai = instantiate(a[i], g);
        if (g.uni() < e) {
            const double k = g.uni();
            if (k < 0.6) {
                char c;
                do c = kBases[g.below(4)]; while (c == ai);
                out.push_back(c);
            } else if (k < 0.8) {
                out.push_back(kBases[g.below(4)]);
                out.push_back(ai);
            }   // else deletion
        } else {
            out.push_back(ai);
        }
    }
}

static void gen_one(const SynthParams& p, const char* const* p1, const int* l1,
                    const char* const* p2, const int* l2, uint64_t seed, uint64_t idx, char* out,
                    uint32_t* out_len, int32_t* truth) {
    Rng g(read_seed(seed, idx));
    const uint32_t L = draw_length(p, g);
    std::vector<char> s;
    s.reserve(L + 2 * p.flank_max + 64);
    const bool adapterless = g.uni() < p.adapterless_fraction;
    const bool rc = g.uni() < p.rc_fraction;
    int i = -1, j = -1;
    if (adapterless) {
        for (uint32_t x = 0; x < L; ++x) s.push_back(kBases[g.below(4)]);
    } else {
        i = (int)g.below((uint32_t)p.n1_used);
        j = p.linked ? i : (int)g.below((uint32_t)p.n2_used);
        bool no1 = false, no2 = false;   // linked: one primer missing
        if (p.linked && g.uni() < p.missing_fraction) {
            if (g.uni() < 0.5) no1 = true;
            else no2 = true;
        }
        const int f1 = p.flank_max ? (int)g.below((uint32_t)p.flank_max + 1) : 0;
        const int f2 = p.flank_max ? (int)g.below((uint32_t)p.flank_max + 1) : 0;
        for (int x = 0; x < f1; ++x) s.push_back(kBases[g.below(4)]);
        if (!no1) mutate_into(p1[i], l1[i], p.adapter_error, g, s);
        const int ins = (int)L - l1[i] - l2[j];
        for (int x = 0; x < ins; ++x)
            s.push_back(g.uni() < p.n_fraction ? 'N' : kBases[g.below(4)]);
        if (!no2) mutate_into(p2[j], l2[j], p.adapter_error, g, s);
        if (no1) i = -1;
        if (no2) j = -1;
        for (int x = 0; x < f2; ++x) s.push_back(kBases[g.below(4)]);
    }
    const size_t n = s.size();
    if (rc) {
        for (size_t x = 0; x < n; ++x) out[x] = comp(s[n - 1 - x]);
    } else {
        memcpy(out, s.data(), n);
    }
    *out_len = (uint32_t)n;
    if (truth) {
        truth[0] = i;
        truth[1] = j;
        truth[2] = rc ? 1 : 0;
    }
}

// Generate reads [first, first+n) into out (read r at out + offs[r], offs from synth_lengths
// caps), writing the real lengths; truth (optional) = n x {sp5 idx, sp27 idx, rc}.
void synth_fill(const SynthParams* p, const char* const* p1, const int* l1, const char* const* p2,
                const int* l2, uint64_t seed, uint64_t first, size_t n, const uint64_t* offs,
                char* out, uint32_t* out_lens, int32_t* truth, int threads) {
    if (threads < 1) threads = 1;
    auto work = [&](size_t lo, size_t hi) {
        for (size_t r = lo; r < hi; ++r)
            gen_one(*p, p1, l1, p2, l2, seed, first + r, out + offs[r], &out_lens[r],
                    truth ? truth + 3 * r : nullptr);
    };
    if (threads == 1 || n < 1024) {
        work(0, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (n + threads - 1) / threads;
    for (int t = 0; t < threads; ++t) {
        const size_t lo = (size_t)t * per, hi = lo + per < n ? lo + per : n;
        if (lo >= hi) break;
        th.emplace_back(work, lo, hi);
    }
    for (auto& t : th) t.join();
}

}  // extern "C"
