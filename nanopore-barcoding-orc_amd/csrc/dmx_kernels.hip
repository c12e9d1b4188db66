// dmx_kernels.hip — gfx950 kernels of the two-round demultiplexer and their launch sequence.
//
// Replaces the per-read hot loop of cutadapt 4.9 as driven by scripts/02_cutadapt_loop.sh:64-72
// (round 1: 5' SP5 adapters, --rc) and :91-103 (round 2: 3' SP27rc adapters, --rc, on every SP5
// bin), and scripts/04_cleaning_primers.sh:371-388 (linked primers).  Semantics restated in
// oracle/cutadapt_oracle.c; design and exactness argument in DESIGN.md §3.
//
// Per round: scan -> resolve -> select -> finalize, all on one HIP stream, no host round trip.
#include "dmx_device.h"
#include "dmx_internal.h"

namespace dmx {

// ---------------------------------------------------------------------------------------------
// shared helpers
// ---------------------------------------------------------------------------------------------
struct RoundArgs {
    const uint32_t* seq;
    const uint32_t* nmask;
    const uint64_t* offs;
    const uint32_t* lens;
    const DevPanel* panel;
    const ItemView* items;       // nullptr: item i = read i, whole read (round 0)
    const uint32_t* n_items_dev; // device count of items (when items != nullptr)
    uint32_t n_items;            // host count / upper bound
    int32_t T;                   // tasks per item
    int32_t per_task_slot;       // linked round 0: one winner slot per (read, pair)
    Cluster* cl;
    Outcome* outc;
    uint32_t* cl_count;
    uint32_t cl_cap;
    uint32_t* flags;             // bit0 cluster overflow, bit1 window violation
    unsigned long long* winner;  // per slot, ~0 = none
    int32_t* origin;             // per slot
};

struct TaskView {
    uint32_t read, n, strand, start, len;
    uint64_t off;
    int o, a;
};

__device__ __forceinline__ bool task_view(const RoundArgs& R, uint32_t item, int sub, int A,
                                          TaskView& tv) {
    if (R.items) {
        const ItemView v = R.items[item];
        tv.read = v.read;
        tv.start = v.start;
        tv.len = v.len;
        tv.strand = v.strand;
        if (v.only_adapter >= 0) {   // linked: exactly one task per item, no RC
            tv.o = 0;
            tv.a = v.only_adapter;
        } else {
            tv.o = sub / A;
            tv.a = sub % A;
        }
    } else {
        tv.read = item;
        tv.start = 0;
        tv.strand = 0;
        tv.len = R.lens[item];
        tv.o = sub / A;
        tv.a = sub % A;
        if (R.per_task_slot) {
            tv.o = 0;
            tv.a = sub;
        }
    }
    tv.n = R.lens[tv.read];
    tv.off = R.offs[tv.read];
    if (tv.o) {   // reverse complement of the view (strand s, start st, len l) of a read of n nt
        tv.start = tv.n - tv.start - tv.len;
        tv.strand ^= 1u;
    }
    return true;
}

__device__ __forceinline__ uint32_t slot_of(const RoundArgs& R, uint32_t item, int sub) {
    return R.per_task_slot ? item * (uint32_t)R.T + (uint32_t)sub : item;
}

__device__ __forceinline__ void load_panel_lds(const DevPanel* P, uint64_t* s_peq, int8_t* s_acc) {
    const int A = P->n_adapters;
    for (int x = threadIdx.x; x < 8 * A; x += blockDim.x) {
        const int c = x / A, a = x % A;
        s_peq[x] = P->ad[a].peq[c];   // code-major: lanes of one read hit consecutive words
    }
    for (int x = threadIdx.x; x < 72 * A; x += blockDim.x) s_acc[x] = P->ad[x / 72].acc[x % 72];
}

// ---------------------------------------------------------------------------------------------
// scan: one lane per (item, orientation, adapter); full-read Myers; emits candidate clusters.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void emit_cluster(const RoundArgs& R, uint32_t item, int sub,
                                             uint32_t j1, uint32_t j2, int lastcol) {
    const uint32_t idx = atomicAdd(R.cl_count, 1u);
    if (idx < R.cl_cap) {
        Cluster c;
        c.item = item;
        c.sub = (uint16_t)sub;
        c.lastcol = (uint8_t)lastcol;
        c.pad = 0;
        c.j1 = j1;
        c.j2 = j2;
        R.cl[idx] = c;
    } else {
        atomicOr(R.flags, 1u);
    }
}

__global__ __launch_bounds__(kScanBlock) void scan_kernel(RoundArgs R) {
    __shared__ uint64_t s_peq[8 * kMaxAdapters];
    __shared__ int8_t s_acc[72 * kMaxAdapters];
    load_panel_lds(R.panel, s_peq, s_acc);
    __syncthreads();

    const int A = R.panel->n_adapters;
    const int T = R.T;
    const int rpb = kScanBlock / T;
    const int tid = threadIdx.x;
    if (tid >= rpb * T) return;
    const uint32_t item = blockIdx.x * (uint32_t)rpb + (uint32_t)(tid / T);
    const int sub = tid % T;
    const uint32_t n_items = R.items ? *R.n_items_dev : R.n_items;
    if (item >= n_items) return;

    TaskView tv;
    task_view(R, item, sub, A, tv);
    const DevAdapter& ad = R.panel->ad[tv.a];
    const int m = ad.m;
    const int kk = ad.kk;
    const bool front = ad.where == kFront;
    const uint32_t hbit = (uint32_t)(m - 1);
    const uint32_t gap = (uint32_t)(m + ad.k + 1);
    const uint64_t* peq = s_peq + tv.a;   // peq[code * A]

    uint64_t pv = front ? 0ull : ~0ull, mv = 0ull;
    int d = front ? 0 : m;
    bool have = false;
    uint32_t cj1 = 0, cj2 = 0;

#define DMX_SCAN_STEP(q)                                                                  \
    {                                                                                     \
        const uint32_t code = ((codes >> (2 * (q))) & 3u) | (((nb >> (q)) & 1u) << 2);    \
        myers_step(peq[code * A], pv, mv, d, hbit);                                       \
        if (d <= kk) {                                                                    \
            const uint32_t j = p0 + (q) + 1;                                              \
            if (have && j - cj2 <= gap) {                                                 \
                cj2 = j;                                                                  \
            } else {                                                                      \
                if (have) emit_cluster(R, item, sub, cj1, cj2, 0);                        \
                have = true;                                                              \
                cj1 = cj2 = j;                                                            \
            }                                                                             \
        }                                                                                 \
    }

    const uint32_t len = tv.len;
    uint32_t p0 = 0;
    for (; p0 + 16 <= len; p0 += 16) {
        uint32_t codes, nb;
        fetch16(R.seq, R.nmask, tv.off, tv.n, tv.strand, tv.start, p0, codes, nb);
#pragma unroll
        for (int q = 0; q < 16; ++q) DMX_SCAN_STEP(q)
    }
    if (p0 < len) {
        uint32_t codes, nb;
        fetch16(R.seq, R.nmask, tv.off, tv.n, tv.strand, tv.start, p0, codes, nb);
        const int cnt = (int)(len - p0);
        for (int q = 0; q < cnt; ++q) DMX_SCAN_STEP(q)
    }
#undef DMX_SCAN_STEP

    // 3' adapters: cutadapt also scans the last column (cells (i, n), i < m: adapter suffix
    // hanging off the read end).  Flag it if any such cell could be accepted.
    if (!front && len > 0) {
        int dd = 0;
        bool any = false;
        const int8_t* acc = s_acc + 72 * tv.a;
        for (int i = 1; i < m; ++i) {
            dd += (int)((pv >> (i - 1)) & 1ull) - (int)((mv >> (i - 1)) & 1ull);
            any |= dd <= (int)acc[i];
        }
        if (any) {
            if (have && len - cj2 <= gap) {
                emit_cluster(R, item, sub, cj1, len, 1);
            } else {
                if (have) emit_cluster(R, item, sub, cj1, cj2, 0);
                emit_cluster(R, item, sub, len, len, 1);
            }
            have = false;
        }
    }
    if (have) emit_cluster(R, item, sub, cj1, cj2, 0);
}

// ---------------------------------------------------------------------------------------------
// resolve: one lane per cluster; restricted Myers window + cutadapt tie-broken traceback.
// ---------------------------------------------------------------------------------------------
struct Walker {
    const uint32_t* seq;
    const uint32_t* nmask;
    uint32_t* flags;
    TaskView tv;
    const uint64_t* peq;    // LDS, + adapter, stride A
    int A;
    const uint64_t* rp;     // LDS ring (P), lane-interleaved: rp[(j % kRing) * 64]
    const uint64_t* rm;
    int js;
    bool real, front;

    // Walk cutadapt's DP pointers from cell (i, j) back to the alignment start.
    // Pointer rule (_align.pyx locate): equal characters -> diagonal; else mismatch if
    // diag <= deletion and diag <= insertion; else insertion (up) if insertion <= deletion;
    // else deletion (left).  Scores: +1 match, -1 mismatch, -2 indel.
    __device__ void trace(int i, int j, int& origin, int& score) const {
        score = 0;
        while (i > 0) {
            if (j == js) {
                if (real) {
                    if (front) {
                        origin = -i;           // FRONT column 0: origin -i, score 0
                    } else {
                        score -= 2 * i;        // BACK column 0: cost i, score -2i, origin 0
                        origin = 0;
                    }
                } else {
                    atomicOr(flags, 2u);    // unreachable for cost <= k
                    score -= 2 * i;
                    origin = js;
                }
                return;
            }
            uint32_t codes, nb;
            fetch16(seq, nmask, tv.off, tv.n, tv.strand, tv.start, (uint32_t)(j - 1),
                    codes, nb);
            const uint32_t code = (codes & 3u) | ((nb & 1u) << 2);
            if ((peq[code * A] >> (i - 1)) & 1ull) {
                --i;
                --j;
                ++score;
                continue;
            }
            const int s1 = ((j - 1) & (kRing - 1)) * 64;
            const int s0 = (j & (kRing - 1)) * 64;
            const uint64_t p1 = rp[s1], m1 = rm[s1];
            const int cdel = col_cost(p1, m1, i);                                   // D(i, j-1)
            const int cd = cdel - (int)((p1 >> (i - 1)) & 1ull) + (int)((m1 >> (i - 1)) & 1ull);
            const int cins = col_cost(rp[s0], rm[s0], i - 1);                       // D(i-1, j)
            if (cd <= cdel && cd <= cins) {
                --i;
                --j;
                score -= 1;
            } else if (cins <= cdel) {
                --i;
                score -= 2;
            } else {
                --j;
                score -= 2;
            }
        }
        origin = j;
    }
};

__global__ __launch_bounds__(kResolveBlock) void resolve_kernel(RoundArgs R) {
    __shared__ uint64_t s_peq[8 * kMaxAdapters];
    __shared__ int8_t s_acc[72 * kMaxAdapters];
    __shared__ uint64_t s_rp[kRing * kResolveBlock];
    __shared__ uint64_t s_rm[kRing * kResolveBlock];
    load_panel_lds(R.panel, s_peq, s_acc);
    __syncthreads();

    const int A = R.panel->n_adapters;
    const uint32_t total = min(*R.cl_count, R.cl_cap);
    const int lane = threadIdx.x;
    uint64_t* rp = s_rp + lane;
    uint64_t* rm = s_rm + lane;

    for (uint32_t ci = blockIdx.x * kResolveBlock + lane; ci < total;
         ci += gridDim.x * kResolveBlock) {
        const Cluster c = R.cl[ci];
        TaskView tv;
        task_view(R, c.item, c.sub, A, tv);
        const DevAdapter& ad = R.panel->ad[tv.a];
        const int m = ad.m, k = ad.k, kk = ad.kk;
        const bool front = ad.where == kFront;
        const uint32_t slot = slot_of(R, c.item, c.sub);
        const uint64_t snapshot = R.winner[slot];
        const int8_t* acc = s_acc + 72 * tv.a;

        int js = (int)c.j1 - m - k - 1;
        const bool real = js <= 0;
        if (real) js = 0;
        uint64_t pv = (front && real) ? 0ull : ~0ull, mv = 0ull;
        int d = (front && real) ? 0 : m;
        rp[(js & (kRing - 1)) * 64] = pv;
        rm[(js & (kRing - 1)) * 64] = mv;

        Walker W{R.seq, R.nmask, R.flags, tv, s_peq + tv.a, A, rp, rm, js, real, front};
        bool found = false;
        int bs = 0, bc = 0, bo = 0;
        uint64_t bt = 0;

        auto consider = [&](int iend, int j, int cost, uint64_t t) {
            const int ub = iend - 2 * cost;   // score <= aligned adapter length - 2 * cost
            if (found && (ub < bs || (ub == bs && cost >= bc))) return;
            if (make_key(ub, tv.o, cost, tv.a, t) > snapshot) return;
            int origin, score;
            if (cost == 0) {                  // exact: the pointer chain is the pure diagonal
                if (j >= iend) {
                    origin = j - iend;
                    score = iend;
                } else {
                    origin = j - iend;        // FRONT only: reaches column 0 at row iend - j
                    score = j;
                }
            } else {
                W.trace(iend, j, origin, score);
            }
            const int lr = iend + (origin < 0 ? origin : 0);
            if (lr < 0 || cost > (int)acc[lr]) return;
            if (!found || score > bs || (score == bs && cost < bc)) {
                found = true;
                bs = score;
                bc = cost;
                bt = t;
                bo = origin;
            }
        };

        const uint32_t hbit = (uint32_t)(m - 1);
        const uint64_t* peq = s_peq + tv.a;
        for (uint32_t p0 = (uint32_t)js; p0 < c.j2; p0 += 16) {
            uint32_t codes, nb;
            fetch16(R.seq, R.nmask, tv.off, tv.n, tv.strand, tv.start, p0, codes, nb);
            const uint32_t cnt = min(16u, c.j2 - p0);
            for (uint32_t q = 0; q < cnt; ++q) {
                const uint32_t code = ((codes >> (2 * q)) & 3u) | (((nb >> q) & 1u) << 2);
                myers_step(peq[code * A], pv, mv, d, hbit);
                const uint32_t j = p0 + q + 1;
                rp[(j & (kRing - 1)) * 64] = pv;
                rm[(j & (kRing - 1)) * 64] = mv;
                if (j >= c.j1 && d <= kk) consider(m, (int)j, d, j);
            }
        }
        if (c.lastcol && !front) {
            int dd = 0;
            for (int i = 1; i < m; ++i) {
                dd += (int)((pv >> (i - 1)) & 1ull) - (int)((mv >> (i - 1)) & 1ull);
                if (dd <= (int)acc[i]) consider(i, (int)tv.len, dd, (uint64_t)tv.len + 1 + i);
            }
        }
        Outcome out;
        out.key = ~0ull;
        out.origin = 0;
        out.pad = 0;
        if (found) {
            out.key = make_key(bs, tv.o, bc, tv.a, bt);
            out.origin = bo;
            atomicMin(&R.winner[slot], (unsigned long long)out.key);
        }
        R.outc[ci] = out;
    }
}

// select: the cluster whose outcome is the slot's winner publishes its origin.
__global__ void select_kernel(RoundArgs R) {
    const uint32_t total = min(*R.cl_count, R.cl_cap);
    for (uint32_t ci = blockIdx.x * blockDim.x + threadIdx.x; ci < total;
         ci += gridDim.x * blockDim.x) {
        const Outcome o = R.outc[ci];
        if (o.key == ~0ull) continue;
        const Cluster c = R.cl[ci];
        const uint32_t slot = slot_of(R, c.item, c.sub);
        if (R.winner[slot] == o.key) R.origin[slot] = o.origin;
    }
}

// ---------------------------------------------------------------------------------------------
// finalize
// ---------------------------------------------------------------------------------------------
// Decode a winning key into a cutadapt Match on a view of length vlen.
__device__ __forceinline__ void decode_match(uint64_t key, int origin, uint32_t vlen,
                                             const DevPanel* P, dmx_match& mt, int& a, int& o) {
    a = key_adapter(key);
    o = key_orient(key);
    const uint64_t t = key_t(key);
    int refstop, qstop;
    if (t <= vlen) {
        qstop = (int)t;
        refstop = P->ad[a].m;
    } else {
        refstop = (int)(t - vlen - 1);
        qstop = (int)vlen;
    }
    mt.rstop = qstop;
    mt.astop = (int16_t)refstop;
    if (origin >= 0) {
        mt.astart = 0;
        mt.rstart = origin;
    } else {
        mt.astart = (int16_t)(-origin);
        mt.rstart = 0;
    }
    mt.score = (int16_t)key_score(key);
    mt.errors = (int16_t)key_cost(key);
}

struct FinalArgs {
    const uint32_t* lens;
    const DevPanel* p0;
    const DevPanel* p1;
    const unsigned long long* winner;
    const int32_t* origin;
    dmx_result* res;
    ItemView* items;            // round-1 item list (out for finalize0, in for finalize1)
    uint32_t* n_items;
    uint32_t n_reads;
    int32_t mode;
    int32_t A0, A1;             // adapters per panel
    unsigned long long* counts; // (A0+1)*(A1+1) + 2
};

// Round 0 epilogue (one thread per read): write m1/bin1, build the round-1 view (the
// round-0-trimmed sequence: FRONT -> view[rstop:], BACK -> view[:rstart]) and queue it.
__global__ __launch_bounds__(256) void finalize0_kernel(FinalArgs F) {
    __shared__ unsigned int s_hist[2 * (kMaxAdapters + 1) + 1];
    const int nh = F.A0 + 1;
    for (int x = threadIdx.x; x < nh + 1; x += blockDim.x) s_hist[x] = 0;
    __syncthreads();
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < F.n_reads) {
        dmx_result out;
        out.bin1 = -1;
        out.bin2 = -1;
        out.rc1 = out.rc2 = 0;
        out.flags = 0;
        out._pad = 0;
        out.m1 = dmx_match{0, 0, 0, 0, 0, 0};
        out.m2 = out.m1;
        const uint64_t key = F.winner[r];
        if (key != ~0ull) {
            int a, o;
            const uint32_t n = F.lens[r];
            decode_match(key, F.origin[r], n, F.p0, out.m1, a, o);
            out.bin1 = (int16_t)a;
            out.rc1 = (uint8_t)o;
            if (F.mode == DMX_MODE_TWO_ROUND) {
                ItemView v;
                v.read = r;
                v.strand = (uint8_t)o;
                v.pad = 0;
                v.only_adapter = -1;
                if (F.p0->ad[a].where == kFront) {
                    v.start = (uint32_t)out.m1.rstop;
                    v.len = n - (uint32_t)out.m1.rstop;
                } else {
                    v.start = 0;
                    v.len = (uint32_t)out.m1.rstart;
                }
                const uint32_t idx = atomicAdd(F.n_items, 1u);
                F.items[idx] = v;
            } else {
                atomicAdd(&s_hist[a + 1], 1u);
            }
            if (o) atomicAdd(&s_hist[nh], 1u);
        } else {
            atomicAdd(&s_hist[0], 1u);
        }
        F.res[r] = out;
    }
    __syncthreads();
    const int stride1 = F.mode == DMX_MODE_TWO_ROUND ? F.A1 + 1 : 1;
    const int ncounts = (F.A0 + 1) * stride1;
    for (int x = threadIdx.x; x < nh + 1; x += blockDim.x) {
        const unsigned int v = s_hist[x];
        if (!v) continue;
        if (x == nh) atomicAdd(&F.counts[ncounts], (unsigned long long)v);
        else atomicAdd(&F.counts[x * stride1], (unsigned long long)v);
    }
}

// Round 1 epilogue (one thread per queued item): m2/bin2 and the (bin1, bin2) histogram.
__global__ __launch_bounds__(256) void finalize1_kernel(FinalArgs F) {
    extern __shared__ unsigned int s_hist2[];
    const int nbins = (F.A0 + 1) * (F.A1 + 1);
    for (int x = threadIdx.x; x < nbins + 1; x += blockDim.x) s_hist2[x] = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < *F.n_items) {
        const ItemView v = F.items[i];
        dmx_result& out = F.res[v.read];
        const uint64_t key = F.winner[i];
        int b = -1;
        if (key != ~0ull) {
            int a, o;
            decode_match(key, F.origin[i], v.len, F.p1, out.m2, a, o);
            out.bin2 = (int16_t)a;
            out.rc2 = (uint8_t)o;
            b = a;
            if (o) atomicAdd(&s_hist2[nbins], 1u);
        }
        atomicAdd(&s_hist2[(out.bin1 + 1) * (F.A1 + 1) + (b + 1)], 1u);
    }
    __syncthreads();
    for (int x = threadIdx.x; x < nbins + 1; x += blockDim.x) {
        const unsigned int c = s_hist2[x];
        if (c) atomicAdd(&F.counts[x == nbins ? nbins + 1 : x], (unsigned long long)c);
    }
}

// ---------------------------------------------------------------------------------------------
// host-side launch sequence
// ---------------------------------------------------------------------------------------------
static int resolve_grid(const Ctx* c) {
    (void)c;
    return 256 * 8;   // grid-stride; one 64-lane block per CU is LDS-limited (ring)
}

int launch_round(Ctx* c, int round, hipStream_t st) {
    RoundArgs R;
    R.seq = c->d_seq;
    R.nmask = c->d_nmask;
    R.offs = c->d_offs;
    R.lens = c->d_lens;
    R.panel = c->d_panel[round];
    const HostPanel& hp = c->panel[round];
    const bool linked = c->mode == DMX_MODE_LINKED;
    R.per_task_slot = (linked && round == 0) ? 1 : 0;
    if (round == 0) {
        R.items = nullptr;
        R.n_items_dev = nullptr;
        R.n_items = (uint32_t)c->n_reads;
        R.T = linked ? hp.n : hp.n * hp.n_orient;
    } else {
        R.items = c->d_items;
        R.n_items_dev = c->d_counters + 2;
        R.n_items = (uint32_t)c->item_cap;
        R.T = linked ? 1 : hp.n * hp.n_orient;
    }
    R.cl = c->d_cl[round];
    R.outc = c->d_outc[round];
    R.cl_count = c->d_counters + round;
    R.cl_cap = (uint32_t)c->cl_cap;
    R.flags = c->d_counters + 3;
    R.winner = c->d_winner[round];
    R.origin = c->d_origin[round];
    if (R.T > kScanBlock) return DMX_E_UNSUPPORTED;

    const uint32_t rpb = kScanBlock / R.T;
    const uint32_t grid = (uint32_t)((R.n_items + rpb - 1) / rpb);
    hipEventRecord(c->ev[round * 3 + 0], st);
    if (grid > 0) hipLaunchKernelGGL(scan_kernel, dim3(grid), dim3(kScanBlock), 0, st, R);
    hipEventRecord(c->ev[round * 3 + 1], st);
    hipLaunchKernelGGL(resolve_kernel, dim3(resolve_grid(c)), dim3(kResolveBlock), 0, st, R);
    hipLaunchKernelGGL(select_kernel, dim3(1024), dim3(256), 0, st, R);
    hipEventRecord(c->ev[round * 3 + 2], st);
    return hipGetLastError() == hipSuccess ? DMX_OK : DMX_E_HIP;
}

int launch_finalize(Ctx* c, int round, hipStream_t st) {
    FinalArgs F;
    F.lens = c->d_lens;
    F.p0 = c->d_panel[0];
    F.p1 = c->d_panel[1];
    F.winner = c->d_winner[round];
    F.origin = c->d_origin[round];
    F.res = c->d_res;
    F.items = c->d_items;
    F.n_items = c->d_counters + 2;
    F.n_reads = (uint32_t)c->n_reads;
    F.mode = c->mode;
    F.A0 = c->panel[0].n;
    F.A1 = c->mode == DMX_MODE_SINGLE ? 0 : c->panel[1].n;
    F.counts = c->d_counts;
    if (round == 0) {
        const uint32_t grid = (uint32_t)((c->n_reads + 255) / 256);
        if (grid) hipLaunchKernelGGL(finalize0_kernel, dim3(grid), dim3(256), 0, st, F);
    } else {
        const uint32_t grid = (uint32_t)((c->item_cap + 255) / 256);
        const size_t shm = sizeof(unsigned int) * ((size_t)(F.A0 + 1) * (F.A1 + 1) + 1);
        if (grid) hipLaunchKernelGGL(finalize1_kernel, dim3(grid), dim3(256), shm, st, F);
    }
    hipEventRecord(c->ev[6 + round], st);
    return hipGetLastError() == hipSuccess ? DMX_OK : DMX_E_HIP;
}

}  // namespace dmx
