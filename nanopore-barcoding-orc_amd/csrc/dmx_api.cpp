// dmx_api.cpp — C-ABI of libdmx (include/dmx.h): context, panels, packing, batch execution.
//
// Panel rules restate cutadapt 4.9 adapter construction (parser.py / adapters.py, not vendored
// in /root/reference): name/sequence come from the FASTA, sequences are
// uppercase with U->T, adapter wildcards are enabled iff a non-ACGT character is present,
// k = int(max_error_rate * m), acceptance `cost <= effective_length * max_error_rate` in IEEE
// double with effective length excluding adapter N's, minimum overlap -O (default 3).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <utility>
#include <vector>

#include "dmx_internal.h"
#include "pack.h"

using namespace dmx;

#define CK(call)                                                                        \
    do {                                                                                \
        hipError_t e_ = (call);                                                         \
        if (e_ != hipSuccess) {                                                         \
            c->err = std::string(#call) + ": " + hipGetErrorString(e_);                 \
            return DMX_E_HIP;                                                           \
        }                                                                               \
    } while (0)

namespace {

constexpr int kMinFilterLen = 10; // shortest shared suffix worth a filter pass
// kGuardWords (dmx_device.h): zeroed words before/after the packed device buffers

uint8_t iupac_mask(char ch) {
    switch (ch) {
        case 'A': return 1;
        case 'C': return 2;
        case 'G': return 4;
        case 'T': return 8;
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

template <typename T>
int dev_alloc(Ctx* c, T** p, size_t count) {
    if (*p) {
        hipFree(*p);
        *p = nullptr;
    }
    if (count == 0) count = 1;
    CK(hipMalloc((void**)p, count * sizeof(T)));
    return DMX_OK;
}


// (A0+1)(A1+1) per-bin counts + 2 RC counts (include/dmx.h dmx_counts)
size_t counts_size(const Ctx* c) {
    const size_t a1 = c->mode == DMX_MODE_SINGLE ? 0 : (size_t)c->panel[1].n;
    return ((size_t)c->panel[0].n + 1) * (a1 + 1) + 2;
}

int ensure_pipeline(Ctx* c) {
    const size_t n = c->n_reads;
    const bool linked = c->mode == DMX_MODE_LINKED;
    const size_t slots0 = linked ? n * (size_t)std::max(1, c->panel[0].n) : n;
    const size_t items = linked ? slots0 : n;
    // non-linked rounds may need one winner slot per (item, orientation): see orient_slot
    const size_t need = std::max(slots0, items) * (linked ? 1 : 2);
    if (!c->d_res || c->res_cap < n) {   // the resident input set's result array
        int rc;
        if ((rc = dev_alloc(c, &c->d_res, n))) return rc;
        c->res_cap = n;
    }
    if (c->slot_cap < need || c->cap_reads < n) {
        const size_t s = need;
        int rc;
        for (int r = 0; r < 2; ++r) {
            if ((rc = dev_alloc(c, &c->d_winner[r], s))) return rc;
            if ((rc = dev_alloc(c, &c->d_origin[r], s))) return rc;
            if ((rc = dev_alloc(c, &c->d_lb[r], s))) return rc;
        }
        if ((rc = dev_alloc(c, &c->d_linked, n))) return rc;
        c->slot_cap = s;
        c->cap_reads = n;
    }
    // The item list has its own capacity: a linked batch needs reads x pairs items, which can
    // exceed what an earlier two-round batch allocated (reads) while its winner slots (2 x
    // reads) still suffice.  Sizing it only with the slots let finalize0_linked write past
    // d_items (an illegal memory access in a parity sweep that ran a two-round case, then a
    // linked one of fewer reads, on one context).
    if (c->item_alloc < items) {
        int rc;
        if ((rc = dev_alloc(c, &c->d_items, items))) return rc;
        c->item_alloc = items;
    }
    c->item_cap = items;
    const size_t want_cl = 4 * std::max(slots0, n) + 65536;
    if (c->cl_cap < want_cl) {
        int rc;
        for (int r = 0; r < 2; ++r) {
            if ((rc = dev_alloc(c, &c->d_cl[r], want_cl))) return rc;
            if ((rc = dev_alloc(c, &c->d_outc[r], want_cl))) return rc;
        }
        c->cl_cap = want_cl;
    }
    const size_t want_cand = 4 * std::max(slots0, n) + 65536;
    if (c->cand_cap < want_cand) {
        int rc;
        for (int r = 0; r < 2; ++r)
            for (int l = 0; l < 2; ++l) {
                if ((rc = dev_alloc(c, &c->d_cand[r][l], want_cand))) return rc;
                if ((rc = dev_alloc(c, &c->d_cand_out[r][l], want_cand))) return rc;
            }
        c->cand_cap = want_cand;
    }
    const size_t want_win = 4 * 2 * std::max(slots0, n) + 65536;
    if (c->win_cap < want_win) {
        int rc;
        if ((rc = dev_alloc(c, &c->d_win, want_win))) return rc;
        if ((rc = dev_alloc(c, &c->d_win2, want_win))) return rc;
        if ((rc = dev_alloc(c, &c->d_tasks, 4 * want_win))) return rc;
        if ((rc = dev_alloc(c, &c->d_ftask, want_win))) return rc;
        c->win_cap = want_win;
        c->task_cap = 4 * want_win;
        c->ftask_cap = want_win;
    }
    // window code slots: verified windows are about one per view and round; later ones gather
    const size_t want_stage = std::min<size_t>(c->win_cap, 2 * std::max(slots0, n) + 65536);
    if (c->use_stage && c->stage_cap < want_stage) {
        int rc;
        if ((rc = dev_alloc(c, &c->d_stage, want_stage * kStageWords))) return rc;
        c->stage_cap = want_stage;
    }
    const size_t nc = counts_size(c);
    if (c->n_counts != nc) {
        int rc;
        if ((rc = dev_alloc(c, &c->d_counts, nc))) return rc;
        c->n_counts = nc;
    }
    return DMX_OK;
}

// The pipeline counters (dmx_internal.h) with the sharded lists' totals (records kept, over
// every shard) folded into their old slots: cnt[4 + r] windows, cnt[10 + r] verified windows,
// cnt[12 + r] screen tasks, cnt[6 + 2r + l] candidates.  *ovf: flag bits of overflowed lists
// (4 windows / tasks, 8 candidates).
hipError_t read_counters(Ctx* c, uint32_t* cnt, int* ovf) {
    hipError_t e = hipMemcpy(cnt, c->d_counters, 32 * sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    std::vector<uint32_t> sh((size_t)kShLists * kShards * kShardStride);
    e = hipMemcpy(sh.data(), c->d_shard, sh.size() * sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return e;
    int o = 0;
    for (int x = 0; x < kShLists; ++x) {
        const bool cand = x >= kShCand && x < kShFtask;
        const uint32_t scap = (uint32_t)((cand ? c->cand_cap : x >= kShFtask ? c->ftask_cap
                                          : x >= kShTasks ? c->task_cap : c->win_cap) /
                                         kShards);
        uint64_t t = 0;
        for (int s = 0; s < kShards; ++s) {
            const uint32_t v = sh[(size_t)(x * kShards + s) * kShardStride];
            t += std::min(v, scap);
            if (v > scap) o |= cand ? 8 : 4;
        }
        const int slot = x < kShWin2 ? 4 + x : x < kShTasks ? 10 + (x - kShWin2)
                       : x < kShCand ? 12 + (x - kShTasks) : x < kShFtask ? 6 + (x - kShCand)
                       : 14 + (x - kShFtask);
        cnt[slot] = (uint32_t)t;
    }
    if (ovf) *ovf = o;
    return hipSuccess;
}

int grow_cands(Ctx* c) {
    const size_t want = c->cand_cap * 2;
    int rc;
    for (int r = 0; r < 2; ++r)
        for (int l = 0; l < 2; ++l) {
            if ((rc = dev_alloc(c, &c->d_cand[r][l], want))) return rc;
            if ((rc = dev_alloc(c, &c->d_cand_out[r][l], want))) return rc;
        }
    c->cand_cap = want;
    return DMX_OK;
}

int grow_windows(Ctx* c) {
    const size_t want = c->win_cap * 2;
    int rc;
    if ((rc = dev_alloc(c, &c->d_win, want))) return rc;
    if ((rc = dev_alloc(c, &c->d_win2, want))) return rc;
    if ((rc = dev_alloc(c, &c->d_tasks, 4 * want))) return rc;
    if ((rc = dev_alloc(c, &c->d_ftask, want))) return rc;
    c->win_cap = want;
    c->task_cap = 4 * want;
    c->ftask_cap = want;
    return DMX_OK;
}

int grow_clusters(Ctx* c) {
    const size_t want = c->cl_cap * 2;
    int rc;
    for (int r = 0; r < 2; ++r) {
        if ((rc = dev_alloc(c, &c->d_cl[r], want))) return rc;
        if ((rc = dev_alloc(c, &c->d_outc[r], want))) return rc;
    }
    c->cl_cap = want;
    return DMX_OK;
}

}  // namespace

namespace dmx {

namespace {
std::mutex g_proc_err_mu;
std::string g_proc_err;
}  // namespace

void set_process_error(const std::string& msg) {
    std::lock_guard<std::mutex> lk(g_proc_err_mu);
    g_proc_err = msg;
}

std::string process_error() {
    std::lock_guard<std::mutex> lk(g_proc_err_mu);
    return g_proc_err;
}

// The kernels' reach around a view, per panel.  A 16-position gather at view
// position p physically loads two aligned u32 words, i.e. view positions [p - 16, p + 32) on
// either strand; whole-block loads (ViewBlocks: filter, verify) cover [p - 63, p + 64 s + 127]
// for s 64-position stretches from p.  Per kernel, the first gather position before the view:
//   filter, verify, window scan, scan, resolve, chop: >= 0 (their ranges start at column 0);
//   index screen: x1 - 15 >= -(m_max - pre_len) - kf - 15 (the I_a band's warm-up, both the
//     last-row test and the 3' last-column test; D' only lowers D there);
//   edge bands: dx - H >= -(m + 7) (end cell (i, j) with j >= 0, H <= 7 diagonals);
// and past the view end: ViewBlocks' in-flight block (<= 190 nt), fetch16 prefetches (<= 54).
// Positions before -kViewReachPre are read at -kViewReachPre (fetch16s).  A read on strand 1
// maps view positions past its end to nt before its offset, and positions before the view to
// nt past its end, so both directions must fit either side of the buffer.
PanelReach panel_reach(const HostPanel& hp, const DevPanel& dp) {
    int m_max = 0;
    bool band = true;
    for (int a = 0; a < hp.n; ++a) {
        m_max = std::max(m_max, (int)hp.ad[a].m);
        band &= hp.ad[a].kk <= 7;
    }
    PanelReach r;
    int pre = 63 + 16;   // ViewBlocks' floor to a block, fetch16's floor to a word
    if (hp.screen) pre = std::max(pre, m_max - dp.pre_len + dp.kf + 15 + 16);
    if (band) pre = std::max(pre, m_max + 7 + 16);
    r.pre_raw = pre;
    r.pre = std::min(pre, std::max(63 + 16, kViewReachPre + 16));
    r.post = 63 + 64 + 63;   // ViewBlocks: the block after the last stretch's two, in flight
    // strand 0: before the view -> before the offset; strand 1: before the view -> past the end
    r.need_pre = std::max(r.pre, r.post) - kMinOffset;
    r.need_post = std::max(r.pre, r.post) + 32 - kMinTail;   // (+ the 8-byte word pair)
    return r;
}

int reset_counts(Ctx* c) {
    CK(hipSetDevice(c->device));
    const size_t nc = counts_size(c);
    if (c->n_counts != nc || !c->d_counts) {
        int rc;
        if ((rc = dev_alloc(c, &c->d_counts, nc))) return rc;
        c->n_counts = nc;
    }
    CK(hipMemsetAsync(c->d_counts, 0, nc * sizeof(unsigned long long), c->stream));
    CK(hipStreamSynchronize(c->stream));
    c->counts_reduced = false;
    return DMX_OK;
}

}  // namespace dmx


extern "C" {

int dmx_abi_version(void) { return DMX_ABI_VERSION; }

int dmx_open(int device, dmx_ctx** out) {
    if (!out) return DMX_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return DMX_E_HIP;
    dmx_ctx* c = new dmx_ctx();
    c->device = device;
    const char* nf = std::getenv("DMX_NO_FILTER");
    c->no_filter = nf && nf[0] == '1';
    const char* nv = std::getenv("DMX_NO_VERIFY");
    c->no_verify = nv && nv[0] == '1';
    const char* np = std::getenv("DMX_NO_PIECES");   // A/B: the full filter pass
    c->no_pieces = np && np[0] == '1';
    const char* rs = std::getenv("DMX_RESOLVE");
    c->force_ring = rs && std::strcmp(rs, "ring") == 0;
    const char* stg = std::getenv("DMX_STAGE");   // A/B: window code slots
    c->use_stage = DMX_STAGE_SLOTS && stg && stg[0] == '1';
    const char* ns = std::getenv("DMX_NO_SCREEN");   // A/B: no index screen before the
    c->no_screen = ns && ns[0] == '1';               // window scan
    const char* s1 = std::getenv("DMX_SCREEN_V1");   // A/B: the unpacked index screen
    c->screen_v1 = s1 && s1[0] == '1';
    if (hipSetDevice(device) != hipSuccess ||
        hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return DMX_E_HIP;
    }
    for (auto& e : c->ev) hipEventCreate(&e);
    for (int r = 0; r < 2; ++r) {
        hipMalloc((void**)&c->d_panel[r], sizeof(DevPanel));
        hipMalloc((void**)&c->d_pieces[r], sizeof(DevPieces));
    }
    hipMalloc((void**)&c->d_counters, 32 * sizeof(uint32_t));
    hipMalloc((void**)&c->d_shard, kShLists * kShards * kShardStride * sizeof(uint32_t));
    *out = c;
    return DMX_OK;
}

void dmx_close(dmx_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    chop_release(c);
    comm_release(c);
    void* bufs[] = {c->d_seq_alloc, c->d_nmask_alloc,     c->d_offs,     c->d_lens,      c->d_res,
                    c->d_winner[0], c->d_winner[1], c->d_origin[0], c->d_origin[1], c->d_lb[0], c->d_lb[1], c->d_cl[0],
                    c->d_cl[1],     c->d_outc[0],   c->d_outc[1],  c->d_items, c->d_win, c->d_win2, c->d_linked, c->d_tasks, c->d_counters, c->d_shard,
                    c->d_counts,    c->d_panel[0],  c->d_panel[1], c->d_pieces[0], c->d_pieces[1],
                    c->d_ftask, c->d_stage, c->d_pieces_flat, c->d_cells[0], c->d_cells[1], c->d_cells[2],
                    c->d_cells[3]};
    for (void* b : bufs)
        if (b) hipFree(b);
    for (int r = 0; r < 2; ++r)
        for (int l = 0; l < 2; ++l) {
            if (c->d_cand[r][l]) hipFree(c->d_cand[r][l]);
            if (c->d_cand_out[r][l]) hipFree(c->d_cand_out[r][l]);
        }
    void* alt[] = {c->alt.seq_alloc, c->alt.nmask_alloc, c->alt.offs, c->alt.lens, c->alt.res,
                   c->alt.exc, c->d_exc};
    for (void* b : alt)
        if (b) hipFree(b);
    for (auto& e : c->ev)
        if (e) hipEventDestroy(e);
    if (c->cstream) hipStreamDestroy(c->cstream);
    if (c->dstream) hipStreamDestroy(c->dstream);
    hipStreamDestroy(c->stream);
    delete c;
}

const char* dmx_last_error(dmx_ctx* c) {
    if (c) return c->err.c_str();
    // no context: the last context-free failure (thread-local copy: the pointer stays valid
    // until this thread's next call)
    thread_local std::string msg;
    msg = dmx::process_error();
    if (msg.empty()) msg = "null context";
    return msg.c_str();
}

int dmx_set_mode(dmx_ctx* c, int mode) {
    if (!c) return DMX_E_INVALID;
    if (mode != DMX_MODE_SINGLE && mode != DMX_MODE_TWO_ROUND && mode != DMX_MODE_LINKED) {
        c->err = "unknown mode";
        return DMX_E_INVALID;
    }
    c->mode = mode;
    ++c->panel_gen;
    return DMX_OK;
}

static int set_panel_impl(dmx_ctx* c, int round, const char* const* seqs, const int* lens,
                          const int* wheres, int n, double max_errors, int min_overlap,
                          int flags);

int dmx_set_panel(dmx_ctx* c, int round, const char* const* seqs, const int* lens, int n,
                  double max_errors, int min_overlap, int flags) {
    return set_panel_impl(c, round, seqs, lens, nullptr, n, max_errors, min_overlap, flags);
}

int dmx_set_panel_mixed(dmx_ctx* c, int round, const char* const* seqs, const int* lens,
                        const int* wheres, int n, double max_errors, int min_overlap, int rc) {
    if (!wheres) return DMX_E_INVALID;
    for (int a = 0; a < n; ++a)
        if (wheres[a] != DMX_FRONT && wheres[a] != DMX_BACK) return DMX_E_INVALID;
    return set_panel_impl(c, round, seqs, lens, wheres, n, max_errors, min_overlap,
                          DMX_FRONT | (rc ? DMX_RC : 0));
}

// Piece screen tables (dmx_device.h DevPieces).  Adapter a of an ACGT panel
// with K_a = acc[m_a] >= 0 (the largest accepted cost of an alignment covering all m_a rows) is
// cut into K_a + 1 disjoint row pieces of near-equal length (at most 16 nt each: a piece may be
// any sub-range of its rows).  An accepted full alignment has <= K_a edits, so some piece is
// aligned without one: an exact copy in the read, after which the alignment ends within
// (m_a - r1) +- K_a columns (r1 = the piece's end row).  Pieces are deduplicated per
// (codes, length, orientation) with the union of their end ranges; every piece contributes its
// 8-mers at offsets 0 .. s-1 (s = the sampling stride), so a copy starting anywhere has one of
// them at a sampled position.  Off (piece_step 0) for IUPAC panels, pieces shorter than 8 nt,
// tables that do not fit, or DMX_NO_PIECES=1.
static void build_pieces(const Ctx* c, const char* const* seqs, const int* lens, int n,
                         HostPanel& hp) {
    hp.piece_step = 0;
    DevPieces& Q = hp.pieces;
    memset(&Q, 0, sizeof(Q));
    if (!hp.filter || c->no_pieces) return;
    struct Pc {
        uint32_t val;
        int len, o, dlo, dhi;
    };
    std::vector<Pc> pcs;
    auto code = [](char ch) -> int {
        switch (ch) {
            case 'A': return 0;
            case 'C': return 1;
            case 'G': return 2;
            case 'T': return 3;
            default: return -1;
        }
    };
    int minlen = 64;
    for (int a = 0; a < n; ++a) {
        const int m = lens[a];
        for (int i = 0; i < m; ++i)
            if (code(seqs[a][i]) < 0) return;   // IUPAC adapter: the full filter pass
        const int K = hp.ad[a].acc[m];
        if (K < 0) continue;                    // never accepted with every row aligned
        const int np = K + 1;
        if (m / np < kPieceK) return;
        for (int p = 0; p < np; ++p) {
            const int r0 = p * m / np, r1 = (p + 1) * m / np;
            const int len = std::min(16, r1 - r0), re = r0 + len;
            minlen = std::min(minlen, len);
            for (int o = 0; o < hp.n_orient; ++o) {
                uint32_t v = 0;
                for (int i = 0; i < len; ++i) {
                    // orientation 1: the reverse complement, as it appears in the view-0 codes
                    const int cd = o == 0 ? code(seqs[a][r0 + i]) : 3 - code(seqs[a][re - 1 - i]);
                    v |= (uint32_t)cd << (2 * i);
                }
                pcs.push_back({v, len, o, (m - re) - K, (m - re) + K});
            }
        }
    }
    // dedup by (codes, length, orientation), union of the end ranges
    std::sort(pcs.begin(), pcs.end(), [](const Pc& x, const Pc& y) {
        return std::make_tuple(x.val, x.len, x.o) < std::make_tuple(y.val, y.len, y.o);
    });
    std::vector<Pc> uq;
    for (const Pc& p : pcs) {
        if (!uq.empty() && uq.back().val == p.val && uq.back().len == p.len && uq.back().o == p.o) {
            uq.back().dlo = std::min(uq.back().dlo, p.dlo);
            uq.back().dhi = std::max(uq.back().dhi, p.dhi);
        } else {
            uq.push_back(p);
        }
    }
    if (uq.empty() || (int)uq.size() > kMaxPieceEntries) return;
    int step = minlen - kPieceK + 1 >= 4 ? 4 : (minlen - kPieceK + 1 >= 2 ? 2 : 1);
    if (const char* e = std::getenv("DMX_PIECE_STEP"))   // A/B: a denser sampling
        step = std::min(step, std::max(1, std::atoi(e)));
    while (step > 1 && (int)uq.size() * step > kMaxPieceEntries) step /= 2;
    if ((int)uq.size() * step > kMaxPieceEntries) return;
    // Sampled offsets: any `step` consecutive offsets j0 .. j0+step-1 of a piece cover every copy
    // (one of its 8-mers sits at a sampled position).  Per piece take the window whose 8-mers the
    // fewest other pieces share (pieces of different adapters that overlap a shared constant
    // block share 8-mers, and every entry of a key is checked on each sampled hit of it).  The
    // offset is a 2-bit field that both screens read the copy back with (the flat scan holds the
    // codes of nt [X - 3, X + 29) per sampled nt X), so the window ends at offset kPieceMaxOff.
    std::map<uint32_t, int> mult;
    for (const Pc& x : uq)
        for (int off = 0; off + kPieceK <= x.len; ++off) ++mult[(x.val >> (2 * off)) & 0xFFFFu];
    std::vector<std::pair<uint32_t, uint64_t>> ents;   // (8-mer, entry)
    int lo_off = 1 << 20, dlo_min = 0, len_max = 0, dhi_max = 0;
    bool any1 = false;
    for (const Pc& x : uq) {
        int best = 0, bcost = 1 << 30;
        for (int j0 = 0; j0 + step - 1 <= kPieceMaxOff && j0 + step - 1 + kPieceK <= x.len; ++j0) {
            int cost = 0;
            for (int off = j0; off < j0 + step; ++off) cost += mult[(x.val >> (2 * off)) & 0xFFFFu];
            if (cost < bcost) bcost = cost, best = j0;
        }
        for (int off = best; off < best + step; ++off)
            ents.push_back({(x.val >> (2 * off)) & 0xFFFFu,
                            piece_entry(x.val, x.len, x.o, off, x.dlo, x.dhi)});
        if (x.o == 0) {
            lo_off = std::min(lo_off, x.len + x.dlo - 1);
        } else {
            dlo_min = any1 ? std::min(dlo_min, x.dlo) : x.dlo;
            any1 = true;
        }
        len_max = std::max(len_max, x.len);
        dhi_max = std::max(dhi_max, x.dhi);
    }
    std::sort(ents.begin(), ents.end());
    int nk = 0;
    for (size_t e = 0; e < ents.size(); ++e) {
        if (e == 0 || ents[e].first != ents[e - 1].first) {
            Q.key[nk++] = (uint32_t)e;
            Q.bitmap[ents[e].first >> 5] |= 1u << (ents[e].first & 31);
        }
        Q.key[nk - 1] += 1u << 16;
        Q.entry[e] = ents[e].second;
    }
    for (int w = 0, r = 0; w < kPieceBitmapWords; ++w) {
        Q.rank_base[w] = (uint16_t)r;
        r += __builtin_popcount(Q.bitmap[w]);
    }
    int reach = 0;   // FRONT: alignments entering at column 0 (rows skipped) end before it
    if (hp.ad[0].where == kFront)
        for (int a = 0; a < n; ++a)
            for (int L = 1; L <= (int)hp.ad[a].m; ++L)
                if (hp.ad[a].acc[L] >= 0) reach = std::max(reach, L + (int)hp.ad[a].acc[L]);
    // every cell a part can mark lies within 64 cells of its mask base (pscreen_kernel)
    int pmax = (992 - std::max(len_max + dhi_max, dhi_max - dlo_min)) / 16 * 16;
    pmax = std::min(pmax, 768);
    if (const char* e = std::getenv("DMX_PIECE_PART"))   // A/B: positions per screen lane
        pmax = std::min(pmax, std::max(64, std::atoi(e) / 16 * 16));
    if (pmax < 64) return;
    Q.on = 1;
    Q.step = step;
    Q.n_pieces = (int)uq.size();
    Q.n_keys = nk;
    Q.n_entries = (int)ents.size();
    Q.front_reach = reach;
    Q.part_max = pmax;
    Q.lo_off = std::max(0, lo_off == (1 << 20) ? 0 : lo_off);
    Q.dlo_min = dlo_min;
    hp.piece_step = step;
}

// The host and device forms of a panel (parser.py / adapters.py rules above), the filter /
// verification / screen blocks and the reach check; uses only c->err, c->no_filter, c->no_verify
// (dmx_panel_reach runs it on a context that was never opened).
static int build_panel(Ctx* c, const char* const* seqs, const int* lens, const int* wheres, int n,
                       double max_errors, int min_overlap, int flags, HostPanel& hp,
                       DevPanel& dp) {
    if (!seqs || !lens) return DMX_E_INVALID;
    if (n <= 0 || n > kMaxAdapters) {
        c->err = "panel must hold 1..64 adapters";
        return DMX_E_INVALID;
    }
    if (!(flags & (DMX_FRONT | DMX_BACK)) || ((flags & DMX_FRONT) && (flags & DMX_BACK))) {
        c->err = "panel flags need exactly one of DMX_FRONT / DMX_BACK";
        return DMX_E_INVALID;
    }
    if (!(max_errors >= 0.0)) {
        c->err = "max_errors must be >= 0";
        return DMX_E_INVALID;
    }
    hp = HostPanel();
    hp.n = n;
    hp.n_orient = (flags & DMX_RC) ? 2 : 1;
    for (int a = 0; a < n; ++a) {
        const int m = lens[a];
        if (m <= 0 || m > kMaxLen) {
            c->err = "adapter length must be 1..64 (one 64-bit Myers word)";
            return DMX_E_UNSUPPORTED;
        }
        DevAdapter& ad = hp.ad[a];
        memset(&ad, 0, sizeof(ad));
        bool wild = false;
        for (int i = 0; i < m; ++i) {
            const char ch = seqs[a][i];
            if (!iupac_mask(ch)) {
                c->err = std::string("adapter character not IUPAC uppercase: ") + ch;
                return DMX_E_INVALID;
            }
            if (ch != 'A' && ch != 'C' && ch != 'G' && ch != 'T') wild = true;
        }
        const double rate = max_errors >= 1.0 ? max_errors / (double)m : max_errors;
        const int k = (int)(rate * m);
        if (m + k + 2 + 4 > kRingSmall) hp.ring_small = false;
        if (m + k + 2 + 4 > kRingLarge) {
            c->err = "error rate too high for the resolve window (m + k + 6 > 128)";
            return DMX_E_UNSUPPORTED;
        }
        int ncount[kMaxLen + 1];
        int nc = 0;
        for (int i = 0; i < m; ++i) {
            ncount[i] = nc;
            if (seqs[a][i] == 'N') ++nc;
        }
        ncount[m] = nc;
        const int eff_len = wild ? m - nc : m;
        if (eff_len == 0) {
            c->err = "adapter consists only of N wildcards";
            return DMX_E_INVALID;
        }
        for (int i = 0; i < m; ++i) {
            // Adapter wildcards: IUPAC mask vs read base; otherwise ASCII equality. Read codes
            // 4..7 (any non-ACGT byte) match nothing in either mode.
            const uint8_t mask = wild ? iupac_mask(seqs[a][i]) : iupac_mask(seqs[a][i]);
            for (int code = 0; code < 4; ++code)
                if (mask & (1u << code)) ad.peq[code] |= 1ull << i;
        }
        int kk = -1;
        for (int L = 0; L < 72; ++L) {
            int allow = -1;
            if (L <= m && L >= min_overlap) {
                const int eff = wild ? (L < m ? L - ncount[L] : eff_len) : L;
                const double lim = (double)eff * rate;
                for (int cst = 0; cst <= 127 && (double)cst <= lim; ++cst) allow = cst;
            }
            ad.acc[L] = (int8_t)allow;
            kk = std::max(kk, allow);
            ad.pacc[L] = (int8_t)kk;
        }
        // score = aligned adapter length - 2 cost - (adapter chars facing a gap) >= L - 3 cost
        for (int L = 1; L < 72; ++L)
            if (ad.acc[L] >= 0 && L - 3 * (int)ad.acc[L] <= 0) hp.nonpos = true;
        ad.m = (uint8_t)m;
        ad.k = (uint8_t)k;
        ad.kk = (int8_t)std::min(kk, k);
        ad.where = wheres ? (wheres[a] == DMX_FRONT ? kFront : kBack)
                          : ((flags & DMX_FRONT) ? kFront : kBack);
    }
    hp.set = true;
    memset(&dp, 0, sizeof(dp));
    dp.n_adapters = hp.n;
    dp.n_orient = hp.n_orient;
    dp.where = hp.ad[0].where;
    for (int a = 1; a < n; ++a)
        if (hp.ad[a].where != hp.ad[0].where) dp.where = 0;
    // Shared-suffix filter block: the longest suffix common to every adapter (<= 32 chars).
    int common = lens[0];
    for (int a = 1; a < n; ++a) {
        int l = 0;
        while (l < common && l < lens[a] &&
               seqs[a][lens[a] - 1 - l] == seqs[0][lens[0] - 1 - l])
            ++l;
        common = l;
    }
    int flen = std::min(common, 32);
    if (const char* fm = std::getenv("DMX_FILTER_MAXLEN"))   // A/B: a shorter suffix block
        flen = std::min(flen, std::max(1, std::atoi(fm)));
    bool uniform = true;
    for (int a = 1; a < n; ++a) uniform &= hp.ad[a].where == hp.ad[0].where;
    int kf_all = -1;
    for (int a = 0; a < n; ++a) kf_all = std::max(kf_all, (int)hp.ad[a].kk);
    // The filter's first 64 columns per segment carry per-column thresholds: the warm-up
    // W = flen + kf and the near-start acceptance pf[j + kf] < kf must both end within them.
    int8_t pf_all[72];
    for (int L = 0; L < 72; ++L) {
        pf_all[L] = -1;
        for (int a = 0; a < n; ++a) pf_all[L] = std::max(pf_all[L], hp.ad[a].pacc[L]);
    }
    const int kf_far = std::min(kf_all, (int)pf_all[71]);
    bool near_ok = true;
    for (int j = 65; j + kf_all < 71; ++j) near_ok &= pf_all[j + kf_all] >= kf_far;
    hp.filter = uniform && flen >= kMinFilterLen && flen + kf_all <= 64 && near_ok &&
                !(c->no_filter);
    if (hp.filter) {
        dp.filter_len = flen;
        int slen = flen;
        if (const char* fs = std::getenv("DMX_FILTER_SCANLEN"))   // A/B: scan a shorter suffix
            slen = std::min(flen, std::max(kMinFilterLen, std::atoi(fs)));
        dp.scan_len = slen;
        // the scanned rows in the top slen bits (last row = bit 31); the rows below match
        // every code, N included, so they stay at cost 0 like row 0 (filter_kernel)
        const int pad = 32 - slen;
        for (int code = 0; code < 8; ++code)
            dp.filter_peq[code] = pad > 0 ? (1u << pad) - 1u : 0u;
        const char* blk = seqs[0] + lens[0] - slen;
        for (int i = 0; i < slen; ++i) {
            const uint8_t mask = iupac_mask(blk[i]);
            for (int code = 0; code < 4; ++code)
                if (mask & (1u << code)) dp.filter_peq[code] |= 1u << (pad + i);
        }
        int kf = -1, mk = 0;
        for (int L = 0; L < 72; ++L) dp.pf[L] = -1;
        for (int a = 0; a < n; ++a) {
            kf = std::max(kf, (int)hp.ad[a].kk);
            mk = std::max(mk, (int)hp.ad[a].m + (int)hp.ad[a].k + 1);
            for (int L = 0; L < 72; ++L) dp.pf[L] = std::max(dp.pf[L], hp.ad[a].pacc[L]);
        }
        dp.kf = kf;
        dp.max_mk = mk;
        // clean flags: the exact stages read a window's view from j1 - (m + k
        // + 1) (window scan) and j1 - (m + 7) (band DP); off when that exceeds 128 positions
        int reach = 0;
        for (int a = 0; a < n; ++a)
            reach = std::max(reach, (int)hp.ad[a].m + std::max((int)hp.ad[a].k + 1, 7));
        reach = (reach + 15) / 16 * 16;
        dp.clean_reach = reach <= 128 && !std::getenv("DMX_NO_CLEAN") ? reach : 0;

        // shared prefix for the verification pass
        int pre = lens[0];
        int mmin = 1 << 30, mmax = 0;
        for (int a = 0; a < n; ++a) {
            int l = 0;
            while (l < pre && l < lens[a] && seqs[a][l] == seqs[0][l]) ++l;
            pre = l;
            mmin = std::min(mmin, lens[a]);
            mmax = std::max(mmax, lens[a]);
        }
        pre = std::min(pre, 32);
        if (pre >= kMinFilterLen && pre + flen <= mmin && !c->no_verify) {
            hp.verify = true;
            dp.pre_len = pre;
            dp.off_min = mmin - pre;
            dp.off_max = mmax - pre;
            dp.m_max = mmax;
            // index screen: every adapter's middle block I_a = rows [pre, m - flen) fits a
            // 32-bit word
            int lmin = 64, lmx = 0, js = 0;
            for (int a = 0; a < n; ++a) {
                lmin = std::min(lmin, lens[a] - pre - flen);
                lmx = std::max(lmx, lens[a] - pre - flen);
                js = std::max(js, lens[a] - pre + (int)hp.ad[a].kk);
            }
            hp.screen = lmin >= 1 && lmx <= 32;
            dp.jsplit = js;
            bool shared = true;   // rows <= pre: identical acceptance for every adapter
            for (int a = 1; a < n; ++a)
                for (int L = 0; L <= pre; ++L) shared &= hp.ad[a].acc[L] == hp.ad[0].acc[L];
            dp.pshared = shared ? 1 : 0;
            for (int i = 0; i < pre; ++i) {
                const uint8_t mask = iupac_mask(seqs[0][i]);
                for (int code = 0; code < 4; ++code)
                    if (mask & (1u << code)) dp.pre_peq[code] |= 1u << i;
            }
        }
    }
    // Every gather of every kernel must stay inside the device guard words for every offset the
    // loaders accept (>= kMinOffset nt, >= kMinTail nt before the end): the deepest warm-up
    // before a view (index screen, edge bands), clamped at -kViewReachPre, and the block loads
    // past it.  Adapters of <= 64 nt always fit; the check keeps it explicit.
    build_pieces(c, seqs, lens, n, hp);
    hp.reach = panel_reach(hp, dp);
    if (hp.reach.need_pre > kGuardNt || hp.reach.need_post > kGuardNt) {
        c->err = "panel: the kernels' reach around a view (" + std::to_string(hp.reach.pre) +
                 " nt before, " + std::to_string(hp.reach.post) +
                 " after) exceeds the device guard";
        return DMX_E_UNSUPPORTED;
    }
    for (int a = 0; a < n; ++a) dp.ad[a] = hp.ad[a];
    // window code slots: from m + k + 1 columns before a window's first hit
    // column (the window scan's restricted start), never below the band's own warm-up
    hp.pre_len = dp.pre_len;
    int mk = 0, m_max = 0;
    for (int a = 0; a < n; ++a) {
        mk = std::max(mk, (int)hp.ad[a].m + (int)hp.ad[a].k + 1);
        m_max = std::max(m_max, (int)hp.ad[a].m);
    }
    hp.stage_back = mk;
    hp.stage_lo = -std::min(kViewReachPre, m_max + 7);
    return DMX_OK;
}

static int set_panel_impl(dmx_ctx* c, int round, const char* const* seqs, const int* lens,
                          const int* wheres, int n, double max_errors, int min_overlap,
                          int flags) {
    if (!c || round < 0 || round > 1 || !seqs || !lens) return DMX_E_INVALID;
    HostPanel hp;
    DevPanel dp;
    const int brc = build_panel(c, seqs, lens, wheres, n, max_errors, min_overlap, flags, hp, dp);
    if (brc) return brc;
    c->panel[round] = hp;
    ++c->panel_gen;
    c->ring_small[round] = hp.ring_small;
    c->band_ok[round] = true;
    int kkmax = 0;
    for (int a = 0; a < n; ++a) {
        c->band_ok[round] &= hp.ad[a].kk <= 7;
        kkmax = std::max(kkmax, (int)hp.ad[a].kk);
    }
    c->band_wide[round] = kkmax > 5;   // list 1 (costs 4..kk): 11 diagonals cover kk <= 5
    CK(hipSetDevice(c->device));
    CK(hipMemcpy(c->d_panel[round], &dp, sizeof(dp), hipMemcpyHostToDevice));
    if (hp.piece_step)
        CK(hipMemcpy(c->d_pieces[round], &hp.pieces, sizeof(DevPieces), hipMemcpyHostToDevice));
    return DMX_OK;
}

size_t dmx_pack_words(uint64_t total_nt, size_t n_reads) {
    const uint64_t nt = 2 * (uint64_t)DMX_PACK_PAD + total_nt + (uint64_t)kPackAlign * n_reads;
    return (size_t)((nt + 31) / 32 * 2 + 4);
}

int dmx_pack(const uint8_t* ascii, const uint64_t* offsets, const uint32_t* lens, size_t n_reads,
             uint32_t* out_seq2b, uint32_t* out_nmask, uint64_t* out_offsets) {
    if ((n_reads && (!offsets || !lens)) || !out_seq2b || !out_nmask || !out_offsets)
        return DMX_E_INVALID;
    uint64_t g = DMX_PACK_PAD;
    uint64_t total = 0;
    for (size_t r = 0; r < n_reads; ++r) {
        out_offsets[r] = g;
        g += ((uint64_t)lens[r] + kPackAlign - 1) / kPackAlign * kPackAlign;
        total += lens[r];
    }
    if (!ascii && total) return DMX_E_INVALID;   // a batch of empty reads needs no text
    const size_t words = dmx_pack_words(total, n_reads);
    memset(out_seq2b, 0, words * sizeof(uint32_t));
    memset(out_nmask, 0, words * sizeof(uint32_t));
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const size_t nth = n_reads < 4096 ? 1 : hw;
    if (nth == 1) {
        pack_range(ascii, offsets, lens, 0, n_reads, out_offsets, out_seq2b, out_nmask);
    } else {
        std::vector<std::thread> th;
        const size_t per = (n_reads + nth - 1) / nth;
        for (size_t t = 0; t < nth; ++t) {
            const size_t lo = t * per, hi = std::min(n_reads, lo + per);
            if (lo >= hi) break;
            th.emplace_back(pack_range, ascii, offsets, lens, lo, hi, out_offsets, out_seq2b,
                            out_nmask);
        }
        for (auto& t : th) t.join();
    }
    return DMX_OK;
}

}  // extern "C"

namespace {

// Mask words [mw0, mw0 + nmw) of the caller's batch into the resident set's d_nmask on stream s:
// a copy of the dense bitmap, or zero-fill + a scatter of the exceptions in that range (sorted
// by index, so the range is one binary search).  The exceptions are staged in the set's d_exc.
int upload_mask(Ctx* c, const MaskSrc& m, size_t mw0, size_t nmw, hipStream_t s) {
    if (m.dense) {
        CK(hipMemcpyAsync(c->d_nmask, m.dense + mw0, nmw * 4, hipMemcpyHostToDevice, s));
        return DMX_OK;
    }
    CK(hipMemsetAsync(c->d_nmask, 0, nmw * 4, s));
    const uint32_t* lo = std::lower_bound(m.idx, m.idx + m.n, (uint32_t)mw0);
    const uint32_t* hi = std::lower_bound(lo, m.idx + m.n, (uint32_t)(mw0 + nmw));
    const size_t n = (size_t)(hi - lo), first = (size_t)(lo - m.idx);
    if (!n) return DMX_OK;
    if (c->exc_cap < n || !c->d_exc) {
        int rc;
        if ((rc = dev_alloc(c, &c->d_exc, 2 * n))) return rc;
        c->exc_cap = n;
    }
    CK(hipMemcpyAsync(c->d_exc, m.idx + first, n * 4, hipMemcpyHostToDevice, s));
    CK(hipMemcpyAsync(c->d_exc + n, m.val + first, n * 4, hipMemcpyHostToDevice, s));
    return launch_mask_scatter(c->d_nmask, c->d_exc, (uint32_t)n, (uint32_t)mw0, s);
}

int load_impl(dmx_ctx* c, const uint32_t* seq2b, const MaskSrc& mask, const uint64_t* offsets,
              const uint32_t* lens, size_t n_words, size_t n_reads) {
    if (n_reads >= (1ull << 31)) {
        c->err = "too many reads in one batch";
        return DMX_E_UNSUPPORTED;
    }
    for (size_t r = 0; r < n_reads; ++r) {
        if (offsets[r] < 16 || (offsets[r] + lens[r] + 64) > (uint64_t)n_words * 16 ||
            lens[r] >= (1u << 30)) {
            c->err = "read offsets/lengths do not fit the packed buffer (use dmx_pack)";
            return DMX_E_INVALID;
        }
    }
    CK(hipSetDevice(c->device));
    int rc;
    if (c->cap_words < n_words || !c->d_seq_alloc) {
        const size_t total = n_words + 2 * kGuardWords;
        if ((rc = dev_alloc(c, &c->d_seq_alloc, total))) return rc;
        if ((rc = dev_alloc(c, &c->d_nmask_alloc, total))) return rc;
        CK(hipMemsetAsync(c->d_seq_alloc, 0, total * 4, c->stream));
        CK(hipMemsetAsync(c->d_nmask_alloc, 0, total * 4, c->stream));
        c->d_seq = c->d_seq_alloc + kGuardWords;
        c->d_nmask = c->d_nmask_alloc + kGuardWords;
        c->cap_words = n_words;
    }
    // the mask has 1 bit per nt: only its first half (of n_words words) carries data
    const size_t nmw = std::min(n_words, (n_words + 1) / 2 + 2);
    if (c->d_seq_alloc && c->n_words > n_words)   // stale tail of a longer batch: guard zero
        CK(hipMemsetAsync(c->d_seq + n_words, 0, (c->n_words - n_words) * 4, c->stream));
    if (c->d_nmask_alloc && c->n_words > nmw)
        CK(hipMemsetAsync(c->d_nmask + nmw, 0, (std::min(c->n_words, c->cap_words) - nmw) * 4,
                          c->stream));
    if (!c->d_offs || c->in_cap_reads < n_reads) {
        if ((rc = dev_alloc(c, &c->d_offs, n_reads))) return rc;
        if ((rc = dev_alloc(c, &c->d_lens, n_reads))) return rc;
        c->in_cap_reads = n_reads;
    }
    c->n_reads = n_reads;
    c->n_words = n_words;
    CK(hipMemcpyAsync(c->d_seq, seq2b, n_words * 4, hipMemcpyHostToDevice, c->stream));
    if ((rc = upload_mask(c, mask, 0, nmw, c->stream))) return rc;
    if (n_reads) {
        CK(hipMemcpyAsync(c->d_offs, offsets, n_reads * 8, hipMemcpyHostToDevice, c->stream));
        CK(hipMemcpyAsync(c->d_lens, lens, n_reads * 4, hipMemcpyHostToDevice, c->stream));
    }
    CK(hipStreamSynchronize(c->stream));
    c->executed = false;
    c->chunked = false;
    chop_invalidate(c);
    return DMX_OK;
}

}  // namespace

extern "C" {

int dmx_load(dmx_ctx* c, const uint32_t* seq2b, const uint32_t* nmask, const uint64_t* offsets,
             const uint32_t* lens, size_t n_words, size_t n_reads) {
    if (!c || (n_reads && (!seq2b || !nmask || !offsets || !lens))) return DMX_E_INVALID;
    MaskSrc m;
    m.dense = nmask;
    return load_impl(c, seq2b, m, offsets, lens, n_words, n_reads);
}

int dmx_panel_pieces(const char* const* seqs, const int* lens, int n, double max_errors,
                     int min_overlap, int flags, int32_t* out, int n_out, uint64_t* entries,
                     int cap) {
    if (!out || n_out < 8) return DMX_E_INVALID;
    Ctx tmp;   // never opened: build_panel reads only the A/B switches dmx_open would set
    const char* np = std::getenv("DMX_NO_PIECES");
    tmp.no_pieces = np && np[0] == '1';
    HostPanel hp;
    DevPanel dp;
    const int rc = build_panel(&tmp, seqs, lens, nullptr, n, max_errors, min_overlap, flags, hp,
                               dp);
    for (int i = 0; i < n_out; ++i) out[i] = 0;
    if (rc != DMX_OK) return rc;
    const DevPieces& Q = hp.pieces;
    const int32_t v[8] = {hp.piece_step, Q.n_pieces, Q.n_keys, Q.n_entries, Q.front_reach,
                          Q.part_max, Q.lo_off, Q.dlo_min};
    for (int i = 0; i < 8; ++i) out[i] = v[i];
    if (entries)
        for (int e = 0; e < Q.n_entries && e < cap; ++e) entries[e] = Q.entry[e];
    return DMX_OK;
}

int dmx_panel_reach(const char* const* seqs, const int* lens, const int* wheres, int n,
                    double max_errors, int min_overlap, int flags, int32_t* out, int n_out) {
    if (!out || n_out < 6) return DMX_E_INVALID;
    if (wheres) {   // dmx_set_panel_mixed's form
        for (int a = 0; a < n; ++a)
            if (wheres[a] != DMX_FRONT && wheres[a] != DMX_BACK) return DMX_E_INVALID;
        flags = DMX_FRONT | (flags & DMX_RC);
    }
    Ctx tmp;   // never opened: build_panel reads only the A/B switches dmx_open would set
    const char* nf = std::getenv("DMX_NO_FILTER");
    tmp.no_filter = nf && nf[0] == '1';
    const char* nv = std::getenv("DMX_NO_VERIFY");
    tmp.no_verify = nv && nv[0] == '1';
    HostPanel hp;
    DevPanel dp;
    PanelReach r;
    const int rc = build_panel(&tmp, seqs, lens, wheres, n, max_errors, min_overlap, flags, hp, dp);
    if (rc == DMX_OK) r = hp.reach;
    else if (rc == DMX_E_UNSUPPORTED && hp.set) r = hp.reach;   // refused by the reach check
    else return rc;
    const int32_t v[6] = {r.pre_raw, r.pre, r.post, r.need_pre, r.need_post, kGuardNt};
    for (int i = 0; i < 6; ++i) out[i] = v[i];
    return rc;
}

int dmx_debug_bounds_selftest(dmx_ctx* c, uint32_t* out3) {
    if (!c || !out3) return DMX_E_INVALID;
    CK(hipSetDevice(c->device));
    return bounds_selftest(c, out3);
}

int dmx_exec(dmx_ctx* c) {
    if (!c) return DMX_E_INVALID;
    if (!c->panel[0].set || (c->mode != DMX_MODE_SINGLE && !c->panel[1].set)) {
        c->err = "panels not set for this mode";
        return DMX_E_STATE;
    }
    CK(hipSetDevice(c->device));
    int rc = ensure_pipeline(c);
    if (rc) return rc;
    hipStream_t st = c->stream;
    CK(hipEventRecord(c->ev[8], st));
    CK(hipMemsetAsync(c->d_counters, 0, 32 * sizeof(uint32_t), st));
    CK(hipMemsetAsync(c->d_shard, 0, kShLists * kShards * kShardStride * sizeof(uint32_t), st));
    CK(hipMemsetAsync(c->d_counts, 0, c->n_counts * sizeof(unsigned long long), st));
    c->counts_reduced = false;
    // A panel whose accepted matches can score <= 0 keeps one winner per orientation:
    // ReverseComplementer compares the two orientations' best scores with "no match" = 0, so
    // a read whose only forward match scores -1 is taken reverse-complemented (and unmatched).
    for (int r = 0; r < 2; ++r)
        c->orient_slot[r] = c->mode != DMX_MODE_LINKED && c->panel[r].n_orient == 2 &&
                            c->panel[r].nonpos;
    const size_t slots0 = c->mode == DMX_MODE_LINKED ? c->n_reads * (size_t)c->panel[0].n
                                                     : c->n_reads * (c->orient_slot[0] ? 2 : 1);
    CK(hipMemsetAsync(c->d_winner[0], 0xFF, slots0 * sizeof(unsigned long long), st));
    if ((rc = prepare_flat(c, st))) return rc;
    if ((rc = launch_round(c, 0, st))) return rc;
    if ((rc = launch_finalize(c, 0, st))) return rc;
    if (c->mode != DMX_MODE_SINGLE) {
        CK(hipMemsetAsync(c->d_winner[1], 0xFF, c->item_cap * (c->orient_slot[1] ? 2 : 1) *
                                                     sizeof(unsigned long long), st));
        if ((rc = launch_round(c, 1, st))) return rc;
        if ((rc = launch_finalize(c, 1, st))) return rc;
    }
    c->executed = true;
    return bounds_check(c, "dmx_exec");   // DMX_DEBUG_BOUNDS builds only (else DMX_OK)
}

int dmx_sync(dmx_ctx* c) {
    if (!c) return DMX_E_INVALID;
    CK(hipStreamSynchronize(c->stream));
    return DMX_OK;
}

int dmx_fetch(dmx_ctx* c, dmx_result* out) {
    if (!c || (!out && c->n_reads)) return DMX_E_INVALID;
    if (!c->executed) {
        c->err = "dmx_fetch before dmx_exec";
        return DMX_E_STATE;
    }
    if (c->chunked) {
        c->err = "dmx_fetch after a chunked dmx_run (its results went to dmx_run's out)";
        return DMX_E_STATE;
    }
    CK(hipSetDevice(c->device));
    if (c->n_reads)
        CK(hipMemcpyAsync(out, c->d_res, c->n_reads * sizeof(dmx_result), hipMemcpyDeviceToHost,
                          c->stream));
    CK(hipStreamSynchronize(c->stream));
    return DMX_OK;
}

int dmx_counts(dmx_ctx* c, uint64_t* out, size_t n_out) {
    if (!c || !out) return DMX_E_INVALID;
    if (!c->executed) {
        c->err = "dmx_counts before dmx_exec";
        return DMX_E_STATE;
    }
    if (n_out < c->n_counts) {
        c->err = "counts buffer too small";
        return DMX_E_INVALID;
    }
    CK(hipSetDevice(c->device));
    CK(hipMemcpyAsync(out, c->d_counts, c->n_counts * 8, hipMemcpyDeviceToHost, c->stream));
    CK(hipStreamSynchronize(c->stream));
    return (int)c->n_counts;
}

int dmx_stats(dmx_ctx* c, float* stage_ms, int n_stage, uint64_t* counts, int n_counts,
              int* flags) {
    if (!c) return DMX_E_INVALID;
    if (!c->executed) {
        c->err = "dmx_stats before dmx_exec";
        return DMX_E_STATE;
    }
    CK(hipSetDevice(c->device));
    CK(hipStreamSynchronize(c->stream));
    const int rounds = c->mode == DMX_MODE_SINGLE ? 1 : 2;
    float t[17] = {};
    for (int r = 0; r < rounds; ++r) {
        hipEventElapsedTime(&t[3 * r + 0], c->ev[3 * r + 0], c->ev[3 * r + 1]);
        hipEventElapsedTime(&t[3 * r + 1], c->ev[3 * r + 1], c->ev[3 * r + 2]);
        hipEventElapsedTime(&t[3 * r + 2], c->ev[3 * r + 2], c->ev[6 + r]);
        const bool f = c->panel[r].filter && !(c->mode == DMX_MODE_LINKED);
        if (f) {
            hipEventElapsedTime(&t[7 + 2 * r], c->ev[3 * r + 0], c->ev[9 + 2 * r]);
            hipEventElapsedTime(&t[8 + 2 * r], c->ev[9 + 2 * r], c->ev[10 + 2 * r]);
            hipEventElapsedTime(&t[11 + 2 * r], c->ev[10 + 2 * r], c->ev[13 + r]);
            hipEventElapsedTime(&t[12 + 2 * r], c->ev[13 + r], c->ev[3 * r + 1]);
            if (c->panel[r].piece_step)   // the piece screen's share of the filter stage
                hipEventElapsedTime(&t[15 + r], c->ev[3 * r + 0], c->ev[15 + r]);
        }
    }
    hipEventElapsedTime(&t[6], c->ev[8], c->ev[6 + rounds - 1]);
    for (int i = 0; i < n_stage && i < 17; ++i) stage_ms[i] = t[i];
    uint32_t cnt[32];
    int list_ovf = 0;
    CK(read_counters(c, cnt, &list_ovf));
    if (getenv("DMX_DEBUG_STATS"))
        fprintf(stderr,
                "dmx stats: filter tasks %u %u windows raw %u %u verified %u %u screened tasks "
                "%u %u (by 3' cells only %u %u) cand %u %u %u %u\n",
                cnt[14], cnt[15], cnt[4], cnt[5], cnt[10], cnt[11], cnt[12], cnt[13], cnt[19],
                cnt[23], cnt[6], cnt[7], cnt[8], cnt[9]);
    if (counts) {
        const bool b0 = c->band_ok[0] && !c->force_ring, b1 = c->band_ok[1] && !c->force_ring;
        const uint64_t v[14] = {cnt[0],
                                cnt[1],
                                c->panel[0].verify ? cnt[10] : cnt[4],
                                c->panel[1].verify ? cnt[11] : cnt[5],
                                b0 ? (uint64_t)cnt[6] + cnt[7] : cnt[16],
                                b1 ? (uint64_t)cnt[8] + cnt[9] : cnt[20],
                                cnt[17],
                                cnt[21],
                                cnt[4],
                                cnt[5],
                                cnt[12],
                                cnt[13],
                                cnt[14],
                                cnt[15]};
        for (int i = 0; i < n_counts && i < 14; ++i) counts[i] = v[i];
    }
    if (flags) {
        int f = (int)cnt[3];
        if (cnt[0] > c->cl_cap || cnt[1] > c->cl_cap) f |= 1;
        f |= list_ovf;
        *flags = f;
    }
    return DMX_OK;
}

int dmx_debug_fetch(dmx_ctx* c, int what, int round, void* out, size_t cap_bytes) {
    if (!c || round < 0 || round > 1 || (!out && cap_bytes)) return DMX_E_INVALID;
    if (!c->executed) {
        c->err = "dmx_debug_fetch before dmx_exec";
        return DMX_E_STATE;
    }
    CK(hipSetDevice(c->device));
    CK(hipStreamSynchronize(c->stream));
    uint32_t cnt[32];
    CK(read_counters(c, cnt, nullptr));
    if (what == DMX_DBG_FLAGS) {
        if (cap_bytes >= 4) std::memcpy(out, &cnt[3], 4);
        return 4;
    }
    // every list is sharded: gather its shards (windows and tasks of round 1 share buffers with
    // round 0: only the last executed round's are resident)
    int slot;
    const char* base;
    size_t cap, rec;
    switch (what) {
        case DMX_DBG_WINDOWS: slot = kShWin + round; base = (const char*)c->d_win; cap = c->win_cap; rec = sizeof(Window); break;
        case DMX_DBG_VERIFIED: slot = kShWin2 + round; base = (const char*)c->d_win2; cap = c->win_cap; rec = sizeof(Window); break;
        case DMX_DBG_TASKS: slot = kShTasks + round; base = (const char*)c->d_tasks; cap = c->task_cap; rec = sizeof(Window); break;
        case DMX_DBG_CANDS0: slot = kShCand + 2 * round; base = (const char*)c->d_cand[round][0]; cap = c->cand_cap; rec = sizeof(Cand); break;
        case DMX_DBG_CANDS1: slot = kShCand + 2 * round + 1; base = (const char*)c->d_cand[round][1]; cap = c->cand_cap; rec = sizeof(Cand); break;
        default: return DMX_E_INVALID;
    }
    uint32_t sh[kShards * kShardStride];
    CK(hipMemcpy(sh, c->d_shard + slot * kShards * kShardStride, sizeof(sh),
                 hipMemcpyDeviceToHost));
    const size_t scap = cap / kShards;
    size_t done = 0;
    for (int s = 0; s < kShards; ++s) {
        const size_t nb = std::min<size_t>(sh[s * kShardStride], scap) * rec;
        const size_t take = out ? std::min(nb, cap_bytes > done ? cap_bytes - done : 0) : 0;
        if (take) CK(hipMemcpy((char*)out + done, base + s * scap * rec, take, hipMemcpyDeviceToHost));
        done += nb;
    }
    if (out) {   // records name their window code slot in off's top bits: clear them
        for (size_t r = 0; (r + 1) * rec <= std::min(done, cap_bytes); ++r) {
            uint64_t off;
            std::memcpy(&off, (char*)out + r * rec + 32, 8);
            off &= kOffMask;
            std::memcpy((char*)out + r * rec + 32, &off, 8);
        }
    }
    return (int)std::min<size_t>(done, (size_t)1 << 30);
}

namespace {

// One chunk of a chunked dmx_run: reads [lo, hi) of the caller's dmx_pack batch, rebased.
struct Chunk {
    size_t lo, hi, w0, words;
    uint64_t g0;      // the chunk's nt base: its offsets are rebased by -g0 on the device
    size_t exc_lo, exc_n;   // its range of the sparse mask's exceptions
};

// The buffers of the resident batch (Ctx fields) <-> the second set.
void swap_inputs(Ctx* c) {
    std::swap(c->d_seq_alloc, c->alt.seq_alloc);
    std::swap(c->d_nmask_alloc, c->alt.nmask_alloc);
    std::swap(c->d_offs, c->alt.offs);
    std::swap(c->d_lens, c->alt.lens);
    std::swap(c->d_res, c->alt.res);
    std::swap(c->cap_words, c->alt.cap_words);
    std::swap(c->in_cap_reads, c->alt.cap_reads);
    std::swap(c->res_cap, c->alt.res_cap);
    std::swap(c->d_exc, c->alt.exc);
    std::swap(c->exc_cap, c->alt.exc_cap);
    std::swap(c->n_words, c->alt.n_words);
    c->d_seq = c->d_seq_alloc + kGuardWords;
    c->d_nmask = c->d_nmask_alloc + kGuardWords;
}

// Upload one chunk into the current set on the copy stream (host-blocking for pageable
// memory, while the compute stream keeps running), zeroing a longer previous chunk's tail.
// Upload one chunk into the current set on the copy stream (asynchronous: the caller syncs
// cstream before the set is used), zeroing a longer previous chunk's tail.  Offsets go up as the
// caller gave them and are rebased on the device.
int upload_chunk(Ctx* c, const Chunk& k, const uint32_t* seq2b, const MaskSrc& mask,
                 const uint64_t* offsets, const uint32_t* lens) {
    hipStream_t s = c->cstream;
    // the nmask words of a range (1 bit per nt: half as many); the rest of the buffer stays
    // zero (the guard)
    const auto mask_words = [](size_t w) { return std::min(w, (w + 1) / 2 + 2); };
    const size_t nmw = mask_words(k.words), old_nmw = mask_words(c->n_words);
    if (c->n_words > k.words)
        CK(hipMemsetAsync(c->d_seq + k.words, 0, (c->n_words - k.words) * 4, s));
    if (old_nmw > nmw) CK(hipMemsetAsync(c->d_nmask + nmw, 0, (old_nmw - nmw) * 4, s));
    CK(hipMemcpyAsync(c->d_seq, seq2b + k.w0, k.words * 4, hipMemcpyHostToDevice, s));
    int rc;
    if ((rc = upload_mask(c, mask, k.w0 / 2, nmw, s))) return rc;
    const size_t n = k.hi - k.lo;
    CK(hipMemcpyAsync(c->d_offs, offsets + k.lo, n * 8, hipMemcpyHostToDevice, s));
    if ((rc = launch_rebase_offsets(c->d_offs, (uint32_t)n, k.g0, s))) return rc;
    CK(hipMemcpyAsync(c->d_lens, lens + k.lo, n * 4, hipMemcpyHostToDevice, s));
    c->n_words = k.words;
    return DMX_OK;
}

// fn(lo, hi) over [0, n) on up to 16 host threads
extern "C++" template <class F>
void parallel_ranges(size_t n, F fn) {
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const size_t nth = n < (1u << 16) ? 1 : hw;
    if (nth == 1) {
        fn((size_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (n + nth - 1) / nth;
    for (size_t t = 0; t < nth; ++t) {
        const size_t lo = t * per, hi = std::min(n, lo + per);
        if (lo < hi) th.emplace_back(fn, lo, hi);
    }
    for (auto& x : th) x.join();
}

int alloc_set(Ctx* c, size_t words, size_t reads) {
    int rc;
    const size_t total = words + 2 * kGuardWords;
    if ((rc = dev_alloc(c, &c->d_seq_alloc, total))) return rc;
    if ((rc = dev_alloc(c, &c->d_nmask_alloc, total))) return rc;
    CK(hipMemsetAsync(c->d_seq_alloc, 0, total * 4, c->stream));
    CK(hipMemsetAsync(c->d_nmask_alloc, 0, total * 4, c->stream));
    if ((rc = dev_alloc(c, &c->d_offs, reads))) return rc;
    if ((rc = dev_alloc(c, &c->d_lens, reads))) return rc;
    if ((rc = dev_alloc(c, &c->d_res, reads))) return rc;
    c->d_seq = c->d_seq_alloc + kGuardWords;
    c->d_nmask = c->d_nmask_alloc + kGuardWords;
    c->cap_words = words;
    c->in_cap_reads = reads;
    c->res_cap = reads;
    c->n_words = 0;
    CK(hipStreamSynchronize(c->stream));
    return DMX_OK;
}

// dmx_run of a batch larger than one chunk: chunks of `per` reads alternate between two input
// and result sets.  While chunk k's kernels run on the compute stream, the host uploads chunk
// k+1 and downloads chunk k-1's results on the copy stream; per-bin counts are summed on the
// host and left in d_counts for dmx_counts / dmx_allreduce_counts.  The batch must come from
// dmx_pack (offsets on kPackAlign boundaries after DMX_PACK_PAD).
int run_chunked(dmx_ctx* c, const uint32_t* seq2b, const MaskSrc& nmask,
                const uint64_t* offsets, const uint32_t* lens, size_t n_words, size_t n_reads,
                dmx_result* out, size_t per) {
    std::vector<Chunk> ch;
    size_t maxw = 0, maxn = 0, maxe = 0;
    for (size_t lo = 0; lo < n_reads; lo += per) {
        Chunk k;
        k.lo = lo;
        k.hi = std::min(n_reads, lo + per);
        if (offsets[lo] < (uint64_t)DMX_PACK_PAD || offsets[lo] % kPackAlign) {
            c->err = "dmx_run: offsets must come from dmx_pack";
            return DMX_E_INVALID;
        }
        k.g0 = offsets[lo] - DMX_PACK_PAD;   // a 32-nt (nmask word) boundary
        ch.push_back(k);
    }
    // each chunk's end (the largest rebased offset + length): one parallel pass over the reads
    std::vector<uint64_t> ends(ch.size(), 0);
    {
        std::vector<std::vector<uint64_t>> part;
        std::mutex mu;
        parallel_ranges(n_reads, [&](size_t lo, size_t hi) {
            std::vector<uint64_t> e(ch.size(), 0);
            for (size_t r = lo; r < hi; ++r) {
                const size_t k = r / per;
                e[k] = std::max<uint64_t>(e[k], offsets[r] + lens[r] - ch[k].g0);
            }
            std::lock_guard<std::mutex> g(mu);
            part.push_back(std::move(e));
        });
        for (const auto& e : part)
            for (size_t k = 0; k < ch.size(); ++k) ends[k] = std::max(ends[k], e[k]);
    }
    for (size_t k = 0; k < ch.size(); ++k) {
        Chunk& x = ch[k];
        x.w0 = (size_t)(x.g0 / 16);
        if (x.w0 >= n_words) {
            c->err = "dmx_run: offsets beyond the packed buffer";
            return DMX_E_INVALID;
        }
        x.words = std::min(n_words - x.w0, (size_t)((ends[k] + DMX_PACK_PAD + 31) / 32 * 2 + 4));
        maxw = std::max(maxw, x.words);
        maxn = std::max(maxn, x.hi - x.lo);
        if (!nmask.dense) {   // the chunk's exceptions: mask words [w0 / 2, w0 / 2 + nmw)
            const size_t mw0 = x.w0 / 2, nmw = std::min(x.words, (x.words + 1) / 2 + 2);
            const uint32_t* a = std::lower_bound(nmask.idx, nmask.idx + nmask.n, (uint32_t)mw0);
            const uint32_t* b = std::lower_bound(a, nmask.idx + nmask.n, (uint32_t)(mw0 + nmw));
            maxe = std::max(maxe, (size_t)(b - a));
        }
    }
    CK(hipSetDevice(c->device));
    if (!c->cstream) CK(hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking));
    if (!c->dstream) CK(hipStreamCreateWithFlags(&c->dstream, hipStreamNonBlocking));
    int rc;
    // both sets sized for the largest chunk; each set's capacities travel with its buffers
    // (swap_inputs), apart from the pipeline's cap_reads
    if (c->cap_words < maxw || c->in_cap_reads < maxn || c->res_cap < maxn || !c->d_offs ||
        !c->d_res) {
        if ((rc = alloc_set(c, maxw, maxn))) return rc;
    }
    if (c->alt.cap_words < maxw || c->alt.cap_reads < maxn || c->alt.res_cap < maxn ||
        !c->alt.offs || !c->alt.res) {
        swap_inputs(c);
        rc = alloc_set(c, maxw, maxn);
        swap_inputs(c);
        if (rc) return rc;
    }
    for (int set = 0; set < 2 && maxe; ++set) {   // exception staging, sized before the loop
        if (c->exc_cap < maxe || !c->d_exc) {
            if ((rc = dev_alloc(c, &c->d_exc, 2 * maxe))) return rc;
            c->exc_cap = maxe;
        }
        swap_inputs(c);
    }
    c->n_reads = maxn;
    chop_invalidate(c);
    c->chunked = false;
    std::vector<uint64_t> total, part;
    if ((rc = upload_chunk(c, ch[0], seq2b, nmask, offsets, lens))) return rc;
    CK(hipStreamSynchronize(c->cstream));
    for (size_t i = 0; i < ch.size(); ++i) {
        const size_t n = ch[i].hi - ch[i].lo;
        c->n_reads = n;
        int attempt = 0;
        for (;; ++attempt) {
            if ((rc = dmx_exec(c))) return rc;
            // meanwhile: the next chunk into the other set, the previous chunk's results out
            // (uploads on cstream and the download on dstream run in both directions at once;
            // the other set's inputs and its result array are disjoint buffers)
            if (attempt == 0) {
                swap_inputs(c);
                if (i + 1 < ch.size() &&
                    (rc = upload_chunk(c, ch[i + 1], seq2b, nmask, offsets, lens)))
                    return rc;
                if (i > 0) {
                    const size_t pn = ch[i - 1].hi - ch[i - 1].lo;
                    CK(hipMemcpyAsync(out + ch[i - 1].lo, c->d_res, pn * sizeof(dmx_result),
                                      hipMemcpyDeviceToHost, c->dstream));
                }
                swap_inputs(c);
            }
            uint64_t cl[8];
            int flags = 0;
            float ms[7];
            if ((rc = dmx_stats(c, ms, 7, cl, 8, &flags))) return rc;
            if (flags & 18) {
                c->err = (flags & 2) ? "internal: traceback left the exact window (please report)"
                                     : "internal: filter task invariant violated (please report)";
                return DMX_E_STATE;
            }
            if (!(flags & 13)) break;
            if (attempt >= 7) {
                c->err = "candidate cluster buffer overflow";
                return DMX_E_NOMEM;
            }
            if ((flags & 1) && (rc = grow_clusters(c))) return rc;
            if ((flags & 4) && (rc = grow_windows(c))) return rc;
            if ((flags & 8) && (rc = grow_cands(c))) return rc;
        }
        part.assign(c->n_counts, 0);
        CK(hipMemcpy(part.data(), c->d_counts, c->n_counts * 8, hipMemcpyDeviceToHost));
        if (total.size() != part.size()) total.assign(part.size(), 0);
        for (size_t x = 0; x < part.size(); ++x) total[x] += part[x];
        CK(hipStreamSynchronize(c->cstream));   // the next chunk is in, the previous one out
        CK(hipStreamSynchronize(c->dstream));
        swap_inputs(c);   // the next chunk (uploaded above) becomes the resident batch
    }
    // the last chunk's results sit in the other set now
    swap_inputs(c);
    {
        const Chunk& k = ch.back();
        CK(hipMemcpy(out + k.lo, c->d_res, (k.hi - k.lo) * sizeof(dmx_result),
                     hipMemcpyDeviceToHost));
    }
    CK(hipMemcpy(c->d_counts, total.data(), total.size() * 8, hipMemcpyHostToDevice));
    c->counts_reduced = false;
    c->chunked = true;
    return DMX_OK;
}

}  // namespace

namespace {

int run_impl(dmx_ctx* c, const uint32_t* seq2b, const MaskSrc& mask, const uint64_t* offsets,
             const uint32_t* lens, size_t n_words, size_t n_reads, dmx_result* out) {
    size_t per = (size_t)1 << 21;   // reads per chunk of an overlapped run
    if (const char* e = std::getenv("DMX_RUN_CHUNK")) per = (size_t)std::strtoull(e, nullptr, 10);
    // chunking rebases every chunk on a 32-nt boundary, which needs dmx_pack's layout at the
    // chunk starts; any other (caller-packed) batch runs in one shot, whatever its size
    bool chunkable = per > 0 && n_reads > per + per / 2;
    for (size_t lo = 0; chunkable && lo < n_reads; lo += per)
        chunkable = offsets[lo] >= (uint64_t)DMX_PACK_PAD && offsets[lo] % kPackAlign == 0;
    if (chunkable) {
        if (!c->panel[0].set || (c->mode != DMX_MODE_SINGLE && !c->panel[1].set)) {
            c->err = "panels not set for this mode";
            return DMX_E_STATE;
        }
        // Every read must also sit at or after its chunk's base g0 = offsets[chunk lo] -
        // DMX_PACK_PAD (+16, the guard any offset keeps): the device rebases offsets by g0, so
        // a read below it (a permuted batch) would wrap.  Such a batch runs in one shot.
        std::atomic<bool> bad{false}, permuted{false};
        parallel_ranges(n_reads, [&](size_t lo, size_t hi) {
            for (size_t r = lo; r < hi; ++r) {
                if (offsets[r] < 16 || (offsets[r] + lens[r] + 64) > (uint64_t)n_words * 16 ||
                    lens[r] >= (1u << 30)) {
                    bad = true;
                    return;
                }
                if (offsets[r] < offsets[r / per * per] - (uint64_t)DMX_PACK_PAD + 16u)
                    permuted = true;
            }
        });
        if (bad) {
            c->err = "read offsets/lengths do not fit the packed buffer (use dmx_pack)";
            return DMX_E_INVALID;
        }
        chunkable = !permuted;
    }
    if (chunkable)
        return run_chunked(c, seq2b, mask, offsets, lens, n_words, n_reads, out, per);
    int rc = load_impl(c, seq2b, mask, offsets, lens, n_words, n_reads);
    if (rc) return rc;
    for (int attempt = 0; attempt < 8; ++attempt) {
        if ((rc = dmx_exec(c))) return rc;
        uint64_t cl[8];
        int flags = 0;
        float ms[7];
        if ((rc = dmx_stats(c, ms, 7, cl, 8, &flags))) return rc;
        if (flags & 18) {
            c->err = (flags & 2) ? "internal: traceback left the exact window (please report)"
                                 : "internal: filter task invariant violated (please report)";
            return DMX_E_STATE;
        }
        if (!(flags & 13)) return dmx_fetch(c, out);
        // candidate overflow: retry with more room, never truncate
        if ((flags & 1) && (rc = grow_clusters(c))) return rc;
        if ((flags & 4) && (rc = grow_windows(c))) return rc;
        if ((flags & 8) && (rc = grow_cands(c))) return rc;
    }
    c->err = "candidate cluster buffer overflow";
    return DMX_E_NOMEM;
}

}  // namespace

int dmx_run(dmx_ctx* c, const uint32_t* seq2b, const uint32_t* nmask, const uint64_t* offsets,
            const uint32_t* lens, size_t n_words, size_t n_reads, dmx_result* out) {
    if (!c || (n_reads && (!seq2b || !nmask || !offsets || !lens || !out))) return DMX_E_INVALID;
    MaskSrc m;
    m.dense = nmask;
    return run_impl(c, seq2b, m, offsets, lens, n_words, n_reads, out);
}

int dmx_run_sparse(dmx_ctx* c, const uint32_t* seq2b, const uint32_t* exc_idx,
                   const uint32_t* exc_val, size_t n_exc, const uint64_t* offsets,
                   const uint32_t* lens, size_t n_words, size_t n_reads, dmx_result* out) {
    if (!c || (n_reads && (!seq2b || !offsets || !lens || !out)) ||
        (n_exc && (!exc_idx || !exc_val)))
        return DMX_E_INVALID;
    const size_t nmw = std::min(n_words, (n_words + 1) / 2 + 2);
    std::atomic<bool> bad{false};
    parallel_ranges(n_exc, [&](size_t lo, size_t hi) {
        for (size_t i = lo; i < hi; ++i)
            if (exc_idx[i] >= nmw || (i && exc_idx[i] <= exc_idx[i - 1])) {
                bad = true;
                return;
            }
    });
    if (bad) {
        c->err = "dmx_run_sparse: exception indices must be strictly increasing mask words";
        return DMX_E_INVALID;
    }
    MaskSrc m;
    m.idx = exc_idx;
    m.val = exc_val;
    m.n = n_exc;
    return run_impl(c, seq2b, m, offsets, lens, n_words, n_reads, out);
}

size_t dmx_mask_exceptions(const uint32_t* nmask, size_t n_words, uint32_t* out_idx,
                           uint32_t* out_val, size_t cap) {
    if (!nmask) return 0;
    const size_t nmw = std::min(n_words, (n_words + 1) / 2 + 2);   // the words carrying data
    const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    const size_t nth = nmw < (1u << 20) ? 1 : hw;
    std::vector<size_t> cnt(nth + 1, 0);
    const size_t per = (nmw + nth - 1) / nth;
    auto count = [&](size_t t) {
        size_t n = 0;
        for (size_t w = t * per, e = std::min(nmw, w + per); w < e; ++w) n += nmask[w] != 0;
        cnt[t + 1] = n;
    };
    auto fill = [&](size_t t) {
        size_t o = cnt[t];
        for (size_t w = t * per, e = std::min(nmw, w + per); w < e; ++w)
            if (nmask[w]) {
                if (o < cap) {
                    out_idx[o] = (uint32_t)w;
                    out_val[o] = nmask[w];
                }
                ++o;
            }
    };
    auto par = [&](auto fn) {
        if (nth == 1) return fn((size_t)0);
        std::vector<std::thread> th;
        for (size_t t = 0; t < nth; ++t) th.emplace_back(fn, t);
        for (auto& x : th) x.join();
    };
    par(count);
    for (size_t t = 0; t < nth; ++t) cnt[t + 1] += cnt[t];
    if (out_idx && out_val && cap) par(fill);
    return cnt[nth];
}

int dmx_host_register(void* p, size_t bytes) {
    if (!p || !bytes) return DMX_E_INVALID;
    return hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess ? DMX_OK : DMX_E_HIP;
}

int dmx_host_unregister(void* p) {
    if (!p) return DMX_E_INVALID;
    return hipHostUnregister(p) == hipSuccess ? DMX_OK : DMX_E_HIP;
}

int dmx_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int dmx_run_multi(dmx_ctx* const* ctxs, int n_ctx, const uint32_t* seq2b, const uint32_t* nmask,
                  const uint64_t* offsets, const uint32_t* lens, size_t n_words, size_t n_reads,
                  dmx_result* out, uint64_t* out_counts, size_t n_counts) {
    if (!ctxs || n_ctx <= 0 || !ctxs[0]) return DMX_E_INVALID;
    dmx_ctx* c0 = ctxs[0];
    if (n_reads && (!seq2b || !nmask || !offsets || !lens || !out)) return DMX_E_INVALID;
    for (int k = 1; k < n_ctx; ++k) {
        if (!ctxs[k] || ctxs[k]->mode != c0->mode || ctxs[k]->panel[0].n != c0->panel[0].n ||
            ctxs[k]->panel[1].n != c0->panel[1].n) {
            c0->err = "dmx_run_multi: contexts must share mode and panels";
            return DMX_E_INVALID;
        }
    }
    // contiguous read ranges balanced by total length; outputs land in place,
    // so shard order = input order
    std::vector<size_t> cut(n_ctx + 1, n_reads);
    cut[0] = 0;
    {
        uint64_t total = 0;
        for (size_t r = 0; r < n_reads; ++r) total += lens[r];
        uint64_t acc = 0;
        int k = 1;
        for (size_t r = 0; r < n_reads && k < n_ctx; ++r) {
            acc += lens[r];
            while (k < n_ctx && acc * (uint64_t)n_ctx >= total * (uint64_t)k) cut[k++] = r + 1;
        }
        for (int j = 1; j <= n_ctx; ++j) cut[j] = std::max(cut[j], cut[j - 1]);
    }
    // one dmx_comm_init_all set over exactly these contexts: the counts are summed on the
    // devices by RCCL; otherwise (contexts sharing a device, no communicator) on the host
    bool rccl = out_counts && c0->comm_group != 0 && c0->comm_ranks == n_ctx;
    for (int k = 1; k < n_ctx && rccl; ++k)
        rccl = ctxs[k]->comm_group == c0->comm_group && ctxs[k]->comm_rank == k;
    if (rccl && c0->comm_rank != 0) rccl = false;
    std::vector<int> rcs(n_ctx, DMX_OK);
    std::vector<std::vector<uint64_t>> cnt(n_ctx);
    auto shard = [&](int k) {
        dmx_ctx* c = ctxs[k];
        const size_t lo = cut[k], hi = cut[k + 1];
        const size_t n = hi - lo;
        if (!n) {   // nothing to run; its counts are zero
            if (rccl) rcs[k] = reset_counts(c);
            return;
        }
        uint64_t g0 = 0;
        {
            if (offsets[lo] < (uint64_t)DMX_PACK_PAD || offsets[lo] % kPackAlign) {
                c->err = "dmx_run_multi: offsets must come from dmx_pack";
                rcs[k] = DMX_E_INVALID;
                return;
            }
            g0 = offsets[lo] - DMX_PACK_PAD;
        }
        std::vector<uint64_t> offs(n);
        uint64_t end = 0;
        for (size_t r = 0; r < n; ++r) {
            offs[r] = offsets[lo + r] - g0;
            end = std::max<uint64_t>(end, offs[r] + lens[lo + r]);
        }
        const size_t w0 = (size_t)(g0 / 16);
        if (w0 >= n_words) {
            c->err = "dmx_run_multi: offsets beyond the packed buffer";
            rcs[k] = DMX_E_INVALID;
            return;
        }
        const size_t words =
            std::min(n_words - w0, (size_t)((end + DMX_PACK_PAD + 31) / 32 * 2 + 4));
        int rc = dmx_run(c, seq2b + w0, nmask + g0 / 32, offs.data(), lens + lo, words, n, out + lo);
        if (rc == DMX_OK && out_counts && !rccl) {
            cnt[k].assign(c->n_counts, 0);
            rc = dmx_counts(c, cnt[k].data(), cnt[k].size());
            if (rc > 0) rc = DMX_OK;
        }
        rcs[k] = rc;
    };
    if (n_ctx == 1) {
        shard(0);
    } else {
        std::vector<std::thread> th;
        for (int k = 0; k < n_ctx; ++k) th.emplace_back(shard, k);
        for (auto& t : th) t.join();
    }
    for (int k = 0; k < n_ctx; ++k) {
        if (rcs[k] != DMX_OK) {
            if (k) c0->err = "device " + std::to_string(ctxs[k]->device) + ": " + ctxs[k]->err;
            return rcs[k];
        }
    }
    if (rccl) return allreduce_counts_group(ctxs, n_ctx, out_counts, n_counts);
    if (out_counts) {
        size_t nc = 0;
        for (int k = 0; k < n_ctx; ++k) nc = std::max(nc, cnt[k].size());
        if (n_counts < nc) {
            c0->err = "counts buffer too small";
            return DMX_E_INVALID;
        }
        for (size_t i = 0; i < n_counts; ++i) out_counts[i] = 0;
        for (int k = 0; k < n_ctx; ++k)
            for (size_t i = 0; i < cnt[k].size(); ++i) out_counts[i] += cnt[k][i];
        return (int)nc;
    }
    return DMX_OK;
}

}  // extern "C"
