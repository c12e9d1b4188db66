// dmx_internal.h — host-side context of libdmx (not part of the public ABI).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/dmx.h"
#include "dmx_device.h"

struct ncclComm;   // RCCL (rccl/rccl.h: ncclComm_t = ncclComm*)

namespace dmx {

struct ChopState;   // read reorientation (dmx_chop.hip)

// Reach of a panel's gathers around a view, in nt (panel_reach below).
struct PanelReach {
    int pre_raw = 0;     // before view position 0, as the kernels' formulas ask
    int pre = 0;         // ... after the fetch16s clamp at -kViewReachPre
    int post = 0;        // past the view end
    int need_pre = 0;    // guard nt needed below the buffer for a read at offset kMinOffset
    int need_post = 0;   // guard nt needed past n_words for reads keeping kMinTail nt of tail
};

struct HostPanel {
    bool screen = false;      // index screen usable (filter + verify, index blocks 1..32)
    int n = 0;
    int n_orient = 1;
    bool set = false;
    bool ring_small = true;
    bool filter = false;
    bool verify = false;
    bool nonpos = false;      // an accepted match may score <= 0 (needs per-orientation winners)
    PanelReach reach;
    DevAdapter ad[kMaxAdapters];
    int pre_len = 0;          // DevPanel::pre_len (0: no verification, the window scan reads
                              // the filter's windows)
    int stage_back = 0;       // window code slots start this many columns before j1 (m + k + 1),
    int stage_lo = 0;         // and not before this view position
    int piece_step = 0;       // piece screen sampling stride (0 = off: the full filter pass)
    DevPieces pieces;         // its tables
};

struct Ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    int mode = DMX_MODE_SINGLE;
    bool no_filter = false;   // DMX_NO_FILTER=1: always full scans (A/B testing)
    bool no_verify = false;   // DMX_NO_VERIFY=1: skip the shared-prefix window verification
    bool no_pieces = false;   // DMX_NO_PIECES=1: the full filter pass instead of the piece screen
    HostPanel panel[2];
    DevPanel* d_panel[2] = {nullptr, nullptr};
    DevPieces* d_pieces[2] = {nullptr, nullptr};

    // resident batch
    size_t n_reads = 0, n_words = 0;
    size_t cap_reads = 0;     // pipeline buffers (winner slots, items, linked keys)
    size_t cap_words = 0;     // d_seq / d_nmask of the resident input set
    size_t in_cap_reads = 0;  // d_offs / d_lens of the resident input set
    size_t res_cap = 0;       // d_res of the resident input set
    uint32_t* d_seq = nullptr;          // = d_seq_alloc + kGuardWords
    uint32_t* d_nmask = nullptr;
    uint32_t* d_seq_alloc = nullptr;    // packed buffers with zeroed guard words on both sides
    uint32_t* d_nmask_alloc = nullptr;  // (the filter loads whole aligned 64-nt blocks)
    uint64_t* d_offs = nullptr;
    uint32_t* d_lens = nullptr;
    uint32_t* d_exc = nullptr;          // sparse no-match mask staging: [idx][val] (dmx_run_sparse)
    size_t exc_cap = 0;

    // dmx_run of a large batch: chunks alternate between the buffers above and this second
    // set (inputs + results), so the next chunk's upload and the previous chunk's download
    // overlap the current chunk's kernels (dmx_api.cpp run_chunked)
    struct InSet {
        uint32_t* seq_alloc = nullptr;
        uint32_t* nmask_alloc = nullptr;
        uint64_t* offs = nullptr;
        uint32_t* lens = nullptr;
        dmx_result* res = nullptr;
        uint32_t* exc = nullptr;
        // capacities travel with their buffers (swap_inputs): words, offs/lens, res, exceptions
        size_t cap_words = 0, cap_reads = 0, res_cap = 0, n_words = 0, exc_cap = 0;
    } alt;
    hipStream_t cstream = nullptr;      // uploads of chunked runs
    hipStream_t dstream = nullptr;      // result downloads of chunked runs (the other direction)
    bool chunked = false;               // the last dmx_run was chunked: dmx_fetch is refused

    // pipeline state
    dmx_result* d_res = nullptr;
    unsigned long long* d_winner[2] = {nullptr, nullptr};
    int32_t* d_origin[2] = {nullptr, nullptr};
    int32_t* d_lb[2] = {nullptr, nullptr};
    bool ring_small[2] = {true, true};
    bool band_ok[2] = {true, true};
    bool band_wide[2] = {true, true};      // some adapter has kk 6..7: list 1 needs 15 diagonals
    bool orient_slot[2] = {false, false};   // per round: one winner slot per (item, orientation)   // every adapter has kk <= 7: banded resolve
    bool force_ring = false;          // DMX_RESOLVE=ring (A/B testing)
    size_t slot_cap = 0;
    Cluster* d_cl[2] = {nullptr, nullptr};
    Outcome* d_outc[2] = {nullptr, nullptr};
    size_t cl_cap = 0;
    Cand* d_cand[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
    Outcome* d_cand_out[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};
    size_t cand_cap = 0;
    Window* d_win = nullptr;
    Window* d_win2 = nullptr;
    size_t win_cap = 0;
    ItemView* d_items = nullptr;
    size_t item_cap = 0;                 // round-2 items of the current mode and batch
    size_t item_alloc = 0;               // entries allocated in d_items (>= item_cap)
    uint32_t* d_shard = nullptr;      // [kShLists][kShards] per-shard list counters (dmx_device.h)
    uint32_t* d_counters = nullptr;   // [0..1] clusters, [2] items, [3] flags, [4..5] windows, [6+2r..] candidates, [10+r] verified windows, [16+4r..] diag, [24..27] DMX_DEBUG_BOUNDS record
    unsigned long long* d_counts = nullptr;
    unsigned long long* d_linked = nullptr;
    Window* d_tasks = nullptr;           // index screen survivors (window piece of one adapter)
    size_t task_cap = 0;
    uint32_t* d_stage = nullptr;         // window code slots (wstage_kernel), kStageWords each
    size_t stage_cap = 0;
    bool use_stage = false;              // DMX_STAGE=1 (A/B, measured slower: DESIGN.md §3.13)
    FTask* d_ftask = nullptr;            // piece screen -> filter tasks
    size_t ftask_cap = 0;
    // flat piece scan (prepare_flat): one scan of the batch against the flat rounds' combined
    // table marks cells[2 r + strand] for every flat round r
    DevPieces* d_pieces_flat = nullptr;
    int flat_rounds = 0;                 // bit r: round r's screen is the flat scan (this exec)
    int flat_want = 0;                   // the rounds the combined table was built for
    int flat_step = 0;                   // its sampling stride (0: no table)
    size_t flat_lds = 0;                 // its LDS image
    uint64_t panel_gen = 1;              // bumped by set_panel / set_mode
    uint64_t flat_gen = 0;               // panel_gen the combined table was built for
    uint32_t* d_cells[4] = {nullptr, nullptr, nullptr, nullptr};
    size_t cells_cap[4] = {0, 0, 0, 0};
    size_t cells_words = 0;
    bool no_screen = false;              // DMX_NO_SCREEN=1: every window runs every adapter
    bool screen_v1 = false;              // DMX_SCREEN_V1=1: one lane per (window, adapter) screen
    size_t n_counts = 0;
    hipEvent_t ev[17] = {};   // [3r..3r+2] round r stages, [6+r] finalize, [8] start,
                              // [9+2r] after filter, [10+2r] after verify, [13+r] after screen,
                              // [15+r] after the piece screen (its filter tasks follow)
    bool executed = false;
    ChopState* chop = nullptr;   // dmx_chop_* state, created by dmx_chop_set

    // RCCL communicator for the per-bin count exchange (dmx_comm.cpp)
    ncclComm* comm = nullptr;
    int comm_ranks = 0, comm_rank = 0;
    uint64_t comm_group = 0;     // nonzero: made by dmx_comm_init_all (one process, grouped calls)
    bool counts_reduced = false; // d_counts already summed over the ranks (cleared by dmx_exec)
};

void chop_release(Ctx* c);
void comm_release(Ctx* c);
int reset_counts(Ctx* c);      // size d_counts for the current panels/mode and zero it (sync)
// The last error of a call that has no context to keep it in (dmx_comm_unique_id's RCCL load),
// returned by dmx_last_error(NULL).
void set_process_error(const std::string& msg);
std::string process_error();
void chop_invalidate(Ctx* c);   // a new dmx_load makes the last dmx_chop_exec's results stale
int launch_round(Ctx* c, int round, hipStream_t st);
int prepare_flat(Ctx* c, hipStream_t st);   // the flat piece scan's index (dmx_kernels.hip)
int launch_finalize(Ctx* c, int round, hipStream_t st);
// offs[i] -= g0 for a chunk's offsets uploaded as the caller gave them (stream st)
int launch_rebase_offsets(uint64_t* offs, uint32_t n, uint64_t g0, hipStream_t st);
// mask[idx[i] - base] = val[i] for the n staged exceptions at d_exc ([idx][val]); stream st
int launch_mask_scatter(uint32_t* mask, const uint32_t* d_exc, uint32_t n, uint32_t base,
                        hipStream_t st);

// DMX_DEBUG_BOUNDS builds (dmx_device.h Bounds): the extents of c's device buffers for a launch
// of kernel `kid`; a reset of the violation record (d_counters[24..27]); the check after a run
// (synchronises, and fails naming the kernel, buffer and index of the first violation).  In
// release builds make_bounds is empty, set_kid / bounds_reset do nothing and bounds_check
// returns DMX_OK without synchronising.
Bounds make_bounds(const Ctx* c, int kid);
inline void set_kid(Bounds& b, int kid) {
#ifdef DMX_DEBUG_BOUNDS
    b.kid = kid;
#else
    (void)b, (void)kid;
#endif
}
hipError_t bounds_reset(Ctx* c, hipStream_t st);
int bounds_check(Ctx* c, const char* where);

// Deepest reach of the kernels' gathers around a view for panel `hp` (nt before position 0,
// before and after the -kViewReachPre clamp, and past the view end), and the smallest guard
// that covers them for every offset dmx_load / dmx_run accept.
PanelReach panel_reach(const HostPanel& hp, const DevPanel& dp);
int bounds_selftest(Ctx* c, uint32_t* host_out);   // dmx_debug_bounds_selftest

// Where a batch's no-match mask comes from: the dense bitmap (1 bit per nt) of dmx_pack, or its
// nonzero words as sorted (index, value) exceptions (dmx_mask_exceptions, dmx_run_sparse).
struct MaskSrc {
    const uint32_t* dense = nullptr;
    const uint32_t* idx = nullptr;
    const uint32_t* val = nullptr;
    size_t n = 0;
};

}  // namespace dmx

// The public opaque handle (include/dmx.h) is the host context.
struct dmx_ctx : dmx::Ctx {};

namespace dmx {
// dmx_run_multi's grouped RCCL count all-reduce (dmx_comm.cpp)
int allreduce_counts_group(dmx_ctx* const* ctxs, int n_ctx, uint64_t* out, size_t n_out);
}  // namespace dmx
