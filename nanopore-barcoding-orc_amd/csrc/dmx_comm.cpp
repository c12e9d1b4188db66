// dmx_comm.cpp — per-bin count exchange over RCCL (xGMI) for sharded runs (include/dmx.h,
// "Multi-GPU count exchange").
//
// Reads are independent, so sharding needs no data-path collective; the only
// exchange is the (A0+1)(A1+1)+2 u64 per-bin counts each shard accumulates on its device
// (cutadapt's per-adapter totals, report.py; one cutadapt -j 24 call per panel in the reference:
// scripts/02_cutadapt_loop.sh:21,64-72,91-103).  The counts are summed in place in HBM by one
// ncclAllReduce on the context's stream, ordered after the pipeline that produced them.
//
// Two ways to build a communicator:
//   * dmx_comm_init_all — one process driving several GPUs (the CLI, the fused loop, and
//     dmx_run_multi): ncclCommInitAll over the contexts' devices, grouped calls;
//   * dmx_comm_unique_id + dmx_comm_init_rank — one process per GPU (bench.py under torchrun):
//     rank 0 draws the id, the launcher's control plane hands it to the other ranks.
//
// librccl.so is opened on the first communicator, not linked: its fat binary (573 MB in this
// ROCm) made ~570 MB of every single-GPU process's resident set, CLI calls and the resident
// server included, against the reference jobs' --mem=4G / 2G (profiles/r5_rss_probe*.json).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <type_traits>

#include "dmx_internal.h"

using namespace dmx;

static_assert(sizeof(ncclUniqueId) == DMX_COMM_ID_BYTES, "RCCL unique id size");

namespace {

// The RCCL entry points dmx uses, resolved from librccl.so.1 at first use.
struct Rccl {
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
    std::string err;   // why loading failed ("" = loaded)
};

const Rccl* rccl(std::string* why = nullptr) {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* name = getenv("DMX_RCCL_LIB");
        void* h = dlopen(name && *name ? name : "librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char* e = dlerror();
            r.err = std::string("cannot load RCCL: ") + (e ? e : "dlopen failed");
            return;
        }
        bool ok = true;
        auto sym = [&](auto& fn, const char* s) {
            fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, s));
            ok = ok && fn != nullptr;
        };
        sym(r.GetUniqueId, "ncclGetUniqueId");
        sym(r.CommInitRank, "ncclCommInitRank");
        sym(r.CommInitAll, "ncclCommInitAll");
        sym(r.CommDestroy, "ncclCommDestroy");
        sym(r.AllReduce, "ncclAllReduce");
        sym(r.GroupStart, "ncclGroupStart");
        sym(r.GroupEnd, "ncclGroupEnd");
        sym(r.GetErrorString, "ncclGetErrorString");
        if (!ok) r.err = "cannot load RCCL: a symbol is missing from the library";
    });
    if (!r.err.empty()) {
        if (why) *why = r.err;
        return nullptr;
    }
    return &r;
}

}  // namespace

namespace dmx {

void comm_release(Ctx* c) {
    if (c->comm) {
        hipSetDevice(c->device);
        if (const Rccl* R = rccl()) R->CommDestroy(c->comm);
        c->comm = nullptr;
    }
    c->comm_ranks = 0;
    c->comm_rank = 0;
    c->comm_group = 0;
}

int reset_counts(Ctx* c);   // dmx_api.cpp

}  // namespace dmx

namespace {

std::atomic<uint64_t> g_group{0};   // distinguishes communicator sets made by dmx_comm_init_all

int nccl_fail(Ctx* c, const char* what, ncclResult_t r) {
    c->err = std::string(what) + ": " + rccl()->GetErrorString(r);
    return DMX_E_HIP;
}

// RCCL for ctx c's call, or nullptr with c->err set.
const Rccl* rccl_for(Ctx* c) {
    std::string why;
    const Rccl* R = rccl(&why);
    if (!R && c) c->err = why;
    return R;
}

}  // namespace

extern "C" {

int dmx_comm_unique_id(uint8_t* id) {
    if (!id) return DMX_E_INVALID;
    std::string why;   // no context to keep it in: the process-wide message (dmx_last_error(NULL))
    const Rccl* R = rccl(&why);
    if (!R) {
        dmx::set_process_error(why);
        return DMX_E_UNSUPPORTED;
    }
    ncclUniqueId u;
    const ncclResult_t r = R->GetUniqueId(&u);
    if (r != ncclSuccess) {
        dmx::set_process_error(std::string("ncclGetUniqueId: ") + R->GetErrorString(r));
        return DMX_E_HIP;
    }
    std::memcpy(id, &u, sizeof(u));
    return DMX_OK;
}

int dmx_comm_init_rank(dmx_ctx* c, const uint8_t* id, int n_ranks, int rank) {
    if (!c || !id || n_ranks <= 0 || rank < 0 || rank >= n_ranks) return DMX_E_INVALID;
    const Rccl* R = rccl_for(c);
    if (!R) return DMX_E_UNSUPPORTED;
    comm_release(c);
    if (hipSetDevice(c->device) != hipSuccess) {
        c->err = "dmx_comm_init_rank: hipSetDevice failed";
        return DMX_E_HIP;
    }
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = R->CommInitRank(&comm, n_ranks, u, rank);
    if (r != ncclSuccess) return nccl_fail(c, "ncclCommInitRank", r);
    c->comm = comm;
    c->comm_ranks = n_ranks;
    c->comm_rank = rank;
    c->comm_group = 0;
    return DMX_OK;
}

int dmx_comm_init_all(dmx_ctx* const* ctxs, int n_ctx) {
    if (!ctxs || n_ctx <= 0 || n_ctx > 64) return DMX_E_INVALID;
    std::set<int> devs;
    int devlist[64];
    for (int k = 0; k < n_ctx; ++k) {
        if (!ctxs[k]) return DMX_E_INVALID;
        devlist[k] = ctxs[k]->device;
        devs.insert(devlist[k]);
    }
    if ((int)devs.size() != n_ctx) {   // RCCL needs one rank per device
        ctxs[0]->err = "dmx_comm_init_all: contexts must be on distinct devices";
        return DMX_E_UNSUPPORTED;
    }
    const Rccl* R = rccl_for(ctxs[0]);
    if (!R) return DMX_E_UNSUPPORTED;
    for (int k = 0; k < n_ctx; ++k) comm_release(ctxs[k]);
    ncclComm_t comms[64] = {};
    const ncclResult_t r = R->CommInitAll(comms, n_ctx, devlist);
    if (r != ncclSuccess) return nccl_fail(ctxs[0], "ncclCommInitAll", r);
    const uint64_t group = ++g_group;
    for (int k = 0; k < n_ctx; ++k) {
        ctxs[k]->comm = comms[k];
        ctxs[k]->comm_ranks = n_ctx;
        ctxs[k]->comm_rank = k;
        ctxs[k]->comm_group = group;
    }
    return DMX_OK;
}

int dmx_comm_size(dmx_ctx* c) { return c ? c->comm_ranks : DMX_E_INVALID; }

int dmx_allreduce_counts(dmx_ctx* c, uint64_t* out, size_t n_out) {
    if (!c) return DMX_E_INVALID;
    if (!c->comm) {
        c->err = "dmx_allreduce_counts: no communicator (dmx_comm_init_rank / _all)";
        return DMX_E_STATE;
    }
    if (!c->executed) {
        c->err = "dmx_allreduce_counts before dmx_exec";
        return DMX_E_STATE;
    }
    if (out && n_out < c->n_counts) {
        c->err = "counts buffer too small";
        return DMX_E_INVALID;
    }
    if (hipSetDevice(c->device) != hipSuccess) return DMX_E_HIP;
    // idempotent per exec: a second call returns the summed counts without summing them again
    // (every rank follows the same call sequence, so either all ranks reduce or none does)
    if (!c->counts_reduced) {
        const ncclResult_t r = rccl()->AllReduce(c->d_counts, c->d_counts, c->n_counts,
                                                 ncclUint64, ncclSum, c->comm, c->stream);
        if (r != ncclSuccess) return nccl_fail(c, "ncclAllReduce", r);
        c->counts_reduced = true;
    }
    if (out &&
        hipMemcpyAsync(out, c->d_counts, c->n_counts * 8, hipMemcpyDeviceToHost, c->stream) !=
            hipSuccess) {
        c->err = "dmx_allreduce_counts: D2H copy failed";
        return DMX_E_HIP;
    }
    if (hipStreamSynchronize(c->stream) != hipSuccess) {
        c->err = "dmx_allreduce_counts: stream failed";
        return DMX_E_HIP;
    }
    return (int)c->n_counts;
}

}  // extern "C"

namespace dmx {

// dmx_run_multi's exchange: every context of one dmx_comm_init_all set sums its device counts
// in place (one grouped ncclAllReduce), then ctxs[0]'s copy comes to the host.  Every context's
// d_counts must hold this batch's shard (dmx_run_multi zeroes those of empty shards).
int allreduce_counts_group(dmx_ctx* const* ctxs, int n_ctx, uint64_t* out, size_t n_out) {
    const size_t nc = ctxs[0]->n_counts;
    for (int k = 1; k < n_ctx; ++k)
        if (ctxs[k]->n_counts != nc) {
            ctxs[0]->err = "count all-reduce: shards disagree on the count layout";
            return DMX_E_STATE;
        }
    if (n_out < nc) {
        ctxs[0]->err = "counts buffer too small";
        return DMX_E_INVALID;
    }
    const Rccl* R = rccl();   // loaded: every context here has a communicator
    ncclResult_t r = R->GroupStart();
    for (int k = 0; k < n_ctx && r == ncclSuccess; ++k) {
        Ctx* c = ctxs[k];
        hipSetDevice(c->device);
        r = R->AllReduce(c->d_counts, c->d_counts, nc, ncclUint64, ncclSum, c->comm, c->stream);
    }
    const ncclResult_t r2 = R->GroupEnd();
    if (r != ncclSuccess) return nccl_fail(ctxs[0], "ncclAllReduce", r);
    if (r2 != ncclSuccess) return nccl_fail(ctxs[0], "ncclGroupEnd", r2);
    for (int k = 0; k < n_ctx; ++k) {
        hipSetDevice(ctxs[k]->device);
        if (hipStreamSynchronize(ctxs[k]->stream) != hipSuccess) {
            ctxs[0]->err = "count all-reduce: stream failed";
            return DMX_E_HIP;
        }
    }
    hipSetDevice(ctxs[0]->device);
    if (hipMemcpy(out, ctxs[0]->d_counts, nc * 8, hipMemcpyDeviceToHost) != hipSuccess) {
        ctxs[0]->err = "count all-reduce: D2H copy failed";
        return DMX_E_HIP;
    }
    for (size_t i = nc; i < n_out; ++i) out[i] = 0;
    return (int)nc;
}

}  // namespace dmx
