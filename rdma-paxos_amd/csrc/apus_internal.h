// Internal (non-ABI) declarations shared by the libapus_gpu translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <condition_variable>
#include <mutex>

#include "../../include/apus_gpu.h"

namespace apus {

// Per-stream launch scratch.  Launches on one stream are ordered, so they may
// share one buffer; launches on different streams of one context get their
// own (the per-block partial statistics and commit_wave_kernel's deferred
// group list are written by one launch and read by the next on its stream).
struct StreamScratch {
    hipStream_t stream;
    bool used;
    uint64_t *partials;     // device scratch for per-block partial statistics
    size_t partials_cap;    // uint64 slots
    uint32_t *slow;         // device [1 + slow_cap]: count, then groups commit_wave_kernel deferred
    size_t slow_cap;        // groups
    uint32_t *ticket;       // device word: quorum_tail_kernel's block arrivals (0 between launches)
    uint64_t last_use;      // apus_ctx::scr_tick at the last launch (least recently used is reclaimed)
    int pins;               // calls between stream_scratch and their last launch (ScratchPin)
    bool reclaiming;        // being handed to another stream (the device drains first)
    bool growing;           // its buffers are being regrown (outside the context lock)
};
constexpr int kMaxStreams = 16;

}  // namespace apus

struct apus_ctx {
    int device = 0;
    int n_cu = 256;
    uint64_t *stats = nullptr;        // device uint64[APUS_STAT_COUNT], shared by every stream
    std::mutex mu;                    // guards scr[] and occ[]
    std::condition_variable scr_cv;   // a pin released / a reclaim finished
    apus::StreamScratch scr[apus::kMaxStreams] = {};
    uint64_t scr_tick = 0;
    int occ[64] = {};                 // commit kernel blocks per CU: (checksum) x (wave, segments, wave + hop) x epilogue
    void *walk_ev[2] = {};            // apus_commit_mark_walk: hipEvent_t pair around the next walk kernel
    void *tail_ev[2] = {};            // apus_commit_mark_tail: the same around the next tail kernel
    void *comm = nullptr;             // ncclComm_t or NULL
    // scalar drop-in scratch: one call at a time (scalar_mu held from the
    // upload of its inputs to the read-back of its outputs)
    std::mutex scalar_mu;
    uint8_t *s_buf = nullptr;
    size_t s_cap = 0;
    uint8_t *h_pinned = nullptr;
    size_t h_cap = 0;
    hipStream_t s_stream = nullptr;
    // staging image of the scalar calls on logs the library did not allocate
    uint8_t *stage = nullptr;         // pinned, mapped host memory
    uint8_t *stage_dev = nullptr;     // its device address
    size_t stage_cap = 0;
    // one-launch scalar calls: their results, pinned and mapped (the kernel
    // stores them and a sequence number last; the caller waits on the number)
    uint8_t *q_host = nullptr;
    uint8_t *q_dev = nullptr;
    uint32_t q_seq = 0;
};

namespace apus {

void log_error(const char *fmt, ...);

// commit walk (+checksum) and median launches (apus_commit.hip)
hipError_t launch_commit(apus_ctx *ctx, const apus_batch_t &b, const apus_commit_out_t &o,
                         uint32_t flags, hipStream_t s);
// vote / rank / prune / validate / nc build (apus_quorum.hip)
// the walk kernel a commit call would launch: info[0] kind (0 lane, 1 wave,
// 2 segment), [1] hop walk, [2] block counter, [3] grid, [4] NC epilogue,
// [5] last-determinant rows
hipError_t commit_walk_info(apus_ctx *ctx, const apus_batch_t &b, uint32_t flags, uint32_t *info);
hipError_t launch_vote(apus_ctx *ctx, const apus_batch_t &b, const apus_vote_out_t &o,
                       hipStream_t s);
hipError_t launch_rank(apus_ctx *ctx, const apus_batch_t &b, const apus_rank_out_t &o,
                       hipStream_t s);
hipError_t launch_prune(apus_ctx *ctx, const apus_batch_t &b, const apus_prune_out_t &o,
                        hipStream_t s);
hipError_t launch_validate(apus_ctx *ctx, const apus_batch_t &b, const apus_nc_batch_t &nc,
                           uint64_t *out, hipStream_t s);
hipError_t launch_nc_build(apus_ctx *ctx, const apus_batch_t &b, apus_entry_det_t *dets,
                           uint32_t max_dets, uint32_t *len, hipStream_t s);
hipError_t launch_last_idx_term(const apus_batch_t &b, uint64_t *out, hipStream_t s);
// log append + ack production (apus_append.hip)
hipError_t launch_append(apus_ctx *ctx, const apus_batch_t &b, const apus_append_in_t &in,
                         const apus_append_out_t &o, hipStream_t s);
hipError_t launch_persist(apus_ctx *ctx, const apus_batch_t &b, const apus_persist_in_t &in, hipStream_t s);
hipError_t launch_config_scan(apus_ctx *ctx, const apus_batch_t &b, const apus_config_io_t &io, hipStream_t s);
hipError_t launch_apply(apus_ctx *ctx, const apus_batch_t &b, const apus_apply_io_t &io, hipStream_t s);
// the election-win transition (apus_win.hip)
hipError_t launch_vote_win(apus_ctx *ctx, const apus_batch_t &b, const apus_win_io_t &io, hipStream_t s);
// the proxy's stable-storage records (apus_records.hip)
hipError_t launch_records_store(apus_ctx *ctx, const apus_batch_t &b, const apus_records_io_t &io, hipStream_t s);
hipError_t launch_records_load(apus_ctx *ctx, const apus_records_load_io_t &io, hipStream_t s);
// log replication step machine (apus_quorum.hip)
hipError_t launch_lr_completion(apus_ctx *ctx, const apus_batch_t &b, const apus_lr_io_t &io, hipStream_t s);
hipError_t launch_log_adjust(apus_ctx *ctx, const apus_batch_t &b, const apus_lr_io_t &io, hipStream_t s);
// generator (apus_gen.hip)
hipError_t launch_gen(apus_ctx *ctx, const apus_batch_t &b, const apus_gen_cfg_t &c,
                      hipStream_t s);

uint32_t grid_for(uint64_t units, uint32_t per_block, int n_cu, uint32_t per_cu);
// the scratch of stream s, grown to at least `slots` partial-statistic slots
// and `slow_groups` deferred-group entries (0: not needed)
// blocks of 256 threads of kernel fn resident per CU (cached per context in
// occ[slot]; slots 40.. belong to the non-commit kernels)
int resident_blocks(apus_ctx *ctx, int slot, const void *fn);
// A call's hold on its stream's scratch, from stream_scratch to the end of
// the call (after its last launch): a pinned slot is never handed to another
// stream, and its buffers are not regrown under another call of the same
// stream.  release() ends the hold early (before a nested stream_scratch).
struct ScratchPin {
    apus_ctx *ctx = nullptr;
    StreamScratch *sc = nullptr;
    void release();
    ~ScratchPin() { release(); }
};
hipError_t stream_scratch(apus_ctx *ctx, hipStream_t s, size_t slots, uint64_t slow_groups, ScratchPin &pin);
void free_scratch(apus_ctx *ctx);

}  // namespace apus
