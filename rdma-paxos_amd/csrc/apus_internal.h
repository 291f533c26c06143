// Internal (non-ABI) declarations shared by the libapus_gpu translation units.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/apus_gpu.h"

struct apus_ctx {
    int device;
    int n_cu;
    uint64_t *stats;        // device uint64[APUS_STAT_COUNT]
    uint64_t *partials;     // device scratch for per-block partial sums
    size_t partials_cap;    // uint64 slots
    uint32_t *slow;         // device [1 + slow_cap]: count, then groups commit_wave_kernel deferred
    size_t slow_cap;        // groups
    void *comm;             // ncclComm_t or NULL
    // scalar drop-in scratch (lazily grown)
    uint8_t *s_buf;
    size_t s_cap;
    uint8_t *h_pinned;
    size_t h_cap;
    hipStream_t s_stream;
};

namespace apus {

void log_error(const char *fmt, ...);

// commit walk (+checksum) and median launches (apus_commit.hip)
hipError_t launch_commit(apus_ctx *ctx, const apus_batch_t &b, const apus_commit_out_t &o,
                         uint32_t flags, hipStream_t s);
// vote / rank / prune / validate / nc build (apus_quorum.hip)
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
// log replication step machine (apus_quorum.hip)
hipError_t launch_lr_completion(apus_ctx *ctx, const apus_batch_t &b, const apus_lr_io_t &io, hipStream_t s);
hipError_t launch_log_adjust(apus_ctx *ctx, const apus_batch_t &b, const apus_lr_io_t &io, hipStream_t s);
// generator (apus_gen.hip)
hipError_t launch_gen(apus_ctx *ctx, const apus_batch_t &b, const apus_gen_cfg_t &c,
                      hipStream_t s);

uint32_t grid_for(uint64_t units, uint32_t per_block, int n_cu, uint32_t per_cu);
hipError_t ensure_partials(apus_ctx *ctx, size_t slots);

}  // namespace apus
