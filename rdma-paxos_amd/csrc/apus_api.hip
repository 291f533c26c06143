// libapus_gpu C ABI: contexts, batched entry points, scalar drop-ins and the
// RCCL statistics all-reduce.  See include/apus_gpu.h for the contract.
//
// No CPU compute path exists: every result is produced by a HIP kernel.  The
// scalar drop-ins run the batched kernels with G = 1 over the ring of a log
// the library allocated (apus_log_new, read in place) or over a staged copy
// of the bytes the call reads (any other log).
#include "apus_device.h"
#include "apus_group_ops.h"
#include "apus_internal.h"

#include <rccl/rccl.h>

#include <atomic>
#include <mutex>
#include <new>
#include <vector>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

namespace {
FILE *g_log_fp = nullptr;
std::mutex g_mu;
apus_ctx *g_default = nullptr;

// Logs the library allocated (apus_log_new): pinned, mapped host memory the
// library owns, read in place by the scalar calls.  Any other log is staged:
// the bytes a call reads are copied into the default context's own pinned
// image (Stager below).  The library never registers or maps memory it did
// not allocate.
struct OwnedLog {
    apus_log_t *host;
    uint8_t *dev;          // device address of `host`
    size_t bytes;          // header + len + pad
};
std::vector<OwnedLog> g_owned;
std::atomic<uint64_t> g_calls_in_place{0}, g_calls_staged{0}, g_bytes_staged{0};

#define CHECK_HIP(expr)                                                                     \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) {                                                             \
            apus::log_error("%s:%d %s: %s\n", __FILE__, __LINE__, #expr, hipGetErrorString(_e)); \
            return APUS_ERROR;                                                              \
        }                                                                                   \
    } while (0)

__global__ void stats_reset_kernel(uint64_t *s)
{
    if (threadIdx.x < APUS_STAT_COUNT) s[threadIdx.x] = threadIdx.x == APUS_STAT_MIN_WATERMARK ? ~0ull : 0ull;
}

}  // namespace

namespace apus {
void log_error(const char *fmt, ...)
{
    if (!g_log_fp) return;
    va_list ap;
    va_start(ap, fmt);
    fprintf(g_log_fp, "[APUS-GPU ERROR] ");
    vfprintf(g_log_fp, fmt, ap);
    va_end(ap);
    fflush(g_log_fp);
}
}  // namespace apus

extern "C" {

const char *apus_version(void) { return "libapus_gpu 0.7 (gfx950, ABI 7)"; }

int apus_abi_version(void) { return APUS_ABI_VERSION; }

void apus_set_log(FILE *fp) { g_log_fp = fp; }

int apus_ctx_create(int device, apus_ctx_t **out)
{
    if (!out) return APUS_ERROR;
    *out = nullptr;
    CHECK_HIP(hipSetDevice(device));
    apus_ctx *c = new (std::nothrow) apus_ctx();
    if (!c) return APUS_ERROR;
    c->device = device;
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
        c->n_cu = 256;
    if (hipMalloc(&c->stats, APUS_STAT_COUNT * sizeof(uint64_t)) != hipSuccess) {
        delete c;
        apus::log_error("apus_ctx_create: cannot allocate stats\n");
        return APUS_ERROR;
    }
    hipLaunchKernelGGL(stats_reset_kernel, dim3(1), dim3(64), 0, 0, c->stats);
    if (hipDeviceSynchronize() != hipSuccess) {
        (void)hipFree(c->stats);
        delete c;
        return APUS_ERROR;
    }
    *out = c;
    return APUS_OK;
}

int apus_ctx_destroy(apus_ctx_t *c)
{
    if (!c) return APUS_ERROR;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    if (c->comm) ncclCommDestroy((ncclComm_t)c->comm);
    if (c->stats) (void)hipFree(c->stats);
    apus::free_scratch(c);
    if (c->s_buf) (void)hipFree(c->s_buf);
    if (c->h_pinned) (void)hipHostFree(c->h_pinned);
    if (c->stage) (void)hipHostFree(c->stage);
    if (c->q_host) (void)hipHostFree(c->q_host);
    if (c->s_stream) (void)hipStreamDestroy(c->s_stream);
    delete c;
    return APUS_OK;
}

uint64_t *apus_ctx_stats(apus_ctx_t *c) { return c ? c->stats : nullptr; }

int apus_stats_reset(apus_ctx_t *c, apus_stream_t stream)
{
    if (!c) return APUS_ERROR;
    hipLaunchKernelGGL(stats_reset_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, c->stats);
    CHECK_HIP(hipGetLastError());
    return APUS_OK;
}

int apus_stats_read(apus_ctx_t *c, uint64_t out[APUS_STAT_COUNT], apus_stream_t stream)
{
    if (!c || !out) return APUS_ERROR;
    CHECK_HIP(hipMemcpyAsync(out, c->stats, APUS_STAT_COUNT * sizeof(uint64_t), hipMemcpyDeviceToHost,
                             (hipStream_t)stream));
    CHECK_HIP(hipStreamSynchronize((hipStream_t)stream));
    return APUS_OK;
}

// A batch of dare_log_t images (APUS_BATCH_LOG_IMAGE) reads its offsets from
// the images' headers and config.cid from b->cid; `state` is then unused.
static bool is_image(const apus_batch_t *b) { return (b->flags & APUS_BATCH_LOG_IMAGE) != 0; }

static bool batch_ok(const apus_batch_t *b)
{
    if (!b || !b->self_idx) return false;
    if (b->n_replicas == 0 || b->n_replicas > APUS_MAX_SERVER_COUNT) return false;
    if (is_image(b)) {
        // the header of group 0 lies in front of ring; entries[] u64-aligned
        if (!b->ring || !b->cid || ((uintptr_t)b->ring & 7u) || (b->ring_stride & 7u) ||
            b->ring_stride < APUS_LOG_HDR_BYTES) {
            apus::log_error("log-image batch: ring, cid, 8-B aligned entries and stride >= header required\n");
            return false;
        }
        return true;
    }
    return b->state != nullptr;
}

// the synthetic generator writes state rows: it takes state-row batches only
// (every other writer updates a log image's header in place, offsets_of)
static bool rows_ok(const apus_batch_t *b)
{
    if (!batch_ok(b)) return false;
    if (is_image(b)) {
        apus::log_error("apus_gen_batch writes state rows: APUS_BATCH_LOG_IMAGE batches are not generated\n");
        return false;
    }
    return true;
}

int apus_commit_mark_walk(apus_ctx_t *c, void *start, void *stop)
{
    if (!c || (!start) != (!stop)) return APUS_ERROR;
    std::lock_guard<std::mutex> lk(c->mu);
    c->walk_ev[0] = start;
    c->walk_ev[1] = stop;
    return APUS_OK;
}

int apus_commit_mark_tail(apus_ctx_t *c, void *start, void *stop)
{
    if (!c || (!start) != (!stop)) return APUS_ERROR;
    std::lock_guard<std::mutex> lk(c->mu);
    c->tail_ev[0] = start;
    c->tail_ev[1] = stop;
    return APUS_OK;
}

int apus_commit_walk_info(apus_ctx_t *c, const apus_batch_t *b, uint32_t flags, uint32_t info[6])
{
    if (!c || !batch_ok(b) || !info) return APUS_ERROR;
    CHECK_HIP(apus::commit_walk_info(c, *b, flags, info));
    return APUS_OK;
}

int apus_commit_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_commit_out_t *o, uint32_t flags,
                      apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !o) return APUS_ERROR;
    if (b->n_groups >> 32) {
        apus::log_error("apus_commit_batch: n_groups must be below 2^32\n");
        return APUS_ERROR;
    }
    if ((flags & (APUS_COMMIT_WALK | APUS_COMMIT_CHECKSUM)) && (!b->ring || b->ring_stride % 16)) {
        apus::log_error("apus_commit_batch: ring missing or ring_stride %% 16 != 0\n");
        return APUS_ERROR;
    }
    if ((flags & APUS_COMMIT_MEDIAN) && (!b->remote_end || !b->lr_step || !b->fail_count)) {
        apus::log_error("apus_commit_batch: median needs remote_end, lr_step, fail_count\n");
        return APUS_ERROR;
    }
    if ((flags & APUS_COMMIT_NC) && (!o->nc_dets || !o->nc_len || !o->nc_max || o->nc_max > (1u << 31) ||
                                     ((uintptr_t)o->nc_dets & 7u))) {
        apus::log_error("apus_commit_batch: APUS_COMMIT_NC needs nc_dets (8-B aligned), nc_len and nc_max\n");
        return APUS_ERROR;
    }
    if ((flags & APUS_COMMIT_PRUNE) && (!b->apply_offsets || !b->ring)) {
        apus::log_error("apus_commit_batch: pruning needs apply_offsets and ring\n");
        return APUS_ERROR;
    }
    if ((flags & APUS_COMMIT_LAST_IT) && (!o->last_idx_term || !b->ring)) {
        apus::log_error("apus_commit_batch: APUS_COMMIT_LAST_IT needs last_idx_term and ring\n");
        return APUS_ERROR;
    }
    if ((flags & APUS_COMMIT_VOTE) && !b->vote_ack) {
        apus::log_error("apus_commit_batch: APUS_COMMIT_VOTE needs vote_ack\n");
        return APUS_ERROR;
    }
    if ((flags & APUS_COMMIT_RANK) &&
        (!b->sid || !b->hb || !b->vote_req || !((flags & APUS_COMMIT_LAST_IT) || b->last_idx_term))) {
        apus::log_error("apus_commit_batch: APUS_COMMIT_RANK needs sid, hb, vote_req and APUS_COMMIT_LAST_IT "
                        "or last_idx_term\n");
        return APUS_ERROR;
    }
    const bool walks = (flags & (APUS_COMMIT_WALK | APUS_COMMIT_CHECKSUM)) != 0;
    if ((flags & APUS_COMMIT_PUBLISH) &&
        (!b->remote_end || !b->remote_commit || !b->lr_step || !b->fail_count || (walks && !o->new_commit))) {
        apus::log_error("apus_commit_batch: APUS_COMMIT_PUBLISH needs remote_end, remote_commit, lr_step, fail_count "
                        "(and new_commit when the call walks)\n");
        return APUS_ERROR;
    }
    if ((flags & APUS_COMMIT_FORCE_PRUNE) && (!b->apply_offsets || !b->ring || !b->sid)) {
        apus::log_error("apus_commit_batch: APUS_COMMIT_FORCE_PRUNE needs apply_offsets, ring, sid\n");
        return APUS_ERROR;
    }
    // force_log_pruning runs after apply_committed_entries in polling()
    // (dare_server.c:1100-1123) and starts from log->apply: after a walk that
    // moves commit the leader's apply has not run yet, so the two are not one
    // call (commit call, apus_apply_batch, then a FORCE_PRUNE call)
    if ((flags & APUS_COMMIT_FORCE_PRUNE) && walks) {
        apus::log_error("apus_commit_batch: APUS_COMMIT_FORCE_PRUNE does not combine with a walk: "
                        "apply_committed_entries runs between them (dare_server.c:1100-1123)\n");
        return APUS_ERROR;
    }
    CHECK_HIP(apus::launch_commit(c, *b, *o, flags, (hipStream_t)stream));
    return APUS_OK;
}

int apus_vote_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_vote_out_t *o, apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !o || !b->vote_ack) return APUS_ERROR;
    CHECK_HIP(apus::launch_vote(c, *b, *o, (hipStream_t)stream));
    return APUS_OK;
}

int apus_vote_rank_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_rank_out_t *o, apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !o || !b->sid || !b->hb || !b->vote_req) return APUS_ERROR;
    if (!b->last_idx_term) {
        apus::log_error("apus_vote_rank_batch: last_idx_term required (see apus_last_idx_term_batch)\n");
        return APUS_ERROR;
    }
    CHECK_HIP(apus::launch_rank(c, *b, *o, (hipStream_t)stream));
    return APUS_OK;
}

int apus_last_idx_term_batch(apus_ctx_t *c, const apus_batch_t *b, uint64_t *out, apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !b->ring || !out) return APUS_ERROR;
    CHECK_HIP(apus::launch_last_idx_term(*b, out, (hipStream_t)stream));
    return APUS_OK;
}

int apus_prune_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_prune_out_t *o, apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !o || !b->apply_offsets || !b->ring) return APUS_ERROR;
    CHECK_HIP(apus::launch_prune(c, *b, *o, (hipStream_t)stream));
    return APUS_OK;
}

int apus_validate_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_nc_batch_t *nc, uint64_t *out,
                        apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !nc || !out || !b->ring || !b->remote_commit) return APUS_ERROR;
    if (nc->max_dets > APUS_MAX_NC_ENTRIES || !nc->dets || !nc->det_len || !nc->follower) return APUS_ERROR;
    if (nc->n_followers > APUS_MAX_SERVER_COUNT || ((uintptr_t)nc->dets & 7u)) return APUS_ERROR;
    if (nc->leader_dets && (!nc->leader_len || !nc->leader_max || ((uintptr_t)nc->leader_dets & 7u))) {
        apus::log_error("apus_validate_batch: leader_dets needs leader_len, leader_max and 8-B alignment\n");
        return APUS_ERROR;
    }
    CHECK_HIP(apus::launch_validate(c, *b, *nc, out, (hipStream_t)stream));
    return APUS_OK;
}

int apus_nc_build_batch(apus_ctx_t *c, const apus_batch_t *b, apus_entry_det_t *dets, uint32_t max_dets,
                        uint32_t *len, apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !b->ring || !dets || !len) return APUS_ERROR;
    CHECK_HIP(apus::launch_nc_build(c, *b, dets, max_dets, len, (hipStream_t)stream));
    return APUS_OK;
}

int apus_append_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_append_in_t *in,
                      const apus_append_out_t *o, apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !in || !o || !b->ring) return APUS_ERROR;
    if (in->max_entries && !in->entries) return APUS_ERROR;
    if (!in->term && !b->sid) return APUS_ERROR;
    if (in->payload_bytes && !in->payload) return APUS_ERROR;
    CHECK_HIP(apus::launch_append(c, *b, *in, *o, (hipStream_t)stream));
    return APUS_OK;
}

int apus_persist_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_persist_in_t *in, apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !in || !in->old_end || !b->ring || !b->self_idx) return APUS_ERROR;
    CHECK_HIP(apus::launch_persist(c, *b, *in, (hipStream_t)stream));
    return APUS_OK;
}

int apus_config_scan_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_config_io_t *io,
                           apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !io || !b->ring) return APUS_ERROR;
    if (!io->cid_offset || !io->cid_idx || !io->req_id || !io->clt_id) return APUS_ERROR;
    CHECK_HIP(apus::launch_config_scan(c, *b, *io, (hipStream_t)stream));
    return APUS_OK;
}

int apus_apply_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_apply_io_t *io, apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !io || !b->ring || !b->self_idx || !b->sid) return APUS_ERROR;
    if (!io->req_id || !io->clt_id || !io->last_applied || !io->last_csm_idx || !io->n_cfg) return APUS_ERROR;
    if (io->max_cfg && (!io->cfg_entries || !io->cfg_payload)) return APUS_ERROR;
    CHECK_HIP(apus::launch_apply(c, *b, *io, (hipStream_t)stream));
    return APUS_OK;
}

int apus_vote_win_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_win_io_t *io, apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !io || !b->ring || !b->sid || !b->vote_ack || !b->remote_commit || !b->lr_step ||
        !b->apply_offsets)
        return APUS_ERROR;
    if (!io->won || !io->voters || !io->new_commit || !io->cid_offset || !io->cid_idx || !io->req_id ||
        !io->clt_id || !io->last_applied || !io->last_csm_idx || !io->last_write_csm_idx || !io->outcome)
        return APUS_ERROR;
    CHECK_HIP(apus::launch_vote_win(c, *b, *io, (hipStream_t)stream));
    return APUS_OK;
}

int apus_lr_completion_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_lr_io_t *io, apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !io || !b->lr_step || !io->wc || !io->send_flag || !io->send_count)
        return APUS_ERROR;
    CHECK_HIP(apus::launch_lr_completion(c, *b, *io, (hipStream_t)stream));
    return APUS_OK;
}

int apus_log_adjust_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_lr_io_t *io, apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !io || !b->ring || !b->self_idx || !b->fail_count || !b->lr_step || !b->vote_ack ||
        !b->remote_commit || !b->remote_end)
        return APUS_ERROR;
    if (!io->send_flag || !io->nc_len || !io->ssn || !io->post) return APUS_ERROR;
    if (io->max_dets > APUS_MAX_NC_ENTRIES || (io->max_dets && !io->nc_dets) || ((uintptr_t)io->nc_dets & 7u))
        return APUS_ERROR;
    // an NC buffer without a row length would skip every LR_SET_END walk
    // (log_find_remote_end_offset, dare_ibv_rc.c:1406-1422): refuse it
    if (io->nc_dets && io->max_dets == 0) {
        apus::log_error("apus_log_adjust_batch: nc_dets given with max_dets == 0\n");
        return APUS_ERROR;
    }
    CHECK_HIP(apus::launch_log_adjust(c, *b, *io, (hipStream_t)stream));
    return APUS_OK;
}

int apus_records_store_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_records_io_t *io,
                             apus_stream_t stream)
{
    if (!c || !batch_ok(b) || !io || !b->ring || !io->cursor || !io->dump_len) return APUS_ERROR;
    if (io->cap && !io->dump) return APUS_ERROR;
    if (io->cap > 0xFFFFFFFFull) {                  // records_len is a uint32_t (db-interface.c:21)
        apus::log_error("apus_records_store_batch: cap must fit records_len (uint32_t)\n");
        return APUS_ERROR;
    }
    CHECK_HIP(apus::launch_records_store(c, *b, *io, (hipStream_t)stream));
    return APUS_OK;
}

int apus_records_load_batch(apus_ctx_t *c, const apus_records_load_io_t *io, apus_stream_t stream)
{
    if (!c || !io || !io->size || !io->n_records || !io->status) return APUS_ERROR;
    if (io->n && !io->dump) return APUS_ERROR;
    if (io->max_plan && !io->plan) return APUS_ERROR;
    if (((uintptr_t)io->plan & 3u) || ((uintptr_t)io->counts & 3u)) return APUS_ERROR;
    CHECK_HIP(apus::launch_records_load(c, *io, (hipStream_t)stream));
    return APUS_OK;
}

int apus_gen_batch(apus_ctx_t *c, const apus_batch_t *b, const apus_gen_cfg_t *cfg, apus_stream_t stream)
{
    if (!c || !rows_ok(b) || !cfg || !b->ring) return APUS_ERROR;
    hipError_t e = apus::launch_gen(c, *b, *cfg, (hipStream_t)stream);
    if (e != hipSuccess) {
        apus::log_error("apus_gen_batch: %s\n", hipGetErrorString(e));
        return APUS_ERROR;
    }
    return APUS_OK;
}

// ---------------------------------------------------------------------------
// RCCL
// ---------------------------------------------------------------------------
int apus_comm_get_unique_id(char id_out[128])
{
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return APUS_ERROR;
    memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return APUS_OK;
}

int apus_comm_init_rank(apus_ctx_t *c, int nranks, const char id[128], int rank)
{
    if (!c) return APUS_ERROR;
    ncclUniqueId uid;
    memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t comm;
    CHECK_HIP(hipSetDevice(c->device));
    if (ncclCommInitRank(&comm, nranks, uid, rank) != ncclSuccess) {
        apus::log_error("ncclCommInitRank failed\n");
        return APUS_ERROR;
    }
    c->comm = comm;
    return APUS_OK;
}

int apus_stats_allreduce(apus_ctx_t *c, apus_stream_t stream)
{
    if (!c || !c->comm) return APUS_ERROR;
    ncclComm_t comm = (ncclComm_t)c->comm;
    hipStream_t s = (hipStream_t)stream;
    // one fused launch: SUM over the counters, MIN over the watermark
    static_assert(APUS_STAT_SLOW == APUS_STAT_MIN_WATERMARK + 1 && APUS_STAT_COUNT > APUS_STAT_SLOW,
                  "stats layout: sums, the watermark (min), sums");
    if (ncclGroupStart() != ncclSuccess) return APUS_ERROR;
    ncclResult_t r = ncclAllReduce(c->stats, c->stats, APUS_STAT_MIN_WATERMARK, ncclUint64, ncclSum, comm, s);
    if (r == ncclSuccess)
        r = ncclAllReduce(c->stats + APUS_STAT_MIN_WATERMARK, c->stats + APUS_STAT_MIN_WATERMARK, 1, ncclUint64,
                          ncclMin, comm, s);
    if (r == ncclSuccess)
        r = ncclAllReduce(c->stats + APUS_STAT_SLOW, c->stats + APUS_STAT_SLOW, APUS_STAT_COUNT - APUS_STAT_SLOW,
                          ncclUint64, ncclSum, comm, s);
    const ncclResult_t g = ncclGroupEnd();
    return (r == ncclSuccess && g == ncclSuccess) ? APUS_OK : APUS_ERROR;
}

int apus_allreduce_stats(apus_ctx_t *c, apus_stream_t stream) { return apus_stats_allreduce(c, stream); }

}  // extern "C"

// ---------------------------------------------------------------------------
// scalar drop-ins
// ---------------------------------------------------------------------------
namespace {

// device image of one group for the scalar calls (all [1][13] arrays)
struct ScalarIn {
    apus_group_state_t st;
    uint64_t remote_end[APUS_MAX_SERVER_COUNT];
    uint64_t remote_commit[APUS_MAX_SERVER_COUNT];
    uint64_t vote_ack[APUS_MAX_SERVER_COUNT];
    uint64_t apply_offsets[APUS_MAX_SERVER_COUNT];
    uint64_t hb[APUS_MAX_SERVER_COUNT];
    apus_vote_req_t vote_req[APUS_MAX_SERVER_COUNT];
    uint64_t sid;
    uint64_t lit[2];
    uint8_t lr_step[APUS_MAX_SERVER_COUNT];
    uint8_t fail_count[APUS_MAX_SERVER_COUNT];
    uint8_t self;
    uint8_t prev_head;
    uint8_t pad[4];
};
struct ScalarOut {
    uint64_t new_commit, median, u64a, u64b;
    uint32_t n_entries, digest, len;
    uint16_t u16a;
    uint8_t committed, u8a, u8b[2];
    apus_cid_t cid;
};

// determinant scratch: one dare_nc_buf_t worth per server (log_adjustment's
// LR_SET_END walks read log->nc_buf[i]); find_remote_end / nc_build use row 0
constexpr size_t kScalarDets = (size_t)APUS_MAX_SERVER_COUNT * APUS_MAX_NC_ENTRIES;
// step-machine columns of the scalar log_adjustment / completion
struct ScalarLr {
    uint64_t nc_len[APUS_MAX_SERVER_COUNT];
    uint64_t ssn;
    uint16_t rc_connected;
    uint8_t send_flag[APUS_MAX_SERVER_COUNT];
    uint8_t send_count[APUS_MAX_SERVER_COUNT];
    uint8_t wc[APUS_MAX_SERVER_COUNT];
    uint8_t post[APUS_MAX_SERVER_COUNT];
};
constexpr size_t kScalarLrOff = 4096 + kScalarDets * sizeof(apus_entry_det_t);
constexpr size_t kScalarBytes = kScalarLrOff + 512;
// the one-launch scalar calls' mapped pages: results, then the ring window
constexpr size_t kQPages = 4096;
static_assert(sizeof(ScalarLr) <= 512, "scratch layout");

int default_ctx(apus_ctx **out)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (!g_default) {
        const char *d = getenv("APUS_DEVICE");
        apus_ctx *c = nullptr;
        if (apus_ctx_create(d ? atoi(d) : 0, &c) != APUS_OK) return APUS_ERROR;
        if (hipMalloc(&c->s_buf, kScalarBytes) != hipSuccess) return APUS_ERROR;
        if (hipHostMalloc(&c->h_pinned, kScalarBytes, hipHostMallocDefault) != hipSuccess) return APUS_ERROR;
        if (hipStreamCreateWithFlags(&c->s_stream, hipStreamNonBlocking) != hipSuccess) return APUS_ERROR;
        void *qd = nullptr;
        // coherent by request, not by default: the one-launch scalar calls'
        // result handshake relies on it (scalar_q_kernel / q_run)
        if (hipHostMalloc((void **)&c->q_host, kQPages, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
            hipHostGetDevicePointer(&qd, c->q_host, 0) != hipSuccess)
            return APUS_ERROR;
        memset(c->q_host, 0, kQPages);
        c->q_dev = (uint8_t *)qd;
        c->s_cap = kScalarBytes;
        c->h_cap = kScalarBytes;
        g_default = c;
    }
    (void)hipSetDevice(g_default->device);
    *out = g_default;
    return APUS_OK;
}

// The staging image: a pinned, mapped buffer of the default context holding
// copies of the caller's ring bytes at their own offsets.  A call stages the
// circular ranges the reference's walk reads for it (every entry of a log
// built by log_append_entry lies in [head, end)) and the 64-B headers at the
// offsets it looks up; the kernels read the image in place.  Bytes outside the
// staged ranges are not the caller's: only a corrupt log, whose entry chain
// leaves [head, end), would read them (apus_log_new logs are read in place and
// have no such limit).  They hold kPoison, whatever earlier calls staged: the
// ranges a call staged are poisoned again when it ends (unpoison), so a
// chain that leaves the staged ranges reads the same bytes on every call,
// never another log's: its results are deterministic.  They are not
// necessarily a rejection: a poison header (type 0xFF, cmd.len 0xFFFF) is an
// entry of 65,599 B, which fits a log of 64 KiB or more, so such a chain may
// walk on through poison "entries" (their reply bytes are 0xFF, never an ack:
// the reply walk stops at the first one) until the step guard or end.
constexpr uint8_t kPoison = 0xFF;
struct Stager {
    const uint8_t *src;    // the caller's entries[]
    uint8_t *dst;          // the staging image (host side)
    uint64_t len;
    uint64_t bytes = 0;
    // the ranges staged (no allocation per call: past kRanges, their extent)
    static constexpr int kRanges = 64;
    uint64_t ra[kRanges], rb[kRanges];
    int nr = 0;
    uint64_t lo = ~0ull, hi = 0;

    void range(uint64_t a, uint64_t b)
    {
        if (b > len) b = len;
        if (a >= b) return;
        memcpy(dst + a, src + a, b - a);
        bytes += b - a;
        if (a < lo) lo = a;
        if (b > hi) hi = b;
        for (int i = 0; i < nr && nr <= kRanges; ++i)
            if (ra[i] <= a && b <= rb[i]) return;
        if (nr < kRanges) { ra[nr] = a; rb[nr] = b; }
        ++nr;
    }
    // the staged bytes back to kPoison (the call's kernels have finished)
    void unpoison()
    {
        if (nr > kRanges) {
            memset(dst + lo, kPoison, hi - lo);
        } else {
            for (int i = 0; i < nr; ++i) memset(dst + ra[i], kPoison, rb[i] - ra[i]);
        }
        nr = 0;
        lo = ~0ull;
        hi = 0;
    }
    // the entries log_get_entry returns from `from` while dist > 0
    // (dare_log.h:255-262, 316-332); an empty log (end == len) has none
    void chain(uint64_t from, uint64_t end)
    {
        if (end >= len || from == end) return;
        if (from < end) {
            range(from, end);
        } else {
            range(from, len);
            range(0, end);
        }
        range(0, 64);      // a header that does not fit is read at 0
    }
    // one entry header looked up at `o` (log_get_entry: at 0 when it does not fit)
    void header(uint64_t o)
    {
        if (o < len) range(o, o + 64);
        range(0, 64);
    }
    // log_get_tail (dare_log.h:402-457): the tail entry, or the scans from
    // commit, apply and head
    void tail(const apus_group_state_t &st)
    {
        if (st.tail != st.len) {
            header(st.tail);
            return;
        }
        chain(st.commit, st.end);
        chain(st.apply, st.end);
        chain(st.head, st.end);
    }
};

void fill_state(apus_group_state_t &st, const apus_log_t *log, const apus_server_config_t *cfg)
{
    st.head = log->head;
    st.apply = log->apply;
    st.commit = log->commit;
    st.end = log->end;     // snapshot `end` once (dare_log.h:258,274)
    st.tail = log->tail;
    st.len = log->len;
    st.cid = cfg->cid;
}

// the device address of a log the library allocated (apus_log_new), else null
uint8_t *owned_ring(const apus_log_t *log)
{
    std::lock_guard<std::mutex> lk(g_mu);
    for (const OwnedLog &o : g_owned)
        if (o.host == log) return o.dev + offsetof(apus_log_t, entries);
    return nullptr;
}

// the staging image holds at least `len` ring bytes plus the 16-B tail the
// window loads may read past len; grown only between calls (every scalar call
// has synchronised its stream before it returns)
int ensure_stage(apus_ctx *c, uint64_t len)
{
    const size_t need = ((size_t)len + 64 + 4095) & ~(size_t)4095;
    if (c->stage_cap >= need) return APUS_OK;
    if (c->stage) (void)hipHostFree(c->stage);
    c->stage = nullptr;
    c->stage_dev = nullptr;
    c->stage_cap = 0;
    void *h = nullptr, *d = nullptr;
    CHECK_HIP(hipHostMalloc(&h, need, hipHostMallocMapped));
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(h);
        apus::log_error("staging image: no device address\n");
        return APUS_ERROR;
    }
    c->stage = (uint8_t *)h;
    c->stage_dev = (uint8_t *)d;
    c->stage_cap = need;
    memset(h, kPoison, need);
    return APUS_OK;
}

// build a G=1 batch over the scratch image; returns host/device views
struct Scalar {
    std::unique_lock<std::mutex> lk;   // c->scalar_mu, held until the call returns
    apus_ctx *c;
    ScalarIn *hin;
    ScalarOut *hout;
    ScalarIn *din;
    ScalarOut *dout;
    apus_entry_det_t *ddets, *hdets;
    apus_batch_t b;
    bool staged = false;               // false: an apus_log_new log, read in place
    Stager stg;                        // the ranges this call reads (staged logs)

    // the staged ranges are poisoned again once the call's work has drained
    // (scalar_finish synchronised the stream; an early error return has not)
    ~Scalar()
    {
        if (staged && stg.nr) {
            (void)hipStreamSynchronize(c->s_stream);
            stg.unpoison();
        }
    }

    // stage what a walk from `from` reads, the tail lookup, one header
    void chain(uint64_t from) { if (staged) stg.chain(from, hin->st.end); }
    void tail() { if (staged) stg.tail(hin->st); }
    void header(uint64_t o) { if (staged) stg.header(o); }
};

int scalar_begin(Scalar &s, const apus_log_t *log, const apus_server_config_t *cfg)
{
    if (!log || !cfg) return APUS_ERROR;
    if (default_ctx(&s.c) != APUS_OK) return APUS_ERROR;
    s.lk = std::unique_lock<std::mutex>(s.c->scalar_mu);
    s.hin = (ScalarIn *)s.c->h_pinned;
    s.hout = (ScalarOut *)(s.c->h_pinned + 2048);
    s.hdets = (apus_entry_det_t *)(s.c->h_pinned + 4096);
    s.din = (ScalarIn *)s.c->s_buf;
    s.dout = (ScalarOut *)(s.c->s_buf + 2048);
    s.ddets = (apus_entry_det_t *)(s.c->s_buf + 4096);
    static_assert(sizeof(ScalarIn) <= 2048 && sizeof(ScalarOut) <= 2048, "scratch layout");
    memset(s.hin, 0, sizeof(ScalarIn));
    memset(s.hout, 0, sizeof(ScalarOut));
    fill_state(s.hin->st, log, cfg);
    s.hin->self = cfg->idx;
    memset(&s.b, 0, sizeof s.b);
    s.b.n_groups = 1;
    s.b.n_replicas = APUS_MAX_SERVER_COUNT;
    const uint64_t len = s.hin->st.len;
    // stride == len: the window loads of commit_wave_kernel then never read
    // more than 16 B past the ring (apus_commit.hip `lim`)
    s.b.ring_stride = len;
    s.b.ring = owned_ring(log);
    s.staged = s.b.ring == nullptr;
    if (s.staged) {
        if (ensure_stage(s.c, len) != APUS_OK) return APUS_ERROR;
        s.stg = Stager{log->entries, s.c->stage, len};
        s.b.ring = s.c->stage_dev;
        ++g_calls_staged;
    } else {
        ++g_calls_in_place;
    }
    s.b.state = &s.din->st;
    s.b.self_idx = &s.din->self;
    s.b.remote_end = s.din->remote_end;
    s.b.remote_commit = s.din->remote_commit;
    s.b.lr_step = s.din->lr_step;
    s.b.fail_count = s.din->fail_count;
    s.b.vote_ack = s.din->vote_ack;
    s.b.apply_offsets = s.din->apply_offsets;
    s.b.vote_req = s.din->vote_req;
    s.b.hb = s.din->hb;
    s.b.sid = &s.din->sid;
    s.b.last_idx_term = s.din->lit;
    s.b.prev_head = &s.din->prev_head;
    return APUS_OK;
}

int scalar_upload(Scalar &s)
{
    if (s.staged) g_bytes_staged += s.stg.bytes;
    CHECK_HIP(hipMemcpyAsync(s.din, s.hin, sizeof(ScalarIn), hipMemcpyHostToDevice, s.c->s_stream));
    return APUS_OK;
}

int scalar_finish(Scalar &s, size_t n_dets = 0, bool inputs_back = false)
{
    CHECK_HIP(hipMemcpyAsync(s.hout, s.dout, sizeof(ScalarOut), hipMemcpyDeviceToHost, s.c->s_stream));
    // the kernels that update ctrl_data in place, as the reference does
    if (inputs_back)
        CHECK_HIP(hipMemcpyAsync(s.hin, s.din, sizeof(ScalarIn), hipMemcpyDeviceToHost, s.c->s_stream));
    if (n_dets)
        CHECK_HIP(hipMemcpyAsync(s.hdets, s.ddets, n_dets * sizeof(apus_entry_det_t), hipMemcpyDeviceToHost,
                                 s.c->s_stream));
    CHECK_HIP(hipStreamSynchronize(s.c->s_stream));
    return APUS_OK;
}

// ---------------------------------------------------------------------------
// One-launch scalar calls.  The staged path above makes a call
// an H2D copy of the scratch, one to three launches, a D2H copy and a stream
// synchronisation (23-43 us).  Here the group's state and columns travel in
// the kernel arguments (256 B), and -- for the reply walk and log_get_tail --
// the ring bytes the staging would copy ([commit, end), wrapped, and the
// header at 0) as a window of at most kQWin bytes after them, in the smallest
// of five argument sizes that holds it (a window read by the kernel from the
// mapped page instead made the walk 2.4 us slower: one PCIe round trip more
// than the runtime's argument copy, profiles/r05/scalar/).  Lane 0 computes
// into LDS; the lanes store the results to the context's pinned mapped page
// write-through at system scope (no L2 write-back: a system-scope release
// fence writes back the whole L2, about 1.7 us clean), wait for them, and
// lane 0 then stores the call's sequence number, which the caller waits on.
// One launch, no copy, no synchronisation call.  Bytes outside the window
// read as kPoison, exactly as bytes outside the staged ranges do; a walk that
// reads one on a log the library owns (read in place by the staged path) is
// redone on that path.
// ---------------------------------------------------------------------------
using namespace apus;
constexpr uint32_t kQWin = 3072;
constexpr uint8_t kQWalk = 1, kQMedian = 2, kQVote = 3, kQPrune = 4, kQPublish = 5;
struct QArgs {
    apus_group_state_t st;
    uint64_t col[APUS_MAX_SERVER_COUNT];     // remote_end (median), vote_ack (vote), apply_offsets (pruning),
                                             // log_offsets[i].commit (publish)
    uint64_t col2[APUS_MAX_SERVER_COUNT];    // log_offsets[i].end (publish)
    uint16_t conn;                           // rc_connected bits (publish)
    uint16_t pad3[3];
    uint8_t step[APUS_MAX_SERVER_COUNT], fail[APUS_MAX_SERVER_COUNT];
    uint8_t self, op, prev, pad;
    uint32_t seq;
    uint32_t bytes;                          // of this struct the kernel reads: the header and the window used
    uint32_t pad2;
    uint64_t seg[4];                         // the window: ring [seg0, seg1), then [seg2, seg3)
    alignas(16) uint8_t win[kQWin];
};
static_assert(offsetof(QArgs, win) + 24 <= 4096, "kernel arguments");
static_assert(offsetof(QArgs, win) % 16 == 0, "16-B copy");
// what a launch passes: QArgs' header and a window of W bytes (the smallest
// of 0, 512, 1152, 2048, 3072 that holds the call's window: the reply walk
// of 8 x 128-B entries reads 1,088 B)
template <uint32_t W>
struct QArgsT {
    uint8_t head[offsetof(QArgs, win)];
    uint8_t win[W ? W : 16];
};
static_assert(sizeof(QArgsT<0>) % 16 == 0 && sizeof(QArgsT<1152>) % 16 == 0, "16-B chunks");
struct QRes {
    uint64_t new_commit, median, vote_commit, new_head, min_apply;
    uint64_t col[APUS_MAX_SERVER_COUNT];     // publish: the servers' commit offsets after it
    uint32_t n_entries;
    uint16_t voters, reset;                  // reset: the OFF servers whose apply offset became log->apply
    uint8_t committed, won, vc[2], outside, append;
    uint8_t pad[2];
    uint32_t seq;                            // stored last
    uint32_t pad4;
};
static_assert(sizeof(QRes) % 8 == 0 && offsetof(QRes, seq) == sizeof(QRes) - 8, "result words, seq last");

__device__ __forceinline__ uint32_t qbyte(const QArgs &a, uint64_t o, bool &outside)
{
    if (o >= a.seg[0] && o < a.seg[1]) return a.win[o - a.seg[0]];
    if (o >= a.seg[2] && o < a.seg[3]) return a.win[(a.seg[1] - a.seg[0]) + (o - a.seg[2])];
    outside = true;
    return kPoison;
}

// log_get_tail (dare_log.h:402-457) over the window
__device__ uint64_t q_get_tail(const QArgs &a, const apus_group_state_t &st, bool &outside)
{
    if (st.tail != st.len) return st.tail;
    if (st.end == st.len) return st.len;
    const uint64_t len = st.len, end = st.end, guard = len / kHdr + 4;
    const uint64_t starts[3] = { st.commit, st.apply, st.head };
    for (int s = 0; s < 3; ++s) {
        uint64_t o = starts[s], tail = len, n = 0;
        for (;;) {
            if (dist(end, len, o) == 0) break;                          // log_get_entry: NULL
            if (len - o < kHdr) o = 0;
            if (!(o <= len - kHdr) || n++ >= guard) break;
            tail = o;
            const uint32_t el = entry_len(qbyte(a, o + kType, outside),
                                          qbyte(a, o + kData, outside) | (qbyte(a, o + kData + 1, outside) << 8));
            if (len - o < el) o = 0;
            o += el;
        }
        if (tail != len) return tail;
    }
    return len;
}

// the computation of a one-launch scalar call (lane 0), results into r
__device__ __forceinline__ void scalar_q_compute(const QArgs &a, QRes *r)
{
    const apus_group_state_t st = a.st;
    const uint32_t self = a.self;
    if (a.op == kQWalk) {
        // the APUS reply walk, as lane_group walks it (dare_ibv_rc.c:1725-1758)
        const uint64_t len = st.len, end = st.end, commit0 = st.commit;
        const uint32_t size = walk_size(st.cid), need = size / 2 + 1;
        const uint64_t guard = len / kHdr + 4;
        uint64_t m = commit0, steps = 0;
        uint32_t n = 0;
        bool outside = false, corrupt = commit0 > len || end > len;
        while (!corrupt && dist(end, len, m)) {
            if (++steps > guard) { corrupt = true; break; }
            if (len - m < kHdr) m = 0;                                   // log_get_entry
            // a header wholly inside one window segment: its bytes read
            // together, unconditionally (one LDS round trip per entry); else
            // byte by byte in the reference's order (a ghost header's replies
            // are not read)
            int64_t hb = -1;
            if (m >= a.seg[0] && m + kHdr <= a.seg[1]) hb = (int64_t)(m - a.seg[0]);
            else if (m >= a.seg[2] && m + kHdr <= a.seg[3]) hb = (int64_t)((a.seg[1] - a.seg[0]) + (m - a.seg[2]));
            uint32_t type, clen, rb[16];
            if (hb >= 0) {
                const uint8_t *h = a.win + hb;
                type = h[kType];
                clen = h[kData] | ((uint32_t)h[kData + 1] << 8);
#pragma unroll
                for (uint32_t i = 0; i < 16; ++i) rb[i] = h[kReply + i];
            } else {
                type = qbyte(a, m + kType, outside);
                clen = qbyte(a, m + kData, outside) | (qbyte(a, m + kData + 1, outside) << 8);
            }
            const uint32_t elen = entry_len(type, clen);
            if (len - m < elen) { m = 0; continue; }                     // ghost header
            if (hb < 0) {
#pragma unroll
                for (uint32_t i = 0; i < 16; ++i) rb[i] = i < size && i != self ? qbyte(a, m + kReply + i, outside) : 0u;
            }
            uint32_t votes = 0;
#pragma unroll
            for (uint32_t i = 0; i < 16; ++i) votes += (i < size && (i == self || rb[i] == 1)) ? 1u : 0u;
            for (uint32_t i = 16; i < size; ++i) votes += (i == self || qbyte(a, m + kReply + i, outside) == 1) ? 1u : 0u;
            if (votes < need) break;
            ++n;
            m += elen;
        }
        const bool adv = !corrupt && larger(end, len, m, commit0);
        r->new_commit = adv ? m : commit0;
        r->committed = corrupt ? 0xFF : (uint8_t)adv;
        r->n_entries = n;
        r->outside = outside ? 1 : 0;
    } else if (a.op == kQMedian) {
        // the DARE median (dare_ibv_rc.c:1650-1723), as the tail computes it for R = 13
        // (both sizes at most 8: the slots past 8 hold no replica and sort
        // last, so 8 slots give the value at rank (size - 1) / 2 -- median_of's
        // argument; 64 rank comparisons instead of 240)
        if (st.cid.size[0] <= 8 && st.cid.size[1] <= 8) {
            QuorumIn<8> q;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                q.rend[i] = a.col[i];
                q.step[i] = a.step[i];
                q.fail[i] = a.fail[i];
                q.ap[i] = 0;
            }
            q.self = self;
            q.prev = 0;
            q.base = ~0ull;
            r->median = median_slots<8, 8>(APUS_MAX_SERVER_COUNT, st, q);
        } else {
            QuorumIn<16> q;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                q.rend[i] = i < APUS_MAX_SERVER_COUNT ? a.col[i] : 0;
                q.step[i] = i < APUS_MAX_SERVER_COUNT ? a.step[i] : 0;
                q.fail[i] = i < APUS_MAX_SERVER_COUNT ? a.fail[i] : 0;
                q.ap[i] = 0;
            }
            q.self = self;
            q.prev = 0;
            q.base = ~0ull;
            r->median = median_of<16, 16>(APUS_MAX_SERVER_COUNT, st, q);
        }
    } else if (a.op == kQPublish) {
        // update_remote_logs' lazy remote-commit publish (dare_ibv_rc.c:1760-1822), as publish_from
        const uint32_t size = walk_size(st.cid);
        uint32_t mask = 0;
        for (uint32_t i = 0; i < APUS_MAX_SERVER_COUNT; ++i) {
            uint64_t rc = a.col[i];
            if (i < size && i != self && ((st.cid.bitmask >> i) & 1u) && a.fail[i] < APUS_PERMANENT_FAILURE &&
                ((a.conn >> i) & 1u) && a.step[i] == APUS_LR_UPDATE_LOG && rc != a.col2[i] && rc != st.commit) {
                rc = larger(st.end, st.len, st.commit, a.col2[i]) ? a.col2[i] : st.commit;
                mask |= 1u << i;
            }
            r->col[i] = rc;
        }
        r->voters = (uint16_t)mask;
    } else if (a.op == kQPrune) {
        // log_pruning's minimum (dare_server.c:2026-2058), as prune_calc computes it for R = 13
        const uint32_t size = ext_group_size(st.cid);
        uint64_t mn = st.apply;
        uint32_t reset = 0;
        bool outside = false;
        for (uint32_t i = 0; i < APUS_MAX_SERVER_COUNT; ++i) {
            if (i >= size) continue;
            uint64_t v = a.col[i];
            if (!((st.cid.bitmask >> i) & 1u)) { v = st.apply; reset |= 1u << i; }    // OFF server
            if (larger(st.end, st.len, mn, v)) mn = v;
        }
        if (dist(st.end, st.len, mn) == 0) mn = q_get_tail(a, st, outside);
        const bool app = larger(st.end, st.len, mn, st.head) && !a.prev;
        r->new_head = app ? mn : st.head;
        r->append = app ? 1 : 0;
        r->min_apply = mn;
        r->reset = (uint16_t)reset;
        r->outside = outside ? 1 : 0;
    } else {
        // poll_vote_count's tally (dare_server.c:1330-1373), vote_from on the arguments
        apus_batch_t b;
        __builtin_memset(&b, 0, sizeof b);
        b.n_groups = 1;
        b.n_replicas = APUS_MAX_SERVER_COUNT;
        FailIn<16> f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            f.ack[i] = i < APUS_MAX_SERVER_COUNT ? a.col[i] : ~0ull;
            f.hb[i] = f.rs[i] = f.ri[i] = f.rt[i] = 0;
        }
        f.sid = 0;
        f.lrec = nullptr;
        apus_vote_out_t o;
        o.won = &r->won;
        o.vote_count = r->vc;
        o.new_commit = &r->vote_commit;
        o.voters = &r->voters;
        (void)vote_from<16, false>(b, 0, st, self, f, o);
    }
}

// The reply walk with the wave (the common case: every header inside the
// window, at most 64 entries, sizes at most 16): the lanes check at once the
// chain that speculates every entry has the first one's length (lane k: the
// header at m0 + k * e0), lane 0 follows the rest of the chain alone
// (log_get_entry's wrap, the ghost-header jump, the step guard), recording
// each entry's window position; then lane k counts entry k's replies and a
// ballot finds the first entry short of a quorum -- the entry the serial walk
// stops at, with the same offsets, count and flags.  Any
// other case returns false: lane 0 runs the exact serial walk
// (scalar_q_compute).  One LDS round trip per entry on lane 0 instead of the
// header and its 16 reply bytes (lane 0's vote arithmetic was 0.5 us per
// entry: profiles/r05/scalar/).
__device__ __forceinline__ bool q_walk_wave(const QArgs &a, QRes *r)
{
    constexpr uint32_t kMaxE = 64;
    __shared__ uint32_t pos[kMaxE];          // entry k's header: its window offset
    __shared__ uint64_t moff[kMaxE + 1];     // entry k's ring offset; [n]: where the chain ended
    __shared__ uint32_t nent, ok, s_e0, s_k;
    __shared__ uint64_t s_m0;
    const apus_group_state_t st = a.st;
    const uint32_t size = walk_size(st.cid), need = size / 2 + 1, self = a.self;
    const uint64_t len = st.len, end = st.end, commit0 = st.commit;
    const bool sane = size <= 16 && !(commit0 > len || end > len);
    // a header wholly inside one window segment: its window offset
    auto wpos = [&](uint64_t m, uint32_t &hb) -> bool {
        if (m >= a.seg[0] && m + kHdr <= a.seg[1]) { hb = (uint32_t)(m - a.seg[0]); return true; }
        if (m >= a.seg[2] && m + kHdr <= a.seg[3]) {
            hb = (uint32_t)((a.seg[1] - a.seg[0]) + (m - a.seg[2]));
            return true;
        }
        return false;
    };
    // 1. the first entry (lane 0), the speculation's base: the chain from it,
    // if every entry has its length (lane k reads the header at m0 + k * e0
    // and checks it), as the batched walks speculate
    if (threadIdx.x == 0) {
        s_e0 = 0;
        if (sane && dist(end, len, commit0)) {
            uint64_t m = commit0;
            if (len - m < kHdr) m = 0;                                   // log_get_entry
            uint32_t hb;
            if (wpos(m, hb)) {
                const uint8_t *h = a.win + hb;
                const uint32_t e = entry_len(h[kType], h[kData] | ((uint32_t)h[kData + 1] << 8));
                if (len - m >= e) { s_m0 = m; s_e0 = e; }                // (a ghost header: the serial walk)
            }
        }
    }
    __syncthreads();
    {
        const uint32_t e0 = s_e0, k = threadIdx.x;
        uint32_t K = 0;
        if (e0) {
            const uint64_t m0 = s_m0, c = m0 + (uint64_t)k * e0;
            // before end on the chain, no wrap, inside the window, the same length
            bool okk = (m0 < end ? c < end : true) && c + e0 <= len;
            uint32_t hb = 0;
            okk = okk && wpos(c, hb);
            if (okk) {
                const uint8_t *h = a.win + hb;
                okk = entry_len(h[kType], h[kData] | ((uint32_t)h[kData + 1] << 8)) == e0;
            }
            const uint64_t bad = __ballot(!okk);
            K = bad ? (uint32_t)__builtin_ctzll(bad) : 64u;
            if (k < K) { pos[k] = hb; moff[k] = c; }
        }
        if (threadIdx.x == 0) s_k = K;
    }
    __syncthreads();
    // 2. lane 0: the rest of the chain (log_get_entry's wrap, the ghost-header
    // jump, the step guard), recording each entry's window position
    if (threadIdx.x == 0) {
        const uint64_t guard = len / kHdr + 4;
        const uint32_t K = s_k;
        uint64_t m = K ? s_m0 + (uint64_t)K * s_e0 : commit0, steps = K;
        uint32_t n = K, good = sane && steps <= guard;
        while (good && dist(end, len, m)) {
            if (++steps > guard) { good = 0; break; }
            if (len - m < kHdr) m = 0;                                   // log_get_entry
            uint32_t hb;
            if (!wpos(m, hb)) { good = 0; break; }
            const uint8_t *h = a.win + hb;
            const uint32_t elen = entry_len(h[kType], h[kData] | ((uint32_t)h[kData + 1] << 8));
            if (len - m < elen) { m = 0; continue; }                     // ghost header
            if (n == kMaxE) { good = 0; break; }
            pos[n] = hb;
            moff[n] = m;
            ++n;
            m += elen;
        }
        moff[n < kMaxE + 1 ? n : kMaxE] = m;
        nent = n;
        ok = good;
    }
    __syncthreads();
    if (!ok) return false;
    const uint32_t n = nent, k = threadIdx.x;
    bool pass = true;
    if (k < n) {
        const uint8_t *h = a.win + pos[k] + kReply;
        uint32_t votes = 0;
#pragma unroll
        for (uint32_t i = 0; i < 16; ++i) votes += (i < size && (i == self || h[i] == 1)) ? 1u : 0u;
        pass = votes >= need;
    }
    const uint64_t fail = __ballot(!pass);
    if (threadIdx.x == 0) {
        const uint32_t k0 = fail ? (uint32_t)__builtin_ctzll(fail) : n;   // the first entry short of a quorum
        const uint64_t m = moff[k0];
        const bool adv = larger(st.end, st.len, m, st.commit);
        r->new_commit = adv ? m : st.commit;
        r->committed = (uint8_t)adv;
        r->n_entries = k0;
        r->outside = 0;
    }
    return true;
}

template <uint32_t W>
__global__ void __launch_bounds__(64) scalar_q_kernel(const QArgsT<W> args, QRes *out)
{
    // the arguments into LDS with every lane at once (one round trip), then
    // lane 0 computes from there into LDS
    constexpr uint32_t kN = sizeof(QArgsT<W>) / 16;
    __shared__ uint4 lds[kN + 1];
    __shared__ QRes res;
    {
        // every chunk of the argument block, unconditionally (a load behind a
        // per-lane test is waited for before the next one is issued): all
        // loads in flight at once, then the stores
        const uint4 *src = reinterpret_cast<const uint4 *>(&args);
        constexpr uint32_t kR = (kN + 63) / 64;
        uint4 v[kR];
#pragma unroll
        for (uint32_t k = 0; k < kR; ++k) {
            const uint32_t i = threadIdx.x + 64 * k;
            v[k] = src[i < kN ? i : kN - 1];
        }
        // (the copy loop is otherwise lowered as a memcpy: load, wait, store,
        // one chunk at a time; consuming every value here keeps the loads
        // together, one wait for all)
#pragma unroll
        for (uint32_t k = 0; k < kR; ++k) asm volatile("" : "+v"(v[k].x), "+v"(v[k].y), "+v"(v[k].z), "+v"(v[k].w));
#pragma unroll
        for (uint32_t k = 0; k < kR; ++k) {
            const uint32_t i = threadIdx.x + 64 * k;
            if (i < kN) lds[i] = v[k];
        }
        if (threadIdx.x < sizeof(QRes) / 8) reinterpret_cast<uint64_t *>(&res)[threadIdx.x] = 0;
    }
    __syncthreads();
    {
        const QArgs &qa = *reinterpret_cast<const QArgs *>(lds);
        const bool done = qa.op == kQWalk && q_walk_wave(qa, &res);
        if (!done && threadIdx.x == 0) scalar_q_compute(qa, &res);
    }
    __syncthreads();

    // the result words at system scope, every lane's done (the barrier), then
    // the sequence number with a system-scope RELEASE: the host's acquire
    // load of it (q_run) then sees every result word -- the HIP memory
    // model's release / acquire pair, on a page allocated
    // hipHostMallocMapped | hipHostMallocCoherent (default_ctx), so no
    // HIP_HOST_COHERENT setting changes it
    const uint32_t seq = reinterpret_cast<const QArgs *>(lds)->seq;
    if (threadIdx.x < offsetof(QRes, seq) / 8)
        __hip_atomic_store(reinterpret_cast<uint64_t *>(out) + threadIdx.x,
                           reinterpret_cast<const uint64_t *>(&res)[threadIdx.x], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(&out->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one launch; waits for the kernel's sequence number in the mapped page (the
// stream is synchronised only when it does not come: an error)
int q_run(apus_ctx *c, QArgs &a, const QRes *&res)
{
    a.seq = ++c->q_seq;
    if (a.seq == 0) a.seq = ++c->q_seq;
    a.bytes = (uint32_t)offsetof(QArgs, win) + (uint32_t)((a.seg[1] - a.seg[0]) + (a.seg[3] - a.seg[2]));
    QRes *hr = (QRes *)c->q_host;
    const uint32_t w = a.bytes - (uint32_t)offsetof(QArgs, win);
#define APUS_Q_LAUNCH(W)                                                                                  \
    {                                                                                                     \
        QArgsT<W> t;                                                                                      \
        memcpy(&t, &a, offsetof(QArgs, win) + w);                                                         \
        hipLaunchKernelGGL(scalar_q_kernel<W>, dim3(1), dim3(64), 0, c->s_stream, t, (QRes *)c->q_dev);   \
    }
    if (w == 0) APUS_Q_LAUNCH(0)
    else if (w <= 512) APUS_Q_LAUNCH(512)
    else if (w <= 1152) APUS_Q_LAUNCH(1152)
    else if (w <= 2048) APUS_Q_LAUNCH(2048)
    else APUS_Q_LAUNCH(kQWin)
#undef APUS_Q_LAUNCH
    CHECK_HIP(hipGetLastError());
    // the kernel's release store of seq, acquired (its result words are then visible)
    uint32_t *seq = &hr->seq;
    for (uint64_t spin = 0; __atomic_load_n(seq, __ATOMIC_ACQUIRE) != a.seq; ++spin) {
        if ((spin & 0xFFFFF) == 0xFFFFF) {
            // not there after a while: the stream tells whether the kernel failed
            const hipError_t e = hipStreamQuery(c->s_stream);
            if (e != hipSuccess && e != hipErrorNotReady) {
                apus::log_error("scalar call: %s\n", hipGetErrorString(e));
                return APUS_ERROR;
            }
            if (e == hipSuccess && __atomic_load_n(seq, __ATOMIC_ACQUIRE) != a.seq) {
                apus::log_error("scalar call: the kernel finished without its result\n");
                return APUS_ERROR;
            }
        }
        __builtin_ia32_pause();
    }
    res = hr;
    return APUS_OK;
}

// the window of a walk from commit: the ranges Stager::chain would stage;
// false when they exceed kQWin (the call takes the staged path)
bool q_window(QArgs &a, const apus_log_t *log)
{
    const uint64_t len = a.st.len, end = a.st.end, from = a.st.commit;
    a.seg[0] = a.seg[1] = a.seg[2] = a.seg[3] = 0;
    if (end >= len || from == end || from > len) return true;          // nothing is read
    uint64_t a0 = from, a1 = from < end ? end : len, b1 = from < end ? 0 : end;
    if (b1 < 64) b1 = len < 64 ? len : 64;                             // a header that does not fit is read at 0
    if ((a1 - a0) + b1 > kQWin) return false;
    memcpy(a.win, log->entries + a0, a1 - a0);
    memcpy(a.win + (a1 - a0), log->entries, b1);
    a.seg[0] = a0;
    a.seg[1] = a1;
    a.seg[2] = 0;
    a.seg[3] = b1;
    return true;
}

// the window of a log_get_tail lookup: the tail header (and the header at 0),
// or -- tail unknown -- the chains from commit / apply / head, when they fit
// two segments (the union of Stager::tail's ranges); false otherwise
bool q_tail_window(QArgs &a, const apus_log_t *log)
{
    const apus_group_state_t &st = a.st;
    const uint64_t len = st.len, end = st.end;
    a.seg[0] = a.seg[1] = a.seg[2] = a.seg[3] = 0;
    if (len < 64) return true;
    uint64_t a0, a1, b1;
    if (st.tail != len) {
        if (st.tail >= len) return true;
        a0 = st.tail;
        a1 = st.tail + 64 < len ? st.tail + 64 : len;
        b1 = 64;
    } else {
        if (end >= len) return true;
        // the chains start at commit, apply or head and run to end: the
        // earliest (circularly farthest from end) start covers the others
        auto far = [&](uint64_t o) { return end >= o ? end - o : len - (o - end); };
        if (st.commit > len || st.apply > len || st.head > len) return false;
        uint64_t from = st.commit;
        if (far(st.apply) > far(from)) from = st.apply;
        if (far(st.head) > far(from)) from = st.head;
        if (far(from) == 0) return true;                                   // every chain is empty
        a0 = from;
        a1 = from < end ? end : len;
        b1 = from < end ? 64 : (end > 64 ? end : 64);
    }
    if ((a1 - a0) + b1 > kQWin) return false;
    memcpy(a.win, log->entries + a0, a1 - a0);
    memcpy(a.win + (a1 - a0), log->entries, b1);
    a.seg[0] = a0;
    a.seg[1] = a1;
    a.seg[2] = 0;
    a.seg[3] = b1;
    return true;
}

// the fast path's common part: state and self from the reference's structs
void q_begin(QArgs &a, const apus_log_t *log, const apus_server_config_t *cfg, uint8_t op)
{
    memset(&a, 0, offsetof(QArgs, win));
    fill_state(a.st, log, cfg);
    a.self = cfg->idx;
    a.op = op;
}

}  // namespace

extern "C" {

int apus_log_new(uint64_t len, apus_log_t **out)
{
    if (!out) return APUS_ERROR;
    *out = nullptr;
    if (len < APUS_ENTRY_HDR || len > (1ull << 40)) return APUS_ERROR;
    apus_ctx *c;
    if (default_ctx(&c) != APUS_OK) return APUS_ERROR;
    const size_t bytes = sizeof(apus_log_t) + (size_t)len + 64;   // + the window loads' 16-B tail
    void *h = nullptr, *d = nullptr;
    CHECK_HIP(hipHostMalloc(&h, bytes, hipHostMallocMapped));
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(h);
        return APUS_ERROR;
    }
    // log_new (dare_log.h:120-137): zeroed, end = tail = old_end = len
    memset(h, 0, bytes);
    apus_log_t *log = (apus_log_t *)h;
    log->len = len;
    log->end = len;
    log->tail = len;
    log->old_end = len;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        g_owned.push_back(OwnedLog{log, (uint8_t *)d, bytes});
    }
    *out = log;
    return APUS_OK;
}

int apus_log_free(apus_log_t *log)
{
    if (!log) return APUS_ERROR;
    apus_ctx *c;
    if (default_ctx(&c) != APUS_OK) return APUS_ERROR;
    // a scalar call reading the log in place finishes first (lock order:
    // scalar_mu, then g_mu)
    std::lock_guard<std::mutex> sl(c->scalar_mu);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        size_t k = 0;
        while (k < g_owned.size() && g_owned[k].host != log) ++k;
        if (k == g_owned.size()) return APUS_INSUCCESS;      // not allocated by apus_log_new
        g_owned.erase(g_owned.begin() + (long)k);
    }
    CHECK_HIP(hipHostFree(log));
    return APUS_OK;
}

int apus_scalar_path_stats(uint64_t *in_place_calls, uint64_t *staged_calls, uint64_t *staged_bytes,
                           uint32_t *owned_logs)
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (in_place_calls) *in_place_calls = g_calls_in_place.load();
    if (staged_calls) *staged_calls = g_calls_staged.load();
    if (staged_bytes) *staged_bytes = g_bytes_staged.load();
    if (owned_logs) *owned_logs = (uint32_t)g_owned.size();
    return APUS_OK;
}

int apus_commit_reply_walk(const apus_log_t *log, const apus_server_config_t *config, uint64_t *new_commit,
                           int *committed)
{
    if (!new_commit || !log || !config) return APUS_ERROR;
    {
        // one launch: the walked bytes in the arguments (most calls)
        apus_ctx *c;
        if (default_ctx(&c) != APUS_OK) return APUS_ERROR;
        std::unique_lock<std::mutex> lk(c->scalar_mu);
        QArgs a;
        q_begin(a, log, config, kQWalk);
        if (q_window(a, log)) {
            const bool owned = owned_ring(log) != nullptr;
            const QRes *r;
            if (q_run(c, a, r) != APUS_OK) return APUS_ERROR;
            if (!(owned && r->outside)) {
                (owned ? g_calls_in_place : g_calls_staged)++;
                if (r->committed == 0xFF) return APUS_ERROR;
                *new_commit = r->new_commit;
                if (committed) *committed = r->committed;
                return APUS_OK;
            }
            // an owned log's walk left the window: read it in place (below)
        }
    }
    Scalar s;
    if (scalar_begin(s, log, config) != APUS_OK) return APUS_ERROR;
    s.chain(s.hin->st.commit);
    if (scalar_upload(s) != APUS_OK) return APUS_ERROR;
    apus_commit_out_t o;
    memset(&o, 0, sizeof o);
    o.new_commit = &s.dout->new_commit;
    o.committed = &s.dout->committed;
    o.n_entries = &s.dout->n_entries;
    CHECK_HIP(apus::launch_commit(s.c, s.b, o, APUS_COMMIT_WALK, s.c->s_stream));
    if (scalar_finish(s) != APUS_OK) return APUS_ERROR;
    if (s.hout->committed == 0xFF) return APUS_ERROR;
    *new_commit = s.hout->new_commit;
    if (committed) *committed = s.hout->committed;
    return APUS_OK;
}

int apus_commit_median(const apus_log_t *log, const apus_server_config_t *config, const apus_ctrl_data_t *ctrl,
                       uint64_t *median)
{
    if (!ctrl || !median || !config || !config->servers || !log) return APUS_ERROR;
    apus_ctx *c;
    if (default_ctx(&c) != APUS_OK) return APUS_ERROR;
    std::unique_lock<std::mutex> lk(c->scalar_mu);
    QArgs a;
    q_begin(a, log, config, kQMedian);
    for (int i = 0; i < APUS_MAX_SERVER_COUNT; ++i) {
        a.col[i] = ctrl->log_offsets[i].end;
        const bool have = i < config->len || config->len == 0;
        a.step[i] = have ? config->servers[i].next_lr_step : 0;
        a.fail[i] = have ? config->servers[i].fail_count : APUS_PERMANENT_FAILURE;
    }
    const QRes *r;
    if (q_run(c, a, r) != APUS_OK) return APUS_ERROR;
    *median = r->median;
    return APUS_OK;
}

int apus_vote_tally(const apus_log_t *log, const apus_server_config_t *config, const apus_ctrl_data_t *ctrl,
                    uint8_t vc[2], uint64_t *new_commit, uint16_t *voters)
{
    if (!ctrl || !log || !config) return APUS_INSUCCESS;
    apus_ctx *c;
    if (default_ctx(&c) != APUS_OK) return APUS_INSUCCESS;
    std::unique_lock<std::mutex> lk(c->scalar_mu);
    QArgs a;
    q_begin(a, log, config, kQVote);
    memcpy(a.col, ctrl->vote_ack, sizeof a.col);
    const QRes *r;
    if (q_run(c, a, r) != APUS_OK) return APUS_INSUCCESS;
    if (vc) { vc[0] = r->vc[0]; vc[1] = r->vc[1]; }
    if (new_commit) *new_commit = r->vote_commit;
    if (voters) *voters = r->voters;
    return r->won;
}

int apus_vote_rank(const apus_log_t *log, const apus_server_config_t *config, apus_ctrl_data_t *ctrl,
                   uint8_t *outcome, uint64_t *new_sid, apus_cid_t *new_cid, uint16_t *cleared)
{
    if (!ctrl) return APUS_ERROR;
    Scalar s;
    if (scalar_begin(s, log, config) != APUS_OK) return APUS_ERROR;
    s.hin->sid = ctrl->sid;
    memcpy(s.hin->hb, ctrl->hb, sizeof s.hin->hb);
    memcpy(s.hin->vote_req, ctrl->vote_req, sizeof s.hin->vote_req);
    // the local (idx, term): the NC walk from commit, else the tail (dare_server.c:1598-1620)
    s.chain(s.hin->st.commit);
    s.tail();
    if (scalar_upload(s) != APUS_OK) return APUS_ERROR;
    // local (idx, term) from the log on the device, then the ranking
    CHECK_HIP(apus::launch_last_idx_term(s.b, s.din->lit, s.c->s_stream));
    apus_rank_out_t o;
    o.outcome = &s.dout->u8a;
    o.new_sid = &s.dout->u64a;
    o.new_cid = &s.dout->cid;
    o.cleared = &s.dout->u16a;
    CHECK_HIP(apus::launch_rank(s.c, s.b, o, s.c->s_stream));
    if (scalar_finish(s) != APUS_OK) return APUS_ERROR;
    // requests the ranking consumed or dropped: the reference zeroes their
    // sid in place (dare_server.c:1566-1580, 1627-1652)
    for (int i = 0; i < APUS_MAX_SERVER_COUNT; ++i)
        if (s.hout->u16a & (1u << i)) ctrl->vote_req[i].sid = 0;
    if (outcome) *outcome = s.hout->u8a;
    if (new_sid) *new_sid = s.hout->u64a;
    if (new_cid) *new_cid = s.hout->cid;
    if (cleared) *cleared = s.hout->u16a;
    return APUS_OK;
}

int apus_min_apply(const apus_log_t *log, const apus_server_config_t *config, apus_ctrl_data_t *ctrl,
                   int prev_log_entry_head, uint64_t *new_head, int *append_head)
{
    if (!ctrl || !log || !config) return APUS_ERROR;
    {
        // one launch; a log_get_tail that leaves the window is redone below
        apus_ctx *c;
        if (default_ctx(&c) != APUS_OK) return APUS_ERROR;
        std::unique_lock<std::mutex> lk(c->scalar_mu);
        QArgs a;
        q_begin(a, log, config, kQPrune);
        memcpy(a.col, ctrl->apply_offsets, sizeof a.col);
        a.prev = prev_log_entry_head ? 1 : 0;
        if (q_tail_window(a, log)) {
            const QRes *r;
            if (q_run(c, a, r) != APUS_OK) return APUS_ERROR;
            if (!r->outside) {
                // OFF servers' apply offsets reset to log->apply (dare_server.c:2031-2034)
                for (int i = 0; i < APUS_MAX_SERVER_COUNT; ++i)
                    if ((r->reset >> i) & 1u) ctrl->apply_offsets[i] = log->apply;
                if (new_head) *new_head = r->new_head;
                if (append_head) *append_head = r->append;
                return APUS_OK;
            }
        }
    }
    Scalar s;
    if (scalar_begin(s, log, config) != APUS_OK) return APUS_ERROR;
    memcpy(s.hin->apply_offsets, ctrl->apply_offsets, sizeof s.hin->apply_offsets);
    s.hin->prev_head = prev_log_entry_head ? 1 : 0;
    s.tail();                                   // dist(min) == 0 -> log_get_tail (dare_server.c:2043-2046)
    if (scalar_upload(s) != APUS_OK) return APUS_ERROR;
    apus_prune_out_t o;
    o.new_head = &s.dout->u64a;
    o.append_head = &s.dout->u8a;
    o.min_apply = &s.dout->u64b;
    CHECK_HIP(apus::launch_prune(s.c, s.b, o, s.c->s_stream));
    if (scalar_finish(s, 0, true) != APUS_OK) return APUS_ERROR;
    // OFF servers' apply offsets reset to log->apply (dare_server.c:2031-2034)
    memcpy(ctrl->apply_offsets, s.hin->apply_offsets, sizeof s.hin->apply_offsets);
    if (new_head) *new_head = s.hout->u64a;
    if (append_head) *append_head = s.hout->u8a;
    return APUS_OK;
}

int apus_publish_commit(const apus_log_t *log, const apus_server_config_t *config, apus_ctrl_data_t *ctrl,
                        uint16_t rc_connected, uint64_t *ssn, uint16_t *post)
{
    if (!log || !config || !config->servers || !ctrl || !ssn || !post) return APUS_ERROR;
    apus_ctx *c;
    if (default_ctx(&c) != APUS_OK) return APUS_ERROR;
    std::unique_lock<std::mutex> lk(c->scalar_mu);
    QArgs a;
    q_begin(a, log, config, kQPublish);
    for (int i = 0; i < APUS_MAX_SERVER_COUNT; ++i) {
        a.col[i] = ctrl->log_offsets[i].commit;
        a.col2[i] = ctrl->log_offsets[i].end;
        const bool have = i < config->len || config->len == 0;
        a.step[i] = have ? config->servers[i].next_lr_step : 0;
        a.fail[i] = have ? config->servers[i].fail_count : APUS_PERMANENT_FAILURE;
    }
    a.conn = rc_connected;
    const QRes *r;
    if (q_run(c, a, r) != APUS_OK) return APUS_ERROR;
    for (int i = 0; i < APUS_MAX_SERVER_COUNT; ++i) ctrl->log_offsets[i].commit = r->col[i];
    *post = r->voters;
    if (r->voters) ++*ssn;                                  // `if (!init) ssn++`, :1788-1789
    return APUS_OK;
}

int apus_force_log_pruning(apus_log_t *log, apus_server_config_t *config, apus_ctrl_data_t *ctrl,
                           int *prev_log_entry_head, uint8_t *target, uint64_t *cfg_idx, uint64_t *new_head,
                           int *append_head)
{
    if (!log || !config || !ctrl || !prev_log_entry_head) return APUS_INSUCCESS;
    Scalar s;
    if (scalar_begin(s, log, config) != APUS_OK) return APUS_INSUCCESS;
    memcpy(s.hin->apply_offsets, ctrl->apply_offsets, sizeof s.hin->apply_offsets);
    s.hin->sid = ctrl->sid;
    s.hin->prev_head = *prev_log_entry_head ? 1 : 0;
    // the CONFIG append's index (the tail entry) and log_pruning's tail lookup
    s.tail();
    // the header the CONFIG append writes, at end (at 0 when a header does not
    // fit): the bytes log_append_entry leaves (sender, padding) are the
    // caller's, copied back with the entry
    {
        const uint64_t e = log->end, l = log->len;
        s.header(e >= l || l - e < APUS_ENTRY_HDR ? 0 : e);
    }
    if (scalar_upload(s) != APUS_OK) return APUS_INSUCCESS;
    apus_commit_out_t o;
    memset(&o, 0, sizeof o);
    o.new_head = &s.dout->u64a;
    o.append_head = &s.dout->u8a;
    o.min_apply = &s.dout->u64b;
    o.force.action = &s.dout->committed;
    o.force.target = &s.dout->u8b[0];
    o.force.cfg_idx = &s.dout->new_commit;
    if (apus::launch_commit(s.c, s.b, o, APUS_COMMIT_FORCE_PRUNE, s.c->s_stream) != hipSuccess)
        return APUS_INSUCCESS;
    if (scalar_finish(s, 0, true) != APUS_OK) return APUS_INSUCCESS;
    const int action = s.hout->committed;
    if (action == APUS_FORCE_REMOVE) {
        config->cid = s.hin->st.cid;                          // CID_SERVER_RM (:2101)
        config->req_id = 0;                                   // :2104-2105
        config->clt_id = 0;
        if (s.hout->new_commit) {
            // the CONFIG entry (at the new tail): written in place on an owned
            // log; on a staged one, back into the caller's log and the image poisoned again
            const uint64_t at = s.hin->st.tail;
            if (s.staged && at + APUS_ENTRY_HDR <= log->len) {
                memcpy((uint8_t *)log->entries + at, s.c->stage + at, APUS_ENTRY_HDR);
                memset(s.c->stage + at, kPoison, APUS_ENTRY_HDR);
            }
        }
        *prev_log_entry_head = s.hin->prev_head;
    }
    // log_append_entry's end / tail (the tail also when the log was full: it is
    // looked up before the full test, dare_log.h:483-495)
    log->end = s.hin->st.end;
    log->tail = s.hin->st.tail;
    memcpy(ctrl->apply_offsets, s.hin->apply_offsets, sizeof s.hin->apply_offsets);
    if (target) *target = s.hout->u8b[0];
    if (cfg_idx) *cfg_idx = s.hout->new_commit;
    if (new_head) *new_head = s.hout->u64a;
    if (append_head) *append_head = s.hout->u8a;
    return action;
}

int apus_log_adjustment(apus_log_t *log, apus_server_config_t *config, apus_ctrl_data_t *ctrl,
                        uint16_t rc_connected, uint64_t *ssn, uint8_t post[APUS_MAX_SERVER_COUNT])
{
    if (!ctrl || !ssn || !post || !config || !config->servers || config->len > APUS_MAX_SERVER_COUNT)
        return APUS_ERROR;
    Scalar s;
    if (scalar_begin(s, log, config) != APUS_OK) return APUS_ERROR;
    ScalarLr *hl = (ScalarLr *)(s.c->h_pinned + kScalarLrOff);
    ScalarLr *dl = (ScalarLr *)(s.c->s_buf + kScalarLrOff);
    memset(hl, 0, sizeof(ScalarLr));
    const uint32_t n = config->len;
    for (uint32_t i = 0; i < n; ++i) {
        const apus_server_t &sv = config->servers[i];
        s.hin->fail_count[i] = sv.fail_count;
        s.hin->lr_step[i] = sv.next_lr_step;
        hl->send_flag[i] = sv.send_flag;
    }
    for (uint32_t i = 0; i < APUS_MAX_SERVER_COUNT; ++i) {
        s.hin->vote_ack[i] = ctrl->vote_ack[i];
        s.hin->remote_commit[i] = ctrl->log_offsets[i].commit;
        s.hin->remote_end[i] = ctrl->log_offsets[i].end;
        hl->nc_len[i] = log->nc_buf[i].len;
    }
    hl->ssn = *ssn;
    hl->rc_connected = rc_connected;
    // the determinants of the servers at LR_SET_END (the only step that reads
    // them) and the local headers log_find_remote_end_offset looks up
    for (uint32_t i = 0; i < n; ++i) {
        if (config->servers[i].next_lr_step != APUS_LR_SET_END || !log->nc_buf[i].len) continue;
        const size_t k = log->nc_buf[i].len < APUS_MAX_NC_ENTRIES ? log->nc_buf[i].len : APUS_MAX_NC_ENTRIES;
        apus_entry_det_t *h = s.hdets + (size_t)i * APUS_MAX_NC_ENTRIES;
        memcpy(h, log->nc_buf[i].entries, k * sizeof(apus_entry_det_t));
        for (size_t j = 0; j < k; ++j) s.header(h[j].offset);
    }
    if (scalar_upload(s) != APUS_OK) return APUS_ERROR;
    CHECK_HIP(hipMemcpyAsync(dl, hl, sizeof(ScalarLr), hipMemcpyHostToDevice, s.c->s_stream));
    for (uint32_t i = 0; i < n; ++i) {
        if (config->servers[i].next_lr_step != APUS_LR_SET_END || !log->nc_buf[i].len) continue;
        const size_t k = log->nc_buf[i].len < APUS_MAX_NC_ENTRIES ? log->nc_buf[i].len : APUS_MAX_NC_ENTRIES;
        const apus_entry_det_t *h = s.hdets + (size_t)i * APUS_MAX_NC_ENTRIES;
        CHECK_HIP(hipMemcpyAsync(s.ddets + (size_t)i * APUS_MAX_NC_ENTRIES, h, k * sizeof(apus_entry_det_t),
                                 hipMemcpyHostToDevice, s.c->s_stream));
    }
    apus_lr_io_t io;
    memset(&io, 0, sizeof io);
    io.send_flag = dl->send_flag;
    io.rc_connected = &dl->rc_connected;
    io.nc_len = dl->nc_len;
    io.nc_dets = s.ddets;
    io.ssn = &dl->ssn;
    io.post = dl->post;
    io.max_dets = APUS_MAX_NC_ENTRIES;
    CHECK_HIP(apus::launch_log_adjust(s.c, s.b, io, s.c->s_stream));
    CHECK_HIP(hipMemcpyAsync(hl, dl, sizeof(ScalarLr), hipMemcpyDeviceToHost, s.c->s_stream));
    if (scalar_finish(s, 0, true) != APUS_OK) return APUS_ERROR;
    // write back what log_adjustment updates in place
    log->commit = s.hin->st.commit;
    for (uint32_t i = 0; i < n; ++i) {
        config->servers[i].next_lr_step = s.hin->lr_step[i];
        config->servers[i].send_flag = hl->send_flag[i];
    }
    for (uint32_t i = 0; i < APUS_MAX_SERVER_COUNT; ++i) {
        ctrl->log_offsets[i].commit = s.hin->remote_commit[i];
        ctrl->log_offsets[i].end = s.hin->remote_end[i];
        post[i] = hl->post[i];
    }
    *ssn = hl->ssn;
    return APUS_OK;
}

int apus_lr_work_completion(apus_server_t *server, int wc)
{
    if (!server || wc < APUS_WC_NONE || wc > APUS_WC_STALE) return APUS_ERROR;
    apus_ctx *c;
    if (default_ctx(&c) != APUS_OK) return APUS_ERROR;
    std::lock_guard<std::mutex> lk(c->scalar_mu);
    ScalarLr *hl = (ScalarLr *)(c->h_pinned + kScalarLrOff);
    ScalarLr *dl = (ScalarLr *)(c->s_buf + kScalarLrOff);
    memset(hl, 0, sizeof(ScalarLr));
    hl->wc[0] = (uint8_t)wc;
    hl->post[0] = server->next_lr_step;        // the step column of this one-pair batch
    hl->send_flag[0] = server->send_flag;
    hl->send_count[0] = server->send_count;
    CHECK_HIP(hipMemcpyAsync(dl, hl, sizeof(ScalarLr), hipMemcpyHostToDevice, c->s_stream));
    apus_batch_t b;
    memset(&b, 0, sizeof b);
    b.n_groups = 1;
    b.n_replicas = 1;
    b.lr_step = dl->post;
    apus_lr_io_t io;
    memset(&io, 0, sizeof io);
    io.send_flag = dl->send_flag;
    io.send_count = dl->send_count;
    io.wc = dl->wc;
    CHECK_HIP(apus::launch_lr_completion(c, b, io, c->s_stream));
    CHECK_HIP(hipMemcpyAsync(hl, dl, sizeof(ScalarLr), hipMemcpyDeviceToHost, c->s_stream));
    CHECK_HIP(hipStreamSynchronize(c->s_stream));
    server->next_lr_step = hl->post[0];
    server->send_flag = hl->send_flag[0];
    server->send_count = hl->send_count[0];
    return APUS_OK;
}

int apus_find_remote_end(const apus_log_t *log, const apus_nc_buf_t *nc, uint64_t *remote_end)
{
    if (!log || !nc || !remote_end) return APUS_ERROR;
    if (nc->len == 0 || nc->len > APUS_MAX_NC_ENTRIES) return APUS_ERROR;
    apus_server_config_t cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.cid.size[0] = 1;
    Scalar s;
    if (scalar_begin(s, log, &cfg) != APUS_OK) return APUS_ERROR;
    memcpy(s.hdets, nc->entries, nc->len * sizeof(apus_entry_det_t));
    for (uint64_t i = 0; i < nc->len; ++i) s.header(s.hdets[i].offset);
    if (scalar_upload(s) != APUS_OK) return APUS_ERROR;
    CHECK_HIP(hipMemcpyAsync(s.ddets, s.hdets, nc->len * sizeof(apus_entry_det_t), hipMemcpyHostToDevice,
                             s.c->s_stream));
    // det_len and follower live in the output scratch
    s.hout->len = (uint32_t)nc->len;
    CHECK_HIP(hipMemcpyAsync(&s.dout->len, &s.hout->len, sizeof(uint32_t), hipMemcpyHostToDevice, s.c->s_stream));
    apus_nc_batch_t b;
    memset(&b, 0, sizeof b);               // no leader determinants: the leader's headers are gathered
    b.n_followers = 1;
    b.max_dets = (uint32_t)nc->len;
    b.dets = s.ddets;
    b.det_len = &s.dout->len;
    b.follower = &s.dout->u8a;
    CHECK_HIP(apus::launch_validate(s.c, s.b, b, &s.dout->u64a, s.c->s_stream));
    if (scalar_finish(s) != APUS_OK) return APUS_ERROR;
    *remote_end = s.hout->u64a;
    return APUS_OK;
}

int apus_entries_to_nc_buf(const apus_log_t *log, apus_nc_buf_t *nc)
{
    if (!log || !nc) return APUS_ERROR;
    apus_server_config_t cfg;
    memset(&cfg, 0, sizeof cfg);
    cfg.cid.size[0] = 1;
    Scalar s;
    if (scalar_begin(s, log, &cfg) != APUS_OK) return APUS_ERROR;
    s.chain(s.hin->st.commit);
    if (scalar_upload(s) != APUS_OK) return APUS_ERROR;
    CHECK_HIP(apus::launch_nc_build(s.c, s.b, s.ddets, (uint32_t)kScalarDets, &s.dout->len, s.c->s_stream));
    CHECK_HIP(hipMemcpyAsync(&s.hout->len, &s.dout->len, sizeof(uint32_t), hipMemcpyDeviceToHost, s.c->s_stream));
    CHECK_HIP(hipStreamSynchronize(s.c->s_stream));
    const uint32_t n = s.hout->len;
    if (scalar_finish(s, n) != APUS_OK) return APUS_ERROR;
    nc->len = n;
    memcpy(nc->entries, s.hdets, n * sizeof(apus_entry_det_t));
    return APUS_OK;
}

}  // extern "C"
