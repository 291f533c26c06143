// Apply / config scan for gfx950: one LANE per group walks its
// log chain (log_get_entry / log_fit_entry, src/include/dare/dare_log.h:
// 241-247,316-332) with the aligned-load helpers of apus_device.h.
//
//   config_scan_kernel  poll_config_entries, src/dare/dare_server.c:2133-2187,
//                       update_cid :2193-2226, equal_cid dare_config.h:48-56
//   apply_kernel        apply_committed_entries, dare_server.c:1815-1974; the
//                       leader's CONFIG re-appends leave as apus_append_batch
//                       input (apus_gpu.h)
//
// Both are chains of dependent header reads with a few bytes used per entry:
// lane per group keeps 64 independent chains in flight per wave.
#include "apus_device.h"
#include "apus_internal.h"
#include "apus_log_ops.h"

namespace apus {

__global__ void __launch_bounds__(256) config_scan_kernel(const apus_batch_t b, const apus_config_io_t io,
                                                          uint64_t *stats)
{
    uint64_t corrupt = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t *const offs = offsets_of(b, g);
        uint64_t *const cw = cid_words(b, g);
        const apus_group_state_t st = load_state(b, g);
        uint64_t off = io.cid_offset[g];
        if (!ring_ok(st, ring_cap(b)) || off > st.len) { ++corrupt; continue; }
        uint64_t c_lo = st.cid.epoch, c_hi = cw[1];
        uint64_t rq = io.req_id[g], head_off = st.head;
        uint32_t cl = io.clt_id[g], dep = 0;
        bool changed = false;
        const bool ok = scan_config(b.ring + g * b.ring_stride, st, io.cid_idx[g], off, c_lo, c_hi, rq, cl, dep,
                                    changed, head_off);
        if (changed) {
            cw[0] = c_lo;
            cw[1] = c_hi;
            io.req_id[g] = rq;
            io.clt_id[g] = (uint16_t)cl;
        }
        if (io.departed) io.departed[g] = (uint16_t)dep;
        if (!ok) { ++corrupt; continue; }
        io.cid_offset[g] = larger(st.end, st.len, off, st.commit) ? st.commit : off;
        if (larger(st.end, st.len, head_off, st.head)) offs[kOffHead] = head_off;
    }
    if (corrupt) atomicAdd((unsigned long long *)&stats[APUS_STAT_CORRUPT], (unsigned long long)corrupt);
}

__global__ void __launch_bounds__(256) apply_kernel(const apus_batch_t b, const apus_apply_io_t io,
                                                    uint64_t *stats)
{
    uint64_t corrupt = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t *const offs = offsets_of(b, g);
        uint64_t *const cw = cid_words(b, g);
        apus_group_state_t st = load_state(b, g);
        if (!ring_ok(st, ring_cap(b))) { ++corrupt; continue; }
        const uint32_t self = b.self_idx[g];
        const uint64_t sid = b.sid[g];
        const bool leader = ((sid >> 8) & 1ull) && (uint32_t)(sid & 0xFFu) == self;   // IS_LEADER
        ApplyAcc a{};
        a.c_lo = st.cid.epoch;
        a.c_hi = cw[1];
        a.rq = io.req_id[g];
        a.cl = io.clt_id[g];
        uint32_t prev = 0;
        const bool ok = apply_walk<false>(b, g, st, self, leader, sid >> 9, a, &io, prev);
        offs[kOffApply] = st.apply;
        if (a.cfg_changed) {
            cw[1] = a.c_hi;
            io.req_id[g] = a.rq;
            io.clt_id[g] = (uint16_t)a.cl;
        }
        if (a.na) {
            uint64_t la0, la1;
            ld_idx_term(b.ring + g * b.ring_stride + a.la_off, la0, la1);
            io.last_applied[3 * g] = la0;
            io.last_applied[3 * g + 1] = la1;
            io.last_applied[3 * g + 2] = a.la2;
            io.last_csm_idx[g] = la0;
        }
        if (io.n_applied) io.n_applied[g] = a.na;
        if (io.departed) io.departed[g] = (uint16_t)a.dep;
        if (io.events) io.events[g] = (uint8_t)a.ev;
        io.n_cfg[g] = a.nc;
        if (!ok) ++corrupt;
    }
    if (corrupt) atomicAdd((unsigned long long *)&stats[APUS_STAT_CORRUPT], (unsigned long long)corrupt);
}

hipError_t launch_config_scan(apus_ctx *ctx, const apus_batch_t &b, const apus_config_io_t &io, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    // (no more blocks than are resident: grid-strided lanes, no partial last round)
    const uint32_t grid = grid_for(b.n_groups, 256, ctx->n_cu,
                                   (uint32_t)min(8, resident_blocks(ctx, 43, (const void *)config_scan_kernel)));
    hipLaunchKernelGGL(config_scan_kernel, dim3(grid), dim3(256), 0, s, b, io, ctx->stats);
    return hipGetLastError();
}

hipError_t launch_apply(apus_ctx *ctx, const apus_batch_t &b, const apus_apply_io_t &io, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    // (capped at the resident blocks, as config_scan_kernel is, it measured
    // 2-4% slower: profiles/r03/grid/ab_grid.log)
    const uint32_t grid = grid_for(b.n_groups, 256, ctx->n_cu, 8);
    hipLaunchKernelGGL(apply_kernel, dim3(grid), dim3(256), 0, s, b, io, ctx->stats);
    return hipGetLastError();
}

}  // namespace apus
