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

namespace apus {

// dare_cid_t as two words: lo = epoch; hi = size0 | size1 << 8 | state << 16
// | pad << 24 | bitmask << 32 (apus_gpu.h apus_cid_t)
constexpr uint64_t kCidCmpMask = ~0xFF000000ull;     // equal_cid ignores pad
__device__ __forceinline__ uint32_t cid_size0(uint64_t hi) { return (uint32_t)hi & 0xFFu; }
__device__ __forceinline__ uint32_t cid_size1(uint64_t hi) { return (uint32_t)(hi >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t cid_state(uint64_t hi) { return (uint32_t)(hi >> 16) & 0xFFu; }
__device__ __forceinline__ bool cid_on(uint64_t hi, uint32_t i) { return i < 32 && ((hi >> (32 + i)) & 1ull); }

__device__ __forceinline__ bool ring_ok(const apus_group_state_t &st, uint64_t stride)
{
    return st.len >= kHdr && st.len <= stride && st.end <= st.len && st.commit <= st.len && st.apply <= st.len &&
           st.head <= st.len;
}

__global__ void __launch_bounds__(256) config_scan_kernel(const apus_batch_t b, const apus_config_io_t io,
                                                          uint64_t *stats)
{
    uint64_t corrupt = 0;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t *const offs = offsets_of(b, g);
        uint64_t *const cw = cid_words(b, g);
        const apus_group_state_t st = load_state(b, g);
        const uint64_t len = st.len, end = st.end, commit = st.commit;
        uint64_t off = io.cid_offset[g];
        if (!ring_ok(st, ring_cap(b)) || off > len) { ++corrupt; continue; }
        const uint8_t *ring = b.ring + g * b.ring_stride;
        const uint64_t cid_idx = io.cid_idx[g];
        uint64_t c_lo = st.cid.epoch;
        uint64_t c_hi = cw[1];
        uint64_t rq = io.req_id[g], head_off = st.head;
        uint32_t cl = io.clt_id[g], dep = 0;
        const uint64_t guard = len / kHdr + 4;
        uint64_t steps = 0;
        bool bad = false, changed = false;
        while (dist(end, len, off) != 0) {
            if (++steps > guard) { bad = true; break; }
            if (len - off < kHdr) off = 0;                            // log_get_entry
            const uint8_t *e = ring + off;
            const uint32_t type = e[kType];
            const uint32_t el = entry_len(type, ld_u16(e + kData));
            if (len - off < el) { off = 0; continue; }                // !log_fit_entry
            if (type == APUS_CONFIG) {
                if (ld_u64(e + kIdx) > cid_idx) {
                    const uint64_t n_lo = ld_u64(e + kData), n_hi = ld_u64(e + kData + 8);
                    if (n_lo != c_lo || ((n_hi ^ c_hi) & kCidCmpMask) != 0) {     // update_cid
                        const uint32_t size = max(cid_size0(n_hi), cid_size1(n_hi));
                        for (uint32_t i = 0; i < size && i < 16; ++i)
                            if (!cid_on(n_hi, i) && cid_on(c_hi, i)) dep |= 1u << i;
                        c_lo = n_lo;
                        c_hi = n_hi;
                        changed = true;
                        rq = ld_u64(e + 16);
                        cl = ld_u16(e + 24);
                    }
                }
            } else if (type == APUS_HEAD) {
                if (!larger(end, len, off, commit)) head_off = ld_u64(e + kData);
            }
            off += el;
        }
        if (changed) {
            cw[0] = c_lo;
            cw[1] = c_hi;
            io.req_id[g] = rq;
            io.clt_id[g] = (uint16_t)cl;
        }
        if (io.departed) io.departed[g] = (uint16_t)dep;
        if (bad) { ++corrupt; continue; }
        io.cid_offset[g] = larger(end, len, off, commit) ? commit : off;
        if (larger(end, len, head_off, st.head)) offs[kOffHead] = head_off;
    }
    if (corrupt) atomicAdd((unsigned long long *)&stats[APUS_STAT_CORRUPT], (unsigned long long)corrupt);
}

__global__ void __launch_bounds__(256) apply_kernel(const apus_batch_t b, const apus_apply_io_t io,
                                                    uint64_t *stats)
{
    uint64_t corrupt = 0;
    const uint32_t M = io.max_cfg;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t *const offs = offsets_of(b, g);
        uint64_t *const cw = cid_words(b, g);
        const apus_group_state_t st = load_state(b, g);
        if (!ring_ok(st, ring_cap(b))) { ++corrupt; continue; }
        const uint64_t len = st.len, end = st.end, commit = st.commit;
        const uint8_t *ring = b.ring + g * b.ring_stride;
        const uint32_t self = b.self_idx[g];
        const uint64_t sid = b.sid[g];
        const bool leader = ((sid >> 8) & 1ull) && (uint32_t)(sid & 0xFFu) == self;   // IS_LEADER
        uint64_t c_lo = st.cid.epoch;
        uint64_t c_hi = cw[1];
        uint64_t rq_cfg = io.req_id[g], la2 = 0, la_off = 0;
        uint32_t cl_cfg = io.clt_id[g], na = 0, nc = 0, dep = 0, ev = 0;
        uint64_t apply = st.apply;
        const uint64_t guard = len / kHdr + 4;
        uint64_t steps = 0;
        bool bad = false, cfg_changed = false;
        // while (log_is_offset_larger(log, commit, apply))
        while (dist(end, len, commit) < dist(end, len, apply)) {
            if (++steps > guard) { bad = true; break; }
            if (len - apply < kHdr) apply = 0;                        // log_get_entry
            const uint8_t *e = ring + apply;
            const uint32_t type = e[kType];
            const uint32_t el = entry_len(type, ld_u16(e + kData));
            if (len - apply < el) { apply = 0; continue; }            // !log_fit_entry
            if (leader && type == APUS_CONFIG) {
                const uint64_t e_lo = ld_u64(e + kData), e_hi = ld_u64(e + kData + 8);
                uint64_t rq = ld_u64(e + 16);
                uint32_t cl = ld_u16(e + 24);
                const uint32_t es = cid_state(e_hi);
                if (es == APUS_CID_STABLE) {
                    if (rq != 0) ev |= APUS_EV_CFG_REPLY;                  // :1862-1875
                } else if (!(c_lo > e_lo)) {                                // :1877-1881
                    if (nc == M) { ev |= APUS_EV_CFG_FULL; break; }
                    if (es == APUS_CID_EXTENDED) {                          // :1888-1902
                        c_hi = (c_hi & ~0xFF0000ull) | ((uint64_t)APUS_CID_TRANSIT << 16);
                        if (rq != 0) { ev |= APUS_EV_JOIN_REPLY; rq = 0; cl = 0; }
                    } else if (es == APUS_CID_TRANSIT) {                   // :1903-1931
                        c_hi = (c_hi & ~0xFF0000ull) | ((uint64_t)APUS_CID_STABLE << 16);
                        const uint32_t s0 = cid_size0(c_hi), s1 = cid_size1(c_hi);
                        for (uint32_t i = s1; i < s0; ++i) {
                            if (i == self) {
                                ev |= APUS_EV_SELF_REMOVED;
                                if (i < 32) c_hi &= ~(1ull << (32 + i));
                                continue;
                            }
                            if (!cid_on(c_hi, i)) continue;
                            c_hi &= ~(1ull << (32 + i));
                            if (i < 16) dep |= 1u << i;
                        }
                        c_hi = (c_hi & ~0xFFFFull) | s1;                    // size[0] = size[1]; size[1] = 0
                    }
                    rq_cfg = rq;
                    cl_cfg = cl;
                    cfg_changed = true;
                    // log_append_entry(..., CONFIG, &data.config.cid), :1935-1937
                    const uint64_t j = g * M + nc;
                    uint64_t *r = reinterpret_cast<uint64_t *>(io.cfg_entries + j);
                    r[0] = rq;
                    r[1] = 16ull * j;
                    r[2] = (uint64_t)cl | ((uint64_t)APUS_CONFIG << 16);
                    uint64_t *pl = reinterpret_cast<uint64_t *>(io.cfg_payload + 16ull * j);
                    pl[0] = c_lo;
                    pl[1] = c_hi;
                    ++nc;
                }
            } else if (!bare_type(type)) {                                  // apply_entry, :1939-1965
                // only the last applied entry's (idx, term) survives the scan:
                // its offset is kept and the pair read once after the walk
                la_off = apply;
                la2 = apply + el;
                ++na;
            }
            apply += el;                                                    // apply_next_entry
        }
        offs[kOffApply] = apply;
        if (cfg_changed) {
            cw[1] = c_hi;
            io.req_id[g] = rq_cfg;
            io.clt_id[g] = (uint16_t)cl_cfg;
        }
        if (na) {
            uint64_t la0, la1;
            ld_idx_term(ring + la_off, la0, la1);
            io.last_applied[3 * g] = la0;
            io.last_applied[3 * g + 1] = la1;
            io.last_applied[3 * g + 2] = la2;
            io.last_csm_idx[g] = la0;
        }
        if (io.n_applied) io.n_applied[g] = na;
        if (io.departed) io.departed[g] = (uint16_t)dep;
        if (io.events) io.events[g] = (uint8_t)ev;
        io.n_cfg[g] = nc;
        if (bad) ++corrupt;
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
