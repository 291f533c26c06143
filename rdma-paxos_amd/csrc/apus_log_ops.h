// The log walks of one group that several kernels share (lane per group):
//   scan_config  poll_config_entries, src/dare/dare_server.c:2133-2187, with
//                update_cid :2193-2226 and equal_cid dare_config.h:48-56
//                (config_scan_kernel, vote_win_kernel)
//   apply_walk   apply_committed_entries, dare_server.c:1815-1974 (apply_kernel:
//                the leader's CONFIG re-appends leave as apus_append_batch
//                input; vote_win_kernel: they are appended in place when they
//                are met, as the reference appends them)
// Both follow the entry chain with log_get_entry / log_fit_entry
// (src/include/dare/dare_log.h:241-247,316-332) and the aligned-load helpers
// of apus_device.h.
#pragma once

#include "apus_device.h"
#include "apus_group_ops.h"

namespace apus {

// dare_cid_t as two words: lo = epoch; hi = size0 | size1 << 8 | state << 16
// | pad << 24 | bitmask << 32 (apus_gpu.h apus_cid_t)
constexpr uint64_t kCidCmpMask = ~0xFF000000ull;     // equal_cid ignores pad
__device__ __forceinline__ uint32_t cid_size0(uint64_t hi) { return (uint32_t)hi & 0xFFu; }
__device__ __forceinline__ uint32_t cid_size1(uint64_t hi) { return (uint32_t)(hi >> 8) & 0xFFu; }
__device__ __forceinline__ uint32_t cid_state(uint64_t hi) { return (uint32_t)(hi >> 16) & 0xFFu; }
__device__ __forceinline__ bool cid_on(uint64_t hi, uint32_t i) { return i < 32 && ((hi >> (32 + i)) & 1ull); }
__device__ __forceinline__ uint64_t cid_with_state(uint64_t hi, uint32_t s) { return (hi & ~0xFF0000ull) | ((uint64_t)s << 16); }
// get_extended_group_size (dare_config.h:78-86) of a cid word
__device__ __forceinline__ uint32_t cid_ext_size(uint64_t hi)
{
    const uint32_t s0 = cid_size0(hi), s1 = cid_size1(hi);
    if (cid_state(hi) == APUS_CID_STABLE) return s0;
    return s0 < s1 ? s1 : s0;
}

__device__ __forceinline__ bool ring_ok(const apus_group_state_t &st, uint64_t stride)
{
    return st.len >= kHdr && st.len <= stride && st.end <= st.len && st.commit <= st.len && st.apply <= st.len &&
           st.head <= st.len;
}

// poll_config_entries over [off, end): a CONFIG entry with idx > cid_idx whose
// cid differs from (c_lo, c_hi) replaces it and records the entry's req_id /
// clt_id (rq, cl; changed set), departures into dep; a HEAD entry at or before
// commit moves head_off.  off ends where the walk ends.  Returns false when
// the walk passes the step guard (the reference would not terminate).
__device__ inline bool scan_config(const uint8_t *ring, const apus_group_state_t &st, uint64_t cid_idx,
                                   uint64_t &off, uint64_t &c_lo, uint64_t &c_hi, uint64_t &rq, uint32_t &cl,
                                   uint32_t &dep, bool &changed, uint64_t &head_off)
{
    const uint64_t len = st.len, end = st.end, commit = st.commit;
    const uint64_t guard = len / kHdr + 4;
    uint64_t steps = 0;
    while (dist(end, len, off) != 0) {
        if (++steps > guard) return false;
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
    return true;
}

// apply_committed_entries' walk state (the config words, the config's req /
// clt, the bookkeeping of the applied client entries and the events)
struct ApplyAcc {
    uint64_t c_lo, c_hi;
    uint64_t rq, la_off, la2;
    uint32_t cl, na, nc, dep, ev;
    bool cfg_changed;
};

// The walk of apply_committed_entries from st.apply while commit is
// circularly larger.  IS_LEADER (leader): client entries applied (the last
// one's offset kept; its (idx, term) read once after the walk), NOOP / HEAD
// stepped over, a STABLE CONFIG with req_id != 0 -> APUS_EV_CFG_REPLY, an
// unstable CONFIG not older than the configuration's epoch moves it
// EXTENDED -> TRANSIT or TRANSIT -> STABLE (servers size[1]..size[0]-1
// removed) and re-appends a CONFIG entry: INLINE, log_append_entry in place
// (append_bare; st.end / tail move and the walk compares against the new end;
// prev cleared); else recorded in io's cfg rows (at most io.max_cfg, then
// APUS_EV_CFG_FULL and the walk stops).  Followers apply every type.
// st.apply is advanced in place.  Returns false on a walk past the step guard
// or an append refused (stopped).
template <bool INLINE>
__device__ inline bool apply_walk(const apus_batch_t &b, uint64_t g, apus_group_state_t &st, uint32_t self,
                                  bool leader, uint64_t term, ApplyAcc &a, const apus_apply_io_t *io,
                                  uint32_t &prev)
{
    const uint8_t *ring = b.ring + g * b.ring_stride;
    const uint64_t len = st.len, commit = st.commit;
    const uint64_t guard = len / kHdr + 4;
    const uint32_t M = INLINE ? 0u : io->max_cfg;
    uint64_t steps = 0;
    // while (log_is_offset_larger(log, commit, apply))
    while (dist(st.end, len, commit) < dist(st.end, len, st.apply)) {
        if (++steps > guard) return false;
        if (len - st.apply < kHdr) st.apply = 0;                       // log_get_entry
        const uint8_t *e = ring + st.apply;
        const uint32_t type = e[kType];
        const uint32_t el = entry_len(type, ld_u16(e + kData));
        if (len - st.apply < el) { st.apply = 0; continue; }           // !log_fit_entry
        if (leader && type == APUS_CONFIG) {
            const uint64_t e_lo = ld_u64(e + kData), e_hi = ld_u64(e + kData + 8);
            uint64_t rq = ld_u64(e + 16);
            uint32_t cl = ld_u16(e + 24);
            const uint32_t es = cid_state(e_hi);
            if (es == APUS_CID_STABLE) {
                if (rq != 0) a.ev |= APUS_EV_CFG_REPLY;                  // :1862-1875
            } else if (!(a.c_lo > e_lo)) {                                // :1877-1881
                if (!INLINE && a.nc == M) { a.ev |= APUS_EV_CFG_FULL; break; }
                if (es == APUS_CID_EXTENDED) {                            // :1888-1902
                    a.c_hi = cid_with_state(a.c_hi, APUS_CID_TRANSIT);
                    if (rq != 0) { a.ev |= APUS_EV_JOIN_REPLY; rq = 0; cl = 0; }
                } else if (es == APUS_CID_TRANSIT) {                     // :1903-1931
                    a.c_hi = cid_with_state(a.c_hi, APUS_CID_STABLE);
                    const uint32_t s0 = cid_size0(a.c_hi), s1 = cid_size1(a.c_hi);
                    for (uint32_t i = s1; i < s0; ++i) {
                        if (i == self) {
                            a.ev |= APUS_EV_SELF_REMOVED;
                            if (i < 32) a.c_hi &= ~(1ull << (32 + i));
                            continue;
                        }
                        if (!cid_on(a.c_hi, i)) continue;
                        a.c_hi &= ~(1ull << (32 + i));
                        if (i < 16) a.dep |= 1u << i;
                    }
                    a.c_hi = (a.c_hi & ~0xFFFFull) | s1;                  // size[0] = size[1]; size[1] = 0
                }
                a.rq = rq;
                a.cl = cl;
                a.cfg_changed = true;
                // log_append_entry(..., CONFIG, &data.config.cid), :1935-1937
                if (INLINE) {
                    const uint64_t w[2] = { a.c_lo, a.c_hi };
                    bool stopped = false;
                    (void)append_bare(b, g, st, prev, term, APUS_CONFIG, rq, cl, w, stopped);
                    if (stopped) return false;
                } else {
                    const uint64_t j = g * M + a.nc;
                    uint64_t *r = reinterpret_cast<uint64_t *>(io->cfg_entries + j);
                    r[0] = rq;
                    r[1] = 16ull * j;
                    r[2] = (uint64_t)cl | ((uint64_t)APUS_CONFIG << 16);
                    uint64_t *pl = reinterpret_cast<uint64_t *>(io->cfg_payload + 16ull * j);
                    pl[0] = a.c_lo;
                    pl[1] = a.c_hi;
                }
                ++a.nc;
            }
        } else if (!bare_type(type)) {                                  // apply_entry, :1939-1965
            // only the last applied entry's (idx, term) survives the walk:
            // its offset is kept and the pair read once after it
            a.la_off = st.apply;
            a.la2 = st.apply + el;
            ++a.na;
        }
        // apply_next_entry: the length read again after an inline append (an
        // append into a nearly full ring may overwrite this entry's bytes)
        st.apply += INLINE ? entry_len(e[kType], ld_u16(e + kData)) : el;
    }
    return true;
}

}  // namespace apus
