// Device-side helpers shared by the libapus_gpu kernels (gfx950 only).
//
// Circular-log arithmetic of src/include/dare/dare_log.h restated for the
// GPU: every comparison is by distance to `end` (dare_log.h:255-282), never
// numeric, except where the reference itself sorts numerically
// (dare_ibv_rc.c:1688-1696).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/apus_gpu.h"

namespace apus {

constexpr uint32_t kHdr = APUS_ENTRY_HDR;   // sizeof(dare_log_entry_t)
constexpr uint32_t kAdlerMod = 65521u;      // RFC 1950

// entry header byte offsets (dare_log.h:33-48)
constexpr uint32_t kIdx = 0, kTerm = 8, kType = 26, kSender = 27, kReply = 28, kData = 48;

__device__ __forceinline__ uint64_t dist(uint64_t end, uint64_t len, uint64_t o)
{
    // log_offset_end_distance, dare_log.h:255-262
    if (end == len) return 0;
    return end >= o ? end - o : len - (o - end);
}

// the same in 32-bit offsets (rings below 2 GiB)
__device__ __forceinline__ uint32_t dist32(uint32_t end, uint32_t len, uint32_t o)
{
    if (end == len) return 0;
    return end >= o ? end - o : len - (o - end);
}

__device__ __forceinline__ bool larger(uint64_t end, uint64_t len, uint64_t a, uint64_t b)
{
    // log_is_offset_larger, dare_log.h:269-282
    return dist(end, len, a) < dist(end, len, b);
}

__device__ __forceinline__ bool bare_type(uint32_t t)
{
    // log_entry_len, dare_log.h:228-234
    return t == APUS_NOOP || t == APUS_CONFIG || t == APUS_HEAD;
}

__device__ __forceinline__ uint32_t entry_len(uint32_t type, uint32_t clen)
{
    return bare_type(type) ? kHdr : kHdr + clen;
}

// bytes of the entry's data that enter the build-defined checksum image
// (apus_oracle.c image_data_len)
__device__ __forceinline__ uint32_t image_data_len(uint32_t type, uint32_t clen)
{
    return type == APUS_NOOP ? 0u : type == APUS_CONFIG ? 16u : type == APUS_HEAD ? 8u : 2u + clen;
}

// `size` the APUS reply walk uses: what the median loop leaves behind
// (dare_ibv_rc.c:1656,1733) = cid.size[1] in CID_TRANSIT, else cid.size[0]
// (both sizes are read as values and then selected: a select between
// c.size[0] and c.size[1] folds into a variable index, and a variable index
// into a local cid makes the compiler keep it in LDS)
__device__ __forceinline__ uint32_t walk_size(const apus_cid_t &c)
{
    const uint32_t s0 = c.size[0], s1 = c.size[1];
    return c.state == APUS_CID_TRANSIT ? s1 : s0;
}

__device__ __forceinline__ uint32_t group_size(const apus_cid_t &c)
{
    // get_group_size, dare_config.h:89-97
    const uint32_t s0 = c.size[0], s1 = c.size[1];
    if (c.state != APUS_CID_TRANSIT) return s0;
    return s0 < s1 ? s1 : s0;
}

__device__ __forceinline__ uint32_t ext_group_size(const apus_cid_t &c)
{
    // get_extended_group_size, dare_config.h:78-86
    const uint32_t s0 = c.size[0], s1 = c.size[1];
    if (c.state == APUS_CID_STABLE) return s0;
    return s0 < s1 ? s1 : s0;
}

// little-endian reads at arbitrary byte offsets of global memory: aligned
// wide loads where the address allows, a dword funnel (v_alignbyte) for a
// misaligned u64 -- lane-per-group walkers touch a different line per lane,
// so every load instruction saved is a 64-line address pass saved
__device__ __forceinline__ uint32_t ld_u8(const uint8_t *p) { return *p; }
__device__ __forceinline__ uint32_t ld_u16(const uint8_t *p)
{
    if (((uintptr_t)p & 1u) == 0) return *reinterpret_cast<const uint16_t *>(p);
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8);
}
__device__ __forceinline__ uint64_t ld_u64(const uint8_t *p)
{
    const uintptr_t a = (uintptr_t)p;
    if ((a & 7u) == 0) return *reinterpret_cast<const uint64_t *>(p);
    const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3u), d0 = w[0], d1 = w[1], d2 = w[2];
    return (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sh) |
           ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32);
}
// idx@0 and term@8 of an entry header (16 bytes from p)
__device__ __forceinline__ void ld_idx_term(const uint8_t *p, uint64_t &idx, uint64_t &term)
{
    const uintptr_t a = (uintptr_t)p;
    if ((a & 7u) == 0) {
        idx = *reinterpret_cast<const uint64_t *>(p);
        term = *reinterpret_cast<const uint64_t *>(p + 8);
        return;
    }
    const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3u), d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3], d4 = w[4];
    idx = (uint64_t)__builtin_amdgcn_alignbyte(d1, d0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(d2, d1, sh) << 32);
    term = (uint64_t)__builtin_amdgcn_alignbyte(d3, d2, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(d4, d3, sh) << 32);
}

__device__ __forceinline__ uint32_t adler_mod(uint32_t x) { return x % kAdlerMod; }

// v_writelane (lane `lane` of `old` := uniform v).  clang exposes no builtin
// for it; the LLVM intrinsic is bound by name, so the compiler still does the
// register allocation and the SGPR lane-select hazard padding.
extern "C" __device__ uint32_t apus_writelane_i32(uint32_t v, uint32_t lane, uint32_t old)
    __asm("llvm.amdgcn.writelane.i32");

// uniform value helpers
__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v)
{
    uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Cross-lane prefix sums with gfx9 DPP moves instead of ds_bpermute: a scan
// step costs a VALU op, not an LDS round trip (a 6-step __shfl_up scan is a
// chain of six).  row_shr:n inside each 16-lane row (bound_ctrl: lanes whose
// source lies outside the row read 0), then row_bcast:15 (rows 1, 3 take the
// last lane of the row before) and row_bcast:31 (rows 2, 3 take lane 31).
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ uint32_t dpp0(uint32_t x)
{
    return __builtin_amdgcn_update_dpp(0u, x, CTRL, ROWS, 0xF, true);
}
// inclusive prefix sum within each 16-lane row
__device__ __forceinline__ uint32_t row_scan_incl(uint32_t x)
{
    uint32_t y = x + dpp0<0x111>(x);     // row_shr:1
    y += dpp0<0x112>(x);                 // row_shr:2
    y += dpp0<0x113>(x);                 // row_shr:3 (sums of 4)
    y += dpp0<0x114>(y);                 // row_shr:4 (sums of 8)
    y += dpp0<0x118>(y);                 // row_shr:8 (the row)
    return y;
}
// inclusive prefix sum over the wave
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x)
{
    uint32_t y = row_scan_incl(x);
    y += dpp0<0x142, 0xA>(y);            // row_bcast:15
    y += dpp0<0x143, 0xC>(y);            // row_bcast:31
    return y;
}
// lane l takes lane l - 1's value (lane 0: 0): wave_shr:1
__device__ __forceinline__ uint32_t wave_shr1(uint32_t x) { return dpp0<0x138>(x); }
__device__ __forceinline__ uint64_t wave_shr1_64(uint64_t x)
{
    return ((uint64_t)wave_shr1((uint32_t)(x >> 32)) << 32) | wave_shr1((uint32_t)x);
}

// SplitMix64 and the keyed draw of the synthetic generator
// (oracle/apus_oracle.c sm64 / draw)
__host__ __device__ __forceinline__ uint64_t sm64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__host__ __device__ __forceinline__ uint64_t draw(uint64_t gkey, uint64_t k)
{
    return sm64(gkey ^ (k * 0xD1B54A32D192ED03ull));
}

// ---------------------------------------------------------------------------
// group g's log offsets + configuration: the 64-B state row, or, for a batch
// of dare_log_t images (APUS_BATCH_LOG_IMAGE), the image's own header fields
// (dare_log.h:79-95) and config.cid from b.cid
// ---------------------------------------------------------------------------
static_assert(APUS_LOG_HDR_BYTES == sizeof(apus_log_t), "dare_log_t header size");
__device__ __forceinline__ const uint64_t *log_header(const apus_batch_t &b, uint64_t g)
{
    return reinterpret_cast<const uint64_t *>(b.ring + g * b.ring_stride - APUS_LOG_HDR_BYTES);
}
__device__ __forceinline__ apus_group_state_t load_state(const apus_batch_t &b, uint64_t g)
{
    if (b.flags & APUS_BATCH_LOG_IMAGE) {
        const uint64_t *h = log_header(b, g);
        apus_group_state_t s;
        s.head = h[0];
        s.apply = h[1];
        s.commit = h[2];
        s.end = h[3];
        s.tail = h[4];
        s.len = h[7];
        s.cid = b.cid[g];
        return s;
    }
    return b.state[g];
}

// The offsets the writers update, in place: head@0 apply@8 commit@16 end@24
// tail@32 in both layouts (the state row and the dare_log_t header share
// them; len is at 40 in a row, 56 in a header), and config.cid (the row's, or
// b.cid[g] for an image).  The reference's writers update the same fields of
// its dare_log_t (log_append_entry: end/tail, apply_committed_entries: apply,
// poll_config_entries: head, log_adjustment: commit) and data.config.cid.
constexpr int kOffHead = 0, kOffApply = 1, kOffCommit = 2, kOffEnd = 3, kOffTail = 4;
__device__ __forceinline__ uint64_t *offsets_of(const apus_batch_t &b, uint64_t g)
{
    if (b.flags & APUS_BATCH_LOG_IMAGE) return const_cast<uint64_t *>(log_header(b, g));
    return reinterpret_cast<uint64_t *>(b.state + g);
}
__device__ __forceinline__ uint64_t *cid_words(const apus_batch_t &b, uint64_t g)
{
    return reinterpret_cast<uint64_t *>((b.flags & APUS_BATCH_LOG_IMAGE) ? b.cid + g : &b.state[g].cid);
}

// Bytes of group g's ring a kernel may touch: the stride, less the next
// image's dare_log_t header for APUS_BATCH_LOG_IMAGE (batch_ok: stride >=
// header).  A valid group has len <= ring_cap; every kernel bounds its ring
// accesses by it, so a corrupt len never reaches past the group's ring.
__host__ __device__ __forceinline__ uint64_t ring_cap(const apus_batch_t &b)
{
    return (b.flags & APUS_BATCH_LOG_IMAGE) ? b.ring_stride - APUS_LOG_HDR_BYTES : b.ring_stride;
}

// ---------------------------------------------------------------------------
// walker over the entries in [o, end) in the style of log_get_tail /
// log_entries_to_nc_buf (offset recorded BEFORE the ghost test)
// ---------------------------------------------------------------------------
struct RingView {
    const uint8_t *ring;
    uint64_t end, len;
    uint64_t cap;          // ring_cap: the bytes at `ring` that belong to the group
    __device__ __forceinline__ bool get_entry(uint64_t &o) const
    {
        // log_get_entry, dare_log.h:316-332
        if (end == len) return false;
        if (dist(end, len, o) == 0) return false;
        if (len - o < kHdr) o = 0;
        // an offset past the ring (never produced by a valid log; undefined in
        // the reference) must not turn into an out-of-bounds device read
        return len >= kHdr && o <= len - kHdr && cap >= kHdr && o <= cap - kHdr;   // o + kHdr <= len, cap
    }
    __device__ __forceinline__ uint32_t elen_at(uint64_t o) const
    {
        const uint8_t *e = ring + o;
        return entry_len(e[kType], ld_u16(e + kData));
    }
};

__device__ __forceinline__ RingView ring_view(const apus_batch_t &b, uint64_t g, const apus_group_state_t &st)
{
    return RingView{ b.ring + g * b.ring_stride, st.end, st.len, ring_cap(b) };
}

// log_get_tail, dare_log.h:402-457
__device__ inline uint64_t device_get_tail(const RingView &v, const apus_group_state_t &st)
{
    if (st.tail != st.len) return st.tail;
    if (st.end == st.len) return st.len;
    const uint64_t guard = st.len / kHdr + 4;
    const uint64_t starts[3] = { st.commit, st.apply, st.head };
#pragma unroll
    for (int s = 0; s < 3; ++s) {
        uint64_t o = starts[s], tail = st.len, n = 0;
        while (v.get_entry(o) && n++ < guard) {
            tail = o;
            const uint32_t el = v.elen_at(o);
            if (v.len - o < el) o = 0;
            o += el;
        }
        if (tail != st.len) return tail;
    }
    return st.len;
}

}  // namespace apus
