// Commit-path kernels for gfx950 (MI355X).
//
//   commit_wave_kernel  — one WAVE per consensus group.  Streams the group's
//       not-committed byte range [commit, end) of the circular log through a
//       per-wave LDS window with 16-B coalesced loads, walks the entry chain
//       (wave-uniform scalar walk, one LDS read per entry), tallies the
//       follower acks of up to 63 entries at once (lane per entry, exact
//       byte==1 test + popcount) and, fused in the same pass, computes the
//       Adler-32 of the walked entries' immutable images from per-window
//       prefix sums (v_dot4_u32_u8), so every log byte is read from HBM once.
//       Reference: APUS reply-count commit rule, update_remote_logs(),
//       src/dare/dare_ibv_rc.c:1725-1758 (walk), log primitives
//       src/include/dare/dare_log.h:255-332.
//   commit_lane_kernel  — one LANE per group, byte loads straight from global
//       memory; the same semantics in the reference's own shape (kept as a
//       second implementation for cross-checking, APUS_BATCH_LANE_IMPL).
//   median_kernel       — one lane per group, DARE median-offset quorum with
//       an in-register Batcher sorting network, dare_ibv_rc.c:1650-1723.
#include "apus_device.h"
#include "apus_internal.h"
#include "apus_stats.h"

#include <stdlib.h>
#include <string.h>

namespace apus {

constexpr int kWaves = 4;                 // waves per 256-thread block
constexpr int kCommitStats = 5;           // decisions, committed, advanced, corrupt, slow path
constexpr uint64_t kCommitStatMap = (uint64_t)APUS_STAT_DECISIONS | ((uint64_t)APUS_STAT_COMMITTED << 8) |
                                    ((uint64_t)APUS_STAT_ADVANCED << 16) | ((uint64_t)APUS_STAT_CORRUPT << 24) |
                                    ((uint64_t)APUS_STAT_SLOW << 32);

// ---------------------------------------------------------------------------
// small wave utilities
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_sum_mod(uint32_t v)
{
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        uint32_t t = __shfl_xor(v, d);
        v += t;
        v = v >= kAdlerMod ? v - kAdlerMod : v;
    }
    return v;
}

// 4-bit mask of the bytes of r equal to 1 (exact, no borrow false positives)
__device__ __forceinline__ uint32_t eq1_nibble(uint32_t r)
{
    const uint32_t x = r ^ 0x01010101u;
    const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
    return ((z >> 7) * 0x10204080u) >> 28;
}

__device__ __forceinline__ uint32_t udot4(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_udot4(a, b, c, false); }
__device__ __forceinline__ uint32_t byte_sum(uint32_t w) { return __builtin_amdgcn_udot4(w, 0x01010101u, 0u, false); }
// sum_j (j + 4i) * byte_j(w) for word i of a 16-byte piece
__device__ __forceinline__ uint32_t byte_wsum(uint32_t w, uint32_t i)
{
    return __builtin_amdgcn_udot4(w, 0x03020100u + 0x04040404u * i, 0u, false);
}

// sums (or mins) partials[nblk][nstat]; statistic k -> stats[(map >> 8k) & 0xFF]
__global__ void __launch_bounds__(256) stats_finalize_kernel(const uint64_t *partials, uint32_t nblk,
                                                             uint32_t nstat, uint64_t *stats,
                                                             uint64_t map, int is_min)
{
    __shared__ uint64_t red[256];
    for (uint32_t k = 0; k < nstat; ++k) {
        uint64_t s = is_min ? ~0ull : 0ull;
        for (uint32_t i = threadIdx.x; i < nblk; i += 256) {
            const uint64_t y = partials[(uint64_t)i * nstat + k];
            s = is_min ? (y < s ? y : s) : s + y;
        }
        red[threadIdx.x] = s;
        __syncthreads();
        for (int d = 128; d >= 1; d >>= 1) {
            if (threadIdx.x < (uint32_t)d) {
                const uint64_t y = red[threadIdx.x + d];
                red[threadIdx.x] = is_min ? (y < red[threadIdx.x] ? y : red[threadIdx.x]) : red[threadIdx.x] + y;
            }
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            unsigned long long *dst = (unsigned long long *)&stats[(map >> (8 * k)) & 0xFFu];
            if (is_min) atomicMin(dst, (unsigned long long)red[0]);
            else if (red[0]) atomicAdd(dst, (unsigned long long)red[0]);
        }
        __syncthreads();
    }
}

hipError_t launch_stats_finalize(const uint64_t *partials, uint32_t nblk, uint32_t nstat,
                                 uint64_t *stats, uint64_t map, bool is_min, hipStream_t s)
{
    hipLaunchKernelGGL(stats_finalize_kernel, dim3(1), dim3(256), 0, s, partials, nblk, nstat, stats, map,
                       is_min ? 1 : 0);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// One group walked by one lane, straight from global memory, 64-bit offsets:
// commit_lane_kernel's body, and commit_wave_kernel's path for rings of 2 GiB
// and more.  Writes the group's outputs; returns n_entries and
// flags = advanced | corrupt << 1.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t adler_bytes(const uint8_t *p, uint32_t n, uint32_t ad)
{
    uint32_t a = ad & 0xFFFF, bb = ad >> 16;
    for (uint32_t i = 0; i < n; ++i) {
        a += p[i];
        a = a >= kAdlerMod ? a - kAdlerMod : a;
        bb += a;
        bb = bb >= kAdlerMod ? bb - kAdlerMod : bb;
    }
    return (bb << 16) | a;
}

template <bool CHECKSUM>
__device__ __forceinline__ void lane_group(const apus_batch_t &b, const apus_commit_out_t &o, uint64_t g,
                                        uint32_t *n_out, uint32_t *flags_out)
{
    const apus_group_state_t st = b.state[g];
    const uint64_t len = st.len, end = st.end, commit0 = st.commit;
    const uint32_t self = b.self_idx[g];
    const uint32_t size = walk_size(st.cid);
    const uint32_t need = size / 2 + 1;
    const uint8_t *ring = b.ring + g * b.ring_stride;
    const uint64_t guard = len / kHdr + 4;
    uint64_t m = commit0, steps = 0, stop = 0;
    uint32_t n = 0, ad = 1;
    bool committing = true, stopped = false;
    // commit or end beyond len: corrupt (oracle/apus_oracle.c); else m <= len throughout
    bool corrupt = commit0 > len || end > len;
    while (!corrupt && dist(end, len, m)) {
        // the step guard flags the commit walk; past its stop it only ends the checksum
        if (++steps > guard) { corrupt = committing; break; }
        if (len - m < kHdr) m = 0;                        // log_get_entry
        const uint8_t *e = ring + m;
        const uint32_t type = e[kType];
        const uint32_t clen = ld_u16(e + kData);
        const uint32_t elen = entry_len(type, clen);
        if (len - m < elen) { m = 0; continue; }          // ghost header
        if (committing) {
            uint32_t votes = 0;
            for (uint32_t i = 0; i < size; ++i) votes += (i == self || e[kReply + i] == 1) ? 1u : 0u;
            if (votes < need) {
                committing = false; stopped = true; stop = m;
                if (!CHECKSUM) break;
            } else {
                ++n;
            }
        }
        if (CHECKSUM) {          // span with bytes 27..47 zeroed
            ad = adler_bytes(e, 27, ad);
            const uint32_t a0 = ad & 0xFFFF;
            ad = (((ad >> 16) + 21u * a0) % kAdlerMod << 16) | a0;
            ad = adler_bytes(e + kData, elen - kData, ad);
        }
        m += elen;
    }
    const uint64_t res = stopped ? stop : m;
    const bool adv = !corrupt && larger(end, len, res, commit0);
    if (o.new_commit) o.new_commit[g] = adv ? res : commit0;
    if (o.committed) o.committed[g] = corrupt ? 0xFF : (uint8_t)adv;
    if (o.n_entries) o.n_entries[g] = n;
    if (CHECKSUM && o.digest) o.digest[g] = ad;
    *n_out = n;
    *flags_out = (adv ? 1u : 0u) | (corrupt ? 2u : 0u);
}

// rings at least this long take lane_group inside commit_wave_kernel
constexpr uint64_t kWaveMaxLen = 1ull << 31;

// ---------------------------------------------------------------------------
// commit_wave_kernel
// ---------------------------------------------------------------------------
// One consensus group per wave, streamed through a per-wave LDS window.
//
// Windows: [ws, ws + WIN) with ws 16-B aligned in device memory; consecutive
// windows overlap by 64 B (ws' = ws + WIN - 64) so every entry header that
// starts in a window lies wholly inside it; after the ring end the sequence
// restarts at offset 0 (the walk's wrap).  The next window is prefetched into
// registers (16-B coalesced loads, 1 KiB per wave instruction) while the
// current one is processed.  Piece k (16 B) of a window lives at LDS slot
// k + k/8: entries of 128 B then hit 16 different banks per ds_read_b128.
//
// Walk: the APUS walk (dare_ibv_rc.c:1725-1758) is a chain -- the next entry
// starts where the current one ends.  Lanes walk it speculatively: lane j
// reads the header at m + j*elen (elen = the last length seen), and the
// chain is confirmed up to the first lane whose entry has another length or
// fails a walk condition (end reached, header/entry does not fit: the
// header-wrap of log_get_entry, dare_log.h:327-330, and the ghost-header jump
// are then taken by the wave-uniform prologue).  Equal-length runs of up to
// 64 entries are confirmed per LDS round trip with a handful of scalar ops.
//
// Acks: each lane tests reply[0..size) of its entry (byte == 1 exactly, self
// always counts); the first confirmed entry without a majority stops the
// commit (ballot + ctz).
//
// Checksum (APUS_COMMIT_CHECKSUM): Adler-32 over the concatenated entry spans
// with bytes 27..47 zeroed (oracle/apus_oracle.c).  Contiguous entries form a
// stretch whose image positions are ring position + constant, so per window
// the image sums are the byte sums of one ring range (per-piece v_dot4 sums
// computed while staging) minus each entry's bytes 27..47 (taken from the
// header registers) -- no per-byte walk.
__device__ __forceinline__ uint32_t pslot(uint32_t k) { return k + (k >> 3); }

// v_cndmask with a lane mask: LLVM turns select chains over an array into a
// dynamically indexed stack array (scratch); this keeps them in VGPRs
__device__ __forceinline__ uint32_t lsel(uint64_t lanes, uint32_t if_set, uint32_t if_clear)
{
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(lanes));
    return r;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// streaming 16-B load: every log byte is read once per batch
__device__ __forceinline__ uint4 ld_stream16(const uint8_t *p)
{
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t mod_add(uint32_t a, uint32_t b)
{
    const uint32_t c = a + b;
    return c >= kAdlerMod ? c - kAdlerMod : c;
}
__device__ __forceinline__ uint32_t mod_sub(uint32_t a, uint32_t b) { return mod_add(a, kAdlerMod - b); }

// bytes [lo, hi) of a 4-byte word (0 <= lo <= hi <= 4)
__device__ __forceinline__ uint32_t byte_mask(int lo, int hi)
{
    const uint32_t up = hi >= 4 ? 0xFFFFFFFFu : ((1u << (8 * hi)) - 1u);
    const uint32_t dn = lo >= 4 ? 0xFFFFFFFFu : ((1u << (8 * lo)) - 1u);
    return up & ~dn;
}

template <int WIN, bool CHECKSUM>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
commit_wave_kernel(const apus_batch_t b, const apus_commit_out_t o, uint64_t *partials)
{
    constexpr int NP = WIN / 16;          // 16-B pieces per window
    constexpr int PPL = NP / 64;          // pieces per lane
    constexpr int SLOTS = NP + NP / 8 + 16;
    constexpr int kMaxSlow = 32;          // per-wave list of groups for the exact slow path
    static_assert(NP % 64 == 0 && WIN >= 1024, "window must be a multiple of 1 KiB");

    __shared__ __attribute__((aligned(16))) uint4 s_win[kWaves][SLOTS];
    __shared__ uint32_t s_slow[kWaves][kMaxSlow];

    const uint32_t lane = lane_id();
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint4 *win = s_win[wv];
    // statistics in VGPR lanes 0..4 (decisions, committed, advanced, corrupt, slow):
    // scalar registers are the scarce resource of this kernel
    uint32_t acc_v = 0;
    auto account = [&](uint32_t n, uint32_t adv, uint32_t cor) {
        acc_v += lane == 0 ? 1u : lane == 1 ? n : lane == 2 ? adv : lane == 3 ? cor : 0u;
    };
    uint32_t elen_g = 128;                // speculation stride, carried across groups

    const uint32_t G = (uint32_t)b.n_groups;          // launch_commit: n_groups < 2^32
    const uint32_t gstride = gridDim.x * kWaves;
    // Group state rows are fetched one group ahead with VECTOR loads into
    // lanes 0..3 (16 B each; a scalar load would be waited for together with
    // the walk's LDS reads), and the next group's first window is prefetched
    // during this group's last window: group starts do not wait on HBM.
    auto load_state = [&](uint32_t gg, uint4 &sv, uint32_t &sf) {
        const uint32_t gc = gg < G ? gg : G - 1;
        sv = reinterpret_cast<const uint4 *>(b.state + gc)[lane & 3u];
        sf = b.self_idx[gc];
    };
    auto rl64 = [](uint32_t lo, uint32_t hi, int src) -> uint64_t {
        return (uint64_t)__builtin_amdgcn_readlane(lo, src) | ((uint64_t)__builtin_amdgcn_readlane(hi, src) << 32);
    };
    // Groups take the fast path when their ring is a 16-B aligned device
    // image padded by 16 B and shorter than 2 GiB (every batch this library
    // generates; the reference's rings are 64 MiB).  `fast_ring` is per batch.
    const bool fast_ring = (((uintptr_t)b.ring | b.ring_stride) & 15u) == 0;
    auto fast_group = [&](uint64_t len64, uint32_t hi_words) {
        return fast_ring && hi_words == 0 && len64 < kWaveMaxLen && b.ring_stride >= len64 + 16;
    };
    // a window's pieces: out-of-window lanes re-read piece 0 (dropped when the
    // window is staged), so the PPL loads issue back to back with no branch
    auto load_window = [&](uint4 (&r)[PPL], const uint8_t *base, uint32_t npc) {
#pragma unroll
        for (int j = 0; j < PPL; ++j) {
            const uint32_t k = lane + 64u * j;
            r[j] = ld_stream16(base + 16u * (k < npc ? k : 0u));
        }
    };

    uint32_t g = blockIdx.x * kWaves + wv;
    uint4 sv = make_uint4(0u, 0u, 0u, 0u);
    uint32_t sf = 0;
    if (g < G) load_state(g, sv, sf);
    bool pf_next = false;                 // nxt holds the first window of group g
    uint4 nxt[PPL];
    uint32_t n_slow = 0;                  // groups deferred to the slow path
    bool slow_all = false;                // list overflowed: redo every deferred group

    for (; g < G; g += gstride) {
        const uint64_t len64 = rl64(sv.z, sv.w, 2);
        const uint32_t hi_words = __builtin_amdgcn_readlane(sv.w, 1) | __builtin_amdgcn_readlane(sv.y, 1) |
                                  __builtin_amdgcn_readlane(sv.w, 2);
        const uint32_t cw = __builtin_amdgcn_readlane(sv.z, 3);
        const uint32_t self = uni(sf);
        const uint32_t gn = g + gstride;
        uint4 svn;
        uint32_t sfn;
        load_state(gn, svn, sfn);         // in flight while this group is walked

        // every offset of the walk fits 32 bits from here on
        const uint32_t len = (uint32_t)len64;
        const uint32_t end = __builtin_amdgcn_readlane(sv.z, 1), commit0 = __builtin_amdgcn_readlane(sv.x, 1);
        bool bail = !fast_group(len64, hi_words) || commit0 > len || end > len;
        const uint32_t st_size0 = cw & 0xFFu, st_size1 = (cw >> 8) & 0xFFu, st_state = (cw >> 16) & 0xFFu;
        const uint32_t size = st_state == APUS_CID_TRANSIT ? st_size1 : st_size0;   // walk_size
        const uint32_t need = size / 2 + 1;
        const uint32_t size_mask = size >= 16 ? 0xFFFFu : ((1u << size) - 1u);
        const uint32_t self_bit = self < 16 ? (1u << self) : 0u;
        const uint8_t *ring = b.ring + (uint64_t)g * b.ring_stride;

        // The window schedule, from the state alone: segment 0 is
        // [commit, wrapped ? len : end), segment 1 is [0, end) when the log
        // wraps; windows advance by WIN - 64 inside a segment (a header that
        // starts in a window lies wholly in it or in the next one).  A walk
        // that needs a byte outside the schedule (a malformed ring) bails to
        // the exact one-lane walk after the main loop.
        const bool wrapped = end < commit0;
        const uint32_t e0 = wrapped ? len : end;
        uint32_t m = commit0;
        bool walk_done = bail || dist32(end, len, m) == 0;
        bool forced = false, committing = true, stopped = false;
        uint32_t stop = 0, n_commit = 0;
        const uint32_t guard = len / kHdr + 4;
        uint32_t steps = 0;
        // checksum: per-lane image sums S = sum b, T = sum pos * b (mod M)
        uint32_t S = 0, T = 0;
        bool stretch = false, carry = false;   // stretch: an entry was confirmed in this segment
        uint32_t e_last = 0;              // end of the last confirmed entry
        uint32_t gap0 = 0;                // where segment 0's entries end (the wrap point)
        bool first_in_seg = true;         // no overlap with a previous window
        bool seg1 = false;                // in segment 1 (after the jump to offset 0)
        bool pending = false;             // jumped; the last entry's checksum still needs segment 0
        uint32_t ws = commit0 & ~15u;
        uint32_t we = min(ws + WIN, e0);
        if (!pf_next && !walk_done) load_window(nxt, ring + ws, (we - ws + 15) >> 4);
        pf_next = false;

        while (!walk_done || carry) {
            const uint32_t npc = (we - ws + 15) >> 4;

            // ---- 1. stage the window; sums over every staged byte ----
            // piece k = lane + 64 j holds window bytes [16k, 16k + 16):
            // s_pos = sum b, t_pos = sum (pos in piece) * b, j_pos = sum j * b
            uint32_t s_pos = 0, t_pos = 0, j_pos = 0;
#pragma unroll
            for (int j = 0; j < PPL; ++j) {
                const uint32_t k = lane + 64u * j;
                const uint4 v = k < npc ? nxt[j] : make_uint4(0u, 0u, 0u, 0u);
                win[pslot(k)] = v;
                if (CHECKSUM) {
                    const uint32_t s0 = udot4(v.w, 0x01010101u, udot4(v.z, 0x01010101u,
                                        udot4(v.y, 0x01010101u, udot4(v.x, 0x01010101u, 0u))));
                    s_pos += s0;
                    j_pos += (uint32_t)j * s0;
                    t_pos = udot4(v.w, 0x0F0E0D0Cu, udot4(v.z, 0x0B0A0908u,
                            udot4(v.y, 0x07060504u, udot4(v.x, 0x03020100u, t_pos))));
                }
            }
            // the window is in LDS and summed before the next one is
            // requested: its registers are reused by the prefetch
            if (CHECKSUM) asm volatile("" : "+v"(s_pos), "+v"(t_pos), "+v"(j_pos));
            asm volatile("" ::: "memory");

            // ---- 2. prefetch the next window of the schedule, or the next group's first ----
            const bool more0 = we < (seg1 ? end : e0);          // this segment continues
            const bool to_seg1 = !more0 && wrapped && !seg1;
            const uint32_t pws = more0 ? ws + WIN - 64 : 0u;
            const uint32_t pwe = more0 ? min(ws + 2 * WIN - 64, seg1 ? end : e0) : min((uint32_t)WIN, end);
            if (more0 || to_seg1) {
                load_window(nxt, ring + pws, (pwe - pws + 15) >> 4);
            } else if (gn < G) {
                const uint64_t l_n = rl64(svn.z, svn.w, 2);
                const uint32_t hi_n = __builtin_amdgcn_readlane(svn.w, 1) | __builtin_amdgcn_readlane(svn.y, 1) |
                                      __builtin_amdgcn_readlane(svn.w, 2);
                const uint32_t c_n = __builtin_amdgcn_readlane(svn.x, 1), e_n = __builtin_amdgcn_readlane(svn.z, 1);
                const uint32_t ln = (uint32_t)l_n;
                if (fast_group(l_n, hi_n) && dist32(e_n, ln, c_n) != 0) {
                    const uint32_t w0 = c_n & ~15u;
                    const uint32_t w1 = min(w0 + WIN, e_n < c_n ? ln : e_n);
                    load_window(nxt, b.ring + (uint64_t)gn * b.ring_stride + w0, (w1 - w0 + 15) >> 4);
                    pf_next = true;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

            // ---- 3. speculative walk over the headers of this window ----
            uint32_t exb = 0, exxb = 0;   // per-lane sums of the zeroed bytes 27..47
            bool jumped = false, jforced = false;
            while (!walk_done && !pending) {
                if (!forced && dist32(end, len, m) == 0) { walk_done = true; break; }
                if (len - m < kHdr) {                  // header does not fit: log_get_entry
                    jumped = true;                     // returns the entry at 0 unchecked
                    jforced = true;
                    break;
                }
                if (m < ws || m + kHdr > we) break;    // next window

                const uint32_t p = m + lane * elen_g;
                const bool inw = (lane == 0) | (p + kHdr <= we);
                // lanes past the window read entry 0's header (results dropped)
                const uint32_t rel = (inw ? p : m) - ws;
                const uint32_t k0 = (rel + 24u) >> 4;
                const uint4 a = win[pslot(k0)], bq = win[pslot(k0 + 1)], c = win[pslot(k0 + 2)];
                const uint32_t r[12] = { a.x, a.y, a.z, a.w, bq.x, bq.y, bq.z, bq.w, c.x, c.y, c.z, c.w };
                const uint32_t q = (rel + 24u) & 15u, qb = q & 3u;
                const uint64_t q1 = __ballot((q & 4u) != 0), q2 = __ballot((q & 8u) != 0);
                uint32_t u[11];
#pragma unroll
                for (int i = 0; i < 11; ++i) u[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], qb);
                uint32_t ev[7];          // ev[i] = entry bytes [24 + 4i, 28 + 4i)
#pragma unroll
                for (int i = 0; i < 7; ++i)
                    ev[i] = lsel(q2, lsel(q1, u[i + 3], u[i + 2]), lsel(q1, u[i + 1], u[i]));
                const uint32_t type = (ev[0] >> 16) & 0xFFu;    // byte 26
                const uint32_t clen = ev[6] & 0xFFFFu;          // bytes 48..49
                const uint32_t elen = bare_type(type) ? kHdr : kHdr + clen;
                const bool ok = inw & ((lane == 0) | (p != end)) & (len - p >= elen);
                const bool cont = ok & (elen == elen_g) & (lane < 63);
                const uint64_t okb = __ballot(ok);
                const uint32_t fb = (uint32_t)__builtin_ctzll(__ballot(!cont));
                const uint32_t nconf = fb + (uint32_t)((okb >> fb) & 1ull);
                if (nconf == 0) {                      // ghost header at m: continue at 0
                    jumped = true;                     // (the loop re-checks the distance)
                    break;
                }
                const bool conf = lane < nconf;
                if (committing) {
                    uint32_t msk = eq1_nibble(ev[1]) | (eq1_nibble(ev[2]) << 4) | (eq1_nibble(ev[3]) << 8) |
                                   (eq1_nibble(ev[4]) << 12);
                    msk = (msk | self_bit) & size_mask;
                    const uint64_t fbits = __ballot(conf & ((uint32_t)__builtin_popcount(msk) < need));
                    const uint32_t ef = fbits ? (uint32_t)__builtin_ctzll(fbits) : nconf;
                    stop = m + ef * elen_g;
                    stopped = fbits != 0;
                    committing = !stopped;
                    n_commit += ef;
                }
                if (CHECKSUM) {
                    // the zeroed bytes 27..47 of confirmed entries
                    const uint32_t snd = ev[0] >> 24;          // byte 27
                    const uint32_t sb = snd + byte_sum(ev[1]) + byte_sum(ev[2]) + byte_sum(ev[3]) +
                                        byte_sum(ev[4]) + byte_sum(ev[5]);
                    const uint32_t stb = 27u * snd + byte_wsum(ev[1], 7) + byte_wsum(ev[2], 8) +
                                         byte_wsum(ev[3], 9) + byte_wsum(ev[4], 10) + byte_wsum(ev[5], 11);
                    exb = (exb + (conf ? sb : 0u)) % kAdlerMod;
                    exxb = (exxb + (conf ? rel * sb + stb : 0u)) % kAdlerMod;   // rel < 2^14, sb < 2^13
                    stretch = true;
                }
                const uint32_t elen_last = __builtin_amdgcn_readlane(elen, nconf - 1);
                m = m + (nconf - 1) * elen_g + elen_last;
                e_last = m;
                elen_g = elen_last;
                forced = false;
                steps += nconf;
                if (!CHECKSUM && !committing) { walk_done = true; break; }
            }

            // ---- 4. checksum: fold this window's image bytes into S, T ----
            if (CHECKSUM) {
                // staged but not new image bytes: the overlap with the previous
                // window (or the bytes before commit), and everything from the
                // wrap point (segment 0 once the jump is seen) or from `we` on
                const uint32_t rel_hi = we - ws, rel_pc = npc * 16u;
                const uint32_t rel_lo = first_in_seg ? (seg1 ? 0u : commit0 - ws) : 64u;
                const uint32_t gap_now = jumped ? m : gap0;
                const uint32_t gap_rel = (jumped || pending) ? min(gap_now - ws, rel_hi) : rel_hi;
                uint32_t s_neg = exb, t_neg = exxb;
                auto sub_range = [&](uint32_t lo, uint32_t hi) {
                    for (uint32_t base = lo & ~3u; base < hi; base += 256u) {
                        const uint32_t x0 = base + 4u * lane;
                        const uint32_t d = (x0 < hi ? x0 : base) >> 2;       // stay inside the window
                        uint32_t x = reinterpret_cast<const uint32_t *>(win + pslot(d >> 2))[d & 3u];
                        const int blo = (int)lo - (int)x0, bhi = (int)hi - (int)x0;
                        x &= byte_mask(blo < 0 ? 0 : blo > 4 ? 4 : blo, bhi < 0 ? 0 : bhi > 4 ? 4 : bhi);
                        const uint32_t s0 = byte_sum(x);
                        s_neg += s0;
                        t_neg += udot4(x, 0x03020100u, x0 * s0);
                    }
                };
                sub_range(0u, rel_lo);
                sub_range(gap_rel, rel_pc);
                // image position of window byte 0
                const uint32_t coef = seg1 ? (gap0 - commit0 + ws) % kAdlerMod
                                           : (ws % kAdlerMod + kAdlerMod - commit0 % kAdlerMod) % kAdlerMod;
                // window-relative positions: piece k byte i sits at 16 k + i
                const uint32_t tp = (t_pos + 16u * (lane * s_pos + 64u * j_pos)) % kAdlerMod;   // < 2^28
                const uint32_t dS = mod_sub(s_pos % kAdlerMod, s_neg % kAdlerMod);
                const uint32_t dT = mod_sub(tp, t_neg % kAdlerMod);
                S = mod_add(S, dS);
                T = (T + coef * dS + dT) % kAdlerMod;   // 65521^2 + 2*65521 < 2^32
            }
            carry = CHECKSUM && stretch && e_last > we;

            // ---- 5. the next window ----
            if (jumped) {
                // log_get_entry's header wrap / the ghost-header jump: legal
                // only from segment 0 of a wrapped log, into segment 1
                if (!wrapped || seg1 || pending) { bail = true; break; }
                gap0 = m;
                m = 0;
                forced = jforced;
                ++steps;
                pending = true;
            }
            // segment 1 starts once the entry before the jump is summed
            const bool next_seg1 = pending && !carry;
            if (next_seg1) { pending = false; stretch = false; seg1 = true; }
            first_in_seg = next_seg1;
            if (steps > guard) { bail = true; break; }         // corrupt ring: the slow path decides
            if (!next_seg1 && !pending && walk_done && !carry) break;
            if (!next_seg1 && !more0) { bail = true; break; }   // the walk leaves the schedule
            if (next_seg1) {
                ws = 0u;
                we = min((uint32_t)WIN, end);
                // jumped before segment 0's last window: the prefetch was segment 0's
                if (!to_seg1) load_window(nxt, ring, (we + 15) >> 4);
            } else {
                ws = pws;                                     // the prefetched window
                we = pwe;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }

        if (bail) {
            // the exact one-lane walk after the main loop
            if (n_slow < kMaxSlow) {
                if (lane == 0) s_slow[wv][n_slow] = g;
            } else {
                slow_all = true;
            }
            ++n_slow;
        } else {
            const uint32_t res = stopped ? stop : m;
            const bool adv = dist32(end, len, res) < dist32(end, len, commit0);
            uint32_t digest = 1;
            if (CHECKSUM) {
                // image length: the entries tile [commit, end), or [commit, gap0) ++ [0, end)
                const uint32_t N = dist32(end, len, commit0) == 0 ? 0u
                                 : (wrapped ? gap0 - commit0 + end : end - commit0) % kAdlerMod;
                const uint32_t Sa = wave_sum_mod(S), Ta = wave_sum_mod(T);
                const uint32_t A = (1u + Sa) % kAdlerMod;
                const uint32_t B = (N + N * Sa + kAdlerMod - Ta) % kAdlerMod;
                digest = (B << 16) | A;
            }
            if (lane == 0) {
                if (o.new_commit) o.new_commit[g] = adv ? (uint64_t)res : (uint64_t)commit0;
                if (o.committed) o.committed[g] = (uint8_t)adv;
                if (o.n_entries) o.n_entries[g] = n_commit;
                if (CHECKSUM && o.digest) o.digest[g] = digest;
            }
            account(n_commit, adv ? 1u : 0u, 0u);
        }
        sv = svn;
        sf = sfn;
    }

    if (n_slow) {
        // the one-lane walk in 64-bit offsets (lane_group, exact for every
        // input), lane 0 of this wave, over the groups this wave deferred
        // list overflow: every group of this wave is walked again (the
        // outputs are rewritten with the same values) and counted afresh
        const uint32_t g0 = blockIdx.x * kWaves + wv;
        const uint32_t cnt = slow_all ? (G - 1 - g0) / gstride + 1 : n_slow;
        if (slow_all) acc_v = 0;
        for (uint32_t i = 0; i < cnt; ++i) {
            const uint32_t gb = slow_all ? g0 + i * gstride : s_slow[wv][i];
            uint32_t n = 0, fl = 0;
            if (lane == 0) lane_group<CHECKSUM>(b, o, gb, &n, &fl);
            account(uni(n), uni(fl) & 1u, uni(fl) >> 1);
            acc_v += lane == 4 ? 1u : 0u;
        }
    }
    uint64_t mine[kCommitStats];   // lane k holds statistic k: count it once per wave
#pragma unroll
    for (int k = 0; k < kCommitStats; ++k) mine[k] = lane == 0 ? __builtin_amdgcn_readlane(acc_v, k) : 0u;
    block_partials<kCommitStats>(partials, mine);
}

// ---------------------------------------------------------------------------
// commit_lane_kernel: one lane per group (APUS_BATCH_LANE_IMPL)
// ---------------------------------------------------------------------------
template <bool CHECKSUM>
__global__ void __launch_bounds__(256) commit_lane_kernel(const apus_batch_t b, const apus_commit_out_t o,
                                                          uint64_t *partials)
{
    uint64_t acc[kCommitStats] = { 0, 0, 0, 0, 0 };
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t n, fl;
        lane_group<CHECKSUM>(b, o, g, &n, &fl);
        acc[0] += 1; acc[1] += n; acc[2] += fl & 1u; acc[3] += fl >> 1;
    }
    block_partials<kCommitStats>(partials, acc);
}

// ---------------------------------------------------------------------------
// median_kernel: DARE median-offset quorum, one lane per group
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void sort_network(uint64_t (&a)[N])
{
    // Batcher odd-even merge sort; every index is a compile-time constant
#pragma unroll
    for (int p = 1; p < N; p <<= 1)
#pragma unroll
        for (int k = p; k >= 1; k >>= 1)
#pragma unroll
            for (int j = k % p; j + k < N; j += 2 * k)
#pragma unroll
                for (int i = 0; i < k; ++i)
                    if (i + j + k < N && (i + j) / (2 * p) == (i + j + k) / (2 * p)) {
                        const uint64_t x = a[i + j], y = a[i + j + k];
                        a[i + j] = x < y ? x : y;
                        a[i + j + k] = x < y ? y : x;
                    }
}

template <int N>
__global__ void __launch_bounds__(256) median_kernel(const apus_batch_t b, uint64_t *median)
{
    const uint32_t R = b.n_replicas;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const apus_group_state_t st = b.state[g];
        const uint64_t len = st.len, end = st.end, commit = st.commit;
        const uint32_t self = b.self_idx[g];
        const bool transit = st.cid.state == APUS_CID_TRANSIT;
        const uint64_t *rend = b.remote_end + g * R;
        const uint8_t *step = b.lr_step + g * R;
        const uint8_t *fail = b.fail_count + g * R;
        // offsets the reference gathers for i < size (dare_ibv_rc.c:1660-1676);
        // slot values do not depend on j, only which slots are live does
        uint64_t off[N];
        uint32_t upd = 0;    // bit i: replica i contributes its remote end
#pragma unroll
        for (int i = 0; i < N; ++i) {
            uint64_t v = commit;
            if ((uint32_t)i == self) v = end;
            else if ((uint32_t)i < R && ((st.cid.bitmask >> i) & 1u) && fail[i] < APUS_PERMANENT_FAILURE &&
                     step[i] == APUS_LR_UPDATE_LOG) {
                v = rend[i];
                upd |= 1u << i;
            }
            off[i] = v;
        }
        uint64_t minv = commit;
        for (int j = 0; j < 2;) {
            const uint32_t size = st.cid.size[j];
            int cnt = 0;
#pragma unroll
            for (int i = 0; i < N; ++i)
                if ((uint32_t)i < size && ((upd >> i) & 1u) && larger(end, len, off[i], minv)) ++cnt;
            if (cnt < (int)(size / 2)) {
                if (!transit) break;
                if (j == 0) { ++j; continue; }
                break;
            }
            uint64_t srt[N];
#pragma unroll
            for (int i = 0; i < N; ++i) srt[i] = (uint32_t)i < size ? off[i] : ~0ull;
            sort_network<N>(srt);
            const uint32_t mi = (size - 1) / 2;
            uint64_t med = srt[0];
#pragma unroll
            for (int i = 0; i < N; ++i)
                if ((uint32_t)i == mi) med = srt[i];
            if (!transit) { minv = med; break; }
            if (j == 0) minv = med;
            else if (larger(end, len, minv, med)) minv = med;
            ++j;
        }
        median[g] = minv;
    }
}

// ---------------------------------------------------------------------------
// launches
// ---------------------------------------------------------------------------
uint32_t grid_for(uint64_t units, uint32_t per_block, int n_cu, uint32_t per_cu)
{
    uint64_t need = (units + per_block - 1) / per_block;
    uint64_t cap = (uint64_t)(n_cu > 0 ? n_cu : 256) * per_cu;
    if (need > cap) need = cap;
    return need ? (uint32_t)need : 1u;
}

hipError_t ensure_partials(apus_ctx *ctx, size_t slots)
{
    if (slots <= ctx->partials_cap) return hipSuccess;
    if (ctx->partials) (void)hipFree(ctx->partials);
    ctx->partials = nullptr;
    ctx->partials_cap = 0;
    hipError_t e = hipMalloc(&ctx->partials, slots * sizeof(uint64_t));
    if (e == hipSuccess) ctx->partials_cap = slots;
    return e;
}

static int commit_win()
{
    static int w = -1;
    if (w < 0) {
        const char *e = getenv("APUS_COMMIT_WIN");
        w = (e && atoi(e) == 4096) ? 4096 : 8192;
    }
    return w;
}

template <int WIN>
static hipError_t launch_wave(apus_ctx *ctx, const apus_batch_t &b, const apus_commit_out_t &o, bool ck,
                              hipStream_t s, uint32_t *grid_out)
{
    static int occ[2] = { 0, 0 };
    int &oc = occ[ck ? 1 : 0];
    if (!oc) {
        if (ck) (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&oc, commit_wave_kernel<WIN, true>, 256, 0);
        else (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&oc, commit_wave_kernel<WIN, false>, 256, 0);
        if (oc <= 0) oc = 2;
    }
    // persistent: exactly the blocks that are resident at once
    const uint32_t grid = grid_for(b.n_groups, kWaves, ctx->n_cu, (uint32_t)oc);
    hipError_t e = ensure_partials(ctx, (size_t)grid * kCommitStats);
    if (e != hipSuccess) return e;
    if (ck) hipLaunchKernelGGL((commit_wave_kernel<WIN, true>), dim3(grid), dim3(256), 0, s, b, o, ctx->partials);
    else hipLaunchKernelGGL((commit_wave_kernel<WIN, false>), dim3(grid), dim3(256), 0, s, b, o, ctx->partials);
    *grid_out = grid;
    return hipGetLastError();
}

hipError_t launch_commit(apus_ctx *ctx, const apus_batch_t &b, const apus_commit_out_t &o,
                         uint32_t flags, hipStream_t s)
{
    if (b.n_groups == 0) return hipSuccess;
    const bool ck = (flags & APUS_COMMIT_CHECKSUM) != 0;
    if (flags & (APUS_COMMIT_WALK | APUS_COMMIT_CHECKSUM)) {
        uint32_t grid;
        hipError_t e;
        if (b.flags & APUS_BATCH_LANE_IMPL) {
            grid = grid_for(b.n_groups, 256, ctx->n_cu, 8);
            if ((e = ensure_partials(ctx, (size_t)grid * kCommitStats)) != hipSuccess) return e;
            if (ck) hipLaunchKernelGGL(commit_lane_kernel<true>, dim3(grid), dim3(256), 0, s, b, o, ctx->partials);
            else hipLaunchKernelGGL(commit_lane_kernel<false>, dim3(grid), dim3(256), 0, s, b, o, ctx->partials);
            e = hipGetLastError();
        } else if (commit_win() == 8192) {
            e = launch_wave<8192>(ctx, b, o, ck, s, &grid);
        } else {
            e = launch_wave<4096>(ctx, b, o, ck, s, &grid);
        }
        if (e != hipSuccess) return e;
        e = launch_stats_finalize(ctx->partials, grid, kCommitStats, ctx->stats, kCommitStatMap, false, s);
        if (e != hipSuccess) return e;
    }
    if ((flags & APUS_COMMIT_MEDIAN) && o.median) {
        const uint32_t grid = grid_for(b.n_groups, 256, ctx->n_cu, 8);
        if (b.n_replicas <= 8) hipLaunchKernelGGL(median_kernel<8>, dim3(grid), dim3(256), 0, s, b, o.median);
        else hipLaunchKernelGGL(median_kernel<16>, dim3(grid), dim3(256), 0, s, b, o.median);
        return hipGetLastError();
    }
    return hipSuccess;
}

}  // namespace apus
