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
//   quorum_tail_kernel  — one launch after the walk: the deferred groups'
//       exact walks, per group the DARE median-offset quorum
//       (dare_ibv_rc.c:1650-1723) and log_pruning's minimum
//       (dare_server.c:2026-2058) from one read of the state row, and the
//       statistics fold in the last arriving block.
#include "apus_device.h"
#include "apus_group_ops.h"
#include "apus_internal.h"
#include "apus_stats.h"

#include <hip/hip_ext.h>
#include <stdlib.h>
#include <string.h>

namespace apus {

constexpr int kWaves = 4;                 // waves per 256-thread block
constexpr int kCommitStats = 5;           // decisions, committed, advanced, corrupt, slow path
constexpr int kWaveStats = 3;             // commit_wave_kernel's: decisions, committed, advanced
constexpr uint64_t kCommitStatMap = (uint64_t)APUS_STAT_DECISIONS | ((uint64_t)APUS_STAT_COMMITTED << 8) |
                                    ((uint64_t)APUS_STAT_ADVANCED << 16) | ((uint64_t)APUS_STAT_CORRUPT << 24) |
                                    ((uint64_t)APUS_STAT_SLOW << 32);
// commit_wave_kernel: the NC determinants (a9) written by the walk (checksum builds only)
constexpr uint32_t kEpiNc = 4;

// ---------------------------------------------------------------------------
// small wave utilities
// ---------------------------------------------------------------------------
// 4-bit mask of the bytes of r equal to 1 (exact, no borrow false positives)
__device__ __forceinline__ uint32_t eq1_nibble(uint32_t r)
{
    const uint32_t x = r ^ 0x01010101u;
    const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);
    return ((z >> 7) * 0x10204080u) >> 28;
}

__device__ __forceinline__ uint32_t udot4(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_udot4(a, b, c, false); }
__device__ __forceinline__ uint32_t byte_sum(uint32_t w) { return __builtin_amdgcn_udot4(w, 0x01010101u, 0u, false); }
// sums (or mins: bit k of min_mask) partials[nblk][nstat]; statistic k -> stats[(map >> 8k) & 0xFF]
__global__ void __launch_bounds__(256) stats_finalize_kernel(const uint64_t *partials, uint32_t nblk,
                                                             uint32_t nstat, uint64_t *stats,
                                                             uint64_t map, uint32_t min_mask, uint32_t *reset)
{
    __shared__ uint64_t red[256];
    for (uint32_t k = 0; k < nstat; ++k) {
        const bool is_min = (min_mask >> k) & 1u;
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
    if (reset && threadIdx.x == 0) *reset = 0;     // the slow list of the launch before
}

hipError_t launch_stats_finalize(const uint64_t *partials, uint32_t nblk, uint32_t nstat,
                                 uint64_t *stats, uint64_t map, uint32_t min_mask, hipStream_t s, uint32_t *reset)
{
    hipLaunchKernelGGL(stats_finalize_kernel, dim3(1), dim3(256), 0, s, partials, nblk, nstat, stats, map,
                       min_mask, reset);
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

// The outputs the walk kernels and the tail's deferred walks write: the
// apus_commit_out_t fields up to last_idx_term, 96 B of kernel arguments.
// The failover outputs go to quorum_tail_kernel as arguments of their own,
// after these: with the whole 160-B apus_commit_out_t as one argument the
// tail reloaded its arguments (s_load_dwordx16) inside its group loop, and
// the C2 tail ran 28 us slower (profiles/r04/tail/).
struct WalkOut {
    uint64_t *new_commit;
    uint8_t *committed;
    uint32_t *n_entries;
    uint32_t *digest;
    uint64_t *median;
    uint64_t *new_head;
    uint8_t *append_head;
    uint64_t *min_apply;
    apus_entry_det_t *nc_dets;
    uint32_t *nc_len;
    uint32_t nc_max;
    uint32_t pad;
    uint64_t *last_idx_term;
};
static_assert(sizeof(WalkOut) == offsetof(apus_commit_out_t, vote), "WalkOut: apus_commit_out_t's head");
inline WalkOut walk_out(const apus_commit_out_t &o)
{
    WalkOut w;
    memcpy(&w, &o, sizeof w);
    return w;
}

template <bool CHECKSUM>
__device__ __forceinline__ void lane_group(const apus_batch_t &b, const WalkOut &o, uint64_t g,
                                        uint32_t *n_out, uint32_t *flags_out)
{
    const apus_group_state_t st = load_state(b, g);
    const uint64_t len = st.len, end = st.end, commit0 = st.commit;
    const uint32_t self = b.self_idx[g];
    const uint32_t size = walk_size(st.cid);
    const uint32_t need = size / 2 + 1;
    const uint8_t *ring = b.ring + g * b.ring_stride;
    const uint64_t guard = len / kHdr + 4;
    uint64_t m = commit0, steps = 0, stop = 0;
    uint32_t n = 0, ad = 1;
    bool committing = true, stopped = false;
    // commit or end beyond len: corrupt (oracle/apus_oracle.c); else m <= len throughout.
    // A len beyond the group's ring (ring_cap) is corrupt too: the walk never
    // reads past it (the next image's header, or past the batch)
    bool corrupt = commit0 > len || end > len || len > ring_cap(b);
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
    if (o.nc_dets && o.nc_len) {
        // APUS_COMMIT_NC: log_entries_to_nc_buf from commit (dare_log.h:339-359),
        // as nc_build_kernel walks it
        const RingView v = ring_view(b, g, st);
        apus_entry_det_t *d = o.nc_dets + g * o.nc_max;
        uint64_t q = commit0;
        uint32_t k = 0;
        while (k < o.nc_max && v.get_entry(q)) {
            const uint8_t *e = v.ring + q;
            apus_entry_det_t x;
            ld_idx_term(e, x.idx, x.term);
            x.offset = q;
            d[k++] = x;
            const uint32_t el = entry_len(e[kType], ld_u16(e + kData));
            if (v.len - q < el) q = 0;
            q += el;
        }
        o.nc_len[g] = k;
    }
    *n_out = n;
    *flags_out = (adv ? 1u : 0u) | (corrupt ? 2u : 0u);
}

// ---------------------------------------------------------------------------
// commit_wave_kernel
// ---------------------------------------------------------------------------
// One consensus group per wave, streamed through a per-wave LDS window.
//
// Virtual offsets.  The walk of a wrapped log runs [commit, gap0) then jumps
// to offset 0 (log_get_entry's header wrap, dare_log.h:327-330, or the
// ghost-header jump, dare_ibv_rc.c:1741-1744 via log_fit_entry).  The kernel
// walks an unwrapped view: ring offset r of the second segment sits at
// virtual offset V + r, V = align16(len).  A window is a 16-B aligned
// virtual range [ws, ws + kWin) whose pieces load from ring(v) =
// v < V ? v : v - V, so the wrap costs no extra window and a C2 batch
// (64 x 128 B) is ONE window per group.  Consecutive windows of a long walk
// overlap by 64 B (a header that starts in a window lies wholly in it or in
// the next).  The first window of the next group is prefetched (16-B buffer
// loads, nt, out-of-window pieces zeroed by the descriptor's range check)
// while the current group is walked.
//
// Walk: the APUS walk (dare_ibv_rc.c:1725-1758) is a chain -- the next
// entry starts where the current one ends.  Lane j reads the header at
// m + j*elen (elen = the last length seen); the chain is confirmed up to the
// first lane whose entry has another length or fails a walk condition (end
// reached, entry does not fit).  A ghost header found that way is jumped
// over without another step.
//
// Acks: each lane tests reply[0..size) of its entry (byte == 1 exactly, self
// always counts); the first confirmed entry without a majority stops the
// commit (ballot + ctz).
//
// Checksum (APUS_COMMIT_CHECKSUM): Adler-32 over the concatenated entry spans
// with bytes 27..47 zeroed (oracle/apus_oracle.c).  Every staged piece's byte
// sum and position-weighted sum are taken while it is written to LDS
// (v_dot4_u32_u8); after the walk, a window contributes the bytes from the
// last counted position to the walk frontier: the staged sums minus the
// bytes outside that range (lane-parallel range sums over LDS: the 64-B
// overlap, the bytes past the frontier, the wrap gap) minus bytes 27..47 of
// each confirmed entry (from its header registers).  Image positions are
// virtual offset - commit, less (V - gap0) past the jump.  Per-lane sums are
// exact 64-bit integers reduced mod 65521 once per group.
//
// Fast path: 16-B aligned ring, len < 2^28, ring_cap >= align16(len),
// commit/end within the ring.  Anything else, and any walk that leaves the
// window schedule (a malformed ring), is deferred to the exact one-lane walk
// (lane_group) after the main loop.
constexpr int kWin = 9216;         // window bytes: 64 x 128-B entries + alignment + slack
constexpr int kNP = kWin / 16;             // 16-B pieces per window
constexpr uint32_t kFastMaxLen = 1u << 28; // keeps every image sum inside 64 bits
constexpr uint32_t kOOB = 0xFFFFFFF0u;     // buffer offset past every range check
static_assert(kNP % 64 == 0, "whole pieces per lane");

// piece k of a window lives at LDS slot k + k/16: lanes reading 128-B or
// 64-B strided headers then hit 16 distinct 4-bank groups per ds_read_b128
__device__ __forceinline__ uint32_t pslot(uint32_t k) { return k + (k >> 4); }

// v_cndmask with a lane mask: LLVM turns select chains over an array into a
// dynamically indexed stack array (scratch); this keeps them in VGPRs
__device__ __forceinline__ uint32_t lsel(uint64_t lanes, uint32_t if_set, uint32_t if_clear)
{
    uint32_t r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(lanes));
    return r;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ring_rsrc(const uint8_t *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(p), (short)0, (int)bytes, 0x00020000);
}
// streaming 16-B load (nt: every log byte is read once per batch)
__device__ __forceinline__ uint4 ld_piece(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 2);
    return make_uint4(v.x, v.y, v.z, v.w);
}

// bytes [lo, hi) of a 4-byte word (0 <= lo <= hi <= 4)
__device__ __forceinline__ uint32_t byte_mask(int lo, int hi)
{
    const uint32_t up = hi >= 4 ? 0xFFFFFFFFu : ((1u << (8 * hi)) - 1u);
    const uint32_t dn = lo >= 4 ? 0xFFFFFFFFu : ((1u << (8 * lo)) - 1u);
    return up & ~dn;
}

// x mod 65521 with 2^16 = 15 (mod 65521): fold 16-bit limbs, no division
__device__ __forceinline__ uint32_t mod_adler64(uint64_t x)
{
    const uint32_t l0 = (uint32_t)x & 0xFFFFu, l1 = ((uint32_t)x >> 16), l2 = (uint32_t)(x >> 32) & 0xFFFFu,
                   l3 = (uint32_t)(x >> 48);
    uint32_t y = l0 + 15u * l1 + 225u * l2 + 3375u * l3;        // < 2^28
    y = (y & 0xFFFFu) + 15u * (y >> 16);                        // < 2^16 + 61440
    y = y >= kAdlerMod ? y - kAdlerMod : y;
    return y >= kAdlerMod ? y - kAdlerMod : y;
}
// a lane's exact sum held as a wrapped int64 -> its residue in [0, 65521)
__device__ __forceinline__ uint32_t mod_adler_signed(uint64_t x)
{
    const bool neg = (int64_t)x < 0;
    const uint32_t r = mod_adler64(neg ? 0ull - x : x);
    return neg && r ? kAdlerMod - r : r;
}

// wave-wide sum of per-lane residues (< 2^16: 64 of them fit 22 bits), uniform
// result: DPP row shifts (zero fill) leave each 16-lane row's sum in its
// lane 15, and the four rows are added in SGPRs
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_shr(uint32_t x)
{
    return __builtin_amdgcn_update_dpp(0u, x, CTRL, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t wave_sum_res(uint32_t x)
{
    x += dpp_shr<0x111>(x);   // row_shr:1
    x += dpp_shr<0x112>(x);   // row_shr:2
    x += dpp_shr<0x114>(x);   // row_shr:4
    x += dpp_shr<0x118>(x);   // row_shr:8
    return (uint32_t)__builtin_amdgcn_readlane(x, 15) + (uint32_t)__builtin_amdgcn_readlane(x, 31) +
           (uint32_t)__builtin_amdgcn_readlane(x, 47) + (uint32_t)__builtin_amdgcn_readlane(x, 63);
}

// walk flags (one scalar word)
constexpr uint32_t kDone = 1, kBail = 2, kForced = 4, kJumpReq = 8, kStopped = 16, kSeg1 = 32, kDrain = 64;
// APUS_COMMIT_NC: a ghost header was recorded as a determinant, so the entry
// the walk reads at 0 next is its copy and no determinant of its own
constexpr uint32_t kGhSkip = 128;
// commit_seg_kernel (APUS_COMMIT_LAST_IT): the wrap was a ghost-header jump
constexpr uint32_t kGhJump = 256;

// a pointer held in VGPRs (the compiler would otherwise keep it in SGPRs)
template <typename T>
__device__ __forceinline__ T *vptr(T *p)
{
    uint64_t x = (uint64_t)p;
    asm volatile("" : "+v"(x));
    return (T *)x;
}

// Groups are taken in blocks of 64 consecutive gids, one block per wave at a
// time (blocks grid-strided over the waves).  Lane i of a block holds group
// blk*64 + i's window-schedule fields, computed once per block in VALU from
// its state row (blk_t), and the group's results (slot registers) until the
// block epilogue computes the 64 digests in VALU and writes every output
// with coalesced stores.  Per group only v_readlane / v_writelane touch these.
constexpr uint32_t kPkWrapped = 1, kPkWindowed = 2, kPkFast = 4;
struct blk_raw_t {                 // the state-row dwords the schedule reads
    uint4 ce;                      // commit lo/hi, end lo/hi   (row bytes 16..31)
    uint2 ln;                      // len lo/hi                 (row bytes 40..47)
    uint32_t cw;                   // cid size[0], size[1], state (row bytes 56..59)
    uint32_t self;                 // config.idx
};
struct blk_t {
    uint32_t commit, end, len, vend;
    uint32_t pk;                   // size | self << 8 | need << 16 | kPk* << 24
};

// (a dare_log_t image keeps commit/end at the same offsets, len at 56 and the
// cid in b.cid: APUS_BATCH_LOG_IMAGE)
__device__ __forceinline__ blk_raw_t load_blk_raw(const apus_batch_t &b, uint64_t g, uint32_t G)
{
    const uint32_t gc = g < G ? (uint32_t)g : G - 1;
    blk_raw_t r;
    if (b.flags & APUS_BATCH_LOG_IMAGE) {
        const uint8_t *hdr = reinterpret_cast<const uint8_t *>(log_header(b, gc));
        r.ce = *reinterpret_cast<const uint4 *>(hdr + 16);
        r.ln = *reinterpret_cast<const uint2 *>(hdr + 56);
        r.cw = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(b.cid + gc) + 8);
    } else {
        const uint8_t *row = reinterpret_cast<const uint8_t *>(b.state + gc);
        r.ce = *reinterpret_cast<const uint4 *>(row + 16);
        r.ln = *reinterpret_cast<const uint2 *>(row + 40);
        r.cw = *reinterpret_cast<const uint32_t *>(row + 56);
    }
    r.self = b.self_idx[gc];
    return r;
}

// cap: ring_cap(b), the bytes of a group's ring the window loads may read
__device__ __forceinline__ blk_t blk_of(const blk_raw_t &r, uint32_t cap)
{
    const uint32_t len = r.ln.x, end = r.ce.z, commit = r.ce.x;
    const uint32_t hi = r.ce.y | r.ce.w | r.ln.y;
    const uint32_t V = (len + 15u) & ~15u;
    const bool wrapped = end < commit;
    const uint32_t vend = wrapped ? V + end : end;
    const uint32_t vend2 = (wrapped && end == 0) ? len : 0xFFFFFFFFu;   // ring offset len ~ 0 when end == 0
    const bool fast = (hi == 0) & (len < kFastMaxLen) & (cap >= V) & (commit <= len) & (end <= len);
    // dist(commit) == 0: nothing to walk
    const bool empty = (end == len) | (commit == vend) | (commit == vend2);
    const uint32_t state = (r.cw >> 16) & 0xFFu;
    const uint32_t size = state == APUS_CID_TRANSIT ? (r.cw >> 8) & 0xFFu : r.cw & 0xFFu;   // walk_size
    blk_t f;
    f.commit = commit;
    f.end = end;
    f.len = len;
    f.vend = vend;
    f.pk = size | (r.self << 8) | ((size / 2 + 1) << 16) |
           (((wrapped ? kPkWrapped : 0u) | ((fast & !empty) ? kPkWindowed : 0u) | (fast ? kPkFast : 0u)) << 24);
    return f;
}

// slot flags (lane i of sl_f): advanced, deferred to the slow path
constexpr uint32_t kSlAdv = 1, kSlBail = 2;

// WIN: window bytes.  kWin (9 KiB) holds a whole C2 batch; kWinShort (3 KiB,
// APUS_BATCH_SHORT_WALKS) needs a third of the LDS and of the prefetch
// registers, so twice the waves per SIMD hide the per-group latency chain of
// short batches (C5's 16 entries).  Results are the same for any window size.
constexpr int kWinShort = 3072;
// kWinHop (12 KiB, APUS_BATCH_VAR_LEN): the hop build walks a C3 group (about
// 137 KB) in many windows, and what each window costs besides its bytes (the
// wait, the staging sums, one lane-parallel pass over its few entries, the
// fold) is paid per window: 12-KiB windows at 3 waves per SIMD (LDS) walk C3
// 5-7% faster than 9-KiB ones at 4, and 16-KiB ones at 2 waves 4% faster
// (same rings, one process: profiles/r05/win/)
constexpr int kWinHop = 12288;
// HOP (APUS_BATCH_VAR_LEN): the walk may switch to following the chain hop by
// hop when speculation keeps failing (variable entry lengths, C3); the
// fixed-size build (C2) carries no hop code at all.
// EPI & kEpiNc: the walk also writes the NC determinants (a9) of [commit, end)
// from the headers it holds (APUS_COMMIT_NC).  (Running the median quorum
// and the pruning minimum inside this kernel was measured and dropped, DESIGN
// §3.1: in the block epilogue it cost what their own launches cost, as a tail
// pass after the walks it cost twice that.)
// DYN: blocks after each wave's first are handed out by an atomic counter
// (the stream's ticket word 1, reset by quorum_tail_kernel), two ids ahead, so
// waves on slower CUs take fewer of them.  Taken on checksum walks of >= 8
// blocks per wave: the C4 shard (32 per wave) 12.4 -> 11.1 ms; at C2 (4 per
// wave) there is nothing to even out and the counter costs 1-5%
// (profiles/r03/dyn/).
// groups per block of the wave kernel (experiment builds: 16 / 32)
constexpr uint32_t kWB = 64;
static_assert(kWB >= 1 && kWB <= 64, "a block is at most one group per lane");
template <bool CHECKSUM, int WIN, bool HOP, uint32_t EPI, bool DYN>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WIN == kWinShort ? (CHECKSUM ? 5 : 6) : WIN == kWinHop ? 3 : 4)))
commit_wave_kernel(const apus_batch_t b, const WalkOut o, uint64_t *partials, uint32_t *slow, uint32_t *ctr)
{
    constexpr int kWin = WIN;
    constexpr int kNP = kWin / 16;
    constexpr int kPPL = kNP / 64;
    // the speculation across a wrap (fixed-size build without NC determinants)
    constexpr bool XW = !HOP && !(EPI & kEpiNc);
    constexpr int kSlots = kNP + kNP / 16 + 4;
    static_assert(kNP % 64 == 0, "whole pieces per lane");
    __shared__ __attribute__((aligned(16))) uint4 s_win[kWaves][kSlots];

    const uint32_t lane = lane_id();
    const uint32_t lane16 = 16u * lane;
    const uint32_t wl = lane < kWB ? lane : kWB - 1u;   // the block's row this lane loads
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t *const slow_v = vptr(slow);
    uint4 *win = s_win[wv];
    // (an unpadded window for the hop build, a hop's three byte reads then
    // being one address with immediate offsets, measured slower: C3 6.03 ->
    // 6.16 ms, the lane pass's header reads conflict on LDS banks)
    const uint32_t *win32 = reinterpret_cast<const uint32_t *>(win);
    // statistics, per lane: decisions | advanced << 16, committed entries
    uint32_t acc_da = 0, acc_n = 0;
    uint32_t elen_g = 128;                // speculation stride, carried across groups
    bool hop = false;                     // walk mode, carried across groups: hop by hop (variable lengths)

    const uint32_t G = (uint32_t)b.n_groups;          // launch_commit: n_groups < 2^32
    const uint32_t nblk = (G + kWB - 1u) / kWB;
    const uint32_t wid = blockIdx.x * kWaves + wv, nw = gridDim.x * kWaves;
    const uint32_t cap = (uint32_t)ring_cap(b);       // <= ring_stride < 2^32 (launch_commit)

    // issue the loads of virtual window [ws, ws + kWin) of a group.  Virtual
    // offsets below V are ring offsets; from V on they are ring offset v - V
    // (the wrapped second segment).  Window bytes [0, nA) come from the first
    // segment, [nA, span) from the second; pieces past span (all of them when
    // !valid) read zero through the buffer range checks.  Whole rows of
    // pieces are addressed by descriptor (base = the segment's ring address
    // at window offset 0, offset = the lane's window offset), so only the one
    // row that straddles V computes per-lane ring offsets.  One code path, so
    // the prefetch registers are written in one place.
    auto load_window = [&](uint4 (&r)[kPPL], const uint8_t *ring, uint32_t ws, uint32_t vend, uint32_t V,
                           bool valid) {
        const uint32_t we_al = min(ws + (uint32_t)kWin, (vend + 15u) & ~15u);
        const uint32_t span = (valid && we_al > ws) ? we_al - ws : 0u;
        const uint32_t nA = ws < V ? min(V - ws, span) : 0u;
        const __amdgpu_buffer_rsrc_t rA = ring_rsrc(ring + ws, nA);
        const __amdgpu_buffer_rsrc_t rB = ring_rsrc((const uint8_t *)((uintptr_t)ring + ws - V), span);
        // The fixed-size build (C2: one window per group) keeps a load per
        // branch: the branch-free form below measured 1.5-2.5% slower there
        // (its selects cost more than the straddle wait, which the window's
        // walk hides), and 1.7% faster on the hop build (C3: several windows
        // per group; var walk 6.19 -> 6.09 ms, walk only 5.85 -> 5.65 ms,
        // profiles/r03/waveab/)
        if constexpr (!HOP) {
        // the straddle row's offsets computed before the first row's load, so
        // its branch writes no register a pending load may target (computed
        // in the branch, they cost a vmcnt(0) there: 0.3-0.6% at C2 in three
        // same-box rounds, profiles/r03/waveab/ab_c2_soearly.log)
        const uint32_t oS = lane16 + 1024u * uni(nA >> 10);
        uint32_t so = oS < nA ? ws + oS : (oS < span ? ws + oS - V : kOOB);
        asm volatile("" : "+v"(so));
#pragma unroll
        for (int j = 0; j < kPPL; ++j) {
            const uint32_t o = lane16 + 1024u * j;
            if (nA >= 1024u * (j + 1)) {
                r[j] = ld_piece(rA, o);
            } else if (nA <= 1024u * j) {
                r[j] = ld_piece(rB, o);
            } else {
                const __amdgpu_buffer_rsrc_t r0 = ring_rsrc(ring, valid ? cap : 0u);
                r[j] = ld_piece(r0, so);
            }
        }
        } else {
        // Rows below jS lie in the first segment, rows above it in the second;
        // row jS (which may straddle V) takes per-lane ring offsets, computed
        // before any load.  One load per row, descriptor and offset selected,
        // no branches: with a load per branch, the straddle row's offset was
        // computed in registers the other branch loads into, and the
        // write-after-write wait on them (vmcnt(0)) stalled the prefetch for a
        // memory round trip in every wrapped group's window.
        const uint32_t jS = uni(nA >> 10);
        const uint32_t oS = lane16 + 1024u * jS;
        const uint32_t so = oS < nA ? ws + oS : (oS < span ? ws + oS - V : kOOB);
        const __amdgpu_buffer_rsrc_t r0 = ring_rsrc(ring, valid ? cap : 0u);
#pragma unroll
        for (int j = 0; j < kPPL; ++j) {
            const __amdgpu_buffer_rsrc_t rj = (uint32_t)j < jS ? rA : ((uint32_t)j == jS ? r0 : rB);
            r[j] = ld_piece(rj, (uint32_t)j == jS ? so : lane16 + 1024u * j);
        }
        }
    };

    uint32_t blk = wid;
    blk_t F = {}, NF = {};
    blk_raw_t raw = {};
    uint32_t nb1 = 0, nb2v = 0;           // DYN: the next block, the one after it (lane 0, a block ahead)
    if (DYN) {
        if (lane == 0) nb1 = nw + atomicAdd(ctr, 1u);
        nb1 = __builtin_amdgcn_readfirstlane(nb1);
        if (lane == 0) nb2v = nw + atomicAdd(ctr, 1u);
    }
    auto next_blk = [&]() -> uint32_t { return DYN ? nb1 : blk + nw; };
    // nxt holds the first window of the next group to walk (zeros when it
    // has nothing to walk).  It is written at exactly two sites, here and the
    // window loop's prefetch, so it stays in one register set.
    uint4 nxt[kPPL];
    if (blk < nblk) {
        F = blk_of(load_blk_raw(b, blk * kWB + wl, G), cap);
        raw = load_blk_raw(b, (uint64_t)next_blk() * kWB + wl, G);
        const uint32_t c0 = __builtin_amdgcn_readlane(F.commit, 0), l0 = __builtin_amdgcn_readlane(F.len, 0);
        const uint32_t v0 = __builtin_amdgcn_readlane(F.vend, 0), p0 = __builtin_amdgcn_readlane(F.pk, 0);
        load_window(nxt, b.ring + (uint64_t)blk * kWB * b.ring_stride, c0 & ~15u, v0, (l0 + 15u) & ~15u,
                    ((p0 >> 24) & kPkWindowed) != 0);
    }

    while (blk < nblk) {
        // slot registers: lane i = group blk*64 + i
        uint32_t sl_c = 0, sl_f = 0, sl_n = 0, sl_s = 0, sl_t = 0, sl_len = 0, sl_nw = 0;
        const uint32_t g0 = blk * kWB;
        const uint32_t nin = min(kWB, G - g0);
        for (uint32_t i = 0; i < nin; ++i) {
            const uint32_t g = g0 + i;
            const uint32_t commit0 = __builtin_amdgcn_readlane(F.commit, i);
            const uint32_t end = __builtin_amdgcn_readlane(F.end, i);
            const uint32_t len = __builtin_amdgcn_readlane(F.len, i);
            const uint32_t vend = __builtin_amdgcn_readlane(F.vend, i);
            const uint32_t pk = __builtin_amdgcn_readlane(F.pk, i);
            const uint32_t pkf = pk >> 24;
            const uint32_t V = (len + 15u) & ~15u;
            const uint32_t vend2 = ((pkf & kPkWrapped) && end == 0) ? len : 0xFFFFFFFFu;
            const uint32_t lim1 = V + len;    // end of the second segment (virtual)
            const uint32_t size = pk & 0xFFu, self = (pk >> 8) & 0xFFu, need = (pk >> 16) & 0xFFu;
            const uint32_t size_mask = size >= 16 ? 0xFFFFu : ((1u << size) - 1u);
            const uint32_t self_bit = self < 16 ? (1u << self) : 0u;
            const uint8_t *ring = b.ring + (uint64_t)g * b.ring_stride;

            uint32_t m = commit0;
            // walk flags in one scalar (bools would each take a 64-bit lane mask)
            uint32_t fl = (!(pkf & kPkFast) ? kBail : 0u) | ((pkf & kPkWindowed) ? 0u : kDone);
            uint32_t stop = 0, n_commit = 0, gap0 = 0;
            uint32_t nwalk = 0, gh_len = 0;   // APUS_COMMIT_NC: determinants so far, the recorded ghost's length
            const uint32_t guard = len / kHdr + 4;
            uint32_t steps = 0;
            // checksum: per-lane exact image sums (wrap-around intermediates)
            uint64_t S = 0, T = 0;
            uint32_t cnt_lo = commit0;        // first virtual byte not yet counted
            uint32_t ws = commit0 & ~15u;

            // The window loop runs at least once per group: the iteration whose
            // schedule has no further window prefetches the next group's first
            // window.  A group that leaves early (nothing to walk, a bail, a walk-
            // only stop) spends one more iteration (kDrain) doing only that.
            for (;;) {
                const bool active = !(fl & kDrain) && (!(fl & kDone) || (CHECKSUM && cnt_lo < m));
                const uint32_t we = min(ws + (uint32_t)kWin, vend);
                const uint32_t we_al = min(ws + (uint32_t)kWin, (vend + 15u) & ~15u);
                const bool more = active && ws + (uint32_t)kWin < vend;   // the schedule has another window
                const bool straddle = ws < V && V < we_al;

                // ---- 1. stage the window; sums over every staged byte ----
                // piece k = lane + 64 j holds window bytes [16k, 16k + 16)
                uint32_t s_pos = 0, t_in = 0, r_pre = 0, s_hi = 0;
                if (active) {
                    uint4 *wl = win + lane + (lane >> 4);
                    if (!CHECKSUM || !straddle) {
#pragma unroll
                        for (int j = 0; j < kPPL; ++j) {
                            const uint4 v = nxt[j];
                            wl[68 * j] = v;
                            if (CHECKSUM) {
                                s_pos = udot4(v.w, 0x01010101u, udot4(v.z, 0x01010101u,
                                        udot4(v.y, 0x01010101u, udot4(v.x, 0x01010101u, s_pos))));
                                r_pre += s_pos;       // sum_j (prefix through j) = kPPL*S - sum_j j*s_j
                                t_in = udot4(v.w, 0x0F0E0D0Cu, udot4(v.z, 0x0B0A0908u,
                                       udot4(v.y, 0x07060504u, udot4(v.x, 0x03020100u, t_in))));
                            }
                        }
                        if (CHECKSUM && ws >= V) s_hi = s_pos;
                    } else {
                        // the window straddles V: s_hi = the bytes of the pieces past
                        // it (window offset >= V - ws), as all minus the prefix below
                        const uint32_t kVb = V - ws;
                        uint32_t s_lo = 0;
#pragma unroll
                        for (int j = 0; j < kPPL; ++j) {
                            const uint4 v = nxt[j];
                            wl[68 * j] = v;
                            s_pos = udot4(v.w, 0x01010101u, udot4(v.z, 0x01010101u,
                                    udot4(v.y, 0x01010101u, udot4(v.x, 0x01010101u, s_pos))));
                            r_pre += s_pos;
                            if (lane16 + 1024u * j < kVb) s_lo = s_pos;
                            t_in = udot4(v.w, 0x0F0E0D0Cu, udot4(v.z, 0x0B0A0908u,
                                   udot4(v.y, 0x07060504u, udot4(v.x, 0x03020100u, t_in))));
                        }
                        s_hi = s_pos - s_lo;
                    }
                }
                // the window is in LDS and summed before the next one is
                // requested: its registers are reused by the prefetch
                if (CHECKSUM) asm volatile("" : "+v"(s_pos), "+v"(t_in), "+v"(r_pre), "+v"(s_hi));
                asm volatile("" ::: "memory");

                // ---- 2. prefetch the next window of the schedule, or the next group's first ----
                {
                    const uint8_t *pring = ring;
                    uint32_t pws = ws + kWin - 64, pvend = vend, pV = V;
                    bool pvalid = true;
                    if (!more) {
                        // the next group of the block (lane i + 1 of F), or the
                        // first of the wave's next block (lane 0 of NF, whose
                        // fields are computed now from the rows loaded a block ago)
                        uint32_t nc, nl, nv, np;
                        uint64_t ng;
                        if (i + 1 < kWB) {
                            nc = __builtin_amdgcn_readlane(F.commit, i + 1);
                            nl = __builtin_amdgcn_readlane(F.len, i + 1);
                            nv = __builtin_amdgcn_readlane(F.vend, i + 1);
                            np = __builtin_amdgcn_readlane(F.pk, i + 1);
                            ng = g + 1;
                        } else {
                            NF = blk_of(raw, cap);
                            nc = __builtin_amdgcn_readlane(NF.commit, 0);
                            nl = __builtin_amdgcn_readlane(NF.len, 0);
                            nv = __builtin_amdgcn_readlane(NF.vend, 0);
                            np = __builtin_amdgcn_readlane(NF.pk, 0);
                            ng = (uint64_t)next_blk() * kWB;
                        }
                        pring = b.ring + (uint64_t)ng * b.ring_stride;
                        pws = nc & ~15u;
                        pvend = nv;
                        pV = (nl + 15u) & ~15u;
                        pvalid = ng < G && ((np >> 24) & kPkWindowed);
                    }
                    load_window(nxt, pring, pws, pvend, pV, pvalid);
                }
                if (!active) break;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

                // ---- 3. speculative walk over the headers of this window ----
                uint32_t exb = 0, exb1 = 0;   // per-lane sums of the zeroed bytes 27..47 (all / second segment)
                uint64_t exxb = 0;            // and their window-relative position-weighted sums
                while (!(fl & kDone)) {
                    if (!(fl & kForced) && (m == vend || m == vend2)) { fl |= kDone; break; }
                    const uint32_t lim = (fl & kSeg1) ? lim1 : len;
                    if ((fl & kJumpReq) || lim - m < kHdr) {
                        // log_get_entry's header wrap (forced: the entry at 0 is
                        // read unchecked) or the ghost-header jump: legal only
                        // from the first segment of a wrapped log
                        if (!(pkf & kPkWrapped) || (fl & kSeg1)) { fl |= kBail; break; }
                        fl = (fl & ~(kJumpReq | kForced)) | kSeg1 | ((fl & kJumpReq) ? 0u : kForced);
                        gap0 = m;
                        m = V;
                        if (++steps > guard) { fl |= kBail; break; }
                        continue;
                    }
                    if (m + kHdr > we) break;              // next window

                    // the votes of the confirmed lanes (lane < nconf, headers in ev)
                    // and the first entry without a majority; the zeroed bytes
                    // 27..47 of the confirmed entries into the checksum corrections
                    // s1: this lane's entry lies past the wrap (second segment)
                    auto tally = [&](const uint32_t (&ev)[7], bool conf, uint32_t nconf, uint32_t rel,
                                     bool s1) -> uint32_t {
                        uint32_t ef = nconf;
                        if (!(fl & kStopped)) {
                            uint32_t msk = eq1_nibble(ev[1]);
                            if (size > 4) msk |= eq1_nibble(ev[2]) << 4;
                            if (size > 8) msk |= (eq1_nibble(ev[3]) << 8) | (eq1_nibble(ev[4]) << 12);
                            msk = (msk | self_bit) & size_mask;
                            const uint64_t fbits = __ballot(conf & ((uint32_t)__builtin_popcount(msk) < need));
                            if (fbits) {
                                ef = (uint32_t)__builtin_ctzll(fbits);
                                fl |= kStopped;
                            }
                            n_commit += ef;
                        }
                        if (CHECKSUM) {
                            const uint32_t snd = ev[0] >> 24;          // byte 27
                            const uint32_t sb = udot4(ev[5], 0x01010101u, udot4(ev[4], 0x01010101u,
                                                udot4(ev[3], 0x01010101u, udot4(ev[2], 0x01010101u,
                                                udot4(ev[1], 0x01010101u, snd)))));
                            const uint32_t stb = udot4(ev[5], 0x2F2E2D2Cu, udot4(ev[4], 0x2B2A2928u,
                                                 udot4(ev[3], 0x27262524u, udot4(ev[2], 0x23222120u,
                                                 udot4(ev[1], 0x1F1E1D1Cu, 27u * snd)))));
                            const uint32_t csb = conf ? sb : 0u;
                            exb += csb;
                            if (s1) exb1 += csb;
                            exxb += (uint64_t)rel * csb + (conf ? stb : 0u);
                        }
                        return ef;     // < nconf: the stop entry
                    };
                    // 48 bytes of LDS from window byte 24 + rel, funnelled per lane
                    // to ev[i] = entry bytes [24 + 4i, 28 + 4i), any alignment
                    // APUS_COMMIT_NC: lane-local determinant (idx, term at window
                    // byte rel, ring offset) as log_entries_to_nc_buf records it
                    // (dare_log.h:346-350); every lane reads, `on` lanes store
                    auto put_det = [&](bool on, uint32_t k, uint32_t rel, uint32_t roff) {
                        const uint32_t k0 = rel >> 4;
                        const uint4 a = win[pslot(k0)], bq = win[pslot(k0 + 1)];
                        const uint32_t r[8] = { a.x, a.y, a.z, a.w, bq.x, bq.y, bq.z, bq.w };
                        const uint32_t qd = rel & 15u, qb = qd & 3u;
                        const uint64_t q1 = __ballot((qd & 4u) != 0), q2 = __ballot((qd & 8u) != 0);
                        uint32_t u[7], w[4];
#pragma unroll
                        for (int i2 = 0; i2 < 7; ++i2) u[i2] = __builtin_amdgcn_alignbyte(r[i2 + 1], r[i2], qb);
#pragma unroll
                        for (int i2 = 0; i2 < 4; ++i2)
                            w[i2] = lsel(q2, lsel(q1, u[i2 + 3], u[i2 + 2]), lsel(q1, u[i2 + 1], u[i2]));
                        if (on && k < o.nc_max) {
                            uint64_t *d = reinterpret_cast<uint64_t *>(o.nc_dets + (uint64_t)g * o.nc_max + k);
                            d[0] = ((uint64_t)w[1] << 32) | w[0];
                            d[1] = ((uint64_t)w[3] << 32) | w[2];
                            d[2] = roff;
                        }
                    };
                    auto header_any = [&](uint32_t rel, uint32_t (&ev)[7]) {
                        const uint32_t k0 = (rel + 24u) >> 4;
                        const uint4 a = win[pslot(k0)], bq = win[pslot(k0 + 1)], c = win[pslot(k0 + 2)];
                        const uint32_t r[12] = { a.x, a.y, a.z, a.w, bq.x, bq.y, bq.z, bq.w, c.x, c.y, c.z, c.w };
                        const uint32_t q = (rel + 24u) & 15u, qb = q & 3u;
                        const uint64_t q1 = __ballot((q & 4u) != 0), q2 = __ballot((q & 8u) != 0);
                        uint32_t u[11];
#pragma unroll
                        for (int i2 = 0; i2 < 11; ++i2) u[i2] = __builtin_amdgcn_alignbyte(r[i2 + 1], r[i2], qb);
#pragma unroll
                        for (int i2 = 0; i2 < 7; ++i2)
                            ev[i2] = lsel(q2, lsel(q1, u[i2 + 3], u[i2 + 2]), lsel(q1, u[i2 + 1], u[i2]));
                    };

                    if (HOP && hop) {
                        // Variable lengths: a speculative step would confirm one
                        // entry for a whole wave step.  Follow the chain from m one
                        // header per hop instead -- type@26 and cmd.len@48 as three
                        // uniform byte reads from LDS (window byte y lives at LDS
                        // byte y + 16*(y >> 8), pslot) -- recording entry j's offset
                        // in lane j; one lane-parallel pass then tallies and sums
                        // them all.  The chain stops where the speculative step
                        // stops: the next header leaves the window, the walk
                        // reaches end, or an entry does not fit (a ghost when its
                        // header does).
                        const uint8_t *win8 = reinterpret_cast<const uint8_t *>(win);
                        uint32_t q = m, p = m, nh = 0, gel = 0;
                        bool ghost = false;
                        for (;;) {
                            const uint32_t y = q - ws;
                            const uint32_t a0 = y + 26u, a1 = y + 48u, a2 = y + 49u;
                            const uint32_t t = win8[a0 + ((a0 >> 8) << 4)];
                            const uint32_t c0 = win8[a1 + ((a1 >> 8) << 4)];
                            const uint32_t c1 = win8[a2 + ((a2 >> 8) << 4)];
                            const uint32_t el = uni(bare_type(t) ? kHdr : kHdr + (c0 | (c1 << 8)));
                            if (q + el > lim) { ghost = q + kHdr <= lim; gel = el; break; }   // log_fit_entry
                            p = apus_writelane_i32(q, nh, p);
                            ++nh;
                            q += el;
                            // (q == end implies q + kHdr > we: the window ends at end)
                            if (nh == 64u || q + kHdr > we) break;
                        }
                        if (nh == 0) {                           // ghost header at m
                            if (EPI & kEpiNc) {
                                if (fl & kGhSkip) { fl |= kBail; break; }
                                put_det(lane == 0, nwalk, m - ws, (fl & kSeg1) ? m - V : m);
                                ++nwalk;
                                gh_len = gel;
                                fl |= kGhSkip;
                            }
                            fl |= kJumpReq;
                            continue;
                        }
                        const bool conf = lane < nh;
                        const uint32_t rel = (conf ? p : m) - ws;
                        uint32_t ev[7];
                        header_any(rel, ev);
                        const uint32_t ef = tally(ev, conf, nh, rel, (fl & kSeg1) != 0);
                        if (ef < nh) stop = __builtin_amdgcn_readlane(p, ef) - ((fl & kSeg1) ? V : 0u);   // ring offset
                        const uint32_t type = (ev[0] >> 16) & 0xFFu;
                        const uint32_t elen = bare_type(type) ? kHdr : kHdr + (ev[6] & 0xFFFFu);
                        if (EPI & kEpiNc) {
                            uint32_t lo = 0;
                            if (fl & kGhSkip) {
                                // lane 0 is the recorded ghost's copy at 0: no determinant
                                // of its own; a copy of another length would part the chains
                                if ((uint32_t)__builtin_amdgcn_readlane(elen, 0) != gh_len) { fl |= kBail; break; }
                                lo = 1;
                                fl &= ~kGhSkip;
                            }
                            const uint32_t sv = (fl & kSeg1) ? V : 0u;
                            put_det(conf && lane >= lo, nwalk + lane - lo, rel, p - sv);
                            nwalk += nh - lo;
                            if (ghost) {                          // the ghost header the hops stopped at
                                put_det(lane == 0, nwalk, q - ws, q - sv);
                                ++nwalk;
                                gh_len = gel;
                                fl |= kGhSkip;
                            }
                        }
                        elen_g = __builtin_amdgcn_readlane(elen, nh - 1);
                        // back to speculation once the chain's lengths repeat
                        if (nh >= 2u && __ballot(conf & (elen != elen_g)) == 0) hop = false;
                        m = q;
                        fl &= ~kForced;
                        steps += nh;
                        if (ghost) fl |= kJumpReq;
                    } else {
                        uint32_t p = m + lane * elen_g;
                        // XW: in a wrapped log's first segment the speculation runs on
                        // across the wrap (as in commit_seg_kernel): the jw lanes whose
                        // entries end by len, then at q the ghost header (its header
                        // fits; lane jw checks it) or a header wrap (the entry at 0 is
                        // read unchecked), then the entries at V, V + elen, ...  A
                        // wrapped C2 batch is then one step, not two.
                        bool xw = false, crossed = false, fz = false;
                        uint32_t q = 0;
                        if (XW && (pkf & kPkWrapped) && !(fl & kSeg1)) {
                            const uint32_t jw = (uint32_t)__builtin_popcountll(__ballot(m + (lane + 1u) * elen_g <= len));
                            q = m + jw * elen_g;
                            const bool gcase = q + kHdr <= len;         // a ghost header at q, else a header wrap
                            xw = jw < 64u && (!gcase || q + kData + 2u <= we);
                            if (xw && gcase) {
                                // the ghost must not fit: its type@26 and cmd.len@48 from LDS
                                const uint8_t *win8 = reinterpret_cast<const uint8_t *>(win);
                                const uint32_t y = q - ws, a0 = y + 26u, a1 = y + 48u, a2 = y + 49u;
                                const uint32_t t = win8[a0 + ((a0 >> 8) << 4)];
                                const uint32_t c0 = win8[a1 + ((a1 >> 8) << 4)], c1 = win8[a2 + ((a2 >> 8) << 4)];
                                xw = q + uni(bare_type(t) ? kHdr : kHdr + (c0 | (c1 << 8))) > len;
                            }
                            if (xw) {
                                crossed = lane >= jw;
                                if (crossed) p = V + (lane - jw) * elen_g;
                                fz = !gcase && lane == jw;
                            }
                        }
                        const bool inw = (lane == 0 && !crossed) | (p + kHdr <= we);
                        // lanes past the window read entry 0's header (results dropped)
                        const uint32_t rel = (inw ? p : m) - ws;
                        uint32_t ev[7];          // ev[i] = entry bytes [24 + 4i, 28 + 4i)
                        // (past the wrap every header sits at 0 mod 16: one shift only if m does)
                        if ((elen_g & 15u) == 0 && (!xw || (m & 15u) == 0)) {
                            // every lane's header sits at the same offset mod 16 (p = m
                            // + lane*elen_g): one funnel per dword, no lane selects
                            const uint32_t k0 = (rel + 24u) >> 4;
                            const uint4 a = win[pslot(k0)], bq = win[pslot(k0 + 1)], c = win[pslot(k0 + 2)];
                            const uint32_t r[12] = { a.x, a.y, a.z, a.w, bq.x, bq.y, bq.z, bq.w, c.x, c.y, c.z, c.w };
                            const uint32_t q = uni((m - ws + 24u) & 15u), qb = q & 3u;
                            switch (q >> 2) {
                            case 0:
#pragma unroll
                                for (int i2 = 0; i2 < 7; ++i2) ev[i2] = __builtin_amdgcn_alignbyte(r[i2 + 1], r[i2], qb);
                                break;
                            case 1:
#pragma unroll
                                for (int i2 = 0; i2 < 7; ++i2) ev[i2] = __builtin_amdgcn_alignbyte(r[i2 + 2], r[i2 + 1], qb);
                                break;
                            case 2:
#pragma unroll
                                for (int i2 = 0; i2 < 7; ++i2) ev[i2] = __builtin_amdgcn_alignbyte(r[i2 + 3], r[i2 + 2], qb);
                                break;
                            default:
#pragma unroll
                                for (int i2 = 0; i2 < 7; ++i2) ev[i2] = __builtin_amdgcn_alignbyte(r[i2 + 4], r[i2 + 3], qb);
                                break;
                            }
                        } else {
                            header_any(rel, ev);
                        }
                        const uint32_t type = (ev[0] >> 16) & 0xFFu;    // byte 26
                        const uint32_t clen = ev[6] & 0xFFFFu;          // bytes 48..49
                        const uint32_t elen = bare_type(type) ? kHdr : kHdr + clen;
                        const bool live = inw & ((lane == 0 && !crossed) | fz | (p != vend));
                        const uint32_t liml = xw ? (p >= V ? lim1 : len) : lim;
                        const bool fit = p + elen <= liml;              // log_fit_entry
                        const bool ok = live & fit;
                        const bool cont = ok & (elen == elen_g) & (lane < 63);
                        const uint64_t okb = __ballot(ok);
                        // a ghost header (header fits, entry does not) ends the chain
                        const uint64_t ghb = __ballot(live & !fit & (p + kHdr <= liml));
                        const uint32_t fb = (uint32_t)__builtin_ctzll(__ballot(!cont));
                        const uint32_t nconf = fb + (uint32_t)((okb >> fb) & 1ull);
                        if (nconf == 0) {                                // ghost header at m
                            if (EPI & kEpiNc) {
                                if (fl & kGhSkip) { fl |= kBail; break; }
                                put_det(lane == 0, nwalk, rel, (fl & kSeg1) ? m - V : m);
                                ++nwalk;
                                gh_len = (uint32_t)__builtin_amdgcn_readlane(elen, 0);
                                fl |= kGhSkip;
                            }
                            fl |= kJumpReq;
                            continue;
                        }
                        const uint32_t ef = tally(ev, lane < nconf, nconf, rel, p >= V);
                        if (ef < nconf) {
                            const uint32_t pv = __builtin_amdgcn_readlane(p, ef);
                            stop = pv >= V ? pv - V : pv;                // ring offset
                        }
                        if (EPI & kEpiNc) {
                            uint32_t lo = 0;
                            if (fl & kGhSkip) {                          // see the hop pass
                                if ((uint32_t)__builtin_amdgcn_readlane(elen, 0) != gh_len) { fl |= kBail; break; }
                                lo = 1;
                                fl &= ~kGhSkip;
                            }
                            // the confirmed entries, and a ghost header right after them
                            const bool gh_next = nconf <= fb && ((ghb >> fb) & 1ull);
                            const uint32_t sv = (fl & kSeg1) ? V : 0u;
                            put_det((lane >= lo && lane < nconf) || (gh_next && lane == fb), nwalk + lane - lo, rel,
                                    p - sv);
                            nwalk += nconf - lo;
                            if (gh_next) {
                                ++nwalk;
                                gh_len = (uint32_t)__builtin_amdgcn_readlane(elen, fb);
                                fl |= kGhSkip;
                            }
                        }
                        const uint32_t elen_last = __builtin_amdgcn_readlane(elen, nconf - 1);
                        const uint32_t p_last = __builtin_amdgcn_readlane(p, nconf - 1);
                        if (xw && p_last >= V) {                        // crossed the wrap
                            fl |= kSeg1;
                            gap0 = q;
                            ++steps;
                        }
                        m = p_last + elen_last;
                        elen_g = elen_last;
                        fl &= ~kForced;
                        steps += nconf;
                        if (nconf <= fb && ((ghb >> fb) & 1ull)) fl |= kJumpReq;   // ghost right after the chain
                        // the chain broke on another length after a short run: hop
                        if (HOP && nconf < 8u && nconf > fb) hop = true;
                    }
                    if (steps > guard) { fl |= kBail; break; }  // corrupt ring: the slow path decides
                    if (!CHECKSUM && (fl & kStopped)) { fl |= kDone; break; }
                }
                if (fl & kBail) {
                    if (more) { fl |= kDrain; continue; }
                    break;
                }

                // ---- 4. checksum: this window's counted bytes [cnt_lo, hi) less the gap ----
                if (CHECKSUM) {
                    const uint32_t hi = min(m, we);
                    uint32_t s_neg = exb, sh_neg = exb1, t_neg = 0;
                    const uint32_t vrel = V > ws ? V - ws : 0u;
                    // window-relative byte range [lo, hi) of LDS, 4 B per lane per round
                    auto sub_range = [&](uint32_t lo, uint32_t hi_r) {
                        for (uint32_t base = lo & ~3u; base < hi_r; base += 256u) {
                            const uint32_t x0 = base + 4u * lane;
                            const uint32_t xc = x0 < hi_r ? x0 : base;          // stay inside the window
                            uint32_t x = win32[4u * pslot(xc >> 4) + ((xc >> 2) & 3u)];
                            const int blo = (int)lo - (int)x0, bhi = (int)hi_r - (int)x0;
                            x &= byte_mask(blo < 0 ? 0 : blo > 4 ? 4 : blo, bhi < 0 ? 0 : bhi > 4 ? 4 : bhi);
                            const uint32_t s0 = byte_sum(x);
                            s_neg += s0;
                            if (x0 >= vrel) sh_neg += s0;
                            t_neg += udot4(x, 0x03020100u, x0 * s0);
                        }
                    };
                    if (cnt_lo > ws) sub_range(0u, cnt_lo - ws);
                    if (we_al > hi) sub_range(hi - ws, we_al - ws);
                    if (fl & kSeg1) {
                        const uint32_t glo = max(gap0, cnt_lo), ghi = min(V, hi);
                        if (glo < ghi) sub_range(glo - ws, ghi - ws);
                    }
                    // staged sums: t = sum (16 k + i) b, k = lane + 64 j
                    const uint32_t t_pos = t_in + lane16 * s_pos + 1024u * ((uint32_t)kPPL * s_pos - r_pre);
                    const int64_t s_cnt = (int64_t)(int32_t)(s_pos - s_neg);
                    const int64_t s1_cnt = (int64_t)(int32_t)(s_hi - sh_neg);
                    const int64_t t_cnt = (int64_t)(int32_t)(t_pos - t_neg) - (int64_t)exxb;
                    S += (uint64_t)s_cnt;
                    T += (uint64_t)(t_cnt + (int64_t)((int32_t)(ws - commit0)) * s_cnt -
                                    (int64_t)(V - gap0) * s1_cnt);
                    cnt_lo = hi;
                }
                if ((fl & kDone) && (!CHECKSUM || cnt_lo >= m)) {
                    if (more) { fl |= kDrain; continue; }
                    break;
                }
                if (!more) { fl |= kBail; break; }          // the walk leaves the schedule
                ws += kWin - 64;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }

            if ((EPI & kEpiNc) && (fl & kGhSkip)) fl |= kBail;       // the walk ended on a recorded ghost
            if (fl & kBail) {
                // deferred to quorum_tail_kernel (the exact one-lane walk)
                if (lane == 0) slow_v[1 + atomicAdd(slow_v, 1u)] = g;
                sl_f = apus_writelane_i32(kSlBail, i, sl_f);
            } else {
                const uint32_t res = (fl & kStopped) ? stop : ((fl & kSeg1) ? m - V : m);
                const bool adv = dist32(end, len, res) < dist32(end, len, commit0);
                sl_c = apus_writelane_i32(adv ? res : commit0, i, sl_c);
                sl_f = apus_writelane_i32(adv ? kSlAdv : 0u, i, sl_f);
                sl_n = apus_writelane_i32(n_commit, i, sl_n);
                if (EPI & kEpiNc) sl_nw = apus_writelane_i32(nwalk, i, sl_nw);
                if (CHECKSUM) {
                    // image length: the entries tile [commit, gap0) ++ [V, m), or [commit, m);
                    // the residue sums (< 2^22) are reduced mod 65521 in the block epilogue
                    sl_len = apus_writelane_i32((fl & kSeg1) ? (gap0 - commit0) + (m - V) : m - commit0,
                                                        i, sl_len);
                    sl_s = apus_writelane_i32(wave_sum_res(mod_adler_signed(S)), i, sl_s);
                    sl_t = apus_writelane_i32(wave_sum_res(mod_adler_signed(T)), i, sl_t);
                }
            }
        }

        // ---- block epilogue: lane i writes group blk*64 + i (coalesced) ----
        {
            const uint32_t g = g0 + lane;
            const bool okg = lane < nin && !(sl_f & kSlBail);
            // a deferred group's commit reads ~0 until the tail walks it (the
            // mark the publish / force tail looks for; real offsets are < 2^32)
            if (lane < nin && (sl_f & kSlBail) && o.new_commit) o.new_commit[g] = ~0ull;
            if (okg) {
                if (o.new_commit) o.new_commit[g] = (uint64_t)sl_c;
                if (o.committed) o.committed[g] = (uint8_t)(sl_f & kSlAdv);
                if (o.n_entries) o.n_entries[g] = sl_n;
                if (EPI & kEpiNc) o.nc_len[g] = sl_nw < o.nc_max ? sl_nw : o.nc_max;
                if (CHECKSUM && o.digest) {
                    const uint32_t Sa = mod_adler64(sl_s), Ta = mod_adler64(sl_t), Nm = mod_adler64(sl_len);
                    const uint32_t A = mod_adler64(1u + Sa);
                    const uint32_t B = mod_adler64((uint64_t)Nm * Sa + Nm + kAdlerMod - Ta);
                    o.digest[g] = (B << 16) | A;
                }
                acc_da += 1u | ((sl_f & kSlAdv) << 16);
                acc_n += sl_n;
            }
        }
        F = NF;
        if (DYN) {
            blk = nb1;
            nb1 = __builtin_amdgcn_readfirstlane(nb2v);
            raw = load_blk_raw(b, (uint64_t)nb1 * kWB + wl, G);
            if (lane == 0) nb2v = nw + atomicAdd(ctr, 1u);
        } else {
            raw = load_blk_raw(b, ((uint64_t)blk + 2u * nw) * kWB + wl, G);
            blk += nw;
        }
    }

    uint64_t mine[kWaveStats] = { acc_da & 0xFFFFu, acc_n, acc_da >> 16 };
    block_partials<kWaveStats>(vptr(partials), mine);
}

// ---------------------------------------------------------------------------
// commit_seg_kernel: short walks (APUS_BATCH_SHORT_WALKS), FOUR groups per
// wave, one per 16-lane segment.  A group's whole walk span [commit, end)
// (virtual offsets, as above) must fit one 2,304-B segment window (16 lanes x
// 9 pieces of 16 B: 16 entries of 128 B at any 16-B phase); a group whose
// walk leaves the window, and every group off the fast path, is deferred to
// quorum_tail_kernel.  Per wave step the four segments run the walk of
// commit_wave_kernel side by side: lane s of a segment reads the header at
// m + s*elen, the segment's 16 ballot bits confirm the chain and find the
// first entry without a majority.  Every segment value (walk offset, flags,
// stop, counts) lives in a VGPR that is uniform across its 16 lanes, so the
// per-group scalar bookkeeping of the wave kernel is paid once per four
// groups.  Checksum: staged byte / position sums of every loaded piece
// (v_dot4), less the bytes outside the image ([window start, commit), the
// wrap gap [gap0, V), [frontier, window end)) and bytes 27..47 of each
// confirmed entry; a window of 2,304 B keeps every sum below 2^32, so the
// Adler (A, B) come from exact 32-bit integers reduced once per group.
// ---------------------------------------------------------------------------
constexpr uint32_t kSegL = 16;                          // lanes per segment
constexpr uint32_t kNSeg = 64 / kSegL;                  // groups per wave
constexpr uint32_t kSegPPL = 9;                         // pieces per lane
constexpr uint32_t kSegWin = kSegL * 16 * kSegPPL;      // 2,304 window bytes
static_assert(kSegWin / 64u < 256u, "a segment's entry count fits 8 bits (LIT slot packing)");
constexpr uint32_t kSegSlots = kSegL * kSegPPL + kSegPPL;       // 144 pieces + 1 pad per 16 (the last read ends at 151)
constexpr uint32_t kSegMaxStride = 1u << 29;            // 4 rings per descriptor stay below 2^31

// LIT (APUS_COMMIT_LAST_IT, checksum walks): each group's row of
// o.last_idx_term receives the ring offset of the last NC determinant of its
// walk (the last entry, or the ghost header whose copy at 0 it is), or ~0 when
// the tail must walk (nothing walked, deferred, a ghost whose copy differs in
// length); quorum_tail_kernel replaces it with that header's (idx, term).
// DYN: blocks handed out by an atomic counter, as in commit_wave_kernel
// (checksum builds at 3 waves per SIMD: 149-152 VGPRs and no spills; at 4 they
// spilled 4-11 VGPRs, and walked the same rings 2-5% slower: profiles/r05/seg3/)
template <bool CHECKSUM, bool LIT, bool DYN>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CHECKSUM ? 3 : 4)))
commit_seg_kernel(const apus_batch_t b, const WalkOut o, uint64_t *partials, uint32_t *slow,
                  uint32_t *ctr)
{
    __shared__ __attribute__((aligned(16))) uint4 s_win[kWaves][kNSeg][kSegSlots];

    const uint32_t lane = lane_id();
    const uint32_t seg = lane >> 4, sl = lane & 15u, sh = 16u * seg;
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t *const slow_v = vptr(slow);
    uint4 *win = s_win[wv][seg];
    // statistics, wave-uniform (SGPRs): per-lane accumulators were spilled,
    // and their scratch reloads waited for every memory operation in flight
    uint32_t acc_dec = 0, acc_adv = 0, acc_ent = 0;
    uint32_t elen_g = 128;                // the segment's speculation stride, carried across groups

    const uint32_t G = (uint32_t)b.n_groups;
    const uint32_t nq = (G + kNSeg - 1) / kNSeg;
    const uint32_t wid = blockIdx.x * kWaves + wv, nw = gridDim.x * kWaves;
    const uint32_t stride = (uint32_t)b.ring_stride;
    const uint32_t cap = (uint32_t)ring_cap(b);       // <= stride < 2^32 (launch_commit)

    // pieces of quad q's windows: segment s loads group 4q + s's span; one
    // descriptor for the quad's four rings, pieces past a span (all of them
    // for a group with nothing to walk) read zero through the range check
    auto load_window = [&](uint4 (&r)[kSegPPL], uint32_t q, const blk_t &f) {
        // q is wave-uniform; said explicitly (readfirstlane), or the compiler
        // builds the descriptor in VGPRs and wraps every load in a waterfall
        // loop (9 per quad: ~55 VALU + 45 SALU)
        const uint32_t qu = uni(q);
        const uint32_t g0 = qu * kNSeg;
        const uint32_t ng = qu < nq ? min(kNSeg, G - g0) : 0u;
        const __amdgpu_buffer_rsrc_t rs =
            ring_rsrc((const uint8_t *)uni64((uint64_t)(b.ring + (uint64_t)g0 * b.ring_stride)),
                      uni(ng ? (ng - 1u) * stride + cap : 0u));
        const bool valid = seg < ng && ((f.pk >> 24) & kPkWindowed);
        const uint32_t V = (f.len + 15u) & ~15u, ws = f.commit & ~15u;
        const uint32_t we_al = min(ws + kSegWin, (f.vend + 15u) & ~15u);
        // (piece offsets in the SGPR offset field, two compares and two
        // selects per piece, measured no faster: the kernel moves 1.10x its
        // algorithmic bytes at 5.9 TB/s, HBM-bound, not issue-bound)
        const uint32_t base = seg * stride;
#pragma unroll
        for (int j = 0; j < (int)kSegPPL; ++j) {
            const uint32_t v = ws + 16u * sl + 256u * j;
            r[j] = ld_piece(rs, (valid && v < we_al) ? base + (v < V ? v : v - V) : kOOB);
        }
    };

    // Groups are taken in blocks of 64 (16 quads), one block per wave at a
    // time, as in commit_wave_kernel: lane i loads group blk*64 + i's state
    // row once per block (coalesced, a block ahead), each quad's segments
    // take their fields from it (shfl), and the 64 results wait in slot
    // registers for one coalesced store per output in the block epilogue.
    // (Four stores per quad made every next quad's wait on its window wait
    // for them as well: 8% of the kernel at the C4 1-GPU shape.)
    const uint32_t nblk = (G + 63u) >> 6;
    uint32_t blk = wid;
    blk_t FB = {}, F = {};
    blk_raw_t rawB = {};
    uint4 nxt[kSegPPL];
    // segment s's group in quad qi of a block: lane 4 qi + s of the block's fields
    auto seg_f = [&](const blk_t &x, uint32_t qi) -> blk_t {
        const int src = (int)(4u * qi + seg);
        blk_t r;
        r.commit = (uint32_t)__shfl((int)x.commit, src);
        r.end = (uint32_t)__shfl((int)x.end, src);
        r.len = (uint32_t)__shfl((int)x.len, src);
        r.vend = (uint32_t)__shfl((int)x.vend, src);
        r.pk = (uint32_t)__shfl((int)x.pk, src);
        return r;
    };
    // DYN: nb1 the next block; the one after it is requested in each block's
    // last quad (nb2v, lane 0) and read at the block's end (held across the
    // whole block it was spilled, and the spill waited for the atomic)
    uint32_t nb1 = 0, nb2v = 0;
    if (DYN) {
        if (lane == 0) nb1 = nw + atomicAdd(ctr, 1u);
        nb1 = __builtin_amdgcn_readfirstlane(nb1);
    }
    auto next_blk = [&]() -> uint32_t { return DYN ? nb1 : blk + nw; };
    if (blk < nblk) {
        FB = blk_of(load_blk_raw(b, (uint64_t)blk * 64u + lane, G), cap);
        rawB = load_blk_raw(b, (uint64_t)next_blk() * 64u + lane, G);
        F = seg_f(FB, 0);
        load_window(nxt, blk * 16u, F);
    }

    while (blk < nblk) {
    // slot registers: lane i = group blk*64 + i (new commit, flags, entries, digest)
    // (entries in the low 24 bits, the kSl* flags above: one register, so the
    // LIT build's extra slot fits without a spill in the block loop)
    // (LIT: the entries in bits 0..7 -- at most kSegWin / kHdr per group --
    // the term in bits 8..23, the index in sl_li: no register more than the
    // other builds, which spilled in the quad loop)
    uint32_t sl_c = 0, sl_nf = 0, sl_d = 0, sl_li = ~0u;
    const uint32_t g0b = blk * 64u;
    const uint32_t nin = min(64u, G - g0b);
    const uint32_t nqb = (nin + 3u) >> 2;
    for (uint32_t qi = 0; qi < nqb; ++qi) {
        const uint32_t q = blk * 16u + qi;
        const uint32_t g = q * kNSeg + seg;
        const uint32_t commit0 = F.commit, end = F.end, len = F.len, vend = F.vend, pk = F.pk;
        const uint32_t pkf = pk >> 24;
        const uint32_t V = (len + 15u) & ~15u;
        const uint32_t vend2 = ((pkf & kPkWrapped) && end == 0) ? len : 0xFFFFFFFFu;
        const uint32_t lim1 = V + len;
        const uint32_t size = pk & 0xFFu, self = (pk >> 8) & 0xFFu, need = (pk >> 16) & 0xFFu;
        const uint32_t size_mask = size >= 16 ? 0xFFFFu : ((1u << size) - 1u);
        const uint32_t self_bit = self < 16 ? (1u << self) : 0u;
        const uint32_t ws = commit0 & ~15u;
        const uint32_t we = min(ws + kSegWin, vend);
        const uint32_t we_al = min(ws + kSegWin, (vend + 15u) & ~15u);

        // ---- 1. stage the four windows; sums over every staged byte ----
        // piece k = sl + 16 j of a segment holds window bytes [16k, 16k + 16)
        uint32_t s_pos = 0, t_in = 0, r_pre = 0, s_lo = 0;
        {
            uint4 *wl = win + sl;
#pragma unroll
            for (int j = 0; j < (int)kSegPPL; ++j) {
                const uint4 v = nxt[j];
                wl[17 * j] = v;
                if (CHECKSUM) {
                    s_pos = udot4(v.w, 0x01010101u, udot4(v.z, 0x01010101u,
                            udot4(v.y, 0x01010101u, udot4(v.x, 0x01010101u, s_pos))));
                    r_pre += s_pos;       // sum_j (prefix through j) = kSegPPL*S - sum_j j*s_j
                    if (ws + 16u * sl + 256u * j < V) s_lo = s_pos;   // bytes of the first segment
                    t_in = udot4(v.w, 0x0F0E0D0Cu, udot4(v.z, 0x0B0A0908u,
                           udot4(v.y, 0x07060504u, udot4(v.x, 0x03020100u, t_in))));
                }
            }
        }
        if (CHECKSUM) asm volatile("" : "+v"(s_pos), "+v"(t_in), "+v"(r_pre), "+v"(s_lo));
        asm volatile("" ::: "memory");

        // ---- 2. the next quad's windows (the next block's rows came a block ago) ----
        const bool last_q = qi + 1u >= nqb;
        if (DYN && last_q && lane == 0) nb2v = nw + atomicAdd(ctr, 1u);
        const blk_t NF = last_q ? seg_f(blk_of(rawB, cap), 0) : seg_f(FB, qi + 1u);
        load_window(nxt, last_q ? next_blk() * 16u : q + 1u, NF);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        // ---- 3. the four walks, side by side ----
        // the checksum needs every byte of the span in the window: the last
        // entry's header may lie inside it and its data past it
        const bool off_path = !(pkf & kPkFast) || (CHECKSUM && ((vend + 15u) & ~15u) - ws > kSegWin);
        uint32_t fl = g >= G ? kDone : ((off_path ? kBail : 0u) | ((pkf & kPkWindowed) ? 0u : kDone));
        uint32_t m = commit0, stop = 0, n_commit = 0, gap0 = V, steps = 0;
        uint32_t lp = ~0u;                        // LIT: the last confirmed entry (virtual offset)
        const uint32_t guard = len / kHdr + 4;
        uint32_t exb = 0, exb1 = 0, exxb = 0;     // bytes 27..47 of confirmed entries (all / past V), weighted
        // (testing the end after each step instead, and not before the first,
        // measured slower: 1.79-1.99 vs 1.67 ms, spills in the quad loop)
        for (;;) {
            bool act = !(fl & (kDone | kBail));
            if (act && !(fl & kForced) && (m == vend || m == vend2)) { fl |= kDone; act = false; }
            if (__ballot(act) == 0) break;
            if (act && ((fl & kJumpReq) || ((fl & kSeg1) ? lim1 : len) - m < kHdr)) {
                // header wrap / ghost jump (see commit_wave_kernel), then the
                // walk goes on at V in this same step: the four segments move
                // in lock-step, so a step spent on the jump alone would cost
                // the whole wave a step (most C4-shaped groups wrap once)
                if (!(pkf & kPkWrapped) || (fl & kSeg1)) {
                    fl |= kBail;
                    act = false;
                } else {
                    const bool forced = !(fl & kJumpReq);    // log_get_entry's wrap reads the entry at 0 unchecked
                    fl = (fl & ~(kJumpReq | kForced)) | kSeg1 | (forced ? kForced : kGhJump);
                    gap0 = m;
                    m = V;
                    if (++steps > guard) { fl |= kBail; act = false; }
                    // a ghost jump lands at 0 as a new loop turn would: end there stops the walk
                    else if (!forced && (m == vend || m == vend2)) { fl |= kDone; act = false; }
                }
            }
            if (act && m + kHdr > we) { fl |= kBail; act = false; }   // the walk leaves the window

            // Lane sl speculates that the chain's entries all have the last
            // length seen.  In a wrapped log's first segment the speculation
            // runs on across the wrap: the jw lanes whose entries end by len
            // read [m, q), q = m + jw*elen; the entry at q cannot fit, so q
            // holds a ghost header (its header fits; its type and cmd.len are
            // read as three LDS bytes to confirm that the entry does not) or
            // the header itself does not fit (the entry at 0 is then read
            // unchecked, log_get_entry's wrap); lanes jw.. read V, V + elen, ...
            // (virtual V = ring offset 0).  A 16-entry batch that wraps is then
            // one step, not two or three.
            const bool xw = act && (pkf & kPkWrapped) && !(fl & kSeg1);
            const uint32_t jw =
                (uint32_t)__builtin_popcount((uint32_t)(__ballot(xw && m + (sl + 1u) * elen_g <= len) >> sh) &
                                             0xFFFFu);
            const uint32_t q = m + jw * elen_g;                     // the wrap point (xw)
            const bool gcase = q + kHdr <= len;                     // a ghost header at q, else a header wrap
            bool xok = xw && jw < 16u && (!gcase || q + kData + 2u <= we);
            if (__ballot(xok && gcase)) {
                // the ghost's type@26 and cmd.len@48 (window byte y at LDS byte y + 16*(y >> 8))
                const uint8_t *win8 = reinterpret_cast<const uint8_t *>(win);
                const uint32_t y = (xok && gcase) ? q - ws : 0u;
                const uint32_t a0 = y + 26u, a1 = y + 48u, a2 = y + 49u;
                const uint32_t t = win8[a0 + ((a0 >> 8) << 4)];
                const uint32_t c0 = win8[a1 + ((a1 >> 8) << 4)], c1 = win8[a2 + ((a2 >> 8) << 4)];
                if (gcase) xok = xok && q + (bare_type(t) ? kHdr : kHdr + (c0 | (c1 << 8))) > len;   // !log_fit_entry
            }
            const bool crossed = xok && sl >= jw;
            uint32_t p = crossed ? V + (sl - jw) * elen_g : m + sl * elen_g;
            const bool fz = crossed && !gcase && sl == jw;          // the entry at 0 after a header wrap
            const bool inw = (sl == 0 && !crossed) | (p + kHdr <= we);
            const uint32_t rel = act ? (inw ? p : m) - ws : 0u;
            const uint32_t k0 = (rel + 24u) >> 4;
            const uint4 a = win[pslot(k0)], bq = win[pslot(k0 + 1)], c = win[pslot(k0 + 2)];
            const uint32_t r[12] = { a.x, a.y, a.z, a.w, bq.x, bq.y, bq.z, bq.w, c.x, c.y, c.z, c.w };
            uint32_t ev[7];          // ev[i] = entry bytes [24 + 4i, 28 + 4i)
            {
                const uint32_t qq = (rel + 24u) & 15u, qb = qq & 3u;
                const uint64_t q1 = __ballot((qq & 4u) != 0), q2 = __ballot((qq & 8u) != 0);
                uint32_t u[11];
#pragma unroll
                for (int i2 = 0; i2 < 11; ++i2) u[i2] = __builtin_amdgcn_alignbyte(r[i2 + 1], r[i2], qb);
#pragma unroll
                for (int i2 = 0; i2 < 7; ++i2)
                    ev[i2] = lsel(q2, lsel(q1, u[i2 + 3], u[i2 + 2]), lsel(q1, u[i2 + 1], u[i2]));
            }
            const uint32_t type = (ev[0] >> 16) & 0xFFu;    // byte 26
            const uint32_t clen = ev[6] & 0xFFFFu;          // bytes 48..49
            const uint32_t elen = bare_type(type) ? kHdr : kHdr + clen;
            const bool live = act & inw & ((sl == 0 && !crossed) | fz | (p != vend));
            const uint32_t liml = p >= V ? lim1 : len;        // (p < len <= V before the wrap)
            const bool fit = p + elen <= liml;                // log_fit_entry
            const bool ok = live & fit;
            const bool cont = ok & (elen == elen_g) & (sl < 15u);
            const uint32_t okS = (uint32_t)(__ballot(ok) >> sh) & 0xFFFFu;
            const uint32_t ghS = (uint32_t)(__ballot(live & !fit & (p + kHdr <= liml)) >> sh) & 0xFFFFu;
            const uint32_t fb = (uint32_t)__builtin_ctz(((uint32_t)(__ballot(!cont) >> sh) & 0xFFFFu) | 0x8000u);
            const uint32_t nconf = fb + ((okS >> fb) & 1u);
            if (act && nconf == 0) { fl |= kJumpReq; act = false; }   // ghost header at m
            const bool conf = act & (sl < nconf);
            uint32_t msk = eq1_nibble(ev[1]);
            if (size > 4) msk |= eq1_nibble(ev[2]) << 4;
            if (size > 8) msk |= (eq1_nibble(ev[3]) << 8) | (eq1_nibble(ev[4]) << 12);
            msk = (msk | self_bit) & size_mask;
            const uint32_t fS = (uint32_t)(__ballot(conf & ((uint32_t)__builtin_popcount(msk) < need)) >> sh) & 0xFFFFu;
            if (CHECKSUM) {
                // the zeroed bytes 27..47 of confirmed entries
                const uint32_t snd = ev[0] >> 24;          // byte 27
                const uint32_t sb = udot4(ev[5], 0x01010101u, udot4(ev[4], 0x01010101u,
                                    udot4(ev[3], 0x01010101u, udot4(ev[2], 0x01010101u,
                                    udot4(ev[1], 0x01010101u, snd)))));
                const uint32_t stb = udot4(ev[5], 0x2F2E2D2Cu, udot4(ev[4], 0x2B2A2928u,
                                     udot4(ev[3], 0x27262524u, udot4(ev[2], 0x23222120u,
                                     udot4(ev[1], 0x1F1E1D1Cu, 27u * snd)))));
                const uint32_t csb = conf ? sb : 0u;
                exb += csb;
                if (p >= V) exb1 += csb;
                exxb += rel * csb + (conf ? stb : 0u);
            }
            const uint32_t lastl = sh + (nconf ? nconf - 1u : 0u);
            const uint32_t elen_last = (uint32_t)__shfl((int)elen, (int)lastl);
            const uint32_t p_last = (uint32_t)__shfl((int)p, (int)lastl);
            const uint32_t ef = fS ? (uint32_t)__builtin_ctz(fS) : nconf;
            const uint32_t p_stop = (uint32_t)__shfl((int)p, (int)(sh + (ef < 16u ? ef : 15u)));
            if (act) {
                if (!(fl & kStopped)) {
                    if (fS) {
                        stop = p_stop >= V ? p_stop - V : p_stop;     // ring offset
                        fl |= kStopped;
                    }
                    n_commit += ef;
                }
                if (p_last >= V && !(fl & kSeg1)) {           // crossed the wrap
                    fl |= kSeg1 | (gcase ? kGhJump : 0u);
                    gap0 = q;
                    ++steps;
                }
                if (LIT) lp = p_last;
                m = p_last + elen_last;
                elen_g = elen_last;
                fl &= ~kForced;
                steps += nconf;
                if (nconf <= fb && ((ghS >> fb) & 1u)) fl |= kJumpReq;   // ghost right after the chain
                if (steps > guard) fl |= kBail;
                if (!CHECKSUM && (fl & kStopped)) fl |= kDone;
            }
        }

        // ---- LIT: where the last NC determinant lies ----
        // log_entries_to_nc_buf records a ghost header and steps over its
        // copy at 0 by the ghost's length; the walk above reads the copy.  So
        // the copy stands for the ghost when it is the last entry, and a copy
        // of another length than its ghost sends the group to the tail's walk.
        uint32_t lidx = ~0u, lterm = 0xFFFFu;
        if (LIT) {
            const bool walked = (fl & (kDone | kBail)) == kDone && g < G && (pkf & kPkWindowed);
            const bool gh = (fl & kGhJump) != 0 && gap0 + kHdr <= V;
            // the candidate header's two pieces, requested before the ghost test
            // below decides whether it counts (a window offset in every lane)
            const uint32_t yh = walked && lp != ~0u ? ((gh && lp == V) ? gap0 : lp) - ws : 0u;
            const uint32_t k = yh >> 4, yb = yh & 3u;
            const uint64_t d1 = __ballot((yh & 4u) != 0), d2 = __ballot((yh & 8u) != 0);
            const uint4 a = win[pslot(k)], c = win[pslot(k + 1u)];
            uint32_t glen = 0, clen0 = 0;
            if (__ballot(walked && gh)) {
                const uint8_t *win8 = reinterpret_cast<const uint8_t *>(win);
                const uint32_t yg = (walked && gh) ? gap0 - ws : 0u, yc = (walked && gh) ? V - ws : 0u;
                auto byte_at = [&](uint32_t y) { return (uint32_t)win8[y + ((y >> 8) << 4)]; };
                const uint32_t tg = byte_at(yg + 26u), tc = byte_at(yc + 26u);
                glen = bare_type(tg) ? kHdr : kHdr + (byte_at(yg + 48u) | (byte_at(yg + 49u) << 8));
                clen0 = bare_type(tc) ? kHdr : kHdr + (byte_at(yc + 48u) | (byte_at(yc + 49u) << 8));
            }
            // (a ghost whose copy the walk never reached: the tail walks)
            const bool have = walked && lp != ~0u && (!gh || (lp >= V && glen == clen0));
            // that header's (idx, term): words aligned by byte (alignbyte) and
            // by word (lane-mask selects).  An index past 32 bits or a term
            // past 16 is left to the tail's exact walk (the same result)
            const uint32_t r[8] = { a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w };
            uint32_t u[7], w[4];
#pragma unroll
            for (int i2 = 0; i2 < 7; ++i2) u[i2] = __builtin_amdgcn_alignbyte(r[i2 + 1], r[i2], yb);
#pragma unroll
            for (int i2 = 0; i2 < 4; ++i2)
                w[i2] = lsel(d2, lsel(d1, u[i2 + 3], u[i2 + 2]), lsel(d1, u[i2 + 1], u[i2]));
            const bool fits = have && w[1] == 0u && w[3] == 0u && w[2] < 0xFFFFu;
            lidx = fits ? w[0] : ~0u;
            lterm = fits ? w[2] : 0xFFFFu;
        }

        // ---- 4. checksum: the staged sums less the bytes outside the image ----
        uint32_t dig = 0;
        if (CHECKSUM) {
            const bool walked = (fl & (kDone | kBail)) == kDone && g < G && (pkf & kPkWindowed);
            // window-relative excluded ranges of this segment, in ONE pass of
            // 16-B pieces (the three used to take a 64-B loop each):
            //   R1 [0, commit0 - ws)       inside piece 0            -> lane 0
            //   R3 [frontier, window end)  inside the frontier's piece -> lane 1
            //   R2 the wrap gap [gap0, V)  its pieces                -> lanes 2..15, 14 per round
            uint32_t s_neg = exb, sh_neg = exb1, t_neg = exxb;
            const uint32_t vrel = V - ws;      // first window offset of the second segment (V > ws, 16-B aligned)
            {
                const uint32_t mr = m - ws, e3 = we_al - ws, r3 = mr < e3 ? mr : e3;
                const uint32_t g2 = (fl & kSeg1) ? gap0 - ws : vrel;
                const uint32_t lo = sl == 0 ? 0u : sl == 1 ? r3 : g2;
                const uint32_t hi = !walked ? 0u : sl == 0 ? commit0 - ws : sl == 1 ? e3 : vrel;
                uint32_t k = sl == 0 ? 0u : sl == 1 ? (r3 >> 4) : (g2 >> 4) + sl - 2u;
                for (uint32_t it = 0;; ++it) {
                    const uint32_t X = 16u * k;
                    // bytes [a, b) of piece k (a < b only where the lane has work)
                    const uint32_t a = lo > X ? lo - X : 0u;
                    const uint32_t bb = hi > X ? (hi - X < 16u ? hi - X : 16u) : 0u;
                    const bool in = a < bb && (it == 0 || sl >= 2u);
                    if (!__ballot(in)) break;
                    const uint4 w = win[pslot(in ? k : 0u)];
                    // 16-bit byte mask of [a, b), each nibble spread to a 0x01-per-byte word
                    const uint32_t M = in ? ((1u << bb) - 1u) & ~((1u << a) - 1u) : 0u;
                    const uint32_t m0 = ((M & 0xFu) * 0x00204081u) & 0x01010101u;
                    const uint32_t m1 = (((M >> 4) & 0xFu) * 0x00204081u) & 0x01010101u;
                    const uint32_t m2 = (((M >> 8) & 0xFu) * 0x00204081u) & 0x01010101u;
                    const uint32_t m3 = ((M >> 12) * 0x00204081u) & 0x01010101u;
                    const uint32_t s0 = udot4(w.w, m3, udot4(w.z, m2, udot4(w.y, m1, udot4(w.x, m0, 0u))));
                    const uint32_t t0 = udot4(w.w, (m3 * 0xFFu) & 0x0F0E0D0Cu, udot4(w.z, (m2 * 0xFFu) & 0x0B0A0908u,
                                        udot4(w.y, (m1 * 0xFFu) & 0x07060504u, udot4(w.x, (m0 * 0xFFu) & 0x03020100u,
                                                                                    X * s0))));
                    s_neg += s0;
                    if (X >= vrel) sh_neg += s0;
                    t_neg += t0;
                    k += 14u;
                }
            }
            // staged position sums: t = sum (16 k + i) b, k = sl + 16 j
            const uint32_t t_pos = t_in + 16u * sl * s_pos + 256u * (kSegPPL * s_pos - r_pre);
            uint32_t s_c = s_pos - s_neg, s1_c = (s_pos - s_lo) - sh_neg, t_c = t_pos - t_neg;
            // segment sums (DPP row = the 16 lanes of a segment) land in its lane 15
            s_c += dpp_shr<0x111>(s_c); s_c += dpp_shr<0x112>(s_c); s_c += dpp_shr<0x114>(s_c); s_c += dpp_shr<0x118>(s_c);
            s1_c += dpp_shr<0x111>(s1_c); s1_c += dpp_shr<0x112>(s1_c); s1_c += dpp_shr<0x114>(s1_c); s1_c += dpp_shr<0x118>(s1_c);
            t_c += dpp_shr<0x111>(t_c); t_c += dpp_shr<0x112>(t_c); t_c += dpp_shr<0x114>(t_c); t_c += dpp_shr<0x118>(t_c);
            // image positions: v - commit0 before V, v - V + (gap0 - commit0) past it;
            // every true value is below 2^32, so wrapping u32 arithmetic is exact
            const uint32_t T = t_c + (ws - commit0) * s_c - (V - gap0) * s1_c;
            const uint32_t N = (fl & kSeg1) ? (gap0 - commit0) + (m - V) : m - commit0;
            const uint32_t A = (1u + s_c) % kAdlerMod;
            const uint32_t B = (N * s_c + N - T) % kAdlerMod;
            dig = (B << 16) | A;
        }

        // ---- 5. results into the block's slots: lane 4 qi + s takes segment s's ----
        {
            const uint32_t res = (fl & kStopped) ? stop : ((fl & kSeg1) ? m - V : m);
            const bool adv = dist32(end, len, res) < dist32(end, len, commit0);
            const uint32_t oc = adv ? res : commit0;
            const uint32_t of = (fl & kBail) ? kSlBail : (adv ? kSlAdv : 0u);
            if (sl == 15u && g < G && (fl & kBail))
                slow_v[1 + atomicAdd(slow_v, 1u)] = g;            // quorum_tail_kernel decides
            const int src = (int)(16u * (lane & 3u) + 15u);       // segment (lane & 3)'s lane 15 (dig lives there)
            const uint32_t v_c = (uint32_t)__shfl((int)oc, src), v_f = (uint32_t)__shfl((int)of, src);
            const uint32_t v_n = (uint32_t)__shfl((int)n_commit, src), v_d = (uint32_t)__shfl((int)dig, src);
            const uint32_t v_li = LIT ? (uint32_t)__shfl((int)lidx, src) : 0u;
            const uint32_t v_lt = LIT ? (uint32_t)__shfl((int)lterm, src) : 0u;
            if ((lane >> 2) == qi) {
                sl_c = v_c;
                sl_nf = (LIT ? v_n | (v_lt << 8) : v_n) | (v_f << 24);
                sl_d = v_d;
                if (LIT) sl_li = v_li;
            }
        }
        F = NF;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    // ---- block epilogue: lane i writes group blk*64 + i (coalesced) ----
    {
        const uint32_t g = g0b + lane;
        const uint32_t sl_f = sl_nf >> 24, sl_n = sl_nf & (LIT ? 0xFFu : 0xFFFFFFu);
        const uint32_t sl_lt = (sl_nf >> 8) & 0xFFFFu;
        const bool w = lane < nin && !(sl_f & kSlBail);     // deferred groups: quorum_tail_kernel writes them
        // (the ~0 mark of a deferred group's commit, as in commit_wave_kernel)
        if (lane < nin && (sl_f & kSlBail) && o.new_commit) o.new_commit[g] = ~0ull;
        if (w) {
            if (o.new_commit) o.new_commit[g] = (uint64_t)sl_c;
            if (o.committed) o.committed[g] = (uint8_t)(sl_f & kSlAdv);
            if (o.n_entries) o.n_entries[g] = sl_n;
            if (CHECKSUM && o.digest) o.digest[g] = sl_d;
        }
        // LIT: every group of the block, its (idx, term) or "none" as the
        // u64 pair (~0, ~0) (a deferred group: none, the tail walks it)
        if (LIT && lane < nin) {
            const bool none = (sl_f & kSlBail) || sl_lt == 0xFFFFu;
            o.last_idx_term[2u * (uint64_t)g] = none ? ~0ull : (uint64_t)sl_li;
            o.last_idx_term[2u * (uint64_t)g + 1u] = none ? ~0ull : (uint64_t)sl_lt;
        }
        acc_dec += (uint32_t)__builtin_popcountll(__ballot(w));
        acc_adv += (uint32_t)__builtin_popcountll(__ballot(w && (sl_f & kSlAdv)));
        acc_ent += wave_sum_res(w ? sl_n : 0u);
    }
    FB = blk_of(rawB, cap);
    // the old rows die before the new ones are requested, so the loads land in
    // the loop-carried registers: scheduled the other way round, a register copy
    // of a loaded byte waited for every load in flight once per block
    asm volatile("" ::"v"(FB.commit), "v"(FB.end), "v"(FB.len), "v"(FB.vend), "v"(FB.pk) : "memory");
    if (DYN) {
        blk = nb1;
        nb1 = __builtin_amdgcn_readfirstlane(nb2v);
        rawB = load_blk_raw(b, (uint64_t)nb1 * 64u + lane, G);
    } else {
        rawB = load_blk_raw(b, (uint64_t)(blk + 2u * nw) * 64u + lane, G);
        blk += nw;
    }
    }

    uint64_t mine[kWaveStats] = { lane == 0 ? acc_dec : 0u, lane == 0 ? acc_ent : 0u, lane == 0 ? acc_adv : 0u };
    block_partials<kWaveStats>(vptr(partials), mine);
}

// ---------------------------------------------------------------------------
// commit_lane_kernel: one lane per group (APUS_BATCH_LANE_IMPL)
// ---------------------------------------------------------------------------
template <bool CHECKSUM>
__global__ void __launch_bounds__(256) commit_lane_kernel(const apus_batch_t b, const WalkOut o,
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
// quorum_tail_kernel: everything a commit call does after its walk, in ONE
// launch (before: the deferred-walk kernel, a statistics fold, the median
// kernel, the pruning kernel and a second fold -- five launches, the group
// state rows read twice):
//   1. the groups the walk deferred (slow[0] of them in slow[1..]): the exact
//      one-lane walk (lane_group), as commit_slow_kernel did;
//   2. per group, one read of the state row for the DARE median quorum (a4,
//      median_group) and log_pruning's minimum (a7, prune_group);
//   3. the block that arrives last folds the walk launch's block partials
//      and every block's partials of this launch into the context statistics
//      and clears the deferred list and the arrival ticket.
// Hand-off to the last block (MI355X_MICROARCH.md, inter-workgroup
// visibility): partial rows stored sc1 (write-through), every storing wave
// drained, a block barrier, one relaxed agent-scope ticket add per block;
// the last arriver reads the rows with sc1 loads.  The walk launch's
// partials come from an earlier kernel (plain loads would do; sc1 too).
// ---------------------------------------------------------------------------
constexpr int kTailStats = 7;   // decisions, committed, advanced, corrupt, slow; watermark (min); votes won
constexpr uint32_t kTailMed = 1u, kTailPrune = 2u, kTailWm = 4u, kTailFresh = 8u, kTailLit = 16u, kTailLitRows = 32u,
                   kTailVote = 64u, kTailRank = 128u, kTailPrev = 256u, kTailPub = 512u, kTailForce = 1024u,
                   kTailWalked = 2048u, kTailList = 4096u;
// kTailList (run time only): the launch after quorum_row_kernel -- it works
// the list alone (the walk's deferred groups, walked here, and the groups the
// row kernel handed over, bit 31 set: their tail work only), then folds.
// Flag sets with an instantiation of their own, every flag a compile-time
// constant (SF): the loads of a group are then straight-line code.  With the
// flags read at run time every flag-dependent load sits in a branch of its
// own, and the waits the compiler places at those joins serialise them
// (profiles/r04/tail/).  kTailFresh only steers the fold; it may be either.
constexpr uint32_t kTailSetC2 = kTailMed | kTailPrune | kTailWm | kTailPrev;
constexpr uint32_t kTailSetC5 = kTailSetC2 | kTailLit | kTailLitRows | kTailVote | kTailRank;
// the bench steps with update_remote_logs' publish (C2, C5) and, at C4,
// force_log_pruning in place of log_pruning
constexpr uint32_t kTailSetC2P = kTailSetC2 | kTailPub | kTailWalked;
constexpr uint32_t kTailSetC5P = kTailSetC5 | kTailPub | kTailWalked;

struct TailArgs {
    const uint32_t *slow;     // the walk's deferred list (NULL: none)
    const uint64_t *wpart;    // the walk launch's block partials (NULL: none)
    uint32_t wblk, wstat;     // their rows and columns (column k -> kCommitStatMap's k-th statistic)
    uint64_t *tpart;          // this launch's rows [gridDim.x][kTailStats]
    uint32_t *ticket;         // arrivals; 0 between launches
    uint64_t *stats;          // ctx->stats
    uint32_t *slow_reset;     // slow[0], cleared by the last block (NULL: none)
    uint32_t flags;           // kTail*
    const uint64_t *rpart;    // quorum_row_kernel's block rows [rblk][kTailStats] (NULL: none)
    uint32_t rblk;
};
// kTailPub: update_remote_logs' publish on the walk's commit (kTailWalked:
// the call walked; o.new_commit holds it, or ~0 for a group the walk
// deferred: such a group is walked by the lane that finishes it, not by the
// deferred-walk loop, so its commit is known there).  kTailForce:
// force_log_pruning on the log as given (never beside a walk: polling() runs
// apply_committed_entries between the two, apus_commit_batch).
struct TailOut2 {
    uint16_t *publish;
    uint64_t *ssn;
    apus_force_out_t force;
};
// kTailLit: o.last_idx_term from the walk's rows (kTailLitRows: each row holds
// the group's (idx, term) already, or the pair (~0, ~0): walked here) or
// walked here for every group.
// kTailVote / kTailRank (FAIL instantiations only): the failover pass of every
// group after its median and pruning, on the state row already in registers
// (vote_of / rank_of, the code apus_vote_batch / apus_vote_rank_batch run);
// the ranking takes the local (idx, term) just produced (kTailLit) or
// b.last_idx_term.

__device__ __forceinline__ uint64_t ld_sc1(const uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// (the bench sets with the ranking: two waves per SIMD asked for -- their
// LDS slabs allow two blocks per CU -- which keeps the 7-replica form, at the
// edge of 256 VGPRs, from taking a third register bank and one wave)
template <int N, int NR, bool CHECKSUM, bool FAIL, uint32_t SF>
constexpr int tail_min_waves() { return FAIL && SF != 0 && (SF & kTailRank) != 0 && NR <= 8 ? 2 : 1; }

template <int N, int NR, bool CHECKSUM, bool FAIL, uint32_t SF>
__global__ void __launch_bounds__(256, (tail_min_waves<N, NR, CHECKSUM, FAIL, SF>())) quorum_tail_kernel(const apus_batch_t b, const WalkOut o, const TailArgs t,
                                                          const apus_vote_out_t vo, const apus_rank_out_t ro,
                                                          const TailOut2 o2)
{
    // the flags: compile-time (SF) or read at run time (SF == 0)
    const uint32_t tf = SF ? SF : t.flags;
    const bool listmode = (t.flags & kTailList) != 0;
    // the ranking's request rows staged in LDS (the bench sets with the
    // ranking, R = 3, 5, 7): one slab per wave, 64 rows of up to 5 u64 per
    // replica, rounded up to whole 1-KiB DMA instructions
    constexpr bool kStage = FAIL && SF != 0 && (SF & kTailRank) != 0 && (NR == 3 || NR == 5 || NR == 7);
    constexpr uint32_t kSlabQ = kStage ? ((64u * NR * 5u * 8u + 1023u) / 1024u) * 128u : 1u;
    uint64_t acc[kTailStats] = { 0, 0, 0, 0, 0, ~0ull, 0 };
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
    // publish / force: the deferred groups are walked in the main loop
    const bool own = (tf & (kTailPub | kTailForce)) != 0;
    const bool work = (tf & (kTailMed | kTailPrune | kTailLit | kTailVote | kTailRank | kTailPub | kTailForce)) != 0;
    {
        const bool med = (tf & kTailMed) != 0, lit = (tf & kTailLit) != 0;
        const bool pub = (tf & kTailPub) != 0, force = (tf & kTailForce) != 0;
        const bool pr = (tf & kTailPrune) != 0 && !force;       // force_log_pruning replaces log_pruning
        const bool vote = FAIL && (tf & kTailVote) != 0, rank = FAIL && (tf & kTailRank) != 0;
        const bool prev = (tf & kTailPrev) != 0, base = (tf & kTailWm) != 0, walked = (tf & kTailWalked) != 0;
        // lrow: the group's request row in LDS (rq u64 per replica; records:
        // the 40-B vote_req_t records), or null: read from HBM per lane
        auto tail_group = [&](uint64_t g, const uint64_t *lrow, uint32_t rq, bool records) {
            // every input first (one memory round trip), then the results
            constexpr bool EX = NR != 8 && NR != 16;
            const apus_group_state_t st = load_state(b, g);
            QuorumIn<NR> q;
            load_quorum_in<NR, EX>(b, g, med || pub, pr || force, prev, base, q);
            uint64_t rc[NR] = {};
            uint32_t conn = 0xFFFFu;
            uint64_t commit = st.commit;
            if (pub) {
                const uint32_t R = EX ? (uint32_t)NR : b.n_replicas;
#pragma unroll
                for (int i = 0; i < NR; ++i) rc[i] = (EX || (uint32_t)i < R) ? col_ld(b.remote_commit + g * R + i) : 0ull;
                if (b.rc_connected) conn = col_ld(b.rc_connected + g);
            }
            if (walked) commit = col_ld(o.new_commit + g);
            uint64_t lr0 = ~0ull, lr1 = ~0ull;
            if (tf & kTailLitRows) { lr0 = col_ld(o.last_idx_term + 2 * g); lr1 = col_ld(o.last_idx_term + 2 * g + 1); }
            FailIn<FAIL ? NR : 1> f;
            if (FAIL) {
                if (lrow) load_fail_in_lds<FAIL ? NR : 1, EX>(b, g, vote, f);
                else load_fail_in<FAIL ? NR : 1, EX>(b, g, vote, rank, f);
            }
            const uint32_t self = (FAIL || pub || force) ? (uint32_t)b.self_idx[g] : 0u;
            if (own && walked && commit == ~0ull) {
                // deferred by the walk kernel (the ~0 mark): the exact one-lane walk here
                uint32_t c, fl;
                lane_group<CHECKSUM>(b, o, g, &c, &fl);
                acc[0] += 1; acc[1] += c; acc[2] += fl & 1u; acc[3] += fl >> 1; acc[4] += 1;
                commit = o.new_commit[g];
            }
            if (med) col_st(o.median + g, median_of<N, NR>(b.n_replicas, st, q));
            if (pr) {
                const uint64_t w = prune_of<NR>(b, g, st, q, o.new_head, o.append_head, o.min_apply);
                acc[5] = w < acc[5] ? w : acc[5];
            }
            if (pub) {
                const uint32_t m = publish_from<NR, EX>(b, g, st, self, commit, q, rc, conn);
                if (o2.publish) col_st(o2.publish + g, (uint16_t)m);
                if (o2.ssn && m) o2.ssn[g] += 1;
            }
            uint64_t idx = 0, term = 0;
            if (lit) {
                // the (idx, term) the walk read (a6's local (idx, term)), or
                // the determinant walk of apus_last_idx_term_batch (the pair
                // (~0, ~0) is also a value a log may hold: walking it again
                // gives the same result)
                if (lr0 != ~0ull || lr1 != ~0ull) {
                    idx = lr0;
                    term = lr1;
                } else {
                    local_idx_term(b, g, st, idx, term);
                    o.last_idx_term[2 * g] = idx;
                    o.last_idx_term[2 * g + 1] = term;
                }
            }
            if (FAIL && (vote || rank)) {
                if (vote) acc[6] += vote_from<FAIL ? NR : 1, EX>(b, g, st, self, f, vo) ? 1u : 0u;
                if (rank) {
                    if (!lit) { idx = b.last_idx_term[2 * g]; term = b.last_idx_term[2 * g + 1]; }
                    if (lrow) fail_rows_lds<FAIL ? NR : 1, EX>(b, lrow, rq, records, f);
                    rank_from<FAIL ? NR : 1, EX>(b, g, st, self, idx, term, f, ro);
                }
            }
            if (force) {
                // force_log_pruning last (polling(), dare_server.c:1121-1124),
                // on the log as given (a non-walking call: commit = state's)
                apus_group_state_t cur = st;
                cur.commit = commit;
                bool stopped = false;
                const uint64_t w = force_prune_of<NR, EX>(b, g, cur, self, q, b.sid, o.new_head, o.append_head,
                                                          o.min_apply, o2.force, stopped);
                acc[5] = w < acc[5] ? w : acc[5];
                acc[3] += stopped ? 1u : 0u;
            }
        };
        // (chunks of 1024 groups per wave from a counter, as the walks take
        // their blocks, measured no faster at the C4 1-GPU point and 130 us
        // slower at C2: profiles/r03/tail_dyn/ab_tail.log; two groups per lane
        // per round, the second's inputs requested before the first's results,
        // 157 VGPRs: 2.96 vs 2.91 ms there, profiles/r04/tail_u2/)
        if (t.slow && (!own || listmode)) {
            // the walk's deferred groups (walked here); in list mode, after
            // quorum_row_kernel, also their tail work when the row kernel left
            // it (own: it skipped them) and the groups it handed over (bit 31)
            const uint32_t n = t.slow[0];
            for (uint32_t i = tid; i < n; i += nth) {
                const uint32_t e = t.slow[1 + i];
                const uint64_t g = e & 0x7FFFFFFFu;
                if (!(e >> 31) || !listmode) {
                    uint32_t c, fl;
                    lane_group<CHECKSUM>(b, o, listmode ? g : (uint64_t)e, &c, &fl);
                    acc[0] += 1; acc[1] += c; acc[2] += fl & 1u; acc[3] += fl >> 1; acc[4] += 1;
                }
                if (listmode && work && (own || (e >> 31))) tail_group(g, nullptr, 0, false);
            }
        }
        if (work && !listmode) {
            if constexpr (kStage) {
                // The request rows of the wave's 64 groups (R records of 40 B,
                // or the packed 24-B rows, per group: one contiguous run) come
                // in by LDS-DMA, 1 KiB per wave instruction, before the
                // group's other loads; each lane then reads its own row from
                // LDS.  Lane-per-group loads of the same bytes touch 64 lines
                // per instruction (21 such instructions per wave at R = 7).
                // A partial last wave, or a row base not 16-B aligned, takes
                // 4-B pieces (u64 columns are 8-B aligned).
                __shared__ __attribute__((aligned(16))) uint64_t slab_all[4 * kSlabQ];
                const uint32_t lane = threadIdx.x & 63u;
                uint64_t *const slab = slab_all + (threadIdx.x >> 6) * kSlabQ;
                const bool packed = b.vote_sit != nullptr;
                const uint64_t *const req = packed ? b.vote_sit : reinterpret_cast<const uint64_t *>(b.vote_req);
                const uint32_t rq = packed ? 3u : (uint32_t)(sizeof(apus_vote_req_t) / 8);
                const uint32_t rowq = (uint32_t)NR * rq;          // u64 per group
                const bool al = (reinterpret_cast<uintptr_t>(req) & 15u) == 0;
                for (uint64_t g0 = tid - lane; g0 < b.n_groups; g0 += nth) {
                    const uint64_t left = b.n_groups - g0;
                    const uint32_t rows = left < 64u ? (uint32_t)left : 64u;
                    const uint64_t *const src = req + g0 * rowq;
                    // the previous group's reads of the slab retired
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (al && rows == 64u) {
                        const uint32_t pieces = rowq * 32u;       // 16-B pieces of 64 rows
                        for (uint32_t c = 0; c < pieces; c += 64) {
                            // lanes past the last piece re-read it into the slab's padding
                            const uint32_t p = c + lane < pieces ? c + lane : pieces - 1;
                            __builtin_amdgcn_global_load_lds(
                                (const void *)(src + 2 * p),
                                (__attribute__((address_space(3))) void *)(slab + 2 * c), 16, 0, 0);
                        }
                    } else {
                        const uint32_t pieces = rows * rowq * 2u;  // 4-B pieces
                        const uint32_t *const s4 = reinterpret_cast<const uint32_t *>(src);
                        for (uint32_t c = 0; c < pieces; c += 64) {
                            const uint32_t p = c + lane < pieces ? c + lane : pieces - 1;
                            __builtin_amdgcn_global_load_lds(
                                (const void *)(s4 + p),
                                (__attribute__((address_space(3))) void *)(reinterpret_cast<uint32_t *>(slab) + c), 4,
                                0, 0);
                        }
                    }
                    if (lane < rows) tail_group(g0 + lane, slab + lane * rowq, rq, !packed);
                }
            } else {
                for (uint64_t g = tid; g < b.n_groups; g += nth) tail_group(g, nullptr, 0, false);
            }
        }
    }
    block_partials<kTailStats, 1u << 5, true>(t.tpart, acc);
    __shared__ uint32_t last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    // The hand-off is the form MI355X_MICROARCH.md's inter-workgroup table
    // lists for "ONE lane of each storing workgroup, for ALL that workgroup's
    // stores: an agent-scope atomic add ... the workgroup whose add came
    // last": every partial-row store sc1 (write-through) and drained by its
    // wave (vmcnt(0) above) before the barrier, one relaxed agent-scope add
    // per block, the last block's loads all sc1 (ld_sc1).  The HIP-memory-model
    // form -- a release fence before an acq_rel add, an acquire fence in the
    // last block -- writes back the XCD's L2 in every
    // block (buffer_wbl2): the C2 tail took 132 us against 55 us, the C5
    // tail 0.60 against 0.43 ms (same box, profiles/r04/tail/ab_tail2.log).
    if (threadIdx.x == 0) {
        last = __hip_atomic_fetch_add(t.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    // the last arriver: fold (sums over both launches' rows, one minimum)
    __shared__ uint64_t red[kTailStats + 5][4];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint64_t s[kTailStats + 5];
#pragma unroll
    for (int k = 0; k < kTailStats + 5; ++k) s[k] = k == 5 ? ~0ull : 0ull;   // column 5: the watermark (min)
    for (uint32_t i = threadIdx.x; i < gridDim.x; i += blockDim.x) {
#pragma unroll
        for (int k = 0; k < kTailStats; ++k) {
            const uint64_t y = ld_sc1(&t.tpart[(uint64_t)i * kTailStats + k]);
            s[k] = k == 5 ? (y < s[k] ? y : s[k]) : s[k] + y;
        }
    }
    if (t.rpart)
        for (uint32_t i = threadIdx.x; i < t.rblk; i += blockDim.x) {
#pragma unroll
            for (int k = 0; k < kTailStats; ++k) {
                const uint64_t y = ld_sc1(&t.rpart[(uint64_t)i * kTailStats + k]);
                s[k] = k == 5 ? (y < s[k] ? y : s[k]) : s[k] + y;
            }
        }
    if (t.wpart)
        for (uint32_t i = threadIdx.x; i < t.wblk; i += blockDim.x)
#pragma unroll
            for (int k = 0; k < 5; ++k)
                if ((uint32_t)k < t.wstat) s[kTailStats + k] += ld_sc1(&t.wpart[(uint64_t)i * t.wstat + k]);
#pragma unroll
    for (int k = 0; k < kTailStats + 5; ++k) {
        uint64_t x = s[k];
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
            const uint64_t y = __shfl_xor(x, d);
            x = k == 5 ? (y < x ? y : x) : x + y;
        }
        if (lane == 0) red[k][wv] = x;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t v[kTailStats + 5];
#pragma unroll
        for (int k = 0; k < kTailStats + 5; ++k) {
            uint64_t x = red[k][0];
            for (int w = 1; w < 4; ++w) x = k == 5 ? (red[k][w] < x ? red[k][w] : x) : x + red[k][w];
            v[k] = x;
        }
        uint64_t add[APUS_STAT_COUNT] = {};
        // walk columns (decisions, committed, advanced[, corrupt, slow]) and
        // the deferred walks' tallies, mapped as the separate fold mapped them
#pragma unroll
        for (int k = 0; k < 5; ++k) add[(kCommitStatMap >> (8 * k)) & 0xFFu] += v[k] + v[kTailStats + k];
        add[APUS_STAT_VOTES_WON] += v[6];
        const bool wm = (t.flags & kTailWm) != 0;
        if (t.flags & kTailFresh) {
            // the statistics of this call replace the accumulated ones
            // (apus_stats_reset folded in)
#pragma unroll
            for (int k = 0; k < APUS_STAT_COUNT; ++k)
                t.stats[k] = k == APUS_STAT_MIN_WATERMARK ? (wm ? v[5] : ~0ull) : add[k];
        } else {
#pragma unroll
            for (int k = 0; k < APUS_STAT_COUNT; ++k)
                if (k != APUS_STAT_MIN_WATERMARK && add[k])
                    atomicAdd((unsigned long long *)&t.stats[k], (unsigned long long)add[k]);
            if (wm) atomicMin((unsigned long long *)&t.stats[APUS_STAT_MIN_WATERMARK], (unsigned long long)v[5]);
        }
        if (t.slow_reset) __hip_atomic_store(t.slow_reset, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(t.ticket + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // the walk's block counter
        __hip_atomic_store(t.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------------------
// quorum_row_kernel: the tail's per-group work with EIGHT lanes per group
// (VERDICT r4 #3).  quorum_tail_kernel gives every group one lane: each of
// its column loads takes 8 B per lane from 64 groups' rows (a 7-replica row
// is 56 B: 28 lines per load instruction), and the failover instantiation
// holds every input of a group in registers at once (239-252 VGPRs: 2 waves
// per SIMD).  Here lane r of a row of 8 holds replica r of its group: each
// column load is one contiguous run of the row's bytes (8 groups per wave,
// 8 x 56 B = 448 B per load instruction), a lane holds one replica's values,
// and the per-group arithmetic runs across the row with the rows' own
// ballots, shuffles and 3-step reductions:
//   median (a4)   slot r's value; counts by ballot; the rank of slot r among
//                 the row's keys from 7 xor shuffles; the slot of rank
//                 (size - 1) / 2 broadcast (median_slots over 8 slots);
//   pruning (a7)  the OFF servers reset in place; the first circular minimum
//                 as a 3-step (distance, index) reduction, log->apply first;
//   publish       each lane its own server's condition and store;
//   vote (a5)     counts and voters by ballot, the commit as a (distance,
//                 index) reduction;
//   ranking (a6)  loop 1 as an exclusive prefix maximum across the row, loop
//                 2 (a chain through the accepted requests) as 8 broadcast
//                 steps every lane of the row runs alike.
// Every flag is a compile-time constant (SF: the bench sets), NR = R <= 8.
// A group it cannot take -- configuration sizes past 8, or (kTailWalked) a
// walk the walk kernel deferred (new_commit ~0) -- is left to the list
// launch that follows (quorum_tail_kernel, kTailList): a deferred group is
// already on the walk's list; a size case is appended with bit 31.  Results
// are bit-identical to quorum_tail_kernel's (the same formulas per slot).
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T rw_shfl(T v, uint32_t src) { return __shfl(v, (int)src, 8); }
template <typename T>
__device__ __forceinline__ T rw_xor(T v, int m) { return __shfl_xor(v, m, 8); }
template <typename T>
__device__ __forceinline__ T rw_up(T v, uint32_t d) { return __shfl_up(v, d, 8); }
// the row's 8 predicate bits (bit r = lane r of the row)
__device__ __forceinline__ uint32_t rw_bits(bool p, uint32_t lane)
{
    return (uint32_t)(__ballot(p) >> (lane & 56u)) & 0xFFu;
}

struct RowArgs {
    uint32_t *list;      // the walk's deferred list (count, then entries): handed-over groups appended
    uint64_t *rpart;     // this launch's block rows [gridDim.x][kTailStats]
};

// median_slots<8, NR> for a group whose sizes are <= 8: lane r holds slot r
template <int NR>
__device__ __forceinline__ uint64_t rw_median(const apus_group_state_t &st, uint32_t r, uint32_t lane, uint32_t self,
                                              uint64_t rend, uint32_t step, uint32_t fail)
{
    const uint64_t len = st.len, end = st.end, commit = st.commit;
    const bool transit = st.cid.state == APUS_CID_TRANSIT;
    const bool upd = r < (uint32_t)NR && r != self && ((st.cid.bitmask >> r) & 1u) &&
                     fail < APUS_PERMANENT_FAILURE && step == APUS_LR_UPDATE_LOG;
    const uint64_t off = r == self ? end : upd ? rend : commit;
    const uint32_t size0 = st.cid.size[0], size1 = st.cid.size[1];
    // the value at rank (size - 1) / 2 of the slots' keys (slot order breaks ties)
    auto select = [&](uint32_t size) {
        const uint64_t key = r < size ? off : ~0ull;
        uint32_t rank = 0;
#pragma unroll
        for (int x = 1; x < 8; ++x) {
            const uint64_t kk = rw_xor(key, x);
            const uint32_t k = r ^ (uint32_t)x;
            rank += (kk < key || (kk == key && k < r)) ? 1u : 0u;
        }
        const uint32_t mi = (size - 1) / 2;
        const uint32_t want = mi < 8u ? mi : 0u;
        const uint32_t sel = (uint32_t)__builtin_ctz(rw_bits(rank == want, lane) | 0x100u) & 7u;
        return rw_shfl(key, sel);
    };
    uint64_t minv = commit;
    const uint32_t cnt0 = (uint32_t)__builtin_popcount(rw_bits(r < size0 && upd && larger(end, len, off, minv), lane));
    const bool ok0 = cnt0 >= size0 / 2;
    const uint64_t med0 = select(size0);
    if (ok0) minv = med0;
    if (transit) {
        // j = 1 on the new configuration, against the j = 0 minimum (or the
        // commit: median_slots compares at j = 1 either way)
        const uint32_t cnt1 =
            (uint32_t)__builtin_popcount(rw_bits(r < size1 && upd && larger(end, len, off, minv), lane));
        const uint64_t med1 = select(size1);
        if (cnt1 >= size1 / 2 && larger(end, len, minv, med1)) minv = med1;
    }
    return minv;
}

template <int NR, uint32_t SF>
__global__ void __launch_bounds__(256) quorum_row_kernel(const apus_batch_t b, const WalkOut o, const apus_vote_out_t vo,
                                                         const apus_rank_out_t ro, const TailOut2 o2, const RowArgs ra)
{
    static_assert(NR >= 2 && NR <= 8, "eight lanes per group");
    // (force_log_pruning never runs beside a walk, apus_commit_batch: no
    // row-kernel set carries it)
    static_assert(!(SF & kTailForce), "force_log_pruning is a call of its own");
    constexpr bool med = (SF & kTailMed) != 0, pr = (SF & kTailPrune) != 0, lit = (SF & kTailLit) != 0;
    constexpr bool litrows = (SF & kTailLitRows) != 0, vote = (SF & kTailVote) != 0, rank = (SF & kTailRank) != 0;
    constexpr bool pub = (SF & kTailPub) != 0, walked = (SF & kTailWalked) != 0, prev = (SF & kTailPrev) != 0;
    constexpr bool base = (SF & kTailWm) != 0;
    uint64_t acc[kTailStats] = { 0, 0, 0, 0, 0, ~0ull, 0 };
    const uint32_t lane = threadIdx.x & 63u, r = lane & 7u;
    const bool lead = r == 0;
    const uint64_t rows = (uint64_t)gridDim.x * (blockDim.x / 8u);
    const bool col = r < (uint32_t)NR;
    for (uint64_t g = (uint64_t)blockIdx.x * (blockDim.x / 8u) + (threadIdx.x >> 3); g < b.n_groups; g += rows) {
        // ---- every input of the group first: the state row and the group's
        // scalars (every lane of the row, the same bytes), lane r's replica r
        const apus_group_state_t st = load_state(b, g);
        const uint64_t gr = g * NR + r;
        uint64_t rend = 0, ap = 0, rc = 0, ack = ~0ull, hbv = 0, rs = 0, ri = 0, rt = 0;
        uint32_t step = 0, fail = 0;
        if (col) {
            if (med || pub) {
                rend = b.remote_end[gr];
                step = b.lr_step[gr];
                fail = b.fail_count[gr];
            }
            if (pr) ap = b.apply_offsets[gr];
            if (pub) rc = b.remote_commit[gr];
            if (vote) ack = b.vote_ack[gr];
            if (rank) {
                hbv = b.hb[gr];
                const uint64_t *rq = b.vote_sit ? b.vote_sit + 3 * gr
                                                : reinterpret_cast<const uint64_t *>(b.vote_req + gr);
                rs = rq[0];
                ri = rq[1];
                rt = rq[2];
            }
        }
        const uint32_t self = b.self_idx[g];
        const uint32_t pv = prev ? (uint32_t)b.prev_head[g] : 0u;
        const uint64_t bs = base ? b.abs_base[g] : ~0ull;
        const uint64_t sid = rank ? b.sid[g] : 0ull;
        const uint32_t conn = pub && b.rc_connected ? (uint32_t)b.rc_connected[g] : 0xFFFFu;
        const uint64_t commit = walked ? o.new_commit[g] : st.commit;
        uint64_t lr0 = ~0ull, lr1 = ~0ull;
        if (litrows) { lr0 = o.last_idx_term[2 * g]; lr1 = o.last_idx_term[2 * g + 1]; }
        if (walked && commit == ~0ull) continue;                    // deferred: the list launch finishes it
        if (st.cid.size[0] > 8u || st.cid.size[1] > 8u) {
            if (lead) ra.list[1 + atomicAdd(ra.list, 1u)] = (uint32_t)g | 0x80000000u;
            continue;
        }
        const uint32_t cidw = st.cid.bitmask;
        const bool on = ((cidw >> r) & 1u) != 0;
        // ---- a4: the DARE median
        if (med) {
            const uint64_t m = rw_median<NR>(st, r, lane, self, rend, step, fail);
            if (lead) o.median[g] = m;
        }
        // ---- a7: log_pruning's minimum
        if (pr) {
            const uint32_t esz = ext_group_size(st.cid);
            const bool in = col && r < esz;
            uint64_t a = ap;
            if (in && !on) { a = st.apply; b.apply_offsets[gr] = a; }          // OFF server
            // the first value of largest distance, log->apply first (larger() is strict)
            uint64_t d = in ? dist(st.end, st.len, a) : 0ull, v = a;
            uint32_t ix = in ? r : 15u;
#pragma unroll
            for (int x = 1; x < 8; x <<= 1) {
                const uint64_t d2 = rw_xor(d, x), v2 = rw_xor(v, x);
                const uint32_t i2 = rw_xor(ix, x);
                if (d2 > d || (d2 == d && i2 < ix)) { d = d2; v = v2; ix = i2; }
            }
            uint64_t mn = d > dist(st.end, st.len, st.apply) ? v : st.apply;
            if (dist(st.end, st.len, mn) == 0) {
                uint64_t tl = 0;
                if (lead) tl = device_get_tail(ring_view(b, g, st), st);
                mn = rw_shfl(tl, 0);
            }
            const bool app = larger(st.end, st.len, mn, st.head) && !pv;
            const uint64_t nh = app ? mn : st.head;
            if (lead) {
                if (o.new_head) o.new_head[g] = nh;
                if (o.append_head) o.append_head[g] = app ? 1 : 0;
                if (o.min_apply) o.min_apply[g] = mn;
                if (b.abs_base) { const uint64_t w = bs + nh; acc[5] = w < acc[5] ? w : acc[5]; }
            }
        }
        // ---- update_remote_logs' publish
        if (pub) {
            const bool pc = col && r < walk_size(st.cid) && r != self && on && fail < APUS_PERMANENT_FAILURE &&
                            ((conn >> r) & 1u) && step == APUS_LR_UPDATE_LOG && rc != rend && rc != commit;
            if (pc) b.remote_commit[gr] = larger(st.end, st.len, commit, rend) ? rend : commit;
            const uint32_t m = rw_bits(pc, lane);
            if (lead) {
                if (o2.publish) o2.publish[g] = (uint16_t)m;
                if (o2.ssn && m) o2.ssn[g] += 1;
            }
        }
        // ---- the candidate's local (idx, term)
        uint64_t idx = 0, term = 0;
        if (lit) {
            if (lr0 != ~0ull || lr1 != ~0ull) {
                idx = lr0;
                term = lr1;
            } else {
                if (lead) {
                    local_idx_term(b, g, st, idx, term);
                    o.last_idx_term[2 * g] = idx;
                    o.last_idx_term[2 * g + 1] = term;
                }
                idx = rw_shfl(idx, 0);
                term = rw_shfl(term, 0);
            }
        } else if (rank) {
            idx = b.last_idx_term[2 * g];
            term = b.last_idx_term[2 * g + 1];
        }
        const uint32_t gsz = group_size(st.cid);
        // ---- a5: poll_vote_count's tally
        if (vote) {
            const uint32_t s0 = st.cid.size[0], s1 = st.cid.size[1];
            const bool cnt = col && r < gsz && r != self && ack != st.len;
            const uint32_t c0 = (1u + (uint32_t)__builtin_popcount(rw_bits(cnt && r < s0, lane))) & 0xFFu;
            const uint32_t c1 = (1u + (uint32_t)__builtin_popcount(rw_bits(cnt && r < s1, lane))) & 0xFFu;
            const uint32_t voters = rw_bits(cnt, lane);
            // the first value of smallest distance, the commit first (larger() is strict)
            uint64_t d = cnt ? dist(st.end, st.len, ack) : ~0ull, v = ack;
            uint32_t ix = cnt ? r : 15u;
#pragma unroll
            for (int x = 1; x < 8; x <<= 1) {
                const uint64_t d2 = rw_xor(d, x), v2 = rw_xor(v, x);
                const uint32_t i2 = rw_xor(ix, x);
                if (d2 < d || (d2 == d && i2 < ix)) { d = d2; v = v2; ix = i2; }
            }
            const uint64_t vc = d < dist(st.end, st.len, st.commit) ? v : st.commit;
            bool won = c0 >= s0 / 2 + 1;
            if (won && st.cid.state != APUS_CID_STABLE) won = c1 >= s1 / 2 + 1;
            if (lead) {
                if (vo.won) vo.won[g] = won ? 1 : 0;
                if (vo.vote_count) { vo.vote_count[2 * g] = (uint8_t)c0; vo.vote_count[2 * g + 1] = (uint8_t)c1; }
                if (vo.new_commit) vo.new_commit[g] = vc;
                if (vo.voters) vo.voters[g] = (uint16_t)voters;
                acc[6] += won ? 1u : 0u;
            }
        }
        // ---- a6: poll_vote_requests' ranking
        if (rank) {
            uint8_t outcome;
            uint64_t new_sid = sid, nc0 = 0, nc1 = 0;
            uint32_t clr = 0;
            if (APUS_SID_L(sid)) {
                outcome = APUS_RANK_LEADER_KNOWN;
            } else {
                const uint32_t pl = (uint32_t)(sid & 0xFF);
                const uint64_t hv = rw_shfl(hbv, pl & 7u);
                const uint64_t h = pl < (uint32_t)NR ? hv : 0ull;
                if (h != 0 && APUS_SID_TERM(h) == APUS_SID_TERM(sid)) {
                    outcome = APUS_RANK_ADOPT_HB;
                    new_sid = h;
                } else {
                    const uint64_t old = sid | (1ull << 8);
                    // loop 1 (dare_server.c:1558-1578): a request at or below the
                    // best before it is cleared: an exclusive prefix maximum
                    const uint64_t rsv = r < gsz ? rs : 0ull;
                    const bool part = r < gsz && r != self;
                    uint64_t inc = part ? rsv : 0ull;
#pragma unroll
                    for (uint32_t s = 1; s < 8; s <<= 1) {
                        const uint64_t y = rw_up(inc, s);
                        if (r >= s && y > inc) inc = y;
                    }
                    uint64_t exc = rw_up(inc, 1u);
                    if (r == 0) exc = 0;
                    const uint64_t bb = exc > old ? exc : old;
                    const bool cl1 = part && bb >= rsv;
                    const uint64_t top = rw_shfl(inc, 7u);
                    const uint64_t best = top > old ? top : old;
                    const uint64_t rs2 = cl1 ? 0ull : rsv;
                    if (best == old) {
                        outcome = APUS_RANK_NO_BETTER;
                        clr = rw_bits(cl1, lane);
                    } else {
                        // loop 2 (:1622-1655): the chain of accepted requests, every
                        // request examined cleared
                        uint64_t hterm = APUS_SID_TERM(best), bsid = old, bidx = idx, bterm = term;
                        uint32_t bi = 0;
#pragma unroll
                        for (uint32_t i = 0; i < 8; ++i) {
                            const uint64_t si = rw_shfl(rs2, i), ti = rw_shfl(rt, i), xi = rw_shfl(ri, i);
                            if (i >= gsz || bsid > si) continue;
                            if (hterm < APUS_SID_TERM(si)) hterm = APUS_SID_TERM(si);
                            if (bterm > ti || (bterm == ti && bidx > xi)) continue;
                            bidx = xi;
                            bterm = ti;
                            bsid = si;
                            bi = i;
                        }
                        clr = gsz >= 8u ? 0xFFu : (1u << gsz) - 1u;
                        if (bsid == old) {
                            uint64_t s = sid;
                            s = (hterm << 9) | (s & 0x1FF);
                            s = (uint64_t)self | ((s >> 8) << 8);
                            new_sid = s;
                            outcome = APUS_RANK_RAISE_TERM;
                        } else {
                            new_sid = bsid;
                            if (lead) {
                                const uint64_t *cw = reinterpret_cast<const uint64_t *>(&b.vote_req[g * NR + bi].cid);
                                nc0 = cw[0];
                                nc1 = cw[1];
                            }
                            outcome = APUS_RANK_VOTE;
                        }
                    }
                }
            }
            if (lead) {
                if (ro.outcome) ro.outcome[g] = outcome;
                if (ro.new_sid) ro.new_sid[g] = new_sid;
                if (ro.new_cid) {
                    uint64_t *ow = reinterpret_cast<uint64_t *>(ro.new_cid + g);
                    ow[0] = nc0;
                    ow[1] = nc1;
                }
                if (ro.cleared) ro.cleared[g] = (uint16_t)clr;
            }
        }
    }
    block_partials<kTailStats, 1u << 5, false>(ra.rpart, acc);
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

// per-stream scratch (apus_internal.h): a buffer that must grow is freed
// only after the work already queued on its stream has drained
static hipError_t grow(hipStream_t s, void **p, size_t *cap, size_t want, size_t unit, bool zero_head)
{
    if (want <= *cap) return hipSuccess;
    if (*p) {
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
        (void)hipFree(*p);
    }
    *p = nullptr;
    *cap = 0;
    const size_t n = want + (zero_head ? 1 : 0);
    hipError_t e = hipMalloc(p, n * unit);
    if (e != hipSuccess) return e;
    *cap = want;
    return zero_head ? hipMemsetAsync(*p, 0, unit, s) : hipSuccess;
}

void ScratchPin::release()
{
    if (!sc) return;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        --sc->pins;
    }
    ctx->scr_cv.notify_all();
    sc = nullptr;
}

hipError_t stream_scratch(apus_ctx *ctx, hipStream_t s, size_t slots, uint64_t slow_groups, ScratchPin &pin)
{
    pin.release();
    std::unique_lock<std::mutex> lk(ctx->mu);
    StreamScratch *sc = nullptr;
    for (;;) {
        StreamScratch *free_slot = nullptr, *lru = nullptr;
        sc = nullptr;
        for (auto &x : ctx->scr) {
            if (x.used && x.stream == s) { sc = &x; break; }
            if (!x.used && !free_slot) free_slot = &x;
            if (x.used && !x.pins && !x.reclaiming && !x.growing && (!lru || x.last_use < lru->last_use)) lru = &x;
        }
        if (sc) {
            // the slot is being handed to this stream, or another call of
            // this stream holds the buffers this one must regrow: wait
            const bool regrow = slots > sc->partials_cap || slow_groups > sc->slow_cap || !sc->ticket;
            if (sc->reclaiming || sc->growing || (regrow && sc->pins)) { ctx->scr_cv.wait(lk); continue; }
            ++sc->pins;
            break;
        }
        if (free_slot) {
            sc = free_slot;
            *sc = StreamScratch{};
            sc->stream = s;
            sc->used = true;
            sc->pins = 1;
            break;
        }
        if (!lru) { ctx->scr_cv.wait(lk); continue; }    // 16 calls in flight on 16 other streams
        // every slot holds another stream: reclaim the least recently used
        // unpinned one once the work queued on it has drained (its stream may
        // since have been destroyed, so the device is synchronised, not the
        // stream; without holding the context lock); its buffers are kept
        sc = lru;
        sc->reclaiming = true;
        sc->stream = s;
        sc->pins = 1;
        lk.unlock();
        const hipError_t e = hipDeviceSynchronize();
        lk.lock();
        sc->reclaiming = false;
        ctx->scr_cv.notify_all();
        if (e != hipSuccess) {      // (the slot now belongs to this stream, unpinned)
            --sc->pins;
            return e;
        }
        break;
    }
    pin.ctx = ctx;
    pin.sc = sc;
    sc->last_use = ++ctx->scr_tick;
    if (slots <= sc->partials_cap && sc->ticket && (!slow_groups || slow_groups <= sc->slow_cap)) return hipSuccess;
    // regrow outside the context lock (grow synchronises the stream): every
    // other call of this slot waits on `growing`, no other slot is held up
    sc->growing = true;
    lk.unlock();
    hipError_t e = grow(s, (void **)&sc->partials, &sc->partials_cap, slots, sizeof(uint64_t), false);
    if (e == hipSuccess && !sc->ticket) {
        e = hipMalloc((void **)&sc->ticket, 64);
        if (e == hipSuccess) e = hipMemsetAsync(sc->ticket, 0, 64, s);
        else sc->ticket = nullptr;
    }
    if (e == hipSuccess && slow_groups)
        e = grow(s, (void **)&sc->slow, &sc->slow_cap, slow_groups, sizeof(uint32_t), true);
    lk.lock();
    sc->growing = false;
    ctx->scr_cv.notify_all();
    return e;
}

int resident_blocks(apus_ctx *ctx, int slot, const void *fn)
{
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        if (ctx->occ[slot]) return ctx->occ[slot];
    }
    int oc = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&oc, fn, 256, 0);
    if (oc <= 0) oc = 1;
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->occ[slot] = oc;
    return oc;
}

void free_scratch(apus_ctx *ctx)
{
    std::lock_guard<std::mutex> lk(ctx->mu);
    for (auto &x : ctx->scr) {
        if (x.partials) (void)hipFree(x.partials);
        if (x.slow) (void)hipFree(x.slow);
        if (x.ticket) (void)hipFree(x.ticket);
        x = StreamScratch{};
    }
}

typedef void (*commit_fn)(const apus_batch_t, const WalkOut, uint64_t *, uint32_t *, uint32_t *);

// Which walk kernel a batch takes: the lane-per-group kernel when asked for
// or when the ring array is not 16-B aligned (or strided past 4 GiB), else
// the segment kernel for short-walk batches, else the wave kernel
static bool walk_on_lanes(const apus_batch_t &b)
{
    const bool wave_ok = ((((uintptr_t)b.ring) | b.ring_stride) & 15u) == 0 && b.ring_stride < (1ull << 32);
    return (b.flags & APUS_BATCH_LANE_IMPL) || !wave_ok;
}
static bool walk_on_segments(const apus_batch_t &b)
{
    return !walk_on_lanes(b) && (b.flags & APUS_BATCH_SHORT_WALKS) != 0 && b.ring_stride <= kSegMaxStride;
}

// apus_commit_mark_walk's events, taken by the next walk launch on any stream
static void take_walk_events(apus_ctx *ctx, hipEvent_t *ev)
{
    std::lock_guard<std::mutex> lk(ctx->mu);
    ev[0] = (hipEvent_t)ctx->walk_ev[0];
    ev[1] = (hipEvent_t)ctx->walk_ev[1];
    ctx->walk_ev[0] = ctx->walk_ev[1] = nullptr;
}

// apus_commit_mark_tail's events, taken by the next tail launch
static void take_tail_events(apus_ctx *ctx, hipEvent_t *ev)
{
    std::lock_guard<std::mutex> lk(ctx->mu);
    ev[0] = (hipEvent_t)ctx->tail_ev[0];
    ev[1] = (hipEvent_t)ctx->tail_ev[1];
    ctx->tail_ev[0] = ctx->tail_ev[1] = nullptr;
}

// the walk kernel of a commit call: commit_wave_kernel (persistent, one wave
// per group), commit_seg_kernel (APUS_BATCH_SHORT_WALKS: four groups per
// wave) or commit_lane_kernel (APUS_BATCH_LANE_IMPL, unaligned rings), and
// the scratch its tail needs: *wblk x *wstat block partials at
// sc->partials[0..], then tblk x kTailStats rows for quorum_tail_kernel;
// *slow is the deferred list (NULL for the lane kernel, which defers
// nothing).  epi & kEpiNc: the walk writes the NC determinants.
// The walk kernel a commit call launches and its grid (launch_walk; also
// apus_commit_walk_info): kind 0 lane, 1 wave, 2 segment; hop: the wave
// kernel's hop walk; dyn: blocks handed out by the counter
struct WalkPlan {
    uint32_t kind, hop, dyn, grid, slot;
    bool rows;
    commit_fn fn;
};

static WalkPlan walk_plan(apus_ctx *ctx, const apus_batch_t &b, bool ck, uint32_t &epi, bool lit)
{
    WalkPlan p{};
    if (walk_on_lanes(b)) {
        p.kind = 0;
        p.grid = grid_for(b.n_groups, 256, ctx->n_cu, 8);
        return p;
    }
    // APUS_BATCH_SHORT_WALKS: four groups per wave (commit_seg_kernel)
    const bool sh = walk_on_segments(b);
    p.kind = sh ? 2u : 1u;
    // APUS_BATCH_VAR_LEN: the wave kernel with the hop walk
    const bool hp = !sh && (b.flags & APUS_BATCH_VAR_LEN) != 0;
    if (sh || !ck) epi = 0;
    const bool nc = (epi & kEpiNc) != 0;
    // (the segment kernel records the last determinants' offsets on checksum walks)
    const bool rows = sh && ck && lit;
#define APUS_WALK_FN(D)                                                                                               \
    (sh ? (ck ? (rows ? commit_seg_kernel<true, true, D> : commit_seg_kernel<true, false, D>)                          \
            : commit_seg_kernel<false, false, D>)                                                                    \
        : hp ? (ck ? (nc ? commit_wave_kernel<true, kWinHop, true, kEpiNc, D> : commit_wave_kernel<true, kWinHop, true, 0, D>) \
                   : commit_wave_kernel<false, kWinHop, true, 0, D>)                                                 \
             : (ck ? (nc ? commit_wave_kernel<true, kWin, false, kEpiNc, D> : commit_wave_kernel<true, kWin, false, 0, D>) \
                   : commit_wave_kernel<false, kWin, false, 0, D>))
    const commit_fn fn_st = APUS_WALK_FN(false), fn_dy = APUS_WALK_FN(true);
#undef APUS_WALK_FN
    const int slot = ((ck ? 1 : 0) + (sh ? 2 : hp ? 4 : 0)) * 2 + ((nc || rows) ? 1 : 0);
    int oc;
    {
        std::lock_guard<std::mutex> lk(ctx->mu);
        oc = ctx->occ[slot];
    }
    if (!oc) {
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&oc, fn_st, 256, 0);
        if (oc <= 0) oc = 2;
        std::lock_guard<std::mutex> lk(ctx->mu);
        ctx->occ[slot] = oc;
    }
    const uint32_t grid = grid_for(sh ? (b.n_groups + kNSeg - 1) / kNSeg : b.n_groups, kWaves, ctx->n_cu,
                                   (uint32_t)oc);
    // blocks of 64 groups handed out by a counter once there are >= 8 per wave,
    // on checksum walks (walk-only segment walks measured 11% slower with it:
    // their quads are too short to hide the counter's round trip)
    const uint64_t bs = sh ? 64u : kWB;
    const uint64_t nblk = (b.n_groups + bs - 1) / bs;
    p.dyn = (ck && nblk >= (uint64_t)8 * grid * kWaves) ? 1u : 0u;
    p.fn = p.dyn ? fn_dy : fn_st;
    p.hop = hp ? 1u : 0u;
    p.grid = grid;
    p.rows = rows;
    return p;
}

static hipError_t launch_walk(apus_ctx *ctx, const apus_batch_t &b, const apus_commit_out_t &o, bool ck,
                              uint32_t epi, bool lit, uint32_t tblk, uint64_t nslow, hipStream_t s, ScratchPin &pin,
                              uint32_t *wblk, uint32_t *wstat, uint32_t **slow)
{
    hipEvent_t ev[2];
    take_walk_events(ctx, ev);
    hipError_t e;
    const WalkPlan p = walk_plan(ctx, b, ck, epi, lit);
    if (p.kind == 0) {
        const uint32_t grid = p.grid;
        if ((e = stream_scratch(ctx, s, (size_t)grid * kCommitStats + (size_t)tblk * kTailStats, 0, pin)) != hipSuccess)
            return e;
        StreamScratch *sc = pin.sc;
        // (lane_group writes the NC determinants with its own exact walk)
        WalkOut ol = walk_out(o);
        if (!(epi & kEpiNc)) { ol.nc_dets = nullptr; ol.nc_len = nullptr; }
        // (the events, when given, take the kernel's own start and end
        // timestamps: no marker packets between the launches)
        hipExtLaunchKernelGGL(ck ? commit_lane_kernel<true> : commit_lane_kernel<false>, dim3(grid), dim3(256), 0, s,
                              ev[0], ev[1], 0u, b, ol, sc->partials);
        *wblk = grid; *wstat = kCommitStats; *slow = nullptr;
        return hipGetLastError();
    }
    if ((e = stream_scratch(ctx, s, (size_t)p.grid * kWaveStats + (size_t)tblk * kTailStats, nslow, pin)) != hipSuccess)
        return e;
    StreamScratch *sc = pin.sc;
    hipExtLaunchKernelGGL(p.fn, dim3(p.grid), dim3(256), 0, s, ev[0], ev[1], 0u, b, walk_out(o), sc->partials, sc->slow,
                          sc->ticket + 1);
    *wblk = p.grid; *wstat = kWaveStats; *slow = sc->slow;
    return hipGetLastError();
}

hipError_t commit_walk_info(apus_ctx *ctx, const apus_batch_t &b, uint32_t flags, uint32_t *info)
{
    const bool ck = (flags & APUS_COMMIT_CHECKSUM) != 0;
    uint32_t epi = (flags & APUS_COMMIT_NC) ? kEpiNc : 0u;
    const WalkPlan p = walk_plan(ctx, b, ck, epi, (flags & APUS_COMMIT_LAST_IT) != 0);
    info[0] = p.kind;
    info[1] = p.hop;
    info[2] = p.dyn;
    info[3] = p.grid;
    info[4] = (epi & kEpiNc) ? 1u : 0u;
    info[5] = p.rows ? 1u : 0u;
    return hipSuccess;
}

hipError_t launch_commit(apus_ctx *ctx, const apus_batch_t &b, const apus_commit_out_t &o,
                         uint32_t flags, hipStream_t s)
{
    if (b.n_groups == 0) return hipSuccess;
    const bool ck = (flags & APUS_COMMIT_CHECKSUM) != 0;
    const bool walk = (flags & (APUS_COMMIT_WALK | APUS_COMMIT_CHECKSUM)) != 0;
    const bool want_med = (flags & APUS_COMMIT_MEDIAN) && o.median;
    const bool want_pr = (flags & APUS_COMMIT_PRUNE) != 0;
    const bool want_nc = (flags & APUS_COMMIT_NC) && o.nc_dets && o.nc_len;
    const bool want_lit = (flags & APUS_COMMIT_LAST_IT) && o.last_idx_term;
    const bool want_vote = (flags & APUS_COMMIT_VOTE) != 0, want_rank = (flags & APUS_COMMIT_RANK) != 0;
    const bool want_pub = (flags & APUS_COMMIT_PUBLISH) != 0, want_force = (flags & APUS_COMMIT_FORCE_PRUNE) != 0;
    const bool fail = want_vote || want_rank;
    const bool fresh = (flags & APUS_COMMIT_STATS_FRESH) != 0;
    if (!walk && !want_med && !want_pr && !want_lit && !fail && !fresh && !want_pub && !want_force) {
        if (want_nc) return launch_nc_build(ctx, b, o.nc_dets, o.nc_max, o.nc_len, s);
        return hipSuccess;
    }
    // the NC determinants come from the walk itself when it checksums (the
    // wave and lane kernels; not the segment kernel), else from their own launch
    const bool sh = walk_on_segments(b), lane = walk_on_lanes(b);
    const uint32_t epi = walk && want_nc && (lane || (ck && !sh)) ? kEpiNc : 0u;
    // the tail's grid: 4 blocks per CU (all resident at once for the C2 set;
    // 8 measured 53 vs 44 us at C2, 16 75 us; the 64M-group and C5 tails
    // the same within noise: profiles/r04/tail_grid/ab_tgrid.log)
    uint32_t tblk = grid_for(b.n_groups, 256, ctx->n_cu, 4);
    const uint32_t R = b.n_replicas;
    // the flags of the tail
    const bool pruning = (want_pr && !want_force) || want_force;   // log_pruning's, or force_log_pruning's
    const uint32_t tflags = (want_med ? kTailMed : 0u) | (want_pr && !want_force ? kTailPrune : 0u) |
                            (pruning && b.abs_base ? kTailWm : 0u) | (pruning && b.prev_head ? kTailPrev : 0u) |
                            (fresh ? kTailFresh : 0u) | (want_lit ? kTailLit : 0u) |
                            (want_lit && walk && sh && ck ? kTailLitRows : 0u) | (want_vote ? kTailVote : 0u) |
                            (want_rank ? kTailRank : 0u) | (want_pub ? kTailPub : 0u) |
                            (want_force ? kTailForce : 0u) | ((want_pub || want_force) && walk ? kTailWalked : 0u);
    const uint32_t set = tflags & ~kTailFresh;
    const bool fast_set = ck && (R == 3 || R == 5 || R == 7) &&
                          (set == kTailSetC2 || set == kTailSetC5 || set == kTailSetC2P || set == kTailSetC5P);
    // APUS_BATCH_TAIL_ROWS: eight lanes per group (quorum_row_kernel), then
    // the list launch, for the bench sets behind a wave or segment walk (its
    // deferred list carries the groups the row kernel hands over: up to 2 G
    // entries); measured slower than one lane per group
    const bool rows = fast_set && walk && !lane && (b.flags & APUS_BATCH_TAIL_ROWS) && b.n_groups < (1ull << 31);
    typedef void (*row_fn)(const apus_batch_t, const WalkOut, const apus_vote_out_t, const apus_rank_out_t,
                           const TailOut2, const RowArgs);
    row_fn rf = nullptr;
    uint32_t rblk = 0;
    if (rows) {
#define APUS_ROW_SET(S) \
    (R == 3 ? quorum_row_kernel<3, S> : R == 5 ? quorum_row_kernel<5, S> : quorum_row_kernel<7, S>)
        rf = set == kTailSetC2    ? APUS_ROW_SET(kTailSetC2)
             : set == kTailSetC5  ? APUS_ROW_SET(kTailSetC5)
             : set == kTailSetC2P ? APUS_ROW_SET(kTailSetC2P)
                                  : APUS_ROW_SET(kTailSetC5P);
#undef APUS_ROW_SET
        // the grid: every block resident (occ slots 48..59: set x R)
        const int slot = 48 +
                         3 * (set == kTailSetC2    ? 0
                              : set == kTailSetC5  ? 1
                              : set == kTailSetC2P ? 2
                                                   : 3) +
                         (R == 3 ? 0 : R == 5 ? 1 : 2);
        rblk = grid_for(b.n_groups, 32, ctx->n_cu, (uint32_t)resident_blocks(ctx, slot, (const void *)rf));
    }
    if (rows) tblk = grid_for(b.n_groups, 256, ctx->n_cu, 1);
    hipError_t e;
    ScratchPin pin;
    uint32_t wblk = 0, wstat = 0, *slow = nullptr;
    if (walk) {
        if ((e = launch_walk(ctx, b, o, ck, epi, want_lit, tblk + rblk, rows ? 2 * b.n_groups : b.n_groups, s, pin,
                             &wblk, &wstat, &slow)) != hipSuccess) {
            // a walk that was queued leaves its block counter (ticket word 1)
            // for the tail's last block to reset: without the tail, reset it here
            if (pin.sc && pin.sc->ticket) (void)hipMemsetAsync(pin.sc->ticket, 0, 8, s);
            if (pin.sc && pin.sc->slow) (void)hipMemsetAsync(pin.sc->slow, 0, sizeof(uint32_t), s);
            return e;
        }
    } else if ((e = stream_scratch(ctx, s, (size_t)tblk * kTailStats, 0, pin)) != hipSuccess) {
        return e;
    }
    StreamScratch *sc = pin.sc;
    // one tail launch: deferred walks, median, pruning and the statistics fold
    TailArgs t;
    t.slow = slow;
    t.wpart = walk ? sc->partials : nullptr;
    t.wblk = wblk;
    t.wstat = wstat;
    t.tpart = sc->partials + (size_t)wblk * wstat;
    t.ticket = sc->ticket;
    t.stats = ctx->stats;
    t.slow_reset = slow;
    t.flags = tflags;
    t.rpart = nullptr;
    t.rblk = 0;
    TailOut2 o2;
    o2.publish = want_pub ? o.publish : nullptr;
    o2.ssn = want_pub ? o.ssn : nullptr;
    if (want_force) o2.force = o.force;
    else memset(&o2.force, 0, sizeof o2.force);
    // the deferred walks write the NC determinants only when the walk kernel
    // writes them for the others
    WalkOut ot = walk_out(o);
    if (!(epi & kEpiNc)) { ot.nc_dets = nullptr; ot.nc_len = nullptr; }
    // sort slots N (8, or 16 beyond 8 replicas); inputs loaded for NR = R
    // replicas where R is 3, 5 or 7
    typedef void (*tail_fn)(const apus_batch_t, const WalkOut, const TailArgs, const apus_vote_out_t,
                            const apus_rank_out_t, const TailOut2);
    // (the failover pass is its own instantiation: its columns would cost
    // every other tail registers)
#define APUS_TAIL_FN(F)                                                                                   \
    (R > 8 ? (ck ? quorum_tail_kernel<16, 16, true, F, 0> : quorum_tail_kernel<16, 16, false, F, 0>)      \
     : R == 3 ? (ck ? quorum_tail_kernel<8, 3, true, F, 0> : quorum_tail_kernel<8, 3, false, F, 0>)       \
     : R == 5 ? (ck ? quorum_tail_kernel<8, 5, true, F, 0> : quorum_tail_kernel<8, 5, false, F, 0>)       \
     : R == 7 ? (ck ? quorum_tail_kernel<8, 7, true, F, 0> : quorum_tail_kernel<8, 7, false, F, 0>)       \
              : (ck ? quorum_tail_kernel<8, 8, true, F, 0> : quorum_tail_kernel<8, 8, false, F, 0>))
    tail_fn fn = fail ? APUS_TAIL_FN(true) : APUS_TAIL_FN(false);
#undef APUS_TAIL_FN
    // the bench configurations' flag sets (checksum walks; R = 3, 5, 7):
    // their own instantiations, every flag a constant
    if (fast_set) {
#define APUS_TAIL_SET(S, F)                                                                                 \
    (R == 3 ? quorum_tail_kernel<8, 3, true, F, S> : R == 5 ? quorum_tail_kernel<8, 5, true, F, S>          \
            : quorum_tail_kernel<8, 7, true, F, S>)
        fn = set == kTailSetC2    ? APUS_TAIL_SET(kTailSetC2, false)
             : set == kTailSetC5  ? APUS_TAIL_SET(kTailSetC5, true)
             : set == kTailSetC2P ? APUS_TAIL_SET(kTailSetC2P, false)
                                  : APUS_TAIL_SET(kTailSetC5P, true);
#undef APUS_TAIL_SET
    }
    // the failover outputs are read only when their flags are set (a caller
    // built against an older, shorter apus_commit_out_t never sets them)
    apus_vote_out_t vo;
    apus_rank_out_t ro;
    memset(&vo, 0, sizeof vo);
    memset(&ro, 0, sizeof ro);
    if (want_vote) vo = o.vote;
    if (want_rank) ro = o.rank;
    if (rows) {
        RowArgs ra;
        ra.list = slow;
        ra.rpart = t.tpart;
        hipLaunchKernelGGL(rf, dim3(rblk), dim3(256), 0, s, b, ot, vo, ro, o2, ra);
        if ((e = hipGetLastError()) != hipSuccess) {
            (void)hipMemsetAsync(sc->ticket, 0, 8, s);
            (void)hipMemsetAsync(slow, 0, sizeof(uint32_t), s);
            return e;
        }
        // the list launch: its rows after the row kernel's
        t.rpart = t.tpart;
        t.rblk = rblk;
        t.tpart += (size_t)rblk * kTailStats;
        t.flags |= kTailList;
    }
    // (apus_commit_mark_tail: the kernel's own start and end timestamps)
    hipEvent_t tev[2];
    take_tail_events(ctx, tev);
    hipExtLaunchKernelGGL(fn, dim3(tblk), dim3(256), 0, s, tev[0], tev[1], 0u, b, ot, t, vo, ro, o2);
    if ((e = hipGetLastError()) != hipSuccess) {
        // the tail resets the arrival ticket and the walk's block counter:
        // a tail that did not launch leaves both to be reset here
        (void)hipMemsetAsync(sc->ticket, 0, 8, s);
        if (slow) (void)hipMemsetAsync(slow, 0, sizeof(uint32_t), s);
        return e;
    }
    pin.release();
    if (want_nc && !(epi & kEpiNc)) return launch_nc_build(ctx, b, o.nc_dets, o.nc_max, o.nc_len, s);
    return hipSuccess;
}

}  // namespace apus


