// Election / pruning / log-adjustment kernels for gfx950 (MI355X).
//
//   vote_tally_kernel   lane per group   poll_vote_count tally,
//                                        src/dare/dare_server.c:1327-1373
//   vote_rank_kernel    lane per group   poll_vote_requests ranking / up-to-date
//                                        test, dare_server.c:1526-1655
//   prune_kernel        lane per group   log_pruning minimum, dare_server.c:2026-2058
//                                        (+ log_get_tail, dare_log.h:402-457)
//   validate_kernel     wave per group   log_find_remote_end_offset,
//                                        dare_log.h:367-394: lane k checks NC
//                                        determinant k, ballot -> first mismatch
//   nc_build_kernel     lane per group   log_entries_to_nc_buf, dare_log.h:339-359
//   last_idx_term_kernel lane per group  local (idx, term), dare_server.c:1598-1620
//   lr_completion_kernel 4 (group, server) pairs per lane: handle_lr_work_completion,
//                                        dare_ibv_rc.c:3126-3196
//   log_adjust_kernel   lane per group   log_adjustment, dare_ibv_rc.c:1292-1451; LR_SET_END
//                                        walks wave-cooperative (lanes over determinants)
//
// Control data is tiny per group (R <= 13 replicas); these kernels are
// HBM-bound streams over [G][R] arrays: one lane per group, per-replica loops
// fully unrolled over a compile-time bound so every array stays in registers.
#include "apus_device.h"
#include "apus_group_ops.h"
#include "apus_internal.h"
#include "apus_stats.h"

namespace apus {

constexpr int kMaxR = 16;

// ---------------------------------------------------------------------------
// vote_of / rank_of (apus_group_ops.h) over N replica slots (EXACT: R == N)
template <int N, bool EXACT>
__global__ void __launch_bounds__(256) vote_tally_kernel(const apus_batch_t b, const apus_vote_out_t o,
                                                         uint64_t *partials)
{
    uint64_t won_cnt[1] = { 0 };
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        FailIn<N> f;
        load_fail_in<N, EXACT>(b, g, true, false, f);
        const apus_group_state_t st = load_state(b, g);
        won_cnt[0] += vote_from<N, EXACT>(b, g, st, b.self_idx[g], f, o) ? 1 : 0;
    }
    block_partials<1>(partials, won_cnt);
}

// ---------------------------------------------------------------------------
template <int N, bool EXACT>
__global__ void __launch_bounds__(256) vote_rank_kernel(const apus_batch_t b, const apus_rank_out_t o,
                                                        const uint64_t *lit)
{
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        FailIn<N> f;
        load_fail_in<N, EXACT>(b, g, false, true, f);
        const apus_group_state_t st = load_state(b, g);
        rank_from<N, EXACT>(b, g, st, b.self_idx[g], lit[2 * g], lit[2 * g + 1], f, o);
    }
}

// ---------------------------------------------------------------------------
template <int N>
__global__ void __launch_bounds__(256) prune_kernel(const apus_batch_t b, const apus_prune_out_t o,
                                                    uint64_t *partials)
{
    uint64_t wm[1] = { ~0ull };
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const apus_group_state_t st = load_state(b, g);
        QuorumIn<N> q;
        load_quorum_in<N, false>(b, g, false, true, b.prev_head != nullptr, b.abs_base != nullptr, q);
        const uint64_t w = prune_of<N>(b, g, st, q, o.new_head, o.append_head, o.min_apply);
        wm[0] = w < wm[0] ? w : wm[0];
    }
    block_partials<1, 1u>(partials, wm);
}

// ---------------------------------------------------------------------------
// validate_kernel: log_find_remote_end_offset (dare_log.h:367-394) for every
// follower of a group at once.  One wave per group; lane k checks determinant
// base + k of kValFB followers per pass, their determinant loads issued back
// to back.  The leader's (idx, term) at a determinant's offset is gathered
// once per distinct offset: a follower that replicates the leader's log
// carries the offsets of the pass's first follower, so its check reuses that
// gather.  Entry lengths are read only where a follower's last determinant
// sits.  The next group's NC lengths are requested while this group's leader
// headers are in flight, so a group costs two dependent round trips per
// 64 determinants (determinants, then leader headers).
// Deviations (undefined in the reference): det_len above max_dets reads
// max_dets determinants; an empty buffer whose follower index is not below
// n_replicas yields 0 (no remote_commit column to read).
// ---------------------------------------------------------------------------
#ifndef APUS_VAL_FB
#define APUS_VAL_FB 4
#endif
#ifndef APUS_VAL_WPE
#define APUS_VAL_WPE 6
#endif
constexpr uint32_t kValFB = APUS_VAL_FB;   // followers per pass

__device__ __forceinline__ uint64_t rl64(uint64_t x, uint32_t k)
{
    return ((uint64_t)__builtin_amdgcn_readlane((uint32_t)(x >> 32), k) << 32) |
           __builtin_amdgcn_readlane((uint32_t)x, k);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(APUS_VAL_WPE))) validate_kernel(const apus_batch_t b, const apus_nc_batch_t nc,
                                                       uint64_t *out, uint64_t *partials)
{
    const uint32_t lane = lane_id();
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint32_t F = nc.n_followers, M = nc.max_dets, R = b.n_replicas;
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    uint64_t mism = 0;
    // lane f < F: follower f's NC length, clamped to the row
    auto load_len = [&](uint64_t gg) -> uint32_t {
        if (gg >= b.n_groups || lane >= F) return 0u;
        const uint32_t n = nc.det_len[gg * F + lane];
        return n < M ? n : M;
    };
    // the leader's determinant count, clamped (0 without leader_dets)
    auto load_lead = [&](uint64_t gg) -> uint32_t {
        if (!nc.leader_dets || gg >= b.n_groups) return 0u;
        const uint32_t n = nc.leader_len[gg];
        return n < nc.leader_max ? n : nc.leader_max;
    };
    uint64_t g = (uint64_t)blockIdx.x * 4 + wv;
    uint32_t nl = load_len(g), lead_nx = load_lead(g);
    for (; g < b.n_groups; g += nw) {
        const apus_group_state_t st = load_state(b, g);
        const RingView v = ring_view(b, g, st);
        const uint64_t gF = g * F;
        // requested with the previous group's gathers (one round trip less)
        const uint32_t lead_n = lead_nx;
        uint64_t myres = 0;                 // lane f: follower f's remote end
        uint32_t nl_next = 0;
        bool next_req = false;
        // empty buffers: the caller's rule, end = log_offsets[i].commit (dare_ibv_rc.c:1378-1384)
        if (lane < F && nl == 0) {
            const uint32_t fol = nc.follower[gF + lane];
            myres = fol < R ? b.remote_commit[g * R + fol] : 0ull;
        }
        for (uint32_t fb = 0; fb < F; fb += kValFB) {
            uint32_t n[kValFB];
            uint32_t pend = 0, nmax = 0;
#pragma unroll
            for (uint32_t j = 0; j < kValFB; ++j) {
                n[j] = fb + j < F ? __builtin_amdgcn_readlane(nl, fb + j) : 0u;
                if (n[j]) pend |= 1u << j;
                nmax = n[j] > nmax ? n[j] : nmax;
            }
            uint64_t res[kValFB] = {};
            for (uint32_t base = 0; pend && base < nmax; base += 64) {
                const uint32_t k = base + lane;
                // the leader's own determinant k (nc.leader_dets): a follower
                // determinant at its offset is checked against it, no gather
                const bool lead_ok = k < lead_n;              // lead_n == 0 without leader_dets
                apus_entry_det_t ld = { 0, 0, 0 };
                if (lead_ok) ld = nc.leader_dets[g * nc.leader_max + k];
                apus_entry_det_t det[kValFB];
                bool live[kValFB];
#pragma unroll
                for (uint32_t j = 0; j < kValFB; ++j) {
                    live[j] = ((pend >> j) & 1u) && k < n[j];
                    det[j] = { 0, 0, 0 };
                    if (live[j]) det[j] = nc.dets[(gF + fb + j) * M + k];
                }
                if (!next_req) {          // overlap the next group's lengths with the gathers
                    nl_next = load_len(g + nw);
                    lead_nx = load_lead(g + nw);
                    next_req = true;
                }
                uint64_t off[kValFB], li[kValFB], lt[kValFB];
                uint32_t el[kValFB];
                bool ok[kValFB], hit[kValFB];
#pragma unroll
                for (uint32_t j = 0; j < kValFB; ++j) {
                    off[j] = det[j].offset;
                    // the leader recorded an entry at exactly this offset (its
                    // header fits there: get_entry leaves the offset as it is)
                    hit[j] = lead_ok && live[j] && off[j] == ld.offset;
                    ok[j] = hit[j] || (live[j] && v.get_entry(off[j]));
                    li[j] = hit[j] ? ld.idx : 0;
                    lt[j] = hit[j] ? ld.term : 0;
                    el[j] = 0;
                }
#pragma unroll
                for (uint32_t j = 0; j < kValFB; ++j) {
                    const bool dup = j > 0 && ok[0] && off[j] == off[0];
                    if (ok[j] && !dup && !hit[j]) ld_idx_term(v.ring + off[j], li[j], lt[j]);
                    if (ok[j] && k + 1 == n[j]) el[j] = v.elen_at(off[j]);
                }
#pragma unroll
                for (uint32_t j = 1; j < kValFB; ++j)
                    if (ok[j] && ok[0] && off[j] == off[0]) { li[j] = li[0]; lt[j] = lt[0]; }
#pragma unroll
                for (uint32_t j = 0; j < kValFB; ++j) {
                    if (!((pend >> j) & 1u)) continue;
                    const bool bad = live[j] && (!ok[j] || li[j] != det[j].idx || lt[j] != det[j].term);
                    const uint64_t bb = __ballot(bad);
                    if (bb) {
                        res[j] = rl64(off[j], (uint32_t)__builtin_ctzll(bb));
                        pend &= ~(1u << j);
                        mism += 1;
                    } else if (base + 64 >= n[j]) {
                        const uint64_t nx = (v.len - off[j] < el[j] ? 0 : off[j]) + el[j];
                        res[j] = rl64(nx, n[j] - 1 - base);
                        pend &= ~(1u << j);
                    }
                }
            }
#pragma unroll
            for (uint32_t j = 0; j < kValFB; ++j)
                if (n[j] && lane == fb + j) myres = res[j];
        }
        if (lane < F) out[gF + lane] = myres;
        if (!next_req) lead_nx = load_lead(g + nw);
        nl = next_req ? nl_next : load_len(g + nw);
    }
    uint64_t mine[1] = { lane == 0 ? mism : 0 };
    block_partials<1>(partials, mine);
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) nc_build_kernel(const apus_batch_t b, apus_entry_det_t *dets,
                                                       uint32_t max_dets, uint32_t *len)
{
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const apus_group_state_t st = load_state(b, g);
        const RingView v = ring_view(b, g, st);
        apus_entry_det_t *out = dets + g * max_dets;
        uint64_t o = st.commit;
        uint32_t n = 0;
        while (n < max_dets && v.get_entry(o)) {
            const uint8_t *e = v.ring + o;
            apus_entry_det_t d;
            ld_idx_term(e, d.idx, d.term);
            d.offset = o;
            out[n++] = d;
            const uint32_t el = entry_len(e[kType], ld_u16(e + kData));
            if (v.len - o < el) o = 0;
            o += el;
        }
        len[g] = n;
    }
}

// ---------------------------------------------------------------------------
// nc_build_seg_kernel: log_entries_to_nc_buf with 16 lanes per group (four
// groups per wave), speculatively as commit_seg_kernel walks: lane j takes
// the entry at o + j*el (el the last entry's length) and the segment's ballot
// bits confirm the longest prefix of entries of that length that are in the
// walk (get_entry: not end, header in the ring) and need no jump, plus the
// first entry that breaks the run -- another length, or a ghost header, which
// log_entries_to_nc_buf records at its own offset before jumping to 0.  The
// confirmed lanes write their determinants side by side (16 x 24 B), so a
// log of equal-size entries (C2, C5) advances 16 entries per wave step; the
// header wrap is taken at the segment's first entry, as the walk does.
// ---------------------------------------------------------------------------
template <uint32_t W>
__device__ __forceinline__ uint32_t segw(uint64_t ballot, uint32_t seg)
{
    return (uint32_t)(ballot >> (W * seg)) & (uint32_t)((1ull << W) - 1ull);
}

// W lanes per group (16 in the product build)
// (The same segment walk for the local last (idx, term), which writes
// nothing per entry, measured slower than last_idx_term_kernel's lane walk:
// C2 1.54 vs 1.47 ms, C5 1.65 vs 1.52 ms, C3 5.0 vs 0.42 ms.)
template <uint32_t W>
__global__ void __launch_bounds__(256) nc_build_seg_kernel(const apus_batch_t b, apus_entry_det_t *dets,
                                                           uint32_t max_dets, uint32_t *len)
{
    constexpr uint32_t kSh = W == 16 ? 4 : W == 8 ? 3 : 2;
    const uint32_t lane = lane_id();
    const uint32_t seg = lane >> kSh, sl = lane & (W - 1u);
    const uint64_t nseg = (uint64_t)gridDim.x * (blockDim.x >> kSh);
    for (uint64_t g0 = ((uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) >> kSh; g0 < b.n_groups;
         g0 += nseg) {
        const uint64_t g = g0 + seg;
        const bool live = g < b.n_groups;
        apus_group_state_t st = {};
        if (live) st = load_state(b, g);
        const uint64_t end = st.end, ln = st.len;
        const uint8_t *ring = b.ring + (live ? g : 0) * b.ring_stride;
        apus_entry_det_t *out = dets + (live ? g : 0) * max_dets;
        uint64_t o = st.commit;
        uint32_t n = 0, elg = 128;
        const uint64_t cap = max_dets, rcap = ring_cap(b);
        bool done = !live || cap == 0;
        while (__ballot(!done)) {
            // log_get_entry at the segment's first entry (dare_log.h:316-332)
            if (!done) {
                if (end == ln || dist(end, ln, o) == 0) done = true;
                else {
                    if (ln - o < kHdr) o = 0;
                    if (!(ln >= kHdr && o <= ln - kHdr && rcap >= kHdr && o <= rcap - kHdr))
                        done = true;                               // past the ring (RingView::get_entry)
                }
            }
            const uint64_t p = o + (uint64_t)sl * elg;
            const bool in = !done && n + sl < cap && p <= ln && ln - p >= kHdr && p + kHdr <= rcap &&
                            (sl == 0 || p != end);
            uint64_t idx = 0, term = 0;
            uint32_t el = 0;
            if (in) {
                const uint8_t *e = ring + p;
                ld_idx_term(e, idx, term);
                el = entry_len(e[kType], ld_u16(e + kData));
            }
            const bool ghost = in && ln - p < el;               // !log_fit_entry: the walk jumps to 0
            const bool cont = in && !ghost && el == elg && sl < W - 1u;
            const uint32_t inb = segw<W>(__ballot(in), seg);
            const uint32_t fb = (uint32_t)__builtin_ctz(segw<W>(__ballot(!cont), seg) | (1u << W));
            const uint32_t nconf = fb + ((inb >> fb) & 1u);
            if (!done && sl < nconf) {
                uint64_t *d = reinterpret_cast<uint64_t *>(out + n + sl);
                d[0] = idx;
                d[1] = term;
                d[2] = p;
            }
            if (!done) {
                if (nconf == 0) {
                    done = true;                                   // max_dets reached
                } else {
                    const uint32_t last = (lane & ~(W - 1u)) + nconf - 1u;
                    const uint64_t p_last = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(p >> 32), last) << 32) |
                                            (uint32_t)__shfl((int)(uint32_t)p, last);
                    const uint32_t el_last = __shfl(el, last);
                    const bool gh_last = __shfl(ghost ? 1 : 0, last) != 0;
                    o = (gh_last ? 0 : p_last) + el_last;
                    elg = el_last;
                    n += nconf;
                }
            }
        }
        if (live && sl == 0) len[g] = n;
    }
}

// ---------------------------------------------------------------------------
// nc_build_quad_kernel: log_entries_to_nc_buf with FOUR lanes per group.  Per
// entry the quad reads the 64 B from the header's 16-B aligned base with one
// 16-B load per lane (plus a fifth piece when the header starts at 15 mod 16),
// parks them in LDS and every lane takes idx, term, type and cmd.len from
// there.  The lane-per-group walk issues four to eight narrow loads per
// entry, each its own request to a different line; here a wave instruction
// covers 16 headers with one or two 64-B requests each.
// ---------------------------------------------------------------------------
constexpr uint32_t kQuadSlot = 80;          // LDS bytes per group: 5 pieces of 16 B

__device__ __forceinline__ uint32_t lds_u32_at(const uint8_t *p, uint32_t off)
{
    const uint32_t *w = reinterpret_cast<const uint32_t *>(p + (off & ~3u));
    return __builtin_amdgcn_alignbyte(w[1], w[0], off & 3u);
}

__global__ void __launch_bounds__(256) nc_build_quad_kernel(const apus_batch_t b, apus_entry_det_t *dets,
                                                            uint32_t max_dets, uint32_t *len)
{
    __shared__ __attribute__((aligned(16))) uint8_t s_hdr[256 / 4][kQuadSlot];
    const uint32_t sub = threadIdx.x & 3u;
    uint8_t *slot = s_hdr[threadIdx.x >> 2];
    const uint64_t nq = (uint64_t)gridDim.x * 64u;
    for (uint64_t g0 = (uint64_t)blockIdx.x * 64u; g0 < b.n_groups; g0 += nq) {
        const uint64_t g = g0 + (threadIdx.x >> 2);
        const bool live = g < b.n_groups;
        apus_group_state_t st = {};
        if (live) st = load_state(b, g);
        const RingView v = ring_view(b, live ? g : 0, st);
        apus_entry_det_t *out = dets + (live ? g : 0) * max_dets;
        uint64_t o = st.commit;
        uint32_t n = 0;
        bool go = live;
        // the quad's lanes hold the same walk state; the loop runs until every
        // quad of the wave is done
        while (__ballot(go)) {
            if (go) go = n < max_dets && v.get_entry(o);
            uint4 pc = make_uint4(0, 0, 0, 0), p4 = pc;
            const uint8_t *e = v.ring + o;
            const uintptr_t base = (uintptr_t)e & ~(uintptr_t)15;
            const uint32_t r = (uint32_t)((uintptr_t)e & 15u);
            // cmd.len's second byte lies in a fifth piece when r == 15; near the
            // end of the ring array that piece is replaced by the byte itself
            const bool p4_ok = base + 80u <= (uintptr_t)(v.ring + v.cap);
            if (go) {
                pc = *reinterpret_cast<const uint4 *>(base + 16u * sub);
                if (sub == 0 && r == 15u) {
                    if (p4_ok) p4 = *reinterpret_cast<const uint4 *>(base + 64u);
                    else p4.x = e[kData + 1];
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (go) {
                reinterpret_cast<uint4 *>(slot)[sub] = pc;
                if (sub == 0 && r == 15u) reinterpret_cast<uint4 *>(slot)[4] = p4;   // byte 64 = e[49] either way
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (go) {
                // lane sub writes det field sub (idx, term, offset)
                uint64_t f;
                if (sub == 0) f = (uint64_t)lds_u32_at(slot, r) | ((uint64_t)lds_u32_at(slot, r + 4u) << 32);
                else if (sub == 1) f = (uint64_t)lds_u32_at(slot, r + 8u) | ((uint64_t)lds_u32_at(slot, r + 12u) << 32);
                else f = o;
                if (sub < 3) reinterpret_cast<uint64_t *>(out + n)[sub] = f;
                const uint32_t type = slot[r + kType];
                const uint32_t clen = (uint32_t)slot[r + kData] | ((uint32_t)slot[r + kData + 1] << 8);
                const uint32_t el = entry_len(type, clen);
                if (v.len - o < el) o = 0;
                o += el;
                ++n;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        if (live && sub == 0) len[g] = n;
    }
}

__global__ void __launch_bounds__(256) last_idx_term_kernel(const apus_batch_t b, uint64_t *lit)
{
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const apus_group_state_t st = load_state(b, g);
        uint64_t idx, term;
        local_idx_term(b, g, st, idx, term);
        lit[2 * g] = idx;
        lit[2 * g + 1] = term;
    }
}


// ---------------------------------------------------------------------------
// log replication step machine
// ---------------------------------------------------------------------------
// handle_lr_work_completion on one (g, i) pair; bytes in, bytes out
__device__ __forceinline__ void lr_complete(uint32_t wc, uint32_t &step, uint32_t &sf, uint32_t &sc)
{
    if (wc == APUS_WC_NONE || wc == APUS_WC_STALE) return;          // :3136 wr_id != next_wr_id
    if (wc == APUS_WC_SUCCESS) {
        if (step == APUS_LR_UPDATE_LOG) {                            // :3138-3155
            if (sc == 0) sf = 1;
            else if (sc == 1) { step = APUS_LR_UPDATE_END; sf = 1; }
            else if (sc == 2) sc = 1;
        } else if (step != APUS_LR_UPDATE_END) {                     // :3157-3162 (uint8_t ++)
            step = (step + 1) & 0xFF;
            sf = 1;
        } else {                                                     // :3163-3168
            step = APUS_LR_UPDATE_LOG;
            sf = 1;
        }
    } else if (step == APUS_LR_UPDATE_LOG) {                         // :3171-3183
        if (sc == 2) sc = 0;
        else if (sc <= 1) sf = 1;
    } else {                                                         // :3185-3193
        sf = 1;
    }
}

// The [G][R] byte columns are streamed as dwords (4 pairs per lane, one
// load and one store per column) when every column is 4-byte aligned; the
// last G*R % 4 pairs (and unaligned columns: VEC = false) go byte by byte.
template <bool VEC>
__global__ void __launch_bounds__(256) lr_completion_kernel(uint64_t pairs, const uint8_t *__restrict__ wc,
                                                            uint8_t *__restrict__ step, uint8_t *__restrict__ sf,
                                                            uint8_t *__restrict__ sc)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (VEC) {
        const uint64_t words = pairs >> 2;
        for (uint64_t w = t; w < words; w += stride) {
            const uint32_t c = reinterpret_cast<const uint32_t *>(wc)[w];
            if (c == 0) continue;                                    // no completions in these 4 pairs
            const uint32_t s0 = reinterpret_cast<const uint32_t *>(step)[w];
            const uint32_t f0 = reinterpret_cast<const uint32_t *>(sf)[w];
            const uint32_t n0 = reinterpret_cast<const uint32_t *>(sc)[w];
            uint32_t s1 = 0, f1 = 0, n1 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t a = (s0 >> (8 * k)) & 0xFF, b = (f0 >> (8 * k)) & 0xFF, d = (n0 >> (8 * k)) & 0xFF;
                lr_complete((c >> (8 * k)) & 0xFF, a, b, d);
                s1 |= a << (8 * k); f1 |= b << (8 * k); n1 |= d << (8 * k);
            }
            if (s1 != s0) reinterpret_cast<uint32_t *>(step)[w] = s1;
            if (f1 != f0) reinterpret_cast<uint32_t *>(sf)[w] = f1;
            if (n1 != n0) reinterpret_cast<uint32_t *>(sc)[w] = n1;
        }
        t += words << 2;
        if (t >= pairs) return;
    }
    for (uint64_t k = t; k < pairs; k += stride) {
        const uint32_t c = wc[k];
        if (c == 0) continue;
        uint32_t a = step[k], b = sf[k], d = sc[k];
        lr_complete(c, a, b, d);
        step[k] = (uint8_t)a; sf[k] = (uint8_t)b; sc[k] = (uint8_t)d;
    }
}

// log_adjustment for one group per lane.  Servers in index order (the
// leader's commit update at LR_GET_NCE_LEN is sequential).  The LR_SET_END
// walks (log_find_remote_end_offset, dare_log.h:367-394) are deferred to a
// wave-cooperative pass: lane segments take the pending (group, server)
// walks and check S determinants per step, the first mismatch found by
// ballot (as validate_kernel).  The group loop runs in whole waves (lanes
// past n_groups idle through the per-group part) so every lane joins the
// cooperative pass.
// MAXR: compile-time bound on R (4 / 8 / 16) so the preloaded server columns
// stay in registers; every column a server can reach is loaded up front
// (back-to-back, no dependent round trips through the skip tests).
__device__ __forceinline__ uint64_t shfl64(uint64_t x, uint32_t src)
{
    return ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(x >> 32), (int)src) << 32) |
           (uint32_t)__shfl((int)(uint32_t)x, (int)src);
}

template <int MAXR, uint32_t S>
__global__ void __launch_bounds__(256) log_adjust_kernel(const apus_batch_t b, const apus_lr_io_t io)
{
    const uint32_t R = b.n_replicas;
    const uint32_t lane = lane_id();
    const uint64_t wstride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < b.n_groups;
         base += wstride) {
        const uint64_t g = base + lane;
        const uint64_t gR = g * R;
        uint32_t walk = 0;                     // servers whose LR_SET_END walk is pending
        apus_group_state_t st = {};
        if (g < b.n_groups) {
            st = load_state(b, g);
            const uint32_t self = b.self_idx[g];
            const uint32_t size = ext_group_size(st.cid);           // :1313
            const uint32_t conn = io.rc_connected ? io.rc_connected[g] : 0xFFFFu;
            uint64_t commit = st.commit;
            bool init = false;
            uint32_t fc[MAXR], sf[MAXR], sp[MAXR];
            uint64_t va[MAXR];
#pragma unroll
            for (int i = 0; i < MAXR; ++i) {
                if ((uint32_t)i >= R) continue;
                fc[i] = b.fail_count[gR + i];
                sf[i] = io.send_flag[gR + i];
                sp[i] = b.lr_step[gR + i];
                va[i] = b.vote_ack[gR + i];
            }
#pragma unroll
            for (int i = 0; i < MAXR; ++i) {
                if ((uint32_t)i >= R) continue;
                uint32_t p = APUS_LR_POST_NONE;
                if ((uint32_t)i < size && (uint32_t)i != self && ((st.cid.bitmask >> i) & 1u) &&   // :1315-1317
                    fc[i] < APUS_PERMANENT_FAILURE &&                                               // :1321
                    sf[i] && ((conn >> i) & 1u)) {                                                 // :1325, :1331
                    const uint64_t rc = va[i];                                                      // :1335
                    if (rc != st.len) {                                                             // :1336
                        uint32_t s = sp[i];
                        if (!init && s < APUS_LR_UPDATE_LOG) { init = true; io.ssn[g] += 1; }       // :1341-1345
                        if (s == APUS_LR_GET_WRITE) {                                               // :1348-1353
                            b.remote_commit[gR + i] = rc;
                            s = APUS_LR_GET_NCE_LEN;
                        }
                        if (s == APUS_LR_GET_NCE_LEN) {                                             // :1354-1379
                            if (larger(st.end, st.len, rc, commit)) commit = rc;
                            p = APUS_LR_POST_READ_NC_LEN;
                        } else if (s == APUS_LR_GET_NCE) {                                          // :1380-1405
                            if (io.nc_len[gR + i] == 0) {
                                b.remote_end[gR + i] = b.remote_commit[gR + i];
                                s = APUS_LR_UPDATE_LOG;
                            } else {
                                p = APUS_LR_POST_READ_NC;
                            }
                        } else if (s == APUS_LR_SET_END) {                                          // :1406-1422
                            // empty buffer (or a len past the ring): the caller's rule, no walk
                            if (io.nc_len[gR + i] && io.max_dets && st.len <= ring_cap(b))
                                walk |= 1u << i;
                            else
                                b.remote_end[gR + i] = b.remote_commit[gR + i];
                            p = APUS_LR_POST_WRITE_END;
                        }
                        if (s != sp[i]) b.lr_step[gR + i] = (uint8_t)s;
                        if (p != APUS_LR_POST_NONE) io.send_flag[gR + i] = 0;                       // :1433
                    }
                }
                io.post[gR + i] = (uint8_t)p;
            }
            if (commit != st.commit) offsets_of(b, g)[kOffCommit] = commit;
        }
        // wave-cooperative determinant walks: 64/S pending walks per step,
        // S lanes each (segment j = lanes [jS, jS+S)), S >= max_dets when
        // max_dets <= 16 so a short NC buffer takes one step
        constexpr uint32_t W = 64 / S;
        const uint32_t seg = lane / S, sl = lane % S;
        const uint64_t segmask = S == 64 ? ~0ull : ((1ull << (S & 63)) - 1);
        for (uint64_t bal = __ballot(walk != 0); bal; bal = __ballot(walk != 0)) {
            uint32_t myL = 64, myI = 0;
            const uint32_t wmine = walk ? (uint32_t)__builtin_ctz(walk) : 0u;
            uint64_t m = bal;
#pragma unroll
            for (uint32_t j = 0; j < W; ++j) {
                if (m) {
                    const uint32_t Lj = (uint32_t)__builtin_ctzll(m);
                    m &= m - 1;
                    const uint32_t ij = __builtin_amdgcn_readlane(wmine, Lj);
                    if (seg == j) { myL = Lj; myI = ij; }
                    if (lane == Lj) walk &= walk - 1;
                }
            }
            const bool act = myL < 64 && base + myL < b.n_groups;
            const uint32_t src = myL & 63u;
            const uint64_t endL = shfl64(st.end, src), lenL = shfl64(st.len, src);
            const uint64_t gL = base + src;
            const uint64_t k_gi = gL * R + myI;
            const apus_entry_det_t *d = io.nc_dets + k_gi * io.max_dets;
            // the first step's determinant is requested together with nc_len
            // (the buffer holds max_dets of them): one dependent load less
            uint32_t n = 0;
            apus_entry_det_t det0 = { 0, 0, 0 };
            if (act) {
                if (sl < io.max_dets) det0 = d[sl];
                const uint64_t nl = io.nc_len[k_gi];
                n = nl < io.max_dets ? (uint32_t)nl : io.max_dets;
            }
            const RingView v = { b.ring + gL * b.ring_stride, endL, lenL, ring_cap(b) };
            uint64_t res = 0;
            bool found = false;
            for (uint32_t k0 = 0;; k0 += S) {
                const bool more = act && !found && k0 < n;
                if (!__ballot(more)) break;
                const uint32_t k = k0 + sl;
                bool bad = false;
                uint64_t ro = 0, nx = 0;
                if (more && k < n) {
                    const apus_entry_det_t det = k0 == 0 ? det0 : d[k];
                    uint64_t off = det.offset;
                    if (!v.get_entry(off)) {
                        bad = true;
                        ro = off;
                    } else {
                        const uint8_t *e = v.ring + off;
                        uint64_t l_idx, l_term;
                        ld_idx_term(e, l_idx, l_term);
                        if (l_idx != det.idx || l_term != det.term) {
                            bad = true;
                            ro = off;
                        } else {
                            const uint32_t el = entry_len(e[kType], ld_u16(e + kData));
                            nx = (v.len - off < el ? 0 : off) + el;
                        }
                    }
                }
                const uint64_t segbits = (__ballot(bad) >> (seg * S)) & segmask;
                const uint64_t vbad = shfl64(ro, seg * S + (segbits ? (uint32_t)__builtin_ctzll(segbits) : 0u));
                const uint64_t vlast = shfl64(nx, seg * S + ((n - 1 - k0) & (S - 1)));
                if (more) {
                    if (segbits) { res = vbad; found = true; }
                    else if (k0 + S >= n) res = vlast;
                }
            }
            if (act && sl == 0) b.remote_end[k_gi] = res;
        }
    }
}

// ---------------------------------------------------------------------------
// launches
// ---------------------------------------------------------------------------
hipError_t launch_vote(apus_ctx *ctx, const apus_batch_t &b, const apus_vote_out_t &o, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    const uint32_t grid = grid_for(b.n_groups, 256, ctx->n_cu, 8);
    ScratchPin pin;
    hipError_t e = stream_scratch(ctx, s, grid, 0, pin);
    StreamScratch *sc = pin.sc;
    if (e != hipSuccess) return e;
    typedef void (*fn_t)(const apus_batch_t, const apus_vote_out_t, uint64_t *);
    const uint32_t R = b.n_replicas;
    const fn_t fn = R == 3 ? vote_tally_kernel<3, true> : R == 5 ? vote_tally_kernel<5, true>
                  : R == 7 ? vote_tally_kernel<7, true> : R <= 8 ? vote_tally_kernel<8, false>
                           : vote_tally_kernel<kMaxR, false>;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, s, b, o, sc->partials);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return launch_stats_finalize(sc->partials, grid, 1, ctx->stats, APUS_STAT_VOTES_WON, false, s);
}

hipError_t launch_last_idx_term(const apus_batch_t &b, uint64_t *out, hipStream_t s)
{
    // (a quad-per-group form of this walk, and the 16-lane segment walk,
    // measured no faster: it writes nothing per entry)
    const uint32_t grid = grid_for(b.n_groups, 256, 256, 8);
    hipLaunchKernelGGL(last_idx_term_kernel, dim3(grid), dim3(256), 0, s, b, out);
    return hipGetLastError();
}

hipError_t launch_rank(apus_ctx *ctx, const apus_batch_t &b, const apus_rank_out_t &o, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    const uint32_t grid = grid_for(b.n_groups, 256, ctx->n_cu, 8);
    typedef void (*fn_t)(const apus_batch_t, const apus_rank_out_t, const uint64_t *);
    const uint32_t R = b.n_replicas;
    const fn_t fn = R == 3 ? vote_rank_kernel<3, true> : R == 5 ? vote_rank_kernel<5, true>
                  : R == 7 ? vote_rank_kernel<7, true> : R <= 8 ? vote_rank_kernel<8, false>
                           : vote_rank_kernel<kMaxR, false>;
    hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, s, b, o, b.last_idx_term);
    return hipGetLastError();
}

hipError_t launch_prune(apus_ctx *ctx, const apus_batch_t &b, const apus_prune_out_t &o, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    const uint32_t grid = grid_for(b.n_groups, 256, ctx->n_cu, 8);
    ScratchPin pin;
    hipError_t e = stream_scratch(ctx, s, grid, 0, pin);
    StreamScratch *sc = pin.sc;
    if (e != hipSuccess) return e;
    if (b.n_replicas > 8) hipLaunchKernelGGL(prune_kernel<16>, dim3(grid), dim3(256), 0, s, b, o, sc->partials);
    else hipLaunchKernelGGL(prune_kernel<8>, dim3(grid), dim3(256), 0, s, b, o, sc->partials);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (!b.abs_base) return hipSuccess;
    return launch_stats_finalize(sc->partials, grid, 1, ctx->stats, APUS_STAT_MIN_WATERMARK, true, s);
}

hipError_t launch_validate(apus_ctx *ctx, const apus_batch_t &b, const apus_nc_batch_t &nc, uint64_t *out,
                           hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    // (no more blocks than are resident: grid-strided waves, no partial last round)
    const uint32_t grid = grid_for(b.n_groups, 4, ctx->n_cu,
                                   (uint32_t)min(16, resident_blocks(ctx, 44, (const void *)validate_kernel)));
    ScratchPin pin;
    hipError_t e = stream_scratch(ctx, s, grid, 0, pin);
    StreamScratch *sc = pin.sc;
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(validate_kernel, dim3(grid), dim3(256), 0, s, b, nc, out, sc->partials);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return launch_stats_finalize(sc->partials, grid, 1, ctx->stats, APUS_STAT_MISMATCHES, false, s);
}

hipError_t launch_nc_build(apus_ctx *ctx, const apus_batch_t &b, apus_entry_det_t *dets, uint32_t max_dets,
                           uint32_t *len, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    // A ring array that is not 16-B aligned (or APUS_BATCH_LANE_IMPL) keeps the
    // lane-per-group walk.  Logs of equal entries (C2, C5) take the 16-lane
    // speculative segments (C2 3.12 -> 2.16 ms, C5 2.87 -> 2.06 ms against the
    // quad kernel); with APUS_BATCH_VAR_LEN the quad kernel, which loads a
    // header in four 16-B pieces at once (C3: 0.87 ms; segments of 16 lanes
    // 6.9 ms, of 4 lanes 2.5 ms: the speculation fails at every entry).
    if ((b.flags & APUS_BATCH_LANE_IMPL) || ((((uintptr_t)b.ring) | b.ring_stride) & 15u)) {
        const uint32_t grid = grid_for(b.n_groups, 256, ctx->n_cu, 8);
        hipLaunchKernelGGL(nc_build_kernel, dim3(grid), dim3(256), 0, s, b, dets, max_dets, len);
    } else if (b.flags & APUS_BATCH_VAR_LEN) {
        const uint32_t grid = grid_for(b.n_groups, 64, ctx->n_cu, 8);
        hipLaunchKernelGGL(nc_build_quad_kernel, dim3(grid), dim3(256), 0, s, b, dets, max_dets, len);
    } else {
        const uint32_t grid = grid_for(b.n_groups, 16, ctx->n_cu, 8);
        hipLaunchKernelGGL(nc_build_seg_kernel<16>, dim3(grid), dim3(256), 0, s, b, dets, max_dets, len);
    }
    return hipGetLastError();
}

hipError_t launch_lr_completion(apus_ctx *ctx, const apus_batch_t &b, const apus_lr_io_t &io, hipStream_t s)
{
    const uint64_t pairs = b.n_groups * b.n_replicas;
    if (!pairs) return hipSuccess;
    const bool vec = (((uintptr_t)io.wc | (uintptr_t)b.lr_step | (uintptr_t)io.send_flag |
                       (uintptr_t)io.send_count) & 3u) == 0;
    const uint32_t grid = grid_for(vec ? (pairs + 3) / 4 : pairs, 256, ctx->n_cu, 8);
    if (vec)
        hipLaunchKernelGGL(lr_completion_kernel<true>, dim3(grid), dim3(256), 0, s, pairs, io.wc, b.lr_step,
                           io.send_flag, io.send_count);
    else
        hipLaunchKernelGGL(lr_completion_kernel<false>, dim3(grid), dim3(256), 0, s, pairs, io.wc, b.lr_step,
                           io.send_flag, io.send_count);
    return hipGetLastError();
}

hipError_t launch_log_adjust(apus_ctx *ctx, const apus_batch_t &b, const apus_lr_io_t &io, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    const bool seg16 = io.max_dets <= 16;
    // (no more blocks than are resident: grid-strided lanes, no partial last round)
#define APUS_ADJ(MR)                                                                                           \
    do {                                                                                                       \
        const void *fn = seg16 ? (const void *)log_adjust_kernel<MR, 16> : (const void *)log_adjust_kernel<MR, 64>; \
        const int slot = 45 + 2 * (MR == 4 ? 0 : MR == 8 ? 1 : 2) + (seg16 ? 1 : 0);                         \
        const uint32_t grid = grid_for(b.n_groups, 256, ctx->n_cu, (uint32_t)min(8, resident_blocks(ctx, slot, fn))); \
        if (seg16) hipLaunchKernelGGL((log_adjust_kernel<MR, 16>), dim3(grid), dim3(256), 0, s, b, io);         \
        else hipLaunchKernelGGL((log_adjust_kernel<MR, 64>), dim3(grid), dim3(256), 0, s, b, io);               \
    } while (0)
    if (b.n_replicas <= 4) APUS_ADJ(4);
    else if (b.n_replicas <= 8) APUS_ADJ(8);
    else APUS_ADJ(kMaxR);
#undef APUS_ADJ
    return hipGetLastError();
}

}  // namespace apus
