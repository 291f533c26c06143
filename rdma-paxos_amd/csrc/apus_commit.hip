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
constexpr int kCommitStats = 4;           // decisions, committed, advanced, corrupt
constexpr uint32_t kCommitStatMap = APUS_STAT_DECISIONS | (APUS_STAT_COMMITTED << 8) |
                                    (APUS_STAT_ADVANCED << 16) | (APUS_STAT_CORRUPT << 24);

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

__device__ __forceinline__ uint32_t byte_sum(uint32_t w) { return __builtin_amdgcn_udot4(w, 0x01010101u, 0u, false); }
// sum_j (j + 4i) * byte_j(w) for word i of a 16-byte piece
__device__ __forceinline__ uint32_t byte_wsum(uint32_t w, uint32_t i)
{
    return __builtin_amdgcn_udot4(w, 0x03020100u + 0x04040404u * i, 0u, false);
}

// sums (or mins) partials[nblk][nstat]; statistic k -> stats[(map >> 8k) & 0xFF]
__global__ void __launch_bounds__(256) stats_finalize_kernel(const uint64_t *partials, uint32_t nblk,
                                                             uint32_t nstat, uint64_t *stats,
                                                             uint32_t map, int is_min)
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
                                 uint64_t *stats, uint32_t map, bool is_min, hipStream_t s)
{
    hipLaunchKernelGGL(stats_finalize_kernel, dim3(1), dim3(256), 0, s, partials, nblk, nstat, stats, map,
                       is_min ? 1 : 0);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// commit_wave_kernel
// ---------------------------------------------------------------------------
// One group per wave.  Per window [ws, we) of the ring (ws 16-B aligned):
//   1. stage: lanes load 16-B pieces k = lane + 64 j (coalesced, 1 KiB per
//      wave instruction) into the wave's LDS window; with CHECKSUM each lane
//      also forms the piece's byte sum and position-weighted byte sum
//      (v_dot4_u32_u8) and the wave scans them into exclusive prefix arrays.
//   2. walk: wave-uniform chain walk over the entry headers inside the
//      window (type @26, cmd.len @48 read with ONE ds_read_b32 + readlane),
//      reproducing log_get_entry's header-wrap and the walk's ghost-header
//      jump; entry e of the window is recorded in lane e's registers.
//   3. acks: lane e tests reply[0..size) of entry e (byte == 1, self always
//      counts) -> ballot -> first failing entry stops the commit.
//   4. checksum: lane e adds the two immutable runs of entry e that fall in
//      the window using the prefix arrays (O(1) per run); lane 63 handles an
//      entry carried over from the previous window.
template <int WIN, bool CHECKSUM>
__global__ void __launch_bounds__(256) commit_wave_kernel(const apus_batch_t b, const apus_commit_out_t o,
                                                          uint64_t *partials)
{
    constexpr int NP = WIN / 16;          // 16-B pieces per window
    constexpr int PPL = NP / 64;          // pieces per lane
    constexpr uint32_t kMaxNew = 63;      // lane 63 is reserved for the carry
    static_assert(NP % 64 == 0, "window must be a multiple of 1 KiB");

    __shared__ __attribute__((aligned(16))) uint32_t s_win[kWaves][WIN / 4 + 16];
    __shared__ __attribute__((aligned(16))) uint2 s_pre[kWaves][CHECKSUM ? NP + 1 : 1];

    const uint32_t lane = lane_id();
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint32_t *win = s_win[wv];
    uint2 *pre = s_pre[wv];

    uint64_t acc[kCommitStats] = { 0, 0, 0, 0 };

    for (uint64_t g = (uint64_t)blockIdx.x * kWaves + wv; g < b.n_groups; g += (uint64_t)gridDim.x * kWaves) {
        const apus_group_state_t st = b.state[g];
        const uint64_t len = st.len, end = st.end, commit0 = st.commit;
        const uint32_t self = b.self_idx[g];
        const uint32_t size = walk_size(st.cid);
        const uint32_t need = size / 2 + 1;
        const uint32_t size_mask = size >= 16 ? 0xFFFFu : ((1u << size) - 1u);
        const uint32_t self_bit = self < 16 ? (1u << self) : 0u;
        const uint8_t *ring = b.ring + g * b.ring_stride;
        // ring + ws must be 16-B aligned: device batches have delta = 0; a
        // host-mapped dare_log_t (scalar drop-ins) has its entries at +8
        const uint32_t delta = (uint32_t)((uintptr_t)ring & 15u);
        // dwords at ring offsets >= lim are never read (mapped logs end at len)
        const uint64_t lim = b.ring_stride >= len + 16 ? ~0ull : len;

        uint64_t m = commit0;
        bool forced = false;
        bool walk_done = dist(end, len, m) == 0;
        bool committing = true, stopped = false, corrupt = false;
        uint64_t stop = 0;
        uint32_t n_commit = 0;
        const uint64_t guard = len / kHdr + 4;
        uint64_t steps = 0, wins = 0;
        const uint64_t win_guard = len / 16 + 8;
        // checksum state: image length (mod M) is uniform, S/T are per-lane
        uint32_t P = 0, S = 0, T = 0;
        bool carry = false;
        uint32_t c_s = 0, c_elen = 0, c_dl = 0, c_p = 0;
        uint64_t cs = m;

        while (!(walk_done && !carry)) {
            if (!CHECKSUM && (walk_done || !committing)) break;
            if (++wins > win_guard) { corrupt = true; break; }
            const int64_t ws = (int64_t)((cs + delta) & ~15ull) - (int64_t)delta;
            const uint64_t we = ((uint64_t)(ws + WIN) < len) ? (uint64_t)(ws + WIN) : len;
            const uint32_t wlen = (int64_t)we > ws ? (uint32_t)((int64_t)we - ws) : 0u;
            const uint32_t np = (wlen + 15) >> 4;

            // ---- 1. stage the window (+ piece sums) ----
            uint32_t ps0[PPL], ps1[PPL];
#pragma unroll
            for (int j = 0; j < PPL; ++j) {
                const uint32_t k = lane + 64u * j;
                uint4 v = make_uint4(0u, 0u, 0u, 0u);
                if (k < np) {
                    const int64_t pos = ws + 16ll * k;
                    if ((uint64_t)(pos + 16) <= lim || pos + 16 <= 0) {
                        v = *reinterpret_cast<const uint4 *>(ring + pos);
                    } else {
                        const uint32_t *q = reinterpret_cast<const uint32_t *>(ring + pos);
                        if ((uint64_t)(pos + 4) <= lim) v.x = q[0];
                        if ((uint64_t)(pos + 8) <= lim) v.y = q[1];
                        if ((uint64_t)(pos + 12) <= lim) v.z = q[2];
                    }
                }
                *reinterpret_cast<uint4 *>(win + 4 * k) = v;
                if (CHECKSUM) {
                    const uint32_t s0 = byte_sum(v.x) + byte_sum(v.y) + byte_sum(v.z) + byte_sum(v.w);
                    const uint32_t sw = byte_wsum(v.x, 0) + byte_wsum(v.y, 1) + byte_wsum(v.z, 2) + byte_wsum(v.w, 3);
                    ps0[j] = s0;
                    ps1[j] = (16u * k * s0 + sw) % kAdlerMod;
                }
            }
            if (CHECKSUM) {
                uint32_t run0 = 0, run1 = 0;
#pragma unroll
                for (int j = 0; j < PPL; ++j) {
                    uint32_t x0 = ps0[j], x1 = ps1[j];
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const uint32_t t0 = __shfl_up(x0, d), t1 = __shfl_up(x1, d);
                        if (lane >= (uint32_t)d) { x0 += t0; x1 += t1; }
                    }
                    pre[lane + 64 * j] = make_uint2(x0 - ps0[j] + run0, x1 - ps1[j] + run1);
                    run0 += __builtin_amdgcn_readlane(x0, 63);
                    run1 += __builtin_amdgcn_readlane(x1, 63);
                }
                if (lane == 0) pre[NP] = make_uint2(run0, run1);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

            // ---- 2. walk the headers inside the window ----
            uint32_t n_new = 0;
            uint32_t e_s = 0, e_elen = 0, e_dl = 0, e_p = 0;   // lane e: entry e of this window
            bool jumped = false;
            while (!walk_done && n_new < kMaxNew) {
                if (!forced && dist(end, len, m) == 0) { walk_done = true; break; }
                if (len - m < kHdr) {                 // header does not fit: entry at 0
                    if (m > we) break;
                    m = 0; forced = true; jumped = true;
                    if (++steps > guard) corrupt = true;
                    break;
                }
                if ((int64_t)m < ws || m + kHdr > we) break;  // header not staged yet
                const uint32_t rel = (uint32_t)(m - ws);
                const uint32_t li = lane & 3u;
                const uint32_t w = win[(rel >> 2) + (li < 2 ? 6u + li : 10u + li)];
                const uint32_t w6 = __builtin_amdgcn_readlane(w, 0), w7 = __builtin_amdgcn_readlane(w, 1);
                const uint32_t w12 = __builtin_amdgcn_readlane(w, 2), w13 = __builtin_amdgcn_readlane(w, 3);
                const uint32_t sh = rel & 3u;
                const uint32_t tw = (sh + 2u >= 4u) ? w7 : w6;
                const uint32_t type = (tw >> (8u * ((sh + 2u) & 3u))) & 0xFFu;
                const uint32_t clen = (uint32_t)(((((uint64_t)w13 << 32) | w12) >> (8u * sh)) & 0xFFFFu);
                const uint32_t elen = entry_len(type, clen);
                if (len - m < elen) {                 // ghost header: continue at 0
                    m = 0; forced = false; jumped = true;
                    if (++steps > guard) corrupt = true;
                    break;
                }
                forced = false;
                const uint32_t dl = image_data_len(type, clen);
                if (lane == n_new) { e_s = (uint32_t)m; e_elen = elen; e_dl = dl; e_p = P; }
                if (CHECKSUM) P = (P + 27u + dl) % kAdlerMod;
                ++n_new;
                m += elen;
                if (++steps > guard) { corrupt = true; break; }
            }
            if (corrupt) break;

            // ---- 3. follower acks of the new entries ----
            if (committing && n_new > 0) {
                bool fail = false;
                if (lane < n_new) {
                    const uint32_t rel = (uint32_t)((int64_t)e_s - ws) + kReply;
                    const uint32_t d = rel >> 2, sh = rel & 3u;
                    const uint32_t q0 = win[d], q1 = win[d + 1], q2 = win[d + 2], q3 = win[d + 3], q4 = win[d + 4];
                    const uint32_t r0 = __builtin_amdgcn_alignbyte(q1, q0, sh);
                    const uint32_t r1 = __builtin_amdgcn_alignbyte(q2, q1, sh);
                    const uint32_t r2 = __builtin_amdgcn_alignbyte(q3, q2, sh);
                    const uint32_t r3 = __builtin_amdgcn_alignbyte(q4, q3, sh);
                    uint32_t mask = eq1_nibble(r0) | (eq1_nibble(r1) << 4) | (eq1_nibble(r2) << 8) |
                                    (eq1_nibble(r3) << 12);
                    mask = (mask | self_bit) & size_mask;
                    fail = (uint32_t)__builtin_popcount(mask) < need;
                }
                const uint64_t fb = __ballot(fail);
                if (fb) {
                    const uint32_t ef = (uint32_t)__builtin_ctzll(fb);
                    stop = __builtin_amdgcn_readlane(e_s, ef);
                    stopped = true;
                    committing = false;
                    n_commit += ef;
                } else {
                    n_commit += n_new;
                }
            }

            // ---- 4. checksum of the entries' bytes inside the window ----
            if (CHECKSUM) {
                bool have = lane < n_new;
                uint32_t s = e_s, dl = e_dl, p = e_p;
                if (lane == 63 && carry) { have = true; s = c_s; dl = c_dl; p = c_p; }
                if (have) {
                    const int64_t weu = (int64_t)we;
                    // two runs: [s, s+27) -> image p, [s+48, s+48+dl) -> image p+27
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        const uint32_t a = r == 0 ? s : s + kData;
                        const uint32_t e = r == 0 ? s + 27u : s + kData + dl;
                        const uint32_t pa = r == 0 ? p : (p + 27u) % kAdlerMod;
                        const int64_t a2 = (int64_t)a > ws ? (int64_t)a : ws;
                        const int64_t e2 = (int64_t)e < weu ? (int64_t)e : weu;
                        if (a2 < e2) {
                            uint32_t sum0[2], sum1[2];
#pragma unroll
                            for (int q = 0; q < 2; ++q) {
                                const uint32_t c = (uint32_t)((q == 0 ? a2 : e2) - ws);
                                const uint32_t k = c >> 4, rr = c & 15u;
                                const uint2 pr = pre[k];
                                uint32_t p0 = pr.x, p1 = pr.y;
                                if (rr) {
                                    const uint4 v = *reinterpret_cast<const uint4 *>(win + 4 * k);
                                    const uint32_t wv4[4] = { v.x, v.y, v.z, v.w };
                                    uint32_t part0 = 0, partw = 0;
#pragma unroll
                                    for (int i = 0; i < 4; ++i) {
                                        const uint32_t lo = 4u * i;
                                        const uint32_t msk = rr >= lo + 4 ? 0xFFFFFFFFu
                                                           : rr <= lo   ? 0u
                                                                        : ((1u << (8u * (rr - lo))) - 1u);
                                        const uint32_t x = wv4[i] & msk;
                                        part0 += byte_sum(x);
                                        partw += byte_wsum(x, i);
                                    }
                                    p0 += part0;
                                    p1 += 16u * k * part0 + partw;
                                }
                                sum0[q] = p0 % kAdlerMod;
                                sum1[q] = p1 % kAdlerMod;
                            }
                            const uint32_t sb = (sum0[1] + kAdlerMod - sum0[0]) % kAdlerMod;
                            const uint32_t sxb = (sum1[1] + kAdlerMod - sum1[0]) % kAdlerMod;
                            const uint32_t pa2 = (pa + (uint32_t)(a2 - (int64_t)a)) % kAdlerMod;  // image pos of a2
                            const uint32_t coef = (pa2 + kAdlerMod - (uint32_t)(a2 - ws) % kAdlerMod) % kAdlerMod;
                            S = (S + sb) % kAdlerMod;
                            T = (uint32_t)(((uint64_t)T + (uint64_t)coef * sb + sxb) % kAdlerMod);
                        }
                    }
                }
                // carry: the entry that still has bytes past `we`
                bool nc = false;
                if (n_new > 0) {
                    const uint32_t last = n_new - 1;
                    const uint32_t ls = __builtin_amdgcn_readlane(e_s, last);
                    const uint32_t le = __builtin_amdgcn_readlane(e_elen, last);
                    if ((uint64_t)ls + le > we) {
                        nc = true;
                        c_s = ls; c_elen = le;
                        c_dl = __builtin_amdgcn_readlane(e_dl, last);
                        c_p = __builtin_amdgcn_readlane(e_p, last);
                    }
                } else if (carry && (uint64_t)c_s + c_elen > we) {
                    nc = true;
                }
                carry = nc;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

            cs = jumped ? 0ull : (carry ? we : m);
        }

        const uint64_t res = stopped ? stop : m;
        const bool adv = !corrupt && larger(end, len, res, commit0);
        uint32_t digest = 1;
        if (CHECKSUM) {
            const uint32_t Sa = wave_sum_mod(S), Ta = wave_sum_mod(T);
            const uint32_t A = (1u + Sa) % kAdlerMod;
            const uint32_t B = (uint32_t)(((uint64_t)P + (uint64_t)P * Sa + kAdlerMod - Ta) % kAdlerMod);
            digest = (B << 16) | A;
        }
        if (lane == 0) {
            if (o.new_commit) o.new_commit[g] = adv ? res : commit0;
            if (o.committed) o.committed[g] = corrupt ? 0xFF : (uint8_t)adv;
            if (o.n_entries) o.n_entries[g] = n_commit;
            if (CHECKSUM && o.digest) o.digest[g] = digest;
        }
        acc[0] += 1;
        acc[1] += n_commit;
        acc[2] += adv ? 1 : 0;
        acc[3] += corrupt ? 1 : 0;
    }
    uint64_t mine[kCommitStats];   // acc is wave-uniform: count it once per wave
#pragma unroll
    for (int k = 0; k < kCommitStats; ++k) mine[k] = lane == 0 ? acc[k] : 0;
    block_partials<kCommitStats>(partials, mine);
}

// ---------------------------------------------------------------------------
// commit_lane_kernel: one lane per group, straight from global memory
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
__global__ void __launch_bounds__(256) commit_lane_kernel(const apus_batch_t b, const apus_commit_out_t o,
                                                          uint64_t *partials)
{
    uint64_t acc[kCommitStats] = { 0, 0, 0, 0 };
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const apus_group_state_t st = b.state[g];
        const uint64_t len = st.len, end = st.end, commit0 = st.commit;
        const uint32_t self = b.self_idx[g];
        const uint32_t size = walk_size(st.cid);
        const uint32_t need = size / 2 + 1;
        const uint8_t *ring = b.ring + g * b.ring_stride;
        const uint64_t guard = len / kHdr + 4;
        uint64_t m = commit0, steps = 0, stop = 0;
        uint32_t n = 0, ad = 1;
        bool committing = true, stopped = false, corrupt = false;
        while (dist(end, len, m)) {
            if (++steps > guard) { corrupt = true; break; }
            if (len - m < kHdr) m = 0;                        // log_get_entry
            if (m + kHdr > len) { corrupt = true; break; }    // offset past the ring
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
            if (CHECKSUM) {
                ad = adler_bytes(e, 27, ad);
                ad = adler_bytes(e + kData, image_data_len(type, clen), ad);
            }
            m += elen;
        }
        const uint64_t res = stopped ? stop : m;
        const bool adv = !corrupt && larger(end, len, res, commit0);
        if (o.new_commit) o.new_commit[g] = adv ? res : commit0;
        if (o.committed) o.committed[g] = corrupt ? 0xFF : (uint8_t)adv;
        if (o.n_entries) o.n_entries[g] = n;
        if (CHECKSUM && o.digest) o.digest[g] = ad;
        acc[0] += 1; acc[1] += n; acc[2] += adv; acc[3] += corrupt;
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

hipError_t launch_commit(apus_ctx *ctx, const apus_batch_t &b, const apus_commit_out_t &o,
                         uint32_t flags, hipStream_t s)
{
    if (b.n_groups == 0) return hipSuccess;
    const bool ck = (flags & APUS_COMMIT_CHECKSUM) != 0;
    if (flags & (APUS_COMMIT_WALK | APUS_COMMIT_CHECKSUM)) {
        uint32_t grid;
        const bool lane_impl = (b.flags & APUS_BATCH_LANE_IMPL) != 0;
        if (lane_impl) grid = grid_for(b.n_groups, 256, ctx->n_cu, 8);
        else grid = grid_for(b.n_groups, kWaves, ctx->n_cu, 20);
        hipError_t e = ensure_partials(ctx, (size_t)grid * kCommitStats);
        if (e != hipSuccess) return e;
        if (lane_impl) {
            if (ck) hipLaunchKernelGGL(commit_lane_kernel<true>, dim3(grid), dim3(256), 0, s, b, o, ctx->partials);
            else hipLaunchKernelGGL(commit_lane_kernel<false>, dim3(grid), dim3(256), 0, s, b, o, ctx->partials);
        } else {
            if (ck) hipLaunchKernelGGL((commit_wave_kernel<4096, true>), dim3(grid), dim3(256), 0, s, b, o, ctx->partials);
            else hipLaunchKernelGGL((commit_wave_kernel<4096, false>), dim3(grid), dim3(256), 0, s, b, o, ctx->partials);
        }
        e = hipGetLastError();
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
