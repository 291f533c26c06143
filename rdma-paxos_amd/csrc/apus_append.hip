// Producer side of the commit walk for gfx950:
//
//   append_kernel   — one WAVE per consensus group appends the group's queued
//       messages in order with log_append_entry's semantics
//       (src/include/dare/dare_log.h:466-558, driven by get_tailq_message,
//       src/dare/dare_ibv_ud.c:780-790).  The placement recurrence (index
//       from the tail entry, header wrap, ghost header + rewrite at 0, full
//       log) is scalar; every entry's 64-B header is written by the 64 lanes
//       as one coalesced byte-masked store (sender@27 and bytes 41..47 are
//       left untouched, as the reference never writes them) and its command
//       bytes by lane-strided copies.
//   persist_kernel  — one LANE per (group, replica copy): persist_new_entries
//       (src/dare/dare_server.c:1792-1810).  The leader stamps sender, each
//       follower sets its reply[] byte in the leader's entries
//       (rc_send_entries_reply, src/dare/dare_ibv_rc.c:1828-1863): the
//       prefix-monotone ack traces the commit walk consumes.
#include "apus_device.h"
#include "apus_internal.h"

namespace apus {

constexpr uint32_t kAppendWaves = 4;

__device__ __forceinline__ bool csm_type(uint32_t t) { return !bare_type(t); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ring_rsrc_of(uint8_t *ring, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(ring, (short)0, (int)bytes, 0x00020000);
}

// lane k's u64 as a wave-uniform value
__device__ __forceinline__ uint64_t rl64c(uint64_t x, uint32_t k)
{
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(x >> 32), k) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((uint32_t)x, k);
}

// bytes of a 64-B header written by log_append_entry (dare_log.h:494-499,
// 507-535): idx, term, req_id, clt_id, type, reply[13] = 0, then the data
// prefix: dmode 1 = cmd.len (CSM-class), 2 = dare_cid_t (16 B), 3 = head (8 B)
__device__ __forceinline__ void write_header(uint8_t *e, uint32_t lane, uint64_t idx, uint64_t term, uint64_t req,
                                             uint32_t clt, uint32_t type, uint32_t dmode, uint32_t clen,
                                             const uint8_t *dsrc)
{
    uint32_t v = 0;
    bool w = true;
    if (lane < 24) {
        const uint64_t x = lane < 8 ? idx : lane < 16 ? term : req;
        v = (uint32_t)(x >> (8 * (lane & 7))) & 0xFFu;
    } else if (lane < 26) {
        v = (clt >> (8 * (lane - 24))) & 0xFFu;
    } else if (lane == 26) {
        v = type;
    } else if (lane == kSender || (lane >= kReply + APUS_MAX_SERVER_COUNT && lane < kData)) {
        w = false;
    } else if (lane < kData) {
        v = 0;                                                  // memset(entry->reply, 0, ...)
    } else if (dmode == 1) {
        w = lane < kData + 2;
        v = (clen >> (8 * (lane - kData))) & 0xFFu;
    } else if (dmode == 2) {
        v = dsrc[lane - kData];
    } else if (dmode == 3) {
        w = lane < kData + 8;
        if (w) v = dsrc[lane - kData];
    } else {
        w = false;
    }
    if (w) e[lane] = (uint8_t)v;
}

// data = each message's sm_cmd_t {len, cmd[len]} verbatim, for messages
// [k0, k1) of the chunk (lane k holds message k's data_off, entry offset and
// cmd.len): the wave copies kB entries at a time, every load of a batch in
// flight before its stores, in the widest unit all sources and destinations
// of the batch are aligned to
__device__ __forceinline__ void copy_cmds(uint8_t *ring, const uint8_t *pay, uint32_t k0, uint32_t k1,
                                          uint64_t m_doff, uint32_t s_v, uint32_t m_clen, uint32_t lane)
{
    constexpr int kB = 8;
    for (uint32_t kb = k0; kb < k1; kb += kB) {
        uint64_t src[kB], dst[kB];
        uint32_t nb[kB], mx = 0, al = 0;
#pragma unroll
        for (int i = 0; i < kB; ++i) {
            const uint32_t kk = min(kb + i, k1 - 1);
            src[i] = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(m_doff >> 32), kk) << 32) |
                     (uint32_t)__builtin_amdgcn_readlane((uint32_t)m_doff, kk);
            dst[i] = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(s_v, kk) + kData;
            nb[i] = kb + i < k1 ? 2u + (uint32_t)__builtin_amdgcn_readlane(m_clen, kk) : 0u;
            mx = max(mx, nb[i]);
            al |= (uint32_t)src[i] | (uint32_t)dst[i];
        }
        if ((al & 3u) == 0) {
            for (uint32_t j = 4 * lane; j < mx; j += 256) {
                uint32_t v[kB];
#pragma unroll
                for (int i = 0; i < kB; ++i)
                    v[i] = j + 4 <= nb[i] ? *reinterpret_cast<const uint32_t *>(pay + src[i] + j) : 0u;
#pragma unroll
                for (int i = 0; i < kB; ++i) {
                    if (j + 4 <= nb[i]) *reinterpret_cast<uint32_t *>(ring + dst[i] + j) = v[i];
                    else for (uint32_t t = j; t < nb[i]; ++t) ring[dst[i] + t] = pay[src[i] + t];
                }
            }
        } else if ((al & 1u) == 0) {
            for (uint32_t j = 2 * lane; j < mx; j += 128) {
                uint32_t v[kB];
#pragma unroll
                for (int i = 0; i < kB; ++i)
                    v[i] = j + 2 <= nb[i] ? *reinterpret_cast<const uint16_t *>(pay + src[i] + j) : 0u;
#pragma unroll
                for (int i = 0; i < kB; ++i) {
                    if (j + 2 <= nb[i]) *reinterpret_cast<uint16_t *>(ring + dst[i] + j) = (uint16_t)v[i];
                    else if (j < nb[i]) ring[dst[i] + j] = pay[src[i] + j];
                }
            }
        } else {
            for (uint32_t j = lane; j < mx; j += 64) {
                uint32_t v[kB];
#pragma unroll
                for (int i = 0; i < kB; ++i) v[i] = j < nb[i] ? pay[src[i] + j] : 0u;
#pragma unroll
                for (int i = 0; i < kB; ++i)
                    if (j < nb[i]) ring[dst[i] + j] = (uint8_t)v[i];
            }
        }
    }
}

// log_append_entry's header of a CSM-class entry (dare_log.h:494-499,
// 507-512): idx, term, req_id, clt_id, type, reply[13] = 0; sender@27 and the
// pad bytes 41..47 are not written.  at(o) is the address of the entry's byte
// o (a ring address, or its place in a padded LDS image of the ring: the pad
// is a multiple of 16 B, so the alignment is the same, and no store below
// crosses a 16-B boundary).  Stores as wide as that alignment allows.
template <typename At>
__device__ __forceinline__ void write_csm_header_at(At at, uint64_t idx, uint64_t term, uint64_t req, uint32_t clt,
                                                    uint32_t type)
{
    const uint32_t al = (uint32_t)(uintptr_t)at(0) & 7u;
    if (al == 0) {
        *reinterpret_cast<uint64_t *>(at(0)) = idx;
        *reinterpret_cast<uint64_t *>(at(8)) = term;
        *reinterpret_cast<uint64_t *>(at(16)) = req;
        *reinterpret_cast<uint16_t *>(at(24)) = (uint16_t)clt;
        *at(26) = (uint8_t)type;
        *reinterpret_cast<uint32_t *>(at(28)) = 0u;         // reply[0..3]
        *reinterpret_cast<uint64_t *>(at(32)) = 0ull;       // reply[4..11]
        *at(40) = 0;                                        // reply[12]
    } else if ((al & 3u) == 0) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            *reinterpret_cast<uint32_t *>(at(4 * i)) = (uint32_t)(idx >> (32 * i));
            *reinterpret_cast<uint32_t *>(at(8 + 4 * i)) = (uint32_t)(term >> (32 * i));
            *reinterpret_cast<uint32_t *>(at(16 + 4 * i)) = (uint32_t)(req >> (32 * i));
        }
        *reinterpret_cast<uint16_t *>(at(24)) = (uint16_t)clt;
        *at(26) = (uint8_t)type;
#pragma unroll
        for (int i = 7; i < 10; ++i) *reinterpret_cast<uint32_t *>(at(4 * i)) = 0u;
        *at(40) = 0;
    } else if ((al & 1u) == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            *reinterpret_cast<uint16_t *>(at(2 * i)) = (uint16_t)(idx >> (16 * i));
            *reinterpret_cast<uint16_t *>(at(8 + 2 * i)) = (uint16_t)(term >> (16 * i));
            *reinterpret_cast<uint16_t *>(at(16 + 2 * i)) = (uint16_t)(req >> (16 * i));
        }
        *reinterpret_cast<uint16_t *>(at(24)) = (uint16_t)clt;
        *at(26) = (uint8_t)type;
#pragma unroll
        for (int i = 14; i < 20; ++i) *reinterpret_cast<uint16_t *>(at(2 * i)) = 0;   // reply[0..11]
        *at(40) = 0;
    } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            *at(i) = (uint8_t)(idx >> (8 * i));
            *at(8 + i) = (uint8_t)(term >> (8 * i));
            *at(16 + i) = (uint8_t)(req >> (8 * i));
        }
        *at(24) = (uint8_t)clt;
        *at(25) = (uint8_t)(clt >> 8);
        *at(26) = (uint8_t)type;
#pragma unroll
        for (int i = kReply; i < kReply + APUS_MAX_SERVER_COUNT; ++i) *at(i) = 0;
    }
}

__device__ __forceinline__ void write_csm_header(uint8_t *e, uint64_t idx, uint64_t term, uint64_t req, uint32_t clt,
                                                 uint32_t type)
{
    write_csm_header_at([e](uint32_t o) { return e + o; }, idx, term, req, clt, type);
}

// ---------------------------------------------------------------------------
// Fast-prefix entries assembled in LDS.  For messages [kk, kl) placed back to
// back from s_v[kk] (no wrap), a sub-chunk whose ring span and command bytes
// fit the wave's LDS is built as an image of the ring span: the span's 16-B
// pieces are read into LDS (so the bytes log_append_entry never writes --
// sender@27, pad 41..47, the neighbours' bytes in the edge pieces -- keep
// their values), every message's command dwords are read into LDS, all with
// no wait between them (buffer loads straight to LDS); then lane k writes
// entry k's header and funnels its command into the image, and the span goes
// back to the ring as 16-B coalesced stores.  A handful of wide memory
// instructions per sub-chunk replace a header store per field and a command
// copy per message (append_kernel was bound by vector-memory instruction
// issue).  A message that does not fit, or whose last payload dword is cut by
// the end of the payload array, keeps the per-message path.
// ---------------------------------------------------------------------------
// A whole C2 group (64 entries of 128 B at any 16-B phase, 64 command images
// of <= 72 B) is one sub-chunk.  13 KB per wave, 52 KB per 4-wave block: the
// 3 blocks per CU that 161 VGPRs allow fit the 160 KB of LDS (4 KiB + 2.5 KiB
// per wave, two or three sub-chunks per C2 group: 7.64 -> 6.80 ms with the
// 16-B command loads below)
constexpr uint32_t kSpanLds = 8448;         // ring-span bytes per wave
constexpr uint32_t kPayLds = 4608;          // command-image bytes per wave
// The span image is padded: 32 B after every 1 KiB of span (span byte y at
// LDS byte y + 32 (y >> 10); one buffer_load ... lds of 64 pieces fills one
// KiB).  Lane k builds entry k, so with an unpadded image all lanes of a store
// hit one bank when the entries have one length (128 B: 32-way conflicts, 78%
// of the LDS cycles of append_kernel at C2, SQ_LDS_BANK_CONFLICT /
// SQ_LDS_IDX_ACTIVE).  The pad moves every eighth 128-B entry 8 banks on and
// the command funnel starts lane k at dword (k & 7) of its command, so a
// 32-lane store group touches 32 banks.
constexpr uint32_t kSpanImg = kSpanLds + 32u * ((kSpanLds + 1023u) / 1024u);
__device__ __forceinline__ uint32_t img_pos(uint32_t y) { return y + ((y >> 10) << 5); }

// lane-parallel LDS -> LDS copy of n bytes into the padded span image at span
// byte dpos (any alignment; dword body funnelled from the source dwords, in
// an order rotated by rot)
__device__ __forceinline__ void lds_funnel(uint8_t *img, uint32_t dpos, const uint8_t *pim, uint32_t spos, uint32_t n,
                                           uint32_t rot)
{
    const uint32_t h = min((4u - (dpos & 3u)) & 3u, n);
    for (uint32_t i = 0; i < h; ++i) img[img_pos(dpos + i)] = pim[spos + i];
    const uint32_t nw = (n - h) >> 2, t = (n - h) & 3u;
    const uint32_t sh = (spos + h) & 3u, q0 = (spos + h) >> 2, d0 = dpos + h;
    const uint32_t *s32 = reinterpret_cast<const uint32_t *>(pim);
    uint32_t w = rot < nw ? rot : 0u;
    for (uint32_t i = 0; i < nw; ++i) {
        *reinterpret_cast<uint32_t *>(img + img_pos(d0 + 4u * w)) =
            __builtin_amdgcn_alignbyte(s32[q0 + w + 1], s32[q0 + w], sh);
        w = w + 1u == nw ? 0u : w + 1u;
    }
    for (uint32_t i = 0; i < t; ++i) img[img_pos(dpos + h + 4u * nw + i)] = pim[spos + h + 4u * nw + i];
}

// the per-message path: header stores + wave-strided command copy
__device__ __forceinline__ void entry_direct(uint8_t *ring, const uint8_t *pay, uint32_t k, uint32_t lane, uint64_t idx,
                                             uint64_t term, uint64_t m_req, uint32_t m_ct, uint64_t m_doff, uint32_t s_v,
                                             uint32_t m_clen)
{
    if (lane == k) write_csm_header(ring + s_v, idx, term, m_req, m_ct & 0xFFFFu, (m_ct >> 16) & 0xFFu);
    copy_cmds(ring, pay, k, k + 1, m_doff, s_v, m_clen, lane);
}

__device__ __forceinline__ uint64_t span_write(uint8_t *ring, __amdgpu_buffer_rsrc_t rrs,
                                           const uint8_t *pay, uint64_t pb, uint32_t kk, uint32_t kl, uint32_t lane,
                                           uint64_t idx0, const uint8_t *tp, uint64_t term, uint64_t m_req,
                                           uint32_t m_ct, uint64_t m_doff, uint32_t s_v, uint32_t m_clen, uint8_t *img,
                                           uint8_t *pim
                                           )
{
    // tp: the tail entry whose idx + 1 is idx0 (NULL: idx0 is known).  Its
    // three dwords are requested with the first sub-chunk's loads and
    // funnelled after their wait, so the index costs no round trip of its own.
    uint32_t t0 = 0, t1 = 0, t2 = 0, tsh = 0;
    bool t_pending = false;
    if (tp) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>((uintptr_t)tp & ~(uintptr_t)3);
        tsh = (uint32_t)(uintptr_t)tp & 3u;
        t0 = w[0];
        t1 = w[1];
        t2 = w[2];
        t_pending = true;
    }
    auto take_idx = [&]() {
        if (t_pending) {
            asm volatile("" : "+v"(t0), "+v"(t1), "+v"(t2));
            idx0 = ((uint64_t)__builtin_amdgcn_alignbyte(t1, t0, tsh) |
                    ((uint64_t)__builtin_amdgcn_alignbyte(t2, t1, tsh) << 32)) + 1;
            t_pending = false;
        }
    };
    const bool in_c = lane >= kk && lane < kl;
    const uint32_t el = kHdr + m_clen, nb = 2u + m_clen, sa = (uint32_t)m_doff & 3u;
    const uint32_t pimg = in_c ? 4u * ((sa + nb + 3u) >> 2) : 0u;
    const uint32_t px = wave_scan_incl(pimg);   // inclusive prefix of the command images
    const uint32_t px_ex = px - pimg;
    // a command that follows its predecessor in the payload array
    const uint64_t m_end = m_doff + nb;
    const uint64_t prev_end = wave_shr1_64(m_end);
    const uint64_t contig = __ballot(lane > kk && lane < kl && m_doff == prev_end);
    const uint64_t edge = __ballot(in_c && m_end > (pb & ~3ull));
    uint32_t k0 = kk;
    while (k0 < kl) {
        const uint32_t A0 = (uint32_t)__builtin_amdgcn_readlane(s_v, k0) & ~15u;
        const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane(px_ex, k0);
        const uint64_t stopm = __ballot(lane >= k0 && lane < kl &&
                                        (s_v + el - A0 > kSpanLds || px - p0 > kPayLds || ((edge >> lane) & 1ull)));
        const uint32_t k1 = stopm ? min(kl, (uint32_t)__builtin_ctzll(stopm)) : kl;
        if (k1 == k0) {
            take_idx();
            entry_direct(ring, pay, k0, lane, idx0 + (k0 - kk), term, m_req, m_ct, m_doff, s_v, m_clen);
            ++k0;
            continue;
        }
        // the sub-chunk's commands through one descriptor based at their
        // lowest dword (32-bit offsets whatever the payload array's size).
        // Back to back in the payload array (one run): the first command's
        // start and the last one's end; else a reduction over the lanes.
        const uint64_t inner = (k1 - k0 > 1) ? (((~0ull) >> (64 - (k1 - k0 - 1))) << (k0 + 1)) : 0ull;
        const bool run = (contig & inner) == inner;
        uint64_t mn, mx;
        if (run) {
            mn = rl64c(m_doff, k0);
            mx = rl64c(m_end, k1 - 1);
        } else {
            const bool mine = lane >= k0 && lane < k1;
            mn = mine ? m_doff : ~0ull;
            mx = mine ? m_end : 0ull;
#pragma unroll
            for (int d = 1; d < 64; d <<= 1) {
                const uint64_t a = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(mn >> 32), d) << 32) |
                                   (uint32_t)__shfl_xor((int)(uint32_t)mn, d);
                const uint64_t z = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(mx >> 32), d) << 32) |
                                   (uint32_t)__shfl_xor((int)(uint32_t)mx, d);
                mn = a < mn ? a : mn;
                mx = z > mx ? z : mx;
            }
            mn = uni64(mn);
            mx = uni64(mx);
        }
        const uint64_t sbase = mn & ~3ull;
        if (mx - sbase >= (1ull << 30)) {   // commands too far apart for one descriptor
            take_idx();
            entry_direct(ring, pay, k0, lane, idx0 + (k0 - kk), term, m_req, m_ct, m_doff, s_v, m_clen);
            ++k0;
            continue;
        }
        const uint64_t prem = pb - sbase;
        const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t *>(pay + sbase), (short)0, (int)(prem < (1ull << 30) ? prem : (1ull << 30)), 0x00020000);
        const uint32_t src = (uint32_t)(m_doff - sbase);
        const uint32_t A1 = ((uint32_t)__builtin_amdgcn_readlane(s_v, k1 - 1) +
                             (uint32_t)__builtin_amdgcn_readlane(el, k1 - 1) + 15u) & ~15u;
        const uint32_t npc = (A1 - A0) >> 4;
        // ---- 1. ring span and command bytes -> LDS, no wait in between ----
        for (uint32_t c = 0; c < npc; c += 64u)
            if (c + lane < npc)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rrs, img + img_pos(16u * c), 16, A0 + 16u * (c + lane), 0, 0, 0);
        // the sub-chunk's commands lie back to back in the payload array: one
        // run of dwords; else a run per command
        const uint32_t s0 = (uint32_t)__builtin_amdgcn_readlane(src, k0) & ~3u;
        if (run) {
            const uint32_t nd = ((uint32_t)__builtin_amdgcn_readlane(src + nb, k1 - 1) - s0 + 3u) >> 2;
            // the run as 16-B pieces, a quarter of the dword loads (the last
            // may read up to 12 bytes past it: into the 16-B pad of the command
            // image, or zeros past the array through the range check)
            const uint32_t n16 = (nd + 3u) >> 2;
            for (uint32_t c = 0; c < n16; c += 64u)
                if (c + lane < n16) __builtin_amdgcn_raw_ptr_buffer_load_lds(prs, pim + 16u * c, 16, s0 + 16u * (c + lane), 0, 0, 0);
        } else {
            for (uint32_t k = k0; k < k1; ++k) {
                const uint32_t sk = (uint32_t)__builtin_amdgcn_readlane(src, k);
                const uint32_t nd = ((sk & 3u) + (uint32_t)__builtin_amdgcn_readlane(nb, k) + 3u) >> 2;
                const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(px_ex, k) - p0;
                for (uint32_t c = 0; c < nd; c += 64u)
                    if (c + lane < nd)
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(prs, pim + lo + 4u * c, 4, (sk & ~3u) + 4u * (c + lane), 0, 0, 0);
            }
        }
        __builtin_amdgcn_s_waitcnt(0);        // every piece landed in LDS
        asm volatile("" ::: "memory");
        take_idx();
        // ---- 2. lane k builds entry k in the image ----
        if (lane >= k0 && lane < k1) {
            const uint32_t e = s_v - A0;
            // header bytes from cut on lie past a 1-KiB boundary: 32 B further
            uint8_t *const he = img + img_pos(e);
            const uint32_t cut = 1024u - (e & 1023u);
            write_csm_header_at([he, cut](uint32_t o) { return he + o + (o >= cut ? 32u : 0u); }, idx0 + (lane - kk), term,
                                m_req, m_ct & 0xFFFFu, (m_ct >> 16) & 0xFFu);
            const uint32_t spos = run ? src - s0 : px_ex - p0 + (src & 3u);
            lds_funnel(img, e + kData, pim, spos, nb, lane & 7u);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- 3. the span back to the ring, 16-B coalesced stores ----
        const uint4 *img16 = reinterpret_cast<const uint4 *>(img);
        for (uint32_t c = 0; c < npc; c += 64u)
            if (c + lane < npc) *reinterpret_cast<uint4 *>(ring + A0 + 16u * (c + lane)) = img16[c + lane + 2u * ((c + lane) >> 6)];
        asm volatile("" ::: "memory");
        k0 = k1;
    }
    take_idx();
    return idx0;
}

// Two fast prefixes around the ring's end in ONE load -> build -> store round
// trip (a group whose batch wraps: before, span_write ran twice, the second
// sub-chunk's loads waiting for the first's stores).  Messages [kk, kw) are
// placed from the current end up to len (lane k's s_v: its ring offset),
// message kw wraps to 0 -- with a ghost header at gpos when its header fits
// before len but the entry does not (dare_log.h:500-515), gpos = ~0 when the
// header does not fit either -- and [kw, kl) are placed from 0 (s_v: offsets
// from 0).  The ghost header is built in the first span's image.  Returns
// false, having loaded and written nothing, when both spans, their commands
// and the ghost do not fit one sub-chunk (the caller then appends the two
// prefixes one after the other); the caller has checked the spans do not
// overlap.  Bytes log_append_entry never writes keep their values, as in
// span_write.
__device__ __forceinline__ bool span_write_wrap(uint8_t *ring, __amdgpu_buffer_rsrc_t rrs, const uint8_t *pay,
                                                uint64_t pb, uint32_t kk, uint32_t kw, uint32_t kl, uint32_t lane,
                                                uint64_t &idx0, const uint8_t *tp, uint64_t term, uint64_t m_req,
                                                uint32_t m_ct, uint64_t m_doff, uint32_t s_v, uint32_t m_clen,
                                                uint32_t gpos, uint32_t A0, uint32_t A1, uint32_t B1, uint8_t *img,
                                                uint8_t *pim)
{
    const bool in_c = lane >= kk && lane < kl;
    const uint32_t nb = 2u + m_clen, sa = (uint32_t)m_doff & 3u;
    const uint32_t pimg = in_c ? 4u * ((sa + nb + 3u) >> 2) : 0u;
    const uint32_t px = wave_scan_incl(pimg);
    const uint32_t px_ex = px - pimg;
    const uint64_t m_end = m_doff + nb;
    const uint64_t prev_end = wave_shr1_64(m_end);
    const uint64_t contig = __ballot(lane > kk && lane < kl && m_doff == prev_end);
    const uint64_t edge = __ballot(in_c && m_end > (pb & ~3ull));
    const uint32_t nA = (A1 - A0) >> 4, nB = B1 >> 4;
    if (edge || 16u * (nA + nB) > kSpanLds || (uint32_t)__builtin_amdgcn_readlane(px, kl - 1) > kPayLds) return false;
    const uint64_t inner = (kl - kk > 1) ? (((~0ull) >> (64 - (kl - kk - 1))) << (kk + 1)) : 0ull;
    const bool run = (contig & inner) == inner;
    uint64_t mn, mx;
    if (run) {
        mn = rl64c(m_doff, kk);
        mx = rl64c(m_end, kl - 1);
    } else {
        mn = in_c ? m_doff : ~0ull;
        mx = in_c ? m_end : 0ull;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t a = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(mn >> 32), d) << 32) |
                               (uint32_t)__shfl_xor((int)(uint32_t)mn, d);
            const uint64_t z = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(mx >> 32), d) << 32) |
                               (uint32_t)__shfl_xor((int)(uint32_t)mx, d);
            mn = a < mn ? a : mn;
            mx = z > mx ? z : mx;
        }
        mn = uni64(mn);
        mx = uni64(mx);
    }
    const uint64_t sbase = mn & ~3ull;
    if (mx - sbase >= (1ull << 30)) return false;          // commands too far apart for one descriptor
    // the tail entry's index with the loads (span_write)
    uint32_t t0 = 0, t1 = 0, t2 = 0, tsh = 0;
    if (tp) {
        const uint32_t *w = reinterpret_cast<const uint32_t *>((uintptr_t)tp & ~(uintptr_t)3);
        tsh = (uint32_t)(uintptr_t)tp & 3u;
        t0 = w[0];
        t1 = w[1];
        t2 = w[2];
    }
    const uint64_t prem = pb - sbase;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t *>(pay + sbase), (short)0, (int)(prem < (1ull << 30) ? prem : (1ull << 30)), 0x00020000);
    const uint32_t src = (uint32_t)(m_doff - sbase);
    // ---- 1. both ring spans and the command bytes -> LDS, no wait between ----
    // (image piece p: the first span's piece p, then the second's p - nA; one
    // buffer_load ... lds fills one KiB of the padded image, so the loads go
    // by image KiB with each lane's ring offset from its own span)
    const uint32_t np = nA + nB;
    for (uint32_t c = 0; c < np; c += 64u) {
        const uint32_t pc = c + lane;
        if (pc < np)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rrs, img + img_pos(16u * c), 16,
                                                     pc < nA ? A0 + 16u * pc : 16u * (pc - nA), 0, 0, 0);
    }
    const uint32_t s0 = (uint32_t)__builtin_amdgcn_readlane(src, kk) & ~3u;
    const uint32_t p0 = (uint32_t)__builtin_amdgcn_readlane(px_ex, kk);
    if (run) {
        const uint32_t nd = ((uint32_t)__builtin_amdgcn_readlane(src + nb, kl - 1) - s0 + 3u) >> 2;
        const uint32_t n16 = (nd + 3u) >> 2;
        for (uint32_t c = 0; c < n16; c += 64u)
            if (c + lane < n16) __builtin_amdgcn_raw_ptr_buffer_load_lds(prs, pim + 16u * c, 16, s0 + 16u * (c + lane), 0, 0, 0);
    } else {
        for (uint32_t k = kk; k < kl; ++k) {
            const uint32_t sk = (uint32_t)__builtin_amdgcn_readlane(src, k);
            const uint32_t nd = ((sk & 3u) + (uint32_t)__builtin_amdgcn_readlane(nb, k) + 3u) >> 2;
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(px_ex, k) - p0;
            for (uint32_t c = 0; c < nd; c += 64u)
                if (c + lane < nd)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(prs, pim + lo + 4u * c, 4, (sk & ~3u) + 4u * (c + lane), 0, 0, 0);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);        // every piece landed in LDS
    asm volatile("" ::: "memory");
    if (tp) {
        asm volatile("" : "+v"(t0), "+v"(t1), "+v"(t2));
        idx0 = ((uint64_t)__builtin_amdgcn_alignbyte(t1, t0, tsh) | ((uint64_t)__builtin_amdgcn_alignbyte(t2, t1, tsh) << 32)) + 1;
    }
    // ---- 2. lane k builds entry k in its span's image; lane kw the ghost ----
    auto build = [&](uint32_t e, bool ghost) {
        uint8_t *const he = img + img_pos(e);
        const uint32_t cut = 1024u - (e & 1023u);
        write_csm_header_at([he, cut](uint32_t o) { return he + o + (o >= cut ? 32u : 0u); }, idx0 + (lane - kk), term,
                            m_req, m_ct & 0xFFFFu, (m_ct >> 16) & 0xFFu);
        if (ghost) {                    // cmd.len, the ghost's only data bytes (write_header, dmode 1)
            img[img_pos(e + kData)] = (uint8_t)m_clen;
            img[img_pos(e + kData + 1)] = (uint8_t)(m_clen >> 8);
        }
    };
    if (in_c) {
        const uint32_t e = lane < kw ? s_v - A0 : 16u * nA + s_v;
        build(e, false);
        const uint32_t spos = run ? src - s0 : px_ex - p0 + (src & 3u);
        lds_funnel(img, e + kData, pim, spos, nb, lane & 7u);
        if (lane == kw && gpos != ~0u) build(gpos - A0, true);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // ---- 3. both spans back to the ring, 16-B coalesced stores ----
    const uint4 *img16 = reinterpret_cast<const uint4 *>(img);
    for (uint32_t c = 0; c < np; c += 64u) {
        const uint32_t pc = c + lane;
        if (pc < np)
            *reinterpret_cast<uint4 *>(ring + (pc < nA ? A0 + 16u * pc : 16u * (pc - nA))) = img16[pc + 2u * (pc >> 6)];
    }
    asm volatile("" ::: "memory");
    return true;
}

// One group, wave-wide: log_append_entry over the group's queued messages,
// fast prefixes assembled in LDS (span_write) and the general step otherwise.
// c_row is the group's state row (lanes 0..7: a row, or its dare_log_t
// header), c_req / c_doff / c_ct / c_clen its first 64 message records with
// their cmd.len (lane k: message k).  on_first() runs once: after the first
// fast prefix's loads landed, or at the end (append_kernel requests the next
// group's first cmd.len there).
template <typename OnFirst>
__device__ __forceinline__ void append_group(const apus_batch_t &b, const apus_append_in_t &in,
                                             const apus_append_out_t &o, uint64_t *stats, uint64_t g, uint32_t lane,
                                             uint8_t *img, uint8_t *pim, uint64_t c_row, uint64_t c_req,
                                             uint64_t c_doff, uint32_t c_ct, uint32_t c_clen, OnFirst on_first
                                             )
{
    const uint64_t stride = b.ring_stride, cap = ring_cap(b), pb = in.payload_bytes;
    const uint32_t max_e = in.max_entries;
    // fast-prefix entries are assembled in LDS (span_write): command dwords
    // are read from a 4-B aligned payload array; ring spans are read and
    // written in 16-B pieces (the last one may reach into the ring's tail pad,
    // below ring_stride: read and written unchanged)
    const bool span_ok = ((uintptr_t)in.payload & 3u) == 0 && ((((uintptr_t)b.ring) | stride) & 15u) == 0 &&
                         stride < (1ull << 31);
    apus_group_state_t st;
    st.head = rl64c(c_row, 0);
    st.apply = rl64c(c_row, 1);
    st.commit = rl64c(c_row, 2);
    st.end = rl64c(c_row, 3);
    st.tail = rl64c(c_row, 4);
    st.len = rl64c(c_row, (b.flags & APUS_BATCH_LOG_IMAGE) ? 7 : 5);      // len@40 (row) / @56 (header)
    const uint64_t len = st.len, head = st.head;
    uint64_t end = st.end, tail = st.tail;
    const uint32_t n = in.n_entries ? min(in.n_entries[g], max_e) : max_e;
    const uint64_t term = in.term ? in.term[g] : (b.sid[g] >> 9);     // SID_GET_TERM
    uint32_t prev_head = b.prev_head ? b.prev_head[g] : 0u;
    uint64_t last_ret = o.last_idx ? o.last_idx[g] : 0ull;
    uint8_t *ring = b.ring + g * stride;
    const apus_append_entry_t *q = in.entries + g * max_e;
    // offsets the device could not honour without reading or writing
    // outside the ring (undefined in the reference) stop the group
    bool stop = !(len >= kHdr && len <= cap && end <= len && tail <= len);
    bool bad = stop && n > 0;
    uint64_t known_off = ~0ull, known_idx = 0;
    bool fired = false;                     // on_first() called

    for (uint32_t c0 = 0; c0 < n; c0 += 64) {
        const uint32_t cn = min(64u, n - c0);
        // lane k holds message c0 + k
        uint64_t m_req = 0, m_doff = 0;
        uint32_t m_ct = 0, m_clen = 0;
        if (c0 == 0) {
            if (lane < cn) {                                  // prefetched a group ago
                m_req = c_req;
                m_doff = c_doff;
                m_ct = c_ct;
                m_clen = c_clen;
            }
        } else if (lane < cn) {
            const apus_append_entry_t r = q[c0 + lane];
            m_req = r.req_id;
            m_doff = r.data_off;
            m_ct = (uint32_t)r.clt_id | ((uint32_t)r.type << 16);
            if (csm_type(r.type) && r.data_off <= pb && pb - r.data_off >= 2)
                m_clen = ld_u16(in.payload + r.data_off);
        }
        uint64_t idx_v = 0;
        const bool m_ok = csm_type(m_ct >> 16) && m_doff <= pb && pb - m_doff >= 2u + m_clen &&
                          (uint64_t)kHdr + m_clen <= len;
        const uint64_t ok_m = __ballot(m_ok);
        uint32_t kk = 0;
        while (kk < cn && !stop) {
            // ---- fast prefix: messages kk.. that are valid CSM-class
            // commands landing in [end, len) without a wrap, a ghost header
            // or a full log (no start equals head), the tail being known.
            // Placement is an exclusive prefix sum of the entry lengths and
            // the index of entry k is idx0 + k: log_append_entry
            // (dare_log.h:487-550) with every branch but the straight one
            // provably not taken.
            uint32_t nf = 0, s_v = 0, x = 0, before = 0;
            if (tail != len && end != len && len < (1ull << 31)) {
                const bool in_c = lane >= kk && lane < cn;
                const uint32_t el = in_c ? kHdr + m_clen : 0u;
                x = wave_scan_incl(el);
                before = kk ? (uint32_t)__builtin_amdgcn_readlane(x, kk - 1) : 0u;
                s_v = (uint32_t)end + (x - el - before);
                const bool ok = in_c && m_ok && (uint64_t)s_v + el <= len && (uint64_t)s_v != head;
                const uint64_t fail = __ballot(!ok) & (~0ull << kk);
                nf = (fail ? (uint32_t)__builtin_ctzll(fail) : 64u) - kk;
            }
            if (nf) {
                const uint32_t kl = kk + nf;                             // last + 1
                uint64_t idx0 = 1;
                const uint8_t *tp = nullptr;                             // the tail entry, idx not known
                if (dist(end, len, tail) != 0) {                          // end != len already
                    const uint64_t off = len - tail < kHdr ? 0 : tail;
                    if (off == known_off) idx0 = known_idx + 1;
                    else tp = ring + off;
                }
                // A batch that wraps at message kl: the prefix after the wrap
                // (from 0) in the same round trip when the wrap is one the
                // general step below would take exactly so (the conditions of
                // "the wrap of a valid message" there, evaluated after this
                // prefix) and the second span ends before the first begins
                uint32_t kl2 = kl, gpos = ~0u, A1 = 0, B1 = 0, sv2 = s_v;
                if (span_ok && kl < cn && ((ok_m >> kl) & 1ull) && head != 0) {
                    const uint32_t s_w = (uint32_t)__builtin_amdgcn_readlane(s_v, kl);
                    const uint32_t c_w = (uint32_t)__builtin_amdgcn_readlane(m_clen, kl);
                    const uint32_t endA = s_w;                               // the prefix's end
                    const uint32_t tailA = (uint32_t)__builtin_amdgcn_readlane(s_v, kl - 1);
                    if ((uint64_t)s_w + kHdr + c_w > len && (uint64_t)s_w != head && endA != len && endA != head &&
                        tailA != 0) {
                        const bool ghost = len - endA >= kHdr;               // header fits, the entry does not
                        gpos = ghost ? endA : ~0u;
                        const uint32_t before2 = (uint32_t)__builtin_amdgcn_readlane(x, kl - 1);
                        const bool in_b = lane >= kl && lane < cn;
                        const uint32_t el = in_b ? kHdr + m_clen : 0u;
                        const uint32_t sb = x - el - before2;                // offset from 0
                        const bool okb = in_b && m_ok && (uint64_t)sb + el <= len && (uint64_t)sb != head;
                        const uint64_t failb = __ballot(!okb) & (~0ull << kl);
                        const uint32_t kb = failb ? (uint32_t)__builtin_ctzll(failb) : 64u;
                        if (kb > kl) {
                            const uint32_t bend = (uint32_t)__builtin_amdgcn_readlane(sb + el, kb - 1);
                            const uint32_t A0 = (uint32_t)__builtin_amdgcn_readlane(s_v, kk) & ~15u;
                            A1 = (max(endA, ghost ? endA + kData + 2u : endA) + 15u) & ~15u;
                            B1 = (bend + 15u) & ~15u;
                            if (B1 <= A0) {
                                kl2 = kb;
                                sv2 = lane >= kl ? sb : s_v;
                            }
                        }
                    }
                }
                if (span_ok && kl2 > kl) {
                    const uint32_t A0 = (uint32_t)__builtin_amdgcn_readlane(s_v, kk) & ~15u;
                    if (span_write_wrap(ring, ring_rsrc_of(ring, (uint32_t)((cap + 15u) & ~15ull)), in.payload, pb, kk,
                                        kl, kl2, lane, idx0, tp, term, m_req, m_ct, m_doff, sv2, m_clen, gpos, A0, A1, B1,
                                        img, pim)) {
                        if (!fired) {
                            on_first();
                            fired = true;
                        }
                        if (lane >= kk && lane < kl2) idx_v = idx0 + (lane - kk);
                        prev_head = 0;                                   // dare_log.h:478-481
                        const uint32_t lb = (uint32_t)__builtin_amdgcn_readlane(sv2, kl2 - 1);
                        tail = lb;
                        end = lb + (uint32_t)__builtin_amdgcn_readlane(kHdr + m_clen, kl2 - 1);
                        known_off = lb;
                        known_idx = idx0 + (kl2 - kk) - 1;
                        last_ret = known_idx;
                        kk = kl2;
                        continue;
                    }
                }
                if (span_ok) {
                    idx0 = span_write(ring, ring_rsrc_of(ring, (uint32_t)((cap + 15u) & ~15ull)), in.payload, pb, kk, kl,
                                      lane, idx0, tp, term, m_req, m_ct, m_doff, s_v, m_clen, img, pim
                                      );
                    if (!fired) {
                        on_first();                            // e.g. the next group's first cmd.len, early
                        fired = true;
                    }
                } else {
                    if (tp) idx0 = ld_u64(tp) + 1;
                    // headers: lane k writes entry k's (sender@27 and 41..47 untouched)
                    if (lane >= kk && lane < kl)
                        write_csm_header(ring + s_v, idx0 + (lane - kk), term, m_req, m_ct & 0xFFFFu,
                                         (m_ct >> 16) & 0xFFu);
                    copy_cmds(ring, in.payload, kk, kl, m_doff, s_v, m_clen, lane);
                }
                if (lane >= kk && lane < kl) idx_v = idx0 + (lane - kk);
                prev_head = 0;                                           // dare_log.h:478-481
                const uint64_t last = (uint64_t)(uint32_t)__builtin_amdgcn_readlane(s_v, kl - 1);
                tail = last;
                end += (uint32_t)__builtin_amdgcn_readlane(x, kl - 1) - before;
                known_off = last;
                known_idx = idx0 + nf - 1;
                last_ret = known_idx;
                kk = kl;
                continue;
            }
            // ---- the wrap of a valid message at the end of the ring ----
            // log_append_entry (dare_log.h:500-515) with the tail's index
            // known: the entry goes to 0 (a ghost header stays at end when
            // the header fits but the entry does not), and the next fast
            // prefix starts there.  Taken only where that prefix computes
            // what the reference does: end != len and the tail's distance
            // nonzero at end and at 0 (the same tail index), head != 0 (the
            // reference's second full test after a ghost, and no entry
            // written over head at 0 without a test).
            if (span_ok && ((ok_m >> kk) & 1ull) && tail != len && end != len && end != head && head != 0 &&
                tail != 0 && len < (1ull << 31) && dist(end, len, tail) != 0) {
                const uint32_t clen = (uint32_t)__builtin_amdgcn_readlane(m_clen, kk);
                if (len - end < kHdr) {                                  // the header does not fit
                    end = 0;
                    continue;
                }
                const uint64_t off = len - tail < kHdr ? 0 : tail;
                if (len - end < (uint64_t)kHdr + clen && off == known_off) {
                    const uint64_t req = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(m_req >> 32), kk) << 32) |
                                         (uint32_t)__builtin_amdgcn_readlane((uint32_t)m_req, kk);
                    const uint32_t ct = (uint32_t)__builtin_amdgcn_readlane(m_ct, kk);
                    write_header(ring + end, lane, known_idx + 1, term, req, ct & 0xFFFFu, (ct >> 16) & 0xFFu, 1u,
                                 clen, nullptr);                         // the ghost header
                    end = 0;
                    continue;
                }
            }
            // ---- one message the general way ----
            do {
                const uint64_t req = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(m_req >> 32), kk) << 32) |
                                     (uint32_t)__builtin_amdgcn_readlane((uint32_t)m_req, kk);
                const uint64_t doff = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(m_doff >> 32), kk) << 32) |
                                      (uint32_t)__builtin_amdgcn_readlane((uint32_t)m_doff, kk);
                const uint32_t ct = (uint32_t)__builtin_amdgcn_readlane(m_ct, kk);
                const uint32_t clt = ct & 0xFFFFu, type = (ct >> 16) & 0xFFu;
                const bool csm = csm_type(type);
                const uint32_t clen = csm ? (uint32_t)__builtin_amdgcn_readlane(m_clen, kk) : 0u;
                const uint64_t need = type == APUS_CONFIG ? 16u : type == APUS_HEAD ? 8u : csm ? 2u + clen : 0u;
                if ((need && (doff > pb || pb - doff < need)) || (csm && (uint64_t)kHdr + clen > len)) {
                    stop = bad = true;
                    break;
                }
                const uint8_t *dsrc = in.payload + doff;

                if (type != APUS_HEAD) prev_head = 0;                    // dare_log.h:478-481
                if (tail == len) {                                       // dare_log.h:484-486
                    st.end = end;
                    st.tail = tail;
                    tail = device_get_tail(RingView{ ring, end, len, len }, st);   // len <= ring_cap (checked)
                }
                // log_get_entry(log, &tail): the last entry's index (dare_log.h:487-489)
                uint64_t idx = 1;
                if (end != len && dist(end, len, tail) != 0) {
                    const uint64_t off = len - tail < kHdr ? 0 : tail;
                    idx = (off == known_off ? known_idx : ld_u64(ring + off)) + 1;
                }
                // log_add_new_entry (dare_log.h:214-221)
                if (end == head) { last_ret = 0; break; }             // the LOG is full
                uint64_t loc = (end == len || len - end < kHdr) ? 0 : end;
                write_header(ring + loc, lane, idx, term, req, clt, type,
                             csm ? 1u : type == APUS_CONFIG ? 2u : type == APUS_HEAD ? 3u : 0u, clen, dsrc);
                if (len - end < kHdr) end = 0;                            // dare_log.h:500-502
                uint64_t elen = kHdr;
                if (csm) {
                    elen = (uint64_t)kHdr + clen;
                    if (len - end < elen) {
                        // a ghost header stays at loc; the entry restarts at 0
                        end = 0;
                        if (end == head) { last_ret = 0; break; }
                        loc = 0;
                        write_header(ring, lane, idx, term, req, clt, type, 1u, clen, dsrc);
                    }
                    for (uint32_t j = lane; j < clen; j += 64) ring[loc + kData + 2 + j] = dsrc[2 + j];
                }
                tail = end;                                              // dare_log.h:547-550
                end += elen;
                known_off = loc;
                known_idx = idx;
                last_ret = idx;
                if (lane == kk) idx_v = idx;
            } while (0);
            ++kk;
        }
        if (o.idx && lane < cn) o.idx[g * max_e + c0 + lane] = idx_v;
    }
    if (lane == 0) {
        if (n) {
            uint64_t *offs = offsets_of(b, g);
            offs[kOffEnd] = end;
            offs[kOffTail] = tail;
        }
        if (b.prev_head) b.prev_head[g] = (uint8_t)prev_head;
        if (o.last_idx) o.last_idx[g] = last_ret;
        if (bad) atomicAdd((unsigned long long *)&stats[APUS_STAT_CORRUPT], 1ull);
    }
    if (!fired) on_first();
}

// LIST: the groups append_quad_kernel handed back, one slice per wave of the
// same grid (list[gw] of them at list[nw + gw * per ...]); else every group.
// DYN (!LIST): groups in chunks of kAppChunk consecutive ids; every chunk
// after a wave's first is handed out by an atomic counter (*ctr, zeroed before
// the launch), the next chunk's id requested a chunk ahead.  (One id per group
// from the counter ran 2.3x slower at C2: 2^20 returning atomics on one word.)
constexpr uint32_t kAppChunk = 16;
template <bool LIST, bool DYN>
__global__ void __launch_bounds__(256) append_kernel(const apus_batch_t b, const apus_append_in_t in,
                                                     const apus_append_out_t o, uint64_t *stats, const uint32_t *list,
                                                     uint32_t nw, uint32_t per, uint32_t *ctr)
{
    __shared__ __attribute__((aligned(16))) uint8_t s_img[kAppendWaves][kSpanImg];
    __shared__ __attribute__((aligned(16))) uint8_t s_pim[kAppendWaves][kPayLds + 16];
    const uint32_t lane = lane_id();
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint64_t G = b.n_groups, pb = in.payload_bytes;
    const uint32_t max_e = in.max_entries;
    const uint64_t gw = (uint64_t)blockIdx.x * kAppendWaves + wv;
    // iteration i appends group grp(i), i from i0 by step while i < lim
    const uint32_t *ids = LIST ? list + nw + gw * per : nullptr;
    const uint64_t i0 = LIST ? 0 : gw, step = LIST ? 1 : (uint64_t)gridDim.x * kAppendWaves,
                   lim = LIST ? (gw < nw ? list[gw] : 0u) : G;
    auto grp = [&](uint64_t i) -> uint64_t { return LIST ? (uint64_t)ids[i] : i; };
    // The next group's state row (lanes 0..7, one u64 each) and its first
    // 64 message records are requested while the current group is worked on;
    // their cmd.len loads after the current group's first fast prefix.
    const uint32_t pre_n = min(64u, max_e);
    uint64_t p_row = 0, p_req = 0, p_doff = 0;
    uint32_t p_ct = 0, p_clen = 0;
    auto load_next = [&](uint64_t i) {
        p_row = 0; p_req = 0; p_doff = 0; p_ct = 0;
        if (i < lim) {
            const uint64_t gg = grp(i);
            if (lane < 8) p_row = offsets_of(b, gg)[lane];     // a row, or a dare_log_t header
            if (lane < pre_n) {
                const apus_append_entry_t r = in.entries[gg * max_e + lane];
                p_req = r.req_id;
                p_doff = r.data_off;
                p_ct = (uint32_t)r.clt_id | ((uint32_t)r.type << 16);
            }
        }
    };
    auto load_clen = [&](uint64_t doff, uint32_t ct) -> uint32_t {
        return (csm_type(ct >> 16) && doff <= pb && pb - doff >= 2) ? ld_u16(in.payload + doff) : 0u;
    };
    // DYN: chunk c covers groups [c K, c K + K); chunks [0, nw) are the
    // waves' first, the rest come from the counter.  nxc: the chunk after the
    // current one (uniform); nxv: lane 0's pending counter value for the one after
    const uint64_t nwv = (uint64_t)gridDim.x * kAppendWaves;
    uint64_t nxc = 0;
    uint32_t nxv = 0;
    if (DYN) {
        if (lane == 0) nxv = atomicAdd(ctr, 1u);
        nxc = nwv + __builtin_amdgcn_readfirstlane(nxv);
        if (lane == 0) nxv = atomicAdd(ctr, 1u);
    }
    // (DYN: i0 = gw is the first chunk's index; groups are chunk * K + k)
    const uint64_t cur = DYN ? (uint64_t)gw * kAppChunk : i0;
    load_next(cur);
    p_clen = load_clen(p_doff, p_ct);
    for (uint64_t i = cur; i < lim; ) {
        // the group after this one
        uint64_t nxt;
        if (DYN) {
            if ((i + 1) % kAppChunk != 0) {
                nxt = i + 1;
            } else {
                nxt = nxc * kAppChunk;
                nxc = nwv + __builtin_amdgcn_readfirstlane(nxv);
                if (lane == 0) nxv = atomicAdd(ctr, 1u);
            }
        } else {
            nxt = i + step;
        }
        const uint64_t g = grp(i);
        const uint64_t c_row = p_row, c_req = p_req, c_doff = p_doff;
        const uint32_t c_ct = p_ct, c_clen = p_clen;
        load_next(nxt);
        append_group(b, in, o, stats, g, lane, s_img[wv], s_pim[wv], c_row, c_req, c_doff, c_ct, c_clen,
                     [&]() { p_clen = load_clen(p_doff, p_ct); }
                     );
        i = nxt;
    }
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src)
{
    return ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(v >> 32), (int)src) << 32) |
           (uint32_t)__shfl((int)(uint32_t)v, (int)src);
}

// ---------------------------------------------------------------------------
// Short batches (max_entries <= 16, e.g. C5's 16-entry groups): four groups
// per wave, 16 lanes each (lane 16 q + k holds message k of the wave's group
// q).  append_kernel pays a group's round trips -- the tail entry's index,
// the span and command loads, the next group's cmd.len -- once per group
// whatever its length; here one wait serves four groups.  The wave places the
// four batches (segmented prefix sums), issues every group's span, command and
// tail-index loads, waits once, builds the four entry images in LDS and writes
// them back.  A group goes this way only when its whole batch is one fast
// prefix in append_group's sense (valid CSM-class commands landing in
// [end, len) with no wrap, no ghost header and no start at head; the tail
// known) whose span and command images fit a quarter of the wave's LDS;
// every other group is appended afterwards by append_group, by the whole wave.
// Same results as append_kernel (tests/test_append.py runs both).
// ---------------------------------------------------------------------------
constexpr uint32_t kQuadSpan = 2080;                    // ring-span bytes per group (130 pieces)
constexpr uint32_t kQuadImg = kQuadSpan + 64;           // its image, padded 32 B after each KiB
constexpr uint32_t kQuadPay = kPayLds / 4;              // command-image bytes per group
static_assert(4 * kQuadImg <= kSpanImg && 4 * kQuadPay <= kPayLds && kQuadImg % 16 == 0 && kQuadPay % 16 == 0,
              "four group slots fit the wave's LDS images");

__global__ void __launch_bounds__(256) append_quad_kernel(const apus_batch_t b, const apus_append_in_t in,
                                                          const apus_append_out_t o, uint64_t *stats, uint32_t *list,
                                                          uint32_t nw, uint32_t per)
{
    __shared__ __attribute__((aligned(16))) uint8_t s_img[kAppendWaves][kSpanImg];
    __shared__ __attribute__((aligned(16))) uint8_t s_pim[kAppendWaves][kPayLds + 16];
    const uint32_t lane = lane_id(), q = lane >> 4, k = lane & 15u, sl = lane & ~15u;   // sl: the segment's lane 0
    const uint32_t wv = uni(threadIdx.x >> 6);
    uint8_t *const img = s_img[wv];
    uint8_t *const pim = s_pim[wv];
    const uint64_t G = b.n_groups, stride = b.ring_stride, cap = ring_cap(b), pb = in.payload_bytes;
    const uint32_t max_e = in.max_entries;                 // <= 16 (launch_append)
    const uint32_t cap16 = (uint32_t)((cap + 15u) & ~15ull);
    const uint32_t len_w = (b.flags & APUS_BATCH_LOG_IMAGE) ? 7u : 5u;    // len@40 (row) / @56 (header)
    const uint64_t gs = (uint64_t)gridDim.x * kAppendWaves * 4u;
    // the next four groups' state rows (lanes 16 q + 0..7), records (lane
    // 16 q + k), batch lengths and terms are requested while the current four
    // are worked on; their cmd.len after the current four's loads landed
    uint64_t p_row = 0, p_req = 0, p_doff = 0, p_term = 0;
    uint32_t p_ct = 0, p_n = 0, p_clen = 0;
    auto load_next = [&](uint64_t g0) {
        const uint64_t gg = g0 + q;
        p_row = 0; p_req = 0; p_doff = 0; p_ct = 0; p_n = 0; p_term = 0;
        if (gg < G) {
            if (k < 8) p_row = offsets_of(b, gg)[k];
            if (k < max_e) {
                const apus_append_entry_t r = in.entries[gg * max_e + k];
                p_req = r.req_id;
                p_doff = r.data_off;
                p_ct = (uint32_t)r.clt_id | ((uint32_t)r.type << 16);
            }
            p_n = in.n_entries ? min(in.n_entries[gg], max_e) : max_e;
            p_term = in.term ? in.term[gg] : (b.sid[gg] >> 9);        // SID_GET_TERM
        }
    };
    auto load_clen = [&]() {
        p_clen = (k < max_e && csm_type(p_ct >> 16) && p_doff <= pb && pb - p_doff >= 2) ? ld_u16(in.payload + p_doff)
                                                                                          : 0u;
    };
    const uint64_t gw = (uint64_t)blockIdx.x * kAppendWaves + wv;
    uint32_t *const ids = list + nw + gw * per;
    uint32_t n_def = 0;
    uint64_t g0 = gw * 4u;
    load_next(g0);
    load_clen();
    for (; g0 < G; g0 += gs) {
        const uint64_t c_row = p_row, c_req = p_req, c_doff = p_doff, term = p_term;
        const uint32_t c_ct = p_ct, c_clen = p_clen, n = p_n;
        load_next(g0 + gs);
        const uint64_t g = g0 + q;
        const uint64_t head = shfl64(c_row, sl), end = shfl64(c_row, sl + 3), tail = shfl64(c_row, sl + 4),
                       len = shfl64(c_row, sl + len_w);
        // ---- placement: the batch as one fast prefix (append_group) ----
        const bool in_c = k < n;
        const uint32_t clen = in_c ? c_clen : 0u;
        const uint32_t el = in_c ? kHdr + clen : 0u;
        const uint32_t x = row_scan_incl(el);              // inclusive prefix in the segment (a DPP row)
        const uint32_t tot = __shfl(x, sl + 15);
        const uint32_t s_v = (uint32_t)end + (x - el);
        const bool m_ok = csm_type(c_ct >> 16) && c_doff <= pb && pb - c_doff >= 2u + clen &&
                          (uint64_t)kHdr + clen <= len;
        const bool grp_ok = g < G && n > 0 && len >= kHdr && len <= cap && end <= len && tail <= len && tail != len &&
                            end != len && len < (1ull << 31);
        // the commands: one 4-B aligned base per group, one run when they lie
        // back to back in the payload array
        const uint32_t nb = 2u + clen, sa = (uint32_t)c_doff & 3u;
        const uint64_t m_end = c_doff + nb;
        const uint64_t prev_end = wave_shr1_64(m_end);     // (read where k > 0)
        uint64_t mn = in_c ? c_doff : ~0ull, mx = in_c ? m_end : 0ull;
#pragma unroll
        for (int d = 1; d < 16; d <<= 1) {
            const uint64_t a = shfl64(mn, lane ^ (uint32_t)d), z = shfl64(mx, lane ^ (uint32_t)d);
            mn = a < mn ? a : mn;
            mx = z > mx ? z : mx;
        }
        const uint64_t sbase = mn & ~3ull;
        const uint32_t pimg = in_c ? 4u * ((sa + nb + 3u) >> 2) : 0u;
        const uint32_t px = row_scan_incl(pimg);           // inclusive prefix of the command images
        const uint32_t ptot = __shfl(px, sl + 15);
        const uint64_t brk = __ballot(in_c && k > 0 && c_doff != prev_end);
        const uint64_t bad = __ballot(in_c && (!m_ok || (uint64_t)s_v + el > len || (uint64_t)s_v == head ||
                                               m_end > (pb & ~3ull)));
        const bool run = ((brk >> sl) & 0xFFFFull) == 0;
        const uint32_t A0 = (uint32_t)end & ~15u;
        const uint32_t npc = ((((uint32_t)end + tot + 15u) & ~15u) - A0) >> 4;
        const uint64_t span_c = mx - sbase;                // command bytes from the base
        const uint32_t n16 = (uint32_t)((span_c + 15u) >> 4);
        const bool fast = grp_ok && ((bad >> sl) & 0xFFFFull) == 0 && span_c < (1ull << 30) && 16u * npc <= kQuadSpan &&
                          (run ? 16ull * n16 <= kQuadPay : ptot <= kQuadPay);
        const uint64_t fm = __ballot(fast && k == 0);     // the fast groups' lane 0
        // the tail entry's index (log_get_entry(log, &tail), dare_log.h:487-489):
        // three dwords per lane of a fast group that has a tail, funnelled after the wait
        uint8_t *const ring = b.ring + g * stride;
        const bool has_tail = fast && dist(end, len, tail) != 0;
        uint32_t t0 = 0, t1 = 0, t2 = 0, tsh = 0;
        if (has_tail) {
            const uint8_t *tp = ring + (len - tail < kHdr ? 0 : tail);
            const uint32_t *w = reinterpret_cast<const uint32_t *>((uintptr_t)tp & ~(uintptr_t)3);
            tsh = (uint32_t)(uintptr_t)tp & 3u;
            t0 = w[0];
            t1 = w[1];
            t2 = w[2];
        }
        // ---- every fast group's span and commands -> its LDS slot, no wait in between ----
        const uint32_t src = (uint32_t)(c_doff - sbase);
        for (uint64_t m = fm; m; m &= m - 1) {
            const uint32_t L = (uint32_t)__builtin_ctzll(m), sq = L >> 4;
            uint8_t *const rq = b.ring + (g0 + sq) * stride;
            const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane(A0, L), np = (uint32_t)__builtin_amdgcn_readlane(npc, L);
            const __amdgpu_buffer_rsrc_t rrs = ring_rsrc_of(rq, cap16);
            uint8_t *const qimg = img + sq * kQuadImg;
            for (uint32_t c = 0; c < np; c += 64u)
                if (c + lane < np)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(rrs, qimg + img_pos(16u * c), 16, a0 + 16u * (c + lane), 0, 0, 0);
            const uint64_t sb = rl64c(sbase, L);
            const uint64_t prem = pb - sb;
            const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<uint8_t *>(in.payload + sb), (short)0, (int)(prem < (1ull << 30) ? prem : (1ull << 30)), 0x00020000);
            uint8_t *const qpim = pim + sq * kQuadPay;
            if (__builtin_amdgcn_readlane((uint32_t)run, L)) {
                // the run as 16-B pieces (the last may read up to 12 bytes past it,
                // inside the slot: 16 n16 <= kQuadPay)
                const uint32_t nn = (uint32_t)__builtin_amdgcn_readlane(n16, L);
                for (uint32_t c = 0; c < nn; c += 64u)
                    if (c + lane < nn) __builtin_amdgcn_raw_ptr_buffer_load_lds(prs, qpim + 16u * c, 16, 16u * (c + lane), 0, 0, 0);
            } else {
                const uint32_t nq = (uint32_t)__builtin_amdgcn_readlane(n, L);
                for (uint32_t j = 0; j < nq; ++j) {
                    const uint32_t sk = (uint32_t)__builtin_amdgcn_readlane(src, L + j);
                    const uint32_t nd = ((sk & 3u) + (uint32_t)__builtin_amdgcn_readlane(nb, L + j) + 3u) >> 2;
                    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane(px - pimg, L + j);
                    for (uint32_t c = 0; c < nd; c += 64u)
                        if (c + lane < nd)
                            __builtin_amdgcn_raw_ptr_buffer_load_lds(prs, qpim + lo + 4u * c, 4, (sk & ~3u) + 4u * (c + lane), 0, 0, 0);
                }
            }
        }
        __builtin_amdgcn_s_waitcnt(0);        // every piece landed in LDS
        asm volatile("" ::: "memory");
        load_clen();                          // the next four groups' first cmd.len (their records landed)
        // ---- lane 16 q + k builds entry k of group q in the group's slot ----
        uint64_t idx = 0;
        if (fast) {
            asm volatile("" : "+v"(t0), "+v"(t1), "+v"(t2));
            const uint64_t idx0 = has_tail ? ((uint64_t)__builtin_amdgcn_alignbyte(t1, t0, tsh) |
                                              ((uint64_t)__builtin_amdgcn_alignbyte(t2, t1, tsh) << 32)) + 1
                                           : 1ull;
            idx = idx0 + k;
            if (in_c) {
                uint8_t *const qimg = img + q * kQuadImg;
                const uint32_t e = s_v - A0;
                // header bytes from cut on lie past a 1-KiB boundary: 32 B further
                uint8_t *const he = qimg + img_pos(e);
                const uint32_t cut = 1024u - (e & 1023u);
                write_csm_header_at([he, cut](uint32_t o) { return he + o + (o >= cut ? 32u : 0u); }, idx, term, c_req,
                                    c_ct & 0xFFFFu, (c_ct >> 16) & 0xFFu);
                lds_funnel(qimg, e + kData, pim + q * kQuadPay, run ? src : px - pimg + sa, nb, k & 7u);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- the spans back to the rings, 16-B coalesced stores ----
        for (uint64_t m = fm; m; m &= m - 1) {
            const uint32_t L = (uint32_t)__builtin_ctzll(m), sq = L >> 4;
            uint8_t *const rq = b.ring + (g0 + sq) * stride;
            const uint32_t a0 = (uint32_t)__builtin_amdgcn_readlane(A0, L), np = (uint32_t)__builtin_amdgcn_readlane(npc, L);
            const uint4 *img16 = reinterpret_cast<const uint4 *>(img + sq * kQuadImg);
            for (uint32_t c = 0; c < np; c += 64u)
                if (c + lane < np)
                    *reinterpret_cast<uint4 *>(rq + a0 + 16u * (c + lane)) = img16[c + lane + 2u * ((c + lane) >> 6)];
        }
        asm volatile("" ::: "memory");
        // ---- a fast group's outputs: log_append_entry's idx per message,
        // end/tail (dare_log.h:547-550), prev_head cleared (:478-481), the last idx ----
        const uint32_t last_s = __shfl(s_v, sl + (n ? n - 1u : 0u));
        if (fast) {
            if (o.idx && in_c) o.idx[g * max_e + k] = idx;
            if (k == 0) {
                uint64_t *offs = offsets_of(b, g);
                offs[kOffEnd] = end + tot;
                offs[kOffTail] = last_s;
                if (b.prev_head) b.prev_head[g] = 0;
                if (o.last_idx) o.last_idx[g] = idx + n - 1;
            }
        }
        // ---- every other group with messages: handed to append_kernel<true>,
        // in this wave's slice of the list ----
        const uint64_t dm = __ballot(k == 0 && g < G && n > 0 && !fast);
        if (k == 0 && g < G && n > 0 && !fast)
            ids[n_def + __builtin_popcountll(dm & ((1ull << lane) - 1ull))] = (uint32_t)g;
        n_def += (uint32_t)__builtin_popcountll(dm);
    }
    if (lane == 0) {
        list[gw] = n_def;
        if (n_def) atomicAdd((unsigned long long *)&stats[APUS_STAT_APPEND_SLOW], (unsigned long long)n_def);
    }
}

__global__ void __launch_bounds__(256) persist_kernel(const apus_batch_t b, const apus_persist_in_t in,
                                                      uint64_t *stats)
{
    const uint32_t R = b.n_replicas;
    const uint64_t total = b.n_groups * R;
    uint64_t corrupt = 0;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t g = t / R;
        const uint32_t i = (uint32_t)(t - g * R);
        const apus_group_state_t st = load_state(b, g);
        const uint64_t end = st.end, len = st.len;
        const uint32_t self = b.self_idx[g];
        uint8_t *ring = b.ring + g * b.ring_stride;
        uint64_t oe = in.old_end[t];
        const uint32_t lim = in.limit ? in.limit[t] : 0xFFFFFFFFu;
        if (!(len >= kHdr && len <= ring_cap(b) && end <= len && oe <= len)) { ++corrupt; continue; }
        const uint64_t guard = len / kHdr + 4;
        uint64_t steps = 0;
        uint32_t n = 0;
        // while (log_is_offset_larger(log, log->end, log->old_end))
        while (dist(end, len, oe) != 0) {
            if (n >= lim) break;
            if (++steps > guard) { ++corrupt; break; }
            if (len - oe < kHdr) oe = 0;                         // log_get_entry
            uint8_t *e = ring + oe;
            const uint64_t elen = entry_len(e[kType], ld_u16(e + kData));
            if (len - oe < elen) { oe = 0; continue; }          // !log_fit_entry: ghost header
            if (i == self) e[kSender] = (uint8_t)i;             // IS_LEADER: entry->sender
            else e[kReply + i] = 1;                             // rc_send_entries_reply
            oe += elen;
            ++n;
        }
        in.old_end[t] = oe;
    }
    if (corrupt) atomicAdd((unsigned long long *)&stats[APUS_STAT_CORRUPT], (unsigned long long)corrupt);
}

// (persist_new_entries in 16-lane speculative segments per (group, replica
// copy), as nc_build_seg_kernel walks, measured slower than persist_kernel:
// C2 3.39 vs 3.02 ms, C5 6.18 vs 3.60 ms -- a copy writes one byte per entry,
// nothing a segment could coalesce.)

constexpr bool kAppDyn = true;

hipError_t launch_append(apus_ctx *ctx, const apus_batch_t &b, const apus_append_in_t &in,
                         const apus_append_out_t &o, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    // four groups per wave for short batches (append_quad_kernel), the groups
    // it hands back then by append_kernel<true> over the same grid
    const bool quad = !(in.flags & APUS_APPEND_PER_GROUP) && in.max_entries <= 16 && b.n_groups < (1ull << 32) &&
                      ((uintptr_t)in.payload & 3u) == 0 && ((((uintptr_t)b.ring) | b.ring_stride) & 15u) == 0 &&
                      b.ring_stride < (1ull << 31);
    // grids no larger than what is resident at once (LDS holds 3 blocks per CU):
    // a wave walks its share of groups grid-strided, and blocks queued behind
    // the resident ones would run as a partial last round at the kernel's end
    if (quad) {
        const uint32_t oc = (uint32_t)resident_blocks(ctx, 40, (const void *)append_quad_kernel);
        const uint32_t grid = grid_for((b.n_groups + 3) / 4, kAppendWaves, ctx->n_cu, oc);
        const uint32_t nw = grid * kAppendWaves;
        const uint64_t per = 4 * ((b.n_groups + 4ull * nw - 1) / (4ull * nw));
        ScratchPin pin;
        hipError_t e = stream_scratch(ctx, s, 1, 1 + nw + (uint64_t)nw * per, pin);
        StreamScratch *sc = pin.sc;
        if (e != hipSuccess) return e;
        uint32_t *list = sc->slow + 1;       // slow[0] is the commit walk's deferred count: left at 0
        hipLaunchKernelGGL(append_quad_kernel, dim3(grid), dim3(256), 0, s, b, in, o, ctx->stats, list, nw,
                           (uint32_t)per);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        hipLaunchKernelGGL((append_kernel<true, false>), dim3(grid), dim3(256), 0, s, b, in, o, ctx->stats, list, nw,
                           (uint32_t)per, nullptr);
        return hipGetLastError();
    }
    const uint32_t grid = grid_for(b.n_groups, kAppendWaves, ctx->n_cu,
                                   (uint32_t)resident_blocks(ctx, 41, (const void *)append_kernel<false, kAppDyn>));
    // groups after each wave's first from a counter (the stream's ticket word 2)
    ScratchPin pin;
    hipError_t e = stream_scratch(ctx, s, 1, 0, pin);
    StreamScratch *sc = pin.sc;
    if (e != hipSuccess) return e;
    if (kAppDyn && (e = hipMemsetAsync(sc->ticket + 2, 0, sizeof(uint32_t), s)) != hipSuccess) return e;
    hipLaunchKernelGGL((append_kernel<false, kAppDyn>), dim3(grid), dim3(256), 0, s, b, in, o, ctx->stats, nullptr,
                       0u, 0u, sc->ticket + 2);
    return hipGetLastError();
}

hipError_t launch_persist(apus_ctx *ctx, const apus_batch_t &b, const apus_persist_in_t &in, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    const uint32_t grid = grid_for(b.n_groups * b.n_replicas, 256, ctx->n_cu, 8);
    hipLaunchKernelGGL(persist_kernel, dim3(grid), dim3(256), 0, s, b, in, ctx->stats);
    return hipGetLastError();
}

}  // namespace apus

