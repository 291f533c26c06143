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

__global__ void __launch_bounds__(256) append_kernel(const apus_batch_t b, const apus_append_in_t in,
                                                     const apus_append_out_t o, uint64_t *stats)
{
    const uint32_t lane = lane_id();
    const uint32_t wv = uni(threadIdx.x >> 6);
    const uint64_t G = b.n_groups, stride = b.ring_stride, pb = in.payload_bytes;
    const uint32_t max_e = in.max_entries;
    // The next group's state row (lanes 0..7, one u64 each) and its first
    // 64 message records are requested while the current group is worked on;
    // their cmd.len loads at the end of the current group.
    const uint64_t gs = (uint64_t)gridDim.x * kAppendWaves;
    const uint32_t pre_n = min(64u, max_e);
    uint64_t p_row = 0, p_req = 0, p_doff = 0;
    uint32_t p_ct = 0, p_clen = 0;
    auto load_next = [&](uint64_t gg) {
        p_row = 0; p_req = 0; p_doff = 0; p_ct = 0;
        if (gg < G) {
            if (lane < 8) p_row = reinterpret_cast<const uint64_t *>(b.state + gg)[lane];
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
    uint64_t g = (uint64_t)blockIdx.x * kAppendWaves + wv;
    load_next(g);
    p_clen = load_clen(p_doff, p_ct);
    for (; g < G; g += gs) {
        const uint64_t c_row = p_row, c_req = p_req, c_doff = p_doff;
        const uint32_t c_ct = p_ct, c_clen = p_clen;
        load_next(g + gs);
        apus_group_state_t st;
        st.head = rl64c(c_row, 0);
        st.apply = rl64c(c_row, 1);
        st.commit = rl64c(c_row, 2);
        st.end = rl64c(c_row, 3);
        st.tail = rl64c(c_row, 4);
        st.len = rl64c(c_row, 5);
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
        bool stop = !(len >= kHdr && len <= stride && end <= len && tail <= len);
        bool bad = stop && n > 0;
        uint64_t known_off = ~0ull, known_idx = 0;

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
                    x = el;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const uint32_t y = __shfl_up(x, d);
                        if (lane >= (uint32_t)d) x += y;
                    }
                    before = kk ? (uint32_t)__builtin_amdgcn_readlane(x, kk - 1) : 0u;
                    s_v = (uint32_t)end + (x - el - before);
                    const bool ok = in_c && m_ok && (uint64_t)s_v + el <= len && (uint64_t)s_v != head;
                    const uint64_t fail = __ballot(!ok) & (~0ull << kk);
                    nf = (fail ? (uint32_t)__builtin_ctzll(fail) : 64u) - kk;
                }
                if (nf) {
                    const uint32_t kl = kk + nf;                             // last + 1
                    uint64_t idx0 = 1;
                    if (dist(end, len, tail) != 0) {                          // end != len already
                        const uint64_t off = len - tail < kHdr ? 0 : tail;
                        idx0 = (off == known_off ? known_idx : ld_u64(ring + off)) + 1;
                    }
                    // headers: lane k writes entry k's (sender@27 and 41..47 untouched)
                    if (lane >= kk && lane < kl) {
                        const uint64_t idx = idx0 + (lane - kk);
                        uint8_t *e = ring + s_v;
                        const uint32_t clt = m_ct & 0xFFFFu, type = (m_ct >> 16) & 0xFFu;
                        if ((s_v & 7u) == 0) {
                            uint64_t *e64 = reinterpret_cast<uint64_t *>(e);
                            e64[0] = idx;
                            e64[1] = term;
                            e64[2] = m_req;
                            *reinterpret_cast<uint16_t *>(e + 24) = (uint16_t)clt;
                            e[26] = (uint8_t)type;
                            *reinterpret_cast<uint32_t *>(e + 28) = 0u;        // reply[0..3]
                            e64[4] = 0ull;                                     // reply[4..11]
                            e[40] = 0;                                         // reply[12]
                        } else {
#pragma unroll
                            for (int i = 0; i < 8; ++i) {
                                e[i] = (uint8_t)(idx >> (8 * i));
                                e[8 + i] = (uint8_t)(term >> (8 * i));
                                e[16 + i] = (uint8_t)(m_req >> (8 * i));
                            }
                            e[24] = (uint8_t)clt;
                            e[25] = (uint8_t)(clt >> 8);
                            e[26] = (uint8_t)type;
#pragma unroll
                            for (int i = kReply; i < kReply + APUS_MAX_SERVER_COUNT; ++i) e[i] = 0;
                        }
                        idx_v = idx;
                    }
                    copy_cmds(ring, in.payload, kk, kl, m_doff, s_v, m_clen, lane);
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
                        tail = device_get_tail(RingView{ ring, end, len }, st);
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
                b.state[g].end = end;
                b.state[g].tail = tail;
            }
            if (b.prev_head) b.prev_head[g] = (uint8_t)prev_head;
            if (o.last_idx) o.last_idx[g] = last_ret;
            if (bad) atomicAdd((unsigned long long *)&stats[APUS_STAT_CORRUPT], 1ull);
        }
        p_clen = load_clen(p_doff, p_ct);
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
        const apus_group_state_t st = b.state[g];
        const uint64_t end = st.end, len = st.len;
        const uint32_t self = b.self_idx[g];
        uint8_t *ring = b.ring + g * b.ring_stride;
        uint64_t oe = in.old_end[t];
        const uint32_t lim = in.limit ? in.limit[t] : 0xFFFFFFFFu;
        if (!(len >= kHdr && len <= b.ring_stride && end <= len && oe <= len)) { ++corrupt; continue; }
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

hipError_t launch_append(apus_ctx *ctx, const apus_batch_t &b, const apus_append_in_t &in,
                         const apus_append_out_t &o, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    const uint32_t grid = grid_for(b.n_groups, kAppendWaves, ctx->n_cu, 8);
    hipLaunchKernelGGL(append_kernel, dim3(grid), dim3(256), 0, s, b, in, o, ctx->stats);
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
