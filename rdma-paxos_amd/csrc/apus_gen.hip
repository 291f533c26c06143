// Synthetic trace generator on the device (bench / parity inputs).
//
// Byte-for-byte the same traces as oracle/apus_oracle.c apus_oracle_gen_batch
// (the specification): counter-keyed SplitMix64 draws per (group, purpose),
// entry placement restating log_append_entry (src/include/dare/dare_log.h:
// 466-558: header-wrap to 0, ghost header when the command does not fit),
// prefix-monotone follower acks (persist_new_entries / rc_send_entries_reply,
// src/dare/dare_server.c:1792-1810, src/dare/dare_ibv_rc.c:1828-1863).
//
//   gen_fill_kernel   every ring byte from draw(gkey, FILL + word)  (coalesced)
//   gen_place_kernel  one lane per group: placement, headers, control data
#include "apus_device.h"
#include "apus_internal.h"

namespace apus {

#define K_G(f) (0x100ull + (f))
#define K_R(r, f) (0x1000ull + (uint64_t)(r) * 64 + (f))
#define K_E(e, f) (0x100000ull + (uint64_t)(e) * 16 + (f))
#define K_RG(e, r) (0x10000000ull + (uint64_t)(e) * 16 + (r))
#define K_FILL(w) ((1ull << 40) + (w))

constexpr uint32_t kGenMaxEntries = 256;

__device__ __forceinline__ uint64_t gkey_of(const apus_gen_cfg_t &c, uint64_t g)
{
    return sm64(c.seed ^ sm64(c.gid_base + g));
}

__global__ void __launch_bounds__(256) gen_fill_kernel(const apus_batch_t b, const apus_gen_cfg_t c)
{
    const uint64_t pps = b.ring_stride / 16;
    const uint64_t total = b.n_groups * pps;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t g = t / pps, k = t - g * pps;
        const uint64_t key = gkey_of(c, g);
        const uint64_t w0 = draw(key, K_FILL(2 * k)), w1 = draw(key, K_FILL(2 * k + 1));
        *reinterpret_cast<uint4 *>(b.ring + g * b.ring_stride + 16 * k) =
            make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
    }
}

__device__ __forceinline__ void st64(uint8_t *p, uint64_t v)
{
#pragma unroll
    for (int i = 0; i < 8; ++i) p[i] = (uint8_t)(v >> (8 * i));
}
__device__ __forceinline__ void st16(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
}

__device__ __forceinline__ uint32_t gen_type(const apus_gen_cfg_t &c, uint64_t key, uint32_t e)
{
    if (!c.type_mix) return 5;
    switch (draw(key, K_E(e, 0)) % 16) {
    case 0: return APUS_NOOP;
    case 1: return APUS_CONFIG;
    case 2: return APUS_HEAD;
    case 3: return 4;
    case 4: return 6;
    default: return 5;
    }
}

// one lane per group; `after` = per-lane LDS column of N u32 (end after entry e)
__global__ void __launch_bounds__(64) gen_place_kernel(const apus_batch_t b, const apus_gen_cfg_t c)
{
    extern __shared__ __attribute__((aligned(16))) uint32_t s_after[];
    const uint32_t R = b.n_replicas, H = c.n_history, E = c.n_entries, N = H + E;
    uint32_t *after = s_after + threadIdx.x * N;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t key = gkey_of(c, g);
        uint8_t *ring = b.ring + g * b.ring_stride;
        const uint64_t len = c.ring_len;

        // ---- group parameters (oracle gen_group_params) ----
        uint32_t size0 = R, size1 = 0, state = APUS_CID_STABLE;
        if (c.cid_mix) {
            const uint64_t u = draw(key, K_G(4)) % 100;
            if (u >= 60 && u < 80) { state = APUS_CID_EXTENDED; size0 = R - 1; size1 = R; }
            else if (u >= 80) {
                state = APUS_CID_TRANSIT;
                if (draw(key, K_G(5)) & 1) { size0 = R - 2; size1 = R; }
                else { size0 = R; size1 = R - 2; }
            }
        }
        const uint32_t self = c.self_random ? (uint32_t)(draw(key, K_G(1)) % size0) : 0u;
        const uint64_t term_g = 1 + draw(key, K_G(2)) % 8;
        const uint64_t idx_base = 1 + draw(key, K_G(3)) % 1000000;
        const uint64_t epoch = draw(key, K_G(6)) % 4;
        uint32_t bitmask = (R >= 32) ? 0xFFFFFFFFu : ((1u << R) - 1u);
        if (draw(key, K_G(7)) % 8 == 0) {
            const uint32_t off = (self + 1 + (uint32_t)(draw(key, K_G(8)) % (R - 1))) % R;
            bitmask &= ~(1u << off);
        }
        const uint64_t h0 = (draw(key, K_G(0)) % len) & ~7ull;
        apus_cid_t cid;
        cid.epoch = epoch; cid.size[0] = (uint8_t)size0; cid.size[1] = (uint8_t)size1;
        cid.state = (uint8_t)state; cid.pad[0] = 0; cid.bitmask = bitmask;

        // ---- follower ack counts ----
        uint32_t kr[APUS_MAX_SERVER_COUNT];
        const uint32_t rs = (self + 1 + (uint32_t)(draw(key, K_G(10)) % (R - 1))) % R;
#pragma unroll
        for (uint32_t r = 0; r < APUS_MAX_SERVER_COUNT; ++r) {
            uint32_t k = 0;
            if (r < R) {
                k = (draw(key, K_R(r, 0)) % 65536 < c.p_full_ack || E == 0) ? E : (uint32_t)(draw(key, K_R(r, 1)) % E);
                if (c.straggler && r == rs) k = (uint32_t)(draw(key, K_R(r, 2)) % (E / 4 + 1));
            }
            kr[r] = k;
        }

        // ---- placement + headers ----
        uint64_t end = h0, tail = 0;
        for (uint32_t e = 0; e < N; ++e) {
            const uint32_t t = gen_type(c, key, e);
            const bool csm = !bare_type(t);
            uint32_t clen = 0;
            const uint32_t lmax = (e < H && c.hist_len_max) ? c.hist_len_max : c.len_max;
            if (csm) clen = c.len_min + (uint32_t)(draw(key, K_E(e, 1)) % (lmax - c.len_min + 1));
            const uint64_t elen = kHdr + (csm ? clen : 0);
            const uint64_t idx = idx_base + e;
            const uint64_t term = (e < H / 2 && term_g > 1) ? term_g - 1 : term_g;
            const uint64_t req = draw(key, K_E(e, 2));
            const uint32_t clt = (uint32_t)(draw(key, K_E(e, 3)) & 0xFFFF);
            uint64_t o = end;
            if (end == len || len - o < kHdr) o = 0;
            if (len - o < elen) {                               // ghost header at o
                uint8_t *gh = ring + o;
                st64(gh + 0, idx); st64(gh + 8, term); st64(gh + 16, req);
                st16(gh + 24, clt); gh[kType] = (uint8_t)t;
                for (int i = 0; i < APUS_MAX_SERVER_COUNT; ++i) gh[kReply + i] = 0;
                st16(gh + kData, clen);
                o = 0;
            }
            uint8_t *en = ring + o;
            st64(en + 0, idx); st64(en + 8, term); st64(en + 16, req);
            st16(en + 24, clt); en[kType] = (uint8_t)t;
            en[kSender] = (uint8_t)self;
#pragma unroll
            for (uint32_t r = 0; r < APUS_MAX_SERVER_COUNT; ++r) {
                uint8_t rb = 0;
                if (r < R && r != self) {
                    if (e < H) rb = 1;
                    else if (e - H < kr[r]) rb = (draw(key, K_RG(e, r)) % 65536 < c.garbage_reply) ? 2 : 1;
                }
                en[kReply + r] = rb;
            }
            if (t == APUS_CONFIG) {
                st64(en + kData, cid.epoch);
                en[kData + 8] = cid.size[0]; en[kData + 9] = cid.size[1];
                en[kData + 10] = cid.state; en[kData + 11] = 0;
                st16(en + kData + 12, cid.bitmask); st16(en + kData + 14, cid.bitmask >> 16);
            } else if (t == APUS_HEAD) {
                st64(en + kData, h0);
            } else if (csm) {
                st16(en + kData, clen);
            }
            tail = o;
            end = o + elen;
            after[e] = (uint32_t)end;
        }

        // ---- group state ----
        const uint64_t commit = H ? after[H - 1] : h0;
        const uint32_t a = (uint32_t)(draw(key, K_G(9)) % (H + 1));
        apus_group_state_t st;
        st.head = h0;
        st.apply = a ? after[a - 1] : h0;
        st.commit = commit;
        st.end = end;
        st.tail = tail;
        st.len = len;
        st.cid = cid;
        b.state[g] = st;
        b.self_idx[g] = (uint8_t)self;

        // ---- per-replica control data ----
        for (uint32_t r = 0; r < R; ++r) {
            const uint64_t gr = g * R + r;
            const uint32_t krr = kr[r < APUS_MAX_SERVER_COUNT ? r : 0];
            if (b.remote_end) b.remote_end[gr] = (r == self) ? end : (krr ? after[H + krr - 1] : commit);
            if (b.remote_commit) b.remote_commit[gr] = commit;
            if (b.lr_step)
                b.lr_step[gr] = (draw(key, K_R(r, 3)) % 16 == 0) ? (uint8_t)(1 + draw(key, K_R(r, 4)) % 6)
                                                                : (uint8_t)APUS_LR_UPDATE_LOG;
            if (b.fail_count)
                b.fail_count[gr] = (draw(key, K_R(r, 5)) % 32 == 0) ? (uint8_t)APUS_PERMANENT_FAILURE : 0;
            if (b.vote_ack) {
                uint64_t va = len;
                if (r != self && draw(key, K_R(r, 6)) % 65536 < c.p_vote_ack) {
                    const uint32_t j = (uint32_t)(draw(key, K_R(r, 7)) % (N + 1));
                    va = j ? after[j - 1] : h0;
                }
                b.vote_ack[gr] = va;
            }
            if (b.apply_offsets) {
                const uint32_t j = (uint32_t)(draw(key, K_R(r, 8)) % (H + 1));
                b.apply_offsets[gr] = j ? after[j - 1] : h0;
            }
            if (b.hb)
                b.hb[gr] = (draw(key, K_R(r, 9)) % 8 == 0)
                               ? (((term_g + draw(key, K_R(r, 10)) % 2) << 9) | (1ull << 8) | r) : 0ull;
            if (b.vote_req) {
                apus_vote_req_t q;
                q.sid = 0; q.index = 0; q.term = 0;
                q.cid.epoch = 0; q.cid.size[0] = 0; q.cid.size[1] = 0; q.cid.state = 0; q.cid.pad[0] = 0;
                q.cid.bitmask = 0;
                if (r != self && (draw(key, K_R(r, 11)) & 1)) {
                    const uint64_t last_idx = idx_base + N - 1;
                    const uint64_t last_term = term_g;
                    q.sid = ((term_g + draw(key, K_R(r, 12)) % 3) << 9) |
                            ((uint64_t)(draw(key, K_R(r, 13)) % 8 == 0) << 8) | r;
                    const int64_t di = (int64_t)(draw(key, K_R(r, 14)) % 5) - 2;
                    const int64_t dt = (int64_t)(draw(key, K_R(r, 15)) % 3) - 1;
                    q.index = (uint64_t)((int64_t)last_idx + di);
                    q.term = (uint64_t)((int64_t)last_term + dt);
                    q.cid = cid;
                    q.cid.epoch = draw(key, K_R(r, 16)) % 8;
                }
                b.vote_req[gr] = q;
            }
        }
        if (b.sid) {
            const uint64_t L = draw(key, K_G(11)) % 4 == 0;
            const uint64_t sidx = draw(key, K_G(12)) % R;
            b.sid[g] = (term_g << 9) | (L << 8) | sidx;
        }
        if (b.last_idx_term) {   // end == len reads as an empty log: (0, 0)
            b.last_idx_term[2 * g] = end == len ? 0 : idx_base + N - 1;
            b.last_idx_term[2 * g + 1] = end == len ? 0 : term_g;
        }
        if (b.prev_head) b.prev_head[g] = draw(key, K_G(13)) % 4 == 0;
        if (b.abs_base) b.abs_base[g] = (draw(key, K_G(14)) % 1000) * len;
    }
}

hipError_t launch_gen(apus_ctx *ctx, const apus_batch_t &b, const apus_gen_cfg_t &c, hipStream_t s)
{
    const uint32_t N = c.n_entries + c.n_history;
    if (N == 0 || N > kGenMaxEntries || b.n_replicas < 2 || b.n_replicas > APUS_MAX_SERVER_COUNT ||
        c.len_min > c.len_max || c.len_max > 65535 || b.ring_stride % 16 || c.ring_len > b.ring_stride ||
        c.ring_len < 256 || (c.hist_len_max && (c.hist_len_max < c.len_min || c.hist_len_max > c.len_max)))
        return hipErrorInvalidValue;
    // the placed entries plus one wrap gap must not reach the head
    const uint64_t hmax = c.hist_len_max ? c.hist_len_max : c.len_max;
    const uint64_t worst = (uint64_t)c.n_history * (kHdr + hmax) + (uint64_t)c.n_entries * (kHdr + c.len_max) + kHdr +
                           c.len_max + 8;
    if (worst >= c.ring_len) return hipErrorInvalidValue;
    if (c.cid_mix && b.n_replicas < 3) return hipErrorInvalidValue;
    if (!b.n_groups) return hipSuccess;
    const uint64_t pieces = b.n_groups * (b.ring_stride / 16);
    uint64_t fg = (pieces + 255) / 256;
    const uint64_t fcap = (uint64_t)(ctx->n_cu > 0 ? ctx->n_cu : 256) * 16;
    if (fg > fcap) fg = fcap;
    hipLaunchKernelGGL(gen_fill_kernel, dim3((uint32_t)fg), dim3(256), 0, s, b, c);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t lds = (size_t)64 * N * sizeof(uint32_t);
    uint64_t pg = (b.n_groups + 63) / 64;
    const uint64_t pcap = (uint64_t)(ctx->n_cu > 0 ? ctx->n_cu : 256) * 8;
    if (pg > pcap) pg = pcap;
    hipLaunchKernelGGL(gen_place_kernel, dim3((uint32_t)pg), dim3(64), lds, s, b, c);
    return hipGetLastError();
}

}  // namespace apus
