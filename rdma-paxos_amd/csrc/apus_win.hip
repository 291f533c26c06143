// The election-win transition for gfx950 (BASELINE config 5's
// reconfiguration): the rest of poll_vote_count after the tally,
// src/dare/dare_server.c:1355-1362 and 1389-1510, one LANE per group
// (apus_gpu.h apus_vote_win_batch).
//
// vote_win_gate_kernel tests every group (IS_CANDIDATE, :49-51) and lists
// the candidates; vote_win_kernel takes the list: a candidate applies the
// tally's side effects, and a winner then walks its log three times
// (poll_config_entries, apply_committed_entries, the blank-entry scan) with
// the shared walks of apus_log_ops.h and appends with append_bare
// (apus_group_ops.h) -- chains of dependent header reads, a few bytes used per
// entry, as apply_kernel.
#include "apus_device.h"
#include "apus_internal.h"
#include "apus_log_ops.h"

namespace apus {

// IS_CANDIDATE (dare_server.c:49-51): SID_GET_IDX == idx, L clear, a term
// (not IS_NONE)
__device__ __forceinline__ bool is_candidate(uint64_t sid, uint32_t self)
{
    return (uint32_t)(sid & 0xFFu) == self && !((sid >> 8) & 1ull) && (sid >> 9) != 0;
}

// The candidate test of every group (a few bytes each, every lane busy): a
// group polling() would not ask to count votes gets APUS_WIN_NOT_CANDIDATE and
// zero counts; a candidate goes to its block's region of the list (LDS
// atomics only: one global counter would serialise a wave per group run)
// that the same block of vote_win_kernel works through.
// list: counts [grid], then grid regions of `cap` ids.
__global__ void __launch_bounds__(256) vote_win_gate_kernel(const apus_batch_t b, const apus_win_io_t io,
                                                            uint32_t *list, uint32_t cap)
{
    __shared__ uint32_t n;
    if (threadIdx.x == 0) n = 0;
    __syncthreads();
    uint32_t *const region = list + gridDim.x + (uint64_t)blockIdx.x * cap;
    for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < b.n_groups;
         g += (uint64_t)gridDim.x * blockDim.x) {
        if (is_candidate(b.sid[g], b.self_idx[g])) {
            region[atomicAdd(&n, 1u)] = (uint32_t)g;
        } else {
            io.outcome[g] = APUS_WIN_NOT_CANDIDATE;
            if (io.events) io.events[g] = 0;
            if (io.departed) io.departed[g] = 0;
            if (io.n_applied) io.n_applied[g] = 0;
            if (io.n_cfg) io.n_cfg[g] = 0;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) list[blockIdx.x] = n;
}

__global__ void __launch_bounds__(256) vote_win_kernel(const apus_batch_t b, const apus_win_io_t io,
                                                       const uint32_t *list, uint32_t cap, uint64_t *stats)
{
    uint64_t corrupt = 0;
    const uint32_t R = b.n_replicas;
    const uint32_t n = list[blockIdx.x];
    const uint32_t *const region = list + gridDim.x + (uint64_t)blockIdx.x * cap;
    for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
        const uint64_t g = region[k];
        const uint32_t self = b.self_idx[g];
        const uint64_t sid = b.sid[g];
        uint32_t outcome = APUS_WIN_NOT_CANDIDATE, ev = 0, dep = 0, na = 0, nc = 0;
        {
            uint64_t *const offs = offsets_of(b, g);
            uint64_t *const cw = cid_words(b, g);
            apus_group_state_t st = load_state(b, g);
            // 1. the tally's side effects (:1355-1362)
            const uint32_t voters = io.voters[g];
            for (uint32_t i = 0; i < R && i < 16; ++i)
                if ((voters >> i) & 1u) {
                    b.remote_commit[g * R + i] = b.vote_ack[g * R + i];
                    b.lr_step[g * R + i] = APUS_LR_GET_NCE_LEN;
                }
            st.commit = io.new_commit[g];
            offs[kOffCommit] = st.commit;
            outcome = APUS_WIN_LOST;
            if (io.won[g]) {
                outcome = APUS_WIN_CORRUPT;   // until an outcome below
                // 2. SID_SET_L + server_update_sid (:1389-1395, :2288-2297): a
                // compare-and-swap on the value read
                const uint64_t ns = sid | (1ull << 8);
                const bool cas = atomicCAS(reinterpret_cast<unsigned long long *>(b.sid + g),
                                           (unsigned long long)sid, (unsigned long long)ns) == sid;
                uint64_t off = io.cid_offset[g];
                do {
                    if (!cas || !ring_ok(st, ring_cap(b)) || off > st.len) break;
                    const uint64_t term = ns >> 9;
                    uint64_t c_lo = st.cid.epoch, c_hi = cw[1];
                    uint64_t rq = io.req_id[g], head_off = st.head;
                    uint32_t cl = io.clt_id[g];
                    bool changed = false;
                    // 3. poll_config_entries (:1404)
                    const bool ok3 = scan_config(b.ring + g * b.ring_stride, st, io.cid_idx[g], off, c_lo, c_hi, rq,
                                                 cl, dep, changed, head_off);
                    if (changed) {
                        cw[0] = c_lo;
                        cw[1] = c_hi;
                        io.req_id[g] = rq;
                        io.clt_id[g] = (uint16_t)cl;
                    }
                    if (!ok3) break;
                    off = larger(st.end, st.len, off, st.commit) ? st.commit : off;
                    io.cid_offset[g] = off;
                    if (larger(st.end, st.len, head_off, st.head)) {
                        st.head = head_off;
                        offs[kOffHead] = head_off;
                    }
                    // 4. apply_committed_entries as the leader (:1409), the
                    // CONFIG re-appends appended when they are met
                    uint32_t prev = b.prev_head ? b.prev_head[g] : 0u;
                    ApplyAcc a{};
                    a.c_lo = c_lo;
                    a.c_hi = c_hi;
                    a.rq = rq;
                    a.cl = cl;
                    const bool ok4 = apply_walk<true>(b, g, st, self, true, term, a, nullptr, prev);
                    offs[kOffApply] = st.apply;
                    c_hi = a.c_hi;
                    if (a.cfg_changed) {
                        cw[1] = c_hi;
                        rq = a.rq;
                        cl = a.cl;
                        io.req_id[g] = rq;
                        io.clt_id[g] = (uint16_t)cl;
                    }
                    if (a.na) {
                        uint64_t la0, la1;
                        ld_idx_term(b.ring + g * b.ring_stride + a.la_off, la0, la1);
                        io.last_applied[3 * g] = la0;
                        io.last_applied[3 * g + 1] = la1;
                        io.last_applied[3 * g + 2] = a.la2;
                        io.last_csm_idx[g] = la0;
                    }
                    na = a.na;
                    nc = a.nc;
                    dep |= a.dep;
                    ev |= a.ev;
                    if (b.prev_head) b.prev_head[g] = (uint8_t)prev;
                    if (!ok4) break;
                    // 5. the blank entry (:1411-1491)
                    const uint64_t len = st.len;
                    const uint8_t *ring = b.ring + g * b.ring_stride;
                    uint32_t type = APUS_CONFIG, next = APUS_WIN_CONFIG;
                    bool append = true;
                    if (cid_state(c_hi) == APUS_CID_STABLE) {
                        rq = 0;
                        cl = 0;
                        io.req_id[g] = 0;
                        io.clt_id[g] = 0;
                    } else {
                        // the scan from cid_offset for a CONFIG entry past cid_idx
                        const uint64_t guard = len / kHdr + 4, cidx = io.cid_idx[g];
                        uint64_t o = off, last = ~0ull, steps = 0;
                        bool bad = false;
                        while (dist(st.end, len, o) != 0) {
                            if (++steps > guard) { bad = true; break; }
                            if (len - o < kHdr) o = 0;                                // log_get_entry
                            last = o;
                            const uint8_t *e = ring + o;
                            const uint32_t t = e[kType];
                            const uint32_t el = entry_len(t, ld_u16(e + kData));
                            if (len - o < el) { o = 0; continue; }                    // !log_fit_entry
                            if (t == APUS_CONFIG && ld_u64(e + kIdx) > cidx) break;
                            o += el;
                        }
                        if (bad) break;
                        if (dist(st.end, len, o) != 0) {
                            type = APUS_NOOP;                     // an un-applied CONFIG: a NOOP (:1441-1448)
                            rq = 0;
                            cl = 0;
                            next = APUS_WIN_NOOP;
                        } else if (last == ~0ull) {
                            append = false;                       // :1456 reads an uninitialised entry
                            next = APUS_WIN_UNDEFINED;
                        } else if (ring[last + kData + 10] == APUS_CID_EXTENDED) {   // entry->data.cid.state
                            c_hi = cid_with_state(c_hi, APUS_CID_TRANSIT);
                            next = APUS_WIN_TRANSIT;
                        } else {
                            // STABLE, servers size[0]-1 down to size[1]+1 removed (:1460-1486)
                            c_hi = cid_with_state(c_hi, APUS_CID_STABLE);
                            const uint32_t s1 = cid_size1(c_hi);
                            for (uint32_t i = (cid_size0(c_hi) - 1u) & 0xFFu; i > s1; --i) {
                                if (i == self) {
                                    ev |= APUS_EV_SELF_REMOVED;   // DIE_AF_COMMIT
                                    if (i < 32) c_hi &= ~(1ull << (32 + i));
                                    continue;
                                }
                                if (!cid_on(c_hi, i)) continue;
                                c_hi &= ~(1ull << (32 + i));
                                if (i < 16) dep |= 1u << i;
                            }
                            c_hi = (c_hi & ~0xFFFFull) | s1;      // size[0] = size[1]; size[1] = 0
                            next = APUS_WIN_STABLE;
                        }
                        cw[1] = c_hi;
                    }
                    if (append) {
                        const uint64_t w[2] = { c_lo, c_hi };
                        bool stopped = false;
                        const uint64_t idx = append_bare(b, g, st, prev, term, type, rq, cl, w, stopped);
                        if (b.prev_head) b.prev_head[g] = (uint8_t)prev;
                        if (stopped) break;
                        io.last_write_csm_idx[g] = idx;
                    }
                    // 6. become_leader: apply_offsets[i] = head (:1505-1508)
                    const uint32_t esz = cid_ext_size(c_hi);
                    for (uint32_t i = 0; i < esz && i < R; ++i) b.apply_offsets[g * R + i] = st.head;
                    outcome = next;
                } while (false);
                if (outcome == APUS_WIN_CORRUPT) ++corrupt;
            }
        }
        io.outcome[g] = (uint8_t)outcome;
        if (io.events) io.events[g] = (uint8_t)ev;
        if (io.departed) io.departed[g] = (uint16_t)dep;
        if (io.n_applied) io.n_applied[g] = na;
        if (io.n_cfg) io.n_cfg[g] = nc;
    }
    if (corrupt) atomicAdd((unsigned long long *)&stats[APUS_STAT_CORRUPT], (unsigned long long)corrupt);
}

hipError_t launch_vote_win(apus_ctx *ctx, const apus_batch_t &b, const apus_win_io_t &io, hipStream_t s)
{
    if (!b.n_groups) return hipSuccess;
    if (b.n_groups >> 32) return hipErrorInvalidValue;
    const uint32_t grid = grid_for(b.n_groups, 256, ctx->n_cu, 8);
    // the candidate lists in the stream's deferred-group scratch: a count per
    // block, then one region per block as large as the groups it tests
    const uint64_t per = (b.n_groups + (uint64_t)grid * 256 - 1) / ((uint64_t)grid * 256);
    const uint32_t cap = (uint32_t)(per * 256);
    ScratchPin pin;
    hipError_t e = stream_scratch(ctx, s, 0, (uint64_t)grid * cap + grid, pin);
    if (e != hipSuccess) return e;
    uint32_t *list = pin.sc->slow;
    hipLaunchKernelGGL(vote_win_gate_kernel, dim3(grid), dim3(256), 0, s, b, io, list, cap);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(vote_win_kernel, dim3(grid), dim3(256), 0, s, b, io, (const uint32_t *)list, cap, ctx->stats);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // (the commit call's walk expects the list's first word at 0)
    return hipMemsetAsync(list, 0, sizeof(uint32_t), s);
}

}  // namespace apus
