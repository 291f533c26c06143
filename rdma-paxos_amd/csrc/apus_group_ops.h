// Per-group quorum operations of quorum_tail_kernel (apus_commit.hip) and
// prune_kernel (apus_quorum.hip): the DARE median quorum (a4) and
// log_pruning's minimum (a7).  Every input a group's median and pruning read
// (its replica columns, self index, previous-HEAD flag, base) is requested
// in one batch of loads before any is used (QuorumIn), so a lane pays one
// memory round trip per group, not one per dependent load.
#pragma once

#include "apus_device.h"

namespace apus {

// the inputs of group g's median (MED) and pruning (PR), for replicas
// i < R <= N (kernels instantiate N = R for the common R = 3, 5, 7: fewer
// registers, and no per-replica branch between the loads, which the
// compiler would otherwise close with a wait each)
template <int N>
struct QuorumIn {
    uint64_t rend[N];         // remote_end (MED)
    uint64_t ap[N];           // apply_offsets (PR)
    uint32_t step[N], fail[N];   // lr_step, fail_count (MED)
    uint32_t self;            // self_idx (MED)
    uint32_t prev;            // prev_head (PR)
    uint64_t base;            // abs_base (PR; ~0 without)
};

// EXACT: the batch has exactly N replicas
template <int N, bool EXACT>
__device__ __forceinline__ void load_quorum_in(const apus_batch_t &b, uint64_t g, bool med, bool pr, QuorumIn<N> &q)
{
    const uint32_t R = EXACT ? (uint32_t)N : b.n_replicas;
    const uint64_t *rend = b.remote_end + g * R, *ap = b.apply_offsets + g * R;
    const uint8_t *step = b.lr_step + g * R, *fail = b.fail_count + g * R;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        q.rend[i] = q.ap[i] = 0;
        q.step[i] = q.fail[i] = 0;
    }
    if (med) {
#pragma unroll
        for (int i = 0; i < N; ++i) {
            if (EXACT || (uint32_t)i < R) {
                q.rend[i] = rend[i];
                q.step[i] = step[i];
                q.fail[i] = fail[i];
            }
        }
    }
    if (pr) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (EXACT || (uint32_t)i < R) q.ap[i] = ap[i];
    }
    q.self = med ? b.self_idx[g] : 0u;
    q.prev = pr && b.prev_head ? b.prev_head[g] : 0u;
    q.base = pr && b.abs_base ? b.abs_base[g] : ~0ull;
}

// DARE median-offset quorum of a group (dare_ibv_rc.c:1650-1723) over N
// sort slots (N >= R; inputs for NR <= N replicas): the quirks are the
// reference's -- numeric sort, circular gate, TRANSIT min
template <int N, int NR>
__device__ __forceinline__ uint64_t median_of(uint32_t R, const apus_group_state_t &st, const QuorumIn<NR> &q)
{
    const uint64_t len = st.len, end = st.end, commit = st.commit;
    const uint32_t self = q.self;
    const bool transit = st.cid.state == APUS_CID_TRANSIT;
    // offsets the reference gathers for i < size (dare_ibv_rc.c:1660-1676);
    // slot values do not depend on j, only which slots are live does
    uint64_t off[N];
    uint32_t upd = 0;    // bit i: replica i contributes its remote end
#pragma unroll
    for (int i = 0; i < N; ++i) {
        uint64_t v = commit;
        if ((uint32_t)i == self) v = end;
        else if (i < NR && (uint32_t)i < R && ((st.cid.bitmask >> i) & 1u) &&
                 q.fail[i < NR ? i : 0] < APUS_PERMANENT_FAILURE &&
                 q.step[i < NR ? i : 0] == APUS_LR_UPDATE_LOG) {
            v = q.rend[i < NR ? i : 0];
            upd |= 1u << i;
        }
        off[i] = v;
    }
    // the two sizes as scalars: indexing st.cid.size[j] by the loop's j
    // made the compiler keep st in LDS (64 B per lane, bank-conflicted)
    const uint32_t size0 = st.cid.size[0], size1 = st.cid.size[1];
    uint64_t minv = commit;
    for (int j = 0; j < 2;) {
        const uint32_t size = j ? size1 : size0;
        int cnt = 0;
#pragma unroll
        for (int i = 0; i < N; ++i)
            if ((uint32_t)i < size && ((upd >> i) & 1u) && larger(end, len, off[i], minv)) ++cnt;
        if (cnt < (int)(size / 2)) {
            if (!transit) break;
            if (j == 0) { ++j; continue; }
            break;
        }
        // the value the reference's numeric insertion sort (dare_ibv_rc.c:
        // 1688-1696) leaves at offsets[(size-1)/2]: slot i's key is off[i] for
        // i < size, else ~0 (past the sort); the slot of rank mi is the one
        // with exactly mi keys before it (ties by slot index).  Rank selection
        // needs no sorted copy: it runs in the commit kernel's block epilogue,
        // where registers are scarce (the sorting network there spilled).
        const uint32_t mi = (size - 1) / 2;
        const uint32_t want = mi < (uint32_t)N ? mi : 0u;   // size 0 or > 2N: the smallest key (a sorted copy's [0])
        uint64_t med = 0;
#pragma unroll
        for (int i = 0; i < N; ++i) {
            const uint64_t ki = (uint32_t)i < size ? off[i] : ~0ull;
            uint32_t r = 0;
#pragma unroll
            for (int k = 0; k < N; ++k) {
                if (k == i) continue;
                const uint64_t kk = (uint32_t)k < size ? off[k] : ~0ull;
                r += (kk < ki || (kk == ki && k < i)) ? 1u : 0u;
            }
            if (r == want) med = ki;
        }
        if (!transit) { minv = med; break; }
        if (j == 0) minv = med;
        else if (larger(end, len, minv, med)) minv = med;
        ++j;
    }
    return minv;
}

// log_pruning's minimum of a group (dare_server.c:2026-2058, + log_get_tail
// when dist(min) == 0, dare_log.h:402-457): writes the apus_prune_out_t
// fields given (NULL = not wanted), resets OFF servers' apply offsets in
// place as the reference does, and returns the group's absolute watermark
// abs_base + new_head (~0 without abs_base)
template <int N>
__device__ __forceinline__ uint64_t prune_of(const apus_batch_t &b, uint64_t g, const apus_group_state_t &st,
                                             const QuorumIn<N> &q, uint64_t *new_head, uint8_t *append_head,
                                             uint64_t *min_apply)
{
    const uint32_t R = b.n_replicas;
    const uint32_t size = ext_group_size(st.cid);
    uint64_t *ap = b.apply_offsets + g * R;
    uint64_t mn = st.apply;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if ((uint32_t)i >= size || (uint32_t)i >= R) continue;
        uint64_t a = q.ap[i];
        if (!((st.cid.bitmask >> i) & 1u)) { a = st.apply; ap[i] = a; }   // OFF server
        if (larger(st.end, st.len, mn, a)) mn = a;
    }
    if (dist(st.end, st.len, mn) == 0) mn = device_get_tail(ring_view(b, g, st), st);
    const bool app = larger(st.end, st.len, mn, st.head) && !q.prev;
    const uint64_t nh = app ? mn : st.head;
    if (new_head) new_head[g] = nh;
    if (append_head) append_head[g] = app ? 1 : 0;
    if (min_apply) min_apply[g] = mn;
    return b.abs_base ? q.base + nh : ~0ull;
}

// The local (idx, term) of a candidate (poll_vote_requests,
// dare_server.c:1598-1620): the last of log_entries_to_nc_buf's determinants
// (dare_log.h:339-359: a ghost header is the determinant, the copy at 0 is
// stepped over), else the entry at log_get_tail (dare_log.h:402-457), else
// (0, 0).  A walk over a corrupt ring stops after len / 64 + 4 steps.
__device__ inline void local_idx_term(const apus_batch_t &b, uint64_t g, const apus_group_state_t &st, uint64_t &idx,
                                      uint64_t &term)
{
    const RingView v = ring_view(b, g, st);
    const uint64_t guard = st.len / kHdr + 4;
    uint64_t o = st.commit, last = ~0ull, n = 0;
    while (v.get_entry(o) && n++ < guard) {
        last = o;
        const uint32_t el = v.elen_at(o);
        if (v.len - o < el) o = 0;
        o += el;
    }
    idx = 0;
    term = 0;
    if (last == ~0ull) {
        uint64_t t = device_get_tail(v, st);
        if (t != st.len && v.get_entry(t)) last = t;
    }
    if (last != ~0ull) ld_idx_term(v.ring + last, idx, term);
}

}  // namespace apus
