// Per-group quorum operations shared by their own lane-per-group kernels
// (median_kernel, prune_kernel) and by commit_wave_kernel's block epilogue,
// which runs them for the 64 groups of a block after the block's walks
// (APUS_COMMIT_MEDIAN / APUS_COMMIT_PRUNE fused into the commit pass).
#pragma once

#include "apus_device.h"

namespace apus {

// DARE median-offset quorum of group g (dare_ibv_rc.c:1650-1723), N >= R:
// the quirks are the reference's -- numeric sort, circular gate, TRANSIT min
template <int N>
__device__ __forceinline__ uint64_t median_group(const apus_batch_t &b, uint64_t g, const apus_group_state_t &st)
{
    const uint32_t R = b.n_replicas;
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

// log_pruning's minimum of group g (dare_server.c:2026-2058, + log_get_tail
// when dist(min) == 0, dare_log.h:402-457): writes the apus_prune_out_t
// fields given (NULL = not wanted), resets OFF servers' apply offsets in
// place as the reference does, and returns the group's absolute watermark
// abs_base + new_head (~0 without abs_base)
constexpr int kPruneMaxR = 16;
__device__ __forceinline__ uint64_t prune_group(const apus_batch_t &b, uint64_t g, const apus_group_state_t &st,
                                                uint64_t *new_head, uint8_t *append_head, uint64_t *min_apply)
{
    const uint32_t R = b.n_replicas;
    const uint32_t size = ext_group_size(st.cid);
    uint64_t *ap = b.apply_offsets + g * R;
    uint64_t mn = st.apply;
#pragma unroll
    for (int i = 0; i < kPruneMaxR; ++i) {
        if ((uint32_t)i >= size || (uint32_t)i >= R) continue;
        uint64_t a = ap[i];
        if (!((st.cid.bitmask >> i) & 1u)) { a = st.apply; ap[i] = a; }   // OFF server
        if (larger(st.end, st.len, mn, a)) mn = a;
    }
    if (dist(st.end, st.len, mn) == 0) mn = device_get_tail(ring_view(b, g, st), st);
    const bool prev = b.prev_head ? b.prev_head[g] != 0 : false;
    const bool app = larger(st.end, st.len, mn, st.head) && !prev;
    const uint64_t nh = app ? mn : st.head;
    if (new_head) new_head[g] = nh;
    if (append_head) append_head[g] = app ? 1 : 0;
    if (min_apply) min_apply[g] = mn;
    return b.abs_base ? b.abs_base[g] + nh : ~0ull;
}

}  // namespace apus
