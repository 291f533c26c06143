// Per-group quorum operations of quorum_tail_kernel (apus_commit.hip) and
// prune_kernel (apus_quorum.hip): the DARE median quorum (a4) and
// log_pruning's minimum (a7).  Every input a group's median and pruning read
// (its replica columns, self index, previous-HEAD flag, base) is requested
// in one batch of loads before any is used (QuorumIn), so a lane pays one
// memory round trip per group, not one per dependent load.
#pragma once

#include "apus_device.h"

namespace apus {

// Column loads and stores of the tail (plain: nontemporal forms measured no
// faster, profiles/r04/tail/; the dropped experiment branches are kept in
// profiles/r04/exp_knobs.diff).
template <typename T>
__device__ __forceinline__ T col_ld(const T *p)
{
    return *p;
}
template <typename T>
__device__ __forceinline__ void col_st(T *p, T v)
{
    *p = v;
}

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
// prev / base: the batch has prev_head / abs_base (kernels whose flags are
// compile-time constants pass them as constants: no branch between the loads)
template <int N, bool EXACT>
__device__ __forceinline__ void load_quorum_in(const apus_batch_t &b, uint64_t g, bool med, bool pr, bool prev,
                                               bool base, QuorumIn<N> &q)
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
                q.rend[i] = col_ld(rend + i);
                q.step[i] = col_ld(step + i);
                q.fail[i] = col_ld(fail + i);
            }
        }
    }
    if (pr) {
#pragma unroll
        for (int i = 0; i < N; ++i)
            if (EXACT || (uint32_t)i < R) q.ap[i] = col_ld(ap + i);
    }
    q.self = med ? col_ld(b.self_idx + g) : 0u;
    q.prev = pr && prev ? col_ld(b.prev_head + g) : 0u;
    q.base = pr && base ? col_ld(b.abs_base + g) : ~0ull;
}

// DARE median-offset quorum of a group (dare_ibv_rc.c:1650-1723) over N
// sort slots (N >= R; inputs for NR <= N replicas): the quirks are the
// reference's -- numeric sort, circular gate, TRANSIT min
template <int N, int NR>
__device__ __forceinline__ uint64_t median_slots(uint32_t R, const apus_group_state_t &st, const QuorumIn<NR> &q)
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

// The median over N sort slots, or over the NR replica slots alone when both
// configuration sizes are at most NR: slots past NR then hold no replica
// (never counted) and sort last (key ~0, the highest indices), so the value
// at rank (size - 1) / 2 < size is the same -- a third of the rank
// comparisons for N = 8, NR = 5
template <int N, int NR>
__device__ __forceinline__ uint64_t median_of(uint32_t R, const apus_group_state_t &st, const QuorumIn<NR> &q)
{
    if (NR < N && st.cid.size[0] <= (uint32_t)NR && st.cid.size[1] <= (uint32_t)NR)
        return median_slots<(NR < N ? NR : N), NR>(R, st, q);
    return median_slots<N, NR>(R, st, q);
}

// log_pruning's minimum of a group (dare_server.c:2026-2058, + log_get_tail
// when dist(min) == 0, dare_log.h:402-457): writes the apus_prune_out_t
// fields given (NULL = not wanted), resets OFF servers' apply offsets in
// place as the reference does, and returns the group's absolute watermark
// abs_base + new_head (~0 without abs_base)
template <int N>
__device__ __forceinline__ uint64_t prune_calc(const apus_batch_t &b, uint64_t g, const apus_group_state_t &st,
                                               const QuorumIn<N> &q, uint64_t &nh_out, bool &app_out,
                                               uint64_t &mn_out)
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
    nh_out = nh;
    app_out = app;
    mn_out = mn;
    return b.abs_base ? q.base + nh : ~0ull;
}
// the same, its results stored (NULL = not wanted)
template <int N>
__device__ __forceinline__ uint64_t prune_of(const apus_batch_t &b, uint64_t g, const apus_group_state_t &st,
                                             const QuorumIn<N> &q, uint64_t *new_head, uint8_t *append_head,
                                             uint64_t *min_apply)
{
    uint64_t nh, mn;
    bool app;
    const uint64_t w = prune_calc<N>(b, g, st, q, nh, app, mn);
    if (new_head) col_st(new_head + g, nh);
    if (append_head) col_st(append_head + g, (uint8_t)(app ? 1 : 0));
    if (min_apply) col_st(min_apply + g, mn);
    return w;
}

// ---------------------------------------------------------------------------
// The lazy remote-commit publish (dare_ibv_rc.c:1760-1822) of a group, on the
// commit `commit` the walk left: servers i < size (the walk's size) that are
// on, not self, not permanently failed, rc_connected and in LR_UPDATE_LOG, and
// whose commit is neither their end nor the leader's, get the leader's commit
// clamped to their end (in place); returns the mask of posted writes.
// rc: remote_commit[g][0..N), conn: rc_connected bits.  Columns past R are
// never visited.
// ---------------------------------------------------------------------------
template <int N, bool EXACT>
__device__ __forceinline__ uint32_t publish_from(const apus_batch_t &b, uint64_t g, const apus_group_state_t &st,
                                                 uint32_t self, uint64_t commit, const QuorumIn<N> &q,
                                                 const uint64_t (&rc)[N], uint32_t conn)
{
    const uint32_t R = EXACT ? (uint32_t)N : b.n_replicas;
    const uint32_t size = walk_size(st.cid);
    uint64_t *rcp = b.remote_commit + g * R;
    uint32_t mask = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if ((uint32_t)i >= size || (!EXACT && (uint32_t)i >= R) || (uint32_t)i == self) continue;
        if (!((st.cid.bitmask >> i) & 1u) || q.fail[i] >= APUS_PERMANENT_FAILURE || !((conn >> i) & 1u) ||
            q.step[i] != APUS_LR_UPDATE_LOG)
            continue;
        if (rc[i] == q.rend[i] || rc[i] == commit) continue;
        rcp[i] = larger(st.end, st.len, commit, q.rend[i]) ? q.rend[i] : commit;
        mask |= 1u << i;
    }
    return mask;
}

// the offsets log_append_entry may write at, as the batched append accepts
// them (apus_gpu.h): len within the ring, end and tail within len
__device__ __forceinline__ bool append_ok(const apus_batch_t &b, const apus_group_state_t &st)
{
    return st.len >= kHdr && st.len <= ring_cap(b) && st.end <= st.len && st.tail <= st.len;
}

// log_append_entry (dare_log.h:466-558) of one bare entry (NOOP or CONFIG;
// a CONFIG entry carries the cid words cw), as apus_append_batch appends it:
// the index from the tail entry (log_get_tail when tail == len), the header at
// end (at 0 when fewer than 64 B are left), a full log (end == head) appends
// nothing and returns 0.  st.end / st.tail are updated here and in memory
// (offsets_of), prev (prev_log_entry_head) is cleared.  Offsets the batched
// append refuses (append_ok) stop it: nothing is written, *stopped is set.
// The fields log_append_entry sets are stored (not sender@27, not bytes
// 41..47, no data for a NOOP); bytes one at a time (entries lie at any byte
// offset; rare groups).
__device__ inline uint64_t append_bare(const apus_batch_t &b, uint64_t g, apus_group_state_t &st, uint32_t &prev,
                                       uint64_t term, uint32_t type, uint64_t req_id, uint32_t clt_id,
                                       const uint64_t cw[2], bool &stopped)
{
    const uint64_t len = st.len, head = st.head;
    uint64_t end = st.end, tail = st.tail;
    if (!append_ok(b, st)) {
        stopped = true;
        return 0;
    }
    prev = 0;
    uint8_t *ring = b.ring + g * b.ring_stride;
    if (tail == len) tail = device_get_tail(ring_view(b, g, st), st);
    uint64_t idx = 1;
    if (end != len && dist(end, len, tail) != 0) {
        const uint64_t off = len - tail < kHdr ? 0 : tail;
        idx = ld_u64(ring + off) + 1;
    }
    uint64_t ret = 0;
    if (end != head) {
        uint8_t *e = ring + ((end == len || len - end < kHdr) ? 0 : end);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            e[kIdx + k] = (uint8_t)(idx >> (8 * k));
            e[kTerm + k] = (uint8_t)(term >> (8 * k));
            e[16 + k] = (uint8_t)(req_id >> (8 * k));
        }
        e[24] = (uint8_t)clt_id;
        e[25] = (uint8_t)(clt_id >> 8);
        e[kType] = (uint8_t)type;
#pragma unroll
        for (int k = 0; k < APUS_MAX_SERVER_COUNT; ++k) e[kReply + k] = 0;
        if (type == APUS_CONFIG) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                e[kData + k] = (uint8_t)(cw[0] >> (8 * k));      // data.cid
                e[kData + 8 + k] = (uint8_t)(cw[1] >> (8 * k));
            }
        }
        if (len - end < kHdr) end = 0;
        tail = end;
        end += kHdr;
        ret = idx;
    }
    st.end = end;
    st.tail = tail;
    uint64_t *off = offsets_of(b, g);
    off[kOffEnd] = end;
    off[kOffTail] = tail;
    return ret;
}

// force_log_pruning (dare_server.c:2069-2122) of a group on the log `st` as
// the commit call leaves it (st.commit = the walk's result): nothing when
// log_size < 0.75 * len (compared in double, as the reference does); else the
// first server with the smallest apply offset is the target; an ON target
// other than the leader is removed (cid bitmask in place, req_id / clt_id
// reset, the CONFIG append, apply_offsets[size] = apply where that column
// exists) and log_pruning (dare_server.c:2026-2058) runs on the log the
// append left (a log whose CONFIG append would be refused is left unchanged:
// APUS_FORCE_REFUSED).  Writes the apus_force_out_t fields and the pruning outputs;
// returns the group's absolute watermark (abs_base + new head; ~0 without).
template <int N, bool EXACT>
__device__ inline uint64_t force_prune_of(const apus_batch_t &b, uint64_t g, apus_group_state_t st, uint32_t self,
                                          const QuorumIn<N> &q, const uint64_t *sid, uint64_t *new_head,
                                          uint8_t *append_head, uint64_t *min_apply, const apus_force_out_t &fo,
                                          bool &stopped)
{
    const uint32_t R = EXACT ? (uint32_t)N : b.n_replicas;
    uint64_t *ap = b.apply_offsets + g * R;
    uint32_t action = APUS_FORCE_NONE, tg = self, prev = q.prev;
    uint64_t cfg = 0, nh = st.head, mn = 0;
    bool app = false;
    const uint64_t log_size = dist(st.end, st.len, st.head);
    if (!((double)log_size < 0.75 * (double)st.len)) {
        uint64_t apv[N];
#pragma unroll
        for (int i = 0; i < N; ++i) apv[i] = q.ap[i];
        const uint32_t size = ext_group_size(st.cid);
        uint64_t m = st.apply;
#pragma unroll
        for (int i = 0; i < N; ++i)
            if ((uint32_t)i < size && (EXACT || (uint32_t)i < R) && larger(st.end, st.len, m, apv[i])) {
                m = apv[i];
                tg = (uint32_t)i;
            }
        action = APUS_FORCE_PRUNE;
        const bool remove = tg != self && ((st.cid.bitmask >> tg) & 1u);
        // the CONFIG append's offsets first: a log the batched append refuses
        // is left unchanged (APUS_FORCE_REFUSED: no removal, no pruning)
        if (remove && !append_ok(b, st)) {
            action = APUS_FORCE_REFUSED;
            stopped = true;
        } else if (remove) {
            action = APUS_FORCE_REMOVE;
            st.cid.bitmask &= ~(1u << tg);                               // CID_SERVER_RM
            uint64_t *cw = cid_words(b, g);
            uint64_t w[2];
            __builtin_memcpy(w, &st.cid, sizeof w);
            cw[1] = w[1];
            if (fo.req_id) fo.req_id[g] = 0;
            if (fo.clt_id) fo.clt_id[g] = 0;
            cfg = append_bare(b, g, st, prev, sid[g] >> 9, APUS_CONFIG, 0, 0, w, stopped);   // (sid read only here)
            if (b.prev_head) b.prev_head[g] = (uint8_t)prev;
            if (size < R) {                                              // :2113, i == size
                ap[size] = st.apply;
#pragma unroll
                for (int i = 0; i < N; ++i)
                    if ((uint32_t)i == size) apv[i] = st.apply;
            }
        }
        if (action != APUS_FORCE_REFUSED) {
            // log_pruning over the replica columns that exist
            const uint32_t esz = ext_group_size(st.cid);
            mn = st.apply;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                if ((uint32_t)i >= esz || (!EXACT && (uint32_t)i >= R)) continue;
                uint64_t a = apv[i];
                if (!((st.cid.bitmask >> i) & 1u)) { a = st.apply; ap[i] = a; }      // OFF server
                if (larger(st.end, st.len, mn, a)) mn = a;
            }
            if (dist(st.end, st.len, mn) == 0) mn = device_get_tail(ring_view(b, g, st), st);
            app = larger(st.end, st.len, mn, st.head) && !prev;
            nh = app ? mn : st.head;
        }
    }
    if (fo.action) fo.action[g] = (uint8_t)action;
    if (fo.target) fo.target[g] = (uint8_t)tg;
    if (fo.cfg_idx) fo.cfg_idx[g] = cfg;
    if (new_head) new_head[g] = nh;
    if (append_head) append_head[g] = app ? 1 : 0;
    if (min_apply) min_apply[g] = mn;
    return b.abs_base ? q.base + nh : ~0ull;
}

// ---------------------------------------------------------------------------
// The failover pass of a group (a5, a6): shared by vote_tally_kernel /
// vote_rank_kernel (apus_quorum.hip) and quorum_tail_kernel's fused form
// (APUS_COMMIT_VOTE / APUS_COMMIT_RANK), so both call forms compute with the
// same code.  Replica slots i < N (N >= R; EXACT: R == N); every column a
// group reads is requested before any is used.
// ---------------------------------------------------------------------------

// The failover columns of a group, every one requested before any is used
// (in the tail after its median and pruning inputs, before its first store)
template <int N>
struct FailIn {
    uint64_t ack[N];                  // vote_ack (a5)
    uint64_t sid;                     // ctrl->sid (a6)
    uint64_t hb[N];                   // hb
    uint64_t rs[N], ri[N], rt[N];     // vote_req[i].sid / index / term
    const uint64_t *lrec;             // the group's 40-B records staged in LDS (the winner's cid), or null
};

template <int N, bool EXACT>
__device__ __forceinline__ void load_fail_in(const apus_batch_t &b, uint64_t g, bool vote, bool rank, FailIn<N> &f)
{
    const uint32_t R = EXACT ? (uint32_t)N : b.n_replicas;
    const uint64_t *ackp = b.vote_ack + g * R, *hbp = b.hb + g * R;
    // the requests' (sid, index, term): the packed vote_sit rows (24 B per
    // replica) when the batch has them, else the 40-B records -- an address
    // choice, not a branch between the loads
    const bool packed = b.vote_sit != nullptr;
    const uint64_t *req = packed ? b.vote_sit + g * R * 3 : reinterpret_cast<const uint64_t *>(b.vote_req + g * R);
    const uint32_t rq = packed ? 3u : (uint32_t)(sizeof(apus_vote_req_t) / 8);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const bool in = EXACT || (uint32_t)i < R;
        f.ack[i] = vote && in ? col_ld(ackp + i) : ~0ull;
        f.hb[i] = rank && in ? col_ld(hbp + i) : 0ull;
        f.rs[i] = rank && in ? col_ld(req + i * rq) : 0ull;
        f.ri[i] = rank && in ? col_ld(req + i * rq + 1) : 0ull;
        f.rt[i] = rank && in ? col_ld(req + i * rq + 2) : 0ull;
    }
    f.sid = rank ? col_ld(b.sid + g) : 0ull;
    f.lrec = nullptr;
}

// load_fail_in for a group whose request row is staged in LDS (the wave's
// LDS-DMA pieces, quorum_tail_kernel): the global columns only; the row is
// read by fail_rows_lds just before the ranking, once the group's other
// inputs are consumed (the wait for the pieces is then a wait for them alone).
template <int N, bool EXACT>
__device__ __forceinline__ void load_fail_in_lds(const apus_batch_t &b, uint64_t g, bool vote, FailIn<N> &f)
{
    const uint32_t R = EXACT ? (uint32_t)N : b.n_replicas;
    const uint64_t *ackp = b.vote_ack + g * R, *hbp = b.hb + g * R;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const bool in = EXACT || (uint32_t)i < R;
        f.ack[i] = vote && in ? col_ld(ackp + i) : ~0ull;
        f.hb[i] = in ? col_ld(hbp + i) : 0ull;
        f.rs[i] = f.ri[i] = f.rt[i] = 0;
    }
    f.sid = col_ld(b.sid + g);
    f.lrec = nullptr;
}

// the staged row (rq u64 per replica; records: 40-B vote_req_t records,
// whose cid the ranking's winner takes from LDS too)
template <int N, bool EXACT>
__device__ __forceinline__ void fail_rows_lds(const apus_batch_t &b, const uint64_t *lrow, uint32_t rq, bool records,
                                              FailIn<N> &f)
{
    const uint32_t R = EXACT ? (uint32_t)N : b.n_replicas;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < N; ++i) {
        const bool in = EXACT || (uint32_t)i < R;
        f.rs[i] = in ? lrow[i * rq] : 0ull;
        f.ri[i] = in ? lrow[i * rq + 1] : 0ull;
        f.rt[i] = in ? lrow[i * rq + 2] : 0ull;
    }
    f.lrec = records ? lrow : nullptr;
}

// poll_vote_count's tally (dare_server.c:1330-1373): vote_count[0..1] start at
// 1 (the candidate's own vote); for i < get_group_size, i != self, with a reply
// (vote_ack[i] != log->len): count i in the old (i < size[0]) and new
// (i < size[1]) configuration, mark it a voter (its log_offsets[i].commit and
// next_lr_step are updated there) and take the circular max into commit.  Won
// iff the old configuration has a majority and, outside CID_STABLE, the new
// one too.  Columns past n_replicas do not exist in a batch (never counted).
template <int N, bool EXACT>
__device__ __forceinline__ bool vote_from(const apus_batch_t &b, uint64_t g, const apus_group_state_t &st,
                                          uint32_t self, const FailIn<N> &f, const apus_vote_out_t &o)
{
    const uint32_t R = EXACT ? (uint32_t)N : b.n_replicas;
    const uint32_t size = group_size(st.cid);
    const uint32_t s0 = st.cid.size[0], s1 = st.cid.size[1];
    uint32_t c0 = 1, c1 = 1, mask = 0;
    uint64_t commit = st.commit;
#pragma unroll
    for (int i = 0; i < N; ++i) {
        if ((uint32_t)i >= size || (!EXACT && (uint32_t)i >= R) || (uint32_t)i == self) continue;
        const uint64_t rc = f.ack[i];
        if (rc == st.len) continue;                          // no reply
        if ((uint32_t)i < s0) ++c0;
        if ((uint32_t)i < s1) ++c1;
        mask |= 1u << i;
        if (larger(st.end, st.len, rc, commit)) commit = rc;
    }
    c0 &= 0xFF; c1 &= 0xFF;                                   // uint8_t vote_count[2]
    bool won = c0 >= s0 / 2 + 1;
    if (won && st.cid.state != APUS_CID_STABLE) won = c1 >= s1 / 2 + 1;
    if (o.won) o.won[g] = won ? 1 : 0;
    if (o.vote_count) { o.vote_count[2 * g] = (uint8_t)c0; o.vote_count[2 * g + 1] = (uint8_t)c1; }
    if (o.new_commit) o.new_commit[g] = commit;
    if (o.voters) o.voters[g] = (uint16_t)mask;
    return won;
}

#define APUS_SID_L(s) ((s) & (1ull << 8))
#define APUS_SID_TERM(s) ((s) >> 9)

// poll_vote_requests' ranking (dare_server.c:1526-1655) given the local last
// (idx, term) (lidx, lterm; :1598-1620): own SID with the L bit -> ignore the
// requests; a heartbeat of the possible leader with the same term -> adopt it;
// else the best request SID above [TERM|1|IDX] (requests at or below the best
// so far are cleared, :1558-1578), then the up-to-date test over every request
// (:1622-1655): the last request not older than the local log (or than the
// previous winner) takes the vote, every request examined is cleared.  The
// columns past n_replicas hold no request (sid 0): a slot i in [R, size) is
// cleared as the reference clears an empty request.
template <int N, bool EXACT>
__device__ __forceinline__ void rank_from(const apus_batch_t &b, uint64_t g, const apus_group_state_t &st,
                                          uint32_t self, uint64_t lidx, uint64_t lterm, const FailIn<N> &f,
                                          const apus_rank_out_t &o)
{
    const uint32_t R = EXACT ? (uint32_t)N : b.n_replicas;
    const uint32_t size = group_size(st.cid);
    const uint64_t sid = f.sid;
    uint64_t rs[N];
#pragma unroll
    for (int i = 0; i < N; ++i) rs[i] = (uint32_t)i < size ? f.rs[i] : 0ull;
    // slots [R, min(size, 16)): no column, an empty request
    const uint32_t hi = size < 16u ? size : 16u;
    const uint32_t ghost = hi > R ? ((1u << hi) - 1u) & ~((1u << R) - 1u) : 0u;
    const uint32_t selfbit = self < 32u ? 1u << self : 0u;
    uint8_t outcome;
    uint64_t new_sid = sid, ncid0 = 0, ncid1 = 0;    // the adopted cid, as its two 8-B words
    uint32_t clr = 0;
    if (APUS_SID_L(sid)) {
        outcome = APUS_RANK_LEADER_KNOWN;
    } else {
        const uint32_t pl = (uint32_t)(sid & 0xFF);
        uint64_t h = 0;
#pragma unroll
        for (int i = 0; i < N; ++i)
            if ((uint32_t)i == pl) h = f.hb[i];
        if (h != 0 && APUS_SID_TERM(h) == APUS_SID_TERM(sid)) {
            outcome = APUS_RANK_ADOPT_HB;
            new_sid = h;
        } else {
            const uint64_t old = sid | (1ull << 8);
            uint64_t best = old;
#pragma unroll
            for (int i = 0; i < N; ++i) {
                if ((uint32_t)i >= size || (uint32_t)i == self) continue;
                if (best >= rs[i]) { rs[i] = 0; clr |= 1u << i; continue; }
                best = rs[i];
            }
            clr |= ghost & ~selfbit;
            if (best == old) {
                outcome = APUS_RANK_NO_BETTER;
            } else {
                uint64_t hterm = APUS_SID_TERM(best);
                uint64_t bsid = old, bidx = lidx, bterm = lterm;
                int bi = -1;
#pragma unroll
                for (int i = 0; i < N; ++i) {
                    if ((uint32_t)i >= size) continue;
                    if (bsid > rs[i]) { rs[i] = 0; clr |= 1u << i; continue; }
                    if (hterm < APUS_SID_TERM(rs[i])) hterm = APUS_SID_TERM(rs[i]);
                    if (bterm > f.rt[i] || (bterm == f.rt[i] && bidx > f.ri[i])) { rs[i] = 0; clr |= 1u << i; continue; }
                    bidx = f.ri[i]; bterm = f.rt[i]; bsid = rs[i]; bi = i;
                    rs[i] = 0; clr |= 1u << i;
                }
                clr |= ghost;
                if (bsid == old) {
                    uint64_t s = sid;
                    s = (hterm << 9) | (s & 0x1FF);
                    s = (uint64_t)self | ((s >> 8) << 8);
                    new_sid = s;
                    outcome = APUS_RANK_RAISE_TERM;
                } else {
                    new_sid = bsid;
                    // the winner's cid: the one column read after the others
                    // (from LDS when the records are staged there)
                    if (f.lrec) {
                        ncid0 = f.lrec[bi * 5 + 3];
                        ncid1 = f.lrec[bi * 5 + 4];
                    } else {
                        const uint64_t *cw = reinterpret_cast<const uint64_t *>(&b.vote_req[g * R + bi].cid);
                        ncid0 = cw[0];
                        ncid1 = cw[1];
                    }
                    outcome = APUS_RANK_VOTE;
                }
            }
        }
    }
    if (o.outcome) o.outcome[g] = outcome;
    if (o.new_sid) o.new_sid[g] = new_sid;
    if (o.new_cid) {
        uint64_t *ow = reinterpret_cast<uint64_t *>(o.new_cid + g);
        ow[0] = ncid0;
        ow[1] = ncid1;
    }
    if (o.cleared) o.cleared[g] = (uint16_t)clr;
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
