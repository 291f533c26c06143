/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see apus_oracle.h).
 *
 * Clean-room C restatement of the APUS quorum/commit hot path.  Every
 * function names the reference code (file:line, relative to the reference
 * tree) whose behaviour it restates.  No reference source is copied; the
 * reference's own dare_log.h is compiled separately (oracle/_ref) to check
 * this file (tests/test_oracle_vs_ref.py).
 *
 * The synthetic trace generator (apus_oracle_gen_*) is the specification the
 * device generator (rdma-paxos_amd/csrc/apus_gen.hip) must reproduce byte
 * for byte; see DESIGN.md "Synthetic traces".
 */
#include "apus_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ */
/* byte image access (entries are not aligned: log_entry_len = 64+len) */
/* ------------------------------------------------------------------ */
static inline uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint16_t rd16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline void wr64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
static inline void wr16(uint8_t *p, uint16_t v) { memcpy(p, &v, 2); }

#define E_IDX    0
#define E_TERM   8
#define E_REQ   16
#define E_CLT   24
#define E_TYPE  26
#define E_SNDR  27
#define E_REPLY 28
#define E_DATA  48

typedef struct {
    const uint8_t *ring;
    uint64_t end, len;
} view_t;

static inline view_t mkview(const uint8_t *ring, const apus_group_state_t *st)
{
    view_t v = { ring, st->end, st->len };
    return v;
}

/* log_offset_end_distance, dare_log.h:255-262 (inline here; the exported
 * form below is for the tests -- a call through the PLT per step doubled the
 * walk's CPU time) */
static inline uint64_t dist_(uint64_t end, uint64_t len, uint64_t off)
{
    if (end == len) return 0;
    return end >= off ? end - off : len - (off - end);
}
uint64_t apus_oracle_dist(uint64_t end, uint64_t len, uint64_t off) { return dist_(end, len, off); }

/* log_is_offset_larger, dare_log.h:269-282 */
static inline int larger_(uint64_t end, uint64_t len, uint64_t a, uint64_t b)
{
    return dist_(end, len, a) < dist_(end, len, b);
}
int apus_oracle_larger(uint64_t end, uint64_t len, uint64_t a, uint64_t b) { return larger_(end, len, a, b); }

static inline uint64_t vdist(const view_t *v, uint64_t o) { return dist_(v->end, v->len, o); }
static inline int vlarger(const view_t *v, uint64_t a, uint64_t b) { return larger_(v->end, v->len, a, b); }

/* log_entry_len, dare_log.h:228-234: NOOP/CONFIG/HEAD are bare headers,
 * every other type carries sm_cmd_t bytes */
static inline uint32_t ent_len(const uint8_t *e)
{
    uint8_t t = e[E_TYPE];
    if (t == APUS_NOOP || t == APUS_CONFIG || t == APUS_HEAD) return APUS_ENTRY_HDR;
    return APUS_ENTRY_HDR + (uint32_t)rd16(e + E_DATA);
}

/* log_fit_entry_header / log_fit_entry, dare_log.h:201-205, 241-247
 * (unsigned arithmetic kept: an offset past len "fits") */
static inline int fit_hdr(const view_t *v, uint64_t o) { return v->len - o >= APUS_ENTRY_HDR; }
static inline int fit_ent(const view_t *v, uint64_t o, const uint8_t *e) { return v->len - o >= ent_len(e); }

/* log_get_entry, dare_log.h:316-332 */
static inline const uint8_t *get_entry(const view_t *v, uint64_t *o)
{
    if (v->end == v->len) return NULL;
    if (vdist(v, *o) == 0) return NULL;
    if (!fit_hdr(v, *o)) *o = 0;
    return v->ring + *o;
}

static inline uint64_t step_guard(uint64_t len) { return len / APUS_ENTRY_HDR + 4; }

/* ------------------------------------------------------------------ */
/* a3: APUS reply-count commit walk, dare_ibv_rc.c:1725-1758           */
/* `size` is the value left by the median loop (dare_ibv_rc.c:1656):   */
/* cid.size[1] in CID_TRANSIT, cid.size[0] otherwise.                  */
/* ------------------------------------------------------------------ */
static inline uint8_t walk_size(const apus_cid_t *cid)
{
    return cid->state == APUS_CID_TRANSIT ? cid->size[1] : cid->size[0];
}

uint64_t apus_oracle_commit_walk(const uint8_t *ring, const apus_group_state_t *st,
                                 uint8_t self, int *advanced, uint32_t *n_committed,
                                 int *corrupt)
{
    view_t v = mkview(ring, st);
    uint8_t size = walk_size(&st->cid);
    int need = size / 2 + 1;
    uint64_t m = st->commit, steps = 0, guard = step_guard(st->len);
    uint32_t n = 0;
    /* Build-defined (the reference spins forever or reads past entries[]):
     * a state with commit or end beyond len, or a walk longer than
     * len/64 + 4 steps before it stops, is corrupt and leaves commit. */
    *corrupt = 0;
    *n_committed = 0;
    *advanced = 0;
    if (st->commit > st->len || st->end > st->len) { *corrupt = 1; return st->commit; }
    while (vdist(&v, m)) {
        if (++steps > guard) { *corrupt = 1; break; }
        const uint8_t *e = get_entry(&v, &m);
        if (!fit_ent(&v, m, e)) { m = 0; continue; }      /* ghost header */
        int votes = 0;
        for (int i = 0; i < size; i++)
            if (i == self || e[E_REPLY + i] == 1) votes++;
        if (votes < need) break;
        m += ent_len(e);
        n++;
    }
    *n_committed = n;
    if (!*corrupt && vlarger(&v, m, st->commit)) { *advanced = 1; return m; }
    return st->commit;
}

/* ------------------------------------------------------------------ */
/* a12 (build-defined): Adler-32 (RFC 1950) over the concatenated      */
/* images of the entries from commit to end, in walk order.  An        */
/* entry's image is its whole span [0, log_entry_len) with bytes        */
/* [27, 48) -- sender, reply[13], pad -- read as zero.  DARE replicates */
/* the leader's raw byte range [remote_end, end) (dare_ibv_rc.c:1532-   */
/* 1545), so every replica holds each span byte-identically except     */
/* these bytes, which are rewritten in place after replication          */
/* (reply: dare_ibv_rc.c:1839; sender: dare_server.c:1804).  Ghost      */
/* headers and wrap gaps belong to no entry and are not in the image.   */
/* ------------------------------------------------------------------ */
#define ADLER_MOD 65521u
uint32_t apus_oracle_adler32(const uint8_t *buf, size_t n, uint32_t adler)
{
    /* RFC 1950 with zlib's deferred reduction: at most NMAX = 5552 bytes
     * between reductions keep b below 2^32 */
    uint32_t a = adler & 0xFFFF, b = adler >> 16;
    while (n) {
        size_t k = n < 5552 ? n : 5552;
        n -= k;
        while (k--) {
            a += *buf++;
            b += a;
        }
        a %= ADLER_MOD;
        b %= ADLER_MOD;
    }
    return (b << 16) | a;
}

static const uint8_t k_zero21[21];

uint32_t apus_oracle_checksum(const uint8_t *ring, const apus_group_state_t *st)
{
    view_t v = mkview(ring, st);
    uint32_t ad = 1;
    uint64_t m = st->commit, steps = 0, guard = step_guard(st->len);
    if (st->commit > st->len || st->end > st->len) return ad;     /* corrupt state */
    while (vdist(&v, m)) {
        if (++steps > guard) break;                               /* truncated */
        const uint8_t *e = get_entry(&v, &m);
        if (!fit_ent(&v, m, e)) { m = 0; continue; }
        uint32_t el = ent_len(e);
        ad = apus_oracle_adler32(e, 27, ad);
        ad = apus_oracle_adler32(k_zero21, 21, ad);
        ad = apus_oracle_adler32(e + E_DATA, el - E_DATA, ad);
        m += el;
    }
    return ad;
}

/* ------------------------------------------------------------------ */
/* a4: DARE median-offset quorum, dare_ibv_rc.c:1650-1723              */
/* ------------------------------------------------------------------ */
uint64_t apus_oracle_median(const apus_group_state_t *st, uint8_t self,
                            const uint64_t *remote_end, const uint8_t *lr_step,
                            const uint8_t *fail_count)
{
    view_t v = { NULL, st->end, st->len };
    uint64_t offs[APUS_MAX_SERVER_COUNT + 3];
    uint64_t min = st->commit;
    int transit = st->cid.state == APUS_CID_TRANSIT;
    memset(offs, 0, sizeof offs);
    for (int j = 0; j < 2; ) {
        uint8_t size = st->cid.size[j];
        int cnt = 0;
        for (int i = 0; i < size; i++) {
            if (i == self) { offs[i] = st->end; continue; }
            if (!((st->cid.bitmask >> i) & 1u) || fail_count[i] >= APUS_PERMANENT_FAILURE ||
                lr_step[i] != APUS_LR_UPDATE_LOG) {
                offs[i] = st->commit;
                continue;
            }
            offs[i] = remote_end[i];
            if (vlarger(&v, offs[i], min)) cnt++;
        }
        if (cnt < size / 2) {
            if (!transit) break;
            if (j == 0) { j++; continue; }
            break;
        }
        /* ascending, by raw numeric value (not circular order) */
        for (int i = 1; i < size; i++) {
            uint64_t x = offs[i];
            int k = i;
            for (; k > 0 && offs[k - 1] > x; k--) offs[k] = offs[k - 1];
            offs[k] = x;
        }
        uint64_t med = offs[(size - 1) / 2];
        if (!transit) { min = med; break; }
        if (j == 0) min = med;
        else if (vlarger(&v, min, med)) min = med;
        j++;
    }
    return min;
}

/* ------------------------------------------------------------------ */
/* a5: poll_vote_count tally, dare_server.c:1327-1373                  */
/* ------------------------------------------------------------------ */
static inline uint8_t group_size(const apus_cid_t *c)      /* dare_config.h:89-97 */
{
    if (c->state != APUS_CID_TRANSIT) return c->size[0];
    return c->size[0] < c->size[1] ? c->size[1] : c->size[0];
}
static inline uint8_t ext_group_size(const apus_cid_t *c)  /* dare_config.h:78-86 */
{
    if (c->state == APUS_CID_STABLE) return c->size[0];
    return c->size[0] < c->size[1] ? c->size[1] : c->size[0];
}

int apus_oracle_vote_tally(const apus_group_state_t *st, uint8_t self,
                           const uint64_t *vote_ack, uint8_t vc[2],
                           uint64_t *new_commit, uint16_t *voters)
{
    view_t v = { NULL, st->end, st->len };
    uint8_t size = group_size(&st->cid);
    uint8_t c0 = 1, c1 = 1;
    uint64_t commit = st->commit;
    uint16_t mask = 0;
    for (int i = 0; i < size; i++) {
        if (i == self) continue;
        uint64_t rc = vote_ack[i];
        if (rc == st->len) continue;                 /* no reply */
        if (i < st->cid.size[0]) c0++;
        if (i < st->cid.size[1]) c1++;
        mask |= (uint16_t)(1u << i);
        if (vlarger(&v, rc, commit)) commit = rc;
    }
    vc[0] = c0; vc[1] = c1;
    *new_commit = commit;
    *voters = mask;
    if (c0 < st->cid.size[0] / 2 + 1) return 0;
    if (st->cid.state != APUS_CID_STABLE && c1 < st->cid.size[1] / 2 + 1) return 0;
    return 1;
}

/* ------------------------------------------------------------------ */
/* a6: poll_vote_requests ranking, dare_server.c:1526-1655             */
/* SID = [TERM(55)|L(1)|IDX(8)], dare_server.h:52-72                   */
/* ------------------------------------------------------------------ */
#define SID_L(s)    ((s) & (1ull << 8))
#define SID_TERM(s) ((s) >> 9)
#define SID_IDX(s)  ((uint8_t)((s) & 0xFF))

uint8_t apus_oracle_vote_rank(const apus_group_state_t *st, uint8_t self, uint64_t sid,
                              const uint64_t *hb, uint32_t n_hb,
                              const apus_vote_req_t *req, uint64_t local_idx,
                              uint64_t local_term, uint64_t *new_sid,
                              apus_cid_t *new_cid, uint16_t *cleared)
{
    uint8_t size = group_size(&st->cid);
    uint64_t rs[APUS_MAX_SERVER_COUNT];
    uint16_t clr = 0;
    memset(new_cid, 0, sizeof *new_cid);
    *cleared = 0;
    *new_sid = sid;
    if (SID_L(sid)) return APUS_RANK_LEADER_KNOWN;
    uint8_t pl = SID_IDX(sid);
    uint64_t h = pl < n_hb ? hb[pl] : 0;
    if (h != 0 && SID_TERM(h) == SID_TERM(sid)) { *new_sid = h; return APUS_RANK_ADOPT_HB; }

    for (int i = 0; i < size; i++) rs[i] = req[i].sid;
    uint64_t old = sid | (1ull << 8), best = old;
    for (int i = 0; i < size; i++) {
        if (i == self) continue;
        if (best >= rs[i]) { rs[i] = 0; clr |= (uint16_t)(1u << i); continue; }
        best = rs[i];
    }
    if (best == old) { *cleared = clr; return APUS_RANK_NO_BETTER; }

    uint64_t hterm = SID_TERM(best);
    uint64_t bsid = old, bidx = local_idx, bterm = local_term;
    apus_cid_t bcid;
    memset(&bcid, 0, sizeof bcid);
    for (int i = 0; i < size; i++) {
        if (bsid > rs[i]) { rs[i] = 0; clr |= (uint16_t)(1u << i); continue; }
        if (hterm < SID_TERM(rs[i])) hterm = SID_TERM(rs[i]);
        if (bterm > req[i].term || (bterm == req[i].term && bidx > req[i].index)) {
            rs[i] = 0; clr |= (uint16_t)(1u << i);
            continue;
        }
        bidx = req[i].index; bterm = req[i].term; bsid = rs[i]; bcid = req[i].cid;
        rs[i] = 0; clr |= (uint16_t)(1u << i);
    }
    *cleared = clr;
    if (bsid == old) {
        uint64_t s = sid;
        s = (hterm << 9) | (s & 0x1FF);            /* SID_SET_TERM */
        s = (uint64_t)self | ((s >> 8) << 8);      /* SID_SET_IDX  */
        *new_sid = s;
        return APUS_RANK_RAISE_TERM;
    }
    *new_sid = bsid;
    *new_cid = bcid;
    return APUS_RANK_VOTE;
}

/* ------------------------------------------------------------------ */
/* log_get_tail, dare_log.h:402-457 (tail recorded BEFORE the ghost    */
/* test, unlike the commit walk)                                       */
/* ------------------------------------------------------------------ */
static uint64_t tail_scan(const view_t *v, uint64_t o, uint64_t guard)
{
    uint64_t tail = v->len, steps = 0;
    const uint8_t *e;
    while ((e = get_entry(v, &o)) != NULL) {
        if (++steps > guard) break;
        tail = o;
        if (!fit_ent(v, o, e)) o = 0;
        o += ent_len(e);
    }
    return tail;
}

uint64_t apus_oracle_log_get_tail(const uint8_t *ring, const apus_group_state_t *st)
{
    view_t v = mkview(ring, st);
    if (st->tail != st->len) return st->tail;
    if (st->end == st->len) return st->len;
    uint64_t g = step_guard(st->len), t;
    if ((t = tail_scan(&v, st->commit, g)) != st->len) return t;
    if ((t = tail_scan(&v, st->apply, g)) != st->len) return t;
    return tail_scan(&v, st->head, g);
}

/* ------------------------------------------------------------------ */
/* a7: log_pruning minimum, dare_server.c:2026-2058                    */
/* ------------------------------------------------------------------ */
uint64_t apus_oracle_min_apply(const uint8_t *ring, const apus_group_state_t *st,
                               uint64_t *apply_offsets, int prev_head,
                               uint64_t *new_head, int *append_head)
{
    view_t v = mkview(ring, st);
    uint8_t size = ext_group_size(&st->cid);
    uint64_t min = st->apply;
    for (int i = 0; i < size; i++) {
        if (!((st->cid.bitmask >> i) & 1u)) apply_offsets[i] = st->apply;
        if (vlarger(&v, min, apply_offsets[i])) min = apply_offsets[i];
    }
    uint64_t m = min;
    if (!vdist(&v, m)) m = apus_oracle_log_get_tail(ring, st);
    if (vlarger(&v, m, st->head) && !prev_head) { *new_head = m; *append_head = 1; }
    else { *new_head = st->head; *append_head = 0; }
    return m;
}

/* ------------------------------------------------------------------ */
/* The lazy remote-commit publish that ends update_remote_logs,        */
/* dare_ibv_rc.c:1760-1822.  `size` is the walk's (the median loop's   */
/* leftover, :1656).  A server is skipped when it is the leader or OFF */
/* (:1762-1764), permanently failed, not rc_connected or not in        */
/* LR_UPDATE_LOG (:1769-1775), or when its commit already equals its   */
/* end or the leader's commit (:1778-1782); otherwise its commit is    */
/* set to the leader's, clamped to its end when that is circularly     */
/* smaller (:1783-1787), and an 8-B write is posted (:1810).  Columns  */
/* past R do not exist in a batch: those servers are not visited.     */
/* ------------------------------------------------------------------ */
uint16_t apus_oracle_publish(const apus_group_state_t *st, uint8_t self, uint32_t R, uint64_t commit,
                             const uint64_t *rend, uint64_t *rcommit, const uint8_t *step,
                             const uint8_t *fail, uint16_t rc_conn)
{
    view_t v = { NULL, st->end, st->len };
    uint8_t size = walk_size(&st->cid);
    uint16_t mask = 0;
    for (uint32_t i = 0; i < size && i < R; i++) {
        if (i == self || !((st->cid.bitmask >> i) & 1u)) continue;
        if (fail[i] >= APUS_PERMANENT_FAILURE || !((rc_conn >> i) & 1u) || step[i] != APUS_LR_UPDATE_LOG)
            continue;
        if (rcommit[i] == rend[i] || rcommit[i] == commit) continue;
        rcommit[i] = commit;
        if (vlarger(&v, rcommit[i], rend[i])) rcommit[i] = rend[i];
        mask |= (uint16_t)(1u << i);
    }
    return mask;
}

/* ------------------------------------------------------------------ */
/* force_log_pruning, dare_server.c:2069-2122: nothing below           */
/* log_size < 0.75 * len (compared in double, as the reference does);  */
/* else the server with the smallest apply offset (strict: the first   */
/* minimum) is the target.  target == self -> log_pruning; target OFF  */
/* -> log_pruning; otherwise the target is removed from the cid, the   */
/* config's req_id / clt_id are reset, a CONFIG entry carrying the new */
/* cid is appended (log_append_entry: it also clears prev_head),       */
/* apply_offsets[size] = apply (the loop variable after the loop,      */
/* :2113; skipped when that column does not exist) and log_pruning     */
/* runs on the log the append left.                                    */
/* ------------------------------------------------------------------ */
int apus_oracle_force_prune(uint8_t *ring, uint64_t stride, apus_group_state_t *st, uint8_t self,
                            uint32_t R, uint64_t sid, uint64_t *apply_offsets, uint8_t *prev_head,
                            uint64_t *req_id, uint16_t *clt_id, uint64_t *new_head, int *append_head,
                            uint64_t *min_apply, uint8_t *target, uint64_t *cfg_idx, int *corrupt)
{
    view_t v = mkview(ring, st);
    uint64_t log_size = vdist(&v, st->head);
    int action = APUS_FORCE_PRUNE;
    *new_head = st->head;
    *append_head = 0;
    *min_apply = 0;
    *target = self;
    *cfg_idx = 0;
    *corrupt = 0;
    if ((double)log_size < 0.75 * (double)st->len) return APUS_FORCE_NONE;
    uint8_t size = ext_group_size(&st->cid), tg = self;
    uint64_t min = st->apply;
    for (uint32_t i = 0; i < size && i < R; i++) {
        if (vlarger(&v, min, apply_offsets[i])) { min = apply_offsets[i]; tg = (uint8_t)i; }
    }
    *target = tg;
    if (tg != self && ((st->cid.bitmask >> tg) & 1u)) {
        /* the CONFIG append's offsets checked first: a log the batched append
         * refuses is left as it is (APUS_FORCE_REFUSED, apus_gpu.h) */
        if (!(st->len >= APUS_ENTRY_HDR && st->len <= stride && st->end <= st->len && st->tail <= st->len)) {
            *corrupt = 1;
            return APUS_FORCE_REFUSED;
        }
        action = APUS_FORCE_REMOVE;
        st->cid.bitmask &= ~(1u << tg);                           /* CID_SERVER_RM */
        *req_id = 0;
        *clt_id = 0;
        apus_append_entry_t q;
        memset(&q, 0, sizeof q);
        q.type = APUS_CONFIG;                                     /* req_id 0, clt_id 0, data = cid */
        uint64_t idx = 0, last = 0;
        *corrupt = apus_oracle_append_group(ring, stride, st, prev_head, sid >> 9, &q, 1,
                                            (const uint8_t *)&st->cid, sizeof(apus_cid_t), &idx, &last);
        *cfg_idx = idx;
        if (size < R) apply_offsets[size] = st->apply;           /* :2113, i == size */
    }
    int app;
    uint64_t nh;
    /* log_pruning (:2026-2058) over the replica columns that exist */
    view_t w = mkview(ring, st);
    uint8_t esz = ext_group_size(&st->cid);
    uint64_t mn = st->apply;
    for (uint32_t i = 0; i < esz && i < R; i++) {
        if (!((st->cid.bitmask >> i) & 1u)) apply_offsets[i] = st->apply;
        if (vlarger(&w, mn, apply_offsets[i])) mn = apply_offsets[i];
    }
    if (!vdist(&w, mn)) mn = apus_oracle_log_get_tail(ring, st);
    app = vlarger(&w, mn, st->head) && !*prev_head;
    nh = app ? mn : st->head;
    *new_head = nh;
    *append_head = app;
    *min_apply = mn;
    return action;
}

/* ------------------------------------------------------------------ */
/* a8: log_find_remote_end_offset, dare_log.h:367-394                  */
/* ------------------------------------------------------------------ */
int apus_oracle_find_remote_end(const uint8_t *ring, const apus_group_state_t *st,
                                const apus_entry_det_t *dets, uint64_t n, uint64_t *out)
{
    view_t v = mkview(ring, st);
    uint64_t o = 0;
    if (n == 0) return 1;
    for (uint64_t i = 0; i < n; i++) {
        o = dets[i].offset;
        const uint8_t *e = get_entry(&v, &o);
        if (!e) { *out = o; return 0; }
        if (rd64(e + E_IDX) != dets[i].idx || rd64(e + E_TERM) != dets[i].term) {
            *out = o;
            return 0;
        }
        if (!fit_ent(&v, o, e)) o = 0;
        o += ent_len(e);
    }
    *out = o;
    return 0;
}

/* ------------------------------------------------------------------ */
/* a9: log_entries_to_nc_buf, dare_log.h:339-359 (capped at max_dets)  */
/* ------------------------------------------------------------------ */
uint32_t apus_oracle_nc_build(const uint8_t *ring, const apus_group_state_t *st,
                              apus_entry_det_t *dets, uint32_t max_dets)
{
    view_t v = mkview(ring, st);
    uint64_t o = st->commit;
    uint32_t n = 0;
    const uint8_t *e;
    while (n < max_dets && (e = get_entry(&v, &o)) != NULL) {
        dets[n].idx = rd64(e + E_IDX);
        dets[n].term = rd64(e + E_TERM);
        dets[n].offset = o;
        n++;
        if (!fit_ent(&v, o, e)) o = 0;
        o += ent_len(e);
    }
    return n;
}

/* local last (idx, term) as poll_vote_requests derives it,
 * dare_server.c:1598-1620 */
void apus_oracle_last_idx_term(const uint8_t *ring, const apus_group_state_t *st,
                               uint64_t out[2])
{
    view_t v = mkview(ring, st);
    uint64_t o = st->commit, steps = 0, guard = step_guard(st->len);
    const uint8_t *e, *last = NULL;
    while ((e = get_entry(&v, &o)) != NULL) {
        if (++steps > guard) break;
        last = e;
        if (!fit_ent(&v, o, e)) o = 0;
        o += ent_len(e);
    }
    if (!last) {
        uint64_t t = apus_oracle_log_get_tail(ring, st);
        if (t == st->len) { out[0] = out[1] = 0; return; }
        last = get_entry(&v, &t);
        if (!last) { out[0] = out[1] = 0; return; }
    }
    out[0] = rd64(last + E_IDX);
    out[1] = rd64(last + E_TERM);
}

/* ================================================================== */
/* Log append: log_append_entry, src/include/dare/dare_log.h:466-558    */
/* (called per queued message by get_tailq_message,                   */
/*  src/dare/dare_ibv_ud.c:780-790)                                    */
/* ================================================================== */
static int csm_class(uint8_t t) { return !(t == APUS_NOOP || t == APUS_CONFIG || t == APUS_HEAD); }

/* the header fields log_append_entry sets (dare_log.h:494-499): idx, term,
 * req_id, clt_id, type, and memset(reply, 0, MAX_SERVER_COUNT).  sender
 * (@27) and bytes 41..47 are not written. */
static void put_fields(uint8_t *e, uint64_t idx, uint64_t term, uint64_t req, uint16_t clt, uint8_t type)
{
    wr64(e + 0, idx);
    wr64(e + 8, term);
    wr64(e + 16, req);
    wr16(e + 24, clt);
    e[26] = type;
    memset(e + 28, 0, APUS_MAX_SERVER_COUNT);
}

int apus_oracle_append_group(uint8_t *ring, uint64_t stride, apus_group_state_t *st,
                             uint8_t *prev_head, uint64_t term,
                             const apus_append_entry_t *q, uint32_t n,
                             const uint8_t *payload, uint64_t payload_bytes,
                             uint64_t *idx_out, uint64_t *last_idx)
{
    const uint64_t len = st->len, head = st->head;
    uint64_t end = st->end, tail = st->tail;
    for (uint32_t k = 0; k < n; k++) idx_out[k] = 0;
    if (n == 0) return 0;
    /* offsets a device cannot honour in bounds (undefined in the reference) */
    if (!(len >= APUS_ENTRY_HDR && len <= stride && end <= len && tail <= len)) return 1;
    int stopped = 0;
    for (uint32_t k = 0; k < n; k++) {
        const apus_append_entry_t *m = &q[k];
        const int csm = csm_class(m->type);
        uint64_t need = 0, clen = 0;
        if (csm) {
            if (m->data_off > payload_bytes || payload_bytes - m->data_off < 2) { stopped = 1; break; }
            clen = rd16(payload + m->data_off);               /* sm_cmd_t.len */
            need = 2 + clen;
        } else if (m->type == APUS_CONFIG) {
            need = sizeof(apus_cid_t);
        } else if (m->type == APUS_HEAD) {
            need = 8;
        }
        if (need && (m->data_off > payload_bytes || payload_bytes - m->data_off < need)) { stopped = 1; break; }
        if (csm && APUS_ENTRY_HDR + clen > len) { stopped = 1; break; }
        const uint8_t *data = payload + m->data_off;

        if (m->type != APUS_HEAD) *prev_head = 0;                          /* :478-481 */
        if (tail == len) {                                                 /* :484-486 */
            apus_group_state_t cur = *st;
            cur.end = end;
            cur.tail = tail;
            tail = apus_oracle_log_get_tail(ring, &cur);
        }
        /* log_get_entry(log, &offset = tail) -> idx (:487-489) */
        uint64_t idx = 1;
        if (end != len && dist_(end, len, tail) != 0) {
            uint64_t off = tail;
            if (len - off < APUS_ENTRY_HDR) off = 0;
            idx = rd64(ring + off) + 1;
        }
        /* log_add_new_entry (:214-221) */
        if (end == head) { *last_idx = 0; continue; }                     /* log full: return 0 */
        uint8_t *e = ring + ((end == len || len - end < APUS_ENTRY_HDR) ? 0 : end);
        put_fields(e, idx, term, m->req_id, m->clt_id, m->type);
        if (len - end < APUS_ENTRY_HDR) end = 0;                          /* :500-502 */
        uint64_t elen = APUS_ENTRY_HDR;
        if (m->type == APUS_CONFIG) {
            memcpy(e + 48, data, sizeof(apus_cid_t));
        } else if (m->type == APUS_HEAD) {
            memcpy(e + 48, data, 8);
        } else if (csm) {
            wr16(e + 48, (uint16_t)clen);
            elen = APUS_ENTRY_HDR + clen;
            if (len - end < elen) {                                       /* !log_fit_entry */
                end = 0;                                                  /* ghost header stays */
                if (end == head) { *last_idx = 0; continue; }
                e = ring;
                put_fields(e, idx, term, m->req_id, m->clt_id, m->type);
                wr16(e + 48, (uint16_t)clen);
            }
            memcpy(e + 50, data + 2, clen);
        }
        tail = end;                                                       /* :547-550 */
        end += elen;
        idx_out[k] = idx;
        *last_idx = idx;
    }
    st->end = end;
    st->tail = tail;
    return stopped;
}

/* persist_new_entries, src/dare/dare_server.c:1792-1810, for replica copy
 * i (all copies are byte-identical, so the leader's ring stands for each):
 * the leader stamps sender, a follower's rc_send_entries_reply
 * (src/dare/dare_ibv_rc.c:1828-1863) sets reply[i] of the entry. */
int apus_oracle_persist_one(uint8_t *ring, uint64_t stride, const apus_group_state_t *st,
                            uint8_t self, uint32_t i, uint64_t *old_end, uint32_t limit)
{
    const uint64_t end = st->end, len = st->len;
    uint64_t oe = *old_end;
    if (!(len >= APUS_ENTRY_HDR && len <= stride && end <= len && oe <= len)) return 1;
    const uint64_t guard = step_guard(len);
    uint64_t steps = 0;
    uint32_t n = 0;
    int corrupt = 0;
    while (larger_(end, len, end, oe)) {
        if (n >= limit) break;
        if (++steps > guard) { corrupt = 1; break; }
        if (len - oe < APUS_ENTRY_HDR) oe = 0;                            /* log_get_entry */
        uint8_t *e = ring + oe;
        if (len - oe < ent_len(e)) { oe = 0; continue; }                  /* ghost header */
        if (i == self) e[27] = (uint8_t)i;                                /* entry->sender */
        else e[28 + i] = 1;                                               /* reply[config.idx] */
        oe += ent_len(e);
        n++;
    }
    *old_end = oe;
    return corrupt;
}

void apus_oracle_append_batch(const apus_batch_t *b, const apus_append_in_t *in, const apus_append_out_t *out,
                              uint64_t *stopped)
{
    uint64_t bad = 0;
    for (uint64_t g = 0; g < b->n_groups; g++) {
        uint32_t n = in->n_entries ? in->n_entries[g] : in->max_entries;
        if (n > in->max_entries) n = in->max_entries;
        uint8_t ph = b->prev_head ? b->prev_head[g] : 0;
        uint64_t term = in->term ? in->term[g] : (b->sid[g] >> 9);
        uint64_t last = out->last_idx ? out->last_idx[g] : 0;
        uint64_t *idx = out->idx + g * in->max_entries;
        bad += (uint64_t)apus_oracle_append_group(b->ring + g * b->ring_stride, b->ring_stride, &b->state[g], &ph,
                                                  term, in->entries + g * in->max_entries, n, in->payload,
                                                  in->payload_bytes, idx, &last);
        for (uint32_t k = n; k < in->max_entries; k++) idx[k] = 0;
        if (b->prev_head) b->prev_head[g] = ph;
        if (out->last_idx) out->last_idx[g] = last;
    }
    if (stopped) *stopped = bad;
}

void apus_oracle_persist_batch(const apus_batch_t *b, const apus_persist_in_t *in, uint64_t *corrupt)
{
    uint64_t bad = 0;
    const uint32_t R = b->n_replicas;
    for (uint64_t g = 0; g < b->n_groups; g++)
        for (uint32_t i = 0; i < R; i++)
            bad += (uint64_t)apus_oracle_persist_one(b->ring + g * b->ring_stride, b->ring_stride, &b->state[g],
                                                     b->self_idx[g], i, &in->old_end[g * R + i],
                                                     in->limit ? in->limit[g * R + i] : 0xFFFFFFFFu);
    if (corrupt) *corrupt = bad;
}

/* ------------------------------------------------------------------ */
/* The proxy's stable-storage records (the BDB record format, 8f.3)    */
/* ------------------------------------------------------------------ */
/* stablestorage_save_request, src/proxy/proxy.c:269-291: the entry's bytes
 * from clt_id (entry + 24) read as a proxy message (proxy.h: header
 * {u16 connection_id, u8 action} -> 4 B; proxy_send_msg's data at +8, so
 * cmd.len = the u16 at entry + 32); bytes of the record, 0 = none */
static inline uint32_t rec_bytes(const uint8_t *e)
{
    const uint8_t action = e[26];
    if (action == 4 || action == 6) return APUS_REC_CONNECT_BYTES;          /* CONNECT, CLOSE */
    if (action == 5) return APUS_REC_SEND_BYTES + (uint32_t)(e[32] | (e[33] << 8));   /* SEND */
    return 0;
}

/* persist_new_entries' walk (dare_server.c:1792-1810) from *cursor, each
 * record appended to the dump (store_record, db-interface.c:65-95: DB_APPEND,
 * records_len += size) */
int apus_oracle_records_store_one(const uint8_t *ring, const apus_group_state_t *st, uint64_t *cursor,
                                  uint8_t *dump, uint64_t cap, uint32_t *dump_len, uint32_t *n_rec)
{
    const uint64_t end = st->end, len = st->len;
    uint64_t oe = *cursor, dl = *dump_len;
    uint32_t n = 0;
    int corrupt = 0;
    if (!(len >= APUS_ENTRY_HDR && end <= len && oe <= len)) {
        *n_rec = 0;
        return 1;
    }
    const uint64_t guard = step_guard(len);
    uint64_t steps = 0;
    while (larger_(end, len, end, oe)) {
        if (++steps > guard) { corrupt = 1; break; }
        if (len - oe < APUS_ENTRY_HDR) oe = 0;                            /* log_get_entry */
        const uint8_t *e = ring + oe;
        if (len - oe < ent_len(e)) { oe = 0; continue; }                  /* ghost header */
        const uint32_t nb = rec_bytes(e);
        if (nb) {
            /* bytes past the log or the dump: the reference reads past its log */
            if (24u + (uint64_t)nb > len - oe || dl + nb > cap) { corrupt = 1; break; }
            memcpy(dump + dl, e + 24, nb);
            dl += nb;
            n++;
        }
        oe += ent_len(e);
    }
    *cursor = oe;
    *dump_len = (uint32_t)dl;
    *n_rec = n;
    return corrupt;
}

void apus_oracle_records_store_batch(const apus_batch_t *b, const apus_records_io_t *io, uint64_t *corrupt)
{
    uint64_t bad = 0;
    for (uint64_t g = 0; g < b->n_groups; g++) {
        uint32_t n = 0;
        bad += (uint64_t)apus_oracle_records_store_one(b->ring + g * b->ring_stride, &b->state[g], &io->cursor[g],
                                                       io->dump + g * io->cap, io->cap, &io->dump_len[g], &n);
        if (io->n_records) io->n_records[g] = n;
    }
    if (corrupt) *corrupt = bad;
}

/* stablestorage_load_records, src/proxy/proxy.c:306-336 */
void apus_oracle_records_load_batch(const apus_records_load_io_t *io)
{
    for (uint64_t k = 0; k < io->n; k++) {
        const uint8_t *d = io->dump + k * io->stride;
        const uint32_t size = io->size[k] < io->stride ? io->size[k] : (uint32_t)io->stride;   /* apus_gpu.h */
        uint32_t len = 0, n = 0, c[3] = { 0, 0, 0 }, status = 0;
        while (len < size) {
            if (size - len < APUS_REC_CONNECT_BYTES) { status = 2; break; }      /* header past size */
            const uint8_t action = d[len + 2];
            uint32_t rb, dl = 0;
            if (action == 5) {                                                  /* SEND */
                if (size - len < APUS_REC_DATA_OFF + 2) { status = 2; break; }
                dl = (uint32_t)(d[len + 8] | (d[len + 9] << 8));
                rb = APUS_REC_SEND_BYTES + dl;                                  /* PROXY_SEND_MSG_SIZE */
            } else if (action == 4 || action == 6) {                            /* CONNECT, CLOSE */
                rb = APUS_REC_CONNECT_BYTES;
            } else {
                status = 1;                                                     /* the reference spins */
                break;
            }
            if (rb > size - len) { status = 2; break; }
            if (io->plan && n < io->max_plan) {
                apus_record_ref_t *r = &io->plan[k * io->max_plan + n];
                memset(r, 0, sizeof *r);
                r->offset = len;
                r->data_len = dl;
                r->connection_id = (uint16_t)(d[len] | (d[len + 1] << 8));
                r->action = action;
            }
            n++;
            c[action - 4]++;
            len += rb;
        }
        io->n_records[k] = n;
        io->status[k] = status;
        if (io->stop) io->stop[k] = len;
        if (io->counts) {
            io->counts[3 * k] = c[0];
            io->counts[3 * k + 1] = c[1];
            io->counts[3 * k + 2] = c[2];
        }
    }
}

/* ================================================================== */
/* Synthetic trace generator (specification for the device generator) */
/* ================================================================== */
static inline uint64_t sm64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static inline uint64_t draw(uint64_t gkey, uint64_t k) { return sm64(gkey ^ (k * 0xD1B54A32D192ED03ull)); }

#define K_G(f)        (0x100ull + (f))
#define K_R(r, f)     (0x1000ull + (uint64_t)(r) * 64 + (f))
#define K_E(e, f)     (0x100000ull + (uint64_t)(e) * 16 + (f))
#define K_RG(e, r)    (0x10000000ull + (uint64_t)(e) * 16 + (r))
#define K_FILL(w)     ((1ull << 40) + (w))

#define GEN_MAX_ENTRIES 256

/* Where log_append_entry (dare_log.h:466-558) puts an entry of elen bytes
 * when the log ends at `end`: at 0 if the header does not fit, else at end;
 * a CSM-class entry whose command does not fit leaves a ghost header at end
 * and is rewritten at 0.  (Bare headers always fit once the header fits.)
 * *ghost = UINT64_MAX when no ghost header is written. */
static inline uint64_t place_entry(uint64_t len, uint64_t end, uint64_t elen, uint64_t *ghost)
{
    uint64_t o = end;
    *ghost = UINT64_MAX;
    if (end == len || len - o < APUS_ENTRY_HDR) o = 0;
    if (len - o < elen) { *ghost = o; o = 0; }
    return o;
}

int apus_oracle_place_seq(uint64_t len, uint64_t start, uint32_t n, const uint32_t *elen,
                          uint64_t *off, uint64_t *ghost, uint64_t *end_out)
{
    uint64_t end = start;
    for (uint32_t k = 0; k < n; k++) {
        off[k] = place_entry(len, end, elen[k], &ghost[k]);
        end = off[k] + elen[k];
    }
    *end_out = end;
    return 0;
}


int apus_oracle_gen_check(const apus_batch_t *b, const apus_gen_cfg_t *c)
{
    uint64_t n = (uint64_t)c->n_entries + c->n_history;
    if (n == 0 || n > GEN_MAX_ENTRIES) return 1;
    if (b->n_replicas < 2 || b->n_replicas > APUS_MAX_SERVER_COUNT) return 1;
    if (c->len_min > c->len_max || c->len_max > 65535) return 1;
    if (c->hist_len_max && (c->hist_len_max < c->len_min || c->hist_len_max > c->len_max)) return 1;
    if (b->ring_stride % 16 || c->ring_len > b->ring_stride || c->ring_len < 256) return 1;
    /* the placed entries plus one wrap gap must not reach the head */
    uint64_t hmax = c->hist_len_max ? c->hist_len_max : c->len_max;
    uint64_t worst = (uint64_t)c->n_history * (APUS_ENTRY_HDR + hmax) +
                     (uint64_t)c->n_entries * (APUS_ENTRY_HDR + (uint64_t)c->len_max) + APUS_ENTRY_HDR + c->len_max + 8;
    if (worst >= c->ring_len) return 1;
    return 0;
}

typedef struct {
    uint8_t  self, size0, size1, state;
    uint32_t bitmask;
    uint64_t epoch, term, idx_base, h0;
} gen_group_t;

static void gen_group_params(const apus_batch_t *b, const apus_gen_cfg_t *c, uint64_t gkey,
                             gen_group_t *p)
{
    uint32_t R = b->n_replicas;
    p->size0 = (uint8_t)R; p->size1 = 0; p->state = APUS_CID_STABLE;
    if (c->cid_mix) {
        uint64_t u = draw(gkey, K_G(4)) % 100;
        if (u >= 60 && u < 80) { p->state = APUS_CID_EXTENDED; p->size0 = (uint8_t)(R - 1); p->size1 = (uint8_t)R; }
        else if (u >= 80) {
            p->state = APUS_CID_TRANSIT;
            if (draw(gkey, K_G(5)) & 1) { p->size0 = (uint8_t)(R - 2); p->size1 = (uint8_t)R; }
            else { p->size0 = (uint8_t)R; p->size1 = (uint8_t)(R - 2); }
        }
    }
    p->self = c->self_random ? (uint8_t)(draw(gkey, K_G(1)) % p->size0) : 0;
    p->term = 1 + draw(gkey, K_G(2)) % 8;
    p->idx_base = 1 + draw(gkey, K_G(3)) % 1000000;
    p->epoch = draw(gkey, K_G(6)) % 4;
    p->bitmask = (R >= 32) ? 0xFFFFFFFFu : ((1u << R) - 1u);
    if (draw(gkey, K_G(7)) % 8 == 0) {
        uint32_t off = (p->self + 1 + (uint32_t)(draw(gkey, K_G(8)) % (R - 1))) % R;
        p->bitmask &= ~(1u << off);
    }
    p->h0 = (draw(gkey, K_G(0)) % c->ring_len) & ~7ull;
}

static inline uint8_t gen_type(const apus_gen_cfg_t *c, uint64_t gkey, uint32_t e)
{
    if (!c->type_mix) return 5;
    switch (draw(gkey, K_E(e, 0)) % 16) {
    case 0: return APUS_NOOP;
    case 1: return APUS_CONFIG;
    case 2: return APUS_HEAD;
    case 3: return 4;
    case 4: return 6;
    default: return 5;
    }
}

void apus_oracle_gen_batch(const apus_batch_t *b, const apus_gen_cfg_t *c,
                           uint64_t g0, uint64_t g1, int threads)
{
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
#endif
    for (int64_t gi = (int64_t)g0; gi < (int64_t)g1; gi++) {
        uint64_t g = (uint64_t)gi;
        uint32_t R = b->n_replicas, H = c->n_history, E = c->n_entries, N = H + E;
        uint64_t gkey = sm64(c->seed ^ sm64(c->gid_base + g));
        uint8_t *ring = b->ring + g * b->ring_stride;
        uint64_t len = c->ring_len;
        gen_group_t p;
        gen_group_params(b, c, gkey, &p);

        /* 1. fill: every ring byte (payload source and stale bytes) */
        for (uint64_t w = 0; w < b->ring_stride / 8; w++) wr64(ring + 8 * w, draw(gkey, K_FILL(w)));

        /* 2. placement, restating log_append_entry, dare_log.h:466-558 */
        uint64_t off[GEN_MAX_ENTRIES], after[GEN_MAX_ENTRIES];
        uint64_t end = p.h0;
        apus_cid_t cid = { p.epoch, { p.size0, p.size1 }, p.state, { 0 }, p.bitmask };
        uint32_t kr[APUS_MAX_SERVER_COUNT];
        uint32_t rs = (p.self + 1 + (uint32_t)(draw(gkey, K_G(10)) % (R - 1))) % R;
        for (uint32_t r = 0; r < R; r++) {
            kr[r] = (draw(gkey, K_R(r, 0)) % 65536 < c->p_full_ack || E == 0)
                        ? E : (uint32_t)(draw(gkey, K_R(r, 1)) % E);
            if (c->straggler && r == rs) kr[r] = (uint32_t)(draw(gkey, K_R(r, 2)) % (E / 4 + 1));
        }
        for (uint32_t e = 0; e < N; e++) {
            uint8_t t = gen_type(c, gkey, e);
            uint16_t clen = 0;
            int csm = !(t == APUS_NOOP || t == APUS_CONFIG || t == APUS_HEAD);
            uint32_t lmax = (e < H && c->hist_len_max) ? c->hist_len_max : c->len_max;
            if (csm) clen = (uint16_t)(c->len_min + draw(gkey, K_E(e, 1)) % (lmax - c->len_min + 1));
            uint64_t elen = APUS_ENTRY_HDR + (csm ? clen : 0);
            uint64_t idx = p.idx_base + e;
            uint64_t term = (e < H / 2 && p.term > 1) ? p.term - 1 : p.term;
            uint64_t req = draw(gkey, K_E(e, 2));
            uint16_t clt = (uint16_t)draw(gkey, K_E(e, 3));
            uint64_t ghost;
            uint64_t o = place_entry(len, end, elen, &ghost);
            if (ghost != UINT64_MAX) {                     /* ghost header        */
                uint8_t *gh = ring + ghost;
                wr64(gh + E_IDX, idx); wr64(gh + E_TERM, term); wr64(gh + E_REQ, req);
                wr16(gh + E_CLT, clt); gh[E_TYPE] = t;
                memset(gh + E_REPLY, 0, APUS_MAX_SERVER_COUNT);
                wr16(gh + E_DATA, clen);
            }
            uint8_t *en = ring + o;
            wr64(en + E_IDX, idx); wr64(en + E_TERM, term); wr64(en + E_REQ, req);
            wr16(en + E_CLT, clt); en[E_TYPE] = t;
            en[E_SNDR] = p.self;                           /* persist_new_entries */
            for (uint32_t r = 0; r < APUS_MAX_SERVER_COUNT; r++) {
                uint8_t rb = 0;
                if (r < R && r != p.self) {
                    if (e < H) rb = 1;
                    else if (e - H < kr[r])
                        rb = (draw(gkey, K_RG(e, r)) % 65536 < c->garbage_reply) ? 2 : 1;
                }
                en[E_REPLY + r] = rb;
            }
            if (t == APUS_CONFIG) memcpy(en + E_DATA, &cid, 16);
            else if (t == APUS_HEAD) wr64(en + E_DATA, p.h0);
            else if (csm) wr16(en + E_DATA, clen);
            off[e] = o;
            end = o + elen;
            after[e] = end;
        }

        /* 3. group state */
        apus_group_state_t *st = &b->state[g];
        uint64_t commit = H ? after[H - 1] : p.h0;
        uint32_t a = (uint32_t)(draw(gkey, K_G(9)) % (H + 1));
        st->head = p.h0;
        st->apply = a ? after[a - 1] : p.h0;
        st->commit = commit;
        st->end = end;
        st->tail = off[N - 1];
        st->len = len;
        st->cid = cid;
        b->self_idx[g] = p.self;

        /* 4. per-replica control data */
        for (uint32_t r = 0; r < R; r++) {
            uint64_t gr = g * R + r;
            if (b->remote_end)
                b->remote_end[gr] = (r == p.self) ? end : (kr[r] ? after[H + kr[r] - 1] : commit);
            if (b->remote_commit) b->remote_commit[gr] = commit;
            if (b->lr_step)
                b->lr_step[gr] = (draw(gkey, K_R(r, 3)) % 16 == 0)
                                     ? (uint8_t)(1 + draw(gkey, K_R(r, 4)) % 6) : APUS_LR_UPDATE_LOG;
            if (b->fail_count)
                b->fail_count[gr] = (draw(gkey, K_R(r, 5)) % 32 == 0) ? APUS_PERMANENT_FAILURE : 0;
            if (b->vote_ack) {
                uint64_t va = len;
                if (r != p.self && draw(gkey, K_R(r, 6)) % 65536 < c->p_vote_ack) {
                    uint32_t j = (uint32_t)(draw(gkey, K_R(r, 7)) % (N + 1));
                    va = j ? after[j - 1] : p.h0;
                }
                b->vote_ack[gr] = va;
            }
            if (b->apply_offsets) {
                uint32_t j = (uint32_t)(draw(gkey, K_R(r, 8)) % (H + 1));
                b->apply_offsets[gr] = j ? after[j - 1] : p.h0;
            }
            if (b->hb)
                b->hb[gr] = (draw(gkey, K_R(r, 9)) % 8 == 0)
                    ? (((p.term + draw(gkey, K_R(r, 10)) % 2) << 9) | (1ull << 8) | r) : 0;
            if (b->vote_req) {
                apus_vote_req_t *q = &b->vote_req[gr];
                memset(q, 0, sizeof *q);
                if (r != p.self && (draw(gkey, K_R(r, 11)) & 1)) {
                    uint64_t last_idx = p.idx_base + N - 1;
                    uint64_t last_term = p.term;
                    q->sid = ((p.term + draw(gkey, K_R(r, 12)) % 3) << 9) |
                             ((uint64_t)(draw(gkey, K_R(r, 13)) % 8 == 0) << 8) | r;
                    int64_t di = (int64_t)(draw(gkey, K_R(r, 14)) % 5) - 2;
                    int64_t dt = (int64_t)(draw(gkey, K_R(r, 15)) % 3) - 1;
                    q->index = (uint64_t)((int64_t)last_idx + di);
                    q->term = (uint64_t)((int64_t)last_term + dt);
                    q->cid = cid;
                    q->cid.epoch = draw(gkey, K_R(r, 16)) % 8;
                }
            }
        }
        if (b->sid) {
            uint64_t L = draw(gkey, K_G(11)) % 4 == 0;
            uint64_t sidx = draw(gkey, K_G(12)) % R;
            b->sid[g] = (p.term << 9) | (L << 8) | sidx;
        }
        if (b->last_idx_term) {   /* end == len reads as an empty log: (0, 0) */
            b->last_idx_term[2 * g] = end == len ? 0 : p.idx_base + N - 1;
            b->last_idx_term[2 * g + 1] = end == len ? 0 : p.term;
        }
        if (b->prev_head) b->prev_head[g] = draw(gkey, K_G(13)) % 4 == 0;
        if (b->abs_base) b->abs_base[g] = (draw(gkey, K_G(14)) % 1000) * len;
    }
}

/* follower NC buffers for (idx, term) validation (config C3): follower r's
 * buffer is the leader's determinant list truncated to n_r entries, with
 * the term of every entry from m_r on bumped by one (divergent suffix). */
void apus_oracle_gen_nc(const apus_batch_t *b, const apus_gen_cfg_t *c,
                        const apus_nc_batch_t *nc, uint64_t g0, uint64_t g1)
{
    uint32_t F = nc->n_followers, M = nc->max_dets;
    apus_entry_det_t *tmp = (apus_entry_det_t *)malloc(sizeof(apus_entry_det_t) * (M ? M : 1));
    for (uint64_t g = g0; g < g1; g++) {
        uint64_t gkey = sm64(c->seed ^ sm64(c->gid_base + g));
        const uint8_t *ring = b->ring + g * b->ring_stride;
        uint32_t n = apus_oracle_nc_build(ring, &b->state[g], tmp, M);
        uint8_t self = b->self_idx[g];
        for (uint32_t f = 0; f < F; f++) {
            uint32_t r = (self + 1 + f) % b->n_replicas;
            uint32_t m = (uint32_t)(draw(gkey, K_R(r, 17)) % (n + 1));
            uint32_t k = m + (uint32_t)(draw(gkey, K_R(r, 18)) % (n - m + 1));
            uint64_t base = (g * F + f) * (uint64_t)M;
            for (uint32_t i = 0; i < k; i++) {
                nc->dets[base + i] = tmp[i];
                if (i >= m) nc->dets[base + i].term += 1;
            }
            nc->det_len[g * F + f] = k;
            nc->follower[g * F + f] = (uint8_t)r;
        }
    }
    free(tmp);
}

/* ================================================================== */
/* batch drivers                                                       */
/* ================================================================== */
void apus_oracle_commit_batch(const apus_batch_t *b, const apus_commit_out_t *out,
                              uint32_t flags, uint64_t g0, uint64_t g1, int threads)
{
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
#endif
    for (int64_t gi = (int64_t)g0; gi < (int64_t)g1; gi++) {
        uint64_t g = (uint64_t)gi;
        const uint8_t *ring = b->ring + g * b->ring_stride;
        const apus_group_state_t *st = &b->state[g];
        uint8_t self = b->self_idx[g];
        if (flags & APUS_COMMIT_WALK) {
            int adv, bad;
            uint32_t n;
            uint64_t c = apus_oracle_commit_walk(ring, st, self, &adv, &n, &bad);
            if (out->new_commit) out->new_commit[g] = c;
            if (out->committed) out->committed[g] = bad ? 0xFF : (uint8_t)adv;
            if (out->n_entries) out->n_entries[g] = n;
        }
        if ((flags & APUS_COMMIT_CHECKSUM) && out->digest)
            out->digest[g] = apus_oracle_checksum(ring, st);
        if ((flags & APUS_COMMIT_MEDIAN) && out->median) {
            uint64_t R = b->n_replicas;
            out->median[g] = apus_oracle_median(st, self, b->remote_end + g * R,
                                                b->lr_step + g * R, b->fail_count + g * R);
        }
    }
}

void apus_oracle_vote_batch(const apus_batch_t *b, const apus_vote_out_t *out,
                            uint64_t g0, uint64_t g1)
{
    for (uint64_t g = g0; g < g1; g++) {
        uint8_t vc[2];
        uint64_t c;
        uint16_t m;
        int won = apus_oracle_vote_tally(&b->state[g], b->self_idx[g],
                                         b->vote_ack + g * b->n_replicas, vc, &c, &m);
        if (out->won) out->won[g] = (uint8_t)won;
        if (out->vote_count) { out->vote_count[2 * g] = vc[0]; out->vote_count[2 * g + 1] = vc[1]; }
        if (out->new_commit) out->new_commit[g] = c;
        if (out->voters) out->voters[g] = m;
    }
}

void apus_oracle_rank_batch(const apus_batch_t *b, const apus_rank_out_t *out,
                            uint64_t g0, uint64_t g1)
{
    uint32_t R = b->n_replicas;
    for (uint64_t g = g0; g < g1; g++) {
        uint64_t lit[2];
        if (b->last_idx_term) { lit[0] = b->last_idx_term[2 * g]; lit[1] = b->last_idx_term[2 * g + 1]; }
        else apus_oracle_last_idx_term(b->ring + g * b->ring_stride, &b->state[g], lit);
        uint64_t ns;
        apus_cid_t nc;
        uint16_t clr;
        uint8_t oc = apus_oracle_vote_rank(&b->state[g], b->self_idx[g], b->sid[g],
                                           b->hb + g * R, R, b->vote_req + g * R,
                                           lit[0], lit[1], &ns, &nc, &clr);
        if (out->outcome) out->outcome[g] = oc;
        if (out->new_sid) out->new_sid[g] = ns;
        if (out->new_cid) out->new_cid[g] = nc;
        if (out->cleared) out->cleared[g] = clr;
    }
}

void apus_oracle_prune_batch(const apus_batch_t *b, const apus_prune_out_t *out,
                             uint64_t g0, uint64_t g1, uint64_t *watermark)
{
    uint32_t R = b->n_replicas;
    uint64_t wm = UINT64_MAX;
    for (uint64_t g = g0; g < g1; g++) {
        uint64_t nh;
        int ap;
        uint64_t m = apus_oracle_min_apply(b->ring + g * b->ring_stride, &b->state[g],
                                           b->apply_offsets + g * R,
                                           b->prev_head ? b->prev_head[g] : 0, &nh, &ap);
        if (out->new_head) out->new_head[g] = nh;
        if (out->append_head) out->append_head[g] = (uint8_t)ap;
        if (out->min_apply) out->min_apply[g] = m;
        if (b->abs_base) { uint64_t w = b->abs_base[g] + nh; if (w < wm) wm = w; }
    }
    if (watermark) *watermark = wm;
}

void apus_oracle_tail_batch(const apus_batch_t *b, const apus_commit_out_t *out, uint32_t flags,
                            const uint64_t *commit, uint64_t g0, uint64_t g1, uint64_t *watermark,
                            uint64_t *corrupt)
{
    const uint32_t R = b->n_replicas;
    uint64_t wm = UINT64_MAX, bad = 0;
    for (uint64_t g = g0; g < g1; g++) {
        apus_group_state_t *st = &b->state[g];
        const uint8_t self = b->self_idx[g];
        const uint64_t c = commit ? commit[g] : st->commit;
        if (flags & APUS_COMMIT_PUBLISH) {
            uint16_t conn = b->rc_connected ? b->rc_connected[g] : 0xFFFFu;
            uint16_t m = apus_oracle_publish(st, self, R, c, b->remote_end + g * R, b->remote_commit + g * R,
                                             b->lr_step + g * R, b->fail_count + g * R, conn);
            if (out->publish) out->publish[g] = m;
            if (out->ssn && m) out->ssn[g] += 1;
        }
        if (flags & APUS_COMMIT_FORCE_PRUNE) {
            /* the log as the commit call leaves it: commit = the walk's */
            apus_group_state_t cur = *st;
            cur.commit = c;
            uint8_t ph = b->prev_head ? b->prev_head[g] : 0, tg;
            uint64_t rq = out->force.req_id ? out->force.req_id[g] : 0;
            uint16_t cl = out->force.clt_id ? out->force.clt_id[g] : 0;
            uint64_t nh, mn, ci;
            int app, bd;
            int a = apus_oracle_force_prune(b->ring + g * b->ring_stride, b->ring_stride, &cur, self, R, b->sid[g],
                                            b->apply_offsets + g * R, &ph, &rq, &cl, &nh, &app, &mn, &tg, &ci, &bd);
            st->end = cur.end;
            st->tail = cur.tail;
            st->cid = cur.cid;
            if (b->prev_head) b->prev_head[g] = ph;
            if (out->force.req_id) out->force.req_id[g] = rq;
            if (out->force.clt_id) out->force.clt_id[g] = cl;
            if (out->force.action) out->force.action[g] = (uint8_t)a;
            if (out->force.target) out->force.target[g] = tg;
            if (out->force.cfg_idx) out->force.cfg_idx[g] = ci;
            if (out->new_head) out->new_head[g] = nh;
            if (out->append_head) out->append_head[g] = (uint8_t)app;
            if (out->min_apply) out->min_apply[g] = mn;
            if (b->abs_base) { uint64_t w = b->abs_base[g] + nh; if (w < wm) wm = w; }
            bad += (uint64_t)bd;
        }
    }
    if (watermark) *watermark = wm;
    if (corrupt) *corrupt = bad;
}

void apus_oracle_validate_batch(const apus_batch_t *b, const apus_nc_batch_t *nc,
                                uint64_t *remote_end_out, uint64_t g0, uint64_t g1)
{
    uint32_t F = nc->n_followers;
    for (uint64_t g = g0; g < g1; g++) {
        for (uint32_t f = 0; f < F; f++) {
            uint64_t gf = g * F + f, o;
            uint32_t n = nc->det_len[gf];
            /* build-defined: a length above the row reads max_dets entries */
            if (n > nc->max_dets) n = nc->max_dets;
            if (n == 0) {                       /* dare_ibv_rc.c:1378-1384 */
                uint8_t fol = nc->follower[gf];
                remote_end_out[gf] = fol < b->n_replicas ? b->remote_commit[g * b->n_replicas + fol] : 0;
                continue;
            }
            apus_oracle_find_remote_end(b->ring + g * b->ring_stride, &b->state[g],
                                        nc->dets + gf * nc->max_dets, n, &o);
            remote_end_out[gf] = o;
        }
    }
}

void apus_oracle_nc_build_batch(const apus_batch_t *b, apus_entry_det_t *dets,
                                uint32_t max_dets, uint32_t *len, uint64_t g0, uint64_t g1)
{
    for (uint64_t g = g0; g < g1; g++)
        len[g] = apus_oracle_nc_build(b->ring + g * b->ring_stride, &b->state[g],
                                      dets + g * max_dets, max_dets);
}

double apus_oracle_time_commit(const apus_batch_t *b, const apus_commit_out_t *out,
                               uint32_t flags, int reps, int threads)
{
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; r++) apus_oracle_commit_batch(b, out, flags, 0, b->n_groups, threads);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

static double secs(const struct timespec *a, const struct timespec *b)
{
    return (double)(b->tv_sec - a->tv_sec) + 1e-9 * (double)(b->tv_nsec - a->tv_nsec);
}

double apus_oracle_time_step(const apus_batch_t *b, const apus_commit_out_t *out,
                             const apus_prune_out_t *pout, uint32_t flags, int reps, int threads)
{
    return apus_oracle_time_step_full(b, out, pout, NULL, NULL, NULL, NULL, flags, reps, threads);
}

/* The CPU baseline of bench.py's whole GPU step: per rep, the commit walk
 * (+ checksum, + median per flags), update_remote_logs' publish
 * (APUS_COMMIT_PUBLISH: out->new_commit needed) and the pruning minimum or
 * (APUS_COMMIT_FORCE_PRUNE) force_log_pruning, then -- where the
 * GPU step runs them -- the vote tally (vout; dare_server.c:1330-1373), each
 * log's local (idx, term) walk + the vote-request ranking (rout;
 * :1526-1655), and the followers' (idx, term) validation (nc, rend_out;
 * dare_log.h:367-394 with the caller's empty-buffer rule), every leg an
 * OpenMP loop over the groups. */
double apus_oracle_time_step_full(const apus_batch_t *b, const apus_commit_out_t *out,
                                  const apus_prune_out_t *pout, const apus_vote_out_t *vout,
                                  const apus_rank_out_t *rout, const apus_nc_batch_t *nc, uint64_t *rend_out,
                                  uint32_t flags, int reps, int threads)
{
    struct timespec t0, t1;
    const uint32_t R = b->n_replicas;
    const int64_t G = (int64_t)b->n_groups;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; r++) {
        apus_oracle_commit_batch(b, out, flags, 0, b->n_groups, threads);
        uint64_t wm = UINT64_MAX;
        if (flags & APUS_COMMIT_PUBLISH) {
            /* update_remote_logs' publish on the walk's commit (dare_ibv_rc.c:1760-1822) */
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
            for (int64_t gi = 0; gi < G; gi++) {
                const uint64_t g = (uint64_t)gi;
                const uint16_t conn = b->rc_connected ? b->rc_connected[g] : 0xFFFFu;
                const uint16_t m = apus_oracle_publish(&b->state[g], b->self_idx[g], R, out->new_commit[g],
                                                       b->remote_end + g * R, b->remote_commit + g * R,
                                                       b->lr_step + g * R, b->fail_count + g * R, conn);
                if (out->publish) out->publish[g] = m;
            }
        }
        if (flags & APUS_COMMIT_FORCE_PRUNE) {
            /* force_log_pruning (dare_server.c:2069-2122) in place of log_pruning */
#ifdef _OPENMP
#pragma omp parallel for schedule(static) reduction(min : wm)
#endif
            for (int64_t gi = 0; gi < G; gi++) {
                const uint64_t g = (uint64_t)gi;
                apus_group_state_t cur = b->state[g];
                cur.commit = out->new_commit[g];
                uint8_t ph = b->prev_head ? b->prev_head[g] : 0, tg;
                uint64_t rq = 0, nh, mn, ci;
                uint16_t cl = 0;
                int app, bd;
                (void)apus_oracle_force_prune(b->ring + g * b->ring_stride, b->ring_stride, &cur, b->self_idx[g], R,
                                              b->sid[g], b->apply_offsets + g * R, &ph, &rq, &cl, &nh, &app, &mn,
                                              &tg, &ci, &bd);
                b->state[g].end = cur.end;
                b->state[g].tail = cur.tail;
                b->state[g].cid = cur.cid;
                if (b->prev_head) b->prev_head[g] = ph;
                if (pout->new_head) pout->new_head[g] = nh;
                if (pout->append_head) pout->append_head[g] = (uint8_t)app;
                if (pout->min_apply) pout->min_apply[g] = mn;
                if (b->abs_base) { uint64_t w = b->abs_base[g] + nh; if (w < wm) wm = w; }
            }
        } else {
#ifdef _OPENMP
        if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static) reduction(min : wm)
#endif
        for (int64_t gi = 0; gi < G; gi++) {
            const uint64_t g = (uint64_t)gi;
            uint64_t nh;
            int ap;
            uint64_t m = apus_oracle_min_apply(b->ring + g * b->ring_stride, &b->state[g],
                                               b->apply_offsets + g * R,
                                               b->prev_head ? b->prev_head[g] : 0, &nh, &ap);
            if (pout->new_head) pout->new_head[g] = nh;
            if (pout->append_head) pout->append_head[g] = (uint8_t)ap;
            if (pout->min_apply) pout->min_apply[g] = m;
            if (b->abs_base) { uint64_t w = b->abs_base[g] + nh; if (w < wm) wm = w; }
        }
        }
        if (wm == 1) fprintf(stderr, "%s", "");      /* keep the reduction live */
        if (vout) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
            for (int64_t gi = 0; gi < G; gi++) {
                const uint64_t g = (uint64_t)gi;
                uint8_t vc[2];
                uint64_t c;
                uint16_t m;
                int won = apus_oracle_vote_tally(&b->state[g], b->self_idx[g], b->vote_ack + g * R, vc, &c, &m);
                if (vout->won) vout->won[g] = (uint8_t)won;
                if (vout->vote_count) { vout->vote_count[2 * g] = vc[0]; vout->vote_count[2 * g + 1] = vc[1]; }
                if (vout->new_commit) vout->new_commit[g] = c;
                if (vout->voters) vout->voters[g] = m;
            }
        }
        if (rout) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
            for (int64_t gi = 0; gi < G; gi++) {
                const uint64_t g = (uint64_t)gi;
                uint64_t lit[2], ns;
                apus_cid_t ncid;
                uint16_t clr;
                apus_oracle_last_idx_term(b->ring + g * b->ring_stride, &b->state[g], lit);
                uint8_t oc = apus_oracle_vote_rank(&b->state[g], b->self_idx[g], b->sid[g], b->hb + g * R, R,
                                                   b->vote_req + g * R, lit[0], lit[1], &ns, &ncid, &clr);
                if (rout->outcome) rout->outcome[g] = oc;
                if (rout->new_sid) rout->new_sid[g] = ns;
                if (rout->new_cid) rout->new_cid[g] = ncid;
                if (rout->cleared) rout->cleared[g] = clr;
            }
        }
        if (nc && rend_out) {
            const uint32_t F = nc->n_followers;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
            for (int64_t gi = 0; gi < G; gi++) {
                const uint64_t g = (uint64_t)gi;
                for (uint32_t f = 0; f < F; f++) {
                    const uint64_t gf = g * F + f;
                    uint32_t n = nc->det_len[gf];
                    if (n > nc->max_dets) n = nc->max_dets;
                    if (n == 0) {
                        const uint8_t fol = nc->follower[gf];
                        rend_out[gf] = fol < R ? b->remote_commit[g * R + fol] : 0;
                        continue;
                    }
                    uint64_t o;
                    apus_oracle_find_remote_end(b->ring + g * b->ring_stride, &b->state[g],
                                                nc->dets + gf * nc->max_dets, n, &o);
                    rend_out[gf] = o;
                }
            }
        }
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return secs(&t0, &t1);
}

double apus_oracle_time_group(const uint8_t *ring, const apus_group_state_t *st, uint8_t self,
                              const uint64_t *remote_end, const uint8_t *lr_step,
                              const uint8_t *fail_count, uint64_t *apply_offsets, int reps)
{
    struct timespec t0, t1;
    volatile uint64_t sink = 0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; r++) {
        int adv, bad, ap;
        uint32_t n;
        uint64_t nh;
        sink += apus_oracle_commit_walk(ring, st, self, &adv, &n, &bad);
        sink += apus_oracle_median(st, self, remote_end, lr_step, fail_count);
        sink += apus_oracle_min_apply(ring, st, apply_offsets, 0, &nh, &ap);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    (void)sink;
    return secs(&t0, &t1);
}

double apus_oracle_host_read_bw(uint64_t bytes, int threads, int reps)
{
    const uint64_t n = bytes / 8;
    uint64_t *buf = (uint64_t *)malloc(n * 8);
    if (!buf) return 0.0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
#endif
    for (int64_t i = 0; i < (int64_t)n; i++) buf[i] = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    struct timespec t0, t1;
    uint64_t acc = 0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; r++) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static) reduction(+ : acc)
#endif
        for (int64_t i = 0; i < (int64_t)n; i++) acc += buf[i];
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    free(buf);
    if (acc == 42) fprintf(stderr, "%s", "");
    return (double)bytes * reps / secs(&t0, &t1);
}

/* ------------------------------------------------------------------ */
/* 8f.2: poll_config_entries, dare_server.c:2133-2187, with update_cid */
/* :2193-2226 and equal_cid, dare_config.h:48-56                        */
/* ------------------------------------------------------------------ */
static int cid_eq(const apus_cid_t *a, const apus_cid_t *b)
{
    return a->epoch == b->epoch && a->state == b->state && a->size[0] == b->size[0] &&
           a->size[1] == b->size[1] && a->bitmask == b->bitmask;
}
static int cid_on(const apus_cid_t *c, uint32_t i) { return i < 32 && ((c->bitmask >> i) & 1u); }

/* update_cid: 1 when equal (nothing done), else the departures and 0 */
static int update_cid(apus_cid_t *cur, const apus_cid_t *cid, uint16_t *departed)
{
    if (cid_eq(cur, cid)) return 1;
    uint8_t size = cid->size[0] > cid->size[1] ? cid->size[0] : cid->size[1];
    for (uint32_t i = 0; i < size; i++)
        if (!cid_on(cid, i) && cid_on(cur, i) && i < 16) *departed |= (uint16_t)(1u << i);
    *cur = *cid;
    return 0;
}

int apus_oracle_config_scan(const uint8_t *ring, apus_group_state_t *st, uint64_t *cid_offset,
                            uint64_t cid_idx, uint64_t *req_id, uint16_t *clt_id, uint16_t *departed)
{
    view_t v = mkview(ring, st);
    uint64_t head_off = st->head, off = *cid_offset, commit = st->commit;
    uint64_t steps = 0, guard = step_guard(st->len);
    uint16_t dep = 0;
    int corrupt = 0;
    while (vdist(&v, off)) {
        if (++steps > guard) { corrupt = 1; break; }
        const uint8_t *e = get_entry(&v, &off);
        if (!fit_ent(&v, off, e)) { off = 0; continue; }
        if (e[E_TYPE] == APUS_CONFIG) {
            if (rd64(e + E_IDX) > cid_idx) {
                apus_cid_t c;
                memcpy(&c, e + E_DATA, sizeof c);
                if (update_cid(&st->cid, &c, &dep) == 0) {
                    *req_id = rd64(e + E_REQ);
                    *clt_id = rd16(e + E_CLT);
                }
            }
        } else if (e[E_TYPE] == APUS_HEAD) {
            /* only committed HEAD entries (dare_server.c:2164-2170) */
            if (!vlarger(&v, off, commit)) head_off = rd64(e + E_DATA);
        }
        off += ent_len(e);
    }
    if (departed) *departed = dep;
    if (corrupt) return 1;
    *cid_offset = vlarger(&v, off, commit) ? commit : off;
    if (vlarger(&v, head_off, st->head)) st->head = head_off;
    return 0;
}

/* ------------------------------------------------------------------ */
/* 8f.2: apply_committed_entries, dare_server.c:1815-1974               */
/* ------------------------------------------------------------------ */
/* The loop of apply_committed_entries.  prev_head == NULL: the leader's
 * CONFIG re-appends are returned as apus_append_batch input (cfg, at most
 * max_cfg, APUS_EV_CFG_FULL past that); prev_head != NULL: they are appended
 * to the log when they are met (log_append_entry, as the reference appends
 * them; the loop then compares offsets against the new end), counted in
 * *n_cfg.  Returns 1 on a walk past the step guard or an append refused. */
static int apply_core(uint8_t *ring, uint64_t stride, apus_group_state_t *st, uint8_t self, uint64_t sid,
                      uint64_t *req_id, uint16_t *clt_id, uint64_t last_applied[3], uint64_t *last_csm_idx,
                      uint32_t *n_applied, uint16_t *departed, uint8_t *events,
                      apus_append_entry_t *cfg, uint8_t *cfg_payload, uint64_t payload_base,
                      uint32_t max_cfg, uint32_t *n_cfg, uint8_t *prev_head)
{
    view_t v = mkview(ring, st);
    /* IS_LEADER, dare_server.c:46-48 */
    const int leader = ((sid >> 8) & 1u) && (uint8_t)(sid & 0xFF) == self;
    uint64_t steps = 0, guard = step_guard(st->len);
    uint32_t na = 0, nc = 0;
    uint16_t dep = 0;
    uint8_t ev = 0;
    int rc = 0;
    while (vlarger(&v, st->commit, st->apply)) {
        if (++steps > guard) { rc = 1; break; }
        const uint8_t *e = get_entry(&v, &st->apply);          /* cannot be NULL */
        if (!fit_ent(&v, st->apply, e)) { st->apply = 0; continue; }
        const uint8_t t = e[E_TYPE];
        const int csm = !(t == APUS_NOOP || t == APUS_CONFIG || t == APUS_HEAD);
        if (leader && t == APUS_CONFIG) {
            apus_cid_t ec;
            memcpy(&ec, e + E_DATA, sizeof ec);
            uint64_t rq = rd64(e + E_REQ);
            uint16_t cl = rd16(e + E_CLT);
            if (ec.state == APUS_CID_STABLE) {
                if (rq != 0) ev |= APUS_EV_CFG_REPLY;                /* :1862-1875 */
            } else if (!(st->cid.epoch > ec.epoch)) {                /* :1877-1881 */
                if (!prev_head && nc == max_cfg) { ev |= APUS_EV_CFG_FULL; break; }
                if (ec.state == APUS_CID_EXTENDED) {                 /* :1888-1902 */
                    st->cid.state = APUS_CID_TRANSIT;
                    if (rq != 0) { ev |= APUS_EV_JOIN_REPLY; rq = 0; cl = 0; }
                } else if (ec.state == APUS_CID_TRANSIT) {           /* :1903-1931 */
                    st->cid.state = APUS_CID_STABLE;
                    for (uint32_t i = st->cid.size[1]; i < st->cid.size[0]; i++) {
                        if (i == self) {
                            ev |= APUS_EV_SELF_REMOVED;
                            if (i < 32) st->cid.bitmask &= ~(1u << i);
                            continue;
                        }
                        if (!cid_on(&st->cid, i)) continue;
                        st->cid.bitmask &= ~(1u << i);
                        if (i < 16) dep |= (uint16_t)(1u << i);
                    }
                    st->cid.size[0] = st->cid.size[1];
                    st->cid.size[1] = 0;
                }
                *req_id = rq;
                *clt_id = cl;
                /* log_append_entry(..., CONFIG, &data.config.cid), :1935-1937 */
                if (prev_head) {
                    apus_append_entry_t q;
                    memset(&q, 0, sizeof q);
                    q.req_id = rq;
                    q.clt_id = cl;
                    q.type = APUS_CONFIG;
                    uint64_t idx = 0, last = 0;
                    apus_cid_t c = st->cid;
                    if (apus_oracle_append_group(ring, stride, st, prev_head, sid >> 9, &q, 1, (const uint8_t *)&c,
                                                 sizeof c, &idx, &last)) { rc = 1; break; }
                    v = mkview(ring, st);                            /* end moved */
                } else {
                    apus_append_entry_t *r = &cfg[nc];
                    memset(r, 0, sizeof *r);
                    r->req_id = rq;
                    r->clt_id = cl;
                    r->type = APUS_CONFIG;
                    r->data_off = payload_base + 16ull * nc;
                    memcpy(cfg_payload + 16ull * nc, &st->cid, 16);
                }
                nc++;
            }
        } else if (csm) {                                            /* apply_entry, :1939-1965 */
            last_applied[0] = rd64(e + E_IDX);
            last_applied[1] = rd64(e + E_TERM);
            last_applied[2] = st->apply + ent_len(e);
            *last_csm_idx = last_applied[0];
            na++;
        }
        /* (read after an inline append, as the reference reads it: an append
         * into a nearly full ring may overwrite this entry's bytes) */
        st->apply += ent_len(e);
    }
    if (n_applied) *n_applied = na;
    if (departed) *departed = dep;
    if (events) *events = ev;
    *n_cfg = nc;
    return rc;
}

int apus_oracle_apply(const uint8_t *ring, apus_group_state_t *st, uint8_t self, uint64_t sid,
                      uint64_t *req_id, uint16_t *clt_id, uint64_t last_applied[3], uint64_t *last_csm_idx,
                      uint32_t *n_applied, uint16_t *departed, uint8_t *events,
                      apus_append_entry_t *cfg, uint8_t *cfg_payload, uint64_t payload_base,
                      uint32_t max_cfg, uint32_t *n_cfg)
{
    return apply_core((uint8_t *)ring, 0, st, self, sid, req_id, clt_id, last_applied, last_csm_idx, n_applied,
                      departed, events, cfg, cfg_payload, payload_base, max_cfg, n_cfg, NULL);
}

/* ------------------------------------------------------------------ */
/* The election-win transition: the rest of poll_vote_count after the  */
/* tally, dare_server.c:1355-1362 and 1389-1510 (apus_gpu.h            */
/* apus_vote_win_batch): the tally's side effects, the SID's L bit     */
/* (server_update_sid :2288-2297), poll_config_entries, the leader's   */
/* apply_committed_entries with its CONFIG re-appends, the blank entry */
/* (CONFIG / NOOP / EXTENDED->TRANSIT / ->STABLE with the removals,    */
/* log_append_entry) and become_leader's apply_offsets = head.         */
/* ------------------------------------------------------------------ */
static int append_one(uint8_t *ring, uint64_t stride, apus_group_state_t *st, uint8_t *prev_head, uint64_t term,
                      uint8_t type, uint64_t req_id, uint16_t clt_id, uint64_t *idx)
{
    apus_append_entry_t q;
    memset(&q, 0, sizeof q);
    q.req_id = req_id;
    q.clt_id = clt_id;
    q.type = type;
    apus_cid_t c = st->cid;
    uint64_t last = 0, k = 0;
    /* *idx = log_append_entry's return; left as it was when refused */
    const int r = apus_oracle_append_group(ring, stride, st, prev_head, term, &q, 1, (const uint8_t *)&c,
                                           type == APUS_CONFIG ? sizeof c : 0, &k, &last);
    if (!r) *idx = k;
    return r;
}

int apus_oracle_vote_win(uint8_t *ring, uint64_t stride, apus_group_state_t *st, uint8_t self, uint32_t R,
                         uint64_t *sid, const uint64_t *vote_ack, uint64_t *rcommit, uint8_t *step,
                         uint64_t *apply_offsets, uint8_t *prev_head, uint8_t won, uint16_t voters,
                         uint64_t new_commit, uint64_t *cid_offset, uint64_t cid_idx, uint64_t *req_id,
                         uint16_t *clt_id, uint64_t last_applied[3], uint64_t *last_csm_idx,
                         uint64_t *last_write_csm_idx, uint8_t *events, uint16_t *departed, uint32_t *n_applied,
                         uint32_t *n_cfg)
{
    uint64_t s = *sid;
    uint8_t ev = 0;
    uint16_t dep = 0;
    *events = 0;
    *departed = 0;
    *n_applied = 0;
    *n_cfg = 0;
    /* IS_CANDIDATE, dare_server.c:49-51 (polling() :1110-1112) */
    if (!((uint8_t)(s & 0xFF) == self && !((s >> 8) & 1u) && (s >> 9) != 0)) return APUS_WIN_NOT_CANDIDATE;
    /* 1. the tally's side effects, :1355-1362 */
    for (uint32_t i = 0; i < R && i < 16; i++)
        if ((voters >> i) & 1u) { rcommit[i] = vote_ack[i]; step[i] = APUS_LR_GET_NCE_LEN; }
    st->commit = new_commit;
    if (!won) return APUS_WIN_LOST;
    /* 2. SID_SET_L + server_update_sid, :1389-1395 */
    s |= 1ull << 8;
    *sid = s;
    const uint64_t term = s >> 9;
    /* 3. poll_config_entries, :1404 */
    if (apus_oracle_config_scan(ring, st, cid_offset, cid_idx, req_id, clt_id, &dep)) {
        *departed = dep;
        return APUS_WIN_CORRUPT;
    }
    /* 4. apply_committed_entries as the leader, :1409 */
    uint8_t ph = prev_head ? *prev_head : 0, ev4 = 0;
    uint16_t dep4 = 0;
    int bad = apply_core(ring, stride, st, self, s, req_id, clt_id, last_applied, last_csm_idx, n_applied, &dep4,
                         &ev4, NULL, NULL, 0, 0, n_cfg, &ph);
    dep |= dep4;
    ev |= ev4;
    int outcome;
    if (bad) { outcome = APUS_WIN_CORRUPT; goto out; }
    /* 5. the blank entry, :1411-1491 */
    if (st->cid.state == APUS_CID_STABLE) {
        *req_id = 0;
        *clt_id = 0;
        if (append_one(ring, stride, st, &ph, term, APUS_CONFIG, 0, 0, last_write_csm_idx)) {
            outcome = APUS_WIN_CORRUPT;
            goto out;
        }
        outcome = APUS_WIN_CONFIG;
    } else {
        view_t v = mkview(ring, st);
        uint64_t off = *cid_offset, steps = 0, guard = step_guard(st->len);
        const uint8_t *e = NULL;
        while (vdist(&v, off)) {
            if (++steps > guard) { outcome = APUS_WIN_CORRUPT; goto out; }
            e = get_entry(&v, &off);
            if (!fit_ent(&v, off, e)) { off = 0; continue; }
            if (e[E_TYPE] == APUS_CONFIG && rd64(e + E_IDX) > cid_idx) break;
            off += ent_len(e);
        }
        if (vdist(&v, off)) {
            /* an un-applied CONFIG entry past cid_idx: a NOOP, :1441-1448 */
            if (append_one(ring, stride, st, &ph, term, APUS_NOOP, 0, 0, last_write_csm_idx)) {
                outcome = APUS_WIN_CORRUPT;
                goto out;
            }
            outcome = APUS_WIN_NOOP;
        } else if (!e) {
            outcome = APUS_WIN_UNDEFINED;                 /* :1456 reads an uninitialised entry */
        } else {
            if (e[E_DATA + 10] == APUS_CID_EXTENDED) {     /* entry->data.cid.state, :1456-1459 */
                st->cid.state = APUS_CID_TRANSIT;
                outcome = APUS_WIN_TRANSIT;
            } else {                                        /* :1460-1486 */
                st->cid.state = APUS_CID_STABLE;
                for (uint8_t i = (uint8_t)(st->cid.size[0] - 1); i > st->cid.size[1]; i--) {
                    if (i == self) {
                        ev |= APUS_EV_SELF_REMOVED;       /* DIE_AF_COMMIT */
                        if (i < 32) st->cid.bitmask &= ~(1u << i);
                        continue;
                    }
                    if (!cid_on(&st->cid, i)) continue;
                    st->cid.bitmask &= ~(1u << i);
                    if (i < 16) dep |= (uint16_t)(1u << i);
                }
                st->cid.size[0] = st->cid.size[1];
                st->cid.size[1] = 0;
                outcome = APUS_WIN_STABLE;
            }
            if (append_one(ring, stride, st, &ph, term, APUS_CONFIG, *req_id, *clt_id, last_write_csm_idx)) {
                outcome = APUS_WIN_CORRUPT;
                goto out;
            }
        }
    }
    /* 6. become_leader: apply_offsets[i] = head, :1505-1508 */
    {
        const uint8_t esz = ext_group_size(&st->cid);
        for (uint32_t i = 0; i < esz && i < R; i++) apply_offsets[i] = st->head;
    }
out:
    if (prev_head) *prev_head = ph;
    *events = ev;
    *departed = dep;
    return outcome;
}

void apus_oracle_vote_win_batch(const apus_batch_t *b, const apus_win_io_t *io, uint64_t g0, uint64_t g1,
                                uint64_t *corrupt)
{
    const uint32_t R = b->n_replicas;
    uint64_t bad = 0;
    for (uint64_t g = g0; g < g1; g++) {
        uint8_t ev = 0;
        uint16_t dep = 0;
        uint32_t na = 0, nc = 0;
        const int oc = apus_oracle_vote_win(b->ring + g * b->ring_stride, b->ring_stride, &b->state[g], b->self_idx[g],
                                            R, &b->sid[g], b->vote_ack + g * R, b->remote_commit + g * R,
                                            b->lr_step + g * R, b->apply_offsets + g * R,
                                            b->prev_head ? &b->prev_head[g] : NULL, io->won[g], io->voters[g],
                                            io->new_commit[g], &io->cid_offset[g], io->cid_idx[g], &io->req_id[g],
                                            &io->clt_id[g], io->last_applied + 3 * g, &io->last_csm_idx[g],
                                            &io->last_write_csm_idx[g], &ev, &dep, &na, &nc);
        io->outcome[g] = (uint8_t)oc;
        if (io->events) io->events[g] = ev;
        if (io->departed) io->departed[g] = dep;
        if (io->n_applied) io->n_applied[g] = na;
        if (io->n_cfg) io->n_cfg[g] = nc;
        bad += oc == APUS_WIN_CORRUPT;
    }
    if (corrupt) *corrupt = bad;
}

void apus_oracle_config_scan_batch(const apus_batch_t *b, const apus_config_io_t *io,
                                   uint64_t g0, uint64_t g1, uint64_t *corrupt)
{
    uint64_t bad = 0;
    for (uint64_t g = g0; g < g1; g++) {
        uint16_t d = 0;
        bad += (uint64_t)apus_oracle_config_scan(b->ring + g * b->ring_stride, &b->state[g], &io->cid_offset[g],
                                                 io->cid_idx[g], &io->req_id[g], &io->clt_id[g], &d);
        if (io->departed) io->departed[g] = d;
    }
    if (corrupt) *corrupt = bad;
}

void apus_oracle_apply_batch(const apus_batch_t *b, const apus_apply_io_t *io,
                             uint64_t g0, uint64_t g1, uint64_t *corrupt)
{
    uint64_t bad = 0;
    for (uint64_t g = g0; g < g1; g++) {
        uint32_t na = 0, nc = 0;
        uint16_t d = 0;
        uint8_t ev = 0;
        const uint64_t k0 = g * io->max_cfg;
        bad += (uint64_t)apus_oracle_apply(b->ring + g * b->ring_stride, &b->state[g], b->self_idx[g], b->sid[g],
                                           &io->req_id[g], &io->clt_id[g], io->last_applied + 3 * g,
                                           &io->last_csm_idx[g], &na, &d, &ev, io->cfg_entries + k0,
                                           io->cfg_payload + 16 * k0, 16 * k0, io->max_cfg, &nc);
        if (io->n_applied) io->n_applied[g] = na;
        if (io->departed) io->departed[g] = d;
        if (io->events) io->events[g] = ev;
        io->n_cfg[g] = nc;
    }
    if (corrupt) *corrupt = bad;
}

/* ------------------------------------------------------------------ */
/* 8f.2: log replication step machine                                  */
/* ------------------------------------------------------------------ */

/* handle_lr_work_completion, dare_ibv_rc.c:3126-3196, one (g, i) pair */
void apus_oracle_lr_completion(uint8_t wc, uint8_t *step, uint8_t *send_flag, uint8_t *send_count)
{
    if (wc == APUS_WC_NONE || wc == APUS_WC_STALE) return;   /* :3136 wr_id != next_wr_id */
    if (wc == APUS_WC_SUCCESS) {
        if (*step == APUS_LR_UPDATE_LOG) {                     /* :3138-3155 */
            if (*send_count == 0) *send_flag = 1;
            else if (*send_count == 1) { *step = APUS_LR_UPDATE_END; *send_flag = 1; }
            else if (*send_count == 2) (*send_count)--;
        } else if (*step != APUS_LR_UPDATE_END) {              /* :3157-3162 */
            (*step)++;
            *send_flag = 1;
        } else {                                               /* :3163-3168 */
            *step = APUS_LR_UPDATE_LOG;
            *send_flag = 1;
        }
    } else {
        if (*step == APUS_LR_UPDATE_LOG) {                     /* :3171-3183 */
            if (*send_count == 2) *send_count = 0;
            else if (*send_count <= 1) *send_flag = 1;
        } else {                                               /* :3185-3193 */
            *send_flag = 1;
        }
    }
}

/* log_adjustment, dare_ibv_rc.c:1292-1451, one group.  Arrays are the
 * group's [R] rows; dets is [R][max_dets]. */
void apus_oracle_log_adjust(const uint8_t *ring, apus_group_state_t *st, uint8_t self, uint32_t R,
                            const uint8_t *fail_count, uint8_t *step, uint8_t *send_flag, uint16_t rc_conn,
                            const uint64_t *vote_ack, uint64_t *rcommit, uint64_t *rend,
                            const uint64_t *nc_len, const apus_entry_det_t *dets, uint32_t max_dets,
                            uint64_t *ssn, uint8_t *post)
{
    view_t v = { NULL, st->end, st->len };
    uint8_t size = ext_group_size(&st->cid);                  /* :1313 */
    int init = 0;
    for (uint32_t i = 0; i < R; i++) post[i] = APUS_LR_POST_NONE;
    for (uint32_t i = 0; i < size && i < R; i++) {
        if (i == self || !((st->cid.bitmask >> i) & 1u)) continue;          /* :1315-1317 */
        if (fail_count[i] >= APUS_PERMANENT_FAILURE) continue;             /* :1321 */
        if (!send_flag[i]) continue;                                       /* :1325 */
        if (!((rc_conn >> i) & 1u)) continue;                              /* :1331 */
        uint64_t remote_commit = vote_ack[i];                              /* :1335 */
        if (st->len == remote_commit) continue;                            /* :1336 */
        uint8_t s = step[i];
        if (!init && s < APUS_LR_UPDATE_LOG) { (*ssn)++; init = 1; }        /* :1341-1345 */
        uint8_t p;
        switch (s) {
        case APUS_LR_GET_WRITE:                                            /* :1348-1353 */
            rcommit[i] = remote_commit;
            s = APUS_LR_GET_NCE_LEN;
            /* fall through */
        case APUS_LR_GET_NCE_LEN:                                          /* :1354-1379 */
            if (vlarger(&v, remote_commit, st->commit)) st->commit = remote_commit;
            p = APUS_LR_POST_READ_NC_LEN;
            break;
        case APUS_LR_GET_NCE:                                              /* :1380-1405 */
            if (nc_len[i] == 0) {
                rend[i] = rcommit[i];
                step[i] = APUS_LR_UPDATE_LOG;
                continue;
            }
            p = APUS_LR_POST_READ_NC;
            break;
        case APUS_LR_SET_END: {                                            /* :1406-1422 */
            uint64_t n = nc_len[i] < max_dets ? nc_len[i] : max_dets, o;
            if (n == 0) o = rcommit[i];
            else apus_oracle_find_remote_end(ring, st, dets + (uint64_t)i * max_dets, n, &o);
            rend[i] = o;
            p = APUS_LR_POST_WRITE_END;
            break;
        }
        default:
            continue;
        }
        step[i] = s;
        send_flag[i] = 0;                                                  /* :1433 */
        post[i] = p;
    }
}

void apus_oracle_lr_completion_batch(const apus_batch_t *b, const apus_lr_io_t *io, uint64_t g0, uint64_t g1)
{
    uint32_t R = b->n_replicas;
    for (uint64_t k = g0 * R; k < g1 * R; k++)
        apus_oracle_lr_completion(io->wc[k], &b->lr_step[k], &io->send_flag[k], &io->send_count[k]);
}

void apus_oracle_log_adjust_batch(const apus_batch_t *b, const apus_lr_io_t *io, uint64_t g0, uint64_t g1)
{
    uint32_t R = b->n_replicas;
    for (uint64_t g = g0; g < g1; g++)
        apus_oracle_log_adjust(b->ring + g * b->ring_stride, &b->state[g], b->self_idx[g], R,
                               b->fail_count + g * R, b->lr_step + g * R, io->send_flag + g * R,
                               io->rc_connected ? io->rc_connected[g] : 0xFFFFu, b->vote_ack + g * R,
                               b->remote_commit + g * R, b->remote_end + g * R, io->nc_len + g * R,
                               io->nc_dets + g * R * io->max_dets, io->max_dets, &io->ssn[g],
                               io->post + g * R);
}
