/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Built into oracle/_ref/libapusref.so
 * by oracle/Makefile, in this container only (it needs /root/reference).
 *
 * This translation unit includes the REFERENCE's own header
 *   /root/reference/src/include/dare/dare_log.h   (+ dare.h, dare_config.h,
 *   dare_sm.h, dare_kvs_sm.h, debug.h — all standard-C only)
 * so every circular-log primitive used below is the reference code itself:
 * log_offset_end_distance, log_is_offset_larger, log_get_entry,
 * log_fit_entry, log_entry_len, log_get_tail, log_entries_to_nc_buf,
 * log_find_remote_end_offset, log_append_entry, get_group_size,
 * get_extended_group_size, CID_IS_SERVER_ON.
 *
 * dare_ibv_rc.c / dare_server.c need <ev.h> and <infiniband/verbs.h>, which
 * this image does not have, so they are not built (no stand-in headers).
 * Their hot-path loop bodies are restated here on top of the real
 * primitives (cited line by line); this is the "reference-composed" oracle
 * the clean-room restatement in apus_oracle.c is checked against.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "dare_log.h"   /* -I /root/reference/src/include/dare */

/* externs the reference header declares (debug.h:110, dare_log.h:26) */
FILE *log_fp;
int prev_log_entry_head;

static dare_log_t *g_log;
static size_t g_cap;
/* set by the batch checkers: mklog clears the offsets and every nc_buf's len
 * instead of the whole 319,656-B header (equivalent for every reader: an
 * nc_buf is read up to its len) */
static int g_light;

/* one dare_log_t whose len is overridden to the group's ring length; all
 * primitives read log->len (dare_log.h:255-282), so small rings are valid */
static dare_log_t *mklog(const uint8_t *ring, uint64_t ring_len, const uint64_t st[6])
{
    size_t need = sizeof(dare_log_t) + ring_len + 64;
    if (!log_fp) log_fp = fopen("/dev/null", "w");
    if (!log_fp) log_fp = stderr;
    if (need > g_cap) {
        free(g_log);
        g_log = (dare_log_t *)calloc(1, need);
        g_cap = need;
    }
    if (g_light) {
        memset(g_log, 0, offsetof(dare_log_t, nc_buf));
        for (int i = 0; i < MAX_SERVER_COUNT; i++) g_log->nc_buf[i].len = 0;
    } else {
        memset(g_log, 0, sizeof(dare_log_t));
    }
    if (ring) memcpy(g_log->entries, ring, ring_len);
    g_log->head = st[0]; g_log->apply = st[1]; g_log->commit = st[2];
    g_log->end = st[3]; g_log->tail = st[4]; g_log->len = st[5];
    g_log->old_end = st[3];
    return g_log;
}

static server_config_t mkcfg(const uint8_t cid16[16], uint8_t self)
{
    server_config_t c;
    memset(&c, 0, sizeof c);
    memcpy(&c.cid, cid16, 16);
    c.idx = self;
    return c;
}

/* ---- layout probe for tests/test_abi.py ---- */
int ref_layout(uint64_t *out, int n)
{
    uint64_t v[] = {
        sizeof(dare_log_entry_t), offsetof(dare_log_entry_t, idx), offsetof(dare_log_entry_t, term),
        offsetof(dare_log_entry_t, req_id), offsetof(dare_log_entry_t, clt_id),
        offsetof(dare_log_entry_t, type), offsetof(dare_log_entry_t, sender),
        offsetof(dare_log_entry_t, reply), offsetof(dare_log_entry_t, data),
        sizeof(dare_log_entry_det_t), sizeof(dare_nc_buf_t), offsetof(dare_nc_buf_t, entries),
        sizeof(dare_log_t), offsetof(dare_log_t, head), offsetof(dare_log_t, apply),
        offsetof(dare_log_t, commit), offsetof(dare_log_t, end), offsetof(dare_log_t, tail),
        offsetof(dare_log_t, old_end), offsetof(dare_log_t, old_commit), offsetof(dare_log_t, len),
        offsetof(dare_log_t, nc_buf), offsetof(dare_log_t, entries),
        sizeof(dare_cid_t), offsetof(dare_cid_t, epoch), offsetof(dare_cid_t, size),
        offsetof(dare_cid_t, state), offsetof(dare_cid_t, bitmask),
        sizeof(server_config_t), offsetof(server_config_t, cid), offsetof(server_config_t, cid_offset),
        offsetof(server_config_t, cid_idx), offsetof(server_config_t, req_id),
        offsetof(server_config_t, servers), offsetof(server_config_t, clt_id),
        offsetof(server_config_t, idx), offsetof(server_config_t, len),
        sizeof(log_offsets_t), LOG_SIZE, MAX_SERVER_COUNT, MAX_NC_ENTRIES,
    };
    int k = (int)(sizeof v / sizeof v[0]);
    for (int i = 0; i < k && i < n; i++) out[i] = v[i];
    return k;
}

uint64_t ref_dist(const uint64_t st[6], uint64_t o) { return log_offset_end_distance(mklog(NULL, 0, st), o); }
int ref_larger(const uint64_t st[6], uint64_t a, uint64_t b) { return log_is_offset_larger(mklog(NULL, 0, st), a, b); }

/* a3 — restates dare_ibv_rc.c:1725-1758 with the real primitives.  `size`
 * is what the median loop leaves behind (dare_ibv_rc.c:1656): cid.size[1]
 * in CID_TRANSIT (the loop always reaches j = 1), cid.size[0] otherwise. */
static uint64_t walk_on(dare_log_t *log, server_config_t cfg, int *committed_out)
{
    uint8_t size = (CID_TRANSIT == cfg.cid.state) ? cfg.cid.size[1] : cfg.cid.size[0];
    uint8_t i;
    int replies, committed = 0;
    uint64_t mo;
    const uint64_t commit0 = log->commit;
    uint64_t guard = log->len / 64 + 4;                                               /* BUILD-ONLY */
    *committed_out = 0;
    if (log->commit > log->len || log->end > log->len) return log->commit;            /* BUILD-ONLY */
    /* TRANSCRIPTION walk (dare_ibv_rc.c:1725-1758) */
    mo = log->commit;
    while (log_offset_end_distance(log, mo)) {
        if (!guard--) return log->commit;                    /* BUILD-ONLY: the step guard (corrupt ring) */
        dare_log_entry_t *entry = log_get_entry(log, &mo);
        if (!log_fit_entry(log, mo, entry)) {
            mo = 0;
            continue;
        }
        replies = 0;
        for (i = 0; i < size; ++i) {
            if ((i == cfg.idx) || (entry->reply[i] == 1)) {
                replies++;
            }
        }
        if (replies < (size / 2 + 1)) {
            break;
        }
        mo += log_entry_len(entry);
    }
    if (log_is_offset_larger(log, mo, log->commit)) {
        log->commit = mo;
        cfg.cid_offset = log->commit;
        committed = 1;
    }
    /* END TRANSCRIPTION walk */
    /* the result; the log is left as it was (the CPU-baseline leg walks it again) */
    mo = log->commit;
    log->commit = commit0;
    *committed_out = committed;
    return mo;
}

uint64_t ref_commit_walk(const uint8_t *ring, const uint64_t st[6], const uint8_t cid16[16],
                         uint8_t self, int *committed)
{
    return walk_on(mklog(ring, st[5], st), mkcfg(cid16, self), committed);
}

/* a4 — restates dare_ibv_rc.c:1650-1723 (server_t gates passed as arrays) */
static uint64_t median_on(dare_log_t *log, server_config_t cfg, const uint64_t *rend, const uint8_t *step,
                          const uint8_t *fail)
{
    uint64_t offsets[MAX_SERVER_COUNT + 3];
    uint8_t i, size;
    memset(offsets, 0, sizeof offsets);
    /* TRANSCRIPTION median (dare_ibv_rc.c:1652-1723) */
    uint64_t min_offset = log->commit;
    int j = 0;
    while (j < 2) {
        int cnt = 0;
        size = cfg.cid.size[j];
        for (i = 0; i < size; i++) {
            if (i == cfg.idx) {
                offsets[i] = log->end;
                continue;
            }
            if (!CID_IS_SERVER_ON(cfg.cid, i) || (fail[i] >= 2) || (step[i] != 5)) {
                offsets[i] = log->commit;
                continue;
            }
            offsets[i] = rend[i];
            if (log_is_offset_larger(log, offsets[i], min_offset)) {
                cnt++;
            }
        }
        if (cnt < size / 2) {
            if (CID_TRANSIT != cfg.cid.state)
                break;
            if (!j) {
                j++; continue;
            }
            break;
        }
        uint64_t tmp; int k;
        for (i = 1; i < size; i++) {
            tmp = offsets[i];
            k = i;
            while ((k > 0) && (offsets[k - 1] > tmp)) {
                offsets[k] = offsets[k - 1];
                k--;
            }
            offsets[k] = tmp;
        }
        if (CID_TRANSIT != cfg.cid.state) {
            min_offset = offsets[(size - 1) / 2];
            break;
        }
        else {
            uint64_t median = offsets[(size - 1) / 2];
            if (!j) min_offset = median;
            else if (log_is_offset_larger(log, min_offset, median))
                min_offset = offsets[(size - 1) / 2];
        }
        j++;
    }
    /* END TRANSCRIPTION median */
    return min_offset;
}

uint64_t ref_median(const uint64_t st[6], const uint8_t cid16[16], uint8_t self,
                    const uint64_t *rend, const uint8_t *step, const uint8_t *fail)
{
    return median_on(mklog(NULL, 0, st), mkcfg(cid16, self), rend, step, fail);
}

/* a5 — restates dare_server.c:1330-1373 with the real get_group_size; the
 * voters' log_offsets[i].commit / next_lr_step updates land in local columns */
static void vote_on(dare_log_t *log, server_config_t cfg, const uint64_t *vote_ack, uint8_t vc[2], int *won)
{
    uint64_t voted[MAX_SERVER_COUNT];
    uint8_t vstep[MAX_SERVER_COUNT];
    *won = 0;
    /* TRANSCRIPTION vote (dare_server.c:1332-1373) */
    vc[0] = 1;
    vc[1] = 1;
    uint8_t i, size = get_group_size(cfg);
    uint64_t rc;
    for (i = 0; i < size; i++) {
        if (i == cfg.idx) continue;
        rc = vote_ack[i];
        if (log->len == rc) {
            continue;
        }
        if (i < cfg.cid.size[0]) {
            vc[0]++;
        }
        if (i < cfg.cid.size[1]) {
            vc[1]++;
        }
        voted[i] = rc;
        vstep[i] = 2;       /* LR_GET_NCE_LEN */
        if (log_is_offset_larger(log, rc, log->commit)) {
            log->commit = rc;
        }
    }
    if (vc[0] < cfg.cid.size[0] / 2 + 1) {
        return;
    }
    if (CID_STABLE != cfg.cid.state) {
        if (vc[1] < cfg.cid.size[1] / 2 + 1) {
            return;
        }
    }
    /* END TRANSCRIPTION vote */
    (void)voted;
    (void)vstep;
    *won = 1;
}

int ref_vote_tally(const uint64_t st[6], const uint8_t cid16[16], uint8_t self,
                   const uint64_t *vote_ack, uint8_t vc[2], uint64_t *new_commit)
{
    dare_log_t *log = mklog(NULL, 0, st);
    int won;
    vote_on(log, mkcfg(cid16, self), vote_ack, vc, &won);
    *new_commit = log->commit;
    return won;
}

/* The SID macros and the vote request of dare_server.h:52-60,98-104, restated
 * (dare_server.h includes <ev.h>, which this image does not have). */
#define SID_GET_IDX(sid) (uint8_t)((sid) & (0xFF))
#define SID_SET_IDX(sid, idx) (sid) = (idx | ((sid >> 8) << 8))
#define SID_GET_L(sid) ((sid) & (1 << 8))
#define SID_SET_L(sid) (sid) |= 1 << 8
#define SID_GET_TERM(sid) ((sid) >> 9)
#define SID_SET_TERM(sid, term) (sid) = (((term) << 9) | ((sid) & 0x1FF))
typedef struct vote_req_t {
    uint64_t sid;
    uint64_t index;
    uint64_t term;
    dare_cid_t cid;
} vote_req_t;

/* local (idx, term) as poll_vote_requests derives it (dare_server.c:1598-1620),
 * with the real log_entries_to_nc_buf / log_get_tail / log_get_entry */
void ref_last_idx_term(const uint8_t *ring, const uint64_t st[6], uint64_t out[2])
{
    dare_log_t *log = mklog(ring, st[5], st);
    static dare_nc_buf_t nc_store[MAX_SERVER_COUNT];
    const uint8_t self = 0;
    const uint64_t old_sid = 0;
    /* (BUILD-ONLY below: end == len with entries present makes log_get_entry
     * return NULL, which the reference dereferences, dare_server.c:1612-1614;
     * this build reports (0, 0) instead of crashing) */
    /* TRANSCRIPTION rank_local (dare_server.c:1598-1620) */
    vote_req_t best_request;
    best_request.sid = old_sid;
    dare_nc_buf_t *nc_buf = &nc_store[self];
    log_entries_to_nc_buf(log, nc_buf);
    if (0 == nc_buf->len) {
        uint64_t tail = log_get_tail(log);
        if (tail == log->len) {
            best_request.index = 0;
            best_request.term  = 0;
        }
        else {
            dare_log_entry_t* last_entry =
                    log_get_entry(log, &tail);
            if (!last_entry) { best_request.index = 0; best_request.term = 0; goto done; }   /* BUILD-ONLY: NULL */
            best_request.index = last_entry->idx;
            best_request.term  = last_entry->term;
        }
    }
    else {
        best_request.index = nc_buf->entries[nc_buf->len-1].idx;
        best_request.term  = nc_buf->entries[nc_buf->len-1].term;
    }
    /* END TRANSCRIPTION rank_local */
done:
    out[0] = best_request.index;
    out[1] = best_request.term;
}

/* the candidate's ctrl_data fields the ranking reads and writes (sid, hb[],
 * vote_req[]); hb is 256 wide so that hb[possible_leader] reads 0 past the
 * group's columns (the reference reads past ctrl_data there) */
typedef struct rank_ctrl {
    uint64_t sid;
    uint64_t hb[256];
    vote_req_t vote_req[MAX_SERVER_COUNT];
} rank_ctrl;
static __thread uint64_t g_rank_sid;
static __thread uint64_t *g_sid_cell;
/* server_update_sid (dare_server.c:2288-2297) compare-and-swaps ctrl_data->sid;
 * here it records the SID the call would install, and installs it in
 * g_sid_cell (poll_vote_count's data.ctrl_data->sid) when that is set */
static int server_update_sid(uint64_t new_sid, uint64_t old_sid)
{
    g_rank_sid = new_sid;
    if (g_sid_cell) {
        if (*g_sid_cell != old_sid) return 1;
        *g_sid_cell = new_sid;
    }
    return 0;
}

/* a6 — poll_vote_requests (dare_server.c:1526-1655) on the candidate's local
 * (idx, term) (ref_last_idx_term): the outcome (APUS_RANK_*: 0 leader known, 1
 * adopt the heartbeat, 2 no better SID, 3 raise the term, 4 vote), the SID it
 * would install, the adopted cid and which requests it zeroed */
static void rank_on(rank_ctrl *ctrl, server_config_t cfg, uint64_t lidx, uint64_t lterm, int *outcome,
                    uint16_t *clr, uint8_t new_cid[16])
{
    uint8_t i, size = get_group_size(cfg);
    uint64_t new_sid;
    vote_req_t *request;
    int rc;
    /* TRANSCRIPTION rank_best (dare_server.c:1535-1579) */
    if (SID_GET_L(ctrl->sid)) {
        *outcome = 0;   /* BUILD-ONLY */
        return;
    }
    uint8_t possible_leader = SID_GET_IDX(ctrl->sid);
    uint64_t hb = ctrl->hb[possible_leader];
    if ( (0 != hb) && (SID_GET_TERM(hb) == SID_GET_TERM(ctrl->sid)) ) {
        server_update_sid(hb, ctrl->sid);
        *outcome = 1;   /* BUILD-ONLY */
        return;
    }
    uint64_t old_sid = ctrl->sid; SID_SET_L(old_sid);
    uint64_t best_sid = old_sid;
    for (i = 0; i < size; i++) {
        if (i == cfg.idx) continue;
        request = &(ctrl->vote_req[i]);
        if (request->sid != 0) {
        }
        if (best_sid >= request->sid) {
            request->sid = 0;
            *clr |= (uint16_t)(1u << i);   /* BUILD-ONLY */
            continue;
        }
        best_sid = request->sid;
    }
    if (best_sid == old_sid) {
        *outcome = 2;   /* BUILD-ONLY */
        return;
    }
    /* END TRANSCRIPTION rank_best */
    uint64_t highest_term = SID_GET_TERM(best_sid);
    vote_req_t best_request;
    best_request.sid = old_sid;
    best_request.index = lidx;
    best_request.term = lterm;
    /* TRANSCRIPTION rank_uptodate (dare_server.c:1626-1667) */
    for (i = 0; i < size; i++) {
        request = &(ctrl->vote_req[i]);
        if (best_request.sid > request->sid) {
            request->sid = 0;
            *clr |= (uint16_t)(1u << i);   /* BUILD-ONLY */
            continue;
        }
        if (highest_term < SID_GET_TERM(request->sid))
            highest_term = SID_GET_TERM(request->sid);
        if ( (best_request.term > request->term) ||
             ((best_request.term == request->term) &&
              (best_request.index > request->index)) )
        {
            request->sid = 0;
            *clr |= (uint16_t)(1u << i);   /* BUILD-ONLY */
            continue;
        }
        best_request.index = request->index;
        best_request.term = request->term;
        best_request.sid = request->sid;
        best_request.cid = request->cid;
        request->sid = 0;
        *clr |= (uint16_t)(1u << i);   /* BUILD-ONLY */
    }
    if (best_request.sid == old_sid) {
        new_sid = ctrl->sid;
        SID_SET_TERM(new_sid, highest_term);
        SID_SET_IDX(new_sid, cfg.idx);
        rc = server_update_sid(new_sid, ctrl->sid);
        if (0 != rc) {
            return;
        }
        *outcome = 3;   /* BUILD-ONLY */
        return;
    }
    /* END TRANSCRIPTION rank_uptodate */
    /* dare_server.c:1682-1689: vote for the best request, adopt its cid */
    rc = server_update_sid(best_request.sid, ctrl->sid);
    memcpy(new_cid, &best_request.cid, 16);
    *outcome = 4;
}

/* a6 entry: the group's columns (hb[n_hb], req[n_hb][5] = sid, index, term,
 * cid) into a candidate's ctrl_data; slots past n_hb hold no request */
int ref_vote_rank(const uint64_t st[6], const uint8_t cid16[16], uint8_t self, uint64_t sid,
                  const uint64_t *hb, int n_hb, const uint64_t *req /* [n][5]: sid,index,term,cid */,
                  uint64_t lidx, uint64_t lterm, uint64_t *new_sid, uint8_t new_cid[16],
                  uint16_t *cleared)
{
    static rank_ctrl ctrl;
    (void)st;
    memset(&ctrl, 0, sizeof ctrl);
    ctrl.sid = sid;
    for (int i = 0; i < n_hb && i < MAX_SERVER_COUNT; i++) {
        ctrl.hb[i] = hb[i];
        ctrl.vote_req[i].sid = req[5 * i];
        ctrl.vote_req[i].index = req[5 * i + 1];
        ctrl.vote_req[i].term = req[5 * i + 2];
        memcpy(&ctrl.vote_req[i].cid, req + 5 * i + 3, 16);
    }
    int outcome = -1;
    uint16_t clr = 0;
    memset(new_cid, 0, 16);
    g_rank_sid = sid;
    rank_on(&ctrl, mkcfg(cid16, self), lidx, lterm, &outcome, &clr, new_cid);
    *new_sid = g_rank_sid;
    *cleared = clr;
    return outcome;
}

/* a7 — restates dare_server.c:2026-2058 with the real primitives */
static uint64_t min_apply_on(dare_log_t *log, server_config_t cfg, uint64_t *apply_offsets, int prev_head,
                             uint64_t *new_head, int *append)
{
    uint8_t i, size;
    *append = 0;
    /* TRANSCRIPTION prune (dare_server.c:2026-2050) */
    size = get_extended_group_size(cfg);
    uint64_t min_offset = log->apply;
    for (i = 0; i < size; i++) {
        if (!CID_IS_SERVER_ON(cfg.cid, i)) {
            apply_offsets[i] = log->apply;
        }
        if (log_is_offset_larger(log, min_offset,
                    apply_offsets[i]))
            min_offset = apply_offsets[i];
    }
    if (!log_offset_end_distance(log, min_offset)) {
        min_offset = log_get_tail(log);
    }
    if (log_is_offset_larger(log, min_offset, log->head) &&
            !prev_head)
    {
        log->head = min_offset;
    /* END TRANSCRIPTION prune */
        *append = 1;
    }
    *new_head = log->head;
    return min_offset;
}

uint64_t ref_min_apply(const uint8_t *ring, const uint64_t st[6], const uint8_t cid16[16],
                       uint64_t *apply_offsets, int prev_head, uint64_t *new_head, int *append)
{
    return min_apply_on(mklog(ring, st[5], st), mkcfg(cid16, 0), apply_offsets, prev_head, new_head, append);
}

/* CPU-baseline leg: `reps` cache-hot repetitions of walk + median + pruning
 * minimum on one group, on the reference's own primitives (the log image is
 * built once, outside the timed loop); seconds.  apus_oracle_time_group times
 * the same work on the clean-room restatement. */
double ref_time_group(const uint8_t *ring, const uint64_t st[6], const uint8_t cid16[16], uint8_t self,
                      const uint64_t *rend, const uint8_t *step, const uint8_t *fail, uint64_t *apply, int reps)
{
    dare_log_t *log = mklog(ring, st[5], st);
    server_config_t cfg = mkcfg(cid16, self);
    server_config_t cfg0 = mkcfg(cid16, 0);
    struct timespec t0, t1;
    volatile uint64_t sink = 0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; r++) {
        int c, a;
        uint64_t nh;
        sink += walk_on(log, cfg, &c);
        sink += median_on(log, cfg, rend, step, fail);
        sink += min_apply_on(log, cfg0, apply, 0, &nh, &a);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    (void)sink;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* a8 — the real log_find_remote_end_offset */
uint64_t ref_find_remote_end(const uint8_t *ring, const uint64_t st[6],
                             const uint64_t *dets /* [n][3] */, uint64_t n)
{
    dare_log_t *log = mklog(ring, st[5], st);
    static dare_nc_buf_t nc;
    nc.len = n;
    memcpy(nc.entries, dets, n * sizeof(dare_log_entry_det_t));
    return log_find_remote_end_offset(log, &nc);
}

/* a9 — the real log_entries_to_nc_buf; returns len, dets [len][3] */
uint64_t ref_nc_build(const uint8_t *ring, const uint64_t st[6], uint64_t *dets, uint64_t max)
{
    dare_log_t *log = mklog(ring, st[5], st);
    static dare_nc_buf_t nc;
    log_entries_to_nc_buf(log, &nc);
    uint64_t n = nc.len < max ? nc.len : max;
    memcpy(dets, nc.entries, n * sizeof(dare_log_entry_det_t));
    return nc.len;
}

uint64_t ref_get_tail(const uint8_t *ring, const uint64_t st[6])
{
    return log_get_tail(mklog(ring, st[5], st));
}

/* the real log_append_entry on an initially empty log of ring_len bytes.
 * types/clens/terms: n entries; out_ring receives the entries[] image,
 * out_st the final {head, apply, commit, end, tail, len}, out_off the offset
 * of every appended entry's header (log->tail after each append). */
int ref_append_seq(uint64_t ring_len, uint64_t start, int n, const uint8_t *types,
                   const uint16_t *clens, const uint64_t *terms, const uint8_t cid16[16],
                   uint8_t *out_ring, uint64_t out_st[6], uint64_t *out_off)
{
    /* head = len + 7 is never reached by end (<= len), so is_log_full never
     * fires; tail = start with no entry there gives idx 1 without a tail
     * scan (dare_log.h:478-484).  start == len keeps the log empty. */
    uint64_t st[6] = { ring_len + 7, start, start, start, start, ring_len };
    dare_log_t *log = mklog(NULL, ring_len, st);
    static uint8_t cmdbuf[2 + 65536];
    memset(log->entries, 0, ring_len);
    for (int k = 0; k < n; k++) {
        uint64_t h = 7;
        uint16_t l = clens[k];
        memcpy(cmdbuf, &l, 2);
        memset(cmdbuf + 2, 0xA5, l);
        void *data = cmdbuf;
        if (types[k] == CONFIG) data = (void *)cid16;
        else if (types[k] == HEAD) data = &h;
        else if (types[k] == NOOP) data = NULL;
        uint64_t idx = log_append_entry(log, terms[k], 0, 0, types[k], data);
        if (idx == 0) return -1;
        out_off[k] = log->tail;
    }
    memcpy(out_ring, log->entries, ring_len);
    out_st[0] = log->head; out_st[1] = log->apply; out_st[2] = log->commit;
    out_st[3] = log->end; out_st[4] = log->tail; out_st[5] = log->len;
    return 0;
}

/* 8f.1 — the real log_append_entry (dare_log.h:466-558) over one group's
 * queued messages, in order, as get_tailq_message does
 * (dare_ibv_ud.c:780-790).  q holds apus_append_entry_t records (24 B:
 * req_id@0, data_off@8, clt_id@16, type@18).  The messages the batched API
 * stops on (apus_gpu.h: an entry that can never fit, data outside the
 * payload -- undefined in the reference) are pre-checked the same way and
 * end the sequence (return 1).  ring/st/prev_head/last_idx are in/out. */
/* the messages of one group on a log image already holding its ring and
 * offsets (ref_append_group, ref_append_batch) */
static int append_on(dare_log_t *log, uint8_t *prev_head, uint64_t term, const uint8_t *q, uint32_t n,
                     const uint8_t *payload, uint64_t payload_bytes, uint64_t *idx_out, uint64_t *last_idx)
{
    prev_log_entry_head = *prev_head;
    int stopped = 0;
    for (uint32_t k = 0; k < n; k++) {
        const uint8_t *r = q + 24 * (size_t)k;
        uint64_t req_id, doff;
        uint16_t clt_id;
        memcpy(&req_id, r, 8);
        memcpy(&doff, r + 8, 8);
        memcpy(&clt_id, r + 16, 2);
        uint8_t type = r[18];
        int csm = !(type == NOOP || type == CONFIG || type == HEAD);
        uint64_t need = 0, clen = 0;
        if (csm) {
            if (doff > payload_bytes || payload_bytes - doff < 2) { stopped = 1; break; }
            clen = ((const sm_cmd_t *)(payload + doff))->len;
            need = 2 + clen;
        } else if (type == CONFIG) {
            need = sizeof(dare_cid_t);
        } else if (type == HEAD) {
            need = sizeof(uint64_t);
        }
        if (need && (doff > payload_bytes || payload_bytes - doff < need)) { stopped = 1; break; }
        if (csm && sizeof(dare_log_entry_t) + clen > log->len) { stopped = 1; break; }
        uint64_t idx = log_append_entry(log, term, req_id, clt_id, type, (void *)(payload + doff));
        idx_out[k] = idx;
        *last_idx = idx;
    }
    *prev_head = (uint8_t)prev_log_entry_head;
    return stopped;
}

int ref_append_group(uint8_t *ring, uint64_t stride, uint64_t st[6], uint8_t *prev_head, uint64_t term,
                     const uint8_t *q, uint32_t n, const uint8_t *payload, uint64_t payload_bytes,
                     uint64_t *idx_out, uint64_t *last_idx)
{
    for (uint32_t k = 0; k < n; k++) idx_out[k] = 0;
    if (n == 0) return 0;
    if (!(st[5] >= sizeof(dare_log_entry_t) && st[5] <= stride && st[3] <= st[5] && st[4] <= st[5])) return 1;
    dare_log_t *log = mklog(ring, st[5], st);
    const int stopped = append_on(log, prev_head, term, q, n, payload, payload_bytes, idx_out, last_idx);
    memcpy(ring, log->entries, st[5]);
    st[3] = log->end;
    st[4] = log->tail;
    return stopped;
}

/* one image per caller: the header cleared once (neither the append nor the
 * persist walk reads nc_buf), its offsets and ring set per group as mklog sets them */
static void light_log(dare_log_t *log, const uint8_t *ring, const uint64_t st[6])
{
    memcpy(log->entries, ring, st[5]);
    log->head = st[0]; log->apply = st[1]; log->commit = st[2];
    log->end = st[3]; log->tail = st[4]; log->len = st[5];
    log->old_end = st[3]; log->old_commit = 0;
}

/* ref_append_group over every group of a batch, in place (rings [n][stride],
 * state rows [n][64], prev_head [n]; q [n][M] records; term [n] or, NULL,
 * SID_GET_TERM(sid[g]) as the batched API; idx_out [n][M], last_idx [n],
 * stopped [n]).  One thread: log_append_entry runs on the reference's global
 * prev_log_entry_head.  0, or 1 without memory. */
int ref_append_batch(uint64_t n, uint64_t stride, uint8_t *rings, uint8_t *state, uint8_t *prev_head,
                     const uint64_t *term, const uint64_t *sid, const uint8_t *q, uint32_t M, const uint32_t *n_msg,
                     const uint8_t *payload, uint64_t payload_bytes, uint64_t *idx_out, uint64_t *last_idx,
                     uint8_t *stopped)
{
    if (!log_fp) log_fp = fopen("/dev/null", "w");
    dare_log_t *log = (dare_log_t *)calloc(1, sizeof(dare_log_t) + stride + 64);
    if (!log) return 1;
    for (uint64_t g = 0; g < n; g++) {
        uint64_t *st = (uint64_t *)(state + 64 * g);
        uint8_t *ring = rings + g * stride;
        const uint32_t m = n_msg ? (n_msg[g] < M ? n_msg[g] : M) : M;
        uint64_t *io = idx_out + g * M;
        for (uint32_t k = 0; k < M; k++) io[k] = 0;
        stopped[g] = 0;
        if (m == 0) continue;
        if (!(st[5] >= sizeof(dare_log_entry_t) && st[5] <= stride && st[3] <= st[5] && st[4] <= st[5])) {
            stopped[g] = 1;
            continue;
        }
        light_log(log, ring, st);
        const uint64_t t = term ? term[g] : (sid[g] >> 9);
        stopped[g] = (uint8_t)append_on(log, prev_head + g, t, q + 24ull * M * g, m, payload, payload_bytes, io,
                                        last_idx + g);
        memcpy(ring, log->entries, st[5]);
        st[3] = log->end;
        st[4] = log->tail;
    }
    free(log);
    return 0;
}

/* 8f.1 — persist_new_entries (dare_server.c:1792-1810) restated on the real
 * primitives for replica copy i: the leader stamps entry->sender, a
 * follower's rc_send_entries_reply (dare_ibv_rc.c:1828-1863) sets
 * reply[config.idx] of the entry at old_end.  `limit` caps the entries
 * persisted (straggler model); the step guard is the build's (apus_gpu.h). */
/* the walk of replica copy i on a log image holding the group's ring and offsets */
static int persist_on(dare_log_t *log, uint8_t self, uint32_t i, uint64_t *old_end, uint32_t limit)
{
    log->old_end = *old_end;
    uint64_t guard = log->len / 64 + 4, steps = 0;
    uint32_t n = 0;
    int corrupt = 0;
    dare_log_entry_t *entry;
    while (log_is_offset_larger(log, log->end, log->old_end)) {
        if (n >= limit) break;
        if (++steps > guard) { corrupt = 1; break; }
        entry = log_get_entry(log, &log->old_end);
        if (!log_fit_entry(log, log->old_end, entry)) {
            log->old_end = 0;
            continue;
        }
        if (i == self) entry->sender = (uint8_t)i;
        else entry->reply[i] = 1;
        log->old_end += log_entry_len(entry);
        n++;
    }
    *old_end = log->old_end;
    return corrupt;
}

int ref_persist_one(uint8_t *ring, uint64_t stride, const uint64_t st[6], uint8_t self, uint32_t i,
                    uint64_t *old_end, uint32_t limit)
{
    if (!(st[5] >= sizeof(dare_log_entry_t) && st[5] <= stride && st[3] <= st[5] && *old_end <= st[5])) return 1;
    dare_log_t *log = mklog(ring, st[5], st);
    const int corrupt = persist_on(log, self, i, old_end, limit);
    memcpy(ring, log->entries, st[5]);
    return corrupt;
}

/* ref_persist_one for every copy i < R of every group, copies in index order
 * (they write distinct bytes), OpenMP over the groups with a log image per
 * thread; old_end [n][R] in/out, limit [n][R] or NULL; corrupt [n] (the copies
 * that stopped on the step guard or a bad cursor).  0, or 1 without memory. */
int ref_persist_batch(uint64_t n, uint32_t R, uint64_t stride, uint8_t *rings, const uint8_t *state,
                      const uint8_t *self, uint64_t *old_end, const uint32_t *limit, uint32_t *corrupt, int threads)
{
    int bad = 0;
    if (!log_fp) log_fp = fopen("/dev/null", "w");
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel reduction(| : bad)
#endif
    {
        dare_log_t *log = (dare_log_t *)calloc(1, sizeof(dare_log_t) + stride + 64);
        if (!log) bad = 1;
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t g = 0; g < (int64_t)n; g++) {
            if (!log) continue;
            const uint64_t *st = (const uint64_t *)(state + 64 * g);
            uint8_t *ring = rings + g * stride;
            uint32_t c = 0;
            if (!(st[5] >= sizeof(dare_log_entry_t) && st[5] <= stride && st[3] <= st[5])) {
                corrupt[g] = R;
                continue;
            }
            light_log(log, ring, st);
            for (uint32_t i = 0; i < R; i++) {
                uint64_t *oe = old_end + g * R + i;
                if (*oe > st[5]) { c++; continue; }
                c += (uint32_t)persist_on(log, self[g], i, oe, limit ? limit[g * R + i] : 0xFFFFFFFFu);
            }
            memcpy(ring, log->entries, st[5]);
            corrupt[g] = c;
        }
        free(log);
    }
    return bad;
}

/* 8f.3 — the proxy's stable-storage records: persist_new_entries'
 * (dare_server.c:1792-1810) walk on the real primitives, handing every
 * entry's &entry->clt_id to proxy_store_cmd = stablestorage_save_request,
 * restated in ref_records.c on the reference's proxy.h (its sink appends the
 * record to the group's snapshot, `dump` of `cap` bytes holding *dump_len).
 * The walk stops where the record would run past the log or the snapshot
 * (the sink's BUILD-ONLY stop) and on the build's step guard. */
extern void ref_save_request(void *data, void *arg);
extern size_t ref_rec_sink_size(void);
extern void ref_rec_sink_init(void *s, uint8_t *buf, uint64_t cap, uint64_t len);
extern void ref_rec_sink_avail(void *s, uint64_t avail);
extern int ref_rec_sink_stopped(const void *s);
extern uint64_t ref_rec_sink_len(const void *s);
extern uint32_t ref_rec_sink_n(const void *s);

int ref_records_store_one(const uint8_t *ring, const uint64_t st[6], uint64_t *cursor, uint8_t *dump, uint64_t cap,
                          uint32_t *dump_len, uint32_t *n_rec)
{
    if (!(st[5] >= sizeof(dare_log_entry_t) && st[3] <= st[5] && *cursor <= st[5])) {   /* BUILD-ONLY */
        *n_rec = 0;
        return 1;
    }
    dare_log_t *log = mklog(ring, st[5], st);
    log->old_end = *cursor;
    uint64_t sink[16];
    ref_rec_sink_init(sink, dump, cap, *dump_len);
    uint64_t guard = log->len / 64 + 4, steps = 0;                    /* BUILD-ONLY */
    int corrupt = 0;
    dare_log_entry_t *entry;
    /* TRANSCRIPTION persist (dare_server.c:1796-1802) */
    while (log_is_offset_larger(log, log->end, log->old_end)) {
        if (++steps > guard) { corrupt = 1; break; }                   /* BUILD-ONLY */
        entry = log_get_entry(log, &log->old_end);
        if (!log_fit_entry(log, log->old_end, entry)) {
            log->old_end = 0;
            continue;
        }
        ref_rec_sink_avail(sink, log->len - log->old_end - offsetof(dare_log_entry_t, clt_id));   /* BUILD-ONLY */
        ref_save_request(&entry->clt_id, sink);
    /* END TRANSCRIPTION persist */
        if (ref_rec_sink_stopped(sink)) { corrupt = 1; break; }         /* BUILD-ONLY */
        log->old_end += log_entry_len(entry);
    }
    *cursor = log->old_end;
    *dump_len = (uint32_t)ref_rec_sink_len(sink);
    *n_rec = ref_rec_sink_n(sink);
    return corrupt;
}

/* ref_records_store_one over every group (state rows [n][64], cursor [n],
 * dumps [n][cap], dump_len / n_rec [n]) and ref_records_load_one over every
 * snapshot (dumps at k * stride, size [n]; plan [n][max_plan] 16-B rows,
 * counts [n][3], status / stop / n_records [n]), in place
 * (tests/test_whole_batch.py).  One thread, light log images.  The store
 * returns the groups that stopped (corrupt walk or a full snapshot). */
extern int ref_records_load_one(const uint8_t *buf_in, uint32_t size, void *plan, uint32_t max_plan, uint32_t *n_out,
                                uint32_t counts[3], uint32_t *stop);
uint64_t ref_records_store_batch(uint64_t n, uint64_t stride, const uint8_t *rings, const uint8_t *state,
                                 uint64_t *cursor, uint8_t *dumps, uint64_t cap, uint32_t *dump_len, uint32_t *n_rec)
{
    uint64_t bad = 0;
    g_light = 1;
    for (uint64_t g = 0; g < n; g++)
        bad += (uint64_t)ref_records_store_one(rings + g * stride, (const uint64_t *)(state + 64 * g), cursor + g,
                                               dumps + g * cap, cap, dump_len + g, n_rec + g);
    g_light = 0;
    return bad;
}

void ref_records_load_batch(uint64_t n, const uint8_t *dumps, uint64_t stride, const uint32_t *size, uint8_t *plan,
                            uint32_t max_plan, uint32_t *n_records, uint32_t *counts, uint32_t *status,
                            uint32_t *stop)
{
    for (uint64_t k = 0; k < n; k++) {
        const uint32_t sz = size[k] < stride ? size[k] : (uint32_t)stride;   /* apus_gpu.h: the stride at most */
        status[k] = (uint32_t)ref_records_load_one(dumps + k * stride, sz, max_plan ? plan + 16ull * max_plan * k : NULL,
                                                   max_plan, n_records + k, counts + 3 * k, stop + k);
    }
}

/* 8f.2 — poll_config_entries (dare_server.c:2133-2187) and update_cid
 * (:2193-2227) transcribed on the server's own `data.log` / `data.config`
 * (a struct of those two members here, so every path reads as in the
 * reference), with the real primitives, equal_cid / CID_IS_SERVER_ON
 * (dare_config.h:26,48-56) and PRINT_CONF_TRANSIT.  SNAPSHOT / dare_state
 * (dare_server.c:62-64) restated; dare_ib_disconnect_server(i) records bit i
 * of `departed`, dare_server_shutdown() a flag.  st[0] (head) and cid16 are
 * updated. */
#define SNAPSHOT        0x40
#define DIE_AF_COMMIT   0x80
static uint64_t dare_state;
/* the members of the server's `data` (dare_server.h) these bodies touch */
typedef struct ref_ctrl {
    uint64_t sid;
    uint64_t apply_offsets[MAX_SERVER_COUNT + 1];   /* force_log_pruning (+1: the :2113 write) */
    uint64_t vote_ack[MAX_SERVER_COUNT];            /* poll_vote_count */
    log_offsets_t log_offsets[MAX_SERVER_COUNT];
} ref_ctrl;
typedef struct ref_sm {
    void (*proxy_do_action)(uint16_t clt_id, uint8_t type, size_t len, uint8_t *cmd, void *arg);
    void (*proxy_update_state)(void *arg);
    void *up_para;
} ref_sm;
static struct {
    dare_log_t *log;
    server_config_t config;
    ref_ctrl *ctrl_data;
    ref_sm *sm;
    uint64_t last_cmt_write_csm_idx;
    uint64_t last_write_csm_idx;
    int endpoints;
    void *loop;
} data;
static uint16_t g_departed;
static int g_shutdown;
static void dare_server_shutdown(void) { g_shutdown = 1; }
static void dare_ib_disconnect_server(uint8_t i) { if (i < 16) g_departed |= (uint16_t)(1u << i); }

static int update_cid(dare_cid_t cid)
{
    /* TRANSCRIPTION update_cid (dare_server.c:2195-2226) */
    if (equal_cid(data.config.cid, cid)) {
        return 1;
    }
    PRINT_CONF_TRANSIT(data.config.cid, cid);

    uint8_t i, size = cid.size[0];
    if (cid.size[1] > size) {
        size = cid.size[1];
    }

    for (i = 0; i < size; i++) {
        if ( CID_IS_SERVER_ON(cid, i) &&
            !CID_IS_SERVER_ON(data.config.cid, i) )
        {
        }
        else if ( !CID_IS_SERVER_ON(cid, i) &&
                  CID_IS_SERVER_ON(data.config.cid, i) )
        {
            if (i == data.config.idx) {
                dare_server_shutdown();
            }
            dare_ib_disconnect_server(i);
        }
    }
    data.config.cid = cid;
    return 0;
    /* END TRANSCRIPTION update_cid */
}

static int g_scan_corrupt;
static void poll_config_entries(void)
{
    uint64_t steps = 0, guard = data.log->len / sizeof(dare_log_entry_t) + 4;
    g_scan_corrupt = 0;
    /* TRANSCRIPTION config_scan (dare_server.c:2136-2186) */
    uint64_t head_offset = data.log->head;
    uint64_t offset = data.config.cid_offset;
    uint64_t commit = data.log->commit;
    dare_log_entry_t *entry;
    while (log_offset_end_distance(data.log, offset)) {
        if (++steps > guard) { g_scan_corrupt = 1; return; }   /* BUILD-ONLY: the reference would spin */
        entry = log_get_entry(data.log, &offset);

        if (!log_fit_entry(data.log, offset, entry)) {
            offset = 0;
            continue;
        }
        if (CONFIG == entry->type) {
            if (entry->idx > data.config.cid_idx) {
                if (0 == update_cid(entry->data.cid)) {
                    data.config.req_id = entry->req_id;
                    data.config.clt_id = entry->clt_id;
                }
            }
        }
        else if (HEAD == entry->type) {
            if (!log_is_offset_larger(data.log, offset, commit)) {
                head_offset = entry->data.head;
                dare_state &= ~SNAPSHOT;
            }
        }
        offset += log_entry_len(entry);
    }
    if (log_is_offset_larger(data.log, offset, commit)) {
        data.config.cid_offset = commit;
    }
    else {
        data.config.cid_offset = offset;
    }
    if (log_is_offset_larger(data.log, head_offset, data.log->head)) {
        data.log->head = head_offset;
    }
    /* END TRANSCRIPTION config_scan */
}

int ref_config_scan(const uint8_t *ring, uint64_t st[6], uint8_t cid16[16], uint64_t *cid_offset,
                    uint64_t cid_idx, uint64_t *req_id, uint16_t *clt_id, uint16_t *departed)
{
    data.log = mklog(ring, st[5], st);
    data.config = mkcfg(cid16, 0);
    data.config.cid_offset = *cid_offset;
    data.config.cid_idx = cid_idx;
    data.config.req_id = *req_id;
    data.config.clt_id = *clt_id;
    g_departed = 0;
    g_shutdown = 0;
    dare_state = 0;
    poll_config_entries();
    memcpy(cid16, &data.config.cid, 16);
    *departed = g_departed;
    *req_id = data.config.req_id;
    *clt_id = data.config.clt_id;
    if (g_scan_corrupt) return 1;
    *cid_offset = data.config.cid_offset;
    st[0] = data.log->head;
    return 0;
}

/* 8f.2 — apply_committed_entries (dare_server.c:1815-1974) transcribed on
 * the same `data`, with IS_NONE / IS_LEADER (dare_server.c:42-48) restated.
 * The reference's side effects are recorded instead of performed: client
 * replies (events 1: a STABLE CONFIG's reply, 2: an EXTENDED one's join
 * reply), DIE_AF_COMMIT (event 4), server disconnects (departed), the CONFIG
 * re-append (cfg_cids[n_cfg] + req / clt: the device returns it as append
 * input; event 8 when max_cfg is reached), the state machine call
 * (n_applied).  st[1] (apply) and cid16 are updated. */
#define IS_NONE \
    ( (SID_GET_IDX(data.ctrl_data->sid) == data.config.idx) && \
      (!SID_GET_L(data.ctrl_data->sid)) && \
      (SID_GET_TERM(data.ctrl_data->sid) == 0) )
#define IS_LEADER \
    ( !IS_NONE && (SID_GET_IDX(data.ctrl_data->sid) == data.config.idx) && \
      (SID_GET_L(data.ctrl_data->sid)) )
#define IS_CANDIDATE \
    ( !IS_NONE && (SID_GET_IDX(data.ctrl_data->sid) == data.config.idx) && \
      (!SID_GET_L(data.ctrl_data->sid)) )
static dare_log_entry_det_t last_applied_entry;
static struct {
    uint8_t events, cfg_state;
    uint32_t n_applied, n_cfg, max_cfg;
    uint64_t *cfg_req;
    uint16_t *cfg_clt;
    uint8_t *cfg_cids;
    uint64_t stride;     /* != 0: the re-appends go to the log (log_append_entry), as the reference appends them */
    int refused;         /* such an append met offsets the batched append refuses */
} g_ap;
static int dare_ib_send_clt_reply(uint16_t clt_id, uint64_t req_id, int type)
{
    (void)clt_id; (void)req_id; (void)type;
    g_ap.events |= g_ap.cfg_state == CID_STABLE ? 1 : 2;
    return 0;
}
static void sm_do_action(uint16_t clt_id, uint8_t type, size_t len, uint8_t *cmd, void *arg)
{
    (void)clt_id; (void)type; (void)len; (void)cmd; (void)arg;
    g_ap.n_applied++;
}
static void sm_update_state(void *arg) { (void)arg; g_ap.n_applied++; }
static void ep_dp_reply_read_req(void *ep, uint64_t idx) { (void)ep; (void)idx; }
/* the CONFIG re-append, recorded (log_append_entry in the reference) */
static int fp_append_ok(uint64_t stride);
static uint64_t cfg_append(dare_log_t *log, uint64_t term, uint64_t req_id, uint16_t clt_id, int type, void *cid)
{
    if (g_ap.stride) {
        if (!fp_append_ok(g_ap.stride)) { g_ap.refused = 1; return 0; }
        g_ap.n_cfg++;
        return log_append_entry(log, term, req_id, clt_id, (uint8_t)type, cid);
    }
    if (g_ap.n_cfg < g_ap.max_cfg) {
        g_ap.cfg_req[g_ap.n_cfg] = req_id;
        g_ap.cfg_clt[g_ap.n_cfg] = clt_id;
        memcpy(g_ap.cfg_cids + 16 * g_ap.n_cfg, cid, 16);
        g_ap.n_cfg++;
    }
    return 0;
}

static int g_apply_corrupt;
static void apply_committed_entries(void)
{
    uint64_t steps = 0, guard = data.log->len / sizeof(dare_log_entry_t) + 4;
    int rc;
    int once = 0;
    g_apply_corrupt = 0;
    /* TRANSCRIPTION apply (dare_server.c:1821-1974) */
    uint64_t old_apply = data.log->apply;
    dare_log_entry_t *entry;
    while (log_is_offset_larger(data.log,
                data.log->commit, data.log->apply))
    {
        if (++steps > guard) { g_apply_corrupt = 1; break; }   /* BUILD-ONLY: the reference would spin */
        if (!IS_LEADER) {
        }
        else {
            if (!once) {
                once = 1;
            }
        }

        entry = log_get_entry(data.log, &data.log->apply);
        if (!log_fit_entry(data.log, data.log->apply, entry)) {
            data.log->apply = 0;
            continue;
        }

        if (!IS_LEADER)
            goto apply_entry;

        if ( (NOOP == entry->type) || (HEAD == entry->type) )
            goto apply_next_entry;
        if (CONFIG != entry->type && NOOP != entry->type && HEAD != entry->type) {
            if (entry->req_id != 0) {
            }
            goto apply_entry;
        }

        g_ap.cfg_state = entry->data.cid.state;   /* BUILD-ONLY: which reply */
        if (CID_STABLE == entry->data.cid.state) {
            if (entry->req_id != 0) {
                rc = dare_ib_send_clt_reply(entry->clt_id,
                            entry->req_id, CONFIG);
                if (0 != rc) {
                    error(log_fp, "Cannot send client reply\n");
                }
                if (dare_state & DIE_AF_COMMIT) {
                    dare_server_shutdown();
                }
            }
            goto apply_next_entry;
        }
        if (data.config.cid.epoch > entry->data.cid.epoch) {
            goto apply_next_entry;
        }
        if (g_ap.n_cfg == g_ap.max_cfg) { g_ap.events |= 8; break; }   /* BUILD-ONLY: CFG_FULL */

        dare_cid_t old_cid = data.config.cid;
        uint64_t req_id = entry->req_id;
        uint16_t clt_id = entry->clt_id;

        if (CID_EXTENDED == entry->data.cid.state) {
            data.config.cid.state = CID_TRANSIT;
            if (entry->req_id != 0) {
                rc = dare_ib_send_clt_reply(entry->clt_id,
                            entry->req_id, CONFIG);
                if (0 != rc) {
                    error(log_fp, "Cannot send client reply\n");
                }
                req_id = 0;
                clt_id = 0;
            }
        }
        else if (CID_TRANSIT == entry->data.cid.state) {
            uint8_t i;
            data.config.cid.state = CID_STABLE;
            for (i = data.config.cid.size[1];
                i < data.config.cid.size[0]; i++)
            {
                if (i == data.config.idx) {
                    dare_state |= DIE_AF_COMMIT;
                    CID_SERVER_RM(data.config.cid, i);
                    continue;
                }
                if (!CID_IS_SERVER_ON(data.config.cid, i)) {
                    continue;
                }
                CID_SERVER_RM(data.config.cid, i);
                dare_ib_disconnect_server(i);
            }
            data.config.cid.size[0] = data.config.cid.size[1];
            data.config.cid.size[1] = 0;
        }
        data.config.req_id = req_id;
        data.config.clt_id = clt_id;
        PRINT_CONF_TRANSIT(old_cid, data.config.cid);
        cfg_append(data.log, SID_GET_TERM(data.ctrl_data->sid),
                        req_id, clt_id, CONFIG, &data.config.cid);
        if (g_ap.refused) { g_apply_corrupt = 1; break; }   /* BUILD-ONLY: an append the batched append refuses */
        goto apply_next_entry;

apply_entry:
        if (CONFIG != entry->type && NOOP != entry->type && HEAD != entry->type) {
            if (!IS_LEADER) {
                if (entry->idx % 10000 == 0) {
                    info_wtime(log_fp, "APPLY LOG ENTRY: (%"PRIu64"; %"PRIu64")\n",
                                entry->idx, entry->term);
                }
            }
            if (!IS_LEADER)
                data.sm->proxy_do_action(entry->clt_id, entry->type, entry->data.cmd.len, &entry->data.cmd.cmd, data.sm->up_para);
            else
                data.sm->proxy_update_state(data.sm->up_para);

            last_applied_entry.idx = entry->idx;
            last_applied_entry.term = entry->term;
            last_applied_entry.offset = data.log->apply + log_entry_len(entry);
            data.last_cmt_write_csm_idx = entry->idx;
        }

apply_next_entry:
        data.log->apply += log_entry_len(entry);
    }

    if ((old_apply != data.log->apply) && IS_LEADER) {
        ep_dp_reply_read_req(&data.endpoints, data.last_cmt_write_csm_idx);
    }
    /* END TRANSCRIPTION apply */
}

int ref_apply(const uint8_t *ring, uint64_t st[6], uint8_t cid16[16], uint8_t self, uint64_t sid,
              uint64_t *req_id_io, uint16_t *clt_id_io, uint64_t last_applied[3], uint64_t *last_csm_idx,
              uint32_t *n_applied, uint16_t *departed, uint8_t *events, uint64_t *cfg_req, uint16_t *cfg_clt,
              uint8_t *cfg_cids, uint32_t max_cfg, uint32_t *n_cfg)
{
    static ref_ctrl ctrl;
    static ref_sm sm = { sm_do_action, sm_update_state, NULL };
    data.log = mklog(ring, st[5], st);
    data.config = mkcfg(cid16, self);
    data.config.req_id = *req_id_io;
    data.config.clt_id = *clt_id_io;
    ctrl.sid = sid;
    data.ctrl_data = &ctrl;
    data.sm = &sm;
    data.last_cmt_write_csm_idx = *last_csm_idx;
    last_applied_entry.idx = last_applied[0];
    last_applied_entry.term = last_applied[1];
    last_applied_entry.offset = last_applied[2];
    memset(&g_ap, 0, sizeof g_ap);
    g_ap.max_cfg = max_cfg; g_ap.cfg_req = cfg_req; g_ap.cfg_clt = cfg_clt; g_ap.cfg_cids = cfg_cids;
    g_departed = 0;
    dare_state = 0;
    apply_committed_entries();
    if (dare_state & DIE_AF_COMMIT) g_ap.events |= 4;
    memcpy(cid16, &data.config.cid, 16);
    st[1] = data.log->apply;
    *req_id_io = data.config.req_id;
    *clt_id_io = data.config.clt_id;
    last_applied[0] = last_applied_entry.idx;
    last_applied[1] = last_applied_entry.term;
    last_applied[2] = last_applied_entry.offset;
    *last_csm_idx = data.last_cmt_write_csm_idx;
    *n_applied = g_ap.n_applied;
    *departed = g_departed;
    *events = g_ap.events;
    *n_cfg = g_ap.n_cfg;
    return g_apply_corrupt;
}

/* ref_config_scan / ref_apply over every group of a batch, in place on the
 * state rows [n][64] (the offsets, then the cid) and the io rows, as the
 * batched calls take them (tests/test_whole_batch.py).  One thread: the
 * transcriptions run on the reference's process-wide `data`.  The apply's
 * CONFIG re-appends are written as apus_append_batch records (req_id,
 * data_off = 16 j, clt_id, type CONFIG) with their cid at payload + 16 j,
 * j = g * max_cfg + k.  Returns the groups that stopped on the step guard. */
uint64_t ref_config_scan_batch(uint64_t n, uint64_t stride, const uint8_t *rings, uint8_t *state, uint64_t *cid_offset,
                               const uint64_t *cid_idx, uint64_t *req_id, uint16_t *clt_id, uint16_t *departed)
{
    uint64_t bad = 0;
    g_light = 1;
    for (uint64_t g = 0; g < n; g++)
        bad += (uint64_t)ref_config_scan(rings + g * stride, (uint64_t *)(state + 64 * g), state + 64 * g + 48,
                                         cid_offset + g, cid_idx[g], req_id + g, clt_id + g, departed + g);
    g_light = 0;
    return bad;
}

uint64_t ref_apply_batch(uint64_t n, uint64_t stride, const uint8_t *rings, uint8_t *state, const uint8_t *self,
                         const uint64_t *sid, uint64_t *req_id, uint16_t *clt_id, uint64_t *last_applied,
                         uint64_t *last_csm_idx, uint32_t *n_applied, uint16_t *departed, uint8_t *events,
                         uint8_t *cfg_entries, uint8_t *cfg_payload, uint32_t max_cfg, uint32_t *n_cfg)
{
    uint64_t bad = 0;
    const uint32_t M = max_cfg ? max_cfg : 1;
    uint64_t *creq = (uint64_t *)calloc(M, 8);
    uint16_t *cclt = (uint16_t *)calloc(M, 2);
    uint8_t *ccid = (uint8_t *)calloc(M, 16);
    if (!creq || !cclt || !ccid) { free(creq); free(cclt); free(ccid); return ~0ull; }
    g_light = 1;
    for (uint64_t g = 0; g < n; g++) {
        bad += (uint64_t)ref_apply(rings + g * stride, (uint64_t *)(state + 64 * g), state + 64 * g + 48, self[g],
                                   sid[g], req_id + g, clt_id + g, last_applied + 3 * g, last_csm_idx + g,
                                   n_applied + g, departed + g, events + g, creq, cclt, ccid, max_cfg, n_cfg + g);
        for (uint32_t k = 0; k < n_cfg[g] && k < max_cfg; k++) {
            const uint64_t j = g * max_cfg + k, off = 16 * j;
            uint8_t *r = cfg_entries + 24 * j;
            memset(r, 0, 24);
            memcpy(r, creq + k, 8);
            memcpy(r + 8, &off, 8);
            memcpy(r + 16, cclt + k, 2);
            r[18] = CONFIG;
            memcpy(cfg_payload + off, ccid + 16 * k, 16);
        }
    }
    g_light = 0;
    free(creq); free(cclt); free(ccid);
    return bad;
}

/* 8f.2 — handle_lr_work_completion, dare_ibv_rc.c:3126-3196, on the
 * server_t fields it reads and writes (dare_server.h:86-95); the LR_* steps
 * (dare_server.h:83-84) and WC_SUCCESS (dare_ibv_rc.c:32) restated, as those
 * files need <ev.h> / <infiniband/verbs.h>.  wc: 0 no WC, 1 success, 2 failed,
 * 3 a wr_id other than server->next_wr_id (:3136) */
#define LR_GET_WRITE      1
#define LR_GET_NCE_LEN    2
#define LR_GET_NCE        3
#define LR_SET_END        4
#define LR_UPDATE_LOG     5
#define LR_UPDATE_END     6
#define PERMANENT_FAILURE 2          /* dare_server.h:76 */
#define WC_SUCCESS        0
typedef struct lr_server {
    uint8_t fail_count, next_lr_step, send_flag, send_count;
} lr_server;

void ref_lr_completion(uint8_t wc, uint8_t *step, uint8_t *send_flag, uint8_t *send_count)
{
    if (wc == 0 || wc == 3) return;
    lr_server srv = { 0, *step, *send_flag, *send_count };
    lr_server *server = &srv;
    const int wc_rc = wc == 1 ? WC_SUCCESS : 1;
    /* TRANSCRIPTION lr_completion (dare_ibv_rc.c:3137-3194) */
        if (WC_SUCCESS == wc_rc) {
            if (server->next_lr_step == LR_UPDATE_LOG) {
                switch (server->send_count) {
                    case 0:
                        server->send_flag = 1;
                        break;
                    case 1:
                        server->next_lr_step = LR_UPDATE_END;
                        server->send_flag = 1;
                        break;
                    case 2:
                        server->send_count--;
                        break;
                }
            }
            else if (server->next_lr_step != LR_UPDATE_END) {
                server->next_lr_step++;
                server->send_flag = 1;
            }
            else {
                server->next_lr_step = LR_UPDATE_LOG;
                server->send_flag = 1;
            }
        }
        else {
            if (server->next_lr_step == LR_UPDATE_LOG) {
                switch (server->send_count) {
                    case 0:
                    case 1:
                        server->send_flag = 1;
                        break;
                    case 2:
                        server->send_count = 0;
                        break;
                }
            }
            else if (server->next_lr_step != LR_UPDATE_END) {
                server->send_flag = 1;
            }
            else {
                server->send_flag = 1;
            }
        }
    /* END TRANSCRIPTION lr_completion */
    *step = server->next_lr_step;
    *send_flag = server->send_flag;
    *send_count = server->send_count;
}

/* 8f.2 — log_adjustment, dare_ibv_rc.c:1292-1451, transcribed (region
 * log_adjust, drift-checked) on the real get_extended_group_size,
 * CID_IS_SERVER_ON, log_is_offset_larger and log_find_remote_end_offset over
 * the log's own nc_buf[i].  The transport it posts through is restated here
 * (those headers need <infiniband/verbs.h>): struct server_t (dare_server.h:
 * 86-95), the endpoint's rc_connected / remote MR (dare_ib.h), LOG_QP /
 * CTRL_QP (dare_ibv.h:41-42), SIGNALED and the WRID_SET_* macros
 * (dare_ibv_rc.h:18,32,43), RC_ERROR (dare_ibv_rc.c:27), the two verbs
 * opcodes, and post_send, which records the work request instead of posting
 * it: post[i] 1 = RDMA READ of nc_buf[self].len, 2 = READ of its entries,
 * 3 = WRITE of end (from the remote address it is given).  The BUILD-ONLY
 * lines are the build's documented deviations (apus_gpu.h): servers past R are
 * never visited, an LR_SET_END buffer of length 0 (undefined in the
 * reference) yields log_offsets[i].commit. */
#define LOG_QP   1
#define CTRL_QP  0
#define SIGNALED 1
#define RC_ERROR 1
#define WRID_SET_CONN(wrid, conn) (wrid) = (conn | ((wrid >> 8) << 8))
#define WRID_SET_SSN(wrid, ssn) (wrid) = (((ssn) << 10) | ((wrid) & 0x3FF))
enum ibv_wr_opcode { IBV_WR_RDMA_WRITE = 0, IBV_WR_RDMA_READ = 4 };
struct ibv_mr;
typedef struct rem_mem_t { uint64_t raddr; uint32_t rkey; } rem_mem_t;
typedef struct dare_ib_ep_t {
    int rc_connected;
    struct { struct { uint64_t raddr; uint32_t rkey; } rmt_mr[2]; } rc_ep;
} dare_ib_ep_t;
struct server_t {
    uint64_t next_wr_id, cached_end_offset, last_get_read_ssn;
    void *ep;
    uint8_t fail_count, next_lr_step, send_flag, send_count;
};
static struct { struct ibv_mr *lcl_mr[2]; } g_ibdev;
#define IBDEV (&g_ibdev)
typedef struct rc_ctrl {
    log_offsets_t log_offsets[MAX_SERVER_COUNT];
    uint64_t vote_ack[MAX_SERVER_COUNT];
} rc_ctrl;
typedef struct rc_data { dare_log_t *log; server_config_t config; rc_ctrl *ctrl_data; } rc_data;

static uint8_t *g_posted;
static int post_send(uint8_t server_id, uint8_t qp_id, void *buf, uint32_t len, struct ibv_mr *mr,
                     enum ibv_wr_opcode opcode, uint8_t signaled, rem_mem_t rm, void *posted_sends)
{
    const uint64_t nc = offsetof(dare_log_t, nc_buf) + sizeof(dare_nc_buf_t) * server_id;
    g_posted[server_id] = rm.raddr == nc + offsetof(dare_nc_buf_t, len) ? 1
                        : rm.raddr == nc + offsetof(dare_nc_buf_t, entries) ? 2
                        : rm.raddr == offsetof(dare_log_t, end) ? 3 : 0xFF;
    return 0;
}

static rc_ctrl g_rc_ctrl;
static struct server_t g_rc_servers[MAX_SERVER_COUNT];
static dare_ib_ep_t g_rc_eps[MAX_SERVER_COUNT];

/* the server-side state of one group in the reference's shapes */
static void rc_world(rc_data *srv, const uint64_t st[6], const uint8_t *ring, const uint8_t cid16[16], uint8_t self,
                     uint32_t R, uint16_t rc_conn)
{
    memset(&g_rc_ctrl, 0, sizeof g_rc_ctrl);
    memset(g_rc_servers, 0, sizeof g_rc_servers);
    memset(g_rc_eps, 0, sizeof g_rc_eps);
    srv->log = mklog(ring, ring ? st[5] : 0, st);
    srv->config = mkcfg(cid16, self);
    srv->config.servers = g_rc_servers;
    srv->ctrl_data = &g_rc_ctrl;
    for (uint32_t i = 0; i < MAX_SERVER_COUNT; i++) {
        g_rc_eps[i].rc_connected = i < 16 ? (rc_conn >> i) & 1 : 0;
        g_rc_servers[i].ep = &g_rc_eps[i];
        if (i >= R) g_rc_servers[i].fail_count = PERMANENT_FAILURE;     /* no column: never visited */
    }
}

int ref_log_adjust(const uint8_t *ring, uint64_t st[6], const uint8_t cid16[16], uint8_t self, uint32_t R,
                   const uint8_t *fail_count, uint8_t *step, uint8_t *send_flag, uint16_t rc_conn,
                   const uint64_t *vote_ack, uint64_t *rcommit, uint64_t *rend, const uint64_t *nc_len,
                   const uint64_t *dets /* [R][max_dets][3] */, uint32_t max_dets, uint64_t *ssn_io, uint8_t *post)
{
    rc_data srv;
    rc_data *SRV_DATA = &srv;
    int rc, init;
    struct server_t *server;
    dare_ib_ep_t *ep;
    void *local_buf;
    uint32_t local_buf_len;
    struct ibv_mr *local_mr;
    enum ibv_wr_opcode rdma_opcode;
    rem_mem_t rm;
    uint8_t i, size;
    uint32_t offset;
    uint64_t remote_commit, *remote_end;
    dare_nc_buf_t *nc_buf;
    uint64_t ssn = *ssn_io;
    rc_world(&srv, st, ring, cid16, self, R, rc_conn);
    memset(&rm, 0, sizeof rm);
    for (i = 0; i < R && i < MAX_SERVER_COUNT; i++) {
        uint64_t n = nc_len[i] < max_dets ? nc_len[i] : max_dets;
        srv.log->nc_buf[i].len = n;
        memcpy(srv.log->nc_buf[i].entries, dets + (uint64_t)i * max_dets * 3, n * sizeof(dare_log_entry_det_t));
        g_rc_servers[i].fail_count = fail_count[i];
        g_rc_servers[i].next_lr_step = step[i];
        g_rc_servers[i].send_flag = send_flag[i];
        g_rc_ctrl.vote_ack[i] = vote_ack[i];
        g_rc_ctrl.log_offsets[i].commit = rcommit[i];
        g_rc_ctrl.log_offsets[i].end = rend[i];
        post[i] = 0;
    }
    g_posted = post;
    /* TRANSCRIPTION log_adjust (dare_ibv_rc.c:1313-1446) */
    size = get_extended_group_size(SRV_DATA->config);
    for (i = 0, init = 0; i < size; i++) {
        if ( (i == SRV_DATA->config.idx) ||
            !CID_IS_SERVER_ON(SRV_DATA->config.cid, i) )
            continue;

        server = &SRV_DATA->config.servers[i];
        if (server->fail_count >= PERMANENT_FAILURE) {
            continue;
        }
        if (!server->send_flag) {
            continue;
        }

        ep = (dare_ib_ep_t*)server->ep;
        if (0 == ep->rc_connected) {
            continue;
        }
        remote_commit = SRV_DATA->ctrl_data->vote_ack[i];
        if (SRV_DATA->log->len == remote_commit) {
            continue;
        }

        if ( (!init) && (server->next_lr_step < LR_UPDATE_LOG) ) {
            ssn++;
            init = 1;
        }
        switch(server->next_lr_step) {
            case LR_GET_WRITE:
            {
                SRV_DATA->ctrl_data->log_offsets[i].commit = remote_commit;
                server->next_lr_step = LR_GET_NCE_LEN;
            }
            case LR_GET_NCE_LEN:
            {
                if (log_is_offset_larger(SRV_DATA->log, remote_commit,
                                             SRV_DATA->log->commit))
                {
                    SRV_DATA->log->commit = remote_commit;
                }
                offset = (uint32_t) (offsetof(dare_log_t, nc_buf)
                            + sizeof(dare_nc_buf_t) * i
                            + offsetof(dare_nc_buf_t, len));
                local_buf = &SRV_DATA->log->nc_buf[i].len;
                local_buf_len = sizeof(uint64_t);
                local_mr = IBDEV->lcl_mr[LOG_QP];;
                rdma_opcode = IBV_WR_RDMA_READ;
                break;
            }
            case LR_GET_NCE:
            {
                nc_buf = &SRV_DATA->log->nc_buf[i];
                if (0 == nc_buf->len) {
                    SRV_DATA->ctrl_data->log_offsets[i].end =
                                SRV_DATA->ctrl_data->log_offsets[i].commit;
                    server->next_lr_step = LR_UPDATE_LOG;
                    continue;
                }
                offset = (uint32_t) (offsetof(dare_log_t, nc_buf)
                            + sizeof(dare_nc_buf_t) * i
                            + offsetof(dare_nc_buf_t, entries));
                local_buf = nc_buf->entries;
                local_buf_len = nc_buf->len * sizeof(dare_log_entry_det_t);
                local_mr = IBDEV->lcl_mr[LOG_QP];;
                rdma_opcode = IBV_WR_RDMA_READ;
                break;
            }
            case LR_SET_END:
            {
                offset = (uint32_t) (offsetof(dare_log_t, end));
                remote_end = &SRV_DATA->ctrl_data->log_offsets[i].end;
                if (0 == SRV_DATA->log->nc_buf[i].len) *remote_end = SRV_DATA->ctrl_data->log_offsets[i].commit; else /* BUILD-ONLY: len 0 */
                *remote_end = log_find_remote_end_offset(SRV_DATA->log,
                                            &SRV_DATA->log->nc_buf[i]);
                local_buf = remote_end;
                local_buf_len = sizeof(uint64_t);
                local_mr = IBDEV->lcl_mr[CTRL_QP];;
                rdma_opcode = IBV_WR_RDMA_WRITE;
                break;
            }
            default:
            {
                continue;
            }
        }
        rm.raddr = ep->rc_ep.rmt_mr[LOG_QP].raddr + offset;
        rm.rkey = ep->rc_ep.rmt_mr[LOG_QP].rkey;

        server->send_flag = 0;
        WRID_SET_SSN(server->next_wr_id, ssn);
        WRID_SET_CONN(server->next_wr_id, i);

        rc = post_send(i, LOG_QP, local_buf, local_buf_len, local_mr,
                        rdma_opcode, SIGNALED, rm, NULL);
        if (0 != rc) {
            error_return(RC_ERROR, log_fp, "Cannot post send operation\n");
        }
    }
    /* END TRANSCRIPTION log_adjust */
    for (i = 0; i < R && i < MAX_SERVER_COUNT; i++) {
        step[i] = g_rc_servers[i].next_lr_step;
        send_flag[i] = g_rc_servers[i].send_flag;
        rcommit[i] = g_rc_ctrl.log_offsets[i].commit;
        rend[i] = g_rc_ctrl.log_offsets[i].end;
    }
    st[2] = srv.log->commit;
    *ssn_io = ssn;
    return 0;
}

/* ref_log_adjust over every group / ref_lr_completion over every (group,
 * server) pair of a batch, in place (state rows [n][64]; columns [n][R];
 * nc_len [n][R] u64; dets [n][R][max_dets][3]; ssn [n]; post [n][R]; conn [n]
 * or NULL = all connected), as the batched calls take them
 * (tests/test_whole_batch.py).  One thread (the reference's process-wide
 * state), light log images. */
void ref_log_adjust_batch(uint64_t n, uint32_t R, uint64_t stride, const uint8_t *rings, uint8_t *state,
                          const uint8_t *self, const uint8_t *fail_count, uint8_t *step, uint8_t *send_flag,
                          const uint16_t *conn, const uint64_t *vote_ack, uint64_t *rcommit, uint64_t *rend,
                          const uint64_t *nc_len, const uint64_t *dets, uint32_t max_dets, uint64_t *ssn, uint8_t *post)
{
    g_light = 1;
    for (uint64_t g = 0; g < n; g++)
        (void)ref_log_adjust(rings + g * stride, (uint64_t *)(state + 64 * g), state + 64 * g + 48, self[g], R,
                             fail_count + g * R, step + g * R, send_flag + g * R, conn ? conn[g] : 0xFFFF,
                             vote_ack + g * R, rcommit + g * R, rend + g * R, nc_len + g * R,
                             dets + 3ull * max_dets * R * g, max_dets, ssn + g, post + g * R);
    g_light = 0;
}

void ref_lr_completion_batch(uint64_t pairs, const uint8_t *wc, uint8_t *step, uint8_t *send_flag, uint8_t *send_count)
{
    for (uint64_t k = 0; k < pairs; k++) ref_lr_completion(wc[k], step + k, send_flag + k, send_count + k);
}

/* The lazy remote-commit publish that ends update_remote_logs
 * (dare_ibv_rc.c:1760-1822), transcribed (region publish) on the reference's
 * log primitives and CID_IS_SERVER_ON, in the shapes log_adjustment's
 * transcription restates above.  `size` is what the median loop leaves
 * (dare_ibv_rc.c:1656, as walk_on).  The post of the 8-B commit write
 * (:1799-1812) is recorded in mask; servers past R (no column in a batch) are
 * never visited.  rcommit / ssn in/out. */
/* the publish on a server world (rc_data: the log as the commit rule left
 * it, config, ctrl_data); returns the mask of posted commit writes */
static uint16_t publish_on(rc_data *SRV_DATA, uint32_t R, uint64_t *ssn_io)
{
    uint8_t i, size;
    int init;
    uint32_t offset = 0;
    uint64_t ssn = *ssn_io;
    uint64_t *remote_end, *remote_commit;
    struct server_t *server;
    dare_ib_ep_t *ep;
    uint16_t mask = 0;
    size = (CID_TRANSIT == SRV_DATA->config.cid.state) ? SRV_DATA->config.cid.size[1] : SRV_DATA->config.cid.size[0];
    /* TRANSCRIPTION publish (dare_ibv_rc.c:1761-1794) */
    for (init = 0, i = 0; i < size; i++) {
        if (i >= R) break;                                        /* BUILD-ONLY: no column past R */
        if ( (i == SRV_DATA->config.idx) ||
            !CID_IS_SERVER_ON(SRV_DATA->config.cid, i) )
            continue;

        server = &SRV_DATA->config.servers[i];
        ep = (dare_ib_ep_t*)server->ep;
        if ( (server->fail_count >= PERMANENT_FAILURE)
                || (0 == ep->rc_connected)
                || (server->next_lr_step != LR_UPDATE_LOG) )
        {
            continue;
        }
        remote_commit = &SRV_DATA->ctrl_data->log_offsets[i].commit;
        remote_end = &SRV_DATA->ctrl_data->log_offsets[i].end;
        if ( (*remote_commit == *remote_end) ||
            (*remote_commit == SRV_DATA->log->commit) )
        {
            continue;
        }
        *remote_commit = SRV_DATA->log->commit;
        if (log_is_offset_larger(SRV_DATA->log, *remote_commit, *remote_end)) {
            *remote_commit = *remote_end;
        }
        if (!init) {
            ssn++;
            offset = (uint32_t) (offsetof(dare_log_t, commit));
            init = 1;
        }
    /* END TRANSCRIPTION publish */
        mask |= (uint16_t)(1u << i);                  /* post_send of remote_commit (:1799-1812) */
    }
    (void)offset;
    *ssn_io = ssn;
    return mask;
}

void ref_publish(const uint64_t st[6], const uint8_t cid16[16], uint8_t self, uint32_t R, uint64_t commit,
                 const uint64_t *rend, uint64_t *rcommit, const uint8_t *step, const uint8_t *fail,
                 uint16_t rc_conn, uint16_t *mask_out, uint64_t *ssn_io)
{
    rc_data srv;
    uint8_t i;
    rc_world(&srv, st, NULL, cid16, self, R, rc_conn);
    srv.log->commit = commit;                       /* the log as the commit rule left it (:1747) */
    for (i = 0; i < R && i < MAX_SERVER_COUNT; i++) {
        g_rc_servers[i].fail_count = fail[i];
        g_rc_servers[i].next_lr_step = step[i];
        g_rc_ctrl.log_offsets[i].end = rend[i];
        g_rc_ctrl.log_offsets[i].commit = rcommit[i];
    }
    *mask_out = publish_on(&srv, R, ssn_io);
    for (i = 0; i < R && i < MAX_SERVER_COUNT; i++) rcommit[i] = g_rc_ctrl.log_offsets[i].commit;
}

/* force_log_pruning (dare_server.c:2069-2122) on the real log_append_entry,
 * get_extended_group_size, CID_IS_SERVER_ON / CID_SERVER_RM and
 * log_is_offset_larger; log_pruning is min_apply_on (the "prune"
 * transcription) on the same `data`, its new head / HEAD-append decision
 * recorded as apus_prune_out_t reports them (the HEAD entry is the caller's
 * append).  On offsets the batched append refuses (apus_gpu.h) the removal
 * stops before it changes anything (BUILD-ONLY), as the oracle and the device
 * do.  Servers past R hold apply offsets equal to end (never a minimum).
 * Returns APUS_FORCE_* (0 none, 1 prune, 2 remove, 3 refused). */
static int g_fp_pruned, g_fp_refused;
static uint64_t g_fp_new_head, g_fp_min, g_fp_cfg_idx;
static int g_fp_append;

static void log_pruning(void)
{
    g_fp_pruned = 1;
    g_fp_min = min_apply_on(data.log, data.config, data.ctrl_data->apply_offsets, prev_log_entry_head,
                            &g_fp_new_head, &g_fp_append);
}

static int fp_append_ok(uint64_t stride)
{
    dare_log_t *l = data.log;
    return l->len >= sizeof(dare_log_entry_t) && l->len <= stride && l->end <= l->len && l->tail <= l->len;
}

static uint8_t target;                 /* the reference's local, kept for the report */
static void force_log_pruning_on(uint64_t stride, int *corrupt)
{
    uint8_t i, size;
    /* TRANSCRIPTION force_prune (dare_server.c:2073-2121) */
    uint64_t log_size = log_offset_end_distance(data.log, data.log->head);

    if (log_size < 0.75 * data.log->len)
        return;

    size = get_extended_group_size(data.config);
    target = data.config.idx;
    uint64_t min_offset = data.log->apply;
    for (i = 0; i < size; i++) {
        if (log_is_offset_larger(data.log, min_offset,
                        data.ctrl_data->apply_offsets[i]))
        {
            min_offset = data.ctrl_data->apply_offsets[i];
            target = i;
        }
    }
    if (target != data.config.idx) {
        if (!CID_IS_SERVER_ON(data.config.cid, target)) {
            log_pruning();
            return;
        }
        if (!fp_append_ok(stride)) { *corrupt = 1; g_fp_refused = 1; return; }   /* BUILD-ONLY: APUS_FORCE_REFUSED */
        dare_cid_t old_cid = data.config.cid;
        CID_SERVER_RM(data.config.cid, target);
        dare_ib_disconnect_server(target);
        data.config.req_id = 0;
        data.config.clt_id = 0;

        g_fp_cfg_idx =                                                 /* BUILD-ONLY: the index is reported */
        log_append_entry(data.log, SID_GET_TERM(data.ctrl_data->sid),
                        0, 0, CONFIG, &data.config.cid);

        if (i < MAX_SERVER_COUNT + 1)                                  /* BUILD-ONLY: the ctrl array's bound */
        data.ctrl_data->apply_offsets[i] = data.log->apply;

        log_pruning();
    }
    else {
        log_pruning();
    }
    /* END TRANSCRIPTION force_prune */
}

int ref_force_prune(uint8_t *ring, uint64_t stride, uint64_t st[6], uint8_t cid16[16], uint8_t self, uint32_t R,
                    uint64_t sid, uint64_t *apply_offsets, uint8_t *prev_head, uint64_t *req_id, uint16_t *clt_id,
                    uint64_t *new_head, int *append_head, uint64_t *min_apply, uint8_t *target_out, uint64_t *cfg_idx,
                    int *corrupt)
{
    static ref_ctrl ctrl;
    uint8_t i;
    data.log = mklog(ring, st[5], st);
    data.config = mkcfg(cid16, self);
    data.config.req_id = *req_id;
    data.config.clt_id = *clt_id;
    memset(&ctrl, 0, sizeof ctrl);
    ctrl.sid = sid;
    for (i = 0; i < MAX_SERVER_COUNT + 1; i++) ctrl.apply_offsets[i] = i < R ? apply_offsets[i] : data.log->end;
    data.ctrl_data = &ctrl;
    prev_log_entry_head = *prev_head;
    g_departed = 0;
    g_fp_pruned = 0;
    g_fp_refused = 0;
    g_fp_cfg_idx = 0;
    g_fp_append = 0;
    g_fp_min = 0;
    g_fp_new_head = data.log->head;
    *corrupt = 0;
    target = self;
    force_log_pruning_on(stride, corrupt);
    int action = g_fp_refused ? 3 : g_departed ? 2 : g_fp_pruned ? 1 : 0;
    *target_out = target;
    *new_head = g_fp_new_head;
    *append_head = g_fp_append;
    *min_apply = g_fp_pruned ? g_fp_min : 0;
    *cfg_idx = g_fp_cfg_idx;
    *req_id = data.config.req_id;
    *clt_id = data.config.clt_id;
    *prev_head = (uint8_t)prev_log_entry_head;
    memcpy(ring, data.log->entries, st[5]);
    st[3] = data.log->end;
    st[4] = data.log->tail;
    memcpy(cid16, &data.config.cid, 16);
    for (i = 0; i < R && i < MAX_SERVER_COUNT; i++) apply_offsets[i] = ctrl.apply_offsets[i];
    return action;
}

/* ref_force_prune over every group of a batch, in place on the rings, the
 * state rows [n][64] (commit = the walk's, as the caller sets it between the
 * calls), apply_offsets [n][R], prev_head, req_id, clt_id; outputs [n]
 * (tests/test_whole_batch.py).  One thread, light log images.  Returns the
 * groups whose walk stopped on the step guard. */
uint64_t ref_force_prune_batch(uint64_t n, uint32_t R, uint64_t stride, uint8_t *rings, uint8_t *state,
                               const uint8_t *self, const uint64_t *sid, uint64_t *apply_offsets, uint8_t *prev_head,
                               uint64_t *req_id, uint16_t *clt_id, uint64_t *new_head, uint8_t *append_head,
                               uint64_t *min_apply, uint8_t *target, uint64_t *cfg_idx, uint8_t *action)
{
    uint64_t bad = 0;
    g_light = 1;
    for (uint64_t g = 0; g < n; g++) {
        int app = 0, corrupt = 0;
        action[g] = (uint8_t)ref_force_prune(rings + g * stride, stride, (uint64_t *)(state + 64 * g), state + 64 * g + 48,
                                             self[g], R, sid[g], apply_offsets + g * R, prev_head + g, req_id + g,
                                             clt_id + g, new_head + g, &app, min_apply + g, target + g, cfg_idx + g,
                                             &corrupt);
        append_head[g] = (uint8_t)app;
        bad += corrupt != 0;
    }
    g_light = 0;
    return bad;
}

/* BASELINE config 5's reconfiguration — poll_vote_count (dare_server.c:
 * 1327-1518) whole, on the same `data`: the tally (:1332-1373), then the
 * election-win transition (:1389-1510): server_update_sid's L bit,
 * poll_config_entries and apply_committed_entries above (their CONFIG
 * re-appends now appended to the log, g_ap.stride), the blank entry through
 * the real log_append_entry and become_leader's apply_offsets = head
 * (region vote_count, drift-checked).  The event-loop calls of become_leader
 * (ep_dp_reset_wait_idx, ev_set_cb, ev_timer_again and the timers) are
 * recorders: the host keeps them (apus_gpu.h).  BUILD-ONLY lines: the
 * outcome report (APUS_WIN_*), the stops where a walk passes the step guard
 * or an append meets offsets the batched append refuses, and the
 * uninitialised `entry` of :1426 (read at :1456 when the scan examined no
 * entry) reported instead of dereferenced. */
/* the outcome codes of apus_gpu.h (APUS_WIN_*), restated: this file builds on
 * the reference's headers only */
enum { APUS_WIN_NOT_CANDIDATE, APUS_WIN_LOST, APUS_WIN_CONFIG, APUS_WIN_NOOP, APUS_WIN_TRANSIT, APUS_WIN_STABLE,
       APUS_WIN_UNDEFINED, APUS_WIN_CORRUPT };
typedef struct ev_timer { double repeat; } ev_timer;
static ev_timer hb_event, to_adjust_event, prune_event;
static void hb_send_cb(void) {}
static void ev_set_cb(ev_timer *w, void (*cb)(void)) { (void)w; (void)cb; }
static void ev_timer_again(void *loop, ev_timer *w) { (void)loop; (void)w; }
static void ep_dp_reset_wait_idx(int *endpoints) { (void)endpoints; }
static struct server_t g_win_servers[MAX_SERVER_COUNT];
static int g_win_outcome;

static void poll_vote_count(void)
{
    int rc;
    uint64_t steps = 0, guard = data.log->len / sizeof(dare_log_entry_t) + 4;
    uint8_t vote_count[2];
    /* TRANSCRIPTION vote_count (dare_server.c:1332-1510) */
    vote_count[0] = 1;
    vote_count[1] = 1;
    uint8_t i, size = get_group_size(data.config);
    uint64_t remote_commit;

    for (i = 0; i < size; i++) {
        if (i == data.config.idx) continue;
        remote_commit = data.ctrl_data->vote_ack[i];
        if (data.log->len == remote_commit) {
            continue;
        }
        if (i < data.config.cid.size[0]) {
            vote_count[0]++;
        }
        if (i < data.config.cid.size[1]) {
            vote_count[1]++;
        }

        data.ctrl_data->log_offsets[i].commit = remote_commit;
        data.config.servers[i].next_lr_step = LR_GET_NCE_LEN;
        if (log_is_offset_larger(data.log, remote_commit, data.log->commit)) {
            data.log->commit = remote_commit;
        }
    }

    if (vote_count[0] <  data.config.cid.size[0] / 2 + 1) {
        return;
    }
    if (CID_STABLE != data.config.cid.state) {
        if (vote_count[1] <  data.config.cid.size[1] / 2 + 1) {
            return;
        }
    }
    info(log_fp, "Votes:");
    for (i = 0; i < size; i++) {
        if (i == data.config.idx) continue;
        remote_commit = data.ctrl_data->vote_ack[i];
        if (data.log->len != remote_commit) {
            info(log_fp, " (p%"PRIu8")", i);
        }
    }
    info(log_fp, "\n");

    g_win_outcome = APUS_WIN_CORRUPT;   /* BUILD-ONLY: until an outcome below */
    uint64_t new_sid = data.ctrl_data->sid;
    SID_SET_L(new_sid);
    rc = server_update_sid(new_sid, data.ctrl_data->sid);
    if (0 != rc) {
        return;
    }

    poll_config_entries();
    if (g_scan_corrupt) return;   /* BUILD-ONLY: the scan passed the step guard */

    apply_committed_entries();
    if (g_apply_corrupt) return;   /* BUILD-ONLY: the apply passed the guard / an append refused */

    if (CID_STABLE == data.config.cid.state) {
        data.config.req_id = 0;
        data.config.clt_id = 0;
        if (!fp_append_ok(g_ap.stride)) return;   /* BUILD-ONLY: an append the batched append refuses */
        data.last_write_csm_idx = log_append_entry(data.log,
            SID_GET_TERM(data.ctrl_data->sid), 0, 0, CONFIG, &data.config.cid);
        g_win_outcome = APUS_WIN_CONFIG;   /* BUILD-ONLY */
        goto become_leader;
    }

    uint64_t offset = data.config.cid_offset;
    dare_log_entry_t *entry;
    entry = NULL;   /* BUILD-ONLY: :1426 leaves it uninitialised */
    while (log_offset_end_distance(data.log, offset)) {
        if (++steps > guard) return;   /* BUILD-ONLY: the reference would spin */
        entry = log_get_entry(data.log, &offset);
        if (!log_fit_entry(data.log, offset, entry)) {
            offset = 0;
            continue;
        }
        if ( (CONFIG == entry->type) &&
            (entry->idx > data.config.cid_idx) )
            break;

        offset += log_entry_len(entry);
    }
    if (log_offset_end_distance(data.log, offset)) {
        if (!fp_append_ok(g_ap.stride)) return;   /* BUILD-ONLY: an append the batched append refuses */
        data.last_write_csm_idx = log_append_entry(data.log,
            SID_GET_TERM(data.ctrl_data->sid), 0, 0, NOOP, NULL);
        g_win_outcome = APUS_WIN_NOOP;   /* BUILD-ONLY */
        goto become_leader;
    }

    if (!entry) { g_win_outcome = APUS_WIN_UNDEFINED; goto become_leader; }   /* BUILD-ONLY: :1456 undefined */
    dare_cid_t old_cid = data.config.cid;
    if (CID_EXTENDED == entry->data.cid.state) {
        data.config.cid.state = CID_TRANSIT;
        g_win_outcome = APUS_WIN_TRANSIT;   /* BUILD-ONLY */
    }
    else {
        data.config.cid.state = CID_STABLE;
        g_win_outcome = APUS_WIN_STABLE;   /* BUILD-ONLY */
        uint8_t i;
        for (i = data.config.cid.size[0] - 1;
            i > data.config.cid.size[1]; i--)
        {
            if (i == data.config.idx) {
                dare_state |= DIE_AF_COMMIT;
                CID_SERVER_RM(data.config.cid, i);
                continue;
            }
            if (!CID_IS_SERVER_ON(data.config.cid, i)) {
                continue;
            }
            CID_SERVER_RM(data.config.cid, i);
            dare_ib_disconnect_server(i);
        }
        data.config.cid.size[0] = data.config.cid.size[1];
        data.config.cid.size[1] = 0;
    }
    PRINT_CONF_TRANSIT(old_cid, data.config.cid);
    if (!fp_append_ok(g_ap.stride)) { g_win_outcome = APUS_WIN_CORRUPT; return; }   /* BUILD-ONLY */
    data.last_write_csm_idx = log_append_entry(data.log,
        SID_GET_TERM(data.ctrl_data->sid), data.config.req_id,
        data.config.clt_id, CONFIG, &data.config.cid);

become_leader:
    ep_dp_reset_wait_idx(&data.endpoints);
    ev_set_cb(&hb_event, hb_send_cb);
    hb_event.repeat = NOW;
    ev_timer_again(data.loop, &hb_event);

    to_adjust_event.repeat = 0;
    ev_timer_again(data.loop, &to_adjust_event);

    size = get_extended_group_size(data.config);
    for (i = 0; i < size; i++) {
        data.ctrl_data->apply_offsets[i] = data.log->head;
    }
    prune_event.repeat = NOW;
    ev_timer_again(data.loop, &prune_event);
    /* END TRANSCRIPTION vote_count */
}

/* one group through polling()'s candidate step: IS_CANDIDATE
 * (dare_server.c:1110-1112) -> poll_vote_count.  Columns past R hold no
 * reply (vote_ack = len).  In/out as apus_vote_win_batch; returns APUS_WIN_*. */
/* the body on a log image already holding the group's ring and offsets */
static int vote_count_core(dare_log_t *log, uint8_t *ring, uint64_t stride, uint64_t st[6], uint8_t cid16[16],
                           uint8_t self, uint32_t R, uint64_t *sid, const uint64_t *vote_ack, uint64_t *rcommit,
                           uint8_t *step, uint64_t *apply_offsets, uint8_t *prev_head, uint64_t *cid_offset,
                           uint64_t cid_idx, uint64_t *req_id, uint16_t *clt_id, uint64_t last_applied[3],
                           uint64_t *last_csm_idx, uint64_t *last_write_csm_idx, uint8_t *events, uint16_t *departed,
                           uint32_t *n_applied, uint32_t *n_cfg)
{
    static ref_ctrl ctrl;
    static ref_sm sm = { sm_do_action, sm_update_state, NULL };
    uint32_t i;
    data.log = log;
    data.config = mkcfg(cid16, self);
    memset(g_win_servers, 0, sizeof g_win_servers);
    data.config.servers = g_win_servers;
    data.config.cid_offset = *cid_offset;
    data.config.cid_idx = cid_idx;
    data.config.req_id = *req_id;
    data.config.clt_id = *clt_id;
    memset(&ctrl, 0, sizeof ctrl);
    ctrl.sid = *sid;
    for (i = 0; i < MAX_SERVER_COUNT; i++) {
        ctrl.vote_ack[i] = i < R ? vote_ack[i] : data.log->len;
        ctrl.log_offsets[i].commit = i < R ? rcommit[i] : 0;
        ctrl.apply_offsets[i] = i < R ? apply_offsets[i] : 0;
        g_win_servers[i].next_lr_step = i < R ? step[i] : 0;
    }
    data.ctrl_data = &ctrl;
    data.sm = &sm;
    data.last_cmt_write_csm_idx = *last_csm_idx;
    data.last_write_csm_idx = *last_write_csm_idx;
    last_applied_entry.idx = last_applied[0];
    last_applied_entry.term = last_applied[1];
    last_applied_entry.offset = last_applied[2];
    memset(&g_ap, 0, sizeof g_ap);
    g_ap.stride = stride;
    g_ap.max_cfg = 0xFFFFFFFFu;
    g_departed = 0;
    g_shutdown = 0;
    dare_state = 0;
    g_scan_corrupt = g_apply_corrupt = 0;
    prev_log_entry_head = prev_head ? *prev_head : 0;
    g_win_outcome = APUS_WIN_NOT_CANDIDATE;
    g_sid_cell = &ctrl.sid;
    if (IS_CANDIDATE) {
        g_win_outcome = APUS_WIN_LOST;
        poll_vote_count();
    }
    g_sid_cell = NULL;
    memcpy(ring, data.log->entries, st[5]);
    st[0] = data.log->head; st[1] = data.log->apply; st[2] = data.log->commit;
    st[3] = data.log->end; st[4] = data.log->tail;
    memcpy(cid16, &data.config.cid, 16);
    *sid = ctrl.sid;
    for (i = 0; i < R && i < MAX_SERVER_COUNT; i++) {
        rcommit[i] = ctrl.log_offsets[i].commit;
        step[i] = g_win_servers[i].next_lr_step;
        apply_offsets[i] = ctrl.apply_offsets[i];
    }
    if (prev_head) *prev_head = (uint8_t)prev_log_entry_head;
    *cid_offset = data.config.cid_offset;
    *req_id = data.config.req_id;
    *clt_id = data.config.clt_id;
    last_applied[0] = last_applied_entry.idx;
    last_applied[1] = last_applied_entry.term;
    last_applied[2] = last_applied_entry.offset;
    *last_csm_idx = data.last_cmt_write_csm_idx;
    *last_write_csm_idx = data.last_write_csm_idx;
    *events = g_ap.events | ((dare_state & DIE_AF_COMMIT) ? 4 : 0);
    *departed = g_departed;
    *n_applied = g_ap.n_applied;
    *n_cfg = g_ap.n_cfg;
    return g_win_outcome;
}

int ref_vote_count(uint8_t *ring, uint64_t stride, uint64_t st[6], uint8_t cid16[16], uint8_t self, uint32_t R,
                   uint64_t *sid, const uint64_t *vote_ack, uint64_t *rcommit, uint8_t *step,
                   uint64_t *apply_offsets, uint8_t *prev_head, uint64_t *cid_offset, uint64_t cid_idx,
                   uint64_t *req_id, uint16_t *clt_id, uint64_t last_applied[3], uint64_t *last_csm_idx,
                   uint64_t *last_write_csm_idx, uint8_t *events, uint16_t *departed, uint32_t *n_applied,
                   uint32_t *n_cfg)
{
    return vote_count_core(mklog(ring, st[5], st), ring, stride, st, cid16, self, R, sid, vote_ack, rcommit, step,
                           apply_offsets, prev_head, cid_offset, cid_idx, req_id, clt_id, last_applied,
                           last_csm_idx, last_write_csm_idx, events, departed, n_applied, n_cfg);
}

/* poll_vote_count (the whole of ref_vote_count) over every group of a batch,
 * in place (tests/test_whole_batch.py: the C5 shard's election win): rings
 * [n][stride], state rows [n][64] (the offsets, then the cid), columns [n][R],
 * the win io's rows.  One thread (the transcription runs on the reference's
 * process-wide `data`, and log_append_entry on its global
 * prev_log_entry_head); one dare_log_t image whose header is cleared once
 * (the path writes no nc_buf), its offsets and ring set per group as mklog
 * sets them.  A group IS_CANDIDATE does not select (dare_server.c:49-51,
 * evaluated on the same `data`) is left as ref_vote_count leaves it: nothing
 * moved, APUS_WIN_NOT_CANDIDATE, zero counts.  0, or 1 without memory. */
int ref_vote_count_batch(uint64_t n, uint32_t R, uint64_t stride, uint8_t *rings, uint8_t *state, const uint8_t *self,
                         uint64_t *sid, const uint64_t *vote_ack, uint64_t *rcommit, uint8_t *step,
                         uint64_t *apply_offsets, uint8_t *prev_head, uint64_t *cid_offset, const uint64_t *cid_idx,
                         uint64_t *req_id, uint16_t *clt_id, uint64_t *last_applied, uint64_t *last_csm_idx,
                         uint64_t *last_write_csm_idx, uint8_t *events, uint16_t *departed, uint32_t *n_applied,
                         uint32_t *n_cfg, uint8_t *outcome)
{
    if (!log_fp) log_fp = fopen("/dev/null", "w");
    if (R > MAX_SERVER_COUNT) return 1;
    dare_log_t *log = (dare_log_t *)calloc(1, sizeof(dare_log_t) + stride + 64);
    if (!log) return 1;
    ref_ctrl probe;
    memset(&probe, 0, sizeof probe);
    for (uint64_t g = 0; g < n; g++) {
        uint64_t *st = (uint64_t *)(state + 64 * g);
        uint8_t *cid16 = state + 64 * g + 48;
        probe.sid = sid[g];
        data.ctrl_data = &probe;
        data.config = mkcfg(cid16, self[g]);
        if (!IS_CANDIDATE) {
            outcome[g] = APUS_WIN_NOT_CANDIDATE;
            events[g] = 0; departed[g] = 0; n_applied[g] = 0; n_cfg[g] = 0;
            continue;
        }
        uint8_t *ring = rings + g * stride;
        memcpy(log->entries, ring, st[5]);
        log->head = st[0]; log->apply = st[1]; log->commit = st[2];
        log->end = st[3]; log->tail = st[4]; log->len = st[5];
        log->old_end = st[3]; log->old_commit = 0;
        outcome[g] = (uint8_t)vote_count_core(log, ring, stride, st, cid16, self[g], R, sid + g, vote_ack + g * R,
                                              rcommit + g * R, step + g * R, apply_offsets + g * R, prev_head + g,
                                              cid_offset + g, cid_idx[g], req_id + g, clt_id + g,
                                              last_applied + 3 * g, last_csm_idx + g, last_write_csm_idx + g,
                                              events + g, departed + g, n_applied + g, n_cfg + g);
    }
    free(log);
    return 0;
}

/* ======================================================================
 * CPU baseline of bench.py's step on the reference's own code (bench.py
 * cpu_baseline, kind "reference"): a sample of groups laid out as the
 * reference keeps them -- one dare_log_t image per group (dare_log.h:77-103:
 * the offsets, nc_buf[MAX_SERVER_COUNT], entries[]; one lazily backed
 * mapping, so only the pages a group touches are resident), and per group the
 * server_t array and ctrl_data columns -- built once, outside the timed loop.
 * Each pass runs, for every group, the transcribed bodies above on the
 * compiled dare_log.h: walk_on (dare_ibv_rc.c:1725-1758), the build-defined
 * Adler-32 of the walked entries (the GPU step's checksum; the reference has
 * none: SURVEY 8a a12), median_on (:1650-1723), publish_on (:1760-1822, on the
 * walk's commit), min_apply_on (dare_server.c:2026-2058); with votes
 * vote_on (:1330-1373), the local (idx, term) through log_entries_to_nc_buf
 * into the image's own nc_buf[idx] (dare_server.c:1598-1620) and rank_on
 * (:1526-1655, on a copy of the group's vote_req rows: it clears them in
 * place); with NC buffers the followers' log_find_remote_end_offset over the
 * image's nc_buf[i] (dare_log.h:367-394, dare_ibv_rc.c:1378-1422).  OpenMP
 * static partition of the groups, as the restatement's CPU baseline.
 * ====================================================================== */
#ifdef _OPENMP
#include <omp.h>
#endif
#include <sys/mman.h>

typedef struct ref_bench {
    uint64_t n, img_stride, ring_len;
    uint32_t R, votes, F;
    uint8_t *imgs;                       /* n dare_log_t images                      */
    server_config_t *cfg;                /* [n], servers -> srv + 13 g              */
    struct server_t *srv;                /* [n][13]                                  */
    rc_ctrl *ctrl;                       /* [n] log_offsets (end, commit), vote_ack  */
    dare_ib_ep_t *eps;                   /* [n][13] rc_connected                     */
    uint64_t *rend, *apply, *ack, *ssn;  /* [n][R] / [n] (the batch's columns)       */
    uint8_t *step, *fail, *prev;
    rank_ctrl *rk;                       /* [n] sid, hb, vote_req                    */
    uint8_t *fol;                        /* [n][F] follower index                    */
    uint64_t *out;                       /* [n][4] results kept live                 */
} ref_bench;

static dare_log_t *rb_log(ref_bench *b, uint64_t g) { return (dare_log_t *)(b->imgs + g * b->img_stride); }

/* st [n][6] (head, apply, commit, end, tail, len), cid [n][16], rings [n][ring_stride];
 * columns [n][R]: rend, rcommit, step, fail, apply, vote_ack (NULL: no votes);
 * hb [n][R], req [n][R][5] (sid, index, term, cid16) with votes; sid [n];
 * prev [n]; conn [n] (NULL: all connected); F followers' NC buffers (dets
 * [n][F][M][3], det_len [n][F], follower [n][F]; F = 0: none) */
void *ref_bench_new(uint64_t n, uint32_t R, uint64_t ring_len, const uint8_t *rings, uint64_t ring_stride,
                    const uint64_t *st, const uint8_t *cid, const uint8_t *self, const uint64_t *rend,
                    const uint64_t *rcommit, const uint8_t *step, const uint8_t *fail, const uint64_t *apply,
                    const uint8_t *prev, const uint16_t *conn, const uint64_t *vote_ack, const uint64_t *hb,
                    const uint64_t *req, const uint64_t *sid, uint32_t F, uint32_t M, const uint64_t *dets,
                    const uint32_t *det_len, const uint8_t *follower)
{
    ref_bench *b = (ref_bench *)calloc(1, sizeof *b);
    if (!b || R > MAX_SERVER_COUNT) return NULL;
    if (!log_fp) log_fp = fopen("/dev/null", "w");
    b->n = n; b->R = R; b->ring_len = ring_len; b->votes = vote_ack != NULL; b->F = F;
    b->img_stride = (sizeof(dare_log_t) + ring_len + 64 + 4095) & ~(uint64_t)4095;
    b->imgs = (uint8_t *)mmap(NULL, n * b->img_stride, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE,
                              -1, 0);
    if (b->imgs == MAP_FAILED) { free(b); return NULL; }
    b->cfg = (server_config_t *)calloc(n, sizeof *b->cfg);
    b->srv = (struct server_t *)calloc(n * MAX_SERVER_COUNT, sizeof *b->srv);
    b->ctrl = (rc_ctrl *)calloc(n, sizeof *b->ctrl);
    b->eps = (dare_ib_ep_t *)calloc(n * MAX_SERVER_COUNT, sizeof *b->eps);
    b->rend = (uint64_t *)malloc(n * R * 8); b->apply = (uint64_t *)malloc(n * R * 8);
    b->step = (uint8_t *)malloc(n * R); b->fail = (uint8_t *)malloc(n * R); b->prev = (uint8_t *)malloc(n);
    b->ssn = (uint64_t *)calloc(n, 8); b->out = (uint64_t *)calloc(n * 4, 8);
    memcpy(b->rend, rend, n * R * 8); memcpy(b->apply, apply, n * R * 8);
    memcpy(b->step, step, n * R); memcpy(b->fail, fail, n * R); memcpy(b->prev, prev, n);
    if (b->votes) {
        b->ack = (uint64_t *)malloc(n * R * 8);
        memcpy(b->ack, vote_ack, n * R * 8);
        b->rk = (rank_ctrl *)calloc(n, sizeof *b->rk);
    }
    if (F) b->fol = (uint8_t *)malloc(n * F);
    for (uint64_t g = 0; g < n; g++) {
        dare_log_t *log = rb_log(b, g);
        const uint64_t *s6 = st + 6 * g;
        log->head = s6[0]; log->apply = s6[1]; log->commit = s6[2]; log->end = s6[3]; log->tail = s6[4];
        log->len = s6[5]; log->old_end = s6[3];
        memcpy(log->entries, rings + g * ring_stride, ring_len);
        b->cfg[g] = mkcfg(cid + 16 * g, self[g]);
        b->cfg[g].servers = b->srv + g * MAX_SERVER_COUNT;
        b->cfg[g].len = (uint8_t)R;
        for (uint32_t i = 0; i < MAX_SERVER_COUNT; i++) {
            struct server_t *sv = b->srv + g * MAX_SERVER_COUNT + i;
            dare_ib_ep_t *ep = b->eps + g * MAX_SERVER_COUNT + i;
            ep->rc_connected = conn ? (i < 16 ? (conn[g] >> i) & 1 : 0) : 1;
            sv->ep = ep;
            sv->fail_count = i < R ? fail[g * R + i] : PERMANENT_FAILURE;   /* no column: never visited */
            sv->next_lr_step = i < R ? step[g * R + i] : 0;
            b->ctrl[g].log_offsets[i].end = i < R ? rend[g * R + i] : 0;
            b->ctrl[g].log_offsets[i].commit = i < R ? rcommit[g * R + i] : 0;
            b->ctrl[g].vote_ack[i] = b->votes && i < R ? vote_ack[g * R + i] : log->len;
        }
        if (b->votes) {
            rank_ctrl *k = b->rk + g;
            k->sid = sid[g];
            for (uint32_t i = 0; i < R; i++) {
                k->hb[i] = hb[g * R + i];
                k->vote_req[i].sid = req[5 * (g * R + i)];
                k->vote_req[i].index = req[5 * (g * R + i) + 1];
                k->vote_req[i].term = req[5 * (g * R + i) + 2];
                memcpy(&k->vote_req[i].cid, req + 5 * (g * R + i) + 3, 16);
            }
        }
        for (uint32_t f = 0; f < F; f++) {
            /* the follower's NC buffer where the leader reads it: log->nc_buf[i] */
            const uint8_t i = follower[g * F + f];
            b->fol[g * F + f] = i;
            if (i >= MAX_SERVER_COUNT) continue;
            dare_nc_buf_t *nb = &log->nc_buf[i];
            uint32_t k = det_len[g * F + f] < M ? det_len[g * F + f] : M;
            nb->len = k;
            memcpy(nb->entries, dets + 3 * (uint64_t)M * (g * F + f), 24ull * k);
        }
    }
    return b;
}

void ref_bench_free(void *h)
{
    ref_bench *b = (ref_bench *)h;
    if (!b) return;
    munmap(b->imgs, b->n * b->img_stride);
    free(b->cfg); free(b->srv); free(b->ctrl); free(b->eps); free(b->rend); free(b->apply); free(b->step);
    free(b->fail); free(b->prev); free(b->ssn); free(b->out); free(b->ack); free(b->rk); free(b->fol);
    free(b);
}

/* the build-defined Adler-32 (RFC 1950) of the walked entries' images --
 * [0, 27) ++ 21 zero bytes ++ [48, log_entry_len) from commit to end, on the
 * reference's log_get_entry / log_fit_entry / log_entry_len */
static uint32_t adler_bytes(const uint8_t *p, uint64_t n, uint32_t ad)
{
    uint32_t a = ad & 0xFFFF, c = ad >> 16;
    while (n) {
        uint64_t k = n < 5552 ? n : 5552;
        n -= k;
        while (k--) { a += *p++; c += a; }
        a %= 65521u;
        c %= 65521u;
    }
    return (c << 16) | a;
}
static const uint8_t k_zero21[21];
static uint32_t adler_walk(dare_log_t *log)
{
    uint32_t ad = 1;
    uint64_t o = log->commit, guard = log->len / 64 + 4;
    dare_log_entry_t *entry;
    while ((entry = log_get_entry(log, &o)) != NULL && guard--) {
        if (!log_fit_entry(log, o, entry)) { o = 0; continue; }
        const uint32_t el = log_entry_len(entry);
        ad = adler_bytes((const uint8_t *)entry, 27, ad);
        ad = adler_bytes(k_zero21, 21, ad);
        ad = adler_bytes((const uint8_t *)entry + 48, el - 48, ad);
        o += el;
    }
    return ad;
}

/* group g's step (the results folded into out[4g..], kept live) */
static void ref_bench_group(ref_bench *b, uint64_t g, int checksum)
{
    dare_log_t *log = rb_log(b, g);
    server_config_t cfg = b->cfg[g];
    const uint32_t R = b->R;
    int committed, app;
    uint64_t nh;
    const uint64_t commit0 = log->commit;
    const uint64_t mo = walk_on(log, cfg, &committed);
    const uint32_t dg = checksum ? adler_walk(log) : 0;
    const uint64_t med = median_on(log, cfg, b->rend + g * R, b->step + g * R, b->fail + g * R);
    rc_data srv = { log, cfg, &b->ctrl[g] };
    log->commit = mo;                                      /* the log as the commit rule left it */
    const uint16_t pm = publish_on(&srv, R, &b->ssn[g]);
    log->commit = commit0;
    const uint64_t head0 = log->head;
    const uint64_t mn = min_apply_on(log, cfg, b->apply + g * R, b->prev[g], &nh, &app);
    log->head = head0;                                     /* (the HEAD append is the caller's) */
    b->out[4 * g] = mo ^ med ^ nh;
    b->out[4 * g + 1] = ((uint64_t)dg << 16) ^ pm ^ mn;
    if (b->votes) {
        uint8_t vc[2];
        int won;
        const uint64_t c1 = log->commit;
        vote_on(log, cfg, b->ctrl[g].vote_ack, vc, &won);
        log->commit = c1;                                  /* vote_on raises it (the tally's write) */
        /* the local (idx, term): log_entries_to_nc_buf into nc_buf[idx] */
        dare_nc_buf_t *nb = &log->nc_buf[cfg.idx < MAX_SERVER_COUNT ? cfg.idx : 0];
        log_entries_to_nc_buf(log, nb);
        uint64_t li = 0, lt = 0;
        if (nb->len) { li = nb->entries[nb->len - 1].idx; lt = nb->entries[nb->len - 1].term; }
        else {
            uint64_t t = log_get_tail(log);
            dare_log_entry_t *e = t == log->len ? NULL : log_get_entry(log, &t);
            if (e) { li = e->idx; lt = e->term; }
        }
        rank_ctrl k;
        k.sid = b->rk[g].sid;
        memcpy(k.vote_req, b->rk[g].vote_req, sizeof k.vote_req);   /* rank_on clears them in place */
        for (uint32_t i = 0; i < R; i++) k.hb[i] = b->rk[g].hb[i];
        if (SID_GET_IDX(k.sid) >= R) k.hb[SID_GET_IDX(k.sid)] = 0;   /* the one slot past R it reads */
        int outcome = -1;
        uint16_t clr = 0;
        uint8_t ncid[16];
        g_sid_cell = NULL;
        rank_on(&k, cfg, li, lt, &outcome, &clr, ncid);
        b->out[4 * g + 2] = (uint64_t)won ^ ((uint64_t)outcome << 8) ^ clr ^ g_rank_sid;
    }
    for (uint32_t f = 0; f < b->F; f++) {
        const uint8_t i = b->fol[g * b->F + f];
        if (i >= MAX_SERVER_COUNT) continue;
        dare_nc_buf_t *nb = &log->nc_buf[i];
        /* dare_ibv_rc.c:1378-1384: an empty buffer leaves the remote end at its commit */
        b->out[4 * g + 3] ^= nb->len ? log_find_remote_end_offset(log, nb) : b->ctrl[g].log_offsets[i].commit;
    }
}

/* seconds for `reps` passes over the sample with `threads` OpenMP threads;
 * *digest0 = group 0's checksum (the caller compares it with the port's) */
double ref_bench_time(void *h, int reps, int threads, int checksum, uint64_t *digest0)
{
    ref_bench *b = (ref_bench *)h;
    struct timespec t0, t1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#endif
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int r = 0; r < reps; r++) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
        for (int64_t g = 0; g < (int64_t)b->n; g++) ref_bench_group(b, (uint64_t)g, checksum);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (digest0) *digest0 = b->n ? b->out[1] >> 16 : 0;
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

/* ---- whole-batch check (tests/test_whole_batch.py) ------------------------
 * The GPU step's per-group results from the reference's own code, for every
 * group of a host batch (the device batch's inputs downloaded chunk by
 * chunk): per group the ring is copied into a thread's dare_log_t image
 * (entries[] + the header offsets; nc_buf[idx] is written by
 * log_entries_to_nc_buf), server_t / ctrl_data are built from the columns,
 * and the composed step of ref_bench_group runs with every result kept in its
 * own array: walk_on (dare_ibv_rc.c:1725-1758) + the build's Adler-32, median_on
 * (:1650-1723), publish_on on the walk's commit (:1760-1794; remote_commit
 * written as the RDMA posts would), min_apply_on (dare_server.c:2026-2050; OFF
 * servers' apply offsets reset), and with votes vote_on (:1330-1373), the
 * local (idx, term) (:1598-1620) and rank_on (:1526-1689).  The log is the one
 * the step reads (log->commit back to its input between the calls, as
 * ref_bench_group does). */
typedef struct ref_check_io {
    uint64_t n, ring_stride;
    uint32_t R, votes;
    /* inputs: rings [n][stride], state rows [n][64], self [n], columns [n][R]
     * (lr_step / fail_count u8), prev_head [n], rc_connected [n] (NULL: all),
     * vote_ack / hb [n][R], vote_req [n][R][5 u64], sid [n] */
    const uint8_t *rings, *state, *self, *step, *fail, *prev;
    const uint16_t *conn;
    const uint64_t *rend, *rcommit, *apply, *vote_ack, *hb, *req, *sid;
    /* outputs [n] (remote_commit / apply_offsets [n][R] after the step;
     * vote_count / last_idx_term [n][2]; new_cid [n][16]) */
    uint64_t *new_commit, *median, *ssn, *rcommit_out, *new_head, *min_apply, *apply_out;
    uint64_t *vote_commit, *lit, *new_sid;
    uint8_t *committed, *append_head, *won, *vc, *outcome, *new_cid;
    uint32_t *digest;
    uint16_t *publish, *cleared;
    /* optional (0 / NULL: none): the leader's NC buffer as
     * log_entries_to_nc_buf lists it (dare_log.h:339-359), at most nc_max
     * determinants per group row [n][nc_max][3] with its length [n]; F
     * followers' NC buffers (dets [n][F][M][3], det_len [n][F], follower
     * [n][F]) validated with log_find_remote_end_offset (dare_log.h:367-394;
     * an empty buffer leaves the remote end at log_offsets[i].commit,
     * dare_ibv_rc.c:1378-1384) into rend_follow [n][F] */
    uint32_t nc_max, F, M, pad;
    uint64_t *nc_dets_out;
    uint32_t *nc_len_out;
    const uint64_t *dets;
    const uint32_t *det_len;
    const uint8_t *follower;
    uint64_t *rend_follow;
} ref_check_io;

static void ref_check_group(const ref_check_io *io, uint64_t g, dare_log_t *log, struct server_t *srv,
                            dare_ib_ep_t *eps, rank_ctrl *k)
{
    const uint32_t R = io->R;
    const uint8_t *row = io->state + 64 * g;
    uint64_t s6[6];
    memcpy(s6, row, sizeof s6);
    log->head = s6[0]; log->apply = s6[1]; log->commit = s6[2]; log->end = s6[3]; log->tail = s6[4];
    log->len = s6[5]; log->old_end = s6[3]; log->old_commit = s6[2];
    memcpy(log->entries, io->rings + g * io->ring_stride, s6[5] < io->ring_stride ? s6[5] : io->ring_stride);
    server_config_t cfg = mkcfg(row + 48, io->self[g]);
    cfg.servers = srv;
    cfg.len = (uint8_t)R;
    rc_ctrl ctrl;
    memset(&ctrl, 0, sizeof ctrl);
    for (uint32_t i = 0; i < MAX_SERVER_COUNT; i++) {
        eps[i].rc_connected = io->conn ? (i < 16 ? (io->conn[g] >> i) & 1 : 0) : 1;
        srv[i].ep = &eps[i];
        srv[i].fail_count = i < R ? io->fail[g * R + i] : PERMANENT_FAILURE;
        srv[i].next_lr_step = i < R ? io->step[g * R + i] : 0;
        ctrl.log_offsets[i].end = i < R ? io->rend[g * R + i] : 0;
        ctrl.log_offsets[i].commit = i < R ? io->rcommit[g * R + i] : 0;
        ctrl.vote_ack[i] = io->votes && i < R ? io->vote_ack[g * R + i] : log->len;
    }
    int committed, app;
    uint64_t nh;
    const uint64_t commit0 = log->commit;
    const uint64_t mo = walk_on(log, cfg, &committed);
    io->new_commit[g] = mo;
    io->committed[g] = (uint8_t)committed;
    io->digest[g] = adler_walk(log);
    io->median[g] = median_on(log, cfg, io->rend + g * R, io->step + g * R, io->fail + g * R);
    rc_data srv_data = { log, cfg, &ctrl };
    uint64_t ssn = 0;
    log->commit = mo;                                      /* the publish reads the walk's commit */
    io->publish[g] = publish_on(&srv_data, R, &ssn);
    log->commit = commit0;
    io->ssn[g] = ssn;
    for (uint32_t i = 0; i < R; i++) io->rcommit_out[g * R + i] = ctrl.log_offsets[i].commit;
    uint64_t ap[MAX_SERVER_COUNT];
    memset(ap, 0, sizeof ap);
    memcpy(ap, io->apply + g * R, 8ull * R);
    const uint64_t head0 = log->head;
    io->min_apply[g] = min_apply_on(log, cfg, ap, io->prev[g], &nh, &app);
    log->head = head0;
    io->new_head[g] = nh;
    io->append_head[g] = (uint8_t)app;
    memcpy(io->apply_out + g * R, ap, 8ull * R);
    if (io->nc_max) {
        dare_nc_buf_t *nb = &log->nc_buf[cfg.idx < MAX_SERVER_COUNT ? cfg.idx : 0];
        log_entries_to_nc_buf(log, nb);
        const uint32_t k = nb->len < io->nc_max ? (uint32_t)nb->len : io->nc_max;
        io->nc_len_out[g] = k;
        memcpy(io->nc_dets_out + 3ull * io->nc_max * g, nb->entries, 24ull * k);
    }
    for (uint32_t f = 0; f < io->F; f++) {
        const uint8_t i = io->follower[g * io->F + f];
        if (i >= MAX_SERVER_COUNT || i == cfg.idx) { io->rend_follow[g * io->F + f] = ~0ull; continue; }
        dare_nc_buf_t *nb = &log->nc_buf[i];
        const uint32_t k = io->det_len[g * io->F + f] < io->M ? io->det_len[g * io->F + f] : io->M;
        nb->len = k;
        memcpy(nb->entries, io->dets + 3ull * io->M * (g * io->F + f), 24ull * k);
        io->rend_follow[g * io->F + f] = k ? log_find_remote_end_offset(log, nb) : ctrl.log_offsets[i].commit;
    }
    if (!io->votes) return;
    uint8_t vc[2];
    int won;
    vote_on(log, cfg, ctrl.vote_ack, vc, &won);
    io->won[g] = (uint8_t)won;
    io->vc[2 * g] = vc[0];
    io->vc[2 * g + 1] = vc[1];
    io->vote_commit[g] = log->commit;
    log->commit = commit0;
    dare_nc_buf_t *nb = &log->nc_buf[cfg.idx < MAX_SERVER_COUNT ? cfg.idx : 0];
    log_entries_to_nc_buf(log, nb);
    uint64_t li = 0, lt = 0;
    if (nb->len) { li = nb->entries[nb->len - 1].idx; lt = nb->entries[nb->len - 1].term; }
    else {
        uint64_t t = log_get_tail(log);
        dare_log_entry_t *e = t == log->len ? NULL : log_get_entry(log, &t);
        if (e) { li = e->idx; lt = e->term; }             /* (NULL: (0, 0), as ref_last_idx_term) */
    }
    io->lit[2 * g] = li;
    io->lit[2 * g + 1] = lt;
    k->sid = io->sid[g];
    for (uint32_t i = 0; i < MAX_SERVER_COUNT; i++) {
        const uint64_t *q = io->req + 5 * (g * R + i);
        k->vote_req[i].sid = i < R ? q[0] : 0;            /* slots past R hold no request */
        k->vote_req[i].index = i < R ? q[1] : 0;
        k->vote_req[i].term = i < R ? q[2] : 0;
        if (i < R) memcpy(&k->vote_req[i].cid, q + 3, 16);
        else memset(&k->vote_req[i].cid, 0, 16);
        if (i < R) k->hb[i] = io->hb[g * R + i];
    }
    if (SID_GET_IDX(k->sid) >= R) k->hb[SID_GET_IDX(k->sid)] = 0;   /* the one slot past R it reads */
    int outcome = -1;
    uint16_t clr = 0;
    uint8_t ncid[16];
    memset(ncid, 0, sizeof ncid);
    g_sid_cell = NULL;
    g_rank_sid = k->sid;
    rank_on(k, cfg, li, lt, &outcome, &clr, ncid);
    io->outcome[g] = (uint8_t)outcome;
    io->new_sid[g] = g_rank_sid;
    memcpy(io->new_cid + 16 * g, ncid, 16);
    io->cleared[g] = clr;
}

/* every group of io, `threads` OpenMP threads; 0 = done, 1 = no memory */
int ref_check_batch(const ref_check_io *io, int threads)
{
    int bad = 0;
    if (!log_fp) log_fp = fopen("/dev/null", "w");
    if (io->R > MAX_SERVER_COUNT) return 1;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel reduction(| : bad)
#endif
    {
        dare_log_t *log = (dare_log_t *)malloc(sizeof(dare_log_t) + io->ring_stride + 64);
        struct server_t *srv = (struct server_t *)calloc(MAX_SERVER_COUNT, sizeof *srv);
        dare_ib_ep_t *eps = (dare_ib_ep_t *)calloc(MAX_SERVER_COUNT, sizeof *eps);
        rank_ctrl *k = (rank_ctrl *)calloc(1, sizeof *k);
        const int ok = log && srv && eps && k;
        if (ok) memset(log, 0, sizeof(dare_log_t));
        else bad = 1;                                      /* (its groups left unchecked: reported) */
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t g = 0; g < (int64_t)io->n; g++)
            if (ok) ref_check_group(io, (uint64_t)g, log, srv, eps, k);
        free(log); free(srv); free(eps); free(k);
    }
    return bad;
}
